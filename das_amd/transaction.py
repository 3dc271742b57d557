"""Transaction with the reference's API (das/transaction.py:1-10)."""


class Transaction:

    def __init__(self):
        self.metta_string = ""

    def add(self, metta_expression: str) -> None:
        self.metta_string += metta_expression + "\n"
