"""The service's postfix query language (service/server.py:34-81).

A query is a comma-separated list of chunks, e.g.

    Node n1 Concept human, Node n2 Concept mammal, Link Inheritance $1 n1,
    Link Inheritance $1 n2, AND

`Node <alias> <type> <name>` chunks come first and name the grounded targets;
then `Link <type> <arg>...` chunks push a Link (an argument is a `$variable`
or a node alias; the link is unordered iff its type is in
UNORDERED_LINK_TYPES); `AND` / `OR` fold the whole stack into one term, `NOT`
negates the top.  Malformed queries return None, exactly where the reference
does; an empty chunk raises IndexError as the reference's `chunk[0]` does.
"""
from ..database.db_interface import UNORDERED_LINK_TYPES
from ..pattern_matcher.pattern_matcher import And, Link, Node, Not, Or, Variable


def _parse_query(query_str: str):
    reading_nodes = True            # server.py:35 current_state 0 / 1
    nodes = {}
    stack = []
    for raw in query_str.split(","):
        words = raw.strip().split()
        head = words[0]
        if reading_nodes:
            if head == "Node":
                if len(words) != 4:
                    return None
                nodes[words[1]] = Node(words[2], words[3])
                continue
            reading_nodes = False
        if head == "Link":
            if len(words) < 3:
                return None
            targets = []
            for arg in words[2:]:
                if arg.startswith("$"):
                    targets.append(Variable(arg))
                elif arg in nodes:
                    targets.append(nodes[arg])
                else:
                    return None
            stack.append(Link(words[1], targets, words[1] not in UNORDERED_LINK_TYPES))
            continue
        if not stack:
            return None
        if head == "AND":
            stack = [And(stack)]
        elif head == "OR":
            stack = [Or(stack)]
        elif head == "NOT":
            stack.append(Not(stack.pop()))
        else:
            return None
    if len(stack) != 1:
        return None
    return stack[0]


parse_query = _parse_query
