"""Summarise rocprofv3 --pmc databases: per kernel (name filter), the counter
values of the LAST dispatches matching, one row per dispatch."""
import re
import sqlite3
import sys


def short(n):
    n = n.replace('das::(anonymous namespace)::', '').replace('das::', '').replace('void ', '')
    return re.sub(r'\(.*', '', n)[:28]


def main(dbs, pat, last=6):
    rows = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for disp, name, cn, v, dur in c.execute(
                "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
            if re.search(pat, name):
                rows.setdefault((db, disp), {"name": short(name), "dur_us": dur / 1000})[cn] = v
    for db in dbs:
        keys = sorted(k for k in rows if k[0] == db)[-last:]
        for k in keys:
            print(db.split('/')[-2], k[1], rows[k])


if __name__ == "__main__":
    main(sys.argv[2:], sys.argv[1])
