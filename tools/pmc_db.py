"""Summarize a rocprofv3 rocpd database (run_results.db): per kernel, the mean
over dispatches of each counter (summed over its per-SE/XCD rows) and the mean
dispatch duration. Usage: python tools/pmc_db.py <db> [kernel-substring]"""
import collections
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"hrs::\(anonymous namespace\)::", "", name)
    return name[:80]


def summarize(db, pat=""):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = {}
    for d, k, c, v, du in rows:
        if pat and pat not in k:
            continue
        per[d][c] += v
        dur[d] = du
        names[d] = short(k)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, cs in per.items():
        for c, v in cs.items():
            agg[names[d]][c].append(v)
        agg[names[d]]["duration_ns"].append(dur[d])
    out = {}
    for k, cs in agg.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = len(cs["duration_ns"])
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    for k, cs in res.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {v:,.0f}")
