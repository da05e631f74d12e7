"""Summarize a rocprofv3 SQ counter pass (CSV: run_counter_collection.csv)
per kernel: the mean over dispatches of each counter (summed over its rows),
plus the wave-cycle split the round profiles quote (parked on s_waitcnt,
issue-stalled, issuing, VALU per wave-cycle). Usage:
  python tools/sq_summary.py <csv> [out.json]"""
import collections
import csv
import json
import re
import sys


def short(name):
    name = re.sub(r"hrs::\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name)[:90]


def summarize(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            d = row["Dispatch_Id"]
            per[d][row["Counter_Name"]] += float(row["Counter_Value"])
            names[d] = short(row["Kernel_Name"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d, cs in per.items():
        for c, v in cs.items():
            agg[names[d]][c].append(v)
    out = {}
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["dispatches"] = len(next(iter(cs.values())))
        wc = m.get("SQ_WAVE_CYCLES", 0)
        if wc:
            m["frac_parked_waitcnt"] = round(m.get("SQ_WAIT_ANY", 0) / wc, 3)
            m["frac_issue_stalled"] = round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
            m["frac_issuing"] = round(m.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
            m["valu_per_wave_cycle"] = round(m.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3)
        out[k] = m
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1])
    res = {k: v for k, v in res.items() if "rocclr" not in k and "elementwise" not in k}
    text = json.dumps(res, indent=1)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(text + "\n")
    else:
        print(text)
