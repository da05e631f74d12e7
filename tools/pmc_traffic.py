"""Per-kernel HBM bytes per dispatch from rocprofv3 --pmc passes
(profiles/run_rocprof.sh): FETCH_SIZE and WRITE_SIZE from separate runs,
corrected as MI355X_MICROARCH.md prescribes (KiB units; gfx950 reports half of
a 16-B-per-lane streaming read, so FETCH_SIZE is doubled), averaged over the
dispatches of each libhrs kernel, and the kernel-trace average duration beside.

  python tools/pmc_traffic.py <profile dir> [--update profiles/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name):
    m = re.search(r"hrs::\(anonymous namespace\)::([a-z_]+(?:<[^>]*>)?)", name)
    return m.group(1).replace(", ", ",") if m else None


def per_kernel(path, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                k = short(row["Kernel_Name"])
                if k:
                    vals[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def durations(path):
    out = {}
    for f in glob.glob(os.path.join(path, "*kernel_stats.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Name"])
                if k:
                    out[k] = {"calls": int(row["Calls"]), "avg_ms": float(row["AverageNs"]) / 1e6}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profile_dir")
    ap.add_argument("--update", help="pmc_traffic.json to update with the bench kernels")
    a = ap.parse_args()
    fetch = per_kernel(os.path.join(a.profile_dir, "pmc_fetch"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.profile_dir, "pmc_write"), "WRITE_SIZE")
    dur = durations(os.path.join(a.profile_dir, "trace"))
    table = {}
    for k in sorted(set(fetch) | set(write) | set(dur)):
        t = {}
        if k in fetch and k in write:
            t["hbm_bytes_per_dispatch"] = int(round((2 * fetch[k] + write[k]) * 1024))
            t["read_bytes"] = int(round(2 * fetch[k] * 1024))
            t["write_bytes"] = int(round(write[k] * 1024))
        if k in dur:
            t.update(dur[k])
        table[k] = t
    print(json.dumps(table, indent=1))
    if a.update:
        with open(a.update) as fh:
            cur = json.load(fh)
        for k, t in table.items():  # every libhrs kernel the profiled run launched (bench.py looks them up by name)
            if "hbm_bytes_per_dispatch" in t:
                cur[k] = t["hbm_bytes_per_dispatch"]
        cur["_note"] = (cur.get("_note", "").split("; source")[0] + "; source " + a.profile_dir + "/pmc_*/")
        with open(a.update, "w") as fh:
            json.dump(cur, fh, indent=1)
            fh.write("\n")


if __name__ == "__main__":
    main()
