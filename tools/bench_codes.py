"""Device-resident encode / decode rates of every code family behind the
boundary (rs = ReedSolomonCode, nrs = NativeReedSolomonCode, xor = XORCode),
one JSON line per (code, op). Same layout and timing as bench.py: [S, n, L]
hops-order stripes in HBM, HIP events on the launching (current) stream,
algorithmic bytes = rows read + rows written.

decode e: e lost locations repaired from the survivors
locationsToReadForDecode picks (rs/xor: the first e data locations; nrs: the
same not-to-read set, outputs in the Java's Apache order). Each timed
output is checked against the stripe it reproduces.

  python tools/bench_codes.py [--stripes 1024 --cell 1048576 --iters 10]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lambdafs_amd import HipNativeReedSolomonCode, HipReedSolomonCode, HipXORCode, device  # noqa: E402

GB = 1e9


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / iters


def run(name, code, S, L, iters, out):
    k, p = code.stripeSize(), code.paritySize()
    n = k + p
    st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda")
    ms = timed(lambda: device.encode_stripes(code, st), iters)
    out.append({"code": name, "k": k, "p": p, "op": "encode", "stripes": S, "cell": L, "ms": round(ms, 4),
                "GBps_hbm": round(n * L * S / (ms * 1e-3) / GB, 1),
                "GiBps_user": round(k * L * S / (ms * 1e-3) / 2 ** 30, 1)})
    for e in range(1, p + 1):
        lost = [p + i for i in range(e)]
        to_read = sorted(code.locationsToReadForDecode(lost))
        ntr = [x for x in range(n) if x not in to_read]
        if name == "nrs":  # outputs follow the Apache-sorted not-to-read list
            lost = sorted(ntr, key=lambda loc: loc + k if loc < p else loc - p)[:e]
        res = torch.empty((S, e, L), dtype=torch.uint8, device="cuda")
        ms = timed(lambda: device.decode_stripes(code, st, lost, ntr, res), iters)
        if not torch.equal(res, st[:, lost, :]):
            raise RuntimeError(f"{name} decode of {lost} did not reproduce the stripe")
        out.append({"code": name, "k": k, "p": p, "op": f"decode{e}", "stripes": S, "cell": L,
                    "ms": round(ms, 4), "GBps_hbm": round((k + e) * L * S / (ms * 1e-3) / GB, 1),
                    "GiBps_user": round(k * L * S / (ms * 1e-3) / 2 ** 30, 1)})
    del st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=1024)
    ap.add_argument("--cell", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--codes", default="rs,nrs,xor", help="comma list of rs, nrs, xor")
    args = ap.parse_args()
    torch.manual_seed(7)
    rows = []
    codes = args.codes.split(",")
    if "rs" in codes:
        run("rs", HipReedSolomonCode(10, 4), args.stripes, args.cell, args.iters, rows)
    if "nrs" in codes:
        run("nrs", HipNativeReedSolomonCode(10, 4), args.stripes, args.cell, args.iters, rows)
        run("nrs", HipNativeReedSolomonCode(6, 3), args.stripes, args.cell, args.iters, rows)
    if "xor" in codes:
        run("xor", HipXORCode(10, 1), args.stripes, args.cell, args.iters, rows)
    for r in rows:
        r["blocks_per_cu_env"] = os.environ.get("HRS_BLOCKS_PER_CU", "default")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
