"""Which window order (HRS_TASK_ORDER: 1 grid-stride, 2 block-cyclic pairs,
0 block range) suits which job shape: the static encode and the pipelined
1-erasure repair over cell sizes 64 KiB-4 MiB and small / large stripe
counts (tools/bench_order.py found block range +3-6 % on bench.py's 1 MiB x
1,024 encode but -16-30 % on configs 4/5's 256 KiB x 512). Medians of
HIP-event times, orders interleaved per rep; outputs compared across orders.
Run: python tools/order_shapes.py [--iters 8] [--reps 3]   (one JSON line per shape x op)
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lambdafs_amd import HipReedSolomonCode, device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=8)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--orders", default="1,2,0")
args = ap.parse_args()
ORDERS = [int(x) for x in args.orders.split(",")]
KiB = 1 << 10
SHAPES = [(10, 4, 64 * KiB, 1024), (10, 4, 64 * KiB, 16384), (10, 4, 256 * KiB, 512), (10, 4, 256 * KiB, 4096),
          (10, 4, 1024 * KiB, 128), (10, 4, 1024 * KiB, 1024), (10, 4, 4096 * KiB, 256),
          (12, 4, 256 * KiB, 512), (12, 4, 256 * KiB, 4096), (12, 4, 1024 * KiB, 1024)]


def timed(fn):
    ms = []
    for _ in range(args.iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return float(np.median(ms))


def sweep(name, fn, target, nbytes, extra):
    outs, times = {}, {o: [] for o in ORDERS}
    for o in ORDERS:
        os.environ["HRS_TASK_ORDER"] = str(o)
        target.fill_(0xA5)
        fn()
        torch.cuda.synchronize()
        outs[o] = target.clone()
    for _ in range(args.reps):
        for o in ORDERS:
            os.environ["HRS_TASK_ORDER"] = str(o)
            fn()
            times[o].append(timed(fn))
    ms = {o: float(np.median(times[o])) for o in ORDERS}
    row = {"op": name, **extra, "ms": {str(o): round(ms[o], 4) for o in ORDERS},
           "TBps": {str(o): round(nbytes / 1e12 / (ms[o] * 1e-3), 3) for o in ORDERS},
           "block_range_vs_grid_stride": round(ms[1] / ms[0], 4) if 0 in ms and 1 in ms else None,
           "identical": all(torch.equal(outs[o], outs[ORDERS[0]]) for o in ORDERS)}
    print(json.dumps(row), flush=True)
    return row["identical"]


def main():
    ok = True
    for k, p, L, S in SHAPES:
        n = k + p
        code = HipReedSolomonCode(k, p)
        st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda")
        extra = {"shape": f"RS({k},{p}) {L // KiB} KiB x {S}", "GiB": round(S * n * L / 2**30, 2),
                 "windows_per_block": S * (L // 2048) // 512}
        ok &= sweep("encode", lambda: device.encode_stripes(code, st), st[:, :p], n * L * S, extra)
        er = [p]
        to_read = sorted(code.locationsToReadForDecode(er))
        ntr = [x for x in range(n) if x not in to_read]
        out = torch.empty((S, 1, L), dtype=torch.uint8, device="cuda")
        ok &= sweep("decode [p]", lambda: device.decode_stripes(code, st, er, ntr, out), out, (k + 1) * L * S, extra)
        del st, out
        torch.cuda.empty_cache()
    os.environ.pop("HRS_TASK_ORDER", None)
    assert ok, "an order changed an output"


if __name__ == "__main__":
    main()
