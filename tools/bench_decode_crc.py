"""Decoder's repair + block check on the bench batch (1,024 RS(10,4) stripes,
1 MiB cells, device-resident): fused hrs_decode_crc_dev vs the two passes it
replaces (hrs_decode_dev, then hrs_crc32_dev over the repaired cells) and vs
the plain repair. Kernel times from HIP events on the launch stream (medians
of --iters, variants interleaved per rep); algorithmic bytes = k survivors
read + e repaired cells written (the fused CRC reads nothing extra)."""
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
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--p", type=int, default=4)
ap.add_argument("--cell", type=int, default=1 << 20)
ap.add_argument("--stripes", type=int, default=1024)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--erased", default="4;0,5;1,6,11")
args = ap.parse_args()
k, p, L, S = args.k, args.p, args.cell, args.stripes
n = k + p
code = HipReedSolomonCode(k, p)
st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda")
device.encode_stripes(code, st)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(args.iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return float(np.median(ms))


for rep in range(args.reps):
    for pat in args.erased.split(";"):
        erased = [int(x) for x in pat.split(",")]
        to_read = sorted(code.locationsToReadForDecode(erased))
        ntr = [x for x in range(n) if x not in to_read]
        out = torch.empty((S, len(erased), L), dtype=torch.uint8, device="cuda")
        out2 = torch.empty_like(out)
        orows = [out2[:, i, :] for i in range(len(erased))]

        def fused():
            return device.decode_stripes_crc(code, st, erased, ntr, out)

        def plain():
            device.decode_stripes(code, st, erased, ntr, out2)

        def two_pass():
            plain()
            return device.crc32_rows(code, orows)

        t_f = timed(fused)
        kern = code.lastKernel()
        t_p = timed(plain)
        t_2 = timed(two_pass)
        a, b = fused(), two_pass()
        torch.cuda.synchronize()
        same = bool(torch.equal(a, b)) and bool(torch.equal(out, out2))
        ok = all(bool(torch.equal(out[:, i], st[:, e])) for i, e in enumerate(erased))
        nbytes = (len(to_read) + len(erased)) * L * S
        print(json.dumps({
            "rep": rep, "erased": erased, "kernel": kern, "fused_ms": round(t_f, 4), "plain_ms": round(t_p, 4),
            "two_pass_ms": round(t_2, 4), "fused_GBps": round(nbytes / (t_f * 1e-3) / 1e9, 1),
            "fused_over_plain": round(t_f / t_p, 3), "speedup_vs_two_pass": round(t_2 / t_f, 3),
            "fused_equals_two_pass": same, "repaired_equals_lost": ok,
        }), flush=True)
        del out, out2
