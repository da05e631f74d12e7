"""Encoder with computeBlockChecksum on the bench batch (1,024 RS(10,4)
stripes, 1 MiB cells, device-resident): fused hrs_encode_crc_dev vs the two
passes it replaces (hrs_encode_dev, then hrs_crc32_dev over the 14 cells).
Kernel times from HIP events on the launch stream; algorithmic bytes = each
cell once: read k, write p (the CRC reads nothing extra when fused)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lambdafs_amd import HipNativeReedSolomonCode, HipReedSolomonCode, device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--p", type=int, default=4)
ap.add_argument("--cell", type=int, default=1 << 20)
ap.add_argument("--stripes", type=int, default=1024)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--nrs", action="store_true")
args = ap.parse_args()
k, p, L, S = args.k, args.p, args.cell, args.stripes
code = (HipNativeReedSolomonCode if args.nrs else HipReedSolomonCode)(k, p)
st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda")
rows = [st[:, p + c, :] for c in range(k)] + [st[:, r, :] for r in range(p)]


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
    return float(np.median(ms)), float(np.min(ms))


def two_pass():
    device.encode_stripes(code, st)
    return device.crc32_rows(code, rows)


fused_med, fused_min = timed(lambda: device.encode_stripes_crc(code, st))
two_med, two_min = timed(two_pass)
enc_med, _ = timed(lambda: device.encode_stripes(code, st))
a = device.encode_stripes_crc(code, st)
b = two_pass()
torch.cuda.synchronize()
same = bool(torch.equal(a, b))
nbytes = (k + p) * L * S
print(json.dumps({
    "what": f"{'nrs' if args.nrs else 'rs'}({k},{p}) encode + CRC32 of all {k + p} cells, {S} x {L >> 10} KiB",
    "fused_ms": round(fused_med, 3), "fused_min_ms": round(fused_min, 3),
    "fused_GBps": round(nbytes / (fused_med * 1e-3) / 1e9, 1),
    "two_pass_ms": round(two_med, 3), "two_pass_min_ms": round(two_min, 3),
    "encode_only_ms": round(enc_med, 3),
    "speedup": round(two_med / fused_med, 3), "fused_equals_two_pass": same,
}), flush=True)
