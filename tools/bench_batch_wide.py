"""Heterogeneous repair batches of wide codes (hrs_decode_batch_dev): a
seeded random erasure pattern (1..p lost) per stripe, device-resident,
HIP-event time of one decode_batch call; algorithmic bytes = the survivors
each stripe's pattern reads + its repaired rows.

  python tools/bench_batch_wide.py [--k 20 --p 8 --stripes 512 --cell 262144]
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
ap.add_argument("--k", type=int, default=20)
ap.add_argument("--p", type=int, default=8)
ap.add_argument("--stripes", type=int, default=512)
ap.add_argument("--cell", type=int, default=256 << 10)
ap.add_argument("--iters", type=int, default=10)
args = ap.parse_args()
k, p, S, L = args.k, args.p, args.stripes, args.cell
n = k + p
code = HipReedSolomonCode(k, p)
st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda")
device.encode_stripes(code, st)
rnd = np.random.default_rng(5)
er = np.full((S, p), -1, dtype=np.int32)
for s in range(S):
    e = sorted(rnd.choice(n, size=int(rnd.integers(1, p + 1)), replace=False).tolist())
    er[s, :len(e)] = e
out = torch.empty((S, p, L), dtype=torch.uint8, device="cuda")
device.decode_batch(code, st, er, out)
torch.cuda.synchronize()
ms = []
for _ in range(args.iters):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    device.decode_batch(code, st, er, out)
    b.record()
    b.synchronize()
    ms.append(a.elapsed_time(b))
ok = all(torch.equal(out[s, :int((er[s] >= 0).sum())], st[s, [int(x) for x in er[s] if x >= 0]]) for s in range(S))
nbytes = sum((k + int((er[s] >= 0).sum())) * L for s in range(S))
med = float(np.median(ms))
print(json.dumps({"k": k, "p": p, "stripes": S, "cell": L, "median_ms": round(med, 4), "min_ms": round(min(ms), 4),
                  "TBps": round(nbytes / (med * 1e-3) / 1e12, 3), "bit_exact": ok}), flush=True)
