"""A/B of the fused encode + CRC kernel's slicing-table replication
(HRS_CRC_REP = 32 | 16 | 8 | 4: lane l reads copy l % R of the bank-private
tables; read per call), interleaved in one process on the bench batch
(RS(10,4), 1,024 x 1 MiB stripes). Occupancy is the same for every R (the
kernel is VGPR-bound at 4 waves/SIMD), so this isolates what
fewer copies cost in LDS bank conflicts. Every variant's CRCs are checked
against the R = 32 run.
  python tools/bench_crc_rep.py [--reps 3 --iters 10 --reps-list 32,16,8,4]
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
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--reps-list", default="32,16,8,4")
ap.add_argument("--no-check", action="store_true", help="skip the R = 32 reference (counter passes: one variant only)")
a = ap.parse_args()
k, p, L, S = 10, 4, 1 << 20, 1024
code = HipReedSolomonCode(k, p)
st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda")
os.environ["HRS_CRC_REP"] = "32"
ref = None if a.no_check else device.encode_stripes_crc(code, st).clone()
for rep in range(a.reps):
    for r in [int(x) for x in a.reps_list.split(",")]:
        os.environ["HRS_CRC_REP"] = str(r)
        got = device.encode_stripes_crc(code, st)
        torch.cuda.synchronize()
        if ref is not None and not torch.equal(got, ref):
            raise SystemExit(f"R={r}: CRCs differ")
        ms = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            device.encode_stripes_crc(code, st)
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        med = float(np.median(ms))
        print(json.dumps({"rep": rep, "copies": r, "kernel": code.lastKernel(), "median_ms": round(med, 4),
                          "min_ms": round(float(np.min(ms)), 4),
                          "TBps": round((k + p) * L * S / (med * 1e-3) / 1e12, 3)}), flush=True)
os.environ.pop("HRS_CRC_REP", None)
