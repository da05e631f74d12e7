"""Throughput of hrs_crc32_dev on the bench batch: CRC-32 of every source and
parity cell of 1,024 RS(10,4) stripes with 1 MiB cells (14 GiB), device-resident."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lambdafs_amd import HipReedSolomonCode, device  # noqa: E402

k, p, L, S = 10, 4, 1 << 20, 1024
code = HipReedSolomonCode(k, p)
st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda")
rows = [st[:, r, :] for r in range(k + p)]
device.crc32_rows(code, rows)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 10
e0.record()
for _ in range(reps):
    device.crc32_rows(code, rows)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
nbytes = (k + p) * L * S
print(json.dumps({"crc32_rows": k + p, "stripes": S, "cell": L, "ms": round(ms, 3),
                  "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1), "frac_of_8TBps": round(nbytes / (ms * 1e-3) / 8e12, 3)}))
