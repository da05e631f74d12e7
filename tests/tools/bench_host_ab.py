"""Synchronous host-buffer calls (the JNI encodeBulk / decodeBulk path), A/B
in one process, calls interleaved: copy engine (pinned staging -> H2D ->
kernel -> D2H, HRS_ZEROCOPY=0) vs zero copy (the kernel reads the staging and
writes its outputs there across the host link), at one RS(10,4) 1 MiB-cell
stripe per call — the shape Encoder.java:442 / Decoder.java:352 issue.
Run: python tests/tools/bench_host_ab.py [--calls 40] [--chunks 524288 ...]   (one JSON line)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from lambdafs_amd import HipReedSolomonCode  # noqa: E402
from oracle import rs_oracle as C  # noqa: E402

GiB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=40)
    args = ap.parse_args()
    k, p, L = 10, 4, 1 << 20
    n = k + p
    code = HipReedSolomonCode(k, p, device=0, zero_inputs_after_encode=False)
    rng = np.random.default_rng(0)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    ref = C.encode_bulk(k, p, [d.copy() for d in data])
    par = [np.zeros(L, np.uint8) for _ in range(p)]
    stripe = ref + data
    erased = [p]
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(n) if x not in to_read]
    reads = [stripe[i] if i in to_read else None for i in range(n)]
    out = [np.zeros(L, np.uint8)]
    modes = {"copy_engine": "0", "zero_copy": "1"}
    t = {m: {"encode": [], "decode": []} for m in modes}
    for r in range(args.calls + 2):
        for m, v in modes.items():
            os.environ["HRS_ZEROCOPY"] = v
            t0 = time.perf_counter()
            code.encodeBulk(data, par)
            t1 = time.perf_counter()
            code.decodeBulk(reads, out, erased, to_read, ntr)
            t2 = time.perf_counter()
            if r >= 2:
                t[m]["encode"].append((t1 - t0) * 1e3)
                t[m]["decode"].append((t2 - t1) * 1e3)
            assert all(np.array_equal(a, b) for a, b in zip(par, ref)), m
            assert np.array_equal(out[0], data[0]), m
            for x in par + out:
                x[:] = 0
    os.environ.pop("HRS_ZEROCOPY")
    line = {"path": "synchronous host-buffer calls, pageable rows, 1 RS(10,4) 1 MiB-cell stripe per call",
            "copy_threads": os.environ.get("HRS_HOST_THREADS", "2 (default)"),
            "chunk_bytes": os.environ.get("HRS_HOST_CHUNK", "524288 (default)"), "bit_exact": True}
    for m in modes:
        for op in ("encode", "decode"):
            med = float(np.median(t[m][op]))
            line[f"{m}_{op}_ms"] = round(med, 3)
            line[f"{m}_{op}_GiBps_user"] = round(k * L / GiB / (med * 1e-3), 2)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
