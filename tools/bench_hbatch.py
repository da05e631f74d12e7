"""Host-memory batch pipelines (hrs_decode_batch_host / hrs_encode_batch_host)
A/B, interleaved rep by rep in one process:
  ring     H2D -> kernel -> D2H on each slot's stream (round 3; HRS_ZEROCOPY=0)
  duplex   H2D / D2H on per-direction streams (HRS_ZEROCOPY=0 HRS_HBATCH_DUPLEX=1)
  zc       zero copy: the kernels read and write the pinned host memory itself
           (pinned callers: one launch over the caller's stripes; pageable:
           over the slots' pinned staging), default
  zc_bN    zc with the grid capped at N blocks (HRS_ZC_BLOCKS=N; default 64)
  zc_24m / zc_96m  chunk device image 24 / 96 MiB (HRS_HBATCH_BYTES; default 48)
  zc_nomerge  a slot's copy-out and the next copy-in as two pool batches (HRS_HBATCH_MERGE=0)
Workload = BASELINE configs[4] per GPU: RS(12,4), 256 KiB cells, 512 stripes,
a seeded random lost pair per stripe; pinned and pageable host memory.

Run: python tools/bench_hbatch.py [--reps 5]   (one JSON line)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import synth  # noqa: E402
from lambdafs_amd import HipReedSolomonCode, device  # noqa: E402

GiB = float(1 << 30)
KNOBS = ("HRS_ZEROCOPY", "HRS_HBATCH_DUPLEX", "HRS_ZC_BLOCKS", "HRS_HBATCH_BYTES", "HRS_HBATCH_MERGE")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stripes", type=int, default=512)
    ap.add_argument("--zc-blocks", type=int, nargs="*", default=[128, 32, 16])
    args = ap.parse_args()
    k, p, L, S = 12, 4, 256 << 10, args.stripes
    n = k + p
    code = HipReedSolomonCode(k, p, device=0)
    st_dev = torch.zeros((S, n, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, st_dev, 5, 0, k, p)
    device.encode_stripes(code, st_dev)
    ref = st_dev.cpu()
    st = torch.empty((S, n, L), dtype=torch.uint8, pin_memory=True)
    st.copy_(ref)
    stn = st.numpy()
    er = np.array([np.sort(np.random.default_rng([0x5EED0005, s]).choice(n, 2, replace=False)) for s in range(S)],
                  dtype=np.int32)
    out = torch.empty((S, 2, L), dtype=torch.uint8, pin_memory=True)
    outn = out.numpy()
    pg = np.array(stn)
    pout = np.zeros((S, 2, L), np.uint8)
    idx = np.arange(S)[:, None]
    want = ref.numpy()[idx, er]
    pge = np.array(stn)
    legs = {
        "decode_pinned": lambda: device.decode_batch_host(code, stn, er, outn),
        "decode_pageable": lambda: device.decode_batch_host(code, pg, er, pout),
        "encode_pinned": lambda: device.encode_batch_host(code, stn),
        "encode_pageable": lambda: device.encode_batch_host(code, pge),
    }
    modes = {"ring": {"HRS_ZEROCOPY": "0"}, "duplex": {"HRS_ZEROCOPY": "0", "HRS_HBATCH_DUPLEX": "1"},
             "zc": {}, "zc_uncapped": {"HRS_ZC_BLOCKS": "0"},
             "zc_24m": {"HRS_HBATCH_BYTES": str(24 << 20)}, "zc_96m": {"HRS_HBATCH_BYTES": str(96 << 20)},
             "zc_nomerge": {"HRS_HBATCH_MERGE": "0"}}
    for b in args.zc_blocks:
        modes[f"zc_b{b}"] = {"HRS_ZC_BLOCKS": str(b)}
    res = {m: {leg: [] for leg in legs} for m in modes}
    for r in range(args.reps + 1):
        for m, env in modes.items():
            for key in KNOBS:
                os.environ.pop(key, None)
            os.environ.update(env)
            for leg, fn in legs.items():
                if leg == "encode_pinned":
                    stn[:, :p] = 0
                if leg == "encode_pageable":
                    pge[:, :p] = 0
                t0 = time.perf_counter()
                fn()
                dt = (time.perf_counter() - t0) * 1e3
                if r:
                    res[m][leg].append(dt)
                ok = (np.array_equal(outn, want) if leg == "decode_pinned" else
                      np.array_equal(pout, want) if leg == "decode_pageable" else
                      np.array_equal(stn, ref.numpy()) if leg == "encode_pinned" else
                      np.array_equal(pge, ref.numpy()))
                if not ok:
                    raise RuntimeError(f"{m} {leg}: output differs")
                outn[:] = 0
                pout[:] = 0
    for key in KNOBS:
        os.environ.pop(key, None)
    line = {"workload": f"RS({k},{p}) {L >> 10} KiB cells x {S} stripes, random lost pair per stripe",
            "bit_exact": True}
    for m in res:
        for leg, v in res[m].items():
            med = float(np.median(v))
            line[f"{m}_{leg}_ms"] = round(med, 3)
            line[f"{m}_{leg}_min_ms"] = round(float(np.min(v)), 3)
            line[f"{m}_{leg}_GiBps_user"] = round(k * L * S / GiB / (med * 1e-3), 2)
    for m in modes:
        for leg in legs:
            line[f"gain_{m}_vs_ring_{leg}"] = round(line[f"ring_{leg}_ms"] / line[f"{m}_{leg}_ms"], 3)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
