"""Why bench.py's e2e_config5 pageable leg (35-36 ms) is slower than
tools/bench_hbatch.py's (30 ms) on the same box: the same pageable decode
(RS(12,4), 256 KiB cells, 512 stripes, random lost pair) timed bench-style
(fresh arrays, one warm-up, 3 reps) and then in the variants below, in one
process. One JSON line. Usage: python tools/labs/pageable_gap_probe.py (tools/labs is gpurun-ignored: copy it to tools/ to run it on the box)"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from lambdafs_amd import HipReedSolomonCode, device  # noqa: E402


def main():
    k, p, L, S = 12, 4, 256 << 10, 512
    n = k + p
    code = HipReedSolomonCode(k, p, device=0)
    st_dev = torch.zeros((S, n, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, st_dev, 5, 0, k, p)
    device.encode_stripes(code, st_dev)
    st = torch.empty((S, n, L), dtype=torch.uint8, pin_memory=True)
    st.copy_(st_dev.cpu())
    stn = st.numpy()
    er = np.array([np.sort(np.random.default_rng([0x5EED0005, s]).choice(n, 2, replace=False)) for s in range(S)],
                  dtype=np.int32)
    want = stn[np.arange(S)[:, None], er]

    def timed(fn, between=None, reps=3):
        fn()
        ms = []
        for _ in range(reps):
            if between:
                between()
            t0 = time.perf_counter()
            fn()
            ms.append((time.perf_counter() - t0) * 1e3)
        return round(float(np.median(ms)), 3)

    res = {}
    hold_gib = int(os.environ.get("PROBE_HOLD_GIB", "0"))  # device memory held, as bench.py's workload does
    held = torch.empty(hold_gib << 30, dtype=torch.uint8, device="cuda") if hold_gib else None
    if held is not None:
        held.fill_(1)
        torch.cuda.synchronize()
    res["held_gib"] = hold_gib
    pg = np.array(stn)
    pout = np.zeros((S, 2, L), np.uint8)
    dec = lambda: device.decode_batch_host(code, pg, er, pout)  # noqa: E731
    res["bench_style"] = timed(dec)
    res["again"] = timed(dec)
    res["zero_out_between"] = timed(dec, between=lambda: pout.fill(0))
    os.environ["HRS_HOST_NT"] = "0"
    res["cached_stores"] = timed(dec)
    os.environ.pop("HRS_HOST_NT")
    res["again_nt"] = timed(dec)
    out2 = np.empty((S, 2, L), np.uint8)
    out2.fill(1)  # pages touched by this thread first
    res["prefaulted_out"] = timed(lambda: device.decode_batch_host(code, pg, er, out2))
    res["ok"] = bool(np.array_equal(pout, want) and np.array_equal(out2, want))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
