"""End-to-end (host-memory) rate of BASELINE configs[4]: RS(12,4) 2-erasure
decode, 256 KiB cells, stripes starting and ending in pinned host memory.

HDFS stripes live in host memory (DataNode sockets / block files), so this
measures the repair path including PCIe: per chunk of stripes, the k=12
survivor cells (as `StripeReader` would assemble them, contiguous per stripe)
are copied H2D, decoded by the engine, and the 2 repaired cells copied D2H.
Three HIP streams (H2D, decode, D2H) and a ring of device slots overlap the
chunks (double/triple buffering). Reported per GPU; the 8-GPU config scales
by per-GPU PCIe links (each MI355X has its own x16 Gen5 link) until host DRAM
bandwidth binds.

Run: python tools/bench_e2e.py [--stripes 512 --chunk 32 --slots 3]
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lambdafs_amd import HipReedSolomonCode, device  # noqa: E402

GiB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=12)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--cell", type=int, default=256 << 10)
    ap.add_argument("--stripes", type=int, default=512, help="per GPU (4096 over 8 GPUs)")
    ap.add_argument("--chunk", type=int, default=32)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    k, p, L, S, C = args.k, args.p, args.cell, args.stripes, args.chunk
    n = k + p
    dev = torch.device("cuda:0")
    code = HipReedSolomonCode(k, p, device=0)
    rnd = random.Random(5)
    erased = sorted(rnd.sample(range(n), 2))
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(n) if x not in to_read]
    D = code.decodeMatrix(erased, ntr)[:, to_read]

    # build the host-side stripes: encode on the device once, then keep only
    # the survivors (pinned, [S, k, L]) and the expected erased cells
    gen = torch.Generator(device=dev)
    gen.manual_seed(12)
    host_surv = torch.empty((S, k, L), dtype=torch.uint8, pin_memory=True)
    expect = torch.empty((S, 2, L), dtype=torch.uint8)
    for s0 in range(0, S, 64):
        s1 = min(S, s0 + 64)
        st = torch.randint(0, 256, (s1 - s0, n, L), dtype=torch.uint8, device=dev, generator=gen)
        device.encode_stripes(code, st)
        host_surv[s0:s1].copy_(st[:, to_read].cpu())
        expect[s0:s1].copy_(st[:, erased].cpu())
    host_out = torch.empty((S, 2, L), dtype=torch.uint8, pin_memory=True)
    torch.cuda.synchronize()

    slots = [(torch.empty((C, k, L), dtype=torch.uint8, device=dev),
              torch.empty((C, 2, L), dtype=torch.uint8, device=dev)) for _ in range(args.slots)]
    s_in, s_comp, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()

    def run():
        done_out = [None] * args.slots  # event: slot's D2H finished (slot reusable)
        for ci, s0 in enumerate(range(0, S, C)):
            s1 = min(S, s0 + C)
            m = s1 - s0
            inb, outb = slots[ci % args.slots]
            with torch.cuda.stream(s_in):
                if done_out[ci % args.slots] is not None:
                    s_in.wait_event(done_out[ci % args.slots])
                inb[:m].copy_(host_surv[s0:s1], non_blocking=True)
                ev_in = torch.cuda.Event()
                ev_in.record(s_in)
            with torch.cuda.stream(s_comp):
                s_comp.wait_event(ev_in)
                device.apply_rows(code, D, [inb[:m, i] for i in range(k)], [outb[:m, j] for j in range(2)])
                ev_c = torch.cuda.Event()
                ev_c.record(s_comp)
            with torch.cuda.stream(s_out):
                s_out.wait_event(ev_c)
                host_out[s0:s1].copy_(outb[:m], non_blocking=True)
                ev_o = torch.cuda.Event()
                ev_o.record(s_out)
                done_out[ci % args.slots] = ev_o
        torch.cuda.synchronize()

    run()  # warm
    times = []
    for _ in range(args.reps):
        host_out.zero_()
        t0 = time.perf_counter()
        run()
        times.append(time.perf_counter() - t0)
    ok = torch.equal(host_out, expect)
    t = min(times)
    # device-only decode rate of the same batch for comparison
    big_in = torch.empty((S, k, L), dtype=torch.uint8, device=dev)
    big_in.copy_(host_surv)
    big_out = torch.empty((S, 2, L), dtype=torch.uint8, device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    device.apply_rows(code, D, [big_in[:, i] for i in range(k)], [big_out[:, j] for j in range(2)])
    ev0.record()
    for _ in range(5):
        device.apply_rows(code, D, [big_in[:, i] for i in range(k)], [big_out[:, j] for j in range(2)])
    ev1.record()
    torch.cuda.synchronize()
    dev_ms = ev0.elapsed_time(ev1) / 5
    # pure PCIe reference: pinned H2D of the survivor bytes alone
    t0 = time.perf_counter()
    big_in.copy_(host_surv, non_blocking=True)
    torch.cuda.synchronize()
    h2d = time.perf_counter() - t0
    res = {
        "config": f"RS({k},{p}) decode of {erased} (2 erasures), {L >> 10} KiB cells, {S} stripes/GPU, "
                  f"end-to-end from pinned host memory; chunk {C} stripes, {args.slots} device slots, 3 streams",
        "bit_exact": bool(ok),
        "e2e_GiBps_user_data": round(k * L * S / GiB / t, 2),
        "e2e_ms": round(t * 1e3, 2),
        "pcie_GBps_h2d_plus_d2h": round((k + 2) * L * S / t / 1e9, 2),
        "device_only_decode_GiBps_user_data": round(k * L * S / GiB / (dev_ms * 1e-3), 1),
        "device_only_decode_ms": round(dev_ms, 3),
        "plain_pinned_h2d_GBps": round(k * L * S / h2d / 1e9, 2),
    }
    print(json.dumps(res), flush=True)
    if not ok:
        raise SystemExit("end-to-end decode differs from the erased cells")


if __name__ == "__main__":
    main()
