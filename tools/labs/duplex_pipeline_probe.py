"""Which stream structure lets a chunked H2D -> kernel -> D2H pipeline use
both directions of the host link at once? (the plain
duplex probe, tools/duplex_probe.py, shows the link is full duplex for
independent chunked copies on two streams.) Job = BASELINE configs[4] per
GPU: 512 stripes x 12 cells x 256 KiB in (1.61 GB), 2 cells per stripe out,
chunks of 12 stripes through a ring of 3 device slots, pinned host memory; the
"kernel" is a small torch op standing in for the repair. Variants:
  ring      each slot's stream runs H2D, kernel, D2H (the round-3 pipeline);
  dir2      H2D and kernel on one copy-in stream, D2H on a copy-out stream
            (one event per chunk; slot reuse via the in-order streams and
            one wait for the slot's previous D2H before its kernel);
  dir3      H2D on copy-in, kernel on the slot's stream, D2H on copy-out
            (three events per chunk);
each with one H2D copy per stripe ("stripe") or per chunk ("chunk").
Run: python tools/duplex_pipeline_probe.py [--reps 5]   (one JSON line)
"""
import argparse
import json
import time

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    L, S, nin, nout, chunk, nslots = 256 << 10, 512, 12, 2, 12, 3
    dev = torch.device("cuda", 0)
    hin = torch.empty((S, nin, L), dtype=torch.uint8, pin_memory=True)
    hin.copy_(torch.randint(0, 256, (S, nin, L), dtype=torch.uint8))
    hout = torch.empty((S, nout, L), dtype=torch.uint8, pin_memory=True)
    want = hin[:, :nout] ^ 0x5A
    dimg = [torch.empty((chunk, nin, L), dtype=torch.uint8, device=dev) for _ in range(nslots)]
    dout = [torch.empty((chunk, nout, L), dtype=torch.uint8, device=dev) for _ in range(nslots)]
    slot_st = [torch.cuda.Stream() for _ in range(nslots)]
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    ev = {n: [torch.cuda.Event() for _ in range(nslots)] for n in ("in", "comp", "done")}

    def h2d(sl, s0, ns, per):
        if per == "chunk":
            dimg[sl][:ns].copy_(hin[s0:s0 + ns], non_blocking=True)
        else:
            for i in range(ns):
                dimg[sl][i].copy_(hin[s0 + i], non_blocking=True)

    def kern(sl, ns):
        torch.bitwise_xor(dimg[sl][:ns, :nout], 0x5A, out=dout[sl][:ns])

    def d2h(sl, s0, ns, per):
        if per == "chunk":
            hout[s0:s0 + ns].copy_(dout[sl][:ns], non_blocking=True)
        else:
            for i in range(ns):
                hout[s0 + i].copy_(dout[sl][i], non_blocking=True)

    def run(variant, per):
        used = [False] * nslots
        for j, s0 in enumerate(range(0, S, chunk)):
            sl, ns = j % nslots, min(chunk, S - s0)
            if variant == "ring":
                with torch.cuda.stream(slot_st[sl]):
                    h2d(sl, s0, ns, per)
                    kern(sl, ns)
                    d2h(sl, s0, ns, per)
            elif variant == "dir2":
                with torch.cuda.stream(s_in):
                    h2d(sl, s0, ns, per)
                    if used[sl]:
                        s_in.wait_event(ev["done"][sl])
                    kern(sl, ns)
                    ev["comp"][sl].record(s_in)
                s_out.wait_event(ev["comp"][sl])
                with torch.cuda.stream(s_out):
                    d2h(sl, s0, ns, per)
                    ev["done"][sl].record(s_out)
            else:  # dir3
                if used[sl]:
                    s_in.wait_event(ev["comp"][sl])
                with torch.cuda.stream(s_in):
                    h2d(sl, s0, ns, per)
                    ev["in"][sl].record(s_in)
                slot_st[sl].wait_event(ev["in"][sl])
                if used[sl]:
                    slot_st[sl].wait_event(ev["done"][sl])
                with torch.cuda.stream(slot_st[sl]):
                    kern(sl, ns)
                    ev["comp"][sl].record(slot_st[sl])
                s_out.wait_event(ev["comp"][sl])
                with torch.cuda.stream(s_out):
                    d2h(sl, s0, ns, per)
                    ev["done"][sl].record(s_out)
            used[sl] = True
        torch.cuda.synchronize()

    res = {"job": f"{S} stripes x {nin} x {L >> 10} KiB in, {nout} cells out, chunks of {chunk}, {nslots} slots"}
    variants = [(v, per) for v in ("ring", "dir2", "dir3") for per in ("stripe", "chunk")]
    times = {f"{v}_{per}": [] for v, per in variants}
    for r in range(args.reps + 1):
        for v, per in variants:
            hout.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(v, per)
            dt = (time.perf_counter() - t0) * 1e3
            if not torch.equal(hout, want):
                raise RuntimeError(f"{v}_{per}: wrong output")
            if r:
                times[f"{v}_{per}"].append(dt)
    for key, t in times.items():
        res[f"{key}_ms"] = round(float(np.median(t)), 3)
    # the link alone: one pinned H2D of the input bytes
    big = torch.empty((S, nin, L), dtype=torch.uint8, device=dev)
    t = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        big.copy_(hin, non_blocking=True)
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
    res["h2d_alone_ms"] = round(float(np.median(t)), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
