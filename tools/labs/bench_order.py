"""Window -> wave order sweep (HRS_TASK_ORDER, hrs_device.hpp wave_tasks:
C >= 1 = block-cyclic chunks of C windows per wave, 1 = the grid-stride order
of rounds 1-4; 0 = block range) over every streaming kernel the bench and the
BASELINE configs run, in one process: the orders alternate per rep (the
variable is read per launch), medians of HIP-event times on the launch
stream; every order's outputs are compared with order 1's.
Workloads: bench.py's RS(10,4) 1 MiB x 1,024 (encode, fused encode + CRC,
1-4 erasure repairs, fused repair + CRC, random-location repair batches of
1 and 2 losses, CRC-32 of the data rows) and configs 4/5's RS(12,4)
256 KiB x 512 (encode, 2-loss batch).
Run: python tools/bench_order.py [--iters 10] [--reps 3]   (one JSON line per workload)
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
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--orders", default="1,2,4,8,16,32,0")
args = ap.parse_args()
ORDERS = [int(x) for x in args.orders.split(",")]


def timed(fn):
    ms = []
    for _ in range(args.iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return float(np.median(ms))


def set_order(o):
    os.environ["HRS_TASK_ORDER"] = str(o)


def random_losses(S, n, e, seed):
    rng = np.random.default_rng(seed)
    return np.array([np.sort(rng.choice(n, e, replace=False)) for _ in range(S)], dtype=np.int32)


def workloads():
    out = []
    for (k, p, L, S) in ((10, 4, 1 << 20, 1024), (12, 4, 256 << 10, 512)):
        n = k + p
        code = HipReedSolomonCode(k, p)
        st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda")
        device.encode_stripes(code, st)
        shape = f"RS({k},{p}) {L >> 10} KiB x {S}"
        par = st[:, :p]
        out.append((f"{shape} encode", code, lambda code=code, st=st: device.encode_stripes(code, st),
                    lambda r, par=par: par.clone(), par, (k + p) * L * S))
        if k == 10:
            out.append((f"{shape} encode+crc", code, lambda code=code, st=st: device.encode_stripes_crc(code, st),
                        lambda r, par=par: torch.cat([par.flatten(), r.view(torch.uint8).flatten()]), par,
                        (k + p) * L * S))
            for er in ([4], [0, 5], [1, 6, 11], [0, 4, 9, 13]):
                to_read = sorted(code.locationsToReadForDecode(er))
                ntr = [x for x in range(n) if x not in to_read]
                o = torch.empty((S, len(er), L), dtype=torch.uint8, device="cuda")
                out.append((f"{shape} decode {er}", code,
                            lambda code=code, st=st, er=er, ntr=ntr, o=o: device.decode_stripes(code, st, er, ntr, o),
                            lambda r, o=o: o.clone(), o, (k + len(er)) * L * S))
                if len(er) <= 2:
                    o2 = torch.empty_like(o)
                    out.append((f"{shape} decode+crc {er}", code,
                                lambda code=code, st=st, er=er, ntr=ntr, o=o2: device.decode_stripes_crc(
                                    code, st, er, ntr, o),
                                lambda r, o=o2: torch.cat([o.flatten(), r.view(torch.uint8).flatten()]), o2,
                                (k + len(er)) * L * S))
            out.append((f"{shape} crc32 data rows", code,
                        lambda code=code, st=st, p=p, k=k: device.crc32_rows(code, [st[:, p + c] for c in range(k)]),
                        lambda r: r.clone(), None, k * L * S))
        for e in ((1, 2) if k == 10 else (2,)):
            er = random_losses(S, n, e, 0x5EED0000 + e)
            o = torch.empty((S, e, L), dtype=torch.uint8, device="cuda")
            out.append((f"{shape} batch repair {e} random", code,
                        lambda code=code, st=st, er=er, o=o: device.decode_batch(code, st, er, o),
                        lambda r, o=o: o.clone(), o, (k + e) * L * S))
    return out


def main():
    bad = []
    for name, code, fn, snap, target, nbytes in workloads():
        times = {o: [] for o in ORDERS}
        outs, kern = {}, {}
        for o in ORDERS:
            set_order(o)
            if target is not None:
                target.fill_(0xA5)  # a task the order skips would leave this behind
            r = fn()
            torch.cuda.synchronize()
            outs[o] = snap(r)
            kern[o] = code.lastKernel()
        for _ in range(args.reps):
            for o in ORDERS:
                set_order(o)
                fn()
                torch.cuda.synchronize()
                times[o].append(timed(fn))
        ms = {o: float(np.median(times[o])) for o in ORDERS}
        best = min(ORDERS, key=lambda o: ms[o])
        ident = {o: bool(torch.equal(outs[o], outs[ORDERS[0]])) for o in ORDERS}
        row = {"workload": name, "kernel": kern[ORDERS[0]], "ms": {str(o): round(ms[o], 4) for o in ORDERS},
               "best_order": best, "best_vs_grid_stride": round(ms[1] / ms[best], 4) if 1 in ms else None,
               "best_TBps": round(nbytes / 1e12 / (ms[best] * 1e-3), 3), "identical": all(ident.values()),
               "same_kernel": len(set(kern.values())) == 1}
        print(json.dumps(row), flush=True)
        if not row["identical"]:
            bad.append(name)
        del outs
    os.environ.pop("HRS_TASK_ORDER", None)
    assert not bad, f"order changed an output: {bad}"


if __name__ == "__main__":
    main()
