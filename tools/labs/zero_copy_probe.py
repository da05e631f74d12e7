"""Kernels reading and writing pinned host memory directly ("zero copy")
instead of H2D -> kernel -> D2H. A kernel's loads and
stores to pinned host memory cross the link as they issue, reads and writes
in flight together, so a coding kernel run over host stripes would use both
link directions at once with no copy engine and no per-stripe copy calls.
Measured here on one GPU, pinned host memory from torch (hipHostMalloc):
  link_read   hrs_probe_stream COPY host -> device (1.5 GiB): the kernel's PCIe read rate
  link_write  COPY device -> host: its PCIe write rate
  link_both   COPY host -> host: reads and writes at once
  dma_h2d     the copy engine's H2D of the same bytes, for comparison
  encode      hrs_encode_dev over BASELINE configs[4]'s shape (RS(12,4), 256 KiB
              cells, 512 stripes) resident in pinned host memory, vs the
              product's hrs_encode_batch_host (H2D, kernel, D2H pipeline)
  repair      hrs_decode_batch_dev over the same host stripes with config 5's
              seeded random lost pairs, outputs in pinned host memory, vs
              hrs_decode_batch_host
Outputs are checked against the device-resident results.
Run: python tools/zero_copy_probe.py [--reps 5]   (one JSON line)
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
from lambdafs_amd import HipReedSolomonCode, _lib, device  # noqa: E402
from lambdafs_amd._lib import ptr_array  # noqa: E402

GiB = float(1 << 30)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(t)), 3)


def device_pointer(t):
    """hipHostGetDevicePointer of a pinned tensor: the address a kernel uses
    for it. The probe runs only where that is the host address itself (HIP's
    unified addressing), so no kernel dereferences an unmapped pointer."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    dp = ctypes.c_void_p()
    st = hip.hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(t.data_ptr()), 0)
    return dp.value if st == 0 else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    reps = args.reps
    k, p, L, S = 12, 4, 256 << 10, 512
    n = k + p
    res = {"what": "kernels on pinned host memory vs copy-engine pipelines", "shape": f"RS({k},{p}) {L >> 10} KiB x {S}"}
    P = _lib.probe_lib()
    stream = torch.cuda.current_stream().cuda_stream
    nbytes = 12 * L * S
    hsrc = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    hsrc.fill_(0x3C)
    hdst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for t in (hsrc, hdst):
        if device_pointer(t) != t.data_ptr():
            raise SystemExit(f"pinned buffer not mapped at its host address: {device_pointer(t)} != {t.data_ptr()}")

    def pcopy(src, dst, sched=2, depth=8, nt=1, blk=1024, bpc=1):
        st = P.hrs_probe_stream(0, src.data_ptr(), dst.data_ptr(), nbytes, sched, depth, nt, blk, bpc, stream)
        assert st == 0, st

    for name, a, b in (("link_read", hsrc, dbuf), ("link_write", dbuf, hdst), ("link_both", hsrc, hdst)):
        best = None
        for shape in ((2, 8, 1, 1024, 1), (2, 8, 0, 1024, 1), (1, 4, 0, 256, 2), (0, 4, 0, 256, 4)):
            ms = timed(lambda: pcopy(a, b, *shape), reps)
            if best is None or ms < best[0]:
                best = (ms, shape)
        res[name + "_ms"] = best[0]
        res[name + "_GBps"] = round(nbytes / 1e9 / (best[0] * 1e-3), 2)
        res[name + "_shape"] = list(best[1])
    assert bool((hdst[:: 1 << 16] == 0x3C).all()) and bool((dbuf[:: 1 << 16] == 0x3C).all())
    res["dma_h2d_ms"] = timed(lambda: dbuf.copy_(hsrc, non_blocking=True), reps)
    res["dma_h2d_GBps"] = round(nbytes / 1e9 / (res["dma_h2d_ms"] * 1e-3), 2)
    del hsrc, hdst, dbuf

    code = HipReedSolomonCode(k, p, device=0)
    st_dev = torch.zeros((S, n, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, st_dev, 5, 0, k, p)
    device.encode_stripes(code, st_dev)
    ref = st_dev.cpu()
    host = torch.empty((S, n, L), dtype=torch.uint8, pin_memory=True)
    host.copy_(ref)
    host[:, :p] = 0
    out = torch.empty((S, 2, L), dtype=torch.uint8, pin_memory=True)
    for t in (host, out):
        if device_pointer(t) != t.data_ptr():
            raise SystemExit("pinned stripes not mapped at their host address")
    # encode with the kernel reading / writing the pinned host stripes
    stride = n * L
    ins = ptr_array([host[0, p + c].data_ptr() for c in range(k)])
    outs = ptr_array([host[0, r].data_ptr() for r in range(p)])

    def enc_zero_copy():
        code._check(_lib.lib().hrs_encode_dev(code._handle(), ins, stride, outs, stride, L, S, stream))

    host[:, :p] = 0
    res["encode_zero_copy_ms"] = timed(enc_zero_copy, reps)
    res["encode_zero_copy_kernel"] = code.lastKernel()
    res["encode_zero_copy_ok"] = bool(torch.equal(host, ref))
    hn = host.numpy()
    host[:, :p] = 0
    res["encode_batch_host_ms"] = timed(lambda: device.encode_batch_host(code, hn), reps)
    res["encode_batch_host_ok"] = bool(torch.equal(host, ref))
    # repairs of config 5's seeded lost pairs, one batch launch over host memory
    er = np.array([np.sort(np.random.default_rng([0x5EED0005, s]).choice(n, 2, replace=False)) for s in range(S)],
                  dtype=np.int32)
    want = ref.numpy()[np.arange(S)[:, None], er]

    def rep_zero_copy():
        code._check(_lib.lib().hrs_decode_batch_dev(
            code._handle(), host.data_ptr(), host.stride(1), host.stride(0), er.ctypes.data, 2, out.data_ptr(),
            out.stride(1), out.stride(0), L, S, stream))

    out.zero_()
    res["repair_zero_copy_ms"] = timed(rep_zero_copy, reps)
    res["repair_zero_copy_kernel"] = code.lastKernel()
    res["repair_zero_copy_ok"] = bool(np.array_equal(out.numpy(), want))
    out.zero_()
    on = out.numpy()
    res["repair_batch_host_ms"] = timed(lambda: device.decode_batch_host(code, hn, er, on), reps)
    res["repair_batch_host_ok"] = bool(np.array_equal(on, want))
    user = k * L * S
    for key in ("encode_zero_copy", "encode_batch_host", "repair_zero_copy", "repair_batch_host"):
        res[key + "_GiBps_user"] = round(user / GiB / (res[key + "_ms"] * 1e-3), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
