"""Could a PAGEABLE host batch (hrs_decode_batch_host / hrs_encode_batch_host
over ordinary memory) run at the pinned rate by registering its pages with
HIP for the call, as the synchronous calls do (hrs_hostpath.cpp
host_apply_direct)? Config 5's shape: RS(12,4), 256 KiB cells, 512 stripes
(2 GiB of stripes), a random lost pair per stripe.

Per repetition, in one process: the staged pageable call (the product's
current path), then hipHostRegister of the stripes and output buffers + the
same call (now zero copy: the buffers count as pinned) + hipHostUnregister,
timing registration, call and unregistration apart. Outputs are compared with
the staged call's. One JSON line.
Usage: python tools/register_batch_probe.py [stripes] [reps]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lambdafs_amd import HipReedSolomonCode, device  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    k, p, L = 12, 4, 256 << 10
    n = k + p
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    code = HipReedSolomonCode(k, p, device=0)
    # page-aligned pageable buffers (np.empty of this size is an mmap; align by hand anyway)
    raw = np.empty(S * n * L + 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    st = raw[off:off + S * n * L].reshape(S, n, L)
    st[:] = (np.arange(L, dtype=np.uint32) * 2654435761 >> 13).astype(np.uint8)[None, None, :]
    st ^= np.arange(S * n, dtype=np.uint8).reshape(S, n, 1)
    er = np.array([np.sort(np.random.default_rng([5, g]).choice(n, 2, replace=False)) for g in range(S)], np.int32)
    oraw = np.empty(S * 2 * L + 4096, np.uint8)
    ooff = (-oraw.ctypes.data) % 4096
    out = oraw[ooff:ooff + S * 2 * L].reshape(S, 2, L)
    ref = np.empty_like(out)
    res = {"what": __doc__.split("\n")[0], "stripes": S, "L": L, "bytes_registered": st.nbytes + out.nbytes,
           "staged_ms": [], "register_ms": [], "call_ms": [], "unregister_ms": [], "ok": True}
    device.decode_batch_host(code, st, er, ref)  # warm
    for _ in range(reps):
        out[:] = 0
        t0 = time.perf_counter()
        device.decode_batch_host(code, st, er, out)
        res["staged_ms"].append((time.perf_counter() - t0) * 1e3)
        res["ok"] &= bool(np.array_equal(out, ref))
        out[:] = 0
        t0 = time.perf_counter()
        e1 = hip.hipHostRegister(st.ctypes.data, st.nbytes, 2)  # hipHostRegisterMapped
        e2 = hip.hipHostRegister(out.ctypes.data, out.nbytes, 2)
        t1 = time.perf_counter()
        if e1 or e2:
            res["register_error"] = [e1, e2]
            res["ok"] = False
            break
        device.decode_batch_host(code, st, er, out)
        t2 = time.perf_counter()
        hip.hipHostUnregister(st.ctypes.data)
        hip.hipHostUnregister(out.ctypes.data)
        t3 = time.perf_counter()
        res["register_ms"].append((t1 - t0) * 1e3)
        res["call_ms"].append((t2 - t1) * 1e3)
        res["unregister_ms"].append((t3 - t2) * 1e3)
        res["ok"] &= bool(np.array_equal(out, ref))
    for key in ("staged_ms", "register_ms", "call_ms", "unregister_ms"):
        res[key] = [round(x, 3) for x in res[key]]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
