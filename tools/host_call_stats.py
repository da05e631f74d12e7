"""Per-call time distribution of the synchronous host-buffer calls from
Python (ctypes), the shape of bench.py's host_calls leg: RS(10,4), one stripe
of 1 MiB pageable rows per call. Prints one JSON line with mean / median /
p90 per call kind, so a mean inflated by a few slow calls shows as such.
Usage: python tools/host_call_stats.py [calls] [label]"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from lambdafs_amd import _lib  # noqa: E402
from lambdafs_amd._lib import ptr_array  # noqa: E402
from lambdafs_amd.erasure_code import HipReedSolomonCode  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    label = sys.argv[2] if len(sys.argv) > 2 else ""
    import ctypes
    k, p, L = 10, 4, 1 << 20
    code = HipReedSolomonCode(k, p, device=0, zero_inputs_after_encode=False)
    rng = np.random.default_rng(0x5EED000A)
    rows = [np.zeros(L, np.uint8) for _ in range(p)] + [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    h = code._handle()
    lib = _lib.lib()
    ins, outs = ptr_array([r.ctypes.data for r in rows[p:]]), ptr_array([r.ctypes.data for r in rows[:p]])
    crc = (ctypes.c_uint32 * (k + p))()
    res = {"label": label, "calls": calls}
    for name, fn in (("encodeBulk", lambda: lib.hrs_encode(h, ins, outs, L)),
                     ("encodeBulkCrc", lambda: lib.hrs_encode_crc(h, ins, outs, L, None, crc))):
        for _ in range(5):
            code._check(fn())
        t = np.empty(calls)
        for i in range(calls):
            t0 = time.perf_counter()
            code._check(fn())
            t[i] = time.perf_counter() - t0
        t *= 1e3
        res[name] = {"mean": round(float(t.mean()), 4), "median": round(float(np.median(t)), 4),
                     "p90": round(float(np.percentile(t, 90)), 4), "min": round(float(t.min()), 4),
                     "path": code.lastHostPath()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
