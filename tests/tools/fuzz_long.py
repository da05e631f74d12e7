"""Long runs of the seeded differential fuzz suites (tests/test_gpu_fuzz.py,
tests/test_host_memory.py::test_host_call_fuzz) with other seeds and more cases
than the default `-m gpu` run affords: a bug hunt, not a test. Each seed is
one call of the suite's own test function, so a failure names its case.
Usage: python tests/tools/fuzz_long.py [seeds] [cases] (one JSON line per seed)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import test_gpu_fuzz as F  # noqa: E402
import test_host_memory as D  # noqa: E402


def main():
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cases = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    if "--no-thp" in sys.argv:  # numpy stops madvise(MADV_HUGEPAGE) on its large arrays
        import numpy._core.multiarray as ma
        ma._set_madvise_hugepage(False)
    if "--local-mempolicy" in sys.argv:
        # MPOL_LOCAL for the whole process: with an explicit policy (no
        # MPOL_F_NUMA_BALANCING) the kernel's NUMA balancing leaves its pages alone
        import ctypes
        libc = ctypes.CDLL(None, use_errno=True)
        if libc.syscall(238, 4, None, 0) != 0:  # SYS_set_mempolicy, MPOL_LOCAL
            raise SystemExit(f"set_mempolicy failed: errno {ctypes.get_errno()}")
    if not torch.cuda.is_available():
        raise SystemExit("no HIP device")
    F.CASES = cases
    for i in range(seeds):
        F.SEED = 0x5EED_F100 + 7919 * i
        t0 = time.time()
        F.test_differential_fuzz(torch)
        print(json.dumps({"suite": "test_gpu_fuzz", "seed": F.SEED, "cases": cases, "ok": True,
                          "s": round(time.time() - t0, 1)}), flush=True)
        D.FUZZ_SEED, D.FUZZ_CASES = 0xD1EC7 + 104729 * (i + 1), max(40, cases // 10)
        t0 = time.time()
        D.test_host_call_fuzz(torch)
        print(json.dumps({"suite": "test_host_memory.test_host_call_fuzz", "seed": D.FUZZ_SEED,
                          "cases": D.FUZZ_CASES, "ok": True, "s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
