"""Debug aid: synchronous (staged) calls over a FRESH buffer each iteration,
the previous one freed first (numpy -> munmap), so a new buffer often lands
at the same virtual addresses as the last one, now backed by other physical
pages. Checks every call against the oracle and reports address reuse and
mismatches. Usage: python tests/tools/fresh_buffer_repro.py [iters] [gap]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from lambdafs_amd import HipReedSolomonCode, HipXORCode  # noqa: E402
from oracle import rs_oracle as C  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    gap = int(sys.argv[2]) if len(sys.argv) > 2 else 48
    L = 1 << 20
    seen, reused, bad = set(), 0, 0
    for it in range(iters):
        xor = it % 2 == 1
        k, p = (3, 1) if xor else (10, 4)
        n = k + p
        code = HipXORCode(k, 1) if xor else HipReedSolomonCode(k, p)
        code.zero_inputs_after_encode = False
        nbuf = 2 * n + 2
        buf = np.random.default_rng(it).integers(0, 256, nbuf * (L + gap) + 8192, dtype=np.uint8)
        base = buf.ctypes.data
        reused += base in seen
        seen.add(base)
        start = (-base) % 4096 + 16 * (it % 256)
        rows = [buf[start + i * (L + gap): start + i * (L + gap) + L] for i in range(nbuf)]
        data, par = rows[p:n], rows[:p]
        ref = [C.xor_encode_bulk(k, [np.array(d) for d in data])] if xor else C.encode_bulk(k, p, [np.array(d) for d in data])
        code.encodeBulk(data, par)
        ep = code.lastHostPath()
        e_ok = all(np.array_equal(par[o], ref[o]) for o in range(p))
        for r in rows[:p]:
            r[:] = np.random.default_rng(it + 1000).integers(0, 256, L, dtype=np.uint8)
        if xor:
            reads = [np.zeros(L, np.uint8)] + rows[1:n]
            want = C.xor_decode_bulk(k, [np.array(r) for r in reads], 0)
            erased, tr, ntr = [0], list(range(1, n)), [0]
        else:
            erased = [p]
            tr = sorted(C.locations_to_read(k, p, erased))
            ntr = [x for x in range(n) if x not in tr]
            reads = [rows[x] if x in tr else None for x in range(n)]
            want = C.decode_bulk5(k, p, [np.zeros(L, np.uint8) if r is None else np.array(r) for r in reads],
                                  erased, tr, ntr)[0]
        outs = rows[n:n + 1]
        code.decodeBulk(reads, outs, erased, tr, ntr)
        dp = code.lastHostPath()
        diff = np.flatnonzero(outs[0] != want)
        if not e_ok or diff.size:
            bad += 1
            print(f"iter {it} {'xor' if xor else 'rs'} base reused={base in seen} encode ok={e_ok} ({ep}) "
                  f"decode ndiff={diff.size} ({dp}) first={diff[0] if diff.size else -1}", flush=True)
        code.close()
        del buf, rows, data, par, outs, reads
    print(f"iterations {iters}, base address reused {reused}, bad {bad}", flush=True)


if __name__ == "__main__":
    main()
