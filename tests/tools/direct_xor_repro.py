"""Debug aid: XOR(3) decode of the parity over rows sharing pages (48-byte
gaps) through the direct path, for every 16-byte start offset within a page;
prints the offsets whose repaired row differs from the oracle and where the
first difference lies (head / middle / tail columns)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from lambdafs_amd import HipXORCode  # noqa: E402
from oracle import rs_oracle as C  # noqa: E402


def main():
    k, p, L, gap = 3, 1, 1 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 48
    n = k + p
    bad = 0
    for step in range(256):
        code = HipXORCode(k, 1)
        code.zero_inputs_after_encode = False
        nbuf = 2 * n + 2
        buf = np.random.default_rng(step).integers(0, 256, nbuf * (L + gap) + 8192, dtype=np.uint8)
        start = (-buf.ctypes.data) % 4096 + 16 * step
        rows = [buf[start + i * (L + gap): start + i * (L + gap) + L] for i in range(nbuf)]
        reads = [np.zeros(L, np.uint8)] + rows[1:n]
        outs = rows[n:n + 1]
        want = C.xor_decode_bulk(k, [np.array(r) for r in reads], 0)
        code.decodeBulk(reads, outs, [0], [x for x in range(1, n)], [0])
        path = code.lastHostPath()
        diff = np.flatnonzero(outs[0] != want)
        if diff.size:
            bad += 1
            offs = [(rows[i].ctypes.data % 4096) for i in range(1, n + 1)]
            print(f"start%4096={(buf.ctypes.data + start) % 4096} path={path} row offsets={offs} "
                  f"ndiff={diff.size} first={diff[0]} last={diff[-1]}", flush=True)
        code.close()
    print(f"bad offsets: {bad} of 256", flush=True)


if __name__ == "__main__":
    main()
