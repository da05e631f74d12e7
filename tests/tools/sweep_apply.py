"""Sweep hrs_apply_dev over every (nout, nin) shape the runtime kernels take
(1..8 outputs x 1..20 inputs, incl. host chunking) against a numpy GF(2^8)
reference; prints failing shapes. Debug aid for the bit-sliced kernels."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lambdafs_amd import HipReedSolomonCode, device  # noqa: E402
from oracle import rs_oracle as C  # noqa: E402

MUL = np.array([[C.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)


def main():
    code = HipReedSolomonCode(10, 4)
    rng = np.random.default_rng(5)
    L, S = 2048 * 2, 2
    bad = []
    for nout in range(1, 9):
        for nin in range(1, 21):
            m = rng.integers(0, 256, (nout, nin), dtype=np.uint8)
            x = torch.randint(0, 256, (S, nin, L), dtype=torch.uint8, device="cuda")
            y = torch.empty((S, nout, L), dtype=torch.uint8, device="cuda")
            device.apply_rows(code, m, [x[:, i] for i in range(nin)], [y[:, o] for o in range(nout)])
            xh, yh = x.cpu().numpy(), y.cpu().numpy()
            ref = np.zeros((S, nout, L), np.uint8)
            for o in range(nout):
                for i in range(nin):
                    ref[:, o] ^= MUL[m[o, i]][xh[:, i]]
            if not (ref == yh).all():
                wrong = [o for o in range(nout) if not (ref[:, o] == yh[:, o]).all()]
                bad.append((nout, nin, wrong))
    print("variant", os.environ.get("HRS_RUNTIME_BRANCHY", "masked"), "failing (nout, nin, outputs):", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
