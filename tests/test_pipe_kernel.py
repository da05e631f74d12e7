"""bitsliced_pipe_kernel (hrs_kernels.hip): the software-pipelined runtime
kernel that serves 1- and 2-output applies of <= 12 inputs (the 1- and
2-erasure repairs of ReedSolomonCode.decodeBulk, ReedSolomonCode.java:191-211).

GPU only. Each wave holds two register sets and alternates between them, so
the cases here make the per-wave task count uneven (more tasks than waves,
not a multiple of the wave count, 1 task for some waves and 4 for others),
add row tails (len mod 2 KiB, bytewise kernel) and go through the host's
input chunking (nin > 16: the last chunk runs with accumulate = 1). Checked
byte for byte against GF(2^8) products from the oracle's multiply
(GaloisField.java:148-160).
"""
import numpy as np
import pytest
import torch

from lambdafs_amd import HipReedSolomonCode, device
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu

MUL = np.array([[C.gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)


def _reference(m, x):
    S, nin, L = x.shape
    ref = np.zeros((S, m.shape[0], L), np.uint8)
    for o in range(m.shape[0]):
        for i in range(nin):
            ref[:, o] ^= MUL[m[o, i]][x[:, i]]
    return ref


@pytest.mark.parametrize(
    "nout,nin,S,L",
    [
        (1, 10, 313, 7 * 2048),        # 2,191 tasks: some waves 1 task, some 2
        (1, 10, 700, 9 * 2048 + 96),   # 6,300 tasks + a 96-byte row tail
        (1, 12, 257, 16 * 2048),       # 4,112 tasks: 2 or 3 per wave
        (2, 12, 129, 33 * 2048),       # 2 outputs, 4,257 tasks
        (1, 5, 1000, 5 * 2048 + 16),   # NINB 8 instance, 16-byte tail
        (2, 3, 3, 2048),               # fewer tasks than waves
        (1, 20, 300, 8 * 2048),        # chunked 16 + 4: pipelined chunk accumulates
        (2, 17, 200, 8 * 2048),        # chunked 16 + 1
    ],
)
def test_pipe_apply_matches_gf_products(nout, nin, S, L):
    code = HipReedSolomonCode(10, 4)
    rng = np.random.default_rng(nout * 1000 + nin * 10 + S)
    m = rng.integers(1, 256, (nout, nin), dtype=np.uint8)
    g = torch.Generator(device="cuda")
    g.manual_seed(S + L)
    x = torch.randint(0, 256, (S, nin, L), dtype=torch.uint8, device="cuda", generator=g)
    y = torch.full((S, nout, L), 0xA5, dtype=torch.uint8, device="cuda")
    device.apply_rows(code, m, [x[:, i] for i in range(nin)], [y[:, o] for o in range(nout)])
    torch.cuda.synchronize()
    ref = _reference(m, x.cpu().numpy())
    got = y.cpu().numpy()
    assert np.array_equal(got, ref), [
        (o, int(np.argmax((got[:, o] != ref[:, o]).reshape(-1)))) for o in range(nout) if not np.array_equal(got[:, o], ref[:, o])
    ]


def test_pipe_decode_uneven_batch_round_trip():
    """RS(10,4) repair of data shard 0 over a stripe count that leaves waves
    with uneven task counts; the repaired cells must equal the originals."""
    k, p = 10, 4
    code = HipReedSolomonCode(k, p)
    S, L = 517, 3 * 2048 + 48
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda", generator=g)
    device.encode_stripes(code, st)
    erased = [p]
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(k + p) if x not in to_read]
    out = torch.empty((S, 1, L), dtype=torch.uint8, device="cuda")
    device.decode_stripes(code, st, erased, ntr, out)
    torch.cuda.synchronize()
    assert torch.equal(out[:, 0], st[:, p])
