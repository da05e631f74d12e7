"""hrs_decode_batch_dev: one launch repairs stripes that lost different
locations (a repair job over many stripes; Decoder.fixErasedBlockImpl per
stripe, Decoder.java:291-338). SURVEY §8(d) config 3's second run (a seeded
random lost location per stripe) goes through it.

GPU only: per-stripe round trips for RS (aligned rows, row tails, unaligned
rows), nrs (Apache output order), xor; equality with the single-pattern
hrs_decode_dev on non-codeword rows; wide codes (per-stripe fallback);
TooManyErasedLocations; back-to-back calls reusing the upload slots.
"""
import random

import numpy as np
import pytest

from lambdafs_amd import HipNativeReedSolomonCode, HipReedSolomonCode, HipXORCode, TooManyErasedLocations, device
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu


def _patterns(n, p, S, seed, max_e=None):
    rnd = random.Random(seed)
    E = max_e if max_e is not None else p
    er = np.full((S, E), -1, dtype=np.int32)
    for s in range(S):
        e = rnd.randint(0, E)
        er[s, :e] = sorted(rnd.sample(range(n), e))
    return er


def _stripes(torch, S, n, L, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)


@pytest.mark.parametrize("L", [4096, 2048 * 3 + 40, 1001, 7])
def test_rs_batch_round_trip(cuda, L):
    torch = cuda
    k, p, S = 10, 4, 96
    n = k + p
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, n, L, L)
    device.encode_stripes(code, st)
    er = _patterns(n, p, S, L)
    out = torch.full((S, p, L), 0xEE, dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    torch.cuda.synchronize()
    for s in range(S):
        lost = [int(x) for x in er[s] if x >= 0]
        if lost:
            assert torch.equal(out[s, :len(lost)], st[s, lost]), (s, lost)
        assert (out[s, len(lost):] == 0xEE).all()  # rows past a stripe's erasures untouched


def test_rs_batch_single_random_location(cuda):
    # config 3, second run: one seeded random lost location per stripe
    torch = cuda
    k, p, S, L = 10, 4, 256, 65536
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, k + p, L, 3)
    device.encode_stripes(code, st)
    rnd = random.Random(0x5EED0003)
    er = np.array([[rnd.randrange(k + p)] for _ in range(S)], dtype=np.int32)
    out = torch.empty((S, 1, L), dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    idx = torch.as_tensor(er[:, 0], dtype=torch.long, device="cuda")
    assert torch.equal(out[:, 0], st[torch.arange(S, device="cuda"), idx])


def test_batch_equals_single_pattern_decode_on_random_rows(cuda):
    # non-codeword rows: the batch applies exactly the per-pattern matrix
    torch = cuda
    k, p, S, L = 10, 4, 40, 2048 + 100
    n = k + p
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, n, L, 11)
    er = _patterns(n, p, S, 12)
    out = torch.zeros((S, p, L), dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    for s in range(S):
        lost = [int(x) for x in er[s] if x >= 0]
        if not lost:
            continue
        to_read = code.locationsToReadForDecode(lost)
        ntr = [x for x in range(n) if x not in to_read]
        ref = torch.empty((1, len(lost), L), dtype=torch.uint8, device="cuda")
        device.decode_stripes(code, st[s:s + 1], lost, ntr, ref)
        assert torch.equal(out[s, :len(lost)], ref[0]), (s, lost)


def test_nrs_batch_apache_order(cuda):
    torch = cuda
    k, p, S, L = 10, 4, 64, 4096 + 16
    n = k + p
    code = HipNativeReedSolomonCode(k, p)
    st = _stripes(torch, S, n, L, 21)
    device.encode_stripes(code, st)
    er = _patterns(n, p, S, 22)
    out = torch.empty((S, p, L), dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    for s in range(S):
        lost = [int(x) for x in er[s] if x >= 0]
        if not lost:
            continue
        to_read = code.locationsToReadForDecode(lost)
        ntr = [x for x in range(n) if x not in to_read]
        order = sorted(ntr, key=lambda loc: loc + k if loc < p else loc - p)[:len(lost)]
        assert torch.equal(out[s, :len(lost)], st[s, order]), (s, lost, order)


def test_xor_batch(cuda):
    torch = cuda
    k, S, L = 10, 50, 3000
    code = HipXORCode(k, 1)
    st = _stripes(torch, S, k + 1, L, 31)
    device.encode_stripes(code, st)
    er = _patterns(k + 1, 1, S, 32)
    out = torch.empty((S, 1, L), dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    for s in range(S):
        if er[s, 0] >= 0:
            assert torch.equal(out[s, 0], st[s, int(er[s, 0])])


def test_wide_code_batch_round_trip(cuda):
    torch = cuda
    k, p, S, L = 30, 6, 6, 2048 + 9
    n = k + p
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, n, L, 41)
    device.encode_stripes(code, st)
    er = _patterns(n, p, S, 42)
    out = torch.empty((S, p, L), dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    for s in range(S):
        lost = [int(x) for x in er[s] if x >= 0]
        if lost:
            assert torch.equal(out[s, :len(lost)], st[s, lost])


def test_batch_too_many_erased(cuda):
    torch = cuda
    code = HipReedSolomonCode(10, 4)
    st = _stripes(torch, 2, 14, 2048, 51)
    er = np.array([[0, -1, -1, -1, -1], [0, 1, 2, 3, 4]], dtype=np.int32)
    out = torch.empty((2, 5, 2048), dtype=torch.uint8, device="cuda")
    with pytest.raises(TooManyErasedLocations):
        device.decode_batch(code, st, er, out)


def test_batch_back_to_back_calls_reuse_slots(cuda):
    torch = cuda
    k, p, S, L = 6, 3, 128, 8192
    n = k + p
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, n, L, 61)
    device.encode_stripes(code, st)
    outs, ers = [], []
    for i in range(5):  # no sync in between: slots alternate, each waits for its last use
        er = _patterns(n, p, S, 100 + i)
        out = torch.empty((S, p, L), dtype=torch.uint8, device="cuda")
        device.decode_batch(code, st, er, out)
        outs.append(out)
        ers.append(er)
    torch.cuda.synchronize()
    for er, out in zip(ers, outs):
        for s in range(0, S, 7):
            lost = [int(x) for x in er[s] if x >= 0]
            if lost:
                assert torch.equal(out[s, :len(lost)], st[s, lost])


def test_wide_batches_stream_vs_oracle(cuda):
    """Patterns beyond the register-resident batch kernel (> 16 survivors, or
    > 8 with 6-8 outputs) take batch_stream_kernel in one launch; beyond 32
    survivors, one launch per stripe. Non-codeword rows: every coefficient
    of every pattern's matrix is checked against the oracle's decodeBulk."""
    torch = cuda
    rnd = np.random.default_rng(77)
    for k, p, S, L in [(20, 8, 12, 4096 + 48), (12, 6, 10, 2048), (40, 4, 3, 2048 + 16)]:
        n = k + p
        code = HipReedSolomonCode(k, p)
        st = _stripes(torch, S, n, L, 80 + k)
        er = np.full((S, p), -1, dtype=np.int32)
        for s in range(S):
            e = sorted(rnd.choice(n, size=int(rnd.integers(0, p + 1)), replace=False).tolist())
            er[s, :len(e)] = e
        out = torch.full((S, p, L), 0x5A, dtype=torch.uint8, device="cuda")
        device.decode_batch(code, st, er, out)
        host, got = st.cpu().numpy(), out.cpu().numpy()
        for s in range(S):
            lost = [int(x) for x in er[s] if x >= 0]
            if not lost:
                continue
            tr = sorted(C.locations_to_read(k, p, lost))
            ntr = [x for x in range(n) if x not in tr]
            reads = [host[s, x] if x in tr else np.zeros(L, np.uint8) for x in range(n)]
            ref = C.decode_bulk5(k, p, reads, lost, tr, ntr)
            assert all((got[s, j] == ref[j]).all() for j in range(len(lost))), (k, p, s, lost)
