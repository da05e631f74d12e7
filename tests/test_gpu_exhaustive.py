"""Exhaustive and extreme-size parity on the GPU (through the C ABI).

- every erasure pattern of RS(10,4) with 1..4 erasures (1,470 patterns), each
  decoded on the GPU from the survivors `locationsToReadForDecode` picks, on a
  batch of codewords (round trip) — and the decode matrices of all of them
  checked against the oracle's reference loops on CPU (tests/test_abi.py
  covers 1-2 erasures; here all 4 levels);
- wide codes: RS(100,10) and the maximum RS(245,10) (k + p = 255 < 256,
  ReedSolomonCode.java:57), exercising the host's input/output chunking;
- decodes with more than 8 erased rows (output chunking);
- every 1..p erasure pattern of each BASELINE shape (RS(3,2), RS(6,3),
  RS(10,4), RS(12,4): 30 / 129 / 1,470 / 2,516 patterns) as ONE heterogeneous
  batch launch (hrs_decode_batch_dev, a different pattern per stripe) on
  NON-codeword stripes, every stripe vs the oracle's per-byte decodeBulk
  5-arg (ReedSolomonCode.java:191-211) with the Decoder's zero rows for the
  unread locations (StripeReader.java:106-124).
"""
import itertools
import random

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, device
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu


def test_all_rs104_erasure_patterns_round_trip(cuda):
    torch = cuda
    k, p, L, S = 10, 4, 4096 + 96, 4
    n = k + p
    code = HipReedSolomonCode(k, p)
    g = torch.Generator(device="cuda")
    g.manual_seed(104)
    st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)
    device.encode_stripes(code, st)
    count = 0
    for e in range(1, p + 1):
        for erased in itertools.combinations(range(n), e):
            erased = list(erased)
            to_read = sorted(code.locationsToReadForDecode(erased))
            ntr = [x for x in range(n) if x not in to_read]
            out = torch.empty((S, e, L), dtype=torch.uint8, device="cuda")
            device.decode_stripes(code, st, erased, ntr, out)
            assert torch.equal(out, st[:, erased, :]), erased
            count += 1
    assert count == 14 + 91 + 364 + 1001


def test_rs104_decode_matrices_all_patterns_vs_oracle_sampled_columns(cuda):
    # every pattern's matrix against the oracle's per-byte decode on random
    # (non-codeword) stripes: 3 random columns per pattern keep it fast
    k, p = 10, 4
    n = k + p
    code = HipReedSolomonCode(k, p)
    rng = np.random.default_rng(7)
    for e in range(3, p + 1):
        for erased in itertools.combinations(range(n), e):
            erased = list(erased)
            to_read = sorted(C.locations_to_read(k, p, erased))
            ntr = [x for x in range(n) if x not in to_read]
            D = code.decodeMatrix(erased, ntr)
            cols = rng.integers(0, 256, (3, n)).tolist()
            for col in cols:
                data = [0 if i in ntr else v for i, v in enumerate(col)]
                ref = C.decode5(k, p, list(data), erased, to_read, ntr)
                got = [0] * e
                for t in range(e):
                    acc = 0
                    for l_ in range(n):
                        acc ^= C.gf_mul(int(D[t, l_]), data[l_])
                    got[t] = acc
                assert got == ref, erased


@pytest.mark.parametrize("k,p", [(100, 10), (245, 10), (30, 20)])
def test_wide_codes_encode_and_decode(cuda, k, p):
    torch = cuda
    n = k + p
    L, S = 2048 * 3 + 5, 2
    code = HipReedSolomonCode(k, p)
    g = torch.Generator(device="cuda")
    g.manual_seed(k)
    st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)
    device.encode_stripes(code, st)
    host = st.cpu().numpy()
    ref = np.stack(C.encode_bulk(k, p, [host[0, p + c] for c in range(k)]))
    assert (host[0, :p] == ref).all()
    rnd = random.Random(k)
    for e in (1, p // 2, p):
        erased = sorted(rnd.sample(range(n), e))
        to_read = sorted(code.locationsToReadForDecode(erased))
        ntr = [x for x in range(n) if x not in to_read]
        out = torch.empty((S, e, L), dtype=torch.uint8, device="cuda")
        device.decode_stripes(code, st, erased, ntr, out)
        assert torch.equal(out, st[:, erased, :]), (k, p, erased)


@pytest.mark.parametrize("k,p", [(3, 2), (6, 3), (10, 4), (12, 4)])
def test_every_pattern_in_one_batch_vs_oracle(cuda, k, p):
    torch = cuda
    n, L = k + p, 2048 + 48  # one fused window and a ragged tail
    pats = [list(e) for m in range(1, p + 1) for e in itertools.combinations(range(n), m)]
    S = len(pats)
    er = np.full((S, p), -1, dtype=np.int32)
    for s, e in enumerate(pats):
        er[s, :len(e)] = e
    g = torch.Generator(device="cuda")
    g.manual_seed(k * 100 + p)
    st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)  # non-codewords
    out = torch.full((S, p, L), 0xEE, dtype=torch.uint8, device="cuda")
    code = HipReedSolomonCode(k, p)
    device.decode_batch(code, st, er, out)
    host, got = st.cpu().numpy(), out.cpu().numpy()
    for s, erased in enumerate(pats):
        to_read = sorted(C.locations_to_read(k, p, erased))
        ntr = [x for x in range(n) if x not in to_read or x in erased]
        reads = [np.zeros(L, np.uint8) if x in ntr else host[s, x] for x in range(n)]
        ref = C.decode_bulk5(k, p, reads, erased, to_read, ntr)
        for j in range(len(erased)):
            assert np.array_equal(got[s, j], ref[j]), (erased, j)
