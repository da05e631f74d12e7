"""The `nrs` codec (NativeReedSolomonCode.java over libhadoop's ISA-L shim,
erasure_coder.c) behind the same boundary.

Parity status: UNPINNED. ISA-L is a third-party library absent from
/root/reference (libhadoop links it at build time; no version is pinned in the
tree), and no JDK is here to run the Java, so the oracle
(oracle/rs_oracle.c, orc_nrs_*) restates ISA-L's published
gf_gen_cauchy1_matrix / gf_invert_matrix / ec_encode_data over GF(2^8)/0x11D
and transcribes the shim (erasure_coder.c:102-230) and the Java's hops<->Apache
remapping (NativeReedSolomonCode.java:90-152). The reference's own test,
TestNativeErasureCodes.testNativeEncodeDecode (RS(10,4), 4 data units lost,
1 KiB cells, round trip), is mirrored below on both the oracle and the GPU.

CPU: the product's matrices against the oracle on every RS(10,4)
not-to-read pattern, the ordering quirk, argument rules. GPU (-m gpu):
encodeBulk / decodeBulk bit-exact against the oracle through host and device
rows, every RS(10,4) pattern round-tripped on device batches, wide codes.
"""
import itertools
import random

import numpy as np
import pytest

from lambdafs_amd import Codec, HipNativeReedSolomonCode, HrsError, device
from lambdafs_amd import codec as codec_mod
from oracle import rs_oracle as C

NONE = -2


def _mul_table():
    t = np.zeros((256, 256), dtype=np.uint8)
    for a in range(256):
        for b in range(a, 256):
            t[a, b] = t[b, a] = C.gf_mul(a, b)
    return t


MUL = _mul_table()


def _apply(D, rows):
    """out_t = XOR_l D[t, l] * rows[l] (host numpy, rows None -> unused)."""
    out = []
    for t in range(D.shape[0]):
        acc = np.zeros_like(next(r for r in rows if r is not None))
        for l_, r in enumerate(rows):
            if D[t, l_]:
                acc ^= MUL[D[t, l_]][r]
        out.append(acc)
    return out


def _apache_sorted(k, p, ntr):
    return sorted(loc + k if loc < p else loc - p for loc in ntr)


def _hops(k, p, a):
    return a + p if a < k else a - k


@pytest.mark.parametrize("k,p", [(10, 4), (6, 3), (3, 2), (1, 1), (20, 8), (100, 10), (245, 10)])
def test_nrs_encode_matrix_matches_oracle(k, p):
    code = HipNativeReedSolomonCode(k, p, device=NONE)
    G = code.encodeMatrix()
    A = C.nrs_encode_matrix(k, p)
    assert (A[:k] == np.eye(k, dtype=np.uint8)).all()
    assert (G == A[k:]).all()
    rng = np.random.default_rng(k)
    data = [rng.integers(0, 256, 33, dtype=np.uint8) for _ in range(k)]
    par = C.nrs_encode_bulk(k, p, data)
    for r, x in enumerate(_apply(G, data)):
        assert (x == par[r]).all()


def test_oracle_native_encode_decode_round_trip():
    # TestNativeErasureCodes.testNativeEncodeDecode on the oracle: RS(10,4),
    # 1 KiB cells, four data units unavailable
    k, p, L = 10, 4, 1024
    rng = np.random.default_rng(1)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    stripe = C.nrs_encode_bulk(k, p, data) + data
    erased = [p + 0, p + 2, p + 5, p + 9]
    reads = [None if i in erased else stripe[i] for i in range(k + p)]
    out = C.nrs_decode_bulk(k, p, reads, erased, erased)
    for o, e in zip(out, erased):
        assert (o == stripe[e]).all()


@pytest.mark.parametrize("k,p", [(10, 4), (6, 3)])
def test_nrs_decode_matrices_every_pattern_vs_oracle(k, p):
    # every not-to-read set of size 1..p, erased = the not-to-read set (hops
    # order); random (non-codeword) rows so every coefficient is exercised
    n = k + p
    code = HipNativeReedSolomonCode(k, p, device=NONE)
    rng = np.random.default_rng(n)
    rows = [rng.integers(0, 256, 24, dtype=np.uint8) for _ in range(n)]
    count = 0
    for m in range(1, p + 1):
        for ntr in itertools.combinations(range(n), m):
            ntr = list(ntr)
            erased = list(ntr)
            D = code.decodeMatrix(erased, ntr)
            assert not D[:, ntr].any()
            reads = [None if i in ntr else rows[i] for i in range(n)]
            ref = C.nrs_decode_bulk(k, p, reads, erased, ntr)
            for got, want in zip(_apply(D, reads), ref):
                assert (got == want).all(), ntr
            count += 1
    assert count == sum(len(list(itertools.combinations(range(n), m))) for m in range(1, p + 1))


def test_nrs_output_order_quirk():
    # Erasing hops parity 2 alone: locationsToReadForDecode keeps the k
    # highest locations, so not-to-read = parity 0..3, Apache [10..13]; the
    # Java hands writeBufs[0] the first of those -> parity 0, not parity 2.
    k, p = 10, 4
    code = HipNativeReedSolomonCode(k, p, device=NONE)
    erased = [2]
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(k + p) if x not in to_read]
    assert ntr == [0, 1, 2, 3]
    D = code.decodeMatrix(erased, ntr)
    G = code.encodeMatrix()
    assert (D[0, p:] == G[0]).all() and not D[0, :p].any()
    rng = np.random.default_rng(2)
    data = [rng.integers(0, 256, 64, dtype=np.uint8) for _ in range(k)]
    stripe = C.nrs_encode_bulk(k, p, data) + data
    out = C.nrs_decode_bulk(k, p, [None if i in ntr else stripe[i] for i in range(k + p)], erased, ntr)
    assert (out[0] == stripe[0]).all() and not (out[0] == stripe[2]).all()
    # apache-sorted order decides: not-to-read [13, 5] -> data 1 (Apache 1) first
    D2 = code.decodeMatrix([13, 5], [13, 5])
    assert [_hops(k, p, a) for a in _apache_sorted(k, p, [13, 5])] == [5, 13]
    assert D2.shape == (2, k + p)


def test_nrs_rules():
    code = HipNativeReedSolomonCode(10, 4, device=NONE)
    with pytest.raises(HrsError):
        code.decodeMatrix([0], [0, 1, 2, 3, 4])  # fewer than k survivors
    with pytest.raises(HrsError):
        code.decodeMatrix([0, 1], [0])  # more outputs than not-to-read buffers
    with pytest.raises(HrsError):
        code.decodeMatrix([0], [0, 0])
    with pytest.raises(HrsError):
        code.decodeMatrix([0], [14])
    with pytest.raises(NotImplementedError):
        code.encode([0] * 10, [0] * 4)
    with pytest.raises(NotImplementedError):
        code.decode([0] * 14, [0], [0])
    with pytest.raises(NotImplementedError):
        code.symbolSize()
    with pytest.raises(NotImplementedError):
        code.decodeBulk([np.zeros(4, np.uint8)] * 14, [np.zeros(4, np.uint8)], [0])
    with pytest.raises(IndexError):
        code.decodeBulk([np.zeros(4, np.uint8)] * 14, [np.zeros(4, np.uint8)] * 2, [0, 1], [], [0])
    assert code.stripeSize() == 10 and code.paritySize() == 4


def test_nrs_codec_registry_resolves_class():
    conf = {codec_mod.ERASURE_CODING_CODECS_KEY: codec_mod.DEFAULT_CODECS_JSON}
    Codec.initializeCodecs(conf)
    c = Codec.getCodec("nrs")
    assert (c.stripeLength, c.parityLength) == (10, 4)
    assert codec_mod.ERASURE_CODE_CLASSES[HipNativeReedSolomonCode.JAVA_CLASS] is HipNativeReedSolomonCode
    with pytest.raises(codec_mod.ClassNotFoundException):
        c.createErasureCode(conf)  # the JSON's NativeReedSolomonCode is not this engine's class


# ---------------------------------------------------------------- GPU parity

@pytest.mark.gpu
def test_native_encode_decode_host_rows(cuda):
    # TestNativeErasureCodes.testNativeEncodeDecode through the product
    k, p, L = 10, 4, 1024
    code = HipNativeReedSolomonCode(k, p)
    rng = np.random.default_rng(3)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    keep = [d.copy() for d in data]
    parity = [np.zeros(L, np.uint8) for _ in range(p)]
    code.encodeBulk(data, parity)
    assert all((a == b).all() for a, b in zip(data, keep))  # inputs untouched (copied to direct buffers)
    ref = C.nrs_encode_bulk(k, p, data)
    assert all((a == b).all() for a, b in zip(parity, ref))
    stripe = parity + data
    erased = [p + 0, p + 2, p + 5, p + 9]
    reads = [None if i in erased else stripe[i] for i in range(k + p)]
    out = [np.zeros(L, np.uint8) for _ in erased]
    code.decodeBulk(reads, out, erased, [i for i in range(k + p) if i not in erased], erased)
    for o, e in zip(out, erased):
        assert (o == stripe[e]).all()
    # the parity-2 quirk through the product
    ntr = [0, 1, 2, 3]
    out = [np.zeros(L, np.uint8)]
    code.decodeBulk([None if i in ntr else stripe[i] for i in range(k + p)], out, [2], list(range(4, 14)), ntr)
    assert (out[0] == stripe[0]).all()


@pytest.mark.gpu
def test_nrs_every_rs104_pattern_round_trip_device(cuda):
    torch = cuda
    k, p, L, S = 10, 4, 4096 + 96, 3
    n = k + p
    code = HipNativeReedSolomonCode(k, p)
    g = torch.Generator(device="cuda")
    g.manual_seed(1014)
    st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)
    device.encode_stripes(code, st)
    host = st.cpu().numpy()
    ref = C.nrs_encode_bulk(k, p, [host[0, p + c] for c in range(k)])
    assert all((host[0, r] == ref[r]).all() for r in range(p))
    count = 0
    for m in range(1, p + 1):
        for ntr in itertools.combinations(range(n), m):
            order = [_hops(k, p, a) for a in _apache_sorted(k, p, ntr)]
            out = torch.empty((S, m, L), dtype=torch.uint8, device="cuda")
            device.decode_stripes(code, st, order, list(ntr), out)
            assert torch.equal(out, st[:, order, :]), ntr
            count += 1
    assert count == 1470


@pytest.mark.gpu
@pytest.mark.parametrize("k,p", [(10, 4), (6, 3), (20, 8), (100, 10)])
def test_nrs_random_rows_vs_oracle_device(cuda, k, p):
    # non-codeword rows, ragged lengths (bit-sliced body + byte tail)
    torch = cuda
    n = k + p
    code = HipNativeReedSolomonCode(k, p)
    rnd = random.Random(k * 7 + p)
    for L in (1, 777, 2048 * 2 + 13):
        g = torch.Generator(device="cuda")
        g.manual_seed(L + k)
        st = torch.randint(0, 256, (2, n, L), dtype=torch.uint8, device="cuda", generator=g)
        host = st.cpu().numpy()
        par = torch.empty((2, p, L), dtype=torch.uint8, device="cuda")
        device.encode_rows(code, [st[:, p + c, :] for c in range(k)], [par[:, r, :] for r in range(p)])
        ref = C.nrs_encode_bulk(k, p, [host[1, p + c] for c in range(k)])
        assert (par[1].cpu().numpy() == np.stack(ref)).all()
        for m in sorted({1, p // 2 or 1, p}):
            ntr = sorted(rnd.sample(range(n), m))
            ne = rnd.randint(1, m)
            erased = ntr[:ne]
            out = torch.empty((2, ne, L), dtype=torch.uint8, device="cuda")
            device.decode_stripes(code, st, erased, ntr, out)
            want = C.nrs_decode_bulk(k, p, [None if i in ntr else host[1, i] for i in range(n)], erased, ntr)
            assert (out[1].cpu().numpy() == np.stack(want)).all(), (k, p, L, ntr, erased)
