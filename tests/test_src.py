"""The `src` codec (SimpleRegeneratingCode.java:28-482) behind the same boundary.

Parity: the oracle (orc_src_* in oracle/rs_oracle.c) transcribes the Java
loop for loop (init's adjustment loop, groups, remainder encode, the three
decode cases, locationsToReadForDecode) over ErasureCode's default bulk loops;
the product builds the same maps as matrices (hrs_matrix.cpp: src_encode_matrix,
build_src_decode_matrix). The reference holds no SRC test or fixture, so the
pin is the transcription plus the round-trip property over every erasure
pattern (as for RS).

CPU: layout, encode matrices, locationsToReadForDecode and every decode
matrix of SRC(10,6,2) (all 1..6-erasure patterns, Decoder-style
not-to-read sets) against the oracle on non-codeword columns. GPU (-m gpu):
bulk and scalar calls vs the oracle, every decodable pattern round-tripped on
device batches, the heterogeneous batch decode, the codec registry.
"""
import itertools
import random

import numpy as np
import pytest

from lambdafs_amd import Codec, HipSimpleRegeneratingCode, TooManyErasedLocations, device
from lambdafs_amd import codec as codec_mod
from oracle import rs_oracle as C

NONE = -2
PARAMS = [(10, 6, 2), (10, 4, 3), (6, 3, 2), (12, 6, 3), (10, 6, 0), (5, 5, 5), (20, 8, 4)]


def _mul_table():
    t = np.zeros((256, 256), dtype=np.uint8)
    for a in range(256):
        for b in range(a, 256):
            t[a, b] = t[b, a] = C.gf_mul(a, b)
    return t


MUL = _mul_table()


def _apply(D, cols):
    """D (ne x n) applied to cols (n x C) over GF(2^8)."""
    out = np.zeros((D.shape[0], cols.shape[1]), dtype=np.uint8)
    for t in range(D.shape[0]):
        for l_ in range(D.shape[1]):
            if D[t, l_]:
                out[t] ^= MUL[D[t, l_]][cols[l_]]
    return out


def _decoder_sets(code, erased):
    """Decoder.java:303-338: ascending erased / toRead / notToRead arrays."""
    n = code.stripeSize() + code.paritySize()
    to_read = code.locationsToReadForDecode(erased)
    return sorted(erased), sorted(to_read), [x for x in range(n) if x not in to_read or x in erased]


@pytest.mark.parametrize("k,p,s", PARAMS)
def test_src_layout_and_encode_matrix_match_oracle(k, p, s):
    code = HipSimpleRegeneratingCode(k, p, s, device=NONE)
    assert code.srcLayout() == C.src_params(k, p, s)
    G = code.encodeMatrix()
    for c in range(k):
        unit = [1 if j == c else 0 for j in range(k)]
        assert list(G[:, c]) == C.src_encode(k, p, s, unit), c
    rng = np.random.default_rng(k * 100 + p * 10 + s)
    data = [rng.integers(0, 256, 40, dtype=np.uint8) for _ in range(k)]
    par = C.src_encode_bulk(k, p, s, data)
    assert (_apply(G, np.stack(data)) == np.stack(par)).all()


@pytest.mark.parametrize("k,p,s", [(10, 6, 2), (6, 3, 2), (10, 4, 3)])
def test_src_locations_and_decode_matrices_every_pattern(k, p, s):
    code = HipSimpleRegeneratingCode(k, p, s, device=NONE)
    n = k + p
    rng = np.random.default_rng(n + s)
    cols = rng.integers(0, 256, (n, 6), dtype=np.uint8)
    decodable = too_many = 0
    for e in range(1, p + 1):
        for erased in itertools.combinations(range(n), e):
            erased = list(erased)
            ref = C.src_locations_to_read(k, p, s, erased)
            if ref is None:
                with pytest.raises(TooManyErasedLocations):
                    code.locationsToReadForDecode(erased)
                too_many += 1
                continue
            assert code.locationsToReadForDecode(erased) == ref, erased
            er, tr, ntr = _decoder_sets(code, erased)
            D = code.decodeMatrix(er, ntr)
            reads = [None if x in ntr else cols[x] for x in range(n)]
            want = C.src_decode_bulk(k, p, s, [np.zeros(6, np.uint8) if r is None else r for r in reads], er, tr, ntr)
            assert want is not None
            assert (_apply(D, np.stack([np.zeros(6, np.uint8) if r is None else r for r in reads])) ==
                    np.stack(want)).all(), erased
            decodable += 1
    assert decodable > 0 and decodable + too_many == sum(
        len(list(itertools.combinations(range(n), e))) for e in range(1, p + 1))


def test_src_oracle_round_trip_every_pattern():
    k, p, s = 10, 6, 2
    n = k + p
    rng = np.random.default_rng(3)
    data = [rng.integers(0, 256, 24, dtype=np.uint8) for _ in range(k)]
    st = C.src_encode_bulk(k, p, s, data) + data
    count = 0
    for e in range(1, p + 1):
        for erased in itertools.combinations(range(n), e):
            erased = list(erased)
            tr = C.src_locations_to_read(k, p, s, erased)
            if tr is None:
                continue
            ntr = [x for x in range(n) if x not in tr or x in erased]
            reads = [np.zeros(24, np.uint8) if x in ntr else st[x] for x in range(n)]
            out = C.src_decode_bulk(k, p, s, reads, erased, sorted(tr), ntr)
            assert all((o == st[x]).all() for o, x in zip(out, erased)), erased
            count += 1
    assert count == 5883  # decodable SRC(10,6,2) patterns with 1..6 erasures


def test_src_rules():
    code = HipSimpleRegeneratingCode(10, 6, 2, device=NONE)
    with pytest.raises(NotImplementedError):
        code.decode([0] * 16, [3], [0])
    with pytest.raises(NotImplementedError):
        code.decodeBulk([np.zeros(4, np.uint8)] * 16, [np.zeros(4, np.uint8)], [3])
    with pytest.raises(Exception):
        HipSimpleRegeneratingCode(10, 4, 5, device=NONE)  # more SRC parities than parities
    assert code.symbolSize() == 8
    assert code.locationsToReadForDecode([]) == []


# ---------------------------------------------------------------- GPU parity

@pytest.mark.gpu
@pytest.mark.parametrize("k,p,s", [(10, 6, 2), (12, 6, 3), (20, 8, 4)])
def test_src_bulk_host_rows_vs_oracle(cuda, k, p, s):
    code = HipSimpleRegeneratingCode(k, p, s)
    n = k + p
    rng = np.random.default_rng(k + p + s)
    L = 3000
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    par = [np.zeros(L, np.uint8) for _ in range(p)]
    code.encodeBulk(data, par)
    assert all((a == b).all() for a, b in zip(par, C.src_encode_bulk(k, p, s, data)))
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(n)]  # non-codeword
    rnd = random.Random(n)
    for _ in range(12):
        erased = sorted(rnd.sample(range(n), rnd.randint(1, p)))
        try:
            er, tr, ntr = _decoder_sets(code, erased)
        except TooManyErasedLocations:
            continue
        out = [np.zeros(L, np.uint8) for _ in er]
        code.decodeBulk([None if x in ntr else rows[x] for x in range(n)], out, er, tr, ntr)
        want = C.src_decode_bulk(k, p, s, [np.zeros(L, np.uint8) if x in ntr else rows[x] for x in range(n)],
                                 er, tr, ntr)
        assert all((a == b).all() for a, b in zip(out, want)), er
    # scalar paths
    msg = [int(v) for v in rng.integers(0, 256, k)]
    parity = [0] * p
    code.encode(msg, parity)
    assert parity == C.src_encode(k, p, s, msg)
    word = parity + msg
    er, tr, ntr = _decoder_sets(code, [p, p + 1])
    vals = [0, 0]
    code.decode([0 if x in ntr else word[x] for x in range(n)], er, vals, tr, ntr)
    assert vals == [word[p], word[p + 1]]


@pytest.mark.gpu
@pytest.mark.parametrize("k,p,s", [(10, 4, 1), (6, 3, 1), (12, 4, 1), (3, 2, 1), (10, 4, 2)])
def test_src_encode_at_compiled_rs_shapes(cuda, k, p, s):
    """SRC shares (k, p) with the compiled-in RS encode kernels; its G (XOR
    groups over RS(k, r)) must never take them (the static kernel
    used to run for any non-XOR code). Host rows, device batches and the
    encode + CRC path, vs the oracle, at window-multiple lengths plus a tail."""
    torch = cuda
    import zlib
    code = HipSimpleRegeneratingCode(k, p, s, device=0)
    assert code.srcLayout()[0] >= 1
    rng = np.random.default_rng(100 * k + 10 * p + s)
    L = (64 << 10) + 77
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    want = C.src_encode_bulk(k, p, s, data)
    par = [np.zeros(L, np.uint8) for _ in range(p)]
    code.encodeBulk(data, par)
    assert all((a == b).all() for a, b in zip(par, want))
    crcs = code.encodeBulkCrc(data, [np.zeros(L, np.uint8) for _ in range(p)])
    assert crcs == [zlib.crc32(r.tobytes()) for r in data] + [zlib.crc32(r.tobytes()) for r in want]
    S, Ld = 3, 64 << 10  # a multiple of the fused kernel's 32 KiB window
    st = torch.randint(0, 256, (S, k + p, Ld), dtype=torch.uint8, device="cuda")
    device.encode_stripes(code, st)
    host = st.cpu().numpy()
    for i in range(S):
        ref = C.src_encode_bulk(k, p, s, [host[i, p + c] for c in range(k)])
        assert all((host[i, r] == ref[r]).all() for r in range(p)), i
    code.setKernelMode(3)  # the fused encode + CRC whenever the shape allows
    st2 = st.clone()
    st2[:, :p] = 0
    crc_dev = device.encode_stripes_crc(code, st2)
    assert torch.equal(st2, st)
    host_crc = crc_dev.cpu().numpy().view(np.uint32).reshape(S, k + p)
    for i in range(S):
        rows = [host[i, p + c] for c in range(k)] + [host[i, r] for r in range(p)]
        assert [int(x) for x in host_crc[i]] == [zlib.crc32(r.tobytes()) for r in rows]


@pytest.mark.gpu
def test_src_every_pattern_round_trip_device(cuda):
    torch = cuda
    k, p, s = 10, 6, 2
    n = k + p
    L, S = 2048 + 64, 2
    code = HipSimpleRegeneratingCode(k, p, s)
    g = torch.Generator(device="cuda")
    g.manual_seed(16)
    st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)
    device.encode_stripes(code, st)
    host = st.cpu().numpy()
    ref = C.src_encode_bulk(k, p, s, [host[0, p + c] for c in range(k)])
    assert all((host[0, r] == ref[r]).all() for r in range(p))
    count = 0
    for e in range(1, p + 1):
        for erased in itertools.combinations(range(n), e):
            erased = list(erased)
            try:
                er, tr, ntr = _decoder_sets(code, erased)
            except TooManyErasedLocations:
                continue
            out = torch.empty((S, e, L), dtype=torch.uint8, device="cuda")
            device.decode_stripes(code, st, er, ntr, out)
            assert torch.equal(out, st[:, er, :]), erased
            count += 1
    assert count == 5883


@pytest.mark.gpu
def test_src_batch_decode(cuda):
    torch = cuda
    k, p, s = 10, 6, 2
    n = k + p
    S, L = 80, 4096 + 30
    code = HipSimpleRegeneratingCode(k, p, s)
    st = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda")
    device.encode_stripes(code, st)
    rnd = random.Random(5)
    er = np.full((S, 4), -1, dtype=np.int32)
    for i in range(S):
        while True:
            e = sorted(rnd.sample(range(n), rnd.randint(0, 4)))
            if C.src_locations_to_read(k, p, s, e) is not None or not e:
                break
        er[i, :len(e)] = e
    out = torch.empty((S, 4, L), dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    for i in range(S):
        lost = [int(x) for x in er[i] if x >= 0]
        if lost:
            assert torch.equal(out[i, :len(lost)], st[i, lost]), (i, lost)


@pytest.mark.gpu
def test_src_codec_registry(cuda):
    conf = {codec_mod.ERASURE_CODING_CODECS_KEY: codec_mod.DEFAULT_CODECS_JSON,
            "hdfs.raid.erasure.code.src": HipSimpleRegeneratingCode.JAVA_CLASS}
    Codec.initializeCodecs(conf)
    code = Codec.getCodec("src").createErasureCode(conf)
    assert isinstance(code, HipSimpleRegeneratingCode)
    assert (code.stripeSize(), code.paritySize(), code.srcLayout()) == (10, 6, (2, 4, 5))
