"""The hops `rs` code against the reference's second source of the same
polynomial code: hadoop-common's legacy pure-Java coder,
RSLegacyRawEncoder / RSLegacyRawDecoder over its own util/GaloisField and
util/RSUtil (hadoop-common-project/hadoop-common/src/main/java/org/apache/
hadoop/io/erasurecode/rawcoder/), restated loop for loop as orc_legacy_* in
oracle/rs_oracle.c.

It is a third transcription, from separate reference files, of the code hops'
ReedSolomonCode implements: the same generator prod (x + 2^i), i < p
(RSLegacyRawEncoder.java:36-53 vs ReedSolomonCode.java:56-82), the same
[parity..., data...] bulk remainder (:91-128 vs :103-125), and syndromes plus
a Vandermonde solve for decode (RSLegacyRawDecoder.java:98-165 vs
ReedSolomonCode.java:127-211). CPU: the legacy coder equals the hops
restatement (orc_rs_*) for every 1..p erasure pattern of RS(10,4), (6,3),
(12,4) and (3,2), on non-codeword stripes, reading the k survivors
locationsToReadForDecode picks and reading every survivor. GPU: the product's
device encode and repairs equal the legacy coder. RS parity stays "parity
unpinned" in the strict sense (no reference-executed vector: no JDK here),
now held by three transcriptions from two reference sources.
"""
import itertools

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, device
from oracle import rs_oracle as C

SHAPES = [(10, 4), (6, 3), (12, 4), (3, 2)]


@pytest.mark.parametrize("k,p", SHAPES + [(1, 1), (20, 8), (100, 10), (200, 55)])
def test_generator_equals_hops(k, p):
    assert C.legacy_generator(k, p) == C.generator(k, p)


@pytest.mark.parametrize("k,p", SHAPES + [(20, 8), (1, 1)])
@pytest.mark.parametrize("L", [1, 7, 64, 4099])
def test_encode_equals_hops(k, p, L):
    rng = np.random.default_rng(k * 1000 + p * 10 + L)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    legacy = C.legacy_rs_encode(k, p, data)
    hops = C.encode_bulk(k, p, [d.copy() for d in data])  # encodeBulk zeroes its inputs
    for a, b in zip(legacy, hops):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("k,p", SHAPES)
def test_decode_equals_hops_every_pattern(k, p):
    """Every pattern of 1..p lost locations, non-codeword stripe (every byte
    random, so every syndrome coefficient counts), two survivor sets: the k
    locationsToReadForDecode picks (the Decoder's call) and every survivor."""
    n, L = k + p, 24
    rng = np.random.default_rng(k * 31 + p)
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(n)]
    count = 0
    for m in range(1, p + 1):
        for erased in itertools.combinations(range(n), m):
            erased = list(erased)
            to_read = sorted(C.locations_to_read(k, p, erased))
            for ntr in ([x for x in range(n) if x not in to_read], erased):
                reads = [np.zeros(L, np.uint8) if j in ntr else rows[j] for j in range(n)]
                tr = [x for x in range(n) if x not in ntr]
                hops = C.decode_bulk5(k, p, reads, erased, tr, ntr)
                legacy = C.hops_decode_via_legacy(k, p, rows, erased, ntr)
                for a, b in zip(hops, legacy):
                    assert np.array_equal(a, b), (erased, ntr)
                count += 1
    assert count == 2 * sum(len(list(itertools.combinations(range(n), m))) for m in range(1, p + 1))


def test_decode_round_trip_and_java_order():
    """A codeword round-trips, and outputs follow the caller's erasedIndexes
    in Apache order (data units, then parity units: adjustOrder,
    RSLegacyRawDecoder.java:222-253)."""
    k, p, L = 6, 3, 100
    rng = np.random.default_rng(5)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    units = data + C.legacy_rs_encode(k, p, data)  # Apache order
    erased = [1, 4, 7]  # data 1, data 4, parity 1
    inputs = [None if i in erased else units[i] for i in range(k + p)]
    out = C.legacy_rs_decode(k, p, inputs, erased)
    for e, o in zip(erased, out):
        assert np.array_equal(o, units[e])


def test_decode_errors_match_the_java():
    k, p, L = 6, 3, 16
    rows = [np.full(L, i, np.uint8) for i in range(k + p)]
    with pytest.raises(ValueError, match="not enough valid inputs"):  # ByteArrayDecodingState.java:111-114
        C.legacy_rs_decode(k, p, [None] * 4 + rows[4:], [0])
    with pytest.raises(ValueError, match="not fully corresponding"):  # RSLegacyRawDecoder.java:146-149
        C.legacy_rs_decode(k, p, [None] + rows[1:], [2])


@pytest.mark.gpu
@pytest.mark.parametrize("k,p,L", [(10, 4, (64 << 10) + 5), (6, 3, 8192), (12, 4, 4096), (3, 2, 2048 * 3)])
def test_device_equals_legacy_coder(cuda, k, p, L):
    """The product's device encode equals RSLegacyRawEncoder, and its repairs
    (decodeBulk 5-arg through hrs_decode_dev) of sampled patterns of a
    non-codeword batch equal RSLegacyRawDecoder with the same rows unread."""
    torch = cuda
    n, S = k + p, 4
    rng = np.random.default_rng(L + k)
    host = rng.integers(0, 256, (S, n, L), dtype=np.uint8)
    code = HipReedSolomonCode(k, p, device=0)
    st = torch.from_numpy(host.copy()).cuda()
    device.encode_stripes(code, st)
    enc = st.cpu().numpy()
    for s in range(S):
        legacy = C.legacy_rs_encode(k, p, [host[s, p + c] for c in range(k)])
        assert all(np.array_equal(enc[s, r], legacy[r]) for r in range(p)), s
    dev_rows = torch.from_numpy(host).cuda()  # non-codewords: every coefficient of the repair counts
    pats = [[p], [0], list(range(p))] + [sorted(rng.choice(n, 1 + t % p, replace=False).tolist()) for t in range(6)]
    for erased in pats:
        to_read = sorted(code.locationsToReadForDecode(erased))
        ntr = [x for x in range(n) if x not in to_read]
        out = torch.empty((S, len(erased), L), dtype=torch.uint8, device="cuda")
        device.decode_stripes(code, dev_rows, erased, ntr, out)
        got = out.cpu().numpy()
        for s in range(S):
            legacy = C.hops_decode_via_legacy(k, p, list(host[s]), erased, ntr)
            for t in range(len(erased)):
                assert np.array_equal(got[s, t], legacy[t]), (erased, s, t)


def _golden():
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "tests", "golden", "bench_digests.json")) as f:
        return json.load(f)


def test_golden_config2_block0_through_the_legacy_coder():
    """The committed full-size digests (made by the hops restatement) are
    reproduced by the legacy coder alone: config 2's parity of global stripes
    0-255 (RS(6,3), 64 KiB cells, SURVEY 8(d) synthetic stripes), encoded by
    RSLegacyRawEncoder's restatement."""
    import hashlib
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import stripe_digests as SD
    import synth
    k, p, L = 6, 3, 64 << 10
    d = {}
    for g in range(256):
        data = synth.stripe_numpy(2, g, k, L)
        h = hashlib.sha256()
        for r in C.legacy_rs_encode(k, p, [data[c] for c in range(k)]):
            h.update(r.tobytes())
        d[g] = h.digest()
    assert SD.combine(d) == {"0": _golden()["config2"]["parity"]["0"]}


def test_golden_config5_block0_through_the_legacy_coder():
    """Config 5's repaired cells of global stripes 0-255 (RS(12,4), 256 KiB
    cells, each stripe's seeded lost pair): parity from the legacy encoder,
    then the legacy decoder reading the k survivors locationsToReadForDecode
    picks — equal to the committed digest the hops restatement made (~20 s)."""
    import hashlib
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import stripe_digests as SD
    import synth
    k, p, L = 12, 4, 256 << 10
    n = k + p
    d = {}
    for g in range(256):
        data = synth.stripe_numpy(5, g, k, L)
        parity = C.legacy_rs_encode(k, p, [data[c] for c in range(k)])
        hops_rows = list(parity) + [data[c] for c in range(k)]  # hops order [parity..., data...]
        er = sorted(int(x) for x in np.random.default_rng([0x5EED0005, g]).choice(n, 2, replace=False))
        tr = sorted(C.locations_to_read(k, p, er))
        ntr = [x for x in range(n) if x not in tr]
        h = hashlib.sha256()
        for o in C.hops_decode_via_legacy(k, p, hops_rows, er, ntr):
            h.update(o.tobytes())
        d[g] = h.digest()
    assert SD.combine(d) == {"0": _golden()["config5"]["repaired"]["0"]}
