"""The XOR code (`xor` codec, XORCode.java:24-146) behind the same boundary.

CPU: the product's XOR matrices and argument rules against the oracle's
transcription of XORCode. GPU (-m gpu): encodeBulk / decodeBulk / scalar
paths bit-exact against the oracle, through the dedicated XOR kernel, the
byte-granular tail kernel and input chunking.
"""
import random

import numpy as np
import pytest

from lambdafs_amd import Codec, HipXORCode, HrsError, device
from lambdafs_amd import codec as codec_mod
from oracle import rs_oracle as C

NONE = -2


def test_xor_matrices_match_oracle():
    for k in (1, 3, 10, 40):
        code = HipXORCode(k, 1, device=NONE)
        G = code.encodeMatrix()
        for c in range(k):
            assert int(G[0, c]) == C.xor_encode(k, [1 if j == c else 0 for j in range(k)])[0]
        for e in range(k + 1):
            D = code.decodeMatrix([e], [])
            for col in range(k + 1):
                unit = [1 if j == col else 0 for j in range(k + 1)]
                assert int(D[0, col]) == C.xor_decode(k, unit, [e])[0]


def test_xor_rules():
    with pytest.raises(HrsError):
        HipXORCode(10, 2, device=NONE)  # XORCode.init asserts paritySize == 1
    code = HipXORCode(10, 1, device=NONE)
    with pytest.raises(HrsError):
        code.decodeMatrix([1, 2], [])  # exactly one erasure
    assert C.xor_decode(3, [1, 2, 3, 4], [0, 1]) == [-1, -1]  # reference: no-op unless one erasure


def test_xor_oracle_round_trip():
    rng = np.random.default_rng(4)
    k = 10
    data = [rng.integers(0, 256, 999, dtype=np.uint8) for _ in range(k)]
    par = C.xor_encode_bulk(k, data)
    stripe = [par] + data
    for e in range(k + 1):
        reads = [np.zeros(999, np.uint8) if i == e else stripe[i] for i in range(k + 1)]
        assert (C.xor_decode_bulk(k, reads, e) == stripe[e]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 3, 10, 16, 17, 40])
def test_xor_encode_decode_gpu(cuda, k):
    torch = cuda
    code = HipXORCode(k, 1)
    for L, S in [(1, 2), (2048, 3), (5000, 2), (65536 + 7, 2)]:
        g = torch.Generator(device="cuda")
        g.manual_seed(k * 31 + L)
        st = torch.randint(0, 256, (S, k + 1, L), dtype=torch.uint8, device="cuda", generator=g)
        device.encode_stripes(code, st)
        host = st.cpu().numpy()
        for s in range(S):
            assert (host[s, 0] == C.xor_encode_bulk(k, [host[s, 1 + c] for c in range(k)])).all(), (k, L)
        for e in sorted({0, 1, k}):
            out = torch.empty((S, 1, L), dtype=torch.uint8, device="cuda")
            device.decode_stripes(code, st, [e], [e], out)
            assert torch.equal(out[:, 0], st[:, e]), (k, L, e)


@pytest.mark.gpu
def test_xor_host_api_and_scalar(cuda):
    rnd = random.Random(3)
    k = 10
    code = HipXORCode(k, 1)
    data = [bytes(rnd.randrange(256) for _ in range(300)) for _ in range(k)]
    par = [bytearray(300)]
    code.encodeBulk(data, par)
    ref = C.xor_encode_bulk(k, [np.frombuffer(d, np.uint8) for d in data])
    assert bytes(par[0]) == bytes(ref)
    stripe = [bytes(par[0])] + data
    for e in range(k + 1):
        reads = [bytes(300) if i == e else stripe[i] for i in range(k + 1)]
        out = [bytearray(300)]
        code.decodeBulk(reads, out, [e], [], [e])
        assert bytes(out[0]) == stripe[e]
        out3 = [bytearray(300)]
        code.decodeBulk(reads, out3, [e])
        assert bytes(out3[0]) == stripe[e]
    msg = [rnd.randrange(256) for _ in range(k)]
    p = [0]
    code.encode(msg, p)
    assert p == C.xor_encode(k, msg)
    data_sym = p + msg
    vals = [0]
    code.decode(list(data_sym), [4], vals)
    assert vals == [data_sym[4]]
    untouched = [123, 45]
    code.decode(list(data_sym), [1, 2], untouched)  # reference no-op
    assert untouched == [123, 45]


@pytest.mark.gpu
def test_xor_codec_registry(cuda):
    conf = {codec_mod.ERASURE_CODING_CODECS_KEY: codec_mod.DEFAULT_CODECS_JSON,
            "hdfs.raid.erasure.code.xor": HipXORCode.JAVA_CLASS}
    Codec.initializeCodecs(conf)
    code = Codec.getCodec("xor").createErasureCode(conf)
    assert isinstance(code, HipXORCode) and (code.stripeSize(), code.paritySize()) == (10, 1)
