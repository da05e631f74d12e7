"""The synchronous host-buffer calls (hrs_encode / hrs_decode, the JNI path)
through the pipelined pinned-staging host path: rows longer than one chunk
(HRS_HOST_CHUNK, default 512 KiB), ragged last chunks, several calls in a row
(slot reuse), bit-exact against the oracle."""
import numpy as np
import pytest

from lambdafs_amd import HipNativeReedSolomonCode, HipReedSolomonCode, HipXORCode
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["zero_copy", "copy_engine"])
def transfer_mode(request, monkeypatch):
    """Every test runs each way the synchronous host-buffer calls can move
    bytes: the staged zero-copy path (the default: rows copied into pinned
    staging, the kernel works on the staging across the link) and the copy
    engine (HRS_ZEROCOPY=0: pinned staging, H2D, kernel, D2H). Which caller memory runs in place
    (runtime-pinned only) is test_host_memory.py."""
    monkeypatch.delenv("HRS_ZEROCOPY", raising=False)
    if request.param == "copy_engine":
        monkeypatch.setenv("HRS_ZEROCOPY", "0")
    return request.param


@pytest.mark.parametrize("L", [(3 << 20) + 777, (2 << 20), 4096 + 5, 1])
def test_host_encode_decode_multi_chunk(cuda, L):
    k, p = 10, 4
    n = k + p
    code = HipReedSolomonCode(k, p, zero_inputs_after_encode=False)
    rng = np.random.default_rng(L % 1000)
    for call in range(3):
        data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        par = [np.zeros(L, np.uint8) for _ in range(p)]
        code.encodeBulk(data, par)
        ref = C.encode_bulk(k, p, data)
        assert all((a == b).all() for a, b in zip(par, ref)), call
        stripe = par + data
        erased = [p + call, 1]
        to_read = sorted(code.locationsToReadForDecode(erased))
        ntr = [x for x in range(n) if x not in to_read]
        out = [np.zeros(L, np.uint8) for _ in erased]
        code.decodeBulk([stripe[i] if i in to_read else None for i in range(n)], out, erased, to_read, ntr)
        assert all((o == stripe[e]).all() for o, e in zip(out, erased)), call


def test_host_nrs_and_xor_multi_chunk(cuda):
    L = (2 << 20) + 3
    rng = np.random.default_rng(9)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(10)]
    nrs = HipNativeReedSolomonCode(10, 4)
    par = [np.zeros(L, np.uint8) for _ in range(4)]
    nrs.encodeBulk(data, par)
    assert all((a == b).all() for a, b in zip(par, C.nrs_encode_bulk(10, 4, data)))
    xor = HipXORCode(10, 1)
    xp = [np.zeros(L, np.uint8)]
    xor.encodeBulk(data, xp)
    assert (xp[0] == C.xor_encode_bulk(10, data)).all()


@pytest.mark.parametrize("L", [1 << 20, (1 << 20) + 48, 4096 + 16])
def test_host_calls_on_pinned_rows(cuda, transfer_mode, L):
    """Rows the caller holds in pinned memory (torch pin_memory, i.e.
    hipHostMalloc) go straight to the zero-copy kernel in place ("pinned"; the
    copy engine mode stages them): encodeBulk, encodeBulkCrc and the 5-arg
    decodeBulkCrc vs the oracle and zlib."""
    import zlib
    torch = cuda
    k, p = 10, 4
    n = k + p
    code = HipReedSolomonCode(k, p, zero_inputs_after_encode=False)
    buf = torch.empty((n + 2, L), dtype=torch.uint8, pin_memory=True).numpy()
    rng = np.random.default_rng(L)
    buf[p:n] = rng.integers(0, 256, (k, L), dtype=np.uint8)
    data, par = list(buf[p:n]), list(buf[:p])
    ref = C.encode_bulk(k, p, [d.copy() for d in data])
    want_path = "copy_engine" if transfer_mode == "copy_engine" else "pinned"
    code.encodeBulk(data, par)
    assert code.lastHostPath() == want_path
    assert all(np.array_equal(par[o], ref[o]) for o in range(p))
    buf[:p] = 0
    crcs = code.encodeBulkCrc(data, par, [3] * n)
    assert all(np.array_equal(par[o], ref[o]) for o in range(p))
    assert crcs == [zlib.crc32(r.tobytes(), 3) for r in data + list(ref)]
    stripe = list(buf[:n])
    erased = [p + 2]
    tr = sorted(C.locations_to_read(k, p, erased))
    ntr = [x for x in range(n) if x not in tr]
    out = [buf[n]]
    dcrc = code.decodeBulkCrc([stripe[x] if x in tr else None for x in range(n)], out, erased, tr, ntr, [9])
    assert np.array_equal(out[0], data[2])
    assert dcrc == [zlib.crc32(data[2].tobytes(), 9)]
    if L % 2048 == 0:  # a ragged checksummed repair has no one-pass kernel: it is staged
        assert code.lastHostPath() == want_path
