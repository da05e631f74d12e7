"""The synchronous host-buffer calls (hrs_encode / hrs_decode, the JNI path)
through the pipelined pinned-staging host path: rows longer than one chunk
(HRS_HOST_CHUNK, default 128 KiB over 8 slots), ragged last chunks, several calls in a row
(slot reuse), bit-exact against the oracle."""
import numpy as np
import pytest

from lambdafs_amd import HipNativeReedSolomonCode, HipReedSolomonCode, HipXORCode
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["zero_copy", "copy_engine", "gated", "wide_chunks"])
def transfer_mode(request, monkeypatch):
    """Every test runs each way the synchronous host-buffer calls can move
    bytes: the staged zero-copy path (the default: rows copied into pinned
    staging, the kernel works on the staging across the link) and the copy
    engine (HRS_ZEROCOPY=0: pinned staging, H2D, kernel, D2H), and the gated
    queue (HRS_HOST_GATE=1, 128 KiB chunks after a 64 KiB first one over 4
    slots: every chunk's kernels queued ahead behind gate kernels the host
    opens after each copy-in), and 512 KiB chunks over 2 slots (wide_chunks:
    the 1,024-thread fused encode + CRC blocks). Copy-in stores: the default
    (nontemporal) for zero_copy and gated, nontemporal only off the GPU's NUMA
    node (HRS_HOST_NT=auto) for wide_chunks, cached (0) for copy_engine.
    Which caller memory runs in place (runtime-pinned only) is
    test_host_memory.py."""
    monkeypatch.delenv("HRS_ZEROCOPY", raising=False)
    for var in ("HRS_HOST_GATE", "HRS_HOST_CHUNK", "HRS_HOST_SLOTS", "HRS_HOST_FIRST", "HRS_HOST_NT"):
        monkeypatch.delenv(var, raising=False)
    if request.param == "copy_engine":
        monkeypatch.setenv("HRS_ZEROCOPY", "0")
        monkeypatch.setenv("HRS_HOST_GATE", "0")
        monkeypatch.setenv("HRS_HOST_NT", "0")
    elif request.param == "gated":  # gated queued chunks, small and many (hrs_hostpath.cpp staged_run)
        monkeypatch.setenv("HRS_HOST_GATE", "1")
        monkeypatch.setenv("HRS_HOST_CHUNK", "131072")
        monkeypatch.setenv("HRS_HOST_SLOTS", "4")
        monkeypatch.setenv("HRS_HOST_FIRST", "65536")
    elif request.param == "wide_chunks":  # 512 KiB x 2 slots (round 5's default)
        monkeypatch.setenv("HRS_HOST_GATE", "0")
        monkeypatch.setenv("HRS_HOST_CHUNK", "524288")
        monkeypatch.setenv("HRS_HOST_SLOTS", "2")
        monkeypatch.setenv("HRS_HOST_NT", "auto")
    else:
        monkeypatch.setenv("HRS_HOST_GATE", "0")
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


def test_gate_miss_reruns_without_gates(cuda, transfer_mode, monkeypatch):
    """A gate kernel that gives up waiting (its host stalled past the timeout; test
    hooks HRS_GATE_TIMEOUT_US / HRS_GATE_DELAY_US) lets its chunk's kernels
    run on stale staging; the call must notice the miss, discard those
    results and run again without gates: bit-exact outputs and CRCs."""
    import time
    import zlib
    if transfer_mode != "gated":
        pytest.skip("gated pipeline only")
    k, p, L = 10, 4, 1 << 20
    code = HipReedSolomonCode(k, p, zero_inputs_after_encode=False)
    rng = np.random.default_rng(77)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    par = [np.zeros(L, np.uint8) for _ in range(p)]
    ref = C.encode_bulk(k, p, data)
    code.encodeBulk(data, par)  # first run of these chunk shapes: no gates yet
    code.encodeBulkCrc(data, par)
    monkeypatch.setenv("HRS_GATE_TIMEOUT_US", "200")
    monkeypatch.setenv("HRS_GATE_DELAY_US", "20000")
    for x in par:
        x[:] = 0xC3
    t0 = time.perf_counter()
    code.encodeBulk(data, par)
    assert time.perf_counter() - t0 >= 0.02  # the stall happened inside the gated run
    assert all((a == b).all() for a, b in zip(par, ref))
    for x in par:
        x[:] = 0x3C
    run = [int(v) for v in rng.integers(0, 1 << 32, k + p, dtype=np.uint64)]
    crcs = code.encodeBulkCrc(data, par, run)
    assert all((a == b).all() for a, b in zip(par, ref))
    cells = data + list(ref)
    assert crcs == [zlib.crc32(cells[i].tobytes(), run[i]) & 0xFFFFFFFF for i in range(k + p)]
