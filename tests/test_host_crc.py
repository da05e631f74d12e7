"""Host-buffer calls with block checksums (hrs_encode_crc / hrs_decode_crc):
the JNI path of Encoder.encodeStripe with computeBlockChecksum
(Encoder.java:408-450: sourceChecksums over readBufs, encodeBulk,
parityChecksums over writeBufs) and of the Decoder's repaired-block check
(Decoder.java:222-229, :645-655).

Cells pass through the pinned-staging pipeline in column chunks
(HRS_HOST_CHUNK, default 128 KiB over 8 slots); each chunk's raw window CRCs are computed
on the GPU next to the encode (fused kernel on 32 KiB-multiple chunks, two
passes on ragged ones), folded on the host as the chunk is copied out
(HRS_HOST_FOLD) and chained with zlib's crc32_combine operator. Parity and repaired rows are checked
against the oracle, CRCs against zlib.crc32 (the JDK's java.util.zip.CRC32
is zlib's CRC-32)."""
import zlib

import numpy as np
import pytest

from lambdafs_amd import HipNativeReedSolomonCode, HipReedSolomonCode, HipXORCode, _lib
from oracle import rs_oracle as C


def test_host_crc_exported():
    L = _lib.lib()
    assert hasattr(L, "hrs_encode_crc") and hasattr(L, "hrs_decode_crc")


@pytest.fixture(params=["zero_copy", "copy_engine", "gated", "wide_chunks"])
def transfer_mode(request, monkeypatch):
    """Every test runs each way the synchronous host-buffer calls can move
    bytes: the staged zero-copy path (the default: rows copied into pinned
    staging, the kernel works on the staging across the link) and the copy
    engine (HRS_ZEROCOPY=0: pinned staging, H2D, kernel, D2H), and the gated
    queue (HRS_HOST_GATE=1, 128 KiB chunks after a 64 KiB first one over 4
    slots: every chunk's kernels queued ahead behind gate kernels the host
    opens after each copy-in), and 512 KiB chunks over 2 slots (wide_chunks:
    the 1,024-thread fused encode + CRC blocks). Which caller memory runs in place
    (runtime-pinned only) is test_host_memory.py."""
    monkeypatch.delenv("HRS_ZEROCOPY", raising=False)
    for var in ("HRS_HOST_GATE", "HRS_HOST_CHUNK", "HRS_HOST_SLOTS", "HRS_HOST_FIRST"):
        monkeypatch.delenv(var, raising=False)
    if request.param == "copy_engine":
        monkeypatch.setenv("HRS_ZEROCOPY", "0")
        monkeypatch.setenv("HRS_HOST_GATE", "0")
    elif request.param == "gated":  # gated queued chunks, small and many (hrs_hostpath.cpp staged_run)
        monkeypatch.setenv("HRS_HOST_GATE", "1")
        monkeypatch.setenv("HRS_HOST_CHUNK", "131072")
        monkeypatch.setenv("HRS_HOST_SLOTS", "4")
        monkeypatch.setenv("HRS_HOST_FIRST", "65536")
    elif request.param == "wide_chunks":  # 512 KiB x 2 slots (round 5's default)
        monkeypatch.setenv("HRS_HOST_GATE", "0")
        monkeypatch.setenv("HRS_HOST_CHUNK", "524288")
        monkeypatch.setenv("HRS_HOST_SLOTS", "2")
    else:
        monkeypatch.setenv("HRS_HOST_GATE", "0")
    return request.param


def _zcrc(rows, start=None):
    return [zlib.crc32(r.tobytes(), 0 if start is None else start[i]) for i, r in enumerate(rows)]


@pytest.mark.gpu
@pytest.mark.usefixtures("transfer_mode")
@pytest.mark.parametrize("L", [1 << 20, (1 << 20) + 777, (2 << 20) + (32 << 10), 4096 + 5, 1])
def test_encode_crc_host_rs104(cuda, L):
    k, p = 10, 4
    code = HipReedSolomonCode(k, p, zero_inputs_after_encode=False)
    rng = np.random.default_rng(L % 997)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    par = [np.full(L, 0x5A, np.uint8) for _ in range(p)]
    crcs = code.encodeBulkCrc(data, par)
    ref = C.encode_bulk(k, p, data)
    assert all((a == b).all() for a, b in zip(par, ref))
    assert crcs == _zcrc(data) + _zcrc(ref)


@pytest.mark.gpu
@pytest.mark.usefixtures("transfer_mode")
def test_encode_crc_host_chained_block(cuda):
    """A block encoded cell by cell: the running CRCs after the last call
    equal the CRC32 of each whole block (CRC32.update chaining)."""
    k, p, cell, cells = 6, 3, 64 << 10, 5
    code = HipReedSolomonCode(k, p)  # zero_inputs_after_encode: checksums see the inputs first
    rng = np.random.default_rng(5)
    blocks = [rng.integers(0, 256, cell * cells, dtype=np.uint8) for _ in range(k)]
    pblocks = [np.zeros(cell * cells, np.uint8) for _ in range(p)]
    crcs = None
    for j in range(cells):
        ins = [b[j * cell:(j + 1) * cell].copy() for b in blocks]
        outs = [np.zeros(cell, np.uint8) for _ in range(p)]
        crcs = code.encodeBulkCrc(ins, outs, crcs)
        assert all((v == 0).all() for v in ins)  # the reference's in-place side effect
        for o in range(p):
            pblocks[o][j * cell:(j + 1) * cell] = outs[o]
    ref = C.encode_bulk(k, p, [b for b in blocks])
    assert all((a == b).all() for a, b in zip(pblocks, ref))
    assert crcs == _zcrc(blocks) + _zcrc(ref)


@pytest.mark.gpu
@pytest.mark.usefixtures("transfer_mode")
@pytest.mark.parametrize("make", [lambda: HipNativeReedSolomonCode(10, 4), lambda: HipXORCode(10, 1),
                                  lambda: HipReedSolomonCode(12, 4, zero_inputs_after_encode=False)])
def test_encode_crc_host_codes(cuda, make):
    code = make()
    k, p = code.stripeSize(), code.paritySize()
    L = (1 << 20) + 3
    rng = np.random.default_rng(k * 10 + p)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    par = [np.zeros(L, np.uint8) for _ in range(p)]
    start = [int(x) for x in rng.integers(0, 1 << 32, k + p, dtype=np.uint64)]
    crcs = code.encodeBulkCrc(data, par, start)
    plain = [np.zeros(L, np.uint8) for _ in range(p)]
    code.encodeBulk(data, plain)
    assert all((a == b).all() for a, b in zip(par, plain))
    assert crcs == _zcrc(data + par, start)


@pytest.mark.gpu
@pytest.mark.usefixtures("transfer_mode")
@pytest.mark.parametrize("L,erased", [((1 << 20) + 11, [4]), (256 << 10, [0, 13]), (3 << 20, [2, 5, 7, 11])])
def test_decode_crc_host(cuda, L, erased):
    k, p = 10, 4
    n = k + p
    code = HipReedSolomonCode(k, p, zero_inputs_after_encode=False)
    rng = np.random.default_rng(L % 991)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    stripe = C.encode_bulk(k, p, data) + data
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(n) if x not in to_read]
    out = [np.zeros(L, np.uint8) for _ in erased]
    crcs = code.decodeBulkCrc([stripe[i] if i in to_read else None for i in range(n)], out, erased, to_read, ntr)
    assert all((o == stripe[e]).all() for o, e in zip(out, erased))
    assert crcs == _zcrc([stripe[e] for e in erased])
    start = [123456789 + e for e in erased]
    crcs2 = code.decodeBulkCrc([stripe[i] if i in to_read else None for i in range(n)], out, erased, to_read, ntr,
                               start)
    assert crcs2 == _zcrc([stripe[e] for e in erased], start)


@pytest.mark.gpu
@pytest.mark.usefixtures("transfer_mode")
def test_crc_host_empty_rows(cuda):
    code = HipReedSolomonCode(3, 2, zero_inputs_after_encode=False)
    data = [np.zeros(0, np.uint8) for _ in range(3)]
    par = [np.zeros(0, np.uint8) for _ in range(2)]
    assert code.encodeBulkCrc(data, par) == [0] * 5
    assert code.encodeBulkCrc(data, par, [7, 8, 9, 10, 11]) == [7, 8, 9, 10, 11]
