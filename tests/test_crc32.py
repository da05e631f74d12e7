"""GPU CRC-32 of device-resident cells (hrs_crc32_dev), bit-exact with
java.util.zip.CRC32 — the checksum Encoder.java:408-450 keeps per source and
parity block and Decoder.java:222-229 re-checks after repair. The JDK's CRC32
is zlib's CRC-32 (the JDK bundles zlib), so Python's zlib.crc32 (system zlib
1.2.11) is the oracle here."""
import os
import subprocess
import zlib

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, device
from oracle import rs_oracle as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_crc_kernel_model_against_zlib():
    """CPU model of the kernels' decomposition (same tables) vs zlib."""
    binary = os.path.join(ROOT, "tests", "cpp", "crc_model")
    if not os.path.exists(binary):
        subprocess.check_call(["make", "-C", ROOT, "tests/cpp/crc_model"])
    out = subprocess.run([binary], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr


def _u32(x):
    return int(x) & 0xFFFFFFFF


@pytest.mark.parametrize("d,W", [(4080, 4096), (16, 4096), (1, 2048), (2048, 2048), (0, 2048), (5000, 6144)])
def test_leading_pad_correction(d, W):
    """The identity the direct host path (hrs_hostpath.cpp host_apply_direct,
    pad_fix) uses for its head / tail segments, which it runs right-aligned
    behind a zero pad: crc32(0, D) = crc32(0, 0^m || D) ^ Z_W(~0) ^ Z_d(~0),
    with Z_n(~0) = ~crc32(0, 0^n) (a raw CRC ignores leading zeros; only the
    length term differs)."""
    D = np.random.default_rng(d).integers(0, 256, d, dtype=np.uint8).tobytes()
    padded = bytes(W - d) + D

    def z(n):
        return ~zlib.crc32(bytes(n)) & 0xFFFFFFFF

    assert zlib.crc32(D) == zlib.crc32(padded) ^ z(W) ^ z(d)


@pytest.mark.gpu
@pytest.mark.parametrize("L", [0, 1, 100, 4095, 4096, 4097, 65536 + 13, 1 << 20, (1 << 20) + 4096 * 70 + 33])
def test_crc32_rows_match_zlib(cuda, L):
    torch = cuda
    code = HipReedSolomonCode(10, 4)
    S, n = 3, 14
    g = torch.Generator(device="cuda")
    g.manual_seed(L + 1)
    st = torch.randint(0, 256, (S, n, max(L, 1)), dtype=torch.uint8, device="cuda", generator=g)[:, :, :L]
    crcs = device.crc32_rows(code, [st[:, r, :] for r in range(n)])
    host = st.cpu().numpy()
    got = crcs.cpu().numpy()
    for s in range(S):
        for r in range(n):
            assert _u32(got[s, r]) == zlib.crc32(host[s, r].tobytes()), (L, s, r)


@pytest.mark.gpu
def test_crc32_chaining_like_CRC32_update(cuda):
    """Running block CRC over successive 1 MiB cells == CRC of the block."""
    torch = cuda
    code = HipReedSolomonCode(10, 4)
    block = torch.randint(0, 256, (2, 4 << 20), dtype=torch.uint8, device="cuda")
    crc = None
    for off in range(0, 4 << 20, 1 << 20):
        cells = [block[:, off:off + (1 << 20)]]
        crc = device.crc32_rows(code, cells, crc)
    host = block.cpu().numpy()
    for s in range(2):
        assert _u32(crc[s, 0]) == zlib.crc32(host[s].tobytes())


@pytest.mark.gpu
def test_crc32_unaligned_rows(cuda):
    torch = cuda
    code = HipReedSolomonCode(10, 4)
    buf = torch.randint(0, 256, (3, 20000), dtype=torch.uint8, device="cuda")
    view = buf[:, 3:3 + 12345]  # rows start 3 bytes into each 20000-byte line
    crcs = device.crc32_rows(code, [view])
    host = view.cpu().numpy()
    for s in range(3):
        assert _u32(crcs[s, 0]) == zlib.crc32(host[s].tobytes())


@pytest.mark.gpu
def test_encode_then_block_checksums(cuda):
    """The Encoder's pattern on device-resident stripes: encode, then CRC32 of
    every source and parity cell (Encoder.java:434-450)."""
    torch = cuda
    k, p, L, S = 10, 4, 1 << 20, 16
    code = HipReedSolomonCode(k, p)
    st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda")
    device.encode_stripes(code, st)
    crcs = device.crc32_rows(code, [st[:, r, :] for r in range(k + p)]).cpu().numpy()
    host = st.cpu().numpy()
    for s in (0, S - 1):
        for r in range(k + p):
            assert _u32(crcs[s, r]) == zlib.crc32(host[s, r].tobytes())


@pytest.mark.gpu
def test_fold_table_shared_by_slot_streams_survives_eviction(cuda):
    """two asynchronous checksummed encodes of the same row length
    run their folds on two different slot streams with one fold table; 64
    device CRC calls of other lengths then evict that table while both may
    still be queued. Each table keeps the latest use on every stream that
    read it, so the eviction waits for both folds. Every CRC vs zlib."""
    torch = cuda
    k, p, L = 10, 4, (256 << 10) + 40
    code = HipReedSolomonCode(k, p)
    rng = np.random.default_rng(78)
    rounds = [[rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] for _ in range(2)]
    keep = [[r.copy() for r in rnd] for rnd in rounds]
    tickets = [code.encodeBulkAsync(rnd, checksums=True) for rnd in rounds]
    side = []
    for i in range(66):
        Li = 8192 + 64 * i
        rows = torch.from_numpy(rng.integers(0, 256, (2, Li), dtype=np.uint8)).cuda()
        side.append((rows, device.crc32_rows(code, [rows[r:r + 1] for r in range(2)])))
    for t, kept in zip(tickets, keep):
        out = [np.zeros(L, np.uint8) for _ in range(p)]
        crcs = code.collect(t, out)
        ref = C.encode_bulk(k, p, [x.copy() for x in kept])
        assert all(np.array_equal(o, r) for o, r in zip(out, ref))
        assert crcs == [zlib.crc32(b.tobytes()) for b in kept + list(ref)]
    torch.cuda.synchronize()
    for rows, got in side:
        host = rows.cpu().numpy()
        assert [int(x) & 0xFFFFFFFF for x in got[0].tolist()] == [zlib.crc32(host[r].tobytes()) for r in range(2)]


@pytest.mark.gpu
def test_fold_table_cache_eviction_across_streams(cuda):
    """More distinct row lengths than the fold-table cache holds (64): the
    least recently used entry is evicted after the event behind its latest
    fold, with calls queued on two streams and never synchronized in between;
    lengths evicted early come back (rebuilt) at the end. Every CRC vs zlib."""
    torch = cuda
    code = HipReedSolomonCode(10, 4)
    lens = [4096 + 48 * i for i in range(72)] + [4096, 4096 + 48]
    rng = np.random.default_rng(77)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = []
    for i, L in enumerate(lens):
        rows = torch.from_numpy(rng.integers(0, 256, (3, L), dtype=np.uint8)).cuda()
        torch.cuda.synchronize()
        with torch.cuda.stream(streams[i % 2]):
            jobs.append((rows, device.crc32_rows(code, [rows[r:r + 1] for r in range(3)])))
    torch.cuda.synchronize()
    for rows, got in jobs:
        host = rows.cpu().numpy()
        want = [zlib.crc32(host[r].tobytes()) for r in range(3)]
        assert [int(x) & 0xFFFFFFFF for x in got[0].tolist()] == want
