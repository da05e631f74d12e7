"""Fused encode + CRC-32 (hrs_encode_crc_dev): the parity and the
java.util.zip.CRC32 of every source and parity cell that Encoder.encodeStripe
produces with computeBlockChecksum (Encoder.java:408-450: sourceChecksums over
readBufs, encodeBulk, parityChecksums over writeBufs), in one pass.

Parity is checked against the engine's own encode (itself pinned to the
oracle in test_gpu_parity.py) and, on sampled stripes, against the oracle
directly; CRCs against zlib.crc32 (the JDK's CRC32 is zlib's CRC-32). Both the
fused kernel (static shapes, 2 KiB-multiple cells; large jobs in 32 KiB
windows, small ones in windows of 1-8 sub-windows of 2 KiB) and the two-pass
fallback (other shapes, ragged cells, unaligned rows, forced runtime kernel)
are covered."""
import zlib

import numpy as np
import pytest

from lambdafs_amd import HipNativeReedSolomonCode, HipReedSolomonCode, _lib, device
from oracle import rs_oracle as C


def _u32(x):
    return int(x) & 0xFFFFFFFF


def test_encode_crc_exported():
    assert hasattr(_lib.lib(), "hrs_encode_crc_dev")


def _check(torch, code, st, crc, ref_parity, cin_host=None):
    """crc [S, k+p] vs zlib over the stripe's cells; parity rows vs ref."""
    k, p = code.stripeSize(), code.paritySize()
    host = st.cpu().numpy()
    got = crc.cpu().numpy()
    assert np.array_equal(host[:, :p], ref_parity), "parity differs from the separate encode"
    for s in range(host.shape[0]):
        for r in range(k + p):
            row = host[s, p + r] if r < k else host[s, r - k]
            start = 0 if cin_host is None else _u32(cin_host[s, r])
            assert _u32(got[s, r]) == zlib.crc32(row.tobytes(), start), (s, r)


def _reference_parity(torch, code, st):
    ref = st.clone()
    device.encode_stripes(code, ref)
    return ref[:, :code.paritySize()].cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("cls,k,p", [(HipReedSolomonCode, 10, 4), (HipReedSolomonCode, 6, 3),
                                     (HipReedSolomonCode, 3, 2), (HipReedSolomonCode, 12, 4),
                                     (HipNativeReedSolomonCode, 10, 4), (HipNativeReedSolomonCode, 6, 3)])
def test_fused_static_shapes(cuda, cls, k, p):
    torch = cuda
    code = cls(k, p)
    code.setKernelMode(3)  # the fused kernel even for a 10-window batch
    S, L = 5, 64 << 10
    g = torch.Generator(device="cuda")
    g.manual_seed(k * 100 + p)
    st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda", generator=g)
    ref = _reference_parity(torch, code, st)
    st[:, :p] = 0x5A  # stale parity must be overwritten
    crc = device.encode_stripes_crc(code, st)
    torch.cuda.synchronize()
    _check(torch, code, st, crc, ref)


@pytest.mark.gpu
def test_fused_rs104_1mib_vs_oracle(cuda):
    """BASELINE config 3 cells (RS(10,4), 1 MiB), incl. all-0x00 / all-0xFF / ramp
    edge stripes; parity of sampled stripes against the oracle's encodeBulk."""
    torch = cuda
    k, p, L, S = 10, 4, 1 << 20, 12
    code = HipReedSolomonCode(k, p)
    code.setKernelMode(3)
    st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda")
    st[0] = 0
    st[1] = 0xFF
    st[2] = (torch.arange(L, device="cuda") % 256).to(torch.uint8)
    ref = _reference_parity(torch, code, st)
    crc = device.encode_stripes_crc(code, st)
    torch.cuda.synchronize()
    _check(torch, code, st, crc, ref)
    host = st.cpu().numpy()
    for s in (0, 1, 2, S - 1):
        want = C.encode_bulk(k, p, [host[s, p + c] for c in range(k)])
        assert all(np.array_equal(host[s, r], want[r]) for r in range(p)), s


@pytest.mark.gpu
def test_fused_chaining_like_CRC32_update(cuda):
    """Successive bufSize rounds of one block: crc_in carries the running CRC."""
    torch = cuda
    k, p, L, S, rounds = 10, 4, 256 << 10, 3, 4
    code = HipReedSolomonCode(k, p)
    code.setKernelMode(3)
    cells = [torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda") for _ in range(rounds)]
    crc = None
    for c in cells:
        crc = device.encode_stripes_crc(code, c, crc)
    torch.cuda.synchronize()
    got = crc.cpu().numpy()
    hosts = [c.cpu().numpy() for c in cells]
    for s in range(S):
        for r in range(k + p):
            loc = p + r if r < k else r - k
            want = 0
            for h in hosts:
                want = zlib.crc32(h[s, loc].tobytes(), want)
            assert _u32(got[s, r]) == want, (s, r)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["ragged", "shape", "forced_runtime", "unaligned"])
def test_two_pass_fallback(cuda, case):
    torch = cuda
    k, p, L, S = 10, 4, 96 << 10, 3
    if case == "ragged":
        L = 100000 + 7
    if case == "shape":
        k, p = 5, 2
    code = HipReedSolomonCode(k, p)
    if case == "forced_runtime":
        code.setKernelMode(1)
    if case == "unaligned":
        buf = torch.randint(0, 256, (S, k + p, L + 3), dtype=torch.uint8, device="cuda")
        st = buf[:, :, 3:]
    else:
        st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda")
    ref = st.clone()
    device.encode_stripes(code, ref) if case != "unaligned" else None
    crc = device.encode_stripes_crc(code, st)
    torch.cuda.synchronize()
    host = st.cpu().numpy()
    if case == "unaligned":
        refp = np.stack([np.stack(C.encode_bulk(k, p, [host[s, p + c] for c in range(k)])) for s in range(S)])
    else:
        refp = ref[:, :p].cpu().numpy()
    _check(torch, code, st, crc, refp)


@pytest.mark.gpu
def test_fused_crc_in_layout_and_errors(cuda):
    torch = cuda
    code = HipReedSolomonCode(10, 4)
    st = torch.zeros((2, 14, 32 << 10), dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        device.encode_stripes_crc(code, st, torch.zeros((2, 13), dtype=torch.int32, device="cuda"))
    cin = torch.full((2, 14), 0x1234567, dtype=torch.int32, device="cuda")
    crc = device.encode_stripes_crc(code, st, cin)
    torch.cuda.synchronize()
    _check(torch, code, st, crc, np.zeros((2, 4, 32 << 10), np.uint8), cin.cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("S,L", [(1, 2 << 10), (1, 6 << 10), (2, 34 << 10), (1, 512 << 10), (1, 1 << 20),
                                 (7, 192 << 10), (64, 256 << 10), (300, 64 << 10)])
def test_fused_window_sizes(cuda, S, L):
    """The fused kernel's window choice (1..16 sub-windows of 2 KiB, by how
    many waves the job gives each CU): the Encoder's single-stripe 512 KiB /
    1 MiB rounds, odd sub-window counts, many small stripes. Parity vs the
    engine's encode (pinned to the oracle), CRCs vs zlib, continued from a
    running value."""
    torch = cuda
    k, p = 10, 4
    code = HipReedSolomonCode(k, p)
    g = torch.Generator(device="cuda")
    g.manual_seed(S * 7 + L)
    st = torch.randint(0, 256, (S, k + p, L), dtype=torch.uint8, device="cuda", generator=g)
    ref = _reference_parity(torch, code, st)
    st[:, :p] = 0xA5
    cin = torch.randint(-2**31, 2**31 - 1, (S, k + p), dtype=torch.int32, device="cuda", generator=g)
    crc = device.encode_stripes_crc(code, st, cin)
    torch.cuda.synchronize()
    _check(torch, code, st, crc, ref, cin.cpu().numpy())
