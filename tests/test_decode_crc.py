"""Fused repair + CRC-32 (hrs_decode_crc_dev): the repaired cells and the
java.util.zip.CRC32 of each of them, as the Decoder produces them per lost
block (decodeBulk, then the repaired block's CRC32 compared with the
NameNode's checksum; Decoder.java:222-229, :352-353, :645-655), in one pass.

Repaired cells are checked against the oracle's decodeBulk (5-arg, the
survivors locationsToReadForDecode picks, every other location not read, as
Decoder.java:303-338 builds the arrays) on non-codeword inputs, so every
coefficient of the decode matrix counts; CRCs against zlib.crc32 (the JDK's
CRC32 is zlib's CRC-32). Both the fused kernel (1-4 repaired locations from
<= 12 live survivors, 2 KiB-multiple aligned cells) and the fallback (apply,
then the CRC pass: 4 locations of RS(10,4) read 10 survivors, ragged cells,
unaligned rows, a forced runtime kernel) are covered."""
import itertools
import random
import zlib

import numpy as np
import pytest

from lambdafs_amd import (HipNativeReedSolomonCode, HipReedSolomonCode, HipSimpleRegeneratingCode, HipXORCode,
                          _lib, device)
from oracle import rs_oracle as C


def _u32(x):
    return int(x) & 0xFFFFFFFF


def test_decode_crc_exported():
    assert hasattr(_lib.lib(), "hrs_decode_crc_dev")


def _stripes(torch, S, n, L, seed, pad=0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    buf = torch.randint(0, 256, (S, n, L + pad), dtype=torch.uint8, device="cuda", generator=g)
    return buf[:, :, pad:] if pad else buf


def _pattern(code, erased):
    n = code.stripeSize() + code.paritySize()
    to_read = sorted(code.locationsToReadForDecode(list(erased)))
    return to_read, [x for x in range(n) if x not in to_read]


def _run(torch, code, st, erased, crc_in=None):
    _, ntr = _pattern(code, erased)
    S, L = st.shape[0], st.shape[2]
    out = torch.full((S, len(erased), L), 0x5A, dtype=torch.uint8, device="cuda")
    crc = device.decode_stripes_crc(code, st, erased, ntr, out, crc_in)
    _run.kernel = code.lastKernel()  # before the reference decode below renames it
    ref = torch.full_like(out, 0xA5)
    device.decode_stripes(code, st, erased, ntr, ref)
    torch.cuda.synchronize()
    return out.cpu().numpy(), crc.cpu().numpy(), ref.cpu().numpy()


def _check_crcs(got_out, crc, crc_in=None):
    S, e = crc.shape
    for s in range(S):
        for t in range(e):
            start = 0 if crc_in is None else _u32(crc_in[s, t])
            assert _u32(crc[s, t]) == zlib.crc32(got_out[s, t].tobytes(), start), (s, t)


def _check_vs_oracle(k, p, host, got_out, erased, to_read, ntr, stripes):
    n = k + p
    L = host.shape[2]
    for s in stripes:
        reads = [host[s, i] if i in to_read else np.zeros(L, np.uint8) for i in range(n)]
        ref = C.decode_bulk5(k, p, reads, erased, to_read, ntr)
        assert all(np.array_equal(got_out[s, i], ref[i]) for i in range(len(erased))), (erased, s)


@pytest.mark.gpu
@pytest.mark.parametrize("k,p", [(10, 4), (6, 3), (12, 4), (3, 2)])
def test_fused_repairs_vs_oracle(cuda, k, p):
    """1..p lost locations (every single loss, sampled pairs/triples/quads)
    on random non-codeword stripes; 1-3 losses (and 4 with <= 8 live
    survivors) take the fused kernel."""
    torch = cuda
    code = HipReedSolomonCode(k, p)
    n = k + p
    rnd = random.Random(k * 31 + p)
    pats = [[x] for x in range(n)]
    for e in range(2, p + 1):
        pats += [sorted(c) for c in rnd.sample(list(itertools.combinations(range(n), e)), 4)]
    S, L = 3, 10 << 10
    st = _stripes(torch, S, n, L, seed=k * 100 + p)
    host = st.cpu().numpy()
    for erased in pats:
        to_read, ntr = _pattern(code, erased)
        got, crc, ref = _run(torch, code, st, erased)
        assert np.array_equal(got, ref), erased
        _check_crcs(got, crc)
        _check_vs_oracle(k, p, host, got, erased, to_read, ntr, range(S))
        live = int((code.decodeMatrix(erased, ntr) != 0).any(axis=0).sum())  # columns the kernel reads
        fused = live <= (8 if len(erased) == 4 else 12)
        assert _run.kernel.startswith("decode_crc") == fused, (erased, _run.kernel)


@pytest.mark.gpu
def test_fused_config3_cells(cuda):
    """BASELINE config 3's repair (RS(10,4), 1 MiB cells, data shard 0 = hops
    location 4 lost) over 48 stripes incl. all-0x00 / all-0xFF / ramp edge
    stripes; sampled stripes against the oracle."""
    torch = cuda
    k, p, L, S = 10, 4, 1 << 20, 48
    code = HipReedSolomonCode(k, p)
    st = _stripes(torch, S, k + p, L, seed=3)
    st[0] = 0
    st[1] = 0xFF
    st[2] = (torch.arange(L, device="cuda") % 256).to(torch.uint8)
    device.encode_stripes(code, st)
    erased = [4]
    to_read, ntr = _pattern(code, erased)
    got, crc, ref = _run(torch, code, st, erased)
    assert _run.kernel.startswith("decode_crc_pipe_kernel<1, 12")
    host = st.cpu().numpy()
    assert np.array_equal(got[:, 0], host[:, 4])  # codewords: the lost cell comes back
    assert np.array_equal(got, ref)
    _check_crcs(got, crc)
    _check_vs_oracle(k, p, host, got, erased, to_read, ntr, (0, 1, 2, S - 1))


@pytest.mark.gpu
def test_chaining_like_CRC32_update(cuda):
    """Successive bufSize rounds of one lost block: crc_in carries the running CRC."""
    torch = cuda
    k, p, L, S, rounds = 10, 4, 256 << 10, 3, 4
    code = HipReedSolomonCode(k, p)
    erased = [2, 9]
    crc = None
    outs = []
    for r in range(rounds):
        got, crc_h, _ = _run(torch, code, _stripes(torch, S, k + p, L, seed=50 + r), erased,
                             None if crc is None else crc)
        crc = torch.from_numpy(crc_h).cuda()
        outs.append(got)
    for s in range(S):
        for t in range(len(erased)):
            want = 0
            for o in outs:
                want = zlib.crc32(o[s, t].tobytes(), want)
            assert _u32(crc_h[s, t]) == want, (s, t)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["ragged", "unaligned", "forced_runtime", "four_of_ten", "small"])
def test_fallback_and_edges(cuda, case):
    torch = cuda
    k, p, L, S = 10, 4, 96 << 10, 3
    erased = [0, 4]
    pad = 0
    code = HipReedSolomonCode(k, p)
    if case == "ragged":
        L = 100000 + 7
    if case == "unaligned":
        pad = 3
    if case == "forced_runtime":
        code.setKernelMode(1)
    if case == "four_of_ten":
        erased = [0, 3, 6, 11]
    if case == "small":
        L, S = 2048, 1
    st = _stripes(torch, S, k + p, L, seed=7, pad=pad)
    got, crc, ref = _run(torch, code, st, erased)
    assert np.array_equal(got, ref)
    _check_crcs(got, crc)
    to_read, ntr = _pattern(code, erased)
    _check_vs_oracle(k, p, st.cpu().numpy(), got, erased, to_read, ntr, range(S))
    fused = case == "small"
    assert _run.kernel.startswith("decode_crc") == fused, _run.kernel


@pytest.mark.gpu
def test_crc_in_layout_and_errors(cuda):
    torch = cuda
    code = HipReedSolomonCode(10, 4)
    st = torch.zeros((2, 14, 32 << 10), dtype=torch.uint8, device="cuda")
    out = torch.empty((2, 1, 32 << 10), dtype=torch.uint8, device="cuda")
    _, ntr = _pattern(code, [5])
    with pytest.raises(ValueError):
        device.decode_stripes_crc(code, st, [5], ntr, out, torch.zeros((2, 2), dtype=torch.int32, device="cuda"))
    cin = torch.full((2, 1), 0x1234567, dtype=torch.int32, device="cuda")
    crc = device.decode_stripes_crc(code, st, [5], ntr, out, cin)
    torch.cuda.synchronize()
    _check_crcs(out.cpu().numpy(), crc.cpu().numpy(), cin.cpu().numpy())


@pytest.mark.gpu
def test_other_codes(cuda):
    """nrs (ISA-L Cauchy), xor and src repairs through the same call: outputs
    equal the plain device decode (itself pinned to the oracle in the codes'
    suites), CRCs equal zlib."""
    torch = cuda
    L, S = 16 << 10, 2
    cases = [(HipNativeReedSolomonCode(10, 4), [[3], [0, 12], [1, 5, 9]]),
             (HipNativeReedSolomonCode(6, 3), [[7], [0, 8]]),
             (HipXORCode(10, 1), [[0], [6]]),
             (HipSimpleRegeneratingCode(10, 6, 2), [[0], [8], [2, 13]])]
    for code, pats in cases:
        n = code.stripeSize() + code.paritySize()
        st = _stripes(torch, S, n, L, seed=n)
        for erased in pats:
            got, crc, ref = _run(torch, code, st, erased)
            assert np.array_equal(got, ref), (type(code).__name__, erased)
            _check_crcs(got, crc)


@pytest.mark.gpu
def test_mirror_checksum_methods_take_device_rows(cuda):
    """HipReedSolomonCode.encodeBulkCrc / decodeBulkCrc with device rows
    (one stripe, 1-D uint8 tensors) run the fused device calls and agree with
    the same methods on host rows (the pinned pipeline) and with zlib."""
    torch = cuda
    k, p, L = 10, 4, 512 << 10
    code = HipReedSolomonCode(k, p)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    data = [torch.randint(0, 256, (L,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    par = [torch.zeros(L, dtype=torch.uint8, device="cuda") for _ in range(p)]
    start = [(0x9E3779B9 * (i + 1)) & 0xFFFFFFFF for i in range(k + p)]
    crcs = code.encodeBulkCrc(data, par, start)
    hdata = [d.cpu().numpy() for d in data]
    hpar = [np.zeros(L, np.uint8) for _ in range(p)]
    assert crcs == HipReedSolomonCode(k, p, zero_inputs_after_encode=False).encodeBulkCrc(hdata, hpar, start)
    assert all(np.array_equal(a.cpu().numpy(), b) for a, b in zip(par, hpar))
    assert crcs == [zlib.crc32(r.tobytes(), s) for r, s in zip(hdata + hpar, start)]
    stripe = par + data  # hops order: parity first
    erased = [1, 7]
    to_read, ntr = _pattern(code, erased)
    outs = [torch.empty(L, dtype=torch.uint8, device="cuda") for _ in erased]
    got = code.decodeBulkCrc([stripe[i] if i in to_read else None for i in range(k + p)], outs, erased, to_read, ntr,
                             [5, 6])
    assert all(torch.equal(o, stripe[e]) for o, e in zip(outs, erased))
    assert got == [zlib.crc32(stripe[e].cpu().numpy().tobytes(), s) for e, s in zip(erased, [5, 6])]
