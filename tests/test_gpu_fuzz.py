"""Seeded differential fuzz of the HIP engine against the oracle (restated
reference loops) and zlib, through the product's entry points.

The structured suites pin each feature at chosen shapes; this one walks the
cross product they sample sparsely: code family (rs / nrs / xor / src) x
(k, p) x cell length (1 byte, 16-byte and 2 KiB window edges, 32 KiB fused
windows, ragged) x row placement (16-byte aligned or not, padded stripe
pitch) x entry point (device encode, device decode, heterogeneous repair
batch, host-row encode/decode, fused encode + CRC-32, the host calls with
block checksums, asynchronous submit/collect rounds, host-memory batches).
Every case uses
non-codeword inputs where the entry point allows it, so every coefficient of
every matrix is exercised, and is compared bit for bit.

Reference anchors: ReedSolomonCode.encodeBulk/decodeBulk
(ReedSolomonCode.java:103-125, :191-211), NativeReedSolomonCode
(NativeReedSolomonCode.java:55-152), XORCode (XORCode.java:99-145),
SimpleRegeneratingCode (SimpleRegeneratingCode.java:28-482),
ErasureCode.locationsToReadForDecode (ErasureCode.java:89-113), CRC32 of
cells (Encoder.java:408-450).
"""
import random
import zlib

import numpy as np
import pytest

from lambdafs_amd import (HipNativeReedSolomonCode, HipReedSolomonCode, HipSimpleRegeneratingCode, HipXORCode,
                          device)
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu

CASES = 400
SEED = 0x5EED_F022
LENGTHS = [1, 15, 16, 17, 100, 2047, 2048, 2049, 4096 + 17, 32768, 65536, 32768 * 3 + 2048 + 5]
SRC_SHAPES = [(10, 6, 2), (6, 3, 2), (10, 4, 3), (10, 4, 1), (6, 3, 1), (12, 4, 1), (3, 2, 1), (10, 4, 2)]
STATIC_RS = [(10, 4), (6, 3), (3, 2), (12, 4)]
STATIC_NRS = [(10, 4), (6, 3)]


ENTRIES = {"rs": ["enc", "dec", "batch", "host", "crc", "hcrc", "async", "hbatch"],
           "nrs": ["enc", "dec", "host", "crc", "hcrc", "async"],
           "xor": ["enc", "dec", "host", "hcrc", "async"], "src": ["enc", "dec", "batch", "hbatch"]}
PAIRS = [(f, e) for f in ENTRIES for e in ENTRIES[f]]  # case i draws pair i % len(PAIRS), the rest at random


def _case(rnd, fam, entry):
    s = 0
    if fam == "rs":
        k, p = rnd.choice(STATIC_RS) if rnd.random() < 0.4 else (rnd.randint(1, 24), rnd.randint(1, 8))
    elif fam == "nrs":
        k, p = rnd.choice(STATIC_NRS) if rnd.random() < 0.4 else (rnd.randint(1, 20), rnd.randint(1, 6))
    elif fam == "xor":
        k, p = rnd.randint(1, 20), 1
    else:
        k, p, s = rnd.choice(SRC_SHAPES)
    L = rnd.choice(LENGTHS) if rnd.random() < 0.7 else rnd.randint(1, 70000)
    S = rnd.randint(1, 3)
    while S * (k + p) * L > (4 << 20) and S > 1:
        S -= 1
    if S * (k + p) * L > (4 << 20):
        L = max(1, (4 << 20) // (k + p))
    off = rnd.choice([0, 0, 16, 1, 3, 8])  # byte offset of the batch in its buffer
    pad = rnd.choice([0, 0, 16, 5])        # extra bytes of stripe pitch
    return fam, k, p, s, entry, L, S, off, pad


def _code(fam, k, p, s):
    if fam == "rs":
        return HipReedSolomonCode(k, p)
    if fam == "nrs":
        return HipNativeReedSolomonCode(k, p)
    if fam == "xor":
        return HipXORCode(k, 1)
    return HipSimpleRegeneratingCode(k, p, s)


def _stripes(torch, S, n, L, off, pad, seed):
    """[S, n, L] view into a flat device buffer at byte offset `off` with
    stripe pitch n*L + pad (rows unaligned whenever off or pitch is)."""
    pitch = n * L + pad
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    buf = torch.randint(0, 256, (off + S * pitch,), dtype=torch.uint8, device="cuda", generator=g)
    return buf[off:].as_strided((S, n, L), (pitch, L, 1))


def _ref_encode(fam, k, p, s, data):
    if fam == "rs":
        return C.encode_bulk(k, p, data)
    if fam == "nrs":
        return C.nrs_encode_bulk(k, p, data)
    if fam == "xor":
        return [C.xor_encode_bulk(k, data)]
    return C.src_encode_bulk(k, p, s, data)


def _pattern(fam, k, p, s, rnd, allow_empty=False):
    """(erased, not_to_read, to_read) as Decoder.java:303-338 builds them, or
    None when the code cannot repair the drawn pattern."""
    n = k + p
    if fam == "xor":
        e = rnd.randrange(n)
        return [e], [e], [x for x in range(n) if x != e]
    if fam == "nrs":
        m = rnd.randint(1, p)
        ntr = sorted(rnd.sample(range(n), m))
        return ntr[:rnd.randint(1, m)], ntr, [x for x in range(n) if x not in ntr]
    ne = rnd.randint(0 if allow_empty else 1, p)
    erased = sorted(rnd.sample(range(n), ne))
    tr = C.locations_to_read(k, p, erased) if fam == "rs" else C.src_locations_to_read(k, p, s, erased)
    if tr is None:
        return None
    tr = sorted(tr)
    return erased, [x for x in range(n) if x not in tr or x in erased], tr


def _ref_decode(fam, k, p, s, reads, erased, ntr, tr):
    if fam == "rs":
        return C.decode_bulk5(k, p, reads, erased, tr, ntr)
    if fam == "nrs":
        return C.nrs_decode_bulk(k, p, reads, erased, ntr)
    if fam == "xor":
        rows = [np.zeros_like(next(r for r in reads if r is not None)) if r is None else r for r in reads]
        return [C.xor_decode_bulk(k, rows, erased[0])]
    return C.src_decode_bulk(k, p, s, reads, erased, tr, ntr)


def _check_encode(torch, fam, k, p, s, st, host_before):
    S = st.shape[0]
    par = torch.full((S, p, st.shape[2]), 0xA5, dtype=torch.uint8, device="cuda")
    device.encode_rows(_code(fam, k, p, s), [st[:, p + c, :] for c in range(k)], [par[:, r, :] for r in range(p)])
    got = par.cpu().numpy()
    for i in range(S):
        ref = _ref_encode(fam, k, p, s, [host_before[i, p + c] for c in range(k)])
        assert all((got[i, r] == ref[r]).all() for r in range(p)), i
    return S * p


def _check_decode(torch, fam, k, p, s, st, host, rnd):
    n, rows = k + p, 0
    for _ in range(3):
        pat = _pattern(fam, k, p, s, rnd)
        if pat is None:
            continue
        erased, ntr, tr = pat
        out = torch.full((st.shape[0], len(erased), st.shape[2]), 0x5A, dtype=torch.uint8, device="cuda")
        device.decode_stripes(_code(fam, k, p, s), st, erased, ntr, out)
        got = out.cpu().numpy()
        for i in range(st.shape[0]):
            reads = [None if x in ntr else host[i, x] for x in range(n)]
            if fam == "rs":  # the reference reads zeros where the stream reader left none
                reads = [np.zeros_like(host[i, 0]) if r is None else r for r in reads]
            ref = _ref_decode(fam, k, p, s, reads, erased, ntr, tr)
            assert ref is not None
            assert all((got[i, j] == ref[j]).all() for j in range(len(erased))), (erased, ntr, i)
            rows += len(erased)
    return rows


def _check_batch(torch, fam, k, p, s, st, host, rnd):
    n, S, L = k + p, st.shape[0], st.shape[2]
    pats = []
    for _ in range(S):
        pat = None
        while pat is None:
            pat = _pattern(fam, k, p, s, rnd, allow_empty=True)
        pats.append(pat)
    E = max(1, max(len(pt[0]) for pt in pats))
    er = np.full((S, E), -1, dtype=np.int32)
    for i, pt in enumerate(pats):
        er[i, :len(pt[0])] = pt[0]
    out = torch.full((S, E, L), 0x5A, dtype=torch.uint8, device="cuda")
    device.decode_batch(_code(fam, k, p, s), st, er, out)
    got = out.cpu().numpy()
    rows = 0
    for i, (erased, ntr, tr) in enumerate(pats):
        if not erased:
            continue
        rows += len(erased)
        reads = [None if x in ntr else host[i, x] for x in range(n)]
        if fam == "rs":
            reads = [np.zeros_like(host[i, 0]) if r is None else r for r in reads]
        ref = _ref_decode(fam, k, p, s, reads, erased, ntr, tr)
        assert all((got[i, j] == ref[j]).all() for j in range(len(erased))), (i, erased)
    return rows


def _check_host(fam, k, p, s, host, rnd):
    n, L = k + p, host.shape[2]
    code = _code(fam, k, p, s)
    code.zero_inputs_after_encode = False
    data = [host[0, p + c].copy() for c in range(k)]
    par = [np.full(L, 0xA5, np.uint8) for _ in range(p)]
    code.encodeBulk(data, par)
    ref = _ref_encode(fam, k, p, s, data)
    assert all((a == b).all() for a, b in zip(par, ref))
    pat = _pattern(fam, k, p, s, rnd)
    if pat is None:
        return p
    erased, ntr, tr = pat
    reads = [None if x in ntr else host[0, x].copy() for x in range(n)]
    if fam == "xor":
        reads = [np.zeros(L, np.uint8) if r is None else r for r in reads]
    outs = [np.full(L, 0x5A, np.uint8) for _ in erased]
    code.decodeBulk(reads, outs, erased, tr, ntr)
    if fam == "rs":
        reads = [np.zeros(L, np.uint8) if r is None else r for r in reads]
    ref = _ref_decode(fam, k, p, s, reads, erased, ntr, tr)
    assert all((a == b).all() for a, b in zip(outs, ref)), (erased, ntr)
    return p + len(erased)


def _check_crc(torch, fam, k, p, s, st, host_before):
    S = st.shape[0]
    crc = device.encode_stripes_crc(_code(fam, k, p, s), st)
    after = st.cpu().numpy()
    got = crc.cpu().numpy().view(np.uint32)
    for i in range(S):
        data = [host_before[i, p + c] for c in range(k)]
        ref = _ref_encode(fam, k, p, s, data)
        assert all((after[i, r] == ref[r]).all() for r in range(p)), i
        want = [zlib.crc32(d.tobytes()) for d in data] + [zlib.crc32(r.tobytes()) for r in ref]
        assert list(got[i]) == want, i
    return S * (k + p)


def _host_pattern_reads(fam, k, p, s, host, rnd):
    """One decodable pattern and the reads the reference decoder sees for it."""
    pat = None
    while pat is None:
        pat = _pattern(fam, k, p, s, rnd)
    erased, ntr, tr = pat
    reads = [None if x in ntr else host[x].copy() for x in range(k + p)]
    if fam == "xor":
        reads = [np.zeros_like(host[0]) if r is None else r for r in reads]
    ref_reads = [np.zeros_like(host[0]) if (r is None and fam == "rs") else r for r in reads]
    return erased, ntr, tr, reads, ref_reads


def _check_hcrc(fam, k, p, s, host, rnd):
    """encodeBulkCrc / decodeBulkCrc (the Encoder's and Decoder's block
    checksums) with running CRCs continued from random values."""
    L = host.shape[2]
    code = _code(fam, k, p, s)
    code.zero_inputs_after_encode = False
    data = [host[0, p + c].copy() for c in range(k)]
    par = [np.full(L, 0xA5, np.uint8) for _ in range(p)]
    run = [rnd.randrange(1 << 32) for _ in range(k + p)]
    got = code.encodeBulkCrc(data, par, run)
    ref = _ref_encode(fam, k, p, s, data)
    assert all((a == b).all() for a, b in zip(par, ref))
    assert got == [zlib.crc32(r.tobytes(), c) for r, c in zip(data + list(ref), run)]
    erased, ntr, tr, reads, ref_reads = _host_pattern_reads(fam, k, p, s, host[0], rnd)
    outs = [np.full(L, 0x5A, np.uint8) for _ in erased]
    run = [rnd.randrange(1 << 32) for _ in erased]
    got = code.decodeBulkCrc(reads, outs, erased, tr, ntr, run)
    want = _ref_decode(fam, k, p, s, ref_reads, erased, ntr, tr)
    assert all((a == b).all() for a, b in zip(outs, want))
    assert got == [zlib.crc32(w.tobytes(), c) for w, c in zip(want, run)]
    return p + 2 * len(erased)


def _check_async(fam, k, p, s, host, rnd):
    """Asynchronous rounds: every stripe submitted (encode, then a decode of
    a fresh pattern) before any is collected, collected out of order."""
    L, S = host.shape[2], host.shape[0]
    code = _code(fam, k, p, s)
    code.zero_inputs_after_encode = False
    subs = []
    for i in range(min(S, 2)):
        data = [host[i, p + c].copy() for c in range(k)]
        subs.append(("enc", code.encodeBulkAsync(data, checksums=bool(i % 2)), data, i % 2))
        erased, ntr, tr, reads, ref_reads = _host_pattern_reads(fam, k, p, s, host[i], rnd)
        subs.append(("dec", code.decodeBulkAsync(reads, erased, tr, ntr), (erased, ntr, tr, ref_reads), 0))
    rows = 0
    for kind, ticket, arg, ck in reversed(subs):
        if kind == "enc":
            outs = [np.full(L, 0xA5, np.uint8) for _ in range(p)]
            crcs = code.collect(ticket, outs)
            ref = _ref_encode(fam, k, p, s, arg)
            assert all((a == b).all() for a, b in zip(outs, ref))
            if ck:
                assert crcs == [zlib.crc32(r.tobytes()) for r in list(arg) + list(ref)]
            rows += p
        else:
            erased, ntr, tr, ref_reads = arg
            outs = [np.full(L, 0x5A, np.uint8) for _ in erased]
            code.collect(ticket, outs)
            want = _ref_decode(fam, k, p, s, ref_reads, erased, ntr, tr)
            assert all((a == b).all() for a, b in zip(outs, want))
            rows += len(erased)
    assert code.pending() == 0
    return rows


def _check_hbatch(fam, k, p, s, host, rnd):
    """Host-memory batches (hrs_encode_batch_host, hrs_decode_batch_host):
    parity in place, then a per-stripe random pattern repaired from host
    memory, survivors only over PCIe."""
    n, S, L = k + p, host.shape[0], host.shape[2]
    code = _code(fam, k, p, s)
    st = host.copy()
    st[:, :p] = 0xA5
    device.encode_batch_host(code, st)
    for i in range(S):
        ref = _ref_encode(fam, k, p, s, [host[i, p + c] for c in range(k)])
        assert all((st[i, r] == ref[r]).all() for r in range(p)), i
    pats = []
    for _ in range(S):
        pat = None
        while pat is None:
            pat = _pattern(fam, k, p, s, rnd, allow_empty=True)
        pats.append(pat)
    E = max(1, max(len(pt[0]) for pt in pats))
    er = np.full((S, E), -1, dtype=np.int32)
    for i, pt in enumerate(pats):
        er[i, :len(pt[0])] = pt[0]
    src = host.copy()  # non-codeword rows: every coefficient counts
    out = np.full((S, E, L), 0x5A, np.uint8)
    device.decode_batch_host(code, src, er, out)
    rows = S * p
    for i, (erased, ntr, tr) in enumerate(pats):
        if not erased:
            continue
        reads = [None if x in ntr else src[i, x] for x in range(n)]
        if fam == "rs":
            reads = [np.zeros_like(src[i, 0]) if r is None else r for r in reads]
        want = _ref_decode(fam, k, p, s, reads, erased, ntr, tr)
        assert all((out[i, j] == want[j]).all() for j in range(len(erased))), (i, erased)
        rows += len(erased)
    return rows


def test_differential_fuzz(cuda):
    torch = cuda
    rnd = random.Random(SEED)
    rows = {pair: 0 for pair in PAIRS}  # output rows compared, per (family, entry point)
    for case in range(CASES):
        fam, k, p, s, entry, L, S, off, pad = _case(rnd, *PAIRS[case % len(PAIRS)])
        n = k + p
        st = _stripes(torch, S, n, L, off, pad, seed=SEED + case)
        host = st.cpu().numpy()
        where = (case, fam, k, p, s, entry, L, S, off, pad)
        try:
            if entry == "enc":
                got = _check_encode(torch, fam, k, p, s, st, host)
            elif entry == "dec":
                got = _check_decode(torch, fam, k, p, s, st, host, rnd)
            elif entry == "batch":
                got = _check_batch(torch, fam, k, p, s, st, host, rnd)
            elif entry == "host":
                got = _check_host(fam, k, p, s, host, rnd)
            elif entry == "hcrc":
                got = _check_hcrc(fam, k, p, s, host, rnd)
            elif entry == "async":
                got = _check_async(fam, k, p, s, host, rnd)
            elif entry == "hbatch":
                got = _check_hbatch(fam, k, p, s, host, rnd)
            else:
                got = _check_crc(torch, fam, k, p, s, st, host)
            rows[(fam, entry)] += got
        except AssertionError as e:
            raise AssertionError(f"fuzz case {where}: {e}") from None
    print("rows compared per (family, entry):", rows)
    assert all(v >= 10 for v in rows.values()), rows
