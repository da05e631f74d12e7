"""Synchronous host-buffer calls straight over the caller's rows (round 5,
VERDICT r4 item 4; opt-in, HRS_HOST_DIRECT=1): the pages under a call's rows
are registered with HIP for the call and the zero-copy kernel reads the
inputs and writes the outputs in place (hrs_hostpath.cpp host_apply_direct),
instead of the staged copies.
Checked against the oracle (ReedSolomonCode.encodeBulk / decodeBulk 5-arg,
ReedSolomonCode.java:103-125, :191-211) and zlib, for the row layouts a JNI
caller produces (rows sharing pages with their neighbours included: only
pages wholly inside a row are registered, the head and tail columns go
through the staging), and for every case that must fall back to the staged
path (misaligned rows, pages already pinned, short rows).
hrs_last_host_path says which path a call took."""
import os
import threading
import zlib

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu

K, P, L = 10, 4, 1 << 20
DIRECT_FUZZ_SEED, DIRECT_FUZZ_CASES = 0xD1EC7, 16  # tests/tools/fuzz_long.py runs other seeds


@pytest.fixture(autouse=True)
def direct_on(monkeypatch):
    """The direct path is opt-in (HRS_HOST_DIRECT=1; hrs_hostpath.cpp
    host_direct_on): these tests turn it on."""
    monkeypatch.setenv("HRS_HOST_DIRECT", "1")
    monkeypatch.delenv("HRS_ZEROCOPY", raising=False)


def test_direct_path_is_opt_in(cuda, monkeypatch):
    """Without HRS_HOST_DIRECT=1 a call that qualifies takes the staged path."""
    monkeypatch.delenv("HRS_HOST_DIRECT")
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    rng = np.random.default_rng(12)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(K)]
    par = [np.zeros(L, np.uint8) for _ in range(P)]
    _encode_check(code, data, par, "staged")


def _rows_in(buf, n, length, offset, gap):
    """n rows of `length` bytes carved out of one buffer: the first at
    `offset`, each next one `gap` bytes after the previous row's end (a heap:
    rows share pages)."""
    return [buf[offset + i * (length + gap): offset + i * (length + gap) + length] for i in range(n)]


def _encode_check(code, data, par, path):
    code.encodeBulk(data, par)
    assert code.lastHostPath() == path
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    for o in range(P):
        assert np.array_equal(par[o], ref[o]), o


def test_direct_separate_rows(cuda):
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    rng = np.random.default_rng(1)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(K)]
    par = [np.full(L, 0xEE, np.uint8) for _ in range(P)]
    _encode_check(code, data, par, "direct")
    for x in par:
        x[:] = 0x11
    _encode_check(code, data, par, "direct")  # the first call unregistered its pages


def test_direct_rows_sharing_pages(cuda):
    """Rows laid out like small heap objects: 16-byte headers between them,
    so neighbouring rows share pages. Only the pages wholly inside a row are
    registered; the columns in the shared pages go through the staging."""
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    n = K + P
    Ls = (256 << 10) + 48  # a multiple of 16: every row stays 16-byte aligned
    buf = np.random.default_rng(2).integers(0, 256, n * (Ls + 16) + 64, dtype=np.uint8)
    rows = _rows_in(buf, n, Ls, 16, 16)
    data, par = rows[:K], rows[K:]
    code.encodeBulk(data, par)
    assert code.lastHostPath() == "direct"
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))


def test_fallbacks(cuda):
    torch = cuda
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    rng = np.random.default_rng(3)
    # misaligned rows: the staged path (the vector kernels need 16-byte rows)
    buf = rng.integers(0, 256, (K + P) * (L + 8) + 64, dtype=np.uint8)
    rows = _rows_in(buf, K + P, L, 8, 8)
    _encode_check(code, rows[:K], rows[K:], "staged")
    # pinned rows (hipHostMalloc'd by torch): nothing to register, the kernel
    # runs over them in place (the "pinned" path comes first)
    pin = torch.empty((K + P, L), dtype=torch.uint8, pin_memory=True).numpy()
    pin[:K] = rng.integers(0, 256, (K, L), dtype=np.uint8)
    _encode_check(code, list(pin[:K]), list(pin[K:]), "pinned")
    # short rows: below HRS_HOST_DIRECT_MIN the copies cost less than registering
    small = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(K)]
    out = [np.zeros(4096, np.uint8) for _ in range(P)]
    _encode_check(code, small, out, "staged")


def test_direct_thresholds(cuda):
    """96 KiB rows: a plain call stays staged (below HRS_HOST_DIRECT_MIN,
    128 KiB), a checksummed one goes direct (HRS_HOST_DIRECT_MIN_CRC, 48 KiB)."""
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    rng = np.random.default_rng(10)
    Ls = 96 << 10
    data = [rng.integers(0, 256, Ls, dtype=np.uint8) for _ in range(K)]
    par = [np.zeros(Ls, np.uint8) for _ in range(P)]
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    code.encodeBulk(data, par)
    assert code.lastHostPath() == "staged"
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    for x in par:
        x[:] = 0
    crcs = code.encodeBulkCrc(data, par)
    assert code.lastHostPath() == "direct"
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    assert crcs == [zlib.crc32(r.tobytes()) for r in data + list(ref)]


def test_direct_decode_with_unread_rows(cuda):
    """decodeBulk 5-arg with the Decoder's arrays (Decoder.java:303-338): the
    not-to-read rows are None and never registered; the repaired rows are
    written in place."""
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    rng = np.random.default_rng(4)
    n = K + P
    erased = [1, 4]
    tr = sorted(C.locations_to_read(K, P, erased))
    ntr = [x for x in range(n) if x not in tr]
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(n)]  # non-codeword: every coefficient counts
    reads = [rows[i] if i in tr else None for i in range(n)]
    outs = [np.zeros(L, np.uint8) for _ in erased]
    code.decodeBulk(reads, outs, erased, tr, ntr)
    assert code.lastHostPath() == "direct"
    ref = C.decode_bulk5(K, P, [r if r is not None else np.zeros(L, np.uint8) for r in reads], erased, tr, ntr)
    assert all(np.array_equal(outs[i], ref[i]) for i in range(len(erased)))


def test_direct_checksummed_calls(cuda):
    """encodeBulkCrc / decodeBulkCrc (Encoder.java:408-450, Decoder.java:222-229)
    straight over the caller's rows, CRCs continued from running values."""
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    rng = np.random.default_rng(5)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(K)]
    par = [np.zeros(L, np.uint8) for _ in range(P)]
    run = [int(x) for x in rng.integers(0, 1 << 32, K + P, dtype=np.uint64)]
    crcs = code.encodeBulkCrc(data, par, run)
    assert code.lastHostPath() == "direct"
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    cells = data + list(ref)
    assert crcs == [zlib.crc32(cells[i].tobytes(), run[i]) & 0xFFFFFFFF for i in range(K + P)]
    stripe = list(ref) + data
    erased = [P]
    tr = sorted(C.locations_to_read(K, P, erased))
    ntr = [x for x in range(K + P) if x not in tr]
    out = [np.zeros(L, np.uint8)]
    dcrc = code.decodeBulkCrc([stripe[i] if i in tr else None for i in range(K + P)], out, erased, tr, ntr, [7])
    assert code.lastHostPath() == "direct"
    assert np.array_equal(out[0], data[0])
    assert dcrc == [zlib.crc32(data[0].tobytes(), 7) & 0xFFFFFFFF]


def test_direct_rows_of_one_array(cuda):
    """Page-aligned rows back to back (one 2-D array, as the Python mirror's
    callers hold a stripe): their page ranges touch and merge into one
    registration; no head or tail columns."""
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    n = K + P
    raw = np.random.default_rng(9).integers(0, 256, (n + 2) * L + 4096, dtype=np.uint8)
    base = (-raw.ctypes.data) % 4096
    rows = _rows_in(raw[base:], n + 2, L, 0, 0)
    data, par = rows[P:n], rows[:P]
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    run = [7 * i for i in range(n)]
    crcs = code.encodeBulkCrc(data, par, run)
    assert code.lastHostPath() == "direct"
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    assert crcs == [zlib.crc32(np.array(r).tobytes(), c) for r, c in zip(data + list(ref), run)]
    erased = [0, P + 3]
    tr = sorted(C.locations_to_read(K, P, erased))
    ntr = [x for x in range(n) if x not in tr]
    want = [np.array(rows[e]) for e in erased]
    outs = rows[n:n + 2]
    code.decodeBulk([rows[i] if i in tr else None for i in range(n)], outs, erased, tr, ntr)
    assert code.lastHostPath() == "direct"
    assert all(np.array_equal(outs[j], want[j]) for j in range(2))


def _page_rows(n, length, offset, rng):
    """n rows, each `offset` bytes past a page boundary of its own buffer."""
    rows = []
    for _ in range(n):
        raw = rng.integers(0, 256, length + offset + 8192, dtype=np.uint8)
        base = (-raw.ctypes.data) % 4096
        rows.append(raw[base + offset: base + offset + length])
    return rows


@pytest.mark.parametrize("offset", [0, 16, 2048, 4000])
@pytest.mark.parametrize("length", [1 << 20, (1 << 20) + 784, (300 << 10) + 48])
def test_direct_head_tail_shapes(cuda, offset, length):
    """Head / tail columns of every width (none, 16 B, 2 KiB, 4,080 B; tails of
    0 to ~6 KiB): they run as one two-stripe launch, right-aligned behind a
    zero pad, and a checksummed call's segment CRCs are chained with the pad's
    length term removed. Parity, repaired rows and CRCs vs the oracle / zlib."""
    rng = np.random.default_rng(offset * 7 + length)
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    data = _page_rows(K, length, offset, rng)
    par = _page_rows(P, length, offset, rng)
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    code.encodeBulk(data, par)
    assert code.lastHostPath() == "direct"
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    for x in par:
        x[:] = 0x3C
    run = [int(x) for x in rng.integers(0, 1 << 32, K + P, dtype=np.uint64)]
    crcs = code.encodeBulkCrc(data, par, run)
    assert code.lastHostPath() == "direct"
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    cells = data + list(ref)
    assert crcs == [zlib.crc32(cells[i].tobytes(), run[i]) & 0xFFFFFFFF for i in range(K + P)]
    stripe = list(ref) + data
    erased = [P + 1, 2]
    tr = sorted(C.locations_to_read(K, P, erased))
    ntr = [x for x in range(K + P) if x not in tr]
    outs = _page_rows(len(erased), length, offset, rng)
    dcrc = code.decodeBulkCrc([stripe[i] if i in tr else None for i in range(K + P)], outs, erased, tr, ntr, [5, 6])
    assert code.lastHostPath() == "direct"
    assert all(np.array_equal(outs[j], stripe[e]) for j, e in enumerate(erased))
    assert dcrc == [zlib.crc32(stripe[e].tobytes(), 5 + j) & 0xFFFFFFFF for j, e in enumerate(erased)]


@pytest.fixture(params=["exclusive", "overlapping"])
def direct_turns(request, monkeypatch):
    """Concurrent callers: by default one direct call at a time (the others
    staged); HRS_HOST_DIRECT_EXCL=0 lets direct calls overlap, which is where
    the page claims (PageClaims) keep two calls off the same pages."""
    if request.param == "overlapping":
        monkeypatch.setenv("HRS_HOST_DIRECT_EXCL", "0")
    else:
        monkeypatch.delenv("HRS_HOST_DIRECT_EXCL", raising=False)
    return request.param


@pytest.mark.usefixtures("direct_turns")
def test_concurrent_calls_rows_sharing_pages(cuda):
    """Four threads, one codec each (one Encoder per mapper thread), whose
    rows are neighbours in one buffer (pages shared between the threads' rows):
    no call registers a page another row reaches into, so overlapping direct
    calls run side by side; every result is bit-exact."""
    n = K + P
    Ls = (128 << 10) + 16
    T, R = 4, 6
    buf = np.random.default_rng(6).integers(0, 256, T * n * (Ls + 16) + 64, dtype=np.uint8)
    rows = _rows_in(buf, T * n, Ls, 16, 16)
    errs, paths = [], []

    def body(t):
        try:
            code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
            mine = rows[t * n:(t + 1) * n]
            data, par = mine[:K], mine[K:]
            ref = C.encode_bulk(K, P, [np.array(d) for d in data])
            for _ in range(R):
                for x in par:
                    x[:] = 0
                code.encodeBulk(data, par)
                paths.append(code.lastHostPath())
                if not all(np.array_equal(par[o], ref[o]) for o in range(P)):
                    raise AssertionError(f"thread {t}: parity differs ({code.lastHostPath()} path)")
        except Exception as e:  # noqa: BLE001 - reported after the join
            errs.append(e)

    ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]
    assert set(paths) <= {"direct", "staged"} and "direct" in paths


@pytest.mark.usefixtures("direct_turns")
def test_concurrent_calls_sharing_input_rows(cuda):
    """Four threads encode the SAME input rows at once (a stripe read by
    several codecs): HIP would accept the same pages registered twice and
    then drop the mapping under the other call, so each call first claims its
    pages process-wide (PageClaims); a call that finds them held takes the
    staged path. Every result is bit-exact and the process stays healthy."""
    T, R = 4, 8
    rng = np.random.default_rng(8)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(K)]
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    errs, paths = [], []

    def body(t):
        try:
            code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
            par = [np.zeros(L, np.uint8) for _ in range(P)]
            for _ in range(R):
                code.encodeBulk(data, par)
                paths.append(code.lastHostPath())
                if not all(np.array_equal(par[o], ref[o]) for o in range(P)):
                    raise AssertionError(f"thread {t}: parity differs ({code.lastHostPath()} path)")
        except Exception as e:  # noqa: BLE001 - reported after the join
            errs.append(e)

    ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]
    assert set(paths) <= {"direct", "staged"} and len(paths) == T * R
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    par = [np.zeros(L, np.uint8) for _ in range(P)]
    code.encodeBulk(data, par)  # every claim was released
    assert code.lastHostPath() == "direct"


def _fz_code(fam, k, p, s):
    from lambdafs_amd import HipNativeReedSolomonCode, HipSimpleRegeneratingCode, HipXORCode
    code = {"rs": lambda: HipReedSolomonCode(k, p), "nrs": lambda: HipNativeReedSolomonCode(k, p),
            "xor": lambda: HipXORCode(k, 1), "src": lambda: HipSimpleRegeneratingCode(k, p, s)}[fam]()
    code.zero_inputs_after_encode = False
    return code


def _fz_encode_ref(fam, k, p, s, data):
    if fam == "rs":
        return C.encode_bulk(k, p, data)
    if fam == "nrs":
        return C.nrs_encode_bulk(k, p, data)
    if fam == "xor":
        return [C.xor_encode_bulk(k, data)]
    return C.src_encode_bulk(k, p, s, data)


def _fz_pattern(fam, k, p, s, rnd):
    """(erased, not_to_read, to_read) as Decoder.java:303-338 builds them."""
    n = k + p
    while True:
        if fam == "xor":
            e = rnd.randrange(n)
            return [e], [e], [x for x in range(n) if x != e]
        if fam == "nrs":
            m = rnd.randint(1, p)
            ntr = sorted(rnd.sample(range(n), m))
            return ntr[:rnd.randint(1, m)], ntr, [x for x in range(n) if x not in ntr]
        erased = sorted(rnd.sample(range(n), rnd.randint(1, p)))
        tr = C.locations_to_read(k, p, erased) if fam == "rs" else C.src_locations_to_read(k, p, s, erased)
        if tr is not None:
            tr = sorted(tr)
            return erased, [x for x in range(n) if x not in tr or x in erased], tr


def _fz_decode_ref(fam, k, p, s, reads, erased, ntr, tr):
    if fam == "rs":
        return C.decode_bulk5(k, p, reads, erased, tr, ntr)
    if fam == "nrs":
        return C.nrs_decode_bulk(k, p, reads, erased, ntr)
    if fam == "xor":
        return [C.xor_decode_bulk(k, reads, erased[0])]
    return C.src_decode_bulk(k, p, s, reads, erased, tr, ntr)


def _fz_report(case, fam, k, p, L, gap, rows, outs, want, erased, ntr, path):
    """What a failed direct-fuzz decode looked like: where the differing bytes
    lie relative to the rows' page boundaries, and whether the output still
    differs after a pause (a write that became visible late) and after the
    same call once more."""
    import time
    lines = [f"case {case} {fam} RS({k},{p}) L={L} gap={gap} erased={erased} ntr={ntr} path={path}",
             "row page offsets " + str([r.ctypes.data % 4096 for r in rows[:k + p + len(erased)]])]
    for j in range(len(erased)):
        d = np.flatnonzero(outs[j] != want[j])
        if d.size:
            lines.append(f"out {j}: {d.size} bytes differ, first {d[0]}, last {d[-1]}")
    time.sleep(0.05)
    lines.append("after 50 ms: " + str([int(np.count_nonzero(outs[j] != want[j])) for j in range(len(erased))]))
    return "\n".join(lines)


def test_direct_fuzz(cuda):
    """Seeded differential fuzz of the synchronous host calls over the
    caller's rows: code family (rs static / runtime shapes, nrs, xor, src) x
    row length (64 KiB .. 1.3 MiB, ragged) x row placement (16-byte offsets
    in a shared heap-like buffer, rows sharing pages) x call (encodeBulk,
    decodeBulk 5-arg, encodeBulkCrc / decodeBulkCrc for rs, nrs and xor).
    Non-codeword reads, bit-exact vs the oracle and zlib; at least half the
    calls must take the direct path (the rest are the staged fallbacks)."""
    import random
    rnd = random.Random(DIRECT_FUZZ_SEED)
    fams = ["rs", "rs", "nrs", "xor", "src"]
    paths = []
    for case in range(DIRECT_FUZZ_CASES):
        fam = fams[case % len(fams)]
        s = 0
        if fam == "rs":
            k, p = rnd.choice([(10, 4), (6, 3), (12, 4), (3, 2)]) if case % 2 else (rnd.randint(2, 14), rnd.randint(1, 5))
        elif fam == "nrs":
            k, p = rnd.choice([(10, 4), (6, 3), (rnd.randint(2, 12), rnd.randint(1, 4))])
        elif fam == "xor":
            k, p = rnd.randint(2, 12), 1
        else:
            k, p, s = rnd.choice([(10, 6, 2), (6, 3, 2), (10, 4, 3), (10, 4, 1)])
        n = k + p
        L = rnd.choice([1 << 20, (1 << 20) + 16 * rnd.randint(1, 400), 16 * rnd.randint(4096, 80000),
                        rnd.randint(65536, 1 << 20)])
        gap = rnd.choice([16, 48, 4096, 4096 * 3 + 16])
        nbuf = 2 * n + 2
        buf = np.random.default_rng(case).integers(0, 256, nbuf * (L + gap) + 8192, dtype=np.uint8)
        start = (-buf.ctypes.data) % 4096 + 16 * rnd.randint(0, 255)
        rows = _rows_in(buf[start:], nbuf, L, 0, gap)
        code = _fz_code(fam, k, p, s)
        data, par = rows[p:n], rows[:p]
        ref = _fz_encode_ref(fam, k, p, s, [np.array(d) for d in data])
        crc_ok = fam != "src" and rnd.random() < 0.5
        if crc_ok:
            run = [rnd.randrange(1 << 32) for _ in range(n)]
            got = code.encodeBulkCrc(data, par, run)
            want_crc = [zlib.crc32(np.array(r).tobytes(), c) for r, c in zip(data + list(ref), run)]
            if got != want_crc:
                raise AssertionError(f"encode CRCs: rows {[i for i in range(n) if got[i] != want_crc[i]]} differ; "
                                     + _fz_report(case, fam, k, p, L, gap, rows, par, ref, list(range(p)), [],
                                                  code.lastHostPath()))
        else:
            code.encodeBulk(data, par)
        paths.append(code.lastHostPath())
        if not all(np.array_equal(par[o], ref[o]) for o in range(p)):
            raise AssertionError("encode: " + _fz_report(case, fam, k, p, L, gap, rows, par, ref, list(range(p)), [],
                                                         paths[-1]))
        for r in rows[:p]:  # non-codeword reads: every decode coefficient counts
            r[:] = np.frombuffer(rnd.randbytes(L), np.uint8)
        erased, ntr, tr = _fz_pattern(fam, k, p, s, rnd)
        src = [np.array(r) for r in rows[:n]]  # the rows before the decode
        reads = [None if x in ntr else rows[x] for x in range(n)]
        outs = rows[n:n + len(erased)]
        if fam == "xor":
            reads = [np.zeros(L, np.uint8) if r is None else r for r in reads]
        ref_reads = [np.zeros(L, np.uint8) if (r is None and fam == "rs") else (None if r is None else np.array(r))
                     for r in reads]
        want = _fz_decode_ref(fam, k, p, s, ref_reads, erased, ntr, tr)
        if crc_ok:
            run = [rnd.randrange(1 << 32) for _ in erased]
            got = code.decodeBulkCrc(reads, outs, erased, tr, ntr, run)
            if got != [zlib.crc32(w.tobytes(), c) for w, c in zip(want, run)]:
                raise AssertionError("decode CRCs differ; " + _fz_report(case, fam, k, p, L, gap, rows, outs, want,
                                                                          erased, ntr, code.lastHostPath()))
        else:
            code.decodeBulk(reads, outs, erased, tr, ntr)
        paths.append(code.lastHostPath())
        if not all(np.array_equal(outs[j], want[j]) for j in range(len(erased))):
            raise AssertionError(_fz_report(case, fam, k, p, L, gap, rows, outs, want, erased, ntr, paths[-1]))
        assert all(np.array_equal(rows[x], src[x]) for x in range(n)), case  # the reads are left as they were
    # ragged lengths misalign every row after the first, and xor has no
    # one-pass CRC: those calls take the staged path
    if os.environ.get("HRS_HOST_DIRECT") == "1":
        assert paths.count("direct") >= len(paths) // 2, paths


@pytest.mark.parametrize("offset", [0, 48])
def test_direct_pageable_batches(cuda, offset):
    """Host batches on pageable memory with the direct path on: the whole
    pages of the batch are registered for the call and the stripes inside them
    run zero copy; with the batch 48 bytes past a page boundary the first and
    last stripes reach into partial pages and are staged; a device set {0, 0}
    registers each member's range. Parity vs the oracle, repaired cells vs the
    lost ones."""
    from lambdafs_amd import device
    k, p, S, Lc = 10, 4, 12, 64 << 10
    n = k + p
    rng = np.random.default_rng(offset + 5)
    raw = np.empty(S * n * Lc + 8192 + offset, np.uint8)
    base = (-raw.ctypes.data) % 4096 + offset
    st = raw[base:base + S * n * Lc].reshape(S, n, Lc)
    st[:, p:] = rng.integers(0, 256, (S, k, Lc), dtype=np.uint8)
    code = HipReedSolomonCode(k, p, device=0)
    device.encode_batch_host(code, st)
    assert code.lastHostPath() == "direct"
    for s in range(S):
        ref = C.encode_bulk(k, p, [st[s, p + c].copy() for c in range(k)])
        assert all((st[s, r] == ref[r]).all() for r in range(p)), s
    er = np.array([sorted(rng.choice(n, 2, replace=False)) for _ in range(S)], dtype=np.int32)
    out = np.full((S, 2, Lc), 0xEE, np.uint8)
    device.decode_batch_host(code, st, er, out)
    assert code.lastHostPath() == "direct"
    assert all(np.array_equal(out[s], st[s, er[s]]) for s in range(S))
    codes = [HipReedSolomonCode(k, p, device=0) for _ in range(2)]
    out[:] = 0xEE
    device.decode_batch_host_multi(codes, st, er, out)
    assert [c.lastHostPath() for c in codes] == ["direct", "direct"]
    assert all(np.array_equal(out[s], st[s, er[s]]) for s in range(S))
