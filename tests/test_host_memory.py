"""Which host memory the GPU may read and write in place (round 6, VERDICT r5
item 1). The synchronous host-buffer calls (hrs_encode / hrs_decode and their
checksummed forms, the JNI path) and the host batches run the zero-copy kernel
directly over the caller's memory ONLY when the runtime allocated it pinned
(hipHostMalloc, torch pin_memory: hrs_last_host_path "pinned"). Every other
host buffer is copied through the library's own pinned staging ("staged"),
including pageable memory the caller registered with hipHostRegister: a
registration maps the pages for the GPU without pinning them, and round 5's
long fuzz runs lost GPU writes to registered pages that moved during a kernel
("Platform constraint"). The round-5 "direct" path, which
registered the caller's pageable pages itself, is gone.

Every call is checked bit-exact against the oracle (ReedSolomonCode
encodeBulk / decodeBulk 5-arg, ReedSolomonCode.java:103-125, :191-211) and
zlib (java.util.zip.CRC32)."""
import ctypes
import random
import threading
import zlib

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, device
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu

K, P, L = 10, 4, 1 << 20
FUZZ_SEED, FUZZ_CASES = 0xD1EC7, 16  # tests/tools/fuzz_long.py runs other seeds
PAGE = 4096


def _hip():
    # the HIP runtime torch loaded (libhrs.so binds the same one: one soname)
    return ctypes.CDLL("libamdhip64.so.7")


def _page_aligned(nbytes, rng=None):
    raw = np.empty(nbytes + 2 * PAGE, np.uint8)
    base = (-raw.ctypes.data) % PAGE
    v = raw[base:base + (nbytes + PAGE - 1) // PAGE * PAGE]
    if rng is not None:
        v[:] = rng.integers(0, 256, v.size, dtype=np.uint8)
    return v, raw


class Registered:
    """hipHostRegister(mapped) of a numpy buffer for the `with` block."""

    def __init__(self, arr):
        self.arr = arr

    def __enter__(self):
        hip = _hip()
        st = hip.hipHostRegister(ctypes.c_void_p(self.arr.ctypes.data), ctypes.c_size_t(self.arr.nbytes),
                                 ctypes.c_uint(2))  # hipHostRegisterMapped
        assert st == 0, f"hipHostRegister: {st}"
        return self.arr

    def __exit__(self, *exc):
        assert _hip().hipHostUnregister(ctypes.c_void_p(self.arr.ctypes.data)) == 0


class HostMalloc:
    """A hipHostMalloc'd buffer as a numpy array."""

    def __init__(self, nbytes):
        self.p = ctypes.c_void_p()
        assert _hip().hipHostMalloc(ctypes.byref(self.p), ctypes.c_size_t(nbytes), ctypes.c_uint(0)) == 0
        self.arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self.p.value))

    def close(self):
        assert _hip().hipHostFree(self.p) == 0


def _all_calls(code, data, par, path, run_seed):
    """encodeBulk, encodeBulkCrc, decodeBulk and decodeBulkCrc over the rows;
    each must take `path` and match the oracle / zlib."""
    n = K + P
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    code.encodeBulk(data, par)
    assert code.lastHostPath() == path
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    for x in par:
        x[:] = 0x5A
    rng = np.random.default_rng(run_seed)
    run = [int(x) for x in rng.integers(0, 1 << 32, n, dtype=np.uint64)]
    crcs = code.encodeBulkCrc(data, par, run)
    assert code.lastHostPath() == path
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    cells = [np.array(d) for d in data] + list(ref)
    assert crcs == [zlib.crc32(cells[i].tobytes(), run[i]) & 0xFFFFFFFF for i in range(n)]
    stripe = list(par) + list(data)
    erased = [P + 1, 2]
    tr = sorted(C.locations_to_read(K, P, erased))
    ntr = [x for x in range(n) if x not in tr]
    want = [np.array(stripe[e]) for e in erased]
    return stripe, erased, tr, ntr, want


def test_registered_rows_are_staged(cuda):
    """Rows in pageable memory the caller registered with hipHostRegister:
    the zero-copy kernel must NOT run over them (its writes could land in a
    page that moved); every call copies through the pinned staging."""
    rng = np.random.default_rng(1)
    buf, _keep = _page_aligned((K + P + 2) * L, rng)
    rows = [buf[i * L:(i + 1) * L] for i in range(K + P + 2)]
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    with Registered(buf):
        data, par = rows[P:K + P], rows[:P]
        stripe, erased, tr, ntr, want = _all_calls(code, data, par, "staged", 2)
        outs = rows[K + P:]
        code.decodeBulk([stripe[i] if i in tr else None for i in range(K + P)], outs, erased, tr, ntr)
        assert code.lastHostPath() == "staged"
        assert all(np.array_equal(outs[j], want[j]) for j in range(2))
        for o in outs:
            o[:] = 0
        dcrc = code.decodeBulkCrc([stripe[i] if i in tr else None for i in range(K + P)], outs, erased, tr, ntr,
                                  [5, 6])
        assert code.lastHostPath() == "staged"
        assert all(np.array_equal(outs[j], want[j]) for j in range(2))
        assert dcrc == [zlib.crc32(want[j].tobytes(), 5 + j) & 0xFFFFFFFF for j in range(2)]
        # a 3-arg decode reading the registered rows
        o3 = [np.zeros(L, np.uint8) for _ in erased]
        code.decodeBulk(stripe, o3, erased)
        assert code.lastHostPath() == "staged"
        assert all(np.array_equal(o3[j], w) for j, w in
                   enumerate(C.decode_bulk3(K, P, [np.array(r) for r in stripe], erased)))


def test_registered_batches_are_staged(cuda):
    """Host batches (hrs_encode_batch_host / hrs_decode_batch_host and the
    device-set form) over a registered pageable array: staged, bit-exact."""
    k, p, S, Lc = 10, 4, 12, 64 << 10
    n = k + p
    rng = np.random.default_rng(3)
    flat, _keep = _page_aligned(S * n * Lc)
    st = flat[:S * n * Lc].reshape(S, n, Lc)
    st[:, p:] = rng.integers(0, 256, (S, k, Lc), dtype=np.uint8)
    oflat, _keep2 = _page_aligned(S * 2 * Lc)
    out = oflat[:S * 2 * Lc].reshape(S, 2, Lc)
    code = HipReedSolomonCode(k, p, device=0)
    with Registered(flat), Registered(oflat):
        device.encode_batch_host(code, st)
        assert code.lastHostPath() == "staged"
        for s in range(S):
            ref = C.encode_bulk(k, p, [st[s, p + c].copy() for c in range(k)])
            assert all((st[s, r] == ref[r]).all() for r in range(p)), s
        er = np.array([sorted(rng.choice(n, 2, replace=False)) for _ in range(S)], dtype=np.int32)
        out[:] = 0xEE
        device.decode_batch_host(code, st, er, out)
        assert code.lastHostPath() == "staged"
        assert all(np.array_equal(out[s], st[s, er[s]]) for s in range(S))
        codes = [HipReedSolomonCode(k, p, device=0) for _ in range(2)]
        out[:] = 0xEE
        device.decode_batch_host_multi(codes, st, er, out)
        assert [c.lastHostPath() for c in codes] == ["staged", "staged"]
        assert all(np.array_equal(out[s], st[s, er[s]]) for s in range(S))


def test_runtime_pinned_rows_take_pinned(cuda):
    """Rows the runtime allocated pinned (torch pin_memory, hipHostMalloc):
    the kernel runs over them in place, one launch, no staging."""
    torch = cuda
    rng = np.random.default_rng(4)
    n = K + P
    pin = torch.empty((n + 2, L), dtype=torch.uint8, pin_memory=True).numpy()
    pin[:] = rng.integers(0, 256, pin.shape, dtype=np.uint8)
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    stripe, erased, tr, ntr, want = _all_calls(code, list(pin[P:n]), list(pin[:P]), "pinned", 5)
    outs = [pin[n], pin[n + 1]]
    code.decodeBulk([stripe[i] if i in tr else None for i in range(n)], outs, erased, tr, ntr)
    assert code.lastHostPath() == "pinned"
    assert all(np.array_equal(outs[j], want[j]) for j in range(2))
    hm = HostMalloc((n + 2) * L)
    try:
        rows = [hm.arr[i * L:(i + 1) * L] for i in range(n + 2)]
        for r in rows:
            r[:] = rng.integers(0, 256, L, dtype=np.uint8)
        stripe, erased, tr, ntr, want = _all_calls(code, rows[P:n], rows[:P], "pinned", 6)
        code.decodeBulk([stripe[i] if i in tr else None for i in range(n)], rows[n:], erased, tr, ntr)
        assert code.lastHostPath() == "pinned"
        assert all(np.array_equal(rows[n + j], want[j]) for j in range(2))
    finally:
        hm.close()
    # a pinned batch: one zero-copy launch over the caller's stripes
    S, Lc = 8, 64 << 10
    st = torch.empty((S, n, Lc), dtype=torch.uint8, pin_memory=True).numpy()
    st[:, P:] = rng.integers(0, 256, (S, K, Lc), dtype=np.uint8)
    device.encode_batch_host(code, st)
    assert code.lastHostPath() == "pinned"
    for s in range(S):
        ref = C.encode_bulk(K, P, [st[s, P + c].copy() for c in range(K)])
        assert all((st[s, r] == ref[r]).all() for r in range(P)), s


def test_mixed_and_misaligned_rows_are_staged(cuda):
    """One pageable row among pinned ones, or pinned rows off 16-byte
    alignment: the call is staged, with the same results."""
    torch = cuda
    rng = np.random.default_rng(7)
    n = K + P
    pin = torch.empty((n, L), dtype=torch.uint8, pin_memory=True).numpy()
    pin[:] = rng.integers(0, 256, pin.shape, dtype=np.uint8)
    code = HipReedSolomonCode(K, P, zero_inputs_after_encode=False)
    data = list(pin[P:n])
    data[3] = np.array(data[3])  # pageable copy
    ref = C.encode_bulk(K, P, [np.array(d) for d in data])
    par = list(pin[:P])
    code.encodeBulk(data, par)
    assert code.lastHostPath() == "staged"
    assert all(np.array_equal(par[o], ref[o]) for o in range(P))
    flat = torch.empty(n * (L + 8) + 64, dtype=torch.uint8, pin_memory=True).numpy()
    flat[:] = rng.integers(0, 256, flat.size, dtype=np.uint8)
    rows = [flat[8 + i * (L + 8): 8 + i * (L + 8) + L] for i in range(n)]
    ref = C.encode_bulk(K, P, [np.array(r) for r in rows[P:]])
    code.encodeBulk(rows[P:], rows[:P])
    assert code.lastHostPath() == "staged"
    assert all(np.array_equal(rows[o], ref[o]) for o in range(P))


def test_concurrent_calls_sharing_input_rows(cuda):
    """Four threads, one codec each (one Encoder per mapper thread), encode
    the SAME pageable input rows at once: every call staged, bit-exact."""
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
    assert set(paths) == {"staged"} and len(paths) == T * R


def _rows_in(buf, n, length, offset, gap):
    """n rows of `length` bytes carved out of one buffer: the first at
    `offset`, each next one `gap` bytes after the previous row's end (a heap:
    rows share pages)."""
    return [buf[offset + i * (length + gap): offset + i * (length + gap) + length] for i in range(n)]


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
    """Where the differing bytes of a failed fuzz call lie."""
    lines = [f"case {case} {fam} RS({k},{p}) L={L} gap={gap} erased={erased} ntr={ntr} path={path}",
             "row page offsets " + str([r.ctypes.data % PAGE for r in rows[:k + p + len(erased)]])]
    for j in range(len(erased)):
        d = np.flatnonzero(outs[j] != want[j])
        if d.size:
            lines.append(f"out {j}: {d.size} bytes differ, first {d[0]}, last {d[-1]}")
    return "\n".join(lines)


def test_host_call_fuzz(cuda):
    """Seeded differential fuzz of the synchronous host calls: code family
    (rs static / runtime shapes, nrs, xor, src) x row length (64 KiB ..
    1.3 MiB, ragged) x row placement (16-byte offsets in a shared heap-like
    pageable buffer, rows sharing pages; one case in four in a pin_memory
    buffer) x call (encodeBulk, decodeBulk 5-arg, encodeBulkCrc /
    decodeBulkCrc for rs, nrs and xor). Non-codeword reads, bit-exact vs the
    oracle and zlib; the reads are left as they were."""
    torch = cuda
    rnd = random.Random(FUZZ_SEED)
    fams = ["rs", "rs", "nrs", "xor", "src"]
    paths = []
    for case in range(FUZZ_CASES):
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
        L_ = rnd.choice([1 << 20, (1 << 20) + 16 * rnd.randint(1, 400), 16 * rnd.randint(4096, 80000),
                         rnd.randint(65536, 1 << 20)])
        gap = rnd.choice([16, 48, 4096, 4096 * 3 + 16])
        nbuf = 2 * n + 2
        size = nbuf * (L_ + gap) + 8192
        if case % 4 == 3:
            buf = torch.empty(size, dtype=torch.uint8, pin_memory=True).numpy()
            buf[:] = np.random.default_rng(case).integers(0, 256, size, dtype=np.uint8)
        else:
            buf = np.random.default_rng(case).integers(0, 256, size, dtype=np.uint8)
        start = (-buf.ctypes.data) % PAGE + 16 * rnd.randint(0, 255)
        rows = _rows_in(buf[start:], nbuf, L_, 0, gap)
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
                                     + _fz_report(case, fam, k, p, L_, gap, rows, par, ref, list(range(p)), [],
                                                  code.lastHostPath()))
        else:
            code.encodeBulk(data, par)
        paths.append(code.lastHostPath())
        if not all(np.array_equal(par[o], ref[o]) for o in range(p)):
            raise AssertionError("encode: " + _fz_report(case, fam, k, p, L_, gap, rows, par, ref, list(range(p)),
                                                         [], paths[-1]))
        for r in rows[:p]:  # non-codeword reads: every decode coefficient counts
            r[:] = np.frombuffer(rnd.randbytes(L_), np.uint8)
        erased, ntr, tr = _fz_pattern(fam, k, p, s, rnd)
        src = [np.array(r) for r in rows[:n]]  # the rows before the decode
        reads = [None if x in ntr else rows[x] for x in range(n)]
        outs = rows[n:n + len(erased)]
        if fam == "xor":
            reads = [np.zeros(L_, np.uint8) if r is None else r for r in reads]
        ref_reads = [np.zeros(L_, np.uint8) if (r is None and fam == "rs") else (None if r is None else np.array(r))
                     for r in reads]
        want = _fz_decode_ref(fam, k, p, s, ref_reads, erased, ntr, tr)
        if crc_ok:
            run = [rnd.randrange(1 << 32) for _ in erased]
            got = code.decodeBulkCrc(reads, outs, erased, tr, ntr, run)
            if got != [zlib.crc32(w.tobytes(), c) for w, c in zip(want, run)]:
                raise AssertionError("decode CRCs differ; " + _fz_report(case, fam, k, p, L_, gap, rows, outs, want,
                                                                          erased, ntr, code.lastHostPath()))
        else:
            code.decodeBulk(reads, outs, erased, tr, ntr)
        paths.append(code.lastHostPath())
        if not all(np.array_equal(outs[j], want[j]) for j in range(len(erased))):
            raise AssertionError(_fz_report(case, fam, k, p, L_, gap, rows, outs, want, erased, ntr, paths[-1]))
        assert all(np.array_equal(rows[x], src[x]) for x in range(n)), case  # the reads are left as they were
    # ragged rows and chunks no one-pass CRC kernel takes use the copy engine
    assert set(paths) <= {"staged", "pinned", "copy_engine"}, paths
