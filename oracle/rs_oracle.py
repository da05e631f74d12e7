"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C oracle (liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, as the checker or the timed CPU baseline. Rows are numpy uint8
arrays. The C code restates the reference Java loop for loop (rs_oracle.c).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    """Compile oracle/rs_oracle.c with gcc into oracle/liboracle.so."""
    src = os.path.join(_HERE, "rs_oracle.c")
    if os.path.exists(_LIB_PATH) and os.path.getmtime(_LIB_PATH) >= max(
        os.path.getmtime(src), os.path.getmtime(os.path.join(_HERE, "rs_oracle.h"))
    ):
        return _LIB_PATH
    subprocess.check_call(
        ["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-Wall", "-o", _LIB_PATH, src]
    )
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        I, P = ctypes.c_int, ctypes.c_void_p
        S = ctypes.c_size_t
        IP = ctypes.POINTER(ctypes.c_int)
        PP = ctypes.POINTER(ctypes.c_void_p)
        sigs = {
            "orc_gf_mul": ([I, I], I),
            "orc_gf_div": ([I, I], I),
            "orc_gf_power": ([I, I], I),
            "orc_gf_log": ([I], I),
            "orc_gf_pow_table": ([I], I),
            "orc_gf_poly_mul": ([IP, I, IP, I, IP], None),
            "orc_gf_poly_add": ([IP, I, IP, I, IP], None),
            "orc_gf_remainder": ([IP, I, IP, I], None),
            "orc_gf_substitute": ([IP, I, I], I),
            "orc_gf_solve_vandermonde": ([IP, IP, I], None),
            "orc_gf_gaussian_elimination": ([IP, I, I], None),
            "orc_rs_generator": ([I, I, IP], I),
            "orc_rs_encode": ([I, I, IP, IP], None),
            "orc_rs_encode_bulk": ([I, I, PP, PP, S], None),
            "orc_rs_decode3": ([I, I, IP, IP, I, IP], None),
            "orc_rs_decode5": ([I, I, IP, IP, I, IP, IP, I, IP, I], None),
            "orc_rs_decode_bulk5": ([I, I, PP, PP, IP, I, IP, I, IP, I, S], None),
            "orc_rs_decode_bulk3": ([I, I, PP, PP, IP, I, S], None),
            "orc_locations_to_read": ([I, I, IP, I, IP], I),
            "orc_rs_compute_error_locations": ([I, I, IP, IP, IP], I),
            "orc_xor_encode": ([I, IP, IP], None),
            "orc_xor_decode": ([I, IP, IP, I, IP], None),
            "orc_xor_encode_bulk": ([I, PP, ctypes.c_void_p, S], None),
            "orc_xor_decode_bulk": ([I, PP, ctypes.c_void_p, I, S], None),
            "orc_nrs_encode_matrix": ([I, I, ctypes.c_void_p], None),
            "orc_nrs_encode_bulk": ([I, I, PP, PP, S], None),
            "orc_nrs_decode_bulk": ([I, I, PP, PP, IP, I, IP, I, S], I),
            "orc_apache_gf_base": ([I], I),
            "orc_apache_gf_log_base": ([I], I),
            "orc_apache_gf_mul": ([I, I], I),
            "orc_apache_gf_inv": ([I], I),
            "orc_apache_gen_cauchy": ([ctypes.c_void_p, I, I], None),
            "orc_apache_rs_encode": ([I, I, PP, PP, S], None),
            "orc_apache_rs_decode": ([I, I, PP, IP, I, PP, S], I),
            "orc_legacy_generator": ([I, I, IP], I),
            "orc_legacy_rs_encode": ([I, I, PP, PP, S], None),
            "orc_legacy_rs_decode": ([I, I, PP, IP, I, PP, S], I),
            "orc_src_params": ([I, I, I, IP, IP, IP], I),
            "orc_src_encode": ([I, I, I, IP, IP], None),
            "orc_src_decode5": ([I, I, I, IP, IP, I, IP, IP, I, IP, I], I),
            "orc_src_locations_to_read": ([I, I, I, IP, I, IP], I),
            "orc_src_encode_bulk": ([I, I, I, PP, PP, S], None),
            "orc_src_decode_bulk": ([I, I, I, PP, PP, IP, I, IP, I, IP, I, S], I),
        }
        for name, (args, res) in sigs.items():
            f = getattr(_lib, name)
            f.argtypes = args
            f.restype = res
        del P
    return _lib


def _ints(values):
    arr = (ctypes.c_int * max(1, len(values)))(*values)
    return arr


def _rowptrs(rows):
    ptrs = (ctypes.c_void_p * max(1, len(rows)))()
    for i, r in enumerate(rows):
        if r is None:
            ptrs[i] = None
        else:
            assert r.dtype == np.uint8 and r.flags["C_CONTIGUOUS"]
            ptrs[i] = r.ctypes.data
    return ptrs


# --------------------------------------------------------------- GaloisField

def gf_mul(x, y):
    return lib().orc_gf_mul(x, y)


def gf_div(x, y):
    return lib().orc_gf_div(x, y)


def gf_power(x, n):
    return lib().orc_gf_power(x, n)


def poly_mul(p, q):
    out = _ints([0] * (len(p) + len(q) - 1))
    lib().orc_gf_poly_mul(_ints(p), len(p), _ints(q), len(q), out)
    return list(out)[: len(p) + len(q) - 1]


def poly_add(p, q):
    n = max(len(p), len(q))
    out = _ints([0] * n)
    lib().orc_gf_poly_add(_ints(p), len(p), _ints(q), len(q), out)
    return list(out)[:n]


def remainder(dividend, divisor):
    d = _ints(dividend)
    lib().orc_gf_remainder(d, len(dividend), _ints(divisor), len(divisor))
    return list(d)[: len(dividend)]


def substitute(p, x):
    return lib().orc_gf_substitute(_ints(p), len(p), x)


def solve_vandermonde(x, y):
    yy = _ints(y)
    lib().orc_gf_solve_vandermonde(_ints(x), yy, len(y))
    return list(yy)[: len(y)]


def gaussian_elimination(matrix):
    h, w = len(matrix), len(matrix[0])
    flat = _ints([v for row in matrix for v in row])
    lib().orc_gf_gaussian_elimination(flat, h, w)
    vals = list(flat)
    return [vals[i * w:(i + 1) * w] for i in range(h)]


# ------------------------------------------------------------ ReedSolomonCode

def generator(k, p):
    out = _ints([0] * (p + 1))
    assert lib().orc_rs_generator(k, p, out) == 0
    return list(out)[: p + 1]


def encode(k, p, message):
    par = _ints([0] * p)
    lib().orc_rs_encode(k, p, _ints(message), par)
    return list(par)[:p]


def encode_bulk(k, p, inputs, zero_inputs_ok=False):
    """ReedSolomonCode.encodeBulk. Returns the p parity rows. The Java zeroes
    its inputs; unless zero_inputs_ok, the rows are copied first."""
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in inputs]
    if not zero_inputs_ok:
        rows = [r.copy() for r in rows]
    L = rows[0].size
    outs = [np.zeros(L, dtype=np.uint8) for _ in range(p)]
    lib().orc_rs_encode_bulk(k, p, _rowptrs(rows), _rowptrs(outs), L)
    return outs


def decode3(k, p, data, erased):
    d = _ints(data)
    vals = _ints([0] * len(erased))
    lib().orc_rs_decode3(k, p, d, _ints(erased), len(erased), vals)
    return list(vals)[: len(erased)], list(d)[: len(data)]


def decode5(k, p, data, erased, to_read, not_to_read, values=None, with_data=False):
    """ReedSolomonCode.decode 5-arg (:144-166). `values` pre-fills erasedValues
    (the Java leaves an entry whose location is not in not_to_read as the caller
    passed it); with_data also returns `data` after the call (zeroed at
    not_to_read by the 3-arg decode it runs)."""
    d = _ints(data)
    vals = _ints(list(values) if values is not None else [0] * len(erased))
    lib().orc_rs_decode5(k, p, d, _ints(erased), len(erased), vals, _ints(to_read), len(to_read),
                         _ints(not_to_read), len(not_to_read))
    if with_data:
        return list(vals)[: len(erased)], list(d)[: len(data)]
    return list(vals)[: len(erased)]


def decode_bulk5(k, p, read_bufs, erased, to_read, not_to_read):
    rows = [None if r is None else np.ascontiguousarray(r, dtype=np.uint8) for r in read_bufs]
    L = max(r.size for r in rows if r is not None)
    outs = [np.zeros(L, dtype=np.uint8) for _ in erased]
    lib().orc_rs_decode_bulk5(k, p, _rowptrs(rows), _rowptrs(outs), _ints(erased), len(erased),
                              _ints(to_read), len(to_read), _ints(not_to_read), len(not_to_read), L)
    return outs


def decode_bulk3(k, p, read_bufs, erased):
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in read_bufs]
    L = rows[0].size
    outs = [np.zeros(L, dtype=np.uint8) for _ in erased]
    lib().orc_rs_decode_bulk3(k, p, _rowptrs(rows), _rowptrs(outs), _ints(erased), len(erased), L)
    return outs


def locations_to_read(k, p, erased):
    out = _ints([0] * k)
    got = lib().orc_locations_to_read(k, p, _ints(erased), len(erased), out)
    return list(out)[:got] if got == k else None


def compute_error_locations(k, p, data):
    d = _ints(data)
    locs = _ints([0] * (k + p))
    nloc = ctypes.c_int(0)
    ok = lib().orc_rs_compute_error_locations(k, p, d, locs, ctypes.byref(nloc))
    return bool(ok), set(list(locs)[: nloc.value]), list(d)[: len(data)]


# ------------------------------------------------------------------ XORCode

def xor_encode(k, message):
    par = _ints([0])
    lib().orc_xor_encode(k, _ints(message), par)
    return [par[0]]


def xor_decode(k, data, erased):
    vals = _ints([-1] * max(1, len(erased)))
    lib().orc_xor_decode(k, _ints(data), _ints(erased), len(erased), vals)
    return list(vals)[: len(erased)]


def xor_encode_bulk(k, inputs):
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in inputs]
    out = np.zeros(rows[0].size, dtype=np.uint8)
    lib().orc_xor_encode_bulk(k, _rowptrs(rows), out.ctypes.data, out.size)
    return out


def xor_decode_bulk(k, read_bufs, erased):
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in read_bufs]
    out = np.zeros(rows[0].size, dtype=np.uint8)
    lib().orc_xor_decode_bulk(k, _rowptrs(rows), out.ctypes.data, int(erased), out.size)
    return out


# ------------------------------------------------- nrs (ISA-L Cauchy RS)

def nrs_encode_matrix(k, p):
    a = np.zeros((k + p, k), dtype=np.uint8)
    lib().orc_nrs_encode_matrix(k, p, a.ctypes.data)
    return a


def nrs_encode_bulk(k, p, inputs):
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in inputs]
    outs = [np.zeros(rows[0].size, dtype=np.uint8) for _ in range(p)]
    lib().orc_nrs_encode_bulk(k, p, _rowptrs(rows), _rowptrs(outs), rows[0].size)
    return outs


def nrs_decode_bulk(k, p, read_bufs, erased, not_to_read):
    rows = [None if r is None else np.ascontiguousarray(r, dtype=np.uint8) for r in read_bufs]
    L = max(r.size for r in rows if r is not None)
    outs = [np.zeros(L, dtype=np.uint8) for _ in erased]
    st = lib().orc_nrs_decode_bulk(k, p, _rowptrs(rows), _rowptrs(outs), _ints(erased), len(erased),
                                   _ints(not_to_read), len(not_to_read), L)
    assert st == 0
    return outs


# ------------------------- Apache Java RS coder (RSRawEncoder / RSRawDecoder)

def apache_gen_cauchy(m, k):
    a = np.zeros((m, k), dtype=np.uint8)
    lib().orc_apache_gen_cauchy(a.ctypes.data, m, k)
    return a


def apache_rs_encode(k, p, inputs):
    """RSRawEncoder.encode: k data units -> p parity units (Apache order)."""
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in inputs]
    outs = [np.zeros(rows[0].size, dtype=np.uint8) for _ in range(p)]
    lib().orc_apache_rs_encode(k, p, _rowptrs(rows), _rowptrs(outs), rows[0].size)
    return outs


def apache_rs_decode(k, p, inputs, erased):
    """RSRawDecoder.decode: inputs[k + p] in Apache order (None = not read),
    erased unit indexes (ascending) -> their values."""
    rows = [None if r is None else np.ascontiguousarray(r, dtype=np.uint8) for r in inputs]
    L = max(r.size for r in rows if r is not None)
    outs = [np.zeros(L, dtype=np.uint8) for _ in erased]
    st = lib().orc_apache_rs_decode(k, p, _rowptrs(rows), _ints(erased), len(erased), _rowptrs(outs), L)
    assert st == 0, "RSRawDecoder: fewer than k inputs or singular"
    return outs


def hops_nrs_decode_via_apache(k, p, read_bufs, erased, not_to_read):
    """NativeReedSolomonCode.decodeBulk (NativeReedSolomonCode.java:90-148)
    with the reference's pure-Java RSRawDecoder in place of the native one it
    is interoperable with: hops rows [parity, data] -> Apache units [data,
    parity], the not-to-read units nulled and their sorted Apache indexes
    decoded, the first len(erased) outputs returned (the Java copies
    bwriteBufs[i] into writeBufs[i] for i < writeBufs.length)."""
    n = k + p
    units = [None] * n
    for i in range(p):
        units[i + k] = read_bufs[i]
    for i in range(k):
        units[i] = read_bufs[i + p]
    mod = []
    for loc in not_to_read:
        a = loc + k if loc < p else loc - p
        units[a] = None
        mod.append(a)
    mod.sort()
    outs = apache_rs_decode(k, p, units, mod)
    return outs[:len(erased)]


# ------------- hadoop-common's legacy RS coder (RSLegacyRawEncoder / Decoder)

def legacy_generator(k, p):
    g = (ctypes.c_int * (p + 1))()
    assert lib().orc_legacy_generator(k, p, g) == p + 1
    return list(g)


def legacy_rs_encode(k, p, inputs):
    """RSLegacyRawEncoder.encode: k data units -> p parity units (the same
    polynomial code as ReedSolomonCode.encodeBulk)."""
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in inputs]
    outs = [np.zeros(rows[0].size, dtype=np.uint8) for _ in range(p)]
    lib().orc_legacy_rs_encode(k, p, _rowptrs(rows), _rowptrs(outs), rows[0].size)
    return outs


def legacy_rs_decode(k, p, inputs, erased):
    """RSLegacyRawDecoder.decode: inputs[k + p] in Apache order [data,
    parity] (None = not read), erased Apache indexes -> their values, in the
    order given. Raises ValueError where the Java throws."""
    rows = [None if r is None else np.ascontiguousarray(r, dtype=np.uint8) for r in inputs]
    L = max(r.size for r in rows if r is not None)
    outs = [np.zeros(L, dtype=np.uint8) for _ in erased]
    st = lib().orc_legacy_rs_decode(k, p, _rowptrs(rows), _ints(erased), len(erased), _rowptrs(outs), L)
    if st != 0:
        raise ValueError({-1: "not enough valid inputs", -2: "inputs not fully corresponding to erasedIndexes",
                          -3: "more null inputs than parity units"}[st])
    return outs


def hops_to_apache(k, p, loc):
    """hops location (parity first) -> Apache unit index (data first)."""
    return loc + k if loc < p else loc - p


def hops_decode_via_legacy(k, p, read_bufs, erased, not_to_read):
    """ReedSolomonCode.decodeBulk 5-arg (ReedSolomonCode.java:191-211) worked
    by the legacy Apache coder: hops rows [parity, data] -> Apache units, the
    not-to-read units nulled, the erased units decoded (erased must be a
    subset of not_to_read, as Decoder.java:303-338 builds them); returns the
    erased values in hops `erased` order."""
    n = k + p
    units = [None] * n
    ntr = set(not_to_read)
    for loc in range(n):
        if loc not in ntr:
            units[hops_to_apache(k, p, loc)] = read_bufs[loc]
    ap = sorted(hops_to_apache(k, p, e) for e in erased)
    outs = legacy_rs_decode(k, p, units, ap)
    by_unit = dict(zip(ap, outs))
    return [by_unit[hops_to_apache(k, p, e)] for e in erased]


# ------------------------------------------- SimpleRegeneratingCode (src)

def src_params(k, p, s):
    """(s, r, d) after SimpleRegeneratingCode.init's adjustment loop."""
    a, b, c = _ints([0]), _ints([0]), _ints([0])
    lib().orc_src_params(k, p, s, a, b, c)
    return a[0], b[0], c[0]


def src_encode(k, p, s, message):
    par = _ints([0] * p)
    lib().orc_src_encode(k, p, s, _ints(message), par)
    return list(par)[:p]


def src_decode5(k, p, s, data, erased, to_read, not_to_read):
    """One symbol column; None where the Java would throw."""
    d = _ints(data)
    vals = _ints([0] * len(erased))
    st = lib().orc_src_decode5(k, p, s, d, _ints(erased), len(erased), vals, _ints(to_read), len(to_read),
                               _ints(not_to_read), len(not_to_read))
    return None if st else list(vals)[: len(erased)]


def src_locations_to_read(k, p, s, erased):
    """Ordered list, or None for TooManyErasedLocations."""
    out = _ints([0] * (k + p))
    m = lib().orc_src_locations_to_read(k, p, s, _ints(erased), len(erased), out)
    return None if m < 0 else list(out)[:m]


def src_encode_bulk(k, p, s, inputs):
    rows = [np.ascontiguousarray(r, dtype=np.uint8) for r in inputs]
    outs = [np.zeros(rows[0].size, dtype=np.uint8) for _ in range(p)]
    lib().orc_src_encode_bulk(k, p, s, _rowptrs(rows), _rowptrs(outs), rows[0].size)
    return outs


def src_decode_bulk(k, p, s, read_bufs, erased, to_read, not_to_read):
    rows = [None if r is None else np.ascontiguousarray(r, dtype=np.uint8) for r in read_bufs]
    L = max(r.size for r in rows if r is not None)
    outs = [np.zeros(L, dtype=np.uint8) for _ in erased]
    st = lib().orc_src_decode_bulk(k, p, s, _rowptrs(rows), _rowptrs(outs), _ints(erased), len(erased),
                                   _ints(to_read), len(to_read), _ints(not_to_read), len(not_to_read), L)
    return None if st else outs


# Raw entry points for the CPU baseline (pointer arrays prepared once).
def encode_bulk_ptrs(k, p, in_ptrs, out_ptrs, L):
    lib().orc_rs_encode_bulk(k, p, in_ptrs, out_ptrs, L)


def decode_bulk5_ptrs(k, p, in_ptrs, out_ptrs, erased, to_read, not_to_read, L):
    lib().orc_rs_decode_bulk5(k, p, in_ptrs, out_ptrs, _ints(erased), len(erased), _ints(to_read),
                              len(to_read), _ints(not_to_read), len(not_to_read), L)


rowptrs = _rowptrs
