"""CPU tests of the product boundary: libhrs.so loads, exports every symbol
include/*.h declares (and nothing else), and its host-side logic (encode/decode matrices,
locationsToReadForDecode, argument and error handling) agrees with the
oracle. No coding call runs here (no GPU in this container)."""
import ctypes
import itertools
import os
import re

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, HrsError, TooManyErasedLocations, _lib
from oracle import rs_oracle as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NONE = -2  # HRS_DEVICE_NONE


def declared_symbols(header="hrs.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hrs_[a-z0-9_]+)\s*\(", src)))


def dynamic_symbols(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True)
    return {ln.split()[-1] for ln in out.stdout.splitlines() if ln.strip()} 


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = declared_symbols()
    assert len(names) >= 17
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(_lib.EXPORTS)
    assert b"gfx950" in _lib.lib().hrs_version()


@pytest.mark.parametrize("path,header", [(_lib.LIB_PATH, "hrs.h"), (_lib.PROBE_LIB_PATH, "hrs_probe.h")])
def test_library_exports_only_its_header(path, header):
    """The version scripts (lambdafs_amd/csrc/libhrs.map, libhrs_probe.map)
    keep the C++ internals local: each library's dynamic symbol table holds
    exactly the hrs_* entry points its header declares (plus HIP's per-TU
    __hip_cuid_ markers). In particular the product library carries no
    diagnostics: the HBM probes live in libhrs_probe.so only."""
    syms = {s for s in dynamic_symbols(path) if not s.startswith("__hip_cuid_")}
    assert syms == set(declared_symbols(header)), sorted(syms ^ set(declared_symbols(header)))[:10]
    if header == "hrs.h":
        assert not any(s.startswith("hrs_probe") for s in syms)
        assert b"rows_kernel" not in open(path, "rb").read()  # no probe kernels in the product code object
    else:
        assert set(syms) == set(_lib.PROBE_EXPORTS)


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"encode_static_kernel" in blob and b"bitsliced_kernel" in blob


@pytest.mark.parametrize("k,p", [(3, 2), (6, 3), (10, 4), (12, 4), (1, 1), (100, 10), (200, 55)])
def test_encode_matrix_matches_oracle(k, p):
    code = HipReedSolomonCode(k, p, device=NONE)
    G = code.encodeMatrix()
    for c in range(k):
        unit = [1 if j == c else 0 for j in range(k)]
        assert list(G[:, c]) == C.encode(k, p, unit)


def _probe_decode5(k, p, erased, to_read, ntr):
    n = k + p
    D = np.zeros((len(erased), n), dtype=np.uint8)
    for col in range(n):
        unit = [1 if j == col else 0 for j in range(n)]
        D[:, col] = C.decode5(k, p, unit, erased, to_read, ntr)
    return D


@pytest.mark.parametrize("k,p", [(10, 4), (6, 3), (12, 4)])
def test_decode_matrix_matches_oracle_all_small_patterns(k, p):
    code = HipReedSolomonCode(k, p, device=NONE)
    n = k + p
    for e in range(1, 3):
        for erased in itertools.combinations(range(n), e):
            erased = list(erased)
            to_read = sorted(C.locations_to_read(k, p, erased))
            ntr = [x for x in range(n) if x not in to_read]
            assert (code.decodeMatrix(erased, ntr) == _probe_decode5(k, p, erased, to_read, ntr)).all(), erased


def test_decode_matrix_odd_semantics():
    """Reference quirks the matrices must reproduce (ReedSolomonCode.java:144-166):
    an erased location missing from notToRead decodes to 0, and fewer
    notToRead locations than p use fewer syndromes."""
    k, p = 10, 4
    code = HipReedSolomonCode(k, p, device=NONE)
    for erased, ntr in [([4], [1, 2]), ([4, 9], [4]), ([0], [0, 13, 7]), ([5], [])]:
        D = code.decodeMatrix(erased, ntr)
        assert (D == _probe_decode5(k, p, erased, [], ntr)).all()


def test_decode3_matrix_matches_oracle():
    k, p = 10, 4
    n = k + p
    code = HipReedSolomonCode(k, p, device=NONE)
    for erased in ([4], [1, 5, 7], [0, 3, 9, 13]):
        D = code.decodeMatrix(erased, erased, zero_not_to_read=False)
        for col in range(n):
            rows = [np.full(1, 1 if j == col else 0, dtype=np.uint8) for j in range(n)]
            out = C.decode_bulk3(k, p, rows, erased)
            assert list(D[:, col]) == [int(o[0]) for o in out]


REPEATED5 = [([3], [3, 3]), ([3, 5], [3, 5, 5]), ([3, 3], [3, 5, 5]), ([3, 3], [3, 3]), ([4], [4, 4, 4, 4]),
             ([0, 13], [13, 0, 13]), ([7, 7, 7], [1, 7, 7, 2]), ([99, -1, 4], [4, 2]), ([5, 5], [])]
REPEATED3 = [[3, 3], [1, 5, 1], [2, 2, 2, 2], [13, 0, 13]]


def _gf_apply(D, rows):
    """out_t = XOR_l D[t][l] * rows[l] over GF(2^8), through the oracle's tables."""
    from oracle import rs_ref
    mul = np.array(rs_ref.MUL, dtype=np.uint8)
    out = np.zeros((D.shape[0], rows.shape[1]), dtype=np.uint8)
    for t in range(D.shape[0]):
        for l in range(D.shape[1]):
            if D[t, l]:
                out[t] ^= mul[D[t, l]][rows[l]]
    return out


@pytest.mark.parametrize("k,p", [(10, 4), (6, 3)])
def test_decode_matrix_repeated_locations_match_java(k, p):
    """VERDICT r5 missing #3: lists the Java accepts with repeated entries (a
    division by zero in solveVandermondeSystem is divTable[y][0] = 0,
    GaloisField.java:107-118) and, in the 5-arg form, erased locations of any
    value (ReedSolomonCode.java:158-165 only compares them). The matrix must
    reproduce the reference's per-byte bulk loops on arbitrary bytes."""
    n = k + p
    code = HipReedSolomonCode(k, p, device=NONE)
    rng = np.random.default_rng(k * 100 + p)
    rows = rng.integers(0, 256, (n, 257), dtype=np.uint8)
    for erased, ntr in REPEATED5:
        ntr = [x for x in ntr if x < n]
        D = code.decodeMatrix(erased, ntr)
        want = C.decode_bulk5(k, p, [r.copy() for r in rows], erased, [], ntr)
        assert (_gf_apply(D, rows) == np.array(want)).all(), (erased, ntr)
        assert (D == _probe_decode5(k, p, erased, [], ntr)).all(), (erased, ntr)
    for erased in REPEATED3:
        erased = [x for x in erased if x < n]
        D = code.decodeMatrix(erased, erased, zero_not_to_read=False)
        want = C.decode_bulk3(k, p, [r.copy() for r in rows], erased)
        assert (_gf_apply(D, rows) == np.array(want)).all(), erased


def test_decode_matrix_repeated_two_transcriptions():
    """The C oracle and the independent Python transcription agree on the
    repeated-location cases the engine now accepts (pins the oracle there)."""
    from oracle.rs_ref import ReedSolomonRef
    k, p = 10, 4
    ref = ReedSolomonRef(k, p)
    rng = np.random.default_rng(7)
    data = [int(v) for v in rng.integers(0, 256, k + p)]
    for erased, ntr in REPEATED5:
        assert ref.decode5(list(data), erased, [], ntr) == C.decode5(k, p, list(data), erased, [], ntr), (erased, ntr)


def test_decode_matrix_rejects_what_java_rejects():
    """A not-to-read location outside [0, n) throws in the Java
    (primitivePower / data index); so does a 3-arg erased one."""
    code = HipReedSolomonCode(10, 4, device=NONE)
    for erased, ntr, zero in [([3], [14], True), ([3], [-1], True), ([14], [14], False), ([-1], [-1], False)]:
        with pytest.raises(HrsError):
            code.decodeMatrix(erased, ntr, zero_not_to_read=zero)


def test_locations_to_read_matches_java():
    code = HipReedSolomonCode(10, 4, device=NONE)
    lib = _lib.lib()
    for erased in ([7], [], [0, 13], [4, 1, 5, 7]):
        out = (ctypes.c_int * 10)()
        assert lib.hrs_locations_to_read(code._h, _lib.int_array(erased), len(erased), out) == 0
        assert list(out) == C.locations_to_read(10, 4, erased) == code.locationsToReadForDecode(erased)
    out = (ctypes.c_int * 10)()
    st = lib.hrs_locations_to_read(code._h, _lib.int_array([0, 1, 2, 3, 4]), 5, out)
    assert st == _lib.HRS_ETOOMANY
    assert b"Locations  0 1 2 3 4" in lib.hrs_last_error(code._h)
    with pytest.raises(TooManyErasedLocations):
        code.locationsToReadForDecode([0, 1, 2, 3, 4])


def test_create_rejects_bad_geometry():
    for k, p in [(0, 4), (10, 0), (200, 56), (255, 1)]:
        with pytest.raises(HrsError) as ei:
            HipReedSolomonCode(k, p, device=NONE)
        assert ei.value.status == _lib.HRS_EINVAL
    assert HipReedSolomonCode(254, 1, device=NONE).stripeSize() == 254


def test_host_only_handle_refuses_coding():
    code = HipReedSolomonCode(3, 2, device=NONE)
    with pytest.raises(HrsError) as ei:
        code.encodeBulk([bytes(8)] * 3, [bytearray(8) for _ in range(2)])
    assert ei.value.status == _lib.HRS_EDEVICE


def test_geometry_accessors():
    code = HipReedSolomonCode(10, 4, device=NONE)
    assert (code.stripeSize(), code.paritySize(), code.symbolSize()) == (10, 4, 8)


def test_scalar_decode5_host_logic_keeps_unlisted_values(monkeypatch):
    """The mirror's scalar 5-arg decode (erasure_code.py) around its bulk call:
    data zeroed at locationsNotToRead, and erasedValues[i] written only when
    erasedLocations[i] is listed there (ReedSolomonCode.java:144-166). The bulk
    call is stood in for by the oracle's decodeBulk here (no GPU); the GPU test
    test_gpu_parity.py::test_scalar_decode5_leaves_unlisted_erased_values runs
    the engine."""
    import random
    k, p = 10, 4
    code = HipReedSolomonCode()
    code._k, code._p = k, p

    def bulk(rows, outs, erased, to_read, ntr):
        got = C.decode_bulk5(k, p, [np.asarray(r) for r in rows], erased, to_read, ntr)
        for o, g in zip(outs, got):
            o[:] = g

    monkeypatch.setattr(code, "decodeBulk", bulk)
    rnd = random.Random(7)
    for _ in range(30):
        data = [rnd.randrange(256) for _ in range(k + p)]
        ntr = sorted(rnd.sample(range(k + p), rnd.randrange(1, p + 1)))
        erased = sorted(rnd.sample(range(k + p), rnd.randrange(1, p + 1)))
        prefill = [rnd.randrange(256) for _ in erased]
        want_vals, want_data = C.decode5(k, p, data, erased, [], ntr, values=prefill, with_data=True)
        vals = list(prefill)
        code.decode(data, erased, vals, [], ntr)
        assert vals == want_vals and data == want_data
