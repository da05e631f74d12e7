"""The `nrs` codec pinned to reference source.

NativeReedSolomonCode calls libhadoop's native ISA-L coder, and ISA-L itself
is not in the reference, so the oracle's ISA-L restatement (orc_nrs_*) had no
reference-held anchor. The reference does hold a pure-Java port of that coder
— hadoop-common's RSRawEncoder / RSRawDecoder over RSUtil and GF256, "ported
from Intel ISA-L ... compatible with the native/ISA-L coder" — and its own
interop tests hold the two equal (TestRSRawCoderInteroperable1.java: Java
encode, native decode; ...Interoperable2.java: the reverse). oracle/rs_oracle.c
now restates that Java loop for loop (orc_apache_*), and this file checks:
  - the field tables of GF256.java (literal GF_BASE / GF_LOG_BASE, extracted
    as numbers by tools/extract_gf256_tables.py) against the Java
    restatement's, the hops GaloisField restatement's and the engine's;
  - the Cauchy matrix, every encode, and the hops wrapper's decode of every
    not-to-read pattern of RS(10,4) and RS(6,3) against the ISA-L restatement
    and the product's matrices (CPU);
  - the product's device encode / decode against the Java restatement, the
    interop pattern of the reference's tests (GPU).
"""
import itertools
import json
import os
import subprocess

import numpy as np
import pytest

from lambdafs_amd import HipNativeReedSolomonCode, device
from oracle import rs_oracle as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NONE = -2  # HRS_DEVICE_NONE


@pytest.fixture(scope="module")
def gf256():
    with open(os.path.join(ROOT, "tests", "golden", "gf256_tables.json")) as f:
        g = json.load(f)
    return g["GF_BASE"]["values"], g["GF_LOG_BASE"]["values"]


def test_java_restatement_tables_equal_reference_literals(gf256):
    base, logb = gf256
    assert len(base) == len(logb) == 256
    assert [C.lib().orc_apache_gf_base(i) for i in range(256)] == base
    assert [C.lib().orc_apache_gf_log_base(i) for i in range(256)] == logb
    assert logb[1] == 0xFF  # log(1) stored as 255: the quirk gfMul / gfInv rely on


def test_hops_and_engine_field_tables_equal_reference_literals(gf256):
    """The hops GaloisField (poly 285, computed tables) and the engine's
    gf256.hpp tables are the same field as GF256.java's literals."""
    base, logb = gf256
    L = C.lib()
    assert [L.orc_gf_pow_table(i) for i in range(255)] == base[:255]
    assert [L.orc_gf_log(x) for x in range(2, 256)] == logb[2:]
    tool = os.path.join(ROOT, "tests", "cpp", "crc_tables")
    if not os.path.exists(tool):
        subprocess.check_call(["make", "-C", ROOT, "tests/cpp/crc_tables"])
    eng = json.loads(subprocess.run([tool], capture_output=True, text=True, check=True).stdout)
    assert eng["gf_exp"][:255] == base[:255] and eng["gf_exp"][255:510] == base[:255]
    assert eng["gf_log"][2:] == logb[2:] and eng["gf_log"][1] == 0


def test_java_multiply_and_inverse_equal_hops_field():
    L = C.lib()
    for a in range(256):
        for b in range(0, 256, 7):
            assert L.orc_apache_gf_mul(a, b) == L.orc_gf_mul(a, b)
        if a:
            assert L.orc_apache_gf_mul(a, L.orc_apache_gf_inv(a)) == 1


@pytest.mark.parametrize("k,p", [(10, 4), (6, 3), (3, 2), (20, 8), (100, 10)])
def test_cauchy_matrix_three_ways(k, p):
    a = C.apache_gen_cauchy(k + p, k)
    assert (a == C.nrs_encode_matrix(k, p)).all()
    code = HipNativeReedSolomonCode(k, p, device=NONE)
    assert (code.encodeMatrix() == a[k:]).all()  # parity r = Apache unit k + r


@pytest.mark.parametrize("k,p,L", [(10, 4, 1000), (6, 3, 77), (3, 2, 8), (20, 8, 64), (100, 10, 33)])
def test_encode_java_vs_isal_restatement(k, p, L):
    rng = np.random.default_rng(k * 100 + p)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    a = C.apache_rs_encode(k, p, data)
    b = C.nrs_encode_bulk(k, p, data)
    assert all((x == y).all() for x, y in zip(a, b))


@pytest.mark.parametrize("k,p", [(10, 4), (6, 3)])
def test_every_not_to_read_pattern_java_vs_isal_and_product(k, p):
    """Non-codeword rows (every coefficient counts); outputs in the Java's
    order (output t = the t-th not-to-read unit in Apache order)."""
    n, L = k + p, 48
    rng = np.random.default_rng(7 + k)
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(n)]
    code = HipNativeReedSolomonCode(k, p, device=NONE)
    mul = np.array([[C.lib().orc_gf_mul(a, b) for b in range(256)] for a in range(256)], np.uint8)
    count = 0
    for m in range(1, p + 1):
        for ntr in itertools.combinations(range(n), m):
            ntr = list(ntr)
            rb = [None if j in ntr else rows[j] for j in range(n)]
            java = C.hops_nrs_decode_via_apache(k, p, rb, ntr, ntr)
            isal = C.nrs_decode_bulk(k, p, rb, ntr, ntr)
            assert all((x == y).all() for x, y in zip(java, isal)), ntr
            D = code.decodeMatrix(ntr, ntr)  # product: ne x n over hops locations
            prod = [np.zeros(L, np.uint8) for _ in ntr]
            for t in range(len(ntr)):
                for j in range(n):
                    if D[t, j]:
                        prod[t] ^= mul[D[t, j]][rows[j]]
            assert all((x == y).all() for x, y in zip(java, prod)), ntr
            count += 1
    assert count == sum(len(list(itertools.combinations(range(n), m))) for m in range(1, p + 1))


@pytest.mark.gpu
@pytest.mark.parametrize("k,p,L", [(10, 4, (64 << 10) + 5), (6, 3, 8192)])
def test_device_nrs_interoperates_with_java_coder(cuda, k, p, L):
    """TestRSRawCoderInteroperable1/2 pattern with the product as one side:
    device encode vs the Java encoder, and device repairs of random patterns
    of a Java-encoded stripe batch vs the Java decoder (through the hops
    wrapper's index mapping)."""
    torch = cuda
    n, S = k + p, 6
    rng = np.random.default_rng(L)
    host = np.zeros((S, n, L), np.uint8)
    for s in range(S):
        data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        host[s, p:] = np.stack(data)
        host[s, :p] = np.stack(C.apache_rs_encode(k, p, data))  # Java-encoded parity, hops order
    code = HipNativeReedSolomonCode(k, p, device=0)
    st = torch.from_numpy(host).cuda()
    st_enc = st.clone()
    st_enc[:, :p] = 0
    device.encode_stripes(code, st_enc)
    assert torch.equal(st_enc, st)  # device encode == Java encode
    for trial in range(4):
        m = 1 + trial % p
        ntr = sorted(rng.choice(n, m, replace=False).tolist())
        out = torch.empty((S, m, L), dtype=torch.uint8, device="cuda")
        device.decode_stripes(code, st, ntr, ntr, out)
        got = out.cpu().numpy()
        for s in range(S):
            rb = [None if j in ntr else host[s, j] for j in range(n)]
            java = C.hops_nrs_decode_via_apache(k, p, rb, ntr, ntr)
            for t in range(m):
                assert np.array_equal(got[s, t], java[t]), (ntr, s, t)
