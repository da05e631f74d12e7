"""GPU parity tests: the HIP engine (through libhrs.so's C ABI) against the CPU
oracle (restated reference loops) and the committed golden vectors.

Bar: bit-exact. Small sizes are compared in full against the oracle; the
BASELINE.json full-size configs are checked through size-independent
properties (encode -> erase -> decode round trips over every stripe) plus a
full oracle comparison of sampled stripes.
"""
import itertools
import random

import numpy as np
import pytest

from lambdafs_amd import Codec, HipReedSolomonCode, HrsError, TooManyErasedLocations, device
from lambdafs_amd import codec as codec_mod
from oracle import rs_oracle as C

pytestmark = pytest.mark.gpu


def rand_stripes(torch, S, n, L, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)


def oracle_parity(k, p, stripe_np):
    return np.stack(C.encode_bulk(k, p, [stripe_np[p + c] for c in range(k)]))


# ------------------------------------------------------------- golden vectors

def test_golden_vectors_host_api(cuda, golden):
    for cs in golden["cases"]:
        k, p, L = cs["k"], cs["p"], cs["len"]
        code = HipReedSolomonCode(k, p)
        data = [bytearray.fromhex(h) for h in cs["data_hex"]]
        par = [bytearray(L) for _ in range(p)]
        code.encodeBulk(data, par)
        assert [x.hex() for x in par] == cs["parity_hex"], cs["name"]
        assert all(not any(d) for d in data)  # reference side effect: inputs zeroed
        stripe = [bytes.fromhex(h) for h in cs["parity_hex"] + cs["data_hex"]]
        for d in cs["decodes"]:
            reads = [stripe[i] if i in d["locations_to_read_array"] else bytes(L) for i in range(k + p)]
            outs = [bytearray(L) for _ in d["erased"]]
            code.decodeBulk(reads, outs, d["erased"], d["locations_to_read_array"], d["locations_not_to_read_array"])
            assert [o.hex() for o in outs] == d["outputs_hex"], (cs["name"], d["erased"])
            if d["decode3_outputs_hex"] is not None:
                reads3 = [bytes(L) if i in d["erased"] else stripe[i] for i in range(k + p)]
                outs3 = [bytearray(L) for _ in d["erased"]]
                code.decodeBulk(reads3, outs3, d["erased"])
                assert [o.hex() for o in outs3] == d["decode3_outputs_hex"]


def test_golden_vectors_device_rows(cuda, golden):
    torch = cuda
    for cs in golden["cases"]:
        k, p = cs["k"], cs["p"]
        code = HipReedSolomonCode(k, p)
        data = [torch.tensor(list(bytes.fromhex(h)), dtype=torch.uint8, device="cuda") for h in cs["data_hex"]]
        par = [torch.zeros(cs["len"], dtype=torch.uint8, device="cuda") for _ in range(p)]
        code.encodeBulk(data, par)
        torch.cuda.synchronize()
        assert [bytes(x.cpu().numpy()).hex() for x in par] == cs["parity_hex"]


# ------------------------------------------------------ encode vs oracle, sizes

@pytest.mark.parametrize("k,p", [(3, 2), (6, 3), (10, 4), (12, 4), (5, 2), (20, 7), (40, 9), (1, 1), (64, 12)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_encode_batch_matches_oracle(cuda, k, p, mode):
    torch = cuda
    code = HipReedSolomonCode(k, p)
    code.setKernelMode(mode)
    for L, S in [(1, 3), (16, 2), (2047, 2), (2048, 3), (2049, 2), (6244, 3), (65536, 2)]:
        st = rand_stripes(torch, S, k + p, L, seed=L * 7 + k)
        st[:, :p, :] = 0xA5  # poison: must be overwritten
        device.encode_stripes(code, st)
        torch.cuda.synchronize()
        host = st.cpu().numpy()
        for s in range(S):
            assert (host[s, :p] == oracle_parity(k, p, host[s])).all(), (k, p, mode, L, s)


def test_kernel_modes_agree_at_full_cell_size(cuda):
    torch = cuda
    k, p, L, S = 10, 4, 1 << 20, 8
    st = rand_stripes(torch, S, k + p, L, seed=3)
    outs = []
    for mode in (0, 1, 2):
        code = HipReedSolomonCode(k, p)
        code.setKernelMode(mode)
        x = st.clone()
        device.encode_stripes(code, x)
        outs.append(x[:, :p].clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    host = st.cpu().numpy()
    ref = oracle_parity(k, p, host[5])
    assert (outs[0][5].cpu().numpy() == ref).all()


def test_unaligned_rows_use_bytewise_kernel(cuda):
    torch = cuda
    k, p, L = 10, 4, 5000
    code = HipReedSolomonCode(k, p)
    buf = torch.randint(0, 256, ((k + p) * (L + 1) + 64,), dtype=torch.uint8, device="cuda")
    data = [buf[1 + i * (L + 1): 1 + i * (L + 1) + L] for i in range(k)]  # odd offsets
    par = [torch.zeros(L + 3, dtype=torch.uint8, device="cuda")[3:] for _ in range(p)]
    code.encodeBulk(data, par)
    torch.cuda.synchronize()
    ref = C.encode_bulk(k, p, [d.cpu().numpy() for d in data])
    assert all((a.cpu().numpy() == b).all() for a, b in zip(par, ref))


# --------------------------------------------------------- decode vs oracle

def _decode_case(code, torch, k, p, erased, L, S, seed, codeword):
    n = k + p
    st = rand_stripes(torch, S, n, L, seed)
    if codeword:
        device.encode_stripes(code, st)
    to_read = sorted(C.locations_to_read(k, p, erased))
    ntr = [x for x in range(n) if x not in to_read]
    out = torch.full((S, len(erased), L), 0x5A, dtype=torch.uint8, device="cuda")
    device.decode_stripes(code, st, erased, ntr, out)
    torch.cuda.synchronize()
    host, got = st.cpu().numpy(), out.cpu().numpy()
    for s in range(S):
        reads = [host[s, i] if i in to_read else np.zeros(L, np.uint8) for i in range(n)]
        ref = C.decode_bulk5(k, p, reads, erased, to_read, ntr)
        assert all((got[s, i] == ref[i]).all() for i in range(len(erased))), (erased, s)
        if codeword:
            assert all((got[s, i] == host[s, e]).all() for i, e in enumerate(erased))


@pytest.mark.parametrize("k,p", [(10, 4), (6, 3), (12, 4), (3, 2)])
def test_decode_every_one_and_two_erasure_pattern(cuda, k, p):
    code = HipReedSolomonCode(k, p)
    n = k + p
    pats = [list(c) for e in (1, 2) for c in itertools.combinations(range(n), e) if e <= p]
    for i, erased in enumerate(pats):
        # arbitrary (non-codeword) inputs exercise the whole linear map
        _decode_case(code, cuda, k, p, erased, L=2048 + 33, S=2, seed=i, codeword=(i % 3 == 0))


def test_decode_random_three_and_four_erasures(cuda):
    rnd = random.Random(7)
    for k, p in [(10, 4), (12, 4), (6, 3)]:
        code = HipReedSolomonCode(k, p)
        for t in range(25):
            e = rnd.choice([x for x in (3, 4) if x <= p])
            erased = sorted(rnd.sample(range(k + p), e))
            _decode_case(code, cuda, k, p, erased, L=rnd.choice([1, 100, 4096, 10000]), S=2, seed=100 + t,
                         codeword=bool(t % 2))


def test_decode_host_api_with_null_unread_rows(cuda):
    k, p, L = 10, 4, 3000
    n = k + p
    code = HipReedSolomonCode(k, p)
    rng = np.random.default_rng(1)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    par = [np.zeros(L, np.uint8) for _ in range(p)]
    code.zero_inputs_after_encode = False
    code.encodeBulk(data, par)
    stripe = par + data
    erased = [4]
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(n) if x not in to_read]
    reads = [stripe[i] if i in to_read else None for i in range(n)]
    out = [np.zeros(L, np.uint8)]
    code.decodeBulk(reads, out, erased, to_read, ntr)
    assert (out[0] == data[0]).all()


def test_decode3_matches_oracle(cuda):
    torch = cuda
    rng = np.random.default_rng(9)
    for k, p in [(10, 4), (3, 3)]:
        code = HipReedSolomonCode(k, p)
        n = k + p
        for erased in ([p], [0, n - 1], list(range(p))):
            rows = [rng.integers(0, 256, 5000, dtype=np.uint8) for _ in range(n)]
            outs = [np.zeros(5000, np.uint8) for _ in erased]
            code.decodeBulk(rows, outs, erased)
            ref = C.decode_bulk3(k, p, rows, erased)
            assert all((a == b).all() for a, b in zip(outs, ref))
            # device rows take the hrs_apply_dev path
            drows = [torch.from_numpy(r).cuda() for r in rows]
            douts = [torch.zeros(5000, dtype=torch.uint8, device="cuda") for _ in erased]
            code.decodeBulk(drows, douts, erased)
            torch.cuda.synchronize()
            assert all((a.cpu().numpy() == b).all() for a, b in zip(douts, ref))


# ----------------------------------------------- full-size BASELINE configs

def test_config1_rs32_1mib_fixture_on_gpu(cuda):
    """BASELINE configs[0]: RS(3,2) encode of one 1 MiB stripe, the input
    java.util.Random(0x5EED0001).nextBytes (HEC-T/Util.java:97-106), through
    the host API (the JNI path) and a device row batch; both must reproduce
    the committed parity SHA-256 of tests/golden/config1_rs_3_2_1mib.json."""
    import hashlib
    import json
    import os
    from oracle.java_random import random_bytes
    torch = cuda
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "tests", "golden", "config1_rs_3_2_1mib.json")) as f:
        cfg = json.load(f)
    L = cfg["len"]
    buf = random_bytes(0x5EED0001, 3 * L)
    assert hashlib.sha256(buf).hexdigest() == cfg["input_sha256"]
    rows = [np.frombuffer(buf[i * L:(i + 1) * L], dtype=np.uint8).copy() for i in range(3)]
    code = HipReedSolomonCode(3, 2, device=0, zero_inputs_after_encode=False)
    par = [np.zeros(L, np.uint8) for _ in range(2)]
    code.encodeBulk(rows, par)
    assert [hashlib.sha256(r.tobytes()).hexdigest() for r in par] == cfg["parity_sha256"]
    st = torch.zeros((1, 5, L), dtype=torch.uint8, device="cuda")
    st[0, 2:] = torch.from_numpy(np.stack(rows)).cuda()
    device.encode_stripes(code, st)
    host = st.cpu().numpy()
    assert [hashlib.sha256(host[0, r].tobytes()).hexdigest() for r in range(2)] == cfg["parity_sha256"]


def test_config2_rs63_64k_10k_stripes(cuda):
    """RS(6,3), 64 KiB cells, 10,000 stripes: full oracle compare on a seeded
    sample, plus every stripe checked through decode round trips."""
    torch = cuda
    k, p, L, S = 6, 3, 64 << 10, 10000
    code = HipReedSolomonCode(k, p)
    st = rand_stripes(torch, S, k + p, L, seed=2)
    device.encode_stripes(code, st)
    for s in sorted(random.Random(2).sample(range(S), 30)):
        host = st[s].cpu().numpy()
        assert (host[:p] == oracle_parity(k, p, host)).all(), s
    for erased in ([3], [0, 8], [3, 4, 5]):
        to_read = sorted(C.locations_to_read(k, p, erased))
        ntr = [x for x in range(k + p) if x not in to_read]
        out = torch.empty((S, len(erased), L), dtype=torch.uint8, device="cuda")
        device.decode_stripes(code, st, erased, ntr, out)
        assert torch.equal(out, st[:, erased, :]), erased


def test_config3_rs104_1mib_1024_stripes(cuda):
    torch = cuda
    k, p, L, S = 10, 4, 1 << 20, 1024
    code = HipReedSolomonCode(k, p)
    st = rand_stripes(torch, S, k + p, L, seed=3)
    device.encode_stripes(code, st)
    for s in (0, 511, 1023):
        host = st[s].cpu().numpy()
        assert (host[:p] == oracle_parity(k, p, host)).all(), s
    erased = [4]
    to_read = sorted(C.locations_to_read(k, p, erased))
    ntr = [x for x in range(k + p) if x not in to_read]
    out = torch.empty((S, 1, L), dtype=torch.uint8, device="cuda")
    device.decode_stripes(code, st, erased, ntr, out)
    assert torch.equal(out[:, 0], st[:, 4])
    # seeded random single location per stripe (second run of config 3), grouped by location
    locs = torch.tensor([random.Random(s).randrange(k + p) for s in range(S)])
    for loc in range(k + p):
        idx = (locs == loc).nonzero().flatten().cuda()
        if idx.numel() == 0:
            continue
        sub = st.index_select(0, idx)
        to_read = sorted(C.locations_to_read(k, p, [loc]))
        ntr = [x for x in range(k + p) if x not in to_read]
        o = torch.empty((sub.shape[0], 1, L), dtype=torch.uint8, device="cuda")
        device.decode_stripes(code, sub, [loc], ntr, o)
        assert torch.equal(o[:, 0], sub[:, loc]), loc


def test_config5_rs124_256k_two_erasures(cuda):
    torch = cuda
    k, p, L, S = 12, 4, 256 << 10, 512
    code = HipReedSolomonCode(k, p)
    st = rand_stripes(torch, S, k + p, L, seed=5)
    device.encode_stripes(code, st)
    host = st[7].cpu().numpy()
    assert (host[:p] == oracle_parity(k, p, host)).all()
    rnd = random.Random(5)
    for _ in range(6):
        erased = sorted(rnd.sample(range(k + p), 2))
        to_read = sorted(C.locations_to_read(k, p, erased))
        ntr = [x for x in range(k + p) if x not in to_read]
        out = torch.empty((S, 2, L), dtype=torch.uint8, device="cuda")
        device.decode_stripes(code, st, erased, ntr, out)
        assert torch.equal(out, st[:, erased, :]), erased


def test_edge_stripes_all_zero_all_ff_ramp(cuda):
    torch = cuda
    k, p, L = 10, 4, 4096
    code = HipReedSolomonCode(k, p)
    st = torch.zeros((3, k + p, L), dtype=torch.uint8, device="cuda")
    st[1, p:] = 0xFF
    st[2, p:] = (torch.arange(k * L, device="cuda") % 256).to(torch.uint8).view(k, L)
    device.encode_stripes(code, st)
    host = st.cpu().numpy()
    assert (host[0, :p] == 0).all()
    for s in range(3):
        assert (host[s, :p] == oracle_parity(k, p, host[s])).all()


# ------------------------------------------- reference API surface on the GPU

def test_scalar_encode_decode_like_TestErasureCodes(cuda):  # TestErasureCodes.java:33-69
    rnd = random.Random(17)
    for _ in range(6):
        k = rnd.randrange(99) + 1
        p = rnd.randrange(9) + 1
        code = HipReedSolomonCode(k, p)
        for _ in range(4):
            msg = [rnd.randrange(256) for _ in range(k)]
            par = [0] * p
            code.encode(msg, par)
            assert par == C.encode(k, p, msg)
            data = par + msg
            copy = list(data)
            e = 1 if p == 1 else rnd.randrange(p - 1) + 1
            erased = rnd.sample(range(k + p), e)
            vals = [0] * e
            code.decode(data, erased, vals)
            assert vals == [copy[x] for x in erased]
            assert all(data[x] == 0 for x in erased)  # Java zeroes data[erased]


def test_scalar_decode5_leaves_unlisted_erased_values(cuda):  # ReedSolomonCode.java:144-166
    """An erased location missing from locationsNotToRead: the Java copies no
    recovered value for it (:158-165), so erasedValues[i] keeps what the
    caller passed; the listed ones are decoded; data is zeroed at
    locationsNotToRead only. Compared with the oracle on pre-filled values."""
    rnd = random.Random(29)
    for k, p in [(10, 4), (6, 3), (3, 2), (12, 4)]:
        code = HipReedSolomonCode(k, p)
        n = k + p
        for _ in range(12):
            data = [rnd.randrange(256) for _ in range(n)]
            ntr = sorted(rnd.sample(range(n), rnd.randrange(1, p + 1)))
            outside = [x for x in range(n) if x not in ntr]
            erased = sorted(rnd.sample(ntr, rnd.randrange(0, len(ntr) + 1)) + rnd.sample(outside, rnd.randrange(1, 3)))
            prefill = [rnd.randrange(1, 256) for _ in erased]
            to_read = [x for x in range(n) if x not in ntr]
            want_vals, want_data = C.decode5(k, p, data, erased, to_read, ntr, values=prefill, with_data=True)
            got_data, got_vals = list(data), list(prefill)
            code.decode(got_data, erased, got_vals, to_read, ntr)
            assert got_vals == want_vals, (k, p, erased, ntr)
            assert got_data == want_data
            for i, loc in enumerate(erased):
                if loc not in ntr:
                    assert got_vals[i] == prefill[i]


REPEATED5 = [([3], [3, 3]), ([3, 5], [3, 5, 5]), ([3, 3], [3, 5, 5]), ([4], [4, 4, 4, 4]),
             ([99, -1, 4], [4, 2]), ([0, 13], [13, 0, 13]), ([7, 7, 7], [1, 7, 7, 2])]
REPEATED3 = [[3, 3], [1, 5, 1], [2, 2, 2, 2], [13, 0, 13]]


@pytest.mark.parametrize("L", [1, 4099, 256 << 10])
def test_repeated_locations_match_java(cuda, L):
    """VERDICT r5 missing #3: location lists the Java accepts with repeated
    entries (its solve divides by zero: divTable[y][0] = 0,
    GaloisField.java:107-118) and 5-arg erased values outside the stripe
    (only compared, ReedSolomonCode.java:158-165). Host rows (sync and
    checksummed), device rows, the 3-arg decodeBulk and the scalar decodes,
    all bit-exact vs the oracle's per-byte reference loops."""
    import zlib
    torch = cuda
    k, p = 10, 4
    n = k + p
    code = HipReedSolomonCode(k, p)
    rng = np.random.default_rng(L)
    rows = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(n)]
    drows = [torch.from_numpy(r).cuda() for r in rows]
    for erased, ntr in REPEATED5:
        want = C.decode_bulk5(k, p, [r.copy() for r in rows], erased, [], ntr)
        outs = [np.zeros(L, np.uint8) for _ in erased]
        code.decodeBulk([r.copy() for r in rows], outs, erased, [], ntr)
        assert all((o == w).all() for o, w in zip(outs, want)), (erased, ntr, "host")
        outs = [np.zeros(L, np.uint8) for _ in erased]
        crcs = code.decodeBulkCrc([r.copy() for r in rows], outs, erased, [], ntr)
        assert all((o == w).all() for o, w in zip(outs, want)), (erased, ntr, "host crc")
        assert crcs == [zlib.crc32(w.tobytes()) for w in want]
        douts = [torch.zeros(L, dtype=torch.uint8, device="cuda") for _ in erased]
        code.decodeBulk(drows, douts, erased, [], ntr)
        torch.cuda.synchronize()
        assert all((o.cpu().numpy() == w).all() for o, w in zip(douts, want)), (erased, ntr, "device")
        if L == 1:
            data = [int(r[0]) for r in rows]
            vals = [0x55] * len(erased)
            want_vals, want_data = C.decode5(k, p, list(data), erased, [], ntr, values=list(vals), with_data=True)
            code.decode(data, erased, vals, [], ntr)
            assert vals == want_vals and data == want_data, (erased, ntr, "scalar")
    for erased in REPEATED3:
        want = C.decode_bulk3(k, p, [r.copy() for r in rows], erased)
        outs = [np.zeros(L, np.uint8) for _ in erased]
        code.decodeBulk([r.copy() for r in rows], outs, erased)
        assert all((o == w).all() for o, w in zip(outs, want)), (erased, "decode3 host")
        douts = [torch.zeros(L, dtype=torch.uint8, device="cuda") for _ in erased]
        code.decodeBulk(drows, douts, erased)
        torch.cuda.synchronize()
        assert all((o.cpu().numpy() == w).all() for o, w in zip(douts, want)), (erased, "decode3 device")
        if L == 1:
            data = [int(r[0]) for r in rows]
            vals = [0] * len(erased)
            want_vals, want_data = C.decode3(k, p, list(data), erased)
            code.decode(data, erased, vals)
            assert vals == want_vals and data == want_data, (erased, "scalar decode3")


def test_codec_registry_plugs_in_hip_code(cuda):
    conf = {codec_mod.ERASURE_CODING_CODECS_KEY: codec_mod.DEFAULT_CODECS_JSON,
            "hdfs.raid.erasure.code.rs": HipReedSolomonCode.JAVA_CLASS}
    Codec.initializeCodecs(conf)
    code = Codec.getCodec("rs").createErasureCode(conf)
    assert isinstance(code, HipReedSolomonCode)
    assert (code.stripeSize(), code.paritySize()) == (10, 4)
    data = [bytes(range(i, i + 64)) for i in range(10)]
    par = [bytearray(64) for _ in range(4)]
    code.encodeBulk(data, par)
    ref = C.encode_bulk(10, 4, [np.frombuffer(d, np.uint8) for d in data])
    assert [bytes(x) for x in par] == [bytes(r) for r in ref]


def test_errors_are_ioexceptions(cuda):
    code = HipReedSolomonCode(10, 4)
    with pytest.raises(TooManyErasedLocations):
        code.locationsToReadForDecode([0, 1, 2, 3, 4])
    with pytest.raises(HrsError):  # more not-to-read than p: the Java throws (errSignature[p])
        code.decodeBulk([bytes(8)] * 14, [bytearray(8)], [0], [], [0, 1, 2, 3, 4])
    with pytest.raises(ValueError):
        code.encodeBulk([bytes(8)] * 9, [bytearray(8)] * 4)
