"""CPU tests of the oracle-digest machinery bench.py uses to check its timed
outputs: per-stripe digests combined per block of 256
global stripes (tools/stripe_digests.py) give the same blocks for every
partition of the stripes over ranks, the comparison with the oracle's
digests fails loudly on a mismatch, on a block the oracle cannot check and
on a run with nothing checked; the mix-ceiling arithmetic; and one block of
tests/golden/bench_digests.json recomputed from the C oracle here (config 2,
global stripes 0-255: the generator's output is reproducible)."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import stripe_digests as SD  # noqa: E402


def _rows(n=1100, width=8):
    return np.arange(n * width, dtype=np.uint64).astype(np.uint8).reshape(n, width) ^ \
        (np.arange(n, dtype=np.uint64)[:, None] * 37).astype(np.uint8)


def test_block_is_hash_of_stripe_hashes_in_global_order():
    rows = _rows()
    d = SD.combine(SD.stripe_digests(lambda a, b: rows[a:b], 600, 0))
    assert list(d) == ["0", "256", "512+88"]
    want = hashlib.sha256(b"".join(hashlib.sha256(rows[i].tobytes()).digest() for i in range(256, 512)))
    assert d["256"] == want.hexdigest()


@pytest.mark.parametrize("nranks", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("total", [1024, 1100, 256])
def test_any_partition_gives_the_same_blocks(nranks, total):
    """Strong scaling splits `total` stripes into contiguous ranges that start
    mid-block (8 ranks x 128 stripes: every block spans two ranks); the union
    of the ranks' per-stripe digests combines to the 1-rank blocks."""
    from lambdafs_amd.parallel import stripe_range
    rows = _rows(total)
    one = SD.combine(SD.stripe_digests(lambda a, b: rows[a:b], total, 0))
    union = {}
    for r in range(nranks):
        lo, hi = stripe_range(total, nranks, r)
        union.update(SD.stripe_digests(lambda a, b: rows[lo + a:lo + b], hi - lo, lo))
    assert SD.combine(union) == one


def test_combine_keys_for_runs_that_start_mid_block():
    digs = {g: bytes([g % 251]) * 32 for g in list(range(300, 600)) + list(range(1000, 1030))}
    assert list(SD.combine(digs)) == ["300+212", "512+88", "1000+24", "1024+6"]
    assert SD.key_span("300+212") == (300, 212) and SD.key_span("512") == (512, 256)


def test_compare_rules():
    want = {"parity": {"0": "aa", "256": "bb", "9984+16": "ee"}, "decode": {"0": "cc"}}
    assert SD.compare({"parity": {"0": "aa"}, "decode": {"0": "cc"}}, want, ("parity", "decode"), 10_000) == \
        {"blocks": 2, "match": True, "checked_stripes": 256, "unchecked_stripes": 0, "partial_blocks": 0}
    with pytest.raises(RuntimeError, match="no block"):  # only a partial block: nothing checkable
        SD.compare({"parity": {"0+128": "zz"}, "decode": {}}, want, ("parity", "decode"), 10_000)
    # an ad-hoc run of 384 stripes: block 0 checked, the partial block 256+128 counted, not fatal
    got = SD.compare({"parity": {"0": "aa", "256+128": "zz"}, "decode": {"0": "cc", "256+128": "yy"}}, want,
                     ("parity", "decode"), 10_000)
    assert got == {"blocks": 2, "match": True, "checked_stripes": 256, "unchecked_stripes": 128, "partial_blocks": 2}
    with pytest.raises(RuntimeError, match="!= oracle"):
        SD.compare({"parity": {"256": "xx"}, "decode": {}}, want, ("parity", "decode"), 10_000)
    with pytest.raises(RuntimeError, match="no block"):  # entirely outside the oracle's range
        SD.compare({"parity": {"10240": "xx"}}, want, ("parity",), 10_000)
    # a run past the oracle's range: the covered part is checked, the rest counted
    got = SD.compare({"parity": {"0": "aa", "10240": "xx"}}, want, ("parity",), 10_000)
    assert got["checked_stripes"] == 256 and got["unchecked_stripes"] == 256
    assert SD.compare({"parity": {"9984+16": "ee"}}, want, ("parity",), 10_000)["blocks"] == 1


def test_mix_ceiling():
    probes = {"read_GBps": 6000.0, "write_GBps": 4000.0}
    assert bench.mix_ceiling(probes, 1, 0) == 6000.0
    assert bench.mix_ceiling(probes, 0, 1) == 4000.0
    assert abs(bench.mix_ceiling(probes, 10, 4) - 14 / (10 / 6000 + 4 / 4000)) < 1e-9


def test_golden_file_covers_the_bench_workloads():
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        g = json.load(f)
    assert "stripe" in g["scheme"]  # the per-stripe-digest scheme bench.py assembles
    assert (g["config3"]["k"], g["config3"]["p"], g["config3"]["cell"]) == (10, 4, 1 << 20)
    assert g["config3"]["stripes"] == 8 * 1024
    assert len(g["config3"]["parity"]) == len(g["config3"]["decode"]) == 32  # 8 GPUs x 1,024 stripes
    assert len(g["config2"]["parity"]) == 40 and "9984+16" in g["config2"]["parity"]
    assert len(g["config5"]["repaired"]) == 16  # 8 GPUs x 512 stripes


def test_golden_config2_block0_from_the_oracle():
    """Recompute one golden block (config 2, stripes 0-255, ~3 s) with the C
    oracle: the committed digests are what the generator produces."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_bench_digests as M
    _, _, key, par, _ = M.block_job((2, 6, 3, 64 << 10, 0, 256, "parity"))
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        assert json.load(f)["config2"]["parity"][key] == par


def test_pattern_fields():
    probes = {"pattern": {"encode": {"GBps": 5000.0}, "decode": {"error": "not instantiated"}}}
    assert bench.pattern_fields(probes, "encode", 4500.0) == {"pattern_ceiling": 5000.0, "frac_vs_pattern": 0.9}
    assert bench.pattern_fields(probes, "decode", 4500.0) == {"pattern_ceiling": None, "frac_vs_pattern": None}
    assert bench.pattern_fields(probes, "other", 1.0)["frac_vs_pattern"] is None


GiB = 1 << 30


def test_e2e_memory_guard():
    """The config-5 leg's host-memory guard (bench.e2e_plan): the full 512
    stripes per rank when every rank on the host fits in 3/4 of the available
    memory, 256 (one oracle block, still checkable) when only that fits, and a
    recorded skip below; unknown memory runs the full leg."""
    need512, need256 = bench.e2e_host_bytes(512), bench.e2e_host_bytes(256)
    assert 5 * GiB < need512 < 7 * GiB and need256 < need512
    assert bench.e2e_plan(None, 8) == (512, None)
    assert bench.e2e_plan(256 * GiB, 8) == (512, None)
    S, why = bench.e2e_plan(8 * need512 / 0.75 - 1, 8)
    assert S == 256 and "256 stripes per rank" in why
    S, why = bench.e2e_plan(8 * need256 / 0.75 - 1, 8)
    assert S == 0 and why.startswith("skipped")
    assert bench.e2e_plan(need512 / 0.75, 1) == (512, None)


def test_host_available_bytes_is_sane():
    v = bench.host_available_bytes()
    assert v is None or 0 < v < (1 << 50)


def test_load_traffic_never_raises():
    wl = {"k": 10, "p": 4, "cell": 1 << 20, "stripes": 1024}
    v, why = bench.load_traffic("encode_static_kernel<10, 4>(...)", wl)
    assert v and why is None
    v, why = bench.load_traffic("no_such_kernel<1>", wl)
    assert v is None and "no PMC pass" in why
    v, why = bench.load_traffic("encode_static_kernel<10, 4>", dict(wl, stripes=128))
    assert v is None and "this run is" in why
