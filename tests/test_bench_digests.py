"""CPU tests of the oracle-digest machinery bench.py uses to check its timed
outputs: the block layout of block_sha256, the
comparison rules of compare_blocks, the mix-ceiling arithmetic, and one
block of tests/golden/bench_digests.json recomputed from the C oracle here
(config 2, global stripes 0-255: the generator's output is reproducible)."""
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


def test_block_sha256_aligns_blocks_to_global_stripes():
    rows = np.arange(600 * 8, dtype=np.uint8).reshape(600, 8)  # 600 stripes of 8 bytes
    d = bench.block_sha256(lambda a, b: rows[a:b], 600, 0)
    assert list(d) == ["0", "256", "512+88"]
    assert d["256"] == hashlib.sha256(rows[256:512].tobytes()).hexdigest()
    # a rank starting at global stripe 300: a partial first block, then aligned ones
    d = bench.block_sha256(lambda a, b: rows[a:b], 600, 300)
    assert list(d) == ["300+212", "512", "768+132"]
    assert d["512"] == hashlib.sha256(rows[212:468].tobytes()).hexdigest()


def test_compare_blocks_rules():
    want = {"parity": {"0": "aa", "256": "bb"}, "decode": {"0": "cc"}}
    assert bench.compare_blocks({"parity": {"0": "aa"}, "decode": {"0": "cc"}}, want, ("parity", "decode")) == \
        {"blocks": 2, "match": True}
    assert bench.compare_blocks({"parity": {"0+128": "zz"}, "decode": {}}, want, ("parity", "decode")) is None
    with pytest.raises(RuntimeError):
        bench.compare_blocks({"parity": {"256": "xx"}, "decode": {}}, want, ("parity", "decode"))


def test_mix_ceiling():
    probes = {"read_GBps": 6000.0, "write_GBps": 4000.0}
    assert bench.mix_ceiling(probes, 1, 0) == 6000.0
    assert bench.mix_ceiling(probes, 0, 1) == 4000.0
    assert abs(bench.mix_ceiling(probes, 10, 4) - 14 / (10 / 6000 + 4 / 4000)) < 1e-9


def test_golden_file_covers_the_bench_workloads():
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        g = json.load(f)
    assert (g["config3"]["k"], g["config3"]["p"], g["config3"]["cell"]) == (10, 4, 1 << 20)
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
    import bench
    probes = {"pattern": {"encode": {"GBps": 5000.0}, "decode": {"error": "not instantiated"}}}
    assert bench.pattern_fields(probes, "encode", 4500.0) == {"pattern_ceiling": 5000.0, "frac_vs_pattern": 0.9}
    assert bench.pattern_fields(probes, "decode", 4500.0) == {"pattern_ceiling": None, "frac_vs_pattern": None}
    assert bench.pattern_fields(probes, "other", 1.0)["frac_vs_pattern"] is None
