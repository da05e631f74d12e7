"""Full-size parity against the oracle (-m gpu): every
stripe of the BASELINE workloads, not a sample. The product's outputs on the
SURVEY §8(d) synthetic stripes are hashed stripe by stripe, the digests
combined per block of 256 global stripes (tools/stripe_digests.py), and
compared with the digests the C oracle computed for the same stripes
(tests/golden/bench_digests.json, made by tests/golden/make_bench_digests.py
from oracle/rs_oracle.c — ReedSolomonCode.encodeBulk / decodeBulk 5-arg
restated). A fault confined to any stripe range shows up as a block mismatch.

  config 3: RS(10,4) 1 MiB x 1,024 — parity of every stripe (encode) and the
            row decodeBulk repairs for lost data shard 0 (decode);
  config 2: RS(6,3) 64 KiB x 10,000 — parity of every stripe;
  config 5: RS(12,4) 256 KiB x 512 — the two cells of each stripe's seeded
            random lost pair, repaired in one heterogeneous batch launch.
"""
import json
import os
import sys

import numpy as np
import pytest

from lambdafs_amd import HipReedSolomonCode, device

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
import synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        return json.load(f)


def digests(rows_of, S, g0=0):
    import stripe_digests as SD
    return SD.combine(SD.stripe_digests(rows_of, S, g0))


def check(got, want):
    assert got, "nothing hashed"
    for key, d in got.items():
        assert want[key] == d, f"block {key}"


def test_config3_every_stripe_vs_oracle(cuda, golden):
    torch = cuda
    k, p, L, S = 10, 4, 1 << 20, 1024
    code = HipReedSolomonCode(k, p)
    st = torch.zeros((S, k + p, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, st, 3, 0, k, p)
    device.encode_stripes(code, st)
    to_read = sorted(code.locationsToReadForDecode([p]))
    ntr = [x for x in range(k + p) if x not in to_read]
    out = torch.empty((S, 1, L), dtype=torch.uint8, device="cuda")
    device.decode_stripes(code, st, [p], ntr, out)
    torch.cuda.synchronize()
    check(digests(lambda a, b: st[a:b, :p], S), golden["config3"]["parity"])
    check(digests(lambda a, b: out[a:b], S), golden["config3"]["decode"])


def test_config3_other_ranks_blocks(cuda, golden):
    """Global stripes 7,168 .. 8,191 (rank 7 of an 8-GPU weak-scaling run):
    the inputs are keyed by global index, so rank 7's blocks are checked here
    on one GPU."""
    torch = cuda
    k, p, L, S, g0 = 10, 4, 1 << 20, 512, 7 * 1024 + 512
    code = HipReedSolomonCode(k, p)
    st = torch.zeros((S, k + p, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, st, 3, g0, k, p)
    device.encode_stripes(code, st)
    torch.cuda.synchronize()
    got = digests(lambda a, b: st[a:b, :p], S, g0)
    assert set(got) == {"7680", "7936"}
    check(got, golden["config3"]["parity"])


def test_config2_every_stripe_vs_oracle(cuda, golden):
    torch = cuda
    k, p, L, S = 6, 3, 64 << 10, 10_000
    code = HipReedSolomonCode(k, p)
    st = torch.zeros((S, k + p, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, st, 2, 0, k, p)
    device.encode_stripes(code, st)
    torch.cuda.synchronize()
    got = digests(lambda a, b: st[a:b, :p], S)
    assert len(got) == 40 and "9984+16" in got
    check(got, golden["config2"]["parity"])


def test_config5_seeded_pairs_vs_oracle(cuda, golden):
    torch = cuda
    k, p, L, S = 12, 4, 256 << 10, 512
    n = k + p
    code = HipReedSolomonCode(k, p)
    st = torch.zeros((S, n, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, st, 5, 0, k, p)
    device.encode_stripes(code, st)
    er = np.array([sorted(np.random.default_rng([0x5EED0005, g]).choice(n, 2, replace=False)) for g in range(S)],
                  dtype=np.int32)
    out = torch.empty((S, 2, L), dtype=torch.uint8, device="cuda")
    device.decode_batch(code, st, er, out)
    torch.cuda.synchronize()
    check(digests(lambda a, b: out[a:b], S), golden["config5"]["repaired"])
