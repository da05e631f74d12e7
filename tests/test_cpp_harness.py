"""The native C++ harness (tests/cpp/codec_harness.cpp) drives libhrs through
include/hrs.hpp as Encoder.encodeStripe / Decoder.fixErasedBlockImpl drive the
Java codec: per-bufSize rounds, zlib CRC32 block checksums, the Decoder's
erased / toRead / notToRead arrays, zero-filled unread inputs; every round is
checked against the oracle and every repaired block against its stored CRC32."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "tests", "cpp", "codec_harness")


def run(*args, timeout=600, env=None):
    if not os.path.exists(HARNESS):
        subprocess.check_call(["make", "-C", ROOT, "tests/cpp/codec_harness"])
    out = subprocess.run([HARNESS, *map(str, args)], capture_output=True, text=True, timeout=timeout,
                         env=None if env is None else dict(os.environ, **env))
    line = out.stdout.strip().splitlines()[-1]
    return out.returncode, json.loads(line)


def test_host_logic_vs_oracle():
    """tests/cpp/host_logic.cpp through host-only handles: every code family's
    matrices and survivor lists vs the oracle, the decode cache past its
    eviction bound, batch plans, argument errors (also the `make asan` run)."""
    exe = os.path.join(ROOT, "tests", "cpp", "host_logic")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", ROOT, "tests/cpp/host_logic"])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and res["ok"], res


@pytest.mark.parametrize("threads", [0, 1, 4, 8])
def test_copy_pool_concurrent_callers(threads):
    """The host copy pool (hrs_host.hpp) under 4 concurrent callers posting
    batches of 1-14 pieces of random sizes (0 B - 1 MiB): every byte lands,
    with 0 (caller-only), 1, 4 and 8 workers draining the batches they join."""
    exe = os.path.join(ROOT, "tests", "cpp", "copy_pool_test")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", ROOT, "tests/cpp/copy_pool_test"])
    env = dict(os.environ, HRS_HOST_THREADS=str(threads))
    out = subprocess.run([exe, "4", "40"], capture_output=True, text=True, timeout=300, env=env)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and res["ok"] and res["bad_jobs"] == 0, res


@pytest.mark.parametrize("k,p", [(10, 4), (12, 4), (6, 3), (3, 2)])
def test_harness_host_only(k, p):
    rc, res = run("--host-only", k, p)
    assert rc == 0 and res["mismatches"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    (10, 4, 4 << 20, 1 << 20, 1, 3),          # the `rs` codec, 1 MiB bufSize, one lost block
    (10, 4, 4 << 20, 1 << 20, 4, 5),          # four lost blocks
    (12, 4, 2 << 20, 256 << 10, 2, 9),        # RS(12,4), 256 KiB cells
    (6, 3, (3 << 20) + 12345, 1 << 20, 3, 11),  # partial last round (tail bytes)
    (3, 2, 1 << 20, 1 << 20, 2, 13),
])
def test_harness_rs_encoder_decoder(cuda, args):
    rc, res = run(*args)
    assert rc == 0 and res["ok"], res


@pytest.mark.gpu
def test_harness_xor(cuda):
    rc, res = run("--xor", 10, 1, 4 << 20, 1 << 20, 1, 17)
    assert rc == 0 and res["ok"], res


@pytest.mark.gpu
@pytest.mark.parametrize("nerased,seed", [(1, 3), (1, 4), (2, 5), (3, 6), (4, 7), (4, 8)])
def test_harness_nrs(cuda, nerased, seed):
    # NativeReedSolomonCode semantics: every round equals the oracle's
    # orc_nrs_decode_bulk, and each repaired block's CRC equals the stored CRC
    # of the block the Java hands back (res["quirk"]: not the erased one)
    rc, res = run("--nrs", 10, 4, 3 << 20, 1 << 20, nerased, seed)
    assert rc == 0 and res["ok"], res


@pytest.mark.gpu
@pytest.mark.parametrize("nerased,seed", [(1, 3), (2, 4), (2, 9), (3, 5), (4, 6)])
def test_harness_src(cuda, nerased, seed):
    # SimpleRegeneratingCode(10, 6, 2): local-group and RS repairs, each round
    # equal to the oracle's transcription, repaired CRCs equal to the stored ones
    rc, res = run("--src=2", 10, 6, 3 << 20, 1 << 20, nerased, seed)
    assert rc == 0 and res["ok"], res


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    (10, 4, 4 << 20, 1 << 20, 2, 21),            # lost at round 2 of 4
    (12, 4, 2 << 20, 256 << 10, 3, 22),          # RS(12,4), 256 KiB cells, round 3 of 8
    (6, 3, (3 << 20) + 4097, 1 << 20, 3, 23),    # the partial last round
    (10, 4, 4 << 20, 1 << 20, 0, 24),            # lost in the very first round
])
def test_harness_decoder_restart_mid_block(cuda, args):
    """Decoder.java:373-387: a read error mid-block adds an erased location,
    the arrays are rebuilt and the round is redone; the repaired block and its
    chained CRC32 must equal the stored ones (the decode-matrix cache is keyed
    on the new pattern)."""
    k, p, block, buf, grow, seed = args
    rc, res = run(f"--grow={grow}", k, p, block, buf, 1, seed)
    assert rc == 0 and res["ok"], res
    assert res["restarts"] == 1 and res["patterns"] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [2, 4])
def test_harness_concurrent_handles(cuda, threads):
    """One codec per thread (Encoder.java:80, Decoder.java:90,
    MapReduceBlockRepairManager.java:426): threads interleave encodeBulk and
    decodeBulk (1-4 lost locations, changing every round) of RS(10,4) 1 MiB
    cells on their own handles (pageable, so staged); every round bit-exact
    vs the oracle's parity and the original cells."""
    rc, res = run(f"--threads={threads}", "--rounds=12", 10, 4, 1 << 20, 1 << 20, 1, 31)
    assert rc == 0 and res["ok"], res


@pytest.mark.gpu
@pytest.mark.parametrize("depth,nerased", [(2, 2), (4, 4)])
def test_harness_async_rounds_vs_sync(cuda, depth, nerased):
    """Encoder.encodeStripe / Decoder.fixErasedBlockImpl of an RS(10,4)
    stripe (16 MiB blocks + a ragged tail, 1 MiB rounds) pipelined `depth`
    rounds deep through encodeBulkSubmit / decodeBulkSubmit / collect and
    synchronously: every parity / repaired cell vs the oracle and the chained
    block CRC32s vs zlib, in both modes."""
    rc, res = run(f"--async={depth}", 10, 4, (16 << 20) + 4097, 1 << 20, nerased, 17)
    assert rc == 0 and res["ok"], res
    assert res["mismatches"] == 0 and res["erased"] == nerased
