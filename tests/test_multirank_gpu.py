"""Multi-rank bench on the HIP path (-m gpu): bench.py under
torch.distributed.run with 2 ranks sharing the box's one GPU (gloo carries the
matrix broadcast, barriers and max-over-ranks; RCCL needs one GPU per rank,
which only the driver's 8-GPU node has). Each rank encodes + decodes its own
contiguous range of GLOBAL stripes (weak scaling, no data exchange), inputs
keyed by global stripe index, so the per-block parity digests
of the 2-rank run must equal those of a 1-rank run over the same stripes —
the cross-N check the round-1 verdict asked for, through the product's
kernels rather than the CPU rehearsal of tests/test_multiproc.py."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def bench_line(nproc, stripes, port, self_launch=False, strong=False):
    common = ["--stripes", str(stripes), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-e2e"]
    common += ["--strong"] if strong else []
    if nproc == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + common
    elif self_launch:  # bench.py starts its own torch.distributed.run child (no launcher here)
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--dist-backend", "gloo"] + common
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
               "--gpus", str(nproc), "--dist-backend", "gloo"] + common
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MASTER_ADDR"] = "127.0.0.1"
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert lines, out.stdout[-2000:]
    return json.loads(lines[-1])


def test_two_ranks_match_one_rank_stripe_for_stripe(cuda):
    one = bench_line(1, 512, 0)
    two = bench_line(2, 256, 29517)
    assert two["n_gpus"] == 2 and two["config"]["stripes_total"] == 512
    assert one["parity_sha256"]["blocks"] == two["parity_sha256"]["blocks"]
    assert set(one["parity_sha256"]["blocks"]) == {"0", "256"}
    assert two["value"] > 0 and two["scaling"] == "weak"


def test_gpus_two_without_launcher_runs_two_ranks(cuda):
    """`bench.py --gpus 2` with no launcher must start two
    ranks itself (a torch.distributed.run child), report n_gpus 2 and print
    the same per-block digests as the 1-rank run over the same stripes."""
    one = bench_line(1, 512, 0)
    two = bench_line(2, 256, 0, self_launch=True)
    assert two["n_gpus"] == 2 and two["config"]["stripes_total"] == 512
    assert one["parity_sha256"]["blocks"] == two["parity_sha256"]["blocks"]
    assert one["parity_sha256"]["decode_blocks"] == two["parity_sha256"]["decode_blocks"]
    assert two["parity_vs_oracle"]["blocks"] == 4 and two["parity_vs_oracle"]["match"]
    assert two["parity_vs_oracle"]["checked_stripes"] == 512


def test_eight_ranks_real_bench_weak_and_strong(cuda):
    """the real bench.py with 8 ranks (gloo; they share
    the box's GPU), as the driver's 8-GPU SCALE run starts it, weak
    (128 stripes per rank) and strong (1,024 in total, 128 per rank: every
    256-stripe oracle block is split over two ranks). Both runs must report 8
    ranks, carry per-rank kernel times, check every stripe against the
    oracle's digests, and print the same blocks."""
    weak = bench_line(8, 128, 0, self_launch=True)
    strong = bench_line(8, 1024, 0, self_launch=True, strong=True)
    for line, scaling in ((weak, "weak"), (strong, "strong")):
        assert line["n_gpus"] == 8 and line["scaling"] == scaling
        assert line["config"]["stripes_total"] == 1024 and line["config"]["stripes_per_gpu"] == 128
        vs = line["parity_vs_oracle"]
        assert vs["match"] and vs["blocks"] == 8 and vs["checked_stripes"] == 1024 and vs["unchecked_stripes"] == 0
        assert [r["rank"] for r in line["per_rank"]] == list(range(8))
        assert sorted(r["g0"] for r in line["per_rank"]) == list(range(0, 1024, 128))
        assert all(r["encode_ms"]["median"] > 0 and r["decode_ms"]["median"] > 0 for r in line["per_rank"])
        assert line["decode_roofline"]["entry_point"] == "hrs_decode_dev"
    assert weak["parity_sha256"]["blocks"] == strong["parity_sha256"]["blocks"]
    assert weak["parity_sha256"]["decode_blocks"] == strong["parity_sha256"]["decode_blocks"]


def test_rccl_collectives_single_rank(cuda):
    """The RCCL path on the box's one GPU: --force-dist creates an nccl
    (= RCCL) process group with one rank bound to its device, so every
    collective bench.py makes at N GPUs really runs through RCCL here — the
    uint8 matrix broadcasts, the int64 MIN / float64 MAX / int32 MIN
    all-reduces, the barriers, and all_gather_object of the digest blocks,
    the config-5 leg included. (Two ranks cannot share one GPU under RCCL;
    the N-rank curve is the driver's.)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-dist", "--dist-backend", "nccl",
           "--stripes", "256", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["config"]["collectives"] == "nccl" and line["n_gpus"] == 1
    assert line["parity_vs_oracle"]["blocks"] == 2 and line["parity_vs_oracle"]["match"]
    e2e = line["e2e_config5"]
    assert e2e["bit_exact"] and e2e["repaired_vs_oracle"]["blocks"] == 2 and e2e["repaired_vs_oracle"]["match"]
