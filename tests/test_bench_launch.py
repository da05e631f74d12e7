"""CPU tests of bench.py's launch contract: `--gpus N`
without a launcher starts N ranks itself through torch.distributed.run — a
child process started before this process touches the GPU — and a launcher
whose WORLD_SIZE differs from --gpus is refused, so a 1..8-GPU scaling run can
never silently measure one rank. Also the PMC-traffic lookup by the name of
the kernel the run launched."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def plan(args, world=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if world is not None:
        env["WORLD_SIZE"] = str(world)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--print-launch"] + args,
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_n_without_launcher_spawns_n_ranks_before_cuda(n):
    p = plan(["--gpus", str(n), "--steps", "3"])
    assert p["plan"] == "spawn" and p["cuda_initialized"] is False
    cmd = p["command"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert f"--nproc-per-node={n}" in cmd and "127.0.0.1" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--print-launch", "--gpus", str(n), "--steps", "3"]  # argv passed through as given


def test_one_gpu_runs_in_process():
    p = plan([])
    assert p == {"plan": "run", "why": None, "cuda_initialized": False, "command": None}


def test_launcher_rank_runs_when_world_matches():
    assert plan(["--gpus", "4"], world=4)["plan"] == "run"


def test_world_size_mismatch_is_refused():
    p = plan(["--gpus", "8"], world=1)
    assert p["plan"] == "error" and "WORLD_SIZE=1" in p["why"]
    env = dict(os.environ, WORLD_SIZE="2")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], capture_output=True,
                         text=True, env=env, timeout=300)
    assert out.returncode == 2 and "WORLD_SIZE=2" in out.stderr


def test_launch_plan_function():
    import bench
    a = bench.parse(["--gpus", "8"])
    assert bench.launch_plan(a, {}) == ("spawn", None)
    assert bench.launch_plan(a, {"WORLD_SIZE": "8"}) == ("run", None)
    assert bench.launch_plan(a, {"WORLD_SIZE": "1"})[0] == "error"
    assert bench.launch_plan(bench.parse([]), {}) == ("run", None)


def test_traffic_key_matches_rocprof_names():
    import bench
    assert bench.traffic_key("encode_static_kernel<10, 4>") == "encode_static_kernel<10,4>"
    assert bench.traffic_key("batch_bitsliced_kernel<1, 12, true>") == "batch_bitsliced_kernel<1,12,true>"
    # the demangled form rocprofv3 writes, as tools/pmc_traffic.py shortens it
    from tools.pmc_traffic import short
    full = "void hrs::(anonymous namespace)::bitsliced_pipe_kernel<1, 12>(hrs::RowArgs)"
    assert bench.traffic_key("bitsliced_pipe_kernel<1, 12>") == short(full) == "bitsliced_pipe_kernel<1,12>"


def test_traffic_table_has_the_bench_kernels():
    """The kernels the default bench launches have PMC entries for the
    default workload; a missing entry, or another workload, reports null
    traffic with the reason (never raise on rank 0 while the other
    ranks wait in a collective, never a figure of another workload)."""
    import bench
    wl = {"k": 10, "p": 4, "cell": 1 << 20, "stripes": 1024}
    for name in ("encode_static_kernel<10, 4>", "bitsliced_pipe_kernel<1, 12>", "batch_bitsliced_kernel<1, 12, true>",
                 "decode_crc_pipe_kernel<1, 12, true>"):
        t, why = bench.load_traffic(name, wl)
        assert isinstance(t, int) and t > 10 ** 10 and why is None
    t, why = bench.load_traffic("no_such_kernel<1>", wl)
    assert t is None and "no_such_kernel" in why
    t, why = bench.load_traffic("encode_static_kernel<10, 4>", dict(wl, stripes=512))
    assert t is None and "512" in why
