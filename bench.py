"""Benchmark of the MI355X RS engine on BASELINE.json's metric.

Metric: "RS encode+decode GiB/s device-resident; 1/2/4/8 MI355X; %HBM roofline".
Workload (configs[2]): RS(10,4) encode + 1-erasure decode, 1 MiB cells.
One step = one pass of the hot path over one batch resident in HBM:
  encode  : parity of all S stripes           (ReedSolomonCode.encodeBulk)
  decode  : data shard 0 (hops location 4) of all S stripes from the k
            survivors locationsToReadForDecode picks (ReedSolomonCode.decodeBulk)
S = 1024 stripes per GPU (weak scaling: each rank owns its own stripe range;
no data crosses xGMI). RCCL carries only the coding matrices (broadcast from
rank 0) and the barriers around the timed region.

value = user-data bytes (k * L per stripe, counted once for the encode and
once for the decode) of all ranks / max-over-ranks wall time, in GiB/s.

Run: python bench.py [--gpus N --steps K --warmup W]
     --gpus N > 1 without a launcher: bench.py starts
         python -m torch.distributed.run --nproc-per-node N bench.py ...
     as a child process before anything touches the GPU, relays its output and
     exits with its status (the driver's `python -m torch.distributed.run ...
     bench.py --gpus N` form runs the ranks directly). A launcher whose
     WORLD_SIZE differs from --gpus is an error.

The decode is timed through the decodeBulk boundary itself (hrs_decode_dev:
the product's argument checks and decode-matrix cache lookup on every call);
the matrix rank 0 broadcasts over RCCL is a cross-check only.

After timing, every stripe's parity and decoded row get a SHA-256; rank 0
gets every rank's per-stripe digests and hashes them per block of 256 global
stripes (tools/stripe_digests.py), so any partition of the stripes over the
ranks (weak or strong scaling) is compared with the C oracle's digests of the
same synthetic stripes (tests/golden/bench_digests.json). On a workload the
oracle covers, a mismatch, a block the oracle has no digest for, or no
checked block at all fails the run.
"""
import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

# Product imports happen in main(), after the launch decision (launch_plan):
# a relaunching parent must not touch the GPU before it starts its child.
synth = SD = HipReedSolomonCode = device = parallel = None

GiB = float(1 << 30)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # ~0.5 s timed at N=1: long enough for an SMI sampler to see it
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=1024, help="stripes per GPU (weak scaling)")
    ap.add_argument("--strong", action="store_true",
                    help="--stripes is the job total, split into contiguous ranges over the ranks")
    ap.add_argument("--cell", type=int, default=1 << 20, help="cell bytes (bufSize)")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--cpu-stripes", type=int, default=0,
                    help="stripes in the CPU baseline sample (0: 8 per thread)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the config-5 end-to-end (host memory) legs")
    ap.add_argument("--e2e-devices", default="all",
                    help="device set of the one-process config-5 leg (hdfs.raid.hip.devices syntax; world size 1)")
    ap.add_argument("--no-sha", action="store_true", help="skip the per-rank parity SHA-256")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-calls", action="store_true",
                    help="skip the synchronous C-ABI call leg (its small launches of the bench's kernels would mix "
                         "into a rocprofv3 per-kernel average: profiles/run_rocprof.sh passes this)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend (nccl = RCCL; gloo only to rehearse ranks sharing one GPU)")
    ap.add_argument("--force-dist", action="store_true",
                    help="create the process group even with one rank, so the collectives really run "
                         "(one-GPU rehearsal of the RCCL calls)")
    ap.add_argument("--print-launch", action="store_true",
                    help="print the launch decision as JSON and exit (no GPU work; tests)")
    return ap.parse_args(argv)


def launch_plan(args, env):
    """What this process does, decided from --gpus and the launcher's
    environment alone (no GPU call): "run" the rank(s) here, "spawn" a
    torch.distributed.run child with --gpus ranks, or refuse a mismatch."""
    world = env.get("WORLD_SIZE")
    if world is None:
        return ("spawn", None) if args.gpus > 1 else ("run", None)
    if int(world) != args.gpus:
        return "error", f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks"
    return "run", None


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_command(args, argv):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend != "nccl":  # rehearsal: several ranks may share a GPU
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1 or args.force_dist:
        if world == 1:  # single-rank group: a rendezvous of its own
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    return world, rank, local


def host_cpus():
    """CPUs this process may use: its affinity set (what `nproc` prints),
    capped by a cgroup CPU quota when one is set (the GPU boxes give one GPU's
    job a share of a larger machine), plus the CPU model string."""
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return nproc, quota, model


def cpu_baseline(k, p, L, nstripes, threads=None):
    """Restated reference CPU path (oracle/: C transcription of
    ReedSolomonCode.encodeBulk + per-byte decodeBulk 5-arg) on a bounded
    sample of the same workload (the same synthetic stripes, global indices
    3..), stripes spread over host threads."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import rs_oracle as C
    C.lib()
    n = k + p
    nproc, quota, model = host_cpus()
    cores = threads or min(nproc, quota or nproc)
    nstripes = nstripes or 8 * cores
    data = [list(synth.stripe_numpy(3, synth.EDGE_STRIPES + i, k, L)) for i in range(min(nstripes, cores))]
    erased = [p]
    to_read = sorted(C.locations_to_read(k, p, erased))
    ntr = [x for x in range(n) if x not in to_read]

    def one(i):
        src = [x.copy() for x in data[i % len(data)]]  # encodeBulk zeroes its inputs, like the Java
        par = [np.zeros(L, np.uint8) for _ in range(p)]
        C.encode_bulk_ptrs(k, p, C.rowptrs(src), C.rowptrs(par), L)
        stripe = par + data[i % len(data)]
        reads = [stripe[j] if j in to_read else np.zeros(L, np.uint8) for j in range(n)]
        out = [np.zeros(L, np.uint8)]
        C.decode_bulk5_ptrs(k, p, C.rowptrs(reads), C.rowptrs(out), erased, to_read, ntr, L)
        return bool((out[0] == data[i % len(data)][0]).all())

    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        ok = all(ex.map(one, range(nstripes)))
    dt = time.perf_counter() - t0
    if not ok:
        raise RuntimeError("CPU baseline round trip failed")
    return {
        "value": round(2 * k * L * nstripes / GiB / dt, 4),
        "unit": "GiB/s",
        "cores": cores,
        "kind": "port",
        "nproc": nproc,
        "cgroup_cpu_quota": quota,
        "cpu_model": model,
        "sample": f"{nstripes} stripes RS({k},{p}) x {L >> 10} KiB cells, encode + 1-erasure decode, "
                  f"{cores} threads (nproc {nproc}, cgroup quota {quota or 'none'} CPUs), {dt:.1f} s wall",
    }


def placement(local):
    """NUMA node of the CPU the calling thread runs on and of the GPU's PCI
    function (sysfs): a staged call from the GPU's socket is ~10-20 us faster
    than from the other one (profiles/r06/NOTES.md §4). None where unknown."""
    out = {"caller_node": None, "gpu_node": None}
    try:
        import ctypes
        cpu = ctypes.CDLL(None).sched_getcpu()
        for name in os.listdir(f"/sys/devices/system/cpu/cpu{cpu}"):
            if name.startswith("node") and name[4:].isdigit():
                out["caller_node"] = int(name[4:])
    except (OSError, AttributeError, ValueError):
        pass
    try:
        pr = torch.cuda.get_device_properties(local)
        bus = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            out["gpu_node"] = int(f.read().strip())
    except (OSError, AttributeError, ValueError, RuntimeError):
        pass
    return out


def host_calls(local, calls=100):
    """The drop-in's synchronous call rate:
    one RS(10,4) stripe of 1 MiB pageable rows per call through the C ABI the
    JNI shim calls (hrs_encode / hrs_decode / hrs_encode_crc / hrs_decode_crc,
    the Encoder.java:442 / Decoder.java:352 shapes), argument arrays built
    once so the loop times the engine, not Python. Data shard 0 lost for the
    decodes; the repaired row is checked."""
    import ctypes
    from lambdafs_amd import _lib
    from lambdafs_amd._lib import int_array, ptr_array
    k, p, L = 10, 4, 1 << 20
    n = k + p
    code = HipReedSolomonCode(k, p, device=local, zero_inputs_after_encode=False)
    rng = np.random.default_rng(0x5EED000A)
    rows = [np.zeros(L, np.uint8) for _ in range(p)] + [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    h = code._handle()
    lib = _lib.lib()
    ins, outs = ptr_array([r.ctypes.data for r in rows[p:]]), ptr_array([r.ctypes.data for r in rows[:p]])
    lost = np.zeros(L, np.uint8)
    erased = [p]
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(n) if x not in to_read]
    reads = ptr_array([rows[i].ctypes.data if i in to_read else None for i in range(n)])
    lostp = ptr_array([lost.ctypes.data])
    e_a, t_a, n_a = int_array(erased), int_array(to_read), int_array(ntr)
    crc = (ctypes.c_uint32 * n)()
    dcrc = (ctypes.c_uint32 * 1)()

    def per_call(fn):
        for _ in range(5):
            code._check(fn())
        t0 = time.perf_counter()
        for _ in range(calls):
            code._check(fn())
        return (time.perf_counter() - t0) * 1e3 / calls

    res = {"what": "synchronous host-buffer calls through the C ABI (the JNI shim's calls), RS(10,4), one stripe of "
                   "1 MiB pageable rows per call (pinned_rows: the same on caller-pinned rows)", "calls": calls}
    res["encodeBulk_ms"] = per_call(lambda: lib.hrs_encode(h, ins, outs, L))
    res["decodeBulk_ms"] = per_call(lambda: lib.hrs_decode(h, reads, lostp, e_a, 1, t_a, k, n_a, len(ntr), L))
    ok = bool(np.array_equal(lost, rows[p]))
    res["encodeBulkCrc_ms"] = per_call(lambda: lib.hrs_encode_crc(h, ins, outs, L, None, crc))
    res["decodeBulkCrc_ms"] = per_call(lambda: lib.hrs_decode_crc(h, reads, lostp, e_a, 1, t_a, k, n_a, len(ntr), L,
                                                                 None, dcrc))
    ok &= bool(np.array_equal(lost, rows[p]))
    for key in ("encodeBulk", "decodeBulk", "encodeBulkCrc", "decodeBulkCrc"):
        res[key + "_ms"] = round(res[key + "_ms"], 4)
        res[key + "_GiBps_user"] = round(k * L / GiB / (res[key + "_ms"] * 1e-3), 2)
    # the same calls on rows the caller holds in pinned memory (hipHostMalloc,
    # via torch): the kernel runs over them in place, no staging ("pinned")
    pin = torch.empty((n, L), dtype=torch.uint8, pin_memory=True).numpy()
    pin[:] = np.stack(rows)
    pins = ptr_array([pin[i].ctypes.data for i in range(p, n)])
    pouts = ptr_array([pin[i].ctypes.data for i in range(p)])
    res["pinned_rows"] = {"encodeBulk_ms": round(per_call(lambda: lib.hrs_encode(h, pins, pouts, L)), 4),
                          "encodeBulkCrc_ms": round(per_call(lambda: lib.hrs_encode_crc(h, pins, pouts, L, None, crc)),
                                                    4),
                          "path": code.lastHostPath()}
    ok &= all(np.array_equal(pin[r], rows[r]) for r in range(p))
    res["bit_exact"] = ok
    res["placement"] = placement(local)
    if not ok:
        raise RuntimeError("host-buffer decode did not reproduce the lost row")
    return res


def sync_threads(local, codecs=(1, 2, 4), calls=48):
    """The unmodified Encoder at raid.encoder.parallelism = T (Encoder.java:
    77-80: T Encoders, one codec and one thread each, every round a
    synchronous encodeBulk, :442): T host threads each calling hrs_encode on
    their own RS(10,4) stripe of 1 MiB pageable rows, back to back, on one
    GPU. Per T: the aggregate user-data rate, the per-call time and the host
    path the calls took. Every thread's last parity is checked against the
    first thread's first call (same data rows)."""
    import threading
    from lambdafs_amd import _lib
    from lambdafs_amd._lib import ptr_array
    k, p, L = 10, 4, 1 << 20
    lib = _lib.lib()
    rng = np.random.default_rng(0x5EED000C)
    data0 = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    workers = []
    for _ in range(max(codecs)):
        code = HipReedSolomonCode(k, p, device=local, zero_inputs_after_encode=False)
        data = [d.copy() for d in data0]  # each thread its own rows, as each Encoder reads its own
        outs = [np.zeros(L, np.uint8) for _ in range(p)]
        workers.append({"code": code, "h": code._handle(), "data": data, "outs": outs,
                        "ins": ptr_array([d.ctypes.data for d in data]),
                        "outp": ptr_array([o.ctypes.data for o in outs])})
    w0 = workers[0]
    w0["code"]._check(lib.hrs_encode(w0["h"], w0["ins"], w0["outp"], L))
    ref = [o.copy() for o in w0["outs"]]
    res = {"what": "T threads x one RS(10,4) codec each, back-to-back synchronous hrs_encode calls on one 1 MiB "
                   "pageable stripe per call (the unmodified Encoder at raid.encoder.parallelism = T), one GPU",
           "calls_per_thread": calls}

    def run(T):
        errs, per = [], []
        lock = threading.Lock()

        def body(w):
            ms = []
            try:
                for _ in range(calls):
                    t0 = time.perf_counter()
                    w["code"]._check(lib.hrs_encode(w["h"], w["ins"], w["outp"], L))
                    ms.append((time.perf_counter() - t0) * 1e3)
            except Exception as e:  # noqa: BLE001 - reported after the join
                errs.append(e)
            with lock:
                per.extend(ms)

        ths = [threading.Thread(target=body, args=(w,)) for w in workers[:T]]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        wall = time.perf_counter() - t0
        if errs:
            raise errs[0]
        if not all(np.array_equal(a, b) for w in workers[:T] for a, b in zip(w["outs"], ref)):
            raise RuntimeError("concurrent synchronous encodes differ")
        return {"threads": T, "wall_ms": round(wall * 1e3, 2),
                "GiBps_user": round(T * calls * k * L / GiB / wall, 2),
                "call_ms": {"median": round(float(np.median(per)), 4), "p90": round(float(np.percentile(per, 90)), 4)},
                "paths": sorted({w["code"].lastHostPath() for w in workers[:T]})}

    run(max(codecs))  # warm every codec's staging and streams
    res["by_threads"] = [run(T) for T in codecs]
    res["bit_exact"] = True
    return res


def async_rounds(local, codecs=4, depths=(1, 2, 4), rounds=48):
    """The asynchronous drop-in under Encoder-shaped traffic (VERDICT r4 item
    5; HipReedSolomonCode.encodeBulkAsync / collect, Encoder.java:421-453):
    `codecs` host threads, one codec each (raid.encoder.parallelism = 4
    Encoders, Encoder.java:77-80), each keeping `depth` RS(10,4) rounds of one
    1 MiB pageable stripe in flight (submit, and once `depth` are pending
    collect the oldest). Per depth: the aggregate user-data rate, the wall
    time of a round (submit to collected) and its GPU-side launch-to-completion
    time (hrs_set_timing / hrs_ticket_gpu_ms, read after hrs_wait). The first
    round of every codec is checked against the synchronous encode."""
    import ctypes
    import threading
    from lambdafs_amd import _lib
    from lambdafs_amd._lib import ptr_array
    k, p, L = 10, 4, 1 << 20
    lib = _lib.lib()
    rng = np.random.default_rng(0x5EED000B)
    workers = []
    for c in range(codecs):
        code = HipReedSolomonCode(k, p, device=local, zero_inputs_after_encode=False)
        code._check(lib.hrs_set_timing(code._handle(), 1))
        data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        ref = [np.zeros(L, np.uint8) for _ in range(p)]
        code.encodeBulk(data, ref)
        outs = [[np.zeros(L, np.uint8) for _ in range(p)] for _ in range(4)]
        workers.append({"code": code, "h": code._handle(), "data": data,  # data: keeps the rows `ins` points at alive
                        "ins": ptr_array([d.ctypes.data for d in data]),
                        "ref": ref, "outs": outs, "outp": [ptr_array([o.ctypes.data for o in ob]) for ob in outs]})
    res = {"what": f"{codecs} threads x one RS(10,4) codec each, D rounds of one 1 MiB pageable stripe in flight "
                   "per codec (hrs_encode_submit / hrs_wait / hrs_collect), one GPU", "rounds_per_codec": rounds}

    def run_depth(depth):
        errs, lat, gpu = [], [], []
        lock = threading.Lock()

        def body(w):
            h, tq = w["h"], []
            t = ctypes.c_uint64(0)
            ms = ctypes.c_float(0)
            my_lat, my_gpu = [], []
            try:
                for r in range(rounds + depth):
                    if r < rounds:
                        w["code"]._check(lib.hrs_encode_submit(h, w["ins"], L, 0, ctypes.byref(t)))
                        tq.append((t.value, time.perf_counter(), r))
                    if len(tq) == depth or (r >= rounds and tq):
                        tk, t0, rr = tq.pop(0)
                        w["code"]._check(lib.hrs_wait(h, tk))
                        w["code"]._check(lib.hrs_ticket_gpu_ms(h, tk, ctypes.byref(ms)))
                        slot = rr % 4
                        w["code"]._check(lib.hrs_collect(h, tk, w["outp"][slot], None))
                        my_lat.append((time.perf_counter() - t0) * 1e3)
                        my_gpu.append(ms.value)
                        if rr == 0 and not all(np.array_equal(a, b) for a, b in zip(w["outs"][slot], w["ref"])):
                            raise RuntimeError("asynchronous encode differs from the synchronous one")
            except Exception as e:  # noqa: BLE001 - reported after the join
                errs.append(e)
            with lock:
                lat.extend(my_lat)
                gpu.extend(my_gpu)

        ths = [threading.Thread(target=body, args=(w,)) for w in workers]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        wall = time.perf_counter() - t0
        if errs:
            raise errs[0]
        return {"depth": depth, "wall_ms": round(wall * 1e3, 2),
                "GiBps_user": round(codecs * rounds * k * L / GiB / wall, 2),
                "round_wall_ms": {"median": round(float(np.median(lat)), 4), "p90": round(float(np.percentile(lat, 90)), 4)},
                "round_gpu_ms": {"median": round(float(np.median(gpu)), 4), "p90": round(float(np.percentile(gpu, 90)), 4)}}

    run_depth(1)  # warm every codec's slots and staging
    res["by_depth"] = [run_depth(d) for d in depths]
    res["bit_exact"] = True
    return res


def e2e_config5(local, rank, world, golden, S=512, L=256 << 10, reps=3):
    """BASELINE configs[4] end to end through the product's host batch API
    (hrs_decode_batch_host): RS(12,4), 256 KiB cells, S stripes per GPU (4,096
    over 8), a seeded random PAIR of lost locations per stripe (keyed by the
    global stripe index), the stripes in pinned host memory; only each
    stripe's 12 survivors cross PCIe H2D, only the 2 repaired cells come back.
    Also the same call on pageable memory, and the host batch encode
    (hrs_encode_batch_host: 12 data cells H2D, 4 parity cells D2H). The
    repaired cells are hashed per 256-stripe block and compared with the
    oracle's digests (golden["config5"]).
    Host memory per rank at S = 512: ~2.3 GiB pinned (stripes + repaired
    cells) and ~2.8 GiB pageable at peak (the pageable copy, its outputs, the
    check copies), plus the process: e2e_host_bytes(), which run()'s guard
    (e2e_plan) holds against the host's available memory."""
    k, p = 12, 4
    n = k + p
    code = HipReedSolomonCode(k, p, device=local)
    dev = f"cuda:{local}"
    g0 = rank * S
    st_dev = torch.zeros((S, n, L), dtype=torch.uint8, device=dev)
    synth.fill_data_rows(torch, st_dev, 5, g0, k, p)
    st = torch.empty((S, n, L), dtype=torch.uint8, pin_memory=True)
    st.copy_(st_dev)
    st[:, :p] = 0
    device.encode_stripes(code, st_dev)  # device-resident parity, to check the host batch encode
    torch.cuda.synchronize()
    stn = st.numpy()

    def timed(fn):
        fn()
        ms = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ms.append((time.perf_counter() - t0) * 1e3)
        return ms

    enc_ms = timed(lambda: device.encode_batch_host(code, stn))
    enc_ok = bool(torch.equal(st, st_dev.cpu()))
    er = np.full((S, 2), -1, dtype=np.int32)
    for s in range(S):
        er[s] = np.sort(np.random.default_rng([0x5EED0005, g0 + s]).choice(n, 2, replace=False))
    out = torch.empty((S, 2, L), dtype=torch.uint8, pin_memory=True)
    outn = out.numpy()
    dec_ms = timed(lambda: device.decode_batch_host(code, stn, er, outn))
    idx = np.arange(S)[:, None]
    dec_ok = bool(np.array_equal(outn, stn[idx, er]))
    mine = SD.stripe_digests(lambda a, b: outn[a:b], S, g0)
    # pageable host memory: staged through the handle's pinned slots (the
    # GPU never writes into memory the runtime did not allocate pinned)
    pg = np.array(stn)
    pout = np.zeros((S, 2, L), np.uint8)
    pg_ms = timed(lambda: device.decode_batch_host(code, pg, er, pout))
    pg_path = code.lastHostPath()
    pg_ok = bool(np.array_equal(pout, pg[idx, er]))
    del pg, pout
    # the link's own rate for the same survivor bytes: one pinned H2D copy
    nbytes = k * L * S
    src = st.view(-1)[:nbytes]
    dst = st_dev.view(-1)[:nbytes]
    h2d_ms = timed(lambda: (dst.copy_(src, non_blocking=True), torch.cuda.synchronize()))
    del st_dev, dst
    torch.cuda.empty_cache()
    t_dec = parallel.max_over_ranks(float(np.median(dec_ms)), dev)
    t_enc = parallel.max_over_ranks(float(np.median(enc_ms)), dev)
    t_pg = parallel.max_over_ranks(float(np.median(pg_ms)), dev)
    ok = parallel.all_ok(enc_ok and dec_ok and pg_ok, dev)
    repaired = SD.combine(gather_digests(mine))
    user = k * L * S * world

    def rate(t_ms, nbytes):
        return round(nbytes / GiB / (t_ms * 1e-3), 3)

    return {
        "what": "configs[4] end-to-end from host memory through hrs_decode_batch_host: RS(12,4) 256 KiB cells, "
                f"{S} stripes/GPU, seeded random lost pair per stripe; pinned host stripes, survivors H2D, "
                "repaired cells D2H, pipelined chunks",
        "decode_ms": stats(dec_ms),
        "decode_GiBps_user": rate(t_dec, user),
        "decode_pcie_GBps": round((k + 2) * L * S * world / 1e9 / (t_dec * 1e-3), 2),
        "h2d_peak_GBps": round(nbytes / 1e9 / (float(np.median(h2d_ms)) * 1e-3), 2),
        "h2d_peak_how": "one pinned-host to device copy of the same 12 * 256 KiB * S survivor bytes",
        "decode_pageable_ms": stats(pg_ms),
        "decode_pageable_GiBps_user": rate(t_pg, user),
        "decode_pageable_path": pg_path,
        "encode_ms": stats(enc_ms),
        "encode_GiBps_user": rate(t_enc, user),
        "encode_pcie_GBps": round((k + p) * L * S * world / 1e9 / (t_enc * 1e-3), 2),
        "bit_exact": ok,
        "repaired_vs_oracle": SD.compare({"repaired": repaired}, golden.get("config5", {}), ("repaired",),
                                         golden.get("config5", {}).get("stripes", 0)),
        "stripes_per_gpu": S,
        "n_gpus": world,
    }


def e2e_device_set(golden, spec, avail, per=512, L=256 << 10, reps=3):
    """BASELINE configs[4] end to end through the drop-in's device set, in ONE
    process: hrs_decode_batch_host_multi /
    hrs_encode_batch_host_multi over one codec per device of `spec`
    (hdfs.raid.hip.devices syntax, default every visible device): `per`
    stripes per device, global stripes 0 .. per * members - 1 (4,096 on an
    8-GPU node = config 5's total), pinned host memory, contiguous ranges, one
    host thread per device. The repaired cells are checked against the
    oracle's config-5 digests, the re-encoded parity against the device
    encode. Runs at world size 1 only (one process drives every device)."""
    from lambdafs_amd import devset
    k, p = 12, 4
    n = k + p
    devs = devset.parse_device_set(spec, devset.device_count())
    m = len(devs)
    S = per * m
    need = m * (per * (n + 2 + p) * L) + (2 << 30)  # pinned stripes + repaired cells + parity copy + process
    if need > 0.75 * avail:
        return {"skipped": f"device set {devs}: needs {need / GiB:.1f} GiB of host memory, "
                           f"{avail / GiB:.1f} GiB available"}
    st = torch.empty((S, n, L), dtype=torch.uint8, pin_memory=True)
    gen = HipReedSolomonCode(k, p, device=devs[0])
    chunk = torch.zeros((per, n, L), dtype=torch.uint8, device=f"cuda:{devs[0]}")
    for g0 in range(0, S, per):  # synthetic stripes keyed by global index, parity from the device encode
        synth.fill_data_rows(torch, chunk, 5, g0, k, p)
        device.encode_stripes(gen, chunk)
        st[g0:g0 + per].copy_(chunk)
    del chunk
    torch.cuda.synchronize()
    par_ref = st[:, :p].clone()
    stn = st.numpy()
    er = np.array([np.sort(np.random.default_rng([0x5EED0005, g]).choice(n, 2, replace=False)) for g in range(S)],
                  dtype=np.int32)
    out = torch.zeros((S, 2, L), dtype=torch.uint8, pin_memory=True)
    outn = out.numpy()
    codes = [HipReedSolomonCode(k, p, device=d) for d in devs]

    def timed(fn):
        fn()
        ms = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ms.append((time.perf_counter() - t0) * 1e3)
        return ms

    dec_ms = timed(lambda: device.decode_batch_host_multi(codes, stn, er, outn))
    idx = np.arange(S)[:, None]
    dec_ok = bool(np.array_equal(outn, stn[idx, er]))
    repaired = SD.combine(SD.stripe_digests(lambda a, b: outn[a:b], S, 0))
    st[:, :p] = 0
    enc_ms = timed(lambda: device.encode_batch_host_multi(codes, stn))
    enc_ok = bool(torch.equal(st[:, :p], par_ref))
    user = k * L * S
    t_dec, t_enc = float(np.median(dec_ms)), float(np.median(enc_ms))
    res = {
        "what": "configs[4] end to end through hrs_decode_batch_host_multi / hrs_encode_batch_host_multi: one "
                f"process, one codec per device of {devs}, {per} stripes per device (global 0..{S - 1}), RS(12,4) "
                "256 KiB cells, seeded random lost pair per stripe, pinned host memory, contiguous ranges, one host "
                "thread per device",
        "devices": devs, "members": m, "stripes": S,
        "decode_ms": stats(dec_ms), "decode_GiBps_user": round(user / GiB / (t_dec * 1e-3), 3),
        "decode_pcie_GBps_per_device": round((k + 2) * L * per / 1e9 / (t_dec * 1e-3), 2),
        "encode_ms": stats(enc_ms), "encode_GiBps_user": round(user / GiB / (t_enc * 1e-3), 3),
        "bit_exact": dec_ok and enc_ok,
        "repaired_vs_oracle": SD.compare({"repaired": repaired}, golden.get("config5", {}), ("repaired",),
                                         golden.get("config5", {}).get("stripes", 0)),
    }
    del st, out, par_ref
    return res


def gather_digests(mine):
    """Union of every rank's per-stripe digests ({global stripe: digest}),
    on every rank."""
    merged = {}
    for d in parallel.gather_objects(mine):
        merged.update(d)
    return merged


def oracle_blocks(rows_of, S, g0):
    """Block digests of this job's outputs: each rank hashes its own stripes,
    every rank assembles the union (tools/stripe_digests.py)."""
    return SD.combine(gather_digests(SD.stripe_digests(rows_of, S, g0)))


def load_golden():
    path = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def host_available_bytes():
    """Host memory this process can still use: MemAvailable, capped by the
    cgroup v2 limit less its current usage when a limit is set (the GPU boxes
    give each job a share of a larger machine). None if neither is readable."""
    vals = []
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    vals.append(int(line.split()[1]) * 1024)
    except (OSError, ValueError, IndexError):
        pass
    try:
        with open("/sys/fs/cgroup/memory.max") as f:
            lim = f.read().strip()
        if lim != "max":
            with open("/sys/fs/cgroup/memory.current") as f:
                vals.append(int(lim) - int(f.read().strip()))
    except (OSError, ValueError):
        pass
    return min(vals) if vals else None


E2E_BASE_BYTES = 3 << 29  # per rank besides the stripes: torch, HIP runtime, pinned slot staging


def e2e_host_bytes(S, L=256 << 10, n=16, e=2):
    """Peak host bytes of one rank's config-5 leg (e2e_config5): the pinned
    stripes and repaired cells, then the pageable copy, its outputs and the
    two fancy-indexed check copies, alive together."""
    return (2 * n + 3 * e) * L * S + E2E_BASE_BYTES


def e2e_plan(avail, local_ranks, S=512):
    """Stripes per rank for the config-5 leg under the host-memory guard:
    S, or S/2 (down to one 256-stripe oracle block, so the repaired cells stay
    checkable), if every rank on this host fits in 3/4 of what is available;
    else 0 and the reason. `avail` None (unknown) runs the full leg."""
    if avail is None:
        return S, None
    s = S
    while s >= 256:
        if local_ranks * e2e_host_bytes(s) <= 0.75 * avail:
            return s, (None if s == S else f"host memory: {avail / GiB:.1f} GiB available for {local_ranks} "
                                           f"rank(s) on this host; {s} stripes per rank instead of {S}")
        s //= 2
    return 0, (f"skipped: {local_ranks} rank(s) x {e2e_host_bytes(256) / GiB:.1f} GiB for the smallest checkable "
               f"leg exceed 3/4 of the {avail / GiB:.1f} GiB of host memory available")


# hrs_probe_stream shapes swept for the copy / read / write ceilings:
# (schedule, depth, nontemporal, block threads, blocks per CU). The first is
# the fastest copy of tools/copy_lab.hip's 252-variant sweep on this pool
# (block ranges: each 1024-thread block streams its own contiguous 1/256 of the
# buffer, 8 loads per thread in flight; profiles/r04/copy_lab/), then the
# runner-ups of other schedules, and the grid-stride float4 loop of the
# guide's STREAM figure (MI355X_MICROARCH.md: 6.29 TB/s).
PROBE_SHAPES = (
    ("block8_nt_1024x1", 2, 8, True, 1024, 1),
    ("block8_plain_1024x1", 2, 8, False, 1024, 1),
    ("block4_plain_1024x1", 2, 4, False, 1024, 1),
    ("wave4K_plain_256x1", 0, 4, False, 256, 1),
    ("wave1K_nt_256x4", 0, 1, True, 256, 4),
    ("grid4_nt_256x1", 1, 4, True, 256, 1),
    ("grid1_nt_256x4", 1, 1, True, 256, 4),
    ("grid1_plain_1024x1", 1, 1, False, 1024, 1),
)


def hbm_probes(dev, stripes=None, patterns=(), nbytes=4 << 30, reps=5):
    """This GPU's streaming ceilings, measured in this run by the probes of
    libhrs_probe.so (include/hrs_probe.h), median of `reps` launches each;
    every figure is the fastest of the PROBE_SHAPES sweep:
      copy    : 4 GiB read + 4 GiB written (hrs_probe_stream COPY, and
                torch's D2D copy_) — SURVEY §8d's "device-copy STREAM peak";
      read    : read-only stream of 4 GiB;
      write   : write-only stream of 4 GiB;
      pattern : for each (name, nread, nwrite) in `patterns`, the coding
                kernels' access pattern without the math (hrs_probe_rows) over
                `stripes` [S, n, L] itself — same buffer, same bytes, same
                2 KiB-window order — under four load schedules (all loads
                first; or D rows in flight with VALU filler standing in for
                the math, which HBM serves better than a burst:
                tools/pace_probe.hip). This is the ceiling of the pattern: a 1:1
                copy is not one for the codec's read-heavy mixes, and the mix
                of the read-only and write-only peaks ((R + W) / (R / read +
                W / write), mix_ceiling) is optimistic, because HBM pays for
                turning its bus between reads and writes.
    The pattern probe overwrites rows [0, nwrite) of every stripe: call it
    after the stripes' outputs have been checked."""
    src = torch.empty((nbytes >> 20, 1 << 20), dtype=torch.uint8, device=dev)
    src.fill_(0x5A)
    dst = torch.empty_like(src)
    sink = torch.zeros(4096, dtype=torch.uint8, device=dev)

    def timed(fn):
        fn()
        times = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b))
        return float(np.median(times))

    def rate(moved, fn):
        return round(moved / (timed(fn) * 1e-3) / 1e9, 1)

    def kw(shape):
        _, sc, d, nt, blk, bpc = shape
        return dict(schedule=sc, depth=d, nontemporal=nt, block_threads=blk, blocks_per_cu=bpc)

    copies = {}
    for shape in PROBE_SHAPES:
        copies[shape[0]] = rate(2 * nbytes, lambda: device.probe_copy(src, dst, **kw(shape)))
        if not torch.equal(dst[::97], src[::97]):
            raise RuntimeError(f"copy probe {shape[0]} mismatch")
        dst.zero_()
    copies["torch_copy"] = rate(2 * nbytes, lambda: dst.copy_(src))
    reads = {sh[0]: rate(nbytes, lambda: device.probe_read(src, sink, **kw(sh))) for sh in PROBE_SHAPES}
    writes = {sh[0]: rate(nbytes, lambda: device.probe_write(dst, **kw(sh))) for sh in PROBE_SHAPES}
    if int(sink.sum().item()) != 0 or dst[0, 4:8].tolist() != [0x5A] * 4:  # element 0 = (0, 0x5A5A5A5A, ..)
        raise RuntimeError("read / write probes did not run as intended")
    del src, dst, sink
    torch.cuda.empty_cache()
    best = lambda d: max(d, key=d.get)
    out = {
        "copy": {"GBps": copies[best(copies)], "best": best(copies), "variants": copies,
                 "guide_copy_GBps": 6290.0,
                 "how": "4 GiB D2D (bytes read + written), hrs_probe_stream COPY over PROBE_SHAPES and torch "
                        "copy_; GBps = the fastest. guide_copy_GBps: MI355X_MICROARCH.md's float4 copy figure "
                        "(box-to-box spread on this pool: profiles/r04/DESIGN_history.md §5)"},
        "read_GBps": reads[best(reads)], "read_best": best(reads),
        "write_GBps": writes[best(writes)], "write_best": best(writes),
        "read_variants": reads, "write_variants": writes,
        "how": "hrs_probe_stream READ / WRITE over 4 GiB, fastest of PROBE_SHAPES (schedule, depth, policy, "
               "block size, blocks per CU), median of 5 launches each",
        "pattern": {},
    }
    if stripes is not None:
        S, n, L = stripes.shape
        for name, nr, nw in patterns:
            moved = (nr + nw) * L * S
            try:
                v = {f"sched{sc}_{bpc}cu": rate(moved, lambda: device.probe_rows(stripes, nr, nw, bpc, sc))
                     for sc in (0, 1, 2, 3) for bpc in (1, 2)}
            except Exception as e:  # a (nread, nwrite) pair hrs_probe_rows does not instantiate
                out["pattern"][name] = {"error": str(e)}
                continue
            out["pattern"][name] = {"GBps": v[best(v)], "best": best(v), "variants": v, "reads": nr, "writes": nw,
                                    "how": f"hrs_probe_rows over the bench's own {S} x {n} x {L} stripes: "
                                           f"{nr} rows read / {nw} written per 2 KiB window, no GF math; "
                                           "load schedules 0-3 x 1-2 blocks/CU (include/hrs_probe.h)"}
    return out


def mix_ceiling(probes, rbytes, wbytes):
    """Ceiling of a stream of rbytes read and wbytes written on this GPU:
    reads and writes share the HBM data bus, each at its own measured peak."""
    return (rbytes + wbytes) / (rbytes / probes["read_GBps"] + wbytes / probes["write_GBps"])


def pattern_fields(probes, name, gbps):
    """roofline.pattern_ceiling / frac_vs_pattern: the kernel against the
    no-math probe of its own access pattern (hbm_probes "pattern")."""
    pat = probes["pattern"].get(name, {})
    if "GBps" not in pat:
        return {"pattern_ceiling": None, "frac_vs_pattern": None}
    return {"pattern_ceiling": pat["GBps"], "frac_vs_pattern": round(gbps / pat["GBps"], 4)}


def stats(ms):
    return {"mean": round(float(np.mean(ms)), 4), "median": round(float(np.median(ms)), 4),
            "min": round(float(np.min(ms)), 4)}


def traffic_key(name):
    """rocprofv3 kernel name -> the key tools/pmc_traffic.py files it under:
    the name up to its first '>' without namespace or parameters, ", " -> ","."""
    name = re.sub(r"^.*::", "", name.split("(")[0]) if "::" in name.split("<")[0] else name
    m = re.match(r"([A-Za-z_0-9]+(?:<[^>]*>)?)", name)
    return m.group(1).replace(", ", ",") if m else name


def load_traffic(kernel, workload):
    """PMC HBM bytes per launch of `kernel` (the name the run launched) from
    profiles/pmc_traffic.json, measured on the workload its "_workload" entry
    names. Returns (bytes, None), or (None, reason) when the kernel has no
    entry or this run's workload (k, p, cell, stripes per launch) is not the
    profiled one — never a stale or rescaled figure, and never an exception
    on one rank while the others wait in a collective."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            table = json.load(f)
    except (OSError, ValueError) as e:
        return None, f"cannot read {path}: {e}"
    key = traffic_key(kernel)
    prof = table.get("_workload")
    if prof != workload:
        return None, f"PMC passes were taken on {prof}, this run is {workload}"
    if key not in table:
        return None, f"no PMC pass for kernel {key} (profiles/run_rocprof.sh)"
    return table[key], None


def main():
    argv = sys.argv[1:]
    args = parse(argv)
    plan, why = launch_plan(args, os.environ)
    if args.print_launch:
        print(json.dumps({"plan": plan, "why": why, "cuda_initialized": torch.cuda.is_initialized(),
                          "command": spawn_command(args, argv) if plan == "spawn" else None}))
        return 0
    if plan == "error":
        print(f"bench.py: {why}", file=sys.stderr)
        return 2
    if plan == "spawn":
        # one rank per GPU, started before this process makes any GPU call
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        return subprocess.call(spawn_command(args, argv), env=env)
    return run(args)


def run(args):
    global synth, SD, HipReedSolomonCode, device, parallel
    import synth as _synth  # SURVEY §8(d) synthetic stripes: splitmix64 per global stripe
    import stripe_digests as _SD  # per-stripe digests, combined per 256-stripe block
    from lambdafs_amd import HipReedSolomonCode as _Code, device as _device, parallel as _parallel
    synth, SD, HipReedSolomonCode, device, parallel = _synth, _SD, _Code, _device, _parallel

    world, rank, local = setup_dist(args)
    k, p, L = args.k, args.p, args.cell
    if args.strong:
        lo, hi = parallel.stripe_range(args.stripes, world, rank)
        S = hi - lo
    else:
        S = args.stripes
    n = k + p
    dev = f"cuda:{local}"
    code = HipReedSolomonCode(k, p, device=local)
    golden = load_golden()
    # the config-5 leg's host-memory guard, decided before any large allocation
    # and agreed over the ranks (every rank runs the leg with the same S, or none)
    local_ranks = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    e2e_S, e2e_why = (0, "skipped: --no-e2e") if args.no_e2e else e2e_plan(host_available_bytes(), local_ranks)
    e2e_S = parallel.min_over_ranks(e2e_S, dev)

    # coding matrices: built on rank 0, broadcast over RCCL, checked everywhere
    # (the timed decode goes through hrs_decode_dev; the broadcast D is the
    # cross-check of its output below)
    erased = [p]  # data shard 0 = hops location p
    to_read = sorted(code.locationsToReadForDecode(erased))
    ntr = [x for x in range(n) if x not in to_read]
    G = parallel.broadcast_matrix(code.encodeMatrix(), dev)
    D = parallel.broadcast_matrix(code.decodeMatrix(erased, ntr), dev)
    D_live = np.ascontiguousarray(D[:, to_read])

    # synthetic stripes, resident in HBM before timing: [S, n, L] hops order;
    # data rows = splitmix64 keyed by (config 3, GLOBAL stripe index) with the
    # edge stripes (all-0x00, all-0xFF, ramp) at global 0..2
    g0 = (parallel.stripe_range(args.stripes, world, rank)[0] if args.strong else rank * S)
    stripes = torch.zeros((S, n, L), dtype=torch.uint8, device=dev)
    synth.fill_data_rows(torch, stripes, 3, g0, k, p)
    out = torch.empty((S, len(erased), L), dtype=torch.uint8, device=dev)
    in_rows = [stripes[:, loc, :] for loc in to_read]
    assert G.shape == (p, k)

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        device.encode_stripes(code, stripes)  # encodeBulk over S stripes (hrs_encode_dev)
        if ev is not None:
            ev[1].record()
        device.decode_stripes(code, stripes, erased, ntr, out)  # decodeBulk 5-arg (hrs_decode_dev)
        if ev is not None:
            ev[2].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    parallel.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    parallel.barrier()
    elapsed = parallel.max_over_ranks(wall, dev)
    dec_kernel = code.lastKernel()  # the decode step's kernel (decode_stripes ran last)
    device.encode_stripes(code, stripes)  # idempotent: same parity; names the encode kernel
    enc_kernel = code.lastKernel()
    torch.cuda.synchronize()

    enc_all = [e[0].elapsed_time(e[1]) for e in events]
    dec_all = [e[1].elapsed_time(e[2]) for e in events]
    enc_ms = float(np.mean(enc_all))
    dec_ms = float(np.mean(dec_all))
    # per-rank evidence for the scaling line: which rank or phase lagged
    per_rank = parallel.gather_objects({
        "rank": rank, "local_rank": local, "host": socket.gethostname(), "g0": g0, "stripes": S,
        "wall_s": round(wall, 6), "encode_ms": stats(enc_all), "decode_ms": stats(dec_all),
        "encode_kernel": traffic_key(enc_kernel), "decode_kernel": traffic_key(dec_kernel)})

    # correctness of what was timed: the decode must reproduce data shard 0,
    # and equal the broadcast matrix applied to the same survivors
    ok = bool(torch.equal(out[:, 0], stripes[:, p]))
    ok &= bool(torch.equal(stripes[min(S - 1, S // 2), p:].cpu(),
                           torch.from_numpy(synth.stripe_numpy(3, g0 + min(S - 1, S // 2), k, L))))
    xcheck = torch.empty_like(out)
    device.apply_rows(code, D_live, in_rows, [xcheck[:, 0, :]])
    ok &= bool(torch.equal(xcheck, out))
    del xcheck
    if not parallel.all_ok(ok, dev):
        raise RuntimeError("benchmark output failed its round-trip check")

    # SURVEY §8(d) config 3, second run: a seeded random lost location per
    # stripe (keyed by the global stripe index), all repaired in one launch
    # (hrs_decode_batch_dev); reported beside the headline, outside its timed region
    er_rand = np.array([[np.random.default_rng([0x5EED0003, g0 + s]).integers(0, n)] for s in range(S)],
                       dtype=np.int32)
    out_rand = torch.empty((S, 1, L), dtype=torch.uint8, device=dev)
    device.decode_batch(code, stripes, er_rand, out_rand)
    torch.cuda.synchronize()
    batch_kernel = code.lastKernel()
    rand_ms = []
    for _ in range(max(3, min(args.steps, 10))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        device.decode_batch(code, stripes, er_rand, out_rand)
        b.record()
        b.synchronize()
        rand_ms.append(a.elapsed_time(b))
    idx = torch.as_tensor(er_rand[:, 0], dtype=torch.long, device=dev)
    ok_rand = bool(torch.equal(out_rand[:, 0], stripes[torch.arange(S, device=dev), idx]))
    if not parallel.all_ok(ok_rand, dev):
        raise RuntimeError("random-location batch decode failed its round-trip check")
    del out_rand

    # the Encoder's block checksums (Encoder.java:408-450) fused
    # into the encode (hrs_encode_crc_dev) vs the two passes it replaces
    # (encode, then hrs_crc32_dev over the 14 cells); outside the timed region
    def med_ms(fn, reps):
        fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ms.append(a.elapsed_time(b))
        return ms

    cells = [stripes[:, p + c, :] for c in range(k)] + [stripes[:, r, :] for r in range(p)]
    crc_fused = device.encode_stripes_crc(code, stripes)
    fused_kernel = code.lastKernel()
    crc_two = device.crc32_rows(code, cells)
    if not parallel.all_ok(bool(torch.equal(crc_fused, crc_two)), dev):
        raise RuntimeError("fused encode+CRC differs from encode then CRC")
    reps = max(3, min(args.steps, 10))
    fused_ms = med_ms(lambda: device.encode_stripes_crc(code, stripes), reps)
    two_ms = med_ms(lambda: (device.encode_stripes(code, stripes), device.crc32_rows(code, cells)), reps)

    # ... and the Decoder's check of a repaired block (Decoder.java:222-229,
    # :645-655): repair + CRC-32 of the repaired cells fused
    # (hrs_decode_crc_dev) vs the repair then hrs_crc32_dev over its outputs
    out_crc = torch.empty_like(out)
    dcrc_fused = device.decode_stripes_crc(code, stripes, erased, ntr, out_crc)
    dfused_kernel = code.lastKernel()
    dcrc_two = device.crc32_rows(code, [out[:, 0, :]])
    if not parallel.all_ok(bool(torch.equal(out_crc, out)) and bool(torch.equal(dcrc_fused, dcrc_two)), dev):
        raise RuntimeError("fused decode+CRC differs from decode then CRC")
    dfused_ms = med_ms(lambda: device.decode_stripes_crc(code, stripes, erased, ntr, out_crc), reps)
    dtwo_ms = med_ms(lambda: (device.decode_stripes(code, stripes, erased, ntr, out),
                              device.crc32_rows(code, [out[:, 0, :]])), reps)
    del out_crc

    # the timed outputs against the oracle: every stripe's parity and decoded
    # row hashed on its rank, the union hashed per block of 256 global stripes
    # and compared with tests/golden/bench_digests.json (SD.compare raises on
    # a mismatch, on a block the oracle cannot check, and on no block checked
    # — on every rank alike, since every rank holds the union)
    sha = None
    want = golden.get("config3", {})
    golden_workload = (k, p, L) == (want.get("k"), want.get("p"), want.get("cell"))
    if args.no_sha:
        vs_oracle = {"skipped": "--no-sha"}
    else:
        digs = {"parity": oracle_blocks(lambda a, b: stripes[a:b, :p], S, g0),
                "decode": oracle_blocks(lambda a, b: out[a:b], S, g0)}
        sha = {"block_stripes": SD.BLOCK, "scheme": "sha256 of the per-stripe sha256 digests in global order",
               "blocks": digs["parity"], "decode_blocks": digs["decode"]}
        if golden_workload:
            vs_oracle = SD.compare(digs, want, ("parity", "decode"), want.get("stripes", 8 * 1024))
        else:
            vs_oracle = {"skipped": f"no oracle digests for RS({k},{p}) x {L} B cells"}
    e2e = {"skipped": e2e_why} if e2e_S == 0 else None
    if e2e_S:
        del cells
        torch.cuda.empty_cache()
        e2e = e2e_config5(local, rank, world, golden, S=e2e_S)
        if e2e_why:
            e2e["memory_guard"] = e2e_why
        if not e2e["bit_exact"]:
            raise RuntimeError("config 5 end-to-end leg: outputs differ from the device-resident ones")
    e2e_set = None
    if world == 1 and not args.no_e2e:  # one process over the device set (hrs_*_batch_host_multi)
        torch.cuda.empty_cache()
        e2e_set = e2e_device_set(golden, args.e2e_devices, host_available_bytes())
        if e2e_set.get("bit_exact") is False:
            raise RuntimeError("config 5 device-set leg: outputs differ from the device-resident ones")

    total_stripes = args.stripes if args.strong else S * world
    user_bytes = 2 * k * L * total_stripes * args.steps
    enc_bytes = (k + p) * L * S  # algorithmic bytes per encode launch (read k, write p)
    dec_bytes = (k + len(erased)) * L * S
    enc_gbps = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbps = dec_bytes / (dec_ms * 1e-3) / 1e9
    res = None
    # after the digests: the pattern probe overwrites parity rows of `stripes`
    probes = (hbm_probes(dev, stripes, (("encode", k, p), ("decode", k, len(erased)))) if rank == 0 else None)
    if rank == 0:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            traffic_note = json.load(f).get("_note")
        wl = {"k": k, "p": p, "cell": L, "stripes": S}
        enc_traffic, enc_traffic_why = load_traffic(enc_kernel, wl)
        dec_traffic, dec_traffic_why = load_traffic(dec_kernel, wl)
        rand_traffic, rand_traffic_why = load_traffic(batch_kernel, wl)
        dcrc_traffic, dcrc_traffic_why = load_traffic(dfused_kernel, wl)
        res = {
            "metric": "RS encode+decode GiB/s device-resident; 1/2/4/8 MI355X; %HBM roofline",
            "value": round(user_bytes / GiB / elapsed, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: splitmix64 per global stripe (base seed 0x5EED0003), edge stripes "
                    "0x00/0xFF/ramp at global 0..2 (SURVEY §8d)",
            "config": {
                "workload": f"RS({k},{p}) encode + 1-erasure decode (data shard 0), {L >> 10} KiB cells, "
                            f"{S} stripes/GPU, device-resident; encodeBulk / decodeBulk via hrs_encode_dev / "
                            "hrs_decode_dev",
                "stripes_per_gpu": S, "stripes_total": total_stripes, "cell_bytes": L, "k": k, "p": p,
                "parallelism": f"stripe-sharded x{world} (RCCL: matrix broadcast + barriers only)",
                "collectives": (dist.get_backend() if dist.is_available() and dist.is_initialized() else None),
            },
            "parity_vs_oracle": vs_oracle,
            "encode_GiBps_per_gpu": round(k * L * S / GiB / (enc_ms * 1e-3), 3),
            "decode_GiBps_per_gpu": round(k * L * S / GiB / (dec_ms * 1e-3), 3),
            "per_rank": per_rank,
            "roofline": {
                "kernel": traffic_key(enc_kernel),
                "bound": "hbm",
                "achieved": round(enc_gbps, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(enc_gbps / HBM_PEAK_GBPS, 4),
                "traffic": enc_traffic,
                "traffic_source": traffic_note if enc_traffic is not None else enc_traffic_why,
                "avg_launch_ms": round(enc_ms, 4),
                "launch_ms": stats(enc_all),
                "algorithmic_bytes_per_launch": enc_bytes,
                "copy_peak": probes["copy"]["GBps"],
                "frac_vs_copy": round(enc_gbps / probes["copy"]["GBps"], 4),
                "mix_ceiling": round(mix_ceiling(probes, k, p), 1),
                "frac_vs_mix_ceiling": round(enc_gbps / mix_ceiling(probes, k, p), 4),
                **pattern_fields(probes, "encode", enc_gbps),
            },
            "decode_roofline": {
                "kernel": traffic_key(dec_kernel), "entry_point": "hrs_decode_dev",
                "achieved": round(dec_gbps, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(dec_gbps / HBM_PEAK_GBPS, 4), "avg_launch_ms": round(dec_ms, 4),
                "launch_ms": stats(dec_all), "frac_vs_copy": round(dec_gbps / probes["copy"]["GBps"], 4),
                "mix_ceiling": round(mix_ceiling(probes, k, len(erased)), 1),
                "frac_vs_mix_ceiling": round(dec_gbps / mix_ceiling(probes, k, len(erased)), 4),
                **pattern_fields(probes, "decode", dec_gbps),
                "traffic": dec_traffic,
                "traffic_source": traffic_note if dec_traffic is not None else dec_traffic_why,
                "algorithmic_bytes_per_launch": dec_bytes,
            },
            "random_location_decode": {
                "what": "config 3 second run: one seeded random lost location per stripe "
                        "(default_rng([0x5EED0003, global stripe])), one batch launch",
                "launch_ms": stats(rand_ms),
                "kernel": traffic_key(batch_kernel),
                "GBps_algorithmic": round((k + 1) * L * S / (float(np.median(rand_ms)) * 1e-3) / 1e9, 1),
                "algorithmic_bytes_per_launch": (k + 1) * L * S,
                "traffic": rand_traffic,
                "traffic_source": None if rand_traffic is not None else rand_traffic_why,
                "GiBps_user_per_gpu": round(k * L * S / GiB / (float(np.median(rand_ms)) * 1e-3), 3),
            },
            "encode_crc": {
                "what": "encode + java.util.zip.CRC32 of all k+p cells (Encoder with computeBlockChecksum)",
                "kernel": traffic_key(fused_kernel) + " + crc_fold_kernel",
                "fused_ms": stats(fused_ms),
                "two_pass_ms": stats(two_ms),
                "fused_GBps_algorithmic": round(enc_bytes / (float(np.median(fused_ms)) * 1e-3) / 1e9, 1),
                "fused_frac": round(enc_bytes / (float(np.median(fused_ms)) * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "speedup_vs_two_pass": round(float(np.median(two_ms)) / float(np.median(fused_ms)), 3),
            },
            "decode_crc": {
                "what": "repair of data shard 0 + java.util.zip.CRC32 of the repaired cell (Decoder's block check)",
                "kernel": traffic_key(dfused_kernel) + " + crc_fold_kernel",
                "fused_ms": stats(dfused_ms),
                "two_pass_ms": stats(dtwo_ms),
                "traffic": dcrc_traffic,
                "traffic_source": None if dcrc_traffic is not None else dcrc_traffic_why,
                "algorithmic_bytes_per_launch": dec_bytes,
                "fused_GBps_algorithmic": round(dec_bytes / (float(np.median(dfused_ms)) * 1e-3) / 1e9, 1),
                "fused_frac": round(dec_bytes / (float(np.median(dfused_ms)) * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "speedup_vs_two_pass": round(float(np.median(dtwo_ms)) / float(np.median(dfused_ms)), 3),
            },
            "hbm_probes": probes,
            "parity_sha256": sha,
            "e2e_config5": e2e,
            "e2e_device_set": e2e_set,
            "cpu_baseline": None,
        }
        res["host_calls"] = None if args.no_host_calls else host_calls(local)
        res["async_rounds"] = None if args.no_host_calls else async_rounds(local)
        res["sync_threads"] = None if args.no_host_calls else sync_threads(local)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(k, p, L, args.cpu_stripes)
            res["cpu_baseline_1thread"] = cpu_baseline(k, p, L, 40, threads=1)
            res["cpu_baseline"]["gpu_vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
        print(json.dumps(res), flush=True)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
