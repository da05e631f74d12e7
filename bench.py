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
     (N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402  (SURVEY §8(d) synthetic stripes: splitmix64 per global stripe)
from lambdafs_amd import HipReedSolomonCode, device, parallel  # noqa: E402

GiB = float(1 << 30)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--stripes", type=int, default=1024, help="stripes per GPU (weak scaling)")
    ap.add_argument("--strong", action="store_true",
                    help="--stripes is the job total, split into contiguous ranges over the ranks")
    ap.add_argument("--cell", type=int, default=1 << 20, help="cell bytes (bufSize)")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--cpu-stripes", type=int, default=0,
                    help="stripes in the CPU baseline sample (0: 8 per thread)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the config-5 end-to-end (host memory) leg")
    ap.add_argument("--no-sha", action="store_true", help="skip the per-rank parity SHA-256")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify a sample against the oracle after timing")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend (nccl = RCCL; gloo only to rehearse ranks sharing one GPU)")
    return ap.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend != "nccl":  # rehearsal: several ranks may share a GPU
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
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


def e2e_config5(local, rank, world, S=512, L=256 << 10, reps=3):
    """BASELINE configs[4] end to end through the product's host batch API
    (hrs_decode_batch_host): RS(12,4), 256 KiB cells, S stripes per GPU (4,096
    over 8), a seeded random PAIR of lost locations per stripe (keyed by the
    global stripe index), the stripes in pinned host memory; only each
    stripe's 12 survivors cross PCIe H2D, only the 2 repaired cells come back.
    Also the same path staged from pageable memory, and the host batch encode
    (hrs_encode_batch_host: 12 data cells H2D, 4 parity cells D2H)."""
    import torch
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
    # pageable host memory: the same call stages through pinned slots
    pg = np.array(stn)
    pout = np.zeros((S, 2, L), np.uint8)
    pg_ms = timed(lambda: device.decode_batch_host(code, pg, er, pout))
    pg_ok = bool(np.array_equal(pout, pg[idx, er]))
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
        "encode_ms": stats(enc_ms),
        "encode_GiBps_user": rate(t_enc, user),
        "encode_pcie_GBps": round((k + p) * L * S * world / 1e9 / (t_enc * 1e-3), 2),
        "bit_exact": ok,
        "n_gpus": world,
    }


def parity_sha256(stripes, p, g0, block=256):
    """SHA-256 of this rank's parity rows (rows 0..p-1, L bytes each, stripe
    by stripe) over each block of `block` consecutive GLOBAL stripes starting
    at a multiple of `block`: {first global stripe of the block: digest}.
    Inputs are keyed by global stripe index, so any N-GPU run covering a
    block must print the same digest for it as any other run."""
    import hashlib
    S = stripes.shape[0]
    out = {}
    s = 0
    while s < S:
        g = g0 + s
        n = min(block - g % block, S - s)
        h = hashlib.sha256()
        for s0 in range(s, s + n, 64):
            h.update(stripes[s0:min(s + n, s0 + 64), :p].contiguous().cpu().numpy().tobytes())
        key = f"{g}" if n == block else f"{g}+{n}"
        out[key] = h.hexdigest()
        s += n
    return out


def copy_peak(dev, code, nbytes=4 << 30, reps=5):
    """Measured device-copy (STREAM-copy) rate on this GPU, read + write of a
    4 GiB buffer, median of `reps`, two ways: the runtime's D2D copy (torch
    copy_) and the engine's own streaming copy (a 1 x 1 all-ones apply runs
    xor_kernel: the same NT loads/stores and grid as the coding kernels, no
    math). SURVEY §8d asks for the roofline against both 8 TB/s and a
    measured copy peak; frac_vs_copy uses the faster of the two."""
    rows = nbytes >> 20
    src = torch.empty((rows, 1 << 20), dtype=torch.uint8, device=dev)
    src.fill_(0x5A)
    dst = torch.empty_like(src)
    out = {}
    for name, fn in (("torch_copy", lambda: dst.copy_(src)),
                     ("engine_copy", lambda: device.apply_rows(code, [[1]], [src], [dst]))):
        fn()
        times = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            times.append(a.elapsed_time(b))
        out[name] = round(2 * nbytes / (float(np.median(times)) * 1e-3) / 1e9, 1)
    if not torch.equal(dst[::97], src[::97]):
        raise RuntimeError("copy probe mismatch")
    del src, dst
    torch.cuda.empty_cache()
    out["GBps"] = max(out["torch_copy"], out["engine_copy"])
    out["how"] = "4 GiB D2D, median of 5: torch copy_ and the engine's 1x1 streaming copy; GBps = max"
    return out


def stats(ms):
    return {"mean": round(float(np.mean(ms)), 4), "median": round(float(np.median(ms)), 4),
            "min": round(float(np.min(ms)), 4)}


# The software-pipelined kernels are the default (HRS_PIPE=0: the plain ones);
# names as rocprofv3 reports them, keys of profiles/pmc_traffic.json.
PIPE = os.environ.get("HRS_PIPE", "1") != "0"
DEC_KERNEL = "bitsliced_pipe_kernel<1,12>" if PIPE else "bitsliced_kernel<1,12>"
BATCH_KERNEL = ("batch_bitsliced_kernel<1,12,true>" if os.environ.get("HRS_BATCH_PATV", "1") != "0"
                else "batch_bitsliced_kernel<1,12,false>")


def enc_kernel_name(k, p):
    return f"encode_static_kernel<{k},{p}>"


def load_traffic(kernel):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(kernel)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    k, p, L = args.k, args.p, args.cell
    if args.strong:
        lo, hi = parallel.stripe_range(args.stripes, world, rank)
        S = hi - lo
    else:
        S = args.stripes
    n = k + p
    dev = f"cuda:{local}"
    code = HipReedSolomonCode(k, p, device=local)

    # coding matrices: built on rank 0, broadcast over RCCL, checked everywhere
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
    out_rows = [out[:, 0, :]]
    assert G.shape == (p, k)

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        device.encode_stripes(code, stripes)
        if ev is not None:
            ev[1].record()
        device.apply_rows(code, D_live, in_rows, out_rows)
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
    parallel.barrier()
    elapsed = parallel.max_over_ranks(time.perf_counter() - t0, dev)

    enc_all = [e[0].elapsed_time(e[1]) for e in events]
    dec_all = [e[1].elapsed_time(e[2]) for e in events]
    enc_ms = float(np.mean(enc_all))
    dec_ms = float(np.mean(dec_all))

    # correctness of what was timed: the decode must reproduce data shard 0
    ok = bool(torch.equal(out[:, 0], stripes[:, p]))
    ok &= bool(torch.equal(stripes[min(S - 1, S // 2), p:].cpu(),
                           torch.from_numpy(synth.stripe_numpy(3, g0 + min(S - 1, S // 2), k, L))))
    if args.check:
        from oracle import rs_oracle as C
        for s_chk in sorted({0, S // 2, S - 1}):
            host = stripes[s_chk].cpu().numpy()
            ref = np.stack(C.encode_bulk(k, p, [host[p + c] for c in range(k)]))
            ok &= bool((host[:p] == ref).all())
    if not parallel.all_ok(ok, dev):
        raise RuntimeError("benchmark output failed its round-trip check")

    # SURVEY §8(d) config 3, second run: a seeded random lost location per
    # stripe, all repaired in one launch (hrs_decode_batch_dev); reported
    # beside the headline, outside its timed region
    rnd = np.random.default_rng(0x5EED0003 + rank)
    er_rand = rnd.integers(0, n, (S, 1)).astype(np.int32)
    out_rand = torch.empty((S, 1, L), dtype=torch.uint8, device=dev)
    device.decode_batch(code, stripes, er_rand, out_rand)
    torch.cuda.synchronize()
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
    crc_two = device.crc32_rows(code, cells)
    if not parallel.all_ok(bool(torch.equal(crc_fused, crc_two)), dev):
        raise RuntimeError("fused encode+CRC differs from encode then CRC")
    reps = max(3, min(args.steps, 10))
    fused_ms = med_ms(lambda: device.encode_stripes_crc(code, stripes), reps)
    two_ms = med_ms(lambda: (device.encode_stripes(code, stripes), device.crc32_rows(code, cells)), reps)

    sha = None
    if not args.no_sha:
        mine = parity_sha256(stripes, p, g0)
        allv = [mine]
        if world > 1:
            allv = [None] * world
            dist.all_gather_object(allv, mine)
        sha = {"block_stripes": 256, "blocks": {}}
        for d in allv:
            sha["blocks"].update(d)
    e2e = None
    if not args.no_e2e:
        del cells
        torch.cuda.empty_cache()
        e2e = e2e_config5(local, rank, world)

    total_stripes = args.stripes if args.strong else S * world
    user_bytes = 2 * k * L * total_stripes * args.steps
    enc_bytes = (k + p) * L * S  # algorithmic bytes per encode launch (read k, write p)
    dec_bytes = (k + len(erased)) * L * S
    enc_gbps = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbps = dec_bytes / (dec_ms * 1e-3) / 1e9
    kernel = enc_kernel_name(k, p)
    res = None
    peak = copy_peak(dev, code) if rank == 0 else None
    if rank == 0:
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
                            f"{S} stripes/GPU, device-resident",
                "stripes_per_gpu": S, "stripes_total": total_stripes, "cell_bytes": L, "k": k, "p": p,
                "parallelism": f"stripe-sharded x{world} (RCCL: matrix broadcast + barriers only)",
            },
            "encode_GiBps_per_gpu": round(k * L * S / GiB / (enc_ms * 1e-3), 3),
            "decode_GiBps_per_gpu": round(k * L * S / GiB / (dec_ms * 1e-3), 3),
            "roofline": {
                "kernel": kernel,
                "bound": "hbm",
                "achieved": round(enc_gbps, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(enc_gbps / HBM_PEAK_GBPS, 4),
                "traffic": load_traffic(kernel),
                "avg_launch_ms": round(enc_ms, 4),
                "launch_ms": stats(enc_all),
                "algorithmic_bytes_per_launch": enc_bytes,
                "copy_peak": peak["GBps"],
                "frac_vs_copy": round(enc_gbps / peak["GBps"], 4),
            },
            "decode_roofline": {
                "kernel": DEC_KERNEL, "achieved": round(dec_gbps, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(dec_gbps / HBM_PEAK_GBPS, 4), "avg_launch_ms": round(dec_ms, 4),
                "launch_ms": stats(dec_all), "frac_vs_copy": round(dec_gbps / peak["GBps"], 4),
                "traffic": load_traffic(DEC_KERNEL),
                "algorithmic_bytes_per_launch": dec_bytes,
            },
            "random_location_decode": {
                "what": "config 3 second run: one seeded random lost location per stripe, one batch launch",
                "launch_ms": stats(rand_ms),
                "kernel": BATCH_KERNEL,
                "GBps_algorithmic": round((k + 1) * L * S / (float(np.median(rand_ms)) * 1e-3) / 1e9, 1),
                "algorithmic_bytes_per_launch": (k + 1) * L * S,
                "traffic": load_traffic(BATCH_KERNEL),
                "GiBps_user_per_gpu": round(k * L * S / GiB / (float(np.median(rand_ms)) * 1e-3), 3),
            },
            "encode_crc": {
                "what": "encode + java.util.zip.CRC32 of all k+p cells (Encoder with computeBlockChecksum)",
                "kernel": f"encode_crc_grouped_kernel<{k},{p},G={4 if k >= 12 else 2},factored> + crc_fold_kernel",
                "fused_ms": stats(fused_ms),
                "two_pass_ms": stats(two_ms),
                "fused_GBps_algorithmic": round(enc_bytes / (float(np.median(fused_ms)) * 1e-3) / 1e9, 1),
                "speedup_vs_two_pass": round(float(np.median(two_ms)) / float(np.median(fused_ms)), 3),
            },
            "copy_peak": peak,
            "parity_sha256": sha,
            "e2e_config5": e2e,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(k, p, L, args.cpu_stripes)
            res["cpu_baseline_1thread"] = cpu_baseline(k, p, L, 40, threads=1)
            res["cpu_baseline"]["gpu_vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
