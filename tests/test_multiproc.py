"""world_size-2 gloo test of the stripe-sharded multi-GPU path (CPU only).

Each rank: builds its coding matrices (host-only libhrs handle), receives rank
0's over the collective and checks them, computes its contiguous stripe range
with the oracle standing in for the kernel, and reports a max-over-ranks time.
The union of the ranks' outputs must equal a single-process run.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(r, nranks, port, total, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(nranks))
    import torch.distributed as dist

    from lambdafs_amd import HipReedSolomonCode, parallel
    from oracle import rs_oracle as C
    dist.init_process_group("gloo", rank=r, world_size=nranks)
    try:
        k, p, L = 10, 4, 512
        code = HipReedSolomonCode(k, p, device=-2)
        G = parallel.broadcast_matrix(code.encodeMatrix())
        erased = [4]
        to_read = sorted(code.locationsToReadForDecode(erased))
        ntr = [x for x in range(k + p) if x not in to_read]
        D = parallel.broadcast_matrix(code.decodeMatrix(erased, ntr))
        lo, hi = parallel.stripe_range(total, nranks, r)
        parity = {}
        for s in range(lo, hi):
            rng = np.random.default_rng(1000 + s)  # stripe-keyed inputs: same bytes at any rank count
            data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
            par = C.encode_bulk(k, p, data)
            stripe = par + data
            reads = [stripe[i] if i in to_read else np.zeros(L, np.uint8) for i in range(k + p)]
            rec = C.decode_bulk5(k, p, reads, erased, to_read, ntr)[0]
            assert (rec == data[0]).all()
            parity[s] = np.stack(par)
        parallel.barrier()
        t = parallel.max_over_ranks(0.5 + r)
        ok = parallel.all_ok(True)
        np.savez(os.path.join(outdir, f"rank{r}.npz"), G=G, D=D, t=t, ok=ok,
                 stripes=np.array(sorted(parity)), parity=np.stack([parity[s] for s in sorted(parity)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [7, 8])
def test_two_rank_sharding_matches_single_process(tmp_path, total):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, total, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0 = np.load(tmp_path / "rank0.npz")
    r1 = np.load(tmp_path / "rank1.npz")
    assert float(r0["t"]) == float(r1["t"]) == 1.5  # max over ranks
    assert bool(r0["ok"]) and bool(r1["ok"])
    assert (r0["G"] == r1["G"]).all() and (r0["D"] == r1["D"]).all()
    got = sorted(r0["stripes"].tolist() + r1["stripes"].tolist())
    assert got == list(range(total))  # contiguous, disjoint, complete
    from oracle import rs_oracle as C
    for z in (r0, r1):
        for s, par in zip(z["stripes"], z["parity"]):
            rng = np.random.default_rng(1000 + int(s))
            data = [rng.integers(0, 256, 512, dtype=np.uint8) for _ in range(10)]
            assert (np.stack(C.encode_bulk(10, 4, data)) == par).all()


def test_stripe_range_partition():
    from lambdafs_amd.parallel import stripe_range
    for total in (0, 1, 7, 1024, 1025):
        for n in (1, 2, 3, 8):
            spans = [stripe_range(total, n, r) for r in range(n)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - lo for lo, h in spans) - min(h - lo for lo, h in spans) <= 1


def _bench_flow_worker(r, nranks, port, outdir):
    """bench.py's collective sequence under gloo with host-only handles:
    matrix broadcasts, the barriers and max-over-ranks around the timed
    region, the all-ok checks, the per-block digest gathers (parity, decode,
    config-5 repairs) and their comparison with the oracle's digests, the
    e2e leg's reductions, and the final barrier — in bench.py's order."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(nranks))
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from lambdafs_amd import HipReedSolomonCode, parallel
    dist.init_process_group("gloo", rank=r, world_size=nranks)
    try:
        k, p = 10, 4
        code = HipReedSolomonCode(k, p, device=-2)
        erased = [p]
        to_read = sorted(code.locationsToReadForDecode(erased))
        ntr = [x for x in range(k + p) if x not in to_read]
        G = parallel.broadcast_matrix(code.encodeMatrix())
        D = parallel.broadcast_matrix(code.decodeMatrix(erased, ntr))
        parallel.barrier()
        parallel.barrier()
        elapsed = parallel.max_over_ranks(1.0 + r / 10)
        ok = parallel.all_ok(True) and parallel.all_ok(True)
        golden = bench.load_golden()
        S, g0 = 1024, r * 1024
        # each rank's digests: the oracle's own blocks for its global range
        par = {key: v for key, v in golden["config3"]["parity"].items() if g0 <= int(key) < g0 + S}
        dec = {key: v for key, v in golden["config3"]["decode"].items() if g0 <= int(key) < g0 + S}
        digs = {"parity": bench.gather_blocks(par, nranks), "decode": bench.gather_blocks(dec, nranks)}
        vs = bench.compare_blocks(digs, golden["config3"], ("parity", "decode"))
        # e2e leg (config 5, 512 stripes per rank)
        t = [parallel.max_over_ranks(float(r + i)) for i in range(3)]
        ok_e2e = parallel.all_ok(r != nranks + 1)
        rep = {key: v for key, v in golden["config5"]["repaired"].items() if r * 512 <= int(key) < (r + 1) * 512}
        rep_all = bench.gather_blocks(rep, nranks)
        vs5 = bench.compare_blocks({"repaired": rep_all}, golden["config5"], ("repaired",))
        dist.barrier()
        np.savez(os.path.join(outdir, f"flow{r}.npz"), G=G, D=D, elapsed=elapsed, ok=ok and ok_e2e,
                 nblocks=vs["blocks"], nrep=vs5["blocks"], t=np.array(t), keys=np.array(sorted(digs["parity"])))
    finally:
        dist.destroy_process_group()


def test_bench_collective_flow_world8(tmp_path):
    """bench.py's multi-rank control flow with 8 ranks
    (gloo on CPU): no collective is rank-conditional, the per-block digests of
    8 x 1,024 stripes gather into the full set and match the oracle's, and
    every rank returns."""
    port = _free_port()
    mp.start_processes(_bench_flow_worker, args=(8, port, str(tmp_path)), nprocs=8, join=True, start_method="spawn")
    res = [np.load(tmp_path / f"flow{r}.npz") for r in range(8)]
    for z in res:
        assert float(z["elapsed"]) == 1.7 and bool(z["ok"])
        assert int(z["nblocks"]) == 64 and int(z["nrep"]) == 16  # 32 parity + 32 decode blocks; 16 repaired
        assert z["t"].tolist() == [7.0, 8.0, 9.0]
        assert len(z["keys"]) == 32
        assert (z["G"] == res[0]["G"]).all() and (z["D"] == res[0]["D"]).all()
