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


def _toy_rows(total, width=64):
    """Stand-in outputs for `total` global stripes (stripe g: its own bytes)."""
    g = np.arange(total, dtype=np.uint64)[:, None]
    return ((g * 2654435761 + np.arange(width, dtype=np.uint64)[None, :] * 40503) >> 7).astype(np.uint8)


def _bench_flow_worker(r, nranks, port, outdir, strong):
    """bench.py's collective sequence under gloo with host-only handles and
    bench.py's own helpers: the e2e guard's MIN, matrix broadcasts, the
    barriers and max-over-ranks around the timed region, the per-rank
    evidence gather, the all-ok checks, the per-stripe digest gathers
    (parity, decode, config-5 repairs) combined per block and compared with
    an oracle table, and the final barrier — in bench.py's order. With
    `strong`, 1,024 stripes are split over the ranks (8 x 128: every 256-block
    spans two ranks), as `bench.py --strong --stripes 1024 --gpus 8` does."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(nranks))
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tools"))
    import bench
    import stripe_digests as SD
    from lambdafs_amd import HipReedSolomonCode, parallel
    bench.parallel, bench.SD = parallel, SD
    dist.init_process_group("gloo", rank=r, world_size=nranks)
    try:
        k, p = 10, 4
        code = HipReedSolomonCode(k, p, device=-2)
        e2e_S = parallel.min_over_ranks(bench.e2e_plan(None if r else 64 << 30, 8)[0])
        erased = [p]
        to_read = sorted(code.locationsToReadForDecode(erased))
        ntr = [x for x in range(k + p) if x not in to_read]
        G = parallel.broadcast_matrix(code.encodeMatrix())
        D = parallel.broadcast_matrix(code.decodeMatrix(erased, ntr))
        total = 1024 if strong else 1024 * nranks
        lo, hi = parallel.stripe_range(total, nranks, r) if strong else (r * 1024, (r + 1) * 1024)
        parallel.barrier()
        parallel.barrier()
        elapsed = parallel.max_over_ranks(1.0 + r / 10)
        per_rank = parallel.gather_objects({"rank": r, "g0": lo, "stripes": hi - lo, "wall_s": 1.0 + r / 10})
        ok = parallel.all_ok(True) and parallel.all_ok(True)
        rows = _toy_rows(total)
        table = {"parity": SD.combine(SD.stripe_digests(lambda a, b: rows[a:b], total, 0)),
                 "decode": SD.combine(SD.stripe_digests(lambda a, b: rows[a:b] ^ 0x5A, total, 0))}
        digs = {"parity": bench.oracle_blocks(lambda a, b: rows[lo + a:lo + b], hi - lo, lo),
                "decode": bench.oracle_blocks(lambda a, b: rows[lo + a:lo + b] ^ 0x5A, hi - lo, lo)}
        vs = SD.compare(digs, table, ("parity", "decode"), total)
        # e2e leg (config 5: e2e_S stripes per rank)
        t = [parallel.max_over_ranks(float(r + i)) for i in range(3)]
        ok_e2e = parallel.all_ok(r != nranks + 1)
        rep_rows = _toy_rows(e2e_S * nranks, 32)
        rep = SD.combine(bench.gather_digests(SD.stripe_digests(lambda a, b: rep_rows[r * e2e_S + a:r * e2e_S + b],
                                                                e2e_S, r * e2e_S)))
        vs5 = SD.compare({"repaired": rep}, {"repaired": SD.combine(SD.stripe_digests(
            lambda a, b: rep_rows[a:b], e2e_S * nranks, 0))}, ("repaired",), e2e_S * nranks)
        dist.barrier()
        np.savez(os.path.join(outdir, f"flow{r}.npz"), G=G, D=D, elapsed=elapsed, ok=ok and ok_e2e,
                 nblocks=vs["blocks"], checked=vs["checked_stripes"], nrep=vs5["blocks"], t=np.array(t),
                 keys=np.array(sorted(digs["parity"])), ranks=np.array([d["rank"] for d in per_rank]),
                 e2e_S=e2e_S)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("strong", [False, True])
def test_bench_collective_flow_world8(tmp_path, strong):
    """bench.py's multi-rank control flow with
    8 ranks (gloo on CPU): no collective is rank-conditional, the per-stripe
    digests of every rank combine into the same blocks as one process would
    hash — also when strong scaling leaves each rank half a block — and every
    block is checked; the e2e guard's decision is the same on every rank; and
    every rank returns."""
    port = _free_port()
    mp.start_processes(_bench_flow_worker, args=(8, port, str(tmp_path), strong), nprocs=8, join=True,
                       start_method="spawn")
    res = [np.load(tmp_path / f"flow{r}.npz") for r in range(8)]
    nblk = 4 if strong else 32
    for z in res:
        assert float(z["elapsed"]) == 1.7 and bool(z["ok"])
        assert int(z["nblocks"]) == 2 * nblk and int(z["checked"]) == (1024 if strong else 8192)
        # rank 0 sees 64 GiB for 8 ranks: the guard shrinks the leg to 256
        # stripes per rank (one oracle block each), and every rank agrees
        assert int(z["e2e_S"]) == 256 and int(z["nrep"]) == 8
        assert z["t"].tolist() == [7.0, 8.0, 9.0]
        assert len(z["keys"]) == nblk and all("+" not in k for k in z["keys"].tolist())
        assert z["ranks"].tolist() == list(range(8))
        assert (z["G"] == res[0]["G"]).all() and (z["D"] == res[0]["D"]).all()
