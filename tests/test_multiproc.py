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
