"""Multi-GPU plumbing for stripe-sharded coding (one process per GPU).

Stripes are independent (every byte column is), so ranks share no data: each
rank encodes/decodes its own contiguous stripe range. torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" in CPU tests) carries only
  - the coding matrix, broadcast from rank 0 and checked by every rank
    against the one it built itself (a cheap cross-rank consistency check), and
  - the barriers and the max-over-ranks reduction around timed regions, and
  - after timing, small gathers of per-rank evidence (output digests, kernel
    times) for rank 0's report.
"""
import numpy as np
import torch
import torch.distributed as dist


def active():
    """A process group exists: every collective below goes through it, even
    with one rank (bench.py --force-dist runs the RCCL calls on one GPU)."""
    return dist.is_available() and dist.is_initialized()


def world():
    return dist.get_world_size() if active() else 1


def rank():
    return dist.get_rank() if active() else 0


def stripe_range(total, nranks, r):
    """Contiguous [lo, hi) share of `total` stripes for rank r (strong scaling)."""
    base, extra = divmod(total, nranks)
    lo = r * base + min(r, extra)
    return lo, lo + base + (1 if r < extra else 0)


def broadcast_matrix(m, device="cpu"):
    """Broadcast rank 0's uint8 coding matrix; raise if any rank's own differs."""
    m = np.ascontiguousarray(np.asarray(m, dtype=np.uint8))
    t = torch.from_numpy(m.copy()).to(device)
    if active():
        dist.broadcast(t, src=0)
    got = t.cpu().numpy()
    same = torch.tensor([1 if np.array_equal(got, m) else 0], device=device)
    if active():
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
    if int(same.item()) != 1:
        raise RuntimeError("coding matrices differ across ranks")
    return got


def barrier():
    if active():
        dist.barrier()


def max_over_ranks(x, device="cpu"):
    if not active():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(x, device="cpu"):
    """Smallest int over the ranks (every rank gets it)."""
    if not active():
        return int(x)
    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def gather_objects(obj):
    """[obj of rank 0, obj of rank 1, ...] on every rank (all_gather_object)."""
    if not active():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def all_ok(flag, device="cpu"):
    if not active():
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())
