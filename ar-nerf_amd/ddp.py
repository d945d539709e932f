"""Data parallelism of the training step over one process per GPU
(torch.distributed; backend "nccl" = RCCL over xGMI on MI355X).

The reference's only parallelism is Lightning DDP over per-rank 8192-ray
batches (train.py:288): gradients all-reduced every step, buffers broadcast
from rank 0 every forward (SURVEY.md §2 "Collective call sites").  Here:
  * ZeRO-1 over the flat parameter vector: the fp32 gradient is
    reduce-scattered (SUM) in 1 + K buckets -- [MLP | coarse hash levels],
    then the binned levels in K level ranges (level_cuts; K =
    the trainer's dp_fine_buckets, 2 by default) -- each rank
    runs FusedAdam on its 1/world shard of every bucket only (fp32 master,
    moments; the 1/world mean is folded into Adam), and the updated fp16
    shadow the kernels read is all-gathered; a bucket's reduce-scatter, Adam
    and all-gather run on the comm stream as soon as its gradient is complete
    (trainer._replay), beside the rest of the backward.
    Exact per element (the same Adam on the same summed gradient), a third
    less traffic than an all-reduce of the fp32 gradient (RS fp32 + AG fp16)
    and 1/world of the Adam work per rank;
  * no per-step buffer broadcast: the occupancy update is made identical on
    every rank by construction -- all ranks draw the same cells and jitter
    (rank-independent seeds), each evaluates a disjoint 1/world share of the
    list, one MAX all-reduce of the 64-bit (list position, sigma) key grid
    combines them with the reference's last-writer-wins rule (every 16
    steps, C*128^3 x 8 B = 16 MB), and rank 0's threshold is broadcast
    (8 bytes) so all ranks pack the same bitfield.
All functions are no-ops for world_size 1.  With the gloo backend (CPU
tests, and the 2-process test on one GPU) device tensors are staged through
host memory.
"""
import torch
import torch.distributed as dist


# (tests) run the collectives through the process group even at world size 1 -- a world-1
# RCCL group then executes the real reduce_scatter_tensor / all_gather_into_tensor calls
# of the data-parallel step (tests/test_ddp_gpu.py), not the world-1 copies
FORCE_COLLECTIVES = False


def comm_active(group=None):
    """True when the collectives below go through the process group."""
    return world_info(group)[1] > 1 or (FORCE_COLLECTIVES and dist.is_available() and dist.is_initialized())


def world_info(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_range(n, rank, world):
    """Contiguous [lo, hi) share of n items for `rank` (covers 0..n exactly once)."""
    return n * rank // world, n * (rank + 1) // world


def shard_cells(indices, coords, rank, world):
    lo, hi = shard_range(indices.shape[0], rank, world)
    return indices[lo:hi], coords[lo:hi]


def level_cuts(lo, n_levels, k):
    """[lo, c_1, ..., n_levels]: levels lo..n_levels-1 in k (at most one per
    level) contiguous ranges whose sizes differ by at most one; [] when
    there is no level to split."""
    n = n_levels - lo
    if n <= 0:
        return []
    k = max(1, min(int(k), n))
    return [lo + (n * r) // k for r in range(k + 1)]


def zero_buckets(n_params, splits, world, align=4):
    """ZeRO-1 bucket bounds over a flat vector padded to n_pad: buckets
    [0, s_1), [s_1, s_2), ..., [s_k, n_pad), all multiples of world*align
    (equal 16-byte aligned shards); each split rounded DOWN, so a bucket holds
    only entries complete at its split (a few of them fall into the next
    bucket).  Empty buckets are dropped.  splits: an int or an ascending list."""
    q = world * align
    n_pad = ((n_params + q - 1) // q) * q
    cuts = [0] + [(s // q) * q for s in ([splits] if isinstance(splits, int) else splits)] + [n_pad]
    return n_pad, [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]


def _gloo(group):
    return dist.get_backend(group) == "gloo"


def reduce_scatter_(full, out, group=None):
    """out (len/world) = this rank's shard of SUM over ranks of full (len)."""
    if not comm_active(group):
        out.copy_(full)
        return out
    if _gloo(group) and full.is_cuda:
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(o, full.cpu(), op=dist.ReduceOp.SUM, group=group)
        out.copy_(o)
    else:
        dist.reduce_scatter_tensor(out, full, op=dist.ReduceOp.SUM, group=group)
    return out


def all_gather_(full, shard, group=None):
    """full (len) = concatenation over ranks of shard (len/world)."""
    if not comm_active(group):
        full.copy_(shard)
        return full
    if _gloo(group) and full.is_cuda:
        f = torch.empty(full.shape, dtype=full.dtype)
        dist.all_gather_into_tensor(f, shard.cpu(), group=group)
        full.copy_(f)
    else:
        dist.all_gather_into_tensor(full, shard, group=group)
    return full


def allreduce_grad_(grad, group=None):
    """Sum the flat gradient over ranks (the mean is applied in Adam)."""
    if comm_active(group):
        if _gloo(group) and grad.is_cuda:
            g = grad.cpu()
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
            grad.copy_(g)
        else:
            dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return grad


def combine_density_tmp_(tmp, group=None):
    """Cell-wise MAX of the per-rank density_grid_tmp keys ((list position + 1)
    << 32 | sigma bits, 0 = unevaluated; ngp_density_scatter_last): the
    largest list position wins across ranks as within one, so the result
    equals a single process evaluating the whole list."""
    if comm_active(group):
        if _gloo(group) and tmp.is_cuda:
            t = tmp.cpu()
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            tmp.copy_(t)
        else:
            dist.all_reduce(tmp, op=dist.ReduceOp.MAX, group=group)
    return tmp


def sync_threshold_(thr, group=None):
    """Broadcast rank 0's occupancy threshold so bitfields are identical."""
    if comm_active(group):
        src = dist.get_global_rank(group, 0) if group is not None else 0
        if _gloo(group) and thr.is_cuda:
            t = thr.cpu()
            dist.broadcast(t, src=src, group=group)
            thr.copy_(t)
        else:
            dist.broadcast(thr, src=src, group=group)
    return thr
