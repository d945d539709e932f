"""Data parallelism of the training step over one process per GPU
(torch.distributed; backend "nccl" = RCCL over xGMI on MI355X).

The reference's only parallelism is Lightning DDP over per-rank 8192-ray
batches (train.py:288): gradients all-reduced every step, buffers broadcast
from rank 0 every forward (SURVEY.md §2 "Collective call sites").  Here:
  * one all-reduce (SUM) of the flat fp32 gradient per step; the Adam kernel
    folds in the 1/world mean (grad_scale), so no extra pass;
  * no per-step buffer broadcast: the occupancy update is made identical on
    every rank by construction -- all ranks draw the same cells and jitter
    (rank-independent seeds), each evaluates a disjoint 1/world share of the
    list, one MAX all-reduce of the 64-bit (list position, sigma) key grid
    combines them with the reference's last-writer-wins rule (every 16
    steps, C*128^3 x 8 B = 16 MB), and rank 0's threshold is broadcast
    (8 bytes) so all ranks pack the same bitfield.
All functions are no-ops for world_size 1 and work with gloo on CPU tensors.
"""
import torch
import torch.distributed as dist


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


def allreduce_grad_(grad, group=None):
    """Sum the flat gradient over ranks (the mean is applied in Adam)."""
    if world_info(group)[1] > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM, group=group)
    return grad


def combine_density_tmp_(tmp, group=None):
    """Cell-wise MAX of the per-rank density_grid_tmp keys ((list position + 1)
    << 32 | sigma bits, 0 = unevaluated; ngp_density_scatter_last): the
    largest list position wins across ranks as within one, so the result
    equals a single process evaluating the whole list."""
    if world_info(group)[1] > 1:
        dist.all_reduce(tmp, op=dist.ReduceOp.MAX, group=group)
    return tmp


def sync_threshold_(thr, group=None):
    """Broadcast rank 0's occupancy threshold so bitfields are identical."""
    if world_info(group)[1] > 1:
        dist.broadcast(thr, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return thr
