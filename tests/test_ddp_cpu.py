"""Multi-process (world_size 2, gloo, CPU) tests of the data-parallel
pieces used by trainer.NGPTrainer (ar-nerf_amd/ddp.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ddp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cells():
    g = torch.Generator().manual_seed(0)
    idx = torch.randint(0, 4096, (3000,), generator=g)  # many duplicates
    sig = torch.rand(3000, generator=g) * 10
    return idx, sig


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        # 1) gradient all-reduce == sum of the ranks' gradients
        g = torch.arange(10, dtype=torch.float32) * (rank + 1)
        ddp.allreduce_grad_(g)
        out["grad"] = g
        # 2) sharded occupancy evaluation + MAX combine of the (position, sigma)
        # keys == single-process last-writer-wins result (duplicate cells, some
        # duplicated across the shard boundary)
        idx, sig = _cells()
        lo, hi = ddp.shard_range(idx.shape[0], rank, world)
        key = torch.zeros(4096, dtype=torch.int64)
        pos = torch.arange(lo, hi, dtype=torch.int64)
        kv = ((pos + 1) << 32) | sig[lo:hi].view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        key.scatter_reduce_(0, idx[lo:hi], kv, reduce="amax")
        ddp.combine_density_tmp_(key)
        out["tmp"] = torch.where(key != 0, (key & 0xFFFFFFFF).to(torch.int32).view(torch.float32), 0.)
        # 3) threshold broadcast from rank 0
        thr = torch.tensor([1.0 + rank, 2.0])
        ddp.sync_threshold_(thr)
        out["thr"] = thr
        # numpy, not torch tensors: torch's queue shares tensor storage through
        # file descriptors that vanish when this process exits first
        q.put((rank, {k: v.numpy() for k, v in out.items()}))
    finally:
        dist.destroy_process_group()


def test_ddp_pieces_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: {k: torch.from_numpy(v) for k, v in o.items()} for r, o in (q.get(timeout=120) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    base = torch.arange(10, dtype=torch.float32)
    for r in range(2):
        torch.testing.assert_close(res[r]["grad"], base * 3)
        assert res[r]["thr"].tolist() == [1.0, 2.0]
    idx, sig = _cells()
    nt = torch.get_num_threads()
    torch.set_num_threads(1)  # torch's sequential index_put_: the last duplicate wins
    try:
        full = torch.zeros(4096)
        full[idx] = sig
    finally:
        torch.set_num_threads(nt)
    assert torch.equal(res[0]["tmp"], full)
    assert torch.equal(res[0]["tmp"], res[1]["tmp"])


@pytest.mark.parametrize("n,world", [(10, 3), (2_097_152, 8), (7, 8)])
def test_shard_range_covers_exactly_once(n, world):
    seen = []
    for r in range(world):
        lo, hi = ddp.shard_range(n, r, world)
        seen += list(range(lo, hi)) if n < 100 else [lo, hi]
    if n < 100:
        assert sorted(seen) == list(range(n))
    else:
        assert seen[0] == 0 and seen[-1] == n and all(seen[2 * i + 1] == seen[2 * i + 2] for i in range(world - 1))


@pytest.mark.parametrize("world", [1, 2, 8])
@pytest.mark.parametrize("lo,k", [(8, 4), (8, 2), (0, 4), (16, 4)])
def test_zero_buckets_split_where_the_gradient_is_complete(world, lo, k):
    """The trainer's ZeRO-1 buckets ([MLP | coarse levels], then the binned
    levels lo..16 in k ranges, ddp.level_cuts; trainer.NGPTrainer.__init__):
    contiguous, cover the padded vector once, equal 16-byte shards per rank,
    and each split is rounded DOWN -- a bucket never holds an entry of a later
    level range, so its reduce-scatter may start once its own range is
    complete."""
    import hashgrid as HG
    grid = HG.HashGrid(0.5)
    n = HG.MLP_PARAMS + 2 * int(grid.offsets[grid.n_levels])
    cuts = ddp.level_cuts(lo, grid.n_levels, k)
    if lo == grid.n_levels:
        assert cuts == []
        return
    assert cuts[0] == lo and cuts[-1] == grid.n_levels and len(cuts) == min(k, grid.n_levels - lo) + 1
    sizes = [b - a for a, b in zip(cuts[:-1], cuts[1:])]
    assert min(sizes) >= 1 and max(sizes) - min(sizes) <= 1
    splits = [HG.MLP_PARAMS + 2 * int(grid.offsets[lv]) for lv in cuts[:-1]]
    n_pad, b = ddp.zero_buckets(n, splits, world)
    assert n_pad >= n and n_pad % (4 * world) == 0
    assert b[0][0] == 0 and b[-1][1] == n_pad and all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    assert len(b) == len(cuts) and all((hi - lo_) % (4 * world) == 0 for lo_, hi in b)
    for i, sp in enumerate(splits):
        assert b[i][1] <= sp and sp - b[i][1] < 4 * world
    assert ddp.zero_buckets(n, splits[0], world)[1][0][1] == b[0][1]  # (an int split: two buckets)
