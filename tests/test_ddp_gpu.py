"""Data-parallel training step on the device: two
processes on the one GPU (gloo backend, device tensors staged through the
host; the graph replays run in segments with the collectives between them)
train the ZeRO-1 path (reduce-scatter of the gradient buckets, Adam on each
rank's shards, all-gather of the fp16 shadow, sharded occupancy updates with
the MAX-combined key grid).  Against one process training the concatenated
batch (rank r draws rays [r*R, (r+1)*R) of the same global batch):

* both ranks hold identical fp16 shadows and identical bitfields every
  checked step;
* the per-step losses agree (the loss is a mean over rays: rank means
  averaged by the 1/world folded into Adam = the 2R-ray mean);
* the parameters agree up to summation order: gradients are sums of fp32
  atomics whose order differs, and Adam maps a tiny-gradient element's
  noise to a +-lr step, so a small fraction of elements may differ by up to
  2*lr per step while the rest agree to fp32 rounding.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
R, STEPS = 2048, 300


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(batch, steps):
    import synthetic as S
    from trainer import NGPTrainer
    sc = S.AnalyticScene(W=100, H=100, n_images=10)
    dev = torch.device("cuda", 0)
    gt, dirs, poses = sc.gt_images(device=dev), sc.directions.to(dev), sc.poses.to(dev)
    tr = NGPTrainer(scale=0.5, batch_size=batch, device=dev, seed=3)
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    losses, bitfields = [], []
    for it in range(steps):
        losses.append(tr.train_step(gt, dirs, poses).sum())
        if it in (100, 260, steps - 1):
            bitfields.append(tr.density_bitfield.clone())
    tr.drain()
    torch.cuda.synchronize()
    return tr, torch.stack(losses).cpu(), [b.cpu() for b in bitfields]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "ar-nerf_amd")]
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr, losses, bfs = _train(R, STEPS)
        p = tr.full_params().cpu().clone()
        # numpy: pickled by value (a torch CPU tensor would travel as a shared-memory fd the exiting
        # child could no longer serve)
        q.put((rank, {"params": p.numpy(), "p16": tr.params16.cpu().numpy(), "losses": losses.numpy(),
                      "bitfields": [b.numpy() for b in bfs], "prefetched": tr.n_prefetched}))
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_one_process_on_the_concatenated_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    res = {r: {k: (v if k == "prefetched" else [torch.from_numpy(x) for x in v] if k == "bitfields"
                   else torch.from_numpy(v)) for k, v in d.items()} for r, d in res.items()}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    r0, r1 = res[0], res[1]
    assert torch.equal(r0["p16"], r1["p16"])
    for a, b in zip(r0["bitfields"], r1["bitfields"]):
        assert torch.equal(a, b)
    assert torch.equal(r0["params"], r1["params"])
    assert r0["prefetched"] > STEPS // 2  # the segmented graph replays ran
    tr, losses, bfs = _train(2 * R, STEPS)
    one = tr.params.cpu()
    # loss of the concatenated batch = mean of the ranks' losses
    two = (r0["losses"] + r1["losses"]) / 2  # each rank's loss is the mean over its rays
    rel = (two - losses).abs() / losses.abs()
    print(f"relative loss difference: step 0 {float(rel[0]):.2e}, max over the first 20 steps "
          f"{float(rel[:20].max()):.2e}, mean over {STEPS} steps {float(rel.mean()):.2e}")
    assert float(rel[0]) < 1e-5  # same parameters, same rays: only summation order differs
    assert float(rel[:20].max()) < 1e-3
    assert float(rel.mean()) < 2e-2
    d = (r0["params"] - one).abs()
    frac = float((d > 1e-5).float().mean())
    print(f"params: {frac:.2e} of elements differ by > 1e-5, max {float(d.max()):.2e}, "
          f"relative L2 {float((r0['params'] - one).norm() / one.norm()):.2e}")
    assert frac < 5e-2
    assert float((r0["params"] - one).norm() / one.norm()) < 5e-2
    assert float(d.max()) <= 2 * 1e-2 * STEPS
    for a, b in zip(r0["bitfields"], bfs):
        flips = int(np.unpackbits(torch.bitwise_xor(a, b).numpy()).sum())
        print(f"bitfield: {flips} of {a.numel() * 8} cells differ from the one-process run")
        assert flips <= 1e-2 * a.numel() * 8
