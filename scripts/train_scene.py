#!/usr/bin/env python3
"""Train on a real scene and report test PSNR -- the reference's train.py
flow (NeRFSystem: mark_invisible_cells, 8192-ray batches, occupancy updates
every 16 steps, Adam + cosine lr, test renders at the end) on the native
trainer.  Usage:
  python scripts/train_scene.py --dataset nsvf --root /data/Synthetic_NeRF/Lego --steps 30000
Prints one JSON line: rays/s of the training loop and the mean test PSNR
(render(test_time=True): device-resident loop, black background -> the
reference evaluates synthetic scenes on white GT, so bg=1 like train.py's
validation for esf == 0)."""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]

import torch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="nsvf")
    ap.add_argument("--root", required=True)
    ap.add_argument("--downsample", type=float, default=1.0)
    ap.add_argument("--scale", type=float, default=0.5)
    ap.add_argument("--steps", type=int, default=30000)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--test-views", type=int, default=0, help="0 = all")
    ap.add_argument("--exact", action="store_true",
                    help="exact mode: every marched sample through the field (chunk_first=0) and the per-sample "
                         "atomic hash backward, instead of the chunked field + binned fine-level backward")
    ap.add_argument("--seed", type=int, default=4)
    ap.add_argument("--sync-every", type=int, default=0, help="(diagnostics) synchronize + report every N steps")
    a = ap.parse_args(argv)
    from datasets import dataset_dict
    from trainer import NGPTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    train = dataset_dict[a.dataset](a.root, split='train', downsample=a.downsample)
    test = dataset_dict[a.dataset](a.root, split='test', downsample=a.downsample)
    gt = train.gt_f32().to(dev)  # float targets, as the reference's loss sees them
    dirs, poses = train.directions.to(dev).contiguous(), train.poses.to(dev).contiguous()
    # erode for COLMAP scenes, as train.py:176-178 passes erode=dataset_name=='colmap'
    mode = dict(chunk_first=0, hash_backward="atomic") if a.exact else {}
    tr = NGPTrainer(scale=a.scale, batch_size=a.batch, device=dev, num_epochs=max(1, a.steps // 1000),
                    erode=a.dataset == "colmap", seed=a.seed, **mode)
    tr.mark_invisible_cells(train.K.to(dev), poses, train.img_wh)  # train.py:169-172
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(a.steps):
        tr.train_step(gt, dirs, poses)
        if a.sync_every and (it + 1) % a.sync_every == 0:
            torch.cuda.synchronize()
            print(f"[train_scene] step {it + 1} ok, samples {int(tr.n_samples.item())}, occupied-cell count "
                  f"{int(tr._occ_count.item())}", file=sys.stderr, flush=True)
    tr.drain()
    torch.cuda.synchronize()
    t_train = time.perf_counter() - t0
    n = len(test.poses) if a.test_views <= 0 else min(a.test_views, len(test.poses))
    tdirs = test.directions.to(dev)
    psnrs = []
    for i in range(n):
        P = test.poses[i].to(dev)
        d = (tdirs @ P[:, :3].t()).contiguous()
        o = P[:, 3].expand_as(d).contiguous()
        out = tr.render(o, d, bg=1.0 if tr.esf == 0 else 0.0)
        mse = torch.mean((out["rgb"].clamp(0, 1) - test.rays[i].to(dev)) ** 2).item()
        psnrs.append(-10 * math.log10(max(mse, 1e-12)))
    import vren
    res = {"dataset": a.dataset, "root": a.root, "steps": a.steps, "mode": "exact" if a.exact else "default",
           "guard_hits": int(vren.lib().ngp_guard_hits()),
           "train_rays_per_s": round(a.steps * a.batch / t_train, 1),
           "test_psnr": round(sum(psnrs) / max(1, len(psnrs)), 3), "test_views": n}
    print(json.dumps(res))
    return res


if __name__ == "__main__":
    main()
