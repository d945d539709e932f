#!/usr/bin/env python3
"""Occupancy-update check (diagnostic): after every density-grid EMA of a
training run, compare the device sum/count/threshold with torch's."""
import json
import os
import sys

ROOT = os.environ.get("NGP_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

dev = torch.device("cuda")
sc = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
gt = sc.gt_images(device=dev)
dirs, poses = sc.directions.to(dev).contiguous(), sc.poses.to(dev).contiguous()
tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev, hash_backward="atomic")
tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
orig = tr.update_density_grid
log = []


def wrapped(*a, **k):
    orig(*a, **k)
    g = tr.density_grid
    pos = g[g > 0]
    log.append({"step": tr.global_step, "kernel_sum": float(tr._sum_cnt[0]), "kernel_cnt": float(tr._sum_cnt[1]),
                "torch_sum": float(pos.double().sum()), "torch_cnt": int(pos.numel()),
                "thr": float(tr.threshold[0]), "torch_mean": float(pos.double().mean()) if pos.numel() else None})


tr.update_density_grid = wrapped
g = torch.Generator(device=dev).manual_seed(1)
for _ in range(int(os.environ.get("STEPS", "600"))):
    img = torch.randint(0, 100, (8192,), device=dev, generator=g)
    pix = torch.randint(0, 800 * 800, (8192,), device=dev, generator=g)
    tr.step(img, pix, gt[img, pix].float() / 255, dirs, poses)
torch.cuda.synchronize()
print(json.dumps(log[::4] + log[-2:]))
