#!/usr/bin/env python3
"""Dump per-row marched counts and gradient-carrying counts of steady-state
training steps (diagnostic for the chunk-round schedule) to an .npz."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402


def main():
    dev = torch.device("cuda")
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = scene.gt_images(device=dev)
    dirs, poses = scene.directions.to(dev), scene.poses.to(dev)
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev)
    tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    for _ in range(2000):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    n, a = [], []
    for _ in range(8):
        tr.train_step(gt, dirs, poses)
        tr.drain()
        torch.cuda.synchronize()
        n.append(tr.rays_a[:, 2].cpu().numpy().copy())
        a.append(tr.n_active.cpu().numpy().copy())
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez("gpurun_out/rows.npz", n=np.stack(n), a=np.stack(a))
    print("ok", np.stack(n).mean(), np.stack(a).mean())


if __name__ == "__main__":
    main()
