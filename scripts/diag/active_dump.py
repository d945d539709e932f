#!/usr/bin/env python3
"""Dump the gradient-carrying samples of steady-state training steps (their
positions in list order, the per-ray counts) to gpurun_out/active.npz -- input
of scripts/diag/coarse_requests.py, which counts the coarse hash backward's
memory-side atomic requests under different merge schemes on the CPU."""
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
    out = {}
    for s in range(4):
        tr.train_step(gt, dirs, poses, allow_pair=False)
        tr.drain()
        torch.cuda.synchronize()
        na = int(tr.n_active_total.item())
        idx = tr.sample_idx[:na].long()
        out[f"xyz{s}"] = tr.xyzs[idx].cpu().numpy()
        out[f"nact{s}"] = tr.n_active.cpu().numpy()
        out[f"nmarch{s}"] = np.int64(tr.n_samples.item())
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed("gpurun_out/active.npz", **out)
    print("ok", [out[f"xyz{s}"].shape[0] for s in range(4)])


if __name__ == "__main__":
    main()
