#!/usr/bin/env python3
"""Per-ray marched vs gradient-carrying (up to termination) sample counts on
a steady-state batch, and the samples a chunked forward would evaluate
(first K per ray, then the rest of the rays still alive)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
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
    torch.cuda.synchronize()
    N = tr.rays_a[:, 2].float()
    A = tr.n_active.float()
    term = A < N  # terminated before exhausting
    out = {"marched": int(N.sum()), "active": int(A.sum()), "rays_hit": int((N > 0).sum()),
           "terminated_rays": int(term.sum()), "mean_N_hit": float(N[N > 0].mean()),
           "mean_active_hit": float(A[N > 0].mean())}
    for K in (16, 32, 48, 64, 96, 128):
        first = torch.minimum(N, torch.full_like(N, K))
        alive = (A >= K) & (N > K)  # not terminated within the first K evaluated
        rest = torch.where(alive, N - K, torch.zeros_like(N))
        out[f"eval_K{K}"] = int(first.sum() + rest.sum())
        for K2 in (2 * K,):
            alive2 = (A >= K2) & (N > K2)
            second = torch.where(alive, torch.minimum(N, torch.full_like(N, K2)) - K, torch.zeros_like(N))
            rest2 = torch.where(alive2, N - K2, torch.zeros_like(N))
            out[f"eval_K{K}_{K2}"] = int(first.sum() + second.sum() + rest2.sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
