#!/usr/bin/env python3
"""Profiling driver for the test-time renderer (BASELINE config 5): trains the
bench's synthetic Lego-shaped scene for --pretrain steps, then renders
--frames full frames with renderer.TestRenderer.  Run under rocprofv3
--kernel-trace and summarise with scripts/render_kstats.py."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ar-nerf_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pretrain", type=int, default=2000)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--iters-per-graph", type=int, default=16)
    a = ap.parse_args()
    import synthetic as S
    from trainer import NGPTrainer
    torch.cuda.set_device(0)
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    tr = NGPTrainer(scale=0.5, batch_size=8192, device="cuda")
    gt = scene.gt_images(device="cuda")
    dirs, poses = scene.directions.cuda().contiguous(), scene.poses.cuda().contiguous()
    t0 = time.time()
    for _ in range(a.pretrain):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    print(f"pretrain {a.pretrain} steps {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    out = bench.inference_bench(tr, a.res, a.frames, 1, 0)
    print(out, flush=True)


if __name__ == "__main__":
    main()
