#!/usr/bin/env python3
"""Host (enqueue) and wall time per steady-state train_step, graphs on/off,
and the host cost of one bare graph replay (diagnostic)."""
import json
import os
import sys
import time

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
    for _ in range(500):
        tr.train_step(gt, dirs, poses)
    torch.cuda.synchronize()
    out = {}
    for graphs in (True, False):
        tr.use_graphs = graphs
        for _ in range(32):
            tr.train_step(gt, dirs, poses)
        torch.cuda.synchronize()
        c0 = time.perf_counter()
        for _ in range(160):
            tr.train_step(gt, dirs, poses)
        c1 = time.perf_counter()
        torch.cuda.synchronize()
        c2 = time.perf_counter()
        out[f"graphs{int(graphs)}_host_us"] = round((c1 - c0) / 160 * 1e6, 1)
        out[f"graphs{int(graphs)}_wall_us"] = round((c2 - c0) / 160 * 1e6, 1)
    g = next(iter(tr._graphs.values()))
    torch.cuda.synchronize()
    c0 = time.perf_counter()
    for _ in range(50):
        g.replay()
    c1 = time.perf_counter()
    torch.cuda.synchronize()
    c2 = time.perf_counter()
    out["bare_replay_host_us"] = round((c1 - c0) / 50 * 1e6, 1)
    out["bare_replay_wall_us"] = round((c2 - c0) / 50 * 1e6, 1)
    out["n_graphs"] = len(tr._graphs)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
