#!/usr/bin/env python3
"""Training-march launch time vs rays per wave (diagnostic): the walk is a
serial latency-bound chain per ray, so the number of SIMDs it spreads over
matters more than lane efficiency.  Runs the trainer to a steady-state
occupancy grid first, then times ngp_march_train_slots alone (no overlap)."""
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
    for _ in range(int(os.environ.get("PRETRAIN", "2000"))):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    out = {"samples": int(tr.n_samples.item())}
    src = ("sample", 12345, gt)
    cur = torch.cuda.current_stream()
    for ser, stage, rpw in [(1, 0, 4), (0, 0, 16), (0, 1, 16), (0, 2, 16)]:
        os.environ["NGP_MARCH_SERIAL"] = str(ser)
        os.environ["NGP_MARCH_DIAG"] = str(stage)
        os.environ["NGP_MARCH_RPW"] = str(rpw)
        os.environ["NGP_MARCH_STAGE"] = str(stage)
        for _ in range(3):
            tr._march(0, src, dirs, poses, cur)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            tr._march(0, src, dirs, poses, cur)
        e1.record()
        torch.cuda.synchronize()
        out[f"ser{ser}_s{stage}_rpw{rpw}_us"] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
    os.environ["NGP_MARCH_RPW"] = "16"
    os.environ["NGP_MARCH_STAGE"] = "0"
    os.environ["NGP_MARCH_SERIAL"] = "0"
    os.environ["NGP_MARCH_DIAG"] = "0"
    saved = tr.density_bitfield.clone()
    for name, val in (("empty", 0), ("full", 255)):
        tr.density_bitfield.fill_(val)
        tr._march(0, src, dirs, poses, cur)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            tr._march(0, src, dirs, poses, cur)
        e1.record()
        torch.cuda.synchronize()
        out[f"{name}_us"] = round(e0.elapsed_time(e1) / 10 * 1e3, 1)
        out[f"{name}_samples"] = int(tr.msets[0]["n_samples"].item())
    tr.density_bitfield.copy_(saved)
    c = tr.msets[0]["counts"]
    tr._march(0, src, dirs, poses, cur)
    torch.cuda.synchronize()
    out["count_max"] = int(c.max())
    out["count_mean_hit"] = float(c[c > 0].float().mean())
    out["hit_frac"] = float((c > 0).float().mean())
    ht = tr.msets[0]["hits_t"]
    span = (ht[:, 1] - ht[:, 0]).clamp(min=0)
    out["tspan_mean"] = float(span.mean())
    out["tspan_max"] = float(span.max())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
