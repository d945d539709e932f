#!/usr/bin/env python3
"""The reference's loop on the drop-in surface (bench.DropinLoop: render_rays +
NeRFLoss + backward + FusedAdam on models.networks.NGP), timed after the
bench's setup training, with its steps bracketed by trace markers so a
rocprofv3 kernel trace of this command can be cut to them
(scripts/kstats.py); prints the wall time per step and, with torch's
profiler, the host-side ops that take the most CPU time per step.
usage: dropin_profile.py [setup_steps=2000] [steps=40] [--torch-profile]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from trainer import NGPTrainer  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n_setup = int(args[0]) if args else 2000
    steps = int(args[1]) if len(args) > 1 else 40
    dev = torch.device("cuda")
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = scene.gt_images(device=dev)
    dirs, poses = scene.directions.to(dev).contiguous(), scene.poses.to(dev).contiguous()
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev)
    tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    for i in range(n_setup):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    loop = bench.DropinLoop(tr, gt, dirs, poses, 8192)
    for _ in range(5):
        loop.step()
    torch.cuda.synchronize()
    vren._ok(vren.lib().ngp_trace_marker(1, vren._stream()), "trace_marker")
    t0 = time.perf_counter()
    rm = vr = 0
    for _ in range(steps):
        _, res = loop.step()
        rm += res["rm_samples"]
        vr += res["vr_samples"]
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    vren._ok(vren.lib().ngp_trace_marker(2, vren._stream()), "trace_marker")
    torch.cuda.synchronize()
    out = {"ms_per_step": round(t * 1e3, 3), "rays_per_s": round(8192 / t), "rm_per_ray": round(float(rm) / steps / 8192, 2),
           "vr_per_ray": round(float(vr) / steps / 8192, 2)}
    if "--torch-profile" in sys.argv:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            for _ in range(10):
                loop.step()
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25), file=sys.stderr)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
