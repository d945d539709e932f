#!/usr/bin/env python3
"""composite_loss launch time on a steady-state training batch, with and
without the fused sample-index compaction (diagnostic)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import synthetic as S  # noqa: E402
import vren  # noqa: E402
from trainer import NGPTrainer, ctypes_float  # noqa: E402
import hashgrid as HG  # noqa: E402


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
    p = HG._ptr
    L = tr.L
    s = vren._stream()
    out = {}
    for name, with_idx in (("plain", False), ("compact", True)):
        def f():
            vren._ok(L.ngp_composite_loss(p(tr.sigmas), p(tr.rgbs), p(tr.deltas), p(tr.ts), p(tr.rays_a), 8192,
                                          p(tr.rgb_gt), p(tr.bg), 0, ctypes_float(1e-3), ctypes_float(0.0), ctypes_float(0.0),
                                          ctypes_float(0.5), ctypes_float(1e-4), p(tr.dsig), p(tr.drgb), p(tr.out_rgb),
                                          p(tr.out_op), p(tr.out_depth), p(tr.out_loss), p(tr.n_active),
                                          p(tr.sample_idx) if with_idx else None, p(tr._alloc_ws),
                                          p(tr.n_active_total), None, s), "cl")
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
    out["n_active_total"] = int(tr.n_active_total.item())
    out["samples"] = int(tr.n_samples.item())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
