#!/usr/bin/env python3
"""Field forward over one steady-state batch (all marched samples): fused
gathers+MLP (ngp_field_forward) vs the split path (ngp_hash_encode, level pair
per XCD, then ngp_field_mlp_forward), each stage alone."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd"), os.path.join(ROOT, "scripts", "diag")]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from stages import timed  # noqa: E402
from trainer import NGPTrainer  # noqa: E402


def main():
    dev = torch.device("cuda")
    scene = S.AnalyticScene(W=800, H=800, n_images=100, scale=0.5)
    gt = scene.gt_images(device=dev)
    dirs, poses = scene.directions.to(dev), scene.poses.to(dev)
    tr = NGPTrainer(scale=0.5, batch_size=8192, device=dev)
    tr.mark_invisible_cells(scene.K, scene.poses, (scene.W, scene.H))
    for _ in range(int(os.environ.get("PRETRAIN", "1000"))):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    p, HGL, s = HG._ptr, HG._lib(), vren._stream()
    n = int(tr.n_samples.item())
    enc_pm = torch.empty(8, tr.cap, 4, dtype=torch.float16, device=dev)
    st = {"n": n}
    st["fused"] = timed(lambda: vren._ok(HGL.ngp_field_forward(
        p(tr.xyzs), p(tr.dirs), tr.cap, p(tr.n_samples), HG.ctypes.byref(tr.grid.desc), p(tr.params16[HG.MLP_PARAMS:]),
        p(tr.params16), p(tr.sigmas), p(tr.rgbs), p(tr.enc), None, s), "ff"))
    st["density_only"] = timed(lambda: vren._ok(HGL.ngp_density_forward(
        p(tr.xyzs), tr.cap, p(tr.n_samples), HG.ctypes.byref(tr.grid.desc), p(tr.params16[HG.MLP_PARAMS:]),
        p(tr.params16), p(tr.sigmas), None, s), "df"))
    st["encode_split"] = timed(lambda: vren._ok(HGL.ngp_hash_encode(
        p(tr.xyzs), tr.cap, p(tr.n_samples), None, HG.ctypes.byref(tr.grid.desc), p(tr.params16[HG.MLP_PARAMS:]),
        p(enc_pm), s), "he"))
    st["mlp_only"] = timed(lambda: vren._ok(HGL.ngp_field_mlp_forward(
        p(enc_pm), p(tr.dirs), tr.cap, p(tr.n_samples), None, p(tr.params16), p(tr.sigmas), p(tr.rgbs), None, s),
        "mf"))
    print(json.dumps(st))


if __name__ == "__main__":
    main()
