#!/usr/bin/env python3
"""Samples per chunk round of the chunked field evaluation and the GPU time
of the encode / MLP forward of each round on a steady-state step
(diagnostic).  Prints one JSON line."""
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
from trainer import NGPTrainer, ctypes_float  # noqa: E402


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
    p, L, HGL, R, K = HG._ptr, tr.L, HG._lib(), 8192, tr.chunk_first
    st = {"marched": int(tr.n_samples.item())}

    def enc():
        vren._ok(HGL.ngp_hash_encode(p(tr.xyzs), tr.cap, p(tr.eval_total), p(tr.eval_idx), HG.ctypes.byref(tr.grid.desc),
                                     p(tr.params16[HG.MLP_PARAMS:]), p(tr.enc), vren._stream()), "enc")

    def mlp():
        vren._ok(HGL.ngp_field_mlp_forward(p(tr.enc), p(tr.dirs), tr.cap, p(tr.eval_total), p(tr.eval_idx),
                                           p(tr.params16), p(tr.sigmas), p(tr.rgbs), None, vren._stream()), "mlp")
    s = vren._stream()
    vren._ok(L.ngp_ray_segments_capped(p(tr.rays_a), R, K, p(tr.act_start), p(tr.eval_total), None, p(tr.eval_idx), s), "sc")
    torch.cuda.synchronize()
    st["round1"] = int(tr.eval_total.item())
    st["round1_encode_us"], st["round1_mlp_us"] = timed(enc), timed(mlp)
    vren._ok(L.ngp_chunk_counts(p(tr.rays_a), R, K, p(tr.sigmas), p(tr.deltas), ctypes_float(1e-4), p(tr.eval_counts), s), "cc")
    vren._ok(L.ngp_ray_segments(p(tr.eval_counts), p(tr.rays_a), R, K, p(tr.act_start), p(tr.eval_total), None,
                                p(tr.eval_idx), s), "sg")
    torch.cuda.synchronize()
    st["round2"] = int(tr.eval_total.item())
    st["round2_encode_us"], st["round2_mlp_us"] = timed(enc), timed(mlp)
    st["segments_capped_us"] = timed(lambda: vren._ok(L.ngp_ray_segments_capped(
        p(tr.rays_a), R, K, p(tr.act_start), p(tr.eval_total), None, p(tr.eval_idx), vren._stream()), "sc"))
    print(json.dumps(st))


if __name__ == "__main__":
    main()
