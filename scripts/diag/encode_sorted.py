#!/usr/bin/env python3
"""hash_encode / field_fwd / hash_bwd launch time on the real training samples
in ray order vs sorted by a spatial Morton key (diagnostic: how much of the
gather/scatter cost is locality)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

vp = ctypes.c_void_p


def spread(v):
    v = v & 0x3FF
    v = (v | (v << 16)) & 0x030000FF
    v = (v | (v << 8)) & 0x0300F00F
    v = (v | (v << 4)) & 0x030C30C3
    v = (v | (v << 2)) & 0x09249249
    return v


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
    n = int(tr.n_samples.item())
    xyz = tr.xyzs[:n].clone()
    d = tr.dirs[:n].clone()
    q = ((xyz / 0.5 + 1) * 0.5 * 1023).clamp(0, 1023).long()
    key = spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)
    t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    perm = torch.argsort(key)
    t1.record()
    torch.cuda.synchronize()
    out = {"n": n, "torch_argsort_us": round(t0.elapsed_time(t1) * 1e3, 1)}
    L = HG._lib()
    s = vp(torch.cuda.current_stream().cuda_stream)
    p = lambda t: vp(t.data_ptr())  # noqa: E731
    grid = tr.grid
    p16 = tr.params16
    enc_pm = torch.empty(8, n, 4, dtype=torch.float16, device=dev)
    sig, rgb = torch.empty(n, device=dev), torch.empty(n, 3, device=dev)
    enc = torch.empty(n, 32, dtype=torch.float16, device=dev)
    denc = torch.randn(n, 32, device=dev) * 1e-3
    grad = torch.zeros(tr.params.numel(), device=dev)
    for name, (x, dd) in (("ray_order", (xyz, d)), ("morton_sorted", (xyz[perm].contiguous(), d[perm].contiguous()))):
        fns = {
            "encode": lambda: L.ngp_hash_encode(p(x), n, None, None, ctypes.byref(grid.desc), p(p16[HG.MLP_PARAMS:]),
                                                p(enc_pm), s),
            "fused_fwd": lambda: L.ngp_field_forward(p(x), p(dd), n, None, ctypes.byref(grid.desc),
                                                     p(p16[HG.MLP_PARAMS:]), p(p16), p(sig), p(rgb), p(enc), None, s),
            "hash_bwd_atomic": lambda: L.ngp_hash_backward(p(x), n, None, None, ctypes.byref(grid.desc), p(denc),
                                                           p(grad[HG.MLP_PARAMS:]), s),
        }
        for k, f in fns.items():
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            out[f"{name}_{k}_us"] = round(e0.elapsed_time(e1) / 10 * 1e3, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
