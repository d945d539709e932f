#!/usr/bin/env python3
"""Standalone GPU time of each stage of a steady-state training step
(diagnostic): each stage re-run 20x back to back on the same inputs, no
overlap with the side-stream march.  Stages mutate only their outputs
(Adam is re-run on the same gradient: params drift, times don't)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd")]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from trainer import NGPTrainer, ctypes_float  # noqa: E402


def timed(f, reps=20):
    """Average GPU time of f: reps calls captured in one HIP graph and
    replayed (no host launch overhead in the number); eager if the stage
    cannot be captured."""
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                f()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
    except RuntimeError:
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)


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
    p, L, HGL, s, R = HG._ptr, tr.L, HG._lib(), vren._stream(), 8192
    cur = torch.cuda.current_stream()
    st = {}
    st["march"] = timed(lambda: tr._march(tr.cur, ("sample", 777, gt), dirs, poses, torch.cuda.current_stream()))
    st["field_fwd"] = timed(lambda: vren._ok(HGL.ngp_field_forward(
        p(tr.xyzs), p(tr.dirs), tr.cap, p(tr.n_samples), HG.ctypes.byref(tr.grid.desc), p(tr.params16[HG.MLP_PARAMS:]),
        p(tr.params16), p(tr.sigmas), p(tr.rgbs), p(tr.enc), None, vren._stream()), "ff"))
    K = 64
    def chunk_round(first_round):
        if first_round:
            vren._ok(L.ngp_chunk_counts(p(tr.rays_a), R, K, None, None, ctypes_float(1e-4), p(tr.eval_counts), vren._stream()), "c")
            vren._ok(L.ngp_ray_segments(p(tr.eval_counts), p(tr.rays_a), R, 0, p(tr.act_start), p(tr.eval_total), None,
                                        p(tr.eval_idx), vren._stream()), "sg")
        else:
            vren._ok(L.ngp_chunk_counts(p(tr.rays_a), R, K, p(tr.sigmas), p(tr.deltas), ctypes_float(1e-4),
                                        p(tr.eval_counts), vren._stream()), "c")
            vren._ok(L.ngp_ray_segments(p(tr.eval_counts), p(tr.rays_a), R, K, p(tr.act_start), p(tr.eval_total), None,
                                        p(tr.eval_idx), vren._stream()), "sg")
    field_ix = lambda: tr._field_indexed(vren._stream())  # noqa: E731
    st["chunk1_list"] = timed(lambda: chunk_round(True))
    st["chunk1_field"] = timed(field_ix)
    st["chunk1_n"] = int(tr.eval_total.item())
    st["chunk2_list"] = timed(lambda: chunk_round(False))
    st["chunk2_field"] = timed(field_ix)
    st["chunk2_n"] = int(tr.eval_total.item())
    st["composite"] = timed(lambda: vren._ok(L.ngp_composite_loss(
        p(tr.sigmas), p(tr.rgbs), p(tr.deltas), p(tr.ts), p(tr.rays_a), R, p(tr.rgb_gt), p(tr.bg), 0,
        ctypes_float(1e-3), ctypes_float(0.0), ctypes_float(0.0), ctypes_float(0.5), ctypes_float(1e-4), p(tr.dsig), p(tr.drgb),
        p(tr.out_rgb), p(tr.out_op), p(tr.out_depth), p(tr.out_loss), p(tr.n_active), None, None, None, None, vren._stream()), "cl"))
    st["active_samples"] = timed(lambda: vren._ok(L.ngp_active_samples(
        p(tr.n_active), p(tr.rays_a), R, p(tr.act_start), p(tr.n_active_total), p(tr.sample_idx), vren._stream()), "as"))
    st["mlp_bwd"] = timed(lambda: vren._ok(HGL.ngp_field_backward_mlp(
        p(tr.dirs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), p(tr.enc), 0, p(tr.params16), p(tr.dsig),
        p(tr.drgb), p(tr.denc), p(tr.grad), vren._stream()), "mb"))
    st["hash_bwd_binned_fine"] = timed(lambda: vren._ok(HGL.ngp_hash_backward_binned(
        p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), HG.ctypes.byref(tr.grid.desc), p(tr.denc),
        p(tr.grad[HG.MLP_PARAMS:]), p(tr.bin_ws), tr.bin_max_samples, tr.bin_level_lo, 0, vren._stream()), "hb"))
    st["hash_bwd_atomic_coarse"] = timed(lambda: vren._ok(HGL.ngp_hash_backward_levels(
        p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), HG.ctypes.byref(tr.grid.desc), p(tr.denc),
        p(tr.grad[HG.MLP_PARAMS:]), 0, tr.bin_level_lo, vren._stream()), "ha"))
    for lo, hi in ((0, 2), (2, 4), (4, 6), (6, 8), (8, 10), (10, 12), (12, 14), (14, 16)):
        st[f"hash_atomic_L{lo}_{hi}"] = timed(lambda: vren._ok(HGL.ngp_hash_backward_levels(
            p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), HG.ctypes.byref(tr.grid.desc), p(tr.denc),
            p(tr.grad[HG.MLP_PARAMS:]), lo, hi, vren._stream()), "hl"))
    for lo in (4, 6, 10, 12):
        st[f"hash_binned_from_L{lo}"] = timed(lambda: vren._ok(HGL.ngp_hash_backward_binned(
            p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), HG.ctypes.byref(tr.grid.desc), p(tr.denc),
            p(tr.grad[HG.MLP_PARAMS:]), p(tr.bin_ws), tr.bin_max_samples, lo, 0, vren._stream()), "hb"))
    st["hash_bwd_atomic_all"] = timed(lambda: vren._ok(HGL.ngp_hash_backward(
        p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), HG.ctypes.byref(tr.grid.desc), p(tr.denc),
        p(tr.grad[HG.MLP_PARAMS:]), vren._stream()), "hall"))
    st["adam"] = timed(lambda: vren._ok(L.ngp_adam_step(
        p(tr.params), p(tr.grad), p(tr.exp_avg), p(tr.exp_avg_sq), p(tr.params16), tr.params.numel(),
        ctypes_float(1e-2), ctypes_float(0.9), ctypes_float(0.999), ctypes_float(1e-15), 100, ctypes_float(1.0), 0,
        vren._stream()), "adam"))
    st["occupancy_update"] = timed(lambda: tr.update_density_grid(0.01 * 1024 / 3 ** 0.5), reps=5)
    st["density_fwd_1M"] = timed(lambda: HG.density_forward(tr.xyzs[:1 << 20].contiguous(), tr.grid, tr.params16), reps=5)
    import time
    torch.cuda.synchronize()
    c0 = time.perf_counter()
    for _ in range(48):
        tr.train_step(gt, dirs, poses)
    c1 = time.perf_counter()
    torch.cuda.synchronize()
    c2 = time.perf_counter()
    st["cpu_enqueue_us_per_step"] = round((c1 - c0) / 48 * 1e6, 1)
    st["wall_us_per_step"] = round((c2 - c0) / 48 * 1e6, 1)
    st["samples"] = int(tr.n_samples.item())
    st["active"] = int(tr.n_active_total.item())
    print(json.dumps(st))


if __name__ == "__main__":
    main()
