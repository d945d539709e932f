#!/usr/bin/env python3
"""The binned hash backward's passes alone on a steady-state Lego-shaped step
(diagnostic; scripts/diag/hashbin_diag.hip): plan (count + scan + plan), the
record write in its variants, the accumulation, the coarse atomic levels.
Prints one JSON line of average µs per launch (graph-replayed)."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HERE = os.path.join(ROOT, "scripts", "diag")
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd"), HERE]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from stages import timed  # noqa: E402
from trainer import NGPTrainer  # noqa: E402


class _S:  # the current stream at each call (timed() captures on a side stream)
    @property
    def _as_parameter_(self):
        return vren._stream()


def main():
    lib_path = os.path.join(HERE, "libhashbindiag.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-C", HERE, "libhashbindiag.so"], check=True)
    D = ctypes.CDLL(lib_path)
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    D.ngp_diag_hash_write.argtypes = [ci, vp, i64, vp, vp, vp, vp, vp, vp, i64, ci, ci, vp]
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
    p, HGL, s = HG._ptr, HG._lib(), _S()
    g = HG.ctypes.byref(tr.grid.desc)
    grad = torch.zeros_like(tr.grad)
    t = HG.MLP_PARAMS
    args = (p(tr.xyzs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), g)
    st = {"n_active": int(tr.n_active_total.item()), "bin_level_lo": tr.bin_level_lo}
    st["plan"] = timed(lambda: vren._ok(HGL.ngp_hash_binned_plan(*args, p(tr.bin_ws), tr.bin_max_samples,
                                                                  tr.bin_level_lo, 0, s), "plan"))
    for mode in (2, 3, 6, 0):
        st[f"write_mode{mode}"] = timed(lambda: vren._ok(D.ngp_diag_hash_write(
            mode, *args, p(tr.denc), p(grad[t:]), p(tr.bin_ws), tr.bin_max_samples, tr.bin_level_lo, 0, s), "w"))
    vren._ok(HGL.ngp_hash_binned_write(*args, p(tr.denc), p(grad[t:]), p(tr.bin_ws), tr.bin_max_samples,
                                       tr.bin_level_lo, 0, s), "write")
    st["accum"] = timed(lambda: vren._ok(HGL.ngp_hash_binned_accum(g, p(grad[t:]), p(tr.bin_ws), tr.bin_max_samples,
                                                                   tr.bin_level_lo, 0, s), "accum"))
    st["coarse_atomic_0_8"] = timed(lambda: vren._ok(HGL.ngp_hash_backward_levels(
        *args, p(tr.denc), p(grad[t:]), 0, tr.bin_level_lo, s), "coarse"))
    st["mlp_bwd"] = timed(lambda: vren._ok(HGL.ngp_field_backward_mlp(
        p(tr.dirs), tr.cap, p(tr.n_active_total), p(tr.sample_idx), p(tr.enc), tr.cap, p(tr.params16), p(tr.dsig),
        p(tr.drgb), p(tr.denc), p(grad), s), "mlpb"))
    print(json.dumps(st))


if __name__ == "__main__":
    main()
