#!/usr/bin/env python3
"""Where an item (bucket chunk) of the binned accumulation + fused Adam
(hash_accum_kernel<true>) spends its time (diagnostic; scripts/diag/accum_phases.hip):
the product kernel built with wall-clock stamps per item, run on the records of
steady-state Lego-shaped steps (the trainer pretrained like bench.py; each run
applies one extra Adam step to the trainer's state -- a measurement only).
Prints one JSON line: per-phase median / mean microseconds over items, items
per block, and the block span."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
HERE = os.path.join(ROOT, "scripts", "diag")
sys.path[:0] = [os.path.join(ROOT, "ar-nerf_amd"), HERE]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import synthetic as S  # noqa: E402
import vren  # noqa: E402
from trainer import NGPTrainer, _p, ctypes_float  # noqa: E402

PHASES = ["search", "zero_prefetch", "records", "adam_flush"]


def main():
    lib_path = os.path.join(HERE, "libaccdiag.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-C", HERE, "libaccdiag.so"], check=True)
    D = ctypes.CDLL(lib_path)
    vp, i64, ci, cf = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
    P = ctypes.POINTER(HG.ngp_hashgrid_t)
    D.ngp_hash_binned_plan.argtypes = [vp, i64, vp, vp, P, vp, i64, ci, ci, vp]
    D.ngp_hash_binned_apply_adam.argtypes = [vp, i64, vp, vp, P, vp, vp, vp, i64, ci, ci, vp, vp, vp, vp, vp, cf, cf,
                                             cf, vp, cf, vp]
    D.ngp_diag_acc_stamps.argtypes = [vp, ci]
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
    host = np.zeros(1024 * 8 * 5, dtype=np.uint64)
    d_all, spans, nitems, launch = [], [], [], []
    t = HG.MLP_PARAMS
    g = ctypes.byref(tr.grid.desc)
    for rep in range(12):
        tr.train_step(gt, dirs, poses)
        tr.drain()
        torch.cuda.synchronize()
        s = vren._stream()
        vren._ok(D.ngp_hash_binned_plan(_p(tr.xyzs), tr.cap, _p(tr.n_active_total), _p(tr.sample_idx), g,
                                        _p(tr.bin_ws), tr.bin_max_samples, tr.bin_level_lo, tr.bin_merge_hi, s),
                 "plan")
        torch.cuda.synchronize()
        assert D.ngp_diag_acc_stamps(None, 1) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        vren._ok(D.ngp_hash_binned_apply_adam(
            _p(tr.xyzs), tr.cap, _p(tr.n_active_total), _p(tr.sample_idx), g, _p(tr.denc), _p(tr.grad[t:]),
            _p(tr.bin_ws), tr.bin_max_samples, tr.bin_level_lo, tr.bin_merge_hi, _p(tr.params[t:]),
            _p(tr.exp_avg[t:]), _p(tr.exp_avg_sq[t:]), _p(tr.params16[t:]), _p(tr.lr_dev), ctypes_float(0.9),
            ctypes_float(0.999), ctypes_float(1e-15), _p(tr.dctr), ctypes_float(1.0), s), "apply_adam")
        e1.record()
        torch.cuda.synchronize()
        if rep < 2:
            continue
        launch.append(e0.elapsed_time(e1) * 1e3)
        assert D.ngp_diag_acc_stamps(host.ctypes.data, 0) == 0
        st = host.reshape(1024, 8, 5).astype(np.int64)
        t0 = st[st > 0].min()
        for b in range(1024):
            k = int((st[b, :, 0] > 0).sum())
            if k == 0:
                continue
            nitems.append(k)
            rows = st[b, :k]
            ok = (rows > 0).all(1)
            d_all.extend(list(np.diff(rows[ok], axis=1) * 10e-3))
            spans.append((rows[k - 1, 4] - rows[0, 0]) * 10e-3 if rows[k - 1, 4] > 0 else np.nan)
    d = np.array(d_all)
    res = {"apply_launch_us_median": round(float(np.median(launch)), 2),
           "items_per_block": {str(k): int(v) for k, v in zip(*np.unique(nitems, return_counts=True))},
           "phase_us_median": {p: round(float(np.median(d[:, i])), 3) for i, p in enumerate(PHASES)},
           "phase_us_mean": {p: round(float(d[:, i].mean()), 3) for i, p in enumerate(PHASES)},
           "phase_us_p90": {p: round(float(np.percentile(d[:, i], 90)), 3) for i, p in enumerate(PHASES)},
           "block_span_us": {"median": round(float(np.nanmedian(spans)), 2), "max": round(float(np.nanmax(spans)), 2)}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
