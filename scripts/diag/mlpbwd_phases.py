#!/usr/bin/env python3
"""Where a block iteration of the MLP backward (field_bwd_mlp_coop_kernel) spends
its time (diagnostic; scripts/diag/mlpbwd_phases.hip): the product kernel built
with wall-clock stamps at its phase boundaries, run on the gradient-carrying
samples of steady-state Lego-shaped steps (the trainer pretrained like bench.py).
Prints one JSON line: per-phase median / mean microseconds over blocks and
iterations, iterations per block, and the launch time."""
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
from trainer import NGPTrainer, _p  # noqa: E402

PHASES = ["fwd_recompute", "data_chain", "exp_barrier", "put1_barrier", "dw1_barrier", "put2_barrier", "dw2"]


def main():
    lib_path = os.path.join(HERE, "libmlpdiag.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-C", HERE, "libmlpdiag.so"], check=True)
    D = ctypes.CDLL(lib_path)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    D.ngp_field_backward_mlp.argtypes = [vp, i64, vp, vp, vp, i64, vp, vp, vp, vp, vp, vp]
    D.ngp_diag_bwd_stamps.argtypes = [vp, vp, ctypes.c_int]
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
    host = np.zeros(1024 * 8 * 8, dtype=np.uint64)
    edges = np.zeros(1024 * 4, dtype=np.uint64)
    edge_d = []
    deltas, iters, launch = [], [], []
    grad = torch.zeros_like(tr.grad[:HG.MLP_PARAMS])
    for rep in range(12):
        tr.train_step(gt, dirs, poses)
        tr.drain()
        torch.cuda.synchronize()
        n_act = int(tr.n_active_total.item())
        assert D.ngp_diag_bwd_stamps(None, None, 1) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        vren._ok(D.ngp_field_backward_mlp(_p(tr.dirs), tr.cap, _p(tr.n_active_total), _p(tr.sample_idx), _p(tr.enc),
                                          tr.cap, _p(tr.params16), _p(tr.dsig), _p(tr.drgb), _p(tr.denc), _p(grad),
                                          vren._stream()), "bwd_diag")
        e1.record()
        torch.cuda.synchronize()
        if rep < 2:
            continue
        launch.append(e0.elapsed_time(e1) * 1e3)
        assert D.ngp_diag_bwd_stamps(host.ctypes.data, edges.ctypes.data, 0) == 0
        ed = edges.reshape(1024, 4).astype(np.int64)
        ed = ed[ed[:, 0] > 0]
        t0 = ed[:, 0].min()
        # per block: start offset vs the first block, staging, loop, atomics, end offset
        edge_d.append(np.stack([ed[:, 0] - t0, ed[:, 1] - ed[:, 0], ed[:, 2] - ed[:, 1], ed[:, 3] - ed[:, 2],
                                ed[:, 3] - t0], 1) * 10e-3)
        st = host.reshape(1024, 8, 8).astype(np.int64)
        for b in range(1024):
            nit = int((st[b, :, 0] > 0).sum())
            if nit == 0:
                continue
            iters.append(nit)
            for it in range(nit):
                row = st[b, it]
                if (row > 0).all():
                    deltas.append(np.diff(row) * 10e-3)  # 100 MHz ticks -> us
        out_n = n_act
    d = np.array(deltas)
    res = {"n_active": out_n, "launch_us_median": float(np.median(launch)),
           "iterations_per_block": {str(k): int(v) for k, v in zip(*np.unique(iters, return_counts=True))},
           "phase_us_median": {p: round(float(np.median(d[:, i])), 3) for i, p in enumerate(PHASES)},
           "phase_us_mean": {p: round(float(d[:, i].mean()), 3) for i, p in enumerate(PHASES)},
           "iteration_us_median": round(float(np.median(d.sum(1))), 3)}
    e = np.concatenate(edge_d)
    for i, name in enumerate(["start_offset", "staging", "loop", "atomics", "end_offset"]):
        res[f"edge_{name}_us"] = {"median": round(float(np.median(e[:, i])), 2), "max": round(float(e[:, i].max()), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
