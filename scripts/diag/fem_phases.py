#!/usr/bin/env python3
"""When the waves of the fused encode + MLP forward gather and when they run
their MLPs (diagnostic; scripts/diag/fem_phases.hip): the product kernel built
with per-wave wall-clock stamps, run on 155 K marched samples of a steady-state
Lego-shaped batch (the trainer pretrained like bench.py).  Prints one JSON
line: percentiles (us from the first wave's start) of wave start, gathers done
and MLPs done, and per-wave gather / MLP durations."""
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


def main():
    lib_path = os.path.join(HERE, "libfemdiag.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-C", HERE, "libfemdiag.so"], check=True)
    D = ctypes.CDLL(lib_path)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    P = ctypes.POINTER(HG.ngp_hashgrid_t)
    D.ngp_field_encode_mlp.argtypes = [vp, vp, i64, vp, vp, P, vp, vp, vp, vp, vp, vp, vp]
    D.ngp_diag_fem_stamps.argtypes = [vp, ctypes.c_int]
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
    n = min(int(tr.n_samples.item()), 155000)
    x, d = tr.xyzs[:n].contiguous(), tr.dirs[:n].contiguous()
    enc = torch.zeros(8, n, 4, dtype=torch.float16, device=dev)
    sig, rgb = torch.empty(n, device=dev), torch.empty(n, 3, device=dev)
    table = tr.params16[HG.MLP_PARAMS:]
    host = np.zeros(4096 * 16 * 3, dtype=np.uint64)
    rows = []
    launch = []
    for rep in range(10):
        assert D.ngp_diag_fem_stamps(None, 1) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        vren._ok(D.ngp_field_encode_mlp(_p(x), _p(d), n, None, None, ctypes.byref(tr.grid.desc), _p(table),
                                        _p(tr.params16), _p(enc), _p(sig), _p(rgb), None, vren._stream()), "fem")
        e1.record()
        torch.cuda.synchronize()
        if rep < 2:
            continue
        launch.append(e0.elapsed_time(e1) * 1e3)
        assert D.ngp_diag_fem_stamps(host.ctypes.data, 0) == 0
        st = host.reshape(-1, 3).astype(np.int64)
        st = st[st[:, 0] > 0]
        st = (st - st[:, 0].min()) * 10e-3
        rows.append(st)
    st = np.concatenate(rows)
    q = [10, 50, 90, 99, 100]
    pct = lambda a: {str(p): round(float(np.percentile(a, p)), 2) for p in q}  # noqa: E731
    res = {"n": n, "launch_us_median": round(float(np.median(launch)), 2), "waves": int(len(st) / len(rows)),
           "start": pct(st[:, 0]), "gathers_done": pct(st[:, 1]), "mlp_done": pct(st[:, 2]),
           "gather_us": pct(st[:, 1] - st[:, 0]), "mlp_us": pct(st[:, 2] - st[:, 1])}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
