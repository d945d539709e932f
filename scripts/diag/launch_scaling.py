#!/usr/bin/env python3
"""GPU time of the encode and the MLP forward vs the sample count (the
device-side count n_dev; same capacity and grid) on a steady-state model:
separates each kernel's fixed cost from its per-sample cost (diagnostic)."""
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
    for _ in range(500):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    p, HGL = HG._ptr, HG._lib()
    nd = torch.zeros(1, dtype=torch.int64, device=dev)
    st = {"marched": int(tr.n_samples.item())}
    for n in (64, 20000, 80000, 160000, 320000, 560000):
        nd.fill_(min(n, st["marched"]))
        st[f"encode_{n}"] = timed(lambda: vren._ok(HGL.ngp_hash_encode(
            p(tr.xyzs), tr.cap, p(nd), None, HG.ctypes.byref(tr.grid.desc), p(tr.params16[HG.MLP_PARAMS:]),
            p(tr.enc), vren._stream()), "enc"))
        st[f"mlp_fwd_{n}"] = timed(lambda: vren._ok(HGL.ngp_field_mlp_forward(
            p(tr.enc), p(tr.dirs), tr.cap, p(nd), None, p(tr.params16), p(tr.sigmas), p(tr.rgbs), None,
            vren._stream()), "mlp"))
    print(json.dumps(st))


if __name__ == "__main__":
    main()
