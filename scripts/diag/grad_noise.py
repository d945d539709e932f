"""Run-to-run spread of the training-step gradient (fp32 atomic summation
order) per parameter group / hash level: the same step from the same state
several times, each compared with the first."""
import os
import sys

H = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(H, "..", ".."), os.path.join(H, "..", "..", "tests"), os.path.join(H, "..", "..", "ar-nerf_amd")]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import test_trainer_gpu as T  # noqa: E402

REP = int(os.environ.get("REP", "5"))
gs = []
for _ in range(REP):
    sc, tr, img, pix, noise = T._setup(table_init=2.0)
    tr.chunk_first = 0
    dirs, poses = sc.directions.to("cuda"), sc.poses.to("cuda")
    o, d = sc.rays(img, pix)
    gt = sc.gt_rgb_rays(o, d).to("cuda")
    tr.step(img.to("cuda"), pix.to("cuda"), gt, dirs, poses, noise=noise.to("cuda"), apply_adam=False)
    torch.cuda.synchronize()
    gs.append(tr.grad.clone())
off = [0, HG.MLP_PARAMS] + [HG.MLP_PARAMS + 2 * o for o in tr.grid.offsets[1:]]
bad = 0
for r in range(1, REP):
    x, y = gs[r], gs[0]
    segs = [float((x[a:b] - y[a:b]).norm() / (y[a:b].norm() + 1e-30)) for a, b in zip(off[:-1], off[1:])]
    worst = max(range(len(segs)), key=lambda i: segs[i])
    bad += segs[worst] > 1e-4
    print(f"run {r}: total {float((x - y).norm() / y.norm()):.2e} worst seg {worst} {segs[worst]:.2e}")
print("corrupted runs:", bad, "of", REP - 1)
