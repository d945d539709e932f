"""One training step's gradient (trainer.NGPTrainer, the product) against the
oracle trainer with fp32 autograd and with the MLP backward's fp16 gradient
storage modelled (oracle.OracleNGPField.grad16), from the same state, rays and
noise (tests/test_trainer_gpu.py's setup).  Prints the relative L2 error per
parameter group for both oracles -- the calibration of the test bars.
Diagnostics only (GPU box): python scripts/diag/grad16_trainer.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "ar-nerf_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import oracle as O  # noqa: E402
import synthetic as S  # noqa: E402
from trainer import NGPTrainer  # noqa: E402

DEV = "cuda"


def main(R=2048, table_init=0.2, seed=3):
    sc = S.AnalyticScene(W=200, H=200, n_images=10)
    tr = NGPTrainer(scale=0.5, batch_size=R, device=DEV, seed=seed)
    with torch.no_grad():
        g = torch.Generator().manual_seed(11)
        tr.params[10240:] = ((torch.rand(tr.params.numel() - 10240, generator=g) * 2 - 1) * table_init).to(DEV)
        tr.params16.copy_(tr.params.half())
    tr.density_bitfield.copy_(sc.bitfield.to(DEV))
    tr.global_step = 1
    gen = torch.Generator().manual_seed(seed)
    img, pix = sc.sample_batch(R, gen)
    noise = torch.rand(R, generator=gen)
    o, d = sc.rays(img, pix)
    gt = sc.gt_rgb_rays(o, d)
    p0 = tr.params.detach().cpu().clone()
    tr.step(img.to(DEV), pix.to(DEV), gt.to(DEV), sc.directions.to(DEV), sc.poses.to(DEV), noise=noise.to(DEV),
            apply_adam=False)
    torch.cuda.synchronize()
    g_gpu = tr.grad.cpu()
    rays_o, rays_d, hits_t = tr.rays_o.cpu(), tr.rays_d.cpu(), tr.hits_t.cpu()
    refs = {}
    for g16 in (False, True):
        ot = O.OracleTrainer(p0, 0.5, tr.density_bitfield.cpu(), 1)
        ot.field.grad16 = g16
        ot.step(rays_o, rays_d, hits_t, gt, noise, torch.ones(3), apply_adam=False)
        refs[g16] = ot.flat_grad()
    for name, lo, hi in (("density MLP", 0, 3072), ("colour MLP", 3072, 10240), ("table", 10240, g_gpu.numel())):
        e32 = float((g_gpu[lo:hi] - refs[False][lo:hi]).norm() / refs[False][lo:hi].norm())
        e16 = float((g_gpu[lo:hi] - refs[True][lo:hi]).norm() / refs[True][lo:hi].norm())
        print(f"{name}: vs fp32 autograd {e32:.3e}, vs fp16-storage model {e16:.3e}")


if __name__ == "__main__":
    main()
