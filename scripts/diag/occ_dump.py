"""Dump the product's occupancy grids (GPU) for the fixture cases of
tests/golden/occupancy_erode.npz / density_update.npz, to compare cell by
cell with a local glue run (scripts/diag/occ_glue_dump.py)."""
import os
import sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "ar-nerf_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import torch
from test_occupancy_gpu import _scene, _ngp, cpu_rng_replay, THR, load
from trainer import NGPTrainer

out = {}
fx = load("occupancy_erode")
for tag, scale in (("lego", 0.5), ("garden", 16.0)):
    sc = _scene(fx, scale)
    tr = NGPTrainer(scale=scale, batch_size=256, sample_capacity=256 * 64, device="cuda")
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    out[f"{tag}_count"] = tr.count_grid.cpu().numpy()
seed, amp = int(fx["seed"]), float(fx["amp"])
sc = _scene(fx, 0.5)
m = _ngp(0.5, seed, amp)
m.mark_invisible_cells(sc.K.cuda(), sc.poses.cuda(), (sc.W, sc.H))
torch.manual_seed(seed)
with cpu_rng_replay():
    m.update_density_grid(THR, warmup=True, erode=True)
    out["e_warm1"] = m.density_grid.cpu().numpy()
    m.update_density_grid(THR, warmup=True, erode=True)
    out["e_warm2"] = m.density_grid.cpu().numpy()
torch.manual_seed(seed + 1)
with cpu_rng_replay():
    m.update_density_grid(THR, warmup=False, erode=True)
out["e_upd"] = m.density_grid.cpu().numpy()
fx = load("density_update")
seed, amp = int(fx["seed"]), float(fx["amp"])
m = _ngp(0.5, seed, amp)
torch.manual_seed(seed)
with cpu_rng_replay():
    m.update_density_grid(THR, warmup=True)
out["d_warm"] = m.density_grid.cpu().numpy()
torch.manual_seed(seed + 1)
with cpu_rng_replay():
    m.update_density_grid(THR, warmup=False)
out["d_upd"] = m.density_grid.cpu().numpy()
os.makedirs("gpurun_out/occdump", exist_ok=True)
np.savez_compressed("gpurun_out/occdump/product.npz", **out)
print("saved", {k: v.shape for k, v in out.items()})
