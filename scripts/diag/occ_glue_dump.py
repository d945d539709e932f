"""Run the reference glue's occupancy cases locally (as make_golden.py does)
and compare with the product dump from scripts/diag/occ_dump.py."""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path[:0] = [os.path.join(ROOT, "tests", "golden")]
import numpy as np
import torch
import make_golden as MG
MG.install_stubs()
import synthetic as S
from models.networks import NGP
torch.set_num_threads(1)
P = np.load(os.path.join(ROOT, "gpurun_out/occdump/product.npz"))
thr = 0.01 * 1024 / 3 ** 0.5


def model(scale):
    m = NGP(scale)
    G = m.grid_size
    ax = torch.arange(G, dtype=torch.int32)
    m.register_buffer("density_grid", torch.zeros(m.cascades, G ** 3))
    m.register_buffer("grid_coords", torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3))
    return m


def cmp(name, a, b):
    d = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
    print(f"{name}: {len(d)} cells differ", end="")
    if len(d):
        print(f"; e.g. {[(int(i), float(a.reshape(-1)[i]), float(b.reshape(-1)[i])) for i in d[:5]]}")
    else:
        print()
    return d


for tag, scale in (("lego", 0.5), ("garden", 16.0)):
    sc = S.AnalyticScene(W=64, H=48, n_images=10, scale=scale)
    m = model(scale)
    m.mark_invisible_cells(sc.K, sc.poses, (64, 48))
    k_ref = torch.round(m.count_grid * 10).numpy()
    k_got = np.round(P[f"{tag}_count"] * 10)
    cmp(f"{tag} k", k_got, k_ref)
# erode chain
seed, amp = 5, 1.0
sc = S.AnalyticScene(W=64, H=48, n_images=10, scale=0.5)
m = model(0.5)
MG.table_override(m, 100 + seed, amp)
m.mark_invisible_cells(sc.K, sc.poses, (64, 48))
torch.manual_seed(seed)
m.update_density_grid(thr, warmup=True, erode=True)
w1 = m.density_grid.numpy().copy()
d = cmp("erode warm1", P["e_warm1"], w1)
m.update_density_grid(thr, warmup=True, erode=True)
w2 = m.density_grid.numpy().copy()
d = cmp("erode warm2", P["e_warm2"], w2)
torch.manual_seed(seed + 1)
m.update_density_grid(thr, warmup=False, erode=True)
cmp("erode upd", P["e_upd"], m.density_grid.numpy())
# density_update
seed = 4
m = model(0.5)
MG.table_override(m, 100 + seed, amp)
torch.manual_seed(seed)
m.update_density_grid(thr, warmup=True)
dw = cmp("plain warm", P["d_warm"], m.density_grid.numpy())
g = m.density_grid
print("occupied (> thr) after warm: glue", int((g > thr).sum()), "product", int((torch.from_numpy(P["d_warm"]) > thr).sum()))
torch.manual_seed(seed + 1)
m.update_density_grid(thr, warmup=False)
cmp("plain upd", P["d_upd"], m.density_grid.numpy())
for i in (1383506,):
    print("cell", i, "product warm1/warm2", P["e_warm1"][0, i], P["e_warm2"][0, i], "glue", w1[0, i], w2[0, i])
for name, g in (("erode warm2", w2), ("plain warm", P["d_warm"])):
    lg = np.abs(np.log(np.maximum(g, 1e-30)) - np.log(thr))
    print(name, "cells within 0.02 / 0.05 of thr (log):", int((lg < 0.02).sum()), int((lg < 0.05).sum()))
