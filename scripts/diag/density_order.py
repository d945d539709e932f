"""Density-forward cost of the occupancy update's 1M points: random cell
order (as drawn) vs sorted by Morton code (cache locality of the coarse
levels inside a wave), plus torch.sort's own cost."""
import os
import sys

H = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(H, "..", ".."), os.path.join(H, "..", "..", "ar-nerf_amd")]
import torch  # noqa: E402

import hashgrid as HG  # noqa: E402
import vren  # noqa: E402


def timed(f, reps=10):
    for _ in range(2):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)


G, s = 128, 0.5
grid = HG.HashGrid(s)
p16 = (torch.rand(grid.n_params, device="cuda") * 2e-2 - 1e-2).half()
M = G ** 3 // 2
cells = torch.randint(0, G ** 3, (M,), device="cuda", dtype=torch.int32)


def points(c):
    xyz = vren.morton3D_invert(c.contiguous()).float()
    xyz = (xyz + torch.rand_like(xyz)) / G * 2 - 1
    return (xyz * s).contiguous()


res = {}
x_rand = points(cells)
res["random"] = timed(lambda: HG.density_forward(x_rand, grid, p16))
x_sort = points(torch.sort(cells)[0])
res["morton_sorted"] = timed(lambda: HG.density_forward(x_sort, grid, p16))
res["torch_sort_1M_int32"] = timed(lambda: torch.sort(cells))
xl = x_rand[torch.argsort(x_rand[:, 0])].contiguous()
res["x_sorted"] = timed(lambda: HG.density_forward(xl, grid, p16))
print(res)
