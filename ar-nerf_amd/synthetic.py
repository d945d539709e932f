"""Seeded synthetic Lego-shaped workload (BASELINE.md "CPU-baseline plan",
SURVEY.md §8d): no dataset or checkpoint is reachable, so the benchmark and
the parity tests run on synthetic cameras, rays and occupancy of the exact
shapes the reference trains on.

* Camera: W x H pinhole, fx = fy = 0.5*W/tan(0.5*fov) (800 px -> 1111.111),
  cx = W/2, cy = H/2; directions through pixel centres
  (datasets/ray_utils.py:24-42, kornia create_meshgrid(H, W, False): u =
  column, v = row, pixel index = v*W + u).
* Poses: cameras on the upper hemisphere of radius 1.5 looking at the origin,
  Blender convention converted to "right down front" like
  datasets/nerf.py:70-73 (c2w[:, 1:3] *= -1).
* Occupancy: a thin spherical shell |r - 0.3| < 2/128 plus 2 % random cells,
  in Morton order, thresholded through packbits.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def intrinsics(W: int, H: int, focal: float | None = None):
    if focal is None:
        focal = 0.5 * 800 / math.tan(0.5 * 0.6911112070083618) * (W / 800)  # Lego camera_angle_x
    return torch.tensor([[focal, 0, W / 2], [0, focal, H / 2], [0, 0, 1]], dtype=torch.float32)


def get_ray_directions(H: int, W: int, K: torch.Tensor) -> torch.Tensor:
    """datasets/ray_utils.py:7-42 (random=False, flatten=True)."""
    v, u = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    d = torch.stack([(u - cx + 0.5) / fx, (v - cy + 0.5) / fy, torch.ones_like(u)], -1)
    return d.reshape(-1, 3)


def make_poses(n: int = 100, radius: float = 1.5, seed: int = 0) -> torch.Tensor:
    """(n,3,4) c2w on the upper hemisphere, looking at the origin."""
    g = np.random.default_rng(seed)
    poses = []
    for _ in range(n):
        theta = g.uniform(0, 2 * np.pi)
        phi = g.uniform(0.1, 0.45 * np.pi)  # elevation
        c = radius * np.array([np.cos(phi) * np.cos(theta), np.cos(phi) * np.sin(theta), np.sin(phi)])
        back = c / np.linalg.norm(c)  # OpenGL camera looks along -z
        right = np.cross(np.array([0.0, 0.0, 1.0]), back)
        right /= np.linalg.norm(right)
        up = np.cross(back, right)
        c2w = np.stack([right, up, back, c], 1)  # Blender/OpenGL
        c2w[:, 1:3] *= -1  # datasets/nerf.py:70-73 -> right, down, front
        poses.append(c2w)
    return torch.tensor(np.stack(poses), dtype=torch.float32)


def morton3(x, y, z):
    def spread(v):
        v = v.astype(np.uint64)
        v = (v * 0x00010001) & 0xFF0000FF
        v = (v * 0x00000101) & 0x0F00F00F
        v = (v * 0x00000011) & 0xC30C30C3
        v = (v * 0x00000005) & 0x49249249
        return v
    return (spread(x) | (spread(y) << 1) | (spread(z) << 2)).astype(np.int64)


def shell_density_grid(grid_size: int = 128, cascades: int = 1, scale: float = 0.5, radius: float = 0.3,
                       rand_frac: float = 0.02, seed: int = 2) -> torch.Tensor:
    """(cascades, G^3) f32 density grid in Morton order: 20 inside a thin
    shell around the origin plus `rand_frac` random cells, 0 elsewhere."""
    G = grid_size
    g = np.random.default_rng(seed)
    ax = np.arange(G)
    X, Y, Z = np.meshgrid(ax, ax, ax, indexing="ij")
    X, Y, Z = X.ravel(), Y.ravel(), Z.ravel()
    idx = morton3(X, Y, Z)
    grid = np.zeros((cascades, G ** 3), np.float32)
    for c in range(cascades):
        s = min(2.0 ** (c - 1), scale)
        cx = ((X + 0.5) / G * 2 - 1) * s
        cy = ((Y + 0.5) / G * 2 - 1) * s
        cz = ((Z + 0.5) / G * 2 - 1) * s
        r = np.sqrt(cx * cx + cy * cy + cz * cz)
        occ = (np.abs(r - radius) < 2.0 / G) | (g.random(G ** 3) < rand_frac)
        grid[c, idx] = np.where(occ, 20.0, 0.0)
    return torch.from_numpy(grid)


def packbits_cpu(grid: torch.Tensor, thr: float) -> torch.Tensor:
    b = (grid.reshape(-1, 8) > thr).to(torch.uint8)
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8)
    return (b * w).sum(1).to(torch.uint8)


class SyntheticScene:
    """Everything the training step needs, on the host."""

    def __init__(self, W=800, H=800, n_images=100, scale=0.5, grid_size=128, seed=0):
        self.W, self.H, self.scale, self.G = W, H, scale, grid_size
        self.K = intrinsics(W, H)
        self.directions = get_ray_directions(H, W, self.K)
        self.poses = make_poses(n_images, seed=seed)
        self.cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)  # models/networks.py:27
        self.density_grid = shell_density_grid(grid_size, self.cascades, scale)
        self.bitfield = packbits_cpu(self.density_grid, 0.5)
        g = np.random.default_rng(seed + 7)
        # synthetic ground-truth colour per image/pixel is generated lazily
        self._rgb_seed = int(g.integers(1 << 30))

    def sample_batch(self, n_rays: int, gen: torch.Generator):
        """datasets/base.py:25-31: uniform image and pixel indices."""
        img = torch.randint(0, self.poses.shape[0], (n_rays,), generator=gen)
        pix = torch.randint(0, self.W * self.H, (n_rays,), generator=gen)
        return img, pix

    def target_rgb(self, img: torch.Tensor, pix: torch.Tensor) -> torch.Tensor:
        """Deterministic smooth pseudo-colour per (image, pixel)."""
        u = (pix % self.W).float() / self.W
        v = (pix // self.W).float() / self.H
        t = img.float() / max(1, self.poses.shape[0])
        return torch.stack([0.5 + 0.5 * torch.sin(6 * u + t), 0.5 + 0.5 * torch.cos(5 * v - t),
                            0.5 + 0.5 * torch.sin(3 * (u + v))], -1)

    def rays(self, img: torch.Tensor, pix: torch.Tensor):
        """datasets/ray_utils.py:45-70 (host reference for tests)."""
        P = self.poses[img]
        d = self.directions[pix]
        rays_d = torch.einsum("nc,nac->na", d, P[:, :, :3])
        rays_o = P[:, :, 3].clone()
        return rays_o, rays_d


class AnalyticScene(SyntheticScene):
    """SyntheticScene whose ground truth is an analytic object, so training
    has a consistent target and the occupancy grid converges onto a surface
    the way it does on Lego: an opaque sphere (radius 0.3) plus a box, with
    procedural colours, on a white background (Blender scenes are composited
    on white, datasets/nerf.py read_image)."""

    SPHERE_R = 0.3
    BOX_MIN = torch.tensor([-0.42, -0.12, -0.40])
    BOX_MAX = torch.tensor([-0.18, 0.18, 0.05])

    def gt_rgb_rays(self, rays_o: torch.Tensor, rays_d: torch.Tensor) -> torch.Tensor:
        o, d = rays_o.double(), rays_d.double()
        dn = d / d.norm(dim=1, keepdim=True)
        inf = torch.full((o.shape[0],), float("inf"), dtype=torch.float64, device=o.device)
        # sphere
        b = (o * dn).sum(1)
        c = (o * o).sum(1) - self.SPHERE_R ** 2
        disc = b * b - c
        ts = torch.where(disc > 0, -b - torch.sqrt(disc.clamp(min=0)), inf)
        ts = torch.where(ts > 0, ts, inf)
        # box (slabs)
        bmin, bmax = self.BOX_MIN.double().to(o.device), self.BOX_MAX.double().to(o.device)
        inv = 1.0 / dn
        t0, t1 = (bmin - o) * inv, (bmax - o) * inv
        tn = torch.minimum(t0, t1).max(1).values
        tf = torch.maximum(t0, t1).min(1).values
        tb = torch.where((tn < tf) & (tn > 0), tn, inf)
        hit_s = ts <= tb
        t = torch.minimum(ts, tb)
        p = o + t[:, None] * dn
        n_s = p / self.SPHERE_R
        col_s = 0.5 + 0.45 * torch.stack([torch.sin(7 * p[:, 0]) * n_s[:, 2], torch.cos(9 * p[:, 1]),
                                          torch.sin(5 * (p[:, 2] + p[:, 0]))], 1)
        checker = ((torch.floor(p[:, 0] * 20) + torch.floor(p[:, 1] * 20) + torch.floor(p[:, 2] * 20)) % 2)
        col_b = torch.stack([0.8 - 0.5 * checker, 0.3 + 0.4 * checker, 0.2 + 0.1 * checker], 1)
        col = torch.where(hit_s[:, None], col_s, col_b)
        hit = torch.isfinite(t)
        col = torch.where(hit[:, None], col, torch.ones_like(col))
        return col.clamp(0, 1).float()

    def gt_images(self, device="cpu", chunk=1 << 20) -> torch.Tensor:
        """(n_images, H*W, 3) uint8 ground truth for every view."""
        n, HW = self.poses.shape[0], self.H * self.W
        out = torch.empty(n, HW, 3, dtype=torch.uint8, device=device)
        dirs = self.directions.to(device)
        for i in range(n):
            P = self.poses[i].to(device)
            for s in range(0, HW, chunk):
                d = dirs[s:s + chunk] @ P[:, :3].t()
                o = P[:, 3].expand_as(d)
                out[i, s:s + chunk] = (self.gt_rgb_rays(o, d) * 255 + 0.5).to(torch.uint8)
        return out


def write_nsvf_scene(root, res=100, n_train=24, n_test=2, seed=7):
    """The analytic scene as an NSVF-format dataset on disk (the Synthetic-
    NeRF layout datasets/nsvf.py reads): rgb/{0,2}_XXXX.png (split 0 = train,
    2 = test), pose/*.txt (4x4 c2w), intrinsics.txt, bbox.txt -- so the whole
    ingest -> train -> test-PSNR flow of train.py runs on it.  The reader
    assumes 800-px Synthetic-NeRF frames scaled by its `downsample`: read the
    scene with downsample = res / 800."""
    import os

    from datasets.png import write_png
    os.makedirs(os.path.join(root, "rgb"), exist_ok=True)
    os.makedirs(os.path.join(root, "pose"), exist_ok=True)
    fx = 0.5 * 800 / np.tan(0.5 * 0.6911112070083618)  # of the 800-px frame
    with open(os.path.join(root, "intrinsics.txt"), "w") as f:
        f.write(f"{fx} 0. 0. 0.\n")
    b = 0.5 / 1.05  # NSVF scale = 1.05 * half side = 0.5, shift 0: poses unchanged
    with open(os.path.join(root, "bbox.txt"), "w") as f:
        f.write(f"{-b} {-b} {-b} {b} {b} {b} 0.01\n")
    sc = AnalyticScene(W=res, H=res, n_images=n_train + n_test, seed=seed)
    for i in range(n_train + n_test):
        split = "0" if i < n_train else "2"
        P = sc.poses[i]
        d = sc.directions @ P[:, :3].t()
        o = P[:, 3].expand_as(d)
        rgb = sc.gt_rgb_rays(o.contiguous(), d.contiguous()).reshape(res, res, 3)
        write_png(os.path.join(root, "rgb", f"{split}_{i:04d}.png"),
                  (rgb.clamp(0, 1) * 255 + 0.5).to(torch.uint8).numpy())
        c2w = np.eye(4)
        c2w[:3] = P.numpy()
        np.savetxt(os.path.join(root, "pose", f"{split}_{i:04d}.txt"), c2w)
    return root
