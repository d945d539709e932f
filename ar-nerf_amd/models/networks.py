"""Drop-in for the reference's models/networks.py (NGP) on the MI355X
kernels.  tinycudann's three modules are replaced by one fused field
(hashgrid.py) over a single flat fp32 master parameter:
    params = [W1 | W2 | W3 | W4 | W5 | hash table]
(`xyz_encoder.params` of tcnn = [W1 | W2 | table]; `rgb_net.params` =
[W3 | W4 | W5]; see load_tcnn_params / tcnn_params for the mapping)."""
import numpy as np
import torch
from torch import nn

import hashgrid as HG
import vren
from .custom_functions import TruncExp  # noqa: F401  (reference export)
from .rendering import NEAR_DISTANCE


class _DensityFn(torch.autograd.Function):
    """NGP.density with gradients for the params (sigma and, optionally, h)."""

    @staticmethod
    def forward(ctx, xyzs, params, grid, shadow):
        p16 = shadow.get()
        n = xyzs.shape[0]
        dirs = torch.zeros(n, 3, device=xyzs.device)
        dirs[:, 2] = 1
        sig, _, enc, h = HG.field_forward(xyzs.contiguous(), dirs, grid, p16, save_enc=True, want_h=True)
        ctx.save_for_backward(xyzs, dirs, enc)
        ctx.grid, ctx.p16 = grid, p16
        ctx.mark_non_differentiable(h)
        return sig, h

    @staticmethod
    def backward(ctx, dsig, dh):
        xyzs, dirs, enc = ctx.saved_tensors
        n = xyzs.shape[0]
        dsig = torch.zeros(n, device=xyzs.device) if dsig is None else dsig.float().contiguous()
        grad = dx = None
        if ctx.needs_input_grad[1]:
            grad = torch.zeros(ctx.grid.n_params, device=xyzs.device)
            HG.field_backward(xyzs.contiguous(), dirs, ctx.grid, ctx.p16, enc, dsig,
                              torch.zeros(n, 3, device=xyzs.device), grad)
        if ctx.needs_input_grad[0]:  # d sigma / d x through the hash grid (render_surface_normal)
            dx = HG.density_input_grad(xyzs.float().contiguous(), ctx.grid, ctx.p16, dsig)
        return dx, grad, None, None


class NGP(nn.Module):
    """models/networks.py:12-281."""

    def __init__(self, scale, rgb_act='Sigmoid', use_raw_HDR=False, seed=4):
        super().__init__()
        if rgb_act != 'Sigmoid' or use_raw_HDR:
            raise NotImplementedError("HDR / exposure tonemapper branch (networks.py:80-93) is out of scope")
        self.rgb_act = rgb_act
        self.use_raw_HDR = use_raw_HDR
        self.scale = scale
        self.register_buffer('center', torch.zeros(1, 3))
        self.register_buffer('xyz_min', -torch.ones(1, 3) * scale)
        self.register_buffer('xyz_max', torch.ones(1, 3) * scale)
        self.register_buffer('half_size', (self.xyz_max - self.xyz_min) / 2)
        self.cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)
        self.grid_size = 128
        self.register_buffer('density_bitfield', torch.zeros(self.cascades * self.grid_size ** 3 // 8,
                                                             dtype=torch.uint8))
        L, F, log2_T, N_min = 16, 2, 19, 16
        b = np.exp(np.log(2048 * scale / N_min) / (L - 1))
        self.grid = HG.HashGrid(scale, L, log2_T, N_min, float(b))
        self.params = nn.Parameter(HG.init_params(self.grid, seed=seed, device="cpu"))
        self._shadow = HG.FP16Shadow(self.params)
        # optimizers.FusedAdam writes this shadow in its Adam launch (no re-cast before the next forward)
        self.params._ngp_shadow = self._shadow

    # -------------------------------------------------- tcnn param mapping
    def tcnn_params(self):
        """(xyz_encoder.params, rgb_net.params) in tcnn's flat layouts."""
        p = self.params.detach()
        m = HG.MLP_PARAMS
        return torch.cat([p[:3072], p[m:]]), p[3072:m].clone()

    @torch.no_grad()
    def load_tcnn_params(self, xyz_params, rgb_params):
        m = HG.MLP_PARAMS
        self.params[:3072] = xyz_params[:3072].to(self.params)
        self.params[m:] = xyz_params[3072:].to(self.params)
        self.params[3072:m] = rgb_params.to(self.params)

    # ---------------------------------------------------------- forward
    def density(self, x, return_feat=False):
        """networks.py:95-108 -> sigmas (N) [, h (N,16) fp16]"""
        x = x.float().contiguous()
        if torch.is_grad_enabled() and (self.params.requires_grad or x.requires_grad):
            sig, h = _DensityFn.apply(x, self.params, self.grid, self._shadow)
        else:
            sig, h = HG.density_forward(x, self.grid, self._shadow.get(), want_h=return_feat)
        return (sig, h) if return_feat else sig

    def forward(self, x, d, **kwargs):
        """networks.py:133-165 (Sigmoid rgb branch) -> sigmas (N) f32, rgbs (N,3) f32."""
        x, d = x.float().contiguous(), d.float().contiguous()
        if torch.is_grad_enabled() and self.params.requires_grad:
            return HG.field(x, d, self.params, self.grid, self._shadow)
        sig, rgb, _, _ = HG.field_forward(x, d, self.grid, self._shadow.get(), save_enc=False)
        return sig, rgb

    # ---------------------------------------------------- occupancy grid
    @torch.no_grad()
    def get_all_cells(self):
        """networks.py:167-179"""
        indices = vren.morton3D(self.grid_coords).long()
        return [(indices, self.grid_coords)] * self.cascades

    @torch.no_grad()
    def sample_uniform_and_occupied_cells(self, M, density_threshold):
        """networks.py:181-207"""
        cells = []
        for c in range(self.cascades):
            coords1 = torch.randint(self.grid_size, (M, 3), dtype=torch.int32, device=self.density_grid.device)
            indices1 = vren.morton3D(coords1).long()
            indices2 = torch.nonzero(self.density_grid[c] > density_threshold)[:, 0]
            if len(indices2) > 0:
                rand_idx = torch.randint(len(indices2), (M,), device=self.density_grid.device)
                indices2 = indices2[rand_idx]
            coords2 = vren.morton3D_invert(indices2.int().contiguous())
            cells += [(torch.cat([indices1, indices2]), torch.cat([coords1, coords2]))]
        return cells

    @torch.no_grad()
    def mark_invisible_cells(self, K, poses, img_wh, chunk=64 ** 3):
        """networks.py:209-250"""
        N_cams = poses.shape[0]
        self.count_grid = torch.zeros_like(self.density_grid)
        w2c_R = poses[:, :3, :3].transpose(1, 2)
        w2c_T = -w2c_R @ poses[:, :3, 3:]
        cells = self.get_all_cells()
        for c in range(self.cascades):
            indices, coords = cells[c]
            for i in range(0, len(indices), chunk):
                xyzs = coords[i:i + chunk] / (self.grid_size - 1) * 2 - 1
                s = min(2 ** (c - 1), self.scale)
                half_grid_size = s / self.grid_size
                xyzs_w = (xyzs * (s - half_grid_size)).T
                xyzs_c = w2c_R @ xyzs_w + w2c_T
                uvd = K @ xyzs_c
                uv = uvd[:, :2] / uvd[:, 2:]
                in_image = (uvd[:, 2] >= 0) & (uv[:, 0] >= 0) & (uv[:, 0] < img_wh[0]) & \
                           (uv[:, 1] >= 0) & (uv[:, 1] < img_wh[1])
                covered_by_cam = (uvd[:, 2] >= NEAR_DISTANCE) & in_image
                self.count_grid[c, indices[i:i + chunk]] = count = covered_by_cam.sum(0) / N_cams
                too_near_to_any_cam = ((uvd[:, 2] < NEAR_DISTANCE) & in_image).any(0)
                valid_mask = (count > 0) & (~too_near_to_any_cam)
                self.density_grid[c, indices[i:i + chunk]] = torch.where(valid_mask, 0., -1.)

    @torch.no_grad()
    def update_density_grid(self, density_threshold, warmup=False, decay=0.95, erode=False):
        """networks.py:252-281 (threshold kept on the device: no .item() sync)."""
        density_grid_tmp = torch.zeros_like(self.density_grid)
        if warmup:
            cells = self.get_all_cells()
        else:
            cells = self.sample_uniform_and_occupied_cells(self.grid_size ** 3 // 4, density_threshold)
        for c in range(self.cascades):
            indices, coords = cells[c]
            s = min(2 ** (c - 1), self.scale)
            half_grid_size = s / self.grid_size
            xyzs_w = (coords / (self.grid_size - 1) * 2 - 1) * (s - half_grid_size)
            xyzs_w += (torch.rand_like(xyzs_w) * 2 - 1) * half_grid_size
            # density_grid_tmp[c, indices] = density (last duplicate wins, deterministically)
            vren.density_scatter_last(density_grid_tmp[c], indices, self.density(xyzs_w))
        if erode:  # clamp(decay**(1/count_grid), 0.1, 0.95), evaluated once on the host (vren.erode_decay)
            key = (self.count_grid.data_ptr(), self.count_grid._version, float(decay))
            if getattr(self, "_erode_key", None) != key:
                self._erode_decay = vren.erode_decay(self.count_grid, decay).to(self.count_grid.device)
                self._erode_key = key
            decay = self._erode_decay
        self.density_grid = torch.where(self.density_grid < 0, self.density_grid,
                                        torch.maximum(self.density_grid * decay, density_grid_tmp))
        pos = self.density_grid > 0
        mean_density = self.density_grid[pos].sum() / pos.sum()
        vren.packbits(self.density_grid, torch.minimum(mean_density, torch.tensor(
            density_threshold, device=mean_density.device)).reshape(1).float(), self.density_bitfield)
