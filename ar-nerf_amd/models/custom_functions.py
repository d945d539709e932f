"""Autograd surface of the reference (models/custom_functions.py:8-173),
same class names, `apply` signatures and outputs, over the MI355X `vren`
(libngp_amd.so).  No torch_scatter / einops dependency."""
import torch

import vren

try:  # torch >= 2.4
    from torch.amp import custom_bwd as _cbwd, custom_fwd as _cfwd

    def custom_fwd(cast_inputs=None):
        return _cfwd(device_type="cuda", cast_inputs=cast_inputs)

    custom_bwd = _cbwd(device_type="cuda")
except ImportError:  # pragma: no cover
    from torch.cuda.amp import custom_bwd, custom_fwd  # noqa: F401


class RayAABBIntersector(torch.autograd.Function):
    """custom_functions.py:8-29 -> (hits_cnt (N), hits_t (N,max_hits,2), hits_voxel_idx (N,max_hits))."""

    @staticmethod
    @custom_fwd(cast_inputs=torch.float32)
    def forward(ctx, rays_o, rays_d, center, half_size, max_hits):
        return tuple(vren.ray_aabb_intersect(rays_o, rays_d, center, half_size, max_hits))


class RaySphereIntersector(torch.autograd.Function):
    """custom_functions.py:32-52 -- never called by the reference; out of scope."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, center, radii, max_hits):
        return tuple(vren.ray_sphere_intersect(rays_o, rays_d, center, radii, max_hits))


def _segment_sum(values, rays_a, n_rays):
    """segment_csr(values, [starts..., end]) of custom_functions.py:107-110 with
    the ray-ordered layout: row r of rays_a IS ray r, so per-row sums are
    per-ray sums (the reference's atomic row order made this assumption
    silently)."""
    ray_of = torch.repeat_interleave(rays_a[:, 0], rays_a[:, 2], output_size=values.shape[0])
    out = torch.zeros(n_rays, *values.shape[1:], device=values.device, dtype=values.dtype)
    return out.index_add_(0, ray_of, values)


# Test hook: when set, called as NOISE_HOOK(rays_o) -> (N,) f32 noise instead of
# torch.rand_like (parity tests replay the reference run's noise).
NOISE_HOOK = None


class RayMarcher(torch.autograd.Function):
    """custom_functions.py:55-112 -> (rays_a, xyzs, dirs, deltas, ts, total_samples)."""

    @staticmethod
    @custom_fwd(cast_inputs=torch.float32)
    def forward(ctx, rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, grid_size,
                max_samples):
        noise = torch.rand_like(rays_o[:, 0]) if NOISE_HOOK is None else NOISE_HOOK(rays_o)  # :83
        rays_a, xyzs, dirs, deltas, ts, counter = vren.raymarching_train(
            rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, noise, grid_size, max_samples)
        total_samples = counter[0]
        ctx.save_for_backward(rays_a, ts)
        ctx.n_rays = rays_o.shape[0]
        return rays_a, xyzs, dirs, deltas, ts, total_samples

    @staticmethod
    @custom_bwd
    def backward(ctx, dL_drays_a, dL_dxyzs, dL_ddirs, dL_ddeltas, dL_dts, dL_dtotal_samples):
        rays_a, ts = ctx.saved_tensors
        dL_drays_o = _segment_sum(dL_dxyzs, rays_a, ctx.n_rays)
        dL_drays_d = _segment_sum(dL_dxyzs * ts[:, None] + dL_ddirs, rays_a, ctx.n_rays)
        return dL_drays_o, dL_drays_d, None, None, None, None, None, None, None


class VolumeRenderer(torch.autograd.Function):
    """custom_functions.py:115-159 -> (total_samples, opacity, depth, rgb, ws)."""

    @staticmethod
    @custom_fwd(cast_inputs=torch.float32)
    def forward(ctx, sigmas, rgbs, deltas, ts, rays_a, T_threshold):
        total_samples, opacity, depth, rgb, ws = vren.composite_train_fw(sigmas, rgbs, deltas, ts, rays_a,
                                                                         T_threshold)
        ctx.save_for_backward(sigmas, rgbs, deltas, ts, rays_a, opacity, depth, rgb, ws)
        ctx.T_threshold = T_threshold
        return total_samples.sum(), opacity, depth, rgb, ws

    @staticmethod
    @custom_bwd
    def backward(ctx, dL_dtotal_samples, dL_dopacity, dL_ddepth, dL_drgb, dL_dws):
        sigmas, rgbs, deltas, ts, rays_a, opacity, depth, rgb, ws = ctx.saved_tensors
        dL_dsigmas, dL_drgbs = vren.composite_train_bw(dL_dopacity.contiguous(), dL_ddepth.contiguous(),
                                                       dL_drgb.contiguous(), dL_dws.contiguous(), sigmas, rgbs, ws,
                                                       deltas, ts, rays_a, opacity, depth, rgb, ctx.T_threshold)
        return dL_dsigmas, dL_drgbs, None, None, None, None


class TruncExp(torch.autograd.Function):
    """custom_functions.py:162-173."""

    @staticmethod
    @custom_fwd(cast_inputs=torch.float32)
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    @custom_bwd
    def backward(ctx, dL_dout):
        x = ctx.saved_tensors[0]
        return dL_dout * torch.exp(x.clamp(-15, 15))
