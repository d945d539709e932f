"""Drop-in for the reference's losses.py (NeRFLoss, DistortionLoss)."""
import torch
from torch import nn

import vren


class DistortionLoss(torch.autograd.Function):
    """losses.py:7-38: Mip-NeRF 360 distortion loss in the DVGO-v2 form, per
    ray (off by default, opt.py:25), on the gfx950 kernels."""

    @staticmethod
    def forward(ctx, ws, deltas, ts, rays_a):
        loss, ws_inclusive_scan, wts_inclusive_scan = vren.distortion_loss_fw(ws, deltas, ts, rays_a)
        ctx.save_for_backward(ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a)
        return loss

    @staticmethod
    def backward(ctx, dL_dloss):
        ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a = ctx.saved_tensors
        dL_dws = vren.distortion_loss_bw(dL_dloss.contiguous(), ws_inclusive_scan, wts_inclusive_scan, ws, deltas,
                                         ts, rays_a)
        return dL_dws, None, None, None


_LOSS_TYPE = {'raw': 0, 'log': 2, 'tanh': 3}


class _NeRFLossFn(torch.autograd.Function):
    """NeRFLoss's per-ray rgb / opacity / depth terms (losses.py:63-76) and their
    backward, one launch each way (ngp_nerf_loss_fw / _bw) instead of ~15
    elementwise ops and their autograd nodes; the same expressions op for op."""

    @staticmethod
    def forward(ctx, rgb, gt, opacity, depth, loss_type, lam_op, lam_depth, grid_scale):
        n = rgb.shape[0]
        l_rgb, l_op, l_dep = torch.empty_like(rgb), torch.empty_like(opacity), torch.empty_like(depth)
        vren._ok(vren.lib().ngp_nerf_loss_fw(vren._check("rgb", rgb, torch.float32), vren._check("rgb_gt", gt, torch.float32),
                                             vren._check("opacity", opacity, torch.float32),
                                             vren._check("depth", depth, torch.float32), n, loss_type, lam_op, lam_depth,
                                             grid_scale, vren._check("l", l_rgb), vren._check("l", l_op),
                                             vren._check("l", l_dep), vren._stream()), "nerf_loss_fw")
        ctx.save_for_backward(rgb, gt, opacity, depth)
        ctx.args = (loss_type, lam_op, lam_depth, grid_scale)
        return l_rgb, l_op, l_dep

    @staticmethod
    def backward(ctx, g_rgb, g_op, g_dep):
        rgb, gt, opacity, depth = ctx.saved_tensors
        n = rgb.shape[0]
        d_rgb, d_op, d_dep = torch.empty_like(rgb), torch.empty_like(opacity), torch.empty_like(depth)
        c = lambda t: vren._check("grad", t.contiguous(), torch.float32) if t is not None else None  # noqa: E731
        vren._ok(vren.lib().ngp_nerf_loss_bw(vren._check("rgb", rgb), vren._check("rgb_gt", gt),
                                             vren._check("opacity", opacity), vren._check("depth", depth), n,
                                             *ctx.args, c(g_rgb), c(g_op), c(g_dep), vren._check("d", d_rgb),
                                             vren._check("d", d_op), vren._check("d", d_dep), vren._stream()),
                 "nerf_loss_bw")
        return d_rgb, None, d_op, d_dep, None, None, None, None


class NeRFLoss(nn.Module):
    """losses.py:41-82."""

    def __init__(self, epoch, loss_set, grid_scale, lambda_depth, lambda_opacity=1e-3, lambda_distortion=1e-3):
        super().__init__()
        self.num_epoch = epoch
        self.grid_scale = grid_scale
        self.lambda_opacity = lambda_opacity
        self.lambda_depth = lambda_depth
        self.lambda_distortion = lambda_distortion
        losses = {
            'raw': lambda x_est, x_gt: (x_est - x_gt) / (x_est.detach() + 1e-3),
            'log': lambda x_est, x_gt: torch.log((0.2935 + x_est) / (0.2935 + x_gt)) * 0.7607,
            'tanh': lambda x_est, x_gt: torch.tanh(x_est) - torch.tanh(x_gt),
        }
        if loss_set not in losses:
            raise ValueError(f"Unknown loss function {loss_set!r}")
        self.rgb_loss = losses[loss_set]
        self.loss_type = _LOSS_TYPE[loss_set]

    def forward(self, results, target, **kwargs):
        d = {}
        rgb, gt, op, dep = results['rgb'], target['rgb'], results['opacity'], results['depth']
        if all(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
               for t in (rgb, gt, op, dep)) and rgb.dim() == 2 and rgb.shape[1] == 3:
            d['rgb'], d['opacity'], d['depth'] = _NeRFLossFn.apply(rgb, gt, op, dep, self.loss_type,
                                                                    float(self.lambda_opacity),
                                                                    float(self.lambda_depth), float(self.grid_scale))
        else:  # (the reference's torch expressions, e.g. for CPU tensors)
            d['rgb'] = self.rgb_loss(rgb, gt) ** 2
            o = op + 1e-10
            d['opacity'] = self.lambda_opacity * (-o * torch.log(o))
            d['depth'] = -self.lambda_depth * torch.log((dep / self.grid_scale + 1e-10).clip(max=1.0))
        if self.lambda_distortion > 0:
            d['distortion'] = self.lambda_distortion * DistortionLoss.apply(results['ws'], results['deltas'],
                                                                            results['ts'], results['rays_a'])
        return d
