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

    def forward(self, results, target, **kwargs):
        d = {}
        d['rgb'] = self.rgb_loss(results['rgb'], target['rgb']) ** 2
        o = results['opacity'] + 1e-10
        d['opacity'] = self.lambda_opacity * (-o * torch.log(o))
        d['depth'] = -self.lambda_depth * torch.log((results['depth'] / self.grid_scale + 1e-10).clip(max=1.0))
        if self.lambda_distortion > 0:
            d['distortion'] = self.lambda_distortion * DistortionLoss.apply(results['ws'], results['deltas'],
                                                                            results['ts'], results['rays_a'])
        return d
