"""d sigma / d x through the hash grid (ngp_density_input_grad) and
render_surface_normal (models/rendering.py:300-313) vs the oracle's fp32
autograd restatement (oracle.density_input_grad; tcnn's input-gradient
arithmetic is unavailable: parity unpinned).  Tolerance: per point, relative
error of the gradient vector <= 2e-2 for >= 99% of points (fp16 storage
points; a ReLU whose pre-activation sits within rounding of 0 may flip), and
normal directions within cos >= 0.999 for >= 99%."""
import pytest
import torch

import hashgrid as HG
import oracle as O
from models.networks import NGP
from models.rendering import render_surface_normal

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(seed=3):
    m = NGP(0.5, seed=seed)
    with torch.no_grad():  # table values large enough that the field has structure
        g = torch.Generator().manual_seed(seed)
        m.params[HG.MLP_PARAMS:] = (torch.rand(m.params.numel() - HG.MLP_PARAMS, generator=g) * 2 - 1) * 0.5
    return m.to(DEV)


def test_density_input_grad_matches_oracle():
    m = _model()
    g = torch.Generator().manual_seed(1)
    x = (torch.rand(4096, 3, generator=g) * 2 - 1) * 0.45
    p16 = m._shadow.get()
    got = HG.density_input_grad(x.to(DEV).contiguous(), m.grid, p16).cpu()
    xyz_params, rgb_params = m.tcnn_params()
    ref = O.density_input_grad(xyz_params.cpu(), 3072, O.HashGridSpec(16, 19, 16, scale=0.5), x,
                               m.xyz_min.cpu(), m.xyz_max.cpu())
    rel = (got - ref).norm(dim=1) / ref.norm(dim=1).clamp_min(1e-12)
    assert float((rel <= 2e-2).float().mean()) >= 0.99, float(rel.median())
    # a weighted dL/dsigma scales the per-point gradient
    w = torch.rand(4096, generator=g)
    got_w = HG.density_input_grad(x.to(DEV).contiguous(), m.grid, p16, w.to(DEV)).cpu()
    want = got * w[:, None]  # (the weight enters before the sums: rounding differs)
    rel_w = (got_w - want).norm(dim=1) / want.norm(dim=1).clamp_min(1e-12)
    assert float((rel_w <= 1e-3).float().mean()) >= 0.99


def test_render_surface_normal_via_autograd():
    m = _model(5)
    g = torch.Generator().manual_seed(2)
    pts = ((torch.rand(32, 48, 3, generator=g) * 2 - 1) * 0.45).to(DEV)
    n = render_surface_normal(m, pts)
    assert n.shape == (32, 48, 3)
    xyz_params, _ = m.tcnn_params()
    ref = O.density_input_grad(xyz_params.cpu(), 3072, O.HashGridSpec(16, 19, 16, scale=0.5), pts.reshape(-1, 3).cpu(),
                               m.xyz_min.cpu(), m.xyz_max.cpu())
    ref = -ref / (ref.norm(dim=1, keepdim=True) + 1e-6)
    cos = (n.reshape(-1, 3).cpu() * ref).sum(1)
    assert float((cos >= 0.999).float().mean()) >= 0.99
    # params-gradient path unaffected: density under autograd w.r.t. the params
    sig = m.density(pts.reshape(-1, 3))
    sig.sum().backward()
    assert m.params.grad is not None and float(m.params.grad.abs().sum()) > 0
