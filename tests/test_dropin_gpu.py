"""The drop-in surface as the reference's training loop uses it: apex
FusedAdam's replacement (optimizers.FusedAdam, train.py:146-152) and the
whole loop (bench.DropinLoop: render_rays + NeRFLoss + backward + FusedAdam on
models.networks.NGP, train.py:84-200)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_fused_adam_matches_torch_adam():
    """optimizers.FusedAdam (one ngp_adam_step launch per tensor) against
    torch.optim.Adam with the reference's settings (eps 1e-15, no weight
    decay) over 5 steps with changing gradients and a learning-rate change:
    parameters within 2 fp32 ulps-ish (1e-6 relative), and the fp16 shadow an
    NGP parameter carries equals the new master rounded to fp16 after every
    step (no stale shadow for the next forward)."""
    from models.networks import NGP
    from optimizers import FusedAdam
    m = NGP(0.5).to(DEV)
    ref = m.params.detach().clone().requires_grad_(True)
    opt = FusedAdam([m.params], 1e-2, eps=1e-15)
    opt_ref = torch.optim.Adam([ref], 1e-2, eps=1e-15)
    g = torch.Generator(device=DEV).manual_seed(3)
    for it in range(5):
        grad = torch.randn(m.params.shape, device=DEV, generator=g) * (10.0 ** -it)
        m.params.grad = grad.clone()
        ref.grad = grad.clone()
        if it == 3:
            for grp in (opt.param_groups[0], opt_ref.param_groups[0]):
                grp["lr"] = 3e-3
        opt.step()
        opt_ref.step()
        torch.testing.assert_close(m.params.detach(), ref.detach(), rtol=1e-6, atol=1e-7)
        assert torch.equal(m._shadow.get(), m.params.detach().half())
        assert m._shadow.half.data_ptr() == m._shadow.get().data_ptr()  # the launch wrote the shadow in place
    with pytest.raises(RuntimeError):  # 6 elements: not a multiple of 4 (no CPU / scalar fallback)
        _step_on(FusedAdam, torch.zeros(6, device=DEV, requires_grad=True))
    with pytest.raises(RuntimeError):  # a CPU tensor
        _step_on(FusedAdam, torch.zeros(8, requires_grad=True))


def _step_on(cls, p):
    p.grad = torch.ones_like(p)
    cls([p], 1e-2).step()


def test_dropin_loop_trains():
    """bench.DropinLoop -- the reference's loop on the drop-in surface -- from
    a briefly trained NGPTrainer state: 40 steps with occupancy updates every
    16, finite losses that go down, the NGP's shadow current after each Adam
    step, and the model's parameters moved by the optimizer."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import synthetic as S
    from trainer import NGPTrainer
    sc = S.AnalyticScene(W=100, H=100, n_images=10)
    gt = sc.gt_images(device=DEV)
    dirs, poses = sc.directions.to(DEV), sc.poses.to(DEV)
    tr = NGPTrainer(scale=0.5, batch_size=2048, device=DEV, seed=3)
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    for _ in range(300):
        tr.train_step(gt, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    loop = bench.DropinLoop(tr, gt, dirs, poses, 2048)
    p0 = loop.model.params.detach().clone()
    losses = []
    for _ in range(40):
        loss, res = loop.step()
        losses.append(float(loss))
        assert torch.equal(loop.model._shadow.get(), loop.model.params.detach().half())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert sum(losses[-10:]) < 1.5 * sum(losses[:10])
    assert float((loop.model.params.detach() - p0).abs().max()) > 0
    assert int(res["rm_samples"]) > 0 and int(res["vr_samples"]) > 0


@pytest.mark.parametrize("loss_set", ["raw", "log", "tanh"])
def test_fused_nerf_loss_matches_the_reference_expressions(loss_set):
    """losses.NeRFLoss on CUDA tensors (one ngp_nerf_loss_fw / _bw launch) against
    the reference's torch expressions (losses.py:63-76, run here on the same
    tensors): every term within fp32 rounding of the op-by-op values, and the
    gradients w.r.t. rgb, opacity and depth through autograd the same, with
    the depth clip's zero gradient where it clips."""
    from losses import NeRFLoss
    g = torch.Generator().manual_seed(3)
    n = 5000
    rgb = torch.rand(n, 3, generator=g).to(DEV).requires_grad_(True)
    gt = torch.rand(n, 3, generator=g).to(DEV)
    op = (torch.rand(n, generator=g) * 0.999 + 1e-4).to(DEV).requires_grad_(True)
    dep = (torch.rand(n, generator=g) * 1.2).to(DEV).requires_grad_(True)  # some past the clip at depth / scale = 1
    L = NeRFLoss(30, loss_set, 1.0, 1e-2, lambda_opacity=1e-3, lambda_distortion=0.0)
    d = L({"rgb": rgb, "opacity": op, "depth": dep}, {"rgb": gt})
    loss = sum(v.mean() for v in d.values())
    gr = torch.autograd.grad(loss, (rgb, op, dep))
    rr, oo, dd = rgb.detach().clone().requires_grad_(True), op.detach().clone().requires_grad_(True), \
        dep.detach().clone().requires_grad_(True)
    ref = {"rgb": L.rgb_loss(rr, gt) ** 2}
    o = oo + 1e-10
    ref["opacity"] = L.lambda_opacity * (-o * torch.log(o))
    ref["depth"] = -L.lambda_depth * torch.log((dd / L.grid_scale + 1e-10).clip(max=1.0))
    lref = sum(v.mean() for v in ref.values())
    gref = torch.autograd.grad(lref, (rr, oo, dd))
    for k in ("rgb", "opacity", "depth"):
        torch.testing.assert_close(d[k], ref[k], rtol=2e-6, atol=1e-9)
    for a, b in zip(gr, gref):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=1e-12)
    assert int((gr[2] == 0).sum()) == int((dep.detach() / 1.0 + 1e-10 > 1.0).sum())
