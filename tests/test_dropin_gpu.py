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
