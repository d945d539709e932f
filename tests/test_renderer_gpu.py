"""Graph-captured test-time renderer (renderer.TestRenderer) vs the host loop
of models/rendering.py:162-253 (our render(test_time=True), itself pinned to
the reference glue's golden fixture in test_golden_gpu.py): bit-exact per
ray, and within the golden tolerance of the fixture directly."""
import pytest
import torch

import renderer as R
import synthetic as S
import vren
from fixture_model import load
from models.networks import NGP
from models.rendering import NEAR_DISTANCE, render
from test_golden_gpu import _product_model

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _hits(model, o, d):
    _, ht, _ = vren.ray_aabb_intersect(o, d, model.center, model.half_size, 1)
    ht = ht[:, 0].contiguous()
    ht[(ht[:, 0] >= 0) & (ht[:, 0] < NEAR_DISTANCE), 0] = NEAR_DISTANCE
    return ht


def _host_loop(model, o, d, **kw):
    with torch.no_grad():
        return render(model, o, d, test_time=True, device_loop=False, **kw)


def _assert_same(res, ref):
    for k in ("rgb", "opacity", "depth"):
        assert torch.equal(res[k], ref[k]), k
    assert int(res["total_samples"]) == int(ref["total_samples"])


@pytest.mark.parametrize("graphs,K", [(True, 16), (True, 2), (False, 4)])
def test_renderer_matches_golden_and_host_loop(graphs, K):
    fx = load("lego_test")
    model = _product_model(fx)
    o, d = torch.from_numpy(fx["rays_o"]).to(DEV), torch.from_numpy(fx["rays_d"]).to(DEV)
    ref = _host_loop(model, o, d)
    rr = R.for_model(model, o.shape[0], iters_per_graph=K, use_graphs=graphs)
    res = rr.render(o, d, _hits(model, o, d))
    _assert_same(res, ref)
    for k in ("rgb", "opacity", "depth"):
        torch.testing.assert_close(res[k].cpu(), torch.from_numpy(fx[k]), atol=2e-3, rtol=0)
    # a second frame through the same captured graphs gives the same image
    res2 = {k: v.clone() for k, v in rr.render(o, d, _hits(model, o, d)).items()}
    _assert_same(res2, ref)


def _scene_model(scale, occ_frac, seed):
    m = NGP(scale)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        m.params.uniform_(-1, 1, generator=g)
        bits = (torch.rand(m.density_bitfield.numel() * 8, generator=g) < occ_frac).to(torch.uint8)
        m.density_bitfield.copy_((bits.view(-1, 8) << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8))
    return m.to(DEV)


@pytest.mark.parametrize("scale,esf,occ", [(0.5, 0.0, 0.02), (16.0, 1 / 256, 0.01)])
def test_renderer_full_frame_bit_exact(scale, esf, occ):
    """A 160x160 frame: many iterations, N_samples growing as rays die;
    cascaded grid + exp step (esf > 0: min_samples 4, the calc_dt `cascades`
    quirk) in the second case."""
    model = _scene_model(scale, occ, seed=5)
    sc = S.AnalyticScene(W=160, H=160, n_images=2)
    n = 160 * 160
    pix = torch.arange(n)
    o, d = sc.rays(torch.zeros(n, dtype=torch.int64), pix)
    o, d = (o * (2 * scale)).to(DEV).contiguous(), d.to(DEV).contiguous()
    ref = _host_loop(model, o, d, exp_step_factor=esf)
    rr = R.for_model(model, n, exp_step_factor=esf, iters_per_graph=8)
    res = rr.render(o, d, _hits(model, o, d))
    _assert_same(res, ref)
    assert rr.last_iterations > 2
    assert float(res["opacity"].max()) > 0


def test_render_api_uses_the_device_loop_bit_exact():
    """render(test_time=True) routes an NGP through the cached TestRenderer:
    same pixels as the host loop, and a parameter update reaches it."""
    fx = load("lego_test")
    model = _product_model(fx)
    o, d = torch.from_numpy(fx["rays_o"]).to(DEV), torch.from_numpy(fx["rays_d"]).to(DEV)
    with torch.no_grad():
        dev = render(model, o, d, test_time=True)
    _assert_same(dev, _host_loop(model, o, d))
    assert len(model._test_renderers) == 1
    with torch.no_grad():
        model.params.mul_(0.5)
        dev2 = render(model, o, d, test_time=True)
    _assert_same(dev2, _host_loop(model, o, d))
    assert not torch.equal(dev2["rgb"], dev["rgb"])


def test_render_pose_equals_rays_path():
    fx = load("lego_test")
    model = _product_model(fx)
    sc = S.AnalyticScene(W=96, H=96, n_images=3)
    n = 96 * 96
    rr = R.for_model(model, n)
    rr.set_camera(sc.directions.to(DEV), model.center, model.half_size)
    res = {k: v.clone() for k, v in rr.render_pose(sc.poses[1].to(DEV)).items()}
    o, d, _ = vren.raygen_aabb(sc.directions.to(DEV), sc.poses.to(DEV), torch.ones(n, dtype=torch.int64, device=DEV),
                               torch.arange(n, device=DEV), model.center, model.half_size, NEAR_DISTANCE)
    _assert_same(res, _host_loop(model, o, d))
