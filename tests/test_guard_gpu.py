"""Capacity guards: a device-side count past the capacity a
kernel was given is clamped AND counted (ngp_guard_hits), never silently
truncated.  These tests overflow a capacity on purpose, see the count, and
reset it so the conftest check (guard hits == 0 after every GPU test) holds
for every other test."""
import pytest
import torch

import hashgrid as HG
import vren

pytestmark = pytest.mark.gpu


def _inputs(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    xyz = ((torch.rand(n, 3, generator=g) - 0.5) * 0.9).cuda()
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g), dim=1).cuda()
    return xyz, d


def test_count_past_capacity_is_counted_not_silent():
    L = vren.lib()
    assert L.ngp_guard_reset() == 0 and L.ngp_guard_hits() == 0
    grid = HG.HashGrid(0.5)
    p16 = HG.init_params(grid, seed=1, table_init=1.0).half()
    n = 3000
    xyz, d = _inputs(n)
    try:
        # within capacity: no hit, same outputs as the host count
        sig0, rgb0, _, _ = HG.field_forward(xyz, d, grid, p16, save_enc=False)
        sig1, rgb1, _, _ = HG.field_forward(xyz, d, grid, p16, save_enc=False,
                                            n_dev=torch.tensor([n], dtype=torch.int64, device="cuda"))
        torch.cuda.synchronize()
        assert L.ngp_guard_hits() == 0
        assert torch.equal(sig0, sig1) and torch.equal(rgb0, rgb1)
        # a device count 5000 past the capacity: clamped (outputs = the n in range) and counted
        sig2, rgb2, _, _ = HG.field_forward(xyz, d, grid, p16, save_enc=False,
                                            n_dev=torch.tensor([n + 5000], dtype=torch.int64, device="cuda"))
        torch.cuda.synchronize()
        h1 = int(L.ngp_guard_hits())
        assert h1 >= 1, "an overflowing count must be counted"
        assert torch.equal(sig0, sig2) and torch.equal(rgb0, rgb2)
        # the density forward's launch counts too
        HG.density_forward(xyz, grid, p16, n_dev=torch.tensor([2 * n], dtype=torch.int64, device="cuda"))
        torch.cuda.synchronize()
        assert int(L.ngp_guard_hits()) > h1
    finally:
        assert L.ngp_guard_reset() == 0
    assert L.ngp_guard_hits() == 0


def test_trainer_overflow_of_the_round2_list_is_counted():
    """The row forward's round-2 list bounded by its capacity (field.hip,
    ngp_field_forward_first_pre): a list smaller than the rows' remaining
    samples drops the tail -- and says so."""
    import synthetic as S
    from trainer import NGPTrainer
    L = vren.lib()
    assert L.ngp_guard_reset() == 0
    sc = S.AnalyticScene(W=64, H=64, n_images=6)
    dev = torch.device("cuda", 0)
    tr = NGPTrainer(scale=0.5, batch_size=512, device=dev, seed=2, warmup_steps=0, update_interval=10 ** 6)
    tr.density_bitfield.copy_(sc.bitfield.to(dev))
    tr.global_step = 1
    gt, dirs, poses = sc.gt_images(device="cuda"), sc.directions.cuda(), sc.poses.cuda()
    try:
        tr.train_step(gt, dirs, poses)
        torch.cuda.synchronize()
        assert L.ngp_guard_hits() == 0  # the real capacity holds every sample
        # shrink the capacity the round-1 launch is told about to 16 list entries
        m = tr.msets[tr.cur]  # the batch this step ran (its rows, rays_a and samples intact)
        HGm = HG
        R = tr.batch_size
        cap_small = 16
        vren._ok(HGm._lib().ngp_field_forward_first_pre(
            HGm._ptr(m["xyzs"]), HGm._ptr(m["dirs"]), HGm._ptr(m["deltas"]), HGm._ptr(m["rays_a"]),
            HGm._ptr(m["rows_ne"]), HGm._ptr(m["n_rows_ne"]), R, cap_small, HGm.c_float(1e-4),
            HGm.ctypes.byref(tr.grid.desc), HGm._ptr(tr.params16[HGm.MLP_PARAMS:]), HGm._ptr(tr.params16),
            None, HGm._ptr(tr.sigmas), HGm._ptr(tr.rgbs), None, HGm._ptr(tr.eval_idx),
            HGm._ptr(torch.zeros(1, dtype=torch.int64, device=dev)), HGm._ptr(tr.eval_stats), 0,
            vren._stream()), "field_forward_first_pre")
        torch.cuda.synchronize()
        assert int(m["n_rows_ne"]) > 0
        assert L.ngp_guard_hits() >= 1
    finally:
        assert L.ngp_guard_reset() == 0
