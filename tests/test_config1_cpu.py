"""BASELINE.json config 1 -- "Lego 64x64, 256 rays/batch, L=4 hash levels,
32-wide MLP on the pure-PyTorch CPU path (plumbing, no GPU)" -- on the
oracle (the CPU restatement; the reference hard-codes L=16 / 64-wide MLPs,
networks.py:33,54,75, and has no CPU path at all, SURVEY.md §0, so this
configuration exists only here): the level table tcnn's sizing gives for
L=4, then training steps of the reference's step math (march, field with
fp16 storage points, VolumeRenderer fw/bw, raw NeRFLoss, autograd, Adam)
that drive the loss down.  The padded MLP input (8 -> 16) follows tcnn's
padding with ones: parity unpinned (tcnn is not in the container)."""
import torch

import oracle as O
import synthetic as S


def test_config1_level_table():
    spec = O.HashGridSpec(n_levels=4, log2_T=19, base_resolution=16, scale=0.5)
    assert abs(spec.b - 4.0) < 1e-6  # b = exp(ln(2048 * 0.5 / 16) / 3)
    assert spec.res.tolist() == [16, 64, 256, 1024]
    assert spec.sizes.tolist() == [4096, 262144, 1 << 19, 1 << 19]  # two dense levels, two hashed
    f = O.OracleNGPField(scale=0.5, n_levels=4, width=32)
    assert f.dens_dims == (16, 32, 16) and f.color_dims == (32, 32, 32, 16)
    assert f.n_dens == 16 * 32 + 32 * 16 and f.rgb_params.numel() == 32 * 32 + 32 * 32 + 16 * 32


def test_config1_trains_on_the_cpu():
    sc = S.AnalyticScene(W=64, H=64, n_images=20, scale=0.5)
    torch.manual_seed(0)
    ot = O.OracleTrainer(None, 0.5, sc.bitfield, 1, n_levels=4, width=32, table_init=1e-4)
    gen = torch.Generator().manual_seed(1)
    c = torch.zeros(1, 3)
    h = torch.ones(1, 3) * 0.5
    losses, samples = [], []
    for _ in range(160):
        img, pix = sc.sample_batch(256, gen)
        o, d = sc.rays(img, pix)
        _, ht, _ = O.ray_aabb_intersect(o, d, c, h, 1)
        ht = ht[:, 0].contiguous()
        ht[(ht[:, 0] >= 0) & (ht[:, 0] < 0.01), 0] = 0.01  # models/rendering.py:29-31
        loss, n = ot.step(o.contiguous(), d.contiguous(), ht, sc.gt_rgb_rays(o, d), torch.rand(256, generator=gen),
                          torch.ones(3))
        losses.append(loss)
        samples.append(n)
    assert all(torch.isfinite(torch.tensor(losses)))
    assert min(samples) > 0
    assert sum(losses[-20:]) / 20 < 0.9 * sum(losses[:20]) / 20, losses
