"""The CPU oracle against the known answers the reference itself states
(SURVEY.md §8c): comments of models/csrc/raymarching.cu, its Morton/packbits
bit conventions, and compositing edge cases.  No GPU."""
import math

import numpy as np
import pytest
import torch

import oracle as O


def test_morton_known_answers():
    c = torch.tensor([[1, 0, 0], [0, 1, 0], [0, 0, 1], [127, 127, 127], [3, 5, 6]], dtype=torch.int32)
    m = O.morton3D(c).tolist()
    assert m[:4] == [1, 2, 4, 2 ** 21 - 1]  # raymarching.cu:35-50, x in bit 0
    # (3,5,6): x=011 y=101 z=110 -> bits z2y2x2 z1y1x1 z0y0x0 = 110 101 011
    assert m[4] == 0b110101011


def test_morton_invert_is_identity_on_grid():
    ax = torch.arange(128, dtype=torch.int32)
    c = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)
    m = O.morton3D(c)
    assert torch.equal(O.morton3D_invert(m), c)
    assert torch.equal(m.sort().values, torch.arange(128 ** 3, dtype=torch.int32))  # a permutation


def test_packbits_lsb_first():
    g = torch.zeros(16)
    g[0] = 1; g[9] = 1; g[15] = 1  # raymarching.cu:136-138: bit i of byte n <- cell 8n+i
    bf = torch.zeros(2, dtype=torch.uint8)
    O.packbits(g, 0.5, bf)
    assert bf.tolist() == [0b00000001, 0b10000010]
    O.packbits(g, 1.0, bf)  # strict '>'
    assert bf.tolist() == [0, 0]


def test_calc_dt_and_mips_known_answers():
    L = O.lib()
    assert L.or_calc_dt(0.7, 0.0, 1024, 128, 0.5) == np.float32(1.73205080757 / 1024)
    # exponential stepping clamps to [sqrt3/1024, 2 sqrt3 scale/128] (raymarching.cu:11-13)
    assert L.or_calc_dt(200.0, 1 / 256, 1024, 128, 16.0) == np.float32(np.float32(1.73205080757) * 2 * 16 / 128)
    assert L.or_calc_dt(1.0, 1 / 256, 1024, 128, 16.0) == np.float32(1 / 256)
    # raymarching.cu:15-18: |xyz| in [0,.5) -> 0, [.5,1) -> 1, [1,2) -> 2
    for x, want in ((0.0, 0), (0.49, 0), (0.5, 1), (0.99, 1), (1.0, 2), (1.99, 2), (3.0, 3)):
        assert L.or_mip_from_pos(x, -0.1, 0.2, 6) == want
    assert L.or_mip_from_pos(7.0, 0, 0, 2) == 1  # clamped to cascades-1
    # raymarching.cu:25-28: dt in [0,1/G) -> 0, [1/G,2/G) -> 1, [2/G,4/G) -> 2
    for dt, want in ((0.5 / 128, 0), (1 / 128, 1), (1.9 / 128, 1), (2 / 128, 2), (3.9 / 128, 2)):
        assert L.or_mip_from_dt(dt, 128, 6) == want


def test_f16_rounding_matches_torch():
    g = torch.Generator().manual_seed(0)
    x = torch.cat([torch.randn(20000, generator=g) * s for s in (1e-7, 1e-5, 1e-2, 1, 100, 7e4)])
    ours = torch.tensor([O.lib().or_f32_to_f16(float(v)) for v in x[::37]], dtype=torch.int32)
    ref = x[::37].half().view(torch.int16).to(torch.int32) & 0xFFFF
    assert torch.equal(ours, ref)


def test_single_opaque_sample_terminates_before_count():
    # volumerendering.cu:40-41: break BEFORE samples++ -> total 0, opacity 1
    rays_a = torch.tensor([[0, 0, 3]])
    sig = torch.tensor([1e6, 1.0, 1.0]); rgb = torch.rand(3, 3)
    dl = torch.full((3,), 0.01); ts = torch.tensor([0.1, 0.2, 0.3])
    tot, op, dep, c, ws = O.composite_train_fw(sig, rgb, dl, ts, rays_a, 1e-4)
    assert tot.tolist() == [0] and op.item() == pytest.approx(1.0)
    assert ws[1:].abs().max() == 0
    torch.testing.assert_close(c[0], rgb[0])


def test_march_constant_step_and_monotone_t():
    o = torch.tensor([[-0.6, 0.01, 0.02]]); d = torch.tensor([[1.0, 0.0, 0.0]])
    ht = torch.tensor([[0.1, 1.1]])
    bf = torch.full((128 ** 3 // 8,), 255, dtype=torch.uint8)  # everything occupied
    rays_a, xyzs, dirs, deltas, ts, cnt = O.raymarching_train(o, d, ht, bf, 1, 0.5, 0.0, torch.zeros(1), 128, 1024)
    n = int(cnt[0])
    assert n == rays_a[0, 2] and abs(n - (1.1 - 0.1) / (1.73205080757 / 1024)) <= 1
    assert torch.all(deltas == np.float32(1.73205080757 / 1024))
    assert torch.all(ts[1:] > ts[:-1]) and ts[0] == 0.1
    torch.testing.assert_close(xyzs[:, 0], -0.6 + ts, atol=1e-6, rtol=0)
    # max_samples caps the count AND sets the minimum step sqrt(3)/max_samples
    _, x2, _, d2, _, c2 = O.raymarching_train(o, d, ht, bf, 1, 0.5, 0.0, torch.zeros(1), 128, 5)
    assert int(c2[0]) <= 5 and torch.all(d2 == np.float32(np.float32(1.73205080757) / 5))
    ht3 = torch.tensor([[0.1, 100.0]])
    _, _, _, _, _, c3 = O.raymarching_train(o, d, ht3, bf, 1, 0.5, 0.0, torch.zeros(1), 128, 5)
    assert int(c3[0]) == 5


def test_march_empty_grid_and_missing_rays():
    o = torch.tensor([[-0.6, 0.0, 0.0], [5.0, 5.0, 5.0]]); d = torch.tensor([[1.0, 0.0, 0.0], [1.0, 0, 0]])
    ht = torch.tensor([[0.1, 1.1], [-1.0, -1.0]])
    bf = torch.zeros(128 ** 3 // 8, dtype=torch.uint8)
    rays_a, xyzs, *_, cnt = O.raymarching_train(o, d, ht, bf, 1, 0.5, 0.0, torch.zeros(2), 128, 1024)
    assert int(cnt[0]) == 0 and rays_a[:, 2].tolist() == [0, 0] and xyzs.shape == (0, 3)


def test_hash_levels_and_param_count():
    spec = O.HashGridSpec(16, 19, 16, scale=0.5)
    # fp32 level scales like tcnn: level 5 -> res 65 (exact arithmetic would give 64)
    assert spec.res.tolist() == [16, 22, 28, 37, 49, 65, 85, 112, 148, 195, 257, 338, 446, 589, 777, 1025]
    assert spec.sizes.tolist()[:6] == [4096, 10648, 21952, 50656, 117656, 274632]
    assert all(s == 2 ** 19 for s in spec.sizes.tolist()[6:])
    assert spec.n_entries * 2 == 11_445_040
    spec16 = O.HashGridSpec(16, 19, 16, scale=16.0)
    assert spec16.res.tolist()[:4] == [16, 27, 45, 74] and spec16.n_entries == 6_811_592


def test_hash_corner_indices_dense_and_hashed():
    spec = O.HashGridSpec(16, 19, 16, scale=0.5)
    x = torch.tensor([[0.1, -0.2, 0.3]])
    idx, w = O.hash_corners(spec, x, -torch.ones(3) * 0.5, torch.ones(3) * 0.5)
    x01 = ((x + 0.5) / 1.0)[0]
    for l in (0, 8):
        s = float(spec.scales[l]); res = int(spec.res[l]); size = int(spec.sizes[l])
        p = np.array([np.float32(s) * np.float32(v) + np.float32(0.5) for v in x01.tolist()], np.float32)
        g = np.floor(p).astype(np.int64)
        f = p - g
        for c in range(8):
            q = [g[d] + ((c >> d) & 1) for d in range(3)]
            if res ** 3 <= size:
                e = (q[0] + q[1] * res + q[2] * res * res) % size
            else:
                e = ((q[0] * 1) ^ (q[1] * 2654435761) ^ (q[2] * 805459861)) % (2 ** 32) % size
            assert int(idx[0, l, c]) == int(spec.offsets[l]) + e
            wt = np.prod([f[d] if (c >> d) & 1 else 1 - f[d] for d in range(3)])
            assert abs(float(w[0, l, c]) - wt) < 1e-6
        assert abs(float(w[0, l].sum()) - 1) < 1e-6


def test_sh4_known_values():
    sh = O.sh4(torch.tensor([[0.0, 0.0, 2.0], [1.0, 0.0, 0.0]])).float()
    torch.testing.assert_close(sh[0, 0], torch.tensor(0.28209479177387814).half().float())
    torch.testing.assert_close(sh[0, 2], torch.tensor(0.48860251190291987).half().float())  # z
    torch.testing.assert_close(sh[1, 3], torch.tensor(-0.48860251190291987).half().float())  # -x
    torch.testing.assert_close(sh[0, 6], torch.tensor(0.94617469575755997 - 0.31539156525251999).half().float())


def test_adam_matches_torch():
    g = torch.Generator().manual_seed(1)
    p = torch.randn(1000, generator=g); gr = torch.randn(1000, generator=g)
    p_ref = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=1e-2, eps=1e-15)
    m = torch.zeros(1000); v = torch.zeros(1000)
    for step in (1, 2, 3):
        O.adam_(p, gr, m, v, 1e-2, step)
        p_ref.grad = gr.clone()
        opt.step()
    torch.testing.assert_close(p, p_ref.detach(), atol=1e-6, rtol=1e-5)


def test_grid_encode_fp32_vs_half_fma_accumulation():
    """Deviation of the encoding's corner sum accumulated in fp32 (this oracle
    and the product, bit-exact with each other) from tcnn's kernel_grid, which
    accumulates result = fma((T)weight, val, result) in T = __half (every
    corner's fma rounded to fp16).  Measured on ray samples with tcnn-scale
    table values: the features agree exactly or within 2 fp16 ulps of the
    half-accumulated value (documented in DESIGN.md §4)."""
    import synthetic as S
    spec = O.HashGridSpec(16, 19, 16, scale=0.5)
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(20000, 3, generator=g) - 0.5)
    table = (torch.rand(spec.n_entries * 2, generator=g) * 2 - 1) * 1.0
    mn, mx = -torch.ones(1, 3) * 0.5, torch.ones(1, 3) * 0.5
    enc32 = O.hash_encode_fwd(spec, x, mn, mx, table).float()  # (N, 32)
    idx, w = O.hash_corners(spec, x, mn, mx)  # (N, L, 8) entry index per corner, fp32 weight
    tab = table.half().double().view(-1, 2)
    wh = w.half().double()  # (T)weight
    r = torch.zeros(x.shape[0], spec.L, 2, dtype=torch.float64)
    for c in range(8):  # fma in half: exact product + sum, one rounding to fp16
        v = tab[idx[:, :, c].long()]
        r = (wh[:, :, c:c + 1] * v + r).half().double()
    enc16 = r.reshape(x.shape[0], 2 * spec.L).float()
    # scale of the accumulation: sum_c |w_c v_c| (fp16 ulps of the partial sums)
    mag = (wh.unsqueeze(-1) * tab[idx.long()].abs()).sum(2).reshape(x.shape[0], 2 * spec.L).float()
    ulps = (enc32 - enc16).abs() / O.ulp16(mag)
    same = float((enc32 == enc16).float().mean())
    print(f"grid encode, fp32 vs __half fma accumulation: {same:.2%} identical, "
          f"{float((ulps <= 1).float().mean()):.2%} within 1 fp16 ulp of sum|w v|, max {float(ulps.max()):.2f} ulps, "
          f"max abs {float((enc32 - enc16).abs().max()):.2e}")
    # 8 fma roundings of partial sums <= sum|w v|, each <= half an ulp
    assert float(ulps.max()) <= 4


def test_mlp_weight_gradient_operand_rounding():
    """The MLP weight gradients dW = sum_s G[o][s] H[i][s] take fp16 operands
    on the GPU (field.hip field_bwd_mlp_coop_kernel, tcnn's precision): each
    sample's gradient column is rounded to fp16 at its own power-of-two scale
    (largest |g| of the sample in [2^13, 2^14)), then re-scaled exactly to the
    128-sample block's common scale (factors <= 1: a second rounding only
    where a value becomes an fp16 subnormal); H is the fp16 activation.
    Operand rounding alone, over a step's ~150k samples with gradient
    magnitudes spread over decades like the training step's: relative L2 vs
    fp32 operands, next to bf16 operands (rounds 1-2's choice) for scale."""
    g = torch.Generator().manual_seed(1)
    n = 1172 * 128
    H = torch.relu(torch.randn(64, n, generator=g)).half().float()  # fp16 activations
    G = torch.randn(16, n, generator=g) * 1e-4 * torch.exp(2 * torch.randn(1, n, generator=g))
    ref = G.double() @ H.double().t()

    def rel(a):
        return float((a.double() - ref).norm() / ref.norm())

    bf = G.bfloat16().float() @ H.bfloat16().float().t()
    # the kernel's scheme: per-sample exponent E_s, block exponent B = min_s E_s over 128 samples
    E = 13 - torch.floor(torch.log2(G.abs().amax(0)))  # 2^E * max|g_s| in [2^13, 2^14)
    Gs = (G * torch.pow(2.0, E)).half()
    B = E.view(-1, 128).amin(1).repeat_interleave(128)
    Gb = (Gs.float() * torch.pow(2.0, B - E)).half().float()  # exact unless subnormal
    hf = (Gb * torch.pow(2.0, -B)) @ H.t()
    e_bf, e_hf = rel(bf), rel(hf)
    print(f"dW operand rounding, relative L2 vs fp32 operands: fp16 (per-sample, then block scale) {e_hf:.2e}, "
          f"bf16 {e_bf:.2e}")
    assert e_hf < 1e-3 and e_bf < 5e-3


def test_rg16_rounds_gradients_like_fp16_over_an_unbounded_exponent_range():
    """oracle.rg16 (the MLP backward's fp16 gradient storage model): identity
    forward; its backward equals a cast to fp16 wherever the value is in
    fp16's normal range, and keeps 11 significant bits far outside it (the
    power-of-two scales put every stored gradient in range)."""
    import oracle as O
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4096, generator=g) * torch.exp2(torch.randint(-12, 14, (4096,), generator=g).float())
    x = torch.cat([x, torch.tensor([0.0, -0.0, 1.0, 65504.0, 2.0 ** -14, 1 + 2.0 ** -11, 1 + 3 * 2.0 ** -11])])
    t = torch.zeros_like(x, requires_grad=True)
    y = O.rg16(t)
    assert torch.equal(y, t)
    y.backward(x)
    normal = (x.abs() >= 2.0 ** -14) | (x == 0)
    assert int(normal.sum()) > 3500
    assert torch.equal(t.grad[normal], x[normal].half().float())
    # far outside fp16's range: the same 11-bit mantissa, scaled
    xn = x[normal]
    big = xn * 2.0 ** 60
    t2 = torch.zeros_like(big, requires_grad=True)
    O.rg16(t2).backward(big)
    assert torch.equal(t2.grad, xn.half().float() * 2.0 ** 60)
