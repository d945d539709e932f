"""GPU parity: libngp_amd.so (through the reference-shaped `vren`) vs the CPU
oracle on the same seeded inputs.  Integer outputs (Morton codes, bitfields,
per-ray sample counts, rays_a) and the marcher's fp32 sample positions are
compared BIT-EXACTLY (both sides evaluate the reference's expressions with
no FMA contraction); compositing within 1e-5 abs/rel (the reference itself
uses __expf)."""
import numpy as np
import pytest
import torch

import oracle as O
import synthetic as S
import vren

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _scene_rays(n_rays, scale=0.5, seed=1, W=800):
    sc = S.SyntheticScene(W=W, H=W, n_images=20, scale=scale)
    gen = torch.Generator().manual_seed(seed)
    img, pix = sc.sample_batch(n_rays, gen)
    o, d = sc.rays(img, pix)
    return sc, o.contiguous(), d.contiguous(), img, pix


def _hits(o, d, scale):
    c = torch.zeros(1, 3); h = torch.ones(1, 3) * scale
    _, ht, _ = O.ray_aabb_intersect(o, d, c, h, 1)
    ht = ht.clone()
    m = (ht[:, 0, 0] >= 0) & (ht[:, 0, 0] < 0.01)
    ht[m, 0, 0] = 0.01
    return ht[:, 0].contiguous()


def _true_div255(u8):
    """u8 / 255 correctly rounded (numpy's astype(float32) / 255.0, the
    reference's read_image); torch turns division by a scalar into a
    multiplication by its reciprocal."""
    x = u8.float()
    return x / torch.full_like(x, 255.0)


def test_library_loads_on_gpu():
    assert torch.cuda.is_available()
    assert vren.lib().ngp_version().startswith(b"ngp_amd")


@pytest.mark.parametrize("max_hits,nv", [(1, 1), (3, 4)])
def test_ray_aabb_intersect(max_hits, nv):
    g = torch.Generator().manual_seed(0)
    o = (torch.rand(2000, 3, generator=g) - 0.5) * 4
    d = torch.randn(2000, 3, generator=g)
    d[:10, 0] = 0.0  # axis-parallel rays: inf/NaN slab handling
    c = (torch.rand(nv, 3, generator=g) - 0.5)
    h = torch.rand(nv, 3, generator=g) * 0.5 + 0.1
    ref = O.ray_aabb_intersect(o, d, c, h, max_hits)
    out = vren.ray_aabb_intersect(o.to(DEV), d.to(DEV), c.to(DEV), h.to(DEV), max_hits)
    assert torch.equal(out[0].cpu(), ref[0])
    assert torch.equal(out[1].cpu(), ref[1])
    assert torch.equal(out[2].cpu(), ref[2])


def test_raygen_aabb_matches_host_rays():
    sc, o, d, img, pix = _scene_rays(8192)
    center = torch.zeros(1, 3, device=DEV); half = torch.ones(1, 3, device=DEV) * 0.5
    ro, rd, ht = vren.raygen_aabb(sc.directions.to(DEV), sc.poses.to(DEV), img.to(DEV), pix.to(DEV), center, half,
                                  0.01)
    assert torch.allclose(ro.cpu(), o, atol=0, rtol=0)
    assert torch.allclose(rd.cpu(), d, atol=1e-6, rtol=1e-6)
    ref = _hits(ro.cpu(), rd.cpu(), 0.5)  # same rays -> bit-exact AABB + clamp
    assert torch.equal(ht.cpu(), ref)


def test_sample_batch_on_device():
    """ngp_sample_batch (datasets/base.py:22-35 + get_rays + AABB + noise on
    device): the rays equal raygen_aabb on the drawn pixels bit for bit, the
    ground truth is the u8 gather / 255 (or the f32 gather), indices and
    noise are in range and roughly uniform, the draw is a pure function of
    (seed, step, global ray index): two ranks with ray_offset 0 / R/2 draw
    the two halves of the single-process batch."""
    import ctypes
    sc = S.SyntheticScene(W=200, H=200, n_images=20, scale=0.5)
    gt = torch.randint(0, 256, (20, 200 * 200, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(0)).to(DEV)
    dirs, poses = sc.directions.to(DEV), sc.poses.to(DEV)
    center = torch.zeros(1, 3, device=DEV); half = torch.ones(1, 3, device=DEV) * 0.5
    R = 1 << 16

    gtf = torch.rand(20, 200 * 200, 3, generator=torch.Generator().manual_seed(1)).to(DEV)

    def draw(seed, step, n=R, offset=0, g=gt):
        out = dict(img=torch.empty(n, dtype=torch.int64, device=DEV), pix=torch.empty(n, dtype=torch.int64, device=DEV),
                   rgb=torch.empty(n, 3, device=DEV), noise=torch.empty(n, device=DEV),
                   o=torch.empty(n, 3, device=DEV), d=torch.empty(n, 3, device=DEV), ht=torch.empty(n, 2, device=DEV))
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        vren._ok(vren.lib().ngp_sample_batch(seed, step, offset, p(g), int(g.dtype == torch.float32), 20, 200 * 200,
                                             p(dirs), p(poses), n, p(center), p(half), 0.01, p(out["img"]),
                                             p(out["pix"]), p(out["rgb"]), p(out["noise"]), p(out["o"]), p(out["d"]),
                                             p(out["ht"]), vren._stream()),
                 "sample_batch")
        return out

    a, b, c = draw(5, 1), draw(5, 1), draw(5, 2)
    for k in a:
        assert torch.equal(a[k], b[k])
    assert not torch.equal(a["pix"], c["pix"])
    assert int(a["img"].min()) >= 0 and int(a["img"].max()) < 20
    assert int(a["pix"].min()) >= 0 and int(a["pix"].max()) < 200 * 200
    assert float(a["noise"].min()) >= 0 and float(a["noise"].max()) < 1
    hist = torch.bincount(a["img"], minlength=20).float()
    assert float(hist.min()) > 0.9 * R / 20 and float(hist.max()) < 1.1 * R / 20
    assert abs(float(a["noise"].mean()) - 0.5) < 0.01
    ro, rd, ht = vren.raygen_aabb(dirs, poses, a["img"], a["pix"], center, half, 0.01)
    assert torch.equal(ro, a["o"]) and torch.equal(rd, a["d"]) and torch.equal(ht, a["ht"])
    assert torch.equal(a["rgb"], _true_div255(gt[a["img"], a["pix"]]))
    h0, h1 = draw(5, 1, R // 2, 0), draw(5, 1, R // 2, R // 2)
    for k in a:
        assert torch.equal(torch.cat([h0[k], h1[k]]), a[k])
    f = draw(5, 1, g=gtf)
    assert torch.equal(f["pix"], a["pix"]) and torch.equal(f["rgb"], gtf[a["img"], a["pix"]])


def test_morton_packbits():
    g = torch.Generator().manual_seed(3)
    coords = torch.randint(0, 128, (100000, 3), generator=g, dtype=torch.int32)
    m = vren.morton3D(coords.to(DEV))
    assert torch.equal(m.cpu(), O.morton3D(coords))
    assert torch.equal(vren.morton3D_invert(m).cpu(), coords)
    grid = torch.rand(6 * 128 ** 3 // 64 * 64, generator=g)
    bf = torch.zeros(grid.numel() // 8, dtype=torch.uint8, device=DEV)
    vren.packbits(grid.to(DEV), 0.7, bf)
    ref = torch.zeros(grid.numel() // 8, dtype=torch.uint8)
    O.packbits(grid, 0.7, ref)
    assert torch.equal(bf.cpu(), ref)
    thr = torch.tensor([0.3], device=DEV)
    vren.packbits(grid.to(DEV), thr, bf)  # device-side threshold
    O.packbits(grid, 0.3, ref)
    assert torch.equal(bf.cpu(), ref)


@pytest.mark.parametrize("scale,esf,n_rays,max_samples", [(0.5, 0.0, 8192, 1024), (16.0, 1 / 256, 4096, 1024),
                                                         (0.5, 0.0, 3000, 7)])
def test_march_train_bit_exact(scale, esf, n_rays, max_samples):
    sc, o, d, _, _ = _scene_rays(n_rays, scale=scale, W=400)
    ht = _hits(o, d, scale)
    noise = torch.rand(n_rays, generator=torch.Generator().manual_seed(3))
    bf = sc.bitfield
    ref = O.raymarching_train(o, d, ht, bf, sc.cascades, scale, esf, noise, 128, max_samples)
    out = vren.raymarching_train(o.to(DEV), d.to(DEV), ht.to(DEV), bf.to(DEV), sc.cascades, scale, esf,
                                 noise.to(DEV), 128, max_samples)
    assert int(out[5][0]) == int(ref[5][0]) and int(out[5][1]) == n_rays
    assert int(ref[5][0]) > (n_rays if max_samples > 100 else n_rays // 10)  # the shell is actually hit
    for a, b in zip(out[:5], ref[:5]):
        assert torch.equal(a.cpu(), b)


@pytest.mark.parametrize("occ,scale,max_samples", [("scene", 0.5, 1024), ("rand0.01", 0.5, 1024),
                                                   ("rand0.2", 0.5, 1024), ("rand0.7", 0.5, 1024),
                                                   ("scene", 0.25, 1024), ("rand0.05", 0.3, 1024),
                                                   ("scene", 0.5, 40), ("blocks", 0.5, 1024)])
def test_march_train_occupancy_patterns_bit_exact(occ, scale, max_samples):
    """The training march (the wave-per-ray lattice walk) equals the oracle's serial
    walk bit for bit -- counts, rays_a, xyz, dirs, t, dt -- on the scene's shell, on
    random bitfields of several densities (many short empty / occupied runs: the
    walk's chain through a window alternates between steps and jumps), on sparse
    Morton-aligned 4^3 blocks (the summary's early out), at scales whose mip bound
    is below 0.5 and with a max_samples cut."""
    n_rays = 4096
    sc, o, d, _, _ = _scene_rays(n_rays, scale=scale, W=400)
    ht = _hits(o, d, scale)
    noise = torch.rand(n_rays, generator=torch.Generator().manual_seed(5))
    g = torch.Generator().manual_seed(7)
    if occ == "scene":
        bf = sc.bitfield
    elif occ == "blocks":  # whole Morton-aligned 4^3 blocks (64-bit words) on or off
        words = (torch.rand(128 ** 3 // 64, generator=g) < 0.03)
        bf = words.repeat_interleave(8).to(torch.uint8) * 255
    else:
        frac = float(occ[4:])
        bits = (torch.rand(128 ** 3, generator=g) < frac).to(torch.uint8)
        bf = (bits.view(-1, 8) << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
    ref = O.raymarching_train(o, d, ht, bf, 1, scale, 0.0, noise, 128, max_samples)
    out = vren.raymarching_train(o.to(DEV), d.to(DEV), ht.to(DEV), bf.to(DEV), 1, scale, 0.0, noise.to(DEV), 128,
                                 max_samples)
    assert int(out[5][0]) == int(ref[5][0])
    for a, b in zip(out[:5], ref[:5]):
        assert torch.equal(a.cpu(), b)


def test_march_train_empty_and_misses():
    o = torch.tensor([[5.0, 5.0, 5.0]]); d = torch.tensor([[1.0, 0.0, 0.0]])
    ht = torch.tensor([[-1.0, -1.0]])
    bf = torch.full((128 ** 3 // 8,), 255, dtype=torch.uint8)
    out = vren.raymarching_train(o.to(DEV), d.to(DEV), ht.to(DEV), bf.to(DEV), 1, 0.5, 0.0,
                                 torch.zeros(1, device=DEV), 128, 1024)
    assert int(out[5][0]) == 0 and out[1].shape == (0, 3)
    assert out[0].cpu().tolist() == [[0, 0, 0]]


def test_composite_train_fw_bw():
    sc, o, d, _, _ = _scene_rays(4096, W=400)
    ht = _hits(o, d, 0.5)
    noise = torch.rand(4096, generator=torch.Generator().manual_seed(4))
    rays_a, xyzs, dirs, deltas, ts, cnt = O.raymarching_train(o, d, ht, sc.bitfield, 1, 0.5, 0.0, noise, 128, 1024)
    N = xyzs.shape[0]
    g = torch.Generator().manual_seed(5)
    sig = torch.rand(N, generator=g) * 200
    rgbs = torch.rand(N, 3, generator=g)
    ref = O.composite_train_fw(sig, rgbs, deltas, ts, rays_a, 1e-4)
    D = lambda x: x.to(DEV)
    out = vren.composite_train_fw(D(sig), D(rgbs), D(deltas), D(ts), D(rays_a), 1e-4)
    # composited counts: a ray may end one sample earlier / later only where the
    # transmittance lands on the threshold within fp32 rounding: each factor
    # exp(-sigma delta) is an __expf (a few fp32 ulps) and the product of k
    # factors is reassociated -- bound |ln T - ln T_thr| <= (k + 1) 2^-20 on
    # the exact (fp64) transmittance after the boundary sample k
    cg, cr = out[0].cpu(), ref[0]
    assert (cg - cr).abs().max() <= 1
    flipped = torch.nonzero(cg != cr)[:, 0]
    for r in flipped.tolist():
        st, n = int(rays_a[r, 1]), int(rays_a[r, 2])
        T = torch.cumprod(torch.exp(-(sig[st:st + n].double() * deltas[st:st + n].double())), 0)
        k = int(min(cg[r], cr[r]))
        assert abs(float(torch.log(T[k])) - float(torch.log(torch.tensor(1e-4, dtype=torch.float64)))) <= \
            (k + 1) * 2.0 ** -20, (r, k)
    print(f"composited counts: {flipped.numel()} of 4096 rays end one sample apart, all at T = T_thr within the bound")
    for a, b in zip(out[1:], ref[1:]):
        torch.testing.assert_close(a.cpu(), b, atol=1e-5, rtol=1e-4)
    gop, gdep, grgb, gws = torch.randn(4096, generator=g), torch.randn(4096, generator=g), \
        torch.randn(4096, 3, generator=g), torch.randn(N, generator=g)
    refb = O.composite_train_bw(gop, gdep, grgb, gws, sig, rgbs, ref[4], deltas, ts, rays_a, ref[1], ref[2], ref[3],
                                1e-4)
    outb = vren.composite_train_bw(D(gop), D(gdep), D(grgb), D(gws), D(sig), D(rgbs), D(ref[4]), D(deltas), D(ts),
                                   D(rays_a), D(ref[1]), D(ref[2]), D(ref[3]), 1e-4)
    torch.testing.assert_close(outb[0].cpu(), refb[0], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(outb[1].cpu(), refb[1], atol=1e-5, rtol=1e-4)


def test_march_test_and_composite_test():
    sc, o, d, _, _ = _scene_rays(5000, W=400)
    ht = _hits(o, d, 0.5)
    alive = torch.arange(5000, dtype=torch.int64)[::2].contiguous()
    ht_ref = ht.clone()
    ref = O.raymarching_test(o, d, ht_ref, alive, sc.bitfield, 1, 0.5, 0.0, 128, 1024, 8)
    ht_gpu = ht.to(DEV)
    out = vren.raymarching_test(o.to(DEV), d.to(DEV), ht_gpu, alive.to(DEV), sc.bitfield.to(DEV), 1, 0.5, 0.0, 128,
                                1024, 8)
    for a, b in zip(out, ref):
        assert torch.equal(a.cpu(), b)
    assert torch.equal(ht_gpu.cpu(), ht_ref)
    n = alive.numel()
    g = torch.Generator().manual_seed(6)
    sig = torch.rand(n, 8, generator=g) * 100; rgbs = torch.rand(n, 8, 3, generator=g)
    op = torch.rand(5000, generator=g) * 0.5; dep = torch.zeros(5000); rgb = torch.zeros(5000, 3)
    al_ref = alive.clone(); op_ref, dep_ref, rgb_ref = op.clone(), dep.clone(), rgb.clone()
    O.composite_test_fw(sig, rgbs, ref[2], ref[3], ht_ref, al_ref, 1e-4, ref[4], op_ref, dep_ref, rgb_ref)
    al_g, op_g, dep_g, rgb_g = alive.to(DEV), op.to(DEV), dep.to(DEV), rgb.to(DEV)
    vren.composite_test_fw(sig.to(DEV), rgbs.to(DEV), out[2], out[3], ht_gpu, al_g, 1e-4, out[4], op_g, dep_g, rgb_g)
    assert (al_g.cpu() != al_ref).sum() <= 2
    torch.testing.assert_close(op_g.cpu(), op_ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rgb_g.cpu(), rgb_ref, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(dep_g.cpu(), dep_ref, atol=1e-5, rtol=1e-5)


def test_check_input_errors_like_reference():
    x = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        vren.morton3D(x.int())
    y = torch.zeros(4, 6, dtype=torch.int32, device=DEV)[:, ::2]
    with pytest.raises(RuntimeError, match="must be contiguous"):
        vren.morton3D(y)


@pytest.mark.parametrize("sorted_", [False, True])
def test_device_occupancy_sampling(sorted_):
    """ngp_occupied_cells lists exactly the cells above the threshold;
    ngp_occupancy_samples draws M uniform + M occupied cells (none when the
    list is empty) with positions inside the jittered cell (networks.py:
    181-207, 262-266), a pure function of the device counter.  The sorted
    variant emits each half in ascending order with the same distribution:
    the empirical CDFs stay within a DKW band of the uniform ones."""
    import ctypes
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    L = vren.lib()
    G, s = 128, 0.5
    hgs = s / G
    g = torch.Generator(device=DEV).manual_seed(0)
    grid = torch.rand(G ** 3, device=DEV, generator=g) * 10
    grid[torch.rand(G ** 3, device=DEV, generator=g) < 0.3] = -1
    thr = 5.9
    lst = torch.empty(G ** 3, dtype=torch.int32, device=DEV)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    ws_l = torch.empty((L.ngp_occupied_cells_workspace(G ** 3) + 3) // 4, dtype=torch.int32, device=DEV)
    vren._ok(L.ngp_occupied_cells(p(grid), G ** 3, thr, p(lst), p(cnt), p(ws_l), vren._stream()), "occ")
    ref = torch.nonzero(grid > thr)[:, 0]
    n = int(cnt.item())
    assert n == ref.numel()
    assert torch.equal(lst[:n].long(), ref)  # torch.nonzero's order: ascending, deterministic
    M = G ** 3 // 4
    ctr = torch.tensor([7], dtype=torch.int64, device=DEV)
    xyz = torch.empty(2 * M, 3, device=DEV)
    flat = torch.empty(2 * M, dtype=torch.int64, device=DEV)

    ws = torch.empty((L.ngp_occupancy_sorted_workspace(M) + 7) // 8, dtype=torch.float64, device=DEV)

    def draw(c_lst, c_cnt, lo=0, hi=2 * M):
        if sorted_:
            vren._ok(L.ngp_occupancy_samples_sorted(99, p(ctr), 0, G, M, s - hgs, hgs, p(c_lst), p(c_cnt), lo, hi,
                                                    p(ws), p(xyz), p(flat), vren._stream()), "samples_sorted")
        else:
            vren._ok(L.ngp_occupancy_samples(99, p(ctr), 0, G, M, s - hgs, hgs, p(c_lst), p(c_cnt), lo, hi, p(xyz),
                                             p(flat), vren._stream()), "samples")
        return xyz[:hi - lo].clone(), flat[:hi - lo].clone()

    x, f = draw(lst, cnt)
    assert int(f.min()) >= 0 and int(f.max()) < G ** 3
    occ = torch.zeros(G ** 3, dtype=torch.bool, device=DEV)
    occ[ref] = True
    assert bool(occ[f[M:]].all())  # second half drawn from the occupied list
    coords = vren.morton3D_invert(f.int().contiguous()).float()
    centre = (coords / (G - 1) * 2 - 1) * (s - hgs)
    assert float((x - centre).abs().max()) <= hgs + 4e-7  # a few fp32 ulps at |x| <= 0.5
    # uniform half: roughly uniform over cells
    assert abs(float(occ[f[:M]].float().mean()) - n / G ** 3) < 0.01
    if sorted_:
        pos = torch.empty(G ** 3, dtype=torch.int64, device=DEV)
        pos[lst[:n].long()] = torch.arange(n, device=DEV)
        lp = pos[f[M:]]  # list positions of the occupied half
        assert bool((f[1:M] >= f[:M - 1]).all()) and bool((lp[1:] >= lp[:-1]).all())
        k = (torch.arange(M, device=DEV, dtype=torch.float64) + 0.5) / M
        band = 2.0 / M ** 0.5  # DKW: P(sup|F_M - F| > 2/sqrt(M)) = 2 exp(-8) ~ 7e-4
        assert float((f[:M].double() / G ** 3 - k).abs().max()) < band + 1.0 / G ** 3
        assert float((lp.double() / n - k).abs().max()) < band + 1.0 / n
    # shards of the same draw are slices of it
    x2, f2 = draw(lst, cnt, lo=1000, hi=5000)
    assert torch.equal(f2, f[1000:5000]) and torch.equal(x2, x[1000:5000])
    # empty occupied list: the second half is skipped (-1)
    cnt.zero_()
    _, f3 = draw(lst, cnt)
    assert bool((f3[M:] == -1).all()) and torch.equal(f3[:M], f[:M])


@pytest.mark.parametrize("n_rows", [1, 63, 64, 8192, 8193, 70000])
def test_ray_segments_lists(n_rows):
    """ngp_ray_segments / ngp_active_samples / ngp_ray_segments_capped (fused
    scan + map up to 65536 rows, scan + map launches above): start offsets,
    totals and index lists equal a torch cumsum / repeat_interleave, incl.
    empty rows."""
    import ctypes
    L = vren.lib()
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator().manual_seed(n_rows)
    N = torch.randint(0, 200, (n_rows,), generator=g)
    N[torch.rand(n_rows, generator=g) < 0.2] = 0
    start = torch.cumsum(N, 0) - N
    rays_a = torch.stack([torch.arange(n_rows), start, N], 1).to(DEV)
    first = 5
    counts = torch.clamp(N - first, min=0).to(torch.int32)

    def expect(c, off):
        c64 = c.long()
        st = torch.cumsum(c64, 0) - c64
        idx = torch.repeat_interleave(start + off, c64) + (torch.arange(int(c64.sum())) -
                                                            torch.repeat_interleave(st, c64))
        return st, int(c64.sum()), idx

    st_ws = torch.empty(n_rows, dtype=torch.int64, device=DEV)
    tot = torch.zeros(1, dtype=torch.int64, device=DEV)
    acc = torch.full((1,), 7, dtype=torch.int64, device=DEV)
    sidx = torch.full((int(N.sum()) + 1,), -1, dtype=torch.int32, device=DEV)
    cd = counts.to(DEV)
    vren._ok(L.ngp_ray_segments(p(cd), p(rays_a), n_rows, first, p(st_ws), p(tot), p(acc), p(sidx), vren._stream()),
             "segments")
    st, total, idx = expect(counts, first)
    assert torch.equal(st_ws.cpu(), st) and int(tot) == total and int(acc) == 7 + total
    assert torch.equal(sidx[:total].cpu().long(), idx)
    # active samples: offset 0, no accumulator
    vren._ok(L.ngp_active_samples(p(cd), p(rays_a), n_rows, p(st_ws), p(tot), p(sidx), vren._stream()), "active")
    st, total, idx = expect(counts, 0)
    assert int(tot) == total and torch.equal(sidx[:total].cpu().long(), idx)
    # capped (round 1 of the chunked forward)
    K = 64
    rc = L.ngp_ray_segments_capped(p(rays_a), n_rows, K, p(st_ws), p(tot), None, p(sidx), vren._stream())
    if n_rows > 65536:
        assert rc != 0
        return
    vren._ok(rc, "capped")
    st, total, idx = expect(torch.clamp(N, max=K), 0)
    assert torch.equal(st_ws.cpu(), st) and int(tot) == total
    assert torch.equal(sidx[:total].cpu().long(), idx)


@pytest.mark.parametrize("n_rows,first,last", [(1, 64, 0), (63, 64, 0), (8192, 64, 0), (8193, 5, 0), (8192, 100, 150),
                                               (70000, 64, 0)])
def test_chunk_segments_equals_counts_then_segments(n_rows, first, last):
    """ngp_chunk_segments (one launch: round-2 counts + look-back scan + map)
    equals ngp_chunk_counts_range followed by ngp_ray_segments: start
    offsets, total, accumulator and the index list, bit for bit -- three
    launches in a row on one workspace (the ticket / generation reset), incl.
    grids larger than the GPU holds at once (70000 rows: 1094 blocks) and
    rows longer than one 64-sample chunk (first 100)."""
    import ctypes
    L = vren.lib()
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator().manual_seed(n_rows + first)
    N = torch.randint(0, 260, (n_rows,), generator=g)
    N[torch.rand(n_rows, generator=g) < 0.2] = 0
    start = torch.cumsum(N, 0) - N
    n_s = int(N.sum()) + 1
    rays_a = torch.stack([torch.arange(n_rows), start, N], 1).to(DEV)
    dense = torch.rand(n_rows, generator=g) < 0.5  # rows terminating in the first chunk vs transparent ones
    row = torch.repeat_interleave(torch.arange(n_rows), N)
    sig = torch.rand(n_s, generator=g) * 2
    sig[:-1] *= torch.where(dense[row], 50.0, 1.0)
    sig = sig.to(DEV)
    dl = (torch.rand(n_s, generator=g) * 0.02).to(DEV)
    cnt = torch.empty(n_rows, dtype=torch.int32, device=DEV)
    vren._ok(L.ngp_chunk_counts_range(p(rays_a), n_rows, first, last, p(sig), p(dl), ctypes.c_float(1e-4), p(cnt),
                                      vren._stream()), "counts")
    st_ref = torch.empty(n_rows, dtype=torch.int64, device=DEV)
    tot_ref, acc_ref = torch.zeros(1, dtype=torch.int64, device=DEV), torch.full((1,), 7, dtype=torch.int64, device=DEV)
    idx_ref = torch.full((n_s,), -1, dtype=torch.int32, device=DEV)
    vren._ok(L.ngp_ray_segments(p(cnt), p(rays_a), n_rows, first, p(st_ref), p(tot_ref), p(acc_ref), p(idx_ref),
                                vren._stream()), "segments")
    ws = torch.zeros((L.ngp_chunk_segments_workspace(n_rows) + 7) // 8, dtype=torch.int64, device=DEV)
    acc = torch.full((1,), 7, dtype=torch.int64, device=DEV)
    add = torch.full((1,), 11, dtype=torch.int64, device=DEV)  # total_acc_add: a round-1 count added with it
    acc_expect = 7
    for it in range(3):
        st = torch.full((n_rows,), -5, dtype=torch.int64, device=DEV)
        tot = torch.zeros(1, dtype=torch.int64, device=DEV)
        idx = torch.full((n_s,), -1, dtype=torch.int32, device=DEV)
        vren._ok(L.ngp_chunk_segments(p(sig), p(dl), p(rays_a), n_rows, first, last, ctypes.c_float(1e-4), p(ws),
                                      p(st), p(tot), p(acc), p(add) if it % 2 else None, p(idx), vren._stream()),
                 "chunk_segments")
        torch.cuda.synchronize()
        T = int(tot_ref)
        acc_expect += T + (11 if it % 2 else 0)
        assert int(tot) == T and int(acc) == acc_expect
        assert torch.equal(st, st_ref) and torch.equal(idx[:T], idx_ref[:T])
    if n_rows >= 1000:  # some rows terminate inside the first chunk, some go on
        assert 0 < int(tot_ref) < int(N.sum())


@pytest.mark.parametrize("n_rows", [1, 100, 8192, 70000])
def test_rays_nonempty_lists_rows_and_zeroes_empty_counts(n_rows):
    """ngp_rays_nonempty: the rows with N > 0 in ascending order and their
    count; rest[r] = 0 for every empty row, the others untouched (the row
    forward's round 1 writes them); the round-2 list length zeroed."""
    import ctypes
    L = vren.lib()
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator().manual_seed(n_rows)
    N = torch.randint(0, 300, (n_rows,), generator=g)
    N[torch.rand(n_rows, generator=g) < 0.67] = 0
    rays_a = torch.stack([torch.arange(n_rows), torch.cumsum(N, 0) - N, N], 1).to(DEV)
    rows = torch.full((n_rows,), -1, dtype=torch.int32, device=DEV)
    n_ne = torch.full((1,), -3, dtype=torch.int64, device=DEV)
    rest = torch.full((n_rows,), 7, dtype=torch.int32, device=DEV)
    z = torch.full((1,), 5, dtype=torch.int64, device=DEV)
    vren._ok(L.ngp_rays_nonempty(p(rays_a), n_rows, p(rows), p(n_ne), p(rest), p(z), vren._stream()), "rays_nonempty")
    torch.cuda.synchronize()
    ref = torch.nonzero(N > 0).flatten()
    assert int(n_ne) == ref.numel()
    assert torch.equal(rows[:ref.numel()].cpu().long(), ref)
    assert torch.equal(rest.cpu(), torch.where(N > 0, 7, 0).int()) and int(z) == 0


@pytest.mark.timeout(60)
def test_march_ends_a_degenerate_ray_instead_of_spinning():
    """A ray whose t is so large that t + dt == t in fp32 (camera 4e4 units away:
    ulp(t) > 2 dt) never advances in the reference's `do t += dt while (t <
    t_target)` -- an endless loop.  The marcher ends such a ray (counted as a
    guard hit) and every other ray of the batch is marched as usual."""
    import vren as V
    sc, o, d, _, _ = _scene_rays(256, W=64)
    o = o.clone()
    o[0] = torch.tensor([4.0e4, 0.0, 0.0])
    d = d.clone()
    d[0] = torch.tensor([-1.0, 0.0, 0.0])
    ht = _hits(o, d, 0.5)
    noise = torch.rand(256, generator=torch.Generator().manual_seed(2))
    # one occupied cell, at the centre: the far ray passes within a block of it (no early out),
    # and its first probe at the box's face is empty -- the jump that never advances
    bf = torch.zeros(128 ** 3 // 8, dtype=torch.uint8)
    c = int(vren.morton3D(torch.tensor([[64, 64, 64]], dtype=torch.int32, device=DEV))[0])
    bf[c // 8] = 1 << (c % 8)
    L = V.lib()
    assert L.ngp_guard_reset() == 0
    try:
        out = vren.raymarching_train(o.to(DEV), d.to(DEV), ht.to(DEV), bf.to(DEV), 1, 0.5, 0.0,
                                     noise.to(DEV), 128, 1024)
        torch.cuda.synchronize()
        assert int(out[0][0, 2]) == 0 and int(L.ngp_guard_hits()) >= 1
        ref = O.raymarching_train(o[1:], d[1:], ht[1:], bf, 1, 0.5, 0.0, noise[1:], 128, 1024)
        assert torch.equal(out[0][1:, 2].cpu(), ref[0][:, 2])
    finally:
        assert L.ngp_guard_reset() == 0
