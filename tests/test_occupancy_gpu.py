"""Occupancy-grid upkeep on the MI355X against the reference glue
(tests/golden/occupancy_erode.npz, density_update.npz; make_golden.py runs
models/networks.py mark_invisible_cells / update_density_grid with the
oracle as tcnn, on one thread so duplicate cells resolve last-writer-wins).

* mark_invisible_cells (networks.py:209-250): the number of covering cameras
  per cell and the -1 marks bit-exact (sha256 of the whole grids) outside
  the cells whose projection lies within 1e-5 (relative, fp64) of an image
  border or the near plane (oracle.mark_borderline_cells, ~0.04 % of cells:
  there the in_image tests depend on the float32 matmul's summation order,
  which differs between BLAS builds and devices), Lego (1 cascade) and
  garden-sized (scale 16, 6 cascades).  count_grid = covered.sum(0) / N_cams:
  on a GPU torch divides a tensor by a scalar as a multiplication by the
  fp32 reciprocal (k * fl(1/N), what the reference's CUDA run computes), on
  the CPU it rounds k / N directly (the fixture's glue run) -- the last bit
  differs for some k; the product's count_grid is exactly k * fl(1/N).
* grid EMA with the erode decay (networks.py:270-276): the device kernel is
  bit-exact vs the torch expression on random grids, threshold from the
  fp64 mean within 1 fp32 ulp of torch's.
* the erode chain (2 warm-up updates + 1 sampled update, the glue's torch RNG
  draws replayed from the CPU generator) and the plain warm-up + sampled
  update through the drop-in NGP: bitfields vs the glue.  A cell may differ
  only if its product density is within the oracle's error bound of the
  threshold: sigma = exp(h0), and |h0 - h0_oracle| is bounded per sample by
  oracle.mlp_forward_bound (one fp16 ulp at every storage point + fp32
  accumulation in any order) -- checked for every differing cell, their
  number reported.  Before a sampled update the cells within 5 % of the
  threshold are pinned to the glue's values (fixture pins), so both draw
  from the same occupied-cell list.
* NGPTrainer's device update == the drop-in NGP's bit for bit on the same
  jitter (same density kernels; the EMA is exact).
"""
import contextlib
import hashlib

import numpy as np
import pytest
import torch

import oracle as O
import synthetic as S
import vren
from fixture_model import FixtureModel, load
from models.networks import NGP
from trainer import NGPTrainer

pytestmark = pytest.mark.gpu
DEV = "cuda"
THR = 0.01 * 1024 / 3 ** 0.5


def _sha(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def _scene(fx, scale):
    return S.AnalyticScene(W=int(fx["W"]), H=int(fx["H"]), n_images=int(fx["n_cams"]), scale=scale)


def _ngp(scale, seed=None, amp=None):
    m = NGP(scale)
    if seed is not None:
        fm = FixtureModel(scale, seed, amp)
        m.load_tcnn_params(fm.xyz_encoder.params.detach(), fm.rgb_net.params.detach())
    G = m.grid_size
    ax = torch.arange(G, dtype=torch.int32)
    m.register_buffer("density_grid", torch.zeros(m.cascades, G ** 3))
    m.register_buffer("grid_coords", torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3))
    return m.to(DEV)


@contextlib.contextmanager
def cpu_rng_replay(log=None):
    """torch.randint / torch.rand_like draw on the CPU default generator (as
    the reference glue did when the fixture was made) and move to the device."""
    ri, rl = torch.randint, torch.rand_like

    def randint(*a, device=None, **k):
        out = ri(*a, **k)
        if log is not None:
            log.append(("randint", out))
        return out.to(device) if device is not None else out

    def rand_like(x, **k):
        out = torch.rand(x.shape, dtype=x.dtype)
        if log is not None:
            log.append(("rand", out))
        return out.to(x.device)

    torch.randint, torch.rand_like = randint, rand_like
    try:
        yield
    finally:
        torch.randint, torch.rand_like = ri, rl


G = 128
_COORDS = torch.stack(torch.meshgrid(*[torch.arange(G, dtype=torch.int32)] * 3, indexing="ij"), -1).reshape(-1, 3)
_MORTON = O.morton3D(_COORDS).long()  # grid_coords row -> cell
_ROW = torch.argsort(_MORTON)  # cell -> grid_coords row


def _xyz(coords, jit, scale=0.5, c=0):
    """networks.py:263-267 in fp32, as both sides compute it."""
    s = min(2 ** (c - 1), scale)
    hgs = s / G
    return (coords / (G - 1) * 2 - 1) * (s - hgs) + (jit * 2 - 1) * hgs


def _sigma_bound(fm, xyz):
    """log-space bound on |ln sigma_product - ln sigma_oracle| per point:
    the h0 bound of oracle.mlp_forward_bound plus fp32 exp rounding."""
    p = fm.xyz_encoder.params.detach()
    spec = O.HashGridSpec(scale=fm.scale)
    enc = O.hash_encode_fwd(spec, xyz.float(), fm.xyz_min, fm.xyz_max, p[3072:])
    Ws, _ = O.mlp_layers(p[:3072], (32, 64, 16))
    _, b = O.mlp_forward_bound(enc, Ws)
    return b[:, 0].double() + 4 * 2.0 ** -24


def _flipped(got, ref):
    diff = np.unpackbits(got ^ ref, bitorder="little").astype(bool)
    return torch.from_numpy(np.nonzero(diff)[0]).long()


def _check_flips(cells, grid, bound, what):
    """every differing cell's product density within its bound of thr (log)"""
    g = grid.reshape(-1).cpu()[cells].double()
    dist = (torch.log(g.clamp_min(1e-30)) - np.log(THR)).abs()
    bad = dist > bound + 2 * 2.0 ** -23  # (+ erode decay ulps: its count differs in the last bit)
    print(f"{what}: {cells.numel()} of {G ** 3} cells differ from the glue, all within the error bound "
          f"(max bound {float(bound.max()) if bound.numel() else 0:.2e})" if not bad.any() else
          f"{what}: cells {cells[bad][:8].tolist()} differ beyond the bound ({dist[bad][:8].tolist()} > "
          f"{bound[bad][:8].tolist()})")
    assert not bad.any()


def _warm_bounds(fm, cells, jits):
    """bound per cell over the warm-up evaluations (one per update, jitter j)"""
    rows = _ROW[cells]
    b = torch.zeros(cells.numel(), dtype=torch.float64)
    for j in jits:
        b = torch.maximum(b, _sigma_bound(fm, _xyz(_COORDS[rows].float(), j[rows])))
    return b


def _sampled_bounds(fm, cells, log, occupied):
    """bound per cell for a sampled update: the evaluation at the LAST list
    entry of the cell (sample_uniform_and_occupied_cells' list, rebuilt from
    the replayed draws and the occupied list it resampled)"""
    (_, coords1), (_, ridx), (_, jit) = [e for e in log if e[0] in ("randint", "rand")]
    idx = torch.cat([O.morton3D(coords1.int()).long(), occupied[ridx]])
    coords = torch.cat([coords1.int(), _COORDS[_ROW[occupied[ridx]]]])
    last = torch.full((G ** 3,), -1, dtype=torch.int64)
    last.scatter_reduce_(0, idx, torch.arange(idx.numel()), reduce="amax")
    pos = last[cells]
    b = torch.zeros(cells.numel(), dtype=torch.float64)
    hit = pos >= 0
    if hit.any():
        b[hit] = _sigma_bound(fm, _xyz(coords[pos[hit]].float(), jit[pos[hit]]))
    return b


def _pin(m, fx, key):
    idx = torch.from_numpy(fx[f"{key}_pin_idx"]).long().to(DEV)
    m.density_grid[0, idx] = torch.from_numpy(fx[f"{key}_pin_val"]).to(DEV)
    return torch.nonzero(m.density_grid[0] > THR)[:, 0].cpu()


@pytest.mark.parametrize("tag,scale", [("lego", 0.5), ("garden", 16.0)])
def test_mark_invisible_cells_bit_exact(tag, scale):
    fx = load("occupancy_erode")
    sc = _scene(fx, scale)
    tr = NGPTrainer(scale=scale, batch_size=256, sample_capacity=256 * 64, device=DEV)
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    N = int(fx["n_cams"])
    k = torch.round(tr.count_grid.cpu() * N)
    assert torch.equal(tr.count_grid.cpu(), k * torch.tensor(1 / N, dtype=torch.float32))
    bl = O.mark_borderline_cells(sc.K, sc.poses, (sc.W, sc.H), G, scale, tr.cascades)
    assert int(bl.sum()) == int(fx[f"{tag}_n_borderline"])
    assert _sha(torch.where(bl, 255, k.long()).to(torch.uint8)) == str(fx[f"{tag}_k_masked_sha"])
    assert _sha(torch.where(bl, 7.0, tr.density_grid.cpu())) == str(fx[f"{tag}_mark_masked_sha"])
    m = _ngp(scale)  # the drop-in model computes the same grids
    m.mark_invisible_cells(sc.K.to(DEV), sc.poses.to(DEV), (sc.W, sc.H))
    assert torch.equal(m.count_grid, tr.count_grid)
    assert torch.equal(m.density_grid, tr.density_grid)


def test_grid_ema_erode_kernel_matches_torch_expression():
    g = torch.Generator().manual_seed(0)
    n = 1 << 20
    grid = torch.rand(n, generator=g) * 20
    grid[torch.rand(n, generator=g) < 0.1] = -1.0
    grid[torch.rand(n, generator=g) < 0.1] = 0.0
    count = torch.randint(0, 11, (n,), generator=g) / 10
    tmp = torch.rand(n, generator=g) * 25
    tmp[torch.rand(n, generator=g) < 0.5] = 0.0  # unsampled cells
    decay = vren.erode_decay(count)
    ref = torch.where(grid < 0, grid, torch.maximum(grid * decay, tmp))  # networks.py:273-276
    mean = ref[ref > 0].double().mean()
    gd = grid.to(DEV)
    key = torch.where(tmp > 0, (torch.arange(n, dtype=torch.int64) + 1) << 32 |
                      (tmp.view(torch.int32).to(torch.int64) & 0xFFFFFFFF), 0).to(DEV)
    sum_cnt = torch.zeros(2, dtype=torch.float64, device=DEV)
    thr = torch.zeros(2, device=DEV)
    L = vren.lib()
    vren._ok(L.ngp_density_grid_ema(gd.data_ptr(), key.data_ptr(), n, vren.c_float(0.95),
                                    decay.to(DEV).data_ptr(), vren.c_float(THR), sum_cnt.data_ptr(),
                                    thr.data_ptr(), vren._stream()), "ema")
    torch.cuda.synchronize()
    assert torch.equal(gd.cpu(), ref)
    assert int(key.abs().sum()) == 0  # consumed
    assert float(thr[1]) == pytest.approx(float(mean), rel=2 ** -23)
    assert float(thr[0]) == min(float(thr[1]), np.float32(THR))


def test_erode_chain_matches_reference_glue():
    fx = load("occupancy_erode")
    seed, amp = int(fx["seed"]), float(fx["amp"])
    fm = FixtureModel(0.5, seed, amp)
    sc = _scene(fx, 0.5)
    m = _ngp(0.5, seed, amp)
    m.mark_invisible_cells(sc.K.to(DEV), sc.poses.to(DEV), (sc.W, sc.H))
    torch.manual_seed(seed)
    log = []
    with cpu_rng_replay(log):
        m.update_density_grid(THR, warmup=True, erode=True)
        m.update_density_grid(THR, warmup=True, erode=True)
    jits = [t for _, t in log]
    cells = _flipped(m.density_bitfield.cpu().numpy(), fx["warm2_bitfield"])
    _check_flips(cells, m.density_grid, _warm_bounds(fm, cells, jits), "warm-up x2 (erode)")
    # the device trainer's update == the drop-in NGP's on the same jitter
    tr = NGPTrainer(scale=0.5, batch_size=256, sample_capacity=256 * 64, device=DEV, erode=True)
    tr.params.copy_(m.params.detach())
    tr.params16.copy_(m.params.detach().half())
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    for j in jits:
        tr.update_density_grid(THR, warmup=True, jitter=j.view(1, -1, 3))
    assert torch.equal(tr.density_grid, m.density_grid)
    assert torch.equal(tr.density_bitfield, m.density_bitfield)
    # one sampled (non-warm-up) update with the glue's draws, from the glue's occupied list
    occupied = _pin(m, fx, "warm2")
    torch.manual_seed(seed + 1)
    log2 = []
    with cpu_rng_replay(log2):
        m.update_density_grid(THR, warmup=False, erode=True)
    cells = _flipped(m.density_bitfield.cpu().numpy(), fx["upd_bitfield"])
    b = torch.maximum(_warm_bounds(fm, cells, jits), _sampled_bounds(fm, cells, log2, occupied))
    _check_flips(cells, m.density_grid, b, "sampled update (erode)")


def test_sampled_update_matches_reference_glue():
    """density_update.npz: warm-up then one sampled update (no erode)."""
    fx = load("density_update")
    seed, amp = int(fx["seed"]), float(fx["amp"])
    fm = FixtureModel(0.5, seed, amp)
    m = _ngp(0.5, seed, amp)
    torch.manual_seed(seed)
    log = []
    with cpu_rng_replay(log):
        m.update_density_grid(THR, warmup=True)
    jits = [t for _, t in log]
    cells = _flipped(m.density_bitfield.cpu().numpy(), fx["warm_bitfield"])
    _check_flips(cells, m.density_grid, _warm_bounds(fm, cells, jits), "warm-up")
    occupied = _pin(m, fx, "warm")
    torch.manual_seed(seed + 1)
    log2 = []
    with cpu_rng_replay(log2):
        m.update_density_grid(THR, warmup=False)
    got = m.density_bitfield.cpu().numpy()
    cells = _flipped(got, fx["upd_bitfield"])
    b = torch.maximum(_warm_bounds(fm, cells, jits), _sampled_bounds(fm, cells, log2, occupied))
    _check_flips(cells, m.density_grid, b, "sampled update")
    assert abs(int(np.unpackbits(got).sum()) - int(fx["upd_popcount"])) <= cells.numel()


@pytest.mark.parametrize("lo_hi", ["all", "head", "tail", "empty"])
def test_occupancy_keep_lists_each_cells_last_draw(lo_hi):
    """ngp_occupancy_keep: of a 2M-sample list shaped as the sorted sampler
    emits it (each half ascending, duplicates adjacent, some cells in both
    halves, empty-list markers -1), exactly the positions in [lo, hi) that no
    later position repeats -- the samples density_grid_tmp's last-write-wins
    keeps (networks.py:268) -- with their count; then ngp_density_scatter_kept
    over the shards [0, lo), [lo, hi), [hi, 2M) leaves the key grid
    ngp_density_scatter_last leaves over the whole list."""
    g = torch.Generator().manual_seed(7)
    G3, M, cascade = 4096, 3000, 1
    base = cascade * G3
    uni = torch.sort(torch.randint(0, G3, (M,), generator=g)).values
    occ_cells = torch.sort(torch.randperm(G3, generator=g)[:300]).values
    occ = torch.sort(occ_cells[torch.randint(0, 300, (M,), generator=g)]).values
    flat = torch.cat([uni, occ]).to(torch.int64) + base
    flat[2 * M - 5:] = -1  # (markers: skipped)
    lo, hi = {"all": (0, 2 * M), "head": (0, M + 7), "tail": (M - 5, 2 * M), "empty": (1234, 1234)}[lo_hi]
    last = {}
    for i, f in enumerate(flat.tolist()):
        if f >= 0:
            last[f] = i
    want = sorted(i for i in last.values() if lo <= i < hi)
    L = vren.lib()
    dflat = flat.to(DEV)
    mark = torch.empty(G3 // 4, dtype=torch.int32, device=DEV)
    kept = torch.full((2 * M,), -7, dtype=torch.int32, device=DEV)
    cnt = torch.full((1,), 99, dtype=torch.int64, device=DEV)
    vren._ok(L.ngp_occupancy_keep(dflat.data_ptr(), M, base, G3, lo, hi, mark.data_ptr(), kept.data_ptr(),
                                  cnt.data_ptr(), vren._stream()), "occupancy_keep")
    torch.cuda.synchronize()
    n = int(cnt.item())
    assert n == len(want)
    assert sorted(kept[:n].cpu().tolist()) == want
    # scatter: the kept samples of [0, lo), [lo, hi), [hi, 2M) (three ranks' shards, MAX-combined by
    # scattering into one key grid) == every sample of the list (the last position wins)
    sig = torch.rand(2 * M, generator=g).to(DEV)
    k_all = torch.zeros(2 * G3, dtype=torch.int64, device=DEV)
    k_kept = torch.zeros_like(k_all)
    vren._ok(L.ngp_density_scatter_last(dflat.data_ptr(), sig.data_ptr(), 2 * M, 0, k_all.data_ptr(),
                                        vren._stream()), "scatter_last")
    for a, b in ((0, lo), (lo, hi), (hi, 2 * M)):
        vren._ok(L.ngp_occupancy_keep(dflat.data_ptr(), M, base, G3, a, b, mark.data_ptr(), kept.data_ptr(),
                                      cnt.data_ptr(), vren._stream()), "occupancy_keep")
        vren._ok(L.ngp_density_scatter_kept(kept.data_ptr(), cnt.data_ptr(), b - a, dflat.data_ptr(),
                                            sig.data_ptr(), 0, k_kept.data_ptr(), vren._stream()), "scatter_kept")
    torch.cuda.synchronize()
    assert torch.equal(k_all, k_kept)


def test_trainer_update_with_kept_samples_is_bit_identical():
    """NGPTrainer's sampled occupancy update evaluating only the kept samples
    (occ_keep, the default) leaves the density grid, threshold and bitfield
    bit for bit as evaluating all 2M samples, from the same trained state."""
    sc = S.AnalyticScene(W=100, H=100, n_images=10)
    dirs, poses = sc.directions.to(DEV), sc.poses.to(DEV)
    gt_img = sc.gt_images(device=DEV)
    tr = NGPTrainer(scale=0.5, batch_size=4096, device=DEV, seed=3, warmup_steps=16)
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    for _ in range(60):
        tr.train_step(gt_img, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    state = [t.clone() for t in (tr.density_grid, tr.density_bitfield, tr.dctr, tr.threshold)]
    outs = []
    for keep in (False, True):
        for t, v in zip((tr.density_grid, tr.density_bitfield, tr.dctr, tr.threshold), state):
            t.copy_(v)
        tr.occ_keep = keep
        tr.update_density_grid(THR, warmup=False)
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (tr.density_grid, tr.density_bitfield, tr.threshold)])
        if keep:
            n_kept = int(tr._occ_kept_n.item())
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    M2 = 2 * (tr.G ** 3 // 4)
    print(f"kept {n_kept} of {M2} samples ({n_kept / M2:.3f})")
    assert 0 < n_kept < M2
    assert not torch.equal(outs[0][0], state[0])  # (the update did change the grid)


def test_update_with_its_draws_beside_the_step_is_bit_identical():
    """The captured step before an update draws the update's cells on the
    march stream beside itself (NGPTrainer._occ_draw), and the update then
    starts from those draws (update_density_grid(drawn=True)): the same grid,
    bitfield and threshold bit for bit as the update drawing them itself, from
    the same trained state."""
    sc = S.AnalyticScene(W=100, H=100, n_images=10)
    dirs, poses = sc.directions.to(DEV), sc.poses.to(DEV)
    gt_img = sc.gt_images(device=DEV)
    tr = NGPTrainer(scale=0.5, batch_size=4096, device=DEV, seed=3, warmup_steps=16)
    tr.mark_invisible_cells(sc.K, sc.poses, (sc.W, sc.H))
    for _ in range(60):
        tr.train_step(gt_img, dirs, poses)
    tr.drain()
    torch.cuda.synchronize()
    state = [t.clone() for t in (tr.density_grid, tr.density_bitfield, tr.dctr, tr.threshold)]
    outs = []
    for drawn in (False, True):
        for t, v in zip((tr.density_grid, tr.density_bitfield, tr.dctr, tr.threshold), state):
            t.copy_(v)
        cs = torch.cuda.current_stream()
        if drawn:
            tr.march_stream.wait_stream(cs)
            with torch.cuda.stream(tr.march_stream):
                tr._occ_draw(0, THR, vren._stream())
            cs.wait_stream(tr.march_stream)
        tr.update_density_grid(THR, warmup=False, drawn=drawn)
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (tr.density_grid, tr.density_bitfield, tr.threshold, tr.dctr)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert not torch.equal(outs[0][0], state[0])  # (the update did change the grid)
