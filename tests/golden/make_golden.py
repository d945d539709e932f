"""Generate the golden fixtures in tests/golden/*.npz by running the
REFERENCE's own Python glue (read from /root/reference, never copied):
models/rendering.py render (train + test), models/custom_functions.py
(RayMarcher / VolumeRenderer autograd), models/networks.py NGP
(update_density_grid), losses.py NeRFLoss -- with this repo's CPU oracle
plugged in as `vren` and as `tinycudann` (oracle.tcnn_stub), since neither
the CUDA extension nor tiny-cuda-nn can be built here (DESIGN.md "Oracle").

What this pins: the reference glue's orchestration (near clamp, noise
perturbation, slicing, background blending, loss formulas and their autograd
wiring, occupancy EMA / threshold / cell sampling) on top of the oracle's
restatement of the kernels.  Params are NOT stored: they are regenerated from
torch CPU generator seeds (tcnn_stub init + the table override below) and
checked against the stored checksums.

Run:  python tests/golden/make_golden.py   (needs /root/reference; ~1 min)
"""
import hashlib
import math
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("AR_NERF_REFERENCE", "/root/reference")
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "ar-nerf_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
import synthetic as S  # noqa: E402

NOISE_LOG = []


def install_stubs():
    vren = types.ModuleType("vren")
    for name in ("ray_aabb_intersect", "morton3D", "morton3D_invert", "packbits", "raymarching_test",
                 "composite_train_fw", "composite_train_bw", "composite_test_fw"):
        setattr(vren, name, getattr(O, name))

    def raymarching_train(*a):
        NOISE_LOG.append(a[7].detach().clone())
        return O.raymarching_train(*a)

    vren.raymarching_train = raymarching_train
    sys.modules["vren"] = vren
    tcnn = types.ModuleType("tinycudann")
    tcnn.NetworkWithInputEncoding = O.tcnn_stub.NetworkWithInputEncoding
    tcnn.Encoding = O.tcnn_stub.Encoding
    tcnn.Network = O.tcnn_stub.Network
    sys.modules["tinycudann"] = tcnn
    ts = types.ModuleType("torch_scatter")

    def segment_csr(src, indptr):
        out = torch.zeros(indptr.numel() - 1, *src.shape[1:], dtype=src.dtype)
        for i in range(indptr.numel() - 1):
            out[i] = src[indptr[i]:indptr[i + 1]].sum(0)
        return out

    ts.segment_csr = segment_csr
    sys.modules["torch_scatter"] = ts
    for name in ("open3d", "cv2", "kornia", "pyransac3d"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.path.insert(0, REF)
    # On a CUDA box `render` runs under autocast, so every custom_fwd(
    # cast_inputs=torch.float32) Function of models/custom_functions.py casts
    # its floating inputs to fp32 (e.g. TruncExp gets h[:,0] as fp32).  Autocast
    # is disabled on this CPU host, so re-apply exactly that cast.
    import models.custom_functions as cf
    for cls in (cf.RayAABBIntersector, cf.RayMarcher, cf.VolumeRenderer, cf.TruncExp):
        orig = cls.apply

        def apply(*a, _orig=orig):
            return _orig(*[x.float() if torch.is_tensor(x) and x.is_floating_point() else x for x in a])

        cls.apply = staticmethod(apply)


def table_override(model, seed, amp, sigma_gain=40.0):
    """Replace the hash table part of xyz_encoder.params by U(-amp, amp) and
    amplify the density head (row 0 of W2) so that rays become opaque and the
    T <= T_threshold early termination is exercised."""
    g = torch.Generator().manual_seed(seed)
    enc = model.xyz_encoder
    with torch.no_grad():
        n = enc.params.numel() - enc.n_mlp
        enc.params[enc.n_mlp:] = (torch.rand(n, generator=g) * 2 - 1) * amp
        enc.params[2048:2048 + 64] *= sigma_gain


def sha(t):
    return hashlib.sha256(t.detach().cpu().contiguous().numpy().tobytes()).hexdigest()


def checksum(p):
    p = p.detach().double()
    return np.array([p.sum().item(), (p * p).sum().item(), p[:8].sum().item(), p[-8:].sum().item()])


def scene_rays(W, n_rays, scale, seed):
    sc = S.AnalyticScene(W=W, H=W, n_images=10, scale=scale)
    gen = torch.Generator().manual_seed(seed)
    img, pix = sc.sample_batch(n_rays, gen)
    o, d = sc.rays(img, pix)
    return sc, o.contiguous(), d.contiguous(), sc.gt_rgb_rays(o, d)


def train_case(name, scale, esf, n_rays, amp, seed):
    from losses import NeRFLoss
    from models.networks import NGP
    from models.rendering import render
    model = NGP(scale)
    table_override(model, 100 + seed, amp)
    sc, o, d, gt = scene_rays(64, n_rays, scale, seed)
    model.density_bitfield.copy_(S.packbits_cpu(S.shell_density_grid(128, model.cascades, scale), 0.5))
    torch.manual_seed(seed)
    NOISE_LOG.clear()
    kw = {"exp_step_factor": esf} if esf > 0 else {}
    res = render(model, o, d, **kw)
    loss_d = NeRFLoss(30, "raw", scale, 0.0, lambda_distortion=0.0)(res, {"rgb": gt})
    loss = sum(v.mean() for v in loss_d.values())
    loss.backward()
    gx, gr = model.xyz_encoder.params.grad, model.rgb_net.params.grad
    nm = model.xyz_encoder.n_mlp
    gidx = torch.randint(0, gx.numel() - nm, (4096,), generator=torch.Generator().manual_seed(7))
    return {
        "case": name, "scale": scale, "esf": esf, "seed": seed, "amp": amp, "n_rays": n_rays,
        "rays_o": o.numpy(), "rays_d": d.numpy(), "gt": gt.numpy(), "noise": NOISE_LOG[0].numpy(),
        "xyz_params_ck": checksum(model.xyz_encoder.params), "rgb_params_ck": checksum(model.rgb_net.params),
        "bitfield_sha": sha(model.density_bitfield),
        "rgb": res["rgb"].detach().numpy(), "opacity": res["opacity"].detach().numpy(),
        "depth": res["depth"].detach().numpy(), "ws": res["ws"].detach().numpy(),
        "deltas": res["deltas"].numpy(), "ts": res["ts"].numpy(), "rays_a": res["rays_a"].numpy(),
        "rm_samples": int(res["rm_samples"]), "vr_samples": int(res["vr_samples"]), "loss": float(loss.detach()),
        "grad_mlp_density": gx[:nm].numpy(), "grad_rgb_net": gr.numpy(), "grad_table_idx": gidx.numpy(),
        "grad_table_vals": gx[nm:][gidx].numpy(), "grad_table_norm": float(gx[nm:].norm()),
        "grad_table_nnz": int((gx[nm:] != 0).sum()),
    }


def test_render_case(scale, amp, seed):
    from models.networks import NGP
    from models.rendering import render
    model = NGP(scale)
    table_override(model, 100 + seed, amp)
    sc = S.AnalyticScene(W=16, H=16, n_images=2, scale=scale)
    P = sc.poses[0]
    d = (sc.directions @ P[:, :3].t()).contiguous()
    o = P[:, 3].expand_as(d).contiguous()
    model.density_bitfield.copy_(S.packbits_cpu(S.shell_density_grid(128, model.cascades, scale), 0.5))
    with torch.no_grad():
        res = render(model, o, d, test_time=True)
    return {"case": "lego_test", "scale": scale, "seed": seed, "amp": amp, "rays_o": o.numpy(), "rays_d": d.numpy(),
            "rgb": res["rgb"].numpy(), "opacity": res["opacity"].numpy(), "depth": res["depth"].numpy(),
            "total_samples": int(res["total_samples"])}


def pins(grid, thr, band=0.05):
    """Cells whose density is within `band` of thr in log space, with their
    values: the sampled update resamples torch.nonzero(grid > thr), so a test
    pins these cells to the glue's values first, and the list it draws from
    is the glue's (the product's densities differ from the oracle's within the
    fp16 storage-point error bound, far below the band)."""
    g = grid.reshape(-1)
    near = (torch.log(g.clamp_min(1e-30)) - math.log(thr)).abs() < band
    idx = torch.nonzero(near)[:, 0]
    return idx.int().numpy(), g[idx].numpy()


def density_case(seed, amp):
    from models.networks import NGP
    model = NGP(0.5)
    table_override(model, 100 + seed, amp)
    G = model.grid_size
    ax = torch.arange(G, dtype=torch.int32)
    model.register_buffer("density_grid", torch.zeros(model.cascades, G ** 3))
    model.register_buffer("grid_coords", torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3))
    thr = 0.01 * 1024 / 3 ** 0.5
    out = {"case": "density_update", "seed": seed, "amp": amp}
    torch.manual_seed(seed)
    model.update_density_grid(thr, warmup=True)
    out["warm_bitfield"] = model.density_bitfield.numpy().copy()
    g = model.density_grid
    out["warm_pin_idx"], out["warm_pin_val"] = pins(g, thr)
    out["warm_grid_sha"] = sha(g)
    out["warm_mean"] = float(g[g > 0].mean())
    torch.manual_seed(seed + 1)
    model.update_density_grid(thr, warmup=False)
    out["upd_bitfield_sha"] = sha(model.density_bitfield)
    out["upd_bitfield"] = model.density_bitfield.numpy().copy()
    out["upd_popcount"] = int(np.unpackbits(model.density_bitfield.numpy()).sum())
    g = model.density_grid
    out["upd_mean"] = float(g[g > 0].mean())
    return out


def occupancy_case(seed, amp, n_cams=10, W=64, H=48):
    """mark_invisible_cells (networks.py:209-250) on a Lego-sized (scale 0.5,
    1 cascade) and a garden-sized (scale 16, 6 cascades) grid, then the erode
    occupancy chain on the Lego grid (train.py:175-178 with erode=True):
    two warm-up updates (the second one decays by the per-cell erode factor)
    and one sampled update.  Grids are stored as sha256 + summaries (the
    count grid takes n_cams+1 values: a histogram of count*n_cams); the final
    bitfields in full."""
    from models.networks import NGP
    out = {"case": "occupancy_erode", "seed": seed, "amp": amp, "n_cams": n_cams, "W": W, "H": H}
    thr = 0.01 * 1024 / 3 ** 0.5
    for tag, scale in (("lego", 0.5), ("garden", 16.0)):
        sc = S.AnalyticScene(W=W, H=H, n_images=n_cams, scale=scale)
        model = NGP(scale)
        G = model.grid_size
        ax = torch.arange(G, dtype=torch.int32)
        model.register_buffer("density_grid", torch.zeros(model.cascades, G ** 3))
        model.register_buffer("grid_coords", torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3))
        model.mark_invisible_cells(sc.K, sc.poses, (W, H))
        cg = model.count_grid
        k = torch.round(cg * n_cams).long()
        assert torch.equal(cg, (k / n_cams).float()), "count grid values are k / n_cams"
        out[f"{tag}_count_sha"] = sha(cg)  # torch CPU: k / n_cams correctly rounded
        out[f"{tag}_k_sha"] = sha(k.to(torch.uint8))  # the number of covering cameras per cell
        # cells whose projections sit on an image border / the near plane (fp64,
        # oracle.mark_borderline_cells) depend on float32 matmul order: masked
        bl = O.mark_borderline_cells(sc.K, sc.poses, (W, H), G, scale, model.cascades)
        out[f"{tag}_n_borderline"] = int(bl.sum())
        out[f"{tag}_k_masked_sha"] = sha(torch.where(bl, 255, k).to(torch.uint8))
        out[f"{tag}_mark_masked_sha"] = sha(torch.where(bl, 7.0, model.density_grid))
        out[f"{tag}_count_hist"] = torch.stack([torch.bincount(k[c], minlength=n_cams + 1)
                                                for c in range(model.cascades)]).numpy()
        out[f"{tag}_mark_sha"] = sha(model.density_grid)
        out[f"{tag}_invisible"] = (model.density_grid < 0).sum(1).numpy()
        if tag != "lego":
            continue
        table_override(model, 100 + seed, amp)
        torch.manual_seed(seed)
        model.update_density_grid(thr, warmup=True, erode=True)
        model.update_density_grid(thr, warmup=True, erode=True)
        g = model.density_grid
        out["warm2_bitfield"] = model.density_bitfield.numpy().copy()
        out["warm2_pin_idx"], out["warm2_pin_val"] = pins(g, thr)
        out["warm2_grid_sha"] = sha(g)
        out["warm2_mean"] = float(g[g > 0].mean())
        torch.manual_seed(seed + 1)
        model.update_density_grid(thr, warmup=False, erode=True)
        g = model.density_grid
        out["upd_bitfield"] = model.density_bitfield.numpy().copy()
        out["upd_grid_sha"] = sha(g)
        out["upd_mean"] = float(g[g > 0].mean())
    return out


def main():
    install_stubs()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cases = [
        train_case("lego_train", 0.5, 0.0, 256, 1.0, 1),
        train_case("garden_train", 16.0, 1 / 256, 128, 1.0, 2),
        test_render_case(0.5, 1.0, 3),
    ]
    # update_density_grid writes density_grid_tmp[c, indices] with duplicate
    # cells: torch's parallel CPU index_put_ lets threads race on them, so
    # the occupancy cases run on one thread (sequential: the last duplicate
    # in list order wins, the semantics the product reproduces)
    torch.set_num_threads(1)
    cases += [density_case(4, 1.0), occupancy_case(5, 1.0)]
    for c in cases:
        path = os.path.join(HERE, f"{c['case']}.npz")
        np.savez_compressed(path, **{k: np.asarray(v) for k, v in c.items()})
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
