"""CPU oracle for the Instant-NGP hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.  The product path (ar-nerf_amd/) never
imports it; its kernels fail loudly without the HIP library.

Layers
------
* ``vren``-shaped functions (same names/argument meaning as the pybind module
  the reference builds, models/csrc/binding.cpp:234-250) over CPU torch
  tensors, backed by oracle/vren_oracle.c (restates models/csrc/*.cu).
* tcnn-semantics hash grid / SH / fully-fused MLP (models/networks.py:33-78),
  with fp16 rounding at tcnn's storage points: params, encoding output,
  hidden activations, network outputs.  Parity for this part is UNPINNED:
  tiny-cuda-nn is not vendored by the reference and not in this container.
* ``tcnn_stub`` -- torch modules shaped like tinycudann's
  NetworkWithInputEncoding / Encoding / Network (flat ``.params``), so the
  reference's own models/networks.py can run on CPU for fixture generation.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from ctypes import POINTER, c_float, c_int, c_int64, c_uint32, c_void_p

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp = c_void_p
        L.or_ray_aabb_intersect.argtypes = [c_int, vp, vp, c_int, vp, vp, c_int, vp, vp, vp]
        L.or_morton3D.argtypes = [c_int, vp, vp]
        L.or_morton3D_invert.argtypes = [c_int, vp, vp]
        L.or_packbits.argtypes = [c_int, vp, c_float, vp]
        L.or_march_train.argtypes = [c_int, vp, vp, vp, vp, c_int, c_int, c_float, c_float, vp, c_int,
                                     vp, vp, vp, vp, vp, vp]
        L.or_march_train.restype = c_int64
        L.or_march_test.argtypes = [c_int, vp, vp, vp, vp, vp, c_int, c_int, c_float, c_float, c_int,
                                    c_int, vp, vp, vp, vp, vp]
        L.or_composite_train_fw.argtypes = [c_int, vp, vp, vp, vp, vp, c_float, vp, vp, vp, vp, vp]
        L.or_composite_train_bw.argtypes = [c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                            c_float, vp, vp]
        L.or_composite_test_fw.argtypes = [c_int, c_int, vp, vp, vp, vp, vp, c_float, vp, vp, vp, vp]
        L.or_distortion_loss_fw.argtypes = [c_int, vp, vp, vp, vp, vp, vp, vp]
        L.or_distortion_loss_bw.argtypes = [c_int, vp, vp, vp, vp, vp, vp, vp, vp]
        L.or_hash_levels.argtypes = [c_int, c_int, c_int, c_float, vp, vp, vp, vp]
        L.or_hash_levels.restype = c_uint32
        L.or_hash_encode_fwd.argtypes = [c_int, vp, vp, vp, c_int, vp, vp, vp, vp, vp, vp]
        L.or_hash_encode_bwd.argtypes = [c_int, vp, vp, vp, c_int, vp, vp, vp, vp, vp, vp]
        L.or_hash_corners.argtypes = [c_int, vp, vp, vp, c_int, vp, vp, vp, vp, vp, vp]
        L.or_sh4.argtypes = [c_int, vp, vp]
        L.or_sh4_unit01.argtypes = [c_int, vp, vp]
        L.or_adam.argtypes = [c_int64, vp, vp, vp, vp, c_float, c_float, c_float, c_float, c_float, c_float]
        L.or_calc_dt.argtypes = [c_float, c_float, c_int, c_int, c_float]
        L.or_calc_dt.restype = c_float
        L.or_mip_from_pos.argtypes = [c_float, c_float, c_float, c_int]
        L.or_mip_from_dt.argtypes = [c_float, c_int, c_int]
        L.or_f32_to_f16.argtypes = [c_float]
        L.or_f32_to_f16.restype = ctypes.c_uint16
        _lib = L
    return _lib


def _p(t: torch.Tensor):
    assert t.device.type == "cpu" and t.is_contiguous(), "oracle takes contiguous CPU tensors"
    return c_void_p(t.data_ptr())


def _c(t, dtype):
    return t.detach().to("cpu", dtype).contiguous()


# --------------------------------------------------------------- vren API
def ray_aabb_intersect(rays_o, rays_d, centers, half_sizes, max_hits):
    """intersection.cu:59-100 -> [hit_cnt i32 (N), hits_t f32 (N,max_hits,2), voxel_idx i64]"""
    o, d = _c(rays_o, torch.float32), _c(rays_d, torch.float32)
    c, h = _c(centers, torch.float32).reshape(-1, 3), _c(half_sizes, torch.float32).reshape(-1, 3)
    n, nv = o.shape[0], c.shape[0]
    cnt = torch.zeros(n, dtype=torch.int32)
    ht = torch.empty(n, max_hits, 2, dtype=torch.float32)
    hv = torch.empty(n, max_hits, dtype=torch.int64)
    lib().or_ray_aabb_intersect(n, _p(o), _p(d), nv, _p(c), _p(h), max_hits, _p(cnt), _p(ht), _p(hv))
    return [cnt, ht, hv]


def morton3D(coords):
    c = _c(coords, torch.int32)
    out = torch.empty(c.shape[0], dtype=torch.int32)
    lib().or_morton3D(c.shape[0], _p(c), _p(out))
    return out


def morton3D_invert(indices):
    i = _c(indices, torch.int32)
    out = torch.empty(i.shape[0], 3, dtype=torch.int32)
    lib().or_morton3D_invert(i.shape[0], _p(i), _p(out))
    return out


def packbits(density_grid, density_threshold, density_bitfield):
    g = _c(density_grid, torch.float32)
    out = torch.empty(density_bitfield.numel(), dtype=torch.uint8)
    lib().or_packbits(out.numel(), _p(g), float(density_threshold), _p(out))
    density_bitfield.copy_(out.view_as(density_bitfield))


def raymarching_train(rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor,
                      noise, grid_size, max_samples):
    """raymarching.cu:283-332.  Ray-ordered layout, exact-size outputs;
    counter = [total_samples, n_rays] like the reference's (2,) int32."""
    o, d = _c(rays_o, torch.float32), _c(rays_d, torch.float32)
    ht, bf, nz = _c(hits_t, torch.float32).reshape(-1, 2), _c(density_bitfield, torch.uint8), _c(noise, torch.float32)
    n = o.shape[0]
    counts = torch.empty(n, dtype=torch.int32)
    rays_a = torch.empty(n, 3, dtype=torch.int64)
    L = lib()
    args = (n, _p(o), _p(d), _p(ht), _p(bf), int(cascades), int(grid_size), float(scale),
            float(exp_step_factor), _p(nz), int(max_samples), _p(counts), _p(rays_a))
    total = L.or_march_train(*args, None, None, None, None)
    xyzs = torch.zeros(total, 3); dirs = torch.zeros(total, 3)
    deltas = torch.zeros(total); ts = torch.zeros(total)
    L.or_march_train(*args, _p(xyzs), _p(dirs), _p(deltas), _p(ts))
    counter = torch.tensor([total, n], dtype=torch.int32)
    return [rays_a, xyzs, dirs, deltas, ts, counter]


def raymarching_test(rays_o, rays_d, hits_t, alive_indices, density_bitfield, cascades, scale,
                     exp_step_factor, grid_size, max_samples, N_samples):
    """raymarching.cu:407-454; hits_t (N_rays,2) is updated IN PLACE."""
    o, d = _c(rays_o, torch.float32), _c(rays_d, torch.float32)
    ht = hits_t if (hits_t.is_contiguous() and hits_t.device.type == "cpu") else _c(hits_t, torch.float32)
    al, bf = _c(alive_indices, torch.int64), _c(density_bitfield, torch.uint8)
    n = al.shape[0]
    xyzs = torch.zeros(n, N_samples, 3); dirs = torch.zeros(n, N_samples, 3)
    deltas = torch.zeros(n, N_samples); ts = torch.zeros(n, N_samples)
    neff = torch.zeros(n, dtype=torch.int32)
    lib().or_march_test(n, _p(o), _p(d), _p(ht), _p(al), _p(bf), int(cascades), int(grid_size),
                        float(scale), float(exp_step_factor), int(N_samples), int(max_samples),
                        _p(xyzs), _p(dirs), _p(deltas), _p(ts), _p(neff))
    if ht is not hits_t:
        hits_t.copy_(ht)
    return [xyzs, dirs, deltas, ts, neff]


def composite_train_fw(sigmas, rgbs, deltas, ts, rays_a, T_threshold):
    s, c = _c(sigmas, torch.float32), _c(rgbs, torch.float32)
    dl, t, ra = _c(deltas, torch.float32), _c(ts, torch.float32), _c(rays_a, torch.int64)
    nr, N = ra.shape[0], s.shape[0]
    op, dep, rgb = torch.zeros(nr), torch.zeros(nr), torch.zeros(nr, 3)
    ws, tot = torch.zeros(N), torch.zeros(nr, dtype=torch.int64)
    lib().or_composite_train_fw(nr, _p(s), _p(c), _p(dl), _p(t), _p(ra), float(T_threshold), _p(tot),
                                _p(op), _p(dep), _p(rgb), _p(ws))
    return [tot, op, dep, rgb, ws]


def composite_train_bw(dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts,
                       rays_a, opacity, depth, rgb, T_threshold):
    f = lambda x: _c(x, torch.float32)
    a = [f(dL_dopacity), f(dL_ddepth), f(dL_drgb), f(dL_dws), f(sigmas), f(rgbs), f(ws), f(deltas),
         f(ts), _c(rays_a, torch.int64), f(opacity), f(depth), f(rgb)]
    N, nr = a[4].shape[0], a[9].shape[0]
    dsig, drgbs = torch.zeros(N), torch.zeros(N, 3)
    lib().or_composite_train_bw(nr, *[_p(x) for x in a], float(T_threshold), _p(dsig), _p(drgbs))
    return [dsig, drgbs]


def composite_test_fw(sigmas, rgbs, deltas, ts, hits_t, alive_indices, T_threshold, N_eff_samples,
                      opacity, depth, rgb):
    """volumerendering.cu:251-284; alive/opacity/depth/rgb updated in place."""
    s, c = _c(sigmas, torch.float32), _c(rgbs, torch.float32)
    dl, t, ne = _c(deltas, torch.float32), _c(ts, torch.float32), _c(N_eff_samples, torch.int32)
    n, Ns = s.shape[0], s.shape[1] if s.dim() == 2 else 1
    for x in (alive_indices, opacity, depth, rgb):
        assert x.is_contiguous() and x.device.type == "cpu"
    lib().or_composite_test_fw(n, Ns, _p(s), _p(c), _p(dl), _p(t), _p(alive_indices), float(T_threshold),
                               _p(ne), _p(opacity), _p(depth), _p(rgb))


def distortion_loss_fw(ws, deltas, ts, rays_a):
    """losses.cu:62-107 -> [loss (N_rays), ws_inclusive_scan (N), wts_inclusive_scan (N)]"""
    w, dl, t, ra = (_c(ws, torch.float32), _c(deltas, torch.float32), _c(ts, torch.float32),
                    _c(rays_a, torch.int64))
    nr, N = ra.shape[0], w.shape[0]
    loss, wsi, wtsi = torch.zeros(nr), torch.zeros(N), torch.zeros(N)
    lib().or_distortion_loss_fw(nr, _p(w), _p(dl), _p(t), _p(ra), _p(loss), _p(wsi), _p(wtsi))
    return [loss, wsi, wtsi]


def distortion_loss_bw(dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a):
    """losses.cu:143-173 -> dL_dws (N)"""
    f = lambda x: _c(x, torch.float32)
    a = [f(dL_dloss), f(ws_inclusive_scan), f(wts_inclusive_scan), f(ws), f(deltas), f(ts), _c(rays_a, torch.int64)]
    dws = torch.zeros(a[3].shape[0])
    lib().or_distortion_loss_bw(a[6].shape[0], *[_p(x) for x in a], _p(dws))
    return dws


# ------------------------------------------------ tcnn-semantics hash grid
class HashGridSpec:
    """Level table of the multires hash grid (models/networks.py:33-49)."""

    def __init__(self, n_levels=16, log2_T=19, base_resolution=16, per_level_scale=None, scale=0.5):
        if per_level_scale is None:
            per_level_scale = float(np.exp(np.log(2048 * scale / base_resolution) / (n_levels - 1)))
        self.L, self.log2_T, self.N_min, self.b = n_levels, log2_T, base_resolution, per_level_scale
        self.scales = torch.empty(n_levels, dtype=torch.float32)
        self.res = torch.empty(n_levels, dtype=torch.int32)
        self.offsets = torch.empty(n_levels + 1, dtype=torch.int32)
        self.sizes = torch.empty(n_levels, dtype=torch.int32)
        self.n_entries = int(lib().or_hash_levels(n_levels, log2_T, base_resolution, float(per_level_scale),
                                                  _p(self.scales), _p(self.res), _p(self.offsets), _p(self.sizes)))

    def _args(self):
        return (self.L, _p(self.scales), _p(self.res), _p(self.offsets), _p(self.sizes))


def f16_bits(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.float16).view(torch.int16)


def hash_encode_fwd(spec: HashGridSpec, x, xyz_min, xyz_max, table_f32):
    """(N,3) world xyz -> (N, 2L) fp16 encoding (tcnn Grid/Hash/Linear)."""
    xx = _c(x, torch.float32); mn = _c(xyz_min, torch.float32).reshape(3); mx = _c(xyz_max, torch.float32).reshape(3)
    tab = f16_bits(_c(table_f32, torch.float32)).contiguous()
    enc = torch.empty(xx.shape[0], 2 * spec.L, dtype=torch.int16)
    lib().or_hash_encode_fwd(xx.shape[0], _p(xx), _p(mn), _p(mx), *spec._args(), _p(tab), _p(enc))
    return enc.view(torch.float16)


def hash_encode_bwd(spec: HashGridSpec, x, xyz_min, xyz_max, denc):
    xx = _c(x, torch.float32); mn = _c(xyz_min, torch.float32).reshape(3); mx = _c(xyz_max, torch.float32).reshape(3)
    g = _c(denc, torch.float32)
    dtab = torch.zeros(spec.n_entries * 2, dtype=torch.float32)
    lib().or_hash_encode_bwd(xx.shape[0], _p(xx), _p(mn), _p(mx), *spec._args(), _p(g), _p(dtab))
    return dtab


def hash_corners(spec: HashGridSpec, x, xyz_min, xyz_max):
    xx = _c(x, torch.float32); mn = _c(xyz_min, torch.float32).reshape(3); mx = _c(xyz_max, torch.float32).reshape(3)
    n = xx.shape[0]
    idx = torch.empty(n, spec.L, 8, dtype=torch.int32); w = torch.empty(n, spec.L, 8)
    lib().or_hash_corners(n, _p(xx), _p(mn), _p(mx), *spec._args(), _p(idx), _p(w))
    return idx, w


def sh4(dirs):
    d = _c(dirs, torch.float32)
    out = torch.empty(d.shape[0], 16, dtype=torch.int16)
    lib().or_sh4(d.shape[0], _p(d), _p(out))
    return out.view(torch.float16)


def sh4_unit01(d01):
    d = _c(d01, torch.float32)
    out = torch.empty(d.shape[0], 16, dtype=torch.int16)
    lib().or_sh4_unit01(d.shape[0], _p(d), _p(out))
    return out.view(torch.float16)


def adam_(p, g, m, v, lr, step, b1=0.9, b2=0.999, eps=1e-15):
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    lib().or_adam(p.numel(), _p(p), _p(g), _p(m), _p(v), lr, b1, b2, eps, bc1, bc2)


# --------------------------------------------------- fp16-point MLP oracle
class _RoundHalf(torch.autograd.Function):
    """Round to fp16 in the forward, identity gradient (tcnn's fp16 storage)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.float16).to(torch.float32)

    @staticmethod
    def backward(ctx, g):
        return g


rh = _RoundHalf.apply


class _RoundGrad16(torch.autograd.Function):
    """Identity in the forward; in the backward the gradient rounded to fp16's
    11 significant bits (round to nearest even) over an unbounded exponent
    range.  This is where tcnn's fused MLP backward stores a layer's gradient
    in fp16 (the pre-activation gradient of every layer, ReLU' applied), at a
    power-of-two scale that keeps it in fp16's normal range -- a power-of-two
    scale is exact, so the rounding is the mantissa's alone.  The product's
    MLP backward (field.hip field_bwd_mlp_coop_kernel) rounds at the same five
    points with per-sample power-of-two scales."""

    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        m, e = torch.frexp(g)
        return torch.ldexp(torch.round(m * 2048.0) / 2048.0, e.to(g.dtype))


rg16 = _RoundGrad16.apply


def mlp_layers(params, dims):
    """Split flat params into row-major [out][in] weight matrices."""
    Ws, o = [], 0
    for i in range(len(dims) - 1):
        n = dims[i + 1] * dims[i]
        Ws.append(params[o:o + n].view(dims[i + 1], dims[i]))
        o += n
    return Ws, o


def mlp_forward(x16, Ws, out_act=None, grad16=False):
    """FullyFusedMLP: ReLU hidden, fp32 accumulate, fp16 at every layer output.
    grad16: the backward stores each layer's pre-activation gradient in fp16
    (rg16), tcnn's backward storage points; default: fp32 autograd throughout."""
    h = x16.float()
    for i, W in enumerate(Ws):
        z = h @ rh(W).t()
        h = rh(rg16(z) if grad16 else z)
        if i < len(Ws) - 1:
            h = torch.relu(h)
    if out_act == "Sigmoid":
        h = rh(torch.sigmoid(h))
    return h


U32 = 2.0 ** -24  # fp32 unit roundoff


def ulp16(v):
    """fp16 ulp at |v| (2^-24 in the subnormal range)."""
    a = v.abs().clamp_min(2.0 ** -14)
    return torch.exp2(torch.floor(torch.log2(a)) - 10)


def mlp_forward_bound(x16, Ws, d_in=None):
    """mlp_forward (ReLU hidden, no output activation) plus, per output, a
    bound on |out - out'| for ANY implementation with the same fp16 storage
    points (fp16 weights and layer outputs) that accumulates each dot
    product in fp32 in any order (e.g. MFMA tiles vs this oracle's GEMM):
    products of fp16 operands are exact in fp32; a length-n fp32 sum is off
    by at most gamma_n * sum|terms| (gamma_n = n u / (1 - n u)); an error d
    in a layer's inputs moves its outputs by at most |W| d; rounding to fp16
    then adds at most one fp16 ulp (the two values may straddle a rounding
    boundary); ReLU is 1-Lipschitz.  d_in: a bound on the inputs' own error
    (default exact).  Returns (out, bound), both fp32."""
    h = x16.float()
    d = torch.zeros_like(h) if d_in is None else d_in.float()
    for i, W in enumerate(Ws):
        W16 = rh(W.detach()).float()
        n = W16.shape[1]
        gam = n * U32 / (1 - n * U32)
        z = h @ W16.t()
        dz = d @ W16.abs().t() + gam * (h.abs() @ W16.abs().t())
        if i < len(Ws) - 1:
            z = torch.relu(z)
        hn = rh(z)
        d = dz + ulp16(z.abs() + dz)
        h = hn
    return h, d


# density net 32->64->16, color net 32->64->64->16(pad; 3 used)
DENSITY_DIMS = (32, 64, 16)  # the reference's (networks.py:51-57, 68-78)
COLOR_DIMS = (32, 64, 64, 16)


def xavier_mlp(dims, gen):
    out = []
    for i in range(len(dims) - 1):
        a = math.sqrt(6.0 / (dims[i] + dims[i + 1]))
        out.append((torch.rand(dims[i + 1] * dims[i], generator=gen) * 2 - 1) * a)
    return torch.cat(out)


class _HashEncodeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, x, spec, xyz_min, xyz_max):
        ctx.save_for_backward(x)
        ctx.spec, ctx.mn, ctx.mx = spec, xyz_min, xyz_max
        return hash_encode_fwd(spec, x, xyz_min, xyz_max, table).float()

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return hash_encode_bwd(ctx.spec, x, ctx.mn, ctx.mx, g), None, None, None, None


class OracleNGPField(torch.nn.Module):
    """CPU oracle of NGP.density / NGP.forward (models/networks.py:95-165) with
    tcnn semantics; flat params like the tcnn torch modules:
      xyz_params = [W1 (w x in), W2 (16 x w), hash table (entries x 2)]
      rgb_params = [W3 (w x 32), W4 (w x w), W5 (16 x w)]
    w = width (64 in the reference, networks.py:54,75), in = 2 L padded to a
    multiple of 16 (tcnn's FullyFusedMLP input granularity; the padded
    encoding dims hold 1.0, tcnn's padding value -- parity unpinned: only
    BASELINE config 1, L = 4, w = 32, pads: 8 -> 16)."""

    def __init__(self, scale=0.5, n_levels=16, log2_T=19, base_resolution=16, seed=4,
                 table_init=1e-4, width=64):
        super().__init__()
        self.scale, self.width = scale, width
        self.spec = HashGridSpec(n_levels, log2_T, base_resolution, scale=scale)
        self.n_in = (2 * n_levels + 15) // 16 * 16
        self.dens_dims = (self.n_in, width, 16)
        self.color_dims = (32, width, width, 16)
        self.register_buffer("xyz_min", -torch.ones(1, 3) * scale)
        self.register_buffer("xyz_max", torch.ones(1, 3) * scale)
        gen = torch.Generator().manual_seed(seed)
        dens = xavier_mlp(self.dens_dims, gen)
        table = (torch.rand(self.spec.n_entries * 2, generator=gen) * 2 - 1) * table_init
        col = xavier_mlp(self.color_dims, gen)
        self.xyz_params = torch.nn.Parameter(torch.cat([dens, table]))
        self.rgb_params = torch.nn.Parameter(col)
        self.n_dens = dens.numel()
        self.grad16 = False  # True: the MLP backward's fp16 gradient storage points (mlp_forward)

    def density_feat(self, x):
        Ws, _ = mlp_layers(self.xyz_params[:self.n_dens], self.dens_dims)
        table = self.xyz_params[self.n_dens:]
        enc = _HashEncodeFn.apply(table, x, self.spec, self.xyz_min, self.xyz_max)
        if enc.shape[1] < self.n_in:  # tcnn pads the encoding to the MLP's input width with ones
            enc = torch.cat([enc, torch.ones(enc.shape[0], self.n_in - enc.shape[1], dtype=enc.dtype)], 1)
        h = mlp_forward(enc, Ws, grad16=self.grad16)
        return h

    def density(self, x, return_feat=False):
        h = self.density_feat(x)
        sig = TruncExpCPU.apply(h[:, 0])
        return (sig, h) if return_feat else sig

    def forward(self, x, d):
        sig, h = self.density(x, return_feat=True)
        sh = sh4(d).float()
        Ws, _ = mlp_layers(self.rgb_params, self.color_dims)
        out = mlp_forward(torch.cat([sh, h], 1), Ws, grad16=self.grad16)
        rgb = rh(torch.sigmoid(out[:, :3]))
        return sig, rgb


def density_input_grad(xyz_params, n_dens, spec: "HashGridSpec", x, xyz_min, xyz_max):
    """d sigma / d x of NGP.density (models/networks.py:95-108) for
    render_surface_normal (models/rendering.py:300-313), by fp32 autograd:
    trilinear weights of tcnn's grid encoding as functions of x (corner
    indices from or_hash_corners), fp16 table / weights, the encoding's VALUE
    taken bit-exact from or_hash_encode_fwd (straight-through), fp16 storage
    points in the MLP, TruncExp.backward's clamp.  tcnn's own input-gradient
    arithmetic is not available here: parity unpinned."""
    x = _c(x, torch.float32)
    mn, mx = xyz_min.reshape(1, 3).float(), xyz_max.reshape(1, 3).float()
    idx, _ = hash_corners(spec, x, mn, mx)
    table = xyz_params[n_dens:].detach().half().float().view(-1, 2)
    enc_exact = hash_encode_fwd(spec, x, mn, mx, xyz_params[n_dens:].detach()).float()
    xg = x.clone().requires_grad_(True)
    x01 = (xg - mn) / (mx - mn)
    feats = []
    for l in range(spec.L):
        p = x01 * float(spec.scales[l]) + 0.5
        f = p - torch.floor(p).detach()
        w = []
        for c in range(8):
            wc = 1.0
            for d in range(3):
                wc = wc * (f[:, d] if (c >> d) & 1 else 1 - f[:, d])
            w.append(wc)
        w = torch.stack(w, 1)  # (n, 8)
        vals = table[idx[:, l, :].long()]  # (n, 8, 2); or_hash_corners returns global entries
        feats.append((w[:, :, None] * vals).sum(1))
    enc = torch.cat(feats, 1)
    enc = enc_exact + (enc - enc.detach())
    Ws, _ = mlp_layers(xyz_params[:n_dens].detach(), (2 * spec.L, 64, 16))
    h = mlp_forward(enc, Ws)
    sig = TruncExpCPU.apply(h[:, 0])
    return torch.autograd.grad(sig.sum(), xg)[0]


class TruncExpCPU(torch.autograd.Function):
    """custom_functions.py:162-173"""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.exp(x)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * torch.exp(x.clamp(-15, 15))


# ------------------------------------------------------------ tcnn stub
class tcnn_stub:
    """Module-shaped like `tinycudann` for importing the reference's
    models/networks.py on CPU (fixture generation only)."""

    class NetworkWithInputEncoding(torch.nn.Module):
        def __init__(self, n_input_dims, n_output_dims, encoding_config, network_config, seed=4):
            super().__init__()
            ec = encoding_config
            L = ec["n_levels"]
            self.spec = HashGridSpec(L, ec["log2_hashmap_size"], ec["base_resolution"], ec["per_level_scale"])
            gen = torch.Generator().manual_seed(seed)
            dims = (2 * L,) + (network_config["n_neurons"],) * network_config["n_hidden_layers"] + (n_output_dims,)
            self.dims = dims
            mlp = xavier_mlp(dims, gen)
            self.n_mlp = mlp.numel()
            table = (torch.rand(self.spec.n_entries * 2, generator=gen) * 2 - 1) * 1e-4
            self.params = torch.nn.Parameter(torch.cat([mlp, table]))
            self.register_buffer("_mn", torch.zeros(3))
            self.register_buffer("_mx", torch.ones(3))

        def forward(self, x01):
            Ws, _ = mlp_layers(self.params[:self.n_mlp], self.dims)
            enc = _HashEncodeFn.apply(self.params[self.n_mlp:], x01.float().contiguous(), self.spec,
                                      self._mn, self._mx)
            return mlp_forward(enc, Ws).half()

    class Encoding(torch.nn.Module):
        def __init__(self, n_input_dims, encoding_config):
            super().__init__()
            assert encoding_config["otype"] == "SphericalHarmonics" and encoding_config["degree"] == 4
            self.register_parameter("params", None)

        def forward(self, d01):
            return sh4_unit01(d01).half()

    class Network(torch.nn.Module):
        def __init__(self, n_input_dims, n_output_dims, network_config, seed=5):
            super().__init__()
            gen = torch.Generator().manual_seed(seed)
            dims = (n_input_dims,) + (network_config["n_neurons"],) * network_config["n_hidden_layers"] + (16,)
            self.dims, self.n_out, self.act = dims, n_output_dims, network_config["output_activation"]
            self.params = torch.nn.Parameter(xavier_mlp(dims, gen))

        def forward(self, x):
            Ws, _ = mlp_layers(self.params, self.dims)
            out = mlp_forward(x.float(), Ws)[:, :self.n_out]
            if self.act == "Sigmoid":
                out = rh(torch.sigmoid(out))
            return out.half()


# ------------------------------------------------ CPU training step (baseline)
class _VolumeRendererCPU(torch.autograd.Function):
    """custom_functions.py:115-159 on the oracle kernels."""

    @staticmethod
    def forward(ctx, sigmas, rgbs, deltas, ts, rays_a, T_threshold):
        tot, op, dep, rgb, ws = composite_train_fw(sigmas, rgbs, deltas, ts, rays_a, T_threshold)
        ctx.save_for_backward(sigmas, rgbs, deltas, ts, rays_a, op, dep, rgb, ws)
        ctx.T = T_threshold
        return tot.sum(), op, dep, rgb, ws

    @staticmethod
    def backward(ctx, dtot, dop, ddep, drgb, dws):
        sigmas, rgbs, deltas, ts, rays_a, op, dep, rgb, ws = ctx.saved_tensors
        dsig, drgbs = composite_train_bw(dop, ddep, drgb, dws, sigmas, rgbs, ws, deltas, ts, rays_a, op, dep, rgb,
                                         ctx.T)
        return dsig, drgbs, None, None, None, None


def nerf_loss_raw(rgb, gt, opacity, lambda_opacity=1e-3):
    """losses.py:63-82 with the default 'raw' rgb loss and depth weight 0."""
    d_rgb = ((rgb - gt) / (rgb.detach() + 1e-3)) ** 2
    o = opacity + 1e-10
    d_op = lambda_opacity * (-o * torch.log(o))
    return d_rgb.mean() + d_op.mean()


class OracleTrainer:
    """One reference training step (train.py:174-200 + FusedAdam) on the CPU
    oracle: march (C), field (torch MLP with fp16 storage points + C hash),
    VolumeRenderer fw/bw (C), NeRFLoss (torch), autograd, Adam (C)."""

    def __init__(self, flat_params, scale, bitfield, cascades, grid_size=128, lr=1e-2, n_levels=16, width=64,
                 seed=4, table_init=0.0):
        """flat_params: the product's flat layout [W1 W2 | W3 W4 W5 | table],
        or None to train the oracle field's own initialisation (any L / width:
        BASELINE config 1 runs L = 4, width 32 on the CPU only)."""
        self.field = OracleNGPField(scale=scale, table_init=table_init, n_levels=n_levels, width=width, seed=seed)
        nd = self.field.n_dens
        self.n_mlp = nd + self.field.rgb_params.numel()
        if flat_params is not None:
            flat = flat_params.detach().float().cpu()
            with torch.no_grad():
                self.field.xyz_params.copy_(torch.cat([flat[:nd], flat[self.n_mlp:]]))
                self.field.rgb_params.copy_(flat[nd:self.n_mlp])
        self.scale, self.cascades, self.G, self.lr = scale, cascades, grid_size, lr
        self.bitfield = bitfield.cpu().contiguous()
        self.state = {p: (torch.zeros_like(p), torch.zeros_like(p)) for p in (self.field.xyz_params,
                                                                             self.field.rgb_params)}
        self.t = 0

    def flat_grad(self):
        nd = self.field.n_dens
        gx, gr = self.field.xyz_params.grad, self.field.rgb_params.grad
        return torch.cat([gx[:nd], gr, gx[nd:]])

    def flat_params(self):
        nd = self.field.n_dens
        px, pr = self.field.xyz_params.detach(), self.field.rgb_params.detach()
        return torch.cat([px[:nd], pr, px[nd:]])

    def step(self, rays_o, rays_d, hits_t, rgb_gt, noise, bg, apply_adam=True):
        rays_a, xyzs, dirs, deltas, ts, cnt = raymarching_train(rays_o, rays_d, hits_t, self.bitfield, self.cascades,
                                                                self.scale, 0.0, noise, self.G, 1024)
        sig, rgbs = self.field(xyzs, dirs)
        vr, op, dep, rgb, ws = _VolumeRendererCPU.apply(sig, rgbs.contiguous(), deltas, ts, rays_a, 1e-4)
        rgb = rgb + bg * (1 - op)[:, None]
        loss = nerf_loss_raw(rgb, rgb_gt, op)
        for p in self.state:
            p.grad = None
        loss.backward()
        self.last = dict(rays_a=rays_a, rgb=rgb.detach(), opacity=op.detach(), depth=dep.detach(), vr=int(vr))
        if not apply_adam:
            return float(loss.detach()), int(cnt[0])
        self.t += 1
        for p, (m, v) in self.state.items():
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            adam_(p.data, g.contiguous(), m, v, self.lr, self.t)
        return float(loss.detach()), int(cnt[0])


def mark_borderline_cells(K, poses, img_wh, grid_size, scale, cascades, near=0.01, rel=1e-5):
    """(cascades, G^3) bool in Morton order: cells whose projection into some
    camera lies within `rel` (relative, float64) of an image border, of the
    near plane or of the camera plane -- there mark_invisible_cells'
    in_image / covered tests (models/networks.py:229-248) depend on the last
    bits of a float32 matmul whose summation order differs between devices
    and BLAS builds; everywhere else they are decided with a margin.
    Test infrastructure (tests/test_occupancy_gpu.py, make_golden.py)."""
    G = grid_size
    W, H = img_wh
    ax = torch.arange(G, dtype=torch.int64)
    coords = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)
    idx = morton3D(coords.int()).long()
    P = poses.double()
    R = P[:, :3, :3].transpose(1, 2)
    T = -R @ P[:, :3, 3:]
    Kd = K.double()
    out = torch.zeros(cascades, G ** 3, dtype=torch.bool)
    for c in range(cascades):
        s = min(2 ** (c - 1), scale)
        hgs = s / G
        for i in range(0, G ** 3, 1 << 18):
            x = (coords[i:i + (1 << 18)].double() / (G - 1) * 2 - 1) * (s - hgs)
            uvd = Kd @ (R @ x.T + T)  # (N_cams, 3, chunk)
            dd = uvd[:, 2]
            uv = uvd[:, :2] / torch.where(dd == 0, torch.full_like(dd, 1e-300), dd)[:, None]
            bu = torch.minimum(uv[:, 0].abs(), (uv[:, 0] - W).abs()) / W
            bv = torch.minimum(uv[:, 1].abs(), (uv[:, 1] - H).abs()) / H
            scale_d = 1 + dd.abs()
            b = (bu < rel) | (bv < rel) | ((dd - near).abs() < rel * scale_d) | (dd.abs() < rel * scale_d)
            out[c, idx[i:i + (1 << 18)]] = b.any(0)
    return out
