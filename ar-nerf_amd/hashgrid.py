"""Hash-grid + fused-MLP field on MI355X (replaces tinycudann as used by
models/networks.py:37-78 of the reference).

Parameters follow tcnn's flat-params model, but as ONE fp32 master buffer
    params = [W1 64x32 | W2 16x64 | W3 64x32 | W4 64x64 | W5 16x64 | table (entries x 2)]
(W* row-major [out][in]; W1,W2 = xyz_encoder's MLP, W3..W5 = rgb_net, W5
rows 3..15 padding) and an fp16 shadow of the same layout that the kernels
read (tcnn keeps the same fp32-master / fp16-compute split).  The shadow is
refreshed lazily whenever the master's version counter changes.

All compute goes through libngp_amd.so; nothing here runs on the CPU.
"""
from __future__ import annotations

import ctypes
import math
from ctypes import c_float, c_int, c_int64, c_uint32, c_void_p

import numpy as np
import torch

import vren

N_LEVELS = 16
MLP_PARAMS = 10240
OW = {"W1": (0, 64, 32), "W2": (2048, 16, 64), "W3": (3072, 64, 32), "W4": (5120, 64, 64), "W5": (9216, 16, 64)}


class ngp_hashgrid_t(ctypes.Structure):
    _fields_ = [("n_levels", c_int), ("scales", c_float * 16), ("res", c_uint32 * 16), ("offsets", c_uint32 * 17),
                ("sizes", c_uint32 * 16), ("xyz_min", c_float * 3), ("xyz_max", c_float * 3)]


_declared = False


def _lib():
    global _declared
    L = vren.lib()
    if not _declared:
        vp = c_void_p
        P = ctypes.POINTER(ngp_hashgrid_t)
        L.ngp_field_forward.argtypes = [vp, vp, c_int64, vp, P, vp, vp, vp, vp, vp, vp, vp]
        L.ngp_density_forward.argtypes = [vp, c_int64, vp, P, vp, vp, vp, vp, vp]
        L.ngp_density_input_grad.argtypes = [vp, c_int64, P, vp, vp, vp, vp, vp]
        L.ngp_field_backward.argtypes = [vp, vp, c_int64, vp, P, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ngp_field_backward_mlp.argtypes = [vp, c_int64, vp, vp, vp, c_int64, vp, vp, vp, vp, vp, vp]
        L.ngp_hash_encode.argtypes = [vp, c_int64, vp, vp, P, vp, vp, vp]
        L.ngp_field_forward_indexed.argtypes = [vp, vp, c_int64, vp, vp, P, vp, vp, vp, vp, vp, vp]
        L.ngp_field_mlp_forward.argtypes = [vp, vp, c_int64, vp, vp, vp, vp, vp, vp, vp]
        L.ngp_field_encode_mlp.argtypes = [vp, vp, c_int64, vp, vp, P, vp, vp, vp, vp, vp, vp, vp]
        L.ngp_field_forward_first.argtypes = [vp, vp, vp, vp, vp, vp, c_int64, c_int64, c_float, P, vp, vp, vp, vp, vp,
                                              vp, vp, vp, vp, vp]
        L.ngp_field_forward_first_pre.argtypes = [vp, vp, vp, vp, vp, vp, c_int64, c_int64, c_float, P, vp, vp, vp,
                                                  vp, vp, vp, vp, vp, vp, c_int, vp]
        L.ngp_field_encode_first_coarse.argtypes = [vp, vp, vp, vp, c_int64, c_int64, P, vp, vp, vp]
        L.ngp_hash_backward.argtypes = [vp, c_int64, vp, vp, P, vp, vp, vp]
        L.ngp_hash_backward_binned.argtypes = [vp, c_int64, vp, vp, P, vp, vp, vp, c_int64, c_int, c_int, vp]
        L.ngp_hash_backward_levels.argtypes = [vp, c_int64, vp, vp, P, vp, vp, c_int, c_int, vp]
        L.ngp_hash_backward_levels_rep.argtypes = [vp, c_int64, vp, vp, P, vp, vp, c_int, c_int, vp, c_int, c_int, c_int,
                                                   vp]
        L.ngp_hash_backward_rep_floats.argtypes = [P, c_int, c_int]
        L.ngp_hash_backward_rep_floats.restype = ctypes.c_size_t
        L.ngp_hash_binned_plan.argtypes = [vp, c_int64, vp, vp, P, vp, c_int64, c_int, c_int, vp]
        L.ngp_hash_binned_apply.argtypes = [vp, c_int64, vp, vp, P, vp, vp, vp, c_int64, c_int, c_int, vp]
        L.ngp_hash_binned_write.argtypes = [vp, c_int64, vp, vp, P, vp, vp, vp, c_int64, c_int, c_int, vp]
        L.ngp_hash_binned_accum.argtypes = [P, vp, vp, c_int64, c_int, c_int, vp]
        L.ngp_hash_binned_accum_levels.argtypes = [P, vp, vp, c_int64, c_int, c_int, c_int, c_int, vp]
        L.ngp_hash_binned_apply_adam.argtypes = [vp, c_int64, vp, vp, P, vp, vp, vp, c_int64, c_int, c_int, vp, vp, vp,
                                                 vp, vp, c_float, c_float, c_float, vp, c_float, vp]
        L.ngp_hash_binned_accum_adam.argtypes = [P, vp, vp, c_int64, c_int, c_int, vp, vp, vp, vp, vp, c_float, c_float,
                                                 c_float, vp, c_float, vp]
        L.ngp_hash_backward_binned_workspace.argtypes = [c_int64]
        L.ngp_hash_backward_binned_workspace.restype = ctypes.c_size_t
        for f in (L.ngp_field_forward, L.ngp_density_forward, L.ngp_density_input_grad, L.ngp_field_backward, L.ngp_field_backward_mlp,
                  L.ngp_hash_encode, L.ngp_field_mlp_forward, L.ngp_field_forward_indexed, L.ngp_field_encode_mlp,
                  L.ngp_hash_backward, L.ngp_hash_backward_binned, L.ngp_hash_backward_levels,
                  L.ngp_hash_backward_levels_rep,
                  L.ngp_hash_binned_plan, L.ngp_hash_binned_apply, L.ngp_hash_binned_write,
                  L.ngp_hash_binned_accum, L.ngp_hash_binned_accum_levels, L.ngp_hash_binned_apply_adam,
                  L.ngp_hash_binned_accum_adam):
            f.restype = c_int
        _declared = True
    return L


def _ptr(t):
    return c_void_p(t.data_ptr()) if t is not None else None


class HashGrid:
    """Level table for the reference's encoding config (models/networks.py:33-49)."""

    def __init__(self, scale: float, n_levels=16, log2_T=19, base_resolution=16, per_level_scale=None):
        if per_level_scale is None:
            per_level_scale = float(np.exp(np.log(2048 * scale / base_resolution) / (n_levels - 1)))
        self.scale, self.n_levels, self.log2_T = scale, n_levels, log2_T
        self.base_resolution, self.per_level_scale = base_resolution, per_level_scale
        d = ngp_hashgrid_t()
        d.n_levels = n_levels
        self.n_entries = int(vren.lib().ngp_hashgrid_levels(n_levels, log2_T, base_resolution, c_float(per_level_scale),
                                                            ctypes.cast(d.scales, c_void_p),
                                                            ctypes.cast(d.res, c_void_p),
                                                            ctypes.cast(d.offsets, c_void_p),
                                                            ctypes.cast(d.sizes, c_void_p)))
        for i in range(3):
            d.xyz_min[i] = -scale
            d.xyz_max[i] = scale
        self.desc = d

    @property
    def resolutions(self):
        return list(self.desc.res)[: self.n_levels]

    @property
    def offsets(self):
        return list(self.desc.offsets)[: self.n_levels + 1]

    @property
    def n_params(self):
        return MLP_PARAMS + 2 * self.n_entries


def init_params(grid: HashGrid, seed=4, table_init=1e-4, device="cuda"):
    """tcnn init: hash table U(-1e-4, 1e-4); MLPs Xavier-uniform per matrix."""
    g = torch.Generator().manual_seed(seed)
    parts = []
    for name in ("W1", "W2", "W3", "W4", "W5"):
        _, out_d, in_d = OW[name]
        a = math.sqrt(6.0 / (in_d + out_d))
        parts.append((torch.rand(out_d * in_d, generator=g) * 2 - 1) * a)
    parts.append((torch.rand(2 * grid.n_entries, generator=g) * 2 - 1) * table_init)
    return torch.cat(parts).to(device)


def _check(x, name, dtype, numel=None):
    vren._check(name, x, dtype)
    if numel is not None and x.numel() != numel:
        raise RuntimeError(f"{name} must have {numel} elements, got {x.numel()}")


def field_forward(xyzs, dirs, grid: HashGrid, params16, save_enc=True, n_dev=None, want_h=False):
    """Fused NGP.forward (models/networks.py:133-146) -> sigmas (n), rgbs (n,3), enc (n,32) fp16 | None, h | None"""
    n = xyzs.shape[0]
    dev = xyzs.device
    _check(xyzs, "xyzs", torch.float32); _check(dirs, "dirs", torch.float32)
    _check(params16, "params16", torch.float16, grid.n_params)
    sig = torch.empty(n, device=dev)
    rgb = torch.empty(n, 3, device=dev)
    enc = torch.empty(n, 32, dtype=torch.float16, device=dev) if save_enc else None
    h = torch.empty(n, 16, dtype=torch.float16, device=dev) if want_h else None
    st = _lib().ngp_field_forward(_ptr(xyzs), _ptr(dirs), n, _ptr(n_dev), ctypes.byref(grid.desc),
                                  _ptr(params16[MLP_PARAMS:]), _ptr(params16), _ptr(sig), _ptr(rgb), _ptr(enc),
                                  _ptr(h), vren._stream())
    vren._ok(st, "ngp_field_forward")
    return sig, rgb, enc, h


def density_forward(xyzs, grid: HashGrid, params16, want_h=False, n_dev=None):
    """NGP.density (models/networks.py:95-108) -> sigmas (n), h (n,16) fp16 | None"""
    n = xyzs.shape[0]
    _check(xyzs, "xyzs", torch.float32)
    _check(params16, "params16", torch.float16, grid.n_params)
    sig = torch.empty(n, device=xyzs.device)
    h = torch.empty(n, 16, dtype=torch.float16, device=xyzs.device) if want_h else None
    st = _lib().ngp_density_forward(_ptr(xyzs), n, _ptr(n_dev), ctypes.byref(grid.desc), _ptr(params16[MLP_PARAMS:]),
                                    _ptr(params16), _ptr(sig), _ptr(h), vren._stream())
    vren._ok(st, "ngp_density_forward")
    return sig, h


def density_input_grad(xyzs, grid: HashGrid, params16, dL_dsigma=None):
    """dL/dx (n,3) of NGP.density through hash grid + density MLP + TruncExp
    (dL_dsigma None = ones: d sigma / d x, render_surface_normal)."""
    n = xyzs.shape[0]
    _check(xyzs, "xyzs", torch.float32)
    _check(params16, "params16", torch.float16, grid.n_params)
    if dL_dsigma is not None:
        _check(dL_dsigma, "dL_dsigma", torch.float32)
    out = torch.empty(n, 3, device=xyzs.device)
    st = _lib().ngp_density_input_grad(_ptr(xyzs), n, ctypes.byref(grid.desc), _ptr(params16[MLP_PARAMS:]),
                                       _ptr(params16), _ptr(dL_dsigma), _ptr(out), vren._stream())
    vren._ok(st, "ngp_density_input_grad")
    return out


def field_backward(xyzs, dirs, grid: HashGrid, params16, enc, dL_dsig, dL_drgb, grad, n_dev=None, denc_ws=None):
    """Accumulates dL/dparams (fp32, params layout) into `grad`."""
    n = xyzs.shape[0]
    _check(grad, "grad", torch.float32, grid.n_params)
    _check(enc, "enc", torch.float16)
    _check(dL_dsig, "dL_dsigmas", torch.float32); _check(dL_drgb, "dL_drgbs", torch.float32)
    if denc_ws is None:
        denc_ws = torch.empty(n, 32, device=xyzs.device)
    st = _lib().ngp_field_backward(_ptr(xyzs), _ptr(dirs), n, _ptr(n_dev), ctypes.byref(grid.desc), _ptr(enc),
                                   _ptr(params16), _ptr(dL_dsig), _ptr(dL_drgb), _ptr(denc_ws), _ptr(grad),
                                   _ptr(grad[MLP_PARAMS:]), vren._stream())
    vren._ok(st, "ngp_field_backward")


BIN_LEVEL_LO, BIN_MERGE_HI = 8, 11  # the trainer's hybrid split on object scenes (trainer.NGPTrainer)
BIN_WS_SAMPLES = 1 << 20  # binned workspace: gradient-carrying samples it holds (the rest: atomic path, exact)
COARSE_REP, COARSE_REP_LEVELS = 8, 4  # the trainer's gradient replicas of the coarsest atomic levels
_bin_ws = {}
_rep_bufs = {}


def _binned_workspace(device):
    """The binned hash backward's workspace (ngp_hash_backward_binned_workspace(BIN_WS_SAMPLES) bytes),
    one per device, allocated on first use and reused by every drop-in backward."""
    ws = _bin_ws.get(device)
    if ws is None:
        nbytes = _lib().ngp_hash_backward_binned_workspace(BIN_WS_SAMPLES)
        ws = _bin_ws[device] = torch.empty((nbytes + 255) // 256, 64, dtype=torch.int32, device=device)
    return ws


def _rep_buffer(grid, device):
    """Replicas of the coarse levels' gradient (ngp_hash_backward_levels_rep; zero between calls)."""
    key = (device, tuple(grid.offsets))
    rep = _rep_bufs.get(key)
    if rep is None:
        nrep = _lib().ngp_hash_backward_rep_floats(ctypes.byref(grid.desc), COARSE_REP_LEVELS, COARSE_REP)
        rep = _rep_bufs[key] = torch.zeros(nrep, device=device)
    return rep


def field_backward_sparse(xyzs, dirs, grid: HashGrid, params16, enc, dL_dsig, dL_drgb, grad):
    """field_backward over the samples that carry gradient only, with the
    training step's hybrid hash backward: the rows with a nonzero dL/dsigma or
    dL/drgb are listed on the device (ngp_gradient_rows: no host sync) -- the
    compositing backward leaves every sample past its ray's termination at
    exact zero, and a zero row adds exactly nothing -- then the MLP backward,
    the atomic coarse levels [0, 8) (levels 0-3 into 8 gradient replicas, folded
    after) and the binned levels [8, 16) over that list
    (the same gradient as field_backward up to fp32 summation order)."""
    n = xyzs.shape[0]
    _check(grad, "grad", torch.float32, grid.n_params)
    _check(enc, "enc", torch.float16)
    _check(dL_dsig, "dL_dsigmas", torch.float32); _check(dL_drgb, "dL_drgbs", torch.float32)
    if n == 0:
        return
    dev = xyzs.device
    L, s = _lib(), vren._stream()
    idx = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    vren._ok(vren.lib().ngp_gradient_rows(_ptr(dL_dsig), _ptr(dL_drgb), n, _ptr(idx), _ptr(cnt), s), "gradient_rows")
    denc = torch.empty(n, 32, device=dev)
    vren._ok(L.ngp_field_backward_mlp(_ptr(dirs), n, _ptr(cnt), _ptr(idx), _ptr(enc), 0, _ptr(params16),
                                      _ptr(dL_dsig), _ptr(dL_drgb), _ptr(denc), _ptr(grad), s), "field_backward_mlp")
    gt = grad[MLP_PARAMS:]
    vren._ok(L.ngp_hash_backward_levels_rep(_ptr(xyzs), n, _ptr(cnt), _ptr(idx), ctypes.byref(grid.desc), _ptr(denc),
                                            _ptr(gt), 0, BIN_LEVEL_LO, _ptr(_rep_buffer(grid, dev)),
                                            COARSE_REP_LEVELS, COARSE_REP, 1, s), "hash_backward_levels_rep")
    vren._ok(L.ngp_hash_backward_binned(_ptr(xyzs), n, _ptr(cnt), _ptr(idx), ctypes.byref(grid.desc), _ptr(denc),
                                        _ptr(gt), _ptr(_binned_workspace(dev)), BIN_WS_SAMPLES, BIN_LEVEL_LO,
                                        BIN_MERGE_HI, s), "hash_backward_binned")


class FP16Shadow:
    """fp16 copy of an fp32 master parameter, refreshed when the master changes."""

    def __init__(self, master: torch.Tensor):
        self.master = master
        self.version = None
        self.half = None

    def get(self):
        v = self.master._version
        if self.half is None or v != self.version or self.half.data_ptr() == 0:
            self.half = self.master.detach().to(torch.float16)
            self.version = v
        return self.half


class _FieldFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xyzs, dirs, params, grid, shadow):
        p16 = shadow.get()
        sig, rgb, enc, _ = field_forward(xyzs.contiguous(), dirs.contiguous(), grid, p16, save_enc=True)
        ctx.save_for_backward(xyzs, dirs, enc)
        ctx.grid, ctx.p16 = grid, p16
        return sig, rgb

    @staticmethod
    def backward(ctx, dsig, drgb):
        xyzs, dirs, enc = ctx.saved_tensors
        grid = ctx.grid
        dsig = torch.zeros(xyzs.shape[0], device=xyzs.device) if dsig is None else dsig.float().contiguous()
        drgb = torch.zeros(xyzs.shape[0], 3, device=xyzs.device) if drgb is None else drgb.float().contiguous()
        grad = torch.zeros(grid.n_params, device=xyzs.device)
        field_backward_sparse(xyzs.contiguous(), dirs.contiguous(), grid, ctx.p16, enc, dsig, drgb, grad)
        return None, None, grad, None, None


def field(xyzs, dirs, params, grid, shadow):
    """Differentiable (w.r.t. params) fused field: -> sigmas (n), rgbs (n,3)."""
    return _FieldFn.apply(xyzs, dirs, params, grid, shadow)
