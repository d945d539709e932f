"""`vren` for MI355X: the reference's pybind extension surface
(models/csrc/binding.cpp:234-250) re-implemented over the C-ABI library
libngp_amd.so (include/ngp_amd.h, hand-written gfx950 HIP kernels).

Same function names, argument order and meaning, same output tensors and
the same CHECK_INPUT error behaviour ("x must be a CUDA tensor" /
"x must be contiguous" as RuntimeError, models/csrc/include/utils.h:4-6).
There is NO CPU fallback: importing works on any host (so the library can
be inspected), but every call needs the library and GPU tensors, and fails
loudly otherwise.

Differences from the reference, all deliberate and documented in DESIGN.md:
  * raymarching_train returns exact-size outputs in a deterministic
    RAY-ORDERED layout (rays_a[r] = [r, start_r, n_r]); the reference fills
    a N_rays*1024 zero-initialised scratch in atomic order.
  * composite_train_fw's first output is the per-ray sample count, as in
    the reference (the autograd wrapper sums it).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_int64, c_void_p

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NGP_AMD_LIB", os.path.join(_HERE, "lib", "libngp_amd.so"))

_lib = None


class NGPError(RuntimeError):
    pass


def _declare(L):
    vp = c_void_p
    sig = {
        "ngp_ray_aabb_intersect": [vp, vp, c_int64, vp, vp, c_int, c_int, vp, vp, vp, vp],
        "ngp_raygen_aabb": [vp, vp, vp, vp, c_int64, vp, vp, c_float, vp, vp, vp, vp],
        "ngp_sample_batch": [ctypes.c_uint64, ctypes.c_uint64, c_int64, vp, c_int, c_int64, c_int64, vp, vp, c_int64,
                             vp, vp, c_float, vp, vp, vp, vp, vp, vp, vp, vp],
        "ngp_sample_batch_dev": [ctypes.c_uint64, vp, c_int64, c_int64, vp, c_int, c_int64, c_int64, vp, vp, c_int64,
                                 vp, vp, c_float, vp, vp, vp, vp, vp, vp, vp, vp],
        "ngp_adam_step_dev": [vp, vp, vp, vp, vp, c_int64, vp, c_float, c_float, c_float, vp, c_float, c_int, vp],
        "ngp_adam_step_dev_zero": [vp, vp, vp, vp, vp, c_int64, vp, c_float, c_float, c_float, vp, c_float, c_int, vp,
                                   c_int64, vp],
        "ngp_adam_step_dev_rep": [vp, vp, vp, vp, vp, c_int64, vp, c_float, c_float, c_float, vp, c_float, c_int, vp,
                                  c_int64, c_int64, c_int, vp],
        "ngp_counters_inc": [vp, c_int, vp],
        "ngp_random_bg": [ctypes.c_uint64, vp, c_int64, vp, vp],
        "ngp_occupied_cells": [vp, c_int64, c_float, vp, vp, vp, vp],
        "ngp_occupancy_samples": [ctypes.c_uint64, vp, c_int, c_int, c_int64, c_float, c_float, vp, vp, c_int64,
                                  c_int64, vp, vp, vp],
        "ngp_occupancy_samples_sorted": [ctypes.c_uint64, vp, c_int, c_int, c_int64, c_float, c_float, vp, vp,
                                         c_int64, c_int64, vp, vp, vp, vp],
        "ngp_morton3d": [vp, c_int64, vp, vp],
        "ngp_morton3d_invert": [vp, c_int64, vp, vp],
        "ngp_packbits": [vp, c_int64, c_float, vp, vp, vp],
        "ngp_march_train_count": [vp, vp, vp, c_int64, vp, c_int, c_int, c_float, c_float, vp, c_int, vp, vp, vp, vp],
        "ngp_march_train_write": [vp, vp, vp, c_int64, vp, c_int, c_int, c_float, c_float, vp, c_int, vp, vp, vp, vp,
                                  vp, vp],
        "ngp_march_train_slots": [vp, vp, vp, c_int64, vp, c_int, c_int, c_float, c_float, vp, c_int, vp, vp, vp, vp,
                                  vp, vp, vp],
        "ngp_bitfield_summary": [vp, c_int64, c_int, vp, vp],
        "ngp_march_train_compact": [vp, vp, vp, c_int64, vp, vp, c_int, vp, vp, vp, vp, vp],
        "ngp_march_test": [vp, vp, vp, vp, c_int64, vp, c_int, c_int, c_float, c_float, c_int, c_int, vp, vp, vp, vp,
                           vp, vp, vp],
        "ngp_composite_train_fw": [vp, vp, vp, vp, vp, c_int64, c_float, vp, vp, vp, vp, vp, vp],
        "ngp_composite_train_bw": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, c_int64, vp, vp, vp, c_float, vp, vp, vp],
        "ngp_composite_test_fw": [vp, vp, vp, vp, c_int64, c_int, vp, c_float, vp, vp, vp, vp, vp],
        "ngp_composite_loss": [vp, vp, vp, vp, vp, c_int64, vp, vp, c_int, c_float, c_float, c_float, c_float, c_float,
                               vp,
                               vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
        "ngp_active_samples": [vp, vp, c_int64, vp, vp, vp, vp],
        "ngp_gradient_rows": [vp, vp, c_int64, vp, vp, vp],
        "ngp_nerf_loss_fw": [vp, vp, vp, vp, c_int64, c_int, c_float, c_float, c_float, vp, vp, vp, vp],
        "ngp_nerf_loss_bw": [vp, vp, vp, vp, c_int64, c_int, c_float, c_float, c_float, vp, vp, vp, vp, vp, vp, vp],
        "ngp_chunk_counts": [vp, c_int64, c_int, vp, vp, c_float, vp, vp],
        "ngp_chunk_counts_range": [vp, c_int64, c_int, c_int, vp, vp, c_float, vp, vp],
        "ngp_ray_segments": [vp, vp, c_int64, c_int, vp, vp, vp, vp, vp],
        "ngp_rays_nonempty": [vp, c_int64, vp, vp, vp, vp, vp],
        "ngp_chunk_segments": [vp, vp, vp, c_int64, c_int, c_int, c_float, vp, vp, vp, vp, vp, vp, vp],
        "ngp_ray_segments_capped": [vp, c_int64, c_int, vp, vp, vp, vp, vp],
        "ngp_adam_step": [vp, vp, vp, vp, vp, c_int64, c_float, c_float, c_float, c_float, c_int64, c_float, c_int,
                          vp],
        "ngp_density_scatter_last": [vp, vp, c_int64, c_int64, vp, vp],
        "ngp_occupancy_keep": [vp, c_int64, c_int64, c_int64, c_int64, c_int64, vp, vp, vp, vp],
        "ngp_density_scatter_kept": [vp, vp, c_int64, vp, vp, c_int64, vp, vp],
        "ngp_density_grid_ema": [vp, vp, c_int64, c_float, vp, c_float, vp, vp, vp],
        "ngp_distortion_loss_fw": [vp, vp, vp, vp, c_int64, vp, vp, vp, vp],
        "ngp_distortion_loss_bw": [vp, vp, vp, vp, vp, vp, vp, c_int64, vp, vp],
        "ngp_render_test_begin": [c_int64, vp, vp, vp, vp, vp, vp],
        "ngp_render_test_march": [vp, vp, vp, c_int64, vp, c_int, c_int, c_float, c_float, c_int, c_int, c_int64,
                                  c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp],
        "ngp_render_test_composite": [vp, vp, vp, vp, vp, c_int64, c_int, vp, vp, vp, c_float, vp, vp, vp, vp],
        "ngp_render_test_finish": [vp, c_int64, vp, vp, vp],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = c_int
    L.ngp_version.restype = ctypes.c_char_p
    L.ngp_hashgrid_levels.argtypes = [c_int, c_int, c_int, c_float, vp, vp, vp, vp]
    L.ngp_hashgrid_levels.restype = ctypes.c_uint32
    L.ngp_occupancy_sorted_workspace.argtypes = [c_int64]
    L.ngp_occupancy_sorted_workspace.restype = ctypes.c_size_t
    L.ngp_occupied_cells_workspace.argtypes = [c_int64]
    L.ngp_occupied_cells_workspace.restype = ctypes.c_size_t
    L.ngp_chunk_segments_workspace.argtypes = [c_int64]
    L.ngp_chunk_segments_workspace.restype = ctypes.c_size_t
    L.ngp_render_test_capacity.argtypes = [c_int64, c_int]
    L.ngp_render_test_capacity.restype = c_int64
    L.ngp_guard_hits.argtypes = []
    L.ngp_guard_hits.restype = ctypes.c_ulonglong
    L.ngp_guard_reset.argtypes = []
    L.ngp_guard_reset.restype = c_int
    # measurement hook (ktimer.py)
    L.ngp_timing_set.argtypes = [vp, vp, c_int64, c_int, c_int, ctypes.c_uint64, ctypes.c_uint64]
    L.ngp_timing_set.restype = c_int
    L.ngp_timing_counts.argtypes = [vp, c_int]
    L.ngp_timing_counts.restype = c_int
    L.ngp_timing_tick_ns.argtypes = []
    L.ngp_timing_tick_ns.restype = ctypes.c_double
    L.ngp_probe_set.argtypes = [vp, vp, c_int64]
    L.ngp_probe_set.restype = c_int
    L.ngp_probe_count.argtypes = []
    L.ngp_probe_count.restype = c_int
    L.ngp_trace_marker.argtypes = [c_int, vp]
    L.ngp_trace_marker.restype = c_int


def lib():
    """Load libngp_amd.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NGPError(f"libngp_amd.so not found at {LIB_PATH}: run `make -C ar-nerf_amd` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def _stream():
    return c_void_p(torch.cuda.current_stream().cuda_stream)


def _check(name, x, dtype=None):
    # models/csrc/include/utils.h:4-6 (CHECK_CUDA, CHECK_CONTIGUOUS)
    if not isinstance(x, torch.Tensor) or not x.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not x.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    if dtype is not None and x.dtype != dtype:
        raise RuntimeError(f"{name} must be {dtype}, got {x.dtype}")
    return c_void_p(x.data_ptr())


def _ok(st, what):
    if st != 0:
        raise NGPError(f"{what} failed with status {st}")


# ------------------------------------------------------------------ rays
def ray_aabb_intersect(rays_o, rays_d, centers, half_sizes, max_hits):
    """intersection.cu:59-100 -> [hit_cnt (N) i32, hits_t (N,max_hits,2), hits_voxel_idx (N,max_hits) i64]"""
    po, pd = _check("rays_o", rays_o, torch.float32), _check("rays_d", rays_d, torch.float32)
    pc, ph = _check("centers", centers, torch.float32), _check("half_sizes", half_sizes, torch.float32)
    n, nv = rays_o.shape[0], centers.numel() // 3
    dev = rays_o.device
    cnt = torch.empty(n, dtype=torch.int32, device=dev)
    ht = torch.empty(n, max_hits, 2, dtype=torch.float32, device=dev)
    hv = torch.empty(n, max_hits, dtype=torch.int64, device=dev)
    _ok(lib().ngp_ray_aabb_intersect(po, pd, n, pc, ph, nv, int(max_hits), c_void_p(cnt.data_ptr()),
                                     c_void_p(ht.data_ptr()), c_void_p(hv.data_ptr()), _stream()),
        "ray_aabb_intersect")
    return [cnt, ht, hv]


def raygen_aabb(directions, poses, img_idxs, pix_idxs, center, half_size, near_distance):
    """Fused get_rays (datasets/ray_utils.py:45-70) on the gathered training
    batch (train.py:85-87) + AABB + near clamp (models/rendering.py:29-31).
    Returns rays_o, rays_d (N,3) and hits_t (N,2)."""
    n = img_idxs.shape[0]
    dev = directions.device
    rays_o = torch.empty(n, 3, device=dev)
    rays_d = torch.empty(n, 3, device=dev)
    hits_t = torch.empty(n, 2, device=dev)
    _ok(lib().ngp_raygen_aabb(_check("directions", directions, torch.float32), _check("poses", poses, torch.float32),
                              _check("img_idxs", img_idxs, torch.int64), _check("pix_idxs", pix_idxs, torch.int64), n,
                              _check("center", center, torch.float32), _check("half_size", half_size, torch.float32),
                              float(near_distance), c_void_p(rays_o.data_ptr()), c_void_p(rays_d.data_ptr()),
                              c_void_p(hits_t.data_ptr()), _stream()), "raygen_aabb")
    return rays_o, rays_d, hits_t


# -------------------------------------------------------- occupancy grid
def morton3D(coords):
    p = _check("coords", coords, torch.int32)
    out = torch.empty(coords.shape[0], dtype=torch.int32, device=coords.device)
    _ok(lib().ngp_morton3d(p, coords.shape[0], c_void_p(out.data_ptr()), _stream()), "morton3D")
    return out


def morton3D_invert(indices):
    p = _check("indices", indices, torch.int32)
    out = torch.empty(indices.shape[0], 3, dtype=torch.int32, device=indices.device)
    _ok(lib().ngp_morton3d_invert(p, indices.shape[0], c_void_p(out.data_ptr()), _stream()), "morton3D_invert")
    return out


def packbits(density_grid, density_threshold, density_bitfield):
    """In place on density_bitfield.  density_threshold may be a float or a
    1-element device tensor (then no host sync is needed)."""
    pg = _check("density_grid", density_grid, torch.float32)
    pb = _check("density_bitfield", density_bitfield, torch.uint8)
    if density_grid.numel() != 8 * density_bitfield.numel():
        raise RuntimeError("density_grid must hold 8 cells per bitfield byte")
    if isinstance(density_threshold, torch.Tensor):
        thr_dev, thr = _check("density_threshold", density_threshold, torch.float32), 0.0
    else:
        thr_dev, thr = None, float(density_threshold)
    _ok(lib().ngp_packbits(pg, density_bitfield.numel(), thr, thr_dev, pb, _stream()), "packbits")


def bitfield_summary(density_bitfield, grid_size=128, out=None):
    """ngp_bitfield_summary: 2 x (n_bytes/256) i32 words: bit w = (64-bit word w
    of the bitfield != 0), then the same dilated by one 4^3 block.  The
    marchers keep it in LDS to skip empty blocks without a global load and
    rays that pass no occupied block (same results with or without it)."""
    pb = _check("density_bitfield", density_bitfield, torch.uint8)
    n = density_bitfield.numel()
    if out is None:
        out = torch.empty(2 * ((n + 255) // 256), dtype=torch.int32, device=density_bitfield.device)
    _ok(lib().ngp_bitfield_summary(pb, n, int(grid_size), c_void_p(out.data_ptr()), _stream()), "bitfield_summary")
    return out


def _summary_arg(density_bitfield, cascades, grid_size):
    """Summary for a marcher launch, or None when the grid is not whole
    2048-cell words (the marcher then reads the bitfield directly)."""
    if (int(cascades) * int(grid_size) ** 3) % 2048 != 0 or density_bitfield.numel() % 8 != 0:
        return None
    return bitfield_summary(density_bitfield, grid_size)


# ----------------------------------------------------------- marching
def march_train_count(rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, noise,
                      grid_size, max_samples):
    """Pass 1 -> (counts i32 (N), rays_a i64 (N,3) ray-ordered, total i64 (1)), no host sync."""
    n = rays_o.shape[0]
    dev = rays_o.device
    counts = torch.empty(n, dtype=torch.int32, device=dev)
    rays_a = torch.empty(n, 3, dtype=torch.int64, device=dev)
    total = torch.empty(1, dtype=torch.int64, device=dev)
    _ok(lib().ngp_march_train_count(_check("rays_o", rays_o, torch.float32), _check("rays_d", rays_d, torch.float32),
                                    _check("hits_t", hits_t, torch.float32), n,
                                    _check("density_bitfield", density_bitfield, torch.uint8), int(cascades),
                                    int(grid_size), float(scale), float(exp_step_factor),
                                    _check("noise", noise, torch.float32), int(max_samples),
                                    c_void_p(counts.data_ptr()), c_void_p(rays_a.data_ptr()),
                                    c_void_p(total.data_ptr()), _stream()), "march_train_count")
    return counts, rays_a, total


def march_train_write(rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, noise,
                      grid_size, max_samples, rays_a, xyzs, dirs, deltas, ts):
    """Pass 2 into caller buffers (capacity >= total)."""
    _ok(lib().ngp_march_train_write(_check("rays_o", rays_o, torch.float32), _check("rays_d", rays_d, torch.float32),
                                    _check("hits_t", hits_t, torch.float32), rays_o.shape[0],
                                    _check("density_bitfield", density_bitfield, torch.uint8), int(cascades),
                                    int(grid_size), float(scale), float(exp_step_factor),
                                    _check("noise", noise, torch.float32), int(max_samples),
                                    _check("rays_a", rays_a, torch.int64), _check("xyzs", xyzs, torch.float32),
                                    _check("dirs", dirs, torch.float32), _check("deltas", deltas, torch.float32),
                                    _check("ts", ts, torch.float32), _stream()), "march_train_write")


def raymarching_train(rays_o, rays_d, hits_t, density_bitfield, cascades, scale, exp_step_factor, noise,
                      grid_size, max_samples):
    """raymarching.cu:283-332 -> [rays_a, xyzs, dirs, deltas, ts, counter].
    counter = [total_samples, n_rays] (int32, like the reference's).  Single
    walk per ray into slot scratch, then one host sync to size the outputs
    (the reference syncs on counter[0] slicing, custom_functions.py:91-96)."""
    n = rays_o.shape[0]
    dev = rays_o.device
    counts = torch.empty(n, dtype=torch.int32, device=dev)
    rays_a = torch.empty(n, 3, dtype=torch.int64, device=dev)
    total = torch.empty(1, dtype=torch.int64, device=dev)
    slot_t = torch.empty(n * int(max_samples), device=dev)
    slot_dt = torch.empty(n * int(max_samples), device=dev)
    po, pd = _check("rays_o", rays_o, torch.float32), _check("rays_d", rays_d, torch.float32)
    summ = _summary_arg(density_bitfield, cascades, grid_size)
    _ok(lib().ngp_march_train_slots(po, pd, _check("hits_t", hits_t, torch.float32), n,
                                    _check("density_bitfield", density_bitfield, torch.uint8), int(cascades),
                                    int(grid_size), float(scale), float(exp_step_factor),
                                    _check("noise", noise, torch.float32), int(max_samples),
                                    c_void_p(counts.data_ptr()), c_void_p(rays_a.data_ptr()),
                                    c_void_p(total.data_ptr()), c_void_p(slot_t.data_ptr()),
                                    c_void_p(slot_dt.data_ptr()), c_void_p(summ.data_ptr()) if summ is not None else None,
                                    _stream()), "march_train_slots")
    N = int(total.item())
    xyzs = torch.empty(N, 3, device=dev)
    dirs = torch.empty(N, 3, device=dev)
    deltas = torch.empty(N, device=dev)
    ts = torch.empty(N, device=dev)
    if N > 0:
        _ok(lib().ngp_march_train_compact(po, pd, c_void_p(rays_a.data_ptr()), n, c_void_p(slot_t.data_ptr()),
                                          c_void_p(slot_dt.data_ptr()), int(max_samples), c_void_p(xyzs.data_ptr()),
                                          c_void_p(dirs.data_ptr()), c_void_p(deltas.data_ptr()),
                                          c_void_p(ts.data_ptr()), _stream()), "march_train_compact")
    counter = torch.stack([total[0].to(torch.int32), torch.full_like(total[0], n, dtype=torch.int32)])
    return [rays_a, xyzs, dirs, deltas, ts, counter]


def raymarching_test(rays_o, rays_d, hits_t, alive_indices, density_bitfield, cascades, scale, exp_step_factor,
                     grid_size, max_samples, N_samples):
    """raymarching.cu:407-454; hits_t (N_rays,2) is updated in place."""
    n = alive_indices.shape[0]
    dev = rays_o.device
    xyzs = torch.empty(n, N_samples, 3, device=dev)
    dirs = torch.empty(n, N_samples, 3, device=dev)
    deltas = torch.empty(n, N_samples, device=dev)
    ts = torch.empty(n, N_samples, device=dev)
    neff = torch.empty(n, dtype=torch.int32, device=dev)
    summ = _summary_arg(density_bitfield, cascades, grid_size)
    _ok(lib().ngp_march_test(_check("rays_o", rays_o, torch.float32), _check("rays_d", rays_d, torch.float32),
                             _check("hits_t", hits_t, torch.float32), _check("alive_indices", alive_indices, torch.int64),
                             n, _check("density_bitfield", density_bitfield, torch.uint8), int(cascades),
                             int(grid_size), float(scale), float(exp_step_factor), int(N_samples), int(max_samples),
                             c_void_p(xyzs.data_ptr()), c_void_p(dirs.data_ptr()), c_void_p(deltas.data_ptr()),
                             c_void_p(ts.data_ptr()), c_void_p(neff.data_ptr()),
                             c_void_p(summ.data_ptr()) if summ is not None else None, _stream()), "raymarching_test")
    return [xyzs, dirs, deltas, ts, neff]


# ---------------------------------------------------------- compositing
def composite_train_fw(sigmas, rgbs, deltas, ts, rays_a, T_threshold):
    """volumerendering.cu:47-83 -> [total_samples (N_rays) i64, opacity, depth, rgb, ws]"""
    nr, N = rays_a.shape[0], sigmas.shape[0]
    dev = sigmas.device
    op = torch.empty(nr, device=dev)
    dep = torch.empty(nr, device=dev)
    rgb = torch.empty(nr, 3, device=dev)
    ws = torch.empty(N, device=dev)
    tot = torch.empty(nr, dtype=torch.int64, device=dev)
    _ok(lib().ngp_composite_train_fw(_check("sigmas", sigmas, torch.float32), _check("rgbs", rgbs, torch.float32),
                                     _check("deltas", deltas, torch.float32), _check("ts", ts, torch.float32),
                                     _check("rays_a", rays_a, torch.int64), nr, float(T_threshold),
                                     c_void_p(tot.data_ptr()), c_void_p(op.data_ptr()), c_void_p(dep.data_ptr()),
                                     c_void_p(rgb.data_ptr()), c_void_p(ws.data_ptr()), _stream()),
        "composite_train_fw")
    return [tot, op, dep, rgb, ws]


def composite_train_bw(dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts, rays_a, opacity,
                       depth, rgb, T_threshold):
    """volumerendering.cu:153-201 -> [dL_dsigmas (N), dL_drgbs (N,3)]"""
    N, nr = sigmas.shape[0], rays_a.shape[0]
    dev = sigmas.device
    dsig = torch.empty(N, device=dev)
    drgbs = torch.empty(N, 3, device=dev)
    _ok(lib().ngp_composite_train_bw(
        _check("dL_dopacity", dL_dopacity, torch.float32), _check("dL_ddepth", dL_ddepth, torch.float32),
        _check("dL_drgb", dL_drgb, torch.float32), _check("dL_dws", dL_dws, torch.float32),
        _check("sigmas", sigmas, torch.float32), _check("rgbs", rgbs, torch.float32), _check("ws", ws, torch.float32),
        _check("deltas", deltas, torch.float32), _check("ts", ts, torch.float32), _check("rays_a", rays_a, torch.int64),
        nr, _check("opacity", opacity, torch.float32), _check("depth", depth, torch.float32),
        _check("rgb", rgb, torch.float32), float(T_threshold), c_void_p(dsig.data_ptr()), c_void_p(drgbs.data_ptr()),
        _stream()), "composite_train_bw")
    return [dsig, drgbs]


def composite_test_fw(sigmas, rgbs, deltas, ts, hits_t, alive_indices, T_threshold, N_eff_samples, opacity, depth,
                      rgb):
    """volumerendering.cu:251-284; alive/opacity/depth/rgb updated in place."""
    n = alive_indices.shape[0]
    Ns = sigmas.shape[1] if sigmas.dim() == 2 else 1
    _ok(lib().ngp_composite_test_fw(_check("sigmas", sigmas, torch.float32), _check("rgbs", rgbs, torch.float32),
                                    _check("deltas", deltas, torch.float32), _check("ts", ts, torch.float32), n, Ns,
                                    _check("alive_indices", alive_indices, torch.int64), float(T_threshold),
                                    _check("N_eff_samples", N_eff_samples, torch.int32),
                                    _check("opacity", opacity, torch.float32), _check("depth", depth, torch.float32),
                                    _check("rgb", rgb, torch.float32), _stream()), "composite_test_fw")


def ray_sphere_intersect(*args, **kwargs):
    raise NotImplementedError("ray_sphere_intersect is never called by the reference (intersection.cu:103-197); "
                              "out of scope (SURVEY.md §2 row 3)")


def distortion_loss_fw(ws, deltas, ts, rays_a):
    """losses.cu:62-107 -> [loss (N_rays), ws_inclusive_scan (N), wts_inclusive_scan (N)]
    (zero-initialised like the reference's torch::zeros outputs)."""
    pw, pd, pt = (_check("ws", ws, torch.float32), _check("deltas", deltas, torch.float32),
                  _check("ts", ts, torch.float32))
    pr = _check("rays_a", rays_a, torch.int64)
    nr, N = rays_a.shape[0], ws.shape[0]
    loss = torch.zeros(nr, device=ws.device)
    wsi, wtsi = torch.zeros(N, device=ws.device), torch.zeros(N, device=ws.device)
    _ok(lib().ngp_distortion_loss_fw(pw, pd, pt, pr, nr, c_void_p(loss.data_ptr()), c_void_p(wsi.data_ptr()),
                                     c_void_p(wtsi.data_ptr()), _stream()), "distortion_loss_fw")
    return [loss, wsi, wtsi]


def distortion_loss_bw(dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a):
    """losses.cu:143-173 -> dL_dws (N)"""
    a = [_check("dL_dloss", dL_dloss, torch.float32), _check("ws_inclusive_scan", ws_inclusive_scan, torch.float32),
         _check("wts_inclusive_scan", wts_inclusive_scan, torch.float32), _check("ws", ws, torch.float32),
         _check("deltas", deltas, torch.float32), _check("ts", ts, torch.float32),
         _check("rays_a", rays_a, torch.int64)]
    dws = torch.zeros(ws.shape[0], device=ws.device)
    _ok(lib().ngp_distortion_loss_bw(*a, rays_a.shape[0], c_void_p(dws.data_ptr()), _stream()), "distortion_loss_bw")
    return dws


def density_scatter_last(tmp, indices, sigmas):
    """tmp.view(-1)[indices] = sigmas (models/networks.py:268) with torch's
    sequential index_put_ semantics on duplicate indices (the last one in
    list order wins), deterministically on the GPU (a device index_put_
    leaves the winner to the scheduler): ngp_density_scatter_last's 64-bit
    (position, sigma) keys, then the winners' sigmas into tmp (f32, in place;
    cells not listed keep their value; sigma is clamped at 0)."""
    _check("tmp", tmp, torch.float32)
    idx = indices.reshape(-1).long().contiguous()
    sig = sigmas.reshape(-1).float().contiguous()
    key = torch.zeros(tmp.numel(), dtype=torch.int64, device=tmp.device)
    _ok(lib().ngp_density_scatter_last(idx.data_ptr(), sig.data_ptr(), idx.numel(), 0, key.data_ptr(), _stream()),
        "density_scatter_last")
    hit = key != 0
    val = (key & 0xFFFFFFFF).to(torch.int32).view(torch.float32)
    flat = tmp.view(-1)
    flat.copy_(torch.where(hit, val, flat))
    return tmp


def erode_decay(count_grid, decay=0.95):
    """Per-cell erode decay clamp(decay**(1/count_grid), 0.1, 0.95)
    (models/networks.py:270-272), for ngp_density_grid_ema's decay_cells.
    count_grid is fixed once mark_invisible_cells ran, so this is evaluated
    once, with torch on the host: the values are the reference expression's
    CPU evaluation bit for bit (a device pow may differ in the last ulp).
    Cells no camera sees (count 0 -> 0.1) hold density -1 and never decay."""
    return torch.clamp(decay ** (1 / count_grid.detach().float().cpu()), 0.1, 0.95)
