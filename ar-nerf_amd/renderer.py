"""Graph-captured test-time renderer (BASELINE config 5).

The reference renders a frame with the host loop of __render_rays_test
(models/rendering.py:162-253): per iteration a host-side N_samples decision,
vren.raymarching_test, model(xyzs, dirs) on the valid samples,
vren.composite_test_fw and a boolean-mask compaction of the alive rays --
a host sync and ~10 launches per iteration, ~20-40 iterations per frame.

TestRenderer runs the same loop with every decision in device memory
(include/ngp_amd.h "device-resident test-time render"): one iteration is
  ngp_render_test_march   (loop test, N_samples, march, valid-sample list)
  ngp_field_encode_mlp over the list (NGP.forward: encode + MLPs in one launch)
  ngp_render_test_composite (composite_test_fw + survivor compaction)
and the iterations are captured in HIP graphs: a frame is graph A (begin +
summary + `iters_per_graph` iterations), then graph B (`iters_tail` more)
only while the device says the loop is still running -- one host sync per
graph; iterations after the loop ends are no-ops (early exits).
Results (opacity, depth, rgb, total_samples) equal the host loop's bit for
bit: tests/test_renderer_gpu.py.
"""
from __future__ import annotations

import ctypes
from ctypes import c_float, c_void_p

import torch

import hashgrid as HG
import vren

MAX_SAMPLES = 1024     # models/rendering.py:7
NEAR_DISTANCE = 0.01   # models/rendering.py:8
STATE_WORDS = 8        # NGP_RENDER_STATE_WORDS
RS_ACTIVE, RS_VALID, RS_TOTAL, RS_ITERS = 4, 5, 6, 7


def _p(t):
    return c_void_p(t.data_ptr())


class TestRenderer:
    """Fixed-shape renderer for batches of n_rays rays (a full frame:
    n_rays = W*H).  params16 / density_bitfield are read through stable
    device buffers: `params16` is used in place (refresh it with copy_), the
    bitfield is re-read every frame (its summary is rebuilt inside graph A)."""

    def __init__(self, n_rays, grid: HG.HashGrid, params16, density_bitfield, cascades, scale, grid_size=128,
                 exp_step_factor=0.0, T_threshold=1e-4, max_samples=MAX_SAMPLES, iters_per_graph=16,
                 bg_rgb=(0.0, 0.0, 0.0), use_graphs=True, iters_tail=None):
        iters_tail = iters_per_graph if iters_tail is None else iters_tail
        if min(iters_per_graph, iters_tail) < 2 or iters_per_graph % 2 or iters_tail % 2:
            raise ValueError("iters_per_graph / iters_tail must be even (alive lists alternate per iteration)")
        dev = params16.device
        vren._check("params16", params16, torch.float16)
        vren._check("density_bitfield", density_bitfield, torch.uint8)
        self.n_rays, self.grid, self.params16, self.bitfield = int(n_rays), grid, params16, density_bitfield
        self.cascades, self.scale, self.grid_size = int(cascades), float(scale), int(grid_size)
        self.esf, self.T_threshold, self.max_samples = float(exp_step_factor), float(T_threshold), int(max_samples)
        # rendering.py:185: min_samples = 1 if exp_step_factor == 0 else 4
        self.min_samples = 1 if self.esf == 0 else 4
        # graph A: frame opening + K iterations; graph B (replayed while the loop runs): K_tail
        self.K, self.K_tail, self.use_graphs = int(iters_per_graph), int(iters_tail), bool(use_graphs)
        self.bg = (ctypes.c_float * 3)(*[float(b) for b in bg_rgb])
        L = HG._lib()
        self.cap = int(L.ngp_render_test_capacity(self.n_rays, self.min_samples))
        n, cap = self.n_rays, self.cap
        f = dict(device=dev, dtype=torch.float32)
        self.rays_o = torch.zeros(n, 3, **f)
        self.rays_d = torch.zeros(n, 3, **f)
        self.hits_t = torch.zeros(n, 2, **f)
        self.opacity = torch.zeros(n, **f)
        self.depth = torch.zeros(n, **f)
        self.rgb = torch.zeros(n, 3, **f)
        self.state = torch.zeros(STATE_WORDS, dtype=torch.int64, device=dev)
        self.alive = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
        self.n_eff = torch.zeros(n, dtype=torch.int32, device=dev)
        self.xyzs = torch.zeros(cap, 3, **f)
        self.dirs = torch.zeros(cap, 3, **f)
        self.deltas = torch.zeros(cap, **f)
        self.ts = torch.zeros(cap, **f)
        self.sigmas = torch.zeros(cap, **f)
        self.rgbs = torch.zeros(cap, 3, **f)
        self.sample_idx = torch.zeros(cap, dtype=torch.int32, device=dev)
        self.enc = torch.zeros(8 * cap * 4, dtype=torch.float16, device=dev)  # pair-major (8, cap, 4)
        self.summary = torch.zeros(2 * ((density_bitfield.numel() + 255) // 256), dtype=torch.int32, device=dev)
        self.n_valid_ptr = c_void_p(self.state.data_ptr() + 8 * RS_VALID)
        self._graphs = {}
        self.last_iterations = 0
        # full-frame camera (render_pose)
        self._dirs = None

    # ------------------------------------------------------------ pieces
    def _iteration(self, k):
        """One loop iteration (rendering.py:186-236) on the current stream."""
        L, s, par = HG._lib(), vren._stream(), k & 1
        vren._ok(L.ngp_render_test_march(_p(self.rays_o), _p(self.rays_d), _p(self.hits_t), self.n_rays,
                                         _p(self.bitfield), self.cascades, self.grid_size, c_float(self.scale),
                                         c_float(self.esf), MAX_SAMPLES, self.min_samples, self.max_samples, par,
                                         _p(self.state), _p(self.alive[par]), _p(self.summary), _p(self.xyzs),
                                         _p(self.dirs), _p(self.deltas), _p(self.ts), _p(self.n_eff),
                                         _p(self.sample_idx), s), "render_test_march")
        # model(xyzs[valid], dirs[valid]) (rendering.py:204-218): NGP.forward over the list
        # (encode + MLPs in one launch; no encoding kept: nothing goes backward)
        vren._ok(L.ngp_field_encode_mlp(_p(self.xyzs), _p(self.dirs), self.cap, self.n_valid_ptr, _p(self.sample_idx),
                                        ctypes.byref(self.grid.desc), _p(self.params16[HG.MLP_PARAMS:]),
                                        _p(self.params16), None, _p(self.sigmas), _p(self.rgbs), None, s),
                 "field_encode_mlp")
        vren._ok(L.ngp_render_test_composite(_p(self.sigmas), _p(self.rgbs), _p(self.deltas), _p(self.ts),
                                             _p(self.n_eff), self.n_rays, par, _p(self.state), _p(self.alive[par]),
                                             _p(self.alive[par ^ 1]), c_float(self.T_threshold), _p(self.opacity),
                                             _p(self.depth), _p(self.rgb), s), "render_test_composite")

    def _begin(self):
        L, s = HG._lib(), vren._stream()
        vren._ok(L.ngp_render_test_begin(self.n_rays, _p(self.state), _p(self.alive[0]), _p(self.opacity),
                                         _p(self.depth), _p(self.rgb), s), "render_test_begin")
        vren.bitfield_summary(self.bitfield, self.grid_size, out=self.summary)

    def _run(self, first):
        """K iterations (graph A, which also opens the frame) or K_tail (graph B)."""
        if first:
            self._begin()
        for k in range(self.K if first else self.K_tail):
            self._iteration(k)

    def _launch(self, first):
        if not self.use_graphs:
            self._run(first)
            return
        g = self._graphs.get(first)
        if g is None:
            g = torch.cuda.CUDAGraph()
            torch.cuda.current_stream().synchronize()
            with torch.cuda.graph(g):
                self._run(first)
            self._graphs[first] = g
            # capture does not execute: run the frame opening for real below
        g.replay()

    # --------------------------------------------------------------- API
    @torch.no_grad()
    def render_loaded(self):
        """Render the rays already in self.rays_o / rays_d / hits_t."""
        self._launch(True)
        while int(self.state[RS_ACTIVE].item()):
            self._launch(False)
        self.last_iterations = int(self.state[RS_ITERS].item())
        vren._ok(HG._lib().ngp_render_test_finish(_p(self.opacity), self.n_rays, self.bg, _p(self.rgb),
                                                  vren._stream()), "render_test_finish")
        return {"opacity": self.opacity, "depth": self.depth, "rgb": self.rgb,
                "total_samples": self.state[RS_TOTAL]}

    @torch.no_grad()
    def render(self, rays_o, rays_d, hits_t):
        """__render_rays_test(model, rays_o, rays_d, hits_t) for hits_t (n_rays,2)
        (the caller's hits_t[:, 0], near-clamped): returns views of the
        renderer's buffers (copy them to keep them past the next frame)."""
        if rays_o.shape[0] != self.n_rays:
            raise RuntimeError(f"TestRenderer was built for {self.n_rays} rays, got {rays_o.shape[0]}")
        self.rays_o.copy_(rays_o.reshape(-1, 3))
        self.rays_d.copy_(rays_d.reshape(-1, 3))
        self.hits_t.copy_(hits_t.reshape(-1, 2))
        return self.render_loaded()

    def set_camera(self, directions, center, half_size):
        """Per-pixel camera directions (H*W, 3) (datasets/ray_utils.py:7-42)
        and the scene box, for render_pose."""
        if directions.shape[0] != self.n_rays:
            raise RuntimeError("directions must have n_rays rows")
        self._dirs = directions.float().contiguous()
        self._center, self._half = center.float().contiguous(), half_size.float().contiguous()
        dev = self._dirs.device
        self._img = torch.zeros(self.n_rays, dtype=torch.int64, device=dev)
        self._pix = torch.arange(self.n_rays, dtype=torch.int64, device=dev)
        self._pose = torch.zeros(1, 3, 4, device=dev)

    @torch.no_grad()
    def render_pose(self, c2w):
        """get_rays(directions, c2w) (ray_utils.py:45-70) + AABB + near clamp
        (rendering.py:25-31) + the test loop, for one (3,4) camera-to-world pose."""
        if self._dirs is None:
            raise RuntimeError("call set_camera() first")
        self._pose.copy_(c2w.reshape(1, 3, 4))
        vren._ok(vren.lib().ngp_raygen_aabb(_p(self._dirs), _p(self._pose), _p(self._img), _p(self._pix),
                                            self.n_rays, _p(self._center), _p(self._half), c_float(NEAR_DISTANCE),
                                            _p(self.rays_o), _p(self.rays_d), _p(self.hits_t), vren._stream()),
                 "raygen_aabb")
        return self.render_loaded()


def for_model(model, n_rays, **kwargs):
    """TestRenderer over a models.networks.NGP (its fp16 shadow and bitfield)."""
    return TestRenderer(n_rays, model.grid, model._shadow.get(), model.density_bitfield, model.cascades,
                        model.scale, model.grid_size, **kwargs)
