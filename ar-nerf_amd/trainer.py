"""The reference's training step (train.py NeRFSystem, Lightning + apex +
tcnn + vren) as a chain of libngp_amd.so kernels on one MI355X per process.

One step (train.py:174-200), all on the current HIP stream, no host sync:
  raygen_aabb (ray_utils.get_rays + RayAABBIntersector + near clamp)
  -> march_train_count / scan / write (RayMarcher; sample count stays on device)
  -> field_forward (hash grid + density MLP + SH + colour MLP)
  -> composite_loss (VolumeRenderer fw + bg blend + NeRFLoss + VolumeRenderer bw)
  -> field_backward (MLP backward + hash scatter)
  -> [all_reduce(grad) over RCCL when world_size > 1]  (DDP, train.py:288)
  -> adam_step (FusedAdam + fp16 shadow + grad zeroing)
and every `update_interval` steps the occupancy update
(models/networks.py:252-281) before the batch (train.py:175-178).

Per-sample buffers are allocated once at capacity n_rays * max_samples; the
kernels read the live sample count from device memory.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.distributed as dist

import ddp
import hashgrid as HG
import vren

MAX_SAMPLES = 1024  # models/rendering.py:9
NEAR_DISTANCE = 0.01  # models/rendering.py:10
LOSS_TYPES = {"raw": 0, "mse": 1, "log": 2, "tanh": 3}


def _p(t):
    return HG._ptr(t)


STAT_STRIPES, STAT_STRIDE = 32, 16  # include/ngp_amd.h NGP_STAT_*
THROTTLE_EVERY, THROTTLE_DEPTH = 32, 4  # host run-ahead bound: <= 160 steps enqueued
COARSE_REP, COARSE_REP_LEVELS = 8, 4  # gradient replicas of the coarsest atomic levels


class NGPTrainer:
    def __init__(self, scale=0.5, batch_size=8192, lr=1e-2, num_epochs=30, steps_per_epoch=1000, loss="raw",
                 lambda_opacity=1e-3, lambda_depth=0.0, random_bg=False, exp_step_factor=None, grid_size=128,
                 update_interval=16, warmup_steps=256, max_samples=MAX_SAMPLES, sample_capacity=None, seed=4,
                 device="cuda", process_group=None, hash_backward="hybrid", bin_samples_per_ray=None, bin_level_lo=None,
                 chunk_first=64, erode=False, lambda_distortion=0.0, bin_merge_hi=None, fused_adam=True, use_graphs=True,
                 pair_steps=False, emulate_dp=False, dp_fine_buckets=2):
        self.dev = torch.device(device)
        self.scale = float(scale)
        self.batch_size = batch_size
        self.lr0, self.num_epochs, self.steps_per_epoch = lr, num_epochs, steps_per_epoch
        self.loss_type = LOSS_TYPES[loss]
        self.lambda_opacity, self.lambda_depth = lambda_opacity, lambda_depth
        self.lambda_distortion = float(lambda_distortion)  # losses.py:77-80 (opt.py:25 default 0)
        self.random_bg = random_bg
        # train.py:104-105
        self.esf = exp_step_factor if exp_step_factor is not None else (1 / 256 if scale > 0.5 else 0.0)
        self.G = grid_size
        # erode (networks.py:270-272): per-cell decay from mark_invisible_cells'
        # count_grid; train.py:178 turns it on for COLMAP scenes
        self.erode = bool(erode)
        self.count_grid = None
        self.decay_cells = None
        self._decay_for = None
        self.cascades = max(1 + int(np.ceil(np.log2(2 * scale))), 1)  # models/networks.py:27
        self.update_interval, self.warmup_steps, self.max_samples = update_interval, warmup_steps, max_samples
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world > 1 else 0
        # the data-parallel (ZeRO-1, graph-segmented) step; emulate_dp = N runs it in one process
        # with the shards of a world of N (this process = rank 0) and the collectives replaced by
        # local copies of its shard -- one rank's compute at world N without the xGMI transfers
        # (bench --emulate-dp N; only shard 0 of each bucket is stepped, so N > 1 is for timing)
        self.dp = self.world > 1 or bool(emulate_dp)
        self.dp_world = self.world if self.world > 1 else max(1, int(emulate_dp))
        dev = self.dev
        # ---- field parameters: fp32 master, fp16 shadow, Adam state, grad
        self.grid = HG.HashGrid(scale)
        init = HG.init_params(self.grid, seed=seed, device=dev)
        self.n_params = n = init.numel()
        # hash backward: "atomic": per-sample fp32 atomics (ngp_hash_backward); "binned": all
        # levels through the counting-sort path; "hybrid" (default): coarse levels
        # [0, bin_level_lo) atomic -- their in-wave run merge keeps the requests few --
        # fine levels binned (DESIGN.md "hash backward").  Defaults by scene size (measured,
        # DESIGN.md §9): one cascade (object scenes, ~70 samples/ray) 8 atomic levels + 128
        # binned samples/ray; cascaded (unbounded) scenes have ~2x the gradient-carrying
        # samples and 4 more hashed levels: all levels binned (+17 % at scale 16) with room
        # for 512 samples/ray.  Resolved before the ZeRO-1 buckets, which split at it.
        assert hash_backward in ("atomic", "binned", "hybrid")
        big = self.cascades > 1
        if bin_level_lo is None:
            bin_level_lo = 0 if big else 8
        if bin_samples_per_ray is None:
            bin_samples_per_ray = 512 if big else 128
        self.hash_backward = hash_backward
        self.bin_level_lo = 0 if hash_backward == "binned" else min(max(int(bin_level_lo), 0), self.grid.n_levels)
        # ZeRO-1 layout (ddp.zero_buckets): buffers padded to n_pad; bucket 0 =
        # [MLP | coarse levels], then the binned levels in dp_fine_buckets level
        # ranges (bin_cuts: [lo, c_1), [c_1, c_2), ...), each split where its
        # gradient is complete -- the world > 1 step accumulates the ranges in
        # turn and reduce-scatters / steps / all-gathers each range's bucket
        # on the comm stream while the next range accumulates, so only the
        # last range's chain is exposed after the backward; rank r owns shard
        # r of each bucket.  All levels binned (bin_level_lo 0): bucket 0 is
        # the MLP alone.
        self.bin_cuts = ddp.level_cuts(self.bin_level_lo, self.grid.n_levels, dp_fine_buckets)
        splits = [HG.MLP_PARAMS + 2 * int(self.grid.offsets[lv]) for lv in self.bin_cuts[:-1]] or \
            [HG.MLP_PARAMS + 2 * int(self.grid.offsets[self.grid.n_levels])]
        self.n_pad, self.buckets = ddp.zero_buckets(n, splits, self.dp_world)
        pb = torch.zeros(self.n_pad, device=dev)
        pb[:n] = init
        self._pbuf = pb
        self.params = pb[:n]  # fp32 master (a rank updates its shards only when world > 1)
        self._p16buf = pb.half()
        self.params16 = self._p16buf[:n]
        self._gbuf = torch.zeros(self.n_pad, device=dev)
        self.grad = self._gbuf[:n]
        self.exp_avg = torch.zeros(self.n_pad, device=dev)
        self.exp_avg_sq = torch.zeros(self.n_pad, device=dev)
        self.shards = [(a + (b - a) * self.rank // self.dp_world, a + (b - a) * (self.rank + 1) // self.dp_world)
                       for a, b in self.buckets]
        self._gshard = [torch.zeros(hi - lo, device=dev) for lo, hi in self.shards] if self.dp else None
        self._bk = None  # (_bucket_host)
        self.global_step = 0
        # ---- occupancy (models/networks.py:20-30, train.py:78-82)
        self.center = torch.zeros(1, 3, device=dev)
        self.half_size = torch.ones(1, 3, device=dev) * scale
        self.density_grid = torch.zeros(self.cascades, self.G ** 3, device=dev)
        self.density_bitfield = torch.zeros(self.cascades * self.G ** 3 // 8, dtype=torch.uint8, device=dev)
        ax = torch.arange(self.G, dtype=torch.int32, device=dev)
        self.grid_coords = torch.stack(torch.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3).contiguous()
        self.all_indices = vren.morton3D(self.grid_coords).long()
        self._sum_cnt = torch.zeros(2, dtype=torch.float64, device=dev)
        # device-side occupancy sampling buffers (update_density_grid)
        M2 = 2 * (self.G ** 3 // 4)
        # density_grid_tmp as 64-bit (list position, sigma) keys: last writer wins (ngp_density_scatter_last)
        self._occ_key = torch.zeros(self.density_grid.shape, dtype=torch.int64, device=dev)
        self._occ_list = torch.empty(self.G ** 3, dtype=torch.int32, device=dev)
        self._occ_count = torch.zeros(1, dtype=torch.int64, device=dev)
        self._occ_list_ws = torch.empty((vren.lib().ngp_occupied_cells_workspace(self.G ** 3) + 3) // 4,
                                        dtype=torch.int32, device=dev)
        self._occ_xyz = torch.empty(M2, 3, device=dev)
        self._occ_flat = torch.empty(M2, dtype=torch.int64, device=dev)
        self._occ_sig = torch.empty(M2, device=dev)
        # only the samples whose sigma the update keeps are evaluated (ngp_occupancy_keep:
        # a cell's last draw; bit-identical grid, 362 -> 302 us per update; occ_keep = False
        # (tests): all 2M, as the reference evaluates them)
        self.occ_keep = True
        self._occ_mark = torch.empty((self.G ** 3 + 15) // 16, 4, dtype=torch.int32, device=dev)
        self._occ_kept = torch.empty(M2, dtype=torch.int32, device=dev)
        self._occ_kept_n = torch.zeros(1, dtype=torch.int64, device=dev)
        self._occ_ws = torch.empty((vren.lib().ngp_occupancy_sorted_workspace(M2 // 2) + 7) // 8, dtype=torch.float64,
                                   device=dev)
        self.threshold = torch.zeros(2, device=dev)
        # ---- per-step buffers
        R = batch_size
        if sample_capacity is not None:  # never let a ray overflow the sample buffers
            self.max_samples = max_samples = max(1, min(max_samples, sample_capacity // R))
        cap = R * max_samples
        self.cap = cap
        f = dict(device=dev, dtype=torch.float32)
        # Two sets of ray / march buffers: the next batch is marched on a side
        # stream while the current batch's field, loss, backward and Adam run.
        self.msets = [self._march_buffers(R, cap, f, self.density_bitfield.numel()) for _ in range(2)]
        self.cur = 0
        self.march_stream = torch.cuda.Stream(device=dev)
        self._pending = None  # (set index, event) of a batch marched ahead
        self.n_prefetched = 0
        self.no_prefetch = False  # (diagnostics) march every batch inline
        # pair_steps: two consecutive steady-state steps per graph replay (_replay_pair)
        self.pair_steps = bool(pair_steps)
        self._ran_ahead = False
        self._pair_key = None
        self._bind(self.msets[0])
        self.sigmas, self.rgbs = torch.zeros(cap, **f), torch.zeros(cap, 3, **f)  # (finite where never evaluated)
        # saved encoding: pair-major (8, cap, 4) for the split forward, else row-major (cap, 32)
        # hybrid hash backward: the atomic coarse levels run on their own
        # stream beside the binned fine levels (disjoint gradient ranges;
        # memory-side atomics vs LDS-bound passes overlap)
        # (Single process) the Adam of the MLP + coarse levels runs on that side stream
        # right after the coarse levels' backward, beside the binned levels'
        # accumulation, whose own FusedAdam is fused into it (+5 %,
        # profiles/r02/ab/fused_adam.txt; bit-identical to one FusedAdam launch after the
        # backward, which fused_adam=False restores).
        # (its own stream: sharing the march's side stream -- their work never overlaps in time --
        # measured 6 % slower, the graph's branches then map onto fewer hardware queues)
        self.bwd_stream = torch.cuda.Stream(device=dev)
        self.fused_adam = bool(fused_adam)
        self._adam_hi = None
        # the training forward: encode + MLPs in one launch (ngp_field_encode_mlp), the
        # pair-major encoding kept for the backward (+1.8 %, profiles/r02/ab/fused_field.txt)
        self.enc = torch.empty(8 * cap * 4, dtype=torch.float16, device=dev)
        self.dsig, self.drgb = torch.empty(cap, **f), torch.empty(cap, 3, **f)
        self.denc = torch.empty(cap, 32, **f)
        self.out_rgb, self.out_op = torch.empty(R, 3, **f), torch.empty(R, **f)
        self.out_depth, self.out_loss = torch.empty(R, **f), torch.empty(R, **f)
        # running totals: [0] marched, [1] composited (vr_samples), [2] gradient-carrying,
        # [3] field-evaluated samples
        # striped counters (ngp_composite_loss: NGP_STAT_STRIPES x NGP_STAT_STRIDE), written by the
        # compositing kernel only; field-evaluated samples in their own 128-B line (eval_stats[0],
        # main stream only: the list launches of the step that evaluates them add both rounds'
        # totals, device-scope atomics) -- no counter word shares a cache line with a writer on
        # another stream
        self.stats = torch.zeros(STAT_STRIPES * STAT_STRIDE, dtype=torch.int64, device=dev)
        self.eval_stats = torch.zeros(STAT_STRIDE, dtype=torch.int64, device=dev)
        # chunked field evaluation (ngp_chunk_counts): first `chunk_first` samples of
        # every row, then the rest of the rows not yet terminated (0 = every sample).
        # (More rounds evaluate 22 % fewer samples, but each extra encode launch costs
        # more than it saves: profiles/r02/ab/chunk_rounds.txt)
        self.chunk_first = int(chunk_first)
        self.eval_counts = torch.empty(R, dtype=torch.int32, device=dev)
        # round-2 list in one launch (counts + look-back scan + map): its look-back workspace, zeroed once
        self._cs_ws = torch.zeros((vren.lib().ngp_chunk_segments_workspace(R) + 7) // 8, dtype=torch.int64,
                                  device=dev)
        # row forward (the default since round 4: +2 %, 9 of 9 alternating pairs,
        # profiles/r04/ab/row_forward_variants.txt): round 1 one wave per non-empty row with the
        # row's transmittance in its epilogue, which appends the row's round-2 samples to the
        # round-2 list itself (ngp_field_forward_first: no list launch); row_forward = 0 (tests)
        # or chunk_first != 64: the two-round lists below
        self.row_forward = 1
        assert self.row_forward in (0, 1)
        # where the next batch's march forks off the step: after the row forward's round 1 on the
        # single-cascade (Lego-shaped) scenes (round 1 runs alone, the march beside round 2 /
        # composite / MLP backward: +2.1 %, 6 of 6 pairs, profiles/r04/ab/march_fork_position.txt);
        # at the step's start on cascaded scenes, whose march is 3/4 of a forward-sized step and
        # beside the MLP backward slows it 1.7x (garden-shaped: -6 %, profiles/r04/ab/garden_r4.txt);
        # (march_at = start | r1 | fwd | mlp: diagnostics, scripts/diag/skip_cost.py)
        self.march_at = "r1" if self.cascades == 1 else "start"
        # round 1's coarse levels 0-7 encoded ahead (the next batch's first chunks, once the MLP + coarse
        # levels' Adam of this step has run, beside the binned levels' accumulation): round 1 then gathers
        # only levels 8-15 (pre_coarse = False, tests: off)
        self.pre_coarse = True
        self.pre_levels = 8  # (the kernel's PRE_LEVELS: levels 0-7, final once the side stream's Adam has run)
        assert self.march_at in ("start", "r1", "fwd", "mlp")
        self.eval_total = torch.zeros(1, dtype=torch.int64, device=dev)
        self.eval_idx = torch.empty(cap, dtype=torch.int32, device=dev)
        self.act_start = torch.empty(R, dtype=torch.int64, device=dev)
        # gradient-carrying samples (up to each ray's termination): index map
        self.n_active = torch.empty(R, dtype=torch.int32, device=dev)
        self.n_active_total = torch.zeros(1, dtype=torch.int64, device=dev)
        self.sample_idx = torch.empty(cap, dtype=torch.int32, device=dev)
        # binned hash backward: workspace for bin_samples_per_ray gradient-
        # carrying samples per ray on average (1 KiB each; the rest take the
        # atomic path, still exact)
        # binned levels [bin_level_lo, bin_merge_hi) merge runs of equal corner pairs along a ray
        # in the record write (one single-entry record per corner for a whole run: fewer records
        # written and accumulated).  Default for one-cascade scenes: levels 8-10 (consecutive
        # samples share a level-10 cell ~3 times on Lego; +1.2 % mean of 5 alternating pairs, 4 of 5,
        # profiles/r03/ab/bin_merge_hi.txt); cascaded scenes, whose every level is binned: all 16
        # (garden-shaped step 7.0 -> 8.3 M rays/s, profiles/r03/ab/garden_bin_merge_hi.txt).
        if bin_merge_hi is None:
            bin_merge_hi = 16 if big else 11
        self.bin_merge_hi = int(bin_merge_hi)
        if hash_backward != "atomic":
            self.bin_max_samples = R * bin_samples_per_ray
            nbytes = HG._lib().ngp_hash_backward_binned_workspace(self.bin_max_samples)
            self.bin_ws = torch.empty((nbytes + 255) // 256, 64, dtype=torch.int32, device=dev)
        # coarse atomic levels [0, coarse_rep_levels) add into coarse_rep replicas of their
        # gradient range, folded afterwards (ngp_hash_backward_levels_rep): the coarsest
        # levels are a few hundred KB every sample touches (levels 0-3 x 8 measured best,
        # profiles/r02/ab/coarse_replicas.txt); single process: folded by the MLP + coarse
        # levels' Adam launch
        self.coarse_rep = COARSE_REP
        self.coarse_rep_levels = min(COARSE_REP_LEVELS, self.bin_level_lo) if hash_backward != "atomic" else 0
        self.rep_buf = None
        if self.coarse_rep > 0 and self.coarse_rep_levels > 0:
            nrep = HG._lib().ngp_hash_backward_rep_floats(HG.ctypes.byref(self.grid.desc), self.coarse_rep_levels,
                                                          self.coarse_rep)
            self.rep_buf = torch.zeros(nrep, **f)
        self.bg = torch.ones(3, **f) if self.esf == 0 else torch.zeros(3, **f)  # models/rendering.py:287-296
        self._bg_rand = torch.zeros(3, **f)
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(1000 + seed + self.rank)
        # ngp_sample_batch key: one seed for all ranks, rank r draws rays [r*R, (r+1)*R) of the global
        # batch (independent uniform draws per ray, as the reference's per-rank DataLoaders)
        self.sample_seed = (1000003 * (seed + 1)) & 0xFFFFFFFFFFFFFFFF
        # occupancy draws: rank-independent (every rank draws the same cells and
        # jitter; each evaluates its shard), so any world size builds one grid
        self.occ_seed = ((1000003 * (seed + 1)) ^ 0x5DEECE66D) & 0xFFFFFFFFFFFFFFFF
        self.occ_gen = torch.Generator(device=dev)
        self.occ_gen.manual_seed(2000 + seed)
        # device step counters: [0] Adam steps taken, [1] batches drawn (RNG
        # counter), [2] device-sampled occupancy updates (their RNG counter)
        self.dctr = torch.zeros(3, dtype=torch.int64, device=dev)
        # (Measured and removed in round 5's clean-up, DESIGN.md §9: a completion ticket by which
        # the step's Adam launches advanced dctr themselves, -2..-4 %; the coarse levels scattered
        # by the MLP backward launch, -4 %.)
        self._updated_for = -1  # global step whose occupancy update already ran (end of the previous graph)
        self.lr_dev = torch.full((1,), float(lr), device=dev)
        self._lr_set = float(lr)
        # HIP graphs of the steady-state step, one per buffer set (see train_step)
        self.use_graphs = bool(use_graphs)
        self._graphs = {}
        self._graph_post = {}
        self.L = vren.lib()
        HG._lib()
        # {"field_fwd"|"mlp_bwd"|"hash_bwd"|stage: (start, end) torch.cuda.Event} (eager diagnostics)
        self.kernel_events = None
        # ktimer.KernelTimer (bench): graph replays carry HIP events around every kernel
        self.timer = None
        # world > 1 graph replays run as segments with the collectives between them
        self._segmented = False
        self.comm_stream = torch.cuda.Stream(device=dev) if torch.cuda.is_available() else None
        self._throttle_q = []  # events of every THROTTLE_EVERY-th step (train_step)

    @staticmethod
    def _march_buffers(R, cap, f, cap_bits):
        dev = f["device"]
        return dict(rays_o=torch.empty(R, 3, **f), rays_d=torch.empty(R, 3, **f), hits_t=torch.empty(R, 2, **f),
                    noise=torch.empty(R, **f), counts=torch.empty(R, dtype=torch.int32, device=dev),
                    img_idxs=torch.empty(R, dtype=torch.int64, device=dev),
                    pix_idxs=torch.empty(R, dtype=torch.int64, device=dev), rgb_gt=torch.empty(R, 3, **f),
                    occ_summary=torch.empty(2 * ((cap_bits + 255) // 256), dtype=torch.int32, device=dev),
                    rays_a=torch.empty(R, 3, dtype=torch.int64, device=dev),
                    n_samples=torch.zeros(1, dtype=torch.int64, device=dev),
                    xyzs=torch.empty(cap, 3, **f), dirs=torch.empty(cap, 3, **f), deltas=torch.empty(cap, **f),
                    ts=torch.empty(cap, **f), slot_t=torch.empty(cap, **f), slot_dt=torch.empty(cap, **f),
                    # the chunked forward's round-1 list (first chunk_first samples of every row),
                    # built by the march itself (_march): off the step's critical path
                    eval_idx1=torch.empty(cap, dtype=torch.int32, device=dev),
                    eval_total1=torch.zeros(1, dtype=torch.int64, device=dev),
                    act_start1=torch.empty(R, dtype=torch.int64, device=dev), eval1_K=0,
                    # row-forward round 1: the non-empty rows (built by the march), the round-2 counts
                    rows_ne=torch.empty(R, dtype=torch.int32, device=dev),
                    n_rows_ne=torch.zeros(1, dtype=torch.int64, device=dev),
                    eval_total2=torch.zeros(1, dtype=torch.int64, device=dev),
                    # round 1's coarse levels 0-7 already in self.enc for this set's first chunks
                    # (ngp_field_encode_first_coarse, run by the previous step beside its accumulation)
                    pre_ready=False)

    def _bind(self, m):
        for k, v in m.items():
            setattr(self, k, v)

    # ------------------------------------------------------------ schedule
    def lr(self):
        """CosineAnnealingLR(T_max=num_epochs, eta_min=lr/30), stepped per epoch (train.py:149-151)."""
        e = self.global_step // self.steps_per_epoch
        eta_min = self.lr0 / 30
        return eta_min + (self.lr0 - eta_min) * (1 + math.cos(math.pi * e / self.num_epochs)) / 2

    # ------------------------------------------------------ occupancy grid
    @torch.no_grad()
    def mark_invisible_cells(self, K, poses, img_wh, chunk=64 ** 3):
        """models/networks.py:209-250 (once, before training): density -1 for
        cells no camera sees (or too near one), and count_grid = the fraction
        of cameras that see each cell, from which the erode decay is derived."""
        K, poses = K.to(self.dev), poses.to(self.dev)
        N_cams = poses.shape[0]
        self.count_grid = torch.zeros_like(self.density_grid)
        w2c_R = poses[:, :3, :3].transpose(1, 2)
        w2c_T = -w2c_R @ poses[:, :3, 3:]
        for c in range(self.cascades):
            indices, coords = self.all_indices, self.grid_coords
            for i in range(0, len(indices), chunk):
                xyzs = coords[i:i + chunk] / (self.G - 1) * 2 - 1
                s = min(2 ** (c - 1), self.scale)
                half_grid_size = s / self.G
                xyzs_w = (xyzs * (s - half_grid_size)).T
                xyzs_c = w2c_R @ xyzs_w + w2c_T
                uvd = K @ xyzs_c
                uv = uvd[:, :2] / uvd[:, 2:]
                in_image = (uvd[:, 2] >= 0) & (uv[:, 0] >= 0) & (uv[:, 0] < img_wh[0]) & (uv[:, 1] >= 0) & \
                           (uv[:, 1] < img_wh[1])
                covered_by_cam = (uvd[:, 2] >= NEAR_DISTANCE) & in_image
                count = covered_by_cam.sum(0) / N_cams
                self.count_grid[c, indices[i:i + chunk]] = count
                too_near_to_any_cam = ((uvd[:, 2] < NEAR_DISTANCE) & in_image).any(0)
                valid_mask = (count > 0) & (~too_near_to_any_cam)
                self.density_grid[c, indices[i:i + chunk]] = torch.where(valid_mask, 0., -1.)
        self.decay_cells = vren.erode_decay(self.count_grid).to(self.dev)
        self._decay_for = 0.95

    @torch.no_grad()
    def _occ_draw(self, c, density_threshold, s):
        """The parameter-independent head of a past-warmup update of cascade c:
        the occupied-cell list from density_grid, the sorted draws, and (keep)
        the kept draws -- launched on stream s.  Returns (lo, hi, M)."""
        L, G = self.L, self.G
        sc = min(2 ** (c - 1), self.scale)
        half_grid_size = sc / G
        M = G ** 3 // 4
        vren._ok(L.ngp_occupied_cells(_p(self.density_grid[c]), G ** 3, ctypes_float(density_threshold),
                                      _p(self._occ_list), _p(self._occ_count), _p(self._occ_list_ws), s),
                 "occupied_cells")
        lo, hi = ddp.shard_range(2 * M, self.rank, self.world)
        # (keep: every rank draws the whole list, positions = list positions, so that
        # the kept ones -- a cell's last draw -- are found over the whole list)
        glo, ghi = (0, 2 * M) if self.occ_keep else (lo, hi)
        args = (self.occ_seed, _p(self.dctr[2:]), c, G, M, ctypes_float(sc - half_grid_size),
                ctypes_float(half_grid_size), _p(self._occ_list), _p(self._occ_count), glo, ghi)
        # each half's cells drawn in ascending order: the density forward's waves
        # stay cache-local (1.8x faster than draw order, scripts/diag/density_order.py)
        vren._ok(L.ngp_occupancy_samples_sorted(*args, _p(self._occ_ws), _p(self._occ_xyz),
                                                _p(self._occ_flat), s), "occupancy_samples_sorted")
        if self.occ_keep:
            vren._ok(L.ngp_occupancy_keep(_p(self._occ_flat), M, c * G ** 3, G ** 3, lo, hi,
                                          _p(self._occ_mark), _p(self._occ_kept), _p(self._occ_kept_n), s),
                     "occupancy_keep")
        return lo, hi, M

    def update_density_grid(self, density_threshold, warmup=False, decay=0.95, erode=None, jitter=None,
                            drawn=False):
        """models/networks.py:252-281.  Past warmup the cells are drawn on device
        (ngp_occupied_cells + ngp_occupancy_samples: no host sync, so the update
        can sit inside a captured graph).  Multi-GPU: each rank evaluates its
        1/world share of the (identically drawn) cells and the cell maxima are
        combined with one MAX all-reduce, so every rank packs an identical
        bitfield.  erode (default: the trainer's setting) decays each cell by
        clamp(decay**(1/count_grid), 0.1, 0.95) (networks.py:270-272).
        jitter (tests): the warm-up's U[0,1) jitter per cell (C, G^3, 3) in
        grid_coords order instead of the trainer's own draw.  drawn (one
        cascade, past warmup): _occ_draw already ran for this update (the
        captured step launches it beside the step before the update)."""
        C, G = self.cascades, self.G
        erode = self.erode if erode is None else erode
        if erode and self.decay_cells is None:
            raise RuntimeError("update_density_grid(erode=True) needs count_grid: call mark_invisible_cells first")
        if erode and decay != self._decay_for:  # (host evaluation: not inside a graph capture)
            self.decay_cells = vren.erode_decay(self.count_grid, decay).to(self.dev)
            self._decay_for = decay
        L, s = self.L, vren._stream()
        key = self._occ_key  # zero on entry; the EMA consumes (re-zeroes) it
        for c in range(C):
            sc = min(2 ** (c - 1), self.scale)
            half_grid_size = sc / G
            if warmup:  # get_all_cells (networks.py:167-179)
                # the jitter is drawn for every cell from a rank-independent
                # generator, then each rank evaluates its share of the cells:
                # any world size builds the same grid
                jit = (torch.rand(self.grid_coords.shape, device=self.dev, generator=self.occ_gen) if jitter is None
                       else jitter[c].to(self.dev))
                lo, hi = ddp.shard_range(self.grid_coords.shape[0], self.rank, self.world)
                indices, coords = self.all_indices[lo:hi], self.grid_coords[lo:hi]
                xyzs_w = (coords / (G - 1) * 2 - 1) * (sc - half_grid_size)
                xyzs_w += (jit[lo:hi] * 2 - 1) * half_grid_size
                sig, _ = HG.density_forward(xyzs_w.float().contiguous(), self.grid, self.params16)
                flat = (indices + c * G ** 3).contiguous()
                n = flat.shape[0]
            else:  # sample_uniform_and_occupied_cells (networks.py:181-207), on device
                if drawn:
                    assert C == 1, "update_density_grid(drawn=True) needs one cascade"
                    M = G ** 3 // 4
                    lo, hi = ddp.shard_range(2 * M, self.rank, self.world)
                else:
                    lo, hi, M = self._occ_draw(c, density_threshold, s)
                n = hi - lo
                if self.occ_keep:
                    # encode + density net of the kept samples only (sigma written at their position)
                    vren._ok(HG._lib().ngp_field_encode_mlp(_p(self._occ_xyz), None, n, _p(self._occ_kept_n),
                                                            _p(self._occ_kept), HG.ctypes.byref(self.grid.desc),
                                                            _p(self.params16[HG.MLP_PARAMS:]), _p(self.params16),
                                                            None, _p(self._occ_sig), None, None, s),
                             "density_encode_mlp")
                    vren._ok(L.ngp_density_scatter_kept(_p(self._occ_kept), _p(self._occ_kept_n), n,
                                                        _p(self._occ_flat), _p(self._occ_sig), 0, _p(key), s),
                             "density_scatter_kept")
                    continue
                # encode + density net in one launch (no encoding kept)
                vren._ok(HG._lib().ngp_field_encode_mlp(_p(self._occ_xyz), None, n, None, None,
                                                        HG.ctypes.byref(self.grid.desc),
                                                        _p(self.params16[HG.MLP_PARAMS:]), _p(self.params16), None,
                                                        _p(self._occ_sig), None, None, s), "density_encode_mlp")
                sig, flat = self._occ_sig, self._occ_flat
            # density_grid_tmp[c, indices] = sigma, list positions lo + i (rank shards)
            vren._ok(L.ngp_density_scatter_last(_p(flat), _p(sig), n, lo, _p(key), s), "density_scatter_last")
        if not warmup:
            vren._ok(L.ngp_counters_inc(_p(self.dctr[2:]), 1, s), "counters_inc")
        ddp.combine_density_tmp_(key, self.pg)
        st = L.ngp_density_grid_ema(_p(self.density_grid), _p(key), self.density_grid.numel(), ctypes_float(decay),
                                    _p(self.decay_cells) if erode else None, ctypes_float(density_threshold),
                                    _p(self._sum_cnt), _p(self.threshold), s)
        vren._ok(st, "density_grid_ema")
        ddp.sync_threshold_(self.threshold, self.pg)  # identical threshold on every rank
        vren.packbits(self.density_grid, self.threshold[:1], self.density_bitfield)

    def _march(self, k, src, directions, poses, stream):
        """Ray generation + AABB + single-pass march of one batch into buffer
        set k.  src = ("idx", img_idxs, pix_idxs, noise | None): rays of the
        given pixels (noise drawn from self.gen when None); or ("sample", add,
        gt_u8): the whole batch drawn on device (ngp_sample_batch_dev: pixels,
        ground truth, noise from Philox keyed by (seed, batch counter + add),
        the counter in device memory so a replayed graph draws fresh batches)."""
        m = self.msets[k]
        m["pre_ready"] = False  # (the set's coarse-level round-1 encoding is stale from here on)
        L, R = self.L, self.batch_size
        side = stream is self.march_stream
        with torch.cuda.stream(stream):
            if side:
                self._ev("march_side", 0, stream)
            s = HG.c_void_p(stream.cuda_stream)
            if src[0] == "sample":
                _, add, gt = src
                n_img, hw = gt.shape[0], gt.shape[1]
                assert gt.dtype in (torch.uint8, torch.float32) and gt.is_contiguous()
                vren._ok(L.ngp_sample_batch_dev(self.sample_seed, _p(self.dctr[1:]), add, self.rank * R, _p(gt),
                                                int(gt.dtype == torch.float32), n_img, hw,
                                                _p(directions), _p(poses), R, _p(self.center), _p(self.half_size),
                                                ctypes_float(NEAR_DISTANCE), _p(m["img_idxs"]), _p(m["pix_idxs"]),
                                                _p(m["rgb_gt"]), _p(m["noise"]), _p(m["rays_o"]), _p(m["rays_d"]),
                                                _p(m["hits_t"]), s), "sample_batch")
            else:
                _, img_idxs, pix_idxs, noise = src
                assert img_idxs.shape[0] == R
                vren._ok(L.ngp_raygen_aabb(_p(directions), _p(poses), _p(img_idxs), _p(pix_idxs), R, _p(self.center),
                                           _p(self.half_size), ctypes_float(NEAR_DISTANCE), _p(m["rays_o"]),
                                           _p(m["rays_d"]), _p(m["hits_t"]), s), "raygen")
                if noise is None:
                    torch.rand(R, out=m["noise"], generator=self.gen)  # custom_functions.py:83
                else:
                    m["noise"].copy_(noise)
            # the bitfield's block summary, rebuilt per march: any writer of
            # density_bitfield (update_density_grid, tests, tools) stays valid
            vren.bitfield_summary(self.density_bitfield, self.G, out=m["occ_summary"])
            vren._ok(L.ngp_march_train_slots(_p(m["rays_o"]), _p(m["rays_d"]), _p(m["hits_t"]), R,
                                             _p(self.density_bitfield), self.cascades, self.G,
                                             ctypes_float(self.scale), ctypes_float(self.esf), _p(m["noise"]),
                                             self.max_samples, _p(m["counts"]), _p(m["rays_a"]),
                                             _p(m["n_samples"]), _p(m["slot_t"]), _p(m["slot_dt"]),
                                             _p(m["occ_summary"]), s), "march_slots")
            vren._ok(L.ngp_march_train_compact(_p(m["rays_o"]), _p(m["rays_d"]), _p(m["rays_a"]), R,
                                               _p(m["slot_t"]), _p(m["slot_dt"]), self.max_samples, _p(m["xyzs"]),
                                               _p(m["dirs"]), _p(m["deltas"]), _p(m["ts"]), s), "march_compact")
            # round 1 of the chunked forward: the list of each row's first chunk_first samples
            # (counts min(N_r, K) + scan + list in one launch), here beside the previous step
            # instead of at the head of this batch's step; its length eval_total1 is counted
            # into eval_stats by the round-2 list launch of the step that evaluates it
            K = self.chunk_first
            rows = self._rows_fwd(K)
            m["eval1_K"] = K if (K > 0 and R <= 65536 and not rows) else 0
            if m["eval1_K"]:
                vren._ok(L.ngp_ray_segments_capped(_p(m["rays_a"]), R, K, _p(m["act_start1"]), _p(m["eval_total1"]),
                                                   None, _p(m["eval_idx1"]), s), "segments_capped")
            elif rows:
                vren._ok(L.ngp_rays_nonempty(_p(m["rays_a"]), R, _p(m["rows_ne"]), _p(m["n_rows_ne"]), None,
                                             _p(m["eval_total2"]), s), "rays_nonempty")
            if side:
                self._ev("march_side", 1, stream)

    def _rows_fwd(self, K):
        """The row forward runs the chunked evaluation (its first chunk is one
        wave: chunk_first 64; other chunk sizes take the two-round lists)."""
        return bool(self.row_forward) and K == 64

    def march_fork_point(self):
        """Where the next batch's march forks off the step (march_at; "r1"
        needs the row forward's own round-1 launch, else the step's start)."""
        if self.march_at == "r1" and not (self._rows_fwd(self.chunk_first) and self.row_forward == 1):
            return "start"
        return self.march_at

    def _can_prefetch(self):
        """The next batch may be marched ahead unless the next step begins with
        an occupancy update (that batch must see the new bitfield)."""
        return (self._pending is None and (self.global_step + 1) % self.update_interval != 0
                and not self.no_prefetch)

    def prefetch(self, src, directions, poses):
        """March the NEXT batch into the idle buffer set on the side stream so
        it overlaps the current step's field / loss / backward / Adam.  Called
        by step() once the current set is bound: everything the side stream
        needs (the next batch's indices, the bitfield, the idle set's last
        readers = the previous step's backward) is already enqueued on the
        main stream, which one event captures.  (Callers that edit
        density_bitfield between steps must not pass next_batch; callers that
        edit params / params16 between steps call invalidate_pre_encode, or
        use load_params.)"""
        if not self._can_prefetch():
            return False
        k = 1 - self.cur
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream())
        self.march_stream.wait_event(ready)
        self._march(k, src, directions, poses, self.march_stream)
        ev = torch.cuda.Event()
        ev.record(self.march_stream)
        self._pending = (k, ev)
        self.n_prefetched += 1
        return True

    def invalidate_pre_encode(self):
        """Forget every buffer set's round-1 coarse-level encoding done ahead
        (pre_ready): it was encoded from the parameters of its time, so any
        write to params / params16 between steps (checkpoint load, state
        transplant, hand edits) must call this (load_params does) -- the next
        round 1 then gathers all 16 levels itself instead of mixing levels 0-7
        of the old parameters with 8-15 of the new."""
        for m in self.msets:
            m["pre_ready"] = False

    @torch.no_grad()
    def load_params(self, params, params16=None):
        """Overwrite the fp32 master (and the fp16 shadow: params16, or the
        master rounded) between steps, invalidating the pre-encoded round 1."""
        n = self.n_params
        self.params.copy_(params[:n].to(self.params))
        self.params16.copy_(params[:n].half() if params16 is None else params16[:n].to(self.params16))
        self.invalidate_pre_encode()

    def drain(self):
        """Order the current stream after a batch marched ahead on the side
        stream (the batch stays pending for the next train_step)."""
        if self._pending is not None and self._pending[1] is not None:
            torch.cuda.current_stream().wait_event(self._pending[1])

    def _ev(self, name, i, stream=None):
        """Breakdown instrumentation (eager steps only): i = 0 opens a new
        (start, end) HIP-event pair for `name` on `stream` (default: the
        current one), i = 1 closes the last one.  kernel_events maps a name to
        the list of its pairs (a kernel launched twice per step has two)."""
        ev = self.kernel_events
        if ev is None:
            return
        st = stream if stream is not None else torch.cuda.current_stream()
        if i == 0:
            pair = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            pair[0].record(st)
            ev.setdefault(name, []).append(pair)
        else:
            ev[name][-1][1].record(st)

    # ---------------------------------------------------------------- step
    def reset_stats(self):
        """Zero the sample counters (stat_totals) on the current stream."""
        self.stats.zero_()
        self.eval_stats.zero_()

    def stat_totals(self):
        """(marched, composited, active, evaluated) samples of the steps run
        since reset_stats() (sum over the stripes; evaluated = both chunked
        rounds, 0 when chunk_first == 0: every marched sample is evaluated)."""
        t = [int(v) for v in self.stats.view(STAT_STRIPES, STAT_STRIDE)[:, :3].sum(0).tolist()]
        return t + [int(self.eval_stats[0])]

    def step(self, img_idxs, pix_idxs, rgb_gt, directions, poses, noise=None, apply_adam=True, next_batch=None):
        """One training step on a batch (train.py:174-200).  img/pix (R) i64,
        rgb_gt (R,3) f32, directions (HW,3), poses (n_img,3,4), all on device.
        next_batch = (img, pix) of the following step: marched ahead on the
        side stream."""
        nxt = None if next_batch is None else ("idx", next_batch[0], next_batch[1], None)
        return self._step(("idx", img_idxs, pix_idxs, noise), rgb_gt, directions, poses, apply_adam, nxt)

    def train_step(self, gt, directions, poses, allow_pair=True):
        """One training step on a batch drawn on device from the training set
        (gt (n_img, HW, 3) u8 images -- or f32 colours, e.g. alpha-blended
        data -- directions (HW,3), poses (n_img,3,4)):
        the reference's DataLoader + training_step with nothing on the host.
        The next step's batch is drawn and marched ahead on the side stream.
        Steady-state steps (batch already marched ahead, no occupancy update
        now or next step) replay a captured HIP graph of the whole step
        (NGP_GRAPHS=0: always eager).  pair_steps: a call may run this step
        AND the next in one replay (the next call then only advances the
        count); allow_pair=False keeps this call to one step, e.g. the last
        step of a measured window."""
        gs, ui = self.global_step, self.update_interval
        self._throttle()
        if self._ran_ahead:  # this step was the second half of the previous call's two-step graph
            if self._pair_key != (gt.data_ptr(), directions.data_ptr(), poses.data_ptr(), gt.shape, gt.dtype):
                raise RuntimeError("pair_steps: the second step of a two-step graph replay must be given the same "
                                   "gt / directions / poses as the first (it already ran on them)")
            self._ran_ahead = False
            self.global_step += 1
            return self.out_loss
        if (self.use_graphs and self._pending is not None and (gs % ui != 0 or self._updated_for == gs)
                and gs >= self.warmup_steps and self.kernel_events is None and not self.no_prefetch):
            if (allow_pair and self.pair_steps and not self.dp and self.timer is None and (gs + 1) % ui != 0
                    and (gs + 2) % ui != 0 and gs // self.steps_per_epoch == (gs + 1) // self.steps_per_epoch):
                return self._replay_pair(gt, directions, poses)
            return self._replay(gt, directions, poses, (gs + 1) % ui == 0)
        return self._step(("sample", 0, gt), None, directions, poses, True, ("sample", 1, gt))

    def _throttle(self):
        """Back-pressure on the host: an event every THROTTLE_EVERY steps, and
        before enqueueing more the host waits for the one THROTTLE_DEPTH events
        back, so at most ~160 steps are ever enqueued ahead of the GPU (that
        step finished long ago when the GPU is the bottleneck: the queue never
        drains, measured no slower).  It bounds the host's lead -- a caller
        that stops, reads out_loss or edits the scene waits for at most that
        many steps, and the runtime's command queue stays bounded -- and is not
        a fault fix.  (The memory faults once seen in long graph-replayed runs
        had another cause, found and fixed in d87e59d: a captured
        hipMemsetAsync of the occupancy-list counter was not ordered before the
        list kernel, which then read stale counts and wrote past the list;
        counters are now zeroed by a kernel node, and the list is built from
        per-block counts with no counter to zero at all.)"""
        if self.global_step % THROTTLE_EVERY:
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self._throttle_q.append(ev)
        if len(self._throttle_q) > THROTTLE_DEPTH:
            self._throttle_q.pop(0).synchronize()

    def _set_lr(self):
        lr = self.lr()
        if lr != self._lr_set:
            self.lr_dev.fill_(lr)
            self._lr_set = lr

    def _replay(self, gt, directions, poses, update_after):
        """Graph-replayed steady-state step for the batch pending in set k.
        Plain variant: the step's kernels on the capture stream, the next
        batch's march forked onto the side stream and joined before the end,
        the device counters advanced last.  update_after (the next step opens
        with an occupancy update): no fork; after the step the update
        (networks.py:252-281, cells drawn on device) and then the next batch's
        march against the new bitfield, all inside the graph."""
        k, ev = self._pending
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        self._set_lr()
        key = (k, bool(update_after), gt.data_ptr(), directions.data_ptr(), poses.data_ptr(), gt.shape, gt.dtype,
               self.msets[k]["pre_ready"])
        if not self.dp:
            self._run_graph(key, lambda: self._graph_body(k, gt, directions, poses, update_after))
        else:
            if self._capture_comm():  # the whole step, its collectives included, in ONE graph
                self._run_graph(key + ("whole",), lambda: self._dp_sequence(k, gt, directions, poses, update_after,
                                                                          lambda sub, fn: fn()))
            else:  # collectives between graph segments
                self._dp_sequence(k, gt, directions, poses, update_after,
                                  lambda sub, fn: self._run_graph(key + sub, fn))
            if update_after:  # (every 16 steps) eager: the update has its own collectives
                self.update_density_grid(0.01 * MAX_SAMPLES / 3 ** 0.5, warmup=False)
                self._march(1 - k, ("sample", 0, gt), directions, poses, torch.cuda.current_stream())
        self.cur = k
        self._bind(self.msets[k])
        self._pending = (1 - k, None)  # marched (and joined) inside the graph
        self.n_prefetched += 1
        self.global_step += 1
        if update_after:
            self._updated_for = self.global_step
        return self.out_loss

    def _capture_comm(self):
        """The data-parallel step's collectives captured into the step's graph
        (one replay per step, no segment boundaries): emulated worlds (local
        copies) and a world-1 RCCL group (tests) by default.  A real world > 1
        keeps the graph segments with eager RCCL calls between them unless
        NGP_DP_CAPTURE=1 opts in (captured multi-rank RCCL
        collectives, with the occupancy update's eager ones between the
        replays, have not run on a multi-GPU node; the segmented step measured
        ~4 % slower emulated).  gloo stages device tensors
        through the host and cannot be captured.  NGP_DP_CAPTURE=0: segments
        always."""
        opt = os.environ.get("NGP_DP_CAPTURE", "")
        if opt == "0":
            return False
        if not ddp.comm_active(self.pg):
            return True
        if dist.get_backend(self.pg) != "nccl":
            return False
        return self.world == 1 or opt == "1"

    def _dp_sequence(self, k, gt, directions, poses, update_after, run):
        """The data-parallel step (ZeRO-1, per-bucket pipeline): run(sub, fn)
        executes one graph segment -- its own graph (segmented replay,
        collectives between the segments) or inline (the whole step captured
        as one graph).  Compute segment; coarse levels on the side stream ->
        bucket 0's reduce-scatter, Adam, all-gather on the comm stream while
        the binned levels run range by range (bin_cuts), each range's bucket
        following it on the comm stream while the next range accumulates;
        joined; device counters advanced."""
        cs, comm = torch.cuda.current_stream(), self.comm_stream
        run(("compute",), lambda: self._segment_compute(k, gt, directions, poses, update_after))
        if self.hash_backward != "atomic":
            self.bwd_stream.wait_stream(cs)
            with torch.cuda.stream(self.bwd_stream):
                run(("coarse",), self._segment_coarse)
            comm.wait_stream(self.bwd_stream)
            self._bucket_update(0)
            nr = len(self.bin_cuts) - 1
            if nr <= 0:  # every level atomic (bin_level_lo == n_levels): the buckets past the
                # alignment cut hold the last params, complete once the coarse segment is
                for j in range(1, len(self.buckets)):
                    self._bucket_update(j)
            for r in range(nr):
                run(("apply", r), lambda r=r: self._segment_apply(r))
                comm.wait_stream(cs)
                # (a range's bucket; a bucket emptied by the alignment was dropped: the rest
                # follow the last range)
                for j in ([1 + r] if r < nr - 1 else range(1 + r, len(self.buckets))):
                    if j < len(self.buckets):
                        self._bucket_update(j)
        else:
            comm.wait_stream(cs)
            for i in range(len(self.buckets)):
                self._bucket_update(i)
        cs.wait_stream(comm)
        vren._ok(self.L.ngp_counters_inc(_p(self.dctr), 2, vren._stream()), "counters_inc")

    def _replay_pair(self, gt, directions, poses):
        """Two consecutive steady-state steps (no occupancy update at, between
        or right after them; one epoch, so one learning rate) as ONE graph
        replay: the replay boundary (the GPU finishing one graph before it
        starts the next) is paid once per two steps.  The second step's
        train_step call then only advances the host step count
        (self._ran_ahead); out_loss holds the second step's losses."""
        k, ev = self._pending
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        self._set_lr()
        key = ("pair", k, gt.data_ptr(), directions.data_ptr(), poses.data_ptr(), gt.shape, gt.dtype,
               self.msets[k]["pre_ready"])

        def body():
            self._graph_body(k, gt, directions, poses, False)
            self._graph_body(1 - k, gt, directions, poses, False)
        self._run_graph(key, body)
        self.cur = 1 - k
        self._bind(self.msets[1 - k])
        self._pending = (k, None)  # the batch after both, marched inside the graph
        self.n_prefetched += 2
        self.global_step += 1
        self._ran_ahead = True
        self._pair_key = key[2:7]
        return self.out_loss

    def _run_graph(self, key, body):
        """Replay the graph captured for `key` (capturing body() first if new;
        with a measurement timer set, one with its stamps)."""
        tm = self.timer  # (measurement) graphs with wall-clock stamp kernels around every kernel
        if tm is not None:
            key = key + (tm.uid,)
        if key not in self._graphs:
            g = torch.cuda.CUDAGraph()
            # capture on a side stream, ordered after everything enqueued so far
            torch.cuda.current_stream().synchronize()
            if tm is not None:
                tm.arm()
            try:
                with torch.cuda.graph(g):
                    body()
            finally:
                if tm is not None:
                    tm.disarm()
            # host-side state the body leaves (which buffer set has its round-1 coarse levels
            # encoded ahead): a replay does not run the body, so it restores this instead
            self._graph_post[key] = tuple(m["pre_ready"] for m in self.msets)
            self._graphs[key] = g
        self._graphs[key].replay()
        for m, f in zip(self.msets, self._graph_post[key]):
            m["pre_ready"] = f

    def _segment_compute(self, k, gt, directions, poses, update_after):
        """world > 1, first segment: the step up to the gradient (and the next
        batch's march on the side stream, joined, unless an update follows)."""
        self.cur = k
        self._bind(self.msets[k])
        cs = torch.cuda.current_stream()
        fork = None
        if not update_after:
            def fork():
                self.march_stream.wait_stream(cs)
                self._march(1 - k, ("sample", 1, gt), directions, poses, self.march_stream)
                return True
        self._segmented = True
        try:
            self._compute(self.rgb_gt, True, fork)
        finally:
            self._segmented = False
        if fork is not None:
            cs.wait_stream(self.march_stream)

    def _coarse_levels(self, fold=True):
        """The atomic coarse hash levels [0, bin_level_lo) on the current stream
        (fold=False: their replicated part stays in rep_buf for the accumulation)."""
        vren._ok(HG._lib().ngp_hash_backward_levels_rep(
            _p(self.xyzs), self.cap, _p(self.n_active_total), _p(self.sample_idx), HG.ctypes.byref(self.grid.desc),
            _p(self.denc), _p(self.grad[HG.MLP_PARAMS:]), 0, self.bin_level_lo,
            _p(self.rep_buf) if self.rep_buf is not None else None,
            self.coarse_rep_levels if self.rep_buf is not None else 0, max(1, self.coarse_rep), int(fold),
            vren._stream()), "hash_backward_levels")

    def _segment_coarse(self):
        """world > 1 graph segment (side stream): the atomic coarse hash levels."""
        self._coarse_levels()

    def _segment_apply(self, r):
        """world > 1 graph segment r (main stream): accumulation of the binned
        level range [bin_cuts[r], bin_cuts[r + 1]) (beside the previous
        range's bucket chain on the comm stream); segment 0 first writes the
        binned levels' records."""
        if r == 0:
            HGL = HG._lib()
            vren._ok(HGL.ngp_hash_binned_write(_p(self.xyzs), self.cap, _p(self.n_active_total),
                                               _p(self.sample_idx), HG.ctypes.byref(self.grid.desc), _p(self.denc),
                                               _p(self.grad[HG.MLP_PARAMS:]), _p(self.bin_ws), self.bin_max_samples,
                                               self.bin_level_lo, self.bin_merge_hi, vren._stream()),
                     "hash_binned_write")
        self._accum_levels(self.bin_cuts[r], self.bin_cuts[r + 1])

    def _accum_levels(self, lo, hi):
        vren._ok(HG._lib().ngp_hash_binned_accum_levels(
            HG.ctypes.byref(self.grid.desc), _p(self.grad[HG.MLP_PARAMS:]), _p(self.bin_ws), self.bin_max_samples,
            self.bin_level_lo, self.bin_merge_hi, lo, hi, vren._stream()), "hash_binned_accum_levels")

    def _bucket_update(self, i):
        """On the comm stream: reduce-scatter of gradient bucket i into this
        rank's shard, FusedAdam on the shard (the same launch clears the
        bucket's local gradient), all-gather of the shard's fp16 shadow.  The
        step runs this for every bucket, so its host path is lean: views and
        launch arguments built once (_bucket_host)."""
        h = self._bucket_host()[i]
        cs = self.comm_stream
        with torch.cuda.stream(cs):
            comm = ddp.comm_active(self.pg)
            if not comm:  # (emulation: this rank's shard of the local gradient)
                h["shard"].copy_(h["src"])
            else:
                ddp.reduce_scatter_(h["full"], h["shard"], self.pg)
            self._adam_shard(i, HG.c_void_p(cs.cuda_stream), zero=True)
            if comm:
                ddp.all_gather_(h["p16full"], h["p16shard"], self.pg)

    def _bucket_host(self):
        """per bucket: the tensors its collectives take and the argument tuple
        of its Adam launch (ngp_adam_step_dev_zero minus the stream)"""
        if getattr(self, "_bk", None) is None:
            self._bk = []
            f = ctypes_float
            for i, ((a, b), (lo, hi)) in enumerate(zip(self.buckets, self.shards)):
                q = lambda t: _p(t[lo:hi])  # noqa: E731
                adam = (q(self._pbuf), _p(self._gshard[i]), q(self.exp_avg), q(self.exp_avg_sq), q(self._p16buf),
                        hi - lo, _p(self.lr_dev), f(0.9), f(0.999), f(1e-15), _p(self.dctr), f(1.0 / self.world), 1,
                        _p(self._gbuf[a:b]), b - a)
                self._bk.append({"full": self._gbuf[a:b], "src": self._gbuf[lo:hi], "shard": self._gshard[i],
                                 "p16full": self._p16buf[a:b], "p16shard": self._p16buf[lo:hi], "adam": adam})
        return self._bk

    def _rs(self, i):
        (a, b), (lo, hi), gs = self.buckets[i], self.shards[i], self._gshard[i]
        if not ddp.comm_active(self.pg):  # (emulation: this rank's shard of the local gradient)
            gs.copy_(self._gbuf[lo:hi])
        else:
            ddp.reduce_scatter_(self._gbuf[a:b], gs, self.pg)

    def _ag(self, i):
        (a, b), (lo, hi) = self.buckets[i], self.shards[i]
        if ddp.comm_active(self.pg):  # (emulation: the shard's shadow is in place already)
            ddp.all_gather_(self._p16buf[a:b], self._p16buf[lo:hi], self.pg)

    def _graph_body(self, k, gt, directions, poses, update_after=False):
        self.cur = k
        self._bind(self.msets[k])
        cs = torch.cuda.current_stream()
        if not update_after:
            def fork():
                self.march_stream.wait_stream(cs)
                self._march(1 - k, ("sample", 1, gt), directions, poses, self.march_stream)
                return True

            self._compute(self.rgb_gt, True, fork)
            cs.wait_stream(self.march_stream)
            vren._ok(self.L.ngp_counters_inc(_p(self.dctr), 2, vren._stream()), "counters_inc")
        else:
            thr = 0.01 * MAX_SAMPLES / 3 ** 0.5
            drawn = self.cascades == 1
            if drawn:
                # the update's parameter-independent head (occupied cells, draws, kept draws: they
                # read density_grid and the occupancy counter only) beside this step, on the march
                # stream (idle: no prefetch before an update)
                self.march_stream.wait_stream(cs)
                with torch.cuda.stream(self.march_stream):
                    self._occ_draw(0, thr, vren._stream())
            self._compute(self.rgb_gt, True, None)
            vren._ok(self.L.ngp_counters_inc(_p(self.dctr), 2, vren._stream()), "counters_inc")
            if drawn:
                cs.wait_stream(self.march_stream)
            self.update_density_grid(thr, warmup=False, drawn=drawn)
            self._march(1 - k, ("sample", 0, gt), directions, poses, cs)

    def _step(self, src, rgb_gt, directions, poses, apply_adam, next_src):
        self._ev("occupancy_update", 0)
        if self.global_step % self.update_interval == 0 and self._updated_for != self.global_step:
            self.update_density_grid(0.01 * MAX_SAMPLES / 3 ** 0.5, warmup=self.global_step < self.warmup_steps)
        self._ev("occupancy_update", 1)
        self._ev("raygen_march", 0)
        if self._pending is not None:  # this batch was marched ahead on the side stream
            k, ev = self._pending
            self._pending = None
            self.cur = k
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
        else:
            self._march(self.cur, src, directions, poses, torch.cuda.current_stream())
        self._bind(self.msets[self.cur])
        if rgb_gt is None:
            rgb_gt = self.rgb_gt
        self._ev("raygen_march", 1)
        fork = None
        if next_src is not None and apply_adam:
            fork = lambda: self.prefetch(next_src, directions, poses)  # noqa: E731
        if apply_adam:
            self._set_lr()
        out = self._compute(rgb_gt, apply_adam, fork)
        if apply_adam:
            vren._ok(self.L.ngp_counters_inc(_p(self.dctr), 2, vren._stream()), "counters_inc")
            self.global_step += 1
        return out

    def _compute(self, rgb_gt, apply_adam, fork):
        """Field forward (chunked), compositing + loss + its backward, field
        backward, [all-reduce], Adam -- on the current stream, no host sync.
        fork() (nullable) launches the next batch's march on the side stream
        and returns whether it did (prefetch() declines before an occupancy
        update or with no_prefetch), where self.march_at says: by default right after the row forward's
        round 1 (which then has the chip to itself; the march overlaps round
        2, the composite and the MLP backward: +2.1 %,
        profiles/r04/ab/march_fork_position.txt); before the row forward, at
        the step's start (round 2: +1.5 % against after the composite,
        profiles/r02/ab/prefetch_at.txt)."""
        L, s, HGL, R = self.L, vren._stream(), HG._lib(), self.batch_size
        at = self.march_fork_point()
        marched = False  # the next batch marched beside this step (fork() said so)
        if fork is not None and at == "start":
            marched = bool(fork())
        self._ev("field_fwd", 0)
        if self._rows_fwd(self.chunk_first):
            # round 1: a wave per non-empty row (the list built by the march), its transmittance
            # deciding the row's round 2, whose samples it appends to the round-2 list itself (no
            # list pass); round 2: the field over that list
            self._ev("hash_encode", 0)
            m = self.msets[self.cur]
            pre = 8 if m["pre_ready"] else 0
            m["pre_ready"] = False
            vren._ok(HGL.ngp_field_forward_first_pre(_p(self.xyzs), _p(self.dirs), _p(self.deltas), _p(self.rays_a),
                                                     _p(self.rows_ne), _p(self.n_rows_ne), R, self.cap,
                                                     ctypes_float(1e-4), HG.ctypes.byref(self.grid.desc),
                                                     _p(self.params16[HG.MLP_PARAMS:]), _p(self.params16),
                                                     _p(self.enc), _p(self.sigmas), _p(self.rgbs), None,
                                                     _p(self.eval_idx), _p(self.eval_total2), _p(self.eval_stats),
                                                     pre, s), "field_forward_first")
            self._ev("hash_encode", 1)
            if fork is not None and at == "r1":
                # (captured before round 2: round 2 captured first and the march forked from an event
                # recorded after round 1 -- the same dependencies -- ran 27 % slower: the graph's
                # queue assignment follows the capture order, profiles/r06/ab/capture_order.txt)
                marched = bool(fork())
            self._field_indexed(s, self.eval_idx, self.eval_total2)
        elif self.chunk_first > 0:  # two rounds: first K samples per row, then the rest of unterminated rows
            K = self.chunk_first
            if self.eval1_K == K:  # built by this batch's march
                self._field_indexed(s, self.eval_idx1, self.eval_total1)
            else:
                vren._ok(L.ngp_chunk_counts(_p(self.rays_a), R, K, None, None, ctypes_float(1e-4),
                                            _p(self.eval_counts), s), "chunk_counts")
                vren._ok(L.ngp_ray_segments(_p(self.eval_counts), _p(self.rays_a), R, 0, _p(self.act_start),
                                            _p(self.eval_total), _p(self.eval_stats), _p(self.eval_idx), s),
                         "segments")
                self._field_indexed(s)
            # second round [K, N_r) of the rows still transparent after K samples: counts, scan
            # and list in one launch (ngp_chunk_segments; the two launches it replaces cost a
            # launch gap and a second pass over rays_a)
            vren._ok(L.ngp_chunk_segments(_p(self.sigmas), _p(self.deltas), _p(self.rays_a), R, K, 0,
                                          ctypes_float(1e-4), _p(self._cs_ws), _p(self.act_start),
                                          _p(self.eval_total), _p(self.eval_stats),
                                          _p(self.eval_total1) if self.eval1_K == K else None, _p(self.eval_idx), s),
                     "chunk_segments")
            self._field_indexed(s)
        else:  # encode + MLPs in one launch over every marched sample
            self._ev("hash_encode", 0)
            vren._ok(HGL.ngp_field_encode_mlp(_p(self.xyzs), _p(self.dirs), self.cap, _p(self.n_samples), None,
                                              HG.ctypes.byref(self.grid.desc), _p(self.params16[HG.MLP_PARAMS:]),
                                              _p(self.params16), _p(self.enc), _p(self.sigmas), _p(self.rgbs), None,
                                              s), "field_encode_mlp")
            self._ev("hash_encode", 1)
        self._ev("field_fwd", 1)
        if fork is not None and at == "fwd":
            marched = bool(fork())
        bg = self.bg
        if self.random_bg:  # rendering.py:287-288, one colour per batch, drawn on device (graph-safe)
            bg = self._bg_rand
            vren._ok(L.ngp_random_bg(self.sample_seed ^ 0x6267, _p(self.dctr[1:]), 0, _p(bg), s), "random_bg")
        self._ev("composite_loss", 0)
        self._ev("composite", 0)
        vren._ok(L.ngp_composite_loss(_p(self.sigmas), _p(self.rgbs), _p(self.deltas), _p(self.ts), _p(self.rays_a), R,
                                      _p(rgb_gt), _p(bg), self.loss_type, ctypes_float(self.lambda_opacity),
                                      ctypes_float(self.lambda_depth), ctypes_float(self.lambda_distortion),
                                      ctypes_float(self.scale), ctypes_float(1e-4),
                                      _p(self.dsig), _p(self.drgb), _p(self.out_rgb), _p(self.out_op),
                                      _p(self.out_depth), _p(self.out_loss), _p(self.n_active), None, None, None,
                                      _p(self.stats), s), "composite_loss")
        self._ev("composite", 1)
        # compacted gradient-carrying samples: scan + map (a per-block atomic reservation inside
        # composite_loss serialises on one address, and an ordered decoupled look-back across its
        # 2048 four-row blocks made the launch 5x longer: both measured slower)
        vren._ok(L.ngp_active_samples(_p(self.n_active), _p(self.rays_a), R, _p(self.act_start),
                                      _p(self.n_active_total), _p(self.sample_idx), s), "active_samples")
        self._ev("composite_loss", 1)
        cs = torch.cuda.current_stream()
        hybrid = self.hash_backward != "atomic"
        binned = hybrid and self.bin_level_lo < self.grid.n_levels  # (hybrid at bin_level_lo == L: all atomic)
        bs = self.bwd_stream
        def plan(after=None):  # bucket plan of the binned fine levels (xyzs / sample_idx only) beside the MLP backward
            if after is None:
                bs.wait_stream(cs)
            else:
                bs.wait_event(after)
            with torch.cuda.stream(bs):
                vren._ok(HGL.ngp_hash_binned_plan(_p(self.xyzs), self.cap, _p(self.n_active_total),
                                                  _p(self.sample_idx), HG.ctypes.byref(self.grid.desc),
                                                  _p(self.bin_ws), self.bin_max_samples, self.bin_level_lo,
                                                  self.bin_merge_hi, vren._stream()), "hash_binned_plan")
                ev = torch.cuda.Event()
                ev.record(bs)
            return ev

        # capture order (the graph's queue assignment follows it; dependencies unchanged): the MLP
        # backward, then the plan forked from an event recorded before it; the binned accumulation, then
        # the coarse branch forked from an event after the MLP backward -- +0.8 % against the reverse
        # order (5 of 7 alternating pairs, profiles/r06/ab/capture_order.txt)
        planned = seg_done = None
        if binned:
            seg_done = torch.cuda.Event()
            seg_done.record(cs)
        self._ev("mlp_bwd", 0)
        vren._ok(HGL.ngp_field_backward_mlp(_p(self.dirs), self.cap, _p(self.n_active_total), _p(self.sample_idx),
                                            _p(self.enc), self.cap, _p(self.params16), _p(self.dsig), _p(self.drgb),
                                            _p(self.denc), _p(self.grad), s), "field_backward_mlp")
        self._ev("mlp_bwd", 1)
        if seg_done is not None:
            planned = plan(seg_done)
        if fork is not None and at == "mlp":
            marched = bool(fork())
        if self._segmented and hybrid:
            # (world > 1 graph segments: the hash backward runs as two more
            # graphs -- coarse levels on the side stream, binned levels here --
            # so the reduce-scatter of the [MLP | coarse] bucket overlaps the
            # binned levels; _replay / _segment_coarse / _segment_apply)
            cs.wait_stream(bs)
            return self.out_loss
        self._ev("hash_bwd", 0)
        if hybrid:
            # atomic coarse levels on the side stream and binned fine levels
            # (after the plan) here, side by side: disjoint gradient ranges
            split = HG.MLP_PARAMS + 2 * self.grid.offsets[self.bin_level_lo]
            # single process: the MLP + coarse levels' Adam right after them on the side stream
            # (no all-reduce orders it after the whole gradient), folding the coarse gradient
            # replicas itself; the binned levels' Adam inside their accumulation (fused_adam)
            adam_split = apply_adam and not self.dp
            fused = self.fused_adam and adam_split
            self._adam_hi = split if fused else self.n_params
            fold_in_adam = adam_split and self.rep_buf is not None

            # the next batch's round-1 pre-encode after the Adam below (only while levels 0-7 are all
            # stepped by that Adam: the binned levels' parameters change inside the accumulation)
            # (any fork point: the next batch's march is captured before this point)
            pre = (adam_split and self.pre_coarse and marched
                   and self._rows_fwd(self.chunk_first) and self.bin_level_lo >= self.pre_levels)
            def side(after=None):
                if after is None:
                    bs.wait_stream(cs)
                else:
                    bs.wait_event(after)
                if pre:
                    # its dependency on the next batch's march (done long before) taken by the coarse
                    # kernel, which waits on the main stream anyway (a second cross-queue wait on the
                    # pre-encode itself started it ~12 us after the Adam's end instead of ~7: r5tl / r5ii)
                    bs.wait_stream(self.march_stream)
                with torch.cuda.stream(bs):
                    self._ev("hash_bwd_coarse", 0)
                    self._coarse_levels(fold=not fold_in_adam)
                    self._ev("hash_bwd_coarse", 1)
                    if adam_split:
                        self._adam(0, split, vren._stream(), rep=fold_in_adam)
                        if pre:
                            # the next batch (marched beside this step) gets its round-1 coarse levels now
                            nx = self.msets[1 - self.cur]
                            vren._ok(HGL.ngp_field_encode_first_coarse(
                                _p(nx["xyzs"]), _p(nx["rays_a"]), _p(nx["rows_ne"]), _p(nx["n_rows_ne"]), R,
                                self.cap, HG.ctypes.byref(self.grid.desc), _p(self.params16[HG.MLP_PARAMS:]),
                                _p(self.enc), vren._stream()), "encode_first_coarse")
                            nx["pre_ready"] = True

            mlp_done = None
            if binned:
                mlp_done = torch.cuda.Event()
                mlp_done.record(cs)
            else:
                side()
            self._ev("hash_binned_apply", 0)
            t = HG.MLP_PARAMS
            if binned:  # (none at bin_level_lo == L: the side stream took every level and its Adam)
                cs.wait_event(planned)
                if fused:  # + FusedAdam of the binned levels inside the accumulation
                    vren._ok(HGL.ngp_hash_binned_apply_adam(
                        _p(self.xyzs), self.cap, _p(self.n_active_total), _p(self.sample_idx),
                        HG.ctypes.byref(self.grid.desc), _p(self.denc), _p(self.grad[t:]), _p(self.bin_ws),
                        self.bin_max_samples, self.bin_level_lo, self.bin_merge_hi, _p(self.params[t:]),
                        _p(self.exp_avg[t:]), _p(self.exp_avg_sq[t:]), _p(self.params16[t:]), _p(self.lr_dev),
                        ctypes_float(0.9), ctypes_float(0.999), ctypes_float(1e-15), _p(self.dctr),
                        ctypes_float(1.0 / self.world), s), "hash_binned_apply_adam")
                else:
                    vren._ok(HGL.ngp_hash_binned_apply(_p(self.xyzs), self.cap, _p(self.n_active_total),
                                                       _p(self.sample_idx), HG.ctypes.byref(self.grid.desc),
                                                       _p(self.denc), _p(self.grad[t:]), _p(self.bin_ws),
                                                       self.bin_max_samples, self.bin_level_lo, self.bin_merge_hi, s),
                             "hash_binned_apply")
                    if adam_split:
                        self._adam(split, self.n_params, s)
            self._ev("hash_binned_apply", 1)
            if mlp_done is not None:
                side(mlp_done)
            cs.wait_stream(bs)
            if adam_split:
                self._ev("hash_bwd", 1)
                return self.out_loss
        else:
            vren._ok(HGL.ngp_hash_backward(_p(self.xyzs), self.cap, _p(self.n_active_total), _p(self.sample_idx),
                                           HG.ctypes.byref(self.grid.desc),
                                           _p(self.denc), _p(self.grad[HG.MLP_PARAMS:]), s), "hash_backward")
        self._ev("hash_bwd", 1)
        if not self.dp and apply_adam:
            self._ev("adam", 0)
            self._adam(0, self.n_params, s)
            self._ev("adam", 1)
        elif self.dp and not self._segmented:
            self._reduce_grads()
            if apply_adam:
                self._adam_shards()
                self._gather_params16()
        return self.out_loss

    # ------------------------------------------------- data parallel (ZeRO-1)
    def _reduce_grads(self):
        """Reduce-scatter (SUM) of each gradient bucket into this rank's shard
        buffers, then the local gradient is zeroed for the next step (RCCL over
        xGMI; outside graph captures).  apply_adam=False callers (tests) find
        the summed shards in _gshard."""
        for i in range(len(self.buckets)):
            self._rs(i)
        self._gbuf.zero_()

    def _adam_shards(self):
        for i in range(len(self.buckets)):
            self._adam_shard(i, vren._stream())

    def _adam_shard(self, i, s, zero=False):
        """FusedAdam on this rank's shard of bucket i: fp32 master, moments
        and fp16 shadow of the shard, from the reduced gradient shard (the
        1/world mean folded in; the shard buffer zeroed).  zero: the launch
        also clears the bucket's local gradient."""
        args = self._bucket_host()[i]["adam"]
        if not zero:
            args = args[:-2] + (None, 0)
        vren._ok(self.L.ngp_adam_step_dev_zero(*args, s), "adam")

    def _gather_params16(self):
        """All-gather of the updated fp16 shadow the kernels read."""
        for i in range(len(self.buckets)):
            self._ag(i)

    def full_params(self):
        """The fp32 master vector, complete on every rank (world > 1: each rank
        updates only its shards; this all-gathers them -- checkpoints, tests)."""
        if self.world > 1:
            for (a, b), (lo, hi) in zip(self.buckets, self.shards):
                ddp.all_gather_(self._pbuf[a:b], self._pbuf[lo:hi].clone(), self.pg)
        return self.params

    def fused_params(self):
        """Parameters whose Adam runs inside the binned accumulation (the binned
        hash levels; single process, hybrid/binned backward), 0 otherwise."""
        if not (self.fused_adam and not self.dp and self.hash_backward != "atomic"):
            return 0
        return self.n_params - (HG.MLP_PARAMS + 2 * self.grid.offsets[self.bin_level_lo])

    def _adam(self, lo, hi, s, rep=False):
        """FusedAdam over params[lo:hi] (16-byte aligned bounds).  lr and the
        step count from device memory (graph replays); dctr[0] = steps taken
        so far, advanced after the step by ngp_counters_inc.  rep: the coarse
        levels' gradient replicas (unfolded, fold=False) are folded here
        (lo <= MLP_PARAMS, hi past the replicated levels)."""
        q = lambda t: _p(t[lo:hi])  # noqa: E731
        if rep:
            vren._ok(self.L.ngp_adam_step_dev_rep(
                q(self.params), q(self.grad), q(self.exp_avg), q(self.exp_avg_sq), q(self.params16), hi - lo,
                _p(self.lr_dev), ctypes_float(0.9), ctypes_float(0.999), ctypes_float(1e-15), _p(self.dctr),
                ctypes_float(1.0 / self.world), 1, _p(self.rep_buf), HG.MLP_PARAMS - lo,
                2 * self.grid.offsets[self.coarse_rep_levels], self.coarse_rep, s), "adam")
            return
        vren._ok(self.L.ngp_adam_step_dev(q(self.params), q(self.grad), q(self.exp_avg), q(self.exp_avg_sq),
                                          q(self.params16), hi - lo, _p(self.lr_dev), ctypes_float(0.9),
                                          ctypes_float(0.999), ctypes_float(1e-15), _p(self.dctr),
                                          ctypes_float(1.0 / self.world), 1, s), "adam")

    def _field_indexed(self, s, idx=None, total=None):
        """Field forward (encode + MLPs in one launch) over the listed samples
        idx[:total] (default eval_idx[:eval_total]); the pair-major encoding
        kept for the backward."""
        idx = self.eval_idx if idx is None else idx
        total = self.eval_total if total is None else total
        self._ev("hash_encode", 0)
        vren._ok(HG._lib().ngp_field_encode_mlp(_p(self.xyzs), _p(self.dirs), self.cap, _p(total),
                                                _p(idx), HG.ctypes.byref(self.grid.desc),
                                                _p(self.params16[HG.MLP_PARAMS:]), _p(self.params16), _p(self.enc),
                                                _p(self.sigmas), _p(self.rgbs), None, s), "field_encode_mlp")
        self._ev("hash_encode", 1)

    # ---------------------------------------------------- test-time render
    @torch.no_grad()
    def render(self, rays_o, rays_d, T_threshold=1e-4, max_samples=MAX_SAMPLES, bg=0.0):
        """__render_rays_test (models/rendering.py:162-253) on the native kernels."""
        N_rays = rays_o.shape[0]
        dev = self.dev
        _, hits_t, _ = vren.ray_aabb_intersect(rays_o, rays_d, self.center, self.half_size, 1)
        m = (hits_t[:, 0, 0] >= 0) & (hits_t[:, 0, 0] < NEAR_DISTANCE)
        hits_t[m, 0, 0] = NEAR_DISTANCE
        ht = hits_t[:, 0]
        opacity = torch.zeros(N_rays, device=dev)
        depth = torch.zeros(N_rays, device=dev)
        rgb = torch.zeros(N_rays, 3, device=dev)
        samples = total = 0
        alive = torch.arange(N_rays, device=dev)
        min_samples = 1 if self.esf == 0 else 4
        while samples < max_samples:
            N_alive = len(alive)
            if N_alive == 0:
                break
            Ns = max(min(N_rays // N_alive, 64), min_samples)
            samples += Ns
            xyzs, dirs, deltas, ts, neff = vren.raymarching_test(rays_o, rays_d, ht, alive, self.density_bitfield,
                                                                 self.cascades, self.scale, self.esf, self.G,
                                                                 MAX_SAMPLES, Ns)
            total += int(neff.sum())
            xyzs = xyzs.reshape(-1, 3)
            dirs = dirs.reshape(-1, 3)
            valid = ~torch.all(dirs == 0, dim=1)
            if valid.sum() == 0:
                break
            sig = torch.zeros(len(xyzs), device=dev)
            rgbs = torch.zeros(len(xyzs), 3, device=dev)
            sv, rv, _, _ = HG.field_forward(xyzs[valid].contiguous(), dirs[valid].contiguous(), self.grid,
                                            self.params16, save_enc=False)
            sig[valid] = sv
            rgbs[valid] = rv
            vren.composite_test_fw(sig.view(-1, Ns), rgbs.view(-1, Ns, 3), deltas, ts, ht, alive, T_threshold, neff,
                                   opacity, depth, rgb)
            alive = alive[alive >= 0].contiguous()
        rgb = rgb + bg * (1 - opacity)[:, None]
        return {"rgb": rgb, "opacity": opacity, "depth": depth, "total_samples": total}


def ctypes_float(x):
    return HG.c_float(float(x))

