/*
 * ngp_amd.h -- C-ABI of the MI355X-native Instant-NGP hot path
 * (libngp_amd.so, built from the ar-nerf_amd/csrc .hip sources for gfx950).
 *
 * Every entry point takes plain device pointers + sizes and an opaque HIP
 * stream (`void* stream` = hipStream_t; NULL = the null stream), launches
 * asynchronously, never allocates or frees caller memory, never
 * synchronises, and returns 0 on success, a negative NGP_E* code for a bad
 * argument, or a positive hipError_t from the launch.  The Python layer
 * (ar-nerf_amd/vren.py) allocates every buffer with the PyTorch caching
 * allocator, exactly like the reference's `vren` extension allocates its
 * outputs with torch::zeros.
 *
 * Each function names the reference interface it replaces (paths relative
 * to the YessionCC/AR-NeRF tree).  The pybind module `vren`
 * (models/csrc/binding.cpp:234-250) is replaced by the ngp_* functions
 * below; tinycudann's NetworkWithInputEncoding / Encoding / Network
 * (models/networks.py:37-78) by the ngp_field_* functions.
 */
#ifndef NGP_AMD_H
#define NGP_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGP_OK 0
#define NGP_EINVAL (-1)      /* null pointer / non-positive size               */
#define NGP_ERANGE (-2)      /* a size exceeds what the kernel supports        */

/* Library build tag (gfx950 code object version string). */
const char* ngp_version(void);

/* ------------------------------------------------------ kernel timing */
/* Measurement hook (bench.py, scripts/): when a table is set, every
 * instrumented kernel launch is bracketed by two one-lane kernels on its
 * stream that store the GPU wall clock (wall_clock64) into
 * stamps[(*step_dev % ring) * (n_ids * per_id * 2) + (id * per_id + i) * 2 +
 * {0 = before, 1 = after}] for the i-th launch of kernel id since this call
 * (launches beyond per_id and ids >= n_ids are not stamped; the stamp before
 * a launch of id only if bit id of begin_mask is set, the one after only if
 * bit id of end_mask is: one stamp before the first and one after the last
 * of consecutive launches times them together with the least perturbation).  Captured into a HIP graph, the stamps time every
 * kernel of every replay, the row chosen by the device step counter at run
 * time.  stamps == NULL disables the hook.  Host-side global state: not for
 * concurrent callers.  ngp_timing_counts: launches bracketed per id since
 * ngp_timing_set; ngp_timing_tick_ns: ns per wall-clock tick. */
enum {
    NGP_K_SAMPLE_BATCH = 0, NGP_K_SUMMARY, NGP_K_MARCH, NGP_K_SCAN_RAYS, NGP_K_COMPACT, NGP_K_SEGMENTS,
    NGP_K_HASH_ENCODE, NGP_K_FIELD_MLP, NGP_K_CHUNK, NGP_K_COMPOSITE, NGP_K_HASH_COUNT, NGP_K_HASH_SCAN,
    NGP_K_HASH_PLAN, NGP_K_MLP_BWD, NGP_K_HASH_BWD_COARSE, NGP_K_HASH_WRITE, NGP_K_HASH_ACCUM, NGP_K_ADAM,
    NGP_K_COUNT
};
int ngp_timing_set(uint64_t* stamps, const int64_t* step_dev, int64_t ring, int n_ids, int per_id, uint64_t begin_mask,
                   uint64_t end_mask);
int ngp_timing_counts(int32_t* counts, int n_ids);
double ngp_timing_tick_ns(void);

/* Device probes (bench.py's roofline window): lane 0 of every wave of the
 * probed kernels below stores its start and its end (GPU wall-clock ticks)
 * into buf[(((*step_dev % ring) * NGP_P_COUNT + id) * NGP_PROBE_WAVES + wave %
 * NGP_PROBE_WAVES) * 2 + {0, 1}] (plain stores; the caller zeroes buf and
 * takes the min start / max end of the nonzero slots) -- a kernel's
 * execution span as a dispatch trace (rocprofv3 --kernel-trace) measures it,
 * without extra graph nodes: the control block is a device symbol the kernels
 * read at run time, so graphs captured with the probes off replay with them
 * on.  buf == NULL disables.  A kernel launched twice in one step row leaves
 * the slots of both (the caller discards such rows).  Host-side global state. */
#define NGP_PROBE_WAVES 65536
enum {
    NGP_P_MARCH = 0, NGP_P_FIRST_CHUNK, NGP_P_FIELD_ENCODE_MLP, NGP_P_COMPOSITE, NGP_P_MLP_BWD, NGP_P_HASH_BWD_COARSE,
    NGP_P_HASH_COUNT, NGP_P_HASH_WRITE, NGP_P_HASH_ACCUM, NGP_P_ADAM, NGP_P_SEGMENTS, NGP_P_NONEMPTY, NGP_P_COUNTERS,
    NGP_P_HASH_PLAN, NGP_P_RESIDUAL, NGP_P_COMPACT, NGP_P_SAMPLE_BATCH, NGP_P_PRE_ENCODE,
    NGP_P_COUNT
};
int ngp_probe_set(uint64_t* buf, const int64_t* step_dev, int64_t ring);
int ngp_probe_count(void);
/* Launches an empty kernel named trace_marker_kernel (tag >= 0) on `stream`:
 * brackets a window of a rocprofv3 dispatch trace (scripts/roofline_check.py). */
int ngp_trace_marker(int tag, void* stream);

/* ---------------------------------------------------------------- rays */
/* Replaces vren.ray_aabb_intersect (binding.cpp:9-20 -> intersection.cu:59-100).
 * rays_o/rays_d (n_rays,3) f32; centers/half_sizes (n_voxels,3) f32.
 * Out: hit_cnt (n_rays) i32, hits_t (n_rays,max_hits,2) f32 (-1 = no hit),
 * hits_voxel_idx (n_rays,max_hits) i64 (-1 = no hit); hits sorted by t1
 * ascending exactly as the reference's torch::sort (misses first). */
int ngp_ray_aabb_intersect(const float* rays_o, const float* rays_d, int64_t n_rays,
                           const float* centers, const float* half_sizes, int n_voxels,
                           int max_hits, int32_t* hit_cnt, float* hits_t, int64_t* hits_voxel_idx,
                           void* stream);

/* Fused training ray generation (datasets/ray_utils.py:7-70 get_ray_directions
 * + get_rays, train.py:85-87 gathers) + AABB intersection + near clamp
 * (models/rendering.py:29-31, NEAR_DISTANCE).  directions (HW,3) f32 camera
 * space; poses (n_img,3,4) f32 c2w; img_idx/pix_idx (n_rays) i64.
 * Out: rays_o, rays_d (n_rays,3) f32, hits_t (n_rays,2) f32. */
int ngp_raygen_aabb(const float* directions, const float* poses, const int64_t* img_idx,
                    const int64_t* pix_idx, int64_t n_rays, const float* center,
                    const float* half_size, float near_distance, float* rays_o, float* rays_d,
                    float* hits_t, void* stream);

/* One training batch generated on device (replaces the DataLoader path
 * BaseDataset.__getitem__, datasets/base.py:22-35, the batch gathers of
 * train.py:85-97 and the marcher's torch.rand noise, custom_functions.py:83):
 * img_idx ~ U{0..n_img-1}, pix_idx ~ U{0..hw-1}, noise ~ U[0,1) from
 * Philox-4x32-10 keyed by (seed, step, ray_offset + ray) -- a pure function of
 * those, so ranks drawing rays [rank*R, (rank+1)*R) of one global batch
 * (ray_offset = rank*R) together draw exactly the single-process batch;
 * rgb_gt (n_rays,3) = gt[img, pix, :] with gt (n_img,hw,3) either u8
 * (gt_f32 = 0; value / 255 in fp32, read_image's astype(float32)/255) or
 * f32 (gt_f32 = 1; e.g. alpha-blended images, datasets/color_utils.py);
 * rays and hits_t as ngp_raygen_aabb. */
int ngp_sample_batch(uint64_t seed, uint64_t step, int64_t ray_offset, const void* gt, int gt_f32, int64_t n_img,
                     int64_t hw, const float* directions, const float* poses, int64_t n_rays, const float* center,
                     const float* half_size, float near_distance, int64_t* img_idx, int64_t* pix_idx,
                     float* rgb_gt, float* noise, float* rays_o, float* rays_d, float* hits_t, void* stream);

/* random_bg (models/rendering.py:287-288: one U[0,1)^3 background colour per
 * training batch) drawn on device: bg (3) f32 from Philox keyed by (seed,
 * *counter_dev + add) -- graph replays draw a fresh colour per batch. */
int ngp_random_bg(uint64_t seed, const int64_t* counter_dev, int64_t add, float* bg, void* stream);

/* ngp_sample_batch with the RNG counter in device memory: step = *step_dev +
 * step_add (a captured graph replays with the counter advanced on device). */
int ngp_sample_batch_dev(uint64_t seed, const int64_t* step_dev, int64_t step_add, int64_t ray_offset, const void* gt,
                         int gt_f32, int64_t n_img, int64_t hw, const float* directions, const float* poses,
                         int64_t n_rays, const float* center, const float* half_size, float near_distance,
                         int64_t* img_idx, int64_t* pix_idx, float* rgb_gt, float* noise, float* rays_o,
                         float* rays_d, float* hits_t, void* stream);

/* ------------------------------------------------- occupancy grid utils */
/* Replaces vren.morton3D (binding.cpp:36-40 -> raymarching.cu:62-88). */
int ngp_morton3d(const int32_t* coords, int64_t n, int32_t* indices, void* stream);
/* Replaces vren.morton3D_invert (binding.cpp:43-47 -> raymarching.cu:90-119). */
int ngp_morton3d_invert(const int32_t* indices, int64_t n, int32_t* coords, void* stream);
/* Replaces vren.packbits (binding.cpp:26-33 -> raymarching.cu:122-161):
 * bit i of byte n = (grid[8n+i] > threshold).  If threshold_dev != NULL the
 * threshold is read from device memory (no host sync; see
 * ngp_density_grid_ema) and `threshold` is ignored. */
int ngp_packbits(const float* density_grid, int64_t n_bytes, float threshold,
                 const float* threshold_dev, uint8_t* bitfield, void* stream);

/* ------------------------------------------------------- ray marching */
/* Replaces vren.raymarching_train (binding.cpp:50-67 -> raymarching.cu:166-332),
 * split into count + write so that the layout is deterministic and exact-size.
 * Pass 1: counts (n_rays) i32, rays_a (n_rays,3) i64 in RAY order
 * (row r = [r, start_r, n_r], start = exclusive prefix sum), total (1) i64.
 * hits_t is (n_rays,2) f32 (= the reference's hits_t[:,0]); noise (n_rays) f32
 * in [0,1) perturbs the first sample (custom_functions.py:83). */
int ngp_march_train_count(const float* rays_o, const float* rays_d, const float* hits_t,
                          int64_t n_rays, const uint8_t* bitfield, int cascades, int grid_size,
                          float scale, float exp_step_factor, const float* noise, int max_samples,
                          int32_t* counts, int64_t* rays_a, int64_t* total, void* stream);
/* Pass 2: writes xyzs, dirs (N,3), deltas, ts (N) f32 at rays_a starts. */
int ngp_march_train_write(const float* rays_o, const float* rays_d, const float* hits_t,
                          int64_t n_rays, const uint8_t* bitfield, int cascades, int grid_size,
                          float scale, float exp_step_factor, const float* noise, int max_samples,
                          const int64_t* rays_a, float* xyzs, float* dirs, float* deltas,
                          float* ts, void* stream);

/* Single-pass variant of the two calls above (same outputs, bit-identical):
 * ngp_march_train_slots walks each ray ONCE, storing its samples' (t, dt) in
 * caller scratch slot_t/slot_dt (n_rays*max_samples f32 each) and producing
 * counts/rays_a/total; ngp_march_train_compact then writes the dense
 * ray-ordered xyzs/dirs/deltas/ts (capacity >= total). */
int ngp_march_train_slots(const float* rays_o, const float* rays_d, const float* hits_t,
                          int64_t n_rays, const uint8_t* bitfield, int cascades, int grid_size,
                          float scale, float exp_step_factor, const float* noise, int max_samples,
                          int32_t* counts, int64_t* rays_a, int64_t* total, float* slot_t,
                          float* slot_dt, const uint32_t* occ_summary, void* stream);
int ngp_march_train_compact(const float* rays_o, const float* rays_d, const int64_t* rays_a,
                            int64_t n_rays, const float* slot_t, const float* slot_dt, int max_samples,
                            float* xyzs, float* dirs, float* deltas, float* ts, void* stream);

/* Replaces vren.raymarching_test (binding.cpp:70-88 -> raymarching.cu:335-454).
 * hits_t (n_rays_total,2) updated in place; alive (n_alive) i64.  Out:
 * xyzs, dirs (n_alive,N_samples,3), deltas, ts (n_alive,N_samples) -- slots
 * past the last sample are written 0 like the reference's torch::zeros --
 * n_eff (n_alive) i32.  Keeps the reference quirk: calc_dt gets `cascades`
 * as its scale (raymarching.cu:370,399). */
int ngp_march_test(const float* rays_o, const float* rays_d, float* hits_t, const int64_t* alive,
                   int64_t n_alive, const uint8_t* bitfield, int cascades, int grid_size,
                   float scale, float exp_step_factor, int N_samples, int max_samples,
                   float* xyzs, float* dirs, float* deltas, float* ts, int32_t* n_eff,
                   const uint32_t* occ_summary, void* stream);

/* Occupancy summary of a bitfield, for the marchers above (occ_summary,
 * nullable there): 2 x ceil(n_bytes/256) uint32 words.  First half: bit w =
 * (64-bit bitfield word w != 0), i.e. whether the Morton-aligned 4x4x4 cell
 * block w holds any occupied cell; second half: the same dilated by one
 * block in each direction (grid_size a power of two; else all ones).  The
 * marchers keep both in LDS: a ray crossing empty blocks never waits on a
 * global load, and the training marcher skips rays that pass no occupied
 * block exactly; results are identical with or without it.  Recompute
 * after every change of the bitfield. */
int ngp_bitfield_summary(const uint8_t* bitfield, int64_t n_bytes, int grid_size, uint32_t* summary,
                         void* stream);

/* -------------------------------------------------------- compositing */
/* Replaces vren.composite_train_fw (binding.cpp:91-101 -> volumerendering.cu:5-83).
 * rays_a (n_rays,3) i64 (any row order); every output element is written
 * (ws = 0 past early termination).  total_samples (n_rays) i64 per ray. */
int ngp_composite_train_fw(const float* sigmas, const float* rgbs, const float* deltas,
                           const float* ts, const int64_t* rays_a, int64_t n_rays, float T_threshold,
                           int64_t* total_samples, float* opacity, float* depth, float* rgb,
                           float* ws, void* stream);
/* Replaces vren.composite_train_bw (binding.cpp:104-127 -> volumerendering.cu:86-201). */
int ngp_composite_train_bw(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drgb,
                           const float* dL_dws, const float* sigmas, const float* rgbs,
                           const float* ws, const float* deltas, const float* ts,
                           const int64_t* rays_a, int64_t n_rays, const float* opacity,
                           const float* depth, const float* rgb, float T_threshold,
                           float* dL_dsigmas, float* dL_drgbs, void* stream);
/* Replaces vren.composite_test_fw (binding.cpp:130-151 -> volumerendering.cu:204-284).
 * sigmas/deltas/ts (n_alive,N_samples), rgbs (n_alive,N_samples,3); alive,
 * opacity, depth, rgb updated in place. */
int ngp_composite_test_fw(const float* sigmas, const float* rgbs, const float* deltas,
                          const float* ts, int64_t n_alive, int N_samples, int64_t* alive,
                          float T_threshold, const int32_t* n_eff, float* opacity, float* depth,
                          float* rgb, void* stream);

/* ---------------------------------------------------- distortion loss */
/* Replace vren.distortion_loss_fw / _bw (binding.cpp, losses.cu:62-107,143-173;
 * autograd wrapper losses.py:7-38).  ws, deltas, ts (N) f32; rays_a (n_rays,3)
 * i64.  fw: loss (indexed by rays_a[:,0]) and the two inclusive scans (N);
 * samples of no row and rows not listed are left untouched (the reference
 * zero-fills: pass zeroed buffers for its outputs).  bw: dL_dws (N) for the
 * listed rows' samples. */
int ngp_distortion_loss_fw(const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                           int64_t n_rays, float* loss, float* ws_inclusive_scan, float* wts_inclusive_scan,
                           void* stream);
int ngp_distortion_loss_bw(const float* dL_dloss, const float* ws_inclusive_scan, const float* wts_inclusive_scan,
                           const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                           int64_t n_rays, float* dL_dws, void* stream);

/* ------------------------------------ device-resident test-time render */
/* Replaces the host loop of __render_rays_test (models/rendering.py:162-253:
 * per iteration vren.raymarching_test, model(), vren.composite_test_fw and the
 * alive compaction, with a host sync on len(alive_indices)) by a loop whose
 * every decision lives in device memory, so iterations can be captured in a
 * HIP graph and replayed (renderer.py).  state: int64[NGP_RENDER_STATE_WORDS]
 *   [0],[1] alive counts of list 0/1, [2] samples (loop budget, rendering.py:186),
 *   [3] N_samples of the current iteration, [4] active (0 once finished),
 *   [5] valid samples listed this iteration (the n_dev of the field kernels),
 *   [6] total_samples (sum of N_eff), [7] iterations run.
 * Iteration k uses parity p = k & 1: ngp_render_test_march reads alive list p,
 * ngp_render_test_composite writes the survivors to list p^1.  Buffers:
 * alive lists (n_rays) i32; slots xyzs/dirs (cap,3), deltas/ts/sigmas (cap),
 * rgbs (cap,3) f32; n_eff (n_rays) i32; sample_idx (cap) i32, cap =
 * ngp_render_test_capacity(n_rays, min_samples).  Per-ray results equal the
 * host loop's bit for bit (compaction order does not enter them). */
#define NGP_RENDER_STATE_WORDS 8
int64_t ngp_render_test_capacity(int64_t n_rays, int min_samples);
/* state init, alive list 0 = arange(n_rays), opacity/depth/rgb = 0 (rendering.py:177-183) */
int ngp_render_test_begin(int64_t n_rays, int64_t* state, int32_t* alive0, float* opacity, float* depth, float* rgb,
                          void* stream);
/* Loop test + N_samples (rendering.py:186-195), then raymarching_test
 * (raymarching.cu:335-404, `cascades` as calc_dt's scale) over the alive rays
 * into slots [s*N_alive + n] (sample-major) (hits_t (n_rays,2) t1 advanced in place), and
 * the valid slots appended to sample_idx (count in state[5]). */
int ngp_render_test_march(const float* rays_o, const float* rays_d, float* hits_t, int64_t n_rays,
                          const uint8_t* bitfield, int cascades, int grid_size, float scale, float exp_step_factor,
                          int max_samples, int min_samples, int64_t sample_budget, int parity, int64_t* state,
                          const int32_t* alive, const uint32_t* occ_summary, float* xyzs, float* dirs, float* deltas,
                          float* ts, int32_t* n_eff, int32_t* sample_idx, void* stream);
/* composite_test_fw (volumerendering.cu:204-284) + total_samples + survivors
 * (n_eff > 0 and T > T_threshold) appended to alive_out. */
int ngp_render_test_composite(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                              const int32_t* n_eff, int64_t n_rays, int parity, int64_t* state,
                              const int32_t* alive_in, int32_t* alive_out, float T_threshold, float* opacity,
                              float* depth, float* rgb, void* stream);
/* rgb += bg_rgb (host float[3]) * (1 - opacity) (rendering.py:240-251) */
int ngp_render_test_finish(const float* opacity, int64_t n_rays, const float* bg_rgb, float* rgb, void* stream);

/* --------------------------------------------- hash grid + fused MLPs */
/* Level table of tcnn's Grid/Hash encoding as configured at
 * models/networks.py:33-49 (host function; fp32 arithmetic like tcnn).
 * Fills scales/res/sizes (L) and offsets (L+1); returns total entries. */
uint32_t ngp_hashgrid_levels(int n_levels, int log2_hashmap_size, int base_resolution,
                             float per_level_scale, float* scales, uint32_t* res,
                             uint32_t* offsets, uint32_t* sizes);

/* Hash-grid description passed by value to the field kernels.  Only the
 * reference's configuration is supported on the GPU: 16 levels x 2 features
 * (a 32-wide MLP input), any log2T / base resolution / per-level scale. */
#define NGP_MAX_LEVELS 16
typedef struct {
    int n_levels;                       /* must be 16 */
    float scales[NGP_MAX_LEVELS];
    uint32_t res[NGP_MAX_LEVELS];
    uint32_t offsets[NGP_MAX_LEVELS + 1];
    uint32_t sizes[NGP_MAX_LEVELS];
    float xyz_min[3], xyz_max[3];        /* models/networks.py:22-23 */
} ngp_hashgrid_t;

/* MLP weights, fp16, one contiguous buffer of NGP_MLP_PARAMS halfs, each
 * matrix row-major [out][in] (tcnn FullyFusedMLP layout, no biases):
 *   W1 64x32, W2 16x64   density net  (xyz_encoder's MLP, networks.py:50-56)
 *   W3 64x32, W4 64x64, W5 16x64 (rows 3..15 padding)  rgb_net (networks.py:68-78) */
#define NGP_MLP_PARAMS 10240

/* Replaces tcnn NetworkWithInputEncoding + Encoding(SH4) + Network as used by
 * NGP.forward (models/networks.py:133-146), fused: per sample
 *   x01 = (x - xyz_min)/(xyz_max - xyz_min); enc = hash(x01) (32, fp16)
 *   h = W2 relu(W1 enc) (16, fp16); sigma = exp(h[0]) (TruncExp, fp32)
 *   rgb = sigmoid(W5 relu(W4 relu(W3 [SH4(d/|d|), h])))[0:3]
 * xyzs, dirs (n,3) f32; table_f16 (entries,2) fp16, 16-byte aligned; mlp_f16 as above.
 * Out: sigmas (n) f32, rgbs (n,3) f32 (fp16 values), optional enc_f16 (n,32)
 * (saved for the backward) and h_f16 (n,16).  If n_dev != NULL the sample
 * count is read from device memory (n = capacity, for graph capture). */
int ngp_field_forward(const float* xyzs, const float* dirs, int64_t n, const int64_t* n_dev,
                      const ngp_hashgrid_t* grid, const void* table_f16, const void* mlp_f16,
                      float* sigmas, float* rgbs, void* enc_f16, void* h_f16, void* stream);

/* NGP.density (models/networks.py:95-108): hash + density MLP only.
 * Out: sigmas (n) f32, optional h_f16 (n,16). */
int ngp_density_forward(const float* xyzs, int64_t n, const int64_t* n_dev, const ngp_hashgrid_t* grid,
                        const void* table_f16, const void* mlp_f16, float* sigmas, void* h_f16,
                        void* stream);

/* Input gradient of NGP.density (models/networks.py:95-108) through the hash
 * grid, density MLP and TruncExp (custom_functions.py:162-173): dL_dx (n,3) =
 * dL_dsigma (n, nullable = ones) * dsigma/dx -- what render_surface_normal
 * (models/rendering.py:300-313) takes from torch.autograd.grad. */
int ngp_density_input_grad(const float* xyzs, int64_t n, const ngp_hashgrid_t* grid, const void* table_f16,
                           const void* mlp_f16, const float* dL_dsigma, float* dL_dx, void* stream);

/* Backward of ngp_field_forward (tcnn's backward for the three modules +
 * TruncExp.backward, custom_functions.py:169-173).  enc_f16 is the forward's
 * saved encoding; dL_dsigmas (n) f32, dL_drgbs (n,3) f32.  denc_ws (n,32) f32
 * is scratch (receives dL/denc).  ACCUMULATES (+=) into grad_mlp
 * (NGP_MLP_PARAMS f32, layout of mlp_f16) and grad_table ((entries,2) f32). */
int ngp_field_backward(const float* xyzs, const float* dirs, int64_t n, const int64_t* n_dev,
                       const ngp_hashgrid_t* grid, const void* enc_f16, const void* mlp_f16,
                       const float* dL_dsigmas, const float* dL_drgbs, float* denc_ws, float* grad_mlp,
                       float* grad_table, void* stream);

/* ngp_field_forward split in two launches (the training path):
 * ngp_hash_encode writes the encoding PAIR-MAJOR, enc_pm (8, n, 4) fp16 with
 * enc_pm[p][i][k] = enc[i][4p + k] (levels 2p, 2p+1 of sample i; the row
 * stride of the pair planes is n, the capacity, also with n_dev); one lane
 * per sample encodes all 16 levels, so each gather instruction serves one
 * level for 64 consecutive samples.  ngp_field_mlp_forward runs the density
 * net, SH4 and colour net on it.  sample_idx (nullable): process rows j <
 * *n_dev (or n) = samples sample_idx[j] (< n), as ngp_field_forward_indexed.
 * dirs == rgbs == NULL: the density net only (ngp_density_forward's values).
 * Same values as ngp_field_forward, bit for bit. */
int ngp_hash_encode(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                    const ngp_hashgrid_t* grid, const void* table_f16, void* enc_pm, void* stream);
/* ngp_hash_encode + ngp_field_mlp_forward in one launch (same values): the
 * pair-major encoding enc_pm (plane stride n; nullable: not stored) of the
 * listed samples, their sigmas / rgbs (dirs == NULL: density net only, rgbs
 * NULL) and h (nullable).
 * Replaces NGP.forward / NGP.density (models/networks.py:95-146). */
int ngp_field_encode_mlp(const float* xyzs, const float* dirs, int64_t n, const int64_t* n_dev,
                         const int32_t* sample_idx, const ngp_hashgrid_t* grid, const void* table_f16,
                         const void* mlp_f16, void* enc_pm, float* sigmas, float* rgbs, void* h_f16, void* stream);
/* The non-empty rows (N > 0) of rays_a, ascending, into rows[0..*n_rows);
 * rest (nullable): rest[r] = 0 for every empty row (ngp_field_forward_first
 * writes the others); zero (nullable): *zero = 0 (the round-2 list length
 * ngp_field_forward_first appends to).  One launch (one workgroup; the list
 * of a batch of rays, built beside the previous step). */
int ngp_rays_nonempty(const int64_t* rays_a, int64_t n_rays, int32_t* rows, int64_t* n_rows, int32_t* rest,
                      int64_t* zero, void* stream);
/* Round 1 of the chunked training forward with the round-2 counts: for the
 * rows rows[j], j < *n_rows_dev (rows NULL: rows 0..n_rows-1; n_rows_dev
 * NULL: n_rows) of rays_a (ray, start, N), the first min(N, 64) samples
 * encoded and run through the MLPs (enc_pm (plane stride n, nullable),
 * sigmas, rgbs: ngp_field_encode_mlp's values bit for bit), then the row's
 * transmittance over them (the compositing kernel's product scan) -> rc =
 * N - 64 if it is still above T_threshold after them, else 0.  rest
 * (nullable): rest[r] = rc -- the counts ngp_chunk_counts_range(first = 64)
 * gives, so ngp_ray_segments(rest, first = 64) lists the round-2 samples.
 * list2 (nullable; rest or list2 required): the round-2 samples themselves,
 * start + 64 .. start + N of every row with rc > 0, appended at ranges
 * reserved on *total2 (zero at the launch; its final value = the list's
 * length): rows in no fixed order, each row's samples contiguous and
 * ascending; list2 holds n entries (writes past it are dropped, and readers
 * of a device count clamp it to their capacity).  *evaluated (nullable) += the samples evaluated here plus, with
 * list2, the listed ones.  With ngp_rays_nonempty's list: one wave per
 * non-empty row.
 * Replaces, for the model(xyzs, dirs) call of __render_rays_train
 * (models/rendering.py:278), round 1's ngp_field_encode_mlp + the round-2
 * count / scan / list launch ngp_chunk_segments. */
int ngp_field_forward_first(const float* xyzs, const float* dirs, const float* deltas, const int64_t* rays_a,
                            const int32_t* rows, const int64_t* n_rows_dev, int64_t n_rows, int64_t n,
                            float T_threshold, const ngp_hashgrid_t* grid, const void* table_f16, const void* mlp_f16,
                            void* enc_pm, float* sigmas, float* rgbs, int32_t* rest, int32_t* list2,
                            int64_t* total2, int64_t* evaluated, void* stream);
/* ngp_field_forward_first whose levels [0, pre_levels) (pre_levels 0 or 8) are
 * already in enc_pm for the first-chunk samples (ngp_field_encode_first_coarse
 * with the same rows and parameters): read back instead of gathered, and not
 * rewritten.  Same outputs bit for bit. */
int ngp_field_forward_first_pre(const float* xyzs, const float* dirs, const float* deltas, const int64_t* rays_a,
                                const int32_t* rows, const int64_t* n_rows_dev, int64_t n_rows, int64_t n,
                                float T_threshold, const ngp_hashgrid_t* grid, const void* table_f16,
                                const void* mlp_f16, void* enc_pm, float* sigmas, float* rgbs, int32_t* rest,
                                int32_t* list2, int64_t* total2, int64_t* evaluated, int pre_levels, void* stream);
/* The coarse levels 0-7 of ngp_field_forward_first's encoding, ahead of time:
 * for the rows rows[j], j < *n_rows_dev (as there), the first min(N, 64)
 * samples' level features written to enc_pm pairs 0-3 (plane stride n).  The
 * training step runs it for the NEXT batch once the coarse levels' Adam has
 * run, beside the binned levels' accumulation. */
int ngp_field_encode_first_coarse(const float* xyzs, const int64_t* rays_a, const int32_t* rows,
                                  const int64_t* n_rows_dev, int64_t n_rows, int64_t n, const ngp_hashgrid_t* grid,
                                  const void* table_f16, void* enc_pm, void* stream);
int ngp_field_mlp_forward(const void* enc_pm, const float* dirs, int64_t n, const int64_t* n_dev,
                          const int32_t* sample_idx, const void* mlp_f16, float* sigmas, float* rgbs, void* h_f16,
                          void* stream);

/* ngp_field_forward over the listed samples only: rows j < n (or *n_dev) of
 * sample_idx; sample i = sample_idx[j] reads xyzs/dirs row i and writes
 * sigmas/rgbs/enc_f16 row i (other rows untouched). */
int ngp_field_forward_indexed(const float* xyzs, const float* dirs, int64_t n, const int64_t* n_dev,
                              const int32_t* sample_idx, const ngp_hashgrid_t* grid, const void* table_f16,
                              const void* mlp_f16, float* sigmas, float* rgbs, void* enc_f16, void* stream);

/* The two halves of ngp_field_backward as separate launches (so each can be
 * timed / overlapped): the MLP backward (writes dL/denc to denc_ws, += grad_mlp)
 * and the hash-table scatter (+= grad_table from denc).  sample_idx (nullable):
 * process only the samples sample_idx[0..n) (compact row j of denc_ws <->
 * sample sample_idx[j]); see ngp_active_samples.  enc_pm_stride: 0 = enc_f16
 * is row-major (n,32) (ngp_field_forward), > 0 = pair-major (ngp_hash_encode)
 * with that plane stride. */
int ngp_field_backward_mlp(const float* dirs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                           const void* enc_f16, int64_t enc_pm_stride, const void* mlp_f16,
                           const float* dL_dsigmas, const float* dL_drgbs, float* denc_ws, float* grad_mlp,
                           void* stream);
int ngp_hash_backward(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                      const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* stream);

/* Binned form of ngp_hash_backward (same gradient up to fp32 summation order):
 * records per (level, 16384-entry range) are staged in `workspace`, then each
 * range is summed in LDS and written once -- no per-sample global atomics
 * (DESIGN.md "hash backward").  Only levels [level_lo, 16) are processed
 * (pair it with ngp_hash_backward_levels for the others).  max_samples =
 * samples the workspace holds (1 KiB each; samples beyond it take the atomic
 * path, still exact); workspace = ngp_hash_backward_binned_workspace(
 * max_samples) bytes, 256-byte aligned device memory.  Levels [level_lo,
 * merge_hi) merge runs of consecutive samples (sample_idx order: along rays)
 * that share a corner pair into one summed record per corner (the coarse
 * levels, where a ray stays in a cell for many samples); merge_hi <= level_lo
 * disables it.  Replaces the same tcnn grid backward. */
size_t ngp_hash_backward_binned_workspace(int64_t max_samples);
int ngp_hash_backward_binned(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                             const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                             int64_t max_samples, int level_lo, int merge_hi, void* stream);
/* ngp_hash_backward_binned in two phases on the same workspace and inputs:
 * _plan (record counts, bucket regions: reads xyzs / sample_idx only, so it
 * can run beside the MLP backward that produces denc) then _apply (records,
 * LDS range sums, gradient). */
int ngp_hash_binned_plan(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                         const ngp_hashgrid_t* grid, void* workspace, int64_t max_samples, int level_lo,
                         int merge_hi, void* stream);
int ngp_hash_binned_apply(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                          const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                          int64_t max_samples, int level_lo, int merge_hi, void* stream);
/* The two launches of ngp_hash_binned_apply separately (write the records,
 * then sum them per bucket into grad_table), so a caller can order other
 * work between them (the trainer runs the coarse levels' atomic scatter
 * beside the accumulation instead of beside the record write). */
int ngp_hash_binned_write(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                          const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                          int64_t max_samples, int level_lo, int merge_hi, void* stream);
int ngp_hash_binned_accum(const ngp_hashgrid_t* grid, float* grad_table, void* workspace, int64_t max_samples,
                          int level_lo, int merge_hi, void* stream);
/* ngp_hash_binned_accum over the buckets of levels [acc_level_lo,
 * acc_level_hi) only (levels below level_lo have none): the data-parallel
 * step sums the binned levels in two level ranges so that the first range's
 * gradient reduce-scatter overlaps the second range's accumulation. */
int ngp_hash_binned_accum_levels(const ngp_hashgrid_t* grid, float* grad_table, void* workspace, int64_t max_samples,
                                 int level_lo, int merge_hi, int acc_level_lo, int acc_level_hi, void* stream);
/* ngp_hash_binned_apply with FusedAdam of the binned levels' parameters
 * (apex FusedAdam, train.py:146-152, as ngp_adam_step_dev): a bucket whose
 * whole gradient one workgroup sums (one chunk, no direct adds, no overflow)
 * is stepped straight from its LDS image -- its gradient never goes through
 * memory -- and every other bucket of levels [level_lo, 16) from grad_table
 * (which those entries leave zeroed).  params / exp_avg / exp_avg_sq (fp32)
 * and params_f16 have grad_table's layout (the table part of the flat
 * vector); the caller steps the rest (MLP, levels < level_lo) with
 * ngp_adam_step_dev.  Requires the binned levels' gradient to be zero on
 * entry apart from this call's own direct adds (the trainer's invariant:
 * Adam zeroes it).  Results are bit-identical to apply + ngp_adam_step_dev. */
int ngp_hash_binned_apply_adam(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                               const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                               int64_t max_samples, int level_lo, int merge_hi, float* params, float* exp_avg,
                               float* exp_avg_sq, void* params_f16, const float* lr_dev, float beta1, float beta2,
                               float eps, const int64_t* step_dev, float grad_scale, void* stream);
/* The accumulation launch of ngp_hash_binned_apply_adam alone (after
 * ngp_hash_binned_write), so other work can be ordered between the two. */
int ngp_hash_binned_accum_adam(const ngp_hashgrid_t* grid, float* grad_table, void* workspace, int64_t max_samples,
                               int level_lo, int merge_hi, float* params, float* exp_avg, float* exp_avg_sq,
                               void* params_f16, const float* lr_dev, float beta1, float beta2, float eps,
                               const int64_t* step_dev, float grad_scale, void* stream);
/* ngp_hash_backward restricted to levels [level_lo, level_hi). */
int ngp_hash_backward_levels(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                             const ngp_hashgrid_t* grid, const float* denc, float* grad_table, int level_lo,
                             int level_hi, void* stream);
/* ngp_hash_backward_levels whose levels < rep_levels add into n_rep
 * replicas of their gradient range (workgroup w into replica w % n_rep), then
 * one launch folds the replicas into grad_table and zeroes them.  The
 * coarsest levels are a few hundred KB that every sample touches: their
 * memory-side atomics queue on few lines, replicas spread them.  rep holds
 * ngp_hash_backward_rep_floats(grid, rep_levels, n_rep) floats, 16-byte
 * aligned, zero on the first call (each call leaves it zero).  Same sums as
 * ngp_hash_backward_levels up to fp32 summation order.  fold = 0 leaves the
 * sums in the replicas for ngp_adam_step_dev_rep to fold. */
int ngp_hash_backward_levels_rep(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                                 const ngp_hashgrid_t* grid, const float* denc, float* grad_table, int level_lo,
                                 int level_hi, float* rep, int rep_levels, int n_rep, int fold, void* stream);
size_t ngp_hash_backward_rep_floats(const ngp_hashgrid_t* grid, int rep_levels, int n_rep);

/* ------------------------------------------------------ training step */
/* Fused compositing + NeRFLoss + compositing backward for one training batch:
 * composite_train_fw (volumerendering.cu:5-44), background blend
 * (models/rendering.py:287-296, bg = 3 device floats), NeRFLoss
 * (losses.py:63-82; loss_type 0 raw (default), 1 mse, 2 log, 3 tanh;
 * opacity entropy lambda_opacity; depth term lambda_depth with depth_scale;
 * distortion term lambda_distortion, losses.py:77-80 + losses.cu:8-140,
 * 0 = off) and composite_train_bw with dL/dws from the distortion term.
 * rgb_gt (n_rays,3).
 * Out: dL_dsigmas (N), dL_drgbs (N,3) for each row's first n_active samples
 * (later entries are left unwritten: their gradient is exactly zero); per
 * ray out_rgb (n_rays,3) (after bg), out_opacity, out_depth, out_loss
 * (n_rays; sum = the batch loss); n_active (n_rays) i32 (nullable) = samples
 * of each row that can carry gradient (up to and including the terminating
 * one; all later ones get exactly 0).
 * sample_idx (nullable; capacity >= total samples) receives the compacted
 * list of those samples, each row's entries contiguous (row order not
 * fixed), and *n_active_total its length; alloc_ws = 16 bytes of zeroed,
 * 8-byte aligned scratch that the kernel leaves zeroed again.  stats
 * (nullable, NGP_STAT_STRIPES x NGP_STAT_STRIDE i64) accumulates, striped
 * over blocks so that no single address takes every block's atomic,
 * counter k of stripe s at stats[s * NGP_STAT_STRIDE + k]: k = 0 marched,
 * 1 composited (vr_samples), 2 gradient-carrying samples; a counter's value
 * is the sum over stripes. */
#define NGP_STAT_STRIPES 32
#define NGP_STAT_STRIDE 16
int ngp_composite_loss(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                       const int64_t* rays_a, int64_t n_rays, const float* rgb_gt, const float* bg,
                       int loss_type, float lambda_opacity, float lambda_depth, float lambda_distortion,
                       float depth_scale, float T_threshold, float* dL_dsigmas, float* dL_drgbs, float* out_rgb,
                       float* out_opacity, float* out_depth, float* out_loss, int32_t* n_active,
                       int32_t* sample_idx, void* alloc_ws, int64_t* n_active_total, int64_t* stats,
                       void* stream);

/* NeRFLoss (losses.py:41-82) of the drop-in surface: per ray the rgb term
 * (loss_type 0 raw ((x - y) / (x + 1e-3))^2 with the denominator detached, 2
 * log, 3 tanh; (n,3)), the opacity term lambda_opacity * (-o log o), o =
 * opacity + 1e-10, and the depth term -lambda_depth * log(min(depth /
 * grid_scale + 1e-10, 1)) -- one launch; _bw: their gradients w.r.t. rgb,
 * opacity and depth from the terms' upstream gradients (each nullable: no
 * gradient into that term), the derivative of each torch op in order.
 * Replaces ~15 elementwise torch ops and their autograd nodes. */
int ngp_nerf_loss_fw(const float* rgb, const float* rgb_gt, const float* opacity, const float* depth, int64_t n,
                     int loss_type, float lambda_opacity, float lambda_depth, float grid_scale, float* loss_rgb,
                     float* loss_opacity, float* loss_depth, void* stream);
int ngp_nerf_loss_bw(const float* rgb, const float* rgb_gt, const float* opacity, const float* depth, int64_t n,
                     int loss_type, float lambda_opacity, float lambda_depth, float grid_scale, const float* g_rgb,
                     const float* g_opacity, const float* g_depth, float* d_rgb, float* d_opacity, float* d_depth,
                     void* stream);
/* The samples that carry gradient in the drop-in backward: rows i < n with
 * dL_dsigmas[i] != 0 or any dL_drgbs[i][*] != 0 (the compositing backward,
 * volumerendering.cu:86-150, leaves every sample past its ray's termination at
 * exact zero) -> idx[0..*count) (device count, 8-byte aligned, zeroed by the
 * call; rows ascending within each 1024-row block, blocks in any order).  The
 * field backward over that list (ngp_field_backward_mlp / ngp_hash_backward*
 * with sample_idx = idx, n_dev = count) adds exactly what it adds over all n
 * rows.  Replaces nothing in the reference: it lets models.custom_functions'
 * autograd surface skip the zero rows the reference's tcnn backward walks. */
int ngp_gradient_rows(const float* dL_dsigmas, const float* dL_drgbs, int64_t n, int32_t* idx, int64_t* count,
                      void* stream);
/* Compacted list of the gradient-carrying samples: act_start_ws (n_rows) i64
 * scratch, n_active_total (1) i64, sample_idx (>= total) i32 with
 * sample_idx[act_start[r] + k] = rays_a[r].start + k, k < n_active[r]. */
int ngp_active_samples(const int32_t* n_active, const int64_t* rays_a, int64_t n_rows,
                       int64_t* act_start_ws, int64_t* n_active_total, int32_t* sample_idx,
                       void* stream);

/* Chunked field evaluation of a training batch (exact: the step reads a row's
 * samples only up to its termination).  sigmas == NULL: counts[r] =
 * min(N_r, first) (round 1).  Else (after round 1 evaluated them): counts[r] =
 * N_r - first if row r's transmittance over its first min(N_r, first) samples
 * (composite_train_fw's serial product, volumerendering.cu:27-41) stays above
 * T_threshold and N_r > first, else 0 (round 2). */
int ngp_chunk_counts(const int64_t* rays_a, int64_t n_rows, int first, const float* sigmas,
                     const float* deltas, float T_threshold, int32_t* counts, void* stream);
/* ngp_chunk_counts of a later round with a cap: a row still transparent after
 * its first min(N_r, first) samples gets min(N_r, last) - first (last <= 0:
 * N_r - first, the round-2 form above); evaluation rounds over [first, last)
 * let rows that terminate there skip the rest of their samples. */
int ngp_chunk_counts_range(const int64_t* rays_a, int64_t n_rows, int first, int last, const float* sigmas,
                           const float* deltas, float T_threshold, int32_t* counts, void* stream);
/* Sample list of per-row segments: sample_idx[start_r + k] = rays_a[r].start +
 * first + k for k < counts[r] (start = exclusive prefix of counts, in
 * start_ws (n_rows) i64); *total = the list length, *total_acc += it
 * (nullable; a device-scope atomic add). */
/* ngp_chunk_counts_range (sigmas given) + ngp_ray_segments of those counts
 * in ONE launch: the list of round-2 samples [first, min(N_r, last)) of the
 * rows still transparent after `first` samples, its per-row starts and total
 * (total_acc += total).  The prefix across row blocks is a decoupled look-back
 * through `lookback_ws`: ngp_chunk_segments_workspace(n_rows) bytes, 8-byte
 * aligned, ZEROED once by the caller and then owned by the call site (the
 * kernel leaves it ready for the next launch; never shared by concurrent
 * launches).  Same outputs as the two calls.  total_acc_add (nullable, needs
 * total_acc): a device count added into *total_acc with the total -- the
 * round-1 list length of a list built earlier, so a step's evaluated samples
 * are counted by the step that evaluates them. */
size_t ngp_chunk_segments_workspace(int64_t n_rows);
int ngp_chunk_segments(const float* sigmas, const float* deltas, const int64_t* rays_a, int64_t n_rows, int first,
                       int last, float T_threshold, void* lookback_ws, int64_t* start_ws, int64_t* total,
                       int64_t* total_acc, const int64_t* total_acc_add, int32_t* sample_idx, void* stream);
int ngp_ray_segments(const int32_t* counts, const int64_t* rays_a, int64_t n_rows, int first,
                     int64_t* start_ws, int64_t* total, int64_t* total_acc, int32_t* sample_idx,
                     void* stream);
/* ngp_ray_segments of each row's first min(N_r, cap) samples (counts read
 * from rays_a: chunked evaluation round 1 in one launch).  NGP_ERANGE above
 * 65536 rows (use ngp_chunk_counts + ngp_ray_segments there). */
int ngp_ray_segments_capped(const int64_t* rays_a, int64_t n_rows, int cap, int64_t* start_ws, int64_t* total,
                            int64_t* total_acc, int32_t* sample_idx, void* stream);


/* apex FusedAdam step (train.py:146; weight decay 0) over n (multiple of 4)
 * fp32 params with grad *= grad_scale, bias corrections for `step` (1-based);
 * writes the fp16 shadow params_f16 and, if zero_grad, zeroes grads. */
int ngp_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* params_f16,
                  int64_t n, float lr, float beta1, float beta2, float eps, int64_t step,
                  float grad_scale, int zero_grad, void* stream);

/* ngp_adam_step with the learning rate and the step count in device memory
 * (lr_dev f32; step_dev = steps already taken, this is step *step_dev + 1;
 * not advanced here -- see ngp_counters_inc). */
int ngp_adam_step_dev(float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* params_f16,
                      int64_t n, const float* lr_dev, float beta1, float beta2, float eps,
                      const int64_t* step_dev, float grad_scale, int zero_grad, void* stream);
/* ngp_adam_step_dev that also clears zero[0, zero_n) (zero_n a multiple of 4,
 * 16-byte aligned) in the same launch -- the data-parallel step's bucket: its
 * local gradient, read by the reduce-scatter before this Adam on the shard,
 * cleared for the next step without a launch of its own. */
int ngp_adam_step_dev_zero(float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* params_f16,
                           int64_t n, const float* lr_dev, float beta1, float beta2, float eps,
                           const int64_t* step_dev, float grad_scale, int zero_grad, float* zero, int64_t zero_n,
                           void* stream);
/* ngp_adam_step_dev whose gradient over [rep_offset, rep_offset + rep_n) of
 * this range is grads + the n_rep replicas of ngp_hash_backward_levels_rep
 * (fold = 0; replica r at rep + r * rep_n), folded in replica order and
 * zeroed: bit-identical to folding them first (fold = 1) and stepping. */
int ngp_adam_step_dev_rep(float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* params_f16, int64_t n,
                          const float* lr_dev, float beta1, float beta2, float eps, const int64_t* step_dev,
                          float grad_scale, int zero_grad, float* rep, int64_t rep_offset, int64_t rep_n, int n_rep,
                          void* stream);
/* counters[i] += 1, i < n (n <= 64): advances the device step counters. */
int ngp_counters_inc(int64_t* counters, int n, void* stream);

/* Occupancy update (models/networks.py:252-281).  density_grid_tmp is kept as
 * a 64-bit key grid (n = C*G^3 u64, 8-byte aligned, zero between updates):
 * scatter_last: density_grid_tmp[idx[i]] = sigmas[i] (networks.py:268) with
 * torch's sequential index_put_ semantics -- of duplicate cells the one at the
 * largest list position pos_base + i wins, key = (pos+1) << 32 | sigma bits
 * (sigma clamped at 0; negative indices skipped); ranks sharding one list
 * combine key grids with a MAX all-reduce.  grid_ema: grid = where(grid<0,
 * grid, max(grid*decay, tmp)) in place (the key grid is consumed: left
 * zeroed); decay_cells (nullable, n floats) replaces the scalar decay per cell
 * -- the erode branch (networks.py:270-272), decay_cells =
 * clamp(decay**(1/count_grid), 0.1, 0.95); then
 * threshold_out[0] = min(mean(grid[grid>0]), thr_max) (NaN if none, as in
 * Python), threshold_out[1] = the mean; feed threshold_out to ngp_packbits'
 * threshold_dev.  sum_cnt_ws: 16 bytes of scratch (two fp64 accumulators, 8-byte
 * aligned; the mean is taken in fp64). */
/* Capacity guards: the number of times a kernel found a device-side count
 * past the capacity its caller gave it and clamped it (the result is then
 * truncated: samples, rows or cells dropped instead of read or written out of
 * bounds) -- every n_dev / n_rows_dev / count argument of the field, hash
 * backward and occupancy kernels, the row forward's round-2 list, the
 * occupancy list and the bounded look-back spin.  Nonzero only after a
 * capacity overflow or memory corruption (tests assert 0, bench.py reports
 * it).  Synchronises the device.  ngp_guard_reset zeroes the counters. */
unsigned long long ngp_guard_hits(void);
int ngp_guard_reset(void);
int ngp_density_scatter_last(const int64_t* indices, const float* sigmas, int64_t n, int64_t pos_base,
                             uint64_t* grid_key, void* stream);
int ngp_density_grid_ema(float* density_grid, uint64_t* grid_key, int64_t n, float decay,
                         const float* decay_cells, float thr_max, void* sum_cnt_ws, float* threshold_out,
                         void* stream);
/* sample_uniform_and_occupied_cells (models/networks.py:181-207) on device,
 * no host sync: ngp_occupied_cells lists the cells of one cascade (n_cells
 * f32, Morton order) with density > threshold into list (capacity n_cells)
 * in ascending cell order -- torch.nonzero's list, deterministic --
 * *count = their number (8-byte aligned); workspace:
 * ngp_occupied_cells_workspace(n_cells) bytes (4-byte aligned).
 * ngp_occupancy_samples writes samples [lo, hi) of the 2*M list: sample i <
 * M a uniform cell, i >= M a cell drawn uniformly from the occupied list
 * (flat_idx = -1, skipped by ngp_density_scatter_last, when it is empty);
 * xyzs (hi-lo, 3) = (coords/(G-1)*2-1)*(s-hgs) + (U*2-1)*hgs (networks.py:
 * 262-266; s_minus_hgs, hgs as fp32), flat_idx (hi-lo) = cascade*G^3 +
 * Morton index.  Randoms from Philox keyed by (seed, *counter_dev, cascade,
 * i): every rank of a data-parallel job draws the same list and can
 * evaluate a disjoint [lo, hi). */
size_t ngp_occupied_cells_workspace(int64_t n_cells);
int ngp_occupied_cells(const float* grid_cascade, int64_t n_cells, float threshold, int32_t* list,
                       int64_t* count, void* workspace, void* stream);
int ngp_occupancy_samples(uint64_t seed, const int64_t* counter_dev, int cascade, int grid_size, int64_t M,
                          float s_minus_hgs, float hgs, const int32_t* occ_list, const int64_t* occ_count,
                          int64_t lo, int64_t hi, float* xyzs, int64_t* flat_idx, void* stream);
/* ngp_occupancy_samples with each half's cells in ascending order (uniform
 * half: Morton order; occupied half: list order), so the density forward's
 * waves stay local: the same two multisets in distribution (M i.i.d. uniform
 * cells, M i.i.d. picks from the list), drawn as order statistics (running
 * sums of Exp(1) variates); other randoms as ngp_occupancy_samples.
 * workspace: ngp_occupancy_sorted_workspace(M) bytes, 8-byte aligned. */
size_t ngp_occupancy_sorted_workspace(int64_t M);
int ngp_occupancy_samples_sorted(uint64_t seed, const int64_t* counter_dev, int cascade, int grid_size, int64_t M,
                                 float s_minus_hgs, float hgs, const int32_t* occ_list, const int64_t* occ_count,
                                 int64_t lo, int64_t hi, void* workspace, float* xyzs, int64_t* flat_idx,
                                 void* stream);
/* The samples of ngp_occupancy_samples_sorted's full list (positions [0, 2M),
 * flat_idx; each half ascending) whose sigma the update keeps: position i
 * survives density_grid_tmp[c, idx] = sigma's last-write-wins
 * (networks.py:268; ngp_density_scatter_last's rule) iff no later position
 * holds its cell -- the last of its run in its half, and in the uniform half
 * only a cell the occupied half does not draw.  Lists the kept positions of
 * [lo, hi) (ascending within each 8192-position block, blocks in any order)
 * and *count = their number (device, 8-byte aligned).  cell_base = cascade *
 * n_cells; mark_ws: round_up(n_cells, 16) bytes of scratch, 16-byte aligned (cleared in 16-byte words).  Evaluating
 * only these (ngp_field_encode_mlp with sample_idx = list) and scattering them
 * with ngp_density_scatter_kept leaves the same key grid as evaluating and
 * scattering all of [lo, hi). */
int ngp_occupancy_keep(const int64_t* flat_idx, int64_t M, int64_t cell_base, int64_t n_cells, int64_t lo,
                       int64_t hi, void* mark_ws, int32_t* list, int64_t* count, void* stream);
/* ngp_density_scatter_last over the listed positions i = list[j], j <
 * min(*count, n_max): key of cell indices[i] max= (pos_base + i + 1) << 32 |
 * sigma bits of sigmas[i]. */
int ngp_density_scatter_kept(const int32_t* list, const int64_t* count, int64_t n_max, const int64_t* indices,
                             const float* sigmas, int64_t pos_base, uint64_t* grid_key, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NGP_AMD_H */
