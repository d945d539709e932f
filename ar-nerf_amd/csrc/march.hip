// Rays, occupancy-grid utilities and ray marching for gfx950.
//
// Replaces models/csrc/intersection.cu and models/csrc/raymarching.cu of the
// reference.  All fp32 arithmetic on the marching path is compiled with FP
// contraction OFF so that every expression rounds exactly as the reference
// source writes it: per-ray sample counts, Morton/occupancy indices and the
// sample t values are bit-exact targets against the oracle.
//
// Layout decisions (MI355X-first):
//  * one lane per ray in 64-lane workgroups, so an 8192-ray batch spreads
//    over 128 CUs instead of the reference's 32 blocks of 256;
//  * count -> single-workgroup wave-scan -> write, giving a deterministic
//    ray-ordered rays_a and exact-size outputs; the 268 MB zero-fill of the
//    reference (raymarching.cu:302-305) is gone.
#pragma clang fp contract(off)

#include <stdlib.h>

#include <algorithm>

#include "common.h"
#include "march.h"

namespace ngp {

// ------------------------------------------------------------ AABB
__device__ __forceinline__ void aabb_t1t2(const float o[3], const float inv[3], const float* c,
                                          const float* h, float& t1, float& t2) {
    // intersection.cu:5-22
    float lo[3], hi[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float tmin = (c[i] - h[i] - o[i]) * inv[i];
        const float tmax = (c[i] + h[i] - o[i]) * inv[i];
        lo[i] = fminf(tmin, tmax);
        hi[i] = fmaxf(tmin, tmax);
    }
    t1 = fmaxf(fmaxf(lo[0], lo[1]), lo[2]);
    t2 = fminf(fminf(hi[0], hi[1]), hi[2]);
    if (t1 > t2) { t1 = -1.0f; t2 = -1.0f; }
}

__global__ void __launch_bounds__(64) ray_aabb_kernel(const float* __restrict__ rays_o,
                                                      const float* __restrict__ rays_d, int64_t n_rays,
                                                      const float* __restrict__ centers,
                                                      const float* __restrict__ half_sizes, int n_vox,
                                                      int max_hits, int32_t* __restrict__ hit_cnt,
                                                      float* __restrict__ hits_t,
                                                      int64_t* __restrict__ hits_vox) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    const float o[3] = {rays_o[3 * r], rays_o[3 * r + 1], rays_o[3 * r + 2]};
    const float inv[3] = {1.0f / rays_d[3 * r], 1.0f / rays_d[3 * r + 1], 1.0f / rays_d[3 * r + 2]};
    float* ht = hits_t + r * max_hits * 2;
    int64_t* hv = hits_vox + r * max_hits;
    for (int k = 0; k < max_hits; ++k) { ht[2 * k] = -1.0f; ht[2 * k + 1] = -1.0f; hv[k] = -1; }
    int cnt = 0;
    for (int v = 0; v < n_vox; ++v) {
        float t1, t2;
        aabb_t1t2(o, inv, centers + 3 * v, half_sizes + 3 * v, t1, t2);
        if (t2 > 0) {  // intersection.cu:44-51
            if (cnt < max_hits) { ht[2 * cnt] = fmaxf(t1, 0.0f); ht[2 * cnt + 1] = t2; hv[cnt] = v; }
            cnt++;
        }
    }
    hit_cnt[r] = cnt;
    // torch::sort(hits_t[...,0]) + gathers (intersection.cu:95-97): ascending by t1
    for (int a = 1; a < max_hits; ++a) {
        const float k0 = ht[2 * a], k1 = ht[2 * a + 1];
        const int64_t kv = hv[a];
        int b = a - 1;
        while (b >= 0 && ht[2 * b] > k0) {
            ht[2 * b + 2] = ht[2 * b]; ht[2 * b + 3] = ht[2 * b + 1]; hv[b + 1] = hv[b]; b--;
        }
        ht[2 * b + 2] = k0; ht[2 * b + 3] = k1; hv[b + 1] = kv;
    }
}

// datasets/ray_utils.py:45-70 (rays_d = dir_cam @ R^T, rays_o = c2w[:,3]) for
// the gathered training batch (train.py:85-87), then the single-box AABB
// test and the near clamp of models/rendering.py:29-31.
__device__ __forceinline__ void gen_ray(const float* __restrict__ P, const float* __restrict__ dc,
                                        const float* __restrict__ center, const float* __restrict__ half_size,
                                        float near, float* __restrict__ ro, float* __restrict__ rd,
                                        float* __restrict__ ht) {
    const float d0 = dc[0], d1 = dc[1], d2 = dc[2];
    // einsum 'n1c,nba->n1a' of rearranged c2w: d_i = sum_c dc_c * R[i][c],
    // evaluated c-major like the batched matmul (fp32, no contraction).
    float d[3], o[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        d[i] = d0 * P[4 * i + 0] + d1 * P[4 * i + 1] + d2 * P[4 * i + 2];
        o[i] = P[4 * i + 3];
    }
    const float inv[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
    float t1, t2;
    aabb_t1t2(o, inv, center, half_size, t1, t2);
    float h0 = -1.0f, h1 = -1.0f;
    if (t2 > 0) { h0 = fmaxf(t1, 0.0f); h1 = t2; }
    if (h0 >= 0 && h0 < near) h0 = near;
#pragma unroll
    for (int i = 0; i < 3; ++i) { ro[i] = o[i]; rd[i] = d[i]; }
    ht[0] = h0;
    ht[1] = h1;
}

__global__ void __launch_bounds__(256) raygen_aabb_kernel(
    const float* __restrict__ directions, const float* __restrict__ poses,
    const int64_t* __restrict__ img_idx, const int64_t* __restrict__ pix_idx, int64_t n_rays,
    const float* __restrict__ center, const float* __restrict__ half_size, float near,
    float* __restrict__ rays_o, float* __restrict__ rays_d, float* __restrict__ hits_t) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    gen_ray(poses + img_idx[r] * 12, directions + pix_idx[r] * 3, center, half_size, near, rays_o + 3 * r,
            rays_d + 3 * r, hits_t + 2 * r);
}

// One training batch entirely on device: BaseDataset.__getitem__
// (datasets/base.py:22-35: img_idxs ~ U{0..n_img-1}, pix_idxs ~ U{0..HW-1},
// rgb = rays[img, pix, :3]), get_rays + AABB + near clamp (as
// raygen_aabb_kernel) and the marcher's start perturbation noise ~ U[0,1)
// (models/custom_functions.py:83), from Philox keyed by (seed, step).
// gt_u8 (n_img, HW, 3) u8 -> rgb_gt = u8 / 255 (f32).
template <typename GT>
__global__ void __launch_bounds__(256) sample_batch_kernel(
    uint64_t seed, uint64_t step, const int64_t* __restrict__ step_dev, int64_t ray_offset, const GT* __restrict__ gt,
    int64_t n_img, int64_t hw,
    const float* __restrict__ directions, const float* __restrict__ poses, int64_t n_rays,
    const float* __restrict__ center, const float* __restrict__ half_size, float near, int64_t* __restrict__ img_idx,
    int64_t* __restrict__ pix_idx, float* __restrict__ rgb_gt, float* __restrict__ noise,
    float* __restrict__ rays_o, float* __restrict__ rays_d, float* __restrict__ hits_t) {
    NGP_PROBE_BEGIN(NGP_P_SAMPLE_BATCH);
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    if (step_dev) step += (uint64_t)*step_dev;  // device counter + offset (graph replays)
    const int64_t q = r + ray_offset;  // the ray's index in the global batch (data-parallel ranks)
    const uint4 u = philox4x32(make_uint4((uint32_t)q, (uint32_t)(q >> 32), (uint32_t)step, (uint32_t)(step >> 32)),
                               make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    const int64_t img = uniform_index(u.x, n_img), pix = uniform_index(u.y, hw);
    img_idx[r] = img;
    pix_idx[r] = pix;
    noise[r] = (float)(u.z >> 8) * (1.0f / 16777216.0f);
    const GT* g = gt + (img * hw + pix) * 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if constexpr (sizeof(GT) == 1)
            rgb_gt[3 * r + i] = (float)g[i] / 255.0f;  // read_image's astype(float32) / 255
        else
            rgb_gt[3 * r + i] = g[i];
    }
    gen_ray(poses + img * 12, directions + pix * 3, center, half_size, near, rays_o + 3 * r, rays_d + 3 * r,
            hits_t + 2 * r);
    NGP_PROBE_END();
}

// random_bg (models/rendering.py:287-288: rgb_bg = torch.rand(3) per batch),
// drawn on device from Philox keyed by (seed, *counter_dev + add) so that a
// replayed graph draws a fresh colour per batch.
__global__ void random_bg_kernel(uint64_t seed, const int64_t* __restrict__ counter_dev, int64_t add,
                                 float* __restrict__ bg) {
    const uint64_t c = (uint64_t)(*counter_dev + add);
    const uint4 u = philox4x32(make_uint4(0x62u, 0x67u, (uint32_t)c, (uint32_t)(c >> 32)),
                               make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    if (threadIdx.x < 3) {
        const uint32_t v = threadIdx.x == 0 ? u.x : threadIdx.x == 1 ? u.y : u.z;
        bg[threadIdx.x] = (float)(v >> 8) * (1.0f / 16777216.0f);
    }
}

// Bitfield summary: bit w of summary = (64-bit bitfield word w != 0), i.e.
// whether the Morton-aligned 4x4x4 cell block w holds any occupied cell;
// bit w of dilated = OR of that over block w and its 26 neighbours (same
// cascade).  One lane per block: the block index IS the cell Morton code
// without its low 6 bits, so its (bx, by, bz) are compact3 of it.
__global__ void __launch_bounds__(256) bitfield_summary_kernel(const uint64_t* __restrict__ words, int64_t n_words,
                                                               int64_t blocks_per_cascade, int bside,
                                                               uint32_t* __restrict__ summary,
                                                               uint32_t* __restrict__ dilated) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = w < n_words;
    bool s = false, dl = false;
    if (in) {
        s = words[w] != 0ull;
        if (bside <= 0) {
            dl = true;  // no block geometry: every block counts as near (disables the early out)
        } else {
            const int64_t c0 = (w / blocks_per_cascade) * blocks_per_cascade;
            const uint32_t local = (uint32_t)(w - c0);
            const int bx = (int)compact3(local), by = (int)compact3(local >> 1), bz = (int)compact3(local >> 2);
            // all 27 loads independent and in flight together (an early exit on the first
            // occupied neighbour made them 27 dependent round trips: 9-20 us per launch)
            uint64_t any = 0;
#pragma unroll
            for (int dz = -1; dz <= 1; ++dz)
#pragma unroll
                for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                    for (int dx = -1; dx <= 1; ++dx) {
                        const int x = bx + dx, y = by + dy, z = bz + dz;
                        if (x < 0 || y < 0 || z < 0 || x >= bside || y >= bside || z >= bside) continue;
                        any |= words[c0 + morton3((uint32_t)x, (uint32_t)y, (uint32_t)z)];
                    }
            dl = any != 0ull;
        }
    }
    const uint64_t bs = __ballot(s), bd = __ballot(dl);
    const int lane = threadIdx.x & 63;
    const int64_t w0 = w - lane;  // 64 consecutive blocks per wave = two summary words
    if (lane == 0 && w0 < n_words) {
        summary[w0 >> 5] = (uint32_t)bs;
        dilated[w0 >> 5] = (uint32_t)bd;
    }
    if (lane == 32 && w0 + 32 < n_words) {
        summary[(w0 >> 5) + 1] = (uint32_t)(bs >> 32);
        dilated[(w0 >> 5) + 1] = (uint32_t)(bd >> 32);
    }
}

// --------------------------------------------------- morton / packbits
__global__ void morton3d_kernel(const int32_t* __restrict__ coords, int64_t n, int32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = (int32_t)morton3((uint32_t)coords[3 * i], (uint32_t)coords[3 * i + 1], (uint32_t)coords[3 * i + 2]);
}

__global__ void morton3d_invert_kernel(const int32_t* __restrict__ idx, int64_t n, int32_t* __restrict__ coords) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t ind = idx[i];
    coords[3 * i] = (int32_t)compact3((uint32_t)(ind >> 0));
    coords[3 * i + 1] = (int32_t)compact3((uint32_t)(ind >> 1));
    coords[3 * i + 2] = (int32_t)compact3((uint32_t)(ind >> 2));
}

// raymarching.cu:122-141.  One byte per lane from two 16-B loads.
__global__ void __launch_bounds__(256) packbits_kernel(const float* __restrict__ grid, int64_t n_bytes,
                                                       float thr, const float* __restrict__ thr_dev,
                                                       uint8_t* __restrict__ bitfield) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_bytes) return;
    const float t = thr_dev ? *thr_dev : thr;
    const float4 a = reinterpret_cast<const float4*>(grid)[2 * n];
    const float4 b = reinterpret_cast<const float4*>(grid)[2 * n + 1];
    uint32_t bits = (a.x > t) | ((a.y > t) << 1) | ((a.z > t) << 2) | ((a.w > t) << 3) |
                    ((b.x > t) << 4) | ((b.y > t) << 5) | ((b.z > t) << 6) | ((b.w > t) << 7);
    bitfield[n] = (uint8_t)bits;
}

// Pass 1 (raymarching.cu:200-234)
template <bool SIMPLE>
__global__ void __launch_bounds__(64) march_count_kernel(const float* __restrict__ rays_o,
                                                         const float* __restrict__ rays_d,
                                                         const float* __restrict__ hits_t, int64_t n_rays,
                                                         const float* __restrict__ noise, MarchParams p,
                                                         int32_t* __restrict__ counts) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    float o[3], d[3], dinv[3];
    load_ray(rays_o, rays_d, r, o, d, dinv);
    const float t2 = hits_t[2 * r + 1];
    float t = start_t(hits_t, noise, r, p);
    int N = 0;
    float x, y, z, dt;
    WordCache wc;
    while (0 <= t && t < t2 && N < p.max_samples) N += march_step<SIMPLE>(t, o, d, dinv, p, x, y, z, dt, wc) ? 1 : 0;
    counts[r] = N;
}

// Exclusive scan of the per-ray counts -> ray-ordered rays_a + total, in one
// 1024-lane workgroup (8192 rays = 8 elements per lane).  Wave-level
// inclusive scan with DPP-backed __shfl_up, then a 16-wave LDS carry.
__global__ void __launch_bounds__(1024) scan_rays_kernel(const int32_t* __restrict__ counts, int64_t n_rays,
                                                         int64_t* __restrict__ rays_a, int64_t* __restrict__ total) {
    __shared__ int64_t wave_sums[16];
    __shared__ int64_t carry_s;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    constexpr int PER = 8;
    for (int64_t base = 0; base < n_rays; base += 1024 * PER) {
        int64_t v[PER];
        int64_t local = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int64_t i = base + (int64_t)tid * PER + k;
            v[k] = (i < n_rays) ? counts[i] : 0;
            local += v[k];
        }
        int64_t incl = local;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wave_sums[wid] = incl;
        __syncthreads();
        if (wid == 0) {
            int64_t ws = lane < 16 ? wave_sums[lane] : 0;
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                const int64_t y = __shfl_up(ws, off, 64);
                if (lane >= off) ws += y;
            }
            if (lane < 16) wave_sums[lane] = ws;  // inclusive over waves
        }
        __syncthreads();
        const int64_t carry = carry_s;
        int64_t run = carry + (wid > 0 ? wave_sums[wid - 1] : 0) + incl - local;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int64_t i = base + (int64_t)tid * PER + k;
            if (i < n_rays) {
                rays_a[3 * i] = i;
                rays_a[3 * i + 1] = run;
                rays_a[3 * i + 2] = v[k];
            }
            run += v[k];
        }
        __syncthreads();
        if (tid == 1023) carry_s = run;
        __syncthreads();
    }
    if (tid == 0) *total = carry_s;
}

// Pass 2 (raymarching.cu:236-279) at the scanned starts.
template <bool SIMPLE>
__global__ void __launch_bounds__(64) march_write_kernel(const float* __restrict__ rays_o,
                                                         const float* __restrict__ rays_d,
                                                         const float* __restrict__ hits_t, int64_t n_rays,
                                                         const float* __restrict__ noise, MarchParams p,
                                                         const int64_t* __restrict__ rays_a,
                                                         float* __restrict__ xyzs, float* __restrict__ dirs,
                                                         float* __restrict__ deltas, float* __restrict__ ts) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    const int64_t start = rays_a[3 * r + 1];
    const int N = (int)rays_a[3 * r + 2];
    if (N == 0) return;
    float o[3], d[3], dinv[3];
    load_ray(rays_o, rays_d, r, o, d, dinv);
    const float t2 = hits_t[2 * r + 1];
    float t = start_t(hits_t, noise, r, p);
    int samples = 0;
    float x, y, z, dt;
    WordCache wc;
    while (t < t2 && samples < N) {
        const float tc = t;
        if (march_step<SIMPLE>(t, o, d, dinv, p, x, y, z, dt, wc)) {
            const int64_t s = start + samples;
            xyzs[3 * s] = x; xyzs[3 * s + 1] = y; xyzs[3 * s + 2] = z;
            dirs[3 * s] = d[0]; dirs[3 * s + 1] = d[1]; dirs[3 * s + 2] = d[2];
            ts[s] = tc;
            deltas[s] = dt;
            samples++;
        }
    }
}

// Single-pass training march: the walk of raymarching.cu:200-234 run once,
// each occupied sample's (t, dt) stored in the ray's own slot range
// [r*max_samples, r*max_samples + n_r).  The reference's second walk
// (:243-279) re-derives exactly these first n_r samples, so storing them is
// equivalent and halves the latency-bound marching.
// The general (cascaded / esf > 0) walk: one lane per ray, MARCH_RPW rays
// per 64-lane wave (the walk is a serial, latency-bound chain per ray, so
// fewer rays per wave -- more waves on more SIMDs -- finish sooner).
constexpr int MARCH_RPW = 16;
template <bool SIMPLE>
__global__ void __launch_bounds__(256) march_slots_kernel(const float* __restrict__ rays_o,
                                                          const float* __restrict__ rays_d,
                                                          const float* __restrict__ hits_t, int64_t n_rays,
                                                          const float* __restrict__ noise, MarchParams p,
                                                          int32_t* __restrict__ counts, float* __restrict__ slot_t,
                                                          float* __restrict__ slot_dt) {
    extern __shared__ uint32_t ssum[];
    WordCache wc;
    wc.sum = load_summary(p, ssum);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    if (lane >= MARCH_RPW) return;
    const int64_t r = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * MARCH_RPW + lane;
    if (r >= n_rays) return;
    float o[3], d[3], dinv[3];
    load_ray(rays_o, rays_d, r, o, d, dinv);
    const float t2 = hits_t[2 * r + 1];
    float t = start_t(hits_t, noise, r, p);
    int N = 0;
    float x, y, z, dt;
    float* st = slot_t + r * (int64_t)p.max_samples;
    float* sd = slot_dt + r * (int64_t)p.max_samples;
    while (0 <= t && t < t2 && N < p.max_samples) {
        const float tc = t;
        if (march_step<SIMPLE>(t, o, d, dinv, p, x, y, z, dt, wc)) {
            st[N] = tc;
            sd[N] = dt;
            N++;
        }
    }
    counts[r] = N;
}

// (lattice helpers LatSeg / lat_build / lat_jump: march.h)

// The serial walk of one ray on lane 0 (a lattice whose segment table
// overflows: dt below half an ulp of t, or more than LSEG binades -- never on
// the object scenes; kept out of line so its registers do not count against
// the lattice loop's).


// first j > k with t_j >= T, for lane point k with value tk: inside the
// window's segment [Kq, Kn) (value Tq, increment Iq, its reciprocal invIq, in
// registers) from one estimate and exact fix-ups; a jump that would leave the
// segment steps on serially, t_{j+1} = fl(t_j + dt) -- the lattice's own
// definition (march_step's `do t += dt while (t < t_target)`), exact across
// any binade boundary.  The first index with t_j >= T is unique, so the
// estimate only sets the cost.
__device__ __forceinline__ int lat_jump_seg(int k, float tk, float T, float dt, int k_end, int Kq, int Kn, float Tq,
                                            float Iq, float invIq) {
    int j = k + 1;
    if (j < Kn) {
        if (fmaf((float)(j - Kq), Iq, Tq) >= T) return j;
        const float need = (T - fmaf((float)(j - Kq), Iq, Tq)) * invIq;
        int jj = min(j + (need < 4096.f ? max(1, (int)need) : 4096), Kn);
        while (jj > j + 1 && fmaf((float)(jj - 1 - Kq), Iq, Tq) >= T) --jj;
        if (jj < Kn) {
            while (jj < Kn && fmaf((float)(jj - Kq), Iq, Tq) < T) ++jj;
            if (jj < Kn) return jj;
        }
        // every point of the segment from j on lies below T: continue from its last one
        j = Kn;
        tk = fmaf((float)(Kn - 1 - Kq), Iq, Tq);
    }
    float t = tk;
    j -= 1;  // (t = t_j)
    do {
        t = t + dt;
        ++j;
    } while (t < T && j < k_end);
    return min(j, k_end);
}

// (lane 0: the ray's samples into its slot_t / slot_dt range)
__device__ __forceinline__ int march_serial_lane(const float o[3], const float d[3], const float dinv[3], float t,
                                              float t2, const MarchParams& p, WordCache& wc, float* st, float* sd) {
    float x, y, z, dts;
    int N = 0;
    while (0 <= t && t < t2 && N < p.max_samples) {
        const float tc = t;
        if (march_step<true>(t, o, d, dinv, p, x, y, z, dts, wc)) { st[N] = tc; sd[N] = dts; N++; }
    }
    return N;
}

// 8 waves per SIMD (64 VGPRs): every wave of an 8192-ray batch resident at once, no second
// dispatch round (73 -> 57 us alone; 7 waves at 65 VGPRs measured 58 us and -0.8 % end to end,
// profiles/r06/march_variants.txt)
__global__ void __launch_bounds__(256, 8) march_slots_wave_kernel(const float* __restrict__ rays_o,
                                                               const float* __restrict__ rays_d,
                                                               const float* __restrict__ hits_t, int64_t n_rays,
                                                               const float* __restrict__ noise, MarchParams p,
                                                               int32_t* __restrict__ counts,
                                                               float* __restrict__ slot_t,
                                                               float* __restrict__ slot_dt) {
    extern __shared__ uint32_t ssum[];
    __shared__ LatSeg segs[4];
    WordCache wc;
    NGP_PROBE_BEGIN(NGP_P_MARCH);
    wc.sum = load_summary(p, ssum);
    wc.dil = wc.sum ? wc.sum + p.n_sum32 : nullptr;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (wave-uniform: the ray's setup is scalar)
    const ProbeConsts pc = probe_consts(p);
    // one ray per wave (the launch has a wave per ray; no loop: no per-ray invariants held across rays)
    for (int64_t r = (int64_t)blockIdx.x * 4 + w; r < n_rays; r = n_rays) {
        float o[3], d[3], dinv[3];
        load_ray(rays_o, rays_d, r, o, d, dinv);
#pragma unroll
        for (int i = 0; i < 3; ++i) { o[i] = uniform_f(o[i]); d[i] = uniform_f(d[i]); dinv[i] = uniform_f(dinv[i]); }
        const float t2 = uniform_f(hits_t[2 * r + 1]);
        const float t0 = uniform_f(start_t(hits_t, noise, r, p));
        const float dt = NGP_SQRT3 / p.max_samples;
        float* st = slot_t + r * (int64_t)p.max_samples;
        float* sd = slot_dt + r * (int64_t)p.max_samples;
        if (!(0 <= t0) || !(t0 < t2)) {
            if (lane == 0) counts[r] = 0;
            continue;
        }
        // Conservative early out (exact): points every half 4^3-block along
        // [t0, t2]; the walk's every probe lies within one block of one of them,
        // so if no point's block has an occupied cell within one block
        // (dilated summary), the walk emits nothing.  Most rays crossing the box
        // miss the object and cost this instead of a full lattice walk.
        if (wc.dil) {
            const float mb = fminf(0.5f, p.scale);
            const float dn = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            const float step = 0.45f * (4.0f * 2.0f * mb / p.grid_size) / dn;
            const int npts = (int)ceilf((t2 - t0) / step) + 1;
            const float gm1 = p.grid_size - 1.0f, mbi = 1 / mb;
            bool near = false;
            for (int j0 = 0; j0 < npts && !near; j0 += 64) {
                const int j = j0 + lane;
                bool b = false;
                if (j < npts) {
                    const float t = fminf(t0 + (float)j * step, t2);
                    const float x = o[0] + t * d[0], y = o[1] + t * d[1], z = o[2] + t * d[2];
                    const int nx = (int)clampf(0.5f * (x * mbi + 1) * p.grid_size, 0.0f, gm1);
                    const int ny = (int)clampf(0.5f * (y * mbi + 1) * p.grid_size, 0.0f, gm1);
                    const int nz = (int)clampf(0.5f * (z * mbi + 1) * p.grid_size, 0.0f, gm1);
                    const uint32_t wi = morton3((uint32_t)nx >> 2, (uint32_t)ny >> 2, (uint32_t)nz >> 2);
                    b = (wc.dil[wi >> 5] >> (wi & 31u)) & 1u;
                }
                near = __ballot(b) != 0ull;
            }
            if (!near) {
                if (lane == 0) counts[r] = 0;
                    continue;
            }
        }
        LatSeg& sg = segs[w];
        int nseg = 0;
        const int k_end = lat_build(t0, t2, dt, sg, nseg, lane == 0);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (k_end < 0) {  // segment table overflow: the serial walk on lane 0
            if (lane == 0) counts[r] = march_serial_lane(o, d, dinv, t0, t2, p, wc, st, sd);
            continue;
        }
        // the window's segment q0 = [Kq, Kn) in registers (re-read when the window passes Kn)
        int c = 0, N = 0, q0 = 0;
        int Kq = 0, Kn = -1;
        float Tq = 0.f, Iq = 0.f, invIq = 0.f;
        while (c < k_end && N < p.max_samples) {
            if (c >= Kn) {
                while (q0 + 1 < nseg && c >= sg.K[q0 + 1]) ++q0;
                Kq = sg.K[q0];
                Kn = q0 + 1 < nseg ? sg.K[q0 + 1] : k_end;
                Tq = uniform_f(sg.T[q0]);
                Iq = uniform_f(sg.I[q0]);
                invIq = uniform_f(1.0f / Iq);
            }
            const int k = c + lane;
            const bool live = k < k_end;
            bool occ = false;
            int nxt = k_end;
            float tk = 0.f;
            if (live) {
                if (k < Kn) {
                    tk = fmaf((float)(k - Kq), Iq, Tq);
                } else {  // past the window's segment (the window straddles a binade): step on from its last point
                    float t = fmaf((float)(Kn - 1 - Kq), Iq, Tq);
                    for (int i = Kn; i <= k; ++i) t = t + dt;
                    tk = t;
                }
                float T;
                occ = march_probe_simple(tk, o, d, dinv, p, pc, wc, T);
                nxt = occ ? k + 1 : lat_jump_seg(k, tk, T, dt, k_end, Kq, Kn, Tq, Iq, invIq);
            }
            const uint64_t occm = __ballot(occ);
            const uint64_t livem = __ballot(live);
            // The walk's chain through the window.  A window whose live points are all
            // occupied is visited whole (successor k + 1 throughout).  Otherwise, in
            // parallel: J_b(i) = the 2^b-th successor of window point i (64 = out of the
            // window), built by pointer doubling; every lane then climbs from point 0 with
            // binary lifting to the last chain point <= itself -- it is on the chain iff
            // that is itself (successors only move forward).  (A scalar hop per empty
            // chain point instead: ~14 hops per window in empty space, 30 SALU
            // instructions and 3 branches each, the kernel 1.6x slower with every wave
            // resident -- the CU's scalar unit is shared, profiles/r06/march_variants.txt.)
            uint64_t vis;
            int pnt;
            if (occm == livem) {
                vis = livem;
                pnt = (livem >> 63) ? c + 64 : k_end;
            } else {
                int J[6];
                J[0] = live ? min(nxt - c, 64) : 64;
#pragma unroll
                for (int b = 1; b < 6; ++b) {
                    const int prev = J[b - 1];
                    const int v = __builtin_amdgcn_ds_bpermute(min(prev, 63) << 2, prev);
                    J[b] = prev >= 64 ? 64 : v;
                }
                int cu = 0;
#pragma unroll
                for (int b = 5; b >= 0; --b) {
                    const int v = __builtin_amdgcn_ds_bpermute(min(cu, 63) << 2, J[b]);
                    const int to = cu >= 64 ? 64 : v;
                    if (to <= lane) cu = to;
                }
                vis = __ballot(cu == lane);
                const int last = 63 - __builtin_clzll(vis);  // the chain's last point in the window
                pnt = __builtin_amdgcn_readlane(nxt, last);  // k_end if it ends the walk
            }
            vis &= occm;
            // emit the chain's occupied points, at most up to max_samples
            const int room = p.max_samples - N;
            const int nv = __builtin_popcountll(vis);
            if ((vis >> lane) & 1ull) {
                const int rank = __builtin_popcountll(vis & ((1ull << lane) - 1ull));
                if (rank < room) {
                    st[N + rank] = tk;
                    sd[N + rank] = dt;
                }
            }
            N += min(nv, room);
            c = pnt;
        }
        if (lane == 0) counts[r] = N;
    }
    NGP_PROBE_END();
}

// Dense ray-ordered outputs from the slots: one wave per ray, lanes over the
// ray's samples (coalesced 12-B / 4-B stores).  xyz = o + t*d is the same
// fp32 expression march_step evaluates (no contraction): bit-identical.
__global__ void __launch_bounds__(256) march_compact_kernel(const float* __restrict__ rays_o,
                                                            const float* __restrict__ rays_d,
                                                            const int64_t* __restrict__ rays_a, int64_t n_rays,
                                                            const float* __restrict__ slot_t,
                                                            const float* __restrict__ slot_dt, int max_samples,
                                                            float* __restrict__ xyzs, float* __restrict__ dirs,
                                                            float* __restrict__ deltas, float* __restrict__ ts) {
    NGP_PROBE_BEGIN(NGP_P_COMPACT);
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n_rays) return;
    const int64_t start = rays_a[3 * r + 1];
    const int N = (int)rays_a[3 * r + 2];
    const float o0 = rays_o[3 * r], o1 = rays_o[3 * r + 1], o2 = rays_o[3 * r + 2];
    const float d0 = rays_d[3 * r], d1 = rays_d[3 * r + 1], d2 = rays_d[3 * r + 2];
    const float* st = slot_t + r * (int64_t)max_samples;
    const float* sd = slot_dt + r * (int64_t)max_samples;
    for (int k = lane; k < N; k += 64) {
        const float t = st[k];
        const int64_t s = start + k;
        xyzs[3 * s] = o0 + t * d0; xyzs[3 * s + 1] = o1 + t * d1; xyzs[3 * s + 2] = o2 + t * d2;
        dirs[3 * s] = d0; dirs[3 * s + 1] = d1; dirs[3 * s + 2] = d2;
        ts[s] = t;
        deltas[s] = sd[k];
    }
    NGP_PROBE_END();
}

// raymarching.cu:335-404 (test time), zero-filling unused slots itself.
template <bool SIMPLE>
__global__ void __launch_bounds__(64) march_test_kernel(const float* __restrict__ rays_o,
                                                        const float* __restrict__ rays_d,
                                                        float* __restrict__ hits_t,
                                                        const int64_t* __restrict__ alive, int64_t n_alive,
                                                        MarchParams p, int N_samples, float* __restrict__ xyzs,
                                                        float* __restrict__ dirs, float* __restrict__ deltas,
                                                        float* __restrict__ ts, int32_t* __restrict__ n_eff) {
    extern __shared__ uint32_t ssum[];
    WordCache wc;
    wc.sum = load_summary(p, ssum);
    __syncthreads();
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_alive) return;
    const int64_t r = alive[n];
    float o[3], d[3], dinv[3];
    load_ray(rays_o, rays_d, r, o, d, dinv);
    float t = hits_t[2 * r];
    const float t2 = hits_t[2 * r + 1];
    int s = 0;
    float x, y, z, dt;
    const int64_t base = n * (int64_t)N_samples;
    while (t < t2 && s < N_samples) {
        const float tc = t;
        if (march_step<SIMPLE>(t, o, d, dinv, p, x, y, z, dt, wc)) {
            const int64_t q = base + s;
            xyzs[3 * q] = x; xyzs[3 * q + 1] = y; xyzs[3 * q + 2] = z;
            dirs[3 * q] = d[0]; dirs[3 * q + 1] = d[1]; dirs[3 * q + 2] = d[2];
            ts[q] = tc;
            deltas[q] = dt;
            hits_t[2 * r] = t;  // raymarching.cu:390
            s++;
        }
    }
    for (int k = s; k < N_samples; ++k) {
        const int64_t q = base + k;
        xyzs[3 * q] = 0.f; xyzs[3 * q + 1] = 0.f; xyzs[3 * q + 2] = 0.f;
        dirs[3 * q] = 0.f; dirs[3 * q + 1] = 0.f; dirs[3 * q + 2] = 0.f;
        ts[q] = 0.f;
        deltas[q] = 0.f;
    }
    n_eff[n] = s;
}

}  // namespace ngp

using namespace ngp;

static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

extern "C" {

int ngp_ray_aabb_intersect(const float* rays_o, const float* rays_d, int64_t n_rays, const float* centers,
                           const float* half_sizes, int n_voxels, int max_hits, int32_t* hit_cnt,
                           float* hits_t, int64_t* hits_voxel_idx, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && n_voxels >= 1 && max_hits >= 1);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(rays_o && rays_d && centers && half_sizes && hit_cnt && hits_t && hits_voxel_idx);
    ray_aabb_kernel<<<nblk(n_rays, 64), 64, 0, as_stream(stream)>>>(rays_o, rays_d, n_rays, centers, half_sizes,
                                                                   n_voxels, max_hits, hit_cnt, hits_t,
                                                                   hits_voxel_idx);
    return ngp_launch_status();
}

int ngp_raygen_aabb(const float* directions, const float* poses, const int64_t* img_idx, const int64_t* pix_idx,
                    int64_t n_rays, const float* center, const float* half_size, float near_distance,
                    float* rays_o, float* rays_d, float* hits_t, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(directions && poses && img_idx && pix_idx && center && half_size && rays_o && rays_d && hits_t);
    raygen_aabb_kernel<<<nblk(n_rays, 256), 256, 0, as_stream(stream)>>>(
        directions, poses, img_idx, pix_idx, n_rays, center, half_size, near_distance, rays_o, rays_d, hits_t);
    return ngp_launch_status();
}

static int launch_sample_batch(uint64_t seed, uint64_t step, const int64_t* step_dev, int64_t ray_offset,
                               const void* gt, int gt_f32, int64_t n_img, int64_t hw, const float* directions,
                               const float* poses, int64_t n_rays, const float* center, const float* half_size,
                               float near_distance, int64_t* img_idx, int64_t* pix_idx, float* rgb_gt, float* noise,
                               float* rays_o, float* rays_d, float* hits_t, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && n_img >= 1 && hw >= 1 && ray_offset >= 0 && (gt_f32 == 0 || gt_f32 == 1));
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(gt && directions && poses && center && half_size && img_idx && pix_idx && rgb_gt && noise &&
                  rays_o && rays_d && hits_t);
    if (gt_f32)
        NGP_TIMED(NGP_K_SAMPLE_BATCH, as_stream(stream), sample_batch_kernel<float><<<nblk(n_rays, 256), 256, 0, as_stream(stream)>>>(
            seed, step, step_dev, ray_offset, (const float*)gt, n_img, hw, directions, poses, n_rays, center,
            half_size, near_distance, img_idx, pix_idx, rgb_gt, noise, rays_o, rays_d, hits_t));
    else
        NGP_TIMED(NGP_K_SAMPLE_BATCH, as_stream(stream), sample_batch_kernel<uint8_t><<<nblk(n_rays, 256), 256, 0, as_stream(stream)>>>(
            seed, step, step_dev, ray_offset, (const uint8_t*)gt, n_img, hw, directions, poses, n_rays, center,
            half_size, near_distance, img_idx, pix_idx, rgb_gt, noise, rays_o, rays_d, hits_t));
    return ngp_launch_status();
}

int ngp_sample_batch(uint64_t seed, uint64_t step, int64_t ray_offset, const void* gt, int gt_f32, int64_t n_img,
                     int64_t hw, const float* directions, const float* poses, int64_t n_rays, const float* center,
                     const float* half_size, float near_distance, int64_t* img_idx, int64_t* pix_idx,
                     float* rgb_gt, float* noise, float* rays_o, float* rays_d, float* hits_t, void* stream) {
    return launch_sample_batch(seed, step, nullptr, ray_offset, gt, gt_f32, n_img, hw, directions, poses, n_rays,
                               center, half_size, near_distance, img_idx, pix_idx, rgb_gt, noise, rays_o, rays_d,
                               hits_t, stream);
}

int ngp_sample_batch_dev(uint64_t seed, const int64_t* step_dev, int64_t step_add, int64_t ray_offset, const void* gt,
                         int gt_f32, int64_t n_img, int64_t hw, const float* directions, const float* poses,
                         int64_t n_rays, const float* center, const float* half_size, float near_distance,
                         int64_t* img_idx, int64_t* pix_idx, float* rgb_gt, float* noise, float* rays_o,
                         float* rays_d, float* hits_t, void* stream) {
    NGP_CHECK_ARG(step_dev);
    return launch_sample_batch(seed, (uint64_t)step_add, step_dev, ray_offset, gt, gt_f32, n_img, hw, directions,
                               poses, n_rays, center, half_size, near_distance, img_idx, pix_idx, rgb_gt, noise,
                               rays_o, rays_d, hits_t, stream);
}

int ngp_random_bg(uint64_t seed, const int64_t* counter_dev, int64_t add, float* bg, void* stream) {
    NGP_CHECK_ARG(counter_dev && bg);
    random_bg_kernel<<<1, 64, 0, as_stream(stream)>>>(seed, counter_dev, add, bg);
    return ngp_launch_status();
}

int ngp_bitfield_summary(const uint8_t* bitfield, int64_t n_bytes, int grid_size, uint32_t* summary, void* stream) {
    NGP_CHECK_ARG(n_bytes >= 0);
    if (n_bytes == 0) return NGP_OK;
    NGP_CHECK_ARG(bitfield && summary && n_bytes % 8 == 0 && ((uintptr_t)bitfield & 7u) == 0);
    const int64_t n_words = n_bytes / 8;
    // the dilated half needs whole cascades of a power-of-two grid (Morton blocks)
    const int64_t bpc = (int64_t)grid_size * grid_size * grid_size / 64;
    const bool dil = grid_size >= 4 && (grid_size & (grid_size - 1)) == 0 && bpc > 0 && n_words % bpc == 0 &&
                     n_words % 64 == 0;
    NGP_TIMED(NGP_K_SUMMARY, as_stream(stream), bitfield_summary_kernel<<<nblk(n_words, 256), 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const uint64_t*>(bitfield), n_words, dil ? bpc : 1, dil ? grid_size / 4 : 0, summary,
        summary + (n_words + 31) / 32));
    return ngp_launch_status();
}

int ngp_morton3d(const int32_t* coords, int64_t n, int32_t* indices, void* stream) {
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(coords && indices);
    morton3d_kernel<<<nblk(n, 256), 256, 0, as_stream(stream)>>>(coords, n, indices);
    return ngp_launch_status();
}

int ngp_morton3d_invert(const int32_t* indices, int64_t n, int32_t* coords, void* stream) {
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(coords && indices);
    morton3d_invert_kernel<<<nblk(n, 256), 256, 0, as_stream(stream)>>>(indices, n, coords);
    return ngp_launch_status();
}

int ngp_packbits(const float* density_grid, int64_t n_bytes, float threshold, const float* threshold_dev,
                 uint8_t* bitfield, void* stream) {
    NGP_CHECK_ARG(n_bytes >= 0);
    if (n_bytes == 0) return NGP_OK;
    NGP_CHECK_ARG(density_grid && bitfield);
    if (((uintptr_t)density_grid & 15u) != 0) return NGP_EINVAL;  // 16-B loads
    packbits_kernel<<<nblk(n_bytes, 256), 256, 0, as_stream(stream)>>>(density_grid, n_bytes, threshold,
                                                                      threshold_dev, bitfield);
    return ngp_launch_status();
}

int ngp_march_train_count(const float* rays_o, const float* rays_d, const float* hits_t, int64_t n_rays,
                          const uint8_t* bitfield, int cascades, int grid_size, float scale, float exp_step_factor,
                          const float* noise, int max_samples, int32_t* counts, int64_t* rays_a, int64_t* total,
                          void* stream) {
    MarchParams p;
    int st = march_params(bitfield, cascades, grid_size, scale, exp_step_factor, max_samples, p);
    if (st) return st;
    NGP_CHECK_ARG(n_rays >= 0 && total && rays_a && counts);
    hipStream_t s = as_stream(stream);
    if (n_rays > 0) {
        NGP_CHECK_ARG(rays_o && rays_d && hits_t && noise);
        if (march_simple(p)) march_count_kernel<true><<<nblk(n_rays, 64), 64, 0, s>>>(rays_o, rays_d, hits_t, n_rays, noise, p, counts);
        else march_count_kernel<false><<<nblk(n_rays, 64), 64, 0, s>>>(rays_o, rays_d, hits_t, n_rays, noise, p, counts);
    }
    NGP_TIMED(NGP_K_SCAN_RAYS, s, scan_rays_kernel<<<1, 1024, 0, s>>>(counts, n_rays, rays_a, total));
    return ngp_launch_status();
}

int ngp_march_train_write(const float* rays_o, const float* rays_d, const float* hits_t, int64_t n_rays,
                          const uint8_t* bitfield, int cascades, int grid_size, float scale, float exp_step_factor,
                          const float* noise, int max_samples, const int64_t* rays_a, float* xyzs, float* dirs,
                          float* deltas, float* ts, void* stream) {
    MarchParams p;
    int st = march_params(bitfield, cascades, grid_size, scale, exp_step_factor, max_samples, p);
    if (st) return st;
    NGP_CHECK_ARG(n_rays >= 0);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(rays_o && rays_d && hits_t && noise && rays_a && xyzs && dirs && deltas && ts);
    if (march_simple(p))
        march_write_kernel<true><<<nblk(n_rays, 64), 64, 0, as_stream(stream)>>>(rays_o, rays_d, hits_t, n_rays, noise,
                                                                                p, rays_a, xyzs, dirs, deltas, ts);
    else
        march_write_kernel<false><<<nblk(n_rays, 64), 64, 0, as_stream(stream)>>>(rays_o, rays_d, hits_t, n_rays,
                                                                                 noise, p, rays_a, xyzs, dirs, deltas, ts);
    return ngp_launch_status();
}

int ngp_march_train_slots(const float* rays_o, const float* rays_d, const float* hits_t, int64_t n_rays,
                          const uint8_t* bitfield, int cascades, int grid_size, float scale, float exp_step_factor,
                          const float* noise, int max_samples, int32_t* counts, int64_t* rays_a, int64_t* total,
                          float* slot_t, float* slot_dt, const uint32_t* occ_summary, void* stream) {
    MarchParams p;
    int st = march_params(bitfield, cascades, grid_size, scale, exp_step_factor, max_samples, p);
    if (st) return st;
    st = march_attach_summary(p, occ_summary);
    if (st) return st;
    NGP_CHECK_ARG(n_rays >= 0 && total && rays_a && counts);
    hipStream_t s = as_stream(stream);
    if (n_rays > 0) {
        NGP_CHECK_ARG(rays_o && rays_d && hits_t && noise && slot_t && slot_dt);
        const size_t lds = march_summary_lds(p);
        if (march_simple(p))  // one cascade, esf 0: the wave-per-ray lattice walk
            NGP_TIMED(NGP_K_MARCH, s, march_slots_wave_kernel<<<nblk(n_rays, 4), 256, lds, s>>>(
                                          rays_o, rays_d, hits_t, n_rays, noise, p, counts, slot_t, slot_dt));
        else
            NGP_TIMED(NGP_K_MARCH, s, march_slots_kernel<false><<<nblk(n_rays, 4 * MARCH_RPW), 256, lds, s>>>(
                                          rays_o, rays_d, hits_t, n_rays, noise, p, counts, slot_t, slot_dt));
    }
    NGP_TIMED(NGP_K_SCAN_RAYS, s, scan_rays_kernel<<<1, 1024, 0, s>>>(counts, n_rays, rays_a, total));
    return ngp_launch_status();
}

int ngp_march_train_compact(const float* rays_o, const float* rays_d, const int64_t* rays_a, int64_t n_rays,
                            const float* slot_t, const float* slot_dt, int max_samples, float* xyzs, float* dirs,
                            float* deltas, float* ts, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && max_samples >= 1);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(rays_o && rays_d && rays_a && slot_t && slot_dt && xyzs && dirs && deltas && ts);
    NGP_TIMED(NGP_K_COMPACT, as_stream(stream), march_compact_kernel<<<nblk(n_rays, 4), 256, 0, as_stream(stream)>>>(rays_o, rays_d, rays_a, n_rays, slot_t,
                                                                        slot_dt, max_samples, xyzs, dirs, deltas, ts));
    return ngp_launch_status();
}

int ngp_march_test(const float* rays_o, const float* rays_d, float* hits_t, const int64_t* alive, int64_t n_alive,
                   const uint8_t* bitfield, int cascades, int grid_size, float scale, float exp_step_factor,
                   int N_samples, int max_samples, float* xyzs, float* dirs, float* deltas, float* ts,
                   int32_t* n_eff, const uint32_t* occ_summary, void* stream) {
    MarchParams p;
    int st = march_params(bitfield, cascades, grid_size, scale, exp_step_factor, max_samples, p);
    if (st) return st;
    st = march_attach_summary(p, occ_summary);
    if (st) return st;
    p.dt_scale = (float)cascades;  // raymarching.cu:370,399 quirk
    NGP_CHECK_ARG(n_alive >= 0 && N_samples >= 1);
    if (n_alive == 0) return NGP_OK;
    NGP_CHECK_ARG(rays_o && rays_d && hits_t && alive && xyzs && dirs && deltas && ts && n_eff);
    // test-time dt uses `cascades` as its scale: SIMPLE only needs esf == 0 and
    // cascades == 1, where calc_dt is the constant minimum either way.
    if (march_simple(p))
        march_test_kernel<true><<<nblk(n_alive, 64), 64, march_summary_lds(p), as_stream(stream)>>>(
            rays_o, rays_d, hits_t, alive, n_alive, p, N_samples, xyzs, dirs, deltas, ts, n_eff);
    else
        march_test_kernel<false><<<nblk(n_alive, 64), 64, march_summary_lds(p), as_stream(stream)>>>(
            rays_o, rays_d, hits_t, alive, n_alive, p, N_samples, xyzs, dirs, deltas, ts, n_eff);
    return ngp_launch_status();
}

}  // extern "C"
