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

#include "common.h"

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
__global__ void __launch_bounds__(256) raygen_aabb_kernel(
    const float* __restrict__ directions, const float* __restrict__ poses,
    const int64_t* __restrict__ img_idx, const int64_t* __restrict__ pix_idx, int64_t n_rays,
    const float* __restrict__ center, const float* __restrict__ half_size, float near,
    float* __restrict__ rays_o, float* __restrict__ rays_d, float* __restrict__ hits_t) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    const float* P = poses + img_idx[r] * 12;
    const float* dc = directions + pix_idx[r] * 3;
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
    for (int i = 0; i < 3; ++i) { rays_o[3 * r + i] = o[i]; rays_d[3 * r + i] = d[i]; }
    hits_t[2 * r] = h0;
    hits_t[2 * r + 1] = h1;
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

// --------------------------------------------------------- marching
struct MarchParams {
    const uint8_t* bitfield;
    int cascades, grid_size, max_samples;
    float scale, esf, dt_scale;  // dt_scale: `scale` (train) or `cascades` (test quirk)
};

// One step of the reference's occupancy walk (raymarching.cu:205-233):
// returns true and advances t by dt if the sample at t is occupied,
// otherwise jumps t over the empty voxel with repeated calc_dt steps.
// SIMPLE = (cascades == 1 && esf == 0): then mip == 0, mip_bound ==
// min(0.5, scale) and dt == sqrt(3)/max_samples exactly (the general
// expressions fold to these constants), so the compiler drops frexp /
// scalbn / the division per step -- same values, bit for bit.
// `wcache` holds the 64-bit bitfield word (a Morton-aligned 4x4x4 block of
// cells) last loaded by this lane; consecutive samples along a ray mostly
// stay in the same block, so most occupancy tests need no memory access.
struct WordCache {
    uint32_t idx = 0xffffffffu;
    uint64_t word = 0;
};

template <bool SIMPLE>
__device__ __forceinline__ bool march_step(float& t, const float o[3], const float d[3], const float dinv[3],
                                           const MarchParams& p, float& x, float& y, float& z, float& dt,
                                           WordCache& wc) {
    const uint32_t G = (uint32_t)p.grid_size;
    const uint32_t grid_size3 = G * G * G;
    const float grid_size_inv = 1.0f / p.grid_size;
    x = o[0] + t * d[0]; y = o[1] + t * d[1]; z = o[2] + t * d[2];
    int mip;
    float mip_bound, mip_bound_inv;
    if constexpr (SIMPLE) {
        dt = NGP_SQRT3 / p.max_samples;  // = clamp(t*0, sqrt3/max, 2 sqrt3 scale/G), t finite
        mip = 0;
        mip_bound = fminf(0.5f, p.scale);
        mip_bound_inv = 1 / mip_bound;
    } else {
        dt = calc_dt(t, p.esf, p.max_samples, p.grid_size, p.dt_scale);
        mip = max(mip_from_pos(x, y, z, p.cascades), mip_from_dt(dt, p.grid_size, p.cascades));
        mip_bound = fminf(scalbnf(1.0f, mip - 1), p.scale);
        mip_bound_inv = 1 / mip_bound;
    }
    const float gm1 = p.grid_size - 1.0f;
    const int nx = (int)clampf(0.5f * (x * mip_bound_inv + 1) * p.grid_size, 0.0f, gm1);
    const int ny = (int)clampf(0.5f * (y * mip_bound_inv + 1) * p.grid_size, 0.0f, gm1);
    const int nz = (int)clampf(0.5f * (z * mip_bound_inv + 1) * p.grid_size, 0.0f, gm1);
    const uint32_t idx = (uint32_t)mip * grid_size3 + morton3((uint32_t)nx, (uint32_t)ny, (uint32_t)nz);
    const uint32_t wi = idx >> 6;
    if (wi != wc.idx) {  // bitfield is (C*G^3/8) bytes, G^3 a multiple of 64 for G >= 4
        wc.word = reinterpret_cast<const uint64_t*>(p.bitfield)[wi];
        wc.idx = wi;
    }
    const bool occ = (wc.word >> (idx & 63u)) & 1ull;
    if (occ) { t += dt; return true; }
    const float tx = (((nx + 0.5f + 0.5f * copysignf(1.0f, d[0])) * grid_size_inv * 2 - 1) * mip_bound - x) * dinv[0];
    const float ty = (((ny + 0.5f + 0.5f * copysignf(1.0f, d[1])) * grid_size_inv * 2 - 1) * mip_bound - y) * dinv[1];
    const float tz = (((nz + 0.5f + 0.5f * copysignf(1.0f, d[2])) * grid_size_inv * 2 - 1) * mip_bound - z) * dinv[2];
    const float t_target = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    if constexpr (SIMPLE) {
        do { t += dt; } while (t < t_target);
    } else {
        do {
            t += calc_dt(t, p.esf, p.max_samples, p.grid_size, p.dt_scale);
        } while (t < t_target);
    }
    return false;
}

__device__ __forceinline__ void load_ray(const float* rays_o, const float* rays_d, int64_t r, float o[3],
                                         float d[3], float dinv[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        o[i] = rays_o[3 * r + i];
        d[i] = rays_d[3 * r + i];
        dinv[i] = 1.0f / d[i];
    }
}

// custom_functions.py:83 noise + raymarching.cu:193-198 start perturbation
__device__ __forceinline__ float start_t(const float* hits_t, const float* noise, int64_t r, const MarchParams& p) {
    float t1 = hits_t[2 * r];
    if (t1 >= 0) {
        const float dt = calc_dt(t1, p.esf, p.max_samples, p.grid_size, p.scale);
        t1 += dt * noise[r];
    }
    return t1;
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
template <bool SIMPLE>
__global__ void __launch_bounds__(64) march_slots_kernel(const float* __restrict__ rays_o,
                                                         const float* __restrict__ rays_d,
                                                         const float* __restrict__ hits_t, int64_t n_rays,
                                                         const float* __restrict__ noise, MarchParams p,
                                                         int32_t* __restrict__ counts, float* __restrict__ slot_t,
                                                         float* __restrict__ slot_dt) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    float o[3], d[3], dinv[3];
    load_ray(rays_o, rays_d, r, o, d, dinv);
    const float t2 = hits_t[2 * r + 1];
    float t = start_t(hits_t, noise, r, p);
    int N = 0;
    float x, y, z, dt;
    float* st = slot_t + r * (int64_t)p.max_samples;
    float* sd = slot_dt + r * (int64_t)p.max_samples;
    WordCache wc;
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
    WordCache wc;
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

// cascades == 1 and esf == 0 (the Lego configuration): see march_step.
// Also requires the bitfield to be 8-byte aligned for the word loads (torch
// allocations are).  dt_scale must be >= 0 so the constant-dt fold holds.
static bool march_simple(const MarchParams& p) { return p.cascades == 1 && p.esf == 0.0f && p.dt_scale >= 0.0f; }

static int march_params(const uint8_t* bf, int cascades, int grid_size, float scale, float esf, int max_samples,
                        MarchParams& p) {
    if (!bf || cascades < 1 || grid_size < 4 || grid_size > 1024 || max_samples < 1) return NGP_EINVAL;
    if (((uintptr_t)bf & 7u) != 0) return NGP_EINVAL;  // 64-bit word loads
    p.bitfield = bf; p.cascades = cascades; p.grid_size = grid_size; p.max_samples = max_samples;
    p.scale = scale; p.esf = esf; p.dt_scale = scale;
    return NGP_OK;
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
    scan_rays_kernel<<<1, 1024, 0, s>>>(counts, n_rays, rays_a, total);
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
                          float* slot_t, float* slot_dt, void* stream) {
    MarchParams p;
    int st = march_params(bitfield, cascades, grid_size, scale, exp_step_factor, max_samples, p);
    if (st) return st;
    NGP_CHECK_ARG(n_rays >= 0 && total && rays_a && counts);
    hipStream_t s = as_stream(stream);
    if (n_rays > 0) {
        NGP_CHECK_ARG(rays_o && rays_d && hits_t && noise && slot_t && slot_dt);
        if (march_simple(p))
            march_slots_kernel<true><<<nblk(n_rays, 64), 64, 0, s>>>(rays_o, rays_d, hits_t, n_rays, noise, p, counts,
                                                                     slot_t, slot_dt);
        else
            march_slots_kernel<false><<<nblk(n_rays, 64), 64, 0, s>>>(rays_o, rays_d, hits_t, n_rays, noise, p, counts,
                                                                      slot_t, slot_dt);
    }
    scan_rays_kernel<<<1, 1024, 0, s>>>(counts, n_rays, rays_a, total);
    return ngp_launch_status();
}

int ngp_march_train_compact(const float* rays_o, const float* rays_d, const int64_t* rays_a, int64_t n_rays,
                            const float* slot_t, const float* slot_dt, int max_samples, float* xyzs, float* dirs,
                            float* deltas, float* ts, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && max_samples >= 1);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(rays_o && rays_d && rays_a && slot_t && slot_dt && xyzs && dirs && deltas && ts);
    march_compact_kernel<<<nblk(n_rays, 4), 256, 0, as_stream(stream)>>>(rays_o, rays_d, rays_a, n_rays, slot_t,
                                                                        slot_dt, max_samples, xyzs, dirs, deltas, ts);
    return ngp_launch_status();
}

int ngp_march_test(const float* rays_o, const float* rays_d, float* hits_t, const int64_t* alive, int64_t n_alive,
                   const uint8_t* bitfield, int cascades, int grid_size, float scale, float exp_step_factor,
                   int N_samples, int max_samples, float* xyzs, float* dirs, float* deltas, float* ts,
                   int32_t* n_eff, void* stream) {
    MarchParams p;
    int st = march_params(bitfield, cascades, grid_size, scale, exp_step_factor, max_samples, p);
    if (st) return st;
    p.dt_scale = (float)cascades;  // raymarching.cu:370,399 quirk
    NGP_CHECK_ARG(n_alive >= 0 && N_samples >= 1);
    if (n_alive == 0) return NGP_OK;
    NGP_CHECK_ARG(rays_o && rays_d && hits_t && alive && xyzs && dirs && deltas && ts && n_eff);
    // test-time dt uses `cascades` as its scale: SIMPLE only needs esf == 0 and
    // cascades == 1, where calc_dt is the constant minimum either way.
    if (march_simple(p))
        march_test_kernel<true><<<nblk(n_alive, 64), 64, 0, as_stream(stream)>>>(
            rays_o, rays_d, hits_t, alive, n_alive, p, N_samples, xyzs, dirs, deltas, ts, n_eff);
    else
        march_test_kernel<false><<<nblk(n_alive, 64), 64, 0, as_stream(stream)>>>(
            rays_o, rays_d, hits_t, alive, n_alive, p, N_samples, xyzs, dirs, deltas, ts, n_eff);
    return ngp_launch_status();
}

}  // extern "C"
