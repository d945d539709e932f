// Occupancy-grid ray-marching step shared by the training / test marchers
// (march.hip) and the device-resident test render loop (render.hip).
// raymarching.cu:11-60,166-234,335-404 of the reference.
#pragma once
#pragma clang fp contract(off)
#include "common.h"

namespace ngp {

// --------------------------------------------------------- marching
struct MarchParams {
    const uint8_t* bitfield;
    const uint32_t* summary;  // nullable: bit w = (64-bit bitfield word w != 0), see ngp_bitfield_summary
    int n_sum32;              // uint32 words of summary
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
    const uint32_t* sum = nullptr;  // LDS copy of the bitfield summary (nullable)
    const uint32_t* dil = nullptr;  // its one-block dilation (nullable; mip-0 blocks of cascade 0)
};

// Copy the bitfield summary into LDS (whole workgroup; call before any
// early return, followed by __syncthreads()).  Returns the LDS pointer or
// nullptr when the launch has no summary.
__device__ __forceinline__ const uint32_t* load_summary(const MarchParams& p, uint32_t* lds) {
    if (!p.summary) return nullptr;
    for (int i = threadIdx.x; i < 2 * p.n_sum32; i += blockDim.x) lds[i] = p.summary[i];
    return lds;
}

// The occupancy test at t (raymarching.cu:205-221): position, cell, bit.
// Returns the bit; for an empty cell also the voxel-exit target
// t_target (:222-228) that the walk then steps past.
template <bool SIMPLE>
__device__ __forceinline__ bool march_probe(float t, const float o[3], const float d[3], const float dinv[3],
                                            const MarchParams& p, float& x, float& y, float& z, float& dt,
                                            WordCache& wc, float& t_target) {
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
        // an all-empty word is known from the LDS summary: no global load, so
        // a wave crossing empty space never waits on memory
        const bool any = !wc.sum || ((wc.sum[wi >> 5] >> (wi & 31u)) & 1u);
        wc.word = any ? reinterpret_cast<const uint64_t*>(p.bitfield)[wi] : 0ull;
        wc.idx = wi;
    }
    const bool occ = (wc.word >> (idx & 63u)) & 1ull;
    if (occ) return true;
    const float tx = (((nx + 0.5f + 0.5f * copysignf(1.0f, d[0])) * grid_size_inv * 2 - 1) * mip_bound - x) * dinv[0];
    const float ty = (((ny + 0.5f + 0.5f * copysignf(1.0f, d[1])) * grid_size_inv * 2 - 1) * mip_bound - y) * dinv[1];
    const float tz = (((nz + 0.5f + 0.5f * copysignf(1.0f, d[2])) * grid_size_inv * 2 - 1) * mip_bound - z) * dinv[2];
    t_target = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    return false;
}

// march_probe<true>'s per-launch constants, computed once (the wave march
// keeps them in scalar registers: uniform VALU results would otherwise sit in
// VGPRs for the whole kernel)
struct ProbeConsts {
    float mip_bound, mip_bound_inv, grid_f, grid_size_inv, gm1;
};
__device__ __forceinline__ float uniform_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}
__device__ __forceinline__ ProbeConsts probe_consts(const MarchParams& p) {
    ProbeConsts c;
    c.mip_bound = uniform_f(fminf(0.5f, p.scale));
    c.mip_bound_inv = uniform_f(1 / c.mip_bound);
    c.grid_f = uniform_f((float)p.grid_size);
    c.grid_size_inv = uniform_f(1.0f / p.grid_size);
    c.gm1 = uniform_f(p.grid_size - 1.0f);
    return c;
}
// march_probe<true> with the constants precomputed: the same expressions,
// operand for operand (bit-identical)
__device__ __forceinline__ bool march_probe_simple(float t, const float o[3], const float d[3], const float dinv[3],
                                                   const MarchParams& p, const ProbeConsts& k, WordCache& wc,
                                                   float& t_target) {
    const uint32_t G = (uint32_t)p.grid_size;
    const float x = o[0] + t * d[0], y = o[1] + t * d[1], z = o[2] + t * d[2];
    const int nx = (int)clampf(0.5f * (x * k.mip_bound_inv + 1) * k.grid_f, 0.0f, k.gm1);
    const int ny = (int)clampf(0.5f * (y * k.mip_bound_inv + 1) * k.grid_f, 0.0f, k.gm1);
    const int nz = (int)clampf(0.5f * (z * k.mip_bound_inv + 1) * k.grid_f, 0.0f, k.gm1);
    (void)G;
    const uint32_t idx = morton3((uint32_t)nx, (uint32_t)ny, (uint32_t)nz);
    const uint32_t wi = idx >> 6;
    if (wi != wc.idx) {
        const bool any = !wc.sum || ((wc.sum[wi >> 5] >> (wi & 31u)) & 1u);
        wc.word = any ? reinterpret_cast<const uint64_t*>(p.bitfield)[wi] : 0ull;
        wc.idx = wi;
    }
    const bool occ = (wc.word >> (idx & 63u)) & 1ull;
    if (occ) return true;
    const float tx = (((nx + 0.5f + 0.5f * copysignf(1.0f, d[0])) * k.grid_size_inv * 2 - 1) * k.mip_bound - x) * dinv[0];
    const float ty = (((ny + 0.5f + 0.5f * copysignf(1.0f, d[1])) * k.grid_size_inv * 2 - 1) * k.mip_bound - y) * dinv[1];
    const float tz = (((nz + 0.5f + 0.5f * copysignf(1.0f, d[2])) * k.grid_size_inv * 2 - 1) * k.mip_bound - z) * dinv[2];
    t_target = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    return false;
}

template <bool SIMPLE>
__device__ __forceinline__ bool march_step(float& t, const float o[3], const float d[3], const float dinv[3],
                                           const MarchParams& p, float& x, float& y, float& z, float& dt,
                                           WordCache& wc) {
    float t_target;
    if (march_probe<SIMPLE>(t, o, d, dinv, p, x, y, z, dt, wc, t_target)) {
        t += dt;
        return true;
    }
    // (t past 2^24 steps of dt: t + dt == t, the reference's loop would never end -- only a
    // degenerate ray (huge t2) gets there; it ends the ray instead and counts a guard hit.)
    // Every step advances t while dt exceeds half an ulp of each t the loop visits, i.e. when
    // dt > 2^-24 max(|t|, |t_target|) (the general dt only grows along the ray): then the plain
    // loop runs; a per-step check inside it cost the test-time march 20-26 % (r6m)
    const bool advances = dt * 16777216.0f > fmaxf(fabsf(t), fabsf(t_target));
    if constexpr (SIMPLE) {
        if (advances) {
            do { t += dt; } while (t < t_target);
        } else {
            do {
                const float tn = t + dt;
                if (!(tn > t)) { t = INFINITY; ngp_guard_hit(); break; }
                t = tn;
            } while (t < t_target);
        }
    } else {
        if (advances) {
            do { t += calc_dt(t, p.esf, p.max_samples, p.grid_size, p.dt_scale); } while (t < t_target);
        } else {
            do {
                const float tn = t + calc_dt(t, p.esf, p.max_samples, p.grid_size, p.dt_scale);
                if (!(tn > t)) { t = INFINITY; ngp_guard_hit(); break; }
                t = tn;
            } while (t < t_target);
        }
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

// ---------------------------------------------- wave-per-ray lattice march
// For SIMPLE launches (one cascade, esf = 0) every t the walk ever holds is a
// point of the lattice t_0, t_{k+1} = fl(t_k + dt) with a constant dt, and
// that lattice has a closed form: inside one binade [2^e, 2^(e+1)) adding dt
// moves a multiple of the binade's ulp u by the SAME multiple of u every time
// (dt/u has no exact .5 fraction; with one, the increment is constant from
// the second step on), so t_k = t_s + (k - s) * inc_s exactly (fmaf of an
// exact product).  The walk (march_step) from point k goes to k + 1 when the
// cell at t_k is occupied, else to the first j > k with t_j >= t_target(k).
// So one wave takes one ray: lane i evaluates lattice point c + i of a
// 64-point window (occupancy + jump target, in parallel), then the wave
// follows the walk's chain through the window with scalar readlanes and
// writes the visited occupied points with one coalesced store.  Bit-identical
// to the serial walk; ~8192 waves per batch instead of 128 latency-bound ones.
//
// Segment table (per ray, in LDS): segment q starts at lattice index K[q]
// with value T[q] and advances by I[q] per index until K[q + 1].
constexpr int LSEG = 32;
struct LatSeg {
    int K[LSEG + 1];
    float T[LSEG], I[LSEG];
};

__device__ __forceinline__ float lat_t(const LatSeg& sg, int q, int k) {
    return fmaf((float)(k - sg.K[q]), sg.I[q], sg.T[q]);
}

// Builds the segments from t0 (>= 0) until the lattice passes t2 and returns
// k_end = first index with t >= t2 (the walk's stop), or -1 if the table
// overflows (caller falls back to the serial walk).  Wave-uniform.
__device__ __forceinline__ int lat_build(float t0, float t2, float dt, LatSeg& sg, int& nseg, bool write) {
    int k = 0, q = 0;
    float ts = t0;
    while (true) {
        if (!(ts < t2)) {  // this point already stops the walk
            if (write) sg.K[q] = k;
            nseg = q;
            return k;
        }
        if (q == LSEG) return -1;
        int e;
        frexpf(ts, &e);
        const float upper = ldexpf(1.0f, e);  // binade [upper/2, upper)
        const float a = ts + dt, b = a + dt;
        int n_max;  // last index offset of this segment
        float inc;
        if (!(a > ts)) return -1;  // dt below half an ulp: no progress, leave it to the serial walk
        if (!(b < upper) || (b - a) != (a - ts)) {
            n_max = 0;  // single-point segment (binade end or a tie step)
            inc = a - ts;
        } else {
            inc = a - ts;
            n_max = (int)ceilf((upper - ts) / inc) - 1;
            while (fmaf((float)(n_max + 1), inc, ts) < upper) ++n_max;
            while (n_max > 0 && !(fmaf((float)n_max, inc, ts) < upper)) --n_max;
        }
        if (write) { sg.K[q] = k; sg.T[q] = ts; sg.I[q] = inc; }
        // the stop may fall inside this segment
        const float last = fmaf((float)n_max, inc, ts);
        if (!(last < t2)) {
            int n = (int)ceilf((t2 - ts) / inc);
            n = max(0, min(n, n_max));
            while (n > 0 && !(fmaf((float)(n - 1), inc, ts) < t2)) --n;
            while (fmaf((float)n, inc, ts) < t2) ++n;
            if (write) sg.K[q + 1] = k + n_max + 1;
            nseg = q + 1;
            return k + n;
        }
        ts = last + dt;  // the step that leaves the binade, as the walk rounds it
        k += n_max + 1;
        ++q;
    }
}

// first j > k with t_j >= T (capped at k_end), k in segment q
__device__ __forceinline__ int lat_jump(const LatSeg& sg, int nseg, int q, int k, float T, int k_end) {
    int j = k + 1;
    while (q + 1 < nseg && j >= sg.K[q + 1]) ++q;
    while (j < k_end) {
        const float tj = lat_t(sg, q, j);
        if (tj >= T) return j;
        const int send = q + 1 < nseg ? sg.K[q + 1] : k_end;
        const float need = (T - tj) / sg.I[q];
        // jump close to the answer, then fix up with exact lattice values
        int m = need < 4096.f ? max(1, (int)need) : 4096;
        int jj = min(j + m, send);
        while (jj > j + 1 && lat_t(sg, q, jj - 1) >= T) --jj;
        if (jj >= send) {  // target lies beyond this segment
            if (send >= k_end) return k_end;
            j = send;
            ++q;
            continue;
        }
        while (jj < send && lat_t(sg, q, jj) < T) ++jj;
        if (jj < send) return jj;
        if (send >= k_end) return k_end;
        j = send;
        ++q;
    }
    return k_end;
}

}  // namespace ngp

using ngp::MarchParams;

// cascades == 1 and esf == 0 (the Lego configuration): see march_step.
// Also requires the bitfield to be 8-byte aligned for the word loads (torch
// allocations are).  dt_scale must be >= 0 so the constant-dt fold holds.
static inline bool march_simple(const MarchParams& p) { return p.cascades == 1 && p.esf == 0.0f && p.dt_scale >= 0.0f; }

static inline int march_params(const uint8_t* bf, int cascades, int grid_size, float scale, float esf, int max_samples,
                        MarchParams& p) {
    if (!bf || cascades < 1 || grid_size < 4 || grid_size > 1024 || max_samples < 1) return NGP_EINVAL;
    if (((uintptr_t)bf & 7u) != 0) return NGP_EINVAL;  // 64-bit word loads
    p.bitfield = bf; p.summary = nullptr; p.n_sum32 = 0; p.cascades = cascades; p.grid_size = grid_size; p.max_samples = max_samples;
    p.scale = scale; p.esf = esf; p.dt_scale = scale;
    return NGP_OK;
}


// Attach a bitfield summary (ngp_bitfield_summary output for this bitfield).
// Requires the LDS copy to fit the launch's dynamic LDS budget.
constexpr int MAX_SUM32 = 8192;  // 2 x 32 KB of LDS: cascades * G^3 <= 2^24 cells
static inline int march_attach_summary(MarchParams& p, const uint32_t* summary) {
    if (!summary) return NGP_OK;
    const int64_t cells = (int64_t)p.cascades * p.grid_size * p.grid_size * p.grid_size;
    if (cells % 2048 != 0) return NGP_EINVAL;  // whole summary words
    if (cells / 2048 > MAX_SUM32) return NGP_ERANGE;
    p.summary = summary;
    p.n_sum32 = (int)(cells / 2048);
    return NGP_OK;
}
// LDS for the summary and its dilation (both n_sum32 words)
static inline size_t march_summary_lds(const MarchParams& p) { return (size_t)2 * p.n_sum32 * sizeof(uint32_t); }
