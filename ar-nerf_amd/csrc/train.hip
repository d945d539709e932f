// Training-step kernels around the field: fused compositing + loss +
// compositing backward, fused Adam with the fp16 shadow write and gradient
// zeroing, and the occupancy-grid EMA / threshold / scatter of the
// density-grid update.  Replaces (train.py:174-200, losses.py:63-82,
// apex FusedAdam at train.py:146, models/networks.py:252-281).
#pragma clang fp contract(off)

#include "common.h"
#include "transmittance.h"

namespace ngp {

// Zeroes n 64-bit words in stream order.  Used instead of hipMemsetAsync for
// the small counters zeroed inside captured graphs: in the exact-mode step
// graph a captured 8-byte memset was not reliably ordered before the kernel
// that reads the counter (ngp_guard_hits counted the fallout), a kernel node
// is.
__global__ void zero_words_kernel(unsigned long long* __restrict__ p, int n) {
    if ((int)threadIdx.x < n) p[threadIdx.x] = 0ull;
}


// ------------------------------------------------------ composite + loss
// One wave per ray.  Pass 1 = composite_train_fw (volumerendering.cu:5-44),
// the transmittance chain walked sample by sample in lane order (readlane)
// with the reference's early break;
// then the background blend (models/rendering.py:287-296) and NeRFLoss
// (losses.py:63-82: rgb loss of type `loss_type`, opacity entropy, depth
// term, distortion term when lambda_distortion > 0) with its analytic
// gradient; pass 2 = composite_train_bw (volumerendering.cu:86-150) with
// dL/dws from the distortion loss (DistortionLoss fw / bw, losses.cu:8-140,
// over the ray's composited samples: the others have ws = 0 and the
// compositing backward stops at the termination anyway).
// Per-ray outputs: rgb (after bg), opacity, depth, loss contribution
// (already divided by the batch means' denominators).
struct LossArgs {
    int loss_type;  // 0 raw (default, opt.py:34), 1 mse (upstream ngp_pl), 2 log, 3 tanh
    float lambda_opacity, lambda_depth, depth_scale, inv_n_rays, T_thr;
    float lambda_dist;  // losses.py:77-80 (0: off, the default)
};

__device__ __forceinline__ void rgb_loss(int type, float x, float y, float& l, float& dldx) {
    switch (type) {
        case 0: {  // (x - y)/(x.detach() + 1e-3), squared
            const float den = x + 1e-3f, d = (x - y) / den;
            l = d * d; dldx = 2.f * d / den; break;
        }
        case 1: { const float d = x - y; l = d * d; dldx = 2.f * d; break; }
        case 2: {
            const float u = logf((0.2935f + x) / (0.2935f + y)) * 0.7607f;
            l = u * u; dldx = 2.f * u * 0.7607f / (0.2935f + x); break;
        }
        default: {
            const float tx = tanhf(x), u = tx - tanhf(y);
            l = u * u; dldx = 2.f * u * (1.f - tx * tx); break;
        }
    }
}

// wave-wide sum / inclusive prefix sum (the reference's per-ray serial sums,
// reassociated: fp32 sums over <= 64 lanes then carried chunk to chunk)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_incl_scan(float v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const float y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    return v;
}

// (ChunkT / chunk_transmittance: transmittance.h, shared with the field forward)

// One row of rays_a on one wave; returns the composited sample count
// (vr_samples' share of this ray) and, in na_out, the samples that carry
// gradient (up to and including the terminating one).  DIST: the distortion
// loss is on (lambda_dist != 0; its code and registers are left out otherwise).
template <bool DIST>
__device__ __forceinline__ int64_t composite_loss_ray(
    int64_t n, const float* __restrict__ sigmas, const float* __restrict__ rgbs, const float* __restrict__ deltas,
    const float* __restrict__ ts, const int64_t* __restrict__ rays_a, const float* __restrict__ gt,
    const float* __restrict__ bg, const LossArgs& la, float* __restrict__ dL_dsig, float* __restrict__ dL_drgbs,
    float* __restrict__ out_rgb, float* __restrict__ out_op, float* __restrict__ out_depth,
    float* __restrict__ out_loss, int32_t* __restrict__ n_active, int64_t& na_out) {
    const int lane = threadIdx.x & 63;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
    // The first two 64-sample chunks (most rows terminate within them) are
    // loaded together up front and kept in registers for the backward: two
    // memory round trips per row instead of one per chunk and pass.
    struct Chunk {
        float sg, dl, cr, cg, cb, tt, w, Ta;
    };
    auto load = [&](int64_t k0, Chunk& c) {
        const int64_t s = start + k0 + lane;
        c.sg = c.dl = c.cr = c.cg = c.cb = c.tt = 0.f;
        if (k0 + lane < N) {
            c.sg = sigmas[s]; c.dl = deltas[s]; c.tt = ts[s];
            c.cr = rgbs[3 * s]; c.cg = rgbs[3 * s + 1]; c.cb = rgbs[3 * s + 2];
        }
    };
    Chunk c0, c1;
    load(0, c0);
    if (N > 64) load(64, c1);
    // ---- forward
    float T = 1.0f, R = 0.f, G = 0.f, B = 0.f, D = 0.f, O = 0.f;
    int64_t samples = 0, na = 0;
    bool done = false;
    auto fw_chunk = [&](int64_t k0, Chunk& c) {
        const int cnt = (int)(N - k0 < 64 ? N - k0 : 64);
        const float a = 1.0f - __expf(-c.sg * c.dl);
        const float om = 1.0f - a;
        const ChunkT ct = chunk_transmittance(om, cnt, T, la.T_thr, lane);
        const int stop = ct.stop;
        if (ct.hit) done = true;
        T = __shfl(ct.Tn, stop - 1, 64);
        const bool act = lane < stop;
        c.w = act ? a * ct.Tk : 0.f;
        c.Ta = ct.Tk * om;
        R += wave_sum(c.w * c.cr); G += wave_sum(c.w * c.cg); B += wave_sum(c.w * c.cb);
        D += wave_sum(c.w * c.tt); O += wave_sum(c.w);
        samples += done ? stop - 1 : stop;
        na += stop;
    };
    fw_chunk(0, c0);
    if (!done && N > 64) fw_chunk(64, c1);
    if (!done && N > 128) {  // long rows: the next chunk in flight while one is composited; w / T spilled
        Chunk c;
        load(128, c);
        for (int64_t k0 = 128; k0 < N && !done; k0 += 64) {
            Chunk nx;
            if (k0 + 64 < N) load(k0 + 64, nx);
            fw_chunk(k0, c);
            const int64_t s = start + k0 + lane;
            if (k0 + lane < N) { dL_drgbs[3 * s] = c.w; dL_drgbs[3 * s + 1] = c.Ta; }
            c = nx;
        }
    }
    // ---- background + loss (wave-uniform)
    const float bgc[3] = {bg[0], bg[1], bg[2]};
    const float xc[3] = {R + bgc[0] * (1 - O), G + bgc[1] * (1 - O), B + bgc[2] * (1 - O)};
    float loss = 0.f, g[3], gop = 0.f;
    const float inv3n = la.inv_n_rays / 3.0f;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        float l, d;
        rgb_loss(la.loss_type, xc[q], gt[3 * ray + q], l, d);
        loss += l * inv3n;
        g[q] = d * inv3n;
        gop -= g[q] * bgc[q];
    }
    const float o = O + 1e-10f;
    loss += la.lambda_opacity * (-o * logf(o)) * la.inv_n_rays;
    gop += la.lambda_opacity * (-(logf(o) + 1.f)) * la.inv_n_rays;
    float gdep = 0.f;
    if (la.lambda_depth != 0.f) {
        const float v = D / la.depth_scale + 1e-10f;
        loss += -la.lambda_depth * logf(fminf(v, 1.0f)) * la.inv_n_rays;
        if (v < 1.0f) gdep = -la.lambda_depth / v / la.depth_scale * la.inv_n_rays;
    }
    // ---- distortion loss (losses.py:77-80): its forward over the composited
    // samples (W_tot = O, WT_tot = D are the ray's sums of ws and ws*ts) and
    // dL/dws per sample (losses.cu:110-140); the ray's sum of dL/dws * ws is
    // needed before the compositing backward's first sample: a pass of its own.
    // Rows longer than two chunks park dL/dws in dL_dsig[s] (overwritten by
    // pass 2 after it is read).
    float gws_c[2] = {0.f, 0.f}, S_ws = 0.f;
    if (DIST) {
        const float gd2 = (la.lambda_dist * la.inv_n_rays) * 2;
        float cw = 0.f, cwt = 0.f, ld = 0.f;
        auto dist_chunk = [&](int64_t k0, const Chunk& c) {
            const int cnt = (int)(na - k0 < 64 ? na - k0 : 64);
            const bool in = lane < cnt;
            const float w = in ? c.w : 0.f, wt = w * c.tt;
            const float a = cw + wave_incl_scan(w, lane), b = cwt + wave_incl_scan(wt, lane);
            const float we = a - w, wte = b - wt;  // exclusive sums (the reference's serial fold values)
            const float l = 2 * (b * we - a * wte) + ((w * (1.0f / 3)) * w) * c.dl;
            ld += wave_sum(in ? l : 0.f);
            const float A = c.tt * we - wte, Bv = (D - b) - c.tt * (O - a);
            const float gw = in ? gd2 * (A + Bv) + ((gd2 / 3.0f) * w) * c.dl : 0.f;
            S_ws += wave_sum(gw * w);
            cw = __shfl(a, 63, 64); cwt = __shfl(b, 63, 64);
            return gw;
        };
        if (na > 0) gws_c[0] = dist_chunk(0, c0);
        if (na > 64) gws_c[1] = dist_chunk(64, c1);
        for (int64_t k0 = 128; k0 < na; k0 += 64) {
            Chunk c;
            load(k0, c);
            const int64_t s = start + k0 + lane;
            c.w = 0.f;
            if (k0 + lane < na) c.w = dL_drgbs[3 * s];
            const float gw = dist_chunk(k0, c);
            if (k0 + lane < na) dL_dsig[s] = gw;
        }
        loss += la.lambda_dist * ld * la.inv_n_rays;
    }
    if (lane == 0) {
        out_rgb[3 * ray] = xc[0]; out_rgb[3 * ray + 1] = xc[1]; out_rgb[3 * ray + 2] = xc[2];
        out_op[ray] = O;
        out_depth[ray] = D;
        out_loss[ray] = loss;
        if (n_active) n_active[n] = (int32_t)na;
    }
    na_out = na;
    // ---- backward over the na composited samples
    const float gs = gop * (1 - O);
    float rc = 0.f, gc = 0.f, bc = 0.f, dc = 0.f, wc = 0.f;
    auto bw_chunk = [&](int64_t k0, const Chunk& c, float gw) {
        const int cnt = (int)(na - k0 < 64 ? na - k0 : 64);
        const bool in = lane < cnt;
        const int64_t s = start + k0 + lane;
        const float w = in ? c.w : 0.f, Ta = c.Ta;
        const float pr = rc + wave_incl_scan(w * c.cr, lane), pg = gc + wave_incl_scan(w * c.cg, lane);
        const float pb = bc + wave_incl_scan(w * c.cb, lane), pd = dc + wave_incl_scan(w * c.tt, lane);
        float ws_term = 0.f;
        if (DIST) {  // + T g_ws - (S - prefix(g_ws ws)) (volumerendering.cu:138-146)
            const float pw = wc + wave_incl_scan(in ? gw * w : 0.f, lane);
            ws_term = Ta * gw - (S_ws - pw);
            wc = __shfl(pw, 63, 64);
        }
        if (in) {
            dL_drgbs[3 * s] = g[0] * w; dL_drgbs[3 * s + 1] = g[1] * w; dL_drgbs[3 * s + 2] = g[2] * w;
            dL_dsig[s] = c.dl * (g[0] * (c.cr * Ta - (R - pr)) + g[1] * (c.cg * Ta - (G - pg)) +
                                 g[2] * (c.cb * Ta - (B - pb)) + gs + gdep * (c.tt * Ta - (D - pd)) + ws_term);
        }
        rc = __shfl(pr, 63, 64); gc = __shfl(pg, 63, 64); bc = __shfl(pb, 63, 64); dc = __shfl(pd, 63, 64);
    };
    if (na > 0) bw_chunk(0, c0, gws_c[0]);
    if (na > 64) bw_chunk(64, c1, gws_c[1]);
    for (int64_t k0 = 128; k0 < na; k0 += 64) {
        Chunk c;
        load(k0, c);
        const int64_t s = start + k0 + lane;
        c.w = 0.f; c.Ta = 0.f;
        float gw = 0.f;
        if (k0 + lane < na) {
            c.w = dL_drgbs[3 * s]; c.Ta = dL_drgbs[3 * s + 1];
            if (DIST) gw = dL_dsig[s];
        }
        bw_chunk(k0, c, gw);
    }
    return samples;
}

// Each block takes 4 rows per round (one per wave).  Per round the block
// sums its rows' gradient-carrying sample counts and reserves that many
// entries of sample_idx with ONE atomic on alloc[0]; each wave then writes
// its row's entries (start + k, k < na) -- a row's samples stay contiguous,
// which the hash backward's run merging relies on.  The last block to finish
// (alloc[1] ticket) publishes the total to *n_active_total and resets both
// counters, so the kernel needs no memset and no scan launch.  stats
// (nullable): [0] += marched samples, [1] += composited samples (vr_samples),
// [2] += gradient-carrying samples, summed per block in LDS, then one atomic
// per counter per block into stripe blockIdx % NGP_STAT_STRIPES (one address
// for all 2048 blocks serialised ~40 us of the kernel on the memory side).
// ---- decoupled look-back (ordered compaction across blocks in one launch)
// Workspace {ticket, done, generation, pad, status[blocks]}, zeroed once by
// the caller.  A block takes a ticket (its position in dispatch order: it
// only ever waits on blocks that started before it), publishes its
// aggregate, and one wave walks back over the status words 64 at a time,
// summing aggregates until the closest inclusive prefix; the last block to
// finish resets the ticket and advances the generation, so the words of the
// previous launch never match.  A status word carries its own value, so the
// hand-off is one 8-byte agent-scope atomic each way (sc1 store / sc1 poll,
// MI355X_MICROARCH.md "Valid forms"): no release / acquire fences -- an
// acquire poll or a release per block (L2 write-back of the whole XCD) made
// the step 60 % slower.  The lists themselves are read by later launches.
struct LookbackWs {
    uint32_t tick, done, gen, pad;
    unsigned long long status[1];  // [blocks]
};
constexpr unsigned long long LB_AGG = 1ull << 40, LB_INCL = 2ull << 40, LB_VAL = (1ull << 40) - 1;
__device__ __forceinline__ unsigned long long lb_word(uint32_t gen, unsigned long long flag, int64_t v) {
    return ((unsigned long long)(gen & 0x3fffffu) << 42) | flag | ((unsigned long long)v & LB_VAL);
}
// whole wave: publishes aggregate A of block b, returns the exclusive prefix
// of the blocks before it, publishes b's inclusive prefix
__device__ __forceinline__ int64_t lookback_prefix(LookbackWs* __restrict__ lb, uint32_t b, uint32_t gen, int64_t A,
                                                   int lane) {
    if (lane == 0)
        __hip_atomic_store(&lb->status[b], lb_word(gen, b == 0 ? LB_INCL : LB_AGG, A), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    int64_t P = 0;
    for (int64_t j = (int64_t)b - 1; j >= 0; j -= 64) {
        const int64_t q = j - lane;
        unsigned long long wv = LB_INCL;  // (q < 0: before block 0, an inclusive 0)
        // bounded: a predecessor publishes its aggregate without waiting on anyone, so this
        // ends in microseconds; the bound only keeps a corrupted workspace from hanging the
        // GPU (counted as a guard hit, ngp_guard_hits: the result is then wrong)
        for (uint32_t spin = 0;; ++spin) {
            if (q >= 0) wv = __hip_atomic_load(&lb->status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool ok = q < 0 || ((uint32_t)(wv >> 42) == (gen & 0x3fffffu) && (wv & (3ull << 40)) != 0);
            if (__all(ok)) break;
            if (spin == (1u << 22)) {
                if (lane == 0) ngp_guard_hit();
                wv = LB_INCL;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const bool incl = (wv & (3ull << 40)) == LB_INCL;
        const uint64_t m = __ballot(incl);
        const int k = m ? __ffsll((unsigned long long)m) - 1 : 63;
        int64_t v = lane <= k ? (int64_t)(wv & LB_VAL) : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        P += v;
        if (m) break;
    }
    if (lane == 0 && b > 0)
        __hip_atomic_store(&lb->status[b], lb_word(gen, LB_INCL, P + A), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return P;
}
// one thread per block, after the block's last use of its ticket
__device__ __forceinline__ void lookback_finish(LookbackWs* __restrict__ lb, uint32_t gen, uint32_t nb) {
    if (__hip_atomic_fetch_add(&lb->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) {
        __hip_atomic_store(&lb->tick, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&lb->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&lb->gen, gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <bool DIST>
__global__ void __launch_bounds__(256) composite_loss_wave_kernel(
    const float* __restrict__ sigmas, const float* __restrict__ rgbs, const float* __restrict__ deltas,
    const float* __restrict__ ts, const int64_t* __restrict__ rays_a, int64_t n_rays, const float* __restrict__ gt,
    const float* __restrict__ bg, LossArgs la, float* __restrict__ dL_dsig, float* __restrict__ dL_drgbs,
    float* __restrict__ out_rgb, float* __restrict__ out_op, float* __restrict__ out_depth,
    float* __restrict__ out_loss, int32_t* __restrict__ n_active, int32_t* __restrict__ sample_idx,
    unsigned long long* __restrict__ alloc, int64_t* __restrict__ n_active_total, int64_t* __restrict__ stats) {
    __shared__ unsigned long long blk[3];
    __shared__ int64_t s_na[4];
    __shared__ unsigned long long s_base;
    NGP_PROBE_BEGIN(NGP_P_COMPOSITE);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x < 3) blk[threadIdx.x] = 0;
    __syncthreads();
    int64_t rm = 0, vr = 0, act = 0;
    for (int64_t r0 = (int64_t)blockIdx.x * 4; r0 < n_rays; r0 += (int64_t)gridDim.x * 4) {
        const int64_t n = r0 + wid;
        int64_t na = 0, start = 0;
        if (n < n_rays) {
            vr += composite_loss_ray<DIST>(n, sigmas, rgbs, deltas, ts, rays_a, gt, bg, la, dL_dsig, dL_drgbs, out_rgb,
                                     out_op, out_depth, out_loss, n_active, na);
            start = rays_a[3 * n + 1];
            rm += rays_a[3 * n + 2];
            act += na;
        }
        if (sample_idx) {
            if (lane == 0) s_na[wid] = na;
            __syncthreads();
            if (threadIdx.x == 0) {
                const int64_t tot = s_na[0] + s_na[1] + s_na[2] + s_na[3];
                s_base = tot ? atomicAdd(alloc, (unsigned long long)tot) : 0ull;
            }
            __syncthreads();
            int64_t off = (int64_t)s_base;
            for (int w = 0; w < wid; ++w) off += s_na[w];
            for (int64_t k = lane; k < na; k += 64) sample_idx[off + k] = (int32_t)(start + k);
            __syncthreads();  // s_na / s_base are rewritten next round
        }
    }
    if (lane == 0) {
        atomicAdd(&blk[0], (unsigned long long)rm);
        atomicAdd(&blk[1], (unsigned long long)vr);
        atomicAdd(&blk[2], (unsigned long long)act);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (stats) {
            unsigned long long* st = (unsigned long long*)stats + (blockIdx.x % NGP_STAT_STRIPES) * NGP_STAT_STRIDE;
            if (blk[0]) atomicAdd(st, blk[0]);
            if (blk[1]) atomicAdd(st + 1, blk[1]);
            if (blk[2]) atomicAdd(st + 2, blk[2]);
        }
        if (sample_idx) {
            __threadfence();
            const unsigned long long ticket = atomicAdd(alloc + 1, 1ull);
            if (ticket == gridDim.x - 1) {  // last block: every reservation is done
                const unsigned long long total = atomicExch(alloc, 0ull);
                atomicExch(alloc + 1, 0ull);
                *n_active_total = (int64_t)total;
            }
        }
    }
    NGP_PROBE_END();
}

// ------------------------------------------------------------------ Adam
// apex FusedAdam, adam_w_mode with weight_decay 0 == Adam (train.py:146):
//   m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2
//   p -= lr * (m / bc1) / (sqrt(v / bc2) + eps)
// g = grad * grad_scale (1/world_size after an all-reduce SUM).  Writes the
// fp16 shadow the kernels read and zeroes the gradient for the next step.
// 4 params per lane, 16-B loads/stores.
// lr_dev / step_dev (nullable): learning rate and the 0-based count of steps
// already taken read from device memory (graph replays), bias corrections
// for step *step_dev + 1 computed here (same fp32 powf as the host path).
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, float* __restrict__ grad, float* __restrict__ m,
                                                   float* __restrict__ v, _Float16* __restrict__ p16, int64_t n4,
                                                   float lr, float b1, float b2, float eps, float bc1, float bc2,
                                                   float grad_scale, int zero_grad, const float* __restrict__ lr_dev,
                                                   const int64_t* __restrict__ step_dev, float* __restrict__ rep = nullptr,
                                                   int64_t rep_lo4 = 0, int64_t rep4 = 0, int nrep = 0,
                                                   float* __restrict__ zero = nullptr, int64_t zero4 = 0) {
    NGP_PROBE_BEGIN(NGP_P_ADAM);
    adam_bias(lr_dev, step_dev, b1, b2, lr, bc1, bc2);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 P = reinterpret_cast<float4*>(p)[i], Gd = reinterpret_cast<float4*>(grad)[i];
        float4 M = reinterpret_cast<float4*>(m)[i], V = reinterpret_cast<float4*>(v)[i];
        const int64_t j = i - rep_lo4;
        if (rep && j >= 0 && j < rep4) {  // gradient replicas (ngp_hash_backward_levels_rep), folded in order
            // One replica in flight per lane (round 5): the kernel's 60 VGPRs let one Adam wave per SIMD
            // run beside the accumulation's 1024-thread blocks (105 VGPRs), where with all 8 replicas'
            // loads issued first (round 3) it waited for those blocks to retire: +2.0 % end to end with
            // the accumulation's prefetch at one group (profiles/r05/ab/round5_ab.txt r5bb / r5cc).
            float4* r4 = reinterpret_cast<float4*>(rep);
            for (int r = 0; r < nrep; ++r) {
                const float4 c = r4[r * rep4 + j];
                Gd.x += c.x; Gd.y += c.y; Gd.z += c.z; Gd.w += c.w;
                r4[r * rep4 + j] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        float* pp = &P.x; float* gp = &Gd.x; float* mp = &M.x; float* vp = &V.x;
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 out;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            adam_elem(pp[k], mp[k], vp[k], gp[k] * grad_scale, lr, b1, b2, eps, bc1, bc2);
            out[k] = (_Float16)pp[k];
        }
        reinterpret_cast<float4*>(p)[i] = P;
        reinterpret_cast<float4*>(m)[i] = M;
        reinterpret_cast<float4*>(v)[i] = V;
        reinterpret_cast<h4*>(p16)[i] = out;
        if (zero_grad) reinterpret_cast<float4*>(grad)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // (ngp_adam_step_dev_zero) a second range cleared by the same launch
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < zero4; i += stride)
        reinterpret_cast<float4*>(zero)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    NGP_PROBE_END();
}

// --------------------------------------------------- occupancy grid update
// density_grid_tmp[c, idx] = sigma (models/networks.py:268) as a torch
// index_put_ over the cell list: with duplicate cells the LAST write in list
// order wins (torch's sequential semantics; sample_uniform_and_occupied_cells
// draws i.i.d., so a duplicated cell keeps its last draw's sigma, and a cell
// drawn in both halves keeps the occupied-half draw).  Each sample i at list
// position pos_base + i leaves the 64-bit key ((pos + 1) << 32 | sigma bits)
// with a 64-bit atomicMax, so the largest position wins independently of
// execution order; ranks sharding the list combine their key grids with a MAX
// all-reduce, the same rule across ranks.  Negative indices are skipped
// (occupancy samples that do not exist: no occupied cell to resample).
__global__ void scatter_last_kernel(const int64_t* __restrict__ idx, const float* __restrict__ sig, int64_t n,
                                    int64_t pos_base, unsigned long long* __restrict__ key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t j = idx[i];
    if (j < 0) return;
    const unsigned long long k = ((unsigned long long)(pos_base + i + 1) << 32) | __float_as_uint(fmaxf(sig[i], 0.f));
    atomicMax(key + j, k);
}

// ---------------------------------------- occupancy cell sampling on device
// sample_uniform_and_occupied_cells (models/networks.py:181-207) without the
// host sync of torch.nonzero: occ_count_kernel + occ_list_kernel list the
// cells of one cascade with density > threshold in ascending cell order, as
// torch.nonzero does (two launches: per-block counts, then each block sums
// the counts of the blocks before it and writes its run -- deterministic, so
// every rank of a data-parallel job builds the same list);
// occ_sample_kernel draws M uniform cells and M cells uniformly from that
// list (none if it is empty, as the reference's empty nonzero gives none)
// and their jittered world positions (networks.py:262-266).
constexpr int OCC_T = 1024, OCC_PER = 8, OCC_CHUNK = OCC_T * OCC_PER;  // cells per block

__device__ __forceinline__ uint32_t occ_hits(const float* __restrict__ grid_c, int64_t n_cells, float thr, int64_t c0,
                                             bool hit[OCC_PER]) {
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < OCC_PER; ++k) {
        hit[k] = c0 + k < n_cells && grid_c[c0 + k] > thr;
        mine += hit[k];
    }
    return mine;
}

__global__ void __launch_bounds__(OCC_T) occ_count_kernel(const float* __restrict__ grid_c, int64_t n_cells, float thr,
                                                          uint32_t* __restrict__ block_counts) {
    __shared__ uint32_t wcnt[OCC_T / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    bool hit[OCC_PER];
    uint32_t v = occ_hits(grid_c, n_cells, thr, ((int64_t)blockIdx.x * OCC_T + tid) * OCC_PER, hit);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) wcnt[wid] = v;
    __syncthreads();
    if (tid == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < OCC_T / 64; ++w) tot += wcnt[w];
        block_counts[blockIdx.x] = tot;
    }
}

__global__ void __launch_bounds__(OCC_T) occ_list_kernel(const float* __restrict__ grid_c, int64_t n_cells, float thr,
                                                         const uint32_t* __restrict__ block_counts,
                                                         int32_t* __restrict__ list,
                                                         unsigned long long* __restrict__ count) {
    __shared__ uint32_t wcnt[OCC_T / 64];
    __shared__ unsigned long long wbase[OCC_T / 64];
    __shared__ unsigned long long base;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // this block's base: the counts of the blocks before it, summed by every
    // wave over a strided share (a few hundred words, L2-resident)
    unsigned long long before = 0ull;
    for (int64_t b = tid; b < (int64_t)blockIdx.x; b += OCC_T) before += block_counts[b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o, 64);
    if (lane == 0) wbase[wid] = before;
    bool hit[OCC_PER];
    const int64_t c0 = ((int64_t)blockIdx.x * OCC_T + tid) * OCC_PER;
    const uint32_t mine = occ_hits(grid_c, n_cells, thr, c0, hit);
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wcnt[wid] = incl;
    __syncthreads();
    if (tid == 0) {
        unsigned long long b = 0ull;
        for (int w = 0; w < OCC_T / 64; ++w) b += wbase[w];
        uint32_t tot = 0;
        for (int w = 0; w < OCC_T / 64; ++w) { const uint32_t v = wcnt[w]; wcnt[w] = tot; tot += v; }
        base = b;
        if (blockIdx.x == gridDim.x - 1) *count = b + tot;
    }
    __syncthreads();
    // (the list holds at most n_cells entries: a base past that can only come
    // from corrupted counts -- dropped instead of written)
    if (base > (unsigned long long)n_cells) {
        if (tid == 0) ngp_guard_hit();
        return;
    }
    int64_t pos = (int64_t)base + wcnt[wid] + incl - mine;
#pragma unroll
    for (int k = 0; k < OCC_PER; ++k)
        if (hit[k] && pos < n_cells) list[pos++] = (int32_t)(c0 + k);
}

__global__ void __launch_bounds__(256) occ_sample_kernel(uint64_t seed, const int64_t* __restrict__ ctr, int cascade,
                                                         int G, int64_t M, float s_minus_hgs, float hgs,
                                                         const int32_t* __restrict__ list,
                                                         const unsigned long long* __restrict__ count, int64_t lo,
                                                         int64_t hi, float* __restrict__ xyzs,
                                                         int64_t* __restrict__ flat) {
    const int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hi) return;
    const int64_t o = i - lo;
    const uint64_t step = (uint64_t)*ctr;
    const uint4 u = philox4x32(make_uint4((uint32_t)i, (uint32_t)(i >> 32), (uint32_t)step, (uint32_t)cascade),
                               make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    int32_t idx;
    if (i < M) {  // uniform cell: torch.randint(G, (M, 3)) then morton3D
        const uint4 v = philox4x32(make_uint4((uint32_t)i, (uint32_t)(i >> 32), (uint32_t)step, 0x9E3779B9u ^ cascade),
                                   make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
        idx = (int32_t)morton3((uint32_t)uniform_index(v.x, G), (uint32_t)uniform_index(v.y, G),
                               (uint32_t)uniform_index(v.z, G));
    } else {  // a cell drawn from the occupied list
        const unsigned long long cnt0 = *count, cnt = min(cnt0, (unsigned long long)G * G * G);  // (guard: list capacity)
        if (cnt0 != cnt && i == (lo > M ? lo : M)) ngp_guard_hit();
        if (cnt == 0) {
            flat[o] = -1;
            xyzs[3 * o] = 0.f; xyzs[3 * o + 1] = 0.f; xyzs[3 * o + 2] = 0.f;
            return;
        }
        idx = list[uniform_index(u.w, (int64_t)cnt)];
    }
    const uint32_t cx = compact3((uint32_t)idx), cy = compact3((uint32_t)idx >> 1), cz = compact3((uint32_t)idx >> 2);
    // xyzs_w = (coords / (G-1) * 2 - 1) * (s - hgs) + (rand * 2 - 1) * hgs, fp32 as torch evaluates it
    const float gm1 = (float)(G - 1);
    const float jr[3] = {(float)(u.x >> 8) * (1.0f / 16777216.0f), (float)(u.y >> 8) * (1.0f / 16777216.0f),
                         (float)(u.z >> 8) * (1.0f / 16777216.0f)};
    const uint32_t cc[3] = {cx, cy, cz};
#pragma unroll
    for (int d = 0; d < 3; ++d) xyzs[3 * o + d] = ((float)cc[d] / gm1 * 2.0f - 1.0f) * s_minus_hgs + (jr[d] * 2.0f - 1.0f) * hgs;
    flat[o] = (int64_t)cascade * G * G * G + idx;
}

// Sorted variant: the same two multisets of cells (M i.i.d. uniform cells, M
// i.i.d. uniform picks from the occupied list) emitted in ascending order, so
// that a wave's points share cache lines on the coarse hash levels (the
// density forward of the 1M points runs ~1.8x faster Morton-sorted than in
// draw order: scripts/diag/density_order.py).  Ascending i.i.d. uniforms are
// drawn directly as order statistics, U_(k) = S_k / S_M with S the running
// sum of M+1 i.i.d. Exp(1) variates (fp64), so no sort is needed: three
// launches -- block sums, one scan of the block sums, then each block
// regenerates its exponentials, scans them and writes its samples.
constexpr int OSC_T = 256, OSC_PER = 16, OSC_CH = OSC_T * OSC_PER;  // exponentials per block

__device__ __forceinline__ double occ_exp(uint64_t seed, uint64_t step, int cascade, int half, int64_t k) {
    const uint4 v = philox4x32(make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)step,
                                          0x7F4A7C15u ^ (uint32_t)(cascade << 1) ^ (uint32_t)half),
                               make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    const double u = ((double)(v.x >> 11) + 1.0) * (1.0 / 2097152.0);  // (0, 1], 21 bits
    const double u2 = u + (double)(v.y >> 11) * (1.0 / 2097152.0 / 2097152.0);  // 42-bit uniform
    return -log(fmin(u2, 1.0));
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(OSC_T) occ_exp_sums_kernel(uint64_t seed, const int64_t* __restrict__ ctr,
                                                             int cascade, int64_t M, int64_t nb,
                                                             double* __restrict__ sums) {
    __shared__ double red[OSC_T / 64];
    const int half = (int)(blockIdx.x / nb);
    const int64_t c = blockIdx.x % nb;
    const uint64_t step = (uint64_t)*ctr;
    double v = 0.0;
#pragma unroll 4
    for (int j = 0; j < OSC_PER; ++j) {
        const int64_t k = c * OSC_CH + (int64_t)j * OSC_T + threadIdx.x;
        if (k <= M) v += occ_exp(seed, step, cascade, half, k);
    }
    v = block_sum_d(v, red);
    if (threadIdx.x == 0) sums[blockIdx.x] = v;
}

// exclusive prefix of the block sums within each half (in place), totals
// after; one workgroup per half, 1024 sums per round
__global__ void __launch_bounds__(1024) occ_exp_scan_kernel(int64_t nb, double* __restrict__ sums) {
    __shared__ double wsum[16];
    __shared__ double carry_s;
    double* p = sums + blockIdx.x * nb;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) carry_s = 0.0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < nb; b0 += 1024) {
        const int64_t b = b0 + t;
        const double v = b < nb ? p[b] : 0.0;
        double incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const double y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        double before = carry_s;
        for (int q = 0; q < w; ++q) before += wsum[q];
        if (b < nb) p[b] = before + incl - v;
        __syncthreads();
        if (t == 1023) carry_s = before + incl;
        __syncthreads();
    }
    if (t == 0) sums[2 * nb + blockIdx.x] = carry_s;
}

__global__ void __launch_bounds__(OSC_T) occ_sample_sorted_kernel(
    uint64_t seed, const int64_t* __restrict__ ctr, int cascade, int G, int64_t M, int64_t nb, float s_minus_hgs,
    float hgs, const int32_t* __restrict__ list, const unsigned long long* __restrict__ count,
    const double* __restrict__ sums, int64_t lo, int64_t hi, float* __restrict__ xyzs, int64_t* __restrict__ flat) {
    __shared__ double wsum[OSC_T / 64];
    const int half = (int)(blockIdx.x / nb);
    const int64_t c = blockIdx.x % nb;
    const int64_t i0 = half * M + c * OSC_CH;  // sample index of this block's first exponential
    if (i0 >= hi || i0 + OSC_CH <= lo) return;  // (block-uniform)
    const uint64_t step = (uint64_t)*ctr;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // thread t takes the OSC_PER consecutive exponentials k0 + t*OSC_PER + j
    const int64_t k0 = c * OSC_CH + (int64_t)t * OSC_PER;
    double e[OSC_PER], loc = 0.0;
#pragma unroll
    for (int j = 0; j < OSC_PER; ++j) {
        e[j] = k0 + j <= M ? occ_exp(seed, step, cascade, half, k0 + j) : 0.0;
        loc += e[j];
    }
    double incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    double run = sums[blockIdx.x];
    for (int q = 0; q < w; ++q) run += wsum[q];
    run += incl - loc;
    const double inv_tot = 1.0 / sums[2 * nb + half];
    const int64_t n_cells = (int64_t)G * G * G;
    const unsigned long long cnt0 = half ? *count : 0ull, cnt = min(cnt0, (unsigned long long)n_cells);  // (guard: capacity)
    if (cnt0 != cnt && threadIdx.x == 0) ngp_guard_hit();
    const float gm1 = (float)(G - 1);
#pragma unroll 1
    for (int j = 0; j < OSC_PER; ++j) {
        run += e[j];
        const int64_t k = k0 + j, i = half * M + k;
        if (k >= M || i < lo || i >= hi) continue;
        const int64_t o = i - lo;
        const double u = run * inv_tot;  // U_(k), ascending in k
        int32_t idx;
        if (!half) {
            idx = (int32_t)min((int64_t)(u * (double)n_cells), n_cells - 1);
        } else {
            if (cnt == 0) {
                flat[o] = -1;
                xyzs[3 * o] = 0.f; xyzs[3 * o + 1] = 0.f; xyzs[3 * o + 2] = 0.f;
                continue;
            }
            idx = list[min((int64_t)(u * (double)cnt), (int64_t)cnt - 1)];
        }
        const uint4 r = philox4x32(make_uint4((uint32_t)i, (uint32_t)(i >> 32), (uint32_t)step, (uint32_t)cascade),
                                   make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
        const uint32_t cc[3] = {compact3((uint32_t)idx), compact3((uint32_t)idx >> 1), compact3((uint32_t)idx >> 2)};
        const float jr[3] = {(float)(r.x >> 8) * (1.0f / 16777216.0f), (float)(r.y >> 8) * (1.0f / 16777216.0f),
                             (float)(r.z >> 8) * (1.0f / 16777216.0f)};
#pragma unroll
        for (int d = 0; d < 3; ++d)
            xyzs[3 * o + d] = ((float)cc[d] / gm1 * 2.0f - 1.0f) * s_minus_hgs + (jr[d] * 2.0f - 1.0f) * hgs;
        flat[o] = (int64_t)cascade * n_cells + idx;
    }
}

// The occupancy samples whose sigma survives density_grid_tmp[c, idx] =
// sigma's last-write-wins (networks.py:268): of the sorted 2M-sample list
// (each half ascending, ngp_occupancy_samples_sorted), position i is kept iff
// no later position holds its cell -- the last of its run within its half
// (duplicates are adjacent there), and, in the uniform half, only if the
// occupied half does not draw the cell at all.  Only kept positions need a
// density evaluation: the others' sigmas would be overwritten.
// occ_mark_kernel: byte per cell, set for every occupied-half cell (plain
// byte stores of one value: no atomics); occ_keep_kernel: the kept positions
// of [lo, hi), compacted per 8192-position block (one reservation per block).
__global__ void __launch_bounds__(256) zero_u4_kernel(uint4* __restrict__ p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = make_uint4(0u, 0u, 0u, 0u);
}
__global__ void __launch_bounds__(256) occ_mark_kernel(const int64_t* __restrict__ flat, int64_t M, int64_t cell_base,
                                                       int64_t n_cells, uint8_t* __restrict__ mark) {
    const int64_t i = M + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= 2 * M) return;
    const int64_t c = flat[i] - cell_base;
    if (c >= 0 && c < n_cells) mark[c] = 1;
}

constexpr int KEEP_T = 1024, KEEP_PER = 8;
__global__ void __launch_bounds__(KEEP_T) occ_keep_kernel(const int64_t* __restrict__ flat, int64_t M,
                                                          int64_t cell_base, int64_t n_cells,
                                                          const uint8_t* __restrict__ mark, int64_t lo, int64_t hi,
                                                          int32_t* __restrict__ list,
                                                          unsigned long long* __restrict__ count) {
    __shared__ uint32_t wcnt[KEEP_T / 64];
    __shared__ unsigned long long base;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t i0 = lo + ((int64_t)blockIdx.x * KEEP_T + tid) * KEEP_PER;
    bool keep[KEEP_PER];
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < KEEP_PER; ++k) {
        const int64_t i = i0 + k;
        bool kp = false;
        if (i < hi) {
            const int64_t f = flat[i];
            const int64_t end = i < M ? M : 2 * M;  // the end of i's half
            kp = f >= 0 && (i + 1 == end || flat[i + 1] != f);
            if (kp && i < M) {
                const int64_t c = f - cell_base;
                kp = !(c >= 0 && c < n_cells && mark[c]);
            }
        }
        keep[k] = kp;
        mine += kp;
    }
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wcnt[wid] = incl;
    __syncthreads();
    if (tid == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < KEEP_T / 64; ++w) { const uint32_t v = wcnt[w]; wcnt[w] = tot; tot += v; }
        base = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    int64_t pos = (int64_t)base + wcnt[wid] + incl - mine;
#pragma unroll
    for (int k = 0; k < KEEP_PER; ++k)
        if (keep[k]) list[pos++] = (int32_t)(i0 + k);
}

// scatter_last_kernel over the kept positions list[j], j < *count: sample i =
// list[j] (list position pos_base + i) with its cell flat[i] and sigma sig[i]
__global__ void __launch_bounds__(256) scatter_kept_kernel(const int32_t* __restrict__ list,
                                                           const int64_t* __restrict__ count, int64_t n_max,
                                                           const int64_t* __restrict__ flat,
                                                           const float* __restrict__ sig, int64_t pos_base,
                                                           unsigned long long* __restrict__ key) {
    const int64_t nk = ngp_capped_count(count, n_max);
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nk; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = list[j];
        const int64_t c = flat[i];
        if (c < 0) continue;
        const unsigned long long k = ((unsigned long long)(pos_base + i + 1) << 32) | __float_as_uint(fmaxf(sig[i], 0.f));
        atomicMax(key + c, k);
    }
}

// models/networks.py:270-278: grid = where(grid<0, grid, max(grid*decay, tmp)),
// decay per cell when decay_cells != nullptr (erode, networks.py:270-272:
// clamp(decay**(1/count_grid), 0.1, 0.95), evaluated once per count grid by the
// caller);
// accumulates sum and count of grid > 0 for the mean, in fp64 so the mean is
// the correctly rounded one whatever the summation order: at initialisation
// every cell holds sigma ~= 1 and the threshold (= that mean) splits them, so
// a last-digit difference in an fp32 sum flips thousands of cells and sends
// training down a different trajectory.
__global__ void __launch_bounds__(256) grid_ema_kernel(float* __restrict__ grid, unsigned long long* __restrict__ key,
                                                       int64_t n, float decay, const float* __restrict__ decay_cells,
                                                       double* __restrict__ sum_cnt) {
    double s = 0.0, c = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float gv = grid[i];
        const float dc = decay_cells ? decay_cells[i] : decay;
        const unsigned long long kv = key[i];
        const float tv = kv ? __uint_as_float((uint32_t)kv) : 0.f;  // density_grid_tmp (zeros where unsampled)
        const float nv = gv < 0 ? gv : fmaxf(gv * dc, tv);
        grid[i] = nv;
        if (kv) key[i] = 0ull;  // consumed: left zeroed for the next update
        if (nv > 0) { s += (double)nv; c += 1.0; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { s += __shfl_xor(s, o, 64); c += __shfl_xor(c, o, 64); }
    __shared__ double ws[2][4];  // one global add pair per block, not per wave
    if ((threadIdx.x & 63) == 0) { ws[0][threadIdx.x >> 6] = s; ws[1][threadIdx.x >> 6] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(sum_cnt, (ws[0][0] + ws[0][1]) + (ws[0][2] + ws[0][3]));
        atomicAdd(sum_cnt + 1, (ws[1][0] + ws[1][1]) + (ws[1][2] + ws[1][3]));
    }
}

// threshold = min(mean(grid[grid>0]), thr_max)  (models/networks.py:278-281)
__global__ void grid_threshold_kernel(const double* __restrict__ sum_cnt, float thr_max, float* __restrict__ thr) {
    // Python's min(nan, x) is nan (mean of an empty selection), and packbits
    // against a NaN threshold clears every bit -- reproduce that exactly.
    const float nan = __int_as_float(0x7fc00000);
    const float mean = sum_cnt[1] > 0 ? (float)(sum_cnt[0] / sum_cnt[1]) : nan;
    thr[0] = sum_cnt[1] > 0 ? fminf(mean, thr_max) : nan;
    thr[1] = mean;
}

// ---------------------------------------------------- active-sample map
// Exclusive scan of the per-row active counts (one 1024-lane workgroup) and
// the compacted index map sample_idx[j] = rays_a[row].start + k for the
// first n_active[row] samples of every row (one wave per row).
__global__ void __launch_bounds__(1024) active_scan_kernel(const int32_t* __restrict__ n_active, int64_t n_rows,
                                                           int64_t* __restrict__ act_start,
                                                           int64_t* __restrict__ total,
                                                           int64_t* __restrict__ total_acc = nullptr) {
    __shared__ int64_t wave_sums[16];
    __shared__ int64_t carry_s;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    constexpr int PER = 8;
    for (int64_t base = 0; base < n_rows; base += 1024 * PER) {
        int64_t v[PER], local = 0;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int64_t i = base + (int64_t)tid * PER + k;
            v[k] = i < n_rows ? n_active[i] : 0;
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
            if (lane < 16) wave_sums[lane] = ws;
        }
        __syncthreads();
        int64_t run = carry_s + (wid > 0 ? wave_sums[wid - 1] : 0) + incl - local;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int64_t i = base + (int64_t)tid * PER + k;
            if (i < n_rows) act_start[i] = run;
            run += v[k];
        }
        __syncthreads();
        if (tid == 1023) carry_s = run;
        __syncthreads();
    }
    if (tid == 0) {
        *total = carry_s;
        if (total_acc) atomicAdd((unsigned long long*)total_acc, (unsigned long long)carry_s);
    }
}

__global__ void __launch_bounds__(256) active_map_kernel(const int32_t* __restrict__ n_active,
                                                         const int64_t* __restrict__ rays_a,
                                                         const int64_t* __restrict__ act_start, int64_t n_rows,
                                                         int32_t* __restrict__ sample_idx, int first) {
    const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (r >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int na = n_active[r];
    const int64_t src = rays_a[3 * r + 1] + first, dst = act_start[r];
    for (int k = lane; k < na; k += 64) sample_idx[dst + k] = (int32_t)(src + k);
}

// Fused scan + map for batch-sized row counts (one launch instead of a
// one-block scan and a map launch, both latency-bound on the step's critical
// path).  Block b owns rows [b*SEG_ROWS, (b+1)*SEG_ROWS): it first sums the
// counts of every row before its range itself (a redundant reduction over
// L2-resident counts, so no block waits on another), then scans its own rows
// in LDS and writes their sample indices.  CAP > 0: counts[r] = min(N_r, CAP)
// read from rays_a (counts unused).  The last block publishes the total.
constexpr int SEG_ROWS = 64, SEG_THREADS = 512;
constexpr int64_t SEG_MAX_ROWS = 65536;  // beyond: scan + map launches (O(rows^2 / SEG_ROWS) reads here)

template <bool CAPPED>
__global__ void __launch_bounds__(SEG_THREADS) segments_kernel(const int32_t* __restrict__ counts,
                                                               const int64_t* __restrict__ rays_a, int64_t n_rows,
                                                               int cap, int first, int64_t* __restrict__ start_ws,
                                                               int64_t* __restrict__ total,
                                                               int64_t* __restrict__ total_acc,
                                                               int32_t* __restrict__ sample_idx) {
    __shared__ int64_t red[SEG_THREADS / 64];
    __shared__ int32_t lofs[SEG_ROWS + 1];
    __shared__ int64_t src[SEG_ROWS];
    NGP_PROBE_BEGIN(NGP_P_SEGMENTS);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * SEG_ROWS, r1 = min(r0 + SEG_ROWS, n_rows);
    auto count = [&](int64_t r) -> int64_t {
        return CAPPED ? min(rays_a[3 * r + 2], (int64_t)cap) : (int64_t)counts[r];
    };
    // 1) prefix of the rows before this block: 8 independent loads in flight
    // per thread (the L2 round trips overlap instead of chaining)
    int64_t acc = 0;
    int64_t r = t;
    for (; r + 7 * SEG_THREADS < r0; r += 8 * SEG_THREADS) {
        int64_t c[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = count(r + k * SEG_THREADS);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += c[k];
    }
    for (; r < r0; r += SEG_THREADS) acc += count(r);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) red[w] = acc;
    // 2) own rows: exclusive scan in wave 0 (SEG_ROWS = 64 = one wave)
    if (w == 0) {
        const int64_t r = r0 + lane;
        const int32_t c = r < r1 ? (int32_t)count(r) : 0;
        int32_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        lofs[lane] = x - c;
        if (lane == 63) lofs[SEG_ROWS] = x;
        src[lane] = r < r1 ? rays_a[3 * r + 1] + first : 0;
    }
    __syncthreads();
    int64_t prefix = 0;
#pragma unroll
    for (int i = 0; i < SEG_THREADS / 64; ++i) prefix += red[i];
    if (t < r1 - r0) start_ws[r0 + t] = prefix + lofs[t];
    const int32_t nb = lofs[SEG_ROWS];
    if (blockIdx.x == gridDim.x - 1 && t == 0) {
        *total = prefix + nb;
        if (total_acc) atomicAdd((unsigned long long*)total_acc, (unsigned long long)(prefix + nb));
    }
    // 3) map: entry q of this block belongs to the row whose [lofs, lofs+c) holds it
    for (int32_t q = t; q < nb; q += SEG_THREADS) {
        int lo = 0, hi = SEG_ROWS;  // lofs[lo] <= q < lofs[hi]
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int mid = (lo + hi) >> 1;
            if (lofs[mid] <= q) lo = mid; else hi = mid;
        }
        sample_idx[prefix + q] = (int32_t)(src[lo] + (q - lofs[lo]));
    }
    NGP_PROBE_END();
}

static void launch_segments(const int32_t* counts, const int64_t* rays_a, int64_t n_rows, int cap, int first,
                            int64_t* start_ws, int64_t* total, int64_t* total_acc, int32_t* sample_idx,
                            hipStream_t s) {
    const unsigned blocks = (unsigned)((n_rows + SEG_ROWS - 1) / SEG_ROWS);
    if (cap > 0)
        NGP_TIMED(NGP_K_SEGMENTS, s, segments_kernel<true><<<blocks, SEG_THREADS, 0, s>>>(nullptr, rays_a, n_rows, cap, first, start_ws, total,
                                                             total_acc, sample_idx));
    else
        NGP_TIMED(NGP_K_SEGMENTS, s, segments_kernel<false><<<blocks, SEG_THREADS, 0, s>>>(counts, rays_a, n_rows, 0, first, start_ws, total,
                                                              total_acc, sample_idx));
}

// ------------------------------------------- chunked forward (training)
// The training step only ever reads a row's samples up to its termination
// (composite_train_fw breaks there, the backward stops there), so the field
// is evaluated in two rounds: the first `first` samples of every row, then --
// only for rows still not terminated after them -- the rest.  Same outputs as
// evaluating every marched sample.
// Round-1 counts: min(N_r, first).
__global__ void __launch_bounds__(256) chunk_first_kernel(const int64_t* __restrict__ rays_a, int64_t n_rows, int first,
                                                          int32_t* __restrict__ counts) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    counts[r] = (int32_t)min(rays_a[3 * r + 2], (int64_t)first);
}

// Later-round counts: one wave per row computes the transmittance of its
// first min(N_r, first) samples exactly as composite_loss_ray's forward does
// (same expressions, chunk_transmittance); a row that has not terminated there
// and has more samples needs min(N_r, last) - first more (last <= 0: N_r).
__global__ void __launch_bounds__(256) chunk_rest_kernel(const float* __restrict__ sigmas,
                                                         const float* __restrict__ deltas,
                                                         const int64_t* __restrict__ rays_a, int64_t n_rows, int first,
                                                         int last, float T_thr, int32_t* __restrict__ counts) {
    const int64_t n = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (n >= n_rows) return;
    const int lane = threadIdx.x & 63;
    const int64_t start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
    const int64_t M = min(N, (int64_t)first);
    float T = 1.0f;
    bool done = false;
    for (int64_t k0 = 0; k0 < M && !done; k0 += 64) {
        const int cnt = (int)(M - k0 < 64 ? M - k0 : 64);
        float sg = 0.f, dl = 0.f;
        if (lane < cnt) { sg = sigmas[start + k0 + lane]; dl = deltas[start + k0 + lane]; }
        const float om = 1.0f - (1.0f - __expf(-sg * dl));
        const ChunkT ct = chunk_transmittance(om, cnt, T, T_thr, lane);
        done = ct.hit;
        T = __shfl(ct.Tn, ct.stop - 1, 64);
    }
    const int64_t end = last > 0 ? min(N, (int64_t)last) : N;
    if (lane == 0) counts[n] = (!done && N > first) ? (int32_t)(end - first) : 0;
}

// The non-empty rows of rays_a in row order (rows[0..*n_rows)) for
// field_first_chunk_kernel's one-wave-per-row round 1, and rest[r] = 0 for the
// empty ones (that kernel writes the others).  One 1024-thread block, 8 rows
// per thread per tile; runs on the march's side stream right after the
// compaction, off the step's critical path.
__global__ void __launch_bounds__(1024) rays_nonempty_kernel(const int64_t* __restrict__ rays_a, int64_t n_rays,
                                                             int32_t* __restrict__ rows, int64_t* __restrict__ n_out,
                                                             int32_t* __restrict__ rest, int64_t* __restrict__ zero) {
    __shared__ int32_t wave_sums[16];
    __shared__ int64_t carry_s;
    NGP_PROBE_BEGIN(NGP_P_NONEMPTY);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    constexpr int PER = 8;
    for (int64_t base = 0; base < n_rays; base += 1024 * PER) {
        uint32_t f = 0;  // bit k: row base + 8 tid + k is non-empty
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int64_t i = base + (int64_t)tid * PER + k;
            if (i < n_rays && rays_a[3 * i + 2] > 0) f |= 1u << k;
        }
        const int32_t local = __popc(f);
        int32_t incl = local;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wave_sums[wid] = incl;
        __syncthreads();
        if (wid == 0) {
            int32_t ws = lane < 16 ? wave_sums[lane] : 0;
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                const int32_t y = __shfl_up(ws, off, 64);
                if (lane >= off) ws += y;
            }
            if (lane < 16) wave_sums[lane] = ws;  // inclusive over waves
        }
        __syncthreads();
        const int64_t carry = carry_s;
        int64_t o = carry + (wid > 0 ? wave_sums[wid - 1] : 0) + incl - local;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int64_t i = base + (int64_t)tid * PER + k;
            if (i >= n_rays) break;
            if (f >> k & 1u) rows[o++] = (int32_t)i;
            else if (rest) rest[i] = 0;
        }
        __syncthreads();
        if (tid == 0) carry_s = carry + wave_sums[15];
        __syncthreads();
    }
    if (tid == 0) {
        *n_out = carry_s;
        if (zero) *zero = 0;
    }
    NGP_PROBE_END();
}

// Round-2 list in one launch: chunk_rest_kernel's counts + the exclusive scan
// across rows + the map of ray_segments.  Block b owns rows [64b, 64b + 64):
// its waves compute the counts of 8 rows each (first-chunk loads of all 8
// rows issued before any transmittance), wave 0 scans them, and the prefix
// over earlier blocks comes from a decoupled look-back: each block publishes
// its aggregate, then its inclusive prefix, as one 64-bit status word
// {generation, flag, value}; wave 0 reads the 64 predecessors before it at a
// time and stops at the closest inclusive one.  Block ids come from an atomic
// ticket (dispatch order), so a block only ever waits on blocks that started
// before it and publish their aggregate without waiting -- no deadlock at any
// grid size.  The last block to finish resets the ticket and advances the
// generation (stale status words of the previous launch never match).
// (64 rows per block: 32 / 16 measured slower, profiles/r03/ab/chunk_segments_rows.txt)
constexpr int CS_ROWS = 64, CS_THREADS = 512, CS_RPW = CS_ROWS / (CS_THREADS / 64);
constexpr int CS_LOG = CS_ROWS == 64 ? 6 : CS_ROWS == 32 ? 5 : 4;
static_assert(CS_ROWS == 64 || CS_ROWS == 32 || CS_ROWS == 16, "row block");

__global__ void __launch_bounds__(CS_THREADS) chunk_segments_kernel(
    const float* __restrict__ sigmas, const float* __restrict__ deltas, const int64_t* __restrict__ rays_a,
    int64_t n_rows, int first, int last, float T_thr, LookbackWs* __restrict__ lb, int64_t* __restrict__ start_ws,
    int64_t* __restrict__ total, int64_t* __restrict__ total_acc, const int64_t* __restrict__ total_acc_add,
    int32_t* __restrict__ sample_idx) {
    __shared__ int32_t cnt_s[CS_ROWS];
    __shared__ int32_t lofs[65];  // (wave 0 writes all 64 lanes' entries; [CS_ROWS] = the block's total)
    __shared__ int64_t src[64];
    __shared__ uint32_t sh_b;
    __shared__ int64_t sh_prefix;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t nb = gridDim.x;
    const uint32_t gen = __hip_atomic_load(&lb->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == 0) sh_b = __hip_atomic_fetch_add(&lb->tick, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint32_t b = sh_b;
    const int64_t r0 = (int64_t)b * CS_ROWS, r1 = min(r0 + CS_ROWS, n_rows);
    // ---- counts (chunk_rest_kernel's arithmetic)
    int64_t st[CS_RPW], Nr[CS_RPW];
    float sg0[CS_RPW], dl0[CS_RPW];
#pragma unroll
    for (int i = 0; i < CS_RPW; ++i) {
        const int64_t r = r0 + w * CS_RPW + i;
        st[i] = r < r1 ? rays_a[3 * r + 1] : 0;
        Nr[i] = r < r1 ? rays_a[3 * r + 2] : 0;
    }
#pragma unroll
    for (int i = 0; i < CS_RPW; ++i) {
        const int64_t M = min(Nr[i], (int64_t)first);
        sg0[i] = dl0[i] = 0.f;
        if (lane < M) { sg0[i] = sigmas[st[i] + lane]; dl0[i] = deltas[st[i] + lane]; }
    }
#pragma unroll
    for (int i = 0; i < CS_RPW; ++i) {
        const int64_t M = min(Nr[i], (int64_t)first);
        float T = 1.0f;
        bool done = false;
        for (int64_t k0 = 0; k0 < M && !done; k0 += 64) {
            const int cnt = (int)(M - k0 < 64 ? M - k0 : 64);
            float sg = sg0[i], dl = dl0[i];
            if (k0 > 0) {
                sg = dl = 0.f;
                if (lane < cnt) { sg = sigmas[st[i] + k0 + lane]; dl = deltas[st[i] + k0 + lane]; }
            }
            const float om = 1.0f - (1.0f - __expf(-sg * dl));
            const ChunkT ct = chunk_transmittance(om, cnt, T, T_thr, lane);
            done = ct.hit;
            T = __shfl(ct.Tn, ct.stop - 1, 64);
        }
        const int64_t end = last > 0 ? min(Nr[i], (int64_t)last) : Nr[i];
        if (lane == 0) cnt_s[w * CS_RPW + i] = (!done && Nr[i] > first) ? (int32_t)(end - first) : 0;
    }
    __syncthreads();
    if (w == 0) {
        // ---- own rows: exclusive scan
        const int64_t r = r0 + lane;
        const int32_t c = r < r1 ? cnt_s[lane % CS_ROWS] : 0;
        int32_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        lofs[lane] = x - c;
        const int32_t A = __shfl(x, 63, 64);
        if (lane == 63) lofs[CS_ROWS] = x;
        src[lane] = r < r1 ? rays_a[3 * r + 1] + first : 0;
        // ---- look-back
        const int64_t P = lookback_prefix(lb, b, gen, A, lane);
        if (lane == 0) {
            sh_prefix = P;
            if (b == nb - 1) {
                *total = P + A;
                if (total_acc)
                    atomicAdd((unsigned long long*)total_acc,
                              (unsigned long long)(P + A + (total_acc_add ? *total_acc_add : 0)));
            }
        }
    }
    __syncthreads();
    const int64_t prefix = sh_prefix;
    if (t < r1 - r0) start_ws[r0 + t] = prefix + lofs[t];
    const int32_t nbe = lofs[CS_ROWS];
    for (int32_t q = t; q < nbe; q += CS_THREADS) {
        int lo = 0, hi = CS_ROWS;  // lofs[lo] <= q < lofs[hi]
#pragma unroll
        for (int k = 0; k < CS_LOG; ++k) {
            const int mid = (lo + hi) >> 1;
            if (lofs[mid] <= q) lo = mid; else hi = mid;
        }
        sample_idx[prefix + q] = (int32_t)(src[lo] + (q - lofs[lo]));
    }
    if (t == 0) lookback_finish(lb, gen, nb);
}

}  // namespace ngp

using namespace ngp;

extern "C" {

int ngp_composite_loss(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                       const int64_t* rays_a, int64_t n_rays, const float* rgb_gt, const float* bg, int loss_type,
                       float lambda_opacity, float lambda_depth, float lambda_distortion, float depth_scale,
                       float T_threshold,
                       float* dL_dsigmas, float* dL_drgbs, float* out_rgb, float* out_opacity, float* out_depth,
                       float* out_loss, int32_t* n_active, int32_t* sample_idx, void* alloc_ws,
                       int64_t* n_active_total, int64_t* stats, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && loss_type >= 0 && loss_type <= 3 && depth_scale > 0);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(rays_a && rgb_gt && bg && out_rgb && out_opacity && out_depth && out_loss);
    NGP_CHECK_ARG(!sample_idx || (alloc_ws && n_active_total && ((uintptr_t)alloc_ws & 7) == 0));
    LossArgs la{loss_type, lambda_opacity, lambda_depth, depth_scale, 1.0f / (float)n_rays, T_threshold,
                lambda_distortion};
    // one row per wave: every row's dependent load chain in flight at once
    // (a few rows per wave serialised their memory latencies)
    const unsigned nb = (unsigned)std::min<int64_t>((n_rays + 3) / 4, 1 << 20);
    if (la.lambda_dist != 0.f)
        NGP_TIMED(NGP_K_COMPOSITE, as_stream(stream), composite_loss_wave_kernel<true><<<nb, 256, 0, as_stream(stream)>>>(
            sigmas, rgbs, deltas, ts, rays_a, n_rays, rgb_gt, bg, la, dL_dsigmas, dL_drgbs, out_rgb, out_opacity,
            out_depth, out_loss, n_active, sample_idx, (unsigned long long*)alloc_ws, n_active_total, stats));
    else
        NGP_TIMED(NGP_K_COMPOSITE, as_stream(stream), composite_loss_wave_kernel<false><<<nb, 256, 0, as_stream(stream)>>>(
            sigmas, rgbs, deltas, ts, rays_a, n_rays, rgb_gt, bg, la, dL_dsigmas, dL_drgbs, out_rgb, out_opacity,
            out_depth, out_loss, n_active, sample_idx, (unsigned long long*)alloc_ws, n_active_total, stats));
    return ngp_launch_status();
}

int ngp_chunk_counts(const int64_t* rays_a, int64_t n_rows, int first, const float* sigmas, const float* deltas,
                     float T_threshold, int32_t* counts, void* stream) {
    return ngp_chunk_counts_range(rays_a, n_rows, first, 0, sigmas, deltas, T_threshold, counts, stream);
}

int ngp_chunk_counts_range(const int64_t* rays_a, int64_t n_rows, int first, int last, const float* sigmas,
                           const float* deltas, float T_threshold, int32_t* counts, void* stream) {
    NGP_CHECK_ARG(n_rows >= 0 && first >= 1 && counts && rays_a && (last <= 0 || last > first));
    if (n_rows == 0) return NGP_OK;
    if (!sigmas) {
        NGP_TIMED(NGP_K_CHUNK, as_stream(stream), chunk_first_kernel<<<(unsigned)((n_rows + 255) / 256), 256, 0, as_stream(stream)>>>(rays_a, n_rows, first,
                                                                                           counts));
    } else {
        NGP_CHECK_ARG(deltas != nullptr);
        NGP_TIMED(NGP_K_CHUNK, as_stream(stream), chunk_rest_kernel<<<(unsigned)((n_rows + 3) / 4), 256, 0, as_stream(stream)>>>(sigmas, deltas, rays_a, n_rows,
                                                                                      first, last, T_threshold, counts));
    }
    return ngp_launch_status();
}

int ngp_rays_nonempty(const int64_t* rays_a, int64_t n_rays, int32_t* rows, int64_t* n_rows, int32_t* rest,
                      int64_t* zero, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && n_rays <= 0x7fffffff && n_rows);
    NGP_CHECK_ARG(n_rays == 0 || (rays_a && rows));
    NGP_TIMED(NGP_K_SEGMENTS, as_stream(stream), rays_nonempty_kernel<<<1, 1024, 0, as_stream(stream)>>>(rays_a, n_rays, rows, n_rows, rest, zero));
    return ngp_launch_status();
}

size_t ngp_chunk_segments_workspace(int64_t n_rows) {
    const int64_t blocks = n_rows > 0 ? (n_rows + CS_ROWS - 1) / CS_ROWS : 1;
    return 16 + 8 * (size_t)blocks;
}

int ngp_chunk_segments(const float* sigmas, const float* deltas, const int64_t* rays_a, int64_t n_rows, int first,
                       int last, float T_threshold, void* lookback_ws, int64_t* start_ws, int64_t* total,
                       int64_t* total_acc, const int64_t* total_acc_add, int32_t* sample_idx, void* stream) {
    NGP_CHECK_ARG(n_rows >= 0 && first >= 1 && (last <= 0 || last > first) && total);
    NGP_CHECK_ARG(!total_acc_add || total_acc);
    hipStream_t s = as_stream(stream);
    if (n_rows == 0) {
        active_scan_kernel<<<1, 1024, 0, s>>>(nullptr, 0, start_ws, total, total_acc);  // total = 0
        return ngp_launch_status();
    }
    NGP_CHECK_ARG(sigmas && deltas && rays_a && lookback_ws && start_ws && sample_idx &&
                  ((uintptr_t)lookback_ws & 7) == 0);
    const int64_t blocks = (n_rows + CS_ROWS - 1) / CS_ROWS;
    NGP_CHECK_ARG(blocks <= (int64_t)0x7fffffff);
    NGP_TIMED(NGP_K_SEGMENTS, s, chunk_segments_kernel<<<(unsigned)blocks, CS_THREADS, 0, s>>>(
        sigmas, deltas, rays_a, n_rows, first, last, T_threshold, (LookbackWs*)lookback_ws, start_ws, total,
        total_acc, total_acc_add, sample_idx));
    return ngp_launch_status();
}

int ngp_ray_segments(const int32_t* counts, const int64_t* rays_a, int64_t n_rows, int first, int64_t* start_ws,
                     int64_t* total, int64_t* total_acc, int32_t* sample_idx, void* stream) {
    NGP_CHECK_ARG(n_rows >= 0 && total && first >= 0);
    hipStream_t s = as_stream(stream);
    if (n_rows > 0) NGP_CHECK_ARG(counts && rays_a && start_ws && sample_idx);
    if (n_rows > 0 && n_rows <= SEG_MAX_ROWS) {
        launch_segments(counts, rays_a, n_rows, 0, first, start_ws, total, total_acc, sample_idx, s);
        return ngp_launch_status();
    }
    active_scan_kernel<<<1, 1024, 0, s>>>(counts, n_rows, start_ws, total, total_acc);
    if (n_rows > 0)
        active_map_kernel<<<(unsigned)((n_rows + 3) / 4), 256, 0, s>>>(counts, rays_a, start_ws, n_rows, sample_idx,
                                                                      first);
    return ngp_launch_status();
}

int ngp_ray_segments_capped(const int64_t* rays_a, int64_t n_rows, int cap, int64_t* start_ws, int64_t* total,
                            int64_t* total_acc, int32_t* sample_idx, void* stream) {
    NGP_CHECK_ARG(n_rows >= 0 && total && cap >= 1);
    hipStream_t s = as_stream(stream);
    if (n_rows == 0) {
        active_scan_kernel<<<1, 1024, 0, s>>>(nullptr, 0, start_ws, total, total_acc);  // total = 0
        return ngp_launch_status();
    }
    NGP_CHECK_ARG(rays_a && start_ws && sample_idx);
    if (n_rows <= SEG_MAX_ROWS) {
        launch_segments(nullptr, rays_a, n_rows, cap, 0, start_ws, total, total_acc, sample_idx, s);
        return ngp_launch_status();
    }
    return NGP_ERANGE;
}

int ngp_adam_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* params_f16, int64_t n,
                  float lr, float beta1, float beta2, float eps, int64_t step, float grad_scale, int zero_grad,
                  void* stream) {
    NGP_CHECK_ARG(n >= 0 && step >= 1);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && params_f16);
    if (n % 4 != 0) return NGP_ERANGE;
    const float bc1 = 1.0f - powf(beta1, (float)step), bc2 = 1.0f - powf(beta2, (float)step);
    const int64_t n4 = n / 4;
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    NGP_TIMED(NGP_K_ADAM, as_stream(stream), adam_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(params, grads, exp_avg, exp_avg_sq,
                                                                 (_Float16*)params_f16, n4, lr, beta1, beta2, eps, bc1,
                                                                 bc2, grad_scale, zero_grad, nullptr, nullptr));
    return ngp_launch_status();
}

int ngp_adam_step_dev(float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* params_f16, int64_t n,
                      const float* lr_dev, float beta1, float beta2, float eps, const int64_t* step_dev,
                      float grad_scale, int zero_grad, void* stream) {
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && params_f16 && lr_dev && step_dev);
    if (n % 4 != 0) return NGP_ERANGE;
    const int64_t n4 = n / 4;
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    NGP_TIMED(NGP_K_ADAM, as_stream(stream), adam_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(params, grads, exp_avg, exp_avg_sq,
                                                                 (_Float16*)params_f16, n4, 0.f, beta1, beta2, eps, 1.f,
                                                                 1.f, grad_scale, zero_grad, lr_dev, step_dev, nullptr, 0,
                                                                 0, 0));
    return ngp_launch_status();
}

int ngp_adam_step_dev_zero(float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* params_f16, int64_t n,
                           const float* lr_dev, float beta1, float beta2, float eps, const int64_t* step_dev,
                           float grad_scale, int zero_grad, float* zero, int64_t zero_n, void* stream) {
    NGP_CHECK_ARG(n >= 0 && zero_n >= 0 && zero_n % 4 == 0 && (zero_n == 0 || (zero && ((uintptr_t)zero & 15) == 0)));
    if (n == 0 && zero_n == 0) return NGP_OK;
    NGP_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && params_f16 && lr_dev && step_dev);
    if (n % 4 != 0) return NGP_ERANGE;
    const int64_t n4 = n / 4, z4 = zero_n / 4;
    int64_t blocks = (std::max(n4, z4) + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    NGP_TIMED(NGP_K_ADAM, as_stream(stream), adam_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(params, grads, exp_avg, exp_avg_sq,
                                                                 (_Float16*)params_f16, n4, 0.f, beta1, beta2, eps, 1.f,
                                                                 1.f, grad_scale, zero_grad, lr_dev, step_dev, nullptr, 0,
                                                                 0, 0, zero, z4));
    return ngp_launch_status();
}

int ngp_adam_step_dev_rep(float* params, float* grads, float* exp_avg, float* exp_avg_sq, void* params_f16, int64_t n,
                          const float* lr_dev, float beta1, float beta2, float eps, const int64_t* step_dev,
                          float grad_scale, int zero_grad, float* rep, int64_t rep_offset, int64_t rep_n, int n_rep,
                          void* stream) {
    if (!rep || rep_n == 0)
        return ngp_adam_step_dev(params, grads, exp_avg, exp_avg_sq, params_f16, n, lr_dev, beta1, beta2, eps,
                                 step_dev, grad_scale, zero_grad, stream);
    NGP_CHECK_ARG(n >= 0 && rep_offset >= 0 && rep_n > 0 && rep_offset % 4 == 0 && rep_n % 4 == 0 &&
                  rep_offset + rep_n <= n && n_rep >= 1 && n_rep <= 64 && ((uintptr_t)rep & 15) == 0);
    NGP_CHECK_ARG(params && grads && exp_avg && exp_avg_sq && params_f16 && lr_dev && step_dev);
    if (n % 4 != 0) return NGP_ERANGE;
    const int64_t n4 = n / 4;
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    NGP_TIMED(NGP_K_ADAM, as_stream(stream), adam_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(params, grads, exp_avg, exp_avg_sq,
                                                                 (_Float16*)params_f16, n4, 0.f, beta1, beta2, eps, 1.f,
                                                                 1.f, grad_scale, zero_grad, lr_dev, step_dev, rep,
                                                                 rep_offset / 4, rep_n / 4, n_rep));
    return ngp_launch_status();
}

// counters[i] += 1 for i < n (the per-step device counters a replayed graph
// advances at its end: Adam's step count, the batch RNG counter)
__global__ void counters_inc_kernel(int64_t* __restrict__ c, int n) {
    NGP_PROBE_BEGIN(NGP_P_COUNTERS);  // (the row of the step the increment closes: read before it)
    if ((int)threadIdx.x < n) c[threadIdx.x] += 1;
    NGP_PROBE_END();
}

int ngp_counters_inc(int64_t* counters, int n, void* stream) {
    NGP_CHECK_ARG(counters && n >= 1 && n <= 64);
    counters_inc_kernel<<<1, 64, 0, as_stream(stream)>>>(counters, n);
    return ngp_launch_status();
}

int ngp_density_scatter_last(const int64_t* indices, const float* sigmas, int64_t n, int64_t pos_base,
                             uint64_t* grid_key, void* stream) {
    NGP_CHECK_ARG(n >= 0 && pos_base >= 0 && pos_base + n < (1ll << 31));
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(indices && sigmas && grid_key && ((uintptr_t)grid_key & 7) == 0);
    scatter_last_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(
        indices, sigmas, n, pos_base, reinterpret_cast<unsigned long long*>(grid_key));
    return ngp_launch_status();
}

size_t ngp_occupied_cells_workspace(int64_t n_cells) {
    return n_cells > 0 ? (size_t)((n_cells + OCC_CHUNK - 1) / OCC_CHUNK) * sizeof(uint32_t) : 0;
}

int ngp_occupied_cells(const float* grid_cascade, int64_t n_cells, float threshold, int32_t* list, int64_t* count,
                       void* workspace, void* stream) {
    NGP_CHECK_ARG(n_cells > 0 && n_cells < (1ll << 31) && grid_cascade && list && count && workspace &&
                  ((uintptr_t)count & 7) == 0 && ((uintptr_t)workspace & 3) == 0);
    hipStream_t s = as_stream(stream);
    const unsigned nb = (unsigned)((n_cells + OCC_CHUNK - 1) / OCC_CHUNK);
    uint32_t* bc = reinterpret_cast<uint32_t*>(workspace);
    occ_count_kernel<<<nb, OCC_T, 0, s>>>(grid_cascade, n_cells, threshold, bc);
    occ_list_kernel<<<nb, OCC_T, 0, s>>>(grid_cascade, n_cells, threshold, bc, list, (unsigned long long*)count);
    return ngp_launch_status();
}

int ngp_occupancy_samples(uint64_t seed, const int64_t* counter_dev, int cascade, int grid_size, int64_t M,
                          float s_minus_hgs, float hgs, const int32_t* occ_list, const int64_t* occ_count, int64_t lo,
                          int64_t hi, float* xyzs, int64_t* flat_idx, void* stream) {
    NGP_CHECK_ARG(counter_dev && occ_list && occ_count && xyzs && flat_idx && grid_size >= 2 && M >= 0 && lo >= 0 &&
                  lo <= hi && hi <= 2 * M && cascade >= 0);
    if (hi == lo) return NGP_OK;
    occ_sample_kernel<<<(unsigned)((hi - lo + 255) / 256), 256, 0, as_stream(stream)>>>(
        seed, counter_dev, cascade, grid_size, M, s_minus_hgs, hgs, occ_list, (const unsigned long long*)occ_count, lo,
        hi, xyzs, flat_idx);
    return ngp_launch_status();
}

size_t ngp_occupancy_sorted_workspace(int64_t M) {
    const int64_t nb = (M + 1 + OSC_CH - 1) / OSC_CH;
    return (size_t)(2 * nb + 2) * sizeof(double);
}

int ngp_occupancy_samples_sorted(uint64_t seed, const int64_t* counter_dev, int cascade, int grid_size, int64_t M,
                                 float s_minus_hgs, float hgs, const int32_t* occ_list, const int64_t* occ_count,
                                 int64_t lo, int64_t hi, void* workspace, float* xyzs, int64_t* flat_idx,
                                 void* stream) {
    NGP_CHECK_ARG(counter_dev && occ_list && occ_count && xyzs && flat_idx && workspace && grid_size >= 2 &&
                  M >= 0 && lo >= 0 && lo <= hi && hi <= 2 * M && cascade >= 0 && ((uintptr_t)workspace & 7) == 0);
    if (hi == lo) return NGP_OK;
    NGP_CHECK_ARG((int64_t)grid_size * grid_size * grid_size <= (1ll << 31));
    hipStream_t s = as_stream(stream);
    const int64_t nb = (M + 1 + OSC_CH - 1) / OSC_CH;
    double* sums = reinterpret_cast<double*>(workspace);
    occ_exp_sums_kernel<<<(unsigned)(2 * nb), OSC_T, 0, s>>>(seed, counter_dev, cascade, M, nb, sums);
    occ_exp_scan_kernel<<<2, 1024, 0, s>>>(nb, sums);
    occ_sample_sorted_kernel<<<(unsigned)(2 * nb), OSC_T, 0, s>>>(seed, counter_dev, cascade, grid_size, M, nb,
                                                                 s_minus_hgs, hgs, occ_list,
                                                                 (const unsigned long long*)occ_count, sums, lo, hi,
                                                                 xyzs, flat_idx);
    return ngp_launch_status();
}

int ngp_occupancy_keep(const int64_t* flat_idx, int64_t M, int64_t cell_base, int64_t n_cells, int64_t lo, int64_t hi,
                       void* mark_ws, int32_t* list, int64_t* count, void* stream) {
    NGP_CHECK_ARG(M >= 0 && n_cells > 0 && cell_base >= 0 && lo >= 0 && lo <= hi && hi <= 2 * M &&
                  hi < (1ll << 31) && flat_idx && mark_ws && list && count && ((uintptr_t)count & 7) == 0);
    NGP_CHECK_ARG(((uintptr_t)mark_ws & 15) == 0);
    hipStream_t s = as_stream(stream);
    zero_words_kernel<<<1, 64, 0, s>>>((unsigned long long*)count, 1);  // (kernel nodes, not memsets: see above)
    if (hi == lo) return ngp_launch_status();
    const int64_t n16 = (n_cells + 15) / 16;
    zero_u4_kernel<<<(unsigned)((n16 + 255) / 256), 256, 0, s>>>((uint4*)mark_ws, n16);
    if (M > 0)
        occ_mark_kernel<<<(unsigned)((M + 255) / 256), 256, 0, s>>>(flat_idx, M, cell_base, n_cells, (uint8_t*)mark_ws);
    const int64_t per_blk = (int64_t)KEEP_T * KEEP_PER;
    occ_keep_kernel<<<(unsigned)((hi - lo + per_blk - 1) / per_blk), KEEP_T, 0, s>>>(
        flat_idx, M, cell_base, n_cells, (const uint8_t*)mark_ws, lo, hi, list, (unsigned long long*)count);
    return ngp_launch_status();
}

int ngp_density_scatter_kept(const int32_t* list, const int64_t* count, int64_t n_max, const int64_t* indices,
                             const float* sigmas, int64_t pos_base, uint64_t* grid_key, void* stream) {
    NGP_CHECK_ARG(n_max >= 0 && pos_base >= 0 && pos_base + n_max < (1ll << 31));
    if (n_max == 0) return NGP_OK;
    NGP_CHECK_ARG(list && count && indices && sigmas && grid_key && ((uintptr_t)grid_key & 7) == 0);
    static const unsigned cap = resident_blocks(scatter_kept_kernel, 256, 0);
    const unsigned blocks = std::max(1u, std::min(cap, (unsigned)((n_max + 255) / 256)));
    scatter_kept_kernel<<<blocks, 256, 0, as_stream(stream)>>>(list, count, n_max, indices, sigmas, pos_base,
                                                              reinterpret_cast<unsigned long long*>(grid_key));
    return ngp_launch_status();
}

int ngp_density_grid_ema(float* density_grid, uint64_t* grid_key, int64_t n, float decay, const float* decay_cells,
                         float thr_max, void* sum_cnt_ws, float* threshold_out, void* stream) {
    NGP_CHECK_ARG(n > 0 && density_grid && grid_key && sum_cnt_ws && threshold_out && ((uintptr_t)grid_key & 7) == 0);
    NGP_CHECK_ARG(((uintptr_t)sum_cnt_ws & 7) == 0);
    hipStream_t s = as_stream(stream);
    zero_words_kernel<<<1, 64, 0, s>>>(reinterpret_cast<unsigned long long*>(sum_cnt_ws), 2);
    int64_t blocks = (n + 255) / 256;
    if (blocks > 512) blocks = 512;
    grid_ema_kernel<<<(unsigned)blocks, 256, 0, s>>>(density_grid, reinterpret_cast<unsigned long long*>(grid_key), n,
                                                     decay, decay_cells,
                                                     (double*)sum_cnt_ws);
    grid_threshold_kernel<<<1, 1, 0, s>>>((const double*)sum_cnt_ws, thr_max, threshold_out);
    return ngp_launch_status();
}

}  // extern "C"

// NeRFLoss (losses.py:41-82) of the drop-in surface in one launch each way:
// the per-ray terms {rgb (3), opacity, depth} the reference builds from ~15
// elementwise torch ops, and their backward, one lane per ray, each op of the
// reference's expression rounded in fp32 in its order (x.detach() in the rgb
// denominator carries no gradient; division by the grid scale is torch's
// multiplication by its reciprocal; clip's gradient is 0 where it clips).
// loss_type 0 raw, 2 log, 3 tanh (the reference's set).
__device__ __forceinline__ float nerf_rgb_term(int type, float x, float y, float& dtdx) {
    if (type == 0) {
        const float den = x + 1e-3f;
        dtdx = 1.0f / den;  // (only used as grad / den below)
        return (x - y) / den;
    }
    if (type == 2) {
        const float a = 0.2935f + x;
        dtdx = a;
        return logf(a / (0.2935f + y)) * 0.7607f;
    }
    const float tx = tanhf(x);
    dtdx = tx;
    return tx - tanhf(y);
}

__global__ void __launch_bounds__(256) nerf_loss_fw_kernel(const float* __restrict__ rgb, const float* __restrict__ gt,
                                                           const float* __restrict__ opacity,
                                                           const float* __restrict__ depth, int64_t n, int type,
                                                           float lam_op, float neg_lam_depth, float inv_scale,
                                                           float* __restrict__ l_rgb, float* __restrict__ l_op,
                                                           float* __restrict__ l_dep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float dd;
        const float t = nerf_rgb_term(type, rgb[3 * i + c], gt[3 * i + c], dd);
        l_rgb[3 * i + c] = t * t;
    }
    const float o = opacity[i] + 1e-10f;
    l_op[i] = lam_op * (-o * logf(o));
    const float v = fminf(depth[i] * inv_scale + 1e-10f, 1.0f);
    l_dep[i] = neg_lam_depth * logf(v);
}

// (g_*: dL/d of each loss term; null = no gradient flows into that term)
__global__ void __launch_bounds__(256) nerf_loss_bw_kernel(const float* __restrict__ rgb, const float* __restrict__ gt,
                                                           const float* __restrict__ opacity,
                                                           const float* __restrict__ depth, int64_t n, int type,
                                                           float lam_op, float neg_lam_depth, float inv_scale,
                                                           const float* __restrict__ g_rgb,
                                                           const float* __restrict__ g_op,
                                                           const float* __restrict__ g_dep, float* __restrict__ d_rgb,
                                                           float* __restrict__ d_op, float* __restrict__ d_dep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float g = 0.f;
        if (g_rgb) {
            const float x = rgb[3 * i + c];
            float dd;
            const float t = nerf_rgb_term(type, x, gt[3 * i + c], dd);
            const float gt2 = g_rgb[3 * i + c] * (2.0f * t);  // PowBackward: grad * (2 t)
            if (type == 0) g = gt2 / (x + 1e-3f);              // DivBackward (the denominator detached)
            else if (type == 2) g = (gt2 * 0.7607f) / dd;       // MulBackward, LogBackward of (a / b): 1 / a
            else g = gt2 * (1.0f - dd * dd);                    // TanhBackward
        }
        d_rgb[3 * i + c] = g;
    }
    float go = 0.f;
    if (g_op) {
        const float o = opacity[i] + 1e-10f, lo = logf(o);
        const float gl = g_op[i] * lam_op;  // MulBackward of lam * f
        // f = (-o) * log(o): d/d(-o) = gl * log(o) -> d/do = -(gl * log(o)); d/dlog = gl * (-o) -> / o
        go = -(gl * lo) + (gl * (-o)) / o;
    }
    d_op[i] = go;
    float gd = 0.f;
    if (g_dep) {
        const float v = depth[i] * inv_scale + 1e-10f;
        if (v <= 1.0f) gd = ((g_dep[i] * neg_lam_depth) / fminf(v, 1.0f)) * inv_scale;
    }
    d_dep[i] = gd;
}

// The rows of (dL/dsigma, dL/drgb) with a nonzero entry: the samples that
// carry gradient (the compositing backward, volumerendering.cu:86-150, leaves
// every sample past its ray's termination at exact zero, and a zero upstream
// gradient adds exactly nothing to the parameters' gradient) -> idx[0..*count).
// A block takes 1024 consecutive rows (a wave 256 of them), counts them per wave,
// reserves its range with ONE atomic (a per-wave atomic on the one counter
// serialised ~9 K reservations: 57 us per launch) and writes the rows in
// order; blocks land in reservation order.
__global__ void __launch_bounds__(256) grad_rows_kernel(const float* __restrict__ dsig, const float* __restrict__ drgb,
                                                        int64_t n, int32_t* __restrict__ idx,
                                                        unsigned long long* __restrict__ count) {
    __shared__ uint32_t wcnt[4];
    __shared__ unsigned long long base_s;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t b0 = (int64_t)blockIdx.x * 1024; b0 < n; b0 += (int64_t)gridDim.x * 1024) {
        uint64_t m[4];
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // wave w takes rows b0 + 256 w .. + 255, 64 per step
            const int64_t i = b0 + 256 * w + 64 * q + lane;
            bool nz = false;
            if (i < n) nz = dsig[i] != 0.f || drgb[3 * i] != 0.f || drgb[3 * i + 1] != 0.f || drgb[3 * i + 2] != 0.f;
            m[q] = __ballot(nz);
            c += (uint32_t)__popcll(m[q]);
        }
        if (lane == 0) wcnt[w] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
            base_s = tot ? atomicAdd(count, (unsigned long long)tot) : 0ull;
        }
        __syncthreads();
        unsigned long long o = base_s;
        for (int v = 0; v < w; ++v) o += wcnt[v];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if ((m[q] >> lane) & 1ull)
                idx[o + __popcll(m[q] & ((1ull << lane) - 1ull))] = (int32_t)(b0 + 256 * w + 64 * q + lane);
            o += __popcll(m[q]);
        }
        __syncthreads();  // wcnt / base_s are rewritten next round
    }
}

extern "C" {

int ngp_nerf_loss_fw(const float* rgb, const float* rgb_gt, const float* opacity, const float* depth, int64_t n,
                     int loss_type, float lambda_opacity, float lambda_depth, float grid_scale, float* loss_rgb,
                     float* loss_opacity, float* loss_depth, void* stream) {
    NGP_CHECK_ARG(n >= 0 && (loss_type == 0 || loss_type == 2 || loss_type == 3) && grid_scale > 0.f);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(rgb && rgb_gt && opacity && depth && loss_rgb && loss_opacity && loss_depth);
    nerf_loss_fw_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(
        rgb, rgb_gt, opacity, depth, n, loss_type, lambda_opacity, -lambda_depth, 1.0f / grid_scale, loss_rgb,
        loss_opacity, loss_depth);
    return ngp_launch_status();
}

int ngp_nerf_loss_bw(const float* rgb, const float* rgb_gt, const float* opacity, const float* depth, int64_t n,
                     int loss_type, float lambda_opacity, float lambda_depth, float grid_scale, const float* g_rgb,
                     const float* g_opacity, const float* g_depth, float* d_rgb, float* d_opacity, float* d_depth,
                     void* stream) {
    NGP_CHECK_ARG(n >= 0 && (loss_type == 0 || loss_type == 2 || loss_type == 3) && grid_scale > 0.f);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(rgb && rgb_gt && opacity && depth && d_rgb && d_opacity && d_depth);
    nerf_loss_bw_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(
        rgb, rgb_gt, opacity, depth, n, loss_type, lambda_opacity, -lambda_depth, 1.0f / grid_scale, g_rgb,
        g_opacity, g_depth, d_rgb, d_opacity, d_depth);
    return ngp_launch_status();
}

int ngp_gradient_rows(const float* dL_dsigmas, const float* dL_drgbs, int64_t n, int32_t* idx, int64_t* count,
                      void* stream) {
    NGP_CHECK_ARG(n >= 0 && n < (1ll << 31) && count && ((uintptr_t)count & 7) == 0);
    hipStream_t s = as_stream(stream);
    zero_words_kernel<<<1, 64, 0, s>>>(reinterpret_cast<unsigned long long*>(count), 1);
    if (n > 0) {
        NGP_CHECK_ARG(dL_dsigmas && dL_drgbs && idx);
        const int64_t b = (n + 1023) / 1024;
        grad_rows_kernel<<<(unsigned)(b < 4096 ? b : 4096), 256, 0, s>>>(
            dL_dsigmas, dL_drgbs, n, idx, reinterpret_cast<unsigned long long*>(count));
    }
    return ngp_launch_status();
}

int ngp_active_samples(const int32_t* n_active, const int64_t* rays_a, int64_t n_rows, int64_t* act_start_ws,
                       int64_t* n_active_total, int32_t* sample_idx, void* stream) {
    NGP_CHECK_ARG(n_rows >= 0 && n_active_total);
    hipStream_t s = as_stream(stream);
    if (n_rows > 0) NGP_CHECK_ARG(n_active && rays_a && act_start_ws && sample_idx);
    if (n_rows > 0 && n_rows <= SEG_MAX_ROWS) {
        NGP_CHECK_ARG(n_active && rays_a && act_start_ws && sample_idx);
        launch_segments(n_active, rays_a, n_rows, 0, 0, act_start_ws, n_active_total, nullptr, sample_idx, s);
        return ngp_launch_status();
    }
    active_scan_kernel<<<1, 1024, 0, s>>>(n_active, n_rows, act_start_ws, n_active_total);
    if (n_rows > 0)
        active_map_kernel<<<(unsigned)((n_rows + 3) / 4), 256, 0, s>>>(n_active, rays_a, act_start_ws, n_rows,
                                                                      sample_idx, 0);
    return ngp_launch_status();
}

}  // extern "C"
