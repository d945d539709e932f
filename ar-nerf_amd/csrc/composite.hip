// Volume-rendering compositing (forward, backward, test-time) for gfx950.
// Replaces models/csrc/volumerendering.cu of the reference.
//
// One wave per ray (training fw / bw: lanes load a chunk, the serial chain
// runs on scalar copies) or one lane per ray (test time), front-to-back,
// with the same early-termination rule (T <= T_threshold breaks BEFORE the count
// increments, volumerendering.cu:40-41).  Unlike the reference, the kernels
// write every output element themselves (zeros past termination), so the
// caller never needs a zero-fill, and the backward keeps the running prefix
// of dL_dws*ws in a register instead of a per-thread thrust scan
// (volumerendering.cu:118-121) -- same left-to-right fp32 sum.
#pragma clang fp contract(off)

#include "common.h"

namespace ngp {

// fp32 lane value j of a wave, in a scalar register
__device__ __forceinline__ float lane_f(float v, int j) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
}

// The reference's serial transmittance chain over one 64-sample chunk
// (T *= 1 - a, in order): lane j gets T before (Tb) and after (Ta) its
// sample.  Only the product is serial (one multiply per sample, no branch:
// the walk's break is found afterwards as the first lane whose T after its
// sample is <= thr -- the values up to there are exactly the serial loop's).
struct ChainT {
    float Tb, Ta, T;  // per lane; T: the chain's value after the chunk's last sample (uniform)
};
__device__ __forceinline__ ChainT serial_transmittance(float om, int cnt, float T, int lane) {
    ChainT c;
    c.Tb = c.Ta = 0.f;
    for (int j = 0; j < cnt; ++j) {
        const bool me = lane == j;
        if (me) c.Tb = T;
        T *= lane_f(om, j);
        if (me) c.Ta = T;
    }
    c.T = T;
    return c;
}

// volumerendering.cu:5-44 with one wave per ray: the lanes load a 64-sample
// chunk (coalesced) and compute each sample's alpha; the chunk's serial
// transmittance chain (serial_transmittance) gives every lane its T; each
// sample's weight w = a T and its products with rgb / t are formed per lane;
// then the ray's left folds of rgb / depth / opacity add them in order up to
// the terminating sample (independent chains, no branch per sample).  The
// same fp32 operations in the same order as the per-lane serial loop
// (bit-identical), the memory latency paid once per chunk, a wave per ray.
__global__ void __launch_bounds__(256) composite_fw_kernel(const float* __restrict__ sigmas,
                                                           const float* __restrict__ rgbs,
                                                           const float* __restrict__ deltas,
                                                           const float* __restrict__ ts,
                                                           const int64_t* __restrict__ rays_a, int64_t n_rays,
                                                           float T_thr, int64_t* __restrict__ total_samples,
                                                           float* __restrict__ opacity, float* __restrict__ depth,
                                                           float* __restrict__ rgb, float* __restrict__ ws) {
    const int lane = threadIdx.x & 63;
    const int64_t n = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (n >= n_rays) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
    float T = 1.0f, r = 0.f, g = 0.f, b = 0.f, d = 0.f, op = 0.f;
    int64_t samples = 0;
    bool done = false;
    for (int64_t k0 = 0; k0 < N; k0 += 64) {
        const int64_t s = start + k0 + lane;
        const int cnt = (int)(N - k0 < 64 ? N - k0 : 64);
        const bool in = lane < cnt;
        if (done) {  // past the termination: ws = 0 (the reference's tail loop)
            if (in) ws[s] = 0.f;
            continue;
        }
        float a = 0.f, cr = 0.f, cg = 0.f, cb = 0.f, tt = 0.f;
        if (in) {
            a = 1.0f - __expf(-sigmas[s] * deltas[s]);
            cr = rgbs[3 * s]; cg = rgbs[3 * s + 1]; cb = rgbs[3 * s + 2];
            tt = ts[s];
        }
        const ChainT ch = serial_transmittance(1.0f - a, cnt, T, lane);
        const uint64_t hit = __ballot(in && ch.Ta <= T_thr);
        const int last = hit ? __ffsll((unsigned long long)hit) - 1 : cnt - 1;  // the chunk's last composited sample
        const float w = a * ch.Tb;
        const float pr = w * cr, pg = w * cg, pb = w * cb, pd = w * tt;
        for (int j = 0; j <= last; ++j) {
            r += lane_f(pr, j); g += lane_f(pg, j); b += lane_f(pb, j);
            d += lane_f(pd, j);
            op += lane_f(w, j);
        }
        if (in) ws[s] = lane <= last ? w : 0.f;
        if (hit) {
            done = true;
            samples = k0 + last;  // (the break comes before the count)
        } else {
            samples = k0 + cnt;
            T = ch.T;
        }
    }
    if (lane == 0) {
        rgb[3 * ray] = r; rgb[3 * ray + 1] = g; rgb[3 * ray + 2] = b;
        depth[ray] = d;
        opacity[ray] = op;
        total_samples[ray] = samples;
    }
}

// volumerendering.cu:86-150, one wave per ray as composite_fw_kernel: the
// total S of dL_dws * ws (the reference's inclusive scan's last value) as a
// serial left fold; per chunk the serial transmittance chain, then the left
// folds of rgb / depth / dL_dws * ws, each fold's running value handed back
// to its sample's lane, and every sample's gradient formed in its lane from
// those (the reference's expression, operand for operand).
__global__ void __launch_bounds__(256) composite_bw_kernel(
    const float* __restrict__ dL_dop, const float* __restrict__ dL_ddep, const float* __restrict__ dL_drgb,
    const float* __restrict__ dL_dws, const float* __restrict__ sigmas, const float* __restrict__ rgbs,
    const float* __restrict__ ws, const float* __restrict__ deltas, const float* __restrict__ ts,
    const int64_t* __restrict__ rays_a, int64_t n_rays, const float* __restrict__ opacity,
    const float* __restrict__ depth, const float* __restrict__ rgb, float T_thr, float* __restrict__ dL_dsig,
    float* __restrict__ dL_drgbs) {
    const int lane = threadIdx.x & 63;
    const int64_t n = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (n >= n_rays) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
    if (N <= 0) return;
    float S = 0.f;
    for (int64_t k0 = 0; k0 < N; k0 += 64) {
        const int cnt = (int)(N - k0 < 64 ? N - k0 : 64);
        const float pk = lane < cnt ? dL_dws[start + k0 + lane] * ws[start + k0 + lane] : 0.f;
        for (int j = 0; j < cnt; ++j) S += lane_f(pk, j);
    }
    const float R = rgb[3 * ray], G = rgb[3 * ray + 1], B = rgb[3 * ray + 2];
    const float O = opacity[ray], D = depth[ray];
    const float gr = dL_drgb[3 * ray], gg = dL_drgb[3 * ray + 1], gb = dL_drgb[3 * ray + 2];
    const float gop = dL_dop[ray], gdep = dL_ddep[ray];
    float T = 1.0f, r = 0.f, g = 0.f, b = 0.f, d = 0.f, pre = 0.f;
    bool done = false;
    for (int64_t k0 = 0; k0 < N; k0 += 64) {
        const int64_t s = start + k0 + lane;
        const int cnt = (int)(N - k0 < 64 ? N - k0 : 64);
        const bool in = lane < cnt;
        float gs = 0.f, gw = 0.f;  // this lane's dL/dsigma and ws (0 past the termination)
        if (!done) {
            float a = 0.f, cr = 0.f, cg = 0.f, cb = 0.f, tt = 0.f, dl = 0.f, dw = 0.f, pk = 0.f;
            if (in) {
                dl = deltas[s];
                a = 1.0f - __expf(-sigmas[s] * dl);
                cr = rgbs[3 * s]; cg = rgbs[3 * s + 1]; cb = rgbs[3 * s + 2];
                tt = ts[s];
                dw = dL_dws[s];
                pk = dw * ws[s];
            }
            const ChainT ch = serial_transmittance(1.0f - a, cnt, T, lane);
            const uint64_t hit = __ballot(in && ch.Ta <= T_thr);
            const int last = hit ? __ffsll((unsigned long long)hit) - 1 : cnt - 1;
            const float w = a * ch.Tb;
            const float pr = w * cr, pg = w * cg, pb = w * cb, pd = w * tt;
            float rj = 0.f, gj = 0.f, bj = 0.f, dj = 0.f, prej = 0.f;  // the folds' values after this lane's sample
            for (int j = 0; j <= last; ++j) {
                r += lane_f(pr, j); g += lane_f(pg, j); b += lane_f(pb, j);
                d += lane_f(pd, j);
                pre += lane_f(pk, j);
                if (lane == j) { rj = r; gj = g; bj = b; dj = d; prej = pre; }
            }
            const float Ta = ch.Ta;
            if (lane <= last) {
                gs = dl * (gr * (cr * Ta - (R - rj)) + gg * (cg * Ta - (G - gj)) + gb * (cb * Ta - (B - bj)) +
                           gop * (1 - O) + gdep * (tt * Ta - (D - dj)) + Ta * dw - (S - prej));
                gw = w;
            }
            if (hit) done = true;
            else T = ch.T;
        }
        if (in) {
            dL_dsig[s] = gs;
            dL_drgbs[3 * s] = gr * gw; dL_drgbs[3 * s + 1] = gg * gw; dL_drgbs[3 * s + 2] = gb * gw;
        }
    }
}

__global__ void __launch_bounds__(64) composite_test_kernel(const float* __restrict__ sigmas,
                                                            const float* __restrict__ rgbs,
                                                            const float* __restrict__ deltas,
                                                            const float* __restrict__ ts, int64_t n_alive, int Ns,
                                                            int64_t* __restrict__ alive, float T_thr,
                                                            const int32_t* __restrict__ n_eff,
                                                            float* __restrict__ opacity, float* __restrict__ depth,
                                                            float* __restrict__ rgb) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_alive) return;
    const int ne = n_eff[n];
    if (ne == 0) { alive[n] = -1; return; }  // volumerendering.cu:221-224
    const int64_t r = alive[n];
    float op = opacity[r], d = depth[r], cr = rgb[3 * r], cg = rgb[3 * r + 1], cb = rgb[3 * r + 2];
    float T = 1 - op;
    for (int s = 0; s < ne; ++s) {
        const int64_t o = n * (int64_t)Ns + s;
        const float a = 1.0f - __expf(-sigmas[o] * deltas[o]);
        const float w = a * T;
        cr += w * rgbs[3 * o]; cg += w * rgbs[3 * o + 1]; cb += w * rgbs[3 * o + 2];
        d += w * ts[o];
        op += w;
        T *= 1.0f - a;
        if (T <= T_thr) { alive[n] = -1; break; }
    }
    rgb[3 * r] = cr; rgb[3 * r + 1] = cg; rgb[3 * r + 2] = cb;
    depth[r] = d;
    opacity[r] = op;
}

// Distortion loss (losses.cu:8-107, DVGO-v2 form): one lane per row.  The
// reference's per-thread thrust scans / reduce are sequential left folds, so
// the folds stay serial per ray for the reference's bits; rows are independent.
__global__ void __launch_bounds__(256) distortion_fw_kernel(const float* __restrict__ ws,
                                                            const float* __restrict__ deltas,
                                                            const float* __restrict__ ts,
                                                            const int64_t* __restrict__ rays_a, int64_t n_rays,
                                                            float* __restrict__ loss, float* __restrict__ ws_inc,
                                                            float* __restrict__ wts_inc) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_rays) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
    const float third = 1.0f / 3;
    float a = 0.f, b = 0.f, acc = 0.f;
    for (int64_t k = 0; k < N; ++k) {
        const int64_t s = start + k;
        const float w = ws[s];
        const float wts = w * ts[s];  // losses.cu:70
        const float ws_exc = a, wts_exc = b;
        a = a + w;
        b = b + wts;
        ws_inc[s] = a;
        wts_inc[s] = b;
        // losses.cu:92-93, one rounding per torch op
        acc = acc + (2 * (b * ws_exc - a * wts_exc) + ((third * w) * w) * deltas[s]);
    }
    loss[ray] = acc;
}

// losses.cu:110-140: every sample's gradient is independent given the scans,
// so one wave per row, lanes over its samples (coalesced).
__global__ void __launch_bounds__(256) distortion_bw_kernel(const float* __restrict__ dL_dloss,
                                                            const float* __restrict__ ws_inc,
                                                            const float* __restrict__ wts_inc,
                                                            const float* __restrict__ ws,
                                                            const float* __restrict__ deltas,
                                                            const float* __restrict__ ts,
                                                            const int64_t* __restrict__ rays_a, int64_t n_rays,
                                                            float* __restrict__ dL_dws) {
    const int64_t n = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (n >= n_rays) return;
    const int lane = threadIdx.x & 63;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
    if (N <= 0) return;
    const int64_t end = start + N - 1;
    const float ws_sum = ws_inc[end], wts_sum = wts_inc[end], g = dL_dloss[ray];
    for (int64_t s = start + lane; s <= end; s += 64) {
        const float t = ts[s];
        const float A = s == start ? 0.0f : t * ws_inc[s - 1] - wts_inc[s - 1];
        const float B = (wts_sum - wts_inc[s]) - t * (ws_sum - ws_inc[s]);
        dL_dws[s] = (g * 2) * (A + B) + (((g * 2.0f) / 3.0f) * ws[s]) * deltas[s];
    }
}

}  // namespace ngp

using namespace ngp;

static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

extern "C" {

int ngp_composite_train_fw(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                           const int64_t* rays_a, int64_t n_rays, float T_threshold, int64_t* total_samples,
                           float* opacity, float* depth, float* rgb, float* ws, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(rays_a && total_samples && opacity && depth && rgb);
    composite_fw_kernel<<<nblk(n_rays, 4), 256, 0, as_stream(stream)>>>(sigmas, rgbs, deltas, ts, rays_a, n_rays,
                                                                       T_threshold, total_samples, opacity, depth,
                                                                       rgb, ws);
    return ngp_launch_status();
}

int ngp_composite_train_bw(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drgb,
                           const float* dL_dws, const float* sigmas, const float* rgbs, const float* ws,
                           const float* deltas, const float* ts, const int64_t* rays_a, int64_t n_rays,
                           const float* opacity, const float* depth, const float* rgb, float T_threshold,
                           float* dL_dsigmas, float* dL_drgbs, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(dL_dopacity && dL_ddepth && dL_drgb && rays_a && opacity && depth && rgb);
    composite_bw_kernel<<<nblk(n_rays, 4), 256, 0, as_stream(stream)>>>(
        dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts, rays_a, n_rays, opacity, depth, rgb,
        T_threshold, dL_dsigmas, dL_drgbs);
    return ngp_launch_status();
}

int ngp_composite_test_fw(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                          int64_t n_alive, int N_samples, int64_t* alive, float T_threshold, const int32_t* n_eff,
                          float* opacity, float* depth, float* rgb, void* stream) {
    NGP_CHECK_ARG(n_alive >= 0 && N_samples >= 1);
    if (n_alive == 0) return NGP_OK;
    NGP_CHECK_ARG(sigmas && rgbs && deltas && ts && alive && n_eff && opacity && depth && rgb);
    composite_test_kernel<<<nblk(n_alive, 64), 64, 0, as_stream(stream)>>>(sigmas, rgbs, deltas, ts, n_alive,
                                                                          N_samples, alive, T_threshold, n_eff,
                                                                          opacity, depth, rgb);
    return ngp_launch_status();
}

int ngp_distortion_loss_fw(const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                           int64_t n_rays, float* loss, float* ws_inclusive_scan, float* wts_inclusive_scan,
                           void* stream) {
    NGP_CHECK_ARG(n_rays >= 0);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(ws && deltas && ts && rays_a && loss && ws_inclusive_scan && wts_inclusive_scan);
    distortion_fw_kernel<<<nblk(n_rays, 256), 256, 0, as_stream(stream)>>>(ws, deltas, ts, rays_a, n_rays, loss,
                                                                          ws_inclusive_scan, wts_inclusive_scan);
    return ngp_launch_status();
}

int ngp_distortion_loss_bw(const float* dL_dloss, const float* ws_inclusive_scan, const float* wts_inclusive_scan,
                           const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                           int64_t n_rays, float* dL_dws, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(dL_dloss && ws_inclusive_scan && wts_inclusive_scan && ws && deltas && ts && rays_a && dL_dws);
    distortion_bw_kernel<<<nblk(n_rays, 4), 256, 0, as_stream(stream)>>>(
        dL_dloss, ws_inclusive_scan, wts_inclusive_scan, ws, deltas, ts, rays_a, n_rays, dL_dws);
    return ngp_launch_status();
}

}  // extern "C"
