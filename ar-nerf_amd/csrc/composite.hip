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

// volumerendering.cu:5-44 with one wave per ray: the lanes load a 64-sample
// chunk (coalesced) and compute each sample's alpha, then the ray's serial
// chain -- T, the left folds of rgb / depth / opacity, the break before the
// count -- runs in the reference's order on scalar copies of lane j's values:
// the same fp32 operations in the same order as the per-lane serial loop
// (bit-identical), with the memory latency paid once per chunk instead of per
// sample and 64x the waves in flight.
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
        float wl = 0.f;  // lane j's ws
        for (int j = 0; j < cnt; ++j) {
            const float aj = lane_f(a, j);
            const float w = aj * T;
            r += w * lane_f(cr, j); g += w * lane_f(cg, j); b += w * lane_f(cb, j);
            d += w * lane_f(tt, j);
            op += w;
            if (lane == j) wl = w;
            T *= 1.0f - aj;
            if (T <= T_thr) { done = true; samples = k0 + j; break; }
        }
        if (!done) samples = k0 + cnt;
        if (in) ws[s] = wl;  // (0 past the terminating sample)
    }
    if (lane == 0) {
        rgb[3 * ray] = r; rgb[3 * ray + 1] = g; rgb[3 * ray + 2] = b;
        depth[ray] = d;
        opacity[ray] = op;
        total_samples[ray] = samples;
    }
}

// volumerendering.cu:86-150, one wave per ray as composite_fw_kernel: the
// total of dL_dws * ws (the reference's inclusive scan's last value) as a
// serial left fold, then the serial pass in the reference's order, each
// sample's gradient put back into its lane and stored per chunk.
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
        float gs = 0.f, gw = 0.f;  // lane j's dL/dsigma and ws (0 past the termination)
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
            for (int j = 0; j < cnt; ++j) {
                const float aj = lane_f(a, j), crj = lane_f(cr, j), cgj = lane_f(cg, j), cbj = lane_f(cb, j);
                const float ttj = lane_f(tt, j);
                const float w = aj * T;
                r += w * crj; g += w * cgj; b += w * cbj;
                d += w * ttj;
                T *= 1.0f - aj;
                pre += lane_f(pk, j);
                const float gsj = lane_f(dl, j) * (gr * (crj * T - (R - r)) + gg * (cgj * T - (G - g)) +
                                                   gb * (cbj * T - (B - b)) + gop * (1 - O) +
                                                   gdep * (ttj * T - (D - d)) + T * lane_f(dw, j) - (S - pre));
                if (lane == j) { gs = gsj; gw = w; }
                if (T <= T_thr) { done = true; break; }
            }
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
