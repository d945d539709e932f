// Shared device helpers for the gfx950 kernels of libngp_amd.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ngp_amd.h"

#define NGP_SQRT3 1.73205080757f

#define NGP_CHECK_ARG(cond)        \
    do {                           \
        if (!(cond)) return NGP_EINVAL; \
    } while (0)

static inline int ngp_launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NGP_OK : (int)e;
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Kernel timing hook (ngp_timing_set, host.hip): HIP events around one launch.
void ngp_timing_mark(int id, int end, hipStream_t s);
#define NGP_TIMED(id, s, ...)          \
    do {                               \
        ngp_timing_mark((id), 0, (s)); \
        __VA_ARGS__;                   \
        ngp_timing_mark((id), 1, (s)); \
    } while (0)

// Device probes (ngp_probe_set, host.hip): lane 0 of every wave of a probed
// kernel stores its start and end time (GPU wall clock) into its own slot
// of the step row (*step % ring) -- plain stores, no atomics (atomics from
// every wave onto a few lines serialised and slowed the probed kernels 2-6x);
// the host takes the min start / max end: the kernel's execution span as a
// dispatch trace sees it, with no extra graph node and no change to the
// captured graphs (the control block is a device symbol read at run time:
// null = off).  Measurement plumbing only.
struct ProbeCtl {
    unsigned long long* buf;  // [ring][NGP_P_COUNT][NGP_PROBE_WAVES][2] (start, end)
    const int64_t* step;
    int64_t ring;
};
static __device__ ProbeCtl ngp_probe_ctl;
void ngp_probe_register(void (*set)(const ProbeCtl&));
static void ngp_probe_set_tu(const ProbeCtl& c) { (void)hipMemcpyToSymbol(HIP_SYMBOL(ngp_probe_ctl), &c, sizeof c); }
static const int ngp_probe_registered = (ngp_probe_register(ngp_probe_set_tu), 0);
__device__ __forceinline__ unsigned long long* ngp_probe_slot(int id) {
    const ProbeCtl c = ngp_probe_ctl;
    if (!c.buf) return nullptr;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    return c.buf + (((*c.step % c.ring) * NGP_P_COUNT + id) * NGP_PROBE_WAVES + (w & (NGP_PROBE_WAVES - 1))) * 2;
}
#define NGP_PROBE_BEGIN(id)                                          \
    unsigned long long* const ngp_probe_ = ngp_probe_slot(id);       \
    if (ngp_probe_ && (threadIdx.x & 63) == 0) ngp_probe_[0] = (unsigned long long)wall_clock64()
#define NGP_PROBE_END() \
    if (ngp_probe_ && (threadIdx.x & 63) == 0) ngp_probe_[1] = (unsigned long long)wall_clock64()

// Capacity guards (ngp_guard_hits, host.hip): every translation unit counts
// in its own device word and registers a reader/resetter at load time.  A
// kernel that clamps a device-side count to the capacity its caller gave it
// (so an overflow cannot write or read out of bounds) counts the clamp here:
// the result is then truncated, and ngp_guard_hits() > 0 says so.
static __device__ unsigned long long ngp_guard_tu;
void ngp_guard_register(unsigned long long (*get)(int reset));
static unsigned long long ngp_guard_get_tu(int reset) {
    unsigned long long v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(ngp_guard_tu), sizeof v) != hipSuccess) return ~0ull;
    if (reset) {
        const unsigned long long z = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(ngp_guard_tu), &z, sizeof z);
    }
    return v;
}
static const int ngp_guard_registered = (ngp_guard_register(ngp_guard_get_tu), 0);
__device__ __forceinline__ void ngp_guard_hit() { atomicAdd(&ngp_guard_tu, 1ull); }
// *n_dev (a device-side count) clamped to the capacity n; a clamp counts one
// guard hit (thread 0 of block 0 only: one per launch).  n_dev null: n.
__device__ __forceinline__ int64_t ngp_capped_count(const int64_t* n_dev, int64_t n) {
    if (!n_dev) return n;
    const int64_t v = *n_dev;
    if (v <= n) return v;
    if (blockIdx.x == 0 && threadIdx.x == 0) ngp_guard_hit();
    return n;
}

// Workgroups of `kernel` that fit on the whole device at once (occupancy x
// CUs): the grid of a persistent kernel, so per-block prologues (LDS weight
// images) are paid once per resident block, not once per tile.
template <typename K>
static unsigned resident_blocks(K kernel, int threads, size_t dyn_lds) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, dyn_lds) != hipSuccess || per_cu < 1)
        return 256;
    return (unsigned)(per_cu * cus);
}

namespace ngp {

// apex FusedAdam's per-element update (ADAM_MODE_0, no weight decay;
// train.py:146-152), shared by adam_kernel and the binned accumulation's fused
// Adam so the two paths are bit-identical.  g = gradient x grad_scale.
__device__ __forceinline__ void adam_bias(const float* lr_dev, const int64_t* step_dev, float b1, float b2,
                                          float& lr, float& bc1, float& bc2) {
    if (lr_dev) lr = *lr_dev;
    if (step_dev) {
        const float st = (float)(*step_dev + 1);
        bc1 = 1.0f - powf(b1, st);
        bc2 = 1.0f - powf(b2, st);
    }
}
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, float lr, float b1, float b2,
                                          float eps, float bc1, float bc2) {
    m = b1 * m + (1 - b1) * g;
    v = b2 * v + (1 - b2) * g * g;
    const float denom = sqrtf(v / bc2) + eps;
    p = p - lr * ((m / bc1) / denom);
}

// Adam state of one parameter range (same layout as the gradient it steps)
struct AdamArgs {
    float* p;
    float* m;
    float* v;
    _Float16* p16;
    const float* lr_dev;
    const int64_t* step_dev;
    float b1, b2, eps, grad_scale;
};

// helper_math.h:280-283 clamp(f,a,b) = fmaxf(a, fminf(f,b)) -- keeps the
// NaN behaviour of fminf/fmaxf that the marcher relies on.
__device__ __forceinline__ float clampf(float f, float a, float b) { return fmaxf(a, fminf(f, b)); }

// raymarching.cu:11-13
__device__ __forceinline__ float calc_dt(float t, float esf, int max_samples, int grid_size, float scale) {
    return clampf(t * esf, NGP_SQRT3 / max_samples, NGP_SQRT3 * 2 * scale / grid_size);
}

// raymarching.cu:19-23
__device__ __forceinline__ int mip_from_pos(float x, float y, float z, int cascades) {
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    int exponent;
    frexpf(mx, &exponent);
    return min(cascades - 1, max(0, exponent + 1));
}

// raymarching.cu:29-32
__device__ __forceinline__ int mip_from_dt(float dt, int grid_size, int cascades) {
    int exponent;
    frexpf(dt * grid_size, &exponent);
    return min(cascades - 1, max(0, exponent));
}

// raymarching.cu:35-50: 3-D Morton code, x in bit 0 (same magic-number
// spread as the reference so every int input maps identically).
__device__ __forceinline__ uint32_t spread3(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
__device__ __forceinline__ uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    return spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
}
// inverse of one axis (raymarching.cu:52-60)
__device__ __forceinline__ uint32_t compact3(uint32_t x) {
    x &= 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

// Counter-based Philox-4x32-10 (Salmon et al., SC'11): 4 independent
// uniform uint32 per (key, counter), no state to carry between steps.
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}
// uniform integer in [0, n) (multiply-shift; bias <= n / 2^32)
__device__ __forceinline__ int64_t uniform_index(uint32_t u, int64_t n) {
    return (int64_t)(((uint64_t)u * (uint64_t)n) >> 32);
}

}  // namespace ngp
