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

// Step completion ticket (ngp_step_ticket_set): the last kernels of a
// training step (the Adam launches, `parties` of them) advance the per-step
// device counters themselves once every block of every one of them has
// finished -- in place of a separate increment launch that would join their
// streams.  ws (caller-owned, zeroed once): [0..7] blocks arrived per party,
// [8] parties complete; the last arriver resets them.
struct StepTicket {
    uint32_t* ws;
    int64_t* counters;
    int n, parties, party;
};
// every thread of the block, after its last read of the counters
__device__ __forceinline__ void step_ticket_arrive(const StepTicket& t) {
    if (!t.ws) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (this wave's counter loads have returned)
    __syncthreads();                                  // every wave of the block is past its reads
    if (threadIdx.x == 0) {
        const uint32_t nb = gridDim.x * gridDim.y * gridDim.z;
        if (atomicAdd(&t.ws[t.party], 1u) == nb - 1) {  // this launch's last block
            atomicExch(&t.ws[t.party], 0u);
            if (atomicAdd(&t.ws[8], 1u) == (uint32_t)t.parties - 1) {  // the step's last launch
                atomicExch(&t.ws[8], 0u);
                for (int i = 0; i < t.n; ++i) atomicAdd((unsigned long long*)&t.counters[i], 1ull);
            }
        }
    }
}
// the ticket of the next participating launch (host side; none when unset)
StepTicket ngp_step_ticket_next();

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
