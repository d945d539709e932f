// Random-gather microbenchmark (diagnostic): each lane issues K independent
// loads of W bytes at random W-aligned offsets of a T-byte table; sums them
// so the loads stay live.  Measures gathers/s vs W, T, waves per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int W, int K>
__global__ void __launch_bounds__(256) gather_kernel(const uint8_t* __restrict__ table, uint32_t n_slots, int iters,
                                                     uint32_t seed, float* __restrict__ out) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        uint32_t idx[K];
#pragma unroll
        for (int k = 0; k < K; ++k) idx[k] = hash32(tid * 7919u + (uint32_t)(it * K + k) * 104729u + seed) % n_slots;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if constexpr (W == 4) acc += __uint_as_float(*reinterpret_cast<const uint32_t*>(table + (size_t)idx[k] * 4) & 0x3fffffffu);
            if constexpr (W == 8) { const uint2 v = *reinterpret_cast<const uint2*>(table + (size_t)idx[k] * 8); acc += __uint_as_float((v.x ^ v.y) & 0x3fffffffu); }
            if constexpr (W == 16) { const uint4 v = *reinterpret_cast<const uint4*>(table + (size_t)idx[k] * 16); acc += __uint_as_float((v.x ^ v.y ^ v.z ^ v.w) & 0x3fffffffu); }
        }
    }
    if (acc == 1234.5f) out[tid] = acc;
}

extern "C" int diag_gather(const void* table, uint64_t table_bytes, int width, int blocks, int iters, uint32_t seed,
                           float* out, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const uint32_t n = (uint32_t)(table_bytes / width);
    if (width == 4) gather_kernel<4, 8><<<blocks, 256, 0, s>>>((const uint8_t*)table, n, iters, seed, out);
    else if (width == 8) gather_kernel<8, 8><<<blocks, 256, 0, s>>>((const uint8_t*)table, n, iters, seed, out);
    else gather_kernel<16, 8><<<blocks, 256, 0, s>>>((const uint8_t*)table, n, iters, seed, out);
    return (int)hipGetLastError();
}
