// Diagnostic build (NOT part of libngp_amd.so): the product's MLP backward
// (field_bwd_mlp_coop_kernel) with wall-clock stamps (100 MHz) at the phase
// boundaries of each block iteration, taken by lane 0 of wave 0 of every
// block: 0 loop top, 1 forward recomputed, 2 data chain done (dL/denc
// stored), 3 exponent barrier, 4 phase-1 tiles put, 5 phase-1 dW done,
// 6 phase-2 tiles put, 7 phase-2 dW done.  scripts/diag/mlpbwd_phases.py.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_bwd_stamps[1024 * 8 * 8];
#define NGP_BWD_PHASE(k)                                                                              \
    do {                                                                                              \
        if (threadIdx.x == 0) {                                                                       \
            const int64_t it_ = (bb - (int64_t)blockIdx.x * CW * 16) / stride;                        \
            if (blockIdx.x < 1024 && it_ < 8) g_bwd_stamps[(blockIdx.x * 8 + it_) * 8 + (k)] = wall_clock64(); \
        }                                                                                             \
    } while (0)
// kernel edges (lane 0 of wave 0): 0 entry, 1 weights staged, 2 loop done, 3 weight-gradient atomics issued
__device__ unsigned long long g_bwd_edges[1024 * 4];
#define NGP_BWD_EDGE(k)                                                                               \
    do {                                                                                              \
        if (threadIdx.x == 0 && blockIdx.x < 1024) g_bwd_edges[blockIdx.x * 4 + (k)] = wall_clock64(); \
    } while (0)
#include "../../ar-nerf_amd/csrc/field.hip"
#include "../../ar-nerf_amd/csrc/host.hip"

extern "C" int ngp_diag_bwd_stamps(unsigned long long* host, unsigned long long* edges, int clear) {
    const size_t bytes = sizeof(unsigned long long) * 1024 * 8 * 8, eb = sizeof(unsigned long long) * 1024 * 4;
    if (clear) {
        static unsigned long long zeros[1024 * 8 * 8];
        const int st = (int)hipMemcpyToSymbol(HIP_SYMBOL(g_bwd_stamps), zeros, bytes);
        return st ? st : (int)hipMemcpyToSymbol(HIP_SYMBOL(g_bwd_edges), zeros, eb);
    }
    const int st = (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bwd_stamps), bytes);
    return st ? st : (int)hipMemcpyFromSymbol(edges, HIP_SYMBOL(g_bwd_edges), eb);
}
