// Diagnostic build (NOT part of libngp_amd.so): the binned accumulation
// (hash_accum_kernel) with wall-clock stamps (100 MHz) per item, lane 0 of
// every block: 0 item start, 1 bucket found (search), 2 image zeroed (+ Adam
// state prefetch issued), 3 records summed, 4 Adam / flush done.
// scripts/diag/accum_phases.py.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_acc_stamps[1024 * 8 * 5];
#define NGP_ACC_PHASE(k)                                                                              \
    do {                                                                                              \
        if (threadIdx.x == 0 && blockIdx.x < 1024) {                                                  \
            const uint32_t j_ = (it - ws.items[b_lo] - blockIdx.x) / gridDim.x;                       \
            if (j_ < 8) g_acc_stamps[(blockIdx.x * 8 + j_) * 5 + (k)] = wall_clock64();                \
        }                                                                                             \
    } while (0)
#include "../../ar-nerf_amd/csrc/hashbin.hip"
#include "../../ar-nerf_amd/csrc/host.hip"

extern "C" int ngp_diag_acc_stamps(unsigned long long* host, int clear) {
    const size_t bytes = sizeof(unsigned long long) * 1024 * 8 * 5;
    if (clear) {
        static unsigned long long zeros[1024 * 8 * 5];
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_acc_stamps), zeros, bytes);
    }
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_acc_stamps), bytes);
}
