// Diagnostic build (NOT part of libngp_amd.so): the fused encode + MLP forward
// (field_encode_mlp_kernel) with wall-clock stamps (100 MHz) per wave, lane 0:
// 0 iteration start, 1 gathers done (encoding parked), 2 MLPs done -- first
// iteration of each wave.  scripts/diag/fem_phases.py.
#include <hip/hip_runtime.h>
__device__ unsigned long long g_fem[4096 * 16 * 3];
#define NGP_FEM_PHASE(k)                                                                                    \
    do {                                                                                                    \
        if (lane == 0 && base == (int64_t)blockIdx.x * blockDim.x + wv * 64 && blockIdx.x < 4096)           \
            g_fem[(blockIdx.x * FEM_WAVES + wv) * 3 + (k)] = wall_clock64();                                \
    } while (0)
#include "../../ar-nerf_amd/csrc/field.hip"
#include "../../ar-nerf_amd/csrc/host.hip"

extern "C" int ngp_diag_fem_stamps(unsigned long long* host, int clear) {
    const size_t bytes = sizeof(unsigned long long) * 4096 * 16 * 3;
    if (clear) {
        static unsigned long long zeros[4096 * 16 * 3];
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_fem), zeros, bytes);
    }
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fem), bytes);
}
