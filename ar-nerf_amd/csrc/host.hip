// Host-side helpers of libngp_amd.so.
#include <math.h>

#include "common.h"

extern "C" {

const char* ngp_version(void) { return "ngp_amd 0.1 gfx950"; }

// Level table of tcnn's Grid/Hash encoding as the reference configures it
// (models/networks.py:33-49): computed in fp32 the way tcnn does
// (scale_l = exp2f(l*log2f(b))*N_min - 1, res_l = ceilf(scale_l)+1,
// size_l = min(next_multiple(res_l^3, 8), 2^log2T)).  Host-side once, so the
// kernels and every caller use one table (no host/device exp2f mismatch).
uint32_t ngp_hashgrid_levels(int n_levels, int log2T, int base_resolution, float per_level_scale, float* scales,
                             uint32_t* res, uint32_t* offsets, uint32_t* sizes) {
    if (n_levels < 1 || n_levels > 32 || log2T < 1 || log2T > 30 || !scales || !res || !offsets || !sizes) return 0;
    const float l2 = log2f(per_level_scale);
    uint32_t off = 0;
    for (int l = 0; l < n_levels; ++l) {
        const float s = exp2f((float)l * l2) * (float)base_resolution - 1.0f;
        const uint32_t r = (uint32_t)ceilf(s) + 1u;
        const uint32_t max_params = 0xffffffffu / 2u;
        uint32_t p = (powf((float)r, 3.0f) > (float)max_params) ? max_params : r * r * r;
        p = (p + 7u) / 8u * 8u;
        const uint32_t T = 1u << log2T;
        if (p > T) p = T;
        scales[l] = s;
        res[l] = r;
        offsets[l] = off;
        sizes[l] = p;
        off += p;
    }
    offsets[n_levels] = off;
    return off;
}

}  // extern "C"
