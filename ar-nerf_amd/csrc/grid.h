// Hash-grid level description shared by the field kernels (field.hip) and
// the binned hash-table backward (hashbin.hip): tcnn GridEncoding indexing.
#pragma once
#include "common.h"

namespace ngp {

constexpr int L = 16;  // levels (x2 features = the 32-wide MLP input)

struct GridArgs {
    ngp_hashgrid_t g;
    uint32_t dense_mask;  // bit l: level l indexes densely (res^3 <= size)
    uint32_t pow2_mask;   // bit l: size_l is a power of two
};

struct LevelLds {
    float scale[L];
    uint32_t res[L], off[L], size[L];
    uint32_t dense, pow2;
};

__device__ __forceinline__ void load_levels(const GridArgs& ga, LevelLds& lv) {
    const int t = threadIdx.x;
    if (t < L) {
        lv.scale[t] = ga.g.scales[t];
        lv.res[t] = ga.g.res[t];
        lv.off[t] = ga.g.offsets[t];
        lv.size[t] = ga.g.sizes[t];
    }
    if (t == 0) { lv.dense = ga.dense_mask; lv.pow2 = ga.pow2_mask; }
}

// tcnn grid_index for one corner (see oracle or_* restatement).
__device__ __forceinline__ uint32_t corner_index(uint32_t px, uint32_t py, uint32_t pz, uint32_t res, uint32_t size,
                                                 bool dense, bool pow2) {
    uint32_t idx = dense ? (px + py * res + pz * (res * res)) : ((px * 1u) ^ (py * 2654435761u) ^ (pz * 805459861u));
    // idx % size: hashed levels have a power-of-two size; a dense level's
    // corner index is below 2 * size (coordinates <= res, size >= res^3), so
    // one conditional subtract; a real division only for other tables.
    if (pow2) return idx & (size - 1u);
    if (idx >= size) {
        if (dense) idx -= size;
        // (coordinates outside [0, res] -- inputs outside the grid's box:
        // the full modulo keeps every index inside the table)
        if (__builtin_expect(idx >= size, 0)) idx %= size;
    }
    return idx;
}

__device__ __forceinline__ void load_x01(const float* __restrict__ xyzs, int64_t i, bool valid, const GridArgs& ga,
                                         float in[3]) {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float x = valid ? xyzs[3 * i + d] : 0.0f;
        // models/networks.py:104
        in[d] = (x - ga.g.xyz_min[d]) / (ga.g.xyz_max[d] - ga.g.xyz_min[d]);
    }
}

static int grid_args(const ngp_hashgrid_t* grid, GridArgs& ga) {
    if (!grid || grid->n_levels != L) return NGP_ERANGE;
    ga.g = *grid;
    ga.dense_mask = 0;
    ga.pow2_mask = 0;
    for (int l = 0; l < L; ++l) {
        const uint64_t r = grid->res[l];
        if (r * r * r <= (uint64_t)grid->sizes[l]) ga.dense_mask |= 1u << l;
        if ((grid->sizes[l] & (grid->sizes[l] - 1u)) == 0) ga.pow2_mask |= 1u << l;
        if (grid->sizes[l] == 0) return NGP_EINVAL;
    }
    return NGP_OK;
}

static unsigned persistent_blocks(int64_t n, int samples_per_block, unsigned cap) {
    int64_t b = (n + samples_per_block - 1) / samples_per_block;
    if (b < 1) b = 1;
    return (unsigned)(b < cap ? b : cap);
}

}  // namespace ngp
