// Transmittance of a row over one 64-sample chunk: shared by the compositing
// kernels (train.hip), the round-2 list (chunk_segments_kernel) and the
// per-row field forward (field.hip), so every evaluation rule sees exactly
// the composite's termination.
#pragma once
#include "common.h"

namespace ngp {

// Transmittance over one 64-sample chunk of a row, lane j < cnt holding
// om_j = 1 - a_j: T after sample j is T_in x (inclusive product of om, a
// fixed Hillis-Steele order -- the reference's serial product reassociated,
// like the wave sums), Tk the transmittance in front of sample j.  stop = 1 +
// the first j with T after it <= thr (where composite_train_fw breaks), else
// cnt.  chunk_rest_kernel, chunk_segments_kernel and field_rows_kernel call
// the same function, so the chunked field evaluation sees exactly the
// composite's termination.  A serial readlane
// walk here set the kernel time by the longest rows (hundreds of samples).
struct ChunkT {
    float Tk, Tn;
    int stop;
    bool hit;
};
__device__ __forceinline__ ChunkT chunk_transmittance(float om, int cnt, float T_in, float thr, int lane) {
    float p = lane < cnt ? om : 1.0f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const float y = __shfl_up(p, o, 64);
        if (lane >= o) p *= y;
    }
    float pe = __shfl_up(p, 1, 64);
    if (lane == 0) pe = 1.0f;
    ChunkT r;
    r.Tk = T_in * pe;
    r.Tn = T_in * p;
    const uint64_t h = __ballot(lane < cnt && r.Tn <= thr);
    r.hit = h != 0ull;
    r.stop = r.hit ? __ffsll((unsigned long long)h) : cnt;
    return r;
}

}  // namespace ngp
