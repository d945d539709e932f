// Input gradient of NGP.density through the hash grid: dL/dx for
// L = sum_i g_i * sigma_i (models/rendering.py:300-313 render_surface_normal:
// torch.autograd.grad(sigmas, pts) through tcnn's grid encoding + density MLP
// + TruncExp, custom_functions.py:162-173).  One lane per point:
//   pass 1  enc = hash(x01) (fmaf over the 8 corners in tcnn's corner order,
//           rounded to fp16 -- the forward's storage point), density MLP in
//           fp32 on the fp16 weights (hidden rounded to fp16), h0 (fp16);
//   back    dL/dh0 = g * exp(clamp(h0, -15, 15)); dL/dhidden = dL/dh0 * W2[0] *
//           relu'(z); dL/denc = W1^T dL/dhidden (fp32);
//   pass 2  dL/dx01_d = sum_l scale_l * sum_c dw_c/dp_d * <dL/denc_l, table_c>,
//           dL/dx_d = dL/dx01_d / (xyz_max_d - xyz_min_d).
// tcnn's input-gradient arithmetic is not available here (parity unpinned:
// checked against an fp32 autograd restatement, tests/test_normal_gpu.py).
// Not a training-path kernel (AR insertion / normals): per-lane enc/genc
// arrays indexed by level live in scratch; kept simple.
#pragma clang fp contract(off)
#include "grid.h"

namespace ngp {

__global__ void __launch_bounds__(256) density_input_grad_kernel(const float* __restrict__ xyzs, int64_t n,
                                                                 GridArgs ga, const _Float16* __restrict__ table,
                                                                 const _Float16* __restrict__ mlp,
                                                                 const float* __restrict__ dL_dsigma,
                                                                 float* __restrict__ dL_dx) {
    __shared__ LevelLds lv;
    __shared__ float w1[64 * 32], w2[64];
    load_levels(ga, lv);
    for (int i = threadIdx.x; i < 64 * 32; i += blockDim.x) w1[i] = (float)mlp[i];
    if (threadIdx.x < 64) w2[threadIdx.x] = (float)mlp[2048 + threadIdx.x];  // W2 row 0 -> h0
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float in[3];
    load_x01(xyzs, i, true, ga, in);
    float enc[32];
#pragma unroll 1
    for (int l = 0; l < L; ++l) {
        float pos[3];
        uint32_t pg[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float p = fmaf(lv.scale[l], in[d], 0.5f);
            const float fl = floorf(p);
            pg[d] = (uint32_t)(int)fl;
            pos[d] = p - fl;
        }
        const bool dense = (lv.dense >> l) & 1u, pow2 = (lv.pow2 >> l) & 1u;
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float w = 1.0f;
#pragma unroll
            for (int d = 0; d < 3; ++d) w *= (c >> d) & 1 ? pos[d] : 1 - pos[d];
            const uint32_t e = lv.off[l] + corner_index(pg[0] + (c & 1), pg[1] + ((c >> 1) & 1),
                                                        pg[2] + ((c >> 2) & 1), lv.res[l], lv.size[l], dense, pow2);
            a0 = fmaf(w, (float)table[2 * (size_t)e], a0);
            a1 = fmaf(w, (float)table[2 * (size_t)e + 1], a1);
        }
        enc[2 * l] = (float)(_Float16)a0;
        enc[2 * l + 1] = (float)(_Float16)a1;
    }
    // density MLP forward (W1 64x32, ReLU, W2 row 0) and its backward to enc
    float gz[64];
    float h0 = 0.f;
#pragma unroll 4
    for (int j = 0; j < 64; ++j) {
        float z = 0.f;
#pragma unroll
        for (int k = 0; k < 32; ++k) z = fmaf(w1[j * 32 + k], enc[k], z);
        const float a = z > 0.f ? (float)(_Float16)z : 0.f;
        h0 = fmaf(w2[j], a, h0);
        gz[j] = z > 0.f ? w2[j] : 0.f;
    }
    h0 = (float)(_Float16)h0;
    const float g = (dL_dsigma ? dL_dsigma[i] : 1.0f) * expf(fminf(fmaxf(h0, -15.f), 15.f));
    float genc[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) genc[k] = 0.f;
#pragma unroll 4
    for (int j = 0; j < 64; ++j) {
        const float gj = g * gz[j];
#pragma unroll
        for (int k = 0; k < 32; ++k) genc[k] = fmaf(w1[j * 32 + k], gj, genc[k]);
    }
    // pass 2: through the trilinear weights
    float gx[3] = {0.f, 0.f, 0.f};
#pragma unroll 1
    for (int l = 0; l < L; ++l) {
        float pos[3];
        uint32_t pg[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float p = fmaf(lv.scale[l], in[d], 0.5f);
            const float fl = floorf(p);
            pg[d] = (uint32_t)(int)fl;
            pos[d] = p - fl;
        }
        const bool dense = (lv.dense >> l) & 1u, pow2 = (lv.pow2 >> l) & 1u;
        float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t e = lv.off[l] + corner_index(pg[0] + (c & 1), pg[1] + ((c >> 1) & 1),
                                                        pg[2] + ((c >> 2) & 1), lv.res[l], lv.size[l], dense, pow2);
            const float v = genc[2 * l] * (float)table[2 * (size_t)e] + genc[2 * l + 1] * (float)table[2 * (size_t)e + 1];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                float dw = (c >> d) & 1 ? 1.0f : -1.0f;  // d/dpos_d of the corner weight
#pragma unroll
                for (int d2 = 0; d2 < 3; ++d2)
                    if (d2 != d) dw *= (c >> d2) & 1 ? pos[d2] : 1 - pos[d2];
                acc[d] = fmaf(dw, v, acc[d]);
            }
        }
#pragma unroll
        for (int d = 0; d < 3; ++d) gx[d] = fmaf(lv.scale[l], acc[d], gx[d]);
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) dL_dx[3 * i + d] = gx[d] / (ga.g.xyz_max[d] - ga.g.xyz_min[d]);
}

}  // namespace ngp

using namespace ngp;

extern "C" int ngp_density_input_grad(const float* xyzs, int64_t n, const ngp_hashgrid_t* grid,
                                      const void* table_f16, const void* mlp_f16, const float* dL_dsigma,
                                      float* dL_dx, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && table_f16 && mlp_f16 && dL_dx);
    density_input_grad_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(
        xyzs, n, ga, (const _Float16*)table_f16, (const _Float16*)mlp_f16, dL_dsigma, dL_dx);
    return ngp_launch_status();
}
