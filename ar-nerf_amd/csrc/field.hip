// Fused multires hash-grid encoding + tiny MLPs (density 32-64-16, colour
// 32-64-64-16) on gfx950 MFMA.  Replaces tiny-cuda-nn's
// NetworkWithInputEncoding / Encoding(SH4) / Network as the reference uses
// them (models/networks.py:37-78, 95-146).
//
// Work decomposition (one 64-lane wave = one 16-sample column block):
//   lane l -> sample s = l & 15 of the block, lane group g = l >> 4.
//   Lane (s, g) gathers hash levels 4g..4g+3 of sample s (32 independent
//   4-byte gathers of fp16x2 table entries), which lands the 8 encoding
//   values enc[s][8g..8g+7] directly in the B-operand layout of
//   v_mfma_f32_16x16x32_f16 (B[k = 8g + j][n = s]).  Every layer is computed
//   transposed, Y^T = W X^T (M = output units, N = samples), so each MFMA's
//   accumulator (rows 4g + r, column s) is re-packed in registers into the
//   next layer's B operand; the K order of that operand is permuted and the
//   weight columns are stored in LDS with the same permutation (P64/P32).
//   Weights (10240 fp16) live in LDS for the whole persistent wave loop.
// Numerics (tcnn storage points): fp16 params, fp32 interpolation weights
// and feature accumulation (fmaf over corners in tcnn order), fp16 encoding,
// fp32 MFMA accumulation, fp16 layer outputs, fp32 TruncExp / sigmoid.
#pragma clang fp contract(off)

#include <algorithm>

#include "common.h"
#include "grid.h"
#include "transmittance.h"

namespace ngp {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

// fp16 MLP buffer offsets (halfs), matrices row-major [out][in]
constexpr int OW1 = 0, OW2 = 2048, OW3 = 3072, OW4 = 5120, OW5 = 9216;
// LDS image of the forward weights (halfs): rows padded to 40 / 72 halfs
constexpr int R32 = 40, R64 = 72;
constexpr int SW1 = 0, SW2 = SW1 + 64 * R32, SW3 = SW2 + 16 * R64, SW4 = SW3 + 64 * R32, SW5 = SW4 + 64 * R64,
              SWF = SW5 + 16 * R64;

// K permutations matching the register re-pack of accumulator tiles:
// step q, lane group g, element j <- hidden unit 32q + (j<4 ? 4g+j : 16+4g+j-4)
__device__ __forceinline__ int P64(int kp) {
    const int q = kp >> 5, g = (kp >> 3) & 3, j = kp & 7;
    return 32 * q + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
}
// colour-net input c = [SH(16), h(16)]: element j <- j<4 ? SH[4g+j] : h[4g+j-4]
__device__ __forceinline__ int P32(int kp) {
    const int g = kp >> 3, j = kp & 7;
    return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
}

__device__ __forceinline__ f4 mfma32(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

struct __attribute__((aligned(4))) u2a4 {
    uint32_t x, y;
    __device__ operator uint2() const { return make_uint2(x, y); }
};

__device__ __forceinline__ uint32_t pick4(uint4 q, uint32_t k) {
    return k == 0 ? q.x : k == 1 ? q.y : k == 2 ? q.z : q.w;
}

// The two entries i0 (corner x) and i1 (corner x+1) of one y/z pair of a
// level's table tl.  Dense levels: always neighbours, one 8-byte load.
// Hashed levels (x term of the hash is px*1, size a power of two): i1 =
// i0 ^ (px ^ (px+1)), so both sit in one aligned 4-entry group unless px = 3
// mod 4 -- one 16-byte load for 3 of 4 pairs, plus a 4-byte load otherwise
// (the gather cost is per lane request, not per byte).
__device__ __forceinline__ void fetch_pair(const uint32_t* __restrict__ tl, uint32_t i0, uint32_t i1, bool dense,
                                           uint32_t& v0, uint32_t& v1) {
    const uint32_t lo = min(i0, i1), hi = max(i0, i1);
    uint32_t vlo, vhi;
    if (dense) {
        const bool adj = hi - lo == 1u;
        const uint2 pr = *reinterpret_cast<const u2a4*>(tl + (adj ? lo : (lo & ~1u)));
        vlo = adj ? pr.x : ((lo & 1u) ? pr.y : pr.x);
        vhi = pr.y;
        if (!adj) vhi = tl[hi];
    } else {
        const uint4 q = *reinterpret_cast<const uint4*>(tl + (lo & ~3u));
        const bool near = (hi ^ lo) < 4u;
        uint32_t vfar = 0u;
        if (!near) vfar = tl[hi];  // (the branch only issues the load: no wait inside it)
        vlo = pick4(q, lo & 3u);
        vhi = near ? pick4(q, hi & 3u) : vfar;
    }
    v0 = i0 < i1 ? vlo : vhi;
    v1 = i0 < i1 ? vhi : vlo;
}

// Hash-encode level l of one sample: the two features (fp32 accumulation,
// rounded once to fp16 by the caller).
__device__ __forceinline__ void encode_level(const float in[3], int l, const LevelLds& lv,
                                             const uint32_t* __restrict__ table, float& a0, float& a1) {
    const float sc = lv.scale[l];
    const uint32_t res = lv.res[l], size = lv.size[l], off = lv.off[l];
    const bool dense = (lv.dense >> l) & 1u, pow2 = (lv.pow2 >> l) & 1u;
    float pos[3];
    uint32_t pg[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float p = fmaf(sc, in[d], 0.5f);
        const float fl = floorf(p);
        pg[d] = (uint32_t)(int)fl;
        pos[d] = p - fl;
    }
    uint32_t v[8];
    float w[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float wt = 1.0f;
#pragma unroll
        for (int d = 0; d < 3; ++d) wt *= (c & (1 << d)) ? pos[d] : 1 - pos[d];
        w[c] = wt;
    }
    // x-adjacent corner pairs: one 8-byte load when the two entries are
    // neighbours (always on dense levels; on hashed levels when px is
    // even, the x term of the hash being px*1), else two 4-byte loads.
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const uint32_t qy = pg[1] + (yz & 1), qz = pg[2] + (yz >> 1);
        const uint32_t i0 = corner_index(pg[0], qy, qz, res, size, dense, pow2);
        const uint32_t i1 = corner_index(pg[0] + 1, qy, qz, res, size, dense, pow2);
        // (level sizes are multiples of 4 and offsets of 8 entries: the
        // aligned groups stay inside the level)
        fetch_pair(table + off, i0, i1, dense || !pow2, v[2 * yz], v[2 * yz + 1]);
    }
    a0 = 0.f;
    a1 = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const _Float16 f0 = __builtin_bit_cast(_Float16, (uint16_t)(v[c] & 0xffffu));
        const _Float16 f1 = __builtin_bit_cast(_Float16, (uint16_t)(v[c] >> 16));
        a0 = fmaf(w[c], (float)f0, a0);
        a1 = fmaf(w[c], (float)f1, a1);
    }
}

// Hash-encode levels 4g..4g+3 of one sample -> 8 fp16 values (enc[8g..8g+7]).
__device__ __forceinline__ h8 encode4(const float in[3], int g, const LevelLds& lv, const uint32_t* __restrict__ table) {
    h8 e;
#pragma unroll
    for (int jl = 0; jl < 4; ++jl) {
        float a0, a1;
        encode_level(in, 4 * g + jl, lv, table, a0, a1);
        e[2 * jl] = (_Float16)a0;
        e[2 * jl + 1] = (_Float16)a1;
    }
    return e;
}

// tcnn SphericalHarmonics degree 4 of (d/|d|+1)/2 (models/networks.py:144-145),
// returning the 4 values SH[4g..4g+3] this lane group needs.
__device__ __forceinline__ void sh4_select(float dx, float dy, float dz, int g, float out[4]) {
    const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
    const float x = ((dx / nrm + 1) / 2) * 2.f - 1.f;
    const float y = ((dy / nrm + 1) / 2) * 2.f - 1.f;
    const float z = ((dz / nrm + 1) / 2) * 2.f - 1.f;
    const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    float o[16];
    o[0] = 0.28209479177387814f;
    o[1] = -0.48860251190291987f * y;
    o[2] = 0.48860251190291987f * z;
    o[3] = -0.48860251190291987f * x;
    o[4] = 1.0925484305920792f * xy;
    o[5] = -1.0925484305920792f * yz;
    o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
    o[7] = -1.0925484305920792f * xz;
    o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
    o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
    o[10] = 2.8906114426405538f * xy * z;
    o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
    o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
    o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
    o[14] = 1.4453057213202769f * z * (x2 - y2);
    o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
#pragma unroll
    for (int r = 0; r < 4; ++r)
        out[r] = g == 0 ? o[r] : g == 1 ? o[4 + r] : g == 2 ? o[8 + r] : o[12 + r];
}

__device__ __forceinline__ h8 pack(h4 a, h4 b) { return h8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }
// ReLU of an fp32 accumulator tile, rounded to fp16: round first (v_cvt_pk),
// then clear every half whose sign is set (round(c) <= 0 exactly when c <= 0,
// so the result equals round(max(c, 0)) bit for bit, +0 included) -- two
// packed integer ops per pair instead of a canonicalize + max per element.
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t relu_bits(uint32_t x) {
    const uint32_t neg = __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, x) >> (s16x2){15, 15});
    return x & ~neg;
}
__device__ __forceinline__ h4 relu_h(f4 c) {
    const uint2 u = __builtin_bit_cast(uint2, h4{(_Float16)c[0], (_Float16)c[1], (_Float16)c[2], (_Float16)c[3]});
    uint32_t x = u.x, y = u.y;
    asm volatile("" : "+v"(x), "+v"(y));  // (opaque: one v_cvt_pk per pair, not re-derived per use)
    return __builtin_bit_cast(h4, make_uint2(relu_bits(x), relu_bits(y)));
}
__device__ __forceinline__ h4 to_h(f4 c) { return h4{(_Float16)c[0], (_Float16)c[1], (_Float16)c[2], (_Float16)c[3]}; }
__device__ __forceinline__ h8 lds8(const _Float16* p) { return *reinterpret_cast<const h8*>(p); }

// Stage the raw fp16 MLP buffer (row-major, 20 KB) into LDS with coalesced
// 16-byte loads; the permuted / transposed images are then built LDS->LDS
// (strided 2-byte global reads there were latency-bound: one wave per SIMD).
__device__ __forceinline__ void stage_raw_weights(const _Float16* __restrict__ mlp, _Float16* raw) {
    const h8* src = reinterpret_cast<const h8*>(mlp);
    h8* dst = reinterpret_cast<h8*>(raw);
    for (int i = threadIdx.x; i < NGP_MLP_PARAMS / 8; i += blockDim.x) dst[i] = src[i];
}

// Build the forward weight image (permuted columns, padded rows) in LDS from
// the staged raw buffer.
__device__ __forceinline__ void load_fwd_weights(const _Float16* __restrict__ mlp, _Float16* sw, bool color) {
    const int t = threadIdx.x, nt = blockDim.x;
    for (int i = t; i < 64 * 32; i += nt) sw[SW1 + (i >> 5) * R32 + (i & 31)] = mlp[OW1 + i];
    for (int i = t; i < 16 * 64; i += nt) sw[SW2 + (i >> 6) * R64 + (i & 63)] = mlp[OW2 + (i >> 6) * 64 + P64(i & 63)];
    if (!color) return;
    for (int i = t; i < 64 * 32; i += nt) sw[SW3 + (i >> 5) * R32 + (i & 31)] = mlp[OW3 + (i >> 5) * 32 + P32(i & 31)];
    for (int i = t; i < 64 * 64; i += nt) sw[SW4 + (i >> 6) * R64 + (i & 63)] = mlp[OW4 + (i >> 6) * 64 + P64(i & 63)];
    for (int i = t; i < 16 * 64; i += nt) sw[SW5 + (i >> 6) * R64 + (i & 63)] = mlp[OW5 + (i >> 6) * 64 + P64(i & 63)];
}

// Inverses of P64 / P32: weight column i -> its position in the permuted row.
__device__ __forceinline__ int P64inv(int i) {
    const int q = i >> 5, r = i & 31;
    return 32 * q + (r < 16 ? 8 * (r >> 2) + (r & 3) : 8 * ((r - 16) >> 2) + 4 + (r & 3));
}
__device__ __forceinline__ int P32inv(int i) { return i < 16 ? 8 * (i >> 2) + (i & 3) : 8 * ((i - 16) >> 2) + 4 + (i & 3); }

// The forward weight image built straight from global memory: coalesced
// 16-byte loads of the row-major buffer, each half scattered to its permuted
// LDS position (8 consecutive halfs share one row) -- no 20 KB raw staging
// buffer, so the MLP-only forward fits more blocks per CU.
// the 8 halfs v of the row-major buffer at flat index i0 (a multiple of 8) into
// the forward image: their row, each column at its permuted position
__device__ __forceinline__ void place_fwd8(int i0, h8 v, _Float16* sw) {
    int row, col0;  // destination row start, and the first column
    bool p64 = false, p32 = false;
    if (i0 < OW2) { row = SW1 + (i0 >> 5) * R32; col0 = i0 & 31; }
    else if (i0 < OW3) { row = SW2 + ((i0 - OW2) >> 6) * R64; col0 = (i0 - OW2) & 63; p64 = true; }
    else if (i0 < OW4) { row = SW3 + ((i0 - OW3) >> 5) * R32; col0 = (i0 - OW3) & 31; p32 = true; }
    else if (i0 < OW5) { row = SW4 + ((i0 - OW4) >> 6) * R64; col0 = (i0 - OW4) & 63; p64 = true; }
    else { row = SW5 + ((i0 - OW5) >> 6) * R64; col0 = (i0 - OW5) & 63; p64 = true; }
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        const int col = col0 + jj;
        sw[row + (p64 ? P64inv(col) : p32 ? P32inv(col) : col)] = v[jj];
    }
}

__device__ __forceinline__ void load_fwd_weights_direct(const _Float16* __restrict__ mlp, _Float16* sw, bool color) {
    const h8* src = reinterpret_cast<const h8*>(mlp);
    const int nv = (color ? NGP_MLP_PARAMS : OW3) / 8;
    for (int c = threadIdx.x; c < nv; c += blockDim.x) place_fwd8(8 * c, src[c], sw);
}

// Density net on one column block: returns h (rows 4g+r of sample s) and
// the four relu'd hidden tiles.
__device__ __forceinline__ h4 density_net(h8 e, const _Float16* sw, int s, int g, h4 h1[4]) {
    const f4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) h1[t] = relu_h(mfma32(lds8(sw + SW1 + (16 * t + s) * R32 + 8 * g), e, z));
    f4 c = z;
#pragma unroll
    for (int q = 0; q < 2; ++q) c = mfma32(lds8(sw + SW2 + s * R64 + 32 * q + 8 * g), pack(h1[2 * q], h1[2 * q + 1]), c);
    return to_h(c);
}

__device__ __forceinline__ h4 color_net(h8 cin, const _Float16* sw, int s, int g, h4 h3[4], h4 h4v[4]) {
    const f4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) h3[t] = relu_h(mfma32(lds8(sw + SW3 + (16 * t + s) * R32 + 8 * g), cin, z));
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        f4 c = z;
#pragma unroll
        for (int q = 0; q < 2; ++q)
            c = mfma32(lds8(sw + SW4 + (16 * t + s) * R64 + 32 * q + 8 * g), pack(h3[2 * q], h3[2 * q + 1]), c);
        h4v[t] = relu_h(c);
    }
    f4 c = z;
#pragma unroll
    for (int q = 0; q < 2; ++q) c = mfma32(lds8(sw + SW5 + s * R64 + 32 * q + 8 * g), pack(h4v[2 * q], h4v[2 * q + 1]), c);
    return to_h(c);
}

__device__ __forceinline__ float sigmoid_h(_Float16 o) {
    return (float)(_Float16)(1.0f / (1.0f + expf(-(float)o)));
}

// ENC_IN: the encoding comes from ngp_hash_encode (pair-major enc_in with
// row stride enc_stride) instead of being gathered here.
template <bool COLOR, bool ENC_IN = false>
__global__ void __launch_bounds__(256) field_fwd_kernel(const float* __restrict__ xyzs, const float* __restrict__ dirs,
                                                        int64_t n, const int64_t* __restrict__ n_dev, GridArgs ga,
                                                        const uint32_t* __restrict__ table,
                                                        const _Float16* __restrict__ mlp, float* __restrict__ sigmas,
                                                        float* __restrict__ rgbs, _Float16* __restrict__ enc_out,
                                                        _Float16* __restrict__ h_out,
                                                        const _Float16* __restrict__ enc_in = nullptr,
                                                        int64_t enc_stride = 0,
                                                        const int32_t* __restrict__ sidx = nullptr) {
    __shared__ __attribute__((aligned(16))) _Float16 sw[SWF];
    __shared__ LevelLds lv;
    load_fwd_weights_direct(mlp, sw, COLOR);
    if constexpr (!ENC_IN) load_levels(ga, lv);
    __syncthreads();
    const int64_t N = ngp_capped_count(n_dev, n);  // (a device count never past the capacity: a guard hit)
    const int lane = threadIdx.x & 63, s = lane & 15, g = lane >> 4;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16; base < N; base += nw * 16) {
        const int64_t j = base + s;  // row of the launch; sample i (sidx: only the listed samples)
        const bool valid = j < N;
        const int64_t i = valid && sidx ? (int64_t)sidx[j] : j;
        h8 e;
        if constexpr (ENC_IN) {
            const h4 z4 = {0, 0, 0, 0};
            const h4 ea = valid ? *reinterpret_cast<const h4*>(enc_in + ((2 * g) * enc_stride + i) * 4) : z4;
            const h4 eb = valid ? *reinterpret_cast<const h4*>(enc_in + ((2 * g + 1) * enc_stride + i) * 4) : z4;
            e = pack(ea, eb);
        } else {
            float in[3];
            load_x01(xyzs, i, valid, ga, in);
            e = encode4(in, g, lv, table);
        }
        h4 h1[4];
        const h4 hh = density_net(e, sw, s, g, h1);
        if (valid) {
            if (enc_out) *reinterpret_cast<h8*>(enc_out + i * 32 + 8 * g) = e;
            if (h_out) *reinterpret_cast<h4*>(h_out + i * 16 + 4 * g) = hh;
            if (g == 0) sigmas[i] = expf((float)hh[0]);  // TruncExp forward (custom_functions.py:165-167)
        }
        if constexpr (COLOR) {
            const float dx = valid ? dirs[3 * i] : 0.f, dy = valid ? dirs[3 * i + 1] : 0.f,
                        dz = valid ? dirs[3 * i + 2] : 1.f;
            float sh[4];
            sh4_select(dx, dy, dz, g, sh);
            const h8 cin = {(_Float16)sh[0], (_Float16)sh[1], (_Float16)sh[2], (_Float16)sh[3], hh[0], hh[1], hh[2], hh[3]};
            h4 h3[4], h4v[4];
            const h4 o = color_net(cin, sw, s, g, h3, h4v);
            if (valid && g == 0) {
                rgbs[3 * i] = sigmoid_h(o[0]);
                rgbs[3 * i + 1] = sigmoid_h(o[1]);
                rgbs[3 * i + 2] = sigmoid_h(o[2]);
            }
        }
    }
}

// ------------------------------------------------------ hash encode alone
// One level's parameters as wave-uniform (scalar) values, so the per-level
// index variant is chosen by scalar branches, not computed for every lane.
struct LevelU {
    float sc;
    uint32_t res, res2, size, off;
    bool dense, pow2;
};
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ LevelU level_u(const LevelLds& lv, int l) {
    LevelU u;
    u.sc = __uint_as_float(rfl(__float_as_uint(lv.scale[l])));
    u.res = rfl(lv.res[l]);
    u.res2 = u.res * u.res;
    u.size = rfl(lv.size[l]);
    u.off = rfl(lv.off[l]);
    u.dense = (rfl(lv.dense) >> l) & 1u;
    u.pow2 = (rfl(lv.pow2) >> l) & 1u;
    return u;
}

// encode_level with the same values (tcnn grid_index, fmaf corner order), but
// the index reduction specialised per level: hashed levels have a power-of-two
// size (mask); on dense levels the corner index is below 2 * size (corner
// coordinates <= res, size >= res^3), so `% size` is one conditional
// subtract; the generic modulo remains for any other table.
__device__ __forceinline__ uint32_t reduce_idx(uint32_t idx, const LevelU& u) {
    if (u.pow2) return idx & (u.size - 1u);
    if (u.dense) {
        // below 2 * size for coordinates in [0, res]; inputs outside the grid's box
        // (coordinates past it) take the full modulo, as tcnn's grid_index does
        idx = idx >= u.size ? idx - u.size : idx;
        return __builtin_expect(idx >= u.size, 0) ? idx % u.size : idx;
    }
    return idx % u.size;
}

// encode_level_u in two halves, so a caller can issue the gathers of several
// levels before it consumes any: corner weights + the level's loads, then the
// fp32 corner sum (the same fmaf order)
__device__ __forceinline__ void gather_level_u(const float in[3], const LevelU& u, const uint32_t* __restrict__ table,
                                               float w[8], uint32_t v[8]) {
    float pos[3];
    uint32_t pg[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float p = fmaf(u.sc, in[d], 0.5f);
        const float fl = floorf(p);
        pg[d] = (uint32_t)(int)fl;
        pos[d] = p - fl;
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float wt = 1.0f;
#pragma unroll
        for (int d = 0; d < 3; ++d) wt *= (c & (1 << d)) ? pos[d] : 1 - pos[d];
        w[c] = wt;
    }
    uint32_t i0[4], i1[4];
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const uint32_t qy = pg[1] + (yz & 1), qz = pg[2] + (yz >> 1);
        uint32_t r0, r1;
        if (u.dense) {
            r0 = pg[0] + qy * u.res + qz * u.res2;
            r1 = r0 + 1u;
        } else {
            const uint32_t h = (qy * 2654435761u) ^ (qz * 805459861u);
            r0 = (pg[0] * 1u) ^ h;
            r1 = ((pg[0] + 1u) * 1u) ^ h;
        }
        i0[yz] = reduce_idx(r0, u);
        i1[yz] = reduce_idx(r1, u);
    }
    const uint32_t* tl = table + u.off;
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) fetch_pair(tl, i0[yz], i1[yz], u.dense || !u.pow2, v[2 * yz], v[2 * yz + 1]);
}

__device__ __forceinline__ void sum_level(const float w[8], const uint32_t v[8], float& a0, float& a1) {
    a0 = 0.f;
    a1 = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const _Float16 f0 = __builtin_bit_cast(_Float16, (uint16_t)(v[c] & 0xffffu));
        const _Float16 f1 = __builtin_bit_cast(_Float16, (uint16_t)(v[c] >> 16));
        a0 = fmaf(w[c], (float)f0, a0);
        a1 = fmaf(w[c], (float)f1, a1);
    }
}

// gather_level_u in two halves that keep fewer registers live across the
// loads' latency: the loads alone (indices from the cell corner), then -- once
// they have returned -- the corner weights recomputed from the position and
// the fp32 corner sum (the same values, the same fmaf order)
__device__ __forceinline__ void level_cell(const float in[3], const LevelU& u, uint32_t pg[3], float pos[3]) {
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float p = fmaf(u.sc, in[d], 0.5f);
        const float fl = floorf(p);
        pg[d] = (uint32_t)(int)fl;
        pos[d] = p - fl;
    }
}
__device__ __forceinline__ void gather_level_loads(const float in[3], const LevelU& u,
                                                   const uint32_t* __restrict__ table, uint32_t v[8]) {
    float pos[3];
    uint32_t pg[3];
    level_cell(in, u, pg, pos);
    uint32_t i0[4], i1[4];
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const uint32_t qy = pg[1] + (yz & 1), qz = pg[2] + (yz >> 1);
        uint32_t r0, r1;
        if (u.dense) {
            r0 = pg[0] + qy * u.res + qz * u.res2;
            r1 = r0 + 1u;
        } else {
            const uint32_t h = (qy * 2654435761u) ^ (qz * 805459861u);
            r0 = (pg[0] * 1u) ^ h;
            r1 = ((pg[0] + 1u) * 1u) ^ h;
        }
        i0[yz] = reduce_idx(r0, u);
        i1[yz] = reduce_idx(r1, u);
    }
    const uint32_t* tl = table + u.off;
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) fetch_pair(tl, i0[yz], i1[yz], u.dense || !u.pow2, v[2 * yz], v[2 * yz + 1]);
}
__device__ __forceinline__ uint32_t level_sum_h2(const float in[3], const LevelU& u, const uint32_t v[8]) {
    float pos[3];
    uint32_t pg[3];
    level_cell(in, u, pg, pos);
    float w[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float wt = 1.0f;
#pragma unroll
        for (int d = 0; d < 3; ++d) wt *= (c & (1 << d)) ? pos[d] : 1 - pos[d];
        w[c] = wt;
    }
    float a0, a1;
    sum_level(w, v, a0, a1);
    return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a0) | ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a1) << 16);
}

__device__ __forceinline__ void encode_level_u(const float in[3], const LevelU& u, const uint32_t* __restrict__ table,
                                               float& a0, float& a1) {
    float w[8];
    uint32_t v[8];
    gather_level_u(in, u, table, w, v);
    sum_level(w, v, a0, a1);
}

// Multires hash encoding alone (the gathers of field_fwd_kernel, same
// arithmetic, bit-identical values), written pair-major:
//   enc_pm[p][i][0..3] = enc[i][4p .. 4p+3]  (levels 2p, 2p+1; p = 0..7).
// Each lane encodes every level of one sample, so a wave instruction gathers
// ONE level for 64 consecutive samples (a ray's neighbours: shared lines on
// the coarse levels) -- 1.55x the rate of one level pair per XCD and 1.8x
// field_fwd_kernel's lane (sample, level group) layout
// (scripts/diag/encode_split.py).  sidx (nullable): rows j < N encode sample
// sidx[j] (rows of enc_pm are samples).
__global__ void __launch_bounds__(256) hash_encode_kernel(const float* __restrict__ xyzs, int64_t n,
                                                          const int64_t* __restrict__ n_dev,
                                                          const int32_t* __restrict__ sidx, GridArgs ga,
                                                          const uint32_t* __restrict__ table,
                                                          _Float16* __restrict__ enc_pm) {
    __shared__ LevelLds lv;
    load_levels(ga, lv);
    __syncthreads();
    const int64_t N = ngp_capped_count(n_dev, n);  // (a device count never past the capacity: a guard hit)
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < N; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = sidx ? (int64_t)sidx[j] : j;
        float in[3];
        load_x01(xyzs, i, true, ga, in);
#pragma unroll 1
        for (int pr = 0; pr < 8; ++pr) {
            float w[2][8];
            uint32_t v[2][8];
            gather_level_u(in, level_u(lv, 2 * pr), table, w[0], v[0]);
            gather_level_u(in, level_u(lv, 2 * pr + 1), table, w[1], v[1]);
            float a0, a1, b0, b1;
            sum_level(w[0], v[0], a0, a1);
            sum_level(w[1], v[1], b0, b1);
            *reinterpret_cast<h4*>(enc_pm + ((int64_t)pr * n + i) * 4) =
                h4{(_Float16)a0, (_Float16)a1, (_Float16)b0, (_Float16)b1};
        }
    }
}

// ------------------------------ fused encode + MLP forward, register form
// field_encode_mlp_kernel's arithmetic (bit-identical outputs) with two
// changes in the structure:
//  * the encoding never goes through LDS: a lane keeps its sample's 16 level
//    dwords (fp16x2 features) in registers, and a 4 x 4 transpose of 4-dword
//    groups across the wave's four 16-lane rows (two v_permlane32_swap and
//    two v_permlane16_swap stages) lands, for column block c, the operand
//    enc[16c + s][8g .. 8g+7] in lane (s, g) -- the B layout of
//    v_mfma_f32_16x16x32_f16; a block then needs only the 24 KB weight image,
//    so occupancy is set by registers, not by the 40 KB of parked rows;
//  * LPR levels are gathered per round (their loads issued together), so a
//    lane's chain of dependent gather rounds is 16 / LPR long instead of 8;
//  * 64-sample chunks are dealt to waves interleaved over the whole grid
//    (chunk k -> wave k / G of block k % G): every resident block gets the
//    same number of chunks within one, so no CU holds two blocks' worth of
//    work while others hold one (the one-pass ceil(N/512)-block form left
//    ~20 % of the CUs doubly loaded).
// 4 x 4 transpose of 4-dword groups across the wave's 16-lane rows: on entry
// register group r (E[4r..4r+3]) of lane row q holds group r of the row's
// sample; on exit group c of lane row g holds group g of row c's sample.
__device__ __forceinline__ void transpose_rows4(uint32_t E[16]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // stage 1: upper 32 lanes of groups 0 / 1 <-> lower 32 lanes of groups 2 / 3
        const auto a = __builtin_amdgcn_permlane32_swap(E[k], E[8 + k], false, false);
        E[k] = a[0];
        E[8 + k] = a[1];
        const auto b = __builtin_amdgcn_permlane32_swap(E[4 + k], E[12 + k], false, false);
        E[4 + k] = b[0];
        E[12 + k] = b[1];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // stage 2: odd rows of groups 0 / 2 <-> even rows of groups 1 / 3
        const auto a = __builtin_amdgcn_permlane16_swap(E[k], E[4 + k], false, false);
        E[k] = a[0];
        E[4 + k] = a[1];
        const auto b = __builtin_amdgcn_permlane16_swap(E[8 + k], E[12 + k], false, false);
        E[8 + k] = b[0];
        E[12 + k] = b[1];
    }
}

__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)b) << 16);
}

// 8 waves per block; 2 levels per gather round (4: the loads of 4 levels in flight need > 128
// VGPRs and spill, -3 %)
constexpr int FEM2_WAVES = 8, FEM_LPR = 2;
constexpr int PRE_LEVELS = 8;  // coarse levels round 1 may find pre-encoded (encode_coarse_first_kernel)
static_assert(PRE_LEVELS % FEM_LPR == 0 && PRE_LEVELS % 2 == 0, "pre-encoded levels: whole rounds and pairs");
static_assert(L % FEM_LPR == 0, "levels per round");
template <bool COLOR>
__global__ void __launch_bounds__(64 * FEM2_WAVES, FEM2_WAVES / 2) field_encode_mlp_reg_kernel(
    const float* __restrict__ xyzs, const float* __restrict__ dirs, int64_t n, const int64_t* __restrict__ n_dev,
    const int32_t* __restrict__ sidx, GridArgs ga, const uint32_t* __restrict__ table,
    const _Float16* __restrict__ mlp, _Float16* __restrict__ enc_pm, float* __restrict__ sigmas,
    float* __restrict__ rgbs, _Float16* __restrict__ h_out) {
    __shared__ __attribute__((aligned(16))) _Float16 sw[SWF];
    __shared__ LevelLds lv;
    NGP_PROBE_BEGIN(NGP_P_FIELD_ENCODE_MLP);
    const int64_t N = ngp_capped_count(n_dev, n);  // (a device count never past the capacity: a guard hit)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t G = gridDim.x;
    const int64_t chunks = (N + 63) >> 6;
    int64_t k = (int64_t)wv * G + blockIdx.x;  // first chunk of this wave (wave-uniform)
    // the first chunk's index and position (count -> index -> position: dependent round
    // trips) requested before the weight image is built, so the two overlap
    int64_t i_first = 0;
    float in_first[3];
    {
        const int64_t j = k * 64 + lane;
        const bool valid = k < chunks && j < N;
        i_first = valid ? (sidx ? (int64_t)sidx[j] : j) : 0;
        load_x01(xyzs, i_first, valid, ga, in_first);
    }
    load_fwd_weights_direct(mlp, sw, COLOR);
    load_levels(ga, lv);
    __syncthreads();
    bool first = true;
    for (; k < chunks; k += (int64_t)FEM2_WAVES * G) {
        int lane_l = lane;  // (opaque per iteration: lane-derived addresses are not held across the loop)
        asm volatile("" : "+v"(lane_l));
        const int s = lane_l & 15, g = lane_l >> 4;
        const int64_t j = k * 64 + lane_l;
        const bool valid = j < N;
        int64_t i = i_first;
        float in[3] = {in_first[0], in_first[1], in_first[2]};
        if (!first) {
            i = valid ? (sidx ? (int64_t)sidx[j] : j) : 0;
            load_x01(xyzs, i, valid, ga, in);
        }
        first = false;
        uint32_t E[16];  // level l's two features, fp16x2
        // rounds of FEM_LPR levels, not unrolled (an unrolled chain hoists every round's
        // loads: 256 VGPRs); each round shifts its levels into the top of E, so after the
        // last round E[l] holds level l
#pragma unroll 1
        for (int r = 0; r < L / FEM_LPR; ++r) {
            uint32_t v[FEM_LPR][8];
#pragma unroll
            for (int q = 0; q < FEM_LPR; ++q) gather_level_loads(in, level_u(lv, FEM_LPR * r + q), table, v[q]);
#pragma unroll
            for (int q = 0; q < 16 - FEM_LPR; ++q) E[q] = E[q + FEM_LPR];
#pragma unroll
            for (int q = 0; q < FEM_LPR; ++q) E[16 - FEM_LPR + q] = level_sum_h2(in, level_u(lv, FEM_LPR * r + q), v[q]);
        }
        if (valid && enc_pm) {
#pragma unroll
            for (int pr = 0; pr < 8; ++pr)
                *reinterpret_cast<uint2*>(enc_pm + ((int64_t)pr * n + i) * 4) = make_uint2(E[2 * pr], E[2 * pr + 1]);
        }
        transpose_rows4(E);
        const int32_t imine = valid ? (int32_t)i : -1;
        // column blocks in a loop (not unrolled: register pressure); block c's operand is
        // E[0..3] after c rotations by one group
#pragma unroll 1
        for (int c = 0; c < 4; ++c) {
            const int32_t ic = __shfl(imine, 16 * c + s, 64);
            const bool ok = ic >= 0;
            const h8 e = __builtin_bit_cast(h8, make_uint4(E[0], E[1], E[2], E[3]));
#pragma unroll
            for (int q = 0; q < 12; ++q) E[q] = E[q + 4];
            h4 h1[4];
            const h4 hh = density_net(e, sw, s, g, h1);
            if (ok) {
                if (h_out) *reinterpret_cast<h4*>(h_out + (int64_t)ic * 16 + 4 * g) = hh;
                if (g == 0) sigmas[ic] = expf((float)hh[0]);  // TruncExp forward (custom_functions.py:165-167)
            }
            if constexpr (COLOR) {
                const float dx = ok ? dirs[3 * (int64_t)ic] : 0.f, dy = ok ? dirs[3 * (int64_t)ic + 1] : 0.f,
                            dz = ok ? dirs[3 * (int64_t)ic + 2] : 1.f;
                float sh[4];
                sh4_select(dx, dy, dz, g, sh);
                const h8 cin = {(_Float16)sh[0], (_Float16)sh[1], (_Float16)sh[2], (_Float16)sh[3], hh[0], hh[1], hh[2], hh[3]};
                h4 h3[4], h4v[4];
                const h4 o = color_net(cin, sw, s, g, h3, h4v);
                if (ok && g == 0) {
                    rgbs[3 * (int64_t)ic] = sigmoid_h(o[0]);
                    rgbs[3 * (int64_t)ic + 1] = sigmoid_h(o[1]);
                    rgbs[3 * (int64_t)ic + 2] = sigmoid_h(o[2]);
                }
            }
        }
    }
    NGP_PROBE_END();
}

// Encode + MLPs of the 64-sample chunk [i0, i0 + cnt) on one wave (lane =
// sample i0 + lane): field_encode_mlp_reg_kernel's body for a contiguous
// chunk; returns this lane's sigma (0 past cnt) for a transmittance epilogue.
// pre (0 or PRE_LEVELS): levels [0, pre) are already in enc_pm (written by
// encode_coarse_first_kernel with the same arithmetic) and only read back.
template <bool COLOR>
__device__ __forceinline__ float encode_mlp_chunk(const float* __restrict__ xyzs, const float* __restrict__ dirs,
                                                  int64_t i0, int cnt, int64_t n, const GridArgs& ga,
                                                  const LevelLds& lv, const uint32_t* __restrict__ table,
                                                  const _Float16* sw, _Float16* __restrict__ enc_pm,
                                                  float* __restrict__ sigmas, float* __restrict__ rgbs, int pre = 0) {
    int lane_l = threadIdx.x & 63;  // (opaque: lane-derived addresses are rematerialised, not held)
    asm volatile("" : "+v"(lane_l));
    const int s = lane_l & 15, g = lane_l >> 4;
    const bool valid = lane_l < cnt;
    const int64_t i = i0 + lane_l;
    float in[3];
    load_x01(xyzs, i, valid, ga, in);
    uint32_t E[16];
    if (pre) {
        // after pre / FEM_LPR rounds the chain holds levels [0, pre) at the top of E
#pragma unroll
        for (int pr = 0; pr < PRE_LEVELS / 2; ++pr) {
            const uint2 q = valid ? *reinterpret_cast<const uint2*>(enc_pm + ((int64_t)pr * n + i) * 4) : make_uint2(0u, 0u);
            E[16 - PRE_LEVELS + 2 * pr] = q.x;
            E[16 - PRE_LEVELS + 2 * pr + 1] = q.y;
        }
    }
#pragma unroll 1
    for (int rr = pre / FEM_LPR; rr < L / FEM_LPR; ++rr) {
        uint32_t v[FEM_LPR][8];
#pragma unroll
        for (int q = 0; q < FEM_LPR; ++q) gather_level_loads(in, level_u(lv, FEM_LPR * rr + q), table, v[q]);
#pragma unroll
        for (int q = 0; q < 16 - FEM_LPR; ++q) E[q] = E[q + FEM_LPR];
#pragma unroll
        for (int q = 0; q < FEM_LPR; ++q) E[16 - FEM_LPR + q] = level_sum_h2(in, level_u(lv, FEM_LPR * rr + q), v[q]);
    }
    if (valid && enc_pm) {
#pragma unroll
        for (int pr = 0; pr < 8; ++pr)
            if (2 * pr >= pre)
                *reinterpret_cast<uint2*>(enc_pm + ((int64_t)pr * n + i) * 4) = make_uint2(E[2 * pr], E[2 * pr + 1]);
    }
    transpose_rows4(E);
    float sg = 0.f;
#pragma unroll 1
    for (int c = 0; c < 4; ++c) {
        if (16 * c >= cnt) break;  // (wave-uniform: no sample in this or a later column block)
        const bool ok = 16 * c + s < cnt;
        const int64_t ic = i0 + 16 * c + s;
        const h8 e = __builtin_bit_cast(h8, make_uint4(E[0], E[1], E[2], E[3]));
#pragma unroll
        for (int q = 0; q < 12; ++q) E[q] = E[q + 4];
        h4 h1[4];
        const h4 hh = density_net(e, sw, s, g, h1);
        const float sig = expf((float)hh[0]);  // TruncExp forward (custom_functions.py:165-167)
        if (ok && g == 0) sigmas[ic] = sig;
        const float sgc = __shfl(sig, lane_l & 15, 64);  // sample 16 c + s's sigma to lane 16 c + s
        if ((lane_l >> 4) == c) sg = sgc;
        if constexpr (COLOR) {
            const float dx = ok ? dirs[3 * ic] : 0.f, dy = ok ? dirs[3 * ic + 1] : 0.f, dz = ok ? dirs[3 * ic + 2] : 1.f;
            float sh[4];
            sh4_select(dx, dy, dz, g, sh);
            const h8 cin = {(_Float16)sh[0], (_Float16)sh[1], (_Float16)sh[2], (_Float16)sh[3], hh[0], hh[1], hh[2], hh[3]};
            h4 h3[4], h4v[4];
            const h4 o = color_net(cin, sw, s, g, h3, h4v);
            if (ok && g == 0) {
                rgbs[3 * ic] = sigmoid_h(o[0]);
                rgbs[3 * ic + 1] = sigmoid_h(o[1]);
                rgbs[3 * ic + 2] = sigmoid_h(o[2]);
            }
        }
    }
    return sg;
}

// Round 1 of the chunked training forward with the round-2 counts fused in:
// one wave per non-empty row (rows[], built beside the previous step by
// ngp_rays_nonempty, so no wave holds more than its one chunk while rows are
// fewer than resident waves), its first min(N, 64) samples encoded and run
// through the MLPs, then the row's transmittance over them
// (chunk_transmittance, the composite's product scan: the same function and
// expressions as chunk_segments_kernel) -> rc = N - 64 if the row is still
// transparent after its first chunk, else 0.  rest (nullable): rest[r] = rc
// (the counts ngp_chunk_counts_range gives).  list2 (nullable): the row's
// round-2 samples start + 64 .. start + N appended to list2 at a range
// reserved by one atomic on *total2 (zero at launch): the round-2 list
// without any scan -- rows land in reservation order, each row's samples
// contiguous (the forward's outputs are per sample, so the order changes no
// value); their count is added to *evaluated with the first chunks'.  A wave
// per row rather than 64 packed list entries (~8 % idle lanes on this step's
// rows); the sigmas never leave registers.
template <bool COLOR>
__global__ void __launch_bounds__(64 * FEM2_WAVES, FEM2_WAVES / 2) field_first_chunk_kernel(
    const float* __restrict__ xyzs, const float* __restrict__ dirs, const float* __restrict__ deltas,
    const int64_t* __restrict__ rays_a, const int32_t* __restrict__ rows, const int64_t* __restrict__ n_rows_dev,
    int64_t n_rows, int64_t n, float T_thr, GridArgs ga, const uint32_t* __restrict__ table,
    const _Float16* __restrict__ mlp, _Float16* __restrict__ enc_pm, float* __restrict__ sigmas,
    float* __restrict__ rgbs, int32_t* __restrict__ rest, int32_t* __restrict__ list2, int64_t* __restrict__ total2,
    int64_t* __restrict__ evaluated, int pre) {
    __shared__ __attribute__((aligned(16))) _Float16 sw[SWF];
    __shared__ LevelLds lv;
    __shared__ unsigned long long blk_eval;
    NGP_PROBE_BEGIN(NGP_P_FIRST_CHUNK);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t NR = ngp_capped_count(n_rows_dev, n_rows);  // (a device count never past the capacity: a guard hit)
    const int64_t G = gridDim.x, stride = (int64_t)FEM2_WAVES * G;
    int64_t j = (int64_t)wv * G + blockIdx.x;  // the wave's first row (wave-uniform)
    // its row (list -> rays_a: dependent round trips) requested before the weight image is built
    int64_t r = 0, start = 0, N = 0;
    if (j < NR) {
        r = rows ? (int64_t)rows[j] : j;
        start = rays_a[3 * r + 1];
        N = rays_a[3 * r + 2];
    }
    if (threadIdx.x == 0) blk_eval = 0ull;
    load_fwd_weights_direct(mlp, sw, COLOR);
    load_levels(ga, lv);
    __syncthreads();
    int64_t ev = 0;
    for (; j < NR; j += stride) {
        const int cnt = (int)(N < 64 ? N : 64);
        int32_t rc = 0;
        if (cnt > 0) {
            const float dl = lane < cnt ? deltas[start + lane] : 0.f;
            const float sg = encode_mlp_chunk<COLOR>(xyzs, dirs, start, cnt, n, ga, lv, table, sw, enc_pm, sigmas, rgbs,
                                                     pre);
            const float om = 1.0f - (1.0f - __expf(-sg * dl));  // chunk_segments_kernel's expression
            const ChunkT ct = chunk_transmittance(om, cnt, 1.0f, T_thr, lane);
            rc = (!ct.hit && N > 64) ? (int32_t)(N - 64) : 0;
            ev += cnt;
        }
        if (rest && lane == 0) rest[r] = rc;
        if (list2 && rc > 0) {
            unsigned long long o = 0;
            if (lane == 0) o = atomicAdd((unsigned long long*)total2, (unsigned long long)rc);
            const int64_t o2 = (int64_t)__shfl(o, 0, 64);
            if (lane == 0 && o2 + rc > n) ngp_guard_hit();  // (past the list's capacity n: counted, then bounded)
            for (int t = lane; t < rc && o2 + t < n; t += 64) list2[o2 + t] = (int32_t)(start + 64 + t);
            ev += rc;
        }
        const int64_t jn = j + stride;
        if (jn < NR) {
            r = rows ? (int64_t)rows[jn] : jn;
            start = rays_a[3 * r + 1];
            N = rays_a[3 * r + 2];
        }
    }
    if (lane == 0 && ev) atomicAdd(&blk_eval, (unsigned long long)ev);
    __syncthreads();
    if (threadIdx.x == 0 && evaluated && blk_eval) atomicAdd((unsigned long long*)evaluated, blk_eval);
    NGP_PROBE_END();
}

// Levels [0, PRE_LEVELS) of round 1's encoding, ahead of time: for the rows
// rows[j], j < *n_rows_dev, of the NEXT batch (its march and row list are
// done beside the current step), the first min(N, 64) samples' coarse-level
// features, written to the pair-major enc_pm (pairs [0, PRE_LEVELS / 2)) with
// encode_mlp_chunk's arithmetic.  Those levels' parameters are final once the
// MLP + coarse levels' Adam of the current step has run, ~a bucket
// accumulation before the step ends, so this runs beside the binned levels'
// accumulation and round 1 of the next step (field_first_chunk_kernel with
// pre = PRE_LEVELS) gathers only the fine levels: half its dependent gather
// rounds leave the critical path.
__global__ void __launch_bounds__(256) encode_coarse_first_kernel(
    const float* __restrict__ xyzs, const int64_t* __restrict__ rays_a, const int32_t* __restrict__ rows,
    const int64_t* __restrict__ n_rows_dev, int64_t n_rows, int64_t n, GridArgs ga,
    const uint32_t* __restrict__ table, _Float16* __restrict__ enc_pm) {
    __shared__ LevelLds lv;
    NGP_PROBE_BEGIN(NGP_P_PRE_ENCODE);
    load_levels(ga, lv);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t NR = ngp_capped_count(n_rows_dev, n_rows);  // (a device count never past the capacity: a guard hit)
    // a wave item = (row, level pair): one gather round per item, the row's PRE_LEVELS / 2 pairs
    // on consecutive waves (one dependent round each instead of PRE_LEVELS / 2 per row: the rows
    // are ~2.7 K, a third of the waves the chip holds)
    constexpr int NP = PRE_LEVELS / 2;
    const int64_t stride = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t q = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); q < NR * NP; q += stride) {
        const int64_t j = q / NP;
        const int pr = (int)(q - j * NP);
        const int64_t r = rows ? (int64_t)rows[j] : j;
        const int64_t start = rays_a[3 * r + 1], N = rays_a[3 * r + 2];
        const bool valid = lane < N;
        const int64_t i = start + lane;
        float in[3];
        load_x01(xyzs, i, valid, ga, in);
        uint32_t v[2][8];
        gather_level_loads(in, level_u(lv, 2 * pr), table, v[0]);
        gather_level_loads(in, level_u(lv, 2 * pr + 1), table, v[1]);
        const uint32_t e0 = level_sum_h2(in, level_u(lv, 2 * pr), v[0]);
        const uint32_t e1 = level_sum_h2(in, level_u(lv, 2 * pr + 1), v[1]);
        if (valid) *reinterpret_cast<uint2*>(enc_pm + ((int64_t)pr * n + i) * 4) = make_uint2(e0, e1);
    }
    NGP_PROBE_END();
}

// One level of the coarse (atomic) hash backward for the wave's 16 consecutive
// samples, lane = 4 s + 2 cx + f: corner c = cx | cy << 1 | cz << 2 of sample s
// receives w_c * gd (gd = dL/denc[s][2 l + f]); runs of equal corners along the
// 16 samples (lanes 4 apart) are merged by segmented suffix sums, and each
// run's head adds its sum with one memory-side fp32 atomic into dst.
// coarse_level_runs: the corner indices (idx[yz], level-offset included), the
// run sums v[yz] and the run-head masks of one level; coarse_scatter_level
// then adds each head's sum with a memory-side atomic.
__device__ __forceinline__ void coarse_level_runs(const float in[3], bool valid, float gd, int l, const LevelLds& lv,
                                                  int lane, int cx, uint32_t idx[4], float v[4], uint64_t heads[4]) {
    const float sc = lv.scale[l];
    const uint32_t res = lv.res[l], size = lv.size[l], off = lv.off[l];
    const bool dense = (lv.dense >> l) & 1u, pow2 = (lv.pow2 >> l) & 1u;
    float pos[3];
    uint32_t pg[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const float p = fmaf(sc, in[d], 0.5f);
        const float fl = floorf(p);
        pg[d] = (uint32_t)(int)fl;
        pos[d] = p - fl;
    }
    // corner c = cx | (cy<<1) | (cz<<2); weight product in tcnn's d order.
    // The four y/z corners are independent: their shuffles are issued
    // together (one LDS round trip per scan step, not four).
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const int cy = yz & 1, cz = yz >> 1;
        float wt = 1.0f;
        wt *= cx ? pos[0] : 1 - pos[0];
        wt *= cy ? pos[1] : 1 - pos[1];
        wt *= cz ? pos[2] : 1 - pos[2];
        idx[yz] = valid ? off + corner_index(pg[0] + cx, pg[1] + cy, pg[2] + cz, res, size, dense, pow2)
                        : 0xffffffffu;
        v[yz] = wt * gd;
    }
    uint32_t prev[4];
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) prev[yz] = __shfl_up(idx[yz], 4, 64);
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) heads[yz] = __ballot(lane < 4 || prev[yz] != idx[yz]);
    if ((heads[0] & heads[1] & heads[2] & heads[3]) != ~0ull) {
        // some runs: segmented suffix sums at lane stride 4
#pragma unroll
        for (int o4 = 4; o4 < 64; o4 <<= 1) {
            float ov[4];
#pragma unroll
            for (int yz = 0; yz < 4; ++yz) ov[yz] = __shfl_down(v[yz], o4, 64);
            // lanes lane+4, lane+8, ..., lane+o4 must all continue the run
            const uint64_t span = ((0x1111111111111111ull & ((2ull << o4) - 1ull)) & ~1ull) << lane;
#pragma unroll
            for (int yz = 0; yz < 4; ++yz)
                if (lane + o4 < 64 && (heads[yz] & span) == 0) v[yz] += ov[yz];
        }
    }
}

__device__ __forceinline__ void coarse_scatter_level(const float in[3], bool valid, float gd, int l, const LevelLds& lv,
                                                     float* __restrict__ dst, int lane, int cx, int f) {
    uint32_t idx[4];
    float v[4];
    uint64_t heads[4];
    coarse_level_runs(in, valid, gd, l, lv, lane, cx, idx, v, heads);
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const bool head = (heads[yz] >> lane) & 1ull;
        if (head && valid) atomicAdd(&dst[2 * (size_t)idx[yz] + f], v[yz]);
    }
}

// ------------------------------------------------------------------ backward
// MLP backward helpers: v_mfma_f32_16x16x16_f16, whose B operand layout
// B[k = 4g + j][n = s] IS the accumulator layout, so every gradient tile of
// the data chain re-enters the next MFMA from registers.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f4 mfma16(h4 a, h4 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ h4 lds4(const _Float16* p) { return *reinterpret_cast<const h4*>(p); }

constexpr int RT16 = 20, RT64 = 68;  // transposed-weight rows: 16 / 64 halfs + pad
constexpr int BT5 = SWF, BT4 = BT5 + 64 * RT16, BT3 = BT4 + 64 * RT64, BT2 = BT3 + 16 * RT64, BT1 = BT2 + 64 * RT16,
              BTE = BT1 + 32 * RT64;
// operand tiles of the weight-gradient sums: [sample][unit] 16x16 images
// (32-byte rows: the packed 8-byte stores and the ds_read_b64_tr_b16 reads
// of a 32-lane half both cover 64 distinct banks), after the weight images
constexpr int TROW = 16, TTILE = 16 * TROW;
constexpr int SCR = (BTE + 7) & ~7;

__device__ __forceinline__ void load_bwd_weights(const _Float16* __restrict__ mlp, _Float16* sw) {
    const int t = threadIdx.x, nt = blockDim.x;
    // W5T[i][o] = W5[o][i] (64 x 16); W4T (64 x 64); W3hT[i][o] = W3[o][16+i] (16 x 64);
    // W2T[i][o] = W2[o][i] (64 x 16); W1T[i][o] = W1[o][i] (32 x 64)
    for (int e = t; e < 64 * 16; e += nt) { const int i = e >> 4, o = e & 15; sw[BT5 + i * RT16 + o] = mlp[OW5 + o * 64 + i]; }
    for (int e = t; e < 64 * 64; e += nt) { const int i = e >> 6, o = e & 63; sw[BT4 + i * RT64 + o] = mlp[OW4 + o * 64 + i]; }
    for (int e = t; e < 16 * 64; e += nt) { const int i = e >> 6, o = e & 63; sw[BT3 + i * RT64 + o] = mlp[OW3 + o * 32 + 16 + i]; }
    for (int e = t; e < 64 * 16; e += nt) { const int i = e >> 4, o = e & 15; sw[BT2 + i * RT16 + o] = mlp[OW2 + o * 64 + i]; }
    for (int e = t; e < 32 * 64; e += nt) { const int i = e >> 6, o = e & 63; sw[BT1 + i * RT64 + o] = mlp[OW1 + o * 32 + i]; }
}

// The backward's weight images (load_fwd_weights + load_bwd_weights) straight
// from global memory in one pass: a thread item is two rows (o, o+1) x 8
// columns of one matrix, two 16-byte loads; the forward image takes each half
// at its permuted position, the transposed matrices a 4-byte pair {W[o][i],
// W[o+1][i]} per column (no raw staging buffer, no barrier between the
// passes: 6.4 -> ~3 us per block, scripts/diag/mlpbwd_phases.py).
__device__ __forceinline__ void load_bwd_weights_direct(const _Float16* __restrict__ mlp, _Float16* sw) {
    // items: W1 32 row pairs x 4 column blocks, W2 8 x 8, W3 32 x 4, W4 32 x 8, W5 8 x 8
    constexpr int N1 = 128, N2 = 64, N3 = 128, N4 = 256, N5 = 64, NI = N1 + N2 + N3 + N4 + N5;
    for (int it = threadIdx.x; it < NI; it += blockDim.x) {
        int ow, lg_cb, li, bt, rt, skip;  // matrix offset, log2(column blocks), local item, bwd image, row, skipped cols
        if (it < N1) { ow = OW1; lg_cb = 2; li = it; bt = BT1; rt = RT64; skip = 0; }
        else if (it < N1 + N2) { ow = OW2; lg_cb = 3; li = it - N1; bt = BT2; rt = RT16; skip = 0; }
        else if (it < N1 + N2 + N3) { ow = OW3; lg_cb = 2; li = it - N1 - N2; bt = BT3; rt = RT64; skip = 16; }
        else if (it < NI - N5) { ow = OW4; lg_cb = 3; li = it - N1 - N2 - N3; bt = BT4; rt = RT64; skip = 0; }
        else { ow = OW5; lg_cb = 3; li = it - (NI - N5); bt = BT5; rt = RT16; skip = 0; }
        const int in_dim = 8 << lg_cb, o = 2 * (li >> lg_cb), i0 = 8 * (li & ((1 << lg_cb) - 1));
        const int f0 = ow + o * in_dim + i0;
        const h8 a = *reinterpret_cast<const h8*>(mlp + f0);
        const h8 b = *reinterpret_cast<const h8*>(mlp + f0 + in_dim);
        place_fwd8(f0, a, sw);
        place_fwd8(f0 + in_dim, b, sw);
        if (i0 >= skip) {  // (W3: only the h columns 16..31 are transposed)
#pragma unroll
            for (int jj = 0; jj < 8; ++jj)
                *reinterpret_cast<h2v*>(sw + bt + (i0 - skip + jj) * rt + o) = h2v{a[jj], b[jj]};
        }
    }
}

__device__ __forceinline__ float max4(f4 v) { return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))); }
// Per-sample power-of-two scales of the data chain: a gradient tile travels in
// fp16 as value x 2^E, E per sample (the same in its four lanes).  At the
// chain's two inputs (dL/drgb through the sigmoid, dL/dh with TruncExp's dL/dsigma)
// E comes from the sample's largest |value| so that it lands in [2^13, 2^14): a
// full 11-bit mantissa for everything within 2^27 of it.  A layer's MFMA output
// is in units of the previous E; after W^T the next E is the previous one minus
// the block's bound exponent of W^T (colsum_exp: the output stays below 2^14, no
// per-sample max), and one power-of-two factor 2^(E_new - E_prev) re-scales it
// (exact).
constexpr int E_MIN = -100, E_MAX = 100;
__device__ __forceinline__ int fexp(float m) {  // m = f 2^e, f in [0.5, 1) (0 -> 0)
    int e;
    frexpf(m, &e);
    return e;
}
__device__ __forceinline__ int next_exp(float m_scaled, int e_prev) {
    return min(max(e_prev + 14 - fexp(m_scaled), E_MIN), E_MAX);
}
__device__ __forceinline__ h4 cvt4(f4 v, float r) {
    return h4{(_Float16)(v[0] * r), (_Float16)(v[1] * r), (_Float16)(v[2] * r), (_Float16)(v[3] * r)};
}
// ReLU' of an fp16 gradient tile by its layer's activation tile (relu_h's
// output: sign clear): keep a half where act > 0, i.e. its bits are nonzero --
// (act + 0x7fff) has bit 15 set exactly then, an arithmetic shift spreads it.
__device__ __forceinline__ uint32_t mask_h2(uint32_t gv, uint32_t av) {
    const s16x2 t = __builtin_bit_cast(s16x2, __builtin_bit_cast(u16x2, av) + (u16x2){0x7fff, 0x7fff});
    return gv & __builtin_bit_cast(uint32_t, t >> (s16x2){15, 15});
}
__device__ __forceinline__ h4 relu_mask(h4 gr, h4 act) {
    const uint2 gv = __builtin_bit_cast(uint2, gr), av = __builtin_bit_cast(uint2, act);
    return __builtin_bit_cast(h4, make_uint2(mask_h2(gv.x, av.x), mask_h2(gv.y, av.y)));
}
// 2^k (k <= 0) as a pair of fp16 (subnormal down to 2^-24, 0 below)
__device__ __forceinline__ uint32_t f16_pow2_x2(int k) {
    const uint32_t b = k >= -14 ? (uint32_t)(k + 15) << 10 : k >= -24 ? 1u << (k + 24) : 0u;
    return b | (b << 16);
}
// an fp16 tile times a per-lane fp16 factor pair (v_pk_mul_f16; exact for powers of two)
typedef _Float16 hx2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h4 mul_h4(h4 v, uint32_t f2) {
    const uint2 u = __builtin_bit_cast(uint2, v);
    const hx2 f = __builtin_bit_cast(hx2, f2);
    return __builtin_bit_cast(h4, make_uint2(__builtin_bit_cast(uint32_t, __builtin_bit_cast(hx2, u.x) * f),
                                             __builtin_bit_cast(uint32_t, __builtin_bit_cast(hx2, u.y) * f)));
}
// v x 2^k (k <= 0) rounded once to fp16: one v_pk_mul_f16 by the fp16 factor
// while 2^k is representable (k >= -24, subnormal factors included); below,
// where the factor is not but the product may be (an fp16 subnormal or even
// normal value), through fp32 -- the same single rounding
__device__ __forceinline__ h4 scale_h4(h4 v, int k) {
    if (k >= -24) return mul_h4(v, f16_pow2_x2(k));
    const float f = ldexpf(1.0f, k);
    return h4{(_Float16)((float)v[0] * f), (_Float16)((float)v[1] * f), (_Float16)((float)v[2] * f),
              (_Float16)((float)v[3] * f)};
}
// min over the wave's 16 samples of a per-sample int (lanes 0-15 hold samples 0-15)
__device__ __forceinline__ int samples_min(int v) {
#define NGP_DPP_ROR_I(x, n) __builtin_amdgcn_update_dpp(0, (x), 0x120 + (n), 0xf, 0xf, false)
    v = min(v, NGP_DPP_ROR_I(v, 1));
    v = min(v, NGP_DPP_ROR_I(v, 2));
    v = min(v, NGP_DPP_ROR_I(v, 4));
    v = min(v, NGP_DPP_ROR_I(v, 8));
#undef NGP_DPP_ROR_I
    return __builtin_amdgcn_readfirstlane(v);
}
// Accumulator tile X[4g + r][s] (lane (s, g)) -> image row s, units 4g..4g+3.
// The four 8-byte chunks of row s sit XOR-swizzled, chunk c at c ^ ((s >> 2) & 3):
// a ds_write_b64 group (16 lanes, banks mod 32) then covers 32 distinct banks
// (unswizzled, rows 8 dwords apart hit 4 banks 4 ways), and get_tile's reads
// stay conflict-free.
__device__ __forceinline__ void put_tile(_Float16* T, h4 v, int s, int g) {
    *reinterpret_cast<h4*>(T + s * TROW + 4 * (g ^ ((s >> 2) & 3))) = v;
}
// units 8h..8h+7 of row s (chunks 2h, 2h+1; e0 = units 8h..8h+3) under the same swizzle
__device__ __forceinline__ void put_tile_pair(_Float16* T, h4 e0, h4 e1, int s, int h) {
    const int sw = (s >> 2) & 3;
    *reinterpret_cast<h8*>(T + s * TROW + 4 * ((2 * h) ^ (sw & 2))) = (sw & 1) ? pack(e1, e0) : pack(e0, e1);
}
// Transposed read: lane (u = s, g) receives X[u][4g + q], q = 0..3, i.e. the
// K = sample fragment of the 16x16x16 operand.  Lane 4q+p of each 16-lane
// group addresses image row 4g+q, units 4p..4p+3 (= T + 4*lane).
typedef __fp16 hp4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
__device__ __forceinline__ h4 get_tile(const _Float16* T, int s, int g) {
    // row 4g + (s >> 2), chunk s & 3 -> stored at chunk (s & 3) ^ g (put_tile's swizzle)
    const _Float16* a = T + 64 * g + 4 * ((s & 12) | ((s & 3) ^ g));
    return __builtin_bit_cast(h4, __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                                      (__attribute__((address_space(3))) hp4*)(const_cast<_Float16*>(a))));
}
// accumulator tile k -> (matrix offset, in_dim, o0, i0)
__device__ __forceinline__ void acc_tile_info(int k, int& ow, int& in_dim, int& o0, int& i0) {
    if (k < 4) { ow = OW5; in_dim = 64; o0 = 0; i0 = 16 * k; return; }
    k -= 4;
    if (k < 16) { ow = OW4; in_dim = 64; o0 = 16 * (k >> 2); i0 = 16 * (k & 3); return; }
    k -= 16;
    if (k < 8) { ow = OW3; in_dim = 32; o0 = 16 * (k >> 1); i0 = 16 * (k & 1); return; }
    k -= 8;
    if (k < 4) { ow = OW2; in_dim = 64; o0 = 0; i0 = 16 * k; return; }
    k -= 4;
    ow = OW1; in_dim = 32; o0 = 16 * (k >> 1); i0 = 16 * (k & 1);
}

// Kernel A: the MLP backward, block-cooperative.  Eight waves per block (two
// per SIMD -- a per-wave kernel holding all 40 weight-gradient tiles in
// registers ran one wave per SIMD, latency-bound on its dependent MFMA / LDS
// chain: 105.8 vs 78.8 us, profiles/r02/mlp_split_coop.json).  Each wave
// back-propagates its own 16-sample column block (forward recomputed from the
// saved fp16 encoding); the weight gradients are then summed by
// the block: every wave puts its operand tiles into its LDS region and wave w
// accumulates output tiles {k} over all eight regions (K = 128 samples per
// block iteration), 5 of the 40 tiles per wave.  Operands go through LDS in
// two phases (layers 5-3: 19 tiles, then layers 2-1: 11 tiles) so eight
// regions fit beside the weight images.  Gradient operands of the data
// chain are fp16 scaled per SAMPLE (column of the B operand; the four lanes
// of a sample exchange their maxima with v_permlane16/32_swap) by a power of
// two, unscaled exactly in fp32 for dL/denc; the weight gradients take the
// same fp16 values re-scaled to one power of two per layer and block
// (tcnn's fp16 operands with the role of its loss scale, no global scale to
// tune).
// (diagnostics only: scripts/diag/mlpbwd_phases.hip defines these to stamp the
// phases of a block iteration and the kernel's edges; empty in the product build)
#ifndef NGP_BWD_PHASE
#define NGP_BWD_PHASE(k)
#define NGP_BWD_EDGE(k)
#endif
// CW waves per block (CW / 4 per SIMD; 12 fit the LDS at <= 168 VGPRs but measured -3 %, DESIGN.md
// section 9 round 4)
constexpr int CW = 8, NT1 = 19, NT2 = 11, CSCRW = NT1 * TTILE;
constexpr int COOP_LDS_HALFS = SCR + CW * CSCRW;
static_assert(CW % 4 == 0, "waves per block: a multiple of 4");
static_assert(NGP_MLP_PARAMS <= CW * CSCRW && NT2 <= NT1, "raw weight staging / phase-2 tiles exceed the scratch");
static_assert(COOP_LDS_HALFS * 2 <= 160 * 1024, "cooperative MLP backward exceeds the LDS");
// output tiles per phase (phase 1: layers 5, 4, 3 = 4 + 16 + 8; phase 2: layers 2, 1 = 4 + 8), dealt
// to the CW waves in contiguous runs (tiles sharing a G operand stay together), at most KT1 / KT2 each
constexpr int NK1 = 28, NK2 = 12, KT1 = (NK1 + CW - 1) / CW, KT2 = (NK2 + CW - 1) / CW;
// phase-1 / phase-2 tile ids inside a wave's region
constexpr int P_DO = 0, P_DA4 = 1, P_DA3 = 5, P_H4 = 9, P_H3 = 13, P_C = 17;
constexpr int Q_DH = 0, Q_DA1 = 1, Q_H1 = 5, Q_E = 9;

// max over the four lanes of one sample (lanes s, s+16, s+32, s+48)
__device__ __forceinline__ float sample_max(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}

// ceil(log2(max_i sum_o |W^T[i][o]|)) of a transposed weight image (rows of nout halfs,
// pitch rt, nin rows; one row per lane, max over the wave): |W^T x| < 2^k max|x| for
// every x, so a gradient tile scaled below 2^14 stays below 2^14 after W^T and a
// re-scale by 2^-k (the inner layers' exponents without per-sample maxima: only the
// chain's two inputs, dL/drgb and dL/dsigma, set a per-sample exponent).  Whole wave,
// uniform result.
__device__ __forceinline__ int colsum_exp(const _Float16* img, int nin, int nout, int rt, int lane) {
    float a = 0.f;
    if (lane < nin)
        for (int o = 0; o < nout; o += 4) {  // (8-byte row reads; the same sequential sum)
            const h4 v = *reinterpret_cast<const h4*>(img + lane * rt + o);
            a += fabsf((float)v[0]);
            a += fabsf((float)v[1]);
            a += fabsf((float)v[2]);
            a += fabsf((float)v[3]);
        }
    for (int off = 32; off > 0; off >>= 1) a = fmaxf(a, __shfl_xor(a, off, 64));
    int e = 0;
    const float m = frexpf(a, &e);
    e = a == 0.f ? -30 : (m == 0.5f ? e - 1 : e);  // ceil(log2(a)) (a = 2^(e-1) exactly: e - 1)
    return __builtin_amdgcn_readfirstlane(e);
}

// output tile k (acc_tile_info order) -> operand tile ids (G, H) in its phase's region
__device__ __forceinline__ void coop_tile_ops(int k, int& gid, int& hid) {
    if (k < 4) { gid = P_DO; hid = P_H4 + k; return; }
    if (k < 20) { gid = P_DA4 + ((k - 4) >> 2); hid = P_H3 + ((k - 4) & 3); return; }
    if (k < 28) { gid = P_DA3 + ((k - 20) >> 1); hid = P_C + ((k - 20) & 1); return; }
    if (k < 32) { gid = Q_DH; hid = Q_H1 + (k - 28); return; }
    gid = Q_DA1 + ((k - 32) >> 1);
    hid = Q_E + ((k - 32) & 1);
}

// wave w owns tiles [start, start + n) of a phase of NK tiles: the first NK % CW waves one more
template <int NK>
__device__ __forceinline__ int coop_start(int w) { return w * (NK / CW) + min(w, NK % CW); }
template <int NK>
__device__ __forceinline__ int coop_count(int w) { return NK / CW + (w < NK % CW ? 1 : 0); }
__device__ __forceinline__ int coop_k1(int w, int t) { return coop_start<NK1>(w) + t; }
__device__ __forceinline__ int coop_n1(int w) { return coop_count<NK1>(w); }
__device__ __forceinline__ int coop_k2(int w, int t) { return NK1 + coop_start<NK2>(w) + t; }
__device__ __forceinline__ int coop_n2(int w) { return coop_count<NK2>(w); }

// layer of output tile k: 0 = W5 (G = dL/dout), 1 = W4 (dL/da4), 2 = W3 (dL/da3),
// 3 = W2 (dL/dh), 4 = W1 (dL/da1)
__device__ __forceinline__ int tile_layer(int k) { return k < 4 ? 0 : k < 20 ? 1 : k < 28 ? 2 : k < 32 ? 3 : 4; }

// v_mfma_f32_16x16x32_f16 over two source regions at a time: the K order
// (lane group g, element j) <- sample 4g + (j & 3) of region src + (j >> 2) is
// the same for the A and the B operand, so the sum over K is the sum over the
// 32 samples.  The G tiles of one layer carry the block's common scale 2^B, so
// each tile's block sum is added to its accumulator times 2^-B (Bl[layer]).
template <int NTL>
__device__ __forceinline__ void coop_dw(const _Float16* scr, int w, int s, int g, int n, int (*kf)(int, int), f4* acc,
                                        const int* Bl) {
    int gid[NTL], hid[NTL];
    float sc[NTL];
    f4 part[NTL];
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
        const int k = kf(w, t < n ? t : 0);
        coop_tile_ops(k, gid[t], hid[t]);
        const int l = tile_layer(k);  // (wave-uniform: the select stays scalar)
        sc[t] = ldexpf(1.0f, -(l == 0 ? Bl[0] : l == 1 ? Bl[1] : l == 2 ? Bl[2] : l == 3 ? Bl[3] : Bl[4]));
    }
#pragma unroll
    for (int src = 0; src < CW; src += 2) {
        const _Float16* R0 = scr + src * CSCRW;
        const _Float16* R1 = R0 + CSCRW;
        h4 G0 = get_tile(R0 + gid[0] * TTILE, s, g), G1 = get_tile(R1 + gid[0] * TTILE, s, g);
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
            if (t >= n) break;
            if (t > 0 && gid[t] != gid[t - 1]) {
                G0 = get_tile(R0 + gid[t] * TTILE, s, g);
                G1 = get_tile(R1 + gid[t] * TTILE, s, g);
            }
            const h8 H = pack(get_tile(R0 + hid[t] * TTILE, s, g), get_tile(R1 + hid[t] * TTILE, s, g));
            part[t] = mfma32(pack(G0, G1), H, src == 0 ? f4{0.f, 0.f, 0.f, 0.f} : part[t]);
        }
    }
#pragma unroll
    for (int t = 0; t < NTL; ++t)
        if (t < n) acc[t] = part[t] * sc[t] + acc[t];
}

__global__ void __launch_bounds__(64 * CW, CW / 4) field_bwd_mlp_coop_kernel(
    const float* __restrict__ dirs, int64_t n, const int64_t* __restrict__ n_dev, const int32_t* __restrict__ sidx,
    const _Float16* __restrict__ enc, const _Float16* __restrict__ mlp, const float* __restrict__ dL_dsig,
    const float* __restrict__ dL_drgb, float* __restrict__ denc, float* __restrict__ grad_mlp, int64_t enc_pm_stride) {
    extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
    // per-wave minima of the layers' per-sample exponents (double-buffered by iteration parity)
    __shared__ __attribute__((aligned(16))) int emin[2][5][CW];
    _Float16* sw = smem;
    _Float16* scr = smem + SCR;
    NGP_BWD_EDGE(0);
    NGP_PROBE_BEGIN(NGP_P_MLP_BWD);
    const int64_t N = ngp_capped_count(n_dev, n);  // (a device count never past the capacity: a guard hit)
    const int lane = threadIdx.x & 63, s = lane & 15, g = lane >> 4;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    _Float16* mine = scr + wid * CSCRW;
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    f4 acc1[KT1], acc2[KT2];
#pragma unroll
    for (int t = 0; t < KT1; ++t) acc1[t] = z;
#pragma unroll
    for (int t = 0; t < KT2; ++t) acc2[t] = z;
    struct In {
        h8 e;
        float dx, dy, dz, dsig, gr[3];
    };
    // the sample of row jj (-1 past the end): listed rows' indices are loaded
    // two iterations ahead, so the dependent loads of the next iteration's
    // inputs never wait on an index load
    auto row_index = [&](int64_t jj) -> int32_t {
        return jj < N ? (sidx ? sidx[jj] : (int32_t)jj) : -1;
    };
    auto load_in = [&](int32_t ii, In& x) {
        x.e = h8{0, 0, 0, 0, 0, 0, 0, 0};
        x.dx = 0.f; x.dy = 0.f; x.dz = 1.f; x.dsig = 0.f; x.gr[0] = x.gr[1] = x.gr[2] = 0.f;
        if (ii >= 0) {
            if (enc_pm_stride > 0)  // pair-major (ngp_hash_encode): pairs 2g, 2g+1
                x.e = pack(*reinterpret_cast<const h4*>(enc + ((2 * g) * enc_pm_stride + ii) * 4),
                           *reinterpret_cast<const h4*>(enc + ((2 * g + 1) * enc_pm_stride + ii) * 4));
            else
                x.e = *reinterpret_cast<const h8*>(enc + (int64_t)ii * 32 + 8 * g);
            x.dx = dirs[3 * (int64_t)ii]; x.dy = dirs[3 * (int64_t)ii + 1]; x.dz = dirs[3 * (int64_t)ii + 2];
            x.dsig = dL_dsig[ii];
            x.gr[0] = dL_drgb[3 * (int64_t)ii]; x.gr[1] = dL_drgb[3 * (int64_t)ii + 1];
            x.gr[2] = dL_drgb[3 * (int64_t)ii + 2];
        }
    };
    const int64_t stride = (int64_t)gridDim.x * CW * 16;
    const int64_t j0 = (int64_t)blockIdx.x * CW * 16 + 16 * wid + s;
    // the first iteration's inputs (count -> index -> rows: three dependent
    // round trips) are requested before the weight images are staged, so the
    // two overlap
    In cur;
    load_in(row_index(j0), cur);
    int32_t i_next = row_index(j0 + stride);
    load_bwd_weights_direct(mlp, sw);
    __syncthreads();
    // per-block bounds of W5^T, W4^T, W2^T: the inner layers' exponents follow from their input's
    // (round 5; rounds 3-4 took a per-sample max after every layer: 12 % more VALU, 6 % longer);
    // one wave per matrix (round 6: every wave computed all three, ~1.3 M VALU per launch)
    __shared__ int kex[3];
    if (wid < 3) {
        const int e = wid == 0 ? colsum_exp(sw + BT5, 64, 16, RT16, lane)
                    : wid == 1 ? colsum_exp(sw + BT4, 64, 64, RT64, lane) : colsum_exp(sw + BT2, 64, 16, RT16, lane);
        if (lane == 0) kex[wid] = e;
    }
    __syncthreads();
    const int k5 = __builtin_amdgcn_readfirstlane(kex[0]), k4 = __builtin_amdgcn_readfirstlane(kex[1]);
    const int k2 = __builtin_amdgcn_readfirstlane(kex[2]);
    NGP_BWD_EDGE(1);
    int par = 0;
    // block-uniform trip count: every wave reaches every barrier
    for (int64_t bb = (int64_t)blockIdx.x * CW * 16; bb < N; bb += stride, par ^= 1) {
        const int64_t base = bb + 16 * wid;
        In nxt;
        load_in(i_next, nxt);
        i_next = row_index(base + s + 2 * stride);
        NGP_BWD_PHASE(0);
        // the lane's (sample, group) re-derived opaquely per iteration: the LDS / global
        // addresses built from them are recomputed here instead of held (or spilled) across the
        // loop as loop-invariant registers
        int lane_l = lane;
        asm volatile("" : "+v"(lane_l));
        const int s = lane_l & 15, g = lane_l >> 4;
        const int64_t j = base + s;
        const bool valid = j < N;
        const h8 e = cur.e;

        // ---- forward recompute
        h4 h1[4];
        const h4 hh = density_net(e, sw, s, g, h1);
        float sh[4];
        sh4_select(cur.dx, cur.dy, cur.dz, g, sh);
        const h4 shh = {(_Float16)sh[0], (_Float16)sh[1], (_Float16)sh[2], (_Float16)sh[3]};
        h4 h3[4], h4v[4];
        const h4 o = color_net(pack(shh, hh), sw, s, g, h3, h4v);
        NGP_BWD_PHASE(1);
        // ---- output layer: sigmoid backward on rows 0..2
        f4 dout = z;
        if (g == 0) {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const float y = 1.0f / (1.0f + expf(-(float)o[r]));
                dout[r] = cur.gr[r] * (y * (1.0f - y));
            }
        }
        const int Eo = next_exp(sample_max(max4(dout)), 0);
        const h4 do_h = cvt4(dout, ldexpf(1.0f, Eo));
        // ---- dL/da4 = ReLU'(W5^T do)   (MFMA output in units of 2^Eo; |.| < 2^(14 + k5))
        f4 c4[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) c4[t] = mfma16(lds4(sw + BT5 + (16 * t + s) * RT16 + 4 * g), do_h, z);
        const int E4 = max(Eo - k5, E_MIN);
        h4 da4h[4];
        {
            const float r = ldexpf(1.0f, E4 - Eo);
#pragma unroll
            for (int t = 0; t < 4; ++t) da4h[t] = relu_mask(cvt4(c4[t], r), h4v[t]);
        }
        // ---- dL/da3 = ReLU'(W4^T da4)
        f4 c3[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            f4 c = z;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) c = mfma16(lds4(sw + BT4 + (16 * t + s) * RT64 + 16 * kt + 4 * g), da4h[kt], c);
            c3[t] = c;
        }
        const int E3 = max(E4 - k4, E_MIN);
        h4 da3h[4];
        {
            const float r = ldexpf(1.0f, E3 - E4);
#pragma unroll
            for (int t = 0; t < 4; ++t) da3h[t] = relu_mask(cvt4(c3[t], r), h3[t]);
        }
        // ---- dL/dh (colour-net input, h part) = W3h^T da3, + TruncExp backward (true units)
        f4 dh = z;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) dh = mfma16(lds4(sw + BT3 + s * RT64 + 16 * kt + 4 * g), da3h[kt], dh);
        dh = dh * ldexpf(1.0f, -E3);
        if (g == 0) dh[0] += cur.dsig * expf(fminf(fmaxf((float)hh[0], -15.f), 15.f));  // custom_functions.py:169-173
        const int Eh = next_exp(sample_max(max4(dh)), 0);
        const h4 dhh = cvt4(dh, ldexpf(1.0f, Eh));
        // ---- dL/da1 = ReLU'(W2^T dh)
        f4 c1[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) c1[t] = mfma16(lds4(sw + BT2 + (16 * t + s) * RT16 + 4 * g), dhh, z);
        const int E1 = max(Eh - k2, E_MIN);
        h4 da1h[4];
        {
            const float r = ldexpf(1.0f, E1 - Eh);
#pragma unroll
            for (int t = 0; t < 4; ++t) da1h[t] = relu_mask(cvt4(c1[t], r), h1[t]);
        }
        // ---- dL/denc = W1^T da1 (rows 16t + 4g + r of sample s), true units
        {
            const float r = ldexpf(1.0f, -E1);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                f4 c = z;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) c = mfma16(lds4(sw + BT1 + (16 * t + s) * RT64 + 16 * kt + 4 * g), da1h[kt], c);
                c = c * r;
                if (valid) *reinterpret_cast<f4*>(denc + j * 32 + 16 * t + 4 * g) = c;
            }
        }
        NGP_BWD_PHASE(2);
        cur = nxt;
        // ---- weight gradients: fp16 operands (tcnn's precision), K = samples.  The G
        // (gradient) tiles of a layer are re-scaled from their per-sample exponent E_s
        // to the block's common one B = min_s E_s (the block's largest gradient at
        // [2^13, 2^14); factors <= 1, exact down to fp16 subnormals), the H tiles are
        // the fp16 activations / encoding as they are.
        const int Es[5] = {Eo, E4, E3, Eh, E1};
        int wmin[5];
#pragma unroll
        for (int l = 0; l < 5; ++l) wmin[l] = samples_min(Es[l]);  // (uniform: the DPP reads every lane of the row)
        if (lane == 0) {
#pragma unroll
            for (int l = 0; l < 5; ++l) emin[par][l][wid] = wmin[l];
        }
        __syncthreads();  // every wave's phase-2 reads of the previous iteration are done; emin[par] complete
        NGP_BWD_PHASE(3);
        int fk[5];  // per-sample re-scale exponents B - E_s (<= 0)
        int Bl[5];
#pragma unroll
        for (int l = 0; l < 5; ++l) {
            int mn = 1 << 30;
#pragma unroll
            for (int q = 0; q < CW; q += 4) {
                const int4 a = *reinterpret_cast<const int4*>(&emin[par][l][q]);
                mn = min(mn, min(min(a.x, a.y), min(a.z, a.w)));
            }
            Bl[l] = __builtin_amdgcn_readfirstlane(mn);
            fk[l] = Bl[l] - Es[l];
        }
        // phase 1 (layers 5, 4, 3)
        put_tile(mine + P_DO * TTILE, scale_h4(do_h, fk[0]), s, g);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            put_tile(mine + (P_DA4 + t) * TTILE, scale_h4(da4h[t], fk[1]), s, g);
            put_tile(mine + (P_DA3 + t) * TTILE, scale_h4(da3h[t], fk[2]), s, g);
            put_tile(mine + (P_H4 + t) * TTILE, h4v[t], s, g);
            put_tile(mine + (P_H3 + t) * TTILE, h3[t], s, g);
        }
        put_tile(mine + P_C * TTILE, shh, s, g);
        put_tile(mine + (P_C + 1) * TTILE, hh, s, g);
        __syncthreads();
        NGP_BWD_PHASE(4);
        coop_dw<KT1>(scr, wid, s, g, coop_n1(wid), coop_k1, acc1, Bl);
        __syncthreads();  // phase-1 reads done: the regions take the phase-2 tiles
        NGP_BWD_PHASE(5);
        // ---- phase 2 (layers 2, 1)
        put_tile(mine + Q_DH * TTILE, scale_h4(dhh, fk[3]), s, g);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            put_tile(mine + (Q_DA1 + t) * TTILE, scale_h4(da1h[t], fk[4]), s, g);
            put_tile(mine + (Q_H1 + t) * TTILE, h1[t], s, g);
        }
        // enc fragment: lane holds enc[8g + j] of sample s -> tile g>>1, units 8(g&1)+j
        put_tile_pair(mine + (Q_E + (g >> 1)) * TTILE, h4{e[0], e[1], e[2], e[3]}, h4{e[4], e[5], e[6], e[7]}, s, g & 1);
        __syncthreads();
        NGP_BWD_PHASE(6);
        coop_dw<KT2>(scr, wid, s, g, coop_n2(wid), coop_k2, acc2, Bl);
        NGP_BWD_PHASE(7);
    }
    // each output tile lives in exactly one wave of the block: one global add
    // per weight.  Wave w of every block owns the same tiles, so the adds of a
    // lane start at a block-dependent rotation (same-address adds serialise at
    // the memory-side atomic unit: 12 -> 7 us per launch; per-block partial
    // rows + a reduction launch measured slower).
    NGP_BWD_EDGE(2);
    const int n1 = coop_n1(wid), n2 = coop_n2(wid), nadd = 4 * (n1 + n2);
    const int rot = (int)(blockIdx.x % (unsigned)nadd);
    // (q = 4 t + r over the wave's tiles in order, taken from q = rot on: two passes over a fully
    // unrolled tile loop, so each add's accumulator element and weight offset are static -- the
    // dynamically indexed version spent ~1000 VALU per wave selecting them)
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int t = 0; t < KT1 + KT2; ++t) {
            const bool p1 = t < KT1;
            const int tt = p1 ? t : t - KT1;
            if (p1 ? tt >= n1 : tt >= n2) continue;
            const int tflat = p1 ? tt : n1 + tt;
            const f4 a = p1 ? acc1[p1 ? tt : 0] : acc2[p1 ? 0 : tt];
            const int k = p1 ? coop_k1(wid, tt) : coop_k2(wid, tt);
            int ow, in_dim, o0, i0;
            acc_tile_info(k, ow, in_dim, o0, i0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int q = 4 * tflat + r;
                if ((pass == 0) != (q >= rot)) continue;
                atomicAdd(&grad_mlp[ow + (o0 + 4 * g + r) * in_dim + i0 + s], a[r]);
            }
        }
    }
    NGP_BWD_EDGE(3);
    NGP_PROBE_END();
}


// Kernel B: hash-table gradient scatter, dL/dtable[e][f] += w_c * dL/denc[2l+f].
// Lane map: 16 consecutive samples per wave, 4 lanes per sample:
//   lane = 4*s + 2*cx + f  (cx = the corner's x bit, f = feature).
// One wave instruction then carries, per sample, the x-adjacent corner pair
// x both features: 4 floats that sit in 16 contiguous bytes whenever the two
// entries are neighbours (dense levels; hashed levels when px is even, since
// the x term of the hash is px*1), so the atomics leave as one request per
// sample instead of four scattered ones.  Samples of one ray are consecutive,
// so equal indices of the same (cx, f) at lane stride 4 are first summed by a
// segmented suffix scan; only each run's head issues its fp32 atomic.
// Levels [lo, hi) (the hybrid backward's atomic coarse levels; [0, L) for
// the all-atomic API path).
__global__ void __launch_bounds__(256) hash_bwd_kernel(const float* __restrict__ xyzs, int64_t n,
                                                       const int64_t* __restrict__ n_dev,
                                                       const int32_t* __restrict__ sidx, GridArgs ga,
                                                       const float* __restrict__ denc, float* __restrict__ grad,
                                                       int lo, int hi, float* __restrict__ rep = nullptr,
                                                       int rep_hi = 0, uint32_t rep_stride = 0, int nrep = 1) {
    // levels below rep_hi add into this block's replica of their gradient
    // range (ngp_hash_backward_levels_rep): the coarsest levels are a few
    // hundred KB that every sample touches, so their memory-side atomics
    // queue on few lines; nrep copies spread them (summed afterwards)
    float* const grep = rep ? rep + (size_t)(blockIdx.x % nrep) * rep_stride : grad;
    __shared__ LevelLds lv;
    // the wave's 16 denc rows, staged once per iteration with coalesced 16-B
    // loads (one global round trip instead of one per level)
    __shared__ __attribute__((aligned(16))) float drow[4][16][36];
    NGP_PROBE_BEGIN(NGP_P_HASH_BWD_COARSE);
    load_levels(ga, lv);
    __syncthreads();
    const int64_t N = ngp_capped_count(n_dev, n);  // (a device count never past the capacity: a guard hit)
    const int lane = threadIdx.x & 63, s = lane >> 2, cx = (lane >> 1) & 1, f = lane & 1, wv = threadIdx.x >> 6;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t base = ((int64_t)blockIdx.x * (blockDim.x >> 6) + wv) * 16; base < N; base += nw * 16) {
        const int64_t j = base + s;  // compact position (denc row)
        const bool valid = j < N;
        const int64_t i = valid && sidx ? (int64_t)sidx[j] : j;  // sample
        {
            // lane (s, q = lane & 3) copies floats [8q, 8q+8) of row j
            const int q = lane & 3;
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
            if (valid && 8 * q + 8 > 2 * lo && 8 * q < 2 * hi) {
                a = *reinterpret_cast<const float4*>(denc + j * 32 + 8 * q);
                b = *reinterpret_cast<const float4*>(denc + j * 32 + 8 * q + 4);
            }
            __builtin_amdgcn_wave_barrier();  // previous iteration's reads of drow are done (in order per wave)
            *reinterpret_cast<float4*>(&drow[wv][s][8 * q]) = a;
            *reinterpret_cast<float4*>(&drow[wv][s][8 * q + 4]) = b;
        }
        float in[3];
        load_x01(xyzs, i, valid, ga, in);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
        for (int l = lo; l < hi; ++l)
            coarse_scatter_level(in, valid, drow[wv][s][2 * l + f], l, lv, l < rep_hi ? grep : grad, lane, cx, f);
    }
    NGP_PROBE_END();
}

constexpr unsigned HASH_BWD_BLOCKS = 8192;  // grid cap of hash_bwd_kernel, all-level API path (2048 measured slower)
// grid cap of the training step's coarse levels (launch_coarse): 2048 waves, two per SIMD.  Round 5: its
// atomics spread over a longer span beside the record write, now that the coarse levels' Adam runs beside
// the accumulation and no longer waits on it -- with the prefetch-free accumulation +1.2-1.3 %; round 6
// re-check: 256 / 1024 / 2048 blocks -3.2 / -0.5 / -1.2 %, profiles/r06/ab/coarse_grid.txt;
// profiles/r05/ab/round5_ab.txt r5ee / r5ff (rounds 2-4: 8192, when a longer coarse kernel delayed that Adam)
constexpr unsigned COARSE_BLOCKS = 512;

// grad[i] += sum_r rep[r][i]; rep[r][i] = 0 (i < n4 float4 groups), replicas
// summed in order r = 0..nrep-1; all of a lane's loads are issued first
template <int MAXR>
__global__ void __launch_bounds__(256) rep_reduce_kernel(float* __restrict__ grad, float* __restrict__ rep,
                                                         uint32_t n4, uint32_t stride4, int nrep) {
    float4* g4 = reinterpret_cast<float4*>(grad);
    float4* r4 = reinterpret_cast<float4*>(rep);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
        float4 b[MAXR];
#pragma unroll
        for (int r = 0; r < MAXR; ++r)
            if (r < nrep) b[r] = r4[(size_t)r * stride4 + i];
        float4 a = g4[i];
#pragma unroll
        for (int r = 0; r < MAXR; ++r)
            if (r < nrep) {
                a.x += b[r].x; a.y += b[r].y; a.z += b[r].z; a.w += b[r].w;
                r4[(size_t)r * stride4 + i] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        g4[i] = a;
    }
}

static int launch_bwd_mlp(const float* dirs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                          const void* enc_f16, int64_t enc_pm_stride, const void* mlp_f16, const float* dL_dsigmas,
                          const float* dL_drgbs, float* denc_ws, float* grad_mlp, void* stream) {
    static bool attr_set = false;
    const size_t clds = (size_t)COOP_LDS_HALFS * sizeof(_Float16);
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)field_bwd_mlp_coop_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)clds) != hipSuccess)
            return NGP_ERANGE;
        attr_set = true;
    }
    hipStream_t s = as_stream(stream);
    static const unsigned ccap = resident_blocks(field_bwd_mlp_coop_kernel, 64 * CW, clds);
    const unsigned cb = persistent_blocks(n, CW * 16, ccap);
    NGP_TIMED(NGP_K_MLP_BWD, s, field_bwd_mlp_coop_kernel<<<cb, 64 * CW, clds, s>>>(
        dirs, n, n_dev, sample_idx, (const _Float16*)enc_f16, (const _Float16*)mlp_f16, dL_dsigmas, dL_drgbs, denc_ws,
        grad_mlp, enc_pm_stride));
    return ngp_launch_status();
}

}  // namespace ngp

using namespace ngp;

extern "C" {

int ngp_field_forward(const float* xyzs, const float* dirs, int64_t n, const int64_t* n_dev,
                      const ngp_hashgrid_t* grid, const void* table_f16, const void* mlp_f16, float* sigmas,
                      float* rgbs, void* enc_f16, void* h_f16, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && dirs && table_f16 && mlp_f16 && sigmas && rgbs);
    NGP_CHECK_ARG(((uintptr_t)table_f16 & 15) == 0);  // 16-byte group gathers
    NGP_CHECK_ARG(((uintptr_t)mlp_f16 & 15) == 0);
    static const unsigned cap = resident_blocks(field_fwd_kernel<true>, 256, 0);
    field_fwd_kernel<true><<<persistent_blocks(n, 64, cap), 256, 0, as_stream(stream)>>>(
        xyzs, dirs, n, n_dev, ga, (const uint32_t*)table_f16, (const _Float16*)mlp_f16, sigmas, rgbs,
        (_Float16*)enc_f16, (_Float16*)h_f16);
    return ngp_launch_status();
}

int ngp_field_forward_indexed(const float* xyzs, const float* dirs, int64_t n, const int64_t* n_dev,
                              const int32_t* sample_idx, const ngp_hashgrid_t* grid, const void* table_f16,
                              const void* mlp_f16, float* sigmas, float* rgbs, void* enc_f16, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && dirs && sample_idx && table_f16 && mlp_f16 && sigmas && rgbs);
    NGP_CHECK_ARG(((uintptr_t)table_f16 & 15) == 0);  // 16-byte group gathers
    NGP_CHECK_ARG(((uintptr_t)mlp_f16 & 15) == 0);
    static const unsigned cap = resident_blocks(field_fwd_kernel<true>, 256, 0);
    field_fwd_kernel<true><<<persistent_blocks(n, 64, cap), 256, 0, as_stream(stream)>>>(
        xyzs, dirs, n, n_dev, ga, (const uint32_t*)table_f16, (const _Float16*)mlp_f16, sigmas, rgbs,
        (_Float16*)enc_f16, nullptr, nullptr, 0, sample_idx);
    return ngp_launch_status();
}

int ngp_density_forward(const float* xyzs, int64_t n, const int64_t* n_dev, const ngp_hashgrid_t* grid,
                        const void* table_f16, const void* mlp_f16, float* sigmas, void* h_f16, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && table_f16 && mlp_f16 && sigmas);
    NGP_CHECK_ARG(((uintptr_t)table_f16 & 15) == 0);  // 16-byte group gathers
    NGP_CHECK_ARG(((uintptr_t)mlp_f16 & 15) == 0);
    static const unsigned cap = resident_blocks(field_fwd_kernel<false>, 256, 0);
    field_fwd_kernel<false><<<persistent_blocks(n, 64, cap), 256, 0, as_stream(stream)>>>(
        xyzs, nullptr, n, n_dev, ga, (const uint32_t*)table_f16, (const _Float16*)mlp_f16, sigmas, nullptr, nullptr,
        (_Float16*)h_f16);
    return ngp_launch_status();
}

int ngp_hash_encode(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                    const ngp_hashgrid_t* grid, const void* table_f16, void* enc_pm, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && table_f16 && enc_pm && ((uintptr_t)enc_pm & 7) == 0);
    NGP_CHECK_ARG(((uintptr_t)table_f16 & 15) == 0);  // 16-byte group gathers
    hipStream_t s = as_stream(stream);
    static const unsigned cap = resident_blocks(hash_encode_kernel, 256, 0);
    NGP_TIMED(NGP_K_HASH_ENCODE, s, hash_encode_kernel<<<std::max(1u, std::min(cap, (unsigned)((n + 255) / 256))), 256, 0, s>>>(
        xyzs, n, n_dev, sample_idx, ga, (const uint32_t*)table_f16, (_Float16*)enc_pm));
    return ngp_launch_status();
}

int ngp_field_encode_mlp(const float* xyzs, const float* dirs, int64_t n, const int64_t* n_dev,
                         const int32_t* sample_idx, const ngp_hashgrid_t* grid, const void* table_f16,
                         const void* mlp_f16, void* enc_pm, float* sigmas, float* rgbs, void* h_f16, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && table_f16 && mlp_f16 && sigmas && (dirs != nullptr) == (rgbs != nullptr));
    NGP_CHECK_ARG(((uintptr_t)table_f16 & 15) == 0 && ((uintptr_t)mlp_f16 & 15) == 0 && ((uintptr_t)enc_pm & 7) == 0);
    hipStream_t s = as_stream(stream);
    // grid = every resident block (the chunks are dealt over the whole grid)
    if (!dirs) {
        static const unsigned capd = resident_blocks(field_encode_mlp_reg_kernel<false>, 64 * FEM2_WAVES, 0);
        NGP_TIMED(NGP_K_HASH_ENCODE, s, field_encode_mlp_reg_kernel<false><<<std::max(1u, std::min(capd, (unsigned)((n + 64 * FEM2_WAVES - 1) / (64 * FEM2_WAVES)))), 64 * FEM2_WAVES, 0, s>>>(
            xyzs, nullptr, n, n_dev, sample_idx, ga, (const uint32_t*)table_f16, (const _Float16*)mlp_f16,
            (_Float16*)enc_pm, sigmas, nullptr, (_Float16*)h_f16));
        return ngp_launch_status();
    }
    static const unsigned capr = resident_blocks(field_encode_mlp_reg_kernel<true>, 64 * FEM2_WAVES, 0);
    NGP_TIMED(NGP_K_HASH_ENCODE, s, field_encode_mlp_reg_kernel<true><<<std::max(1u, std::min(capr, (unsigned)((n + 64 * FEM2_WAVES - 1) / (64 * FEM2_WAVES)))), 64 * FEM2_WAVES, 0, s>>>(
        xyzs, dirs, n, n_dev, sample_idx, ga, (const uint32_t*)table_f16, (const _Float16*)mlp_f16,
        (_Float16*)enc_pm, sigmas, rgbs, (_Float16*)h_f16));
    return ngp_launch_status();
}

int ngp_field_forward_first_pre(const float* xyzs, const float* dirs, const float* deltas, const int64_t* rays_a,
                                const int32_t* rows, const int64_t* n_rows_dev, int64_t n_rows, int64_t n,
                                float T_threshold, const ngp_hashgrid_t* grid, const void* table_f16,
                                const void* mlp_f16, void* enc_pm, float* sigmas, float* rgbs, int32_t* rest,
                                int32_t* list2, int64_t* total2, int64_t* evaluated, int pre_levels, void* stream) {
    NGP_CHECK_ARG(pre_levels == 0 || (pre_levels == PRE_LEVELS && enc_pm));
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n_rows >= 0 && n >= 0);
    if (n_rows == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && dirs && deltas && rays_a && table_f16 && mlp_f16 && sigmas && rgbs && (rest || list2));
    NGP_CHECK_ARG(!list2 || (total2 && ((uintptr_t)total2 & 7) == 0));
    NGP_CHECK_ARG(((uintptr_t)table_f16 & 15) == 0 && ((uintptr_t)mlp_f16 & 15) == 0 && ((uintptr_t)enc_pm & 7) == 0 &&
                  ((uintptr_t)evaluated & 7) == 0);
    hipStream_t s = as_stream(stream);
    // grid = every resident block: the rows are dealt over all resident waves
    static const unsigned cap = resident_blocks(field_first_chunk_kernel<true>, 64 * FEM2_WAVES, 0);
    const unsigned blocks = std::max(1u, std::min(cap, (unsigned)((n_rows + FEM2_WAVES - 1) / FEM2_WAVES)));
    NGP_TIMED(NGP_K_HASH_ENCODE, s, field_first_chunk_kernel<true><<<blocks, 64 * FEM2_WAVES, 0, s>>>(
        xyzs, dirs, deltas, rays_a, rows, n_rows_dev, n_rows, n, T_threshold, ga, (const uint32_t*)table_f16,
        (const _Float16*)mlp_f16, (_Float16*)enc_pm, sigmas, rgbs, rest, list2, total2, evaluated, pre_levels));
    return ngp_launch_status();
}

int ngp_field_forward_first(const float* xyzs, const float* dirs, const float* deltas, const int64_t* rays_a,
                            const int32_t* rows, const int64_t* n_rows_dev, int64_t n_rows, int64_t n,
                            float T_threshold, const ngp_hashgrid_t* grid, const void* table_f16, const void* mlp_f16,
                            void* enc_pm, float* sigmas, float* rgbs, int32_t* rest, int32_t* list2,
                            int64_t* total2, int64_t* evaluated, void* stream) {
    return ngp_field_forward_first_pre(xyzs, dirs, deltas, rays_a, rows, n_rows_dev, n_rows, n, T_threshold, grid,
                                       table_f16, mlp_f16, enc_pm, sigmas, rgbs, rest, list2, total2, evaluated, 0,
                                       stream);
}

int ngp_field_encode_first_coarse(const float* xyzs, const int64_t* rays_a, const int32_t* rows,
                                  const int64_t* n_rows_dev, int64_t n_rows, int64_t n, const ngp_hashgrid_t* grid,
                                  const void* table_f16, void* enc_pm, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n_rows >= 0 && n >= 0);
    if (n_rows == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && rays_a && table_f16 && enc_pm && ((uintptr_t)table_f16 & 15) == 0 &&
                  ((uintptr_t)enc_pm & 7) == 0);
    hipStream_t s = as_stream(stream);
    static const unsigned cap = resident_blocks(encode_coarse_first_kernel, 256, 0);
    const unsigned blocks = std::max(1u, std::min(cap, (unsigned)((n_rows * (PRE_LEVELS / 2) + 3) / 4)));
    encode_coarse_first_kernel<<<blocks, 256, 0, s>>>(xyzs, rays_a, rows, n_rows_dev, n_rows, n, ga,
                                                      (const uint32_t*)table_f16, (_Float16*)enc_pm);
    return ngp_launch_status();
}

int ngp_field_mlp_forward(const void* enc_pm, const float* dirs, int64_t n, const int64_t* n_dev,
                          const int32_t* sample_idx, const void* mlp_f16, float* sigmas, float* rgbs, void* h_f16,
                          void* stream) {
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(enc_pm && mlp_f16 && sigmas && (dirs != nullptr) == (rgbs != nullptr));
    NGP_CHECK_ARG(((uintptr_t)mlp_f16 & 15) == 0 && ((uintptr_t)enc_pm & 7) == 0);
    GridArgs ga{};
    if (!dirs) {  // density net only (occupancy updates)
        static const unsigned capd = resident_blocks(field_fwd_kernel<false, true>, 256, 0);
        NGP_TIMED(NGP_K_FIELD_MLP, as_stream(stream),
                  field_fwd_kernel<false, true><<<persistent_blocks(n, 64, capd), 256, 0, as_stream(stream)>>>(
                      nullptr, nullptr, n, n_dev, ga, nullptr, (const _Float16*)mlp_f16, sigmas, nullptr, nullptr,
                      (_Float16*)h_f16, (const _Float16*)enc_pm, n, sample_idx));
        return ngp_launch_status();
    }
    static const unsigned cap = resident_blocks(field_fwd_kernel<true, true>, 256, 0);
    NGP_TIMED(NGP_K_FIELD_MLP, as_stream(stream),
              field_fwd_kernel<true, true><<<persistent_blocks(n, 64, cap), 256, 0, as_stream(stream)>>>(
                  nullptr, dirs, n, n_dev, ga, nullptr, (const _Float16*)mlp_f16, sigmas, rgbs, nullptr,
                  (_Float16*)h_f16, (const _Float16*)enc_pm, n, sample_idx));
    return ngp_launch_status();
}

int ngp_field_backward_mlp(const float* dirs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                           const void* enc_f16, int64_t enc_pm_stride, const void* mlp_f16, const float* dL_dsigmas,
                           const float* dL_drgbs, float* denc_ws, float* grad_mlp, void* stream) {
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(dirs && enc_f16 && mlp_f16 && dL_dsigmas && dL_drgbs && denc_ws && grad_mlp);
    NGP_CHECK_ARG(((uintptr_t)mlp_f16 & 15) == 0);
    return launch_bwd_mlp(dirs, n, n_dev, sample_idx, enc_f16, enc_pm_stride, mlp_f16, dL_dsigmas, dL_drgbs,
                          denc_ws, grad_mlp, stream);
}

int ngp_hash_backward(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                      const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && denc && grad_table && ((uintptr_t)denc & 15) == 0);
    NGP_TIMED(NGP_K_HASH_BWD_COARSE, as_stream(stream), hash_bwd_kernel<<<persistent_blocks(n, 64, HASH_BWD_BLOCKS), 256, 0, as_stream(stream)>>>(xyzs, n, n_dev, sample_idx,
                                                                                     ga, denc, grad_table, 0, L));
    return ngp_launch_status();
}

}  // extern "C"

static void launch_coarse(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                          const GridArgs& ga, const float* denc, float* grad_table, int lo, int hi, float* rep,
                          int rep_hi, uint32_t rep_stride, int nrep, hipStream_t s) {
    NGP_TIMED(NGP_K_HASH_BWD_COARSE, s, hash_bwd_kernel<<<persistent_blocks(n, 64, COARSE_BLOCKS), 256, 0, s>>>(
        xyzs, n, n_dev, sample_idx, ga, denc, grad_table, lo, hi, rep, rep_hi, rep_stride, nrep));
}

extern "C" {

int ngp_hash_backward_levels(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                             const ngp_hashgrid_t* grid, const float* denc, float* grad_table, int level_lo,
                             int level_hi, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0 && 0 <= level_lo && level_lo <= level_hi && level_hi <= L);
    if (n == 0 || level_lo == level_hi) return NGP_OK;
    NGP_CHECK_ARG(xyzs && denc && grad_table && ((uintptr_t)denc & 15) == 0);
    launch_coarse(xyzs, n, n_dev, sample_idx, ga, denc, grad_table, level_lo, level_hi, nullptr, 0, 0, 1,
                  as_stream(stream));
    return ngp_launch_status();
}

int ngp_hash_backward_levels_rep(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                                 const ngp_hashgrid_t* grid, const float* denc, float* grad_table, int level_lo,
                                 int level_hi, float* rep, int rep_levels, int n_rep, int fold, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0 && 0 <= level_lo && level_lo <= level_hi && level_hi <= L);
    NGP_CHECK_ARG(0 <= rep_levels && rep_levels <= level_hi && n_rep >= 1 && n_rep <= 64);
    if (rep_levels == 0 || !rep)
        return ngp_hash_backward_levels(xyzs, n, n_dev, sample_idx, grid, denc, grad_table, level_lo, level_hi,
                                        stream);
    if (n == 0 || level_lo == level_hi) return NGP_OK;
    NGP_CHECK_ARG(xyzs && denc && grad_table && ((uintptr_t)denc & 15) == 0);
    NGP_CHECK_ARG(((uintptr_t)grad_table & 15) == 0 && ((uintptr_t)rep & 15) == 0);
    // replicas cover table entries [0, offsets[rep_levels]) (x 2 features)
    const uint32_t nfl = 2u * grid->offsets[rep_levels];
    NGP_CHECK_ARG(nfl % 4 == 0);
    hipStream_t s = as_stream(stream);
    launch_coarse(xyzs, n, n_dev, sample_idx, ga, denc, grad_table, level_lo, level_hi, rep, rep_levels, nfl, n_rep, s);
    if (!fold) return ngp_launch_status();  // the caller folds them (ngp_adam_step_dev_rep)
    const uint32_t n4 = nfl / 4;
    const unsigned rb = std::min(2048u, (n4 + 255) / 256);
    if (n_rep <= 8)
        NGP_TIMED(NGP_K_HASH_BWD_COARSE, s, rep_reduce_kernel<8><<<rb, 256, 0, s>>>(grad_table, rep, n4, n4, n_rep));
    else if (n_rep <= 16)
        NGP_TIMED(NGP_K_HASH_BWD_COARSE, s, rep_reduce_kernel<16><<<rb, 256, 0, s>>>(grad_table, rep, n4, n4, n_rep));
    else
        NGP_TIMED(NGP_K_HASH_BWD_COARSE, s, rep_reduce_kernel<64><<<rb, 256, 0, s>>>(grad_table, rep, n4, n4, n_rep));
    return ngp_launch_status();
}

size_t ngp_hash_backward_rep_floats(const ngp_hashgrid_t* grid, int rep_levels, int n_rep) {
    if (!grid || rep_levels < 0 || rep_levels > L || n_rep < 1) return 0;
    return (size_t)n_rep * 2u * grid->offsets[rep_levels];
}

int ngp_field_backward(const float* xyzs, const float* dirs, int64_t n, const int64_t* n_dev,
                       const ngp_hashgrid_t* grid, const void* enc_f16, const void* mlp_f16,
                       const float* dL_dsigmas, const float* dL_drgbs, float* denc_ws, float* grad_mlp,
                       float* grad_table, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    st = ngp_field_backward_mlp(dirs, n, n_dev, nullptr, enc_f16, 0, mlp_f16, dL_dsigmas, dL_drgbs, denc_ws, grad_mlp,
                                stream);
    if (st) return st;
    return ngp_hash_backward(xyzs, n, n_dev, nullptr, grid, denc_ws, grad_table, stream);
}

}  // extern "C"
