// Diagnostic build (NOT part of libngp_amd.so): variants of the multires
// hash encode, to find what bounds it on realistic sample sets
// (scripts/diag/encode_diag.py).  Every variant writes the pair-major
// encoding of ngp_hash_encode (bit-identical values: the same gather_level_u /
// sum_level arithmetic), so the driver checks them against it.
//   mode 1: one lane per sample, only level pairs [p0, p1)   (time by level range)
//   mode 2: XCD-partitioned: a workgroup reads its XCC id and encodes that
//           XCD's level set for chunks of samples it dequeues from the XCD's
//           own counter (any placement covers every sample); set x = levels
//           {2x, 2x+1}
//   mode 3: as 2 with set x = levels {x, x + 8} (a dense level beside a hashed one)
//   mode 4: dense levels [0, lds_levels) staged into LDS (coalesced 16-B
//           copies) by a persistent 1024-thread workgroup per CU, gathered from
//           there; the other levels from global memory
#include "../../ar-nerf_amd/csrc/field.hip"
#include "../../ar-nerf_amd/csrc/host.hip"

namespace ngp {

__global__ void __launch_bounds__(256) enc_range_kernel(const float* __restrict__ xyzs, int64_t n,
                                                        const int64_t* __restrict__ n_dev, GridArgs ga,
                                                        const uint32_t* __restrict__ table,
                                                        _Float16* __restrict__ enc_pm, int p0, int p1) {
    __shared__ LevelLds lv;
    load_levels(ga, lv);
    __syncthreads();
    const int64_t N = n_dev ? *n_dev : n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        float in[3];
        load_x01(xyzs, i, true, ga, in);
#pragma unroll 1
        for (int pr = p0; pr < p1; ++pr) {
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

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 7u;
}

__global__ void zero8_kernel(uint32_t* c) {  // 8 counters, 16 words apart
    if (threadIdx.x < 128) c[threadIdx.x] = 0u;
}

template <int SET>
__global__ void __launch_bounds__(256) enc_xcd_kernel(const float* __restrict__ xyzs, int64_t n,
                                                      const int64_t* __restrict__ n_dev, GridArgs ga,
                                                      const uint32_t* __restrict__ table,
                                                      _Float16* __restrict__ enc_pm, uint32_t* __restrict__ ctr) {
    __shared__ LevelLds lv;
    __shared__ uint32_t chunk;
    load_levels(ga, lv);
    const uint32_t x = xcc_id();
    const int la = SET == 2 ? 2 * (int)x : (int)x, lb = SET == 2 ? 2 * (int)x + 1 : (int)x + 8;
    const int64_t N = n_dev ? *n_dev : n;
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) chunk = atomicAdd(&ctr[16 * x], 1u);  // (one counter per XCD, 64 B apart)
        __syncthreads();
        const int64_t i = (int64_t)chunk * blockDim.x + threadIdx.x;
        if ((int64_t)chunk * blockDim.x >= N) break;
        if (i >= N) continue;
        float in[3];
        load_x01(xyzs, i, true, ga, in);
        float w[2][8];
        uint32_t v[2][8];
        gather_level_u(in, level_u(lv, la), table, w[0], v[0]);
        gather_level_u(in, level_u(lv, lb), table, w[1], v[1]);
        float a0, a1, b0, b1;
        sum_level(w[0], v[0], a0, a1);
        sum_level(w[1], v[1], b0, b1);
        if (SET == 2) {
            *reinterpret_cast<h4*>(enc_pm + ((int64_t)x * n + i) * 4) =
                h4{(_Float16)a0, (_Float16)a1, (_Float16)b0, (_Float16)b1};
        } else {
            typedef _Float16 h2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<h2*>(enc_pm + ((int64_t)(la >> 1) * n + i) * 4 + 2 * (la & 1)) = h2{(_Float16)a0, (_Float16)a1};
            *reinterpret_cast<h2*>(enc_pm + ((int64_t)(lb >> 1) * n + i) * 4 + 2 * (lb & 1)) = h2{(_Float16)b0, (_Float16)b1};
        }
    }
}

// gather_level_u with the table read through `tl` (LDS or global) for one level
__device__ __forceinline__ void gather_level_at(const float in[3], const LevelU& u, const uint32_t* tl, float w[8],
                                                uint32_t v[8]) {
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
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const uint32_t qy = pg[1] + (yz & 1), qz = pg[2] + (yz >> 1);
        const uint32_t r0 = pg[0] + qy * u.res + qz * u.res2;
        const uint32_t i0 = reduce_idx(r0, u), i1 = reduce_idx(r0 + 1u, u);
        v[2 * yz] = tl[i0];
        v[2 * yz + 1] = tl[i1];
    }
}

__global__ void __launch_bounds__(1024) enc_lds_kernel(const float* __restrict__ xyzs, int64_t n,
                                                       const int64_t* __restrict__ n_dev, GridArgs ga,
                                                       const uint32_t* __restrict__ table,
                                                       _Float16* __restrict__ enc_pm, int lds_levels) {
    extern __shared__ __attribute__((aligned(16))) uint32_t stab[];
    __shared__ LevelLds lv;
    load_levels(ga, lv);
    const uint32_t nent = ga.g.offsets[lds_levels];  // entries of levels [0, lds_levels) (a multiple of 8)
    for (uint32_t e = threadIdx.x; e < nent / 4; e += blockDim.x)
        reinterpret_cast<uint4*>(stab)[e] = reinterpret_cast<const uint4*>(table)[e];
    __syncthreads();
    const int64_t N = n_dev ? *n_dev : n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        float in[3];
        load_x01(xyzs, i, true, ga, in);
#pragma unroll 1
        for (int pr = 0; pr < 8; ++pr) {
            float w[2][8];
            uint32_t v[2][8];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int l = 2 * pr + q;
                const LevelU u = level_u(lv, l);
                if (l < lds_levels) gather_level_at(in, u, stab + u.off, w[q], v[q]);
                else gather_level_u(in, u, table, w[q], v[q]);
            }
            float a0, a1, b0, b1;
            sum_level(w[0], v[0], a0, a1);
            sum_level(w[1], v[1], b0, b1);
            *reinterpret_cast<h4*>(enc_pm + ((int64_t)pr * n + i) * 4) =
                h4{(_Float16)a0, (_Float16)a1, (_Float16)b0, (_Float16)b1};
        }
    }
}


// mode 5: the fused encode + MLP forward software-pipelined per wave: a
// persistent wave walks its 64-sample chunks; while it gathers level pair r of
// the NEXT chunk it runs MLP slice r of the current one (slice 2cb: density net
// of column block cb, 2cb+1: its colour net) from a double-buffered LDS row
// image, so the MFMA / VALU work sits inside the gathers' latency.
template <bool COLOR, int NW>
__global__ void __launch_bounds__(64 * NW) fem_pipe_kernel(const float* __restrict__ xyzs,
                                                           const float* __restrict__ dirs, int64_t n,
                                                           const int64_t* __restrict__ n_dev,
                                                           const int32_t* __restrict__ sidx, GridArgs ga,
                                                           const uint32_t* __restrict__ table,
                                                           const _Float16* __restrict__ mlp,
                                                           _Float16* __restrict__ enc_pm, float* __restrict__ sigmas,
                                                           float* __restrict__ rgbs) {
    __shared__ __attribute__((aligned(16))) _Float16 sw[SWF];
    __shared__ __attribute__((aligned(16))) _Float16 xs[NW][2][64 * XROW];
    __shared__ int32_t xi[NW][2][64];
    __shared__ LevelLds lv;
    load_fwd_weights_direct(mlp, sw, COLOR);
    load_levels(ga, lv);
    __syncthreads();
    const int64_t N = n_dev ? *n_dev : n;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, s = lane & 15, g = lane >> 4;
    const int64_t nwaves = (int64_t)gridDim.x * NW;
    const int64_t c0 = (int64_t)blockIdx.x * NW + wv;
    auto sample_of = [&](int64_t c) -> int32_t {  // the lane's sample of chunk c (-1: none)
        const int64_t j = c * 64 + lane;
        return j < N ? (sidx ? sidx[j] : (int32_t)j) : -1;
    };
    auto fence_wave = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    if (c0 * 64 >= N) return;
    // prologue: chunk c0 into buffer 0
    {
        const int32_t i = sample_of(c0);
        float in[3];
        load_x01(xyzs, i < 0 ? 0 : i, i >= 0, ga, in);
        _Float16* row = &xs[wv][0][lane * XROW];
#pragma unroll 1
        for (int pr = 0; pr < 8; ++pr) {
            float w[2][8];
            uint32_t v[2][8];
            gather_level_u(in, level_u(lv, 2 * pr), table, w[0], v[0]);
            gather_level_u(in, level_u(lv, 2 * pr + 1), table, w[1], v[1]);
            float a0, a1, b0, b1;
            sum_level(w[0], v[0], a0, a1);
            sum_level(w[1], v[1], b0, b1);
            const h4 e4 = h4{(_Float16)a0, (_Float16)a1, (_Float16)b0, (_Float16)b1};
            if (i >= 0 && enc_pm) *reinterpret_cast<h4*>(enc_pm + ((int64_t)pr * n + i) * 4) = e4;
            *reinterpret_cast<h4*>(row + 4 * pr) = e4;
        }
        xi[wv][0][lane] = i;
        fence_wave();
    }
    int32_t i_nx = sample_of(c0 + nwaves);
    int b = 0;
    for (int64_t c = c0; c * 64 < N; c += nwaves, b ^= 1) {
        const bool has_next = (c + nwaves) * 64 < N;  // (wave-uniform)
        const int32_t inx = i_nx;
        i_nx = sample_of(c + 2 * nwaves);
        float in[3];
        load_x01(xyzs, inx < 0 ? 0 : inx, inx >= 0, ga, in);
        _Float16* nrow = &xs[wv][b ^ 1][lane * XROW];
        const _Float16* cur = xs[wv][b];
        h4 hh = h4{0, 0, 0, 0};
#pragma unroll 1
        for (int r = 0; r < 8; ++r) {
            float w[2][8];
            uint32_t v[2][8];
            if (has_next) {
                gather_level_u(in, level_u(lv, 2 * r), table, w[0], v[0]);
                gather_level_u(in, level_u(lv, 2 * r + 1), table, w[1], v[1]);
            }
            // MLP slice r of chunk c
            const int src = 16 * (r >> 1) + s;
            const int32_t ic = xi[wv][b][src];
            const bool ok = ic >= 0;
            if ((r & 1) == 0) {
                const h8 e = *reinterpret_cast<const h8*>(&cur[src * XROW + 8 * g]);
                h4 h1[4];
                hh = density_net(e, sw, s, g, h1);
                if (ok && g == 0) sigmas[ic] = expf((float)hh[0]);  // TruncExp forward (custom_functions.py:165-167)
            } else if constexpr (COLOR) {
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
            if (has_next) {
                float a0, a1, b0, b1;
                sum_level(w[0], v[0], a0, a1);
                sum_level(w[1], v[1], b0, b1);
                const h4 e4 = h4{(_Float16)a0, (_Float16)a1, (_Float16)b0, (_Float16)b1};
                if (inx >= 0 && enc_pm) *reinterpret_cast<h4*>(enc_pm + ((int64_t)r * n + inx) * 4) = e4;
                *reinterpret_cast<h4*>(nrow + 4 * r) = e4;
            }
        }
        if (has_next) xi[wv][b ^ 1][lane] = inx;
        fence_wave();
    }
}

// mode 6: ngp_hash_encode's lane-per-sample encode over rows j -> sidx[j],
// each XCD taking chunks of 256 rows from its own eighth of the rows (per-XCD
// dequeue counters; an XCD that runs dry takes chunks from the others, so any
// placement covers every row): with spatially sorted rows an XCD's L2 only
// holds its region's table entries.
__global__ void __launch_bounds__(256) enc_xcdrange_kernel(const float* __restrict__ xyzs, int64_t n,
                                                           const int32_t* __restrict__ sidx, GridArgs ga,
                                                           const uint32_t* __restrict__ table,
                                                           _Float16* __restrict__ enc_pm, uint32_t* __restrict__ ctr) {
    __shared__ LevelLds lv;
    __shared__ int64_t row0;
    load_levels(ga, lv);
    const uint32_t x = xcc_id();
    const int64_t nch = (n + 255) / 256;  // chunks of 256 rows
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t xr = (x + k) & 7u;  // own range first, then the others'
        const int64_t c_lo = nch * xr / 8, c_hi = nch * (xr + 1) / 8;
        for (;;) {
            __syncthreads();
            if (threadIdx.x == 0) {
                const int64_t c = c_lo + atomicAdd(&ctr[16 * xr], 1u);
                row0 = c < c_hi ? c * 256 : -1;
            }
            __syncthreads();
            if (row0 < 0) break;
            const int64_t j = row0 + threadIdx.x;
            if (j >= n) continue;
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
}

}  // namespace ngp

extern "C" int ngp_diag_encode(int mode, int a, int b, const float* xyzs, int64_t n, const int64_t* n_dev,
                               const ngp_hashgrid_t* grid, const void* table, void* enc_pm, uint32_t* ctr,
                               int blocks, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    hipStream_t s = as_stream(stream);
    const uint32_t* t = (const uint32_t*)table;
    _Float16* e = (_Float16*)enc_pm;
    switch (mode) {
        case 1:
            enc_range_kernel<<<blocks, 256, 0, s>>>(xyzs, n, n_dev, ga, t, e, a, b);
            break;
        case 2:
            zero8_kernel<<<1, 128, 0, s>>>(ctr);
            enc_xcd_kernel<2><<<blocks, 256, 0, s>>>(xyzs, n, n_dev, ga, t, e, ctr);
            break;
        case 3:
            zero8_kernel<<<1, 128, 0, s>>>(ctr);
            enc_xcd_kernel<3><<<blocks, 256, 0, s>>>(xyzs, n, n_dev, ga, t, e, ctr);
            break;
        case 4: {
            const size_t lds = (size_t)grid->offsets[a] * 4;
            if (lds > 150 * 1024) return NGP_ERANGE;
            if (hipFuncSetAttribute((const void*)enc_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds) != hipSuccess)
                return NGP_ERANGE;
            enc_lds_kernel<<<blocks, 1024, lds, s>>>(xyzs, n, n_dev, ga, t, e, a);
            break;
        }
        default:
            return NGP_EINVAL;
    }
    return ngp_launch_status();
}

// mode 5 (a = waves per block: 4 or 8; blocks): the pipelined fused forward
extern "C" int ngp_diag_enc_rows(int mode, const float* xyzs, int64_t n, const int32_t* sidx,
                                 const ngp_hashgrid_t* grid, const void* table, void* enc_pm, uint32_t* ctr, int blocks,
                                 void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    hipStream_t s = as_stream(stream);
    if (mode == 0) {  // the product kernel's grid, rows through sidx
        hash_encode_kernel<<<blocks, 256, 0, s>>>(xyzs, n, nullptr, sidx, ga, (const uint32_t*)table,
                                                  (_Float16*)enc_pm);
    } else {
        zero8_kernel<<<1, 128, 0, s>>>(ctr);
        enc_xcdrange_kernel<<<blocks, 256, 0, s>>>(xyzs, n, sidx, ga, (const uint32_t*)table, (_Float16*)enc_pm, ctr);
    }
    return ngp_launch_status();
}

extern "C" int ngp_diag_fem(int nw, const float* xyzs, const float* dirs, int64_t n, const ngp_hashgrid_t* grid,
                            const void* table, const void* mlp, void* enc_pm, float* sigmas, float* rgbs, int blocks,
                            void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    hipStream_t s = as_stream(stream);
    if (nw == 4)
        fem_pipe_kernel<true, 4><<<blocks, 256, 0, s>>>(xyzs, dirs, n, nullptr, nullptr, ga, (const uint32_t*)table,
                                                        (const _Float16*)mlp, (_Float16*)enc_pm, sigmas, rgbs);
    else if (nw == 2)
        fem_pipe_kernel<true, 2><<<blocks, 128, 0, s>>>(xyzs, dirs, n, nullptr, nullptr, ga, (const uint32_t*)table,
                                                        (const _Float16*)mlp, (_Float16*)enc_pm, sigmas, rgbs);
    else
        fem_pipe_kernel<true, 8><<<blocks, 512, 0, s>>>(xyzs, dirs, n, nullptr, nullptr, ga, (const uint32_t*)table,
                                                        (const _Float16*)mlp, (_Float16*)enc_pm, sigmas, rgbs);
    return ngp_launch_status();
}
