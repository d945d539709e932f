// Device-resident test-time render loop for gfx950: the reference's
// __render_rays_test (models/rendering.py:162-253) with every host decision
// moved into device memory, so a whole frame is a few HIP-graph replays with
// one host sync at the end instead of a sync + ~5 launches per iteration.
//
// Per iteration (parity p = iteration & 1 selects the alive list pair):
//   render_iter_kernel      N_alive = state[p]; stop if 0 or samples >= budget;
//                           N_samples = max(min(N_rays // N_alive, 64), min_samples)
//                           (rendering.py:188-195)
//   render_march_kernel     raymarching_test for the alive rays (raymarching.cu:335-404,
//                           identical walk to march_test_kernel) into SAMPLE-MAJOR
//                           slots [s*N_alive + n] (lane-per-ray stores and the
//                           composite's loads coalesce across lanes); appends the valid slots to a sample
//                           list (the reference's valid_mask, rendering.py:204)
//   (field kernels)         ngp_hash_encode + ngp_field_mlp_forward over the list
//   render_composite_kernel composite_test_fw (volumerendering.cu:204-284) and the
//                           alive compaction (rendering.py:236) into list p^1
//
// Results are per ray and depend on the alive list only through N_alive (an
// order-independent count), so the unordered atomic compaction gives the
// reference's values bit for bit.
#pragma clang fp contract(off)
#include "march.h"

namespace ngp {

// state (int64[NGP_RENDER_STATE_WORDS]) word indices
enum : int { RS_ALIVE0 = 0, RS_ALIVE1 = 1, RS_SAMPLES = 2, RS_NS = 3, RS_ACTIVE = 4, RS_VALID = 5, RS_TOTAL = 6,
             RS_ITERS = 7 };

__global__ void __launch_bounds__(256) render_begin_kernel(int64_t n_rays, int64_t* __restrict__ state,
                                                           int32_t* __restrict__ alive0, float* __restrict__ opacity,
                                                           float* __restrict__ depth, float* __restrict__ rgb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < NGP_RENDER_STATE_WORDS) {
        int64_t v = 0;
        if (i == RS_ALIVE0) v = n_rays;
        if (i == RS_ACTIVE) v = 1;
        state[i] = v;
    }
    if (i >= n_rays) return;
    alive0[i] = (int32_t)i;  // torch.arange(N_rays) (rendering.py:183)
    opacity[i] = 0.f;
    depth[i] = 0.f;
    rgb[3 * i] = 0.f; rgb[3 * i + 1] = 0.f; rgb[3 * i + 2] = 0.f;
}

__global__ void render_iter_kernel(int64_t* __restrict__ state, int parity, int64_t n_rays, int min_samples,
                                   int64_t sample_budget) {
    if (threadIdx.x != 0 || !state[RS_ACTIVE]) return;
    const int64_t n_alive = state[parity];
    if (n_alive == 0 || state[RS_SAMPLES] >= sample_budget) {  // rendering.py:187-190
        state[RS_ACTIVE] = 0;
        state[RS_VALID] = 0;
        return;
    }
    int64_t ns = n_rays / n_alive;
    ns = ns < 64 ? ns : 64;
    ns = ns > min_samples ? ns : min_samples;
    state[RS_SAMPLES] += ns;
    state[RS_NS] = ns;
    state[RS_VALID] = 0;
    state[parity ^ 1] = 0;
    state[RS_ITERS] += 1;
}

// Inclusive prefix sum over the 64 lanes of a wave.
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

// Block-wide append (blockDim 256, called by every thread of the block):
// this thread's first index for `cnt` items; ONE counter atomic per block
// (same-address atomics serialise: one per wave cost ~100 us per iteration
// at 640K rays).
__device__ __forceinline__ int64_t block_append(int cnt, unsigned long long* counter) {
    __shared__ int wtot[4];
    __shared__ int64_t boff;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int incl = wave_incl_scan(cnt);
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int tot = wtot[0] + wtot[1] + wtot[2] + wtot[3];
        boff = tot ? (int64_t)atomicAdd(counter, (unsigned long long)tot) : 0;
    }
    __syncthreads();
    int before = 0;
    for (int i = 0; i < w; ++i) before += wtot[i];
    const int64_t off = boff + before + incl - cnt;
    __syncthreads();  // wtot / boff are reused by the next call
    return off;
}

constexpr int CRPT = 4;  // rays per thread per composite pass

// block_append for CRPT items per thread at positions n = base + k*256 + t:
// offsets in (k, t) order, i.e. the survivors keep their alive-list order
// within the block (the list order is what keeps neighbouring pixels' samples
// adjacent for the encode's gathers), with ONE counter atomic.
__device__ __forceinline__ void block_append_k(const int (&cnt)[CRPT], int64_t (&off)[CRPT],
                                               unsigned long long* counter) {
    __shared__ int wt[CRPT][4];
    __shared__ int64_t boff;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl[CRPT];
#pragma unroll
    for (int k = 0; k < CRPT; ++k) {
        incl[k] = wave_incl_scan(cnt[k]);
        if (lane == 63) wt[k][w] = incl[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
#pragma unroll
        for (int k = 0; k < CRPT; ++k) tot += wt[k][0] + wt[k][1] + wt[k][2] + wt[k][3];
        boff = tot ? (int64_t)atomicAdd(counter, (unsigned long long)tot) : 0;
    }
    __syncthreads();
    int64_t base = boff;
#pragma unroll
    for (int k = 0; k < CRPT; ++k) {
        int before = 0;
        for (int i = 0; i < w; ++i) before += wt[k][i];
        off[k] = base + before + incl[k] - cnt[k];
        base += wt[k][0] + wt[k][1] + wt[k][2] + wt[k][3];
    }
    __syncthreads();  // wt / boff are reused by the next call
}

// ---- wave-per-ray mode (SIMPLE launches, N_samples >= WAVE_NS) ----------
// Late iterations have few alive rays with many samples each: one lane per
// ray leaves most of the chip idle while each lane walks ~N_samples occupied
// points serially.  Here one wave takes one ray and walks it with the
// lattice machinery of march_slots_wave_kernel (march.hip: the fp32 t-lattice
// in closed form per binade, a 64-point window evaluated in parallel, the
// walk's chain resolved by pointer doubling) -- the same points as the serial
// walk, bit for bit.  Sample indices are staged in LDS and appended with one
// global atomic per block flush.
constexpr int WAVE_NS = 16;  // N_samples threshold of the wave-per-ray mode (profiles/r01/render/wave_ns_ab.txt)
constexpr int STAGE = 2048;

struct WaveLds {
    LatSeg segs[4];
    int32_t stage[STAGE];
    int nst;
    int64_t goff;
};

__device__ __forceinline__ void stage_flush(WaveLds& L, int64_t* state, int32_t* sample_idx) {
    if (threadIdx.x == 0)
        L.goff = L.nst ? (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(&state[RS_VALID]),
                                            (unsigned long long)L.nst)
                       : 0;
    __syncthreads();
    for (int i = threadIdx.x; i < L.nst; i += blockDim.x) sample_idx[L.goff + i] = L.stage[i];
    __syncthreads();
    if (threadIdx.x == 0) L.nst = 0;
    __syncthreads();
}

__device__ void render_march_waves(const float* __restrict__ rays_o, const float* __restrict__ rays_d,
                                   float* __restrict__ hits_t, const MarchParams& p, WordCache& wc,
                                   int64_t* __restrict__ state, int64_t n_alive, int Ns,
                                   const int32_t* __restrict__ alive, float* __restrict__ xyzs,
                                   float* __restrict__ dirs, float* __restrict__ deltas, float* __restrict__ ts,
                                   int32_t* __restrict__ n_eff, int32_t* __restrict__ sample_idx, WaveLds& L) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float dt = NGP_SQRT3 / p.max_samples;
    if (threadIdx.x == 0) L.nst = 0;
    __syncthreads();
    for (int64_t b0 = (int64_t)blockIdx.x * 4; b0 < n_alive; b0 += (int64_t)gridDim.x * 4) {  // block-uniform
        const int64_t n = b0 + w;
        if (n < n_alive) {
            const int64_t r = alive[n];
            float o[3], d[3], dinv[3];
            load_ray(rays_o, rays_d, r, o, d, dinv);
            const float t0 = hits_t[2 * r], t2 = hits_t[2 * r + 1];
            int N = 0;
            bool near = t0 < t2;  // raymarching.cu:366 loop condition at entry
            if (near && wc.dil) {
                // exact early out (march_slots_wave_kernel): no occupied block
                // within one block of the segment -> the walk emits nothing
                const float mb = fminf(0.5f, p.scale);
                const float dn = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                const float step = 0.45f * (4.0f * 2.0f * mb / p.grid_size) / dn;
                const int npts = (int)ceilf((t2 - t0) / step) + 1;
                const float gm1 = p.grid_size - 1.0f, mbi = 1 / mb;
                bool any = false;
                for (int j0 = 0; j0 < npts && !any; j0 += 64) {
                    const int j = j0 + lane;
                    bool b = false;
                    if (j < npts) {
                        const float t = fminf(t0 + (float)j * step, t2);
                        const float x = o[0] + t * d[0], y = o[1] + t * d[1], z = o[2] + t * d[2];
                        const int nx = (int)clampf(0.5f * (x * mbi + 1) * p.grid_size, 0.0f, gm1);
                        const int ny = (int)clampf(0.5f * (y * mbi + 1) * p.grid_size, 0.0f, gm1);
                        const int nz = (int)clampf(0.5f * (z * mbi + 1) * p.grid_size, 0.0f, gm1);
                        const uint32_t wi = morton3((uint32_t)nx >> 2, (uint32_t)ny >> 2, (uint32_t)nz >> 2);
                        b = (wc.dil[wi >> 5] >> (wi & 31u)) & 1u;
                    }
                    any = __ballot(b) != 0ull;
                }
                near = any;
            }
            if (near) {
                LatSeg& sg = L.segs[w];
                int nseg = 0;
                const int k_end = t0 >= 0 ? lat_build(t0, t2, dt, sg, nseg, lane == 0) : -1;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (k_end < 0) {  // table overflow: the serial walk on lane 0
                    if (lane == 0) {
                        float t = t0, x, y, z, dts, t_emit = t0;
                        while (t < t2 && N < Ns) {
                            const float tc = t;
                            if (march_step<true>(t, o, d, dinv, p, x, y, z, dts, wc)) {
                                t_emit = t;
                                const int64_t q = N * n_alive + n;
                                xyzs[3 * q] = x; xyzs[3 * q + 1] = y; xyzs[3 * q + 2] = z;
                                dirs[3 * q] = d[0]; dirs[3 * q + 1] = d[1]; dirs[3 * q + 2] = d[2];
                                ts[q] = tc;
                                deltas[q] = dts;
                                N++;
                            }
                        }
                        if (N) hits_t[2 * r] = t_emit;
                    }
                    N = __builtin_amdgcn_readfirstlane(N);
                } else {
                    int c = 0, q0 = 0;
                    while (c < k_end && N < Ns) {
                        while (q0 + 1 < nseg && c >= sg.K[q0 + 1]) ++q0;
                        const int k = c + lane;
                        int q = q0;
                        while (q + 1 < nseg && k >= sg.K[q + 1]) ++q;
                        const bool live = k < k_end;
                        const float tk = live ? lat_t(sg, q, k) : 0.f;
                        bool occ = false;
                        int nxt = k_end;
                        float x = 0.f, y = 0.f, z = 0.f;
                        if (live) {
                            float dts, T;
                            occ = march_probe<true>(tk, o, d, dinv, p, x, y, z, dts, wc, T);
                            nxt = occ ? k + 1 : lat_jump(sg, nseg, q, k, T, k_end);
                        }
                        const uint64_t occm = __ballot(occ && live);
                        int J[6];
                        J[0] = live ? min(nxt - c, 64) : 64;
#pragma unroll
                        for (int b = 1; b < 6; ++b) {
                            const int prev = J[b - 1];
                            const int v = __builtin_amdgcn_ds_bpermute(min(prev, 63) << 2, prev);
                            J[b] = prev >= 64 ? 64 : v;
                        }
                        int cur = 0;
#pragma unroll
                        for (int b = 5; b >= 0; --b) {
                            const int v = __builtin_amdgcn_ds_bpermute(min(cur, 63) << 2, J[b]);
                            const int to = cur >= 64 ? 64 : v;
                            if (to <= lane) cur = to;
                        }
                        uint64_t vis = __ballot(cur == lane);
                        const int last = 63 - __builtin_clzll(vis);
                        const int pnt = __builtin_amdgcn_readlane(nxt, last);
                        vis &= occm;
                        const int room = Ns - N;
                        const int nv = __builtin_popcountll(vis);
                        const int ne = min(nv, room);
                        if ((vis >> lane) & 1ull) {
                            const int rank = __builtin_popcountll(vis & ((1ull << lane) - 1ull));
                            if (rank < room) {
                                const int64_t qq = (N + rank) * n_alive + n;
                                xyzs[3 * qq] = x; xyzs[3 * qq + 1] = y; xyzs[3 * qq + 2] = z;
                                dirs[3 * qq] = d[0]; dirs[3 * qq + 1] = d[1]; dirs[3 * qq + 2] = d[2];
                                ts[qq] = tk;
                                deltas[qq] = dt;
                                if (rank == ne - 1) hits_t[2 * r] = tk + dt;  // raymarching.cu:390
                            }
                        }
                        N += ne;
                        c = pnt;
                    }
                }
            }
            int base = 0;
            if (lane == 0) {
                n_eff[n] = N;
                base = N ? atomicAdd(&L.nst, N) : 0;  // LDS
            }
            base = __builtin_amdgcn_readfirstlane(base);
            for (int k = lane; k < N; k += 64) L.stage[base + k] = (int32_t)(k * n_alive + n);
        }
        __syncthreads();
        if (L.nst > STAGE - 4 * 64) stage_flush(L, state, sample_idx);  // block-uniform (read after the barrier)
    }
    stage_flush(L, state, sample_idx);
}

template <bool SIMPLE>
__global__ void __launch_bounds__(256) render_march_kernel(const float* __restrict__ rays_o,
                                                           const float* __restrict__ rays_d,
                                                           float* __restrict__ hits_t, MarchParams p,
                                                           int64_t* __restrict__ state, int parity,
                                                           const int32_t* __restrict__ alive,
                                                           float* __restrict__ xyzs, float* __restrict__ dirs,
                                                           float* __restrict__ deltas, float* __restrict__ ts,
                                                           int32_t* __restrict__ n_eff,
                                                           int32_t* __restrict__ sample_idx, int wave_ns) {
    if (!state[RS_ACTIVE]) return;
    const int64_t n_alive = state[parity];
    const int Ns = (int)state[RS_NS];
    const bool waves = SIMPLE && Ns >= wave_ns;
    // block-uniform, before the barrier
    if ((int64_t)blockIdx.x * (waves ? 4 : blockDim.x) >= n_alive) return;
    extern __shared__ uint32_t ssum[];
    WordCache wc;
    wc.sum = load_summary(p, ssum);
    wc.dil = wc.sum ? wc.sum + p.n_sum32 : nullptr;
    __syncthreads();
    if constexpr (SIMPLE) {
        if (waves) {
            __shared__ WaveLds L;
            render_march_waves(rays_o, rays_d, hits_t, p, wc, state, n_alive, Ns, alive, xyzs, dirs, deltas, ts,
                               n_eff, sample_idx, L);
            return;
        }
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // block-uniform trip count (block_append synchronises the block)
    for (int64_t bbase = (int64_t)blockIdx.x * blockDim.x; bbase < n_alive; bbase += stride) {
        const int64_t n = bbase + threadIdx.x;
        int s = 0;
        if (n < n_alive) {
            const int64_t r = alive[n];
            float o[3], d[3], dinv[3];
            load_ray(rays_o, rays_d, r, o, d, dinv);
            float t = hits_t[2 * r];
            const float t2 = hits_t[2 * r + 1];
            float x, y, z, dt, t_emit = t;
            while (t < t2 && s < Ns) {  // raymarching.cu:366-400
                const float tc = t;
                if (march_step<SIMPLE>(t, o, d, dinv, p, x, y, z, dt, wc)) {
                    t_emit = t;
                    const int64_t q = s * n_alive + n;  // sample-major: lanes' stores coalesce
                    xyzs[3 * q] = x; xyzs[3 * q + 1] = y; xyzs[3 * q + 2] = z;
                    dirs[3 * q] = d[0]; dirs[3 * q + 1] = d[1]; dirs[3 * q + 2] = d[2];
                    ts[q] = tc;
                    deltas[q] = dt;
                    s++;
                }
            }
            if (s) hits_t[2 * r] = t_emit;  // raymarching.cu:390: t after the last emitted sample
            n_eff[n] = s;
        }
        // append the valid slots to the sample list
        const int64_t off = block_append(s, reinterpret_cast<unsigned long long*>(&state[RS_VALID]));
        for (int k = 0; k < s; ++k) sample_idx[off + k] = (int32_t)(k * n_alive + n);
    }
}

__global__ void __launch_bounds__(256) render_composite_kernel(const float* __restrict__ sigmas,
                                                               const float* __restrict__ rgbs,
                                                               const float* __restrict__ deltas,
                                                               const float* __restrict__ ts,
                                                               const int32_t* __restrict__ n_eff,
                                                               int64_t* __restrict__ state, int parity,
                                                               const int32_t* __restrict__ alive_in,
                                                               int32_t* __restrict__ alive_out, float T_thr,
                                                               float* __restrict__ opacity, float* __restrict__ depth,
                                                               float* __restrict__ rgb) {
    if (!state[RS_ACTIVE]) return;
    const int64_t n_alive = state[parity];
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int my_total = 0;
    // CRPT rays per thread per pass (stride 256): one survivor append per
    // 256*CRPT rays (same-address atomics serialise)
    // (only while the alive rays outnumber the grid's threads: late iterations
    // have few rays with many samples each and want one ray per thread)
    const int rpt = n_alive > stride ? CRPT : 1;
    for (int64_t bbase = (int64_t)blockIdx.x * blockDim.x * rpt; bbase < n_alive; bbase += stride * rpt) {
        int32_t kept[CRPT];  // survivor ray or -1 (static indices: registers)
#pragma unroll
        for (int k = 0; k < CRPT; ++k) {  // block-uniform
            kept[k] = -1;
            const int64_t n = bbase + k * blockDim.x + threadIdx.x;
            if (k >= rpt || n >= n_alive) continue;
            const int ne = n_eff[n];
            const int32_t r = alive_in[n];
            my_total += ne;  // total_samples += N_eff_samples.sum() (rendering.py:199)
            if (ne <= 0) continue;  // volumerendering.cu:221-224: no samples -> dead
            bool keep = true;
            float op = opacity[r], dp = depth[r], cr = rgb[3 * r], cg = rgb[3 * r + 1], cb = rgb[3 * r + 2];
            float T = 1 - op;
            for (int s = 0; s < ne; ++s) {  // volumerendering.cu:228-256
                const int64_t o = s * n_alive + n;  // sample-major slots (render_march_kernel)
                const float a = 1.0f - __expf(-sigmas[o] * deltas[o]);
                const float w = a * T;
                cr += w * rgbs[3 * o]; cg += w * rgbs[3 * o + 1]; cb += w * rgbs[3 * o + 2];
                dp += w * ts[o];
                op += w;
                T *= 1.0f - a;
                if (T <= T_thr) { keep = false; break; }
            }
            rgb[3 * r] = cr; rgb[3 * r + 1] = cg; rgb[3 * r + 2] = cb;
            depth[r] = dp;
            opacity[r] = op;
            if (keep) kept[k] = r;
        }
        int cnt[CRPT];
        int64_t off[CRPT];
#pragma unroll
        for (int k = 0; k < CRPT; ++k) cnt[k] = kept[k] >= 0;
        block_append_k(cnt, off, reinterpret_cast<unsigned long long*>(&state[parity ^ 1]));
#pragma unroll
        for (int k = 0; k < CRPT; ++k)
            if (kept[k] >= 0) alive_out[off[k]] = kept[k];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) my_total += __shfl_xor(my_total, o, 64);
    __shared__ int wsum[4];  // one total atomic per block, not per wave
    if (lane == 0) wsum[threadIdx.x >> 6] = my_total;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (tot) atomicAdd(reinterpret_cast<unsigned long long*>(&state[RS_TOTAL]), (unsigned long long)tot);
    }
}

// rendering.py:240-251: rgb += bg * (1 - opacity)
__global__ void __launch_bounds__(256) render_finish_kernel(const float* __restrict__ opacity, int64_t n_rays, float b0,
                                                            float b1, float b2, float* __restrict__ rgb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_rays) return;
    const float m = 1 - opacity[i];
    rgb[3 * i] += b0 * m; rgb[3 * i + 1] += b1 * m; rgb[3 * i + 2] += b2 * m;
}

}  // namespace ngp

using namespace ngp;

static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

extern "C" {

int64_t ngp_render_test_capacity(int64_t n_rays, int min_samples) {
    if (n_rays < 0 || min_samples < 1) return -1;
    // N_alive * N_samples <= max(N_rays, N_alive * min_samples) <= N_rays * min_samples
    return n_rays * (int64_t)min_samples;
}

int ngp_render_test_begin(int64_t n_rays, int64_t* state, int32_t* alive0, float* opacity, float* depth, float* rgb,
                          void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && n_rays < INT32_MAX && state);
    NGP_CHECK_ARG(n_rays == 0 || (alive0 && opacity && depth && rgb));
    const int64_t n = n_rays > NGP_RENDER_STATE_WORDS ? n_rays : NGP_RENDER_STATE_WORDS;
    render_begin_kernel<<<nblk(n, 256), 256, 0, as_stream(stream)>>>(n_rays, state, alive0, opacity, depth, rgb);
    return ngp_launch_status();
}

int ngp_render_test_march(const float* rays_o, const float* rays_d, float* hits_t, int64_t n_rays,
                          const uint8_t* bitfield, int cascades, int grid_size, float scale, float exp_step_factor,
                          int max_samples, int min_samples, int64_t sample_budget, int parity, int64_t* state,
                          const int32_t* alive, const uint32_t* occ_summary, float* xyzs, float* dirs, float* deltas,
                          float* ts, int32_t* n_eff, int32_t* sample_idx, void* stream) {
    MarchParams p;
    int st = march_params(bitfield, cascades, grid_size, scale, exp_step_factor, max_samples, p);
    if (st) return st;
    st = march_attach_summary(p, occ_summary);
    if (st) return st;
    p.dt_scale = (float)cascades;  // raymarching.cu:370,399 quirk (test time)
    NGP_CHECK_ARG(n_rays >= 0 && n_rays < INT32_MAX && min_samples >= 1 && (parity == 0 || parity == 1) && state);
    NGP_CHECK_ARG(ngp_render_test_capacity(n_rays, min_samples) < INT32_MAX);
    hipStream_t s = as_stream(stream);
    render_iter_kernel<<<1, 64, 0, s>>>(state, parity, n_rays, min_samples, sample_budget);
    if (n_rays == 0) return ngp_launch_status();
    NGP_CHECK_ARG(rays_o && rays_d && hits_t && alive && xyzs && dirs && deltas && ts && n_eff && sample_idx);
    const unsigned blocks = std::min(nblk(n_rays, 256), 2048u);
    const int wave_ns = WAVE_NS;
    if (march_simple(p))
        render_march_kernel<true><<<blocks, 256, march_summary_lds(p), s>>>(
            rays_o, rays_d, hits_t, p, state, parity, alive, xyzs, dirs, deltas, ts, n_eff, sample_idx, wave_ns);
    else
        render_march_kernel<false><<<blocks, 256, march_summary_lds(p), s>>>(
            rays_o, rays_d, hits_t, p, state, parity, alive, xyzs, dirs, deltas, ts, n_eff, sample_idx, wave_ns);
    return ngp_launch_status();
}

int ngp_render_test_composite(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                              const int32_t* n_eff, int64_t n_rays, int parity, int64_t* state,
                              const int32_t* alive_in, int32_t* alive_out, float T_threshold, float* opacity,
                              float* depth, float* rgb, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && (parity == 0 || parity == 1) && state);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(sigmas && rgbs && deltas && ts && n_eff && alive_in && alive_out && alive_in != alive_out &&
                  opacity && depth && rgb);
    const unsigned blocks = std::min(nblk(n_rays, 256 * CRPT), 1024u);
    render_composite_kernel<<<blocks, 256, 0, as_stream(stream)>>>(sigmas, rgbs, deltas, ts, n_eff, state, parity,
                                                                  alive_in, alive_out, T_threshold, opacity, depth,
                                                                  rgb);
    return ngp_launch_status();
}

int ngp_render_test_finish(const float* opacity, int64_t n_rays, const float* bg_rgb, float* rgb, void* stream) {
    NGP_CHECK_ARG(n_rays >= 0 && bg_rgb);
    if (n_rays == 0) return NGP_OK;
    NGP_CHECK_ARG(opacity && rgb);
    render_finish_kernel<<<nblk(n_rays, 256), 256, 0, as_stream(stream)>>>(opacity, n_rays, bg_rgb[0], bg_rgb[1],
                                                                           bg_rgb[2], rgb);
    return ngp_launch_status();
}

}  // extern "C"
