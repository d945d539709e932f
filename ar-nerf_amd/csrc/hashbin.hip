// Binned hash-table backward: dL/dtable without per-sample memory-side
// atomics.  Same result as hash_bwd_kernel (field.hip) / tcnn's
// kernel_grid_backward (the `params.grad` that models/networks.py's
// xyz_encoder receives), up to fp32 rounding/summation order.
//
// Why: gfx950 float atomics execute at the memory side, one 64-byte request
// per touched segment (MI355X_MICROARCH.md "Global float atomics"); the hash
// backward touches ~4 random 16-byte segments per (sample, level), so the
// atomic form runs at the chip's atomic request rate (~20 G/s), far below HBM
// speed.  Here every gradient contribution is moved twice at HBM speed as a
// 16-byte record, summed in LDS, and each table range is written once.
//
//   bucket  = (level l, range of BENT consecutive entries of level l)
//   record  = one (sample, level, y/z corner) = the x-adjacent corner pair:
//             {key = i0 | i1 << 13 | flags, fx, a0, a1} (16 B): i0/i1 are
//             the two corners' entry offsets inside the bucket,
//             a_f = (w_y * w_z) * dL/denc[2l + f]; corner x+c receives
//             (c ? fx : 1 - fx) * a_f.
//   1 count  (hash_count_kernel): records per (tile of TILE samples, bucket),
//            LDS counters, one row per tile -- no global atomics.
//   2 scan   (hash_scan_kernel): per bucket, exclusive prefix over tiles.
//   3 plan   (hash_plan_kernel): bucket regions (prefix of bucket totals)
//            and pass-B work items (chunks of <= CH records per bucket).
//   4 write  (hash_write_kernel): recompute each record and store it at its
//            slot of the bucket's contiguous region (counting sort).
//   5 accum  (hash_accum_kernel): one workgroup per chunk streams its records
//            into an fp64 LDS image of the range (BENT x 2 x 8 B = 128 KB;
//            ds_add_f64 runs ~9x the rate of ds_add_f32 on gfx950, measured
//            by scripts/diag/lds_atomics.py) and
//            writes it out once: a read-add-store when it is the bucket's
//            only chunk and nothing was added to the range directly, else
//            atomic adds of the non-zero entries.
// A dense-level pair split by a bucket boundary adds its x+1 corner with a
// global atomic (and flags the bucket); samples beyond the workspace capacity
// take the per-sample atomic path (and flag every bucket): exact either way.
//
// Run merging (levels of merge_mask, the coarse ones): consecutive samples of
// a ray share a level's cell for dt * res_l < 1 (40 samples per cell at level
// 0, ~6 at level 7 on Lego), i.e. the same (x, x+1) corner pair per y/z
// corner.  Lanes 4 apart in a wave hold consecutive samples of the same y/z
// corner, so the write kernel sums each run of equal pairs in registers
// (segmented suffix sums, as the accumulation does) and its head emits two
// single-entry records {i | F_SINGLE, sum_x, sum_y, 0} -- one per corner of
// the pair, each in its own bucket (no split pair) -- for the whole run; a
// run of one sample emits its pair record as usual.  Records per
// (sample, level) stay <= 4 (a run of L >= 2 samples emits 2), and the count
// kernel makes the same run decisions from the same keys.
#pragma clang fp contract(off)

#include "common.h"
#include "grid.h"

namespace ngp {

// entries per bucket (fp64 LDS image: 2 x BENT x 8 B = 128 KB, one accumulating workgroup per CU;
// 4096-entry buckets at two per CU measured the same accumulation time and a slower count pass)
constexpr int BSHIFT = 13, BENT = 1 << BSHIFT;
constexpr int NBL = (1 << 19) / BENT;            // bucket slots per level (2^19 / BENT)
// accumulation workgroup: 8192-entry buckets (128 KB LDS, one per CU) take
// 1024 threads, 4096-entry buckets (64 KB, two per CU) 512, so that a
// thread covers 4 float4 groups of its bucket either way (PF below)
constexpr int ACC_T = BENT / 8;
constexpr int NSLOT = L * NBL;                   // (level, bucket) slots per tile row
constexpr int MAXB = 2048;                       // buckets over all levels
constexpr int TILE = 256;                        // samples per count/write tile
constexpr int RPT = TILE * 4 / 256;              // records per thread per level
constexpr uint32_t CH = 32768;                   // records per pass-5 chunk
constexpr uint32_t IB_CAP = 8192;                // items with a direct item -> bucket entry
constexpr uint32_t F_C0 = 1u << 28;              // record carries corner x only (pair split)
constexpr uint32_t F_SINGLE = 1u << 29;          // record {i0 | F_SINGLE, g0, g1, 0}: one entry, summed run

struct BinArgs {
    int lo;                 // levels [lo, L) are binned (the others have no buckets)
    uint32_t merge;         // bit l: runs of equal corner pairs are merged at level l
    uint32_t bbase[L + 1];  // first bucket of level l
    int64_t tiles_cap;      // tiles the workspace holds
};

struct BinWs {
    uint32_t* fb;      // [MAXB + 1]: 1 if direct adds hit bucket b; [MAXB]: a tile spilled
    uint32_t* tot;     // [MAXB] records per bucket
    uint32_t* rstart;  // [MAXB + 1] bucket region starts
    uint32_t* items;   // [MAXB + 1] chunk prefix
    uint32_t* ib;      // [IB_CAP] item -> its bucket (the accumulation's lookup; binary search beyond)
    uint32_t* ofs;     // [NSLOT][tiles_cap] counts, then exclusive offsets over tiles
    uint4* rec;        // [tiles_cap * TILE * 4 * L]
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static size_t bin_ws_bytes(int64_t tiles, BinWs* w, void* base) {
    const size_t o_fb = 0, o_tot = align256((MAXB + 1) * 4), o_rs = o_tot + align256(MAXB * 4),
                 o_it = o_rs + align256((MAXB + 1) * 4), o_ib = o_it + align256((MAXB + 1) * 4),
                 o_ofs = o_ib + align256(IB_CAP * 4);
    const size_t o_rec = align256(o_ofs + (size_t)tiles * NSLOT * 4);
    const size_t total = o_rec + (size_t)tiles * TILE * 4 * L * sizeof(uint4);
    if (w) {
        char* b = reinterpret_cast<char*>(base);
        w->fb = reinterpret_cast<uint32_t*>(b + o_fb);
        w->tot = reinterpret_cast<uint32_t*>(b + o_tot);
        w->rstart = reinterpret_cast<uint32_t*>(b + o_rs);
        w->items = reinterpret_cast<uint32_t*>(b + o_it);
        w->ib = reinterpret_cast<uint32_t*>(b + o_ib);
        w->ofs = reinterpret_cast<uint32_t*>(b + o_ofs);
        w->rec = reinterpret_cast<uint4*>(b + o_rec);
    }
    return total;
}

__device__ __forceinline__ void add_pair_direct(float* __restrict__ grad, uint32_t e, float w, float a0, float a1) {
    atomicAdd(grad + 2 * (size_t)e, w * a0);
    atomicAdd(grad + 2 * (size_t)e + 1, w * a1);
}

// One record of sample (in, gd) at level l, y/z corner (cy, cz): the two
// x-adjacent corners' entries of the level and the factors of their weights.
struct Rec {
    uint32_t e0, e1;
    float fx, a0, a1;
};

__device__ __forceinline__ Rec make_rec(const float in[3], float2 gd, int cy, int cz, const LevelLds& lv, int l) {
    const float sc = lv.scale[l];
    const uint32_t res = lv.res[l], size = lv.size[l];
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
    const float wyz = (cy ? pos[1] : 1 - pos[1]) * (cz ? pos[2] : 1 - pos[2]);
    Rec r;
    r.fx = pos[0];
    r.a0 = wyz * gd.x;
    r.a1 = wyz * gd.y;
    r.e0 = corner_index(pg[0], pg[1] + cy, pg[2] + cz, res, size, dense, pow2);
    r.e1 = corner_index(pg[0] + 1, pg[1] + cy, pg[2] + cz, res, size, dense, pow2);
    return r;
}

// Run structure of one level across the wave: lanes 4 apart hold consecutive
// samples of one y/z corner.  head: the lane starts a run of equal (e0, e1)
// (lanes 0-3, an invalid lane or its successor, a changed pair); longrun: a
// head whose run continues to lane + 4.
struct RunInfo {
    bool head, longrun;
    uint64_t heads;
};
__device__ __forceinline__ RunInfo run_info(bool valid, uint32_t e0, uint32_t e1) {
    const int lane = threadIdx.x & 63;
    const uint32_t k0 = valid ? e0 : 0xffffffffu, k1 = valid ? e1 : (0xfffffff0u | (uint32_t)lane);
    const uint32_t p0 = __shfl_up(k0, 4, 64), p1 = __shfl_up(k1, 4, 64);
    RunInfo r;
    r.head = lane < 4 || !valid || p0 != k0 || p1 != k1;
    r.heads = __ballot(r.head);
    r.longrun = r.head && valid && lane + 4 < 64 && !((r.heads >> (lane + 4)) & 1ull);
    return r;
}

__device__ __forceinline__ void tile_inputs(const float* __restrict__ xyzs, const int32_t* __restrict__ sidx,
                                            const GridArgs& ga, int64_t j0, int64_t N, float in[RPT][3],
                                            bool valid[RPT]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int64_t j = j0 + k * 64 + (t >> 2);
        valid[k] = j < N;
        const int64_t i = valid[k] && sidx ? (int64_t)sidx[j] : j;
        load_x01(xyzs, i, valid[k], ga, in[k]);
    }
}

__global__ void __launch_bounds__(256) hash_count_kernel(const float* __restrict__ xyzs, int64_t n,
                                                         const int64_t* __restrict__ n_dev,
                                                         const int32_t* __restrict__ sidx, GridArgs ga, BinArgs ba,
                                                         BinWs ws) {
    __shared__ LevelLds lv;
    __shared__ uint32_t cnt[NSLOT];
    NGP_PROBE_BEGIN(NGP_P_HASH_COUNT);
    load_levels(ga, lv);
    const int64_t N = ngp_capped_count(n_dev, n);  // (a device count never past the capacity: a guard hit)
    const int64_t ntiles = min((N + TILE - 1) / TILE, ba.tiles_cap);
    const int t = threadIdx.x, yz = t & 3, cy = yz & 1, cz = yz >> 1;
    const float2 g0 = make_float2(0.f, 0.f);
    // the bucket flags are set by hash_write_kernel (a later launch): clear them here
    if (blockIdx.x == 0)
        for (int i = t; i <= MAXB; i += blockDim.x) ws.fb[i] = 0u;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int i = t; i < NSLOT; i += 256) cnt[i] = 0;
        __syncthreads();
        float in[RPT][3];
        bool valid[RPT];
        tile_inputs(xyzs, sidx, ga, tile * TILE, N, in, valid);
#pragma unroll 1
        for (int l = ba.lo; l < L; ++l) {
            const bool merge = (ba.merge >> l) & 1u;
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                const Rec r = make_rec(in[k], g0, cy, cz, lv, l);
                if (merge) {  // the write kernel's run decisions, from the same keys
                    const RunInfo ri = run_info(valid[k], r.e0, r.e1);
                    if (!valid[k] || !ri.head) continue;
                    atomicAdd(&cnt[l * NBL + (r.e0 >> BSHIFT)], 1u);
                    if (ri.longrun) atomicAdd(&cnt[l * NBL + (r.e1 >> BSHIFT)], 1u);
                    continue;
                }
                if (!valid[k]) continue;
                atomicAdd(&cnt[l * NBL + (r.e0 >> BSHIFT)], 1u);
            }
        }
        __syncthreads();
        for (int i = t; i < NSLOT; i += 256) ws.ofs[(size_t)i * ba.tiles_cap + tile] = cnt[i];
        __syncthreads();
    }
    NGP_PROBE_END();
}

// one workgroup per (level, bucket) slot: exclusive prefix over tiles in place
__global__ void __launch_bounds__(256) hash_scan_kernel(const int64_t* __restrict__ n_dev, int64_t n, BinArgs ba,
                                                        BinWs ws) {
    __shared__ uint32_t wsum[4];
    const int slot = blockIdx.x, l = slot / NBL, lb = slot % NBL;
    if (lb >= (int)(ba.bbase[l + 1] - ba.bbase[l])) return;
    const int64_t N = ngp_capped_count(n_dev, n);  // (a device count never past the capacity: a guard hit)
    const int64_t ntiles = min((N + TILE - 1) / TILE, ba.tiles_cap);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t carry = 0;
    for (int64_t c0 = 0; c0 < ntiles; c0 += 256) {
        const int64_t tile = c0 + t;
        uint32_t* p = ws.ofs + (size_t)slot * ba.tiles_cap + tile;
        const uint32_t v = tile < ntiles ? *p : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t before = carry;
        for (int i = 0; i < w; ++i) before += wsum[i];
        const uint32_t blk = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (tile < ntiles) *p = before + x - v;
        carry += blk;
        __syncthreads();
    }
    if (t == 0) ws.tot[ba.bbase[l] + lb] = carry;
}

// bucket regions + chunk items (one workgroup of MAXB / 2 threads, two buckets each)
__global__ void __launch_bounds__(MAXB / 2) hash_plan_kernel(uint32_t nbt, BinWs ws) {
    __shared__ uint32_t a[MAXB / 2], c[MAXB / 2];
    NGP_PROBE_BEGIN(NGP_P_HASH_PLAN);
    const uint32_t t = threadIdx.x, b0 = 2 * t, b1 = 2 * t + 1;
    const uint32_t t0 = b0 < nbt ? ws.tot[b0] : 0u, t1 = b1 < nbt ? ws.tot[b1] : 0u;
    const uint32_t c0 = (t0 + CH - 1) / CH, c1 = (t1 + CH - 1) / CH;
    a[t] = t0 + t1;
    c[t] = c0 + c1;
    __syncthreads();
    for (uint32_t o = 1; o < MAXB / 2; o <<= 1) {  // Hillis-Steele inclusive scans over bucket pairs
        const uint32_t va = t >= o ? a[t - o] : 0u, vc = t >= o ? c[t - o] : 0u;
        __syncthreads();
        a[t] += va;
        c[t] += vc;
        __syncthreads();
    }
    ws.rstart[b0 + 1] = a[t] - t1;
    ws.rstart[b1 + 1] = a[t];
    ws.items[b0 + 1] = c[t] - c1;
    ws.items[b1 + 1] = c[t];
    if (t == 0) { ws.rstart[0] = 0; ws.items[0] = 0; }
    // item -> bucket table (one entry per chunk; usually one chunk per bucket)
    for (uint32_t it = c[t] - c1 - c0; it < c[t] - c1 && it < IB_CAP; ++it) ws.ib[it] = b0;
    for (uint32_t it = c[t] - c1; it < c[t] && it < IB_CAP; ++it) ws.ib[it] = b1;
    NGP_PROBE_END();
}

// MODE bits: 2 = store each record from registers at its rank (the product
// path: measured faster than staging a level's records in LDS and writing
// bucket runs, MODE 0); 1 (no record stores) and 4 (no LDS rank atomics) are
// diagnostic variants for scripts/diag.
template <int MODE>
__global__ void __launch_bounds__(256) hash_write_kernel(const float* __restrict__ xyzs, int64_t n,
                                                         const int64_t* __restrict__ n_dev,
                                                         const int32_t* __restrict__ sidx, GridArgs ga, BinArgs ba,
                                                         const float* __restrict__ denc, float* __restrict__ grad,
                                                         BinWs ws) {
    static_assert((MODE & 2) || NBL == 64, "MODE 0 (diagnostics) scans one wave of buckets");
    __shared__ LevelLds lv;
    __shared__ uint32_t base[NSLOT];          // this tile's first slot in each bucket region
    __shared__ uint32_t hist2[2][NBL], loff[NBL + 1];  // MODE 0: one level's counts
    __shared__ uint4 stage[TILE * 4];         // MODE 0: one level's records, sorted by bucket
    __shared__ uint8_t sbk[TILE * 4];
    // MODE 2 ranks every level's records in its own counters (reusing stage[]'s
    // LDS), cleared once per tile: the level loop then has no barrier, so a wave
    // does not wait at every level for the block's slowest wave
    uint32_t* const hall = reinterpret_cast<uint32_t*>(stage);
    static_assert(sizeof(stage) >= NSLOT * sizeof(uint32_t), "stage[] holds the per-level counters");
    NGP_PROBE_BEGIN(NGP_P_HASH_WRITE);
    load_levels(ga, lv);
    const int64_t N = ngp_capped_count(n_dev, n);  // (a device count never past the capacity: a guard hit)
    const int64_t ntiles = (N + TILE - 1) / TILE;
    const int t = threadIdx.x, yz = t & 3, cy = yz & 1, cz = yz >> 1;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const bool spill = tile >= ba.tiles_cap;  // no room: per-sample atomics for this tile
        if (spill && t == 0) ws.fb[MAXB] = 1u;
        if (!spill) {
            for (int i = t; i < NSLOT; i += 256) {
                const int l = i / NBL, lb = i % NBL;
                base[i] = lb < (int)(ba.bbase[l + 1] - ba.bbase[l])
                              ? ws.rstart[ba.bbase[l] + lb] + ws.ofs[(size_t)i * ba.tiles_cap + tile]
                              : 0u;
                if (MODE & 2) hall[i] = 0;
            }
        }
        float in[RPT][3];
        bool valid[RPT];
        const int64_t j0 = tile * TILE;
        tile_inputs(xyzs, sidx, ga, j0, N, in, valid);
        float2 gd[RPT], gn[RPT];
#pragma unroll
        for (int k = 0; k < RPT; ++k)
            gd[k] = valid[k] ? *reinterpret_cast<const float2*>(denc + (j0 + k * 64 + (t >> 2)) * 32 + 2 * ba.lo)
                             : float2{0.f, 0.f};
        if (MODE & 2) __syncthreads();  // base[], hall[] ready
#pragma unroll 1
        for (int l = ba.lo; l < L; ++l) {
            uint32_t* hist = (MODE & 2) ? hall + l * NBL : hist2[l & 1];
            if (!(MODE & 2)) {
                if (t < NBL) hist[t] = 0;
                __syncthreads();  // also: base[] ready; previous level's stage[] reads done
            }
#pragma unroll
            for (int k = 0; k < RPT; ++k)  // next level's dL/denc, loaded ahead
                gn[k] = valid[k] && l + 1 < L
                            ? *reinterpret_cast<const float2*>(denc + (j0 + k * 64 + (t >> 2)) * 32 + 2 * (l + 1))
                            : float2{0.f, 0.f};
            const uint32_t off = lv.off[l];
            uint4 rec[RPT];
            uint32_t slot[RPT];  // bucket << 16 | rank in the tile's run, or ~0u
            if ((ba.merge >> l) & 1u) {  // run-merged level (wave-uniform branch)
#pragma unroll
                for (int k = 0; k < RPT; ++k) {
                    const Rec r = make_rec(in[k], gd[k], cy, cz, lv, l);
                    const RunInfo ri = run_info(valid[k], r.e0, r.e1);
                    const int lane = t & 63;
                    // the fp32 products tcnn adds, summed over the run (segmented suffix sums)
                    float v00 = (1 - r.fx) * r.a0, v01 = (1 - r.fx) * r.a1, v10 = r.fx * r.a0, v11 = r.fx * r.a1;
                    if (ri.heads != ~0ull) {
#pragma unroll
                        for (int o4 = 4; o4 < 64; o4 <<= 1) {
                            const float d00 = __shfl_down(v00, o4, 64), d01 = __shfl_down(v01, o4, 64);
                            const float d10 = __shfl_down(v10, o4, 64), d11 = __shfl_down(v11, o4, 64);
                            const uint64_t span = ((0x1111111111111111ull & ((2ull << o4) - 1ull)) & ~1ull) << lane;
                            if (lane + o4 < 64 && (ri.heads & span) == 0) {
                                v00 += d00; v01 += d01; v10 += d10; v11 += d11;
                            }
                        }
                    }
                    if (!valid[k] || !ri.head) continue;
                    if (spill) {
                        atomicAdd(grad + 2 * (size_t)(off + r.e0), v00);
                        atomicAdd(grad + 2 * (size_t)(off + r.e0) + 1, v01);
                        atomicAdd(grad + 2 * (size_t)(off + r.e1), v10);
                        atomicAdd(grad + 2 * (size_t)(off + r.e1) + 1, v11);
                        continue;
                    }
                    const uint32_t b0 = r.e0 >> BSHIFT, b1 = r.e1 >> BSHIFT;
                    if (ri.longrun) {
                        const uint4 q0 = make_uint4((r.e0 & (BENT - 1)) | F_SINGLE, __float_as_uint(v00),
                                                    __float_as_uint(v01), 0u);
                        const uint4 q1 = make_uint4((r.e1 & (BENT - 1)) | F_SINGLE, __float_as_uint(v10),
                                                    __float_as_uint(v11), 0u);
                        ws.rec[base[l * NBL + b0] + atomicAdd(&hist[b0], 1u)] = q0;
                        ws.rec[base[l * NBL + b1] + atomicAdd(&hist[b1], 1u)] = q1;
                        continue;
                    }
                    uint32_t key = (r.e0 & (BENT - 1)) | ((r.e1 & (BENT - 1)) << BSHIFT);
                    if (b1 != b0) {  // pair split by a bucket boundary: corner x+1 goes direct
                        key |= F_C0;
                        add_pair_direct(grad, off + r.e1, r.fx, r.a0, r.a1);
                        ws.fb[ba.bbase[l] + b1] = 1u;
                    }
                    ws.rec[base[l * NBL + b0] + atomicAdd(&hist[b0], 1u)] =
                        make_uint4(key, __float_as_uint(r.fx), __float_as_uint(r.a0), __float_as_uint(r.a1));
                }
#pragma unroll
                for (int k = 0; k < RPT; ++k) gd[k] = gn[k];
                continue;
            }
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                slot[k] = ~0u;
                if (!valid[k]) continue;
                const Rec r = make_rec(in[k], gd[k], cy, cz, lv, l);
                if (spill) {
                    add_pair_direct(grad, off + r.e0, 1 - r.fx, r.a0, r.a1);
                    add_pair_direct(grad, off + r.e1, r.fx, r.a0, r.a1);
                    continue;
                }
                const uint32_t b0 = r.e0 >> BSHIFT, b1 = r.e1 >> BSHIFT;
                uint32_t key = (r.e0 & (BENT - 1)) | ((r.e1 & (BENT - 1)) << BSHIFT);
                if (b1 != b0) {  // pair split by a bucket boundary: corner x+1 goes direct
                    key |= F_C0;
                    add_pair_direct(grad, off + r.e1, r.fx, r.a0, r.a1);
                    ws.fb[ba.bbase[l] + b1] = 1u;  // idempotent flag
                }
                rec[k] = make_uint4(key, __float_as_uint(r.fx), __float_as_uint(r.a0), __float_as_uint(r.a1));
                slot[k] = (b0 << 16) | ((MODE & 4) ? (uint32_t)(t & 15) : atomicAdd(&hist[b0], 1u));
            }
#pragma unroll
            for (int k = 0; k < RPT; ++k) gd[k] = gn[k];
            if (spill) continue;
            if (MODE & 2) {
#pragma unroll
                for (int k = 0; k < RPT; ++k)
                    if (slot[k] != ~0u && !(MODE & 1))
                        ws.rec[base[l * NBL + (slot[k] >> 16)] + (slot[k] & 0xffffu)] = rec[k];
                continue;
            }
            __syncthreads();
            if (t < 64) {  // exclusive scan of the tile's per-bucket counts (MODE 0, diagnostics: NBL <= 64)
                const uint32_t h = hist[t];
                uint32_t x = h;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(x, o, 64);
                    if (t >= o) x += y;
                }
                loff[t] = x - h;
                if (t == 63) loff[NBL] = x;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                if (slot[k] == ~0u) continue;
                const uint32_t bb = slot[k] >> 16, r = loff[bb] + (slot[k] & 0xffffu);
                stage[r] = rec[k];
                sbk[r] = (uint8_t)bb;
            }
            __syncthreads();
            // runs of one bucket are contiguous in both stage[] and the region
            const uint32_t nrec = loff[NBL];
            for (uint32_t r = t; r < nrec; r += 256) {
                const uint32_t bb = sbk[r];
                if (!(MODE & 1)) ws.rec[base[l * NBL + bb] + (r - loff[bb])] = stage[r];
                else if (stage[r].x == 0xdeadbeefu) ws.fb[0] = 2u;  // keeps the staging live
            }
        }
        __syncthreads();
    }
    NGP_PROBE_END();
}

// A bucket whose summed gradient one workgroup owns: a single chunk, no
// workspace overflow.  With FUSED the accumulation applies Adam to such a
// bucket straight from its LDS image (plus, for a bucket flagged in fb[], the
// direct adds the record write made into its range, read back from memory:
// the same fp32 sum the flush's atomic would form) and
// hash_adam_residual_kernel steps every other bucket from memory.
__device__ __forceinline__ bool fused_bucket(const BinWs& ws, uint32_t b, bool overflow) {
    return !overflow && ws.items[b + 1] - ws.items[b] <= 1u;
}

__device__ __forceinline__ uint32_t bucket_level(const BinArgs& ba, uint32_t b) {
    int l = 0;
    while (l < L - 1 && b >= ba.bbase[l + 1]) ++l;
    return (uint32_t)l;
}

// Adam over params [4e, 4e+4) of a bucket range (entries 2e, 2e+1 x 2 features)
// with gradient g (already x grad_scale) and the state P, M, V already loaded;
// same arithmetic as adam_kernel.
__device__ __forceinline__ void adam4_regs(const AdamArgs& a, size_t base, uint32_t e, float4 g, float4 P, float4 M,
                                           float4 V, float lr, float bc1, float bc2) {
    adam_elem(P.x, M.x, V.x, g.x, lr, a.b1, a.b2, a.eps, bc1, bc2);
    adam_elem(P.y, M.y, V.y, g.y, lr, a.b1, a.b2, a.eps, bc1, bc2);
    adam_elem(P.z, M.z, V.z, g.z, lr, a.b1, a.b2, a.eps, bc1, bc2);
    adam_elem(P.w, M.w, V.w, g.w, lr, a.b1, a.b2, a.eps, bc1, bc2);
    reinterpret_cast<float4*>(a.p + base)[e] = P;
    reinterpret_cast<float4*>(a.m + base)[e] = M;
    reinterpret_cast<float4*>(a.v + base)[e] = V;
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    reinterpret_cast<h4*>(a.p16 + base)[e] = h4{(_Float16)P.x, (_Float16)P.y, (_Float16)P.z, (_Float16)P.w};
}

__device__ __forceinline__ void adam4(const AdamArgs& a, size_t base, uint32_t e, float4 g, float lr, float bc1,
                                      float bc2) {
    adam4_regs(a, base, e, g, reinterpret_cast<const float4*>(a.p + base)[e],
               reinterpret_cast<const float4*>(a.m + base)[e], reinterpret_cast<const float4*>(a.v + base)[e], lr, bc1,
               bc2);
}

// (diagnostics only: scripts/diag/accum_phases.hip stamps an item's phases; empty in the product build)
#ifndef NGP_ACC_PHASE
#define NGP_ACC_PHASE(k)
#endif
template <bool FUSED = false>
__global__ void __launch_bounds__(ACC_T) hash_accum_kernel(GridArgs ga, BinArgs ba, uint32_t nbt,
                                                          float* __restrict__ grad, BinWs ws, AdamArgs adam,
                                                          uint32_t b_lo, uint32_t b_hi) {
    // buckets [b_lo, b_hi) (a level range; all buckets: 0, nbt)
    extern __shared__ __attribute__((aligned(16))) double img[];  // [2][BENT]: feature-major, 8-byte stride
    NGP_PROBE_BEGIN(NGP_P_HASH_ACCUM);
    const uint32_t total = ws.items[b_hi];
    const int t = threadIdx.x, lane = t & 63;
    const bool overflow = ws.fb[MAXB] != 0;
    float lr = 0.f, bc1 = 1.f, bc2 = 1.f;
    if (FUSED) adam_bias(adam.lr_dev, adam.step_dev, adam.b1, adam.b2, lr, bc1, bc2);
    for (uint32_t it = ws.items[b_lo] + blockIdx.x; it < total; it += gridDim.x) {
        NGP_ACC_PHASE(0);
        uint32_t lo = b_lo, hi = b_hi;  // bucket b: items[b] <= it < items[b + 1]
        if (it < IB_CAP) {  // (the plan's item -> bucket table: one load, not a dependent search)
            lo = ws.ib[it];
        } else {
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (ws.items[mid] <= it) lo = mid; else hi = mid;
            }
        }
        const uint32_t b = lo, c = it - ws.items[b], nch = ws.items[b + 1] - ws.items[b];
        int l = 0;
        while (l < L - 1 && b >= ba.bbase[l + 1]) ++l;
        const uint32_t lb = b - ba.bbase[l];
        const uint32_t ne = min((uint32_t)BENT, ga.g.sizes[l] - (lb << BSHIFT));
        const size_t gbase = 2 * ((size_t)ga.g.offsets[l] + ((size_t)lb << BSHIFT));
        const bool own = nch == 1 && !overflow && ws.fb[b] == 0;
        const bool fz = FUSED && nch == 1 && !overflow;  // fused_bucket
        const bool flagged = ws.fb[b] != 0;               // direct adds in the range
        NGP_ACC_PHASE(1);
        const uint32_t ng = 2 * ne / 4;  // float4 groups of the range
        for (uint32_t e = t; e < 2 * BENT / 2; e += blockDim.x)
            reinterpret_cast<double2*>(img)[e] = make_double2(0.0, 0.0);
        __syncthreads();
        NGP_ACC_PHASE(2);
        const uint32_t r0 = ws.rstart[b] + c * CH, r1 = min(ws.rstart[b + 1], r0 + CH);
        constexpr int U = FUSED ? 2 : 4;  // records in flight per thread (FUSED: registers hold the Adam state)
        // software-pipelined: the next iteration's records are loaded before
        // this iteration's are summed (one load latency per item, not per pass)
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t q = r0 + t + u * blockDim.x;
            v[u] = q < r1 ? ws.rec[q] : make_uint4(0u, 0u, 0u, 0u);
        }
        for (uint32_t q0 = r0 + t; q0 < r1; q0 += U * blockDim.x) {
            uint4 vn[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t q = q0 + (U + u) * blockDim.x;
                vn[u] = q < r1 ? ws.rec[q] : make_uint4(0u, 0u, 0u, 0u);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t q = q0 + u * blockDim.x;
                const uint32_t key = v[u].x, i0 = key & (BENT - 1), i1 = (key >> BSHIFT) & (BENT - 1);
                const float fx = __uint_as_float(v[u].y), a0 = __uint_as_float(v[u].z), a1 = __uint_as_float(v[u].w);
                const float w0 = 1 - fx;
                // the fp32 products tcnn would add, summed in fp64; a single-entry
                // record {i0 | F_SINGLE, g0, g1} carries a run's sums for entry i0
                const bool single = key & F_SINGLE;
                const bool c1 = !(key & (F_C0 | F_SINGLE));
                double p00 = single ? (double)fx : (double)(w0 * a0), p01 = single ? (double)a0 : (double)(w0 * a1);
                double p10 = c1 ? (double)(fx * a0) : 0.0, p11 = c1 ? (double)(fx * a1) : 0.0;
                // Runs: records 4 apart in a wave are the same y/z corner of
                // consecutive samples (a ray's), which on coarse levels often
                // share both entries -- sum such runs in registers first
                // (segmented suffix sum at lane stride 4), one LDS add per run.
                const bool pad = q >= r1;
                const uint32_t kk = pad ? 0xf0000000u | lane : key;
                const uint32_t prev = __shfl_up(kk, 4, 64);
                const bool head = lane < 4 || prev != kk;
                const uint64_t heads = __ballot(head);
                if (heads != ~0ull) {
#pragma unroll
                    for (int o4 = 4; o4 < 64; o4 <<= 1) {
                        const double d00 = __shfl_down(p00, o4, 64), d01 = __shfl_down(p01, o4, 64);
                        const double d10 = __shfl_down(p10, o4, 64), d11 = __shfl_down(p11, o4, 64);
                        const uint64_t span = (0x1111111111111111ull & ((2ull << o4) - 1ull)) & ~1ull;
                        if (lane + o4 < 64 && (heads & (span << lane)) == 0) {
                            p00 += d00; p01 += d01; p10 += d10; p11 += d11;
                        }
                    }
                }
                if (!head || pad) continue;
                atomicAdd(&img[i0], p00);
                atomicAdd(&img[BENT + i0], p01);
                if (c1) {
                    atomicAdd(&img[i1], p10);
                    atomicAdd(&img[BENT + i1], p11);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = vn[u];
        }
        __syncthreads();
        NGP_ACC_PHASE(3);
        float* g = grad + gbase;
        // entries 2e, 2e+1 x features 0, 1 -> grad[4e .. 4e+3]
        auto image4 = [&](uint32_t e) {
            const double2 f0 = reinterpret_cast<const double2*>(img)[e];
            const double2 f1 = reinterpret_cast<const double2*>(img + BENT)[e];
            return make_float4((float)f0.x, (float)f1.x, (float)f0.y, (float)f1.y);
        };
        // the range's whole gradient: this image (+ the direct adds of a flagged bucket, zeroed after)
        auto fused_grad = [&](uint32_t e) {
            float4 v = image4(e);
            if (flagged) {
                float4* g4 = reinterpret_cast<float4*>(g) + e;
                const float4 m = *g4;
                v.x = m.x + v.x; v.y = m.y + v.y; v.z = m.z + v.z; v.w = m.w + v.w;
                *g4 = make_float4(0.f, 0.f, 0.f, 0.f);
            }
            const float sc = adam.grad_scale;
            return make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
        };
        // A fused bucket's Adam state (p, m, v) is read here, at the flush, not
        // prefetched before the records (rounds 3-5 held one to four float4
        // groups of it per thread across the record phase): 93 instead of 105-128
        // VGPRs, so beside these whole-CU blocks (4 waves per SIMD) there is room
        // for the MLP + coarse Adam's and the next batch's round-1 pre-encode's
        // waves (round 5, profiles/r05/ab/round5_ab.txt r5dd-r5ff).
        for (uint32_t e = t; e < ng; e += blockDim.x) {
            if (fz) {
                adam4(adam, gbase, e, fused_grad(e), lr, bc1, bc2);
                continue;
            }
            const float4 v = image4(e);
            if (own) {  // sole writer of this range: read-add-store keeps the += contract
                float4 o = reinterpret_cast<const float4*>(g)[e];
                o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
                reinterpret_cast<float4*>(g)[e] = o;
            } else {
                if (v.x != 0.f) atomicAdd(g + 4 * e, v.x);
                if (v.y != 0.f) atomicAdd(g + 4 * e + 1, v.y);
                if (v.z != 0.f) atomicAdd(g + 4 * e + 2, v.z);
                if (v.w != 0.f) atomicAdd(g + 4 * e + 3, v.w);
            }
        }
        __syncthreads();
        NGP_ACC_PHASE(4);
    }
    if (FUSED) {  // buckets without records: Adam with a zero gradient (moments still decay)
        for (uint32_t b = b_lo + blockIdx.x; b < b_hi; b += gridDim.x) {
            if (ws.tot[b] != 0u || !fused_bucket(ws, b, overflow)) continue;
            const uint32_t l = bucket_level(ba, b), lb = b - ba.bbase[l];
            const uint32_t ne = min((uint32_t)BENT, ga.g.sizes[l] - (lb << BSHIFT));
            const size_t gbase = 2 * ((size_t)ga.g.offsets[l] + ((size_t)lb << BSHIFT));
            const bool flagged = ws.fb[b] != 0;  // direct adds only
            float4* g4 = reinterpret_cast<float4*>(grad + gbase);
            for (uint32_t e = t; e < 2 * ne / 4; e += blockDim.x) {
                float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (flagged) {
                    const float sc = adam.grad_scale;
                    const float4 m = g4[e];
                    gv = make_float4(m.x * sc, m.y * sc, m.z * sc, m.w * sc);
                    g4[e] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                adam4(adam, gbase, e, gv, lr, bc1, bc2);
            }
        }
    }
    NGP_PROBE_END();
}

// Adam (+ gradient zeroing) of the binned buckets the fused accumulation did
// not step: one workgroup per bucket, from the gradient in memory.
__global__ void __launch_bounds__(256) hash_adam_residual_kernel(GridArgs ga, BinArgs ba, uint32_t nbt,
                                                                  float* __restrict__ grad, BinWs ws, AdamArgs adam,
                                                                  uint32_t b_lo) {
    NGP_PROBE_BEGIN(NGP_P_RESIDUAL);
    const uint32_t b = b_lo + blockIdx.x;
    const bool mine = b < nbt && !fused_bucket(ws, b, ws.fb[MAXB] != 0);  // (block-uniform)
    float lr = 0.f, bc1 = 1.f, bc2 = 1.f;
    if (mine) adam_bias(adam.lr_dev, adam.step_dev, adam.b1, adam.b2, lr, bc1, bc2);
    if (mine) {
        const uint32_t l = bucket_level(ba, b), lb = b - ba.bbase[l];
        const uint32_t ne = min((uint32_t)BENT, ga.g.sizes[l] - (lb << BSHIFT));
        const size_t gbase = 2 * ((size_t)ga.g.offsets[l] + ((size_t)lb << BSHIFT));
        float4* g4 = reinterpret_cast<float4*>(grad + gbase);
        const float sc = adam.grad_scale;
        for (uint32_t e = threadIdx.x; e < 2 * ne / 4; e += blockDim.x) {
            const float4 gv = g4[e];
            adam4(adam, gbase, e, make_float4(gv.x * sc, gv.y * sc, gv.z * sc, gv.w * sc), lr, bc1, bc2);
            g4[e] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    NGP_PROBE_END();
}

static int bin_args(const ngp_hashgrid_t* grid, int64_t tiles_cap, int lo, int merge_hi, BinArgs& ba,
                    uint32_t& nbt) {
    if (lo < 0 || lo >= L || merge_hi < 0 || merge_hi > L) return NGP_EINVAL;
    ba.lo = lo;
    ba.merge = merge_hi >= 32 ? 0xffffffffu : ((1u << merge_hi) - 1u);
    uint32_t b = 0;
    for (int l = 0; l < L; ++l) {
        ba.bbase[l] = b;
        const uint32_t nb = l < lo ? 0u : (grid->sizes[l] + BENT - 1) >> BSHIFT;
        if (nb > (uint32_t)NBL) return NGP_ERANGE;
        if (grid->offsets[l] & 1u) return NGP_EINVAL;  // flush rows are 16-byte aligned
        b += nb;
    }
    ba.bbase[L] = b;
    ba.tiles_cap = tiles_cap;
    nbt = b;
    return b <= (uint32_t)MAXB ? NGP_OK : NGP_ERANGE;
}

}  // namespace ngp

using namespace ngp;

extern "C" {

size_t ngp_hash_backward_binned_workspace(int64_t max_samples) {
    if (max_samples <= 0) return 0;
    return bin_ws_bytes((max_samples + TILE - 1) / TILE, nullptr, nullptr);
}

// phase bit 1: count + scan + plan (xyzs / sample_idx only); bit 2: write +
// accumulate (needs denc and the plan of the same inputs).
static int hash_binned(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                       const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                       int64_t max_samples, int level_lo, int merge_hi, int phase, void* stream,
                       const AdamArgs* adam = nullptr, int acc_lo = 0, int acc_hi = L) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    NGP_CHECK_ARG(n >= 0 && max_samples > 0);
    if (n == 0) return NGP_OK;
    NGP_CHECK_ARG(xyzs && workspace && ((uintptr_t)workspace & 255) == 0);
    if (phase & 6)
        NGP_CHECK_ARG(grad_table && ((uintptr_t)grad_table & 15) == 0);
    if (phase & 2) NGP_CHECK_ARG(denc && ((uintptr_t)denc & 7) == 0);
    const int64_t tiles_cap = (max_samples + TILE - 1) / TILE;
    // record slots are uint32-indexed
    NGP_CHECK_ARG(tiles_cap * TILE * 4 * L < (int64_t)0xffffffffLL);
    BinArgs ba;
    uint32_t nbt;
    st = bin_args(grid, tiles_cap, level_lo, merge_hi, ba, nbt);
    if (st) return st;
    // phase 4 over the buckets of levels [acc_lo, acc_hi) only (levels below level_lo have none)
    NGP_CHECK_ARG(0 <= acc_lo && acc_lo <= acc_hi && acc_hi <= L);
    const uint32_t b_lo = ba.bbase[acc_lo], b_hi = ba.bbase[acc_hi];
    BinWs ws;
    bin_ws_bytes(tiles_cap, &ws, workspace);
    hipStream_t s = as_stream(stream);
    if (phase & 1) {
        static const unsigned capC = resident_blocks(hash_count_kernel, 256, 0);
        NGP_TIMED(NGP_K_HASH_COUNT, s, hash_count_kernel<<<persistent_blocks(n, TILE, capC), 256, 0, s>>>(xyzs, n, n_dev, sample_idx, ga, ba, ws));
        NGP_TIMED(NGP_K_HASH_SCAN, s, hash_scan_kernel<<<NSLOT, 256, 0, s>>>(n_dev, n, ba, ws));
        NGP_TIMED(NGP_K_HASH_PLAN, s, hash_plan_kernel<<<1, MAXB / 2, 0, s>>>(nbt, ws));
    }
    if (phase & 2) {
        static const unsigned capW = resident_blocks(hash_write_kernel<2>, 256, 0);
        NGP_TIMED(NGP_K_HASH_WRITE, s, hash_write_kernel<2><<<persistent_blocks(n, TILE, capW), 256, 0, s>>>(xyzs, n, n_dev, sample_idx, ga, ba,
                                                                           denc, grad_table, ws));
    }
    if (phase & 4) {
        static bool attr = false;
        const size_t lds = (size_t)BENT * 2 * sizeof(double);
        if (!attr) {
            if (hipFuncSetAttribute((const void*)hash_accum_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds) != hipSuccess ||
                hipFuncSetAttribute((const void*)hash_accum_kernel<true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                return NGP_ERANGE;
            attr = true;
        }
        static const unsigned capB = resident_blocks(hash_accum_kernel<false>, ACC_T, lds);
        if (adam) {
            NGP_TIMED(NGP_K_HASH_ACCUM, s, hash_accum_kernel<true><<<capB, ACC_T, lds, s>>>(ga, ba, nbt, grad_table, ws, *adam, b_lo, b_hi));
            if (b_hi > b_lo)
                NGP_TIMED(NGP_K_ADAM, s, hash_adam_residual_kernel<<<b_hi - b_lo, 256, 0, s>>>(ga, ba, nbt, grad_table, ws, *adam, b_lo));
        } else {
            NGP_TIMED(NGP_K_HASH_ACCUM, s, hash_accum_kernel<false><<<capB, ACC_T, lds, s>>>(ga, ba, nbt, grad_table, ws, AdamArgs{}, b_lo, b_hi));
        }
    }
    return ngp_launch_status();
}

int ngp_hash_backward_binned(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                             const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                             int64_t max_samples, int level_lo, int merge_hi, void* stream) {
    return hash_binned(xyzs, n, n_dev, sample_idx, grid, denc, grad_table, workspace, max_samples, level_lo,
                       merge_hi, 7, stream);
}

int ngp_hash_binned_plan(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                         const ngp_hashgrid_t* grid, void* workspace, int64_t max_samples, int level_lo,
                         int merge_hi, void* stream) {
    return hash_binned(xyzs, n, n_dev, sample_idx, grid, nullptr, nullptr, workspace, max_samples, level_lo,
                       merge_hi, 1, stream);
}

int ngp_hash_binned_apply(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                          const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                          int64_t max_samples, int level_lo, int merge_hi, void* stream) {
    return hash_binned(xyzs, n, n_dev, sample_idx, grid, denc, grad_table, workspace, max_samples, level_lo,
                       merge_hi, 6, stream);
}

int ngp_hash_binned_write(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                          const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                          int64_t max_samples, int level_lo, int merge_hi, void* stream) {
    return hash_binned(xyzs, n, n_dev, sample_idx, grid, denc, grad_table, workspace, max_samples, level_lo,
                       merge_hi, 2, stream);
}

int ngp_hash_binned_apply_adam(const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sample_idx,
                               const ngp_hashgrid_t* grid, const float* denc, float* grad_table, void* workspace,
                               int64_t max_samples, int level_lo, int merge_hi, float* params, float* exp_avg,
                               float* exp_avg_sq, void* params_f16, const float* lr_dev, float beta1, float beta2,
                               float eps, const int64_t* step_dev, float grad_scale, void* stream) {
    NGP_CHECK_ARG(params && exp_avg && exp_avg_sq && params_f16 && lr_dev && step_dev);
    NGP_CHECK_ARG(((uintptr_t)params & 15) == 0 && ((uintptr_t)exp_avg & 15) == 0 && ((uintptr_t)exp_avg_sq & 15) == 0 &&
                  ((uintptr_t)params_f16 & 7) == 0);
    const AdamArgs a{params, exp_avg, exp_avg_sq, (_Float16*)params_f16, lr_dev, step_dev, beta1, beta2, eps,
                     grad_scale};
    return hash_binned(xyzs, n, n_dev, sample_idx, grid, denc, grad_table, workspace, max_samples, level_lo,
                       merge_hi, 6, stream, &a);
}

int ngp_hash_binned_accum_adam(const ngp_hashgrid_t* grid, float* grad_table, void* workspace, int64_t max_samples,
                               int level_lo, int merge_hi, float* params, float* exp_avg, float* exp_avg_sq,
                               void* params_f16, const float* lr_dev, float beta1, float beta2, float eps,
                               const int64_t* step_dev, float grad_scale, void* stream) {
    NGP_CHECK_ARG(params && exp_avg && exp_avg_sq && params_f16 && lr_dev && step_dev);
    NGP_CHECK_ARG(((uintptr_t)params & 15) == 0 && ((uintptr_t)exp_avg & 15) == 0 && ((uintptr_t)exp_avg_sq & 15) == 0 &&
                  ((uintptr_t)params_f16 & 7) == 0);
    const AdamArgs a{params, exp_avg, exp_avg_sq, (_Float16*)params_f16, lr_dev, step_dev, beta1, beta2, eps,
                     grad_scale};
    static const float dummy[1] = {0.f};
    return hash_binned(dummy, 1, nullptr, nullptr, grid, nullptr, grad_table, workspace, max_samples, level_lo,
                       merge_hi, 4, stream, &a);
}

int ngp_hash_binned_accum(const ngp_hashgrid_t* grid, float* grad_table, void* workspace, int64_t max_samples,
                          int level_lo, int merge_hi, void* stream) {
    // (xyzs / n only gate the argument checks here; the accumulation reads the workspace)
    static const float dummy[1] = {0.f};
    return hash_binned(dummy, 1, nullptr, nullptr, grid, nullptr, grad_table, workspace, max_samples, level_lo,
                       merge_hi, 4, stream);
}

int ngp_hash_binned_accum_levels(const ngp_hashgrid_t* grid, float* grad_table, void* workspace, int64_t max_samples,
                                 int level_lo, int merge_hi, int acc_level_lo, int acc_level_hi, void* stream) {
    static const float dummy[1] = {0.f};
    return hash_binned(dummy, 1, nullptr, nullptr, grid, nullptr, grad_table, workspace, max_samples, level_lo,
                       merge_hi, 4, stream, nullptr, acc_level_lo, acc_level_hi);
}

}  // extern "C"
