// Diagnostic build (NOT part of libngp_amd.so): the hash-grid backward with
// atomics removed / replaced / unmerged and restricted level ranges, to split
// its time into compute, scatter-shape and atomic cost.  scripts/diag/hash_bwd.py
#include "../../ar-nerf_amd/csrc/field.hip"
#include "../../ar-nerf_amd/csrc/hashbin.hip"
#include "../../ar-nerf_amd/csrc/host.hip"

extern "C" int ngp_diag_hash_bwd(int mode, int lo, int hi, int blocks_cap, const float* xyzs, int64_t n,
                                 const int64_t* n_dev, const int32_t* sidx, const ngp_hashgrid_t* grid,
                                 const float* denc, float* grad, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    const unsigned b = persistent_blocks(n, 64, blocks_cap);
    hipStream_t s = as_stream(stream);
    switch (mode) {
        case 0: hash_bwd_kernel<0><<<b, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, denc, grad, lo, hi); break;
        case 1: hash_bwd_kernel<1><<<b, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, denc, grad, lo, hi); break;
        case 2: hash_bwd_kernel<2><<<b, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, denc, grad, lo, hi); break;
        case 3: hash_bwd_kernel<3><<<b, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, denc, grad, lo, hi); break;
        default: return NGP_EINVAL;
    }
    return ngp_launch_status();
}

// pass 5 alone, on a workspace filled by ngp_hash_backward_binned
extern "C" int ngp_diag_hash_accum(int mode, int threads, const ngp_hashgrid_t* grid, float* grad, void* workspace,
                                   int64_t max_samples, int lo, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    const int64_t tiles_cap = (max_samples + TILE - 1) / TILE;
    BinArgs ba;
    uint32_t nbt;
    st = bin_args(grid, tiles_cap, lo, 0, ba, nbt);
    if (st) return st;
    BinWs ws;
    bin_ws_bytes(tiles_cap, &ws, workspace);
    const size_t lds = (size_t)BENT * 2 * sizeof(double);
    hipStream_t s = as_stream(stream);
    static bool attr[4] = {false, false, false, false};
    const void* fns[4] = {(const void*)hash_accum_kernel<0>, (const void*)hash_accum_kernel<1>,
                          (const void*)hash_accum_kernel<2>, (const void*)hash_accum_kernel<3>};
    if (!attr[mode]) {
        hipFuncSetAttribute(fns[mode], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr[mode] = true;
    }
    switch (mode) {
        case 0: hash_accum_kernel<0><<<256, threads, lds, s>>>(ga, ba, nbt, grad, ws, AdamArgs{}); break;
        case 1: hash_accum_kernel<1><<<256, threads, lds, s>>>(ga, ba, nbt, grad, ws, AdamArgs{}); break;
        case 2: hash_accum_kernel<2><<<256, threads, lds, s>>>(ga, ba, nbt, grad, ws, AdamArgs{}); break;
        case 3: hash_accum_kernel<3><<<256, threads, lds, s>>>(ga, ba, nbt, grad, ws, AdamArgs{}); break;
        default: return NGP_EINVAL;
    }
    return ngp_launch_status();
}

// LDS atomic throughput microbenchmark: each thread issues `iters` adds to
// pseudo-random words of a 128 KB LDS image (kind 0: ds_add_f32, 1: ds_add_u32,
// 2: ds_add_f64, 3: plain ds read+write (not atomic), 4: ds_add_f32 at
// conflict-free addresses (lane-linear)).
template <int KIND>
__global__ void __launch_bounds__(1024) lds_atomic_bench(int iters, float* out) {
    extern __shared__ __attribute__((aligned(16))) float img[];
    const int t = threadIdx.x;
    for (int e = t; e < 32768; e += blockDim.x) img[e] = 0.f;
    __syncthreads();
    uint32_t h = t * 2654435761u + blockIdx.x * 97u;
    for (int i = 0; i < iters; ++i) {
        h = h * 1664525u + 1013904223u;
        const uint32_t a = KIND == 4 ? ((t + i * 64) & 32767) : (h >> 17);
        if (KIND == 0 || KIND == 4) atomicAdd(&img[a], 1.0f);
        else if (KIND == 1) atomicAdd(reinterpret_cast<uint32_t*>(img) + a, 1u);
        else if (KIND == 2) atomicAdd(reinterpret_cast<double*>(img) + (a >> 1), 1.0);
        else { img[a] += 1.0f; }
    }
    __syncthreads();
    if (t == 0) out[blockIdx.x] = img[t];
}

extern "C" int ngp_diag_lds_atomics(int kind, int iters, float* out, void* stream) {
    const size_t lds = 131072;
    hipStream_t s = as_stream(stream);
    static bool attr[5] = {false, false, false, false, false};
    const void* fns[5] = {(const void*)lds_atomic_bench<0>, (const void*)lds_atomic_bench<1>,
                          (const void*)lds_atomic_bench<2>, (const void*)lds_atomic_bench<3>,
                          (const void*)lds_atomic_bench<4>};
    if (!attr[kind]) {
        hipFuncSetAttribute(fns[kind], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr[kind] = true;
    }
    switch (kind) {
        case 0: lds_atomic_bench<0><<<256, 1024, lds, s>>>(iters, out); break;
        case 1: lds_atomic_bench<1><<<256, 1024, lds, s>>>(iters, out); break;
        case 2: lds_atomic_bench<2><<<256, 1024, lds, s>>>(iters, out); break;
        case 3: lds_atomic_bench<3><<<256, 1024, lds, s>>>(iters, out); break;
        case 4: lds_atomic_bench<4><<<256, 1024, lds, s>>>(iters, out); break;
        default: return NGP_EINVAL;
    }
    return ngp_launch_status();
}

// pass 4 alone (after a full ngp_hash_backward_binned call filled ofs/rstart)
extern "C" int ngp_diag_hash_write(int mode, const float* xyzs, int64_t n, const int64_t* n_dev, const int32_t* sidx,
                                   const ngp_hashgrid_t* grid, const float* denc, float* grad, void* workspace,
                                   int64_t max_samples, int lo, void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    const int64_t tiles_cap = (max_samples + TILE - 1) / TILE;
    BinArgs ba;
    uint32_t nbt;
    st = bin_args(grid, tiles_cap, lo, 0, ba, nbt);
    if (st) return st;
    BinWs ws;
    bin_ws_bytes(tiles_cap, &ws, workspace);
    hipStream_t s = as_stream(stream);
    const unsigned g = persistent_blocks(n, TILE, 2048);
    switch (mode) {
        case 0: hash_write_kernel<0><<<g, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, ba, denc, grad, ws); break;
        case 1: hash_write_kernel<1><<<g, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, ba, denc, grad, ws); break;
        case 2: hash_write_kernel<2><<<g, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, ba, denc, grad, ws); break;
        case 3: hash_write_kernel<3><<<g, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, ba, denc, grad, ws); break;
        case 5: hash_write_kernel<5><<<g, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, ba, denc, grad, ws); break;
        case 7: hash_write_kernel<7><<<g, 256, 0, s>>>(xyzs, n, n_dev, sidx, ga, ba, denc, grad, ws); break;
        default: return NGP_EINVAL;
    }
    return ngp_launch_status();
}
