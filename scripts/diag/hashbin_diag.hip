// Diagnostic build (NOT part of libngp_amd.so): the binned hash backward's
// record write alone in its variants, to split its time into record
// computation, LDS rank atomics and global stores (scripts/diag/hashbin_diag.py).
//   mode 2: the product (records stored from registers at their rank)
//   mode 3: no record stores      mode 6: no LDS rank atomics
//   mode 0: a level's records staged in LDS, bucket runs stored contiguously
#include "../../ar-nerf_amd/csrc/hashbin.hip"
#include "../../ar-nerf_amd/csrc/host.hip"

extern "C" int ngp_diag_hash_write(int mode, const float* xyzs, int64_t n, const int64_t* n_dev,
                                   const int32_t* sample_idx, const ngp_hashgrid_t* grid, const float* denc,
                                   float* grad_table, void* workspace, int64_t max_samples, int level_lo, int blocks,
                                   void* stream) {
    GridArgs ga;
    int st = grid_args(grid, ga);
    if (st) return st;
    const int64_t tiles_cap = (max_samples + TILE - 1) / TILE;
    BinArgs ba;
    uint32_t nbt;
    st = bin_args(grid, tiles_cap, level_lo, 0, ba, nbt);
    if (st) return st;
    BinWs ws;
    bin_ws_bytes(tiles_cap, &ws, workspace);
    hipStream_t s = as_stream(stream);
    const unsigned b = blocks > 0 ? (unsigned)blocks : persistent_blocks(n, TILE, resident_blocks(hash_write_kernel<2>, 256, 0));
    switch (mode) {
        case 2: hash_write_kernel<2><<<b, 256, 0, s>>>(xyzs, n, n_dev, sample_idx, ga, ba, denc, grad_table, ws); break;
        case 3: hash_write_kernel<3><<<b, 256, 0, s>>>(xyzs, n, n_dev, sample_idx, ga, ba, denc, grad_table, ws); break;
        case 6: hash_write_kernel<6><<<b, 256, 0, s>>>(xyzs, n, n_dev, sample_idx, ga, ba, denc, grad_table, ws); break;
        case 0: hash_write_kernel<0><<<b, 256, 0, s>>>(xyzs, n, n_dev, sample_idx, ga, ba, denc, grad_table, ws); break;
        default: return NGP_EINVAL;
    }
    return ngp_launch_status();
}
