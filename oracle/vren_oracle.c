/*
 * vren_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * CPU restatement of the reference's Instant-NGP hot path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the oracle the
 * HIP kernels are compared against.  Nothing under ar-nerf_amd/ links or
 * calls this file.
 *
 * Each function cites the reference file:line it restates (paths relative to
 * the YessionCC/AR-NeRF tree).  Built with -O2 -ffp-contract=off
 * -fno-fast-math so that every fp32 expression is evaluated exactly as the
 * CUDA source writes it (no FMA contraction), which is what makes the
 * occupancy/Morton indexing and per-ray sample counts bit-exact targets.
 *
 * Pinning (see DESIGN.md "Oracle"): the reference's CUDA extension `vren`
 * cannot be built here (needs the CUDA toolkit: helper_math.h includes
 * cuda_runtime.h, volumerendering.cu needs thrust's CUDA backend), so the
 * kernel arithmetic is pinned by (a) the known answers written in the
 * reference's own comments (raymarching.cu:15-18,25-28; morton bit order
 * raymarching.cu:35-60; packbits LSB-first raymarching.cu:136-138) and
 * (b) golden fixtures produced by running the reference's own Python glue
 * (models/rendering.py, models/custom_functions.py, models/networks.py,
 * losses.py) with this oracle plugged in as `vren`.  The tiny-cuda-nn
 * hash-grid / SH / FullyFusedMLP arithmetic is restated from tcnn's
 * published algorithm (not vendored by the reference): parity unpinned.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SQRT3 1.73205080757f

/* ---------------------------------------------------------------- helpers */
/* helper_math.h:280-283  clamp(f,a,b) = fmaxf(a, fminf(f, b)) */
static inline float clampf_(float f, float a, float b) { return fmaxf(a, fminf(f, b)); }
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
/* raymarching.cu:7 */
static inline float signf_(float x) { return copysignf(1.0f, x); }

/* raymarching.cu:11-13 */
static inline float calc_dt(float t, float esf, int max_samples, int grid_size, float scale) {
    return clampf_(t * esf, SQRT3 / max_samples, SQRT3 * 2 * scale / grid_size);
}
/* raymarching.cu:19-23 */
static inline int mip_from_pos(float x, float y, float z, int cascades) {
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    int exponent; frexpf(mx, &exponent);
    return imin(cascades - 1, imax(0, exponent + 1));
}
/* raymarching.cu:29-32 */
static inline int mip_from_dt(float dt, int grid_size, int cascades) {
    int exponent; frexpf(dt * grid_size, &exponent);
    return imin(cascades - 1, imax(0, exponent));
}
/* raymarching.cu:35-42 */
static inline uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
/* raymarching.cu:44-50 */
static inline uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
/* raymarching.cu:52-60 */
static inline uint32_t morton3_invert(uint32_t x) {
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

/* IEEE binary16 <-> binary32, round-to-nearest-even (the rounding the GPU's
 * v_cvt_f16_f32 performs); used for tcnn's fp16 storage points. */
uint16_t or_f32_to_f16(float f) {
    uint32_t x; memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t exp = (x >> 23) & 0xffu;
    uint32_t mant = x & 0x7fffffu;
    if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (mant ? (0x200u | (mant >> 13)) : 0u));
    const int e = (int)exp - 127 + 15;
    if (e >= 0x1f) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        const int shift = 14 - e;
        uint32_t hm = mant >> shift;
        const uint32_t rem = mant & ((1u << shift) - 1u), halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (hm & 1u))) hm++;
        return (uint16_t)(sign | hm);
    }
    const uint32_t hm = mant >> 13, rem = mant & 0x1fffu;
    uint32_t h = sign | ((uint32_t)e << 10) | hm;
    if (rem > 0x1000u || (rem == 0x1000u && (hm & 1u))) h++;
    return (uint16_t)h;
}
float or_f16_to_f32(uint16_t h) {
    const uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu, mant = h & 0x3ffu, x;
    if (exp == 0) {
        if (mant == 0) x = sign;
        else {
            exp = 127 - 15 + 1;
            while (!(mant & 0x400u)) { mant <<= 1; exp--; }
            mant &= 0x3ffu;
            x = sign | (exp << 23) | (mant << 13);
        }
    } else if (exp == 0x1f) x = sign | 0x7f800000u | (mant << 13);
    else x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    float f; memcpy(&f, &x, 4); return f;
}
static inline float rh(float f) { return or_f16_to_f32(or_f32_to_f16(f)); }

/* ------------------------------------------------------- ray / AABB (a2) */
/* intersection.cu:5-22 (_ray_aabb_intersect) and :25-56 (kernel), host side
 * :59-100 including the ascending sort of hits by t1 (misses = -1 first). */
void or_ray_aabb_intersect(int n_rays, const float* rays_o, const float* rays_d,
                           int n_vox, const float* centers, const float* half_sizes,
                           int max_hits, int32_t* hit_cnt, float* hits_t, int64_t* hits_vox) {
    for (int r = 0; r < n_rays; ++r) {
        float* ht = hits_t + (size_t)r * max_hits * 2;
        int64_t* hv = hits_vox + (size_t)r * max_hits;
        for (int k = 0; k < max_hits; ++k) { ht[2 * k] = -1.0f; ht[2 * k + 1] = -1.0f; hv[k] = -1; }
        int cnt = 0;
        const float o[3] = {rays_o[3 * r], rays_o[3 * r + 1], rays_o[3 * r + 2]};
        const float inv[3] = {1.0f / rays_d[3 * r], 1.0f / rays_d[3 * r + 1], 1.0f / rays_d[3 * r + 2]};
        for (int v = 0; v < n_vox; ++v) {
            float t1v[3], t2v[3];
            for (int i = 0; i < 3; ++i) {
                const float tmin = (centers[3 * v + i] - half_sizes[3 * v + i] - o[i]) * inv[i];
                const float tmax = (centers[3 * v + i] + half_sizes[3 * v + i] - o[i]) * inv[i];
                t1v[i] = fminf(tmin, tmax); t2v[i] = fmaxf(tmin, tmax);
            }
            float t1 = fmaxf(fmaxf(t1v[0], t1v[1]), t1v[2]);
            float t2 = fminf(fminf(t2v[0], t2v[1]), t2v[2]);
            if (t1 > t2) { t1 = -1.0f; t2 = -1.0f; }
            if (t2 > 0) {
                if (cnt < max_hits) { ht[2 * cnt] = fmaxf(t1, 0.0f); ht[2 * cnt + 1] = t2; hv[cnt] = v; }
                cnt++;
            }
        }
        hit_cnt[r] = cnt;
        /* torch::sort(hits_t[...,0]) ascending, then gather (intersection.cu:95-97) */
        for (int a = 1; a < max_hits; ++a) {
            const float k0 = ht[2 * a], k1 = ht[2 * a + 1]; const int64_t kv = hv[a];
            int b = a - 1;
            while (b >= 0 && ht[2 * b] > k0) { ht[2 * b + 2] = ht[2 * b]; ht[2 * b + 3] = ht[2 * b + 1]; hv[b + 1] = hv[b]; b--; }
            ht[2 * b + 2] = k0; ht[2 * b + 3] = k1; hv[b + 1] = kv;
        }
    }
}

/* ------------------------------------------------ morton / packbits (a9) */
/* raymarching.cu:62-70 */
void or_morton3D(int n, const int32_t* coords, int32_t* out) {
    for (int i = 0; i < n; ++i)
        out[i] = (int32_t)morton3((uint32_t)coords[3 * i], (uint32_t)coords[3 * i + 1], (uint32_t)coords[3 * i + 2]);
}
/* raymarching.cu:90-101 */
void or_morton3D_invert(int n, const int32_t* idx, int32_t* coords) {
    for (int i = 0; i < n; ++i) {
        const int32_t ind = idx[i];
        coords[3 * i] = (int32_t)morton3_invert((uint32_t)(ind >> 0));
        coords[3 * i + 1] = (int32_t)morton3_invert((uint32_t)(ind >> 1));
        coords[3 * i + 2] = (int32_t)morton3_invert((uint32_t)(ind >> 2));
    }
}
/* raymarching.cu:122-141: bit i of byte n <- grid[8n+i] > thr */
void or_packbits(int n_bytes, const float* grid, float thr, uint8_t* bitfield) {
    for (int n = 0; n < n_bytes; ++n) {
        uint8_t bits = 0;
        for (int i = 0; i < 8; ++i) bits |= (grid[8 * n + i] > thr) ? (uint8_t)(1u << i) : 0;
        bitfield[n] = bits;
    }
}

/* -------------------------------------------------- ray marching (a3) */
/* One step of the occupancy walk shared by raymarching.cu:204-233 (count),
 * :245-278 (write) and :367-401 (test).  Returns 1 if the sample at t is
 * occupied (t advanced by dt), 0 if t jumped to the next voxel boundary. */
static inline int march_step(float* tp, float ox, float oy, float oz, float dx, float dy, float dz,
                             float dx_inv, float dy_inv, float dz_inv, const uint8_t* bf,
                             int cascades, int grid_size, float scale, float dt_scale, float esf,
                             int max_samples, float* px, float* py, float* pz, float* pdt) {
    const uint32_t grid_size3 = (uint32_t)(grid_size * grid_size * grid_size);
    const float grid_size_inv = 1.0f / grid_size;
    float t = *tp;
    const float x = ox + t * dx, y = oy + t * dy, z = oz + t * dz;
    const float dt = calc_dt(t, esf, max_samples, grid_size, dt_scale);
    const int mip = imax(mip_from_pos(x, y, z, cascades), mip_from_dt(dt, grid_size, cascades));
    const float mip_bound = fminf(scalbnf(1.0f, mip - 1), scale);
    const float mip_bound_inv = 1 / mip_bound;
    const int nx = (int)clampf_(0.5f * (x * mip_bound_inv + 1) * grid_size, 0.0f, grid_size - 1.0f);
    const int ny = (int)clampf_(0.5f * (y * mip_bound_inv + 1) * grid_size, 0.0f, grid_size - 1.0f);
    const int nz = (int)clampf_(0.5f * (z * mip_bound_inv + 1) * grid_size, 0.0f, grid_size - 1.0f);
    const uint32_t idx = (uint32_t)mip * grid_size3 + morton3((uint32_t)nx, (uint32_t)ny, (uint32_t)nz);
    const int occ = (bf[idx / 8] & (1u << (idx % 8))) != 0;
    *px = x; *py = y; *pz = z; *pdt = dt;
    if (occ) { t += dt; *tp = t; return 1; }
    const float tx = (((nx + 0.5f + 0.5f * signf_(dx)) * grid_size_inv * 2 - 1) * mip_bound - x) * dx_inv;
    const float ty = (((ny + 0.5f + 0.5f * signf_(dy)) * grid_size_inv * 2 - 1) * mip_bound - y) * dy_inv;
    const float tz = (((nz + 0.5f + 0.5f * signf_(dz)) * grid_size_inv * 2 - 1) * mip_bound - z) * dz_inv;
    const float t_target = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    do { t += calc_dt(t, esf, max_samples, grid_size, dt_scale); } while (t < t_target);
    *tp = t;
    return 0;
}

/* raymarching.cu:166-280 + custom_functions.py:79-100, with a deterministic
 * RAY-ORDERED layout: rays_a row r = (r, start_r, n_r) with start_r the
 * exclusive prefix sum of the counts (the reference assigns rows/starts by
 * two independent atomicAdds; compare per ray).  counts: (n_rays) out.
 * If xyzs == NULL only counts/rays_a are produced.  Returns total samples. */
int64_t or_march_train(int n_rays, const float* rays_o, const float* rays_d, const float* hits_t,
                       const uint8_t* bf, int cascades, int grid_size, float scale, float esf,
                       const float* noise, int max_samples, int32_t* counts, int64_t* rays_a,
                       float* xyzs, float* dirs, float* deltas, float* ts) {
    /* pass 1 (raymarching.cu:184-234): per-ray sample count */
#pragma omp parallel for schedule(dynamic, 64)
    for (int r = 0; r < n_rays; ++r) {
        const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
        const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
        const float dx_inv = 1.0f / dx, dy_inv = 1.0f / dy, dz_inv = 1.0f / dz;
        float t1 = hits_t[2 * r]; const float t2 = hits_t[2 * r + 1];
        if (t1 >= 0) { const float dt = calc_dt(t1, esf, max_samples, grid_size, scale); t1 += dt * noise[r]; }
        float t = t1; int N = 0; float x, y, z, dt;
        while (0 <= t && t < t2 && N < max_samples)
            N += march_step(&t, ox, oy, oz, dx, dy, dz, dx_inv, dy_inv, dz_inv, bf, cascades, grid_size,
                            scale, scale, esf, max_samples, &x, &y, &z, &dt);
        counts[r] = N;
    }
    /* ray-ordered exclusive prefix sum -> rays_a (replaces :237-241 atomics) */
    int64_t total = 0;
    for (int r = 0; r < n_rays; ++r) {
        rays_a[3 * r] = r; rays_a[3 * r + 1] = total; rays_a[3 * r + 2] = counts[r];
        total += counts[r];
    }
    if (!xyzs) return total;
    /* pass 2 (raymarching.cu:243-279): re-march and write */
#pragma omp parallel for schedule(dynamic, 64)
    for (int r = 0; r < n_rays; ++r) {
        const int N = counts[r];
        if (N == 0) continue;
        const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
        const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
        const float dx_inv = 1.0f / dx, dy_inv = 1.0f / dy, dz_inv = 1.0f / dz;
        float t1 = hits_t[2 * r]; const float t2 = hits_t[2 * r + 1];
        if (t1 >= 0) { const float dt = calc_dt(t1, esf, max_samples, grid_size, scale); t1 += dt * noise[r]; }
        const int64_t start = rays_a[3 * r + 1];
        float t = t1; int samples = 0; float x, y, z, dt;
        while (t < t2 && samples < N) {
            const float tcur = t;
            if (march_step(&t, ox, oy, oz, dx, dy, dz, dx_inv, dy_inv, dz_inv, bf, cascades, grid_size,
                           scale, scale, esf, max_samples, &x, &y, &z, &dt)) {
                const int64_t s = start + samples;
                xyzs[3 * s] = x; xyzs[3 * s + 1] = y; xyzs[3 * s + 2] = z;
                dirs[3 * s] = dx; dirs[3 * s + 1] = dy; dirs[3 * s + 2] = dz;
                ts[s] = tcur; deltas[s] = dt; samples++;
            }
        }
    }
    return total;
}

/* raymarching.cu:335-404 (test-time march).  NOTE the reference quirk kept
 * here: calc_dt receives `cascades` as its scale argument (:370,:399), while
 * the mip bound still uses `scale` (:374).  hits_t (n_rays,2) is updated in
 * place (:390).  Output rows are zero where no sample was taken. */
void or_march_test(int n_alive, const float* rays_o, const float* rays_d, float* hits_t,
                   const int64_t* alive, const uint8_t* bf, int cascades, int grid_size, float scale,
                   float esf, int N_samples, int max_samples, float* xyzs, float* dirs,
                   float* deltas, float* ts, int32_t* n_eff) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int n = 0; n < n_alive; ++n) {
        const int64_t r = alive[n];
        const float ox = rays_o[3 * r], oy = rays_o[3 * r + 1], oz = rays_o[3 * r + 2];
        const float dx = rays_d[3 * r], dy = rays_d[3 * r + 1], dz = rays_d[3 * r + 2];
        const float dx_inv = 1.0f / dx, dy_inv = 1.0f / dy, dz_inv = 1.0f / dz;
        float t = hits_t[2 * r]; const float t2 = hits_t[2 * r + 1];
        int s = 0; float x, y, z, dt;
        for (int k = 0; k < N_samples; ++k) {
            const size_t o = (size_t)n * N_samples + k;
            xyzs[3 * o] = xyzs[3 * o + 1] = xyzs[3 * o + 2] = 0.f;
            dirs[3 * o] = dirs[3 * o + 1] = dirs[3 * o + 2] = 0.f;
            deltas[o] = 0.f; ts[o] = 0.f;
        }
        while (t < t2 && s < N_samples) {
            const float tcur = t;
            if (march_step(&t, ox, oy, oz, dx, dy, dz, dx_inv, dy_inv, dz_inv, bf, cascades, grid_size,
                           scale, (float)cascades, esf, max_samples, &x, &y, &z, &dt)) {
                const size_t o = (size_t)n * N_samples + s;
                xyzs[3 * o] = x; xyzs[3 * o + 1] = y; xyzs[3 * o + 2] = z;
                dirs[3 * o] = dx; dirs[3 * o + 1] = dy; dirs[3 * o + 2] = dz;
                ts[o] = tcur; deltas[o] = dt;
                hits_t[2 * r] = t;
                s++;
            }
        }
        n_eff[n] = s;
    }
}

/* -------------------------------------------------- compositing (a7) */
/* volumerendering.cu:5-44.  Outputs must be zeroed by the caller (the
 * reference allocates them with torch::zeros, :57-61). */
void or_composite_train_fw(int n_rays, const float* sigmas, const float* rgbs, const float* deltas,
                           const float* ts, const int64_t* rays_a, float T_thr, int64_t* total_samples,
                           float* opacity, float* depth, float* rgb, float* ws) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int n = 0; n < n_rays; ++n) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        int64_t samples = 0; float T = 1.0f;
        while (samples < N) {
            const int64_t s = start + samples;
            const float a = 1.0f - expf(-sigmas[s] * deltas[s]);
            const float w = a * T;
            rgb[3 * ray] += w * rgbs[3 * s]; rgb[3 * ray + 1] += w * rgbs[3 * s + 1]; rgb[3 * ray + 2] += w * rgbs[3 * s + 2];
            depth[ray] += w * ts[s];
            opacity[ray] += w;
            ws[s] = w;
            T *= 1.0f - a;
            if (T <= T_thr) break;
            samples++;
        }
        total_samples[ray] = samples;
    }
}

/* volumerendering.cu:86-150 (+ the dL_dws*ws auxiliary input, :174).
 * dsig/drgbs zeroed by caller (:171-172). */
void or_composite_train_bw(int n_rays, const float* dL_dop, const float* dL_ddep, const float* dL_drgb,
                           const float* dL_dws, const float* sigmas, const float* rgbs, const float* ws,
                           const float* deltas, const float* ts, const int64_t* rays_a, const float* opacity,
                           const float* depth, const float* rgb, float T_thr, float* dL_dsig, float* dL_drgbs) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int n = 0; n < n_rays; ++n) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        if (N <= 0) continue;
        /* inclusive scan of dL_dws*ws over the ray's samples (:118-122) */
        float* scan = (float*)malloc(sizeof(float) * (size_t)N);
        float acc = 0.f;
        for (int64_t k = 0; k < N; ++k) { acc += dL_dws[start + k] * ws[start + k]; scan[k] = acc; }
        const float S = scan[N - 1];
        const float R = rgb[3 * ray], G = rgb[3 * ray + 1], B = rgb[3 * ray + 2];
        const float O = opacity[ray], D = depth[ray];
        float T = 1.0f, r = 0.f, g = 0.f, b = 0.f, d = 0.f;
        int64_t samples = 0;
        while (samples < N) {
            const int64_t s = start + samples;
            const float a = 1.0f - expf(-sigmas[s] * deltas[s]);
            const float w = a * T;
            r += w * rgbs[3 * s]; g += w * rgbs[3 * s + 1]; b += w * rgbs[3 * s + 2];
            d += w * ts[s];
            T *= 1.0f - a;
            dL_drgbs[3 * s] = dL_drgb[3 * ray] * w;
            dL_drgbs[3 * s + 1] = dL_drgb[3 * ray + 1] * w;
            dL_drgbs[3 * s + 2] = dL_drgb[3 * ray + 2] * w;
            dL_dsig[s] = deltas[s] * (dL_drgb[3 * ray] * (rgbs[3 * s] * T - (R - r)) +
                                      dL_drgb[3 * ray + 1] * (rgbs[3 * s + 1] * T - (G - g)) +
                                      dL_drgb[3 * ray + 2] * (rgbs[3 * s + 2] * T - (B - b)) +
                                      dL_dop[ray] * (1 - O) + dL_ddep[ray] * (ts[s] * T - (D - d)) +
                                      T * dL_dws[s] - (S - scan[samples]));
            if (T <= T_thr) break;
            samples++;
        }
        free(scan);
    }
}

/* volumerendering.cu:204-248.  sigmas/deltas/ts (n_alive, Ns), rgbs
 * (n_alive, Ns, 3); alive/opacity/depth/rgb updated in place. */
void or_composite_test_fw(int n_alive, int Ns, const float* sigmas, const float* rgbs, const float* deltas,
                          const float* ts, int64_t* alive, float T_thr, const int32_t* n_eff,
                          float* opacity, float* depth, float* rgb) {
    for (int n = 0; n < n_alive; ++n) {
        if (n_eff[n] == 0) { alive[n] = -1; continue; }
        const int64_t r = alive[n];
        int s = 0; float T = 1 - opacity[r];
        while (s < n_eff[n]) {
            const size_t o = (size_t)n * Ns + s;
            const float a = 1.0f - expf(-sigmas[o] * deltas[o]);
            const float w = a * T;
            rgb[3 * r] += w * rgbs[3 * o]; rgb[3 * r + 1] += w * rgbs[3 * o + 1]; rgb[3 * r + 2] += w * rgbs[3 * o + 2];
            depth[r] += w * ts[o];
            opacity[r] += w;
            T *= 1.0f - a;
            if (T <= T_thr) { alive[n] = -1; break; }
            s++;
        }
    }
}

/* ------------------------------------------------ distortion loss */
/* losses.cu:8-107 (DVGO-v2 form of the Mip-NeRF 360 distortion loss).
 * thrust::inclusive/exclusive_scan and reduce inside a kernel thread run
 * sequentially (no dynamic parallelism): left folds from 0.  wts = ws*ts and
 * the _loss expression are separate torch ops (:70, :92-93), each rounded.
 * Outputs zeroed by the caller (torch::zeros, :72-75,95). */
void or_distortion_loss_fw(int n_rays, const float* ws, const float* deltas, const float* ts,
                           const int64_t* rays_a, float* loss, float* ws_inc, float* wts_inc) {
    const float third = 1.0f / 3;
#pragma omp parallel for schedule(dynamic, 64)
    for (int n = 0; n < n_rays; ++n) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        float a = 0.f, b = 0.f, acc = 0.f;
        for (int64_t k = 0; k < N; ++k) {
            const int64_t s = start + k;
            const float wts = ws[s] * ts[s];
            const float ws_exc = a, wts_exc = b;
            a = a + ws[s];
            b = b + wts;
            ws_inc[s] = a;
            wts_inc[s] = b;
            const float p = b * ws_exc, q = a * wts_exc;
            const float l = 2 * (p - q) + ((third * ws[s]) * ws[s]) * deltas[s];
            acc = acc + l;
        }
        loss[ray] = acc;
    }
}

/* losses.cu:110-140 */
void or_distortion_loss_bw(int n_rays, const float* dL_dloss, const float* ws_inc, const float* wts_inc,
                           const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                           float* dL_dws) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int n = 0; n < n_rays; ++n) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1], N = rays_a[3 * n + 2];
        if (N <= 0) continue;
        const int64_t end = start + N - 1;
        const float ws_sum = ws_inc[end], wts_sum = wts_inc[end];
        const float g = dL_dloss[ray];
        for (int64_t s = start; s <= end; ++s) {
            const float A = s == start ? 0.0f : ts[s] * ws_inc[s - 1] - wts_inc[s - 1];
            const float B = (wts_sum - wts_inc[s]) - ts[s] * (ws_sum - ws_inc[s]);
            const float x = (g * 2) * (A + B);
            const float y = (((g * 2.0f) / 3.0f) * ws[s]) * deltas[s];
            dL_dws[s] = x + y;
        }
    }
}

/* ------------------------------------------- multires hash grid (a4) */
/* tiny-cuda-nn GridEncoding (Hash, Linear), restated from its published
 * algorithm as configured at models/networks.py:33-49:
 *   scale_l = exp2f(l*log2f(b))*N_min - 1,  res_l = ceilf(scale_l)+1,
 *   size_l  = min(next_multiple(res_l^3, 8), 2^log2T)      (entries)
 * Fills scales/res/offsets(L+1)/sizes; returns total entries. */
uint32_t or_hash_levels(int L, int log2T, int N_min, float per_level_scale, float* scales,
                        uint32_t* res, uint32_t* offsets, uint32_t* sizes) {
    const float l2 = log2f(per_level_scale);
    uint32_t off = 0;
    for (int l = 0; l < L; ++l) {
        const float s = exp2f((float)l * l2) * (float)N_min - 1.0f;
        const uint32_t rr = (uint32_t)ceilf(s) + 1;
        const uint32_t max_params = 0xffffffffu / 2;
        uint32_t p = (powf((float)rr, 3.0f) > (float)max_params) ? max_params : rr * rr * rr;
        p = (p + 7u) / 8u * 8u;
        if (p > (1u << log2T)) p = 1u << log2T;
        scales[l] = s; res[l] = rr; offsets[l] = off; sizes[l] = p;
        off += p;
    }
    offsets[L] = off;
    return off;
}

/* tcnn grid_index: dense strides while they fit the level, else the
 * xor-of-primes spatial hash; then mod the level size. */
static inline uint32_t grid_index(uint32_t size, uint32_t res, uint32_t px, uint32_t py, uint32_t pz) {
    uint32_t stride = 1, index = 0;
    const uint32_t p[3] = {px, py, pz};
    for (int dim = 0; dim < 3 && stride <= size; ++dim) { index += p[dim] * stride; stride *= res; }
    if (size < stride) index = (px * 1u) ^ (py * 2654435761u) ^ (pz * 805459861u);
    return index % size;
}

/* Per-sample level/corner geometry shared by fwd and bwd. */
static inline void level_corners(float x01, float y01, float z01, float scale, uint32_t res, uint32_t size,
                                 uint32_t idx[8], float w[8]) {
    float pos[3]; uint32_t pg[3];
    const float in[3] = {x01, y01, z01};
    for (int d = 0; d < 3; ++d) {
        float p = fmaf(scale, in[d], 0.5f);
        const float g = floorf(p);
        pg[d] = (uint32_t)(int)g;
        pos[d] = p - g;
    }
    for (int c = 0; c < 8; ++c) {
        float wt = 1.0f; uint32_t q[3];
        for (int d = 0; d < 3; ++d) {
            if ((c & (1 << d)) == 0) { wt *= 1 - pos[d]; q[d] = pg[d]; }
            else { wt *= pos[d]; q[d] = pg[d] + 1; }
        }
        w[c] = wt; idx[c] = grid_index(size, res, q[0], q[1], q[2]);
    }
}

/* models/networks.py:104-105 x01 = (x - xyz_min)/(xyz_max - xyz_min), then the
 * hash encoding.  table: fp16 bits (entries,2) = the fp16 copy of the fp32
 * master params.  Feature accumulation: acc = fmaf(w_c, v_c, acc) over the 8
 * corners in tcnn's corner order, fp32; output rounded once to fp16.
 * enc: (n, 2L) fp16 bits, level-major (feature 2l, 2l+1). */
void or_hash_encode_fwd(int n, const float* x, const float* xyz_min, const float* xyz_max, int L,
                        const float* scales, const uint32_t* res, const uint32_t* offsets,
                        const uint32_t* sizes, const uint16_t* table, uint16_t* enc) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        float in[3];
        for (int d = 0; d < 3; ++d) in[d] = (x[3 * i + d] - xyz_min[d]) / (xyz_max[d] - xyz_min[d]);
        for (int l = 0; l < L; ++l) {
            uint32_t idx[8]; float w[8];
            level_corners(in[0], in[1], in[2], scales[l], res[l], sizes[l], idx, w);
            float a0 = 0.f, a1 = 0.f;
            for (int c = 0; c < 8; ++c) {
                const size_t e = (size_t)offsets[l] + idx[c];
                a0 = fmaf(w[c], or_f16_to_f32(table[2 * e]), a0);
                a1 = fmaf(w[c], or_f16_to_f32(table[2 * e + 1]), a1);
            }
            enc[(size_t)i * 2 * L + 2 * l] = or_f32_to_f16(a0);
            enc[(size_t)i * 2 * L + 2 * l + 1] = or_f32_to_f16(a1);
        }
    }
}

/* Backward of the above w.r.t. the table: dtable[e][f] += w_c * denc[2l+f]
 * (fp32, sample order).  denc (n, 2L) fp32; dtable (entries, 2) fp32. */
void or_hash_encode_bwd(int n, const float* x, const float* xyz_min, const float* xyz_max, int L,
                        const float* scales, const uint32_t* res, const uint32_t* offsets,
                        const uint32_t* sizes, const float* denc, float* dtable) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int l = 0; l < L; ++l) {
        for (int i = 0; i < n; ++i) {
            float in[3];
            for (int d = 0; d < 3; ++d) in[d] = (x[3 * i + d] - xyz_min[d]) / (xyz_max[d] - xyz_min[d]);
            uint32_t idx[8]; float w[8];
            level_corners(in[0], in[1], in[2], scales[l], res[l], sizes[l], idx, w);
            const float g0 = denc[(size_t)i * 2 * L + 2 * l], g1 = denc[(size_t)i * 2 * L + 2 * l + 1];
            for (int c = 0; c < 8; ++c) {
                const size_t e = (size_t)offsets[l] + idx[c];
                dtable[2 * e] += w[c] * g0;
                dtable[2 * e + 1] += w[c] * g1;
            }
        }
    }
}

/* Flat corner indices (level offset added) and weights, (n, L, 8): used by
 * tests to check the integer hashing bit-exactly. */
void or_hash_corners(int n, const float* x, const float* xyz_min, const float* xyz_max, int L,
                     const float* scales, const uint32_t* res, const uint32_t* offsets,
                     const uint32_t* sizes, uint32_t* idx_out, float* w_out) {
    for (int i = 0; i < n; ++i) {
        float in[3];
        for (int d = 0; d < 3; ++d) in[d] = (x[3 * i + d] - xyz_min[d]) / (xyz_max[d] - xyz_min[d]);
        for (int l = 0; l < L; ++l) {
            uint32_t idx[8]; float w[8];
            level_corners(in[0], in[1], in[2], scales[l], res[l], sizes[l], idx, w);
            for (int c = 0; c < 8; ++c) {
                idx_out[((size_t)i * L + l) * 8 + c] = offsets[l] + idx[c];
                w_out[((size_t)i * L + l) * 8 + c] = w[c];
            }
        }
    }
}

/* ------------------------------------------------ SH degree 4 (a6) */
/* tcnn SphericalHarmonics (degree 4) on an input already in [0,1]^3: tcnn
 * maps it back with x = 2*in - 1 and evaluates the 16 real SH basis
 * functions; stored fp16.  out: (n,16) fp16 bits. */
static void sh4_core(float in0, float in1, float in2, uint16_t* out) {
    const float x = in0 * 2.f - 1.f, y = in1 * 2.f - 1.f, z = in2 * 2.f - 1.f;
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
    for (int k = 0; k < 16; ++k) out[k] = or_f32_to_f16(o[k]);
}
void or_sh4_unit01(int n, const float* in01, uint16_t* out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) sh4_core(in01[3 * i], in01[3 * i + 1], in01[3 * i + 2], out + (size_t)i * 16);
}
/* models/networks.py:144-145: d/|d| (torch.norm = sqrt of the fp32 sum of
 * squares), (d+1)/2, then the tcnn encoding above. */
void or_sh4(int n, const float* dirs, uint16_t* out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        const float dx = dirs[3 * i], dy = dirs[3 * i + 1], dz = dirs[3 * i + 2];
        const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
        sh4_core((dx / nrm + 1) / 2, (dy / nrm + 1) / 2, (dz / nrm + 1) / 2, out + (size_t)i * 16);
    }
}

/* --------------------------------------------------- Adam (a10) */
/* apex FusedAdam (train.py:146: lr, eps=1e-15; betas (0.9,0.999), no decay):
 * m=b1 m+(1-b1)g; v=b2 v+(1-b2)g^2; p -= lr*(m/bc1)/(sqrt(v/bc2)+eps). */
void or_adam(int64_t n, float* p, const float* g, float* m, float* v, float lr, float b1, float b2,
             float eps, float bc1, float bc2) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const float gi = g[i];
        m[i] = b1 * m[i] + (1 - b1) * gi;
        v[i] = b2 * v[i] + (1 - b2) * gi * gi;
        const float denom = sqrtf(v[i] / bc2) + eps;
        p[i] = p[i] - lr * ((m[i] / bc1) / denom);
    }
}

/* keep rh() referenced for builds that only use part of the file */
float or_round_half(float f) { return rh(f); }

/* Exported for known-answer tests only. */
float or_calc_dt(float t, float esf, int max_samples, int grid_size, float scale) {
    return calc_dt(t, esf, max_samples, grid_size, scale);
}
int or_mip_from_pos(float x, float y, float z, int cascades) { return mip_from_pos(x, y, z, cascades); }
int or_mip_from_dt(float dt, int grid_size, int cascades) { return mip_from_dt(dt, grid_size, cascades); }
