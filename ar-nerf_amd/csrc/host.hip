// Host-side helpers of libngp_amd.so.
#include <math.h>

#include "common.h"

// Kernel timing hook (ngp_timing_set): a one-lane kernel before and after
// each instrumented launch stores the GPU wall clock into the caller's stamp
// table, row = *step_dev % ring -- plain kernel nodes, so a captured HIP
// graph times its kernels on every replay (HIP event nodes inside captured
// graphs are not available with the HIP runtime torch ships).
static uint64_t* g_stamps = nullptr;
static const int64_t* g_step = nullptr;
static int64_t g_ring = 0;
static int g_ids = 0, g_per = 0;
static uint64_t g_begin = 0, g_end = 0;  // ids bracketed before / after
static int32_t g_count[64];

__global__ void stamp_kernel(uint64_t* __restrict__ stamps, const int64_t* __restrict__ step, int64_t ring,
                             int64_t row_len, int64_t col) {
    if (threadIdx.x == 0) stamps[(*step % ring) * row_len + col] = wall_clock64();
}

void ngp_timing_mark(int id, int end, hipStream_t s) {
    if (!g_stamps || id < 0 || id >= g_ids) return;
    const int i = g_count[id];
    if (end) g_count[id] = i + 1;
    if (i >= g_per || !(((end ? g_end : g_begin) >> id) & 1ull)) return;
    stamp_kernel<<<1, 64, 0, s>>>(g_stamps, g_step, g_ring, (int64_t)g_ids * g_per * 2,
                                  ((int64_t)id * g_per + i) * 2 + (end ? 1 : 0));
}

// device probes: every translation unit registers the setter of its copy of
// the control symbol (common.h) at load time
static void (*g_probe_setters[16])(const ProbeCtl&);
static int g_n_probe_setters = 0;
void ngp_probe_register(void (*set)(const ProbeCtl&)) {
    if (g_n_probe_setters < 16) g_probe_setters[g_n_probe_setters++] = set;
}

// capacity guards: each translation unit's counter reader (common.h)
static unsigned long long (*g_guard_getters[16])(int);
static int g_n_guard_getters = 0;
void ngp_guard_register(unsigned long long (*get)(int)) {
    if (g_n_guard_getters < 16) g_guard_getters[g_n_guard_getters++] = get;
}

// a kernel whose only purpose is its name in a dispatch trace (ngp_trace_marker)
__global__ void trace_marker_kernel(int tag) {
    if (tag < 0) __builtin_trap();  // (never: keeps the argument live)
}

extern "C" {

const char* ngp_version(void) { return "ngp_amd 0.2 gfx950"; }

int ngp_timing_set(uint64_t* stamps, const int64_t* step_dev, int64_t ring, int n_ids, int per_id, uint64_t begin_mask,
                   uint64_t end_mask) {
    if (stamps && (!step_dev || ring < 1 || n_ids < 1 || n_ids > 64 || per_id < 1)) return NGP_EINVAL;
    g_stamps = stamps;
    g_step = stamps ? step_dev : nullptr;
    g_ring = stamps ? ring : 0;
    g_ids = stamps ? n_ids : 0;
    g_per = stamps ? per_id : 0;
    g_begin = begin_mask;
    g_end = end_mask;
    for (int i = 0; i < 64; ++i) g_count[i] = 0;
    return NGP_OK;
}

int ngp_probe_set(uint64_t* buf, const int64_t* step_dev, int64_t ring) {
    if (buf && (!step_dev || ring < 1)) return NGP_EINVAL;
    const ProbeCtl c{(unsigned long long*)buf, buf ? step_dev : nullptr, buf ? ring : 0};
    for (int i = 0; i < g_n_probe_setters; ++i) g_probe_setters[i](c);
    const hipError_t e = hipDeviceSynchronize();
    return e == hipSuccess ? NGP_OK : (int)e;
}

int ngp_probe_count(void) { return NGP_P_COUNT; }

unsigned long long ngp_guard_hits(void) {
    unsigned long long s = 0;
    for (int i = 0; i < g_n_guard_getters; ++i) {
        const unsigned long long v = g_guard_getters[i](0);
        if (v == ~0ull) return ~0ull;
        s += v;
    }
    return s;
}

int ngp_guard_reset(void) {
    for (int i = 0; i < g_n_guard_getters; ++i)
        if (g_guard_getters[i](1) == ~0ull) return NGP_EINVAL;
    return NGP_OK;
}

int ngp_trace_marker(int tag, void* stream) {
    NGP_CHECK_ARG(tag >= 0);
    trace_marker_kernel<<<1, 64, 0, as_stream(stream)>>>(tag);
    return ngp_launch_status();
}

int ngp_timing_counts(int32_t* counts, int n_ids) {
    if (!counts || n_ids < 0 || n_ids > 64) return NGP_EINVAL;
    for (int i = 0; i < n_ids; ++i) counts[i] = g_count[i];
    return NGP_OK;
}

double ngp_timing_tick_ns(void) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
        return 0.0;
    return 1e6 / (double)khz;
}

// Level table of tcnn's Grid/Hash encoding as the reference configures it
// (models/networks.py:33-49): computed in fp32 the way tcnn does
// (scale_l = exp2f(l*log2f(b))*N_min - 1, res_l = ceilf(scale_l)+1,
// size_l = min(next_multiple(res_l^3, 8), 2^log2T)).  Host-side once, so the
// kernels and every caller use one table (no host/device exp2f mismatch).
uint32_t ngp_hashgrid_levels(int n_levels, int log2T, int base_resolution, float per_level_scale, float* scales,
                             uint32_t* res, uint32_t* offsets, uint32_t* sizes) {
    if (n_levels < 1 || n_levels > 32 || log2T < 1 || log2T > 30 || !scales || !res || !offsets || !sizes) return 0;
    const float l2 = log2f(per_level_scale);
    uint32_t off = 0;
    for (int l = 0; l < n_levels; ++l) {
        const float s = exp2f((float)l * l2) * (float)base_resolution - 1.0f;
        const uint32_t r = (uint32_t)ceilf(s) + 1u;
        const uint32_t max_params = 0xffffffffu / 2u;
        uint32_t p = (powf((float)r, 3.0f) > (float)max_params) ? max_params : r * r * r;
        p = (p + 7u) / 8u * 8u;
        const uint32_t T = 1u << log2T;
        if (p > T) p = T;
        scales[l] = s;
        res[l] = r;
        offsets[l] = off;
        sizes[l] = p;
        off += p;
    }
    offsets[n_levels] = off;
    return off;
}

}  // extern "C"
