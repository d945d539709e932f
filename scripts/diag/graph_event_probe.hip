// Probe: timing hipEvents recorded as external event nodes inside a captured
// HIP graph (hipEventRecordWithFlags(..., hipEventRecordExternal)).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void spin(float* p, int n, int it) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = p[i];
    for (int k = 0; k < it; ++k) v = __sinf(v) * 1.0001f + 0.5f;
    p[i] = v;
}
int main() {
    const int n = 1 << 20;
    float* p; CK(hipMalloc(&p, n * 4)); CK(hipMemset(p, 0, n * 4));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1, w0, w1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&w0)); CK(hipEventCreate(&w1));
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    spin<<<n / 256, 256, 0, s>>>(p, n, 100);
    CK(hipEventRecordWithFlags(e0, s, hipEventRecordExternal));
    spin<<<n / 256, 256, 0, s>>>(p, n, 2000);
    CK(hipEventRecordWithFlags(e1, s, hipEventRecordExternal));
    spin<<<n / 256, 256, 0, s>>>(p, n, 100);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(w0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(w1, s));
        CK(hipStreamSynchronize(s));
        float ms = -1, wms = -1;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipEventElapsedTime(&wms, w0, w1));
        printf("replay %d: inner kernel %.4f ms (whole graph %.4f ms)\n", r, ms, wms);
    }
    CK(hipEventRecord(w0, s));
    spin<<<n / 256, 256, 0, s>>>(p, n, 2000);
    CK(hipEventRecord(w1, s));
    CK(hipStreamSynchronize(s));
    float ms; CK(hipEventElapsedTime(&ms, w0, w1));
    printf("eager inner kernel %.4f ms\n", ms);
    return 0;
}
