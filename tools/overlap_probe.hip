// overlap_probe.hip -- a stand-in for the loop kernel's footprint (8 workgroups
// x 256 threads, optional 146944 B of LDS, optional dependent-FMA work) that
// runs for a fixed wall time on its own stream, so tools/overlap_probe.py can
// time the matched filter beside it and tell dispatch/residency effects from
// the loop kernel's own activity.
#include <hip/hip_runtime.h>
extern "C" __global__ void sleeper(long long ticks, int busy, float *sink) {
    extern __shared__ float lds[];   // launched with 0 or 146944 bytes
    const long long t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
    float x = threadIdx.x;
    if (threadIdx.x == 0) lds[0] = x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        if (busy) {
#pragma unroll 16
            for (int i = 0; i < 256; ++i) x = x * 1.0000001f + 1e-7f;
        } else {
            __builtin_amdgcn_s_sleep(64);
        }
    }
    if (x == 12345.0f) sink[threadIdx.x] = x;
}
extern "C" int launch_sleeper(void *stream, long long ticks, int lds_bytes, int busy, float *sink, int wgs) {
    hipLaunchKernelGGL(sleeper, dim3(wgs), dim3(256), lds_bytes, (hipStream_t)stream, ticks, busy, sink);
    return hipGetLastError();
}
