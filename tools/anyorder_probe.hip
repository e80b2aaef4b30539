// anyorder_probe.hip -- does a kernel launched with hipExtAnyOrderLaunch on the
// SAME stream start while the previous kernel still runs (AQL barrier bit
// cleared), on gfx950?  Kernel A: 128 workgroups holding 125 KB of LDS each
// (the loop kernel's footprint) that spin for a fixed wall time; kernel B: many
// short workgroups (the FIR's shape).  Each kernel records its first
// workgroup start and last workgroup end (s_memrealtime, 100 MHz) with vector
// atomics.  No kernel waits for another, so no ordering can hang it.
//   hipcc --offload-arch=gfx950 -O2 tools/anyorder_probe.hip -o tools/bin/anyorder_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));             \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__global__ __launch_bounds__(256) void spin_kernel(unsigned long long *t, uint64_t ticks,
                                                   unsigned long long *resident) {
    __shared__ float big[125 * 1024 / 4];
    const uint64_t t0 = wall_clock64();
    if (threadIdx.x == 0) atomicMin(&t[0], t0);
    if (resident && threadIdx.x == 0)
        __hip_atomic_fetch_add(resident, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    big[threadIdx.x] = static_cast<float>(threadIdx.x);
    float acc = 0.f;
    while (wall_clock64() - t0 < ticks) acc += big[(threadIdx.x * 7) & 255];
    __syncthreads();
    if (threadIdx.x == 0) {
        if (acc == -1.f) t[3] = 1;   // keep acc live
        atomicMax(&t[1], wall_clock64());
    }
}

__global__ __launch_bounds__(256) void short_kernel(unsigned long long *t, float *buf) {
    __shared__ float tile[4096];
    const uint64_t t0 = wall_clock64();
    if (threadIdx.x == 0) atomicMin(&t[0], t0);
    float acc = 0.f;
    for (int i = 0; i < 16; ++i) tile[threadIdx.x + 256 * i] = buf[(blockIdx.x * 256 + threadIdx.x + i) & 1048575];
    __syncthreads();
    for (int k = 0; k < 2000; ++k) acc = acc * 0.999f + tile[(threadIdx.x + k) & 4095];
    buf[(blockIdx.x * 256 + threadIdx.x) & 1048575] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&t[1], wall_clock64());
}

int main() {
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    unsigned long long *t;
    float *buf;
    CK(hipMalloc(&t, 8 * sizeof(unsigned long long)));
    CK(hipMalloc(&buf, 1048576 * sizeof(float)));
    CK(hipMemset(buf, 0, 1048576 * sizeof(float)));
    unsigned long long *sig;
    CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&sig), 8, hipMallocSignalMemory));
    CK(hipMemset(sig, 0, 8));
    unsigned long long target = 0;
    int can_wait = 0;
    CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
    std::printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can_wait);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const uint64_t ticks = static_cast<uint64_t>(rate_khz) * 20;   // 20 ms
    const char *names[5] = {"same stream, default", "same stream, B any-order", "two streams",
                            "B first, waits A resident", "B first, no wait"};
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 5; ++mode) {
            unsigned long long init[8] = {~0ull, 0, ~0ull, 0, 0, 0, 0, 0};
            CK(hipMemcpy(t, init, sizeof(init), hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            if (mode >= 3) {
                // the race lost on purpose: B is issued (and ready) before A
                if (mode == 3) {
                    target += 128;
                    CK(hipStreamWaitValue64(s2, sig, target, hipStreamWaitValueGte));
                }
                hipLaunchKernelGGL(short_kernel, dim3(100000), dim3(256), 0, s2, t + 2, buf);
                hipLaunchKernelGGL(spin_kernel, dim3(128), dim3(256), 0, s1, t, ticks, mode == 3 ? sig : nullptr);
            } else {
            hipLaunchKernelGGL(spin_kernel, dim3(128), dim3(256), 0, s1, t, ticks, nullptr);
            hipStream_t sb = mode == 2 ? s2 : s1;
            if (mode == 1)
                hipExtLaunchKernelGGL(short_kernel, dim3(100000), dim3(256), 0, sb, nullptr, nullptr,
                                      hipExtAnyOrderLaunch, t + 2, buf);
            else
                hipLaunchKernelGGL(short_kernel, dim3(100000), dim3(256), 0, sb, t + 2, buf);
            }
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            unsigned long long h[8];
            CK(hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost));
            const double us = 1000.0 / rate_khz;
            const unsigned long long o = h[0] < h[2] ? h[0] : h[2];
            std::printf("%-28s A [%8.1f, %8.1f] us  B [%8.1f, %8.1f] us  %s\n", names[mode], (h[0] - o) * us,
                        (h[1] - o) * us, (h[2] - o) * us, (h[3] - o) * us,
                        h[2] < h[1] ? "OVERLAP" : "serial");
        }
    return 0;
}
