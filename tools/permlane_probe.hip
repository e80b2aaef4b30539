// permlane_probe.hip -- semantics of v_permlane32_swap_b32 on gfx950
// (__builtin_amdgcn_permlane32_swap(old, src, fi, bc) -> {new vdst, new src}).
//   hipcc --offload-arch=gfx950 -O2 tools/permlane_probe.hip -o tools/bin/permlane_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *o) {
    const unsigned a = 1000u + threadIdx.x, b = 2000u + threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    o[2 * threadIdx.x] = r[0];
    o[2 * threadIdx.x + 1] = r[1];
}
int main() {
    unsigned *d, h[128];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int l : {0, 1, 31, 32, 33, 63}) std::printf("lane %2d: r0 %u r1 %u\n", l, h[2 * l], h[2 * l + 1]);
    return 0;
}
