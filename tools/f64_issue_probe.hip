// tools/f64_issue_probe.hip -- issue cost of f64 VALU forms for a lone wave
// per SIMD on gfx950 (the Costas step is ~30 f64 ops per symbol, most of them
// three-source FMAs): independent v_add_f64 / v_mul_f64 / v_fma_f64 (three
// VGPR pairs) / v_fmac_f64 / v_fma_f64 with an SGPR-pair addend, eight
// independent accumulators each.  Diagnostic.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x

template <int V>
__global__ void kern(long long *cyc, double *sink, int iters, double sk) {
    double a0 = 1.0 + threadIdx.x * 1e-9, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
    double b = 0.999999, c = 1e-7;
    asm volatile("" : "+v"(b), "+v"(c));
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (V == 0) {
            R8(asm volatile("v_add_f64 %0, %0, %8\n\tv_add_f64 %1, %1, %8\n\tv_add_f64 %2, %2, %8\n\tv_add_f64 %3, %3, %8\n\t"
                            "v_add_f64 %4, %4, %8\n\tv_add_f64 %5, %5, %8\n\tv_add_f64 %6, %6, %8\n\tv_add_f64 %7, %7, %8"
                            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));)
        } else if (V == 1) {
            R8(asm volatile("v_mul_f64 %0, %0, %8\n\tv_mul_f64 %1, %1, %8\n\tv_mul_f64 %2, %2, %8\n\tv_mul_f64 %3, %3, %8\n\t"
                            "v_mul_f64 %4, %4, %8\n\tv_mul_f64 %5, %5, %8\n\tv_mul_f64 %6, %6, %8\n\tv_mul_f64 %7, %7, %8"
                            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (V == 2) {
            R8(asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\tv_fma_f64 %3, %3, %8, %9\n\t"
                            "v_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\tv_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9"
                            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));)
        } else if (V == 3) {
            R8(asm volatile("v_fmac_f64 %0, %8, %9\n\tv_fmac_f64 %1, %8, %9\n\tv_fmac_f64 %2, %8, %9\n\tv_fmac_f64 %3, %8, %9\n\t"
                            "v_fmac_f64 %4, %8, %9\n\tv_fmac_f64 %5, %8, %9\n\tv_fmac_f64 %6, %8, %9\n\tv_fmac_f64 %7, %8, %9"
                            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));)
        } else if (V == 4) {
            R8(asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %1, %1, %8, %9\n\tv_fma_f64 %2, %2, %8, %9\n\tv_fma_f64 %3, %3, %8, %9\n\t"
                            "v_fma_f64 %4, %4, %8, %9\n\tv_fma_f64 %5, %5, %8, %9\n\tv_fma_f64 %6, %6, %8, %9\n\tv_fma_f64 %7, %7, %8, %9"
                            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "s"(sk));)
        } else if (V == 5) {   // the same three-source FMA with a dependent pair chain: latency
            R8(asm volatile("v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %0, %0, %8, %9\n\t"
                            "v_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %0, %0, %8, %9\n\tv_fma_f64 %0, %0, %8, %9"
                            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));)
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
    long long *cyc;
    double *sink;
    hipMalloc(&cyc, 1024 * 4 * sizeof(long long));
    hipMalloc(&sink, 1024 * 256 * sizeof(double));
    const int iters = 1000;
    const char *names[] = {"v_add_f64 (2 src)", "v_mul_f64 (2 src)", "v_fma_f64 (3 VGPR pairs)",
                           "v_fmac_f64 (2 src + dst)", "v_fma_f64 (SGPR addend)", "v_fma_f64 dependent chain"};
    // blocks = 256 x 4 waves: one wave on every SIMD; blocks = 1, 64 threads:
    // one wave on an otherwise idle GPU (isa_bench's setting)
    auto run = [&](auto kfn, int v, int blocks, int threads) {
        hipLaunchKernelGGL(kfn, dim3(blocks), dim3(threads), 0, 0, cyc, sink, 10, 1e-7);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(kfn, dim3(blocks), dim3(threads), 0, 0, cyc, sink, iters, 1e-7);
        hipDeviceSynchronize();
        long long h[1024];
        hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        const int nw = blocks * threads / 64;
        double s = 0;
        for (int i = 0; i < nw; ++i) s += h[(i / (threads / 64)) * 4 + i % (threads / 64)];
        printf("%-30s %4d waves: %.2f cycles per instruction\n", names[v], nw, s / nw / (iters * 64.0));
    };
    for (int cfg = 0; cfg < 2; ++cfg) {
        const int blocks = cfg ? 1 : 256, threads = cfg ? 64 : 256;
        run(kern<0>, 0, blocks, threads);
        run(kern<1>, 1, blocks, threads);
        run(kern<2>, 2, blocks, threads);
        run(kern<3>, 3, blocks, threads);
        run(kern<4>, 4, blocks, threads);
        run(kern<5>, 5, blocks, threads);
    }
    return 0;
}
