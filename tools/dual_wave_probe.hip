// tools/dual_wave_probe.hip -- does a second wave per SIMD raise VALU issue on
// gfx950?  The FLL (qpsk_fll.hip) runs one wave per SIMD and issues one VALU
// instruction every ~5.2 shader cycles; a split into a chain wave and a helper
// wave only pays if two waves on one SIMD issue faster than one.  Diagnostic.
//
// Each wave runs `iters` x 64 groups of 4 independent packed / f64 ops (or a
// dependent chain), timed with s_memtime; printed: shader cycles per
// instruction of ONE wave, and SIMD cycles per instruction summed over the
// waves that share a SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x

template <int V>
__global__ void kern(long long *cyc, float *sink, int iters) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v pa = {1.0f + threadIdx.x * 1e-6f, 1.0f}, pb = {0.9999f, 1.0001f}, pc = pa, pd = pa, pe = pa;
    double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999, c = 1e-7, d = a, e = a, f = a;
    // waves 4..7 of a 512-thread block share SIMDs with waves 0..3
    const bool second = threadIdx.x >= 256;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (V == 0 || (V == 2 && second)) {   // 4 independent pk_add chains
            REP8(REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n\tv_pk_add_f32 %1, %1, %4\n\t"
                                   "v_pk_add_f32 %2, %2, %4\n\tv_pk_add_f32 %3, %3, %4"
                                   : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pe) : "v"(pb));))
        } else if (V == 1) {   // 4 independent fma_f64 chains
            REP8(REP8(asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_fma_f64 %1, %1, %4, %5\n\t"
                                   "v_fma_f64 %2, %2, %4, %5\n\tv_fma_f64 %3, %3, %4, %5"
                                   : "+v"(a), "+v"(d), "+v"(e), "+v"(f) : "v"(b), "v"(c));))
        } else if (V == 2) {   // first waves: one dependent pk_add chain (latency-bound)
            REP8(REP8(asm volatile("v_pk_add_f32 %0, %0, %1\n\tv_pk_add_f32 %0, %0, %1\n\t"
                                   "v_pk_add_f32 %0, %0, %1\n\tv_pk_add_f32 %0, %0, %1"
                                   : "+v"(pa) : "v"(pb));))
        } else if (V == 3) {   // mixed f64 / packed / int, independent
            int ia = threadIdx.x, ib = 3;
            REP8(REP8(asm volatile("v_fma_f64 %0, %0, %3, %4\n\tv_pk_add_f32 %1, %1, %5\n\t"
                                   "v_add_u32 %2, %2, %6\n\tv_pk_mul_f32 %1, %1, %5"
                                   : "+v"(a), "+v"(pc), "+v"(ia) : "v"(b), "v"(c), "v"(pb), "v"(ib));))
            pa.x += ia;
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = pa.x + pc.x + pd.y + pe.x + (float)(a + d + e + f);
}

int main() {
    long long *cyc;
    float *sink;
    hipMalloc(&cyc, 4096 * 8 * sizeof(long long));
    hipMalloc(&sink, 4096 * 512 * sizeof(float));
    const int iters = 2000;
    const char *names[] = {"4x indep pk_add", "4x indep fma_f64", "dep pk_add | indep pk_add", "mixed indep"};
    auto run = [&](auto kfn, int v, int waves) {
        hipLaunchKernelGGL(kfn, dim3(256), dim3(64 * waves), 0, 0, cyc, sink, 10);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(kfn, dim3(256), dim3(64 * waves), 0, 0, cyc, sink, iters);
        hipDeviceSynchronize();
        long long h[8];
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        const double n = 256.0 * iters;   // instructions per wave
        double w0 = h[0] / n, w4 = waves > 4 ? h[4] / n : 0.0;
        printf("%-28s waves/SIMD %d: wave0 %.2f cyc/instr, wave4 %.2f, SIMD %.2f cyc/instr\n", names[v],
               waves / 4, w0, w4, waves > 4 ? (h[0] > h[4] ? h[0] : h[4]) / (2 * n) : w0);
    };
    run(kern<0>, 0, 4); run(kern<0>, 0, 8);
    run(kern<1>, 1, 4); run(kern<1>, 1, 8);
    run(kern<2>, 2, 4); run(kern<2>, 2, 8);
    run(kern<3>, 3, 4); run(kern<3>, 3, 8);
    return 0;
}
