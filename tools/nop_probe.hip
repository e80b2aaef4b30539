// tools/nop_probe.hip -- does a hazard s_nop cost a lone wave issue time on
// gfx950?  The FLL block (qpsk_fll.hip) carries 36 s_nop per 596 instructions
// (a packed-f32 result read by the next instruction, a DPP source); this
// measures shader cycles per VALU instruction of one wave per SIMD for
// independent packed adds with and without s_nops between them.  Diagnostic.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x

template <int V>
__global__ void kern(long long *cyc, float *sink, int iters) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v pa = {1.0f + threadIdx.x * 1e-6f, 1.0f}, pb = {0.9999f, 1.0001f}, pc = pa, pd = pa, pe = pa;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (V == 0) {   // 4 independent pk_add
            REP8(REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n\tv_pk_add_f32 %1, %1, %4\n\t"
                                   "v_pk_add_f32 %2, %2, %4\n\tv_pk_add_f32 %3, %3, %4"
                                   : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pe) : "v"(pb));))
        } else if (V == 1) {   // the same, s_nop 0 after every second one
            REP8(REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n\tv_pk_add_f32 %1, %1, %4\n\ts_nop 0\n\t"
                                   "v_pk_add_f32 %2, %2, %4\n\tv_pk_add_f32 %3, %3, %4\n\ts_nop 0"
                                   : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pe) : "v"(pb));))
        } else if (V == 2) {   // s_nop 1 after every second one
            REP8(REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n\tv_pk_add_f32 %1, %1, %4\n\ts_nop 1\n\t"
                                   "v_pk_add_f32 %2, %2, %4\n\tv_pk_add_f32 %3, %3, %4\n\ts_nop 1"
                                   : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pe) : "v"(pb));))
        } else if (V == 3) {   // s_nop 0 after every one
            REP8(REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n\ts_nop 0\n\tv_pk_add_f32 %1, %1, %4\n\ts_nop 0\n\t"
                                   "v_pk_add_f32 %2, %2, %4\n\ts_nop 0\n\tv_pk_add_f32 %3, %3, %4\n\ts_nop 0"
                                   : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pe) : "v"(pb));))
        } else if (V == 4) {   // 2 dependent pairs interleaved: mul -> add, no nops needed
            REP8(REP8(asm volatile("v_pk_mul_f32 %0, %0, %4\n\tv_pk_mul_f32 %1, %1, %4\n\t"
                                   "v_pk_add_f32 %0, %0, %4\n\tv_pk_add_f32 %1, %1, %4"
                                   : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pe) : "v"(pb));))
        } else if (V == 5) {   // 1 dependent pair at a time: mul, s_nop 0, add (the FLL's pattern)
            REP8(REP8(asm volatile("v_pk_mul_f32 %0, %0, %4\n\ts_nop 0\n\tv_pk_add_f32 %0, %0, %4\n\t"
                                   "v_pk_mul_f32 %1, %1, %4\n\ts_nop 0\n\tv_pk_add_f32 %1, %1, %4"
                                   : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pe) : "v"(pb));))
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = pa.x + pc.x + pd.y + pe.x;
}

int main() {
    long long *cyc;
    float *sink;
    hipMalloc(&cyc, 1024 * 4 * sizeof(long long));
    hipMalloc(&sink, 1024 * 256 * sizeof(float));
    const int iters = 2000;
    const char *names[] = {"4 indep pk_add", "+ s_nop 0 per 2", "+ s_nop 1 per 2", "+ s_nop 0 per 1",
                           "2 mul->add pairs interleaved", "mul, s_nop 0, add (serial pairs)"};
    auto run = [&](auto kfn, int v) {
        hipLaunchKernelGGL(kfn, dim3(256), dim3(256), 0, 0, cyc, sink, 10);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(kfn, dim3(256), dim3(256), 0, 0, cyc, sink, iters);
        hipDeviceSynchronize();
        long long h[1024];
        hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < 1024; ++i) s += h[i];
        const double per = s / 1024 / (iters * 256.0);
        printf("%-34s %.2f cycles per VALU instruction\n", names[v], per);
    };
    run(kern<0>, 0);
    run(kern<1>, 1);
    run(kern<2>, 2);
    run(kern<3>, 3);
    run(kern<4>, 4);
    run(kern<5>, 5);
    return 0;
}
