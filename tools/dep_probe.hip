// tools/dep_probe.hip -- what one VALU dependency costs a lone wave on gfx950,
// measured without the compiler's inline-asm padding.
//
// tools/isa_bench.hip times a dependent chain as one asm statement per
// instruction, and hipcc pads consecutive inline-asm statements with `s_nop 0`
// (a hazard it cannot rule out inside asm), so its "8.25-8.5 cycles per
// dependent op" counts a nop per op.  Here every chain is ONE asm statement of
// 16 instructions, written out with explicit registers, so the only waits are
// the hardware's; the dependent f64 chains are checked bit for bit against
// the host (a missing hardware interlock would show as a stale read).  Also:
// the same chains with an explicit `s_nop 0` between ops (isa_bench's case),
// operand register banks (bank = VGPR index mod 4), SGPR operands, VCC
// producers and consumers, f32 / packed / integer / conversion chains and two
// interleaved chains.  Diagnostic only; vector stores only.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>

#define R2(x) x x
#define R4(x) R2(x) R2(x)
#define R16(x) R4(R4(x))

// one wave: a (double) chain seed in v[2:3] of every lane
template <int V>
__global__ void kern(double *out, long long *cyc, int iters, double seed, double b, double c) {
    double a = seed + threadIdx.x * 1e-9;
    float fa = (float)a;
    unsigned ua = threadIdx.x;
    long long t0 = 0, t1 = 0;
    // explicit registers: the chain lives in v[10:11]; operands in v[12:13],
    // v[14:15] (banks 0/2), v[16:17] (bank 0, same as v12), v[20:21]
    asm volatile("v_mov_b64 v[10:11], %0\n\tv_mov_b64 v[12:13], %1\n\tv_mov_b64 v[14:15], %2\n\t"
                 "v_mov_b64 v[16:17], %2\n\tv_mov_b64 v[18:19], %1\n\tv_mov_b64 v[20:21], %0\n\t"
                 "v_mov_b32 v24, %3\n\tv_mov_b32 v25, %4\n\tv_mov_b32 v26, 1.0\n\tv_mov_b32 v27, 0x3f800001"
                 :: "v"(a), "v"(b), "v"(c), "v"(fa), "v"(ua)
                 : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v24",
                   "v25", "v26", "v27");
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (V == 0)        // dependent v_fma_f64, operands on banks 0 (chain), 0 (v12), 2 (v14)
            asm volatile(R16("v_fma_f64 v[10:11], v[10:11], v[12:13], v[14:15]\n\t") ::: "v10", "v11");
        else if (V == 1)   // the same with s_nop 0 between (isa_bench's padding)
            asm volatile(R16("v_fma_f64 v[10:11], v[10:11], v[12:13], v[14:15]\n\ts_nop 0\n\t") ::: "v10", "v11");
        else if (V == 2)   // dependent fma, all three sources on bank 0 (v10, v12, v16)
            asm volatile(R16("v_fma_f64 v[10:11], v[10:11], v[12:13], v[16:17]\n\t") ::: "v10", "v11");
        else if (V == 3)   // dependent fma, sources on banks 0, 2, 2 (v10, v18, v14)
            asm volatile(R16("v_fma_f64 v[10:11], v[10:11], v[18:19], v[14:15]\n\t") ::: "v10", "v11");
        else if (V == 4)   // dependent v_add_f64
            asm volatile(R16("v_add_f64 v[10:11], v[10:11], v[14:15]\n\t") ::: "v10", "v11");
        else if (V == 5)   // dependent v_mul_f64
            asm volatile(R16("v_mul_f64 v[10:11], v[10:11], v[12:13]\n\t") ::: "v10", "v11");
        else if (V == 6)   // dependent fma with an SGPR addend
            asm volatile(R16("v_fma_f64 v[10:11], v[10:11], v[12:13], %0\n\t") :: "s"(c) : "v10", "v11");
        else if (V == 7)   // two interleaved dependent fma chains (v10, v20)
            asm volatile(R16("v_fma_f64 v[10:11], v[10:11], v[12:13], v[14:15]\n\t"
                             "v_fma_f64 v[20:21], v[20:21], v[12:13], v[14:15]\n\t") ::: "v10", "v11", "v20", "v21");
        else if (V == 8)   // four independent fmas per step (issue rate)
            asm volatile(R4("v_fma_f64 v[10:11], v[10:11], v[12:13], v[14:15]\n\t"
                            "v_fma_f64 v[20:21], v[20:21], v[12:13], v[14:15]\n\t"
                            "v_fma_f64 v[28:29], v[12:13], v[14:15], v[16:17]\n\t"
                            "v_fma_f64 v[30:31], v[12:13], v[16:17], v[14:15]\n\t")
                         ::: "v10", "v11", "v20", "v21", "v28", "v29", "v30", "v31");
        else if (V == 9)   // dependent v_fma_f32
            asm volatile(R16("v_fma_f32 v24, v24, v26, v27\n\t") ::: "v24");
        else if (V == 10)  // dependent v_pk_add_f32
            asm volatile(R16("v_pk_add_f32 v[10:11], v[10:11], v[26:27]\n\t") ::: "v10", "v11");
        else if (V == 11)  // dependent v_add_u32
            asm volatile(R16("v_add_u32 v25, v25, v26\n\t") ::: "v25");
        else if (V == 12)  // v_cmp -> vcc -> v_cndmask -> v_cmp ... (the Costas decision shape)
            asm volatile(R16("v_cmp_le_f64 vcc, v[12:13], v[10:11]\n\tv_cndmask_b32 v11, v13, v15, vcc\n\t")
                         ::: "v11", "vcc");
        else if (V == 13)  // f64 -> f32 -> f64 conversions, dependent (M&M t = (float)mu, widen)
            asm volatile(R16("v_cvt_f32_f64 v24, v[10:11]\n\tv_cvt_f64_f32 v[10:11], v24\n\t") ::: "v10", "v11",
                         "v24");
        else if (V == 14)  // dependent v_floor_f64 + v_add_f64 (the M&M timing update)
            asm volatile(R16("v_add_f64 v[10:11], v[10:11], v[14:15]\n\tv_floor_f64 v[10:11], v[10:11]\n\t")
                         ::: "v10", "v11");
        else if (V == 15)  // dependent fma with |abs| and neg source modifiers
            asm volatile(R16("v_fma_f64 v[10:11], -|v[10:11]|, v[12:13], v[14:15]\n\t") ::: "v10", "v11");
        else if (V == 16)  // dependent v_fmac_f64 (VOP2, dst = addend)
            asm volatile(R16("v_fmac_f64 v[10:11], v[12:13], v[14:15]\n\tv_mul_f64 v[12:13], v[10:11], v[18:19]\n\t")
                         ::: "v10", "v11", "v12", "v13");
        else if (V == 17)  // dependent v_max_f64 with abs (the Costas range track)
            asm volatile(R16("v_max_f64 v[10:11], v[10:11], |v[14:15]|\n\tv_add_f64 v[14:15], v[10:11], v[14:15]\n\t")
                         ::: "v10", "v11", "v14", "v15");
    }
    t1 = __builtin_amdgcn_s_memtime();
    double r;
    asm volatile("v_mov_b64 %0, v[10:11]" : "=v"(r));
    out[threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

static const int kPerIter[] = {16, 16, 16, 16, 16, 16, 16, 32, 16, 16, 16, 16, 32, 32, 32, 16, 32, 32};
static const char *kName[] = {
    "dep fma_f64 (banks 0,0,2)",      "dep fma_f64 + s_nop 0",          "dep fma_f64 (banks 0,0,0)",
    "dep fma_f64 (banks 0,2,2)",      "dep add_f64",                    "dep mul_f64",
    "dep fma_f64 (SGPR addend)",      "2 interleaved fma_f64 chains",   "4 independent fma_f64",
    "dep fma_f32",                    "dep pk_add_f32",                 "dep add_u32",
    "cmp_f64 -> vcc -> cndmask pairs", "cvt f64->f32->f64 pairs",       "add_f64 + floor_f64 pairs",
    "dep fma_f64 -|a| modifiers",     "fmac_f64 -> mul_f64 pairs",      "max_f64 |b| -> add_f64 pairs"};

template <int V>
static void run(double *out, long long *cyc, int iters) {
    const double seed = 1.25, b = 0.999999, c = 1e-7;
    hipLaunchKernelGGL(kern<V>, dim3(1), dim3(64), 0, 0, out, cyc, 4, seed, b, c);
    hipLaunchKernelGGL(kern<V>, dim3(1), dim3(64), 0, 0, out, cyc, iters, seed, b, c);
    hipDeviceSynchronize();
    long long cy;
    double got;
    hipMemcpy(&cy, cyc, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&got, out, 8, hipMemcpyDeviceToHost);
    char check[48] = "";
    if (V == 0 || V == 1 || V == 3) {   // host replay of lane 0's chain
        double x = seed;
        const double bb = (V == 3) ? b : b, cc = c;
        for (long long i = 0; i < (long long)iters * 16; ++i) x = std::fma(x, bb, cc);
        std::snprintf(check, sizeof check, "  [lane 0 %s host]", std::memcmp(&x, &got, 8) == 0 ? "==" : "!=");
    } else if (V == 2) {
        double x = seed;
        for (long long i = 0; i < (long long)iters * 16; ++i) x = std::fma(x, b, c);
        std::snprintf(check, sizeof check, "  [lane 0 %s host]", std::memcmp(&x, &got, 8) == 0 ? "==" : "!=");
    } else if (V == 4) {
        double x = seed;
        for (long long i = 0; i < (long long)iters * 16; ++i) x = x + c;
        std::snprintf(check, sizeof check, "  [lane 0 %s host]", std::memcmp(&x, &got, 8) == 0 ? "==" : "!=");
    }
    std::printf("%-34s %6.2f cycles per instruction%s\n", kName[V], (double)cy / ((double)iters * kPerIter[V]), check);
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    double *out;
    long long *cyc;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, 8);
    const int iters = 2000;
    run<0>(out, cyc, iters); run<1>(out, cyc, iters); run<2>(out, cyc, iters); run<3>(out, cyc, iters);
    run<4>(out, cyc, iters); run<5>(out, cyc, iters); run<6>(out, cyc, iters); run<7>(out, cyc, iters);
    run<8>(out, cyc, iters); run<9>(out, cyc, iters); run<10>(out, cyc, iters); run<11>(out, cyc, iters);
    run<12>(out, cyc, iters); run<13>(out, cyc, iters); run<14>(out, cyc, iters); run<15>(out, cyc, iters);
    run<16>(out, cyc, iters); run<17>(out, cyc, iters);
    // s_memtime against the wall clock
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<0>, dim3(1), dim3(64), 0, 0, out, cyc, 400000, 1.25, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long cy;
    hipMemcpy(&cy, cyc, 8, hipMemcpyDeviceToHost);
    std::printf("s_memtime: %.3f GHz (ticks / wall)\n", cy / (ms * 1e6));
    return 0;
}
