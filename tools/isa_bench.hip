// tools/isa_bench.hip -- single-wave issue/latency microbenchmarks on gfx950,
// to model the per-symbol cost of the serial loops in qpsk_loop.hip.
// Diagnostic only.  Prints cycles (s_memtime ticks) per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int V>
__global__ void kern(double *out, long long *cyc, int iters) {
    __shared__ double lds[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = 0.0;
    __syncthreads();
    double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999, c = 1e-7, d = 2.0, e = 3.0, f = 4.0;
    float fa = 1.0f + threadIdx.x * 1e-6f, fb = 0.9999f, fc = 1e-7f;
    int ia = threadIdx.x, ib = 3;
    unsigned addr = (threadIdx.x & 63) * 8;
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v pa = {fa, fa}, pb = {0.9999f, 1.0001f}, pc = pa, pd = pa, pe = pa;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (V == 0) {   // dependent v_fma_f64 chain
            REP64(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));)
        } else if (V == 1) {   // 4 independent f64 fma chains, interleaved
            REP8(REP8(asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_fma_f64 %1, %1, %4, %5\n\t"
                                   "v_fma_f64 %2, %2, %4, %5\n\tv_fma_f64 %3, %3, %4, %5"
                                   : "+v"(a), "+v"(d), "+v"(e), "+v"(f) : "v"(b), "v"(c));))
        } else if (V == 2) {   // dependent v_fma_f32 chain
            REP64(asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(fa) : "v"(fb), "v"(fc));)
        } else if (V == 3) {   // independent f32 fma x4
            float fd = fa, fe = fa, ff = fa;
            REP8(REP8(asm volatile("v_fma_f32 %0, %0, %4, %5\n\tv_fma_f32 %1, %1, %4, %5\n\t"
                                   "v_fma_f32 %2, %2, %4, %5\n\tv_fma_f32 %3, %3, %4, %5"
                                   : "+v"(fa), "+v"(fd), "+v"(fe), "+v"(ff) : "v"(fb), "v"(fc));))
            fa += fd + fe + ff;
        } else if (V == 4) {   // dependent v_add_u32 chain
            REP64(asm volatile("v_add_u32 %0, %0, %1" : "+v"(ia) : "v"(ib));)
        } else if (V == 5) {   // dependent LDS read chain (address from previous data)
            REP64(asm volatile("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)" : "+v"(addr));)
        } else if (V == 6) {   // dependent f64 fma with an independent f64 fma between
            REP8(REP8(asm volatile("v_fma_f64 %0, %0, %2, %3\n\tv_fma_f64 %1, %1, %2, %3"
                                   : "+v"(a), "+v"(d) : "v"(b), "v"(c));))
        } else if (V == 7) {   // dependent v_mul_f64 chain
            REP64(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(b));)
        } else if (V == 8) {   // f64 fma chain + v_cndmask pair between
            REP64(asm volatile("v_fma_f64 %0, %0, %2, %3\n\tv_cndmask_b32 %1, %1, %4, vcc" : "+v"(a), "+v"(ia) : "v"(b), "v"(c), "v"(ib) : "vcc");)
        } else if (V == 9) {   // dependent v_rndne_f64 / v_floor style (trans-like) chain
            REP64(asm volatile("v_floor_f64 %0, %0" : "+v"(a));)
        } else if (V == 10) {  // dependent v_cvt_f64_f32 -> v_cvt_f32_f64 pairs
            REP64(asm volatile("v_cvt_f64_f32 %0, %1\n\tv_cvt_f32_f64 %1, %0" : "+v"(a), "+v"(fa));)
        } else if (V == 11) {  // dependent v_add_f64 chain
            REP64(asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(b));)
        } else if (V == 13) {  // dependent v_pk_add_f32 chain
            REP64(asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(pa) : "v"(pb));)
        } else if (V == 14) {  // dependent v_pk_mul_f32 chain
            REP64(asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pa) : "v"(pb));)
        } else if (V == 15) {  // dependent v_add_f32 chain
            REP64(asm volatile("v_add_f32 %0, %0, %1" : "+v"(fa) : "v"(fb));)
        } else if (V == 16) {  // dependent v_add_f32_dpp row_shr:2 chain (2 wait states each)
            REP64(asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %0, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(fa) : "v"(fb));)
        } else if (V == 17) {  // 4 independent v_pk_add_f32 chains, interleaved
            REP8(REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n\tv_pk_add_f32 %1, %1, %4\n\t"
                                   "v_pk_add_f32 %2, %2, %4\n\tv_pk_add_f32 %3, %3, %4"
                                   : "+v"(pa), "+v"(pc), "+v"(pd), "+v"(pe) : "v"(pb));))
        } else if (V == 18) {  // dependent pk_add with op_sel swap + neg (the FLL combine)
            REP64(asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "+v"(pa) : "v"(pb));)
        } else if (V == 19) {  // dependent v_cvt_f32_f64 -> v_pk_mul_f32 (f64 result into packed)
            REP64(asm volatile("v_cvt_f64_f32 %0, %1\n\tv_pk_mul_f32 %2, %2, %3\n\tv_cvt_f32_f64 %1, %0" : "+v"(a), "+v"(fa), "+v"(pa) : "v"(pb));)
        } else if (V == 20) {  // 4 independent v_mul_f64 chains
            REP8(REP8(asm volatile("v_mul_f64 %0, %0, %4\n\tv_mul_f64 %1, %1, %4\n\t"
                                   "v_mul_f64 %2, %2, %4\n\tv_mul_f64 %3, %3, %4"
                                   : "+v"(a), "+v"(d), "+v"(e), "+v"(f) : "v"(b));))
        } else if (V == 21) {  // 4 independent v_add_f64 chains
            REP8(REP8(asm volatile("v_add_f64 %0, %0, %4\n\tv_add_f64 %1, %1, %4\n\t"
                                   "v_add_f64 %2, %2, %4\n\tv_add_f64 %3, %3, %4"
                                   : "+v"(a), "+v"(d), "+v"(e), "+v"(f) : "v"(b));))
        } else if (V == 22) {  // 4 independent fma_f64 chains, lanes 0..31 only
            if (threadIdx.x % 64 < 32) {
                REP8(REP8(asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_fma_f64 %1, %1, %4, %5\n\t"
                                       "v_fma_f64 %2, %2, %4, %5\n\tv_fma_f64 %3, %3, %4, %5"
                                       : "+v"(a), "+v"(d), "+v"(e), "+v"(f) : "v"(b), "v"(c));))
            }
        } else if (V == 23) {  // 2 independent fma_f64 chains + 2 independent add_u32 chains
            int ic = ia;
            REP8(REP8(asm volatile("v_fma_f64 %0, %0, %4, %5\n\tv_add_u32 %2, %2, %6\n\t"
                                   "v_fma_f64 %1, %1, %4, %5\n\tv_add_u32 %3, %3, %6"
                                   : "+v"(a), "+v"(d), "+v"(ia), "+v"(ic) : "v"(b), "v"(c), "v"(ib));))
            ia += ic;
        } else if (V == 24) {  // 4 independent v_mov_b64
            REP8(REP8(asm volatile("v_mov_b64 %0, %4\n\tv_mov_b64 %1, %4\n\t"
                                   "v_mov_b64 %2, %4\n\tv_mov_b64 %3, %4"
                                   : "=v"(a), "=v"(d), "=v"(e), "=v"(f) : "v"(b));))
        } else if (V == 25) {  // 4 independent v_cmp_le_f64 -> distinct SGPR pairs
            unsigned long long m0, m1, m2, m3;
            REP8(REP8(asm volatile("v_cmp_le_f64 %0, %4, %5\n\tv_cmp_le_f64 %1, %4, %6\n\t"
                                   "v_cmp_le_f64 %2, %5, %6\n\tv_cmp_le_f64 %3, %6, %4"
                                   : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3) : "v"(a), "v"(b), "v"(c));))
            ia += (int)(m0 + m1 + m2 + m3);
        } else if (V == 26) {  // dependent f64 chain: mul, add, add (kb -> k shape)
            REP8(REP8(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));))
            REP8(REP8(asm volatile("v_add_f64 %0, %0, %1" : "+v"(d) : "v"(b));))
        } else if (V == 27) {  // ds_read_b128 dependent chain (address from data)
            REP64(asm volatile("ds_read_b128 v[100:103], %0\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 %0, v100" : "+v"(addr) :: "v100", "v101", "v102", "v103");)
        } else if (V == 12) {  // scalar op stream (s_mov: leaves SCC, which the loop branch uses, alone)
            int sa = it, sb = 7;
            REP64(asm volatile("s_mov_b32 %0, %1" : "=s"(sa) : "s"(sb));)
            ia += sa;
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x + blockIdx.x * blockDim.x] = a + d + e + f + fa + ia + addr + pa.x + pc.y + pd.x + pe.y;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    double *out; long long *cyc;
    hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 4096);
    const char *names[] = {"dep fma_f64", "4x indep fma_f64", "dep fma_f32", "4x indep fma_f32",
                           "dep add_u32", "dep ds_read_b32+wait", "2 chains fma_f64",
                           "dep mul_f64", "fma_f64 + cndmask", "dep floor_f64",
                           "cvt f32<->f64 pair", "dep add_f64", "scalar s_add", "dep pk_add_f32",
                           "dep pk_mul_f32", "dep add_f32", "dep add_f32_dpp+nop1", "4x indep pk_add",
                           "dep pk_add opsel/neg", "cvt>pk_mul>cvt", "4x indep mul_f64", "4x indep add_f64",
                           "4x indep fma_f64 32 lanes", "2 fma_f64 + 2 add_u32", "4x v_mov_b64",
                           "4x v_cmp_le_f64", "fma_f64 chain + add_f64 chain (seq)", "dep ds_read_b128+mov"};
    const int iters = 1000;
    auto run = [&](auto kfn, int idx, int waves_per_block, int blocks) {
        hipLaunchKernelGGL(kfn, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, cyc, 10);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(kfn, dim3(blocks), dim3(64 * waves_per_block), 0, 0, out, cyc, iters);
        hipDeviceSynchronize();
        long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-24s waves/blk %d: %.2f ticks per instruction\n", names[idx], waves_per_block,
               (double)c / (iters * 64.0));
    };
    for (int w : {1, 4}) {
        run(kern<0>, 0, w, 1); run(kern<1>, 1, w, 1); run(kern<2>, 2, w, 1); run(kern<3>, 3, w, 1);
        run(kern<4>, 4, w, 1); run(kern<5>, 5, w, 1); run(kern<6>, 6, w, 1); run(kern<7>, 7, w, 1);
        run(kern<8>, 8, w, 1); run(kern<9>, 9, w, 1); run(kern<10>, 10, w, 1); run(kern<11>, 11, w, 1);
        run(kern<12>, 12, w, 1); run(kern<13>, 13, w, 1); run(kern<14>, 14, w, 1);
        run(kern<15>, 15, w, 1); run(kern<16>, 16, w, 1); run(kern<17>, 17, w, 1);
        run(kern<18>, 18, w, 1); run(kern<19>, 19, w, 1);
        run(kern<20>, 20, w, 1); run(kern<21>, 21, w, 1); run(kern<22>, 22, w, 1);
        run(kern<23>, 23, w, 1); run(kern<24>, 24, w, 1); run(kern<25>, 25, w, 1);
        run(kern<26>, 26, w, 1); run(kern<27>, 27, w, 1);
    }
    // s_memtime rate: ticks over a wall-clock interval
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern<0>, dim3(1), dim3(64), 0, 0, out, cyc, 200000);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("s_memtime: %.3f GHz (ticks / wall)\n", c / (ms * 1e6));
    return 0;
}
