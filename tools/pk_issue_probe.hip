// tools/pk_issue_probe.hip -- issue cost of gfx950 packed f32 ops for a lone
// wave: v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32, independent (4 chains
// round-robin) and dependent (one chain), each as ONE asm statement (no
// compiler padding inside).  Diagnostic only; vector stores only.
#include <hip/hip_runtime.h>
#include <cstdio>

#define R2(x) x x
#define R4(x) R2(x) R2(x)
#define R8(x) R4(x) R4(x)

template <int V>
__global__ void kern(float *out, long long *cyc, int iters) {
    float a = threadIdx.x * 1e-3f;
    long long t0, t1;
    asm volatile("v_mov_b32 v10, %0\n\tv_mov_b32 v11, %0\n\tv_mov_b32 v12, 1.0\n\tv_mov_b32 v13, -1.0\n\t"
                 "v_mov_b32 v14, %0\n\tv_mov_b32 v15, %0\n\tv_mov_b32 v16, %0\n\tv_mov_b32 v17, %0\n\t"
                 "v_mov_b32 v18, %0\n\tv_mov_b32 v19, %0\n\tv_mov_b32 v20, %0\n\tv_mov_b32 v21, %0"
                 :: "v"(a) : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21");
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (V == 0)   // independent pk_add, 4 chains
            asm volatile(R4("v_pk_add_f32 v[14:15], v[14:15], v[12:13]\n\tv_pk_add_f32 v[16:17], v[16:17], v[12:13]\n\t"
                            "v_pk_add_f32 v[18:19], v[18:19], v[12:13]\n\tv_pk_add_f32 v[20:21], v[20:21], v[12:13]\n\t")
                         ::: "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21");
        else if (V == 1)   // independent pk_fma, 4 chains
            asm volatile(R4("v_pk_fma_f32 v[14:15], v[14:15], v[12:13], v[10:11]\n\tv_pk_fma_f32 v[16:17], v[16:17], v[12:13], v[10:11]\n\t"
                            "v_pk_fma_f32 v[18:19], v[18:19], v[12:13], v[10:11]\n\tv_pk_fma_f32 v[20:21], v[20:21], v[12:13], v[10:11]\n\t")
                         ::: "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21");
        else if (V == 2)   // independent pk_mul, 4 chains
            asm volatile(R4("v_pk_mul_f32 v[14:15], v[14:15], v[12:13]\n\tv_pk_mul_f32 v[16:17], v[16:17], v[12:13]\n\t"
                            "v_pk_mul_f32 v[18:19], v[18:19], v[12:13]\n\tv_pk_mul_f32 v[20:21], v[20:21], v[12:13]\n\t")
                         ::: "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21");
        else if (V == 3)   // dependent pk_add chain (with the s_nop 0 gfx950 wants between)
            asm volatile(R8("v_pk_add_f32 v[14:15], v[14:15], v[12:13]\n\ts_nop 0\n\t") R8("v_pk_add_f32 v[14:15], v[14:15], v[12:13]\n\ts_nop 0\n\t") ::: "v14", "v15");
        else if (V == 4)   // dependent pk_fma chain (with s_nop 0)
            asm volatile(R8("v_pk_fma_f32 v[14:15], v[14:15], v[12:13], v[10:11]\n\ts_nop 0\n\t") R8("v_pk_fma_f32 v[14:15], v[14:15], v[12:13], v[10:11]\n\ts_nop 0\n\t") ::: "v14", "v15");
        else if (V == 5)   // independent f32 fma (VOP3), 4 chains
            asm volatile(R4("v_fma_f32 v14, v14, v12, v10\n\tv_fma_f32 v16, v16, v12, v10\n\tv_fma_f32 v18, v18, v12, v10\n\tv_fma_f32 v20, v20, v12, v10\n\t")
                         ::: "v14", "v16", "v18", "v20");
    }
    t1 = __builtin_amdgcn_s_memtime();
    float r;
    asm volatile("v_mov_b32 %0, v14" : "=v"(r));
    out[threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

static const char *kName[] = {"independent v_pk_add_f32", "independent v_pk_fma_f32", "independent v_pk_mul_f32",
                              "dependent v_pk_add_f32 + s_nop 0", "dependent v_pk_fma_f32 + s_nop 0", "independent v_fma_f32"};
static const int kPer[] = {16, 16, 16, 16, 16, 16};

template <int V>
static void run(float *out, long long *cyc) {
    const int iters = 4000;
    hipLaunchKernelGGL(kern<V>, dim3(1), dim3(64), 0, 0, out, cyc, 8);
    hipLaunchKernelGGL(kern<V>, dim3(1), dim3(64), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    std::printf("%-36s %6.2f cycles per op (loop branch included)\n", kName[V], (double)c / ((double)iters * kPer[V]));
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    float *out;
    long long *cyc;
    hipMalloc(&out, 256);
    hipMalloc(&cyc, 8);
    run<0>(out, cyc); run<1>(out, cyc); run<2>(out, cyc); run<3>(out, cyc); run<4>(out, cyc); run<5>(out, cyc);
    return 0;
}
