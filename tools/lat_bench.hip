// tools/lat_bench.hip -- dependent-chain latency of single gfx950 VALU idioms
// (v_max_f64, v_cmp->v_cndmask through VCC, v_bfi), one wave.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int V>
__global__ void k(double *out, long long *cyc, int n) {
    double x = 1.0 + threadIdx.x * 1e-3, y = 0.5;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (V == 0) x = x * 1.0000001;                          // dep mul_f64
            if (V == 1) x = __builtin_fmax(x, y) * 1.0000001;        // max + mul
            if (V == 2) x = (x > y ? x : y) * 1.0000001;             // cmp/cndmask + mul
            if (V == 3) x = (fabs(x) > 3.0 ? x - 6.0 : x) + 1e-9;    // wrap-like select + add
            if (V == 4) {                                            // bfi sign + mul
                union { double d; unsigned long long u; } a; a.d = x;
                a.u = (a.u & 0x7fffffffffffffffull) | ((a.u << 1) & 0x8000000000000000ull);
                x = a.d * 1.0000001;
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <int V> void run(const char *nm, double *o, long long *c) {
    hipLaunchKernelGGL(k<V>, dim3(1), dim3(64), 0, 0, o, c, 1000);
    long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("%-32s %6.1f cycles per step\n", nm, h / 16000.0);
}
int main() {
    double *o; long long *c; hipMalloc(&o, 512); hipMalloc(&c, 8);
    run<0>("mul_f64", o, c);
    run<1>("max_f64 + mul_f64", o, c);
    run<2>("cmp/cndmask + mul_f64", o, c);
    run<3>("cmp/cndmask select + add_f64", o, c);
    run<4>("bit ops + mul_f64", o, c);
    return 0;
}
