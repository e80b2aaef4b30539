// tools/loop_latency.hip -- microbenchmark of the per-symbol dependency chain of
// the symbol-sync + Costas loop (qpsk_loop.hip) with operands in registers, to
// separate compute latency from memory/LDS effects.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include "../qpsk-modulator-demodulator_amd/csrc/qpsk_sincos.h"

__device__ __forceinline__ long long stamp() { return __builtin_amdgcn_s_memtime(); }

template <int V>
__global__ void k(double* out, long long* cyc, int iters) {
  double theta = 0.1 * threadIdx.x, freq = 0.0, mu = 0.3, integ = 0.0;
  float xi = 0.5f + threadIdx.x * 1e-3f, xq = -0.4f;
  float pdi = 1, pdq = -1, psi = 0.3f, psq = 0.2f;
  double acc = 0.0;
  float facc = 1.0f;
  long long base = 1;
  __builtin_amdgcn_s_waitcnt(0);
  long long t0 = stamp();
  for (int it = 0; it < iters; ++it) {
    if (V == 0 || V == 2) {   // M&M step (float interp + double loop)
      const float t = (float)mu;
      const float tm1 = t - 1.0f, tm2 = t - 2.0f, tp1 = t + 1.0f;
      const float cm1 = -(t * tm1 * tm2) * (1.0f / 6.0f);
      const float c0 = (tp1 * tm1 * tm2) * (1.0f / 2.0f);
      const float c1 = -(tp1 * t * tm2) * (1.0f / 2.0f);
      const float c2 = (tp1 * t * tm1) * (1.0f / 6.0f);
      const float ci = cm1 * xi + c0 * xq + c1 * xi + c2 * xq;
      const float cq = cm1 * xq + c0 * xi + c1 * xq + c2 * xi;
      const float di = ci >= 0.0f ? 1.0f : -1.0f, dq = cq >= 0.0f ? 1.0f : -1.0f;
      const double t1 = (double)pdi * ci + (double)pdq * cq;
      const double t2 = (double)di * psi + (double)dq * psq;
      const double e = t1 - t2;
      integ += 3.4e-6 * e;
      double corr = 2.6e-3 * e + integ;
      corr = corr > 0.1 ? 0.1 : corr; corr = corr < -0.1 ? -0.1 : corr;
      const double nt = (double)base + mu + (8.0 + corr);
      const double fl = floor(nt);
      base = (long long)fl; mu = nt - fl;
      psi = ci; psq = cq; pdi = di; pdq = dq;
      xi = ci; xq = cq;   // feed back to keep the chain
      if (V == 2) acc += ci;
    }
    if (V == 0 || V == 1) {   // Costas step
      double sn, cs;
      qpsk_sincos(theta, &sn, &cs);
      const double mi = (double)xi * cs + (double)xq * sn;
      const double mq = (double)xq * cs - (double)xi * sn;
      const float ri = (float)mi, rq = (float)mq;
      const float ei = ri >= 0.0f ? 1.0f : -1.0f, eq = rq >= 0.0f ? 1.0f : -1.0f;
      const double pe = (double)ei * mq - (double)eq * mi;
      freq += 0.0101 * pe;
      theta += freq + 0.1375 * pe;
      theta = theta > 3.14159265358979311600 ? theta - 6.283185307179586 : (theta < -3.14159265358979311600 ? theta + 6.283185307179586 : theta);
      acc += ri;
    }
    if (V == 3) {   // sincos chain only
      double sn, cs;
      qpsk_sincos(theta, &sn, &cs);
      theta = sn + 0.5 * cs;
    }
    if (V == 4) {   // 16 dependent fma f64
#pragma unroll
      for (int j = 0; j < 16; ++j) theta = fma(theta, 0.999, 1e-3);
    }
    if (V == 5) {   // 16 dependent fma f32
#pragma unroll
      for (int j = 0; j < 16; ++j) facc = fmaf(facc, 0.999f, 1e-3f);
    }
    if (V == 6) {   // 16 dependent add f64
#pragma unroll
      for (int j = 0; j < 16; ++j) theta = theta + 1e-3 * (double)j;
    }
  }
  long long t1 = stamp();
  out[threadIdx.x + blockIdx.x * blockDim.x] = acc + theta + facc + mu + integ + (double)base;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V> void run(const char* name, int iters, int blocks) {
  double* out; long long* cyc;
  hipMalloc(&out, 64 * blocks * sizeof(double));
  hipMalloc(&cyc, blocks * sizeof(long long));
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, out, cyc, 100);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(64), 0, 0, out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long c; hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-28s blocks=%4d  %8.1f cycles/iter (memtime)  %8.1f ns/iter (wall)\n", name, blocks,
         (double)c / iters, ms * 1e6 / iters);
  hipFree(out); hipFree(cyc);
}

int main() {
  const int it = 20000;
  for (int b : {1, 256}) {
    run<0>("full M&M+Costas", it, b);
    run<1>("Costas only", it, b);
    run<2>("M&M only", it, b);
    run<3>("sincos chain", it, b);
    run<4>("16 dep fma f64", it, b);
    run<5>("16 dep fma f32", it, b);
    run<6>("16 dep add f64", it, b);
  }
  return 0;
}
