// tools/loop_probe.hip -- diagnostic build of the symbol-sync/Costas loop kernel
// with s_memtime stamps: where do the consumer and loader waves spend cycles?
#define QPSK_LOOP_STAMPS 1
#include "../qpsk-modulator-demodulator_amd/csrc/qpsk_loop.hip"
#include <cstdio>
#include <vector>
#include <random>
using namespace qpsk;

// optional load beside the loop kernel (argv[4] = number of workgroups): one
// FMA-bound workgroup per CU (100 KB LDS keeps it off the loop's CUs), run on
// a second stream for ~2x the loop's time, to see whether the loop slows in
// cycles (contention) or only in wall time (clock)
// memory-bound variant: streams a large buffer (read + write) for the same time
__global__ void burn_mem_kernel(const float4 *src, float4 *dst, long long n4, long long ticks) {
  extern __shared__ float lds[];
  if (threadIdx.x == 0) lds[0] = 0.f;
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  const long long stride = (long long)gridDim.x * blockDim.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
  }
}
__global__ void burn_kernel(float *sink, long long ticks) {
  extern __shared__ float lds[];
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  float x = threadIdx.x, y = blockIdx.x;
  if (threadIdx.x == 0) lds[0] = x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
#pragma unroll 32
    for (int i = 0; i < 256; ++i) { x = x * 1.0000001f + 1e-7f; y = y * 0.9999999f + 1e-7f; }
  }
  if (x + y == 12345.0f) sink[threadIdx.x] = x;
}

int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 256;
  const int64_t n = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int spw = argc > 3 ? atoi(argv[3]) : 0;   // loop_variant: 0 auto, 1 16x64, 2 32x64, 3 16x128, 4 24x128
  const int64_t stride = ((kMfPrefix + n + 2 + 63) / 64) * 64;
  // 32 distinct noise rows, replicated over the batch (host generation of a
  // C3-sized batch would take minutes)
  const int SH = S < 32 ? S : 32;
  std::vector<float> h(2 * stride * (size_t)SH);
  std::mt19937 g(1); std::normal_distribution<float> nd(0.f, 0.3f);
  for (auto& v : h) v = nd(g);
  float *mf, *carry; StreamState* st; uint32_t* bits; int64_t *cnt; unsigned long long* probe;
  hipMalloc(&mf, 2 * stride * (size_t)S * 4);
  for (int r0 = 0; r0 < S; r0 += SH)
    hipMemcpy(mf + 2 * stride * (size_t)r0, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&carry, S * kCarryMax * 8); hipMemset(carry, 0, S * kCarryMax * 8);
  std::vector<StreamState> hs(S); for (auto& x : hs) { x = StreamState{}; x.base = 1; }
  hipMalloc(&st, S * sizeof(StreamState)); hipMemcpy(st, hs.data(), S * sizeof(StreamState), hipMemcpyHostToDevice);
  const int64_t words = n / 2;
  hipMalloc(&bits, S * words * 4); hipMalloc(&cnt, 2 * S * 8); hipMalloc(&probe, 16 * S * 8);
  hipMemset(probe, 0, 16 * S * 8);
  LoopArgs a{}; a.mf = mf; a.mf_stride = stride; a.carry = carry; a.n = n; a.state = st; a.bits = bits;
  a.bits_stride_words = words; a.bits_cap_words = words; a.n_bits = cnt; a.n_syms = cnt + S; a.S = S; a.probe = probe;
  LoopParams P{}; P.sps = argc > 6 ? atof(argv[6]) : 8.0; P.kp = 2.622462326512427e-3; P.ki = 3.443172085385801e-06; P.c_alpha = 0.13751550967894244; P.c_beta = 0.010184293139132996; P.differential = 1;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int burn = argc > 4 ? atoi(argv[4]) : 0;
  hipStream_t bs; hipStreamCreateWithFlags(&bs, hipStreamNonBlocking);
  float *sink; hipMalloc(&sink, 4096);
  const int burn_mem = argc > 5 ? atoi(argv[5]) : 0;
  float4 *bsrc = nullptr, *bdst = nullptr;
  const long long bn4 = (1LL << 30) / 16;   // 1 GiB each way
  if (burn > 0 && burn_mem) { hipMalloc(&bsrc, bn4 * 16); hipMalloc(&bdst, bn4 * 16); hipMemset(bsrc, 0, bn4 * 16); }
  auto burn_launch = [&]() {
    if (burn_mem) {
      hipFuncSetAttribute((const void *)burn_mem_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 100 << 10);
      hipLaunchKernelGGL(burn_mem_kernel, dim3(burn), dim3(1024), 100 << 10, bs, bsrc, bdst, bn4, 6000000LL);
    } else {
      hipFuncSetAttribute((const void *)burn_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 100 << 10);
      hipLaunchKernelGGL(burn_kernel, dim3(burn), dim3(256), 100 << 10, bs, sink, 6000000LL);   // 60 ms
    }
  };
  if (burn > 0) {
    burn_launch();
    hipDeviceSynchronize();   // warm: let the clock settle under the load once
    burn_launch();
  }
  const long long rt0 = 0; (void)rt0;
  hipEventRecord(e0);
  launch_loop(a, P, kModeDemodulate, spw, 0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> pr(16 * S); hipMemcpy(pr.data(), probe, pr.size() * 8, hipMemcpyDeviceToHost);
  int64_t ns; hipMemcpy(&ns, cnt + S, 8, hipMemcpyDeviceToHost);
  printf("S=%d n=%lld variant=%d burn=%d: %.3f ms, stream0 symbols %lld -> %.1f ns/symbol, WG0 M&M cycles %.3g -> %.2f GHz effective\n",
         S, (long long)n, spw, burn, ms, (long long)ns, ms * 1e6 / ns, (double)(pr[2] + pr[3]),
         (double)(pr[2] + pr[3]) / (ms * 1e6));
  const int wgs = spw == 0 || spw == 2 ? 32 : (spw == 4 ? 24 : 16);
  const int nwg = (S + wgs - 1) / wgs;
  for (int b = 0; b < nwg; ++b) {
    auto* p = &pr[16 * b];
    printf(" WG %2d:", b);
    for (int w = 0; w < 4; ++w) {
      const unsigned hw = (unsigned)p[12 + w]; const unsigned xcc = (unsigned)(p[12 + w] >> 32);
      printf(" w%d xcc%u se%u cu%2u simd%u |", w, xcc & 0xf, (hw >> 13) & 3, (hw >> 8) & 0xf, (hw >> 4) & 3);
    }
    printf(" M&M %.0f Costas %.0f cyc/sym\n", (double)p[3] / (p[4] & 0xfffff), (double)p[6] / (p[4] & 0xfffff));
  }
  for (int bi = 0; bi < 3; ++bi) {
    const int b = bi < 2 ? bi : nwg - 1;   // the first two and the last (maybe partial) workgroup
    auto* p = &pr[16 * b];
    const double R = (double)p[7];
    printf(" WG %d rounds %llu: per round cycles: loader wait %.0f bar %.0f issue %.0f | M&M bar %.0f loop %.0f | Costas bar %.0f loop %.0f | cyc/sym M&M %.0f Costas %.0f | M&M uniform-loop cycles/round %.0f (%.0f/sym) | Costas uniform %.0f/round (%.0f/sym) | M&M pre %.0f post %.0f\n",
           b, p[7], p[0] / R, (p[1] & 0xffffffffull) / R, (p[1] >> 32) / R, p[2] / R, p[3] / R, p[5] / R, p[6] / R, (double)p[3] / (p[4] & 0xfffff), (double)p[6] / (p[4] & 0xfffff), (double)(p[4] >> 20) / R, p[10] ? (double)(p[4] >> 20) / p[10] : 0.0, p[8] / R, p[9] ? (double)p[8] / p[9] : 0.0, (p[11] & 0xffffffffull) / R, (p[11] >> 32) / R);
  }
  return 0;
}
