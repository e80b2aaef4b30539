// tools/mfma_f32_probe.hip -- can the f32 multi-block MFMAs form the matched
// filter's products?  The reference FIR rounds every product and every add
// separately (FIRFilter.cs:165-180, no FMA), so an MFMA may only supply the
// products: D = A*B + C with K = 1 and C = -0 is round(A*B), the same bits as
// v_mul_f32 (signed zeros included) if the unit rounds like fmaf.
//
//   1. D-register layout of v_mfma_f32_{4x4x1_16b,16x16x1_4b,32x32x1_2b}_f32
//   2. exactness: D vs the host's IEEE float product on random bit patterns,
//      normals, denormal products, signed zeros
//   3. issue cost: back-to-back MFMAs with k v_pk_add_f32 per MFMA consuming
//      the previous MFMA's products, one and two waves per SIMD
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/mfma_f32_probe.hip -o tools/bin/mfma_f32_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f32v __attribute__((ext_vector_type(32)));
typedef float f2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

// one wave: D for given per-lane A, B (C = -0)
__global__ void mfma_once(const float *A, const float *B, float *D4, float *D16, float *D32) {
    const int l = threadIdx.x;
    const float a = A[l], b = B[l];
    f4 c4;
    for (int i = 0; i < 4; ++i) c4[i] = -0.0f;
    f16v c16;
    for (int i = 0; i < 16; ++i) c16[i] = -0.0f;
    f32v c32;
    for (int i = 0; i < 32; ++i) c32[i] = -0.0f;
    const f4 d4 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c4, 0, 0, 0);
    const f16v d16 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c16, 0, 0, 0);
    const f32v d32 = __builtin_amdgcn_mfma_f32_32x32x1f32(a, b, c32, 0, 0, 0);
    for (int i = 0; i < 4; ++i) D4[i * 64 + l] = d4[i];
    for (int i = 0; i < 16; ++i) D16[i * 64 + l] = d16[i];
    for (int i = 0; i < 32; ++i) D32[i * 64 + l] = d32[i];
}

// timing: ITER x (MFMA of form F on fresh operands, NADD packed adds of the
// previous MFMA's D into accumulators); unrolled by two so the D buffers
// alternate (no copies).  Build with -mllvm -amdgpu-mfma-vgpr-form=1 so D
// lands in VGPRs as the FIR would use it.
template <int F> struct DV;
template <> struct DV<4> { typedef f4 t; static constexpr int n = 4; };
template <> struct DV<16> { typedef f16v t; static constexpr int n = 16; };
template <> struct DV<32> { typedef f32v t; static constexpr int n = 32; };
template <int F>
__device__ __forceinline__ typename DV<F>::t mfma1(float a, float b, typename DV<F>::t c) {
    if constexpr (F == 4) return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    else if constexpr (F == 16) return __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_32x32x1f32(a, b, c, 0, 0, 0);
}
template <int F, int NADD>
__global__ __launch_bounds__(256) void mfma_rate(const float *in, float *out, unsigned long long *cyc, int iters) {
    typedef typename DV<F>::t dv;
    constexpr int ND = DV<F>::n;
    const int l = threadIdx.x & 63;
    float a = in[l], b = in[64 + l];
    f2 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f2{0.f, 0.f};
    dv cz;
    for (int i = 0; i < ND; ++i) cz[i] = -0.f;
    dv d0 = cz, d1 = cz;
    auto adds = [&](const dv &d) {
#pragma unroll
        for (int k = 0; k < NADD; ++k) {
            const f2 p = f2{d[(2 * k) % ND], d[(2 * k + 1) % ND]};
            acc[k % 16] = acc[k % 16] + p;
        }
    };
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it += 2) {
        d0 = mfma1<F>(a, b, cz);
        adds(d1);
        a = a + 1.0f;
        d1 = mfma1<F>(a, b, cz);
        adds(d0);
        b = b * 0.5f;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    f2 s = f2{0.f, 0.f};
    for (int i = 0; i < 16; ++i) s = s + acc[i];
    float t = 0.f;
    for (int i = 0; i < ND; ++i) t += d0[i] + d1[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + t;
    if (l == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

// VALU-only reference: the same products on v_pk_mul_f32 + the adds
template <int NMUL>
__global__ __launch_bounds__(256) void valu_rate(const float *in, float *out, unsigned long long *cyc, int iters) {
    const int l = threadIdx.x & 63;
    f2 x[NMUL];
    for (int i = 0; i < NMUL; ++i) x[i] = f2{in[l] + i, in[64 + l] - i};
    float h = in[128 + l];
    f2 acc[NMUL];
    for (int i = 0; i < NMUL; ++i) acc[i] = f2{0.f, 0.f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NMUL; ++i) acc[i] = acc[i] + h * x[i];
        h = h * 0.999f;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    f2 s = f2{0.f, 0.f};
    for (int i = 0; i < NMUL; ++i) s = s + acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
    if (l == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

static float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

template <typename K>
static double time_kernel(K kern, int blocks, int threads, const float *din, float *dout,
                          unsigned long long *dcyc, int iters, double *cyc_per_iter) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, dcyc, iters);   // warm
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, dcyc, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const int nw = blocks * threads / 64;
    std::vector<unsigned long long> c(nw);
    CHECK(hipMemcpy(c.data(), dcyc, nw * 8, hipMemcpyDeviceToHost));
    double s = 0;
    for (auto v : c) s += v;
    *cyc_per_iter = s / nw / iters;
    return ms;
}

int main() {
    // ---- 1. layout
    float *dA, *dB, *dD4, *dD16, *dD32;
    CHECK(hipMalloc(&dA, 256 * 4));
    CHECK(hipMalloc(&dB, 256 * 4));
    CHECK(hipMalloc(&dD4, 4 * 64 * 4));
    CHECK(hipMalloc(&dD16, 16 * 64 * 4));
    CHECK(hipMalloc(&dD32, 32 * 64 * 4));
    std::vector<float> A(64), B(64), D4(256), D16(1024), D32(2048);
    auto run = [&]() {
        CHECK(hipMemcpy(dA, A.data(), 256, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dB, B.data(), 256, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(mfma_once, dim3(1), dim3(64), 0, 0, dA, dB, dD4, dD16, dD32);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(D4.data(), dD4, 4 * 256, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(D16.data(), dD16, 16 * 256, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(D32.data(), dD32, 32 * 256, hipMemcpyDeviceToHost));
    };
    // A = lane + 1, B = 1 -> D says which A lane; then the reverse for B
    for (int l = 0; l < 64; ++l) { A[l] = l + 1; B[l] = 1.0f; }
    run();
    std::vector<float> a4 = D4, a16 = D16, a32 = D32;
    for (int l = 0; l < 64; ++l) { A[l] = 1.0f; B[l] = l + 1; }
    run();
    auto show = [](const char *name, const std::vector<float> &da, const std::vector<float> &db, int nreg) {
        printf("%s: D[reg][lane] = A[lane a] * B[lane b]  (a,b), lanes 0..%d\n", name, 63);
        for (int r = 0; r < nreg; ++r) {
            printf("  reg %2d:", r);
            for (int l = 0; l < 64; ++l) printf(" %d,%d", (int)da[r * 64 + l] - 1, (int)db[r * 64 + l] - 1);
            printf("\n");
        }
    };
    const std::vector<float> b4 = D4, b16 = D16, b32 = D32;
    show("4x4x1_16b", a4, b4, 4);
    show("16x16x1_4b", a16, b16, 16);
    show("32x32x1_2b", a32, b32, 32);

    // ---- 2. exactness (16x16x1 form: every (A lane, B lane) pair of a block)
    std::mt19937 rng(1234);
    long bad[3] = {0, 0, 0}, tot[3] = {0, 0, 0};
    long badz = 0, badd = 0;
    for (int trial = 0; trial < 3000; ++trial) {
        const int kind = trial % 6;
        for (int l = 0; l < 64; ++l) {
            uint32_t ua = rng(), ub = rng();
            if (kind == 0) { A[l] = bits2f(ua); B[l] = bits2f(ub); }
            else if (kind == 1) { A[l] = (float)std::normal_distribution<double>(0, 1)(rng);
                                  B[l] = (float)std::normal_distribution<double>(0, 0.3)(rng); }
            else if (kind == 2) {   // denormal products: tiny * small
                A[l] = ldexpf((float)(rng() % 100000 + 1) / 100000.0f, -(int)(rng() % 30) - 100);
                B[l] = ldexpf((float)(rng() % 100000 + 1) / 100000.0f, -(int)(rng() % 30));
                if (rng() & 1) A[l] = -A[l];
            } else if (kind == 3) {   // signed zeros mixed in
                A[l] = (rng() & 3) == 0 ? ((rng() & 1) ? 0.0f : -0.0f) : (float)std::normal_distribution<double>(0, 1)(rng);
                B[l] = (rng() & 3) == 0 ? ((rng() & 1) ? 0.0f : -0.0f) : (float)std::normal_distribution<double>(0, 1)(rng);
            } else if (kind == 4) {   // denormal inputs
                A[l] = bits2f((rng() & 0x807fffffu));
                B[l] = (float)std::normal_distribution<double>(0, 4)(rng);
            } else {   // products near overflow / underflow rounding boundaries
                A[l] = ldexpf(1.0f + (float)(rng() % 1000) / 1000.0f, (int)(rng() % 250) - 125);
                B[l] = ldexpf(1.0f + (float)(rng() % 1000) / 1000.0f, (int)(rng() % 250) - 125);
            }
        }
        run();
        auto chk = [&](int form, const std::vector<float> &D, const std::vector<float> &la, const std::vector<float> &lb, int nreg) {
            for (int r = 0; r < nreg; ++r)
                for (int l = 0; l < 64; ++l) {
                    const int ia = (int)la[r * 64 + l] - 1, ib = (int)lb[r * 64 + l] - 1;
                    const float want = A[ia] * B[ib];
                    const float got = D[r * 64 + l];
                    const bool same = f2bits(want) == f2bits(got) || (std::isnan(want) && std::isnan(got));
                    ++tot[form];
                    if (!same) {
                        ++bad[form];
                        if (want == 0.0f) ++badz;
                        else if (std::fabs(want) < 1.17549435e-38f) ++badd;
                        if (bad[form] <= 4)
                            printf("  mismatch form %d kind %d: %a * %a = %a, mfma %a\n", form, kind, A[ia], B[ib], want, got);
                    }
                }
        };
        chk(0, D4, a4, b4, 4);
        chk(1, D16, a16, b16, 16);
        chk(2, D32, a32, b32, 32);
    }
    printf("exactness vs host IEEE product (C = -0): 4x4 %ld/%ld bad, 16x16 %ld/%ld bad, 32x32 %ld/%ld bad "
           "(of the bad: %ld zero results, %ld denormal results)\n",
           bad[0], tot[0], bad[1], tot[1], bad[2], tot[2], badz, badd);

    // ---- 3. issue cost
    float *din, *dout;
    unsigned long long *dcyc;
    CHECK(hipMalloc(&din, 256 * 4));
    CHECK(hipMalloc(&dout, 1 << 22));
    CHECK(hipMalloc(&dcyc, 1 << 20));
    std::vector<float> hin(256);
    for (int i = 0; i < 256; ++i) hin[i] = 0.5f + 0.001f * i;
    CHECK(hipMemcpy(din, hin.data(), 256 * 4, hipMemcpyHostToDevice));
    const int iters = 20000;
    int dev = 0;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, dev));
    const int cus = prop.multiProcessorCount;
    double cpi;
    for (int wps = 1; wps <= 2; ++wps) {
        const int blocks = cus * wps;   // 256 threads = 4 waves = one per SIMD
        printf("-- %d wave(s) per SIMD, %d blocks of 256\n", wps, blocks);
#define T(F, N)                                                                                     \
    {                                                                                               \
        double ms = time_kernel(mfma_rate<F, N>, blocks, 256, din, dout, dcyc, iters, &cpi);        \
        const double prod = (F == 4 ? 256.0 : 1024.0) * blocks * 4 * iters;                         \
        printf("  mfma %2dx%-2d + %2d pk_add: %6.1f cyc/iter (s_memtime), %.3f ms, %.2f Tproducts/s\n", F, \
               F, N, cpi, ms, prod / ms / 1e9);                                                     \
    }
        T(4, 0) T(4, 2) T(4, 4) T(4, 6)
        T(16, 0) T(16, 4) T(16, 8) T(16, 12)
        T(32, 0) T(32, 8) T(32, 16)
#undef T
        {
            double ms = time_kernel(valu_rate<8>, blocks, 256, din, dout, dcyc, iters, &cpi);
            const double prod = 16.0 * 64 * blocks * 4 * iters;
            printf("  valu 8 pk_mul + 8 pk_add:   %6.1f cyc/iter, %.3f ms, %.2f Tproducts/s\n", cpi, ms, prod / ms / 1e9);
        }
    }
    return 0;
}
