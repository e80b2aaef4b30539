// tools/mm_bench.hip -- cycles per symbol of the Mueller-Muller step of
// qpsk_loop.hip in isolation (one wave, 32 active lanes, an LDS sample ring per
// lane as in the loop kernel), with variants that stub out one piece each, to
// see where the M&M chain's time goes beyond 4 cycles per instruction (round 6,
// VERDICT r05 "locate the M&M's ~75 unexplained cycles").  The step below is
// the loop kernel's (interp, TED, PI, clamp, advance, tap address, symbol
// store), copied so each piece can be switched off; diagnostic only.
//
//   V0  the kernel's step (float symbol slot, ds_write_b64)
//   V1  no symbol store
//   V2  taps from registers: no LDS read and no tap address on the chain
//   V3  taps from LDS at an address off the chain (a counter): the read is
//       issued early, its latency hidden
//   V4  no clamp (corr = c)
//   V5  the TED without the decision doubles (e from the sums alone)
//   V6  double symbol slot (ds_write_b128, the layout before round 6)
//   V7  V3 + V1
//   V8  V0 with ring rows of 262 float2 instead of 260 (2-way instead of
//       4-way bank conflicts on the tap reads when all lanes sit at one position)
//   V9  V0 with rows of 261 float2 (conflict-free; not 16-B aligned, bench only)
//   V10 V0 with per-lane timing phases spread over the ring (random banks)
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef double d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const f2 lds_f2;

constexpr int kRing = 256, kRS = 29;
template <int V> constexpr int row_of() { return V == 8 ? 262 : (V == 9 ? 261 : 260); }

template <int V>
__global__ __launch_bounds__(64) void mm(const f2 *src, float *out_g, long long *cyc, int reps, double sps) {
    constexpr int kRow = row_of<V>();
    __shared__ f2 ring[32 * 262];
    __shared__ f2 symf[32 * kRS];
    __shared__ d2 symd[32 * kRS];
    const int lane = threadIdx.x;
    for (int i = lane; i < 32 * 262; i += 64) ring[i] = src[i];
    __syncthreads();
    if (lane >= 32) return;
    const double kp = 2.622462326512427e-3, ki = 3.443172085385801e-06;
    double clamp_hi = 0.1, clamp_lo = -0.1;
    asm volatile("" : "+v"(clamp_hi), "+v"(clamp_lo));
    f2 *row = ring + lane * kRow;
    uint32_t tap0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_f2 *)(row + 4 - 3)));
    asm volatile("" : "+v"(tap0));
    const double tap_shift = 6755399441055744.0 + 2.0;
    auto taps_fl = [&](double fl) -> lds_f2 * {
        union { double v; unsigned long long u; } kb;
        kb.v = fl + tap_shift;
        const uint32_t idx = static_cast<uint32_t>(kb.u) & (kRing - 1);
        uint32_t addr;
        asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(addr) : "v"(idx), "v"(tap0));
        return reinterpret_cast<lds_f2 *>(static_cast<uintptr_t>(addr));
    };
    double nt = (V == 10 ? 5.0 + (lane * 37) % 64 : 5.0) + 0.01 * lane, mu = 0.01 * lane, integ = 0.0;
    double psid = 0.3, psqd = -0.2, pdid = 1.0, pdqd = -1.0;
    lds_f2 *tp = taps_fl(floor(nt));
    f2 xm1 = tp[0], x0 = tp[1], x1 = tp[2], x2 = tp[3];
    const f2 rx0 = f2{0.3f, -0.2f}, rx1 = f2{0.9f, 0.4f}, rx2 = f2{-0.5f, 0.7f}, rx3 = f2{0.1f, -0.8f};
    unsigned ctr = 0;
    f2 *outf = symf + lane * kRS;
    d2 *outd = symd + lane * kRS;
    auto step = [&](int k) {
        const float t = static_cast<float>(mu);
        const f2 p1 = f2{t, t} + f2{0.0f, 1.0f};
        const f2 p2 = f2{t, t} + f2{-2.0f, -1.0f};
        const f2 bd = (p1 * p2.y) * p2.x;
        const f2 fg = p2 * (p1.y * p1.x);
        const f2 c01 = bd * f2{-(1.0f / 6.0f), 1.0f / 2.0f};
        const f2 c23 = fg * f2{-(1.0f / 2.0f), 1.0f / 6.0f};
        const f2 acc = ((c01.x * xm1 + c01.y * x0) + c23.x * x1) + c23.y * x2;
        const float ci = acc.x, cq = acc.y;
        const double cid = ci, cqd = cq;
        double e;
        double did = 1.0, dqd = 1.0;
        if (V == 5) {
            e = (cid + cqd) - (psid + psqd);
        } else {
            did = ci >= 0.0f ? 1.0 : -1.0;
            dqd = cq >= 0.0f ? 1.0 : -1.0;
            const double t1 = fma(pdid, cid, pdqd * cqd);
            const double t2 = fma(did, psid, dqd * psqd);
            e = t1 - t2;
        }
        integ = integ + ki * e;
        const double c = kp * e + integ;
        const double corr = V == 4 ? c : __builtin_fmax(__builtin_fmin(c, clamp_hi), clamp_lo);
        psid = cid; psqd = cqd;
        pdid = did; pdqd = dqd;
        nt = nt + (sps + corr);
        const double fl = floor(nt);
        mu = nt - fl;
        if (V == 2) {
            xm1 = rx0 + f2{static_cast<float>(fl) * 1e-30f, 0.f}; x0 = rx1; x1 = rx2; x2 = rx3;
        } else if (V == 3 || V == 7) {
            ctr += 8;
            tp = reinterpret_cast<lds_f2 *>(static_cast<uintptr_t>(tap0 + ((ctr & 255) << 3)));
            xm1 = tp[0]; x0 = tp[1]; x1 = tp[2]; x2 = tp[3];
        } else {
            tp = taps_fl(fl);
            xm1 = tp[0]; x0 = tp[1]; x1 = tp[2]; x2 = tp[3];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (V == 6) outd[k] = d2{cid, cqd};
        else if (V != 1 && V != 7) outf[k] = f2{ci, cq};
    };
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int k = 0; k < 16; ++k) step(k);
    }
    __builtin_amdgcn_s_waitcnt(0);
    long long t1 = __builtin_amdgcn_s_memtime();
    out_g[lane] = static_cast<float>(nt) + static_cast<float>(integ) + symf[lane * kRS + 3].x +
                  static_cast<float>(symd[lane * kRS + 3].x);
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int V>
static void run(const char *name, const f2 *src, float *out, long long *cyc, double sps) {
    const int reps = 4096;
    double best = 1e30;
    for (int t = 0; t < 3; ++t) {
        hipLaunchKernelGGL(mm<V>, dim3(1), dim3(64), 0, 0, src, out, cyc, reps, sps);
        hipDeviceSynchronize();
        long long c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        const double cy = (double)c / (reps * 16);
        best = cy < best ? cy : best;
    }
    printf("V%-2d %-52s %7.1f cycles per symbol\n", V, name, best);
}

int main(int argc, char **argv) {
    const double sps = argc > 1 ? atof(argv[1]) : 4.0;
    f2 *src;
    float *out;
    long long *cyc;
    hipMalloc(&src, 32 * 262 * sizeof(f2));
    hipMalloc(&out, 64 * sizeof(float));
    hipMalloc(&cyc, 8);
    f2 h[32 * 262];
    unsigned s = 12345;
    for (auto &v : h) {
        s = s * 1664525u + 1013904223u;
        const float a = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
        s = s * 1664525u + 1013904223u;
        const float b = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
        v = f2{a, b};
    }
    hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
    printf("M&M step alone, one wave, 32 lanes, sps %.1f (s_memtime cycles)\n", sps);
    run<0>("the kernel's step (float slot)", src, out, cyc, sps);
    run<1>("no symbol store", src, out, cyc, sps);
    run<2>("taps from registers (no LDS read / address)", src, out, cyc, sps);
    run<3>("taps from LDS, address off the chain", src, out, cyc, sps);
    run<4>("no clamp", src, out, cyc, sps);
    run<5>("TED without decision doubles", src, out, cyc, sps);
    run<6>("double symbol slot (ds_write_b128)", src, out, cyc, sps);
    run<7>("address off the chain + no store", src, out, cyc, sps);
    run<8>("ring rows of 262 float2 (2-way conflicts)", src, out, cyc, sps);
    run<9>("ring rows of 261 float2 (conflict-free)", src, out, cyc, sps);
    run<10>("spread per-lane positions (rows of 260)", src, out, cyc, sps);
    return 0;
}
