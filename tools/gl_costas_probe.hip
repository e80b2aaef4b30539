// tools/gl_costas_probe.hip -- cycles per symbol of the glibc-exact Costas
// step of qpsk_loop.hip (costas_trig = 1, fast split form: lanes l and l + 32
// carry one stream, qpsk_glibc_trig.h) in one lone wave, LDS-resident table and
// symbols, with variants that stub out one piece each, to see where the
// chain's ~690 cycles per symbol go beyond its ~114 instructions.
// Diagnostic only; not part of the library.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp \
//         tools/gl_costas_probe.hip -o tools/bin/gl_costas_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../qpsk-modulator-demodulator_amd/csrc/qpsk_glibc_trig.h"

typedef double d2 __attribute__((ext_vector_type(2)));
constexpr int kRS = 41;

__device__ __forceinline__ void swap_halves(double r, double *lower, double *upper) {
    const uint64_t b = __builtin_bit_cast(uint64_t, r);
    const uint32_t lo = static_cast<uint32_t>(b), hi = static_cast<uint32_t>(b >> 32);
    const auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    *lower = __builtin_bit_cast(double, (static_cast<uint64_t>(ph[0]) << 32) | pl[0]);
    *upper = __builtin_bit_cast(double, (static_cast<uint64_t>(ph[1]) << 32) | pl[1]);
}

// lanes 2l and 2l + 1 carry one stream: each gets its partner's value with one
// quad_perm [1,0,3,2] DPP move per word
__device__ __forceinline__ double pair_partner(double r) {
    const uint64_t b = __builtin_bit_cast(uint64_t, r);
    const int lo = static_cast<int>(static_cast<uint32_t>(b)), hi = static_cast<int>(static_cast<uint32_t>(b >> 32));
    const uint32_t plo = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(lo, lo, 0xB1, 0xF, 0xF, false));
    const uint32_t phi = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(hi, hi, 0xB1, 0xF, 0xF, false));
    return __builtin_bit_cast(double, (static_cast<uint64_t>(phi) << 32) | plo);
}

__device__ __forceinline__ double signsel(double x, bool pos) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    float h = __builtin_bit_cast(float, static_cast<uint32_t>(b >> 32));
    asm("" : "+v"(h));
    const float r = pos ? h : -h;
    return __builtin_bit_cast(double, (static_cast<uint64_t>(__builtin_bit_cast(uint32_t, r)) << 32) |
                                          static_cast<uint32_t>(b));
}

// the round-4 split of the pair (qpsk_glibc_trig.h before round 5): the
// argument of this half, then its value
__device__ __forceinline__ double old_fs_prepare(double x, const qpsk_gl_fs_lane *K, double *dxa, uint32_t *t,
                                                 int *swap) {
    const double ax = fabs(x);
    const double tt = fma(ax, QPSK_GL_HPINV, K->toint);
    const double xn = tt - QPSK_GL_TOINT;
    double y = fma(-xn, QPSK_GL_MP1, ax);
    y = fma(-xn, QPSK_GL_MP2, y);
    const double t2 = fma(-xn, QPSK_GL_PP3, y);
    double db = fma(-xn, QPSK_GL_PP3, y - t2);
    const double b = fma(-xn, QPSK_GL_PP4, t2);
    db = db + fma(-xn, QPSK_GL_PP4, t2 - b);
    const double yb = QPSK_GL_HP0 - ax;
    const double xb = yb + K->hp1L;
    const double dB = (yb - xb) + QPSK_GL_HP1;
    const int rA = ax < 0x1.b6p-1;
    const int rB = ax < 0x1.368fdp+1;
    *dxa = rA ? 0.0 : (rB ? dB : db);
    const uint32_t tn = (uint32_t)qpsk_gl_bits(tt) << 30;
    *t = rB ? 0u : tn;
    *swap = rA ? 0 : (rB ? 1 : (int)(tn >> 30) & 1);
    return rA ? ax : (rB ? xb : b);
}

// qpsk_gl_fs_half with pieces switchable: NOTAB reads four register constants
// instead of the LDS row, NOTAY drops the TAYLOR_SIN select
template <bool NOTAB, bool NOTAY>
__device__ __forceinline__ double fs_half_v(double xa, double dxa, uint32_t t, const qpsk_gl_fs_lane *K,
                                            const double *tabh, const double *treg) {
    double ty = 0.0;
    if (!NOTAY) {
        const double ta = xa * xa;
        double tp = fma(ta, QPSK_GL_S5, K->s4);
        tp = fma(ta, tp, QPSK_GL_S3);
        tp = fma(ta, tp, QPSK_GL_S2);
        tp = fma(ta, tp, QPSK_GL_S1);
        ty = xa + fma(ta, fma(tp, xa, -(0.5 * dxa)), dxa);
    }
    const double d = qpsk_gl_with_hi(dxa, qpsk_gl_hi(dxa) ^ (qpsk_gl_hi(xa) & K->sign));
    const double ax = fabs(xa);
    const double u = QPSK_GL_BIG + ax;
    const double xr = fma(d, K->L1, ax - (u - QPSK_GL_BIG));
    const double xx = xr * xr;
    const double q = xr * xx;
    const double p = fma(xx, QPSK_GL_SN5, K->sn3);
    const double dl = d * K->L0;
    const double s = fma(q, p, fma(xr, K->L1, dl)) + xr * K->L0;
    const double c = fma(xr, dl, xx * fma(xx, fma(xx, QPSK_GL_CS6, K->cs4), QPSK_GL_CS2));
    const uint32_t node = (uint32_t)qpsk_gl_bits(u) & 127u;
    double t0, t1, t2, t3;
    if (NOTAB) {
        t0 = treg[0]; t1 = treg[1]; t2 = treg[2]; t3 = treg[3];
    } else {
        typedef __attribute__((address_space(3))) const double lds_double;
        uint32_t addr;
        asm("v_lshl_add_u32 %0, %1, 5, %2" : "=v"(addr) : "v"(node), "v"((uint32_t)(uintptr_t)(lds_double *)tabh));
        lds_double *tb = (lds_double *)(uintptr_t)addr;
        t0 = tb[0]; t1 = tb[1]; t2 = tb[2]; t3 = tb[3];
    }
    double cor = fma(s, t0, t1);
    cor = fma(-c, t2, cor);
    cor = fma(s, t3, cor);
    const double r = t2 + cor;
    double v = qpsk_gl_with_hi(r, qpsk_gl_bfi(K->sgnm, qpsk_gl_hi(xa), qpsk_gl_hi(r)));
    if (!NOTAY && K->sin_half && ax < 0.126) v = ty;
    return qpsk_gl_with_hi(v, qpsk_gl_hi(v) ^ ((t + K->tsh) & K->sign));
}

// the pair with the table row read as early as the argument allows: xa, u and
// the row address first, the row's four loads, a scheduling barrier, then the
// rest (dx, quadrant, polynomials).  MERGEA: region A as region C with n = 0
// (tt = toint when the high word of 1/hp0 is zeroed: then xn = 0 and the
// reduction returns (|x|, +0) exactly), so the argument selects have two ways
template <bool MERGEA>
__device__ __forceinline__ void fs_early(double x, const qpsk_gl_fs_lane *K, const double *tabh, double *s_out,
                                         double *c_out) {
    const double ax = fabs(x);
    const int rA = ax < 0x1.b6p-1;
    const int rB = ax < 0x1.368fdp+1;
    double hpinv = QPSK_GL_HPINV;
    if (MERGEA) {
        const uint64_t hb = qpsk_gl_bits(hpinv);
        hpinv = qpsk_gl_from_bits(rA ? (hb & 0xffffffffull) : hb);
    }
    const double tt = fma(ax, hpinv, K->toint);
    const double xn = tt - QPSK_GL_TOINT;
    double y = fma(-xn, QPSK_GL_MP1, ax);
    y = fma(-xn, QPSK_GL_MP2, y);
    const double t2 = fma(-xn, QPSK_GL_PP3, y);
    const double b = fma(-xn, QPSK_GL_PP4, t2);
    const double yb = QPSK_GL_HP0 - ax;
    const double xb = yb + K->hp1L;
    const int rBo = MERGEA ? (rB && !rA) : rB;
    const double xa = MERGEA ? (rBo ? xb : b) : (rA ? ax : (rB ? xb : b));
    const double axa = fabs(xa);
    const double u = QPSK_GL_BIG + axa;
    const uint32_t node = (uint32_t)qpsk_gl_bits(u) & 127u;
    typedef __attribute__((address_space(3))) const double lds_double;
    uint32_t addr;
    asm("v_lshl_add_u32 %0, %1, 5, %2" : "=v"(addr) : "v"(node), "v"((uint32_t)(uintptr_t)(lds_double *)tabh));
    lds_double *tb = (lds_double *)(uintptr_t)addr;
    const double t0 = tb[0], t1 = tb[1], t2r = tb[2], t3 = tb[3];
    __builtin_amdgcn_sched_barrier(0);
    double db = fma(-xn, QPSK_GL_PP3, y - t2);
    db = db + fma(-xn, QPSK_GL_PP4, t2 - b);
    const double dB = (yb - xb) + QPSK_GL_HP1;
    const double dxa = MERGEA ? (rBo ? dB : db) : (rA ? 0.0 : (rB ? dB : db));
    const uint32_t tn = (uint32_t)qpsk_gl_bits(tt) << 30;
    const uint32_t t = rBo ? 0u : tn;
    const int swap = MERGEA ? (rBo ? 1 : (int)(tn >> 30) & 1) : (rA ? 0 : (rB ? 1 : (int)(tn >> 30) & 1));
    /* qpsk_gl_fs_half from here, with the row already loaded */
    const double ta = xa * xa;
    double tp = fma(ta, QPSK_GL_S5, K->s4);
    tp = fma(ta, tp, QPSK_GL_S3);
    tp = fma(ta, tp, QPSK_GL_S2);
    tp = fma(ta, tp, QPSK_GL_S1);
    const double ty = xa + fma(ta, fma(tp, xa, -(0.5 * dxa)), dxa);
    const double d = qpsk_gl_with_hi(dxa, qpsk_gl_hi(dxa) ^ (qpsk_gl_hi(xa) & K->sign));
    const double xr = fma(d, K->L1, axa - (u - QPSK_GL_BIG));
    const double xx = xr * xr;
    const double q = xr * xx;
    const double p = fma(xx, QPSK_GL_SN5, K->sn3);
    const double dl = d * K->L0;
    const double s = fma(q, p, fma(xr, K->L1, dl)) + xr * K->L0;
    const double c = fma(xr, dl, xx * fma(xx, fma(xx, QPSK_GL_CS6, K->cs4), QPSK_GL_CS2));
    double cor = fma(s, t0, t1);
    cor = fma(-c, t2r, cor);
    cor = fma(s, t3, cor);
    const double r = t2r + cor;
    double v = qpsk_gl_with_hi(r, qpsk_gl_bfi(K->sgnm, qpsk_gl_hi(xa), qpsk_gl_hi(r)));
    if (K->sin_half && axa < 0.126) v = ty;
    const double rh = qpsk_gl_with_hi(v, qpsk_gl_hi(v) ^ ((t + K->tsh) & K->sign));
    double VS, VC;
    swap_halves(rh, &VS, &VC);
    qpsk_gl_fs_finish(x, swap, VS, VC, K, s_out, c_out);
}

// V: 0 the round-4 kernel step, 1 no permlane hand-over, 2 table
// from registers, 3 no TAYLOR_SIN, 4 = 1+2+3, 5 cheap trig (no glibc code),
// 6 the local copy of the step (check that it times like 0), 7 no prepare
// (xa = |theta|, region A only), 8 = 7+2+3, 9 early row read, 10 = 9 +
// region A merged into C, 11 the header's qpsk_gl_fs_pair (= 10), 12 = 11
// without the hand-over, 13 = 11 with lanes 2l, 2l + 1 per stream and a DPP
// hand-over whose selects fold into the swap, 14 = 13 with the hand-over
// as explicit selects by lane parity (then fs_finish)
template <int V>
__global__ __launch_bounds__(64) void gl_costas(const d2 *sym_g, const double *tab_g, float *out_g, long long *cyc,
                                                int reps) {
    __shared__ double tab[880];
    __shared__ d2 sym[32 * kRS];
    __shared__ uint16_t rot[32 * kRS];
    const int lane = threadIdx.x;
    for (int i = lane; i < 110; i += 64) qpsk_gl_half_tables(tab_g, i, tab + 4 * i, tab + 440 + 4 * i);
    for (int i = lane; i < 32 * kRS; i += 64) sym[i] = sym_g[i];
    __syncthreads();
    constexpr bool PAIR = V == 13 || V == 14;
    const int cl = PAIR ? lane >> 1 : lane & 31, half = PAIR ? lane & 1 : lane >> 5;
    const double *tabh = tab + (half ? 440 : 0);
    qpsk_gl_fs_lane KF = qpsk_gl_fs_lane_init(half == 0);
    asm volatile("" : "+v"(KF.L0), "+v"(KF.L1), "+v"(KF.hp1L), "+v"(KF.sgnm), "+v"(KF.tsh), "+v"(KF.sign));
    asm volatile("" : "+v"(KF.toint), "+v"(KF.s4), "+v"(KF.sn3), "+v"(KF.cs4));
    double treg[4] = {tab[4 * 20 + (half ? 440 : 0)], tab[4 * 20 + 1], tab[4 * 20 + 2], tab[4 * 20 + 3]};
    asm volatile("" : "+v"(treg[0]), "+v"(treg[1]), "+v"(treg[2]), "+v"(treg[3]));
    // carrier phases spread over [-3, 3] across the streams
    double theta = -3.0 + 0.19 * ((cl * 13) % 32), freq = 1e-4;
    double ca = 0.13751550967894244, cb = 0.010184293139132996;
    double kTwoPi = 2.0 * 3.14159265358979311600, kPi = 3.14159265358979311600;
    asm volatile("" : "+v"(ca), "+v"(cb), "+v"(kTwoPi), "+v"(kPi));
    const d2 *in = sym + cl * kRS;
    uint16_t *out = rot + cl * kRS;
    double amax = 0.0;
    d2 y = in[0];
    auto step = [&](int k) {
        const d2 yn = in[k + 1];
        double sn, cs;
        if constexpr (V == 5) {
            cs = 1.0 - 0.5 * theta * theta;
            sn = theta;
        } else if constexpr (V == 12) {
            int sw;
            const double rh = qpsk_gl_fs_pair(theta, &KF, tabh, &sw);
            qpsk_gl_fs_finish(theta, sw, rh, rh, &KF, &sn, &cs);
        } else if constexpr (V == 13) {
            int sw;
            const double rh = qpsk_gl_fs_pair(theta, &KF, tabh, &sw);
            const double P = pair_partner(rh);
            const int swp = sw ^ half;
            const double s = swp ? P : rh;
            cs = swp ? rh : P;
            sn = qpsk_gl_with_hi(s, qpsk_gl_hi(s) ^ (qpsk_gl_hi(theta) & KF.sign));
        } else if constexpr (V == 14) {
            int sw;
            const double rh = qpsk_gl_fs_pair(theta, &KF, tabh, &sw);
            const double P = pair_partner(rh);
            const double VS = half ? P : rh, VC = half ? rh : P;
            qpsk_gl_fs_finish(theta, sw, VS, VC, &KF, &sn, &cs);
        } else if constexpr (V == 11) {
            int sw;
            const double rh = qpsk_gl_fs_pair(theta, &KF, tabh, &sw);
            double VS, VC;
            swap_halves(rh, &VS, &VC);
            qpsk_gl_fs_finish(theta, sw, VS, VC, &KF, &sn, &cs);
        } else if constexpr (V == 9 || V == 10) {
            fs_early<V == 10>(theta, &KF, tabh, &sn, &cs);
        } else if constexpr (V == 0) {
            double dxa;
            uint32_t tq;
            int sw;
            const double xa = old_fs_prepare(theta, &KF, &dxa, &tq, &sw);
            const double rh = fs_half_v<false, false>(xa, dxa, tq, &KF, tabh, nullptr);
            double VS, VC;
            swap_halves(rh, &VS, &VC);
            qpsk_gl_fs_finish(theta, sw, VS, VC, &KF, &sn, &cs);
        } else {
            constexpr bool NOSWAP = V == 1 || V == 4;
            constexpr bool NOTAB = V == 2 || V == 4 || V == 8;
            constexpr bool NOTAY = V == 3 || V == 4 || V == 8;
            constexpr bool NOPREP = V == 7 || V == 8;
            double dxa = 0.0, xa;
            uint32_t tq = 0;
            int sw = 0;
            if (NOPREP) xa = fabs(theta);
            else xa = old_fs_prepare(theta, &KF, &dxa, &tq, &sw);
            const double rh = fs_half_v<NOTAB, NOTAY>(xa, dxa, tq, &KF, tabh, treg);
            double VS, VC;
            if (NOSWAP) { VS = rh; VC = rh; }
            else swap_halves(rh, &VS, &VC);
            qpsk_gl_fs_finish(theta, sw, VS, VC, &KF, &sn, &cs);
        }
        const double mi = y.x * cs + y.y * sn;
        const double mq = y.y * cs - y.x * sn;
        const float ri = static_cast<float>(mi), rq = static_cast<float>(mq);
        const bool qpos = rq >= 0.0f;
        const double ei = ri >= 0.0f ? 1.0 : -1.0;
        const double qmi = signsel(mi, qpos);
        const double pe = fma(ei, mq, -qmi);
        freq = freq + cb * pe;
        const double tn = theta + (freq + ca * pe);
        const double tw = tn - copysign(kTwoPi, tn);
        theta = fabs(tn) > kPi ? tw : tn;
        const uint32_t eih = static_cast<uint32_t>(__builtin_bit_cast(uint64_t, ei) >> 32);
        const uint32_t eqh = qpos ? 0x3FF00000u : 0xBFF00000u;
        out[k] = static_cast<uint16_t>(__builtin_amdgcn_perm(eqh, eih, 0x0c0c0703u));
        y = yn;
    };
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        for (int k = 0; k < 32; k += 4) {
            step(k);
            asm volatile("v_max_f64 %0, %0, |%1|" : "+v"(amax) : "v"(theta));
            step(k + 1);
            asm volatile("v_max_f64 %0, %0, |%1|" : "+v"(amax) : "v"(theta));
            step(k + 2);
            asm volatile("v_max_f64 %0, %0, |%1|" : "+v"(amax) : "v"(theta));
            step(k + 3);
            asm volatile("v_max_f64 %0, %0, |%1|" : "+v"(amax) : "v"(theta));
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    long long t1 = __builtin_amdgcn_s_memtime();
    out_g[lane] = rot[cl * kRS + 3] + (float)theta + (float)amax;
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int V>
static void run(const char *name, const d2 *sym, const double *tab, float *out, long long *cyc) {
    const int reps = 1024;
    double best = 1e30;
    for (int t = 0; t < 3; ++t) {
        hipLaunchKernelGGL(gl_costas<V>, dim3(1), dim3(64), 0, 0, sym, tab, out, cyc, reps);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return; }
        long long c = 0;
        if (hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost) != hipSuccess) return;
        const double cy = (double)c / (reps * 32);
        if (cy < best) best = cy;
    }
    printf("%-40s %6.1f cycles/symbol\n", name, best);
}

int main() {
    d2 *sym;
    double *tab;
    float *out;
    long long *cyc;
    if (hipMalloc(&sym, 32 * kRS * sizeof(d2)) != hipSuccess || hipMalloc(&tab, 440 * 8) != hipSuccess ||
        hipMalloc(&out, 64 * 4) != hipSuccess || hipMalloc(&cyc, 8) != hipSuccess)
        return 1;
    static d2 h[32 * kRS];
    for (int i = 0; i < 32 * kRS; ++i) h[i] = d2{0.7 * ((i * 7) % 5 - 2), 0.6 * ((i * 3) % 7 - 3)};
    if (hipMemcpy(sym, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
    if (hipMemcpy(tab, qpsk_gl_sincostab_host, 440 * 8, hipMemcpyHostToDevice) != hipSuccess) return 1;
    run<0>("round-4 step (warm-up)", sym, tab, out, cyc);
    run<0>("round-4 step", sym, tab, out, cyc);
    run<6>("local copy of the step", sym, tab, out, cyc);
    run<1>("no permlane hand-over", sym, tab, out, cyc);
    run<2>("table from registers", sym, tab, out, cyc);
    run<3>("no TAYLOR_SIN", sym, tab, out, cyc);
    run<4>("no hand-over, no table, no Taylor", sym, tab, out, cyc);
    run<7>("no prepare (region A only)", sym, tab, out, cyc);
    run<8>("no prepare, no table, no Taylor", sym, tab, out, cyc);
    run<5>("cheap trig (no glibc code)", sym, tab, out, cyc);
    run<9>("early row read", sym, tab, out, cyc);
    run<10>("early row read, region A merged into C", sym, tab, out, cyc);
    run<11>("qpsk_gl_fs_pair (round-5 header)", sym, tab, out, cyc);
    run<12>("fs_pair, no hand-over", sym, tab, out, cyc);
    run<13>("fs_pair, lane pairs, DPP, folded selects", sym, tab, out, cyc);
    run<14>("fs_pair, lane pairs, DPP, parity selects", sym, tab, out, cyc);
    return 0;
}
