/* tools/check_glibc_sincosf.c -- pins the FLL's float trig to the reference's.
 *
 * .NET's MathF.Sin / MathF.Cos (Band-Edge Filter.cs:108-109) call the C
 * runtime's sinf / cosf, glibc on a Linux host.  This checker compares, for
 * every float input (stride 1 = all 2^32 bit patterns):
 *   glibc sinf / cosf  vs  the oracle restatement or_sinf / or_cosf
 *   (oracle/or_sincos.h)  vs  the product's fused qpsk_sincosf_glibc
 *   (csrc/qpsk_sincosf.h; the _small and branch-free _fast forms and the
 *   FLL's lane-split form, both lanes' views, too where |x| < 120)
 * bit for bit (any NaN equals any NaN).  Prints "<checked> checked, <n> differ".
 *   gcc -O2 -fopenmp -ffp-contract=off -mfma -Ioracle \
 *       -Iqpsk-modulator-demodulator_amd/csrc -o /tmp/chk tools/check_glibc_sincosf.c -lm
 *   /tmp/chk [stride]          (~10 s for all inputs on 8 cores)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "or_sincos.h"
#include "qpsk_sincosf.h"

static int same(float a, float b)
{
    uint32_t x, y;
    memcpy(&x, &a, 4);
    memcpy(&y, &b, 4);
    return x == y || (a != a && b != b);
}

int main(int argc, char **argv)
{
    const long long stride = argc > 1 ? atoll(argv[1]) : 1;
    long long bad = 0, checked = 0;
#pragma omp parallel for reduction(+ : bad, checked) schedule(static)
    for (long long i = 0; i < (1LL << 32); i += stride) {
        const uint32_t u = (uint32_t)i;
        float x;
        memcpy(&x, &u, 4);
        const float gs = sinf(x), gc = cosf(x);
        float ps, pc;
        qpsk_sincosf_glibc(x, &ps, &pc);
        int ok = same(gs, or_sinf(x)) && same(gc, or_cosf(x)) && same(gs, ps) && same(gc, pc);
        if (ok && (fabsf(x) < 120.0f || x != x)) {
            qpsk_sincosf_glibc_small(x, &ps, &pc);
            ok = same(gs, ps) && same(gc, pc);
            qpsk_sincosf_glibc_fast(x, &ps, &pc);
            ok = ok && same(gs, ps) && same(gc, pc);
            if (u != 0x80000000u) {   /* the lane-split form (y != -0): both lanes' views */
                uint32_t ts, tc;
                const uint32_t os = qpsk_sincosf_split_own(x, qpsk_sincosf_lane_init(1), &ts);
                const uint32_t oc = qpsk_sincosf_split_own(x, qpsk_sincosf_lane_init(0), &tc);
                qpsk_sincosf_split_pick(os, oc, ts, &ps, &pc);
                ok = ok && same(gs, ps) && same(gc, pc);
                qpsk_sincosf_split_pick(oc, os, tc, &ps, &pc);
                ok = ok && same(gs, ps) && same(gc, pc);
            }
        }
        if (!ok) {
            if (bad < 4) printf("differ at %08x\n", u);
            ++bad;
        }
        ++checked;
    }
    printf("%lld checked, %lld differ\n", checked, bad);
    return bad != 0;
}
