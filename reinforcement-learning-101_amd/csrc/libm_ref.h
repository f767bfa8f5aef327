// libm_ref.h — the reference's transcendentals, bit for bit: glibc 2.35's
// (License: this file restates GNU C Library code and is LGPL-2.1-or-later,
// like its sources: e_pow.c (c) 2018 Arm Ltd., s_sin.c (c) IBM Corp.
// 2001-2017 / the GNU C Library; see THIRD_PARTY_NOTICES.md.)
//
// pow(x, 2.0), sin and cos as the x86_64 library computes them (the FMA
// builds its ifunc selects on any FMA-capable CPU, compiled with GCC's
// default floating-point contraction), restated from glibc's published
// algorithms:
//
//   pow: sysdeps/ieee754/dbl-64/e_pow.c (Szabolcs Nagy, 2018: log_inline with
//        a 128-entry table and a degree-8 polynomial in double-double, then
//        exp_inline with a 128-entry 2^(k/N) table and a degree-5 polynomial)
//   sin, cos: sysdeps/ieee754/dbl-64/s_sin.c (IBM Accurate Mathematical
//        Library as cleaned up for 2.28: do_sin / do_cos with the 110-entry
//        sin/cos table of i/128, TAYLOR_SIN below 0.126, Cody-Waite reduction
//        by pi/2 in three parts below 105414350)
//
// The reference squares with Python / numpy `v ** 2` (= glibc pow) and takes
// np.sin / np.cos of np.radians(angle); the oracle (oracle/drone_oracle.c)
// calls the same libm.  The fast step path uses v*v and trig.h; frame.h falls
// back to these functions on the rare frame whose predicate quantities sit
// within a hair of a boundary.
//
// Where glibc's C source leaves a*b+c to the compiler, GCC (-ffp-contract=fast,
// -mfma) fuses every product whose only uses are additions; the fma() calls
// below are exactly those fusions (checked bit for bit against the library on
// 10^8+ inputs per function: tools/check_libm_ref.cpp).  This file must be
// compiled with -ffp-contract=off, so no other contraction happens.
//
// The includer defines, before including:
//   DD_LIBM_FN                      function qualifiers (e.g. __device__ __forceinline__)
//   DD_LIBM_ENTRY (optional)        qualifiers of pow2 / sin / cos (default DD_LIBM_FN)
//   DD_LIBM_SINCOS_FN (optional)    qualifiers of sincos (default DD_LIBM_FN)
//   dd_libm_pow_tab[384]            {invc, logc, logctail} x 128   (DD_LIBM_POW_TAB)
//   dd_libm_exp_tab[256]            {tail, sbits} x 128 as uint64  (DD_LIBM_EXP_TAB)
//   dd_libm_sincos_tab[440]         {sn, ssn, cs, ccs} x 110       (DD_LIBM_SINCOS_TAB)
// and includes libm_tables.h (glibc 2.35's tables, committed; tools/gen_libm_tables.py) for the scalar data.
#pragma once

#include <stdint.h>
#include <string.h>

#include "libm_tables.h"

#ifndef DD_LIBM_ENTRY
#define DD_LIBM_ENTRY DD_LIBM_FN
#endif
#ifndef DD_LIBM_SINCOS_FN
#define DD_LIBM_SINCOS_FN DD_LIBM_FN
#endif

namespace dd {
namespace libm {

DD_LIBM_FN uint64_t bits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
DD_LIBM_FN double from_bits(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}

// A double constant as an opaque value in a vector register
// (DD_LIBM_OPAQUE, device builds): these functions run on a kernel's rare
// path, where their ~35 coefficients would otherwise be materialised as SGPR
// pairs and spill the kernel's hot loop SGPRs into VGPR lanes.  Same bits.
#ifdef DD_LIBM_OPAQUE
DD_LIBM_FN double kc(double v) {
    asm volatile("" : "+v"(v));
    return v;
}
#else
DD_LIBM_FN double kc(double v) { return v; }
#endif

// ---- pow ------------------------------------------------------------------
// log(x) for the IEEE bits ix of a positive normal x, as hi + *tail
// (e_pow.c log_inline, the __FP_FAST_FMA branch).
DD_LIBM_FN double pow_log(uint64_t ix, double* tail) {
    constexpr double A[7] = DD_LIBM_POW_POLY;
    constexpr double Ln2hi = DD_LIBM_POW_LN2HI, Ln2lo = DD_LIBM_POW_LN2LO;
    constexpr uint64_t OFF = 0x3fe6955500000000ull;
    const uint64_t tmp = ix - OFF;
    const int i = (int)((tmp >> (52 - 7)) % 128);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & (0xfffull << 52));
    const double z = from_bits(iz);
    const double kd = (double)k;
    const double invc = dd_libm_pow_tab[3 * i], logc = dd_libm_pow_tab[3 * i + 1],
                 logctail = dd_libm_pow_tab[3 * i + 2];
    const double r = fma(z, invc, -1.0);
    const double t1 = fma(kd, kc(Ln2hi), logc);
    const double t2 = t1 + r;
    const double lo1 = fma(kd, kc(Ln2lo), logctail);
    const double lo2 = t1 - t2 + r;
    const double ar = A[0] * r;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double hi = t2 + ar2;
    const double lo3 = fma(ar, r, -ar2);
    const double lo4 = t2 - hi + ar2;
    const double q = fma(ar2, fma(ar2, fma(r, kc(A[6]), kc(A[5])), fma(r, kc(A[4]), kc(A[3]))),
                         fma(r, kc(A[2]), kc(A[1])));
    const double lo = fma(ar3, q, lo1 + lo2 + lo3 + lo4);  // ... + p, p = ar3 * q fused
    const double y = hi + lo;
    *tail = hi - y + lo;
    return y;
}

// exp(x + xtail) (e_pow.c exp_inline with sign_bias 0, and specialcase).
DD_LIBM_FN double pow_exp(double x, double xtail) {
    constexpr double C[4] = DD_LIBM_EXP_POLY;
    constexpr double InvLn2N = DD_LIBM_EXP_INVLN2N, Shift = DD_LIBM_EXP_SHIFT;
    constexpr double NegLn2hiN = DD_LIBM_EXP_NEGLN2HIN, NegLn2loN = DD_LIBM_EXP_NEGLN2LON;
    uint32_t abstop = (uint32_t)(bits(x) >> 52) & 0x7ff;
    if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {  // top12(0x1p-54) = 0x3c9, top12(512) = 0x408
        if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;  // tiny: WANT_ROUNDING
        if (abstop >= 0x409u) return (bits(x) >> 63) ? 0.0 : __builtin_inf();  // |x| >= 1024
        abstop = 0;  // large |x|: specialcase
    }
    double kd = fma(kc(InvLn2N), x, Shift);  // z = InvLn2N * x; kd = z + Shift, fused
    const uint64_t ki = bits(kd);
    kd -= Shift;
    double r = fma(kd, kc(NegLn2loN), fma(kd, kc(NegLn2hiN), x));
    r += xtail;
    const uint64_t idx = 2 * (ki % 128);
    const uint64_t top = ki << (52 - 7);
    const double tail = from_bits(dd_libm_exp_tab[idx]);
    uint64_t sbits = dd_libm_exp_tab[idx + 1] + top;
    const double r2 = r * r;
    const double tmp = fma(r2 * r2, fma(r, kc(C[3]), kc(C[2])), fma(r2, fma(r, kc(C[1]), kc(C[0])), tail + r));
    if (abstop == 0) {  // specialcase
        if ((ki & 0x80000000u) == 0) {
            sbits -= 1009ull << 52;
            const double scale = from_bits(sbits);
            return 0x1p1009 * fma(scale, tmp, scale);
        }
        sbits += 1022ull << 52;
        const double scale = from_bits(sbits);
        // scale * tmp is one product (CSE) with a second use in the branch
        // below, another basic block: GCC fuses neither use
        const double st = scale * tmp;
        double y = scale + st;
        if (fabs(y) < 1.0) {
            const double one = y < 0.0 ? -1.0 : 1.0;
            double lo = scale - y + st;
            const double hi = one + y;
            lo = one - hi + y + lo;
            y = (hi + lo) - one;
            if (y == 0) y = from_bits(sbits & 0x8000000000000000ull);
        }
        return 0x1p-1022 * y;
    }
    const double scale = from_bits(sbits);
    return fma(scale, tmp, scale);
}

// pow(x, 2.0): Python's / numpy's `x ** 2` (e_pow.c __pow with y = 2).
DD_LIBM_ENTRY double pow2(double x) {
    uint64_t ix = bits(x) & 0x7fffffffffffffffull;  // y = 2 is an even integer: pow(-x, 2) = pow(x, 2)
    const uint32_t topx = (uint32_t)(ix >> 52);
    if (topx - 1u >= 0x7feu) {  // zero, subnormal, inf or nan
        if (ix == 0 || topx == 0x7ff) return x * x;
        ix = bits(from_bits(ix) * 0x1p52) & 0x7fffffffffffffffull;  // subnormal: normalise
        ix -= 52ull << 52;
    }
    double lo;
    const double hi = pow_log(ix, &lo);
    const double ehi = 2.0 * hi;
    const double elo = fma(2.0, lo, fma(2.0, hi, -ehi));  // y * lo + fma(y, hi, -ehi), fused
    return pow_exp(ehi, elo);
}

// ---- sin, cos -------------------------------------------------------------
constexpr double kS1 = -0x1.5555555555555p-3, kS2 = 0x1.1111111110ecep-7, kS3 = -0x1.a01a019db08b8p-13,
                 kS4 = 0x1.71de27b9a7ed9p-19, kS5 = -0x1.addffc2fcdf59p-26;
constexpr double kSn3 = -0x1.5555555555515p-3, kSn5 = 0x1.11110e829872fp-7, kCs2 = 0.5,
                 kCs4 = -0x1.5555555555535p-5, kCs6 = 0x1.6c16bedd9e239p-10;
constexpr double kBig = 0x1.8p45, kHp0 = 0x1.921fb54442d18p0, kHp1 = 0x1.1a62633145c07p-54;
constexpr double kMp1 = 0x1.921fb58000000p0, kMp2 = -0x1.dde973c000000p-27, kPp3 = -0x1.cb3b398000000p-55,
                 kPp4 = -0x1.d747f23e32ed7p-83, kHpinv = 0x1.45f306dc9c883p-1, kToint = 0x1.8p52;

// TAYLOR_SIN(xx, a, da)
DD_LIBM_FN double taylor_sin(double xx, double a, double da) {
    const double poly = fma(fma(fma(fma(kc(kS5), xx, kc(kS4)), xx, kc(kS3)), xx, kc(kS2)), xx, kc(kS1));
    const double t = fma(fma(poly, a, -(0.5 * da)), xx, da);
    return a + t;
}

DD_LIBM_FN double do_cos(double x, double dx) {
    if (x < 0) dx = -dx;
    const double u = kBig + fabs(x);
    x = fabs(x) - (u - kBig) + dx;
    const double xx = x * x;
    const double s = fma(x * xx, fma(xx, kc(kSn5), kc(kSn3)), x);
    const double c = xx * fma(xx, fma(xx, kc(kCs6), kc(kCs4)), kCs2);
    const int k = (int)(uint32_t)bits(u) << 2;
    const double sn = dd_libm_sincos_tab[k], ssn = dd_libm_sincos_tab[k + 1], cs = dd_libm_sincos_tab[k + 2],
                 ccs = dd_libm_sincos_tab[k + 3];
    const double cor = fma(-sn, s, fma(-cs, c, fma(-s, ssn, ccs)));
    return cs + cor;
}

DD_LIBM_FN double do_sin(double x, double dx) {
    const double xold = x;
    if (fabs(x) < 0.126) return taylor_sin(x * x, x, dx);
    if (x <= 0) dx = -dx;
    const double u = kBig + fabs(x);
    x = fabs(x) - (u - kBig);
    const double xx = x * x;
    const double s = x + fma(x * xx, fma(xx, kc(kSn5), kc(kSn3)), dx);
    const double c = fma(x, dx, xx * fma(xx, fma(xx, kc(kCs6), kc(kCs4)), kCs2));
    const int k = (int)(uint32_t)bits(u) << 2;
    const double sn = dd_libm_sincos_tab[k], ssn = dd_libm_sincos_tab[k + 1], cs = dd_libm_sincos_tab[k + 2],
                 ccs = dd_libm_sincos_tab[k + 3];
    const double cor = fma(cs, s, fma(-sn, c, fma(s, ccs, ssn)));
    return copysign(sn + cor, xold);
}

DD_LIBM_FN int reduce_sincos(double x, double* a, double* da) {
    const double t = fma(x, kc(kHpinv), kToint);
    const double xn = t - kToint;
    const double y = fma(-xn, kc(kMp2), fma(-xn, kc(kMp1), x));
    const int n = (int)(bits(t) & 3);
    const double pp3 = kc(kPp3), pp4 = kc(kPp4);
    const double t2 = fma(-xn, pp3, y);           // y - t1, t1 = xn * pp3 fused into both uses
    double db = fma(-xn, pp3, y - t2);
    const double b = fma(-xn, pp4, t2);           // t2 - t1, t1 = xn * pp4
    db += fma(-xn, pp4, t2 - b);
    *a = b;
    *da = db;
    return n;
}

DD_LIBM_FN double do_sincos(double a, double da, int n) {
    const double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
    return (n & 2) ? -r : r;
}

// sin(x) for |x| < 105414350 (the reference's angles: |x| <= 3 pi); larger or
// non-finite arguments return NaN (glibc's __branred range is never reached
// from the frame, whose angles a caller-written state keeps below 2^53 deg).
DD_LIBM_ENTRY double sin(double x) {
    const uint32_t k = (uint32_t)(bits(x) >> 32) & 0x7fffffffu;
    if (k < 0x3e500000u) return x;
    if (k < 0x3feb6000u) return do_sin(x, 0);
    if (k < 0x400368fdu) return copysign(do_cos(kc(kHp0) - fabs(x), kc(kHp1)), x);
    if (k < 0x419921fbu) {
        double a, da;
        const int n = reduce_sincos(x, &a, &da);
        return do_sincos(a, da, n);
    }
    return __builtin_nan("");
}

DD_LIBM_ENTRY double cos(double x) {
    const uint32_t k = (uint32_t)(bits(x) >> 32) & 0x7fffffffu;
    if (k < 0x3e400000u) return 1.0;
    if (k < 0x3feb6000u) return do_cos(x, 0);
    if (k < 0x400368fdu) {
        const double hp1 = kc(kHp1);
        const double y = kc(kHp0) - fabs(x);
        const double a = y + hp1;
        const double da = (y - a) + hp1;
        return do_sin(a, da);
    }
    if (k < 0x419921fbu) {
        double a, da;
        const int n = reduce_sincos(x, &a, &da);
        return do_sincos(a, da, n + 1);
    }
    return __builtin_nan("");
}

// sin(x) and cos(x), bit for bit what glibc's separate sin and cos return
// (not its sincos, whose middle range differs), with one do_sin and one
// do_cos per argument and no divergent range branch: whatever the range, sin
// and cos come from do_sin / do_cos of the same reduced argument (swapped,
// negated or sign-copied by range), so the two kernels run once per lane.
DD_LIBM_SINCOS_FN void sincos(double x, double* sp, double* cp) {
    const uint32_t k = (uint32_t)(bits(x) >> 32) & 0x7fffffffu;
    double sa = x, sda = 0.0, ca = x, cda = 0.0;  // arguments of do_sin and do_cos (direct range)
    bool swap = false, neg_s = false, neg_c = false, sign_x = false;
    if (k >= 0x400368fdu) {  // |x| > 2.426265: by pi/2, n = quadrant
        double a, da;
        const int n = reduce_sincos(x, &a, &da);
        sa = ca = a;
        sda = cda = da;
        swap = (n & 1) != 0;  // odd n: sin from do_cos, cos from do_sin
        neg_s = (n & 2) != 0;
        neg_c = ((n + 1) & 2) != 0;
    } else if (k >= 0x3feb6000u) {  // 0.855469 <= |x| <= 2.426265: about pi/2
        const double hp1 = kc(kHp1);
        const double t = kc(kHp0) - fabs(x);
        ca = t;  // sin = copysign(do_cos(t, hp1), x)
        cda = hp1;
        sa = t + hp1;  // cos = do_sin(a, da), a + da = t + hp1
        sda = (t - sa) + hp1;
        swap = true;
        sign_x = true;
    }
    const double rs = do_sin(sa, sda), rc = do_cos(ca, cda);
    double s = swap ? rc : rs, c = swap ? rs : rc;
    s = sign_x ? copysign(s, x) : s;
    s = neg_s ? -s : s;
    c = neg_c ? -c : c;
    s = k < 0x3e500000u ? x : s;    // |x| < 2^-26: sin(x) = x
    c = k < 0x3e400000u ? 1.0 : c;  // |x| < 2^-27: cos(x) = 1
    const bool out = k >= 0x419921fbu;  // beyond __branred's threshold (never reached) or not finite
    *sp = out ? __builtin_nan("") : s;
    *cp = out ? __builtin_nan("") : c;
}

}  // namespace libm
}  // namespace dd
