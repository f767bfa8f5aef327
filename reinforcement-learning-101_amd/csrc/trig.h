// trig.h — double-precision angle math of the drone frame: sin/cos of the
// rotation, exact division by the observation scales, angle wrapping.
//
// The frame takes sin/cos of angle * (pi/180) twice per drone (thrust vector
// and bottom centre, physics.py:6-23).  Angles live in [-180, 180] degrees
// (normalize_angle), so |x| <= pi + 1 ulp and the quadrant is |n| <= 2.  The
// general OCML sincos spends ~100 VALU instructions on its fast path
// (double-double Cody-Waite reduction sized for huge arguments); this one
// spends ~40 for |x| < 2^19 * pi/2:
//   * reduction: a three-part Cody-Waite split of pi/2 as three FMAs (33-bit
//     head and middle, so n * head and n * middle are exact; the first FMA is
//     exact, the second exact whenever it cancels, i.e. whenever the reduced
//     argument is small enough for the tail to matter), no y1 tail word;
//   * kernels: the public-domain fdlibm minimax polynomials (Sun, 1993) for
//     sin and cos on [-pi/4, pi/4], without the tail correction.
// Never more than 1 ulp from glibc's correctly-rounded-in-practice sin/cos
// (the reference's, through numpy); 13 % of results are 1 ulp off (3 % with
// the y1 tail kept, 16 VALU more: tests/test_trig_math.py).  The frame's
// flags do not depend on it (near a boundary the lane is redone with glibc's
// functions, frame.h), and an ulp of sin moves vx by an ulp of 0.15.
// Beyond |x| = 2^19 * pi/2 (angles past 4.7e7 degrees, far outside anything
// step() produces or the reference can normalise) the reduction loses
// accuracy; no library fallback is compiled in, so the kernel carries no
// Payne-Hanek code.  Compiled with -ffp-contract=off: every step below relies
// on the separate roundings it is written with.
#pragma once

#include <math.h>

#if defined(__HIPCC__)
#define DD_HD __host__ __device__
#else
#define DD_HD
#endif

namespace dd {
namespace trig {

constexpr double kInvPio2 = 6.36619772367581382433e-01;  // 0x3FE45F306DC9C883
constexpr double kPio2_1 = 1.57079632673412561417e+00;   // 0x3FF921FB54400000 (33 bits)
constexpr double kPio2_2 = 6.07710050630396597660e-11;   // 0x3DD0B4611A600000 (33 bits)
constexpr double kPio2_2t = 2.02226624879595063154e-21;  // 0x3BA3198A2E037073

constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;

// Horner step a + z * b, fused (the polynomial tails are far below an ulp of
// the result, so fusing only removes roundings).
DD_HD inline double hstep(double a, double z, double b) { return fma(z, b, a); }

// The same Horner step with the constant `a` as an SGPR operand of a VOP3
// v_fma_f64 (device code, kSgpr).  Left to itself the compiler materialises
// each coefficient into the accumulator with two v_mov_b32 and issues a
// v_fmac: three VALU per step.  Here the two moves are s_mov (the scalar
// unit, which another wave's VALU issue overlaps): the step kernel, four
// waves per SIMD.  Same operation, same bits.  The innermost step of each
// chain (two constants) keeps the plain form: a VOP3 reads one SGPR pair.
template <bool kSgpr>
DD_HD inline double hstep_c(double a, double z, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (kSgpr) {
        double r;
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(z), "v"(b), "s"(a));
        return r;
    }
#endif
    return hstep(a, z, b);
}

// sin(y), |y| <= pi/4
template <bool kSgpr = false>
DD_HD inline double ksin(double y) {
    const double z = y * y;
    const double v = z * y;
    const double r =
        hstep_c<kSgpr>(S1, z, hstep_c<kSgpr>(S2, z, hstep_c<kSgpr>(S3, z, hstep_c<kSgpr>(S4, z, hstep(S5, z, S6)))));
    return fma(v, r, y);
}

// cos(y), |y| <= pi/4
template <bool kSgpr = false>
DD_HD inline double kcos(double y) {
    const double z = y * y;
    const double w = z * z;
    const double r = z * hstep_c<kSgpr>(C1, z, hstep(C2, z, C3)) + w * w * hstep_c<kSgpr>(C4, z, hstep(C5, z, C6));
    const double hz = 0.5 * z;
    const double u = 1.0 - hz;
    return u + (((1.0 - u) - hz) + z * r);
}

// (sin x, cos x), within 1 ulp for |x| < 2^19 * pi/2.
template <bool kSgpr = false>
DD_HD inline void sincos(double x, double* s, double* c) {
    const double fn = rint(x * kInvPio2);
    const int n = (int)fn;
    const double t = fma(-fn, kPio2_1, x);  // exact: fn * head has <= 53 bits, Sterbenz
    const double y = fma(-fn, kPio2_2t, fma(-fn, kPio2_2, t));
    const double sv = ksin<kSgpr>(y);
    const double cv = kcos<kSgpr>(y);
    // quadrant n & 3 -> (sv, cv), (cv, -sv), (-sv, -cv), (-cv, sv), as
    // selects and sign flips rather than a divergent switch
    const double a = (n & 1) ? cv : sv;
    const double b = (n & 1) ? sv : cv;
    *s = (n & 2) ? -a : a;
    *c = ((n + 1) & 2) ? -b : b;
}

// (sin x, cos x) of x = deg * (pi/180) for |deg| <= 20 (an upright drone,
// config.py's max landing angle) by Taylor polynomials with no range
// reduction: sin to x^9, cos to x^8, so |error| <= |x|^11/11! + rounding
// < 3e-13 (sin) and |x|^10/10! < 8e-12 (cos) at |x| <= 0.3491.  Not the
// reference's sin/cos to the ulp: only for the landing test's bottom
// centre, which decides on_pad by comparisons whose risky band (2^-19
// relative, frame.h) is ~10^6 times wider than 10 x this error, so every
// decision outside the band is the reference's and the band is redone with
// glibc's functions.  ~11 VALU instead of the general sincos's ~35.
constexpr double kT3 = -1.0 / 6.0, kT5 = 1.0 / 120.0, kT7 = -1.0 / 5040.0, kT9 = 1.0 / 362880.0;
constexpr double kT2 = -0.5, kT4 = 1.0 / 24.0, kT6 = -1.0 / 720.0, kT8 = 1.0 / 40320.0;
template <bool kSgpr = false>
DD_HD inline void sincos_upright_deg(double deg, double* s, double* c) {
    const double x = deg * (3.14159265358979323846 / 180.0);
    const double z = x * x;
    const double ps = hstep_c<kSgpr>(kT3, z, hstep_c<kSgpr>(kT5, z, hstep(kT7, z, kT9)));
    *s = fma(x * z, ps, x);
    const double pc = hstep_c<kSgpr>(kT2, z, hstep_c<kSgpr>(kT4, z, hstep(kT6, z, kT8)));
    *c = fma(z, pc, 1.0);
}

#if defined(__HIPCC__)
// sqrt(x), correctly rounded, for x >= 2^-767, +-0, +inf and NaN: the
// instruction sequence ROCm's compiler emits for a double sqrt on gfx950
// (v_rsq_f64, then Goldschmidt / Newton refinements), without the scaling
// it wraps around them for inputs below 2^-767 (a compare, two selects and
// two v_ldexp_f64 per call).  For every input at or above 2^-767 the scaled
// and unscaled sequences are the same operations on the same operand, so
// the results are bit-identical; callers send smaller inputs to sqrt().
__device__ __forceinline__ double sqrt_unscaled(double x) {
#if !defined(__HIP_DEVICE_COMPILE__)
    return sqrt(x);  // the host pass never runs device code
#else
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    g = fma(d, h, g);
    return __builtin_amdgcn_class(x, 0x260) ? x : g;  // +-0 and +inf pass through
#endif
}
#endif

// x / d, correctly rounded, in three double ops instead of the ~10 of the
// general division sequence.  inv_d = RN(1/d); q0 = RN(x * inv_d) is a
// faithful quotient, so by Markstein's theorem RN(q0 + inv_d * (x - q0 * d))
// = RN(x / d): the reference's quotient, bit for bit (finite operands, no
// underflow).  fma() is always fused, whatever -ffp-contract says.
DD_HD inline double div_exact(double x, double d, double inv_d) {
    const double q0 = x * inv_d;
    const double r = fma(-q0, d, x);
    return fma(r, inv_d, q0);
}

// div_exact with x passed through an empty asm between its two uses.  In the
// kRef = false rollout kernels with f64 storage (d and inv_d in registers)
// ROCm 7.2 wrote q0 over x's register and then read that register back as x
// (v_fma_f64 D, -A, B, A: the quotient of the quotient).  The LLVM IR is
// right; the guard changes the machine code's shape.  It costs registers,
// so only those kernels use it; tools/scan_isa.py checks every build.
DD_HD inline double div_exact_guarded(double x, double d, double inv_d) {
    const double q0 = x * inv_d;
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(x));
#endif
    const double r = fma(-q0, d, x);
    return fma(r, inv_d, q0);
}

// physics.normalize_angle (physics.py:26-39) in O(1).  The reference's loops
// subtract (add) 360 while the angle is > 180 (< -180).  For |a| < 2^55 each
// a - 360 is exact (360 is a multiple of ulp(a)), so k passes of the loop
// equal one exact a - k * 360; k comes from a division plus one correction
// either way.  (Past 2^55 the reference's loop never terminates.)
DD_HD inline double normalize_angle(double a) {
    if (a > 180.0) {
        const double k = ceil((a - 180.0) / 360.0);
        double r = a - k * 360.0;
        r = r > 180.0 ? r - 360.0 : r;    // k one short
        r = r <= -180.0 ? r + 360.0 : r;  // k one past: the loop stops once r <= 180
        return r;
    }
    if (a < -180.0) {
        const double k = ceil((-180.0 - a) / 360.0);
        double r = a + k * 360.0;
        r = r < -180.0 ? r + 360.0 : r;
        r = r >= 180.0 ? r - 360.0 : r;
        return r;
    }
    return a;
}

}  // namespace trig
}  // namespace dd
