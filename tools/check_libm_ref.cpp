// Host check of csrc/libm_ref.h against the C library it restates: pow(x, 2.0),
// sin and cos bit for bit on random and adversarial inputs.
//
//   g++ -O2 -ffp-contract=off -I<dir of libm_tables.h> -Ireinforcement-learning-101_amd/csrc \
//       tools/check_libm_ref.cpp -o /tmp/check_libm_ref -lm && /tmp/check_libm_ref [millions]
//
// Inputs: pow — uniform doubles over the frame's ranges (|v| < 16, |d| < 1200),
// log-uniform over 2^-1074..2^1023, and squares near rounding midpoints (the
// only inputs where glibc's pow differs from x*x); sin / cos — np.radians of
// uniform degrees in [-540, 540] (the frame's angles), of the integer and
// half-integer degrees, and uniform radians in [-10, 10].
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "libm_tables.h"

static const double dd_libm_pow_tab[384] = DD_LIBM_POW_TAB;
static const uint64_t dd_libm_exp_tab[256] = DD_LIBM_EXP_TAB;
static const double dd_libm_sincos_tab[440] = DD_LIBM_SINCOS_TAB;
#define DD_LIBM_FN static inline
#include "libm_ref.h"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next() {  // splitmix64
    uint64_t z = (rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double uni(double lo, double hi) { return lo + (hi - lo) * ((next() >> 11) * 0x1p-53); }
static double as_d(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }
static uint64_t as_u(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }

static long long bad_pow, bad_sin, bad_cos, n_pow, n_trig, pow_ne_mul;

static void check_pow(double x) {
    volatile double two = 2.0;
    const double want = pow(x, two), got = dd::libm::pow2(x);
    ++n_pow;
    pow_ne_mul += want != x * x;
    if (as_u(want) != as_u(got) && !(isnan(want) && isnan(got))) {
        if (bad_pow < 8) printf("pow(%a, 2): libm %a, ref %a\n", x, want, got);
        ++bad_pow;
    }
}

static long long bad_sincos;

static void check_trig(double x) {
    const double ws = sin(x), gs = dd::libm::sin(x), wc = cos(x), gc = dd::libm::cos(x);
    double ss, cc;
    dd::libm::sincos(x, &ss, &cc);
    if (as_u(ss) != as_u(ws) || as_u(cc) != as_u(wc)) {
        if (bad_sincos < 8) printf("sincos(%a): libm %a %a, ref %a %a\n", x, ws, wc, ss, cc);
        ++bad_sincos;
    }
    ++n_trig;
    if (as_u(ws) != as_u(gs)) {
        if (bad_sin < 8) printf("sin(%a): libm %a, ref %a\n", x, ws, gs);
        ++bad_sin;
    }
    if (as_u(wc) != as_u(gc)) {
        if (bad_cos < 8) printf("cos(%a): libm %a, ref %a\n", x, wc, gc);
        ++bad_cos;
    }
}

int main(int argc, char** argv) {
    const long long m = (argc > 1 ? atoll(argv[1]) : 10) * 1000000LL;
    const double deg2rad = 3.14159265358979323846 / 180.0;
    for (long long i = 0; i < m; ++i) {
        check_pow(uni(-16, 16));
        check_pow(uni(-1200, 1200));
        check_pow(as_d(next() & 0x7fefffffffffffffull));  // any finite magnitude
        // near-midpoint squares: x = m * 2^-26 with m odd gives x*x ending in a single 1 bit
        const double y = uni(0.5, 64);
        const double near = as_d((as_u(y) & ~0x7FFFFFFull) | (next() & 0x3) | 0x4000000ull);
        check_pow(near);
        check_trig(uni(-540, 540) * deg2rad);
        if ((i & 7) == 0) check_trig(uni(-10, 10));
        if ((i & 15) == 0) check_trig(uni(-1e-7, 1e-7));  // the tiny ranges
    }
    for (int d = -1080; d <= 1080; ++d) check_trig((d * 0.5) * deg2rad);
    const double special[] = {0.0, -0.0, 1e-310, -1e-310, 5e-324, 1e-160, 1e154, 1.3e154, INFINITY, -INFINITY, NAN, 1.0,
                              -1.0, 3.0, 1e300};
    for (double s : special) check_pow(s);
    const double tsp[] = {0.0, -0.0, 0x1p-27, -0x1p-27, 0x1p-26, 0x1.fffffffffffffp-28, 0.855469, 0.126, -0.126,
                          2.426265, -2.426265, 3.14159265358979323846, 1e8, 105414300.0};
    for (double t : tsp) check_trig(t);
    printf("pow(x, 2): %lld / %lld differ from libm (libm != x*x on %lld)\n", bad_pow, n_pow, pow_ne_mul);
    printf("sin: %lld / %lld differ; cos: %lld / %lld differ; sincos (vs separate sin, cos): %lld differ\n", bad_sin,
           n_trig, bad_cos, n_trig, bad_sincos);
    return (bad_pow || bad_sin || bad_cos || bad_sincos) ? 1 : 0;
}
