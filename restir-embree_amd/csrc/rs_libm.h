/* rs_libm.h -- the transcendental functions of the ReSTIR DI path as fixed sequences of IEEE-754 operations,
 * shared bit for bit by the gfx950 kernels and the CPU restatement (oracle/restir_oracle.c includes this file).
 *
 * Why: the reference calls its platform's libm (MSVC's) for powf / expf / lgammaf / sinf / cosf and Boost's
 * ibeta in double (pg/MaterialPhong.cpp:122-248, pg/Distribution.h:7-68, pg/Sampling.cpp:78-87).  ROCm's ocml
 * and glibc round differently in the last place, and a last-ulp difference can move `U < w / w_sum`
 * (pg/Reservoir.h:33-47) and flip a reservoir's selection -- a flip the capped history then carries for
 * frames.  Neither libm is the reference's, so faithfulness does not prefer either; one shared sequence
 * makes GPU and CPU frames identical.  Every function here is computed in double with polynomial cores
 * accurate to a few double ulps, so the float results are the correctly rounded values except in the rare
 * case that the true value lies within ~1e-16 relative of a float rounding boundary (tests/test_oracle.py
 * checks them against numpy/glibc double precision on dense grids).
 *
 * Only +, -, *, /, conversions and bit moves are used (no fma, no hardware transcendental approximations,
 * no libm calls); both sides compile it with -ffp-contract=off, so the same operations round the same way.
 * Plain C99 (the oracle is C) and HIP (host + device).
 */
#ifndef RS_LIBM_H
#define RS_LIBM_H
#include <stdint.h>

#if defined(__HIP__)
#define RS_LM __host__ __device__ static inline
#else
#define RS_LM static inline
#endif

RS_LM uint64_t rs_lm_bits(double d) { uint64_t u; __builtin_memcpy(&u, &d, 8); return u; }
RS_LM double rs_lm_dbl(uint64_t u) { double d; __builtin_memcpy(&d, &u, 8); return d; }
RS_LM uint32_t rs_lm_fbits(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
RS_LM float rs_lm_flt(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
#define RS_LM_DINF rs_lm_dbl(0x7ff0000000000000ull)
#define RS_LM_DNAN rs_lm_dbl(0x7ff8000000000000ull)
#define RS_LM_FINF rs_lm_flt(0x7f800000u)
#define RS_LM_FNAN rs_lm_flt(0x7fc00000u)
/* 2^k for -1022 <= k <= 1023 */
RS_LM double rs_lm_pow2(int k) { return rs_lm_dbl((uint64_t)(k + 1023) << 52); }

#define RS_LM_LN2_HI 6.93147180369123816490e-01  /* 0x3fe62e42fee00000: 32 significant bits, k * hi exact */
#define RS_LM_LN2_LO 1.90821492927058770002e-10
#define RS_LM_INV_LN2 1.44269504088896338700e+00
#define RS_LM_SQRT2 1.41421356237309514547e+00

/* natural logarithm, double */
RS_LM double rs_log_d(double x) {
    const uint64_t b = rs_lm_bits(x);
    if (x != x) return x;
    if (x < 0.0) return RS_LM_DNAN;
    if (x == 0.0) return -RS_LM_DINF;
    if (b == 0x7ff0000000000000ull) return x;                                     /* +inf */
    int e = 0;
    double m = x;
    if (x < 2.2250738585072014e-308) { m = x * 18014398509481984.0; e = -54; }    /* subnormal: x 2^54 */
    const uint64_t mb = rs_lm_bits(m);
    e += (int)((mb >> 52) & 0x7ff) - 1023;
    m = rs_lm_dbl((mb & 0x000fffffffffffffull) | 0x3ff0000000000000ull);          /* [1, 2) */
    if (m > RS_LM_SQRT2) { m = m * 0.5; e += 1; }                                  /* [0.707, 1.414] */
    /* log(m) = 2 atanh(s), s = (m - 1) / (m + 1), |s| <= 0.1716: 2s + 2s z (1/3 + z/5 + ... + z^9/21), z = s^2 */
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s;
    double p = 1.0 / 21.0;
    p = 1.0 / 19.0 + z * p;
    p = 1.0 / 17.0 + z * p;
    p = 1.0 / 15.0 + z * p;
    p = 1.0 / 13.0 + z * p;
    p = 1.0 / 11.0 + z * p;
    p = 1.0 / 9.0 + z * p;
    p = 1.0 / 7.0 + z * p;
    p = 1.0 / 5.0 + z * p;
    p = 1.0 / 3.0 + z * p;
    const double two_s = s + s;
    const double lm = two_s + two_s * (z * p);
    const double de = (double)e;
    return de * RS_LM_LN2_HI + (lm + de * RS_LM_LN2_LO);
}

/* e^x, double */
RS_LM double rs_exp_d(double x) {
    if (x != x) return x;
    if (x > 709.782712893384) return RS_LM_DINF;
    if (x < -745.2) return 0.0;
    const double t = x * RS_LM_INV_LN2;
    const int k = (int)(t >= 0.0 ? t + 0.5 : t - 0.5);                 /* round to nearest, ties away */
    const double dk = (double)k;
    const double r = (x - dk * RS_LM_LN2_HI) - dk * RS_LM_LN2_LO;    /* |r| <= 0.347 */
    /* Taylor to r^14 / 14! (truncation < 4e-18 relative) */
    double p = 1.0 / 87178291200.0;
    p = 1.0 / 6227020800.0 + r * p;
    p = 1.0 / 479001600.0 + r * p;
    p = 1.0 / 39916800.0 + r * p;
    p = 1.0 / 3628800.0 + r * p;
    p = 1.0 / 362880.0 + r * p;
    p = 1.0 / 40320.0 + r * p;
    p = 1.0 / 5040.0 + r * p;
    p = 1.0 / 720.0 + r * p;
    p = 1.0 / 120.0 + r * p;
    p = 1.0 / 24.0 + r * p;
    p = 1.0 / 6.0 + r * p;
    p = 0.5 + r * p;
    p = r + (r * r) * p;          /* e^r - 1 */
    const double er = 1.0 + p;
    if (k >= -1021 && k <= 1023) return er * rs_lm_pow2(k);
    if (k > 1023) return er * rs_lm_pow2(k - 1) * 2.0;
    return er * rs_lm_pow2(k + 1000) * rs_lm_pow2(-1000);             /* subnormal result: one rounding at the end */
}

/* log(1 + x), double, x > -1 (log(u) * x / (u - 1), u = 1 + x rounded) */
RS_LM double rs_log1p_d(double x) {
    if (x != x) return x;
    const double u = 1.0 + x;
    if (u == 1.0) return x;
    return rs_log_d(u) * (x / (u - 1.0));
}

/* log Gamma(x), double, x > 0 (the path's domain: shininess / 2 + 1/2 and its neighbours); x <= 0 -> +inf / NaN */
RS_LM double rs_lgamma_d(double x) {
    if (x != x) return x;
    if (x == 0.0) return RS_LM_DINF;
    if (x < 0.0) return RS_LM_DNAN;
    if (x == 1.0 || x == 2.0) return 0.0;
    if (x > 1e300) return RS_LM_DINF;
    /* shift up to x >= 10 (lgamma(x) = lgamma(x + n) - log(x (x+1) ... (x+n-1))), then Stirling's series */
    double prod = 1.0;
    while (x < 10.0) { prod = prod * x; x = x + 1.0; }
    const double ix = 1.0 / x, ix2 = ix * ix;
    double s = 1.0 / 156.0;                      /* B_14 / (14 * 13) */
    s = -691.0 / 360360.0 + ix2 * s;
    s = 1.0 / 1188.0 + ix2 * s;
    s = -1.0 / 1680.0 + ix2 * s;
    s = 1.0 / 1260.0 + ix2 * s;
    s = -1.0 / 360.0 + ix2 * s;
    s = 1.0 / 12.0 + ix2 * s;
    const double half_log_2pi = 0.91893853320467274178;
    const double lg = ((x - 0.5) * rs_log_d(x) - x) + (half_log_2pi + s * ix);
    return prod == 1.0 ? lg : lg - rs_log_d(prod);
}

RS_LM float rs_expf(float x) { return (float)rs_exp_d((double)x); }
RS_LM float rs_lgammaf(float x) { return (float)rs_lgamma_d((double)x); }

/* x^y (C99 special cases) */
RS_LM float rs_powf(float x, float y) {
    if (y == 0.0f || x == 1.0f) return 1.0f;
    if (x != x || y != y) return x + y;
    const double ay = y < 0.0f ? -(double)y : (double)y;
    const int y_inf = ay > 3.4028234663852886e38;
    /* y an odd integer: |y| < 2^24 and y == trunc(y) and trunc(y) odd */
    int y_odd = 0, y_int = 0;
    if (!y_inf) {
        if (ay >= 16777216.0) { y_int = 1; }
        else {
            const int64_t iy = (int64_t)ay;
            y_int = (double)iy == ay;
            y_odd = y_int && (iy & 1);
        }
    }
    const float ax = x < 0.0f ? -x : x;
    if (y_inf) {
        if (ax == 1.0f) return 1.0f;
        return ((ax < 1.0f) == (y > 0.0f)) ? 0.0f : RS_LM_FINF;
    }
    const int neg = (rs_lm_fbits(x) >> 31) && y_odd;   /* odd integer power of a negative (or -0) base */
    if (x < 0.0f && !y_int) return RS_LM_FNAN;
    float r;
    if (ax == 0.0f) r = y > 0.0f ? 0.0f : RS_LM_FINF;
    else if (rs_lm_fbits(ax) == 0x7f800000u) r = y > 0.0f ? ax : 0.0f;
    else r = (float)rs_exp_d((double)y * rs_log_d((double)ax));
    return neg ? -r : r;
}

/* sin and cos of a float angle (the path's angles are 2 pi U, U in [0, 1)): Cody-Waite reduction by pi/2 in
 * double, Taylor cores on |r| <= pi/4 */
#define RS_LM_PIO2_HI 1.57079632673412561417e+00   /* 0x3ff921fb54400000: 33 significant bits */
#define RS_LM_PIO2_LO 6.07710050650619224932e-11
#define RS_LM_2_OVER_PI 6.36619772367581382433e-01
RS_LM double rs_lm_sin_core(double r) {          /* |r| <= pi/4, to r^17 / 17! */
    const double z = r * r;
    double p = 1.0 / 355687428096000.0;
    p = -1.0 / 1307674368000.0 + z * p;
    p = 1.0 / 6227020800.0 + z * p;
    p = -1.0 / 39916800.0 + z * p;
    p = 1.0 / 362880.0 + z * p;
    p = -1.0 / 5040.0 + z * p;
    p = 1.0 / 120.0 + z * p;
    p = -1.0 / 6.0 + z * p;
    return r + (r * z) * p;
}
RS_LM double rs_lm_cos_core(double r) {          /* |r| <= pi/4, to r^18 / 18! */
    const double z = r * r;
    double p = -1.0 / 6402373705728000.0;
    p = 1.0 / 20922789888000.0 + z * p;
    p = -1.0 / 87178291200.0 + z * p;
    p = 1.0 / 479001600.0 + z * p;
    p = -1.0 / 3628800.0 + z * p;
    p = 1.0 / 40320.0 + z * p;
    p = -1.0 / 720.0 + z * p;
    p = 1.0 / 24.0 + z * p;
    return 1.0 + z * (-0.5 + z * p);
}
RS_LM void rs_sincosf(float a, float* s, float* c) {
    const double x = (double)a;
    if (x != x || x - x != 0.0) { *s = (float)(x - x); *c = (float)(x - x); return; }   /* NaN, +-inf -> NaN */
    const double t = x * RS_LM_2_OVER_PI;
    const int64_t k = (int64_t)(t >= 0.0 ? t + 0.5 : t - 0.5);
    const double dk = (double)k;
    const double r = (x - dk * RS_LM_PIO2_HI) - dk * RS_LM_PIO2_LO;
    const double sr = rs_lm_sin_core(r), cr = rs_lm_cos_core(r);
    double sv, cv;
    switch ((int)(k & 3)) {
        case 0: sv = sr; cv = cr; break;
        case 1: sv = cr; cv = -sr; break;
        case 2: sv = -sr; cv = -cr; break;
        default: sv = -cr; cv = sr; break;
    }
    *s = (float)sv;
    *c = (float)cv;
}
RS_LM float rs_sinf(float a) { float s, c; rs_sincosf(a, &s, &c); return s; }
RS_LM float rs_cosf(float a) { float s, c; rs_sincosf(a, &s, &c); return c; }

#endif /* RS_LIBM_H */
