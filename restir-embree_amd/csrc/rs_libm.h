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
 * Only +, -, *, /, fma, conversions, bit moves and constant tables are used (no hardware transcendental
 * approximations, no libm calls; fma is exactly rounded everywhere); both sides compile it with -ffp-contract=off, so the same operations round the same way.
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

/* powf's core, e^(y log x) for a positive finite float x and a finite float y, in double with table-driven
 * reductions (the tables: scripts/gen_libm_tables.py).  log: x = 2^e m, m in [1, 2), c = the 21-bit reciprocal of
 * m's 1/128-interval centre, r = m c - 1 exact (|r| < 2^-8), log1p(r) to r^6 (truncation < 2^-58 absolute);
 * exp: t = k ln2/128 + r (|r| <= ln2/256), e^r - 1 to r^5 (truncation < 2^-60), 2^(k/128) from the table.
 * Relative error of the double result below 2^-44 for every |y log x| <= 160, so the float result is the
 * correctly rounded one unless the true value lies within that of a float rounding boundary.  fma is exactly
 * rounded on both sides (v_fma_f64 on gfx950, the C library's fma on the host). */
#define RS_LM_LOG_TAB_INIT { \
    0x1.fe02000000000p-1, 0x1.fefeaa2b11bc0p-9, 0x1.fa11c00000000p-1, 0x1.7dc725f817e07p-7, \
    0x1.f631000000000p-1, 0x1.3ceba4346e1f5p-6, 0x1.f25f600000000p-1, 0x1.b9fc8e7af9b2ap-6, \
    0x1.ee9c800000000p-1, 0x1.1b0d90923d990p-5, 0x1.eae8000000000p-1, 0x1.58a63afc8f4d5p-5, \
    0x1.e741a00000000p-1, 0x1.95c8deec9017cp-5, 0x1.e3a9200000000p-1, 0x1.d2762aadb1f03p-5, \
    0x1.e01e000000000p-1, 0x1.075993598e4f1p-4, 0x1.dca0200000000p-1, 0x1.253f4ff0a14cbp-4, \
    0x1.d92f200000000p-1, 0x1.42eddeea647a5p-4, 0x1.d5cac00000000p-1, 0x1.6065d09375a56p-4, \
    0x1.d272c00000000p-1, 0x1.7da7c0d7b229fp-4, 0x1.cf26e00000000p-1, 0x1.9ab45762038c1p-4, \
    0x1.cbe6e00000000p-1, 0x1.b78c47bb0f46ep-4, 0x1.c8b2600000000p-1, 0x1.d4317066cb872p-4, \
    0x1.c589400000000p-1, 0x1.f0a3820117dd8p-4, 0x1.c26b600000000p-1, 0x1.067118aca65e6p-3, \
    0x1.bf58400000000p-1, 0x1.14785346742c5p-3, 0x1.bc4fe00000000p-1, 0x1.2266c510a6288p-3, \
    0x1.b951e00000000p-1, 0x1.303d7e0e4806fp-3, 0x1.b65e200000000p-1, 0x1.3dfc6d8ecd770p-3, \
    0x1.b374800000000p-1, 0x1.4ba38539a57c9p-3, 0x1.b094c00000000p-1, 0x1.5933509982f0fp-3, \
    0x1.adbe800000000p-1, 0x1.66acfa272b2f5p-3, 0x1.aaf1e00000000p-1, 0x1.740f50d4046e7p-3, \
    0x1.a82e600000000p-1, 0x1.815c229435a43p-3, 0x1.a574200000000p-1, 0x1.8e92426888385p-3, \
    0x1.a2c2a00000000p-1, 0x1.9bb38c67e023ep-3, 0x1.a01a000000000p-1, 0x1.a8bed7c882f59p-3, \
    0x1.9d7a000000000p-1, 0x1.b5b4d1e8fc9e4p-3, 0x1.9ae2400000000p-1, 0x1.c296ce58c2d92p-3, \
    0x1.9853000000000p-1, 0x1.cf6308e09dc6cp-3, 0x1.95cbc00000000p-1, 0x1.dc1b7d0ac03a6p-3, \
    0x1.934c600000000p-1, 0x1.e8c04daaa60c8p-3, 0x1.90d5000000000p-1, 0x1.f5505964b91c7p-3, \
    0x1.8e65200000000p-1, 0x1.00e6d81ad5329p-2, 0x1.8bfce00000000p-1, 0x1.071b9abcd5c6ap-2, \
    0x1.899c000000000p-1, 0x1.0d46dd79ac3cbp-2, 0x1.8742800000000p-1, 0x1.136865293a9a2p-2, \
    0x1.84f0000000000p-1, 0x1.1980f2dd42b6fp-2, 0x1.82a4a00000000p-1, 0x1.1f8ffa248a2f3p-2, \
    0x1.8060200000000p-1, 0x1.2595ebcdf79c1p-2, 0x1.7e22600000000p-1, 0x1.2b92e66b8a3d4p-2, \
    0x1.7beb400000000p-1, 0x1.31870a1544431p-2, 0x1.79baa00000000p-1, 0x1.3772786bfdaf5p-2, \
    0x1.7790800000000p-1, 0x1.3d54fd5c1f722p-2, 0x1.756ca00000000p-1, 0x1.432f13e04f0b7p-2, \
    0x1.734f000000000p-1, 0x1.49008a04012d9p-2, 0x1.7137800000000p-1, 0x1.4ec986260053cp-2, \
    0x1.6f26000000000p-1, 0x1.548a303add283p-2, 0x1.6d1a600000000p-1, 0x1.5a42b1cf4d03dp-2, \
    0x1.6b14a00000000p-1, 0x1.5ff2dbca7a271p-2, 0x1.6914800000000p-1, 0x1.659b34303eb85p-2, \
    0x1.671a000000000p-1, 0x1.6b3b8e2359e5ep-2, 0x1.6525000000000p-1, 0x1.70d41827895fep-2, \
    0x1.6335600000000p-1, 0x1.766502639e472p-2, 0x1.614b400000000p-1, 0x1.7bedc5237b5a8p-2, \
    0x1.5f66400000000p-1, 0x1.816f4b5a0d54ap-2, 0x1.5d86800000000p-1, 0x1.86e90ea330c92p-2, \
    0x1.5babc00000000p-1, 0x1.8c5ba1058bef3p-2, 0x1.59d6200000000p-1, 0x1.91c67bf45a84dp-2, \
    0x1.5805600000000p-1, 0x1.972a345135159p-2, 0x1.5639800000000p-1, 0x1.9c86a32dc09b5p-2, \
    0x1.5472600000000p-1, 0x1.a1dc018d5b9c3p-2, 0x1.52b0000000000p-1, 0x1.a72a2966be1eap-2, \
    0x1.50f2200000000p-1, 0x1.ac71b6e58bf2bp-2, 0x1.4f39000000000p-1, 0x1.b1b1c2ebe0363p-2, \
    0x1.4d84400000000p-1, 0x1.b6eb4d53cf496p-2, 0x1.4bd3e00000000p-1, 0x1.bc1e3370dbb51p-2, \
    0x1.4a28000000000p-1, 0x1.c149ef115f227p-2, 0x1.4880600000000p-1, 0x1.c66f22fff7e95p-2, \
    0x1.46dce00000000p-1, 0x1.cb8e1184d7b9cp-2, 0x1.453da00000000p-1, 0x1.d0a6352721ea6p-2, \
    0x1.43a2800000000p-1, 0x1.d5b7d0ae2d3a6p-2, 0x1.420b600000000p-1, 0x1.dac328a2c67f1p-2, \
    0x1.4078200000000p-1, 0x1.dfc883506e353p-2, 0x1.3ee9000000000p-1, 0x1.e4c6f4868824cp-2, \
    0x1.3d5da00000000p-1, 0x1.e9bf9019865d4p-2, 0x1.3bd6000000000p-1, 0x1.eeb238640ed14p-2, \
    0x1.3a52400000000p-1, 0x1.f39e674811f64p-2, 0x1.38d2200000000p-1, 0x1.f884ceafead5fp-2, \
    0x1.3755c00000000p-1, 0x1.fd64e88f61626p-2, 0x1.35dce00000000p-1, 0x1.011fb4f260110p-1, \
    0x1.3467a00000000p-1, 0x1.0389e65ce6465p-1, 0x1.32f5c00000000p-1, 0x1.05f1649264f2ep-1, \
    0x1.3187800000000p-1, 0x1.0855b704b49d7p-1, 0x1.301c800000000p-1, 0x1.0ab7706ce1523p-1, \
    0x1.2eb4e00000000p-1, 0x1.0d164deb9db4dp-1, 0x1.2d50a00000000p-1, 0x1.0f7241e9b497dp-1, \
    0x1.2befa00000000p-1, 0x1.11cb75587cf44p-1, 0x1.2a91c00000000p-1, 0x1.1422121244125p-1, \
    0x1.2937200000000p-1, 0x1.1675d49aba794p-1, 0x1.27dfa00000000p-1, 0x1.18c6e71f5cf9cp-1, \
    0x1.268b400000000p-1, 0x1.1b153d17da5cbp-1, 0x1.2539e00000000p-1, 0x1.1d6101c677321p-1, \
    0x1.23eb800000000p-1, 0x1.1faa293870b5dp-1, 0x1.22a0200000000p-1, 0x1.21f0a7665c834p-1, \
    0x1.2157a00000000p-1, 0x1.2434a8d483c52p-1, 0x1.2012000000000p-1, 0x1.26762213430f0p-1, \
    0x1.1ecf400000000p-1, 0x1.28b5079f60839p-1, 0x1.1d8f600000000p-1, 0x1.2af14de264542p-1, \
    0x1.1c52200000000p-1, 0x1.2d2b5c72ee932p-1, 0x1.1b17c00000000p-1, 0x1.2f62b5550976ep-1, \
    0x1.19e0200000000p-1, 0x1.319786da80914p-1, 0x1.18ab000000000p-1, 0x1.33ca3aa328d19p-1, \
    0x1.1778a00000000p-1, 0x1.35fa51bd36ec1p-1, 0x1.1648e00000000p-1, 0x1.3827fbc587fd3p-1, \
    0x1.151ba00000000p-1, 0x1.3a536947ebfbdp-1, 0x1.13f0e00000000p-1, 0x1.3c7c905f73636p-1, \
    0x1.12c8c00000000p-1, 0x1.3ea32b76b3250p-1, 0x1.11a3000000000p-1, 0x1.40c7a7880dd0dp-1, \
    0x1.107fc00000000p-1, 0x1.42e9bf1df81afp-1, 0x1.0f5ee00000000p-1, 0x1.4509a4733bb0cp-1, \
    0x1.0e40600000000p-1, 0x1.47274e133ac47p-1, 0x1.0d24400000000p-1, 0x1.4942b27a2fdacp-1, \
    0x1.0c0a800000000p-1, 0x1.4b5bc8156e5bdp-1, 0x1.0af3000000000p-1, 0x1.4d72c2a3a0184p-1, \
    0x1.09ddc00000000p-1, 0x1.4f879935028b7p-1, 0x1.08cac00000000p-1, 0x1.519a42cba359dp-1, \
    0x1.07ba000000000p-1, 0x1.53aab65b9a60dp-1, 0x1.06ab600000000p-1, 0x1.55b9292b40e19p-1, \
    0x1.059ee00000000p-1, 0x1.57c592d36f795p-1, 0x1.0494a00000000p-1, 0x1.59cfabffae921p-1, \
    0x1.038c600000000p-1, 0x1.5bd7e9ae72473p-1, 0x1.0286400000000p-1, 0x1.5dde04b14a866p-1, \
    0x1.0182400000000p-1, 0x1.5fe1f46d189cfp-1, 0x1.0080400000000p-1, 0x1.61e3f01a46467p-1 }
#define RS_LM_EXP2_TAB_INIT { \
    0x1.0000000000000p+0, 0x1.0163da9fb3335p+0, 0x1.02c9a3e778061p+0, 0x1.04315e86e7f85p+0, \
    0x1.059b0d3158574p+0, 0x1.0706b29ddf6dep+0, 0x1.0874518759bc8p+0, 0x1.09e3ecac6f383p+0, \
    0x1.0b5586cf9890fp+0, 0x1.0cc922b7247f7p+0, 0x1.0e3ec32d3d1a2p+0, 0x1.0fb66affed31bp+0, \
    0x1.11301d0125b51p+0, 0x1.12abdc06c31ccp+0, 0x1.1429aaea92de0p+0, 0x1.15a98c8a58e51p+0, \
    0x1.172b83c7d517bp+0, 0x1.18af9388c8deap+0, 0x1.1a35beb6fcb75p+0, 0x1.1bbe084045cd4p+0, \
    0x1.1d4873168b9aap+0, 0x1.1ed5022fcd91dp+0, 0x1.2063b88628cd6p+0, 0x1.21f49917ddc96p+0, \
    0x1.2387a6e756238p+0, 0x1.251ce4fb2a63fp+0, 0x1.26b4565e27cddp+0, 0x1.284dfe1f56381p+0, \
    0x1.29e9df51fdee1p+0, 0x1.2b87fd0dad990p+0, 0x1.2d285a6e4030bp+0, 0x1.2ecafa93e2f56p+0, \
    0x1.306fe0a31b715p+0, 0x1.32170fc4cd831p+0, 0x1.33c08b26416ffp+0, 0x1.356c55f929ff1p+0, \
    0x1.371a7373aa9cbp+0, 0x1.38cae6d05d866p+0, 0x1.3a7db34e59ff7p+0, 0x1.3c32dc313a8e5p+0, \
    0x1.3dea64c123422p+0, 0x1.3fa4504ac801cp+0, 0x1.4160a21f72e2ap+0, 0x1.431f5d950a897p+0, \
    0x1.44e086061892dp+0, 0x1.46a41ed1d0057p+0, 0x1.486a2b5c13cd0p+0, 0x1.4a32af0d7d3dep+0, \
    0x1.4bfdad5362a27p+0, 0x1.4dcb299fddd0dp+0, 0x1.4f9b2769d2ca7p+0, 0x1.516daa2cf6642p+0, \
    0x1.5342b569d4f82p+0, 0x1.551a4ca5d920fp+0, 0x1.56f4736b527dap+0, 0x1.58d12d497c7fdp+0, \
    0x1.5ab07dd485429p+0, 0x1.5c9268a5946b7p+0, 0x1.5e76f15ad2148p+0, 0x1.605e1b976dc09p+0, \
    0x1.6247eb03a5585p+0, 0x1.6434634ccc320p+0, 0x1.6623882552225p+0, 0x1.68155d44ca973p+0, \
    0x1.6a09e667f3bcdp+0, 0x1.6c012750bdabfp+0, 0x1.6dfb23c651a2fp+0, 0x1.6ff7df9519484p+0, \
    0x1.71f75e8ec5f74p+0, 0x1.73f9a48a58174p+0, 0x1.75feb564267c9p+0, 0x1.780694fde5d3fp+0, \
    0x1.7a11473eb0187p+0, 0x1.7c1ed0130c132p+0, 0x1.7e2f336cf4e62p+0, 0x1.80427543e1a12p+0, \
    0x1.82589994cce13p+0, 0x1.8471a4623c7adp+0, 0x1.868d99b4492edp+0, 0x1.88ac7d98a6699p+0, \
    0x1.8ace5422aa0dbp+0, 0x1.8cf3216b5448cp+0, 0x1.8f1ae99157736p+0, 0x1.9145b0b91ffc6p+0, \
    0x1.93737b0cdc5e5p+0, 0x1.95a44cbc8520fp+0, 0x1.97d829fde4e50p+0, 0x1.9a0f170ca07bap+0, \
    0x1.9c49182a3f090p+0, 0x1.9e86319e32323p+0, 0x1.a0c667b5de565p+0, 0x1.a309bec4a2d33p+0, \
    0x1.a5503b23e255dp+0, 0x1.a799e1330b358p+0, 0x1.a9e6b5579fdbfp+0, 0x1.ac36bbfd3f37ap+0, \
    0x1.ae89f995ad3adp+0, 0x1.b0e07298db666p+0, 0x1.b33a2b84f15fbp+0, 0x1.b59728de5593ap+0, \
    0x1.b7f76f2fb5e47p+0, 0x1.ba5b030a1064ap+0, 0x1.bcc1e904bc1d2p+0, 0x1.bf2c25bd71e09p+0, \
    0x1.c199bdd85529cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c67f12e57d14bp+0, 0x1.c8f6d9406e7b5p+0, \
    0x1.cb720dcef9069p+0, 0x1.cdf0b555dc3fap+0, 0x1.d072d4a07897cp+0, 0x1.d2f87080d89f2p+0, \
    0x1.d5818dcfba487p+0, 0x1.d80e316c98398p+0, 0x1.da9e603db3285p+0, 0x1.dd321f301b460p+0, \
    0x1.dfc97337b9b5fp+0, 0x1.e264614f5a129p+0, 0x1.e502ee78b3ff6p+0, 0x1.e7a51fbc74c83p+0, \
    0x1.ea4afa2a490dap+0, 0x1.ecf482d8e67f1p+0, 0x1.efa1bee615a27p+0, 0x1.f252b376bba97p+0, \
    0x1.f50765b6e4540p+0, 0x1.f7bfdad9cbe14p+0, 0x1.fa7c1819e90d8p+0, 0x1.fd3c22b8f71f1p+0 }

#if defined(__HIP__)
static __constant__ const double rs_lm_log_tab_dev[256] = RS_LM_LOG_TAB_INIT;
static __constant__ const double rs_lm_exp2_tab_dev[128] = RS_LM_EXP2_TAB_INIT;
#endif
static const double rs_lm_log_tab_host[256] = RS_LM_LOG_TAB_INIT;
static const double rs_lm_exp2_tab_host[128] = RS_LM_EXP2_TAB_INIT;
#if defined(__HIP_DEVICE_COMPILE__)
#define RS_LM_TAB(n) n##_dev
#else
#define RS_LM_TAB(n) n##_host
#endif
#define RS_LM_LN2_128_HI 0x1.62e42feep-8           /* ln2 / 128 to 33 significant bits: k hi exact */
#define RS_LM_LN2_128_LO 1.4907929134926466e-12
#define RS_LM_128_OVER_LN2 184.6649652337873

RS_LM double rs_lm_pow_core(float ax, float y) {
    uint32_t b = rs_lm_fbits(ax);
    int e = -127;
    if (b < 0x00800000u) { b = rs_lm_fbits(ax * 8388608.0f); e -= 23; }          /* subnormal: x 2^23 */
    e += (int)(b >> 23);
    const int i = (int)((b >> 16) & 127);
    const double m = (double)rs_lm_flt((b & 0x007fffffu) | 0x3f800000u);
    const double r = m * RS_LM_TAB(rs_lm_log_tab)[2 * i] - 1.0;                   /* exact */
    double p = __builtin_fma(r, -1.0 / 6.0, 1.0 / 5.0);
    p = __builtin_fma(r, p, -0.25);
    p = __builtin_fma(r, p, 1.0 / 3.0);
    p = __builtin_fma(r, p, -0.5);
    const double l1p = __builtin_fma(r * r, p, r);
    const double de = (double)e;
    const double lx = __builtin_fma(de, RS_LM_LN2_HI, RS_LM_TAB(rs_lm_log_tab)[2 * i + 1]) +
                      __builtin_fma(de, RS_LM_LN2_LO, l1p);
    const double t = (double)y * lx;
    if (t > 128.0) return RS_LM_DINF;
    if (t < -160.0) return 0.0;
    const double u = t * RS_LM_128_OVER_LN2;
    const int k = (int)(u >= 0.0 ? u + 0.5 : u - 0.5);
    const double dk = (double)k;
    double rr = __builtin_fma(dk, -RS_LM_LN2_128_HI, t);
    rr = __builtin_fma(dk, -RS_LM_LN2_128_LO, rr);
    double q = __builtin_fma(rr, 1.0 / 120.0, 1.0 / 24.0);
    q = __builtin_fma(rr, q, 1.0 / 6.0);
    q = __builtin_fma(rr, q, 0.5);
    const double em1 = __builtin_fma(rr * rr, q, rr);
    const int j = k & 127;
    const int64_t qk = (int64_t)((k - j) / 128);
    const double s = rs_lm_dbl(rs_lm_bits(RS_LM_TAB(rs_lm_exp2_tab)[j]) + ((uint64_t)qk << 52));
    return __builtin_fma(s, em1, s);
}

#if defined(__HIP__)
/* the core as a called function (rs_powf_sel's `call`): its constants and temporaries stay out of the calling
   kernel's register allocation -- a gain in the register-bound per-lane kernels, a loss in the lockstep ones */
__host__ __device__ static __attribute__((noinline)) double rs_lm_pow_core_call(float ax, float y) {
    return rs_lm_pow_core(ax, y);
}
#endif
/* x^y (C99 special cases); call != 0 (a constant at every call site): the core by rs_lm_pow_core_call */
RS_LM float rs_powf_sel(float x, float y, int call) {
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
    float r;
    if (ax == 0.0f) r = y > 0.0f ? 0.0f : RS_LM_FINF;
    else if (rs_lm_fbits(ax) == 0x7f800000u) r = y > 0.0f ? ax : 0.0f;   /* (-inf)^y: sign by y_odd only */
    else if (x < 0.0f && !y_int) return RS_LM_FNAN;
    else {
#if defined(__HIP_DEVICE_COMPILE__)
        r = (float)(call ? rs_lm_pow_core_call(ax, y) : rs_lm_pow_core(ax, y));
#else
        (void)call;
        r = (float)rs_lm_pow_core(ax, y);
#endif
    }
    return neg ? -r : r;
}
RS_LM float rs_powf(float x, float y) { return rs_powf_sel(x, y, 0); }

/* sin and cos of a float angle (the path's angles are 2 pi U, U in [0, 1)): Cody-Waite reduction by pi/2 in
 * double, Taylor cores on |r| <= pi/4 */
#define RS_LM_PIO2_HI 1.57079632673412561417e+00   /* 0x3ff921fb54400000: 33 significant bits */
#define RS_LM_PIO2_LO 6.07710050650619224932e-11
#define RS_LM_2_OVER_PI 6.36619772367581382433e-01
RS_LM double rs_lm_sin_core(double r) {          /* |r| <= pi/4, to r^15 / 15! (truncation < 6e-17 relative) */
    const double z = r * r;
    double p = __builtin_fma(z, -1.0 / 1307674368000.0, 1.0 / 6227020800.0);
    p = __builtin_fma(z, p, -1.0 / 39916800.0);
    p = __builtin_fma(z, p, 1.0 / 362880.0);
    p = __builtin_fma(z, p, -1.0 / 5040.0);
    p = __builtin_fma(z, p, 1.0 / 120.0);
    p = __builtin_fma(z, p, -1.0 / 6.0);
    return __builtin_fma(r * z, p, r);
}
RS_LM double rs_lm_cos_core(double r) {          /* |r| <= pi/4, to r^16 / 16! (truncation < 3e-18) */
    const double z = r * r;
    double p = __builtin_fma(z, 1.0 / 20922789888000.0, -1.0 / 87178291200.0);
    p = __builtin_fma(z, p, 1.0 / 479001600.0);
    p = __builtin_fma(z, p, -1.0 / 3628800.0);
    p = __builtin_fma(z, p, 1.0 / 40320.0);
    p = __builtin_fma(z, p, -1.0 / 720.0);
    p = __builtin_fma(z, p, 1.0 / 24.0);
    return __builtin_fma(z, __builtin_fma(z, p, -0.5), 1.0);
}
RS_LM void rs_sincosf(float a, float* s, float* c) {
    const double x = (double)a;
    if (x != x || x - x != 0.0) { *s = (float)(x - x); *c = (float)(x - x); return; }   /* NaN, +-inf -> NaN */
    const double t = x * RS_LM_2_OVER_PI;
    const int64_t k = (int64_t)(t >= 0.0 ? t + 0.5 : t - 0.5);
    const double dk = (double)k;
    const double r = __builtin_fma(-dk, RS_LM_PIO2_LO, __builtin_fma(-dk, RS_LM_PIO2_HI, x));
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
