/*
 * restir_oracle.c -- CPU restatement of the reference ReSTIR DI hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product (restir-embree_amd/, librestir_amd.so) never links or calls it.
 *
 * Reference: Tonz24/restir-embree @ /root/reference (read-only).  Citation legend:
 *   pg/ = template/src/pg/pg1_embree/
 * Every function below names the reference file:line it restates.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - The reference's hot path cannot be compiled here (Embree/D3D11/OIDN/assimp are
 *     Windows-only binaries; its translation units need stand-ins for stdafx.h and the
 *     Embree library).  This restatement is therefore pinned by
 *       (a) tests/golden/ibeta_kat.json  - generated from the reference's vendored
 *           Boost 1.86 boost::math::beta (oracle/kat/gen_ibeta.cpp), pins calc_I_M;
 *       (b) tests/golden/glm_kat.json    - generated from the reference's vendored glm
 *           0.9.9 (oracle/kat/gen_glm.cpp), pins camera matrices, primary rays,
 *           reflect/normalize/round/trunc semantics;
 *     and everything else (reservoir logic, pass order, MIS modes) is "parity unpinned":
 *     restated line by line from the cited source, no reference fixture exists.
 *   - Embree 3.13.5's triangle/traversal arithmetic is replaced by Moller-Trumbore with
 *     a fixed tie-break (smaller t, then smaller triangle index) -- parity unpinned at the
 *     Embree boundary (no Embree here), identical rule in the HIP product.
 *   - The reference's global mt19937 (pg/utils.cpp:175-202) is replaced by a counter RNG
 *     keyed by (seed, frame, pass, pixel, draw#), consumed in the reference's per-pixel
 *     draw order.  The HIP product uses the identical RNG.
 *
 * Build: oracle/Makefile -> oracle/_build/librestir_oracle.so  (gcc -O2 -fopenmp)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <immintrin.h>
/* the path's transcendental functions: one shared sequence of IEEE operations with the HIP kernels
 * (restir-embree_amd/csrc/rs_libm.h), so frames match bit for bit; glibc's libm is not called on the path */
#include "../restir-embree_amd/csrc/rs_libm.h"
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ constants */
#define OR_PI          3.14159265358979323846264338327950288f   /* glm::pi<float>() */
#define OR_ONE_OVER_PI 0.318309886183790671537767526745028724f  /* glm::one_over_pi */
#define OR_ONE_OVER_2PI 0.159154943091895335768883763372514362f /* glm::one_over_two_pi */
#define OR_TWO_PI      6.28318530717958647692528676655900576f   /* glm::two_pi */
#define OR_ROOT_PI     1.772453850905516027f                     /* glm::root_pi */

enum { MT_NORMAL = 0, MT_LAMBERT = 1, MT_PHONG = 2, MT_MIRROR = 3, MT_DIELECTRIC = 4,
       MT_DIELECTRIC_TRANSPARENT = 5, MT_UNSUPPORTED = 6 };           /* pg/enums.h:3-11 */
enum { MIS_CONSTANT = 0, MIS_DEBIAS_CONTRIB = 1, MIS_DEBIAS_Z = 2, MIS_BALANCE = 3,
       MIS_PAIRWISE = 4 };                                             /* pg/ReSTIRIntegrator.h:19-25 */
enum { PASS_INITIAL = 1, PASS_TEMPORAL = 2, PASS_SPATIAL0 = 3 };

/* ------------------------------------------------------------------ glm-semantics math */
typedef struct { float x, y, z; } v3;
static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scl(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 neg(v3 a) { return V(-a.x, -a.y, -a.z); }
/* glm compute_dot<vec3>: tmp = a*b; tmp.x + tmp.y + tmp.z  (glm/detail/func_geometric.inl:48-55) */
static inline float dot(v3 a, v3 b) { v3 t = mul(a, b); return t.x + t.y + t.z; }
/* glm compute_cross (func_geometric.inl:68-79) */
static inline v3 cross(v3 x, v3 y) {
    return V(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
static inline float len(v3 a) { return sqrtf(dot(a, a)); }
/* glm normalize = v * inversesqrt(dot(v,v)), inversesqrt = 1/sqrt (func_exponential.inl:136-139) */
static inline v3 nrmz(v3 a) { return scl(a, 1.0f / sqrtf(dot(a, a))); }
/* glm reflect: I - N * dot(N, I) * 2 (func_geometric.inl:104-110) */
static inline v3 reflect(v3 I, v3 N) { return sub(I, scl(scl(N, dot(N, I)), 2.0f)); }
/* glm scalar max/min (func_common.inl:17-30): NaN propagation of the select form */
static inline float gmax(float x, float y) { return (x < y) ? y : x; }
static inline float gmin(float x, float y) { return (y < x) ? y : x; }
static inline float maxc(v3 a) { return gmax(gmax(a.x, a.y), a.z); }   /* pg/utils.h:61-63 */
static inline int nonzero_pos(v3 e) { return e.x > 0 || e.y > 0 || e.z > 0; }

/* column-major 4x4, m[c][r] like glm */
typedef struct { float m[4][4]; } m4;

/* glm::lookAtRH (glm/ext/matrix_transform.inl:99-119) */
static m4 look_at_rh(v3 eye, v3 center, v3 up) {
    v3 f = nrmz(sub(center, eye));
    v3 s = nrmz(cross(f, up));
    v3 u = cross(s, f);
    m4 R; memset(&R, 0, sizeof R);
    R.m[0][0] = 1; R.m[1][1] = 1; R.m[2][2] = 1; R.m[3][3] = 1;
    R.m[0][0] = s.x; R.m[1][0] = s.y; R.m[2][0] = s.z;
    R.m[0][1] = u.x; R.m[1][1] = u.y; R.m[2][1] = u.z;
    R.m[0][2] = -f.x; R.m[1][2] = -f.y; R.m[2][2] = -f.z;
    R.m[3][0] = -dot(s, eye); R.m[3][1] = -dot(u, eye); R.m[3][2] = dot(f, eye);
    return R;
}

/* glm compute_inverse<4,4> (glm/detail/func_matrix.inl:294-351) */
static m4 inverse4(const m4* M) {
    const float (*m)[4] = M->m;
    float c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    float F0[4] = {c00, c00, c02, c03}, F1[4] = {c04, c04, c06, c07}, F2[4] = {c08, c08, c10, c11};
    float F3[4] = {c12, c12, c14, c15}, F4[4] = {c16, c16, c18, c19}, F5[4] = {c20, c20, c22, c23};
    float V0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]};
    float V1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
    float V2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]};
    float V3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    m4 I;
    for (int i = 0; i < 4; ++i) {
        float i0 = V1[i] * F0[i] - V2[i] * F1[i] + V3[i] * F2[i];
        float i1 = V0[i] * F0[i] - V2[i] * F3[i] + V3[i] * F4[i];
        float i2 = V0[i] * F1[i] - V1[i] * F3[i] + V3[i] * F5[i];
        float i3 = V0[i] * F2[i] - V1[i] * F4[i] + V2[i] * F5[i];
        I.m[0][i] = i0 * SA[i]; I.m[1][i] = i1 * SB[i]; I.m[2][i] = i2 * SA[i]; I.m[3][i] = i3 * SB[i];
    }
    float d0 = m[0][0] * I.m[0][0], d1 = m[0][1] * I.m[1][0], d2 = m[0][2] * I.m[2][0], d3 = m[0][3] * I.m[3][0];
    float det = (d0 + d1) + (d2 + d3);
    float ood = 1.0f / det;
    for (int c = 0; c < 4; ++c) for (int r = 0; r < 4; ++r) I.m[c][r] = I.m[c][r] * ood;
    return I;
}

/* glm mat4 * vec4 (glm/detail/type_mat4x4.inl:561-572): (m0*x + m1*y) + (m2*z + m3*w) */
static v3 m4_mul_point(const m4* M, v3 p) {
    const float (*m)[4] = M->m;
    float r[3];
    for (int i = 0; i < 3; ++i) {
        float a0 = m[0][i] * p.x + m[1][i] * p.y;
        float a1 = m[2][i] * p.z + m[3][i] * 1.0f;
        r[i] = a0 + a1;
    }
    return V(r[0], r[1], r[2]);
}
/* glm mat3 * vec3 (type_mat3x3.inl:468-474) with mat3(invViewMat) */
static v3 m3_mul(const m4* M, v3 v) {
    const float (*m)[4] = M->m;
    return V(m[0][0] * v.x + m[1][0] * v.y + m[2][0] * v.z,
             m[0][1] * v.x + m[1][1] * v.y + m[2][1] * v.z,
             m[0][2] * v.x + m[1][2] * v.y + m[2][2] * v.z);
}

/* ------------------------------------------------------------------ counter RNG */
/* Replaces Utils::getRandomValue's shared mt19937 (pg/utils.cpp:175-176,199-202). */
static inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
typedef struct { uint32_t key, n; } rng_t;
static inline rng_t rng_init(uint32_t seed, uint32_t frame, uint32_t pass, uint32_t pixel) {
    uint32_t k = hash32(seed ^ 0x6a09e667u);
    k = hash32(k ^ frame);
    k = hash32(k + 0x9e3779b9u * (pass + 1u));
    k = hash32(k ^ pixel);
    rng_t r = {k, 0u};
    return r;
}
static inline float rng_u(rng_t* r) {
    uint32_t x = hash32(r->key ^ hash32(r->n + 0x632be5abu));
    r->n++;
    return (float)(x >> 8) * (1.0f / 16777216.0f);
}
/* Utils::getRandomValue(a, b) = a + (b - a) * U  (pg/utils.cpp:199-202) */
static inline float rnd(rng_t* r, float a, float b) { float u = rng_u(r); return a + (b - a) * u; }
/* Initial-pass draw slots: candidate c (area candidates 0..A-1, then BRDF candidates) owns draws
 * 4c..4c+3 -- up to 3 for its sample, 4c+3 for its reservoir update -- so candidates are independent
 * of one another's outcome (the reference's shared mt19937 stream has no observable order). */
static inline uint32_t cand_slot(int c) { return 4u * (uint32_t)c; }

/* ------------------------------------------------------------------ incomplete beta */
/* Non-normalised incomplete beta B_x(a,b) in double: restates boost::math::beta(a,b,x)
 * (libs/Boost/boost/math/special_functions/beta.hpp:1607-1622, ibeta_imp normalised=false)
 * with the Lentz continued fraction; pinned by tests/golden/ibeta_kat.json. */
static double betacf(double a, double b, double x) {
    const double FPMIN = 1e-300, EPS = 1e-16;
    double qab = a + b, qap = a + 1.0, qam = a - 1.0;
    double c = 1.0, d = 1.0 - qab * x / qap;
    if (fabs(d) < FPMIN) d = FPMIN;
    d = 1.0 / d;
    double h = d;
    for (int m = 1; m <= 10000; ++m) {
        int m2 = 2 * m;
        double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
        d = 1.0 + aa * d; if (fabs(d) < FPMIN) d = FPMIN;
        c = 1.0 + aa / c; if (fabs(c) < FPMIN) c = FPMIN;
        d = 1.0 / d; h *= d * c;
        aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
        d = 1.0 + aa * d; if (fabs(d) < FPMIN) d = FPMIN;
        c = 1.0 + aa / c; if (fabs(c) < FPMIN) c = FPMIN;
        d = 1.0 / d;
        double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < EPS) break;
    }
    return h;
}
double or_ibeta(double x, double a, double b) {
    if (!(x > 0.0)) return 0.0;
    double lbeta = rs_lgamma_d(a) + rs_lgamma_d(b) - rs_lgamma_d(a + b);
    if (x >= 1.0) return rs_exp_d(lbeta);
    double lbt = a * rs_log_d(x) + b * rs_log1p_d(-x);
    if (x < (a + 1.0) / (a + b + 2.0))
        return rs_exp_d(lbt) * betacf(a, b, x) / a;
    return rs_exp_d(lbeta) - rs_exp_d(lbt) * betacf(b, a, 1.0 - x) / b;
}
/* rs_libm.h's functions over arrays (tests/test_oracle.py test_libm_correctly_rounded) */
void or_libm_f1(int which, const float* x, float* o, int n) {
    for (int i = 0; i < n; ++i)
        o[i] = which == 0 ? rs_expf(x[i]) : which == 1 ? rs_lgammaf(x[i]) : which == 2 ? rs_sinf(x[i]) : rs_cosf(x[i]);
}
void or_libm_powf(const float* x, const float* y, float* o, int n) {
    for (int i = 0; i < n; ++i) o[i] = rs_powf(x[i], y[i]);
}
void or_libm_d1(int which, const double* x, double* o, int n) {
    for (int i = 0; i < n; ++i)
        o[i] = which == 0 ? rs_log_d(x[i]) : which == 1 ? rs_exp_d(x[i]) : which == 2 ? rs_log1p_d(x[i]) : rs_lgamma_d(x[i]);
}
/* MaterialPhong::ibeta (pg/MaterialPhong.cpp:246-248): float in, Boost promotes to double, float out */
static inline float ibeta_f(float x, float a, float b) { return (float)or_ibeta((double)x, (double)a, (double)b); }
/* MaterialPhong::gamma_quot (pg/MaterialPhong.cpp:224-226) */
static inline float gamma_quot(float a, float b) { return rs_expf(rs_lgammaf(a) - rs_lgammaf(b)); }
/* MaterialPhong::calc_I_M (pg/MaterialPhong.cpp:228-244) */
float or_calc_I_M(float nDotV, float n) {
    float costerm = nDotV;
    float sinterm_sq = 1.0f - costerm * costerm;
    float halfn = 0.5f * n;
    float negterm = costerm;
    sinterm_sq = gmin(gmax(sinterm_sq, 0.0f), 1.0f);
    if (n >= 1e-18f) negterm *= halfn * ibeta_f(sinterm_sq, halfn, 0.5f);
    return (OR_TWO_PI * costerm + OR_ROOT_PI * gamma_quot(halfn + 0.5f, halfn + 1.0f) *
            (rs_powf(sinterm_sq, halfn) - negterm)) / (n + 2.0f);
}

/* ------------------------------------------------------------------ scene */
typedef struct {
    v3 kd, ks, le; float shin; int type;
} or_mat;

typedef struct { float lo[3], hi[3]; int left, right, first, count; } or_node; /* count>0 => leaf */

typedef struct {
    uint32_t n_tris;
    v3 *p0, *p1, *p2, *n0, *n1, *n2;
    uint32_t* mat;
    int32_t* emis_id;          /* per triangle, -1 if not emissive (pg/ModelLoader.cpp:291-292) */
    uint32_t n_mat; or_mat* mats;
    /* emissive list + TriangleCDF (pg/TriangleCDF.cpp:8-34) */
    uint32_t n_emis; uint32_t* emis_tri;
    float* cdf;                /* cumulative normalised area, cdf2 */
    float* pick_pdf;           /* getTriangle's prob (pg/TriangleCDF.cpp:49-53) */
    float* area;               /* Triangle::area (pg/triangle.cpp:13-16) */
    float total_area;
    /* BVH */
    or_node* nodes; int n_nodes; uint32_t* tri_index;
    struct or_wnode* wn; int n_wn;
    float box_eps;                   /* the closest-hit walks' box margin (or_box_epsilon) */   /* 8-wide tree over the same leaves (or_scene_set_wide), or NULL */
    /* textures: per-material map slots (0-based, -1 none: diffuse, specular,
       shininess, normal), per-triangle uv (6) / tangents (9), textures in FreeImage layout, sky */
    int32_t* maps; float* uv; float* tan;
    struct or_tex* tex; int n_tex; int sky;
} or_scene;

/* Texture after FreeImage_ConvertToRawBits (pg/Texture.cpp:46-50): rows top first, pitch padded to
   4 bytes, 8-bit texels B,G,R(,A), float texels R,G,B(,A); `bytes` has 16 zero guard bytes at the end */
typedef struct or_tex { int w, h, pitch, px; uint8_t* bytes; } or_tex;
typedef struct { uint32_t width, height, channels; int32_t format; const void* data; int32_t srgb_expand; } or_texdesc;

/* Triangle::Triangle area = 0.5 * |cross(v1-v0, v2-v0)|  (pg/triangle.cpp:13-16) */
static float tri_area(v3 a, v3 b, v3 c) { return 0.5f * len(cross(sub(b, a), sub(c, a))); }

/* ---- binned SAH BVH (oracle's own; any correct BVH finds the same hits) */
typedef struct { float lo[3], hi[3]; } aabb;
static void bb_empty(aabb* b) { for (int i = 0; i < 3; ++i) { b->lo[i] = FLT_MAX; b->hi[i] = -FLT_MAX; } }
static void bb_grow_p(aabb* b, v3 p) {
    float q[3] = {p.x, p.y, p.z};
    for (int i = 0; i < 3; ++i) { if (q[i] < b->lo[i]) b->lo[i] = q[i]; if (q[i] > b->hi[i]) b->hi[i] = q[i]; }
}
static void bb_grow(aabb* b, const aabb* o) {
    for (int i = 0; i < 3; ++i) { if (o->lo[i] < b->lo[i]) b->lo[i] = o->lo[i]; if (o->hi[i] > b->hi[i]) b->hi[i] = o->hi[i]; }
}
static float bb_area(const aabb* b) {
    float d0 = b->hi[0] - b->lo[0], d1 = b->hi[1] - b->lo[1], d2 = b->hi[2] - b->lo[2];
    if (d0 < 0) return 0;
    return 2.0f * (d0 * d1 + d1 * d2 + d2 * d0);
}

typedef struct { aabb* tb; float* cen; uint32_t* idx; or_node* nodes; int n_nodes; } bvh_build_t;

/* the closest-hit walks' box margin: 2^-16 x the scene's largest |coordinate| (at least 1), restating rs_wide.h
 * box_epsilon.  Moller-Trumbore accepts hits whose point o + t d lies a few ulps outside the triangle's box; without
 * a margin a closest-hit walk can cull that box after finding a tied neighbour, and which box that is depends on the
 * tree (this oracle's binary and 8-wide trees disagreed on 1 of 8.3 M C3 4K primary rays).  With it every tree
 * returns the triangle test's answer.  The any-hit walks keep the exact boxes (as the kernels do). */
static float or_box_epsilon(const float* pos, size_t nfloats) {
    float m = 1.0f;
    for (size_t i = 0; i < nfloats; ++i) {
        const float a = fabsf(pos[i]);
        if (a - a == 0.0f && a > m) m = a;
    }
    return m * (1.0f / 65536.0f);
}

static int bvh_build_rec(bvh_build_t* B, int first, int count) {
    int ni = B->n_nodes++;
    or_node* N = &B->nodes[ni];
    aabb bb, cb; bb_empty(&bb); bb_empty(&cb);
    for (int i = first; i < first + count; ++i) {
        uint32_t t = B->idx[i];
        bb_grow(&bb, &B->tb[t]);
        bb_grow_p(&cb, V(B->cen[3 * t], B->cen[3 * t + 1], B->cen[3 * t + 2]));
    }
    memcpy(N->lo, bb.lo, sizeof bb.lo); memcpy(N->hi, bb.hi, sizeof bb.hi);
    if (count <= 4) { N->first = first; N->count = count; N->left = N->right = -1; return ni; }
    enum { NB = 16 };
    int best_axis = -1, best_split = -1; float best_cost = FLT_MAX;
    for (int ax = 0; ax < 3; ++ax) {
        float lo = cb.lo[ax], hi = cb.hi[ax];
        if (!(hi > lo)) continue;
        aabb bins[NB]; int cnt[NB];
        for (int b = 0; b < NB; ++b) { bb_empty(&bins[b]); cnt[b] = 0; }
        float k = (float)NB / (hi - lo);
        for (int i = first; i < first + count; ++i) {
            uint32_t t = B->idx[i];
            int b = (int)((B->cen[3 * t + ax] - lo) * k); if (b >= NB) b = NB - 1; if (b < 0) b = 0;
            cnt[b]++; bb_grow(&bins[b], &B->tb[t]);
        }
        float la[NB], ra[NB]; int lc[NB], rc[NB];
        aabb acc; bb_empty(&acc); int c = 0;
        for (int b = 0; b < NB; ++b) { bb_grow(&acc, &bins[b]); c += cnt[b]; la[b] = bb_area(&acc); lc[b] = c; }
        bb_empty(&acc); c = 0;
        for (int b = NB - 1; b >= 0; --b) { bb_grow(&acc, &bins[b]); c += cnt[b]; ra[b] = bb_area(&acc); rc[b] = c; }
        for (int b = 0; b < NB - 1; ++b) {
            if (lc[b] == 0 || rc[b + 1] == 0) continue;
            float cost = la[b] * lc[b] + ra[b + 1] * rc[b + 1];
            if (cost < best_cost) { best_cost = cost; best_axis = ax; best_split = b; }
        }
    }
    int mid;
    if (best_axis < 0) {
        mid = first + count / 2;  /* all centroids equal: median split by index */
    } else {
        float lo = cb.lo[best_axis], hi = cb.hi[best_axis];
        float k = (float)NB / (hi - lo);
        int i = first, j = first + count - 1;
        while (i <= j) {
            uint32_t t = B->idx[i];
            int b = (int)((B->cen[3 * t + best_axis] - lo) * k); if (b >= NB) b = NB - 1; if (b < 0) b = 0;
            if (b <= best_split) ++i; else { uint32_t s = B->idx[i]; B->idx[i] = B->idx[j]; B->idx[j] = s; --j; }
        }
        mid = i;
        if (mid == first || mid == first + count) mid = first + count / 2;
    }
    int l = bvh_build_rec(B, first, mid - first);
    int r = bvh_build_rec(B, mid, first + count - mid);
    N = &B->nodes[ni];
    N->left = l; N->right = r; N->count = 0; N->first = 0;
    return ni;
}

void or_scene_destroy(or_scene* s);

/* Scene ctor (pg/Scene.cpp:8-16) + ModelLoader geometry setup (pg/ModelLoader.cpp:218-321) +
 * TriangleCDF ctor (pg/TriangleCDF.cpp:8-34).  mat_f: per material kd3 ks3 le3 shininess. */
or_scene* or_scene_create(uint32_t n_tris, const float* pos, const float* nrm, const uint32_t* tri_mat,
                          uint32_t n_mat, const float* mat_f, const int32_t* mat_type) {
    or_scene* s = (or_scene*)calloc(1, sizeof(or_scene));
    s->n_tris = n_tris; s->n_mat = n_mat; s->sky = -1;
    s->p0 = malloc(n_tris * sizeof(v3)); s->p1 = malloc(n_tris * sizeof(v3)); s->p2 = malloc(n_tris * sizeof(v3));
    s->n0 = malloc(n_tris * sizeof(v3)); s->n1 = malloc(n_tris * sizeof(v3)); s->n2 = malloc(n_tris * sizeof(v3));
    s->mat = malloc(n_tris * sizeof(uint32_t)); s->emis_id = malloc(n_tris * sizeof(int32_t));
    s->mats = malloc((n_mat ? n_mat : 1) * sizeof(or_mat));
    for (uint32_t m = 0; m < n_mat; ++m) {
        const float* f = mat_f + 10 * m;
        s->mats[m].kd = V(f[0], f[1], f[2]); s->mats[m].ks = V(f[3], f[4], f[5]);
        s->mats[m].le = V(f[6], f[7], f[8]); s->mats[m].shin = f[9]; s->mats[m].type = mat_type[m];
    }
    uint32_t ne = 0;
    for (uint32_t t = 0; t < n_tris; ++t) {
        const float* p = pos + 9 * t; const float* n = nrm + 9 * t;
        s->p0[t] = V(p[0], p[1], p[2]); s->p1[t] = V(p[3], p[4], p[5]); s->p2[t] = V(p[6], p[7], p[8]);
        s->n0[t] = V(n[0], n[1], n[2]); s->n1[t] = V(n[3], n[4], n[5]); s->n2[t] = V(n[6], n[7], n[8]);
        s->mat[t] = tri_mat[t];
        v3 le = s->mats[tri_mat[t]].le;
        /* Material::isEmissive: emission.x + emission.y + emission.z > 0 (pg/material.h:135-137) */
        if (le.x + le.y + le.z > 0) s->emis_id[t] = (int32_t)ne++; else s->emis_id[t] = -1;
    }
    s->n_emis = ne;
    s->emis_tri = malloc((ne ? ne : 1) * sizeof(uint32_t));
    s->cdf = malloc((ne ? ne : 1) * sizeof(float));
    s->pick_pdf = malloc((ne ? ne : 1) * sizeof(float));
    s->area = malloc((ne ? ne : 1) * sizeof(float));
    for (uint32_t t = 0; t < n_tris; ++t) if (s->emis_id[t] >= 0) s->emis_tri[s->emis_id[t]] = t;
    float total = 0.0f;
    for (uint32_t e = 0; e < ne; ++e) {
        uint32_t t = s->emis_tri[e];
        s->area[e] = tri_area(s->p0[t], s->p1[t], s->p2[t]);
        total += s->area[e];
    }
    s->total_area = total;
    for (uint32_t e = 0; e < ne; ++e) {
        float norm_area = s->area[e] / total;
        float pred = e == 0 ? 0.0f : s->cdf[e - 1];
        s->cdf[e] = pred + norm_area;
    }
    /* std::sort by cumulative value (pg/TriangleCDF.cpp:27-29): the sequence is already
       non-decreasing; ties only for zero-area triangles (not produced by our scenes). */
    for (uint32_t e = 0; e < ne; ++e) s->pick_pdf[e] = e == 0 ? s->cdf[0] : s->cdf[e] - s->cdf[e - 1];

    /* BVH */
    bvh_build_t B;
    B.tb = malloc((n_tris ? n_tris : 1) * sizeof(aabb));
    B.cen = malloc((n_tris ? n_tris : 1) * 3 * sizeof(float));
    B.idx = malloc((n_tris ? n_tris : 1) * sizeof(uint32_t));
    B.nodes = malloc((2 * (n_tris ? n_tris : 1)) * sizeof(or_node));
    B.n_nodes = 0;
    for (uint32_t t = 0; t < n_tris; ++t) {
        bb_empty(&B.tb[t]); bb_grow_p(&B.tb[t], s->p0[t]); bb_grow_p(&B.tb[t], s->p1[t]); bb_grow_p(&B.tb[t], s->p2[t]);
        for (int a = 0; a < 3; ++a) B.cen[3 * t + a] = 0.5f * (B.tb[t].lo[a] + B.tb[t].hi[a]);
        B.idx[t] = t;
    }
    s->box_eps = or_box_epsilon(pos, 9 * (size_t)n_tris);
    if (n_tris) bvh_build_rec(&B, 0, (int)n_tris);
    s->nodes = B.nodes; s->n_nodes = B.n_nodes; s->tri_index = B.idx;
    free(B.tb); free(B.cen);
    return s;
}

void or_scene_destroy(or_scene* s) {
    if (!s) return;
    free(s->wn);
    free(s->p0); free(s->p1); free(s->p2); free(s->n0); free(s->n1); free(s->n2);
    free(s->mat); free(s->emis_id); free(s->mats); free(s->emis_tri); free(s->cdf);
    free(s->pick_pdf); free(s->area); free(s->nodes); free(s->tri_index);
    for (int i = 0; i < s->n_tex; ++i) free(s->tex[i].bytes);
    free(s->tex); free(s->maps); free(s->uv); free(s->tan); free(s);
}

/* ------------------------------------------------------------------ textures */
/* Utils::expand (pg/utils.cpp:209-218) */
static float srgb_expand1(float u) {
    if (u <= 0.0f) return 0.0f;
    if (u >= 1.0f) return 1.0f;
    if (u <= 0.04045f) return u / 12.92f;
    return rs_powf((u + 0.055f) / 1.055f, 2.4f);
}
/* Texture ctor (pg/Texture.cpp:9-57) + Texture::expand applied n_expand times (:141-160) */
static int tex_load(or_tex* t, const or_texdesc* d, int n_expand) {
    if (!d->data || d->width < 1 || d->height < 1) return -1;
    if (d->format == 0) { if (d->channels != 1 && d->channels != 3 && d->channels != 4) return -1; t->px = (int)d->channels; }
    else if (d->format == 1) { if (d->channels != 3 && d->channels != 4) return -1; t->px = 4 * (int)d->channels; }
    else return -1;
    t->w = (int)d->width; t->h = (int)d->height;
    t->pitch = (t->w * t->px + 3) & ~3;
    t->bytes = calloc((size_t)t->pitch * t->h + 16, 1);
    size_t rowlen = (size_t)t->w * d->channels;
    for (int y = 0; y < t->h; ++y) {
        uint8_t* dst = t->bytes + (size_t)y * t->pitch;
        if (d->format == 1) { memcpy(dst, (const float*)d->data + (size_t)y * rowlen, rowlen * sizeof(float)); continue; }
        const uint8_t* src = (const uint8_t*)d->data + (size_t)y * rowlen;
        for (int x = 0; x < t->w; ++x) {
            const uint8_t* q = src + (size_t)x * d->channels;
            uint8_t* o = dst + (size_t)x * t->px;
            if (d->channels == 1) { o[0] = q[0]; continue; }
            o[0] = q[2]; o[1] = q[1]; o[2] = q[0];
            if (d->channels == 4) o[3] = q[3];
        }
        for (int k = 0; k < n_expand; ++k)
            for (int x = 0; x < t->w * t->px; ++x) {
                float f = (float)dst[x] / 255.0f;
                f = srgb_expand1(f);
                dst[x] = (uint8_t)(f * 255.0f);
            }
    }
    return 0;
}
/* mat_maps: n_mat x 4 one-based texture indices (0 none); uv: T x 6 or NULL; tan: T x 9 or NULL.
   A colour texture is expanded once per diffuse/specular slot referencing it (ModelLoader expands the
   TextureProxy-shared texture for every such slot, pg/ModelLoader.cpp:124-137). */
int or_scene_set_textures(or_scene* s, const int32_t* mat_maps, const float* uv, const float* tan, uint32_t n_tex,
                          const or_texdesc* descs) {
    int* count = calloc(n_tex ? n_tex : 1, sizeof(int));
    s->maps = malloc((s->n_mat ? s->n_mat : 1) * 4 * sizeof(int32_t));
    for (uint32_t m = 0; m < s->n_mat; ++m)
        for (int k = 0; k < 4; ++k) {
            int32_t v = mat_maps[4 * m + k];
            if (v < 0 || (uint32_t)v > n_tex) { free(count); return -1; }
            s->maps[4 * m + k] = v - 1;
            if (k < 2 && v > 0 && descs[v - 1].srgb_expand) count[v - 1]++;
        }
    s->tex = calloc(n_tex + 1, sizeof(or_tex));
    for (uint32_t i = 0; i < n_tex; ++i)
        if (tex_load(&s->tex[i], &descs[i], count[i])) { free(count); return -1; }
    s->n_tex = (int)n_tex;
    free(count);
    s->uv = calloc((size_t)(s->n_tris ? s->n_tris : 1) * 6, sizeof(float));
    s->tan = calloc((size_t)(s->n_tris ? s->n_tris : 1) * 9, sizeof(float));
    if (uv) memcpy(s->uv, uv, (size_t)s->n_tris * 6 * sizeof(float));
    if (tan) memcpy(s->tan, tan, (size_t)s->n_tris * 9 * sizeof(float));
    return 0;
}
/* Scene::loadSkybox (pg/Scene.cpp:46-50): the sky texture is stored after the material maps */
int or_scene_set_sky(or_scene* s, const or_texdesc* d) {
    if (s->sky >= 0) { free(s->tex[s->sky].bytes); s->n_tex--; s->sky = -1; }
    if (!d) return 0;
    s->tex = realloc(s->tex, (size_t)(s->n_tex + 1) * sizeof(or_tex));
    if (tex_load(&s->tex[s->n_tex], d, 0)) return -1;
    s->sky = s->n_tex++;
    return 0;
}
/* Texture::get_texel(int x, int y) (pg/Texture.cpp:72-107) */
static v3 tex_texel(const or_tex* t, int x, int y, int repeat) {
    int cx, cy;
    if (repeat) { cx = abs(x % t->w); cy = abs(y % t->h); }
    else { cx = x < 0 ? 0 : (x > t->w - 1 ? t->w - 1 : x); cy = y < 0 ? 0 : (y > t->h - 1 ? t->h - 1 : y); }
    const uint8_t* p = t->bytes + (size_t)cy * t->pitch + (size_t)cx * t->px;
    if (t->px > 4) { float f[3]; memcpy(f, p, sizeof f); return V(f[0], f[1], f[2]); }
    return V((float)p[2] / 255.0f, (float)p[1] / 255.0f, (float)p[0] / 255.0f);
}
/* Texture::getTexelBilinear (pg/Texture.cpp:170-194); glm::mix(x, y, a) = x*(1-a) + y*a */
static v3 tex_bilinear(const or_tex* t, float u, float v, int repeat) {
    float pxc = u * (float)t->w, pyc = (1.0f - v) * (float)t->h;
    float fx = floorf(pxc), fy = floorf(pyc);
    float tx = pxc - fx, ty = pyc - fy;
    v3 q00 = tex_texel(t, (int)fx, (int)fy, repeat), q10 = tex_texel(t, (int)(fx + 1.0f), (int)fy, repeat);
    v3 q01 = tex_texel(t, (int)fx, (int)(fy + 1.0f), repeat), q11 = tex_texel(t, (int)(fx + 1.0f), (int)(fy + 1.0f), repeat);
    v3 x1 = add(scl(q00, 1.0f - tx), scl(q10, tx));
    v3 x2 = add(scl(q01, 1.0f - tx), scl(q11, tx));
    return add(scl(x1, 1.0f - ty), scl(x2, ty));
}
/* SphericalMap::getTexel (pg/SphericalMap.cpp:10-14), INVPI = 1.0 / M_PI (double); sky texture is
   BILINEAR + CLAMP_TO_EDGE (pg/Texture.h:27) */
static v3 sky_texel(const or_scene* s, v3 dir) {
    const double invpi = 1.0 / 3.14159265358979323846;
    const float x = (float)(0.5f + (double)(0.5f * atan2f(dir.y, dir.x)) * invpi);
    const float y = (float)(1.0f - (double)acosf(dir.z) * invpi);
    return tex_bilinear(&s->tex[s->sky], x, y, 0);
}
/* Material::getDiffuseColor / getSpecularColor / getShininess (pg/material.cpp:105-134) at the
   interpolated uv and the normal map (pg/Intersection.h:26-39); normal_only: BRDF-sampled emitter hits */
static void apply_maps(const or_scene* s, uint32_t prim, float u, float v, uint32_t m, v3* kd, v3* ks, float* shin,
                       v3* n, int normal_only) {
    if (!s->maps) return;
    const int32_t* mp = s->maps + 4 * m;
    if (mp[0] < 0 && mp[1] < 0 && mp[2] < 0 && mp[3] < 0) return;
    const float* q = s->uv + 6 * (size_t)prim;
    float w = 1.0f - u - v;
    float tu = (q[0] * w + q[2] * u) + q[4] * v, tv = (q[1] * w + q[3] * u) + q[5] * v;
    if (!normal_only) {
        if (mp[0] >= 0) *kd = tex_bilinear(&s->tex[mp[0]], tu, tv, 1);
        if (mp[1] >= 0) *ks = tex_bilinear(&s->tex[mp[1]], tu, tv, 1);
        if (mp[2] >= 0) { v3 r = tex_bilinear(&s->tex[mp[2]], tu, tv, 1); *shin = 2.0f / (r.x * r.x) - 2.0f; }
    }
    if (mp[3] >= 0) {
        const float* g = s->tan + 9 * (size_t)prim;
        v3 T = add(add(scl(V(g[0], g[1], g[2]), w), scl(V(g[3], g[4], g[5]), u)), scl(V(g[6], g[7], g[8]), v));
        T = sub(T, scl(*n, dot(T, *n)));
        T = nrmz(T);
        v3 B = nrmz(cross(*n, T));
        v3 N = sub(scl(tex_bilinear(&s->tex[mp[3]], tu, tv, 1), 2.0f), V(1.0f, 1.0f, 1.0f));
        v3 nn = *n;
        *n = V(T.x * N.x + B.x * N.y + nn.x * N.z, T.y * N.x + B.y * N.y + nn.y * N.z, T.z * N.x + B.z * N.y + nn.z * N.z);
    }
}

/* ------------------------------------------------------------------ ray queries */
/* Moller-Trumbore with fixed operation order; the HIP product uses the same arithmetic.
 * Replaces Embree's rtcIntersect1/rtcOccluded1 triangle test (pg/Intersection.h:43-83). */
static inline int tri_hit(const or_scene* s, uint32_t t, v3 o, v3 d, float tnear, float tfar,
                          float* tt, float* uu, float* vv) {
    v3 v0 = s->p0[t];
    v3 e1 = sub(s->p1[t], v0), e2 = sub(s->p2[t], v0);
    v3 p = cross(d, e2);
    float det = dot(e1, p);
    if (det == 0.0f) return 0;
    float inv = 1.0f / det;
    v3 sv = sub(o, v0);
    float u = dot(sv, p) * inv;
    if (!(u >= 0.0f && u <= 1.0f)) return 0;
    v3 q = cross(sv, e1);
    float v = dot(d, q) * inv;
    if (!(v >= 0.0f && u + v <= 1.0f)) return 0;
    float t_ = dot(e2, q) * inv;
    if (!(t_ >= tnear && t_ <= tfar)) return 0;
    *tt = t_; *uu = u; *vv = v;
    return 1;
}

/* conservative slab test: interval widened by (1 +- 4 eps) so it never culls a box whose
   contents the triangle test would accept */
/* closest-hit margin (or_box_epsilon): olo = o + e, ohi = o - e, the origins the lo / hi planes are taken from,
   i.e. the box widened by e on every side (NULL: no margin; rs_scene.h box_test_m) */
static inline int box_hit(const or_node* n, v3 o, v3 inv, float tnear, float tfar, float* tentry, const float* olo,
                          const float* ohi) {
    float oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z};
    float t0 = tnear, t1 = tfar;
    for (int a = 0; a < 3; ++a) {
        float ta = (n->lo[a] - (olo ? olo[a] : oo[a])) * ii[a];
        float tb = (n->hi[a] - (ohi ? ohi[a] : oo[a])) * ii[a];
        float mn = fminf(ta, tb), mx = fmaxf(ta, tb);
        t0 = fmaxf(t0, mn); t1 = fminf(t1, mx);
    }
    *tentry = t0;
    return t0 * (1.0f - 4.0f * FLT_EPSILON) <= t1 * (1.0f + 4.0f * FLT_EPSILON);
}

typedef struct { int hit; float t, u, v; uint32_t prim; } or_hit;

static or_hit closest_hit_wide(const or_scene* s, v3 o, v3 d, float tnear, float tfar);
static int any_hit_wide(const or_scene* s, v3 o, v3 d, float tnear, float tfar);
static or_hit closest_hit(const or_scene* s, v3 o, v3 d, float tnear, float tfar) {
    or_hit h = {0, tfar, 0, 0, 0xffffffffu};
    if (!s->n_nodes) return h;
    if (s->wn) return closest_hit_wide(s, o, d, tnear, tfar);
    v3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const float e = s->box_eps;
    const float olo[3] = {o.x + e, o.y + e, o.z + e}, ohi[3] = {o.x - e, o.y - e, o.z - e};
    int stack[128]; int sp = 0; stack[sp++] = 0;
    while (sp) {
        const or_node* n = &s->nodes[stack[--sp]];
        float te;
        if (!box_hit(n, o, inv, tnear, h.t, &te, olo, ohi)) continue;
        if (n->count) {
            for (int i = n->first; i < n->first + n->count; ++i) {
                uint32_t t = s->tri_index[i]; float tt, uu, vv;
                if (tri_hit(s, t, o, d, tnear, h.t, &tt, &uu, &vv)) {
                    if (!h.hit || tt < h.t || (tt == h.t && t < h.prim)) {
                        h.hit = 1; h.t = tt; h.u = uu; h.v = vv; h.prim = t;
                    }
                }
            }
        } else {
            stack[sp++] = n->right; stack[sp++] = n->left;
        }
    }
    return h;
}

static int any_hit(const or_scene* s, v3 o, v3 d, float tnear, float tfar) {
    if (!s->n_nodes) return 0;
    if (s->wn) return any_hit_wide(s, o, d, tnear, tfar);
    v3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    int stack[128]; int sp = 0; stack[sp++] = 0;
    while (sp) {
        const or_node* n = &s->nodes[stack[--sp]];
        float te;
        if (!box_hit(n, o, inv, tnear, tfar, &te, NULL, NULL)) continue;
        if (n->count) {
            for (int i = n->first; i < n->first + n->count; ++i) {
                float tt, uu, vv;
                if (tri_hit(s, s->tri_index[i], o, d, tnear, tfar, &tt, &uu, &vv)) return 1;
            }
        } else {
            stack[sp++] = n->right; stack[sp++] = n->left;
        }
    }
    return 0;
}

/* ---- 8-wide walks (the CPU baseline's SIMD traversal; not part of the restatement:
 * any tree finds the same hits).  The binary tree collapsed like the product's wide tree (csrc/rs_wide.h:
 * a wide node's up to 8 children come from opening the largest-area interior child), children kept as
 * the binary nodes' exact boxes in SoA and tested 8 at a time with box_hit's float operations (fminf /
 * fmaxf NaN rules included); leaf children are the binary leaves (<= 4 triangles each). */
typedef struct or_wnode { float lo[3][8], hi[3][8]; int32_t kid[8]; uint32_t valid; } or_wnode;  /* kid < 0: leaf ~node */
enum { OR_WSTACK = 512 };

int or_scene_set_wide(or_scene* s, int on) {
    free(s->wn); s->wn = NULL; s->n_wn = 0;
    if (!on || !s->n_nodes || !__builtin_cpu_supports("avx2")) return 0;
    or_wnode* W = calloc((size_t)s->n_nodes, sizeof(or_wnode));
    int* q = malloc((size_t)s->n_nodes * sizeof(int));
    int* lvl = malloc((size_t)s->n_nodes * sizeof(int));
    int nq = 1, depth = 0;
    q[0] = 0; lvl[0] = 0;
    for (int qi = 0; qi < nq; ++qi) {
        const or_node* b = &s->nodes[q[qi]];
        int kids[8], nk = 0;
        if (b->count) kids[nk++] = q[qi]; else { kids[nk++] = b->left; kids[nk++] = b->right; }
        while (nk < 8) {
            int best = -1; float ba = -1.0f;
            for (int i = 0; i < nk; ++i) {
                const or_node* k = &s->nodes[kids[i]];
                aabb bb; memcpy(bb.lo, k->lo, sizeof bb.lo); memcpy(bb.hi, k->hi, sizeof bb.hi);
                if (!k->count && bb_area(&bb) > ba) { ba = bb_area(&bb); best = i; }
            }
            if (best < 0) break;
            const or_node* x = &s->nodes[kids[best]];
            kids[best] = x->left; kids[nk++] = x->right;
        }
        or_wnode* w = &W[qi];
        for (int c = 0; c < 8; ++c)
            for (int a = 0; a < 3; ++a) { w->lo[a][c] = 0.0f; w->hi[a][c] = 0.0f; }
        for (int c = 0; c < nk; ++c) {
            const or_node* k = &s->nodes[kids[c]];
            for (int a = 0; a < 3; ++a) { w->lo[a][c] = k->lo[a]; w->hi[a][c] = k->hi[a]; }
            if (k->count) w->kid[c] = ~kids[c];
            else { w->kid[c] = nq; lvl[nq] = lvl[qi] + 1; if (lvl[nq] > depth) depth = lvl[nq]; q[nq++] = kids[c]; }
            w->valid |= 1u << c;
        }
    }
    free(q); free(lvl);
    if (7 * (depth + 1) + 1 > OR_WSTACK) { free(W); return 0; }   /* the walks' fixed stacks */
    s->wn = W; s->n_wn = nq;
    return 1;
}

/* box_hit for the 8 children: bit c = child c accepted; tentry[c] = its entry t */
/* OL / OH: the origins of the lo / hi planes (box_hit's olo / ohi; both O without the margin) */
__attribute__((target("avx2"))) static inline uint32_t box8(const or_wnode* w, const __m256* OL, const __m256* OH,
                                                              const __m256* I, float tnear, float tfar, float* tentry) {
    __m256 t0 = _mm256_set1_ps(tnear), t1 = _mm256_set1_ps(tfar);
    for (int a = 0; a < 3; ++a) {
        const __m256 ta = _mm256_mul_ps(_mm256_sub_ps(_mm256_loadu_ps(w->lo[a]), OL[a]), I[a]);
        const __m256 tb = _mm256_mul_ps(_mm256_sub_ps(_mm256_loadu_ps(w->hi[a]), OH[a]), I[a]);
        const __m256 nb = _mm256_cmp_ps(tb, tb, _CMP_UNORD_Q);
        /* fminf / fmaxf(ta, tb): the non-NaN operand if one is NaN (min_ps/max_ps return tb then) */
        __m256 mn = _mm256_blendv_ps(_mm256_min_ps(ta, tb), ta, nb);
        __m256 mx = _mm256_blendv_ps(_mm256_max_ps(ta, tb), ta, nb);
        t0 = _mm256_max_ps(mn, t0);   /* fmaxf(t0, mn): t0 when mn is NaN */
        t1 = _mm256_min_ps(mx, t1);
    }
    _mm256_storeu_ps(tentry, t0);
    const __m256 ok = _mm256_cmp_ps(_mm256_mul_ps(t0, _mm256_set1_ps(1.0f - 4.0f * FLT_EPSILON)),
                                    _mm256_mul_ps(t1, _mm256_set1_ps(1.0f + 4.0f * FLT_EPSILON)), _CMP_LE_OQ);
    return (uint32_t)_mm256_movemask_ps(ok) & w->valid;
}

__attribute__((target("avx2"))) static int any_hit_wide(const or_scene* s, v3 o, v3 d, float tnear, float tfar) {
    const v3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const __m256 O[3] = {_mm256_set1_ps(o.x), _mm256_set1_ps(o.y), _mm256_set1_ps(o.z)};
    const __m256 I[3] = {_mm256_set1_ps(inv.x), _mm256_set1_ps(inv.y), _mm256_set1_ps(inv.z)};
    int stack[OR_WSTACK]; int sp = 0; stack[sp++] = 0;
    float te[8];
    while (sp) {
        const or_wnode* w = &s->wn[stack[--sp]];
        uint32_t m = box8(w, O, O, I, tnear, tfar, te);
        while (m) {
            const int c = __builtin_ctz(m); m &= m - 1;
            const int32_t k = w->kid[c];
            if (k >= 0) { stack[sp++] = k; continue; }
            const or_node* n = &s->nodes[~k];
            for (int i = n->first; i < n->first + n->count; ++i) {
                float tt, uu, vv;
                if (tri_hit(s, s->tri_index[i], o, d, tnear, tfar, &tt, &uu, &vv)) return 1;
            }
        }
    }
    return 0;
}

/* closest hit: leaves tested when met, interior children pushed farthest first (nearest popped next, so
 * the running t culls more of the rest) */
__attribute__((target("avx2"))) static or_hit closest_hit_wide(const or_scene* s, v3 o, v3 d, float tnear, float tfar) {
    or_hit h = {0, tfar, 0, 0, 0xffffffffu};
    const v3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const __m256 I[3] = {_mm256_set1_ps(inv.x), _mm256_set1_ps(inv.y), _mm256_set1_ps(inv.z)};
    const float e = s->box_eps;
    const __m256 OL[3] = {_mm256_set1_ps(o.x + e), _mm256_set1_ps(o.y + e), _mm256_set1_ps(o.z + e)};
    const __m256 OH[3] = {_mm256_set1_ps(o.x - e), _mm256_set1_ps(o.y - e), _mm256_set1_ps(o.z - e)};
    int stack[OR_WSTACK]; int sp = 0; stack[sp++] = 0;
    float te[8];
    while (sp) {
        const or_wnode* w = &s->wn[stack[--sp]];
        uint32_t m = box8(w, OL, OH, I, tnear, h.t, te);
        int near[8]; int nn = 0;
        while (m) {
            const int c = __builtin_ctz(m); m &= m - 1;
            const int32_t k = w->kid[c];
            if (k >= 0) {   /* insertion by entry t, descending */
                int j = nn++;
                while (j > 0 && te[near[j - 1]] < te[c]) { near[j] = near[j - 1]; --j; }
                near[j] = c;
                continue;
            }
            const or_node* n = &s->nodes[~k];
            for (int i = n->first; i < n->first + n->count; ++i) {
                uint32_t t = s->tri_index[i]; float tt, uu, vv;
                if (tri_hit(s, t, o, d, tnear, h.t, &tt, &uu, &vv)) {
                    if (!h.hit || tt < h.t || (tt == h.t && t < h.prim)) {
                        h.hit = 1; h.t = tt; h.u = uu; h.v = vv; h.prim = t;
                    }
                }
            }
        }
        for (int j = 0; j < nn; ++j) stack[sp++] = w->kid[near[j]];
    }
    return h;
}

/* ------------------------------------------------------------------ params / buffers */
typedef struct {
    int32_t m_area, m_brdf, spatial_neighbors, spatial_passes, confidence_cap;
    float spatial_radius, min_normal_similarity, max_depth_difference;
    int32_t do_spatial, do_temporal, do_visibility_pass, reject_dissimilar, spatial_mis;
    int32_t use_skybox; float bg_color[3];
    float tnear_offset, tfar_offset, normal_offset;
    uint32_t seed; int32_t debug_reprojection;
} or_params;  /* snapshot of pg/ReSTIRIntegrator.cpp:13-35 statics + pg/RenderParams.h:5-17 */

typedef struct { v3 pos, nrm, kd, ks, le; float shin, depth; int type; } or_gbe; /* pg/GBufferElement.h:6-17 */
typedef struct { v3 pos; m4 view, inv_view; float focal; } or_gcam;            /* pg/GBufferElement.h:136-139 */
typedef struct { v3 p, n, li; float wsum, W; int conf; } or_res;               /* pg/Reservoir.h:6-59 */

typedef struct {
    int W, H;
    or_gbe* g[2]; or_gcam gc[2]; int gcur;
    or_res* r[3]; int r_last;
    uint64_t frames;          /* frameCtr (pg/simpleguidx11.h:101) */
    int cache_im;             /* 1: cache calc_I_M per pixel (speed only; identical values) */
    float* im_cache[2];       /* 1/calc_I_M per pixel for Phong-dispatched surfaces */
    void* tile;               /* or_tile_state, allocated on first use */
    uint64_t rebuilt;         /* tile mode: G elements the temporal pass rebuilt beyond the tile's rows */
    uint64_t ref_rays;        /* the last frame's reference-equivalent ray count (fold_ref) */
} or_ctx;

or_ctx* or_ctx_create(int W, int H) {
    or_ctx* c = (or_ctx*)calloc(1, sizeof(or_ctx));
    c->W = W; c->H = H;
    size_t n = (size_t)W * H;
    for (int i = 0; i < 2; ++i) { c->g[i] = calloc(n, sizeof(or_gbe)); c->im_cache[i] = calloc(n, sizeof(float)); }
    for (int i = 0; i < 3; ++i) c->r[i] = calloc(n, sizeof(or_res));
    c->r_last = 2;
    c->cache_im = 1;
    return c;
}
static void tile_release(or_ctx* c);
void or_ctx_destroy(or_ctx* c) {
    if (!c) return;
    tile_release(c);
    for (int i = 0; i < 2; ++i) { free(c->g[i]); free(c->im_cache[i]); }
    for (int i = 0; i < 3; ++i) free(c->r[i]);
    free(c);
}
void or_ctx_set_cache_im(or_ctx* c, int on) { c->cache_im = on; }
void or_ctx_reset_history(or_ctx* c) { c->frames = 0; }

static inline or_res res_empty(void) {
    or_res r;
    r.p = V(-FLT_MAX, -FLT_MAX, -FLT_MAX); r.n = r.p; r.li = r.p;
    r.wsum = 0; r.W = 0; r.conf = 0;
    return r;
}
/* LightSample::isValid (pg/Reservoir.h:11-17) */
static inline int sample_valid(const or_res* s) {
    int pok = s->p.x != -FLT_MAX && s->p.y != -FLT_MAX && s->p.z != -FLT_MAX;
    int nok = s->n.x != -FLT_MAX && s->n.y != -FLT_MAX && s->n.z != -FLT_MAX;
    int lok = s->li.x > 0 || s->li.y > 0 || s->li.z > 0;
    return pok && nok && lok;
}
typedef struct { v3 p, n, li; } sample_t;
static inline sample_t smp_of(const or_res* r) { sample_t s = {r->p, r->n, r->li}; return s; }
static inline sample_t smp_invalid(void) { sample_t s; s.p = V(-FLT_MAX, -FLT_MAX, -FLT_MAX); s.n = s.p; s.li = s.p; return s; }
static inline int smp_valid(sample_t s) {
    or_res r; r.p = s.p; r.n = s.n; r.li = s.li; return sample_valid(&r);
}
/* Reservoir::addSample (pg/Reservoir.h:33-47), in two halves so the golden-vector hook below can
 * replay a recorded U stream through the same code: res_update accumulates and says whether a U is
 * drawn (not when w == 0 && w_sum == 0), res_take decides with that U. */
static inline int res_update(or_res* r, float w, int conf) {
    r->wsum += w;
    r->conf += conf;
    return !(w == 0 && r->wsum == 0);
}
static inline int res_take(or_res* r, sample_t s, float w, float u) {
    if (u < w / r->wsum) { r->p = s.p; r->n = s.n; r->li = s.li; return 1; }
    return 0;
}
static inline int res_add(or_res* r, sample_t s, float w, int conf, rng_t* rng) {
    if (!res_update(r, w, conf)) return 0;
    return res_take(r, s, w, rng_u(rng));
}
/* Reservoir::capConfidence (pg/Reservoir.h:54-56) */
static inline void res_cap(or_res* r, int cap) { r->conf = r->conf < cap ? r->conf : cap; }

/* ------------------------------------------------------------------ reference-equivalent ray count
 * Rays the REFERENCE would trace for the same frame: every rtcIntersect1 (primary + BRDF rays) and every
 * testOcclusion its code reaches -- each visibility-tested evaluateF with a valid sample at a
 * non-emissive pixel (pg/ReSTIRIntegrator.cpp:185-206; also when L_i*f_r*G is zero, a ray this
 * restatement and the product skip), the final p-hats it re-evaluates (initial :289, temporal
 * :706/:721/:727, spatial :481) and every pixel of visibilityPass (:302-312).  Per thread (no atomics
 * in the timed CPU baseline), folded once per frame. */
static _Thread_local uint64_t tl_ref;
static uint64_t fold_ref(void) {
    uint64_t t = 0;
#pragma omp parallel reduction(+:t)
    { t += tl_ref; tl_ref = 0; }
    return t;
}

/* ------------------------------------------------------------------ per-frame context */
typedef struct {
    const or_scene* s; or_ctx* c; const or_params* P; uint32_t frame;
    const or_gbe* G; const or_gbe* Gp; const or_gcam* gc; const or_gcam* gcp;
    const float* im; const float* imp;
    int gy0, gy1;             /* G-buffer rows available (tile band + margin) */
} fctx;

/* diagnostic (scripts/anyhit_probe.py): record every occlusion ray whose origin is one of up to 16 given points --
 * origin, direction, tnear, tfar, result (9 floats) -- into a caller buffer */
static struct { int n_pts; float pts[16][3]; float* buf; int cap; int count; } g_rec;
void or_record_rays(int n_pts, const float* pts, float* buf, int cap) {
    g_rec.n_pts = n_pts < 16 ? n_pts : 16;
    for (int i = 0; i < g_rec.n_pts; ++i) for (int a = 0; a < 3; ++a) g_rec.pts[i][a] = pts[3 * i + a];
    g_rec.buf = buf; g_rec.cap = cap; g_rec.count = 0;
}
int or_recorded_rays(void) { return g_rec.count; }
static void record_ray(v3 o, v3 d, float tnear, float tfar, int res) {
    for (int i = 0; i < g_rec.n_pts; ++i)
        if (o.x == g_rec.pts[i][0] && o.y == g_rec.pts[i][1] && o.z == g_rec.pts[i][2]) {
            const int k = __atomic_fetch_add(&g_rec.count, 1, __ATOMIC_RELAXED);
            if (k < g_rec.cap) {
                float* r = g_rec.buf + 9 * (size_t)k;
                r[0] = o.x; r[1] = o.y; r[2] = o.z; r[3] = d.x; r[4] = d.y; r[5] = d.z; r[6] = tnear; r[7] = tfar;
                r[8] = (float)res;
            }
            return;
        }
}

/* Intersection::testOcclusion (pg/Intersection.h:43-60) */
static int occluded(const fctx* F, v3 from, v3 to, uint64_t* rays) {
    float dist = len(sub(to, from));
    v3 dir = nrmz(sub(to, from));
    float tnear = FLT_MIN + F->P->tnear_offset;
    float tfar = dist - F->P->tfar_offset;
    (*rays)++;
    const int res = any_hit(F->s, from, dir, tnear, tfar);
    if (g_rec.n_pts) record_ray(from, dir, tnear, tfar, res);
    return res;
}

/* Intersection::intersectEmbree + getGeometryAttributes (pg/Intersection.h:8-41,85-113) */
typedef struct { int hit; v3 point, normal; uint32_t prim; float t, u, v; } hitinfo;
static hitinfo intersect(const fctx* F, v3 o, v3 d, float tnear, uint64_t* rays) {
    hitinfo hi; hi.hit = 0; hi.prim = 0xffffffffu; hi.t = FLT_MAX; hi.point = V(0, 0, 0); hi.normal = V(0, 0, 0);
    hi.u = 0.0f; hi.v = 0.0f;
    (*rays)++;
    tl_ref++;
    or_hit h = closest_hit(F->s, o, d, tnear, FLT_MAX);
    if (!h.hit) return hi;
    const or_scene* s = F->s; uint32_t t = h.prim;
    /* rtcInterpolate0 slot 0: (1-u-v)*n0 + u*n1 + v*n2 */
    float w = 1.0f - h.u - h.v;
    v3 n = add(add(scl(s->n0[t], w), scl(s->n1[t], h.u)), scl(s->n2[t], h.v));
    n = nrmz(n);
    if (dot(neg(d), n) <= 0.0f) n = scl(n, -1.0f);
    hi.hit = 1; hi.normal = n; hi.prim = t; hi.t = h.t; hi.u = h.u; hi.v = h.v;
    hi.point = add(o, scl(d, h.t));
    return hi;
}

/* CosineWeightedDistribution::getPdf (pg/Distribution.h:33-35) */
static inline float cosine_pdf(v3 n, v3 wi) { return gmax(dot(n, wi), 0.0f) * OR_ONE_OVER_PI; }
/* CosineLobeDistribution::getPdf (pg/Distribution.h:65-67) */
static inline float lobe_pdf(v3 wi, v3 wr, float gamma) {
    return (gamma + 1.0f) * OR_ONE_OVER_2PI * rs_powf(gmax(0.0f, dot(wi, wr)), gamma);
}
/* pdf eval dispatch: always MaterialPhong::evalPdf (pg/ReSTIRIntegrator.h:54-59, pg/MaterialPhong.cpp:150-172) */
static float phong_eval_pdf(const or_gbe* g, v3 cam, v3 wi) {
    float maxD = maxc(g->kd), maxS = maxc(g->ks);
    float pf = maxD / (maxD + maxS);
    float pdf = cosine_pdf(g->nrm, wi) * pf;
    v3 wo = nrmz(sub(g->pos, cam));
    v3 wr = nrmz(reflect(wo, g->nrm));
    pdf += lobe_pdf(wi, wr, g->shin) * (1.0f - pf);
    return pdf;
}

/* brdf eval dispatch (pg/ReSTIRIntegrator.h:32-41) */
static v3 eval_brdf(const or_gbe* g, v3 cam, v3 wi, float im_cached, int use_cache) {
    int phong = g->type == MT_PHONG || g->type == MT_DIELECTRIC;
    if (!phong) return scl(g->kd, OR_ONE_OVER_PI);     /* MaterialLambert::evalBRDF (pg/MaterialLambert.cpp:33-41) */
    /* MaterialPhong::evalBRDF (pg/MaterialPhong.cpp:122-148) */
    v3 Vv = nrmz(sub(cam, g->pos));
    v3 f = scl(g->kd, OR_ONE_OVER_PI);
    float i_m;
    if (use_cache) i_m = im_cached;
    else { float nDotV = dot(Vv, g->nrm); i_m = 1.0f / or_calc_I_M(nDotV, g->shin); }
    v3 wr = nrmz(reflect(neg(Vv), g->nrm));
    float pw = rs_powf(gmax(dot(wi, wr), 0.0f), g->shin);
    f = add(f, scl(scl(g->ks, i_m), pw));
    return f;
}

/* ReSTIRIntegrator::evaluateF (pg/ReSTIRIntegrator.cpp:185-211).  The shadow ray is skipped
 * when L_i*f_r*G is exactly zero in every channel: the product is then 0 whatever V is. */
static v3 evaluate_f(const fctx* F, sample_t smp, v3 cam, const or_gbe* g, float im, int test_vis, uint64_t* rays) {
    if (!smp_valid(smp) || g->le.x > 0 || g->le.y > 0 || g->le.z > 0) return V(0, 0, 0);
    tl_ref += test_vis ? 1u : 0u;
    v3 ld = sub(smp.p, g->pos);
    float r2 = dot(ld, ld);
    ld = nrmz(ld);
    float cI = gmax(dot(ld, g->nrm), 0.0f);
    float cY = fabsf(dot(neg(ld), smp.n));
    float G = cI * cY / r2;
    v3 fr = eval_brdf(g, cam, ld, im, F->c->cache_im);
    v3 L = scl(mul(smp.li, fr), G);
    if (test_vis && !(L.x == 0.0f && L.y == 0.0f && L.z == 0.0f)) {
        int vis = !occluded(F, g->pos, smp.p, rays);
        L = scl(L, (float)vis);
    }
    return L;
}
/* evaluatePHat = length(evaluateF) (pg/ReSTIRIntegrator.cpp:180-183) */
static float eval_phat(const fctx* F, sample_t smp, v3 cam, const or_gbe* g, float im, int test_vis, uint64_t* rays) {
    return len(evaluate_f(F, smp, cam, g, im, test_vis, rays));
}

/* CosineWeightedDistribution::sample (pg/Distribution.h:7-28) */
static v3 ortho(v3 v) {                       /* Utils::orthogonal (pg/utils.cpp:204-207) */
    return fabsf(v.x) > fabsf(v.z) ? V(v.y, -v.x, 0.0f) : V(0.0f, v.z, -v.y);
}
static v3 to_world(v3 smp, v3 n) {
    v3 o2 = nrmz(ortho(n));
    v3 o1 = nrmz(cross(n, o2));
    o2 = nrmz(cross(o1, n));
    /* glm::mat3{o1,o2,n} * smp */
    return V(o1.x * smp.x + o2.x * smp.y + n.x * smp.z,
             o1.y * smp.x + o2.y * smp.y + n.y * smp.z,
             o1.z * smp.x + o2.z * smp.y + n.z * smp.z);
}
static v3 cosine_sample_u(v3 n, float r1, float r2) {
    float ang = OR_PI * 2.0f * r1;
    float x = rs_cosf(ang) * sqrtf(1.0f - r2);
    float y = rs_sinf(ang) * sqrtf(1.0f - r2);
    float z = sqrtf(r2);
    return to_world(nrmz(V(x, y, z)), n);
}
static v3 cosine_sample(v3 n, rng_t* rng) {
    float r1 = rnd(rng, 0, 1), r2 = rnd(rng, 0, 1);
    return cosine_sample_u(n, r1, r2);
}
/* CosineLobeDistribution::sample (pg/Distribution.h:37-57) */
static v3 lobe_sample_u(v3 wr, float gamma, float r1, float r2) {
    float ang = 2.0f * OR_PI * r1;
    float x = rs_cosf(ang) * sqrtf(1.0f - rs_powf(r2, 2.0f / (gamma + 1.0f)));
    float y = rs_sinf(ang) * sqrtf(1.0f - rs_powf(r2, 2.0f / (gamma + 1.0f)));
    float z = rs_powf(r2, 1.0f / (gamma + 1.0f));
    return to_world(nrmz(V(x, y, z)), wr);
}
static v3 lobe_sample(v3 wr, float gamma, rng_t* rng) {
    float r1 = rnd(rng, 0, 1), r2 = rnd(rng, 0, 1);
    return lobe_sample_u(wr, gamma, r1, r2);
}

/* BRDF sampling dispatch (pg/ReSTIRIntegrator.h:43-52): returns omega_i and pdf */
static v3 sample_brdf(const or_gbe* g, v3 cam, rng_t* rng, float* pdf_out) {
    if (g->type == MT_LAMBERT) {
        /* MaterialLambert::sampleBRDF (pg/MaterialLambert.cpp:43-53) */
        v3 wi = cosine_sample(g->nrm, rng);
        *pdf_out = cosine_pdf(g->nrm, wi);
        return wi;
    }
    /* MaterialPhong::sampleBRDF (pg/MaterialPhong.cpp:174-222) */
    v3 wo = nrmz(sub(g->pos, cam));
    float maxD = maxc(g->kd), maxS = maxc(g->ks);
    float r0 = rnd(rng, 0.0f, maxD + maxS);
    float pf = maxD / (maxD + maxS);
    v3 wr = nrmz(reflect(wo, g->nrm));
    v3 wi;
    if (r0 < maxD) wi = cosine_sample(g->nrm, rng);
    else wi = lobe_sample(wr, g->shin, rng);
    float pd = cosine_pdf(g->nrm, wi) * pf;
    float ps = lobe_pdf(wi, wr, g->shin) * (1.0f - pf);
    *pdf_out = pd + ps;
    return wi;
}

/* m_area / m_brdf (pg/ReSTIRIntegrator.h:62-74) */
static inline float m_area(const or_params* P, float pa, float pb) {
    if (pa == 0.0f && pb == 0.0f) return 0.0f;
    return pa / ((float)P->m_area * pa + (float)P->m_brdf * pb);
}
static inline float m_brdf(const or_params* P, float pb, float pa) {
    if (pa == 0.0f && pb == 0.0f) return 0.0f;
    return pb / ((float)P->m_area * pa + (float)P->m_brdf * pb);
}

/* ------------------------------------------------------------------ passes */
/* Camera (pg/camera.cpp:12-58,81-84) */
typedef struct { v3 eye; m4 view, inv_view; float focal; } or_cam;
static or_cam make_cam(const float* cam7, int W, int H) {
    or_cam c;
    v3 from = V(cam7[0], cam7[1], cam7[2]), at = V(cam7[3], cam7[4], cam7[5]);
    float fov = cam7[6];
    /* setFOV: fov_y = radians(fov); f_y = H / (2 tanf(fov_y/2)) */
    float fov_rad = fov * 0.01745329251994329576923690768489f;
    c.focal = (float)H / (2.0f * tanf(fov_rad / 2.0f));
    /* recalculate_m_c_w */
    v3 up = V(0.0f, 0.0f, 1.0f);
    v3 zc = nrmz(sub(from, at));
    v3 xc = nrmz(cross(up, zc));
    v3 yc = nrmz(cross(zc, xc));
    c.view = look_at_rh(from, at, yc);
    c.inv_view = inverse4(&c.view);
    c.eye = from;
    return c;
}
/* Camera::GenerateRay (pg/camera.cpp:20-42), CenterSampler => pixel corner */
static v3 primary_dir(const or_cam* c, int x, int y, int W, int H) {
    v3 dc = V((float)x - (float)W / 2.0f, (float)H / 2.0f - (float)y, -c->focal);
    return nrmz(m3_mul(&c->inv_view, dc));
}

/* gBufferFillPass (pg/ReSTIRIntegrator.cpp:213-234) for one pixel and the camera `cam` (Camera::GenerateRay,
 * pg/camera.cpp:20-42, CenterSampler => pixel corner): the G element and its cached 1/I_M */
static void gbuffer_elem(const fctx* F, const or_gcam* cam, int x, int y, or_gbe* e, float* imv, uint64_t* rc) {
    const or_params* P = F->P; const or_scene* s = F->s; int W = F->c->W, H = F->c->H;
    v3 dc = V((float)x - (float)W / 2.0f, (float)H / 2.0f - (float)y, -cam->focal);
    v3 d = nrmz(m3_mul(&cam->inv_view, dc));
    hitinfo h = intersect(F, cam->pos, d, FLT_MIN + 0.01f, rc);
    memset(e, 0, sizeof *e);
    *imv = 0.0f;
    if (h.hit) {
        const or_mat* m = &s->mats[s->mat[h.prim]];
        e->pos = h.point; e->nrm = h.normal;
        e->depth = len(sub(h.point, cam->pos));
        e->type = m->type; e->kd = m->kd; e->ks = m->ks; e->le = m->le; e->shin = m->shin;
        apply_maps(s, h.prim, h.u, h.v, s->mat[h.prim], &e->kd, &e->ks, &e->shin, &e->nrm, 0);
        if (e->type == MT_PHONG || e->type == MT_DIELECTRIC) {
            v3 Vv = nrmz(sub(cam->pos, e->pos));
            *imv = 1.0f / or_calc_I_M(dot(Vv, e->nrm), e->shin);
        }
    } else {
        e->le = P->use_skybox ? sky_texel(s, d) : V(P->bg_color[0], P->bg_color[1], P->bg_color[2]);
    }
}
static void pass_gbuffer(fctx* F, const or_cam* cam, or_gbe* G, float* im, int y0, int y1, uint64_t* rays) {
    int W = F->c->W;
    or_gcam gc; gc.pos = cam->eye; gc.view = cam->view; gc.inv_view = cam->inv_view; gc.focal = cam->focal;
    uint64_t rc = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+:rc)
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < W; ++x)
            gbuffer_elem(F, &gc, x, y, &G[(size_t)y * W + x], &im[(size_t)y * W + x], &rc);
    *rays += rc;
}

/* areaSampleLight (pg/ReSTIRIntegrator.cpp:89-124) + TriangleCDF::getTriangle (pg/TriangleCDF.cpp:36-54)
 * + Sampling::sampleTriangle (pg/Sampling.cpp:63-76) */
static sample_t area_sample(const fctx* F, const or_gbe* g, v3 cam, rng_t* rng, float* W_out, float* mis_out) {
    const or_scene* s = F->s;
    float ksi = rnd(rng, 0.0f, 1.0f);
    /* std::lower_bound(cdf2, ksi) */
    uint32_t lo = 0, n = s->n_emis;
    while (n > 0) { uint32_t h = n / 2; if (s->cdf[lo + h] < ksi) { lo = lo + h + 1; n = n - h - 1; } else n = h; }
    uint32_t idx = lo;
    if (idx >= s->n_emis) idx = s->n_emis - 1;
    float pick = s->pick_pdf[idx];
    uint32_t t = s->emis_tri[idx];
    float r1 = rnd(rng, 0, 1), r2 = rnd(rng, 0, 1);
    float x = 1.0f - sqrtf(r1);
    float y = sqrtf(r1) * (1.0f - r2);
    float z = sqrtf(r1) * r2;
    v3 pt = add(add(scl(s->p0[t], x), scl(s->p1[t], y)), scl(s->p2[t], z));
    v3 nn = nrmz(add(add(scl(s->n0[t], x), scl(s->n1[t], y)), scl(s->n2[t], z)));
    float tri_pdf = 1.0f / s->area[idx];
    float pdf_area = pick * tri_pdf;
    v3 ld = sub(pt, g->pos);
    float r2s = dot(ld, ld);
    ld = nrmz(ld);
    float cY = gmax(dot(neg(ld), nn), 0.0f);
    float amf = cY / r2s;
    float pb = phong_eval_pdf(g, cam, ld);
    float pba = pb * amf;
    sample_t smp = {pt, nn, s->mats[s->mat[t]].le};
    *mis_out = m_area(F->P, pdf_area, pba);
    *W_out = 1.0f / pdf_area;
    return smp;
}

/* brdfSampleLight (pg/ReSTIRIntegrator.cpp:126-177) */
static sample_t brdf_sample(const fctx* F, const or_gbe* g, v3 cam, rng_t* rng, float* W_out, float* mis_out, uint64_t* rays) {
    const or_scene* s = F->s; const or_params* P = F->P;
    float pdf;
    v3 wi = sample_brdf(g, cam, rng, &pdf);
    v3 org = add(g->pos, scl(g->nrm, P->normal_offset));
    hitinfo h = intersect(F, org, wi, FLT_MIN + P->tnear_offset, rays);
    sample_t smp = smp_invalid();
    *W_out = 0.0f; *mis_out = 0.0f;
    if (h.hit) {
        const or_mat* m = &s->mats[s->mat[h.prim]];
        if (m->le.x + m->le.y + m->le.z > 0) {
            v3 kd_, ks_; float sh_;
            apply_maps(s, h.prim, h.u, h.v, s->mat[h.prim], &kd_, &ks_, &sh_, &h.normal, 1);   /* normal map */
            v3 ld = sub(h.point, g->pos);
            float r2s = dot(ld, ld);
            ld = nrmz(ld);
            float cY = gmax(dot(neg(ld), h.normal), 0.0f);
            float amf = cY / r2s;
            int32_t e = s->emis_id[h.prim];
            /* TriangleCDF::getPDFForTriangle (pg/TriangleCDF.h:25-31) */
            float pdf_area = s->area[e] / s->total_area;
            pdf_area *= 1.0f / s->area[e];
            float bpa = pdf * amf;
            smp.p = h.point; smp.n = h.normal; smp.li = m->le;
            *W_out = 1.0f / bpa;
            *mis_out = m_brdf(P, bpa, pdf_area);
        }
    }
    return smp;
}

/* initialRenderPass (pg/ReSTIRIntegrator.cpp:236-298) */
static void pass_initial(fctx* F, or_res* Rw, int y0, int y1, uint64_t* rays) {
    const or_params* P = F->P; int W = F->c->W; v3 cam = F->gc->pos;
    uint64_t rc = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+:rc)
    for (int y = y0; y < y1; ++y) {
        for (int x = 0; x < W; ++x) {
            size_t p = (size_t)y * W + x;
            const or_gbe* g = &F->G[p];
            float im = F->im[p];
            if (nonzero_pos(g->le) || F->s->n_emis == 0) { Rw[p] = res_empty(); continue; }
            rng_t rng = rng_init(P->seed, F->frame, PASS_INITIAL, (uint32_t)p);
            or_res r = res_empty();
            int tv = !P->do_visibility_pass;
            float best_phat = 0.0f;   /* p-hat of the selected candidate: the final p-hat (:289) */
            if (P->m_area > 0) {
                float inv_ma = 1.0f / (float)P->m_area;
                for (int i = 0; i < P->m_area; ++i) {
                    float Wc, mis;
                    rng.n = cand_slot(i);
                    sample_t smp = area_sample(F, g, cam, &rng, &Wc, &mis);
                    float ph = eval_phat(F, smp, cam, g, im, tv, &rc);
                    float w = P->m_brdf > 0 ? mis * ph * Wc : inv_ma * ph * Wc;
                    rng.n = cand_slot(i) + 3u;
                    if (res_add(&r, smp, w, 1, &rng)) best_phat = ph;
                }
            }
            if (P->m_brdf > 0) {
                float inv_mb = 1.0f / (float)P->m_brdf;
                for (int i = 0; i < P->m_brdf; ++i) {
                    float Wc, mis;
                    rng.n = cand_slot(P->m_area + i);
                    sample_t smp = brdf_sample(F, g, cam, &rng, &Wc, &mis, &rc);
                    float ph = eval_phat(F, smp, cam, g, im, tv, &rc);
                    float w = P->m_area > 0 ? mis * ph * Wc : inv_mb * ph * Wc;
                    rng.n = cand_slot(P->m_area + i) + 3u;
                    if (res_add(&r, smp, w, 1, &rng)) best_phat = ph;
                }
            }
            float ph = sample_valid(&r) ? best_phat : 0.0f;
            tl_ref += (tv && sample_valid(&r)) ? 1u : 0u;        /* :289 re-evaluated with visibility */
            r.W = ph > 0.0f ? 1.0f / ph * r.wsum : 0.0f;
            res_cap(&r, P->confidence_cap);
            Rw[p] = r;
        }
    }
    *rays += rc;
}

/* visibilityPass (pg/ReSTIRIntegrator.cpp:302-312) */
static void pass_visibility(fctx* F, or_res* Rw, int y0, int y1, uint64_t* rays) {
    int W = F->c->W; uint64_t rc = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+:rc)
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < W; ++x) {
            size_t p = (size_t)y * W + x;
            tl_ref++;                    /* the reference traces it for every pixel */
            /* invalid samples only ever carry W == 0 already: skip their (meaningless) ray */
            if (!sample_valid(&Rw[p])) continue;
            if (occluded(F, F->G[p].pos, Rw[p].p, &rc)) Rw[p].W = 0;
        }
    *rays += rc;
}

/* reprojectBackward / reprojectForward (pg/ReSTIRIntegrator.cpp:544-587) */
static int reproject(const or_gcam* gc, v3 ws, int W, int H, int* sx, int* sy) {
    v3 vs = m4_mul_point(&gc->view, ws);
    if (vs.z >= 0) return 0;
    float fx = (-vs.x / vs.z) * gc->focal + (float)W / 2.0f;
    float fy = (vs.y / vs.z) * gc->focal + (float)H / 2.0f;
    float rx = roundf(fx), ry = roundf(fy);   /* glm::round = std::round (half away from zero) */
    /* int conversion of the rounded value; out-of-range values are rejected below */
    if (!(rx >= -2147483648.0f && rx < 2147483648.0f) || !(ry >= -2147483648.0f && ry < 2147483648.0f)) return 0;
    int X = (int)rx, Y = (int)ry;
    if (X < 0 || X > W - 1 || Y < 0 || Y > H - 1) return 0;
    *sx = X; *sy = Y;
    return 1;
}

/* temporalReusePass (pg/ReSTIRIntegrator.cpp:625-732).  debugReprojection (:30, :647-689): the rejection
 * colours go into the current G-buffer's emission AFTER the pass (the reference's OpenMP loop writes them
 * while other pixels read -- a race; here no pixel of the pass sees them), a pixel's own colour winning
 * over a forward-check mark (0,0,100) from another pixel. */
static void pass_temporal(fctx* F, const or_res* Rr, const or_res* Rl, or_res* Rw, int y0, int y1, uint64_t* rays) {
    const or_params* P = F->P; int W = F->c->W, H = F->c->H;
    uint64_t rc = 0, rebuilt = 0;
    const size_t npx = (size_t)W * H;
    uint8_t* dbg = P->debug_reprojection ? (uint8_t*)calloc(2 * npx, 1) : NULL;
#define DBG_OWN(code) do { if (dbg) dbg[p] = (code); } while (0)
#pragma omp parallel for schedule(dynamic, 1) reduction(+:rc, rebuilt)
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < W; ++x) {
            size_t p = (size_t)y * W + x;
            const or_gbe* cur = &F->G[p];
            v3 ccam = F->gc->pos, pcam = F->gcp->pos;
            const or_res* cr = &Rr[p];
            const or_res* pr = &Rl[p];       /* previous reservoir read at the CURRENT pixel (:641) */
            int qx, qy;
            if (!reproject(F->gcp, cur->pos, W, H, &qx, &qy)) { Rw[p] = *cr; DBG_OWN(1); continue; }
            size_t q = (size_t)qy * W + qx;
            const or_gbe* prev = &F->Gp[q];
            float imq = F->imp[q];
            /* tile mode: an element beyond the tile's G-buffer rows is rebuilt from the previous camera
               (full frame: never) -- the product's k_temporal does the same */
            or_gbe prev_alt;
            if (qy < F->gy0 || qy >= F->gy1) {
                gbuffer_elem(F, F->gcp, qx, qy, &prev_alt, &imq, &rc);
                prev = &prev_alt;
                rebuilt++;
            }
            float cd = len(sub(cur->pos, ccam));
            float pd = len(sub(prev->pos, pcam));
            float dr = cd > pd ? pd / cd : cd / pd;
            if (dr < 0.9f) { Rw[p] = *cr; DBG_OWN(2); continue; }
            const or_gbe* pac = &F->Gp[p];
            int fx, fy;
            if (!reproject(F->gc, pac->pos, W, H, &fx, &fy)) { Rw[p] = *cr; DBG_OWN(3); continue; }
            const or_gbe* fw = &F->G[(size_t)fy * W + fx];
            or_gbe fw_alt; float im_unused;
            if (fy < F->gy0 || fy >= F->gy1) {
                gbuffer_elem(F, F->gc, fx, fy, &fw_alt, &im_unused, &rc);
                fw = &fw_alt;
                rebuilt++;
            }
            float cdp = len(sub(pac->pos, pcam));
            float pdp = len(sub(fw->pos, ccam));
            float drp = cdp > pdp ? pdp / cdp : cdp / pdp;
            if (drp < 0.9f) {
                Rw[p] = *cr;
                if (dbg) dbg[npx + (size_t)fy * W + fx] = 1;   /* the same value from any pixel */
                continue;
            }

            rng_t rng = rng_init(P->seed, F->frame, PASS_TEMPORAL, (uint32_t)p);
            or_res res = res_empty();
            float imc = F->im[p];
            sample_t cs = smp_of(cr), ps = smp_of(pr);
            float p_cur = eval_phat(F, cs, ccam, cur, imc, 1, &rc);
            float p_prev = eval_phat(F, cs, pcam, prev, imq, 1, &rc);
            float m_cur = p_cur * (float)cr->conf / (p_cur * (float)cr->conf + p_prev * (float)pr->conf);
            if (!(m_cur > 0)) m_cur = 0.0f;
            float ph_cur = p_cur;  /* :706 re-evaluates the identical p-hat */
            tl_ref += (smp_valid(cs) && !nonzero_pos(cur->le)) ? 1u : 0u;
            float w_cur = m_cur * ph_cur * cr->W;
            int took_cur = res_add(&res, cs, w_cur, cr->conf, &rng);
            p_cur = eval_phat(F, ps, ccam, cur, imc, 1, &rc);
            p_prev = eval_phat(F, ps, pcam, prev, imq, 1, &rc);
            float m_prev = p_prev * (float)pr->conf / (p_cur * (float)cr->conf + p_prev * (float)pr->conf);
            if (!(m_prev > 0)) m_prev = 0.0f;
            float ph_prev = p_cur;  /* :721 re-evaluates the identical p-hat */
            tl_ref += (smp_valid(ps) && !nonzero_pos(cur->le)) ? 1u : 0u;
            float w_prev = m_prev * ph_prev * pr->W;
            int took_prev = res_add(&res, ps, w_prev, pr->conf, &rng);
            res_cap(&res, P->confidence_cap);
            /* final p-hat (:727) of the surviving sample at the current pixel */
            float fph = took_prev ? ph_prev : (took_cur ? ph_cur : 0.0f);
            tl_ref += (sample_valid(&res) && !nonzero_pos(cur->le)) ? 1u : 0u;
            res.W = fph > 0.0f ? res.wsum / fph : 0.0f;
            Rw[p] = res;
        }
#undef DBG_OWN
    if (dbg) {
        or_gbe* G = (or_gbe*)F->G;    /* the context's current G-buffer */
        for (size_t q = 0; q < npx; ++q) {
            const uint8_t own = dbg[q], fwd = dbg[npx + q];
            if (!own && !fwd) continue;
            G[q].le = own == 1 ? V(100, 100, 0) : own == 2 ? V(0, 100, 0) : own == 3 ? V(100, 0, 100) : V(0, 0, 100);
        }
        free(dbg);
    }
    *rays += rc;
    F->c->rebuilt += rebuilt;
}

/* Sampling::sampleDiskUniform (pg/Sampling.cpp:78-87) + vec2 -> ivec2 truncation */
static void disk_offset(float radius, rng_t* rng, int* ox, int* oy) {
    float theta = rnd(rng, 0, 2.0f) * OR_PI;
    float r = sqrtf(rnd(rng, 0, radius));
    float x = r * rs_cosf(theta);
    float y = r * rs_sinf(theta);
    *ox = (int)x; *oy = (int)y;
}

/* spatialReusePass (pg/ReSTIRIntegrator.cpp:316-542) */
static void pass_spatial(fctx* F, const or_res* Rr, or_res* Rw, int pass_idx, int y0, int y1, uint64_t* rays) {
    const or_params* P = F->P; int W = F->c->W, H = F->c->H;
    v3 cam = F->gc->pos;
    uint64_t rc = 0;
    int kmax = P->spatial_neighbors;
#pragma omp parallel for schedule(dynamic, 1) reduction(+:rc)
    for (int y = y0; y < y1; ++y) {
        int* nb = (int*)malloc(sizeof(int) * (size_t)(kmax + 1));
        for (int x = 0; x < W; ++x) {
            size_t p = (size_t)y * W + x;
            const or_gbe* th = &F->G[p];
            if (nonzero_pos(th->le)) { Rw[p] = Rr[p]; continue; }
            rng_t rng = rng_init(P->seed, F->frame, PASS_SPATIAL0 + (uint32_t)pass_idx, (uint32_t)p);
            int M = 1, cnt = 0;
            nb[cnt++] = (int)p;
            for (int i = 0; i < kmax; ++i) {
                int ox, oy;
                disk_offset(P->spatial_radius, &rng, &ox, &oy);
                int nx = x + ox, ny = y + oy;
                nx = nx < 0 ? 0 : (nx > W - 1 ? W - 1 : nx);    /* glm::clamp = min(max()) */
                ny = ny < 0 ? 0 : (ny > H - 1 ? H - 1 : ny);
                size_t q = (size_t)ny * W + nx;
                const or_gbe* ne = &F->G[q];
                if (nonzero_pos(ne->le)) continue;
                if (P->reject_dissimilar) {
                    float ns = dot(ne->nrm, th->nrm);
                    if (ns < P->min_normal_similarity) continue;
                    float dr = 0;
                    if (ne->depth > 0) dr = th->depth / ne->depth;
                    float hd = P->max_depth_difference * 0.5f;
                    if (dr < 1.0f - hd || dr > 1.0f + hd) continue;
                }
                nb[cnt++] = (int)q; M += 1;
            }
            int csum = 0, csum_nc = 0;
            for (int i = 0; i < cnt; ++i) { int c = Rr[nb[i]].conf; csum += c; if (i) csum_nc += c; }
            or_res res = res_empty();
            int sel = 0;
            float rcpM = M > 0 ? 1.0f / (float)M : 0.0f;
            float sel_phat = 0.0f;
            for (int i = 0; i < cnt; ++i) {
                const or_res* ri = &Rr[nb[i]];
                sample_t si = smp_of(ri);
                float mis = rcpM;
                if (P->spatial_mis == MIS_BALANCE) {
                    float num = 0, den = 0; mis = 0.0f;
                    for (int j = 0; j < cnt; ++j) {
                        const or_res* rj = &Rr[nb[j]];
                        float ph = eval_phat(F, si, cam, &F->G[nb[j]], F->im[nb[j]], 1, &rc);
                        den += ph * rj->conf;
                        if (i == j) num = ph * ri->conf;
                    }
                    if (den > 0) mis = num / den;
                }
                if (P->spatial_mis == MIS_PAIRWISE) {
                    mis = 0.0f;
                    if (i == 0) {
                        float sum = 0.0f;
                        float phc = eval_phat(F, si, cam, &F->G[nb[i]], F->im[nb[i]], 1, &rc) * (float)ri->conf;
                        for (int j = 1; j < cnt; ++j) {
                            const or_res* rj = &Rr[nb[j]];
                            float phj = eval_phat(F, si, cam, &F->G[nb[j]], F->im[nb[j]], 1, &rc);
                            float den = phc + phj * (float)csum_nc;
                            if (den > 0) {
                                float cf = (float)rj->conf / (float)csum;
                                sum += cf * (phc / den);
                            }
                        }
                        mis = ((float)ri->conf / (float)csum) + sum;
                    } else {
                        float phi = eval_phat(F, si, cam, &F->G[nb[i]], F->im[nb[i]], 1, &rc);
                        float phc = eval_phat(F, si, cam, &F->G[nb[0]], F->im[nb[0]], 1, &rc);
                        phi *= (float)csum_nc;
                        float den = phi + phc * (float)Rr[nb[0]].conf;
                        if (den > 0 && csum > 0) mis = ((float)ri->conf / (float)csum) * (phi / den);
                    }
                }
                float rph = eval_phat(F, si, cam, th, F->im[p], 1, &rc);
                float rw = mis * rph * ri->W;
                if (res_add(&res, si, rw, ri->conf, &rng)) { sel = i; sel_phat = rph; }
            }
            /* final p-hat (:481): p-hat of the surviving sample at this pixel = sel_phat */
            float fph = sample_valid(&res) ? sel_phat : 0.0f;
            tl_ref += sample_valid(&res) ? 1u : 0u;
            if (P->spatial_mis == MIS_CONSTANT || P->spatial_mis == MIS_BALANCE || P->spatial_mis == MIS_PAIRWISE) {
                res.W = fph > 0.0f ? res.wsum / fph : 0.0f;
            } else if (P->spatial_mis == MIS_DEBIAS_Z) {
                int Z = 0; float corr = 1.0f;
                for (int i = 0; i < cnt; ++i) {
                    tl_ref++;
                    if (!occluded(F, F->G[nb[i]].pos, res.p, &rc)) Z += 1;
                }
                if (Z > 0 && M > 0) corr = (1.0f / (float)Z) / rcpM;
                res.W = fph > 0.0f ? corr * res.wsum / fph : 0.0f;
            } else if (P->spatial_mis == MIS_DEBIAS_CONTRIB) {
                sample_t ss = smp_of(&Rr[nb[sel]]);
                float num = 0, den = 0, cw = 0, corr = 0;
                for (int i = 0; i < cnt; ++i) {
                    const or_res* ri = &Rr[nb[i]];
                    float ph = eval_phat(F, ss, cam, &F->G[nb[i]], F->im[nb[i]], 1, &rc);
                    den += ph * (float)ri->conf;
                    if (i == sel) num = ph * (float)ri->conf;
                }
                if (den > 0) cw = num / den;
                if (M > 0) corr = cw / rcpM;
                res.W = fph > 0.0f ? corr * res.wsum / fph : 0.0f;
            }
            res_cap(&res, P->confidence_cap);
            Rw[p] = res;
        }
        free(nb);
    }
    *rays += rc;
}

/* Integrator::sanitize (pg/Integrator.cpp:6-22) */
static v3 sanitize(v3 l) {
    if (isnan(l.x) || isnan(l.y) || isnan(l.z)) l = V(0, 0, 0);
    if (l.x < 0 || l.y < 0 || l.z < 0) l = V(0, 0, 0);
    return l;
}

/* shade loop (pg/simpleguidx11.cpp:447-472) */
static void pass_shade(fctx* F, const or_res* Rr, float* out, int y0, int y1, uint64_t* rays) {
    int W = F->c->W; v3 cam = F->gc->pos; uint64_t rc = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+:rc)
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < W; ++x) {
            size_t p = (size_t)y * W + x;
            const or_res* r = &Rr[p];
            v3 px;
            if (r->wsum > 0.0f) {     /* Reservoir::hasSample (pg/Reservoir.h:49-52) */
                v3 f = evaluate_f(F, smp_of(r), cam, &F->G[p], F->im[p], 1, &rc);
                px = scl(f, r->W);
            } else px = F->G[p].le;
            px = sanitize(px);
            float* o = out + 3 * (size_t)(y - y0) * W + 3 * (size_t)x;
            o[0] = px.x; o[1] = px.y; o[2] = px.z;
        }
    *rays += rc;
}

/* ------------------------------------------------------------------ frame / tile driver
 * SimpleGuiDX11::produceRestir (pg/simpleguidx11.cpp:359-487) split into the stages a row band of a
 * tile-sharded frame runs (same stages as the HIP product's rs_tile_* C ABI):
 *   begin    : G-buffer rows [y0-margin, y1+margin), initial RIS (+ visibility) rows [y0, y1)
 *   halo     : the caller exchanges reservoir rows [y0-halo, y0) / [y1, y1+halo) between stages
 *   temporal : rows [y0, y1);  spatial(p): rows [y0, y1);  finish: shade rows [y0, y1), swap history */
typedef struct {
    int active, y0, y1, halo, ra, rb, rcur, last, temporal_ran;
    or_params P; fctx F; or_cam cam; uint64_t rays;
} or_tile_state;
static or_tile_state* tile_of(or_ctx* c) {
    if (!c->tile) c->tile = calloc(1, sizeof(or_tile_state));
    return (or_tile_state*)c->tile;
}
static void tile_release(or_ctx* c) { free(c->tile); c->tile = NULL; }

int or_tile_begin(or_ctx* c, const or_scene* s, const float* cam7, const or_params* P, uint32_t frame_index,
                  int y0, int y1, int margin, int halo) {
    int W = c->W, H = c->H;
    /* useSkybox reads the scene's equirect sky (pg/SphericalMap.cpp:10-14) */
    if (P->use_skybox && s->sky < 0) return -2;
    if (y0 < 0 || y1 > H || y0 >= y1 || margin < 0 || halo < 0 || halo > margin) return -1;
    or_tile_state* T = tile_of(c);
    if (!T) return -1;
    (void)fold_ref();            /* drop counts of earlier non-frame calls (trace hooks, MIS frames) */
    T->P = *P; T->y0 = y0; T->y1 = y1; T->halo = halo; T->rays = 0;
    T->cam = make_cam(cam7, W, H);
    /* G-buffer ping-pong instead of gBufferLastFrame.setDataFrom (:480) */
    int gcur = c->gcur ^ 1, gprev = c->gcur;
    c->gc[gcur].pos = T->cam.eye; c->gc[gcur].view = T->cam.view; c->gc[gcur].inv_view = T->cam.inv_view;
    c->gc[gcur].focal = T->cam.focal;
    fctx* F = &T->F;
    F->s = s; F->c = c; F->P = &T->P; F->frame = frame_index;
    F->G = c->g[gcur]; F->Gp = c->g[gprev]; F->gc = &c->gc[gcur]; F->gcp = &c->gc[gprev];
    F->im = c->im_cache[gcur]; F->imp = c->im_cache[gprev];
    F->gy0 = y0 - margin < 0 ? 0 : y0 - margin;
    F->gy1 = y1 + margin > H ? H : y1 + margin;
    pass_gbuffer(F, &T->cam, c->g[gcur], c->im_cache[gcur], F->gy0, F->gy1, &T->rays);
    /* reservoir buffer choice: never overwrite R_last before the temporal pass */
    T->last = c->r_last;
    T->ra = (T->last + 1) % 3; T->rb = (T->last + 2) % 3;
    pass_initial(F, c->r[T->ra], y0, y1, &T->rays);
    if (P->do_visibility_pass) pass_visibility(F, c->r[T->ra], y0, y1, &T->rays);
    T->rcur = T->ra;
    T->temporal_ran = 0;
    T->active = 1;
    c->gcur = gcur;
    return 0;
}

/* which: 0 rows [y0-halo, y0), 1 rows [y1, y1+halo), 2 rows [y0, y0+halo), 3 rows [y1-halo, y1)
   of the current reservoir buffer (48 B per pixel); NULL when outside the frame */
int or_tile_halo_ptr(or_ctx* c, int which, void** ptr, size_t* bytes) {
    or_tile_state* T = tile_of(c);
    if (!T || !T->active) return -1;
    int h = T->halo, r0;
    switch (which) {
        case 0: r0 = T->y0 - h; break;
        case 1: r0 = T->y1; break;
        case 2: r0 = T->y0; break;
        case 3: r0 = T->y1 - h; break;
        default: return -1;
    }
    if (h == 0 || r0 < 0 || r0 + h > c->H) { *ptr = NULL; *bytes = 0; return 0; }
    *ptr = (void*)(c->r[T->rcur] + (size_t)r0 * c->W);
    *bytes = (size_t)h * c->W * sizeof(or_res);
    return 0;
}

int or_tile_temporal(or_ctx* c) {
    or_tile_state* T = tile_of(c);
    if (!T || !T->active) return -1;
    if (T->P.do_temporal && c->frames > 0 && !T->temporal_ran) {
        pass_temporal(&T->F, c->r[T->rcur], c->r[T->last], c->r[T->rb], T->y0, T->y1, &T->rays);
        T->rcur = T->rb;
        T->temporal_ran = 1;
    }
    return 0;
}

int or_tile_spatial(or_ctx* c, int pass_index) {
    or_tile_state* T = tile_of(c);
    if (!T || !T->active) return -1;
    if (!(T->P.do_spatial && pass_index >= 0 && pass_index < T->P.spatial_passes)) return 0;
    or_tile_temporal(c);
    int dst = (T->rcur == T->ra) ? T->rb : T->ra;
    pass_spatial(&T->F, c->r[T->rcur], c->r[dst], pass_index, T->y0, T->y1, &T->rays);
    T->rcur = dst;
    return 0;
}

/* out_rgb: (y1-y0)*W*3 floats of the band */
int or_tile_finish(or_ctx* c, float* out_rgb, uint64_t* rays_out) {
    or_tile_state* T = tile_of(c);
    if (!T || !T->active) return -1;
    or_tile_temporal(c);
    pass_shade(&T->F, c->r[T->rcur], out_rgb, T->y0, T->y1, &T->rays);
    c->ref_rays = fold_ref();
    c->r_last = T->rcur;
    c->frames++;
    T->active = 0;
    if (rays_out) *rays_out = T->rays;
    return 0;
}

/* one full frame (no tiling); out_rgb = W*H*3 floats (frame_data) */
int or_render_frame(or_ctx* c, const or_scene* s, const float* cam7, const or_params* P,
                    uint32_t frame_index, float* out_rgb, uint64_t* rays_out) {
    int rc = or_tile_begin(c, s, cam7, P, frame_index, 0, c->H, 0, 0);
    if (rc) return rc;
    or_tile_temporal(c);
    if (P->do_spatial)
        for (int i = 0; i < P->spatial_passes; ++i) or_tile_spatial(c, i);
    return or_tile_finish(c, out_rgb, rays_out);
}

/* ------------------------------------------------------------------ MIS direct-light ground truth
 * SimpleGuiDX11::produceStandard (pg/simpleguidx11.cpp:336-357) with Raytracer::get_pixel
 * (pg/raytracer.cpp:40-45) and NEEPathIntegrator::integrateImpl2 (pg/NEEPathIntegrator.cpp:72-131)
 * at calcDI = on, calcGI = off (direct illumination only: the quantity ReSTIR DI estimates) and
 * DirectMISIntegrator as the direct integrator (pg/DirectMISIntegrator.cpp:10-143): one BRDF sample,
 * then one light sample, power heuristic.  The material calls are the HitInfo variants --
 * MaterialLambert (pg/MaterialLambert.cpp:10-31) and MaterialPhong (pg/MaterialPhong.cpp:18-119), with
 * Phong for PHONG/DIELECTRIC and Lambert for every other type (the ReSTIR path's BRDF model,
 * pg/ReSTIRIntegrator.h:32-41, so both converge to the same image).  CenterSampler primary ray
 * (pixel corner).  RNG: pass PASS_MIS, draws sequential per pixel over the spp samples. */
#define PASS_MIS 64u
typedef struct { v3 pos, n, dir, kd, ks, wr; float shin, i_m, maxD, maxS, pf; int phong; } mis_surf;

static inline float mis_power(float pdf, float other) {   /* DirectMISIntegrator::powerHeuristic (:10-15) */
    float a = pdf * pdf, b = other * other;
    return a / (b + a);
}
static inline v3 dvs(v3 v, float s) { return V(v.x / s, v.y / s, v.z / s); }   /* glm vec3 / scalar */
/* getPdfForSample (pg/MaterialLambert.cpp:20-23, pg/MaterialPhong.cpp:94-119) */
static float mis_pdf_for(const mis_surf* h, v3 wi) {
    if (!h->phong) return cosine_pdf(h->n, wi);
    float pdf = cosine_pdf(h->n, wi) * h->pf;
    pdf += lobe_pdf(wi, h->wr, h->shin) * (1.0f - h->pf);
    return pdf;
}
/* evaluateBRDF (pg/MaterialLambert.cpp:25-31, pg/MaterialPhong.cpp:69-92) */
static v3 mis_brdf(const mis_surf* h, v3 wi) {
    v3 f = scl(h->kd, OR_ONE_OVER_PI);
    if (!h->phong) return f;
    return add(f, scl(scl(h->ks, h->i_m), rs_powf(gmax(dot(wi, h->wr), 0.0f), h->shin)));
}
/* evaluateLightingGI (pg/MaterialLambert.cpp:10-18, pg/MaterialPhong.cpp:18-67) */
static v3 mis_sample(const mis_surf* h, rng_t* rng, v3* f_r, float* pdf) {
    if (!h->phong) {
        v3 wi = cosine_sample(h->n, rng);
        *pdf = cosine_pdf(h->n, wi);
        *f_r = dvs(h->kd, OR_PI);
        return wi;
    }
    float r0 = rnd(rng, 0.0f, h->maxD + h->maxS);
    v3 wi;
    if (r0 < h->maxD) {
        wi = cosine_sample(h->n, rng);
        *f_r = scl(h->kd, OR_ONE_OVER_PI);
    } else {
        wi = lobe_sample(h->wr, h->shin, rng);
        *f_r = scl(scl(h->ks, h->i_m), rs_powf(gmax(dot(wi, h->wr), 0.0f), h->shin));
    }
    float pd = cosine_pdf(h->n, wi) * h->pf;
    float ps = lobe_pdf(wi, h->wr, h->shin) * (1.0f - h->pf);
    *pdf = pd + ps;
    if (dot(h->n, wi) < 0) *f_r = V(0, 0, 0);
    return wi;
}
/* DirectMISIntegrator::evaluateBRDFSample (pg/DirectMISIntegrator.cpp:94-144) */
static v3 mis_brdf_part(const fctx* F, const mis_surf* h, rng_t* rng, uint64_t* rays) {
    const or_scene* s = F->s; const or_params* P = F->P;
    v3 f_r; float pdf;
    v3 wi = mis_sample(h, rng, &f_r, &pdf);
    hitinfo b = intersect(F, add(h->pos, scl(h->n, P->normal_offset)), wi, FLT_MIN + P->tnear_offset, rays);
    if (!b.hit) return V(0, 0, 0);
    const or_mat* m = &s->mats[s->mat[b.prim]];
    if (!(m->le.x + m->le.y + m->le.z > 0)) return V(0, 0, 0);
    v3 kd_, ks_; float sh_;
    apply_maps(s, b.prim, b.u, b.v, s->mat[b.prim], &kd_, &ks_, &sh_, &b.normal, 1);
    v3 ld = sub(b.point, h->pos);
    float r2 = dot(ld, ld);
    ld = nrmz(ld);
    float cI = gmax(dot(ld, h->n), 0.0f);
    float cY = gmax(dot(neg(ld), b.normal), 0.0f);
    float amf = cY / r2;
    int32_t e = s->emis_id[b.prim];
    float pdf_light = s->area[e] / s->total_area;       /* TriangleCDF::getPDFForTriangle (pg/TriangleCDF.h:25-31) */
    pdf_light *= 1.0f / s->area[e];
    float w = mis_power(pdf * amf, pdf_light);
    return dvs(scl(mul(scl(m->le, w), f_r), cI), pdf);
}
/* DirectMISIntegrator::evaluateLightSample (pg/DirectMISIntegrator.cpp:38-92) */
static v3 mis_light_part(const fctx* F, const mis_surf* h, rng_t* rng, uint64_t* rays) {
    const or_scene* s = F->s;
    if (s->n_emis == 0) return V(0, 0, 0);                /* TriangleCDF::isValid */
    float ksi = rnd(rng, 0.0f, 1.0f);                      /* TriangleCDF::getTriangle (pg/TriangleCDF.cpp:36-54) */
    uint32_t lo = 0, n = s->n_emis;
    while (n > 0) { uint32_t k = n / 2; if (s->cdf[lo + k] < ksi) { lo = lo + k + 1; n = n - k - 1; } else n = k; }
    uint32_t idx = lo < s->n_emis ? lo : s->n_emis - 1;
    uint32_t t = s->emis_tri[idx];
    float r1 = rnd(rng, 0, 1), r2 = rnd(rng, 0, 1);          /* Sampling::sampleTriangle (pg/Sampling.cpp:63-76) */
    float x = 1.0f - sqrtf(r1), y = sqrtf(r1) * (1.0f - r2), z = sqrtf(r1) * r2;
    v3 pt = add(add(scl(s->p0[t], x), scl(s->p1[t], y)), scl(s->p2[t], z));
    v3 nn = nrmz(add(add(scl(s->n0[t], x), scl(s->n1[t], y)), scl(s->n2[t], z)));
    float light_pdf = s->pick_pdf[idx] * (1.0f / s->area[idx]);
    if (light_pdf == 0) return V(0, 0, 0);
    v3 ld = sub(pt, h->pos);
    float r_sqr = dot(ld, ld);
    ld = nrmz(ld);
    if (r_sqr == 0) return V(0, 0, 0);
    float cI = gmax(dot(ld, h->n), 0.0f);
    float cY = gmax(dot(neg(ld), nn), 0.0f);
    float amf = cY / r_sqr;
    if (!(cI > 0 && cY > 0) || occluded(F, h->pos, pt, rays)) return V(0, 0, 0);
    float pba = mis_pdf_for(h, ld) * amf;
    v3 le = s->mats[s->mat[t]].le;
    float w = mis_power(light_pdf, pba);
    if (!(w > 0.0f)) return V(0, 0, 0);
    float G = cI * cY / r_sqr;
    return dvs(scl(mul(scl(le, w), mis_brdf(h, ld)), G), light_pdf);
}

/* out_rgb: W*H*3 floats; spp samples per pixel averaged (sum / spp) -- frame-to-frame accumulation
 * is or_post_apply's running mean, as the reference's accumulator */
int or_render_direct_mis(or_ctx* c, const or_scene* s, const float* cam7, const or_params* P, uint32_t frame_index,
                         int spp, float* out_rgb, uint64_t* rays_out) {
    if (P->use_skybox && s->sky < 0) return -2;
    if (spp < 1) return -1;
    int W = c->W, H = c->H;
    or_cam cam = make_cam(cam7, W, H);
    fctx F; memset(&F, 0, sizeof F);
    F.s = s; F.c = c; F.P = P; F.frame = frame_index;
    uint64_t rc = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+:rc)
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            size_t p = (size_t)y * W + x;
            v3 d = primary_dir(&cam, x, y, W, H);
            hitinfo hi = intersect(&F, cam.eye, d, FLT_MIN + 0.01f, &rc);
            v3 px;
            if (!hi.hit) {
                px = P->use_skybox ? sky_texel(s, d) : V(P->bg_color[0], P->bg_color[1], P->bg_color[2]);
            } else {
                const or_mat* m = &s->mats[s->mat[hi.prim]];
                v3 kd = m->kd, ks = m->ks, hn = hi.normal; float shin = m->shin;
                apply_maps(s, hi.prim, hi.u, hi.v, s->mat[hi.prim], &kd, &ks, &shin, &hn, 0);
                if (nonzero_pos(m->le)) {                  /* Material::isEmitter, camera vertex */
                    px = m->le;
                } else {
                    mis_surf h;
                    h.pos = hi.point; h.n = hn; h.dir = d;
                    h.kd = kd; h.ks = ks; h.shin = shin;
                    h.phong = m->type == MT_PHONG || m->type == MT_DIELECTRIC;
                    h.maxD = maxc(h.kd); h.maxS = maxc(h.ks);
                    h.pf = h.maxD / (h.maxD + h.maxS);
                    h.wr = nrmz(reflect(d, h.n));
                    h.i_m = h.phong ? 1.0f / or_calc_I_M(dot(neg(d), h.n), h.shin) : 0.0f;
                    rng_t rng = rng_init(P->seed, frame_index, PASS_MIS, (uint32_t)p);
                    v3 acc = V(0, 0, 0);
                    for (int k = 0; k < spp; ++k) {
                        v3 L = add(V(0, 0, 0), mis_brdf_part(&F, &h, &rng, &rc));
                        L = add(L, mis_light_part(&F, &h, &rng, &rc));
                        L = sanitize(L);
                        acc = add(acc, add(V(0, 0, 0), L));    /* L_i_indirect (0) + L_i_direct */
                    }
                    px = dvs(acc, (float)spp);
                }
            }
            px = sanitize(px);
            out_rgb[3 * p] = px.x; out_rgb[3 * p + 1] = px.y; out_rgb[3 * p + 2] = px.z;
        }
    }
    if (rays_out) *rays_out = rc;
    return 0;
}

/* ------------------------------------------------------------------ dumps / KAT hooks */
/* G-buffer dump: 19 floats per pixel: pos3 nrm3 kd3 ks3 le3 shin depth type inv_IM */
int or_get_gbuffer(const or_ctx* c, int prev, float* out) {
    int gi = prev ? (c->gcur ^ 1) : c->gcur;
    size_t n = (size_t)c->W * c->H;
    for (size_t p = 0; p < n; ++p) {
        const or_gbe* e = &c->g[gi][p]; float* o = out + 19 * p;
        o[0] = e->pos.x; o[1] = e->pos.y; o[2] = e->pos.z; o[3] = e->nrm.x; o[4] = e->nrm.y; o[5] = e->nrm.z;
        o[6] = e->kd.x; o[7] = e->kd.y; o[8] = e->kd.z; o[9] = e->ks.x; o[10] = e->ks.y; o[11] = e->ks.z;
        o[12] = e->le.x; o[13] = e->le.y; o[14] = e->le.z; o[15] = e->shin; o[16] = e->depth;
        o[17] = (float)e->type; o[18] = c->im_cache[gi][p];
    }
    return 0;
}
/* Final reservoir dump (the buffer shaded last frame = R_last): 12 floats per pixel:
   point3 normal3 Li3 w_sum W confidence */
int or_get_reservoirs(const or_ctx* c, float* out) {
    size_t n = (size_t)c->W * c->H;
    const or_res* R = c->r[c->r_last];
    for (size_t p = 0; p < n; ++p) {
        const or_res* r = &R[p]; float* o = out + 12 * p;
        o[0] = r->p.x; o[1] = r->p.y; o[2] = r->p.z; o[3] = r->n.x; o[4] = r->n.y; o[5] = r->n.z;
        o[6] = r->li.x; o[7] = r->li.y; o[8] = r->li.z; o[9] = r->wsum; o[10] = r->W; o[11] = (float)r->conf;
    }
    return 0;
}
/* camera KAT: view16 (column-major), inv16, focal, dir3 for pixel (px,py) */
int or_camera_kat(const float* cam7, int W, int H, int px, int py, float* out) {
    or_cam c = make_cam(cam7, W, H);
    memcpy(out, c.view.m, 64); memcpy(out + 16, c.inv_view.m, 64);
    out[32] = c.focal;
    v3 d = primary_dir(&c, px, py, W, H);
    out[33] = d.x; out[34] = d.y; out[35] = d.z;
    return 0;
}
int or_reproject_kat(const float* cam7, int W, int H, const float* ws, int* out_xy) {
    or_cam c = make_cam(cam7, W, H);
    or_gcam g; g.pos = c.eye; g.view = c.view; g.inv_view = c.inv_view; g.focal = c.focal;
    int x = -1, y = -1;
    if (!reproject(&g, V(ws[0], ws[1], ws[2]), W, H, &x, &y)) { x = -1; y = -1; }
    out_xy[0] = x; out_xy[1] = y;
    return 0;
}
float or_rng_u(uint32_t seed, uint32_t frame, uint32_t pass, uint32_t pixel, uint32_t n) {
    rng_t r = rng_init(seed, frame, pass, pixel); r.n = n; return rng_u(&r);
}
/* scene introspection for tests */
uint32_t or_scene_n_emissive(const or_scene* s) { return s->n_emis; }
float or_scene_total_area(const or_scene* s) { return s->total_area; }
int or_scene_cdf(const or_scene* s, float* cdf, float* pick, float* area) {
    for (uint32_t e = 0; e < s->n_emis; ++e) { cdf[e] = s->cdf[e]; pick[e] = s->pick_pdf[e]; area[e] = s->area[e]; }
    return 0;
}
/* closest-hit / any-hit probes (ray batches) for traversal parity tests */
int or_trace_closest(const or_scene* s, int n, const float* o, const float* d, float tnear, float tfar,
                     float* t_out, int32_t* prim_out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        or_hit h = closest_hit(s, V(o[3 * i], o[3 * i + 1], o[3 * i + 2]), V(d[3 * i], d[3 * i + 1], d[3 * i + 2]), tnear, tfar);
        t_out[i] = h.hit ? h.t : -1.0f; prim_out[i] = h.hit ? (int32_t)h.prim : -1;
    }
    return 0;
}
int or_trace_any(const or_scene* s, int n, const float* o, const float* d, const float* tnear, const float* tfar, int32_t* hit_out) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i)
        hit_out[i] = any_hit(s, V(o[3 * i], o[3 * i + 1], o[3 * i + 2]), V(d[3 * i], d[3 * i + 1], d[3 * i + 2]), tnear[i], tfar[i]);
    return 0;
}
int or_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
void or_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* ------------------------------------------------------------------ post-frame */
/* The producer loop's per-frame post block (pg/simpleguidx11.cpp:246-333):
 *   accumulator = glm::mix(accumulator, frame, 1/(accFrameCtr+1))          (:246-253; glm
 *                 compute_mix_scalar: x*(1-a) + y*a)
 *   pix = accumulator; if tonemap: Utils::aces (pg/utils.cpp:191-198); if gammaCorrect:
 *   Utils::compress per channel (pg/utils.cpp:219-229, the float compared with the double 0.0031308);
 *   display = vec4(pix, 1)                                                    (:266-294; denoise off)
 *   mean / variance of the accumulator's per-pixel channel mean, float mean, double sums (:304-327).
 * Rows [y0, y1) of a W-wide image; `sum` / `sqr_sum` return the double sums over those rows. */
static inline float post_aces(float x) {
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    float v = (x * (a * x + b)) / (x * (c * x + d) + e);
    return gmin(gmax(v, 0.0f), 1.0f);          /* glm::clamp = min(max(x, lo), hi), select forms */
}
static inline float post_compress(float u) {
    if (u <= 0.0f) return 0.0f;
    if (u >= 1.0f) return 1.0f;
    if ((double)u <= 0.0031308) return u * 12.92f;
    return 1.055f * rs_powf(u, 1.0f / 2.4f) - 0.055f;
}
void or_post_apply(int W, int y0, int y1, const float* frame, float* acc, int acc_frames, int tonemap,
                   int gamma_correct, float* display_rgba, double* sum, double* sqr_sum) {
    const float a = 1.0f / (float)(acc_frames + 1);
    double s = 0.0, q = 0.0;
    for (int y = y0; y < y1; ++y) {
        for (int x = 0; x < W; ++x) {
            size_t p = (size_t)y * W + x;
            float px[3];
            for (int k = 0; k < 3; ++k) {
                float m = acc[3 * p + k] * (1.0f - a) + frame[3 * p + k] * a;
                acc[3 * p + k] = m;
                float v = m;
                if (tonemap) v = post_aces(v);
                if (gamma_correct) v = post_compress(v);
                px[k] = v;
            }
            if (display_rgba) {
                display_rgba[4 * p] = px[0]; display_rgba[4 * p + 1] = px[1];
                display_rgba[4 * p + 2] = px[2]; display_rgba[4 * p + 3] = 1.0f;
            }
            float mean = (acc[3 * p] + acc[3 * p + 1] + acc[3 * p + 2]) / 3.0f;
            s += mean;
            q += (double)(mean * mean);
        }
    }
    if (sum) *sum = s;
    if (sqr_sum) *sqr_sum = q;
}

/* ------------------------------------------------------------------ golden-vector hooks (tests only) */
/* Reference header-only code compiled by oracle/kat/gen_refheaders.cpp (tests/golden/refheaders_kat.json)
 * replays recorded U streams; these hooks run the oracle's own functions over the same streams. */
/* a sequence of addSample(sample_i, w[i], conf[i]) then capConfidence(cap) (pg/Reservoir.h:33-56):
 * out_i = {chosen sample index or -1, draws consumed, confidence before cap, after cap, hasSample,
 * bestSample.isValid}; *out_wsum = w_sum; taken[i] = 1 where addSample returned true */
void or_kat_reservoir(const float* w, const int32_t* conf, int n, const float* u, int nu, int cap,
                      float* out_wsum, int32_t* out_i, int32_t* taken) {
    or_res r = res_empty();
    int used = 0;
    for (int i = 0; i < n; ++i) {
        sample_t s = {V((float)i, 0.5f, -0.5f), V(0.0f, 0.0f, 1.0f), V(1.0f, 2.0f, 3.0f)};
        taken[i] = 0;
        if (res_update(&r, w[i], conf[i])) taken[i] = res_take(&r, s, w[i], u[used++ % nu]);
    }
    out_i[0] = r.p.x == -FLT_MAX ? -1 : (int)r.p.x;
    out_i[1] = used;
    out_i[2] = r.conf;
    res_cap(&r, cap);
    out_i[3] = r.conf;
    out_i[4] = r.wsum > 0.0f;                  /* Reservoir::hasSample (pg/Reservoir.h:49-52) */
    out_i[5] = sample_valid(&r);
    *out_wsum = r.wsum;
}
int or_kat_light_sample_valid(const float* p, const float* n, const float* li) {
    or_res r = res_empty();
    r.p = V(p[0], p[1], p[2]); r.n = V(n[0], n[1], n[2]); r.li = V(li[0], li[1], li[2]);
    return sample_valid(&r);
}
/* CosineWeightedDistribution::sample / getPdf with draws (r1, r2) (pg/Distribution.h:10-35) */
void or_kat_cosine(const float* n, float r1, float r2, const float* other, float* out5) {
    v3 N = V(n[0], n[1], n[2]);
    v3 wi = cosine_sample_u(N, r1, r2);
    out5[0] = wi.x; out5[1] = wi.y; out5[2] = wi.z;
    out5[3] = cosine_pdf(N, wi);
    out5[4] = cosine_pdf(N, V(other[0], other[1], other[2]));
}
/* CosineLobeDistribution::sample / getPdf (pg/Distribution.h:43-67) */
void or_kat_lobe(const float* wr, float gamma, float r1, float r2, const float* other, float* out5) {
    v3 R = V(wr[0], wr[1], wr[2]);
    v3 wi = lobe_sample_u(R, gamma, r1, r2);
    out5[0] = wi.x; out5[1] = wi.y; out5[2] = wi.z;
    out5[3] = lobe_pdf(wi, R, gamma);
    out5[4] = lobe_pdf(V(other[0], other[1], other[2]), R, gamma);
}
float or_kat_power_heuristic(float a, float b) { return mis_power(a, b); }
float or_kat_max_component(const float* v) { return maxc(V(v[0], v[1], v[2])); }
/* ReSTIRIntegrator::m_area(pa, pb) / m_brdf(pb, pa) (pg/ReSTIRIntegrator.h:62-74) at M_Area = A, M_Brdf = B */
void or_kat_mis(int A, int B, float pa, float pb, float* out2) {
    or_params P;
    memset(&P, 0, sizeof P);
    P.m_area = A; P.m_brdf = B;
    out2[0] = m_area(&P, pa, pb);
    out2[1] = m_brdf(&P, pb, pa);
}
uint64_t or_ctx_rebuilt(const or_ctx* c) { return c->rebuilt; }
uint64_t or_ctx_ref_rays(const or_ctx* c) { return c->ref_rays; }
