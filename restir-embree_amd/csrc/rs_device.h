// rs_device.h -- per-pixel maths of the ReSTIR DI path for gfx950 (device side).
//
// Every function states the reference code it follows (pg/ = template/src/pg/pg1_embree/).  The
// arithmetic keeps glm 0.9.9's operation order (the reference's maths library) and the file is
// compiled with -ffp-contract=off so results match the CPU restatement to the last bit (sqrt and division are
// correctly rounded on both sides; sin/cos/pow/exp/lgamma and the double log/exp/log1p/lgamma of the incomplete
// beta are rs_libm.h's fixed operation sequences, shared with the oracle, instead of ocml / glibc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <float.h>
#include "rs_libm.h"

namespace rs {

constexpr float kPi = 3.14159265358979323846264338327950288f;          // glm::pi<float>()
constexpr float kOneOverPi = 0.318309886183790671537767526745028724f;  // glm::one_over_pi
constexpr float kOneOver2Pi = 0.159154943091895335768883763372514362f; // glm::one_over_two_pi
constexpr float kTwoPi = 6.28318530717958647692528676655900576f;        // glm::two_pi
constexpr float kRootPi = 1.772453850905516027f;                        // glm::root_pi

// MaterialType (pg/enums.h:3-11)
enum : int { MT_NORMAL = 0, MT_LAMBERT = 1, MT_PHONG = 2, MT_MIRROR = 3, MT_DIELECTRIC = 4 };
// SpatialWeightCalculation (pg/ReSTIRIntegrator.h:19-25)
enum : int { MIS_CONSTANT = 0, MIS_DEBIAS_CONTRIB = 1, MIS_DEBIAS_Z = 2, MIS_BALANCE = 3, MIS_PAIRWISE = 4 };
// counter-RNG pass keys (shared with the oracle's definition)
enum : uint32_t { PASS_INITIAL = 1, PASS_TEMPORAL = 2, PASS_SPATIAL0 = 3 };

struct vec3 { float x, y, z; };
__device__ __forceinline__ vec3 mk(float x, float y, float z) { return vec3{x, y, z}; }
__device__ __forceinline__ vec3 operator+(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ vec3 operator-(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ vec3 operator*(vec3 a, vec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ vec3 operator*(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ vec3 operator-(vec3 a) { return {-a.x, -a.y, -a.z}; }
// glm compute_dot<vec3>: (a*b).x + (a*b).y + (a*b).z
__device__ __forceinline__ float dot(vec3 a, vec3 b) { vec3 t = a * b; return t.x + t.y + t.z; }
// glm compute_cross
__device__ __forceinline__ vec3 cross(vec3 x, vec3 y) {
    return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
__device__ __forceinline__ float length(vec3 a) { return sqrtf(dot(a, a)); }
// glm normalize = v * (1 / sqrt(dot(v, v)))
__device__ __forceinline__ vec3 normalize(vec3 a) { return a * (1.0f / sqrtf(dot(a, a))); }
// glm reflect: I - N * dot(N, I) * 2
__device__ __forceinline__ vec3 reflect(vec3 I, vec3 N) { return I - (N * dot(N, I)) * 2.0f; }
// glm scalar max/min: select form (NaN propagation as in the reference)
__device__ __forceinline__ float gmax(float x, float y) { return (x < y) ? y : x; }
__device__ __forceinline__ float gmin(float x, float y) { return (y < x) ? y : x; }
__device__ __forceinline__ float maxc(vec3 a) { return gmax(gmax(a.x, a.y), a.z); }      // pg/utils.h:61-63
__device__ __forceinline__ bool any_pos(vec3 e) { return e.x > 0 || e.y > 0 || e.z > 0; }
__device__ __forceinline__ vec3 xyz(float4 v) { return {v.x, v.y, v.z}; }
__device__ __forceinline__ float4 f4(vec3 v, float w) { return make_float4(v.x, v.y, v.z, w); }

// ---------------------------------------------------------------- counter RNG
// Replaces Utils::getRandomValue's shared mt19937 (pg/utils.cpp:175-176,199-202): one independent
// stream per (seed, frame, pass, full-frame pixel), consumed in the reference's per-pixel order.
__device__ __forceinline__ uint32_t hash32(uint32_t x) {   // lowbias32
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
struct Rng {
    uint32_t key, n;
    __device__ __forceinline__ void init(uint32_t seed, uint32_t frame, uint32_t pass, uint32_t pixel) {
        uint32_t k = hash32(seed ^ 0x6a09e667u);
        k = hash32(k ^ frame);
        k = hash32(k + 0x9e3779b9u * (pass + 1u));
        key = hash32(k ^ pixel);
        n = 0;
    }
    __device__ __forceinline__ float at(uint32_t i) const {
        uint32_t x = hash32(key ^ hash32(i + 0x632be5abu));
        return (float)(x >> 8) * (1.0f / 16777216.0f);
    }
    __device__ __forceinline__ float u() { return at(n++); }
    // Utils::getRandomValue(a, b) = a + (b - a) * U
    __device__ __forceinline__ float range(float a, float b) { float v = u(); return a + (b - a) * v; }
};

// ---------------------------------------------------------------- incomplete beta (double)
// boost::math::beta(a, b, x) non-normalised (pg/MaterialPhong.cpp:246-248): Lentz continued fraction.
__device__ inline double betacf(double a, double b, double x) {
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
__device__ inline double ibeta_d(double x, double a, double b) {
    if (!(x > 0.0)) return 0.0;
    double lbeta = rs_lgamma_d(a) + rs_lgamma_d(b) - rs_lgamma_d(a + b);
    if (x >= 1.0) return rs_exp_d(lbeta);
    double lbt = a * rs_log_d(x) + b * rs_log1p_d(-x);
    if (x < (a + 1.0) / (a + b + 2.0)) return rs_exp_d(lbt) * betacf(a, b, x) / a;
    return rs_exp_d(lbeta) - rs_exp_d(lbt) * betacf(b, a, 1.0 - x) / b;
}
// MaterialPhong::calc_I_M (pg/MaterialPhong.cpp:224-244); gamma_quot in float as in the reference.
__device__ inline float calc_I_M(float nDotV, float n) {
    float costerm = nDotV;
    float sinterm_sq = 1.0f - costerm * costerm;
    float halfn = 0.5f * n;
    float negterm = costerm;
    sinterm_sq = gmin(gmax(sinterm_sq, 0.0f), 1.0f);
    if (n >= 1e-18f) negterm *= halfn * (float)ibeta_d((double)sinterm_sq, (double)halfn, 0.5);
    float gq = rs_expf(rs_lgammaf(halfn + 0.5f) - rs_lgammaf(halfn + 1.0f));
    return (kTwoPi * costerm + kRootPi * gq * (rs_powf(sinterm_sq, halfn) - negterm)) / (n + 2.0f);
}

// ---------------------------------------------------------------- G-buffer element
// GBufferElement (pg/GBufferElement.h:6-17) + the per-pixel 1/I_M (depends only on n.v and
// shininess, both fixed per pixel and frame) so p-hat never re-runs the incomplete beta.
struct GElem {
    vec3 pos; float depth;
    vec3 nrm; float shin;
    vec3 kd; float inv_im;
    vec3 ks; int type;
    vec3 le;
};
struct GBuf {   // SoA of float4: g0 (pos,depth) g1 (nrm,shin) g2 (kd,1/I_M) g3 (ks,type) g4 (le,0)
    float4* g0; float4* g1; float4* g2; float4* g3; float4* g4;
    __device__ __forceinline__ GElem load(size_t p) const {
        float4 a = g0[p], b = g1[p], c = g2[p], d = g3[p], e = g4[p];
        GElem g;
        g.pos = xyz(a); g.depth = a.w; g.nrm = xyz(b); g.shin = b.w; g.kd = xyz(c); g.inv_im = c.w;
        g.ks = xyz(d); g.type = __float_as_int(d.w); g.le = xyz(e);
        return g;
    }
    __device__ __forceinline__ void store(size_t p, const GElem& g) const {
        g0[p] = f4(g.pos, g.depth); g1[p] = f4(g.nrm, g.shin); g2[p] = f4(g.kd, g.inv_im);
        g3[p] = f4(g.ks, __int_as_float(g.type)); g4[p] = f4(g.le, 0.0f);
    }
    __device__ __forceinline__ vec3 le(size_t p) const { return xyz(g4[p]); }
    __device__ __forceinline__ vec3 pos(size_t p) const { return xyz(g0[p]); }
};
struct GCam { vec3 pos; float focal; float view[16]; };   // camera of the frame the G-buffer belongs to

// ---------------------------------------------------------------- reservoir (48 B, AoS)
// Reservoir + LightSample (pg/Reservoir.h:6-59): a = (point, w_sum), b = (normal, W), c = (L_i, conf)
struct Res {
    vec3 p, n, li; float wsum, W; int conf;
};
struct ResBuf {
    float4* r;   // 3 float4 per pixel
    __device__ __forceinline__ Res load(size_t p) const {
        float4 a = r[3 * p], b = r[3 * p + 1], c = r[3 * p + 2];
        return Res{xyz(a), xyz(b), xyz(c), a.w, b.w, __float_as_int(c.w)};
    }
    __device__ __forceinline__ void store(size_t p, const Res& s) const {
        r[3 * p] = f4(s.p, s.wsum); r[3 * p + 1] = f4(s.n, s.W); r[3 * p + 2] = f4(s.li, __int_as_float(s.conf));
    }
};
__device__ __forceinline__ Res res_empty() {
    Res r; r.p = mk(-FLT_MAX, -FLT_MAX, -FLT_MAX); r.n = r.p; r.li = r.p; r.wsum = 0; r.W = 0; r.conf = 0;
    return r;
}
struct Sample { vec3 p, n, li; };
__device__ __forceinline__ Sample smp_invalid() { Sample s; s.p = mk(-FLT_MAX, -FLT_MAX, -FLT_MAX); s.n = s.p; s.li = s.p; return s; }
__device__ __forceinline__ Sample smp_of(const Res& r) { return Sample{r.p, r.n, r.li}; }
// LightSample::isValid (pg/Reservoir.h:11-17)
__device__ __forceinline__ bool smp_valid(const Sample& s) {
    bool pok = s.p.x != -FLT_MAX && s.p.y != -FLT_MAX && s.p.z != -FLT_MAX;
    bool nok = s.n.x != -FLT_MAX && s.n.y != -FLT_MAX && s.n.z != -FLT_MAX;
    bool lok = s.li.x > 0 || s.li.y > 0 || s.li.z > 0;
    return pok && nok && lok;
}
// Reservoir::addSample (pg/Reservoir.h:33-47)
// the update without the sample copy: returns whether the new sample is selected
__device__ __forceinline__ bool res_add_w(Res& r, float w, int conf, Rng& rng) {
    r.wsum += w;
    r.conf += conf;
    if (w == 0 && r.wsum == 0) return false;
    return rng.u() < w / r.wsum;
}
__device__ __forceinline__ bool res_add(Res& r, const Sample& s, float w, int conf, Rng& rng) {
    if (!res_add_w(r, w, conf, rng)) return false;
    r.p = s.p; r.n = s.n; r.li = s.li;
    return true;
}
// Initial-pass draw slots (oracle/restir_oracle.c cand_slot): candidate c owns draws 4c..4c+3 --
// up to 3 for its sample, 4c+3 for its reservoir update -- independent of other candidates' outcome.
__device__ __forceinline__ uint32_t cand_slot(int c) { return 4u * (uint32_t)c; }
__device__ __forceinline__ void res_cap(Res& r, int cap) { r.conf = r.conf < cap ? r.conf : cap; }

// ---------------------------------------------------------------- BRDF statics
// The per-pixel invariants of every BRDF evaluation / pdf / sample at a G element seen from `cam`,
// computed once (each in the reference's operation order).  The Phong eval's mirror direction
// normalize(reflect(-normalize(cam - p), n)) and the pdf's normalize(reflect(normalize(p - cam), n))
// are the same bits (p - cam = -(cam - p) exactly; normalize commutes with negation), so one wr.
struct ShadeFrame {
    vec3 nrm; float pf;        // pf = maxD / (maxD + maxS)             (pg/MaterialPhong.cpp:152-154)
    vec3 wr; float omp;        // mirror direction; omp = 1 - pf
    vec3 kd_pi; float shin;    // kd * 1/pi                             (pg/MaterialLambert.cpp:33-41)
    vec3 ks_im; float a;       // ks * 1/I_M;  a = (shin + 1) * 1/(2 pi)  (pg/MaterialPhong.cpp:122-172)
    float maxD, maxS; int type;
};
__device__ __forceinline__ ShadeFrame make_frame(const GElem& g, vec3 cam) {
    ShadeFrame s;
    s.maxD = maxc(g.kd); s.maxS = maxc(g.ks);
    s.pf = s.maxD / (s.maxD + s.maxS);
    s.omp = 1.0f - s.pf;
    s.nrm = g.nrm;
    vec3 wo = normalize(g.pos - cam);
    s.wr = normalize(reflect(wo, g.nrm));
    s.kd_pi = g.kd * kOneOverPi;
    s.ks_im = g.ks * g.inv_im;
    s.shin = g.shin;
    s.a = (g.shin + 1.0f) * kOneOver2Pi;
    s.type = g.type;
    return s;
}
__device__ __forceinline__ bool is_phong(int type) { return type == MT_PHONG || type == MT_DIELECTRIC; }
// MaterialPhong::evalPdf -- the MIS pdf is always Phong's (pg/ReSTIRIntegrator.h:54-59,
// pg/MaterialPhong.cpp:150-172)
// Lambert surfaces (ks = 0: omp = 0) add the lobe term a * pow(..) * 0 = +0 exactly (a finite, the pow in
// [0, 1]), so the powf is skipped for them -- the MIS pdf of every area candidate on a diffuse wall
// (Call: the pow's core as a called function, rs_libm.h rs_powf_sel -- for the register-bound per-lane kernels)
template <bool Call = false>
__device__ __forceinline__ float phong_pdf(const ShadeFrame& s, vec3 wi) {
    float pdf = gmax(dot(s.nrm, wi), 0.0f) * kOneOverPi * s.pf;
    pdf += (s.omp != 0.0f || !isfinite(s.a)) ? s.a * rs_powf_sel(gmax(0.0f, dot(wi, s.wr)), s.shin, Call) * s.omp : 0.0f;
    return pdf;
}
// BRDF eval dispatch (pg/ReSTIRIntegrator.h:32-41): Phong for PHONG/DIELECTRIC
// (pg/MaterialPhong.cpp:122-148, with the cached 1/I_M), Lambert otherwise (pg/MaterialLambert.cpp:33-41)
template <bool Call = false>
__device__ __forceinline__ vec3 eval_brdf(const ShadeFrame& s, vec3 wi) {
    vec3 f = s.kd_pi;
    if (!is_phong(s.type)) return f;
    float pw = rs_powf_sel(gmax(dot(wi, s.wr), 0.0f), s.shin, Call);
    return f + s.ks_im * pw;
}
__device__ __forceinline__ float phong_pdf(const GElem& g, vec3 cam, vec3 wi) { return phong_pdf(make_frame(g, cam), wi); }
__device__ __forceinline__ vec3 eval_brdf(const GElem& g, vec3 cam, vec3 wi) { return eval_brdf(make_frame(g, cam), wi); }

// Utils::orthogonal (pg/utils.cpp:204-207) + the ONB of pg/Distribution.h:15-24
__device__ __forceinline__ vec3 to_world(vec3 s, vec3 n) {
    vec3 o = fabsf(n.x) > fabsf(n.z) ? mk(n.y, -n.x, 0.0f) : mk(0.0f, n.z, -n.y);
    vec3 o2 = normalize(o);
    vec3 o1 = normalize(cross(n, o2));
    o2 = normalize(cross(o1, n));
    return mk(o1.x * s.x + o2.x * s.y + n.x * s.z, o1.y * s.x + o2.y * s.y + n.y * s.z,
              o1.z * s.x + o2.z * s.y + n.z * s.z);
}
// CosineWeightedDistribution::sample (pg/Distribution.h:7-28)
__device__ __forceinline__ vec3 cosine_sample(vec3 n, Rng& rng) {
    float r1 = rng.range(0, 1), r2 = rng.range(0, 1);
    float ang = kPi * 2.0f * r1;
    float sq = sqrtf(1.0f - r2);
    float sn, cs;
    rs_sincosf(ang, &sn, &cs);
    float x = cs * sq, y = sn * sq, z = sqrtf(r2);
    return to_world(normalize(mk(x, y, z)), n);
}
// CosineLobeDistribution::sample (pg/Distribution.h:37-57)
__device__ __forceinline__ vec3 lobe_sample(vec3 wr, float gamma, Rng& rng) {
    float r1 = rng.range(0, 1), r2 = rng.range(0, 1);
    float ang = 2.0f * kPi * r1;
    float sq = sqrtf(1.0f - rs_powf(r2, 2.0f / (gamma + 1.0f)));
    float sn, cs;
    rs_sincosf(ang, &sn, &cs);
    float x = cs * sq, y = sn * sq;
    float z = rs_powf(r2, 1.0f / (gamma + 1.0f));
    return to_world(normalize(mk(x, y, z)), wr);
}
// BRDF sampling dispatch (pg/ReSTIRIntegrator.h:43-52): Lambert (pg/MaterialLambert.cpp:43-53) or
// Phong (pg/MaterialPhong.cpp:174-222; also DIELECTRIC and every other type).  Returns omega_i, pdf.
__device__ __forceinline__ vec3 sample_brdf(const ShadeFrame& s, Rng& rng, float& pdf) {
    if (s.type == MT_LAMBERT) {
        vec3 wi = cosine_sample(s.nrm, rng);
        pdf = gmax(dot(s.nrm, wi), 0.0f) * kOneOverPi;
        return wi;
    }
    float r0 = rng.range(0.0f, s.maxD + s.maxS);
    vec3 wi = (r0 < s.maxD) ? cosine_sample(s.nrm, rng) : lobe_sample(s.wr, s.shin, rng);
    float pd = gmax(dot(s.nrm, wi), 0.0f) * kOneOverPi * s.pf;
    float ps = s.a * rs_powf(gmax(0.0f, dot(wi, s.wr)), s.shin) * s.omp;
    pdf = pd + ps;
    return wi;
}

// Integrator::sanitize (pg/Integrator.cpp:6-22)
__device__ __forceinline__ vec3 sanitize(vec3 l) {
    if (isnan(l.x) || isnan(l.y) || isnan(l.z)) l = mk(0, 0, 0);
    if (l.x < 0 || l.y < 0 || l.z < 0) l = mk(0, 0, 0);
    return l;
}

}  // namespace rs
