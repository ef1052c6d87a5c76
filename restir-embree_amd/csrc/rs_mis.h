// rs_mis.h -- MIS direct-light ground truth: converged references for bias/variance
// checks of the ReSTIR output.
//
// SimpleGuiDX11::produceStandard (pg/simpleguidx11.cpp:336-357) with Raytracer::get_pixel
// (pg/raytracer.cpp:40-45) and NEEPathIntegrator::integrateImpl2 (pg/NEEPathIntegrator.cpp:72-131) at
// calcDI = on, calcGI = off (direct illumination: the quantity ReSTIR DI estimates), with
// DirectMISIntegrator as the direct integrator (pg/DirectMISIntegrator.cpp:10-143): per sample one
// BRDF-sampled ray, then one light sample with its shadow ray, power heuristic.  Material calls are the
// HitInfo variants: MaterialLambert (pg/MaterialLambert.cpp:10-31), MaterialPhong
// (pg/MaterialPhong.cpp:18-119); Phong for PHONG/DIELECTRIC, Lambert for the other types (the ReSTIR
// path's BRDF model, pg/ReSTIRIntegrator.h:32-41, so both converge to the same image).  Pixel-corner
// primary ray (CenterSampler), computed once per pixel; spp samples per launch averaged (sum / spp);
// frames are accumulated by rs_post_frame (the reference's running mean).  RNG: pass kPassMis, draws
// sequential per pixel over the samples.  Restated in oracle/restir_oracle.c or_render_direct_mis.
#pragma once
#include "rs_passes.h"

namespace rs {

constexpr uint32_t kPassMis = 64u;

struct MisSurf { vec3 pos, n, wr, kd, ks; float shin, i_m, maxD, maxS, pf; bool phong; };

// DirectMISIntegrator::powerHeuristic (pg/DirectMISIntegrator.cpp:10-15)
__device__ __forceinline__ float mis_power(float pdf, float other) {
    float a = pdf * pdf, b = other * other;
    return a / (b + a);
}
__device__ __forceinline__ vec3 dvs(vec3 v, float s) { return mk(v.x / s, v.y / s, v.z / s); }   // glm vec3 / scalar
__device__ __forceinline__ float cos_pdf(vec3 n, vec3 wi) { return gmax(dot(n, wi), 0.0f) * kOneOverPi; }
__device__ __forceinline__ float lobe_pdf(vec3 wi, vec3 wr, float g) {      // pg/Distribution.h:65-67
    return (g + 1.0f) * kOneOver2Pi * rs_powf(gmax(0.0f, dot(wi, wr)), g);
}
// getPdfForSample (pg/MaterialLambert.cpp:20-23, pg/MaterialPhong.cpp:94-119)
__device__ __forceinline__ float mis_pdf_for(const MisSurf& h, vec3 wi) {
    if (!h.phong) return cos_pdf(h.n, wi);
    float pdf = cos_pdf(h.n, wi) * h.pf;
    pdf += lobe_pdf(wi, h.wr, h.shin) * (1.0f - h.pf);
    return pdf;
}
// evaluateBRDF (pg/MaterialLambert.cpp:25-31, pg/MaterialPhong.cpp:69-92)
__device__ __forceinline__ vec3 mis_brdf(const MisSurf& h, vec3 wi) {
    vec3 f = h.kd * kOneOverPi;
    if (!h.phong) return f;
    return f + (h.ks * h.i_m) * rs_powf(gmax(dot(wi, h.wr), 0.0f), h.shin);
}
// evaluateLightingGI (pg/MaterialLambert.cpp:10-18, pg/MaterialPhong.cpp:18-67)
__device__ __forceinline__ vec3 mis_sample(const MisSurf& h, Rng& rng, vec3& f_r, float& pdf) {
    if (!h.phong) {
        vec3 wi = cosine_sample(h.n, rng);
        pdf = cos_pdf(h.n, wi);
        f_r = dvs(h.kd, kPi);
        return wi;
    }
    float r0 = rng.range(0.0f, h.maxD + h.maxS);
    vec3 wi;
    if (r0 < h.maxD) {
        wi = cosine_sample(h.n, rng);
        f_r = h.kd * kOneOverPi;
    } else {
        wi = lobe_sample(h.wr, h.shin, rng);
        f_r = (h.ks * h.i_m) * rs_powf(gmax(dot(wi, h.wr), 0.0f), h.shin);
    }
    float pd = cos_pdf(h.n, wi) * h.pf;
    float ps = lobe_pdf(wi, h.wr, h.shin) * (1.0f - h.pf);
    pdf = pd + ps;
    if (dot(h.n, wi) < 0) f_r = mk(0, 0, 0);
    return wi;
}

// DirectMISIntegrator::evaluateBRDFSample (pg/DirectMISIntegrator.cpp:94-144).  BRDF rays are
// incoherent: per-lane walk (as brdf_sample in the ReSTIR passes).
template <int T>
__device__ __forceinline__ vec3 mis_brdf_part(const DevScene& S, const FrameConst& F, const MisSurf& h, bool alive,
                                              Rng& rng, uint32_t& rays) {
    vec3 f_r;
    float pdf;
    vec3 wi = mis_sample(h, rng, f_r, pdf);
    rays += alive ? 1u : 0u;
    SurfHit b = intersect<T | TRAV_LANE>(S, alive, h.pos + h.n * F.normal_off, wi, FLT_MIN + F.tnear_off);
    if (!b.hit) return mk(0, 0, 0);
    MatRec m = load_mat(S, b.mat);
    if (!(m.le.x + m.le.y + m.le.z > 0)) return mk(0, 0, 0);      // Material::isEmissive
    vec3 bn = b.normal;
    if (S.texd) apply_maps(S, b, m, bn, true);
    vec3 ld = b.point - h.pos;
    float r2 = dot(ld, ld);
    ld = normalize(ld);
    float cI = gmax(dot(ld, h.n), 0.0f);
    float cY = gmax(dot(-ld, bn), 0.0f);
    float amf = cY / r2;
    float pdf_light = emis_pdf_brdf(S, b.emis_id);                 // TriangleCDF::getPDFForTriangle
    float w = mis_power(pdf * amf, pdf_light);
    return dvs(((m.le * w) * f_r) * cI, pdf);
}

// DirectMISIntegrator::evaluateLightSample (pg/DirectMISIntegrator.cpp:38-92)
template <int T>
__device__ __forceinline__ vec3 mis_light_part(const DevScene& S, const FrameConst& F, const MisSurf& h, bool alive,
                                               Rng& rng, uint32_t& rays) {
    if (S.n_emis == 0) return mk(0, 0, 0);                          // TriangleCDF::isValid (uniform)
    float ksi = rng.range(0.0f, 1.0f);                              // TriangleCDF::getTriangle
    const uint32_t idx = light_index(S, ksi);
    const EmisRec E = EmisRec::load(S.emis + 8 * idx);
    float r1 = rng.range(0, 1), r2 = rng.range(0, 1);                // Sampling::sampleTriangle
    float sr = sqrtf(r1);
    float bx = 1.0f - sr, by = sr * (1.0f - r2), bz = sr * r2;
    vec3 pt = (E.p0 * bx + E.p1 * by) + E.p2 * bz;
    vec3 nn = normalize((E.n0 * bx + E.n1 * by) + E.n2 * bz);
    float light_pdf = E.pdf_area;                                    // pick prob * (1 / area)
    vec3 ld = pt - h.pos;
    float r_sqr = dot(ld, ld);
    ld = normalize(ld);
    float cI = gmax(dot(ld, h.n), 0.0f);
    float cY = gmax(dot(-ld, nn), 0.0f);
    float amf = cY / r_sqr;
    const bool ok = alive && light_pdf != 0.0f && r_sqr != 0.0f && cI > 0 && cY > 0;
    const bool occ = occluded<T>(S, F, ok, h.pos, pt, rays);
    if (!ok || occ) return mk(0, 0, 0);
    float pba = mis_pdf_for(h, ld) * amf;
    float w = mis_power(light_pdf, pba);
    if (!(w > 0.0f)) return mk(0, 0, 0);
    float G = cI * cY / r_sqr;
    return dvs(((E.le * w) * mis_brdf(h, ld)) * G, light_pdf);
}

template <int T>
__global__ void __launch_bounds__(256) k_direct_mis(DevScene S, FrameConst F, int spp, float* fb, CountSlot C) {
    int x, y;
    const bool in = pixel_of(F, F.y0, F.y1, x, y);
    const uint64_t t0 = wave_clock();
    const uint32_t pix = (uint32_t)y * (uint32_t)F.W + (uint32_t)x;
    uint32_t rays = in ? 1u : 0u;
    vec3 dc = mk((float)x - (float)F.W / 2.0f, (float)F.H / 2.0f - (float)y, -F.cam.focal);
    const float* m = F.inv_view;
    vec3 d = normalize(mk(m[0] * dc.x + m[3] * dc.y + m[6] * dc.z, m[1] * dc.x + m[4] * dc.y + m[7] * dc.z,
                          m[2] * dc.x + m[5] * dc.y + m[8] * dc.z));
    SurfHit hi = intersect<T>(S, in, F.cam.pos, d, FLT_MIN + 0.01f);
    MatRec mr = load_mat(S, hi.mat);
    vec3 hn = hi.normal;
    if (S.texd && hi.hit) apply_maps(S, hi, mr, hn, false);
    const bool surf = in && hi.hit && !any_pos(mr.le);               // Material::isEmitter: camera vertex -> Le
    vec3 px = hi.hit ? mr.le : (F.use_sky ? sky_texel(S, d) : F.bg);  // miss: sky or bgColor (:131)
    MisSurf h;
    h.pos = hi.point; h.n = hn; h.kd = mr.kd; h.ks = mr.ks; h.shin = mr.shin;
    h.phong = is_phong(mr.type);
    h.maxD = maxc(h.kd); h.maxS = maxc(h.ks);
    h.pf = h.maxD / (h.maxD + h.maxS);
    h.wr = normalize(reflect(d, h.n));
    h.i_m = (surf && h.phong) ? 1.0f / calc_I_M(dot(-d, h.n), h.shin) : 0.0f;
    Rng rng; rng.init(F.seed, F.frame, kPassMis, pix);
    vec3 acc = mk(0, 0, 0);
    for (int k = 0; k < spp; ++k) {
        vec3 L = mk(0, 0, 0) + mis_brdf_part<T>(S, F, h, surf, rng, rays);
        L = L + mis_light_part<T>(S, F, h, surf, rng, rays);
        acc = acc + (mk(0, 0, 0) + sanitize(L));                    // L_i_indirect (0) + L_i_direct
    }
    if (surf) px = dvs(acc, (float)spp);
    px = sanitize(px);
    if (in) store_rgb(fb, pix, px);
    count_rays(C, rays, in ? 1u : 0u, t0, y);
}

}  // namespace rs
