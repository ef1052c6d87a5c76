// rs_texture.h -- material textures and the equirectangular sky.
//
// Device layout (restir_capi.hip upload_textures): every texture's texels live in one byte buffer in
// the layout FreeImage_ConvertToRawBits gives the reference (pg/Texture.cpp:46-50): top row first,
// rows padded to 4 bytes (FreeImage_GetPitch), 8-bit texels in B,G,R(,A) byte order, float texels as
// R,G,B(,A) floats.  8-bit diffuse/specular maps are sRGB-expanded at upload (Texture::expand,
// pg/Texture.cpp:141-160).  Descriptor: (byte offset, width, height, pitch), (pixel bytes, format, 0, 0).
//
// Lookups restate Texture::get_texel / getTexelBilinear (pg/Texture.cpp:72-107,170-194) exactly,
// including its quirks: REPEAT wraps with abs(x % w) (negative coordinates mirror), 1-byte texels read
// three consecutive bytes as B,G,R, and v is flipped ((1 - v) * h).
#pragma once
#include "rs_scene.h"

namespace rs {

// Texture::get_texel(int x, int y) (pg/Texture.cpp:72-107)
__device__ __forceinline__ vec3 tex_texel(const DevScene& S, int t, int x, int y, bool repeat) {
    const int4 a = S.texd[2 * t], b = S.texd[2 * t + 1];
    const int w = a.y, h = a.z;
    int cx, cy;
    if (repeat) { cx = abs(x % w); cy = abs(y % h); }
    else { cx = min(max(x, 0), w - 1); cy = min(max(y, 0), h - 1); }   // glm::clamp
    const uint8_t* p = S.tex + (size_t)a.x + (size_t)cy * (size_t)a.w + (size_t)cx * (size_t)b.x;
    if (b.x > 4) {                                                     // HDR / EXR: float texels
        const float* f = reinterpret_cast<const float*>(p);
        return mk(f[0], f[1], f[2]);
    }
    return mk((float)p[2] / 255.0f, (float)p[1] / 255.0f, (float)p[0] / 255.0f);
}

// Texture::getTexelBilinear (pg/Texture.cpp:170-194); glm::mix(x, y, a) = x * (1 - a) + y * a
__device__ __forceinline__ vec3 tex_bilinear(const DevScene& S, int t, float u, float v, bool repeat) {
    const int4 a = S.texd[2 * t];
    const float pxc = u * (float)a.y, pyc = (1.0f - v) * (float)a.z;
    const float fx = floorf(pxc), fy = floorf(pyc);
    const float tx = pxc - fx, ty = pyc - fy;
    const vec3 q00 = tex_texel(S, t, (int)fx, (int)fy, repeat);
    const vec3 q10 = tex_texel(S, t, (int)(fx + 1.0f), (int)fy, repeat);
    const vec3 q01 = tex_texel(S, t, (int)fx, (int)(fy + 1.0f), repeat);
    const vec3 q11 = tex_texel(S, t, (int)(fx + 1.0f), (int)(fy + 1.0f), repeat);
    const vec3 x1 = q00 * (1.0f - tx) + q10 * tx;
    const vec3 x2 = q01 * (1.0f - tx) + q11 * tx;
    return x1 * (1.0f - ty) + x2 * ty;
}

// SphericalMap::getTexel (pg/SphericalMap.cpp:10-14): INVPI = 1.0 / M_PI is a double, so both
// coordinates are finished in double; the sky texture is BILINEAR + CLAMP_TO_EDGE (Texture.h:27)
__device__ __forceinline__ vec3 sky_texel(const DevScene& S, vec3 dir) {
    const double invpi = 1.0 / 3.14159265358979323846;
    const float x = (float)(0.5f + (double)(0.5f * atan2f(dir.y, dir.x)) * invpi);
    const float y = (float)(1.0f - (double)acosf(dir.z) * invpi);
    return tex_bilinear(S, S.sky, x, y, false);
}

// Material::getDiffuseColor / getSpecularColor / getShininess (pg/material.cpp:105-134) at the hit's
// interpolated uv (rtcInterpolate slot 1, pg/Intersection.h:99-100), and the normal map
// (pg/Intersection.h:26-39): N = TBN * (2 t - 1) with T the interpolated tangent (slot 3)
// Gram-Schmidt'ed against the ray-facing normal, B = normalize(cross(n, T)); N is not normalised.
// `normal_only`: hits that only need the shading normal (BRDF-sampled emitter hits).
__device__ __forceinline__ void apply_maps(const DevScene& S, const SurfHit& h, MatRec& m, vec3& n, bool normal_only) {
    const int4 maps = load_maps(S, h.mat);
    if (maps.x < 0 && maps.y < 0 && maps.z < 0 && maps.w < 0) return;
    const float w = 1.0f - h.u - h.v;
    const float4 A = S.tri_uv[2 * h.prim], B = S.tri_uv[2 * h.prim + 1];
    const float u = (A.x * w + A.z * h.u) + B.x * h.v;
    const float v = (A.y * w + A.w * h.u) + B.y * h.v;
    if (!normal_only) {
        if (maps.x >= 0) m.kd = tex_bilinear(S, maps.x, u, v, true);
        if (maps.y >= 0) m.ks = tex_bilinear(S, maps.y, u, v, true);
        if (maps.z >= 0) {
            const vec3 r = tex_bilinear(S, maps.z, u, v, true);
            m.shin = 2.0f / (r.x * r.x) - 2.0f;                        // roughness -> shininess
        }
    }
    if (maps.w >= 0) {
        const float4* Tt = S.tri_tan + 3 * h.prim;
        vec3 T = (xyz(Tt[0]) * w + xyz(Tt[1]) * h.u) + xyz(Tt[2]) * h.v;
        T = T - n * dot(T, n);
        T = normalize(T);
        const vec3 Bn = normalize(cross(n, T));
        const vec3 N = tex_bilinear(S, maps.w, u, v, true) * 2.0f - mk(1.0f, 1.0f, 1.0f);
        n = mk(T.x * N.x + Bn.x * N.y + n.x * N.z, T.y * N.x + Bn.y * N.y + n.y * N.z,
               T.z * N.x + Bn.z * N.y + n.z * N.z);
    }
}

}  // namespace rs
