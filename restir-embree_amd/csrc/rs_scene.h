// rs_scene.h -- device scene layout and BVH traversal (replaces Embree's rtcIntersect1/rtcOccluded1,
// pg/Intersection.h:8-113).
//
// BVH: depth-first ("preorder") node array with skip pointers -- stackless traversal.  Node i is
// 32 B = 2 x float4:  a = (lo.xyz, skip), b = (hi.xyz, leaf)   [skip/leaf as int bits]
//   skip = index of the node following i's subtree (== n_nodes ends traversal)
//   leaf = -1 for an interior node (its first child is i + 1), else (first << 3) | (count - 1)
// Leaf triangles are stored contiguously in leaf order, 48 B each = 3 x float4:
//   (v0.xyz, prim), (e1.xyz, 0), (e2.xyz, 0)   with e1 = v1 - v0, e2 = v2 - v0 (same float ops the
//   CPU restatement does on the fly), prim = original triangle index (int bits).
// Shading attributes are indexed by prim: 3 float4 vertex normals + material/emissive id.
//
// Two traversal kinds, selected per launch as a template parameter (Trav); both return bit-identical
// results (same box/triangle tests, same tie rule), they differ only in how a wave walks the array:
//   TRAV_LOCKSTEP  the wave walks the node array together (coherent rays: C2's shadow/primary rays)
//   TRAV_LANE      every lane walks its own path with vector loads (incoherent rays: C3)
// The context picks the faster kind per scene by timing (restir_capi.hip pick_traversal).
#pragma once
#include "rs_device.h"

namespace rs {

struct DevScene {
    const float4* nodes;      // 2 per node
    const float4* tris;       // 3 per leaf-ordered triangle
    const float4* tri_nrm;    // 3 per prim: n0 (w = material id bits), n1 (w = emissive id bits), n2
    const float4* mats;       // 4 per material: (kd, shin), (ks, type bits), (le, 0), map ids (int bits, -1 none:
                              //   diffuse, specular, shininess, normal)
    const float4* emis;       // 8 per emissive triangle (one 128-B line; layout at EmisRec)
    const float* cdf;         // cumulative normalised area (TriangleCDF::cdf2)
    const int* cdf_guide;     // kCdfGuide+1 entries: lower_bound(cdf, j / kCdfGuide)
    uint32_t n_nodes, n_tris, n_emis, n_mats;
    // textures (rs_texture.h); all null / -1 for untextured scenes
    const float4* tri_uv;     // 2 per prim: (uv0, uv1), (uv2, 0, 0)
    const float4* tri_tan;    // 3 per prim: tangent t0, t1, t2 (normal-mapped scenes only)
    const uint8_t* tex;       // texel bytes of every texture
    const int4* texd;         // 2 per texture: (byte offset, width, height, pitch), (pixel bytes, format, 0, 0)
    int sky;                  // texture index of the equirect sky, -1 none
};
constexpr int kCdfGuide = 1024;

enum Trav : int { TRAV_LOCKSTEP = 0, TRAV_LANE = 1 };

// Moller-Trumbore, fixed op order (identical to oracle/restir_oracle.c tri_hit)
__device__ __forceinline__ bool tri_test(float4 A, float4 B, float4 C, vec3 o, vec3 d, float tnear,
                                         float tfar, float& t_out, float& u_out, float& v_out) {
    vec3 v0 = xyz(A), e1 = xyz(B), e2 = xyz(C);
    vec3 p = cross(d, e2);
    float det = dot(e1, p);
    if (det == 0.0f) return false;
    float inv = 1.0f / det;
    vec3 sv = o - v0;
    float u = dot(sv, p) * inv;
    if (!(u >= 0.0f && u <= 1.0f)) return false;
    vec3 q = cross(sv, e1);
    float v = dot(d, q) * inv;
    if (!(v >= 0.0f && u + v <= 1.0f)) return false;
    float t = dot(e2, q) * inv;
    if (!(t >= tnear && t <= tfar)) return false;
    t_out = t; u_out = u; v_out = v;
    return true;
}

// The same test without early returns (identical arithmetic and acceptance; with det == 0 the
// quotients are inf/NaN and the explicit det check rejects).  Used by the lockstep walks, where the
// triangle is shared by the wave: straight-line VALU instead of three nested exec-mask regions.
__device__ __forceinline__ bool tri_test_nb(float4 A, float4 B, float4 C, vec3 o, vec3 d, float tnear, float tfar,
                                            float& t, float& u, float& v) {
    vec3 v0 = xyz(A), e1 = xyz(B), e2 = xyz(C);
    vec3 p = cross(d, e2);
    float det = dot(e1, p);
    float inv = 1.0f / det;
    vec3 sv = o - v0;
    u = dot(sv, p) * inv;
    vec3 q = cross(sv, e1);
    v = dot(d, q) * inv;
    t = dot(e2, q) * inv;
    const bool ok_u = u >= 0.0f && u <= 1.0f, ok_v = v >= 0.0f && u + v <= 1.0f, ok_t = t >= tnear && t <= tfar;
    return (det != 0.0f) & ok_u & ok_v & ok_t;
}

// conservative slab test (interval widened by 4 ulp-ish so no box the triangle test accepts is culled)
__device__ __forceinline__ bool box_test(float4 a, float4 b, vec3 o, vec3 inv, float tnear, float tfar) {
    float tx0 = (a.x - o.x) * inv.x, tx1 = (b.x - o.x) * inv.x;
    float ty0 = (a.y - o.y) * inv.y, ty1 = (b.y - o.y) * inv.y;
    float tz0 = (a.z - o.z) * inv.z, tz1 = (b.z - o.z) * inv.z;
    float t0 = fmaxf(fmaxf(fmaxf(tnear, fminf(tx0, tx1)), fminf(ty0, ty1)), fminf(tz0, tz1));
    float t1 = fminf(fminf(fminf(tfar, fmaxf(tx0, tx1)), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    return t0 * (1.0f - 4.0f * FLT_EPSILON) <= t1 * (1.0f + 4.0f * FLT_EPSILON);
}

struct Hit { float t, u, v; int prim; };

// uniform-index load through the constant address space -> s_load (scalar cache), no VGPR address
__device__ __forceinline__ float4 sload(const float4* p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const float __attribute__((address_space(4)))* cfloat_ptr;
    cfloat_ptr q = (cfloat_ptr)(const float*)(p + i);
    return make_float4(q[0], q[1], q[2], q[3]);
#else
    return p[i];   // host pass only type-checks device code
#endif
}
// wave-uniform node load for the lockstep walks: scalar cache (default) or, with RS_NODE_VMEM, one
// broadcast vector load through L1 (32 KB/CU) with the control words moved to SGPRs
// (a broadcast vector load through L1 + readfirstlane was measured 10 % slower on C2)
__device__ __forceinline__ void node_load(const float4* nodes, uint32_t m, float4& a, float4& b) {
    a = sload(nodes, 2 * m); b = sload(nodes, 2 * m + 1);
}
template <bool Uniform>
__device__ __forceinline__ float4 ld4(const float4* p, uint32_t i) {
    if (Uniform) return sload(p, i);
    return p[i];
}

// ---------------------------------------------------------------- node visit
// one node of a closest-hit walk (rtcIntersect1; ties: smaller t, then smaller triangle index).  The box
// test culls against the running closest t; with the tie rule applied at every accepted triangle the
// result does not depend on the visit order.
template <bool Uniform>
__device__ __forceinline__ void closest_visit(const DevScene& S, float4 a, float4 b, uint32_t i, vec3 o, vec3 d,
                                              vec3 inv, float tnear, uint32_t& cur, Hit& h) {
    const uint32_t skip = (uint32_t)__float_as_int(a.w);
    if (!box_test(a, b, o, inv, tnear, h.t)) { cur = skip; return; }
    const int leaf = __float_as_int(b.w);
    if (leaf < 0) { cur = i + 1; return; }
    const int first = leaf >> 3, cnt = (leaf & 7) + 1;
    for (int j = 0; j < cnt; ++j) {
        const uint32_t tri = 3u * (uint32_t)(first + j);
        const float4 T0 = ld4<Uniform>(S.tris, tri);
        float t, u, v;
        if (tri_test(T0, ld4<Uniform>(S.tris, tri + 1), ld4<Uniform>(S.tris, tri + 2), o, d, tnear, h.t, t, u, v)) {
            const int prim = __float_as_int(T0.w);
            if (h.prim < 0 || t < h.t || (t == h.t && prim < h.prim)) { h.t = t; h.u = u; h.v = v; h.prim = prim; }
        }
    }
    cur = skip;
}

// ---------------------------------------------------------------- per-lane walks (TRAV_LANE)
// Branch-lean per-lane walks: uniform loop condition, select-based cursor updates, the leaf's
// triangles in a wave-uniform loop up to the largest leaf among the lanes -- no per-lane exec-mask
// regions (C3: +21 % over the branchy loop).  Measured alternatives (kept in git history
// only): child-box records with a short stack, 8-bit quantised and binary16 nodes, a node lookahead,
// deferred leaves and a union walk of a pixel's shadow-ray pair -- all bit-identical, all slower on C3.
// walk from node `i` (0xffffffff: no walk) to the end of the preorder
__device__ __forceinline__ bool occluded_lane_from(const DevScene& S, uint32_t i, vec3 o, vec3 d, vec3 inv, float tnear,
                                                   float tfar) {
    const uint32_t n = S.n_nodes;
    uint32_t occ = 0u;
    while (__ballot(i < n) != 0) {
        const bool live = i < n;
        const uint32_t ii = live ? i : 0u;
        const float4 a = S.nodes[2 * ii], b = S.nodes[2 * ii + 1];
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
        const bool hit = live & box_test(a, b, o, inv, tnear, tfar);
        const bool in_leaf = hit & (leaf >= 0);
        const int first = leaf >> 3, cnt = in_leaf ? (leaf & 7) + 1 : 0;
        for (int j = 0; j < 8; ++j) {
            const bool want = (j < cnt) & (occ == 0u);
            if (__ballot(want) == 0) break;
            const float4* T = S.tris + 3 * (want ? first + j : 0);
            float t, u, v;
            const bool h = tri_test_nb(T[0], T[1], T[2], o, d, tnear, tfar, t, u, v);
            occ = (want & h) ? 1u : occ;
        }
        i = !live ? i : (occ ? 0xffffffffu : ((hit & (leaf < 0)) ? i + 1 : skip));
    }
    return occ != 0u;
}
__device__ __forceinline__ bool occluded_lane(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    return occluded_lane_from(S, active ? 0u : 0xffffffffu, o, d, inv, tnear, tfar);
}
__device__ __forceinline__ void closest_lane_from(const DevScene& S, uint32_t i, vec3 o, vec3 d, vec3 inv, float tnear,
                                                  Hit& h) {
    const uint32_t n = S.n_nodes;
    while (__ballot(i < n) != 0) {
        const bool live = i < n;
        const uint32_t ii = live ? i : 0u;
        const float4 a = S.nodes[2 * ii], b = S.nodes[2 * ii + 1];
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
        const bool hit = live & box_test(a, b, o, inv, tnear, h.t);
        const bool in_leaf = hit & (leaf >= 0);
        const int first = leaf >> 3, cnt = in_leaf ? (leaf & 7) + 1 : 0;
        for (int j = 0; j < 8; ++j) {
            const bool want = j < cnt;
            if (__ballot(want) == 0) break;
            const float4* T = S.tris + 3 * (want ? first + j : 0);
            const float4 T0 = T[0];
            float t, u, v;
            const bool hh = want & tri_test_nb(T0, T[1], T[2], o, d, tnear, h.t, t, u, v);
            const int prim = __float_as_int(T0.w);
            const bool better = hh & (h.prim < 0 || t < h.t || (t == h.t && prim < h.prim));
            h.t = better ? t : h.t; h.u = better ? u : h.u; h.v = better ? v : h.v;
            h.prim = better ? prim : h.prim;
        }
        i = !live ? i : ((hit & (leaf < 0)) ? i + 1 : skip);
    }
}
__device__ __forceinline__ Hit closest_lane(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    Hit h; h.t = tfar; h.u = 0; h.v = 0; h.prim = -1;
    closest_lane_from(S, active ? 0u : 0xffffffffu, o, d, inv, tnear, h);
    return h;
}

// ---------------------------------------------------------------- wave-coherent walks (TRAV_LOCKSTEP)
// The skip-pointer order is a global order and every ray only moves forward through it, so a wave
// can walk the node array together: each step it takes m = min over lanes of their next node, loads
// node m ONCE with scalar loads (uniform address, no 64-address gather), and only the lanes whose
// next node is m test it.  The number of steps is the size of the union of the lanes' paths -- for
// a wave's shadow rays from one 8x8 tile this is ~ the longest single path (scripts/bvh_analysis.py:
// union 30.4 vs longest 28.9 nodes on C2) -- while per-step memory traffic drops from up to 64 cache
// lines to one.  For incoherent rays the union approaches the sum of the paths (C3: 4x slower than
// TRAV_LANE), hence the per-scene choice.

// min over all 64 lanes (EXEC must be all ones): DPP butterfly in-row, then row broadcasts
__device__ __forceinline__ uint32_t wave_min_full(uint32_t v) {
    const int I = (int)0xffffffff;   // identity for unsigned min (lanes masked off by row/bank masks)
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// exact min over the ACTIVE lanes for a partially masked wave (slow path; kernels keep waves full)
__device__ __forceinline__ uint32_t wave_min_partial(uint32_t v) {
    uint32_t m = 0xffffffffu;
    uint64_t act = __ballot(1);
    while (act) {
        int lane = __builtin_ctzll(act);
        act &= act - 1;
        uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
        m = x < m ? x : m;
    }
    return m;
}

__device__ __forceinline__ uint32_t wave_min(bool full, uint32_t v) {
    return full ? wave_min_full(v) : wave_min_partial(v);
}
template <int K>
__device__ __forceinline__ uint32_t lane_min(const uint32_t* cur) {
    uint32_t lm = cur[0];
#pragma unroll
    for (int k = 1; k < K; ++k) lm = cur[k] < lm ? cur[k] : lm;
    return lm;
}
// Next step's node after a lockstep step at m.  Every cursor is > m afterwards (lanes on m moved to
// m + 1, skip(m) > m or done; the others were already > m), so if any lane descended to m + 1 that is
// the minimum -- the cross-lane reduction is only needed when no lane descended.
__device__ __forceinline__ uint32_t next_min(bool full, bool descended, uint32_t m, uint32_t lane_min_v) {
    if (__ballot(descended) != 0) return m + 1;
    return wave_min(full, lane_min_v);
}

// K any-hit rays per lane sharing one origin (a pixel's shadow rays to K light samples), one lockstep
// walk: each lane keeps K cursors, the wave steps through the union of all 64*K paths; each step's node
// (and leaf triangles) is loaded once and tested against every ray whose cursor is on it.
template <int K>
__device__ __forceinline__ void occluded_wave_multi(const DevScene& S, const bool* active, vec3 o, const vec3* d,
                                                    float tnear, const float* tfar, bool* occ) {
    const bool full = __ballot(1) == ~0ull;
    vec3 inv[K];
    uint32_t cur[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        inv[k] = mk(1.0f / d[k].x, 1.0f / d[k].y, 1.0f / d[k].z);
        cur[k] = active[k] ? 0u : 0xffffffffu;
        occ[k] = false;
    }
    const uint32_t n = S.n_nodes;
    // per-lane ray state as integer bit-sets (bit k = ray k) held in VGPRs and updated with selects:
    // bools carried across the loop's control flow would live as SGPR lane masks re-merged with
    // s_andn2/s_and/s_or at every join -- that bookkeeping made SALU the busiest unit.  Only
    // wave-uniform branches remain (leaf or not, ballot tests).
    uint32_t occb = 0u;
    uint32_t m = wave_min(full, lane_min<K>(cur));
    while (m < n) {
        float4 a, b;
        node_load(S.nodes, m, a, b);
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
        uint32_t hbb = 0u;
#pragma unroll
        for (int k = 0; k < K; ++k) hbb |= (cur[k] == m && box_test(a, b, o, inv[k], tnear, tfar[k])) ? (1u << k) : 0u;
        if (leaf >= 0) {                                      // wave-uniform
            const int first = leaf >> 3, cnt = (leaf & 7) + 1;
            for (int j = 0; j < cnt; ++j) {
                const uint32_t want = hbb & ~occb;
                if (__ballot(want != 0u) == 0) break;
                const uint32_t tri = 3u * (uint32_t)(first + j);
                const float4 T0 = sload(S.tris, tri), T1 = sload(S.tris, tri + 1), T2 = sload(S.tris, tri + 2);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    if (__ballot((want >> k) & 1u) != 0) {        // wave-uniform
                        float t, u, v;
                        const bool hit = tri_test_nb(T0, T1, T2, o, d[k], tnear, tfar[k], t, u, v);
                        occb |= (((want >> k) & 1u) && hit) ? (1u << k) : 0u;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < K; ++k)
                cur[k] = cur[k] == m ? (((hbb & occb) >> k) & 1u ? 0xffffffffu : skip) : cur[k];
            m = wave_min(full, lane_min<K>(cur));
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) cur[k] = cur[k] == m ? ((hbb >> k) & 1u ? m + 1 : skip) : cur[k];
            m = next_min(full, hbb != 0u, m, lane_min<K>(cur));
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) occ[k] = (occb >> k) & 1u;
}
// one any-hit ray per lane (the K = 1 walk, written out: the leaf loop exits per lane)
__device__ __forceinline__ bool occluded_wave(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const bool full = __ballot(1) == ~0ull;
    vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const uint32_t n = S.n_nodes;
    uint32_t i = active ? 0u : 0xffffffffu;
    uint32_t occ = 0u;                 // integer, not a bool: see occluded_wave_multi
    uint32_t m = wave_min(full, i);
    while (m < n) {
        float4 a, b;
        node_load(S.nodes, m, a, b);
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
        const bool at = i == m;
        const bool hb = at && box_test(a, b, o, inv, tnear, tfar);
        if (leaf >= 0) {                                      // wave-uniform
            const int first = leaf >> 3, cnt = (leaf & 7) + 1;
            for (int k = 0; k < cnt; ++k) {
                const bool want = hb && occ == 0u;
                if (__ballot(want) == 0) break;
                const uint32_t tri = 3u * (uint32_t)(first + k);
                float t, u, v;
                const bool hit = tri_test_nb(sload(S.tris, tri), sload(S.tris, tri + 1), sload(S.tris, tri + 2), o, d,
                                             tnear, tfar, t, u, v);
                occ = (want && hit) ? 1u : occ;
            }
            i = at ? ((hb && occ) ? 0xffffffffu : skip) : i;
            m = wave_min(full, i);
        } else {
            i = at ? (hb ? m + 1 : skip) : i;
            m = next_min(full, hb, m, i);
        }
    }
    return occ != 0u;
}
__device__ __forceinline__ Hit closest_wave(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const bool full = __ballot(1) == ~0ull;
    vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    Hit h; h.t = tfar; h.u = 0; h.v = 0; h.prim = -1;
    const uint32_t n = S.n_nodes;
    uint32_t i = active ? 0u : 0xffffffffu;
    uint32_t m = wave_min(full, i);
    while (m < n) {
        float4 a, b;
        node_load(S.nodes, m, a, b);
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
        const bool at = i == m;
        const bool hb = at && box_test(a, b, o, inv, tnear, h.t);
        if (leaf >= 0) {                                      // wave-uniform
            if (__ballot(hb) != 0) {
                const int first = leaf >> 3, cnt = (leaf & 7) + 1;
                for (int k = 0; k < cnt; ++k) {
                    const uint32_t tri = 3u * (uint32_t)(first + k);
                    const float4 T0 = sload(S.tris, tri);
                    float t, u, v;
                    const bool hit = hb & tri_test_nb(T0, sload(S.tris, tri + 1), sload(S.tris, tri + 2), o, d, tnear,
                                                       h.t, t, u, v);
                    const int prim = __float_as_int(T0.w);
                    const bool better = hit && (h.prim < 0 || t < h.t || (t == h.t && prim < h.prim));
                    h.t = better ? t : h.t; h.u = better ? u : h.u; h.v = better ? v : h.v;
                    h.prim = better ? prim : h.prim;
                }
            }
            i = at ? skip : i;
            m = wave_min(full, i);
        } else {
            i = at ? (hb ? m + 1 : skip) : i;
            m = next_min(full, hb, m, i);
        }
    }
    return h;
}

// ---------------------------------------------------------------- dispatch
// Every lane of the wave must make the call (convergent call sites); `active` selects the lanes with a ray.
template <int T, int K>
__device__ __forceinline__ void trace_any_multi(const DevScene& S, const bool* active, vec3 o, const vec3* d,
                                                float tnear, const float* tfar, bool* occ) {
    if (T == TRAV_LOCKSTEP) {
        occluded_wave_multi<K>(S, active, o, d, tnear, tfar, occ);
    } else {   // one walk after the other (measured faster than interleaving the K walks, and than one
               // loop running a lane's walks back to back: that spilled the hot loop, 2.5x slower on C3)
#pragma unroll
        for (int k = 0; k < K; ++k) occ[k] = occluded_lane(S, active[k], o, d[k], tnear, tfar[k]);
    }
}
template <int T>
__device__ __forceinline__ bool trace_any(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    if (T == TRAV_LOCKSTEP) return occluded_wave(S, active, o, d, tnear, tfar);
    return occluded_lane(S, active, o, d, tnear, tfar);
}
template <int T>
__device__ __forceinline__ Hit trace_closest(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    if (T == TRAV_LOCKSTEP) return closest_wave(S, active, o, d, tnear, tfar);
    return closest_lane(S, active, o, d, tnear, tfar);
}

// Material record (pg/material.h:105-115)
struct MatRec { vec3 kd; float shin; vec3 ks; int type; vec3 le; };
constexpr int kMatStride = 4;
__device__ __forceinline__ MatRec load_mat(const DevScene& S, uint32_t m) {
    float4 a = S.mats[kMatStride * m], b = S.mats[kMatStride * m + 1], c = S.mats[kMatStride * m + 2];
    return MatRec{xyz(a), a.w, xyz(b), __float_as_int(b.w), xyz(c)};
}
__device__ __forceinline__ int4 load_maps(const DevScene& S, uint32_t m) {
    float4 q = S.mats[kMatStride * m + 3];
    return make_int4(__float_as_int(q.x), __float_as_int(q.y), __float_as_int(q.z), __float_as_int(q.w));
}

// Intersection::intersectEmbree + getGeometryAttributes (pg/Intersection.h:8-41,85-113):
// hit point = org + dir*t, interpolated normal (1-u-v)n0 + u n1 + v n2, normalised, flipped to face
// the ray; material; emissive id (vertex-0 attribute, :103-110).
struct SurfHit { bool hit; vec3 point, normal; uint32_t mat; int emis_id; int prim; float u, v; };
template <int T>
__device__ __forceinline__ SurfHit intersect(const DevScene& S, bool active, vec3 o, vec3 d, float tnear) {
    SurfHit r; r.hit = false; r.mat = 0; r.emis_id = -1; r.point = mk(0, 0, 0); r.normal = mk(0, 0, 0);
    r.prim = -1; r.u = 0.0f; r.v = 0.0f;
    Hit h = trace_closest<T>(S, active, o, d, tnear, FLT_MAX);
    if (h.prim < 0) return r;
    const float4* N = S.tri_nrm + 3 * h.prim;
    float4 n0 = N[0], n1 = N[1], n2 = N[2];
    float w = 1.0f - h.u - h.v;
    vec3 n = (xyz(n0) * w + xyz(n1) * h.u) + xyz(n2) * h.v;
    n = normalize(n);
    if (dot(-d, n) <= 0.0f) n = n * -1.0f;
    r.hit = true; r.normal = n; r.point = o + d * h.t;
    r.mat = (uint32_t)__float_as_int(n0.w); r.emis_id = __float_as_int(n1.w);
    r.prim = h.prim; r.u = h.u; r.v = h.v;
    return r;
}

}  // namespace rs
