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
    // child-box records of the interior nodes (TRAV_LANE walks, see "child-box walks" below)
    const float4* crec;
    const uint32_t* cskip;    // per record: the node after its subtree (skip pointer), overflow fallback
    uint32_t n_crec;          // 0: none (single-leaf tree) -> the skip-pointer walks
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
// node format of the per-lane walks: 0 skip-pointer float nodes, 1/2 child-box records, 3 half nodes
#ifndef RS_CREC
#define RS_CREC 0
#endif
// Node fetch of the per-lane skip-pointer walks.  RS_CREC == 3: one 16-B record per node (half the
// lane-loads of the 32-B float node, which bound these walks -- §3.8 of DESIGN.md): the box as six
// binary16 values rounded OUTWARD (rs_bvh_build.hip k_crec_emit), so it contains the exact box and the
// walk visits a superset of the exact walk's nodes with the same triangle tests -- bit-identical hits;
// w: interior -> skip pointer, leaf -> 1 << 31 | first << 3 | count - 1 (a leaf's skip is i + 1 in the
// preorder).
__device__ __forceinline__ float h2f(uint32_t bits) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(bits & 0xffffu));
}
__device__ __forceinline__ void lane_node(const DevScene& S, uint32_t i, float4& a, float4& b, uint32_t& skip, int& leaf) {
    if (RS_CREC == 3) {   // built for every non-empty tree (bvh_crec_build fails otherwise)
        const uint4 q = ((const uint4*)S.crec)[i];
        a = make_float4(h2f(q.x), h2f(q.x >> 16), h2f(q.y), 0.0f);
        b = make_float4(h2f(q.y >> 16), h2f(q.z), h2f(q.z >> 16), 0.0f);
        const bool lf = (int)q.w < 0;
        skip = lf ? i + 1u : q.w;
        leaf = lf ? (int)(q.w & 0x7fffffffu) : -1;
    } else {
        a = S.nodes[2 * i]; b = S.nodes[2 * i + 1];
        skip = (uint32_t)__float_as_int(a.w);
        leaf = __float_as_int(b.w);
    }
}
// RS_CREC == 3: a leaf whose half box was hit is re-tested against its exact float box before its
// triangles are (the outward-rounded boxes of leaves next to a ray's origin surface would otherwise add
// ~1.3 triangle tests per shadow ray on C3, which cost more than the halved node loads save)
__device__ __forceinline__ bool leaf_exact(const DevScene& S, bool in_leaf, uint32_t i, vec3 o, vec3 inv, float tnear,
                                           float tfar) {
#if RS_CREC == 3 && !defined(RS_HALF_LOOSE_LEAVES)
    if (__ballot(in_leaf) == 0) return false;
    bool r = false;
    if (in_leaf) {                        // only the lanes on a hit leaf load its exact box
        const float4 a = S.nodes[2 * i], b = S.nodes[2 * i + 1];
        r = box_test(a, b, o, inv, tnear, tfar);
    }
    return r;
#else
    return in_leaf;
#endif
}
// RS_LANE_LOOKAHEAD=1: the walk carries node i + 1 beside node i.  The next node is i + 1 after every
// entered interior node and after every leaf (a leaf's skip is i + 1 in the preorder), so those steps
// start without waiting on a dependent load; the load of the new i + 1 (and, after a miss, of the skip
// target) is issued at the end of each step.  Same nodes visited in the same order: bit-identical.
#ifndef RS_LANE_LOOKAHEAD
#define RS_LANE_LOOKAHEAD 0
#endif
#define RS_LA (RS_LANE_LOOKAHEAD && RS_CREC == 0)
__device__ __forceinline__ void la_advance(const DevScene& S, bool next_is_ahead, uint32_t nx, uint32_t n, float4& ca,
                                           float4& cb, float4& na, float4& nb) {
    if (next_is_ahead) { ca = na; cb = nb; }
    else if (nx < n) { ca = S.nodes[2 * nx]; cb = S.nodes[2 * nx + 1]; }
    if (nx < n - 1u) { na = S.nodes[2 * nx + 2]; nb = S.nodes[2 * nx + 3]; }
}
// Branch-lean per-lane walks: uniform loop condition, select-based cursor updates, the leaf's
// triangles in a wave-uniform loop up to the largest leaf among the lanes -- no per-lane exec-mask
// regions (C3: +21 % over the branchy loop).
// walk from node `i` (0xffffffff: no walk) to the end of the preorder
__device__ __forceinline__ bool occluded_lane_from(const DevScene& S, uint32_t i, vec3 o, vec3 d, vec3 inv, float tnear,
                                                   float tfar) {
    const uint32_t n = S.n_nodes;
    uint32_t occ = 0u;
#if RS_LA
    float4 ca = make_float4(0.0f, 0.0f, 0.0f, 0.0f), cb = ca, na = ca, nb = ca;
    la_advance(S, false, i, n, ca, cb, na, nb);
#endif
    while (__ballot(i < n) != 0) {
        const bool live = i < n;
        const uint32_t ii = live ? i : 0u;
#if RS_LA
        const float4 a = ca, b = cb;
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
#else
        float4 a, b;
        uint32_t skip;
        int leaf;
        lane_node(S, ii, a, b, skip, leaf);
#endif
        const bool hit = live & box_test(a, b, o, inv, tnear, tfar);
        const bool in_leaf = leaf_exact(S, hit & (leaf >= 0), ii, o, inv, tnear, tfar);
        const int first = leaf >> 3, cnt = in_leaf ? (leaf & 7) + 1 : 0;
        for (int j = 0; j < 8; ++j) {
            const bool want = (j < cnt) & (occ == 0u);
            if (__ballot(want) == 0) break;
            const float4* T = S.tris + 3 * (want ? first + j : 0);
            float t, u, v;
            const bool h = tri_test_nb(T[0], T[1], T[2], o, d, tnear, tfar, t, u, v);
            occ = (want & h) ? 1u : occ;
        }
        const uint32_t nx = !live ? i : (occ ? 0xffffffffu : ((hit & (leaf < 0)) ? i + 1 : skip));
#if RS_LA
        la_advance(S, live & (nx == i + 1u), nx, n, ca, cb, na, nb);
#endif
        i = nx;
    }
    return occ != 0u;
}
// RS_LANE_DEFER=k: deferred leaves for the any-hit per-lane walk (Aila & Laine's while-while idea): a lane
// whose walk reaches a hit leaf parks there, the others keep stepping through interior nodes, and the
// wave tests the parked lanes' triangles together once >= k lanes are parked (or no lane can step) --
// the wave-wide triangle loop runs for many lanes at once instead of at almost every step.  Every ray
// still makes its own tests in its own order: bit-identical.
#ifndef RS_LANE_DEFER
#define RS_LANE_DEFER 0
#endif
__device__ __forceinline__ bool occluded_lane_defer(const DevScene& S, uint32_t i, vec3 o, vec3 d, vec3 inv, float tnear,
                                                    float tfar) {
    const uint32_t n = S.n_nodes;
    uint32_t occ = 0u, parked = 0u, pskip = 0u;
    int pleaf = 0;
    while (__ballot(i < n) != 0) {
        const bool step = (i < n) & (parked == 0u);
        const uint32_t ii = step ? i : 0u;
        const float4 a = S.nodes[2 * ii], b = S.nodes[2 * ii + 1];
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
        const bool hit = step & box_test(a, b, o, inv, tnear, tfar);
        const bool to_leaf = hit & (leaf >= 0);
        i = (step & !to_leaf) ? (hit ? i + 1 : skip) : i;
        parked = to_leaf ? 1u : parked;
        pleaf = to_leaf ? leaf : pleaf;
        pskip = to_leaf ? skip : pskip;
        const uint64_t pk = __ballot(parked != 0u);
        if (__popcll(pk) >= RS_LANE_DEFER || (pk != 0 && __ballot((i < n) & (parked == 0u)) == 0)) {   // wave-uniform
            const int first = pleaf >> 3, cnt = parked ? (pleaf & 7) + 1 : 0;
            for (int j = 0; j < 8; ++j) {
                const bool want = (j < cnt) & (occ == 0u);
                if (__ballot(want) == 0) break;
                const float4* T = S.tris + 3 * (want ? first + j : 0);
                float t, u, v;
                const bool h = tri_test_nb(T[0], T[1], T[2], o, d, tnear, tfar, t, u, v);
                occ = (want & h) ? 1u : occ;
            }
            i = parked ? (occ ? 0xffffffffu : pskip) : i;
            parked = 0u;
        }
    }
    return occ != 0u;
}
__device__ __forceinline__ bool occluded_lane_skip(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    if (RS_LANE_DEFER > 0 && RS_CREC == 0)
        return occluded_lane_defer(S, active ? 0u : 0xffffffffu, o, d, inv, tnear, tfar);
    return occluded_lane_from(S, active ? 0u : 0xffffffffu, o, d, inv, tnear, tfar);
}
__device__ __forceinline__ void closest_lane_from(const DevScene& S, uint32_t i, vec3 o, vec3 d, vec3 inv, float tnear,
                                                  Hit& h) {
    const uint32_t n = S.n_nodes;
#if RS_LA
    float4 ca = make_float4(0.0f, 0.0f, 0.0f, 0.0f), cb = ca, na = ca, nb = ca;
    la_advance(S, false, i, n, ca, cb, na, nb);
#endif
    while (__ballot(i < n) != 0) {
        const bool live = i < n;
        const uint32_t ii = live ? i : 0u;
#if RS_LA
        const float4 a = ca, b = cb;
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
#else
        float4 a, b;
        uint32_t skip;
        int leaf;
        lane_node(S, ii, a, b, skip, leaf);
#endif
        const bool hit = live & box_test(a, b, o, inv, tnear, h.t);
        const bool in_leaf = leaf_exact(S, hit & (leaf >= 0), ii, o, inv, tnear, h.t);
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
        const uint32_t nx = !live ? i : ((hit & (leaf < 0)) ? i + 1 : skip);
#if RS_LA
        la_advance(S, live & (nx == i + 1u), nx, n, ca, cb, na, nb);
#endif
        i = nx;
    }
}
__device__ __forceinline__ Hit closest_lane_skip(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    Hit h; h.t = tfar; h.u = 0; h.v = 0; h.prim = -1;
    closest_lane_from(S, active ? 0u : 0xffffffffu, o, d, inv, tnear, h);
    return h;
}

// K any-hit rays of one lane sharing an origin (a pixel's area-candidate pair), one per-lane walk over
// the union of their skip-pointer paths: each step fetches the lane's smallest cursor once and tests
// every ray whose cursor is on it, so the paths' common prefix (the top of the tree) is fetched once
// instead of K times.  Each ray's cursor sequence is its own walk's -- the same box and triangle tests,
// bit-identical results.  RS_LANE_UNION=0: the K walks one after the other.
#ifndef RS_LANE_UNION
#define RS_LANE_UNION 0
#endif
template <int K>
__device__ __forceinline__ void occluded_lane_union(const DevScene& S, const bool* active, vec3 o, const vec3* d,
                                                    float tnear, const float* tfar, bool* occ) {
    constexpr uint32_t kDone = 0xffffffffu;
    vec3 inv[K];
    uint32_t cur[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        inv[k] = mk(1.0f / d[k].x, 1.0f / d[k].y, 1.0f / d[k].z);
        cur[k] = active[k] ? 0u : kDone;
    }
    const uint32_t n = S.n_nodes;
    uint32_t occb = 0u;
    uint32_t m = cur[0];
#pragma unroll
    for (int k = 1; k < K; ++k) m = cur[k] < m ? cur[k] : m;
    while (__ballot(m < n) != 0) {
        const bool live = m < n;
        const uint32_t ii = live ? m : 0u;
        float4 a, b;
        uint32_t skip;
        int leaf;
        lane_node(S, ii, a, b, skip, leaf);
        uint32_t hbb = 0u;
#pragma unroll
        for (int k = 0; k < K; ++k) hbb |= (live & (cur[k] == m) && box_test(a, b, o, inv[k], tnear, tfar[k])) ? (1u << k) : 0u;
        const int first = leaf >> 3, cnt = (leaf >= 0) & (hbb != 0u) ? (leaf & 7) + 1 : 0;
        for (int j = 0; j < 8; ++j) {
            const uint32_t want = j < cnt ? hbb & ~occb : 0u;
            if (__ballot(want != 0u) == 0) break;
            const float4* T = S.tris + 3 * (want ? first + j : 0);
            const float4 T0 = T[0], T1 = T[1], T2 = T[2];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (__ballot((want >> k) & 1u) != 0) {
                    float t, u, v;
                    const bool h = tri_test_nb(T0, T1, T2, o, d[k], tnear, tfar[k], t, u, v);
                    occb |= (((want >> k) & 1u) && h) ? (1u << k) : 0u;
                }
            }
        }
        uint32_t nm = kDone;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t nx = ((occb >> k) & 1u) ? kDone : ((((hbb >> k) & 1u) && leaf < 0) ? m + 1u : skip);
            cur[k] = (live & (cur[k] == m)) ? nx : cur[k];
            nm = cur[k] < nm ? cur[k] : nm;
        }
        m = nm;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) occ[k] = (occb >> k) & 1u;
}

// ---------------------------------------------------------------- child-box walks (TRAV_LANE)
// The skip-pointer walk fetches a node to test that node's own box, so every child of every entered
// node costs one dependent load -- about twice the entered nodes.  A child-box record holds BOTH
// children's boxes of an interior node, so a walk loads one record per ENTERED interior node; a leaf
// child's triangles are tested straight from its parent's visit (leaf nodes are never fetched).
//
// The per-lane walks of C3 keep the vector-memory pipeline busy (TA/TD ~90 % busy on k_gbuffer_initial;
// loading every record twice costs +57 % time); a 32-B record (two 16-B loads instead of four) quantises
// the children's boxes to 8 bits:
//   RS_CREC == 2, 2 x uint4:
//     w0..w2  origin O (float; the record's box lo)       w3.b0  biased exponent e of the scale s = 2^(e-127)
//     w3.b1-3 L.lo q    w4.b0-2 L.hi q    w4.b3,w5.b0-1 R.lo q    w5.b2-3,w6.b0 R.hi q
//     w6.b1-3 + w7.b0-3: two 28-bit links (bit 27: leaf; leaf: first tri << 3 | count - 1, else record)
//   coordinate = O + q * s, emitted rounded OUTWARD (rs_bvh_build.hip k_crec_emit checks every one with
//   this same expression), e == 0: a box that could not be quantised -- always entered
//   RS_CREC == 1: 64 B exact records, 4 x float4: (L.lo, Llink) (L.hi, Rlink) (R.lo, skip) (R.hi, 0),
//   link >= 0 a record, < 0 ~leaf word
// Right children whose box was hit wait on a short per-lane stack in registers (RS_CSTACK entries,
// shifted: no scratch); when it overflows the oldest entry is dropped and, once the stack runs empty,
// the walk finishes as a skip-pointer walk: an any-hit walk (always left first, so every dropped entry
// is a right child of an ancestor) from the current record's skip (S.cskip), after which the preorder
// holds every dropped subtree; a closest-hit walk (nearer child first) from the root, culled by the
// closest hit found so far.  Every box the walk tests contains the exact box, the box test is the same
// conservative slab test and the triangle tests are the same (any-hit: existence; closest: the tie
// rule), so results are bit-identical to the skip-pointer walks.  Records are emitted from the nodes at
// build time and after every refit (rs_bvh_build.hip).
#ifndef RS_CSTACK
#define RS_CSTACK 6
#endif
// Default 0 (skip-pointer walks): measured on C3 (k_gbuffer_initial, lane walks, 1080p): skip pointers
// 23.6 ms, 64-B records 23.8-25.1 ms, 32-B quantised records 31.3 ms -- the record walk halves the
// dependent loads and the L1 misses but not the lane-loads, and the dequantisation VALU sits on the
// walk's critical path.  Kept as a build option (-DRS_CREC=1/2), tested bit-identical.
constexpr int kCrecWords = RS_CREC == 2 ? 2 : (RS_CREC == 3 ? 1 : 4);     // float4 per record
#define RS_CREC_REC (RS_CREC == 1 || RS_CREC == 2)   // child-box record walks (3: half-precision nodes)
struct CStack {
    uint32_t s[RS_CSTACK];
    int sp;
    bool dropped;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int k = 0; k < RS_CSTACK; ++k) s[k] = 0u;
        sp = 0; dropped = false;
    }
    __device__ __forceinline__ void push(bool c, uint32_t v) {
        dropped = dropped | (c & (sp == RS_CSTACK));
#pragma unroll
        for (int k = RS_CSTACK - 1; k > 0; --k) s[k] = c ? s[k - 1] : s[k];
        s[0] = c ? v : s[0];
        sp = c ? (sp < RS_CSTACK ? sp + 1 : sp) : sp;
    }
    __device__ __forceinline__ void pop(bool c) {
#pragma unroll
        for (int k = 0; k < RS_CSTACK - 1; ++k) s[k] = c ? s[k + 1] : s[k];
        sp = c ? sp - 1 : sp;
    }
};
// slab test returning the entry distance (closest-hit child order)
__device__ __forceinline__ bool box_test_t(float4 a, float4 b, vec3 o, vec3 inv, float tnear, float tfar, float& tin) {
    float tx0 = (a.x - o.x) * inv.x, tx1 = (b.x - o.x) * inv.x;
    float ty0 = (a.y - o.y) * inv.y, ty1 = (b.y - o.y) * inv.y;
    float tz0 = (a.z - o.z) * inv.z, tz1 = (b.z - o.z) * inv.z;
    float t0 = fmaxf(fmaxf(fmaxf(tnear, fminf(tx0, tx1)), fminf(ty0, ty1)), fminf(tz0, tz1));
    float t1 = fminf(fminf(fminf(tfar, fmaxf(tx0, tx1)), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    tin = t0;
    return t0 * (1.0f - 4.0f * FLT_EPSILON) <= t1 * (1.0f + 4.0f * FLT_EPSILON);
}
// quantised coordinate -> float; the emitter rounds q outward against exactly this expression
__device__ __forceinline__ float crec_deq(float o, uint32_t q, float s) { return o + (float)q * s; }

// One record visit: both children's box tests against [tnear, tfar], decoded links.
struct CVisit {
    bool hL, hR;           // box hit
    float tL, tR;          // entry distances (closest-hit order)
    bool leafL, leafR;
    uint32_t aL, aR;       // interior: record index; leaf: first triangle
    int cL, cR;            // leaf triangle counts
};
template <bool Ordered>   // Ordered: entry distances for the closest-hit child order
__device__ __forceinline__ CVisit crec_visit(const DevScene& S, bool live, uint32_t r, vec3 o, vec3 inv, float tnear,
                                             float tfar) {
    CVisit v;
    v.tL = v.tR = 0.0f;
#if RS_CREC == 2
    const uint4* R4 = (const uint4*)S.crec + 2 * (size_t)r;
    const uint4 a = R4[0], b = R4[1];
    const float ox = __uint_as_float(a.x), oy = __uint_as_float(a.y), oz = __uint_as_float(a.z);
    const uint32_t eb = a.w & 0xffu;
    const float s = __uint_as_float(eb << 23);
    const float4 Llo = make_float4(crec_deq(ox, (a.w >> 8) & 0xffu, s), crec_deq(oy, (a.w >> 16) & 0xffu, s),
                                   crec_deq(oz, a.w >> 24, s), 0.0f);
    const float4 Lhi = make_float4(crec_deq(ox, b.x & 0xffu, s), crec_deq(oy, (b.x >> 8) & 0xffu, s),
                                   crec_deq(oz, (b.x >> 16) & 0xffu, s), 0.0f);
    const float4 Rlo = make_float4(crec_deq(ox, b.x >> 24, s), crec_deq(oy, b.y & 0xffu, s),
                                   crec_deq(oz, (b.y >> 8) & 0xffu, s), 0.0f);
    const float4 Rhi = make_float4(crec_deq(ox, (b.y >> 16) & 0xffu, s), crec_deq(oy, b.y >> 24, s),
                                   crec_deq(oz, b.z & 0xffu, s), 0.0f);
    const bool any = eb == 0u;                       // unquantisable record: enter both children
    if (Ordered) {
        v.hL = live & (any | box_test_t(Llo, Lhi, o, inv, tnear, tfar, v.tL));
        v.hR = live & (any | box_test_t(Rlo, Rhi, o, inv, tnear, tfar, v.tR));
        v.tL = any ? tnear : v.tL; v.tR = any ? tnear : v.tR;
    } else {
        v.hL = live & (any | box_test(Llo, Lhi, o, inv, tnear, tfar));
        v.hR = live & (any | box_test(Rlo, Rhi, o, inv, tnear, tfar));
    }
    const uint32_t lL = (b.z >> 8) | ((b.w & 0xfu) << 24), lR = b.w >> 4;
    v.leafL = (lL >> 27) & 1u; v.leafR = (lR >> 27) & 1u;
    v.aL = v.leafL ? (lL >> 3) & 0xffffffu : lL; v.aR = v.leafR ? (lR >> 3) & 0xffffffu : lR;
    v.cL = (int)(lL & 7u) + 1; v.cR = (int)(lR & 7u) + 1;
#else
    const float4* R4 = S.crec + 4 * (size_t)r;
    const float4 c0 = R4[0], c1 = R4[1], c2 = R4[2], c3 = R4[3];
    if (Ordered) {
        v.hL = live & box_test_t(c0, c1, o, inv, tnear, tfar, v.tL);
        v.hR = live & box_test_t(c2, c3, o, inv, tnear, tfar, v.tR);
    } else {
        v.hL = live & box_test(c0, c1, o, inv, tnear, tfar);
        v.hR = live & box_test(c2, c3, o, inv, tnear, tfar);
    }
    const int lL = __float_as_int(c0.w), lR = __float_as_int(c1.w);
    v.leafL = lL < 0; v.leafR = lR < 0;
    v.aL = v.leafL ? (uint32_t)(~lL) >> 3 : (uint32_t)lL; v.aR = v.leafR ? (uint32_t)(~lR) >> 3 : (uint32_t)lR;
    v.cL = (~lL & 7) + 1; v.cR = (~lR & 7) + 1;
#endif
    return v;
}

__device__ __forceinline__ bool occluded_crec(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    constexpr uint32_t kDone = 0xffffffffu;
    uint32_t cur = active ? 0u : kDone, resume = kDone, occ = 0u;
    CStack st;
    st.init();
    while (__ballot(cur != kDone) != 0) {
        const bool live = cur != kDone;
        const uint32_t r = live ? cur : 0u;
        const CVisit v = crec_visit<false>(S, live, r, o, inv, tnear, tfar);
        const int nL = (v.hL & v.leafL) ? v.cL : 0, nR = (v.hR & v.leafR) ? v.cR : 0;
        for (int j = 0; j < 16; ++j) {
            const bool want = (j < nL + nR) & (occ == 0u);
            if (__ballot(want) == 0) break;
            const uint32_t t = j < nL ? v.aL + j : v.aR + (j - nL);
            const float4* T = S.tris + 3 * (want ? t : 0u);
            float tt, u, w;
            const bool h = tri_test_nb(T[0], T[1], T[2], o, d, tnear, tfar, tt, u, w);
            occ = (want & h) ? 1u : occ;
        }
        const bool iL = v.hL & !v.leafL, iR = v.hR & !v.leafR;
        const bool go = live & (occ == 0u);
        const bool none = !iL & !iR;
        const bool pop = go & none & (st.sp > 0);
        const uint32_t top = st.s[0];
        st.pop(pop);
        st.push(go & iL & iR, v.aR);
        if (go & none & !pop & st.dropped) resume = S.cskip[r];      // rare: the stack overflowed
        const uint32_t nxt = iL ? v.aL : (iR ? v.aR : (pop ? top : kDone));
        cur = !live ? cur : (go ? nxt : kDone);
    }
    if (__ballot(resume != kDone) != 0)            // a stack overflowed: finish as a skip-pointer walk
        occ |= occluded_lane_from(S, occ ? kDone : resume, o, d, inv, tnear, tfar) ? 1u : 0u;
    return occ != 0u;
}

__device__ __forceinline__ Hit closest_crec(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    constexpr uint32_t kDone = 0xffffffffu;
    Hit h; h.t = tfar; h.u = 0; h.v = 0; h.prim = -1;
    uint32_t cur = active ? 0u : kDone, resume = kDone;
    CStack st;
    st.init();
    while (__ballot(cur != kDone) != 0) {
        const bool live = cur != kDone;
        const uint32_t r = live ? cur : 0u;
        const CVisit v = crec_visit<true>(S, live, r, o, inv, tnear, h.t);
        const int nL = (v.hL & v.leafL) ? v.cL : 0, nR = (v.hR & v.leafR) ? v.cR : 0;
        for (int j = 0; j < 16; ++j) {
            const bool want = j < nL + nR;
            if (__ballot(want) == 0) break;
            const uint32_t t = j < nL ? v.aL + j : v.aR + (j - nL);
            const float4* T = S.tris + 3 * (want ? t : 0u);
            const float4 T0 = T[0];
            float tt, u, w;
            const bool hh = want & tri_test_nb(T0, T[1], T[2], o, d, tnear, h.t, tt, u, w);
            const int prim = __float_as_int(T0.w);
            const bool better = hh & (h.prim < 0 || tt < h.t || (tt == h.t && prim < h.prim));
            h.t = better ? tt : h.t; h.u = better ? u : h.u; h.v = better ? w : h.v;
            h.prim = better ? prim : h.prim;
        }
        const bool iL = v.hL & !v.leafL, iR = v.hR & !v.leafR;
        const bool none = !iL & !iR;
        const bool pop = live & none & (st.sp > 0);
        const uint32_t top = st.s[0];
        st.pop(pop);
        const bool rfirst = v.tR < v.tL;              // both entered: the nearer first, the other waits
        st.push(live & iL & iR, rfirst ? v.aL : v.aR);
        // an overflowed closest-hit walk restarts the skip-pointer walk at the root (nearer-first order
        // may have dropped a LEFT child, which precedes the current record in the preorder)
        resume = (live & none & !pop & st.dropped) ? 0u : resume;
        const uint32_t nxt = (iL & iR) ? (rfirst ? v.aR : v.aL) : (iL ? v.aL : (iR ? v.aR : (pop ? top : kDone)));
        cur = !live ? cur : nxt;
    }
    if (__ballot(resume != kDone) != 0) closest_lane_from(S, resume, o, d, inv, tnear, h);
    return h;
}

__device__ __forceinline__ bool occluded_lane(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    if (RS_CREC_REC && S.n_crec) return occluded_crec(S, active, o, d, tnear, tfar);
    return occluded_lane_skip(S, active, o, d, tnear, tfar);
}
__device__ __forceinline__ Hit closest_lane(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    if (RS_CREC_REC && S.n_crec) return closest_crec(S, active, o, d, tnear, tfar);
    return closest_lane_skip(S, active, o, d, tnear, tfar);
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
    } else if (RS_LANE_UNION && !(RS_CREC_REC && S.n_crec)) {
        occluded_lane_union<K>(S, active, o, d, tnear, tfar, occ);
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
