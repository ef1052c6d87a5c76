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
    // 8-wide tree of the per-lane walks (rs_bvh_build.hip build_wide); n_wnodes = 0: skip-pointer walks
    const uint4* wnodes;      // 5 per node
    const float4* wtris;      // 3 per wide-leaf triangle: (v0, prim) (e1) (e2)
    uint32_t n_wnodes;
    // per emissive triangle: its bucket (0..63) in the Morton order of the emitters' centroids -- the key
    // the wave-sorted initial pass groups its shadow rays by (rs_passes.h k_gbuffer_initial_sorted)
    const uint8_t* ebucket;
    vec3 ecen;                // centre of the emitters' centroid bounds (the sorted spatial pass's target cells)
    float box_eps;            // the closest-hit walks' box margin in scene units (rs_wide.h box_epsilon)
};
constexpr int kCdfGuide = 1024;

// Kernel template value T = walk kind (bit 0) | TRAV_WIDE when the scene's 8-wide tree is live (bit 1):
// every pass kernel exists for the four combinations, so each one carries only the walks it uses (a runtime
// wide-or-skip choice inside one kernel doubled the per-lane kernels' code and register pressure).  The
// lockstep kinds still walk BRDF rays per lane (wide with TRAV_WIDE).
enum Trav : int { TRAV_LOCKSTEP = 0, TRAV_LANE = 1, TRAV_WIDE = 2 };
constexpr bool trav_lane(int T) { return (T & TRAV_LANE) != 0; }
constexpr bool trav_wide(int T) { return (T & TRAV_WIDE) != 0; }

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

// the closest-hit walks' test: the box widened by the margin e (rs_wide.h box_epsilon) on every side, written as
// box_test with the ray origin moved by -+e for the lo / hi planes (olo = o + e, ohi = o - e: (lo - e) - o and
// (hi + e) - o up to rounding), so a triangle the test accepts is never culled with its box.  No per-box cost
// over box_test, and a direction component of exactly 0 (1/d = inf) keeps the slab test exact: the widening
// applied in t (e |1/d| added to the t interval) turned inf - inf into NaN there and dropped the axis --
// C2's centre column and row (pixel-corner rays) then walked most of the tree (+27 % on the initial pass)
__device__ __forceinline__ bool box_test_m(float4 a, float4 b, vec3 olo, vec3 ohi, vec3 inv, float tnear, float tfar) {
    float tx0 = (a.x - olo.x) * inv.x, tx1 = (b.x - ohi.x) * inv.x;
    float ty0 = (a.y - olo.y) * inv.y, ty1 = (b.y - ohi.y) * inv.y;
    float tz0 = (a.z - olo.z) * inv.z, tz1 = (b.z - ohi.z) * inv.z;
    float t0 = fmaxf(fmaxf(fmaxf(tnear, fminf(tx0, tx1)), fminf(ty0, ty1)), fminf(tz0, tz1));
    float t1 = fminf(fminf(fminf(tfar, fmaxf(tx0, tx1)), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
    return t0 * (1.0f - 4.0f * FLT_EPSILON) <= t1 * (1.0f + 4.0f * FLT_EPSILON);
}
struct MarginO { vec3 lo, hi; };   // box_test_m's shifted origins
__device__ __forceinline__ MarginO margin_origins(const DevScene& S, vec3 o) {
    const float e = S.box_eps;
    return MarginO{mk(o.x + e, o.y + e, o.z + e), mk(o.x - e, o.y - e, o.z - e)};
}
// the 8-wide walk's form of the margin: e |1/d| per axis in t (wide_hits widens its t bounds per axis already)
__device__ __forceinline__ vec3 box_margin(const DevScene& S, vec3 inv) {
    return mk(S.box_eps * fabsf(inv.x), S.box_eps * fabsf(inv.y), S.box_eps * fabsf(inv.z));
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
                                              vec3 inv, MarginO mo, float tnear, uint32_t& cur, Hit& h) {
    const uint32_t skip = (uint32_t)__float_as_int(a.w);
    if (!box_test_m(a, b, mo.lo, mo.hi, inv, tnear, h.t)) { cur = skip; return; }
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

__device__ __forceinline__ void closest_lane_from(const DevScene& S, uint32_t i, vec3 o, vec3 d, vec3 inv, float tnear,
                                                  Hit& h) {
    const uint32_t n = S.n_nodes;
    const MarginO mo = margin_origins(S, o);
    while (__ballot(i < n) != 0) {
        const bool live = i < n;
        const uint32_t ii = live ? i : 0u;
        const float4 a = S.nodes[2 * ii], b = S.nodes[2 * ii + 1];
        const uint32_t skip = (uint32_t)__float_as_int(a.w);
        const int leaf = __float_as_int(b.w);
        const bool hit = live & box_test_m(a, b, mo.lo, mo.hi, inv, tnear, h.t);
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



// ---------------------------------------------------------------- 8-wide per-lane walks (TRAV_LANE)
// The skip-pointer walk fetches every child of every entered node to test that child's box: ~75 dependent
// 32-B node loads per C3 shadow ray, and the per-lane walks are bound by those lane-loads and the VALU of
// one box test per step.  The 8-wide tree (rs_bvh_build.hip build_wide: 80-B nodes
// holding the quantised boxes of up to 8 children) tests all children of a node per fetch: ~14 node
// fetches per shadow ray (5 x 16-B loads each), i.e. about half the lane-loads, a fifth of the
// dependent-load chain, and 8 box tests per fetch that share the node's per-axis setup.
// Traversal: a group = (first interior child node, mask of its hit slots still to visit); a step pops one
// slot from the current group (pushing the rest on a short per-lane register stack), fetches that node,
// tests its 8 child boxes, tests its hit leaf triangles (one triangle per leaf slot, a wave-uniform loop
// like the skip walk's) and makes the hit interior children the next group; an empty group pops the
// stack.  The box test is conservative: the quantised planes contain the exact child box (built outward)
// and the interval is widened by the float error of t = q * (s / d) + (o - org) / d (relative 4 ulp as in
// box_test, and per axis 2^-22 |(o - org) / d| for the rounding of that term, folded into the offsets) --
// a superset of the exact test, so with the same triangle tests and tie rule the results are those of every
// other walk.  (One bound for all axes was tried first: an axis the ray is nearly parallel to has a huge
// |(o - org) / d|, and that bound opened every box of the tree for such rays -- 100x slower walks.)
// The stack holds one group per level below the root, so a tree of depth <= kWideStack never overflows;
// a deeper tree is not used (rs_scene::wide_on: the walks take the skip pointers) -- a fallback walk after
// the wide one doubled the per-lane kernels' code and register pressure (scratch inside the walk loops).
#ifndef RS_WIDE_STACK
#define RS_WIDE_STACK 8
#endif
constexpr int kWideStack = RS_WIDE_STACK;
struct WideStack {
    uint32_t s[kWideStack];   // s[0] = top: base << 8 | mask
    int n;
    uint32_t lost;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int k = 0; k < kWideStack; ++k) s[k] = 0u;
        n = 0; lost = 0u;
    }
    __device__ __forceinline__ void push(bool c, uint32_t v) {
        lost |= (c & (n == kWideStack)) ? 1u : 0u;
#pragma unroll
        for (int k = kWideStack - 1; k > 0; --k) s[k] = c ? s[k - 1] : s[k];
        s[0] = c ? v : s[0];
        n = c ? (n < kWideStack ? n + 1 : n) : n;
    }
    __device__ __forceinline__ uint32_t pop(bool c) {
        const uint32_t top = s[0];
#pragma unroll
        for (int k = 0; k < kWideStack - 1; ++k) s[k] = c ? s[k + 1] : s[k];
        n = c ? n - 1 : n;
        return top;
    }
};
__device__ __forceinline__ float ubyte_f(uint32_t w, int k) { return (float)((w >> (8 * k)) & 0xffu); }
// the 8 child boxes of node (w0..w4) against the ray; bit c = slot c hit (valid slots only)
__device__ __forceinline__ uint32_t wide_hits(uint4 w0, uint4 w1, uint4 w2, uint4 w3, uint4 w4, vec3 o, vec3 inv,
                                              float tnear, float tfar, vec3 ew = vec3{0.0f, 0.0f, 0.0f}) {
    const uint32_t eb = w0.w;
    const vec3 s = mk(__uint_as_float((eb & 0xffu) << 23), __uint_as_float(((eb >> 8) & 0xffu) << 23),
                      __uint_as_float(((eb >> 16) & 0xffu) << 23));
    const vec3 a = mk(s.x * inv.x, s.y * inv.y, s.z * inv.z);                 // exact (power-of-two scale)
    const vec3 b = mk((__uint_as_float(w0.x) - o.x) * inv.x, (__uint_as_float(w0.y) - o.y) * inv.y,
                      (__uint_as_float(w0.z) - o.z) * inv.z);
    // per axis the near (far) t lowered (raised) by 2^-22 |b|: the rounding of b and of b -+ that bound
    // (an axis the ray is almost parallel to has a huge |b| and widens only itself)
    // (+ ew: the closest-hit walks' box margin, rs_wide.h box_epsilon; 0 for the any-hit walks)
    const float ex = 2.384185791015625e-07f * fabsf(b.x) + ew.x, ey = 2.384185791015625e-07f * fabsf(b.y) + ew.y,
                ez = 2.384185791015625e-07f * fabsf(b.z) + ew.z;
    const vec3 bn = mk(b.x - ex, b.y - ey, b.z - ez), bf = mk(b.x + ex, b.y + ey, b.z + ez);
    // near / far planes per axis by the direction's sign (lo bytes near for a positive direction)
    const bool px = inv.x >= 0.0f, py = inv.y >= 0.0f, pz = inv.z >= 0.0f;
    const uint32_t nx0 = px ? w1.z : w3.x, nx1 = px ? w1.w : w3.y, fx0 = px ? w3.x : w1.z, fx1 = px ? w3.y : w1.w;
    const uint32_t ny0 = py ? w2.x : w3.z, ny1 = py ? w2.y : w3.w, fy0 = py ? w3.z : w2.x, fy1 = py ? w3.w : w2.y;
    const uint32_t nz0 = pz ? w2.z : w4.x, nz1 = pz ? w2.w : w4.y, fz0 = pz ? w4.x : w2.z, fz1 = pz ? w4.y : w2.w;
    const float lo_k = 1.0f - 4.0f * FLT_EPSILON, hi_k = 1.0f + 4.0f * FLT_EPSILON;
    uint32_t hits = 0u;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int k = c & 3;
        const uint32_t qnx = c < 4 ? nx0 : nx1, qny = c < 4 ? ny0 : ny1, qnz = c < 4 ? nz0 : nz1;
        const uint32_t qfx = c < 4 ? fx0 : fx1, qfy = c < 4 ? fy0 : fy1, qfz = c < 4 ? fz0 : fz1;
        const float tnx = fmaf(ubyte_f(qnx, k), a.x, bn.x), tny = fmaf(ubyte_f(qny, k), a.y, bn.y);
        const float tnz = fmaf(ubyte_f(qnz, k), a.z, bn.z);
        const float tfx = fmaf(ubyte_f(qfx, k), a.x, bf.x), tfy = fmaf(ubyte_f(qfy, k), a.y, bf.y);
        const float tfz = fmaf(ubyte_f(qfz, k), a.z, bf.z);
        const float t0 = fmaxf(fmaxf(fmaxf(tnear, tnx), tny), tnz);
        const float t1 = fminf(fminf(fminf(tfar, tfx), tfy), tfz);
        hits |= (t0 * lo_k <= t1 * hi_k) ? (1u << c) : 0u;
    }
    const uint32_t nv = w0.w >> 28;
    return hits & ((1u << nv) - 1u);
}
// Stats (rs_debug_trace only): *stats = node fetches << 16 | triangle tests of this lane's walk
template <bool Any, bool Stats = false, bool NoTri = false>
__device__ __forceinline__ void wide_walk(const DevScene& S, bool active, vec3 o, vec3 d, vec3 inv, float tnear,
                                          float tfar, Hit& h, uint32_t& occ, uint32_t& lost, uint32_t* stats = nullptr) {
    uint32_t gb = 0u, gm = active ? 1u : 0u;       // root group: node 0, slot 0
    uint32_t n_fetch = 0u, n_tri = 0u;
    const vec3 ew = Any ? mk(0.0f, 0.0f, 0.0f) : box_margin(S, inv);
    WideStack st;
    st.init();
    while (__ballot(gm != 0u) != 0) {
        if (Stats) n_fetch += gm != 0u ? 1u : 0u;
        const bool live = gm != 0u;
        const uint32_t slot = (uint32_t)__builtin_ctz(gm | 0x100u);
        const uint32_t node = live ? gb + slot : 0u;
        const uint32_t rest = gm & (gm - 1u);
        st.push(live & (rest != 0u), (gb << 8) | rest);
        const uint4* P = S.wnodes + 5 * (size_t)node;
        const uint4 w0 = P[0], w1 = P[1], w2 = P[2], w3 = P[3], w4 = P[4];
        const float tf = Any ? tfar : h.t;
        uint32_t hits = live ? wide_hits(w0, w1, w2, w3, w4, o, inv, tnear, tf, ew) : 0u;
        const uint32_t ni = (w0.w >> 24) & 0xfu;
        uint32_t tm = NoTri ? 0u : hits >> ni;      // leaf slots ni.. -> triangles tri_base + (slot - ni)
        const uint32_t tb = w1.y;
        while (__ballot(tm != 0u && (!Any || occ == 0u)) != 0) {
            const bool want = tm != 0u && (!Any || occ == 0u);
            if (Stats) n_tri += want ? 1u : 0u;
            const uint32_t j = (uint32_t)__builtin_ctz(tm | 0x100u);
            tm &= tm - 1u;
            const float4* T = S.wtris + 3 * (size_t)(want ? tb + j : 0u);
            const float4 T0 = T[0];
            float t, u, v;
            const bool hh = want & tri_test_nb(T0, T[1], T[2], o, d, tnear, Any ? tfar : h.t, t, u, v);
            if (Any) {
                occ = hh ? 1u : occ;
            } else {
                const int prim = __float_as_int(T0.w);
                const bool better = hh & (h.prim < 0 || t < h.t || (t == h.t && prim < h.prim));
                h.t = better ? t : h.t; h.u = better ? u : h.u; h.v = better ? v : h.v;
                h.prim = better ? prim : h.prim;
            }
        }
        const uint32_t ngm = (Any && occ) ? 0u : (hits & ((1u << ni) - 1u));
        const bool pop = live & (ngm == 0u) & (st.n > 0) & !(Any && occ);
        const uint32_t top = st.pop(pop);
        gb = !live ? gb : (ngm ? w1.x : (pop ? top >> 8 : 0u));
        gm = !live ? 0u : (ngm ? ngm : (pop ? top & 0xffu : 0u));
        if (Any && occ) st.n = 0;
    }
    lost = st.lost;
    if (Stats) *stats = (n_fetch << 16) | (n_tri & 0xffffu);
}

template <bool Wide>
__device__ __forceinline__ bool occluded_lane(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    if (!Wide) return occluded_lane_from(S, active ? 0u : 0xffffffffu, o, d, inv, tnear, tfar);
    uint32_t occ = 0u, lost = 0u;
    Hit h;
    wide_walk<true>(S, active, o, d, inv, tnear, tfar, h, occ, lost);   // lost == 0: depth <= kWideStack
    return occ != 0u;
}
// A list of n any-hit rays walked by one wave on the 8-wide tree, each lane taking the list's next ray when its own
// walk ends (Aila & Laine's persistent "while-while" with dynamic fetch): the rays of a 64-ray batch differ in
// walk length (C3 shadow rays: mean 12.8 node fetches, batch maximum 27; scripts/bvh_lab.cpp DUMP_ITERS), so a
// batch-at-a-time loop idles half its lanes.  Lanes are refilled when at least RS_REFILL_IDLE of them are idle
// (one round of ray loads serves them all; a refill per finished ray would add a load latency to most steps), or
// when every lane is.  ray(j, o, d, tfar) loads ray j; done(j, occ) records its answer.  The box and triangle tests
// are wide_walk<true>'s, so every ray's answer is the one wide_walk gives it -- only the lane and the time differ.
#ifndef RS_REFILL_IDLE
#define RS_REFILL_IDLE 8
#endif
template <class RayF, class DoneF>
__device__ __forceinline__ void occluded_wide_list(const DevScene& S, uint32_t n, float tnear, RayF ray, DoneF done) {
    const uint32_t lane = __lane_id();
    uint32_t j = lane, next = 64u;                 // this lane's ray; the list's next unassigned ray (wave-uniform)
    vec3 o = mk(0.0f, 0.0f, 0.0f), d = mk(1.0f, 1.0f, 1.0f), inv = mk(1.0f, 1.0f, 1.0f);
    float tfar = 0.0f;
    uint32_t gb = 0u, gm = 0u, occ = 0u;
    WideStack st;
    st.init();
    if (j < n) {
        ray(j, o, d, tfar);
        inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        gm = 1u;
    }
    while (true) {
        const uint64_t im = __ballot(gm == 0u);
        const uint32_t nidle = (uint32_t)__popcll(im);
        if (next < n && (nidle >= (uint32_t)RS_REFILL_IDLE || nidle == 64u)) {
            const uint32_t nj = next + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0u));
            next += nidle;
            if (gm == 0u && nj < n) {
                j = nj;
                ray(j, o, d, tfar);
                inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
                gb = 0u; gm = 1u; occ = 0u;
                st.n = 0;
            }
        }
        if (__ballot(gm != 0u) == 0) break;        // every lane idle and the list drained
        const bool live = gm != 0u;
        const uint32_t slot = (uint32_t)__builtin_ctz(gm | 0x100u);
        const uint32_t node = live ? gb + slot : 0u;
        const uint32_t rest = gm & (gm - 1u);
        st.push(live & (rest != 0u), (gb << 8) | rest);
        const uint4* P = S.wnodes + 5 * (size_t)node;
        const uint4 w0 = P[0], w1 = P[1], w2 = P[2], w3 = P[3], w4 = P[4];
        const uint32_t hits = live ? wide_hits(w0, w1, w2, w3, w4, o, inv, tnear, tfar) : 0u;
        const uint32_t ni = (w0.w >> 24) & 0xfu;
        uint32_t tm = hits >> ni;                  // leaf slots ni.. -> triangles tri_base + (slot - ni)
        const uint32_t tb = w1.y;
        while (__ballot(tm != 0u && occ == 0u) != 0) {
            const bool want = tm != 0u && occ == 0u;
            const uint32_t jj = (uint32_t)__builtin_ctz(tm | 0x100u);
            tm &= tm - 1u;
            const float4* T = S.wtris + 3 * (size_t)(want ? tb + jj : 0u);
            float t, u, v;
            const bool hh = want & tri_test_nb(T[0], T[1], T[2], o, d, tnear, tfar, t, u, v);
            occ = hh ? 1u : occ;
        }
        const uint32_t ngm = occ ? 0u : (hits & ((1u << ni) - 1u));
        const bool pop = live & (ngm == 0u) & (st.n > 0) & (occ == 0u);
        const uint32_t top = st.pop(pop);
        gb = !live ? gb : (ngm ? w1.x : (pop ? top >> 8 : 0u));
        gm = !live ? 0u : (ngm ? ngm : (pop ? top & 0xffu : 0u));
        if (occ) st.n = 0;
        if (live && gm == 0u) done(j, occ != 0u);
    }
}
template <bool Wide>
__device__ __forceinline__ Hit closest_lane(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    const vec3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    Hit h; h.t = tfar; h.u = 0; h.v = 0; h.prim = -1;
    if (!Wide) {
        closest_lane_from(S, active ? 0u : 0xffffffffu, o, d, inv, tnear, h);
        return h;
    }
    uint32_t occ = 0u, lost = 0u;
    wide_walk<false>(S, active, o, d, inv, tnear, tfar, h, occ, lost);   // lost == 0: depth <= kWideStack
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
    const MarginO mo = margin_origins(S, o);
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
        const bool hb = at && box_test_m(a, b, mo.lo, mo.hi, inv, tnear, h.t);
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
    if (!trav_lane(T)) {
        occluded_wave_multi<K>(S, active, o, d, tnear, tfar, occ);
    } else {   // one walk after the other (measured faster than interleaving the K walks, and than one
               // loop running a lane's walks back to back: that spilled the hot loop, 2.5x slower on C3)
#pragma unroll
        for (int k = 0; k < K; ++k) occ[k] = occluded_lane<trav_wide(T)>(S, active[k], o, d[k], tnear, tfar[k]);
    }
}
template <int T>
__device__ __forceinline__ bool trace_any(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    if (!trav_lane(T)) return occluded_wave(S, active, o, d, tnear, tfar);
    return occluded_lane<trav_wide(T)>(S, active, o, d, tnear, tfar);
}
template <int T>
__device__ __forceinline__ Hit trace_closest(const DevScene& S, bool active, vec3 o, vec3 d, float tnear, float tfar) {
    if (!trav_lane(T)) return closest_wave(S, active, o, d, tnear, tfar);
    return closest_lane<trav_wide(T)>(S, active, o, d, tnear, tfar);
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
