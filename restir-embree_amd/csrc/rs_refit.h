// rs_refit.h -- in-place BVH refit for moving geometry (device code shared by rs_bvh_build.hip and
// the fused update launch in restir_capi.hip).
//
// The topology stays; every node's box is recomputed from the new vertex positions exactly as the
// builders compute it (per-triangle min/max of the three vertices, unions by fminf/fmaxf -- order
// independent), and the leaf triangles are rewritten from the new positions with the same operations
// as k_ploc_emit.  Since the box test is conservative and the closest-hit tie rule does not depend on
// visit order, a refit tree answers every query bit-identically to a freshly built one
// (tests/test_gpu_parity.py::test_update_positions_refit_matches_fresh_scene).
//
// Nodes are processed deepest level first; an interior node's children (i + 1 and the left child's
// skip) sit exactly one level deeper.  The plan (node ids grouped by depth) is computed once per
// topology on the host (bvh_refit_plan); large levels get a multi-workgroup launch each, runs of small
// levels share one single-workgroup launch with a workgroup barrier between levels (one CU: global
// writes are visible to the workgroup after the barrier).
//
// The 8-wide tree (rs_wide.h layout) is refit the same way: its topology (breadth-first levels, each node's
// slots) stays, every node's 8 child boxes are recomputed bottom-up from the new positions -- triangle slots
// from their vertices, interior slots from the child node's EXACT box (kept beside the tree, `box`, so that
// the outward rounding does not compound level over level) -- and re-quantised with the builder's own
// encoder (rs_wide.h wide_encode: outward, exact), so the walk's box test stays a superset of the exact one.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>
#include "rs_wide.h"

namespace rs {

constexpr int kWideLevels = RS_WIDE_STACK + 1;   // a tree walked by the 8-entry stack has <= 9 levels

// 8-wide tree of the per-lane walks (built on the GPU by rs_wide_build.hip, walked by rs_scene.h; layout
// in rs_wide.h).  Device allocations owned by the scene.
struct WideBvh {
    uint4* nodes = nullptr;      // 5 per node
    float4* tris = nullptr;      // 3 per wide-leaf triangle
    float4* box = nullptr;       // 2 per node: its exact box (lo, hi), the refit's input for the parent
    uint32_t n_nodes = 0;
    uint32_t n_tris = 0;
    int depth = 0;               // deepest level (root = 0)
    int lvl[kWideLevels + 1] = {};   // breadth-first level offsets: level L = nodes [lvl[L], lvl[L + 1])
    int status = 0;              // why there is no tree (include/restir_c.h RS_WIDE_*): 0 live
};

// Workgroup size of the refits and of the per-update kernel (k_scene_update).  Updates run on the next frame's
// lane beside earlier frames' passes, which hold every CU: a workgroup of 1024 threads needs 16 free wave slots
// on one CU at once and waited for the passes' tails to be dispatched (C5: 0.68 ms per update under the profiler)
#ifndef RS_REFIT_BLOCK
#define RS_REFIT_BLOCK 256
#endif
constexpr int kRefitBlock = RS_REFIT_BLOCK;
constexpr int kRefitSmall = 4096;                // levels up to this many nodes go to the 1-block batch

__device__ __forceinline__ void refit_node(float4* nodes, float4* tris, const float* __restrict__ pos, int i) {
    const float4 a = nodes[2 * i], b = nodes[2 * i + 1];
    const int leaf = __float_as_int(b.w);
    float l[3], h[3];
    if (leaf >= 0) {
        const int first = leaf >> 3, cnt = (leaf & 7) + 1;
        l[0] = l[1] = l[2] = INFINITY; h[0] = h[1] = h[2] = -INFINITY;
        for (int j = 0; j < cnt; ++j) {
            const int k = first + j;
            const int prim = __float_as_int(tris[3 * k].w);
            const float* p = pos + 9 * (size_t)prim;
            for (int ax = 0; ax < 3; ++ax) {
                l[ax] = fminf(l[ax], fminf(fminf(p[ax], p[3 + ax]), p[6 + ax]));
                h[ax] = fmaxf(h[ax], fmaxf(fmaxf(p[ax], p[3 + ax]), p[6 + ax]));
            }
            const float v0x = p[0], v0y = p[1], v0z = p[2];
            tris[3 * k] = make_float4(v0x, v0y, v0z, __int_as_float(prim));
            tris[3 * k + 1] = make_float4(p[3] - v0x, p[4] - v0y, p[5] - v0z, 0.0f);
            tris[3 * k + 2] = make_float4(p[6] - v0x, p[7] - v0y, p[8] - v0z, 0.0f);
        }
    } else {
        const int L = i + 1, R = __float_as_int(nodes[2 * L].w);
        const float4 al = nodes[2 * L], ah = nodes[2 * L + 1], bl = nodes[2 * R], bh = nodes[2 * R + 1];
        l[0] = fminf(al.x, bl.x); l[1] = fminf(al.y, bl.y); l[2] = fminf(al.z, bl.z);
        h[0] = fmaxf(ah.x, bh.x); h[1] = fmaxf(ah.y, bh.y); h[2] = fmaxf(ah.z, bh.z);
    }
    nodes[2 * i] = make_float4(l[0], l[1], l[2], a.w);
    nodes[2 * i + 1] = make_float4(h[0], h[1], h[2], b.w);
}

// levels [l0, l1) of the plan (one workgroup walks them with barriers in between)
__device__ __forceinline__ void refit_levels(float4* nodes, float4* tris, const float* __restrict__ pos,
                                             const int* __restrict__ order, const int* __restrict__ lvl_off,
                                             int l0, int l1, int block, int nblocks) {
    for (int lv = l0; lv < l1; ++lv) {
        const int b = lvl_off[lv], e = lvl_off[lv + 1];
        for (int q = b + block * kRefitBlock + threadIdx.x; q < e; q += nblocks * kRefitBlock)
            refit_node(nodes, tris, pos, order[q]);
        if (lv + 1 < l1) __syncthreads();
    }
}
// launch batches: a level with more than kRefitSmall nodes gets its own multi-workgroup launch, runs
// of small levels share one single-workgroup launch
struct RefitBatch { int l0, l1, blocks; };
inline std::vector<RefitBatch> refit_batches(const std::vector<int>& lvl_off) {
    std::vector<RefitBatch> out;
    const int nl = (int)lvl_off.size() - 1;
    int l = 0;
    while (l < nl) {
        const int n = lvl_off[l + 1] - lvl_off[l];
        if (n > kRefitSmall) {
            out.push_back({l, l + 1, (n + kRefitBlock - 1) / kRefitBlock});
            ++l;
        } else {
            int e = l + 1;
            while (e < nl && lvl_off[e + 1] - lvl_off[e] <= kRefitSmall) ++e;
            out.push_back({l, e, 1});
            l = e;
        }
    }
    return out;
}


// ---------------------------------------------------------------- 8-wide tree refit
struct WideRefitArgs {
    uint4* nodes; float4* tris; float4* box; const float* pos;
    int lvl[kWideLevels + 1];
    int l_deep, l_top;           // levels l_deep down to l_top (inclusive), deepest first; l_deep < l_top: none
};
__device__ __forceinline__ void wide_refit_node(const WideRefitArgs& A, uint32_t j) {
    const uint4 w0 = A.nodes[5 * (size_t)j], w1 = A.nodes[5 * (size_t)j + 1];
    const int ni = (int)((w0.w >> 24) & 0xfu), nv = (int)(w0.w >> 28);
    const uint32_t cb = w1.x, tb = w1.y;
    WBox kb[8];
    for (int i = 0; i < nv; ++i) {
        if (i < ni) {
            const float4 l = A.box[2 * (size_t)(cb + i)], h = A.box[2 * (size_t)(cb + i) + 1];
            kb[i] = WBox{{l.x, l.y, l.z}, {h.x, h.y, h.z}};
        } else {
            const size_t t = tb + (uint32_t)(i - ni);
            const int prim = __float_as_int(A.tris[3 * t].w);
            const float* p = A.pos + 9 * (size_t)prim;
            bool fin = true;
            for (int a = 0; a < 3; ++a) {
                kb[i].lo[a] = w_min(w_min(p[a], p[3 + a]), p[6 + a]);
                kb[i].hi[a] = w_max(w_max(p[a], p[3 + a]), p[6 + a]);
                fin = fin && isfinite(kb[i].lo[a]) && isfinite(kb[i].hi[a]);
            }
            // a triangle with a non-finite vertex can never be hit (the triangle test's arithmetic turns NaN,
            // DESIGN.md §3.9); like k_prim_bounds it gets a point box at the origin, so every node above it
            // stays encodable and its planes stay a superset of the finite triangles below
            if (!fin)
                for (int a = 0; a < 3; ++a) kb[i].lo[a] = kb[i].hi[a] = 0.0f;
            const float v0x = p[0], v0y = p[1], v0z = p[2];
            A.tris[3 * t] = make_float4(v0x, v0y, v0z, __int_as_float(prim));
            A.tris[3 * t + 1] = make_float4(p[3] - v0x, p[4] - v0y, p[5] - v0z, 0.0f);
            A.tris[3 * t + 2] = make_float4(p[6] - v0x, p[7] - v0y, p[8] - v0z, 0.0f);
        }
    }
    uint32_t w[20];
    WBox u;
    // every child box is finite now (point boxes above); encoding can only fail for coordinates near FLT_MAX
    // (no power-of-two frame <= 2^127 spans them), where the node keeps its previous planes
    if (!wide_encode(kb, nv, ni, cb, tb, w, &u)) return;
    uint4* P = A.nodes + 5 * (size_t)j;
    for (int k = 0; k < 5; ++k) P[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
    A.box[2 * (size_t)j] = make_float4(u.lo[0], u.lo[1], u.lo[2], 0.0f);
    A.box[2 * (size_t)j + 1] = make_float4(u.hi[0], u.hi[1], u.hi[2], 0.0f);
}
// levels l_deep .. l_top by `nblocks` workgroups of kRefitBlock threads (one workgroup: barriers between levels)
__device__ __forceinline__ void wide_refit_levels(const WideRefitArgs& A, int block, int nblocks) {
    for (int lv = A.l_deep; lv >= A.l_top; --lv) {
        for (int q = A.lvl[lv] + block * kRefitBlock + (int)threadIdx.x; q < A.lvl[lv + 1]; q += nblocks * kRefitBlock)
            wide_refit_node(A, (uint32_t)q);
        if (lv > A.l_top) __syncthreads();
    }
}
// launch batches, deepest first: a level with more than kRefitSmall nodes alone over many workgroups, runs
// of small levels in one workgroup
struct WideBatch { int l_deep, l_top, blocks; };
inline std::vector<WideBatch> wide_refit_batches(const WideBvh& w) {
    std::vector<WideBatch> out;
    int l = w.depth;
    while (l >= 0) {
        const int n = w.lvl[l + 1] - w.lvl[l];
        if (n > kRefitSmall) { out.push_back({l, l, (n + kRefitBlock - 1) / kRefitBlock}); --l; continue; }
        int e = l;
        while (e - 1 >= 0 && w.lvl[e] - w.lvl[e - 1] <= kRefitSmall) --e;
        out.push_back({l, e, 1});
        l = e - 1;
    }
    return out;
}
inline WideRefitArgs wide_refit_args(const WideBvh& w, const float* pos, int l_deep, int l_top) {
    WideRefitArgs A{w.nodes, w.tris, w.box, pos, {}, l_deep, l_top};
    for (int i = 0; i <= kWideLevels; ++i) A.lvl[i] = w.lvl[i];
    return A;
}

}  // namespace rs
