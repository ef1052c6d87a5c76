// rs_wide.h -- the 8-wide tree of the per-lane walks: its node encoding (shared by the host restatement and
// the GPU builder / refit, rs_wide_build.hip) and the host restatement of the build -- a top-down SAH source
// tree and the SAH-optimal collapse -- that the GPU builder reproduces bit for bit (tests/test_wide_bvh.py,
// tests/test_gpu_parity.py::test_wide_tree_gpu_equals_host).  Plain C++ apart from RS_HD: the header is also
// compiled by g++ for tests/cpp/wide_harness.cpp.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#ifndef RS_WIDE_STACK
#define RS_WIDE_STACK 8   // the walk's register stack (rs_scene.h kWideStack, same default): deepest tree walked
#endif
#if defined(__HIP__)
#define RS_HD __host__ __device__
#else
#define RS_HD
#endif

namespace rs {
// ============================================================================================
// 8-wide tree for the per-lane walks (rs_scene.h "8-wide per-lane walks").  Collapsed on the host from
// the PLOC tree (its merge links), once per build: every wide node is a PLOC internal node whose up to 8
// children come from opening, largest surface area first, the internal children of the node until there
// are 8 (Wald et al. 2008 / Ylitie et al. 2017's greedy collapse).  Leaves hold ONE triangle.  Layout
// (breadth-first, so a node's interior children are consecutive nodes and its leaf triangles consecutive
// wide-leaf triangles): interior children occupy slots 0..ni-1, leaf children slots ni..nv-1.
// Node = 5 x uint4 (80 B):
//   w0 = origin o.xyz (float), ex | ey << 8 | ez << 16 | ni << 24 | nv << 28
//   w1 = child_base, tri_base, qlo.x[0..3], qlo.x[4..7]      (q: one byte per slot)
//   w2 = qlo.y[0..3], qlo.y[4..7], qlo.z[0..3], qlo.z[4..7]
//   w3 = qhi.x[0..3], qhi.x[4..7], qhi.y[0..3], qhi.y[4..7]
//   w4 = qhi.z[0..3], qhi.z[4..7], 0, 0
// A child's box is o + q * s per axis, s = 2^(e - 127); o is a multiple of s, so every plane o + q*s is an
// exact float, and the planes are rounded OUTWARD (lo down, hi up) from the exact child box: the walk's
// box test is a superset of the exact one (results cannot change, rs_scene.h).
// ============================================================================================
namespace wide {
struct WBox { float lo[3], hi[3]; };
inline double exp2i(int e) { return std::ldexp(1.0, e); }
inline int h_f2i(float f) { int i; std::memcpy(&i, &f, 4); return i; }
inline uint32_t h_f2u(float f) { uint32_t i; std::memcpy(&i, &f, 4); return i; }
RS_HD inline bool w_finite(float x) { return x - x == 0.0f; }
RS_HD inline float w_min(float a, float b) { return b < a ? b : a; }   // std::min / std::max
RS_HD inline float w_max(float a, float b) { return a < b ? b : a; }
// The closest-hit walks' box margin, in scene units: 2^-16 x the scene's largest |coordinate| (at least 1).
// Moller-Trumbore accepts a hit from its barycentrics, but the point o + t d of its t can lie outside the
// triangle's box by a few ulps of the coordinates (a ray through the shared edge of two triangles, C3: 2.5e-6 m at
// 10 m); along an axis the ray crosses slowly that is far beyond the slab test's 4-eps t margin, so a closest-hit
// walk could cull the box of the tie-winning triangle after finding its neighbour -- and which box that is depends
// on the tree (the oracle's binary and 8-wide trees disagreed on 1 of 8.3 M C3 4K primary rays).  The closest-hit
// slab tests widen every box by this margin (rs_scene.h box_test_m, wide_hits), so every tree returns the triangle
// test's own answer (ties: smaller t, then smaller index).  The any-hit (shadow) walks keep the exact boxes: a
// margin on them lets every ray from a flat layer's surface (walls, the C2 light layer) enter the layer's thin
// boxes, which cost the lockstep walk up to 3.8x (2^-16) and 3 % (2^-22) on C2.  oracle/restir_oracle.c restates it.
inline float box_epsilon(const float* pos, size_t nfloats) {
    float m = 1.0f;
    for (size_t i = 0; i < nfloats; ++i) {
        const float a = pos[i] < 0.0f ? -pos[i] : pos[i];
        if (w_finite(a) && a > m) m = a;
    }
    return m * (1.0f / 65536.0f);
}
// quantisation frame of one axis: s = 2^e >= extent / 255 and >= the float spacing at the box, o = a float
// multiple of s <= lo with o + 255 s >= hi; every child box [clo, chi] quantises OUTWARD to bytes ql, qh with
// o + ql s <= clo and o + qh s >= chi, all checked in double, where o, s and q are exact (the first k that
// satisfies every check is taken).  Host and device run the same double operations.
RS_HD inline bool wide_axis(float lo, float hi, const float* clo, const float* chi, int nv, int& e, float& o, uint8_t* ql,
                            uint8_t* qh) {
    const double ext = (double)hi - (double)lo;
    int k = -126;
    if (ext > 0) { int x; frexp(ext / 255.0, &x); k = x > -126 ? x : -126; }   // ext / 255 < 2^x
    const float big = w_max(fabsf(lo), fabsf(hi));
    if (big > 0) { int x; frexp((double)big, &x); k = k > x - 24 ? k : x - 24; }  // ulp(big) <= 2^(x-24)
    for (; k <= 127; ++k) {
        const double sd = ldexp(1.0, k);
        const float of = (float)(floor((double)lo / sd) * sd);
        const double od = (double)of;
        if (od > (double)lo || od + 255.0 * sd < (double)hi || floor(od / sd) * sd != od) continue;
        bool ok = true;
        for (int i = 0; i < nv && ok; ++i) {
            // estimate in double (the difference chi - od may round), then step to the exact outward byte:
            // od + q * sd is a multiple of sd no larger than the box, exact in double, so the tests are exact
            double a = floor(((double)clo[i] - od) / sd), b = ceil(((double)chi[i] - od) / sd);
            a = a < 0.0 ? 0.0 : (a > 255.0 ? 255.0 : a); b = b < 0.0 ? 0.0 : (b > 255.0 ? 255.0 : b);
            while (a > 0.0 && od + a * sd > (double)clo[i]) a -= 1.0;
            while (b < 255.0 && od + b * sd < (double)chi[i]) b += 1.0;
            ok = od + a * sd <= (double)clo[i] && od + b * sd >= (double)chi[i];
            ql[i] = (uint8_t)a; qh[i] = (uint8_t)b;
        }
        if (ok) { e = k; o = of; return true; }
    }
    return false;
}
// one wide node from its nv <= 8 child boxes (slots 0..ni-1 interior, ni..nv-1 triangles): the 20 words of
// the layout above; *u = the union of the child boxes.  false: a non-finite box, or no conservative frame.
RS_HD inline bool wide_encode(const WBox* kb, int nv, int ni, uint32_t child_base, uint32_t tri_base, uint32_t* w, WBox* u) {
    WBox b = kb[0];
    for (int i = 1; i < nv; ++i)
        for (int a = 0; a < 3; ++a) { b.lo[a] = w_min(b.lo[a], kb[i].lo[a]); b.hi[a] = w_max(b.hi[a], kb[i].hi[a]); }
    *u = b;
    int e[3] = {0, 0, 0};
    float o[3] = {0.0f, 0.0f, 0.0f};
    uint8_t qlo[3][8] = {}, qhi[3][8] = {};
    for (int a = 0; a < 3; ++a) {
        if (!w_finite(b.lo[a]) || !w_finite(b.hi[a])) return false;
        float clo[8], chi[8];
        for (int i = 0; i < nv; ++i) { clo[i] = kb[i].lo[a]; chi[i] = kb[i].hi[a]; }
        if (!wide_axis(b.lo[a], b.hi[a], clo, chi, nv, e[a], o[a], qlo[a], qhi[a])) return false;
    }
    auto pack = [](const uint8_t* q, int first) {
        return (uint32_t)q[first] | ((uint32_t)q[first + 1] << 8) | ((uint32_t)q[first + 2] << 16) | ((uint32_t)q[first + 3] << 24);
    };
    auto bits = [](float f) { union { float f; uint32_t u; } x; x.f = f; return x.u; };
    w[0] = bits(o[0]); w[1] = bits(o[1]); w[2] = bits(o[2]);
    w[3] = (uint32_t)(e[0] + 127) | ((uint32_t)(e[1] + 127) << 8) | ((uint32_t)(e[2] + 127) << 16) | ((uint32_t)ni << 24) |
           ((uint32_t)nv << 28);
    w[4] = child_base; w[5] = tri_base; w[6] = pack(qlo[0], 0); w[7] = pack(qlo[0], 4);
    w[8] = pack(qlo[1], 0); w[9] = pack(qlo[1], 4); w[10] = pack(qlo[2], 0); w[11] = pack(qlo[2], 4);
    w[12] = pack(qhi[0], 0); w[13] = pack(qhi[0], 4); w[14] = pack(qhi[1], 0); w[15] = pack(qhi[1], 4);
    w[16] = pack(qhi[2], 0); w[17] = pack(qhi[2], 4); w[18] = 0u; w[19] = 0u;
    return true;
}
}  // namespace wide
using namespace wide;

// Top-down SAH source tree for the collapse (the PLOC tree stays the binary walks' and the refit's): binned
// SAH (32 bins per axis over the centroid bounds) above kSweepMax triangles, a full sweep over the sorted
// centroids below (C3 lab: thresholds 256 / 2048 / 8192 give the same walk counts) (cost = the children's
// half areas x their triangle counts).  Every choice is a function of the node's triangle SET (ties: axis,
// then position, then triangle index), so the tree does not depend on the order of the arrays -- the GPU
// builder (rs_wide_build.hip) builds the same tree level by level.  Output in the PLOC arrays'
// shape: ids < n triangles (box, hi.w = triangle bits), ids >= n internal (lo.w / hi.w = child id bits).
// pos: 9 floats per triangle, all finite (callers check: NaN centroids would break the sorts' ordering;
// the GPU builder and the test harness build no wide tree for non-finite geometry).  Returns the root id.
inline int build_sah_host(const float* pos, int n, std::vector<float>& nlo, std::vector<float>& nhi,
                          int kSweepMax = 256) {
    constexpr int kBins = 32;
    const size_t total = 2 * (size_t)n - 1;
    nlo.assign(4 * total, 0.0f); nhi.assign(4 * total, 0.0f);
    std::vector<WBox> tb(n);
    std::vector<float> cen(3 * (size_t)n);
    for (int t = 0; t < n; ++t) {
        const float* p = pos + 9 * (size_t)t;
        for (int a = 0; a < 3; ++a) {
            tb[t].lo[a] = std::min(std::min(p[a], p[3 + a]), p[6 + a]);
            tb[t].hi[a] = std::max(std::max(p[a], p[3 + a]), p[6 + a]);
            cen[3 * (size_t)t + a] = 0.5f * tb[t].lo[a] + 0.5f * tb[t].hi[a];
            nlo[4 * (size_t)t + a] = tb[t].lo[a]; nhi[4 * (size_t)t + a] = tb[t].hi[a];
        }
        nlo[4 * (size_t)t + 3] = 0.0f; nhi[4 * (size_t)t + 3] = [&] { float f; std::memcpy(&f, &t, 4); return f; }();
    }
    if (n == 1) return 0;
    auto grow = [](WBox& b, const WBox& c) {
        for (int a = 0; a < 3; ++a) { b.lo[a] = std::min(b.lo[a], c.lo[a]); b.hi[a] = std::max(b.hi[a], c.hi[a]); }
    };
    auto empty = [] { WBox b; for (int a = 0; a < 3; ++a) { b.lo[a] = 3.0e38f; b.hi[a] = -3.0e38f; } return b; };
    auto half_area = [](const WBox& b) {
        const double x = (double)b.hi[0] - b.lo[0], y = (double)b.hi[1] - b.lo[1], z = (double)b.hi[2] - b.lo[2];
        return x * y + y * z + z * x;
    };
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    std::vector<double> rarea(kSweepMax + 1);
    int next = n;
    struct Job { int first, count, id, parent, side; };
    std::vector<Job> st = {{0, n, -1, -1, 0}};
    int root = -1;
    auto link = [&](const Job& j, int id) {
        if (j.parent < 0) { root = id; return; }
        float f; std::memcpy(&f, &id, 4);
        (j.side ? nhi : nlo)[4 * (size_t)j.parent + 3] = f;
    };
    while (!st.empty()) {
        Job j = st.back();
        st.pop_back();
        if (j.count == 1) { link(j, idx[j.first]); continue; }
        const int id = next++;
        link(j, id);
        WBox nb = empty();
        for (int i = j.first; i < j.first + j.count; ++i) grow(nb, tb[idx[i]]);
        for (int a = 0; a < 3; ++a) { nlo[4 * (size_t)id + a] = nb.lo[a]; nhi[4 * (size_t)id + a] = nb.hi[a]; }
        int* I = idx.data() + j.first;
        int split = j.count / 2;
        if (j.count > kSweepMax) {               // binned SAH
            float clo[3] = {3.0e38f, 3.0e38f, 3.0e38f}, chi[3] = {-3.0e38f, -3.0e38f, -3.0e38f};
            for (int i = 0; i < j.count; ++i)
                for (int a = 0; a < 3; ++a) { clo[a] = std::min(clo[a], cen[3 * (size_t)I[i] + a]); chi[a] = std::max(chi[a], cen[3 * (size_t)I[i] + a]); }
            double best = 1e300; int bax = -1, bb = 0;
            for (int a = 0; a < 3; ++a) {
                if (!(chi[a] > clo[a])) continue;
                const double sc = kBins / ((double)chi[a] - clo[a]);
                WBox bx[kBins]; int cnt[kBins] = {};
                for (int b = 0; b < kBins; ++b) bx[b] = empty();
                for (int i = 0; i < j.count; ++i) {
                    const int b = std::min(kBins - 1, (int)(((double)cen[3 * (size_t)I[i] + a] - clo[a]) * sc));
                    ++cnt[b]; grow(bx[b], tb[I[i]]);
                }
                double ra[kBins]; int rc[kBins];
                WBox r = empty(); int c = 0;
                for (int b = kBins - 1; b >= 1; --b) { grow(r, bx[b]); c += cnt[b]; ra[b] = c ? half_area(r) : 0.0; rc[b] = c; }
                WBox l = empty(); c = 0;
                for (int b = 1; b < kBins; ++b) {
                    grow(l, bx[b - 1]); c += cnt[b - 1];
                    if (!c || !rc[b]) continue;
                    const double cost = half_area(l) * c + ra[b] * rc[b];
                    if (cost < best) { best = cost; bax = a; bb = b; }
                }
            }
            if (bax >= 0) {
                const double sc = kBins / ((double)chi[bax] - clo[bax]);
                int* mid = std::partition(I, I + j.count, [&](int t) {
                    return std::min(kBins - 1, (int)(((double)cen[3 * (size_t)t + bax] - clo[bax]) * sc)) < bb;
                });
                split = (int)(mid - I);
            } else {                             // every centroid equal: split at the middle of the triangle-index
                int mn = I[0], mx = I[0];        // range (a rule on the set, not on the array's order; both sides
                for (int i = 1; i < j.count; ++i) { mn = std::min(mn, I[i]); mx = std::max(mx, I[i]); }   // non-empty)
                const int mid = mn + (mx - mn) / 2;
                split = (int)(std::partition(I, I + j.count, [&](int t) { return t <= mid; }) - I);
            }
        } else {                                 // full sweep
            double best = 1e300; int bax = 0, bs = j.count / 2;
            auto by_axis = [&](int a) {
                std::sort(I, I + j.count, [&](int p, int q) {
                    const float cp = cen[3 * (size_t)p + a], cq = cen[3 * (size_t)q + a];
                    return cp < cq || (cp == cq && p < q);
                });
            };
            for (int a = 0; a < 3; ++a) {
                by_axis(a);
                WBox r = empty();
                for (int i = j.count - 1; i >= 1; --i) { grow(r, tb[I[i]]); rarea[i] = half_area(r); }
                WBox l = empty();
                for (int i = 1; i < j.count; ++i) {
                    grow(l, tb[I[i - 1]]);
                    const double cost = half_area(l) * i + rarea[i] * (j.count - i);
                    if (cost < best) { best = cost; bax = a; bs = i; }
                }
            }
            if (bax != 2) by_axis(bax);
            split = bs;
        }
        st.push_back({j.first + split, j.count - split, -1, id, 1});
        st.push_back({j.first, split, -1, id, 0});
    }
    return root;
}

// SAH-optimal collapse (Ylitie, Karras, Laine 2017, "Efficient incoherent ray traversal on GPUs through
// compressed wide BVHs", §3.2), with one triangle per leaf slot and a bound on the wide tree's depth (the
// walk's register stack holds one group per level: rs_scene.h kWideStack).  For binary node x, slot budget
// k <= 8 and height budget g (a wide node placed in a slot may have at most g levels of wide nodes below it):
//   triangle x:  S(x, k, g) = A(x) c_tri
//   S(x, 1, g) = N(x, g) = A(x) c_node + D(x, 8, g - 1)       (x as a wide node; infeasible for g < 0)
//   S(x, k, g) = min(S(x, k - 1, g), D(x, k, g)),  D(x, k, g) = min over a of S(l, a, g) + S(r, k - a, g)
// The root is N(root, depth budget).  plan() fills the tables bottom-up; kids() expands a wide node's choice.
struct SahCollapse {
    static constexpr int kG = 10;                // g = -1 .. 8
    int n = 0, gmax = 8;
    std::vector<float> S;                        // per node [g + 1][k - 1]
    std::vector<uint8_t> open, split;
    size_t at(int x, int g, int k) const { return ((size_t)x * kG + (size_t)(g + 1)) * 8 + (size_t)(k - 1); }
    bool plan(const float* nlo, const float* nhi, int n_, int root, float c_node, float c_tri, int depth_max) {
        n = n_; gmax = depth_max;
        if (gmax < 0 || gmax > kG - 2) return false;
        const size_t total = 2 * (size_t)n - 1;
        S.assign(total * kG * 8, 0.0f); open.assign(total * kG * 8, 0); split.assign(total * kG * 8, 0);
        auto area = [&](int c) { const float* a = nlo + 4 * (size_t)c; const float* z = nhi + 4 * (size_t)c;
            const float ex = z[0] - a[0], ey = z[1] - a[1], ez = z[2] - a[2]; return ex * ey + ey * ez + ez * ex; };
        const float inf = 3.0e38f;
        std::vector<std::pair<int, bool>> st = {{root, false}};   // post-order
        while (!st.empty()) {
            auto [x, done] = st.back();
            st.pop_back();
            if (x < n) { for (int g = -1; g <= gmax; ++g) for (int k = 1; k <= 8; ++k) S[at(x, g, k)] = area(x) * c_tri; continue; }
            const int l = h_f2i(nlo[4 * (size_t)x + 3]), r = h_f2i(nhi[4 * (size_t)x + 3]);
            if (l < 0 || r < 0 || (size_t)l >= total || (size_t)r >= total) return false;
            if (!done) { st.push_back({x, true}); st.push_back({l, false}); st.push_back({r, false}); continue; }
            float Dprev[8] = {};                     // D(x, ., g - 1)
            for (int g = -1; g <= gmax; ++g) {
                float D[8];
                for (int k = 2; k <= 8; ++k) {       // D(x, k, g): a slots to the left child, k - a to the right
                    float best = inf; int ba = 1;
                    for (int a = 1; a < k; ++a) {
                        const float v = S[at(l, g, a)] + S[at(r, g, k - a)];
                        if (v < best) { best = v; ba = a; }
                    }
                    D[k - 1] = best; split[at(x, g, k)] = (uint8_t)ba;
                }
                // N(x, g) needs D(x, 8, g - 1): computed in the previous g iteration (g - 1 >= -1), else infeasible
                float Nx = inf;
                if (g >= 0) {
                    const float d8 = Dprev[7];
                    Nx = d8 < inf ? area(x) * c_node + d8 : inf;
                }
                S[at(x, g, 1)] = Nx;
                for (int k = 2; k <= 8; ++k) {
                    const float prev = S[at(x, g, k - 1)];
                    const bool o = D[k - 1] < prev;
                    S[at(x, g, k)] = o ? D[k - 1] : prev;
                    open[at(x, g, k)] = o ? 1 : 0;
                }
                for (int k = 0; k < 8; ++k) Dprev[k] = D[k];
            }
        }
        return S[at(root, gmax, 1)] < inf || root < n;
    }
    void expand(const float* nlo, const float* nhi, int x, int k, int g, std::vector<int>& out, std::vector<int>& hb) const {
        while (x >= n && k > 1 && !open[at(x, g, k)]) --k;
        if (x < n || k == 1) { out.push_back(x); hb.push_back(g); return; }
        const int a = split[at(x, g, k)];
        expand(nlo, nhi, h_f2i(nlo[4 * (size_t)x + 3]), a, g, out, hb);
        expand(nlo, nhi, h_f2i(nhi[4 * (size_t)x + 3]), k - a, g, out, hb);
    }
    // children of wide node c built under height budget g; hb = each child's own height budget
    std::vector<int> kids(const float* nlo, const float* nhi, int c, int g, std::vector<int>& hb) const {
        std::vector<int> out;
        hb.clear();
        if (c < n) { out.push_back(c); hb.push_back(g); return out; }
        const int a = split[at(c, g - 1, 8)];
        expand(nlo, nhi, h_f2i(nlo[4 * (size_t)c + 3]), a, g - 1, out, hb);
        expand(nlo, nhi, h_f2i(nhi[4 * (size_t)c + 3]), 8 - a, g - 1, out, hb);
        return out;
    }
};

// nlo / nhi: the PLOC nodes as 4 floats each (ids < n: primitives, hi.w = triangle index bits; ids >= n:
// internal, lo.w / hi.w = left / right child id bits); out: 20 words per wide node.  collapse: 0 greedy
// (open the largest-area interior child until 8), 1 SAH-optimal within max_depth levels (SahCollapse,
// costs c_node / c_tri; falls back to greedy when it has no plan).  The CPU restatement the GPU builder
// (rs_wide_build.hip) is checked against (tests/cpp/wide_harness.cpp); no product path calls it.
inline int build_wide_host(const float* nlo, const float* nhi, int n, int root, std::vector<uint32_t>& out,
                           std::vector<int>& tri_prims, int& depth, std::string& err, int collapse = 0,
                           float c_node = 1.0f, float c_tri = 0.3f, int max_depth = 8,
                           std::vector<int>* slot_src = nullptr) {   // optional: 8 per node, the source node of each slot
    out.clear(); tri_prims.clear(); depth = 0;
    if (slot_src) slot_src->clear();
    if (n <= 0) return 0;
    auto is_prim = [&](int c) { return c < n; };
    auto box = [&](int c) { WBox b; const float* a = nlo + 4 * (size_t)c; const float* z = nhi + 4 * (size_t)c;
        for (int k = 0; k < 3; ++k) { b.lo[k] = a[k]; b.hi[k] = z[k]; } return b; };
    auto area = [&](int c) { const float* a = nlo + 4 * (size_t)c; const float* z = nhi + 4 * (size_t)c;
        const float ex = z[0] - a[0], ey = z[1] - a[1], ez = z[2] - a[2]; return ex * ey + ey * ez + ez * ex; };
    SahCollapse sah;
    // the plan's tables take 480 B per binary node (0.24 GB at C3's 248 k triangles): above 2^21 triangles
    // (~1 GB of tables), or without a plan inside the depth, the greedy collapse
    if (collapse == 1 && (n > (1 << 21) || !sah.plan(nlo, nhi, n, root, c_node, c_tri, max_depth)))
        collapse = 0;
    // triangles below every binary node (ids >= n; a primitive counts 1): a node's interior slots are ordered by it,
    // most first, so the walks' lowest-slot-first order enters the fuller subtrees first -- an any-hit ray meets an
    // occluder after fewer node fetches (scripts/bvh_lab.cpp ORDER: C3 shadow rays 13.86 -> 12.73 fetches)
    std::vector<int> ntri(n > 1 ? (size_t)n - 1 : 0, 0);
    if (n > 1) {
        std::vector<std::pair<int, bool>> ps = {{root, false}};
        while (!ps.empty()) {
            auto [x, done] = ps.back();
            ps.pop_back();
            if (x < n) continue;
            const int l = h_f2i(nlo[4 * (size_t)x + 3]), r = h_f2i(nhi[4 * (size_t)x + 3]);
            if (l < 0 || r < 0 || l >= 2 * n - 1 || r >= 2 * n - 1) { err = "wide BVH: bad child id"; return -1; }
            if (!done) { ps.push_back({x, true}); ps.push_back({l, false}); ps.push_back({r, false}); continue; }
            ntri[x - n] = (l < n ? 1 : ntri[l - n]) + (r < n ? 1 : ntri[r - n]);
        }
    }
    auto tri_count = [&](int c) { return c < n ? 1 : ntri[c - n]; };
    std::vector<int> queue = {root}, level = {0}, budget = {max_depth};   // wide node i = PLOC node queue[i]
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const int c = queue[qi];
        std::vector<int> kids, hb;
        if (collapse == 1) kids = sah.kids(nlo, nhi, c, budget[qi], hb);
        else {
            if (is_prim(c)) kids = {c};
            else kids = {h_f2i(nlo[4 * (size_t)c + 3]), h_f2i(nhi[4 * (size_t)c + 3])};
            while (kids.size() < 8) {
                int best = -1; float ba = -1.0f;
                for (int i = 0; i < (int)kids.size(); ++i)
                    if (!is_prim(kids[i]) && area(kids[i]) > ba) { ba = area(kids[i]); best = i; }
                if (best < 0) break;
                const int x = kids[best];
                kids.erase(kids.begin() + best);
                kids.push_back(h_f2i(nlo[4 * (size_t)x + 3]));
                kids.push_back(h_f2i(nhi[4 * (size_t)x + 3]));
            }
        }
        if (collapse != 1) std::stable_partition(kids.begin(), kids.end(), [&](int k) { return !is_prim(k); });
        if (collapse == 1) {                           // keep each slot's height budget with its child
            std::vector<int> order(kids.size());
            for (size_t i = 0; i < kids.size(); ++i) order[i] = (int)i;
            std::stable_partition(order.begin(), order.end(), [&](int i) { return !is_prim(kids[i]); });
            std::vector<int> k2, h2;
            for (int i : order) { k2.push_back(kids[i]); h2.push_back(hb[i]); }
            kids.swap(k2); hb.swap(h2);
        }
        int ni = 0;
        while (ni < (int)kids.size() && !is_prim(kids[ni])) ++ni;
        for (int i = 1; i < ni; ++i)                   // interior slots: most triangles first, ties in expansion order
            for (int j = i; j > 0 && tri_count(kids[j]) > tri_count(kids[j - 1]); --j) {
                std::swap(kids[j], kids[j - 1]);
                if (collapse == 1) std::swap(hb[j], hb[j - 1]);
            }
        const int nv = (int)kids.size();
        const uint32_t child_base = (uint32_t)queue.size(), tri_base = (uint32_t)tri_prims.size();
        for (int i = 0; i < ni; ++i) {
            queue.push_back(kids[i]); level.push_back(level[qi] + 1); depth = std::max(depth, level[qi] + 1);
            budget.push_back(collapse == 1 ? hb[i] : 0);
        }
        for (int i = ni; i < nv; ++i) tri_prims.push_back(h_f2i(nhi[4 * (size_t)kids[i] + 3]));
        WBox kb[8], u;
        for (int i = 0; i < nv; ++i) kb[i] = box(kids[i]);
        uint32_t w[20];
        if (!wide_encode(kb, nv, ni, child_base, tri_base, w, &u)) {
            bool fin = true;
            for (int a = 0; a < 3; ++a) fin = fin && w_finite(u.lo[a]) && w_finite(u.hi[a]);
            err = fin ? "wide BVH: no conservative quantisation" : "wide BVH: non-finite box";
            return -1;
        }
        out.insert(out.end(), w, w + 20);
        if (slot_src) for (int i = 0; i < 8; ++i) slot_src->push_back(i < nv ? kids[i] : -1);
        if (queue.size() >= (1u << 24)) { err = "wide BVH: too many nodes"; return -1; }
    }
    return 0;
}


}  // namespace rs
