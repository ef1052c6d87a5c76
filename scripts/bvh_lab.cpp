#include <chrono>
// bvh_lab.cpp -- offline BVH quality lab (analysis tooling, not product, not test).
// Builds candidate trees on the CPU for a dumped scene and replays the walk the GPU's per-lane kernels
// make (skip-pointer preorder, stackless, conservative slab test, leaf triangles tested in a wave-wide
// loop up to the largest leaf among the lanes), over primary rays and one shadow ray per pixel to a
// random point on a random emissive triangle (scripts/bvh_stats.py's ray set), in 8x8-pixel waves.
// Reports per ray: node visits, triangle tests; per wave: lockstep steps of the per-lane loop (max over
// lanes) and triangle-loop iterations (sum over steps of the max leaf count of the lanes in a hit leaf).
//
//   g++ -O3 -march=native -fopenmp -std=c++17 -o /tmp/bvh_lab scripts/bvh_lab.cpp
//   python scripts/bvh_lab.py            (dumps the scene, runs the builders, prints the table)
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>
#include "../restir-embree_amd/csrc/rs_wide.h"

struct V3 { float x, y, z; };
static inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static inline V3 vmin(V3 a, V3 b) { return {std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)}; }
static inline V3 vmax(V3 a, V3 b) { return {std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)}; }
static inline float comp(V3 a, int k) { return k == 0 ? a.x : (k == 1 ? a.y : a.z); }

struct Box {
    V3 lo{FLT_MAX, FLT_MAX, FLT_MAX}, hi{-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void add(V3 p) { lo = vmin(lo, p); hi = vmax(hi, p); }
    void add(const Box& b) { lo = vmin(lo, b.lo); hi = vmax(hi, b.hi); }
    float half_area() const {
        if (lo.x > hi.x) return 0.0f;
        V3 e = hi - lo;
        return e.x * e.y + e.y * e.z + e.z * e.x;
    }
};

struct Tri { V3 v0, v1, v2; };
static std::vector<Tri> g_tris;

// ---------------------------------------------------------------- binary build tree
struct BNode { Box b; int l = -1, r = -1; std::vector<int> prims; int cnt = 0; };
struct Tree { std::vector<BNode> n; int root = -1; };

static Box tri_box(int t) { Box b; b.add(g_tris[t].v0); b.add(g_tris[t].v1); b.add(g_tris[t].v2); return b; }

// ---- PLOC (the GPU builder's algorithm: Morton order, radius-r nearest neighbour by merged area, mutual merges)
static uint32_t expand10(uint32_t v) {
    v &= 0x3ffu;
    v = (v * 0x00010001u) & 0xFF0000FFu; v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u; v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
static Tree build_ploc(const std::vector<int>& prims, const std::vector<Box>& pbox, int radius) {
    const int n = (int)prims.size();
    Box cb;
    std::vector<V3> cen(n);
    for (int i = 0; i < n; ++i) { const Box& b = pbox[i]; cen[i] = (b.lo + b.hi) * 0.5f; cb.add(cen[i]); }
    std::vector<std::pair<uint64_t, int>> keys(n);
    for (int i = 0; i < n; ++i) {
        uint32_t q[3];
        for (int a = 0; a < 3; ++a) {
            float mn = comp(cb.lo, a), ext = comp(cb.hi, a) - mn;
            float t = ext > 0 ? (comp(cen[i], a) - mn) / ext : 0.0f;
            int v = (int)(t * 1024.0f);
            q[a] = (uint32_t)std::min(1023, std::max(0, v));
        }
        uint32_t m = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
        keys[i] = {((uint64_t)m << 32) | (uint32_t)i, i};
    }
    std::sort(keys.begin(), keys.end());
    Tree T;
    T.n.reserve(2 * n);
    std::vector<int> C(n);
    for (int j = 0; j < n; ++j) {
        BNode L; L.b = pbox[keys[j].second]; L.prims = {prims[keys[j].second]}; L.cnt = 1;
        T.n.push_back(L); C[j] = j;
    }
    while (C.size() > 1) {
        const int k = (int)C.size();
        std::vector<int> N(k);
#pragma omp parallel for schedule(static)
        for (int i = 0; i < k; ++i) {
            float best = INFINITY; int bj = -1;
            for (int o = -radius; o <= radius; ++o) {
                int j = i + o;
                if (o == 0 || j < 0 || j >= k) continue;
                Box m = T.n[C[i]].b; m.add(T.n[C[j]].b);
                float a = m.half_area();
                if (a < best) { best = a; bj = j; }
            }
            N[i] = bj;
        }
        std::vector<int> nc;
        nc.reserve(k);
        for (int i = 0; i < k; ++i) {
            int j = N[i];
            bool mutual = j >= 0 && N[j] == i;
            if (mutual && i < j) {
                BNode P; P.l = C[i]; P.r = C[j]; P.b = T.n[C[i]].b; P.b.add(T.n[C[j]].b);
                P.cnt = T.n[C[i]].cnt + T.n[C[j]].cnt;
                T.n.push_back(P); nc.push_back((int)T.n.size() - 1);
            } else if (!(mutual && j < i)) {
                nc.push_back(C[i]);
            }
        }
        C.swap(nc);
    }
    T.root = C[0];
    return T;
}

// ---- top-down full-sweep SAH over centroids (object splits), to single primitives
static int sweep_rec(Tree& T, std::vector<int>& idx, int first, int count, const std::vector<Box>& pbox,
                     const std::vector<V3>& cen, std::vector<float>& rarea) {
    BNode N;
    for (int i = first; i < first + count; ++i) N.b.add(pbox[idx[i]]);
    N.cnt = count;
    if (count == 1) { N.prims = {idx[first]}; T.n.push_back(N); return (int)T.n.size() - 1; }
    float best = INFINITY; int bax = -1, bsplit = -1;
    std::vector<int> tmp[3];
    for (int a = 0; a < 3; ++a) {
        tmp[a].assign(idx.begin() + first, idx.begin() + first + count);
        std::sort(tmp[a].begin(), tmp[a].end(), [&](int p, int q) {
            float cp = comp(cen[p], a), cq = comp(cen[q], a);
            return cp < cq || (cp == cq && p < q);
        });
        Box rb;
        for (int i = count - 1; i >= 1; --i) { rb.add(pbox[tmp[a][i]]); rarea[i] = rb.half_area(); }
        Box lb;
        for (int i = 1; i < count; ++i) {
            lb.add(pbox[tmp[a][i - 1]]);
            float c = lb.half_area() * i + rarea[i] * (count - i);
            if (c < best) { best = c; bax = a; bsplit = i; }
        }
    }
    std::copy(tmp[bax].begin(), tmp[bax].end(), idx.begin() + first);
    int l = sweep_rec(T, idx, first, bsplit, pbox, cen, rarea);
    int r = sweep_rec(T, idx, first + bsplit, count - bsplit, pbox, cen, rarea);
    N.l = l; N.r = r;
    T.n.push_back(N);
    return (int)T.n.size() - 1;
}
static Tree build_sweep(const std::vector<int>& prims, const std::vector<Box>& pbox) {
    const int n = (int)prims.size();
    std::vector<V3> cen(n);
    for (int i = 0; i < n; ++i) cen[i] = (pbox[i].lo + pbox[i].hi) * 0.5f;
    std::vector<int> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    std::vector<float> rarea(n + 1);
    Tree T;
    T.n.reserve(2 * n);
    T.root = sweep_rec(T, idx, 0, n, pbox, cen, rarea);
    for (auto& x : T.n) for (auto& p : x.prims) p = prims[p];
    return T;
}

// ---- SBVH (Stich et al. 2009): binned object splits + binned spatial splits with reference clipping
struct Ref { Box b; int prim; };
static void clip_tri(int prim, const Box& into, int axis, float pos, Box& left, Box& right) {
    // split the triangle's polygon (clipped to `into`) at axis = pos
    const Tri& T = g_tris[prim];
    V3 v[3] = {T.v0, T.v1, T.v2};
    left = Box(); right = Box();
    for (int i = 0; i < 3; ++i) {
        V3 a = v[i], b = v[(i + 1) % 3];
        float pa = comp(a, axis), pb = comp(b, axis);
        if (pa <= pos) left.add(a);
        if (pa >= pos) right.add(a);
        if ((pa < pos && pb > pos) || (pa > pos && pb < pos)) {
            float t = (pos - pa) / (pb - pa);
            V3 m = a + (b - a) * t;
            if (axis == 0) m.x = pos; else if (axis == 1) m.y = pos; else m.z = pos;
            left.add(m); right.add(m);
        }
    }
    left.lo = vmax(left.lo, into.lo); left.hi = vmin(left.hi, into.hi);
    right.lo = vmax(right.lo, into.lo); right.hi = vmin(right.hi, into.hi);
}
struct SbvhCfg { int bins = 32; float alpha = 1e-5f; int max_leaf = 1; };
static int sbvh_rec(Tree& T, std::vector<Ref> refs, const SbvhCfg& cfg, float root_area, int depth) {
    BNode N;
    Box cb;
    for (auto& r : refs) { N.b.add(r.b); cb.add((r.b.lo + r.b.hi) * 0.5f); }
    N.cnt = (int)refs.size();
    const int n = (int)refs.size();
    if (n <= cfg.max_leaf || depth > 60) {
        for (auto& r : refs) N.prims.push_back(r.prim);
        std::sort(N.prims.begin(), N.prims.end());
        N.prims.erase(std::unique(N.prims.begin(), N.prims.end()), N.prims.end());
        N.cnt = (int)N.prims.size();
        T.n.push_back(N);
        return (int)T.n.size() - 1;
    }
    // object split: full sweep
    float best = INFINITY; int bax = -1, bsplit = -1;
    std::vector<float> rarea(n + 1);
    std::vector<int> ord[3];
    for (int a = 0; a < 3; ++a) {
        ord[a].resize(n);
        std::iota(ord[a].begin(), ord[a].end(), 0);
        std::sort(ord[a].begin(), ord[a].end(), [&](int p, int q) {
            float cp = comp(refs[p].b.lo, a) + comp(refs[p].b.hi, a), cq = comp(refs[q].b.lo, a) + comp(refs[q].b.hi, a);
            return cp < cq || (cp == cq && refs[p].prim < refs[q].prim);
        });
        Box rb;
        for (int i = n - 1; i >= 1; --i) { rb.add(refs[ord[a][i]].b); rarea[i] = rb.half_area(); }
        Box lb;
        for (int i = 1; i < n; ++i) {
            lb.add(refs[ord[a][i - 1]].b);
            float c = lb.half_area() * i + rarea[i] * (n - i);
            if (c < best) { best = c; bax = a; bsplit = i; }
        }
    }
    // overlap of the object split's children
    Box L0, R0;
    for (int i = 0; i < bsplit; ++i) L0.add(refs[ord[bax][i]].b);
    for (int i = bsplit; i < n; ++i) R0.add(refs[ord[bax][i]].b);
    Box ov; ov.lo = vmax(L0.lo, R0.lo); ov.hi = vmin(L0.hi, R0.hi);
    float ov_area = (ov.lo.x <= ov.hi.x && ov.lo.y <= ov.hi.y && ov.lo.z <= ov.hi.z) ? ov.half_area() : 0.0f;
    bool spatial = false; int sax = -1; float spos = 0;
    if (ov_area > cfg.alpha * root_area) {
        for (int a = 0; a < 3; ++a) {
            float lo = comp(N.b.lo, a), hi = comp(N.b.hi, a);
            if (!(hi > lo)) continue;
            const int B = cfg.bins;
            std::vector<Box> bb(B);
            std::vector<int> entry(B, 0), exitc(B, 0);
            float w = (hi - lo) / B;
            for (auto& r : refs) {
                int b0 = std::min(B - 1, std::max(0, (int)((comp(r.b.lo, a) - lo) / w)));
                int b1 = std::min(B - 1, std::max(0, (int)((comp(r.b.hi, a) - lo) / w)));
                entry[b0]++; exitc[b1]++;
                Box cur = r.b;
                for (int b = b0; b < b1; ++b) {
                    float pos = lo + w * (b + 1);
                    Box l, rr;
                    clip_tri(r.prim, cur, a, pos, l, rr);
                    if (l.lo.x <= l.hi.x) bb[b].add(l);
                    cur = rr;
                }
                if (cur.lo.x <= cur.hi.x) bb[b1].add(cur);
            }
            std::vector<float> ra(B);
            std::vector<int> rc(B);
            Box acc; int cnt = 0;
            for (int b = B - 1; b >= 1; --b) { acc.add(bb[b]); cnt += exitc[b]; ra[b] = acc.half_area(); rc[b] = cnt; }
            Box lacc; int lc = 0;
            for (int b = 1; b < B; ++b) {
                lacc.add(bb[b - 1]); lc += entry[b - 1];
                if (lc == 0 || rc[b] == 0) continue;
                float c = lacc.half_area() * lc + ra[b] * rc[b];
                if (c < best) { best = c; spatial = true; sax = a; spos = lo + w * b; }
            }
        }
    }
    std::vector<Ref> Lr, Rr;
    if (!spatial) {
        for (int i = 0; i < n; ++i) (i < bsplit ? Lr : Rr).push_back(refs[ord[bax][i]]);
    } else {
        for (auto& r : refs) {
            float lo = comp(r.b.lo, sax), hi = comp(r.b.hi, sax);
            if (hi <= spos) Lr.push_back(r);
            else if (lo >= spos) Rr.push_back(r);
            else {
                Box l, rr;
                clip_tri(r.prim, r.b, sax, spos, l, rr);
                if (l.lo.x <= l.hi.x && l.lo.y <= l.hi.y && l.lo.z <= l.hi.z) Lr.push_back({l, r.prim});
                if (rr.lo.x <= rr.hi.x && rr.lo.y <= rr.hi.y && rr.lo.z <= rr.hi.z) Rr.push_back({rr, r.prim});
            }
        }
        if (Lr.empty() || Rr.empty()) {   // degenerate: fall back to the object split
            Lr.clear(); Rr.clear();
            for (int i = 0; i < n; ++i) (i < bsplit ? Lr : Rr).push_back(refs[ord[bax][i]]);
        }
    }
    refs.clear(); refs.shrink_to_fit();
    int l = sbvh_rec(T, std::move(Lr), cfg, root_area, depth + 1);
    int r = sbvh_rec(T, std::move(Rr), cfg, root_area, depth + 1);
    N.l = l; N.r = r;
    N.cnt = T.n[l].cnt + T.n[r].cnt;
    T.n.push_back(N);
    return (int)T.n.size() - 1;
}
static Tree build_sbvh(const SbvhCfg& cfg) {
    std::vector<Ref> refs(g_tris.size());
    Box all;
    for (size_t i = 0; i < g_tris.size(); ++i) { refs[i] = {tri_box((int)i), (int)i}; all.add(refs[i].b); }
    Tree T;
    T.root = sbvh_rec(T, std::move(refs), cfg, all.half_area(), 0);
    return T;
}

// ---- SAH collapse (the GPU's k_ploc_collapse rule) into leaves of <= max_leaf references
struct CTree { std::vector<BNode> n; int root; };
static float collapse(Tree& T, int c, int max_leaf, float ctrav, float ctri, std::vector<char>& leafify, std::vector<float>& cost) {
    BNode& N = T.n[c];
    if (N.l < 0) { cost[c] = ctri * (float)N.prims.size(); leafify[c] = 1; return cost[c]; }
    float cl = collapse(T, N.l, max_leaf, ctrav, ctri, leafify, cost);
    float cr = collapse(T, N.r, max_leaf, ctrav, ctri, leafify, cost);
    float A = std::max(N.b.half_area(), 1e-30f);
    float split = ctrav + (T.n[N.l].b.half_area() * cl + T.n[N.r].b.half_area() * cr) / A;
    float leaf = ctri * (float)N.cnt;
    if (N.cnt <= max_leaf && leaf <= split) { cost[c] = leaf; leafify[c] = 1; }
    else { cost[c] = split; leafify[c] = 0; }
    return cost[c];
}
static void gather_prims(const Tree& T, int c, std::vector<int>& out) {
    if (T.n[c].l < 0) { out.insert(out.end(), T.n[c].prims.begin(), T.n[c].prims.end()); return; }
    gather_prims(T, T.n[c].l, out); gather_prims(T, T.n[c].r, out);
}

// ---------------------------------------------------------------- flattened skip-pointer layout
struct FNode { Box b; int skip; int first = -1, cnt = 0; };
struct Flat { std::vector<FNode> n; std::vector<int> leaf_prims; };
enum Order { ORD_LEFT, ORD_BIG_FIRST, ORD_SMALL_FIRST, ORD_MORE_TRIS_FIRST };
static void flatten_rec(const Tree& T, int c, const std::vector<char>& leafify, Order ord, Flat& F) {
    const BNode& N = T.n[c];
    int i = (int)F.n.size();
    F.n.push_back(FNode{N.b, 0});
    if (leafify[c]) {
        std::vector<int> p;
        gather_prims(T, c, p);
        std::sort(p.begin(), p.end());
        p.erase(std::unique(p.begin(), p.end()), p.end());
        F.n[i].first = (int)F.leaf_prims.size(); F.n[i].cnt = (int)p.size();
        F.leaf_prims.insert(F.leaf_prims.end(), p.begin(), p.end());
        F.n[i].skip = i + 1;
        return;
    }
    int a = N.l, b = N.r;
    bool swap = false;
    if (ord == ORD_BIG_FIRST) swap = T.n[b].b.half_area() > T.n[a].b.half_area();
    if (ord == ORD_SMALL_FIRST) swap = T.n[b].b.half_area() < T.n[a].b.half_area();
    if (ord == ORD_MORE_TRIS_FIRST) swap = T.n[b].cnt > T.n[a].cnt;
    if (swap) std::swap(a, b);
    flatten_rec(T, a, leafify, ord, F);
    flatten_rec(T, b, leafify, ord, F);
    F.n[i].skip = (int)F.n.size();
}
static Flat make_flat(Tree& T, int max_leaf, float ctrav, float ctri, Order ord) {
    std::vector<char> leafify(T.n.size(), 0);
    std::vector<float> cost(T.n.size(), 0);
    collapse(T, T.root, max_leaf, ctrav, ctri, leafify, cost);
    Flat F;
    flatten_rec(T, T.root, leafify, ord, F);
    // a leaf holding > 8 prims (SBVH leaves of duplicated refs) is not encodable on the GPU: report
    return F;
}

// ---------------------------------------------------------------- walks
static inline bool box_test(const Box& b, V3 o, V3 inv, float tn, float tf) {
    float tx0 = (b.lo.x - o.x) * inv.x, tx1 = (b.hi.x - o.x) * inv.x;
    float ty0 = (b.lo.y - o.y) * inv.y, ty1 = (b.hi.y - o.y) * inv.y;
    float tz0 = (b.lo.z - o.z) * inv.z, tz1 = (b.hi.z - o.z) * inv.z;
    float t0 = std::max(std::max(std::max(tn, std::min(tx0, tx1)), std::min(ty0, ty1)), std::min(tz0, tz1));
    float t1 = std::min(std::min(std::min(tf, std::max(tx0, tx1)), std::max(ty0, ty1)), std::max(tz0, tz1));
    return t0 * (1.0f - 4.0f * FLT_EPSILON) <= t1 * (1.0f + 4.0f * FLT_EPSILON);
}
static inline bool tri_hit(int p, V3 o, V3 d, float tn, float tf, float& t) {
    const Tri& T = g_tris[p];
    V3 e1 = T.v1 - T.v0, e2 = T.v2 - T.v0;
    V3 pv = cross(d, e2);
    float det = dot(e1, pv);
    if (det == 0.0f) return false;
    float inv = 1.0f / det;
    V3 sv = o - T.v0;
    float u = dot(sv, pv) * inv;
    if (!(u >= 0.0f && u <= 1.0f)) return false;
    V3 q = cross(sv, e1);
    float v = dot(d, q) * inv;
    if (!(v >= 0.0f && u + v <= 1.0f)) return false;
    t = dot(e2, q) * inv;
    return t >= tn && t <= tf;
}
struct Ray { V3 o, d; float tn, tf; bool active; };
// per-lane walk; records per step (node index or -1 done) and the leaf count tested at each step
struct Trace { int visits = 0, tris = 0; std::vector<int> step_cnt; float t = -1; int prim = -1; bool occ = false; };
static Trace walk(const Flat& F, const Ray& r, bool any, std::vector<int>* vis = nullptr) {
    Trace tr;
    if (!r.active) return tr;
    V3 inv{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    float tf = r.tf;
    int i = 0, n = (int)F.n.size();
    while (i < n) {
        const FNode& N = F.n[i];
        ++tr.visits;
        if (vis) vis->push_back(i);
        bool hit = box_test(N.b, r.o, inv, r.tn, tf);
        int cnt = 0;
        if (hit && N.cnt > 0) {
            for (int j = 0; j < N.cnt; ++j) {
                ++cnt; ++tr.tris;
                float t;
                int p = F.leaf_prims[N.first + j];
                if (tri_hit(p, r.o, r.d, r.tn, tf, t)) {
                    if (any) { tr.occ = true; break; }
                    if (tr.prim < 0 || t < tf || (t == tf && p < tr.prim)) { tf = t; tr.prim = p; tr.t = t; }
                }
            }
        }
        tr.step_cnt.push_back(cnt);
        if (tr.occ) break;
        i = (hit && N.cnt == 0) ? i + 1 : N.skip;
    }
    return tr;
}

struct Stats { double visits = 0, tris = 0, wave_steps = 0, wave_tri_iters = 0; long rays = 0, waves = 0; std::vector<int> vis; };
static void wave_stats(const std::vector<Trace>& tr, const std::vector<char>& act, int W, int H, Stats& S) {
    // waves: 8x8 pixel tiles
    for (int ty = 0; ty + 8 <= H; ty += 8)
        for (int tx = 0; tx + 8 <= W; tx += 8) {
            int steps = 0;
            std::vector<const Trace*> lanes;
            for (int y = 0; y < 8; ++y)
                for (int x = 0; x < 8; ++x) {
                    int p = (ty + y) * W + tx + x;
                    if (!act[p]) continue;
                    lanes.push_back(&tr[p]);
                    steps = std::max(steps, (int)tr[p].step_cnt.size());
                }
            if (lanes.empty()) continue;
            double it = 0;
            for (int s = 0; s < steps; ++s) {
                int m = 0;
                for (auto* l : lanes) if (s < (int)l->step_cnt.size()) m = std::max(m, l->step_cnt[s]);
                it += m;
            }
            S.wave_steps += steps; S.wave_tri_iters += it; S.waves++;
        }
    for (size_t p = 0; p < tr.size(); ++p)
        if (act[p]) { S.visits += tr[p].visits; S.tris += tr[p].tris; S.rays++; S.vis.push_back(tr[p].visits); }
}


// ---------------------------------------------------------------- k-wide trees (collapsed from the binary tree)
struct WChild { Box b; int node = -1; int first = -1, cnt = 0; };      // node >= 0: interior; else leaf (first, cnt)
struct WNode { std::vector<WChild> c; };
struct Wide { std::vector<WNode> n; std::vector<int> leaf_prims; };
static int wide_rec(const Tree& T, int c, const std::vector<char>& leafify, int k, Wide& Wd) {
    std::vector<int> kids = {T.n[c].l, T.n[c].r};
    while ((int)kids.size() < k) {          // open the largest interior child
        int best = -1; float ba = -1;
        static const int wh = getenv("WH") ? atoi(getenv("WH")) : 0;   // 0 area, 1 area x count, 2 area x log count
        for (int i = 0; i < (int)kids.size(); ++i) {
            if (leafify[kids[i]]) continue;
            float v = T.n[kids[i]].b.half_area();
            if (wh == 1) v *= (float)T.n[kids[i]].cnt;
            if (wh == 2) v *= std::log2((float)T.n[kids[i]].cnt + 1.0f);
            if (v > ba) { ba = v; best = i; }
        }
        if (best < 0) break;
        int x = kids[best];
        kids.erase(kids.begin() + best);
        kids.push_back(T.n[x].l); kids.push_back(T.n[x].r);
    }
    int me = (int)Wd.n.size();
    Wd.n.push_back(WNode{});
    std::vector<WChild> cs;
    for (int x : kids) {
        WChild ch; ch.b = T.n[x].b;
        if (leafify[x]) {
            std::vector<int> p; gather_prims(T, x, p);
            std::sort(p.begin(), p.end()); p.erase(std::unique(p.begin(), p.end()), p.end());
            ch.first = (int)Wd.leaf_prims.size(); ch.cnt = (int)p.size();
            Wd.leaf_prims.insert(Wd.leaf_prims.end(), p.begin(), p.end());
        } else {
            ch.node = wide_rec(T, x, leafify, k, Wd);
        }
        cs.push_back(ch);
    }
    Wd.n[me].c = cs;
    return me;
}
static inline bool box_test_t(const Box& b, V3 o, V3 inv, float tn, float tf, float& tin) {
    float tx0 = (b.lo.x - o.x) * inv.x, tx1 = (b.hi.x - o.x) * inv.x;
    float ty0 = (b.lo.y - o.y) * inv.y, ty1 = (b.hi.y - o.y) * inv.y;
    float tz0 = (b.lo.z - o.z) * inv.z, tz1 = (b.hi.z - o.z) * inv.z;
    float t0 = std::max(std::max(std::max(tn, std::min(tx0, tx1)), std::min(ty0, ty1)), std::min(tz0, tz1));
    float t1 = std::min(std::min(std::min(tf, std::max(tx0, tx1)), std::max(ty0, ty1)), std::max(tz0, tz1));
    tin = t0;
    return t0 * (1.0f - 4.0f * FLT_EPSILON) <= t1 * (1.0f + 4.0f * FLT_EPSILON);
}
// per-lane stack walk over a wide tree: a step = one node fetch (all child boxes tested) and then the
// hit leaf children's triangles; hit interior children pushed far-to-near (nearest popped first)
static Trace walk_wide(const Wide& Wd, const Ray& r, bool any, int& max_stack) {
    Trace tr;
    if (!r.active) return tr;
    V3 inv{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    float tf = r.tf;
    std::vector<std::pair<float, int>> st;
    st.push_back({r.tn, 0});
    while (!st.empty()) {
        auto [tin0, ni] = st.back(); st.pop_back();
        if (!any && tin0 * (1.0f - 4.0f * FLT_EPSILON) > tf * (1.0f + 4.0f * FLT_EPSILON)) continue;   // culled on pop (no fetch)
        ++tr.visits;
        const WNode& N = Wd.n[ni];
        std::vector<std::pair<float, int>> hits;
        int cnt = 0;
        std::vector<std::pair<float, const WChild*>> leaves;
        for (auto& ch : N.c) {
            float tin;
            if (!box_test_t(ch.b, r.o, inv, r.tn, tf, tin)) continue;
            if (ch.node >= 0) hits.push_back({tin, ch.node});
            else leaves.push_back({tin, &ch});
        }
        std::sort(leaves.begin(), leaves.end(), [](auto& a, auto& b) { return a.first < b.first; });
        for (auto& lf : leaves) {
            for (int j = 0; j < lf.second->cnt; ++j) {
                ++cnt; ++tr.tris;
                float t; int p = Wd.leaf_prims[lf.second->first + j];
                if (tri_hit(p, r.o, r.d, r.tn, tf, t)) {
                    if (any) { tr.occ = true; break; }
                    if (tr.prim < 0 || t < tf || (t == tf && p < tr.prim)) { tf = t; tr.prim = p; tr.t = t; }
                }
            }
            if (tr.occ) break;
        }
        tr.step_cnt.push_back(cnt);
        if (tr.occ) break;
        std::sort(hits.begin(), hits.end(), [](auto& a, auto& b) { return a.first > b.first; });
        for (auto& h : hits) st.push_back(h);
        max_stack = std::max(max_stack, (int)st.size());
    }
    return tr;
}

// the GPU shape: group stack (base node, remaining hit-interior mask), children tested at the parent;
// returns the deepest group stack
static int group_depth(const Wide& Wd, const Ray& r, bool any) {
    if (!r.active) return 0;
    V3 inv{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    float tf = r.tf;
    struct G { int node; std::vector<int> kids; };
    std::vector<std::vector<int>> st;
    std::vector<int> cur = {0};
    int maxd = 0; bool occ = false; int prim = -1;
    while (!occ) {
        if (cur.empty()) { if (st.empty()) break; cur = st.back(); st.pop_back(); }
        int ni = cur.front(); cur.erase(cur.begin());
        if (!cur.empty()) { st.push_back(cur); maxd = std::max(maxd, (int)st.size()); }
        const WNode& N = Wd.n[ni];
        std::vector<int> nxt;
        for (auto& ch : N.c) {
            float tin;
            if (!box_test_t(ch.b, r.o, inv, r.tn, tf, tin)) continue;
            if (ch.node >= 0) { nxt.push_back(ch.node); continue; }
            for (int j = 0; j < ch.cnt; ++j) {
                float t; int p = Wd.leaf_prims[ch.first + j];
                if (tri_hit(p, r.o, r.d, r.tn, tf, t)) { if (any) { occ = true; break; } if (prim < 0 || t < tf || (t == tf && p < prim)) { tf = t; prim = p; } }
            }
            if (occ) break;
        }
        cur = nxt;
    }
    return maxd;
}

// ---- emulation of the product's wide_walk (rs_scene.h) on the product's wide tree (rs_wide.h): per lane,
// the same group/stack logic and quantised box test; counts loop iterations, stack overflows, triangle tests
struct WEmu { int iters = 0, tris = 0, lost = 0, occ = 0; int prim = -1; float t = 0; int maxsp = 0; };
static inline float u2f_(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static const std::vector<float>* g_exact_lo = nullptr;
static const std::vector<float>* g_exact_hi = nullptr;
static const std::vector<int>* g_slot_src = nullptr;
static uint32_t emu_hits_exact(size_t node, const uint32_t* w, V3 o, V3 inv, float tnear, float tfar) {
    uint32_t hits = 0;
    const float iv[3] = {inv.x, inv.y, inv.z}, org[3] = {o.x, o.y, o.z};
    for (int c = 0; c < (int)(w[3] >> 28); ++c) {
        const int k = (*g_slot_src)[8 * node + c];
        float t0 = tnear, t1 = tfar;
        for (int a = 0; a < 3; ++a) {
            const float x0 = ((*g_exact_lo)[4 * (size_t)k + a] - org[a]) * iv[a], x1 = ((*g_exact_hi)[4 * (size_t)k + a] - org[a]) * iv[a];
            t0 = std::fmax(t0, std::fmin(x0, x1)); t1 = std::fmin(t1, std::fmax(x0, x1));
        }
        if (t0 * (1.0f - 4.0f * FLT_EPSILON) <= t1 * (1.0f + 4.0f * FLT_EPSILON)) hits |= 1u << c;
    }
    return hits;
}
static uint32_t emu_hits(const uint32_t* w, V3 o, V3 inv, float tnear, float tfar) {
    const uint32_t eb = w[3];
    const float s[3] = {u2f_((eb & 0xffu) << 23), u2f_(((eb >> 8) & 0xffu) << 23), u2f_(((eb >> 16) & 0xffu) << 23)};
    const float iv[3] = {inv.x, inv.y, inv.z}, org[3] = {o.x, o.y, o.z};
    float a[3], b[3];
    for (int k = 0; k < 3; ++k) { a[k] = s[k] * iv[k]; b[k] = (u2f_(w[k]) - org[k]) * iv[k]; }
    const float E = 2.384185791015625e-07f * std::fmax(std::fmax(std::fabs(b[0]), std::fabs(b[1])), std::fabs(b[2]));
    const uint32_t lo[3][2] = {{w[6], w[7]}, {w[8], w[9]}, {w[10], w[11]}};
    const uint32_t hi[3][2] = {{w[12], w[13]}, {w[14], w[15]}, {w[16], w[17]}};
    const float lo_k = 1.0f - 4.0f * FLT_EPSILON, hi_k = 1.0f + 4.0f * FLT_EPSILON;
    uint32_t hits = 0;
    for (int c = 0; c < 8; ++c) {
        float tn[3], tf[3];
        for (int k = 0; k < 3; ++k) {
            const bool pos = iv[k] >= 0.0f;
            const uint32_t qn = pos ? lo[k][c >> 2] : hi[k][c >> 2], qf = pos ? hi[k][c >> 2] : lo[k][c >> 2];
            tn[k] = std::fma((float)((qn >> (8 * (c & 3))) & 0xffu), a[k], b[k]);
            tf[k] = std::fma((float)((qf >> (8 * (c & 3))) & 0xffu), a[k], b[k]);
        }
        const float t0 = std::fmax(std::fmax(std::fmax(tnear, tn[0]), tn[1]), tn[2]);
        const float t1 = std::fmin(std::fmin(std::fmin(tfar, tf[0]), tf[1]), tf[2]);
        if (std::fma(t0, lo_k, -E) <= std::fma(t1, hi_k, E)) hits |= 1u << c;
    }
    return hits & ((1u << (w[3] >> 28)) - 1u);
}
static WEmu emu_walk(const std::vector<uint32_t>& W, const std::vector<int>& prims, const Ray& r, bool any, int K,
                     std::vector<uint32_t>* seq = nullptr) {
    WEmu e;
    if (!r.active) return e;
    V3 inv{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    uint32_t gb = 0, gm = 1;
    std::vector<uint32_t> st;
    float tf = r.tf;
    while (gm) {
        ++e.iters;
        uint32_t slot = __builtin_ctz(gm), node = gb + slot, rest = gm & (gm - 1);
        if (rest) { if ((int)st.size() == K) { st.erase(st.begin()); e.lost = 1; } st.push_back((gb << 8) | rest); }
        e.maxsp = std::max(e.maxsp, (int)st.size());
        if (seq) seq->push_back(node);
        const uint32_t* w = &W[20 * (size_t)node];
        uint32_t hits = g_slot_src ? emu_hits_exact(node, w, r.o, inv, r.tn, tf) : emu_hits(w, r.o, inv, r.tn, tf);
        uint32_t ni = (w[3] >> 24) & 0xfu, tm = hits >> ni, tb = w[5];
        while (tm && !(any && e.occ)) {
            uint32_t j = __builtin_ctz(tm); tm &= tm - 1; ++e.tris;
            float t; int p = prims[tb + j];
            if (tri_hit(p, r.o, r.d, r.tn, tf, t)) {
                if (any) e.occ = 1;
                else if (e.prim < 0 || t < tf || (t == tf && p < e.prim)) { tf = t; e.prim = p; e.t = t; }
            }
        }
        uint32_t ngm = (any && e.occ) ? 0u : (hits & ((1u << ni) - 1u));
        if (ngm) { gb = w[4]; gm = ngm; }
        else if (!st.empty() && !(any && e.occ)) { uint32_t top = st.back(); st.pop_back(); gb = top >> 8; gm = top & 0xff; }
        else gm = 0;
    }
    return e;
}


// LAB (ORDER=1): any-hit walks that visit a node's hit interior children in another order than the slot order --
// 1 nearest entry first, 2 farthest first, 3 largest (most slots below) first -- node fetches counted
static uint32_t emu_hits_t(const uint32_t* w, V3 o, V3 inv, float tnear, float tfar, float* tent) {
    const uint32_t eb = w[3];
    const float s[3] = {u2f_((eb & 0xffu) << 23), u2f_(((eb >> 8) & 0xffu) << 23), u2f_(((eb >> 16) & 0xffu) << 23)};
    const float iv[3] = {inv.x, inv.y, inv.z}, org[3] = {o.x, o.y, o.z};
    float a[3], b[3];
    for (int k = 0; k < 3; ++k) { a[k] = s[k] * iv[k]; b[k] = (u2f_(w[k]) - org[k]) * iv[k]; }
    const uint32_t lo[3][2] = {{w[6], w[7]}, {w[8], w[9]}, {w[10], w[11]}};
    const uint32_t hi[3][2] = {{w[12], w[13]}, {w[14], w[15]}, {w[16], w[17]}};
    uint32_t hits = 0;
    for (int c = 0; c < 8; ++c) {
        float tn[3], tf[3];
        for (int k = 0; k < 3; ++k) {
            const bool pos = iv[k] >= 0.0f;
            const uint32_t qn = pos ? lo[k][c >> 2] : hi[k][c >> 2], qf = pos ? hi[k][c >> 2] : lo[k][c >> 2];
            tn[k] = std::fma((float)((qn >> (8 * (c & 3))) & 0xffu), a[k], b[k]);
            tf[k] = std::fma((float)((qf >> (8 * (c & 3))) & 0xffu), a[k], b[k]);
        }
        const float t0 = std::fmax(std::fmax(std::fmax(tnear, tn[0]), tn[1]), tn[2]);
        const float t1 = std::fmin(std::fmin(std::fmin(tfar, tf[0]), tf[1]), tf[2]);
        tent[c] = t0;
        if (t0 * 0.9999995f <= t1 * 1.0000005f) hits |= 1u << c;
    }
    return hits & ((1u << (w[3] >> 28)) - 1u);
}
static FILE* g_iters_dump = nullptr;           // DUMP_ITERS=path: each shadow ray's node fetches (int32, pixel order)
static std::vector<int> g_subtree, g_subtri;     // per wide node: nodes / triangles below it (ORDER=3 / 5)
static int emu_walk_order(const std::vector<uint32_t>& W, const std::vector<int>& prims, const Ray& r, int mode,
                          bool any = true) {
    V3 inv{1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z};
    float tfar = r.tf;
    std::vector<uint32_t> st{0u};
    int iters = 0;
    while (!st.empty()) {
        const uint32_t node = st.back(); st.pop_back();
        ++iters;
        const uint32_t* w = &W[20 * (size_t)node];
        float te[8];
        const uint32_t hits = emu_hits_t(w, r.o, inv, r.tn, tfar, te);
        const uint32_t ni = (w[3] >> 24) & 0xfu, tb = w[5];
        for (uint32_t tm = hits >> ni; tm; tm &= tm - 1) {
            float t;
            if (tri_hit(prims[tb + __builtin_ctz(tm)], r.o, r.d, r.tn, tfar, t)) {
                if (any) return iters;
                tfar = std::min(tfar, t);
            }
        }
        std::vector<std::pair<float, uint32_t>> kids;
        for (uint32_t c = 0; c < ni; ++c)
            if ((hits >> c) & 1u) {
                const uint32_t k = w[4] + c;
                float area = 0.0f;
                if (mode == 4) {                         // the child's quantised box (surface area / 2)
                    float e3[3];
                    for (int a = 0; a < 3; ++a) {
                        const float sc = u2f_(((w[3] >> (8 * a)) & 0xffu) << 23);
                        const uint32_t ql = (w[6 + 2 * a + (c >> 2)] >> (8 * (c & 3))) & 0xffu;
                        const uint32_t qh = (w[12 + 2 * a + (c >> 2)] >> (8 * (c & 3))) & 0xffu;
                        e3[a] = (float)(qh - ql) * sc;
                    }
                    area = e3[0] * e3[1] + e3[1] * e3[2] + e3[2] * e3[0];
                }
                const float key = mode == 1 ? -te[c] : mode == 2 ? te[c] : mode == 3 ? (float)g_subtree[k] :
                                  mode == 4 ? area : mode == 5 ? (float)g_subtri[k] : -(float)c;
                kids.push_back({key, k});
            }
        std::sort(kids.begin(), kids.end());      // ascending key: the last pushed (popped first) has the largest key
        for (auto& kv : kids) st.push_back(kv.second);
    }
    return iters;
}

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: bvh_lab scene.bin which [W H]\n"); return 1; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    int32_t nt, ne;
    float cam[7];
    fread(&nt, 4, 1, f); fread(&ne, 4, 1, f); fread(cam, 4, 7, f);
    g_tris.resize(nt);
    fread(g_tris.data(), sizeof(Tri), nt, f);
    std::vector<int32_t> emis(ne);
    fread(emis.data(), 4, ne, f);
    fclose(f);
    std::string which = argv[2];
    const int W = argc > 3 ? atoi(argv[3]) : 480, H = argc > 4 ? atoi(argv[4]) : 272;
    const int max_leaf = argc > 5 ? atoi(argv[5]) : 8;
    const float ctri = argc > 6 ? (float)atof(argv[6]) : 1.0f;
    const Order ord = argc > 7 ? (Order)atoi(argv[7]) : ORD_LEFT;

    std::vector<int> prims(nt);
    std::iota(prims.begin(), prims.end(), 0);
    std::vector<Box> pbox(nt);
    for (int i = 0; i < nt; ++i) pbox[i] = tri_box(i);
    Tree T;
    if (which == "ploc") T = build_ploc(prims, pbox, 16);
    else if (which == "ploc32") T = build_ploc(prims, pbox, 32);
    else if (which == "sweep") T = build_sweep(prims, pbox);
    else if (which == "sbvh") T = build_sbvh(SbvhCfg{32, 1e-5f, 1});
    else if (which == "sbvh4") T = build_sbvh(SbvhCfg{32, 1e-4f, 1});
    else { fprintf(stderr, "unknown builder\n"); return 1; }
    if (getenv("CHECK_WIDE")) {   // the product's collapse (rs_wide.h) on this PLOC tree
        const int n = nt, total = 2 * n - 1;
        // PLOC-shaped arrays: ids < n prims (Morton order j -> the tree's leaf node j), >= n internal
        std::vector<float> lo(4 * (size_t)total), hi(4 * (size_t)total);
        std::vector<int> id(T.n.size(), -1);
        int nx = n, np = 0;
        for (size_t i = 0; i < T.n.size(); ++i) if (T.n[i].l < 0) id[i] = np++;
        for (size_t i = 0; i < T.n.size(); ++i) if (T.n[i].l >= 0) id[i] = nx++;
        for (size_t i = 0; i < T.n.size(); ++i) {
            const BNode& B = T.n[i]; const int k = id[i];
            float* a = &lo[4 * (size_t)k]; float* b = &hi[4 * (size_t)k];
            a[0] = B.b.lo.x; a[1] = B.b.lo.y; a[2] = B.b.lo.z; b[0] = B.b.hi.x; b[1] = B.b.hi.y; b[2] = B.b.hi.z;
            int L = B.l >= 0 ? id[B.l] : -1, R = B.r >= 0 ? id[B.r] : B.prims[0];
            std::memcpy(&a[3], &L, 4); std::memcpy(&b[3], &R, 4);
        }
        int wroot = id[T.root];
        if (getenv("HOST_SAH")) {                 // the product's host SAH source tree (rs_wide.h build_sah_host)
            const auto t0 = std::chrono::steady_clock::now();
            wroot = rs::build_sah_host((const float*)g_tris.data(), n, lo, hi, getenv("SWEEP_MAX") ? atoi(getenv("SWEEP_MAX")) : 2048);
            printf("build_sah_host %.1f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        std::vector<uint32_t> WN; std::vector<int> pr; int depth = 0; std::string err;
        const int coll = getenv("COLLAPSE") ? atoi(getenv("COLLAPSE")) : 0;
        const float c_tri = getenv("C_TRI") ? (float)atof(getenv("C_TRI")) : 0.3f;
        const int sl = getenv("MAX_DEPTH") ? atoi(getenv("MAX_DEPTH")) : 8;
        const auto tw = std::chrono::steady_clock::now();
        std::vector<int> slot_src;
        int rc = rs::build_wide_host(lo.data(), hi.data(), n, wroot, WN, pr, depth, err, coll, 1.0f, c_tri, sl, &slot_src);
        if (getenv("EXACT_BOXES")) {   // LAB: the walk's box test on the exact child boxes instead of the quantised planes
            g_exact_lo = &lo; g_exact_hi = &hi; g_slot_src = &slot_src;
        }
        printf("build_wide_host %.1f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count());
        printf("build_wide_host rc=%d err=%s nodes=%zu depth=%d\n", rc, err.c_str(), WN.size() / 20, depth);
        if (rc || !getenv("EMU")) return 0;
        Flat Fr = make_flat(T, 8, 1.0f, 1.0f, ORD_LEFT);
        // rays as below (primary, then shadow rays to random emitters), emulated walks
        V3 eye{cam[0], cam[1], cam[2]}, at{cam[3], cam[4], cam[5]};
        float fov = cam[6] * 3.14159265358979f / 180.0f;
        V3 zc = eye - at; zc = zc * (1.0f / std::sqrt(dot(zc, zc)));
        V3 up{0, 0, 1};
        V3 xc = cross(up, zc); xc = xc * (1.0f / std::sqrt(dot(xc, xc)));
        V3 yc = cross(zc, xc);
        float focal = (float)H / (2.0f * std::tan(fov / 2.0f));
        std::mt19937 rng(1);
        std::uniform_real_distribution<float> U(0.0f, 1.0f);
        double it_p = 0, it_s = 0, tr_s = 0, it_b = 0, tr_p = 0, tr_b = 0; long lost = 0, ns = 0, nb = 0, mism = 0; int maxsp = 0;
        std::vector<int> wave_it(((W / 8) * (H / 8)), 0);
        // LEVELS: node fetches per breadth-first level (what an LDS copy of the top levels would serve)
        const size_t NN = WN.size() / 20;
        std::vector<int> lvl_of(NN, 0);
        for (size_t j = 0; j < NN; ++j) {
            const uint32_t ni = (WN[20 * j + 3] >> 24) & 0xfu;
            for (uint32_t i = 0; i < ni; ++i) lvl_of[WN[20 * j + 4] + i] = lvl_of[j] + 1;
        }
        std::vector<double> lv_hist[3];
        for (auto& h : lv_hist) h.assign(32, 0.0);
        std::vector<size_t> lv_nodes(32, 0);
        for (size_t j = 0; j < NN; ++j) lv_nodes[lvl_of[j]]++;
        std::vector<uint32_t> lseq;
        const bool order_lab = getenv("ORDER") != nullptr;
        if (getenv("DUMP_ITERS")) g_iters_dump = fopen(getenv("DUMP_ITERS"), "wb");
        double it_ord[6] = {0, 0, 0, 0, 0, 0}, it_ordp[6] = {0, 0, 0, 0, 0, 0};
        if (order_lab) {
            g_subtree.assign(NN, 1);
            g_subtri.assign(NN, 0);
            for (size_t j = NN; j-- > 0;) {              // children after parents (breadth-first ids)
                const uint32_t ni = (WN[20 * j + 3] >> 24) & 0xfu, nv = WN[20 * j + 3] >> 28;
                g_subtri[j] += (int)(nv - ni);
                for (uint32_t i = 0; i < ni; ++i) { g_subtree[j] += g_subtree[WN[20 * j + 4] + i]; g_subtri[j] += g_subtri[WN[20 * j + 4] + i]; }
            }
        }
        auto lv_add = [&](int k) { for (uint32_t v : lseq) lv_hist[k][lvl_of[v]] += 1; lseq.clear(); };
        const bool levels = getenv("LEVELS") != nullptr;
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                V3 dc{(float)x - W / 2.0f, H / 2.0f - (float)y, -focal};
                V3 d = xc * dc.x + yc * dc.y + zc * dc.z;
                d = d * (1.0f / std::sqrt(dot(d, d)));
                Ray pr_{eye, d, 0.01f, 3.0e38f, true};
                WEmu a = emu_walk(WN, pr, pr_, false, 8, levels ? &lseq : nullptr);
                lv_add(0);
                Trace ref = walk(Fr, pr_, false);
                mism += a.prim != ref.prim;
                it_p += a.iters; tr_p += a.tris;
                if (order_lab) for (int m = 0; m < 6; ++m) it_ordp[m] += emu_walk_order(WN, pr, pr_, m, false);
                if (a.prim < 0) continue;
                V3 o = eye + d * a.t;
                {   // a cosine-distributed bounce off the hit triangle (the BRDF candidates' closest-hit rays)
                    const Tri& ht = g_tris[a.prim];
                    V3 nn = cross(ht.v1 - ht.v0, ht.v2 - ht.v0);
                    nn = nn * (1.0f / std::sqrt(std::max(dot(nn, nn), 1e-30f)));
                    if (dot(nn, d) > 0) nn = nn * -1.0f;
                    V3 t1 = std::fabs(nn.x) > 0.5f ? V3{0, 1, 0} : V3{1, 0, 0};
                    t1 = cross(nn, t1); t1 = t1 * (1.0f / std::sqrt(dot(t1, t1)));
                    V3 t2 = cross(nn, t1);
                    float u1 = U(rng), u2 = U(rng), rr = std::sqrt(u1), ph = 6.2831853f * u2;
                    V3 bd = t1 * (rr * std::cos(ph)) + t2 * (rr * std::sin(ph)) + nn * std::sqrt(std::max(0.0f, 1 - u1));
                    Ray br{o, bd, 0.01f, 3.0e38f, true};
                    WEmu c = emu_walk(WN, pr, br, false, 8, levels ? &lseq : nullptr);
                    lv_add(1);
                    Trace rb = walk(Fr, br, false);
                    mism += c.prim != rb.prim;
                    it_b += c.iters; tr_b += c.tris; ++nb;
                }
                int e = emis[rng() % ne];
                float r1 = U(rng), r2 = U(rng), sr = std::sqrt(r1);
                const Tri& t = g_tris[e];
                V3 q = t.v0 * (1 - sr) + t.v1 * (sr * (1 - r2)) + t.v2 * (sr * r2);
                V3 sd = q - o;
                float dist = std::sqrt(dot(sd, sd));
                sd = sd * (1.0f / std::max(dist, 1e-20f));
                Ray sh{o, sd, 0.01f, dist - 0.001f, true};
                WEmu b = emu_walk(WN, pr, sh, true, 8, levels ? &lseq : nullptr);
                lv_add(2);
                Trace rs_ = walk(Fr, sh, true);
                mism += b.occ != (int)rs_.occ;
                it_s += b.iters; tr_s += b.tris; lost += b.lost; ++ns; maxsp = std::max(maxsp, b.maxsp);
                if (g_iters_dump) fwrite(&b.iters, 4, 1, g_iters_dump);
                if (order_lab) for (int m = 0; m < 6; ++m) it_ord[m] += emu_walk_order(WN, pr, sh, m);
                if (y / 8 < H / 8 && x / 8 < W / 8) { int& wv = wave_it[(y / 8) * (W / 8) + x / 8]; wv = std::max(wv, b.iters); }
            }
        if (g_iters_dump) fclose(g_iters_dump);
        if (order_lab)
            printf("ORDER shadow fetches/ray: slot order %.3f, nearest first %.3f, farthest first %.3f, most nodes first %.3f, "
                   "largest area first %.3f, most triangles first %.3f\n",
                   it_ord[0] / ns, it_ord[1] / ns, it_ord[2] / ns, it_ord[3] / ns, it_ord[4] / ns, it_ord[5] / ns);
        if (order_lab)
            printf("ORDER primary (closest hit) fetches/ray: slot %.3f, nearest %.3f, farthest %.3f, most nodes %.3f, "
                   "largest area %.3f, most triangles %.3f\n", it_ordp[0] / (W * H), it_ordp[1] / (W * H), it_ordp[2] / (W * H),
                   it_ordp[3] / (W * H), it_ordp[4] / (W * H), it_ordp[5] / (W * H));
        if (levels) {
            const char* nm[3] = {"primary", "bounce", "shadow"};
            for (int k = 0; k < 3; ++k) {
                double tot = 0, cum = 0, bytes = 0;
                for (double v : lv_hist[k]) tot += v;
                printf("levels %-8s fetches/ray by level (cumulative share, nodes up to it, KB):", nm[k]);
                size_t nodes = 0;
                for (int l = 0; l < 8 && lv_hist[k][l] > 0; ++l) {
                    cum += lv_hist[k][l]; nodes += lv_nodes[l]; bytes = nodes * 80.0;
                    printf(" L%d %.0f%% (%zu, %.1f)", l, 100.0 * cum / tot, nodes, bytes / 1024.0);
                }
                printf("  [%.2f fetches/ray]\n", tot / (k == 0 ? (double)W * H : (k == 1 ? (double)nb : (double)ns)));
            }
        }
        if (getenv("COHERENCE")) {
            // per 16x16 workgroup and candidate: 256 shadow rays (pixel -> random emitter point) walked by
            // 4 waves of 64.  Per wave: lockstep steps (its longest walk) and the node fetches the vector
            // memory path processes, counted as distinct nodes among the lanes per step.  Groupings: the
            // 8x8 pixel quadrants (the kernels' layout) vs the 256 rays sorted by a target key.
            const int K = 8;
            const char* names[4] = {"8x8 pixels", "sorted by emitter", "sorted by target Morton", "sorted by dir octant+Morton"};
            double st[4] = {0, 0, 0, 0}, ds[4] = {0, 0, 0, 0}, un[4] = {0, 0, 0, 0}, lane_f = 0; long nwave = 0;
            std::mt19937 rg2(5);
            for (int ty = 0; ty + 16 <= H; ty += 16)
                for (int tx = 0; tx + 16 <= W; tx += 16) {
                    V3 org[256]; bool ok[256];
                    for (int l = 0; l < 256; ++l) {
                        int q4 = l >> 6, ll = l & 63;
                        int x = tx + (q4 & 1) * 8 + (ll & 7), y = ty + (q4 >> 1) * 8 + (ll >> 3);
                        V3 dc{(float)x - W / 2.0f, H / 2.0f - (float)y, -focal};
                        V3 d = xc * dc.x + yc * dc.y + zc * dc.z;
                        d = d * (1.0f / std::sqrt(dot(d, d)));
                        WEmu a = emu_walk(WN, pr, Ray{eye, d, 0.01f, 3.0e38f, true}, false, 8);
                        ok[l] = a.prim >= 0; org[l] = eye + d * a.t;
                    }
                    for (int k = 0; k < K; ++k) {
                        std::vector<std::vector<uint32_t>> seq(256);
                        uint64_t key[4][256];
                        for (int l = 0; l < 256; ++l) {
                            int e = emis[rg2() % ne];
                            float r1 = U(rg2), r2 = U(rg2), sr = std::sqrt(r1);
                            const Tri& t = g_tris[e];
                            V3 q = t.v0 * (1 - sr) + t.v1 * (sr * (1 - r2)) + t.v2 * (sr * r2);
                            auto qb = [](float v) { return (uint32_t)std::min(1023.0f, std::max(0.0f, (v + 20.0f) * 25.0f)); };
                            uint32_t mx = qb(q.x), my = qb(q.y), mz = qb(q.z); uint64_t m = 0;
                            for (int bb = 0; bb < 10; ++bb) m |= (uint64_t)((((mx >> bb) & 1) << (3 * bb)) | (((my >> bb) & 1) << (3 * bb + 1)) | (((mz >> bb) & 1) << (3 * bb + 2)));
                            V3 sd = q - org[l];
                            const uint64_t oct = (sd.x < 0) | ((sd.y < 0) << 1) | ((sd.z < 0) << 2);
                            key[0][l] = l; key[1][l] = ((uint64_t)e << 8) | l; key[2][l] = (m << 8) | l; key[3][l] = (((oct << 30) | m) << 8) | l;
                            if (!ok[l]) continue;
                            float dist = std::sqrt(dot(sd, sd));
                            sd = sd * (1.0f / std::max(dist, 1e-20f));
                            emu_walk(WN, pr, Ray{org[l], sd, 0.01f, dist - 0.001f, true}, true, 8, &seq[l]);
                            lane_f += seq[l].size();
                        }
                        for (int g = 0; g < 4; ++g) {
                            std::sort(key[g], key[g] + 256);
                            for (int w = 0; w < 4; ++w) {
                                size_t T = 0;
                                for (int i = 0; i < 64; ++i) T = std::max(T, seq[key[g][64 * w + i] & 255].size());
                                st[g] += T;
                                {   // the union of the wave's walks: steps of a wave-lockstep wide walk
                                    std::vector<uint32_t> u;
                                    for (int i = 0; i < 64; ++i) { auto& q = seq[key[g][64 * w + i] & 255]; u.insert(u.end(), q.begin(), q.end()); }
                                    std::sort(u.begin(), u.end()); un[g] += std::unique(u.begin(), u.end()) - u.begin();
                                }
                                for (size_t t = 0; t < T; ++t) {
                                    uint32_t v[64]; int nv = 0;
                                    for (int i = 0; i < 64; ++i) { auto& q = seq[key[g][64 * w + i] & 255]; if (t < q.size()) v[nv++] = q[t]; }
                                    std::sort(v, v + nv); ds[g] += std::unique(v, v + nv) - v;
                                }
                            }
                        }
                        nwave += 4;
                    }
                }
            printf("coherence: lane fetches per ray %.2f\n", lane_f / (nwave * 64.0));
            for (int g = 0; g < 4; ++g)
                printf("  %-28s steps per wave %.1f, distinct node fetches per wave %.1f (per step %.1f), union %.1f\n", names[g],
                       st[g] / nwave, ds[g] / nwave, ds[g] / st[g], un[g] / nwave);
        }
        if (getenv("COHERENCE_WAVE")) {
            // one wave = an 8x8 pixel tile with K area candidates per pixel (64 K shadow rays).  As the kernels
            // run them: candidate by candidate (lane = pixel).  Regrouped: the wave's 64 K rays sorted by a key
            // and traced 64 at a time in sorted order (lane = sorted position).  Per wave: lockstep steps (sum
            // over the K groups of the longest walk) and the distinct nodes per step (the lines the vector
            // memory path returns), summed.
            const int K = getenv("K") ? atoi(getenv("K")) : 32;
            const int RB = getenv("RANK_BITS") ? atoi(getenv("RANK_BITS")) : 12;   // buckets of the emitter's spatial rank
            const char* names[4] = {"per candidate (kernel)", "by emitter spatial rank (bucketed)", "sorted by target Morton", "sorted by octant+Morton"};
            // each emitter's rank in the Morton order of the emitter centroids (a per-scene table)
            std::vector<uint32_t> erank(g_tris.size(), 0);
            {
                std::vector<std::pair<uint64_t, int>> order;
                for (int e : emis) {
                    const Tri& t = g_tris[e];
                    V3 c = (t.v0 + t.v1 + t.v2) * (1.0f / 3.0f);
                    auto qb = [](float v) { return (uint32_t)std::min(1023.0f, std::max(0.0f, (v + 20.0f) * 25.0f)); };
                    uint32_t mx = qb(c.x), my = qb(c.y), mz = qb(c.z); uint64_t m = 0;
                    for (int bb = 0; bb < 10; ++bb) m |= (uint64_t)((((mx >> bb) & 1) << (3 * bb)) | (((my >> bb) & 1) << (3 * bb + 1)) | (((mz >> bb) & 1) << (3 * bb + 2)));
                    order.push_back({m, e});
                }
                std::sort(order.begin(), order.end());
                for (size_t i = 0; i < order.size(); ++i) erank[order[i].second] = (uint32_t)((i << RB) / order.size());
            }
            double st[4] = {0, 0, 0, 0}, ds[4] = {0, 0, 0, 0}, bu[4] = {0, 0, 0, 0}, wu[4] = {0, 0, 0, 0};
            long nwave = 0;
            std::mt19937 rg2(7);
            const int stride = getenv("WSTRIDE") ? atoi(getenv("WSTRIDE")) : 4;   // every stride-th tile in x and y
            for (int ty = 0; ty + 8 <= H; ty += 8 * stride)
                for (int tx = 0; tx + 8 <= W; tx += 8 * stride) {
                    V3 org[64]; bool ok[64];
                    for (int l = 0; l < 64; ++l) {
                        int x = tx + (l & 7), y = ty + (l >> 3);
                        V3 dc{(float)x - W / 2.0f, H / 2.0f - (float)y, -focal};
                        V3 d = xc * dc.x + yc * dc.y + zc * dc.z;
                        d = d * (1.0f / std::sqrt(dot(d, d)));
                        WEmu a = emu_walk(WN, pr, Ray{eye, d, 0.01f, 3.0e38f, true}, false, 8);
                        ok[l] = a.prim >= 0; org[l] = eye + d * a.t;
                    }
                    const int R = 64 * K;
                    std::vector<std::vector<uint32_t>> seq(R);
                    std::vector<std::vector<int>> bvis(R);      // binary skip-pointer walk: visited nodes
                    std::vector<uint64_t> key[4];
                    for (int g = 0; g < 4; ++g) key[g].resize(R);
                    for (int c = 0; c < K; ++c)
                        for (int l = 0; l < 64; ++l) {
                            const int r = c * 64 + l;
                            int e = emis[rg2() % ne];
                            float r1 = U(rg2), r2 = U(rg2), sr = std::sqrt(r1);
                            const Tri& t = g_tris[e];
                            V3 q = t.v0 * (1 - sr) + t.v1 * (sr * (1 - r2)) + t.v2 * (sr * r2);
                            auto qb = [](float v) { return (uint32_t)std::min(1023.0f, std::max(0.0f, (v + 20.0f) * 25.0f)); };
                            uint32_t mx = qb(q.x), my = qb(q.y), mz = qb(q.z); uint64_t m = 0;
                            for (int bb = 0; bb < 10; ++bb) m |= (uint64_t)((((mx >> bb) & 1) << (3 * bb)) | (((my >> bb) & 1) << (3 * bb + 1)) | (((mz >> bb) & 1) << (3 * bb + 2)));
                            V3 sd = q - org[l];
                            const uint64_t oct = (sd.x < 0) | ((sd.y < 0) << 1) | ((sd.z < 0) << 2);
                            static const int use_oct = getenv("OCT") ? atoi(getenv("OCT")) : 0;
                            key[0][r] = (uint64_t)r; key[1][r] = ((((use_oct ? oct : 0) << RB) | (uint64_t)erank[e]) << 12) | r;
                            key[2][r] = (m << 12) | r;
                            key[3][r] = (((oct << 30) | m) << 12) | r;
                            if (!ok[l]) continue;
                            float dist = std::sqrt(dot(sd, sd));
                            sd = sd * (1.0f / std::max(dist, 1e-20f));
                            emu_walk(WN, pr, Ray{org[l], sd, 0.01f, dist - 0.001f, true}, true, 8, &seq[r]);
                            walk(Fr, Ray{org[l], sd, 0.01f, dist - 0.001f, true}, true, &bvis[r]);
                        }
                    for (int g = 0; g < 4; ++g) {
                        std::sort(key[g].begin(), key[g].end());
                        for (int c = 0; c < K; ++c) {   // binary lockstep: the wave steps through the union of its lanes' visits
                            std::vector<int> u;
                            for (int i = 0; i < 64; ++i) { auto& q = bvis[key[g][64 * c + i] & 4095]; u.insert(u.end(), q.begin(), q.end()); }
                            std::sort(u.begin(), u.end());
                            bu[g] += std::unique(u.begin(), u.end()) - u.begin();
                        }
                        for (int c = 0; c < K; ++c) {   // wide lockstep: the wave fetches the union of its lanes' wide nodes
                            std::vector<uint32_t> u;
                            for (int i = 0; i < 64; ++i) { auto& q = seq[key[g][64 * c + i] & 4095]; u.insert(u.end(), q.begin(), q.end()); }
                            std::sort(u.begin(), u.end());
                            wu[g] += std::unique(u.begin(), u.end()) - u.begin();
                        }
                        for (int c = 0; c < K; ++c) {
                            size_t T = 0;
                            for (int i = 0; i < 64; ++i) T = std::max(T, seq[key[g][64 * c + i] & 4095].size());
                            st[g] += T;
                            for (size_t s = 0; s < T; ++s) {
                                uint32_t v[64]; int nv = 0;
                                for (int i = 0; i < 64; ++i) { auto& q = seq[key[g][64 * c + i] & 4095]; if (s < q.size()) v[nv++] = q[s]; }
                                std::sort(v, v + nv); ds[g] += std::unique(v, v + nv) - v;
                            }
                        }
                    }
                    ++nwave;
                }
            printf("wave coherence (8x8 tile, K=%d candidates, %ld waves):\n", K, nwave);
            for (int g = 0; g < 4; ++g)
                printf("  %-26s steps per wave %.1f, distinct node fetches per wave %.1f (per step %.2f) | binary lockstep union %.1f"
                       " | wide lockstep union %.1f\n",
                       names[g], st[g] / nwave, ds[g] / nwave, ds[g] / st[g], bu[g] / nwave, wu[g] / nwave);
        }
        double wsum = 0; for (int v : wave_it) wsum += v;
        printf("emu: primary iters %.2f tris %.2f | bounce iters %.2f tris %.2f | shadow iters %.2f tris %.2f lost %.4f max stack %d wave-max iters %.1f | mismatches %ld | nodes %zu\n",
               it_p / (W * H), tr_p / (W * H), it_b / std::max(nb, 1L), tr_b / std::max(nb, 1L), it_s / ns, tr_s / ns,
               (double)lost / ns, maxsp, wsum / wave_it.size(), mism, WN.size() / 20);
        return 0;
    }
    const int wide_k = getenv("WIDE") ? atoi(getenv("WIDE")) : 0;
    Flat F = make_flat(T, max_leaf, 1.0f, ctri, ord);
    Wide Wd;
    if (wide_k) {
        std::vector<char> leafify(T.n.size(), 0);
        std::vector<float> cost(T.n.size(), 0);
        collapse(T, T.root, max_leaf, 1.0f, ctri, leafify, cost);
        wide_rec(T, T.root, leafify, wide_k, Wd);
    }
    int max_stack = 0;
    int interior = 0, leaves = 0, maxleaf = 0;
    for (auto& n : F.n) { if (n.cnt) { ++leaves; maxleaf = std::max(maxleaf, n.cnt); } else ++interior; }

    // camera: pg/camera.cpp GenerateRay (pixel-corner rays, Z-up lookAt)
    V3 eye{cam[0], cam[1], cam[2]}, at{cam[3], cam[4], cam[5]};
    float fov = cam[6] * 3.14159265358979f / 180.0f;
    V3 zc = eye - at; zc = zc * (1.0f / std::sqrt(dot(zc, zc)));
    V3 up{0, 0, 1};
    V3 xc = cross(up, zc); xc = xc * (1.0f / std::sqrt(dot(xc, xc)));
    V3 yc = cross(zc, xc);
    float focal = (float)H / (2.0f * std::tan(fov / 2.0f));
    const int npx = W * H;
    std::vector<Ray> prim(npx), shad(npx);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            V3 dc{(float)x - W / 2.0f, H / 2.0f - (float)y, -focal};
            V3 d = xc * dc.x + yc * dc.y + zc * dc.z;
            d = d * (1.0f / std::sqrt(dot(d, d)));
            prim[y * W + x] = Ray{eye, d, 0.01f, 3.0e38f, true};
        }
    std::vector<Trace> tp(npx), ts(npx);
#pragma omp parallel for schedule(dynamic, 256)
    for (int p = 0; p < npx; ++p) { int ms = 0; tp[p] = wide_k ? walk_wide(Wd, prim[p], false, ms) : walk(F, prim[p], false);
#pragma omp critical
        max_stack = std::max(max_stack, ms); }
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    std::vector<char> pact(npx, 1), sact(npx, 0);
    for (int p = 0; p < npx; ++p) {
        if (tp[p].prim < 0) { shad[p].active = false; continue; }
        V3 o = prim[p].o + prim[p].d * tp[p].t;
        int e = emis[rng() % ne];
        float r1 = U(rng), r2 = U(rng), sr = std::sqrt(r1);
        const Tri& t = g_tris[e];
        V3 q = t.v0 * (1 - sr) + t.v1 * (sr * (1 - r2)) + t.v2 * (sr * r2);
        V3 d = q - o;
        float dist = std::sqrt(dot(d, d));
        d = d * (1.0f / std::max(dist, 1e-20f));
        shad[p] = Ray{o, d, 0.01f, dist - 0.001f, true};
        sact[p] = 1;
    }
#pragma omp parallel for schedule(dynamic, 256)
    for (int p = 0; p < npx; ++p) { int ms = 0; ts[p] = wide_k ? walk_wide(Wd, shad[p], true, ms) : walk(F, shad[p], true);
#pragma omp critical
        max_stack = std::max(max_stack, ms); }
    if (wide_k) {
        std::vector<long> hist(32, 0);
        for (int p = 0; p < npx; ++p) { hist[std::min(31, group_depth(Wd, prim[p], false))]++; if (sact[p]) hist[std::min(31, group_depth(Wd, shad[p], true))]++; }
        printf("group stack depth histogram:");
        for (int d = 0; d < 16; ++d) if (hist[d]) printf(" %d:%ld", d, hist[d]);
        printf("\n");
    }
    Stats SP, SS;
    wave_stats(tp, pact, W, H, SP);
    wave_stats(ts, sact, W, H, SS);
    long occ = 0;
    for (int p = 0; p < npx; ++p) occ += sact[p] && ts[p].occ;
    auto p95 = [](std::vector<int>& v) { std::sort(v.begin(), v.end()); return v.empty() ? 0 : v[(size_t)(0.95 * v.size())]; };
    if (wide_k) {
        std::vector<int> dep(Wd.n.size(), 0);
        int md = 0;
        for (size_t i = 0; i < Wd.n.size(); ++i)        // parents precede children (preorder ids)
            for (auto& c : Wd.n[i].c) if (c.node >= 0) { dep[c.node] = dep[i] + 1; md = std::max(md, dep[c.node]); }
        printf("[wide %d: %zu nodes, depth %d, max stack (pairs) %d] ", wide_k, Wd.n.size(), md, max_stack);
    }
    printf("%-7s leaf<=%d ctri=%.1f ord=%d nodes=%zu (leaves %d, max leaf %d, refs %zu) | primary visits %.1f p95 %d tris %.2f "
           "wave steps %.1f tri-iters %.1f | shadow visits %.1f p95 %d tris %.2f wave steps %.1f tri-iters %.1f occluded %.3f\n",
           which.c_str(), max_leaf, ctri, (int)ord, F.n.size(), leaves, maxleaf, F.leaf_prims.size(),
           SP.visits / SP.rays, p95(SP.vis), SP.tris / SP.rays, SP.wave_steps / SP.waves, SP.wave_tri_iters / SP.waves,
           SS.visits / SS.rays, p95(SS.vis), SS.tris / SS.rays, SS.wave_steps / SS.waves, SS.wave_tri_iters / SS.waves,
           (double)occ / SS.rays);
    return 0;
}
