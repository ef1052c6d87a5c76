// TEST INFRASTRUCTURE: CPU checks of the 8-wide tree of the per-lane walks (restir-embree_amd/csrc/rs_wide.h,
// the collapse rs_bvh_build.hip runs after every PLOC build) and of the walk's quantised box test
// (rs_scene.h wide_hits, restated here with the same float operations).  Built by tests/test_wide_bvh.py.
//   collapse: 0 greedy, 1 SAH-optimal (both over the random merge tree), 2 SAH-optimal over rs_wide.h
//   build_sah_host's top-down SAH tree (the product's default)
//   wide_check: structure (breadth-first layout, slots, every triangle exactly once, depth) and
//               conservativeness (every dequantised child box contains the exact child box)
//   wide_query: random rays (incl. axis-parallel directions and origins on box planes) through the wide walk
//               restated on the CPU vs brute force over all triangles: closest hit (t, prim, tie rule) and
//               any hit must be identical
#include "../../restir-embree_amd/csrc/rs_wide.h"

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <string>
#include <vector>

namespace {
struct V { float x, y, z; };
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V crs(V a, V b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
float dt(V a, V b) { float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return x + y + z; }

struct Scene {
    std::vector<float> pos;            // 9 per triangle
    std::vector<float> nlo, nhi;       // PLOC-shaped nodes, 4 floats each
    int n = 0, root = 0;
};
float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

// random triangles (clustered, some long and thin, some axis-aligned) and a random binary merge tree
// (ids < n primitives, n.. internal) shaped like the PLOC output
void make_scene(Scene& S, int n, uint32_t seed) {
    std::mt19937 rng(seed);
    std::uniform_real_distribution<float> U(-1.0f, 1.0f);
    S.n = n;
    S.pos.resize(9 * (size_t)n);
    for (int t = 0; t < n; ++t) {
        float c[3] = {U(rng) * 8.0f, U(rng) * 4.0f, U(rng) * 3.0f + 3.0f};
        const int kind = (int)(rng() % 5);
        if (kind == 4) { c[0] = 0.0f; c[1] = (rng() % 2) ? 0.0f : -7.0f; }          // on the zero planes
        for (int v = 0; v < 3; ++v)
            for (int a = 0; a < 3; ++a) {
                float d = U(rng) * (kind == 0 ? 0.05f : kind == 1 ? 0.5f : 0.2f);
                if (kind == 2 && a == 2) d = 0.0f;                           // flat in z (lamp-like)
                if (kind == 3 && a == 0) d = U(rng) * 3.0f;                  // long and thin
                if (kind == 4 && a < 2) d = (rng() % 3 == 0) ? 0.0f : U(rng) * 1e-15f;   // tiny offsets from 0 / -7
                S.pos[9 * (size_t)t + 3 * v + a] = c[a] + d;
            }
    }
    const int total = 2 * n - 1;
    S.nlo.assign(4 * (size_t)total, 0.0f); S.nhi.assign(4 * (size_t)total, 0.0f);
    for (int t = 0; t < n; ++t)
        for (int a = 0; a < 3; ++a) {
            const float* p = &S.pos[9 * (size_t)t];
            S.nlo[4 * t + a] = std::min(std::min(p[a], p[3 + a]), p[6 + a]);
            S.nhi[4 * t + a] = std::max(std::max(p[a], p[3 + a]), p[6 + a]);
        }
    for (int t = 0; t < n; ++t) { S.nlo[4 * t + 3] = u2f(0xffffffffu); S.nhi[4 * t + 3] = u2f((uint32_t)t); }
    // merge neighbours in a spatially sorted order (a few random merges for bad trees)
    std::vector<int> C(n);
    for (int i = 0; i < n; ++i) C[i] = i;
    std::sort(C.begin(), C.end(), [&](int a, int b) { return S.nlo[4 * a] < S.nlo[4 * b]; });
    int next = n;
    while (C.size() > 1) {
        std::vector<int> nc;
        for (size_t i = 0; i < C.size(); i += 2) {
            if (i + 1 == C.size() || rng() % 7 == 0) { nc.push_back(C[i]); if (i + 1 < C.size()) nc.push_back(C[i + 1]); continue; }
            const int L = C[i], R = C[i + 1], id = next++;
            for (int a = 0; a < 3; ++a) {
                S.nlo[4 * id + a] = std::min(S.nlo[4 * L + a], S.nlo[4 * R + a]);
                S.nhi[4 * id + a] = std::max(S.nhi[4 * L + a], S.nhi[4 * R + a]);
            }
            S.nlo[4 * id + 3] = u2f((uint32_t)L); S.nhi[4 * id + 3] = u2f((uint32_t)R);
            nc.push_back(id);
        }
        C.swap(nc);
    }
    S.root = C[0];
}

// rs_scene.h tri_test (Moller-Trumbore, fixed op order, no contraction: compiled with -ffp-contract=off)
bool tri_test(const float* p, V o, V d, float tn, float tf, float& t) {
    V v0{p[0], p[1], p[2]};
    V e1{p[3] - p[0], p[4] - p[1], p[5] - p[2]}, e2{p[6] - p[0], p[7] - p[1], p[8] - p[2]};
    V pv = crs(d, e2);
    float det = dt(e1, pv);
    if (det == 0.0f) return false;
    float inv = 1.0f / det;
    V sv = sub(o, v0);
    float u = dt(sv, pv) * inv;
    if (!(u >= 0.0f && u <= 1.0f)) return false;
    V q = crs(sv, e1);
    float v = dt(d, q) * inv;
    if (!(v >= 0.0f && u + v <= 1.0f)) return false;
    t = dt(e2, q) * inv;
    return t >= tn && t <= tf;
}

// rs_scene.h wide_hits, the same float operations (fmaf = the device's v_fma_f32)
uint32_t wide_hits(const uint32_t* w, V o, V inv, float tnear, float tfar) {
    const uint32_t eb = w[3];
    const float s[3] = {u2f((eb & 0xffu) << 23), u2f(((eb >> 8) & 0xffu) << 23), u2f(((eb >> 16) & 0xffu) << 23)};
    const float iv[3] = {inv.x, inv.y, inv.z}, org[3] = {o.x, o.y, o.z};
    float a[3], b[3];
    float bn[3], bf[3];
    for (int k = 0; k < 3; ++k) {
        a[k] = s[k] * iv[k]; b[k] = (u2f(w[k]) - org[k]) * iv[k];
        const float e = 2.384185791015625e-07f * std::fabs(b[k]);
        bn[k] = b[k] - e; bf[k] = b[k] + e;
    }
    const uint32_t lo[3][2] = {{w[6], w[7]}, {w[8], w[9]}, {w[10], w[11]}};
    const uint32_t hi[3][2] = {{w[12], w[13]}, {w[14], w[15]}, {w[16], w[17]}};
    const float lo_k = 1.0f - 4.0f * FLT_EPSILON, hi_k = 1.0f + 4.0f * FLT_EPSILON;
    uint32_t hits = 0;
    for (int c = 0; c < 8; ++c) {
        float tn[3], tf[3];
        for (int k = 0; k < 3; ++k) {
            const bool pos = iv[k] >= 0.0f;
            const uint32_t qn = pos ? lo[k][c >> 2] : hi[k][c >> 2], qf = pos ? hi[k][c >> 2] : lo[k][c >> 2];
            tn[k] = std::fma((float)((qn >> (8 * (c & 3))) & 0xffu), a[k], bn[k]);
            tf[k] = std::fma((float)((qf >> (8 * (c & 3))) & 0xffu), a[k], bf[k]);
        }
        const float t0 = std::fmax(std::fmax(std::fmax(tnear, tn[0]), tn[1]), tn[2]);
        const float t1 = std::fmin(std::fmin(std::fmin(tfar, tf[0]), tf[1]), tf[2]);
        if (t0 * lo_k <= t1 * hi_k) hits |= 1u << c;
    }
    const uint32_t nv = w[3] >> 28;
    return hits & ((1u << nv) - 1u);
}

// the walk's visit order does not matter for the result; a plain recursive walk over the same tests
void walk(const std::vector<uint32_t>& W, const std::vector<int>& prims, const Scene& S, uint32_t node, V o, V d, V inv,
          float tn, float& tf, int& prim, bool any, bool& occ) {
    const uint32_t* w = &W[20 * (size_t)node];
    const uint32_t hits = wide_hits(w, o, inv, tn, any ? tf : tf);
    const uint32_t ni = (w[3] >> 24) & 0xfu;
    for (uint32_t c = 0; c < 8 && !occ; ++c) {
        if (!((hits >> c) & 1u)) continue;
        if (c < ni) { walk(W, prims, S, w[4] + c, o, d, inv, tn, tf, prim, any, occ); continue; }
        const int p = prims[w[5] + c - ni];
        float t;
        if (tri_test(&S.pos[9 * (size_t)p], o, d, tn, tf, t)) {
            if (any) { occ = true; return; }
            if (prim < 0 || t < tf || (t == tf && p < prim)) { tf = t; prim = p; }
        }
    }
}
}  // namespace

extern "C" {
// the host restatement of the product's build (build_sah_host + SAH-optimal collapse within the walk's depth)
// over caller positions: returns the number of wide nodes (words: 20 each) or -1; *n_prims = leaf triangles.
// The GPU builder (rs_wide_build.hip) must produce the same words (tests/test_gpu_parity.py).
int wide_build_host(const float* pos, int n, uint32_t* words, int cap_nodes, int* prims, int* n_prims, int* depth_out) {
    for (size_t i = 0; i < 9 * (size_t)n; ++i)
        if (!rs::w_finite(pos[i])) return -2;          // non-finite geometry: the GPU builds no tree either
    std::vector<float> nlo, nhi;
    const int root = rs::build_sah_host(pos, n, nlo, nhi);
    rs::SahCollapse sah;
    if (n > 1 && !sah.plan(nlo.data(), nhi.data(), n, root, 1.0f, 0.3f, 8)) return -2;   // the GPU builds no tree
    std::vector<uint32_t> W;
    std::vector<int> P;
    int depth = 0;
    std::string err;
    if (rs::build_wide_host(nlo.data(), nhi.data(), n, root, W, P, depth, err, 1) != 0) return -1;
    const int nn = (int)(W.size() / 20);
    if (nn > cap_nodes) return -3;
    std::memcpy(words, W.data(), W.size() * sizeof(uint32_t));
    std::memcpy(prims, P.data(), P.size() * sizeof(int));
    *n_prims = (int)P.size();
    *depth_out = depth;
    return nn;
}
// structure + conservativeness; returns the number of wide nodes (> 0) or a negative code, msg = reason
int wide_check(int n, uint32_t seed, int* depth_out, char* msg, int msg_len, int collapse) {
    Scene S;
    make_scene(S, n, seed);
    std::vector<uint32_t> W;
    std::vector<int> prims;
    int depth = 0;
    std::string err;
    auto fail = [&](const std::string& m) { if (msg) { std::strncpy(msg, m.c_str(), msg_len - 1); msg[msg_len - 1] = 0; } return -1; };
    if (collapse == 3) {                   // coincident triangles (the source tree's degenerate-centroid split)
        // (a few dozen: the full sweep's ties peel identical boxes off one at a time, so hundreds of copies make
        // a chain too deep for the walk's stack -- the product then builds no wide tree, tests/test_gpu_wide.py)
        for (int t = 1; t < std::min(n / 2, 24); ++t) std::memcpy(&S.pos[9 * (size_t)t], &S.pos[0], 9 * sizeof(float));
        collapse = 2;
    }
    if (collapse == 2) { S.root = rs::build_sah_host(S.pos.data(), S.n, S.nlo, S.nhi); collapse = 1; }   // host SAH source
    if (rs::build_wide_host(S.nlo.data(), S.nhi.data(), S.n, S.root, W, prims, depth, err, collapse) != 0) return fail(err);
    if (depth > 8) return fail("deeper than the walk's stack");
    const size_t nn = W.size() / 20;
    if ((int)prims.size() != n) return fail("triangle count");
    std::vector<int> seen(n, 0);
    for (int p : prims) { if (p < 0 || p >= n) return fail("prim range"); seen[p]++; }
    for (int t = 0; t < n; ++t) if (seen[t] != 1) return fail("triangle not exactly once");
    // exact subtree boxes, bottom-up (breadth-first ids: children after parents)
    std::vector<float> blo(3 * nn, FLT_MAX), bhi(3 * nn, -FLT_MAX);
    std::vector<int> parent(nn, -1), level(nn, 0);
    uint32_t next_child = 1, next_tri = 0;
    for (size_t i = 0; i < nn; ++i) {
        const uint32_t* w = &W[20 * i];
        const uint32_t ni = (w[3] >> 24) & 0xfu, nv = w[3] >> 28;
        if (nv < 1 || nv > 8 || ni > nv) return fail("slot counts");
        if (ni && w[4] != next_child) return fail("interior children not breadth-first contiguous");
        if (nv > ni && w[5] != next_tri) return fail("leaf triangles not contiguous");
        next_child += ni; next_tri += nv - ni;
        for (uint32_t c = 0; c < ni; ++c) { parent[w[4] + c] = (int)i; level[w[4] + c] = level[i] + 1; }
    }
    if (next_child != nn || next_tri != (uint32_t)n) return fail("layout totals");
    int md = 0;
    for (size_t i = 0; i < nn; ++i) md = std::max(md, level[i]);
    if (md != depth) return fail("depth");
    for (size_t ii = nn; ii-- > 0;) {
        const uint32_t* w = &W[20 * ii];
        const uint32_t ni = (w[3] >> 24) & 0xfu, nv = w[3] >> 28;
        const uint32_t e[3] = {w[3] & 0xffu, (w[3] >> 8) & 0xffu, (w[3] >> 16) & 0xffu};
        const uint32_t lo[3][2] = {{w[6], w[7]}, {w[8], w[9]}, {w[10], w[11]}};
        const uint32_t hi[3][2] = {{w[12], w[13]}, {w[14], w[15]}, {w[16], w[17]}};
        for (uint32_t c = 0; c < nv; ++c) {
            float clo[3], chi[3];
            if (c < ni) {
                for (int a = 0; a < 3; ++a) { clo[a] = blo[3 * (w[4] + c) + a]; chi[a] = bhi[3 * (w[4] + c) + a]; }
            } else {
                const float* p = &S.pos[9 * (size_t)prims[w[5] + c - ni]];
                for (int a = 0; a < 3; ++a) {
                    clo[a] = std::min(std::min(p[a], p[3 + a]), p[6 + a]);
                    chi[a] = std::max(std::max(p[a], p[3 + a]), p[6 + a]);
                }
            }
            for (int a = 0; a < 3; ++a) {
                const double s = std::ldexp(1.0, (int)e[a] - 127), o = (double)u2f(w[a]);
                const double ql = (double)((lo[a][c >> 2] >> (8 * (c & 3))) & 0xffu), qh = (double)((hi[a][c >> 2] >> (8 * (c & 3))) & 0xffu);
                if (o + ql * s > (double)clo[a] || o + qh * s < (double)chi[a]) return fail("plane not outward");
                // and the planes are exact floats
                if ((double)(float)(o + ql * s) != o + ql * s || (double)(float)(o + qh * s) != o + qh * s) return fail("plane not a float");
                blo[3 * ii + a] = std::min(blo[3 * ii + a], clo[a]);
                bhi[3 * ii + a] = std::max(bhi[3 * ii + a], chi[a]);
            }
        }
    }
    if (depth_out) *depth_out = depth;
    return (int)nn;
}

// random queries: wide walk (restated) vs brute force; returns the number of rays checked or a negative code
int wide_query(int n, uint32_t seed, int n_rays, int* n_hits, int collapse) {
    Scene S;
    make_scene(S, n, seed);
    std::vector<uint32_t> W;
    std::vector<int> prims;
    int depth = 0;
    std::string err;
    if (collapse == 3) {
        // (a few dozen: the full sweep's ties peel identical boxes off one at a time, so hundreds of copies make
        // a chain too deep for the walk's stack -- the product then builds no wide tree, tests/test_gpu_wide.py)
        for (int t = 1; t < std::min(n / 2, 24); ++t) std::memcpy(&S.pos[9 * (size_t)t], &S.pos[0], 9 * sizeof(float));
        collapse = 2;
    }
    if (collapse == 2) { S.root = rs::build_sah_host(S.pos.data(), S.n, S.nlo, S.nhi); collapse = 1; }
    if (rs::build_wide_host(S.nlo.data(), S.nhi.data(), S.n, S.root, W, prims, depth, err, collapse) != 0) return -1;
    std::mt19937 rng(seed * 7 + 1);
    std::uniform_real_distribution<float> U(-1.0f, 1.0f);
    int hits = 0;
    for (int r = 0; r < n_rays; ++r) {
        V o{U(rng) * 9.0f, U(rng) * 5.0f, U(rng) * 4.0f + 3.0f}, d{U(rng), U(rng), U(rng)};
        const int kind = r % 5;
        if (kind == 1) { d.y = 0.0f; d.z = 0.0f; }                               // axis-parallel
        if (kind == 2) { d.x = 0.0f; }
        if (kind == 3) {                                                          // origin on a triangle's box plane
            const float* p = &S.pos[9 * (size_t)(rng() % n)];
            o.x = std::min(std::min(p[0], p[3]), p[6]);
            d.x = 0.0f;
        }
        if (kind == 4) {                                                          // from a triangle toward another one
            const float* p = &S.pos[9 * (size_t)(rng() % n)];
            const float* q = &S.pos[9 * (size_t)(rng() % n)];
            o = V{(p[0] + p[3] + p[6]) / 3.0f, (p[1] + p[4] + p[7]) / 3.0f, (p[2] + p[5] + p[8]) / 3.0f};
            d = sub(V{(q[0] + q[3] + q[6]) / 3.0f, (q[1] + q[4] + q[7]) / 3.0f, (q[2] + q[5] + q[8]) / 3.0f}, o);
        }
        const float len = std::sqrt(dt(d, d));
        if (!(len > 0.0f)) continue;
        d = V{d.x / len, d.y / len, d.z / len};
        const V inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        const float tn = 0.01f, tf0 = kind == 4 ? len * 0.9f : 3.0e38f;
        // brute force
        float bt = tf0; int bp = -1; bool bocc = false;
        for (int t = 0; t < n; ++t) {
            float th;
            if (tri_test(&S.pos[9 * (size_t)t], o, d, tn, tf0, th)) bocc = true;
            if (tri_test(&S.pos[9 * (size_t)t], o, d, tn, bt, th) && (bp < 0 || th < bt || (th == bt && t < bp))) { bt = th; bp = t; }
        }
        float wt = tf0; int wp = -1; bool occ = false;
        walk(W, prims, S, 0, o, d, inv, tn, wt, wp, false, occ);
        bool wocc = false; float tfa = tf0; int dummy = -1;
        walk(W, prims, S, 0, o, d, inv, tn, tfa, dummy, true, wocc);
        if (wp != bp || (bp >= 0 && f2u(wt) != f2u(bt)) || wocc != bocc) return -(1000 + r);
        hits += bp >= 0;
    }
    if (n_hits) *n_hits = hits;
    return n_rays;
}
}
