// rs_wide_build.hip -- the 8-wide tree of the per-lane walks, built on the GPU (replaces, with the PLOC tree of
// rs_bvh_build.hip, Embree's rtcCommitScene, pg/Scene.cpp:15).  It is the host restatement in rs_wide.h
// (build_sah_host + SahCollapse + build_wide_host, collapse 1) run as data-parallel kernels, and produces the
// same tree word for word (tests/test_gpu_wide.py::test_wide_tree_gpu_equals_host):
//
//   1 k_tri_prep      triangle boxes and centroids (the host's float operations), the identity permutation,
//                     a non-finite flag (no wide tree for non-finite geometry: the walks take the skip pointers)
//   2 large segments  (> kSmall triangles) top-down, one host-driven round per tree level over ALL of the
//                     level's segments at once, split into chunks of kChunk triangles:
//                       k_seg_bounds  centroid / box / triangle-index bounds per segment (ordered-int atomics:
//                                     min / max are order independent, so the result is deterministic)
//                       k_seg_bins    32 bins per axis per segment (LDS per chunk, then global atomics)
//                       k_seg_choose  the binned-SAH split, in double, with the host's loop order and ties
//                       k_seg_side    each triangle's side; per-chunk left counts -> k_seg_scan (per segment)
//                       k_seg_scatter stable partition into a scratch permutation; k_seg_copy copies it back
//                       k_seg_link    the node's child ids
//   3 k_small         every segment of 2..kSmall triangles builds its whole subtree in one workgroup: per node
//                     a bitonic sort of its triangles per axis by (centroid, index) in LDS, prefix / suffix box
//                     scans and the full-sweep SAH costs in double, ties to the first (axis, position)
//   4 k_dp_level      Ylitie et al.'s SAH-optimal collapse tables S(x, k, g), bottom-up one binary depth level
//                     per launch (nodes bucketed by depth with k_depth_count / k_depth_fill)
//   5 k_wide_kids / k_wide_emit   the wide nodes breadth-first, one launch pair per wide level (<= 9): each
//                     node expands its slots from the tables, exclusive scans place its interior children and
//                     leaf triangles, and rs_wide.h wide_encode quantises its child boxes (outward, exact)
//   6 k_wide_gather   the wide-leaf triangles (v0, prim) (e1) (e2)
// Every choice is a function of a node's triangle set, so the arrays' order inside a level never matters.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <float.h>
#include <string>
#include <vector>
#include <algorithm>
#include "rs_refit.h"
#include "../../include/restir_c.h"
#include "rs_wide.h"

namespace rs { hipError_t pool_malloc(void** p, size_t bytes, hipStream_t st); }

namespace rs {
namespace wb {

constexpr int kSmall = 256;         // rs_wide.h build_sah_host kSweepMax
constexpr int kBins = 32;
constexpr int kChunk = 2048;        // triangles per chunk of a large segment (one workgroup)
constexpr int kB = 256;             // threads per workgroup
constexpr float kEmpty = 3.0e38f;   // the host's empty box (rs_wide.h build_sah_host `empty`)
constexpr float kCnode = 1.0f, kCtri = 0.3f;   // build_wide_host's defaults
constexpr int kG = SahCollapse::kG; // g = -1 .. 8
constexpr int kGmax = RS_WIDE_STACK;

__device__ __forceinline__ int f2o(float f) { const int i = __float_as_int(f); return i >= 0 ? i : i ^ 0x7fffffff; }
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }
__device__ __forceinline__ double half_area_d(const float* lo, const float* hi) {   // build_sah_host half_area
    const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
    return x * y + y * z + z * x;
}
__device__ __forceinline__ float area_f(float4 a, float4 z) {                      // SahCollapse area
    const float ex = z.x - a.x, ey = z.y - a.y, ez = z.z - a.z;
    return ex * ey + ey * ez + ez * ex;
}

// ---------------------------------------------------------------- 1 triangles
__global__ void k_tri_prep(const float* __restrict__ pos, int n, float4* tlo, float4* thi, float4* tcen, int* idx,
                           float4* nlo, float4* nhi, int* bad) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const float* p = pos + 9 * (size_t)t;
    float l[3], h[3], c[3];
    bool fin = true;
    for (int a = 0; a < 3; ++a) {
        fin = fin && w_finite(p[a]) && w_finite(p[3 + a]) && w_finite(p[6 + a]);
        l[a] = w_min(w_min(p[a], p[3 + a]), p[6 + a]);
        h[a] = w_max(w_max(p[a], p[3 + a]), p[6 + a]);
        c[a] = 0.5f * l[a] + 0.5f * h[a];
    }
    if (!fin) atomicOr(bad, 1);
    tlo[t] = make_float4(l[0], l[1], l[2], 0.0f);
    thi[t] = make_float4(h[0], h[1], h[2], 0.0f);
    tcen[t] = make_float4(c[0], c[1], c[2], 0.0f);
    idx[t] = t;
    nlo[t] = make_float4(l[0], l[1], l[2], 0.0f);
    nhi[t] = make_float4(h[0], h[1], h[2], __int_as_float(t));
}

// ---------------------------------------------------------------- 2 large segments
struct Seg { int first, count, id, depth; };
struct Chunk { int seg, begin, end, pad; };
struct SegAcc {
    int cb[6];                       // centroid bounds (ordered ints): lo xyz, hi xyz
    int nb[6];                       // node box
    int imin, imax;                  // triangle index range
    int cnt[3][kBins];
    int blo[3][kBins][3], bhi[3][kBins][3];
};
struct SegDec { int bax, bb, mid, left; double sc; float clo; int pad; };

__global__ void k_acc_init(SegAcc* acc, int ns) {
    const int s = blockIdx.x;
    if (s >= ns) return;
    SegAcc& A = acc[s];
    for (int i = threadIdx.x; i < 3 * kBins; i += blockDim.x) {
        const int a = i / kBins, b = i % kBins;
        A.cnt[a][b] = 0;
        for (int k = 0; k < 3; ++k) { A.blo[a][b][k] = f2o(kEmpty); A.bhi[a][b][k] = f2o(-kEmpty); }
    }
    if (threadIdx.x == 0) {
        for (int k = 0; k < 3; ++k) {
            A.cb[k] = f2o(kEmpty); A.cb[3 + k] = f2o(-kEmpty);
            A.nb[k] = f2o(kEmpty); A.nb[3 + k] = f2o(-kEmpty);
        }
        A.imin = INT32_MAX; A.imax = INT32_MIN;
    }
}

__device__ __forceinline__ int wave_min(int v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

__global__ void __launch_bounds__(kB) k_seg_bounds(const Chunk* __restrict__ ch, const int* __restrict__ idx,
                                                  const float4* __restrict__ tlo, const float4* __restrict__ thi,
                                                  const float4* __restrict__ tcen, SegAcc* acc) {
    const Chunk C = ch[blockIdx.x];
    int v[14];
    for (int k = 0; k < 3; ++k) { v[k] = INT32_MAX; v[3 + k] = INT32_MIN; v[6 + k] = INT32_MAX; v[9 + k] = INT32_MIN; }
    v[12] = INT32_MAX; v[13] = INT32_MIN;
    for (int p = C.begin + (int)threadIdx.x; p < C.end; p += kB) {
        const int t = idx[p];
        const float4 l = tlo[t], h = thi[t], c = tcen[t];
        const float cl[3] = {c.x, c.y, c.z}, ll[3] = {l.x, l.y, l.z}, hh[3] = {h.x, h.y, h.z};
        for (int k = 0; k < 3; ++k) {
            v[k] = min(v[k], f2o(cl[k])); v[3 + k] = max(v[3 + k], f2o(cl[k]));
            v[6 + k] = min(v[6 + k], f2o(ll[k])); v[9 + k] = max(v[9 + k], f2o(hh[k]));
        }
        v[12] = min(v[12], t); v[13] = max(v[13], t);
    }
    __shared__ int red[kB / 64][14];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int k = 0; k < 14; ++k) {
        const bool mx = k == 13 || (k >= 3 && k < 6) || (k >= 9 && k < 12);
        const int r = mx ? wave_max(v[k]) : wave_min(v[k]);
        if (lane == 0) red[wv][k] = r;
    }
    __syncthreads();
    if (threadIdx.x < 14) {
        const int k = threadIdx.x;
        const bool mx = k == 13 || (k >= 3 && k < 6) || (k >= 9 && k < 12);
        int r = red[0][k];
        for (int w = 1; w < kB / 64; ++w) r = mx ? max(r, red[w][k]) : min(r, red[w][k]);
        SegAcc& A = acc[C.seg];
        if (k < 3) atomicMin(&A.cb[k], r);
        else if (k < 6) atomicMax(&A.cb[k], r);
        else if (k < 9) atomicMin(&A.nb[k - 6], r);
        else if (k < 12) atomicMax(&A.nb[k - 6], r);
        else if (k == 12) atomicMin(&A.imin, r);
        else atomicMax(&A.imax, r);
    }
}

// the bin of centroid coordinate c on an axis with bounds [clo, chi] (build_sah_host: min(31, (int)((c - clo) * sc)))
__device__ __forceinline__ int bin_of(float c, float clo, double sc) {
    const int b = (int)(((double)c - clo) * sc);
    return b < kBins - 1 ? b : kBins - 1;
}

__global__ void __launch_bounds__(kB) k_seg_bins(const Chunk* __restrict__ ch, const int* __restrict__ idx,
                                                const float4* __restrict__ tlo, const float4* __restrict__ thi,
                                                const float4* __restrict__ tcen, SegAcc* acc) {
    const Chunk C = ch[blockIdx.x];
    SegAcc& A = acc[C.seg];
    __shared__ int s_cnt[3][kBins], s_lo[3][kBins][3], s_hi[3][kBins][3];
    for (int i = threadIdx.x; i < 3 * kBins; i += kB) {
        const int a = i / kBins, b = i % kBins;
        s_cnt[a][b] = 0;
        for (int k = 0; k < 3; ++k) { s_lo[a][b][k] = f2o(kEmpty); s_hi[a][b][k] = f2o(-kEmpty); }
    }
    float clo[3], chi[3];
    double sc[3];
    for (int a = 0; a < 3; ++a) {
        clo[a] = o2f(A.cb[a]); chi[a] = o2f(A.cb[3 + a]);
        sc[a] = kBins / ((double)chi[a] - clo[a]);
    }
    __syncthreads();
    for (int p = C.begin + (int)threadIdx.x; p < C.end; p += kB) {
        const int t = idx[p];
        const float4 l = tlo[t], h = thi[t], c = tcen[t];
        const float cc[3] = {c.x, c.y, c.z};
        const int lo[3] = {f2o(l.x), f2o(l.y), f2o(l.z)}, hi[3] = {f2o(h.x), f2o(h.y), f2o(h.z)};
        for (int a = 0; a < 3; ++a) {
            if (!(chi[a] > clo[a])) continue;
            const int b = bin_of(cc[a], clo[a], sc[a]);
            atomicAdd(&s_cnt[a][b], 1);
            for (int k = 0; k < 3; ++k) { atomicMin(&s_lo[a][b][k], lo[k]); atomicMax(&s_hi[a][b][k], hi[k]); }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * kBins; i += kB) {
        const int a = i / kBins, b = i % kBins;
        if (!s_cnt[a][b]) continue;
        atomicAdd(&A.cnt[a][b], s_cnt[a][b]);
        for (int k = 0; k < 3; ++k) { atomicMin(&A.blo[a][b][k], s_lo[a][b][k]); atomicMax(&A.bhi[a][b][k], s_hi[a][b][k]); }
    }
}

// one workgroup per segment: build_sah_host's binned loop, same precision and the same choice.  Thread (a, b) forms
// the left box (bins 0..b-1) and the right box (bins b..31) of split b on axis a from the bins staged in LDS -- the
// unions are exact float min / max, so any order gives the host's boxes -- and the lowest cost wins with the host's
// tie rule (first axis, then first bin).  (One thread per segment walking the 96 bins through global memory took
// 0.11 ms per level, 1.5 ms of C3's build: VERDICT r4.)
constexpr int kChooseThreads = 128;
__global__ void __launch_bounds__(kChooseThreads) k_seg_choose(const Seg* __restrict__ segs, int ns, const SegAcc* __restrict__ acc,
                                                               SegDec* dec, float4* nlo, float4* nhi) {
    const int s = blockIdx.x;
    if (s >= ns) return;
    const SegAcc& A = acc[s];
    __shared__ int s_cnt[3][kBins];
    __shared__ float s_lo[3][kBins][3], s_hi[3][kBins][3];
    __shared__ double s_cost[3 * kBins];
    for (int i = threadIdx.x; i < 3 * kBins; i += kChooseThreads) {
        const int a = i / kBins, b = i % kBins;
        s_cnt[a][b] = A.cnt[a][b];
        for (int k = 0; k < 3; ++k) { s_lo[a][b][k] = o2f(A.blo[a][b][k]); s_hi[a][b][k] = o2f(A.bhi[a][b][k]); }
    }
    __syncthreads();
    float clo[3], chi[3];
    for (int a = 0; a < 3; ++a) { clo[a] = o2f(A.cb[a]); chi[a] = o2f(A.cb[3 + a]); }
    if (threadIdx.x < 3 * kBins) {
        const int a = threadIdx.x / kBins, b = threadIdx.x % kBins;
        double cost = -1.0;                                   // -1: no split here
        if (b >= 1 && chi[a] > clo[a]) {
            float llo[3] = {kEmpty, kEmpty, kEmpty}, lhi[3] = {-kEmpty, -kEmpty, -kEmpty};
            float rlo[3] = {kEmpty, kEmpty, kEmpty}, rhi[3] = {-kEmpty, -kEmpty, -kEmpty};
            int cl = 0, cr = 0;
            for (int j = 0; j < kBins; ++j) {
                if (j < b) {
                    for (int k = 0; k < 3; ++k) { llo[k] = w_min(llo[k], s_lo[a][j][k]); lhi[k] = w_max(lhi[k], s_hi[a][j][k]); }
                    cl += s_cnt[a][j];
                } else {
                    for (int k = 0; k < 3; ++k) { rlo[k] = w_min(rlo[k], s_lo[a][j][k]); rhi[k] = w_max(rhi[k], s_hi[a][j][k]); }
                    cr += s_cnt[a][j];
                }
            }
            if (cl && cr) cost = half_area_d(llo, lhi) * cl + half_area_d(rlo, rhi) * cr;
        }
        s_cost[threadIdx.x] = cost;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double best = 1e300;
    int bax = -1, bb = 0;
    for (int i = 0; i < 3 * kBins; ++i)                      // axis-major, bin-ascending: the host's loop order
        if (s_cost[i] >= 0.0 && s_cost[i] < best) { best = s_cost[i]; bax = i / kBins; bb = i % kBins; }
    const Seg S = segs[s];
    SegDec D;
    D.bax = bax; D.bb = bb; D.left = 0; D.pad = 0;
    D.mid = A.imin + (A.imax - A.imin) / 2;
    D.clo = bax >= 0 ? clo[bax] : 0.0f;
    D.sc = bax >= 0 ? kBins / ((double)chi[bax] - clo[bax]) : 0.0;
    dec[s] = D;
    // the node box: the union of its triangles' boxes grown from the empty box
    float l[3], h[3];
    for (int k = 0; k < 3; ++k) { l[k] = w_min(kEmpty, o2f(A.nb[k])); h[k] = w_max(-kEmpty, o2f(A.nb[3 + k])); }
    nlo[S.id] = make_float4(l[0], l[1], l[2], 0.0f);
    nhi[S.id] = make_float4(h[0], h[1], h[2], 0.0f);
}

__device__ __forceinline__ bool goes_left(const SegDec& D, int t, const float4* __restrict__ tcen) {
    if (D.bax < 0) return t <= D.mid;
    const float4 c = tcen[t];
    const float v = D.bax == 0 ? c.x : (D.bax == 1 ? c.y : c.z);
    return bin_of(v, D.clo, D.sc) < D.bb;
}

__global__ void __launch_bounds__(kB) k_seg_side(const Chunk* __restrict__ ch, const int* __restrict__ idx,
                                                const float4* __restrict__ tcen, const SegDec* __restrict__ dec,
                                                uint8_t* side, int* chunk_left) {
    const Chunk C = ch[blockIdx.x];
    const SegDec D = dec[C.seg];
    int nl = 0;
    for (int p = C.begin + (int)threadIdx.x; p < C.end; p += kB) {
        const bool l = goes_left(D, idx[p], tcen);
        side[p] = l ? 1 : 0;
        nl += l ? 1 : 0;
    }
    __shared__ int red[kB / 64];
    for (int o = 32; o > 0; o >>= 1) nl += __shfl_xor(nl, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = nl;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kB / 64; ++w) t += red[w];
        chunk_left[blockIdx.x] = t;
    }
}

// per segment: exclusive offsets of its chunks' left / right triangles, and the segment's left count
__global__ void k_seg_scan(const Seg* __restrict__ segs, const int2* __restrict__ seg_chunks, int ns, const Chunk* __restrict__ ch,
                           const int* __restrict__ chunk_left, int2* chunk_off, SegDec* dec) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const int2 r = seg_chunks[s];
    int L = 0, R = 0;
    for (int c = r.x; c < r.y; ++c) {
        chunk_off[c] = make_int2(L, R);
        const int nl = chunk_left[c];
        L += nl;
        R += (ch[c].end - ch[c].begin) - nl;
    }
    dec[s].left = L;
}

__global__ void __launch_bounds__(kB) k_seg_scatter(const Chunk* __restrict__ ch, const Seg* __restrict__ segs,
                                                   const int* __restrict__ idx, const uint8_t* __restrict__ side,
                                                   const int2* __restrict__ chunk_off, const SegDec* __restrict__ dec,
                                                   int* out) {
    const Chunk C = ch[blockIdx.x];
    const Seg S = segs[C.seg];
    const int split = dec[C.seg].left;
    const int2 off = chunk_off[blockIdx.x];
    __shared__ int wl[kB / 64], base_l, base_r;
    if (threadIdx.x == 0) { base_l = 0; base_r = 0; }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int p0 = C.begin; p0 < C.end; p0 += kB) {
        const int p = p0 + (int)threadIdx.x;
        const bool valid = p < C.end;
        const bool l = valid && side[p];
        const uint64_t bl = __ballot(l), bv = __ballot(valid);
        const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
        const int rl = __popcll(bl & below), rr = __popcll(bv & ~bl & below);
        if (lane == 0) wl[wv] = __popcll(bl) | (__popcll(bv & ~bl) << 16);
        __syncthreads();
        int ol = base_l, orr = base_r;
        for (int w = 0; w < wv; ++w) { ol += wl[w] & 0xffff; orr += wl[w] >> 16; }
        if (valid) {
            const int dst = l ? S.first + off.x + ol + rl : S.first + split + off.y + orr + rr;
            out[dst] = idx[p];
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 0; w < kB / 64; ++w) { base_l += wl[w] & 0xffff; base_r += wl[w] >> 16; }
        __syncthreads();
    }
}

__global__ void k_seg_copy(const Chunk* __restrict__ ch, const int* __restrict__ src, int* dst) {
    const Chunk C = ch[blockIdx.x];
    for (int p = C.begin + (int)threadIdx.x; p < C.end; p += blockDim.x) dst[p] = src[p];
}

// child ids: >= 0 a node id, < 0 "the triangle at permutation position -(code + 1)"
__global__ void k_seg_link(const Seg* __restrict__ segs, int ns, const int2* __restrict__ kids, const int* __restrict__ idx,
                           int n, float4* nlo, float4* nhi, int* depth) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ns) return;
    const Seg S = segs[s];
    const int2 k = kids[s];
    const int l = k.x >= 0 ? k.x : idx[-(k.x + 1)], r = k.y >= 0 ? k.y : idx[-(k.y + 1)];
    nlo[S.id].w = __int_as_float(l);
    nhi[S.id].w = __int_as_float(r);
    depth[S.id - n] = S.depth;
}

// ---------------------------------------------------------------- 3 small segments: one workgroup each
struct SmallSeg { int first, count, id, depth; };
// Jobs (nodes) of more than kWaveJob triangles are split by the whole workgroup (bitonic sorts and scans in
// LDS, barriers); smaller ones -- most of a segment's nodes -- go to a list that the four waves drain in
// parallel, each splitting its subtree depth-first in registers (wave_subtree: shuffles, no barriers).  Both
// make the host's decision (build_sah_host: sort by (centroid, triangle id), full-sweep SAH in double, first
// minimum, earlier axes win ties).  Node ids are drawn from one counter in the segment's reserved range; the
// order in which subtrees draw them does not change the wide tree (every later choice is a function of a
// node's triangle set).
constexpr int kWaveJob = 64;

__device__ __forceinline__ bool key_after(int x, float cx, int tx, int y, float cy, int ty) {   // x after y?
    if (x < 0) return y >= 0;                  // padding after everything
    if (y < 0) return false;
    return cy < cx || (cy == cx && ty < tx);
}

__device__ void wave_subtree(int4 J0, int lane, const int* s_tri, float (*s_lo)[kSmall], float (*s_hi)[kSmall],
                             float (*s_cen)[kSmall], int* s_ord, int* s_next, int* s_maxd, int n, float4* nlo,
                             float4* nhi, int* depth) {
    int4 stk = make_int4(0, 0, 0, 0);          // lane i holds stack entry i (depth-first: <= 63 entries)
    if (lane == 0) stk = J0;
    int sp = 1;
    while (sp > 0) {
        int4 J;
        J.x = __shfl(stk.x, sp - 1); J.y = __shfl(stk.y, sp - 1); J.z = __shfl(stk.z, sp - 1); J.w = __shfl(stk.w, sp - 1);
        --sp;
        const int f = J.x, c = J.y;
        int P = 2;                             // sort width: c rounded up to a power of two (lanes >= P idle)
        while (P < c) P <<= 1;
        const bool in = lane < c;
        const int e0 = in ? s_ord[f + lane] : -1;
        double best = 1e300;
        int bax = 0, bs = c / 2;
        int srt[3];
        float pl[3], ph[3];                    // the last axis' prefix box (the node box at lane c - 1)
        for (int a = 0; a < 3; ++a) {
            int x = e0;
            float cx = x >= 0 ? s_cen[a][x] : 0.0f;
            int tx = x >= 0 ? s_tri[x] : 0;
            for (int k = 2; k <= P; k <<= 1)
                for (int j = k >> 1; j > 0; j >>= 1) {
                    const int y = __shfl_xor(x, j);
                    const float cy = __shfl_xor(cx, j);
                    const int ty = __shfl_xor(tx, j);
                    const bool up = (lane & k) == 0, lower = (lane & j) == 0;
                    const bool mine_after = key_after(x, cx, tx, y, cy, ty);
                    // the lower lane of an ascending pair keeps the smaller element
                    const bool take = (lower == up) ? mine_after : key_after(y, cy, ty, x, cx, tx);
                    if (take) { x = y; cx = cy; tx = ty; }
                }
            srt[a] = x;
            float ql[3], qh[3];
            for (int k = 0; k < 3; ++k) {
                pl[k] = in ? s_lo[k][x] : 0.0f; ph[k] = in ? s_hi[k][x] : 0.0f;
                ql[k] = pl[k]; qh[k] = ph[k];
            }
            // inclusive prefix (elements 0..lane) and suffix (lane..c-1) box scans
            for (int o = 1; o < c; o <<= 1) {
                for (int k = 0; k < 3; ++k) {
                    const float ul = __shfl_up(pl[k], o), uh = __shfl_up(ph[k], o);
                    const float dl = __shfl_down(ql[k], o), dh = __shfl_down(qh[k], o);
                    if (in && lane >= o) { pl[k] = w_min(ul, pl[k]); ph[k] = w_max(uh, ph[k]); }
                    if (in && lane + o < c) { ql[k] = w_min(ql[k], dl); qh[k] = w_max(qh[k], dh); }
                }
            }
            // split at i = lane + 1 (left = sorted 0..lane): boxes grown from the empty box
            double cost = 1e300;
            const int i = lane + 1;
            float rl[3], rh[3];
            for (int k = 0; k < 3; ++k) { rl[k] = __shfl_down(ql[k], 1); rh[k] = __shfl_down(qh[k], 1); }
            if (i < c) {
                float ll[3], lh[3], Rl[3], Rh[3];
                for (int k = 0; k < 3; ++k) {
                    ll[k] = w_min(kEmpty, pl[k]); lh[k] = w_max(-kEmpty, ph[k]);
                    Rl[k] = w_min(kEmpty, rl[k]); Rh[k] = w_max(-kEmpty, rh[k]);
                }
                cost = half_area_d(ll, lh) * i + half_area_d(Rl, Rh) * (c - i);
            }
            int bi = i;
            for (int o = 32; o > 0; o >>= 1) {  // first minimum in position order
                const double oc = __shfl_xor(cost, o);
                const int ob = __shfl_xor(bi, o);
                if (oc < cost || (oc == cost && ob < bi)) { cost = oc; bi = ob; }
            }
            if (cost < best) { best = cost; bax = a; bs = bi; }   // earlier axes win ties
        }
        const int xs = bax == 0 ? srt[0] : bax == 1 ? srt[1] : srt[2];
        if (in) s_ord[f + lane] = xs;
        float l[3], h[3];
        for (int k = 0; k < 3; ++k) {
            l[k] = w_min(kEmpty, __shfl(pl[k], c - 1));
            h[k] = w_max(-kEmpty, __shfl(ph[k], c - 1));
        }
        const int cf[2] = {f, f + bs}, cc[2] = {bs, c - bs};
        int cid[2];
        for (int q = 0; q < 2; ++q) {
            if (cc[q] == 1) { cid[q] = s_tri[__shfl(xs, cf[q] - f)]; continue; }
            int id = 0;
            if (lane == 0) { id = atomicAdd(s_next, 1); atomicMax(s_maxd, J.w + 1); }
            cid[q] = __shfl(id, 0);
            if (lane == sp) stk = make_int4(cf[q], cc[q], cid[q], J.w + 1);
            ++sp;
        }
        if (lane == 0) {
            nlo[J.z] = make_float4(l[0], l[1], l[2], __int_as_float(cid[0]));
            nhi[J.z] = make_float4(h[0], h[1], h[2], __int_as_float(cid[1]));
            depth[J.z - n] = J.w;
        }
    }
}

__global__ void __launch_bounds__(kB) k_small(const SmallSeg* __restrict__ segs, const int* __restrict__ idx,
                                             const float4* __restrict__ tlo, const float4* __restrict__ thi,
                                             const float4* __restrict__ tcen, int n, float4* nlo, float4* nhi,
                                             int* depth, int* max_depth) {
    const SmallSeg G = segs[blockIdx.x];
    const int tid = threadIdx.x;
    __shared__ int s_tri[kSmall];
    __shared__ float s_lo[3][kSmall], s_hi[3][kSmall], s_cen[3][kSmall];
    __shared__ int s_ord[kSmall], s_srt[3][kSmall], s_key[kSmall];
    __shared__ float s_plo[3][kSmall], s_phi[3][kSmall], s_qlo[3][kSmall], s_qhi[3][kSmall];
    __shared__ double s_bc[kB / 64];
    __shared__ int s_bi[kB / 64];
    __shared__ int4 s_job[kSmall / kWaveJob + 8];
    __shared__ int4 s_wjob[kSmall / 2];
    __shared__ int s_sp, s_next, s_maxd, s_nw, s_take;
    __shared__ double s_best;
    __shared__ int s_bax, s_bs;
    if (tid < G.count) {
        const int t = idx[G.first + tid];
        s_tri[tid] = t;
        const float4 l = tlo[t], h = thi[t], c = tcen[t];
        s_lo[0][tid] = l.x; s_lo[1][tid] = l.y; s_lo[2][tid] = l.z;
        s_hi[0][tid] = h.x; s_hi[1][tid] = h.y; s_hi[2][tid] = h.z;
        s_cen[0][tid] = c.x; s_cen[1][tid] = c.y; s_cen[2][tid] = c.z;
        s_ord[tid] = tid;
    }
    if (tid == 0) {
        s_sp = 0; s_nw = 0; s_take = 0;
        if (G.count > kWaveJob) s_job[s_sp++] = make_int4(0, G.count, G.id, G.depth);
        else s_wjob[s_nw++] = make_int4(0, G.count, G.id, G.depth);
        s_next = G.id + 1; s_maxd = G.depth;
    }
    __syncthreads();
    while (true) {                             // the workgroup: jobs of more than kWaveJob triangles
        if (s_sp == 0) break;
        const int4 J = s_job[s_sp - 1];
        const int f = J.x, c = J.y;
        int P = 1;
        while (P < c) P <<= 1;
        __syncthreads();
        if (tid == 0) { s_sp--; s_best = 1e300; s_bax = 0; s_bs = c / 2; }
        for (int a = 0; a < 3; ++a) {
            // bitonic sort of the job's slots by (centroid a, triangle id); padding slots (-1) last
            if (tid < P) s_key[tid] = tid < c ? s_ord[f + tid] : -1;
            __syncthreads();
            for (int k = 2; k <= P; k <<= 1)
                for (int j = k >> 1; j > 0; j >>= 1) {
                    if (tid < P) {
                        const int q = tid ^ j;
                        if (q > tid) {
                            const int x = s_key[tid], y = s_key[q];
                            // x after y?  (padding after everything)
                            bool gt;
                            if (x < 0) gt = y >= 0;
                            else if (y < 0) gt = false;
                            else {
                                const float cx = s_cen[a][x], cy = s_cen[a][y];
                                gt = cy < cx || (cy == cx && s_tri[y] < s_tri[x]);
                            }
                            const bool up = (tid & k) == 0;
                            if (gt == up) { s_key[tid] = y; s_key[q] = x; }
                        }
                    }
                    __syncthreads();
                }
            if (tid < c) {
                const int e = s_key[tid];
                s_srt[a][f + tid] = e;
                for (int k = 0; k < 3; ++k) {
                    s_plo[k][tid] = s_lo[k][e]; s_phi[k][tid] = s_hi[k][e];
                    s_qlo[k][tid] = s_lo[k][e]; s_qhi[k][tid] = s_hi[k][e];
                }
            }
            __syncthreads();
            // inclusive prefix (p: elements 0..i) and suffix (q: elements i..c-1) box scans
            for (int o = 1; o < c; o <<= 1) {
                float pl[3], ph[3], ql[3], qh[3];
                const bool dp = tid < c && tid >= o, dq = tid < c && tid + o < c;
                for (int k = 0; k < 3; ++k) {
                    if (dp) { pl[k] = w_min(s_plo[k][tid - o], s_plo[k][tid]); ph[k] = w_max(s_phi[k][tid - o], s_phi[k][tid]); }
                    if (dq) { ql[k] = w_min(s_qlo[k][tid], s_qlo[k][tid + o]); qh[k] = w_max(s_qhi[k][tid], s_qhi[k][tid + o]); }
                }
                __syncthreads();
                for (int k = 0; k < 3; ++k) {
                    if (dp) { s_plo[k][tid] = pl[k]; s_phi[k][tid] = ph[k]; }
                    if (dq) { s_qlo[k][tid] = ql[k]; s_qhi[k][tid] = qh[k]; }
                }
                __syncthreads();
            }
            // split at i (left = sorted 0..i-1): cost = A(l) i + A(r) (c - i), boxes grown from the empty box
            double cost = 1e300;
            const int i = tid + 1;
            if (i < c) {
                float ll[3], lh[3], rl[3], rh[3];
                for (int k = 0; k < 3; ++k) {
                    ll[k] = w_min(kEmpty, s_plo[k][i - 1]); lh[k] = w_max(-kEmpty, s_phi[k][i - 1]);
                    rl[k] = w_min(kEmpty, s_qlo[k][i]); rh[k] = w_max(-kEmpty, s_qhi[k][i]);
                }
                cost = half_area_d(ll, lh) * i + half_area_d(rl, rh) * (c - i);
            }
            // first minimum in position order (strict <, as the host's loop)
            int bi = i;
            for (int o = 32; o > 0; o >>= 1) {
                const double oc = __shfl_xor(cost, o);
                const int ob = __shfl_xor(bi, o);
                if (oc < cost || (oc == cost && ob < bi)) { cost = oc; bi = ob; }
            }
            if ((tid & 63) == 0) { s_bc[tid >> 6] = cost; s_bi[tid >> 6] = bi; }
            __syncthreads();
            if (tid == 0) {
                double bc = s_bc[0]; int b = s_bi[0];
                for (int w = 1; w < kB / 64; ++w)
                    if (s_bc[w] < bc || (s_bc[w] == bc && s_bi[w] < b)) { bc = s_bc[w]; b = s_bi[w]; }
                if (bc < s_best) { s_best = bc; s_bax = a; s_bs = b; }   // earlier axes win ties
            }
            __syncthreads();
        }
        const int bax = s_bax, bs = s_bs;
        if (tid < c) s_ord[f + tid] = s_srt[bax][f + tid];
        __syncthreads();
        if (tid == 0) {
            // node box = the union over the job (prefix of its last element), grown from the empty box
            float l[3], h[3];
            for (int k = 0; k < 3; ++k) { l[k] = w_min(kEmpty, s_plo[k][c - 1]); h[k] = w_max(-kEmpty, s_phi[k][c - 1]); }
            int cid[2];
            const int cf[2] = {f, f + bs}, cc[2] = {bs, c - bs};
            for (int q = 0; q < 2; ++q) {
                if (cc[q] == 1) { cid[q] = s_tri[s_ord[cf[q]]]; continue; }
                cid[q] = s_next++;
                if (cc[q] > kWaveJob) s_job[s_sp++] = make_int4(cf[q], cc[q], cid[q], J.w + 1);
                else s_wjob[s_nw++] = make_int4(cf[q], cc[q], cid[q], J.w + 1);
                s_maxd = max(s_maxd, J.w + 1);
            }
            nlo[J.z] = make_float4(l[0], l[1], l[2], __int_as_float(cid[0]));
            nhi[J.z] = make_float4(h[0], h[1], h[2], __int_as_float(cid[1]));
            depth[J.z - n] = J.w;
        }
        __syncthreads();
    }
    // the waves: subtrees of at most kWaveJob triangles, one list entry at a time
    const int lane = tid & 63;
    for (;;) {
        int j = 0;
        if (lane == 0) j = atomicAdd(&s_take, 1);
        j = __shfl(j, 0);
        if (j >= s_nw) break;
        wave_subtree(s_wjob[j], lane, s_tri, s_lo, s_hi, s_cen, s_ord, &s_next, &s_maxd, n, nlo, nhi, depth);
    }
    __syncthreads();
    if (tid == 0) atomicMax(max_depth, s_maxd);
}

// ---------------------------------------------------------------- 4 SAH-optimal collapse tables
// The internal nodes bucketed by depth.  A workgroup first counts its nodes per depth in LDS and makes ONE global
// atomic per depth it holds (the same-address global atomics of one thread per node serialised: 1.22 ms per
// launch at C3's 248 k nodes).  Order inside a depth bucket is free: k_dp_level's nodes of one
// depth are independent.  nd <= kDepthLds (the host falls back to the per-node atomics above it).
constexpr int kDepthLds = 1024;
__global__ void k_depth_count(const int* __restrict__ depth, int m, int nd, int* cnt) {
    __shared__ int h[kDepthLds];
    for (int d = threadIdx.x; d < nd; d += blockDim.x) h[d] = 0;
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) atomicAdd(&h[depth[i]], 1);
    __syncthreads();
    for (int d = threadIdx.x; d < nd; d += blockDim.x)
        if (h[d]) atomicAdd(&cnt[d], h[d]);
}
__global__ void k_depth_fill(const int* __restrict__ depth, int m, int nd, int* fill, int* order) {
    __shared__ int h[kDepthLds], base[kDepthLds];
    for (int d = threadIdx.x; d < nd; d += blockDim.x) h[d] = 0;
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int dep = i < m ? depth[i] : 0;
    const int rank = i < m ? atomicAdd(&h[dep], 1) : 0;
    __syncthreads();
    for (int d = threadIdx.x; d < nd; d += blockDim.x)
        if (h[d]) base[d] = atomicAdd(&fill[d], h[d]);
    __syncthreads();
    if (i < m) order[base[dep] + rank] = i;
}
__global__ void k_depth_count_flat(const int* __restrict__ depth, int m, int* cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) atomicAdd(&cnt[depth[i]], 1);
}
__global__ void k_depth_fill_flat(const int* __restrict__ depth, int m, int* fill, int* order) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) order[atomicAdd(&fill[depth[i]], 1)] = i;
}
// S(x, k, g) for the internal nodes of one depth level (SahCollapse::plan's loops, same float operations):
// tables per internal node x - n, [g + 1][k - 1].  16 lanes per node, lane g + 1 computes row g: its D(k) from
// the children's rows g (two coalesced 32-B rows), the node term N from D(8) of row g - 1 (the lane below,
// by shuffle).  One lane per node walking all ten rows serially took 25-130 us per level launch (23 launches
// at C3), latency on the children's tables.
constexpr int kDpLanes = 16;
// (+ ntri: the node's triangle count, for build_wide_host's slot order; children are a deeper level, done already)
__global__ void k_dp_level(const int* __restrict__ order, int b, int e, int n, const float4* __restrict__ nlo,
                           const float4* __restrict__ nhi, float* S, uint8_t* open, uint8_t* split, int* ntri) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int q = b + t / kDpLanes, gi = t % kDpLanes, g = gi - 1;
    const bool node = q < e, act = node && gi < kG;
    const float inf = 3.0e38f;
    float D[8];
    D[0] = 0.0f;
    int xi = 0;
    float ax = 0.0f;
    if (act) {
        xi = order[q];
        const int x = n + xi;
        const float4 xl = nlo[x], xh = nhi[x];
        const int l = __float_as_int(xl.w), r = __float_as_int(xh.w);
        ax = area_f(xl, xh);
        if (gi == 0) ntri[xi] = (l < n ? 1 : ntri[l - n]) + (r < n ? 1 : ntri[r - n]);
        float rl[8], rr[8];
        if (l < n) { const float al = area_f(nlo[l], nhi[l]) * kCtri; for (int k = 0; k < 8; ++k) rl[k] = al; }
        else {
            const float4* p = (const float4*)(S + (size_t)(l - n) * kG * 8 + gi * 8);
            const float4 u = p[0], v = p[1];
            rl[0] = u.x; rl[1] = u.y; rl[2] = u.z; rl[3] = u.w; rl[4] = v.x; rl[5] = v.y; rl[6] = v.z; rl[7] = v.w;
        }
        if (r < n) { const float ar = area_f(nlo[r], nhi[r]) * kCtri; for (int k = 0; k < 8; ++k) rr[k] = ar; }
        else {
            const float4* p = (const float4*)(S + (size_t)(r - n) * kG * 8 + gi * 8);
            const float4 u = p[0], v = p[1];
            rr[0] = u.x; rr[1] = u.y; rr[2] = u.z; rr[3] = u.w; rr[4] = v.x; rr[5] = v.y; rr[6] = v.z; rr[7] = v.w;
        }
        uint8_t* Px = split + (size_t)xi * kG * 8 + gi * 8;
#pragma unroll
        for (int k = 2; k <= 8; ++k) {
            float best = inf;
            int ba = 1;
#pragma unroll
            for (int a = 1; a < k; ++a) {
                const float v = rl[a - 1] + rr[k - a - 1];
                if (v < best) { best = v; ba = a; }
            }
            D[k - 1] = best;
            Px[k - 1] = (uint8_t)ba;
        }
        Px[0] = 0;
    } else {
#pragma unroll
        for (int k = 1; k < 8; ++k) D[k] = 0.0f;
    }
    const float d8 = __shfl_up(D[7], 1, kDpLanes);     // D(8) of row g - 1 (Dprev; zeros before row -1)
    if (!act) return;
    float Nx = inf;
    if (g >= 0) Nx = d8 < inf ? ax * kCnode + d8 : inf;
    float* Sx = S + (size_t)xi * kG * 8 + gi * 8;
    uint8_t* Ox = open + (size_t)xi * kG * 8 + gi * 8;
    float prev = Nx;
    Sx[0] = Nx;
    Ox[0] = 0;
#pragma unroll
    for (int k = 2; k <= 8; ++k) {
        const bool o = D[k - 1] < prev;
        prev = o ? D[k - 1] : prev;
        Sx[k - 1] = prev;
        Ox[k - 1] = o ? 1 : 0;
    }
}

// ---------------------------------------------------------------- 5 wide nodes, breadth first
struct WideQ { int node, budget; };
// SahCollapse::kids / expand: the slots of wide node c under height budget g, left-first
__device__ int wide_kids(int c, int g, int n, const float4* __restrict__ nlo, const float4* __restrict__ nhi,
                         const uint8_t* __restrict__ open, const uint8_t* __restrict__ split, int* out) {
    if (c < n) { out[0] = c; return 1; }
    int3 st[16];
    int sp = 0, m = 0;
    const int gg = g - 1;
    const int a = split[(size_t)(c - n) * kG * 8 + (gg + 1) * 8 + 7];
    st[sp++] = make_int3(__float_as_int(nhi[c].w), 8 - a, 0);
    st[sp++] = make_int3(__float_as_int(nlo[c].w), a, 0);
    while (sp > 0 && m < 8) {
        int3 j = st[--sp];
        int x = j.x, k = j.y;
        while (x >= n && k > 1 && !open[(size_t)(x - n) * kG * 8 + (gg + 1) * 8 + (k - 1)]) --k;
        if (x < n || k == 1) { out[m++] = x; continue; }
        const int s = split[(size_t)(x - n) * kG * 8 + (gg + 1) * 8 + (k - 1)];
        if (sp + 2 > 16) return -1;
        st[sp++] = make_int3(__float_as_int(nhi[x].w), k - s, 0);
        st[sp++] = make_int3(__float_as_int(nlo[x].w), s, 0);
    }
    return sp == 0 ? m : -1;
}
__global__ void k_wide_kids(const WideQ* __restrict__ wq, int q0, int q1, int n, const float4* __restrict__ nlo,
                            const float4* __restrict__ nhi, const uint8_t* __restrict__ open,
                            const uint8_t* __restrict__ split, const int* __restrict__ ntri, int* kids, int* n_int,
                            int* n_leaf, int* bad) {
    const int i = q0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= q1) return;
    const WideQ Q = wq[i];
    int k[8];
    const int m = wide_kids(Q.node, Q.budget, n, nlo, nhi, open, split, k);
    if (m <= 0) { atomicOr(bad, 2); n_int[i - q0] = 0; n_leaf[i - q0] = 0; return; }
    // interior slots first, each group in expansion order (build_wide_host's stable partition); the interior slots
    // then by triangle count, most first, ties in expansion order (build_wide_host's insertion sort)
    int o = 0, ni = 0;
    int ki[8], kc[8];
    for (int j = 0; j < m; ++j)
        if (k[j] >= n) {
            int c = ntri[k[j] - n], p = ni++;
            for (; p > 0 && c > kc[p - 1]; --p) { ki[p] = ki[p - 1]; kc[p] = kc[p - 1]; }
            ki[p] = k[j]; kc[p] = c;
        }
    for (int j = 0; j < ni; ++j) kids[8 * (size_t)i + o++] = ki[j];
    for (int j = 0; j < m; ++j) if (k[j] < n) kids[8 * (size_t)i + o++] = k[j];
    for (int j = m; j < 8; ++j) kids[8 * (size_t)i + j] = -1;
    n_int[i - q0] = ni;
    n_leaf[i - q0] = m - ni;
}
__global__ void k_wide_emit(WideQ* wq, int q0, int q1, int tri_off, const int* __restrict__ kids,
                            const int* __restrict__ n_int, const int* __restrict__ n_leaf, const int* __restrict__ s_int,
                            const int* __restrict__ s_leaf, const float4* __restrict__ nlo, const float4* __restrict__ nhi,
                            uint4* nodes, float4* box, int* prims, int* bad) {
    const int i = q0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= q1) return;
    const int ni = n_int[i - q0], nv = ni + n_leaf[i - q0];
    if (nv == 0) return;
    const uint32_t cb = (uint32_t)(q1 + s_int[i - q0]), tb = (uint32_t)(tri_off + s_leaf[i - q0]);
    const int g = wq[i].budget;
    WBox kb[8];
    for (int j = 0; j < nv; ++j) {
        const int x = kids[8 * (size_t)i + j];
        const float4 l = nlo[x], h = nhi[x];
        kb[j] = WBox{{l.x, l.y, l.z}, {h.x, h.y, h.z}};
        if (j < ni) wq[cb + j] = WideQ{x, g - 1};
        else prims[tb + (j - ni)] = __float_as_int(h.w);
    }
    uint32_t w[20];
    WBox u;
    if (!wide_encode(kb, nv, ni, cb, tb, w, &u)) { atomicOr(bad, 4); return; }
    for (int k = 0; k < 5; ++k) nodes[5 * (size_t)i + k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
    box[2 * (size_t)i] = make_float4(u.lo[0], u.lo[1], u.lo[2], 0.0f);
    box[2 * (size_t)i + 1] = make_float4(u.hi[0], u.hi[1], u.hi[2], 0.0f);
}

// ---------------------------------------------------------------- 6 wide-leaf triangles
// a wide level's totals for the host: next-level nodes (scan + last count), leaf triangles, the failure flag
__global__ void k_level_totals(const int* si, const int* ni, const int* sl, const int* nl, int cnt, const int* bad,
                               int* out) {
    if (threadIdx.x == 0) { out[0] = si[cnt - 1]; out[1] = ni[cnt - 1]; out[2] = sl[cnt - 1]; out[3] = nl[cnt - 1]; out[4] = *bad; }
}
__global__ void k_wide_gather(const float* __restrict__ pos, const int* __restrict__ prims, uint32_t m, float4* tris) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const int prim = prims[k];
    const float* p = pos + 9 * (size_t)prim;
    const float v0x = p[0], v0y = p[1], v0z = p[2];
    tris[3 * k] = make_float4(v0x, v0y, v0z, __int_as_float(prim));
    tris[3 * k + 1] = make_float4(p[3] - v0x, p[4] - v0y, p[5] - v0z, 0.0f);
    tris[3 * k + 2] = make_float4(p[6] - v0x, p[7] - v0y, p[8] - v0z, 0.0f);
}

// device scratch freed on every exit
// stream-ordered scratch from the device pool (rs_bvh_build.hip preload_code_objects keeps it cached)
struct Scratch {
    hipStream_t st;
    std::vector<void*> p;
    explicit Scratch(hipStream_t s) : st(s) {}
    template <class T> bool get(T** out, size_t count) {
        *out = nullptr;
        if (pool_malloc((void**)out, std::max<size_t>(1, count) * sizeof(T), st) != hipSuccess) return false;
        p.push_back((void*)*out);
        return true;
    }
    ~Scratch() { for (void* q : p) (void)hipFreeAsync(q, st); }
};

}  // namespace wb

#define WB_CHECK(x, what)                                                                     \
    do {                                                                                      \
        if (!(x)) { err = std::string("wide BVH: ") + (what); return -1; }                    \
    } while (0)
#define WB_HIP(x) WB_CHECK((x) == hipSuccess, #x)

// Builds the 8-wide tree of the n triangles at d_pos (device, 9 floats each) on `st`.  Returns 0 with *w filled
// (device allocations owned by the caller), 1 when no tree applies (non-finite positions, or no plan within the
// walk's depth: the walks then take the skip pointers; *w stays empty), -1 on a HIP error (err set).
// the code object of this file loaded now (HIP loads a file's kernels at its first launch or query; see
// rs::preload_code_objects)
void preload_wide_build() {
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, (const void*)wb::k_small);
}

int build_wide_gpu(const float* d_pos, int n, hipStream_t st, WideBvh* w, std::string& err) {
    using namespace wb;
    *w = WideBvh{};
    if (n <= 0) { w->status = RS_WIDE_EMPTY; return 1; }
    if (n >= (1 << 24)) { w->status = RS_WIDE_TOO_MANY; return 1; }   // the node word's 24-bit child index
    Scratch X(st);
    const int total = 2 * n - 1, m = n - 1;          // binary nodes, internal nodes
    float4 *tlo, *thi, *tcen, *nlo, *nhi;
    int *idx, *tmp, *depth, *bad, *dmax;
    WB_CHECK(X.get(&tlo, n) && X.get(&thi, n) && X.get(&tcen, n) && X.get(&nlo, total) && X.get(&nhi, total) &&
             X.get(&idx, n) && X.get(&tmp, n) && X.get(&depth, std::max(1, m)) && X.get(&bad, 1) && X.get(&dmax, 1),
             "scratch allocation failed");
    WB_HIP(hipMemsetAsync(bad, 0, sizeof(int), st));
    WB_HIP(hipMemsetAsync(dmax, 0, sizeof(int), st));
    k_tri_prep<<<(n + kB - 1) / kB, kB, 0, st>>>(d_pos, n, tlo, thi, tcen, idx, nlo, nhi, bad);
    WB_HIP(hipGetLastError());
    int h_bad = 0;
    WB_HIP(hipMemcpyAsync(&h_bad, bad, sizeof(int), hipMemcpyDeviceToHost, st));
    WB_HIP(hipStreamSynchronize(st));
    if (h_bad) { w->status = RS_WIDE_NONFINITE; return 1; }   // non-finite geometry: no wide tree
    int root = 0, max_depth = 0;
    // ---- source tree
    if (n >= 2) {
        root = n;
        std::vector<Seg> cur;
        std::vector<SmallSeg> small;
        int next = n + 1;
        if (n > kSmall) cur.push_back({0, n, n, 0});
        else { small.push_back({0, n, n, 0}); next = n + (n - 1); }
        Seg* d_seg = nullptr; int2* d_segch = nullptr; Chunk* d_ch = nullptr; SegAcc* d_acc = nullptr; SegDec* d_dec = nullptr;
        int* d_cl = nullptr; int2* d_coff = nullptr; int2* d_kids = nullptr; uint8_t* d_side = nullptr;
        const size_t max_seg = (size_t)n / kSmall + 1, max_ch = (size_t)n / kChunk + max_seg + 1;
        WB_CHECK(X.get(&d_seg, max_seg) && X.get(&d_segch, max_seg) && X.get(&d_ch, max_ch) && X.get(&d_acc, max_seg) &&
                 X.get(&d_dec, max_seg) && X.get(&d_cl, max_ch) && X.get(&d_coff, max_ch) && X.get(&d_kids, max_seg) &&
                 X.get(&d_side, n), "scratch allocation failed");
        std::vector<Chunk> chunks;
        std::vector<int2> segch, kids;
        std::vector<SegDec> dec;
        while (!cur.empty()) {
            const int ns = (int)cur.size();
            chunks.clear(); segch.clear();
            for (int s = 0; s < ns; ++s) {
                const int c0 = (int)chunks.size();
                for (int b = cur[s].first; b < cur[s].first + cur[s].count; b += kChunk)
                    chunks.push_back({s, b, std::min(cur[s].first + cur[s].count, b + kChunk), 0});
                segch.push_back(make_int2(c0, (int)chunks.size()));
            }
            const int nc = (int)chunks.size();
            WB_HIP(hipMemcpyAsync(d_seg, cur.data(), ns * sizeof(Seg), hipMemcpyHostToDevice, st));
            WB_HIP(hipMemcpyAsync(d_segch, segch.data(), ns * sizeof(int2), hipMemcpyHostToDevice, st));
            WB_HIP(hipMemcpyAsync(d_ch, chunks.data(), nc * sizeof(Chunk), hipMemcpyHostToDevice, st));
            k_acc_init<<<ns, kB, 0, st>>>(d_acc, ns);
            k_seg_bounds<<<nc, kB, 0, st>>>(d_ch, idx, tlo, thi, tcen, d_acc);
            k_seg_bins<<<nc, kB, 0, st>>>(d_ch, idx, tlo, thi, tcen, d_acc);
            k_seg_choose<<<ns, kChooseThreads, 0, st>>>(d_seg, ns, d_acc, d_dec, nlo, nhi);
            k_seg_side<<<nc, kB, 0, st>>>(d_ch, idx, tcen, d_dec, d_side, d_cl);
            k_seg_scan<<<(ns + 63) / 64, 64, 0, st>>>(d_seg, d_segch, ns, d_ch, d_cl, d_coff, d_dec);
            k_seg_scatter<<<nc, kB, 0, st>>>(d_ch, d_seg, idx, d_side, d_coff, d_dec, tmp);
            k_seg_copy<<<nc, kB, 0, st>>>(d_ch, tmp, idx);
            WB_HIP(hipGetLastError());
            dec.resize(ns);
            WB_HIP(hipMemcpyAsync(dec.data(), d_dec, ns * sizeof(SegDec), hipMemcpyDeviceToHost, st));
            WB_HIP(hipStreamSynchronize(st));
            std::vector<Seg> nxt;
            kids.assign(ns, make_int2(0, 0));
            for (int s = 0; s < ns; ++s) {
                const Seg& S = cur[s];
                const int L = dec[s].left;
                WB_CHECK(L > 0 && L < S.count, "empty side in a binned split");
                const int cf[2] = {S.first, S.first + L}, cc[2] = {L, S.count - L};
                int id[2];
                for (int q = 0; q < 2; ++q) {
                    if (cc[q] == 1) { id[q] = -(cf[q] + 1); continue; }
                    if (cc[q] <= kSmall) { id[q] = next; small.push_back({cf[q], cc[q], next, S.depth + 1}); next += cc[q] - 1; }
                    else { id[q] = next++; nxt.push_back({cf[q], cc[q], id[q], S.depth + 1}); }
                }
                kids[s] = make_int2(id[0], id[1]);
                max_depth = std::max(max_depth, S.depth);
            }
            WB_HIP(hipMemcpyAsync(d_kids, kids.data(), ns * sizeof(int2), hipMemcpyHostToDevice, st));
            k_seg_link<<<(ns + 63) / 64, 64, 0, st>>>(d_seg, ns, d_kids, idx, n, nlo, nhi, depth);
            WB_HIP(hipGetLastError());
            WB_HIP(hipStreamSynchronize(st));     // the host vectors above are reused next level
            cur.swap(nxt);
        }
        WB_CHECK(next == total, "node count mismatch");
        if (!small.empty()) {
            SmallSeg* d_small = nullptr;
            WB_CHECK(X.get(&d_small, small.size()), "scratch allocation failed");
            WB_HIP(hipMemcpyAsync(d_small, small.data(), small.size() * sizeof(SmallSeg), hipMemcpyHostToDevice, st));
            k_small<<<(unsigned)small.size(), kB, 0, st>>>(d_small, idx, tlo, thi, tcen, n, nlo, nhi, depth, dmax);
            WB_HIP(hipGetLastError());
            int hd = 0;
            WB_HIP(hipMemcpyAsync(&hd, dmax, sizeof(int), hipMemcpyDeviceToHost, st));
            WB_HIP(hipStreamSynchronize(st));
            max_depth = std::max(max_depth, hd);
        }
    }
    // ---- SAH-optimal collapse tables, deepest binary level first
    float* S = nullptr;
    uint8_t *open = nullptr, *split = nullptr;
    WB_CHECK(X.get(&S, (size_t)std::max(1, m) * kG * 8) && X.get(&open, (size_t)std::max(1, m) * kG * 8) &&
             X.get(&split, (size_t)std::max(1, m) * kG * 8), "collapse tables: allocation failed");
    int* ntri = nullptr;                             // triangles below each internal node (k_dp_level, k_wide_kids)
    WB_CHECK(X.get(&ntri, std::max(1, m)), "scratch allocation failed");
    if (m > 0) {
        int *cnt = nullptr, *order = nullptr;
        const int nd = max_depth + 1;
        WB_CHECK(X.get(&cnt, nd) && X.get(&order, m), "scratch allocation failed");
        WB_HIP(hipMemsetAsync(cnt, 0, nd * sizeof(int), st));
        if (nd <= kDepthLds) k_depth_count<<<(m + kB - 1) / kB, kB, 0, st>>>(depth, m, nd, cnt);
        else k_depth_count_flat<<<(m + kB - 1) / kB, kB, 0, st>>>(depth, m, cnt);
        std::vector<int> hc(nd), off(nd + 1, 0);
        WB_HIP(hipMemcpyAsync(hc.data(), cnt, nd * sizeof(int), hipMemcpyDeviceToHost, st));
        WB_HIP(hipStreamSynchronize(st));
        for (int d = 0; d < nd; ++d) off[d + 1] = off[d] + hc[d];
        WB_CHECK(off[nd] == m, "depth buckets");
        WB_HIP(hipMemcpyAsync(cnt, off.data(), nd * sizeof(int), hipMemcpyHostToDevice, st));
        if (nd <= kDepthLds) k_depth_fill<<<(m + kB - 1) / kB, kB, 0, st>>>(depth, m, nd, cnt, order);
        else k_depth_fill_flat<<<(m + kB - 1) / kB, kB, 0, st>>>(depth, m, cnt, order);
        for (int d = nd - 1; d >= 0; --d) {
            const int b = off[d], e = off[d + 1];
            if (e > b) k_dp_level<<<(unsigned)(((size_t)(e - b) * kDpLanes + 127) / 128), 128, 0, st>>>(order, b, e, n, nlo, nhi, S, open, split, ntri);
        }
        WB_HIP(hipGetLastError());
        float s_root = 0.0f;
        WB_HIP(hipMemcpyAsync(&s_root, S + (size_t)(root - n) * kG * 8 + (kGmax + 1) * 8, sizeof(float),
                              hipMemcpyDeviceToHost, st));
        WB_HIP(hipStreamSynchronize(st));
        if (!(s_root < 3.0e38f)) { w->status = RS_WIDE_TOO_DEEP; return 1; }   // no plan within the walk's depth
    }
    // ---- wide nodes, breadth first
    WideQ* wq = nullptr;
    int *kidv = nullptr, *ni = nullptr, *nl = nullptr, *si = nullptr, *sl = nullptr, *prims = nullptr;
    const int maxw = std::max(1, m);                 // every wide node is an internal binary node (or the lone triangle)
    int* tot5 = nullptr;
    WB_CHECK(X.get(&wq, maxw) && X.get(&kidv, (size_t)8 * maxw) && X.get(&ni, maxw) && X.get(&nl, maxw) &&
             X.get(&si, maxw) && X.get(&sl, maxw) && X.get(&prims, n) && X.get(&tot5, 5), "scratch allocation failed");
    size_t scan_bytes = 0;
    WB_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, ni, si, maxw, st));
    void* scan_tmp = nullptr;
    WB_CHECK(X.get((uint8_t**)&scan_tmp, scan_bytes), "scratch allocation failed");
    uint4* nodes = nullptr;
    float4* box = nullptr;
    // (allocated at the exact size after the levels are known: staged in scratch first)
    uint4* nodes_s = nullptr;
    float4* box_s = nullptr;
    WB_CHECK(X.get(&nodes_s, (size_t)5 * maxw) && X.get(&box_s, (size_t)2 * maxw), "scratch allocation failed");
    const WideQ r0{root, kGmax};
    WB_HIP(hipMemcpyAsync(wq, &r0, sizeof r0, hipMemcpyHostToDevice, st));
    int q0 = 0, q1 = 1, tri_off = 0, level = 0;    // level `level` = wide nodes [q0, q1)
    int lvl[kWideLevels + 1] = {};
    while (q0 < q1) {
        WB_CHECK(level < kWideLevels, "deeper than the walk's stack");
        const int cnt = q1 - q0;
        k_wide_kids<<<(cnt + kB - 1) / kB, kB, 0, st>>>(wq, q0, q1, n, nlo, nhi, open, split, ntri, kidv, ni, nl, bad);
        WB_HIP(hipGetLastError());
        WB_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, ni, si, cnt, st));
        WB_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, nl, sl, cnt, st));
        k_wide_emit<<<(cnt + kB - 1) / kB, kB, 0, st>>>(wq, q0, q1, tri_off, kidv, ni, nl, si, sl, nlo, nhi, nodes_s, box_s,
                                                          prims, bad);
        WB_HIP(hipGetLastError());
        int h[5];
        k_level_totals<<<1, 64, 0, st>>>(si, ni, sl, nl, cnt, bad, tot5);   // one read-back per level
        WB_HIP(hipMemcpyAsync(h, tot5, sizeof h, hipMemcpyDeviceToHost, st));
        WB_HIP(hipStreamSynchronize(st));
        if (h[4]) { err = h[4] & 4 ? "wide BVH: no conservative quantisation" : "wide BVH: slot expansion failed"; return -1; }
        const int nq = h[0] + h[1];
        tri_off += h[2] + h[3];
        lvl[level + 1] = q1;
        ++level;
        q0 = q1;
        q1 += nq;
        WB_CHECK(q1 <= maxw && tri_off <= n, "wide node overflow");
    }
    WB_CHECK(tri_off == n, "every triangle in one leaf slot");
    const int nw = q1;
    float4* tris = nullptr;
    const bool ok = hipMalloc(&nodes, (size_t)5 * nw * sizeof(uint4)) == hipSuccess &&
                    hipMalloc(&box, (size_t)2 * nw * sizeof(float4)) == hipSuccess &&
                    hipMalloc(&tris, (size_t)3 * n * sizeof(float4)) == hipSuccess &&
                    hipMemcpyAsync(nodes, nodes_s, (size_t)5 * nw * sizeof(uint4), hipMemcpyDeviceToDevice, st) == hipSuccess &&
                    hipMemcpyAsync(box, box_s, (size_t)2 * nw * sizeof(float4), hipMemcpyDeviceToDevice, st) == hipSuccess &&
                    (k_wide_gather<<<(n + kB - 1) / kB, kB, 0, st>>>(d_pos, prims, (uint32_t)n, tris), hipGetLastError() == hipSuccess) &&
                    hipStreamSynchronize(st) == hipSuccess;
    if (!ok) {
        if (nodes) hipFree(nodes);
        if (box) hipFree(box);
        if (tris) hipFree(tris);
        err = "wide BVH: final allocation / copy failed";
        return -1;
    }
    w->nodes = nodes; w->box = box; w->tris = tris;
    w->n_nodes = (uint32_t)nw;
    w->n_tris = (uint32_t)n;
    w->depth = level - 1;                            // lvl[level] = nw
    for (int i = 0; i <= kWideLevels; ++i) w->lvl[i] = i <= level ? lvl[i] : nw;
    return 0;
}

}  // namespace rs
