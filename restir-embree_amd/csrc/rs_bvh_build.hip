// rs_bvh_build.hip -- wavefront LBVH build on the GPU; replaces Embree's rtcCommitScene
// (pg/Scene.cpp:15).  Every stage is a data-parallel kernel; no inter-workgroup hand-off inside a
// launch (kernel boundaries provide visibility across the 8 non-coherent XCD L2s), so the build is
// placement-independent and deterministic (identical trees on every rank):
//   1 k_prim_bounds   per-triangle AABB + centroid; centroid bounds by block reduce + ordered-int
//                     atomics (min/max are order independent)
//   2 k_morton        64-bit key = morton30(centroid) << 32 | triangle index (unique keys)
//   3 radix sort      hipcub::DeviceRadixSort::SortKeys on 62 bits
//   4 k_karras        Karras 2012 hierarchy: internal node i's range, split, children, parents
//   5 k_depth         depth of every node (walk to the root)
//   6 k_refit_level   bottom-up AABB union + collapsed subtree sizes, one launch per depth level
//   7 k_emit          collapse subtrees of <= kLeafMax triangles into leaves, preorder index by
//                     walking up (idx = idx(parent) + 1 + [right child] * kept(left sibling)),
//                     write the 32-B skip-pointer nodes
//   8 k_leaf_tris     triangles in leaf order as (v0, prim), (e1), (e2)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <float.h>
#include <string>
#include <vector>
#include <cstdlib>
#include <cmath>
#include <utility>
#include <cstring>
#include <algorithm>
#include <mutex>
#include "rs_refit.h"
#include "rs_wide.h"
#include "../../include/restir_c.h"

namespace rs {

constexpr int kLeafMax = 4;

__device__ __forceinline__ int f2o(float f) {   // order-preserving float -> int
    int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

struct BuildNode {        // internal nodes [0, n-1), leaves [n-1, 2n-1)
    float lo[3], hi[3];
    int parent, left, right;
    int first, last;
    int kept;             // nodes this subtree contributes to the output (1 when collapsed)
    int depth;
};

__global__ void k_prim_bounds(const float* __restrict__ pos, uint32_t n, float4* lo, float4* hi, int* cb) {
    __shared__ int s[6][256];
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    int c[6] = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MIN, INT32_MIN, INT32_MIN};
    if (i < n) {
        const float* p = pos + 9 * (size_t)i;
        float l[3], h[3];
        bool fin = true;
        for (int a = 0; a < 3; ++a) {
            l[a] = fminf(fminf(p[a], p[3 + a]), p[6 + a]);
            h[a] = fmaxf(fmaxf(p[a], p[3 + a]), p[6 + a]);
            fin = fin && isfinite(l[a]) && isfinite(h[a]);
        }
        // a triangle with an infinite (or all-NaN) coordinate can never be hit (the triangle test's arithmetic
        // turns NaN and fails); it enters the tree as a point box at the origin so that the centroid bounds,
        // the Morton codes and PLOC's merge distances stay finite (Embree drops such primitives)
        if (!fin)
            for (int a = 0; a < 3; ++a) l[a] = h[a] = 0.0f;
        lo[i] = make_float4(l[0], l[1], l[2], 0.0f);
        hi[i] = make_float4(h[0], h[1], h[2], 0.0f);
        for (int a = 0; a < 3; ++a) {
            float cen = 0.5f * (l[a] + h[a]);
            c[a] = f2o(cen); c[3 + a] = f2o(cen);
        }
    }
    for (int a = 0; a < 6; ++a) s[a][threadIdx.x] = c[a];
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < (unsigned)w) {
            for (int a = 0; a < 3; ++a) s[a][threadIdx.x] = min(s[a][threadIdx.x], s[a][threadIdx.x + w]);
            for (int a = 3; a < 6; ++a) s[a][threadIdx.x] = max(s[a][threadIdx.x], s[a][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        for (int a = 0; a < 3; ++a) atomicMin(&cb[a], s[a][0]);
        for (int a = 3; a < 6; ++a) atomicMax(&cb[a], s[a][0]);
    }
}

__device__ __forceinline__ uint32_t expand10(uint32_t v) {
    v &= 0x3ffu;
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void k_morton(const float4* lo, const float4* hi, uint32_t n, const int* cb, uint64_t* keys) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float l[3] = {lo[i].x, lo[i].y, lo[i].z}, h[3] = {hi[i].x, hi[i].y, hi[i].z};
    uint32_t q[3];
    for (int a = 0; a < 3; ++a) {
        float mn = o2f(cb[a]), mx = o2f(cb[3 + a]);
        float cen = 0.5f * (l[a] + h[a]);
        float ext = mx - mn;
        float t = ext > 0.0f ? (cen - mn) / ext : 0.0f;
        int v = (int)(t * 1024.0f);
        q[a] = (uint32_t)(v < 0 ? 0 : (v > 1023 ? 1023 : v));
    }
    uint32_t m = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
    keys[i] = ((uint64_t)m << 32) | i;
}

__device__ __forceinline__ int delta(const uint64_t* k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    return __clzll(k[i] ^ k[j]);
}

__global__ void k_init_leaves(BuildNode* N, uint32_t n, const uint64_t* keys, const float4* lo, const float4* hi) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint32_t prim = (uint32_t)(keys[j] & 0xffffffffu);
    BuildNode& L = N[(n - 1) + j];
    float4 a = lo[prim], b = hi[prim];
    L.lo[0] = a.x; L.lo[1] = a.y; L.lo[2] = a.z; L.hi[0] = b.x; L.hi[1] = b.y; L.hi[2] = b.z;
    L.left = L.right = -1; L.first = L.last = (int)j; L.kept = 1; L.depth = 0;
    if (n == 1) L.parent = -1;
}

__global__ void k_karras(BuildNode* N, int n, const uint64_t* k) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    int d = (delta(k, n, i, i + 1) - delta(k, n, i, i - 1)) >= 0 ? 1 : -1;
    int dmin = delta(k, n, i, i - d);
    int lmax = 2;
    while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
    int j = i + l * d;
    int dnode = delta(k, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    int gamma = i + s * d + min(d, 0);
    int first = min(i, j), last = max(i, j);
    int left = (first == gamma) ? (n - 1) + gamma : gamma;
    int right = (last == gamma + 1) ? (n - 1) + gamma + 1 : gamma + 1;
    BuildNode& I = N[i];
    I.left = left; I.right = right; I.first = first; I.last = last;
    N[left].parent = i; N[right].parent = i;
    if (i == 0) I.parent = -1;
}

__global__ void k_depth(BuildNode* N, int total, int* max_depth) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int d = 0, c = i;
    while (N[c].parent >= 0) { c = N[c].parent; ++d; }
    N[i].depth = d;
    atomicMax(max_depth, d);
}

__global__ void k_refit_level(BuildNode* N, int n_internal, int level) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_internal || N[i].depth != level) return;
    BuildNode& I = N[i];
    const BuildNode& A = N[I.left];
    const BuildNode& B = N[I.right];
    for (int a = 0; a < 3; ++a) { I.lo[a] = fminf(A.lo[a], B.lo[a]); I.hi[a] = fmaxf(A.hi[a], B.hi[a]); }
    int size = I.last - I.first + 1;
    I.kept = size <= kLeafMax ? 1 : 1 + A.kept + B.kept;
}

__device__ __forceinline__ bool is_collapsed(const BuildNode* N, int n, int c) {
    // internal node turned into a leaf
    return c < n - 1 && (N[c].last - N[c].first + 1) <= kLeafMax;
}
__device__ __forceinline__ bool is_emitted(const BuildNode* N, int n, int c) {
    for (int q = N[c].parent; q >= 0; q = N[q].parent)
        if (is_collapsed(N, n, q)) return false;
    return true;
}

__global__ void k_emit(const BuildNode* N, int n, float4* out) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    int total = 2 * n - 1;
    if (c >= total || !is_emitted(N, n, c)) return;
    int idx = 0;
    for (int ch = c, q = N[c].parent; q >= 0; ch = q, q = N[q].parent) {
        idx += 1;
        if (N[q].right == ch) idx += N[N[q].left].kept;
    }
    const BuildNode& X = N[c];
    bool leaf = (c >= n - 1) || is_collapsed(N, n, c);
    int skip = idx + (leaf ? 1 : X.kept);
    int info = leaf ? ((X.first << 3) | (X.last - X.first)) : -1;
    out[2 * idx] = make_float4(X.lo[0], X.lo[1], X.lo[2], __int_as_float(skip));
    out[2 * idx + 1] = make_float4(X.hi[0], X.hi[1], X.hi[2], __int_as_float(info));
}

__global__ void k_leaf_tris(const float* __restrict__ pos, const uint64_t* keys, uint32_t n, float4* tris) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint32_t prim = (uint32_t)(keys[k] & 0xffffffffu);
    const float* p = pos + 9 * (size_t)prim;
    float v0x = p[0], v0y = p[1], v0z = p[2];
    tris[3 * k] = make_float4(v0x, v0y, v0z, __int_as_float((int)prim));
    tris[3 * k + 1] = make_float4(p[3] - v0x, p[4] - v0y, p[5] - v0z, 0.0f);
    tris[3 * k + 2] = make_float4(p[6] - v0x, p[7] - v0y, p[8] - v0z, 0.0f);
}

#define BVH_CHECK(x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) { err = std::string(#x ": ") + hipGetErrorString(e_); goto fail; } \
    } while (0)

// Builds the BVH for n triangles at d_pos (n*9 floats, device).  On success *d_nodes (2*n_nodes
// float4) and *d_tris (3*n float4) are new device allocations owned by the caller.
int build_bvh_lbvh(const float* d_pos, uint32_t n, hipStream_t st, float4** d_nodes, uint32_t* n_nodes,
                   float4** d_tris, std::string& err) {
    *d_nodes = nullptr; *d_tris = nullptr; *n_nodes = 0;
    if (n == 0) return 0;
    if (n >= (1u << 28)) { err = "too many triangles for the 28-bit leaf index"; return -1; }
    float4 *lo = nullptr, *hi = nullptr, *nodes = nullptr, *tris = nullptr;
    int* cb = nullptr;
    uint64_t *keys = nullptr, *keys_sorted = nullptr;
    BuildNode* N = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int* dmax = nullptr;
    int max_depth = 0, total = 2 * (int)n - 1, kept_root = 1;
    const int B = 256;
    const int gn = (int)((n + B - 1) / B), gt = (total + B - 1) / B;
    int init_cb[6] = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MIN, INT32_MIN, INT32_MIN};

    BVH_CHECK(hipMalloc(&lo, n * sizeof(float4)));
    BVH_CHECK(hipMalloc(&hi, n * sizeof(float4)));
    BVH_CHECK(hipMalloc(&cb, 6 * sizeof(int)));
    BVH_CHECK(hipMalloc(&dmax, sizeof(int)));
    BVH_CHECK(hipMalloc(&keys, n * sizeof(uint64_t)));
    BVH_CHECK(hipMalloc(&keys_sorted, n * sizeof(uint64_t)));
    BVH_CHECK(hipMalloc(&N, (size_t)total * sizeof(BuildNode)));
    BVH_CHECK(hipMemcpyAsync(cb, init_cb, sizeof init_cb, hipMemcpyHostToDevice, st));
    BVH_CHECK(hipMemsetAsync(dmax, 0, sizeof(int), st));

    k_prim_bounds<<<gn, B, 0, st>>>(d_pos, n, lo, hi, cb);
    k_morton<<<gn, B, 0, st>>>(lo, hi, n, cb, keys);
    BVH_CHECK(hipGetLastError());
    BVH_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, keys, keys_sorted, (int)n, 0, 62, st));
    BVH_CHECK(hipMalloc(&tmp, tmp_bytes));
    BVH_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, keys, keys_sorted, (int)n, 0, 62, st));

    k_init_leaves<<<gn, B, 0, st>>>(N, n, keys_sorted, lo, hi);
    if (n > 1) k_karras<<<gn, B, 0, st>>>(N, (int)n, keys_sorted);
    k_depth<<<gt, B, 0, st>>>(N, total, dmax);
    BVH_CHECK(hipGetLastError());
    BVH_CHECK(hipMemcpyAsync(&max_depth, dmax, sizeof(int), hipMemcpyDeviceToHost, st));
    BVH_CHECK(hipStreamSynchronize(st));
    if (n > 1) {
        int gi = (int)((n - 1 + B - 1) / B);
        for (int lv = max_depth; lv >= 0; --lv) k_refit_level<<<gi, B, 0, st>>>(N, (int)n - 1, lv);
        BVH_CHECK(hipGetLastError());
        BVH_CHECK(hipMemcpyAsync(&kept_root, &N[0].kept, sizeof(int), hipMemcpyDeviceToHost, st));
        BVH_CHECK(hipStreamSynchronize(st));
    }
    // + 1 zeroed pad node (node n is readable: room for speculative next-node loads)
    BVH_CHECK(hipMalloc(&nodes, ((size_t)kept_root + 1) * 2 * sizeof(float4)));
    BVH_CHECK(hipMemsetAsync(nodes + 2 * (size_t)kept_root, 0, 2 * sizeof(float4), st));
    BVH_CHECK(hipMalloc(&tris, (size_t)n * 3 * sizeof(float4)));
    if (n > 1) {
        k_emit<<<gt, B, 0, st>>>(N, (int)n, nodes);
    } else {
        k_emit<<<1, B, 0, st>>>(N, 1, nodes);
    }
    k_leaf_tris<<<gn, B, 0, st>>>(d_pos, keys_sorted, n, tris);
    BVH_CHECK(hipGetLastError());
    BVH_CHECK(hipStreamSynchronize(st));
    *d_nodes = nodes; *d_tris = tris; *n_nodes = (uint32_t)kept_root;
    nodes = nullptr; tris = nullptr;
    hipFree(lo); hipFree(hi); hipFree(cb); hipFree(dmax); hipFree(keys); hipFree(keys_sorted); hipFree(N); hipFree(tmp);
    return 0;
fail:
    if (lo) hipFree(lo);
    if (hi) hipFree(hi);
    if (cb) hipFree(cb);
    if (dmax) hipFree(dmax);
    if (keys) hipFree(keys);
    if (keys_sorted) hipFree(keys_sorted);
    if (N) hipFree(N);
    if (tmp) hipFree(tmp);
    if (nodes) hipFree(nodes);
    if (tris) hipFree(tris);
    return -1;
}


// ============================================================================================
// PLOC builder (Meister & Bittner 2018, "Parallel Locally-Ordered Clustering for Bounding Volume
// Hierarchy Construction"): Morton-ordered clusters; every iteration each cluster finds its nearest
// neighbour (smallest merged-box surface area) within +-kRadius positions, mutual nearest pairs merge,
// the cluster array is compacted by a prefix sum.  Near-SAH tree quality from fully data-parallel
// kernels (scripts/bvh_analysis.py: 20 node visits per C2 shadow ray vs 39 for Karras LBVH, 17 for a
// binned-SAH sweep).  Then a bottom-up SAH collapse into leaves of <= 8 triangles and the same
// preorder skip-pointer layout as above.  Deterministic: ties go to the smaller index, node ids come
// from prefix sums, no atomics decide structure.
// ============================================================================================
#ifndef RS_PLOC_RADIUS
#define RS_PLOC_RADIUS 16
#endif
constexpr int kRadius = RS_PLOC_RADIUS;
constexpr int kPlocBlock = 256;
#ifndef RS_LEAF_MAX
#define RS_LEAF_MAX 8
#endif
#ifndef RS_SAH_CTRI
#define RS_SAH_CTRI 1.0f
#endif
constexpr int kLeafMaxSah = RS_LEAF_MAX;          // <= 8 (leaf word: (first << 3) | (count - 1))
constexpr float kCtrav = 1.0f, kCtri = RS_SAH_CTRI;

__device__ __forceinline__ float half_area(float4 lo, float4 hi) {
    float ex = hi.x - lo.x, ey = hi.y - lo.y, ez = hi.z - lo.z;
    return ex * ey + ey * ez + ez * ex;
}

// leaves: node j = j-th prim in Morton order; lo.w = -1 (no left child), hi.w = prim index
__global__ void k_ploc_leaves(const uint64_t* keys, uint32_t n, const float4* lo, const float4* hi, float4* nlo,
                              float4* nhi, int* cnt, int* C) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint32_t prim = (uint32_t)(keys[j] & 0xffffffffu);
    float4 a = lo[prim], b = hi[prim];
    nlo[j] = make_float4(a.x, a.y, a.z, __int_as_float(-1));
    nhi[j] = make_float4(b.x, b.y, b.z, __int_as_float((int)prim));
    cnt[j] = 1;
    C[j] = (int)j;
}

// The iterations run in batches without a host round trip (kPlocBatch per synchronisation): the cluster count
// and the next node id live in a device state that each iteration reads from slot p and writes to slot p ^ 1
// (PlocState); grids are sized by the count at the last synchronisation, and an iteration that finds one
// cluster left (or a failed one) passes the state and the cluster array through unchanged.
struct PlocState { int k, base, err, pad; };
constexpr int kPlocBatch = 4;

__global__ void __launch_bounds__(kPlocBlock) k_ploc_nearest(const int* C, const PlocState* S, const float4* nlo,
                                                             const float4* nhi, int* N) {
    const int k = S->k;
    if (k <= 1 || S->err) return;
    __shared__ float4 slo[kPlocBlock + 2 * kRadius], shi[kPlocBlock + 2 * kRadius];
    const int base = blockIdx.x * kPlocBlock;
    if (base >= k) return;
    for (int t = threadIdx.x; t < kPlocBlock + 2 * kRadius; t += kPlocBlock) {
        int g = base - kRadius + t;
        if (g >= 0 && g < k) {
            int c = C[g];
            slo[t] = nlo[c];
            shi[t] = nhi[c];
        }
    }
    __syncthreads();
    const int i = base + threadIdx.x;
    if (i >= k) return;
    const float4 a = slo[threadIdx.x + kRadius], b = shi[threadIdx.x + kRadius];
    double best = INFINITY;
    int bj = -1;
    for (int o = -kRadius; o <= kRadius; ++o) {
        int j = i + o;
        if (o == 0 || j < 0 || j >= k) continue;
        float4 c = slo[threadIdx.x + kRadius + o], d = shi[threadIdx.x + kRadius + o];
        float ex = fmaxf(b.x, d.x) - fminf(a.x, c.x);
        float ey = fmaxf(b.y, d.y) - fminf(a.y, c.y);
        float ez = fmaxf(b.z, d.z) - fminf(a.z, c.z);
        const float af = ex * ey + ey * ez + ez * ex;
        // a float area that overflows (coordinates beyond ~1e19) is re-formed in double, so the nearest
        // neighbour stays defined and PLOC keeps merging; finite areas compare exactly as before
        const double area = af < INFINITY ? (double)af
                                          : (double)ex * ey + (double)ey * ez + (double)ez * ex;
        if (area < best) { best = area; bj = j; }      // j ascending: ties keep the smaller index
    }
    N[i] = bj;
}

// flags of the k live clusters; zeros over [k, kmax) so the scans may run over the host's bound kmax
__global__ void k_ploc_flags(const int* N, const PlocState* S, int kmax, int* valid, int* merged) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = S->k;
    if (i >= kmax || k <= 1 || S->err) return;
    if (i >= k) { valid[i] = 0; merged[i] = 0; return; }
    int j = N[i];
    bool mutual = j >= 0 && N[j] == i;
    valid[i] = (mutual && j < i) ? 0 : 1;   // the right partner of a merge disappears
    merged[i] = (mutual && i < j) ? 1 : 0;
}

__global__ void k_ploc_merge(const int* C, const PlocState* S, PlocState* Snext, const int* N, const int* valid,
                             const int* merged, const int* pos, const int* mid, float4* nlo, float4* nhi, int* parent,
                             int* cnt, int* Cout) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    const PlocState s = *S;
    if (s.k <= 1 || s.err) {                   // done (or failed): pass everything through
        if (i == 0) { *Snext = s; Cout[0] = C[0]; }
        return;
    }
    if (i >= s.k) return;
    if (i == s.k - 1) {                        // the last cluster knows the totals of the scans
        const int merges = mid[i] + merged[i];
        *Snext = PlocState{pos[i] + valid[i], s.base + merges, merges <= 0 ? 1 : 0, 0};
    }
    if (merged[i]) {
        int id = s.base + mid[i];
        int L = C[i], R = C[N[i]];
        float4 al = nlo[L], ah = nhi[L], bl = nlo[R], bh = nhi[R];
        nlo[id] = make_float4(fminf(al.x, bl.x), fminf(al.y, bl.y), fminf(al.z, bl.z), __int_as_float(L));
        nhi[id] = make_float4(fmaxf(ah.x, bh.x), fmaxf(ah.y, bh.y), fmaxf(ah.z, bh.z), __int_as_float(R));
        parent[L] = id; parent[R] = id;
        cnt[id] = cnt[L] + cnt[R];
        Cout[pos[i]] = id;
    } else if (valid[i]) {
        Cout[pos[i]] = C[i];
    }
}

__global__ void k_ploc_depth(const int* parent, int total, int* depth, int* max_depth) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= total) return;
    int d = 0;
    for (int q = parent[c]; q >= 0; q = parent[q]) ++d;
    depth[c] = d;
    atomicMax(max_depth, d);
}

// bottom-up SAH collapse, one depth level per launch (internal node ids are [n, 2n-1))
__global__ void k_ploc_collapse(const float4* nlo, const float4* nhi, const int* cnt, const int* depth, int n, int level,
                                float* cost, int* kept, int* collapsed) {
    int c = n + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= 2 * n - 1 || depth[c] != level) return;
    int L = __float_as_int(nlo[c].w), R = __float_as_int(nhi[c].w);
    float A = fmaxf(half_area(nlo[c], nhi[c]), 1e-30f);
    float split = kCtrav + (half_area(nlo[L], nhi[L]) * cost[L] + half_area(nlo[R], nhi[R]) * cost[R]) / A;
    float leaf = kCtri * (float)cnt[c];
    if (cnt[c] <= kLeafMaxSah && leaf <= split) {
        cost[c] = leaf; kept[c] = 1; collapsed[c] = 1;
    } else {
        cost[c] = split; kept[c] = 1 + kept[L] + kept[R]; collapsed[c] = 0;
    }
}

__global__ void k_ploc_leaf_init(int n, float* cost, int* kept, int* collapsed) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    cost[c] = kCtri; kept[c] = 1; collapsed[c] = 0;
}

// preorder index + triangle-slot offset by walking to the root; emits the skip-pointer nodes and,
// for every primitive leaf, its triangle in leaf order
__global__ void k_ploc_emit(const float4* nlo, const float4* nhi, const int* parent, const int* cnt, const int* kept,
                            const int* collapsed, int n, const float* __restrict__ pos, float4* out, float4* tris) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= 2 * n - 1) return;
    bool emitted = true;
    int idx = 0, off = 0;
    for (int ch = c, q = parent[c]; q >= 0; ch = q, q = parent[q]) {
        if (collapsed[q]) emitted = false;
        int L = __float_as_int(nlo[q].w);
        idx += 1;
        if (L != ch) { idx += kept[L]; off += cnt[L]; }   // ch is the right child
    }
    if (c < n) {   // primitive: its triangle slot is `off`
        int prim = __float_as_int(nhi[c].w);
        const float* p = pos + 9 * (size_t)prim;
        float v0x = p[0], v0y = p[1], v0z = p[2];
        tris[3 * off] = make_float4(v0x, v0y, v0z, __int_as_float(prim));
        tris[3 * off + 1] = make_float4(p[3] - v0x, p[4] - v0y, p[5] - v0z, 0.0f);
        tris[3 * off + 2] = make_float4(p[6] - v0x, p[7] - v0y, p[8] - v0z, 0.0f);
    }
    if (!emitted) return;
    bool leaf = (c < n) || collapsed[c];
    int skip = idx + (leaf ? 1 : kept[c]);
    int info = leaf ? ((off << 3) | (cnt[c] - 1)) : -1;
    float4 a = nlo[c], b = nhi[c];
    out[2 * idx] = make_float4(a.x, a.y, a.z, __int_as_float(skip));
    out[2 * idx + 1] = make_float4(b.x, b.y, b.z, __int_as_float(info));
}


// The builders' scratch (stream-ordered allocations) comes from a private pool per device, never the device's
// default pool that the host process (PyTorch, other libraries) shares: it caches its blocks across the launches
// of one build (release threshold: unlimited) and is trimmed to empty after every build (builder_pool_trim).
static hipMemPool_t g_builder_pool[64] = {};
static std::mutex g_builder_pool_mu;
hipMemPool_t builder_pool() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(g_builder_pool_mu);
    if (!g_builder_pool[dev]) {
        hipMemPoolProps pp = {};
        pp.allocType = hipMemAllocationTypePinned;
        pp.location.type = hipMemLocationTypeDevice;
        pp.location.id = dev;
        hipMemPool_t pl = nullptr;
        if (hipMemPoolCreate(&pl, &pp) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
        uint64_t keep = ~0ull;
        (void)hipMemPoolSetAttribute(pl, hipMemPoolAttrReleaseThreshold, &keep);
        g_builder_pool[dev] = pl;
    }
    return g_builder_pool[dev];
}
hipError_t pool_malloc(void** p, size_t bytes, hipStream_t st) {
    hipMemPool_t pl = builder_pool();
    return pl ? hipMallocFromPoolAsync(p, bytes, pl, st) : hipMallocAsync(p, bytes, st);
}
// after a build has finished on the host's view (its stream synchronised): return the scratch to the driver
void builder_pool_trim() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return;
    std::lock_guard<std::mutex> lk(g_builder_pool_mu);
    if (g_builder_pool[dev]) (void)hipMemPoolTrimTo(g_builder_pool[dev], 0);
}

#define PLOC_CHECK(x)                                                                  \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) { err = std::string(#x ": ") + hipGetErrorString(e_); goto fail; } \
    } while (0)

int build_bvh_ploc(const float* d_pos, uint32_t n, hipStream_t st, float4** d_nodes, uint32_t* n_nodes,
                   float4** d_tris, std::string& err) {
    *d_nodes = nullptr; *d_tris = nullptr; *n_nodes = 0;
    if (n == 0) return 0;
    if (n >= (1u << 27)) { err = "too many triangles for the leaf index"; return -1; }
    const int total = 2 * (int)n - 1;
    const int B = 256;
    float4 *lo = nullptr, *hi = nullptr, *nlo = nullptr, *nhi = nullptr, *nodes = nullptr, *tris = nullptr;
    int *cb = nullptr, *cnt = nullptr, *parent = nullptr, *C0 = nullptr, *C1 = nullptr, *N = nullptr;
    int *valid = nullptr, *merged = nullptr, *pos = nullptr, *mid = nullptr, *depth = nullptr, *dmax = nullptr;
    int *kept = nullptr, *collapsed = nullptr;
    float* cost = nullptr;
    uint64_t *keys = nullptr, *keys_sorted = nullptr;
    void *tmp = nullptr, *tmp2 = nullptr;
    size_t tmp_bytes = 0, tmp2_bytes = 0;
    int init_cb[6] = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MIN, INT32_MIN, INT32_MIN};
    int k = (int)n, base = (int)n, root = 0, max_depth = 0, kept_root = 1;
    PlocState* pst = nullptr;                  // two slots (the iteration's parity)

    PLOC_CHECK(pool_malloc((void**)&lo, n * sizeof(float4), st));
    PLOC_CHECK(pool_malloc((void**)&hi, n * sizeof(float4), st));
    PLOC_CHECK(pool_malloc((void**)&cb, 6 * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&keys, n * sizeof(uint64_t), st));
    PLOC_CHECK(pool_malloc((void**)&keys_sorted, n * sizeof(uint64_t), st));
    PLOC_CHECK(pool_malloc((void**)&nlo, (size_t)total * sizeof(float4), st));
    PLOC_CHECK(pool_malloc((void**)&nhi, (size_t)total * sizeof(float4), st));
    PLOC_CHECK(pool_malloc((void**)&cnt, (size_t)total * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&parent, (size_t)total * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&depth, (size_t)total * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&kept, (size_t)total * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&collapsed, (size_t)total * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&cost, (size_t)total * sizeof(float), st));
    PLOC_CHECK(pool_malloc((void**)&C0, n * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&C1, n * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&N, n * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&valid, n * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&merged, n * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&pos, n * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&mid, n * sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&dmax, sizeof(int), st));
    PLOC_CHECK(pool_malloc((void**)&pst, 2 * sizeof(PlocState), st));
    PLOC_CHECK(hipMemcpyAsync(cb, init_cb, sizeof init_cb, hipMemcpyHostToDevice, st));
    PLOC_CHECK(hipMemsetAsync(dmax, 0, sizeof(int), st));
    PLOC_CHECK(hipMemsetAsync(parent, 0xff, (size_t)total * sizeof(int), st));   // -1

    k_prim_bounds<<<(n + B - 1) / B, B, 0, st>>>(d_pos, n, lo, hi, cb);
    k_morton<<<(n + B - 1) / B, B, 0, st>>>(lo, hi, n, cb, keys);
    PLOC_CHECK(hipGetLastError());
    PLOC_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, keys, keys_sorted, (int)n, 0, 62, st));
    PLOC_CHECK(pool_malloc(&tmp, tmp_bytes, st));
    PLOC_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, keys, keys_sorted, (int)n, 0, 62, st));
    PLOC_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2_bytes, valid, pos, (int)n, st));
    PLOC_CHECK(pool_malloc(&tmp2, tmp2_bytes, st));
    k_ploc_leaves<<<(n + B - 1) / B, B, 0, st>>>(keys_sorted, n, lo, hi, nlo, nhi, cnt, C0);
    PLOC_CHECK(hipGetLastError());

    {
        PlocState h0{k, base, 0, 0};
        PLOC_CHECK(hipMemcpyAsync(&pst[0], &h0, sizeof h0, hipMemcpyHostToDevice, st));
    }
    for (int par = 0; k > 1;) {                  // batches of kPlocBatch iterations, one round trip each
        const int kmax = k, g = (kmax + B - 1) / B;
        for (int it = 0; it < kPlocBatch; ++it, par ^= 1) {
            k_ploc_nearest<<<(kmax + kPlocBlock - 1) / kPlocBlock, kPlocBlock, 0, st>>>(C0, pst + par, nlo, nhi, N);
            k_ploc_flags<<<g, B, 0, st>>>(N, pst + par, kmax, valid, merged);
            PLOC_CHECK(hipGetLastError());
            PLOC_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp2, tmp2_bytes, valid, pos, kmax, st));
            PLOC_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp2, tmp2_bytes, merged, mid, kmax, st));
            k_ploc_merge<<<g, B, 0, st>>>(C0, pst + par, pst + (par ^ 1), N, valid, merged, pos, mid, nlo, nhi, parent,
                                          cnt, C1);
            PLOC_CHECK(hipGetLastError());
            std::swap(C0, C1);
        }
        PlocState hs{};
        PLOC_CHECK(hipMemcpyAsync(&hs, pst + par, sizeof hs, hipMemcpyDeviceToHost, st));
        PLOC_CHECK(hipStreamSynchronize(st));
        if (hs.err) { err = "PLOC made no progress"; goto fail; }
        k = hs.k;
        base = hs.base;
    }
    PLOC_CHECK(hipMemcpyAsync(&root, C0, sizeof(int), hipMemcpyDeviceToHost, st));
    PLOC_CHECK(hipStreamSynchronize(st));
    if (root != total - 1) { err = "PLOC root id mismatch"; goto fail; }
    k_ploc_depth<<<(total + B - 1) / B, B, 0, st>>>(parent, total, depth, dmax);
    k_ploc_leaf_init<<<(n + B - 1) / B, B, 0, st>>>((int)n, cost, kept, collapsed);
    PLOC_CHECK(hipGetLastError());
    PLOC_CHECK(hipMemcpyAsync(&max_depth, dmax, sizeof(int), hipMemcpyDeviceToHost, st));
    PLOC_CHECK(hipStreamSynchronize(st));
    if (n > 1) {
        int gi = (int)((n - 1 + B - 1) / B);
        for (int lv = max_depth; lv >= 0; --lv)
            k_ploc_collapse<<<gi, B, 0, st>>>(nlo, nhi, cnt, depth, (int)n, lv, cost, kept, collapsed);
        PLOC_CHECK(hipGetLastError());
        PLOC_CHECK(hipMemcpyAsync(&kept_root, kept + root, sizeof(int), hipMemcpyDeviceToHost, st));
        PLOC_CHECK(hipStreamSynchronize(st));
    }
    // + 1 zeroed pad node (node n is readable: room for speculative next-node loads)
    PLOC_CHECK(hipMalloc(&nodes, ((size_t)kept_root + 1) * 2 * sizeof(float4)));
    PLOC_CHECK(hipMemsetAsync(nodes + 2 * (size_t)kept_root, 0, 2 * sizeof(float4), st));
    PLOC_CHECK(hipMalloc(&tris, (size_t)n * 3 * sizeof(float4)));
    k_ploc_emit<<<(total + B - 1) / B, B, 0, st>>>(nlo, nhi, parent, cnt, kept, collapsed, (int)n, d_pos, nodes, tris);
    PLOC_CHECK(hipGetLastError());
    PLOC_CHECK(hipStreamSynchronize(st));
    *d_nodes = nodes; *d_tris = tris; *n_nodes = (uint32_t)kept_root;
    nodes = nullptr; tris = nullptr;
fail: {
        // scratch: stream-ordered frees into the device pool (no synchronisation; the next build's or the wide
        // build's allocations reuse it, see build_pool_setup); the outputs are ordinary allocations
        void* ptrs[] = {lo, hi, nlo, nhi, cb, cnt, parent, C0, C1, N, valid, merged, pos, mid, depth,
                        dmax, kept, collapsed, cost, keys, keys_sorted, tmp, tmp2, pst};
        for (void* p : ptrs) if (p) (void)hipFreeAsync(p, st);
        if (nodes) hipFree(nodes);
        if (tris) hipFree(tris);
    }
    return *d_nodes || n == 0 ? 0 : -1;
}

// ---------------------------------------------------------------- in-place refit (rs_refit.h)
// multi-workgroup launches always get l1 == l0 + 1
__global__ void __launch_bounds__(kRefitBlock) k_refit(float4* nodes, float4* tris, const float* __restrict__ pos,
                                                       const int* __restrict__ order, const int* __restrict__ lvl_off,
                                                       int l0, int l1) {
    refit_levels(nodes, tris, pos, order, lvl_off, l0, l1, blockIdx.x, gridDim.x);
}

// node ids grouped by depth, deepest level first (host, once per topology)
int bvh_refit_plan(const float4* d_nodes, uint32_t n_nodes, hipStream_t st, int** d_order, int** d_lvl_off,
                   std::vector<int>& lvl_off, std::string& err) {
    *d_order = nullptr; *d_lvl_off = nullptr; lvl_off.clear();
    if (n_nodes == 0) return 0;
    std::vector<float4> h(2 * (size_t)n_nodes);
    if (hipMemcpyAsync(h.data(), d_nodes, h.size() * sizeof(float4), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) { err = "refit plan: node download failed"; return -1; }
    std::vector<int> depth(n_nodes), ends;
    int max_d = 0;
    for (uint32_t i = 0; i < n_nodes; ++i) {          // ancestors of i = open subtrees whose skip > i
        while (!ends.empty() && (uint32_t)ends.back() <= i) ends.pop_back();
        depth[i] = (int)ends.size();
        max_d = std::max(max_d, depth[i]);
        int skip, leaf;
        std::memcpy(&skip, &h[2 * i].w, 4); std::memcpy(&leaf, &h[2 * i + 1].w, 4);
        if (leaf < 0) ends.push_back(skip);
    }
    std::vector<int> cnt(max_d + 1, 0), order(n_nodes);
    for (uint32_t i = 0; i < n_nodes; ++i) cnt[max_d - depth[i]]++;
    lvl_off.assign(max_d + 2, 0);
    for (int l = 0; l <= max_d; ++l) lvl_off[l + 1] = lvl_off[l] + cnt[l];
    std::vector<int> fill(lvl_off.begin(), lvl_off.end() - 1);
    for (uint32_t i = 0; i < n_nodes; ++i) order[fill[max_d - depth[i]]++] = (int)i;
    if (hipMalloc(d_order, order.size() * sizeof(int)) != hipSuccess ||
        hipMalloc(d_lvl_off, lvl_off.size() * sizeof(int)) != hipSuccess) { err = "refit plan: hipMalloc failed"; return -1; }
    if (hipMemcpyAsync(*d_order, order.data(), order.size() * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(*d_lvl_off, lvl_off.data(), lvl_off.size() * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) { err = "refit plan: upload failed"; return -1; }
    return 0;
}

// stream-ordered refit; no host synchronisation.  With *tail != nullptr a final single-workgroup
// batch is not launched but returned (levels [tail[0], tail[1])) for the caller to fuse.
int bvh_refit(float4* d_nodes, float4* d_tris, const float* d_pos, const int* d_order, const int* d_lvl_off,
              const std::vector<int>& lvl_off, hipStream_t st, int* tail, std::string& err) {
    const std::vector<RefitBatch> bs = refit_batches(lvl_off);
    if (tail) tail[0] = tail[1] = 0;
    for (size_t i = 0; i < bs.size(); ++i) {
        const RefitBatch& r = bs[i];
        if (tail && i + 1 == bs.size() && r.blocks == 1) { tail[0] = r.l0; tail[1] = r.l1; break; }
        k_refit<<<r.blocks, kRefitBlock, 0, st>>>(d_nodes, d_tris, d_pos, d_order, d_lvl_off, r.l0, r.l1);
    }
    if (hipGetLastError() != hipSuccess) { err = "refit launch failed"; return -1; }
    return 0;
}

// builder selection: PLOC by default; RESTIR_BVH=lbvh selects the Karras LBVH (kept for comparison).  Then the
// 8-wide tree of the per-lane walks from the positions alone (rs_wide_build.hip); it is optional: when it does
// not apply (non-finite positions, no plan within the walk's depth) or its build fails, the scene keeps the
// binary tree and the walks take the skip pointers (RESTIR_WIDE=off: never built).
int build_wide_gpu(const float* d_pos, int n, hipStream_t st, WideBvh* w, std::string& err);
void preload_wide_build();
// HIP loads a source file's code object at the first launch (or attribute query) of one of its kernels: at
// context creation, so that a scene build is not charged the one-time load of the builders (~10 ms at C3)
void preload_code_objects() {
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, (const void*)k_ploc_nearest);
    preload_wide_build();
    (void)builder_pool();
    (void)hipGetLastError();
}
void wide_free(WideBvh& w) {
    void* p[] = {w.nodes, w.tris, w.box};
    for (void* q : p) if (q) hipFree(q);
    w = WideBvh{};
}
int build_bvh(const float* d_pos, uint32_t n, hipStream_t st, float4** d_nodes, uint32_t* n_nodes, float4** d_tris,
              WideBvh* wide, std::string& err) {
    const char* e = getenv("RESTIR_BVH");
    const char* w = getenv("RESTIR_WIDE");
    if (w && std::string(w) == "off") { if (wide) { wide_free(*wide); wide->status = RS_WIDE_OFF; } wide = nullptr; }
    const int rc = (e && std::string(e) == "lbvh") ? build_bvh_lbvh(d_pos, n, st, d_nodes, n_nodes, d_tris, err)
                                                   : build_bvh_ploc(d_pos, n, st, d_nodes, n_nodes, d_tris, err);
    if (rc != 0 || !wide) return rc;
    std::string werr;
    if (const int wr = build_wide_gpu(d_pos, (int)n, st, wide, werr); wr != 0) {   // optional: binary walks
        const int why = wr < 0 ? RS_WIDE_ERROR : (wide->status ? wide->status : RS_WIDE_ERROR);
        wide_free(*wide);
        wide->status = why;
    }
    (void)hipGetLastError();
    return 0;
}

}  // namespace rs
