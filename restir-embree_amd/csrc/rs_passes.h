// rs_passes.h -- the per-pixel ReSTIR passes as device functions + kernels (gfx950).
//
// One thread per pixel; a 64-lane wave covers an 8x8 pixel tile (primary/shadow-ray coherence and
// L1/L2 locality of the neighbour gathers), a 256-thread workgroup a 16x16 tile.
// Passes (SimpleGuiDX11::produceRestir, pg/simpleguidx11.cpp:359-487):
//   k_gbuffer_initial : gBufferFillPass (:368-375) fused with initialRenderPass (:381-388) -- the
//                       initial pass reads only its own pixel's G record, so it stays in registers
//   k_visibility      : visibilityPass (:393-402)
//   k_temporal        : temporalReusePass (:408-420)
//   k_spatial         : spatialReusePass (:428-443), the last pass fused with the shade loop
//                       (:449-472): the shaded f is the selected candidate's (already visibility-
//                       tested) f, cached, so shading costs no extra shadow ray
//   k_shade           : stand-alone shade loop when no reuse pass can carry it
//
// Convergence: every ray query is made by the whole wave (lanes without a ray pass active=false), so
// the lockstep traversal (rs_scene.h) sees a full EXEC mask.  Per-pixel early-outs of the reference
// (emissive pixel, invalid sample, zero contribution) are therefore predicates, not branches; lanes
// outside the image work on a clamped pixel and store nothing.
#pragma once
#include "rs_scene.h"
#include "rs_texture.h"

// waves per SIMD the ray-tracing kernels are register-budgeted for (launch_bounds 2nd argument)
#ifndef RS_INITIAL_WAVES
#define RS_INITIAL_WAVES 4
#endif
#ifndef RS_SPATIAL_WAVES
#define RS_SPATIAL_WAVES 4
#endif
// ... for a small lockstep spatial launch (a rank's band: < 2 rounds of waves), which runs beside the
// other frames in flight (C2 balanced bands, 5 vs 4 waves: 1/4 band 0.373 vs 0.383 ms/frame, 1/8 band
// 0.241 vs 0.244; a full-size launch stays at 4: 5 cost C5 3.7 %)
#ifndef RS_SPATIAL_WAVES_SMALL
#define RS_SPATIAL_WAVES_SMALL RS_SPATIAL_WAVES
#endif
// ... for the per-lane traversal kind (incoherent scenes: the walk loop needs more registers)
#ifndef RS_INITIAL_WAVES_LANE
#define RS_INITIAL_WAVES_LANE RS_INITIAL_WAVES
#endif
#ifndef RS_SPATIAL_WAVES_LANE
#define RS_SPATIAL_WAVES_LANE RS_SPATIAL_WAVES
#endif
#ifndef RS_TEMPORAL_WAVES
#define RS_TEMPORAL_WAVES 4
#endif
#ifndef RS_TEMPORAL_WAVES_LANE
#define RS_TEMPORAL_WAVES_LANE RS_TEMPORAL_WAVES
#endif
#define RS_WAVES(T, lockstep, lane) (((T) & TRAV_LANE) ? (lane) : (lockstep))
// area candidates whose shadow rays share one lockstep traversal (occluded_wave_multi); 4 measured on
// C2 1080p: 694-698 frames/s at a 4-wave budget (700-704 with 2), 560 at 5 waves (register spills)
#ifndef RS_RIS_BATCH
#define RS_RIS_BATCH 2
#endif
// ... for the per-lane walk: one candidate at a time (per-lane walks gain nothing from batching, and a
// second pending ray is register pressure inside the walk loop: C3 +1.3 %)
#ifndef RS_RIS_BATCH_LANE
#define RS_RIS_BATCH_LANE 1
#endif

namespace rs {

struct FrameConst {
    // rs_frame_params snapshot
    int m_area, m_brdf, k, spatial_passes, cap;
    float radius, min_normal_sim, max_depth_diff;
    int do_spatial, do_temporal, do_vis_pass, reject, mis;
    vec3 bg; float tnear_off, tfar_off, normal_off;
    int use_sky;          // useSkybox with a scene sky (rs_texture.h sky_texel)
    uint32_t seed, frame;
    int W, H;             // full frame
    int y0, y1;           // band this context renders
    int gy0, gy1;         // G-buffer rows computed (band + margin, clamped)
    float inv_view[9];    // mat3(invViewMat), column-major (pg/camera.cpp:57)
    float inv_view_prev[9];   // ... of the previous frame (a tile's temporal pass rebuilds G elements)
    GCam cam, camp;       // current / previous frame camera (pg/GBufferElement.h:136-139)
    const int* row_order; // full-frame launches: grid row -> 16-px tile row, costliest first (or null)
    int n_order;          // entries of row_order (== the grid's rows when it applies)
    int debug_reproj;     // debugReprojection: k_temporal records, k_debug_reproj paints (full frames)
    int canon_vis;        // spatial pass: the canonical (own) reservoir's sample is known unoccluded from the pixel
                          //   (restir_capi.hip rs_tile_spatial; §3.2) -- its visibility ray is not traced again
    uint8_t* dbg;         // 2 x W*H bytes: [p] the pixel's own rejection (1..3), [W*H + p] forward-check hit
    float* cand_w;        // the sorted initial pass's phase-A candidate weights (RS_SORT_STORE_W), per 8x8 tile
    float4* cand_ray;     // ... and its needed shadow rays' (direction, tfar) (RS_SORT_STORE_RAY), per 8x8 tile
};

struct Counters { unsigned long long rays, primary, reproj_outside; };   // per-frame totals

// Per-launch ray counting without atomics: every wave stores its (rays, primary) pair into its own
// slot of a per-launch array, k_reduce_counts sums all slots once per frame.  (Same-address device
// atomics from all 8 XCDs serialise at the memory side: one 64-bit atomicAdd per wave cost ~0.7 ms
// per 1080p kernel, more than the G-buffer pass itself -- scripts/initial_breakdown.py.)
struct CountSlot {
    uint2* part;                         // one entry per wave of the launch
    unsigned long long* outside;         // Counters::reproj_outside (rare: tile-edge reprojections)
    float* row_cost;                     // per-image-row wave time (rs_context_track_row_costs), or null
    int y0, y1;                          // rows whose cost is recorded (the rank's band)
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// constant-rate (100 MHz) clock at a wave's start, for the optional per-row cost record
__device__ __forceinline__ uint64_t wave_clock() { return __builtin_amdgcn_s_memrealtime(); }
// load-balancing record (rs_mgpu_rebalance, TiledRenderer.rebalance): the wave's lifetime spread evenly over the 8
// rows of its 8x8 tile from its top row (lanes 0..7 one row each), so band boundaries balance to the row rather than
// to the tile row.  Row-spread atomics, only while tracking is on (calibration frames).
#ifndef RS_ROWCOST_SPREAD
#define RS_ROWCOST_SPREAD 1    // 0: the whole wave's time on its top row (round 4)
#endif
__device__ __forceinline__ void row_cost_add(CountSlot C, uint64_t t0, int y) {
    if (!C.row_cost) return;
    constexpr int kRows = RS_ROWCOST_SPREAD ? 8 : 1;
    const int yt = __builtin_amdgcn_readfirstlane(y) + (int)(threadIdx.x & 63);
    const float w = (float)(wave_clock() - t0) * (1.0f / kRows);
    if ((threadIdx.x & 63) < kRows && yt >= C.y0 && yt < C.y1) atomicAdd(C.row_cost + yt, w);
}
__device__ __forceinline__ void count_rays(CountSlot C, uint32_t rays, uint32_t primary, uint64_t t0, int y) {
    uint32_t r = wave_sum(rays), p = wave_sum(primary);
    if ((threadIdx.x & 63) == 0)
        C.part[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)] = make_uint2(r, p);
    row_cost_add(C, t0, y);
}

// sum n slot pairs into the frame totals (and the context's running totals): kReduceBlocks
// one-wave workgroups reduce contiguous chunks into partials (integer sums: order-free), the last
// one folds them (a single workgroup streaming ~1.6 MB of slots at 1080p was CU-bandwidth bound:
// 40 us).  One wave per workgroup: the reduction runs while other frames' pass kernels fill
// the CUs, and a 1024-thread workgroup (16 free wave slots on one CU at once) waited ~150 us for a
// CU to drain -- on the frame's critical path (a rank's band: 0.36 ms initial + 0.15 ms waiting).
constexpr int kReduceBlocks = 128, kReduceThreads = 64;
__device__ __forceinline__ void block_sum2(unsigned long long& r, unsigned long long& p) {
    __shared__ unsigned long long sr[16], sp[16];
    for (int o = 32; o > 0; o >>= 1) { r += __shfl_xor(r, o, 64); p += __shfl_xor(p, o, 64); }
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) { sr[w] = r; sp[w] = p; }
    __syncthreads();
    r = 0; p = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < nw; ++i) { r += sr[i]; p += sp[i]; }
}
// One launch: every workgroup publishes its partial, and the last one to finish (a device-scope
// ticket; acquire/release at agent scope, since the partials come from all XCDs) folds them into the
// frame's totals and re-arms the ticket for the lane's next frame.  (Two launches cost one more
// ~11 us hipLaunchKernel on the host per frame.)
__global__ void __launch_bounds__(kReduceThreads) k_reduce_counts(const uint2* part, size_t n, ulonglong2* partial,
                                                                  unsigned* ticket, Counters* out, Counters* tot) {
    const size_t chunk = (n + gridDim.x - 1) / gridDim.x, b = blockIdx.x * chunk, e = b + chunk < n ? b + chunk : n;
    unsigned long long r = 0, p = 0;
    for (size_t i = b + threadIdx.x; i < e; i += kReduceThreads) { uint2 v = part[i]; r += v.x; p += v.y; }
    block_sum2(r, p);
    __shared__ bool last;
    if (threadIdx.x == 0) {
        __hip_atomic_store(&partial[blockIdx.x].x, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&partial[blockIdx.x].y, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    r = 0; p = 0;
    for (unsigned i = threadIdx.x; i < gridDim.x; i += kReduceThreads) {
        r += __hip_atomic_load(&partial[i].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        p += __hip_atomic_load(&partial[i].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    block_sum2(r, p);
    if (threadIdx.x == 0) {
        out->rays = r; out->primary = p;
        atomicAdd(&tot->rays, r); atomicAdd(&tot->primary, p);   // frames of several lanes may finish together
        // the frame's temporal pass (same stream, earlier) has finished counting its tile-edge misses
        const unsigned long long o = __hip_atomic_load(&out->reproj_outside, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (o) atomicAdd(&tot->reproj_outside, o);
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Workgroup -> screen tile.  Workgroups are dispatched in grid order, so a full-frame launch takes its
// 16-px tile rows in the context's cost order (costliest first: the longest-running workgroups start
// early and the cheap ones fill the launch's tail -- C2's floor rows cost ~2x its ceiling rows), measured
// during the traversal tuning frames (restir_capi.hip record_traversal_time).  Every pixel's work is
// independent of the order: results are identical for any order.  (Giving each XCD a vertical stripe
// of the frame instead, so neighbouring tiles share an L2, measured 1.85x slower on C2 and 3 % on C3.)
__device__ __forceinline__ int order_row(const int* order, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const int __attribute__((address_space(4)))* cint_ptr;   // uniform index: scalar load
    return ((cint_ptr)(order + i))[0];
#else
    return order[i];
#endif
}
__device__ __forceinline__ void tile_of(const FrameConst& F, int ya, int yb, int& bx, int& by) {
    bx = blockIdx.x; by = blockIdx.y;
    if (F.row_order && ya == 0 && yb == F.H && (uint32_t)F.n_order == gridDim.y) by = order_row(F.row_order, blockIdx.y);
}

// 8x8 tile per wave, 16x16 per workgroup, rows [ya, yb).  Returns whether the pixel exists; x/y are
// clamped into the image so out-of-range lanes can run the (convergent) code on a valid pixel.
__device__ __forceinline__ bool pixel_of(const FrameConst& F, int ya, int yb, int& x, int& y) {
    const int W = F.W;
    int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int bx, by;
    tile_of(F, ya, yb, bx, by);
    x = bx * 16 + (wave & 1) * 8 + (lane & 7);
    y = ya + by * 16 + (wave >> 1) * 8 + (lane >> 3);
    bool in = x < W && y < yb;
    x = x < W ? x : W - 1;
    y = y < yb ? y : yb - 1;
    return in;
}

// Intersection::testOcclusion (pg/Intersection.h:43-60): from the surface point, no normal offset
template <int T>
__device__ __forceinline__ bool occluded(const DevScene& S, const FrameConst& F, bool active, vec3 from, vec3 to,
                                         uint32_t& rays) {
    float dist = length(to - from);
    vec3 dir = normalize(to - from);
    rays += active ? 1u : 0u;
    return trace_any<T>(S, active, from, dir, FLT_MIN + F.tnear_off, dist - F.tfar_off);
}

// ReSTIRIntegrator::evaluateF (pg/ReSTIRIntegrator.cpp:185-211) for the lanes with `alive`.  The
// shadow ray is skipped when L_i*f_r*G is exactly zero in every channel (0 whatever V is).
// Split in two around the shadow ray so callers can batch several rays into one traversal:
// evaluate_f_pre computes the unoccluded L and the testOcclusion ray (dir = normalize(p - pos),
// tfar = |p - pos| - tfarOffset, exactly as occluded<T>() forms them); evaluate_f_post applies V.
struct FPre { vec3 L, dir; float tfar; bool ok, need; };
template <bool Call = false>
__device__ __forceinline__ FPre evaluate_f_pre(const FrameConst& F, const Sample& s, vec3 pos, bool emissive,
                                               const ShadeFrame& sf, bool test_vis, bool alive) {
    FPre r;
    r.ok = alive && smp_valid(s) && !emissive;
    vec3 ld = s.p - pos;
    float r2 = dot(ld, ld);
    ld = normalize(ld);
    float cI = gmax(dot(ld, sf.nrm), 0.0f);
    float cY = fabsf(dot(-ld, s.n));
    float G = cI * cY / r2;
    r.L = (s.li * eval_brdf<Call>(sf, ld)) * G;
    r.need = r.ok && test_vis && !(r.L.x == 0.0f && r.L.y == 0.0f && r.L.z == 0.0f);
    r.dir = ld;
    r.tfar = sqrtf(r2) - F.tfar_off;
    return r;
}
__device__ __forceinline__ FPre evaluate_f_pre(const FrameConst& F, const Sample& s, vec3 cam, const GElem& g,
                                               bool test_vis, bool alive) {
    return evaluate_f_pre(F, s, g.pos, g.le.x > 0 || g.le.y > 0 || g.le.z > 0, make_frame(g, cam), test_vis, alive);
}
__device__ __forceinline__ vec3 evaluate_f_post(const FPre& p, bool occ) {
    vec3 L = p.L;
    if (p.need) L = L * (float)(!occ);
    return p.ok ? L : mk(0, 0, 0);
}
template <int T>
__device__ __forceinline__ vec3 evaluate_f(const DevScene& S, const FrameConst& F, const Sample& s, vec3 pos,
                                           bool emissive, const ShadeFrame& sf, bool test_vis, bool alive,
                                           uint32_t& rays) {
    FPre p = evaluate_f_pre(F, s, pos, emissive, sf, test_vis, alive);
    bool occ = false;
    if (test_vis) {                                                   // test_vis is wave-uniform
        rays += p.need ? 1u : 0u;
        occ = trace_any<T>(S, p.need, pos, p.dir, FLT_MIN + F.tnear_off, p.tfar);
    }
    return evaluate_f_post(p, occ);
}
template <int T>
__device__ __forceinline__ vec3 evaluate_f(const DevScene& S, const FrameConst& F, const Sample& s, vec3 cam,
                                           const GElem& g, bool test_vis, bool alive, uint32_t& rays) {
    FPre p = evaluate_f_pre(F, s, cam, g, test_vis, alive);
    bool occ = false;
    if (test_vis) {                                                   // test_vis is wave-uniform
        rays += p.need ? 1u : 0u;
        occ = trace_any<T>(S, p.need, g.pos, p.dir, FLT_MIN + F.tnear_off, p.tfar);
    }
    return evaluate_f_post(p, occ);
}

// m_area / m_brdf (pg/ReSTIRIntegrator.h:62-74)
__device__ __forceinline__ float m_area(const FrameConst& F, float pa, float pb) {
    if (pa == 0.0f && pb == 0.0f) return 0.0f;
    return pa / ((float)F.m_area * pa + (float)F.m_brdf * pb);
}
__device__ __forceinline__ float m_brdf(const FrameConst& F, float pb, float pa) {
    if (pa == 0.0f && pb == 0.0f) return 0.0f;
    return pb / ((float)F.m_area * pa + (float)F.m_brdf * pb);
}

// gBufferFillPass (pg/ReSTIRIntegrator.cpp:213-234) + Camera::GenerateRay (pg/camera.cpp:20-42) for the
// camera `cam` (mat3(invViewMat) `m`): the current frame's, or the previous frame's when a tile rebuilds
// a G element its rows do not hold (k_temporal)
template <int T>
__device__ __forceinline__ GElem gbuffer_fill_cam(const DevScene& S, const FrameConst& F, const GCam& cam,
                                                  const float* m, int x, int y, bool active) {
    vec3 dc = mk((float)x - (float)F.W / 2.0f, (float)F.H / 2.0f - (float)y, -cam.focal);
    vec3 dw = mk(m[0] * dc.x + m[3] * dc.y + m[6] * dc.z, m[1] * dc.x + m[4] * dc.y + m[7] * dc.z,
                 m[2] * dc.x + m[5] * dc.y + m[8] * dc.z);
    dw = normalize(dw);
    SurfHit h = intersect<T>(S, active, cam.pos, dw, FLT_MIN + 0.01f);
    GElem g;
    g.pos = mk(0, 0, 0); g.nrm = g.pos; g.kd = g.pos; g.ks = g.pos; g.le = g.pos;
    g.shin = 0; g.depth = 0; g.type = 0; g.inv_im = 0;
    if (h.hit) {
        MatRec mr = load_mat(S, h.mat);
        vec3 nrm = h.normal;
        if (S.texd) apply_maps(S, h, mr, nrm, false);                // textured scenes only (uniform)
        g.pos = h.point; g.nrm = nrm; g.depth = length(h.point - cam.pos);
        g.type = mr.type; g.kd = mr.kd; g.ks = mr.ks; g.le = mr.le; g.shin = mr.shin;
        if (g.type == MT_PHONG || g.type == MT_DIELECTRIC) {
            vec3 V = normalize(cam.pos - g.pos);
#ifdef RS_DIAG_NO_IM   // timing diagnostic only (scripts/initial_breakdown.py); breaks parity
            g.inv_im = 1.0f + 0.0f * dot(V, g.nrm);
#else
            g.inv_im = 1.0f / calc_I_M(dot(V, g.nrm), g.shin);
#endif
        }
    } else {
        g.le = F.use_sky ? sky_texel(S, dw) : F.bg;      // useSkybox ? sky : renderParams.bgColor (:231)
    }
    return g;
}
template <int T>
__device__ __forceinline__ GElem gbuffer_fill(const DevScene& S, const FrameConst& F, int x, int y, bool active) {
    return gbuffer_fill_cam<T>(S, F, F.cam, F.inv_view, x, y, active);
}

// TriangleCDF::getTriangle's index (pg/TriangleCDF.cpp:36-54): std::lower_bound(cdf2, ksi), narrowed
// by the guide table: ksi*kCdfGuide is exact (ksi = k*2^-24), and lower_bound(j/G) <= lower_bound(ksi)
// <= lower_bound((j+1)/G) for j = floor(ksi*G)
__device__ __forceinline__ uint32_t light_index(const DevScene& S, float ksi) {
    uint32_t j = (uint32_t)(ksi * (float)kCdfGuide);
    uint32_t lo = (uint32_t)S.cdf_guide[j], n = (uint32_t)S.cdf_guide[j + 1] + 1u - lo;
    if (lo + n > S.n_emis) n = S.n_emis - lo;
    while (n > 0) {
        uint32_t h = n >> 1;
        if (S.cdf[lo + h] < ksi) { lo = lo + h + 1; n = n - h - 1; } else n = h;
    }
    return lo < S.n_emis ? lo : S.n_emis - 1;
}

// the emissive-triangle pick of candidate c alone (its first RNG slot): the CDF search is a chain of
// dependent loads, so the initial pass issues the next batch's picks before the current batch's walk
__device__ __forceinline__ uint32_t area_pick(const DevScene& S, const Rng& rng, int c) {
    Rng q = rng;
    q.n = cand_slot(c);
    return light_index(S, q.range(0.0f, 1.0f));
}
// An emissive triangle's record, 8 float4 (one 128-B line):
//   e0 (p0, pdf_area)  e1 (p1, n0.x)  e2 (p2, n0.y)  e3 (le, n0.z)
//   e4 (n1, pick)      e5 (n2, pdf_brdf)  e6 (area, inv_area, 0, 0)  e7 unused
// pdf_area = pick * inv_area (TriangleCDF pick probability x 1/area, the product areaSampleLight forms),
// its sign bit set when the vertex normals differ.  An area sample of a flat emitter (all vertex normals
// equal -- every quad light) reads e0..e3 only: 4 loads instead of 7 per candidate, the light-table
// gathers being ~18 % of the C2 initial pass.  A flat emitter's n1 = n2 = n0 bit for bit, so the
// interpolated normal is computed with the same operands either way.
struct EmisRec {
    vec3 p0, p1, p2, n0, n1, n2, le;
    float pdf_area;
    __device__ __forceinline__ static EmisRec load(const float4* E) {
        const float4 a = E[0], b = E[1], c = E[2], d = E[3];
        EmisRec r;
        r.p0 = xyz(a); r.p1 = xyz(b); r.p2 = xyz(c); r.le = xyz(d);
        r.n0 = mk(b.w, c.w, d.w);
        r.n1 = r.n0; r.n2 = r.n0;
        if (__float_as_uint(a.w) >> 31) { r.n1 = xyz(E[4]); r.n2 = xyz(E[5]); }
        r.pdf_area = fabsf(a.w);
        return r;
    }
};
__device__ __forceinline__ float emis_pdf_brdf(const DevScene& S, int id) { return S.emis[8 * id + 5].w; }

// areaSampleLight (pg/ReSTIRIntegrator.cpp:89-124), TriangleCDF::getTriangle (pg/TriangleCDF.cpp:36-54),
// Sampling::sampleTriangle (pg/Sampling.cpp:63-76)
template <bool Call = false>
__device__ __forceinline__ Sample area_sample_at(const DevScene& S, const FrameConst& F, vec3 pos, const ShadeFrame& sf,
                                                 Rng& rng, uint32_t idx, float& W_out, float& mis_out) {
    const EmisRec E = EmisRec::load(S.emis + 8 * idx);
    float r1 = rng.range(0, 1), r2 = rng.range(0, 1);
    float sr = sqrtf(r1);
    float bx = 1.0f - sr, by = sr * (1.0f - r2), bz = sr * r2;
    vec3 pt = (E.p0 * bx + E.p1 * by) + E.p2 * bz;
    vec3 nn = normalize((E.n0 * bx + E.n1 * by) + E.n2 * bz);
    float pdf_area = E.pdf_area;            // pick prob * (1 / area)
    vec3 ld = pt - pos;
    float r2s = dot(ld, ld);
    ld = normalize(ld);
    float cY = gmax(dot(-ld, nn), 0.0f);
    float amf = cY / r2s;
    float pba = phong_pdf<Call>(sf, ld) * amf;
    mis_out = m_area(F, pdf_area, pba);
    W_out = 1.0f / pdf_area;
    return Sample{pt, nn, E.le};
}
__device__ __forceinline__ Sample area_sample(const DevScene& S, const FrameConst& F, vec3 pos, const ShadeFrame& sf,
                                              Rng& rng, float& W_out, float& mis_out) {
    const uint32_t idx = light_index(S, rng.range(0.0f, 1.0f));
    return area_sample_at(S, F, pos, sf, rng, idx, W_out, mis_out);
}

// brdfSampleLight (pg/ReSTIRIntegrator.cpp:126-177)
template <int T>
__device__ __forceinline__ Sample brdf_sample(const DevScene& S, const FrameConst& F, vec3 pos, const ShadeFrame& sf,
                                              bool alive, Rng& rng, float& W_out, float& mis_out, uint32_t& rays) {
    float pdf;
    vec3 wi = sample_brdf(sf, rng, pdf);
    vec3 org = pos + sf.nrm * F.normal_off;
    rays += alive ? 1u : 0u;
    // BRDF-sampled directions are incoherent across a tile even when shadow rays are not: the
    // per-lane walk beats the lockstep union for them in either kind (C2: +3 %)
    SurfHit h = intersect<T | TRAV_LANE>(S, alive, org, wi, FLT_MIN + F.tnear_off);
    W_out = 0.0f; mis_out = 0.0f;
    if (h.hit) {
        MatRec mr = load_mat(S, h.mat);
        if (mr.le.x + mr.le.y + mr.le.z > 0) {      // Material::isEmissive (pg/material.h:135-137)
            vec3 hn = h.normal;
            if (S.texd) apply_maps(S, h, mr, hn, true);                // a normal-mapped emitter
            vec3 ld = h.point - pos;
            float r2s = dot(ld, ld);
            ld = normalize(ld);
            float cY = gmax(dot(-ld, hn), 0.0f);
            float amf = cY / r2s;
            float pdf_area = emis_pdf_brdf(S, h.emis_id);   // getPDFForTriangle (pg/TriangleCDF.h:25-31)
            float bpa = pdf * amf;
            W_out = 1.0f / bpa;
            mis_out = m_brdf(F, bpa, pdf_area);
            return Sample{h.point, hn, mr.le};
        }
    }
    return smp_invalid();
}

// The initial pass keeps its pixel's ShadeFrame in LDS (5 float4 per thread, component-major so a
// wave's ds_read_b128 of one component is conflict-free) and re-reads it for every candidate batch:
// the ~20 per-pixel invariants then occupy no VGPRs across the shadow-ray walks (the compiler barrier
// in load() keeps LICM from hoisting the reads back out of the candidate loop).  256 threads x 80 B =
// 20 KB per workgroup.
struct FrameSlot {
    float4* base;   // __shared__ float4[5 * n] (+ n more for the split kernel's (pos, alive))
    int t, n;       // this thread's entry, entries per component (compile-time at every use)
    __device__ __forceinline__ void store(const ShadeFrame& s) const {
        base[t] = f4(s.nrm, s.pf);
        base[n + t] = f4(s.wr, s.omp);
        base[2 * n + t] = f4(s.kd_pi, s.shin);
        base[3 * n + t] = f4(s.ks_im, s.a);
        base[4 * n + t] = make_float4(s.maxD, s.maxS, __int_as_float(s.type), 0.0f);
    }
    __device__ __forceinline__ ShadeFrame load() const {
        asm volatile("" ::: "memory");
        const float4 a = base[t], b = base[n + t], c = base[2 * n + t], d = base[3 * n + t], e = base[4 * n + t];
        ShadeFrame s;
        s.nrm = xyz(a); s.pf = a.w; s.wr = xyz(b); s.omp = b.w; s.kd_pi = xyz(c); s.shin = c.w;
        s.ks_im = xyz(d); s.a = d.w; s.maxD = e.x; s.maxS = e.y; s.type = __float_as_int(e.z);
        return s;
    }
};

// One batch of area candidates [c0, c0 + kB) (initialRenderPass :246-266): sample, unoccluded f, one
// walk for the batch's shadow rays; returns each candidate's RIS weight w in w_out.  Only two weights per
// candidate stay live across the walk -- the unoccluded one and the occluded one, (m * 0) * W -- instead
// of the sample, f, MIS weight and W: an occluded (or invalid) candidate has f = 0 and p-hat = 0, which
// both produce bit for bit.  (The selected candidate's f is re-derived from its re-drawn sample.)
template <int T, int kB>
__device__ __forceinline__ void area_batch(const DevScene& S, const FrameConst& F, vec3 pos, const ShadeFrame& sf,
                                           Rng& rng, int c0, int c_end, bool alive, bool tv, const uint32_t* pick,
                                           float* w_out, uint32_t& rays) {
    float wu[kB], wo[kB];
    bool act[kB], okb[kB], occ[kB];
    vec3 dir[kB];
    float tf[kB];
    const float inv_ma = 1.0f / (float)F.m_area;
#pragma unroll
    for (int k = 0; k < kB; ++k) {
        float Wc, mis;
        rng.n = cand_slot(c0 + k) + 1u;                 // slot +0 was the pick (area_pick)
        const Sample s = area_sample_at(S, F, pos, sf, rng, pick[k], Wc, mis);
        const FPre p = evaluate_f_pre(F, s, pos, false, sf, tv, alive && c0 + k < c_end);
        const float ph = length(p.L);
        const float m = F.m_brdf > 0 ? mis : inv_ma;
        wu[k] = m * ph * Wc;
        wo[k] = m * 0.0f * Wc;
        act[k] = p.need; okb[k] = p.ok; dir[k] = p.dir; tf[k] = p.tfar; occ[k] = false;
        rays += act[k] ? 1u : 0u;
    }
    if (tv) trace_any_multi<T, kB>(S, act, pos, dir, FLT_MIN + F.tnear_off, tf, occ);
#pragma unroll
    for (int k = 0; k < kB; ++k) w_out[k] = (okb[k] && !(act[k] && occ[k])) ? wu[k] : wo[k];   // evaluate_f_post
}
// the selected area candidate's sample and (unoccluded) f, re-drawn from its RNG slots
__device__ __forceinline__ Sample area_redraw(const DevScene& S, const FrameConst& F, vec3 pos, const ShadeFrame& sf,
                                             Rng& rng, int c, bool tv, vec3& f) {
    float Wc, mis;
    rng.n = cand_slot(c);
    const Sample s = area_sample(S, F, pos, sf, rng, Wc, mis);
    f = evaluate_f_pre(F, s, pos, false, sf, tv, true).L;
    return s;
}

// initialRenderPass (pg/ReSTIRIntegrator.cpp:236-298) for the lanes with `in_pass`.  f_sel returns the
// selected candidate's f (for the fused shade); the final p-hat (:289) equals the selected candidate's
// p-hat (same arguments), so it is not re-evaluated.
template <int T>
__device__ __forceinline__ Res initial_ris(const DevScene& S, const FrameConst& F, vec3 pos, bool emissive,
                                           FrameSlot fs, uint32_t pix, bool in_pass, vec3& f_sel, uint32_t& rays) {
    f_sel = mk(0, 0, 0);
    Res r = res_empty();
    const bool alive = in_pass && !emissive && S.n_emis > 0;           // :238-244
    if (__ballot(alive) == 0) return r;                                 // wave-uniform exit
    Rng rng; rng.init(F.seed, F.frame, PASS_INITIAL, pix);
    const bool tv = !F.do_vis_pass;
    constexpr int kB = trav_lane(T) ? RS_RIS_BATCH_LANE : RS_RIS_BATCH;
    float best_phat = 0.0f;
    if (F.m_area > 0) {
        // area candidates in batches of kB (area_batch: one walk per batch), then the reservoir updates
        // in candidate order.  The selected sample and its f are re-drawn from its slots once at the end
        // instead of being carried per candidate (a selected candidate has w > 0: unoccluded, f = L).
        int sel = -1;
        uint32_t pick[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) pick[k] = area_pick(S, rng, k);
        for (int c0 = 0; c0 < F.m_area; c0 += kB) {
            float w[kB];
            uint32_t next[kB];
#pragma unroll
            for (int k = 0; k < kB; ++k) next[k] = area_pick(S, rng, c0 + kB + k);   // in flight during the walk
            area_batch<T, kB>(S, F, pos, fs.load(), rng, c0, F.m_area, alive, tv, pick, w, rays);
#pragma unroll
            for (int k = 0; k < kB; ++k) pick[k] = next[k];
#pragma unroll
            for (int k = 0; k < kB; ++k) {
                if (c0 + k < F.m_area) {
                    rng.n = cand_slot(c0 + k) + 3u;
                    if (alive && res_add_w(r, w[k], 0, rng)) sel = c0 + k;
                }
            }
        }
        if (sel >= 0) {
            const Sample s = area_redraw(S, F, pos, fs.load(), rng, sel, tv, f_sel);
            best_phat = length(f_sel);
            r.p = s.p; r.n = s.n; r.li = s.li;
        }
    }
    if (F.m_brdf > 0) {
        float inv_mb = 1.0f / (float)F.m_brdf;
        for (int i = 0; i < F.m_brdf; ++i) {
            float Wc, mis;
            rng.n = cand_slot(F.m_area + i);
            const ShadeFrame sf = fs.load();
            Sample s = brdf_sample<T>(S, F, pos, sf, alive, rng, Wc, mis, rays);
            vec3 f = evaluate_f<T>(S, F, s, pos, false, sf, tv, alive, rays);
            float ph = length(f);
            float w = F.m_area > 0 ? mis * ph * Wc : inv_mb * ph * Wc;
            rng.n = cand_slot(F.m_area + i) + 3u;
            if (alive && res_add(r, s, w, 0, rng)) { best_phat = ph; f_sel = f; }
        }
    }
    if (!alive) { f_sel = mk(0, 0, 0); return res_empty(); }
    // every candidate adds confidence 1 (Reservoir::addSample, pg/Reservoir.h:35): counted here, not
    // carried through the candidate loops (one register less across every shadow walk)
    r.conf = F.m_area + F.m_brdf;
    float ph = smp_valid(smp_of(r)) ? best_phat : 0.0f;
    r.W = ph > 0.0f ? 1.0f / ph * r.wsum : 0.0f;
    res_cap(r, F.cap);
    return r;
}

// shade of one pixel (pg/simpleguidx11.cpp:456-468) given the reservoir's f (already visibility-tested)
__device__ __forceinline__ vec3 shade_px(const Res& r, vec3 f, vec3 le) {
    vec3 px = r.wsum > 0.0f ? f * r.W : le;   // Reservoir::hasSample (pg/Reservoir.h:49-52)
    return sanitize(px);
}
__device__ __forceinline__ void store_rgb(float* fb, size_t p, vec3 c) {
    fb[3 * p] = c.x; fb[3 * p + 1] = c.y; fb[3 * p + 2] = c.z;
}

// ---------------------------------------------------------------- persistent waves (per-wave tile queue)
// A persistent launch has about one device's worth of resident workgroups; every WAVE pulls 8x8-pixel tiles from a
// per-launch counter (one atomic per tile, lane 0) in the order a full grid would dispatch them -- the 4 waves of a
// 16x16 tile in a row, the tile rows costliest first (tile_of) -- until the queue is empty.  A wave that finishes its
// tile takes the next one at once, where a one-thread-per-pixel grid keeps a workgroup's four wave slots until its
// slowest wave retires.  Counter words: [0] next tile, [1] waves exited; the last wave to exit re-arms both for the
// lane's next launch.  Every pixel's work is independent of which wave does it: frames are bit-identical.
struct TileQ { uint32_t* ctr; uint32_t n; };
__device__ __forceinline__ uint32_t q_pull(const TileQ& Q) {
    uint32_t t = 0u;
    if ((threadIdx.x & 63) == 0) t = atomicAdd(Q.ctr, 1u);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
}
__device__ __forceinline__ void q_exit(const TileQ& Q) {
    if ((threadIdx.x & 63) != 0) return;
    const uint32_t waves = gridDim.x * gridDim.y * (blockDim.x >> 6);
    if (__hip_atomic_fetch_add(Q.ctr + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == waves - 1) {
        __hip_atomic_store(Q.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(Q.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// 8x8 tile t of rows [ya, yb) in dispatch order (4 per 16x16 tile, 16-px rows by the context's cost order on full frames)
__device__ __forceinline__ bool pixel_of_q(const FrameConst& F, int ya, int yb, uint32_t t, int& x, int& y) {
    const int W = F.W, gx = (W + 15) / 16, gy = (yb - ya + 15) / 16;
    const int q = (int)(t >> 2), w = (int)(t & 3u);
    const int bx = q % gx;
    int by = q / gx;
    if (F.row_order && ya == 0 && yb == F.H && F.n_order == gy) by = order_row(F.row_order, (uint32_t)by);
    const int lane = threadIdx.x & 63;
    x = bx * 16 + (w & 1) * 8 + (lane & 7);
    y = ya + by * 16 + (w >> 1) * 8 + (lane >> 3);
    const bool in = x < W && y < yb;
    x = x < W ? x : W - 1;
    y = y < yb ? y : yb - 1;
    return in;
}
// the unclamped origin of 8x8 tile t (pixel_of_q's layout)
__device__ __forceinline__ void tile_origin_q(const FrameConst& F, int ya, int yb, uint32_t t, int& tx0, int& ty0) {
    const int gx = (F.W + 15) / 16, gy = (yb - ya + 15) / 16;
    const int q = (int)(t >> 2), w = (int)(t & 3u);
    const int bx = q % gx;
    int by = q / gx;
    if (F.row_order && ya == 0 && yb == F.H && F.n_order == gy) by = order_row(F.row_order, (uint32_t)by);
    tx0 = bx * 16 + (w & 1) * 8;
    ty0 = ya + by * 16 + (w >> 1) * 8;
}
// count_rays for a persistent wave: the slot of this wave once at the end; the per-row cost per tile
__device__ __forceinline__ void count_store(CountSlot C, uint32_t rays, uint32_t primary) {
    const uint32_t r = wave_sum(rays), p = wave_sum(primary);
    if ((threadIdx.x & 63) == 0)
        C.part[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)] = make_uint2(r, p);
}

// G-buffer + initialRenderPass of one pixel (the body of k_gbuffer_initial)
template <int T>
__device__ __forceinline__ void gbuffer_initial_px(const DevScene& S, const FrameConst& F, const GBuf& G, const ResBuf& Rw,
                                                   float* fb, int fuse_shade, const FrameSlot& fs, int x, int y, bool in,
                                                   uint32_t& rays) {
    const size_t p = (size_t)y * F.W + x;
    GElem g = gbuffer_fill<T>(S, F, x, y, in);
    if (in) G.store(p, g);
    fs.store(make_frame(g, F.cam.pos));
    const bool ris = in && y >= F.y0 && y < F.y1;
    vec3 f;
    Res r = initial_ris<T>(S, F, g.pos, any_pos(g.le), fs, (uint32_t)p, ris, f, rays);
    if (ris) {
        Rw.store(p, r);
        if (fuse_shade) store_rgb(fb, p, shade_px(r, f, g.le));
    }
}
template <int T>
__global__ void __launch_bounds__(256, RS_WAVES(T, RS_INITIAL_WAVES, RS_INITIAL_WAVES_LANE)) k_gbuffer_initial(DevScene S, FrameConst F, GBuf G,
                                                                            ResBuf Rw, float* fb, int fuse_shade,
                                                                            CountSlot C) {
    const uint64_t t0 = wave_clock();
    if ((blockIdx.x | blockIdx.y | threadIdx.x) == 0) *C.outside = 0ull;   // this frame's counter (rs_tile_begin)
    int x, y;
    uint32_t rays = 0;
    const bool in = pixel_of(F, F.gy0, F.gy1, x, y);
    __shared__ float4 frame_lds[5 * 256];
    const FrameSlot fs{frame_lds, (int)threadIdx.x, 256};
    gbuffer_initial_px<T>(S, F, G, Rw, fb, fuse_shade, fs, x, y, in, rays);
    count_rays(C, rays + (in ? 1u : 0u), in ? 1u : 0u, t0, y);
}
// ---------------------------------------------------------------- wave-sorted initial pass (per-lane wide walks)
// The per-lane walks of incoherent scenes (C3) are bound by the vector-memory data path returning a wave's
// divergent node loads (TD busy 0.92): every load instruction touches as many cache lines as its lanes visit
// distinct nodes.  Lane = pixel and candidate by candidate, a wave's 64 shadow rays aim at 64 random lights.
// This kernel regroups them: per chunk of kSortChunk area candidates a wave (an 8x8 pixel tile)
//   A  samples each candidate of its 64 pixels (lane = pixel): a needed shadow ray (its slot = candidate,
//      pixel) takes a rank in one of 64 buckets by its light (S.ebucket: the Morton order of the emitter
//      centroids; one LDS atomic), and its light and rank are kept in the slot's LDS word;
//   then a 64-lane scan turns the bucket counts into offsets and every slot index is scattered to its place:
//      the chunk's rays are in LDS bucket by bucket (a counting sort);
//   B  traces them 64 at a time in that order (lane = ray): each lane re-forms its ray from the slot -- the
//      pixel's surface point from LDS, the candidate's RNG draws, the light record -- with the operations
//      area_sample_at / evaluate_f_pre use, so it is bit for bit the ray the pixel would trace, walks the
//      tree (per lane: the 8-wide tree; lockstep: the wave steps through the union of its rays' binary
//      paths, which the grouping shrinks) and sets the pixel's occlusion bit;
//   C  re-draws each candidate (lane = pixel) for its RIS weight and runs the reference's addSample stream
//      over the chunk in candidate order.  (Re-drawing costs one more sampling pass; keeping the weights
//      would take 4 B per slot of LDS and cost occupancy.)
// Rays aimed at neighbouring lights share their upper tree paths, so a load instruction touches fewer lines
// (CPU lab, scripts/bvh_lab.cpp COHERENCE_WAVE, C3: distinct node fetches per wave -39 %, lockstep steps
// -13 % for 32 candidates in 64 buckets).  The results do not depend on the order rays are traced in:
// frames are bit-identical to k_gbuffer_initial (tests/test_gpu_parity.py).
#ifndef RS_SORT_CHUNK
#define RS_SORT_CHUNK 16
#endif
#ifndef RS_INITIAL_WAVES_SORT
#define RS_INITIAL_WAVES_SORT 5              // per-lane walks (LDS: 29 KB per workgroup -> 5 workgroups per CU)
#endif
#ifndef RS_INITIAL_WAVES_SORT_LOCKSTEP
#define RS_INITIAL_WAVES_SORT_LOCKSTEP 5
#endif
constexpr int kSortChunk = RS_SORT_CHUNK;   // area candidates per sort round
// Phase A's unoccluded candidate weights kept for phase C in global memory (one coalesced 256-B store and load
// per candidate and wave: FrameConst::cand_w) instead of phase C drawing every candidate again (its light pick, the
// emitter record gathers, the sample, both Phong powf).  The region is the wave's hand-off slot: its resident wave
// slot in the persistent launch (reused tile after tile, so the few MB stay in the caches), its 8x8 tile in a
// one-launch grid (restir_capi.hip ensure_handoff sizes both by the launch)
#ifndef RS_SORT_STORE_W
#define RS_SORT_STORE_W 1
#endif
static_assert(!RS_SORT_STORE_W || kSortChunk <= 16, "ok and NaN bits of a chunk share one word");
// ... and the needed shadow rays' (direction, tfar) for phase B (one 16-B load per ray instead of re-forming it
// from the candidate's RNG slots and the emitter's three vertices)
#ifndef RS_SORT_STORE_RAY
#define RS_SORT_STORE_RAY 1
#endif
static_assert(kSortChunk >= 1 && kSortChunk <= 32, "one occlusion word per pixel; 11-bit ranks");
struct SortLds {                            // one wave's region (7.3 KB at 16 candidates)
    uint32_t slot[kSortChunk * 64];         // slot k * 64 + lane: light | rank in its bucket << 21
    uint16_t e[kSortChunk * 64];            // the slots of the chunk's rays, bucket by bucket
    uint32_t cur[64];                       // bucket counts, then bucket offsets
    uint32_t occ[64];                       // per pixel: the chunk's occlusion bits
    float px[64], py[64], pz[64];           // per pixel: its surface point
};
// cross-lane LDS hand-off inside one wave: LDS requests of a wave complete in order, so a fence against
// compiler reordering is all that is needed
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
// the pixel index of lane `l` of this thread's wave tile (pixel_of's layout, unclamped)
__device__ __forceinline__ uint32_t tile_pixel(const FrameConst& F, int ya, int yb, int l) {
    int bx, by;
    tile_of(F, ya, yb, bx, by);
    const int wave = threadIdx.x >> 6;
    const int x = bx * 16 + (wave & 1) * 8 + (l & 7), y = ya + by * 16 + (wave >> 1) * 8 + (l >> 3);
    return (uint32_t)y * (uint32_t)F.W + (uint32_t)x;
}
// the bucket of a shadow ray: RS_SORT_KEY 0 = the light's Morton bucket alone; 1 (default since round 6) = the
// direction's octant x the top 3 bits of the light's Morton bucket (CPU lab, scripts/bvh_lab.cpp COHERENCE_WAVE, 32
// candidates: light bucket alone -- C3 wide-walk distinct fetches -39 %, C2 binary lockstep union -6 %; octant x
// light 3 bits -- C3 -30 %, C2 -45 %.  GPU, C3 1080p, round 4: initial pass 14.97 vs 15.14 ms; round 6 with the
// lane refill: 75.35-75.72 vs 75.11-75.39 frames/s, initial pass 11.88-11.94 vs 11.95-11.99 ms)
#ifndef RS_SORT_KEY
#define RS_SORT_KEY 1
#endif
__device__ __forceinline__ uint32_t ray_bucket(const DevScene& S, uint32_t pick, vec3 d) {
    const uint32_t eb = S.ebucket[pick];
    if (RS_SORT_KEY == 0) return eb;
    const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    return (oct << 3) | (eb >> 3);
}
// candidate c of a pixel: area_batch's sample and unoccluded evaluation (pick, weights, shadow ray need)
struct AreaCand { uint32_t pick, bucket; float wu; bool ok, need, wo_nan; vec3 dir; float tfar; };
// (the sorted pass's candidates take the pow core by call: RS_SORT_POW_CALL, C3 +2 %)
#ifndef RS_SORT_POW_CALL
#define RS_SORT_POW_CALL 1
#endif
__device__ __forceinline__ AreaCand area_cand(const DevScene& S, const FrameConst& F, vec3 pos, const ShadeFrame& sf,
                                              Rng& rng, int c, bool tv, bool alive, float inv_ma) {
    AreaCand a;
    a.pick = area_pick(S, rng, c);
    float Wc, mis;
    rng.n = cand_slot(c) + 1u;
    const Sample s = area_sample_at<RS_SORT_POW_CALL>(S, F, pos, sf, rng, a.pick, Wc, mis);
    const FPre pr = evaluate_f_pre<RS_SORT_POW_CALL>(F, s, pos, false, sf, tv, alive);
    a.bucket = ray_bucket(S, a.pick, pr.dir);
    const float m = F.m_brdf > 0 ? mis : inv_ma;
    a.wu = m * length(pr.L) * Wc;
    const float wo = m * 0.0f * Wc;             // +-0 (the same reservoir update) or NaN
    a.wo_nan = wo != wo;
    a.ok = pr.ok;
    a.need = pr.need;
    a.dir = pr.dir;
    a.tfar = pr.tfar;
    return a;
}

// the sorted kernel's reservoir state around its BRDF candidates' walks: 14 words per lane in the wave's
// slot[] region (word c at c * 64 + lane: conflict-free)
#ifndef RS_SORT_PARK
#define RS_SORT_PARK 1
#endif
static_assert(kSortChunk >= 14 || !RS_SORT_PARK, "brdf_park needs 14 slot words per lane");
__device__ __forceinline__ void brdf_park(uint32_t* sl, int lane, const Res& r, float bp, vec3 fs) {
    const float v[14] = {r.p.x, r.p.y, r.p.z, r.n.x, r.n.y, r.n.z, r.li.x, r.li.y, r.li.z, r.wsum, bp, fs.x, fs.y, fs.z};
#pragma unroll
    for (int c = 0; c < 14; ++c) sl[c * 64 + lane] = __float_as_uint(v[c]);
}
__device__ __forceinline__ void brdf_unpark(const uint32_t* sl, int lane, Res& r, float& bp, vec3& fs) {
    float v[14];
#pragma unroll
    for (int c = 0; c < 14; ++c) v[c] = __uint_as_float(sl[c * 64 + lane]);
    r.p = mk(v[0], v[1], v[2]); r.n = mk(v[3], v[4], v[5]); r.li = mk(v[6], v[7], v[8]); r.wsum = v[9];
    bp = v[10]; fs = mk(v[11], v[12], v[13]);
}
// one wave's 8x8 tile of the sorted pass: lane = pixel (x, y) (clamped; `in` whether it exists), the tile's
// unclamped origin (tx0, ty0) for the pixel index of a ray's source lane, the wave's LDS region L, its hand-off slot
template <int T>
__device__ __forceinline__ void sorted_tile(const DevScene& S, const FrameConst& F, const GBuf& G, const ResBuf& Rw,
                                            float* fb, int fuse_shade, SortLds& L, int lane, int x, int y, bool in,
                                            int tx0, int ty0, size_t hslot, uint32_t& rays) {
    const size_t p = (size_t)y * F.W + x;
    {
        const GElem g = gbuffer_fill<T>(S, F, x, y, in);
        if (in) G.store(p, g);
        L.px[lane] = g.pos.x; L.py[lane] = g.pos.y; L.pz[lane] = g.pos.z;
    }
    const bool ris = in && y >= F.y0 && y < F.y1;
    const vec3 cam = F.cam.pos;
    Res r = res_empty();
    vec3 f_sel = mk(0, 0, 0);
    // (the G element is re-read where it is needed: nothing of it stays live across the walks)
    const bool alive = ris && !any_pos(G.load(p).le) && S.n_emis > 0;          // :238-244
    if (__ballot(alive) != 0) {
        Rng rng; rng.init(F.seed, F.frame, PASS_INITIAL, (uint32_t)p);
        const bool tv = !F.do_vis_pass;
        float best_phat = 0.0f;
        if (F.m_area > 0) {
            int sel = -1;
            const float inv_ma = 1.0f / (float)F.m_area;
            for (int c0 = 0; c0 < F.m_area; c0 += kSortChunk) {
                const int nk = F.m_area - c0 < kSortChunk ? F.m_area - c0 : kSortChunk;
                // ---- A: the chunk's samples (lane = pixel); needed rays take a rank in their light's bucket
                L.cur[lane] = 0u;
                L.occ[lane] = 0u;
                wave_lds_sync();
                uint32_t needm = 0u;
                uint32_t bkt[(kSortChunk + 3) / 4] = {};                // the needed rays' buckets, 8 bits each
                const size_t wtile = hslot;
#if RS_SORT_STORE_W
                uint32_t flg = 0u;                                      // bit k: ok; bit 16 + k: its occluded weight is NaN
                float* const wst = F.cand_w + wtile * (size_t)(kSortChunk * 64) + lane;
#endif
                {
                    const GElem g = G.load(p);
                    const ShadeFrame sf = make_frame(g, cam);
                    for (int k = 0; k < nk; ++k) {
                        const AreaCand a = area_cand(S, F, g.pos, sf, rng, c0 + k, tv, alive, inv_ma);
#if RS_SORT_STORE_W
                        wst[k * 64] = a.wu;
                        flg |= (a.ok ? 1u << k : 0u) | (a.wo_nan ? 1u << (16 + k) : 0u);
#endif
                        if (a.need) {
#if RS_SORT_STORE_RAY
                            F.cand_ray[wtile * (size_t)(kSortChunk * 64) + (size_t)(k * 64 + lane)] = f4(a.dir, a.tfar);
#endif
                            const uint32_t rank = atomicAdd(&L.cur[a.bucket], 1u);
                            L.slot[k * 64 + lane] = a.pick | (rank << 21);
                            bkt[k >> 2] |= a.bucket << (8 * (k & 3));
                            needm |= 1u << k;
                        }
                    }
                }
                wave_lds_sync();
                const uint32_t cnt = L.cur[lane];                       // lane = bucket: exclusive scan
                uint32_t incl = cnt;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t v = __shfl_up(incl, o);
                    incl += lane >= o ? v : 0u;
                }
                const uint32_t n_rays = __shfl(incl, 63);
                L.cur[lane] = incl - cnt;
                wave_lds_sync();
#pragma unroll
                for (int k = 0; k < kSortChunk; ++k)
                    if ((needm >> k) & 1u) {
                        const uint32_t b = (bkt[k >> 2] >> (8 * (k & 3))) & 0xffu;
                        L.e[L.cur[b] + (L.slot[k * 64 + lane] >> 21)] = (uint16_t)(k * 64 + lane);
                    }
                wave_lds_sync();
                // ---- B: the chunk's shadow rays in bucket order (lane = ray)
#if RS_SORT_STORE_RAY
                if constexpr (trav_lane(T) && trav_wide(T)) {          // lanes refilled from the list (rs_scene.h)
                    occluded_wide_list(S, n_rays, FLT_MIN + F.tnear_off,
                        [&](uint32_t j, vec3& o, vec3& ld, float& tfar) {
                            const uint32_t sl = L.e[j], src = sl & 63u;
                            o = mk(L.px[src], L.py[src], L.pz[src]);
                            const float4 dt = F.cand_ray[wtile * (size_t)(kSortChunk * 64) + sl];   // phase A's ray
                            ld = xyz(dt);
                            tfar = dt.w;
                            rays += 1u;
                        },
                        [&](uint32_t j, bool occ) {
                            const uint32_t sl = L.e[j];
                            if (occ) atomicOr(&L.occ[sl & 63u], 1u << (sl >> 6));
                        });
                } else
#endif
                for (uint32_t j0 = 0; j0 < n_rays; j0 += 64u) {
                    const uint32_t j = j0 + (uint32_t)lane;
                    const bool act = j < n_rays;
                    const uint32_t sl = L.e[act ? j : 0u];
                    const uint32_t pick = L.slot[sl] & 0x1fffffu, k = sl >> 6, src = sl & 63u;
                    const vec3 o = mk(L.px[src], L.py[src], L.pz[src]);
#if RS_SORT_STORE_RAY
                    (void)pick;
                    const float4 dt = F.cand_ray[wtile * (size_t)(kSortChunk * 64) + sl];   // phase A's evaluate_f_pre ray
                    const vec3 ld = xyz(dt);
                    const float tfar = dt.w;
#else
                    Rng q;
                    q.init(F.seed, F.frame, PASS_INITIAL,
                           (uint32_t)(ty0 + (int)(src >> 3)) * (uint32_t)F.W + (uint32_t)(tx0 + (int)(src & 7u)));
                    q.n = cand_slot(c0 + (int)k) + 1u;
                    const float r1 = q.range(0, 1), r2 = q.range(0, 1);    // area_sample_at's draws
                    const float4* E = S.emis + 8 * (size_t)pick;
                    const vec3 p0 = xyz(E[0]), p1 = xyz(E[1]), p2 = xyz(E[2]);
                    const float sr = sqrtf(r1);
                    const float bx = 1.0f - sr, by = sr * (1.0f - r2), bz = sr * r2;
                    const vec3 pt = (p0 * bx + p1 * by) + p2 * bz;
                    vec3 ld = pt - o;                                        // evaluate_f_pre's ray
                    const float r2s = dot(ld, ld);
                    ld = normalize(ld);
                    const float tfar = sqrtf(r2s) - F.tfar_off;
#endif
                    const bool occ = trace_any<T>(S, act, o, ld, FLT_MIN + F.tnear_off, tfar);
                    rays += act ? 1u : 0u;
                    if (act && occ) atomicOr(&L.occ[src], 1u << k);
                }
                wave_lds_sync();
                // ---- C: phase A's weights, the reservoir stream in candidate order (lane = pixel)
                const uint32_t occm = L.occ[lane];
#if RS_SORT_STORE_W
                for (int k = 0; k < nk; ++k) {
                    const int c = c0 + k;
                    const bool use_u = ((flg >> k) & 1u) && !(((needm & occm) >> k) & 1u);
                    const float w = use_u ? wst[k * 64] : (((flg >> (16 + k)) & 1u) ? __int_as_float(0x7fc00000) : 0.0f);
                    rng.n = cand_slot(c) + 3u;
                    if (alive && res_add_w(r, w, 0, rng)) sel = c;
                }
#else
                const GElem g = G.load(p);
                const ShadeFrame sf = make_frame(g, cam);
                for (int k = 0; k < nk; ++k) {
                    const int c = c0 + k;
                    const AreaCand a = area_cand(S, F, g.pos, sf, rng, c, tv, alive, inv_ma);
                    const bool use_u = a.ok && !(a.need && ((occm >> k) & 1u));
                    const float w = use_u ? a.wu : (a.wo_nan ? __int_as_float(0x7fc00000) : 0.0f);
                    rng.n = cand_slot(c) + 3u;
                    if (alive && res_add_w(r, w, 0, rng)) sel = c;
                }
#endif
            }
            if (sel >= 0) {
                const GElem g = G.load(p);
                const Sample s = area_redraw(S, F, g.pos, make_frame(g, cam), rng, sel, tv, f_sel);
                best_phat = length(f_sel);
                r.p = s.p; r.n = s.n; r.li = s.li;
            }
        }
        if (F.m_brdf > 0) {
            // the BRDF candidates' two walks (closest hit, then the shadow ray) run with the reservoir state
            // parked in this wave's LDS (slot[] is free after the area chunks) and the pixel's G element
            // re-read around them, so only the sample in flight is live across a walk
            const float inv_mb = 1.0f / (float)F.m_brdf;
            for (int i = 0; i < F.m_brdf; ++i) {
                if (RS_SORT_PARK) brdf_park(L.slot, lane, r, best_phat, f_sel);
                float Wc, mis;
                rng.n = cand_slot(F.m_area + i);
                Sample s;
                {
                    const GElem g = G.load(p);
                    s = brdf_sample<T>(S, F, g.pos, make_frame(g, cam), alive, rng, Wc, mis, rays);
                }
                asm volatile("" ::: "memory");
                vec3 f;
                {
                    const GElem g = G.load(p);
                    f = evaluate_f<T>(S, F, s, g.pos, false, make_frame(g, cam), tv, alive, rays);
                }
                asm volatile("" ::: "memory");
                if (RS_SORT_PARK) brdf_unpark(L.slot, lane, r, best_phat, f_sel);
                float ph = length(f);
                float w = F.m_area > 0 ? mis * ph * Wc : inv_mb * ph * Wc;
                rng.n = cand_slot(F.m_area + i) + 3u;
                if (alive && res_add(r, s, w, 0, rng)) { best_phat = ph; f_sel = f; }
            }
        }
        if (alive) {                                                    // as initial_ris's epilogue
            r.conf = F.m_area + F.m_brdf;
            const float ph = smp_valid(smp_of(r)) ? best_phat : 0.0f;
            r.W = ph > 0.0f ? 1.0f / ph * r.wsum : 0.0f;
            res_cap(r, F.cap);
        } else {
            r = res_empty();
            f_sel = mk(0, 0, 0);
        }
    }
    if (ris) {
        Rw.store(p, r);
        if (fuse_shade) store_rgb(fb, p, shade_px(r, f_sel, G.load(p).le));
    }
}
template <int T>
__global__ void __launch_bounds__(256, RS_WAVES(T, RS_INITIAL_WAVES_SORT_LOCKSTEP, RS_INITIAL_WAVES_SORT))
k_gbuffer_initial_sorted(DevScene S, FrameConst F, GBuf G, ResBuf Rw, float* fb, int fuse_shade, CountSlot C) {
    const uint64_t t0 = wave_clock();
    if ((blockIdx.x | blockIdx.y | threadIdx.x) == 0) *C.outside = 0ull;   // this frame's counter (rs_tile_begin)
    __shared__ SortLds lds[4];
    int x, y, bx, by;
    uint32_t rays = 0;
    const bool in = pixel_of(F, F.gy0, F.gy1, x, y);
    tile_of(F, F.gy0, F.gy1, bx, by);
    const int wave = threadIdx.x >> 6;
    const int tx0 = bx * 16 + (wave & 1) * 8, ty0 = F.gy0 + by * 16 + (wave >> 1) * 8;
    const size_t hslot = (size_t)((ty0 - F.gy0) >> 3) * (size_t)(2 * ((F.W + 15) >> 4)) + (size_t)(tx0 >> 3);   // the launch's 8x8 tile
    sorted_tile<T>(S, F, G, Rw, fb, fuse_shade, lds[wave], threadIdx.x & 63, x, y, in, tx0, ty0, hslot, rays);
    count_rays(C, rays + (in ? 1u : 0u), in ? 1u : 0u, t0, y);
}
// the same pass by persistent waves (RESTIR_PERSIST_SORTED): about one device's worth of resident workgroups,
// every WAVE pulling 8x8 tiles from a per-launch counter in the grid's dispatch order (costliest tile rows first
// on full frames).  The waves of the sorted pass are independent (each its own LDS region), so a wave that
// finishes its tile takes the next at once instead of holding its workgroup's slot until the slowest of the
// four finishes -- per-lane walks vary from tile to tile.
template <int T>
__global__ void __launch_bounds__(256, RS_WAVES(T, RS_INITIAL_WAVES_SORT_LOCKSTEP, RS_INITIAL_WAVES_SORT))
k_gbuffer_initial_sorted_pq(DevScene S, FrameConst F, GBuf G, ResBuf Rw, float* fb, int fuse_shade, CountSlot C,
                            TileQ Q) {
    if ((blockIdx.x | blockIdx.y | threadIdx.x) == 0) *C.outside = 0ull;
    __shared__ SortLds lds[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t rays = 0, prim = 0;
    for (;;) {
        const uint32_t t = q_pull(Q);
        if (t >= Q.n) break;
        const uint64_t t0 = wave_clock();
        int x, y;
        const bool in = pixel_of_q(F, F.gy0, F.gy1, t, x, y);
        int tx0, ty0;
        tile_origin_q(F, F.gy0, F.gy1, t, tx0, ty0);
        sorted_tile<T>(S, F, G, Rw, fb, fuse_shade, lds[wave], lane, x, y, in, tx0, ty0,
                       (size_t)blockIdx.x * 4 + (size_t)wave, rays);   // the resident wave's slot
        rays += in ? 1u : 0u;
        prim += in ? 1u : 0u;
        row_cost_add(C, t0, y);
    }
    count_store(C, rays, prim);
    q_exit(Q);
}

// ---------------------------------------------------------------- candidate-split initial pass
// The same G-buffer + initialRenderPass with the candidates of a pixel spread over kSplit waves: a
// workgroup is ONE 8x8 tile, wave g evaluates candidate group g of its 64 pixels.  A pixel's
// candidates are independent until the reservoir stream (every candidate owns its RNG slots, and
// the shadow ray / p-hat / w of a candidate do not depend on the others), so the groups only
// exchange each candidate's weight w_c through LDS; wave 0 then runs the reference's sequential
// addSample stream over w_0..w_{A+B-1} (the same float additions in the same order, the same U per
// candidate) and re-draws the selected area sample.  Results are bit-identical to k_gbuffer_initial.
// Why: a one-thread-per-pixel launch over a small band (a rank's 1/8 of 1080p: ~4k waves for 5k wave
// slots) runs as ONE round whose time is the slowest tile's; 4x the waves with 1/4 the work each
// fill the chip and average the tiles out.
// A selected candidate always has w > 0, hence p-hat > 0, hence an unoccluded f: its f is the
// evaluate_f_pre L of the re-drawn sample, no shadow ray needed.  BRDF candidates cannot be re-drawn
// without their closest-hit ray, so their sample and f go through LDS too.
#ifndef RS_SPLIT_WAVES
#define RS_SPLIT_WAVES 4
#endif
constexpr int kSplit = RS_SPLIT_WAVES;    // waves (candidate groups) per 8x8 tile
constexpr int kSplitMaxCand = 64;         // A + B the split kernel keeps in LDS
constexpr int kSplitMaxBrdf = 2;          // B the split kernel keeps in LDS
// LDS, sized at launch for the frame's candidate counts (split_lds_bytes): FrameSlot (5 x 64 float4) + (pos,
// alive) per pixel, then w_c of candidate c at pixel lane (n x 64 floats), then BRDF candidate i's (p, f.x)
// (n, f.y) (li, f.z).  C2's 33 candidates take 17.4 KB -- a fixed 64-candidate layout (34.5 KB) held the
// kernel to 3 waves per SIMD
struct SplitLds {
    float4* frame;
    float* w;
    float4* brdf;
    __device__ __forceinline__ SplitLds(float4* base, int n)
        : frame(base), w((float*)(base + 6 * 64)), brdf(base + 6 * 64 + 16 * n) {}
};
__host__ __device__ constexpr size_t split_lds_bytes(int n, int b) {
    return (size_t)6 * 64 * 16 + (size_t)n * 64 * 4 + (size_t)b * 3 * 64 * 16;
}
// candidate range [lo, hi) of group g over the combined list (area 0..A-1, then BRDF A..A+B-1), cut at
// equal estimated cost: a BRDF candidate (a per-lane closest-hit walk, then its shadow ray) counts as
// RS_SPLIT_BRDF_W area candidates, so the last group -- the one holding the BRDF candidates -- takes fewer
// area candidates and the workgroup's waves finish together (C2, 32 + 1 candidates: groups 8 / 9 / 9 / 6 + 1;
// C2's 1/8 bands, every rank timed alone, two sessions: mean 0.2094-0.2108 vs 0.2154-0.2172 ms at weight 1,
// weights 2 and 4 no better than 1: scripts/gpu_split_ab.sh)
#ifndef RS_SPLIT_BRDF_W
#define RS_SPLIT_BRDF_W 3
#endif
__device__ __forceinline__ int split_bound(int A, int B, int k) {
    constexpr int wb = RS_SPLIT_BRDF_W;
    const int e = (k * (A + B * wb)) / kSplit;           // in area-candidate units
    if (e <= A) return e;
    const int b = (e - A) / wb;
    return A + (b < B ? b : B);
}
__device__ __forceinline__ void split_range(int A, int B, int g, int& lo, int& hi) {
    lo = split_bound(A, B, g); hi = split_bound(A, B, g + 1);
}

template <int T>
__global__ void __launch_bounds__(64 * kSplit, RS_WAVES(T, RS_INITIAL_WAVES, RS_INITIAL_WAVES_LANE)) k_gbuffer_initial_split(DevScene S, FrameConst F, GBuf G,
                                                                                  ResBuf Rw, float* fb, int fuse_shade,
                                                                                  CountSlot C) {
    const uint64_t t0 = wave_clock();
    if ((blockIdx.x | blockIdx.y | threadIdx.x) == 0) *C.outside = 0ull;   // this frame's counter (rs_tile_begin)
    extern __shared__ float4 split_lds[];
    const SplitLds L(split_lds, F.m_area + F.m_brdf);
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    int x = blockIdx.x * 8 + (lane & 7), y = F.gy0 + blockIdx.y * 8 + (lane >> 3);
    const bool in = x < F.W && y < F.gy1;
    x = x < F.W ? x : F.W - 1;
    y = y < F.gy1 ? y : F.gy1 - 1;
    const size_t p = (size_t)y * F.W + x;
    const bool ris = in && y >= F.y0 && y < F.y1;
    const FrameSlot fs{L.frame, lane, 64};
    uint32_t rays = 0;
    vec3 le = mk(0, 0, 0);
    if (g == 0) {                                                       // wave-uniform
        GElem gel = gbuffer_fill<T>(S, F, x, y, in);
        if (in) G.store(p, gel);
        fs.store(make_frame(gel, F.cam.pos));
        const bool alive = ris && !any_pos(gel.le) && S.n_emis > 0;    // :238-244
        L.frame[5 * 64 + lane] = f4(gel.pos, alive ? 1.0f : 0.0f);
        le = gel.le;
    }
    __syncthreads();
    const float4 pa = L.frame[5 * 64 + lane];
    const vec3 pos = xyz(pa);
    const bool alive = pa.w != 0.0f;
    const int A = F.m_area, B = F.m_brdf, n = A + B;
    const bool tv = !F.do_vis_pass;
    constexpr int kB = trav_lane(T) ? RS_RIS_BATCH_LANE : RS_RIS_BATCH;
    int lo, hi;
    split_range(A, B, g, lo, hi);
    if (__ballot(alive) != 0) {                                         // wave-uniform
        Rng rng; rng.init(F.seed, F.frame, PASS_INITIAL, (uint32_t)p);
        const int ahi = hi < A ? hi : A;
        for (int c0 = lo; c0 < ahi; c0 += kB) {               // area candidates (:246-266)
            float w[kB];
            uint32_t pick[kB];
#pragma unroll
            for (int k = 0; k < kB; ++k) pick[k] = area_pick(S, rng, c0 + k);
            area_batch<T, kB>(S, F, pos, fs.load(), rng, c0, ahi, alive, tv, pick, w, rays);
#pragma unroll
            for (int k = 0; k < kB; ++k)
                if (c0 + k < ahi) L.w[(c0 + k) * 64 + lane] = w[k];
        }
        for (int c = lo > A ? lo : A; c < hi; ++c) {                     // BRDF candidates (:268-286)
            float Wc, mis;
            rng.n = cand_slot(c);
            const ShadeFrame sf = fs.load();
            Sample s = brdf_sample<T>(S, F, pos, sf, alive, rng, Wc, mis, rays);
            const vec3 f = evaluate_f<T>(S, F, s, pos, false, sf, tv, alive, rays);
            L.w[c * 64 + lane] = A > 0 ? mis * length(f) * Wc : (1.0f / (float)B) * length(f) * Wc;
            float4* q = L.brdf + (c - A) * 3 * 64;
            q[lane] = f4(s.p, f.x); q[64 + lane] = f4(s.n, f.y); q[128 + lane] = f4(s.li, f.z);
        }
    }
    __syncthreads();
    if (g != 0) { count_rays(C, rays, 0, t0, y); return; }
    // wave 0: the reservoir stream in candidate order (Reservoir::addSample, pg/Reservoir.h:33-47)
    Res r = res_empty();
    vec3 f_sel = mk(0, 0, 0);
    float best_phat = 0.0f;
    if (__ballot(alive) != 0) {
        Rng rng; rng.init(F.seed, F.frame, PASS_INITIAL, (uint32_t)p);
        int sel = -1;
        for (int c = 0; c < A; ++c) {
            rng.n = cand_slot(c) + 3u;
            if (alive && res_add_w(r, L.w[c * 64 + lane], 1, rng)) sel = c;
        }
        if (sel >= 0) {                                                 // re-draw the selected area sample
            const Sample s = area_redraw(S, F, pos, fs.load(), rng, sel, tv, f_sel);
            best_phat = length(f_sel);
            r.p = s.p; r.n = s.n; r.li = s.li;
        }
        for (int c = A; c < n; ++c) {
            rng.n = cand_slot(c) + 3u;
            if (alive && res_add_w(r, L.w[c * 64 + lane], 1, rng)) {
                const float4* q = L.brdf + (c - A) * 3 * 64;
                const float4 a = q[lane], b = q[64 + lane], d = q[128 + lane];
                r.p = xyz(a); r.n = xyz(b); r.li = xyz(d);
                f_sel = mk(a.w, b.w, d.w);
                best_phat = length(f_sel);
            }
        }
    }
    if (!alive) { f_sel = mk(0, 0, 0); r = res_empty(); }
    else {
        const float ph = smp_valid(smp_of(r)) ? best_phat : 0.0f;
        r.W = ph > 0.0f ? 1.0f / ph * r.wsum : 0.0f;
        res_cap(r, F.cap);
    }
    if (ris) {
        Rw.store(p, r);
        if (fuse_shade) store_rgb(fb, p, shade_px(r, f_sel, le));
    }
    count_rays(C, rays + (in ? 1u : 0u), in ? 1u : 0u, t0, y);
}

// visibilityPass (pg/ReSTIRIntegrator.cpp:302-312).  Invalid samples always carry W == 0 already,
// so their (meaningless) ray is not traced.
template <int T>
__global__ void __launch_bounds__(256) k_visibility(DevScene S, FrameConst F, GBuf G, ResBuf R, CountSlot C) {
    const uint64_t t0 = wave_clock();
    int x, y;
    uint32_t rays = 0;
    const bool in = pixel_of(F, F.y0, F.y1, x, y);
    const size_t p = (size_t)y * F.W + x;
    Res r = R.load(p);
    const bool need = in && smp_valid(smp_of(r));
    if (occluded<T>(S, F, need, G.pos(p), r.p, rays) && need) R.r[3 * p + 1].w = 0.0f;
    count_rays(C, rays, 0, t0, y);
}

// reprojectBackward / reprojectForward (pg/ReSTIRIntegrator.cpp:544-587)
__device__ __forceinline__ bool reproject(const GCam& c, vec3 ws, int W, int H, int& sx, int& sy) {
    const float* m = c.view;   // glm mat4 * vec4: (m0*x + m1*y) + (m2*z + m3*1)
    float vx = (m[0] * ws.x + m[4] * ws.y) + (m[8] * ws.z + m[12] * 1.0f);
    float vy = (m[1] * ws.x + m[5] * ws.y) + (m[9] * ws.z + m[13] * 1.0f);
    float vz = (m[2] * ws.x + m[6] * ws.y) + (m[10] * ws.z + m[14] * 1.0f);
    if (vz >= 0) return false;
    float fx = (-vx / vz) * c.focal + (float)W / 2.0f;
    float fy = (vy / vz) * c.focal + (float)H / 2.0f;
    float rx = roundf(fx), ry = roundf(fy);
    if (!(rx >= -2147483648.0f && rx < 2147483648.0f) || !(ry >= -2147483648.0f && ry < 2147483648.0f)) return false;
    int X = (int)rx, Y = (int)ry;
    if (X < 0 || X > W - 1 || Y < 0 || Y > H - 1) return false;
    sx = X; sy = Y;
    return true;
}

// k_temporal's per-thread state across its shadow walks: 20 words component-major (a wave's access to
// one word is conflict-free), 20 KB per workgroup
struct TemporalSlot {
    static constexpr int kWords = 20;
    float* base;
    int t;
    __device__ __forceinline__ void put(int c, float v) const { base[c * 256 + t] = v; }
    __device__ __forceinline__ float get(int c) const { return base[c * 256 + t]; }
    __device__ __forceinline__ void put3(int c, vec3 v) const { put(c, v.x); put(c + 1, v.y); put(c + 2, v.z); }
    __device__ __forceinline__ vec3 get3(int c) const { return mk(get(c), get(c + 1), get(c + 2)); }
};

// temporalReusePass (pg/ReSTIRIntegrator.cpp:625-732).  The previous reservoir is read at the
// CURRENT pixel (:641), the previous G-buffer at the reprojected pixel (:652).
// T | TEMPORAL_BAND: the G-buffers hold only the tile's rows +- margin (a band of a multi-GPU frame, a
// tile): the instantiation with the rare rebuilds below; a full-frame launch has none (their walks and the
// state kept around them would otherwise cost every wave registers)
constexpr int TEMPORAL_BAND = 4;
// the bucket of a ray toward a light point: direction octant x the target's cell (one bit per axis against
// the emitters' centroid centre) -- the sorted temporal and spatial passes' key
__device__ __forceinline__ uint32_t point_bucket(const DevScene& S, vec3 pt, vec3 d) {
    const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    const uint32_t cx = pt.x > S.ecen.x ? 1u : 0u, cy = pt.y > S.ecen.y ? 2u : 0u, cz = pt.z > S.ecen.z ? 4u : 0u;
    return (oct << 3) | cx | cy | cz;
}
// T | TEMPORAL_SORT: the four shadow rays of a wave's 64 pixels are counting-sorted by direction octant x
// target cell (as k_spatial_sorted's) and traced 64 at a time in that order (lane = ray); bit-identical
constexpr int TEMPORAL_SORT = 8;
struct TemporalSortLds {                    // one wave's region (1.5 KB)
    uint16_t slot[4 * 64];                  // slot k * 64 + lane: rank of ray k of pixel lane in its bucket
    uint16_t e[4 * 64];                     // the slots, bucket by bucket
    uint32_t cur[64];                       // bucket counts, then offsets
    uint32_t occ[64];                       // per pixel: occlusion bit of ray k
};
template <int T>
// Sp: the previous frame's geometry (== S unless the scene moved since; rs_scene::dev_of), traced when a tile
// rebuilds a previous-frame G element beyond its rows
__global__ void __launch_bounds__(256, RS_WAVES(T, RS_TEMPORAL_WAVES, RS_TEMPORAL_WAVES_LANE)) k_temporal(DevScene S, DevScene Sp, FrameConst F, GBuf G, GBuf Gp, ResBuf Rr, ResBuf Rl,
                                                  ResBuf Rw, CountSlot C) {
    constexpr bool kBand = (T & TEMPORAL_BAND) != 0;
    constexpr bool kSort = (T & TEMPORAL_SORT) != 0;
    const uint64_t t0 = wave_clock();
    int x, y;
    uint32_t rays = 0;
    const bool in = pixel_of(F, F.y0, F.y1, x, y);
    const size_t p = (size_t)y * F.W + x;
    const vec3 cpos = G.pos(p);
    int qx = x, qy = y, fx = x, fy = y;
    bool ok = in && reproject(F.camp, cpos, F.W, F.H, qx, qy);
    uint32_t dcode = (in && !ok) ? 1u : 0u;          // debugReprojection (pg/ReSTIRIntegrator.cpp:647-689)
    bool dfwd = false;
    // A tile holds the G-buffers of its rows +- margin only.  A reprojection beyond them (a miss
    // pixel's position is (0,0,0), which projects anywhere) rebuilds the element it needs from the
    // frame's camera -- gBufferFillPass is a function of (camera, pixel) -- so tiles stay bit-identical
    // to the full frame.  Rare (a few pixels per frame): counted in Counters::reproj_outside.
    // Only positions live across these rebuilds' walks; the full elements are loaded after them (the
    // previous one rebuilt once more for its lanes) so no G element is spilled around a walk.
    const bool q_out = kBand && ok && (qy < F.gy0 || qy >= F.gy1);
    const size_t q = ok && !q_out ? (size_t)qy * F.W + qx : p;
    vec3 ppos = Gp.pos(q);
    if constexpr (kBand) if (__ballot(q_out) != 0) {
        const GElem alt = gbuffer_fill_cam<T>(Sp, F, F.camp, F.inv_view_prev, qx, qy, q_out);
        if (q_out) { ppos = alt.pos; rays += 1u; atomicAdd(C.outside, 1ull); }
    }
    if (ok) {
        float cd = length(cpos - F.cam.pos), pd = length(ppos - F.camp.pos);
        float dr = cd > pd ? pd / cd : cd / pd;
        ok = !(dr < 0.9f);
        dcode = ok ? dcode : 2u;
    }
    vec3 pac = Gp.pos(p);
    const bool fok = ok && reproject(F.cam, pac, F.W, F.H, fx, fy);
    dcode = (ok && !fok) ? 3u : dcode;
    const bool f_out = kBand && fok && (fy < F.gy0 || fy >= F.gy1);
    vec3 fw = G.pos(fok && !f_out ? (size_t)fy * F.W + fx : p);
    if constexpr (kBand) if (__ballot(f_out) != 0) {
        const GElem alt = gbuffer_fill_cam<T>(S, F, F.cam, F.inv_view, fx, fy, f_out);
        if (f_out) { fw = alt.pos; rays += 1u; atomicAdd(C.outside, 1ull); }
    }
    if (ok) {
        ok = fok;
        if (ok) {
            float cdp = length(pac - F.camp.pos), pdp = length(fw - F.cam.pos);
            float drp = cdp > pdp ? pdp / cdp : cdp / pdp;
            ok = !(drp < 0.9f);
            dfwd = !ok;
        }
    }
    if (F.debug_reproj) {                             // recorded; painted by k_debug_reproj after the pass
        const size_t n = (size_t)F.W * F.H;
        if (dcode) F.dbg[p] = (uint8_t)dcode;
        if (dfwd) F.dbg[n + (size_t)fy * F.W + fx] = 1u;
    }
    const bool any_ok = __ballot(ok) != 0;
    float ph[4];
    __shared__ float temporal_lds[TemporalSlot::kWords * 256];
    const TemporalSlot ts{temporal_lds, (int)threadIdx.x};
    if (any_ok) {
        const GElem cur = G.load(p);
        GElem prev = Gp.load(q);
        if constexpr (kBand) if (__ballot(q_out && ok) != 0) {            // the rebuilt element again (its ray counted above)
            const GElem alt = gbuffer_fill_cam<T>(Sp, F, F.camp, F.inv_view_prev, qx, qy, q_out && ok);
            if (q_out) prev = alt;
        }
        // the four evaluateF calls (:700-717: the current and previous samples at the current and previous
        // surfaces).  Their unoccluded f are evaluated first; what the shadow walks need afterwards -- the two
        // origins and two targets, |L| and |L * 0| (the post-visibility lengths bit for bit, evaluate_f_post)
        // -- goes to this thread's LDS slots (TemporalSlot), the need bits stay in a register, and the
        // reservoirs are re-read after the walks (L2-resident), so the walks run with the whole register
        // budget and nothing is spilled around them (r03: 219 scratch ops, the walk loops spill-free)
        const Sample cs = smp_of(Rr.load(p)), ps = smp_of(Rl.load(p));
        uint32_t nd = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const FPre e = evaluate_f_pre(F, k < 2 ? cs : ps, (k & 1) ? F.camp.pos : F.cam.pos, (k & 1) ? prev : cur,
                                          true, ok);
            ts.put(12 + k, e.ok ? length(e.L) : 0.0f);
            ts.put(16 + k, e.ok ? length(e.L * 0.0f) : 0.0f);
            // the current sample at the current surface (k = 0) is the initial pass's selection, found unoccluded
            // from this pixel by the same ray (§3.2): not traced again (F.canon_vis: no visibility pass)
            const bool need = e.need && !(k == 0 && F.canon_vis);
            nd |= need ? 1u << k : 0u;
            rays += need ? 1u : 0u;
        }
        ts.put3(0, cur.pos); ts.put3(3, prev.pos); ts.put3(6, cs.p); ts.put3(9, ps.p);
        if constexpr (kSort) {
            __shared__ TemporalSortLds sort_lds[4];
            TemporalSortLds& L = sort_lds[threadIdx.x >> 6];
            const int lane = threadIdx.x & 63, wbase = threadIdx.x & ~63;
            // ---- A: each needed ray takes a rank in its bucket (lane = pixel)
            L.cur[lane] = 0u;
            L.occ[lane] = 0u;
            wave_lds_sync();
            uint32_t bk = 0u;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((nd >> k) & 1u) {
                    const vec3 tg = ts.get3(6 + 3 * (k >> 1));
                    const uint32_t b = point_bucket(S, tg, tg - ts.get3(3 * (k & 1)));
                    L.slot[k * 64 + lane] = (uint16_t)atomicAdd(&L.cur[b], 1u);
                    bk |= b << (8 * k);
                }
            wave_lds_sync();
            const uint32_t cnt_b = L.cur[lane];
            uint32_t incl = cnt_b;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(incl, o);
                incl += lane >= o ? v : 0u;
            }
            const uint32_t n_rays = __shfl(incl, 63);
            L.cur[lane] = incl - cnt_b;
            wave_lds_sync();
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((nd >> k) & 1u) L.e[L.cur[(bk >> (8 * k)) & 63u] + L.slot[k * 64 + lane]] = (uint16_t)(k * 64 + lane);
            wave_lds_sync();
            // ---- B: the rays in bucket order (lane = ray), re-formed from the pixel's LDS slot
            if constexpr (trav_lane(T) && trav_wide(T)) {              // lanes refilled from the list (rs_scene.h)
                occluded_wide_list(S, n_rays, FLT_MIN + F.tnear_off,
                    [&](uint32_t j, vec3& o, vec3& d, float& tfar) {
                        const uint32_t sl = L.e[j];
                        const int k = (int)(sl >> 6), src = (int)(sl & 63u);
                        const TemporalSlot tq{temporal_lds, wbase + src};
                        o = tq.get3(3 * (k & 1));
                        const vec3 ld = tq.get3(6 + 3 * (k >> 1)) - o;                   // evaluate_f_pre's ray
                        d = normalize(ld);
                        tfar = sqrtf(dot(ld, ld)) - F.tfar_off;
                    },
                    [&](uint32_t j, bool oc) {
                        const uint32_t sl = L.e[j];
                        if (oc) atomicOr(&L.occ[sl & 63u], 1u << (sl >> 6));
                    });
            } else
            for (uint32_t j0 = 0; j0 < n_rays; j0 += 64u) {
                const uint32_t j = j0 + (uint32_t)lane;
                const bool act = j < n_rays;
                const uint32_t sl = L.e[act ? j : 0u];
                const int k = (int)(sl >> 6), src = (int)(sl & 63u);
                const TemporalSlot tq{temporal_lds, wbase + src};
                const vec3 o = tq.get3(3 * (k & 1)), ld = tq.get3(6 + 3 * (k >> 1)) - o;   // evaluate_f_pre's ray
                const bool oc = trace_any<T>(S, act, o, normalize(ld), FLT_MIN + F.tnear_off, sqrtf(dot(ld, ld)) - F.tfar_off);
                if (act && oc) atomicOr(&L.occ[src], 1u << k);
            }
            wave_lds_sync();
            // ---- C: the p-hats (lane = pixel)
            const uint32_t occm = L.occ[lane];
#pragma unroll
            for (int k = 0; k < 4; ++k) ph[k] = ((nd & occm) >> k) & 1u ? ts.get(16 + k) : ts.get(12 + k);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                asm volatile("" ::: "memory");
                const vec3 o = ts.get3(3 * (k & 1)), ld = ts.get3(6 + 3 * (k >> 1)) - o;   // evaluate_f_pre's ray
                const bool need = (nd >> k) & 1u;
                const bool oc = trace_any<T>(S, need, o, normalize(ld), FLT_MIN + F.tnear_off, sqrtf(dot(ld, ld)) - F.tfar_off);
                asm volatile("" ::: "memory");
                ph[k] = need && oc ? ts.get(16 + k) : ts.get(12 + k);
            }
        }
    }
    asm volatile("" ::: "memory");                      // re-read the reservoirs: nothing carried across the walks
    const Res cr = Rr.load(p);
    Res out = cr;
    if (any_ok) {
        const Res pr = Rl.load(p);
        Rng rng; rng.init(F.seed, F.frame, PASS_TEMPORAL, (uint32_t)p);
        Res res = res_empty();
        const Sample cs = smp_of(cr), ps = smp_of(pr);
        const float p_cur = ph[0], p_prev = ph[1];
        float m_cur = p_cur * (float)cr.conf / (p_cur * (float)cr.conf + p_prev * (float)pr.conf);
        if (!(m_cur > 0)) m_cur = 0.0f;
        float ph_cur = p_cur;
        const float p_cur2 = ph[2], p_prev2 = ph[3];
        if (ok) {
            bool took_cur = res_add(res, cs, m_cur * ph_cur * cr.W, cr.conf, rng);
            float m_prev = p_prev2 * (float)pr.conf / (p_cur2 * (float)cr.conf + p_prev2 * (float)pr.conf);
            if (!(m_prev > 0)) m_prev = 0.0f;
            float ph_prev = p_cur2;
            bool took_prev = res_add(res, ps, m_prev * ph_prev * pr.W, pr.conf, rng);
            res_cap(res, F.cap);
            float fph = took_prev ? ph_prev : (took_cur ? ph_cur : 0.0f);
            res.W = fph > 0.0f ? res.wsum / fph : 0.0f;
            out = res;
        }
    }
    if (in) Rw.store(p, out);
    count_rays(C, rays, 0, t0, y);
}

// debugReprojection's colours (pg/ReSTIRIntegrator.cpp:648,663,675,689) into the current G-buffer emission,
// after the temporal pass: a pixel's own rejection wins over a forward-check mark from another pixel
__global__ void k_debug_reproj(GBuf G, const uint8_t* __restrict__ dbg, uint32_t n) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint32_t own = dbg[p], fwd = dbg[n + p];
    if (!own && !fwd) return;
    const vec3 c = own == 1u ? mk(100, 100, 0) : (own == 2u ? mk(0, 100, 0) : (own == 3u ? mk(100, 0, 100) : mk(0, 0, 100)));
    G.g4[p] = f4(c, G.g4[p].w);
}

// Sampling::sampleDiskUniform (pg/Sampling.cpp:78-87) -> glm::vec<2,int> (truncation), clamped to
// the screen (pg/ReSTIRIntegrator.cpp:338-340).  Draws 2i and 2i+1 of the pixel's spatial stream.
__device__ __forceinline__ size_t neighbor_px(const FrameConst& F, const Rng& rng, int i, int x, int y) {
    float u0 = rng.at(2u * i), u1 = rng.at(2u * i + 1u);
    float theta = (0.0f + (2.0f - 0.0f) * u0) * kPi;
    float r = sqrtf(0.0f + (F.radius - 0.0f) * u1);
    float sn, cs;
    rs_sincosf(theta, &sn, &cs);
    float ox = r * cs, oy = r * sn;
    int nx = x + (int)ox, ny = y + (int)oy;
    nx = nx < 0 ? 0 : (nx > F.W - 1 ? F.W - 1 : nx);
    ny = ny < 0 ? 0 : (ny > F.H - 1 ? F.H - 1 : ny);
    return (size_t)ny * F.W + nx;
}

// list position i (0 = canonical) -> pixel index; `acc` bit j set <=> neighbour draw j accepted
__device__ __forceinline__ size_t list_px(const FrameConst& F, const Rng& rng, uint64_t acc, int i, int x, int y,
                                          size_t p) {
    if (i == 0) return p;
    int c = 0;
    for (int j = 0; j < F.k; ++j) {
        if ((acc >> j) & 1ull) {
            if (++c == i) return neighbor_px(F, rng, j, x, y);
        }
    }
    return p;
}

// neighbour-list cache entries per thread in LDS (list positions 1..k; k <= kNbrCache - 1)
constexpr int kNbrCache = 17;

// spatialReusePass (pg/ReSTIRIntegrator.cpp:316-542); shade fused when this is the last pass.
// List loops run to the uniform bound k+1 with `i < cnt` as a predicate (convergent ray queries).
// CM = 1: the CONSTANT-MIS instantiation (the metric point), compiled without the other modes' code
// and register pressure; CM = 0 handles every mode.
template <int T, int CM, int SMALL = 0>
__global__ void __launch_bounds__(256, RS_WAVES(T, SMALL ? RS_SPATIAL_WAVES_SMALL : RS_SPATIAL_WAVES, RS_SPATIAL_WAVES_LANE))
k_spatial(DevScene S, FrameConst F, GBuf G, ResBuf Rr, ResBuf Rw, int pass_idx, int fuse_shade, float* fb, CountSlot C) {
    const int mode = CM ? MIS_CONSTANT : F.mis;
    __shared__ uint32_t nbr[kNbrCache * 256];
    const uint64_t t0 = wave_clock();
    int x, y;
    uint32_t rays = 0;
    const bool in = pixel_of(F, F.y0, F.y1, x, y);
    const size_t p = (size_t)y * F.W + x;
    const vec3 cam = F.cam.pos;
    GElem th = G.load(p);
    const bool emissive = any_pos(th.le);
    const bool alive = in && !emissive;
    if (in && emissive) {                                  // :319-324
        Res r = Rr.load(p);
        Rw.store(p, r);
        if (fuse_shade) store_rgb(fb, p, shade_px(r, mk(0, 0, 0), th.le));
    }
    if (__ballot(alive) != 0) {
        Rng rng; rng.init(F.seed, F.frame, PASS_SPATIAL0 + (uint32_t)pass_idx, (uint32_t)p);
        // neighbour selection (:334-374); the accepted list is cached in LDS when k <= kNbrCache - 1
        // (list position i -> pixel), otherwise list_px re-derives it from the RNG slots
        const bool cached = F.k < kNbrCache;
        uint64_t acc = 0;
        int M = 1;
        for (int i = 0; i < F.k; ++i) {
            size_t q = neighbor_px(F, rng, i, x, y);
            if (any_pos(G.le(q))) continue;
            if (F.reject) {
                float4 nq = G.g1[q];
                float ns = dot(xyz(nq), th.nrm);
                if (ns < F.min_normal_sim) continue;
                float nd = G.g0[q].w;
                float dr = 0;
                if (nd > 0) dr = th.depth / nd;
                float hd = F.max_depth_diff * 0.5f;
                if (dr < 1.0f - hd || dr > 1.0f + hd) continue;
            }
            acc |= 1ull << i;
            if (cached) nbr[M * 256 + threadIdx.x] = (uint32_t)q;
            M += 1;
        }
        auto list_q = [&](int i) -> size_t {
            if (!cached) return list_px(F, rng, acc, i, x, y, p);
            return (i == 0 || i >= M) ? p : (size_t)nbr[i * 256 + threadIdx.x];
        };
        rng.n = 2u * (uint32_t)F.k;
        const int cnt = M;
        const int kk = F.k + 1;                            // uniform list bound
        int csum = 0, csum_nc = 0;                         // :379-385
        for (int i = 0; i < cnt; ++i) {
            int c = __float_as_int(Rr.r[3 * list_q(i) + 2].w);
            csum += c;
            if (i) csum_nc += c;
        }
        Res res = res_empty();
        int sel = 0;
        float rcpM = M > 0 ? 1.0f / (float)M : 0.0f;
        vec3 f_sel = mk(0, 0, 0);
        if (mode == MIS_CONSTANT) {
            // CONSTANT MIS (the metric point): the k+1 candidates' shadow rays all start at this pixel,
            // so pairs share one walk (trace_any_multi); the addSample draws stay in candidate order
            const ShadeFrame sf = make_frame(th, cam);
            for (int i0 = 0; i0 < kk; i0 += 2) {
                FPre pre[2];
                Res rr[2];
                bool act[2], occ[2];
                vec3 dir[2];
                float tf[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int i = i0 + k;
                    rr[k] = Rr.load(list_q(i));
                    pre[k] = evaluate_f_pre(F, smp_of(rr[k]), th.pos, false, sf, true, alive && i < cnt);
                    pre[k].need = pre[k].need && !(i == 0 && F.canon_vis);   // known unoccluded: f = L as traced
                    act[k] = pre[k].need; dir[k] = pre[k].dir; tf[k] = pre[k].tfar; occ[k] = false;
                    rays += act[k] ? 1u : 0u;
                }
                trace_any_multi<T, 2>(S, act, th.pos, dir, FLT_MIN + F.tnear_off, tf, occ);
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int i = i0 + k;
                    if (i < kk) {
                        const vec3 f = evaluate_f_post(pre[k], occ[k]);
                        const float rw = rcpM * length(f) * rr[k].W;
                        if (alive && i < cnt && res_add(res, smp_of(rr[k]), rw, rr[k].conf, rng)) { sel = i; f_sel = f; }
                    }
                }
            }
        } else for (int i = 0; i < kk; ++i) {
            const bool li = alive && i < cnt;
            size_t qi = list_q(i);
            Res ri = Rr.load(qi);
            Sample si = smp_of(ri);
            float mis = rcpM;
            if (mode == MIS_BALANCE) {                    // :407-424
                float num = 0, den = 0;
                mis = 0.0f;
                for (int j = 0; j < kk; ++j) {
                    const bool lj = li && j < cnt;
                    size_t qj = list_q(j);
                    int cj = __float_as_int(Rr.r[3 * qj + 2].w);
                    float ph = length(evaluate_f<T>(S, F, si, cam, G.load(qj), true, lj, rays));
                    if (lj) {
                        den += ph * cj;
                        if (i == j) num = ph * ri.conf;
                    }
                }
                if (den > 0) mis = num / den;
            }
            if (mode == MIS_PAIRWISE) {                   // :427-467
                mis = 0.0f;
                if (i == 0) {
                    float sum = 0.0f;
                    float phc = length(evaluate_f<T>(S, F, si, cam, G.load(qi), true, li, rays)) * (float)ri.conf;
                    for (int j = 1; j < kk; ++j) {
                        const bool lj = li && j < cnt;
                        size_t qj = list_q(j);
                        int cj = __float_as_int(Rr.r[3 * qj + 2].w);
                        float phj = length(evaluate_f<T>(S, F, si, cam, G.load(qj), true, lj, rays));
                        float den = phc + phj * (float)csum_nc;
                        if (lj && den > 0) {
                            float cf = (float)cj / (float)csum;
                            sum += cf * (phc / den);
                        }
                    }
                    mis = ((float)ri.conf / (float)csum) + sum;
                } else {
                    float phi = length(evaluate_f<T>(S, F, si, cam, G.load(qi), true, li, rays));
                    float phc = length(evaluate_f<T>(S, F, si, cam, G.load(p), true, li, rays));
                    phi *= (float)csum_nc;
                    int c0 = __float_as_int(Rr.r[3 * p + 2].w);
                    float den = phi + phc * (float)c0;
                    if (den > 0 && csum > 0) mis = ((float)ri.conf / (float)csum) * (phi / den);
                }
            }
            vec3 f = evaluate_f<T>(S, F, si, cam, th, true, li, rays);     // :472
            float rph = length(f);
            float rw = mis * rph * ri.W;
            if (li && res_add(res, si, rw, ri.conf, rng)) { sel = i; f_sel = f; }
        }
        float fph = smp_valid(smp_of(res)) ? length(f_sel) : 0.0f;  // :481
        if (mode == MIS_CONSTANT || mode == MIS_BALANCE || mode == MIS_PAIRWISE) {
            res.W = fph > 0.0f ? res.wsum / fph : 0.0f;
        } else if (mode == MIS_DEBIAS_Z) {                // :494-506
            int Z = 0;
            float corr = 1.0f;
            for (int i = 0; i < kk; ++i) {
                const bool li = alive && i < cnt;
                size_t qi = list_q(i);
                bool occ = occluded<T>(S, F, li, G.pos(qi), res.p, rays);
                if (li && !occ) Z += 1;
            }
            if (Z > 0 && M > 0) corr = (1.0f / (float)Z) / rcpM;
            res.W = fph > 0.0f ? corr * res.wsum / fph : 0.0f;
        } else if (mode == MIS_DEBIAS_CONTRIB) {          // :515-538
            Sample ss = smp_of(Rr.load(list_q(sel)));
            float num = 0, den = 0, cw = 0, corr = 0;
            for (int i = 0; i < kk; ++i) {
                const bool li = alive && i < cnt;
                size_t qi = list_q(i);
                int ci = __float_as_int(Rr.r[3 * qi + 2].w);
                float ph = length(evaluate_f<T>(S, F, ss, cam, G.load(qi), true, li, rays));
                if (li) {
                    den += ph * (float)ci;
                    if (i == sel) num = ph * (float)ci;
                }
            }
            if (den > 0) cw = num / den;
            if (M > 0) corr = cw / rcpM;
            res.W = fph > 0.0f ? corr * res.wsum / fph : 0.0f;
        }
        res_cap(res, F.cap);
        if (alive) {
            Rw.store(p, res);
            if (fuse_shade) store_rgb(fb, p, shade_px(res, f_sel, th.le));
        }
    }
    count_rays(C, rays, 0, t0, y);
}

// ---------------------------------------------------------------- wave-sorted spatial pass (CONSTANT MIS)
// The same regrouping as k_gbuffer_initial_sorted for the spatial pass's k + 1 visibility rays per pixel (the
// pixel to each listed neighbour's sample): per wave the rays are counting-sorted by octant x the target's cell
// (one bit per axis of the emitters' bounds: the samples are light points) and traced 64 at a time in that
// order; each lane re-forms its ray from the slot (list position, pixel) -- the pixel's surface point from the
// G-buffer, the neighbour's sample from its reservoir -- with evaluate_f_pre's operations, and the reservoir
// stream then runs per pixel in list order.  Bit-identical to k_spatial<T, 1> (tests/test_gpu_parity.py).
// Lists of up to kSpatialSortMax entries (k <= 8); longer lists take k_spatial.
constexpr int kSpatialSortMax = 9;
struct SpatialSortLds {                     // one wave's region (2.9 KB)
    uint16_t slot[kSpatialSortMax * 64];    // slot i * 64 + lane: rank in its bucket
    uint16_t e[kSpatialSortMax * 64];       // the slots of the rays, bucket by bucket
    uint32_t cur[64];                       // bucket counts, then offsets
    uint32_t occ[64];                       // per pixel: occlusion bit of list position i
};

#ifndef RS_SPATIAL_WAVES_SORT_LOCKSTEP
#define RS_SPATIAL_WAVES_SORT_LOCKSTEP RS_SPATIAL_WAVES
#endif
template <int T>
__global__ void __launch_bounds__(256, RS_WAVES(T, RS_SPATIAL_WAVES_SORT_LOCKSTEP, RS_SPATIAL_WAVES_LANE))
k_spatial_sorted(DevScene S, FrameConst F, GBuf G, ResBuf Rr, ResBuf Rw, int pass_idx, int fuse_shade, float* fb, CountSlot C) {
    __shared__ uint32_t nbr[(kSpatialSortMax - 1) * 256];      // list position i >= 1 -> pixel
    __shared__ SpatialSortLds lds[4];
    SpatialSortLds& L = lds[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63, wbase = threadIdx.x & ~63;
    const uint64_t t0 = wave_clock();
    int x, y;
    uint32_t rays = 0;
    const bool in = pixel_of(F, F.y0, F.y1, x, y);
    const size_t p = (size_t)y * F.W + x;
    const vec3 cam = F.cam.pos;
    GElem th = G.load(p);
    const bool emissive = any_pos(th.le);
    const bool alive = in && !emissive;
    if (in && emissive) {                                  // :319-324
        Res r = Rr.load(p);
        Rw.store(p, r);
        if (fuse_shade) store_rgb(fb, p, shade_px(r, mk(0, 0, 0), th.le));
    }
    if (__ballot(alive) != 0) {
        Rng rng; rng.init(F.seed, F.frame, PASS_SPATIAL0 + (uint32_t)pass_idx, (uint32_t)p);
        int M = 1;                                          // neighbour selection (:334-374), as k_spatial
        for (int i = 0; i < F.k; ++i) {
            size_t q = neighbor_px(F, rng, i, x, y);
            if (any_pos(G.le(q))) continue;
            if (F.reject) {
                float4 nq = G.g1[q];
                float ns = dot(xyz(nq), th.nrm);
                if (ns < F.min_normal_sim) continue;
                float nd = G.g0[q].w;
                float dr = 0;
                if (nd > 0) dr = th.depth / nd;
                float hd = F.max_depth_diff * 0.5f;
                if (dr < 1.0f - hd || dr > 1.0f + hd) continue;
            }
            nbr[(M - 1) * 256 + threadIdx.x] = (uint32_t)q;
            M += 1;
        }
        rng.n = 2u * (uint32_t)F.k;
        const int cnt = M, kk = F.k + 1;
        auto list_q = [&](int i) -> size_t { return (i == 0 || i >= M) ? p : (size_t)nbr[(i - 1) * 256 + threadIdx.x]; };
        ShadeFrame sf = make_frame(th, cam);
        // ---- A: every list entry's ray need and bucket rank (lane = pixel)
        L.cur[lane] = 0u;
        L.occ[lane] = 0u;
        wave_lds_sync();
        uint32_t needm = 0u, bkt[3] = {0u, 0u, 0u};         // 9 buckets x 6 bits -> 3 words of 3 x 10 bits
        for (int i = 0; i < kk; ++i) {
            const Res rr = Rr.load(list_q(i));
            const FPre pre = evaluate_f_pre(F, smp_of(rr), th.pos, false, sf, true, alive && i < cnt);
            if (pre.need && !(i == 0 && F.canon_vis)) {       // the canonical sample: known unoccluded, not traced
                const uint32_t b = point_bucket(S, rr.p, pre.dir);
                L.slot[i * 64 + lane] = (uint16_t)atomicAdd(&L.cur[b], 1u);
                bkt[i / 3] |= b << (10 * (i % 3));
                needm |= 1u << i;
            }
        }
        wave_lds_sync();
        const uint32_t cnt_b = L.cur[lane];
        uint32_t incl = cnt_b;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o);
            incl += lane >= o ? v : 0u;
        }
        const uint32_t n_rays = __shfl(incl, 63);
        L.cur[lane] = incl - cnt_b;
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < kSpatialSortMax; ++i)
            if ((needm >> i) & 1u) {
                const uint32_t b = (bkt[i / 3] >> (10 * (i % 3))) & 63u;
                L.e[L.cur[b] + L.slot[i * 64 + lane]] = (uint16_t)(i * 64 + lane);
            }
        wave_lds_sync();
        // ---- B: the rays in bucket order (lane = ray)
        if constexpr (trav_lane(T) && trav_wide(T)) {                  // lanes refilled from the list (rs_scene.h)
            occluded_wide_list(S, n_rays, FLT_MIN + F.tnear_off,
                [&](uint32_t j, vec3& o, vec3& ld, float& tfar) {
                    const uint32_t sl = L.e[j];
                    const uint32_t i = sl >> 6, src = sl & 63u;
                    const uint32_t psrc = tile_pixel(F, F.y0, F.y1, (int)src);
                    const size_t q = i == 0 ? (size_t)psrc : (size_t)nbr[(i - 1) * 256 + wbase + src];
                    o = xyz(G.g0[psrc]);
                    const vec3 sp = xyz(Rr.r[3 * q]);
                    ld = sp - o;                                        // evaluate_f_pre's ray
                    const float r2 = dot(ld, ld);
                    ld = normalize(ld);
                    tfar = sqrtf(r2) - F.tfar_off;
                    rays += 1u;
                },
                [&](uint32_t j, bool occ) {
                    const uint32_t sl = L.e[j];
                    if (occ) atomicOr(&L.occ[sl & 63u], 1u << (sl >> 6));
                });
        } else
        for (uint32_t j0 = 0; j0 < n_rays; j0 += 64u) {
            const uint32_t j = j0 + (uint32_t)lane;
            const bool act = j < n_rays;
            const uint32_t sl = L.e[act ? j : 0u];
            const uint32_t i = sl >> 6, src = sl & 63u;
            const uint32_t psrc = tile_pixel(F, F.y0, F.y1, (int)src);
            const size_t q = i == 0 ? (size_t)psrc : (size_t)nbr[(i - 1) * 256 + wbase + src];
            const vec3 o = xyz(G.g0[psrc]);
            const vec3 sp = xyz(Rr.r[3 * q]);
            vec3 ld = sp - o;                                   // evaluate_f_pre's ray
            const float r2 = dot(ld, ld);
            ld = normalize(ld);
            const float tfar = sqrtf(r2) - F.tfar_off;
            const bool occ = trace_any<T>(S, act, o, ld, FLT_MIN + F.tnear_off, tfar);
            rays += act ? 1u : 0u;
            if (act && occ) atomicOr(&L.occ[src], 1u << i);
        }
        wave_lds_sync();
        // ---- C: the reservoir stream in list order (lane = pixel).  The pixel's G element and frame are
        // re-read / re-derived here rather than carried across B's walks (they would be spilled around them)
        asm volatile("" ::: "memory");
        th = G.load(p);
        sf = make_frame(th, cam);
        const uint32_t occm = L.occ[lane];
        const float rcpM = M > 0 ? 1.0f / (float)M : 0.0f;
        Res res = res_empty();
        vec3 f_sel = mk(0, 0, 0);
        for (int i = 0; i < kk; ++i) {
            const Res rr = Rr.load(list_q(i));
            const FPre pre = evaluate_f_pre(F, smp_of(rr), th.pos, false, sf, true, alive && i < cnt);
            const vec3 f = evaluate_f_post(pre, ((occm >> i) & 1u) != 0u);
            const float rw = rcpM * length(f) * rr.W;
            if (alive && i < cnt && res_add(res, smp_of(rr), rw, rr.conf, rng)) f_sel = f;
        }
        const float fph = smp_valid(smp_of(res)) ? length(f_sel) : 0.0f;  // :481
        res.W = fph > 0.0f ? res.wsum / fph : 0.0f;
        res_cap(res, F.cap);
        if (alive) {
            Rw.store(p, res);
            if (fuse_shade) store_rgb(fb, p, shade_px(res, f_sel, th.le));
        }
    }
    count_rays(C, rays, 0, t0, y);
}

// shade loop (pg/simpleguidx11.cpp:447-472)
template <int T>
__global__ void __launch_bounds__(256) k_shade(DevScene S, FrameConst F, GBuf G, ResBuf Rr, float* fb, CountSlot C) {
    const uint64_t t0 = wave_clock();
    int x, y;
    uint32_t rays = 0;
    const bool in = pixel_of(F, F.y0, F.y1, x, y);
    const size_t p = (size_t)y * F.W + x;
    Res r = Rr.load(p);
    GElem g = G.load(p);
    vec3 f = evaluate_f<T>(S, F, smp_of(r), F.cam.pos, g, true, in && r.wsum > 0.0f, rays);
    if (in) store_rgb(fb, p, shade_px(r, f, g.le));
    count_rays(C, rays, 0, t0, y);
}

}  // namespace rs
