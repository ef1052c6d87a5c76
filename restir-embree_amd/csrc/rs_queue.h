// rs_queue.h -- the queued initial pass (north star: persistent-thread wavefront kernels with ballot-
// compacted ray queues) for incoherent scenes, where one-thread-per-pixel shadow walks leave most of a
// wave idle: on C3 a wave's 64 walks take max-over-lanes ~158 node visits for a mean of ~75, so half
// the lane-steps do nothing.  The same initialRenderPass (pg/ReSTIRIntegrator.cpp:236-298) in three
// launches, bit-identical to k_gbuffer_initial:
//   k_q_generate  one thread per pixel: G-buffer fill, then every area candidate's sample and
//                 unoccluded f (no walk); the candidate's RIS weight for both visibility outcomes goes
//                 to cw[c][pixel], its shadow ray -- if it needs one -- is appended to the wave's
//                 segment of the ray queue (wave ballot + mbcnt: compaction without atomics, in a
//                 deterministic order).  BRDF candidates (closest hit + their own shadow ray) run here
//                 as before and store (w, sample, f).
//   k_q_trace     persistent waves, a grid-stride over segments: a lane whose ray is finished takes
//                 the next ray of the queue at once (ballot of the idle lanes, prefix rank), so every
//                 walk step runs on (nearly) full waves; any-hit result -> occ[c][pixel].
//   k_q_resolve   one thread per pixel: the reference's addSample stream over the candidates in order
//                 (w = occ ? w_occ : w_vis, the same U per candidate), the selected area sample
//                 re-drawn from its RNG slots, BRDF candidates from their records; reservoir write and
//                 the fused shade.
// Queue storage per frame in flight (sized for the launch's rows): rays 20 B x A per pixel, weights
// 8 B x A, occlusion 1 B x A, BRDF records 52 B x B.
#pragma once
#include "rs_passes.h"

#ifndef RS_Q_TRACE_WAVES
#define RS_Q_TRACE_WAVES 8
#endif
#ifndef RS_Q_GEN_WAVES
#define RS_Q_GEN_WAVES 6
#endif

namespace rs {

struct QBuf {
    float4* ray;        // per k_q_generate wave: 64 * A slots, (dir.xyz, tfar)
    uint32_t* rid;      // per slot: (candidate << 24) | local pixel (pixel - gy0 * W)
    uint32_t* cnt;      // per k_q_generate wave: rays in its segment
    float2* cw;         // [c][local pixel]: (w if unoccluded, w if occluded) -- equal when no ray is traced
    uint8_t* occ;       // [c][local pixel]: any-hit of the candidate's shadow ray
    float4* brdf;       // [b][3][local pixel]: (p, f.x) (n, f.y) (li, f.z)
    float* bw;          // [b][local pixel]: the BRDF candidate's RIS weight
    uint32_t P;         // local pixels (rows gy0..gy1 x W): stride of the [c][pixel] arrays
    int A;              // area candidates (segment capacity 64 * A)
};

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {   // set bits of mask below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <int T>
__global__ void __launch_bounds__(256, RS_Q_GEN_WAVES) k_q_generate(DevScene S, FrameConst F, GBuf G, QBuf Q,
                                                                     CountSlot C) {
    const uint64_t t0 = wave_clock();
    if ((blockIdx.x | blockIdx.y | threadIdx.x) == 0) *C.outside = 0ull;   // this frame's counter (rs_tile_begin)
    int x, y;
    uint32_t rays = 0;
    const bool in = pixel_of(F, F.gy0, F.gy1, x, y);
    const size_t p = (size_t)y * F.W + x;
    const uint32_t lp = (uint32_t)(p - (size_t)F.gy0 * F.W);
    __shared__ float4 frame_lds[5 * 256];
    const FrameSlot fs{frame_lds, (int)threadIdx.x, 256};
    const GElem g = gbuffer_fill<T>(S, F, x, y, in);
    if (in) G.store(p, g);
    fs.store(make_frame(g, F.cam.pos));
    const bool ris = in && y >= F.y0 && y < F.y1;
    const bool alive = ris && !any_pos(g.le) && S.n_emis > 0;          // :238-244
    const uint32_t wave = (blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const size_t base = (size_t)wave * 64u * (uint32_t)Q.A;
    uint32_t n = 0;                                                     // rays in the segment (uniform)
    if (__ballot(alive) != 0) {                                         // wave-uniform
        Rng rng; rng.init(F.seed, F.frame, PASS_INITIAL, (uint32_t)p);
        const bool tv = !F.do_vis_pass;
        const float inv_ma = 1.0f / (float)F.m_area;
        for (int c = 0; c < F.m_area; ++c) {                            // :246-266 without the walks
            const ShadeFrame sf = fs.load();
            float Wc, mis;
            const uint32_t pick = area_pick(S, rng, c);
            rng.n = cand_slot(c) + 1u;
            const Sample s = area_sample_at(S, F, g.pos, sf, rng, pick, Wc, mis);
            const FPre pr = evaluate_f_pre(F, s, g.pos, false, sf, tv, alive);
            const float ph = length(pr.L);
            const float m = F.m_brdf > 0 ? mis : inv_ma;
            const float wu = m * ph * Wc, wo = m * 0.0f * Wc;           // area_batch's two outcomes
            const float wf = pr.ok ? wu : wo;                           // no ray: the outcome is known
            if (alive) Q.cw[(size_t)c * Q.P + lp] = pr.need ? make_float2(wu, wo) : make_float2(wf, wf);
            const uint64_t mk_need = __ballot(pr.need);
            if (pr.need) {
                const size_t slot = base + n + lane_rank(mk_need);
                Q.ray[slot] = f4(pr.dir, pr.tfar);
                Q.rid[slot] = ((uint32_t)c << 24) | lp;
            }
            n += (uint32_t)__popcll(mk_need);
        }
        if (F.m_brdf > 0) {                                             // :268-286, as initial_ris
            const float inv_mb = 1.0f / (float)F.m_brdf;
            for (int i = 0; i < F.m_brdf; ++i) {
                float Wc, mis;
                rng.n = cand_slot(F.m_area + i);
                const ShadeFrame sf = fs.load();
                const Sample s = brdf_sample<T>(S, F, g.pos, sf, alive, rng, Wc, mis, rays);
                const vec3 f = evaluate_f<T>(S, F, s, g.pos, false, sf, tv, alive, rays);
                const float ph = length(f);
                if (alive) {
                    Q.bw[(size_t)i * Q.P + lp] = F.m_area > 0 ? mis * ph * Wc : inv_mb * ph * Wc;
                    float4* q = Q.brdf + (size_t)i * 3 * Q.P;
                    q[lp] = f4(s.p, f.x); q[Q.P + lp] = f4(s.n, f.y); q[2 * (size_t)Q.P + lp] = f4(s.li, f.z);
                }
            }
        }
    }
    if ((threadIdx.x & 63) == 0) Q.cnt[wave] = n;
    count_rays(C, rays + (in ? 1u : 0u), in ? 1u : 0u, t0, y);
}

// Persistent any-hit walks over the queue: waves stride over the segments; idle lanes refill from the
// wave's cursor (seg, pos) -- uniform, in SGPRs -- after every step, so lanes do not wait for the
// wave's longest walk.  The walk is occluded_lane's (same box / triangle tests, first hit ends it).
__global__ void __launch_bounds__(256, RS_Q_TRACE_WAVES) k_q_trace(DevScene S, FrameConst F, GBuf G, QBuf Q,
                                                                   uint32_t n_seg, CountSlot C) {
    const uint64_t t0 = wave_clock();
    const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
    uint32_t seg = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    uint32_t pos = 0, cnt = seg < n_seg ? Q.cnt[seg] : 0u;
    const uint32_t cap = 64u * (uint32_t)Q.A;
    const uint32_t n_nodes = S.n_nodes;
    const float tnear = FLT_MIN + F.tnear_off;
    bool have = false;
    uint32_t i = 0, id = 0, occ = 0, rays = 0, tri = 0, tl = 0, after = 0;
    vec3 o = mk(0, 0, 0), d = mk(0, 0, 1), inv = mk(0, 0, 1);
    float tfar = 0.0f;
    while (true) {
        uint64_t idle = __ballot(!have);
        while (idle != 0 && seg < n_seg) {                              // refill the idle lanes
            const uint32_t avail = cnt - pos;
            if (avail == 0) {
                seg += n_waves;
                pos = 0;
                cnt = seg < n_seg ? Q.cnt[seg] : 0u;
                continue;
            }
            const uint32_t k = (uint32_t)__popcll(idle), take = k < avail ? k : avail;
            const uint32_t rk = lane_rank(idle);
            if (!have && rk < take) {
                const size_t slot = (size_t)seg * cap + pos + rk;
                const float4 rr = Q.ray[slot];
                id = Q.rid[slot];
                o = G.pos((size_t)F.gy0 * F.W + (id & 0xffffffu));
                d = xyz(rr); tfar = rr.w;
                inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
                i = 0; occ = 0; tl = 0; have = true;
                ++rays;
            }
            pos += take;
            idle = __ballot(!have);
        }
        if (__ballot(have) == 0) break;                                 // queue drained, every lane done
        // One step per lane: a node visit, or ONE triangle test of the leaf the lane is in.  (Testing
        // a leaf's triangles in a loop inside the node step makes the whole wave wait for the largest
        // leaf any lane entered -- on C3 some lane is in a leaf in most steps.)  Same box and triangle
        // tests as occluded_lane; the first hit ends the walk.
        if (have) {
            if (tl > 0) {
                const float4* Tp = S.tris + 3 * tri;
                float t, u, v;
                if (tri_test_nb(Tp[0], Tp[1], Tp[2], o, d, tnear, tfar, t, u, v)) occ = 1u;
                ++tri;
                --tl;
                if (tl == 0) i = after;
            } else {
                const float4 a = S.nodes[2 * i], b = S.nodes[2 * i + 1];
                const uint32_t skip = (uint32_t)__float_as_int(a.w);
                const int leaf = __float_as_int(b.w);
                const bool hit = box_test(a, b, o, inv, tnear, tfar);
                if (hit && leaf >= 0) { tri = (uint32_t)(leaf >> 3); tl = (leaf & 7) + 1; after = skip; }
                else i = (hit && leaf < 0) ? i + 1 : skip;
            }
            if (occ || (tl == 0 && i >= n_nodes)) {                     // the walk ended: record, go idle
                Q.occ[(size_t)(id >> 24) * Q.P + (id & 0xffffffu)] = (uint8_t)(occ != 0u);
                have = false;
            }
        }
    }
    count_rays(C, rays, 0, t0, -1);
}

// the addSample stream (pg/Reservoir.h:33-47) in candidate order over the queued results
__global__ void __launch_bounds__(256) k_q_resolve(DevScene S, FrameConst F, GBuf G, QBuf Q, ResBuf Rw, float* fb,
                                                   int fuse_shade, CountSlot C) {
    const uint64_t t0 = wave_clock();
    int x, y;
    const bool in = pixel_of(F, F.y0, F.y1, x, y);
    const size_t p = (size_t)y * F.W + x;
    const uint32_t lp = (uint32_t)(p - (size_t)F.gy0 * F.W);
    const GElem g = G.load(p);
    const bool alive = in && !any_pos(g.le) && S.n_emis > 0;
    Res r = res_empty();
    vec3 f_sel = mk(0, 0, 0);
    float best_phat = 0.0f;
    if (__ballot(alive) != 0) {
        Rng rng; rng.init(F.seed, F.frame, PASS_INITIAL, (uint32_t)p);
        const bool tv = !F.do_vis_pass;
        int sel = -1;
        for (int c = 0; c < F.m_area; ++c) {
            const float2 w2 = alive ? Q.cw[(size_t)c * Q.P + lp] : make_float2(0.0f, 0.0f);
            const bool oc = alive && Q.occ[(size_t)c * Q.P + lp] != 0;
            rng.n = cand_slot(c) + 3u;
            if (alive && res_add_w(r, oc ? w2.y : w2.x, 0, rng)) sel = c;
        }
        if (sel >= 0) {                                                 // the selected area sample, re-drawn
            const Sample s = area_redraw(S, F, g.pos, make_frame(g, F.cam.pos), rng, sel, tv, f_sel);
            best_phat = length(f_sel);
            r.p = s.p; r.n = s.n; r.li = s.li;
        }
        for (int b = 0; b < F.m_brdf; ++b) {
            const float w = alive ? Q.bw[(size_t)b * Q.P + lp] : 0.0f;
            rng.n = cand_slot(F.m_area + b) + 3u;
            if (alive && res_add_w(r, w, 0, rng)) {
                const float4* q = Q.brdf + (size_t)b * 3 * Q.P;
                const float4 a = q[lp], bb = q[Q.P + lp], e = q[2 * (size_t)Q.P + lp];
                r.p = xyz(a); r.n = xyz(bb); r.li = xyz(e);
                f_sel = mk(a.w, bb.w, e.w);
                best_phat = length(f_sel);
            }
        }
    }
    if (!alive) { f_sel = mk(0, 0, 0); r = res_empty(); }
    else {
        r.conf = F.m_area + F.m_brdf;                                   // +1 per candidate (pg/Reservoir.h:35)
        const float ph = smp_valid(smp_of(r)) ? best_phat : 0.0f;
        r.W = ph > 0.0f ? 1.0f / ph * r.wsum : 0.0f;
        res_cap(r, F.cap);
    }
    if (in) {
        Rw.store(p, r);
        if (fuse_shade) store_rgb(fb, p, shade_px(r, f_sel, g.le));
    }
    count_rays(C, 0, 0, t0, y);
}

}  // namespace rs
