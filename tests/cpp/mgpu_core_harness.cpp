// TEST INFRASTRUCTURE: the native multi-GPU orchestration (restir-embree_amd/csrc/rs_mgpu_core.h, the
// code rs_mgpu_render_frame runs) driven on the CPU: every rank is an oracle context rendering its band
// with the oracle's tile stages (or_tile_*), the halo exchange and gather are host memcpys between the
// ranks' buffers.  Built by tests/test_mgpu_core.py (g++), loaded with ctypes.
#include "../../restir-embree_amd/csrc/rs_mgpu_core.h"

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
int or_tile_begin(void* c, const void* s, const float* cam7, const void* P, uint32_t frame, int y0, int y1, int margin,
                  int halo);
int or_tile_halo_ptr(void* c, int which, void** ptr, size_t* bytes);
int or_tile_temporal(void* c);
int or_tile_spatial(void* c, int p);
int or_tile_finish(void* c, float* out_rgb, uint64_t* rays);
}

namespace {
struct OracleRank {
    void* ctx;
    const void* scene;
    const float* cam7;
    const void* P;
    uint32_t frame;
    int W, H, y0 = 0, y1 = 0;
    std::vector<float> fb;      // full-frame framebuffer, the band's rows filled by finish
    int begin(int a, int b, int margin, int halo) {
        y0 = a; y1 = b;
        return or_tile_begin(ctx, scene, cam7, P, frame, a, b, margin, halo);
    }
    int temporal() { return or_tile_temporal(ctx); }
    int spatial(int p) { return or_tile_spatial(ctx, p); }
    int finish() {
        fb.assign((size_t)H * W * 3, 0.0f);
        uint64_t rays = 0;
        return or_tile_finish(ctx, fb.data() + (size_t)y0 * W * 3, &rays);
    }
    void* halo(int which, size_t* bytes) {
        void* p = nullptr;
        *bytes = 0;
        or_tile_halo_ptr(ctx, which, &p, bytes);
        return p;
    }
    char* frame_base() { return fb.empty() ? nullptr : (char*)fb.data(); }
};

// host memcpy transport over the same transfer plans rs_mgpu.hip's local mode pairs (rs::mgpu::pair_local)
struct HostComm {
    float* full;
    int W;
    size_t halo_bytes;
    std::vector<int> bounds, ids;
    int exchanges = 0;
    int run(std::vector<OracleRank*>& rk, const std::vector<std::vector<rs::mgpu::Xfer>>& plans) {
        return rs::mgpu::pair_local(plans, ids, [&](int i, const rs::mgpu::Xfer& x, int j, const rs::mgpu::Xfer& y) -> int {
            void *dst, *src;
            if (x.slot == rs::mgpu::kFrameRows) {
                dst = rk[i]->frame_base() + x.offset;
                src = rk[j]->frame_base() + y.offset;
            } else {
                size_t bd = 0, bs = 0;
                dst = rk[i]->halo(x.slot, &bd);
                src = rk[j]->halo(y.slot, &bs);
                if (!dst || !src || bd != x.bytes || bs != y.bytes) return -10;
                ++exchanges;
            }
            std::memcpy(dst, src, x.bytes);
            return 0;
        });
    }
    int exchange_halo(std::vector<OracleRank*>& rk, int) {
        std::vector<std::vector<rs::mgpu::Xfer>> plans;
        for (size_t i = 0; i < rk.size(); ++i) plans.push_back(rs::mgpu::halo_plan(ids[i], (int)rk.size(), halo_bytes));
        return run(rk, plans);
    }
    int gather(std::vector<OracleRank*>& rk) {
        std::vector<std::vector<rs::mgpu::Xfer>> plans;
        for (size_t i = 0; i < rk.size(); ++i) plans.push_back(rs::mgpu::gather_plan(ids[i], bounds, (size_t)W * 3 * sizeof(float)));
        if (int rc = run(rk, plans)) return rc;
        std::memcpy(full, rk[0]->frame_base() + 0, rk[0]->fb.size() * sizeof(float));
        return 0;
    }
};

// Recording link: what issue_plan would post to RCCL, with the lane communicator it would use
struct Op { int rank, lane, peer; bool send; size_t bytes; };
struct RecLink {
    std::vector<Op>* ops; int rank, lane; int groups = 0, open = 0;
    int group_start() { ++open; return 0; }
    int group_end() { ++groups; --open; return 0; }
    int send(const void*, size_t b, int peer) { if (!open) return -5; ops->push_back({rank, lane, peer, true, b}); return 0; }
    int recv(void*, size_t b, int peer) { if (!open) return -5; ops->push_back({rank, lane, peer, false, b}); return 0; }
};
// a rank object whose buffers exist exactly where a tile of rows [y0, y1) has them
struct FakeRank {
    int y0, y1, H, h; size_t halo_bytes; std::vector<char>* mem;
    void* halo(int which, size_t* bytes) {
        const int r0 = which == 0 ? y0 - h : which == 1 ? y1 : which == 2 ? y0 : y1 - h;
        *bytes = 0;
        if (h == 0 || r0 < 0 || r0 + h > H) return nullptr;    // rs_tile_halo_ptr's rule
        *bytes = halo_bytes;
        return mem->data();
    }
    char* frame_base() { return mem->data(); }
};
}  // namespace

extern "C" {
// One frame of `n` ranks (oracle contexts, one scene each) over the row bounds[0..n]; the gathered frame
// into full (H*W*3).  Returns 0 or an error code; *exchanges = halo copies made.
int harness_frame(void** ctxs, const void** scenes, int n, const int32_t* bounds, int W, const float* cam7,
                  const void* params, int spatial_passes, float radius, int spatial, uint32_t frame, float* full,
                  int* exchanges) {
    std::vector<OracleRank> ranks(n);
    std::vector<OracleRank*> ptrs(n);
    std::vector<int> ids(n), b(bounds, bounds + n + 1);
    for (int i = 0; i < n; ++i) {
        ranks[i] = OracleRank{ctxs[i], scenes[i], cam7, params, frame, W, b[n]};
        ptrs[i] = &ranks[i];
        ids[i] = i;
    }
    const int halo = n > 1 ? rs::mgpu::halo_rows(radius, spatial != 0 && spatial_passes > 0) : 0;
    HostComm comm{full, W, (size_t)halo * W * 48, b, ids};
    const int rc = rs::mgpu::render_frame(ptrs, comm, b, ids, spatial ? spatial_passes : 0, halo, halo, true);
    if (exchanges) *exchanges = comm.exchanges;
    return rc;
}

// rs::mgpu::balanced_bounds on host costs
int harness_balanced(const double* costs, int H, int world, int min_rows, int32_t* out) {
    std::vector<double> c(costs, costs + H);
    std::vector<int> b;
    if (!rs::mgpu::balanced_bounds(c, world, min_rows, b)) return -1;
    for (int i = 0; i <= world; ++i) out[i] = b[i];
    return 0;
}
// rs::mgpu::balanced_bounds_grain (rs_mgpu_rebalance's split: boundaries on whole `grain`-row wave tiles)
int harness_balanced_grain(const double* costs, int H, int world, int min_rows, int grain, int32_t* out) {
    std::vector<double> c(costs, costs + H);
    std::vector<int> b;
    if (!rs::mgpu::balanced_bounds_grain(c, world, min_rows, grain, b)) return -1;
    for (int i = 0; i <= world; ++i) out[i] = b[i];
    return 0;
}
int harness_halo(float radius) { return rs::mgpu::halo_rows(radius, true); }

// Every rank of a `world`-rank frame issues its halo and gather plans through issue_plan (the code the
// RCCL branch runs) into a recording link on the frame's lane; the recorded operations are then paired:
// every send needs exactly one recv of equal bytes from the same peer on the same lane communicator.
// Returns the number of operations (> 0) or a negative code; msg receives the first violation.
int harness_plan_check(int world, const int32_t* bounds, int W, int H, int halo, int lane, char* msg, int msg_len) {
    std::vector<int> b(bounds, bounds + world + 1);
    std::vector<Op> ops;
    std::vector<char> mem(16);
    std::vector<std::vector<rs::mgpu::Xfer>> hp, gp;
    const size_t hb = (size_t)halo * W * 48, row = (size_t)W * 12;
    for (int r = 0; r < world; ++r) {
        FakeRank g{b[r], b[r + 1], H, halo, hb, &mem};
        RecLink link{&ops, r, lane};
        hp.push_back(rs::mgpu::halo_plan(r, world, hb));
        gp.push_back(rs::mgpu::gather_plan(r, b, row));
        if (int rc = rs::mgpu::issue_plan(g, hp.back(), link)) return rc < 0 ? rc - 100 : -100;
        if (int rc = rs::mgpu::issue_plan(g, gp.back(), link)) return rc < 0 ? rc - 200 : -200;
        if (link.open) return -300;
    }
    std::string e = rs::mgpu::check_plans(hp);
    if (e.empty()) e = rs::mgpu::check_plans(gp);
    // pair the recorded operations themselves (what the communicators would see)
    std::vector<char> used(ops.size(), 0);
    for (size_t k = 0; k < ops.size() && e.empty(); ++k) {
        if (!ops[k].send) continue;
        size_t hits = 0;
        for (size_t q = 0; q < ops.size(); ++q)
            if (!ops[q].send && !used[q] && ops[q].rank == ops[k].peer && ops[q].peer == ops[k].rank &&
                ops[q].lane == ops[k].lane && ops[q].bytes == ops[k].bytes) { used[q] = 1; ++hits; break; }
        if (hits != 1) e = "send " + std::to_string(ops[k].rank) + "->" + std::to_string(ops[k].peer) + " unmatched";
    }
    for (size_t q = 0; q < ops.size() && e.empty(); ++q)
        if (!ops[q].send && !used[q]) e = "recv " + std::to_string(ops[q].rank) + "<-" + std::to_string(ops[q].peer) + " unmatched";
    if (!e.empty()) {
        if (msg && msg_len > 0) { std::strncpy(msg, e.c_str(), msg_len - 1); msg[msg_len - 1] = 0; }
        return -1;
    }
    // byte totals: 2 (world - 1) halo messages each way; the gather covers every row outside rank 0's band
    size_t halo_sent = 0, gather_recv = 0;
    for (auto& p : hp) halo_sent += rs::mgpu::plan_bytes(p, true);
    for (auto& p : gp) gather_recv += rs::mgpu::plan_bytes(p, false);
    if (halo_sent != 2 * (size_t)(world - 1) * hb) return -2;
    if (gather_recv != (size_t)(H - b[1]) * row) return -3;
    return (int)ops.size();
}
// a deliberately broken plan set must be rejected by check_plans (the checker itself is tested)
int harness_plan_check_negative() {
    std::vector<std::vector<rs::mgpu::Xfer>> p = {rs::mgpu::halo_plan(0, 2, 96), rs::mgpu::halo_plan(1, 2, 96)};
    if (!rs::mgpu::check_plans(p).empty()) return -1;
    p[1][0].bytes = 48;                              // size mismatch
    if (rs::mgpu::check_plans(p).empty()) return -2;
    p[1] = {};                                       // a rank that posts nothing
    if (rs::mgpu::check_plans(p).empty()) return -3;
    // a halo the tile does not have -> issue_plan fails before the group starts
    std::vector<Op> ops;
    std::vector<char> mem(16);
    FakeRank g{0, 10, 20, 0, 96, &mem};              // h = 0: no halo rows
    RecLink link{&ops, 0, 0};
    const int rc = rs::mgpu::issue_plan(g, rs::mgpu::halo_plan(0, 2, 96), link);
    if (rc != -2 || !ops.empty() || link.groups != 0) return -4;
    return 0;
}
}
