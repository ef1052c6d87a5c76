// rs_mgpu.hip -- tile-sharded frames across GPUs behind the C ABI (SURVEY.md §8b rs_mgpu_render_frame,
// §8e): the C++ caller of the reference (SimpleGuiDX11::Producer, pg/simpleguidx11.cpp:240-241) renders an
// N-GPU frame with one call per rank.  One rs_mgpu per process holds
//   * RCCL mode (rs_mgpu_create): this process's rank of `world`, one communicator per run-ahead lane
//     (ncclCommInitRank + ncclCommSplit), so frames in flight on different lanes exchange halos and
//     gather independently; every transfer is a point-to-point ncclSend/ncclRecv group issued on the
//     frame's own lane stream (xGMI links are point-to-point: no ring collective on the data path);
//   * local mode (rs_mgpu_create_local): `world` contexts of this process (e.g. N ranks on one GPU for
//     tests, or one process driving several GPUs), transfers by device copies between the contexts'
//     buffers ordered with events.
// The stage sequence is rs::mgpu::render_frame (rs_mgpu_core.h), shared with the CPU test of the
// orchestration.
#include "rs_mgpu_core.h"
#include "rs_internal.h"
#include "../../include/restir_c.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

using namespace rs;

namespace {

constexpr int kLanes = RS_MAX_AHEAD + 1;   // run-ahead lanes of a context (restir_capi.hip kMaxAhead + 1)

// one rank's tile stages on its context (the interface rs::mgpu::render_frame drives)
struct GpuRank {
    rs_context* ctx = nullptr;
    const rs_scene* scene = nullptr;
    rs_camera cam{};
    rs_frame_params P{};
    uint32_t frame = 0;
    int y0 = 0, y1 = 0;
    const float* band = nullptr;     // band framebuffer after finish
    hipStream_t st = nullptr;        // the frame's stream (a run-ahead lane)
    int lane = 0;
    rs_pass_times* times = nullptr;
    int begin(int a, int b, int margin, int halo) {
        y0 = a; y1 = b;
        rs_tile_desc t{a, b, std::max(margin, halo), halo};
        if (int rc = rs_tile_begin(ctx, scene, &cam, &P, frame, &t)) return rc;
        void* s = nullptr;
        if (int rc = rs_tile_stream(ctx, &s, &lane)) return rc;
        st = (hipStream_t)s;
        return 0;
    }
    int temporal() { return rs_tile_temporal(ctx); }
    int spatial(int p) { return rs_tile_spatial(ctx, p); }
    int finish() { return rs_tile_finish(ctx, &band, times); }
    void* halo(int which, size_t* bytes) {
        void* p = nullptr;
        *bytes = 0;
        if (rs_tile_halo_ptr(ctx, which, &p, bytes) != RS_OK) return nullptr;
        return p;
    }
    // the full-frame framebuffer the band was rendered into (rows at their place)
    char* frame_base() {
        return band ? (char*)const_cast<float*>(band) - (size_t)y0 * ctx_width(ctx) * 3 * sizeof(float) : nullptr;
    }
};

#define NCCLCHK(m, x)                                                                                      \
    do {                                                                                                   \
        ncclResult_t r_ = (x);                                                                             \
        if (r_ != ncclSuccess) return (m)->error(RS_E_HIP, std::string(#x " -> ") + ncclGetErrorString(r_)); \
    } while (0)
#define HIPCHK_M(m, x)                                                                                     \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) return (m)->error(RS_E_HIP, std::string(#x " -> ") + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

struct rs_mgpu {
    bool local = false;
    int world = 1;
    std::vector<int> rank_ids;                  // global rank of each local rank
    std::vector<GpuRank> ranks;
    std::vector<GpuRank*> rank_ptrs;
    std::vector<int> bounds;                    // world + 1 row boundaries
    int W = 0, H = 0;
    ncclComm_t comm[kLanes] = {};
    // local mode: events ordering copies between the contexts' streams
    std::vector<hipEvent_t> ev_a, ev_b;
    int refine = 2;                             // time-based refinement rounds of rs_mgpu_rebalance
    std::vector<std::vector<double>> rebalance_ms;   // per measured round of the last rebalance: every rank's ms
    double* d_red = nullptr;                    // RCCL all-reduce scratch (rows of costs / a few scalars)
    size_t red_cap = 0;
    std::string err;
    int error(int code, const std::string& m) {
        err = m;
        return ctx_fail(ranks.empty() ? nullptr : ranks[0].ctx, code, "rs_mgpu: " + m);
    }

    // ---- transfer statistics (rs_mgpu_get_stats): per frame, HIP events around each halo exchange and
    // the gather on every local rank's frame stream, folded when the ring slot is reused.  stats.halo_ms /
    // gather_ms are local rank 0's (the ABI's figures); halo_ms_rank / gather_ms_rank hold every local
    // rank's, so measure_bands can take each rank's own exchange time out of its band time.
    static constexpr int kStatRing = 8, kTimedPasses = 4, kEvPerRank = 2 * kTimedPasses + 2;
    std::vector<hipEvent_t> sev[kStatRing];     // [local rank * kEvPerRank + event]
    int s_nx[kStatRing] = {};                   // exchanges recorded in the slot
    bool s_gather[kStatRing] = {}, s_pending[kStatRing] = {};
    int s_slot = 0;
    size_t halo_bytes = 0;                      // per halo slot of the frame in progress
    rs_mgpu_stats stats{};
    std::vector<double> halo_ms_rank, gather_ms_rank;
    hipEvent_t& ev(int slot, size_t i, int e) { return sev[slot][i * kEvPerRank + e]; }
    static double span(hipEvent_t a, hipEvent_t b) {
        float ms = 0.0f;
        if (hipEventSynchronize(b) == hipSuccess && hipEventElapsedTime(&ms, a, b) == hipSuccess) return ms;
        return 0.0;
    }
    void fold(int k) {
        if (!s_pending[k]) return;
        s_pending[k] = false;
        for (size_t i = 0; i < ranks.size(); ++i) {
            double h = 0.0, g = 0.0;
            for (int x = 0; x < s_nx[k]; ++x) h += span(ev(k, i, 2 * x), ev(k, i, 2 * x + 1));
            if (s_gather[k]) g = span(ev(k, i, 2 * kTimedPasses), ev(k, i, 2 * kTimedPasses + 1));
            halo_ms_rank[i] += h; gather_ms_rank[i] += g;
            if (i == 0) { stats.halo_ms += h; stats.gather_ms += g; }
        }
    }
    int begin_frame_stats() {
        s_slot = (s_slot + 1) % kStatRing;
        fold(s_slot);
        if (halo_ms_rank.size() != ranks.size()) { halo_ms_rank.assign(ranks.size(), 0.0); gather_ms_rank.assign(ranks.size(), 0.0); }
        if (sev[s_slot].empty()) {
            sev[s_slot].assign(ranks.size() * kEvPerRank, nullptr);
            for (size_t i = 0; i < ranks.size(); ++i) {     // each rank's events on its context's device
                HIPCHK_M(this, hipSetDevice(ctx_device(ranks[i].ctx)));
                for (int e = 0; e < kEvPerRank; ++e) HIPCHK_M(this, hipEventCreate(&ev(s_slot, i, e)));
            }
            HIPCHK_M(this, hipSetDevice(ctx_device(ranks[0].ctx)));
        }
        s_nx[s_slot] = 0; s_gather[s_slot] = false; s_pending[s_slot] = true;
        stats.frames++;
        return 0;
    }
    int record_all(std::vector<GpuRank*>& rk, int e) {
        for (size_t i = 0; i < rk.size(); ++i) HIPCHK_M(this, hipEventRecord(ev(s_slot, i, e), rk[i]->st));
        return 0;
    }

    // RCCL point-to-point link of one frame: its lane's communicator, its stream; every call checked
    struct NcclLink {
        rs_mgpu* m; ncclComm_t comm; hipStream_t st;
        int group_start() { NCCLCHK(m, ncclGroupStart()); return 0; }
        int group_end() { NCCLCHK(m, ncclGroupEnd()); return 0; }
        int send(const void* p, size_t b, int peer) { NCCLCHK(m, ncclSend(p, b, ncclUint8, peer, comm, st)); return 0; }
        int recv(void* p, size_t b, int peer) { NCCLCHK(m, ncclRecv(p, b, ncclUint8, peer, comm, st)); return 0; }
    };

    // local mode: every rank's plan paired with its neighbours' (rs::mgpu::pair_local); each recv is a copy
    // on the receiver's stream after the sender's last stage, and the sender's next stage waits for it
    int local_exchange(std::vector<GpuRank*>& rk, const std::vector<std::vector<mgpu::Xfer>>& plans) {
        const int n = (int)rk.size();
        for (int i = 0; i < n; ++i) HIPCHK_M(this, hipEventRecord(ev_a[i], rk[i]->st));
        std::vector<std::vector<char>> readers(n, std::vector<char>(n, 0));   // readers[j][i]: i copied from j
        int rc = mgpu::pair_local(plans, rank_ids, [&](int i, const mgpu::Xfer& x, int j, const mgpu::Xfer& y) -> int {
            void *dst = nullptr, *src = nullptr;
            if (x.slot == mgpu::kFrameRows) {
                dst = rk[i]->frame_base() + x.offset;
                src = rk[j]->frame_base() + y.offset;
            } else {
                size_t bd = 0, bs = 0;
                dst = rk[i]->halo(x.slot, &bd);
                src = rk[j]->halo(y.slot, &bs);
                if (bd != x.bytes || bs != y.bytes) return -2;
            }
            if (!dst || !src) return -2;
            HIPCHK_M(this, hipStreamWaitEvent(rk[i]->st, ev_a[j], 0));
            HIPCHK_M(this, hipMemcpyAsync(dst, src, x.bytes, hipMemcpyDeviceToDevice, rk[i]->st));
            readers[j][i] = 1;
            return 0;
        });
        if (rc == -1) return error(RS_E_INVALID, "local exchange: a transfer plan has no matching sender");
        if (rc == -2) return error(RS_E_INVALID, "local exchange: a halo or framebuffer is missing or has the wrong size");
        if (rc) return rc;
        for (int i = 0; i < n; ++i) HIPCHK_M(this, hipEventRecord(ev_b[i], rk[i]->st));
        for (int j = 0; j < n; ++j)                  // senders: their next stage writes the buffers read
            for (int i = 0; i < n; ++i)
                if (readers[j][i]) HIPCHK_M(this, hipStreamWaitEvent(rk[j]->st, ev_b[i], 0));
        return 0;
    }

    // ---- halo exchange (the Comm interface of rs::mgpu::render_frame)
    int exchange_halo(std::vector<GpuRank*>& rk, int pass) {
        if (world == 1) return 0;
        const bool timed = pass < kTimedPasses;
        if (timed)
            if (int rc = record_all(rk, 2 * pass)) return rc;
        std::vector<std::vector<mgpu::Xfer>> plans;
        for (size_t i = 0; i < rk.size(); ++i) {
            plans.push_back(mgpu::halo_plan(rank_ids[i], world, halo_bytes));
            stats.halo_bytes_sent += mgpu::plan_bytes(plans.back(), true);
            stats.halo_bytes_recv += mgpu::plan_bytes(plans.back(), false);
        }
        if (!local) {
            GpuRank& g = *rk[0];
            NcclLink link{this, comm[g.lane], g.st};
            const int rc = mgpu::issue_plan(g, plans[0], link);
            if (rc == -2) return error(RS_E_INVALID, "halo exchange: the tile has no halo rows the plan needs");
            if (rc) return rc;
        } else if (int rc = local_exchange(rk, plans)) {
            return rc;
        }
        if (timed) {
            if (int rc = record_all(rk, 2 * pass + 1)) return rc;
            s_nx[s_slot] = pass + 1;
        }
        return 0;
    }

    // ---- gather: band framebuffers -> rank 0's context framebuffer (full frame, rows at their place).
    // Every rank's context stream then waits for the gather (ctx_join): later work there -- the next
    // frame on the context stream, rs_synchronize, an all-reduce on comm[0] -- is ordered after the
    // transfer that reads (senders) or writes (rank 0) this lane's framebuffer.
    int gather(std::vector<GpuRank*>& rk) {
        if (world == 1) return 0;
        if (int rc = record_all(rk, 2 * kTimedPasses)) return rc;
        const size_t row = (size_t)W * 3 * sizeof(float);
        std::vector<std::vector<mgpu::Xfer>> plans;
        for (size_t i = 0; i < rk.size(); ++i) {
            plans.push_back(mgpu::gather_plan(rank_ids[i], bounds, row));
            stats.gather_bytes += mgpu::plan_bytes(plans.back(), false);
        }
        if (!local) {
            GpuRank& g = *rk[0];
            NcclLink link{this, comm[g.lane], g.st};
            const int rc = mgpu::issue_plan(g, plans[0], link);
            if (rc == -2) return error(RS_E_INVALID, "gather: no framebuffer");
            if (rc) return rc;
        } else if (int rc = local_exchange(rk, plans)) {
            return rc;
        }
        if (int rc = record_all(rk, 2 * kTimedPasses + 1)) return rc;
        s_gather[s_slot] = true;
        for (auto* g : rk)
            if (int rc = ctx_join(g->ctx, g->st)) return rc;
        return 0;
    }

    // sum (op 0) or max (op 1) of n doubles over all ranks, in place (host values)
    int allreduce(double* v, int n, int op) {
        if (local || world == 1) return 0;
        GpuRank& g = ranks[0];
        hipStream_t st = ctx_stream(g.ctx);
        if ((size_t)n > red_cap) {
            if (d_red) hipFree(d_red);
            d_red = nullptr; red_cap = 0;
            HIPCHK_M(this, hipSetDevice(ctx_device(g.ctx)));
            HIPCHK_M(this, hipMalloc(&d_red, (size_t)n * sizeof(double)));
            red_cap = (size_t)n;
        }
        HIPCHK_M(this, hipMemcpyAsync(d_red, v, (size_t)n * sizeof(double), hipMemcpyHostToDevice, st));
        NCCLCHK(this, ncclAllReduce(d_red, d_red, (size_t)n, ncclFloat64, op == 1 ? ncclMax : ncclSum, comm[0], st));
        HIPCHK_M(this, hipMemcpyAsync(v, d_red, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK_M(this, hipStreamSynchronize(st));
        return 0;
    }
};

static int check_scenes(rs_mgpu* m, const rs_scene* const* scenes) {
    if (!scenes) return m->error(RS_E_INVALID, "null scene array");
    for (size_t i = 0; i < m->ranks.size(); ++i)
        if (!scenes[i]) return m->error(RS_E_INVALID, "null scene for local rank " + std::to_string(i));
    return RS_OK;
}

extern "C" int rs_mgpu_unique_id(uint8_t id[RS_MGPU_ID_BYTES]) {
    if (!id) return RS_E_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return RS_E_HIP;
    static_assert(sizeof(u.internal) == RS_MGPU_ID_BYTES, "RCCL unique id size");
    std::memcpy(id, u.internal, RS_MGPU_ID_BYTES);
    return RS_OK;
}

extern "C" int rs_mgpu_create(rs_context* ctx, int rank, int world, const uint8_t id[RS_MGPU_ID_BYTES], rs_mgpu** out) {
    if (!ctx || !out || !id || world < 1 || rank < 0 || rank >= world)
        return ctx_fail(ctx, RS_E_INVALID, "rs_mgpu_create: bad arguments");
    *out = nullptr;
    auto m = std::make_unique<rs_mgpu>();
    m->world = world;
    m->W = ctx_width(ctx); m->H = ctx_height(ctx);
    if (world > m->H) return ctx_fail(ctx, RS_E_INVALID, "rs_mgpu_create: more ranks than rows");
    m->ranks.resize(1);
    m->ranks[0].ctx = ctx;
    m->rank_ids = {rank};
    m->bounds = mgpu::equal_bounds(m->H, world);
    if (hipSetDevice(ctx_device(ctx)) != hipSuccess) return ctx_fail(ctx, RS_E_HIP, "rs_mgpu_create: hipSetDevice");
    ncclUniqueId u;
    std::memcpy(u.internal, id, RS_MGPU_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&m->comm[0], world, u, rank);
    if (r != ncclSuccess) return ctx_fail(ctx, RS_E_HIP, std::string("rs_mgpu_create: ncclCommInitRank -> ") + ncclGetErrorString(r));
    for (int k = 1; k < kLanes; ++k) {          // one communicator per run-ahead lane
        r = ncclCommSplit(m->comm[0], 0, rank, &m->comm[k], nullptr);
        if (r != ncclSuccess) {
            for (auto& c : m->comm) if (c) ncclCommDestroy(c);
            return ctx_fail(ctx, RS_E_HIP, std::string("rs_mgpu_create: ncclCommSplit -> ") + ncclGetErrorString(r));
        }
    }
    *out = m.release();
    return RS_OK;
}

extern "C" int rs_mgpu_create_local(rs_context* const* ctxs, int world, rs_mgpu** out) {
    if (!ctxs || !out || world < 1) return ctx_fail(nullptr, RS_E_INVALID, "rs_mgpu_create_local: bad arguments");
    *out = nullptr;
    auto m = std::make_unique<rs_mgpu>();
    m->local = true;
    m->world = world;
    m->W = ctx_width(ctxs[0]); m->H = ctx_height(ctxs[0]);
    if (world > m->H) return ctx_fail(ctxs[0], RS_E_INVALID, "rs_mgpu_create_local: more ranks than rows");
    m->ranks.resize(world);
    for (int i = 0; i < world; ++i) {
        if (!ctxs[i] || ctx_width(ctxs[i]) != m->W || ctx_height(ctxs[i]) != m->H)
            return ctx_fail(ctxs[0], RS_E_INVALID, "rs_mgpu_create_local: contexts must share the frame size");
        m->ranks[i].ctx = ctxs[i];
        m->rank_ids.push_back(i);
    }
    m->bounds = mgpu::equal_bounds(m->H, world);
    m->ev_a.resize(world); m->ev_b.resize(world);
    for (int i = 0; i < world; ++i) {
        if (hipSetDevice(ctx_device(ctxs[i])) != hipSuccess ||
            hipEventCreateWithFlags(&m->ev_a[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&m->ev_b[i], hipEventDisableTiming) != hipSuccess)
            return ctx_fail(ctxs[0], RS_E_HIP, "rs_mgpu_create_local: hipEventCreate");
    }
    *out = m.release();
    return RS_OK;
}

extern "C" void rs_mgpu_destroy(rs_mgpu* m) {
    if (!m) return;
    for (auto& g : m->ranks) if (g.ctx) rs_synchronize(g.ctx);   // every frame's transfers joined it
    for (auto& c : m->comm) if (c) ncclCommDestroy(c);
    for (auto& slot : m->sev)
        for (auto e : slot) if (e) hipEventDestroy(e);
    for (auto e : m->ev_a) if (e) hipEventDestroy(e);
    for (auto e : m->ev_b) if (e) hipEventDestroy(e);
    if (m->d_red) hipFree(m->d_red);
    delete m;
}

extern "C" int rs_mgpu_set_bands(rs_mgpu* m, const int32_t* bounds) {
    if (!m || !bounds) return RS_E_INVALID;
    std::vector<int> b(bounds, bounds + m->world + 1);
    if (!mgpu::valid_bounds(b, m->H, m->world))
        return m->error(RS_E_INVALID, "rs_mgpu_set_bands: bounds must rise from 0 to H, one band per rank");
    for (auto& g : m->ranks) rs_synchronize(g.ctx);
    m->bounds = b;
    return RS_OK;
}

extern "C" int rs_mgpu_get_bands(const rs_mgpu* m, int32_t* bounds) {
    if (!m || !bounds) return RS_E_INVALID;
    for (int i = 0; i <= m->world; ++i) bounds[i] = m->bounds[i];
    return RS_OK;
}

extern "C" int rs_mgpu_render_frame(rs_mgpu* m, const rs_scene* const* scenes, const rs_camera* cam,
                                    const rs_frame_params* P, uint32_t frame_index, int gather, float* frame_rgb_host,
                                    rs_pass_times* times) {
    if (!m || !cam || !P) return RS_E_INVALID;
    if (int rc = check_scenes(m, scenes)) return rc;
    const int halo = m->world > 1 ? mgpu::halo_rows(P->spatial_radius, P->do_spatial && P->spatial_passes > 0) : 0;
    for (int r = 0; r < m->world; ++r)
        if (halo && m->bounds[r + 1] - m->bounds[r] < halo)
            return m->error(RS_E_INVALID, "a band is thinner than the spatial halo: too many ranks for the frame height");
    m->rank_ptrs.clear();
    for (size_t i = 0; i < m->ranks.size(); ++i) {
        GpuRank& g = m->ranks[i];
        g.scene = scenes[i]; g.cam = *cam; g.P = *P; g.frame = frame_index;
        g.times = i == 0 ? times : nullptr;
        m->rank_ptrs.push_back(&g);
    }
    m->halo_bytes = (size_t)halo * m->W * 3 * sizeof(float) * 4;    // h rows x W x 48-B reservoirs
    if (m->world > 1)
        if (int rc = m->begin_frame_stats()) return rc;
    // G-buffer margin = the halo: a temporal reprojection beyond a tile's rows rebuilds its element
    if (int rc = mgpu::render_frame(m->rank_ptrs, *m, m->bounds, m->rank_ids, P->do_spatial ? P->spatial_passes : 0,
                                    halo, halo, gather != 0))
        return rc;
    if (frame_rgb_host && m->rank_ids[0] == 0) {
        uint64_t t = 0;
        if (int rc = rs_frame_readback(m->ranks[0].ctx, frame_rgb_host, &t)) return rc;
        if (int rc = rs_frame_wait(m->ranks[0].ctx, t)) return rc;
    }
    return RS_OK;
}

extern "C" int rs_mgpu_frame_device_ptr(rs_mgpu* m, const float** dptr) {
    if (!m || !dptr) return RS_E_INVALID;
    return rs_get_frame_device_ptr(m->ranks[0].ctx, dptr);
}

extern "C" int rs_mgpu_reset_history(rs_mgpu* m) {
    if (!m) return RS_E_INVALID;
    for (auto& g : m->ranks)
        if (int rc = rs_reset_history(g.ctx)) return rc;
    return RS_OK;
}

extern "C" int rs_mgpu_get_stats(rs_mgpu* m, rs_mgpu_stats* out, int reset) {
    if (!m || !out) return RS_E_INVALID;
    for (auto& g : m->ranks)
        if (int rc = rs_synchronize(g.ctx)) return rc;
    for (int k = 0; k < rs_mgpu::kStatRing; ++k) m->fold(k);
    *out = m->stats;
    if (reset) m->stats = rs_mgpu_stats{};
    return RS_OK;
}

extern "C" int rs_mgpu_allreduce(rs_mgpu* m, double* values, int n, int op) {
    if (!m || !values || n <= 0 || (op != 0 && op != 1)) return RS_E_INVALID;
    return m->allreduce(values, n, op);
}

extern "C" int rs_mgpu_set_rebalance_refine(rs_mgpu* m, int rounds) {
    if (!m || rounds < 0 || rounds > 8) return RS_E_INVALID;
    m->refine = rounds;
    return RS_OK;
}

// Each rank's own time per frame with `bounds`: `warm` unmeasured frames (the history after a boundary move,
// lazily grown buffers), then `n` frames with the gather.  A rank's time is its frames' begin..shade span
// (rs_pass_times.total_ms, event ring, frames in flight as in production) minus the halo exchanges on its
// own stream (which include waiting for slower neighbours), plus -- on global rank 0 -- the gather it
// receives.  Every local rank has its own exchange spans (rs_mgpu::halo_ms_rank), so no local rank looks
// cheaper than another.  The caller's timing totals and transfer statistics are read as deltas, not reset.
// All-reduced, so every rank sees the same vector and makes the same choice.
static int measure_bands(rs_mgpu* m, const rs_scene* const* scenes, const rs_camera* cam, const rs_frame_params* P,
                         uint32_t& frame, int warm, int n, std::vector<double>& t) {
    if (int rc = rs_mgpu_reset_history(m)) return rc;   // the previous G-buffer rows of a moved band
    for (int f = 0; f < warm; ++f)
        if (int rc = rs_mgpu_render_frame(m, scenes, cam, P, frame++, 1, nullptr, nullptr)) return rc;
    const size_t nl = m->ranks.size();
    std::vector<double> ms0(nl), halo0, gather0;
    std::vector<uint32_t> nf0(nl);
    rs_mgpu_stats st{};
    if (int rc = rs_mgpu_get_stats(m, &st, 0)) return rc;   // folds every finished frame's spans
    halo0 = m->halo_ms_rank; gather0 = m->gather_ms_rank;
    for (size_t i = 0; i < nl; ++i) {
        rs_pass_times sum{};
        if (int rc = rs_get_timing_totals(m->ranks[i].ctx, &sum, &nf0[i], 0)) return rc;
        ms0[i] = sum.total_ms;
    }
    for (int f = 0; f < n; ++f)
        if (int rc = rs_mgpu_render_frame(m, scenes, cam, P, frame++, 1, nullptr, nullptr)) return rc;
    if (int rc = rs_mgpu_get_stats(m, &st, 0)) return rc;
    t.assign(m->world, 0.0);
    for (size_t i = 0; i < nl; ++i) {
        rs_pass_times sum{};
        uint32_t nf = 0;
        if (int rc = rs_get_timing_totals(m->ranks[i].ctx, &sum, &nf, 0)) return rc;
        double v = (sum.total_ms - ms0[i]) - (m->halo_ms_rank[i] - halo0[i]);
        if (m->rank_ids[i] == 0) v += m->gather_ms_rank[i] - gather0[i];
        t[m->rank_ids[i]] = std::max(0.0, v) / std::max<uint32_t>(1, nf - nf0[i]);
    }
    return m->allreduce(t.data(), m->world, 0);
}

constexpr int kBandGrain = 8;                // band boundaries on whole 8-row wave tiles (balanced_bounds_grain)

extern "C" int rs_mgpu_rebalance(rs_mgpu* m, const rs_scene* const* scenes, const rs_camera* cam,
                                 const rs_frame_params* P, uint32_t first_frame, int n_frames, int min_rows) {
    if (!m || !cam || !P || n_frames < 1) return RS_E_INVALID;
    if (int rc = check_scenes(m, scenes)) return rc;
    if (m->world == 1) return RS_OK;
    m->rebalance_ms.clear();
    for (auto& g : m->ranks) {
        if (int rc = rs_context_track_row_costs(g.ctx, 1)) return rc;
        std::vector<float> tmp(m->H);
        if (int rc = rs_get_row_costs(g.ctx, tmp.data(), 1)) return rc;   // start from zero
    }
    for (int f = 0; f < n_frames; ++f)
        if (int rc = rs_mgpu_render_frame(m, scenes, cam, P, first_frame + (uint32_t)f, 0, nullptr, nullptr)) return rc;
    std::vector<double> cost(m->H, 0.0);
    std::vector<float> tmp(m->H);
    for (auto& g : m->ranks) {
        if (int rc = rs_get_row_costs(g.ctx, tmp.data(), 1)) return rc;
        for (int y = 0; y < m->H; ++y) cost[y] += tmp[y];
        if (int rc = rs_context_track_row_costs(g.ctx, 0)) return rc;
    }
    if (int rc = m->allreduce(cost.data(), m->H, 0)) return rc;
    const int halo = mgpu::halo_rows(P->spatial_radius, P->do_spatial && P->spatial_passes > 0);
    std::vector<int> b;
    const int rows = std::max(std::max(1, min_rows), halo);
    if (!mgpu::balanced_bounds_grain(cost, m->world, rows, kBandGrain, b))
        return m->error(RS_E_INVALID, "rs_mgpu_rebalance: bands of min_rows do not fit");
    m->bounds = b;
    // Time-based refinement: row costs predict a band's time only to about +-7 % (the per-row
    // wave time misses what a band pays as a launch: rounds of waves, the split pass, halo and gather).  Each
    // round measures every rank's time with the current bounds, rescales each band's row costs so that they sum
    // to its measured time, and balances again; the bounds with the lowest measured maximum are kept.  (C4 at
    // 8 ranks, every band timed alone on one MI355X: slowest band 9.09 -> 8.96 -> 8.80 ms over two rounds,
    // profiles/r04_band_refine_C4_N8.txt.)
    uint32_t frame = first_frame + (uint32_t)n_frames;
    std::vector<int> best = b;
    double best_max = 0.0;
    const int n_meas = std::max(n_frames, 6);
    for (int it = 0; it <= m->refine && m->refine > 0; ++it) {
        std::vector<double> t;
        if (int rc = measure_bands(m, scenes, cam, P, frame, 2, n_meas, t)) return rc;
        const double mx = *std::max_element(t.begin(), t.end());
        m->rebalance_ms.push_back(t);
        if (it == 0 || mx < best_max) { best_max = mx; best = m->bounds; }
        if (it == m->refine) break;
        for (int r = 0; r < m->world; ++r) {    // band r's rows rescaled to its measured time
            double c = 0.0;
            for (int y = m->bounds[r]; y < m->bounds[r + 1]; ++y) c += cost[y];
            if (c > 0.0 && t[r] > 0.0)
                for (int y = m->bounds[r]; y < m->bounds[r + 1]; ++y) cost[y] *= t[r] / c;
        }
        std::vector<int> nb;
        if (!mgpu::balanced_bounds_grain(cost, m->world, rows, kBandGrain, nb)) break;
        if (nb == m->bounds) break;              // converged: nothing left to measure
        m->bounds = nb;
    }
    m->bounds = best;
    return rs_mgpu_reset_history(m);   // the previous G-buffer rows of a moved band belong to another rank
}

extern "C" int rs_mgpu_rebalance_times(const rs_mgpu* m, int round, double* ms) {
    if (!m || !ms || round < 0 || round >= (int)m->rebalance_ms.size()) return RS_E_INVALID;
    for (int r = 0; r < m->world; ++r) ms[r] = m->rebalance_ms[round][r];
    return RS_OK;
}
