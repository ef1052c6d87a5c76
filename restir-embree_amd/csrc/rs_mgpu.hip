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

constexpr int kLanes = 3;   // run-ahead lanes of a context (restir_capi.hip kMaxAhead + 1)

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
        if (rs_tile_halo_ptr(ctx, which, &p, bytes) != RS_OK) return nullptr;
        return p;
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
    double* d_red = nullptr;                    // RCCL all-reduce scratch (rows of costs / a few scalars)
    size_t red_cap = 0;
    std::string err;
    int error(int code, const std::string& m) {
        err = m;
        return ctx_fail(ranks.empty() ? nullptr : ranks[0].ctx, code, "rs_mgpu: " + m);
    }

    // ---- halo exchange (the Comm interface of rs::mgpu::render_frame)
    int exchange_halo(std::vector<GpuRank*>& rk, int pass) {
        (void)pass;
        if (world == 1) return 0;
        if (!local) {
            GpuRank& g = *rk[0];
            const int r = rank_ids[0];
            size_t bs = 0, br = 0;
            NCCLCHK(this, ncclGroupStart());
            for (int side = 0; side < 2; ++side) {
                const int peer = side == 0 ? r - 1 : r + 1;
                if (peer < 0 || peer >= world) continue;
                void* snd = g.halo(side == 0 ? 2 : 3, &bs);
                void* rcv = g.halo(side == 0 ? 0 : 1, &br);
                if (!snd || !rcv) continue;
                ncclSend(snd, bs, ncclUint8, peer, comm[g.lane], g.st);
                ncclRecv(rcv, br, ncclUint8, peer, comm[g.lane], g.st);
            }
            NCCLCHK(this, ncclGroupEnd());
            return 0;
        }
        // local: every rank's stream waits for its neighbours' last stage, copies their edge rows into its
        // halo rows; then the neighbours wait for those copies (their next pass writes the buffer read)
        const int n = (int)rk.size();
        for (int i = 0; i < n; ++i) HIPCHK_M(this, hipEventRecord(ev_a[i], rk[i]->st));
        for (int i = 0; i < n; ++i) {
            for (int side = 0; side < 2; ++side) {
                const int j = side == 0 ? i - 1 : i + 1;
                if (j < 0 || j >= n) continue;
                size_t bs = 0, br = 0;
                void* snd = rk[j]->halo(side == 0 ? 3 : 2, &bs);
                void* rcv = rk[i]->halo(side == 0 ? 0 : 1, &br);
                if (!snd || !rcv || bs != br) continue;
                HIPCHK_M(this, hipStreamWaitEvent(rk[i]->st, ev_a[j], 0));
                HIPCHK_M(this, hipMemcpyAsync(rcv, snd, br, hipMemcpyDeviceToDevice, rk[i]->st));
            }
        }
        for (int i = 0; i < n; ++i) HIPCHK_M(this, hipEventRecord(ev_b[i], rk[i]->st));
        for (int i = 0; i < n; ++i)
            for (int j : {i - 1, i + 1})
                if (j >= 0 && j < n) HIPCHK_M(this, hipStreamWaitEvent(rk[i]->st, ev_b[j], 0));
        return 0;
    }

    // ---- gather: band framebuffers -> rank 0's context framebuffer (full frame, rows at their place)
    int gather(std::vector<GpuRank*>& rk) {
        if (world == 1) return 0;
        const size_t row = (size_t)W * 3;
        if (!local) {
            GpuRank& g = *rk[0];
            const int r = rank_ids[0];
            NCCLCHK(this, ncclGroupStart());
            if (r == 0) {
                float* full = const_cast<float*>(g.band) - (size_t)g.y0 * row;
                for (int q = 1; q < world; ++q)
                    ncclRecv(full + (size_t)bounds[q] * row, (size_t)(bounds[q + 1] - bounds[q]) * row, ncclFloat32, q,
                             comm[g.lane], g.st);
            } else {
                ncclSend(g.band, (size_t)(g.y1 - g.y0) * row, ncclFloat32, 0, comm[g.lane], g.st);
            }
            NCCLCHK(this, ncclGroupEnd());
            if (r == 0) return ctx_join(g.ctx, g.st);
            return 0;
        }
        const int n = (int)rk.size();
        GpuRank& g0 = *rk[0];
        float* full = const_cast<float*>(g0.band) - (size_t)g0.y0 * row;
        for (int i = 1; i < n; ++i) {
            HIPCHK_M(this, hipEventRecord(ev_a[i], rk[i]->st));
            HIPCHK_M(this, hipStreamWaitEvent(g0.st, ev_a[i], 0));
            HIPCHK_M(this, hipMemcpyAsync(full + (size_t)rk[i]->y0 * row, rk[i]->band,
                                          (size_t)(rk[i]->y1 - rk[i]->y0) * row * sizeof(float),
                                          hipMemcpyDeviceToDevice, g0.st));
        }
        HIPCHK_M(this, hipEventRecord(ev_b[0], g0.st));
        for (int i = 1; i < n; ++i) HIPCHK_M(this, hipStreamWaitEvent(rk[i]->st, ev_b[0], 0));   // band reuse
        return ctx_join(g0.ctx, g0.st);
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
    for (auto& g : m->ranks) if (g.ctx) rs_synchronize(g.ctx);
    for (auto& c : m->comm) if (c) ncclCommDestroy(c);
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

extern "C" int rs_mgpu_allreduce(rs_mgpu* m, double* values, int n, int op) {
    if (!m || !values || n <= 0 || (op != 0 && op != 1)) return RS_E_INVALID;
    return m->allreduce(values, n, op);
}

extern "C" int rs_mgpu_rebalance(rs_mgpu* m, const rs_scene* const* scenes, const rs_camera* cam,
                                 const rs_frame_params* P, uint32_t first_frame, int n_frames, int min_rows) {
    if (!m || !cam || !P || n_frames < 1) return RS_E_INVALID;
    if (int rc = check_scenes(m, scenes)) return rc;
    if (m->world == 1) return RS_OK;
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
    if (!mgpu::balanced_bounds(cost, m->world, std::max(std::max(1, min_rows), halo), b))
        return m->error(RS_E_INVALID, "rs_mgpu_rebalance: bands of min_rows do not fit");
    m->bounds = b;
    return rs_mgpu_reset_history(m);   // the previous G-buffer rows of a moved band belong to another rank
}
