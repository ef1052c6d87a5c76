// rs_mgpu_core.h -- orchestration of a row-band sharded frame, independent of the
// device and of the transport, so the same code drives the product (librestir_amd tile stages + RCCL
// over xGMI, or device copies between contexts of one process) and a CPU test (the oracle's tile
// stages + host memcpy, tests/cpp/mgpu_core_harness.cpp via tests/test_mgpu_core.py).
//
// A frame of `world` row bands (the reference renders one frame per produceRestir call,
// pg/simpleguidx11.cpp:359-487; every rank renders its rows of it):
//   begin      every local rank: G-buffer of its rows +- margin, initial RIS (+ visibility) of its rows
//   temporal   every local rank
//   for each spatial pass p:
//     exchange the reservoir halo: rows [y0, y0+h) to the rank above and [y1-h, y1) to the rank below,
//              rows [y0-h, y0) / [y1, y1+h) from them; h = floor(sqrtf(R)) (the largest |offset| the
//              disk sample can produce, pg/Sampling.cpp:78-87 truncated, pg/ReSTIRIntegrator.cpp:338)
//     spatial(p) every local rank
//   finish     shade + history swap; band framebuffer
//   gather     bands -> rank 0's full frame (optional)
// The per-pixel counter RNG is keyed by the full-frame pixel index, so the gathered frame equals the
// single-GPU frame bit for bit whatever the bands are.
#pragma once
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rs {
namespace mgpu {

// halo rows for a spatial radius, float32 semantics as the device forms the offset
inline int halo_rows(float radius, bool spatial) {
    if (!spatial) return 0;
    const float r = radius > 0.0f ? radius : 0.0f;
    return (int)std::floor(std::sqrt(r));     // std::sqrt(float): correctly rounded like sqrtf
}

// equal row bands: rank r gets [r*H/world, (r+1)*H/world)
inline std::vector<int> equal_bounds(int H, int world) {
    std::vector<int> b(world + 1);
    for (int r = 0; r <= world; ++r) b[r] = (int)((long long)r * H / world);
    return b;
}

// Contiguous bands with (as nearly as rows allow) equal summed cost, every band >= min_rows rows.
// Deterministic: every rank computes the same split from the same all-reduced costs.  Same rule as
// restir_amd.distributed.balanced_bands (tests compare the two).
inline bool balanced_bounds(const std::vector<double>& costs_in, int world, int min_rows, std::vector<int>& out) {
    const int H = (int)costs_in.size();
    if (world <= 0 || (long long)world * min_rows > H) return false;
    std::vector<double> c(H);
    double sum = 0.0;
    for (int i = 0; i < H; ++i) {
        const double v = costs_in[i];
        c[i] = (std::isfinite(v) && v > 0.0) ? v : 0.0;
        sum += c[i];
    }
    if (sum <= 0.0) { out = equal_bounds(H, world); return true; }
    const double eps = sum * 1e-6 / H;            // no zero-cost plateaus: boundaries stay put
    std::vector<double> cum(H + 1, 0.0);
    for (int i = 0; i < H; ++i) cum[i + 1] = cum[i] + (c[i] + eps);
    out.assign(world + 1, 0);
    for (int r = 1; r < world; ++r) {
        const double target = cum[H] * r / world;
        // numpy.searchsorted(cum, target) (side='left'): first index with cum[i] >= target
        int lo = 0, hi = H + 1;
        while (lo < hi) { const int m = (lo + hi) / 2; if (cum[m] < target) lo = m + 1; else hi = m; }
        int y = lo;
        const int ymin = out[r - 1] + min_rows, ymax = H - (world - r) * min_rows;
        y = y < ymax ? y : ymax;
        y = y > ymin ? y : ymin;
        out[r] = y;
    }
    out[world] = H;
    return true;
}

// The same split in units of `grain` rows (the last unit may be short): boundaries on multiples of grain, so no
// band but the last ends in a partial 8-row wave tile (a pass launch's tiles start at the band's first row, and a
// partial tile costs a whole one: C2's 1/8 bands measured 1-5 % slower with row-exact boundaries).  Falls back to
// single rows when the height is not a multiple of grain or the bands of min_rows do not fit in whole units.
inline bool balanced_bounds_grain(const std::vector<double>& costs, int world, int min_rows, int grain,
                                  std::vector<int>& out) {
    const int H = (int)costs.size();
    const int G = grain > 1 ? (H + grain - 1) / grain : H, mg = grain > 1 ? (min_rows + grain - 1) / grain : min_rows;
    if (grain <= 1 || H % grain || (long long)world * mg > G) return balanced_bounds(costs, world, min_rows, out);
    std::vector<double> cg(G, 0.0);
    for (int y = 0; y < H; ++y) {
        const double v = costs[y];
        cg[y / grain] += (std::isfinite(v) && v > 0.0) ? v : 0.0;
    }
    if (!balanced_bounds(cg, world, mg, out)) return false;
    for (int r = 1; r < world; ++r) out[r] = std::min(out[r] * grain, H);
    out[world] = H;
    return true;
}

inline bool valid_bounds(const std::vector<int>& b, int H, int world) {
    if ((int)b.size() != world + 1 || b[0] != 0 || b[world] != H) return false;
    for (int r = 0; r < world; ++r)
        if (b[r] >= b[r + 1]) return false;
    return true;
}

// ---------------------------------------------------------------- transfer plans
// Every exchange of a frame is a list of point-to-point transfers per rank, computed from state all
// ranks share (rank, world, bounds, halo rows, frame width), so the ranks agree on every pairing without
// talking.  The same plans drive the RCCL branch (ncclSend/ncclRecv in one group on the frame's stream,
// issue_plan below), the device copies of local mode and the host copies of the CPU test (pair_local),
// and the plan checker the tests run for 2..8 ranks (check_plans).
enum : int {
    kHaloAbove = 0,    // rows [y0-h, y0): received from rank r-1        (rs_tile_halo_ptr which = 0)
    kHaloBelow = 1,    // rows [y1, y1+h): received from rank r+1        (which = 1)
    kEdgeTop = 2,      // rows [y0, y0+h): sent to rank r-1              (which = 2)
    kEdgeBottom = 3,   // rows [y1-h, y1): sent to rank r+1              (which = 3)
    kFrameRows = 4     // framebuffer rows (gather), `offset` bytes from the full frame's first row
};
struct Xfer {
    int peer;          // global rank
    bool send;
    int slot;          // kHalo* / kEdge* / kFrameRows
    size_t offset;     // kFrameRows only
    size_t bytes;
};
// Halo exchange of rank r before a spatial pass (every slot holds halo_bytes = h rows x W x 48 B):
// its top edge rows go to r-1 and r-1's bottom edge rows land in its halo above; symmetrically below.
inline std::vector<Xfer> halo_plan(int r, int world, size_t halo_bytes) {
    std::vector<Xfer> p;
    if (halo_bytes == 0) return p;
    if (r > 0) {
        p.push_back({r - 1, true, kEdgeTop, 0, halo_bytes});
        p.push_back({r - 1, false, kHaloAbove, 0, halo_bytes});
    }
    if (r + 1 < world) {
        p.push_back({r + 1, true, kEdgeBottom, 0, halo_bytes});
        p.push_back({r + 1, false, kHaloBelow, 0, halo_bytes});
    }
    return p;
}
// the neighbour's slot a halo slot is filled from
inline int halo_source_slot(int recv_slot) { return recv_slot == kHaloAbove ? kEdgeBottom : kEdgeTop; }
// Gather into rank 0's full frame: rank q > 0 sends its rows [bounds[q], bounds[q+1]); rank 0 receives each
// band at the same rows of its frame (row_bytes = W x 12 B).
inline std::vector<Xfer> gather_plan(int r, const std::vector<int>& bounds, size_t row_bytes) {
    std::vector<Xfer> p;
    const int world = (int)bounds.size() - 1;
    if (world <= 1) return p;
    if (r == 0) {
        for (int q = 1; q < world; ++q)
            p.push_back({q, false, kFrameRows, (size_t)bounds[q] * row_bytes, (size_t)(bounds[q + 1] - bounds[q]) * row_bytes});
    } else {
        p.push_back({0, true, kFrameRows, (size_t)bounds[r] * row_bytes, (size_t)(bounds[r + 1] - bounds[r]) * row_bytes});
    }
    return p;
}
// does send `s` of rank `rs` fill recv `x` of rank `rx`?
inline bool xfer_matches(const Xfer& x, int rx, const Xfer& s, int rs) {
    if (x.send || !s.send || x.peer != rs || s.peer != rx || x.bytes != s.bytes) return false;
    if (x.slot == kFrameRows) return s.slot == kFrameRows && s.offset == x.offset;
    return s.slot == halo_source_slot(x.slot);
}
// A world of plans (plans[r] = rank r's) is consistent when every recv has exactly one matching send of
// the same size, every send exactly one matching recv, and no rank talks to itself or to a rank outside
// the world.  Returns "" or a description of the first violation.
inline std::string check_plans(const std::vector<std::vector<Xfer>>& plans) {
    const int world = (int)plans.size();
    for (int r = 0; r < world; ++r)
        for (const Xfer& x : plans[r]) {
            if (x.peer < 0 || x.peer >= world || x.peer == r)
                return "rank " + std::to_string(r) + ": transfer with peer " + std::to_string(x.peer);
            int n = 0;
            for (const Xfer& y : plans[x.peer])
                n += x.send ? xfer_matches(y, x.peer, x, r) : xfer_matches(x, r, y, x.peer);
            if (n != 1)
                return "rank " + std::to_string(r) + (x.send ? " send to " : " recv from ") + std::to_string(x.peer) +
                       " (slot " + std::to_string(x.slot) + ", " + std::to_string(x.bytes) + " B): " +
                       std::to_string(n) + " matching entries";
        }
    return "";
}
inline size_t plan_bytes(const std::vector<Xfer>& p, bool send) {
    size_t b = 0;
    for (const Xfer& x : p) b += x.send == send ? x.bytes : 0;
    return b;
}

// Issues one rank's plan through `link` (int group_start(), send(const void*, size_t, int peer),
// recv(void*, size_t, int peer), group_end(); each returns 0 or an error).  Every buffer is resolved and
// size-checked before the first call, so a missing halo is an error raised before the group starts
// instead of a send whose peer never posts the matching recv.  `g` provides
//   void* halo(int slot, size_t* bytes)   and   char* frame_base()   (the full-frame framebuffer).
template <class Rank, class Link>
int issue_plan(Rank& g, const std::vector<Xfer>& plan, Link& link) {
    std::vector<void*> ptr(plan.size());
    for (size_t k = 0; k < plan.size(); ++k) {
        const Xfer& x = plan[k];
        if (x.slot == kFrameRows) {
            char* base = g.frame_base();
            ptr[k] = base ? base + x.offset : nullptr;
        } else {
            size_t b = 0;
            ptr[k] = g.halo(x.slot, &b);
            if (b != x.bytes) ptr[k] = nullptr;
        }
        if (!ptr[k]) return -2;                      // before any transfer of the group is posted
    }
    if (plan.empty()) return 0;
    if (int rc = link.group_start()) return rc;
    for (size_t k = 0; k < plan.size(); ++k) {
        const Xfer& x = plan[k];
        const int rc = x.send ? link.send(ptr[k], x.bytes, x.peer) : link.recv(ptr[k], x.bytes, x.peer);
        if (rc) { link.group_end(); return rc; }
    }
    return link.group_end();
}

// All ranks in one process (local mode, the CPU test): calls copy(i, x, j, y) for every recv x of local rank
// i with the send y of local rank j that fills it (plans[i] belongs to global rank ids[i]).  Returns -1 when
// a recv has no matching send among the local ranks.
template <class F>
int pair_local(const std::vector<std::vector<Xfer>>& plans, const std::vector<int>& ids, F&& copy) {
    const int n = (int)plans.size();
    for (int i = 0; i < n; ++i)
        for (const Xfer& x : plans[i]) {
            if (x.send) continue;
            int j = -1;
            for (int q = 0; q < n; ++q) if (ids[q] == x.peer) j = q;
            if (j < 0) return -1;
            const Xfer* y = nullptr;
            for (const Xfer& s : plans[j]) if (xfer_matches(x, ids[i], s, ids[j])) { y = &s; break; }
            if (!y) return -1;
            if (int rc = copy(i, x, j, *y)) return rc;
        }
    return 0;
}

// One frame through the tile stages of the local ranks.  `Local` is a sequence of rank objects with
//   int begin(int y0, int y1, int margin, int halo)   int temporal()   int spatial(int pass)
//   int finish()   (each returns 0 on success)
// and `Comm` provides
//   int exchange_halo(Local& ranks, int pass)   int gather(Local& ranks)
// Bands and halo come from the caller; every stage is issued for every local rank before the next
// stage, so independent ranks (threads of work on different devices / streams) overlap.
template <class Local, class Comm>
int render_frame(Local& ranks, Comm& comm, const std::vector<int>& bounds, const std::vector<int>& rank_ids,
                 int spatial_passes, int halo, int margin, bool gather) {
    const int n = (int)rank_ids.size();
    const int world = (int)bounds.size() - 1;
    for (int r = 0; r < world; ++r)                  // a neighbour's halo must lie inside the adjacent band
        if (halo > 0 && bounds[r + 1] - bounds[r] < halo) return -1;   // RS_E_INVALID
    for (int i = 0; i < n; ++i) {
        const int r = rank_ids[i];
        if (int rc = ranks[i]->begin(bounds[r], bounds[r + 1], margin, halo)) return rc;
    }
    for (int i = 0; i < n; ++i)
        if (int rc = ranks[i]->temporal()) return rc;
    for (int p = 0; p < spatial_passes; ++p) {
        if (halo > 0)
            if (int rc = comm.exchange_halo(ranks, p)) return rc;
        for (int i = 0; i < n; ++i)
            if (int rc = ranks[i]->spatial(p)) return rc;
    }
    for (int i = 0; i < n; ++i)
        if (int rc = ranks[i]->finish()) return rc;
    if (gather)
        if (int rc = comm.gather(ranks)) return rc;
    return 0;
}

}  // namespace mgpu
}  // namespace rs
