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

inline bool valid_bounds(const std::vector<int>& b, int H, int world) {
    if ((int)b.size() != world + 1 || b[0] != 0 || b[world] != H) return false;
    for (int r = 0; r < world; ++r)
        if (b[r] >= b[r + 1]) return false;
    return true;
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
