// TEST INFRASTRUCTURE: the native multi-GPU orchestration (restir-embree_amd/csrc/rs_mgpu_core.h, the
// code rs_mgpu_render_frame runs) driven on the CPU: every rank is an oracle context rendering its band
// with the oracle's tile stages (or_tile_*), the halo exchange and gather are host memcpys between the
// ranks' buffers.  Built by tests/test_mgpu_core.py (g++), loaded with ctypes.
#include "../../restir-embree_amd/csrc/rs_mgpu_core.h"

#include <cstdint>
#include <cstring>
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
    int W, y0 = 0, y1 = 0;
    std::vector<float> band;
    int begin(int a, int b, int margin, int halo) {
        y0 = a; y1 = b;
        return or_tile_begin(ctx, scene, cam7, P, frame, a, b, margin, halo);
    }
    int temporal() { return or_tile_temporal(ctx); }
    int spatial(int p) { return or_tile_spatial(ctx, p); }
    int finish() {
        band.assign((size_t)(y1 - y0) * W * 3, 0.0f);
        uint64_t rays = 0;
        return or_tile_finish(ctx, band.data(), &rays);
    }
    void* halo(int which, size_t* bytes) {
        void* p = nullptr;
        *bytes = 0;
        or_tile_halo_ptr(ctx, which, &p, bytes);
        return p;
    }
};

struct HostComm {
    float* full;
    int W;
    int exchanges = 0;
    int exchange_halo(std::vector<OracleRank*>& rk, int) {
        const int n = (int)rk.size();
        for (int i = 0; i < n; ++i)
            for (int side = 0; side < 2; ++side) {
                const int j = side == 0 ? i - 1 : i + 1;
                if (j < 0 || j >= n) continue;
                size_t bs = 0, br = 0;
                void* snd = rk[j]->halo(side == 0 ? 3 : 2, &bs);
                void* rcv = rk[i]->halo(side == 0 ? 0 : 1, &br);
                if (!snd || !rcv || bs != br) return -10;
                std::memcpy(rcv, snd, br);
                ++exchanges;
            }
        return 0;
    }
    int gather(std::vector<OracleRank*>& rk) {
        for (auto* r : rk) std::memcpy(full + (size_t)r->y0 * W * 3, r->band.data(), r->band.size() * sizeof(float));
        return 0;
    }
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
        ranks[i] = OracleRank{ctxs[i], scenes[i], cam7, params, frame, W};
        ptrs[i] = &ranks[i];
        ids[i] = i;
    }
    HostComm comm{full, W};
    const int halo = n > 1 ? rs::mgpu::halo_rows(radius, spatial != 0 && spatial_passes > 0) : 0;
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
int harness_halo(float radius) { return rs::mgpu::halo_rows(radius, true); }
}
