// TEST INFRASTRUCTURE: runs the RCCL branch of rs_mgpu (csrc/rs_mgpu.hip: rs_mgpu_create with a unique id,
// per-lane communicators, NcclLink halo exchanges and gathers, rs_mgpu_rebalance's all-reduce) with `world`
// ranks as threads of one process on one GPU, linked against tests/cpp/rccl_stub.cpp instead of librccl, and
// checks every gathered frame bit for bit against one context rendering the same frames.
//   mgpu_rccl_driver <scene.obj> W H world frames eye(3) at(3) fov temporal(0/1)
// Prints one JSON line; exit 0 iff every frame is identical and the stub saw no unpaired / mismatched transfer.
#include "../../include/restir.hpp"

#include <barrier>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

extern "C" void rccl_stub_stats(long* pairs, long* bytes, long* mismatches, long* unpaired, long* allreduces);

int main(int argc, char** argv) {
    if (argc < 14) { std::fprintf(stderr, "usage: %s obj W H world frames ex ey ez ax ay az fov temporal\n", argv[0]); return 2; }
    const char* obj = argv[1];
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), world = std::atoi(argv[4]), frames = std::atoi(argv[5]);
    restir::Camera cam(std::atof(argv[6]), std::atof(argv[7]), std::atof(argv[8]), std::atof(argv[9]), std::atof(argv[10]),
                       std::atof(argv[11]), std::atof(argv[12]));
    restir::Params P;
    P.m_area = 8; P.m_brdf = 1; P.spatial_neighbors = 4; P.spatial_passes = 2; P.do_spatial = 1;
    P.do_temporal = std::atoi(argv[13]);
    const size_t px = (size_t)W * H * 3;
    // frame sequence: `frames` frames, a rebalance (2 frames, history reset), `frames` more
    const uint32_t f_after = (uint32_t)frames + 2;
    std::vector<std::vector<float>> ref;
    try {
        restir::Renderer r(W, H);
        r.LoadScene(obj);
        r.camera_ = cam;
        r.params = P;
        r.timePasses = false;
        for (int i = 0; i < 2 * frames; ++i) {
            if (i == frames) { r.resetHistory(); r.frameCtr = f_after; }
            r.produceRestir();
            ref.emplace_back(r.frame_data(), r.frame_data() + px);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "reference: %s\n", e.what());
        return 1;
    }
    std::vector<restir::Renderer*> rk;
    for (int i = 0; i < world; ++i) {
        rk.push_back(new restir::Renderer(W, H));
        rk.back()->LoadScene(obj);
    }
    uint8_t id[RS_MGPU_ID_BYTES];
    if (rs_mgpu_unique_id(id) != RS_OK) { std::fprintf(stderr, "unique id\n"); return 1; }
    std::vector<int> fail(world, 0);
    std::vector<std::string> msg(world);
    int bad_frames = 0;
    std::vector<int> bands(world + 1, 0);
    int refine_rounds = 0;                      // measured rounds of the rebalance's time-based refinement
    std::barrier sync(world);
    auto run = [&](int i) {
        rs_mgpu* m = nullptr;
        auto chk = [&](int rc, const char* what) {
            if (rc != RS_OK && !fail[i]) { fail[i] = rc; msg[i] = std::string(what) + ": " + rs_last_error(rk[i]->handle()); }
            return rc == RS_OK;
        };
        if (!chk(rs_mgpu_create(rk[i]->handle(), i, world, id, &m), "rs_mgpu_create")) { sync.arrive_and_drop(); return; }
        const rs_scene* s = rk[i]->scene_handle();
        std::vector<float> host(i == 0 ? px : 0);
        auto frame = [&](uint32_t f, int k) {
            if (!chk(rs_mgpu_render_frame(m, &s, &cam, &P, f, 1, i == 0 ? host.data() : nullptr, nullptr), "render")) return;
            if (i == 0 && std::memcmp(host.data(), ref[k].data(), px * sizeof(float)) != 0) ++bad_frames;
        };
        for (int k = 0; k < frames; ++k) frame((uint32_t)k, k);
        chk(rs_mgpu_rebalance(m, &s, &cam, &P, (uint32_t)frames, 2, 6), "rebalance");
        if (i == 0) {
            rs_mgpu_get_bands(m, bands.data());
            std::vector<double> ms(world);
            while (rs_mgpu_rebalance_times(m, refine_rounds, ms.data()) == RS_OK) ++refine_rounds;
        }
        for (int k = 0; k < frames; ++k) frame(f_after + (uint32_t)k, frames + k);
        rs_mgpu_stats st{};
        chk(rs_mgpu_get_stats(m, &st, 0), "stats");
        sync.arrive_and_wait();                 // nobody tears down a communicator a peer still uses
        rs_mgpu_destroy(m);
    };
    std::vector<std::thread> th;
    for (int i = 0; i < world; ++i) th.emplace_back(run, i);
    for (auto& t : th) t.join();
    long pairs, bytes, mism, unp, ar;
    rccl_stub_stats(&pairs, &bytes, &mism, &unp, &ar);
    int nfail = 0;
    for (int i = 0; i < world; ++i) if (fail[i]) { ++nfail; std::fprintf(stderr, "rank %d: %s\n", i, msg[i].c_str()); }
    std::printf("{\"world\": %d, \"frames\": %d, \"bad_frames\": %d, \"rank_errors\": %d, \"bands\": [", world, 2 * frames, bad_frames, nfail);
    for (int i = 0; i <= world; ++i) std::printf("%s%d", i ? ", " : "", bands[i]);
    std::printf("], \"refine_rounds\": %d, \"pairs\": %ld, \"bytes\": %ld, \"mismatches\": %ld, \"unpaired\": %ld, \"allreduces\": %ld}\n",
                refine_rounds, pairs, bytes, mism, unp, ar);
    for (auto* r : rk) delete r;
    return (bad_frames || nfail || mism || unp || pairs == 0 || ar == 0) ? 1 : 0;
}
