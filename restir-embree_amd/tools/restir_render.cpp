// restir_render -- C++ host driver over include/restir.hpp: loads an OBJ/MTL scene (or builds the C1
// Cornell box), renders N frames of the ReSTIR path on the GPU and prints per-pass times; optionally
// writes the last frame as a PFM.  Mirrors the reference's tutorial_3 -> Producer loop
// (pg/tutorials.cpp:27-42, pg/simpleguidx11.cpp:223-334) without the UI.
//
//   restir_render [--obj file.obj] [--w 1920 --h 1080] [--frames 10] [--area 32] [--brdf 1]
//                 [--spatial k] [--temporal] [--out frame.pfm] [--eye x y z --at x y z --fov deg]
//                 [--bench] [--ranks N [--compare]] [--denoise weights.tza [--png display.png]]
// --bench: the drop-in throughput -- frames/s of produceRestir with frame_data landing in host memory
// every frame, pipelined (pipelineDepth 2 and 1: readbacks overlapping the next frames, timePasses off)
// and with the reference's synchronous semantics; one JSON line.
// --ranks N: the frames as N row bands, one context per rank (HIP device rank % device count) driven from
// this thread through rs_mgpu_create_local / rs_mgpu_render_frame (halo exchange + gather by device
// copies); --compare also renders them on one context and reports whether every frame is bit-identical.
#include "../../include/restir.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <memory>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static void quad(std::vector<float>& P, std::vector<float>& N, const float a[3], const float b[3], const float c[3],
                 const float d[3], const float n[3]) {
    const float* t[6] = {a, b, c, a, c, d};
    for (auto* v : t) { P.insert(P.end(), v, v + 3); N.insert(N.end(), n, n + 3); }
}

static void write_pfm(const std::string& path, int W, int H, const float* rgb) {
    FILE* fp = std::fopen(path.c_str(), "wb");
    if (!fp) throw restir::Error(RS_E_IO, "cannot write " + path);
    std::fprintf(fp, "PF\n%d %d\n-1.0\n", W, H);
    for (int y = H - 1; y >= 0; --y) std::fwrite(rgb + (size_t)y * W * 3, 4, (size_t)W * 3, fp);
    std::fclose(fp);
}

int main(int argc, char** argv) {
    std::string obj, out, denoise_w, png;
    int W = 512, H = 512, frames = 5;
    bool bench = false, cam_set = false, compare = false;
    int ranks = 0;
    float eye[3] = {0, 0, 0}, at[3] = {0, 0, 0}, fov = 40.0f;
    restir::Renderer* rp = nullptr;
    restir::Params prm;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() { return i + 1 < argc ? argv[++i] : (char*)"0"; };
        if (a == "--obj") obj = next();
        else if (a == "--w") W = std::atoi(next());
        else if (a == "--h") H = std::atoi(next());
        else if (a == "--frames") frames = std::atoi(next());
        else if (a == "--area") prm.m_area = std::atoi(next());
        else if (a == "--brdf") prm.m_brdf = std::atoi(next());
        else if (a == "--spatial") { prm.do_spatial = 1; prm.spatial_neighbors = std::atoi(next()); }
        else if (a == "--temporal") prm.do_temporal = 1;
        else if (a == "--out") out = next();
        else if (a == "--bench") bench = true;
        else if (a == "--ranks") ranks = std::atoi(next());
        else if (a == "--compare") compare = true;
        else if (a == "--denoise") denoise_w = next();
        else if (a == "--png") png = next();
        else if (a == "--eye") { for (float& v : eye) v = (float)std::atof(next()); cam_set = true; }
        else if (a == "--at") { for (float& v : at) v = (float)std::atof(next()); cam_set = true; }
        else if (a == "--fov") fov = (float)std::atof(next());
    }
    // Raytracer::LoadScene: the OBJ file, or the C1 Cornell box built in memory
    auto load = [&](restir::Renderer& r) {
        if (!obj.empty()) {
            r.LoadScene(obj);
            r.camera_ = restir::Camera(1.878f, -7.724f, 1.602f, 0, 0, 0, 55.0f);   // tutorial_3 camera
            return;
        }
        // C1: Cornell box [-1,1]^2 x [0,2], one ceiling light
        std::vector<float> P, N, LP, LN;
        const float f0[3] = {-1, -1, 0}, f1[3] = {1, -1, 0}, f2[3] = {1, 1, 0}, f3[3] = {-1, 1, 0};
        const float c0[3] = {-1, -1, 2}, c1[3] = {-1, 1, 2}, c2[3] = {1, 1, 2}, c3[3] = {1, -1, 2};
        const float up[3] = {0, 0, 1}, dn[3] = {0, 0, -1}, bk[3] = {0, -1, 0};
        quad(P, N, f0, f1, f2, f3, up);
        quad(P, N, c0, c1, c2, c3, dn);
        const float b0[3] = {-1, 1, 0}, b1[3] = {1, 1, 0}, b2[3] = {1, 1, 2}, b3[3] = {-1, 1, 2};
        quad(P, N, b0, b1, b2, b3, bk);
        const float l0[3] = {-0.25f, -0.25f, 1.98f}, l1[3] = {-0.25f, 0.25f, 1.98f}, l2[3] = {0.25f, 0.25f, 1.98f},
                    l3[3] = {0.25f, -0.25f, 1.98f};
        quad(LP, LN, l0, l1, l2, l3, dn);
        std::vector<rs_mesh_desc> meshes = {{(uint32_t)(P.size() / 9), P.data(), N.data(), 0},
                                            {(uint32_t)(LP.size() / 9), LP.data(), LN.data(), 1}};
        rs_material_desc white{}, light{};
        white.diffuse[0] = white.diffuse[1] = white.diffuse[2] = 0.73f; white.type = 1; white.shininess = 1;
        light.emission[0] = 17; light.emission[1] = 12; light.emission[2] = 4; light.type = 1;
        r.LoadScene(meshes, {white, light});
        r.camera_ = restir::Camera(0.0f, -3.9f, 1.0f, 0.0f, 0.0f, 1.0f, 40.0f);
    };
    try {
        if (ranks > 0) {
            int ndev = 1;
            if (const char* e = std::getenv("RESTIR_DEVICES")) ndev = std::max(1, std::atoi(e));
            restir::MultiGpuRenderer mg(W, H, ranks, ndev);
            for (int i = 0; i < ranks; ++i) load(mg.rank(i));
            mg.camera_ = mg.rank(0).camera_;
            if (cam_set) mg.camera_ = restir::Camera(eye[0], eye[1], eye[2], at[0], at[1], at[2], fov);
            mg.params = prm;
            std::unique_ptr<restir::Renderer> one;
            if (compare) {
                one.reset(new restir::Renderer(W, H));
                load(*one);
                one->camera_ = mg.camera_;
                one->params = prm;
            }
            bool same = true;
            for (int f = 0; f < frames; ++f) {
                mg.produceRestir();
                if (one) {
                    one->produceRestir();
                    same = same && std::memcmp(one->frame_data(), mg.frame_data(), (size_t)W * H * 12) == 0;
                }
            }
            std::printf("{\"ranks\": %d, \"frames\": %d, \"compared\": %s, \"bit_identical\": %s}\n", ranks, frames,
                        compare ? "true" : "false", compare ? (same ? "true" : "false") : "null");
            if (!out.empty()) write_pfm(out, W, H, mg.frame_data());
            return compare && !same ? 2 : 0;
        }
        restir::Renderer r(W, H);
        rp = &r;
        r.params = prm;
        load(r);
        if (cam_set) r.camera_ = restir::Camera(eye[0], eye[1], eye[2], at[0], at[1], at[2], fov);
        if (bench) {
            using clk = std::chrono::steady_clock;
            r.timePasses = false;
            auto run = [&](int depth, int n) {
                r.pipelineDepth = depth;
                for (int f = 0; f < 9; ++f) r.produceRestir();      // traversal tuning (6) + warm-up
                r.finish();
                const auto t0 = clk::now();
                for (int f = 0; f < n; ++f) r.produceRestir();
                r.finish();
                return std::chrono::duration<double>(clk::now() - t0).count();
            };
            const double tp = run(2, frames), t1 = run(1, frames), ts = run(0, frames);
            double sum = 0.0;                                     // touch the last host frame
            for (size_t i = 0; i < (size_t)W * H * 3; i += 997) sum += r.frame_data()[i];
            std::printf("{\"value\": %.4f, \"unit\": \"frames/s\", \"ms_per_step\": %.4f, \"frames\": %d, "
                        "\"mode\": \"pipelineDepth 2: frame_data = the frame 2 back, readbacks overlapped\", "
                        "\"depth1_value\": %.4f, "
                        "\"sync_value\": %.4f, \"sync_mode\": \"reference semantics: frame_data = this frame\", "
                        "\"frame_bytes\": %zu, \"driver\": \"restir-embree_amd/tools/restir_render --bench "
                        "(include/restir.hpp)\", \"checksum\": %.6g}\n",
                        frames / tp, tp / frames * 1e3, frames, frames / t1, frames / ts, (size_t)W * H * 12, sum);
            return 0;
        }
        r.accumulate = true;                 // the producer loop's progressive accumulation
        if (!denoise_w.empty()) {            // SimpleGuiDX11::initOIDN + RenderParams::denoise
            r.initOIDN(denoise_w);
            r.denoise = true;
        }
        for (int f = 0; f < frames; ++f) {
            r.produceRestir();
            r.postFrame();
            std::printf("frame %d: gbuffer+initial %.3f ms, temporal %.3f ms, spatial %.3f ms, shade %.3f ms, "
                        "total %.3f ms, rays %llu, accumulator mean %.6f var %.6f (%u frames)\n", f,
                        r.gBUfferFillDuration, r.temporalReusePassDuration, r.spatialReusePassDuration,
                        r.shadingPassDuration, r.totalFrameDuration, (unsigned long long)r.raysTraced,
                        r.accumulatorMean, r.accumulatorVariance, r.accFrameCtr);
        }
        r.finish();
        if (!out.empty()) write_pfm(out, W, H, r.frame_data());
        if (!png.empty()) {                  // SimpleGuiDX11::exportImage of the (denoised) display
            rs_export_params ep{0.0f, 1};
            restir::check(rs_export_png(r.handle(), png.c_str(), &ep), r.handle());
        }
    } catch (const restir::Error& e) {
        std::fprintf(stderr, "error %d: %s\n", e.code, e.what());
        return 1;
    }
    (void)rp;
    return 0;
}
