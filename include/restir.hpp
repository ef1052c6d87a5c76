// restir.hpp -- C++ host-side mirror of the reference's ReSTIR frame API over the C ABI (restir_c.h).
//
// The reference drives the hot path from C++ members of one object:
//   Raytracer::LoadScene(std::string)        pg/raytracer.cpp:34-38
//   SimpleGuiDX11::produceRestir(float t)    pg/simpleguidx11.cpp:359-487
//   glm::vec3* frame_data                    pg/simpleguidx11.h:152
//   ReSTIRIntegrator static knobs            pg/ReSTIRIntegrator.cpp:13-35 (M_Area, M_Brdf, ...)
//   per-pass timers                          pg/simpleguidx11.h:120-127 (gBUfferFillDuration, ...)
// restir::Renderer keeps those names so a reference caller switches by replacing the object type.
// Errors become restir::Error exceptions on the C++ side (the reference throws std::runtime_error
// for Embree errors, pg/tutorials.cpp:6-24); nothing throws across the C ABI itself.
#pragma once
#include "restir_c.h"

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace restir {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc, const rs_context* ctx) {
    if (rc != RS_OK) throw Error(rc, std::string("librestir_amd: ") + rs_last_error(ctx));
}

// ReSTIRIntegrator's statics + ReSTIR's private RenderParams, with the reference defaults
// (pg/ReSTIRIntegrator.cpp:13-33, pg/RenderParams.h:5-17); useSkybox off (missing sky HDR).
struct Params : rs_frame_params {
    enum SpatialWeightCalculation { CONSTANT = 0, CONSTANT_DEBIAS_CONTRIB = 1, CONSTANT_DEBIAS_Z_TERM = 2,
                                    BALANCE_HEURISTIC = 3, PAIRWISE_MIS = 4 };
    Params() {
        std::memset(static_cast<rs_frame_params*>(this), 0, sizeof(rs_frame_params));
        m_area = 1; m_brdf = 1; spatial_neighbors = 5; spatial_passes = 1; confidence_cap = 20;
        spatial_radius = 30.0f; min_normal_similarity = 0.85f; max_depth_difference = 0.2f;
        spatial_mis = CONSTANT; use_skybox = 0; bg_color[0] = bg_color[1] = bg_color[2] = 0.5f;
        tnear_offset = 0.01f; tfar_offset = 0.001f; normal_offset = 0.001f; seed = 123;
    }
};

struct Camera : rs_camera {   // Camera(width, height, fov_y, view_from, view_at), Z-up
    Camera(float ex = 0, float ey = 0, float ez = 0, float ax = 0, float ay = 0, float az = 0, float fov = 40.0f) {
        eye[0] = ex; eye[1] = ey; eye[2] = ez; at[0] = ax; at[1] = ay; at[2] = az; fov_y_deg = fov;
    }
    void setPosition(float x, float y, float z) { eye[0] = x; eye[1] = y; eye[2] = z; }   // pg/camera.cpp:60-64
    void setViewAt(float x, float y, float z) { at[0] = x; at[1] = y; at[2] = z; }        // pg/camera.h:31-35
    void setFOV(float deg) { fov_y_deg = deg; }                                            // pg/camera.cpp:81-84
};

class Renderer {
public:
    Renderer(int width, int height, int hip_device = 0, void* hip_stream = nullptr) : width_(width), height_(height) {
        check(rs_context_create(hip_device, width, height, hip_stream, &ctx_), nullptr);
        const size_t bytes = (size_t)width * height * 3 * sizeof(float);
        for (auto& b : ring_) {                 // page-locked frame_data ring (asynchronous readback)
            void* p = nullptr;
            check(rs_host_alloc(ctx_, bytes, &p), ctx_);
            b = static_cast<float*>(p);
            std::memset(b, 0, bytes);
        }
        shown_ = ring_[0];
    }
    ~Renderer() {
        if (ctx_) rs_synchronize(ctx_);
        if (scene_) rs_scene_destroy(scene_);
        if (denoiser_) rs_denoiser_destroy(denoiser_);
        if (ctx_) rs_context_destroy(ctx_);
        for (auto b : ring_) rs_host_free(b);
    }
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    // Raytracer::LoadScene(file): OBJ/MTL (Pc/Kd/Ks/Ke/Ns) -> GPU LBVH + emissive CDF
    void LoadScene(const std::string& obj_path) {
        rs_scene* s = nullptr;
        check(rs_scene_load_obj(ctx_, obj_path.c_str(), &s), ctx_);
        replace_scene(s);
    }
    // Scene from in-memory meshes (what ModelLoader hands Embree, pg/ModelLoader.cpp:232-317)
    void LoadScene(const std::vector<rs_mesh_desc>& meshes, const std::vector<rs_material_desc>& materials) {
        rs_scene* s = nullptr;
        check(rs_scene_create(ctx_, meshes.data(), (uint32_t)meshes.size(), materials.data(),
                              (uint32_t)materials.size(), &s), ctx_);
        replace_scene(s);
    }

    // SimpleGuiDX11::produceRestir(t): one frame with the current camera_ and params; frame_data()
    // then holds the linear-HDR framebuffer, the duration members the per-pass device times.
    //   pipelineDepth = 0 (reference semantics): frame_data() is this frame (the call waits for it).
    //   pipelineDepth = d (1..2): the frame's readback into host memory runs while the next frames
    //     render, and frame_data() is the frame d frames back (frameDataIndex() says which; finish()
    //     brings it up to date) -- the producer loop's accumulate/tonemap then lags d frames.  d = 2 keeps
    //     as many frames in flight as the library's run-ahead lanes (3).
    //   timePasses = false: no per-frame pass timing (the duration members are not updated; that saves
    //     the host sync rs_render_frame needs to read the device times back).
    void produceRestir(float t = 0.0f) {
        (void)t;
        if (!scene_) throw Error(RS_E_INVALID, "produceRestir: no scene loaded");
        rs_pass_times pt{};
        check(rs_render_frame(ctx_, scene_, &camera_, &params, frameCtr, nullptr, timePasses ? &pt : nullptr), ctx_);
        Pending p{0, ring_[cur_], (long long)frameCtr};
        check(rs_frame_readback(ctx_, p.buf, &p.ticket), ctx_);
        pending_[n_pending_++] = p;
        cur_ = (cur_ + 1) % kRing;
        const int depth = pipelineDepth < 0 ? 0 : (pipelineDepth > kRing - 1 ? kRing - 1 : pipelineDepth);
        while (n_pending_ > depth) publish();
        if (timePasses) {
            gBUfferFillDuration = pt.gbuffer_initial_ms;   // G-buffer fill and initial RIS run fused
            initialCandidatesGenDuration = 0.0f;
            visibilityPassDuration = pt.visibility_ms;
            temporalReusePassDuration = pt.temporal_ms;
            spatialReusePassDuration = pt.spatial_ms;
            shadingPassDuration = pt.shade_ms;
            bufferCopyDuration = 0.0f;                      // history is a pointer swap
            totalFrameDuration = pt.total_ms;
            raysTraced = pt.rays;
        }
        ++frameCtr;
    }
    // pipelined mode: wait for the outstanding readbacks; frame_data() is then the last frame produced
    void finish() {
        while (n_pending_ > 0) publish();
    }
    // frameCtr of the frame frame_data() holds (-1 before the first one has landed)
    long long frameDataIndex() const { return shown_frame_; }
    void resetHistory() { check(rs_reset_history(ctx_), ctx_); }

    // The producer loop's post block after produceRestir (pg/simpleguidx11.cpp:246-333, OIDN excluded):
    // accumulate into the accumulator, ACES + sRGB into display_data(), accumulatorMean/Variance.
    // SimpleGuiDX11::initOIDN (pg/simpleguidx11.cpp:52-75): the "RT" filter (hdr, auto-exposure) with
    // the weights of an OIDN tensor archive; postFrame() then shows the denoised accumulator when
    // `denoise` (RenderParams::denoise) is set.
    void initOIDN(const std::string& weights_tza) {
        rs_denoiser* d = nullptr;
        check(rs_denoiser_create_from_file(ctx_, weights_tza.c_str(), &d), ctx_);
        if (denoiser_) rs_denoiser_destroy(denoiser_);
        denoiser_ = d;
        check(rs_context_set_denoiser(ctx_, denoiser_), ctx_);
    }
    void postFrame() {
        rs_post_params pp{accumulate ? 1 : 0, tonemap ? 1 : 0, gammaCorrect ? 1 : 0, maxAccCount, denoise ? 1 : 0};
        rs_post_stats st{};
        const float* dptr = nullptr;
        check(rs_post_frame(ctx_, &pp, &dptr, &st), ctx_);
        accFrameCtr = accumulate && st.acc_frames_used + 1 <= (uint32_t)maxAccCount ? st.acc_frames_used + 1 : 0;
        accumulatorMean = st.mean;
        accumulatorVariance = st.variance;
        display_device_ = dptr;
    }
    const float* display_device_data() const { return display_device_; }   // device W*H*4 float RGBA

    const float* frame_data() const { return shown_; }           // W*H*3, row-major, y=0 top
    int width() const { return width_; }
    int height() const { return height_; }
    rs_context* handle() { return ctx_; }
    rs_scene* scene_handle() { return scene_; }

    Camera camera_;
    Params params;
    uint32_t frameCtr = 0;
    int pipelineDepth = 0;
    bool timePasses = true;
    float gBUfferFillDuration = 0, initialCandidatesGenDuration = 0, visibilityPassDuration = 0,
          temporalReusePassDuration = 0, spatialReusePassDuration = 0, shadingPassDuration = 0,
          bufferCopyDuration = 0, totalFrameDuration = 0;
    uint64_t raysTraced = 0;
    // post block (SimpleGuiDX11 accumulate / maxAccCount / accFrameCtr, RenderParams::tonemap,
    // Raytracer::gammaCorrect, accumulatorMean / accumulatorVariance)
    bool accumulate = false, tonemap = true, gammaCorrect = true;
    bool denoise = false;                       // RenderParams::denoise (pg/RenderParams.h:13), needs initOIDN
    int maxAccCount = 300000;
    uint32_t accFrameCtr = 0;
    double accumulatorMean = 0.0, accumulatorVariance = 0.0;

private:
    struct Pending { uint64_t ticket; float* buf; long long frame; };
    static constexpr int kRing = 3;
    void publish() {                            // the oldest outstanding readback becomes frame_data()
        check(rs_frame_wait(ctx_, pending_[0].ticket), ctx_);
        shown_ = pending_[0].buf; shown_frame_ = pending_[0].frame;
        for (int i = 1; i < n_pending_; ++i) pending_[i - 1] = pending_[i];
        --n_pending_;
    }
    float* ring_[kRing] = {};
    float* shown_ = nullptr;
    Pending pending_[kRing] = {};
    int n_pending_ = 0;
    long long shown_frame_ = -1;
    int cur_ = 0;
    const float* display_device_ = nullptr;
    void replace_scene(rs_scene* s) {
        if (scene_) rs_scene_destroy(scene_);
        scene_ = s;
    }
    int width_, height_;
    rs_context* ctx_ = nullptr;
    rs_scene* scene_ = nullptr;
    rs_denoiser* denoiser_ = nullptr;
};

// The N-GPU frame (rs_mgpu_*) with the same member surface: N row bands, one Renderer
// (context) per rank, all driven from this thread (rs_mgpu_create_local: halo exchange and gather by
// device copies; rank i on HIP device i % device_count).  frame_data() is rank 0's gathered frame.  A
// multi-process deployment uses rs_mgpu_create with an RCCL id instead.
class MultiGpuRenderer {
public:
    MultiGpuRenderer(int width, int height, int ranks, int device_count = 1) : width_(width), height_(height) {
        if (ranks < 1 || device_count < 1) throw Error(RS_E_INVALID, "MultiGpuRenderer: ranks and device_count must be >= 1");
        for (int i = 0; i < ranks; ++i) ranks_.emplace_back(new Renderer(width, height, i % device_count));
        frame_.assign((size_t)width * height * 3, 0.0f);
    }
    ~MultiGpuRenderer() {
        if (m_) rs_mgpu_destroy(m_);
        for (auto* r : ranks_) delete r;
    }
    MultiGpuRenderer(const MultiGpuRenderer&) = delete;
    MultiGpuRenderer& operator=(const MultiGpuRenderer&) = delete;

    int ranks() const { return (int)ranks_.size(); }
    Renderer& rank(int i) { return *ranks_[i]; }       // load the scene into every rank (LoadScene)
    // one frame as N bands, gathered into frame_data() (synchronous)
    void produceRestir(float t = 0.0f) {
        (void)t;
        if (!m_) {
            std::vector<rs_context*> ctxs;
            for (auto* r : ranks_) ctxs.push_back(r->handle());
            check(rs_mgpu_create_local(ctxs.data(), (int)ctxs.size(), &m_), ranks_[0]->handle());
        }
        std::vector<const rs_scene*> scenes;
        for (auto* r : ranks_) {
            if (!r->scene_handle()) throw Error(RS_E_INVALID, "MultiGpuRenderer: load the scene into every rank");
            scenes.push_back(r->scene_handle());
        }
        check(rs_mgpu_render_frame(m_, scenes.data(), &camera_, &params, frameCtr, 1, frame_.data(), nullptr),
              ranks_[0]->handle());
        ++frameCtr;
    }
    // cost-balanced bands from n_frames of per-row wave times, then `refine` rounds of time-based refinement
    // (-1: the library's default; resets the history)
    void rebalance(int n_frames = 2, int min_rows = 8, int refine = -1) {
        produceRestir();                              // creates the group
        std::vector<const rs_scene*> scenes;
        for (auto* r : ranks_) scenes.push_back(r->scene_handle());
        if (refine >= 0) check(rs_mgpu_set_rebalance_refine(m_, refine), ranks_[0]->handle());
        check(rs_mgpu_rebalance(m_, scenes.data(), &camera_, &params, frameCtr, n_frames, min_rows), ranks_[0]->handle());
        frameCtr = 0;
    }
    const float* frame_data() const { return frame_.data(); }

    Camera camera_;
    Params params;
    uint32_t frameCtr = 0;

private:
    int width_, height_;
    std::vector<Renderer*> ranks_;
    rs_mgpu* m_ = nullptr;
    std::vector<float> frame_;
};

}  // namespace restir
