// restir_capi.hip -- C ABI (include/restir_c.h) over the gfx950 kernels.
//
// Host side of the drop-in boundary: owns the per-pixel buffers the reference keeps in
// SimpleGuiDX11 (pg/simpleguidx11.cpp:113-119, pg/simpleguidx11.h:27-66), uploads scenes
// (pg/Scene.cpp:8-16, pg/ModelLoader.cpp:218-321, pg/TriangleCDF.cpp:8-34), computes the camera
// (pg/camera.cpp:12-84) and sequences the passes of produceRestir (pg/simpleguidx11.cpp:359-487).
#include "rs_passes.h"
#include "rs_mis.h"
#include "rs_post.h"
#include "rs_refit.h"
#include "../../include/restir_c.h"
#include "rs_image.h"
#include "rs_internal.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>
#include <algorithm>

namespace rs {
int build_bvh(const float* d_pos, uint32_t n, hipStream_t st, float4** d_nodes, uint32_t* n_nodes, float4** d_tris,
              WideBvh* wide, std::string& err);
void preload_code_objects();
void builder_pool_trim();
int bvh_refit_plan(const float4* d_nodes, uint32_t n_nodes, hipStream_t st, int** d_order, int** d_lvl_off,
                   std::vector<int>& lvl_off, std::string& err);
int bvh_refit(float4* d_nodes, float4* d_tris, const float* d_pos, const int* d_order, const int* d_lvl_off,
              const std::vector<int>& lvl_off, hipStream_t st, int* tail, std::string& err);
void wide_free(WideBvh& w);
}

using namespace rs;

static thread_local std::string g_last_error;

struct rs_scene {
    rs_context* ctx = nullptr;
    uint32_t n_tris = 0, n_emis = 0, n_mats = 0, n_nodes = 0;
    float* d_pos = nullptr;
    float4 *d_nodes = nullptr, *d_tris = nullptr, *d_tri_nrm = nullptr, *d_mats = nullptr, *d_emis = nullptr;
    float* d_cdf = nullptr;
    int* d_cdf_guide = nullptr;
    float build_ms = 0.0f;
    float box_eps = 0.0f;                 // closest-hit box margin (rs_wide.h box_epsilon), set at the last full build
    // host copies (rs_scene_rebuild re-derives the tables on the host)
    std::vector<float> h_nrm;
    std::vector<uint32_t> h_tri_mat;
    std::vector<rs_material_desc> h_mats;
    // rs_scene_update_positions: emissive triangle ids, refit plan, pinned upload ring (2 slots)
    int* d_emis_tri = nullptr;
    uint8_t* d_ebucket = nullptr;          // per emitter: its Morton bucket (the sorted initial pass's ray key)
    float ecen[3] = {0.0f, 0.0f, 0.0f};    // centre of the emitter centroids' bounds (the sorted spatial pass's key)
    int *d_refit_order = nullptr, *d_refit_lvl = nullptr;
    std::vector<int> refit_lvl;
    // 8-wide tree of the per-lane walks (rs_scene.h), built on the GPU with the binary tree (rs_wide_build.hip)
    // and refit with it when the positions move (rs_refit.h); a_wide = its second copy for pipelined updates
    // and the previous geometry generation (like a_nodes below)
    WideBvh wide, a_wide;
    bool wide_on = false;
    float* h_stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    int stage_i = 0;
    // pipelined updates (frames in flight): the refit and the light tables go to a second copy of the
    // BVH / triangles / light tables, on the next frame's lane stream, while earlier frames still read the
    // current copy; the copies then swap.  gen counts swaps (a frame remembers the one it read).
    float4 *a_nodes = nullptr, *a_tris = nullptr, *a_emis = nullptr;
    float* a_cdf = nullptr;
    int* a_cdf_guide = nullptr;
    int gen = 0;
    // geometry generation (every rs_scene_update_positions; not a rebuild: same positions) and the
    // generation the a_* copy (+ a_tri_nrm when those normals differ) holds as the previous geometry --
    // a tile's temporal pass rebuilds a previous-frame G element against the previous frame's geometry
    uint32_t geo_gen = 0, a_geo = 0xffffffffu;
    float4* a_tri_nrm = nullptr;
    bool a_nrm = false;
    hipEvent_t update_ev = nullptr;        // the last pipelined update (every later frame waits for it)
    bool update_recorded = false;
    float* d_nrm_stage = nullptr;
    // textures (rs_texture.h): host copies in device layout (re-packed when the sky changes)
    struct HostTex { std::vector<uint8_t> bytes; int w = 0, h = 0, pitch = 0, px = 0; };
    std::vector<HostTex> h_tex;            // material maps, then the sky (if any) last
    int sky = -1;
    uint8_t* d_tex = nullptr;
    int4* d_texd = nullptr;
    float4 *d_uv = nullptr, *d_tan = nullptr;
    // per-scene traversal choice (RS_TRAVERSAL_AUTO): frame times of each kind, tuning frames counted
    mutable int trav_choice = -1;
    mutable int trav_runs[2] = {0, 0};
    mutable float trav_ms[2] = {0.0f, 0.0f};
    DevScene dev() const {
        DevScene S;
        S.nodes = d_nodes; S.tris = d_tris; S.tri_nrm = d_tri_nrm; S.mats = d_mats; S.emis = d_emis; S.cdf = d_cdf; S.cdf_guide = d_cdf_guide;
        S.n_nodes = n_nodes; S.n_tris = n_tris; S.n_emis = n_emis; S.n_mats = n_mats;
        S.tri_uv = d_uv; S.tri_tan = d_tan; S.tex = d_tex; S.texd = d_texd; S.sky = sky;
        S.wnodes = wide_on ? wide.nodes : nullptr; S.wtris = wide.tris; S.n_wnodes = wide_on ? wide.n_nodes : 0u;
        S.ebucket = d_ebucket;
        S.ecen = vec3{ecen[0], ecen[1], ecen[2]};
        S.box_eps = box_eps;
        return S;
    }
    // the geometry of generation `g` if this scene still holds it (current, or the a_* copy of g == a_geo)
    bool dev_of(uint32_t g, DevScene& S) const {
        S = dev();
        if (g == geo_gen) return true;
        if (g != a_geo || !a_nodes) return false;
        S.nodes = a_nodes; S.tris = a_tris;
        if (a_nrm) S.tri_nrm = a_tri_nrm;
        const bool w = wide_on && a_wide.nodes;    // the refit trees of that generation
        S.wnodes = w ? a_wide.nodes : nullptr; S.wtris = w ? a_wide.tris : nullptr; S.n_wnodes = w ? a_wide.n_nodes : 0u;
        return true;
    }
};

enum { EV_BEGIN, EV_INIT, EV_VIS, EV_TEMPORAL, EV_SPATIAL, EV_SHADE, EV_DONE, EV_COUNT };

// Frame pipelining ("run-ahead", depth D <= kMaxAhead): frames rotate over D+1 internal "lane"
// streams, frame f running entirely on lane f mod (D+1), so up to D+1 consecutive frames are in flight
// at once: one frame's G-buffer + initial pass (which reads nothing of earlier frames) overlaps the
// previous frames' later passes, halo exchanges and gathers, and the tails of their kernels.  Only the
// temporal pass depends on the previous frame (its final reservoirs and G-buffer): it waits for that
// frame's completion event.  Each lane owns its framebuffer, ray-count slots and counters; the G ring
// holds D+2 buffers (frames f-D-1..f), the reservoir ring 3D+2 (the buffers frames f-D..f-1 touch stay
// apart from the two frame f writes).  The context's stream waits for every frame's completion, so
// its semantics are those of a sequential renderer.  D = 0 runs everything on the context's stream.
// Work enqueued on the context's stream between frames (geometry updates, MIS frames, sky changes)
// makes the next frame's lane wait for it.
constexpr int kMaxAhead = RS_MAX_AHEAD, kLanes = kMaxAhead + 1, kGRing = kMaxAhead + 2, kRRing = 3 * kMaxAhead + 2;
struct rs_context {
    int device = 0, W = 0, H = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipStream_t lane[kLanes] = {};         // frame streams (run-ahead); frame f on lane f mod (D+1)
    int ahead = kMaxAhead;                 // run-ahead depth D (rs_context_set_run_ahead)
    hipStream_t fs = nullptr;              // stream of the frame in flight (a lane, or `stream` when D = 0)
    int li = 0;                            // its lane index (0 when D = 0)
    bool join_next = true;                 // the next frame waits for the context's stream
    GBuf G[kGRing] = {};
    GCam gcam[kGRing] = {};
    float ginv[kGRing][9] = {};            // each slot's mat3(invViewMat) (a tile's temporal pass rebuilds G)
    int gcur = 0, gprev = 0;
    float4* R[kRRing] = {};
    int r_last = 2;
    int rhist[kMaxAhead][3];               // {ra, rb, last} of the previous frames (most recent first)
    float* fb = nullptr;                   // the framebuffer of the frame in flight / last frame
    float* fbs[kLanes] = {};               // per-lane framebuffers (fbs[0] allocated at create, others on demand)
    int fb_ring = 1;
    float* d_rowcost = nullptr;            // per-row wave time while tracking (rs_context_track_row_costs)
    bool track_rows = false;
    Counters* d_cnt = nullptr;             // = cnts[li]
    Counters* cnts[kLanes] = {};
    Counters* h_cnt = nullptr;
    uint2* d_part = nullptr;               // per-wave ray-count slots of this frame's launches (= parts[pk])
    size_t part_cap = 0, part_used = 0;
    uint2* parts[kLanes] = {};             // per-lane slot buffers
    size_t part_caps[kLanes] = {};
    int pk = 0;
    Counters* d_tot = nullptr;             // running totals over frames (rs_get_timing_totals)
    ulonglong2* d_red = nullptr;           // k_reduce_counts partials + ticket (= reds[li])
    ulonglong2* reds[kLanes] = {};
    uint32_t* qctr[kLanes] = {};           // persistent-wave tile queues (rs_passes.h TileQ): 4 words per lane
    float* candw[kLanes] = {};             // the sorted initial pass's candidate weights (FrameConst::cand_w), per lane
    float4* candr[kLanes] = {};            // ... and its shadow rays (FrameConst::cand_ray), per lane
    size_t cand_slots[kLanes] = {};        // wave slots candw / candr hold (ensure_handoff)
    int persist_sorted = RS_SPLIT_AUTO;    // RESTIR_PERSIST_SORTED: the sorted pass by persistent waves
    int persist_sorted_wgs[4] = {};
    // pass timing without a per-frame host sync: every frame records into its own slot of an event
    // ring; slots are folded into the running totals lazily (when reused, or on rs_get_timing_totals)
    static constexpr int kEvRing = 64;
    hipEvent_t evr[kEvRing][EV_COUNT] = {};
    bool ev_pending[kEvRing] = {};
    int slot = 0;
    uint64_t seq = 0;
    double tot_ms[6] = {};                 // gbuffer_initial, visibility, temporal, spatial, shade, total
    uint64_t tot_frames = 0;
    hipEvent_t ev[EV_COUNT] = {};          // the frame in flight's slot
    hipEvent_t ev_gt[2] = {};              // rs_render_direct_mis launch
    uint64_t frames = 0;
    std::string err;
    // frame / tile in flight
    bool active = false;
    const rs_scene* scene = nullptr;
    FrameConst F = {};
    rs_frame_params P = {};
    rs_tile_desc tile = {};
    int ra = 0, rb = 1, rcur = 0, last = 2;
    bool temporal_ran = false, spatial_ran = false, shade_fused = false, ev_temporal = false;
    // traversal kind (rs_scene.h Trav): requested mode, kind of the frame in flight, tuning frame flag
    int trav_mode = RS_TRAVERSAL_AUTO;
    hipEvent_t last_done = nullptr;        // completion event of the last finished frame
    hipEvent_t prev_done = nullptr;        // ... of the frame before the one in flight (temporal waits)
    hipEvent_t prev_begin = nullptr;       // start event of the last frame begun
    hipEvent_t lane_wait[kLanes] = {};     // a lane's last frame ran on the context's stream: its done event
    // per lane: the scene copy its last frame read and that frame's done event (pipelined scene updates)
    const rs_scene* lane_scene[kLanes] = {};
    int lane_gen[kLanes] = {};
    hipEvent_t lane_done[kLanes] = {};
    bool lane_prevgeo[kLanes] = {};        // the lane's last frame rebuilt G elements from the a_* geometry copy
    // geometry generation of the last finished frame / the frame in progress (a tile's temporal rebuild of
    // a previous-frame G element traces the previous frame's geometry, rs_scene::dev_of)
    const rs_scene* geo_last_scene = nullptr;
    uint32_t geo_last = 0, geo_prev = 0;
    const rs_scene* geo_prev_scene = nullptr;
    bool prevgeo_read = false;
    uint64_t prevgeo_missing = 0;          // rebuilds that had to use the current geometry (two updates between frames)
    const rs_scene* frame_scene = nullptr;   // the frame in progress: scene and copy generation
    int frame_gen = 0;
    int trav = TRAV_LOCKSTEP;
    bool twide = false;                    // the frame's scene has its 8-wide tree live (kernel template bit)
    bool tuning = false;
    hipEvent_t tune_ev[16] = {};           // tuning frame: events around each spatial kernel (halo exchanges excluded)
    int tune_n = 0;
    // tile-row dispatch order (rs_passes.h tile_of): per-row wave time of full-frame tuning frames, one
    // buffer per traversal kind; the chosen kind's costs order the 16-px tile rows, costliest first
    float* d_tune_cost[2] = {nullptr, nullptr};
    int* d_order = nullptr;
    int n_order = 0;
    bool order_on = true;                  // RESTIR_TILE_ORDER=off: row-major dispatch
    bool tune_rows = false;                // this tuning frame records per-row cost
    // candidate-split initial pass (rs_passes.h k_gbuffer_initial_split): requested mode, last frame's
    int split_mode = RS_SPLIT_AUTO;
    bool split = false;
    int wave_slots = 0;                    // resident wave capacity of the device at the initial pass's budget
    // post-frame (rs_post_frame): accumulator (float3, like the reference's glm::vec3 accumulator),
    // display (float4 RGBA), per-workgroup statistic partials, accFrameCtr
    float* acc = nullptr;
    float4* display = nullptr;
    double2* post_part = nullptr;
    double2* post_out = nullptr;
    uint32_t acc_frames = 0;
    uint64_t post_px = 0;                  // pixels the last rs_post_frame's statistics cover
    rs_camera cam_last = {};               // camera of the last frame (rs_export_png's sidecar)
    rs_denoiser* denoiser = nullptr;       // rs_post_frame's RenderParams::denoise (rs_context_set_denoiser)
    std::vector<rs_denoiser*> denoisers;   // every live denoiser created on this context (rs::ctx_track_denoiser)
    // asynchronous framebuffer readback (rs_frame_readback): ticket ring, and per lane the readback its
    // framebuffer is under (that lane's next frame waits for it before writing)
    bool readback_kernel = false;          // DMA engine (default) or a copy kernel (env RESTIR_READBACK=kernel)
    static constexpr int kRb = 8;
    hipEvent_t rb_ev[kRb] = {};
    bool rb_busy[kRb] = {};
    uint64_t rb_seq = 0;
    hipEvent_t fb_read[kLanes] = {};
    hipEvent_t join_ev = nullptr;          // rs::ctx_join
    uint8_t* d_dbg = nullptr;              // debugReprojection marks (FrameConst::dbg), on first use
    int cus = 256;
    int sort_mode = RS_SPLIT_AUTO;         // wave-sorted initial pass (RESTIR_SORT=on|off; AUTO: per-lane walks)
    bool sep_margin = true;                // a band's G-buffer margin rows in their own launch (RESTIR_MARGIN_SPLIT=off)
    int sort_spatial = RS_SPLIT_AUTO;      // wave-sorted spatial pass, CONSTANT MIS, k <= 8 (RESTIR_SORT_SPATIAL=on|off;
                                           // AUTO: per-lane walks -- C3 2.21 -> 1.87 ms; lockstep C5 0.228 -> 0.250)
    int sort_temporal = RS_SPLIT_AUTO;     // wave-sorted temporal rays (RESTIR_SORT_TEMPORAL=off: per-ray walks)
};

// --------------------------------------------------------------------------- helpers
static int fail(rs_context* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    g_last_error = msg;
    return code;
}
#define HIPCHK(c, x)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) return fail((c), RS_E_HIP, std::string(#x " -> ") + hipGetErrorString(e_)); \
    } while (0)

// Every entry point: bind the context's device and drop any stale error another library (e.g. torch's
// pointer-attribute queries) left in HIP's per-thread last-error slot, so the post-launch
// hipGetLastError() checks only see errors of our own launches.
static hipError_t enter(rs_context* c) {
    (void)hipGetLastError();
    return hipSetDevice(c->device);
}
// the context's stream and the run-ahead side streams
static void sync_all(rs_context* c) {
    hipStreamSynchronize(c->stream);
    for (auto st : c->lane) if (st) hipStreamSynchronize(st);
}

// glm-semantics host maths for the camera (pg/camera.cpp:44-58, glm/ext/matrix_transform.inl:99-119,
// glm/detail/func_matrix.inl:294-351)
struct hv3 { float x, y, z; };
static inline hv3 hsub(hv3 a, hv3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline float hdot(hv3 a, hv3 b) { float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return x + y + z; }
static inline hv3 hcross(hv3 x, hv3 y) { return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
static inline hv3 hnorm(hv3 a) { float s = 1.0f / std::sqrt(hdot(a, a)); return {a.x * s, a.y * s, a.z * s}; }
static inline float hlen(hv3 a) { return std::sqrt(hdot(a, a)); }

static void look_at_rh(hv3 eye, hv3 center, hv3 up, float m[4][4]) {
    hv3 f = hnorm(hsub(center, eye));
    hv3 s = hnorm(hcross(f, up));
    hv3 u = hcross(s, f);
    std::memset(m, 0, 64);
    m[0][0] = s.x; m[1][0] = s.y; m[2][0] = s.z;
    m[0][1] = u.x; m[1][1] = u.y; m[2][1] = u.z;
    m[0][2] = -f.x; m[1][2] = -f.y; m[2][2] = -f.z;
    m[3][0] = -hdot(s, eye); m[3][1] = -hdot(u, eye); m[3][2] = hdot(f, eye);
    m[3][3] = 1.0f;
}
static void inverse4(const float m[4][4], float I[4][4]) {
    float c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3], c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3], c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2], c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2], c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3], c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2], c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2], c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1], c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    const float F0[4] = {c00, c00, c02, c03}, F1[4] = {c04, c04, c06, c07}, F2[4] = {c08, c08, c10, c11};
    const float F3[4] = {c12, c12, c14, c15}, F4[4] = {c16, c16, c18, c19}, F5[4] = {c20, c20, c22, c23};
    const float V0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]}, V1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
    const float V2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]}, V3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    for (int i = 0; i < 4; ++i) {
        float i0 = V1[i] * F0[i] - V2[i] * F1[i] + V3[i] * F2[i];
        float i1 = V0[i] * F0[i] - V2[i] * F3[i] + V3[i] * F4[i];
        float i2 = V0[i] * F1[i] - V1[i] * F3[i] + V3[i] * F5[i];
        float i3 = V0[i] * F2[i] - V1[i] * F4[i] + V2[i] * F5[i];
        I[0][i] = i0 * SA[i]; I[1][i] = i1 * SB[i]; I[2][i] = i2 * SA[i]; I[3][i] = i3 * SB[i];
    }
    float d0 = m[0][0] * I[0][0], d1 = m[0][1] * I[1][0], d2 = m[0][2] * I[2][0], d3 = m[0][3] * I[3][0];
    float det = (d0 + d1) + (d2 + d3);
    float ood = 1.0f / det;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) I[c][r] = I[c][r] * ood;
}

// Camera ctor + setFOV + recalculate_m_c_w (pg/camera.cpp:12-18,44-58,81-84)
static void make_camera(const rs_camera* c, int H, GCam& g, float inv3[9]) {
    hv3 from{c->eye[0], c->eye[1], c->eye[2]}, at{c->at[0], c->at[1], c->at[2]};
    float fov_rad = c->fov_y_deg * 0.01745329251994329576923690768489f;
    g.focal = (float)H / (2.0f * tanf(fov_rad / 2.0f));
    hv3 up{0.0f, 0.0f, 1.0f};
    hv3 zc = hnorm(hsub(from, at));
    hv3 xc = hnorm(hcross(up, zc));
    hv3 yc = hnorm(hcross(zc, xc));
    float V[4][4], I[4][4];
    look_at_rh(from, at, yc, V);
    inverse4(V, I);
    std::memcpy(g.view, V, 64);
    g.pos = vec3{from.x, from.y, from.z};
    for (int col = 0; col < 3; ++col)
        for (int r = 0; r < 3; ++r) inv3[3 * col + r] = I[col][r];
}

// --------------------------------------------------------------------------- context
extern "C" int rs_context_create(int hip_device, int width, int height, void* hip_stream, rs_context** out) {
    if (!out || width <= 0 || height <= 0) return fail(nullptr, RS_E_INVALID, "rs_context_create: bad arguments");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(nullptr, RS_E_HIP, "rs_context_create: no HIP device visible");
    if (hip_device < 0 || hip_device >= ndev) return fail(nullptr, RS_E_INVALID, "rs_context_create: bad device index");
    rs_context* c = new rs_context();
    c->device = hip_device; c->W = width; c->H = height;
    auto bail = [&](const std::string& m) { g_last_error = m; rs_context_destroy(c); return RS_E_HIP; };
    if (hipSetDevice(hip_device) != hipSuccess) return bail("hipSetDevice failed");
    if (hip_stream) c->stream = (hipStream_t)hip_stream;
    else {
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail("hipStreamCreate failed");
        c->own_stream = true;
    }
    for (auto& st : c->lane)
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return bail("hipStreamCreate failed");
    for (auto& h : c->rhist) h[0] = h[1] = h[2] = -1;
    size_t n = (size_t)width * height;
    for (int i = 0; i < kGRing; ++i) {
        float4** f[5] = {&c->G[i].g0, &c->G[i].g1, &c->G[i].g2, &c->G[i].g3, &c->G[i].g4};
        for (auto* p : f) {
            if (hipMalloc(p, n * sizeof(float4)) != hipSuccess) return bail("hipMalloc(G-buffer) failed");
            hipMemsetAsync(*p, 0, n * sizeof(float4), c->stream);
        }
    }
    for (int i = 0; i < kRRing; ++i) {
        if (hipMalloc(&c->R[i], n * 3 * sizeof(float4)) != hipSuccess) return bail("hipMalloc(reservoirs) failed");
        hipMemsetAsync(c->R[i], 0, n * 3 * sizeof(float4), c->stream);
    }
    if (hipMalloc(&c->fbs[0], n * 3 * sizeof(float)) != hipSuccess) return bail("hipMalloc(frame) failed");
    hipMemsetAsync(c->fbs[0], 0, n * 3 * sizeof(float), c->stream);
    c->fb = c->fbs[0];
    for (int i = 0; i < kLanes; ++i) {
        if (hipMalloc(&c->cnts[i], sizeof(Counters)) != hipSuccess) return bail("hipMalloc(counters) failed");
        if (hipMalloc(&c->reds[i], (kReduceBlocks + 1) * sizeof(ulonglong2)) != hipSuccess) return bail("hipMalloc(partials) failed");
        hipMemsetAsync(c->reds[i], 0, (kReduceBlocks + 1) * sizeof(ulonglong2), c->stream);   // ticket = 0
        hipMemsetAsync(c->cnts[i], 0, sizeof(Counters), c->stream);
        if (hipMalloc(&c->qctr[i], 4 * sizeof(uint32_t)) != hipSuccess) return bail("hipMalloc(tile queues) failed");
        hipMemsetAsync(c->qctr[i], 0, 4 * sizeof(uint32_t), c->stream);
    }
    c->d_cnt = c->cnts[0]; c->d_red = c->reds[0];
    c->fs = c->stream;
    if (hipHostMalloc(&c->h_cnt, sizeof(Counters), hipHostMallocDefault) != hipSuccess) return bail("hipHostMalloc failed");
    if (hipMalloc(&c->d_tot, sizeof(Counters)) != hipSuccess) return bail("hipMalloc(totals) failed");
    hipMemsetAsync(c->d_tot, 0, sizeof(Counters), c->stream);
    for (auto& slot : c->evr)
        for (auto& e : slot)
            if (hipEventCreate(&e) != hipSuccess) return bail("hipEventCreate failed");
    for (auto& e : c->ev_gt)
        if (hipEventCreate(&e) != hipSuccess) return bail("hipEventCreate failed");
    for (int i = 0; i < EV_COUNT; ++i) c->ev[i] = c->evr[0][i];
    if (hipStreamSynchronize(c->stream) != hipSuccess) return bail("context init failed");
    rs::preload_code_objects();
    if (const char* t = std::getenv("RESTIR_TRAVERSAL")) {     // auto (default) | lockstep | lane
        if (!std::strcmp(t, "lockstep")) c->trav_mode = RS_TRAVERSAL_LOCKSTEP;
        else if (!std::strcmp(t, "lane")) c->trav_mode = RS_TRAVERSAL_LANE;
    }
    if (const char* t = std::getenv("RESTIR_SPLIT")) {         // auto (default) | on | off
        if (!std::strcmp(t, "on")) c->split_mode = RS_SPLIT_ON;
        else if (!std::strcmp(t, "off")) c->split_mode = RS_SPLIT_OFF;
    }
    if (const char* t = std::getenv("RESTIR_PERSIST_SORTED")) {   // persistent-wave sorted pass: auto | on | off
        if (!std::strcmp(t, "on")) c->persist_sorted = RS_SPLIT_ON;
        else if (!std::strcmp(t, "off")) c->persist_sorted = RS_SPLIT_OFF;
        else if (!std::strcmp(t, "auto")) c->persist_sorted = RS_SPLIT_AUTO;
    }
    if (const char* t = std::getenv("RESTIR_SORT")) {          // auto (default) | on | off: wave-sorted initial pass
        if (!std::strcmp(t, "on")) c->sort_mode = RS_SPLIT_ON;
        else if (!std::strcmp(t, "off")) c->sort_mode = RS_SPLIT_OFF;
    }
    if (const char* t = std::getenv("RESTIR_SORT_TEMPORAL")) { // auto (default) | on | off: wave-sorted temporal rays
        if (!std::strcmp(t, "on")) c->sort_temporal = RS_SPLIT_ON;
        else if (!std::strcmp(t, "off")) c->sort_temporal = RS_SPLIT_OFF;
    }
    if (const char* t = std::getenv("RESTIR_MARGIN_SPLIT"))    // on (default) | off
        c->sep_margin = std::strcmp(t, "off") != 0;
    if (const char* t = std::getenv("RESTIR_SORT_SPATIAL")) {  // auto (default) | on | off: wave-sorted spatial pass
        if (!std::strcmp(t, "on")) c->sort_spatial = RS_SPLIT_ON;
        else if (!std::strcmp(t, "off")) c->sort_spatial = RS_SPLIT_OFF;
    }
    if (const char* t = std::getenv("RESTIR_TILE_ORDER"))      // cost (default) | off (row-major)
        c->order_on = std::strcmp(t, "off") != 0;
    if (const char* t = std::getenv("RESTIR_READBACK"))        // sdma (default) | kernel
        c->readback_kernel = std::strcmp(t, "kernel") == 0;
    if (const char* t = std::getenv("RESTIR_RUNAHEAD"))        // run-ahead depth 0..kMaxAhead
        c->ahead = std::max(0, std::min(kMaxAhead, std::atoi(t)));
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus <= 0) cus = 256;
        c->wave_slots = cus * 4 * RS_INITIAL_WAVES;
        c->cus = cus;
    }
    *out = c;
    return RS_OK;
}

extern "C" int rs_context_set_traversal(rs_context* c, int mode) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_context_set_traversal: null context");
    if (mode != RS_TRAVERSAL_AUTO && mode != RS_TRAVERSAL_LOCKSTEP && mode != RS_TRAVERSAL_LANE)
        return fail(c, RS_E_INVALID, "rs_context_set_traversal: mode must be RS_TRAVERSAL_AUTO/LOCKSTEP/LANE");
    c->trav_mode = mode;
    return RS_OK;
}
extern "C" int rs_context_set_initial_split(rs_context* c, int mode) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_context_set_initial_split: null context");
    if (mode != RS_SPLIT_AUTO && mode != RS_SPLIT_OFF && mode != RS_SPLIT_ON)
        return fail(c, RS_E_INVALID, "rs_context_set_initial_split: mode must be RS_SPLIT_AUTO/OFF/ON");
    c->split_mode = mode;
    return RS_OK;
}
extern "C" int rs_max_run_ahead(void) { return kMaxAhead; }
extern "C" int rs_context_set_run_ahead(rs_context* c, int depth) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_context_set_run_ahead: null context");
    if (c->active) return fail(c, RS_E_INVALID, "rs_context_set_run_ahead: a frame is in flight");
    HIPCHK(c, enter(c));
    sync_all(c);                                 // frames in flight keep the buffers of the old depth
    if (depth < 0 || depth > kMaxAhead) return fail(c, RS_E_INVALID, "rs_context_set_run_ahead: depth must be 0.." + std::to_string(kMaxAhead));
    c->ahead = depth;
    c->join_next = true;
    return RS_OK;
}
extern "C" int rs_context_handoff_bytes(const rs_context* c, uint64_t* bytes) {
    if (!c || !bytes) return RS_E_INVALID;
    uint64_t b = 0;
    for (size_t s : c->cand_slots) b += (uint64_t)s * (uint64_t)(kSortChunk * 64) * (sizeof(float) + sizeof(float4));
    *bytes = b;
    return RS_OK;
}

extern "C" int rs_context_set_frame_ring(rs_context* c, int n) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_context_set_frame_ring: null context");
    if (n != 1 && n != 2) return fail(c, RS_E_INVALID, "rs_context_set_frame_ring: n must be 1 or 2");
    if (c->active) return fail(c, RS_E_INVALID, "rs_context_set_frame_ring: a frame is in flight");
    HIPCHK(c, enter(c));
    c->fb_ring = n;
    return RS_OK;
}
extern "C" int rs_context_track_row_costs(rs_context* c, int enable) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_context_track_row_costs: null context");
    if (c->active) return fail(c, RS_E_INVALID, "rs_context_track_row_costs: a frame is in flight");
    HIPCHK(c, enter(c));
    if (enable && !c->d_rowcost) {
        HIPCHK(c, hipMalloc(&c->d_rowcost, (size_t)c->H * sizeof(float)));
        HIPCHK(c, hipMemsetAsync(c->d_rowcost, 0, (size_t)c->H * sizeof(float), c->stream));
    }
    c->track_rows = enable != 0;
    return RS_OK;
}
extern "C" int rs_get_row_costs(rs_context* c, float* costs, int reset) {
    if (!c || !costs) return fail(c, RS_E_INVALID, "rs_get_row_costs: null argument");
    if (c->active) return fail(c, RS_E_INVALID, "rs_get_row_costs: a frame is in flight");
    HIPCHK(c, enter(c));
    const size_t bytes = (size_t)c->H * sizeof(float);
    if (!c->d_rowcost) { std::memset(costs, 0, bytes); return RS_OK; }
    HIPCHK(c, hipMemcpyAsync(costs, c->d_rowcost, bytes, hipMemcpyDeviceToHost, c->stream));
    if (reset) HIPCHK(c, hipMemsetAsync(c->d_rowcost, 0, bytes, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RS_OK;
}
extern "C" int rs_context_get_initial_split(const rs_context* c, int* mode, int* last) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_context_get_initial_split: null context");
    if (mode) *mode = c->split_mode;
    if (last) *last = c->split ? 1 : 0;
    return RS_OK;
}
extern "C" int rs_context_get_traversal(const rs_context* c, const rs_scene* s, int* mode, int* last_kind,
                                        int* scene_choice) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_context_get_traversal: null context");
    if (mode) *mode = c->trav_mode;
    if (last_kind) *last_kind = c->trav;
    if (scene_choice) *scene_choice = s ? s->trav_choice : -1;
    return RS_OK;
}

extern "C" void rs_context_destroy(rs_context* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    for (auto st : c->lane) if (st) hipStreamSynchronize(st);
    for (rs_denoiser* d : c->denoisers) rs::denoiser_detach(d);   // their rs_denoiser_destroy frees the rest
    for (auto e : c->rb_ev) if (e) hipEventDestroy(e);
    if (c->join_ev) hipEventDestroy(c->join_ev);
    for (auto& g : c->G) {
        float4* f[5] = {g.g0, g.g1, g.g2, g.g3, g.g4};
        for (auto* p : f) if (p) hipFree(p);
    }
    for (auto* r : c->R) if (r) hipFree(r);
    for (float* f : c->fbs) if (f) hipFree(f);
    if (c->d_rowcost) hipFree(c->d_rowcost);
    for (auto* p : c->cnts) if (p) hipFree(p);
    for (auto* p : c->reds) if (p) hipFree(p);
    for (auto* p : c->qctr) if (p) hipFree(p);
    for (auto* p : c->candw) if (p) hipFree(p);
    for (auto* p : c->candr) if (p) hipFree(p);
    if (c->d_tot) hipFree(c->d_tot);
    void* post[] = {c->acc, c->display, c->post_part, c->post_out};
    for (void* p : post) if (p) hipFree(p);
    for (uint2* p : c->parts) if (p) hipFree(p);
    if (c->h_cnt) hipHostFree(c->h_cnt);
    for (auto& slot : c->evr)
        for (auto& e : slot) if (e) hipEventDestroy(e);
    for (auto& e : c->ev_gt) if (e) hipEventDestroy(e);
    for (auto& e : c->tune_ev) if (e) hipEventDestroy(e);
    for (float* p : c->d_tune_cost) if (p) hipFree(p);
    if (c->d_order) hipFree(c->d_order);
    for (auto st : c->lane) if (st) hipStreamDestroy(st);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
}

extern "C" const char* rs_last_error(const rs_context* c) {
    return c ? c->err.c_str() : g_last_error.c_str();
}

// --------------------------------------------------------------------------- scene
static int build_geometry(rs_context* c, rs_scene* s, const std::vector<float>& pos, std::string& err);
// Utils::expand (pg/utils.cpp:209-218)
static float srgb_expand1(float u) {
    if (u <= 0.0f) return 0.0f;
    if (u >= 1.0f) return 1.0f;
    if (u <= 0.04045f) return u / 12.92f;
    return rs_powf((u + 0.055f) / 1.055f, 2.4f);
}

// A texture in the layout the reference's Texture holds after FreeImage_ConvertToRawBits
// (pg/Texture.cpp:46-50): rows top first, pitch padded to 4 bytes, 8-bit texels as B,G,R(,A); float
// texels as R,G,B(,A).  srgb_expand times Texture::expand (pg/Texture.cpp:141-160; every byte of the
// pixel, quantised back to a byte each time).
static bool prepare_texture(const rs_texture_desc& d, int srgb_expand, rs_scene::HostTex& t, std::string& err) {
    if (!d.data || d.width < 1 || d.height < 1 || d.width > 65536 || d.height > 65536) { err = "bad texture size"; return false; }
    if (d.format == RS_TEX_U8) {
        if (d.channels != 1 && d.channels != 3 && d.channels != 4) { err = "8-bit textures need 1, 3 or 4 channels"; return false; }
        t.px = (int)d.channels;
    } else if (d.format == RS_TEX_F32) {
        if (d.channels != 3 && d.channels != 4) { err = "float textures need 3 or 4 channels"; return false; }
        t.px = 4 * (int)d.channels;
    } else { err = "bad texture format"; return false; }
    t.w = (int)d.width; t.h = (int)d.height;
    t.pitch = (t.w * t.px + 3) & ~3;                                   // FreeImage_GetPitch
    t.bytes.assign((size_t)t.pitch * t.h, 0);
    const size_t rowlen = (size_t)t.w * d.channels;
    for (int y = 0; y < t.h; ++y) {
        uint8_t* dst = t.bytes.data() + (size_t)y * t.pitch;
        if (d.format == RS_TEX_F32) {
            std::memcpy(dst, (const float*)d.data + (size_t)y * rowlen, rowlen * sizeof(float));
            continue;
        }
        const uint8_t* src = (const uint8_t*)d.data + (size_t)y * rowlen;
        for (int x = 0; x < t.w; ++x) {
            const uint8_t* q = src + (size_t)x * d.channels;
            uint8_t* o = dst + (size_t)x * t.px;
            if (d.channels == 1) { o[0] = q[0]; continue; }
            o[0] = q[2]; o[1] = q[1]; o[2] = q[0];
            if (d.channels == 4) o[3] = q[3];
        }
        for (int k = 0; k < srgb_expand; ++k)
            for (int x = 0; x < t.w * t.px; ++x) {
                float f = (float)dst[x] / 255.0f;
                f = srgb_expand1(f);
                dst[x] = (uint8_t)(f * 255.0f);
            }
    }
    return true;
}

// (re-)upload every texture of the scene: one byte buffer (16-byte aligned offsets, 16 zero guard bytes
// after each texture for the 1-byte texel quirk) + descriptors
static int upload_textures(rs_context* c, rs_scene* s, std::string& err) {
    if (s->d_tex) { hipFree(s->d_tex); s->d_tex = nullptr; }
    if (s->d_texd) { hipFree(s->d_texd); s->d_texd = nullptr; }
    if (s->h_tex.empty()) return 0;
    std::vector<int4> desc;
    size_t total = 0;
    for (const auto& t : s->h_tex) {
        desc.push_back(make_int4((int)total, t.w, t.h, t.pitch));
        desc.push_back(make_int4(t.px, t.px > 4 ? RS_TEX_F32 : RS_TEX_U8, 0, 0));
        total += (t.bytes.size() + 16 + 15) & ~(size_t)15;
    }
    if (total >= (size_t)INT32_MAX) { err = "textures exceed 2 GiB"; return -1; }
    std::vector<uint8_t> all(total, 0);
    for (size_t i = 0; i < s->h_tex.size(); ++i)
        std::memcpy(all.data() + desc[2 * i].x, s->h_tex[i].bytes.data(), s->h_tex[i].bytes.size());
    hipStream_t st = c->stream;
    if (hipMalloc(&s->d_tex, total) != hipSuccess || hipMalloc(&s->d_texd, desc.size() * sizeof(int4)) != hipSuccess) {
        err = "hipMalloc(textures) failed"; return -1;
    }
    if (hipMemcpyAsync(s->d_tex, all.data(), total, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(s->d_texd, desc.data(), desc.size() * sizeof(int4), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) { err = "texture upload failed"; return -1; }
    return 0;
}

static int scene_from_arrays(rs_context* c, const std::vector<float>& pos, const std::vector<float>& nrm,
                             const std::vector<uint32_t>& tri_mat, const rs_material_desc* mats, uint32_t n_mats,
                             const std::vector<float>& uv, const std::vector<float>& tan,
                             const rs_texture_desc* textures, uint32_t n_tex, rs_scene** out) {
    const uint32_t n = (uint32_t)tri_mat.size();
    for (uint32_t t = 0; t < n; ++t)
        if (tri_mat[t] >= n_mats) return fail(c, RS_E_INVALID, "rs_scene_create: material index out of range");
    if (n_tex && !textures) return fail(c, RS_E_INVALID, "rs_scene_create_textured: null textures");
    bool any_map = false, any_normal_map = false;
    std::vector<int> expand_count(n_tex, 0);
    for (uint32_t m = 0; m < n_mats; ++m) {
        const rs_material_desc& d = mats[m];
        if (d.type < 0 || d.type > 6) return fail(c, RS_E_INVALID, "rs_scene_create: bad material type");
        const int32_t maps[4] = {d.diffuse_map, d.specular_map, d.shininess_map, d.normal_map};
        for (int k = 0; k < 4; ++k) {
            if (maps[k] < 0 || (uint32_t)maps[k] > n_tex)
                return fail(c, RS_E_INVALID, "rs_scene_create: texture index out of range");
            any_map |= maps[k] > 0;
        }
        any_normal_map |= d.normal_map > 0;
    }
    // materials (pg/material.h:105-115) + emissive list in triangle order (triIdCtr, pg/ModelLoader.cpp:291-305)
    std::vector<float4> hm(kMatStride * (size_t)std::max(n_mats, 1u));
    for (uint32_t m = 0; m < n_mats; ++m) {
        const rs_material_desc& d = mats[m];
        int type = d.type;
        float tb; std::memcpy(&tb, &type, 4);
        const int mp[4] = {d.diffuse_map - 1, d.specular_map - 1, d.shininess_map - 1, d.normal_map - 1};
        float mf[4]; std::memcpy(mf, mp, sizeof mf);
        hm[kMatStride * m] = make_float4(d.diffuse[0], d.diffuse[1], d.diffuse[2], d.shininess);
        hm[kMatStride * m + 1] = make_float4(d.specular[0], d.specular[1], d.specular[2], tb);
        hm[kMatStride * m + 2] = make_float4(d.emission[0], d.emission[1], d.emission[2], 0.0f);
        hm[kMatStride * m + 3] = make_float4(mf[0], mf[1], mf[2], mf[3]);
    }
    if (n_mats == 0) {
        const int none[4] = {-1, -1, -1, -1};
        float mf[4]; std::memcpy(mf, none, sizeof mf);
        hm[3] = make_float4(mf[0], mf[1], mf[2], mf[3]);
    }
    std::vector<float4> tn(3 * (size_t)std::max(n, 1u));
    std::vector<uint32_t> emis_tri;
    for (uint32_t t = 0; t < n; ++t) {
        const rs_material_desc& d = mats[tri_mat[t]];
        int eid = -1;
        if (d.emission[0] + d.emission[1] + d.emission[2] > 0) {   // Material::isEmissive (pg/material.h:135-137)
            eid = (int)emis_tri.size();
            emis_tri.push_back(t);
        }
        int mi = (int)tri_mat[t];
        float mb, eb; std::memcpy(&mb, &mi, 4); std::memcpy(&eb, &eid, 4);
        const float* q = &nrm[9 * (size_t)t];
        tn[3 * t] = make_float4(q[0], q[1], q[2], mb);
        tn[3 * t + 1] = make_float4(q[3], q[4], q[5], eb);
        tn[3 * t + 2] = make_float4(q[6], q[7], q[8], 0.0f);
    }
    rs_scene* s = new rs_scene();
    s->ctx = c; s->n_tris = n; s->n_mats = n_mats;
    s->h_nrm = nrm; s->h_tri_mat = tri_mat; s->h_mats.assign(mats, mats + n_mats);
    auto bail = [&](int code, const std::string& m) { rs_scene_destroy(s); return fail(c, code, m); };
    std::string err;
    if (any_map) {
        // Texture::expand count per texture: once per material diffuse/specular slot that references it
        // (ModelLoader expands the TextureProxy-shared texture again for every such slot, :127,135)
        for (uint32_t m = 0; m < n_mats; ++m) {
            if (mats[m].diffuse_map > 0) expand_count[mats[m].diffuse_map - 1] += textures[mats[m].diffuse_map - 1].srgb_expand ? 1 : 0;
            if (mats[m].specular_map > 0) expand_count[mats[m].specular_map - 1] += textures[mats[m].specular_map - 1].srgb_expand ? 1 : 0;
        }
        s->h_tex.resize(n_tex);
        for (uint32_t i = 0; i < n_tex; ++i)
            if (!prepare_texture(textures[i], expand_count[i], s->h_tex[i], err))
                return bail(RS_E_INVALID, "texture " + std::to_string(i + 1) + ": " + err);
        if (upload_textures(c, s, err) != 0) return bail(RS_E_HIP, err);
        std::vector<float4> huv(2 * (size_t)std::max(n, 1u), make_float4(0, 0, 0, 0));
        if (!uv.empty())
            for (uint32_t t = 0; t < n; ++t) {
                const float* q = &uv[6 * (size_t)t];
                huv[2 * t] = make_float4(q[0], q[1], q[2], q[3]);
                huv[2 * t + 1] = make_float4(q[4], q[5], 0.0f, 0.0f);
            }
        if (hipMalloc(&s->d_uv, huv.size() * sizeof(float4)) != hipSuccess) return bail(RS_E_HIP, "hipMalloc(uv) failed");
        hipMemcpyAsync(s->d_uv, huv.data(), huv.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream);
        if (any_normal_map) {
            std::vector<float4> ht(3 * (size_t)std::max(n, 1u), make_float4(0, 0, 0, 0));
            if (!tan.empty())
                for (uint32_t t = 0; t < n; ++t)
                    for (int j = 0; j < 3; ++j) {
                        const float* q = &tan[9 * (size_t)t + 3 * j];
                        ht[3 * t + j] = make_float4(q[0], q[1], q[2], 0.0f);
                    }
            if (hipMalloc(&s->d_tan, ht.size() * sizeof(float4)) != hipSuccess) return bail(RS_E_HIP, "hipMalloc(tangents) failed");
            hipMemcpyAsync(s->d_tan, ht.data(), ht.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream);
        }
        if (hipStreamSynchronize(c->stream) != hipSuccess) return bail(RS_E_HIP, "attribute upload failed");
    } else if (n_tex) {
        s->h_tex.resize(n_tex);                                        // unreferenced textures: validate only
        for (uint32_t i = 0; i < n_tex; ++i)
            if (!prepare_texture(textures[i], 0, s->h_tex[i], err)) return bail(RS_E_INVALID, "texture " + std::to_string(i + 1) + ": " + err);
        s->h_tex.clear();
    }
    hipStream_t st = c->stream;
    if (hipMalloc(&s->d_tri_nrm, tn.size() * sizeof(float4)) != hipSuccess) return bail(RS_E_HIP, "hipMalloc(nrm) failed");
    hipMemcpyAsync(s->d_tri_nrm, tn.data(), tn.size() * sizeof(float4), hipMemcpyHostToDevice, st);
    if (hipMalloc(&s->d_mats, hm.size() * sizeof(float4)) != hipSuccess) return bail(RS_E_HIP, "hipMalloc(mats) failed");
    hipMemcpyAsync(s->d_mats, hm.data(), hm.size() * sizeof(float4), hipMemcpyHostToDevice, st);
    if (build_geometry(c, s, pos, err) != 0) return bail(RS_E_HIP, err);
    *out = s;
    return RS_OK;
}

// Everything that depends on the vertex positions: the emissive-triangle table + CDF + guide table
// (TriangleCDF ctor, pg/TriangleCDF.cpp:8-34, pg/TriangleCDF.h:25-31; Triangle::area,
// pg/triangle.cpp:13-16) and the BVH.  Used at scene creation and by rs_scene_update_positions.
static int build_geometry(rs_context* c, rs_scene* s, const std::vector<float>& pos, std::string& err) {
    const uint32_t n = s->n_tris;
    const std::vector<float>& nrm = s->h_nrm;
    const std::vector<uint32_t>& tri_mat = s->h_tri_mat;
    const rs_material_desc* mats = s->h_mats.data();
    std::vector<uint32_t> emis_tri;
    for (uint32_t t = 0; t < n; ++t) {
        const rs_material_desc& d = mats[tri_mat[t]];
        if (d.emission[0] + d.emission[1] + d.emission[2] > 0) emis_tri.push_back(t);   // same order as eid
    }
    const uint32_t ne = (uint32_t)emis_tri.size();
    std::vector<float> area(ne), cdf(std::max(ne, 1u));
    float total = 0.0f;
    for (uint32_t e = 0; e < ne; ++e) {
        const float* p = &pos[9 * (size_t)emis_tri[e]];
        hv3 a{p[0], p[1], p[2]}, b{p[3], p[4], p[5]}, cc{p[6], p[7], p[8]};
        area[e] = 0.5f * hlen(hcross(hsub(b, a), hsub(cc, a)));
        total += area[e];
    }
    for (uint32_t e = 0; e < ne; ++e) {
        float na = area[e] / total;
        float pred = e == 0 ? 0.0f : cdf[e - 1];
        cdf[e] = pred + na;
    }
    std::vector<float4> em(8 * (size_t)std::max(ne, 1u));
    for (uint32_t e = 0; e < ne; ++e) {
        uint32_t t = emis_tri[e];
        const float* p = &pos[9 * (size_t)t];
        const float* q = &nrm[9 * (size_t)t];
        const rs_material_desc& d = mats[tri_mat[t]];
        float pick = e == 0 ? cdf[0] : cdf[e] - cdf[e - 1];
        float inv_area = 1.0f / area[e];
        float pdf_brdf = area[e] / total;
        pdf_brdf *= 1.0f / area[e];
        const bool flat = std::memcmp(q, q + 3, 3 * sizeof(float)) == 0 && std::memcmp(q, q + 6, 3 * sizeof(float)) == 0;
        const float pdf_area = pick * inv_area;           // the product areaSampleLight forms (rs_passes.h EmisRec)
        em[8 * e + 0] = make_float4(p[0], p[1], p[2], flat ? pdf_area : -pdf_area);
        em[8 * e + 1] = make_float4(p[3], p[4], p[5], q[0]);
        em[8 * e + 2] = make_float4(p[6], p[7], p[8], q[1]);
        em[8 * e + 3] = make_float4(d.emission[0], d.emission[1], d.emission[2], q[2]);
        em[8 * e + 4] = make_float4(q[3], q[4], q[5], pick);
        em[8 * e + 5] = make_float4(q[6], q[7], q[8], pdf_brdf);
        em[8 * e + 6] = make_float4(area[e], inv_area, 0.0f, 0.0f);
        em[8 * e + 7] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    // emitter buckets for the sorted initial pass (performance only: any bucketing gives the same frames):
    // the emitters' centroids in Morton order over their bounds, cut into 64 equal runs
    std::vector<uint8_t> ebucket(std::max(ne, 1u), 0);
    if (ne) {
        float lo[3] = {3.0e38f, 3.0e38f, 3.0e38f}, hi[3] = {-3.0e38f, -3.0e38f, -3.0e38f};
        std::vector<float> cen(3 * (size_t)ne);
        for (uint32_t e = 0; e < ne; ++e) {
            const float* p = &pos[9 * (size_t)emis_tri[e]];
            for (int a = 0; a < 3; ++a) {
                const float v = (p[a] + p[3 + a] + p[6 + a]) * (1.0f / 3.0f);
                cen[3 * (size_t)e + a] = std::isfinite(v) ? v : 0.0f;
                lo[a] = std::min(lo[a], cen[3 * (size_t)e + a]); hi[a] = std::max(hi[a], cen[3 * (size_t)e + a]);
            }
        }
        std::vector<std::pair<uint64_t, uint32_t>> ord(ne);
        for (uint32_t e = 0; e < ne; ++e) {
            uint64_t m = 0;
            uint32_t q[3];
            for (int a = 0; a < 3; ++a) {
                const float ext = hi[a] - lo[a];
                const float t = ext > 0.0f ? (cen[3 * (size_t)e + a] - lo[a]) / ext : 0.0f;
                q[a] = (uint32_t)std::min(1023.0f, std::max(0.0f, t * 1024.0f));
            }
            for (int b = 0; b < 10; ++b)
                for (int a = 0; a < 3; ++a) m |= (uint64_t)((q[a] >> b) & 1u) << (3 * b + a);
            ord[e] = {m, e};
        }
        std::sort(ord.begin(), ord.end());
        for (uint32_t i = 0; i < ne; ++i) ebucket[ord[i].second] = (uint8_t)(((uint64_t)i * 64u) / ne);
        for (int a = 0; a < 3; ++a) s->ecen[a] = 0.5f * lo[a] + 0.5f * hi[a];
    }
    std::vector<int> guide(kCdfGuide + 1);     // guide[j] = lower_bound(cdf, j / kCdfGuide)
    for (int j = 0; j <= kCdfGuide; ++j) {
        float key = (float)j / (float)kCdfGuide;
        guide[j] = (int)(std::lower_bound(cdf.begin(), cdf.begin() + ne, key) - cdf.begin());
    }
    hipStream_t st = c->stream;
    c->join_next = true;
    sync_all(c);                                // frames in flight, pipelined updates
    if (hipStreamSynchronize(st) != hipSuccess) { err = "stream sync failed"; return -1; }
    {
        void* alt[] = {s->a_nodes, s->a_tris, s->a_emis, s->a_cdf, s->a_cdf_guide, s->a_tri_nrm};
        for (void* p : alt) if (p) hipFree(p);
        wide_free(s->a_wide);
        s->a_nodes = s->a_tris = s->a_emis = s->a_tri_nrm = nullptr; s->a_cdf = nullptr; s->a_cdf_guide = nullptr;
        s->a_geo = 0xffffffffu; s->a_nrm = false;
        s->update_recorded = false;
    }
    void* old[] = {s->d_pos, s->d_nodes, s->d_tris, s->d_emis, s->d_cdf, s->d_cdf_guide, s->d_emis_tri,
                   s->d_refit_order, s->d_refit_lvl, s->d_ebucket};
    s->d_ebucket = nullptr;
    wide_free(s->wide); s->wide_on = false;
    for (void* p : old) if (p) hipFree(p);
    s->d_pos = nullptr; s->d_nodes = nullptr; s->d_tris = nullptr; s->d_emis = nullptr; s->d_cdf = nullptr;
    s->d_cdf_guide = nullptr; s->d_emis_tri = nullptr; s->d_refit_order = nullptr; s->d_refit_lvl = nullptr;
    s->n_nodes = 0; s->refit_lvl.clear();
    s->n_emis = ne;
    if (n) {
        if (hipMalloc(&s->d_pos, pos.size() * sizeof(float)) != hipSuccess) { err = "hipMalloc(pos) failed"; return -1; }
        hipMemcpyAsync(s->d_pos, pos.data(), pos.size() * sizeof(float), hipMemcpyHostToDevice, st);
    }
    if (hipMalloc(&s->d_emis, em.size() * sizeof(float4)) != hipSuccess) { err = "hipMalloc(emis) failed"; return -1; }
    hipMemcpyAsync(s->d_emis, em.data(), em.size() * sizeof(float4), hipMemcpyHostToDevice, st);
    if (hipMalloc(&s->d_cdf, cdf.size() * sizeof(float)) != hipSuccess) { err = "hipMalloc(cdf) failed"; return -1; }
    hipMemcpyAsync(s->d_cdf, cdf.data(), cdf.size() * sizeof(float), hipMemcpyHostToDevice, st);
    if (hipMalloc(&s->d_cdf_guide, guide.size() * sizeof(int)) != hipSuccess) { err = "hipMalloc(guide) failed"; return -1; }
    hipMemcpyAsync(s->d_cdf_guide, guide.data(), guide.size() * sizeof(int), hipMemcpyHostToDevice, st);
    if (hipMalloc(&s->d_ebucket, ebucket.size()) != hipSuccess) { err = "hipMalloc(emitter buckets) failed"; return -1; }
    hipMemcpyAsync(s->d_ebucket, ebucket.data(), ebucket.size(), hipMemcpyHostToDevice, st);
    if (ne) {
        if (hipMalloc(&s->d_emis_tri, ne * sizeof(int)) != hipSuccess) { err = "hipMalloc(emis ids) failed"; return -1; }
        hipMemcpyAsync(s->d_emis_tri, emis_tri.data(), ne * sizeof(int), hipMemcpyHostToDevice, st);
    }
    if (hipStreamSynchronize(st) != hipSuccess) { err = "geometry upload failed"; return -1; }   // host vectors die
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0, st);
    std::string berr;
    s->box_eps = box_epsilon(pos.data(), pos.size());
    int rc = build_bvh(s->d_pos, n, st, &s->d_nodes, &s->n_nodes, &s->d_tris, &s->wide, berr);
    s->wide_on = rc == 0 && s->wide.n_nodes > 0 && s->wide.depth <= kWideStack;   // deeper: the skip pointers
    hipEventRecord(e1, st);
    if (rc == 0 && hipStreamSynchronize(st) == hipSuccess) hipEventElapsedTime(&s->build_ms, e0, e1);
    else { err = "BVH build failed: " + berr; rc = -1; (void)hipStreamSynchronize(st); }
    builder_pool_trim();                          // the build's scratch back to the driver (stream drained above)
    hipEventDestroy(e0); hipEventDestroy(e1);
    if (rc == 0 && bvh_refit_plan(s->d_nodes, s->n_nodes, st, &s->d_refit_order, &s->d_refit_lvl, s->refit_lvl, berr) != 0) {
        err = berr; rc = -1;
    }
    return rc;
}

// TriangleCDF tables from the positions on the device (rs_scene_update_positions): the same float
// operations in the same order as build_geometry's host loop -- sequential total and prefix sum in
// one lane, everything else data-parallel -- so the tables are bit-identical to a fresh scene's.
constexpr int kLightBlock = kRefitBlock, kLightChunk = 8192;
__device__ __forceinline__ void light_table(const float* __restrict__ pos, const float4* __restrict__ tri_nrm,
                                            const float4* __restrict__ mats, const int* __restrict__ emis_tri,
                                            uint32_t ne, float4* em, float* cdf, int* guide) {
    __shared__ float s_total;
    __shared__ float4 s_a4[kLightChunk / 4];   // 16-B aligned: the sequential chains read 4 values per load
    float* s_a = (float*)s_a4;
    for (uint32_t e = threadIdx.x; e < ne; e += kLightBlock) {
        const int t = emis_tri[e];
        const float* p = pos + 9 * (size_t)t;
        const vec3 a = mk(p[0], p[1], p[2]), b = mk(p[3], p[4], p[5]), c = mk(p[6], p[7], p[8]);
        const float area = 0.5f * length(cross(b - a, c - a));         // Triangle::area, pg/triangle.cpp:13-16
        const float4 n0 = tri_nrm[3 * t], n1 = tri_nrm[3 * t + 1], n2 = tri_nrm[3 * t + 2];
        const int m = __float_as_int(n0.w);
        // record layout: rs_passes.h EmisRec (the .w of e0/e4/e5 and e6.y are set below)
        const bool flat = __float_as_uint(n0.x) == __float_as_uint(n1.x) && __float_as_uint(n0.y) == __float_as_uint(n1.y) &&
                          __float_as_uint(n0.z) == __float_as_uint(n1.z) && __float_as_uint(n0.x) == __float_as_uint(n2.x) &&
                          __float_as_uint(n0.y) == __float_as_uint(n2.y) && __float_as_uint(n0.z) == __float_as_uint(n2.z);
        em[8 * e + 0] = make_float4(p[0], p[1], p[2], flat ? 0.0f : -0.0f);   // sign bit: normals differ
        em[8 * e + 1] = make_float4(p[3], p[4], p[5], n0.x);
        em[8 * e + 2] = make_float4(p[6], p[7], p[8], n0.y);
        em[8 * e + 3] = f4(xyz(mats[kMatStride * m + 2]), n0.z);
        em[8 * e + 4] = make_float4(n1.x, n1.y, n1.z, 0.0f);
        em[8 * e + 5] = make_float4(n2.x, n2.y, n2.z, 0.0f);
        em[8 * e + 6] = make_float4(area, 0.0f, 0.0f, 0.0f);
        em[8 * e + 7] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    __syncthreads();
    // TriangleCDF ctor, pg/TriangleCDF.cpp:8-34: the total and the prefix sum are sequential float
    // sums (host order); one lane runs each chain out of LDS, the loads and divisions are parallel
    float total = 0.0f;
    for (uint32_t c0 = 0; c0 < ne; c0 += kLightChunk) {
        const uint32_t m = min(ne - c0, (uint32_t)kLightChunk);
        for (uint32_t j = threadIdx.x; j < m; j += kLightBlock) s_a[j] = em[8 * (c0 + j) + 6].x;
        __syncthreads();
        if (threadIdx.x == 0) {                 // the host's order: one float add after the other
            const uint32_t m4 = m & ~3u;
#pragma unroll 4
            for (uint32_t j = 0; j < m4; j += 4) {
                const float4 v = s_a4[j >> 2];
                total += v.x; total += v.y; total += v.z; total += v.w;
            }
            for (uint32_t j = m4; j < m; ++j) total += s_a[j];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) s_total = total;
    __syncthreads();
    total = s_total;
    float pred = 0.0f;
    for (uint32_t c0 = 0; c0 < ne; c0 += kLightChunk) {
        const uint32_t m = min(ne - c0, (uint32_t)kLightChunk);
        for (uint32_t j = threadIdx.x; j < m; j += kLightBlock) s_a[j] = em[8 * (c0 + j) + 6].x / total;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t m4 = m & ~3u;
#pragma unroll 4
            for (uint32_t j = 0; j < m4; j += 4) {
                float4 v = s_a4[j >> 2];
                pred = pred + v.x; v.x = pred; pred = pred + v.y; v.y = pred;
                pred = pred + v.z; v.z = pred; pred = pred + v.w; v.w = pred;
                s_a4[j >> 2] = v;
            }
            for (uint32_t j = m4; j < m; ++j) { pred = pred + s_a[j]; s_a[j] = pred; }
        }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < m; j += kLightBlock) cdf[c0 + j] = s_a[j];
        __syncthreads();
    }
    for (uint32_t e = threadIdx.x; e < ne; e += kLightBlock) {
        const float area = em[8 * e + 6].x;
        const float pick = e == 0 ? cdf[0] : cdf[e] - cdf[e - 1];
        float pdf_brdf = area / total;
        pdf_brdf *= 1.0f / area;
        const float inv_area = 1.0f / area, pdf_area = pick * inv_area;
        em[8 * e + 0].w = (__float_as_uint(em[8 * e + 0].w) >> 31) ? -pdf_area : pdf_area;
        em[8 * e + 4].w = pick;
        em[8 * e + 5].w = pdf_brdf;
        em[8 * e + 6].y = inv_area;
    }
    for (int j = threadIdx.x; j <= kCdfGuide; j += kLightBlock) {   // lower_bound(cdf, j / kCdfGuide)
        const float key = (float)j / (float)kCdfGuide;
        uint32_t lo = 0, hi = ne;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (cdf[mid] < key) lo = mid + 1; else hi = mid;
        }
        guide[j] = (int)lo;
    }
}

// one launch for the three independent single-workgroup jobs of an update: workgroup 0 the light
// tables, workgroup 1 the last (small-level) batch of the binary refit, workgroup 2 that of the 8-wide refit
struct RefitArgs { float4* nodes; float4* tris; const float* pos; const int* order; const int* lvl_off; int l0, l1; };
__global__ void __launch_bounds__(kLightBlock) k_scene_update(const float* __restrict__ pos, const float4* __restrict__ tri_nrm,
                                                              const float4* __restrict__ mats, const int* __restrict__ emis_tri,
                                                              uint32_t ne, float4* em, float* cdf, int* guide, RefitArgs R,
                                                              WideRefitArgs W) {
    static_assert(kLightBlock == kRefitBlock, "one workgroup size for every job");
    if (blockIdx.x == 0) {
        if (ne) light_table(pos, tri_nrm, mats, emis_tri, ne, em, cdf, guide);
    } else if (blockIdx.x == 1) {
        refit_levels(R.nodes, R.tris, R.pos, R.order, R.lvl_off, R.l0, R.l1, 0, 1);
    } else if (W.l_deep >= W.l_top) {
        wide_refit_levels(W, 0, 1);
    }
}
__global__ void __launch_bounds__(kRefitBlock) k_wide_refit(WideRefitArgs W) { wide_refit_levels(W, blockIdx.x, gridDim.x); }

// the 8-wide tree's second copy (same topology), allocated and filled on first use
static int wide_copy(rs_context* c, const WideBvh& from, WideBvh& to, hipStream_t st) {
    if (!to.nodes) {
        to = from;
        to.nodes = nullptr; to.tris = nullptr; to.box = nullptr;
        HIPCHK(c, hipMalloc(&to.nodes, (size_t)5 * from.n_nodes * sizeof(uint4)));
        HIPCHK(c, hipMalloc(&to.tris, (size_t)3 * from.n_tris * sizeof(float4)));
        HIPCHK(c, hipMalloc(&to.box, (size_t)2 * from.n_nodes * sizeof(float4)));
    }
    HIPCHK(c, hipMemcpyAsync(to.nodes, from.nodes, (size_t)5 * from.n_nodes * sizeof(uint4), hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(to.tris, from.tris, (size_t)3 * from.n_tris * sizeof(float4), hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(to.box, from.box, (size_t)2 * from.n_nodes * sizeof(float4), hipMemcpyDeviceToDevice, st));
    return RS_OK;
}

__global__ void k_set_normals(const float* __restrict__ nrm, uint32_t n, float4* tri_nrm) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const float* q = nrm + 9 * (size_t)t;
    tri_nrm[3 * t] = make_float4(q[0], q[1], q[2], tri_nrm[3 * t].w);
    tri_nrm[3 * t + 1] = make_float4(q[3], q[4], q[5], tri_nrm[3 * t + 1].w);
    tri_nrm[3 * t + 2] = make_float4(q[6], q[7], q[8], 0.0f);
}

// Moving geometry (C5).  Stream-ordered and free of host synchronisation: the positions go through a
// pinned two-slot ring (a slot is reused once its previous copy has completed), the light tables are
// recomputed on the device and the BVH is refit (same topology; results bit-identical to a fresh build,
// rs_bvh_build.hip).  Frames already enqueued see the old geometry, later ones the new.  With frames in
// flight the refit and the tables are written to the scene's second copy on the next frame's lane
// stream, after the frames that read that copy (two frames back) have finished, and the copies swap:
// the update overlaps the previous frame's temporal / spatial / shade passes instead of waiting for
// every enqueued frame (C5 1080p: 484 -> 537 frames/s).
extern "C" int rs_scene_update_positions(rs_scene* s, const float* positions, const float* normals) {
    if (!s || !positions) return fail(s ? s->ctx : nullptr, RS_E_INVALID, "rs_scene_update_positions: null argument");
    rs_context* c = s->ctx;
    if (c->active) return fail(c, RS_E_INVALID, "rs_scene_update_positions: a frame is in flight");
    HIPCHK(c, enter(c));
    const size_t nf = 9 * (size_t)s->n_tris;
    if (nf == 0) return RS_OK;
    // frames in flight and positions only (no normals): pipelined into the other
    // scene copy; otherwise in place after every enqueued frame (the next frame joins the context stream)
    const bool pipelined = c->ahead > 0 && !normals;
    const int L = c->ahead > 0 ? (int)(c->seq % (uint64_t)(c->ahead + 1)) : 0;
    hipStream_t st = pipelined ? c->lane[L] : c->stream;
    const int k = s->stage_i;
    s->stage_i ^= 1;
    if (!s->h_stage[k]) {
        HIPCHK(c, hipHostMalloc(&s->h_stage[k], 2 * nf * sizeof(float), hipHostMallocDefault));
        HIPCHK(c, hipEventCreateWithFlags(&s->stage_ev[k], hipEventDisableTiming));
    } else {
        HIPCHK(c, hipEventSynchronize(s->stage_ev[k]));
    }
    std::memcpy(s->h_stage[k], positions, nf * sizeof(float));
    if (!s->update_ev) HIPCHK(c, hipEventCreateWithFlags(&s->update_ev, hipEventDisableTiming));
    if (s->update_recorded) HIPCHK(c, hipStreamWaitEvent(st, s->update_ev, 0));   // d_pos and the copies
    float4 *nodes = s->d_nodes, *tris = s->d_tris, *em = s->d_emis;
    float* cdf = s->d_cdf;
    int* guide = s->d_cdf_guide;
    const size_t bn = 2 * ((size_t)s->n_nodes + 1) * sizeof(float4), bt = 3 * (size_t)s->n_tris * sizeof(float4),
                 be = 8 * (size_t)s->n_emis * sizeof(float4), bc = (size_t)std::max(1u, s->n_emis) * sizeof(float),
                 bg = (kCdfGuide + 1) * sizeof(int), bnrm = 3 * (size_t)s->n_tris * sizeof(float4);
    if (!s->a_nodes) {                           // the second copy, on first use: topology and tables copied
        sync_all(c);
        HIPCHK(c, hipMalloc(&s->a_nodes, bn));
        HIPCHK(c, hipMalloc(&s->a_tris, bt));
        HIPCHK(c, hipMalloc(&s->a_emis, std::max<size_t>(be, sizeof(float4))));
        HIPCHK(c, hipMalloc(&s->a_cdf, bc));
        HIPCHK(c, hipMalloc(&s->a_cdf_guide, bg));
        HIPCHK(c, hipMemcpyAsync(s->a_nodes, s->d_nodes, bn, hipMemcpyDeviceToDevice, st));
        HIPCHK(c, hipMemcpyAsync(s->a_tris, s->d_tris, bt, hipMemcpyDeviceToDevice, st));
        if (be) HIPCHK(c, hipMemcpyAsync(s->a_emis, s->d_emis, be, hipMemcpyDeviceToDevice, st));
        HIPCHK(c, hipMemcpyAsync(s->a_cdf, s->d_cdf, bc, hipMemcpyDeviceToDevice, st));
        HIPCHK(c, hipMemcpyAsync(s->a_cdf_guide, s->d_cdf_guide, bg, hipMemcpyDeviceToDevice, st));
        if (s->wide_on) if (int rc = wide_copy(c, s->wide, s->a_wide, st)) return rc;
    }
    WideBvh* wt = &s->wide;                      // the 8-wide tree the refit writes
    if (pipelined) {
        // every frame that read the copy about to be written has finished (a lane's frames in stream order):
        // the frames of that generation, and tile frames that rebuilt elements from it as the previous one
        for (int l = 0; l < kLanes; ++l)
            if (c->lane_scene[l] == s && (((s->gen - c->lane_gen[l]) & 1) || c->lane_prevgeo[l]) && c->lane_done[l])
                HIPCHK(c, hipStreamWaitEvent(st, c->lane_done[l], 0));
        nodes = s->a_nodes; tris = s->a_tris; em = s->a_emis; cdf = s->a_cdf; guide = s->a_cdf_guide;
        wt = &s->a_wide;
        s->a_nrm = false;
    } else {
        c->join_next = true;                     // the next frame's initial pass must see the new geometry
        // in place (after every enqueued frame): the current geometry becomes the a_* copy first, so a
        // tile's next temporal pass can still trace the previous frame's geometry
        HIPCHK(c, hipMemcpyAsync(s->a_nodes, s->d_nodes, bn, hipMemcpyDeviceToDevice, st));
        HIPCHK(c, hipMemcpyAsync(s->a_tris, s->d_tris, bt, hipMemcpyDeviceToDevice, st));
        if (s->wide_on) if (int rc = wide_copy(c, s->wide, s->a_wide, st)) return rc;
        s->a_nrm = normals != nullptr;
        if (s->a_nrm) {
            if (!s->a_tri_nrm) HIPCHK(c, hipMalloc(&s->a_tri_nrm, bnrm));
            HIPCHK(c, hipMemcpyAsync(s->a_tri_nrm, s->d_tri_nrm, bnrm, hipMemcpyDeviceToDevice, st));
        }
    }
    s->a_geo = s->geo_gen;                       // after the update: a_* = this generation, d_* = the next
    s->geo_gen++;
    HIPCHK(c, hipMemcpyAsync(s->d_pos, s->h_stage[k], nf * sizeof(float), hipMemcpyHostToDevice, st));
    if (normals) {
        s->h_nrm.assign(normals, normals + nf);
        if (!s->d_nrm_stage) HIPCHK(c, hipMalloc(&s->d_nrm_stage, nf * sizeof(float)));
        std::memcpy(s->h_stage[k] + nf, normals, nf * sizeof(float));
        HIPCHK(c, hipMemcpyAsync(s->d_nrm_stage, s->h_stage[k] + nf, nf * sizeof(float), hipMemcpyHostToDevice, st));
        k_set_normals<<<(s->n_tris + 255) / 256, 256, 0, st>>>(s->d_nrm_stage, s->n_tris, s->d_tri_nrm);
    }
    HIPCHK(c, hipEventRecord(s->stage_ev[k], st));
    std::string err;
    int tail[2];
    if (bvh_refit(nodes, tris, s->d_pos, s->d_refit_order, s->d_refit_lvl, s->refit_lvl, st, tail, err) != 0)
        return fail(c, RS_E_HIP, "rs_scene_update_positions: " + err);
    RefitArgs R{nodes, tris, s->d_pos, s->d_refit_order, s->d_refit_lvl, tail[0], tail[1]};
    // the 8-wide tree keeps its topology and is refit too (rs_refit.h): large levels alone, the last run of
    // small levels up to the root in the fused launch's third workgroup
    WideRefitArgs W = wide_refit_args(*wt, s->d_pos, -1, 0);
    if (s->wide_on) {
        const std::vector<WideBatch> wb = wide_refit_batches(*wt);
        for (size_t i = 0; i < wb.size(); ++i) {
            if (i + 1 == wb.size() && wb[i].blocks == 1) { W.l_deep = wb[i].l_deep; W.l_top = wb[i].l_top; break; }
            WideRefitArgs A = wide_refit_args(*wt, s->d_pos, wb[i].l_deep, wb[i].l_top);
            k_wide_refit<<<wb[i].blocks, kRefitBlock, 0, st>>>(A);
        }
    }
    // the light tables, the binary refit's last levels and the wide refit's last levels, one workgroup each
    k_scene_update<<<3, kLightBlock, 0, st>>>(s->d_pos, s->d_tri_nrm, s->d_mats, s->d_emis_tri, s->n_emis, em, cdf, guide,
                                              R, W);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(s->update_ev, st));
    s->update_recorded = true;
    if (pipelined) {                             // later frames read the new copy
        std::swap(s->d_nodes, s->a_nodes); std::swap(s->d_tris, s->a_tris); std::swap(s->d_emis, s->a_emis);
        std::swap(s->d_cdf, s->a_cdf); std::swap(s->d_cdf_guide, s->a_cdf_guide);
        std::swap(s->wide, s->a_wide);
        s->gen++;
    }
    return RS_OK;
}

// Full rebuild (light tables on the host + a new PLOC tree) from the scene's current device positions:
// restores tree quality after large motions.  Synchronous.
extern "C" int rs_scene_rebuild(rs_scene* s) {
    if (!s) return fail(nullptr, RS_E_INVALID, "rs_scene_rebuild: null scene");
    rs_context* c = s->ctx;
    if (c->active) return fail(c, RS_E_INVALID, "rs_scene_rebuild: a frame is in flight");
    HIPCHK(c, enter(c));
    std::vector<float> pos(9 * (size_t)s->n_tris);
    if (!pos.empty()) {
        if (s->update_recorded) HIPCHK(c, hipStreamWaitEvent(c->stream, s->update_ev, 0));   // a pipelined update
        HIPCHK(c, hipMemcpyAsync(pos.data(), s->d_pos, pos.size() * sizeof(float), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    std::string err;
    if (build_geometry(c, s, pos, err) != 0) return fail(c, RS_E_HIP, "rs_scene_rebuild: " + err);
    return RS_OK;
}

extern "C" int rs_scene_create_textured(rs_context* c, const rs_mesh_desc* meshes, uint32_t n_meshes,
                                        const rs_material_desc* materials, uint32_t n_materials,
                                        const rs_texture_desc* textures, uint32_t n_textures, rs_scene** out) {
    if (!c || !out || (n_meshes && !meshes) || (n_materials && !materials))
        return fail(c, RS_E_INVALID, "rs_scene_create: null argument");
    *out = nullptr;
    HIPCHK(c, enter(c));
    std::vector<float> pos, nrm, uv, tan;
    std::vector<uint32_t> tri_mat;
    bool any_uv = false, any_tan = false;
    for (uint32_t m = 0; m < n_meshes; ++m) {
        any_uv |= meshes[m].texcoords != nullptr;
        any_tan |= meshes[m].tangents != nullptr;
    }
    for (uint32_t m = 0; m < n_meshes; ++m) {
        const rs_mesh_desc& d = meshes[m];
        if (d.n_tris && (!d.positions || !d.normals)) return fail(c, RS_E_INVALID, "rs_scene_create: null mesh buffer");
        pos.insert(pos.end(), d.positions, d.positions + 9 * (size_t)d.n_tris);
        nrm.insert(nrm.end(), d.normals, d.normals + 9 * (size_t)d.n_tris);
        tri_mat.insert(tri_mat.end(), d.n_tris, d.material);
        if (any_uv) {
            if (d.texcoords) uv.insert(uv.end(), d.texcoords, d.texcoords + 6 * (size_t)d.n_tris);
            else uv.insert(uv.end(), 6 * (size_t)d.n_tris, 0.0f);
        }
        if (any_tan) {
            if (d.tangents) tan.insert(tan.end(), d.tangents, d.tangents + 9 * (size_t)d.n_tris);
            else tan.insert(tan.end(), 9 * (size_t)d.n_tris, 0.0f);
        }
    }
    return scene_from_arrays(c, pos, nrm, tri_mat, materials, n_materials, uv, tan, textures, n_textures, out);
}

extern "C" int rs_scene_create(rs_context* c, const rs_mesh_desc* meshes, uint32_t n_meshes,
                               const rs_material_desc* materials, uint32_t n_materials, rs_scene** out) {
    return rs_scene_create_textured(c, meshes, n_meshes, materials, n_materials, nullptr, 0, out);
}

static rs_texture_desc image_desc(const Image& im, int srgb) {
    rs_texture_desc d;
    d.width = (uint32_t)im.w; d.height = (uint32_t)im.h; d.channels = (uint32_t)im.channels;
    d.format = im.is_float ? RS_TEX_F32 : RS_TEX_U8;
    d.data = im.is_float ? (const void*)im.f32.data() : (const void*)im.u8.data();
    d.srgb_expand = srgb;
    return d;
}

extern "C" int rs_scene_load_obj(rs_context* c, const char* path, rs_scene** out) {
    if (!c || !path || !out) return fail(c, RS_E_INVALID, "rs_scene_load_obj: null argument");
    HIPCHK(c, enter(c));
    ObjScene o;
    std::string err;
    int rc = load_obj_file(path, o, err);
    if (rc) return fail(c, rc == -3 ? RS_E_UNSUPPORTED : RS_E_IO, err);
    std::vector<rs_texture_desc> tex;
    for (size_t i = 0; i < o.images.size(); ++i) tex.push_back(image_desc(o.images[i], o.srgb[i]));
    const bool textured = !tex.empty();
    static const std::vector<float> none;
    return scene_from_arrays(c, o.pos, o.nrm, o.tri_mat, o.mats.data(), (uint32_t)o.mats.size(), textured ? o.uv : none,
                             textured ? o.tan : none, tex.data(), (uint32_t)tex.size(), out);
}

// Scene::loadSkybox / SphericalMap (pg/Scene.cpp:46-50, pg/SphericalMap.h:8-10): the sky is kept as the
// last texture of the scene's buffer (material map indices are unaffected)
extern "C" int rs_scene_set_sky(rs_scene* s, const rs_texture_desc* d) {
    if (!s) return fail(nullptr, RS_E_INVALID, "rs_scene_set_sky: null scene");
    rs_context* c = s->ctx;
    if (c->active) return fail(c, RS_E_INVALID, "rs_scene_set_sky: a frame is in flight");
    HIPCHK(c, enter(c));
    HIPCHK(c, hipStreamSynchronize(c->stream));        // enqueued frames may still read the texture buffer
    c->join_next = true;
    rs_scene::HostTex t;
    std::string err;
    if (d && !prepare_texture(*d, 0, t, err)) return fail(c, RS_E_INVALID, "rs_scene_set_sky: " + err);
    if (s->sky >= 0) { s->h_tex.pop_back(); s->sky = -1; }
    if (d) { s->h_tex.push_back(std::move(t)); s->sky = (int)s->h_tex.size() - 1; }
    if (upload_textures(c, s, err) != 0) return fail(c, RS_E_HIP, "rs_scene_set_sky: " + err);
    return RS_OK;
}

extern "C" int rs_scene_load_sky(rs_scene* s, const char* path) {
    if (!s || !path) return fail(s ? s->ctx : nullptr, RS_E_INVALID, "rs_scene_load_sky: null argument");
    Image im;
    std::string err;
    int rc = load_image(path, im, err);
    if (rc) return fail(s->ctx, rc == -3 ? RS_E_UNSUPPORTED : RS_E_IO, err);
    const rs_texture_desc d = image_desc(im, 0);
    return rs_scene_set_sky(s, &d);
}

extern "C" int rs_image_decode(const char* path, uint32_t* w, uint32_t* h, uint32_t* ch, int32_t* fmt, void* out,
                               size_t out_bytes) {
    if (!path || !w || !h || !ch || !fmt) return fail(nullptr, RS_E_INVALID, "rs_image_decode: null argument");
    Image im;
    std::string err;
    int rc = load_image(path, im, err);
    if (rc) return fail(nullptr, rc == -3 ? RS_E_UNSUPPORTED : RS_E_IO, err);
    *w = (uint32_t)im.w; *h = (uint32_t)im.h; *ch = (uint32_t)im.channels;
    *fmt = im.is_float ? RS_TEX_F32 : RS_TEX_U8;
    if (!out) return RS_OK;
    const size_t need = im.is_float ? im.f32.size() * sizeof(float) : im.u8.size();
    if (out_bytes < need) return fail(nullptr, RS_E_INVALID, "rs_image_decode: output buffer too small");
    std::memcpy(out, im.is_float ? (const void*)im.f32.data() : (const void*)im.u8.data(), need);
    return RS_OK;
}

extern "C" void rs_scene_destroy(rs_scene* s) {
    if (!s) return;
    if (s->ctx) hipSetDevice(s->ctx->device);
    if (s->ctx && s->ctx->stream) hipStreamSynchronize(s->ctx->stream);
    if (s->ctx) sync_all(s->ctx);
    void* ptrs[] = {s->d_pos, s->d_nodes, s->d_tris, s->d_tri_nrm, s->d_mats, s->d_emis, s->d_cdf, s->d_cdf_guide,
                    s->d_emis_tri, s->d_refit_order, s->d_refit_lvl, s->d_nrm_stage, s->d_tex, s->d_texd, s->d_uv,
                    s->d_tan, s->a_tri_nrm, s->a_nodes, s->a_tris, s->a_emis, s->a_cdf, s->a_cdf_guide, s->d_ebucket};
    for (void* p : ptrs) if (p) hipFree(p);
    wide_free(s->wide);
    wide_free(s->a_wide);
    for (int k = 0; k < 2; ++k) {
        if (s->h_stage[k]) hipHostFree(s->h_stage[k]);
        if (s->stage_ev[k]) hipEventDestroy(s->stage_ev[k]);
    }
    if (s->update_ev) hipEventDestroy(s->update_ev);
    {
    }
    delete s;
}

extern "C" int rs_debug_wide_tree(const rs_scene* s, uint32_t* n_nodes, uint32_t* n_tris, int32_t* depth, uint32_t* words,
                                  int32_t* prims) {
    if (!s || !n_nodes || !n_tris) return fail(s ? s->ctx : nullptr, RS_E_INVALID, "rs_debug_wide_tree: null argument");
    rs_context* c = s->ctx;
    HIPCHK(c, enter(c));
    const WideBvh& w = s->wide;
    const bool on = s->wide_on && w.nodes;
    *n_nodes = on ? w.n_nodes : 0u;
    *n_tris = on ? w.n_tris : 0u;
    if (depth) *depth = on ? w.depth : -1;
    if (!on || (!words && !prims)) return RS_OK;
    if (s->update_recorded) HIPCHK(c, hipStreamWaitEvent(c->stream, s->update_ev, 0));
    if (words) HIPCHK(c, hipMemcpyAsync(words, w.nodes, (size_t)w.n_nodes * 5 * sizeof(uint4), hipMemcpyDeviceToHost, c->stream));
    std::vector<float4> t;
    if (prims) {
        t.resize(3 * (size_t)w.n_tris);
        HIPCHK(c, hipMemcpyAsync(t.data(), w.tris, t.size() * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (prims)
        for (uint32_t k = 0; k < w.n_tris; ++k) std::memcpy(&prims[k], &t[3 * (size_t)k].w, 4);
    return RS_OK;
}

extern "C" int rs_scene_walk_info(const rs_scene* s, uint32_t* wide_nodes, int32_t* wide_depth, int32_t* status) {
    if (!s) return fail(nullptr, RS_E_INVALID, "rs_scene_walk_info: null scene");
    const bool on = s->wide_on && s->wide.nodes;
    if (wide_nodes) *wide_nodes = on ? s->wide.n_nodes : 0u;
    if (wide_depth) *wide_depth = on ? s->wide.depth : -1;
    if (status) *status = on ? RS_WIDE_LIVE : (s->wide.status ? s->wide.status : RS_WIDE_TOO_DEEP);
    return RS_OK;
}

extern "C" int rs_scene_info(const rs_scene* s, uint32_t* n_tris, uint32_t* n_emissive, uint32_t* n_nodes,
                             float* build_ms) {
    if (!s) return fail(nullptr, RS_E_INVALID, "rs_scene_info: null scene");
    if (n_tris) *n_tris = s->n_tris;
    if (n_emissive) *n_emissive = s->n_emis;
    if (n_nodes) *n_nodes = s->n_nodes;
    if (build_ms) *build_ms = s->build_ms;
    return RS_OK;
}

// --------------------------------------------------------------------------- frame / tile driver
static dim3 grid_rows(int W, int ya, int yb) { return dim3((W + 15) / 16, (yb - ya + 15) / 16); }

// launch kernel<Trav> for the frame's traversal kind
// the kernel instantiation of the frame: walk kind | TRAV_WIDE when the scene's 8-wide tree is live
// (rs_scene.h Trav; c->twide is taken from the scene when the frame begins)
#define LAUNCH_TRAV_BS_SH_ON(c, st, kernel, grid, bs, sh, ...)                                              \
    do {                                                                                                   \
        switch ((c)->trav | ((c)->twide ? TRAV_WIDE : 0)) {                                                \
            case TRAV_LANE | TRAV_WIDE: kernel<TRAV_LANE | TRAV_WIDE><<<(grid), (bs), (sh), (st)>>>(__VA_ARGS__); break; \
            case TRAV_LANE: kernel<TRAV_LANE><<<(grid), (bs), (sh), (st)>>>(__VA_ARGS__); break;                  \
            case TRAV_WIDE: kernel<TRAV_LOCKSTEP | TRAV_WIDE><<<(grid), (bs), (sh), (st)>>>(__VA_ARGS__); break;  \
            default: kernel<TRAV_LOCKSTEP><<<(grid), (bs), (sh), (st)>>>(__VA_ARGS__); break;                     \
        }                                                                                                  \
    } while (0)
#define LAUNCH_TRAV_BS_ON(c, st, kernel, grid, bs, ...) LAUNCH_TRAV_BS_SH_ON(c, st, kernel, grid, bs, 0, __VA_ARGS__)
#define LAUNCH_TRAV_BS_SH(c, kernel, grid, bs, sh, ...) LAUNCH_TRAV_BS_SH_ON(c, (c)->fs, kernel, grid, bs, sh, __VA_ARGS__)
// the same with extra template bits X (a pass's own variant bits above the traversal kind's)
#define LAUNCH_TRAV_X(c, X, kernel, grid, ...)                                                              \
    do {                                                                                                   \
        switch ((c)->trav | ((c)->twide ? TRAV_WIDE : 0)) {                                                \
            case TRAV_LANE | TRAV_WIDE: kernel<TRAV_LANE | TRAV_WIDE | (X)><<<(grid), 256, 0, (c)->fs>>>(__VA_ARGS__); break; \
            case TRAV_LANE: kernel<TRAV_LANE | (X)><<<(grid), 256, 0, (c)->fs>>>(__VA_ARGS__); break;                  \
            case TRAV_WIDE: kernel<TRAV_LOCKSTEP | TRAV_WIDE | (X)><<<(grid), 256, 0, (c)->fs>>>(__VA_ARGS__); break;  \
            default: kernel<TRAV_LOCKSTEP | (X)><<<(grid), 256, 0, (c)->fs>>>(__VA_ARGS__); break;                     \
        }                                                                                                  \
    } while (0)
#define LAUNCH_TRAV_ON(c, st, kernel, grid, ...) LAUNCH_TRAV_BS_ON(c, st, kernel, grid, 256, __VA_ARGS__)
#define LAUNCH_TRAV(c, kernel, grid, ...) LAUNCH_TRAV_ON(c, (c)->fs, kernel, grid, __VA_ARGS__)
#define LAUNCH_TRAV_BS(c, kernel, grid, bs, ...) LAUNCH_TRAV_BS_ON(c, (c)->fs, kernel, grid, bs, __VA_ARGS__)

// fold a finished frame's pass times (event-ring slot s) into the running totals
static void fold_slot(rs_context* c, int s) {
    if (!c->ev_pending[s]) return;
    c->ev_pending[s] = false;
    hipEvent_t* e = c->evr[s];
    if (hipEventSynchronize(e[EV_SHADE]) != hipSuccess) return;
    float v[6] = {};
    (void)hipEventElapsedTime(&v[0], e[EV_BEGIN], e[EV_INIT]);
    (void)hipEventElapsedTime(&v[1], e[EV_INIT], e[EV_VIS]);
    (void)hipEventElapsedTime(&v[2], e[EV_VIS], e[EV_TEMPORAL]);
    (void)hipEventElapsedTime(&v[3], e[EV_TEMPORAL], e[EV_SPATIAL]);
    (void)hipEventElapsedTime(&v[4], e[EV_SPATIAL], e[EV_SHADE]);
    (void)hipEventElapsedTime(&v[5], e[EV_BEGIN], e[EV_SHADE]);
    for (int i = 0; i < 6; ++i) c->tot_ms[i] += v[i];
    c->tot_frames++;
}

// RS_TRAVERSAL_AUTO: the first 2*kTuneRuns frames of a scene alternate the two kinds; per kind the first
// run is a warm-up (lazy code-object load, cold caches), the next kTuneRuns-1 are timed (their kernels
// only, each tuning frame running alone: record_traversal_time).
constexpr int kTuneRuns = 3;
static void pick_traversal(rs_context* c, const rs_scene* s) {
    c->tuning = false;
    if (c->trav_mode == RS_TRAVERSAL_LOCKSTEP) { c->trav = TRAV_LOCKSTEP; return; }
    if (c->trav_mode == RS_TRAVERSAL_LANE) { c->trav = TRAV_LANE; return; }
    if (s->trav_choice >= 0) { c->trav = s->trav_choice; return; }
    c->trav = s->trav_runs[TRAV_LOCKSTEP] <= s->trav_runs[TRAV_LANE] ? TRAV_LOCKSTEP : TRAV_LANE;
    for (auto& e : c->tune_ev)
        if (!e && hipEventCreate(&e) != hipSuccess) { e = nullptr; return; }   // untimed: stays un-tuned
    c->tune_n = 0;
    c->tuning = true;
    // full-frame tuning frames also record per-row cost for the tile-row dispatch order
    c->tune_rows = false;
    if (c->order_on && !c->track_rows && c->tile.y0 == 0 && c->tile.y1 == c->H) {
        float*& p = c->d_tune_cost[c->trav];
        if (!p && hipMalloc(&p, (size_t)c->H * sizeof(float)) == hipSuccess)
            (void)hipMemsetAsync(p, 0, (size_t)c->H * sizeof(float), c->stream);
        c->tune_rows = p != nullptr;
    }
}
// The tuning frames' per-row wave time of the chosen kind -> tile-row dispatch order, costliest first
// (ties: top row first).  Full frames only; the frames are already synchronised here.
static void order_tile_rows(rs_context* c, int kind) {
    c->tune_rows = false;
    if (!c->d_tune_cost[kind]) return;
    std::vector<float> rc((size_t)c->H);
    if (hipMemcpy(rc.data(), c->d_tune_cost[kind], rc.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return;
    const int n = (c->H + 15) / 16;
    std::vector<double> cost(n, 0.0);
    for (int y = 0; y < c->H; ++y) cost[y / 16] += rc[y];
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
    if (!c->d_order && hipMalloc(&c->d_order, (size_t)n * sizeof(int)) != hipSuccess) { c->d_order = nullptr; return; }
    if (hipMemcpy(c->d_order, order.data(), (size_t)n * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) return;
    c->n_order = n;
}
static void record_traversal_time(rs_context* c) {
    if (!c->tuning) return;
    c->tuning = false;
    // a tuning frame runs alone (rs_tile_begin: on the context's stream, and the next frame waits for
    // it), and only its kernels are timed: begin..temporal, each spatial kernel, spatial..shade -- not
    // the halo exchanges of a multi-GPU frame, which wait for other ranks
    c->join_next = true;
    float ms = 0.0f, t = 0.0f;
    if (hipEventSynchronize(c->ev[EV_SHADE]) != hipSuccess ||
        hipEventElapsedTime(&ms, c->ev[EV_BEGIN], c->ev[EV_TEMPORAL]) != hipSuccess ||
        hipEventElapsedTime(&t, c->ev[c->tune_n ? EV_SPATIAL : EV_TEMPORAL], c->ev[EV_SHADE]) != hipSuccess)
        return;
    ms += t;
    for (int i = 0; i + 1 < c->tune_n; i += 2) {
        if (hipEventElapsedTime(&t, c->tune_ev[i], c->tune_ev[i + 1]) != hipSuccess) return;
        ms += t;
    }
    const rs_scene* s = c->scene;
    if (++s->trav_runs[c->trav] > 1) s->trav_ms[c->trav] += ms;
    if (s->trav_runs[TRAV_LOCKSTEP] >= kTuneRuns && s->trav_runs[TRAV_LANE] >= kTuneRuns) {
        s->trav_choice = s->trav_ms[TRAV_LANE] < s->trav_ms[TRAV_LOCKSTEP] ? TRAV_LANE : TRAV_LOCKSTEP;
        order_tile_rows(c, s->trav_choice);
    }
}
static size_t grid_waves(dim3 g, int waves_per_block = 4) { return (size_t)g.x * g.y * waves_per_block; }

// the ray-count slot buffer k (of two: consecutive frames can be in flight) with >= need slots; the
// frame's launches then take consecutive slices of it (count_slot)
static bool use_parts(rs_context* c, int k, size_t need) {
    c->pk = k;
    c->part_used = 0;
    if (need > c->part_caps[k]) {
        sync_all(c);
        if (c->parts[k]) hipFree(c->parts[k]);
        c->parts[k] = nullptr; c->part_caps[k] = 0;
        if (hipMalloc(&c->parts[k], need * sizeof(uint2)) != hipSuccess) { c->d_part = nullptr; c->part_cap = 0; return false; }
        c->part_caps[k] = need;
    }
    c->d_part = c->parts[k]; c->part_cap = c->part_caps[k];
    return true;
}
// ray-count slots for one launch (rs_passes.h CountSlot); capacity is reserved in rs_tile_begin
static CountSlot count_slot(rs_context* c, dim3 grid, int waves_per_block = 4) {
    const size_t n = grid_waves(grid, waves_per_block);
    if (c->part_used + n > c->part_cap) {       // more launches than reserved (a pass re-run): grow, keep slots
        const size_t cap = 2 * (c->part_used + n);
        uint2* np = nullptr;
        sync_all(c);
        if (hipMalloc(&np, cap * sizeof(uint2)) == hipSuccess) {
            if (c->part_used) hipMemcpy(np, c->d_part, c->part_used * sizeof(uint2), hipMemcpyDeviceToDevice);
            hipFree(c->d_part);
            c->d_part = c->parts[c->pk] = np; c->part_cap = c->part_caps[c->pk] = cap;
        } else {
            c->part_used = 0;                   // out of memory: recount from slot 0 (totals undercount)
        }
    }
    float* rows = c->track_rows ? c->d_rowcost : (c->tune_rows ? c->d_tune_cost[c->trav] : nullptr);
    CountSlot s{c->d_part + c->part_used, &c->d_cnt->reproj_outside, rows, c->F.y0, c->F.y1};
    c->part_used += n;
    return s;
}
// reserve slots for every launch of a frame: initial + visibility + temporal + P spatial + shade
// the wave-sorted initial pass (rs_passes.h k_gbuffer_initial_sorted) for the per-lane walks: sorting a
// tile's shadow rays by octant x light bucket cuts C3's initial pass 16.27 -> 15.25 ms; the lockstep walk
// already shares one node stream per wave and loses to the sort's extra phases (C2: 1.31 -> 1.69 ms)
static bool want_sorted(const rs_context* c, const rs_frame_params* P, const rs_scene* s) {
    if (P->m_area <= 0 || s->n_emis >= (1u << 21) || c->sort_mode == RS_SPLIT_OFF) return false;
    return c->sort_mode == RS_SPLIT_ON || c->trav == TRAV_LANE;
}
static dim3 grid_split(int W, int ya, int yb) { return dim3((W + 7) / 8, (yb - ya + 7) / 8); }
// the initial pass runs candidate-split when asked, or (AUTO) when one thread per pixel would give the
// launch too few rounds of the device's resident waves (a rank's band of a multi-GPU frame) and
// the walks are lockstep: per-lane walks are latency-bound and need the occupancy the split kernel's
// LDS takes away (C3 1/8 band: 5.3 ms split vs 4.2 ms one thread per pixel)
static bool want_split(const rs_context* c, const rs_frame_params* P, int gy0, int gy1) {
    if (P->m_area + P->m_brdf > kSplitMaxCand || P->m_brdf > kSplitMaxBrdf) return false;
    if (c->split_mode == RS_SPLIT_ON) return true;
    if (c->split_mode == RS_SPLIT_OFF) return false;
    // with frames in flight the neighbouring frames fill a launch's tail: split only below one round
    // (C2 1/4 band, 1.4 rounds: 0.363 ms/frame unsplit vs 0.411 split with the cost-weighted groups, r04;
    // 1/8 band, 0.8 rounds: 0.209 split vs 0.26); one frame at a time, below 3 rounds (1/8 band 0.64 -> 0.40 ms)
    const size_t rounds = c->ahead > 0 ? 1 : 3;
    return c->trav == TRAV_LOCKSTEP && grid_waves(grid_rows(c->W, gy0, gy1)) < rounds * c->wave_slots;
}
// the sorted initial pass by persistent waves (RESTIR_PERSIST_SORTED).  AUTO (default): with frames in flight
// (run-ahead > 0) and more than one round of the one-launch kernel's waves, kPersistSortedWgs resident workgroups
// per CU -- fewer than the kernel's occupancy, so the other frames' temporal and spatial passes run beside it.
// The pass alone is slower that way (C3 16.7-16.9 vs 14.9-15.0 ms), the frame throughput higher (C3 60.8-61.6 vs
// 60.0-60.1 frames/s over three sessions; 2 workgroups per CU: 58.3-58.5); one frame in flight keeps
// the one-launch kernel.
constexpr int kPersistSortedWgs = 3;
static int persist_sorted_wgs(rs_context* c) {
    const int kind = c->trav | (c->twide ? TRAV_WIDE : 0);
    int& n = c->persist_sorted_wgs[kind];
    if (!n) {
        hipError_t e = hipSuccess;
        switch (kind) {
            case TRAV_LANE | TRAV_WIDE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gbuffer_initial_sorted_pq<TRAV_LANE | TRAV_WIDE>, 256, 0); break;
            case TRAV_LANE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gbuffer_initial_sorted_pq<TRAV_LANE>, 256, 0); break;
            case TRAV_WIDE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gbuffer_initial_sorted_pq<TRAV_WIDE>, 256, 0); break;
            default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gbuffer_initial_sorted_pq<TRAV_LOCKSTEP>, 256, 0); break;
        }
        if (e != hipSuccess || n <= 0) n = RS_INITIAL_WAVES_SORT;
    }
    return n;
}
static int persist_sorted_grid_wgs(rs_context* c) {     // resident workgroups per CU of the persistent launch
    int n = std::min(persist_sorted_wgs(c), kPersistSortedWgs);
    if (const char* t = std::getenv("RESTIR_PERSIST_SORTED_WGS")) n = std::max(1, std::min(persist_sorted_wgs(c), std::atoi(t)));
    return n;
}
static bool want_persist_sorted(rs_context* c, dim3 grid) {
    if (c->persist_sorted == RS_SPLIT_OFF) return false;
    if (c->persist_sorted == RS_SPLIT_ON) return true;
    // full frames only, and not while row costs are being recorded: a throttled persistent launch charges its
    // early (costly, contended) tiles more and its late ones less than the one-launch kernel a band runs, so
    // bounds balanced on its row costs come out uneven (C4's eight 4K bands: max 9.59 vs 8.96 ms)
    const bool full = c->tile.y0 == 0 && c->tile.y1 == c->H;
    return c->ahead > 0 && full && !c->track_rows && !c->tune_rows &&
           grid_waves(grid) > (size_t)c->cus * 4 * (size_t)persist_sorted_wgs(c);
}
// the sorted initial pass's hand-off buffers of lane k (FrameConst::cand_w, cand_ray: kSortChunk x 64 candidates per
// wave slot, 20 B each) for `slots` wave slots, grown on demand; false (nothing allocated) when the device is out of
// memory.  Sized by the launch, not the frame: the persistent launch's resident waves (C3 1080p: 3 workgroups x 4
// waves x 256 CUs x 20 KB = 63 MB per lane), a one-launch band its own tiles.
static bool ensure_handoff(rs_context* c, int k, size_t slots) {
    if (slots <= c->cand_slots[k]) return true;
    sync_all(c);                                   // frames in flight on the lane may still read the old buffers
    if (c->candw[k]) hipFree(c->candw[k]);
    if (c->candr[k]) hipFree(c->candr[k]);
    c->candw[k] = nullptr; c->candr[k] = nullptr; c->cand_slots[k] = 0;
    const size_t n = slots * (size_t)(kSortChunk * 64);
    if (hipMalloc(&c->candw[k], n * sizeof(float)) != hipSuccess || hipMalloc(&c->candr[k], n * sizeof(float4)) != hipSuccess) {
        (void)hipGetLastError();
        if (c->candw[k]) hipFree(c->candw[k]);
        c->candw[k] = nullptr; c->candr[k] = nullptr;
        return false;
    }
    c->cand_slots[k] = slots;
    return true;
}
static bool reserve_count_slots(rs_context* c, int k, const rs_frame_params* P, int gy0, int gy1, int y0, int y1,
                                size_t extra = 0) {
    const size_t spatial = grid_waves(grid_rows(c->W, y0, y1));
    size_t need = (c->split ? grid_waves(grid_split(c->W, gy0, gy1), kSplit) : grid_waves(grid_rows(c->W, gy0, gy1))) +
                  grid_waves(grid_rows(c->W, y0, y1)) * 4 + spatial * (size_t)std::max(0, P->spatial_passes) + extra;
    return use_parts(c, k, need);
}

extern "C" int rs_tile_begin(rs_context* c, const rs_scene* s, const rs_camera* cam, const rs_frame_params* P,
                             uint32_t frame_index, const rs_tile_desc* tile) {
    if (!c || !s || !cam || !P || !tile) return fail(c, RS_E_INVALID, "rs_tile_begin: null argument");
    if (s->ctx != c) return fail(c, RS_E_INVALID, "rs_tile_begin: scene belongs to another context");
    if (P->use_skybox && s->sky < 0)
        return fail(c, RS_E_UNSUPPORTED, "use_skybox: the scene has no sky map (rs_scene_set_sky / rs_scene_load_sky)");
    if (P->m_area < 0 || P->m_brdf < 0 || P->spatial_passes < 0 || P->confidence_cap < 0)
        return fail(c, RS_E_INVALID, "rs_frame_params: negative count");
    if (P->do_spatial && (P->spatial_neighbors < 0 || P->spatial_neighbors > 64))
        return fail(c, RS_E_INVALID, "rs_frame_params: spatial_neighbors must be in [0, 64]");
    if (P->spatial_mis < 0 || P->spatial_mis > 4) return fail(c, RS_E_INVALID, "rs_frame_params: bad spatial_mis");
    if (P->debug_reprojection && (tile->y0 != 0 || tile->y1 != c->H))
        return fail(c, RS_E_UNSUPPORTED, "debug_reprojection: full frames only (its marks land on any pixel)");
    if (tile->y0 < 0 || tile->y1 > c->H || tile->y0 >= tile->y1 || tile->margin < 0 || tile->halo < 0 ||
        tile->halo > tile->margin)
        return fail(c, RS_E_INVALID, "rs_tile_begin: bad tile (need 0<=y0<y1<=H, 0<=halo<=margin)");
    HIPCHK(c, enter(c));
    c->scene = s; c->P = *P; c->tile = *tile; c->cam_last = *cam;
    FrameConst& F = c->F;
    F.m_area = P->m_area; F.m_brdf = P->m_brdf; F.k = P->spatial_neighbors; F.spatial_passes = P->spatial_passes;
    F.cap = P->confidence_cap; F.radius = P->spatial_radius; F.min_normal_sim = P->min_normal_similarity;
    F.max_depth_diff = P->max_depth_difference; F.do_spatial = P->do_spatial; F.do_temporal = P->do_temporal;
    F.do_vis_pass = P->do_visibility_pass; F.reject = P->reject_dissimilar; F.mis = P->spatial_mis;
    F.bg = vec3{P->bg_color[0], P->bg_color[1], P->bg_color[2]};
    F.tnear_off = P->tnear_offset; F.tfar_off = P->tfar_offset; F.normal_off = P->normal_offset;
    F.use_sky = P->use_skybox ? 1 : 0;
    F.seed = P->seed; F.frame = frame_index;
    F.W = c->W; F.H = c->H;
    F.y0 = tile->y0; F.y1 = tile->y1;
    F.row_order = c->n_order ? c->d_order : nullptr; F.n_order = c->n_order;
    F.debug_reproj = P->debug_reprojection ? 1 : 0;
    if (F.debug_reproj && !c->d_dbg) HIPCHK(c, hipMalloc(&c->d_dbg, 2 * (size_t)c->W * c->H));
    F.dbg = c->d_dbg;
    F.gy0 = std::max(0, tile->y0 - tile->margin); F.gy1 = std::min(c->H, tile->y1 + tile->margin);
    // G-buffer ring (replaces gBufferLastFrame.setDataFrom, pg/simpleguidx11.cpp:480): this frame
    // writes the slot after the current one; G[gcur] becomes the previous frame's
    int gnew = (c->gcur + 1) % kGRing;
    make_camera(cam, c->H, c->gcam[gnew], F.inv_view);
    std::memcpy(c->ginv[gnew], F.inv_view, sizeof F.inv_view);
    std::memcpy(F.inv_view_prev, c->ginv[c->gcur], sizeof F.inv_view_prev);
    F.cam = c->gcam[gnew];
    F.camp = c->gcam[c->gcur];
    // the frame's stream: lane seq mod (D+1) (run-ahead), else the context's stream
    const int D = c->ahead;
    c->li = D > 0 ? (int)(c->seq % (uint64_t)(D + 1)) : (c->fb_ring == 2 ? (int)(c->seq & 1) : 0);
    // a frame that must follow work enqueued on the context's stream since the last frame (geometry
    // updates, ...) simply runs on that stream (it is ordered after every earlier frame there); the next
    // frame on its lane then waits for it
    pick_traversal(c, s);
    c->twide = s->wide_on;
    if (!c->fbs[c->li]) {                       // a lane's framebuffer, on first use: cleared on the context's
        const size_t bytes = (size_t)c->W * c->H * 3 * sizeof(float);   // stream, so this frame runs there too
        HIPCHK(c, hipMalloc(&c->fbs[c->li], bytes));
        HIPCHK(c, hipMemsetAsync(c->fbs[c->li], 0, bytes, c->stream));
        c->join_next = true;
    }
    const bool on_ctx = D == 0 || c->join_next || c->tuning;   // a traversal-tuning frame runs alone
    c->fs = on_ctx ? c->stream : c->lane[c->li];
    if (c->fb_read[c->li]) {                    // the lane's framebuffer is still being read back
        HIPCHK(c, hipStreamWaitEvent(c->fs, c->fb_read[c->li], 0));
        c->fb_read[c->li] = nullptr;
    }
    c->fb = c->fbs[c->li];
    c->d_cnt = c->cnts[c->li]; c->d_red = c->reds[c->li];
    // reservoir ring: `last` = the previous frame's final buffer (reservoirsLastFrame, a pointer swap,
    // :477); this frame writes two buffers none of the D frames before it touches (they may still run)
    c->last = c->r_last;
    {
        auto used = [&](int i) {
            if (i == c->last) return true;
            for (int g = 0; g < D; ++g)
                if (i == c->rhist[g][0] || i == c->rhist[g][1] || i == c->rhist[g][2]) return true;
            return false;
        };
        c->ra = 0;
        while (used(c->ra)) ++c->ra;
        c->rb = c->ra + 1;
        while (used(c->rb)) ++c->rb;            // < kRRing: D frames touch <= 3D buffers, `last` among them
        for (int g = kMaxAhead - 1; g > 0; --g)
            for (int j = 0; j < 3; ++j) c->rhist[g][j] = c->rhist[g - 1][j];
        c->rhist[0][0] = c->ra; c->rhist[0][1] = c->rb; c->rhist[0][2] = c->last;
    }
    c->rcur = c->ra;
    const bool temporal = P->do_temporal && c->frames > 0;
    const bool spatial = P->do_spatial && P->spatial_passes > 0;
    c->shade_fused = !P->do_visibility_pass && !temporal && !spatial;
    c->temporal_ran = c->spatial_ran = c->ev_temporal = false;
    const DevScene S = s->dev();
    // A band's G-buffer margin (the rows of the spatial halo beyond it) needs the G-buffer only.  Its rows get their
    // own small launch, so the initial pass's 8-row tiles start at the band's first row: otherwise the top and
    // bottom tile rows mix margin rows -- whose lanes idle through the whole candidate loop -- with band rows
    // (C2's 1/8 band: 145 G rows in 19 tile rows for 135 RIS rows, 11 % of the pass's waves idle).  Full frames
    // have no margin.
    const bool margins = c->sep_margin && (F.gy0 < F.y0 || F.gy1 > F.y1);
    FrameConst Fi = F;                          // the rows of the initial pass's launch
    if (margins) { Fi.gy0 = F.y0; Fi.gy1 = F.y1; }
    const size_t margin_waves = margins ? grid_waves(grid_rows(c->W, F.gy0, F.y0)) + grid_waves(grid_rows(c->W, F.y1, F.gy1)) : 0;
    c->split = want_split(c, P, Fi.gy0, Fi.gy1);
    // the initial pass's kernel, chosen (and its hand-off buffers grown) before anything of the frame is enqueued:
    // 0 one thread per pixel, 1 wave-sorted (one launch), 2 wave-sorted by persistent waves
    const dim3 gg = grid_rows(c->W, Fi.gy0, Fi.gy1), gb = grid_rows(c->W, F.y0, F.y1);
    int init_kind = 0;
    dim3 gp(1);
    if (!c->split && want_sorted(c, P, s)) {
        init_kind = want_persist_sorted(c, gg) ? 2 : 1;
        if (init_kind == 2)
            gp = dim3((unsigned)std::min<size_t>((size_t)gg.x * gg.y, (size_t)c->cus * (size_t)persist_sorted_grid_wgs(c)));
        // one slot per resident wave of the persistent launch (reused tile after tile), else per 8x8 tile of the launch
        const size_t slots = init_kind == 2 ? (size_t)gp.x * 4 : (size_t)gg.x * gg.y * 4;
        if (!ensure_handoff(c, c->li, slots)) init_kind = 0;   // out of memory: the one-thread-per-pixel pass (same bits)
    }
    if (!reserve_count_slots(c, c->li, P, Fi.gy0, Fi.gy1, F.y0, F.y1, margin_waves))
        return fail(c, RS_E_HIP, "hipMalloc(count slots) failed");
    if (c->fs != c->stream && c->lane_wait[c->li]) {   // this lane's previous frame ran on the context's stream
        HIPCHK(c, hipStreamWaitEvent(c->fs, c->lane_wait[c->li], 0));
    }
    c->lane_wait[c->li] = nullptr;
    // frames start in order (the previous frame has started -- so every frame up to f-D-1 has finished:
    // the one on this lane by stream order, earlier ones by induction): frames f-D..f-1 are the only
    // ones that can still run beside this frame
    if (c->fs != c->stream && c->prev_begin) HIPCHK(c, hipStreamWaitEvent(c->fs, c->prev_begin, 0));
    if (s->update_recorded) HIPCHK(c, hipStreamWaitEvent(c->fs, s->update_ev, 0));   // the scene copy it reads
    c->frame_scene = s; c->frame_gen = s->gen;
    c->geo_prev = c->geo_last; c->geo_prev_scene = c->geo_last_scene; c->prevgeo_read = false;
    c->join_next = false;
    // (the frame's Counters need no memset: k_reduce_counts stores rays/primary, and the initial pass
    // zeroes reproj_outside before the temporal pass can count -- one API call less per frame)
    c->slot = (int)(c->seq++ % rs_context::kEvRing);
    fold_slot(c, c->slot);                      // the slot's previous frame (kEvRing frames ago)
    for (int i = 0; i < EV_COUNT; ++i) c->ev[i] = c->evr[c->slot][i];
    HIPCHK(c, hipEventRecord(c->ev[EV_BEGIN], c->fs));
    c->prev_begin = c->ev[EV_BEGIN];
    if (margins) {                              // the margin rows' G-buffer (no RIS rows: the candidate loops exit)
        const int rr[2][2] = {{F.gy0, F.y0}, {F.y1, F.gy1}};
        for (const auto& r : rr) {
            if (r[0] >= r[1]) continue;
            FrameConst Fm = F;
            Fm.gy0 = r[0]; Fm.gy1 = r[1];
            const dim3 gm = grid_rows(c->W, r[0], r[1]);
            LAUNCH_TRAV(c, k_gbuffer_initial, gm, S, Fm, c->G[gnew], ResBuf{c->R[c->ra]}, c->fb, 0, count_slot(c, gm));
            HIPCHK(c, hipGetLastError());
        }
    }
    if (c->split) {
        const dim3 gs = grid_split(c->W, Fi.gy0, Fi.gy1);
        LAUNCH_TRAV_BS_SH(c, k_gbuffer_initial_split, gs, 64 * kSplit, split_lds_bytes(P->m_area + P->m_brdf, P->m_brdf),
                          S, Fi, c->G[gnew], ResBuf{c->R[c->ra]}, c->fb,
                    c->shade_fused ? 1 : 0, count_slot(c, gs, kSplit));
    } else if (init_kind > 0) {
        Fi.cand_w = c->candw[c->li];
        Fi.cand_ray = c->candr[c->li];
        if (init_kind == 2) {
            // persistent waves, each pulling 8x8 tiles (rs_passes.h k_gbuffer_initial_sorted_pq); the queue's counters
            // from zero on the frame's stream (the last exiting wave also re-arms them, but an aborted launch would
            // leave every later one pulling past the end)
            const uint32_t nt = gg.x * gg.y * 4u;
            HIPCHK(c, hipMemsetAsync(c->qctr[c->li], 0, 4 * sizeof(uint32_t), c->fs));
            LAUNCH_TRAV(c, k_gbuffer_initial_sorted_pq, gp, S, Fi, c->G[gnew], ResBuf{c->R[c->ra]}, c->fb,
                        c->shade_fused ? 1 : 0, count_slot(c, gp), TileQ{c->qctr[c->li], nt});
        } else {
            LAUNCH_TRAV(c, k_gbuffer_initial_sorted, gg, S, Fi, c->G[gnew], ResBuf{c->R[c->ra]}, c->fb, c->shade_fused ? 1 : 0,
                        count_slot(c, gg));
        }
    } else {
        LAUNCH_TRAV(c, k_gbuffer_initial, gg, S, Fi, c->G[gnew], ResBuf{c->R[c->ra]}, c->fb, c->shade_fused ? 1 : 0,
                    count_slot(c, gg));
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev[EV_INIT], c->fs));
    if (P->do_visibility_pass) {
        LAUNCH_TRAV(c, k_visibility, gb, S, F, c->G[gnew], ResBuf{c->R[c->ra]}, count_slot(c, gb));
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(c->ev[EV_VIS], c->fs));
    c->gprev = c->gcur;
    c->gcur = gnew;       // G[gcur] = this frame, G[gprev] = previous frame
    c->prev_done = c->last_done;
    c->active = true;
    return RS_OK;
}

extern "C" int rs_tile_stream(rs_context* c, void** stream, int* lane) {
    if (!c || !stream) return fail(c, RS_E_INVALID, "rs_tile_stream: null argument");
    if (!c->active) return fail(c, RS_E_INVALID, "rs_tile_stream: no frame in flight");
    *stream = (void*)c->fs;
    if (lane) *lane = c->li;
    return RS_OK;
}

extern "C" int rs_tile_halo_ptr(rs_context* c, int which, void** dptr, size_t* bytes) {
    if (!c || !dptr || !bytes || !c->active) return fail(c, RS_E_INVALID, "rs_tile_halo_ptr: no frame in flight");
    const int h = c->tile.halo, W = c->W;
    int r0;
    switch (which) {
        case 0: r0 = c->tile.y0 - h; break;
        case 1: r0 = c->tile.y1; break;
        case 2: r0 = c->tile.y0; break;
        case 3: r0 = c->tile.y1 - h; break;
        default: return fail(c, RS_E_INVALID, "rs_tile_halo_ptr: which must be 0..3");
    }
    if (h == 0 || r0 < 0 || r0 + h > c->H) { *dptr = nullptr; *bytes = 0; return RS_OK; }
    *dptr = (void*)(c->R[c->rcur] + 3 * (size_t)r0 * W);
    *bytes = (size_t)h * W * 3 * sizeof(float4);
    return RS_OK;
}

extern "C" int rs_tile_temporal(rs_context* c) {
    if (!c || !c->active) return fail(c, RS_E_INVALID, "rs_tile_temporal: no frame in flight");
    HIPCHK(c, enter(c));
    if (c->P.do_temporal && c->frames > 0 && !c->temporal_ran) {
        const DevScene S = c->scene->dev();
        const dim3 gb = grid_rows(c->W, c->F.y0, c->F.y1);
        // the previous frame's final reservoirs and G-buffer (another lane may still be finishing it)
        if (c->prev_done && c->fs != c->stream) HIPCHK(c, hipStreamWaitEvent(c->fs, c->prev_done, 0));
        const size_t npx = (size_t)c->W * c->H;
        // a tile rebuilds previous-frame G elements beyond its rows with the previous frame's geometry
        DevScene Sp = S;
        const bool partial = c->F.gy0 > 0 || c->F.gy1 < c->H;
        const bool twide = c->twide;
        if (partial && c->geo_prev_scene == c->scene && c->geo_prev != c->scene->geo_gen) {
            if (c->scene->dev_of(c->geo_prev, Sp)) c->prevgeo_read = true;
            else { Sp = S; c->prevgeo_missing++; }     // two updates between frames: the a_* copy moved on
        }
        // the kernel walks S and Sp with one traversal kind: when either lacks its 8-wide tree (a generation
        // held without one), this launch walks both binary trees (same hits, rs_scene.h)
        if (!S.wnodes || !Sp.wnodes) c->twide = false;
        if (c->F.debug_reproj) HIPCHK(c, hipMemsetAsync(c->d_dbg, 0, 2 * npx, c->fs));
        c->F.canon_vis = c->P.do_visibility_pass ? 0 : 1;   // the current reservoir's sample: tested from this pixel
        // the wave-sorted shadow rays (TEMPORAL_SORT) unless RESTIR_SORT_TEMPORAL=off: C3 (per-lane) temporal
        // 1.54 -> 1.36 ms, C5 (lockstep) 0.210 -> 0.191 ms
        const bool tsort = c->sort_temporal != RS_SPLIT_OFF;
#define RS_TEMPORAL_ARGS S, Sp, c->F, c->G[c->gcur], c->G[c->gprev], ResBuf{c->R[c->rcur]}, ResBuf{c->R[c->last]}, \
                         ResBuf{c->R[c->rb]}, count_slot(c, gb)
        if (partial && tsort) LAUNCH_TRAV_X(c, TEMPORAL_BAND | TEMPORAL_SORT, k_temporal, gb, RS_TEMPORAL_ARGS);
        else if (partial) LAUNCH_TRAV_X(c, TEMPORAL_BAND, k_temporal, gb, RS_TEMPORAL_ARGS);
        else if (tsort) LAUNCH_TRAV_X(c, TEMPORAL_SORT, k_temporal, gb, RS_TEMPORAL_ARGS);
        else LAUNCH_TRAV(c, k_temporal, gb, RS_TEMPORAL_ARGS);
#undef RS_TEMPORAL_ARGS
        c->twide = twide;
        HIPCHK(c, hipGetLastError());
        if (c->F.debug_reproj) {
            k_debug_reproj<<<(unsigned)((npx + 255) / 256), 256, 0, c->fs>>>(c->G[c->gcur], c->d_dbg, (uint32_t)npx);
            HIPCHK(c, hipGetLastError());
        }
        c->rcur = c->rb;
        c->temporal_ran = true;
    }
    if (!c->ev_temporal) {
        HIPCHK(c, hipEventRecord(c->ev[EV_TEMPORAL], c->fs));
        c->ev_temporal = true;
    }
    return RS_OK;
}

extern "C" int rs_tile_spatial(rs_context* c, int pass_index) {
    if (!c || !c->active) return fail(c, RS_E_INVALID, "rs_tile_spatial: no frame in flight");
    if (!(c->P.do_spatial && pass_index >= 0 && pass_index < c->P.spatial_passes)) return RS_OK;
    HIPCHK(c, enter(c));
    if (c->P.do_temporal && c->frames > 0 && !c->temporal_ran) {
        int rc = rs_tile_temporal(c);
        if (rc) return rc;
    }
    if (!c->ev_temporal) {
        HIPCHK(c, hipEventRecord(c->ev[EV_TEMPORAL], c->fs));
        c->ev_temporal = true;
    }
    const DevScene S = c->scene->dev();
    int dst = (c->rcur == c->ra) ? c->rb : c->ra;
    int fuse = (pass_index == c->P.spatial_passes - 1) ? 1 : 0;
    // the canonical reservoir's sample was visibility-tested from this very pixel (same origin, target, tnear and
    // tfar: the same ray) when it was selected -- by the initial pass, the temporal pass (p-hat at the current
    // surface) or the previous spatial pass -- except after a visibility pass, which keeps occluded samples with
    // W = 0 (pg/ReSTIRIntegrator.cpp:302-312); the temporal pass passes such a reservoir through on a failed
    // reprojection, so with the visibility pass only passes >= 1 know it
    c->F.canon_vis = (!c->P.do_visibility_pass || pass_index > 0) ? 1 : 0;
    const dim3 gb = grid_rows(c->W, c->F.y0, c->F.y1);
    {
        const CountSlot cs = count_slot(c, gb);
        const GBuf& G = c->G[c->gcur];
        const ResBuf Rr{c->R[c->rcur]}, Rw{c->R[dst]};
        const bool cm = c->F.mis == MIS_CONSTANT;
        const bool tev = c->tuning && c->tune_n + 2 <= (int)(sizeof(c->tune_ev) / sizeof(c->tune_ev[0]));
        if (tev) HIPCHK(c, hipEventRecord(c->tune_ev[c->tune_n], c->fs));
#define SPATIAL(TK, CM, SM) k_spatial<TK, CM, SM><<<gb, 256, 0, c->fs>>>(S, c->F, G, Rr, Rw, pass_index, fuse, c->fb, cs)
        const bool ssort = c->sort_spatial == RS_SPLIT_ON || (c->sort_spatial == RS_SPLIT_AUTO && c->trav == TRAV_LANE);
        if (ssort && cm && c->F.k + 1 <= kSpatialSortMax) {
            LAUNCH_TRAV(c, k_spatial_sorted, gb, S, c->F, G, Rr, Rw, pass_index, fuse, c->fb, cs);
        } else if (c->trav == TRAV_LANE) {
            if (c->twide) { if (cm) SPATIAL(TRAV_LANE | TRAV_WIDE, 1, 0); else SPATIAL(TRAV_LANE | TRAV_WIDE, 0, 0); }
            else { if (cm) SPATIAL(TRAV_LANE, 1, 0); else SPATIAL(TRAV_LANE, 0, 0); }
        } else if (grid_waves(gb) < (size_t)2 * c->wave_slots) {   // a small launch: RS_SPATIAL_WAVES_SMALL budget
            if (c->twide) { if (cm) SPATIAL(TRAV_WIDE, 1, 1); else SPATIAL(TRAV_WIDE, 0, 1); }
            else { if (cm) SPATIAL(TRAV_LOCKSTEP, 1, 1); else SPATIAL(TRAV_LOCKSTEP, 0, 1); }
        } else {
            if (c->twide) { if (cm) SPATIAL(TRAV_WIDE, 1, 0); else SPATIAL(TRAV_WIDE, 0, 0); }
            else { if (cm) SPATIAL(TRAV_LOCKSTEP, 1, 0); else SPATIAL(TRAV_LOCKSTEP, 0, 0); }
        }
#undef SPATIAL
        if (tev) {
            HIPCHK(c, hipEventRecord(c->tune_ev[c->tune_n + 1], c->fs));
            c->tune_n += 2;
        }
    }
    HIPCHK(c, hipGetLastError());
    c->rcur = dst;
    if (fuse) c->shade_fused = true;
    c->spatial_ran = true;
    HIPCHK(c, hipEventRecord(c->ev[EV_SPATIAL], c->fs));
    return RS_OK;
}

extern "C" int rs_tile_finish(rs_context* c, const float** band_rgb, rs_pass_times* t) {
    if (!c || !c->active) return fail(c, RS_E_INVALID, "rs_tile_finish: no frame in flight");
    HIPCHK(c, enter(c));
    if (c->P.do_temporal && c->frames > 0 && !c->temporal_ran) {
        int rc = rs_tile_temporal(c);
        if (rc) return rc;
    }
    if (!c->ev_temporal) {
        HIPCHK(c, hipEventRecord(c->ev[EV_TEMPORAL], c->fs));
        c->ev_temporal = true;
    }
    if (!c->spatial_ran) HIPCHK(c, hipEventRecord(c->ev[EV_SPATIAL], c->fs));
    if (!c->shade_fused) {
        const DevScene S = c->scene->dev();
        const dim3 gb = grid_rows(c->W, c->F.y0, c->F.y1);
        LAUNCH_TRAV(c, k_shade, gb, S, c->F, c->G[c->gcur], ResBuf{c->R[c->rcur]}, c->fb, count_slot(c, gb));
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(c->ev[EV_SHADE], c->fs));
    c->ev_pending[c->slot] = true;
    k_reduce_counts<<<kReduceBlocks, kReduceThreads, 0, c->fs>>>(c->d_part, c->part_used, c->d_red,
                                                                 (unsigned*)(c->d_red + kReduceBlocks), c->d_cnt, c->d_tot);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->ev[EV_DONE], c->fs));
    c->last_done = c->ev[EV_DONE];
    c->lane_scene[c->li] = c->frame_scene; c->lane_gen[c->li] = c->frame_gen; c->lane_done[c->li] = c->ev[EV_DONE];
    c->lane_prevgeo[c->li] = c->prevgeo_read;
    c->geo_last = c->frame_scene ? c->frame_scene->geo_gen : 0; c->geo_last_scene = c->frame_scene;
    if (c->fs == c->stream && c->ahead > 0) c->lane_wait[c->li] = c->ev[EV_DONE];
    if (c->fs != c->stream) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev[EV_DONE], 0));   // sequential semantics
    record_traversal_time(c);
    c->r_last = c->rcur;   // reservoirsLastFrame = final buffer (pointer swap, :477)
    c->frames++;
    c->active = false;
    if (band_rgb) *band_rgb = c->fb + 3 * (size_t)c->F.y0 * c->W;
    if (t) {
        HIPCHK(c, hipMemcpyAsync(c->h_cnt, c->d_cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->fs));
        HIPCHK(c, hipStreamSynchronize(c->fs));
        float a = 0, b = 0, d = 0, e = 0, f = 0, tot = 0;
        hipEventElapsedTime(&a, c->ev[EV_BEGIN], c->ev[EV_INIT]);
        hipEventElapsedTime(&b, c->ev[EV_INIT], c->ev[EV_VIS]);
        hipEventElapsedTime(&d, c->ev[EV_VIS], c->ev[EV_TEMPORAL]);
        hipEventElapsedTime(&e, c->ev[EV_TEMPORAL], c->ev[EV_SPATIAL]);
        hipEventElapsedTime(&f, c->ev[EV_SPATIAL], c->ev[EV_SHADE]);
        hipEventElapsedTime(&tot, c->ev[EV_BEGIN], c->ev[EV_SHADE]);
        t->gbuffer_initial_ms = a; t->visibility_ms = b; t->temporal_ms = d; t->spatial_ms = e; t->shade_ms = f;
        t->total_ms = tot; t->rays = c->h_cnt->rays; t->primary_rays = c->h_cnt->primary;
        t->reproj_outside = c->h_cnt->reproj_outside;
        fold_slot(c, c->slot);
    }
    return RS_OK;
}

extern "C" int rs_get_timing_totals(rs_context* c, rs_pass_times* sum, uint32_t* n_frames, int reset) {
    if (!c || !sum) return fail(c, RS_E_INVALID, "rs_get_timing_totals: null argument");
    if (c->active) return fail(c, RS_E_INVALID, "rs_get_timing_totals: a frame is in flight");
    HIPCHK(c, enter(c));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int s = 0; s < rs_context::kEvRing; ++s) fold_slot(c, s);
    Counters tot{};
    HIPCHK(c, hipMemcpy(&tot, c->d_tot, sizeof(Counters), hipMemcpyDeviceToHost));
    sum->gbuffer_initial_ms = (float)c->tot_ms[0]; sum->visibility_ms = (float)c->tot_ms[1];
    sum->temporal_ms = (float)c->tot_ms[2]; sum->spatial_ms = (float)c->tot_ms[3];
    sum->shade_ms = (float)c->tot_ms[4]; sum->total_ms = (float)c->tot_ms[5];
    sum->rays = tot.rays; sum->primary_rays = tot.primary; sum->reproj_outside = tot.reproj_outside;
    if (n_frames) *n_frames = (uint32_t)c->tot_frames;
    if (reset) {
        for (double& v : c->tot_ms) v = 0.0;
        c->tot_frames = 0;
        HIPCHK(c, hipMemset(c->d_tot, 0, sizeof(Counters)));
    }
    return RS_OK;
}

extern "C" int rs_render_frame(rs_context* c, const rs_scene* s, const rs_camera* cam, const rs_frame_params* P,
                               uint32_t frame_index, float* frame_rgb_host, rs_pass_times* times) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_render_frame: null context");
    rs_tile_desc full{0, c->H, 0, 0};
    int rc = rs_tile_begin(c, s, cam, P, frame_index, &full);
    if (rc) return rc;
    if ((rc = rs_tile_temporal(c))) return rc;
    if (P->do_spatial)
        for (int i = 0; i < P->spatial_passes; ++i)
            if ((rc = rs_tile_spatial(c, i))) return rc;
    if ((rc = rs_tile_finish(c, nullptr, times))) return rc;
    if (frame_rgb_host) {
        HIPCHK(c, hipMemcpyAsync(frame_rgb_host, c->fb, (size_t)c->W * c->H * 3 * sizeof(float), hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return RS_OK;
}

// MIS direct-light ground truth (rs_mis.h) into the framebuffer: one launch, spp
// samples per pixel.  Does not touch the ReSTIR history (G-buffers, reservoirs, frame counter).
extern "C" int rs_render_direct_mis(rs_context* c, const rs_scene* s, const rs_camera* cam, const rs_frame_params* P,
                                    uint32_t frame_index, uint32_t spp, float* frame_rgb_host, rs_pass_times* t) {
    if (!c || !s || !cam || !P) return fail(c, RS_E_INVALID, "rs_render_direct_mis: null argument");
    if (s->ctx != c) return fail(c, RS_E_INVALID, "rs_render_direct_mis: scene belongs to another context");
    if (c->active) return fail(c, RS_E_INVALID, "rs_render_direct_mis: a tile frame is in flight");
    if (P->use_skybox && s->sky < 0)
        return fail(c, RS_E_UNSUPPORTED, "use_skybox: the scene has no sky map (rs_scene_set_sky / rs_scene_load_sky)");
    if (spp < 1 || spp > 65536) return fail(c, RS_E_INVALID, "rs_render_direct_mis: spp must be in [1, 65536]");
    HIPCHK(c, enter(c));
    FrameConst F = {};
    F.bg = vec3{P->bg_color[0], P->bg_color[1], P->bg_color[2]};
    F.tnear_off = P->tnear_offset; F.tfar_off = P->tfar_offset; F.normal_off = P->normal_offset;
    F.use_sky = P->use_skybox ? 1 : 0;
    F.seed = P->seed; F.frame = frame_index;
    F.W = c->W; F.H = c->H; F.y0 = 0; F.y1 = c->H; F.gy0 = 0; F.gy1 = c->H;
    GCam gc;
    make_camera(cam, c->H, gc, F.inv_view);
    F.cam = gc; F.camp = gc;
    const DevScene S = s->dev();
    const dim3 g = grid_rows(c->W, 0, c->H);
    c->fs = c->stream; c->li = 0;                 // the context's stream (after every frame enqueued so far)
    c->d_cnt = c->cnts[0]; c->d_red = c->reds[0];
    sync_all(c);                                  // lane 0's slots may still be in use
    c->fb = c->fbs[0];
    if (c->fb_read[0]) { HIPCHK(c, hipEventSynchronize(c->fb_read[0])); c->fb_read[0] = nullptr; }
    if (!use_parts(c, 0, grid_waves(g))) return fail(c, RS_E_HIP, "hipMalloc(count slots) failed");
    c->join_next = true;
    HIPCHK(c, hipMemsetAsync(c->d_cnt, 0, sizeof(Counters), c->stream));
    hipEvent_t e0 = c->ev_gt[0], e1 = c->ev_gt[1];
    HIPCHK(c, hipEventRecord(e0, c->stream));
    pick_traversal(c, s);
    c->twide = s->wide_on;
    c->tuning = false;               // the ReSTIR frames own the per-scene traversal tuning
    LAUNCH_TRAV(c, k_direct_mis, g, S, F, (int)spp, c->fb, count_slot(c, g));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(e1, c->stream));
    k_reduce_counts<<<kReduceBlocks, kReduceThreads, 0, c->stream>>>(c->d_part, c->part_used, c->d_red,
                                                                     (unsigned*)(c->d_red + kReduceBlocks), c->d_cnt, c->d_tot);
    HIPCHK(c, hipGetLastError());
    if (t || frame_rgb_host) {
        if (frame_rgb_host)
            HIPCHK(c, hipMemcpyAsync(frame_rgb_host, c->fb, (size_t)c->W * c->H * 3 * sizeof(float), hipMemcpyDeviceToHost,
                                     c->stream));
        HIPCHK(c, hipMemcpyAsync(c->h_cnt, c->d_cnt, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (t) {
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            *t = rs_pass_times{};
            t->shade_ms = ms; t->total_ms = ms;
            t->rays = c->h_cnt->rays; t->primary_rays = c->h_cnt->primary;
        }
    }
    return RS_OK;
}

extern "C" int rs_get_frame_device_ptr(rs_context* c, const float** dptr) {
    if (!c || !dptr) return fail(c, RS_E_INVALID, "rs_get_frame_device_ptr: null argument");
    *dptr = c->fb;
    return RS_OK;
}

// Readback of the framebuffer into page-locked host memory.  Alone, a copy kernel's stores over the host
// link move a 1080p frame (24.9 MB) in 0.46 ms (54 GB/s) against the DMA engine's 0.84 ms (30 GB/s)
// (scripts/host_link_bw.hip); beside the frames in flight the kernel competes with them for CUs and the
// DMA engine wins: C2 1080p drop-in 652 vs 533 frames/s at pipeline depth 2 (scripts/dropin_ab.sh).
// So the DMA engine is the default, the kernel an option (RESTIR_READBACK=kernel).
typedef float rb_v4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_readback(const rb_v4* __restrict__ src, rb_v4* dst, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(src[i], dst + i);
}

extern "C" int rs_frame_readback(rs_context* c, float* dst, uint64_t* ticket) {
    if (!c || !dst || !ticket) return fail(c, RS_E_INVALID, "rs_frame_readback: null argument");
    if (c->active) return fail(c, RS_E_INVALID, "rs_frame_readback: a tile frame is in flight");
    HIPCHK(c, enter(c));
    if (!c->rb_ev[0])
        for (int i = 0; i < rs_context::kRb; ++i) HIPCHK(c, hipEventCreateWithFlags(&c->rb_ev[i], hipEventDisableTiming));
    const uint64_t t = ++c->rb_seq;
    const int k = (int)(t % rs_context::kRb);
    if (c->rb_busy[k]) HIPCHK(c, hipEventSynchronize(c->rb_ev[k]));   // the slot's ticket kRb ago
    const size_t bytes = (size_t)c->W * c->H * 3 * sizeof(float);
    // DMA engine (hipMemcpyAsync; pageable memory is staged by the runtime), or with RESTIR_READBACK=kernel
    // and a page-locked, 16-B aligned destination a copy kernel.  Both on the
    // context's stream, which is ordered after every frame enqueued so far (rs_tile_finish) and runs nothing
    // else while frames run on their lanes: a fifth stream would share one of the process's 4 hardware
    // queues with a lane and serialise the copy with that lane's next frame.
    hipPointerAttribute_t at{};
    void* ddst = nullptr;
    const bool kernel_ok = c->readback_kernel && bytes % 16 == 0 && ((uintptr_t)dst & 15) == 0 &&
                           hipPointerGetAttributes(&at, dst) == hipSuccess && at.type == hipMemoryTypeHost &&
                           hipHostGetDevicePointer(&ddst, dst, 0) == hipSuccess && ddst != nullptr;
    (void)hipGetLastError();                   // a pageable pointer leaves an error in the per-thread slot
    if (kernel_ok) {
        k_readback<<<256, 256, 0, c->stream>>>((const rb_v4*)c->fb, (rb_v4*)ddst, bytes / 16);
        HIPCHK(c, hipGetLastError());
    } else {
        HIPCHK(c, hipMemcpyAsync(dst, c->fb, bytes, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->rb_ev[k], c->stream));
    c->rb_busy[k] = true;
    c->fb_read[c->li] = c->rb_ev[k];
    *ticket = t;
    return RS_OK;
}

extern "C" int rs_frame_wait(rs_context* c, uint64_t t) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_frame_wait: null context");
    if (t == 0 || t > c->rb_seq) return fail(c, RS_E_INVALID, "rs_frame_wait: unknown ticket");
    if (c->rb_seq - t >= (uint64_t)rs_context::kRb) return RS_OK;    // its slot was reused: waited for then
    HIPCHK(c, enter(c));
    HIPCHK(c, hipEventSynchronize(c->rb_ev[t % rs_context::kRb]));
    return RS_OK;
}

extern "C" int rs_host_alloc(rs_context* c, size_t bytes, void** out) {
    if (!c || !out || bytes == 0) return fail(c, RS_E_INVALID, "rs_host_alloc: bad argument");
    HIPCHK(c, enter(c));
    HIPCHK(c, hipHostMalloc(out, bytes, hipHostMallocDefault));
    return RS_OK;
}
extern "C" void rs_host_free(void* p) {
    if (p) hipHostFree(p);
}

extern "C" int rs_reset_history(rs_context* c) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_reset_history: null context");
    c->frames = 0;
    return RS_OK;
}

extern "C" int rs_synchronize(rs_context* c) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_synchronize: null context");
    HIPCHK(c, enter(c));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RS_OK;
}

extern "C" int rs_dump_gbuffer(rs_context* c, int prev, float* out) {
    if (!c || !out) return fail(c, RS_E_INVALID, "rs_dump_gbuffer: null argument");
    HIPCHK(c, enter(c));
    size_t n = (size_t)c->W * c->H;
    const GBuf& g = c->G[prev ? c->gprev : c->gcur];
    std::vector<float4> a(n), b(n), d(n), e(n), f(n);
    HIPCHK(c, hipMemcpyAsync(a.data(), g.g0, n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(b.data(), g.g1, n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(d.data(), g.g2, n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(e.data(), g.g3, n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(f.data(), g.g4, n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (size_t p = 0; p < n; ++p) {
        float* o = out + 19 * p;
        int type; std::memcpy(&type, &e[p].w, 4);
        o[0] = a[p].x; o[1] = a[p].y; o[2] = a[p].z; o[3] = b[p].x; o[4] = b[p].y; o[5] = b[p].z;
        o[6] = d[p].x; o[7] = d[p].y; o[8] = d[p].z; o[9] = e[p].x; o[10] = e[p].y; o[11] = e[p].z;
        o[12] = f[p].x; o[13] = f[p].y; o[14] = f[p].z; o[15] = b[p].w; o[16] = a[p].w; o[17] = (float)type;
        o[18] = d[p].w;
    }
    return RS_OK;
}

extern "C" int rs_dump_reservoirs(rs_context* c, float* out) {
    if (!c || !out) return fail(c, RS_E_INVALID, "rs_dump_reservoirs: null argument");
    HIPCHK(c, enter(c));
    size_t n = (size_t)c->W * c->H;
    std::vector<float4> r(3 * n);
    HIPCHK(c, hipMemcpyAsync(r.data(), c->R[c->r_last], 3 * n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (size_t p = 0; p < n; ++p) {
        float* o = out + 12 * p;
        const float4 &a = r[3 * p], &b = r[3 * p + 1], &d = r[3 * p + 2];
        int conf; std::memcpy(&conf, &d.w, 4);
        o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = b.x; o[4] = b.y; o[5] = b.z;
        o[6] = d.x; o[7] = d.y; o[8] = d.z; o[9] = a.w; o[10] = b.w; o[11] = (float)conf;
    }
    return RS_OK;
}

// --------------------------------------------------------------------------- post-frame (§8f-1)
extern "C" int rs_post_frame(rs_context* c, const rs_post_params* pp, const float** display_rgba_dptr,
                             rs_post_stats* stats) {
    if (!c || !pp) return fail(c, RS_E_INVALID, "rs_post_frame: null argument");
    if (c->active) return fail(c, RS_E_INVALID, "rs_post_frame: a frame is in flight (finish it first)");
    HIPCHK(c, enter(c));
    const size_t npx = (size_t)c->W * c->H;
    const int nblk_max = (int)((npx + 255) / 256);
    if (!c->acc) {
        HIPCHK(c, hipMalloc(&c->acc, npx * 3 * sizeof(float)));
        HIPCHK(c, hipMemsetAsync(c->acc, 0, npx * 3 * sizeof(float), c->stream));   // zeroed accumulator
        HIPCHK(c, hipMalloc(&c->display, npx * sizeof(float4)));
        HIPCHK(c, hipMemsetAsync(c->display, 0, npx * sizeof(float4), c->stream));
        HIPCHK(c, hipMalloc(&c->post_part, (size_t)nblk_max * sizeof(double2)));
        HIPCHK(c, hipMalloc(&c->post_out, sizeof(double2)));
    }
    // rows of the last rendered frame / band (rs_render_frame: all rows)
    const int y0 = c->frames ? c->F.y0 : 0, y1 = c->frames ? c->F.y1 : c->H;
    // a denoised display is validated before the accumulator blends this frame (a rejected call leaves the
    // accumulator and accFrameCtr as they were)
    if (pp->denoise && !c->denoiser) return fail(c, RS_E_INVALID, "rs_post_frame: denoise without a denoiser (rs_context_set_denoiser)");
    if (pp->denoise && (y0 != 0 || y1 != c->H)) return fail(c, RS_E_UNSUPPORTED, "rs_post_frame: denoise needs a full frame, not a tile band");
    PostConst P{c->W, y0, y1, 1.0f / (float)(c->acc_frames + 1), pp->tonemap ? 1 : 0, pp->gamma_correct ? 1 : 0};
    const size_t n = (size_t)(y1 - y0) * c->W;
    const int nblk = (int)((n + 255) / 256);
    if (nblk > 0) {
        k_post<<<nblk, 256, 0, c->stream>>>(c->fb, c->acc, c->display, P, c->post_part);
        HIPCHK(c, hipGetLastError());
        k_post_reduce<<<1, 256, 0, c->stream>>>(c->post_part, nblk, c->post_out);
        HIPCHK(c, hipGetLastError());
    }
    c->post_px = nblk > 0 ? n : 0;
    // accFrameCtr bookkeeping (pg/simpleguidx11.cpp:297-306): the frame is in the accumulator now, whatever
    // the denoise step below returns
    const uint32_t used = c->acc_frames;
    c->acc_frames++;
    const uint32_t max_acc = pp->max_acc_frames > 0 ? (uint32_t)pp->max_acc_frames : 300000u;
    const bool accumulate = pp->accumulate && c->acc_frames <= max_acc;
    if (!accumulate) c->acc_frames = 0;
    if (pp->denoise) {   // oidnFilter.execute on the accumulator, display = the denoised image (:255-280)
        const float* den = nullptr;
        const int rc = rs_denoise_frame(c, c->denoiser, nullptr, &den);
        if (rc != RS_OK) return rc;
        k_post_display<<<nblk, 256, 0, c->stream>>>(den, c->display, P);
        HIPCHK(c, hipGetLastError());
    }
    if (display_rgba_dptr) *display_rgba_dptr = (const float*)c->display;
    if (stats) {
        double2 h{0.0, 0.0};
        if (nblk > 0) HIPCHK(c, hipMemcpyAsync(&h, c->post_out, sizeof(double2), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        stats->sum = h.x; stats->sqr_sum = h.y; stats->pixels = n;
        stats->mean = n ? h.x / (double)n : 0.0;
        const double sqr_mean = n ? h.y / (double)n : 0.0;
        stats->variance = sqr_mean - stats->mean * stats->mean;     // D(X) = E(X^2) - E(X)^2 (:324-325)
        stats->acc_frames_used = used;
    }
    return RS_OK;
}

// glm::to_string(vec3): "vec3(x, y, z)" with %f
static std::string glm_vec3(const float* v) {
    char b[160];
    std::snprintf(b, sizeof b, "vec3(%f, %f, %f)", v[0], v[1], v[2]);
    return b;
}
extern "C" int rs_export_png(rs_context* c, const char* path, const rs_export_params* ep) {
    if (!c || !path) return fail(c, RS_E_INVALID, "rs_export_png: null argument");
    if (!c->display) return fail(c, RS_E_INVALID, "rs_export_png: no display buffer (call rs_post_frame first)");
    HIPCHK(c, enter(c));
    const size_t npx = (size_t)c->W * c->H;
    std::vector<float4> disp(npx);
    double2 st{0.0, 0.0};
    HIPCHK(c, hipMemcpyAsync(disp.data(), c->display, npx * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    if (c->post_px) HIPCHK(c, hipMemcpyAsync(&st, c->post_out, sizeof(double2), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<uint8_t> px(npx * 4);
    for (size_t i = 0; i < npx; ++i) {          // glm::vec<4,uint8_t>(display_data[i] * 255.0f), :617-619
        const float v[4] = {disp[i].x, disp[i].y, disp[i].z, disp[i].w};
        for (int k = 0; k < 4; ++k) {
            const float f = v[k] * 255.0f;
            px[4 * i + k] = (f > 0.0f) ? (uint8_t)(f < 255.0f ? f : 255.0f) : (uint8_t)0;   // out-of-range: clamp
        }
    }
    std::string err;
    if (write_png(path, c->W, c->H, 4, px.data(), err) != 0) return fail(c, RS_E_IO, "rs_export_png: " + err);
    if (ep && ep->write_sidecar) {              // :628-650
        const double n = (double)c->post_px;
        const double mean = n > 0 ? st.x / n : 0.0, var = n > 0 ? st.y / n - mean * mean : 0.0;
        std::FILE* f = std::fopen((std::string(path) + ".txt").c_str(), "w");
        if (!f) return fail(c, RS_E_IO, std::string("rs_export_png: cannot write ") + path + ".txt");
        const rs_frame_params& P = c->P;
        std::ostringstream o;
        o << "Image name: " << path << "\n\n";
        o << "Iteration count: " << c->acc_frames << "\n";
        o << "Area samples: " << P.m_area << "\n";
        o << "BRDF samples: " << P.m_brdf << "\n\n";
        o << "Spatial reuse: " << (P.do_spatial ? "True" : "False") << "\n";
        o << "\tPass count: " << P.spatial_passes << "\n";
        o << "\tNeighbor count: " << P.spatial_neighbors << "\n";
        o << "\tReuse radius: " << P.spatial_radius << "\n\n";
        o << "Temporal reuse: " << (P.do_temporal ? "True" : "False") << "\n\n";
        o << "Render time: " << (ep ? ep->render_time_s : 0.0f) << " s" << "\n";
        o << "Image mean: " << mean << "\n";
        o << "Image variance: " << var << "\n\n";
        o << "Camera position: " << glm_vec3(c->cam_last.eye) << "\n";
        o << "Camera view at: " << glm_vec3(c->cam_last.at) << "\n";
        o << "Camera vertical FOV: " << c->cam_last.fov_y_deg << std::endl;
        const std::string t = o.str();
        const bool ok = std::fwrite(t.data(), 1, t.size(), f) == t.size();
        std::fclose(f);
        if (!ok) return fail(c, RS_E_IO, "rs_export_png: sidecar write failed");
    }
    return RS_OK;
}
extern "C" int rs_image_encode_png(const char* path, uint32_t w, uint32_t h, uint32_t ch, const uint8_t* px) {
    if (!path || !px || !w || !h || ch < 1 || ch > 4) return fail(nullptr, RS_E_INVALID, "rs_image_encode_png: bad arguments");
    std::string err;
    if (write_png(path, (int)w, (int)h, (int)ch, px, err) != 0) return fail(nullptr, RS_E_IO, err);
    return RS_OK;
}

// --------------------------------------------------------------------------- denoiser (§8f-4)
extern "C" int rs_denoise_frame(rs_context* c, rs_denoiser* d, const rs_denoise_params* p, const float** out) {
    if (!c || !d || !out) return fail(c, RS_E_INVALID, "rs_denoise_frame: null argument");
    if (rs::denoiser_ctx(d) != c) return fail(c, RS_E_INVALID, "rs_denoise_frame: the denoiser belongs to another context");
    if (c->active) return fail(c, RS_E_INVALID, "rs_denoise_frame: a frame is in flight (finish it first)");
    if (!c->acc || !c->frames) return fail(c, RS_E_INVALID, "rs_denoise_frame: no accumulator yet (render a frame and call rs_post_frame)");
    if (p && !p->hdr) return fail(c, RS_E_UNSUPPORTED, "rs_denoise_frame: only hdr = true (the reference's setting) is supported");
    HIPCHK(c, enter(c));
    float* o = rs::denoiser_frame_out(d, c->W, c->H);
    if (!o) return fail(c, RS_E_HIP, "rs_denoise_frame: output allocation failed");
    const GBuf& g = c->G[c->gcur];   // the last frame's G-buffer: albedo = kd (g2.xyz), normal = g1.xyz
    const int rc = rs::denoise_run(d, c->stream, c->acc, 3, (const float*)g.g2, 4, (const float*)g.g1, 4, o, 3,
                                   c->H, c->W, p ? p->input_scale : NAN);
    if (rc != RS_OK) return rc;
    *out = o;
    return RS_OK;
}
extern "C" int rs_context_set_denoiser(rs_context* c, rs_denoiser* d) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_context_set_denoiser: null context");
    if (d && rs::denoiser_ctx(d) != c) return fail(c, RS_E_INVALID, "rs_context_set_denoiser: the denoiser belongs to another context");
    c->denoiser = d;
    return RS_OK;
}

extern "C" int rs_post_reset(rs_context* c) {
    if (!c) return fail(nullptr, RS_E_INVALID, "rs_post_reset: null context");
    c->acc_frames = 0;
    return RS_OK;
}

// --------------------------------------------------------------------------- test hook
__global__ void k_debug_trace(DevScene S, uint32_t n, const float* o, const float* d, const float* tn, const float* tf,
                              int any, float* t_out, int32_t* prim_out) {
    // mode (`any`): 0 closest / 1 any-hit with the lockstep wave traversal the passes use,
    //               2 closest / 3 any-hit with the per-lane traversal
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = i0 < n;
    const uint32_t i = act ? i0 : n - 1;
    vec3 O = mk(o[3 * i], o[3 * i + 1], o[3 * i + 2]), D = mk(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
    if (any >= 6 && any <= 10 && S.n_wnodes == 0u) {   // the 8-wide modes need the scene's wide tree
        if (act) { prim_out[i] = -1; t_out[i] = -1.0f; }
        return;
    }
    if (any >= 8 && any <= 10) {  // timing probes of the 8-wide walk: 8 closest walk with the ray's tfar,
        const vec3 inv = mk(1.0f / D.x, 1.0f / D.y, 1.0f / D.z);   // 9 any-hit without triangle tests,
        Hit h; h.t = tf[i]; h.u = h.v = 0.0f; h.prim = -1;        // 10 any-hit with statistics off
        uint32_t occ = 0u, lost = 0u;
        if (any == 8) wide_walk<false>(S, act, O, D, inv, tn[i], tf[i], h, occ, lost);
        else if (any == 9) wide_walk<true, false, true>(S, act, O, D, inv, tn[i], tf[i], h, occ, lost);
        else wide_walk<true>(S, act, O, D, inv, tn[i], tf[i], h, occ, lost);
        if (act) { prim_out[i] = any == 8 ? h.prim : (int32_t)occ; t_out[i] = (float)lost; }
    } else if (any == 6 || any == 7) {   // 8-wide walk statistics: node fetches << 16 | triangle tests; t = stack overflow
        const vec3 inv = mk(1.0f / D.x, 1.0f / D.y, 1.0f / D.z);
        Hit h; h.t = tf[i]; h.u = h.v = 0.0f; h.prim = -1;
        uint32_t occ = 0u, lost = 0u, st = 0u;
        if (any == 7) wide_walk<true, true>(S, act, O, D, inv, tn[i], tf[i], h, occ, lost, &st);
        else wide_walk<false, true>(S, act, O, D, inv, tn[i], tf[i], h, occ, lost, &st);
        if (act) { prim_out[i] = (int32_t)st; t_out[i] = (float)lost; }
    } else if (any == 4 || any == 5) {   // BVH statistics of the per-lane walk: visits << 16 | triangle tests
        vec3 inv = mk(1.0f / D.x, 1.0f / D.y, 1.0f / D.z);
        uint32_t cur = act ? 0u : 0xffffffffu, visits = 0, tris = 0;
        bool occ = false;
        Hit h; h.t = tf[i]; h.u = h.v = 0; h.prim = -1;
        while (cur < S.n_nodes && !occ) {
            const uint32_t k = cur;
            const float4 a = S.nodes[2 * k], b = S.nodes[2 * k + 1];
            const int leaf = __float_as_int(b.w);
            const float tmax = any == 5 ? tf[i] : h.t;
            ++visits;
            if (any == 4 && leaf >= 0 && box_test(a, b, O, inv, tn[i], tmax)) tris += (leaf & 7) + 1;
            if (any == 5) {
                cur = (uint32_t)__float_as_int(a.w);
                if (box_test(a, b, O, inv, tn[i], tf[i])) {
                    if (leaf < 0) cur = k + 1;
                    else
                        for (int j = 0; j < (leaf & 7) + 1 && !occ; ++j) {
                            const float4* T = S.tris + 3 * ((leaf >> 3) + j);
                            float t, u, v;
                            ++tris;
                            occ = tri_test(T[0], T[1], T[2], O, D, tn[i], tf[i], t, u, v);
                        }
                }
            } else {
                closest_visit<false>(S, a, b, k, O, D, inv, margin_origins(S, O), tn[i], cur, h);
            }
        }
        if (act) { prim_out[i] = (int32_t)((visits << 16) | (tris & 0xffff)); t_out[i] = occ ? 1.0f : 0.0f; }
    } else if (any == 1 || any == 3) {         // per-lane: the scene's walk (8-wide when live)
        bool occ = any == 1 ? trace_any<TRAV_LOCKSTEP>(S, act, O, D, tn[i], tf[i])
                            : (S.n_wnodes ? trace_any<TRAV_LANE | TRAV_WIDE>(S, act, O, D, tn[i], tf[i])
                                          : trace_any<TRAV_LANE>(S, act, O, D, tn[i], tf[i]));
        if (act) { prim_out[i] = occ ? 1 : 0; t_out[i] = 0.0f; }
    } else {
        Hit h = any == 0 ? trace_closest<TRAV_LOCKSTEP>(S, act, O, D, tn[i], tf[i])
                         : (S.n_wnodes ? trace_closest<TRAV_LANE | TRAV_WIDE>(S, act, O, D, tn[i], tf[i])
                                       : trace_closest<TRAV_LANE>(S, act, O, D, tn[i], tf[i]));
        if (act) { prim_out[i] = h.prim; t_out[i] = h.prim >= 0 ? h.t : -1.0f; }
    }
}

extern "C" int rs_debug_trace(rs_context* c, const rs_scene* s, uint32_t n, const float* o, const float* d,
                              const float* tnear, const float* tfar, int any_hit, float* t_out, int32_t* prim_out) {
    if (!c || !s || !o || !d || !tnear || !tfar || !t_out || !prim_out) return fail(c, RS_E_INVALID, "rs_debug_trace: null");
    if (n == 0) return RS_OK;
    HIPCHK(c, enter(c));
    float *dd = nullptr;
    int32_t* dp = nullptr;
    size_t fl = (size_t)n * 9;   // o(3n) d(3n) tn(n) tf(n) t(n)
    HIPCHK(c, hipMalloc(&dd, fl * sizeof(float)));
    HIPCHK(c, hipMalloc(&dp, (size_t)n * sizeof(int32_t)));
    hipMemcpyAsync(dd, o, 3 * (size_t)n * 4, hipMemcpyHostToDevice, c->stream);
    hipMemcpyAsync(dd + 3 * (size_t)n, d, 3 * (size_t)n * 4, hipMemcpyHostToDevice, c->stream);
    hipMemcpyAsync(dd + 6 * (size_t)n, tnear, (size_t)n * 4, hipMemcpyHostToDevice, c->stream);
    hipMemcpyAsync(dd + 7 * (size_t)n, tfar, (size_t)n * 4, hipMemcpyHostToDevice, c->stream);
    if (s->update_recorded) HIPCHK(c, hipStreamWaitEvent(c->stream, s->update_ev, 0));   // a pipelined update
    k_debug_trace<<<(n + 255) / 256, 256, 0, c->stream>>>(s->dev(), n, dd, dd + 3 * (size_t)n, dd + 6 * (size_t)n,
                                                          dd + 7 * (size_t)n, any_hit, dd + 8 * (size_t)n, dp);
    hipError_t e = hipGetLastError();
    hipMemcpyAsync(t_out, dd + 8 * (size_t)n, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(prim_out, dp, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream);
    hipError_t e2 = hipStreamSynchronize(c->stream);
    hipFree(dd); hipFree(dp);
    if (e != hipSuccess || e2 != hipSuccess) return fail(c, RS_E_HIP, "rs_debug_trace: kernel failed");
    return RS_OK;
}

// ---------------------------------------------------------------- internal helpers (rs_internal.h)
namespace rs {
hipStream_t ctx_stream(rs_context* c) { return c->stream; }
int ctx_device(const rs_context* c) { return c->device; }
int ctx_width(const rs_context* c) { return c->W; }
int ctx_height(const rs_context* c) { return c->H; }
int ctx_fail(rs_context* c, int code, const std::string& msg) { return fail(c, code, msg); }
void ctx_track_denoiser(rs_context* c, rs_denoiser* d, bool add) {
    auto& v = c->denoisers;
    v.erase(std::remove(v.begin(), v.end(), d), v.end());
    if (add) v.push_back(d);
    else if (c->denoiser == d) c->denoiser = nullptr;
}
int ctx_join(rs_context* c, hipStream_t st) {
    HIPCHK(c, enter(c));
    if (st == c->stream) return RS_OK;
    if (!c->join_ev) HIPCHK(c, hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->join_ev, st));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->join_ev, 0));   // captured now: the event may be re-recorded
    return RS_OK;
}
}  // namespace rs
