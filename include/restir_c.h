/*
 * restir_c.h -- C ABI of the MI355X-native ReSTIR DI renderer (librestir_amd.so).
 *
 * Drop-in boundary for the reference's per-pixel hot path (Tonz24/restir-embree,
 * pg/ = template/src/pg/pg1_embree/).  The reference's seam is three C++ members of one object
 * (SURVEY.md §8b):
 *   scene-load   Raytracer::LoadScene(file)            pg/raytracer.cpp:34-38
 *                -> Scene::Scene(file, RTCDevice)        pg/Scene.cpp:8-16 (rtcCommitScene = BVH build :15)
 *   render       SimpleGuiDX11::produceRestir(float t) pg/simpleguidx11.cpp:359-487
 *   framebuffer  glm::vec3* frame_data                 pg/simpleguidx11.h:152 (linear HDR RGB f32,
 *                                                       row-major y*W+x, y=0 = top row)
 * and the Embree device lifecycle it wraps (rtcNewDevice/rtcReleaseDevice, pg/simpleguidx11.cpp:48,
 * pg/raytracer.cpp:28-32).  Each entry point below cites the call it replaces.
 *
 * Conventions: plain pointers and sizes only; every function returns 0 on success or a negative
 * RS_E* code; rs_last_error() gives the message.  No exceptions cross the ABI, no global state.
 * A context is bound to one HIP device and one host thread.  Rendering is asynchronous on the
 * context's stream and synchronises only when a host output pointer is given.
 */
#ifndef RESTIR_C_H
#define RESTIR_C_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_OK 0
#define RS_E_INVALID (-1)     /* bad argument / shape */
#define RS_E_HIP (-2)         /* HIP runtime error */
#define RS_E_UNSUPPORTED (-3) /* feature the reference has but this build does not (e.g. JPEG textures) */
#define RS_E_IO (-4)          /* file not found / parse error (scene loader) */

typedef struct rs_context rs_context;
typedef struct rs_scene rs_scene;

/* One mesh = one reference Surface / RTCGeometry (pg/ModelLoader.cpp:232-317): de-indexed triangles
 * (3 unique vertices each, :297-299) with per-vertex normals (vertex attribute slot 0, :280-282). */
typedef struct {
    uint32_t n_tris;
    const float* positions;   /* n_tris * 9 floats: v0.xyz v1.xyz v2.xyz */
    const float* normals;     /* n_tris * 9 floats: n0.xyz n1.xyz n2.xyz */
    uint32_t material;        /* index into the material array (Surface::get_material, :213,243) */
    const float* texcoords;   /* n_tris * 6 floats (uv per vertex; attribute slot 1, :284-285) or NULL = 0 */
    const float* tangents;    /* n_tris * 9 floats (attribute slot 3, :287-289) or NULL = 0; normal maps only */
} rs_mesh_desc;

/* Decoded texture (Texture, pg/Texture.cpp:9-57): top row first, rows tightly packed, channels in
 * R,G,B(,A) order.  Lookups are bilinear (Texture::getTexelBilinear, :170-194): REPEAT for material
 * maps (ModelLoader::TextureProxy, pg/ModelLoader.cpp:28), CLAMP_TO_EDGE for the sky (Texture.h:27). */
#define RS_TEX_U8 0           /* 8-bit LDR (PNG/JPG...): texel = byte / 255 */
#define RS_TEX_F32 1          /* float HDR (.hdr/.exr/.pfm): texel = value; 3 or 4 channels */
typedef struct {
    uint32_t width, height;
    uint32_t channels;        /* 1, 3 or 4 (1-channel 8-bit maps keep the reference's 3-byte read quirk) */
    int32_t format;           /* RS_TEX_U8 or RS_TEX_F32 */
    const void* data;         /* width * height * channels elements */
    int32_t srgb_expand;      /* Texture::expand at load (8-bit; pg/Texture.cpp:141-160): ModelLoader sets it
                                 for map_Kd / map_Ks when Raytracer::gammaCorrect (pg/ModelLoader.cpp:127,135) */
} rs_texture_desc;

/* Material record as the ReSTIR statics read it (pg/material.cpp:105-134, pg/material.h:105-115).
 * Colours are linear (the loader's sRGB expansion, pg/ModelLoader.cpp:80-97, already applied). */
typedef struct {
    float diffuse[3];         /* Kd */
    float specular[3];        /* Ks */
    float emission[3];        /* Ke -- emissive iff Ke.x+Ke.y+Ke.z > 0 (pg/material.h:135-137) */
    float shininess;          /* Ns */
    int32_t type;             /* MaterialType (pg/enums.h:3-11): 1 LAMBERT, 2 PHONG, 4 DIELECTRIC, ... */
    /* texture slots (Material::kDiffuseMapSlot..., pg/material.cpp:105-134; Intersection.h:26-39):
       1-based index into the textures passed to rs_scene_create_textured, 0 = none */
    int32_t diffuse_map, specular_map, shininess_map, normal_map;
} rs_material_desc;

/* Camera(width, height, fov_y, view_from, view_at), Z-up (pg/camera.cpp:12-18, pg/camera.h:68). */
typedef struct {
    float eye[3];
    float at[3];
    float fov_y_deg;
} rs_camera;

/* POD snapshot of ReSTIRIntegrator's static knobs (pg/ReSTIRIntegrator.cpp:13-35) and of its private
 * RenderParams (pg/RenderParams.h:5-17), passed by value per frame. */
typedef struct {
    int32_t m_area;                /* M_Area */
    int32_t m_brdf;                /* M_Brdf */
    int32_t spatial_neighbors;     /* spatialReuseNeighborCount (k) */
    int32_t spatial_passes;        /* spatialPassCount (P) */
    int32_t confidence_cap;        /* confidenceCap */
    float spatial_radius;          /* spatialReuseRadius (R) */
    float min_normal_similarity;
    float max_depth_difference;
    int32_t do_spatial;
    int32_t do_temporal;
    int32_t do_visibility_pass;
    int32_t reject_dissimilar;
    int32_t spatial_mis;           /* SpatialWeightCalculation: 0 CONSTANT, 1 DEBIAS_CONTRIB,
                                      2 DEBIAS_Z_TERM, 3 BALANCE_HEURISTIC, 4 PAIRWISE_MIS */
    int32_t use_skybox;            /* primary misses read the scene's sky (rs_scene_set_sky); else bg_color */
    float bg_color[3];
    float tnear_offset;
    float tfar_offset;
    float normal_offset;
    uint32_t seed;                 /* counter-RNG seed (replaces Utils' mt19937{123}, pg/utils.cpp:175) */
    int32_t debug_reprojection;    /* debugReprojection (pg/ReSTIRIntegrator.cpp:30, :647-689): the temporal pass
                                      paints rejected reprojections into the G-buffer emission -- (100,100,0)
                                      no backward reprojection, (0,100,0) depth ratio, (100,0,100) no forward
                                      reprojection at the pixel, (0,0,100) at the forward-reprojected pixel of
                                      a failed forward depth check.  Applied after the pass (the reference's
                                      parallel loop races on them); full frames only (RS_E_UNSUPPORTED on a
                                      partial tile) */
} rs_frame_params;

/* Per-pass device time in ms (the reference's std::chrono pass timers, pg/simpleguidx11.h:120-127). */
typedef struct {
    float gbuffer_initial_ms;      /* gBUfferFillDuration + initialCandidatesGenDuration (fused) */
    float visibility_ms;           /* visibilityPassDuration */
    float temporal_ms;             /* temporalReusePassDuration */
    float spatial_ms;              /* spatialReusePassDuration (all P passes) */
    float shade_ms;                /* shadingPassDuration (0 when fused into the last reuse pass) */
    float total_ms;                /* totalFrameDuration (history copy is a pointer swap: 0) */
    uint64_t rays;                 /* closest-hit + occlusion rays traced this frame (device count) */
    uint64_t primary_rays;
    uint64_t reproj_outside;       /* G-buffer elements the temporal pass rebuilt because a reprojection fell
                                      beyond the tile's rows +- margin (0 for full frames; tiles only) */
} rs_pass_times;

/* ---- device lifecycle (rtcNewDevice / rtcReleaseDevice) ------------------------------------- */
/* Creates a context bound to HIP device `hip_device` rendering width x height frames.  `hip_stream`
 * is a hipStream_t to render on (NULL: the context creates its own).  Owns every per-pixel buffer:
 * 2 G-buffers (current/previous), 3 reservoir buffers, the framebuffer. */
int rs_context_create(int hip_device, int width, int height, void* hip_stream, rs_context** out);
void rs_context_destroy(rs_context* ctx);
const char* rs_last_error(const rs_context* ctx);   /* ctx may be NULL: last global create error */

/* ---- scene load (Scene::Scene + ModelLoader::loadScene + rtcCommitScene) ---------------------- */
/* Uploads the triangles, builds the emissive-triangle CDF (TriangleCDF ctor, pg/TriangleCDF.cpp:8-34)
 * and builds the BVH on the GPU (PLOC agglomerative clustering over Morton-sorted triangles -> SAH
 * leaf collapse -> depth-first skip-pointer layout; env RESTIR_BVH=lbvh selects the Karras LBVH).
 * Replaces rtcNewScene/rtcCommitScene (pg/Scene.cpp:10,15). */
int rs_scene_create(rs_context* ctx, const rs_mesh_desc* meshes, uint32_t n_meshes,
                    const rs_material_desc* materials, uint32_t n_materials, rs_scene** out);
/* OBJ/MTL loader honouring Pc (material class), Kd/Ks (sRGB-expanded), Ke, Ns, vt texture
 * coordinates and map_Kd / map_Ks / map_Ns / norm textures (PNG, .hdr, .pfm, .ppm; pg/ModelLoader.cpp:
 * 41-153 conventions; tangents per triangle from the uv derivatives), then rs_scene_create_textured. */
int rs_scene_load_obj(rs_context* ctx, const char* obj_path, rs_scene** out);
/* rs_scene_create with material textures: diffuse / specular maps replace Kd / Ks, a shininess map gives
 * Ns = 2 / r^2 - 2 (Material::getShininess, pg/material.cpp:123-134), a normal map replaces the
 * (ray-facing) shading normal by TBN * (2 t - 1), unnormalised (pg/Intersection.h:26-39).  Textures are
 * copied to the device; the descriptors may be freed after the call. */
int rs_scene_create_textured(rs_context* ctx, const rs_mesh_desc* meshes, uint32_t n_meshes,
                             const rs_material_desc* materials, uint32_t n_materials,
                             const rs_texture_desc* textures, uint32_t n_textures, rs_scene** out);
/* Equirectangular sky for rs_frame_params.use_skybox (Scene::loadSkybox + SphericalMap,
 * pg/Scene.cpp:46-50, pg/SphericalMap.cpp:10-14): primary-ray misses read it (G-buffer emission,
 * pg/ReSTIRIntegrator.cpp:231; NEE miss, pg/NEEPathIntegrator.cpp:131).  NULL removes it. */
int rs_scene_set_sky(rs_scene* scene, const rs_texture_desc* equirect);
/* Loads the sky from a file (Raytracer::LoadScene's forest.hdr, pg/raytracer.cpp:34-38): Radiance
 * .hdr, .pfm, binary .ppm or PNG (8-bit gray/RGB/RGBA). */
int rs_scene_load_sky(rs_scene* scene, const char* path);
/* The scene loader's image decoder on its own (no device; tests and tools): with out == NULL only
 * width/height/channels/format are returned; else out receives width*height*channels bytes (RS_TEX_U8)
 * or floats (RS_TEX_F32), top row first -- RS_E_INVALID if out_bytes is too small. */
int rs_image_decode(const char* path, uint32_t* width, uint32_t* height, uint32_t* channels, int32_t* format,
                    void* out, size_t out_bytes);
void rs_scene_destroy(rs_scene* scene);
/* Animated geometry (C5 moving lights; the reference cannot move geometry -- the Embree analogue is
 * rtcUpdateGeometryBuffer + rtcCommitGeometry + rtcCommitScene): replaces all n_tris*9 vertex
 * positions (and, if normals != NULL, the vertex normals) in the scene's triangle order, recomputes
 * the emissive-triangle CDF on the device and refits the BVH (same topology; every query answers
 * bit-identically to a freshly built tree).  Materials and triangle count are unchanged.
 * Asynchronous, no host synchronisation (the caller's arrays are copied before return); no tile frame
 * may be open.  Frames already enqueued render the old geometry, later frames the new: with frames in
 * flight (run-ahead > 0) and normals == NULL the refit and tables are written to a second copy of the
 * scene's device data, ordered only after the frames that read that copy, and swapped in (the
 * pipeline keeps running); otherwise the update is written in place after every enqueued frame. */
int rs_scene_update_positions(rs_scene* scene, const float* positions, const float* normals);
/* Full rebuild of the CDF and a new PLOC tree from the scene's current positions -- restores tree
 * quality after large motions, where a refit tree's boxes grow.  Synchronous. */
int rs_scene_rebuild(rs_scene* scene);
/* Scene statistics: n_tris, n_emissive, n_bvh_nodes, bvh build time (ms). */
int rs_scene_info(const rs_scene* scene, uint32_t* n_tris, uint32_t* n_emissive, uint32_t* n_nodes,
                  float* build_ms);
/* The scene's ray-query structure: the 8-wide tree of the per-lane walks (wide_nodes > 0, wide_depth its deepest
 * level) or, without one, the reason (status) -- the walks then take the binary tree's skip pointers, with the same
 * hits.  A tree the walk's 8-entry group stack cannot hold (no SAH collapse within depth 8) is RS_WIDE_TOO_DEEP. */
enum {
    RS_WIDE_LIVE = 0,        /* the per-lane walks use the 8-wide tree */
    RS_WIDE_NONFINITE = 1,   /* a non-finite vertex coordinate at build time */
    RS_WIDE_TOO_DEEP = 2,    /* no collapse within the walk's stack depth (8 levels) */
    RS_WIDE_TOO_MANY = 3,    /* >= 2^24 triangles (the node word's child index) */
    RS_WIDE_EMPTY = 4,       /* no triangles */
    RS_WIDE_OFF = 5,         /* disabled (RESTIR_WIDE=off) */
    RS_WIDE_ERROR = 6        /* the build failed (device error / allocation) */
};
int rs_scene_walk_info(const rs_scene* scene, uint32_t* wide_nodes, int32_t* wide_depth, int32_t* status);

/* ---- render(frame) (SimpleGuiDX11::produceRestir) ----------------------------------------- */
/* Renders one frame: G-buffer -> initial RIS -> [visibility] -> [temporal, if a previous frame
 * exists] -> [spatial x P] -> shade; then swaps history (pointer swap instead of the reference's
 * memcpy, pg/simpleguidx11.cpp:477-481).  `frame_index` keys the counter RNG.  If frame_rgb_host is
 * non-NULL the W*H*3 framebuffer is copied to it (synchronous); `times` (optional) receives
 * per-pass device times (synchronous). */
int rs_render_frame(rs_context* ctx, const rs_scene* scene, const rs_camera* camera,
                    const rs_frame_params* params, uint32_t frame_index, float* frame_rgb_host,
                    rs_pass_times* times);
/* ---- MIS direct-light ground truth ------------------------------------------ */
/* SimpleGuiDX11::produceStandard + NEEPathIntegrator (pg/NEEPathIntegrator.cpp:72-131) with calcDI on,
 * calcGI off and DirectMISIntegrator (pg/DirectMISIntegrator.cpp:10-143: one BRDF sample + one light
 * sample, power heuristic) as the direct integrator: an unbiased estimate of the direct illumination
 * ReSTIR DI converges to.  spp samples per pixel (averaged) into the framebuffer; accumulate frames
 * with rs_post_frame for a converged reference.  Leaves the ReSTIR history untouched.  times (optional)
 * reports the launch in shade_ms/total_ms and the rays traced; synchronises if times or
 * frame_rgb_host is given. */
int rs_render_direct_mis(rs_context* ctx, const rs_scene* scene, const rs_camera* camera,
                         const rs_frame_params* params, uint32_t frame_index, uint32_t spp,
                         float* frame_rgb_host, rs_pass_times* times);

/* Pass times and rays summed over every frame finished since context creation (or the last reset),
 * without a host sync per frame: each frame records into its own slot of an event ring and the rays
 * are summed on the device.  Synchronises the stream; sum->*_ms are totals (divide by *n_frames).
 * Replaces reading the per-pass std::chrono members every frame (pg/simpleguidx11.h:120-127). */
int rs_get_timing_totals(rs_context* ctx, rs_pass_times* sum, uint32_t* n_frames, int reset);
/* Device pointer to the framebuffer (frame_data): W*H*3 floats, valid until the next render (with a
 * frame ring of 2: until the render after next). */
int rs_get_frame_device_ptr(rs_context* ctx, const float** dptr);
/* Asynchronous framebuffer readback (the reference's frame_data, pg/simpleguidx11.h:152, is host memory
 * the passes write in place).  rs_frame_readback enqueues a copy of the last rendered frame's W*H*3
 * floats into host_dst on the context's stream, ordered after that frame, and returns a ticket
 * without waiting; rs_frame_wait blocks until that copy has landed.  The next frame that would overwrite
 * the framebuffer being read (the same run-ahead lane) waits for the copy on the device, so the copy
 * overlaps the following frames' rendering.  host_dst should be page-locked (rs_host_alloc) for the
 * copy to be asynchronous. */
int rs_frame_readback(rs_context* ctx, float* host_dst, uint64_t* ticket);
int rs_frame_wait(rs_context* ctx, uint64_t ticket);
/* Page-locked host memory for rs_frame_readback (hipHostMalloc on the context's device). */
int rs_host_alloc(rs_context* ctx, size_t bytes, void** out);
void rs_host_free(void* p);
/* Forget the previous frame (frameCtr = 0): the next frame skips temporal reuse. */
int rs_reset_history(rs_context* ctx);
/* Wait for all work queued on the context's stream. */
int rs_synchronize(rs_context* ctx);

/* ---- BVH traversal kind (no reference counterpart: Embree picks its own kernels) ---------------
 * LOCKSTEP: a wave walks the node array together (scalar node loads) -- best for coherent rays.
 * LANE: every lane walks its own path (vector loads) -- best for incoherent rays in large scenes.
 * AUTO (default; env RESTIR_TRAVERSAL=lockstep|lane overrides at context creation): the first six
 * frames of a scene alternate the kinds and time them (the first frame of each kind is a warm-up; a
 * tuning frame runs alone, not beside other frames in flight, and only its kernels are timed), later
 * frames use the faster one.  Both kinds return bit-identical frames. */
#define RS_TRAVERSAL_AUTO (-1)
#define RS_TRAVERSAL_LOCKSTEP 0
#define RS_TRAVERSAL_LANE 1
int rs_context_set_traversal(rs_context* ctx, int mode);
/* mode: the requested mode; last_kind: kind the last frame ran with; scene_choice: the kind AUTO
 * settled on for `scene` (-1 while still timing; scene may be NULL). */
int rs_context_get_traversal(const rs_context* ctx, const rs_scene* scene, int* mode, int* last_kind,
                             int* scene_choice);

/* ---- candidate-split initial pass (no reference counterpart: a launch-shape choice) ------------
 * ON: the initial pass spreads a pixel's A+B candidates over 4 waves of one 8x8-tile workgroup
 * (fills the GPU when a rank renders a small band); OFF: one thread carries all candidates of its
 * pixel; AUTO (default; env RESTIR_SPLIT=on|off overrides at context creation): ON when the launch
 * has fewer than one round (frames in flight) or 3 rounds (run-ahead depth 0) of one-thread-per-pixel
 * waves for the device and the frame uses the lockstep traversal.  Needs A+B <= 64 and B <= 2
 * (OFF otherwise).  Frames are bit-identical either way. */
#define RS_SPLIT_AUTO (-1)
#define RS_SPLIT_OFF 0
#define RS_SPLIT_ON 1
int rs_context_set_initial_split(rs_context* ctx, int mode);
/* mode: the requested mode; last: whether the last frame's initial pass ran split (0/1) */
int rs_context_get_initial_split(const rs_context* ctx, int* mode, int* last);
/* Frame pipelining (no reference counterpart): with depth D (0..rs_max_run_ahead(), default the maximum;
 * env RESTIR_RUNAHEAD=D at context creation) frames rotate over D+1 internal streams, so a frame's G-buffer + initial pass
 * (which reads nothing of earlier frames) runs while up to D earlier frames still run their later
 * passes; only the temporal pass waits for the previous frame.  The context's stream waits for every
 * frame, so its semantics are unchanged; a frame's framebuffer pointer (rs_tile_finish,
 * rs_get_frame_device_ptr) stays valid for D+1 frames.  Work enqueued on the context's stream between
 * frames (geometry updates) is waited for by the next frame.  Frames are bit-identical for every D. */
int rs_context_set_run_ahead(rs_context* ctx, int depth);
/* the largest run-ahead depth this build supports (the default depth) */
int rs_max_run_ahead(void);
/* Framebuffer ring (no reference counterpart): n = 1 (default, one frame_data buffer, like
 * pg/simpleguidx11.h:152) or 2 -- consecutive frames alternate between two buffers, so a consumer
 * (the multi-GPU gather, an async copy) may still read frame f while frame f+1 renders. */
int rs_context_set_frame_ring(rs_context* ctx, int n);
/* Device bytes of the wave-sorted initial pass's hand-off buffers (phase A's candidate weights and shadow rays,
 * 20 B per candidate slot), summed over the run-ahead lanes.  They are grown on demand before a frame is
 * enqueued and sized by the launch: one region per resident wave of the persistent launch (C3 1080p: ~63 MB
 * per lane), one per 8x8 tile of a one-launch grid (a band's rows only).  If the device cannot hold them
 * the frame runs the one-thread-per-pixel initial pass instead (the same results). */
int rs_context_handoff_bytes(const rs_context* ctx, uint64_t* bytes);
/* Load-balancing record for tile sharding (no reference counterpart): while enabled, every pass
 * kernel's waves add their lifetime (100 MHz ticks) to the image row at the top of their tile, for rows
 * inside the context's band.  rs_get_row_costs copies the H per-row sums to `costs` (host, H floats;
 * synchronises the stream) and optionally zeroes them. */
int rs_context_track_row_costs(rs_context* ctx, int enable);
int rs_get_row_costs(rs_context* ctx, float* costs, int reset);

/* ---- post-frame: the producer loop's block after produceRestir -------------
 * (pg/simpleguidx11.cpp:246-333, OIDN excluded):  accumulator = mix(accumulator, frame_data,
 * 1/(accFrameCtr+1)); display = vec4(compress(aces(accumulator)), 1) per the tonemap (RenderParams,
 * default on) and gammaCorrect (Raytracer, default on) switches; mean / variance of the
 * accumulator's per-pixel channel mean.  Operates on the rows of the last rendered frame (a tile's
 * band after rs_tile_finish).  Without `accumulate` accFrameCtr restarts at 0 every frame (the
 * accumulator then equals the frame), as in the reference (:297-306).  The accumulator starts at 0. */
typedef struct {
    int32_t accumulate;        /* SimpleGuiDX11::accumulate (default false) */
    int32_t tonemap;           /* RenderParams::tonemap (default true) */
    int32_t gamma_correct;     /* Raytracer::gammaCorrect (default true) */
    int32_t max_acc_frames;    /* maxAccCount (<= 0: the reference's 300000) */
    int32_t denoise;           /* RenderParams::denoise (default false, pg/RenderParams.h:13): display the
                                  denoised accumulator (pg/simpleguidx11.cpp:277-280); needs a denoiser set
                                  with rs_context_set_denoiser and a full frame (not a tile band) */
} rs_post_params;
typedef struct {
    double mean, variance;     /* accumulatorMean / accumulatorVariance over the rows processed */
    double sum, sqr_sum;       /* the double sums behind them (combine across tiles by summing) */
    uint64_t pixels;
    uint32_t acc_frames_used;  /* accFrameCtr this frame was blended with */
    uint32_t reserved;
} rs_post_stats;
/* display_rgba_dptr (optional) receives the device pointer of the W*H float4 display buffer;
 * stats (optional) synchronises the stream. */
int rs_post_frame(rs_context* ctx, const rs_post_params* params, const float** display_rgba_dptr,
                  rs_post_stats* stats);
/* accFrameCtr = 0 (the next rs_post_frame overwrites the accumulator with the frame). */
int rs_post_reset(rs_context* ctx);

/* ---- denoiser: the reference's Open Image Denoise "RT" filter ---------------------
 * pg/simpleguidx11.cpp:52-75 (oidnNewDevice / oidnNewFilter("RT") / setImage color = accumulator, albedo =
 * gBuffer.diffuseColorBuf, normal = gBuffer.wSpaceNormalBuf, output; hdr = true; quality High; commit) and
 * :255-260 (execute every frame; errors printed).  Here: OIDN's UNet on the matrix cores (float16 storage,
 * float32 accumulation; csrc/rs_denoise.hip), weights from an OIDN tensor archive (.tza; OIDN's trained
 * rt_hdr_alb_nrm.tza is not shipped with the reference -- pass it, or any weights of the same topology).
 * Errors: RS_E_INVALID for a malformed archive / topology mismatch (the message names the tensor),
 * RS_E_UNSUPPORTED for hdr = false.  All execution is asynchronous on the context's stream. */
typedef struct rs_denoiser rs_denoiser;
typedef struct {
    int32_t input_channels;    /* 3 colour only, 6 + albedo, 9 + normal (the reference's filter: 9) */
    int32_t channels[16];      /* output channels of enc_conv0..5b, dec_conv4a..dec_conv0 */
    uint64_t parameters;
    double mac_per_pixel;      /* multiply-accumulates per (padded) input pixel */
} rs_denoiser_info;
typedef struct {
    float input_scale;         /* oidn "inputScale": <= 0 or NaN = auto-exposure (OIDN's default) */
    int32_t hdr;               /* oidn "hdr": must be 1 (the reference sets true) */
} rs_denoise_params;
/* Host only (no device work): parse + check an archive against the UNet topology. */
int rs_denoiser_check_weights(const void* tza, size_t bytes, rs_denoiser_info* info);
int rs_denoiser_create(rs_context* ctx, const void* tza, size_t bytes, rs_denoiser** out);
int rs_denoiser_create_from_file(rs_context* ctx, const char* path, rs_denoiser** out);
int rs_denoiser_info_get(const rs_denoiser* d, rs_denoiser_info* info);
/* oidnFilter.execute on device images: colour / albedo / normal / output are W*H float3 rows (the
 * reference's oidn::Format::Float3 shared buffers). */
int rs_denoiser_execute(rs_denoiser* d, const float* color, const float* albedo, const float* normal,
                        float* output, int32_t width, int32_t height, const rs_denoise_params* params);
/* The reference's per-frame call: colour = the context's accumulator (after rs_post_frame), albedo / normal
 * = the last frame's G-buffer diffuse colour / normal; *output_dptr = W*H float3 (owned by the denoiser). */
int rs_denoise_frame(rs_context* ctx, rs_denoiser* d, const rs_denoise_params* params, const float** output_dptr);
/* rs_post_frame with params->denoise runs rs_denoise_frame (auto-exposure) and tonemaps its output. */
int rs_context_set_denoiser(rs_context* ctx, rs_denoiser* d);
/* HIP-event time of the last execute (enable first; waits for it) and the input scale it used (waits). */
int rs_denoiser_set_timing(rs_denoiser* d, int enable);
int rs_denoiser_last_ms(rs_denoiser* d, float* ms);
/* ms[17]: the last timed execute's input transform (+ auto-exposure), then each of the 16 convolutions. */
int rs_denoiser_layer_ms(rs_denoiser* d, float* ms);
int rs_denoiser_get_scale(rs_denoiser* d, float* scale);
/* Test hook: the float16 activation tensor `tensor` of the last execute (0 = network input, then the
 * outputs of enc_conv0, pool(enc_conv1..4), enc_conv5a, enc_conv5b, dec_conv4a .. dec_conv1b) with its
 * one-pixel zero border, NHWC: dims = {rows + 2, cols + 2, channel stride, real channels}; host (optional)
 * receives dims[0] * dims[1] * dims[2] halves.  Synchronises. */
int rs_denoiser_dump(rs_denoiser* d, int tensor, uint16_t* host, int32_t* dims);
void rs_denoiser_destroy(rs_denoiser* d);

/* ---- image export (SimpleGuiDX11::exportImage, pg/simpleguidx11.cpp:607-650) ------
 * Writes the display buffer of the last rs_post_frame as an 8-bit RGBA PNG -- every channel
 * (uint8_t)(display * 255.0f), as the reference's glm::vec<4,uint8_t>(display_data[i] * 255.0f) -- and,
 * with write_sidecar, "<path>.txt" with the reference's fields: iteration count (accFrameCtr), area /
 * BRDF samples, spatial reuse (pass count, neighbour count, radius), temporal reuse, render time,
 * image mean / variance (of the last rs_post_frame) and the last frame's camera.  Synchronises. */
typedef struct {
    float render_time_s;       /* the `time` argument of exportImage (the caller's clock) */
    int32_t write_sidecar;
} rs_export_params;
int rs_export_png(rs_context* ctx, const char* path, const rs_export_params* params);
/* Utility: encode `channels` (1..4) interleaved 8-bit samples, top row first, as a PNG file. */
int rs_image_encode_png(const char* path, uint32_t width, uint32_t height, uint32_t channels,
                        const uint8_t* pixels);

/* ---- state dumps for golden parity ------------------------------------------------------- */
/* G-buffer of the last rendered frame (prev=0) or the one before (prev=1): W*H*19 floats per pixel
 * pos3 normal3 kd3 ks3 Le3 shininess depth type 1/I_M.  Reservoirs shaded last frame: W*H*12
 * floats per pixel point3 normal3 Li3 w_sum W confidence. */
int rs_dump_gbuffer(rs_context* ctx, int prev, float* host_out);
int rs_dump_reservoirs(rs_context* ctx, float* host_out);

/* ---- tile-sharded frames (multi-GPU) ---------------------------------------- */
/* A rank renders rows [y0, y1) of the full width x height frame.  The G-buffer is computed for the
 * rows [y0-margin, y1+margin) (recomputed margin, no exchange); the reservoir rows within `halo` of
 * the band edge are exchanged between neighbouring ranks by the caller (RCCL) between the stages:
 *   rs_tile_begin      : G-buffer (band+margin) + initial RIS (+ visibility) for the band
 *   rs_tile_halo_ptr   : device pointers of the current reservoir buffer's halo rows
 *   rs_tile_temporal   : temporal reuse on the band
 *   rs_tile_spatial    : one spatial pass on the band (reads the halo rows)
 *   rs_tile_finish     : shade, history swap; returns the band's framebuffer device pointer
 * Per-pixel counter RNG keyed by the full-frame pixel index makes the result bit-identical to a
 * single-GPU frame for any margin >= halo: a temporal reprojection beyond the tile's G-buffer rows
 * rebuilds the element it needs from the frame's camera (counted in rs_pass_times.reproj_outside). */
typedef struct {
    int32_t y0, y1;         /* band rows, 0 <= y0 < y1 <= height */
    int32_t margin;         /* G-buffer rows recomputed beyond the band (>= halo) */
    int32_t halo;           /* reservoir rows exchanged each side (floor(sqrt(R)) for spatial reuse) */
} rs_tile_desc;
int rs_tile_begin(rs_context* ctx, const rs_scene* scene, const rs_camera* camera,
                  const rs_frame_params* params, uint32_t frame_index, const rs_tile_desc* tile);
/* which: 0 = rows [y0-halo, y0) (receive from the rank above), 1 = rows [y1, y1+halo) (from below),
 *        2 = rows [y0, y0+halo) (send up), 3 = rows [y1-halo, y1) (send down).
 * *bytes = rows * width * 48; NULL pointer when the rows fall outside the frame. */
int rs_tile_halo_ptr(rs_context* ctx, int which, void** dptr, size_t* bytes);
/* The stream the frame in flight runs on (a run-ahead lane, or the context's stream at depth 0) and its
 * lane index: a multi-GPU driver issues the frame's halo exchange and gather on it, so frames of
 * different lanes communicate independently. */
int rs_tile_stream(rs_context* ctx, void** stream, int* lane);
int rs_tile_temporal(rs_context* ctx);
int rs_tile_spatial(rs_context* ctx, int pass_index);
int rs_tile_finish(rs_context* ctx, const float** band_rgb_dptr, rs_pass_times* times);

/* ---- multi-GPU frames behind the ABI (SURVEY.md §8b rs_mgpu_render_frame, §8e) ------------------
 * The caller of the reference (SimpleGuiDX11::Producer, pg/simpleguidx11.cpp:240-241) renders one frame
 * per produceRestir; here a frame of `world` row bands is rendered by one rs_mgpu_render_frame call per
 * rank (process), each rank on its own GPU context: G-buffer + initial RIS of its rows, temporal, then
 * before every spatial pass a point-to-point halo exchange of floor(sqrt(R)) reservoir rows with each
 * neighbour (RCCL ncclSend/ncclRecv group on the frame's stream; one communicator per run-ahead lane so
 * frames in flight communicate independently), shade, and a gather of the band framebuffers into rank
 * 0's context framebuffer (rs_get_frame_device_ptr / rs_frame_readback on rank 0 then see the full
 * frame).  The gathered frame is bit-identical to a single-GPU frame.
 *   rank 0: rs_mgpu_unique_id(id); distribute id to every rank (MPI, a file, torch.distributed, ...)
 *   every rank: rs_context_create(device) -> rs_scene_* (same scene) -> rs_mgpu_create(ctx, rank, world, id)
 *               per frame: rs_mgpu_render_frame(m, &scene, camera, params, frame, gather=1, host_or_NULL, NULL)
 * rs_mgpu_create_local drives `world` contexts of ONE process (a rank per context; transfers are device
 * copies) -- several GPUs from one thread, or ranks sharing a GPU (tests).  `scenes` holds one scene per
 * local rank (each loaded on that rank's context).  Calls are collective: every rank calls them in the
 * same order. */
typedef struct rs_mgpu rs_mgpu;
#define RS_MGPU_ID_BYTES 128
int rs_mgpu_unique_id(uint8_t id[RS_MGPU_ID_BYTES]);
int rs_mgpu_create(rs_context* ctx, int rank, int world, const uint8_t id[RS_MGPU_ID_BYTES], rs_mgpu** out);
int rs_mgpu_create_local(rs_context* const* ctxs, int world, rs_mgpu** out);
void rs_mgpu_destroy(rs_mgpu* m);
/* row bands: bounds[0] = 0 < bounds[1] < ... < bounds[world] = height (equal bands at creation) */
int rs_mgpu_set_bands(rs_mgpu* m, const int32_t* bounds);
int rs_mgpu_get_bands(const rs_mgpu* m, int32_t* bounds);
/* Cost-balanced bands: renders n_frames (no gather) while the pass kernels record per-row wave time
 * (rs_context_track_row_costs), all-reduces the rows' costs, moves the boundaries to equal cost (every
 * band >= max(min_rows, halo) rows; same split on every rank), resets the history. */
int rs_mgpu_rebalance(rs_mgpu* m, const rs_scene* const* scenes, const rs_camera* camera,
                      const rs_frame_params* params, uint32_t first_frame, int n_frames, int min_rows);
/* Then (rounds > 0, default 2) time-based refinement inside rs_mgpu_rebalance: each round renders frames with
 * the current bands (gathered, frames in flight), all-reduces every rank's own time per frame (its frames'
 * begin..shade span minus its halo exchanges, plus rank 0's gather), rescales each band's row costs to its
 * time and balances again; the measured bands with the lowest maximum are kept.  rounds = 0: row costs only.
 * The setting persists on `m` until set again (the Python wrapper passes 2 whenever its caller gives none).
 * Side effects: rs_mgpu_rebalance renders n_frames frames, plus per measured round 2 + max(n_frames, 6)
 * gathered frames (frame indices first_frame, first_frame + 1, ...), which overwrite rank 0's framebuffer;
 * the contexts' timing totals and the rs_mgpu stats keep counting those frames (read as deltas, never
 * reset); the history is reset on return.
 * rs_mgpu_rebalance_times: the last rebalance's measured ms per rank (world values) of measured round r. */
int rs_mgpu_set_rebalance_refine(rs_mgpu* m, int rounds);
int rs_mgpu_rebalance_times(const rs_mgpu* m, int round, double* ms);
/* One frame.  gather != 0: bands -> rank 0's framebuffer; frame_rgb_host (rank 0, optional) receives it
 * (synchronous).  times (optional, synchronous): the first local rank's pass times. */
int rs_mgpu_render_frame(rs_mgpu* m, const rs_scene* const* scenes, const rs_camera* camera,
                         const rs_frame_params* params, uint32_t frame_index, int gather, float* frame_rgb_host,
                         rs_pass_times* times);
/* the first local rank's framebuffer (on rank 0 after a gather: the full frame) */
int rs_mgpu_frame_device_ptr(rs_mgpu* m, const float** dptr);
int rs_mgpu_reset_history(rs_mgpu* m);
/* host values summed (op 0) or maxed (op 1) over all ranks in place (RCCL all-reduce; synchronous) --
 * for the caller's timing / statistics, not on the frame's data path */
int rs_mgpu_allreduce(rs_mgpu* m, double* values, int n, int op);
/* Transfer statistics of this process's ranks since creation / the last reset (synchronous: waits for
 * every frame enqueued).  Times are HIP-event spans on the frame's stream of the first local rank: a
 * halo exchange (each spatial pass, first 4 timed) and the gather, including any wait for the peer. */
typedef struct rs_mgpu_stats {
    uint64_t frames;
    uint64_t halo_bytes_sent, halo_bytes_recv;   /* reservoir halo rows, all local ranks */
    uint64_t gather_bytes;                       /* framebuffer rows received by rank 0 */
    double halo_ms, gather_ms;
} rs_mgpu_stats;
int rs_mgpu_get_stats(rs_mgpu* m, rs_mgpu_stats* out, int reset);

/* ---- test hook: raw BVH queries (rtcIntersect1 / rtcOccluded1 semantics) ----------------------
 * n rays, host arrays o[3n], d[3n], tnear[n], tfar[n].  any_hit=0: closest hit -> t_out[n] (-1 on miss),
 * prim_out[n] (original triangle index, -1 on miss); any_hit=1: prim_out[n] = 1 if occluded else 0.
 * Modes 0/1 use the lockstep traversal, 2/3 the same queries per-lane (the 8-wide tree when the scene has
 * one); 4 (closest) / 5 (any) return per-ray skip-pointer walk statistics instead: prim_out[n] = node
 * visits << 16 | triangle tests; 6 (closest) / 7 (any) the 8-wide walk's: node fetches << 16 | triangle
 * tests, t_out = 1 if its stack overflowed; 8 / 9 / 10 are timing probes of the 8-wide walk (closest;
 * any-hit without triangle tests; any-hit).  Modes 6-10 return prim -1 / t -1 without a wide tree. */
int rs_debug_trace(rs_context* ctx, const rs_scene* scene, uint32_t n, const float* o, const float* d,
                   const float* tnear, const float* tfar, int any_hit, float* t_out, int32_t* prim_out);

/* ---- test hook: the scene's 8-wide tree (rs_wide.h layout, built on the GPU by rs_wide_build.hip and refit
 * with the positions) ----------------------------------------------------------------------------------
 * *n_nodes / *n_tris = its size (0 / 0: the scene has no wide tree; its walks take the skip pointers);
 * *depth = its deepest level.  With words != NULL (20 * *n_nodes uint32) and prims != NULL (*n_tris int32)
 * it also copies the node words and each wide-leaf triangle's original triangle index (synchronous). */
int rs_debug_wide_tree(const rs_scene* scene, uint32_t* n_nodes, uint32_t* n_tris, int32_t* depth, uint32_t* words,
                       int32_t* prims);

#ifdef __cplusplus
}
#endif
#endif /* RESTIR_C_H */
