// rs_internal.h -- library-internal helpers shared between restir_capi.hip and rs_mgpu.hip (not part of
// the C ABI; hidden symbols).
#pragma once
#include <hip/hip_runtime.h>
#include <string>

struct rs_context;
struct rs_denoiser;

// run-ahead: the deepest frame pipeline a context supports (restir_capi.hip kMaxAhead; frames in flight =
// depth + 1 lanes, each with its own stream, framebuffer and -- in rs_mgpu.hip -- communicator)
#ifndef RS_MAX_AHEAD
#define RS_MAX_AHEAD 2
#endif

namespace rs {
// the context's own stream (ordered after every frame enqueued so far)
__attribute__((visibility("hidden"))) hipStream_t ctx_stream(rs_context* c);
__attribute__((visibility("hidden"))) int ctx_device(const rs_context* c);
__attribute__((visibility("hidden"))) int ctx_width(const rs_context* c);
__attribute__((visibility("hidden"))) int ctx_height(const rs_context* c);
// work enqueued on `st` after the frame (a multi-GPU gather into the frame's framebuffer) becomes part of
// the frame for everything that orders on the context's stream (readback, post-frame, the next frame)
__attribute__((visibility("hidden"))) int ctx_join(rs_context* c, hipStream_t st);
// record an error message on the context (rs_last_error) and return `code`
__attribute__((visibility("hidden"))) int ctx_fail(rs_context* c, int code, const std::string& msg);
// rs_denoise.hip: the denoiser on device images (float3 rows at `*st` floats per pixel), enqueued on `st`;
// input_scale <= 0 / NaN: auto-exposure.  The output buffer rs_denoise_frame writes; the owning context.
__attribute__((visibility("hidden"))) int denoise_run(rs_denoiser* d, hipStream_t st, const float* color, int cst,
                                                      const float* albedo, int ast, const float* normal, int nst,
                                                      float* out, int ost, int H, int W, float input_scale);
__attribute__((visibility("hidden"))) float* denoiser_frame_out(rs_denoiser* d, int W, int H);
__attribute__((visibility("hidden"))) rs_context* denoiser_ctx(const rs_denoiser* d);
// denoiser lifetime: a context tracks the denoisers created on it; rs_denoiser_destroy unregisters one (and
// clears the context's post-frame denoiser when it is that one); rs_context_destroy detaches the rest, which
// then fail their calls with RS_E_INVALID and free only their own memory in rs_denoiser_destroy
__attribute__((visibility("hidden"))) void ctx_track_denoiser(rs_context* c, rs_denoiser* d, bool add);
__attribute__((visibility("hidden"))) void denoiser_detach(rs_denoiser* d);
}  // namespace rs
