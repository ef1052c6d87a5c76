// rs_internal.h -- library-internal helpers shared between restir_capi.hip and rs_mgpu.hip (not part of
// the C ABI; hidden symbols).
#pragma once
#include <hip/hip_runtime.h>
#include <string>

struct rs_context;

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
}  // namespace rs
