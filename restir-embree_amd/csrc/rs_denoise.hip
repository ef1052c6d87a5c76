// rs_denoise.hip -- the reference's denoiser on gfx950 matrix cores.
//
// The reference runs Open Image Denoise's "RT" filter on the accumulator every produced frame, with the
// current G-buffer's diffuse colour as albedo and world-space normal as normal, hdr = true, quality High
// (pg/simpleguidx11.cpp:52-75 setup, :255-256 execute), and displays the result when RenderParams::denoise
// is on (pg/RenderParams.h:13, pg/simpleguidx11.cpp:273-280).  OIDN ships with the reference only as
// Windows binaries (template/src/libs/oidn-2.3.3.x64.windows) and its trained weights are not shipped, so
// this is OIDN 2.3's published network and pre/post-processing restated (oracle/denoise_ref.py is the
// fp32 checker), running weights loaded from an OIDN tensor archive (.tza, restir_amd/tza.py).
//
// Network: OIDN's UNet -- 16 3x3 convolutions (enc_conv0..5b, dec_conv4a..0), ReLU, 2x2 max pooling
// after enc_conv1..4, nearest 2x upsampling + channel concatenation [upsampled, skip] before
// dec_conv4a/3a/2a/1a.  ~120 k MAC per pixel at the default channel counts (0.5 TFLOP per 1080p frame):
// the one GEMM-shaped workload of the renderer, so it runs on MFMA:
//   * activations: NHWC float16, channels padded to a multiple of 16, every level's tensor stored with a
//     one-pixel zero border (the convolutions' zero padding; the border is never written);
//   * one kernel per convolution, an implicit GEMM: a workgroup (4 waves) computes a 16x16-pixel output
//     tile for all output channels; the input halo (18x18 pixels x 32 channels) is staged in LDS (two
//     buffers: the next channel chunk's global loads are in flight while the MFMAs run on this one;
//     XOR-swizzled 16-B slots so a wave's fragment reads are bank-conflict free); each wave owns 8x8
//     pixels = 4 groups of 16 (2x2 quads side by side), A fragments (16 pixels x 32 k) come from LDS, B
//     fragments (32 k x 16 output channels) are pre-packed per lane on the host so each is one coalesced
//     1-KB load; v_mfma_f32_16x16x32_f16, float32 accumulation;
//   * a k-step is one tap x 32 channels, or -- for 16-channel chunks (the 9-channel input, the odd half of
//     48 / 80 / 112-channel tensors) -- two taps x 16 channels;
//   * fused: bias + ReLU; 2x2 max pooling (a lane's 4 accumulator registers ARE a 2x2 quad); the
//     decoder's upsampling and concatenation (the halo loader reads the coarse tensor at (y>>1, x>>1) and
//     each source's channel chunks in turn); the output transform (inverse PU / input scale) in the last
//     convolution, which writes float3 rows at the caller's stride;
//   * input transform + auto-exposure: two small streaming kernels before the first convolution.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/restir_c.h"
#include "rs_internal.h"

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace rs {
namespace dn {

// PU transfer function of OIDN's HDR path (oracle/denoise_ref.py restates the same constants)
constexpr float PU_A = 1.41283765e+03f, PU_B = 1.64593172e+00f, PU_C = 4.31384981e-01f;
constexpr float PU_D = -2.94139609e-03f, PU_E = 1.92653254e-01f, PU_F = 6.26026094e-03f, PU_G = 9.98620152e-01f;
constexpr float PU_Y0 = 1.57945760e-06f, PU_Y1 = 3.22087631e-02f;
constexpr float PU_X0 = 2.23151711e-03f, PU_X1 = 3.70974749e-01f;
constexpr float HDR_Y_MAX = 65504.0f;

__host__ __device__ inline float pu_forward(float y) {
    if (y <= PU_Y0) return PU_A * y;
    if (y <= PU_Y1) return PU_B * powf(y, PU_C) + PU_D;
    return PU_E * logf(y + PU_F) + PU_G;
}
__device__ inline float pu_inverse(float x) {
    if (x <= PU_X0) return x / PU_A;
    if (x <= PU_X1) return powf((x - PU_D) / PU_B, 1.0f / PU_C);
    return expf((x - PU_G) / PU_E) - PU_F;
}

constexpr int kTile = 16;                      // output tile edge (pixels)
constexpr int kHalo = kTile + 2;               // 18
constexpr int kHaloPx = kHalo * kHalo;         // 324
// Halo image of one 32-channel chunk in LDS: pixel (r, c) at r * kRowBytes + c * 64, 16-B slot s at + 16 s.
// ds_read_b128 serves a wave in 4 lane groups of 16 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and the same
// +32; MI355X_MICROARCH.md §LDS); with 64-B pixels and a row pitch of 32 mod 256 bytes (18 x 64 + 160) the
// 16 lanes of every group read 16 distinct 4-bank units at every tap, for 32- and 16-channel chunks
// (an exhaustive check over the linear layouts; the XOR swizzle before it was 2-way, SQ_LDS_BANK_CONFLICT
// ~3 extra cycles per LDS instruction).  Linear addresses: group and tap offsets are immediates.
constexpr int kRowBytes = kHalo * 64 + 160;    // 1312
constexpr int kChunkBytes = kHalo * kRowBytes; // 23616 B
constexpr int kMaxChunks = 12;
constexpr int kStageRegs = (kHaloPx * 4 + 255) / 256;   // 16-B staging slots per thread (6)
constexpr size_t kFillWorkgroups = 256;                   // one workgroup per CU before splitting channels
                                                          // (splitting re-stages the halo: measured slower
                                                          // at 1/4 resolution, faster only at 1/16)
constexpr int kMaxNtw = 4;                                // n-tiles per workgroup: 16 x 4 accumulators per lane

enum Post : int { POST_STORE = 0, POST_POOL = 1, POST_FINAL = 2 };

struct ConvArgs {
    const _Float16* src[2];
    int cs[2];                 // channel stride (elements) of each source tensor
    int sh[2], sw[2];          // interior height / width of each source tensor
    int up[2];                 // source read through nearest 2x upsampling
    int nchunk;
    int ch_src[kMaxChunks], ch_base[kMaxChunks], ch_w[kMaxChunks], ch_step[kMaxChunks];
    const half8* w;            // [k-step][n-tile][64 lanes] B fragments
    const float* bias;         // n-tiles * 16 (zero padded)
    int nt_total;              // n-tiles of the layer; a workgroup computes NT of them from blockIdx.z * NT
    _Float16* dst;             // POST_STORE / POST_POOL: output tensor (bordered NHWC)
    int dcs;                   // its channel stride
    int h, w_;                 // this convolution's output-level interior size
    float* out;                // POST_FINAL: float3 rows, `ostride` floats per pixel
    int ostride, H, W;
    const float* scale;        // device input scale
    float inv_norm;            // 1 / NORM_SCALE = pu_forward(65504)
};

__device__ __forceinline__ void stage_load(const ConvArgs& a, int c, int tx0, int ty0, uint4 (&r)[kStageRegs]) {
    const int s = a.ch_src[c];
    const int spp = a.ch_w[c] >> 3;            // 16-B slots per pixel: 4 (32 ch) or 2 (16 ch)
    const _Float16* src = a.src[s];
    const int cs = a.cs[s], sh = a.sh[s], sw = a.sw[s], up = a.up[s], base = a.ch_base[c];
    const int nslots = kHaloPx * spp;
#pragma unroll
    for (int k = 0; k < kStageRegs; ++k) {
        const int q = (int)threadIdx.x + k * 256;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (q < nslots) {
            const int px = spp == 4 ? (q >> 2) : (q >> 1), sl = q & (spp - 1);
            const int hr = px / kHalo, hc = px - hr * kHalo;
            int y = ty0 - 1 + hr, x = tx0 - 1 + hc;
            if (up) { y >>= 1; x >>= 1; }      // arithmetic: -1 stays -1 (the border)
            if (y >= -1 && y <= sh && x >= -1 && x <= sw)
                v = *(const uint4*)(src + ((size_t)(y + 1) * (size_t)(sw + 2) + (size_t)(x + 1)) * cs + base + 8 * sl);
        }
        r[k] = v;
    }
}
__device__ __forceinline__ void stage_store(uint8_t* buf, int spp, const uint4 (&r)[kStageRegs]) {
    const int nslots = kHaloPx * spp;
#pragma unroll
    for (int k = 0; k < kStageRegs; ++k) {
        const int q = (int)threadIdx.x + k * 256;
        if (q < nslots) {
            const int px = spp == 4 ? (q >> 2) : (q >> 1), sl = q & (spp - 1);
            const int hr = px / kHalo, hc = px - hr * kHalo;
            *(uint4*)(buf + hr * kRowBytes + hc * 64 + (sl << 4)) = r[k];
        }
    }
}

// B fragments: all four waves of a workgroup multiply the same weights, so a chunk's B fragments are
// staged once per workgroup into LDS ([step][n-tile][64 lanes] x 16 B, a wave's fragment read = 1 KB
// contiguous: conflict-free) instead of each wave loading them from L2 -- the per-wave loads were 6x the
// halo staging's vector-memory instructions and kept the texture data path 82 % busy (r03_pmc_denoise).
// Halo and B buffers are single: loads of chunk c + 1 into registers overlap chunk c's MFMAs, then two
// barriers around the LDS writes.
// Only for NT <= 3: a 4-n-tile chunk's 36 KB of B would leave 2 workgroups per CU (measured slower on
// dec_conv1a: 247 vs 219 us); those keep per-wave global B loads (next step's prefetched) and a
// double-buffered halo.
#ifndef RS_DN_HALFB
#define RS_DN_HALFB 1
#endif
template <int NT> struct BStage { static constexpr bool lds = NT <= 3 && !(RS_DN_HALFB && NT == 2); static constexpr int kRegs = lds ? (9 * NT * 64 + 255) / 256 : 1; };
// NT = 4 and 2: B staged through LDS in two stages per 32-channel chunk (steps 0-4, then 5-8: 5 NT KB at a
// time): NT = 4 keeps the LDS budget of the per-wave-B form (3 workgroups per CU) without its per-wave B
// loads, NT = 2 fits 4 workgroups per CU instead of 3 (whole-chunk staging).  NT = 1 and 3 gain nothing
// from it (measured: equal; NT = 3 is register-bound at 3 waves)
#ifndef RS_DN_B4_STEPS
#define RS_DN_B4_STEPS 5
#endif
template <int NT> struct BHalf { static constexpr bool on = RS_DN_HALFB && (NT == 4 || NT == 2);
                                 static constexpr int steps = NT == 4 ? RS_DN_B4_STEPS : 5;   // k-steps per LDS stage
                                 static constexpr int waves = NT == 4 && steps > 3 ? 3 : 4;   // per SIMD (= workgroups per CU by LDS)
                                 static constexpr int kRegs = (steps * NT * 64 + 255) / 256; };
// B fragments of steps [s0, s0 + ns) of chunk c into registers / from registers into bbuf (step s0 first)
template <int NT>
__device__ __forceinline__ void bhalf_load(const ConvArgs& a, int c, int n0, int s0, int ns, uint4 (&r)[BHalf<NT>::kRegs]) {
    const int n = ns * NT * 64;
    const uint4* w = (const uint4*)a.w;
#pragma unroll
    for (int k = 0; k < BHalf<NT>::kRegs; ++k) {
        const int q = (int)threadIdx.x + k * 256;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (q < n) {
            const int st = q / (NT * 64), rem = q - st * (NT * 64);
            v = w[((size_t)(a.ch_step[c] + s0 + st) * a.nt_total + n0) * 64 + rem];
        }
        r[k] = v;
    }
}
template <int NT>
__device__ __forceinline__ void bhalf_store(uint8_t* bbuf, int ns, const uint4 (&r)[BHalf<NT>::kRegs]) {
    const int n = ns * NT * 64;
#pragma unroll
    for (int k = 0; k < BHalf<NT>::kRegs; ++k) {
        const int q = (int)threadIdx.x + k * 256;
        if (q < n) *(uint4*)(bbuf + q * 16) = r[k];
    }
}

template <int NT>
__device__ __forceinline__ void bstage_load(const ConvArgs& a, int c, int n0, uint4 (&r)[BStage<NT>::kRegs]) {
    const int nst = a.ch_w[c] == 32 ? 9 : 5;
    const int n = nst * NT * 64;               // 16-B pieces: (step, n-tile, lane)
    const uint4* w = (const uint4*)a.w;
#pragma unroll
    for (int k = 0; k < BStage<NT>::kRegs; ++k) {
        const int q = (int)threadIdx.x + k * 256;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (q < n) {
            const int st = q / (NT * 64), rem = q - st * (NT * 64);
            v = w[((size_t)(a.ch_step[c] + st) * a.nt_total + n0) * 64 + rem];
        }
        r[k] = v;
    }
}
template <int NT>
__device__ __forceinline__ void bstage_store(uint8_t* bbuf, int nst, const uint4 (&r)[BStage<NT>::kRegs]) {
    const int n = nst * NT * 64;
#pragma unroll
    for (int k = 0; k < BStage<NT>::kRegs; ++k) {
        const int q = (int)threadIdx.x + k * 256;
        if (q < n) *(uint4*)(bbuf + q * 16) = r[k];
    }
}

// steps [s0, s1) of chunk c (s1 < 0: all); BL: B fragments from bbuf (step s0 first), else per wave from global
template <int NT, bool BL = BStage<NT>::lds || BHalf<NT>::on>
__device__ __forceinline__ void compute_chunk(const ConvArgs& a, int c, const uint8_t* buf, const uint8_t* bbuf,
                                              f32x4 (&acc)[4][NT], int lane, int X, int Yb, int n0, int s0 = 0,
                                              int s1 = -1) {
    const int h = lane >> 4;
    const bool w32 = a.ch_w[c] == 32;
    const int nst = s1 >= 0 ? s1 : (w32 ? 9 : 5);
    const half8* bp = (const half8*)bbuf + lane - s0 * NT * 64;                       // BL
    const half8* wp = a.w + ((size_t)a.ch_step[c] * a.nt_total + n0) * 64 + lane;     // otherwise
    half8 bg[NT];
    if constexpr (!BL)
#pragma unroll
        for (int n = 0; n < NT; ++n) bg[n] = wp[n * 64];
    for (int st = s0; st < nst; ++st) {
        int tap, sl;
        if (w32) { tap = st; sl = h; }
        else { tap = 2 * st + (h >> 1); tap = tap > 8 ? 8 : tap; sl = h & 1; }   // tap 9: zero weights
        const int ky = tap / 3, kx = tap - 3 * ky;
        half8 b[NT], bn[NT];
        if constexpr (BL) {
#pragma unroll
            for (int n = 0; n < NT; ++n) b[n] = bp[(st * NT + n) * 64];
        } else {
#pragma unroll
            for (int n = 0; n < NT; ++n) b[n] = bg[n];
            if (st + 1 < nst)
#pragma unroll
                for (int n = 0; n < NT; ++n) bn[n] = wp[((st + 1) * a.nt_total + n) * 64];
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int hr = Yb + 2 * g + ky, hc = X + kx;
            const half8 av = *(const half8*)(buf + hr * kRowBytes + hc * 64 + (sl << 4));
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b[n], acc[g][n], 0, 0, 0);
        }
        if constexpr (!BL)
#pragma unroll
            for (int n = 0; n < NT; ++n) bg[n] = bn[n];
    }
}

template <int NT, int POST>
struct ConvLds {
    static constexpr int kB = 9 * NT * 1024;   // one chunk's B fragments
    static constexpr int kIn = BStage<NT>::lds ? kChunkBytes + kB
                             : BHalf<NT>::on ? kChunkBytes + BHalf<NT>::steps * NT * 1024 : 2 * kChunkBytes;
    static constexpr int kOut = POST == POST_STORE ? 256 * (NT * 16 + 8) * 2 : POST == POST_POOL ? 64 * (NT * 16 + 8) * 2
                                                                                     : 256 * 17 * 4;
    static constexpr int kBytes = kIn > kOut ? kIn : kOut;
};

template <int NT, int POST, bool RELU>
__global__ void __launch_bounds__(256, BHalf<NT>::on ? BHalf<NT>::waves : 1) k_conv3(ConvArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[ConvLds<NT, POST>::kBytes];
    uint8_t* const bbuf = lds + kChunkBytes;
    const int tx0 = blockIdx.x * kTile, ty0 = blockIdx.y * kTile;
    const int n0 = blockIdx.z * NT;            // first n-tile of this workgroup
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wy = wv >> 1, wx = wv & 1;
    const int i = lane & 15, h = lane >> 4;
    // A row i of a group = pixel (x, y) = (2 (i >> 2) + (i & 1), (i >> 1) & 1) of its 8x2 block
    const int X = 8 * wx + 2 * (i >> 2) + (i & 1);
    const int Yb = 8 * wy + ((i >> 1) & 1);

    f32x4 acc[4][NT];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[g][n] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    uint4 st[kStageRegs];
    if constexpr (BStage<NT>::lds) {           // single halo + B buffers, two barriers per chunk
        uint4 bs[BStage<NT>::kRegs];
        stage_load(a, 0, tx0, ty0, st);
        bstage_load<NT>(a, 0, n0, bs);
        stage_store(lds, a.ch_w[0] >> 3, st);
        bstage_store<NT>(bbuf, a.ch_w[0] == 32 ? 9 : 5, bs);
        __syncthreads();
        for (int c = 0; c < a.nchunk; ++c) {
            const bool more = c + 1 < a.nchunk;
            if (more) {                        // in flight during the MFMAs
                stage_load(a, c + 1, tx0, ty0, st);
                bstage_load<NT>(a, c + 1, n0, bs);
            }
            compute_chunk<NT>(a, c, lds, bbuf, acc, lane, X, Yb, n0);
            __syncthreads();
            if (more) {
                stage_store(lds, a.ch_w[c + 1] >> 3, st);
                bstage_store<NT>(bbuf, a.ch_w[c + 1] == 32 ? 9 : 5, bs);
                __syncthreads();
            }
        }
    } else if constexpr (BHalf<NT>::on) {      // single halo buffer, B in LDS stages of S k-steps
        constexpr int S = BHalf<NT>::steps;
        uint4 bs[BHalf<NT>::kRegs];
        auto nsteps = [&](int c) { return a.ch_w[c] == 32 ? 9 : 5; };
        stage_load(a, 0, tx0, ty0, st);
        bhalf_load<NT>(a, 0, n0, 0, S < nsteps(0) ? S : nsteps(0), bs);
        stage_store(lds, a.ch_w[0] >> 3, st);
        bhalf_store<NT>(bbuf, S < nsteps(0) ? S : nsteps(0), bs);
        __syncthreads();
        for (int c = 0; c < a.nchunk; ++c) {
            const int nst = nsteps(c), nsg = (nst + S - 1) / S;
            const bool more = c + 1 < a.nchunk;
            for (int sg = 0; sg < nsg; ++sg) {  // one compute call site: one inlined copy of the step loop
                const bool last = sg + 1 == nsg;
                const int s0 = sg * S, s1 = last ? nst : s0 + S;
                if (!last) {                     // this chunk's next stage
                    const int e = s1 + S < nst ? s1 + S : nst;
                    bhalf_load<NT>(a, c, n0, s1, e - s1, bs);
                } else if (more) {
                    const int nn = nsteps(c + 1);
                    stage_load(a, c + 1, tx0, ty0, st);
                    bhalf_load<NT>(a, c + 1, n0, 0, S < nn ? S : nn, bs);
                }
                compute_chunk<NT, true>(a, c, lds, bbuf, acc, lane, X, Yb, n0, s0, s1);
                __syncthreads();
                if (!last) {
                    const int e = s1 + S < nst ? s1 + S : nst;
                    bhalf_store<NT>(bbuf, e - s1, bs);
                    __syncthreads();
                }
            }
            if (more) {
                const int nn = nsteps(c + 1);
                stage_store(lds, a.ch_w[c + 1] >> 3, st);
                bhalf_store<NT>(bbuf, S < nn ? S : nn, bs);
                __syncthreads();
            }
        }
    } else {                                   // double-buffered halo, per-wave global B
        stage_load(a, 0, tx0, ty0, st);
        stage_store(lds, a.ch_w[0] >> 3, st);
        __syncthreads();
        for (int c = 0; c < a.nchunk; ++c) {
            const bool more = c + 1 < a.nchunk;
            if (more) stage_load(a, c + 1, tx0, ty0, st);      // in flight during the MFMAs
            compute_chunk<NT, false>(a, c, lds + (c & 1) * kChunkBytes, nullptr, acc, lane, X, Yb, n0);
            if (more) stage_store(lds + ((c + 1) & 1) * kChunkBytes, a.ch_w[c + 1] >> 3, st);
            __syncthreads();
        }
    }

    // epilogue.  C/D: lane holds column co = 16 n + i and rows 4 h + r (r = register): pixel
    // (2 h + (r & 1), r >> 1) of the group's 8x2 block -- one 2x2 quad per lane
    // LDS out images: pixel pitch CS + 8 halves (16 B more than the channels; float images 17 floats) so
    // the 4 quads of a wave-instruction's scattered 2-B / 4-B writes fall on different banks
    if constexpr (POST == POST_STORE) {
        constexpr int CS = NT * 16, CP = CS + 8;
        _Float16* o = (_Float16*)lds;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const float bv = a.bias[16 * (n0 + n) + i];
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = acc[g][n][r] + bv;
                    if (RELU) v = v > 0.0f ? v : 0.0f;
                    const int px = (8 * wy + 2 * g + (r >> 1)) * kTile + 8 * wx + 2 * h + (r & 1);
                    o[px * CP + 16 * n + i] = (_Float16)v;
                }
        }
        __syncthreads();
        constexpr int PPP = CS / 8;            // 16-B pieces per pixel
        for (int q = threadIdx.x; q < 256 * PPP; q += 256) {
            const int px = q / PPP, pc = q - px * PPP;
            const int gy = ty0 + (px >> 4), gx = tx0 + (px & 15);
            if (gy < a.h && gx < a.w_)
                *(uint4*)(a.dst + ((size_t)(gy + 1) * (size_t)(a.w_ + 2) + (size_t)(gx + 1)) * a.dcs + 16 * n0 + 8 * pc) =
                    *(const uint4*)(o + px * CP + 8 * pc);
        }
    } else if constexpr (POST == POST_POOL) {
        constexpr int CS = NT * 16, CP = CS + 8;
        _Float16* o = (_Float16*)lds;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const float bv = a.bias[16 * (n0 + n) + i];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 v4 = acc[g][n];
                float m = fmaxf(fmaxf(v4[0], v4[1]), fmaxf(v4[2], v4[3])) + bv;
                if (RELU) m = m > 0.0f ? m : 0.0f;
                const int px = (4 * wy + g) * 8 + 4 * wx + h;   // 8x8 pooled tile
                o[px * CP + 16 * n + i] = (_Float16)m;
            }
        }
        __syncthreads();
        constexpr int PPP = CS / 8;
        const int ph = a.h >> 1, pw = a.w_ >> 1;
        for (int q = threadIdx.x; q < 64 * PPP; q += 256) {
            const int px = q / PPP, pc = q - px * PPP;
            const int gy = (ty0 >> 1) + (px >> 3), gx = (tx0 >> 1) + (px & 7);
            if (gy < ph && gx < pw)
                *(uint4*)(a.dst + ((size_t)(gy + 1) * (size_t)(pw + 2) + (size_t)(gx + 1)) * a.dcs + 16 * n0 + 8 * pc) =
                    *(const uint4*)(o + px * CP + 8 * pc);
        }
    } else {   // POST_FINAL: dec_conv0 (linear) + the output transform, float3 at the caller's stride
        float* o = (float*)lds;
        const float bv = a.bias[i];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int px = (8 * wy + 2 * g + (r >> 1)) * kTile + 8 * wx + 2 * h + (r & 1);
                o[px * 17 + i] = acc[g][0][r] + bv;
            }
        __syncthreads();
        const int px = threadIdx.x;
        const int gy = ty0 + (px >> 4), gx = tx0 + (px & 15);
        if (gy < a.H && gx < a.W) {
            const float inv_scale = 1.0f / *a.scale;
            float* dst = a.out + ((size_t)gy * a.W + gx) * a.ostride;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                float v = o[px * 17 + k];
                v = v > 0.0f ? v : 0.0f;                       // max(x, 0), NaN -> 0
                float y = pu_inverse(v * a.inv_norm) * inv_scale;
                dst[k] = isfinite(y) ? y : 0.0f;
            }
        }
    }
}

// ---------------------------------------------------------------- the pipelined convolution (k_conv3p)
// One workgroup of 8 waves per CU, persistent over 16 x 32-pixel output tiles (a wave: 8 x 8 pixels, the
// fragments and epilogue of k_conv3), for layers with 4 n-tiles (49..64 output channels).  A stage = one
// (tile, channel chunk): its halo image and its B fragments go global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: no staging registers, no ds_write pass) into one of two stage buffers, and the
// next stage's DMA is in flight across the barriers while the MFMAs run on this one -- across tile
// boundaries too, so no tile waits for its first chunk.  Per stage: issue stage s + 1; counted
// `s_waitcnt vmcnt` (this wave's part of stage s has landed; stage s + 1's loads stay in flight); raw
// s_barrier (every wave's part has); MFMAs; raw s_barrier (the buffer may be refilled).  Never
// __syncthreads(): its fence would drain the DMA in flight.
// LDS-DMA writes 64 lanes x 16 B contiguously per instruction, so the halo image is slot-linear: 16-B slot q
// of a stage holds halo pixel (hr, hc), 16-B part s chosen by q's byte offset in a pitched image --
// 64-B pixels at a 2208-B row pitch (32-channel chunks), 32-B pixels at 1152 B (16-channel chunks), pitches
// at which every fragment read is bank-conflict free (scripts/dn_lds_layout.py); the pad slots load zeros.
constexpr int kPTH = 16, kPTW = 32;                     // output tile rows x columns
constexpr int kPHH = kPTH + 2, kPHW = kPTW + 2;         // halo 18 x 34
constexpr int kPPitch32 = 2208, kPPitch16 = 1152;
constexpr int kPHalo32 = (kPHH - 1) * kPPitch32 + kPHW * 64;   // 39712 B
constexpr int kPHalo16 = (kPHH - 1) * kPPitch16 + kPHW * 32;   // 20672 B
constexpr int kPThreads = 512;
// stage buffer: the 32-channel halo image, then the chunk's B fragments (k-step-major, NT KB per k-step)
template <int NT> struct PCfg {
    static constexpr int kBuf = kPHalo32 + 9 * NT * 1024;
    // LDS-DMA instructions wave 7 (the wave with the fewest) issues for n slots: it skips the last round when
    // that round's slots run out before its lanes
    static constexpr int cnt7(int n) { return n > 448 ? (n - 448 + kPThreads - 1) / kPThreads : 0; }
    // s_waitcnt vmcnt count that retires stage s while stage s + 1 (32- or 16-channel) stays in flight
    static constexpr int kWait32 = cnt7(kPHalo32 / 16) + cnt7(9 * NT * 64);
    static constexpr int kWait16 = cnt7(kPHalo16 / 16) + cnt7(5 * NT * 64);
    static_assert(2 * kBuf <= 163840, "two stage buffers fit the CU's LDS");
    static_assert(kPTH * kPTW * (NT * 16 + 8) * 2 <= kBuf, "the epilogue's image fits a stage buffer");
};
static_assert(PCfg<4>::kWait32 == 8 && PCfg<4>::kWait16 == 4, "vmcnt counts");

__device__ __forceinline__ void glds16(const void* g, uint8_t* l) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

struct PTile { int tx0, ty0; };
__device__ __forceinline__ PTile ptile(const ConvArgs& a, int t) {
    const int tw = (a.w_ + kPTW - 1) / kPTW;
    const int ty = t / tw;
    return PTile{(t - ty * tw) * kPTW, ty * kPTH};
}

// timing ablations of k_conv3p (wrong results; analysis builds only): bit 0 skips the B fragments' DMA after the
// first stage, bit 1 the halo's
#ifndef RS_DNP_ABLATE
#define RS_DNP_ABLATE 0
#endif
// LDS-DMA of stage (tile t, chunk c) into buffer `buf`
template <int NT>
__device__ __forceinline__ void pstage_issue(const ConvArgs& a, int t, int c, uint8_t* buf, bool first = true) {
    const PTile T = ptile(a, t);
    const int tid = (int)threadIdx.x, wv = tid >> 6;
    const int s = a.ch_src[c];
    const bool w32 = a.ch_w[c] == 32;
    const _Float16* src = a.src[s];
    const int cs = a.cs[s], sh = a.sh[s], sw = a.sw[s], up = a.up[s], base = a.ch_base[c];
    const int nh = (w32 ? kPHalo32 : kPHalo16) / 16;
#pragma unroll
    for (int r = 0; r < (kPHalo32 / 16 + kPThreads - 1) / kPThreads; ++r) {
        if ((RS_DNP_ABLATE & 2) && !first) break;
        int q = r * kPThreads + tid;
        asm volatile("" : "+v"(q));                    // recomputed per stage: hoisted, the slot maps spill
        if (r * kPThreads + wv * 64 < nh) {                // the wave has slots in this round
            const int o = q * 16;
            int hr, hc, sl;
            if (w32) { hr = o / kPPitch32; const int rem = o - hr * kPPitch32; hc = rem >> 6; sl = (rem >> 4) & 3; }
            else { hr = o / kPPitch16; const int rem = o - hr * kPPitch16; hc = rem >> 5; sl = (rem >> 4) & 1; }
            int y = T.ty0 - 1 + hr, x = T.tx0 - 1 + hc;
            if (up) { y >>= 1; x >>= 1; }              // arithmetic: -1 stays -1 (the border)
            size_t px = 0;                             // pixel 0 = the zero border
            if (hc < kPHW && y <= sh && x <= sw) px = (size_t)(y + 1) * (size_t)(sw + 2) + (size_t)(x + 1);
            if (q < nh)                                // lanes past the image would write the B fragments
                glds16(src + px * cs + base + 8 * sl, buf + r * (kPThreads * 16) + wv * 1024);
        }
    }
    const int nst = w32 ? 9 : 5, nb = nst * NT * 64;
    const uint4* w = (const uint4*)a.w + (size_t)a.ch_step[c] * NT * 64;
    uint8_t* bb = buf + kPHalo32;
#pragma unroll
    for (int r = 0; r < (9 * NT * 64 + kPThreads - 1) / kPThreads; ++r) {
        if ((RS_DNP_ABLATE & 1) && !first) break;
        int q = r * kPThreads + tid;
        asm volatile("" : "+v"(q));
        if (r * kPThreads + wv * 64 < nb) glds16(w + (q < nb ? q : 0), bb + r * (kPThreads * 16) + wv * 1024);
    }
}

// MFMAs of one stage: chunk c's k-steps over the halo image and B fragments in `buf`
template <int NT>
__device__ __forceinline__ void pstage_compute(const ConvArgs& a, int c, const uint8_t* buf, f32x4 (&acc)[4][NT],
                                               int lane, int X, int Yb) {
    const int h = lane >> 4;
    const half8* bp = (const half8*)(buf + kPHalo32) + lane;
    if (a.ch_w[c] == 32) {
        const uint8_t* ab = buf + Yb * kPPitch32 + X * 64 + h * 16;
        for (int st = 0; st < 9; ++st) {
            const int ky = st / 3, kx = st - 3 * ky;
            half8 b[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n) b[n] = bp[(st * NT + n) * 64];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const half8 av = *(const half8*)(ab + (2 * g + ky) * kPPitch32 + kx * 64);
#pragma unroll
                for (int n = 0; n < NT; ++n) acc[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b[n], acc[g][n], 0, 0, 0);
            }
        }
    } else {
        const uint8_t* ab = buf + Yb * kPPitch16 + X * 32 + (h & 1) * 16;
        for (int st = 0; st < 5; ++st) {
            int tap = 2 * st + (h >> 1);
            tap = tap > 8 ? 8 : tap;                   // tap 9: zero weights
            const int ky = tap / 3, kx = tap - 3 * ky;
            half8 b[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n) b[n] = bp[(st * NT + n) * 64];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const half8 av = *(const half8*)(ab + (2 * g + ky) * kPPitch16 + kx * 32);
#pragma unroll
                for (int n = 0; n < NT; ++n) acc[g][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b[n], acc[g][n], 0, 0, 0);
            }
        }
    }
}

// a workgroup barrier that is not a fence (no vmcnt(0): the DMA in flight stays in flight); the empty asm
// keeps the compiler from moving LDS accesses across it
__device__ __forceinline__ void raw_barrier() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
}

template <int NT, int POST, bool RELU>
__global__ void __launch_bounds__(kPThreads) k_conv3p(ConvArgs a) {
    using C = PCfg<NT>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * C::kBuf];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wy = wv >> 2, wx = wv & 3;
    const int i = lane & 15, h = lane >> 4;
    const int X = 8 * wx + 2 * (i >> 2) + (i & 1);
    const int Yb = 8 * wy + ((i >> 1) & 1);
    const int ntiles = ((a.w_ + kPTW - 1) / kPTW) * ((a.h + kPTH - 1) / kPTH);
    int t = blockIdx.x, c = 0, b = 0;
    if (t >= ntiles) return;
    float bv[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        bv[n] = a.bias[16 * n + i];
        asm volatile("" : "+v"(bv[n]));                // loaded before the first DMA is issued
    }
    f32x4 acc[4][NT];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[g][n] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    pstage_issue<NT>(a, t, 0, lds);
    for (;;) {
        int tn = t, cn = c + 1;
        if (cn == a.nchunk) { cn = 0; tn = t + (int)gridDim.x; }
        const bool more = tn < ntiles;
        if (more) {
            pstage_issue<NT>(a, tn, cn, lds + (b ^ 1) * C::kBuf, RS_DNP_ABLATE == 0);
            if (RS_DNP_ABLATE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else if (a.ch_w[cn] == 32) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::kWait32) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::kWait16) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        raw_barrier();                                 // every wave's part of stage (t, c) has landed
        uint8_t* buf = lds + b * C::kBuf;
        pstage_compute<NT>(a, c, buf, acc, lane, X, Yb);
        if (cn == 0 || !more) {                        // tile t done: bias, ReLU (, pool), f16 through LDS, 16-B stores
            const PTile T = ptile(a, t);
            constexpr int CP = NT * 16 + 8;            // LDS image pixel pitch (halves): k_conv3's epilogue
            constexpr bool pool = POST == POST_POOL;
            constexpr int OW = pool ? kPTW / 2 : kPTW, NPX = pool ? kPTH * kPTW / 4 : kPTH * kPTW;
            _Float16* o = (_Float16*)buf;
            lds_barrier();                             // every wave's MFMAs have read the stage
#pragma unroll
            for (int n = 0; n < NT; ++n)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    if constexpr (pool) {
                        const f32x4 v4 = acc[g][n];
                        float m = fmaxf(fmaxf(v4[0], v4[1]), fmaxf(v4[2], v4[3])) + bv[n];
                        if (RELU) m = m > 0.0f ? m : 0.0f;
                        o[((4 * wy + g) * OW + 4 * wx + h) * CP + 16 * n + i] = (_Float16)m;
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            float v = acc[g][n][r] + bv[n];
                            if (RELU) v = v > 0.0f ? v : 0.0f;
                            o[((8 * wy + 2 * g + (r >> 1)) * OW + 8 * wx + 2 * h + (r & 1)) * CP + 16 * n + i] = (_Float16)v;
                        }
                    }
                    acc[g][n] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                }
            lds_barrier();
            // the image's LDS reads in asm: before a compiler-visible ds_read the compiler waits vmcnt(0) --
            // for the next stage's DMA and for every store issued before it
            constexpr int PPP = NT * 2, NQ = NPX * PPP, NK = (NQ + kPThreads - 1) / kPThreads;
            const int oh = pool ? a.h >> 1 : a.h, ow = pool ? a.w_ >> 1 : a.w_;
            const int oy0 = pool ? T.ty0 >> 1 : T.ty0, ox0 = pool ? T.tx0 >> 1 : T.tx0;
            uint4 ov[NK];
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int q = (int)threadIdx.x + k * kPThreads;
                const int px = q / PPP, pc = q - px * PPP;
                const uint32_t la = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(o + px * CP + 8 * pc);
                if (NQ % kPThreads == 0 || q < NQ) asm volatile("ds_read_b128 %0, %1" : "=v"(ov[k]) : "v"(la) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int q = (int)threadIdx.x + k * kPThreads;
                const int px = q / PPP, pc = q - px * PPP;
                const int gy = oy0 + px / OW, gx = ox0 + px % OW;
                if ((NQ % kPThreads == 0 || q < NQ) && gy < oh && gx < ow)
                    *(uint4*)(a.dst + ((size_t)(gy + 1) * (size_t)(ow + 2) + (size_t)(gx + 1)) * a.dcs + 8 * pc) = ov[k];
            }
        }
        if (!more) break;
        lds_barrier();                                 // the buffer may be refilled
        t = tn; c = cn; b ^= 1;
    }
}

// ---------------------------------------------------------------- input transform + auto-exposure
struct InArgs {
    const float* color; const float* albedo; const float* normal;
    int cst, ast, nst;         // floats per pixel of each image
    int H, W, Hp, Wp, ic;
    const float* scale;
    float norm;                // NORM_SCALE
    _Float16* in;              // (Hp + 2) x (Wp + 2) x 16
};
__device__ __forceinline__ float clampf(float x, float lo, float hi) {
    x = x == x ? x : 0.0f;                        // NaN -> 0
    return x < lo ? lo : (x > hi ? hi : x);
}
__global__ void __launch_bounds__(256) k_dn_input(InArgs a) {
    const size_t p = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= (size_t)a.Hp * a.Wp) return;
    const int y = (int)(p / a.Wp), x = (int)(p - (size_t)y * a.Wp);
    _Float16 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = (_Float16)0.0f;
    if (y < a.H && x < a.W) {
        const size_t q = (size_t)y * a.W + x;
        const float s = *a.scale;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            float c = a.color[q * a.cst + k];
            c = clampf((c == c ? c : 0.0f) * s, 0.0f, HDR_Y_MAX);
            v[k] = (_Float16)(pu_forward(c) * a.norm);
        }
        if (a.ic >= 6)
#pragma unroll
            for (int k = 0; k < 3; ++k) v[3 + k] = (_Float16)clampf(a.albedo[q * a.ast + k], 0.0f, 1.0f);
        if (a.ic >= 9)
#pragma unroll
            for (int k = 0; k < 3; ++k) v[6 + k] = (_Float16)(clampf(a.normal[q * a.nst + k], -1.0f, 1.0f) * 0.5f + 0.5f);
    }
    uint4* d = (uint4*)(a.in + ((size_t)(y + 1) * (size_t)(a.Wp + 2) + (size_t)(x + 1)) * 16);
    d[0] = *(const uint4*)&v[0];
    d[1] = *(const uint4*)&v[8];
}

// bins of <= 16x16 pixels: mean luminance -> log2 (NaN marks a bin at or below eps)
__global__ void __launch_bounds__(256) k_dn_ae_bins(const float* color, int cst, int H, int W, int nbh, int nbw,
                                                      float* binlog) {
    __shared__ float s[256];
    const int b = blockIdx.x, bi = b / nbw, bj = b - bi * nbw;
    const int y0 = (int)((long long)bi * H / nbh), y1 = (int)((long long)(bi + 1) * H / nbh);
    const int x0 = (int)((long long)bj * W / nbw), x1 = (int)((long long)(bj + 1) * W / nbw);
    const int bw = x1 - x0, n = (y1 - y0) * bw;
    const int t = threadIdx.x;
    float L = 0.0f;
    if (t < n) {
        const size_t q = (size_t)(y0 + t / bw) * W + (x0 + t % bw);
        const float* c = color + q * cst;
        L = 0.212671f * c[0] + 0.715160f * c[1] + 0.072169f * c[2];
    }
    s[t] = L;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) s[t] += s[t + w];
        __syncthreads();
    }
    if (t == 0) {
        const float m = s[0] / (float)n;
        binlog[b] = m > 1e-8f ? log2f(m) : __builtin_nanf("");
    }
}
__global__ void __launch_bounds__(1024) k_dn_ae_final(const float* binlog, int nb, float* scale) {
    __shared__ float s[1024];
    __shared__ int cn[1024];
    const int t = threadIdx.x;
    float a = 0.0f;
    int c = 0;
    for (int b = t; b < nb; b += 1024) {
        const float v = binlog[b];
        if (v == v) { a += v; ++c; }
    }
    s[t] = a; cn[t] = c;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if (t < w) { s[t] += s[t + w]; cn[t] += cn[t + w]; }
        __syncthreads();
    }
    if (t == 0) *scale = cn[0] > 0 ? 0.18f / exp2f(s[0] / (float)cn[0]) : 1.0f;
}
__global__ void k_dn_set(float* p, float v) { *p = v; }

// ---------------------------------------------------------------- host: weights
struct Tensor { std::vector<int> shape; std::vector<float> data; };

static float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    uint32_t f;
    if (e == 0) {
        if (m == 0) f = s;
        else {                                     // subnormal
            int k = -1; uint32_t mm = m;
            do { ++k; mm <<= 1; } while (!(mm & 0x400));
            f = s | ((uint32_t)(127 - 15 - k) << 23) | ((mm & 0x3ff) << 13);
        }
    } else if (e == 31) f = s | 0x7f800000u | (m << 13);
    else f = s | ((e - 15 + 127) << 23) | (m << 13);
    float out;
    std::memcpy(&out, &f, 4);
    return out;
}

// OIDN tensor archive (restir_amd/tza.py documents the layout)
static bool parse_tza(const uint8_t* p, size_t n, std::map<std::string, Tensor>& out, std::string& err) {
    auto rd = [&](size_t off, void* dst, size_t k) -> bool {
        if (off + k > n || off + k < off) return false;
        std::memcpy(dst, p + off, k);
        return true;
    };
    uint16_t magic = 0; uint8_t major = 0; uint64_t table = 0;
    if (!rd(0, &magic, 2) || !rd(2, &major, 1) || !rd(4, &table, 8)) { err = "truncated header"; return false; }
    if (magic != 0x41D7) { err = "bad magic (not a tensor archive)"; return false; }
    if (major != 2) { err = "unsupported tensor archive version " + std::to_string(major); return false; }
    uint32_t cnt = 0;
    if (!rd(table, &cnt, 4)) { err = "table offset out of range"; return false; }
    size_t q = table + 4;
    for (uint32_t t = 0; t < cnt; ++t) {
        uint16_t ln = 0;
        if (!rd(q, &ln, 2) || q + 2 + ln > n) { err = "truncated tensor table"; return false; }
        std::string name((const char*)p + q + 2, ln);
        q += 2 + ln;
        uint8_t nd = 0;
        if (!rd(q, &nd, 1)) { err = "truncated tensor table"; return false; }
        q += 1;
        Tensor T;
        size_t elems = 1;
        for (int d = 0; d < nd; ++d) {
            uint32_t v = 0;
            if (!rd(q, &v, 4)) { err = "truncated tensor table"; return false; }
            q += 4;
            T.shape.push_back((int)v);
            elems *= v;
        }
        q += nd;                                   // layout characters
        char dt = 0; uint64_t off = 0;
        if (!rd(q, &dt, 1) || !rd(q + 1, &off, 8)) { err = "truncated tensor table"; return false; }
        q += 9;
        const size_t es = dt == 'f' ? 4 : dt == 'h' ? 2 : 0;
        if (!es) { err = "tensor " + name + ": unsupported data type"; return false; }
        if (elems > (1u << 28) || off + elems * es > n || off + elems * es < off) { err = "tensor " + name + " out of range"; return false; }
        T.data.resize(elems);
        if (dt == 'f') std::memcpy(T.data.data(), p + off, elems * 4);
        else for (size_t e = 0; e < elems; ++e) { uint16_t hv; std::memcpy(&hv, p + off + 2 * e, 2); T.data[e] = half_to_float(hv); }
        out[name] = std::move(T);
    }
    return true;
}

enum BufId { B_IN, B_E0, B_P1, B_P2, B_P3, B_P4, B_E5A, B_E5B, B_D4A, B_D4B, B_D3A, B_D3B, B_D2A, B_D2B, B_D1A, B_D1B, B_COUNT };
struct LayerDef { const char* name; int src0, up0, src1, level, post, relu, dst; };
static const LayerDef kNet[16] = {
    {"enc_conv0", B_IN, 0, -1, 0, POST_STORE, 1, B_E0},
    {"enc_conv1", B_E0, 0, -1, 0, POST_POOL, 1, B_P1},
    {"enc_conv2", B_P1, 0, -1, 1, POST_POOL, 1, B_P2},
    {"enc_conv3", B_P2, 0, -1, 2, POST_POOL, 1, B_P3},
    {"enc_conv4", B_P3, 0, -1, 3, POST_POOL, 1, B_P4},
    {"enc_conv5a", B_P4, 0, -1, 4, POST_STORE, 1, B_E5A},
    {"enc_conv5b", B_E5A, 0, -1, 4, POST_STORE, 1, B_E5B},
    {"dec_conv4a", B_E5B, 1, B_P3, 3, POST_STORE, 1, B_D4A},
    {"dec_conv4b", B_D4A, 0, -1, 3, POST_STORE, 1, B_D4B},
    {"dec_conv3a", B_D4B, 1, B_P2, 2, POST_STORE, 1, B_D3A},
    {"dec_conv3b", B_D3A, 0, -1, 2, POST_STORE, 1, B_D3B},
    {"dec_conv2a", B_D3B, 1, B_P1, 1, POST_STORE, 1, B_D2A},
    {"dec_conv2b", B_D2A, 0, -1, 1, POST_STORE, 1, B_D2B},
    {"dec_conv1a", B_D2B, 1, B_IN, 0, POST_STORE, 1, B_D1A},
    {"dec_conv1b", B_D1A, 0, -1, 0, POST_STORE, 1, B_D1B},
    {"dec_conv0", B_D1B, 0, -1, 0, POST_FINAL, 0, -1},
};

struct Chunk { int src, base, w, step; };
struct Layer {
    int co = 0, nt = 0, nsteps = 0;
    int ci[2] = {0, 0};
    std::vector<Chunk> chunks;
    half8* dw = nullptr;
    float* db = nullptr;
};

struct Net {
    int ic = 0;
    int co[16] = {};
    int bufc[B_COUNT] = {};        // real channels of each tensor
    int bufcs[B_COUNT] = {};       // channel stride (multiple of 16)
    int buflev[B_COUNT] = {};
    uint64_t params = 0;
    double mac_per_px = 0.0;       // at the network's input resolution (padded)
};

static int round16(int c) { return (c + 15) / 16 * 16; }

// topology check of the archive against OIDN's UNet; fills channel counts
static bool check_net(const std::map<std::string, Tensor>& T, Net& net, std::string& err) {
    for (int l = 0; l < 16; ++l) {
        const std::string n = kNet[l].name;
        auto w = T.find(n + ".weight"), b = T.find(n + ".bias");
        if (w == T.end() || b == T.end()) { err = "missing tensor " + n + (w == T.end() ? ".weight" : ".bias"); return false; }
        const auto& s = w->second.shape;
        if (s.size() != 4 || s[2] != 3 || s[3] != 3) { err = n + ".weight: expected (O, I, 3, 3)"; return false; }
        if (b->second.shape.size() != 1 || b->second.shape[0] != s[0]) { err = n + ".bias: expected (O)"; return false; }
        if (s[0] < 1 || s[0] > 128) { err = n + ": output channels outside 1..128"; return false; }
        net.co[l] = s[0];
    }
    net.ic = T.at("enc_conv0.weight").shape[1];
    if (net.ic != 3 && net.ic != 6 && net.ic != 9) { err = "enc_conv0: input channels must be 3, 6 or 9"; return false; }
    net.bufc[B_IN] = net.ic;
    net.buflev[B_IN] = 0;
    for (int l = 0; l < 15; ++l) {
        net.bufc[kNet[l].dst] = net.co[l];
        net.buflev[kNet[l].dst] = kNet[l].level + (kNet[l].post == POST_POOL ? 1 : 0);
    }
    if (net.co[15] != 3) { err = "dec_conv0: expected 3 output channels"; return false; }
    net.params = 0;
    net.mac_per_px = 0.0;
    for (int l = 0; l < 16; ++l) {
        const int need = net.bufc[kNet[l].src0] + (kNet[l].src1 >= 0 ? net.bufc[kNet[l].src1] : 0);
        const int got = T.at(std::string(kNet[l].name) + ".weight").shape[1];
        if (got != need) {
            err = std::string(kNet[l].name) + ": " + std::to_string(got) + " input channels, the UNet feeds it " + std::to_string(need);
            return false;
        }
        net.params += (uint64_t)net.co[l] * got * 9 + net.co[l];
        net.mac_per_px += (double)net.co[l] * got * 9 / (double)(1 << (2 * kNet[l].level));
    }
    for (int b = 0; b < B_COUNT; ++b) net.bufcs[b] = round16(net.bufc[b]);
    return true;
}

// B fragments: for k-step s of chunk (src, base, w) and n-tile n, lane l holds 8 halves
//   w = 32: tap s,               channels base + 8 (l >> 4) + j
//   w = 16: tap 2 s + (l >> 5),  channels base + 8 ((l >> 4) & 1) + j   (tap 9: zero)
// of output channel 16 n + (l & 15)  -- the same k order the kernel's A fragments read
static void pack_layer(const Tensor& W, const Tensor& B, const Net& net, int l, Layer& L, std::vector<_Float16>& wout,
                       std::vector<float>& bout) {
    const LayerDef& d = kNet[l];
    L.co = net.co[l];
    L.nt = (L.co + 15) / 16;
    const int srcs[2] = {d.src0, d.src1};
    const int ci_total = W.shape[1];
    L.chunks.clear();
    int step = 0;
    for (int s = 0; s < 2; ++s) {
        if (srcs[s] < 0) continue;
        L.ci[s] = net.bufc[srcs[s]];
        const int cs = net.bufcs[srcs[s]];
        for (int base = 0; base < cs;) {
            const int w = cs - base >= 32 ? 32 : 16;
            L.chunks.push_back({s, base, w, step});
            step += w == 32 ? 9 : 5;
            base += w;
        }
    }
    L.nsteps = step;
    wout.assign((size_t)step * L.nt * 64 * 8, (_Float16)0.0f);
    for (const Chunk& ch : L.chunks) {
        const int nst = ch.w == 32 ? 9 : 5;
        const int coff = ch.src == 0 ? 0 : L.ci[0];
        for (int st = 0; st < nst; ++st)
            for (int n = 0; n < L.nt; ++n)
                for (int ln = 0; ln < 64; ++ln)
                    for (int j = 0; j < 8; ++j) {
                        const int hh = ln >> 4, co = 16 * n + (ln & 15);
                        int tap, c;
                        if (ch.w == 32) { tap = st; c = ch.base + 8 * hh + j; }
                        else { tap = 2 * st + (hh >> 1); c = ch.base + 8 * (hh & 1) + j; }
                        float v = 0.0f;
                        if (tap <= 8 && co < L.co && c < L.ci[ch.src])
                            v = W.data[(((size_t)co * ci_total + coff + c) * 3 + tap / 3) * 3 + tap % 3];
                        wout[((((size_t)(ch.step + st) * L.nt + n) * 64 + ln) * 8) + j] = (_Float16)v;
                    }
    }
    bout.assign((size_t)L.nt * 16, 0.0f);
    for (int co = 0; co < L.co; ++co) bout[co] = B.data[co];
}

}  // namespace dn
}  // namespace rs

using namespace rs::dn;

struct rs_denoiser {
    rs_context* ctx = nullptr;                  // null once the context is destroyed (rs::denoiser_detach)
    int device = 0;
    Net net;
    Layer L[16];
    // activation tensors for the current image size
    int H = 0, W = 0, Hp = 0, Wp = 0;
    _Float16* buf[B_COUNT] = {};
    float* d_scale = nullptr;
    float* d_binlog = nullptr;
    int binlog_cap = 0;
    float* d_out = nullptr;                     // rs_denoise_frame's output (W*H float3)
    int out_w = 0, out_h = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t evl[17] = {};                    // timed: after the input transform, after each convolution
    bool timed = false;
    uint32_t pipe = 0u;                         // layers (bit l) on k_conv3p where it applies (2..4 n-tiles):
                                                // RESTIR_DN_PIPE=<mask> or 1 (all); measured slower, off
    int cus = 256;                              // its workgroups (RESTIR_DN_PIPE_GRID caps them: tests)
};

namespace {
int dfail(rs_denoiser* d, int code, const std::string& m) { return rs::ctx_fail(d ? d->ctx : nullptr, code, m); }
#define DCHK(d, x)                                                                                   \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) return dfail((d), RS_E_HIP, std::string(#x " -> ") + hipGetErrorString(e_)); \
    } while (0)

void free_bufs(rs_denoiser* d) {
    for (auto& b : d->buf) { if (b) hipFree(b); b = nullptr; }
    d->H = d->W = d->Hp = d->Wp = 0;
}

int ensure_bufs(rs_denoiser* d, int H, int W, hipStream_t st) {
    if (H == d->H && W == d->W) return RS_OK;
    free_bufs(d);
    const int Hp = (H + 15) / 16 * 16, Wp = (W + 15) / 16 * 16;
    for (int b = 0; b < B_COUNT; ++b) {
        const int lv = d->net.buflev[b];
        const size_t bytes = (size_t)((Hp >> lv) + 2) * (size_t)((Wp >> lv) + 2) * d->net.bufcs[b] * 2;
        DCHK(d, hipMalloc(&d->buf[b], bytes));
        DCHK(d, hipMemsetAsync(d->buf[b], 0, bytes, st));    // zero borders (never written afterwards)
    }
    const int nb = ((H + 15) / 16) * ((W + 15) / 16);
    if (nb > d->binlog_cap) {
        if (d->d_binlog) hipFree(d->d_binlog);
        DCHK(d, hipMalloc(&d->d_binlog, (size_t)nb * sizeof(float)));
        d->binlog_cap = nb;
    }
    d->H = H; d->W = W; d->Hp = Hp; d->Wp = Wp;
    return RS_OK;
}

template <int NT, int POST, bool RELU>
void launch(const ConvArgs& a, dim3 g, hipStream_t st) { k_conv3<NT, POST, RELU><<<g, 256, 0, st>>>(a); }

bool dispatch(int nt, int post, bool relu, const ConvArgs& a, dim3 g, hipStream_t st) {
#define RS_DN_CASE(N)                                                       \
    case N:                                                                 \
        if (post == POST_POOL) launch<N, POST_POOL, true>(a, g, st);        \
        else if (relu) launch<N, POST_STORE, true>(a, g, st);              \
        else launch<N, POST_STORE, false>(a, g, st);                       \
        return true;
    if (post == POST_FINAL) {
        if (nt != 1) return false;
        launch<1, POST_FINAL, false>(a, g, st);
        return true;
    }
    switch (nt) {
        RS_DN_CASE(1) RS_DN_CASE(2) RS_DN_CASE(3) RS_DN_CASE(4)
        default: return false;
    }
#undef RS_DN_CASE
}

bool dispatch_pipe(int nt, int post, bool relu, const ConvArgs& a, dim3 g, hipStream_t st) {
#define RS_DNP_CASE(N)                                                                          \
    case N:                                                                                     \
        if (post == POST_POOL) k_conv3p<N, POST_POOL, true><<<g, kPThreads, 0, st>>>(a);        \
        else if (relu) k_conv3p<N, POST_STORE, true><<<g, kPThreads, 0, st>>>(a);              \
        else k_conv3p<N, POST_STORE, false><<<g, kPThreads, 0, st>>>(a);                       \
        return true;
    if (post == POST_POOL && !relu) return false;
    switch (nt) {
        RS_DNP_CASE(2) RS_DNP_CASE(3) RS_DNP_CASE(4)
        default: return false;
    }
#undef RS_DNP_CASE
}

int create_impl(rs_context* ctx, const void* tza, size_t bytes, rs_denoiser** out) {
    if (!ctx || !tza || !out) return rs::ctx_fail(ctx, RS_E_INVALID, "rs_denoiser_create: null argument");
    *out = nullptr;
    std::map<std::string, Tensor> T;
    std::string err;
    if (!parse_tza((const uint8_t*)tza, bytes, T, err)) return rs::ctx_fail(ctx, RS_E_INVALID, "rs_denoiser_create: " + err);
    rs_denoiser* d = new rs_denoiser();
    d->ctx = ctx;
    d->device = rs::ctx_device(ctx);
    if (const char* e = std::getenv("RESTIR_DN_PIPE")) d->pipe = std::strcmp(e, "1") == 0 ? 0xffffu : (uint32_t)std::strtoul(e, nullptr, 0);
    if (hipDeviceGetAttribute(&d->cus, hipDeviceAttributeMultiprocessorCount, d->device) != hipSuccess || d->cus < 1) d->cus = 256;
    if (const char* e = std::getenv("RESTIR_DN_PIPE_GRID")) d->cus = std::max(1, std::atoi(e));
    if (!check_net(T, d->net, err)) { delete d; return rs::ctx_fail(ctx, RS_E_INVALID, "rs_denoiser_create: " + err); }
    (void)hipGetLastError();
    if (hipSetDevice(rs::ctx_device(ctx)) != hipSuccess) { delete d; return rs::ctx_fail(ctx, RS_E_HIP, "rs_denoiser_create: hipSetDevice"); }
    hipStream_t st = rs::ctx_stream(ctx);
    int rc = RS_OK;
    for (int l = 0; l < 16 && rc == RS_OK; ++l) {
        std::vector<_Float16> w;
        std::vector<float> b;
        pack_layer(T.at(std::string(kNet[l].name) + ".weight"), T.at(std::string(kNet[l].name) + ".bias"), d->net, l, d->L[l], w, b);
        if ((int)d->L[l].chunks.size() > kMaxChunks) { rc = rs::ctx_fail(ctx, RS_E_INVALID, "rs_denoiser_create: too many input channels"); break; }
        if (hipMalloc(&d->L[l].dw, w.size() * 2) != hipSuccess || hipMalloc(&d->L[l].db, b.size() * 4) != hipSuccess ||
            hipMemcpyAsync(d->L[l].dw, w.data(), w.size() * 2, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d->L[l].db, b.data(), b.size() * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = rs::ctx_fail(ctx, RS_E_HIP, "rs_denoiser_create: weight upload failed");
    }
    if (rc == RS_OK && (hipMalloc(&d->d_scale, sizeof(float)) != hipSuccess || hipEventCreate(&d->ev0) != hipSuccess ||
                        hipEventCreate(&d->ev1) != hipSuccess))
        rc = rs::ctx_fail(ctx, RS_E_HIP, "rs_denoiser_create: allocation failed");
    for (auto& e : d->evl)
        if (rc == RS_OK && hipEventCreate(&e) != hipSuccess) rc = rs::ctx_fail(ctx, RS_E_HIP, "rs_denoiser_create: event");
    if (rc != RS_OK) { rs_denoiser_destroy(d); return rc; }
    rs::ctx_track_denoiser(ctx, d, true);
    *out = d;
    return RS_OK;
}
}  // namespace

namespace rs {
// the filter on device images (float3 rows at the given strides), enqueued on `st`
int denoise_run(rs_denoiser* d, hipStream_t st, const float* color, int cst, const float* albedo, int ast,
                const float* normal, int nst, float* out, int ost, int H, int W, float input_scale) {
    if (!d || !color || !out) return dfail(d, RS_E_INVALID, "rs_denoise: null image");
    if (!d->ctx) return dfail(d, RS_E_INVALID, "rs_denoise: the denoiser's context was destroyed");
    if (H <= 0 || W <= 0) return dfail(d, RS_E_INVALID, "rs_denoise: empty image");
    if (d->net.ic >= 6 && !albedo) return dfail(d, RS_E_INVALID, "rs_denoise: the weights need an albedo image");
    if (d->net.ic >= 9 && !normal) return dfail(d, RS_E_INVALID, "rs_denoise: the weights need a normal image");
    (void)hipGetLastError();
    DCHK(d, hipSetDevice(ctx_device(d->ctx)));
    int rc = ensure_bufs(d, H, W, st);
    if (rc != RS_OK) return rc;
    if (d->timed) DCHK(d, hipEventRecord(d->ev0, st));
    // input scale: auto-exposure unless given
    if (std::isfinite(input_scale) && input_scale > 0.0f) {
        k_dn_set<<<1, 1, 0, st>>>(d->d_scale, input_scale);
    } else {
        const int nbh = (H + 15) / 16, nbw = (W + 15) / 16;
        k_dn_ae_bins<<<nbh * nbw, 256, 0, st>>>(color, cst, H, W, nbh, nbw, d->d_binlog);
        k_dn_ae_final<<<1, 1024, 0, st>>>(d->d_binlog, nbh * nbw, d->d_scale);
    }
    const float norm = 1.0f / pu_forward(HDR_Y_MAX);
    InArgs ia{color, albedo, normal, cst, ast, nst, H, W, d->Hp, d->Wp, d->net.ic, d->d_scale, norm, d->buf[B_IN]};
    const size_t npx = (size_t)d->Hp * d->Wp;
    k_dn_input<<<(unsigned)((npx + 255) / 256), 256, 0, st>>>(ia);
    DCHK(d, hipGetLastError());
    if (d->timed) DCHK(d, hipEventRecord(d->evl[0], st));
    for (int l = 0; l < 16; ++l) {
        const LayerDef& ld = kNet[l];
        const Layer& L = d->L[l];
        ConvArgs a{};
        const int srcs[2] = {ld.src0, ld.src1};
        for (int s = 0; s < 2; ++s) {
            if (srcs[s] < 0) continue;
            const int lv = d->net.buflev[srcs[s]];
            a.src[s] = d->buf[srcs[s]];
            a.cs[s] = d->net.bufcs[srcs[s]];
            a.sh[s] = d->Hp >> lv;
            a.sw[s] = d->Wp >> lv;
            a.up[s] = s == 0 ? ld.up0 : 0;
        }
        a.nchunk = (int)L.chunks.size();
        for (int c = 0; c < a.nchunk; ++c) {
            a.ch_src[c] = L.chunks[c].src; a.ch_base[c] = L.chunks[c].base;
            a.ch_w[c] = L.chunks[c].w; a.ch_step[c] = L.chunks[c].step;
        }
        a.w = L.dw; a.bias = L.db;
        a.h = d->Hp >> ld.level; a.w_ = d->Wp >> ld.level;
        if (ld.post != POST_FINAL) { a.dst = d->buf[ld.dst]; a.dcs = d->net.bufcs[ld.dst]; }
        else {
            a.out = out; a.ostride = ost; a.H = H; a.W = W; a.scale = d->d_scale;
            a.inv_norm = pu_forward(HDR_Y_MAX);
        }
        a.nt_total = L.nt;
        if (((d->pipe >> l) & 1u) && ld.post != POST_FINAL && L.nt >= 2 && L.nt <= 4) {
            // one persistent workgroup per CU over 16 x 32 tiles (or one per tile when there are fewer)
            const size_t nt = (size_t)((a.w_ + kPTW - 1) / kPTW) * (size_t)((a.h + kPTH - 1) / kPTH);
            const dim3 g((unsigned)std::min<size_t>(nt, (size_t)d->cus));
            if (!dispatch_pipe(L.nt, ld.post, ld.relu != 0, a, g, st)) return dfail(d, RS_E_UNSUPPORTED, "rs_denoise: unsupported layer");
            DCHK(d, hipGetLastError());
            if (d->timed) DCHK(d, hipEventRecord(d->evl[l + 1], st));
            continue;
        }
        // n-tiles per workgroup: all of them, unless the layer's tiles cannot fill the chip (the coarse
        // levels): then the output channels split over blockIdx.z (each split re-stages the input halo)
        const unsigned gx = (unsigned)((a.w_ + kTile - 1) / kTile), gy = (unsigned)((a.h + kTile - 1) / kTile);
        a.nt_total = L.nt;
        int ntw = 1;
        if (ld.post != POST_FINAL)
            for (int k = L.nt < kMaxNtw ? L.nt : kMaxNtw; k >= 1; --k)
                if (L.nt % k == 0) { ntw = k; if ((size_t)gx * gy * (L.nt / k) >= kFillWorkgroups) break; }
        const dim3 g(gx, gy, (unsigned)(L.nt / ntw));
        if (!dispatch(ntw, ld.post, ld.relu != 0, a, g, st)) return dfail(d, RS_E_UNSUPPORTED, "rs_denoise: unsupported layer width");
        DCHK(d, hipGetLastError());
        if (d->timed) DCHK(d, hipEventRecord(d->evl[l + 1], st));
    }
    if (d->timed) DCHK(d, hipEventRecord(d->ev1, st));
    return RS_OK;
}
}  // namespace rs

// ---------------------------------------------------------------- C ABI
extern "C" int rs_denoiser_check_weights(const void* tza, size_t bytes, rs_denoiser_info* info) {
    if (!tza) return rs::ctx_fail(nullptr, RS_E_INVALID, "rs_denoiser_check_weights: null argument");
    std::map<std::string, Tensor> T;
    std::string err;
    Net net;
    if (!parse_tza((const uint8_t*)tza, bytes, T, err) || !check_net(T, net, err))
        return rs::ctx_fail(nullptr, RS_E_INVALID, "rs_denoiser_check_weights: " + err);
    if (info) {
        std::memset(info, 0, sizeof *info);
        info->input_channels = net.ic;
        for (int l = 0; l < 16; ++l) info->channels[l] = net.co[l];
        info->parameters = net.params;
        info->mac_per_pixel = net.mac_per_px;
    }
    return RS_OK;
}

extern "C" int rs_denoiser_create(rs_context* ctx, const void* tza, size_t bytes, rs_denoiser** out) {
    return create_impl(ctx, tza, bytes, out);
}

extern "C" int rs_denoiser_create_from_file(rs_context* ctx, const char* path, rs_denoiser** out) {
    if (!ctx || !path || !out) return rs::ctx_fail(ctx, RS_E_INVALID, "rs_denoiser_create_from_file: null argument");
    std::FILE* f = std::fopen(path, "rb");
    if (!f) return rs::ctx_fail(ctx, RS_E_IO, std::string("rs_denoiser_create_from_file: cannot open ") + path);
    std::vector<uint8_t> blob;
    uint8_t tmp[1 << 16];
    size_t k;
    while ((k = std::fread(tmp, 1, sizeof tmp, f)) > 0) blob.insert(blob.end(), tmp, tmp + k);
    std::fclose(f);
    return create_impl(ctx, blob.data(), blob.size(), out);
}

extern "C" int rs_denoiser_info_get(const rs_denoiser* d, rs_denoiser_info* info) {
    if (!d || !info) return rs::ctx_fail(d ? d->ctx : nullptr, RS_E_INVALID, "rs_denoiser_info_get: null argument");
    std::memset(info, 0, sizeof *info);
    info->input_channels = d->net.ic;
    for (int l = 0; l < 16; ++l) info->channels[l] = d->net.co[l];
    info->parameters = d->net.params;
    info->mac_per_pixel = d->net.mac_per_px;
    return RS_OK;
}

extern "C" int rs_denoiser_execute(rs_denoiser* d, const float* color, const float* albedo, const float* normal,
                                   float* output, int32_t width, int32_t height, const rs_denoise_params* p) {
    if (!d) return rs::ctx_fail(nullptr, RS_E_INVALID, "rs_denoiser_execute: null denoiser");
    const float scale = p ? p->input_scale : NAN;
    if (p && !p->hdr) return dfail(d, RS_E_UNSUPPORTED, "rs_denoiser_execute: only hdr = true (the reference's setting) is supported");
    if (!d->ctx) return dfail(d, RS_E_INVALID, "rs_denoiser_execute: the denoiser's context was destroyed");
    return rs::denoise_run(d, rs::ctx_stream(d->ctx), color, 3, albedo, 3, normal, 3, output, 3, height, width, scale);
}

extern "C" int rs_denoiser_set_timing(rs_denoiser* d, int enable) {
    if (!d) return rs::ctx_fail(nullptr, RS_E_INVALID, "rs_denoiser_set_timing: null denoiser");
    d->timed = enable != 0;
    return RS_OK;
}

extern "C" int rs_denoiser_last_ms(rs_denoiser* d, float* ms) {
    if (!d || !ms) return rs::ctx_fail(d ? d->ctx : nullptr, RS_E_INVALID, "rs_denoiser_last_ms: null argument");
    if (!d->timed) return dfail(d, RS_E_INVALID, "rs_denoiser_last_ms: timing is off (rs_denoiser_set_timing)");
    DCHK(d, hipEventSynchronize(d->ev1));
    DCHK(d, hipEventElapsedTime(ms, d->ev0, d->ev1));
    return RS_OK;
}

extern "C" int rs_denoiser_layer_ms(rs_denoiser* d, float* ms) {
    if (!d || !ms) return rs::ctx_fail(d ? d->ctx : nullptr, RS_E_INVALID, "rs_denoiser_layer_ms: null argument");
    if (!d->timed) return dfail(d, RS_E_INVALID, "rs_denoiser_layer_ms: timing is off (rs_denoiser_set_timing)");
    DCHK(d, hipEventSynchronize(d->ev1));
    DCHK(d, hipEventElapsedTime(&ms[0], d->ev0, d->evl[0]));
    for (int l = 0; l < 16; ++l) DCHK(d, hipEventElapsedTime(&ms[l + 1], d->evl[l], d->evl[l + 1]));
    return RS_OK;
}

extern "C" int rs_denoiser_get_scale(rs_denoiser* d, float* scale) {
    if (!d || !scale) return rs::ctx_fail(d ? d->ctx : nullptr, RS_E_INVALID, "rs_denoiser_get_scale: null argument");
    if (!d->ctx) return dfail(d, RS_E_INVALID, "rs_denoiser_get_scale: the denoiser's context was destroyed");
    hipStream_t st = rs::ctx_stream(d->ctx);
    DCHK(d, hipMemcpyAsync(scale, d->d_scale, sizeof(float), hipMemcpyDeviceToHost, st));
    DCHK(d, hipStreamSynchronize(st));
    return RS_OK;
}

extern "C" int rs_denoiser_dump(rs_denoiser* d, int tensor, uint16_t* host, int32_t* dims) {
    if (!d || tensor < 0 || tensor >= B_COUNT) return rs::ctx_fail(d ? d->ctx : nullptr, RS_E_INVALID, "rs_denoiser_dump: bad argument");
    if (!d->buf[tensor]) return dfail(d, RS_E_INVALID, "rs_denoiser_dump: nothing executed yet");
    if (!d->ctx) return dfail(d, RS_E_INVALID, "rs_denoiser_dump: the denoiser's context was destroyed");
    const int lv = d->net.buflev[tensor];
    const int h = (d->Hp >> lv) + 2, w = (d->Wp >> lv) + 2, cs = d->net.bufcs[tensor];
    if (dims) { dims[0] = h; dims[1] = w; dims[2] = cs; dims[3] = d->net.bufc[tensor]; }
    if (host) {
        hipStream_t st = rs::ctx_stream(d->ctx);
        DCHK(d, hipMemcpyAsync(host, d->buf[tensor], (size_t)h * w * cs * 2, hipMemcpyDeviceToHost, st));
        DCHK(d, hipStreamSynchronize(st));
    }
    return RS_OK;
}

extern "C" void rs_denoiser_destroy(rs_denoiser* d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    if (d->ctx) {                               // still attached: its work is on the context's stream
        (void)hipStreamSynchronize(rs::ctx_stream(d->ctx));
        rs::ctx_track_denoiser(d->ctx, d, false);
    }                                           // (detached: the context drained its streams when destroyed)
    free_bufs(d);
    for (auto& L : d->L) { if (L.dw) hipFree(L.dw); if (L.db) hipFree(L.db); }
    if (d->d_scale) hipFree(d->d_scale);
    if (d->d_binlog) hipFree(d->d_binlog);
    if (d->d_out) hipFree(d->d_out);
    if (d->ev0) hipEventDestroy(d->ev0);
    if (d->ev1) hipEventDestroy(d->ev1);
    for (auto e : d->evl) if (e) hipEventDestroy(e);
    delete d;
}

namespace rs {
float* denoiser_frame_out(rs_denoiser* d, int W, int H) {
    if (!d->d_out || d->out_w != W || d->out_h != H) {
        if (d->d_out) hipFree(d->d_out);
        d->d_out = nullptr;
        d->out_w = d->out_h = 0;
        if (hipMalloc(&d->d_out, (size_t)W * H * 3 * sizeof(float)) != hipSuccess) return nullptr;
        d->out_w = W; d->out_h = H;
    }
    return d->d_out;
}
rs_context* denoiser_ctx(const rs_denoiser* d) { return d->ctx; }
void denoiser_detach(rs_denoiser* d) { d->ctx = nullptr; }
}  // namespace rs
