// rs_jpeg.cpp -- JPEG decoder for the scene loader's textures (the reference decodes them with FreeImage,
// pg/Texture.cpp:18-30; every texture the reference ships is a JPEG, e.g. data/room/room.mtl:11,21,32).
// ITU-T T.81 Huffman-coded 8-bit JPEG: baseline / extended sequential (SOF0 / SOF1) and progressive (SOF2:
// spectral selection + successive approximation, EOB runs), interleaved and non-interleaved scans, restart
// intervals, any sampling factors up to 4; grey, YCbCr and RGB (Adobe transform 0).  The sample reconstruction
// restates the Independent JPEG Group's published algorithms as libjpeg-turbo runs them by default:
//   * the "islow" integer IDCT (Loeffler-Ligtenberg-Moschytz, 13-bit constants, 2 extra bits in pass 1, the
//     post-IDCT range-limit table's wraparound mask);
//   * "fancy" (triangle-filter) upsampling for 2x1 / 2x2 chroma (h2v1 / h2v2: 3/4 - 1/4 weights, the
//     alternating +8 / +7 rounding, edge rows and columns replicated), box replication for other factors;
//   * YCbCr -> RGB with the 16-bit fixed-point tables (FIX(1.402), FIX(1.772), FIX(0.71414), FIX(0.34414)).
// Pinned bit-exact against PIL's libjpeg-turbo on every JPEG the reference ships and on synthetic files
// (tests/test_image_io.py).  Not supported (RS_E_UNSUPPORTED): arithmetic coding, lossless, 12-bit, CMYK.
#include "rs_image.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <vector>

namespace rs {
namespace {

const int kZigzag[64 + 16] = {   // natural order of zig-zag index k (+16 guard entries, as libjpeg's)
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huff {
    bool defined = false;
    int32_t maxcode[18];
    int32_t valoff[17];
    uint8_t vals[256];
    uint8_t look_len[512], look_val[512];     // 9-bit lookahead
    bool build(const uint8_t* counts, const uint8_t* v, int nv) {
        std::memcpy(vals, v, (size_t)nv);
        int code = 0, k = 0;
        std::memset(look_len, 0, sizeof look_len);
        for (int l = 1; l <= 16; ++l) {
            valoff[l] = k - code;
            for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
                if (code >= (1 << l)) return false;   // over-subscribed: checked before any table write
                if (l <= 9) {
                    const int sh = 9 - l;
                    for (int f = 0; f < (1 << sh); ++f) { look_len[(code << sh) | f] = (uint8_t)l; look_val[(code << sh) | f] = v[k]; }
                }
            }
            maxcode[l] = counts[l - 1] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        defined = true;
        return true;
    }
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0;
    int bw = 0, bh = 0;                         // blocks of the coefficient array (MCU-padded)
    int cw = 0, ch = 0;                         // component samples (ceil(W * h / hmax), ...)
    std::vector<int16_t> coef;                  // bw * bh blocks of 64 coefficients, natural order
    uint16_t q[64] = {};                        // quantisation table latched at the component's first scan
    bool latched = false;
    int dc_pred = 0;
    std::vector<uint8_t> plane;                 // bw * 8 x bh * 8 samples after the IDCT
};

struct Decoder {
    const uint8_t* f;
    size_t n, p = 0;
    std::string err;
    uint16_t qt[4][64] = {};
    bool qt_def[4] = {};
    Huff dc[4], ac[4];
    std::vector<Comp> comp;
    int W = 0, H = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool progressive = false, sof = false;
    int restart = 0;
    bool adobe = false, jfif = false;
    int adobe_transform = -1;
    // entropy bit reader
    uint32_t bitbuf = 0;
    int bitcnt = 0;
    bool hit_marker = false;
    int eobrun = 0;

    bool fail(const std::string& m) { if (err.empty()) err = m; return false; }
    int u8() { return p < n ? f[p++] : -1; }
    int u16() { const int a = u8(), b = u8(); return (a < 0 || b < 0) ? -1 : (a << 8) | b; }

    void fill() {
        while (bitcnt <= 24) {
            int b = 0;
            if (!hit_marker && p < n) {
                b = f[p];
                if (b == 0xFF) {
                    const int nx = p + 1 < n ? f[p + 1] : -1;
                    if (nx == 0x00) p += 2;
                    else { hit_marker = true; b = 0; }    // a marker: feed zeros (libjpeg's behaviour)
                } else {
                    ++p;
                }
            }
            bitbuf |= (uint32_t)b << (24 - bitcnt);
            bitcnt += 8;
        }
    }
    int bits(int k) {                           // k <= 16
        if (k == 0) return 0;
        if (bitcnt < k) fill();
        const int v = (int)(bitbuf >> (32 - k));
        bitbuf <<= k; bitcnt -= k;
        return v;
    }
    int bit() { return bits(1); }
    int decode(const Huff& h) {
        if (bitcnt < 16) fill();
        const int look = (int)(bitbuf >> 23);
        int l = h.look_len[look];
        if (l) { bitbuf <<= l; bitcnt -= l; return h.look_val[look]; }
        int code = (int)(bitbuf >> 23);
        l = 9;
        bitbuf <<= 9; bitcnt -= 9;
        while (code > h.maxcode[l]) {
            code = (code << 1) | bit();
            if (++l > 16) return -1;
        }
        return h.vals[h.valoff[l] + code];
    }
    static int extend(int v, int s) { return s == 0 ? 0 : (v < (1 << (s - 1)) ? v - (1 << s) + 1 : v); }
    int receive_extend(int s) { return extend(bits(s), s); }

    void reset_entropy() {
        bitbuf = 0; bitcnt = 0; hit_marker = false; eobrun = 0;
        for (auto& c : comp) c.dc_pred = 0;
    }
    bool read_restart() {                       // expect RSTn at the entropy data's end
        bitbuf = 0; bitcnt = 0; hit_marker = false;
        while (p + 1 < n && !(f[p] == 0xFF && f[p + 1] >= 0xD0 && f[p + 1] <= 0xD7)) {
            if (f[p] == 0xFF && f[p + 1] != 0x00 && f[p + 1] != 0xFF) break;   // some other marker: resync there
            ++p;
        }
        if (p + 1 < n && f[p] == 0xFF && f[p + 1] >= 0xD0 && f[p + 1] <= 0xD7) p += 2;
        eobrun = 0;
        for (auto& c : comp) c.dc_pred = 0;
        return true;
    }

    bool parse_sof(int marker) {
        const int len = u16();
        if (len < 8) return fail("bad SOF");
        const int prec = u8();
        H = u16(); W = u16();
        const int nc = u8();
        if (prec != 8) return fail("only 8-bit JPEG is supported");
        if (W <= 0 || H <= 0 || W > 65535 || H > 65535) return fail("bad JPEG size");
        // a header of a few bytes must not commit gigabytes: cap the image at 2^28 pixels, and at 4096 pixels
        // per byte of the file (a real entropy stream codes far fewer; an all-DC 8x8 block still takes >= 1 bit)
        if ((uint64_t)W * (uint64_t)H > (1ull << 28) || (uint64_t)W * (uint64_t)H > 4096ull * (uint64_t)n)
            return fail("JPEG size exceeds the decoder's limit");
        if (nc != 1 && nc != 3) return fail("only grey and 3-component JPEG are supported");
        if (len != 8 + 3 * nc) return fail("bad SOF length");
        comp.assign(nc, Comp{});
        for (auto& c : comp) {
            c.id = u8();
            const int s = u8();
            c.h = s >> 4; c.v = s & 15; c.tq = u8();
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) return fail("bad component sampling");
            hmax = std::max(hmax, c.h); vmax = std::max(vmax, c.v);
        }
        progressive = marker == 0xC2;
        mcux = (W + 8 * hmax - 1) / (8 * hmax);
        mcuy = (H + 8 * vmax - 1) / (8 * vmax);
        for (auto& c : comp) {
            if (hmax % c.h || vmax % c.v) return fail("unsupported sampling factors");
            c.bw = mcux * c.h; c.bh = mcuy * c.v;
            c.cw = (W * c.h + hmax - 1) / hmax; c.ch = (H * c.v + vmax - 1) / vmax;
            c.coef.assign((size_t)c.bw * c.bh * 64, 0);
        }
        sof = true;
        return true;
    }
    bool parse_dqt() {
        int len = u16() - 2;
        while (len > 0) {
            const int pq = u8();
            const int t = pq & 15, prec = pq >> 4;
            if (t > 3 || prec > 1) return fail("bad DQT");
            for (int k = 0; k < 64; ++k) {
                const int v = prec ? u16() : u8();
                if (v < 0) return fail("truncated DQT");
                qt[t][kZigzag[k]] = (uint16_t)v;
            }
            qt_def[t] = true;
            len -= 1 + 64 * (prec + 1);
        }
        return len == 0 ? true : fail("bad DQT length");
    }
    bool parse_dht() {
        int len = u16() - 2;
        while (len > 0) {
            const int tc = u8();
            const int cls = tc >> 4, t = tc & 15;
            if (cls > 1 || t > 3) return fail("bad DHT");
            uint8_t counts[16];
            int tot = 0;
            for (int i = 0; i < 16; ++i) { const int c = u8(); if (c < 0) return fail("truncated DHT"); counts[i] = (uint8_t)c; tot += c; }
            if (tot > 256 || p + (size_t)tot > n) return fail("bad DHT counts");
            if (!(cls ? ac[t] : dc[t]).build(counts, f + p, tot)) return fail("bad Huffman table");
            p += (size_t)tot;
            len -= 17 + tot;
        }
        return len == 0 ? true : fail("bad DHT length");
    }
    void latch(Comp& c) {
        if (c.latched) return;
        std::memcpy(c.q, qt[c.tq], sizeof c.q);
        c.latched = true;
    }

    // one block of a scan
    bool block(Comp& c, int16_t* b, int tdc, int tac, int Ss, int Se, int Ah, int Al) {
        if (!progressive) {
            const int s = decode(dc[tdc]);
            if (s < 0 || s > 11) return fail("bad DC code");
            c.dc_pred += receive_extend(s);
            b[0] = (int16_t)c.dc_pred;
            for (int k = 1; k < 64;) {
                const int rs = decode(ac[tac]);
                if (rs < 0) return fail("bad AC code");
                const int r = rs >> 4, s2 = rs & 15;
                if (s2) {
                    k += r;
                    if (k > 63) return fail("AC coefficient index overflow");
                    b[kZigzag[k]] = (int16_t)receive_extend(s2);
                    ++k;
                } else {
                    if (r != 15) break;
                    k += 16;
                }
            }
            return true;
        }
        if (Ss == 0) {                           // DC scans
            if (Ah == 0) {
                const int s = decode(dc[tdc]);
                if (s < 0 || s > 11) return fail("bad DC code");
                c.dc_pred += receive_extend(s);
                b[0] = (int16_t)(c.dc_pred * (1 << Al));
            } else if (bit()) {
                b[0] = (int16_t)(b[0] | (1 << Al));
            }
            return true;
        }
        if (Ah == 0) {                           // AC first pass
            if (eobrun > 0) { --eobrun; return true; }
            for (int k = Ss; k <= Se;) {
                const int rs = decode(ac[tac]);
                if (rs < 0) return fail("bad AC code");
                const int r = rs >> 4, s = rs & 15;
                if (s) {
                    k += r;
                    if (k > 63) return fail("AC coefficient index overflow");
                    b[kZigzag[k]] = (int16_t)(receive_extend(s) * (1 << Al));
                    ++k;
                } else if (r == 15) {
                    k += 16;
                } else {
                    eobrun = 1 << r;
                    if (r) eobrun += bits(r);
                    --eobrun;
                    break;
                }
            }
            return true;
        }
        // AC refinement (T.81 G.1.2.3; libjpeg's decode_mcu_AC_refine)
        const int p1 = 1 << Al, m1 = -1 * (1 << Al);
        int k = Ss;
        auto refine = [&](int16_t& v) {
            if (bit() && (v & p1) == 0) v = (int16_t)(v >= 0 ? v + p1 : v + m1);
        };
        if (eobrun == 0) {
            for (; k <= Se; ++k) {
                const int rs = decode(ac[tac]);
                if (rs < 0) return fail("bad AC code");
                int r = rs >> 4, s = rs & 15;
                if (s) {
                    if (s != 1) return fail("bad AC refinement size");
                    s = bit() ? p1 : m1;
                } else if (r != 15) {
                    eobrun = 1 << r;
                    if (r) eobrun += bits(r);
                    break;
                }
                do {
                    int16_t& v = b[kZigzag[k]];
                    if (v != 0) refine(v);
                    else if (--r < 0) break;
                    ++k;
                } while (k <= Se);
                if (s && k <= 63) b[kZigzag[k]] = (int16_t)s;
            }
        }
        if (eobrun > 0) {
            for (; k <= Se; ++k) {
                int16_t& v = b[kZigzag[k]];
                if (v != 0) refine(v);
            }
            --eobrun;
        }
        return true;
    }

    bool parse_sos() {
        if (!sof) return fail("SOS before SOF");
        const int len = u16();
        const int ns = u8();
        if (ns < 1 || ns > 4 || len != 6 + 2 * ns) return fail("bad SOS");
        std::vector<int> ci(ns), tdc(ns), tac(ns);
        for (int i = 0; i < ns; ++i) {
            const int id = u8(), t = u8();
            ci[i] = -1;
            for (size_t k = 0; k < comp.size(); ++k) if (comp[k].id == id) ci[i] = (int)k;
            if (ci[i] < 0) return fail("SOS names an unknown component");
            tdc[i] = t >> 4; tac[i] = t & 15;
            if (tdc[i] > 3 || tac[i] > 3) return fail("bad SOS table");
        }
        const int Ss = u8(), Se = u8(), A = u8();
        const int Ah = A >> 4, Al = A & 15;
        if (progressive) {
            if (Ss > Se || Se > 63 || (Ss == 0 && Se != 0) || (Ss > 0 && ns != 1) || Al > 13) return fail("bad progressive scan");
        }
        for (int i = 0; i < ns; ++i) {
            Comp& c = comp[ci[i]];
            if (!qt_def[c.tq]) return fail("missing quantisation table");
            latch(c);
            const bool need_dc = !progressive || (Ss == 0 && Ah == 0);
            const bool need_ac = !progressive || Ss > 0;
            if ((need_dc && !dc[tdc[i]].defined) || (need_ac && !ac[tac[i]].defined)) return fail("missing Huffman table");
        }
        reset_entropy();
        int mcus_left = restart;
        auto mcu_done = [&]() -> bool {
            if (!restart) return true;
            if (--mcus_left == 0) { read_restart(); mcus_left = restart; }
            return true;
        };
        if (ns == 1) {                          // non-interleaved: the component's own blocks, raster order
            Comp& c = comp[ci[0]];
            const int bx = (c.cw + 7) / 8, by = (c.ch + 7) / 8;
            for (int y = 0; y < by; ++y)
                for (int x = 0; x < bx; ++x) {
                    if (!block(c, &c.coef[((size_t)y * c.bw + x) * 64], tdc[0], tac[0], Ss, Se, Ah, Al)) return false;
                    mcu_done();
                }
        } else {
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    for (int i = 0; i < ns; ++i) {
                        Comp& c = comp[ci[i]];
                        for (int v = 0; v < c.v; ++v)
                            for (int h = 0; h < c.h; ++h) {
                                const size_t bi = (size_t)(my * c.v + v) * c.bw + (size_t)(mx * c.h + h);
                                if (!block(c, &c.coef[bi * 64], tdc[i], tac[i], Ss, Se, Ah, Al)) return false;
                            }
                    }
                    mcu_done();
                }
        }
        // skip to the next marker
        bitbuf = 0; bitcnt = 0; hit_marker = false;
        while (p + 1 < n && !(f[p] == 0xFF && f[p + 1] != 0x00 && !(f[p + 1] >= 0xD0 && f[p + 1] <= 0xD7) && f[p + 1] != 0xFF)) ++p;
        return true;
    }

    bool parse() {
        if (n < 4 || f[0] != 0xFF || f[1] != 0xD8) return fail("not a JPEG file");
        p = 2;
        bool scanned = false;
        while (p < n) {
            int b = u8();
            if (b != 0xFF) continue;
            int m = u8();
            while (m == 0xFF) m = u8();
            if (m < 0) break;
            if (m == 0xD9) break;                                   // EOI
            if (m >= 0xD0 && m <= 0xD7) continue;                   // stray RST
            if (m == 0x01) continue;
            if (m == 0xC0 || m == 0xC1 || m == 0xC2) { if (!parse_sof(m)) return false; continue; }
            if ((m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) || m == 0xCC)
                return fail(m == 0xC3 || m == 0xC7 || m == 0xCB || m == 0xCF ? "lossless JPEG is not supported"
                                                                             : "arithmetic-coded JPEG is not supported");
            if (m == 0xC4) { if (!parse_dht()) return false; continue; }
            if (m == 0xDB) { if (!parse_dqt()) return false; continue; }
            if (m == 0xDD) { const int l = u16(); restart = u16(); if (l != 4 || restart < 0) return fail("bad DRI"); continue; }
            if (m == 0xDA) { if (!parse_sos()) return false; scanned = true; continue; }
            const int len = u16();                                  // APPn, COM, DNL, ...
            if (len < 2 || p + (size_t)len - 2 > n) return fail("truncated JPEG marker segment");
            if (m == 0xE0 && len >= 7 && !std::memcmp(f + p, "JFIF", 4)) jfif = true;
            if (m == 0xEE && len >= 14 && !std::memcmp(f + p, "Adobe", 5)) { adobe = true; adobe_transform = f[p + 11]; }
            p += (size_t)len - 2;
        }
        if (!sof || !scanned) return fail("no image data in JPEG");
        return true;
    }

    // ---- islow IDCT (jidctint.c) into the component's sample plane
    static inline int64_t descale(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }
    static inline uint8_t idct_limit(int64_t v) {               // the post-IDCT range-limit table (mask 1023)
        int k = (int)(v & 1023);
        const int x = k >= 512 ? k - 1024 : k;
        const int o = x + 128;
        return (uint8_t)(o < 0 ? 0 : (o > 255 ? 255 : o));
    }
    static void idct_islow(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
        constexpr int CB = 13, P1 = 2;
        constexpr int64_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                          F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
        int ws[64];
        for (int c = 0; c < 8; ++c) {
            const int16_t* i = in + c;
            const uint16_t* qq = q + c;
            int* w = ws + c;
            if (!i[8] && !i[16] && !i[24] && !i[32] && !i[40] && !i[48] && !i[56]) {
                const int dc = (int)((int64_t)i[0] * qq[0] * (1 << P1));
                for (int r = 0; r < 8; ++r) w[8 * r] = dc;
                continue;
            }
            int64_t z2 = (int64_t)i[16] * qq[16], z3 = (int64_t)i[48] * qq[48];
            int64_t z1 = (z2 + z3) * F0541;
            int64_t tmp2 = z1 + z3 * (-F1847), tmp3 = z1 + z2 * F0765;
            z2 = (int64_t)i[0] * qq[0]; z3 = (int64_t)i[32] * qq[32];
            int64_t tmp0 = (z2 + z3) * (1 << CB), tmp1 = (z2 - z3) * (1 << CB);
            const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
            tmp0 = (int64_t)i[56] * qq[56]; tmp1 = (int64_t)i[40] * qq[40];
            tmp2 = (int64_t)i[24] * qq[24]; tmp3 = (int64_t)i[8] * qq[8];
            z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2; int64_t z4 = tmp1 + tmp3;
            const int64_t z5 = (z3 + z4) * F1175;
            tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
            z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
            z3 += z5; z4 += z5;
            tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
            w[0] = (int)descale(t10 + tmp3, CB - P1); w[56] = (int)descale(t10 - tmp3, CB - P1);
            w[8] = (int)descale(t11 + tmp2, CB - P1); w[48] = (int)descale(t11 - tmp2, CB - P1);
            w[16] = (int)descale(t12 + tmp1, CB - P1); w[40] = (int)descale(t12 - tmp1, CB - P1);
            w[24] = (int)descale(t13 + tmp0, CB - P1); w[32] = (int)descale(t13 - tmp0, CB - P1);
        }
        for (int r = 0; r < 8; ++r) {
            const int* w = ws + 8 * r;
            uint8_t* o = out + (size_t)r * stride;
            if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
                const uint8_t v = idct_limit(descale(w[0], P1 + 3));
                for (int c = 0; c < 8; ++c) o[c] = v;
                continue;
            }
            int64_t z2 = w[2], z3 = w[6];
            int64_t z1 = (z2 + z3) * F0541;
            int64_t tmp2 = z1 + z3 * (-F1847), tmp3 = z1 + z2 * F0765;
            int64_t tmp0 = ((int64_t)w[0] + w[4]) * (1 << CB), tmp1 = ((int64_t)w[0] - w[4]) * (1 << CB);
            const int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
            tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
            z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2; int64_t z4 = tmp1 + tmp3;
            const int64_t z5 = (z3 + z4) * F1175;
            tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
            z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
            z3 += z5; z4 += z5;
            tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
            constexpr int S = CB + P1 + 3;
            o[0] = idct_limit(descale(t10 + tmp3, S)); o[7] = idct_limit(descale(t10 - tmp3, S));
            o[1] = idct_limit(descale(t11 + tmp2, S)); o[6] = idct_limit(descale(t11 - tmp2, S));
            o[2] = idct_limit(descale(t12 + tmp1, S)); o[5] = idct_limit(descale(t12 - tmp1, S));
            o[3] = idct_limit(descale(t13 + tmp0, S)); o[4] = idct_limit(descale(t13 - tmp0, S));
        }
    }

    void reconstruct(Comp& c) {
        const int pw = c.bw * 8;
        c.plane.assign((size_t)pw * c.bh * 8, 0);
        const int bx = (c.cw + 7) / 8, by = (c.ch + 7) / 8;    // blocks that hold image samples
        for (int y = 0; y < by; ++y)
            for (int x = 0; x < bx; ++x)
                idct_islow(&c.coef[((size_t)y * c.bw + x) * 64], c.q, &c.plane[(size_t)y * 8 * pw + (size_t)x * 8], pw);
    }

    // component c upsampled to full resolution, one output row
    void upsample_row(const Comp& c, int y, std::vector<uint8_t>& row) const {
        const int pw = c.bw * 8;
        const int sh = hmax / c.h, sv = vmax / c.v;
        if (sh == 1 && sv == 1) { std::memcpy(row.data(), &c.plane[(size_t)y * pw], (size_t)W); return; }
        const int dw = c.cw;
        auto at = [&](int r, int x) -> int { return c.plane[(size_t)r * pw + x]; };
        if (sh == 1 && sv == 2) {
            // h1v2 fancy upsampling: 3/4 nearer row + 1/4 farther row, rounding +1 (upper) / +2 (lower)
            const int r = y / 2;
            const int other = (y & 1) ? std::min(r + 1, c.ch - 1) : std::max(r - 1, 0);
            const int bias = (y & 1) ? 2 : 1;
            for (int x = 0; x < W; ++x) row[x] = (uint8_t)((at(r, x) * 3 + at(other, x) + bias) >> 2);
            return;
        }
        if (sh == 2 && (sv == 1 || sv == 2) && dw > 2) {
            // h2v1 / h2v2 fancy upsampling: column sums (3 * nearer row + farther row for v2), then the horizontal
            // triangle filter with +8 / +7 rounding (>> 4 for v2 column sums, >> 2 for h2v1)
            const int r = y / sv;
            std::vector<int> cs(dw);
            if (sv == 2) {
                const int other = (y & 1) ? std::min(r + 1, c.ch - 1) : std::max(r - 1, 0);
                for (int x = 0; x < dw; ++x) cs[x] = at(r, x) * 3 + at(other, x);
            } else {
                for (int x = 0; x < dw; ++x) cs[x] = at(r, x);
            }
            std::vector<uint8_t> out(2 * (size_t)dw);
            if (sv == 2) {
                if (dw == 1) { out[0] = out[1] = (uint8_t)((cs[0] * 4 + 8) >> 4); }
                else {
                    out[0] = (uint8_t)((cs[0] * 4 + 8) >> 4);
                    out[1] = (uint8_t)((cs[0] * 3 + cs[1] + 7) >> 4);
                    for (int x = 1; x < dw - 1; ++x) {
                        out[2 * x] = (uint8_t)((cs[x] * 3 + cs[x - 1] + 8) >> 4);
                        out[2 * x + 1] = (uint8_t)((cs[x] * 3 + cs[x + 1] + 7) >> 4);
                    }
                    out[2 * (dw - 1)] = (uint8_t)((cs[dw - 1] * 3 + cs[dw - 2] + 8) >> 4);
                    out[2 * (dw - 1) + 1] = (uint8_t)((cs[dw - 1] * 4 + 7) >> 4);
                }
            } else {
                if (dw == 1) { out[0] = out[1] = (uint8_t)cs[0]; }
                else {
                    out[0] = (uint8_t)cs[0];
                    out[1] = (uint8_t)((cs[0] * 3 + cs[1] + 2) >> 2);
                    for (int x = 1; x < dw - 1; ++x) {
                        out[2 * x] = (uint8_t)((cs[x] * 3 + cs[x - 1] + 1) >> 2);
                        out[2 * x + 1] = (uint8_t)((cs[x] * 3 + cs[x + 1] + 2) >> 2);
                    }
                    out[2 * (dw - 1)] = (uint8_t)((cs[dw - 1] * 3 + cs[dw - 2] + 1) >> 2);
                    out[2 * (dw - 1) + 1] = (uint8_t)cs[dw - 1];
                }
            }
            std::memcpy(row.data(), out.data(), (size_t)W);
            return;
        }
        // other integral factors: box replication (libjpeg's int_upsample)
        const int r = y / sv;
        for (int x = 0; x < W; ++x) row[x] = (uint8_t)at(r, x / sh);
    }

    bool output(Image& img) {
        for (auto& c : comp) {
            if (!c.latched) return fail("a component has no scan");
            reconstruct(c);
        }
        const int nc = (int)comp.size();
        img.w = W; img.h = H; img.is_float = false;
        img.channels = nc == 1 ? 1 : 3;
        img.u8.assign((size_t)W * H * img.channels, 0);
        // colour transform: YCbCr unless Adobe says 0 (RGB), or no JFIF / Adobe marker and ids 'R','G','B'
        bool ycc = nc == 3;
        if (nc == 3) {
            if (adobe) ycc = adobe_transform != 0;
            else if (!jfif && comp[0].id == 'R' && comp[1].id == 'G' && comp[2].id == 'B') ycc = false;
        }
        int cr_r[256], cb_b[256];
        int64_t cr_g[256], cb_g[256];
        auto FIX = [](double x) { return (int64_t)(x * 65536.0 + 0.5); };
        for (int i = 0, x = -128; i < 256; ++i, ++x) {
            cr_r[i] = (int)((FIX(1.40200) * x + (1 << 15)) >> 16);
            cb_b[i] = (int)((FIX(1.77200) * x + (1 << 15)) >> 16);
            cr_g[i] = -FIX(0.71414) * x;
            cb_g[i] = -FIX(0.34414) * x + (1 << 15);
        }
        auto clamp8 = [](int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); };
        std::vector<uint8_t> r0(W), r1(W), r2(W);
        for (int y = 0; y < H; ++y) {
            upsample_row(comp[0], y, r0);
            uint8_t* o = &img.u8[(size_t)y * W * img.channels];
            if (nc == 1) { std::memcpy(o, r0.data(), (size_t)W); continue; }
            upsample_row(comp[1], y, r1);
            upsample_row(comp[2], y, r2);
            for (int x = 0; x < W; ++x) {
                if (ycc) {
                    const int Y = r0[x], cb = r1[x], cr = r2[x];
                    o[3 * x] = clamp8(Y + cr_r[cr]);
                    o[3 * x + 1] = clamp8(Y + (int)((cb_g[cb] + cr_g[cr]) >> 16));
                    o[3 * x + 2] = clamp8(Y + cb_b[cb]);
                } else {
                    o[3 * x] = r0[x]; o[3 * x + 1] = r1[x]; o[3 * x + 2] = r2[x];
                }
            }
        }
        return true;
    }
};

}  // namespace

int decode_jpeg(const std::vector<uint8_t>& file, Image& img, std::string& err) {
    Decoder d;
    d.f = file.data();
    d.n = file.size();
    bool ok = false;
    try {
        ok = d.parse() && d.output(img);
    } catch (const std::bad_alloc&) {
        d.fail("out of memory decoding JPEG");
    }
    if (!ok) {
        err = d.err;
        const bool unsup = err.find("not supported") != std::string::npos || err.find("only ") == 0 ||
                           err.find("unsupported") != std::string::npos;
        return unsup ? -3 : -1;
    }
    return 0;
}

}  // namespace rs
