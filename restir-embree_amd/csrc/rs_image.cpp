// rs_image.cpp -- texture file decoders for the scene loader (see rs_image.h).
#include "rs_image.h"

#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <sstream>
#include <utility>

namespace rs {

static bool read_file(const std::string& path, std::vector<uint8_t>& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return true;
}

static uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// ---------------------------------------------------------------- PNG (ISO/IEC 15948)
static void put_be32(std::vector<uint8_t>& o, uint32_t v) {
    o.push_back((uint8_t)(v >> 24)); o.push_back((uint8_t)(v >> 16)); o.push_back((uint8_t)(v >> 8)); o.push_back((uint8_t)v);
}
static void put_chunk(std::vector<uint8_t>& o, const char* type, const uint8_t* d, size_t n) {
    put_be32(o, (uint32_t)n);
    const size_t t = o.size();
    o.insert(o.end(), type, type + 4);
    o.insert(o.end(), d, d + n);
    put_be32(o, (uint32_t)crc32(0L, o.data() + t, (uInt)(n + 4)));
}
int write_png(const std::string& path, int w, int h, int channels, const uint8_t* px, std::string& err) {
    if (w <= 0 || h <= 0 || channels < 1 || channels > 4 || !px) { err = "write_png: bad image"; return -1; }
    static const uint8_t ctypes[5] = {0, 0, 4, 2, 6};          // gray, gray+alpha, RGB, RGBA
    const size_t row = (size_t)w * channels;
    std::vector<uint8_t> raw((row + 1) * h);
    for (int y = 0; y < h; ++y) {                               // filter type 0 (None) per scanline
        raw[(row + 1) * y] = 0;
        std::memcpy(&raw[(row + 1) * y + 1], px + row * y, row);
    }
    uLongf zn = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zn);
    if (compress2(z.data(), &zn, raw.data(), (uLong)raw.size(), 6) != Z_OK) { err = "write_png: deflate failed"; return -1; }
    std::vector<uint8_t> o = {137, 80, 78, 71, 13, 10, 26, 10};
    uint8_t ihdr[13];
    ihdr[0] = (uint8_t)(w >> 24); ihdr[1] = (uint8_t)(w >> 16); ihdr[2] = (uint8_t)(w >> 8); ihdr[3] = (uint8_t)w;
    ihdr[4] = (uint8_t)(h >> 24); ihdr[5] = (uint8_t)(h >> 16); ihdr[6] = (uint8_t)(h >> 8); ihdr[7] = (uint8_t)h;
    ihdr[8] = 8; ihdr[9] = ctypes[channels]; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    put_chunk(o, "IHDR", ihdr, 13);
    put_chunk(o, "IDAT", z.data(), zn);
    put_chunk(o, "IEND", nullptr, 0);
    std::ofstream f(path, std::ios::binary);
    if (!f) { err = "cannot open " + path + " for writing"; return -1; }
    f.write((const char*)o.data(), (std::streamsize)o.size());
    if (!f) { err = "write failed: " + path; return -1; }
    return 0;
}

static int decode_png(const std::vector<uint8_t>& f, Image& img, std::string& err) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) { err = "not a PNG file"; return -1; }
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    size_t p = 8;
    while (p + 12 <= f.size()) {
        const uint32_t len = be32(&f[p]);
        if (p + 12 + (size_t)len > f.size()) { err = "truncated PNG chunk"; return -1; }
        const uint8_t* type = &f[p + 4];
        const uint8_t* d = &f[p + 8];
        if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
            w = be32(d); h = be32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(d, d + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns.assign(d, d + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        p += 12 + (size_t)len;
    }
    if (w == 0 || h == 0 || w > 65536 || h > 65536) { err = "bad PNG size"; return -1; }
    if (depth != 8) { err = "only 8-bit PNG is supported"; return -3; }
    if (interlace) { err = "interlaced PNG is not supported"; return -3; }
    int spp;   // samples per pixel in the file
    switch (ctype) {
        case 0: spp = 1; break;
        case 2: spp = 3; break;
        case 3: spp = 1; break;
        case 4: spp = 2; break;
        case 6: spp = 4; break;
        default: err = "bad PNG colour type"; return -1;
    }
    const size_t stride = (size_t)w * spp;
    std::vector<uint8_t> raw((stride + 1) * h);
    uLongf raw_len = (uLongf)raw.size();
    if (uncompress(raw.data(), &raw_len, idat.data(), (uLong)idat.size()) != Z_OK || raw_len != raw.size()) {
        err = "PNG inflate failed"; return -1;
    }
    std::vector<uint8_t> px(stride * h);
    for (uint32_t y = 0; y < h; ++y) {      // undo the per-row filters
        const uint8_t ft = raw[y * (stride + 1)];
        const uint8_t* src = &raw[y * (stride + 1) + 1];
        uint8_t* cur = &px[y * stride];
        const uint8_t* prev = y ? &px[(y - 1) * stride] : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= (size_t)spp ? cur[i - spp] : 0;
            const int b = prev ? prev[i] : 0;
            const int c = (prev && i >= (size_t)spp) ? prev[i - spp] : 0;
            int v = src[i];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: {
                    const int pp = a + b - c, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - c);
                    v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                    break;
                }
                default: err = "bad PNG filter"; return -1;
            }
            cur[i] = (uint8_t)v;
        }
    }
    img.w = (int)w; img.h = (int)h; img.is_float = false;
    if (ctype == 0 || ctype == 2 || ctype == 6) {
        img.channels = spp;
        img.u8.swap(px);
    } else if (ctype == 4) {                 // gray + alpha -> RGBA (FreeImage loads it as 32-bit)
        img.channels = 4;
        img.u8.resize((size_t)w * h * 4);
        for (size_t i = 0; i < (size_t)w * h; ++i) {
            const uint8_t g = px[2 * i], al = px[2 * i + 1];
            img.u8[4 * i] = g; img.u8[4 * i + 1] = g; img.u8[4 * i + 2] = g; img.u8[4 * i + 3] = al;
        }
    } else {                                 // palette -> RGB(A)
        if (plte.size() < 3) { err = "PNG palette missing"; return -1; }
        const size_t ne = plte.size() / 3;
        img.channels = trns.empty() ? 3 : 4;
        img.u8.resize((size_t)w * h * img.channels);
        for (size_t i = 0; i < (size_t)w * h; ++i) {
            const size_t k = px[i] < ne ? px[i] : 0;
            uint8_t* o = &img.u8[i * img.channels];
            o[0] = plte[3 * k]; o[1] = plte[3 * k + 1]; o[2] = plte[3 * k + 2];
            if (img.channels == 4) o[3] = k < trns.size() ? trns[k] : 255;
        }
    }
    return 0;
}

// ---------------------------------------------------------------- Radiance RGBE (.hdr)
static int decode_hdr(const std::vector<uint8_t>& f, Image& img, std::string& err) {
    size_t p = 0;
    auto line = [&](std::string& s) {
        s.clear();
        while (p < f.size() && f[p] != '\n') s.push_back((char)f[p++]);
        if (p < f.size()) ++p;
    };
    std::string s;
    line(s);
    if (s.rfind("#?", 0) != 0) { err = "not a Radiance HDR file"; return -1; }
    do { line(s); } while (!s.empty() && p < f.size());
    line(s);
    int w = 0, h = 0;
    char a[3] = {}, b[3] = {};
    if (std::sscanf(s.c_str(), "%2s %d %2s %d", a, &h, b, &w) != 4 || std::strcmp(a, "-Y") || std::strcmp(b, "+X")) {
        err = "unsupported HDR orientation (need -Y H +X W)"; return -3;
    }
    if (w <= 0 || h <= 0 || w > 65536 || h > 65536) { err = "bad HDR size"; return -1; }
    std::vector<uint8_t> row(4 * (size_t)w);
    img.w = w; img.h = h; img.channels = 3; img.is_float = true;
    img.f32.resize((size_t)w * h * 3);
    for (int y = 0; y < h; ++y) {
        if (p + 4 > f.size()) { err = "truncated HDR data"; return -1; }
        if (w >= 8 && w < 32768 && f[p] == 2 && f[p + 1] == 2 && ((f[p + 2] << 8) | f[p + 3]) == w) {
            p += 4;                           // adaptive RLE: the four components one after another
            for (int c = 0; c < 4; ++c) {
                int x = 0;
                while (x < w) {
                    if (p >= f.size()) { err = "truncated HDR RLE"; return -1; }
                    int n = f[p++];
                    if (n > 128) {
                        n -= 128;
                        if (p >= f.size() || x + n > w) { err = "bad HDR run"; return -1; }
                        const uint8_t v = f[p++];
                        for (int k = 0; k < n; ++k) row[4 * (size_t)(x++) + c] = v;
                    } else {
                        if (n == 0 || p + n > f.size() || x + n > w) { err = "bad HDR run"; return -1; }
                        for (int k = 0; k < n; ++k) row[4 * (size_t)(x++) + c] = f[p++];
                    }
                }
            }
        } else {                              // flat RGBE pixels
            if (p + 4 * (size_t)w > f.size()) { err = "truncated HDR data"; return -1; }
            std::memcpy(row.data(), &f[p], 4 * (size_t)w);
            p += 4 * (size_t)w;
        }
        for (int x = 0; x < w; ++x) {         // RGBE -> float (Ward's rgbe2float)
            const uint8_t* q = &row[4 * (size_t)x];
            float* o = &img.f32[3 * ((size_t)y * w + x)];
            if (q[3]) {
                const float e = (float)std::ldexp(1.0, (int)q[3] - (128 + 8));
                o[0] = q[0] * e; o[1] = q[1] * e; o[2] = q[2] * e;
            } else {
                o[0] = o[1] = o[2] = 0.0f;
            }
        }
    }
    return 0;
}

// ---------------------------------------------------------------- PFM / PPM / PGM
static bool header_tokens(const std::vector<uint8_t>& f, size_t& p, int n, std::vector<std::string>& tok) {
    while ((int)tok.size() < n && p < f.size()) {
        while (p < f.size() && std::isspace(f[p])) ++p;
        if (p < f.size() && f[p] == '#') { while (p < f.size() && f[p] != '\n') ++p; continue; }
        std::string t;
        while (p < f.size() && !std::isspace(f[p])) t.push_back((char)f[p++]);
        if (!t.empty()) tok.push_back(t);
    }
    if (p < f.size()) ++p;                    // the single whitespace before the raster
    return (int)tok.size() == n;
}

static int decode_pnm(const std::vector<uint8_t>& f, Image& img, std::string& err) {
    size_t p = 0;
    std::vector<std::string> t;
    if (!header_tokens(f, p, 4, t)) { err = "bad PNM header"; return -1; }
    const bool pfm = t[0] == "PF" || t[0] == "Pf";
    const bool color = t[0] == "PF" || t[0] == "P6";
    if (!pfm && t[0] != "P6" && t[0] != "P5") { err = "unsupported PNM variant " + t[0]; return -3; }
    const int w = std::atoi(t[1].c_str()), h = std::atoi(t[2].c_str());
    if (w <= 0 || h <= 0 || w > 65536 || h > 65536) { err = "bad PNM size"; return -1; }
    const int nc = color ? 3 : 1;
    img.w = w; img.h = h;
    if (pfm) {
        const double scale = std::atof(t[3].c_str());
        const bool little = scale < 0;
        if (p + (size_t)w * h * nc * 4 > f.size()) { err = "truncated PFM"; return -1; }
        img.is_float = true; img.channels = 3;
        img.f32.resize((size_t)w * h * 3);
        for (int y = 0; y < h; ++y)           // PFM rows run bottom to top
            for (int x = 0; x < w; ++x)
                for (int c = 0; c < 3; ++c) {
                    const uint8_t* q = &f[p + 4 * (((size_t)y * w + x) * nc + (nc == 3 ? c : 0))];
                    uint8_t b4[4] = {q[0], q[1], q[2], q[3]};
                    if (!little) { std::swap(b4[0], b4[3]); std::swap(b4[1], b4[2]); }
                    float v; std::memcpy(&v, b4, 4);
                    img.f32[3 * ((size_t)(h - 1 - y) * w + x) + c] = v;
                }
        return 0;
    }
    if (std::atoi(t[3].c_str()) != 255) { err = "only maxval 255 PNM is supported"; return -3; }
    if (p + (size_t)w * h * nc > f.size()) { err = "truncated PNM"; return -1; }
    img.is_float = false; img.channels = nc;
    img.u8.assign(f.begin() + p, f.begin() + p + (size_t)w * h * nc);
    return 0;
}

int load_image(const std::string& path, Image& img, std::string& err) {
    std::vector<uint8_t> f;
    if (!read_file(path, f)) { err = "cannot open " + path; return -1; }
    int rc;
    try {   // a decoder's allocation failure is an error return, never an exception through the C ABI
        if (f.size() >= 8 && f[0] == 137 && f[1] == 'P' && f[2] == 'N' && f[3] == 'G') rc = decode_png(f, img, err);
        else if (f.size() >= 2 && f[0] == '#' && f[1] == '?') rc = decode_hdr(f, img, err);
        else if (f.size() >= 2 && f[0] == 'P') rc = decode_pnm(f, img, err);
        else if (f.size() >= 2 && f[0] == 0xFF && f[1] == 0xD8) rc = decode_jpeg(f, img, err);
        else { err = "unknown image format"; rc = -1; }
    } catch (const std::bad_alloc&) {
        err = "out of memory decoding the image"; rc = -1;
    }
    if (rc) err = path + ": " + err;
    return rc;
}

}  // namespace rs
