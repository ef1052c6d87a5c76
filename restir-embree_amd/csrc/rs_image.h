// rs_image.h -- texture file decoding for the scene loader (the reference uses FreeImage,
// pg/Texture.cpp:9-57; not available here).  Formats: JPEG (rs_jpeg.cpp), PNG (8-bit gray / gray+alpha / RGB /
// RGBA / palette, non-interlaced; zlib inflate), Radiance .hdr (flat and RLE scanlines), .pfm, binary .ppm/.pgm.
#pragma once
#include "../../include/restir_c.h"

#include <cstdint>
#include <string>
#include <vector>

namespace rs {

struct Image {
    int w = 0, h = 0, channels = 0;  // 1, 3 or 4
    bool is_float = false;
    std::vector<uint8_t> u8;         // top row first, R,G,B(,A)
    std::vector<float> f32;
};

// 0 on success; -1 I/O or format error, -3 unsupported variant (arithmetic / lossless / 12-bit / CMYK JPEG,
// 16-bit / interlaced PNG)
int load_image(const std::string& path, Image& img, std::string& err);
// rs_jpeg.cpp: baseline / extended / progressive Huffman JPEG, grey or 3 components, libjpeg-turbo's default
// reconstruction (islow IDCT, fancy upsampling, fixed-point YCbCr -> RGB)
int decode_jpeg(const std::vector<uint8_t>& file, Image& img, std::string& err);

// 8-bit PNG writer (stbi_write_png's role in SimpleGuiDX11::exportImage, pg/simpleguidx11.cpp:607-627):
// `channels` = 1..4 interleaved bytes, top row first; 0 on success, -1 I/O error
int write_png(const std::string& path, int w, int h, int channels, const uint8_t* px, std::string& err);

// OBJ/MTL scene (rs_obj_loader.cpp): de-indexed triangles in file order, materials with 1-based map
// slots into `images`; srgb[i] = texture i is a colour map (Texture::expand per referencing slot)
struct ObjScene {
    std::vector<float> pos, nrm, uv, tan;      // 9, 9, 6, 9 floats per triangle
    std::vector<uint32_t> tri_mat;
    std::vector<rs_material_desc> mats;
    std::vector<Image> images;
    std::vector<int> srgb;
};
// 0 on success; -1 parse / I/O error, -3 unsupported texture file
int load_obj_file(const char* path, ObjScene& out, std::string& err);

}  // namespace rs
