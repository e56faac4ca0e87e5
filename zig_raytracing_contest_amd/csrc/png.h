// png.h -- PNG decode (for glTF textures) and encode (output.png) on zlib.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace zrt {

// An 8-bit image expanded to RGBA the way stb_image's req_comp = 4 does
// (gray -> g,g,g; missing alpha -> 255; palette via PLTE/tRNS; 16-bit -> high
// byte).  actual_c = channels in the file (stb's *comp), incl. tRNS alpha.
struct Image8 {
    int w = 0, h = 0;
    int actual_c = 0;
    std::vector<uint8_t> rgba;
};

int png_decode(const uint8_t* data, size_t n, Image8* out);
// JPEG (jpeg.cpp): baseline/extended/progressive Huffman, 8-bit, Gray or YCbCr -> RGBA8
int jpeg_decode(const uint8_t* data, size_t n, Image8* out);
int png_encode_rgb(const uint8_t* rgb, int w, int h, int level, std::vector<uint8_t>* out);
int png_write_rgb(const char* path, const uint8_t* rgb, int w, int h, int level);

// stb_image stbi__ldr_to_hdr with req_comp = 4: colour channels
// (float)(pow(v / 255.0f, 2.2f) * 1.0f), alpha v / 255.0f.
void rgba8_to_linear(const Image8& img, std::vector<float>* rgba_f);

}  // namespace zrt
