// PNG encode time by zlib level on a rendered image (host tool).
//   g++ -O2 -std=c++17 -Iinclude -Izig_raytracing_contest_amd/csrc tools/png_bench.cpp zig_raytracing_contest_amd/csrc/png.cpp zig_raytracing_contest_amd/csrc/capi.cpp -o tools/bin/png_bench -lz -pthread
#include <chrono>
#include <cstdio>
#include <vector>
#include "png.h"
#include "zrt.h"
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb"); std::vector<uint8_t> b; int c; while ((c = fgetc(f)) != EOF) b.push_back((uint8_t)c); fclose(f);
    zrt::Image8 img; if (zrt::png_decode(b.data(), b.size(), &img) != 0) return 1;
    std::vector<uint8_t> rgb((size_t)img.w * img.h * 3);
    for (size_t i = 0; i < (size_t)img.w * img.h; ++i) for (int k = 0; k < 3; ++k) rgb[3 * i + k] = img.rgba[4 * i + k];
    for (int lv : {1, 2, 3, 4, 6}) {
        std::vector<uint8_t> out; auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < 5; ++r) { out.clear(); zrt::png_encode_rgb(rgb.data(), img.w, img.h, lv, &out); }
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / 5;
        printf("level %d: %.2f ms, %zu bytes\n", lv, ms, out.size());
    }
}
