// Host check of the byte parsers under AddressSanitizer + UBSan
// (tests/test_sanitize.py builds it with -fsanitize=address,undefined):
// glTF / GLB (gltf.cpp, json.h), PNG (png.cpp) and JPEG (jpeg.cpp) -- the
// code that reads untrusted files (stage1.zig:30-110, 381-469 on the
// reference side).  Every seed must load; then deterministic mutations of it
// (truncations at 33 lengths, and byte flips) must each either load or return
// an error -- never read or write out of bounds, overflow a signed int,
// shift out of range, or leak (any sanitizer report aborts the run).
//   parser_fuzz <workdir> <mutations per seed> <seed files...>
// .png / .jpg seeds go to the decoders as byte buffers; .gltf / .glb seeds
// are loaded by path from <workdir>, where mutated copies are written (a
// .gltf's sibling .bin / image files are mutated too, one file at a time).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "png.h"
#include "zrt.h"

static std::vector<uint8_t> read_all(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}
static void write_all(const std::string& p, const std::vector<uint8_t>& b) {
    std::ofstream f(p, std::ios::binary | std::ios::trunc);
    f.write((const char*)b.data(), (std::streamsize)b.size());
}
static std::string ext_of(const std::string& p) {
    const size_t d = p.rfind('.');
    return d == std::string::npos ? "" : p.substr(d);
}
static std::string base_of(const std::string& p) {
    const size_t s = p.rfind('/');
    return s == std::string::npos ? p : p.substr(s + 1);
}

// the mutants of one buffer: truncations, then single / multi byte flips
static std::vector<std::vector<uint8_t>> mutants(const std::vector<uint8_t>& b, int n, std::mt19937_64& rng) {
    std::vector<std::vector<uint8_t>> out;
    for (int k = 0; k <= 32; ++k) out.emplace_back(b.begin(), b.begin() + (ptrdiff_t)(b.size() * k / 33));
    const uint8_t interesting[] = {0x00, 0xFF, 0x7F, 0x80, 0x01, 0x10, '{', '}', '"', ',', '9', '-'};
    for (int i = 0; i < n && !b.empty(); ++i) {
        std::vector<uint8_t> m = b;
        const int flips = 1 + (int)(rng() % 4);
        for (int f = 0; f < flips; ++f) {
            // bias towards the head: headers, chunk tables and JSON keys live there
            const size_t pos = (rng() & 1) ? rng() % std::min<size_t>(m.size(), 512) : rng() % m.size();
            m[pos] = (rng() & 1) ? interesting[rng() % sizeof interesting] : (uint8_t)rng();
        }
        out.push_back(std::move(m));
    }
    return out;
}

static int decode_image(const std::string& ext, const std::vector<uint8_t>& b) {
    zrt::Image8 img;
    const int rc = ext == ".png" ? zrt::png_decode(b.data(), b.size(), &img) : zrt::jpeg_decode(b.data(), b.size(), &img);
    if (rc == ZRT_OK) {
        std::vector<float> lin;
        zrt::rgba8_to_linear(img, &lin);
        if (img.rgba.size() != (size_t)img.w * img.h * 4) return -100;
    }
    return rc;
}

static int load_gltf(const std::string& path) {
    zrt_gltf* g = nullptr;
    const int rc = zrt_gltf_load(path.c_str(), 2, &g);
    if (rc == ZRT_OK) {
        const float *p, *nn, *t;
        const uint32_t* m;
        uint32_t n = 0;
        zrt_gltf_soup(g, &p, &nn, &t, &m, &n);
        zrt_scene s{};
        zrt_gltf_materials(g, &s);
        zrt_camera cam;
        (void)zrt_gltf_camera(g, nullptr, -1, 64, &cam);
        zrt_gltf_free(g);
    }
    return rc;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: parser_fuzz <workdir> <mutations> <seeds...>\n");
        return 2;
    }
    const std::string wd = argv[1];
    const int n = atoi(argv[2]);
    std::mt19937_64 rng(20241116);
    long runs = 0, ok = 0, seed_fail = 0;
    for (int a = 3; a < argc; ++a) {
        const std::string seed = argv[a], ext = ext_of(seed);
        if (ext == ".png" || ext == ".jpg") {
            const auto b = read_all(seed);
            if (decode_image(ext, b) != ZRT_OK) { fprintf(stderr, "seed failed: %s\n", seed.c_str()); ++seed_fail; }
            for (const auto& m : mutants(b, n, rng)) { ++runs; ok += decode_image(ext, m) == ZRT_OK; }
        } else if (ext == ".gltf" || ext == ".glb") {
            if (load_gltf(seed) != ZRT_OK) { fprintf(stderr, "seed failed: %s\n", seed.c_str()); ++seed_fail; }
            // mutate the document itself, then each sibling file listed after
            // "--sibling" style: every other argv entry with the seed's stem
            const std::string dir = seed.substr(0, seed.rfind('/') + 1);
            std::vector<std::string> files = {base_of(seed)};
            for (int b = 3; b < argc; ++b) {
                const std::string o = argv[b];
                if (o != seed && o.rfind(dir, 0) == 0 && (ext_of(o) == ".bin" || ext_of(o) == ".png" ||
                                                          ext_of(o) == ".jpg"))
                    files.push_back(base_of(o));
            }
            for (const auto& target : files) {
                for (const auto& f : files) write_all(wd + "/" + f, read_all(dir + f));
                const auto orig = read_all(dir + target);
                for (const auto& m : mutants(orig, target == files[0] ? n : n / 4, rng)) {
                    write_all(wd + "/" + target, m);
                    ++runs;
                    ok += load_gltf(wd + "/" + files[0]) == ZRT_OK;
                }
                write_all(wd + "/" + target, orig);
            }
        }
    }
    printf("{\"runs\": %ld, \"loaded\": %ld, \"seed_failures\": %ld}\n", runs, ok, seed_fail);
    return seed_fail ? 1 : 0;
}
