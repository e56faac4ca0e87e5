// cli.cpp -- `zrt`, the drop-in for the reference executable (src/main.zig).
//
//   zrt [--in input.gltf] [--out output.png] [--camera NAME] [--width N] [--height N]
//
// Same flags and defaults as main.zig:33-39 (zig-args: `--flag value` or
// `--flag=value`), config.json read from the working directory with the same
// keys (main.zig:56-69: grid_resolution, num_threads, num_samples,
// max_bounce), the same phase log lines on stderr ("info: Loaded in ...",
// main.zig:103-142, durations printed like std.fmt.fmtDuration).  The render
// phase runs the HIP path on every GPU listed in ZRT_DEVICES (default: device
// 0) through one libzrt device group (zrt_group_*): the image's interleaved
// tiles split over the GPUs, one context each, gathered over xGMI.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zrt.h"
#include "json.h"

namespace zrt {
unsigned host_threads();   // capi.cpp: CPUs this process may use, capped by OMP_NUM_THREADS
}

extern "C" int zrt_png_write(const char* path, const uint8_t* rgb, uint32_t w, uint32_t h);

namespace {

using Clock = std::chrono::steady_clock;

// std.fmt.fmtDuration (Zig 0.11)
std::string fmt_duration(uint64_t ns) {
    std::string out;
    const struct { uint64_t ns; const char* sep; } big[] = {
        {365ull * 86400 * 1000000000ull, "y"}, {7ull * 86400 * 1000000000ull, "w"},
        {86400ull * 1000000000ull, "d"}, {3600ull * 1000000000ull, "h"}, {60ull * 1000000000ull, "m"}};
    for (const auto& u : big) {
        if (ns >= u.ns) {
            const uint64_t n = ns / u.ns;
            out += std::to_string(n) + u.sep;
            ns -= n * u.ns;
            if (ns == 0) return out;
        }
    }
    const struct { uint64_t ns; const char* sep; } small[] = {
        {1000000000ull, "s"}, {1000000ull, "ms"}, {1000ull, "us"}};
    for (const auto& u : small) {
        const uint64_t k = ns * 1000 / u.ns;
        if (k >= 1000) {
            out += std::to_string(k / 1000);
            const uint64_t frac = k % 1000;
            if (frac) {
                char buf[8];
                snprintf(buf, sizeof buf, ".%03llu", (unsigned long long)frac);
                std::string f(buf);
                while (f.size() > 1 && f.back() == '0') f.pop_back();
                out += f;
            }
            return out + u.sep;
        }
    }
    return out + std::to_string(ns) + "ns";
}

uint64_t since(Clock::time_point t) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t).count();
}

void info(const std::string& s) { fprintf(stderr, "info: %s\n", s.c_str()); }
int fail(const char* what, int rc) {
    fprintf(stderr, "error: %s: %s\n", what, zrt_error_string(rc));
    return 1;
}

struct Config {
    uint32_t res[3] = {128, 128, 128};
    int num_threads = -1;   // null
    uint32_t num_samples = 3, max_bounce = 4;
};

bool load_config(const char* path, Config* c, std::string* err) {
    FILE* f = fopen(path, "rb");
    if (!f) { *err = "FileNotFound: config.json"; return false; }
    std::string s;
    char buf[4096];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    fclose(f);
    zrt::json::Value v;
    if (!zrt::json::parse(s.data(), s.size(), &v) || v.type != zrt::json::Value::Object) {
        *err = "SyntaxError in config.json";
        return false;
    }
    for (const auto& kv : v.obj) {   // std.json rejects unknown fields
        if (kv.first != "grid_resolution" && kv.first != "num_threads" && kv.first != "num_samples" &&
            kv.first != "max_bounce") {
            *err = "UnknownField: " + kv.first;
            return false;
        }
    }
    const zrt::json::Value* g = v.get("grid_resolution");
    if (!g || g->type != zrt::json::Value::Array || g->size() != 3) { *err = "MissingField: grid_resolution"; return false; }
    for (int i = 0; i < 3; ++i) c->res[i] = (uint32_t)(*g)[i].num;
    const zrt::json::Value* t = v.get("num_threads");
    c->num_threads = (t && t->type == zrt::json::Value::Number) ? (int)t->num : -1;
    if (!v.get("num_samples") || !v.get("max_bounce")) { *err = "MissingField"; return false; }
    c->num_samples = (uint32_t)v.number("num_samples", 3);
    c->max_bounce = (uint32_t)v.number("max_bounce", 4);
    return true;
}

void usage() {
    fprintf(stderr,
            "usage: zrt [--in input.gltf] [--out output.png] [--camera NAME] [--width N] [--height N]\n"
            "  config.json (cwd): grid_resolution, num_threads, num_samples, max_bounce\n"
            "  ZRT_DEVICES=0,1,...  GPUs to render on (image tiles split across them)\n");
}

}  // namespace

int main(int argc, char** argv) {
    const auto t_start = Clock::now();
    // HIP start-up (context + code objects of the first render GPU, ~0.1-0.2 s)
    // overlapped with argument parsing and the glTF load; joined before the
    // first GPU use
    int warm_dev = 0;
    if (const char* e = getenv("ZRT_DEVICES")) warm_dev = atoi(e);
    // ZRT_TIMING=1: the start-up split on stderr ("timing:" lines, not the
    // reference's phase lines): when the warm-up thread ran, how long the
    // first GPU use waited for it, the group creation and the grid info
    const bool timing = getenv("ZRT_TIMING") != nullptr;
    uint64_t warm_begin_ns = 0, warm_end_ns = 0;
    std::thread hip_warm([warm_dev, t_start, &warm_begin_ns, &warm_end_ns] {
        warm_begin_ns = since(t_start);
        (void)zrt_device_warmup(warm_dev);
        warm_end_ns = since(t_start);
    });
    struct Join {
        std::thread& t;
        ~Join() { if (t.joinable()) t.join(); }
    } join_warm{hip_warm};
    std::string in = "input.gltf", out = "output.png";
    const char* camera = nullptr;
    std::string camera_s;
    int width = -1, height = -1;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i], val;
        const size_t eq = a.find('=');
        bool has_val = false;
        if (a.rfind("--", 0) == 0 && eq != std::string::npos) { val = a.substr(eq + 1); a = a.substr(0, eq); has_val = true; }
        auto next = [&]() -> bool {
            if (has_val) return true;
            if (i + 1 >= argc) return false;
            val = argv[++i];
            return true;
        };
        if (a == "--help" || a == "-h") { usage(); return 0; }
        if (a != "--in" && a != "--out" && a != "--camera" && a != "--width" && a != "--height") {
            fprintf(stderr, "error: unknown option %s\n", a.c_str());
            usage();
            return 1;
        }
        if (!next()) { fprintf(stderr, "error: missing value for %s\n", a.c_str()); return 1; }
        if (a == "--in") in = val;
        else if (a == "--out") out = val;
        else if (a == "--camera") { camera_s = val; camera = camera_s.c_str(); }
        else {
            char* e = nullptr;
            const long v = strtol(val.c_str(), &e, 10);
            if (!e || *e || v < 0 || v > 65535) { fprintf(stderr, "error: %s must be u16\n", a.c_str()); return 1; }
            (a == "--width" ? width : height) = (int)v;
        }
    }
    Config cfg;
    std::string err;
    if (!load_config("config.json", &cfg, &err)) { fprintf(stderr, "error: %s\n", err.c_str()); return 1; }
    info("Num samples: " + std::to_string(cfg.num_samples) + ", max bounce " + std::to_string(cfg.max_bounce));
    const uint32_t num_threads = cfg.num_threads >= 0 ? (uint32_t)cfg.num_threads
                                                      : zrt::host_threads();
    info("Num threads: " + std::to_string(num_threads));

    // GPUs
    std::vector<int> devices;
    if (const char* e = getenv("ZRT_DEVICES")) {
        std::string s(e);
        size_t p = 0;
        while (p < s.size()) {
            const size_t q = s.find(',', p);
            devices.push_back(atoi(s.substr(p, q == std::string::npos ? std::string::npos : q - p).c_str()));
            if (q == std::string::npos) break;
            p = q + 1;
        }
    }
    if (devices.empty()) devices.push_back(0);

    zrt_scene scene;
    memset(&scene, 0, sizeof scene);
    zrt_camera cam;
    zrt_gltf* gltf = nullptr;
    zrt_geometry* geo = nullptr;
    zrt_group* group = nullptr;     // one context per device (zrt_group_*, libzrt)
    struct GroupFree {
        zrt_group*& g;
        ~GroupFree() { zrt_group_destroy(g); }
    } free_group{group};
    int rc;
    {
        const auto t = Clock::now();
        if ((rc = zrt_gltf_load(in.c_str(), num_threads, &gltf)) != ZRT_OK) return fail("loadGltfFile", rc);
        info("Loaded in " + fmt_duration(since(t)));
    }
    const float *pos, *nrm, *uv;
    const uint32_t* mat;
    uint32_t ntri = 0;
    {
        const auto t = Clock::now();
        if ((rc = zrt_gltf_camera(gltf, camera, width, height, &cam)) != ZRT_OK) return fail("loadCamera", rc);
        info("Pixels count: " + std::to_string((uint64_t)cam.w * cam.h));
        zrt_gltf_materials(gltf, &scene);
        info("Materials count: " + std::to_string(scene.num_materials));
        zrt_gltf_soup(gltf, &pos, &nrm, &uv, &mat, &ntri);
        info("Preprocessed in " + fmt_duration(since(t)));
    }
    const uint32_t ndev = (uint32_t)devices.size();
    {
        const auto t = Clock::now();
        info("Grid resolution: { " + std::to_string(cfg.res[0]) + ", " + std::to_string(cfg.res[1]) + ", " +
             std::to_string(cfg.res[2]) + " }");
        // Default: the grid is built on every render GPU straight into its
        // context (zrt_group_create_built, the builds in parallel; r01: 5-9 ms
        // against 36-97 ms for host build + upload).  ZRT_DEVICE_BUILD=0: host
        // threads, then one upload per device; =1: device build with the host
        // round trip.  Same arrays, bit for bit, on every path.
        const char* db = getenv("ZRT_DEVICE_BUILD");
        const int mode = db ? atoi(db) : 2;
        uint32_t empty = 0, mn = 0xFFFFFFFFu, mx = 0, ncells = 0, nrefs = 0;
        if (mode == 2) {
            const uint64_t join0 = since(t_start);
            if (hip_warm.joinable()) hip_warm.join();
            const uint64_t join1 = since(t_start);
            rc = zrt_group_create_built(pos, nrm, uv, mat, ntri, cfg.res, scene.num_materials, scene.materials,
                                        scene.texels, scene.num_texel_floats, devices.data(), ndev, &group);
            if (rc != ZRT_OK) return fail("Geometry.build", rc);
            const uint64_t built = since(t_start);
            zrt_context* c0 = nullptr;
            uint32_t gi[4];
            if ((rc = zrt_group_context(group, 0, &c0)) != ZRT_OK || (rc = zrt_context_grid_info(c0, nullptr, gi)) != ZRT_OK)
                return fail("Geometry.build", rc);
            if (timing)
                fprintf(stderr, "timing: warm-up thread %s .. %s (%s), joined at %s after waiting %s, "
                        "group_create_built %s, grid info %s\n",
                        fmt_duration(warm_begin_ns).c_str(), fmt_duration(warm_end_ns).c_str(),
                        fmt_duration(warm_end_ns - warm_begin_ns).c_str(), fmt_duration(join1).c_str(),
                        fmt_duration(join1 - join0).c_str(), fmt_duration(built - join1).c_str(),
                        fmt_duration(since(t_start) - built).c_str());
            ncells = cfg.res[0] * cfg.res[1] * cfg.res[2];
            nrefs = gi[0]; empty = gi[1]; mn = gi[2]; mx = gi[3];
        } else {
            if (mode == 1) {
                if (hip_warm.joinable()) hip_warm.join();
                rc = zrt_geometry_build_device(pos, nrm, uv, mat, ntri, cfg.res, devices[0], &geo);
            } else {
                rc = zrt_geometry_build(pos, nrm, uv, mat, ntri, cfg.res, num_threads, &geo);
            }
            if (rc != ZRT_OK) return fail("Geometry.build", rc);
            zrt_geometry_scene(geo, &scene);
            ncells = scene.num_cells;
            nrefs = scene.num_triangles;
            for (uint32_t c = 0; c < scene.num_cells; ++c) {
                const uint32_t k = scene.cells[2 * c + 1] - scene.cells[2 * c];
                if (!k) ++empty;
                else { mn = std::min(mn, k); mx = std::max(mx, k); }
            }
        }
        char buf[256];
        const uint32_t nonempty = ncells - empty;
        snprintf(buf, sizeof buf, "Empty cells: %u/%u (%.2f%%) min triangles: %u max triangles: %u mean_triangles: %u",
                 empty, ncells, 100.0 * empty / ncells, nonempty ? mn : 0xFFFFFFFFu, mx,
                 nonempty ? nrefs / nonempty : 0);
        info(buf);
        snprintf(buf, sizeof buf, "Unique triangle count: %u/%u (%.2f%%)", ntri, nrefs,
                 nrefs ? 100.0 * ntri / nrefs : 0.0);
        info(buf);
        info("Compiled in " + fmt_duration(since(t)));
    }
    if (!group) {
        const auto t = Clock::now();
        if (hip_warm.joinable()) hip_warm.join();
        if ((rc = zrt_group_create(&scene, devices.data(), ndev, &group)) != ZRT_OK) return fail("zrt_group_create", rc);
        info("Uploaded in " + fmt_duration(since(t)));
    }
    std::vector<uint8_t> img((size_t)cam.w * cam.h * 3, 0);
    {
        // Scene.render (main.zig:126): the image's tiles over the devices,
        // one host thread each, gathered into img (zrt_group_render)
        const auto t = Clock::now();
        zrt_render_config rc_{};
        rc_.num_samples = cfg.num_samples;
        rc_.max_bounce = cfg.max_bounce;
        rc_.num_ranks = 1;
        zrt_stats st{};
        if ((rc = zrt_group_render(group, &cam, &rc_, img.data(), &st)) != ZRT_OK) return fail("Scene.render", rc);
        const uint64_t ns = since(t);
        info("Rendered in " + fmt_duration(ns));
        char buf[160];
        snprintf(buf, sizeof buf, "Rays: %llu segments, %.1f Mrays/s on %u GPU(s)", (unsigned long long)st.segments,
                 st.segments / (ns / 1e9) / 1e6, ndev);
        info(buf);
    }
    zrt_group_destroy(group);
    group = nullptr;
    {
        const auto t = Clock::now();
        if ((rc = zrt_png_write(out.c_str(), img.data(), cam.w, cam.h)) != ZRT_OK) return fail("WritePngFail", rc);
        info("Saved in " + fmt_duration(since(t)));
    }
    zrt_geometry_free(geo);
    zrt_gltf_free(gltf);
    info("Done in " + fmt_duration(since(t_start)));
    return 0;
}
