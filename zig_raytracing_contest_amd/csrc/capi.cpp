// capi.cpp -- host-side C ABI helpers: status strings, camera (stage1),
// ziggurat tables, the per-rank tile order of the packed image.
#include <sched.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "zrt_internal.h"

using namespace zrt;

namespace zrt {
unsigned host_threads() {
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) n = (unsigned)CPU_COUNT(&set);
    if (const char* e = getenv("OMP_NUM_THREADS")) {
        const int k = atoi(e);
        if (k > 0) n = std::min(n, (unsigned)k);
    }
    return n;
}
}  // namespace zrt

extern "C" const char* zrt_error_string(int s) {
    switch (s) {
        case ZRT_OK: return "ok";
        case ZRT_ERR_INVALID_ARG: return "invalid argument";
        case ZRT_ERR_NO_DEVICE: return "no HIP device";
        case ZRT_ERR_HIP: return "HIP runtime error";
        case ZRT_ERR_OUT_OF_MEMORY: return "out of memory";
        case ZRT_ERR_UNSUPPORTED: return "unsupported configuration";
        case ZRT_ERR_IO: return "I/O error";
        case ZRT_ERR_PARSE: return "parse error";
        case ZRT_ERR_NOT_FOUND: return "not found";
        case ZRT_ERR_CAMERA: return "camera/output size rules violated";
        default: return "unknown status";
    }
}

extern "C" int zrt_abi_version(void) { return ZRT_ABI_VERSION; }

namespace zrt {

void zig_tables(double zx[257], double zf[257]) {
    static std::once_flag once;
    static double X[257], F[257];
    std::call_once(once, [] {
        X[0] = kNormV / norm_pdf(kNormR);
        X[1] = kNormR;
        for (int i = 2; i < 256; ++i)
            X[i] = std::sqrt(-2.0 * det_log(kNormV / X[i - 1] + norm_pdf(X[i - 1])));
        X[256] = 0.0;
        for (int i = 0; i < 257; ++i) F[i] = norm_pdf(X[i]);
    });
    memcpy(zx, X, sizeof X);
    memcpy(zf, F, sizeof F);
}

int tile_pixels(uint32_t w, uint32_t h, uint32_t tile, uint32_t rank, uint32_t nranks,
                uint32_t* out, uint32_t* count) {
    if (!count || w == 0 || h == 0 || nranks == 0 || rank >= nranks) return ZRT_ERR_INVALID_ARG;
    if (tile == 0) tile = 64;
    if (tile % 8 != 0) return ZRT_ERR_INVALID_ARG;
    const uint32_t tx = (w + tile - 1) / tile, ty = (h + tile - 1) / tile;
    uint64_t n = 0;
    for (uint64_t t = rank; t < (uint64_t)tx * ty; t += nranks) {
        const uint32_t x0 = (uint32_t)(t % tx) * tile, y0 = (uint32_t)(t / tx) * tile;
        for (uint32_t by = 0; by < tile; by += 8)
            for (uint32_t bx = 0; bx < tile; bx += 8)
                for (uint32_t py = 0; py < 8; ++py)
                    for (uint32_t px = 0; px < 8; ++px) {
                        const uint32_t x = x0 + bx + px, y = y0 + by + py;
                        if (x >= w || y >= h) continue;
                        if (out) out[n] = y * w + x;
                        ++n;
                    }
    }
    *count = (uint32_t)n;
    return ZRT_OK;
}

}  // namespace zrt

extern "C" int zrt_tile_pixels(uint32_t w, uint32_t h, uint32_t tile, uint32_t rank,
                               uint32_t nranks, uint32_t* pixels, uint32_t* count) {
    return tile_pixels(w, h, tile, rank, nranks, pixels, count);
}

// stage1.zig:309-371 loadCamera, from the camera node's global matrix.
extern "C" int zrt_camera_from_matrix(const float m[16], float yfov, int has_aspect,
                                      float aspect, int32_t width, int32_t height,
                                      zrt_camera* out) {
    if (!m || !out) return ZRT_ERR_INVALID_ARG;
    uint32_t w, h;
    if (width < 0 && height < 0) return ZRT_ERR_CAMERA;          // OutputImgSizeIsNotSpecified
    if (width >= 0 && height >= 0) {
        if (has_aspect) return ZRT_ERR_CAMERA;                     // CameraHasAspectRatio
        w = (uint32_t)width;
        h = (uint32_t)height;
    } else {
        if (!has_aspect) return ZRT_ERR_CAMERA;                    // CameraHasntAspectRatio
        w = width >= 0 ? (uint32_t)width : f2u((float)height * aspect);
        h = height >= 0 ? (uint32_t)height : f2u((float)width / aspect);
    }
    const float fw = (float)w, fh = (float)h;
    const v3 origin = mk(m[12], m[13], m[14]);                     // col3(3)
    const v3 fwd = normalize(scale(mk(m[8], m[9], m[10]), -1.0f)); // -col3(2)
    const v3 right = normalize(cross(fwd, mk(0, 1, 0)));
    const v3 up = cross(fwd, right);
    const float focal = (fh / 2.0f) / tanf(yfov / 2.0f);
    const v3 llc = sub(sub(scale(fwd, focal), scale(right, fw / 2.0f)), scale(up, fh / 2.0f));
    out->w = w;
    out->h = h;
    const v3* src[4] = {&origin, &llc, &right, &up};
    float* dst[4] = {out->origin, out->lower_left_corner, out->right, out->up};
    for (int k = 0; k < 4; ++k) {
        dst[k][0] = src[k]->x;
        dst[k][1] = src[k]->y;
        dst[k][2] = src[k]->z;
    }
    return ZRT_OK;
}
