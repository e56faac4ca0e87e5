// group.hip -- several GPUs behind one render call (zrt_group_*, and
// zrt_render with a device list).
//
// Reference: Scene.render (src/stage3.zig:247-256) spawns one worker per
// thread over contiguous pixel blocks (stage3.zig:228-229) and joins them
// before it returns.  Here the workers are GPUs: one context per device, the
// image's 32x32 tiles (tile_size overrides) interleaved over them (tile t -> device t % n, for
// balance: sky rows are cheap), one host thread per device driving its
// context, and the join is a gather: every device's packed RGB8 tiles are
// copied to the first device (hipMemcpyPeerAsync: a DMA over xGMI when peer
// access is on), scattered into the row-major image there by one kernel and
// copied to the caller once.  The RNG is keyed by global pixel, so the image
// is the one-device image bit for bit, whatever the list (repeats allowed:
// two contexts on one GPU).  No collective library: within one process a
// peer copy is the gather; RCCL serves the one-process-per-GPU path
// (bench.py / dist.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "zrt_internal.h"

#define GROUP_TRY(expr)                                                          \
    do {                                                                         \
        hipError_t _e = (expr);                                                  \
        if (_e != hipSuccess) return _e == hipErrorOutOfMemory ? ZRT_ERR_OUT_OF_MEMORY : ZRT_ERR_HIP; \
    } while (0)

namespace {

// img[pixel[q]] = packed[q] for the concatenated packed tiles of every device
__global__ __launch_bounds__(256) void unpermute_kernel(const uint8_t* __restrict__ packed,
                                                        const uint32_t* __restrict__ pixels, uint32_t n,
                                                        uint8_t* __restrict__ img) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= n) return;
    const uint32_t p = pixels[q];
    img[3ull * p + 0] = packed[3ull * q + 0];
    img[3ull * p + 1] = packed[3ull * q + 1];
    img[3ull * p + 2] = packed[3ull * q + 2];
}

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct zrt_group {
    std::vector<int> devices;
    std::vector<zrt_context*> ctx;
    hipStream_t stream = nullptr;              // on devices[0]: the gather (the first context's, not owned)
    uint8_t* d_gather = nullptr; size_t gather_cap = 0;   // every device's packed tiles, device order
    uint8_t* d_img = nullptr; size_t img_cap = 0;
    uint32_t* d_pix = nullptr; size_t pix_cap = 0;        // their pixel indices, same order
    uint32_t pix_key[4] = {0, 0, 0, 0};
    bool pix_valid = false;
};

namespace {

int check_devices(const int32_t* devices, uint32_t n) {
    if (!devices || n == 0) return ZRT_ERR_INVALID_ARG;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return ZRT_ERR_NO_DEVICE;
    for (uint32_t i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= count) return ZRT_ERR_NO_DEVICE;
    return ZRT_OK;
}

// The shared tail of both create calls: contexts made on one thread per
// device by `make(i, &ctx)`, peer access from the first device to the others.
template <typename Make>
int group_create(const int32_t* devices, uint32_t n, zrt_group** out, Make make) {
    if (!out) return ZRT_ERR_INVALID_ARG;
    *out = nullptr;
    int rc = check_devices(devices, n);
    if (rc != ZRT_OK) return rc;
    zrt_group* g = new (std::nothrow) zrt_group();
    if (!g) return ZRT_ERR_OUT_OF_MEMORY;
    g->devices.assign(devices, devices + n);
    g->ctx.assign(n, nullptr);
    std::vector<int> rcs(n, ZRT_OK);
    {
        std::vector<std::thread> th;
        for (uint32_t i = 0; i < n; ++i) th.emplace_back([&, i] { rcs[i] = make(i, &g->ctx[i]); });
        for (auto& t : th) t.join();
    }
    for (int r : rcs)
        if (r != ZRT_OK) rc = r;
    if (rc == ZRT_OK)        // repeats of a device render side by side: split its queue budget
        for (uint32_t i = 0; i < n; ++i)
            zrt::context_set_mem_share(g->ctx[i], (uint32_t)std::count(g->devices.begin(), g->devices.end(),
                                                                        g->devices[i]));
    if (rc == ZRT_OK) {
        DevGuard dg(g->devices[0]);
        for (uint32_t i = 1; i < n; ++i) {
            if (g->devices[i] == g->devices[0]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, g->devices[0], g->devices[i]) == hipSuccess && can) {
                const hipError_t e = hipDeviceEnablePeerAccess(g->devices[i], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) rc = ZRT_ERR_HIP;
                (void)hipGetLastError();   // clear an "already enabled" status
            }
        }
        // the gather runs on the first context's stream (on devices[0]; idle
        // once its render has returned): no stream of the group's own
        if (rc == ZRT_OK) g->stream = (hipStream_t)zrt::context_stream(g->ctx[0]);
    }
    if (rc != ZRT_OK) {
        zrt_group_destroy(g);
        return rc;
    }
    *out = g;
    return ZRT_OK;
}

template <typename T>
int grow_on(T** p, size_t* cap, size_t n) {
    if (*cap >= n && *p) return ZRT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    GROUP_TRY(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
    *cap = n;
    return ZRT_OK;
}

}  // namespace

extern "C" int zrt_group_create(const zrt_scene* scene, const int32_t* devices, uint32_t num_devices,
                                zrt_group** out) {
    if (!scene) return ZRT_ERR_INVALID_ARG;
    return group_create(devices, num_devices, out,
                        [&](uint32_t i, zrt_context** c) { return zrt_context_create(scene, devices[i], c); });
}

extern "C" int zrt_group_create_built(const float* positions, const float* normals, const float* texcoords,
                                      const uint32_t* material, uint32_t num_triangles,
                                      const uint32_t resolution[3], uint32_t num_materials,
                                      const zrt_material* materials, const float* texels,
                                      uint64_t num_texel_floats, const int32_t* devices, uint32_t num_devices,
                                      zrt_group** out) {
    return group_create(devices, num_devices, out, [&](uint32_t i, zrt_context** c) {
        return zrt_context_create_built(positions, normals, texcoords, material, num_triangles, resolution,
                                        num_materials, materials, texels, num_texel_floats, devices[i], c);
    });
}

extern "C" int zrt_group_context(zrt_group* g, uint32_t i, zrt_context** out) {
    if (!g || !out || i >= g->ctx.size()) return ZRT_ERR_INVALID_ARG;
    *out = g->ctx[i];
    return ZRT_OK;
}

extern "C" void zrt_group_destroy(zrt_group* g) {
    if (!g) return;
    for (zrt_context* c : g->ctx) zrt_context_destroy(c);
    if (!g->devices.empty()) {
        DevGuard dg(g->devices[0]);
        if (g->d_gather) (void)hipFree(g->d_gather);
        if (g->d_img) (void)hipFree(g->d_img);
        if (g->d_pix) (void)hipFree(g->d_pix);
    }
    delete g;
}

extern "C" int zrt_group_render(zrt_group* g, const zrt_camera* cam, const zrt_render_config* cfg, uint8_t* rgb_out,
                                zrt_stats* stats) {
    if (!g || !cam || !cfg || !rgb_out || g->ctx.empty()) return ZRT_ERR_INVALID_ARG;
    const uint32_t n = (uint32_t)g->ctx.size();
    const uint32_t nr = cfg->num_ranks ? cfg->num_ranks : 1u;
    if (cfg->rank >= nr || (uint64_t)nr * n > 0xFFFFFFFFull) return ZRT_ERR_INVALID_ARG;
    // 32x32 tiles by default over several devices: the 8-rank tile-time
    // spread of cfg3 is 0.934 of ideal against 0.906 with 64x64
    const uint32_t tile = cfg->tile_size ? cfg->tile_size : (n * nr > 1u ? 32u : 64u);
    const bool whole = nr == 1;                // the whole image: gather on device 0
    std::vector<int> rcs(n, ZRT_OK);
    std::vector<zrt_stats> st(n);
    {
        std::vector<std::thread> th;
        for (uint32_t i = 0; i < n; ++i)
            th.emplace_back([&, i] {
                zrt_render_config c = *cfg;
                c.device = g->devices[i];
                // device i takes the i-th of every n of this process's tiles
                // (t % nr == rank, (t / nr) % n == i): t % (nr n) == rank + nr i
                c.rank = cfg->rank + nr * i;
                c.num_ranks = nr * n;
                c.tile_size = tile;
                c.num_devices = 0;
                c.devices = nullptr;
                zrt_outputs o{};
                if (!whole) o.rgb_image = rgb_out;   // disjoint pixels per device
                rcs[i] = zrt_context_render(g->ctx[i], cam, &c, &o, &st[i]);
            });
        for (auto& t : th) t.join();
    }
    for (int r : rcs)
        if (r != ZRT_OK) return r;
    if (whole) {
        const int dev0 = g->devices[0];
        DevGuard dg(dev0);
        const uint64_t npx = (uint64_t)cam->w * cam->h;
        int rc;
        const uint32_t key[4] = {cam->w, cam->h, tile, n};
        if (!g->pix_valid || memcmp(key, g->pix_key, sizeof key) != 0) {
            std::vector<uint32_t> all(npx);
            uint64_t off = 0;
            for (uint32_t i = 0; i < n; ++i) {
                uint32_t cnt = 0;
                if ((rc = zrt::tile_pixels(cam->w, cam->h, tile, i, n, all.data() + off, &cnt)) != ZRT_OK) return rc;
                off += cnt;
            }
            if (off != npx) return ZRT_ERR_INVALID_ARG;
            if ((rc = grow_on(&g->d_pix, &g->pix_cap, npx)) != ZRT_OK) return rc;
            GROUP_TRY(hipMemcpyAsync(g->d_pix, all.data(), npx * 4, hipMemcpyHostToDevice, g->stream));
            GROUP_TRY(hipStreamSynchronize(g->stream));
            memcpy(g->pix_key, key, sizeof key);
            g->pix_valid = true;
        }
        if ((rc = grow_on(&g->d_gather, &g->gather_cap, 3 * npx)) != ZRT_OK) return rc;
        if ((rc = grow_on(&g->d_img, &g->img_cap, 3 * npx)) != ZRT_OK) return rc;
        uint64_t off = 0;
        for (uint32_t i = 0; i < n; ++i) {     // device i's packed tiles -> device 0 (xGMI DMA)
            const uint8_t* src = nullptr;
            uint32_t P = 0;
            int dev = 0;
            if ((rc = zrt::context_device_rgb(g->ctx[i], &src, &P, &dev)) != ZRT_OK) return rc;
            if (P == 0) continue;
            if (dev == dev0)
                GROUP_TRY(hipMemcpyAsync(g->d_gather + 3 * off, src, 3ull * P, hipMemcpyDeviceToDevice, g->stream));
            else
                GROUP_TRY(hipMemcpyPeerAsync(g->d_gather + 3 * off, dev0, src, dev, 3ull * P, g->stream));
            off += P;
        }
        if (off != npx) return ZRT_ERR_INVALID_ARG;
        hipLaunchKernelGGL(unpermute_kernel, dim3((uint32_t)((npx + 255) / 256)), dim3(256), 0, g->stream,
                           (const uint8_t*)g->d_gather, (const uint32_t*)g->d_pix, (uint32_t)npx, g->d_img);
        GROUP_TRY(hipGetLastError());
        GROUP_TRY(hipMemcpyAsync(rgb_out, g->d_img, 3 * npx, hipMemcpyDeviceToHost, g->stream));
        GROUP_TRY(hipStreamSynchronize(g->stream));
    }
    if (stats) {
        zrt_stats s{};
        for (const zrt_stats& x : st) {
            s.segments += x.segments;
            s.cells_visited += x.cells_visited;
            s.triangle_tests += x.triangle_tests;
            s.hits += x.hits;
            s.samples += x.samples;
            s.render_ms = std::max(s.render_ms, x.render_ms);
            s.trace_kernel_ms += x.trace_kernel_ms;
            s.trace_launches += x.trace_launches;
        }
        *stats = s;
    }
    return ZRT_OK;
}
