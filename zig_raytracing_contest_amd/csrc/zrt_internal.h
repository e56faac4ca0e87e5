// zrt_internal.h -- types shared by the host code and the CDNA4 kernels.
#pragma once
#include <cstring>

#include "../../include/zrt.h"
#include "zrt_math.h"

namespace zrt {

// Device texture descriptor (stage3.zig:82-92): offset in floats into the
// texel pool; chans = 3 for colour, 1 for transparency.
struct DevTex {
    uint32_t off;
    int32_t w, h, umin, umax, vmin, vmax;
    uint32_t pad;
};
struct DevMat { DevTex tex[3]; };   // base_color, emissive, transparency
// A 1x1 texture (every material slot without an image, stage1.zig:411-425)
// needs no clamp range (any clamp and @mod by 1 give texel 0), so its texel
// rides in those fields instead: channel k's f32 bits in (umin, umax,
// vmin)[k].  Sampling then reads it from the material (LDS in the shade
// kernel) instead of the texel pool.
ZHD void dev_tex_inline(DevTex& d, const float* texels, int chans) {
    if (d.w != 1 || d.h != 1) return;
    int32_t* f[3] = {&d.umin, &d.umax, &d.vmin};
    for (int k = 0; k < chans; ++k) memcpy(f[k], texels + d.off + k, 4);
}

// Ziggurat NormDist tables (Zig std ziggurat.zig ZigTableGen), computed on the
// host with the deterministic exp/log of zrt_math.h.
void zig_tables(double zx[257], double zf[257]);

// Host threads for "all CPUs" (config.json num_threads null, main.zig:90
// getCpuCount): the CPUs this process may run on, capped by OMP_NUM_THREADS
// when set (the per-GPU CPU share on shared GPU hosts).
unsigned host_threads();

// Whether the park kernel's exact per-cell occupancy (OccX) serves a grid:
// its 4^3-cell bricks need 24-bit indices (__umul24 in the kernels), the
// occupied-brick count before a 32-brick word must fit the u16 prefix, and
// the blob must fit the LDS left beside the per-wave slots.  Otherwise the
// bounces take the lane walk (wf_kernel, coarsened brick bits): the render
// still runs, on every grid the reference accepts (u32 resolution, < 2^31
// cells), with the same image.
inline bool occx_usable(uint64_t bricks, uint64_t occupied, uint64_t lds_bytes, uint64_t budget) {
    return bricks <= (1ull << 24) && occupied < 0xFFFFull && lds_bytes <= budget;
}

// Host-side packed pixel order of one rank (zrt_tile_pixels).
int tile_pixels(uint32_t w, uint32_t h, uint32_t tile, uint32_t rank, uint32_t nranks,
                uint32_t* out, uint32_t* count);

// The packed RGB8 of a context's last render (device memory on its device,
// 3 * pixels bytes in its rank's zrt_tile_pixels order): what a device group
// gathers (group.hip).
int context_device_rgb(const zrt_context* c, const uint8_t** d_rgb, uint32_t* pixels, int* device);

// Contexts of one group that share a device render at the same time: each
// sizes its passes from 1/share of the device's queue budget (group.hip sets
// share = how often the device appears in the list).
void context_set_mem_share(zrt_context* c, uint32_t share);

// The context's main HIP stream (as a void*: this header has no HIP types):
// a group gathers on its first context's stream instead of creating one of
// its own (a stream's first hardware queue cost ~10-17 ms of the CLI's
// start-up, r06d).
void* context_stream(const zrt_context* c);

}  // namespace zrt
