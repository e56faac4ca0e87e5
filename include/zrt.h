/*
 * zrt.h -- C ABI of the MI355X-native render hot path (libzrt.so).
 *
 * Drop-in boundary for the reference's render seam
 *     pub fn render(self: Scene, threads: []std.Thread, camera: Camera,
 *                   img: []RGB) !void                  (src/stage3.zig:247)
 * called once from src/main.zig:126.  The reference has no plugin registry;
 * its only FFI mechanism is @cImport of C headers (src/c.zig:1-5) plus a
 * static C library linked by build.zig:29-48, so a Zig host binds this
 * header the same way.
 *
 * Zig's @Vector(3, f32) (16-byte padded) and std.MultiArrayList are not
 * C-ABI, so the Scene is passed FLATTENED: plain pointers and sizes, caller
 * owned, read-only for the duration of the call.  All functions are
 * synchronous, return 0 (ZRT_OK) or a negative zrt_status, and never throw.
 * No torch types appear anywhere in this interface.
 */
#ifndef ZRT_H
#define ZRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZRT_ABI_VERSION 2      /* 2: device list in zrt_render_config, zrt_group_* */

typedef enum zrt_status {
    ZRT_OK = 0,
    ZRT_ERR_INVALID_ARG = -1,     /* null pointer, zero size, inconsistent scene */
    ZRT_ERR_NO_DEVICE = -2,       /* no HIP device / bad ordinal */
    ZRT_ERR_HIP = -3,             /* a HIP runtime call failed */
    ZRT_ERR_OUT_OF_MEMORY = -4,   /* host or device allocation failed */
    ZRT_ERR_UNSUPPORTED = -5,     /* e.g. max_bounce above the compiled stack depth */
    ZRT_ERR_IO = -6,              /* file open/read/write failed */
    ZRT_ERR_PARSE = -7,           /* glTF / JSON / PNG malformed */
    ZRT_ERR_NOT_FOUND = -8,       /* camera name not found, no cameras (stage1.zig:282-307) */
    ZRT_ERR_CAMERA = -9,          /* stage1.zig:322-342 width/height/aspect-ratio rules */
} zrt_status;

/* ---- scene (stage3.zig:136-143 Scene, flattened) ------------------------ */

/* linalg.zig:407-410 Grid */
typedef struct zrt_grid {
    float bbox_min[3];
    float bbox_max[3];
    uint32_t resolution[3];
    float cell_size[3];              /* (bbox_max - bbox_min) / resolution, f32 */
} zrt_grid;

/* stage3.zig:82-92 Texture(T).  `offset` indexes zrt_scene.texels in floats;
 * colour textures hold 3 floats per texel (linear RGB, factor applied),
 * transparency textures 1 float per texel.  Rows top to bottom.
 * u/v_min/max: [0, w-1] for CLAMP_TO_EDGE, [INT32_MIN, INT32_MAX] for repeat
 * (stage1.zig:381-409); a missing texture is a 1x1 texel = factor
 * (stage1.zig:411-425). */
typedef struct zrt_texture {
    uint64_t offset;
    int32_t w, h;
    int32_t u_min, u_max, v_min, v_max;
    int32_t _pad;
} zrt_texture;

/* stage3.zig:125-129 Material */
typedef struct zrt_material {
    zrt_texture base_color;          /* 3 floats/texel */
    zrt_texture emissive;            /* 3 floats/texel */
    zrt_texture transparency;        /* 1 float/texel  */
} zrt_material;

typedef struct zrt_scene {
    zrt_grid grid;
    uint32_t num_cells;              /* resolution[0]*resolution[1]*resolution[2] */
    const uint32_t* cells;           /* num_cells * {begin, end}   (stage3.zig:131-134) */
    uint32_t num_triangles;          /* baked refs: cell order, duplicated (stage2.zig:137-164) */
    const float* triangles_pos;      /* num_triangles * 9: v0, e1 = v1-v0, e2 = v2-v0 (linalg.zig:683-694) */
    const float* triangles_data;     /* num_triangles * 15: normal[3] x3, texcoord[2] x3 (stage3.zig:44-51) */
    const uint32_t* triangles_material; /* num_triangles (Data.material_idx) */
    uint32_t num_materials;
    const zrt_material* materials;
    const float* texels;
    uint64_t num_texel_floats;
} zrt_scene;

/* stage3.zig:19-26 Camera (built by stage1.zig:309-371) */
typedef struct zrt_camera {
    uint32_t w, h;
    float origin[3];
    float lower_left_corner[3];
    float right[3];
    float up[3];                     /* points world-down: row 0 is the top image row */
} zrt_camera;

/* main.zig:56-61 Config (num_samples/max_bounce) + device-side knobs that
 * the reference's config.json does not have (kept out of config.json). */
typedef struct zrt_render_config {
    uint32_t num_samples;            /* spp, 1..65535 (u16 in the reference) */
    uint32_t max_bounce;             /* recursion depth of traceRayRecursive */
    uint64_t seed;                   /* counter-RNG key (0 = default) */
    int32_t device;                  /* HIP ordinal, -1 = current device */
    uint32_t rank;                   /* this process's shard of the image */
    uint32_t num_ranks;              /* tiles t with t % num_ranks == rank */
    uint32_t tile_size;              /* square tile edge in pixels, 0 = 64 (32 over several devices) */
    uint32_t flags;                  /* ZRT_FLAG_* */
    uint32_t samples_per_pass;       /* samples of every pixel per device pass, 0 = automatic: as few
                                        passes as 144 GiB of path queues allow, at least two for frames
                                        of 2^23 samples or more (the image is the same for any value) */
    /* zrt_render only (ABI 2, in what were reserved words; zero = `device`
     * alone, one = devices[0] alone): the image's tiles split over
     * num_devices HIP ordinals, tile t
     * rendered on devices[t % num_devices] (repeats allowed), gathered into
     * rgb_out over xGMI -- the multi-device fan-out and join that
     * Scene.render does with its worker threads (stage3.zig:247-256). */
    uint32_t num_devices;
    uint32_t _reserved0;
    const int32_t* devices;
} zrt_render_config;

#define ZRT_FLAG_COUNT_STATS  0x1u   /* count cells/tests/hits (slower kernel variant) */
#define ZRT_FLAG_LANE_WALK    0x2u   /* every launch walks + tests per lane (no park kernel) */
/* 0x4, 0x8: reserved (round-2 kernel variants that were measured slower and removed) */
#define ZRT_FLAG_ONE_SET      0x10u  /* every pass on the context's one stream (no second pass set, no
                                        lead): kernels never overlap, so their durations are exclusive
                                        (the roofline measurement); same image */
#define ZRT_FLAG_KERNEL_TIMES 0x20u  /* HIP events around every kernel launch: per-kernel device times
                                        in zrt_context_profile (adds ~10 us per launch) */
#define ZRT_FLAG_ESCAPE       0x40u  /* the park walk always uses the escape table (by default only on
                                        scenes where enough of it is set to pay); same image */
#define ZRT_FLAG_NO_ESCAPE    0x80u  /* the park walk never uses the escape table; same image */
#define ZRT_FLAG_FRUSTUM      0x100u /* the primary launch always uses the frustum bounds (by default
                                        only for frames of 2^23 samples or more, where their build pays);
                                        same image */
#define ZRT_FLAG_NO_FRUSTUM   0x200u /* the primary launch never uses the frustum bounds (wins over
                                        ZRT_FLAG_FRUSTUM); same image */
#define ZRT_FLAG_MT_EXACT     0x400u /* every launch walks + tests per lane with the IEEE f32 division in
                                        Moller-Trumbore: what a context does by itself for a scene with
                                        an edge component of 2^62 or more or infinite (the other kernels'
                                        short reciprocal of the determinant holds for |det| < 2^126);
                                        same image */
#define ZRT_FLAG_RELEASE      0x800u /* the park kernel always skips test rounds with too few parked lanes
                                        that have refs to test (by default only on scenes where enough
                                        entry faces of the occupied cells have nothing left to test); same
                                        image */
#define ZRT_FLAG_NO_RELEASE   0x1000u /* never (wins over ZRT_FLAG_RELEASE); same image */

/* Per-call statistics.  segments = Scene.traceRay calls (primary + bounce +
 * transparency pass-through); Mrays/s = segments / render time. */
typedef struct zrt_stats {
    uint64_t segments;
    uint64_t cells_visited;          /* only with ZRT_FLAG_COUNT_STATS */
    uint64_t triangle_tests;         /* only with ZRT_FLAG_COUNT_STATS */
    uint64_t hits;                   /* only with ZRT_FLAG_COUNT_STATS */
    uint64_t samples;                /* pixels x spp rendered by this call */
    double render_ms;                /* device time: all kernels of the render */
    double trace_kernel_ms;          /* device time: path-trace kernel launches only */
    uint32_t trace_launches;
    uint32_t _pad;
} zrt_stats;

const char* zrt_error_string(int status);
int zrt_abi_version(void);
int zrt_device_count(int* count);
/* Optional: create the device's context and load the library's kernels now
 * (otherwise the first GPU call pays ~0.1-0.2 s), e.g. on a thread while the
 * host loads the scene.  device -1 = 0. */
int zrt_device_warmup(int device);

/* ---- stage 2: grid build + bake (stage2.zig:44-164) --------------------- */
typedef struct zrt_geometry zrt_geometry;

/* positions n*9 (v0,v1,v2 world space), normals n*9, texcoords n*6,
 * material n.  Inputs are read during the call only.  Deterministic:
 * identical to the single-threaded reference order (triangle order within
 * a cell), whatever the host thread count. */
int zrt_geometry_build(const float* positions, const float* normals, const float* texcoords,
                       const uint32_t* material, uint32_t num_triangles,
                       const uint32_t resolution[3], uint32_t num_threads, zrt_geometry** out);
/* The same build on a GPU: SAT binning, cell order and
 * bake as HIP kernels on device `device` (-1 = current).  Output identical
 * to zrt_geometry_build, bit for bit; the result lives in host memory like
 * the host build's.  Replaces Geometry.build + bakeInto (stage2.zig:131-164,
 * called at main.zig:117-118). */
int zrt_geometry_build_device(const float* positions, const float* normals, const float* texcoords,
                              const uint32_t* material, uint32_t num_triangles,
                              const uint32_t resolution[3], int device, zrt_geometry** out);
/* Fills grid/cells/triangle arrays of *scene (views into the geometry,
 * valid until zrt_geometry_free); leaves the material fields untouched. */
int zrt_geometry_scene(const zrt_geometry* g, zrt_scene* scene);
/* Source triangle index of each baked ref (stage2 Geometry.indices). */
int zrt_geometry_indices(const zrt_geometry* g, const uint32_t** indices, uint32_t* count);
void zrt_geometry_free(zrt_geometry* g);

/* ---- stage 3: the render seam ------------------------------------------ */

/* One-shot drop-in for Scene.render: uploads the scene, renders the whole
 * image on `cfg->device` -- or, with cfg->num_devices > 1, on every device of
 * cfg->devices (one host thread and one context per entry, interleaved 32x32
 * tiles by default -- cfg->tile_size overrides -- the packed tiles gathered
 * to the first device over xGMI) -- writes
 * w*h*3 RGB8 into rgb_out (caller-allocated, row 0 = top), frees device
 * memory, returns.  The image is bit-identical for any device list. */
int zrt_render(const zrt_scene* scene, const zrt_camera* camera, const zrt_render_config* cfg,
               uint8_t* rgb_out, zrt_stats* stats);

/* Device-resident path (scene uploaded once, many renders).  A context owns
 * its HIP streams: frames of 2^23 samples or more run their passes on two
 * streams (two pass sets, each with its own queues); zrt_context_render
 * returns once every stream is done, and device_rgb_packed is written on the
 * context's main stream after the join.  One thread at a time per context. */
typedef struct zrt_context zrt_context;

typedef struct zrt_outputs {
    uint8_t* rgb_image;              /* host w*h*3; only this rank's pixels are written */
    uint8_t* rgb_packed;             /* host n_owned*3 in zrt_tile_pixels order */
    float* linear_packed;            /* host n_owned*3: pixel sum * (1/spp), pre-toRGB */
    void* device_rgb_packed;         /* device n_owned*3 on the context's device */
} zrt_outputs;

/* Every finite, infinite or NaN coordinate is taken, as in the reference
 * (linalg.zig:696-722).  A scene with a triangle edge component
 * (scene->triangles_pos e1, e2) of magnitude 2^62 or more or infinite -- a
 * vertex component (positions) of 2^61 or more for the device build --
 * renders through the lane walk with the IEEE division (ZRT_FLAG_MT_EXACT),
 * since the other kernels' short reciprocal of the Moller-Trumbore
 * determinant is exact for |det| < 2^126 only. */
int zrt_context_create(const zrt_scene* scene, int device, zrt_context** out);
/* Geometry.build + bakeInto (stage2.zig:44-164, main.zig:117-118) and the
 * stage-3 upload in one step: the grid is built on `device` straight into the
 * context's HBM arrays (no host copy of the baked scene).  Renders exactly as
 * zrt_geometry_build + zrt_geometry_scene + zrt_context_create. */
int zrt_context_create_built(const float* positions, const float* normals, const float* texcoords,
                             const uint32_t* material, uint32_t num_triangles, const uint32_t resolution[3],
                             uint32_t num_materials, const zrt_material* materials, const float* texels,
                             uint64_t num_texel_floats, int device, zrt_context** out);
int zrt_context_render(zrt_context* ctx, const zrt_camera* camera, const zrt_render_config* cfg,
                       const zrt_outputs* outputs, zrt_stats* stats);
void zrt_context_destroy(zrt_context* ctx);

/* A device group: one context per entry of `devices` (HIP ordinals, repeats
 * allowed), the scene resident on each, rendered by one call -- Scene.render's
 * spawn + join of its workers (stage3.zig:247-256) across GPUs in one
 * process.  zrt_group_render splits this process's share of the image (the
 * tiles t with t % cfg->num_ranks == cfg->rank; cfg->device is ignored) over
 * the devices, device i taking sub-rank i, on one host thread each; with
 * num_ranks <= 1 the devices' packed tiles are copied to devices[0] (peer copy
 * over xGMI), scattered into the image there and copied to rgb_out once,
 * otherwise each device's pixels are written into rgb_out from the host (other
 * pixels untouched).  stats: sums over devices; render_ms = the slowest. */
typedef struct zrt_group zrt_group;
int zrt_group_create(const zrt_scene* scene, const int32_t* devices, uint32_t num_devices, zrt_group** out);
/* Geometry.build + bakeInto on every device of the group (as
 * zrt_context_create_built; the builds run in parallel, bit-identical). */
int zrt_group_create_built(const float* positions, const float* normals, const float* texcoords,
                           const uint32_t* material, uint32_t num_triangles, const uint32_t resolution[3],
                           uint32_t num_materials, const zrt_material* materials, const float* texels,
                           uint64_t num_texel_floats, const int32_t* devices, uint32_t num_devices,
                           zrt_group** out);
int zrt_group_render(zrt_group* g, const zrt_camera* camera, const zrt_render_config* cfg, uint8_t* rgb_out,
                     zrt_stats* stats);
/* The group's i-th context (owned by the group), e.g. for zrt_context_grid_info. */
int zrt_group_context(zrt_group* g, uint32_t i, zrt_context** out);
void zrt_group_destroy(zrt_group* g);

/* Per-kernel breakdown of the context's last zrt_context_render (bench.py's
 * roofline: the dominant kernel's launch time and algorithmic work).
 * ms / launches per kernel class; ms only with ZRT_FLAG_KERNEL_TIMES (else 0).
 * primary_counts: segments, cells visited, triangle tests, hits of the
 * primary (camera) segments, counting renders (ZRT_FLAG_COUNT_STATS) only --
 * the bounce launches' work is zrt_stats' totals minus these. */
enum {
    ZRT_KERNEL_PRIMARY = 0,   /* wf_kernel, primary launch (camera rays) */
    ZRT_KERNEL_PARK = 1,      /* wf_park_kernel, bounce trace */
    ZRT_KERNEL_SHADE = 2,     /* wf_shade_kernel, bounce shading */
    ZRT_KERNEL_BOUNCE = 3,    /* wf_kernel, bounce launch (lane walk / no OccX) */
    ZRT_KERNEL_RESOLVE = 4,   /* wf_resolve_kernel / resolve_kernel */
    ZRT_KERNEL_COUNT = 5,     /* trace_kernel (counting build) */
    ZRT_KERNEL_CLASSES = 8
};
typedef struct zrt_kernel_profile {
    double ms[ZRT_KERNEL_CLASSES];
    uint32_t launches[ZRT_KERNEL_CLASSES];
    uint32_t passes;                 /* passes of the frame */
    uint32_t sets;                   /* pass sets (streams) it ran on */
    uint64_t primary_counts[4];
} zrt_kernel_profile;
int zrt_context_profile(const zrt_context* ctx, zrt_kernel_profile* out);

/* The context's grid and {num_refs, empty cells, min refs of a non-empty cell
 * (0xFFFFFFFF if none), max refs of a cell}: the grid statistics the
 * reference logs after Geometry.build (main.zig:117-118), without a host copy
 * of the cells. */
int zrt_context_grid_info(zrt_context* ctx, zrt_grid* grid, uint32_t info[4]);

/* Pixels owned by `rank` (row-major image indices) in the packed output
 * order: tiles t = rank, rank+num_ranks, ... (row-major tile order), each
 * tile walked in 8x8 blocks.  pixels may be NULL to query *count. */
int zrt_tile_pixels(uint32_t w, uint32_t h, uint32_t tile_size, uint32_t rank,
                    uint32_t num_ranks, uint32_t* pixels, uint32_t* count);

/* ---- stage 1: glTF scene load + camera (stage1.zig) --------------------- */
typedef struct zrt_gltf zrt_gltf;

/* Loads .gltf (+ .bin, + PNG images) or .glb; triangle soup in node order
 * (stage1.zig:217-259), materials (stage1.zig:381-496), cameras. */
int zrt_gltf_load(const char* path, uint32_t num_threads, zrt_gltf** out);
int zrt_gltf_soup(const zrt_gltf* g, const float** positions, const float** normals,
                  const float** texcoords, const uint32_t** material, uint32_t* num_triangles);
/* Fills the material/texel fields of *scene (views valid until free). */
int zrt_gltf_materials(const zrt_gltf* g, zrt_scene* scene);
/* stage1.zig:309-371; width/height < 0 mean "not given". */
int zrt_gltf_camera(const zrt_gltf* g, const char* camera_name, int32_t width, int32_t height,
                    zrt_camera* out);
void zrt_gltf_free(zrt_gltf* g);

/* stage1.zig:309-371 from an explicit node matrix (column-major 16). */
int zrt_camera_from_matrix(const float matrix[16], float yfov, int has_aspect_ratio,
                           float aspect_ratio, int32_t width, int32_t height, zrt_camera* out);

/* ---- device-function parity probes (tests only; run on the GPU) -------- */
enum {
    ZRT_PROBE_TRIANGLE = 0,   /* in n*15 (v0,v1,v2,orig,dir) -> out n*4 (hit,t,u,v) */
    ZRT_PROBE_BBOX = 1,       /* in n*12 (min,max,orig,dir) -> out n*2 (hit,t) */
    ZRT_PROBE_DDA = 2,        /* in n*12 (min,max,orig,dir) + res u32[3] in aux -> out n*(4+4*64):
                                 steps (-1 miss, -2 bad linear index), first cell, (cell, t) per next() */
    ZRT_PROBE_TO_RGB = 3,     /* in n*3 -> out n*3 (as float) */
    ZRT_PROBE_RNG_F32 = 4,    /* in n*3 u32 (seed_lo,pixel,sample) -> out n*16 floats */
    ZRT_PROBE_RNG_NORM = 5,   /* same -> out n*16 floats */
    ZRT_PROBE_EXP_LOG = 6,    /* in n doubles -> out n*2 doubles (exp, log) */
    ZRT_PROBE_TEXTURE = 7,    /* in n*2 (u,v) + aux texture -> out n*3 */
    ZRT_PROBE_TRIANGLE_FLAT = 8, /* as TRIANGLE, through the branch-free test of the park kernel */
    ZRT_PROBE_RECIP = 9,      /* in n floats det -> out n*2: the park / packed kernels' short 1/det
                                 (rcp + six FMAs), the IEEE-division kernels' 1.0f/det */
    ZRT_PROBE_RECIP_SWEEP = 10, /* in n*2 u32 {first float bits, count} -> out n*4 u32 {floats whose
                                 short 1/det differs in any bit from the device's IEEE 1.0f/det (NaN
                                 equals NaN), the smallest such bits (0xFFFFFFFF: none), 0, 0};
                                 every float of each range, on the device */
    ZRT_PROBE_TRIANGLE_EXACT = 11, /* as TRIANGLE, with the IEEE division of the ZRT_FLAG_MT_EXACT kernels */
    ZRT_PROBE_QUOT = 12,      /* in n*2 floats (a, b) -> out n*2: dda_init_fq's quotient quot_rn(a, b,
                                 1/b by the short reciprocal), the IEEE a / b */
    ZRT_PROBE_QUOT_SWEEP = 13, /* in n*2 u32 {first significand s_b, count} -> out n*4 u32 {pairs whose
                                 quot_rn differs in any bit from the IEEE quotient, the first such a's
                                 bits, its b's bits, 0}: every a in [1, 2) against every
                                 b = 1 + s / 2^23, s in [s_b, s_b + count), on the device */
};
int zrt_probe(int which, const void* in, void* out, uint32_t n, const void* aux, int device);
/* Comma-separated substrings of the mangled names of the timed kernel
 * instantiations in the gfx950 code object (build checks; no HIP call). */
const char* zrt_timed_kernels(void);

#ifdef __cplusplus
}
#endif
#endif /* ZRT_H */
