/*
 * zrt_oracle.h -- CPU restatement of the reference render hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / CPU baseline.  The product (zig_raytracing_contest_amd/libzrt.so)
 * never links, loads or calls anything here.
 *
 * What it restates (all paths relative to the reference checkout):
 *   src/linalg.zig   vector ops, Bbox.rayIntersection, Grid + Iterator (DDA),
 *                    intersectsTriangleAabb (SAT), Triangle.rayIntersection,
 *                    toRGB, randomUnitVector
 *   src/stage2.zig   Geometry.build (initGrid/initCells/initIndices) + bakeInto
 *   src/stage3.zig   Camera.getRay, Triangle.Data.interpolate, Texture.sample,
 *                    getEnvColor, traceRay, traceRayRecursive, renderWorker
 *   src/stage1.zig   loadCamera basis (camera from a node matrix + yfov)
 *   Zig 0.11 std     Xoshiro256++/SplitMix64 (DefaultPrng), Random.float,
 *                    ziggurat floatNorm, math.lerp (= @mulAdd), math.pow
 *
 * Pinning: the reference cannot be built here (no zig toolchain, empty
 * submodules).  The oracle is pinned by porting every
 * known-answer test the reference holds for this path (linalg.zig:9-11,
 * 231-241, 352-405, 565-681) -> tests/test_oracle_kat.py.  Everything the
 * reference does not test (Moller-Trumbore, SAT, textures, RNG streams,
 * full images) is "parity unpinned" w.r.t. the reference and is pinned only
 * by analytic cases + committed golden vectors produced by this oracle.
 *
 * Two RNG modes:
 *   ORC_RNG_REF   : Xoshiro256++ seeded per worker thread with its index and
 *                   contiguous pixel blocks, exactly as stage3.zig:222-245.
 *   ORC_RNG_PATH  : counter-based stream keyed by (seed, pixel, sample) --
 *                   the stream the GPU kernel uses, so GPU == oracle bitwise.
 */
#ifndef ZRT_ORACLE_H
#define ZRT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_RNG_REF = 0, ORC_RNG_PATH = 1 };

/* ---- opaque scene ------------------------------------------------------ */
typedef struct orc_scene orc_scene;

/* Build + bake (stage2.zig:44-164).  pos: n*9 floats (v0,v1,v2); nrm: n*9;
 * uv: n*6; mat: n material indices.  Inputs are copied. */
orc_scene* orc_scene_build(const float* pos, const float* nrm, const float* uv,
                           const uint32_t* mat, uint32_t n, const uint32_t res[3]);
void orc_scene_free(orc_scene* s);
uint32_t orc_scene_num_refs(const orc_scene* s);
/* grid6 = bbox min/max, cell3 = cell size; cells = 2*ncells (begin,end);
 * indices = num_refs source-triangle indices in cell order */
void orc_scene_get(const orc_scene* s, float grid_bbox[6], float cell_size[3],
                   uint32_t* cells, uint32_t* indices);

/* Materials: per material 3 textures (base_color, emissive, transparency),
 * each 7 int32: {offset (floats into texels), w, h, u_min, u_max, v_min, v_max}.
 * Colour textures hold 3 floats/texel, transparency 1 float/texel. */
void orc_scene_set_materials(orc_scene* s, uint32_t n_mat, const int32_t* tex_desc,
                             const float* texels, uint64_t n_texel_floats);

/* camera: w,h + origin, lower_left_corner, right, up (12 floats) */
typedef struct orc_camera {
    uint32_t w, h;
    float origin[3], llc[3], right[3], up[3];
} orc_camera;

/* stage1.zig:309-371 given the node's global matrix (column-major 16) */
int orc_camera_from_matrix(const float m[16], float yfov, int has_aspect, float aspect,
                           int width, int height, orc_camera* out);

/* counters: [0]=segments (traceRay calls) [1]=cells visited [2]=triangle tests
 * [3]=hits [4]=samples */
int orc_render(const orc_scene* s, const orc_camera* cam, uint32_t spp, uint32_t max_bounce,
               int rng_mode, uint64_t seed, uint32_t num_threads,
               uint32_t px_begin, uint32_t px_end,
               uint8_t* rgb /* (px_end-px_begin)*3 or NULL */,
               float* linear /* (px_end-px_begin)*3: pixel sum * inv_spp, or NULL */,
               uint64_t counters[5]);

/* Same as orc_render for an explicit list of pixels (the list is the
 * "image" that REF mode partitions into contiguous per-thread blocks). */
int orc_render_pixels(const orc_scene* s, const orc_camera* cam, uint32_t spp,
                      uint32_t max_bounce, int rng_mode, uint64_t seed, uint32_t num_threads,
                      const uint32_t* pixels, uint32_t n, uint8_t* rgb, float* linear,
                      uint64_t counters[5]);

/* ---- unit entry points (known-answer tests, device-function parity) ---- */
int   orc_bbox_ray(const float bbox[6], const float orig[3], const float dir[3], float* t);
/* DDA: writes up to max_steps (cell xyz, t returned by next()); returns #steps
 * written (the last entry has t=+inf if exit was reached); returns -1 on miss. */
int   orc_grid_trace(const float bbox[6], const uint32_t res[3], const float orig[3],
                     const float dir[3], uint32_t* cells_out, float* t_out, int max_steps,
                     uint32_t first_cell[3]);
void  orc_grid_cell_bbox(const float bbox[6], const uint32_t res[3], uint32_t x, uint32_t y,
                         uint32_t z, float out[6]);
int   orc_tri_intersect(const float v0[3], const float v1[3], const float v2[3],
                        const float orig[3], const float dir[3], float tuv[3]);
int   orc_tri_aabb(const float tri[9], const float bbox[6]);
void  orc_cross(const float a[3], const float b[3], float out[3]);
float orc_length(const float v[3]);
void  orc_to_rgb(const float v[3], uint8_t out[3]);
float orc_powf(float x, float y);
double orc_exp(double x);
double orc_log(double x);
void  orc_env(const float dir[3], float out[3]);
/* texture sampling: chans 3 or 1 */
void  orc_tex_sample(const float* data, int chans, int w, int h, int u_min, int u_max,
                     int v_min, int v_max, float u, float v, float* out);
/* RNG streams */
void  orc_xoshiro_u64(uint64_t seed, uint64_t* out, int n);
void  orc_splitmix_u64(uint64_t seed, uint64_t* out, int n);   /* SplitMix64.init(seed).next() x n */
void  orc_path_u64(uint64_t seed, uint32_t pixel, uint32_t sample, uint64_t* out, int n);
void  orc_path_f32(uint64_t seed, uint32_t pixel, uint32_t sample, float* out, int n);
void  orc_path_norm(uint64_t seed, uint32_t pixel, uint32_t sample, float* out, int n);
void  orc_xoshiro_f32(uint64_t seed, float* out, int n);
void  orc_xoshiro_norm(uint64_t seed, float* out, int n);
void  orc_zig_tables(double x[257], double f[257]);

#ifdef __cplusplus
}
#endif
#endif
