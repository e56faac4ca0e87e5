// render.hip -- the render hot path on CDNA4 (gfx950): wavefront path-trace
// kernels + in-order sample resolve, behind the C ABI of include/zrt.h.
//
// Reference: Scene.render / renderWorker / traceRayRecursive / traceRay
// (src/stage3.zig:152-256) over Grid.traceRay + Iterator.next
// (src/linalg.zig:443-496) and Triangle.rayIntersection (linalg.zig:696-722).
//
// Organisation (MI355X-first, not the reference's thread blocks):
//   * a work item is ONE path sample (pixel, sample); items are numbered
//     pixel-major over this rank's packed pixel list (tile_size tiles, 64x64 by
//     default on one device, walked in 8x8 blocks), item = pixel * S + sample of the pass, so one wave64 of
//     the primary launch = 64 samples of one pixel (coherent primary rays)
//     and its records are contiguous;
//   * bounce k of every path of a pass is one launch over a compacted queue
//     of the paths still alive (wavefront organisation); each lane traces one
//     Scene.traceRay segment and shades it (traceRayRecursive's body);
//   * the per-bounce (emissive, albedo) pairs go to HBM planes and the resolve
//     kernel folds them back to front per sample, then sums the samples IN
//     SAMPLE ORDER (renderWorker's `pixel = pixel.add(ray_color)`), scales by
//     the f32 reciprocal of spp and quantizes with toRGB: the image is
//     bit-identical to the recursion's for any scheduling.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <new>
#include <vector>

#include "zrt_internal.h"
#include "dda.h"
#include "escape.h"
#include "device_geometry.h"

using namespace zrt;

#define HIP_TRY(expr)                                                            \
    do {                                                                         \
        hipError_t _e = (expr);                                                  \
        if (_e != hipSuccess) {                                                  \
            if (getenv("ZRT_DEBUG"))                                             \
                fprintf(stderr, "zrt: %s failed: %s (%s:%d)\n", #expr,           \
                        hipGetErrorString(_e), __FILE__, __LINE__);              \
            return _e == hipErrorOutOfMemory ? ZRT_ERR_OUT_OF_MEMORY : ZRT_ERR_HIP; \
        }                                                                        \
    } while (0)

namespace {

constexpr float kFltEps = 1.1920928955078125e-07f;   // std.math.floatEps(f32)
constexpr int kBlock = 256;                          // resolve / probes / helpers
constexpr int kTraceBlock = 512;                     // launch bound of wf_kernel / trace_kernel
constexpr int kTraceThreads = 256;                   // threads per wf_kernel / trace_kernel block
// (r03ze, full spp: 1 -1.3 / -0.6 / -1.5%, 3 -0.6 / -0.2 / -0.6% on cfg3 /
// cfg2 / cfg5; 3 spills inside the primary's cell walk).  Round 6, with the
// entry-face skip testing fewer refs per cell: 1 at 7 waves per SIMD (70
// VGPRs, no spill) against 2 at 6 (r06bi + r06bj, 5 rounds): cfg3 +1.7 /
// -0.05%, cfg2 +2.2 / +1.0%, cfg5 +0.35 / +0.5%; 1 at 6 waves: cfg3 -0.6%
#ifndef ZRT_TRI_BATCH
#define ZRT_TRI_BATCH 1
#endif
constexpr int kTriBatch = ZRT_TRI_BATCH;             // triangle loads in flight per lane
#ifndef ZRT_PARK_BLOCK_T
#define ZRT_PARK_BLOCK_T 1024
#endif
constexpr int kParkBlock = ZRT_PARK_BLOCK_T;         // wf_park_kernel: one workgroup per CU
// (3 entries since r05t: 113 VGPRs, which fit beside the park kernel at 96,
// ZRT_PARK_WPE; one-stream shade 18.9 -> 17.1 ms per cfg3 frame)
#ifndef ZRT_SHADE_N
#define ZRT_SHADE_N 3
#endif
constexpr int kShadeEntries = ZRT_SHADE_N;           // wf_shade_kernel: queue entries per lane per fetch
#ifndef ZRT_WF_CHUNK
#define ZRT_WF_CHUNK 3
#endif
// wf_kernel: 64-entry batches per work atomic (r02d1: 2 vs 1 cfg3 +0.35%,
// cfg2 +0.9%, cfg5 +0.2%; 4: +0.6 / +0.5 / 0%; on round 5's final tree 3 vs
// 2: cfg3 6548 / 6540 vs 6489 / 6499 (+0.8%), cfg2 +0.8%, cfg5 +0.1%,
// profiles/r05/r05ay_ab_chunks_lead.log)
constexpr uint32_t kWfChunk = ZRT_WF_CHUNK;

// Triangle positions per ref (bakeInto's Pos: v0, e1 = v1 - v0, e2 = v2 - v0)
// as 3 float4 (48 B, w unused).  36-byte records touch 25% fewer cache lines
// per cell but cost the park kernel 9 VGPRs (r05f: cfg3 -9%).
// ZRT_PLANES16: a scattering hit's bounce-plane record is (albedo, has
// emissive) in one float4 (16 B, one store) plus a float4 emissive record
// only when the material emits, against 24 B in two stores (stk4 + stk2):
// the lamps are the only emissive materials of the stand-in scenes.  r05j,
// alternating processes, 2 rounds, images identical: cfg3 5894 / 5899 vs
// 5819 / 5812 (+1.4%), cfg5 +1.0%, cfg2 +1.1%; one-stream resolve 6.1 -> 4.3
// ms per cfg3 frame (profiles/r05/r05j_ab_planes16.log)
#ifndef ZRT_PLANES16
#define ZRT_PLANES16 1
#endif
// ZRT_ESCAPE: the park walk stops a segment once its escape-table bit
// (escape.h) says every later cell of its ray is empty
#ifndef ZRT_ESCAPE
#define ZRT_ESCAPE 1
#endif
// ZRT_FRUSTUM: the primary walk fast-forwards (DDAV_FF) over the crossings
// below its pixel block's frustum bound (escape.h frustum_bound lo); with
// ZRT_FRUSTUM_HI it also stops once it has tested the cell whose exit is at
// or past the block's far bound (hi)
#ifndef ZRT_FRUSTUM
#define ZRT_FRUSTUM 1
#endif
#ifndef ZRT_FRUSTUM_HI
#define ZRT_FRUSTUM_HI 1
#endif
// the timed kernels' normalize: 1/length by recip_rn (zrt_math.h; the same
// vector bit for bit)
#ifndef ZRT_NORMALIZE_RN
#define ZRT_NORMALIZE_RN 1
#endif
#if ZRT_NORMALIZE_RN
#define ZRT_NORM_RN normalize_rn
#else
#define ZRT_NORM_RN normalize
#endif
// ZRT_FFN: the frustum fast-forward as DDAV_FFN (dda.h: per axis predicated
// adds and a count, the packed coordinate written once) instead of DDAV_FF4
// (a packed step per crossing); cfg3 camera rays cross 85.6 cells below their
// block's bound (tools/frustum_sim.cpp), cfg5 75.5, cfg2 62.8
#ifndef ZRT_FFN
#define ZRT_FFN 1
#endif
// ZRT_PRIMARY_BMASK: the packed lane walk (primary, lane-walk bounces) on
// brick-major words reads, on entering an occupied brick, the brick's 64-bit
// cell mask from global memory and loads a cell's record only when its own
// bit is set.  With the brick bit alone every cell of an occupied brick cost
// a dependent record load and an empty test: cfg3 camera rays walk 44 cells
// after the frustum bound, 18.9 in occupied bricks, 4.2 non-empty (host
// model, tools/frustum_sim.cpp on the bench scenes; cfg5 27.3 / 11.5 / 2.8)
#ifndef ZRT_PRIMARY_BMASK
#define ZRT_PRIMARY_BMASK 1
#endif
// ZRT_WALK_FACE_SKIP: the packed lane walk (primary, lane-walk bounces) skips
// a cell's refs that the cell it left already tested (test_cell_keep), as
// the park kernel's test rounds do.  The r06aa A/B, before the exact cell
// bits and the counted fast-forward, had it at -0.1% (cfg3); on the tree
// after them (r06af, r06ag, 5 rounds) cfg3 +1.2%, cfg5 +0.3%, cfg2 +0.5%,
// with 6 VGPRs of the 7-wave primary spilled outside its walk (6 waves: no
// spill, cfg3 +0.9%)
#ifndef ZRT_WALK_FACE_SKIP
#define ZRT_WALK_FACE_SKIP 1
#endif
// dda_init_fq (dda.h) in the primary / lane-walk wf_kernel too (the park
// kernel's refill always takes it when ZRT_FAST_QUOT)
#ifndef ZRT_FAST_QUOT_WF
#define ZRT_FAST_QUOT_WF 1
#endif
// primary frustum bounds per (1 << ZRT_FRUSTUM_SHIFT)^2 pixel block: 4x4
// since round 6, when the counted fast-forward (ZRT_FFN) made the crossings
// below the bound cheap (r05ae had 8x8 = 4x4 = 2x2 at ~10 VALU per crossing);
// r06ai / r06ak, 5 rounds: cfg3 +0.8 / +0.5%, cfg2 -0.3 / +0.1%, cfg5 0 / +0.1%
#ifndef ZRT_FRUSTUM_SHIFT
#define ZRT_FRUSTUM_SHIFT 2
#endif
constexpr uint32_t kFrustShift = ZRT_FRUSTUM_SHIFT;
static_assert(kFrustShift <= 3, "a frustum block lies inside one tile (tile edges are multiples of 8)");
// brick-major packed cell words for the grids that allow them (dda.h): r05ag,
// 2 rounds, images identical: cfg3 6076 / 6088 vs 6005 / 5999 (+1.3%), cfg2
// +2.4%, cfg5 +1.2%; the park walk trip 179 -> 165 VALU
// (profiles/r05/r05ag_ab_brick_major.log)
#ifndef ZRT_PACK_BM
#define ZRT_PACK_BM 1
#endif

constexpr double kFrustB = (double)(1u << ZRT_FRUSTUM_SHIFT);
// DDA steps per park walk trip, every cell's brick lookup in flight at once
// (r03h/r03i, full spp: 4 vs 2 cfg3 +2.6%, cfg5 +2.2%, cfg2 -0.2%; 6: cfg3
// +0.4%, cfg5 +4.1%; 8: -8 to -10% everywhere)
#ifndef ZRT_WALK_STEPS
#define ZRT_WALK_STEPS 4
#endif
// the park kernel without the escape table (cfg2, cfg5) at 5 steps: r06ba, 2
// rounds, cfg5 +0.55%, cfg2 +0.4%; with the table 5 steps spill in the walk
// (cfg3 -6.7%) and 6 spill everywhere (cfg5 -8%)
#ifndef ZRT_WALK_STEPS_NOESC
#define ZRT_WALK_STEPS_NOESC 5
#endif
constexpr uint32_t kTriFloats = 12u;

struct TraceParams {
    float bmin[3], bmax[3];
    uint32_t res[3];
    float cs[3];
    float ics[3];             // RN(1 / cs) (host division), for dda_init_fq
    uint32_t cs_ok;           // every cs in [2^-32, 2^32]: dda_init_fq may use ics
    const uint2* cells;
    const float* tri_pos;     // kTriFloats per ref (see kTriFloats)
    const float4* tri_data;   // 4 per ref: n0 n1 n2 uv0 uv1 uv2 mat
    const DevMat* mats;
    uint32_t nmat;
    const float* texels;
    const double* zig;        // zx[257], zf[257]
    const uint32_t* occ;      // brick occupancy bits (brick = 2^occ_shift cells per axis)
    uint32_t occ_shift, occ_nb0, occ_nb01, occ_words;
    // per 4^3 brick in linear brick order (= pc >> 6 of a brick-major word)
    // its 64-bit cell mask (occx_mask_kernel's), for the packed lane walk
    const unsigned long long* bmask;
    // primary launch: per 2^kFrustShift-square pixel block of the image (row-major, tlo_nbx
    // blocks per row) the frustum bounds (lo, hi, unused, unused) of escape.h
    // frustum_bound, or null
    const float4* tlo;
    uint32_t tlo_nbx;
    // packed walks (DdaV): the layout, the cells indexed by the packed word
    // (the cells themselves for power-of-two grids, else a padded copy), the
    // coarse-brick fields of the packed word (offset, width per axis) and
    // their in-brick bits; the 4^3-brick fields for OccX
    PackK pk;
    const uint32_t* cell32;   // 8 u32 per packed cell: begin, end, entry-face masks (see cell32_kernel)
    uint32_t occ_o1, occ_o2, occ_w0, occ_w1, occ_w2, occ_lowm;
    uint32_t ox1, ox2, ow0, ow1, ow2;
    float org[3], llc[3], right[3], up[3];
    uint32_t w;
    const uint32_t* pixlist;
    uint32_t P;               // pixels of this rank
    uint32_t s0;              // first sample index of this pass
    uint32_t total;           // items in this pass: S * P, pixel-major (item = q * S + s)
    uint32_t S;               // samples of every pixel in this pass
    DivS sdiv;                // item / S by multiply and shift (div_magic)
    uint32_t max_bounce;
    uint64_t seed;
    float4* out;              // counting build: sample radiance per item
    uint32_t* counter;
    unsigned long long* stats;   // segments, cells, tests, hits, diagnostics
};

// Ref j's v0, e1, e2.
__device__ __forceinline__ void load_tri(const TraceParams& p, uint32_t j, v3& v0, v3& e1, v3& e2) {
    const float* q = p.tri_pos + (uint64_t)kTriFloats * j;
    const float4 a = *reinterpret_cast<const float4*>(q), b = *reinterpret_cast<const float4*>(q + 4),
                 c = *reinterpret_cast<const float4*>(q + 8);
    v0 = mk(a.x, a.y, a.z); e1 = mk(b.x, b.y, b.z); e2 = mk(c.x, c.y, c.z);
}

// Per-bounce (emissive, albedo) pairs of one path (counting megakernel only).
// The fold reads them back to front: e0 + a0*(e1 + a1*(...)) is
// traceRayRecursive's arithmetic (stage3.zig:219); pass-through bounces
// (stage3.zig:212) add no pair.
template <int N>
struct Stack {
    float e[3 * N], a[3 * N];
    uint32_t used;
    __device__ __forceinline__ void init() { used = 0u; }
    __device__ __forceinline__ void set(uint32_t slot, v3 ee, v3 aa) {
        e[3 * slot] = ee.x; e[3 * slot + 1] = ee.y; e[3 * slot + 2] = ee.z;
        a[3 * slot] = aa.x; a[3 * slot + 1] = aa.y; a[3 * slot + 2] = aa.z;
        used |= 1u << slot;
    }
    __device__ __forceinline__ v3 fold(v3 L) const {
        for (int i = N - 1; i >= 0; --i) {
            if ((used >> i) & 1u) {
                L = add(mk(e[3 * i], e[3 * i + 1], e[3 * i + 2]),
                        mul(mk(a[3 * i], a[3 * i + 1], a[3 * i + 2]), L));
            }
        }
        return L;
    }
};

__device__ __forceinline__ bool brick_occupied(const TraceParams& p, const uint32_t* occ, uint32_t c0,
                                               uint32_t c1, uint32_t c2) {
    const uint32_t s = p.occ_shift;
    const uint32_t b = __umul24(c2 >> s, p.occ_nb01) + __umul24(c1 >> s, p.occ_nb0) + (c0 >> s);   // nb <= 2^24 (context check)
    return (occ[b >> 5] >> (b & 31u)) & 1u;
}

// brick_occupied for a packed cell (DdaV): the brick coordinates are bit
// fields of the word (width 0 when a brick spans the whole axis)
// (brick-major words: the occupancy bricks are 4^3, context_packed, so the
// brick is the word's high part)
template <bool BM>
__device__ __forceinline__ bool brick_occupied_v(const TraceParams& p, const uint32_t* occ, uint32_t pc) {
    if (BM) {
        return __builtin_amdgcn_ubfe(occ[pc >> 11], pc >> 6, 1u);
    }
    const uint32_t b = __umul24(__builtin_amdgcn_ubfe(pc, p.occ_o2, p.occ_w2), p.occ_nb01) +
                       __umul24(__builtin_amdgcn_ubfe(pc, p.occ_o1, p.occ_w1), p.occ_nb0) +
                       __builtin_amdgcn_ubfe(pc, p.occ_shift, p.occ_w0);
    return (occ[b >> 5] >> (b & 31u)) & 1u;
}

// The in-brick cell index k = x | y << 2 | z << 4 of a packed cell: one
// 24-bit multiply of the fields' low two bits sums them, shifted into place
// (pack_layout picks the multiplier and checks every in-brick cell), and the
// 64-bit shift reads only k[5:0].  (6 VALU; 9 with the fields moved by shifts
// and masks.)
template <bool BM>
__device__ __forceinline__ bool occx_cell(unsigned long long bm, const DdaV& s, const PackK& k) {
    if (BM) return (uint32_t)(bm >> (s.pc & 63u)) & 1u;   // (brick-major: the word's low six bits)
    const uint32_t i = __umul24(s.pc & k.low2, k.kmul) >> k.kshr;
    return (uint32_t)(bm >> (i & 63u)) & 1u;
}

// Grid constants as wave-uniform registers (see GridK).
__device__ __forceinline__ GridK grid_consts(const TraceParams& p) {
    GridK g;
    g.rm0 = __builtin_amdgcn_readfirstlane(p.res[0] - 1u);
    g.rm1 = __builtin_amdgcn_readfirstlane(p.res[1] - 1u);
    g.rm2 = __builtin_amdgcn_readfirstlane(p.res[2] - 1u);
    g.str1 = __builtin_amdgcn_readfirstlane(p.res[0]);
    g.str2 = __builtin_amdgcn_readfirstlane(p.res[0] * p.res[1]);
    return g;
}

__device__ __forceinline__ bool first_active_lane() {
    return (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__ballot(1));
}

// All triangles of one cell in reference order (stage3.zig:164-178), TB at
// a time: the TB loads are issued before the first test so their latencies
// overlap (one memory round trip per TB triangles instead of per triangle).
template <int TB, bool STATS, bool MTX = false>
__device__ __forceinline__ void test_cell(const TraceParams& p, uint32_t b, uint32_t e, v3 o, v3 d,
                                          float& nearest, float& hu, float& hv, uint32_t& hidx,
                                          uint32_t& n_tests, uint64_t* wstat) {
    for (uint32_t i = b; i < e; i += TB) {
        if (STATS && first_active_lane()) ++wstat[1];   // wave trips of this loop
        v3 A[TB], B[TB], Cc[TB];
#pragma unroll
        for (int k = 0; k < TB; ++k) load_tri(p, min(i + (uint32_t)k, e - 1u), A[k], B[k], Cc[k]);
#pragma unroll
        for (int k = 0; k < TB; ++k) {
            if (i + (uint32_t)k < e) {
                if (STATS) ++n_tests;
                float t, u, v;
                if (tri_ray<MTX>(A[k], B[k], Cc[k], o, d, &t, &u, &v)) {
                    if (nearest > t && t > 0.0f) { nearest = t; hu = u; hv = v; hidx = i + k; }
                }
            }
        }
    }
}

// test_cell for the packed walk's cells, with the entry-face skip of the
// park kernel's test rounds (cell32_kernel): `keep` is the mask of the cell's
// refs (bit k: ref b + k) still to test for the face the ray entered across,
// all ones for a segment's first cell or cells above 32 refs.  A skipped ref
// is bit-identical to one of the cell the ray just left, already tested
// there, so the kept refs give the same nearest hit, in the same order.
template <int TB, bool MTX>
__device__ __forceinline__ void test_cell_keep(const TraceParams& p, uint32_t b, uint32_t e, uint32_t keep, v3 o,
                                               v3 d, float& nearest, float& hu, float& hv, uint32_t& hidx) {
    const uint32_t cnt = e - b;
    if (cnt > 32u || keep == ~0u) {
        uint32_t dummy = 0;
        test_cell<TB, false, MTX>(p, b, e, o, d, nearest, hu, hv, hidx, dummy, nullptr);
        return;
    }
    uint32_t m = keep & ((cnt < 32u ? (1u << cnt) : 0u) - 1u);
    while (m) {
        uint32_t k[TB];
        bool has[TB];
#pragma unroll
        for (int j = 0; j < TB; ++j) {
            has[j] = m != 0u;
            k[j] = has[j] ? (uint32_t)__builtin_ctz(m) : k[0];
            m &= m - 1u;
        }
        v3 A[TB], B[TB], Cc[TB];
#pragma unroll
        for (int j = 0; j < TB; ++j) load_tri(p, b + k[j], A[j], B[j], Cc[j]);
#pragma unroll
        for (int j = 0; j < TB; ++j) {
            if (has[j]) {
                float t, u, v;
                if (tri_ray<MTX>(A[j], B[j], Cc[j], o, d, &t, &u, &v)) {
                    if (nearest > t && t > 0.0f) { nearest = t; hu = u; hv = v; hidx = b + k[j]; }
                }
            }
        }
    }
}

// Scene.traceRay (stage3.zig:152-186) with empty-space skipping that changes
// nothing in the result: the DDA arithmetic runs for every cell exactly as
// Iterator.next does; only the 8-byte Cell load is skipped when the cell's
// brick holds no triangle (its range would be empty).
// STATS (counting build): n_cells / n_tests per lane; prof[] per wave:
// [6] cell loads, [7] non-empty cells, [8] wave trips of the cell loop,
// [9] wave trips of the triangle-batch loop, [10] cell trips with any test,
// [4] 64-wide rounds if each trip's tests were shared evenly.
// PACKED: the walk state with the cell packed into one word (DdaV, grids of
// at most 1024 cells per axis; same cells, same order, same t_exit), which
// also indexes the cell records (cell32).
// TAU (packed walk): a frustum bound (escape.h frustum_bound lo) for this ray: the
// crossings below it enter only empty cells; +inf: the ray meets no
// occupied cell at all.
template <bool STATS, int TB, bool PACKED = false, bool PK_BM = false, bool MTX = false>
__device__ __forceinline__ float trace_ray(const TraceParams& p, const uint32_t* occ, v3 o, v3 d,
                                           float& hu, float& hv, uint32_t& hidx, uint32_t& n_cells,
                                           uint32_t& n_tests, uint64_t* prof, uint32_t* wcnt = nullptr,
                                           float tau = 0.0f, float tfar = kInf) {
    float nearest = kInf;
    Dda s0;
    // (the counting build and the IEEE-division kernels keep dda_init's
    // divisions; the timed kernels take dda_init_fq's quotients: same state)
    if (ZRT_FAST_QUOT && ZRT_FAST_QUOT_WF && !MTX && !STATS) {
        if (!dda_init_fq(p.bmin, p.bmax, p.res, p.cs, p.ics, p.cs_ok != 0u, o, d, s0)) return nearest;
    } else if (!dda_init(p.bmin, p.bmax, p.res, p.cs, o, d, s0)) {
        return nearest;
    }
    const uint32_t sh = p.occ_shift;
    const GridK gk = grid_consts(p);
    if constexpr (PACKED) {
        static_assert(!STATS, "the counting build walks unpacked");
        DdaV s;
        ddav_from_t<PK_BM>(s0, gk, p.pk, s);
        // the field masks as laundered registers: selected straight from the
        // kernel arguments they became a vector load at a selected offset
        // (v_cndmask of 0x94/0x98/0x9c, global_load_dword, vmcnt(0)) in
        // every step (r03 ISA)
        uint32_t f0 = p.pk.f0, f1 = p.pk.f1, f2 = p.pk.f2;
        asm("" : "+s"(f0), "+s"(f1), "+s"(f2));
        if (ZRT_FRUSTUM && s0.neg < 8u) {
            // the cells before tau are empty (the pixel block's frustum bound):
            // their crossings as plain adds, the walk's exact state after them
            // (DDAV_FF); nearest is +inf here, so no break test fires among them
            if (tau == kInf) return nearest;               // no occupied cell on the ray: the miss
            if (tau > fminf(s.tn0, fminf(s.tn1, s.tn2))) {
                bool exited;
                // (four branch-free crossings per loop trip: r04s, cfg3 5730 vs
                // 5695 Mrays/s with one per trip, DDAV_FF)
                if (ZRT_FFN) DDAV_FFN(s, p.pk, f0, f1, f2, tau, exited);
                else DDAV_FF4(s, f0, f1, f2, tau, exited);
                if (exited) return nearest;
            }
        }
        bool occupied = brick_occupied_v<PK_BM>(p, occ, s.pc);
        constexpr bool kBm = PK_BM && ZRT_PRIMARY_BMASK;
        unsigned long long q = 0ull;        // kBm: the current brick's cell mask
        if (kBm && occupied) q = p.bmask[s.pc >> 6];
        // the walk's stop: the nearest hit so far, or (TFAR, a frustum far
        // bound) the t past which every cell of the ray is empty
        float lim = ZRT_FRUSTUM_HI && s0.neg < 8u ? tfar : kInf;
        // ZRT_WALK_FACE_SKIP: the crossing t of the step into the current
        // cell (NaN: the segment's first tested cell, every ref tested)
        float tcl = __builtin_nanf("");
        for (;;) {
            if (kBm ? ((q >> (s.pc & 63u)) & 1ull) != 0ull : occupied) {
                const uint32_t* rec = p.cell32 + 8ull * s.pc;
                const uint2 cell = *reinterpret_cast<const uint2*>(rec);
                if (ZRT_WALK_FACE_SKIP) {
                    // the face entered: the stepped axis a is the one whose
                    // next crossing is this step's own tc + td_a; exactly one
                    // such axis, or (a tie at tc) every ref is tested
                    const bool x0 = s.tn0 == tcl + s.td0, x1 = s.tn1 == tcl + s.td1, x2 = s.tn2 == tcl + s.td2;
                    uint32_t keep = ~0u;
                    if ((uint32_t)x0 + (uint32_t)x1 + (uint32_t)x2 == 1u) {
                        const uint32_t face = x0 ? (s.d0 >> 31) : (x1 ? 2u + (s.d1 >> 31) : 4u + (s.d2 >> 31));
                        keep = rec[2 + face];
                    }
                    test_cell_keep<TB, MTX>(p, cell.x, cell.y, keep, o, d, nearest, hu, hv, hidx);
                } else {
                    test_cell<TB, false, MTX>(p, cell.x, cell.y, o, d, nearest, hu, hv, hidx, n_tests, prof);
                }
                lim = fminf(lim, nearest);                 // = min(nearest, far bound)
            }
            bool crossed, exited;
            float tc;
            PackK pkl = p.pk;
            pkl.f0 = f0; pkl.f1 = f1; pkl.f2 = f2;
            DDAV_STEPX(s, pkl, p.occ_lowm, crossed, exited, tc);
            if (exited || lim <= tc) break;                // stage3.zig:179-182 (T_EXIT = +inf at the exit)
            tcl = tc;
            if (crossed) {
                occupied = brick_occupied_v<PK_BM>(p, occ, s.pc);
                if (kBm) q = occupied ? p.bmask[s.pc >> 6] : 0ull;
            }
        }
        return nearest;
    }
    DdaW s;
    ddaw_from(s0, gk, s);
    bool occupied = brick_occupied(p, occ, s.c0, s.c1, s.c2);
    for (;;) {
        if (STATS) ++n_cells;
        if (STATS && first_active_lane()) ++prof[8];
        uint32_t ncell = 0;
        if (occupied) {
            const uint2 cell = p.cells[s.lin];
            if (STATS) { prof[6] += 1; prof[7] += cell.y > cell.x ? 1 : 0; ncell = cell.y - cell.x; }
            test_cell<TB, STATS, MTX>(p, cell.x, cell.y, o, d, nearest, hu, hv, hidx, n_tests, prof + 8);
        }
        if (STATS) {
            // wave-shared work of this trip: sum of the lanes' triangle counts
            uint32_t* wc = wcnt + 2 * (threadIdx.x >> 6);
            const bool first = first_active_lane();
            if (first) wc[0] = 0;
            __builtin_amdgcn_wave_barrier();
            atomicAdd(&wc[0], ncell);
            __builtin_amdgcn_wave_barrier();
            if (first) {
                const uint32_t N = wc[0];
                prof[10] += N ? 1 : 0;
                prof[4] += (N + 63) / 64;
            }
        }
        bool crossed;
        float t_exit;
        DDAW_STEP(s, sh, crossed, t_exit);
        if (nearest <= t_exit) break;                      // stage3.zig:179-182
        if (crossed) occupied = brick_occupied(p, occ, s.c0, s.c1, s.c2);
    }
    return nearest;
}

// Texture(T).sample (stage3.zig:111-123).  A 1x1 texture -- the dummy of
// every material slot without an image (stage1.zig:411-425) -- has all four
// texel indices 0 (any clamp, @mod by 1), so it loads its texel once and
// runs the same bilinear arithmetic on it (bit-identical: x - x is not
// folded, NaN/inf weights propagate as before), instead of the index
// arithmetic and four loads per channel.
#ifndef ZRT_TEX1
#define ZRT_TEX1 1
#endif
__device__ __forceinline__ v3 sample3(const float* texels, const DevTex& t, float u, float v) {
    const float* b = texels + t.off;
    if (ZRT_TEX1 && t.w == 1 && t.h == 1) {
        const float fu = tex_frac(u), fv = tex_frac(v);
        // the texel, inlined in the descriptor (dev_tex_inline)
        const float x = __int_as_float(t.umin), y = __int_as_float(t.umax), z = __int_as_float(t.vmin);
        return mk(bilerp(x, x, x, x, fu, fv), bilerp(y, y, y, y, fu, fv), bilerp(z, z, z, z, fu, fv));
    }
    const TexCoords c = tex_coords(t.w, t.h, t.umin, t.umax, t.vmin, t.vmax, u, v);
    v3 r;
    r.x = bilerp(b[3 * c.i11 + 0], b[3 * c.i21 + 0], b[3 * c.i12 + 0], b[3 * c.i22 + 0], c.fu, c.fv);
    r.y = bilerp(b[3 * c.i11 + 1], b[3 * c.i21 + 1], b[3 * c.i12 + 1], b[3 * c.i22 + 1], c.fu, c.fv);
    r.z = bilerp(b[3 * c.i11 + 2], b[3 * c.i21 + 2], b[3 * c.i12 + 2], b[3 * c.i22 + 2], c.fu, c.fv);
    return r;
}
__device__ __forceinline__ float sample1(const float* texels, const DevTex& t, float u, float v) {
    const float* b = texels + t.off;
    if (ZRT_TEX1 && t.w == 1 && t.h == 1) {               // the 1x1 dummy (see sample3)
        const float x = __int_as_float(t.umin);
        return bilerp(x, x, x, x, tex_frac(u), tex_frac(v));
    }
    const TexCoords c = tex_coords(t.w, t.h, t.umin, t.umax, t.vmin, t.vmax, u, v);
    return bilerp(b[c.i11], b[c.i21], b[c.i12], b[c.i22], c.fu, c.fv);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned lo = __shfl_xor((unsigned)x, off);
        const unsigned hi = __shfl_xor((unsigned)(x >> 32), off);
        x += ((unsigned long long)hi << 32) | lo;
    }
    return x;
}

// renderWorker: camera.getRay(x + U, y + U) (stage3.zig:238, :27-35) for
// pass item `item` (= packed pixel * S + s_local: pixel-major, so one
// pixel's samples are consecutive items and a wave's records are
// contiguous); leaves rng after the jitter.
__device__ __forceinline__ void camera_ray(const TraceParams& p, uint32_t item, Rng& rng, v3& o, v3& d,
                                           uint32_t* block = nullptr) {
    const uint32_t q = div_by(item, p.sdiv);
    const uint32_t s_local = item - q * p.S;
    const uint32_t pixel = p.pixlist[q];
    const uint32_t py = pixel / p.w;
    const uint32_t px = pixel - py * p.w;
    if (block) *block = (py >> kFrustShift) * p.tlo_nbx + (px >> kFrustShift);
    rng.s = path_key(p.seed, pixel, p.s0 + s_local);
    const float jx = rng_float(rng);
    const float jy = rng_float(rng);
    o = mk(p.org[0], p.org[1], p.org[2]);
    d = ZRT_NORM_RN(add(add(mk(p.llc[0], p.llc[1], p.llc[2]),
                          scale(mk(p.right[0], p.right[1], p.right[2]), (float)px + jx)),
                      scale(mk(p.up[0], p.up[1], p.up[2]), (float)py + jy)));
}

// The RNG state camera_ray leaves (after the jitter draws), without the ray.
__device__ __forceinline__ Rng camera_rng(const TraceParams& p, uint32_t item) {
    const uint32_t q = div_by(item, p.sdiv);
    const uint32_t s_local = item - q * p.S;
    const uint32_t pixel = p.pixlist[q];
    Rng rng;
    rng.s = path_key(p.seed, pixel, p.s0 + s_local);
    (void)rng_float(rng);
    (void)rng_float(rng);
    return rng;
}

// The counting megakernel: renderWorker's per-sample body (stage3.zig:237-241)
// + traceRayRecursive (stage3.zig:188-220) made iterative, one lane = one
// path from camera to sky, with exact per-lane work counters (segments,
// cells, triangle tests, hits).  Same RNG -> same paths as the timed
// wavefront kernels, so its counts are the timed frame's algorithmic work
// (bench.py's roofline) and the parity tests' traversal counters.
template <int MAXB>
__global__ __launch_bounds__(kTraceBlock, 1) void trace_kernel(const TraceParams p) {
    __shared__ double s_zig[514];
    extern __shared__ __attribute__((aligned(16))) uint32_t s_occ[];
    uint64_t prof[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    __shared__ uint32_t s_wcnt[2 * (kTraceBlock / 64)];
    for (uint32_t i = threadIdx.x; i < 514; i += blockDim.x) s_zig[i] = p.zig[i];
    for (uint32_t i = threadIdx.x; i < p.occ_words; i += blockDim.x) s_occ[i] = p.occ[i];
    __syncthreads();
    const double* zx = s_zig;
    const double* zf = s_zig + 257;

    const uint32_t lane = threadIdx.x & 63u;
    uint32_t n_seg = 0, n_cells = 0, n_tests = 0, n_hits = 0;
    uint32_t p_seg = 0, p_cells = 0, p_tests = 0, p_hits = 0;   // the primary (camera) segments' share

    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(p.counter, 64u);
        base = __builtin_amdgcn_readfirstlane(base);
        if (base >= p.total) break;
        const uint32_t item = base + lane;
        if (item >= p.total) continue;

        Rng rng;
        v3 o, d;
        camera_ray(p, item, rng, o, d);
        Stack<MAXB> stk;
        stk.init();
        v3 L = mk(0, 0, 0);
        uint32_t slot = 0;
        for (uint32_t depth = p.max_bounce; depth > 0; --depth, ++slot) {
            ++n_seg;
            float hu = 0.0f, hv = 0.0f;
            uint32_t hidx = 0;
            const uint32_t c_before = n_cells, t_before = n_tests;
            // (the plain IEEE division in Moller-Trumbore: the counting build is
            // the timed kernels' checker and serves every scene, mt_inv_det)
            const float t = trace_ray<true, kTriBatch, false, false, true>(p, s_occ, o, d, hu, hv, hidx, n_cells,
                                                                           n_tests, prof, s_wcnt);
            if (slot == 0) { ++p_seg; p_cells += n_cells - c_before; p_tests += n_tests - t_before; }
            if (t == kInf) { L = env_color(d); break; }       // stage3.zig:195-197
            ++n_hits;
            if (slot == 0) ++p_hits;
            // stage3.zig:199-206
            const float4* tdp = p.tri_data + 4ull * hidx;
            const float4 d0 = tdp[0], d1 = tdp[1], d2 = tdp[2], d3 = tdp[3];
            const float w0 = 1.0f - hu - hv;
            const float tc0 = (d2.y * w0 + d2.w * hu) + d3.y * hv;
            const float tc1 = (d2.z * w0 + d3.x * hu) + d3.z * hv;
            const DevMat& m = p.mats[__float_as_uint(d3.w)];
            const v3 albedo = sample3(p.texels, m.tex[0], tc0, tc1);
            const v3 emissive = sample3(p.texels, m.tex[1], tc0, tc1);
            const float transparency = sample1(p.texels, m.tex[2], tc0, tc1);
            const v3 nrm = add(add(scale(mk(d0.x, d0.y, d0.z), w0), scale(mk(d0.w, d1.x, d1.y), hu)),
                               scale(mk(d1.z, d1.w, d2.x), hv));
            const v3 no = add(o, scale(d, t + kFltEps));        // ray.at(hit.t + eps)
            if (!(rng_float(rng) > transparency)) {             // stage3.zig:207
                // randomUnitVector (linalg.zig:140-148): 3 x floatNorm, normalize
                const float nx = (float)rng_norm64(rng, zx, zf);
                const float ny = (float)rng_norm64(rng, zx, zf);
                const float nz = (float)rng_norm64(rng, zx, zf);
                d = normalize(add(nrm, normalize(mk(nx, ny, nz))));
                stk.set(slot, emissive, albedo);                // stage3.zig:214-219
            }                                                   // else pass-through :208-212
            o = no;
        }
        L = stk.fold(L);
        p.out[item] = make_float4(L.x, L.y, L.z, 0.0f);
    }
    const unsigned long long s0 = wave_sum(n_seg), s1 = wave_sum(n_cells), s2 = wave_sum(n_tests),
                             s3 = wave_sum(n_hits), s4 = wave_sum(prof[6]), s5 = wave_sum(prof[7]),
                             s6 = wave_sum(prof[8]), s7 = wave_sum(prof[9]), s8 = wave_sum(prof[10]),
                             s9 = wave_sum(prof[4]);
    const unsigned long long q0 = wave_sum(p_seg), q1 = wave_sum(p_cells), q2 = wave_sum(p_tests),
                             q3 = wave_sum(p_hits);
    if (lane == 0) {
        atomicAdd(&p.stats[8], q0);
        atomicAdd(&p.stats[9], q1);
        atomicAdd(&p.stats[10], q2);
        atomicAdd(&p.stats[11], q3);
        atomicAdd(&p.stats[0], s0);
        atomicAdd(&p.stats[1], s1);
        atomicAdd(&p.stats[2], s2);
        atomicAdd(&p.stats[3], s3);
        atomicAdd(&p.stats[4], s4);
        atomicAdd(&p.stats[5], s5);
        atomicAdd(&p.stats[6], s6);
        atomicAdd(&p.stats[7], s7);
        atomicAdd(&p.stats[14], s8);
        atomicAdd(&p.stats[15], s9);
    }
}

// ---------------------------------------------------------------------------
// Wavefront organisation: one launch per bounce over a compacted queue of
// live paths.
//
// A megakernel keeps a lane on one path from camera to sky, so a wave lives
// as long as its longest path.  Here bounce k is its own launch over the
// paths still alive after bounce k-1: every lane traces one segment and
// shades it; a continuing path is appended to the next queue (one returning
// atomic per wave and region, ballot + popcount ranks), a finished one
// stores its terminal radiance (env / 0) and the mask of bounce slots that
// scattered.  The per-bounce (emissive, albedo) pairs go to HBM in
// [slot][item] planes and wf_resolve_kernel folds them back to front.
// Items are pixel-major (item = packed pixel * S + sample of the pass).
//
// A queue record is 48 B: (o.xyz, item) (d.xyz, depth | slot << 16)
// (rng lo, rng hi, mask, 0).
//
// XCD split: blocks are dispatched round-robin over the 8 XCDs, so block
// group g = blockIdx % 8 shares one L2.  The packed pixel list is cut into 8
// ranges (8x8-block aligned) and every queue into 8 regions, region g holding
// the paths of pixel range g (capacity S * P_g).  Group g takes pixel range
// g / region g first, then helps the other groups: a screen region's paths
// stay on one XCD from bounce to bounce.  Same items, other order: same image.
struct WfParams {
    TraceParams t;
    const float4* q_in;
    float4* q_out;
    float4* stk4;             // bounce planes, slot-major: float4 (e, a.x) at [slot * T + item]
    float2* stk2;             //   and float2 (a.y, a.z) at [slot * T + item] (24 B per pair)
                              // ZRT_PLANES16: stk4 = (a, emissive bits != 0), stk2 = float4 e
                              // at [slot * T + item], written for emissive hits only
    float4* term;             // [item]: terminal L.xyz, scatter mask bits
    uint32_t T;               // items in this pass
    uint32_t* fetch8;         // work counter per group of this launch
    const uint32_t* n_in8;    // paths per region of q_in
    uint32_t* n_out8;         // paths per region of q_out
    float4* hit;              // split launches: [entry] (t, u, v, ref) of the segment just traced
    uint32_t* fetch8s;        // split launches: work counter per group of the shade kernel
    // wf_park_kernel: exact per-cell occupancy blob (see OccX) and schedule
    const uint32_t* occx;
    uint32_t occx_words, occx_nbw, occx_moff, occx_nb0, occx_nb01;
    uint32_t occx_ldsw;       // u32 words OccX takes in LDS (multiple of 4): entries + masks
    uint32_t test_min;        // parked lanes before a wave runs a test round
    uint32_t refill_min;      // finished lanes before a wave shades and refills
    uint32_t rel_min;         // park release: a round with fewer parked lanes with refs is skipped (0: off)
    uint32_t rel_emin;        //   ... if at least this many parked lanes have none
    // escape table (escape.h): kEscWords u32 per 4^3 brick, bit b of word
    // w = direction bin 32 w + b; null: not built (the walk never stops early)
    const uint32_t* esc;
};

// Work / append counters: one per 128-byte line (32 u32), so the waves'
// atomics on different counters do not queue on one line (packed counters
// made the region queues 2.4x slower, round 1).
constexpr uint32_t kCtr = 32;

// XCD split: first pixel (packed order) of group g, 8x8-block aligned.
__device__ __forceinline__ uint32_t xcd_q0(uint32_t P, uint32_t g) {
    const uint32_t nblk = (P + 63u) >> 6;
    return min(P, (nblk * g / 8u) * 64u);
}

// First queue entry of region g: S * (the first pixel of pixel range g).
__device__ __forceinline__ uint32_t region_base(const WfParams& w, uint32_t g) { return w.t.S * xcd_q0(w.t.P, g); }

// traceRayRecursive's body after the hit (stage3.zig:195-219) for one
// segment: env colour on a miss, else material lookup, (e, a) pair to the
// bounce planes on a scatter, pass-through otherwise.  Returns true when the
// path continues (o, d, depth, slot, rng, mask updated); false with L set
// when it terminates.
// `mats`: the material descriptors (p.mats, or the shade kernel's LDS copy).
// `sp` (ZRT_SWEEP builds, the shade kernel only): per-wave s_memtime cycles
// and active lanes of the phases (SHADE_STAMP), else null.
#ifdef ZRT_SWEEP
// phase k: cycles into sp[k], active lanes into sp[8 + k]; sp[16] the last
// tick.  `sp` is the wave's row in LDS, updated by the first active lane, so
// a stamp inside a divergent branch (the hit path) counts for the wave
// whichever lanes run it.  `v`: a value the phase produced, so the stamp
// waits for it.
#define SHADE_STAMP(k, v) do { if (sp) { asm volatile("" :: "v"(v)); const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    const uint32_t n_ = (uint32_t)__popcll(__ballot(1)); \
    if (first_active_lane()) { sp[k] += t_ - sp[16]; sp[16] = t_; sp[8 + (k)] += n_; } } } while (0)
#else
#define SHADE_STAMP(k, v) do { (void)sp; } while (0)
#endif
// The hit triangle's Data record (stage3.zig:199-206: normals, uvs, material),
// loaded by the caller so that a lane shading several entries can issue every
// entry's load before the first entry's texel loads (r05c: -4% shade time
// alone, but the kernel no longer fits beside the park kernel).
struct TriRec {
    float4 d0, d1, d2, d3;
};
__device__ __forceinline__ TriRec tri_rec(const TraceParams& p, float t, uint32_t hidx) {
    TriRec r;
    if (t == kInf) {
        r.d0 = r.d1 = r.d2 = r.d3 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        return r;
    }
    const float4* tdp = p.tri_data + 4ull * hidx;
    r.d0 = tdp[0]; r.d1 = tdp[1]; r.d2 = tdp[2]; r.d3 = tdp[3];
    return r;
}
// LAST: the segment is the path's last (depth 1, the last bounce launch):
// traceRayRecursive at depth 1 returns e + a * (the depth-0 call's 0) on a
// scatter and 0 on a pass-through (stage3.zig:188-219), so the terminal
// radiance is e + a * 0 itself -- the resolve's fold step add(e, mul(a, L))
// at L = 0, the same f32 operations, with e = +0 exactly when the material
// emits nothing -- and no bounce plane, scatter bit, normal draws (the
// ziggurat) or queue append is needed.
template <bool LAST = false>
__device__ __forceinline__ bool shade_segment(const WfParams& w, const double* zx, const double* zf,
                                              const DevMat* mats, uint32_t item, float t, float hu, float hv,
                                              const TriRec& tr, v3& o, v3& d, uint32_t& depth, uint32_t& slot,
                                              Rng& rng, uint32_t& mask, v3& L,
                                              unsigned long long* sp = nullptr) {
    SHADE_STAMP(1, t);                                      // the hit record landed
    if (t == kInf) { L = env_color(d); return false; }     // stage3.zig:195-197
    const TraceParams& p = w.t;
    const float4 d0 = tr.d0, d1 = tr.d1, d2 = tr.d2, d3 = tr.d3;   // stage3.zig:199-206
    const float w0 = 1.0f - hu - hv;
    const float tc0 = (d2.y * w0 + d2.w * hu) + d3.y * hv;
    const float tc1 = (d2.z * w0 + d3.x * hu) + d3.z * hv;
    SHADE_STAMP(2, tc1);                                    // triangle data
    const DevMat& m = mats[__float_as_uint(d3.w)];
    const v3 albedo = sample3(p.texels, m.tex[0], tc0, tc1);
    const v3 emissive = sample3(p.texels, m.tex[1], tc0, tc1);
    const float transparency = sample1(p.texels, m.tex[2], tc0, tc1);
    SHADE_STAMP(3, transparency);                           // material + texels
    const v3 nrm = add(add(scale(mk(d0.x, d0.y, d0.z), w0), scale(mk(d0.w, d1.x, d1.y), hu)),
                       scale(mk(d1.z, d1.w, d2.x), hv));
    const v3 no = add(o, scale(d, t + kFltEps));
    const float u_tr = rng_float(rng);
    SHADE_STAMP(4, u_tr);                                   // transparency draw
    if (LAST) {
        // the fold's last step at L = 0 (ZRT_PLANES16: e = +0 exactly when no
        // e was stored, i.e. when every bit of the sampled e is zero: then
        // the sample is that +0)
        L = !(u_tr > transparency) ? add(emissive, mul(albedo, mk(0.0f, 0.0f, 0.0f))) : mk(0, 0, 0);
        return false;
    }
    if (!(u_tr > transparency)) {                           // stage3.zig:207, :214-219
        // the (e, a) pair goes out before the normal draws, so the ziggurat
        // (f64, 64-bit RNG) runs without the six colour registers live; 24 B
        // per pair instead of two float4 (r03zk: cfg3 +0.5%, cfg2 +1.6%,
        // cfg5 +1.3%: this write and wf_resolve_kernel's read are HBM-bound)
        if (ZRT_PLANES16) {
            // (a, has_e) in 16 B; e only for emissive hits (its own plane)
            const uint32_t eb = __float_as_uint(emissive.x) | __float_as_uint(emissive.y) | __float_as_uint(emissive.z);
            w.stk4[(uint64_t)slot * w.T + item] = make_float4(albedo.x, albedo.y, albedo.z, __uint_as_float(eb));
            if (eb != 0u)
                reinterpret_cast<float4*>(w.stk2)[(uint64_t)slot * w.T + item] =
                    make_float4(emissive.x, emissive.y, emissive.z, 0.0f);
        } else {
            w.stk4[(uint64_t)slot * w.T + item] = make_float4(emissive.x, emissive.y, emissive.z, albedo.x);
            w.stk2[(uint64_t)slot * w.T + item] = make_float2(albedo.y, albedo.z);
        }
        const float nx = (float)rng_norm64(rng, zx, zf);
        const float ny = (float)rng_norm64(rng, zx, zf);
        const float nz = (float)rng_norm64(rng, zx, zf);
        d = ZRT_NORM_RN(add(nrm, ZRT_NORM_RN(mk(nx, ny, nz))));
        mask |= 1u << slot;
        SHADE_STAMP(5, d.x);                                // pair store + ziggurat draws
    }
    o = no;
    --depth;
    ++slot;
    L = mk(0, 0, 0);
    return depth != 0;                                      // depth 0: recursion returns 0
}

__device__ __forceinline__ void q_store(const WfParams& w, uint32_t pos, v3 o, v3 d, uint32_t item, uint32_t depth,
                                        uint32_t slot, const Rng& rng, uint32_t mask) {
    w.q_out[3ull * pos] = make_float4(o.x, o.y, o.z, __uint_as_float(item));
    w.q_out[3ull * pos + 1] = make_float4(d.x, d.y, d.z, __uint_as_float(depth | (slot << 16)));
    w.q_out[3ull * pos + 2] = make_float4(__uint_as_float((uint32_t)rng.s), __uint_as_float((uint32_t)(rng.s >> 32)),
                                          __uint_as_float(mask), 0.0f);
}

// Append the continuing paths of the wave (lanes with `cont`) to the next
// queue, each to the region `reg` of its pixel range: one returning atomic
// per distinct region of the wave, ranks from ballot + popcount.
__device__ __forceinline__ void wf_append(const WfParams& w, bool cont, uint64_t below, v3 o, v3 d, uint32_t item,
                                          uint32_t depth, uint32_t slot, const Rng& rng, uint32_t mask,
                                          uint32_t reg) {
    uint64_t pend = __ballot(cont);
    while (pend) {
        const uint32_t lead = (uint32_t)__builtin_ctzll(pend);
        const uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)reg, (int)lead);
        const uint64_t m = __ballot(cont && reg == g);
        uint32_t ob = 0;
        if ((threadIdx.x & 63u) == lead) ob = atomicAdd(&w.n_out8[g * kCtr], (uint32_t)__popcll(m));
        ob = (uint32_t)__builtin_amdgcn_readlane((int)ob, (int)lead) + region_base(w, g);
        if (cont && reg == g) q_store(w, ob + (uint32_t)__popcll(m & below), o, d, item, depth, slot, rng, mask);
        pend &= ~m;
    }
}

// Fetch work for a wave from the XCD group queues, group `grp` first: one
// returning atomic takes `want` consecutive entries of group grp's range
// (primary launch: items of pixel range g for every sample of the pass;
// bounce launches: region g of q_in).  Returns false once every group is
// exhausted.  On true, entries [base, min(base + want, lim)) of group grp
// belong to this wave; entry j maps to the item / queue index of ent_index().
template <bool PRIMARY>
__device__ __forceinline__ bool wf_fetch(const WfParams& w, uint32_t want, uint32_t& grp, uint32_t& tried,
                                         uint32_t& base, uint32_t& lim) {
    const TraceParams& p = w.t;
    const uint32_t S = p.S;
    for (;;) {
        const uint32_t q0 = xcd_q0(p.P, grp);
        const uint32_t pg = xcd_q0(p.P, grp + 1u) - q0;
        lim = PRIMARY ? S * pg : w.n_in8[grp * kCtr];
        uint32_t b = 0;
        if ((threadIdx.x & 63u) == 0) b = atomicAdd(&w.fetch8[grp * kCtr], want);
        base = __builtin_amdgcn_readfirstlane(b);
        if (base < lim) return true;
        if (++tried == 8u) return false;
        grp = (grp + 1u) & 7u;
    }
}
// Primary launch: entry j of group g is sample j % S of pixel q0 + j / S
// (pixel-major), so a wave traces 64 samples of one pixel (or all S samples
// of 64 / S neighbouring pixels in the packed 8x8-block order): rays that
// stay within one pixel's footprint walk the same cells and test the same
// triangles side by side.  Against 64 pixels of one sample (8x8 blocks,
// sample-major) the primary launch took 17.0 vs 22.4-23.2 ms at cfg3 64 spp
// (r02at: cfg3 +6.3%, cfg5 +3.6%, cfg2 +0.5%).  Since r04 the item number
// (what term / the bounce planes / the resolve index) is pixel-major too,
// item = S * pixel + sample = S * q0 + j: a wave's terminal and bounce-pair
// stores are contiguous (sample-major, its 64 lanes stored 64 lines P items
// apart: 126 B of DRAM writes per primary item for <= 72 B of records, r03zm).
// Bounce launches: entry j of region g is queue index S * q0 + j.
template <bool PRIMARY>
__device__ __forceinline__ uint32_t ent_index(const WfParams& w, uint32_t grp, uint32_t j) {
    return region_base(w, grp) + j;
}

// The path state of queue entry / primary item `i` that shading needs.
template <bool PRIMARY>
__device__ __forceinline__ void path_state(const WfParams& w, uint32_t i, uint32_t& item, uint32_t& depth,
                                           uint32_t& slot, Rng& rng, uint32_t& mask) {
    if (PRIMARY) {
        item = i;
        depth = w.t.max_bounce;
        slot = 0;
        mask = 0;
        rng = camera_rng(w.t, i);
    } else {
        const float4 a = w.q_in[3ull * i], b = w.q_in[3ull * i + 1], c = w.q_in[3ull * i + 2];
        item = __float_as_uint(a.w);
        depth = __float_as_uint(b.w) & 0xFFFFu;
        slot = __float_as_uint(b.w) >> 16;
        rng.s = ((uint64_t)__float_as_uint(c.y) << 32) | __float_as_uint(c.x);
        mask = __float_as_uint(c.z);
    }
}

// wf_kernel: one lane = one segment, walked and tested by the lane itself.
// MTX: Moller-Trumbore with the plain IEEE division (mt_inv_det), for the
// scenes whose edges leave the short reciprocal's domain (zrt_context::mt_exact).
template <int MINW, bool PRIMARY, bool PACKED, bool PK_BM = false, bool MTX = false>
__global__ __launch_bounds__(kTraceBlock, MINW) void wf_kernel(const WfParams w) {
    const TraceParams& p = w.t;
    __shared__ double s_zig[514];
    extern __shared__ __attribute__((aligned(16))) uint32_t s_occ[];
    for (uint32_t i = threadIdx.x; i < 514; i += blockDim.x) s_zig[i] = p.zig[i];
    for (uint32_t i = threadIdx.x; i < p.occ_words; i += blockDim.x) s_occ[i] = p.occ[i];
    __syncthreads();
    const double* zx = s_zig;
    const double* zf = s_zig + 257;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
    uint32_t n_seg = 0, dummy = 0;
    uint32_t grp = blockIdx.x & 7u, tried = 0;
#ifdef ZRT_SWEEP
    // ZRT_SWEEP builds: per-wave s_memtime cycles of the walk (camera ray +
    // traceRay), the shading (+ terminal store) and the fetch + append
    unsigned long long wprof[3] = {0, 0, 0};
    uint64_t wtick = __builtin_amdgcn_s_memtime();
#define WF_STAMP(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); wprof[k] += t_ - wtick; wtick = t_; } while (0)
#else
#define WF_STAMP(k) do { } while (0)
#endif

    for (;;) {
        uint32_t base = 0, lim = 0;
        if (!wf_fetch<PRIMARY>(w, 64u * kWfChunk, grp, tried, base, lim)) break;
      for (uint32_t sub = 0; sub < kWfChunk && base + 64u * sub < lim; ++sub) {
        const uint32_t j = base + 64u * sub + lane;
        const bool valid = j < lim;
        const uint32_t i = valid ? ent_index<PRIMARY>(w, grp, j) : 0u;
        bool cont = false;
        uint32_t mask = 0, r_item = 0, r_depth = 0, r_slot = 0;
        v3 r_o = mk(0, 0, 0), r_d = mk(0, 0, 0);
        Rng r_rng;
        r_rng.s = 0;
        if (valid) {
            // the ray only: the rest of the path's state (item, slot, RNG,
            // mask) is re-read after the walk, so it holds no VGPRs in it
            v3 o, d;
            uint32_t depth;
            float tau = 0.0f, tfar = kInf;
            if (PRIMARY) {
                Rng rng0;
                uint32_t blk = 0;
                camera_ray(p, i, rng0, o, d, &blk);
                if (ZRT_FRUSTUM && p.tlo) {
                    const float4 fb = p.tlo[blk];
                    tau = fb.x;
                    tfar = fb.y;
                }
                depth = p.max_bounce;
            } else {
                const float4 a = w.q_in[3ull * i], b = w.q_in[3ull * i + 1];
                o = mk(a.x, a.y, a.z);
                d = mk(b.x, b.y, b.z);
                depth = __float_as_uint(b.w) & 0xFFFFu;
            }
            float t = kInf, hu = 0.0f, hv = 0.0f;
            uint32_t hidx = 0;
            WF_STAMP(2);
            if (depth != 0)
                t = trace_ray<false, kTriBatch, PACKED, PK_BM, MTX>(p, s_occ, o, d, hu, hv, hidx, dummy, dummy, nullptr,
                                                                    nullptr, tau, tfar);
            WF_STAMP(0);
            uint32_t item, slot;
            Rng rng;
            path_state<PRIMARY>(w, i, item, depth, slot, rng, mask);
            v3 L = mk(0, 0, 0);
            if (depth != 0) {
                ++n_seg;
                cont = shade_segment(w, zx, zf, p.mats, item, t, hu, hv, tri_rec(p, t, hidx), o, d, depth, slot, rng,
                                     mask, L);
            }
            if (!cont) w.term[item] = make_float4(L.x, L.y, L.z, __uint_as_float(mask));
            r_item = item; r_depth = depth; r_slot = slot; r_o = o; r_d = d; r_rng = rng;
            WF_STAMP(1);
        }
        wf_append(w, cont, below, r_o, r_d, r_item, r_depth, r_slot, r_rng, mask, grp);
        WF_STAMP(2);
      }
    }
    const unsigned long long s0 = wave_sum(n_seg);
    if (lane == 0) atomicAdd(&p.stats[0], s0);
#ifdef ZRT_SWEEP
    if (PRIMARY && lane == 0)
        for (int k = 0; k < 3; ++k) atomicAdd(&p.stats[29 + k], wprof[k]);
#endif
#undef WF_STAMP
}

// ---------------------------------------------------------------------------
// wf_park_kernel: Scene.traceRay as walk / park / test rounds with exact
// per-cell occupancy in LDS: the bounce launches' kernel.
//
// Counted on the contest stand-in (cfg3, round 1): a segment visits 85
// cells, 4.3 of them non-empty, and tests 18.2 triangles; per wave the
// per-lane triangle loop ran 134 two-triangle trips for 9.1 per lane (6.8%
// of the lanes busy) and the walk 184 trips for 85 steps per lane.  Here:
//  * the exact occupancy of every cell sits in LDS (OccX), so a lane loads a
//    cell's [begin, end) only when the cell holds triangles, and the walk of
//    empty cells is DDA arithmetic plus one LDS lookup per 4^3 brick entered;
//  * a lane that reaches a non-empty cell issues the range load and PARKS
//    (its load is in flight while the others walk on);
//  * once `test_min` lanes are parked (or none walks) the wave runs one test
//    round: the (parked lane, triangle) pairs of all parked lanes are laid
//    out in lane order and tested 64 at a time, one pair per lane; each
//    parked lane keeps the lexicographic min of (t, ref) over its pairs with
//    0 < t < nearest -- exactly what the reference's in-order
//    `nearest > t and t > 0` loop keeps (stage3.zig:164-178: the smallest t,
//    the first ref among equal t; t > 0 orders like its bit pattern) -- and
//    walks on from that cell;
//  * finished lanes wait until `refill_min` of them are done, then write
//    their hit records (t, u, v, ref) together and take fresh paths from the
//    wave's chunk of the queue (persistent waves, dynamic fetch);
//    wf_shade_kernel then shades the hit records with whole waves
//    (traceRayRecursive's body, stage3.zig:195-219) and appends.
// Per lane the cells, the tests, their order semantics and the break test
// after every cell (stage3.zig:179-182) are the reference's: same hit.
//
// OccX (4^3-cell bricks): one bit per brick, 1 + the u16 number of
// occupied bricks before each 32-brick word, the zero mask, then one 64-bit
// cell mask per occupied brick.
// In LDS each 32-brick word sits beside its prefix as one 8-byte entry, so a
// lookup is two dependent LDS reads: (bits, prefix), then the mask.  The
// mask index is (1 + prefix + occupied bricks below b in the word) x (b's
// bit): an empty brick reads the zero mask at index 0, so nothing is
// selected after the load (5 VALU from the entry to the mask address,
// against 11 with the loaded mask zeroed by selects; the bit-field
// extracts use the hardware's 5-bit offset/width, so b needs no & 31).
struct OccX {
    const uint2* ent;                    // (brick bits, 1 + occupied bricks before the word)
    const unsigned long long* masks;     // [0]: zero mask
};
__device__ __forceinline__ unsigned long long occx_mask_at(const OccX& L, uint2 e, uint32_t b) {
    const uint32_t low = __builtin_amdgcn_ubfe(e.x, 0u, b);        // bits of the bricks below b
    const uint32_t bit = __builtin_amdgcn_ubfe(e.x, b, 1u);
    return L.masks[__umul24((uint32_t)__popc(low) + e.y, bit)];
}

__device__ __forceinline__ unsigned long long occx_mask(const OccX& L, uint32_t b) {
    return occx_mask_at(L, L.ent[b >> 5], b);
}
// occx_mask for a brick index that may lie past the grid (a speculative
// step beyond the exit cell): the word index is clamped into the blob, so
// the read stays inside it; the result of such a lookup is never used
__device__ __forceinline__ unsigned long long occx_mask_clamped(const OccX& L, uint32_t b, uint32_t nbw) {
    return occx_mask_at(L, L.ent[min(b >> 5, nbw - 1u)], b);
}
// occx_mask for a brick-major word (no clamp: the word stays inside the
// grid's packed range).  Laundering pc >> 11 saves the compiler's third
// address VALU ((pc >> 8) & ~7 + base) but measured neutral (r05al:
// cfg3 -0.2%, cfg2 / cfg5 +0.5%)
__device__ __forceinline__ unsigned long long occx_mask_bm(const OccX& L, uint32_t pc) {
    return occx_mask_at(L, L.ent[pc >> 11], pc >> 6);
}
// The 4^3 brick of a packed cell (DdaV): its coordinates are the fields'
// bits above their low two.  24-bit multiplies (full rate; v_mul_lo_u32 is
// quarter rate), exact because OccX serves only grids of at most 2^24
// bricks (occx_usable).
template <bool BM>
__device__ __forceinline__ uint32_t occx_brick(const WfParams& w, const DdaV& s) {
    if (BM) return s.pc >> 6;                              // (brick-major: the brick's linear index)
    const TraceParams& p = w.t;
    return __umul24(__builtin_amdgcn_ubfe(s.pc, p.ox2, p.ow2), w.occx_nb01) +
           __umul24(__builtin_amdgcn_ubfe(s.pc, p.ox1, p.ow1), w.occx_nb0) + __builtin_amdgcn_ubfe(s.pc, 2u, p.ow0);
}

// A parked lane's cell range [begin, end) is loaded by LDS-DMA into its
// wave's slots (begin at rng[lane], end at rng[64 + lane]): the load writes
// no VGPR, so the walk loop that keeps stepping the other lanes never waits
// on it (a VGPR destination made the compiler put a vmcnt(0) in the walk:
// its address registers doubled as the previous step's load destination,
// r02k ISA).  Nothing orders an LDS read behind a pending LDS-DMA but the
// wave's own vmcnt, so the test round drains vmcnt(0) before reading them.
constexpr int kParkWaves = kParkBlock / 64;
#ifndef ZRT_PARK_CHUNK
#define ZRT_PARK_CHUNK 256
#endif
// queue entries per work atomic of a park wave (r02d0, two pass sets: 128 vs
// 64 cfg3 +0.8%, cfg2 +1.1%, cfg5 +0.3%; 32 -2%; 256 +1.0 / -0.1 / +0.5%;
// r03za, on the round-3 kernels: 256 vs 128 cfg3 +0.5%, cfg5 +0.4%, cfg2
// -0.5%; 64 -0.7 / -1.0 / -0.5%)
constexpr uint32_t kParkChunk = ZRT_PARK_CHUNK;
// ZRT_PARK_LATE_DRAIN (below, the refill round): r05q, 2 rounds, images
// identical: cfg5 3576 / 3587 vs 3551 / 3553 (+0.8%, park -1%), cfg3 +0.1%,
// cfg2 +0.5% (profiles/r05/r05q_ab_park_late_drain.log)
#ifndef ZRT_PARK_LATE_DRAIN
#define ZRT_PARK_LATE_DRAIN 1
#endif
// ZRT_PARK_QPF: at the end of a refill round the wave pulls the lines of the
// next 64 queue entries of its chunk into L2 (one LDS-DMA dword per lane into
// a per-wave scratch slot that nothing reads), so the next refill round's
// record loads hit L2 instead of HBM.  The walk trips that follow do not wait
// for vector memory; the next test round's vmcnt(0) is the first wait behind
// the prefetch, and its ranges were issued after it.  Off: r06ab, 2 rounds,
// images identical: cfg3 6972 vs 6992 (-0.3%), cfg2 -0.4%, cfg5 3845 vs 3892
// (-1.2%) (profiles/r06/r06ab_ab_queue_prefetch.log): the extra request per
// lane and refill costs more than the record loads' HBM latency, which the
// SIMD's other park waves already hide
#ifndef ZRT_PARK_QPF
#define ZRT_PARK_QPF 0
#endif
// ZRT_PARK_ADAPT: a launch with few entries per wave (the last bounces, an
// 8-rank tile set) takes smaller chunks, down to 64, so the waves' last
// chunks end closer together (the launch tail).  r05e, alternating processes,
// 2 rounds, images identical: cfg3 5801 / 5810 vs 5765 / 5749 (+0.8%), cfg2
// +0.6%, cfg5 +0.1% (profiles/r05/r05e_ab_p96_park_adapt.log)
#ifndef ZRT_PARK_ADAPT
#define ZRT_PARK_ADAPT 1
#endif
// Park release (round 6): a parked lane whose cell has no ref left to test
// for the face it entered across (the entry-face mask is 0: every ref was
// tested in the cell it left) costs a test round nothing but its latency,
// and 54% of the parks on cfg3 are such (r06n).  Once a round's ranges have
// landed, a round with fewer than `rel_min` parked lanes that have refs to
// test is not run while lanes still walk: the empty ones walk on (what the
// round would have done with them), the others stay parked for the next
// round.  The context turns it on for scenes where enough of the occupied
// cells' entry faces have empty masks (context_release; ZRT_FLAG_RELEASE /
// ZRT_FLAG_NO_RELEASE force it): images identical either way.
//
// Issued by inline asm, not the builtin: the compiler treats an LDS-DMA like
// a store whose VGPR operands are read late, so whenever the register
// allocator reuses the address registers inside the walk it guards the reuse
// with a vmcnt(0) there -- every step then waits for the range load just
// issued (r02p ISA: the two-step walk got one after a register shuffle).
// The address is read when the instruction issues; the only consumer of the
// data is the test round, behind its explicit vmcnt(0), and the kernel drains
// vmcnt before it ends.  M0 cannot be declared clobbered (a reserved
// register: the clobber is ignored), so nothing else in the park kernel may
// rely on it: tests/test_codegen.py checks that every M0 access in its code
// object is this sequence.
// Range only (the segment's first cell: no cell was left, every ref is
// tested; the caller writes the all-ones mask itself).
__device__ __forceinline__ void park_load_range(const TraceParams& p, uint32_t pc, uint32_t* rng) {
    const uint32_t* c = p.cell32 + 8ull * pc;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)rng);
    // (an instruction offset would move the LDS destination too: the end
    // word gets its own address)
    asm volatile("s_mov_b32 m0, %2\n\t"
                 "global_load_lds_dword %0, off\n\t"
                 "s_add_u32 m0, m0, 0x100\n\t"
                 "global_load_lds_dword %1, off"
                 :
                 : "v"(c), "v"(c + 1), "s"(m0)
                 : "memory");
}
// Range and the mask of the refs to test for a ray that entered the cell
// across `face` (cell32_kernel) into rng[lane], rng[64 + lane], rng[128 + lane].
__device__ __forceinline__ void park_load_cell(const TraceParams& p, uint32_t pc, uint32_t face, uint32_t* rng) {
    const uint32_t* c = p.cell32 + 8ull * pc;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)rng);
    asm volatile("s_mov_b32 m0, %3\n\t"
                 "global_load_lds_dword %0, off\n\t"
                 "s_add_u32 m0, m0, 0x100\n\t"
                 "global_load_lds_dword %1, off\n\t"
                 "s_add_u32 m0, m0, 0x100\n\t"
                 "global_load_lds_dword %2, off"
                 :
                 : "v"(c), "v"(c + 1), "v"(c + 2 + face), "s"(m0)
                 : "memory");
}

// The escape-table word of a walking lane's current brick into its wave's
// escape slot esc[lane] (same LDS-DMA as park_load_range: no VGPR is written,
// the walk never waits for it; the lane reads the slot at the next trips,
// and a word for an earlier brick of the same ray is as valid as the current
// one: every cell after it lies on the ray further on).
__device__ __forceinline__ void park_load_esc(const uint32_t* word, uint32_t* esc) {
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)esc);
    asm volatile("s_mov_b32 m0, %1\n\t"
                 "global_load_lds_dword %0, off"
                 :
                 : "v"(word), "s"(m0)
                 : "memory");
}

// Per-wave LDS of the test rounds.
struct ParkSlot {
    float4 o[64];                    // lane's ray origin; w: nearest entering the round
    float4 d[64];                    // lane's ray direction; w (bits): ref of its pair slot 0
    unsigned long long best[64];     // per parked lane: (t bits << 32) | ref of its best pair
    float2 uv[64];                   // (u, v) of that pair
    uint32_t mark[64];               // lane + 1 of the parked lane whose pairs start at this slot
};

// Exclusive prefix sum over the wave (the whole wave must be active: every
// DPP read below runs under full EXEC).  Row scans by DPP row_shr with
// bound_ctrl (a source lane outside the row reads 0), rows joined through
// their last lanes.  NOT written as `rl >= k ? dpp(x) : 0`: that puts the
// DPP read under a partial EXEC, and gfx9 DPP treats a disabled source lane
// as invalid (tools/dpp_probe.hip; the cause of round 1's park-mode fault).
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t x, uint32_t lane, uint32_t& total) {
    uint32_t s = x;
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x111, 0xf, 0xf, true);   // row_shr:1
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x112, 0xf, 0xf, true);   // row_shr:2
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x114, 0xf, 0xf, true);   // row_shr:4
    s += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x118, 0xf, 0xf, true);   // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)s, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)s, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)s, 47);
    const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)s, 63);
    const uint32_t row = lane >> 4;
    s += row == 0u ? 0u : (row == 1u ? r0 : (row == 2u ? r0 + r1 : r0 + r1 + r2));
    total = r0 + r1 + r2 + r3;
    return s - x;
}

// ZRT_SWEEP builds only: per-wave s_memtime cycles of the three rounds and
// their activity (printed by zrt_context_render as zrt_park_profile; the
// stamps cost ~10% and never run in the product build).
#ifdef ZRT_SWEEP
#define PARK_PROF_DECL unsigned long long pprof[21] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
    uint64_t ptick = __builtin_amdgcn_s_memtime();
#define PARK_STAMP(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); pprof[k] += t_ - ptick; ptick = t_; } while (0)
#define PARK_COUNT(k, v) (pprof[k] += (v))
#else
#define PARK_PROF_DECL
#define PARK_STAMP(k) do { } while (0)
#define PARK_COUNT(k, v) do { } while (0)
#endif

// ZRT_PARK_WPE: the park kernel compiled for 5 waves per SIMD (at most 96
// VGPRs; it still runs 4, one 1024-thread workgroup per CU), so 4 x 96 leave
// 128 VGPRs per SIMD lane for a shade wave of 3 entries per lane (113) or a
// primary wave (80) of the other pass set.  r05t, 2 rounds, images identical:
// with ZRT_SHADE_N 3, cfg3 6014 / 6034 vs 6011 / 6017, cfg2 3902 / 3897 vs
// 3878 / 3838, cfg5 3584 / 3590 vs 3582 / 3594 (profiles/r05/r05t_ab_park96_shade3.log)
#ifndef ZRT_PARK_WPE
#define ZRT_PARK_WPE 5
#endif
#if ZRT_PARK_WPE
#define ZRT_PARK_ATTR __attribute__((amdgpu_waves_per_eu(ZRT_PARK_WPE, 8)))
#else
#define ZRT_PARK_ATTR
#endif
// ESC: with the escape table (context_escape decides per scene); PK_BM:
// brick-major packed words (dda.h)
template <bool ESC, bool PK_BM>
__global__ __launch_bounds__(kParkBlock) ZRT_PARK_ATTR void wf_park_kernel(const WfParams w) {
    const TraceParams& p = w.t;
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    __shared__ uint32_t s_rng[kParkWaves * 192];            // LDS-DMA range + face-mask slots
    uint32_t* const rng_slot = s_rng + 192u * (threadIdx.x >> 6);
    __shared__ uint32_t s_esc[kParkWaves * 64];             // escape-table words (park_load_esc)
    uint32_t* const esc_slot = s_esc + 64u * (threadIdx.x >> 6);
    __shared__ uint8_t s_sel8[256 * 8];                     // bit position of the r-th set bit of a byte
#if ZRT_PARK_QPF
    __shared__ uint32_t s_qpf[kParkWaves * 64];             // queue-record prefetch landing slots (never read)
    uint32_t* const qpf_slot = s_qpf + 64u * (threadIdx.x >> 6);
#endif
    for (uint32_t i = threadIdx.x; i < 256u * 8u; i += blockDim.x) {
        SEL8_ENTRY(i, pos);
        s_sel8[i] = (uint8_t)pos;
    }
    // OccX into LDS: (bits, prefix) entries, then the masks
    {
        const uint16_t* pre = reinterpret_cast<const uint16_t*>(w.occx + w.occx_nbw);
        uint2* ent = reinterpret_cast<uint2*>(s_dyn);
        for (uint32_t i = threadIdx.x; i < w.occx_nbw; i += blockDim.x) ent[i] = make_uint2(w.occx[i], pre[i]);
        for (uint32_t i = threadIdx.x; i < w.occx_words - w.occx_moff; i += blockDim.x)
            s_dyn[2 * w.occx_nbw + i] = w.occx[w.occx_moff + i];
    }
    __syncthreads();
    OccX L;
    L.ent = reinterpret_cast<const uint2*>(s_dyn);
    L.masks = reinterpret_cast<const unsigned long long*>(s_dyn + 2 * w.occx_nbw);
    ParkSlot& W = reinterpret_cast<ParkSlot*>(s_dyn + w.occx_ldsw)[threadIdx.x >> 6];

    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
    const uint32_t test_min = w.test_min, refill_min = w.refill_min, rel_min = w.rel_min;
    const GridK gk = grid_consts(p);
    constexpr uint32_t kIdle = 0, kWalk = 1, kPark = 2, kDone = 3;
    uint32_t st = kIdle;
    bool more = true;
    uint32_t grp = blockIdx.x & 7u, tried = 0;
    uint32_t cb = 0, ce = 0, cgrp = 0;     // the wave's current chunk of queue entries
    uint32_t chunk = kParkChunk;
    if (ZRT_PARK_ADAPT) {                  // (wave-uniform: the previous launch's final counts)
        uint32_t ntot = 0;
        for (uint32_t g = 0; g < 8u; ++g) ntot += w.n_in8[g * kCtr];
        const uint32_t per = ntot / (gridDim.x * (blockDim.x >> 6) * 4u);
        chunk = __builtin_amdgcn_readfirstlane(max(64u, min(kParkChunk, per & ~63u)));
    }
    // the segment: ray, DDA state, best hit, range
    v3 o = mk(0, 0, 0), d = mk(0, 0, 0);
    DdaV s;                                // grids of <= 1024 cells per axis (zrt_context_render)
    const PackK pk = p.pk;
    uint32_t fv0 = pk.f0, fv1 = pk.f1, fv2 = pk.f2;        // field masks in VGPRs (DDAV_STEPM)
    asm("" : "+v"(fv0), "+v"(fv1), "+v"(fv2));
    memset(&s, 0, sizeof s);
    float nearest = kInf, hu = 0.0f, hv = 0.0f;
    uint32_t hidx = 0;
    uint32_t qi = 0;                       // the path's queue entry
    // the ray's escape-table word (byte offset in a brick's kEscWords) and
    // bit; emask 0: the ray never stops early (no table, or a -inf / NaN
    // crossing sequence)
    uint32_t eoff = 0, emask = 0;
    uint32_t eb = ~0u;                     // the brick of the lane's last escape-table query
    PARK_PROF_DECL

    for (;;) {
        // ---- hit records + refill round, once enough lanes are finished or idle
        const uint64_t busy = __ballot(st == kWalk || st == kPark);
        if ((uint32_t)(64 - __popcll(busy)) >= refill_min || busy == 0ull) {
            PARK_COUNT(8, 1);
            PARK_COUNT(9, __popcll(__ballot(st == kDone)));
            if (__ballot(st == kDone) != 0ull) {
                // the hit record for wf_shade_kernel; then drain the stores:
                // otherwise the compiler guards the walk loop's reuse of their
                // data registers with a vmcnt(0) INSIDE the loop, which then
                // also waits for the previous step's range load, every step
                // (r02f ISA; walk 1304 cycles per step)
                const bool done = st == kDone;
                if (done) {
                    w.hit[qi] = make_float4(nearest, hu, hv, __uint_as_float(hidx));
                    st = kIdle;
                }
                if (!ZRT_PARK_LATE_DRAIN) __builtin_amdgcn_s_waitcnt(0x3f70);   // vmcnt(0)
            }
            bool loaded = false;                                   // (wave-uniform)
            PARK_STAMP(10);
            // idle lanes take entries of the wave's chunk [cb, ce) of group
            // cgrp, a new chunk of kParkChunk entries once it is used up: one
            // returning atomic per chunk instead of one per refill round
            uint64_t idle = __ballot(st == kIdle);
            while (idle != 0ull && (ce > cb || more)) {
                if (cb == ce) {
                    uint32_t base = 0, lim = 0;
                    more = wf_fetch<false>(w, chunk, grp, tried, base, lim);
                    PARK_STAMP(11);
                    if (!more) break;
                    cb = base;
                    ce = min(base + chunk, lim);
                    cgrp = grp;
                }
                const uint32_t take = min((uint32_t)__popcll(idle), ce - cb);
                const uint32_t rank = (uint32_t)__popcll(idle & below);
                if (st == kIdle && rank < take) {
                    {
                        qi = ent_index<false>(w, cgrp, cb + rank);
                        {
                            const float4 qa = w.q_in[3ull * qi], qb = w.q_in[3ull * qi + 1];
                            o = mk(qa.x, qa.y, qa.z);
                            d = mk(qb.x, qb.y, qb.z);
                        }
                        {                                          // queued paths have depth >= 1
                            nearest = kInf;
                            hu = hv = 0.0f;
                            hidx = 0;
                            W.o[lane] = make_float4(o.x, o.y, o.z, 0.0f);
                            W.d[lane] = make_float4(d.x, d.y, d.z, 0.0f);
                            Dda s0;
                            if (ZRT_FAST_QUOT ? dda_init_fq(p.bmin, p.bmax, p.res, p.cs, p.ics, p.cs_ok != 0u, o, d, s0)
                                              : dda_init(p.bmin, p.bmax, p.res, p.cs, o, d, s0)) {   // stage3.zig:153-156
                                ddav_from_t<PK_BM>(s0, gk, pk, s);
                                if (ESC) {
                                    // (every DMA into this slot from the lane's last
                                    // ray has landed before this store: that ray's
                                    // escape DMAs were issued before this refill's
                                    // q_in loads, vector memory completes in order
                                    // (vmcnt), and this store runs only after
                                    // dda_init consumed o and d, i.e. after the
                                    // compiler's wait for those loads.  With
                                    // ZRT_PARK_LATE_DRAIN the kDone drain no longer
                                    // sits between them; the parity suite renders
                                    // every scene with the table forced on)
                                    const uint32_t bin = esc_dir_bin(d);
                                    eoff = (bin >> 5) * 4u;
                                    emask = w.esc && s0.neg < 8u ? 1u << (bin & 31u) : 0u;
                                    eb = ~0u;
                                    esc_slot[lane] = 0u;
                                }
                                if (occx_cell<PK_BM>(occx_mask(L, occx_brick<PK_BM>(w, s)), s, pk)) {
                                    park_load_range(p, s.pc, rng_slot);
                                    rng_slot[128 + lane] = ~0u;    // first cell: every ref
                                    st = kPark;
                                } else {
                                    st = kWalk;
                                }
                            } else {
                                st = kDone;                        // misses the grid: nearest = +inf
                            }
                        }
                    }
                }
                PARK_STAMP(12);
                cb += take;
                loaded = loaded || take != 0u;
                idle = __ballot(st == kIdle);
            }
            // ZRT_PARK_LATE_DRAIN: the hit-record stores drain with the new
            // paths' record loads (vector memory completes in order); only a
            // round that loaded nothing drains them explicitly
            if (ZRT_PARK_LATE_DRAIN && !loaded) __builtin_amdgcn_s_waitcnt(0x3f70);
#if ZRT_PARK_QPF
            if (ce > cb) {
                const uint32_t j = min(cb + lane, ce - 1u);
                park_load_esc(reinterpret_cast<const uint32_t*>(w.q_in + 3ull * ent_index<false>(w, cgrp, j)), qpf_slot);
            }
#endif
            PARK_STAMP(0);
            if (__ballot(st != kIdle) == 0ull) {
                if (!more) break;
                continue;
            }
        }
        // ---- walk until test_min lanes are parked or nobody walks
        for (;;) {
            const uint64_t wk = __ballot(st == kWalk);
            if (wk == 0ull || (uint32_t)__popcll(__ballot(st == kPark)) >= test_min) break;
            PARK_COUNT(3, 1);
            PARK_COUNT(4, __popcll(wk));
            if (st == kWalk) {
                // ZRT_WALK_STEPS DDA steps per trip, every cell's lookup in
                // flight before any is used; the trip ends in the first cell
                // that ends the segment or holds triangles (steps after it
                // are speculative and dropped; their lookups read a clamped
                // brick).  Every boolean of the trip is a lane mask and every
                // select one v_cndmask on it (DDAV_STEPM: 179 VALU and no
                // branch per four-step trip, against 202 VALU, 14 v_mov and
                // four execz branches with per-lane booleans, r03p)
                constexpr int kS = ESC ? ZRT_WALK_STEPS : ZRT_WALK_STEPS_NOESC;
                static_assert(kS >= 2, "the trip keeps the cell before its last step");
                // the escape words landed so far (used at the trip's end, so the
                // read's latency hides behind the trip)
                const uint32_t ew = ESC ? esc_slot[lane] & emask : 0u;
                DdaV ss[kS];
                LaneM ex[kS], stop[kS], dd[kS];
                float te[kS];
                unsigned long long q[kS];
#pragma unroll
                for (int k = 0; k < kS; ++k) {
                    ss[k] = k ? ss[k - 1] : s;
                    DDAV_STEPM(ss[k], fv0, fv1, fv2, ex[k], te[k]);
                }
#pragma unroll
                // (brick-major words never leave the grid's packed range, pk_add
                // wraps inside a field, so their speculative lookups need no clamp)
                for (int k = 0; k < kS; ++k)
                    q[k] = PK_BM ? occx_mask_bm(L, ss[k].pc)
                                 : occx_mask_clamped(L, occx_brick<PK_BM>(w, ss[k]), w.occx_nbw);
#pragma unroll
                for (int k = 0; k < kS; ++k) asm volatile("" : "+v"(q[k]));
#pragma unroll
                for (int k = 0; k < kS; ++k) {
                    dd[k] = lm_or(ex[k], lm_of(nearest <= te[k]));
                    stop[k] = lm_or(dd[k], lm_of(occx_cell<PK_BM>(q[k], ss[k], pk)));
                }
                // the first stopping step wins: from the last step back (the
                // last step's selects are identities)
                DdaV sel = ss[kS - 1];
                uint32_t prev = ss[kS - 2].pc;
                LaneM pkd = lm_andn(stop[kS - 1], dd[kS - 1]), dn = dd[kS - 1];
#pragma unroll
                for (int k = kS - 2; k >= 0; --k) {
                    sel.tn0 = lm_sel(stop[k], ss[k].tn0, sel.tn0);
                    sel.tn1 = lm_sel(stop[k], ss[k].tn1, sel.tn1);
                    sel.tn2 = lm_sel(stop[k], ss[k].tn2, sel.tn2);
                    sel.pc = lm_selu(stop[k], ss[k].pc, sel.pc);
                    prev = lm_selu(stop[k], k ? ss[k - 1].pc : s.pc, prev);
                    pkd = lm_or(lm_andn(pkd, stop[k]), lm_andn(stop[k], dd[k]));
                    dn = lm_or(lm_andn(dn, stop[k]), dd[k]);
                }
#ifdef ZRT_SWEEP
                {   // lane steps taken (up to the stopping one), those into cells of
                    // empty bricks, and those that entered an empty brick
                    LaneM alive = lm_of(true);
                    uint32_t pcp = s.pc;
#pragma unroll
                    for (int k = 0; k < kS; ++k) {
                        const LaneM emp = lm_of(q[k] == 0ull);
                        const LaneM ent = lm_of(((pcp ^ ss[k].pc) & ~pk.low2) != 0u);
                        PARK_COUNT(13, __popcll(alive));
                        PARK_COUNT(14, __popcll(lm_and(alive, emp)));
                        PARK_COUNT(15, __popcll(lm_and(lm_and(alive, emp), ent)));
                        alive = lm_andn(alive, stop[k]);
                        pcp = ss[k].pc;
                    }
                }
#endif
                st = lm_selu(dn, kDone, st);
                s = sel;
                if (lm_selu(pkd, 1u, 0u)) {
                    const uint32_t x = s.pc ^ prev;
                    const uint32_t face = (x & pk.f0) ? (s.d0 >> 31)
                                                      : ((x & pk.f1) ? 2u + (s.d1 >> 31) : 4u + (s.d2 >> 31));
                    park_load_cell(p, s.pc, face, rng_slot);
                    st = kPark;
                }
                if (ESC) {
                    // a set escape bit: no cell of the ray after the queried
                    // brick holds a triangle, so the hit so far stands (this
                    // trip cannot have parked the lane: escape.h)
                    const LaneM esc = lm_and(lm_of(st == kWalk), lm_of(ew != 0u));
                    PARK_COUNT(16, __popcll(esc));
                    st = lm_selu(esc, kDone, st);
                    // one query per brick the ray enters (its word does not
                    // change while the lane walks inside the brick)
                    const uint32_t b = occx_brick<PK_BM>(w, s);
                    if (st == kWalk && emask != 0u && b != eb) {
                        park_load_esc(reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(w.esc) +
                                                                        b * (4u * kEscWords) + eoff),
                                      esc_slot);
                        eb = b;
                    }
                }
            }
        }
        PARK_STAMP(1);
        // ---- test round: the parked lanes' cells, all pairs over all lanes
        if (__ballot(st == kPark) != 0ull) {
            __builtin_amdgcn_s_waitcnt(0x3f70);                    // vmcnt(0): the ranges landed
            PARK_STAMP(20);                                        // (sweep: the round's wait for them)
            const bool ready = st == kPark;
            // the parked cell's refs still to test: those the mask keeps
            // (cells of at most 32 refs; larger ones test every ref)
            const uint32_t rb = rng_slot[lane], re = rng_slot[64 + lane], cnt = re - rb;
            const uint32_t keep = cnt < 32u ? rng_slot[128 + lane] & ((1u << cnt) - 1u) : rng_slot[128 + lane];
            const uint32_t n = ready ? (cnt <= 32u ? (uint32_t)__popc(keep) : cnt) : 0u;
            // park release (above): a round with fewer than rel_min parked
            // lanes that have refs to test is not run while lanes walk
            if (rel_min != 0u && __ballot(st == kWalk) != 0ull &&
                (uint32_t)__popcll(__ballot(ready && n != 0u)) < rel_min &&
                (uint32_t)__popcll(__ballot(ready && n == 0u)) >= w.rel_emin) {
                PARK_COUNT(19, __popcll(__ballot(ready && n == 0u)));
                if (ready && n == 0u) st = kWalk;
                continue;
            }
            uint32_t tot = 0;
            const uint32_t off = wave_excl_sum(n, lane, tot);
            PARK_COUNT(5, 1);
            PARK_COUNT(6, (tot + 63u) / 64u);
            PARK_COUNT(7, tot);
            PARK_COUNT(17, __popcll(__ballot(ready)));               // parked lanes tested
            PARK_COUNT(18, __popcll(__ballot(ready && n == 0u)));    // ... with no ref left to test
            W.o[lane].w = nearest;
            rng_slot[lane] = rb;                                   // (the slots are free until the walk)
            rng_slot[64 + lane] = off;
            rng_slot[128 + lane] = cnt <= 32u ? keep : ~0u;
            W.best[lane] = ~0ull;
            uint32_t carry = 0;
            for (uint32_t r = 0; r < tot; r += 64u) {
                // owner of pair slot r + lane: the last parked lane starting
                // at or before it (mark), or the one running over from r - 1
                W.mark[lane] = 0u;
                __builtin_amdgcn_wave_barrier();
                if (n != 0u && off >= r && off < r + 64u) W.mark[off - r] = lane + 1u;
                __builtin_amdgcn_wave_barrier();
                const uint64_t starts = __ballot(W.mark[lane] != 0u);
                const uint64_t upto = starts & (~0ull >> (63u - lane));
                const uint32_t owner = upto ? W.mark[63u - (uint32_t)__builtin_clzll(upto)] - 1u : carry;
                carry = (uint32_t)__builtin_amdgcn_readlane((int)owner, 63);
                const uint32_t g = r + lane;
                const float4 ro = W.o[owner], rd = W.d[owner];
                // pair g is the owner's (g - off)-th kept ref
                const uint32_t kr = g - rng_slot[64 + owner];
                const uint32_t j = rng_slot[owner] + (kr < 32u ? select_bit(s_sel8, rng_slot[128 + owner], kr) : kr);
                bool cand = false;
                float t = 0.0f, u = 0.0f, v = 0.0f;
                if (g < tot) {
                    v3 A, B, C;
                    load_tri(p, j, A, B, C);
                    cand = tri_ray_flat(A, B, C, mk(ro.x, ro.y, ro.z), mk(rd.x, rd.y, rd.z), &t, &u, &v) &&
                           ro.w > t && t > 0.0f;                   // stage3.zig:172
                }
                const unsigned long long key = ((unsigned long long)__float_as_uint(t) << 32) | j;
                if (cand) atomicMin(&W.best[owner], key);
                __builtin_amdgcn_wave_barrier();
                if (cand && W.best[owner] == key) W.uv[owner] = make_float2(u, v);
                __builtin_amdgcn_wave_barrier();
            }
            if (n != 0u) {
                const unsigned long long k = W.best[lane];
                if (k != ~0ull) {
                    nearest = __uint_as_float((uint32_t)(k >> 32));
                    hidx = (uint32_t)k;
                    const float2 uv = W.uv[lane];
                    hu = uv.x;
                    hv = uv.y;
                }
            }
            if (ready) st = kWalk;                                 // the cell is done: step out of it next
        }
        PARK_STAMP(2);
    }
    __builtin_amdgcn_s_waitcnt(0x3f70);                            // vmcnt(0): no LDS-DMA outlives the wave
#ifdef ZRT_SWEEP
    if (lane == 0)
        for (int k = 0; k < 13; ++k) atomicAdd(&p.stats[16 + k], pprof[k]);
    if (lane == 0)
        for (int k = 13; k < 21; ++k) atomicAdd(&p.stats[48 + k - 13], pprof[k]);
#endif
}

// Split launches: the shading half of a bounce (traceRayRecursive's body
// after traceRay, stage3.zig:195-219) over the hit records wf_park_kernel
// wrote, one lane per path with every lane of the wave busy, appending the
// continuing paths to the next queue.  Same XCD group order as the trace.
// One path of the shading half, its state decoded and its hit record h
// loaded: shades, writes the terminal radiance of an ending path and appends
// a continuing one (the whole wave calls it).
__device__ __forceinline__ void shade_path(const WfParams& w, const double* zx, const double* zf,
                                           const DevMat* mats, bool valid,
                                           uint32_t item, v3 o, v3 d, uint32_t depth, uint32_t slot, Rng rng,
                                           uint32_t mask, float4 h, const TriRec& tr, uint64_t below, uint32_t grp,
                                           uint32_t& n_seg, unsigned long long* sp = nullptr) {
    bool cont = false;
    if (valid) {
        v3 L = mk(0, 0, 0);
        ++n_seg;                               // queued / primary paths have depth >= 1
        cont = shade_segment(w, zx, zf, mats, item, h.x, h.y, h.z, tr, o, d, depth, slot, rng, mask, L, sp);
        if (!cont) w.term[item] = make_float4(L.x, L.y, L.z, __uint_as_float(mask));
    }
    SHADE_STAMP(6, o.x);                       // the rest of the segment (misses, pass-through, terminal store)
    wf_append(w, cont, below, o, d, item, depth, slot, rng, mask, grp);
    SHADE_STAMP(7, o.x);                       // append
}

// One queue entry: its path record (a, b, c) and hit record h already loaded.
__device__ __forceinline__ void shade_entry(const WfParams& w, const double* zx, const double* zf,
                                            const DevMat* mats, bool valid,
                                            float4 a, float4 b, float4 c, float4 h, const TriRec& tr,
                                            uint64_t below, uint32_t grp, uint32_t& n_seg,
                                            unsigned long long* sp = nullptr) {
    Rng rng;
    rng.s = ((uint64_t)__float_as_uint(c.y) << 32) | __float_as_uint(c.x);
    shade_path(w, zx, zf, mats, valid, __float_as_uint(a.w), mk(a.x, a.y, a.z), mk(b.x, b.y, b.z),
               __float_as_uint(b.w) & 0xFFFFu, __float_as_uint(b.w) >> 16, rng, __float_as_uint(c.z), h, tr,
               below, grp, n_seg, sp);
}
// ZRT_SHADE_EARLY_APPEND: whether a path continues is known from its records
// alone (shade_segment: a hit with depth >= 2 continues, whether it scatters
// or passes through; a miss ends), so the wave reserves its appends with one
// returning atomic right after the records land and the atomic's latency
// overlaps the shading chain (triangle data -> texels -> RNG) instead of
// following it; the path is stored at its reserved position.  r05m,
// alternating processes, 2 rounds, images identical: cfg3 6019 / 6008 vs 5895
// / 5877 (+2.2%), cfg5 +0.6%, cfg2 ±0; one-stream shade 23.3-27.0 -> 18.3-18.6
// ms per cfg3 frame (profiles/r05/r05m_ab_shade_early_append.log)
#ifndef ZRT_SHADE_EARLY_APPEND
#define ZRT_SHADE_EARLY_APPEND 1
#endif
#ifndef ZRT_SHADE_LAST
#define ZRT_SHADE_LAST 1
#endif
// its entries per lane per fetch and launch bound: r06f, 3 rounds of
// alternating processes at full spp, images identical, against no LAST
// kernel (6518 / 3851 / 4165 Mrays/s cfg3 / cfg5 / cfg2): 4 entries (78
// VGPRs) 6586 / 3859 / 4193 (+1.0 / +0.2 / +0.7%); 3 entries (65) 6580 /
// 3845 / 4170; 2 entries at 8 waves per SIMD (52 VGPRs: two waves fit beside
// four park waves) 6564 / 3832 / 4123 (profiles/r06/r06f_ab_shade_last.log)
#ifndef ZRT_SHADE_LAST_MINW
#define ZRT_SHADE_LAST_MINW 1
#endif
#ifndef ZRT_SHADE_LAST_N
#define ZRT_SHADE_LAST_N 4
#endif
__device__ __forceinline__ bool shade_continues(bool valid, float4 b, float4 h) {
    return valid && h.x != kInf && (__float_as_uint(b.w) & 0xFFFFu) >= 2u;
}
// One entry (records loaded) shaded: an ending path writes its terminal
// radiance; a continuing one is left in (o, d, item, depth, slot, rng, mask)
// for the caller to store at its reserved position.  Returns shade_segment's
// answer (false for an invalid entry), which must equal shade_continues':
// the ZRT_SWEEP build counts disagreements (stats[60]) and fails the render
// on any.
struct ShadeOut {
    v3 o, d;
    uint32_t item, depth, slot, mask;
    Rng rng;
};
template <bool LAST = false>
__device__ __forceinline__ bool shade_entry_keep(const WfParams& w, const double* zx, const double* zf,
                                                 const DevMat* mats, bool valid, float4 a, float4 b, float4 c,
                                                 float4 h, const TriRec& tr, ShadeOut& so, uint32_t& n_seg,
                                                 unsigned long long* sp = nullptr) {
    if (!valid) return false;
    so.rng.s = ((uint64_t)__float_as_uint(c.y) << 32) | __float_as_uint(c.x);
    so.item = __float_as_uint(a.w);
    so.o = mk(a.x, a.y, a.z);
    so.d = mk(b.x, b.y, b.z);
    so.depth = __float_as_uint(b.w) & 0xFFFFu;
    so.slot = __float_as_uint(b.w) >> 16;
    so.mask = __float_as_uint(c.z);
    v3 L = mk(0, 0, 0);
    ++n_seg;
    const bool cont = shade_segment<LAST>(w, zx, zf, mats, so.item, h.x, h.y, h.z, tr, so.o, so.d, so.depth,
                                          so.slot, so.rng, so.mask, L, sp);
    if (!cont) w.term[so.item] = make_float4(L.x, L.y, L.z, __uint_as_float(so.mask));
    return cont;
}

// LMATS: the material descriptors (at most kLdsMats) copied to dynamic LDS
// (nmat x 96 B: the shade kernel's LDS stays small, so its workgroups still
// fit beside the other pass set's park kernel), so the dependent chain
// hit -> triangle data -> material -> texels takes its material hop from LDS
// instead of L2.
constexpr uint32_t kLdsMats = 64;
// LAST: the launch of a pass's last bounce (every entry has depth 1): the
// terminal radiance only (shade_segment<true>), no append (ZRT_SHADE_LAST)
template <bool LMATS, bool LAST = false>
#ifndef ZRT_SHADE_MINW
#define ZRT_SHADE_MINW 1
#endif
__global__ __launch_bounds__(kTraceBlock, LAST ? ZRT_SHADE_LAST_MINW : ZRT_SHADE_MINW) void wf_shade_kernel(const WfParams w) {
    constexpr int NE = LAST ? ZRT_SHADE_LAST_N : kShadeEntries;   // entries per lane per fetch
    const TraceParams& p = w.t;
    __shared__ double s_zig[514];
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dynm[];    // LMATS: p.nmat DevMat
    DevMat* const s_mats = reinterpret_cast<DevMat*>(s_dynm);
    for (uint32_t i = threadIdx.x; i < 514; i += blockDim.x) s_zig[i] = p.zig[i];
    if (LMATS)
        for (uint32_t i = threadIdx.x; i < p.nmat * (uint32_t)(sizeof(DevMat) / 4); i += blockDim.x)
            reinterpret_cast<uint32_t*>(s_mats)[i] = reinterpret_cast<const uint32_t*>(p.mats)[i];
    __syncthreads();
    const DevMat* const mats = LMATS ? s_mats : p.mats;
    const double* zx = s_zig;
    const double* zf = s_zig + 257;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
    uint32_t n_seg = 0;
    uint32_t grp = blockIdx.x & 7u, tried = 0;
    WfParams ws = w;
    ws.fetch8 = w.fetch8s;
    const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#ifdef ZRT_SWEEP
    // ZRT_SWEEP builds: per-wave cycles and active lanes of the shading phases
    // (SHADE_STAMP; printed as zrt_shade_profile with ZRT_PARK_PROFILE)
    __shared__ unsigned long long s_sprof[kTraceBlock / 64][17];
    unsigned long long* const sp = s_sprof[threadIdx.x >> 6];
    if (lane < 16) sp[lane] = 0;
    if (lane == 16) sp[16] = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_wave_barrier();
#else
    unsigned long long* const sp = nullptr;
#endif
    // NE entries per lane per fetch: every entry's records are
    // loaded before the first is shaded, so their latency overlaps the
    // earlier entries' dependent chains (2: cfg3 +1.2%, cfg2 / cfg5 within
    // noise, 112 VGPRs, r02c6)
    for (;;) {
        uint32_t base = 0, lim = 0;
        if (!wf_fetch<false>(ws, 64u * NE, grp, tried, base, lim)) break;
        SHADE_STAMP(0, base);                  // work atomic
        float4 a[NE], b[NE], c[NE], h[NE];
        bool hit[NE];
        {
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                const uint32_t j = base + 64u * e + lane;
                a[e] = b[e] = c[e] = h[e] = z4;
                hit[e] = j < lim;
                if (j < lim) {
                    const uint32_t i = ent_index<false>(w, grp, j);
                    a[e] = w.q_in[3ull * i]; b[e] = w.q_in[3ull * i + 1]; c[e] = w.q_in[3ull * i + 2]; h[e] = w.hit[i];
                }
            }
        }
        if (LAST) {
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                ShadeOut so;
                (void)shade_entry_keep<true>(w, zx, zf, mats, hit[e], a[e], b[e], c[e], h[e],
                                             tri_rec(p, hit[e] ? h[e].x : kInf, __float_as_uint(h[e].w)), so, n_seg,
                                             sp);
            }
        } else if (ZRT_SHADE_EARLY_APPEND) {
            bool pc[NE];
            uint64_t m[NE];
            uint32_t tot = 0;
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                pc[e] = shade_continues(hit[e], b[e], h[e]);
                m[e] = __ballot(pc[e]);
                tot += (uint32_t)__popcll(m[e]);
            }
            uint32_t ob = 0;
            if (lane == 0 && tot != 0u) ob = atomicAdd(&w.n_out8[grp * kCtr], tot);
            uint32_t before = 0;
            // (each entry's triangle record loaded as its shading starts: all
            // of them up front took 100 VGPRs and lost co-residency, r05c)
#pragma unroll
            for (int e = 0; e < NE; ++e) {
                ShadeOut so;
                const bool cont = shade_entry_keep(w, zx, zf, mats, hit[e], a[e], b[e], c[e], h[e],
                                                   tri_rec(p, hit[e] ? h[e].x : kInf, __float_as_uint(h[e].w)), so,
                                                   n_seg, sp);
#ifdef ZRT_SWEEP
                if (cont != pc[e]) atomicAdd(&p.stats[60], 1ull);
#else
                (void)cont;
#endif
                // (converged again: lane 0's reservation, long returned, reaches every lane)
                const uint32_t base = __builtin_amdgcn_readfirstlane(ob) + region_base(w, grp) + before;
                if (pc[e]) q_store(w, base + (uint32_t)__popcll(m[e] & below), so.o, so.d, so.item, so.depth, so.slot,
                                   so.rng, so.mask);
                before += (uint32_t)__popcll(m[e]);
            }
        } else {
#pragma unroll
            for (int e = 0; e < NE; ++e)
                shade_entry(w, zx, zf, mats, hit[e], a[e], b[e], c[e], h[e],
                            tri_rec(p, hit[e] ? h[e].x : kInf, __float_as_uint(h[e].w)), below, grp, n_seg, sp);
        }
    }
    const unsigned long long s0 = wave_sum(n_seg);
    if (lane == 0) atomicAdd(&p.stats[0], s0);
#ifdef ZRT_SWEEP
    if (lane == 0)
        for (int k = 0; k < 16; ++k) atomicAdd(&p.stats[32 + k], sp[k]);
#endif
}

// Fold + ordered sample sum + toRGB for wavefront mode (stage3.zig:219,
// :236-242): per sample, L = terminal radiance, then e + a*L for every slot
// that scattered, from the last bounce back to the first.  Items are
// pixel-major, so a block takes kResPix pixels and folds their samples
// kResSmp at a time with consecutive lanes on consecutive items (16 lanes
// read one pixel's 16 records: 256-byte runs), parks the radiances in LDS,
// and one thread per pixel then adds them in sample order (renderWorker's
// `pixel = pixel.add(...)` chain, unchanged: the same f32 sum).
constexpr uint32_t kResPix = 64, kResSmp = 16, kResRow = kResSmp * 3 + 1;   // +1: no LDS bank conflict
__global__ __launch_bounds__(kBlock) void wf_resolve_kernel(const float4* __restrict__ term,
                                                            const float4* __restrict__ stk4,
                                                            const float2* __restrict__ stk2, uint32_t T,
                                                            uint32_t P, uint32_t S, uint32_t max_bounce,
                                                            float4* acc, int first, int last,
                                                            float inv_spp, uint8_t* rgb, float* lin) {
    __shared__ float s_l[kResPix * kResRow];
    const uint32_t q0 = blockIdx.x * kResPix;
    const uint32_t np = min(kResPix, P - q0);
    const uint32_t tid = threadIdx.x;
    const uint32_t q = q0 + tid;
    v3 px = mk(0, 0, 0);
    if (tid < np && !first) { const float4 a = acc[q]; px = mk(a.x, a.y, a.z); }
    for (uint32_t c = 0; c < S; c += kResSmp) {
        const uint32_t ns = min(kResSmp, S - c);
        for (uint32_t m = tid; m < kResPix * kResSmp; m += kBlock) {
            const uint32_t i = m / kResSmp, k = m % kResSmp;   // the block's pixel i, sample c + k
            if (i < np && k < ns) {
                const uint32_t item = (q0 + i) * S + c + k;
                const float4 tm = term[item];
                v3 L = mk(tm.x, tm.y, tm.z);
                const uint32_t mask = __float_as_uint(tm.w);
                for (int slot = (int)max_bounce - 1; slot >= 0; --slot) {
                    if ((mask >> slot) & 1u) {
                        if (ZRT_PLANES16) {
                            // e = +0 exactly when the hit stored no emissive plane
                            const float4 a = stk4[(uint64_t)slot * T + item];
                            v3 e = mk(0.0f, 0.0f, 0.0f);
                            if (__float_as_uint(a.w) != 0u) {
                                const float4 ee = reinterpret_cast<const float4*>(stk2)[(uint64_t)slot * T + item];
                                e = mk(ee.x, ee.y, ee.z);
                            }
                            L = add(e, mul(mk(a.x, a.y, a.z), L));
                        } else {
                            const float4 e = stk4[(uint64_t)slot * T + item];
                            const float2 a = stk2[(uint64_t)slot * T + item];
                            L = add(mk(e.x, e.y, e.z), mul(mk(e.w, a.x, a.y), L));
                        }
                    }
                }
                float* dst = s_l + i * kResRow + 3u * k;
                dst[0] = L.x; dst[1] = L.y; dst[2] = L.z;
            }
        }
        __syncthreads();
        if (tid < np) {
            const float* src = s_l + tid * kResRow;
            for (uint32_t k = 0; k < ns; ++k) px = add(px, mk(src[3 * k], src[3 * k + 1], src[3 * k + 2]));
        }
        __syncthreads();
    }
    if (tid >= np) return;
    if (!last) { acc[q] = make_float4(px.x, px.y, px.z, 0.0f); return; }
    const v3 l = mul(px, mk(inv_spp, inv_spp, inv_spp));
    uint8_t c[3];
    to_rgb(l, c);
    rgb[3 * (size_t)q + 0] = c[0];
    rgb[3 * (size_t)q + 1] = c[1];
    rgb[3 * (size_t)q + 2] = c[2];
    if (lin) { lin[3 * (size_t)q] = l.x; lin[3 * (size_t)q + 1] = l.y; lin[3 * (size_t)q + 2] = l.z; }
}

// renderWorker tail (stage3.zig:236-242) for the counting megakernel:
// ordered per-pixel sum over this pass's samples, then (last pass) * (1/spp)
// and toRGB.
__global__ __launch_bounds__(kBlock) void resolve_kernel(const float4* __restrict__ out, uint32_t P,
                                                         uint32_t S, float4* acc, int first, int last,
                                                         float inv_spp, uint8_t* rgb, float* lin) {
    const uint32_t q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= P) return;
    v3 px = mk(0, 0, 0);
    if (!first) { const float4 a = acc[q]; px = mk(a.x, a.y, a.z); }
    for (uint32_t s = 0; s < S; ++s) {
        const float4 c = out[(size_t)q * S + s];          // pixel-major items
        px = add(px, mk(c.x, c.y, c.z));
    }
    if (!last) { acc[q] = make_float4(px.x, px.y, px.z, 0.0f); return; }
    const v3 l = mul(px, mk(inv_spp, inv_spp, inv_spp));
    uint8_t c[3];
    to_rgb(l, c);
    rgb[3 * (size_t)q + 0] = c[0];
    rgb[3 * (size_t)q + 1] = c[1];
    rgb[3 * (size_t)q + 2] = c[2];
    if (lin) { lin[3 * (size_t)q] = l.x; lin[3 * (size_t)q + 1] = l.y; lin[3 * (size_t)q + 2] = l.z; }
}

using TraceFn = void (*)(const TraceParams);
using WfFn = void (*)(const WfParams);

// wf_kernel occupancy (waves per SIMD, __launch_bounds__).  The primary
// launch at 7 (72 VGPRs, no scratch access inside the cell walk): r02ah, one
// box, cfg3 64 spp at 5 / 6 / 7 / 8 waves 3127 / 3155 / 3197 / 3193 Mrays/s
// (8 reloads spills inside the walk).  The lane-walk bounce launches
// (ZRT_FLAG_LANE_WALK) at 6: 7 waves put 2-3 spill reloads in that walk and
// ran cfg3 at 1933 vs 2108 (round 1).  tests/test_codegen.py checks every
// instantiation zrt_timed_kernels names.
#ifndef ZRT_WF_MINW
#define ZRT_WF_MINW 6
#endif
// r04pw (the frustum-bound primary): 6 / 7 / 8 waves cfg3 5732 / 5724 / 5692,
// cfg5 3491 / 3489 / 3493, cfg2 3778 / 3739 / 3725 Mrays/s; at 6 the primary
// has no scratch access at all (12 at 7, 26 and walk reloads at 8).  Built
// without SLP pairing (Makefile) the packed primary fits 7 waves (72 VGPRs,
// no spill): r05ap, cfg3 6412 / 6400 vs 6346 / 6357 (+0.9%), cfg2 +0.7%,
// cfg5 +0.3% (profiles/r05/r05ap_ab_primary7_select.log).  Round 6: the
// entry-face skip (ZRT_WALK_FACE_SKIP) spills 6-10 VGPRs at 7 waves, some in
// the walk loop of the frustum instantiation; at 6 waves it spills nothing
// and measured the same (r06af / r06ag: cfg3 +0.9 / +1.3% vs +1.3 / +1.2%
// at 7 over the 7-wave tree without the skip).  With one triangle load in
// flight per lane (ZRT_TRI_BATCH 1) the primary fits 7 waves again (70
// VGPRs, no spill): r06bi / r06bj
#ifndef ZRT_WF_MINW0
#define ZRT_WF_MINW0 7
#endif
constexpr int kWfMinWaves = ZRT_WF_MINW;
constexpr int kWfMinWaves0 = ZRT_WF_MINW0;
// wf_park_kernel schedule: a test round once 14 lanes are parked, a shade +
// refill round once 16 lanes are finished (cfg3 64 spp sweep, r02d: T 4-16 x
// R 8/16/32; T 12 R 16 3110 Mrays/s, T 8-16 R 16 within 1.3%, R 8 -15%,
// R 32 -13%; cfg5 T 16 R 16 2075, T 8 2055; full spp after the lane-mask
// trip, r03z: T 14 vs 12 cfg3 +0.3%, cfg2 +0.6%, cfg5 +0.5%; T 10 / 16,
// R 12 / 20 no better).  On round 5's final tree (cheaper walk trips and
// test rounds) R 20 is ahead everywhere: r05au / r05av, 2 + 2 rounds, cfg3
// +0.9 / +0.5%, cfg5 +0.25 / +0.3%, cfg2 +0.3 / +0.2%; T 12 / 16 / 18 and
// R 12 / 24 are not (profiles/r05/r05au_ab_o2_park_schedule.log,
// r05av_ab_park_schedule2.log).  ZRT_SWEEP builds read ZRT_PARK_T / ZRT_PARK_R.
#ifndef ZRT_PARK_T
#define ZRT_PARK_T 14
#endif
#ifndef ZRT_PARK_R
#define ZRT_PARK_R 20
#endif
constexpr uint32_t kParkTestMin = ZRT_PARK_T;
#ifndef ZRT_PARK_T_REL
#define ZRT_PARK_T_REL 12
#endif
constexpr uint32_t kParkTestMinRel = ZRT_PARK_T_REL;   // with the park release
constexpr uint32_t kParkRefillMin = ZRT_PARK_R;
// packed walk state when every axis has at most kPackMaxRes cells
const WfFn kWfPrimary = (WfFn)wf_kernel<kWfMinWaves0, true, true>;
const WfFn kWfBounce = (WfFn)wf_kernel<kWfMinWaves, false, true>;
const WfFn kWfPrimaryBM = (WfFn)wf_kernel<kWfMinWaves0, true, true, true>;
const WfFn kWfBounceBM = (WfFn)wf_kernel<kWfMinWaves, false, true, true>;
const WfFn kWfPrimaryWide = (WfFn)wf_kernel<kWfMinWaves, true, false>;   // (6 waves: at 7 it spills)
const WfFn kWfBounceWide = (WfFn)wf_kernel<kWfMinWaves, false, false>;
// scenes with an edge component of 2^62 or more, or infinite
// (zrt_context::mt_exact): the unpacked lane walk with the IEEE division in
// Moller-Trumbore, for every launch
const WfFn kWfPrimaryExact = (WfFn)wf_kernel<kWfMinWaves, true, false, false, true>;
const WfFn kWfBounceExact = (WfFn)wf_kernel<kWfMinWaves, false, false, false, true>;

// max_bounce picks the stack depth the counting kernel is compiled for.
TraceFn count_fn(uint32_t max_bounce) {
    if (max_bounce <= 4) return (TraceFn)trace_kernel<4>;
    if (max_bounce <= 8) return (TraceFn)trace_kernel<8>;
    if (max_bounce <= 16) return (TraceFn)trace_kernel<16>;
    if (max_bounce <= 32) return (TraceFn)trace_kernel<32>;
    return nullptr;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <typename T>
int grow(T** p, size_t* cap, size_t n) {
    if (*cap >= n && *p) return ZRT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
    *cap = n;
    return ZRT_OK;
}

// OccX (wf_park_kernel): LDS left for the blob in one 1024-thread workgroup
// per CU after the per-wave ParkSlots and the static ziggurat tables.
constexpr size_t kLdsPerCu = 160 * 1024;
// pass sets in flight (streams) by default, and at most (ZRT_SWEEP: ZRT_SETS)
constexpr uint32_t kPassSets = 2;
constexpr uint32_t kMaxPassSets = 4;
constexpr uint64_t kSetsMinSamples = 1ull << 23;   // samples of a frame that runs kPassSets
constexpr uint64_t kFrustumMinSamples = 1ull << 23; // samples of a frame that computes the frustum bounds
// % of a pass moved from the last pass to the first when two sets run (r02d7,
// vs 0: 20% cfg3 +3.2%, cfg5 +0.2%, cfg2 -1.0%; 16% cfg3 +1.4%; 25% cfg3
// +3.2%, cfg2 -1.7%; the response is bumpy: r02d5/d6 sweeps)
#ifndef ZRT_LEAD_PCT
#define ZRT_LEAD_PCT 20
#endif
constexpr uint32_t kLeadPct = ZRT_LEAD_PCT;
constexpr size_t kParkSlotsBytes = (kParkBlock / 64) * sizeof(ParkSlot);
constexpr size_t kOccxBudget = kLdsPerCu - kParkSlotsBytes - 514 * sizeof(double) - kParkWaves * 192 * 4 - 256 -
                                256 * 8 -   // the select table
                                kParkWaves * 64 * 4 -  // the escape slots
                                (ZRT_PARK_QPF ? kParkWaves * 64 * 4 : 0);   // the prefetch slots

}  // namespace

struct zrt_context {
    int device = 0;
    uint32_t mem_share = 1;            // contexts rendering on this device at once (a group's repeats)
    hipStream_t stream = nullptr;
    hipEvent_t ev_begin = nullptr, ev_end = nullptr;
    std::vector<hipEvent_t> ev_trace;
    zrt_grid grid{};
    uint32_t ncells = 0, nrefs = 0, nmat = 0;
    uint2* d_cells = nullptr;
    // packed walks (DdaV): the layout and the cells indexed by the packed word
    PackK pk{};
    bool packed = false;
    uint32_t* d_cell32 = nullptr;      // cell records at the packed index (cell32_kernel)
    float* d_pos = nullptr;
    float4* d_data = nullptr;
    DevMat* d_mats = nullptr;
    float* d_texels = nullptr;
    double* d_zig = nullptr;
    uint32_t* d_occ = nullptr;
    uint32_t occ_shift = 0, occ_nb[3] = {0, 0, 0}, occ_words = 0;
    uint32_t* d_occx = nullptr;     // exact per-cell occupancy blob (OccX), if it fits the LDS budget
    unsigned long long* d_bmask = nullptr;   // every 4^3 brick's cell mask, linear brick order (TraceParams::bmask)
    uint32_t* d_esc = nullptr;      // escape table (escape.h), with OccX
    uint32_t* d_sat = nullptr;      // summed-area table of cell occupancy (escape.h EscSat), or null
    // the primary frustum bounds (frustum_kernel) per 8x8 pixel block
    float4* d_tlo = nullptr; size_t tlo_cap = 0;
    bool esc_on = false;            // the park launches use it (dense enough to pay, context_escape)
    // park release (wf_park_kernel): the fraction of the occupied cells'
    // entry-face masks that are 0, and whether the launches use it
    double rel_frac = 0.0;
    bool rel_on = false;
    bool esc_tried = false;         // context_escape ran (at the first render that can use it)
    double esc_density = 0.0;       // fraction of its (brick, bin) bits set
    uint32_t occx_words = 0, occx_nbw = 0, occx_moff = 0, occx_nb[3] = {0, 0, 0};
    bool occx_ok = false;
    // an edge component of 2^62 or more, or infinite: every launch takes the
    // lane walk with the IEEE division in Moller-Trumbore (kWf*Exact), since
    // the park and packed kernels' short reciprocal holds for |det| < 2^126
    // only (zrt_math.h mt_inv_det)
    bool mt_exact = false;
    // grow-only work buffers
    uint32_t* d_pix = nullptr; size_t pix_cap = 0;
    float4* d_out = nullptr; size_t out_cap = 0;     // counting build
    // wavefront buffers of one pass set (queues, terminal radiance, bounce
    // planes, counters, hit records); set k > 0 runs on its own stream
    struct PassSet {
        hipStream_t stream = nullptr;      // set 0: the context stream
        float4* q0 = nullptr; size_t q0_cap = 0;
        float4* q1 = nullptr; size_t q1_cap = 0;
        float4* term = nullptr; size_t term_cap = 0;
        float4* stk4 = nullptr; size_t stk4_cap = 0;   // bounce planes: (e, a.x) per (slot, item)
        float2* stk2 = nullptr; size_t stk2_cap = 0;   //   (a.y, a.z) per (slot, item)
        uint32_t* wfc = nullptr; size_t wfc_cap = 0;
        float4* hit = nullptr; size_t hit_cap = 0;
        hipEvent_t ev_join = nullptr;      // set k > 0: its last pass is done
    };
    PassSet set[kMaxPassSets];
    float4* d_acc = nullptr; size_t acc_cap = 0;
    uint8_t* d_rgb = nullptr; size_t rgb_cap = 0;
    float* d_lin = nullptr; size_t lin_cap = 0;
    std::vector<hipEvent_t> ev_pass;   // per pass: its resolve done
    hipEvent_t ev_fork = nullptr;
    uint32_t* d_counter = nullptr;
    unsigned long long* d_stats = nullptr;
    int num_cus = 0;
    // ZRT_FLAG_KERNEL_TIMES: an event pair per kernel launch and its class
    std::vector<hipEvent_t> ev_k;
    std::vector<uint8_t> ev_k_cls;
    zrt_kernel_profile prof{};         // of the last render (zrt_context_profile)
    // cached pixel list
    std::vector<uint32_t> pix;
    uint32_t pix_key[5] = {0, 0, 0, 0, 0};
    bool pix_valid = false;
};

static int validate_materials(const zrt_scene* s);

// A copy on the context's stream, waited for: the product path never uses
// HIP's null stream, whose first use in a process creates its hardware
// queue (~10 ms of the CLI's start-up, r06d)
static hipError_t copy_sync(void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t st) {
    const hipError_t e = hipMemcpyAsync(dst, src, n, kind, st);
    return e != hipSuccess ? e : hipStreamSynchronize(st);
}

// ZRT_TIMING=1: context creation's stages on stderr ("timing:" lines), each
// closed by a stream sync (the start-up split of VERDICT r5 #6)
struct StageClock {
    bool on = getenv("ZRT_TIMING") != nullptr;
    double t = 0.0;
    static double now_ms() {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
    }
    StageClock() { t = now_ms(); }
    void mark(const zrt_context* c, const char* what);
};

void StageClock::mark(const zrt_context* c, const char* what) {
    if (!on) return;
    (void)hipStreamSynchronize(c->stream);
    const double n = now_ms();
    fprintf(stderr, "timing: context %s %.3f ms\n", what, n - t);
    t = n;
}

static int validate_scene(const zrt_scene* s) {
    if (!s) return ZRT_ERR_INVALID_ARG;
    const uint64_t nc = (uint64_t)s->grid.resolution[0] * s->grid.resolution[1] * s->grid.resolution[2];
    if (nc == 0 || nc != s->num_cells || nc > 0x7FFFFFFFull || !s->cells) return ZRT_ERR_INVALID_ARG;
    if (s->num_triangles && (!s->triangles_pos || !s->triangles_data || !s->triangles_material))
        return ZRT_ERR_INVALID_ARG;
    for (uint64_t c = 0; c < nc; ++c) {
        const uint32_t b = s->cells[2 * c], e = s->cells[2 * c + 1];
        if (b > e || e > s->num_triangles) return ZRT_ERR_INVALID_ARG;
    }
    for (uint32_t i = 0; i < s->num_triangles; ++i)
        if (s->triangles_material[i] >= s->num_materials) return ZRT_ERR_INVALID_ARG;
    return validate_materials(s);
}

// Whether a scene needs the IEEE-division kernels (zrt_context::mt_exact):
// `n` floats of which those with k % stride in [first, stride) are checked
// (baked refs: the e1, e2 components of v0 e1 e2; source triangles: every
// vertex component, at 2^61, so that their differences stay below 2^62).
// NaN components need nothing: both forms propagate them.
static bool needs_mt_exact(const float* v, uint64_t n, uint32_t stride, uint32_t first, float lim) {
    for (uint64_t k = 0; k < n; ++k)
        if (k % stride >= first && fabsf(v[k]) >= lim) return true;
    return false;
}

// Materials and texels only (textures inside the texel array).
static int validate_materials(const zrt_scene* s) {
    if (s->num_materials == 0 || !s->materials || !s->texels) return ZRT_ERR_INVALID_ARG;
    for (uint32_t m = 0; m < s->num_materials; ++m) {
        const zrt_texture* t[3] = {&s->materials[m].base_color, &s->materials[m].emissive,
                                   &s->materials[m].transparency};
        for (int k = 0; k < 3; ++k) {
            const uint64_t ch = k < 2 ? 3 : 1;
            if (t[k]->w <= 0 || t[k]->h <= 0) return ZRT_ERR_INVALID_ARG;
            if (t[k]->offset + (uint64_t)t[k]->w * t[k]->h * ch > s->num_texel_floats)
                return ZRT_ERR_INVALID_ARG;
            if (t[k]->offset > 0xFFFFFFFFull) return ZRT_ERR_UNSUPPORTED;
        }
    }
    return ZRT_OK;
}

int grid_build_warmup();   // grid_build.hip

extern "C" int zrt_device_count(int* count) {
    if (!count) return ZRT_ERR_INVALID_ARG;
    *count = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return ZRT_ERR_NO_DEVICE;
    *count = n;
    return ZRT_OK;
}

// The timed wf_kernel instantiations, as the substrings of their mangled
// names that tools/spill_check.py / tests/test_codegen.py look for in the
// gfx950 code object (primary launch, then bounce launches).  No HIP call.
extern "C" const char* zrt_timed_kernels(void) {
#define ZRT_STR2(x) #x
#define ZRT_STR(x) ZRT_STR2(x)
    // the default launch set: primary wf_kernel, then per bounce the
    // trace-only park kernel + the whole-wave shade kernel (or wf_kernel when
    // the scene's OccX does not fit the LDS)
    // (brick-major packed words, then field words: dda.h)
    // (the last bool of wf_kernel: MTX, the IEEE-division instantiations
    // of the scenes with edges of 2^62 or more, not timed)
    return "wf_kernelILi" ZRT_STR(ZRT_WF_MINW0) "ELb1ELb1ELb1ELb0EE,wf_kernelILi" ZRT_STR(ZRT_WF_MINW0)
           "ELb1ELb1ELb0ELb0EE,"
           "wf_park_kernelILb1ELb1E,wf_park_kernelILb0ELb1E,wf_park_kernelILb1ELb0E,wf_park_kernelILb0ELb0E,"
           "wf_shade_kernelILb1ELb0EE,wf_shade_kernelILb1ELb1EE,wf_kernelILi" ZRT_STR(ZRT_WF_MINW) "ELb0ELb1ELb1ELb0EE,wf_kernelILi" ZRT_STR(
               ZRT_WF_MINW) "ELb0ELb1ELb0ELb0EE";
#undef ZRT_STR
#undef ZRT_STR2
}

// Start-up work of the first GPU call, done ahead: the device's context and
// the library's code objects (one fat binary, loaded on first use: ~0.1-0.2 s
// on MI355X).  Lets a host overlap it with file loading.
extern "C" int zrt_device_warmup(int device) {
    // ZRT_TIMING: the split of the HIP start-up (runtime initialisation,
    // device context, the two code objects) on stderr
    const bool timing = getenv("ZRT_TIMING") != nullptr;
    const double t0 = StageClock::now_ms();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ZRT_ERR_NO_DEVICE;
    const double t1 = StageClock::now_ms();
    if (device < 0) device = 0;
    if (device >= n) return ZRT_ERR_NO_DEVICE;
    DeviceGuard g(device);
    HIP_TRY(hipFree(nullptr));
    const double t2 = StageClock::now_ms();
    hipFuncAttributes fa;
    HIP_TRY(hipFuncGetAttributes(&fa, (const void*)resolve_kernel));
    const double t3 = StageClock::now_ms();
    const int rc = grid_build_warmup();
    if (timing)
        fprintf(stderr, "timing: warm-up: runtime init (hipGetDeviceCount) %.3f ms, device context %.3f ms, "
                "render.hip code object %.3f ms, grid_build.hip code object %.3f ms\n",
                t1 - t0, t2 - t1, t3 - t2, StageClock::now_ms() - t3);
    return rc;
}

extern "C" void zrt_context_destroy(zrt_context* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    if (c->d_cell32) (void)hipFree(c->d_cell32);
    void* bufs[] = {c->d_cells, c->d_pos, c->d_data, c->d_mats, c->d_texels, c->d_zig, c->d_occ, c->d_occx, c->d_esc,
                    c->d_bmask, c->d_sat, c->d_tlo,
                    c->d_pix, c->d_out, c->d_acc, c->d_rgb, c->d_lin, c->d_counter, c->d_stats};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (zrt_context::PassSet& ps : c->set) {
        void* sb[] = {ps.q0, ps.q1, ps.term, ps.stk4, ps.stk2, ps.wfc, ps.hit};
        for (void* b : sb)
            if (b) (void)hipFree(b);
        if (ps.ev_join) (void)hipEventDestroy(ps.ev_join);
        if (ps.stream && ps.stream != c->stream) (void)hipStreamDestroy(ps.stream);
    }
    for (hipEvent_t e : c->ev_trace) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_pass) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_k) (void)hipEventDestroy(e);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_begin) (void)hipEventDestroy(c->ev_begin);
    if (c->ev_end) (void)hipEventDestroy(c->ev_end);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

namespace {

// OccX on the device, pass 1: one thread per 4^3 brick -> its 64-bit cell
// mask (bit (z&3)<<4 | (y&3)<<2 | (x&3) = cell non-empty) and the brick bit.
__global__ __launch_bounds__(kBlock) void occx_mask_kernel(const uint2* __restrict__ cells, uint32_t r0, uint32_t r1,
                                                           uint32_t r2, uint32_t nb0, uint32_t nb1, uint32_t nb,
                                                           unsigned long long* __restrict__ masks,
                                                           uint32_t* __restrict__ bits) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    unsigned long long m = 0ull;
    if (b < nb) {
        const uint32_t bx = b % nb0, by = (b / nb0) % nb1, bz = b / (nb0 * nb1);
        for (uint32_t k = 0; k < 64; ++k) {
            const uint32_t x = bx * 4 + (k & 3u), y = by * 4 + ((k >> 2) & 3u), z = bz * 4 + (k >> 4);
            if (x < r0 && y < r1 && z < r2) {
                const uint2 c = cells[((uint64_t)z * r1 + y) * r0 + x];
                if (c.x < c.y) m |= 1ull << k;
            }
        }
        masks[b] = m;
    }
    const uint64_t bal = __ballot(b < nb && m != 0ull);
    const uint32_t lane = threadIdx.x & 63u;
    if (b < nb && (lane == 0 || lane == 32)) bits[b >> 5] = (uint32_t)(bal >> lane);
}

// Pass 2 (one block): 1 + the u16 prefix of occupied bricks per 32-brick
// word, the zero mask, then the occupied masks compacted in brick order;
// out[0] = the number of occupied bricks.
__global__ __launch_bounds__(1024) void occx_pack_kernel(const uint32_t* __restrict__ bits, uint32_t nbw,
                                                         const unsigned long long* __restrict__ masks,
                                                         uint16_t* __restrict__ prefix,
                                                         unsigned long long* __restrict__ packed,
                                                         uint32_t* __restrict__ out) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (nbw + 1023u) / 1024u;
    const uint32_t w0 = threadIdx.x * per, w1 = min(w0 + per, nbw);
    uint32_t sum = 0;
    for (uint32_t wd = w0; wd < w1; ++wd) sum += (uint32_t)__popc(bits[wd]);
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {            // inclusive Hillis-Steele scan
        const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - sum;
    for (uint32_t wd = w0; wd < w1; ++wd) {
        prefix[wd] = (uint16_t)min(run + 1u, 0xFFFFu);
        for (uint32_t wb = bits[wd]; wb; wb &= wb - 1u)
            packed[1u + run++] = masks[32u * wd + (uint32_t)__builtin_ctz(wb)];
    }
    if (threadIdx.x == 0) packed[0] = 0ull;
    if (threadIdx.x == 1023) out[0] = run;
}

}  // namespace

static int context_base(zrt_context* c) {
    StageClock sc;
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    sc.mark(c, "stream");
    HIP_TRY(hipEventCreate(&c->ev_begin));
    HIP_TRY(hipEventCreate(&c->ev_end));
    sc.mark(c, "events");
    // one attribute, not hipGetDeviceProperties (which fills ~100 fields and
    // took ~10 ms of the CLI's start-up, r06c)
    HIP_TRY(hipDeviceGetAttribute(&c->num_cus, hipDeviceAttributeMultiprocessorCount, c->device));
    sc.mark(c, "CU count");
    return ZRT_OK;
}

static int context_materials(zrt_context* c, const zrt_scene* s);
static int context_occupancy(zrt_context* c, const uint32_t* host_cells);

// Word i of ref k's (v0, e1, e2) in the context's triangle layout.
__device__ __forceinline__ uint32_t tri_word(const float* pos, uint32_t k, uint32_t i) {
    return __float_as_uint(pos[(uint64_t)kTriFloats * k + i + i / 3]);
}
__device__ __forceinline__ bool same_tri(const float* pos, uint32_t a, uint32_t b) {
    for (uint32_t i = 0; i < 9; ++i)
        if (tri_word(pos, a, i) != tri_word(pos, b, i)) return false;
    return true;
}

// The packed walks' cell records: 8 u32 per cell at its packed-word index
// (x | y << o1 | z << o2; the padding of a non-power-of-two grid stays empty):
// begin, end, then for each entry face f = 2 * axis + (the ray steps toward
// -axis) the mask of the refs (bit k: ref begin + k) that a ray entering the
// cell across f must still test.
//
// A ray enters a cell only from the cell it has just left, across the face
// they share, and leaves a cell only after testing all of its refs
// (stage3.zig:164-182).  A ref whose (v0, e1, e2) bits equal those of a ref
// of that neighbour gives the same (hit, t, u, v) as the one already tested
// there: if that one was taken, nearest == t and `nearest > t` fails; if not,
// nearest has only shrunk since.  So skipping it changes no hit, no tie
// (ties resolve within the cell by ref order, and the kept refs keep their
// order and index) and no break test.  Refs of cells with more than 32 refs
// are all kept (mask all ones), and so are those of a face on the grid
// boundary (no ray steps in across it).  About half of all triangle tests on
// the contest stand-in repeat the previous cell's (triangles span ~5.6
// cells), a third on the Sponza-scale one.
__global__ __launch_bounds__(kBlock) void cell32_kernel(const uint2* __restrict__ cells, uint32_t r0, uint32_t r1,
                                                        uint32_t r2, uint32_t ncells, const PackK pk,
                                                        const float* __restrict__ pos, uint32_t* __restrict__ out) {
    for (uint32_t ci = blockIdx.x * kBlock + threadIdx.x; ci < ncells; ci += gridDim.x * kBlock) {
        const uint2 c = cells[ci];
        const uint32_t x = ci % r0, y = (ci / r0) % r1, z = ci / r0 / r1;
        uint32_t* rec = out + 8ull * pack_cellv(pk, x, y, z);
        rec[0] = c.x;
        rec[1] = c.y;
        const uint32_t n = c.y - c.x;
        const uint32_t all = n >= 32u ? ~0u : (1u << n) - 1u;
        for (uint32_t f = 0; f < 6; ++f) {
            const uint32_t axis = f >> 1, toward_neg = f & 1u;
            const uint32_t cc = axis == 0 ? x : (axis == 1 ? y : z), rr = axis == 0 ? r0 : (axis == 1 ? r1 : r2);
            // the cell left: one step back against the ray's direction
            const bool inside = toward_neg ? cc + 1u < rr : cc > 0u;
            uint32_t m = all;
            if (inside && n > 0u && n <= 32u) {
                const uint32_t step = axis == 0 ? 1u : (axis == 1 ? r0 : r0 * r1);
                const uint2 pc = cells[toward_neg ? ci + step : ci - step];
                for (uint32_t k = 0; k < n; ++k)
                    for (uint32_t q = pc.x; q < pc.y; ++q)
                        if (same_tri(pos, c.x + k, q)) {
                            m &= ~(1u << k);
                            break;
                        }
            }
            rec[2 + f] = m;
        }
    }
}

// Park release statistic (context_release): over the occupied cells of the
// packed records, how many (cell, entry face) masks are 0 -- out[0] masks
// of occupied cells, out[1] zero masks among them.
__global__ __launch_bounds__(kBlock) void release_stat_kernel(const uint32_t* __restrict__ rec, uint64_t n,
                                                              unsigned long long* __restrict__ out) {
    unsigned long long faces = 0, zero = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint32_t* r = rec + 8 * i;
        if (r[1] > r[0]) {
            faces += 6;
            for (int f = 0; f < 6; ++f) zero += r[2 + f] == 0u ? 1 : 0;
        }
    }
    faces = wave_sum(faces);
    zero = wave_sum(zero);
    if ((threadIdx.x & 63u) == 0) {
        atomicAdd(&out[0], faces);
        atomicAdd(&out[1], zero);
    }
}

// The packed walks' layout (DdaV) and their cell records (cell32_kernel;
// none beyond 16 GiB, or beyond 1 GiB and 16x the cells' own 8 B -- flat
// grids whose narrow axis pack_layout widened: such a grid walks unpacked).
constexpr uint64_t kCell32Max = 16ull << 30;
constexpr double kRelMinFrac = 0.25;   // park release from this fraction of empty entry-face masks
static int context_packed(zrt_context* c) {
    const uint32_t* r = c->grid.resolution;
    // brick-major words where the grid allows them and the primary's
    // occupancy bricks are 4^3 (it reads them by pc >> 6); else field words
    // (and the dense brick masks exist: trace_ray reads them by pc >> 6)
    c->packed = pack_layout(r, c->pk, ZRT_PACK_BM && c->occ_shift == 2u && c->d_bmask != nullptr);
    if (!c->packed) return ZRT_OK;
    const uint64_t n = 1ull << (c->pk.b0 + c->pk.b1 + c->pk.b2);
    if (32 * n > kCell32Max || (n > 16ull * c->ncells && 32 * n > (1ull << 30))) {
        c->packed = false;
        return ZRT_OK;
    }
    HIP_TRY(hipMalloc((void**)&c->d_cell32, 32 * n));
    if (!pack_is_linear(r, c->pk)) HIP_TRY(hipMemsetAsync(c->d_cell32, 0, 32 * n, c->stream));
    hipLaunchKernelGGL(cell32_kernel, dim3(std::min<uint32_t>((c->ncells + kBlock - 1) / kBlock, 16384)), dim3(kBlock),
                       0, c->stream, c->d_cells, r[0], r[1], r[2], c->ncells, c->pk, c->d_pos,
                       c->d_cell32);
    HIP_TRY(hipGetLastError());
    // the park release pays on scenes whose rays often park in a cell with
    // nothing left to test for their entry face: r06q/r06r, alternating
    // processes, images identical: Cornell box (65% of the occupied cells'
    // entry faces empty) +7%, contest stand-in (29%) +3%, Sponza-scale
    // stand-in (18%) -1.5% (profiles/r06/r06q_ab_park_release.log)
    {
        unsigned long long h[2] = {0, 0};
        unsigned long long* d = nullptr;
        HIP_TRY(hipMalloc((void**)&d, sizeof h));
        hipError_t e = hipMemsetAsync(d, 0, sizeof h, c->stream);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(release_stat_kernel, dim3(std::min<uint64_t>((n + kBlock - 1) / kBlock, 4096)),
                               dim3(kBlock), 0, c->stream, (const uint32_t*)c->d_cell32, n, d);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        (void)hipFree(d);
        HIP_TRY(e);
        c->rel_frac = h[0] ? (double)h[1] / (double)h[0] : 0.0;
        c->rel_on = c->rel_frac >= kRelMinFrac;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ZRT_OK;
}

static int context_counters(zrt_context* c) {
    StageClock sc;
    int rc = context_packed(c);
    if (rc != ZRT_OK) return rc;
    sc.mark(c, "cell records (cell32_kernel)");
    HIP_TRY(hipMalloc((void**)&c->d_counter, 64));
    HIP_TRY(hipMalloc((void**)&c->d_stats, 512));
    return ZRT_OK;
}

static int context_init(zrt_context* c, const zrt_scene* s) {
    int rc = context_base(c);
    if (rc != ZRT_OK) return rc;
    c->grid = s->grid;
    c->ncells = s->num_cells;
    c->nrefs = s->num_triangles;
    c->nmat = s->num_materials;
    c->mt_exact = needs_mt_exact(s->triangles_pos, 9ull * s->num_triangles, 9u, 3u, 0x1p62f);
    HIP_TRY(hipMalloc((void**)&c->d_cells, 8ull * c->ncells));
    HIP_TRY(copy_sync(c->d_cells, s->cells, 8ull * c->ncells, hipMemcpyHostToDevice, c->stream));
    const size_t nr = std::max<size_t>(c->nrefs, 1);
    std::vector<float> pos(kTriFloats * nr, 0.0f);
    std::vector<float4> dat(4 * nr);
    for (uint32_t i = 0; i < c->nrefs; ++i) {
        const float* q = s->triangles_pos + 9ull * i;
        float* o = pos.data() + (size_t)kTriFloats * i;
        memcpy(o, q, 12); memcpy(o + 4, q + 3, 12); memcpy(o + 8, q + 6, 12);
        float tmp[16];
        memcpy(tmp, s->triangles_data + 15ull * i, 15 * sizeof(float));
        memcpy(&tmp[15], &s->triangles_material[i], 4);
        memcpy(&dat[4 * i], tmp, 64);
    }
    HIP_TRY(hipMalloc((void**)&c->d_pos, pos.size() * sizeof(float)));
    HIP_TRY(copy_sync(c->d_pos, pos.data(), pos.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMalloc((void**)&c->d_data, dat.size() * sizeof(float4)));
    HIP_TRY(copy_sync(c->d_data, dat.data(), dat.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    if ((rc = context_materials(c, s)) != ZRT_OK) return rc;
    return context_occupancy(c, s->cells);
}

// Materials, texels, ziggurat tables (stage3.zig:125-129, Zig std ziggurat).
static int context_materials(zrt_context* c, const zrt_scene* s) {
    c->nmat = s->num_materials;
    std::vector<DevMat> mats(c->nmat);
    for (uint32_t m = 0; m < c->nmat; ++m) {
        const zrt_texture* t[3] = {&s->materials[m].base_color, &s->materials[m].emissive,
                                   &s->materials[m].transparency};
        for (int k = 0; k < 3; ++k) {
            DevTex& d = mats[m].tex[k];
            d.off = (uint32_t)t[k]->offset;
            d.w = t[k]->w; d.h = t[k]->h;
            d.umin = t[k]->u_min; d.umax = t[k]->u_max;
            d.vmin = t[k]->v_min; d.vmax = t[k]->v_max;
            d.pad = 0;
            dev_tex_inline(d, s->texels, k < 2 ? 3 : 1);
        }
    }
    StageClock sc;
    HIP_TRY(hipMalloc((void**)&c->d_mats, mats.size() * sizeof(DevMat)));
    HIP_TRY(copy_sync(c->d_mats, mats.data(), mats.size() * sizeof(DevMat), hipMemcpyHostToDevice, c->stream));
    sc.mark(c, "materials");
    HIP_TRY(hipMalloc((void**)&c->d_texels, s->num_texel_floats * sizeof(float)));
    HIP_TRY(copy_sync(c->d_texels, s->texels, s->num_texel_floats * sizeof(float), hipMemcpyHostToDevice, c->stream));
    sc.mark(c, "texels");
    double zig[514];
    zig_tables(zig, zig + 257);
    sc.mark(c, "ziggurat tables (host)");
    HIP_TRY(hipMalloc((void**)&c->d_zig, sizeof zig));
    HIP_TRY(copy_sync(c->d_zig, zig, sizeof zig, hipMemcpyHostToDevice, c->stream));
    sc.mark(c, "ziggurat upload");
    return ZRT_OK;
}

// OccX blob layout for nb bricks (nbw 32-brick words) and `occupied` masks:
// bits | u16 (1 + prefix) per word | (8-byte aligned) the zero mask + masks.
static void occx_layout(uint64_t nbw, uint64_t occupied, uint64_t* moff, uint64_t* words) {
    const uint64_t pw = (nbw + 1) / 2;                   // prefix words
    *moff = (nbw + pw + 1) & ~1ull;
    *words = *moff + 2 * (occupied + 1);
}
// u32 words of the LDS copy: 8-byte (bits, prefix) entries, then the masks
static uint64_t occx_lds_words(uint64_t nbw, uint64_t moff, uint64_t words) {
    return (2 * nbw + (words - moff) + 3) & ~3ull;
}

// Brick occupancy and OccX, from the host cells or (host_cells null) from
// c->d_cells on the device; then the work counters.
//  * OccX (the park kernel) is built on 4^3-cell bricks and used when it fits
//    the LDS budget.
//  * wf_kernel's brick bits sit in LDS beside 7 waves' worth of workgroups:
//    4^3-cell bricks (4 KB of bits for a 128^3 grid, round 1's best) while
//    the bits take at most kOccLdsMax bytes, coarser bricks (8^3, 16^3, ...:
//    OR of the 4^3 ones) for larger grids -- result-invariant, an empty brick
//    only lets the walk skip the range loads of its cells.
#ifndef ZRT_OCC_LDS_KB
#define ZRT_OCC_LDS_KB 16
#endif
#ifndef ZRT_OCC_SH0
#define ZRT_OCC_SH0 2
#endif
constexpr uint64_t kOccLdsMax = (uint64_t)ZRT_OCC_LDS_KB << 10;

__global__ __launch_bounds__(kBlock) void occ_coarsen_kernel(const uint32_t* __restrict__ bits4, uint32_t nb0,
                                                             uint32_t nb1, uint32_t nb, uint32_t dsh, uint32_t cn0,
                                                             uint32_t cn01, uint32_t* __restrict__ out) {
    const uint32_t b = blockIdx.x * kBlock + threadIdx.x;
    if (b >= nb || !((bits4[b >> 5] >> (b & 31u)) & 1u)) return;
    const uint32_t bx = b % nb0, by = (b / nb0) % nb1, bz = b / (nb0 * nb1);
    const uint32_t cb = (bz >> dsh) * cn01 + (by >> dsh) * cn0 + (bx >> dsh);
    atomicOr(&out[cb >> 5], 1u << (cb & 31u));
}

// Coarse brick bits straight from the cells (device-built grids whose 4^3
// bricks are too many for OccX): one thread per cell, atomicOr per non-empty one.
__global__ __launch_bounds__(kBlock) void occ_cells_kernel(const uint2* __restrict__ cells, uint32_t r0, uint32_t r1,
                                                           uint32_t ncells, uint32_t sh, uint32_t cn0, uint32_t cn01,
                                                           uint32_t* __restrict__ out) {
    for (uint32_t ci = blockIdx.x * kBlock + threadIdx.x; ci < ncells; ci += gridDim.x * kBlock) {
        const uint2 c = cells[ci];
        if (c.x >= c.y) continue;
        const uint32_t x = ci % r0, y = (ci / r0) % r1, z = ci / r0 / r1;
        const uint32_t cb = (z >> sh) * cn01 + (y >> sh) * cn0 + (x >> sh);
        atomicOr(&out[cb >> 5], 1u << (cb & 31u));
    }
}

// Escape table (escape.h): a summed-area table of cell occupancy, then one
// thread per (4^3 brick, direction bin).
__global__ __launch_bounds__(kBlock) void esc_sat_fill_kernel(const uint2* __restrict__ cells, uint32_t r0, uint32_t r1,
                                                              uint32_t ncells, uint32_t n0, uint32_t n01,
                                                              uint32_t* __restrict__ sat) {
    for (uint32_t ci = blockIdx.x * kBlock + threadIdx.x; ci < ncells; ci += gridDim.x * kBlock) {
        const uint2 c = cells[ci];
        const uint32_t x = ci % r0, y = (ci / r0) % r1, z = ci / r0 / r1;
        sat[(uint64_t)(z + 1) * n01 + (uint64_t)(y + 1) * n0 + x + 1] = c.x < c.y ? 1u : 0u;
    }
}
// prefix sums along one axis of the (n0 x n1 x n2) volume: one thread per line
__global__ __launch_bounds__(kBlock) void esc_sat_scan_kernel(uint32_t* __restrict__ sat, uint32_t n0, uint32_t n1,
                                                              uint32_t n2, uint32_t axis) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    const uint64_t n01 = (uint64_t)n0 * n1;
    uint64_t base, stride;
    uint32_t len;
    if (axis == 0) {
        if (t >= n1 * n2) return;
        base = (uint64_t)(t / n1) * n01 + (uint64_t)(t % n1) * n0; stride = 1; len = n0;
    } else if (axis == 1) {
        if (t >= n0 * n2) return;
        base = (uint64_t)(t / n0) * n01 + t % n0; stride = n0; len = n1;
    } else {
        if (t >= n0 * n1) return;
        base = t; stride = n01; len = n2;
    }
    uint32_t acc = 0;
    for (uint32_t i = 0; i < len; ++i) {
        acc += sat[base + i * stride];
        sat[base + i * stride] = acc;
    }
}
__global__ __launch_bounds__(kBlock) void esc_build_kernel(const uint32_t* __restrict__ sat, uint32_t r0, uint32_t r1,
                                                           uint32_t r2, float cs0, float cs1, float cs2, uint32_t nb0,
                                                           uint32_t nb1, uint32_t nbr, uint32_t* __restrict__ esc) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (uint64_t)nbr * kEscNBin) return;
    const uint32_t br = (uint32_t)(t / kEscNBin), bin = (uint32_t)(t % kEscNBin);
    const uint32_t res[3] = {r0, r1, r2};
    const float cs[3] = {cs0, cs1, cs2};
    const EscSat S{sat, r0 + 1u, (r0 + 1u) * (r1 + 1u)};
    if (esc_compute(S, res, cs, br % nb0, (br / nb0) % nb1, br / (nb0 * nb1), bin))
        atomicOr(&esc[(uint64_t)br * kEscWords + (bin >> 5)], 1u << (bin & 31u));
}

// Least fraction of set escape bits for the park launches to use the table.
constexpr double kEscMinDensity = 0.12;
// The escape table for a context with OccX (the park walk); none for grids
// whose summed-area table would pass 2^28 entries (the walk then never stops
// early, as before).
// Primary frustum bounds (escape.h frustum_bound): one thread per 8x8 pixel
// block of the w x h image.
struct FrustumArgs {
    uint32_t res[3];
    float bmin[3], bmax[3], cs[3], org[3], llc[3], right[3], up[3];
    uint32_t w, h, nbx, nby;
    // this rank's tiles (capi.cpp tile_pixels: tile t of the tx-wide row-major
    // grid belongs to rank t % nranks): tile edge in blocks, tiles per row,
    // the rank and the rank count; the kernel bounds only their blocks.
    // whole: one wave per block of the image, those of other ranks' tiles
    // leaving at once (tiles larger than the image: fewer waves that way)
    uint32_t tb, tx, rank, nranks, whole;
};
__global__ __launch_bounds__(kBlock) void frustum_kernel(const uint32_t* __restrict__ sat, const FrustumArgs a,
                                                         float4* __restrict__ tlo) {
    const EscSat S{sat, a.res[0] + 1u, (a.res[0] + 1u) * (a.res[1] + 1u)};
    // one wave per block: lane l tests slices l, l + 64, ... of the same
    // march (frustum_cone / frustum_slice), the wave takes the first and
    // last occupied ones (a 1080p frame: 32 K waves of ~4 slices per lane
    // instead of 32 K threads of ~200 dependent slices, 0.42 ms, r04eb2)
    const uint32_t lane = threadIdx.x & 63u;
    // wave i: block i % tb^2 (row-major in the tile) of this rank's tile i / tb^2
    const uint32_t i = (blockIdx.x * kBlock + threadIdx.x) >> 6, bpt = a.tb * a.tb;
    uint32_t bx, by;
    if (a.whole) {                                         // (uniform over the wave)
        if (i >= a.nbx * a.nby) return;
        bx = i % a.nbx;
        by = i / a.nbx;
        if (((by / a.tb) * a.tx + bx / a.tb) % a.nranks != a.rank) return;
    } else {
        const uint32_t t = a.rank + (i / bpt) * a.nranks, k = i % bpt;
        bx = (t % a.tx) * a.tb + k % a.tb;
        by = (t / a.tx) * a.tb + k / a.tb;
        if (bx >= a.nbx || by >= a.nby) return;
    }
    const uint32_t b = by * a.nbx + bx;
    const FrustumCone q = frustum_cone(a.bmin, a.bmax, a.cs, a.org, a.llc, a.right, a.up, kFrustB * bx,
                                       kFrustB * bx + kFrustB, kFrustB * by, kFrustB * by + kFrustB);
    int first = 1 << 30, last = -1;
    if (q.ok)
        for (int it = (int)lane; it < (1 << 16) && !(it * q.ds > q.s_far); it += 64)
            if (frustum_slice(S, q, a.res, a.bmin, a.cs, a.org, it)) {
                first = min(first, it);
                last = max(last, it);
            }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        first = min(first, __shfl_xor(first, off));
        last = max(last, __shfl_xor(last, off));
    }
    if (lane == 0) {
        FrustumBound fb{0.0f, kInf, kInf, kInf};
        if (q.ok) frustum_finish(q, first == (1 << 30) ? -1 : first, last, fb);
        tlo[b] = make_float4(fb.lo, fb.hi, kInf, kInf);
    }
}

// The summed-area table of cell occupancy (escape.h EscSat): kept in the
// context for the escape table and the primary frustum bounds; none for grids
// whose table would pass 2^28 entries (1 GiB).
static int context_sat(zrt_context* c) {
    const uint32_t* r = c->grid.resolution;
    const uint64_t n0 = r[0] + 1ull, n1 = r[1] + 1ull, n2 = r[2] + 1ull;
    if (n0 * n1 * n2 > (1ull << 28)) return ZRT_OK;
    HIP_TRY(hipMalloc((void**)&c->d_sat, 4ull * n0 * n1 * n2));
    HIP_TRY(hipMemsetAsync(c->d_sat, 0, 4ull * n0 * n1 * n2, c->stream));
    hipLaunchKernelGGL(esc_sat_fill_kernel, dim3(4096), dim3(kBlock), 0, c->stream, c->d_cells, r[0], r[1], c->ncells,
                       (uint32_t)n0, (uint32_t)(n0 * n1), c->d_sat);
    const uint64_t lines[3] = {n1 * n2, n0 * n2, n0 * n1};
    for (uint32_t a = 0; a < 3; ++a)
        hipLaunchKernelGGL(esc_sat_scan_kernel, dim3((uint32_t)((lines[a] + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           c->stream, c->d_sat, (uint32_t)n0, (uint32_t)n1, (uint32_t)n2, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    return ZRT_OK;
}

static int context_escape(zrt_context* c) {
    if (!ZRT_ESCAPE || !c->occx_ok || !c->d_sat) return ZRT_OK;
    const uint32_t* r = c->grid.resolution;
    const uint64_t nbr = (uint64_t)c->occx_nb[0] * c->occx_nb[1] * c->occx_nb[2];
    HIP_TRY(hipMalloc((void**)&c->d_esc, 4ull * kEscWords * nbr));
    HIP_TRY(hipMemsetAsync(c->d_esc, 0, 4ull * kEscWords * nbr, c->stream));
    const uint64_t nthr = nbr * kEscNBin;
    hipLaunchKernelGGL(esc_build_kernel, dim3((uint32_t)((nthr + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                       (const uint32_t*)c->d_sat, r[0], r[1], r[2], c->grid.cell_size[0], c->grid.cell_size[1],
                       c->grid.cell_size[2], c->occx_nb[0], c->occx_nb[1], (uint32_t)nbr, c->d_esc);
    HIP_TRY(hipGetLastError());
    // Use it when enough of its bits are set: each walk trip of the park
    // kernel then issues a table query per brick entered (~4% of a launch on
    // scenes whose rays never escape, r04g), and the check itself costs ~1.5%.
    // Measured (r04): contest stand-in 23% of the bits set, +8% frame rate;
    // Cornell box 6%, -1.5%; Sponza-scale 1.6%, -4%.
    std::vector<uint32_t> h(kEscWords * nbr);
    HIP_TRY(hipMemcpyAsync(h.data(), c->d_esc, 4ull * kEscWords * nbr, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    uint64_t set = 0;
    for (uint32_t x : h) set += (uint64_t)__builtin_popcount(x);
    c->esc_density = (double)set / ((double)nbr * kEscNBin);
    c->esc_on = c->esc_density >= kEscMinDensity;
    return ZRT_OK;
}

static int context_occupancy(zrt_context* c, const uint32_t* host_cells) {
    StageClock sc_occ;
    const uint32_t* r = c->grid.resolution;
    for (int i = 0; i < 3; ++i) c->occx_nb[i] = (r[i] + 3u) >> 2;
    const uint64_t nb = (uint64_t)c->occx_nb[0] * c->occx_nb[1] * c->occx_nb[2];
    // more than 2^24 4^3 bricks (> 2^30 cells): no OccX (24-bit brick
    // indices), the bounces take the lane walk over the coarse bits below
    const bool occx_possible = occx_usable(nb, 0, 0, 1);
    const uint64_t nbw = (nb + 31) / 32;
    uint32_t sh = ZRT_OCC_SH0;
    auto words_at = [&](uint32_t k) {
        const uint64_t n = (uint64_t)((r[0] + (1u << k) - 1) >> k) * ((r[1] + (1u << k) - 1) >> k) *
                           ((r[2] + (1u << k) - 1) >> k);
        return (n + 31) / 32;
    };
    while (words_at(sh) * 4 > kOccLdsMax) ++sh;
    c->occ_shift = sh;
    for (int i = 0; i < 3; ++i) c->occ_nb[i] = (r[i] + (1u << sh) - 1) >> sh;
    c->occ_words = (uint32_t)words_at(sh);
    HIP_TRY(hipMalloc((void**)&c->d_occ, 4ull * c->occ_words));
    if (host_cells) {
        std::vector<unsigned long long> mask(occx_possible ? nb : 0, 0ull);
        std::vector<uint32_t> coarse(c->occ_words, 0u);
        for (uint32_t z = 0; z < r[2]; ++z)
            for (uint32_t y = 0; y < r[1]; ++y)
                for (uint32_t x = 0; x < r[0]; ++x) {
                    const uint64_t ci = ((uint64_t)z * r[1] + y) * r[0] + x;
                    if (host_cells[2 * ci] < host_cells[2 * ci + 1]) {
                        const uint64_t b = ((uint64_t)(z >> 2) * c->occx_nb[1] + (y >> 2)) * c->occx_nb[0] + (x >> 2);
                        if (occx_possible) mask[b] |= 1ull << (((z & 3u) << 4) | ((y & 3u) << 2) | (x & 3u));
                        const uint64_t cb = ((uint64_t)(z >> sh) * c->occ_nb[1] + (y >> sh)) * c->occ_nb[0] + (x >> sh);
                        coarse[cb >> 5] |= 1u << (cb & 31);
                    }
                }
        HIP_TRY(copy_sync(c->d_occ, coarse.data(), 4ull * c->occ_words, hipMemcpyHostToDevice, c->stream));
        if (!occx_possible) {
            c->occx_ok = false;
            const int rc = context_sat(c);
            if (rc != ZRT_OK) return rc;
            return context_counters(c);
        }
        HIP_TRY(hipMalloc((void**)&c->d_bmask, nb * 8));
        HIP_TRY(copy_sync(c->d_bmask, mask.data(), nb * 8, hipMemcpyHostToDevice, c->stream));
        std::vector<uint32_t> bits(nbw, 0u);
        std::vector<uint16_t> prefix(nbw, 0);
        std::vector<unsigned long long> masks;
        uint64_t run = 0;
        for (uint64_t wd = 0; wd < nbw; ++wd) {
            prefix[wd] = (uint16_t)std::min<uint64_t>(run + 1, 0xFFFF);
            for (uint64_t b = wd * 32; b < std::min<uint64_t>(nb, wd * 32 + 32); ++b)
                if (mask[b]) { bits[wd] |= 1u << (b & 31); masks.push_back(mask[b]); ++run; }
        }
        masks.insert(masks.begin(), 0ull);
        uint64_t moff, words;
        occx_layout(nbw, run, &moff, &words);
        c->occx_ok = occx_usable(nb, run, occx_lds_words(nbw, moff, words) * 4, kOccxBudget);
        if (c->occx_ok) {
            std::vector<uint32_t> blob(words, 0u);
            memcpy(blob.data(), bits.data(), nbw * 4);
            memcpy(blob.data() + nbw, prefix.data(), nbw * 2);
            memcpy(blob.data() + moff, masks.data(), masks.size() * 8);
            c->occx_words = (uint32_t)words;
            c->occx_nbw = (uint32_t)nbw;
            c->occx_moff = (uint32_t)moff;
            HIP_TRY(hipMalloc((void**)&c->d_occx, words * 4));
            HIP_TRY(copy_sync(c->d_occx, blob.data(), words * 4, hipMemcpyHostToDevice, c->stream));
        }
    } else if (!occx_possible) {
        HIP_TRY(hipMemsetAsync(c->d_occ, 0, 4ull * c->occ_words, c->stream));
        hipLaunchKernelGGL(occ_cells_kernel, dim3(4096), dim3(kBlock), 0, c->stream, c->d_cells, r[0], r[1], c->ncells,
                           sh, c->occ_nb[0], c->occ_nb[0] * c->occ_nb[1], c->d_occ);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(c->stream));
        c->occx_ok = false;
    } else {
        // the blob for the largest possible occupancy, then the real size
        uint64_t moff, words;
        occx_layout(nbw, nb, &moff, &words);
        // the scratch buffers are freed on every exit path (the blob belongs
        // to the context as soon as it exists)
        struct Scratch {
            uint32_t* n = nullptr;
            ~Scratch() {
                if (n) (void)hipFree(n);
            }
        } tmp;
        uint32_t* d_blob = nullptr;
        HIP_TRY(hipMalloc((void**)&c->d_bmask, nb * 8));   // the dense masks stay (TraceParams::bmask)
        HIP_TRY(hipMalloc((void**)&tmp.n, 4));
        HIP_TRY(hipMalloc((void**)&d_blob, words * 4));
        c->d_occx = d_blob;            // freed with the context from here on
        unsigned long long* const d_masks = c->d_bmask;
        uint32_t* const d_n = tmp.n;
        HIP_TRY(hipMemsetAsync(d_blob, 0, words * 4, c->stream));
        hipLaunchKernelGGL(occx_mask_kernel, dim3((uint32_t)((nb + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                           c->d_cells, r[0], r[1], r[2], c->occx_nb[0], c->occx_nb[1], (uint32_t)nb, d_masks, d_blob);
        hipLaunchKernelGGL(occx_pack_kernel, dim3(1), dim3(1024), 0, c->stream, (const uint32_t*)d_blob,
                           (uint32_t)nbw, (const unsigned long long*)d_masks,
                           reinterpret_cast<uint16_t*>(d_blob + nbw),
                           reinterpret_cast<unsigned long long*>(d_blob + moff), d_n);
        hipError_t le = hipGetLastError();
        if (sh == 2) {
            HIP_TRY(hipMemcpyAsync(c->d_occ, d_blob, nbw * 4, hipMemcpyDeviceToDevice, c->stream));
        } else if (sh < 2) {                   // (ZRT_OCC_SH0 builds) bricks finer than OccX's
            HIP_TRY(hipMemsetAsync(c->d_occ, 0, 4ull * c->occ_words, c->stream));
            hipLaunchKernelGGL(occ_cells_kernel, dim3(4096), dim3(kBlock), 0, c->stream, c->d_cells, r[0], r[1],
                               c->ncells, sh, c->occ_nb[0], c->occ_nb[0] * c->occ_nb[1], c->d_occ);
            if (le == hipSuccess) le = hipGetLastError();
        } else {
            HIP_TRY(hipMemsetAsync(c->d_occ, 0, 4ull * c->occ_words, c->stream));
            hipLaunchKernelGGL(occ_coarsen_kernel, dim3((uint32_t)((nb + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                               c->stream, (const uint32_t*)d_blob, c->occx_nb[0], c->occx_nb[1], (uint32_t)nb, sh - 2u,
                               c->occ_nb[0], c->occ_nb[0] * c->occ_nb[1], c->d_occ);
            if (le == hipSuccess) le = hipGetLastError();
        }
        uint32_t run = 0;
        HIP_TRY(hipMemcpyAsync(&run, d_n, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(le);
        occx_layout(nbw, run, &moff, &words);
        c->occx_ok = occx_usable(nb, run, occx_lds_words(nbw, moff, words) * 4, kOccxBudget);
        c->occx_words = (uint32_t)words;
        c->occx_nbw = (uint32_t)nbw;
        c->occx_moff = (uint32_t)moff;
    }
    // (the escape table itself is built by the first render whose frame is
    // large enough to pay for it: context_escape)
    sc_occ.mark(c, "occupancy bits + OccX");
    const int rc = context_sat(c);
    sc_occ.mark(c, "summed-area table");
    if (rc != ZRT_OK) return rc;
    return context_counters(c);
}

extern "C" int zrt_context_create(const zrt_scene* s, int device, zrt_context** out) {
    if (!out) return ZRT_ERR_INVALID_ARG;
    *out = nullptr;
    int rc = validate_scene(s);
    if (rc != ZRT_OK) return rc;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ZRT_ERR_NO_DEVICE;
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) return ZRT_ERR_NO_DEVICE;
    }
    if (device >= n) return ZRT_ERR_NO_DEVICE;
    DeviceGuard g(device);
    zrt_context* c = new (std::nothrow) zrt_context();
    if (!c) return ZRT_ERR_OUT_OF_MEMORY;
    c->device = device;
    rc = context_init(c, s);
    if (rc != ZRT_OK) { zrt_context_destroy(c); return rc; }
    *out = c;
    return ZRT_OK;
}

// Device-built context: Geometry.build + bakeInto (stage2.zig:44-164) on the
// GPU straight into the context's arrays (grid_build.hip), no host copy of the
// baked scene.  Same render results as zrt_geometry_build + zrt_context_create.
extern "C" int zrt_context_create_built(const float* positions, const float* normals, const float* texcoords,
                                        const uint32_t* material, uint32_t num_triangles,
                                        const uint32_t resolution[3], uint32_t num_materials,
                                        const zrt_material* materials, const float* texels,
                                        uint64_t num_texel_floats, int device, zrt_context** out) {
    if (!out) return ZRT_ERR_INVALID_ARG;
    *out = nullptr;
    if (!material) return ZRT_ERR_INVALID_ARG;
    zrt_scene ms{};
    ms.num_materials = num_materials;
    ms.materials = materials;
    ms.texels = texels;
    ms.num_texel_floats = num_texel_floats;
    int rc = validate_materials(&ms);
    if (rc != ZRT_OK) return rc;
    for (uint32_t i = 0; i < num_triangles; ++i)
        if (material[i] >= num_materials) return ZRT_ERR_INVALID_ARG;
    if (num_triangles && !positions) return ZRT_ERR_INVALID_ARG;
    // vertex components of 2^61 or more (or infinite) may give edge
    // components of 2^62 or more: the IEEE-division kernels (mt_exact)
    const bool mt_exact = needs_mt_exact(positions, 9ull * num_triangles, 1u, 0u, 0x1p61f);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ZRT_ERR_NO_DEVICE;
    if (device < 0) {
        if (hipGetDevice(&device) != hipSuccess) return ZRT_ERR_NO_DEVICE;
    }
    if (device >= n) return ZRT_ERR_NO_DEVICE;
    DeviceGuard g(device);
    zrt_context* c = new (std::nothrow) zrt_context();
    if (!c) return ZRT_ERR_OUT_OF_MEMORY;
    c->device = device;
    c->mt_exact = mt_exact;
    StageClock sc;
    rc = context_base(c);
    if (rc == ZRT_OK) {
        sc.mark(c, "stream + device properties");
        zrt::Grid grid;
        DeviceGeometry dg;
        rc = grid_build_into_device(positions, normals, texcoords, material, num_triangles, resolution, c->stream,
                                    &grid, &dg);
        if (rc == ZRT_OK) sc.mark(c, "grid build + bake (grid_build.hip)");
        if (rc == ZRT_OK) {
            for (int i = 0; i < 3; ++i) {
                c->grid.bbox_min[i] = (&grid.bbox.min.x)[i];
                c->grid.bbox_max[i] = (&grid.bbox.max.x)[i];
                c->grid.resolution[i] = grid.res[i];
                c->grid.cell_size[i] = (&grid.cell_size.x)[i];
            }
            c->ncells = resolution[0] * resolution[1] * resolution[2];
            c->nrefs = dg.refs;
            c->d_cells = dg.cells;
            c->d_data = dg.data;               // the context owns both from here (freed by destroy)
            c->d_pos = reinterpret_cast<float*>(dg.pos);   // the device bake's 3 float4 per ref
            if (rc == ZRT_OK && (rc = context_materials(c, &ms)) == ZRT_OK) {
                sc.mark(c, "materials + texels");
                rc = context_occupancy(c, nullptr);
            }
        }
    }
    if (rc != ZRT_OK) { zrt_context_destroy(c); return rc; }
    *out = c;
    return ZRT_OK;
}

// Empty cells and min/max refs of the non-empty ones (the CLI's grid log,
// main.zig:117-118 + stage2 logging), reduced on the device.
__global__ __launch_bounds__(kBlock) void grid_info_kernel(const uint2* __restrict__ cells, uint32_t ncells,
                                                           uint32_t* __restrict__ out) {
    uint32_t empty = 0, mn = 0xFFFFFFFFu, mx = 0;
    for (uint32_t ci = blockIdx.x * kBlock + threadIdx.x; ci < ncells; ci += gridDim.x * kBlock) {
        const uint2 c = cells[ci];
        const uint32_t k = c.y - c.x;
        if (!k) ++empty;
        else { mn = min(mn, k); mx = max(mx, k); }
    }
    for (int o = 32; o > 0; o >>= 1) {
        empty += __shfl_xor(empty, o);
        mn = min(mn, (uint32_t)__shfl_xor(mn, o));
        mx = max(mx, (uint32_t)__shfl_xor(mx, o));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], empty);
        atomicMin(&out[1], mn);
        atomicMax(&out[2], mx);
    }
}

extern "C" int zrt_context_grid_info(zrt_context* c, zrt_grid* grid, uint32_t info[4]) {
    if (!c || !info) return ZRT_ERR_INVALID_ARG;
    DeviceGuard g(c->device);
    if (grid) *grid = c->grid;
    uint32_t h[3] = {0u, 0xFFFFFFFFu, 0u};
    HIP_TRY(hipMemcpyAsync(c->d_counter, h, sizeof h, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(grid_info_kernel, dim3(std::min<uint32_t>((c->ncells + kBlock - 1) / kBlock, 2048)),
                       dim3(kBlock), 0, c->stream, c->d_cells, c->ncells, c->d_counter);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h, c->d_counter, sizeof h, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    info[0] = c->nrefs;
    info[1] = h[0];
    info[2] = h[1];
    info[3] = h[2];
    return ZRT_OK;
}

// Samples per pass: the caller's cfg->samples_per_pass, else as few passes
// as the queue budget allows but at least one per pass set (the sets' kernels
// overlap on their streams), split evenly: cfg3 256 spp = 2 x 128 (r02bq, two
// streams: 2 x 128 265.5 ms, 4 x 64 269.2, 8 x 32 273.1; cfg2 64 spp: 2 x 32
// 18.1 ms vs one pass 20.1).  The budget covers every set: 144 GiB (HBM is
// 288 GB), at most 60% of the free device memory.
// `held`: the bytes of pass buffers this context already holds (grow-only,
// reused by this render), counted as free: otherwise the split would depend
// on the renders before (a warm context saw less free memory and ran 3 passes
// on 2 sets, the last one alone).  The pass count is a multiple of the sets
// (when spp allows), so the streams stay balanced to the end of the frame.
static uint64_t pass_samples(const zrt_render_config* cfg, uint64_t per_item, uint32_t P, uint32_t sets,
                             size_t held, uint32_t share) {
    const uint64_t spp = cfg->num_samples;
    const uint64_t cap = std::max<uint64_t>(1, 0x7FFFFF00ull / P);     // items of a pass < 2^31
    if (cfg->samples_per_pass) return std::min<uint64_t>(std::min<uint64_t>(cfg->samples_per_pass, spp), cap);
    size_t budget = (size_t)144 << 30;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b)
        budget = std::min(budget, (free_b + held) / 10 * 6);
    budget /= std::max<uint32_t>(share, 1u);      // contexts of a group sharing this device
    const uint64_t fit = std::min<uint64_t>(cap, std::max<uint64_t>(1, budget / sets / (per_item * P)));
    uint64_t npass = std::max<uint64_t>(std::min<uint64_t>(sets, spp), (spp + fit - 1) / fit);
    npass = std::min<uint64_t>(spp, (npass + sets - 1) / sets * sets);
    const uint64_t s_pass = (spp + npass - 1) / npass;
    return s_pass;
}

extern "C" int zrt_context_render(zrt_context* c, const zrt_camera* cam, const zrt_render_config* cfg,
                                  const zrt_outputs* outs, zrt_stats* stats) {
    if (!c || !cam || !cfg) return ZRT_ERR_INVALID_ARG;
    if (cfg->num_samples == 0 || cfg->num_samples > 65535) return ZRT_ERR_INVALID_ARG;
    if (cam->w == 0 || cam->h == 0 || (uint64_t)cam->w * cam->h > 0xFFFFFFFFull) return ZRT_ERR_INVALID_ARG;
    const uint32_t nranks = cfg->num_ranks ? cfg->num_ranks : 1;
    if (cfg->rank >= nranks) return ZRT_ERR_INVALID_ARG;
    // the scatter mask holds one bit per bounce slot, the queue 16 bits of depth
    if (cfg->max_bounce > 32) return ZRT_ERR_UNSUPPORTED;
    const bool counting = (cfg->flags & ZRT_FLAG_COUNT_STATS) != 0;
    const TraceFn cfn = count_fn(cfg->max_bounce);
    if (counting && !cfn) return ZRT_ERR_UNSUPPORTED;
    DeviceGuard g(c->device);

    // packed pixel order of this rank (cached across calls)
    const uint32_t key[5] = {cam->w, cam->h, cfg->tile_size ? cfg->tile_size : 64, cfg->rank, nranks};
    if (!c->pix_valid || memcmp(key, c->pix_key, sizeof key) != 0) {
        uint32_t n = 0;
        int rc = tile_pixels(key[0], key[1], key[2], key[3], key[4], nullptr, &n);
        if (rc != ZRT_OK) return rc;
        c->pix.resize(std::max<uint32_t>(n, 1));
        tile_pixels(key[0], key[1], key[2], key[3], key[4], c->pix.data(), &n);
        c->pix.resize(n);
        int r2 = grow(&c->d_pix, &c->pix_cap, std::max<size_t>(n, 1));
        if (r2 != ZRT_OK) return r2;
        if (n) HIP_TRY(copy_sync(c->d_pix, c->pix.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
        memcpy(c->pix_key, key, sizeof key);
        c->pix_valid = true;
    }
    const uint32_t P = (uint32_t)c->pix.size();
    zrt_stats st{};
    if (P == 0) { if (stats) *stats = st; return ZRT_OK; }

    const uint32_t spp = cfg->num_samples;
    const uint32_t mb = cfg->max_bounce;
    const uint32_t nb = std::max<uint32_t>(mb, 1);
    // per-item bytes of a pass: counting megakernel = the float4 sample
    // radiance; wavefront = 2 queues x 48 B + terminal 16 B + the bounce
    // planes per slot ((a, has_e) 16 B + e 16 B with ZRT_PLANES16, else 24 B)
    // (+ the 16 B hit record the park kernel hands the shade kernel)
    const uint64_t per_item = counting ? 16ull : 96ull + 16ull + 16ull + (ZRT_PLANES16 ? 32ull : 24ull) * nb;
    // small frames run one set: a second stream costs its first launches
    // (the zrt CLI's 3-spp 1080p frame rendered in 30-39 vs 12.5-13.3 ms on a
    // fresh process) and does not pay back (cfg3 at 3 spp, warm: 7.1 vs 6.8
    // ms), while cfg2 (16.8 M samples) gains 10% (r02c4)
    const bool big = (uint64_t)P * cfg->num_samples >= kSetsMinSamples;
    uint32_t want_sets = big ? kPassSets : 1u;
#if defined(ZRT_SWEEP) || defined(ZRT_SETS_ENV)
    if (const char* e = getenv("ZRT_SETS")) want_sets = (uint32_t)std::max(1, std::min((int)kMaxPassSets, atoi(e)));
#endif
    const bool ktimes = (cfg->flags & ZRT_FLAG_KERNEL_TIMES) != 0;
    size_t held = 16ull * c->out_cap;
    for (const zrt_context::PassSet& ps : c->set)
        held += 16ull * (ps.q0_cap + ps.q1_cap + ps.term_cap + ps.stk4_cap + ps.hit_cap) + 8ull * ps.stk2_cap +
                4ull * ps.wfc_cap;
    const uint64_t s_pass = pass_samples(cfg, per_item, P, counting ? 1u : want_sets, held, c->mem_share);
    const uint32_t npasses = (uint32_t)((spp + s_pass - 1) / s_pass);
    // pass sets: pass p runs on set p % nsets, each set with its own stream
    // and buffers, so one pass's launches fill the machine while another's
    // drain (tails, the latency-bound shade kernel beside the park kernel):
    // two sets cfg3 -5%, cfg2 -9%, cfg5 -7% frame time, images identical
    // (r02c1, profiles/r02/r02c1_ab_two_streams.log)
    const uint32_t plan_sets = counting ? 1u : std::min<uint32_t>(npasses, want_sets);
    // ZRT_FLAG_ONE_SET: the same passes (split and lead as planned for the
    // sets) run one after another on the context's stream, so no kernel
    // overlaps another: exclusive kernel durations for bench.py's roofline,
    // the same per-launch work as the frame it stands for
    const uint32_t nsets = (cfg->flags & ZRT_FLAG_ONE_SET) ? 1u : plan_sets;
    // lead: samples moved from the last pass to the first.  The second set's
    // first primary launch waits for the first's (it fills every CU), so the
    // second set ends behind the first unless the first has more work.
    uint32_t lead_pct = plan_sets > 1 ? kLeadPct : 0u;
#if defined(ZRT_SWEEP) || defined(ZRT_SETS_ENV)
    if (const char* e = getenv("ZRT_LEAD")) lead_pct = plan_sets > 1 ? (uint32_t)std::max(0, std::min(50, atoi(e))) : 0u;
#endif
    const uint64_t last_n = spp - (uint64_t)(npasses - 1) * s_pass;     // samples of the last pass
    const uint64_t cap_items = std::max<uint64_t>(1, 0x7FFFFF00ull / P);
    const uint32_t lead = npasses > 1 ? (uint32_t)std::min<uint64_t>(
                                            {s_pass * lead_pct / 100, last_n - 1, cap_items - std::min(cap_items, s_pass)})
                                      : 0u;
    auto pass_first = [&](uint32_t pass) -> uint32_t { return pass == 0 ? 0u : (uint32_t)(pass * s_pass + lead); };
    auto pass_count = [&](uint32_t pass) -> uint32_t {
        return pass == 0 ? (uint32_t)std::min<uint64_t>(spp, s_pass + lead)
                         : (uint32_t)std::min<uint64_t>(s_pass, spp - pass_first(pass));
    };
    const uint64_t T = (s_pass + lead) * P;      // the first pass is the largest
    int rc;
    if (counting && (rc = grow(&c->d_out, &c->out_cap, (size_t)T)) != ZRT_OK) return rc;
    for (uint32_t k = 0; k < nsets && !counting; ++k) {
        zrt_context::PassSet& ps = c->set[k];
        if ((rc = grow(&ps.q0, &ps.q0_cap, 3 * T)) != ZRT_OK) return rc;
        if ((rc = grow(&ps.q1, &ps.q1_cap, 3 * T)) != ZRT_OK) return rc;
        if ((rc = grow(&ps.term, &ps.term_cap, T)) != ZRT_OK) return rc;
        if ((rc = grow(&ps.stk4, &ps.stk4_cap, T * nb)) != ZRT_OK) return rc;
        if ((rc = grow(&ps.stk2, &ps.stk2_cap, T * nb * (ZRT_PLANES16 ? 2 : 1))) != ZRT_OK) return rc;
        if ((rc = grow(&ps.wfc, &ps.wfc_cap, 32ull * kCtr * (mb + 2))) != ZRT_OK) return rc;
        if (k == 0) {
            ps.stream = c->stream;
        } else {
            if (!ps.stream) HIP_TRY(hipStreamCreateWithFlags(&ps.stream, hipStreamNonBlocking));
            if (!ps.ev_join) HIP_TRY(hipEventCreateWithFlags(&ps.ev_join, hipEventDisableTiming));
        }
    }
    if (nsets > 1) {
        if (!c->ev_fork) HIP_TRY(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
        while (c->ev_pass.size() < npasses) {
            hipEvent_t e;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->ev_pass.push_back(e);
        }
    }
    if (npasses > 1 && (rc = grow(&c->d_acc, &c->acc_cap, P)) != ZRT_OK) return rc;
    if ((rc = grow(&c->d_rgb, &c->rgb_cap, 3ull * P)) != ZRT_OK) return rc;
    const bool want_lin = outs && outs->linear_packed;
    if (want_lin && (rc = grow(&c->d_lin, &c->lin_cap, 3ull * P)) != ZRT_OK) return rc;
    const uint32_t launches_per_pass = counting ? 1 : nb;
    while (c->ev_trace.size() < 2ull * npasses * launches_per_pass) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        c->ev_trace.push_back(e);
    }

    // per-kernel events: per pass the primary, nb - 1 bounces of up to two
    // kernels, the resolve
    const size_t nk = ktimes ? (size_t)npasses * (2 * nb + 1) : 0;
    while (c->ev_k.size() < 2 * nk) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        c->ev_k.push_back(e);
    }
    c->ev_k_cls.assign(nk, 0);

    // Kernel per launch: the park kernel (traces, writes hit records) +
    // wf_shade_kernel for the bounce launches (incoherent rays) when the
    // scene's OccX fits the LDS budget, wf_kernel for the primary launch
    // (coherent 8x8-pixel waves: 22 vs 42 ms for the park kernel at cfg3 64
    // spp, r02d).  ZRT_FLAG_LANE_WALK: wf_kernel for every launch (round 1's
    // path, and the fallback).
    // (the park walk packs a cell into one word: at most 1024 cells per axis)
    // mtx: Moller-Trumbore with the IEEE division in every launch (scenes
    // whose edges leave the short reciprocal's domain, or as the flag forces):
    // the unpacked lane walk, kWf*Exact
    const bool mtx = c->mt_exact || (cfg->flags & ZRT_FLAG_MT_EXACT);
    const bool park_next = c->occx_ok && !counting && !(cfg->flags & ZRT_FLAG_LANE_WALK) &&
                           c->packed && !mtx;
    // the park release (wf_park_kernel): where enough entry faces are empty
    // (context_packed), or as the flags force it (same image either way);
    // with it the test rounds start at 12 parked lanes instead of 14 (r06u,
    // in one process, images identical: cfg3 7004 vs 6979, cfg2 4795 vs
    // 4632 Mrays/s; 10: 6987 / 4815, 8: 6927 / 4748;
    // profiles/r06/r06u_knobs_release_trigger.log)
    const bool rel = !(cfg->flags & ZRT_FLAG_NO_RELEASE) && (c->rel_on || (cfg->flags & ZRT_FLAG_RELEASE));
    uint32_t test_min = rel ? kParkTestMinRel : kParkTestMin, refill_min = kParkRefillMin;
#if defined(ZRT_SWEEP) || defined(ZRT_SETS_ENV)
    if (const char* e = getenv("ZRT_PARK_T")) test_min = (uint32_t)std::max(1, std::min(64, atoi(e)));
    if (const char* e = getenv("ZRT_PARK_R")) refill_min = (uint32_t)std::max(1, std::min(64, atoi(e)));
#endif
    uint32_t rel_min = test_min;           // park release: the parked lanes with refs a round needs
    uint32_t rel_emin = 1;                 //   and the empty ones that make skipping it worth it
#if defined(ZRT_SWEEP) || defined(ZRT_SETS_ENV)
    if (const char* e = getenv("ZRT_PARK_REL")) rel_min = (uint32_t)std::max(1, std::min(64, atoi(e)));
    if (const char* e = getenv("ZRT_PARK_REL_E")) rel_emin = (uint32_t)std::max(1, std::min(64, atoi(e)));
#endif
    const bool packed = c->packed && !mtx;
    const bool pbm = packed && c->pk.bm;   // brick-major packed words (dda.h)
    const WfFn f_first = mtx ? kWfPrimaryExact : packed ? (pbm ? kWfPrimaryBM : kWfPrimary) : kWfPrimaryWide;
    // the escape table: where dense enough to pay (context_escape), or as
    // the flags force it (both kernels give the same image)
    // (built at the first frame of 2^23 samples or more, or the first the flag
    // forces: 2.1 ms on cfg3 at 384 bins, r04eb2, more than the table saves a
    // 3-spp 1080p frame)
    if (!c->esc_tried && park_next && !(cfg->flags & ZRT_FLAG_NO_ESCAPE) && (big || (cfg->flags & ZRT_FLAG_ESCAPE))) {
        c->esc_tried = true;
        if ((rc = context_escape(c)) != ZRT_OK) return rc;
    }
    const bool esc = c->d_esc && !(cfg->flags & ZRT_FLAG_NO_ESCAPE) &&
                     (c->esc_on || (cfg->flags & ZRT_FLAG_ESCAPE));
    const WfFn f_next = park_next ? (pbm ? (esc ? (WfFn)wf_park_kernel<true, true> : (WfFn)wf_park_kernel<false, true>)
                                         : (esc ? (WfFn)wf_park_kernel<true, false> : (WfFn)wf_park_kernel<false, false>))
                                  : mtx ? kWfBounceExact : (packed ? (pbm ? kWfBounceBM : kWfBounce) : kWfBounceWide);
    const WfFn s_next = c->nmat <= kLdsMats ? (WfFn)wf_shade_kernel<true> : (WfFn)wf_shade_kernel<false>;
    // a pass's last bounce launch: the terminal-radiance-only shade (LAST)
    const WfFn s_last = !ZRT_SHADE_LAST ? s_next
                        : c->nmat <= kLdsMats ? (WfFn)wf_shade_kernel<true, true> : (WfFn)wf_shade_kernel<false, true>;
    const size_t lds_shade = c->nmat <= kLdsMats ? c->nmat * sizeof(DevMat) : 0;
    for (uint32_t k = 0; k < nsets && park_next; ++k)
        if ((rc = grow(&c->set[k].hit, &c->set[k].hit_cap, T)) != ZRT_OK) return rc;

    // Capacity guard: every buffer a launch below writes holds what that
    // launch writes (round 2's counting render once wrote through an
    // unallocated d_out after a refactor of the pass logic; a stale, smaller
    // buffer must not pass silently either).  Queues 3 float4 per item, bounce
    // planes a float4 + a float2 per (slot, item), terminal radiance / hit records / counting
    // output 1 per item, the pass's items S * P <= T (checked per pass).
    {
        auto shortfall = [&](const char* what, const void* ptr, size_t cap, uint64_t need) {
            if (ptr && cap >= need) return false;
            if (getenv("ZRT_DEBUG"))
                fprintf(stderr, "zrt: capacity guard: %s holds %zu, the launch writes %llu\n", what, ptr ? cap : 0,
                        (unsigned long long)need);
            return true;
        };
        bool bad = shortfall("pixel list", c->d_pix, c->pix_cap, P) || shortfall("rgb", c->d_rgb, c->rgb_cap, 3ull * P) ||
                   (npasses > 1 && shortfall("accumulator", c->d_acc, c->acc_cap, P)) ||
                   (want_lin && shortfall("linear", c->d_lin, c->lin_cap, 3ull * P)) ||
                   (counting && shortfall("counting output", c->d_out, c->out_cap, T));
        for (uint32_t k = 0; k < nsets && !counting && !bad; ++k) {
            const zrt_context::PassSet& ps = c->set[k];
            bad = shortfall("q0", ps.q0, ps.q0_cap, 3 * T) || shortfall("q1", ps.q1, ps.q1_cap, 3 * T) ||
                  shortfall("term", ps.term, ps.term_cap, T) || shortfall("planes4", ps.stk4, ps.stk4_cap, T * nb) ||
                  shortfall("planes2", ps.stk2, ps.stk2_cap, T * nb * (ZRT_PLANES16 ? 2 : 1)) ||
                  shortfall("counters", ps.wfc, ps.wfc_cap, 32ull * kCtr * (mb + 2)) ||
                  (park_next && shortfall("hit records", ps.hit, ps.hit_cap, T)) ||
                  (k > 0 && (!ps.stream || !ps.ev_join));
        }
        for (uint32_t pass = 0; pass < npasses && !bad; ++pass)
            bad = (uint64_t)pass_count(pass) * P > T || pass_first(pass) + pass_count(pass) > spp;
        if (bad) return ZRT_ERR_INVALID_ARG;
    }

    // occupancy-sized persistent grids
    const size_t lds_wf = 4ull * c->occ_words;
    int park_block = kParkBlock;
#ifdef ZRT_SWEEP
    if (const char* e = getenv("ZRT_PARK_BLOCK")) park_block = std::max(64, std::min(kParkBlock, atoi(e) / 64 * 64));
#endif
    const uint32_t occx_ldsw = (uint32_t)occx_lds_words(c->occx_nbw, c->occx_moff, c->occx_words);
    const size_t lds_park = 4ull * occx_ldsw + (size_t)(park_block / 64) * sizeof(ParkSlot);
    if (getenv("ZRT_WF_DEBUG"))
        fprintf(stderr, "{\"zrt_park_lds\": {\"occx_bytes\": %u, \"block\": %d, \"lds_per_block\": %zu, "
                "\"release_frac\": %.4f, \"release\": %d}}\n",
                4u * occx_ldsw, park_block, lds_park, c->rel_frac, rel ? 1 : 0);
    auto grid_for = [&](const void* f, int threads, size_t lds, uint32_t* blocks) -> int {
        int bpc = 0;
        HIP_TRY(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, f, threads, lds));
        if (getenv("ZRT_WF_DEBUG"))
            fprintf(stderr, "{\"zrt_grid\": {\"threads\": %d, \"lds\": %zu, \"blocks_per_cu\": %d}}\n", threads, lds, bpc);
        bpc = std::max(1, std::min(bpc, 2048 / threads));
        *blocks = (uint32_t)(c->num_cus * bpc);
        return ZRT_OK;
    };
    uint32_t grid_first = 0, grid_next = 0, grid_count = 0, grid_shade = 0, grid_shade_last = 0;
    const int thr_first = kTraceThreads;
    const int thr_next = park_next ? park_block : kTraceThreads;
    const size_t lds_first = lds_wf, lds_next = park_next ? lds_park : lds_wf;
    if (counting) {
        if ((rc = grid_for((const void*)cfn, kTraceThreads, lds_wf, &grid_count)) != ZRT_OK) return rc;
    } else {
        if ((rc = grid_for((const void*)f_first, thr_first, lds_first, &grid_first)) != ZRT_OK) return rc;
        if ((rc = grid_for((const void*)f_next, thr_next, lds_next, &grid_next)) != ZRT_OK) return rc;
        if ((rc = grid_for((const void*)s_next, kTraceThreads, lds_shade, &grid_shade)) != ZRT_OK) return rc;
        if ((rc = grid_for((const void*)s_last, kTraceThreads, lds_shade, &grid_shade_last)) != ZRT_OK) return rc;
    }

    TraceParams tp;
    memset(&tp, 0, sizeof tp);
    for (int i = 0; i < 3; ++i) {
        tp.bmin[i] = c->grid.bbox_min[i];
        tp.bmax[i] = c->grid.bbox_max[i];
        tp.res[i] = c->grid.resolution[i];
        tp.cs[i] = c->grid.cell_size[i];
        tp.ics[i] = 1.0f / c->grid.cell_size[i];          // IEEE: RN(1 / cs)
        tp.org[i] = cam->origin[i];
        tp.llc[i] = cam->lower_left_corner[i];
        tp.right[i] = cam->right[i];
        tp.up[i] = cam->up[i];
    }
    tp.cs_ok = 1u;
    for (int i = 0; i < 3; ++i)
        if (!(fabsf(tp.cs[i]) >= 0x1p-32f && fabsf(tp.cs[i]) <= 0x1p32f)) tp.cs_ok = 0u;
    tp.cells = c->d_cells;
    tp.pk = c->pk;
    tp.cell32 = c->d_cell32;
    {
        const uint32_t sh = c->occ_shift, b[3] = {c->pk.b0, c->pk.b1, c->pk.b2};
        tp.occ_w0 = b[0] > sh ? b[0] - sh : 0u;
        tp.occ_w1 = b[1] > sh ? b[1] - sh : 0u;
        tp.occ_w2 = b[2] > sh ? b[2] - sh : 0u;
        auto lowbits = [&](int a) { return (1u << std::min(sh, b[a])) - 1u; };
        tp.occ_o1 = c->pk.o1 + sh;
        tp.occ_o2 = c->pk.o2 + sh;
        // (brick-major words: occupancy bricks of 4^3, the word's low six bits)
        tp.occ_lowm = c->pk.bm ? 63u : lowbits(0) | (lowbits(1) << c->pk.o1) | (lowbits(2) << c->pk.o2);
        tp.ox1 = c->pk.o1 + 2u;
        tp.ox2 = c->pk.o2 + 2u;
        tp.ow0 = b[0] - 2u;
        tp.ow1 = b[1] - 2u;
        tp.ow2 = b[2] - 2u;
    }
    tp.tri_pos = c->d_pos;
    tp.tri_data = c->d_data;
    tp.mats = c->d_mats;
    tp.nmat = c->nmat;
    tp.texels = c->d_texels;
    tp.zig = c->d_zig;
    tp.occ = c->d_occ;
    tp.bmask = c->d_bmask;
    tp.occ_shift = c->occ_shift;
    tp.occ_nb0 = c->occ_nb[0];
    tp.occ_nb01 = c->occ_nb[0] * c->occ_nb[1];
    tp.occ_words = c->occ_words;
    tp.w = cam->w;
    tp.pixlist = c->d_pix;
    tp.P = P;
    tp.max_bounce = mb;
    tp.seed = cfg->seed;
    tp.out = c->d_out;
    tp.counter = c->d_counter;
    tp.stats = c->d_stats;
    // stage3.zig:223 inv_num_samples = ones / splat(spp)  (f32 division)
    const float inv_spp = 1.0f / (float)spp;
    size_t kn = 0;                             // kernels launched (ZRT_FLAG_KERNEL_TIMES)
    auto kt_begin = [&](int cls, hipStream_t sm) -> int {
        if (!ktimes) return ZRT_OK;
        c->ev_k_cls[kn] = (uint8_t)cls;
        HIP_TRY(hipEventRecord(c->ev_k[2 * kn], sm));
        return ZRT_OK;
    };
    auto kt_end = [&](hipStream_t sm) -> int {
        if (!ktimes) return ZRT_OK;
        HIP_TRY(hipEventRecord(c->ev_k[2 * kn + 1], sm));
        ++kn;
        return ZRT_OK;
    };
    zrt_kernel_profile kp{};

    HIP_TRY(hipMemsetAsync(c->d_stats, 0, 512, c->stream));
    HIP_TRY(hipEventRecord(c->ev_begin, c->stream));
    // the frustum bounds cost a 78-us launch per render (1080p, one wave per
    // block, r04fk3; 0.42 ms one thread per block) and save ~18% of the
    // primary launch: frames of 2^23 samples or more (a 3-spp 1080p frame's
    // primary takes ~0.5 ms: break-even)
    if (ZRT_FRUSTUM && c->d_sat && !counting && packed && !(cfg->flags & ZRT_FLAG_NO_FRUSTUM) &&
        ((uint64_t)P * cfg->num_samples >= kFrustumMinSamples || (cfg->flags & ZRT_FLAG_FRUSTUM))) {
        // the primary frustum bounds of this camera, every render (inside the
        // timed region: one wave per 4x4 pixel block, 130 K waves at 1080p)
        const uint32_t nbx = (cam->w + (1u << kFrustShift) - 1u) >> kFrustShift;
        const uint32_t nby = (cam->h + (1u << kFrustShift) - 1u) >> kFrustShift;
        if ((rc = grow(&c->d_tlo, &c->tlo_cap, (size_t)nbx * nby)) != ZRT_OK) return rc;
        FrustumArgs fa;
        for (int k = 0; k < 3; ++k) {
            fa.res[k] = c->grid.resolution[k];
            fa.bmin[k] = c->grid.bbox_min[k];
            fa.bmax[k] = c->grid.bbox_max[k];
            fa.cs[k] = c->grid.cell_size[k];
            fa.org[k] = cam->origin[k];
            fa.llc[k] = cam->lower_left_corner[k];
            fa.right[k] = cam->right[k];
            fa.up[k] = cam->up[k];
        }
        fa.w = cam->w; fa.h = cam->h; fa.nbx = nbx; fa.nby = nby;
        // only the blocks of this rank's tiles (a tile edge is a multiple of 8
        // pixels, so of a block edge): an 8-rank frame bounds 1/8 of them
        const uint32_t tile = cfg->tile_size ? cfg->tile_size : 64u;
        fa.tb = tile >> kFrustShift;
        fa.tx = (cam->w + tile - 1u) / tile;
        fa.rank = cfg->rank;
        fa.nranks = nranks;
        const uint64_t ntiles = (uint64_t)fa.tx * ((cam->h + tile - 1u) / tile);
        // (a rank with pixels owns tile `rank`, so ntiles > rank here)
        const uint64_t per_tile = (ntiles - cfg->rank + nranks - 1u) / nranks * fa.tb * fa.tb;
        fa.whole = per_tile > (uint64_t)nbx * nby ? 1u : 0u;
        const uint64_t fthreads = (fa.whole ? (uint64_t)nbx * nby : per_tile) * 64u;
        hipLaunchKernelGGL(frustum_kernel, dim3((uint32_t)((fthreads + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                           (const uint32_t*)c->d_sat, fa, c->d_tlo);
        HIP_TRY(hipGetLastError());
        tp.tlo = c->d_tlo;
        tp.tlo_nbx = nbx;
    }
    if (nsets > 1) {                           // the other sets start after the stats reset
        HIP_TRY(hipEventRecord(c->ev_fork, c->stream));
        for (uint32_t k = 1; k < nsets; ++k) HIP_TRY(hipStreamWaitEvent(c->set[k].stream, c->ev_fork, 0));
    }
    uint32_t launches = 0, ne = 0;
    for (uint32_t pass = 0; pass < npasses; ++pass) {
        // pass set pass % nsets: its own stream and buffers
        const zrt_context::PassSet& ps = c->set[counting ? 0u : pass % nsets];
        hipStream_t sm = counting ? c->stream : ps.stream;
        float4* const q0 = ps.q0;
        float4* const q1 = ps.q1;
        float4* const term = ps.term;
        float4* const stk4 = ps.stk4;
        float2* const stk2 = ps.stk2;
        uint32_t* const wfc = ps.wfc;
        float4* const hit = ps.hit;
        const uint32_t s0 = pass_first(pass);
        const uint32_t S = pass_count(pass);
        tp.s0 = s0;
        tp.total = S * P;
        tp.S = S;
        tp.sdiv = div_magic(S);
        const int first = pass == 0 ? 1 : 0, last = pass + 1 == npasses ? 1 : 0;
        if (!counting) {
            // per launch k: 8 work counters, then 8 region counts of the
            // paths entering launch k (written by launch k - 1)
            HIP_TRY(hipMemsetAsync(wfc, 0, 4ull * 32 * kCtr * (mb + 2), sm));
            WfParams W;
            memset(&W, 0, sizeof W);
            W.t = tp;
            W.stk4 = stk4;
            W.stk2 = stk2;
            W.term = term;
            W.T = (uint32_t)T;
            W.occx = c->d_occx;
            W.occx_words = c->occx_words;
            W.occx_ldsw = occx_ldsw;
            W.occx_nbw = c->occx_nbw;
            W.occx_moff = c->occx_moff;
            W.occx_nb0 = c->occx_nb[0];
            W.occx_nb01 = c->occx_nb[0] * c->occx_nb[1];
            W.test_min = test_min;
            W.refill_min = refill_min;
            W.rel_min = rel ? rel_min : 0u;
            W.rel_emin = rel_emin;
            W.esc = c->d_esc;
            for (uint32_t k = 0; k < nb; ++k) {
                W.q_in = (k & 1) ? q0 : q1;
                W.q_out = (k & 1) ? q1 : q0;
                W.fetch8 = wfc + kCtr * (16 * k);
                W.n_in8 = wfc + kCtr * (16 * k + 8);
                W.n_out8 = wfc + kCtr * (16 * (k + 1) + 8);
                W.hit = hit;
                W.fetch8s = wfc + kCtr * (16 * (mb + 2) + 8 * k);
                HIP_TRY(hipEventRecord(c->ev_trace[ne++], sm));
                const int cls = k == 0 ? ZRT_KERNEL_PRIMARY : (park_next ? ZRT_KERNEL_PARK : ZRT_KERNEL_BOUNCE);
                if ((rc = kt_begin(cls, sm)) != ZRT_OK) return rc;
                if (k == 0)
                    hipLaunchKernelGGL(f_first, dim3(grid_first), dim3(thr_first), lds_first, sm, W);
                else
                    hipLaunchKernelGGL(f_next, dim3(grid_next), dim3(thr_next), lds_next, sm, W);
                HIP_TRY(hipGetLastError());
                if ((rc = kt_end(sm)) != ZRT_OK) return rc;
                ++kp.launches[cls];
                if (k > 0 && park_next) {                    // same bounce, shading half
                    if ((rc = kt_begin(ZRT_KERNEL_SHADE, sm)) != ZRT_OK) return rc;
                    if (k + 1 == nb)
                        hipLaunchKernelGGL(s_last, dim3(grid_shade_last), dim3(kTraceThreads), lds_shade, sm, W);
                    else
                        hipLaunchKernelGGL(s_next, dim3(grid_shade), dim3(kTraceThreads), lds_shade, sm, W);
                    HIP_TRY(hipGetLastError());
                    if ((rc = kt_end(sm)) != ZRT_OK) return rc;
                    ++kp.launches[ZRT_KERNEL_SHADE];
                }
                HIP_TRY(hipEventRecord(c->ev_trace[ne++], sm));
                ++launches;
            }
            // the passes' sums into acc stay in pass order (stage3.zig:236-242)
            if (nsets > 1 && pass > 0) HIP_TRY(hipStreamWaitEvent(sm, c->ev_pass[pass - 1], 0));
            if ((rc = kt_begin(ZRT_KERNEL_RESOLVE, sm)) != ZRT_OK) return rc;
            hipLaunchKernelGGL(wf_resolve_kernel, dim3((P + kResPix - 1) / kResPix), dim3(kBlock), 0, sm,
                               term, stk4, stk2, (uint32_t)T, P, S, mb, c->d_acc, first, last, inv_spp,
                               c->d_rgb, want_lin ? c->d_lin : nullptr);
            if ((rc = kt_end(sm)) != ZRT_OK) return rc;
            ++kp.launches[ZRT_KERNEL_RESOLVE];
            if (nsets > 1) HIP_TRY(hipEventRecord(c->ev_pass[pass], sm));
        } else {
            HIP_TRY(hipMemsetAsync(c->d_counter, 0, 4, c->stream));
            HIP_TRY(hipEventRecord(c->ev_trace[ne++], c->stream));
            if ((rc = kt_begin(ZRT_KERNEL_COUNT, c->stream)) != ZRT_OK) return rc;
            hipLaunchKernelGGL(cfn, dim3(grid_count), dim3(kTraceThreads), lds_wf, c->stream, tp);
            HIP_TRY(hipGetLastError());
            if ((rc = kt_end(c->stream)) != ZRT_OK) return rc;
            ++kp.launches[ZRT_KERNEL_COUNT];
            ++launches;
            HIP_TRY(hipEventRecord(c->ev_trace[ne++], c->stream));
            if ((rc = kt_begin(ZRT_KERNEL_RESOLVE, c->stream)) != ZRT_OK) return rc;
            hipLaunchKernelGGL(resolve_kernel, dim3((P + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream,
                               c->d_out, P, S, c->d_acc, first, last, inv_spp, c->d_rgb,
                               want_lin ? c->d_lin : nullptr);
            if ((rc = kt_end(c->stream)) != ZRT_OK) return rc;
            ++kp.launches[ZRT_KERNEL_RESOLVE];
        }
        HIP_TRY(hipGetLastError());
    }
    for (uint32_t k = 1; k < nsets; ++k) {     // join: the other sets' passes are done
        HIP_TRY(hipEventRecord(c->set[k].ev_join, c->set[k].stream));
        HIP_TRY(hipStreamWaitEvent(c->stream, c->set[k].ev_join, 0));
    }
    HIP_TRY(hipEventRecord(c->ev_end, c->stream));
    if (outs && outs->device_rgb_packed)
        HIP_TRY(hipMemcpyAsync(outs->device_rgb_packed, c->d_rgb, 3ull * P, hipMemcpyDeviceToDevice,
                               c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));

    unsigned long long hs[64];
    HIP_TRY(copy_sync(hs, c->d_stats, sizeof hs, hipMemcpyDeviceToHost, c->stream));
    // diagnostics (debugging only): counting-build walk/test trip counts,
    // per-launch device times
    if (getenv("ZRT_CELL_STATS") && counting)
        fprintf(stderr, "{\"zrt_profile_cells\": {\"visited\": %llu, \"loaded\": %llu, \"non_empty\": %llu, "
                "\"tests\": %llu, \"wave_cell_trips\": %llu, \"wave_tri_trips\": %llu, \"trips_with_tests\": %llu, "
                "\"shared_rounds\": %llu}}\n",
                hs[1], hs[4], hs[5], hs[2], hs[6], hs[7], hs[14], hs[15]);
#ifdef ZRT_SWEEP
    if (hs[60]) {       // the early append's reservation disagreed with shading (shade_entry_keep)
        fprintf(stderr, "zrt: %llu shade continuations differ from their reservations\n", hs[60]);
        return ZRT_ERR_HIP;
    }
    if (getenv("ZRT_PARK_PROFILE") && park_next)
        fprintf(stderr, "{\"zrt_park_profile\": {\"cyc_shade_refill\": %llu, \"cyc_walk\": %llu, \"cyc_test\": %llu, "
                "\"walk_iters\": %llu, \"walk_lanes\": %llu, \"test_rounds\": %llu, \"sub_rounds\": %llu, "
                "\"pairs\": %llu, \"refill_rounds\": %llu, \"shaded_lanes\": %llu, \"cyc_drain\": %llu, "
                "\"cyc_atomic\": %llu, \"cyc_setup\": %llu}}\n",
                hs[16], hs[17], hs[18], hs[19], hs[20], hs[21], hs[22], hs[23], hs[24], hs[25], hs[26], hs[27], hs[28]);
    if (getenv("ZRT_PARK_PROFILE") && park_next)
        fprintf(stderr, "{\"zrt_walk_steps\": {\"lane_steps\": %llu, \"empty_brick_steps\": %llu, "
                "\"empty_brick_entries\": %llu, \"escapes\": %llu, \"parked_tested\": %llu, \"parked_no_refs\": %llu, "
                "\"released_early\": %llu, \"cyc_round_wait\": %llu}}\n",
                hs[48], hs[49], hs[50], hs[51], hs[52], hs[53], hs[54], hs[55]);
    if (getenv("ZRT_PARK_PROFILE") && !counting)
        fprintf(stderr, "{\"zrt_primary_profile\": {\"cyc_walk\": %llu, \"cyc_shade\": %llu, \"cyc_fetch_append\": %llu}}\n",
                hs[29], hs[30], hs[31]);
    if (getenv("ZRT_PARK_PROFILE") && park_next)   // wf_shade_kernel phases: wave cycles, active-lane sums
        fprintf(stderr, "{\"zrt_shade_profile\": {\"cyc\": [%llu, %llu, %llu, %llu, %llu, %llu, %llu, %llu], "
                "\"lanes\": [%llu, %llu, %llu, %llu, %llu, %llu, %llu, %llu], \"phases\": [\"fetch\", \"records\", "
                "\"tri_data\", \"texels\", \"u_draw\", \"pair_ziggurat\", \"tail\", \"append\"]}}\n",
                hs[32], hs[33], hs[34], hs[35], hs[36], hs[37], hs[38], hs[39], hs[40], hs[41], hs[42], hs[43],
                hs[44], hs[45], hs[46], hs[47]);
#endif
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev_begin, c->ev_end));
    st.render_ms = ms;
    const bool wf_debug = getenv("ZRT_WF_DEBUG") != nullptr;
    for (uint32_t e = 0; e + 1 < ne; e += 2) {   // trace launches only (not resolve)
        float t = 0.0f;
        HIP_TRY(hipEventElapsedTime(&t, c->ev_trace[e], c->ev_trace[e + 1]));
        st.trace_kernel_ms += t;
        if (wf_debug) fprintf(stderr, "{\"zrt_launch\": %u, \"ms\": %.3f}\n", e / 2, t);
    }
    st.trace_launches = launches;
    for (size_t k = 0; k < kn; ++k) {
        float t = 0.0f;
        HIP_TRY(hipEventElapsedTime(&t, c->ev_k[2 * k], c->ev_k[2 * k + 1]));
        kp.ms[c->ev_k_cls[k]] += t;
    }
    kp.passes = npasses;
    kp.sets = counting ? 1u : nsets;
    if (counting)
        for (int k = 0; k < 4; ++k) kp.primary_counts[k] = hs[8 + k];
    c->prof = kp;
    st.segments = hs[0];
    st.cells_visited = hs[1];
    st.triangle_tests = hs[2];
    st.hits = hs[3];
    st.samples = (uint64_t)P * spp;

    if (outs && (outs->rgb_packed || outs->rgb_image)) {
        std::vector<uint8_t> tmp;
        uint8_t* dst = outs->rgb_packed;
        if (!dst) { tmp.resize(3ull * P); dst = tmp.data(); }
        HIP_TRY(copy_sync(dst, c->d_rgb, 3ull * P, hipMemcpyDeviceToHost, c->stream));
        if (outs->rgb_image)
            for (uint32_t q = 0; q < P; ++q) memcpy(outs->rgb_image + 3ull * c->pix[q], dst + 3ull * q, 3);
    }
    if (want_lin)
        HIP_TRY(copy_sync(outs->linear_packed, c->d_lin, 3ull * P * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    if (stats) *stats = st;
    return ZRT_OK;
}

extern "C" int zrt_context_profile(const zrt_context* c, zrt_kernel_profile* out) {
    if (!c || !out) return ZRT_ERR_INVALID_ARG;
    *out = c->prof;
    return ZRT_OK;
}

void* zrt::context_stream(const zrt_context* c) { return c ? (void*)c->stream : nullptr; }

void zrt::context_set_mem_share(zrt_context* c, uint32_t share) {
    if (c) c->mem_share = std::max<uint32_t>(share, 1u);
}

int zrt::context_device_rgb(const zrt_context* c, const uint8_t** d_rgb, uint32_t* pixels, int* device) {
    if (!c || !d_rgb || !pixels || !device) return ZRT_ERR_INVALID_ARG;
    *d_rgb = c->d_rgb;
    *pixels = c->pix_valid ? (uint32_t)c->pix.size() : 0u;
    *device = c->device;
    return ZRT_OK;
}

extern "C" int zrt_render(const zrt_scene* scene, const zrt_camera* cam, const zrt_render_config* cfg,
                          uint8_t* rgb_out, zrt_stats* stats) {
    if (!scene || !cam || !cfg || !rgb_out) return ZRT_ERR_INVALID_ARG;
    if (cfg->num_devices > 1) {                // the image's tiles over a device list (group.hip)
        if (!cfg->devices) return ZRT_ERR_INVALID_ARG;
        zrt_group* g = nullptr;
        int rc = zrt_group_create(scene, cfg->devices, cfg->num_devices, &g);
        if (rc != ZRT_OK) return rc;
        zrt_render_config whole = *cfg;
        whole.rank = 0;
        whole.num_ranks = 1;
        rc = zrt_group_render(g, cam, &whole, rgb_out, stats);
        zrt_group_destroy(g);
        return rc;
    }
    // a one-entry list names the device; a null list keeps
    // cfg->device, as ABI-1 callers that set num_devices = 1 for "one device"
    // expect
    const int32_t dev = cfg->num_devices == 1 && cfg->devices ? cfg->devices[0] : cfg->device;
    zrt_context* c = nullptr;
    int rc = zrt_context_create(scene, dev, &c);
    if (rc != ZRT_OK) return rc;
    zrt_render_config one = *cfg;
    one.rank = 0;
    one.num_ranks = 1;
    zrt_outputs o{};
    o.rgb_image = rgb_out;
    rc = zrt_context_render(c, cam, &one, &o, stats);
    zrt_context_destroy(c);
    return rc;
}

// ---------------------------------------------------------------------------
// Device-function parity probes: the exact __device__ code paths of the
// kernel, evaluated on the GPU for the Tier-1 tests.
namespace {

__global__ void probe_kernel(int which, const void* in, void* out, uint32_t n, const void* aux,
                             const double* zig) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    switch (which) {
        case ZRT_PROBE_TRIANGLE: {
            const float* a = (const float*)in + 15ull * i;
            float* o = (float*)out + 4ull * i;
            const v3 v0 = ld3(a), v1 = ld3(a + 3), v2 = ld3(a + 6);
            float t = 0, u = 0, v = 0;
            const bool h = tri_ray(v0, sub(v1, v0), sub(v2, v0), ld3(a + 9), ld3(a + 12), &t, &u, &v);
            o[0] = h ? 1.0f : 0.0f; o[1] = t; o[2] = u; o[3] = v;
            break;
        }
        case ZRT_PROBE_TRIANGLE_EXACT: {  // the IEEE-division test of the mt_exact kernels
            const float* a = (const float*)in + 15ull * i;
            float* o = (float*)out + 4ull * i;
            const v3 v0 = ld3(a), v1 = ld3(a + 3), v2 = ld3(a + 6);
            float t = 0, u = 0, v = 0;
            const bool h = tri_ray<true>(v0, sub(v1, v0), sub(v2, v0), ld3(a + 9), ld3(a + 12), &t, &u, &v);
            o[0] = h ? 1.0f : 0.0f; o[1] = t; o[2] = u; o[3] = v;
            break;
        }
        case ZRT_PROBE_TRIANGLE_FLAT: {   // wf_park_kernel's branch-free test
            const float* a = (const float*)in + 15ull * i;
            float* o = (float*)out + 4ull * i;
            const v3 v0 = ld3(a), v1 = ld3(a + 3), v2 = ld3(a + 6);
            float t = 0, u = 0, v = 0;
            const bool h = tri_ray_flat(v0, sub(v1, v0), sub(v2, v0), ld3(a + 9), ld3(a + 12), &t, &u, &v);
            o[0] = h ? 1.0f : 0.0f; o[1] = h ? t : 0.0f; o[2] = h ? u : 0.0f; o[3] = h ? v : 0.0f;
            break;
        }
        case ZRT_PROBE_BBOX: {
            const float* a = (const float*)in + 12ull * i;
            float* o = (float*)out + 2ull * i;
            Bbox b; b.min = ld3(a); b.max = ld3(a + 3);
            float t = 0;
            const bool h = bbox_ray(b, ld3(a + 6), ld3(a + 9), &t);
            o[0] = h ? 1.0f : 0.0f; o[1] = h ? t : 0.0f;
            break;
        }
        case ZRT_PROBE_DDA: {
            // the kernels' own DDA: dda_init (Grid.traceRay) + DDA_STEP
            // (Iterator.next).  out: [0] steps (-1: misses the bbox, -2: the
            // incremental linear index disagreed with linearlizeCellIdx),
            // [1..3] first cell, then per step (cell after next(), t): the
            // reference's it.cell / it.next() pairs (linalg.zig:583-681)
            const float* a = (const float*)in + 12ull * i;
            const uint32_t* res = (const uint32_t*)aux;
            float* o = (float*)out + (4ull + 4ull * 64) * i;
            Bbox bb; bb.min = ld3(a); bb.max = ld3(a + 3);
            const uint32_t r3[3] = {res[0], res[1], res[2]};
            const Grid g = grid_init(bb, r3);
            const float bmin[3] = {bb.min.x, bb.min.y, bb.min.z}, bmax[3] = {bb.max.x, bb.max.y, bb.max.z};
            const float cs[3] = {g.cell_size.x, g.cell_size.y, g.cell_size.z};
            Dda s;
            // the park kernel's dda_init (dda_init_fq: the quotients from one
            // reciprocal per axis where exact, else dda_init)
            const float ics[3] = {1.0f / cs[0], 1.0f / cs[1], 1.0f / cs[2]};
            bool cs_ok = true;
            for (int k = 0; k < 3; ++k) cs_ok = cs_ok && fabsf(cs[k]) >= 0x1p-32f && fabsf(cs[k]) <= 0x1p32f;
            const bool in = ZRT_FAST_QUOT ? dda_init_fq(bmin, bmax, r3, cs, ics, cs_ok, ld3(a + 6), ld3(a + 9), s)
                                          : dda_init(bmin, bmax, r3, cs, ld3(a + 6), ld3(a + 9), s);
            if (!in) { o[0] = -1.0f; break; }
            GridK gk;
            gk.rm0 = r3[0] - 1u; gk.rm1 = r3[1] - 1u; gk.rm2 = r3[2] - 1u;
            gk.str1 = r3[0]; gk.str2 = r3[0] * r3[1];
            o[1] = (float)s.c0; o[2] = (float)s.c1; o[3] = (float)s.c2;
            int nsteps = 0;
            bool lin_ok = true;
            while (nsteps < 64) {
                const uint32_t c0 = s.c0, c1 = s.c1, c2 = s.c2;
                lin_ok = lin_ok && s.lin == (c2 * r3[1] + c1) * r3[0] + c0;
                bool crossed;
                float te;
                DDA_STEP(s, gk, 0u, crossed, te);
                (void)crossed;
                float* e = o + 4 + 4 * nsteps;
                // at the exit cell next() returns +inf and leaves the cell
                if (te == kInf) { e[0] = (float)c0; e[1] = (float)c1; e[2] = (float)c2; }
                else { e[0] = (float)s.c0; e[1] = (float)s.c1; e[2] = (float)s.c2; }
                e[3] = te;
                ++nsteps;
                if (te == kInf) break;
            }
            o[0] = lin_ok ? (float)nsteps : -2.0f;
            break;
        }
        case ZRT_PROBE_TO_RGB: {
            const float* a = (const float*)in + 3ull * i;
            uint8_t c[3];
            to_rgb(ld3(a), c);
            float* o = (float*)out + 3ull * i;
            o[0] = c[0]; o[1] = c[1]; o[2] = c[2];
            break;
        }
        case ZRT_PROBE_RNG_F32:
        case ZRT_PROBE_RNG_NORM: {
            const uint32_t* a = (const uint32_t*)in + 3ull * i;
            Rng r;
            r.s = path_key((uint64_t)a[0], a[1], a[2]);
            float* o = (float*)out + 16ull * i;
            for (int k = 0; k < 16; ++k)
                o[k] = which == ZRT_PROBE_RNG_F32 ? rng_float(r) : (float)rng_norm64(r, zig, zig + 257);
            break;
        }
        case ZRT_PROBE_EXP_LOG: {
            const double x = ((const double*)in)[i];
            double* o = (double*)out + 2ull * i;
            o[0] = det_exp(x);
            o[1] = det_log(x);
            break;
        }
        case ZRT_PROBE_TEXTURE: {
            // aux: int32 {chans, w, h, umin, umax, vmin, vmax, 0} then texels
            const int32_t* h = (const int32_t*)aux;
            DevTex t;
            t.off = 0; t.w = h[1]; t.h = h[2]; t.umin = h[3]; t.umax = h[4]; t.vmin = h[5]; t.vmax = h[6];
            const float* tex = (const float*)(h + 8);
            dev_tex_inline(t, tex, h[0]);
            const float* a = (const float*)in + 2ull * i;
            float* o = (float*)out + 3ull * i;
            if (h[0] == 3) {
                const v3 r = sample3(tex, t, a[0], a[1]);
                o[0] = r.x; o[1] = r.y; o[2] = r.z;
            } else {
                o[0] = sample1(tex, t, a[0], a[1]); o[1] = 0; o[2] = 0;
            }
            break;
        }
        case ZRT_PROBE_QUOT: {
            const float* a = (const float*)in + 2ull * i;
            float* o = (float*)out + 2ull * i;
            o[0] = quot_rn(a[0], a[1], mt_inv_det<false>(a[1]));
            o[1] = a[0] / a[1];
            break;
        }
        case ZRT_PROBE_RECIP: {
            const float x = ((const float*)in)[i];
            float* o = (float*)out + 2ull * i;
            o[0] = mt_inv_det<false>(x);
            o[1] = mt_inv_det<true>(x);
            break;
        }
        default:
            break;
    }
}

// ZRT_PROBE_RECIP_SWEEP: every float bit pattern of [lo, lo + count), the
// short reciprocal against the IEEE division, bit for bit (NaN == NaN).
__global__ __launch_bounds__(kBlock) void recip_sweep_kernel(uint32_t lo, uint32_t count, uint32_t* out) {
    uint32_t bad = 0, first = 0xFFFFFFFFu;
    for (uint32_t k = blockIdx.x * kBlock + threadIdx.x; k < count; k += gridDim.x * kBlock) {
        const float x = __uint_as_float(lo + k);
        const float a = mt_inv_det<false>(x), b = mt_inv_det<true>(x);
        const bool same = __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
        if (!same) { ++bad; first = min(first, lo + k); }
    }
    for (int o = 32; o > 0; o >>= 1) {
        bad += __shfl_xor(bad, o);
        first = min(first, (uint32_t)__shfl_xor(first, o));
    }
    if ((threadIdx.x & 63u) == 0 && bad) {
        atomicAdd(&out[0], bad);
        atomicMin(&out[1], first);
    }
}

// ZRT_PROBE_QUOT_SWEEP: every significand pair (a in [1, 2), b = 1 + s /
// 2^23 for s in [s0, s0 + ns)), quot_rn against the IEEE division, bit for bit.
__global__ __launch_bounds__(kBlock) void quot_sweep_kernel(uint32_t s0, uint32_t ns, uint32_t* out) {
    const uint64_t total = (uint64_t)ns << 23;
    uint32_t bad = 0;
    unsigned long long first = ~0ull;
    for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < total; k += (uint64_t)gridDim.x * kBlock) {
        const uint32_t ab = 0x3F800000u | (uint32_t)(k & 0x7FFFFFu);
        const uint32_t bb = 0x3F800000u | (s0 + (uint32_t)(k >> 23));
        const float a = __uint_as_float(ab), b = __uint_as_float(bb);
        const float q = quot_rn(a, b, mt_inv_det<false>(b));
        if (__float_as_uint(q) != __float_as_uint(a / b)) {
            ++bad;
            first = min(first, ((unsigned long long)bb << 32) | ab);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        bad += __shfl_xor(bad, o);
        const unsigned lo = __shfl_xor((unsigned)first, o), hi = __shfl_xor((unsigned)(first >> 32), o);
        first = min(first, ((unsigned long long)hi << 32) | lo);
    }
    if ((threadIdx.x & 63u) == 0 && bad) {
        atomicAdd(&out[0], bad);
        atomicMin(reinterpret_cast<unsigned long long*>(out + 2), first);
    }
}

}  // namespace

extern "C" int zrt_probe(int which, const void* in, void* out, uint32_t n, const void* aux, int device) {
    if (!in || !out || n == 0) return ZRT_ERR_INVALID_ARG;
    size_t in_sz = 0, out_sz = 0, aux_sz = 0;
    switch (which) {
        case ZRT_PROBE_TRIANGLE:
        case ZRT_PROBE_TRIANGLE_EXACT:
        case ZRT_PROBE_TRIANGLE_FLAT: in_sz = 60; out_sz = 16; break;
        case ZRT_PROBE_BBOX: in_sz = 48; out_sz = 8; break;
        case ZRT_PROBE_DDA: in_sz = 48; out_sz = 4 * (4 + 4 * 64); aux_sz = 12; break;
        case ZRT_PROBE_TO_RGB: in_sz = 12; out_sz = 12; break;
        case ZRT_PROBE_RNG_F32:
        case ZRT_PROBE_RNG_NORM: in_sz = 12; out_sz = 64; break;
        case ZRT_PROBE_EXP_LOG: in_sz = 8; out_sz = 16; break;
        case ZRT_PROBE_RECIP: in_sz = 4; out_sz = 8; break;
        case ZRT_PROBE_RECIP_SWEEP: in_sz = 8; out_sz = 16; break;
        case ZRT_PROBE_QUOT: in_sz = 8; out_sz = 8; break;
        case ZRT_PROBE_QUOT_SWEEP: in_sz = 8; out_sz = 16; break;
        case ZRT_PROBE_TEXTURE: {
            in_sz = 8; out_sz = 12;
            if (!aux) return ZRT_ERR_INVALID_ARG;
            const int32_t* h = (const int32_t*)aux;
            if ((h[0] != 1 && h[0] != 3) || h[1] <= 0 || h[2] <= 0) return ZRT_ERR_INVALID_ARG;
            aux_sz = 32 + 4ull * h[0] * h[1] * h[2];
            break;
        }
        default: return ZRT_ERR_INVALID_ARG;
    }
    if (aux_sz && !aux) return ZRT_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ZRT_ERR_NO_DEVICE;
    DeviceGuard g(device);
    void *d_in = nullptr, *d_out = nullptr, *d_aux = nullptr;
    double* d_zig = nullptr;
    double zig[514];
    zig_tables(zig, zig + 257);
    int rc = ZRT_OK;
    auto cleanup = [&]() {
        if (d_in) (void)hipFree(d_in);
        if (d_out) (void)hipFree(d_out);
        if (d_aux) (void)hipFree(d_aux);
        if (d_zig) (void)hipFree(d_zig);
    };
    auto run = [&]() -> int {
        HIP_TRY(hipMalloc(&d_in, in_sz * n));
        HIP_TRY(hipMalloc(&d_out, out_sz * n));
        HIP_TRY(hipMalloc((void**)&d_zig, sizeof zig));
        HIP_TRY(hipMemcpy(d_in, in, in_sz * n, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(d_zig, zig, sizeof zig, hipMemcpyHostToDevice));
        if (aux_sz) {
            HIP_TRY(hipMalloc(&d_aux, aux_sz));
            HIP_TRY(hipMemcpy(d_aux, aux, aux_sz, hipMemcpyHostToDevice));
        }
        if (which == ZRT_PROBE_QUOT_SWEEP) {
            // out per range: {mismatches, 0, first (a bits, b bits) as a u64 min}
            const uint32_t* r = (const uint32_t*)in;
            std::vector<uint32_t> init(4ull * n, 0u);
            for (uint32_t k = 0; k < n; ++k) init[4ull * k + 2] = init[4ull * k + 3] = 0xFFFFFFFFu;
            HIP_TRY(hipMemcpy(d_out, init.data(), out_sz * n, hipMemcpyHostToDevice));
            for (uint32_t k = 0; k < n; ++k) {
                if (r[2 * k + 1] == 0) continue;
                if ((uint64_t)r[2 * k] + r[2 * k + 1] > (1ull << 23)) return ZRT_ERR_INVALID_ARG;
                hipLaunchKernelGGL(quot_sweep_kernel, dim3(16384), dim3(kBlock), 0, 0, r[2 * k], r[2 * k + 1],
                                   (uint32_t*)d_out + 4ull * k);
                HIP_TRY(hipGetLastError());
            }
        } else if (which == ZRT_PROBE_RECIP_SWEEP) {
            const uint32_t* r = (const uint32_t*)in;
            std::vector<uint32_t> init(4ull * n, 0u);
            for (uint32_t k = 0; k < n; ++k) init[4ull * k + 1] = 0xFFFFFFFFu;
            HIP_TRY(hipMemcpy(d_out, init.data(), out_sz * n, hipMemcpyHostToDevice));
            for (uint32_t k = 0; k < n; ++k) {
                if (r[2 * k + 1] == 0) continue;
                if ((uint64_t)r[2 * k] + r[2 * k + 1] > 0x100000000ull) return ZRT_ERR_INVALID_ARG;
                const uint32_t blocks = std::min<uint32_t>(8192u, (r[2 * k + 1] + kBlock - 1) / kBlock);
                hipLaunchKernelGGL(recip_sweep_kernel, dim3(blocks), dim3(kBlock), 0, 0, r[2 * k], r[2 * k + 1],
                                   (uint32_t*)d_out + 4ull * k);
                HIP_TRY(hipGetLastError());
            }
        } else {
            hipLaunchKernelGGL(probe_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, which, d_in, d_out, n,
                               d_aux, d_zig);
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(out, d_out, out_sz * n, hipMemcpyDeviceToHost));
        return ZRT_OK;
    };
    rc = run();
    cleanup();
    return rc;
}
