// Uniform-grid DDA (Grid.traceRay / Grid.Iterator, linalg.zig:443-496) and
// the exact empty-brick skip, shared by the HIP kernels (render.hip) and the
// host-side check tests/cpp/dda_skip_check.cpp (g++ -ffp-contract=off).
#pragma once
#include <stdint.h>

#include "zrt_math.h"

namespace zrt {

ZHD uint32_t zmin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// Grid.Iterator state (linalg.zig:471-477) + the running cell index.  The
// exit cell, step and linear-index step of each axis follow from the sign of
// the ray direction (linalg.zig:450-452), kept as 3 bits in `neg`.
struct Dda {
    float tn0, tn1, tn2, td0, td1, td2;
    uint32_t c0, c1, c2;
    uint32_t lin;
    uint32_t neg;             // bit a: dir[a] < 0
};

// Grid.traceRay (linalg.zig:443-469); false if the ray misses the grid bbox.
ZHD bool dda_init(const float* bmin, const float* bmax, const uint32_t* res, const float* cs, v3 o, v3 d,
                  Dda& s) {
    Bbox bb;
    bb.min = mk(bmin[0], bmin[1], bmin[2]);
    bb.max = mk(bmax[0], bmax[1], bmax[2]);
    float t_hit;
    if (!bbox_ray(bb, o, d, &t_hit)) return false;
    t_hit = fmaxf(0.0f, t_hit);
    const v3 local = sub(add(o, scale(d, t_hit)), bb.min);
    const bool n0 = d.x < 0.0f, n1 = d.y < 0.0f, n2 = d.z < 0.0f;
    s.c0 = zmin(f2u(local.x / cs[0]), res[0] - 1u);
    s.c1 = zmin(f2u(local.y / cs[1]), res[1] - 1u);
    s.c2 = zmin(f2u(local.z / cs[2]), res[2] - 1u);
    s.neg = (n0 ? 1u : 0u) | (n1 ? 2u : 0u) | (n2 ? 4u : 0u);
    s.td0 = fabsf(cs[0] / d.x);
    s.td1 = fabsf(cs[1] / d.y);
    s.td2 = fabsf(cs[2] / d.z);
    s.tn0 = t_hit + ((((float)(s.c0 + (n0 ? 0u : 1u))) * cs[0] - local.x) / d.x);
    s.tn1 = t_hit + ((((float)(s.c1 + (n1 ? 0u : 1u))) * cs[1] - local.y) / d.y);
    s.tn2 = t_hit + ((((float)(s.c2 + (n2 ? 0u : 1u))) * cs[2] - local.z) / d.z);
    s.lin = (s.c2 * res[1] + s.c1) * res[0] + s.c0;
    // bit 3: some crossing sequence starts at -inf / NaN (a zero direction
    // component on a boundary), where BRICK_SKIP4's merge argument fails
    const bool ok = s.tn0 > -kInf && s.tn1 > -kInf && s.tn2 > -kInf && s.td0 == s.td0 && s.td1 == s.td1 &&
                    s.td2 == s.td2;
    s.neg |= ok ? 0u : 8u;
    return true;
}

// dda_init with its fifteen f32 divisions (bbox_ray's six, then three cell
// indices, three t_delta and three first crossings) as quot_rn quotients:
// one correctly rounded reciprocal of each direction component (the
// mt_inv_det sequence, exact for normal |d| <= 2^126) shared by the four
// divisions by it, and the cell sizes' reciprocals RN(1 / cs) from the host
// (`ics`, valid when `cs_ok`: every cs in [2^-32, 2^32]).  When every
// numerator is 0 or of magnitude in [2^-64, 2^64] (or NaN) and every |d| in
// [2^-32, 1], each quotient is the division's bit for bit (quot_rn), so the
// state is dda_init's; otherwise the lane recomputes it with dda_init.  The
// check costs ~2 VALU per operand; 11-VALU divisions become 4-VALU quotients
// (DESIGN 5.5e).
#ifndef ZRT_FAST_QUOT
#define ZRT_FAST_QUOT 1
#endif
#if defined(__HIPCC__)
// (bits << 1) - 2 of a float: its magnitude's bits doubled, minus 2 -- zero
// wraps to the top, so a minimum >= 2 * bits(2^-64) - 2 says "0 or >= 2^-64"
ZHD uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
__device__ __forceinline__ uint32_t quot_low3(float a, float b, float c) {
    const uint32_t x = (fbits(a) << 1) - 2u, y = (fbits(b) << 1) - 2u, z = (fbits(c) << 1) - 2u;
    return zmin(x, zmin(y, z));
}
__device__ __forceinline__ float abs_max3(float a, float b, float c) {
    return fmaxf(fabsf(a), fmaxf(fabsf(b), fabsf(c)));
}
__device__ __forceinline__ bool dda_init_fq(const float* bmin, const float* bmax, const uint32_t* res, const float* cs,
                                            const float* ics, bool cs_ok, v3 o, v3 d, Dda& s) {
    const float yx = mt_inv_det<false>(d.x), yy = mt_inv_det<false>(d.y), yz = mt_inv_det<false>(d.z);
    // bbox_ray (linalg.zig:324-349)
    const bool sx = d.x < 0.0f, sy = d.y < 0.0f, sz = d.z < 0.0f;
    const float lx = (sx ? bmax[0] : bmin[0]) - o.x, ly = (sy ? bmax[1] : bmin[1]) - o.y,
                lz = (sz ? bmax[2] : bmin[2]) - o.z;
    const float hx = (sx ? bmin[0] : bmax[0]) - o.x, hy = (sy ? bmin[1] : bmax[1]) - o.y,
                hz = (sz ? bmin[2] : bmax[2]) - o.z;
    const float mnx = quot_rn(lx, d.x, yx), mny = quot_rn(ly, d.y, yy), mnz = quot_rn(lz, d.z, yz);
    const float mxx = quot_rn(hx, d.x, yx), mxy = quot_rn(hy, d.y, yy), mxz = quot_rn(hz, d.z, yz);
    float tmin = mnx, tmax = mxx;
    bool hit = !((tmin > mxy) || (tmax < mny));
    tmin = fmaxf(tmin, mny);
    tmax = fminf(tmax, mxy);
    hit = hit && !((tmin > mxz) || (tmax < mnz));
    tmin = fmaxf(tmin, mnz);
    // Grid.traceRay (linalg.zig:443-469)
    const float t_hit = fmaxf(0.0f, tmin);
    const v3 local = sub(add(o, scale(d, t_hit)), mk(bmin[0], bmin[1], bmin[2]));
    const bool n0 = sx, n1 = sy, n2 = sz;
    const uint32_t c0 = zmin(f2u(quot_rn(local.x, cs[0], ics[0])), res[0] - 1u);
    const uint32_t c1 = zmin(f2u(quot_rn(local.y, cs[1], ics[1])), res[1] - 1u);
    const uint32_t c2 = zmin(f2u(quot_rn(local.z, cs[2], ics[2])), res[2] - 1u);
    const float ax = ((float)(c0 + (n0 ? 0u : 1u))) * cs[0] - local.x;
    const float ay = ((float)(c1 + (n1 ? 0u : 1u))) * cs[1] - local.y;
    const float az = ((float)(c2 + (n2 ? 0u : 1u))) * cs[2] - local.z;
    // the operands' range (quot_rn): numerators 0 or in [2^-64, 2^64] (NaN
    // passes: it stays NaN either way), |d| in [2^-32, 1]
    const float big = fmaxf(fmaxf(abs_max3(lx, ly, lz), abs_max3(hx, hy, hz)),
                            fmaxf(abs_max3(local.x, local.y, local.z), abs_max3(ax, ay, az)));
    const uint32_t low = zmin(zmin(quot_low3(lx, ly, lz), quot_low3(hx, hy, hz)),
                              zmin(quot_low3(local.x, local.y, local.z), quot_low3(ax, ay, az)));
    const float dmin = fminf(fabsf(d.x), fminf(fabsf(d.y), fabsf(d.z)));
    const bool ok = cs_ok && !(big > 0x1p64f) && low >= 2u * 0x1F800000u - 2u && dmin >= 0x1p-32f;
    if (!ok) return dda_init(bmin, bmax, res, cs, o, d, s);
    if (!hit) return false;
    s.c0 = c0; s.c1 = c1; s.c2 = c2;
    s.neg = (n0 ? 1u : 0u) | (n1 ? 2u : 0u) | (n2 ? 4u : 0u);
    s.td0 = fabsf(quot_rn(cs[0], d.x, yx));
    s.td1 = fabsf(quot_rn(cs[1], d.y, yy));
    s.td2 = fabsf(quot_rn(cs[2], d.z, yz));
    s.tn0 = t_hit + quot_rn(ax, d.x, yx);
    s.tn1 = t_hit + quot_rn(ay, d.y, yy);
    s.tn2 = t_hit + quot_rn(az, d.z, yz);
    s.lin = (s.c2 * res[1] + s.c1) * res[0] + s.c0;
    const bool fin = s.tn0 > -kInf && s.tn1 > -kInf && s.tn2 > -kInf && s.td0 == s.td0 && s.td1 == s.td1 &&
                     s.td2 == s.td2;
    s.neg |= fin ? 0u : 8u;
    return true;
}
#endif

// Iterator.next (linalg.zig:478-496), branch-free.  map[k] with
// k = (t0<t1)<<2 | (t0<t2)<<1 | (t1<t2) and map = {2,1,2,1,2,2,0,0} is
// exactly: axis 0 iff t0<t1 && t0<t2; axis 1 iff !(t0<t1) && t1<t2; else 2
// (same booleans, so NaNs pick the same axis).  T_EXIT = the crossing t of
// the chosen axis, or +inf at the exit cell.  On that +inf the state is
// stepped past the exit, which is harmless: traceRay always stops there
// (nearest <= inf).  CROSSED: the step left the current occupancy brick.
// A macro over a local Dda, not a function on a reference: as a function,
// InstCombine turns `a0 ? s.c0 : s.c1` into a load through a selected
// pointer and the whole state lands in scratch memory.  For the same reason
// the grid constants come in as a GridK of laundered registers: selecting
// between res[0..2] directly became a global load from the kernel
// arguments at a selected offset, i.e. a memory round trip in every step.
struct GridK {
    uint32_t rm0, rm1, rm2;   // res[k] - 1: last cell index per axis
    uint32_t str1, str2;      // linear-index strides of axes 1 and 2
};
#define DDA_STEP(S, G, SH, CROSSED, T_EXIT)                                           \
    do {                                                                             \
        const float t0_ = (S).tn0, t1_ = (S).tn1, t2_ = (S).tn2;                     \
        const bool b01_ = t0_ < t1_, b02_ = t0_ < t2_, b12_ = t1_ < t2_;             \
        const bool a0_ = b01_ && b02_;                                               \
        const bool a1_ = !b01_ && b12_;                                              \
        const bool a2_ = !a0_ && !a1_;                                               \
        const float tc_ = a0_ ? t0_ : (a1_ ? t1_ : t2_);                             \
        const uint32_t c0_ = (S).c0, c1_ = (S).c1, c2_ = (S).c2;                     \
        const uint32_t cc_ = a0_ ? c0_ : (a1_ ? c1_ : c2_);                          \
        const uint32_t ax_ = a0_ ? 0u : (a1_ ? 1u : 2u);                             \
        const bool ng_ = ((S).neg >> ax_) & 1u;                                      \
        const uint32_t rm1_ = a0_ ? (G).rm0 : (a1_ ? (G).rm1 : (G).rm2);           \
        const uint32_t ec_ = ng_ ? 0u : rm1_;                                        \
        const uint32_t cn_ = ng_ ? cc_ - 1u : cc_ + 1u;                              \
        const uint32_t str_ = a0_ ? 1u : (a1_ ? (G).str1 : (G).str2);             \
        (CROSSED) = ((cc_ ^ cn_) >> (SH)) != 0u;                                     \
        const float u0_ = t0_ + (S).td0, u1_ = t1_ + (S).td1, u2_ = t2_ + (S).td2;   \
        (S).tn0 = a0_ ? u0_ : t0_;                                                   \
        (S).tn1 = a1_ ? u1_ : t1_;                                                   \
        (S).tn2 = a2_ ? u2_ : t2_;                                                   \
        (S).c0 = a0_ ? cn_ : c0_;                                                    \
        (S).c1 = a1_ ? cn_ : c1_;                                                    \
        (S).c2 = a2_ ? cn_ : c2_;                                                    \
        (S).lin = ng_ ? (S).lin - str_ : (S).lin + str_;                             \
        (T_EXIT) = cc_ == ec_ ? kInf : tc_;                                          \
    } while (0)

// The park kernel's walk state: Dda with every per-axis quantity of a step
// resolved at setup -- the exit cell e_a (0 or res_a - 1), the cell step s_a
// (+1 or -1 mod 2^32) and the linear-index step l_a (+-1, +-str1, +-str2
// mod 2^32; axis 0's is s_0) -- so a step selects them by axis instead of deriving them from
// the sign bits and the grid constants (DDA_STEP: 44 VALU per step in the
// r02m ISA, this: 29).  Same booleans, same f32 adds, same cells and T_EXIT
// as DDA_STEP (tests/cpp/dda_skip_check.cpp compares the two step by step).
struct DdaW {
    float tn0, tn1, tn2, td0, td1, td2;
    uint32_t c0, c1, c2;
    uint32_t lin;
    uint32_t e0, e1, e2;
    uint32_t s0, s1, s2;      // s0 is also axis 0's linear-index step
    uint32_t l1, l2;
};
ZHD void ddaw_from(const Dda& d, const GridK& g, DdaW& w) {
    w.tn0 = d.tn0; w.tn1 = d.tn1; w.tn2 = d.tn2;
    w.td0 = d.td0; w.td1 = d.td1; w.td2 = d.td2;
    w.c0 = d.c0; w.c1 = d.c1; w.c2 = d.c2;
    w.lin = d.lin;
    const bool n0 = d.neg & 1u, n1 = (d.neg >> 1) & 1u, n2 = (d.neg >> 2) & 1u;
    w.e0 = n0 ? 0u : g.rm0;
    w.e1 = n1 ? 0u : g.rm1;
    w.e2 = n2 ? 0u : g.rm2;
    w.s0 = n0 ? 0xFFFFFFFFu : 1u;
    w.s1 = n1 ? 0xFFFFFFFFu : 1u;
    w.s2 = n2 ? 0xFFFFFFFFu : 1u;
    w.l1 = n1 ? 0u - g.str1 : g.str1;
    w.l2 = n2 ? 0u - g.str2 : g.str2;
}
#define DDAW_STEP(S, SH, CROSSED, T_EXIT)                                            \
    do {                                                                             \
        const float t0_ = (S).tn0, t1_ = (S).tn1, t2_ = (S).tn2;                     \
        const bool b01_ = t0_ < t1_, b02_ = t0_ < t2_, b12_ = t1_ < t2_;             \
        const bool a0_ = b01_ && b02_;                                               \
        const bool a1_ = !b01_ && b12_;                                              \
        const bool a2_ = !a0_ && !a1_;                                               \
        const float tc_ = a0_ ? t0_ : (a1_ ? t1_ : t2_);                             \
        const float dt_ = a0_ ? (S).td0 : (a1_ ? (S).td1 : (S).td2);                 \
        const uint32_t cc_ = a0_ ? (S).c0 : (a1_ ? (S).c1 : (S).c2);                 \
        const uint32_t ec_ = a0_ ? (S).e0 : (a1_ ? (S).e1 : (S).e2);                 \
        const uint32_t cn_ = cc_ + (a0_ ? (S).s0 : (a1_ ? (S).s1 : (S).s2));         \
        (S).lin += a0_ ? (S).s0 : (a1_ ? (S).l1 : (S).l2);                           \
        (CROSSED) = ((cc_ ^ cn_) >> (SH)) != 0u;                                     \
        const float un_ = tc_ + dt_;                                                 \
        (S).tn0 = a0_ ? un_ : t0_;                                                   \
        (S).tn1 = a1_ ? un_ : t1_;                                                   \
        (S).tn2 = a2_ ? un_ : t2_;                                                   \
        (S).c0 = a0_ ? cn_ : (S).c0;                                                 \
        (S).c1 = a1_ ? cn_ : (S).c1;                                                 \
        (S).c2 = a2_ ? cn_ : (S).c2;                                                 \
        (T_EXIT) = cc_ == ec_ ? kInf : tc_;                                          \
    } while (0)

// Field-wise select of a walk state (a struct-level `c ? a : b` may become a
// load through a selected pointer, see DDA_STEP).  Fields that are equal in
// A and B (the per-axis constants) fold away.
#define DDAW_SEL(D, C, A, B)                                                          \
    do {                                                                             \
        (D).tn0 = (C) ? (A).tn0 : (B).tn0; (D).tn1 = (C) ? (A).tn1 : (B).tn1;        \
        (D).tn2 = (C) ? (A).tn2 : (B).tn2; (D).td0 = (C) ? (A).td0 : (B).td0;        \
        (D).td1 = (C) ? (A).td1 : (B).td1; (D).td2 = (C) ? (A).td2 : (B).td2;        \
        (D).c0 = (C) ? (A).c0 : (B).c0; (D).c1 = (C) ? (A).c1 : (B).c1;              \
        (D).c2 = (C) ? (A).c2 : (B).c2; (D).lin = (C) ? (A).lin : (B).lin;           \
        (D).e0 = (C) ? (A).e0 : (B).e0; (D).e1 = (C) ? (A).e1 : (B).e1;              \
        (D).e2 = (C) ? (A).e2 : (B).e2; (D).s0 = (C) ? (A).s0 : (B).s0;              \
        (D).s1 = (C) ? (A).s1 : (B).s1; (D).s2 = (C) ? (A).s2 : (B).s2;              \
        (D).l1 = (C) ? (A).l1 : (B).l1; (D).l2 = (C) ? (A).l2 : (B).l2;              \
    } while (0)

// The packed walk state (the park walk and the primary lane walk, grids of
// at most 1024 cells per axis): the cell in one word of per-grid fields,
// pc = c0 | c1 << o1 | c2 << o2, field a B_a = max(2, ceil(log2 res_a)) bits
// wide (o1 = B0, o2 = B0 + B1, B0 + B1 + B2 <= 30).  For res_a = 2^B_a the
// word IS linearlizeCellIdx (linalg.zig:429-431), and otherwise it indexes a
// copy of the cells padded to 2^B0 x 2^B1 x 2^B2, so the walk keeps no
// separate linear index.  A step adds the axis's packed step d_a
// (+-1 << o_a mod 2^32); the brick-crossing test is one xor and mask; the
// exit test compares the axis's field with the packed exit cells pe.  Same
// booleans, same f32 adds, same cells and T_EXIT as DDA_STEP
// (tests/cpp/dda_skip_check.cpp, step by step on random grids).  A step past
// the exit (T_EXIT = +inf) may carry into the next field; the walk ends there
// (the park kernel's speculative second step only reads a clamped brick).
// Brick-major words (bm = 1; grids of 4 to 1024 cells per axis, powers of
// two): bits [0, 6) hold every axis's low two bits (x | y << 2 | z << 4, the
// cell's index inside its 4^3 brick) and the fields' high parts follow (x
// from bit 6, y from o1, z from o2), so the word >> 6 is the brick's linear
// index and its low six bits the in-brick index (no multiply, no field
// extracts: 8 VALU less per OccX lookup).  A field is then two bit runs, and
// a step adds +-lowbit(f_a) across the gap (pk_add: 3 VALU more per step).
// The kernels take the layout as a template parameter (PK_BM, which the step
// macros below name).
struct PackK {
    uint32_t o1, o2;          // bit offsets of fields 1 and 2 (field 0 at bit 0; bm: of their high parts)
    uint32_t b0, b1, b2;      // field widths
    uint32_t f0, f1, f2;      // field masks
    uint32_t low2;            // in-brick bits of every field, 4^3 bricks
    uint32_t kmul, kshr;      // in-brick cell index: ((pc & low2) * kmul) >> kshr = x | y << 2 | z << 4
    uint32_t bm;              // brick-major layout (then low2 = 63, kmul = 1, kshr = 0)
};
constexpr uint32_t kPackMaxRes = 1024;                         // cells per axis a packed walk holds
ZHD uint32_t ceil_log2u(uint32_t x) {
    uint32_t b = 0;
    while (b < 32 && (1ull << b) < x) ++b;
    return b;
}
// The layout for given field widths; false if the in-brick index multiplier
// does not work for it.  The multiplier sums the three fields' low two bits,
// shifted to x | y << 2 | z << 4: exact when no two of the nine shifted bit
// pairs overlap (then the sum has no carry); checked here for every in-brick
// cell, which is exactly the function the kernels compute.
ZHD bool pack_fields(uint32_t b0, uint32_t b1, uint32_t b2, PackK& k) {
    if (b0 + b1 + b2 > 30u) return false;
    k.b0 = b0; k.b1 = b1; k.b2 = b2;
    k.o1 = b0;
    k.o2 = b0 + b1;
    k.f0 = (1u << b0) - 1u;
    k.f1 = ((1u << b1) - 1u) << k.o1;
    k.f2 = ((1u << b2) - 1u) << k.o2;
    k.low2 = 3u | (3u << k.o1) | (3u << k.o2);
    uint32_t sh = 0;
    if (k.o1 > 2u + sh) sh = k.o1 - 2u;
    if (k.o2 > 4u + sh) sh = k.o2 - 4u;
    k.kshr = sh;
    k.kmul = (1u << sh) + (1u << (sh + 2u - k.o1)) + (1u << (sh + 4u - k.o2));
    if (k.kmul >= (1u << 24)) return false;                    // a 24-bit multiply operand
    if (k.o2 + 2u > 24u) return false;                         // pc & low2 must fit 24 bits too
    for (uint32_t c = 0; c < 64; ++c) {
        const uint32_t t = (c & 3u) | (((c >> 2) & 3u) << k.o1) | ((c >> 4) << k.o2);
        // exactly the kernels' __umul24 (24-bit operands, low 32 bits of the product)
        if (((((t & 0xFFFFFFu) * (k.kmul & 0xFFFFFFu)) >> k.kshr) & 63u) != c) return false;
    }
    return true;
}
// Division of a pass item (< 2^31) by the pass's samples per pixel S, as one
// 32x32->64 multiply and a shift (Granlund-Montgomery with N = 31:
// m = ceil(2^(31+l) / S), l = ceil(log2 S), so 2^(31+l) <= m S < 2^(31+l) + 2^l
// and floor(n m / 2^(31+l)) = floor(n / S) for every n < 2^31; m < 2^32 for
// S < 2^31).  Items are pixel-major (item = q S + s), so q = item / S is the
// pixel and item - q S the sample (tests/cpp/div_check.cpp: every S < 2^16).
struct DivS {
    uint32_t m, sh;
};
ZHD DivS div_magic(uint32_t S) {
    uint32_t l = 0;
    while (l < 31 && (1ull << l) < S) ++l;
    DivS r;
    r.sh = 31u + l;
    r.m = (uint32_t)(((1ull << r.sh) + S - 1) / S);
    return r;
}
ZHD uint32_t div_by(uint32_t n, const DivS& d) { return (uint32_t)(((uint64_t)n * d.m) >> d.sh); }

// The layout for a grid; false if it does not pack (an axis above 1024
// cells).  Fields as narrow as the resolution allows (then the word is the
// linear index on power-of-two grids), widened where close fields would make
// the in-brick multiplier's bit pairs overlap (small grids; they then index a
// padded copy of the cells).
// The brick-major layout, if the grid allows it.
ZHD bool pack_layout_bm(const uint32_t res[3], PackK& k) {
    uint32_t bb[3];
    for (int a = 0; a < 3; ++a) {
        if (res[a] < 4u || res[a] > kPackMaxRes || (res[a] & (res[a] - 1u)) != 0u) return false;
        bb[a] = ceil_log2u(res[a]);
    }
    if (bb[0] + bb[1] + bb[2] > 30u) return false;
    k.b0 = bb[0]; k.b1 = bb[1]; k.b2 = bb[2];
    k.o1 = 6u + (bb[0] - 2u);
    k.o2 = k.o1 + (bb[1] - 2u);
    k.f0 = 3u | (((1u << (bb[0] - 2u)) - 1u) << 6u);
    k.f1 = (3u << 2u) | (((1u << (bb[1] - 2u)) - 1u) << k.o1);
    k.f2 = (3u << 4u) | (((1u << (bb[2] - 2u)) - 1u) << k.o2);
    k.low2 = 63u;
    k.kmul = 1u;
    k.kshr = 0u;
    k.bm = 1u;
    return true;
}
// BM_OK: the brick-major layout where the grid allows it (pack_layout_bm).
ZHD bool pack_layout(const uint32_t res[3], PackK& k, bool bm_ok = false) {
    if (bm_ok && pack_layout_bm(res, k)) return true;
    k.bm = 0u;
    uint32_t b[3];
    for (int a = 0; a < 3; ++a) {
        if (res[a] == 0 || res[a] > kPackMaxRes) return false;
        b[a] = ceil_log2u(res[a]) < 2u ? 2u : ceil_log2u(res[a]);
    }
    for (uint32_t extra = 0; extra <= 16; ++extra)            // fewest added bits first
        for (uint32_t e0 = 0; e0 <= extra; ++e0)
            if (pack_fields(b[0] + e0, b[1] + (extra - e0), b[2], k)) return true;
    return false;
}
template <bool BM>
ZHD uint32_t pack_cellt(const PackK& k, uint32_t c0, uint32_t c1, uint32_t c2) {
    if (BM)
        return (c0 & 3u) | ((c1 & 3u) << 2) | ((c2 & 3u) << 4) | ((c0 >> 2) << 6) | ((c1 >> 2) << k.o1) |
               ((c2 >> 2) << k.o2);
    return c0 | (c1 << k.o1) | (c2 << k.o2);
}
ZHD uint32_t pack_cellv(const PackK& k, uint32_t c0, uint32_t c1, uint32_t c2) {
    return k.bm ? pack_cellt<true>(k, c0, c1, c2) : pack_cellt<false>(k, c0, c1, c2);
}
// whether the packed word equals the linear cell index (no padded copy needed)
ZHD bool pack_is_linear(const uint32_t res[3], const PackK& k) {
    return !k.bm && res[0] == (1u << k.b0) && res[1] == (1u << k.b1) && res[2] == (1u << k.b2);
}
// Axis a's cell coordinate of a packed word
ZHD uint32_t pack_coord(const PackK& k, uint32_t pc, int a) {
    const uint32_t o = a == 0 ? 0u : (a == 1 ? k.o1 : k.o2), b = a == 0 ? k.b0 : (a == 1 ? k.b1 : k.b2);
    if (k.bm) return ((pc >> (2 * a)) & 3u) | (((pc >> (a == 0 ? 6u : o)) & ((1u << (b - 2u)) - 1u)) << 2);
    return (pc >> o) & (b >= 32u ? ~0u : (1u << b) - 1u);
}
template <bool BM>
ZHD uint32_t pack_coordt(const PackK& k, uint32_t pc, int a) {
    const uint32_t o = a == 0 ? 0u : (a == 1 ? k.o1 : k.o2), b = a == 0 ? k.b0 : (a == 1 ? k.b1 : k.b2);
    if (BM) return ((pc >> (2 * a)) & 3u) | (((pc >> (a == 0 ? 6u : o)) & ((1u << (b - 2u)) - 1u)) << 2);
    return (pc >> o) & (b >= 32u ? ~0u : (1u << b) - 1u);
}
// The packed word with axis a's coordinate (field F) replaced by c
template <bool BM>
ZHD uint32_t pk_setc(const PackK& k, uint32_t pc, uint32_t f, int a, uint32_t c) {
    const uint32_t o = a == 0 ? 0u : (a == 1 ? k.o1 : k.o2);
    if (BM) return (pc & ~f) | ((c & 3u) << (2 * a)) | ((c >> 2) << (a == 0 ? 6u : o));
    return (pc & ~f) | (c << o);
}
// pc + D on field F (D = +-lowbit(F), one cell): one add for contiguous
// fields; for brick-major ones the gap between the field's two runs is filled
// with ones (forward: the carry crosses it) or cleared (backward: the borrow
// does), the sum masked to F and the other fields kept.  No carry leaves the
// field.  (pk_addn: n cells.)
#ifndef ZRT_PK_BITOP3
#define ZRT_PK_BITOP3 1
#endif
template <bool BM>
ZHD uint32_t pk_add(uint32_t pc, uint32_t f, uint32_t d) {
    if (!BM) return pc + d;
    const uint32_t s = (uint32_t)((int32_t)d >> 31);
#if defined(__HIP_DEVICE_COMPILE__) && defined(__gfx950__) && ZRT_PK_BITOP3
    // (v_bitop3 is a gfx950 instruction: an ARCH= build for another target
    // takes the plain expression below)
    // g = (pc & f) | (~f & ~s) as ONE v_bitop3 (table index pc*4 + f*2 + s:
    // rows 0, 4, 6, 7 set); left to itself the compiler selects ~f by the
    // sign with a compare, a select and a v_not (6 VALU per step, not 4)
    uint32_t g;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xd1" : "=v"(g) : "v"(pc), "v"(f), "v"(s));
#else
    const uint32_t g = (pc & f) | (~f & ~s);
#endif
    return ((g + d) & f) | (pc & ~f);
}
// (a masked add of n * D is NOT n steps on a brick-major field: n's bits
// above the low run would land in the gap; pk_setc writes the coordinate)
template <bool BM>
ZHD uint32_t pk_addn(uint32_t pc, uint32_t f, uint32_t n, uint32_t d) {
    if (!BM) return pc + n * d;
    for (uint32_t i = 0; i < n; ++i) pc = pk_add<true>(pc, f, d);
    return pc;
}
struct DdaV {
    float tn0, tn1, tn2, td0, td1, td2;
    uint32_t pc, pe;
    uint32_t d0, d1, d2;      // packed cell step per axis
};
template <bool BM>
ZHD void ddav_from_t(const Dda& d, const GridK& g, const PackK& k, DdaV& w) {
    w.tn0 = d.tn0; w.tn1 = d.tn1; w.tn2 = d.tn2;
    w.td0 = d.td0; w.td1 = d.td1; w.td2 = d.td2;
    w.pc = pack_cellt<BM>(k, d.c0, d.c1, d.c2);
    const bool n0 = d.neg & 1u, n1 = (d.neg >> 1) & 1u, n2 = (d.neg >> 2) & 1u;
    w.pe = pack_cellt<BM>(k, n0 ? 0u : g.rm0, n1 ? 0u : g.rm1, n2 ? 0u : g.rm2);
    const uint32_t s1 = BM ? 4u : (1u << k.o1), s2 = BM ? 16u : (1u << k.o2);
    w.d0 = n0 ? 0xFFFFFFFFu : 1u;
    w.d1 = n1 ? 0u - s1 : s1;
    w.d2 = n2 ? 0u - s2 : s2;
}
ZHD void ddav_from(const Dda& d, const GridK& g, const PackK& k, DdaV& w) {
    if (k.bm) ddav_from_t<true>(d, g, k, w);
    else ddav_from_t<false>(d, g, k, w);
}
// An opaque copy: keeps the compiler from merging `a0 ? t2 : (a1 ? t2 : u)`
// into `(a0 || a1) ? t2 : u`, whose or-of-compares it turns into a select of
// booleans materialised in VGPRs (7 VALU per step in the r02e5 ISA instead of
// the second v_cndmask).
ZHD float opaque_f(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    asm("" : "+v"(x));    // not volatile: a volatile asm is a scheduling barrier (r02e8: -0.5 to -1.5%)
#endif
    return x;
}
// One Iterator.next on the packed state.  LOWM: the in-brick bits of every
// field for the walk's occupancy bricks (CROSSED: the step left its brick).
// T_EXIT = EXITED ? +inf : TC, so traceRay's break test nearest <= T_EXIT is
// EXITED || nearest <= TC (nearest is +inf or a hit t, never NaN): one
// compare and a scalar or, not a select and two compares.
#define DDAV_STEPX(S, K, LOWM, CROSSED, EXITED, TC)                                   \
    do {                                                                             \
        const float t0_ = (S).tn0, t1_ = (S).tn1, t2_ = (S).tn2;                     \
        const bool b01_ = t0_ < t1_, b02_ = t0_ < t2_, b12_ = t1_ < t2_;             \
        const bool a0_ = b01_ && b02_;                                               \
        const bool a1_ = !b01_ && b12_;                                              \
        const float tc_ = a0_ ? t0_ : (a1_ ? t1_ : t2_);                             \
        const float dt_ = a0_ ? (S).td0 : (a1_ ? (S).td1 : (S).td2);                 \
        const uint32_t fm_ = a0_ ? (K).f0 : (a1_ ? (K).f1 : (K).f2);                 \
        const uint32_t pn_ = pk_add<PK_BM>((S).pc, fm_, a0_ ? (S).d0 : (a1_ ? (S).d1 : (S).d2)); \
        (CROSSED) = (((S).pc ^ pn_) & ~(LOWM)) != 0u;                                \
        (EXITED) = (((S).pc ^ (S).pe) & fm_) == 0u;                                  \
        (TC) = tc_;                                                                  \
        const float un_ = tc_ + dt_;                                                 \
        (S).tn0 = a0_ ? un_ : t0_;                                                   \
        (S).tn1 = a1_ ? un_ : t1_;                                                   \
        (S).tn2 = a0_ ? t2_ : (a1_ ? opaque_f(t2_) : un_);    /* a2: neither */       \
        (S).pc = pn_;                                                                \
    } while (0)
// Lane masks for the park walk trip.  On the device a LaneM is the wave's
// 64-bit lane mask (a ballot, i.e. the compare result in an SGPR pair) and
// lm_sel is one v_cndmask_b32 on it, so the compiler can neither turn a
// select's condition into booleans materialised in VGPRs nor wrap a select
// in a branch (the r03k ISA of DDAV_STEPX: 4 execz branches and 8
// SGPR-to-VGPR copies per four-step trip).  On the host (the step check in
// tests/cpp/dda_skip_check.cpp) a LaneM is one lane's bool: same booleans,
// same selects.
#if defined(__HIP_DEVICE_COMPILE__)
typedef uint64_t LaneM;
__device__ __forceinline__ LaneM lm_of(bool c) { return __builtin_amdgcn_ballot_w64(c); }
__device__ __forceinline__ LaneM lm_and(LaneM a, LaneM b) { return a & b; }
__device__ __forceinline__ LaneM lm_andn(LaneM a, LaneM b) { return a & ~b; }
__device__ __forceinline__ LaneM lm_or(LaneM a, LaneM b) { return a | b; }
__device__ __forceinline__ float lm_sel(LaneM m, float t, float f) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}
__device__ __forceinline__ uint32_t lm_selu(LaneM m, uint32_t t, uint32_t f) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}
#else
typedef bool LaneM;
ZHD LaneM lm_of(bool c) { return c; }
ZHD LaneM lm_and(LaneM a, LaneM b) { return a && b; }
ZHD LaneM lm_andn(LaneM a, LaneM b) { return a && !b; }
ZHD LaneM lm_or(LaneM a, LaneM b) { return a || b; }
ZHD float lm_sel(LaneM m, float t, float f) { return m ? t : f; }
ZHD uint32_t lm_selu(LaneM m, uint32_t t, uint32_t f) { return m ? t : f; }
#endif
// DDAV_STEPX on lane masks: A0 = t0<t1 && t0<t2, A1 = !(t0<t1) && t1<t2,
// else axis 2 (DDA_STEP's booleans); FV0..FV2: the field masks (in VGPRs
// for the park walk: a select between two SGPR operands needs a copy
// first).  The core selects the step's axis quantities and updates the
// crossing ts; FM: the axis's field mask, DP: its packed cell step.
#define DDAV_STEPM_CORE(S, FV0, FV1, FV2, FM, DP, TC)                                \
    const float t0_ = (S).tn0, t1_ = (S).tn1, t2_ = (S).tn2;                         \
    const LaneM m01_ = lm_of(t0_ < t1_), m02_ = lm_of(t0_ < t2_), m12_ = lm_of(t1_ < t2_); \
    const LaneM a0_ = lm_and(m01_, m02_);                                            \
    const LaneM a1_ = lm_andn(m12_, m01_);                                           \
    const LaneM a01_ = lm_or(a0_, a1_);                                              \
    const float tc_ = lm_sel(a0_, t0_, lm_sel(a1_, t1_, t2_));                       \
    const float dt_ = lm_sel(a0_, (S).td0, lm_sel(a1_, (S).td1, (S).td2));           \
    const uint32_t FM = lm_selu(a0_, (FV0), lm_selu(a1_, (FV1), (FV2)));             \
    const uint32_t DP = lm_selu(a0_, (S).d0, lm_selu(a1_, (S).d1, (S).d2));          \
    (TC) = tc_;                                                                      \
    const float un_ = tc_ + dt_;                                                     \
    (S).tn0 = lm_sel(a0_, un_, t0_);                                                 \
    (S).tn1 = lm_sel(a1_, un_, t1_);                                                 \
    (S).tn2 = lm_sel(a01_, t2_, un_);
// EXM: the lane mask of the lanes whose step's axis is at its exit cell
#define DDAV_STEPM(S, FV0, FV1, FV2, EXM, TC)                                        \
    do {                                                                             \
        DDAV_STEPM_CORE(S, FV0, FV1, FV2, fm_, dp_, TC)                              \
        (EXM) = lm_of((((S).pc ^ (S).pe) & fm_) == 0u);                              \
        (S).pc = pk_add<PK_BM>((S).pc, fm_, dp_);                                           \
    } while (0)
// The same with DDAV_STEPX's per-lane outputs (the lane walk)
#define DDAV_STEPMB(S, FV0, FV1, FV2, LOWM, CROSSED, EXITED, TC)                     \
    do {                                                                             \
        DDAV_STEPM_CORE(S, FV0, FV1, FV2, fm_, dp_, TC)                              \
        const uint32_t pn_ = pk_add<PK_BM>((S).pc, fm_, dp_);                               \
        (CROSSED) = (((S).pc ^ pn_) & ~(LOWM)) != 0u;                                \
        (EXITED) = (((S).pc ^ (S).pe) & fm_) == 0u;                                  \
        (S).pc = pn_;                                                                \
    } while (0)
#define DDAV_SEL(D, C, A, B)                                                          \
    do {                                                                             \
        (D).tn0 = (C) ? (A).tn0 : (B).tn0; (D).tn1 = (C) ? (A).tn1 : (B).tn1;        \
        (D).tn2 = (C) ? (A).tn2 : (B).tn2; (D).td0 = (C) ? (A).td0 : (B).td0;        \
        (D).td1 = (C) ? (A).td1 : (B).td1; (D).td2 = (C) ? (A).td2 : (B).td2;        \
        (D).pc = (C) ? (A).pc : (B).pc; (D).pe = (C) ? (A).pe : (B).pe;              \
        (D).d0 = (C) ? (A).d0 : (B).d0; (D).d1 = (C) ? (A).d1 : (B).d1;              \
        (D).d2 = (C) ? (A).d2 : (B).d2;                                              \
    } while (0)

// Empty-brick skip, 4^3 bricks (occ_shift 2): the state Iterator.next would
// reach at the step that leaves the current brick, computed at once.  Axis
// a's crossings form the sequence T_a(1) = tn_a, T_a(j+1) = T_a(j) + td_a
// (the same f32 adds the DDA does); Iterator.next always takes the smallest
// head, ties to the higher axis (DDA_STEP's booleans), so the steps are the
// merge of the three sequences ordered by (t, -axis).  The brick is left by
// the first, in that order, of the brick-exit crossings E_a = T_a(m_a)
// (m_a = cells to the brick face along a), and every other axis b has then
// taken exactly the crossings T_b(j), j < m_b, that precede it.  Not used
// with a -inf/NaN sequence (neg bit 3).  EXITED: the skip left the grid
// (Iterator.next returned +inf there).  T_EXIT: the exit t of the last cell
// passed = the largest of the passed cells' exit ts (the merge is
// nondecreasing), +inf if EXITED: traceRay's break test (stage3.zig:179-182)
// fires inside the skipped cells iff nearest <= T_EXIT, and they hold no
// triangle, so the skip is exact for any nearest.
#define SKIP_AXIS(S, G, A)                                                                    \
    const bool n##A##_ = ((S).neg >> A) & 1u;                                                 \
    const uint32_t lo##A##_ = (S).c##A & ~3u;                                                 \
    const uint32_t hi##A##_ = zmin(lo##A##_ + 3u, (G).rm##A);                                  \
    const uint32_t m##A##_ = n##A##_ ? (S).c##A - lo##A##_ + 1u : hi##A##_ - (S).c##A + 1u;   \
    const bool out##A##_ = n##A##_ ? lo##A##_ == 0u : hi##A##_ == (G).rm##A;                  \
    const float T##A##1_ = (S).tn##A;                                                         \
    const float T##A##2_ = T##A##1_ + (S).td##A;                                              \
    const float T##A##3_ = T##A##2_ + (S).td##A;                                              \
    const float T##A##4_ = T##A##3_ + (S).td##A;                                              \
    const float E##A##_ = m##A##_ == 1u ? T##A##1_                                            \
                        : (m##A##_ == 2u ? T##A##2_ : (m##A##_ == 3u ? T##A##3_ : T##A##4_));
#define SKIP_COUNT(S, A, TIE)                                                                 \
    uint32_t k##A##_ = 0;                                                                     \
    k##A##_ += (1u < m##A##_ && (T##A##1_ < ex_ || (T##A##1_ == ex_ && (TIE)))) ? 1u : 0u;     \
    k##A##_ += (2u < m##A##_ && (T##A##2_ < ex_ || (T##A##2_ == ex_ && (TIE)))) ? 1u : 0u;     \
    k##A##_ += (3u < m##A##_ && (T##A##3_ < ex_ || (T##A##3_ == ex_ && (TIE)))) ? 1u : 0u;     \
    k##A##_ = x##A##_ ? m##A##_ : k##A##_;                                                    \
    (S).tn##A = k##A##_ == 0u ? T##A##1_                                                      \
              : (k##A##_ == 1u ? T##A##2_                                                     \
              : (k##A##_ == 2u ? T##A##3_ : (k##A##_ == 3u ? T##A##4_ : T##A##4_ + (S).td##A))); \
    (S).c##A = n##A##_ ? (S).c##A - k##A##_ : (S).c##A + k##A##_;
#define BRICK_SKIP4(S, G, EXITED, T_EXIT)                                                     \
    do {                                                                                      \
        SKIP_AXIS(S, G, 0)                                                                    \
        SKIP_AXIS(S, G, 1)                                                                    \
        SKIP_AXIS(S, G, 2)                                                                    \
        const bool x0_ = E0_ < E1_ && E0_ < E2_;                                              \
        const bool x1_ = !(E0_ < E1_) && E1_ < E2_;                                           \
        const bool x2_ = !x0_ && !x1_;                                                        \
        const float ex_ = x0_ ? E0_ : (x1_ ? E1_ : E2_);                                      \
        SKIP_COUNT(S, 0, false)                                                               \
        SKIP_COUNT(S, 1, x0_)                                                                 \
        SKIP_COUNT(S, 2, !x2_)                                                                \
        (EXITED) = x0_ ? out0_ : (x1_ ? out1_ : out2_);                                       \
        (T_EXIT) = (EXITED) ? kInf : ex_;                                                     \
        (S).lin = (S).c2 * (G).str2 + (S).c1 * (G).str1 + (S).c0;                             \
    } while (0)

// BRICK_SKIP4 on the packed state (DdaV, PackK): the primary lane walk's
// empty-brick skip.  Same merge argument: per axis a the cells left inside
// the 4^3 brick (or to the grid exit, whichever is nearer) m1_a, the
// brick-exit crossing E_a = T_a(m1_a + 1) from the same f32 adds, the exit
// axis X = the first E_a in (t, -axis) order, and every other axis takes the
// crossings T_b(j) that precede E_X in that order (ties to the higher axis,
// as Iterator.next's booleans); axis X takes m1_X + 1.  The signs come from
// the packed steps (d_a < 0 as u32 top bit).  Not used with a -inf/NaN
// crossing sequence (Dda.neg bit 3).  EXITED / TC as DDAV_STEPX: the break
// test nearest <= T_EXIT of the last skipped cell is EXITED || nearest <= TC
// (tests/cpp/dda_skip_check.cpp checks it against the cell walk).
#if defined(__HIP_DEVICE_COMPILE__)
#define ZRT_UBFE(X, O, W) __builtin_amdgcn_ubfe((X), (O), (W))
#else
#define ZRT_UBFE(X, O, W) ((W) == 0u ? 0u : (((X) >> (O)) & (0xFFFFFFFFu >> (32u - (W)))))
#endif
#define SKIPV_AXIS(S, K, A)                                                                    \
    const uint32_t c##A##_ = pack_coord((K), (S).pc, A);                                        \
    const uint32_t xn##A##_ = (uint32_t)((int32_t)(S).d##A >> 31);                              \
    const uint32_t rem##A##_ = ~(c##A##_ ^ xn##A##_) & 3u;                                      \
    const uint32_t te##A##_ = xn##A##_ ? c##A##_ : pack_coord((K), (S).pe, A) - c##A##_;        \
    const uint32_t m1##A##_ = zmin(rem##A##_, te##A##_);                                        \
    const bool out##A##_ = te##A##_ <= rem##A##_;                                               \
    const float T##A##1_ = (S).tn##A;                                                           \
    const float T##A##2_ = T##A##1_ + (S).td##A;                                                \
    const float T##A##3_ = T##A##2_ + (S).td##A;                                                \
    const float T##A##4_ = T##A##3_ + (S).td##A;                                                \
    const float E##A##_ = m1##A##_ == 0u ? T##A##1_                                             \
                        : (m1##A##_ == 1u ? T##A##2_ : (m1##A##_ == 2u ? T##A##3_ : T##A##4_));
#define SKIPV_COUNT(S, A, TIE)                                                                 \
    uint32_t k##A##_ = ((T##A##1_ < ex_ || (T##A##1_ == ex_ && (TIE))) ? 1u : 0u) +             \
                       ((T##A##2_ < ex_ || (T##A##2_ == ex_ && (TIE))) ? 1u : 0u) +             \
                       ((T##A##3_ < ex_ || (T##A##3_ == ex_ && (TIE))) ? 1u : 0u);              \
    k##A##_ = x##A##_ ? m1##A##_ + 1u : k##A##_;                                                \
    (S).tn##A = k##A##_ == 0u ? T##A##1_                                                        \
              : (k##A##_ == 1u ? T##A##2_                                                       \
              : (k##A##_ == 2u ? T##A##3_ : (k##A##_ == 3u ? T##A##4_ : T##A##4_ + (S).td##A)));
#define BRICK_SKIPV(S, K, EXITED, TC)                                                          \
    do {                                                                                       \
        SKIPV_AXIS(S, K, 0)                                                                    \
        SKIPV_AXIS(S, K, 1)                                                                    \
        SKIPV_AXIS(S, K, 2)                                                                    \
        const bool x0_ = E0_ < E1_ && E0_ < E2_;                                               \
        const bool x1_ = !(E0_ < E1_) && E1_ < E2_;                                            \
        const bool x2_ = !x0_ && !x1_;                                                         \
        const float ex_ = x0_ ? E0_ : (x1_ ? E1_ : E2_);                                       \
        SKIPV_COUNT(S, 0, false)                                                               \
        SKIPV_COUNT(S, 1, x0_)                                                                 \
        SKIPV_COUNT(S, 2, !x2_)                                                                \
        (EXITED) = x0_ ? out0_ : (x1_ ? out1_ : out2_);                                        \
        (TC) = ex_;                                                                            \
        (S).pc = pk_addn<PK_BM>(pk_addn<PK_BM>(pk_addn<PK_BM>((S).pc, (K).f0, k0_, (S).d0), (K).f1, k1_, (S).d1), (K).f2, \
                         k2_, (S).d2);                                                         \
    } while (0)

// Fast-forward of the packed walk through space known to be empty: every
// Iterator.next step whose crossing t is below TAU, as plain f32 adds per
// axis (the same adds, in the same order per axis, as the cell-by-cell
// walk).  The steps are the merge of the three crossing sequences in
// (t, -axis) order, so the crossings with t < TAU are exactly a prefix of the
// walk, and the state after them is the walk's state after that many steps.
// EXITED: one of them was the exit crossing of its axis (Iterator.next
// returned +inf there; the walk has ended).  The caller guarantees that the
// cells those steps enter hold no triangle and that nearest > TAU (so no break
// test fires among them); not used with a -inf/NaN crossing sequence
// (Dda.neg bit 3).  tests/cpp/dda_skip_check.cpp checks it step for step.
#define FF_AXIS(S, A, FA, TAU, EXITED)                                                         \
    while ((S).tn##A < (TAU)) {                                                                \
        if ((((S).pc ^ (S).pe) & (FA)) == 0u) { (EXITED) = true; break; }                     \
        (S).tn##A += (S).td##A;                                                                \
        (S).pc = pk_add<PK_BM>((S).pc, (FA), (S).d##A);                                               \
    }
#define DDAV_FF(S, F0, F1, F2, TAU, EXITED)                                                    \
    do {                                                                                       \
        (EXITED) = false;                                                                      \
        FF_AXIS(S, 0, F0, TAU, EXITED)                                                         \
        if (!(EXITED)) { FF_AXIS(S, 1, F1, TAU, EXITED) }                                      \
        if (!(EXITED)) { FF_AXIS(S, 2, F2, TAU, EXITED) }                                      \
    } while (0)

// DDAV_FF with four conditional crossings per loop trip and the selects
// branch-free (fewer exec-mask updates per crossing; same crossings, same
// state, same EXITED).
#define FF_AXIS4(S, A, FA, TAU, EXITED)                                                        \
    for (;;) {                                                                                 \
        _Pragma("unroll") for (int u_ = 0; u_ < 4; ++u_) {                                     \
            const bool go_ = (S).tn##A < (TAU) && !(EXITED);                                   \
            const bool at_ = (((S).pc ^ (S).pe) & (FA)) == 0u;                                 \
            (EXITED) = (EXITED) || (go_ && at_);                                               \
            const bool mv_ = go_ && !at_;                                                      \
            (S).tn##A = mv_ ? (S).tn##A + (S).td##A : (S).tn##A;                               \
            (S).pc = mv_ ? pk_add<PK_BM>((S).pc, (FA), (S).d##A) : (S).pc;                           \
        }                                                                                      \
        if (!((S).tn##A < (TAU)) || (EXITED)) break;                                           \
    }
#define DDAV_FF4(S, F0, F1, F2, TAU, EXITED)                                                   \
    do {                                                                                       \
        (EXITED) = false;                                                                      \
        FF_AXIS4(S, 0, F0, TAU, EXITED)                                                        \
        if (!(EXITED)) { FF_AXIS4(S, 1, F1, TAU, EXITED) }                                     \
        if (!(EXITED)) { FF_AXIS4(S, 2, F2, TAU, EXITED) }                                     \
    } while (0)

// DDAV_FF with the packed cell stepped once per axis: per axis the crossings
// below TAU as predicated f32 adds (four per loop trip) and their count n,
// then the coordinate written once (pk_setc); EXITED when n reaches past the axis's exit
// cell (FF_AXIS stops there: its crossing j is the exit one iff j - 1 cells
// remained, so EXITED iff n > cells left).  The loop stops within four
// crossings of n > left, so it runs at most left + 4 adds whatever TAU is.
// Same crossings (the adds stop at the first t >= TAU), same state, same
// EXITED as DDAV_FF; ~4 VALU per crossing instead of ~10.
#define FFN_AXIS(S, K, A, FA, TAU, EXITED)                                                     \
    {                                                                                          \
        const uint32_t c_ = pack_coordt<PK_BM>((K), (S).pc, A), e_ = pack_coordt<PK_BM>((K), (S).pe, A); \
        const uint32_t left_ = c_ > e_ ? c_ - e_ : e_ - c_;   /* cells before the exit one */  \
        uint32_t n_ = 0;                                                                       \
        while ((S).tn##A < (TAU) && n_ <= left_) {                                             \
            _Pragma("unroll") for (int u_ = 0; u_ < 4; ++u_) {                                 \
                const bool go_ = (S).tn##A < (TAU);                                            \
                (S).tn##A = go_ ? (S).tn##A + (S).td##A : (S).tn##A;                           \
                n_ += go_ ? 1u : 0u;                                                           \
            }                                                                                  \
        }                                                                                      \
        if (n_ > left_) (EXITED) = true;                                                       \
        else (S).pc = pk_setc<PK_BM>((K), (S).pc, (FA), A, c_ > e_ ? c_ - n_ : c_ + n_);       \
    }
#define DDAV_FFN(S, K, F0, F1, F2, TAU, EXITED)                                                \
    do {                                                                                       \
        (EXITED) = false;                                                                      \
        FFN_AXIS(S, K, 0, F0, TAU, EXITED)                                                     \
        if (!(EXITED)) { FFN_AXIS(S, K, 1, F1, TAU, EXITED) }                                  \
        if (!(EXITED)) { FFN_AXIS(S, K, 2, F2, TAU, EXITED) }                                  \
    } while (0)

// DDAV_FF for long jumps: per axis first a run of n crossings known to lie
// below TAU and before the exit cell -- n from a float estimate with a safety
// margin, capped by the cells left to the exit -- done as n plain adds (the
// same adds in the same order: the state is the one the cell walk reaches
// after them) and one packed-cell step of n cells, then FF_AXIS for the last
// few.  Same crossings, same state, same EXITED as DDAV_FF.
#define FFC_AXIS(S, K, A, FA, TAU, EXITED)                                                     \
    {                                                                                          \
        const float est_ = ((TAU) - (S).tn##A) / (S).td##A;                                    \
        /* a lower bound on the crossings below TAU: the n adds' rounding drifts by at most */ \
        /* n TAU 2^-24 <= 6e-5 n td while TAU < 1000 td, inside the 1e-4 n + 2 margin     */ \
        uint32_t n_ = est_ > 3.0f && (TAU) < 1000.0f * (S).td##A ? (uint32_t)(est_ * 0.9999f) - 2u : 0u; \
        const uint32_t c_ = pack_coord((K), (S).pc, A), e_ = pack_coord((K), (S).pe, A);      \
        const uint32_t left_ = c_ > e_ ? c_ - e_ : e_ - c_;   /* cells before the exit one */  \
        n_ = zmin(n_, left_);                                                                  \
        for (uint32_t k_ = 0; k_ < n_; ++k_) (S).tn##A += (S).td##A;                           \
        (S).pc = pk_addn<PK_BM>((S).pc, (FA), n_, (S).d##A);                                          \
    }                                                                                          \
    FF_AXIS(S, A, FA, TAU, EXITED)
#define DDAV_FFC(S, K, F0, F1, F2, TAU, EXITED)                                                \
    do {                                                                                       \
        (EXITED) = false;                                                                      \
        FFC_AXIS(S, K, 0, F0, TAU, EXITED)                                                     \
        if (!(EXITED)) { FFC_AXIS(S, K, 1, F1, TAU, EXITED) }                                  \
        if (!(EXITED)) { FFC_AXIS(S, K, 2, F2, TAU, EXITED) }                                  \
    } while (0)

// Select of the park kernel's pair refill (render.hip): position of the r-th
// (from 0) set bit of m, r < popcount(m).  The byte holding it comes from
// three prefix popcounts, its position within the byte from a 2 KB LDS table
// (sel8[byte * 8 + rank], filled with SEL8_ENTRY).  ~20 VALU + one LDS read
// against ~35 dependent VALU for a binary search over the halves' popcounts
// (r03v: cfg3 +0.7%, cfg5 +0.6%).  tests/cpp/select_check.cpp checks it
// against a bit loop on the host.
// A macro rather than a function: as a call the table fill reshuffles the park
// kernel's register allocation (same instructions, other registers).
#define SEL8_ENTRY(I, POS)                                                         \
    uint32_t POS = 0;                                                              \
    {                                                                              \
        uint32_t m_ = (I) >> 3, r_ = (I) & 7u;                                     \
        for (uint32_t k_ = 0; k_ < 8; ++k_)                                        \
            if ((m_ >> k_) & 1u) { if (r_ == 0) { POS = k_; break; } --r_; }       \
    }
ZHD uint32_t select_bit(const uint8_t* sel8, uint32_t m, uint32_t r) {
    const uint32_t c0 = (uint32_t)__builtin_popcount(m & 0xFFu), c1 = (uint32_t)__builtin_popcount(m & 0xFFFFu),
                   c2 = (uint32_t)__builtin_popcount(m & 0xFFFFFFu);
    const uint32_t k = (r >= c0 ? 1u : 0u) + (r >= c1 ? 1u : 0u) + (r >= c2 ? 1u : 0u);
    // (the bits below byte k counted again rather than picked from c0..c2:
    // the pick compiled to three nested exec-mask branches, r05aq ISA)
    const uint32_t below = (uint32_t)__builtin_popcount(m & ((1u << (8u * k)) - 1u));
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t byte = __builtin_amdgcn_ubfe(m, 8u * k, 8u);
#else
    const uint32_t byte = (m >> (8u * k)) & 0xFFu;
#endif
    return 8u * k + sel8[byte * 8u + (r - below)];
}

}  // namespace zrt
