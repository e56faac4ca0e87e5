// Escape table for the park walk (render.hip wf_park_kernel), shared by the
// device build kernel and the host check tests/cpp/escape_check.cpp.
//
// traceRay (stage3.zig:152-185) tests the triangles of every cell the DDA
// visits until nearest <= t_next_crossing.  If no cell after the current one
// holds a triangle, nothing after it can change the result: the walk may
// stop there with the nearest hit so far (a miss stays +inf).  The table
// proves that conservatively, per 4^3 brick B and direction bin:
//   * a bin is a cone of directions: the dominant axis a and its sign (the
//     cube face), and the slopes u = d_b / |d_a|, v = d_c / |d_a| of the
//     other two axes in one of kEscBins x kEscBins cells of [-1, 1]^2;
//   * the bit is set when the region swept by every ray that starts in B with
//     a direction in the cone (its slopes widened by kEscEps), dilated by one
//     cell on every side, holds no occupied cell of the grid.
// A DDA walk is the ray's line up to f32 rounding, far below a cell, so every
// cell it visits after one in B lies in that region: a set bit means every
// later cell is empty.  Rays whose crossing sequences start at -inf / NaN (a
// zero direction component on a cell boundary, Dda.neg bit 3) never use it.
//
// The region is tested slab by slab along a: the cells of slab i that the
// cone can reach form a rectangle in the other two axes, and a summed-area
// table of cell occupancy answers "any occupied cell in it" with 8 loads.
#pragma once
#include <stdint.h>

#include "zrt_math.h"

namespace zrt {

#ifndef ZRT_ESC_BINS
#define ZRT_ESC_BINS 8
#endif
constexpr uint32_t kEscBins = ZRT_ESC_BINS;                    // per face axis
constexpr uint32_t kEscNBin = 6 * kEscBins * kEscBins;         // 384 bins (r04q: 8 x 8 per face vs 4 x 4: cfg3 +0.9%)
constexpr uint32_t kEscWords = kEscNBin <= 128 ? 4 : (kEscNBin + 31) / 32;   // u32 words per brick
constexpr double kEscEps = 1e-3;                               // slope margin of a bin's cone

// The bin of a direction (any consistent face choice on |d_a| ties: both
// faces' cones hold the direction, their slopes reach +-1 + kEscEps).
ZHD uint32_t esc_dir_bin(v3 d) {
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    uint32_t a;
    float m, u, v;
    // (the slopes need not be exact: a bin's cone is kEscEps wider than its
    // cell, far more than the reciprocal's error)
#if defined(__HIP_DEVICE_COMPILE__)
#define ZRT_ESC_RCP(x) __builtin_amdgcn_rcpf(x)
#else
#define ZRT_ESC_RCP(x) (1.0f / (x))
#endif
    if (ax >= ay && ax >= az) { a = 0; m = d.x; const float r = ZRT_ESC_RCP(ax); u = d.y * r; v = d.z * r; }
    else if (ay >= az) { a = 1; m = d.y; const float r = ZRT_ESC_RCP(ay); u = d.x * r; v = d.z * r; }
    else { a = 2; m = d.z; const float r = ZRT_ESC_RCP(az); u = d.x * r; v = d.y * r; }
#undef ZRT_ESC_RCP
    const uint32_t f = 2u * a + (m < 0.0f ? 1u : 0u);
    const float fb = (float)kEscBins;
    const uint32_t iu = (uint32_t)fminf(fmaxf((u + 1.0f) * 0.5f * fb, 0.0f), fb - 1.0f);
    const uint32_t iv = (uint32_t)fminf(fmaxf((v + 1.0f) * 0.5f * fb, 0.0f), fb - 1.0f);
    return (f * kEscBins + iu) * kEscBins + iv;
}

// Summed-area table of cell occupancy, (res0 + 1) x (res1 + 1) x (res2 + 1):
// S[z][y][x] = occupied cells in [0, x) x [0, y) x [0, z).
struct EscSat {
    const uint32_t* s;
    uint32_t n0, n01;      // res0 + 1, (res0 + 1) (res1 + 1)
};
// occupied cells in the inclusive cell box [x0, x1] x [y0, y1] x [z0, z1]
ZHD uint32_t esc_box(const EscSat& S, uint32_t x0, uint32_t x1, uint32_t y0, uint32_t y1, uint32_t z0, uint32_t z1) {
    const uint64_t X0 = x0, X1 = x1 + 1ull, Y0 = (uint64_t)y0 * S.n0, Y1 = (uint64_t)(y1 + 1) * S.n0;
    const uint64_t Z0 = (uint64_t)z0 * S.n01, Z1 = (uint64_t)(z1 + 1) * S.n01;
    return S.s[Z1 + Y1 + X1] - S.s[Z1 + Y1 + X0] - S.s[Z1 + Y0 + X1] + S.s[Z1 + Y0 + X0] - S.s[Z0 + Y1 + X1] +
           S.s[Z0 + Y1 + X0] + S.s[Z0 + Y0 + X1] - S.s[Z0 + Y0 + X0];
}

// The bit of brick (bx, by, bz) and `bin` (see the header comment).
// A grid with a zero-extent (or non-finite) axis -- every triangle in one
// plane, Grid.init's cell_size 0 (linalg.zig:412-441) -- has walks whose
// crossings on that axis do not advance t, which the cell-unit geometry below
// does not model: such grids get no proof (no escape bit, no frustum bound).
ZHD bool esc_cells_regular(const float cs[3]) {
    return cs[0] > 0.0f && cs[1] > 0.0f && cs[2] > 0.0f && cs[0] < kInf && cs[1] < kInf && cs[2] < kInf;
}

ZHD bool esc_compute(const EscSat& S, const uint32_t res[3], const float cs[3], uint32_t bx, uint32_t by,
                     uint32_t bz, uint32_t bin) {
    if (!esc_cells_regular(cs)) return false;
    const uint32_t fc = bin / (kEscBins * kEscBins), iu = (bin / kEscBins) % kEscBins, iv = bin % kEscBins;
    const int a = (int)(fc / 2u), sg = (fc & 1u) ? -1 : 1;
    const int b = a == 0 ? 1 : 0, c = a == 2 ? 1 : 2;
    const double nb = (double)kEscBins;
    const double u0 = -1.0 + 2.0 * iu / nb - kEscEps, u1 = -1.0 + 2.0 * (iu + 1) / nb + kEscEps;
    const double v0 = -1.0 + 2.0 * iv / nb - kEscEps, v1 = -1.0 + 2.0 * (iv + 1) / nb + kEscEps;
    const uint32_t B[3] = {bx, by, bz};
    double lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = 4.0 * B[k];
        hi[k] = fmin(4.0 * B[k] + 4.0, (double)res[k]);
    }
    // a cell-unit step along a moves cs_a / cs_b cells along b
    const double kb = (double)cs[a] / (double)cs[b], kc = (double)cs[a] / (double)cs[c];
    const int ra = (int)res[a];
    for (int i = sg > 0 ? (int)lo[a] : (int)hi[a] - 1; i >= 0 && i < ra; i += sg) {
        double smin, smax;                      // a-distance from the brick to slab i
        if (sg > 0) { smin = fmax(0.0, i - hi[a]); smax = fmax(0.0, i + 1.0 - lo[a]); }
        else { smin = fmax(0.0, lo[a] - (i + 1.0)); smax = fmax(0.0, hi[a] - i); }
        const double ylo = lo[b] + kb * fmin(smin * u0, smax * u0), yhi = hi[b] + kb * fmax(smin * u1, smax * u1);
        const double zlo = lo[c] + kc * fmin(smin * v0, smax * v0), zhi = hi[c] + kc * fmax(smin * v1, smax * v1);
        // the cells the interval touches, one more on each side
        const double yf0 = floor(ylo) - 1.0, yf1 = ceil(yhi), zf0 = floor(zlo) - 1.0, zf1 = ceil(zhi);
        if (yf1 < 0.0 || yf0 > res[b] - 1.0 || zf1 < 0.0 || zf0 > res[c] - 1.0) {
            // the region lies beside the grid in this slab; it only moves
            // further out when neither slope range straddles 0 on that side
            const bool out_y = (yf1 < 0.0 && u1 <= 0.0) || (yf0 > res[b] - 1.0 && u0 >= 0.0);
            const bool out_z = (zf1 < 0.0 && v1 <= 0.0) || (zf0 > res[c] - 1.0 && v0 >= 0.0);
            if (out_y || out_z) break;
            continue;
        }
        const uint32_t y0 = (uint32_t)fmax(0.0, yf0), y1 = (uint32_t)fmin(res[b] - 1.0, yf1);
        const uint32_t z0 = (uint32_t)fmax(0.0, zf0), z1 = (uint32_t)fmin(res[c] - 1.0, zf1);
        uint32_t lo3[3], hi3[3];
        lo3[a] = hi3[a] = (uint32_t)i;
        lo3[b] = y0; hi3[b] = y1;
        lo3[c] = z0; hi3[c] = z1;
        if (esc_box(S, lo3[0], hi3[0], lo3[1], hi3[1], lo3[2], hi3[2]) != 0u) return false;
    }
    return true;
}

// Primary-ray frustum bound (the primary launch, render.hip frustum_kernel).
// Every camera ray of the pixel block [u0, u1) x [v0, v1) (pixel x + jitter,
// stage3.zig:234-238) starts at the camera origin o with direction
// normalize(llc + right u + up v): the points o + s D(u, v), s >= 0, form a
// cone over the parallelogram of D's, and its slice s in [s0, s1] is the
// convex hull of the eight corner points.  Marching slices of about two cells
// along the cone's dominant axis, the first slice whose box (dilated by one
// cell) holds an occupied cell ends the march: every point of the block's
// rays with normalized t < s0 |D|min lies in earlier, empty slices, so a walk
// may fast-forward (DDAV_FF) over every crossing below that t.  +inf: the cone
// meets no occupied cell at all, so every ray of the block misses
// (traceRay's +inf).  0: no bound (a degenerate cone).
// hi: the march goes on to the last slice [s0, s1] that holds an occupied
// cell: every point of the block's rays with t >= s1 |D|max lies in later,
// empty slices, so once the walk has tested a cell whose exit crossing is at
// or past hi no later cell can change the result (+inf: no bound).
// [ga, gb]: the longest run of at least kFrustumGapSlices empty slices
// between occupied ones, as t: every point of the block's rays with t in
// [ga, gb] lies in it (ga = s_start |D|max rounded up, gb = s_end |D|min
// rounded down), so a walk that enters a cell at a crossing in [ga, gb) may
// fast-forward over every crossing below gb (+inf, +inf: no gap).
constexpr int kFrustumGapSlices = 2;
struct FrustumBound {
    float lo, hi, ga, gb;
};
ZHD bool s_far_finite(double x) { return x * 0.0 == 0.0; }

// The block's cone: corner directions, |D| bounds, the march's slice width
// along the dominant axis and its end (frustum_bound; frustum_kernel runs the
// slices over a wave's lanes with the same arithmetic).
struct FrustumCone {
    double D[4][3];
    double dmin, dmax, s_far, ds;
    bool ok;
};
ZHD FrustumCone frustum_cone(const float bmin[3], const float bmax[3], const float cs[3], const float org[3],
                             const float llc[3], const float right[3], const float up[3], double u0, double u1,
                             double v0, double v1) {
    FrustumCone q;
    q.ok = false;
    q.dmax = 0.0;
    q.s_far = q.ds = 0.0;
    const double uu[2] = {u0, u1}, vv[2] = {v0, v1};
    double dmin = 1e300, mid[3] = {0, 0, 0};
    for (int c = 0; c < 4; ++c) {
        double n2 = 0.0;
        for (int k = 0; k < 3; ++k) {
            q.D[c][k] = (double)llc[k] + (double)right[k] * uu[c & 1] + (double)up[k] * vv[c >> 1];
            n2 += q.D[c][k] * q.D[c][k];
            mid[k] += 0.25 * q.D[c][k];
        }
        dmin = fmin(dmin, sqrt(n2));
        q.dmax = fmax(q.dmax, sqrt(n2));
    }
    // |D| over the parallelogram >= the corners' least |D| minus its diagonals
    double rl = 0.0, ul = 0.0;
    for (int k = 0; k < 3; ++k) {
        rl += (double)right[k] * right[k];
        ul += (double)up[k] * up[k];
    }
    dmin -= sqrt(rl) * (u1 - u0) + sqrt(ul) * (v1 - v0);
    q.dmin = dmin;
    if (!(dmin > 0.0) || !esc_cells_regular(cs)) return q;
    // beyond s_far every point of the cone is farther from o than any grid point
    double far2 = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double a = fabs((double)bmin[k] - org[k]), b = fabs((double)bmax[k] - org[k]);
        far2 += fmax(a, b) * fmax(a, b);
    }
    q.s_far = sqrt(far2) / dmin;
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (fabs(mid[k]) / cs[k] > fabs(mid[ax]) / cs[ax]) ax = k;
    q.ds = 2.0 * (double)cs[ax] / fmax(fabs(mid[ax]), 1e-30);
    // the march must reach s_far within its 2^16 slices
    q.ok = q.ds > 0.0 && s_far_finite(q.s_far) && (double)(1 << 16) * q.ds > q.s_far;
    return q;
}
// Slice it of the march: [it ds, it ds + ds]; whether its box (the eight
// corner points, dilated by one cell) holds an occupied cell.
ZHD bool frustum_slice(const EscSat& S, const FrustumCone& q, const uint32_t res[3], const float bmin[3],
                       const float cs[3], const float org[3], int it) {
    const double s0 = it * q.ds, s1 = s0 + q.ds;
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (int c = 0; c < 4; ++c)
        for (int k = 0; k < 3; ++k) {
            const double p0 = org[k] + s0 * q.D[c][k], p1 = org[k] + s1 * q.D[c][k];
            lo[k] = fmin(lo[k], fmin(p0, p1));
            hi[k] = fmax(hi[k], fmax(p0, p1));
        }
    uint32_t c0[3], c1[3];
    if (!esc_cells_regular(cs)) return true;                  // (no bound: frustum_cone refuses these)
    for (int k = 0; k < 3; ++k) {
        const double a = floor((lo[k] - bmin[k]) / cs[k]) - 1.0, b = floor((hi[k] - bmin[k]) / cs[k]) + 1.0;
        if (b < 0.0 || a > res[k] - 1.0) return false;
        c0[k] = (uint32_t)fmax(0.0, a);
        c1[k] = (uint32_t)fmin(res[k] - 1.0, b);
    }
    return esc_box(S, c0[0], c1[0], c0[1], c1[1], c0[2], c1[2]) != 0u;
}
// lo and hi from the first and last occupied slices (-1: none).
ZHD void frustum_finish(const FrustumCone& q, int first, int last, FrustumBound& fb) {
    if (first < 0) {
        fb.lo = kInf;
        return;
    }
    const double tl = (first * q.ds) * q.dmin, th = (last * q.ds + q.ds) * q.dmax;
    fb.lo = (float)tl;
    if ((double)fb.lo > tl) fb.lo = nextafterf(fb.lo, 0.0f);     // round down
    fb.hi = (float)th;
    if ((double)fb.hi < th) fb.hi = nextafterf(fb.hi, kInf);     // round up
}
ZHD FrustumBound frustum_bound(const EscSat& S, const uint32_t res[3], const float bmin[3], const float bmax[3],
                               const float cs[3], const float org[3], const float llc[3], const float right[3],
                               const float up[3], double u0, double u1, double v0, double v1) {
    FrustumBound fb{0.0f, kInf, kInf, kInf};
    const FrustumCone q = frustum_cone(bmin, bmax, cs, org, llc, right, up, u0, u1, v0, v1);
    if (!q.ok) return fb;                                          // no bound
    int first = -1, last = -1, gap_it = -1, best0 = 0, best1 = 0, run = 0;
    double best_len = -1.0;
    for (int it = 0; it < 1 << 16 && !(it * q.ds > q.s_far); ++it) {
        if (frustum_slice(S, q, res, bmin, cs, org, it)) {
            const double len = (it * q.ds) * q.dmin - (gap_it * q.ds) * q.dmax;
            if (first >= 0 && run >= kFrustumGapSlices && len > best_len) {
                best_len = len;
                best0 = gap_it;
                best1 = it;
            }
            if (first < 0) first = it;
            last = it;
            run = 0;
        } else {
            if (run == 0) gap_it = it;
            ++run;
        }
    }
    frustum_finish(q, first, last, fb);
    if (first >= 0 && best_len > 0.0) {
        const double ta = (best0 * q.ds) * q.dmax, tb = (best1 * q.ds) * q.dmin;
        float ga = (float)ta, gb = (float)tb;
        if ((double)ga < ta) ga = nextafterf(ga, kInf);          // round up
        if ((double)gb > tb) gb = nextafterf(gb, 0.0f);          // round down
        if (ga < gb) {
            fb.ga = ga;
            fb.gb = gb;
        }
    }
    return fb;
}

}  // namespace zrt
