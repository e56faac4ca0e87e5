// zrt_math.h -- f32 math of the render hot path, shared by the host grid
// build (geometry.cpp) and the CDNA4 kernels (render.hip).
//
// Semantics follow the reference exactly (file:line per function) so that the
// GPU image is bit-identical to the CPU oracle's build-mode image:
//   * compiled with -ffp-contract=off: Zig never contracts a*b+c;
//   * every @reduce(.Add) is evaluated left to right (ordered LLVM reduction);
//   * @min/@max are minnum/maxnum (fminf/fmaxf), division and sqrt are
//     correctly rounded (hipcc default), normalize multiplies by 1/len;
//   * std.math.lerp is @mulAdd -> fmaf.
#pragma once

#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define ZHD __host__ __device__ __forceinline__
#else
#define ZHD inline
#endif

namespace zrt {

constexpr float kInf = __builtin_inff();

struct v3 { float x, y, z; };
ZHD v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
ZHD v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
ZHD v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
ZHD v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
ZHD v3 divv(v3 a, v3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
ZHD v3 scale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
ZHD v3 vmin(v3 a, v3 b) { return mk(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
ZHD v3 vmax(v3 a, v3 b) { return mk(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
ZHD float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }      // linalg.zig:190
ZHD float length(v3 a) { return sqrtf(dot(a, a)); }                             // linalg.zig:119
ZHD v3 normalize(v3 a) { return scale(a, 1.0f / length(a)); }                  // linalg.zig:123
ZHD v3 cross(v3 a, v3 b) {                                                      // linalg.zig:173
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
ZHD v3 vabs(v3 a) { return mk(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
ZHD v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

// @intFromFloat f32 -> u32 / i32, defined (saturating) where the reference
// is UB; the oracle uses the same definition (oracle/zrt_oracle.c f2u/f2i).
// Written as selects around one in-range conversion (4294967040 and
// 2147483520 are the largest floats below 2^32 and 2^31): with early returns
// the compiler nested three execz branches around every conversion.
ZHD uint32_t f2u(float f) {
    const uint32_t c = (uint32_t)fminf(fmaxf(f, 0.0f), 4294967040.0f);
    const uint32_t s = f >= 4294967296.0f ? 0xFFFFFFFFu : c;
    return f > -1.0f ? s : 0u;
}
ZHD int32_t f2i(float f) {
    const int32_t c = (int32_t)fminf(fmaxf(f, -2147483648.0f), 2147483520.0f);
    const int32_t s = f >= 2147483648.0f ? 2147483647 : c;
    return f != f ? 0 : s;
}

// ---- Bbox / Grid (linalg.zig:294-469) ------------------------------------
struct Bbox { v3 min, max; };
struct Grid { Bbox bbox; uint32_t res[3]; v3 cell_size; };

// linalg.zig:324-349
ZHD bool bbox_ray(const Bbox& b, v3 o, v3 d, float* t) {
    const bool sx = d.x < 0.0f, sy = d.y < 0.0f, sz = d.z < 0.0f;
    const v3 lo = mk(sx ? b.max.x : b.min.x, sy ? b.max.y : b.min.y, sz ? b.max.z : b.min.z);
    const v3 hi = mk(sx ? b.min.x : b.max.x, sy ? b.min.y : b.max.y, sz ? b.min.z : b.max.z);
    const v3 mn = divv(sub(lo, o), d);
    const v3 mx = divv(sub(hi, o), d);
    float tmin = mn.x, tmax = mx.x;
    if ((tmin > mx.y) || (tmax < mn.y)) return false;
    tmin = fmaxf(tmin, mn.y);
    tmax = fminf(tmax, mx.y);
    if ((tmin > mx.z) || (tmax < mn.z)) return false;
    tmin = fmaxf(tmin, mn.z);
    *t = tmin;
    return true;
}

ZHD Grid grid_init(Bbox b, const uint32_t res[3]) {                              // linalg.zig:412
    Grid g;
    g.bbox = b;
    g.res[0] = res[0]; g.res[1] = res[1]; g.res[2] = res[2];
    g.cell_size = divv(sub(b.max, b.min), mk((float)res[0], (float)res[1], (float)res[2]));
    return g;
}
ZHD void grid_cell_idx(const Grid& g, v3 p, uint32_t out[3]) {                   // linalg.zig:424
    const v3 q = divv(sub(p, g.bbox.min), g.cell_size);
    const uint32_t c[3] = {f2u(q.x), f2u(q.y), f2u(q.z)};
    for (int i = 0; i < 3; ++i) out[i] = c[i] < g.res[i] - 1u ? c[i] : g.res[i] - 1u;
}
ZHD Bbox grid_cell_bbox(const Grid& g, uint32_t x, uint32_t y, uint32_t z) {     // linalg.zig:433
    Bbox b;
    b.min = add(g.bbox.min, mul(g.cell_size, mk((float)x, (float)y, (float)z)));
    b.max = add(b.min, g.cell_size);
    return b;
}

// ---- SAT triangle/AABB (linalg.zig:500-563) ------------------------------
ZHD bool sat_axis(v3 v0, v3 v1, v3 v2, v3 ext, v3 axis) {
    const float p0 = dot(v0, axis), p1 = dot(v1, axis), p2 = dot(v2, axis);
    // dot((1,0,0), axis) literally: 1*ax + 0*ay + 0*az (NaN axes stay NaN)
    const float r = ext.x * fabsf(dot(mk(1, 0, 0), axis)) +
                    ext.y * fabsf(dot(mk(0, 1, 0), axis)) +
                    ext.z * fabsf(dot(mk(0, 0, 1), axis));
    const float maxp = fmaxf(p0, fmaxf(p1, p2));
    const float minp = fminf(p0, fminf(p1, p2));
    return !(fmaxf(-maxp, minp) > r);
}
ZHD bool tri_aabb(v3 t0, v3 t1, v3 t2, const Bbox& b) {
    const v3 center = scale(add(b.max, b.min), 0.5f);
    const v3 ext = scale(sub(b.max, b.min), 0.5f);
    const v3 a = sub(t0, center), bb = sub(t1, center), c = sub(t2, center);
    const v3 ab = normalize(sub(bb, a));
    const v3 bc = normalize(sub(c, bb));
    const v3 ca = normalize(sub(a, c));
    if (!sat_axis(a, bb, c, ext, mk(0.0f, -ab.z, ab.y))) return false;
    if (!sat_axis(a, bb, c, ext, mk(0.0f, -bc.z, bc.y))) return false;
    if (!sat_axis(a, bb, c, ext, mk(0.0f, -ca.z, ca.y))) return false;
    if (!sat_axis(a, bb, c, ext, mk(ab.z, 0.0f, -ab.x))) return false;
    if (!sat_axis(a, bb, c, ext, mk(bc.z, 0.0f, -bc.x))) return false;
    if (!sat_axis(a, bb, c, ext, mk(ca.z, 0.0f, -ca.x))) return false;
    if (!sat_axis(a, bb, c, ext, mk(-ab.y, ab.x, 0.0f))) return false;
    if (!sat_axis(a, bb, c, ext, mk(-bc.y, bc.x, 0.0f))) return false;
    if (!sat_axis(a, bb, c, ext, mk(-ca.y, ca.x, 0.0f))) return false;
    if (!sat_axis(a, bb, c, ext, mk(1, 0, 0))) return false;
    if (!sat_axis(a, bb, c, ext, mk(0, 1, 0))) return false;
    if (!sat_axis(a, bb, c, ext, mk(0, 0, 1))) return false;
    if (!sat_axis(a, bb, c, ext, cross(ab, bc))) return false;
    return true;
}

// ---- deterministic f64 exp / log ----------------------------------------
// ONE definition shared with the oracle (oracle/zrt_oracle.c orc_exp/orc_log,
// restated there independently): used for the ziggurat tables and pdf
// (Zig std ziggurat.zig NormDist) and for toRGB's pow.
ZHD double dbits(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
ZHD uint64_t bitsd(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }

ZHD double det_exp(double x) {
    const double LN2_HI = 6.93147180369123816490e-01;
    const double LN2_LO = 1.90821492927058770002e-10;
    const double INV_LN2 = 1.44269504088896338700e+00;
    if (x != x) return x;
    if (x > 709.782712893384) return (double)kInf;
    if (x < -745.1332191019412) return 0.0;
    const double kd = floor(x * INV_LN2 + 0.5);
    int k = (int)kd;
    const double r = (x - kd * LN2_HI) - kd * LN2_LO;
    double p = 1.0 / 6227020800.0;
    p = p * r + 1.0 / 479001600.0;
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    if (k > 1023) { p *= dbits((uint64_t)(1023 + 1023) << 52); k -= 1023; }
    if (k < -1022) { p *= dbits((uint64_t)(1023 - 1000) << 52); k += 1000; }
    if (k < -1022) { p *= dbits((uint64_t)(1023 - 1000) << 52); k += 1000; }
    return p * dbits((uint64_t)(k + 1023) << 52);
}

ZHD double det_log(double x) {
    const double LN2_HI = 6.93147180369123816490e-01;
    const double LN2_LO = 1.90821492927058770002e-10;
    if (x != x) return x;
    if (x < 0.0) return dbits(0x7ff8000000000000ull);
    if (x == 0.0) return -(double)kInf;
    if (x == (double)kInf) return x;
    uint64_t b = bitsd(x);
    int e = (int)((b >> 52) & 0x7ff);
    if (e == 0) {
        x *= dbits((uint64_t)(1023 + 54) << 52);
        b = bitsd(x);
        e = (int)((b >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    double m = dbits((b & 0x000FFFFFFFFFFFFFull) | ((uint64_t)1023 << 52));
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s;
    double p = 1.0 / 23.0;
    p = p * z + 1.0 / 21.0;
    p = p * z + 1.0 / 19.0;
    p = p * z + 1.0 / 17.0;
    p = p * z + 1.0 / 15.0;
    p = p * z + 1.0 / 13.0;
    p = p * z + 1.0 / 11.0;
    p = p * z + 1.0 / 9.0;
    p = p * z + 1.0 / 7.0;
    p = p * z + 1.0 / 5.0;
    p = p * z + 1.0 / 3.0;
    const double lm = 2.0 * s + (2.0 * s) * (z * p);
    const double ed = (double)e;
    return ed * LN2_HI + (ed * LN2_LO + lm);
}

// std.math.pow(f32, x, 1/2.2) as called by toRGB (linalg.zig:66-72,153):
// x>0 finite -> exp(y*log(x)); the Zig/Go special cases otherwise.
ZHD float pow_gamma(float x, float y) {
    if (x == 1.0f) return 1.0f;
    if (x != x) return x;
    if (x == 0.0f) return 0.0f;                        // y > 0, not an odd integer
    if (x == kInf || x == -kInf) return kInf;          // pow(-inf,y) = pow(-0,-y) = +inf
    if (x < 0.0f) return __builtin_nanf("");
    return (float)det_exp((double)y * det_log((double)x));
}

// linalg.zig:150-159 toRGB: clamp has no lower bound (quirk, :58-60)
ZHD void to_rgb(v3 c, uint8_t out[3]) {
    const float g = 0.454545454545454545f;
    const float r[3] = {pow_gamma(c.x, g), pow_gamma(c.y, g), pow_gamma(c.z, g)};
    for (int i = 0; i < 3; ++i) out[i] = (uint8_t)f2u(fminf(r[i], fmaxf(0.0f, 0.999999f)) * 256.0f);
}

// ---- RNG ------------------------------------------------------------------
// Counter-based stream keyed by (seed, pixel, sample): SplitMix64 started at
// mix64(path_id ^ mix64(seed + golden)).  Draw ORDER per sample is the
// reference's (stage3.zig:238 jx, jy; per bounce :207 U, :214 3 x floatNorm).
ZHD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
constexpr uint64_t kGolden = 0x9e3779b97f4a7c15ull;
ZHD uint64_t path_key(uint64_t seed, uint32_t pixel, uint32_t sample) {
    return mix64((((uint64_t)pixel << 16) | (uint64_t)sample) ^ mix64(seed + kGolden));
}
struct Rng {
    uint64_t s;
    ZHD uint64_t next() { s += kGolden; return mix64(s); }
};
ZHD int clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }
// Zig 0.11 Random.float(f32)
ZHD float rng_float(Rng& r) {
    const uint64_t rnd = r.next();
    uint32_t lz = (uint32_t)clz64(rnd);
    if (lz >= 41) {
        lz = 41 + (uint32_t)clz64(r.next());
        if (lz == 41 + 64) lz += (uint32_t)__builtin_clz((uint32_t)r.next() | 0x7FFu);
    }
    const uint32_t bits = ((126u - lz) << 23) | ((uint32_t)rnd & 0x7FFFFFu);
    float f; memcpy(&f, &bits, 4); return f;
}
// Zig 0.11 Random.float(f64)
ZHD double rng_double(Rng& r) {
    const uint64_t rnd = r.next();
    uint64_t lz = (uint64_t)clz64(rnd);
    if (lz >= 12) {
        lz = 12;
        for (;;) {
            const uint64_t addl = (uint64_t)clz64(r.next());
            lz += addl;
            if (addl != 64) break;
            if (lz >= 1022) { lz = 1022; break; }
        }
    }
    return dbits(((1022 - lz) << 52) | (rnd & 0xFFFFFFFFFFFFFull));
}
constexpr double kNormR = 3.6541528853610088;
constexpr double kNormV = 0.00492867323399;
ZHD double norm_pdf(double x) { return det_exp(-x * x / 2.0); }
// ziggurat.zig next_f64(NormDist); zx/zf: 257-entry tables (zig_tables()).
ZHD double rng_norm64(Rng& r, const double* zx, const double* zf) {
    for (;;) {
        const uint64_t bits = r.next();
        const unsigned i = (unsigned)(bits & 0xff);
        const double u = dbits(((uint64_t)(0x3ff + 1) << 52) | (bits >> 12)) - 3.0;
        const double x = u * zx[i];
        if (fabs(x) < zx[i + 1]) return x;
        if (i == 0) {
            double xx = 1.0, yy = 0.0;
            while (-2.0 * yy < xx * xx) {
                xx = det_log(rng_double(r)) / kNormR;
                yy = det_log(rng_double(r));
            }
            return u < 0.0 ? xx - kNormR : kNormR - xx;
        }
        if (zf[i + 1] + (zf[i] - zf[i + 1]) * rng_double(r) < norm_pdf(x)) return x;
    }
}

// ---- Moller-Trumbore, back faces culled (linalg.zig:696-722) --------------
#ifndef ZRT_MT_RCP
#define ZRT_MT_RCP 1
#endif
// 1.0f / det, correctly rounded.  On the device: the compiler's IEEE f32
// division sequence (rcp, then the fma refinements) without its
// v_div_scale / v_div_fmas / v_div_fixup steps, which are identities for a
// numerator of 1 and 2^-95 < |det| < 2^126 (no scaling, no special value):
// 7 VALU instead of 11 (r05am).  A det below 1e-8 is rejected whatever this
// returns, and |det| <= |e1| |e2| |d| < 2^126 for the kernels' unit
// directions when every edge component is below 2^62 (NaN aside, which both
// forms propagate).  Scenes with a larger or infinite edge component render
// through the IEEE instantiation (IEEE = true: the plain division, every
// operand) that the contexts select at creation (zrt_context::mt_exact):
// a guard per wave instead split the test loop and spilled.  The device
// probe ZRT_PROBE_RECIP_SWEEP checks the short form against the division
// on every float of the domain (tests/test_gpu_parity.py).
template <bool IEEE = false>
ZHD float mt_inv_det(float det) {
#if defined(__HIP_DEVICE_COMPILE__) && ZRT_MT_RCP
    if (!IEEE) {
        const float r = __builtin_amdgcn_rcpf(det);
        const float f1 = __builtin_fmaf(__builtin_fmaf(-det, r, 1.0f), r, r);
        const float f3 = __builtin_fmaf(__builtin_fmaf(-det, f1, 1.0f), f1, f1);
        return __builtin_fmaf(__builtin_fmaf(-det, f3, 1.0f), f1, f3);
    }
#endif
    return 1.0f / det;
}
// a / b, correctly rounded, from y = RN(1 / b): Markstein's correction
// q0 = a y, r = a - b q0 (exact, one fma), q = q0 + r y.  The IEEE quotient bit
// for bit when b and a / b are normal and r is representable: checked on the
// device for every pair of significands (a, b in [1, 2):
// ZRT_PROBE_QUOT_SWEEP), which extends by exact power-of-two scaling to
// 2^-64 <= |a| <= 2^64 and 2^-32 <= |b| <= 2^32 (quot_operands_ok; the
// remainder stays exact down there), and a = +-0 (q0 is the signed zero the
// division gives, the copysign keeps it: r y may add a zero of the other
// sign).  NaN operands give NaN either way.
ZHD float quot_rn(float a, float b, float y) {
    const float q0 = a * y;
    const float r = fmaf(-b, q0, a);
    return copysignf(fmaf(r, y, q0), q0);
}
// 1.0f / x, correctly rounded, for every x: the short reciprocal (equal to
// the division for every normal |x| <= 2^126, the r06b sweep), the division
// itself for zero, subnormal, larger, infinite or NaN x (a branch that a
// normalize of a ray direction never takes).
ZHD float recip_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__) && ZRT_MT_RCP
    float r = mt_inv_det<false>(x);
    if (__builtin_expect(!(fabsf(x) >= 0x1p-126f && fabsf(x) <= 0x1p126f), 0)) r = 1.0f / x;
    return r;
#else
    return 1.0f / x;
#endif
}
// normalize (linalg.zig:123) with recip_rn: the same vector bit for bit
ZHD v3 normalize_rn(v3 a) { return scale(a, recip_rn(length(a))); }
template <bool IEEE = false>
ZHD bool tri_ray(v3 v0, v3 e1, v3 e2, v3 o, v3 d, float* t, float* uu, float* vv) {
    const v3 pvec = cross(d, e2);
    const float det = dot(e1, pvec);
    if (det < 0.00000001f) return false;
    const float inv_det = mt_inv_det<IEEE>(det);
    const v3 tvec = sub(o, v0);
    const float u = dot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return false;
    const v3 qvec = cross(tvec, e1);
    const float v = dot(d, qvec) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return false;
    *t = dot(e2, qvec) * inv_det;
    *uu = u;
    *vv = v;
    return true;
}

// tri_ray without early returns, for lanes that test different triangles
// side by side (wf_park_kernel's test rounds): every quantity is evaluated by
// the same f32 operations in the same order and the rejections are combined
// at the end, so for an accepted hit t, u and v are tri_ray's bit for bit, and
// the hit/miss answer is tri_ray's for every input (a NaN passes a rejection
// here exactly when tri_ray's `<` / `>` against it lets it continue).
template <bool IEEE = false>
ZHD bool tri_ray_flat(v3 v0, v3 e1, v3 e2, v3 o, v3 d, float* t, float* uu, float* vv) {
    const v3 pvec = cross(d, e2);
    const float det = dot(e1, pvec);
    const float inv_det = mt_inv_det<IEEE>(det);
    const v3 tvec = sub(o, v0);
    const float u = dot(tvec, pvec) * inv_det;
    const v3 qvec = cross(tvec, e1);
    const float v = dot(d, qvec) * inv_det;
    *t = dot(e2, qvec) * inv_det;
    *uu = u;
    *vv = v;
    const bool rej = (det < 0.00000001f) | (u < 0.0f) | (u > 1.0f) | (v < 0.0f) | (u + v > 1.0f);
    return !rej;
}

// ---- textures (stage3.zig:94-121) -----------------------------------------
ZHD float tex_frac(float v) { return fabsf(v - truncf(v)); }
ZHD int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }
// @mod(a, b) for b > 0 (texture extents).  On the device, a in [0, b) --
// texture coordinates inside the image -- returns a, and |a| < 2^21 takes a
// float quotient: a * rcp(b) is within 0.5 of a / b there (rcp's 1-ulp
// error times |a / b| < 2^21), so its floor is the quotient or one off, and
// one correction each way gives the residue exactly.  The rest takes the
// integer division (~25 VALU with quarter-rate multiplies) in a call: inline,
// its registers made the primary kernel spill inside its cell walk, and
// without the [0, b) return cfg3 lost 3% (r03t/r03u).
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __noinline__ int32_t fmod_i_slow(int32_t a, int32_t b) {
    const int32_t r = a % b;
    return r < 0 ? r + b : r;
}
#endif
ZHD int32_t fmod_i(int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if ((uint32_t)a < (uint32_t)b) return a;
    if (b > 0 && a > -(1 << 21) && a < (1 << 21)) {
        const int32_t q = (int32_t)floorf((float)a * __builtin_amdgcn_rcpf((float)b));
        int32_t r = a - q * b;
        r = r < 0 ? r + b : r;
        return r >= b ? r - b : r;
    }
    return fmod_i_slow(a, b);
#else
    const int32_t r = a % b;
    return r < 0 ? r + b : r;
#endif
}
ZHD float lerpf(float a, float b, float t) { return fmaf(b - a, t, a); }       // @mulAdd

struct TexCoords { int32_t i11, i21, i12, i22; float fu, fv; };
ZHD TexCoords tex_coords(int32_t w_int, int32_t h_int, int32_t u_min, int32_t u_max,
                         int32_t v_min, int32_t v_max, float u, float v) {
    const int32_t ui = f2i(floorf((float)w_int * u));
    const int32_t vi = f2i(floorf((float)h_int * v));
    const int32_t ui1 = (int32_t)((uint32_t)ui + 1u), vi1 = (int32_t)((uint32_t)vi + 1u);
    const int32_t x1 = fmod_i(clampi(ui, u_min, u_max), w_int);
    const int32_t y1 = fmod_i(clampi(vi, v_min, v_max), h_int);
    const int32_t x2 = fmod_i(clampi(ui1, u_min, u_max), w_int);
    const int32_t y2 = fmod_i(clampi(vi1, v_min, v_max), h_int);
    TexCoords c;
    c.i11 = y1 * w_int + x1; c.i21 = y1 * w_int + x2;
    c.i12 = y2 * w_int + x1; c.i22 = y2 * w_int + x2;
    c.fu = tex_frac(u); c.fv = tex_frac(v);
    return c;
}
ZHD float bilerp(float p11, float p21, float p12, float p22, float fu, float fv) {
    return lerpf(lerpf(p11, p21, fu), lerpf(p12, p22, fu), fv);
}

// stage3.zig:144-150
ZHD v3 env_color(v3 d) {
    const float t = 0.5f * (d.y + 1.0f);
    return add(scale(mk(1, 1, 1), 1.0f - t), scale(mk(0.5f, 0.7f, 1.0f), t));
}

}  // namespace zrt
