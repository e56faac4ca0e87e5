/*
 * zrt_oracle.c -- CPU restatement of the reference render hot path.
 * TEST INFRASTRUCTURE ONLY (see zrt_oracle.h for scope, pinning and modes).
 *
 * Compiled with -O2 -ffp-contract=off (no FMA contraction: Zig does not
 * contract), every float literal is f32 (Zig coerces comptime floats to f32
 * before the arithmetic), every reduction is evaluated left to right
 * (@reduce(.Add) on a non-fast-math @Vector is an ordered LLVM reduction).
 */
#define _GNU_SOURCE
#include "zrt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================= */
/* Vec3 (linalg.zig:13-222)                                                 */
/* ======================================================================= */
typedef struct { float x, y, z; } v3;

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vdiv(v3 a, v3 b) { return V(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 vscale(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
/* @min/@max on floats lower to LLVM minnum/maxnum == C fminf/fmaxf */
static inline v3 vmin(v3 a, v3 b) { return V(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
static inline v3 vmax(v3 a, v3 b) { return V(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
/* linalg.zig:190 dot = @reduce(.Add, a*b), ordered */
static inline float vdot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
/* linalg.zig:119 */
static inline float vlength(v3 a) { return sqrtf(vdot(a, a)); }
/* linalg.zig:123: scale by the f32 reciprocal, not a division */
static inline v3 vnormalize(v3 a) { return vscale(a, 1.0f / vlength(a)); }
/* linalg.zig:173-178 */
static inline v3 vcross(v3 a, v3 b) {
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline v3 vabs(v3 a) { return V(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
static inline float vget(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline v3 vload(const float* p) { return V(p[0], p[1], p[2]); }

typedef struct { v3 orig, dir; } ray_t;
/* linalg.zig:284 */
static inline v3 ray_at(ray_t r, float t) { return vadd(r.orig, vscale(r.dir, t)); }

/* @intFromFloat(f32 -> u32): UB outside [0, 2^32) in ReleaseFast.  The
 * restatement defines it: truncate toward zero, (-1,0) -> 0 (what Zig
 * accepts), anything below or NaN -> 0, >= 2^32 -> UINT32_MAX.  The GPU
 * kernel implements the same definition. */
static inline uint32_t f2u(float f) {
    if (!(f > -1.0f)) return 0u;          /* NaN or <= -1 */
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    if (f < 0.0f) return 0u;
    return (uint32_t)f;
}
/* @intFromFloat(f32 -> i32) with the same saturating definition */
static inline int32_t f2i(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (int32_t)0x80000000;
    return (int32_t)f;
}

/* ======================================================================= */
/* Deterministic exp/log (f64).  Zig's std.math.pow(f32) computes           */
/* @exp(yf*@log(x)) and the ziggurat tables/pdf use exp/log in f64.  The    */
/* restatement pins ONE definition, implemented identically in the GPU      */
/* kernel, so that oracle and device agree bit for bit:                     */
/*   exp: k = floor(x/ln2 + 1/2), r = (x - k*ln2hi) - k*ln2lo, Horner       */
/*        Taylor to degree 13, scale by 2^k through the exponent bits.      */
/*   log: x = m*2^e, m in [sqrt(1/2), sqrt(2)), s = (m-1)/(m+1),            */
/*        log m = 2s(1 + z/3 + ... + z^11/23), z = s*s.                     */
/* ======================================================================= */
static const double LN2_HI = 6.93147180369123816490e-01;
static const double LN2_LO = 1.90821492927058770002e-10;
static const double INV_LN2 = 1.44269504088896338700e+00;

static inline double dbits(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static inline uint64_t bitsd(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }

double orc_exp(double x) {
    if (x != x) return x;
    if (x > 709.782712893384) return INFINITY;
    if (x < -745.1332191019412) return 0.0;
    double kd = floor(x * INV_LN2 + 0.5);
    int k = (int)kd;
    double r = (x - kd * LN2_HI) - kd * LN2_LO;
    double p = 1.0 / 6227020800.0;               /* 1/13! */
    p = p * r + 1.0 / 479001600.0;               /* 1/12! */
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

double orc_log(double x) {
    if (x != x) return x;
    if (x < 0.0) return NAN;
    if (x == 0.0) return -INFINITY;
    if (x == INFINITY) return x;
    uint64_t b = bitsd(x);
    int e = (int)((b >> 52) & 0x7ff);
    if (e == 0) { /* subnormal */
        x *= dbits((uint64_t)(1023 + 54) << 52);
        b = bitsd(x);
        e = (int)((b >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    double m = dbits((b & 0x000FFFFFFFFFFFFFull) | ((uint64_t)1023 << 52));
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double z = s * s;
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
    double lm = 2.0 * s + (2.0 * s) * (z * p);
    double ed = (double)e;
    return ed * LN2_HI + (ed * LN2_LO + lm);
}

/* Zig std.math.pow(f32, x, y) (Go-derived) special cases for the one call
 * site (toRGB, y = 1/2.2, linalg.zig:66-72,153); general branch
 * exp(yf*log(x)) evaluated with the deterministic f64 exp/log above. */
float orc_powf(float x, float y) {
    if (y == 0.0f || x == 1.0f) return 1.0f;
    if (x != x || y != y) return NAN;
    if (y == 1.0f) return x;
    float yi_f = truncf(fabsf(y));
    int y_is_int = (yi_f == fabsf(y));
    int y_odd = y_is_int && fabsf(y) < 16777216.0f && (((int64_t)yi_f) & 1);
    if (x == 0.0f) {
        if (y < 0.0f) return y_odd ? copysignf(INFINITY, x) : INFINITY;
        return y_odd ? x : 0.0f;
    }
    if (isinf(y)) {
        if (x == -1.0f) return 1.0f;
        if ((fabsf(x) < 1.0f) == (y > 0.0f)) return 0.0f;
        return INFINITY;
    }
    if (isinf(x)) {
        if (x < 0.0f) return orc_powf(1.0f / x, -y);
        return y < 0.0f ? 0.0f : INFINITY;
    }
    if (y == 0.5f) return sqrtf(x);
    if (y == -0.5f) return 1.0f / sqrtf(x);
    if (!y_is_int && x < 0.0f) return NAN;
    if (!y_is_int) {
        /* restated general branch (only reached with non-integer y here):
         * yf in (0,1): yf > 0.5 -> yf-1, yi+1, then x^yi by the frexp loop.
         * For the toRGB exponent yi = 0 and yf = y. */
        double t = (double)y * orc_log((double)x);
        return (float)orc_exp(t);
    }
    /* integer exponents: not reached by the reference hot path */
    return (float)orc_exp((double)y * orc_log((double)fabsf(x))) * ((x < 0.0f && y_odd) ? -1.0f : 1.0f);
}

/* ======================================================================= */
/* Zig std.rand (0.11): SplitMix64, Xoshiro256++, Random.float, ziggurat    */
/* ======================================================================= */
static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
#define GOLDEN 0x9e3779b97f4a7c15ull

typedef struct {
    int mode;
    uint64_t s[4];   /* xoshiro state (REF) or s[0] = splitmix counter (PATH) */
} rng_t;

static void rng_init_ref(rng_t* r, uint64_t seed) {
    /* Xoshiro256.init -> seed(): four SplitMix64.next() outputs */
    uint64_t sm = seed;
    r->mode = ORC_RNG_REF;
    for (int i = 0; i < 4; ++i) { sm += GOLDEN; r->s[i] = mix64(sm); }
}
/* Build-mode stream (the GPU's): a SplitMix64 sequence whose start is
 * keyed by (seed, pixel, sample).  Any (pixel,sample) ordering or device
 * split replays the same numbers. */
static void rng_init_path(rng_t* r, uint64_t seed, uint32_t pixel, uint32_t sample) {
    r->mode = ORC_RNG_PATH;
    uint64_t path_id = ((uint64_t)pixel << 16) | (uint64_t)sample;
    r->s[0] = mix64(path_id ^ mix64(seed + GOLDEN));
}
static inline uint64_t rng_next(rng_t* r) {
    if (r->mode == ORC_RNG_PATH) {
        r->s[0] += GOLDEN;
        return mix64(r->s[0]);
    }
    uint64_t* s = r->s;
    const uint64_t res = rotl64(s[0] + s[3], 23) + s[0];
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return res;
}
static inline int clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }

/* Random.float(f32): 23 mantissa bits + exponent from leading zeros */
static inline float rng_float(rng_t* r) {
    uint64_t rnd = rng_next(r);
    uint32_t lz = (uint32_t)clz64(rnd);
    if (lz >= 41) {
        lz = 41 + (uint32_t)clz64(rng_next(r));
        if (lz == 41 + 64) {
            uint32_t u = (uint32_t)rng_next(r) | 0x7FFu;
            lz += (uint32_t)__builtin_clz(u);
        }
    }
    uint32_t bits = ((126u - lz) << 23) | ((uint32_t)rnd & 0x7FFFFFu);
    float f; memcpy(&f, &bits, 4); return f;
}
/* Random.float(f64) */
static inline double rng_double(rng_t* r) {
    uint64_t rnd = rng_next(r);
    uint64_t lz = (uint64_t)clz64(rnd);
    if (lz >= 12) {
        lz = 12;
        for (;;) {
            uint64_t addl = (uint64_t)clz64(rng_next(r));
            lz += addl;
            if (addl != 64) break;
            if (lz >= 1022) { lz = 1022; break; }
        }
    }
    uint64_t bits = ((1022 - lz) << 52) | (rnd & 0xFFFFFFFFFFFFFull);
    return dbits(bits);
}

/* ziggurat.zig NormDist tables (ZigTableGen) */
static const double NORM_R = 3.6541528853610088;
static const double NORM_V = 0.00492867323399;
static double ZX[257], ZF[257];
static pthread_once_t zig_once = PTHREAD_ONCE_INIT;
static double norm_f(double x) { return orc_exp(-x * x / 2.0); }
static double norm_f_inv(double y) { return sqrt(-2.0 * orc_log(y)); }
static void zig_init(void) {
    ZX[0] = NORM_V / norm_f(NORM_R);
    ZX[1] = NORM_R;
    for (int i = 2; i < 256; ++i) ZX[i] = norm_f_inv(NORM_V / ZX[i - 1] + norm_f(ZX[i - 1]));
    ZX[256] = 0.0;
    for (int i = 0; i < 257; ++i) ZF[i] = norm_f(ZX[i]);
}
void orc_zig_tables(double x[257], double f[257]) {
    pthread_once(&zig_once, zig_init);
    memcpy(x, ZX, sizeof ZX);
    memcpy(f, ZF, sizeof ZF);
}
/* ziggurat.next_f64(random, NormDist) */
static double rng_norm64(rng_t* r) {
    for (;;) {
        uint64_t bits = rng_next(r);
        unsigned i = (unsigned)(bits & 0xff);
        double u = dbits(((uint64_t)(0x3ff + 1) << 52) | (bits >> 12)) - 3.0;
        double x = u * ZX[i];
        double test_x = fabs(x);
        if (test_x < ZX[i + 1]) return x;
        if (i == 0) {
            /* norm_zero_case */
            double xx = 1.0, yy = 0.0;
            while (-2.0 * yy < xx * xx) {
                xx = orc_log(rng_double(r)) / NORM_R;
                yy = orc_log(rng_double(r));
            }
            return u < 0.0 ? xx - NORM_R : NORM_R - xx;
        }
        if (ZF[i + 1] + (ZF[i] - ZF[i + 1]) * rng_double(r) < norm_f(x)) return x;
    }
}
/* Random.floatNorm(f32) = @floatCast(next_f64) */
static inline float rng_norm(rng_t* r) { return (float)rng_norm64(r); }

/* linalg.zig:140-148 (args evaluated left to right) */
static inline v3 random_unit_vector(rng_t* r) {
    float a = rng_norm(r);
    float b = rng_norm(r);
    float c = rng_norm(r);
    return vnormalize(V(a, b, c));
}

/* ======================================================================= */
/* Bbox + Grid + DDA iterator (linalg.zig:294-498)                          */
/* ======================================================================= */
typedef struct { v3 min, max; } bbox_t;
typedef struct { bbox_t bbox; uint32_t res[3]; v3 cell_size; } grid_t;
typedef struct { uint32_t cell[3], exit[3], step[3]; float t_delta[3], t_next[3]; } iter_t;

/* linalg.zig:324-349 */
static int bbox_ray(bbox_t b, ray_t ray, float* t) {
    int sx = ray.dir.x < 0.0f, sy = ray.dir.y < 0.0f, sz = ray.dir.z < 0.0f;
    v3 lo = V(sx ? b.max.x : b.min.x, sy ? b.max.y : b.min.y, sz ? b.max.z : b.min.z);
    v3 hi = V(sx ? b.min.x : b.max.x, sy ? b.min.y : b.max.y, sz ? b.min.z : b.max.z);
    v3 mn = vdiv(vsub(lo, ray.orig), ray.dir);
    v3 mx = vdiv(vsub(hi, ray.orig), ray.dir);
    float tmin = mn.x, tmax = mx.x;
    if ((tmin > mx.y) || (tmax < mn.y)) return 0;
    tmin = fmaxf(tmin, mn.y);
    tmax = fminf(tmax, mx.y);
    if ((tmin > mx.z) || (tmax < mn.z)) return 0;
    tmin = fmaxf(tmin, mn.z);
    tmax = fminf(tmax, mx.z);
    *t = tmin;
    return 1;
}

/* linalg.zig:412-418 */
static grid_t grid_init(bbox_t b, const uint32_t res[3]) {
    grid_t g;
    g.bbox = b;
    g.res[0] = res[0]; g.res[1] = res[1]; g.res[2] = res[2];
    g.cell_size = vdiv(vsub(b.max, b.min), V((float)res[0], (float)res[1], (float)res[2]));
    return g;
}
/* linalg.zig:424-427 */
static void grid_cell_idx(const grid_t* g, v3 p, uint32_t out[3]) {
    v3 q = vdiv(vsub(p, g->bbox.min), g->cell_size);
    uint32_t c[3] = {f2u(q.x), f2u(q.y), f2u(q.z)};
    for (int i = 0; i < 3; ++i) out[i] = c[i] < g->res[i] - 1u ? c[i] : g->res[i] - 1u;
}
/* linalg.zig:429-431 */
static inline uint64_t grid_lin(const grid_t* g, uint64_t x, uint64_t y, uint64_t z) {
    return z * g->res[0] * g->res[1] + y * g->res[0] + x;
}
/* linalg.zig:433-441 */
static bbox_t grid_cell_bbox(const grid_t* g, uint64_t x, uint64_t y, uint64_t z) {
    bbox_t b;
    b.min = vadd(g->bbox.min, vmul(g->cell_size, V((float)x, (float)y, (float)z)));
    b.max = vadd(b.min, g->cell_size);
    return b;
}
/* linalg.zig:443-469 */
static int grid_trace(const grid_t* g, ray_t ray, iter_t* it) {
    float t_hit;
    if (!bbox_ray(g->bbox, ray, &t_hit)) return 0;
    t_hit = fmaxf(0.0f, t_hit);
    int sg[3] = {ray.dir.x < 0.0f, ray.dir.y < 0.0f, ray.dir.z < 0.0f};
    v3 t_delta = vabs(vdiv(g->cell_size, ray.dir));
    v3 local = vsub(ray_at(ray, t_hit), g->bbox.min);
    v3 q = vdiv(local, g->cell_size);
    float qa[3] = {q.x, q.y, q.z};
    float cs[3] = {g->cell_size.x, g->cell_size.y, g->cell_size.z};
    float la[3] = {local.x, local.y, local.z};
    float da[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
    float td[3] = {t_delta.x, t_delta.y, t_delta.z};
    for (int i = 0; i < 3; ++i) {
        uint32_t c = f2u(qa[i]);
        uint32_t rm1 = g->res[i] - 1u;
        c = c < rm1 ? c : rm1;
        it->cell[i] = c;
        it->step[i] = sg[i] ? 0xFFFFFFFFu : 1u;
        it->exit[i] = sg[i] ? 0u : rm1;
        it->t_delta[i] = td[i];
        float next_cell = (float)(uint32_t)(c + (sg[i] ? 0u : 1u));
        it->t_next[i] = t_hit + ((next_cell * cs[i] - la[i]) / da[i]);
    }
    return 1;
}
/* linalg.zig:478-496 */
static inline float iter_next(iter_t* it) {
    unsigned k = ((unsigned)(it->t_next[0] < it->t_next[1]) << 2) +
                 ((unsigned)(it->t_next[0] < it->t_next[2]) << 1) +
                 ((unsigned)(it->t_next[1] < it->t_next[2]));
    static const unsigned char map[8] = {2, 1, 2, 1, 2, 2, 0, 0};
    unsigned axis = map[k];
    if (it->cell[axis] == it->exit[axis]) return INFINITY;
    float t = it->t_next[axis];
    it->cell[axis] = it->cell[axis] + it->step[axis];
    it->t_next[axis] += it->t_delta[axis];
    return t;
}

/* ======================================================================= */
/* SAT triangle/AABB (linalg.zig:500-563)                                  */
/* ======================================================================= */
static int sat_axis(v3 v0, v3 v1, v3 v2, v3 ext, v3 axis) {
    float p0 = vdot(v0, axis), p1 = vdot(v1, axis), p2 = vdot(v2, axis);
    float r = ext.x * fabsf(vdot(V(1, 0, 0), axis)) +
              ext.y * fabsf(vdot(V(0, 1, 0), axis)) +
              ext.z * fabsf(vdot(V(0, 0, 1), axis));
    float maxp = fmaxf(p0, fmaxf(p1, p2));
    float minp = fminf(p0, fminf(p1, p2));
    return !(fmaxf(-maxp, minp) > r);
}
static int tri_aabb(const v3 tri[3], bbox_t b) {
    v3 center = vscale(vadd(b.max, b.min), 0.5f);
    v3 ext = vscale(vsub(b.max, b.min), 0.5f);
    v3 a = vsub(tri[0], center), bb = vsub(tri[1], center), c = vsub(tri[2], center);
    v3 ab = vnormalize(vsub(bb, a));
    v3 bc = vnormalize(vsub(c, bb));
    v3 ca = vnormalize(vsub(a, c));
    v3 axes[13] = {
        V(0.0f, -ab.z, ab.y), V(0.0f, -bc.z, bc.y), V(0.0f, -ca.z, ca.y),
        V(ab.z, 0.0f, -ab.x), V(bc.z, 0.0f, -bc.x), V(ca.z, 0.0f, -ca.x),
        V(-ab.y, ab.x, 0.0f), V(-bc.y, bc.x, 0.0f), V(-ca.y, ca.x, 0.0f),
        V(1, 0, 0), V(0, 1, 0), V(0, 0, 1), vcross(ab, bc)};
    for (int i = 0; i < 13; ++i)
        if (!sat_axis(a, bb, c, ext, axes[i])) return 0;
    return 1;
}

/* ======================================================================= */
/* Moller-Trumbore with back-face culling (linalg.zig:683-722)              */
/* ======================================================================= */
typedef struct { v3 v0, e1, e2; } tripos_t;
static inline int tri_ray(const tripos_t* tr, ray_t ray, float* t, float* uu, float* vv) {
    v3 pvec = vcross(ray.dir, tr->e2);
    float det = vdot(tr->e1, pvec);
    if (det < 0.00000001f) return 0;
    float inv_det = 1.0f / det;
    v3 tvec = vsub(ray.orig, tr->v0);
    float u = vdot(tvec, pvec) * inv_det;
    if (u < 0.0f || u > 1.0f) return 0;
    v3 qvec = vcross(tvec, tr->e1);
    float v = vdot(ray.dir, qvec) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return 0;
    *t = vdot(tr->e2, qvec) * inv_det;
    *uu = u;
    *vv = v;
    return 1;
}

/* ======================================================================= */
/* Scene (stage2 build/bake + stage3 data)                                  */
/* ======================================================================= */
typedef struct {
    int32_t off, w, h, u_min, u_max, v_min, v_max;
} tex_t;
typedef struct { tex_t base, emis, transp; } mat_t;

struct orc_scene {
    grid_t grid;
    uint32_t ncells;
    uint32_t* cells;      /* 2*ncells begin,end */
    uint32_t nrefs;
    uint32_t* indices;    /* nrefs */
    tripos_t* pos;        /* nrefs, cell order (bakeInto duplicates) */
    float* data;          /* nrefs * 15 : n0 n1 n2 uv0 uv1 uv2 */
    uint32_t* mat;        /* nrefs */
    uint32_t nmat;
    mat_t* mats;
    float* texels;
};

static void tri_minmax(const float* p, v3* mn, v3* mx) {
    v3 a = vload(p), b = vload(p + 3), c = vload(p + 6);
    *mn = vmin(a, vmin(b, c));
    *mx = vmax(a, vmax(b, c));
}

orc_scene* orc_scene_build(const float* pos, const float* nrm, const float* uv,
                           const uint32_t* mat, uint32_t n, const uint32_t res[3]) {
    orc_scene* s = (orc_scene*)calloc(1, sizeof *s);
    /* stage2.zig:44-57 initGrid */
    bbox_t b = {V(INFINITY, INFINITY, INFINITY), V(-INFINITY, -INFINITY, -INFINITY)};
    for (uint32_t t = 0; t < n; ++t)
        for (int i = 0; i < 3; ++i) {
            v3 p = vload(pos + 9 * (size_t)t + 3 * i);
            b.min = vmin(b.min, p);
            b.max = vmax(b.max, p);
        }
    s->grid = grid_init(b, res);
    const grid_t* g = &s->grid;
    s->ncells = res[0] * res[1] * res[2];
    uint32_t* first = (uint32_t*)calloc(s->ncells, 4);
    uint32_t* num = (uint32_t*)calloc(s->ncells, 4);
    /* stage2.zig:59-102 initCells (count) */
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t t = 0; t < n; ++t) {
            const float* p = pos + 9 * (size_t)t;
            v3 tri[3] = {vload(p), vload(p + 3), vload(p + 6)};
            v3 mn, mx;
            tri_minmax(p, &mn, &mx);
            uint32_t lo[3], hi[3];
            grid_cell_idx(g, mn, lo);
            grid_cell_idx(g, mx, hi);
            for (uint64_t z = lo[2]; z <= hi[2]; ++z)
                for (uint64_t y = lo[1]; y <= hi[1]; ++y)
                    for (uint64_t x = lo[0]; x <= hi[0]; ++x) {
                        bbox_t cb = grid_cell_bbox(g, x, y, z);
                        if (tri_aabb(tri, cb)) {
                            uint64_t ci = grid_lin(g, x, y, z);
                            if (pass == 0) num[ci] += 1;
                            else { s->indices[first[ci] + num[ci]] = t; num[ci] += 1; }
                        }
                    }
        }
        if (pass == 0) {
            uint32_t total = 0;
            for (uint32_t c = 0; c < s->ncells; ++c) { first[c] = total; total += num[c]; num[c] = 0; }
            s->nrefs = total;
            s->indices = (uint32_t*)malloc(sizeof(uint32_t) * (total ? total : 1));
        }
    }
    /* stage2.zig:137-164 bakeInto */
    s->cells = (uint32_t*)malloc(8 * (size_t)s->ncells);
    for (uint32_t c = 0; c < s->ncells; ++c) {
        s->cells[2 * c] = first[c];
        s->cells[2 * c + 1] = first[c] + num[c];
    }
    free(first); free(num);
    s->pos = (tripos_t*)malloc(sizeof(tripos_t) * (s->nrefs ? s->nrefs : 1));
    s->data = (float*)malloc(sizeof(float) * 15 * (s->nrefs ? s->nrefs : 1));
    s->mat = (uint32_t*)malloc(4 * (s->nrefs ? s->nrefs : 1));
    for (uint32_t i = 0; i < s->nrefs; ++i) {
        uint32_t t = s->indices[i];
        const float* p = pos + 9 * (size_t)t;
        v3 v0 = vload(p), v1 = vload(p + 3), v2 = vload(p + 6);
        s->pos[i].v0 = v0;
        s->pos[i].e1 = vsub(v1, v0);
        s->pos[i].e2 = vsub(v2, v0);
        memcpy(s->data + 15 * (size_t)i, nrm + 9 * (size_t)t, 9 * sizeof(float));
        memcpy(s->data + 15 * (size_t)i + 9, uv + 6 * (size_t)t, 6 * sizeof(float));
        s->mat[i] = mat[t];
    }
    return s;
}

void orc_scene_free(orc_scene* s) {
    if (!s) return;
    free(s->cells); free(s->indices); free(s->pos); free(s->data); free(s->mat);
    free(s->mats); free(s->texels); free(s);
}
uint32_t orc_scene_num_refs(const orc_scene* s) { return s->nrefs; }
void orc_scene_get(const orc_scene* s, float gb[6], float cs[3], uint32_t* cells, uint32_t* idx) {
    gb[0] = s->grid.bbox.min.x; gb[1] = s->grid.bbox.min.y; gb[2] = s->grid.bbox.min.z;
    gb[3] = s->grid.bbox.max.x; gb[4] = s->grid.bbox.max.y; gb[5] = s->grid.bbox.max.z;
    cs[0] = s->grid.cell_size.x; cs[1] = s->grid.cell_size.y; cs[2] = s->grid.cell_size.z;
    if (cells) memcpy(cells, s->cells, 8 * (size_t)s->ncells);
    if (idx) memcpy(idx, s->indices, 4 * (size_t)s->nrefs);
}
void orc_scene_set_materials(orc_scene* s, uint32_t n_mat, const int32_t* td,
                             const float* texels, uint64_t n) {
    free(s->mats); free(s->texels);
    s->nmat = n_mat;
    s->mats = (mat_t*)malloc(sizeof(mat_t) * (n_mat ? n_mat : 1));
    for (uint32_t m = 0; m < n_mat; ++m) {
        tex_t* t[3] = {&s->mats[m].base, &s->mats[m].emis, &s->mats[m].transp};
        for (int k = 0; k < 3; ++k) {
            const int32_t* d = td + 21 * (size_t)m + 7 * k;
            t[k]->off = d[0]; t[k]->w = d[1]; t[k]->h = d[2];
            t[k]->u_min = d[3]; t[k]->u_max = d[4]; t[k]->v_min = d[5]; t[k]->v_max = d[6];
        }
    }
    s->texels = (float*)malloc(sizeof(float) * (n ? n : 1));
    memcpy(s->texels, texels, sizeof(float) * n);
}

/* ======================================================================= */
/* stage3.zig shading                                                       */
/* ======================================================================= */
/* stage3.zig:94-96 */
static inline float tex_frac(float v) { return fabsf(v - truncf(v)); }
static inline int32_t clampi(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }
/* @mod on i32 with positive divisor: floor modulo */
static inline int32_t fmod_i(int32_t a, int32_t b) { int32_t r = a % b; return r < 0 ? r + b : r; }
/* std.math.lerp = @mulAdd(b - a, t, a) (fused) */
static inline float lerpf(float a, float b, float t) { return fmaf(b - a, t, a); }

/* stage3.zig:111-121, chans = 3 (Vec3) or 1 (f32) */
static void tex_sample_raw(const float* data, int chans, int32_t w_int, int32_t h_int,
                           int32_t u_min, int32_t u_max, int32_t v_min, int32_t v_max,
                           float u, float v, float* out) {
    float w = (float)w_int, h = (float)h_int;
    int32_t ui = f2i(floorf(w * u));
    int32_t vi = f2i(floorf(h * v));
    /* ui + 1 with i32 wrap (overflow is UB in the reference) */
    int32_t ui1 = (int32_t)((uint32_t)ui + 1u), vi1 = (int32_t)((uint32_t)vi + 1u);
    int32_t x1 = fmod_i(clampi(ui, u_min, u_max), w_int);
    int32_t y1 = fmod_i(clampi(vi, v_min, v_max), h_int);
    int32_t x2 = fmod_i(clampi(ui1, u_min, u_max), w_int);
    int32_t y2 = fmod_i(clampi(vi1, v_min, v_max), h_int);
    float fu = tex_frac(u), fv = tex_frac(v);
    for (int c = 0; c < chans; ++c) {
        float p11 = data[(size_t)(y1 * w_int + x1) * chans + c];
        float p21 = data[(size_t)(y1 * w_int + x2) * chans + c];
        float p12 = data[(size_t)(y2 * w_int + x1) * chans + c];
        float p22 = data[(size_t)(y2 * w_int + x2) * chans + c];
        float r1 = lerpf(p11, p21, fu);
        float r2 = lerpf(p12, p22, fu);
        out[c] = lerpf(r1, r2, fv);
    }
}
static inline void tex_sample(const orc_scene* s, const tex_t* t, int chans, float u, float v, float* out) {
    tex_sample_raw(s->texels + t->off, chans, t->w, t->h, t->u_min, t->u_max, t->v_min, t->v_max, u, v, out);
}

/* stage3.zig:144-150 */
static inline v3 env_color(ray_t r) {
    float t = 0.5f * (r.dir.y + 1.0f);
    return vadd(vscale(V(1, 1, 1), 1.0f - t), vscale(V(0.5f, 0.7f, 1.0f), t));
}

typedef struct { uint64_t seg, cells, tests, hits; } ctr_t;

/* stage3.zig:152-186 */
static inline float trace(const orc_scene* s, ray_t ray, float* hu, float* hv, uint32_t* hidx, ctr_t* ctr) {
    float nearest = INFINITY;
    iter_t it;
    ctr->seg++;
    if (grid_trace(&s->grid, ray, &it)) {
        for (;;) {
            uint64_t ci = grid_lin(&s->grid, it.cell[0], it.cell[1], it.cell[2]);
            uint32_t b = s->cells[2 * ci], e = s->cells[2 * ci + 1];
            ctr->cells++;
            for (uint32_t ti = b; ti < e; ++ti) {
                float t, u, v;
                ctr->tests++;
                if (tri_ray(&s->pos[ti], ray, &t, &u, &v)) {
                    if (nearest > t && t > 0.0f) { nearest = t; *hu = u; *hv = v; *hidx = ti; }
                }
            }
            float t_exit = iter_next(&it);
            if (nearest <= t_exit) break;
        }
    }
    return nearest;
}

/* stage3.zig:188-220 (recursive, literal) */
static v3 trace_recursive(const orc_scene* s, ray_t ray, uint32_t depth, rng_t* rng, ctr_t* ctr) {
    if (depth == 0) return V(0, 0, 0);
    float u = 0, v = 0;
    uint32_t idx = 0;
    float t = trace(s, ray, &u, &v, &idx, ctr);
    if (t == INFINITY) return env_color(ray);
    ctr->hits++;
    const float* d = s->data + 15 * (size_t)idx;
    const mat_t* m = &s->mats[s->mat[idx]];
    /* stage3.zig:53-66 interpolate */
    float w0 = 1.0f - u - v;
    float tc0 = d[9] * w0 + d[11] * u + d[13] * v;
    float tc1 = d[10] * w0 + d[12] * u + d[14] * v;
    float alb[3], emi[3], tr;
    tex_sample(s, &m->base, 3, tc0, tc1, alb);
    tex_sample(s, &m->emis, 3, tc0, tc1, emi);
    tex_sample(s, &m->transp, 1, tc0, tc1, &tr);
    v3 nrm = vadd(vadd(vscale(vload(d), w0), vscale(vload(d + 3), u)), vscale(vload(d + 6), v));
    if (rng_float(rng) > tr) {
        ray_t nr = {ray_at(ray, t + 1.1920928955078125e-07f), ray.dir};
        return trace_recursive(s, nr, depth - 1, rng, ctr);
    }
    v3 sc = vnormalize(vadd(nrm, random_unit_vector(rng)));
    ray_t nr = {ray_at(ray, t + 1.1920928955078125e-07f), sc};
    v3 li = trace_recursive(s, nr, depth - 1, rng, ctr);
    return vadd(V(emi[0], emi[1], emi[2]), vmul(V(alb[0], alb[1], alb[2]), li));
}

/* linalg.zig:150-159 toRGB: pow(1/2.2), clamp (upper only: the quirk at
 * linalg.zig:58-60), *256, truncate */
static inline void to_rgb(v3 c, uint8_t out[3]) {
    const float g = 0.454545454545454545f;
    float r[3] = {orc_powf(c.x, g), orc_powf(c.y, g), orc_powf(c.z, g)};
    for (int i = 0; i < 3; ++i) {
        float q = fminf(r[i], fmaxf(0.0f, 0.999999f)) * 256.0f;
        out[i] = (uint8_t)f2u(q);
    }
}

/* stage3.zig:27-35 */
static inline ray_t camera_ray(const orc_camera* c, float x, float y) {
    ray_t r;
    r.orig = vload(c->origin);
    r.dir = vnormalize(vadd(vadd(vload(c->llc), vscale(vload(c->right), x)), vscale(vload(c->up), y)));
    return r;
}

/* ---- renderWorker (stage3.zig:222-245) ---------------------------------- */
typedef struct {
    const orc_scene* s; const orc_camera* cam;
    uint32_t spp, max_bounce; int mode; uint64_t seed;
    const uint32_t* pixels; uint32_t px_begin; uint32_t n;  /* list or range */
    uint32_t thread_idx, thread_num;
    uint8_t* rgb; float* linear; ctr_t ctr;
} job_t;

static inline void shade_pixel(job_t* j, uint32_t slot, uint32_t pix, rng_t* rng) {
    const orc_camera* cam = j->cam;
    float inv = 1.0f / (float)j->spp;
    float x = (float)(pix % cam->w);
    float y = (float)(pix / cam->w);
    v3 pixel = V(0, 0, 0);
    for (uint32_t s = 0; s < j->spp; ++s) {
        if (j->mode == ORC_RNG_PATH) rng_init_path(rng, j->seed, pix, s);
        float jx = rng_float(rng);
        float jy = rng_float(rng);
        ray_t r = camera_ray(cam, x + jx, y + jy);
        v3 c = trace_recursive(j->s, r, j->max_bounce, rng, &j->ctr);
        pixel = vadd(pixel, c);
    }
    v3 lin = vmul(pixel, V(inv, inv, inv));
    if (j->linear) { j->linear[3 * (size_t)slot] = lin.x; j->linear[3 * (size_t)slot + 1] = lin.y; j->linear[3 * (size_t)slot + 2] = lin.z; }
    if (j->rgb) to_rgb(lin, j->rgb + 3 * (size_t)slot);
}

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    rng_t rng;
    rng_init_ref(&rng, j->thread_idx);       /* DefaultPrng.init(thread_idx) */
    uint32_t ppt = (j->n + j->thread_num - 1) / j->thread_num;
    uint32_t i = ppt * j->thread_idx;
    for (uint32_t k = 0; k < ppt; ++k, ++i) {
        if (i >= j->n) break;
        uint32_t pix = j->pixels ? j->pixels[i] : j->px_begin + i;
        shade_pixel(j, i, pix, &rng);
    }
    return NULL;
}

static int render_common(const orc_scene* s, const orc_camera* cam, uint32_t spp, uint32_t max_bounce,
                         int mode, uint64_t seed, uint32_t num_threads, const uint32_t* pixels,
                         uint32_t px_begin, uint32_t n, uint8_t* rgb, float* linear, uint64_t counters[5]) {
    pthread_once(&zig_once, zig_init);
    if (!s || !cam || spp == 0 || spp > 65535) return -1;
    if (num_threads == 0) num_threads = 1;
    job_t* jobs = (job_t*)calloc(num_threads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc(num_threads, sizeof(pthread_t));
    for (uint32_t t = 0; t < num_threads; ++t) {
        job_t* j = &jobs[t];
        j->s = s; j->cam = cam; j->spp = spp; j->max_bounce = max_bounce; j->mode = mode;
        j->seed = seed; j->pixels = pixels; j->px_begin = px_begin; j->n = n;
        j->thread_idx = t; j->thread_num = num_threads; j->rgb = rgb; j->linear = linear;
    }
    if (num_threads == 1) worker(&jobs[0]);
    else {
        for (uint32_t t = 0; t < num_threads; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
        for (uint32_t t = 0; t < num_threads; ++t) pthread_join(th[t], NULL);
    }
    if (counters) {
        memset(counters, 0, 5 * sizeof(uint64_t));
        for (uint32_t t = 0; t < num_threads; ++t) {
            counters[0] += jobs[t].ctr.seg; counters[1] += jobs[t].ctr.cells;
            counters[2] += jobs[t].ctr.tests; counters[3] += jobs[t].ctr.hits;
        }
        counters[4] = (uint64_t)n * spp;
    }
    free(jobs); free(th);
    return 0;
}

int orc_render(const orc_scene* s, const orc_camera* cam, uint32_t spp, uint32_t max_bounce,
               int rng_mode, uint64_t seed, uint32_t num_threads, uint32_t px_begin, uint32_t px_end,
               uint8_t* rgb, float* linear, uint64_t counters[5]) {
    if (px_end < px_begin) return -1;
    return render_common(s, cam, spp, max_bounce, rng_mode, seed, num_threads, NULL, px_begin,
                         px_end - px_begin, rgb, linear, counters);
}

int orc_render_pixels(const orc_scene* s, const orc_camera* cam, uint32_t spp, uint32_t max_bounce,
                      int rng_mode, uint64_t seed, uint32_t num_threads, const uint32_t* pixels,
                      uint32_t n, uint8_t* rgb, float* linear, uint64_t counters[5]) {
    return render_common(s, cam, spp, max_bounce, rng_mode, seed, num_threads, pixels, 0, n, rgb,
                         linear, counters);
}

/* ---- stage1.zig:309-371 loadCamera (from the node's global matrix) ------ */
int orc_camera_from_matrix(const float m[16], float yfov, int has_aspect, float aspect,
                           int width, int height, orc_camera* out) {
    uint32_t w, h;
    if (width < 0 && height < 0) return -1;                 /* OutputImgSizeIsNotSpecified */
    if (width >= 0 && height >= 0) {
        if (has_aspect) return -2;                          /* CameraHasAspectRatio */
        w = (uint32_t)width; h = (uint32_t)height;
    } else {
        if (!has_aspect) return -3;                         /* CameraHasntAspectRatio */
        w = width >= 0 ? (uint32_t)width : f2u((float)height * aspect);
        h = height >= 0 ? (uint32_t)height : f2u((float)width / aspect);
    }
    float fw = (float)w, fh = (float)h;
    v3 origin = V(m[12], m[13], m[14]);
    v3 fwd = vnormalize(vscale(V(m[8], m[9], m[10]), -1.0f));
    v3 right = vnormalize(vcross(fwd, V(0, 1, 0)));
    v3 up = vcross(fwd, right);
    float focal = (fh / 2.0f) / tanf(yfov / 2.0f);
    v3 llc = vsub(vsub(vscale(fwd, focal), vscale(right, fw / 2.0f)), vscale(up, fh / 2.0f));
    out->w = w; out->h = h;
    out->origin[0] = origin.x; out->origin[1] = origin.y; out->origin[2] = origin.z;
    out->llc[0] = llc.x; out->llc[1] = llc.y; out->llc[2] = llc.z;
    out->right[0] = right.x; out->right[1] = right.y; out->right[2] = right.z;
    out->up[0] = up.x; out->up[1] = up.y; out->up[2] = up.z;
    return 0;
}

/* ======================================================================= */
/* unit entry points                                                        */
/* ======================================================================= */
static bbox_t bb6(const float b[6]) { bbox_t r = {vload(b), vload(b + 3)}; return r; }

int orc_bbox_ray(const float b[6], const float o[3], const float d[3], float* t) {
    ray_t r = {vload(o), vload(d)};
    return bbox_ray(bb6(b), r, t);
}
int orc_grid_trace(const float b[6], const uint32_t res[3], const float o[3], const float d[3],
                   uint32_t* cells_out, float* t_out, int max_steps, uint32_t first[3]) {
    grid_t g = grid_init(bb6(b), res);
    ray_t r = {vload(o), vload(d)};
    iter_t it;
    if (!grid_trace(&g, r, &it)) return -1;
    first[0] = it.cell[0]; first[1] = it.cell[1]; first[2] = it.cell[2];
    int n = 0;
    while (n < max_steps) {
        float t = iter_next(&it);
        cells_out[3 * n] = it.cell[0]; cells_out[3 * n + 1] = it.cell[1]; cells_out[3 * n + 2] = it.cell[2];
        t_out[n] = t;
        ++n;
        if (t == INFINITY) break;
    }
    return n;
}
void orc_grid_cell_bbox(const float b[6], const uint32_t res[3], uint32_t x, uint32_t y, uint32_t z,
                        float out[6]) {
    grid_t g = grid_init(bb6(b), res);
    bbox_t c = grid_cell_bbox(&g, x, y, z);
    out[0] = c.min.x; out[1] = c.min.y; out[2] = c.min.z;
    out[3] = c.max.x; out[4] = c.max.y; out[5] = c.max.z;
}
int orc_tri_intersect(const float v0[3], const float v1[3], const float v2[3], const float o[3],
                      const float d[3], float tuv[3]) {
    tripos_t tr;
    tr.v0 = vload(v0);
    tr.e1 = vsub(vload(v1), tr.v0);
    tr.e2 = vsub(vload(v2), tr.v0);
    ray_t r = {vload(o), vload(d)};
    return tri_ray(&tr, r, &tuv[0], &tuv[1], &tuv[2]);
}
int orc_tri_aabb(const float tri[9], const float b[6]) {
    v3 t[3] = {vload(tri), vload(tri + 3), vload(tri + 6)};
    return tri_aabb(t, bb6(b));
}
void orc_cross(const float a[3], const float b[3], float out[3]) {
    v3 c = vcross(vload(a), vload(b));
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
float orc_length(const float v[3]) { return vlength(vload(v)); }
void orc_to_rgb(const float v[3], uint8_t out[3]) { to_rgb(vload(v), out); }
void orc_env(const float d[3], float out[3]) {
    ray_t r = {V(0, 0, 0), vload(d)};
    v3 c = env_color(r);
    out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
void orc_tex_sample(const float* data, int chans, int w, int h, int u_min, int u_max, int v_min,
                    int v_max, float u, float v, float* out) {
    tex_sample_raw(data, chans, w, h, u_min, u_max, v_min, v_max, u, v, out);
}
void orc_splitmix_u64(uint64_t seed, uint64_t* out, int n) {
    uint64_t s = seed;
    for (int i = 0; i < n; ++i) { s += GOLDEN; out[i] = mix64(s); }
}
void orc_xoshiro_u64(uint64_t seed, uint64_t* out, int n) {
    rng_t r; rng_init_ref(&r, seed);
    for (int i = 0; i < n; ++i) out[i] = rng_next(&r);
}
void orc_path_u64(uint64_t seed, uint32_t pixel, uint32_t sample, uint64_t* out, int n) {
    rng_t r; rng_init_path(&r, seed, pixel, sample);
    for (int i = 0; i < n; ++i) out[i] = rng_next(&r);
}
void orc_path_f32(uint64_t seed, uint32_t pixel, uint32_t sample, float* out, int n) {
    rng_t r; rng_init_path(&r, seed, pixel, sample);
    for (int i = 0; i < n; ++i) out[i] = rng_float(&r);
}
void orc_path_norm(uint64_t seed, uint32_t pixel, uint32_t sample, float* out, int n) {
    pthread_once(&zig_once, zig_init);
    rng_t r; rng_init_path(&r, seed, pixel, sample);
    for (int i = 0; i < n; ++i) out[i] = rng_norm(&r);
}
void orc_xoshiro_f32(uint64_t seed, float* out, int n) {
    rng_t r; rng_init_ref(&r, seed);
    for (int i = 0; i < n; ++i) out[i] = rng_float(&r);
}
void orc_xoshiro_norm(uint64_t seed, float* out, int n) {
    pthread_once(&zig_once, zig_init);
    rng_t r; rng_init_ref(&r, seed);
    for (int i = 0; i < n; ++i) out[i] = rng_norm(&r);
}
