// Host emulation of trace_wave (render.hip): 64 rays walked in lockstep with
// the triangle tests of each step laid out over the wave and reduced per
// owner by min (t bits, ref).  Compared ray by ray with the sequential
// traceRay walk (trace_ray): same nearest, ref, u, v.  Built as a shared
// library by tests/test_wave_traversal.py and called through ctypes on the
// baked arrays of a real scene.
#include <cstdint>
#include <cstring>
#include <vector>

#include "dda.h"

using namespace zrt;

namespace {

struct Scn {
    const float *bmin, *bmax, *cs;
    const uint32_t *res, *cells;
    const float* pos;   // 9 per ref
    GridK gk;
};

bool test_tri(const Scn& S, uint32_t j, v3 o, v3 d, float* t, float* u, float* v) {
    const float* q = S.pos + 9ull * j;
    return tri_ray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]), o, d, t, u, v);
}

// stage3.zig:152-186, one ray
void trace_seq(const Scn& S, v3 o, v3 d, float out[4]) {
    float nearest = kInf, hu = 0, hv = 0;
    uint32_t hidx = 0;
    Dda s;
    if (dda_init(S.bmin, S.bmax, S.res, S.cs, o, d, s)) {
        for (;;) {
            const uint32_t b = S.cells[2 * s.lin], e = S.cells[2 * s.lin + 1];
            for (uint32_t j = b; j < e; ++j) {
                float t, u, v;
                if (test_tri(S, j, o, d, &t, &u, &v) && nearest > t && t > 0.0f) {
                    nearest = t; hu = u; hv = v; hidx = j;
                }
            }
            bool crossed;
            float t_exit;
            DDA_STEP(s, S.gk, 2, crossed, t_exit);
            (void)crossed;
            if (nearest <= t_exit) break;
        }
    }
    out[0] = nearest; out[1] = hu; out[2] = hv;
    memcpy(&out[3], &hidx, 4);
}

// trace_wave, 64 lanes (fewer at the tail)
void trace_wave_emul(const Scn& S, const v3* o, const v3* d, int nl, float* out) {
    float nearest[64], hu[64], hv[64];
    uint32_t hidx[64];
    Dda s[64];
    bool active[64];
    for (int l = 0; l < nl; ++l) {
        nearest[l] = kInf; hu[l] = hv[l] = 0; hidx[l] = 0;
        active[l] = dda_init(S.bmin, S.bmax, S.res, S.cs, o[l], d[l], s[l]);
    }
    for (;;) {
        bool any = false;
        for (int l = 0; l < nl; ++l) any |= active[l];
        if (!any) break;
        uint32_t b[64] = {0}, n[64] = {0}, off[64] = {0};
        uint32_t N = 0;
        for (int l = 0; l < nl; ++l) {
            if (active[l]) { b[l] = S.cells[2 * s[l].lin]; n[l] = S.cells[2 * s[l].lin + 1] - b[l]; }
            off[l] = N;
            N += n[l];
        }
        if (N) {
            uint64_t best[64];
            float bu[64], bv[64];
            for (int l = 0; l < 64; ++l) best[l] = ~0ull;
            for (uint32_t q = 0; q < N; ++q) {        // all rounds, all lanes
                int owner = 0;
                for (int l = 0; l < nl; ++l)
                    if (n[l] && q >= off[l] && q < off[l] + n[l]) owner = l;
                const uint32_t j = b[owner] - off[owner] + q;
                float t, u, v;
                if (test_tri(S, j, o[owner], d[owner], &t, &u, &v) && nearest[owner] > t && t > 0.0f) {
                    uint32_t tb;
                    memcpy(&tb, &t, 4);
                    const uint64_t key = ((uint64_t)tb << 32) | j;
                    if (key < best[owner]) { best[owner] = key; bu[owner] = u; bv[owner] = v; }
                }
            }
            for (int l = 0; l < nl; ++l) {
                if (n[l] && best[l] != ~0ull) {
                    const uint32_t tb = (uint32_t)(best[l] >> 32);
                    memcpy(&nearest[l], &tb, 4);
                    hidx[l] = (uint32_t)best[l];
                    hu[l] = bu[l]; hv[l] = bv[l];
                }
            }
        }
        for (int l = 0; l < nl; ++l) {
            if (!active[l]) continue;
            bool crossed;
            float t_exit;
            DDA_STEP(s[l], S.gk, 2, crossed, t_exit);
            (void)crossed;
            if (nearest[l] <= t_exit) active[l] = false;
        }
    }
    for (int l = 0; l < nl; ++l) {
        out[4 * l] = nearest[l]; out[4 * l + 1] = hu[l]; out[4 * l + 2] = hv[l];
        memcpy(&out[4 * l + 3], &hidx[l], 4);
    }
}

// The park kernel's entry-face skip (render.hip cell32_kernel): refs whose
// (v0, e1, e2) equal a ref of the cell the ray just left are not tested.
// mask[8 * cell + 2 + f] as the kernel builds it (dense cell index here).
std::vector<uint32_t> face_masks(const Scn& S, uint32_t ncells) {
    std::vector<uint32_t> m(8ull * ncells);
    const uint32_t r0 = S.res[0], r1 = S.res[1], r2 = S.res[2];
    auto same = [&](uint32_t a, uint32_t b) { return !memcmp(S.pos + 9ull * a, S.pos + 9ull * b, 36); };
    for (uint32_t ci = 0; ci < ncells; ++ci) {
        const uint32_t x = ci % r0, y = (ci / r0) % r1, z = ci / r0 / r1;
        const uint32_t b = S.cells[2 * ci], e = S.cells[2 * ci + 1], n = e - b;
        const uint32_t all = n >= 32u ? ~0u : (1u << n) - 1u;
        for (uint32_t f = 0; f < 6; ++f) {
            const uint32_t axis = f >> 1, neg = f & 1u;
            const uint32_t cc = axis == 0 ? x : (axis == 1 ? y : z), rr = axis == 0 ? r0 : (axis == 1 ? r1 : r2);
            const bool inside = neg ? cc + 1u < rr : cc > 0u;
            uint32_t mk_ = all;
            if (inside && n > 0 && n <= 32) {
                const uint32_t step = axis == 0 ? 1u : (axis == 1 ? r0 : r0 * r1);
                const uint32_t pci = neg ? ci + step : ci - step;
                for (uint32_t k = 0; k < n; ++k)
                    for (uint32_t q = S.cells[2 * pci]; q < S.cells[2 * pci + 1]; ++q)
                        if (same(b + k, q)) { mk_ &= ~(1u << k); break; }
            }
            m[8ull * ci + 2 + f] = mk_;
        }
    }
    return m;
}

// trace_seq with the skip: same walk, each cell's refs filtered by the mask
// of the face the ray entered across (all refs in the first cell)
void trace_skip(const Scn& S, const std::vector<uint32_t>& fm, v3 o, v3 d, float out[4], uint64_t* tests,
                uint64_t* kept) {
    float nearest = kInf, hu = 0, hv = 0;
    uint32_t hidx = 0;
    Dda s;
    if (dda_init(S.bmin, S.bmax, S.res, S.cs, o, d, s)) {
        int face = -1;
        for (;;) {
            const uint32_t b = S.cells[2 * s.lin], e = S.cells[2 * s.lin + 1], n = e - b;
            const uint32_t m = (face < 0 || n > 32) ? ~0u : fm[8ull * s.lin + 2 + face];
            for (uint32_t j = b; j < e; ++j) {
                ++*tests;
                if (j - b < 32 && !((m >> (j - b)) & 1u)) continue;
                ++*kept;
                float t, u, v;
                if (test_tri(S, j, o, d, &t, &u, &v) && nearest > t && t > 0.0f) {
                    nearest = t; hu = u; hv = v; hidx = j;
                }
            }
            const uint32_t c0 = s.c0, c1 = s.c1, c2 = s.c2;
            bool crossed;
            float t_exit;
            DDA_STEP(s, S.gk, 2, crossed, t_exit);
            (void)crossed;
            if (nearest <= t_exit) break;
            const int axis = s.c0 != c0 ? 0 : (s.c1 != c1 ? 1 : 2);
            face = 2 * axis + (int)((s.neg >> axis) & 1u);
            (void)c2;
        }
    }
    out[0] = nearest; out[1] = hu; out[2] = hv;
    memcpy(&out[3], &hidx, 4);
}

}  // namespace

// Sequential traceRay with and without the entry-face skip: mismatching
// output words; stats[0] tests of the full walk, stats[1] tests kept.
extern "C" int skip_check(const float* bmin, const float* bmax, const uint32_t* res, const float* cs,
                          const uint32_t* cells, const float* pos, uint32_t nrays, const float* rays,
                          uint64_t* stats) {
    Scn S{bmin, bmax, cs, res, cells, pos, GridK{res[0] - 1, res[1] - 1, res[2] - 1, res[0], res[0] * res[1]}};
    const std::vector<uint32_t> fm = face_masks(S, res[0] * res[1] * res[2]);
    uint32_t bad = 0;
    stats[0] = stats[1] = 0;
    for (uint32_t i = 0; i < nrays; ++i) {
        const v3 o = mk(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        const v3 d = mk(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        float a[4], b[4];
        trace_seq(S, o, d, a);
        trace_skip(S, fm, o, d, b, &stats[0], &stats[1]);
        if (memcmp(a, b, 16)) ++bad;
    }
    return (int)bad;
}

extern "C" int wave_check(const float* bmin, const float* bmax, const uint32_t* res, const float* cs,
                          const uint32_t* cells, const float* pos, uint32_t nrays, const float* rays,
                          float* out_seq, float* out_wave) {
    Scn S{bmin, bmax, cs, res, cells, pos, GridK{res[0] - 1, res[1] - 1, res[2] - 1, res[0], res[0] * res[1]}};
    std::vector<v3> o(nrays), d(nrays);
    for (uint32_t i = 0; i < nrays; ++i) {
        o[i] = mk(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        d[i] = mk(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        trace_seq(S, o[i], d[i], out_seq + 4ull * i);
    }
    for (uint32_t i = 0; i < nrays; i += 64) {
        const int nl = (int)(nrays - i < 64 ? nrays - i : 64);
        trace_wave_emul(S, &o[i], &d[i], nl, out_wave + 4ull * i);
    }
    uint32_t bad = 0;
    for (uint64_t k = 0; k < 4ull * nrays; ++k)
        if (memcmp(&out_seq[k], &out_wave[k], 4)) ++bad;
    return (int)bad;
}
