// Host check of BRICK_SKIP4 (csrc/dda.h): on random grids, occupancies and
// rays (including axis-aligned and exact-diagonal ones that produce crossing
// ties), the skip walk must enter exactly the same cells of occupied bricks,
// with bit-identical DDA state, as the cell-by-cell walk of Iterator.next
// (DDA_STEP), and leave the grid at the same point.  And DDAW_STEP (the park
// kernel's walk) must step exactly like DDA_STEP.
//   g++ -O2 -std=c++17 -ffp-contract=off -I<csrc> dda_skip_check.cpp
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "dda.h"

using namespace zrt;

// PK_BM_TEST=1: the brick-major packed words (dda.h; the step macros name PK_BM)
#ifndef PK_BM_TEST
#define PK_BM_TEST 0
#endif
constexpr bool PK_BM = PK_BM_TEST != 0;

struct TestGrid {
    float bmin[3], bmax[3], cs[3];
    uint32_t res[3];
    uint32_t nb[3];
    std::vector<uint8_t> occ;   // per 4^3 brick
    bool occupied(uint32_t c0, uint32_t c1, uint32_t c2) const {
        return occ[((c2 >> 2) * nb[1] + (c1 >> 2)) * nb[0] + (c0 >> 2)] != 0;
    }
};

struct Rec {
    uint32_t c0, c1, c2, lin;
    float tn0, tn1, tn2;
    bool operator==(const Rec& o) const {
        return c0 == o.c0 && c1 == o.c1 && c2 == o.c2 && lin == o.lin &&
               !memcmp(&tn0, &o.tn0, 4) && !memcmp(&tn1, &o.tn1, 4) && !memcmp(&tn2, &o.tn2, 4);
    }
};

static Rec rec(const Dda& s) { return Rec{s.c0, s.c1, s.c2, s.lin, s.tn0, s.tn1, s.tn2}; }

// reference: every cell; keep the ones in occupied bricks
static std::vector<Rec> walk_cells(const TestGrid& g, const GridK& k, Dda s) {
    std::vector<Rec> out;
    for (int guard = 0; guard < 100000; ++guard) {
        if (g.occupied(s.c0, s.c1, s.c2)) out.push_back(rec(s));
        bool crossed;
        float t_exit;
        DDA_STEP(s, k, 2, crossed, t_exit);
        (void)crossed;
        if (t_exit == kInf) return out;
    }
    out.push_back(Rec{~0u, ~0u, ~0u, ~0u, 0, 0, 0});
    return out;
}

static uint64_t g_texit_fails = 0;
static uint64_t g_walk_fails = 0, g_walk_steps = 0;

// DDAW_STEP (the unpacked walk) against DDA_STEP, step by step: cells,
// linear index, crossing flag, T_EXIT and the next crossing ts bit for bit;
// and DDAV_STEPX (the packed walks, per-grid field widths) the same way: the
// packed word equals the cell's packing (and, on power-of-two grids, the
// linear index), the crossing flag, T_EXIT = EXITED ? +inf : TC and the ts bit
// for bit up to the exit step (past it the packed fields may carry; the walk
// has ended there), and the in-brick index of the park walk's OccX test;
// DDAV_STEPM / DDAV_STEPMB (the same step on lane masks) must equal
// DDAV_STEPX bit for bit.
static void walk_w(const GridK& k, Dda s) {
    DdaW w;
    ddaw_from(s, k, w);
    const uint32_t res[3] = {k.rm0 + 1, k.rm1 + 1, k.rm2 + 1};
    PackK pk;
    const bool packs = pack_layout(res, pk, PK_BM);
    if (!packs || pk.bm != (uint32_t)PK_BM) {    // (brick-major words pack power-of-two grids only)
        if (!PK_BM) ++g_walk_fails;
        return;
    }
    const bool linear = pack_is_linear(res, pk);
    DdaV x;
    ddav_from(s, k, pk, x);
    DdaV y = x;                              // DDAV_STEPM (lane-mask form of the park walk trip)
    DdaV z = x;                              // DDAV_STEPMB (its lane-walk form)
    for (int guard = 0; guard < 100000; ++guard) {
        bool c1, c2, c4, ex4;
        float e1, e2, tc4;
        const uint32_t pc_before = x.pc;
        DDA_STEP(s, k, 2, c1, e1);
        DDAW_STEP(w, 2, c2, e2);
        DDAV_STEPX(x, pk, pk.low2, c4, ex4, tc4);
        LaneM ex5;
        float tc5;
        const bool y_in_step = y.pc == pc_before;
        DDAV_STEPM(y, pk.f0, pk.f1, pk.f2, ex5, tc5);
        bool c6, ex6;
        float tc6;
        DDAV_STEPMB(z, pk.f0, pk.f1, pk.f2, pk.low2, c6, ex6, tc6);
        if (!y_in_step || ex5 != ex4 || memcmp(&tc5, &tc4, 4) || y.pc != x.pc || memcmp(&y.tn0, &x.tn0, 4) ||
            memcmp(&y.tn1, &x.tn1, 4) || memcmp(&y.tn2, &x.tn2, 4) || c6 != c4 || ex6 != ex4 ||
            memcmp(&tc6, &tc4, 4) || z.pc != x.pc || memcmp(&z.tn0, &x.tn0, 4) || memcmp(&z.tn1, &x.tn1, 4) ||
            memcmp(&z.tn2, &x.tn2, 4)) {
            ++g_walk_fails;
            return;
        }
        ++g_walk_steps;
        const bool same = c1 == c2 && !memcmp(&e1, &e2, 4) && s.c0 == w.c0 && s.c1 == w.c1 && s.c2 == w.c2 &&
                          s.lin == w.lin && !memcmp(&s.tn0, &w.tn0, 4) && !memcmp(&s.tn1, &w.tn1, 4) &&
                          !memcmp(&s.tn2, &w.tn2, 4);
        const float e4 = ex4 ? kInf : tc4;
        bool same_v = !memcmp(&e1, &e4, 4) && !memcmp(&s.tn0, &x.tn0, 4) && !memcmp(&s.tn1, &x.tn1, 4) &&
                      !memcmp(&s.tn2, &x.tn2, 4);
        if (e1 != kInf) {
            const uint32_t kk = (((x.pc & pk.low2) * pk.kmul) >> pk.kshr) & 63u;
            const uint32_t kw = (s.c0 & 3u) | (s.c1 & 3u) << 2 | (s.c2 & 3u) << 4;
            same_v = same_v && c1 == c4 && x.pc == pack_cellv(pk, s.c0, s.c1, s.c2) && kk == kw &&
                     (!linear || x.pc == s.lin);
        }
        if (!same || !same_v) {
            ++g_walk_fails;
            return;
        }
        if (e1 == kInf) return;
    }
}

// product: skip unoccupied bricks whole; each skip's T_EXIT must be the exit
// t of the last cell the cell walk passes in that brick (+inf at the grid
// exit), and its state the cell walk's state on entering the next brick
static std::vector<Rec> walk_skip(const TestGrid& g, const GridK& k, Dda s, uint64_t* skips) {
    std::vector<Rec> out;
    for (int guard = 0; guard < 100000; ++guard) {
        const bool occ = g.occupied(s.c0, s.c1, s.c2);
        if (!occ && s.neg < 8u) {
            Dda q = s;
            float last = 0.0f;
            for (;;) {
                bool cr;
                DDA_STEP(q, k, 2, cr, last);
                if (cr || last == kInf) break;
            }
            bool exited;
            float te;
            BRICK_SKIP4(s, k, exited, te);
            ++*skips;
            if (memcmp(&te, &last, 4) != 0 || (!exited && !(rec(s) == rec(q)))) ++g_texit_fails;
            if (exited) return out;
            continue;
        }
        if (occ) out.push_back(rec(s));
        bool crossed;
        float t_exit;
        DDA_STEP(s, k, 2, crossed, t_exit);
        (void)crossed;
        if (t_exit == kInf) return out;
    }
    out.push_back(Rec{~0u, ~0u, ~0u, ~0u, 0, 0, 0});
    return out;
}

// BRICK_SKIPV (the primary lane walk's skip on the packed state) with
// DDAV_STEPX in occupied bricks: the same cells of occupied bricks with the
// same crossing ts as the cell walk, each skip's TC the exit t of the last
// cell the cell walk passes in that brick, EXITED exactly at the grid exit
static uint64_t g_skipv_fails = 0, g_skipv = 0;
static void walk_skipv(const TestGrid& g, const GridK& k, const Dda& s0, const std::vector<Rec>& ref) {
    const uint32_t res[3] = {k.rm0 + 1, k.rm1 + 1, k.rm2 + 1};
    PackK pk;
    if (!pack_layout(res, pk, PK_BM) || pk.bm != (uint32_t)PK_BM) return;
    DdaV x;
    ddav_from(s0, k, pk, x);
    Dda q = s0;                                   // the cell walk alongside
    size_t n = 0;
    for (int guard = 0; guard < 100000; ++guard) {
        const uint32_t c0 = pack_coord(pk, x.pc, 0), c1 = pack_coord(pk, x.pc, 1), c2 = pack_coord(pk, x.pc, 2);
        const bool occ = g.occupied(c0, c1, c2);
        if (occ) {
            if (n >= ref.size() || ref[n].c0 != c0 || ref[n].c1 != c1 || ref[n].c2 != c2 ||
                memcmp(&ref[n].tn0, &x.tn0, 4) || memcmp(&ref[n].tn1, &x.tn1, 4) || memcmp(&ref[n].tn2, &x.tn2, 4)) {
                ++g_skipv_fails;
                return;
            }
            ++n;
        }
        bool exited, crossed;
        float tc;
        if (!occ && s0.neg < 8u) {
            float last = 0.0f;
            for (;;) {                                // the cell walk to the brick's last cell
                bool cr;
                DDA_STEP(q, k, 2, cr, last);
                if (cr || last == kInf) break;
            }
            BRICK_SKIPV(x, pk, exited, tc);
            ++g_skipv;
            const float te = exited ? kInf : tc;
            if (memcmp(&te, &last, 4) != 0) { ++g_skipv_fails; return; }
        } else {
            float last;
            bool cr;
            DDA_STEP(q, k, 2, cr, last);
            DDAV_STEPX(x, pk, pk.low2, crossed, exited, tc);
            const float te = exited ? kInf : tc;
            if (memcmp(&te, &last, 4) != 0) { ++g_skipv_fails; return; }
        }
        if (exited) break;
        if (x.pc != pack_cellv(pk, q.c0, q.c1, q.c2) || memcmp(&q.tn0, &x.tn0, 4) || memcmp(&q.tn1, &x.tn1, 4) ||
            memcmp(&q.tn2, &x.tn2, 4)) {
            ++g_skipv_fails;
            return;
        }
    }
    if (n != ref.size() && !(ref.size() == n + 1 && ref[n].c0 == ~0u)) ++g_skipv_fails;
}

// DDAV_FF (the primary walk's fast-forward) against the cell walk: from
// random points of the walk, the packed state after every crossing with
// t < tau must be the cell walk's state after its steps with TC < tau (ts bit
// for bit, same cell), and EXITED must be set exactly when the cell walk meets
// its exit crossing among them.
static uint64_t g_ff_fails = 0, g_ff = 0, g_ff_steps = 0;
static void walk_ff(const GridK& k, const Dda& s0, std::mt19937_64& rng) {
    const uint32_t res[3] = {k.rm0 + 1, k.rm1 + 1, k.rm2 + 1};
    PackK pk;
    if (!pack_layout(res, pk, PK_BM) || pk.bm != (uint32_t)PK_BM || s0.neg >= 8u) return;
    Dda q = s0;
    for (int guard = 0; guard < 100000; ++guard) {
        if (rng() % 3 == 0) {                       // fast-forward from here
            DdaV x;
            ddav_from(q, k, pk, x);
            const float tmin = fminf(q.tn0, fminf(q.tn1, q.tn2));
            const float dmin = fminf(q.td0, fminf(q.td1, q.td2));
            const float tau = tmin + (float)(1 + rng() % 120) * dmin;
            bool exited, exited4, exitedc, exitedn;
            DdaV x4 = x, xc = x, xn = x;
            DDAV_FF(x, pk.f0, pk.f1, pk.f2, tau, exited);
            DDAV_FF4(x4, pk.f0, pk.f1, pk.f2, tau, exited4);
            DDAV_FFC(xc, pk, pk.f0, pk.f1, pk.f2, tau, exitedc);
            DDAV_FFN(xn, pk, pk.f0, pk.f1, pk.f2, tau, exitedn);
            if (exitedn != exited || (!exited && (xn.pc != x.pc || memcmp(&xn.tn0, &x.tn0, 4) ||
                                                  memcmp(&xn.tn1, &x.tn1, 4) || memcmp(&xn.tn2, &x.tn2, 4)))) {
                ++g_ff_fails;
                return;
            }
            if (exited4 != exited || (!exited && (x4.pc != x.pc || memcmp(&x4.tn0, &x.tn0, 4) ||
                                                  memcmp(&x4.tn1, &x.tn1, 4) || memcmp(&x4.tn2, &x.tn2, 4)))) {
                ++g_ff_fails;
                return;
            }
            if (exitedc != exited || (!exited && (xc.pc != x.pc || memcmp(&xc.tn0, &x.tn0, 4) ||
                                                  memcmp(&xc.tn1, &x.tn1, 4) || memcmp(&xc.tn2, &x.tn2, 4)))) {
                ++g_ff_fails;
                return;
            }
            Dda r = q;                              // the cell walk: steps with TC < tau
            bool rexit = false;
            for (int g2 = 0; g2 < 100000; ++g2) {
                Dda t = r;
                bool cr;
                float te;
                DDA_STEP(t, k, 2, cr, te);
                const float tc = fminf(r.tn0, fminf(r.tn1, r.tn2));   // the step's crossing t
                if (!(tc < tau)) break;
                if (te == kInf) { rexit = true; break; }
                r = t;
                ++g_ff_steps;
            }
            ++g_ff;
            if (exited != rexit ||
                (!exited && (x.pc != pack_cellv(pk, r.c0, r.c1, r.c2) || memcmp(&x.tn0, &r.tn0, 4) ||
                             memcmp(&x.tn1, &r.tn1, 4) || memcmp(&x.tn2, &r.tn2, 4)))) {
                ++g_ff_fails;
                return;
            }
        }
        bool cr;
        float te;
        DDA_STEP(q, k, 2, cr, te);
        if (te == kInf) return;
    }
}

int main(int argc, char** argv) {
    const int n_grids = argc > 1 ? atoi(argv[1]) : 40;
    const int n_rays = argc > 2 ? atoi(argv[2]) : 4000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    uint64_t total = 0, skips = 0, ties = 0, fails = 0, g_layout_grids = 0;
    for (int gi = 0; gi < n_grids; ++gi) {
        TestGrid g;
        const bool pow2 = gi % 3 == 0;     // exact arithmetic -> many crossing ties
        for (int a = 0; a < 3; ++a) {
            g.res[a] = gi == 0 ? 128u : 1u + (uint32_t)(rng() % 40);
            if (PK_BM && gi % 2 == 1) g.res[a] = 4u << (rng() % 5);   // (grids the brick-major words pack)
            g.bmin[a] = pow2 ? 0.0f : -5.0f + 10.0f * U(rng);
            g.cs[a] = pow2 ? 0.25f : 0.05f + U(rng);
            g.bmax[a] = g.bmin[a] + g.cs[a] * (float)g.res[a];
            g.nb[a] = (g.res[a] + 3) / 4;
        }
        g.occ.resize((size_t)g.nb[0] * g.nb[1] * g.nb[2]);
        const float dens = (gi % 4) * 0.1f;
        for (auto& o : g.occ) o = U(rng) < dens;
        GridK k{g.res[0] - 1, g.res[1] - 1, g.res[2] - 1, g.res[0], g.res[0] * g.res[1]};
        {   // grids whose packed words take this build's layout (the walk_skipv / walk_ff checks run on them)
            PackK pk;
            if (pack_layout(g.res, pk, PK_BM) && pk.bm == (uint32_t)PK_BM) ++g_layout_grids;
        }
        for (int r = 0; r < n_rays; ++r) {
            v3 o, d;
            const int kind = r % 4;
            float c[3];
            for (int a = 0; a < 3; ++a) {
                const float ext = g.bmax[a] - g.bmin[a];
                c[a] = g.bmin[a] - 0.5f * ext + 2.0f * ext * U(rng);
                if (kind >= 2) c[a] = g.bmin[a] + g.cs[a] * (float)(rng() % (g.res[a] + 1));   // on cell corners
            }
            o = mk(c[0], c[1], c[2]);
            if (kind == 0) {
                d = normalize(mk(U(rng) - 0.5f, U(rng) - 0.5f, U(rng) - 0.5f));
            } else if (kind == 1) {                 // one or two zero components
                float v[3] = {U(rng) - 0.5f, U(rng) - 0.5f, U(rng) - 0.5f};
                v[rng() % 3] = 0.0f;
                if (rng() & 1) v[rng() % 3] = 0.0f;
                if (v[0] == 0 && v[1] == 0 && v[2] == 0) v[0] = 1.0f;
                d = normalize(mk(v[0], v[1], v[2]));
            } else {                                // exact diagonals: equal |d| per axis
                const float sx = (rng() & 1) ? 1.0f : -1.0f, sy = (rng() & 1) ? 1.0f : -1.0f,
                            sz = (rng() & 1) ? 1.0f : -1.0f;
                d = kind == 2 ? normalize(mk(sx, sy, sz)) : normalize(mk(sx, 2.0f * sy, sz));
            }
            Dda s;
            if (!dda_init(g.bmin, g.bmax, g.res, g.cs, o, d, s)) continue;
            ++total;
            if (s.tn0 == s.tn1 || s.tn1 == s.tn2 || s.tn0 == s.tn2) ++ties;
            walk_w(k, s);
            const auto a = walk_cells(g, k, s);
            const auto b = walk_skip(g, k, s, &skips);
            walk_skipv(g, k, s, a);
            walk_ff(k, s, rng);
            if (!(a.size() == b.size() && std::equal(a.begin(), a.end(), b.begin()))) {
                if (++fails <= 5)
                    fprintf(stderr, "MISMATCH grid %d ray %d: %zu vs %zu cells (o=%g,%g,%g d=%g,%g,%g)\n", gi, r,
                            a.size(), b.size(), o.x, o.y, o.z, d.x, d.y, d.z);
            }
        }
    }
    fails += g_texit_fails + g_walk_fails + g_skipv_fails + g_ff_fails;
    printf("{\"rays\": %llu, \"skips\": %llu, \"tie_starts\": %llu, \"t_exit_fails\": %llu, "
           "\"walk_steps\": %llu, \"walk_fails\": %llu, \"skipv\": %llu, \"skipv_fails\": %llu, \"ff\": %llu, \"ff_steps\": %llu, \"ff_fails\": %llu, \"layout_grids\": %llu, \"fails\": %llu}\n",
           (unsigned long long)total, (unsigned long long)skips, (unsigned long long)ties,
           (unsigned long long)g_texit_fails, (unsigned long long)g_walk_steps, (unsigned long long)g_walk_fails,
           (unsigned long long)g_skipv, (unsigned long long)g_skipv_fails, (unsigned long long)g_ff,
           (unsigned long long)g_ff_steps, (unsigned long long)g_ff_fails, (unsigned long long)g_layout_grids,
           (unsigned long long)fails);
    return fails ? 1 : 0;
}
