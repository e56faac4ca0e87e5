// Host model of the primary frustum bounds (csrc/escape.h frustum_bound) on a
// real scene (planning tool, not product code): per 8x8 pixel block of the
// camera the bounds (lo, hi), then random camera rays walked as traceRay does
// (stage3.zig:152-185, triangles tested): how many walk steps lie in cells
// exited below lo (the fast-forward's share) and after the exit that passes
// hi (the far stop's share), and whether any occupied cell lies past hi.
//   g++ -O2 -std=c++17 -fopenmp -ffp-contract=off -Izig_raytracing_contest_amd/csrc -Iinclude tools/frustum_sim.cpp -o /tmp/frustum_sim
//   frustum_sim <scene.bin> <cam.bin> [rays=50000] [block=8]
// (block: the pixel block edge of the bounds; the product's is 8)
// scene.bin: as tools/walk_sim.cpp; cam.bin: origin, lower_left_corner, right,
// up (3 f32 each), w, h (f32).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "dda.h"
#include "escape.h"

using namespace zrt;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int nrays = argc > 3 ? atoi(argv[3]) : 50000;
    const uint32_t B = argc > 4 ? (uint32_t)atoi(argv[4]) : 8u;
    FILE* f = fopen(argv[1], "rb");
    float bmin[3], bmax[3], cs[3];
    uint32_t res[3], ncells, nrefs;
    if (fread(bmin, 4, 3, f) != 3 || fread(bmax, 4, 3, f) != 3 || fread(res, 4, 3, f) != 3 ||
        fread(cs, 4, 3, f) != 3 || fread(&ncells, 4, 1, f) != 1 || fread(&nrefs, 4, 1, f) != 1)
        return 3;
    std::vector<uint32_t> cells(2ull * ncells);
    std::vector<float> tp(9ull * nrefs);
    if (fread(cells.data(), 8, ncells, f) != ncells || fread(tp.data(), 36, nrefs, f) != nrefs) return 3;
    fclose(f);
    float cam[14];
    f = fopen(argv[2], "rb");
    if (fread(cam, 4, 14, f) != 14) return 3;
    fclose(f);
    const uint32_t W = (uint32_t)cam[12], H = (uint32_t)cam[13];
    const uint32_t n0 = res[0] + 1, n1 = res[1] + 1, n2 = res[2] + 1;
    std::vector<uint32_t> sat((size_t)n0 * n1 * n2, 0);
    for (uint32_t z = 0; z < res[2]; ++z)
        for (uint32_t y = 0; y < res[1]; ++y)
            for (uint32_t x = 0; x < res[0]; ++x) {
                const size_t c = ((size_t)z * res[1] + y) * res[0] + x;
                sat[((size_t)(z + 1) * n1 + y + 1) * n0 + x + 1] = cells[2 * c + 1] > cells[2 * c];
            }
    for (uint32_t z = 0; z < n2; ++z)
        for (uint32_t y = 0; y < n1; ++y)
            for (uint32_t x = 1; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)z * n1 + y) * n0 + x - 1];
    for (uint32_t z = 0; z < n2; ++z)
        for (uint32_t y = 1; y < n1; ++y)
            for (uint32_t x = 0; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)z * n1 + y - 1) * n0 + x];
    for (uint32_t z = 1; z < n2; ++z)
        for (uint32_t y = 0; y < n1; ++y)
            for (uint32_t x = 0; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)(z - 1) * n1 + y) * n0 + x];
    const EscSat S{sat.data(), n0, n0 * n1};
    const uint32_t nbx = (W + B - 1) / B, nby = (H + B - 1) / B;
    std::vector<FrustumBound> fb(nbx * nby);
#pragma omp parallel for
    for (int b = 0; b < (int)(nbx * nby); ++b) {
        const uint32_t bx = b % nbx, by = b / nbx;
        fb[b] = frustum_bound(S, res, bmin, bmax, cs, cam, cam + 3, cam + 6, cam + 9, (double)B * bx,
                              (double)B * bx + B, (double)B * by, (double)B * by + B);
    }
    const GridK g{res[0] - 1, res[1] - 1, res[2] - 1, res[0], res[0] * res[1]};
    const v3 o = mk(cam[0], cam[1], cam[2]), llc = mk(cam[3], cam[4], cam[5]), right = mk(cam[6], cam[7], cam[8]),
             up = mk(cam[9], cam[10], cam[11]);
    uint64_t steps = 0, below = 0, above = 0, rays = 0, misses = 0, bad = 0, infr = 0;
#pragma omp parallel for reduction(+ : steps, below, above, rays, misses, bad, infr)
    for (int r = 0; r < nrays; ++r) {
        std::mt19937_64 rng(r * 7919ull + 5);
        std::uniform_real_distribution<float> U(0.0f, 1.0f);
        const uint32_t px = rng() % W, py = rng() % H;
        const float ux = px + U(rng), vy = py + U(rng);
        const v3 d = normalize(add(add(llc, scale(right, ux)), scale(up, vy)));
        const FrustumBound b = fb[(py / B) * nbx + px / B];
        Dda s;
        if (!dda_init(bmin, bmax, res, cs, o, d, s)) continue;
        ++rays;
        if (b.lo == kInf) ++infr;
        float nearest = kInf;
        bool past = false;
        for (int guard = 0; guard < 100000; ++guard) {
            ++steps;
            const size_t c = ((size_t)s.c2 * res[1] + s.c1) * res[0] + s.c0;
            if (fminf(s.tn0, fminf(s.tn1, s.tn2)) <= b.lo) ++below;      // exited below lo
            if (past) {
                ++above;
                if (cells[2 * c + 1] > cells[2 * c]) ++bad;
            }
            for (uint32_t j = cells[2 * c]; j < cells[2 * c + 1]; ++j) {
                const float* q = &tp[9ull * j];
                float t, u, v;
                if (tri_ray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]), o, d, &t, &u, &v))
                    if (nearest > t && t > 0.0f) nearest = t;
            }
            bool crossed;
            float te;
            DDA_STEP(s, g, 2, crossed, te);
            (void)crossed;
            if (nearest <= te) break;
            if (te >= b.hi) past = true;
        }
        if (nearest == kInf) ++misses;
    }
    printf("rays %llu (misses %.3f, in +inf blocks %.3f): steps/ray %.1f, exited below lo %.1f, after hi %.1f, "
           "occupied after hi %llu\n",
           (unsigned long long)rays, (double)misses / rays, (double)infr / rays, (double)steps / rays,
           (double)below / rays, (double)above / rays, (unsigned long long)bad);
    return bad ? 1 : 0;
}
