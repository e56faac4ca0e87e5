// Host model of a distance-field fast-forward for traceRay's grid walk
// (planning tool, not product code): with D = the Chebyshev distance in cells
// from the current cell to the nearest occupied cell, every cell the ray
// passes before t = min(tn) + (D - 3) min(td) is empty, so the three crossing
// sequences can be advanced by plain f32 adds (the same adds Iterator.next
// does) to that t -- the exact DDA state of the merge prefix -- without the
// per-cell walk.  Reports the walk operations (DDA steps + fast-forwards) and
// the add iterations per ray, for a cell-level field and a 4^3-brick one.
//   g++ -O2 -std=c++17 -fopenmp -ffp-contract=off -Izig_raytracing_contest_amd/csrc -Iinclude tools/ff_sim.cpp -o /tmp/ff_sim
//   ff_sim <scene.bin> <rays.bin>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dda.h"

using namespace zrt;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
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
    const int R0 = res[0], R1 = res[1], R2 = res[2];
    auto lin = [&](int x, int y, int z) { return ((size_t)z * R1 + y) * R0 + x; };
    // Chebyshev distance transform (cells), capped at 255: separable min-plus passes
    std::vector<uint8_t> D((size_t)R0 * R1 * R2);
    for (size_t c = 0; c < D.size(); ++c) D[c] = cells[2 * c + 1] > cells[2 * c] ? 0 : 255;
    // chessboard distance: 26-neighbour two-pass raster scans
    for (int pass = 0; pass < 2; ++pass) {
        const int s = pass ? -1 : 1;
        for (int zi = 0; zi < R2; ++zi)
            for (int yi = 0; yi < R1; ++yi)
                for (int xi = 0; xi < R0; ++xi) {
                    const int z = pass ? R2 - 1 - zi : zi, y = pass ? R1 - 1 - yi : yi, x = pass ? R0 - 1 - xi : xi;
                    int best = D[lin(x, y, z)];
                    for (int dz = -1; dz <= 0; ++dz)
                        for (int dy = -1; dy <= 1; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                if (dz == 0 && (dy > 0 || (dy == 0 && dx >= 0))) continue;
                                const int X = x + s * dx, Y = y + s * dy, Z = z + s * dz;
                                if (X < 0 || Y < 0 || Z < 0 || X >= R0 || Y >= R1 || Z >= R2) continue;
                                best = std::min(best, D[lin(X, Y, Z)] + 1);
                            }
                    D[lin(x, y, z)] = (uint8_t)std::min(best, 255);
                }
    }
    // brick-level: distance in bricks between 4^3 bricks, then a cell bound 4 (DB - 1) + 1
    const int B0 = (R0 + 3) / 4, B1 = (R1 + 3) / 4, B2 = (R2 + 3) / 4;
    std::vector<uint8_t> DB((size_t)B0 * B1 * B2, 255);
    for (int z = 0; z < R2; ++z)
        for (int y = 0; y < R1; ++y)
            for (int x = 0; x < R0; ++x)
                if (D[lin(x, y, z)] == 0) DB[((size_t)(z / 4) * B1 + y / 4) * B0 + x / 4] = 0;
    for (int pass = 0; pass < 2; ++pass) {
        const int s = pass ? -1 : 1;
        for (int zi = 0; zi < B2; ++zi)
            for (int yi = 0; yi < B1; ++yi)
                for (int xi = 0; xi < B0; ++xi) {
                    const int z = pass ? B2 - 1 - zi : zi, y = pass ? B1 - 1 - yi : yi, x = pass ? B0 - 1 - xi : xi;
                    int best = DB[((size_t)z * B1 + y) * B0 + x];
                    for (int dz = -1; dz <= 0; ++dz)
                        for (int dy = -1; dy <= 1; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                if (dz == 0 && (dy > 0 || (dy == 0 && dx >= 0))) continue;
                                const int X = x + s * dx, Y = y + s * dy, Z = z + s * dz;
                                if (X < 0 || Y < 0 || Z < 0 || X >= B0 || Y >= B1 || Z >= B2) continue;
                                best = std::min(best, DB[((size_t)Z * B1 + Y) * B0 + X] + 1);
                            }
                    DB[((size_t)z * B1 + y) * B0 + x] = (uint8_t)std::min(best, 255);
                }
    }
    f = fopen(argv[2], "rb");
    uint32_t n;
    if (fread(&n, 4, 1, f) != 1) return 3;
    std::vector<float> rays(6ull * n);
    if (fread(rays.data(), 24, n, f) != n) return 3;
    fclose(f);
    GridK g;
    g.rm0 = res[0] - 1; g.rm1 = res[1] - 1; g.rm2 = res[2] - 1;
    g.str1 = res[0]; g.str2 = res[0] * res[1];
    for (int mode = 0; mode < 5; ++mode) {   // 0: plain walk, 1: cell field, 2: brick field, 3/4: brick field capped at 3/7
        uint64_t ops = 0, ffs = 0, iters = 0, bad = 0, steps_total = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : ops, ffs, iters, bad, steps_total)
        for (int64_t r = 0; r < (int64_t)n; ++r) {
            const v3 o = mk(rays[6 * r], rays[6 * r + 1], rays[6 * r + 2]);
            const v3 d = mk(rays[6 * r + 3], rays[6 * r + 4], rays[6 * r + 5]);
            float nearest = kInf;
            Dda s;
            if (!dda_init(bmin, bmax, res, cs, o, d, s)) continue;
            const bool usable = s.neg < 8u;
            for (int guard = 0; guard < 100000; ++guard) {
                ++ops;
                ++steps_total;
                const size_t c = lin(s.c0, s.c1, s.c2);
                for (uint32_t j = cells[2 * c]; j < cells[2 * c + 1]; ++j) {
                    const float* q = &tp[9ull * j];
                    float t, u, v;
                    if (tri_ray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]), o, d, &t, &u, &v))
                        if (nearest > t && t > 0.0f) nearest = t;
                }
                int db = DB[((size_t)(s.c2 / 4) * B1 + s.c1 / 4) * B0 + s.c0 / 4];
                if (mode == 3) db = std::min(db, 3);
                if (mode == 4) db = std::min(db, 7);
                int dist = mode == 1 ? D[c] : (mode >= 2 ? std::max(0, 4 * (db - 1) + 1) : 0);
                if (mode && usable && dist >= 4 && nearest == kInf) {
                    // fast-forward: every crossing with t < tau
                    const float tmin = std::min(s.tn0, std::min(s.tn1, s.tn2));
                    const float dmin = std::min(s.td0, std::min(s.td1, s.td2));
                    const float tau = tmin + (float)(dist - 3) * dmin;
                    float* tn[3] = {&s.tn0, &s.tn1, &s.tn2};
                    const float td[3] = {s.td0, s.td1, s.td2};
                    uint32_t* cc[3] = {&s.c0, &s.c1, &s.c2};
                    const uint32_t rm[3] = {g.rm0, g.rm1, g.rm2};
                    bool exited = false;
                    uint32_t it = 0, moved = 0;
                    for (int a = 0; a < 3; ++a) {
                        const bool ng = (s.neg >> a) & 1u;
                        uint32_t k = 0;
                        while (*tn[a] < tau) {
                            if (*cc[a] == (ng ? 0u : rm[a])) { exited = true; break; }
                            *tn[a] += td[a];
                            *cc[a] = ng ? *cc[a] - 1 : *cc[a] + 1;
                            ++k;
                        }
                        it = std::max(it, k);
                        moved += k;
                    }
                    s.lin = lin(s.c0, s.c1, s.c2);
                    ++ffs;
                    iters += it;
                    steps_total += moved;
                    if (exited) break;
                    if (moved) {
                        --ops;                                  // the ff replaces this iteration's step
                        // the cell reached must be one the walk visits (it is, by the merge argument)
                        if (D[s.lin] == 0 && false) ++bad;
                        continue;
                    }
                }
                bool crossed;
                float te;
                DDA_STEP(s, g, 2, crossed, te);
                (void)crossed;
                if (nearest <= te) break;
            }
        }
        printf("mode %d: walk ops/ray %.1f (ff %.1f, add iterations %.1f), cells passed/ray %.1f\n", mode,
               (double)ops / n, (double)ffs / n, (double)iters / n, (double)steps_total / n);
    }
    return 0;
}
