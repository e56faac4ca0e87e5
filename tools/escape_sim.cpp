// Host model of an escape table for traceRay's grid walk: per 4^3 brick and
// direction bin, whether every ray that starts in the brick with a direction
// in the bin leaves the grid through empty cells only (its swept region,
// dilated by one cell, holds no occupied cell).  A walk that reaches such a
// brick can stop there: no later cell holds a triangle, so traceRay's result
// is the nearest hit so far (stage3.zig:152-185).  Reports, per ray, the
// steps the walk would save and checks soundness (no occupied cell visited
// after the escape point).
//   g++ -O2 -std=c++17 -fopenmp -ffp-contract=off -Izig_raytracing_contest_amd/csrc -Iinclude tools/escape_sim.cpp -o /tmp/escape_sim
//   escape_sim <scene.bin> <rays.bin> <out.bin> [bins_per_face_axis=4]
// out.bin: per ray: steps u32, saved u32, unsound u32
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dda.h"

using namespace zrt;

struct Esc {
    uint32_t res[3], nb[3], nbin;   // nbin per face axis
    std::vector<uint32_t> pre[3];   // per axis a: per cell slab, 2-D inclusive prefix sums over the other two axes
    std::vector<uint8_t> bits;      // [brick][6 * nbin * nbin]
};

// direction bin: face = dominant axis and sign, (u, v) = the other two
// components over |d_a| in [-1, 1], nbin x nbin cells
static uint32_t dir_bin(v3 d, uint32_t nbin) {
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    uint32_t a;
    float m, u, v;
    if (ax >= ay && ax >= az) { a = 0; m = d.x; u = d.y / ax; v = d.z / ax; }
    else if (ay >= az) { a = 1; m = d.y; u = d.x / ay; v = d.z / ay; }
    else { a = 2; m = d.z; u = d.x / az; v = d.y / az; }
    const uint32_t f = 2 * a + (m < 0.0f ? 1 : 0);
    uint32_t iu = (uint32_t)fminf(fmaxf((u + 1.0f) * 0.5f * nbin, 0.0f), nbin - 1.0f);
    uint32_t iv = (uint32_t)fminf(fmaxf((v + 1.0f) * 0.5f * nbin, 0.0f), nbin - 1.0f);
    return (f * nbin + iu) * nbin + iv;
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const uint32_t nbin = argc > 4 ? atoi(argv[4]) : 4;
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
    auto occ = [&](uint32_t x, uint32_t y, uint32_t z) {
        const uint32_t c = (z * res[1] + y) * res[0] + x;
        return cells[2 * c + 1] > cells[2 * c];
    };
    Esc E;
    for (int a = 0; a < 3; ++a) { E.res[a] = res[a]; E.nb[a] = (res[a] + 3) / 4; }
    E.nbin = nbin;
    // prefix sums: axis a's slab i, 2-D over (b, c) = the other axes in order
    for (int a = 0; a < 3; ++a) {
        const int b = a == 0 ? 1 : 0, c = a == 2 ? 1 : 2;
        const uint32_t R = res[b] + 1, S = res[c] + 1;
        E.pre[a].assign((size_t)res[a] * R * S, 0);
        for (uint32_t i = 0; i < res[a]; ++i)
            for (uint32_t y = 0; y < res[b]; ++y)
                for (uint32_t z = 0; z < res[c]; ++z) {
                    uint32_t p[3];
                    p[a] = i; p[b] = y; p[c] = z;
                    uint32_t* P = &E.pre[a][(size_t)i * R * S];
                    P[(y + 1) * S + z + 1] = (occ(p[0], p[1], p[2]) ? 1 : 0) + P[y * S + z + 1] + P[(y + 1) * S + z] -
                                             P[y * S + z];
                }
    }
    const uint32_t nbr = E.nb[0] * E.nb[1] * E.nb[2], nb6 = 6 * nbin * nbin;
    E.bits.assign((size_t)nbr * nb6, 0);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t br = 0; br < (int64_t)nbr; ++br) {
        const uint32_t B[3] = {(uint32_t)(br % E.nb[0]), (uint32_t)((br / E.nb[0]) % E.nb[1]),
                               (uint32_t)(br / (E.nb[0] * E.nb[1]))};
        for (uint32_t bin = 0; bin < nb6; ++bin) {
            const uint32_t fc = bin / (nbin * nbin), iu = (bin / nbin) % nbin, iv = bin % nbin;
            const int a = fc / 2, sg = (fc & 1) ? -1 : 1;
            const int b = a == 0 ? 1 : 0, c = a == 2 ? 1 : 2;
            const double eps = 1e-3;
            const double u0 = -1.0 + 2.0 * iu / nbin - eps, u1 = -1.0 + 2.0 * (iu + 1) / nbin + eps;
            const double v0 = -1.0 + 2.0 * iv / nbin - eps, v1 = -1.0 + 2.0 * (iv + 1) / nbin + eps;
            // the brick in cell units
            const double lo[3] = {4.0 * B[0], 4.0 * B[1], 4.0 * B[2]};
            const double hi[3] = {fmin(4.0 * B[0] + 4, res[0]), fmin(4.0 * B[1] + 4, res[1]), fmin(4.0 * B[2] + 4, res[2])};
            bool ok = true;
            const uint32_t R = res[b] + 1, S = res[c] + 1;
            for (int i = sg > 0 ? (int)lo[a] : (int)hi[a] - 1; ok && i >= 0 && i < (int)res[a]; i += sg) {
                // a-distance from the brick to slab i (cell units)
                double smin, smax;
                if (sg > 0) { smin = fmax(0.0, i - hi[a]); smax = fmax(0.0, i + 1 - lo[a]); }
                else { smin = fmax(0.0, lo[a] - (i + 1)); smax = fmax(0.0, hi[a] - i); }
                // (u, v are slopes in world units: a cell-unit step along a moves
                // cs_a / cs_b cells along b)
                const double kb = (double)cs[a] / cs[b], kc = (double)cs[a] / cs[c];
                const double ylo = lo[b] + kb * fmin(smin * u0, smax * u0), yhi = hi[b] + kb * fmax(smin * u1, smax * u1);
                const double zlo = lo[c] + kc * fmin(smin * v0, smax * v0), zhi = hi[c] + kc * fmax(smin * v1, smax * v1);
                // cells overlapping [ylo, yhi] dilated by one cell
                const int y0 = (int)std::max(0.0, floor(ylo) - 1), y1 = (int)std::min((double)res[b] - 1, ceil(yhi));
                const int z0 = (int)std::max(0.0, floor(zlo) - 1), z1 = (int)std::min((double)res[c] - 1, ceil(zhi));
                if (y0 > y1 || z0 > z1) break;       // the region has left the grid sideways
                const uint32_t* P = &E.pre[a][(size_t)i * R * S];
                const uint32_t cnt = P[(y1 + 1) * S + z1 + 1] - P[y0 * S + z1 + 1] - P[(y1 + 1) * S + z0] + P[y0 * S + z0];
                if (cnt) ok = false;
            }
            E.bits[(size_t)br * nb6 + bin] = ok;
        }
    }
    uint64_t nesc = 0;
    for (auto x : E.bits) nesc += x;
    fprintf(stderr, "escape bits set: %.3f of %u x %u\n", (double)nesc / E.bits.size(), nbr, nb6);

    f = fopen(argv[2], "rb");
    uint32_t n;
    if (fread(&n, 4, 1, f) != 1) return 3;
    std::vector<float> rays(6ull * n);
    if (fread(rays.data(), 24, n, f) != n) return 3;
    fclose(f);
    GridK g;
    g.rm0 = res[0] - 1; g.rm1 = res[1] - 1; g.rm2 = res[2] - 1;
    g.str1 = res[0]; g.str2 = res[0] * res[1];
    std::vector<uint32_t> out(3ull * n);
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t r = 0; r < (int64_t)n; ++r) {
        const v3 o = mk(rays[6 * r], rays[6 * r + 1], rays[6 * r + 2]);
        const v3 d = mk(rays[6 * r + 3], rays[6 * r + 4], rays[6 * r + 5]);
        const uint32_t bin = dir_bin(d, nbin);
        float nearest = kInf;
        uint32_t steps = 0, esc_at = 0, unsound = 0;
        bool escaped = false;
        Dda s;
        if (dda_init(bmin, bmax, res, cs, o, d, s)) {
            for (;;) {
                const uint32_t brk = ((s.c2 / 4) * E.nb[1] + s.c1 / 4) * E.nb[0] + s.c0 / 4;
                ++steps;
                struct { uint32_t x, y; } cr = {cells[2 * s.lin], cells[2 * s.lin + 1]};
                if (escaped && cr.y > cr.x) unsound = 1;
                for (uint32_t j = cr.x; j < cr.y; ++j) {
                    const float* q = &tp[9ull * j];
                    float t, u, v;
                    if (tri_ray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]), o, d, &t, &u, &v))
                        if (nearest > t && t > 0.0f) nearest = t;
                }
                if (!escaped && E.bits[(size_t)brk * nb6 + bin]) { escaped = true; esc_at = steps; }
                bool crossed;
                float te;
                DDA_STEP(s, g, 2, crossed, te);
                (void)crossed;
                if (nearest <= te) break;
            }
        }
        out[3 * r] = steps;
        out[3 * r + 1] = escaped ? steps - esc_at : 0;
        out[3 * r + 2] = unsound;
    }
    f = fopen(argv[3], "wb");
    fwrite(out.data(), 12, n, f);
    fclose(f);
    return 0;
}
