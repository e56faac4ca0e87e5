// Host model of traceRay's grid walk (stage3.zig:152-185, linalg.zig:443-496)
// for planning the empty-brick skip: per ray, the cells Iterator.next visits,
// how many of them lie in empty 4^3 bricks, and how many empty bricks the walk
// enters.  Also emits the hit (t, ref) so the caller can spawn bounce rays.
//   g++ -O2 -std=c++17 -ffp-contract=off -Izig_raytracing_contest_amd/csrc -Iinclude tools/walk_sim.cpp -o /tmp/walk_sim
//   walk_sim <scene.bin> <rays.bin> <out.bin>
// scene.bin: bbox[6] f32, res[3] u32, cs[3] f32, ncells u32, nrefs u32,
//            cells (begin, end) u32 x ncells, tri_pos 9 f32 x nrefs (v0, e1, e2)
// rays.bin:  n u32, then (o, d) 6 f32 x n
// out.bin:   per ray: steps u16 | first occupied-cell step << 16, empty_steps u32, empty_entries u32,
//            occ_steps u16 | last occupied-brick step << 16, t f32, ref u32
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dda.h"

using namespace zrt;

int main(int argc, char** argv) {
    if (argc != 4) return 2;
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
    const uint32_t bx = (res[0] + 3) / 4, by = (res[1] + 3) / 4, bz = (res[2] + 3) / 4;
    std::vector<uint8_t> brick(bx * by * bz, 0);
    for (uint32_t z = 0; z < res[2]; ++z)
        for (uint32_t y = 0; y < res[1]; ++y)
            for (uint32_t x = 0; x < res[0]; ++x) {
                const uint32_t c = (z * res[1] + y) * res[0] + x;
                if (cells[2 * c + 1] > cells[2 * c]) brick[((z / 4) * by + y / 4) * bx + x / 4] = 1;
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
    std::vector<uint32_t> out(6ull * n);
    for (uint32_t r = 0; r < n; ++r) {
        const v3 o = mk(rays[6 * r], rays[6 * r + 1], rays[6 * r + 2]);
        const v3 d = mk(rays[6 * r + 3], rays[6 * r + 4], rays[6 * r + 5]);
        float nearest = kInf;
        uint32_t hidx = ~0u, steps = 0, esteps = 0, eent = 0, osteps = 0, lastocc = 0, firstocc = 0;
        Dda s;
        if (dda_init(bmin, bmax, res, cs, o, d, s)) {
            uint32_t pb = ~0u;
            for (;;) {
                const uint32_t b = ((s.c2 / 4) * by + s.c1 / 4) * bx + s.c0 / 4;
                ++steps;
                if (!brick[b]) {
                    ++esteps;
                    if (b != pb) ++eent;
                } else {
                    ++osteps;
                    lastocc = steps;
                }
                pb = b;
                if (!firstocc && cells[2 * s.lin + 1] > cells[2 * s.lin]) firstocc = steps;
                for (uint32_t j = cells[2 * s.lin]; j < cells[2 * s.lin + 1]; ++j) {
                    const float* q = &tp[9ull * j];
                    float t, u, v;
                    if (tri_ray(mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), mk(q[6], q[7], q[8]), o, d, &t, &u, &v))
                        if (nearest > t && t > 0.0f) { nearest = t; hidx = j; }
                }
                bool crossed;
                float te;
                DDA_STEP(s, g, 2, crossed, te);
                (void)crossed;
                if (nearest <= te) break;
            }
        }
        uint32_t* w = &out[6ull * r];
        w[0] = steps | (firstocc << 16); w[1] = esteps; w[2] = eent; w[3] = osteps | (lastocc << 16);
        memcpy(&w[4], &nearest, 4);
        w[5] = hidx;
    }
    f = fopen(argv[3], "wb");
    fwrite(out.data(), 24, n, f);
    fclose(f);
    return 0;
}
