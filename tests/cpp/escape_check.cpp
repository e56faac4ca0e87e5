// Host check of the escape table (csrc/escape.h): on random grids
// (anisotropic cells, clustered occupancy so that many bits are set) and
// random rays, every cell the cell-by-cell walk (DDA_STEP, Iterator.next)
// visits after a cell whose brick has the ray's escape bit set must be
// empty.  Also checks the summed-area box query against a direct count.
//   g++ -O2 -std=c++17 -ffp-contract=off -I<csrc> escape_check.cpp
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "dda.h"
#include "escape.h"

using namespace zrt;

int main(int argc, char** argv) {
    const int n_grids = argc > 1 ? atoi(argv[1]) : 24;
    const int n_rays = argc > 2 ? atoi(argv[2]) : 20000;
    std::mt19937_64 rng(777);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    uint64_t rays = 0, escapes = 0, saved = 0, steps = 0, unsound = 0, box_fails = 0, bits_set = 0, bits = 0;
    for (int gi = 0; gi < n_grids; ++gi) {
        uint32_t res[3];
        float bmin[3], bmax[3], cs[3];
        for (int a = 0; a < 3; ++a) {
            res[a] = gi == 0 ? 64u : 4u + (uint32_t)(rng() % 60);
            bmin[a] = -5.0f + 10.0f * U(rng);
            cs[a] = 0.02f + U(rng);
            bmax[a] = bmin[a] + cs[a] * (float)res[a];
        }
        // occupancy: a few random blobs and planes
        std::vector<uint8_t> occ((size_t)res[0] * res[1] * res[2], 0);
        const int nblob = 1 + (int)(rng() % 6);
        for (int k = 0; k < nblob; ++k) {
            uint32_t c[3], r[3];
            for (int a = 0; a < 3; ++a) { c[a] = rng() % res[a]; r[a] = 1 + rng() % (res[a] / 4 + 1); }
            const bool plane = rng() % 3 == 0;
            if (plane) r[rng() % 3] = 0;
            for (uint32_t z = c[2] > r[2] ? c[2] - r[2] : 0; z <= std::min(res[2] - 1, c[2] + r[2]); ++z)
                for (uint32_t y = c[1] > r[1] ? c[1] - r[1] : 0; y <= std::min(res[1] - 1, c[1] + r[1]); ++y)
                    for (uint32_t x = c[0] > r[0] ? c[0] - r[0] : 0; x <= std::min(res[0] - 1, c[0] + r[0]); ++x)
                        if (plane || U(rng) < 0.3f) occ[((size_t)z * res[1] + y) * res[0] + x] = 1;
        }
        const uint32_t n0 = res[0] + 1, n1 = res[1] + 1, n2 = res[2] + 1;
        std::vector<uint32_t> sat((size_t)n0 * n1 * n2, 0);
        for (uint32_t z = 0; z < res[2]; ++z)
            for (uint32_t y = 0; y < res[1]; ++y)
                for (uint32_t x = 0; x < res[0]; ++x)
                    sat[((size_t)(z + 1) * n1 + y + 1) * n0 + x + 1] = occ[((size_t)z * res[1] + y) * res[0] + x];
        for (uint32_t z = 0; z < n2; ++z)          // prefix along x, then y, then z
            for (uint32_t y = 0; y < n1; ++y)
                for (uint32_t x = 1; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)z * n1 + y) * n0 + x - 1];
        for (uint32_t z = 0; z < n2; ++z)
            for (uint32_t y = 1; y < n1; ++y)
                for (uint32_t x = 0; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)z * n1 + y - 1) * n0 + x];
        for (uint32_t z = 1; z < n2; ++z)
            for (uint32_t y = 0; y < n1; ++y)
                for (uint32_t x = 0; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)(z - 1) * n1 + y) * n0 + x];
        EscSat S{sat.data(), n0, n0 * n1};
        for (int q = 0; q < 200; ++q) {            // box queries against a direct count
            uint32_t lo[3], hi[3];
            for (int a = 0; a < 3; ++a) {
                lo[a] = rng() % res[a];
                hi[a] = lo[a] + rng() % (res[a] - lo[a]);
            }
            uint32_t cnt = 0;
            for (uint32_t z = lo[2]; z <= hi[2]; ++z)
                for (uint32_t y = lo[1]; y <= hi[1]; ++y)
                    for (uint32_t x = lo[0]; x <= hi[0]; ++x) cnt += occ[((size_t)z * res[1] + y) * res[0] + x];
            if (esc_box(S, lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]) != cnt) ++box_fails;
        }
        const uint32_t nb[3] = {(res[0] + 3) / 4, (res[1] + 3) / 4, (res[2] + 3) / 4};
        std::vector<uint8_t> tab((size_t)nb[0] * nb[1] * nb[2] * kEscNBin);
        for (uint32_t bz = 0; bz < nb[2]; ++bz)
            for (uint32_t by = 0; by < nb[1]; ++by)
                for (uint32_t bx = 0; bx < nb[0]; ++bx)
                    for (uint32_t bin = 0; bin < kEscNBin; ++bin) {
                        const bool e = esc_compute(S, res, cs, bx, by, bz, bin);
                        tab[(((size_t)bz * nb[1] + by) * nb[0] + bx) * kEscNBin + bin] = e;
                        bits_set += e;
                        ++bits;
                    }
        const GridK k{res[0] - 1, res[1] - 1, res[2] - 1, res[0], res[0] * res[1]};
        for (int r = 0; r < n_rays; ++r) {
            float c[3];
            for (int a = 0; a < 3; ++a) {
                const float ext = bmax[a] - bmin[a];
                c[a] = r % 3 == 0 ? bmin[a] - 0.5f * ext + 2.0f * ext * U(rng) : bmin[a] + ext * U(rng);
                if (r % 7 == 0) c[a] = bmin[a] + cs[a] * (float)(rng() % (res[a] + 1));   // on cell corners
            }
            v3 d;
            if (r % 5 == 0) {                                                          // diagonals: face ties
                d = normalize(mk((rng() & 1) ? 1.0f : -1.0f, (rng() & 1) ? 1.0f : -1.0f, (rng() & 1) ? 1.0f : -1.0f));
            } else {
                d = normalize(mk(U(rng) - 0.5f, U(rng) - 0.5f, U(rng) - 0.5f));
            }
            Dda s;
            if (!dda_init(bmin, bmax, res, cs, mk(c[0], c[1], c[2]), d, s)) continue;
            ++rays;
            const bool usable = s.neg < 8u;
            const uint32_t bin = esc_dir_bin(d);
            bool escaped = false;
            for (int guard = 0; guard < 100000; ++guard) {
                ++steps;
                const bool o = occ[((size_t)s.c2 * res[1] + s.c1) * res[0] + s.c0] != 0;
                if (escaped) {
                    ++saved;
                    if (o) { ++unsound; break; }
                }
                const size_t brk = ((size_t)(s.c2 / 4) * nb[1] + s.c1 / 4) * nb[0] + s.c0 / 4;
                if (!escaped && usable && tab[brk * kEscNBin + bin]) { escaped = true; ++escapes; }
                bool crossed;
                float te;
                DDA_STEP(s, k, 2, crossed, te);
                (void)crossed;
                if (te == kInf) break;
            }
        }
    }
    // the primary frustum bounds: per 8x8 pixel block of a random camera, no
    // ray of the block (random jitter, the kernel's f32 ray) enters an
    // occupied cell at a crossing below the block's lo bound, nor starts in one
    // before it (a +inf bound: the ray enters no occupied cell at all), nor
    // at a crossing at or past its hi bound
    uint64_t f_rays = 0, f_skipped = 0, f_steps = 0, f_unsound = 0, f_miss_blocks = 0, f_blocks = 0;
    uint64_t f_far = 0, f_far_unsound = 0, f_gap = 0, f_gap_unsound = 0, f_gap_blocks = 0;
    for (int gi = 0; gi < n_grids; ++gi) {
        uint32_t res[3];
        float bmin[3], bmax[3], cs[3];
        for (int a = 0; a < 3; ++a) {
            res[a] = 8u + (uint32_t)(rng() % 56);
            bmin[a] = -5.0f + 10.0f * U(rng);
            cs[a] = 0.02f + U(rng);
            bmax[a] = bmin[a] + cs[a] * (float)res[a];
        }
        std::vector<uint8_t> occ((size_t)res[0] * res[1] * res[2], 0);
        const int nblob = 1 + (int)(rng() % 5);
        for (int k = 0; k < nblob; ++k) {
            uint32_t c[3], r[3];
            for (int a = 0; a < 3; ++a) { c[a] = rng() % res[a]; r[a] = rng() % (res[a] / 6 + 1); }
            for (uint32_t z = c[2] > r[2] ? c[2] - r[2] : 0; z <= std::min(res[2] - 1, c[2] + r[2]); ++z)
                for (uint32_t y = c[1] > r[1] ? c[1] - r[1] : 0; y <= std::min(res[1] - 1, c[1] + r[1]); ++y)
                    for (uint32_t x = c[0] > r[0] ? c[0] - r[0] : 0; x <= std::min(res[0] - 1, c[0] + r[0]); ++x)
                        occ[((size_t)z * res[1] + y) * res[0] + x] = 1;
        }
        const uint32_t n0 = res[0] + 1, n1 = res[1] + 1, n2 = res[2] + 1;
        std::vector<uint32_t> sat((size_t)n0 * n1 * n2, 0);
        for (uint32_t z = 0; z < res[2]; ++z)
            for (uint32_t y = 0; y < res[1]; ++y)
                for (uint32_t x = 0; x < res[0]; ++x)
                    sat[((size_t)(z + 1) * n1 + y + 1) * n0 + x + 1] = occ[((size_t)z * res[1] + y) * res[0] + x];
        for (uint32_t z = 0; z < n2; ++z)
            for (uint32_t y = 0; y < n1; ++y)
                for (uint32_t x = 1; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)z * n1 + y) * n0 + x - 1];
        for (uint32_t z = 0; z < n2; ++z)
            for (uint32_t y = 1; y < n1; ++y)
                for (uint32_t x = 0; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)z * n1 + y - 1) * n0 + x];
        for (uint32_t z = 1; z < n2; ++z)
            for (uint32_t y = 0; y < n1; ++y)
                for (uint32_t x = 0; x < n0; ++x) sat[((size_t)z * n1 + y) * n0 + x] += sat[((size_t)(z - 1) * n1 + y) * n0 + x];
        EscSat S{sat.data(), n0, n0 * n1};
        const GridK k{res[0] - 1, res[1] - 1, res[2] - 1, res[0], res[0] * res[1]};
        for (int cam = 0; cam < 4; ++cam) {
            // camera: outside or inside the grid, looking at a random grid point
            float org[3], tgt[3];
            for (int a = 0; a < 3; ++a) {
                const float ext = bmax[a] - bmin[a];
                org[a] = cam % 2 ? bmin[a] + ext * U(rng) : bmin[a] - ext + 3.0f * ext * U(rng);
                tgt[a] = bmin[a] + ext * U(rng);
            }
            const uint32_t W = 64, H = 48;
            const v3 f = normalize(mk(tgt[0] - org[0], tgt[1] - org[1], tgt[2] - org[2]));
            v3 rt = cross(f, mk(0.3f, 1.0f, 0.2f));
            rt = normalize(rt);
            const v3 upn = cross(rt, f);
            const float px = (0.2f + U(rng)) / (float)W;      // image plane width ~0.2-1.2 at distance 1
            const v3 right = scale(rt, px), upv = scale(upn, px);
            const v3 llc = sub(sub(f, scale(right, 0.5f * W)), scale(upv, 0.5f * H));
            const float llc_[3] = {llc.x, llc.y, llc.z}, right_[3] = {right.x, right.y, right.z},
                        up_[3] = {upv.x, upv.y, upv.z};
            for (uint32_t by = 0; by < H / 8; ++by)
                for (uint32_t bx = 0; bx < W / 8; ++bx) {
                    const FrustumBound fb = frustum_bound(S, res, bmin, bmax, cs, org, llc_, right_, up_, 8.0 * bx,
                                                          8.0 * bx + 8.0, 8.0 * by, 8.0 * by + 8.0);
                    const float tlo = fb.lo, thi = fb.hi, ga = fb.ga, gb = fb.gb;
                    f_gap_blocks += ga < gb;
                    ++f_blocks;
                    f_miss_blocks += tlo == kInf;
                    for (int r = 0; r < 40; ++r) {
                        const float ux = (float)(8 * bx + rng() % 8) + U(rng), vy = (float)(8 * by + rng() % 8) + U(rng);
                        const v3 o = mk(org[0], org[1], org[2]);
                        const v3 d = normalize(add(add(llc, scale(right, ux)), scale(upv, vy)));
                        Dda s;
                        if (!dda_init(bmin, bmax, res, cs, o, d, s)) continue;
                        ++f_rays;
                        float tin = 0.0f;              // the t the current cell was entered at
                        {
                            Bbox bb;
                            bb.min = mk(bmin[0], bmin[1], bmin[2]);
                            bb.max = mk(bmax[0], bmax[1], bmax[2]);
                            bbox_ray(bb, o, d, &tin);
                            tin = fmaxf(0.0f, tin);
                        }
                        for (int guard = 0; guard < 100000; ++guard) {
                            ++f_steps;
                            const bool o_ = occ[((size_t)s.c2 * res[1] + s.c1) * res[0] + s.c0] != 0;
                            if (tin < tlo) {
                                ++f_skipped;
                                if (o_) { ++f_unsound; break; }
                            }
                            if (guard > 0 && tin >= thi) {       // entered past the far bound
                                ++f_far;
                                if (o_) { ++f_far_unsound; break; }
                            }
                            if (guard > 0 && tin >= ga && tin < gb) {   // entered inside the gap
                                ++f_gap;
                                if (o_) { ++f_gap_unsound; break; }
                            }
                            bool crossed;
                            float te;
                            const float tc = fminf(s.tn0, fminf(s.tn1, s.tn2));
                            DDA_STEP(s, k, 2, crossed, te);
                            (void)crossed;
                            if (te == kInf) break;
                            tin = tc;
                        }
                    }
                }
        }
    }
    printf("{\"frustum_blocks\": %llu, \"frustum_miss_blocks\": %llu, \"frustum_rays\": %llu, \"frustum_steps\": %llu, "
           "\"frustum_cells_below_bound\": %llu, \"frustum_unsound\": %llu, \"frustum_cells_past_far\": %llu, "
           "\"frustum_far_unsound\": %llu, \"frustum_gap_blocks\": %llu, \"frustum_cells_in_gap\": %llu, "
           "\"frustum_gap_unsound\": %llu}\n",
           (unsigned long long)f_blocks, (unsigned long long)f_miss_blocks, (unsigned long long)f_rays,
           (unsigned long long)f_steps, (unsigned long long)f_skipped, (unsigned long long)f_unsound,
           (unsigned long long)f_far, (unsigned long long)f_far_unsound, (unsigned long long)f_gap_blocks,
           (unsigned long long)f_gap, (unsigned long long)f_gap_unsound);
    unsound += f_unsound + f_far_unsound + f_gap_unsound;
    // flat grids (a zero or non-finite cell_size axis, linalg.zig:412-441 on
    // coplanar scenes): no escape bit and no frustum bound, whatever the
    // occupancy (the kernels' guard against dividing by them)
    uint64_t flat_bits = 0, flat_bounds = 0;
    {
        const uint32_t fres[3] = {8, 8, 8};
        std::vector<uint32_t> fsat(9 * 9 * 9, 0u);    // an empty grid: every bit would be set
        const EscSat FS{fsat.data(), 9u, 81u};
        const float bad[4][3] = {{0.5f, 0.5f, 0.0f}, {0.0f, 0.5f, 0.5f}, {0.0f, 0.0f, 0.0f},
                                 {0.5f, kInf, 0.5f}};
        for (const auto& c3 : bad) {
            for (uint32_t bin = 0; bin < kEscNBin; ++bin) flat_bits += esc_compute(FS, fres, c3, 0, 1, 0, bin);
            const float fbmin[3] = {0, 0, 0}, fbmax[3] = {4 * c3[0], 4 * c3[1], 4 * c3[2]};
            const float forg[3] = {-1, -2, -3}, fllc[3] = {1, 2, 3}, fr[3] = {0.01f, 0, 0}, fu[3] = {0, 0.01f, 0};
            const FrustumBound fb = frustum_bound(FS, fres, fbmin, fbmax, c3, forg, fllc, fr, fu, 0, 8, 0, 8);
            flat_bounds += !(fb.lo == 0.0f && fb.hi == kInf);
        }
    }
    printf("{\"flat_grid_bits\": %llu, \"flat_grid_bounds\": %llu}\n", (unsigned long long)flat_bits,
           (unsigned long long)flat_bounds);
    unsound += flat_bits + flat_bounds;
    printf("{\"rays\": %llu, \"steps\": %llu, \"escapes\": %llu, \"steps_after_escape\": %llu, \"bits_set\": %.4f, "
           "\"unsound\": %llu, \"box_fails\": %llu}\n",
           (unsigned long long)rays, (unsigned long long)steps, (unsigned long long)escapes,
           (unsigned long long)saved, bits ? (double)bits_set / bits : 0.0, (unsigned long long)unsound,
           (unsigned long long)box_fails);
    return unsound || box_fails ? 1 : 0;
}
