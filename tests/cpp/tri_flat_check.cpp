// Host check of tri_ray_flat (csrc/zrt_math.h): the branch-free Moller-Trumbore
// of the park kernel's test rounds must accept exactly the (ray, triangle)
// pairs tri_ray accepts, with bit-identical t, u, v - on random, degenerate,
// back-facing, edge-grazing and NaN/inf inputs.
//   g++ -O2 -std=c++17 -ffp-contract=off -I<csrc> tri_flat_check.cpp
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>

#include "zrt_math.h"

using namespace zrt;

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 rng(777);
    std::uniform_real_distribution<float> U(-2.0f, 2.0f);
    const float specials[] = {0.0f, -0.0f, 1.0f, -1.0f, 1e-8f, 1e-30f, kInf, -kInf, __builtin_nanf("")};
    long fails = 0, hits = 0;
    for (long i = 0; i < n; ++i) {
        float f[15];
        for (float& x : f) x = U(rng);
        const int kind = (int)(i % 8);
        if (kind == 1) { f[6] = f[3] * 0.5f; f[7] = f[4] * 0.5f; f[8] = f[5] * 0.5f; }          // degenerate
        if (kind == 2) f[(size_t)(rng() % 15)] = specials[rng() % 9];                          // specials
        if (kind == 3) { f[0] = f[1] = f[2] = 0.0f; f[3] = 1.0f; f[4] = f[5] = 0.0f;           // unit triangle,
                         f[6] = f[8] = 0.0f; f[7] = 1.0f; f[9] = f[10] = 0.25f * (float)(rng() % 5);  // ray on
                         f[11] = 1.0f; f[12] = f[13] = 0.0f; f[14] = -1.0f; }                // edges/corners
        const v3 v0 = mk(f[0], f[1], f[2]), e1 = mk(f[3], f[4], f[5]), e2 = mk(f[6], f[7], f[8]);
        const v3 o = mk(f[9], f[10], f[11]);
        const v3 d = kind == 3 ? mk(f[12], f[13], f[14]) : normalize(mk(f[12], f[13], f[14]));
        float t0 = 0, u0 = 0, w0 = 0, t1 = 0, u1 = 0, w1 = 0;
        const bool a = tri_ray(v0, e1, e2, o, d, &t0, &u0, &w0);
        const bool b = tri_ray_flat(v0, e1, e2, o, d, &t1, &u1, &w1);
        hits += a;
        if (a != b || (a && (memcmp(&t0, &t1, 4) || memcmp(&u0, &u1, 4) || memcmp(&w0, &w1, 4)))) {
            if (++fails <= 5) fprintf(stderr, "MISMATCH case %ld kind %d: %d vs %d\n", i, kind, a, b);
        }
    }
    printf("{\"pairs\": %ld, \"hits\": %ld, \"fails\": %ld}\n", n, hits, fails);
    return fails ? 1 : 0;
}
