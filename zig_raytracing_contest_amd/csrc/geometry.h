// geometry.h -- the stage-2 result (Geometry.build + bakeInto,
// src/stage2.zig:44-164) shared by the host build (geometry.cpp) and the
// device build (grid_build.hip).
#pragma once

#include <vector>

#include "zrt_internal.h"

struct zrt_geometry {
    zrt::Grid grid;
    uint32_t ncells = 0;
    std::vector<uint32_t> cells;     // 2*ncells {begin, end}
    std::vector<uint32_t> indices;   // refs -> source triangle
    std::vector<float> pos;          // refs*9 : v0, e1, e2
    std::vector<float> data;         // refs*15
    std::vector<uint32_t> mat;       // refs
};

namespace zrt {

// stage2.zig:44-57 initGrid: scene bbox over every vertex in order, then
// Grid.init.  Sequential on purpose: fminf/fmaxf in the reference's order
// (signed zeros included); ~1 ms for 300k triangles.
inline Grid scene_grid(const float* positions, uint32_t n, const uint32_t res[3]) {
    Bbox bb{mk(kInf, kInf, kInf), mk(-kInf, -kInf, -kInf)};
    for (uint64_t i = 0; i < 3ull * n; ++i) {
        const v3 p = ld3(positions + 3 * i);
        bb.min = vmin(bb.min, p);
        bb.max = vmax(bb.max, p);
    }
    return grid_init(bb, res);
}

// Argument checks shared by both builds.
inline int check_build_args(const float* positions, const float* normals, const float* texcoords,
                            const uint32_t* material, uint32_t n, const uint32_t* resolution) {
    if (!positions || !normals || !texcoords || !material || !resolution || n == 0) return ZRT_ERR_INVALID_ARG;
    const uint64_t ncells = (uint64_t)resolution[0] * resolution[1] * resolution[2];
    if (resolution[0] == 0 || resolution[1] == 0 || resolution[2] == 0 || ncells > 0x7FFFFFFFull)
        return ZRT_ERR_INVALID_ARG;
    return ZRT_OK;
}

}  // namespace zrt
