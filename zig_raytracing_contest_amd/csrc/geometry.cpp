// geometry.cpp -- stage 2 of the reference (src/stage2.zig:44-164): scene
// bbox, uniform grid, SAT binning of triangles into cells, exclusive prefix
// sum, and the bake that DUPLICATES triangles into cell order.  This is the
// exact memory the render kernel reads, so it is parity-critical: the output
// must equal the single-threaded reference order (triangles within a cell in
// source order) bit for bit.
//
// MI355X-host design: the SAT tests (the O(sum of overlapped cells) part) run
// on all host threads over contiguous triangle chunks; each chunk records its
// (triangle -> cells) hits in order, and a stable counting pass in chunk order
// reproduces the reference's sequential fill exactly.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "geometry.h"

using namespace zrt;

namespace {

struct Chunk {
    uint32_t t0 = 0;
    std::vector<uint32_t> hit_cells;  // cell index of every (triangle, cell) overlap, triangle order
    std::vector<uint32_t> tri_hits;   // overlaps per triangle of the chunk
};

void bin_chunk(const Grid& g, const float* pos, uint32_t t0, uint32_t t1, Chunk* out) {
    out->hit_cells.clear();
    out->t0 = t0;
    out->tri_hits.assign(t1 - t0, 0);
    for (uint32_t t = t0; t < t1; ++t) {
        const float* p = pos + 9ull * t;
        const v3 a = ld3(p), b = ld3(p + 3), c = ld3(p + 6);
        // stage2.zig:65-66: vertex bbox -> cell range
        uint32_t lo[3], hi[3];
        grid_cell_idx(g, vmin(a, vmin(b, c)), lo);
        grid_cell_idx(g, vmax(a, vmax(b, c)), hi);
        for (uint32_t z = lo[2]; z <= hi[2]; ++z)
            for (uint32_t y = lo[1]; y <= hi[1]; ++y)
                for (uint32_t x = lo[0]; x <= hi[0]; ++x) {
                    const Bbox cb = grid_cell_bbox(g, x, y, z);
                    if (tri_aabb(a, b, c, cb)) {
                        out->hit_cells.push_back((z * g.res[1] + y) * g.res[0] + x);
                        out->tri_hits[t - t0] += 1;
                    }
                }
    }
}

}  // namespace

extern "C" int zrt_geometry_build(const float* positions, const float* normals,
                                  const float* texcoords, const uint32_t* material,
                                  uint32_t n, const uint32_t resolution[3],
                                  uint32_t num_threads, zrt_geometry** out) {
    if (!out) return ZRT_ERR_INVALID_ARG;
    *out = nullptr;
    const int arc = check_build_args(positions, normals, texcoords, material, n, resolution);
    if (arc != ZRT_OK) return arc;
    const uint64_t ncells64 = (uint64_t)resolution[0] * resolution[1] * resolution[2];
    zrt_geometry* geo = new (std::nothrow) zrt_geometry();
    if (!geo) return ZRT_ERR_OUT_OF_MEMORY;
    try {
        geo->grid = scene_grid(positions, n, resolution);   // stage2.zig:44-57
        geo->ncells = (uint32_t)ncells64;

        // SAT binning on host threads (stage2.zig:59-79 / 104-124)
        unsigned nt = num_threads ? num_threads : host_threads();
        nt = std::min<unsigned>(nt, 64);
        const uint32_t nchunks = std::min<uint32_t>(n, nt * 8);
        std::vector<Chunk> chunks(nchunks);
        std::atomic<uint32_t> next{0};
        auto work = [&]() {
            for (;;) {
                const uint32_t k = next.fetch_add(1);
                if (k >= nchunks) break;
                const uint32_t t0 = (uint32_t)((uint64_t)n * k / nchunks);
                const uint32_t t1 = (uint32_t)((uint64_t)n * (k + 1) / nchunks);
                bin_chunk(geo->grid, positions, t0, t1, &chunks[k]);
            }
        };
        std::vector<std::thread> pool;
        for (unsigned i = 1; i < nt; ++i) pool.emplace_back(work);
        work();
        for (auto& th : pool) th.join();

        // counts + exclusive prefix sum (stage2.zig:85-95)
        std::vector<uint32_t> first(geo->ncells, 0), fill(geo->ncells, 0);
        for (const Chunk& c : chunks)
            for (uint32_t ci : c.hit_cells) fill[ci] += 1;
        uint64_t total = 0;
        for (uint32_t c = 0; c < geo->ncells; ++c) {
            first[c] = (uint32_t)total;
            total += fill[c];
            fill[c] = 0;
        }
        if (total > 0xFFFFFFFFull) { delete geo; return ZRT_ERR_UNSUPPORTED; }
        // fill in triangle order (stage2.zig:104-124): chunks are contiguous
        // triangle ranges walked in order, and each chunk's hit list is in
        // (triangle, z, y, x) order -- exactly the reference's sequence.
        geo->indices.resize(total);
        for (uint32_t k = 0; k < nchunks; ++k) {
            const auto& hits = chunks[k].hit_cells;
            const auto& cnt = chunks[k].tri_hits;
            size_t h = 0;
            for (size_t j = 0; j < cnt.size(); ++j) {
                const uint32_t t = chunks[k].t0 + (uint32_t)j;
                for (uint32_t q = 0; q < cnt[j]; ++q, ++h) {
                    const uint32_t ci = hits[h];
                    geo->indices[first[ci] + fill[ci]] = t;
                    fill[ci] += 1;
                }
            }
        }
        // bakeInto (stage2.zig:137-164)
        geo->cells.resize(2ull * geo->ncells);
        for (uint32_t c = 0; c < geo->ncells; ++c) {
            geo->cells[2ull * c] = first[c];
            geo->cells[2ull * c + 1] = first[c] + fill[c];
        }
        const uint64_t refs = total;
        geo->pos.resize(9 * refs);
        geo->data.resize(15 * refs);
        geo->mat.resize(refs);
        auto bake = [&](uint64_t r0, uint64_t r1) {
            for (uint64_t i = r0; i < r1; ++i) {
                const uint32_t t = geo->indices[i];
                const float* p = positions + 9ull * t;
                const v3 v0 = ld3(p), v1 = ld3(p + 3), v2 = ld3(p + 6);
                const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
                float* q = &geo->pos[9 * i];
                q[0] = v0.x; q[1] = v0.y; q[2] = v0.z;
                q[3] = e1.x; q[4] = e1.y; q[5] = e1.z;
                q[6] = e2.x; q[7] = e2.y; q[8] = e2.z;
                memcpy(&geo->data[15 * i], normals + 9ull * t, 9 * sizeof(float));
                memcpy(&geo->data[15 * i + 9], texcoords + 6ull * t, 6 * sizeof(float));
                geo->mat[i] = material[t];
            }
        };
        pool.clear();
        for (unsigned i = 0; i < nt; ++i)
            pool.emplace_back(bake, refs * i / nt, refs * (i + 1) / nt);
        for (auto& th : pool) th.join();
    } catch (const std::bad_alloc&) {
        delete geo;
        return ZRT_ERR_OUT_OF_MEMORY;
    }
    *out = geo;
    return ZRT_OK;
}

extern "C" int zrt_geometry_scene(const zrt_geometry* g, zrt_scene* s) {
    if (!g || !s) return ZRT_ERR_INVALID_ARG;
    for (int i = 0; i < 3; ++i) {
        s->grid.bbox_min[i] = (&g->grid.bbox.min.x)[i];
        s->grid.bbox_max[i] = (&g->grid.bbox.max.x)[i];
        s->grid.resolution[i] = g->grid.res[i];
        s->grid.cell_size[i] = (&g->grid.cell_size.x)[i];
    }
    s->num_cells = g->ncells;
    s->cells = g->cells.data();
    s->num_triangles = (uint32_t)g->indices.size();
    s->triangles_pos = g->pos.data();
    s->triangles_data = g->data.data();
    s->triangles_material = g->mat.data();
    return ZRT_OK;
}

extern "C" int zrt_geometry_indices(const zrt_geometry* g, const uint32_t** idx, uint32_t* count) {
    if (!g || !idx || !count) return ZRT_ERR_INVALID_ARG;
    *idx = g->indices.data();
    *count = (uint32_t)g->indices.size();
    return ZRT_OK;
}

extern "C" void zrt_geometry_free(zrt_geometry* g) { delete g; }
