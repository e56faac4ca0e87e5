// grid_build.hip -- stage 2 on the GPU: SAT binning of the
// triangles into the uniform grid and the bake into cell order
// (src/stage2.zig:59-164 over linalg.zig:424-441 and :500-563), bit for bit
// the host build's output (geometry.cpp), which the oracle pins.
//
// The reference walks the triangles in order and, per triangle, the cells of
// its vertex-bbox cell range in (z, y, x) order, appending the triangle to
// every cell whose box passes the SAT test (stage2.zig:104-124).  A cell's
// refs therefore sit in increasing triangle order, each triangle at most once.
// On the device:
//   1. cand_kernel       one thread per triangle: the cell range
//                        (stage2.zig:108-109) and its cell count;
//   2. exclusive scan    of the per-triangle candidate counts (u64);
//   3. sat_kernel<0>     one thread per candidate (triangle, cell): the
//                        triangle by binary search in the scanned counts, the
//                        cell from the candidate's rank in the range, the SAT
//                        test (stage2.zig:114-115); a hit counts into its cell;
//   4. exclusive scan    of the cell counts = first ref of every cell
//                        (stage2.zig:85-95);
//   5. sat_kernel<1>     the same tests again; a hit takes a slot of its cell
//                        (atomic, any order) and stores the key (cell, triangle);
//   6. radix sort of the keys (LSD, 8-bit digits, below): per cell, the refs in increasing
//                        triangle order -- exactly the reference's fill order --
//                        whatever the cell's size (a 1x1x1 grid is one cell of
//                        every triangle);
//   7. bake_kernel       refs -> Pos {v0, v1 - v0, v2 - v0}, Data, material
//                        (stage2.zig:137-164); cells_kernel -> {begin, end}.
// The scene bbox and Grid.init stay on the host (geometry.h scene_grid): one
// sequential pass, bit-exact with initGrid's fmin/fmax order.
//
// Bound: the SAT tests are ~150 flops per candidate (1-10 M candidates:
// microseconds of VALU); the passes over the 2 M cells (counts, scan, order,
// cells: ~50 MB) and the baked arrays (~80 MB written) make it HBM-bound,
// a few ms in total.  Costlier for the wall clock: the host<->device copies.
//
// The scans and the sort are this file's own (no hipCUB): hipCUB's scan and
// radix-sort instantiations were 3.9 MB of the library's 4.2 MB of code
// objects, and loading them on the first HIP call took 8-25 ms of the CLI's
// wall clock on the GPU host (tools/hip_init_probe.cpp, r02ap / r02aq).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <new>
#include <vector>

#include "device_geometry.h"
#include "geometry.h"

using namespace zrt;

namespace {

constexpr int kB = 256;

// stage2.zig:108-109: the triangle's cell range; the candidate count is the
// range's size (the host loop `z <= hi` runs zero times if lo > hi).
__global__ __launch_bounds__(kB) void cand_kernel(const float* __restrict__ pos, uint32_t n, Grid g,
                                                  uint32_t* __restrict__ range,
                                                  unsigned long long* __restrict__ cnt) {
    const uint32_t t = blockIdx.x * kB + threadIdx.x;
    if (t > n) return;
    if (t == n) { cnt[n] = 0ull; return; }   // scan slot n: the total
    const float* p = pos + 9ull * t;
    const v3 a = ld3(p), b = ld3(p + 3), c = ld3(p + 6);
    uint32_t lo[3], hi[3];
    grid_cell_idx(g, vmin(a, vmin(b, c)), lo);
    grid_cell_idx(g, vmax(a, vmax(b, c)), hi);
    unsigned long long m = 1ull;
    for (int k = 0; k < 3; ++k) {
        range[6ull * t + k] = lo[k];
        range[6ull * t + 3 + k] = hi[k];
        m *= hi[k] >= lo[k] ? (unsigned long long)(hi[k] - lo[k] + 1u) : 0ull;
    }
    cnt[t] = m;
}

// One candidate per thread (grid-stride).  FILL = false: count the hits per
// cell (+ the total); FILL = true: store each hit's (cell, triangle) key in its cell.
template <bool FILL>
__global__ __launch_bounds__(kB) void sat_kernel(const float* __restrict__ pos, uint32_t n, Grid g,
                                                 const uint32_t* __restrict__ range,
                                                 const unsigned long long* __restrict__ off,
                                                 unsigned long long total, uint32_t* __restrict__ count,
                                                 const uint32_t* __restrict__ first,
                                                 unsigned long long* __restrict__ keys,
                                                 unsigned long long* __restrict__ nrefs) {
    const unsigned long long stride = (unsigned long long)gridDim.x * kB;
    uint32_t hits = 0;
    for (unsigned long long q = (unsigned long long)blockIdx.x * kB + threadIdx.x; q < total; q += stride) {
        // the triangle: the last t with off[t] <= q (off[0] = 0 <= q < total = off[n])
        uint32_t lo = 0, hi = n;
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) >> 1;
            if (off[mid] <= q) lo = mid;
            else hi = mid;
        }
        const uint32_t t = lo;
        const uint32_t* r = range + 6ull * t;
        const unsigned long long k = q - off[t];           // rank in (z, y, x) order
        const unsigned long long nx = r[3] - r[0] + 1u, nxy = nx * (r[4] - r[1] + 1u);
        const uint32_t z = r[2] + (uint32_t)(k / nxy);
        const uint32_t y = r[1] + (uint32_t)((k % nxy) / nx);
        const uint32_t x = r[0] + (uint32_t)(k % nx);
        const float* p = pos + 9ull * t;
        if (!tri_aabb(ld3(p), ld3(p + 3), ld3(p + 6), grid_cell_bbox(g, x, y, z))) continue;
        const uint32_t cell = (z * g.res[1] + y) * g.res[0] + x;
        if (FILL) {
            keys[first[cell] + atomicAdd(&count[cell], 1u)] = ((unsigned long long)cell << 32) | t;
        } else {
            atomicAdd(&count[cell], 1u);
            ++hits;
        }
    }
    if (!FILL) {
        unsigned long long h = hits;
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned lo32 = __shfl_xor((unsigned)h, o), hi32 = __shfl_xor((unsigned)(h >> 32), o);
            h += ((unsigned long long)hi32 << 32) | lo32;
        }
        if ((threadIdx.x & 63u) == 0 && h) atomicAdd(nrefs, h);
    }
}

// sorted (cell, triangle) keys -> the triangle of every ref
__global__ __launch_bounds__(kB) void key_tri_kernel(const unsigned long long* __restrict__ keys, uint32_t refs,
                                                     uint32_t* __restrict__ idx) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i < refs) idx[i] = (uint32_t)keys[i];
}

__global__ __launch_bounds__(kB) void cells_kernel(const uint32_t* __restrict__ first,
                                                   const uint32_t* __restrict__ count, uint32_t ncells,
                                                   uint2* __restrict__ cells) {
    const uint32_t c = blockIdx.x * kB + threadIdx.x;
    if (c < ncells) cells[c] = make_uint2(first[c], first[c] + count[c]);   // stage2.zig:141-146
}

// bakeInto (stage2.zig:151-158): Pos.init(v0, v1, v2) and Data per ref.
__global__ __launch_bounds__(kB) void bake_kernel(const float* __restrict__ pos, const float* __restrict__ nrm,
                                                  const float* __restrict__ uv, const uint32_t* __restrict__ mat,
                                                  const uint32_t* __restrict__ idx, uint32_t refs,
                                                  float* __restrict__ opos, float* __restrict__ odata,
                                                  uint32_t* __restrict__ omat) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i >= refs) return;
    const uint32_t t = idx[i];
    const float* p = pos + 9ull * t;
    const v3 v0 = ld3(p), e1 = sub(ld3(p + 3), v0), e2 = sub(ld3(p + 6), v0);
    float* q = opos + 9ull * i;
    q[0] = v0.x; q[1] = v0.y; q[2] = v0.z;
    q[3] = e1.x; q[4] = e1.y; q[5] = e1.z;
    q[6] = e2.x; q[7] = e2.y; q[8] = e2.z;
    float* d = odata + 15ull * i;
    for (int k = 0; k < 9; ++k) d[k] = nrm[9ull * t + k];
    for (int k = 0; k < 6; ++k) d[9 + k] = uv[6ull * t + k];
    omat[i] = mat[t];
}

// bakeInto straight into the render context's layout (render.hip
// context_init): Pos as 3 float4 (v0 | shape id 0, e1 | 0, e2 | 0), Data as 4
// float4 (9 normal + 6 texcoord floats, material index bits).
__global__ __launch_bounds__(kB) void ctx_bake_kernel(const float* __restrict__ pos, const float* __restrict__ nrm,
                                                      const float* __restrict__ uv,
                                                      const uint32_t* __restrict__ mat,
                                                      const uint32_t* __restrict__ idx, uint32_t refs,
                                                      float4* __restrict__ opos, float4* __restrict__ odata) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i >= refs) return;
    const uint32_t t = idx[i];
    const float* p = pos + 9ull * t;
    const v3 v0 = ld3(p), e1 = sub(ld3(p + 3), v0), e2 = sub(ld3(p + 6), v0);
    opos[3ull * i] = make_float4(v0.x, v0.y, v0.z, 0.0f);
    opos[3ull * i + 1] = make_float4(e1.x, e1.y, e1.z, 0.0f);
    opos[3ull * i + 2] = make_float4(e2.x, e2.y, e2.z, 0.0f);
    const float* nn = nrm + 9ull * t;
    const float* uu = uv + 6ull * t;
    odata[4ull * i] = make_float4(nn[0], nn[1], nn[2], nn[3]);
    odata[4ull * i + 1] = make_float4(nn[4], nn[5], nn[6], nn[7]);
    odata[4ull * i + 2] = make_float4(nn[8], uu[0], uu[1], uu[2]);
    odata[4ull * i + 3] = make_float4(uu[3], uu[4], uu[5], __uint_as_float(mat[t]));
}

// Device buffers of one build, freed on every exit path.
struct DevBufs {
    std::vector<void*> p;
    ~DevBufs() {
        for (void* x : p) (void)hipFree(x);
    }
    template <typename T>
    hipError_t alloc(T** out, size_t n) {
        void* q = nullptr;
        const hipError_t e = hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) p.push_back(q);
        *out = static_cast<T*>(q);
        return e;
    }
};

#define GB_TRY(expr)                                                                  \
    do {                                                                              \
        const hipError_t e_ = (expr);                                                 \
        if (e_ != hipSuccess) return e_ == hipErrorOutOfMemory ? ZRT_ERR_OUT_OF_MEMORY : ZRT_ERR_HIP; \
    } while (0)

uint32_t blocks_for(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, (n + kB - 1) / kB); }

// ---- exclusive scan, three passes over tiles of kScanTile items: per-tile
// sums, their scan (one workgroup), then each tile scanned from its offset.
// Integer sums: the same result for any tiling.
constexpr int kScanItems = 8;
constexpr uint32_t kScanTile = kB * kScanItems;

// exclusive scan of one value per thread over the workgroup; total to *tot
template <typename T>
__device__ __forceinline__ T block_excl_scan(T v, T* sh, T* tot) {
    const uint32_t tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (uint32_t o = 1; o < (uint32_t)kB; o <<= 1) {
        const T add = tid >= o ? sh[tid - o] : T(0);
        __syncthreads();
        sh[tid] += add;
        __syncthreads();
    }
    const T incl = sh[tid];
    if (tot) *tot = sh[kB - 1];
    __syncthreads();
    return incl - v;
}

template <typename T>
__global__ __launch_bounds__(kB) void scan_tile_sums(const T* __restrict__ in, uint64_t n, T* __restrict__ sums) {
    __shared__ T sh[kB];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    T v = 0;
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < n) v += in[base + k];
    T tot;
    (void)block_excl_scan(v, sh, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// one workgroup: the tile sums scanned in place (exclusive)
template <typename T>
__global__ __launch_bounds__(kB) void scan_sums(T* __restrict__ sums, uint32_t nt) {
    __shared__ T sh[kB];
    const uint32_t per = (nt + kB - 1) / kB;
    const uint32_t b0 = threadIdx.x * per, b1 = min(b0 + per, nt);
    T v = 0;
    for (uint32_t i = b0; i < b1; ++i) v += sums[i];
    T run = block_excl_scan(v, sh, (T*)nullptr);
    for (uint32_t i = b0; i < b1; ++i) {
        const T x = sums[i];
        sums[i] = run;
        run += x;
    }
}

template <typename T>
__global__ __launch_bounds__(kB) void scan_tiles(const T* __restrict__ in, uint64_t n, const T* __restrict__ sums,
                                                 T* __restrict__ out) {
    __shared__ T sh[kB];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    T x[kScanItems];
    T v = 0;
    for (int k = 0; k < kScanItems; ++k) {
        x[k] = base + k < n ? in[base + k] : T(0);
        v += x[k];
    }
    T run = block_excl_scan(v, sh, (T*)nullptr) + sums[blockIdx.x];
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < n) {
            out[base + k] = run;
            run += x[k];
        }
}

// out[i] = in[0] + ... + in[i-1]; tmp: at least scan_tmp_items(n) T's
uint64_t scan_tmp_items(uint64_t n) { return std::max<uint64_t>(1, (n + kScanTile - 1) / kScanTile); }
template <typename T>
hipError_t exclusive_scan(const T* in, T* out, uint64_t n, T* tmp, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint32_t nt = (uint32_t)scan_tmp_items(n);
    hipLaunchKernelGGL(scan_tile_sums<T>, dim3(nt), dim3(kB), 0, st, in, n, tmp);
    hipLaunchKernelGGL(scan_sums<T>, dim3(1), dim3(kB), 0, st, tmp, nt);
    hipLaunchKernelGGL(scan_tiles<T>, dim3(nt), dim3(kB), 0, st, in, n, (const T*)tmp, out);
    return hipGetLastError();
}

// ---- stable LSD radix sort of u64 keys, 8-bit digits.  Per pass: a digit
// histogram per tile of kSortTile keys (digit-major, so the exclusive scan
// of all of them gives each (digit, tile) its first output slot), then the
// scatter: each tile walks its keys in index order, 256 at a time; a key's
// slot is its (digit, tile) base + the keys of that digit already written
// by the tile + those ahead of it in the same round (earlier waves, then
// earlier lanes: the lanes of a wave with the same digit found by ballots
// over the 8 digit bits).  Stable, so after the passes over the low 32 bits
// (the triangle) and then the cell bits the keys are in (cell, triangle)
// order -- the reference's fill order.
constexpr int kSortRounds = 16;
constexpr uint32_t kSortTile = kB * kSortRounds;
constexpr int kWaves = kB / 64;

__global__ __launch_bounds__(kB) void sort_hist_kernel(const unsigned long long* __restrict__ keys, uint32_t n,
                                                       uint32_t shift, uint32_t nt, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kSortTile;
    for (int r = 0; r < kSortRounds; ++r) {
        const uint32_t i = base + (uint32_t)r * kB + threadIdx.x;
        if (i < n) atomicAdd(&h[(uint32_t)(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * nt + blockIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(kB) void sort_scatter_kernel(const unsigned long long* __restrict__ keys, uint32_t n,
                                                          uint32_t shift, uint32_t nt, const uint32_t* __restrict__ off,
                                                          unsigned long long* __restrict__ out) {
    __shared__ uint32_t run[256];            // keys of each digit this tile has placed
    __shared__ uint32_t wc[kWaves][256];     // this round: keys of each digit per wave
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
    run[tid] = off[(size_t)tid * nt + blockIdx.x];
    const uint32_t base = blockIdx.x * kSortTile;
    for (int r = 0; r < kSortRounds; ++r) {
        for (int w = 0; w < kWaves; ++w) wc[w][tid] = 0;
        __syncthreads();
        const uint32_t i = base + (uint32_t)r * kB + tid;
        const bool valid = i < n;
        const unsigned long long key = valid ? keys[i] : 0ull;
        const uint32_t d = (uint32_t)(key >> shift) & 255u;
        // lanes of this wave holding a valid key with the same digit
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < 8; ++b) {
            const uint64_t m = __ballot(valid && ((d >> b) & 1u));
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        if (valid && (peers & below) == 0ull) wc[wave][d] = (uint32_t)__popcll(peers);   // the digit's first lane
        __syncthreads();
        if (valid) {
            uint32_t ahead = run[d];
            for (int w = 0; w < (int)wave; ++w) ahead += wc[w][d];
            out[ahead + (uint32_t)__popcll(peers & below)] = key;
        }
        __syncthreads();
        uint32_t add = 0;
        for (int w = 0; w < kWaves; ++w) add += wc[w][tid];
        run[tid] += add;
        __syncthreads();
    }
}

// sorts keys[0, n) on bits [0, nbits); the result ends in *keys or *alt
// (returned through *result); tmp: 256 * tiles + scan_tmp_items of that
hipError_t radix_sort(unsigned long long* keys, unsigned long long* alt, uint32_t n, uint32_t nbits, uint32_t* tmp,
                      hipStream_t st, unsigned long long** result) {
    const uint32_t nt = std::max<uint32_t>(1, (n + kSortTile - 1) / kSortTile);
    uint32_t* hist = tmp;
    uint32_t* off = tmp + 256ull * nt;
    uint32_t* stmp = off + 256ull * nt;
    unsigned long long *a = keys, *b = alt;
    for (uint32_t shift = 0; shift < nbits; shift += 8) {
        hipLaunchKernelGGL(sort_hist_kernel, dim3(nt), dim3(kB), 0, st, (const unsigned long long*)a, n, shift, nt,
                           hist);
        hipError_t e = exclusive_scan<uint32_t>(hist, off, 256ull * nt, stmp, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(sort_scatter_kernel, dim3(nt), dim3(kB), 0, st, (const unsigned long long*)a, n, shift, nt,
                           (const uint32_t*)off, b);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        std::swap(a, b);
    }
    *result = a;
    return hipSuccess;
}
uint64_t radix_tmp_items(uint32_t n) {
    const uint64_t nt = std::max<uint32_t>(1, (n + kSortTile - 1) / kSortTile);
    return 512ull * nt + scan_tmp_items(256ull * nt);
}

}  // namespace

namespace {

// geo: host result (zrt_geometry_build_device); dg: the render context's
// device arrays instead (no host round trip).  Exactly one is non-null.
int build_on_device(const float* positions, const float* normals, const float* texcoords,
                    const uint32_t* material, uint32_t n, hipStream_t st, zrt_geometry* geo,
                    const Grid& grid, uint32_t ncells_in, DeviceGeometry* dg) {
    DevBufs B;
    const Grid g = grid;
    const uint32_t ncells = ncells_in;
    float* d_pos;
    uint32_t* d_range;
    unsigned long long *d_cnt, *d_off, *d_nrefs;
    GB_TRY(B.alloc(&d_pos, 9ull * n));
    GB_TRY(B.alloc(&d_range, 6ull * n));
    GB_TRY(B.alloc(&d_cnt, n + 1ull));
    GB_TRY(B.alloc(&d_off, n + 1ull));
    GB_TRY(B.alloc(&d_nrefs, 1));
    GB_TRY(hipMemcpyAsync(d_pos, positions, 36ull * n, hipMemcpyHostToDevice, st));
    GB_TRY(hipMemsetAsync(d_nrefs, 0, 8, st));

    // 1-2: candidates per triangle, scanned
    hipLaunchKernelGGL(cand_kernel, dim3(blocks_for(n + 1ull)), dim3(kB), 0, st, d_pos, n, g, d_range, d_cnt);
    GB_TRY(hipGetLastError());
    unsigned long long* d_stmp64;
    GB_TRY(B.alloc(&d_stmp64, scan_tmp_items(n + 1ull)));
    GB_TRY(exclusive_scan<unsigned long long>(d_cnt, d_off, n + 1ull, d_stmp64, st));
    unsigned long long total = 0;
    GB_TRY(hipMemcpyAsync(&total, d_off + n, 8, hipMemcpyDeviceToHost, st));
    GB_TRY(hipStreamSynchronize(st));

    // 3-4: hits per cell, scanned into the first ref of every cell
    uint32_t *d_count, *d_first;
    GB_TRY(B.alloc(&d_count, ncells));
    GB_TRY(B.alloc(&d_first, ncells));
    GB_TRY(hipMemsetAsync(d_count, 0, 4ull * ncells, st));
    const uint32_t sat_blocks = (uint32_t)std::min<unsigned long long>(blocks_for(total), 65536ull);
    if (total) {
        hipLaunchKernelGGL(sat_kernel<false>, dim3(sat_blocks), dim3(kB), 0, st, d_pos, n, g, d_range, d_off,
                           total, d_count, nullptr, nullptr, d_nrefs);
        GB_TRY(hipGetLastError());
    }
    unsigned long long refs64 = 0;
    GB_TRY(hipMemcpyAsync(&refs64, d_nrefs, 8, hipMemcpyDeviceToHost, st));
    uint32_t* d_stmp32;
    GB_TRY(B.alloc(&d_stmp32, scan_tmp_items(ncells)));
    GB_TRY(exclusive_scan<uint32_t>(d_count, d_first, ncells, d_stmp32, st));
    GB_TRY(hipStreamSynchronize(st));
    if (refs64 > 0x7FFFFFFFull) return ZRT_ERR_UNSUPPORTED;   // u32 slots (refs of a 2^31-ref grid: 16 GB of Pos)
    const uint32_t refs = (uint32_t)refs64;

    // 5-6: fill, then the reference's order within each cell
    uint32_t* d_idx;
    unsigned long long *d_keys, *d_keys2;
    GB_TRY(B.alloc(&d_idx, refs));
    GB_TRY(B.alloc(&d_keys, refs));
    GB_TRY(B.alloc(&d_keys2, refs));
    GB_TRY(hipMemsetAsync(d_count, 0, 4ull * ncells, st));
    if (total) {
        hipLaunchKernelGGL(sat_kernel<true>, dim3(sat_blocks), dim3(kB), 0, st, d_pos, n, g, d_range, d_off, total,
                           d_count, d_first, d_keys, nullptr);
        GB_TRY(hipGetLastError());
    }
    if (refs) {
        uint32_t cell_bits = 1;
        while (cell_bits < 31 && (1u << cell_bits) < ncells) ++cell_bits;
        uint32_t* d_rtmp;
        GB_TRY(B.alloc(&d_rtmp, radix_tmp_items(refs)));
        unsigned long long* sorted = nullptr;
        GB_TRY(radix_sort(d_keys, d_keys2, refs, 32 + cell_bits, d_rtmp, st, &sorted));
        hipLaunchKernelGGL(key_tri_kernel, dim3(blocks_for(refs)), dim3(kB), 0, st, (const unsigned long long*)sorted,
                           refs, d_idx);
        GB_TRY(hipGetLastError());
    }
    uint2* d_cells;
    if (dg) {
        GB_TRY(hipMalloc((void**)&dg->cells, 8ull * std::max<uint32_t>(ncells, 1)));
        d_cells = dg->cells;
    } else {
        GB_TRY(B.alloc(&d_cells, ncells));
    }
    hipLaunchKernelGGL(cells_kernel, dim3(blocks_for(ncells)), dim3(kB), 0, st, d_first, d_count, ncells, d_cells);
    GB_TRY(hipGetLastError());

    // 7: bake
    float *d_nrm, *d_uv, *d_opos, *d_odata;
    uint32_t *d_mat, *d_omat;
    GB_TRY(B.alloc(&d_nrm, 9ull * n));
    GB_TRY(B.alloc(&d_uv, 6ull * n));
    GB_TRY(B.alloc(&d_mat, n));
    if (dg) {   // straight into the context's layout
        dg->refs = refs;
        GB_TRY(hipMalloc((void**)&dg->pos, 48ull * std::max<uint32_t>(refs, 1)));
        GB_TRY(hipMalloc((void**)&dg->data, 64ull * std::max<uint32_t>(refs, 1)));
        GB_TRY(hipMemcpyAsync(d_nrm, normals, 36ull * n, hipMemcpyHostToDevice, st));
        GB_TRY(hipMemcpyAsync(d_uv, texcoords, 24ull * n, hipMemcpyHostToDevice, st));
        GB_TRY(hipMemcpyAsync(d_mat, material, 4ull * n, hipMemcpyHostToDevice, st));
        if (refs) {
            hipLaunchKernelGGL(ctx_bake_kernel, dim3(blocks_for(refs)), dim3(kB), 0, st, d_pos, d_nrm, d_uv, d_mat,
                               d_idx, refs, dg->pos, dg->data);
            GB_TRY(hipGetLastError());
        }
        GB_TRY(hipStreamSynchronize(st));
        return ZRT_OK;
    }
    GB_TRY(B.alloc(&d_opos, 9ull * refs));
    GB_TRY(B.alloc(&d_odata, 15ull * refs));
    GB_TRY(B.alloc(&d_omat, refs));
    GB_TRY(hipMemcpyAsync(d_nrm, normals, 36ull * n, hipMemcpyHostToDevice, st));
    GB_TRY(hipMemcpyAsync(d_uv, texcoords, 24ull * n, hipMemcpyHostToDevice, st));
    GB_TRY(hipMemcpyAsync(d_mat, material, 4ull * n, hipMemcpyHostToDevice, st));
    if (refs) {
        hipLaunchKernelGGL(bake_kernel, dim3(blocks_for(refs)), dim3(kB), 0, st, d_pos, d_nrm, d_uv, d_mat, d_idx,
                           refs, d_opos, d_odata, d_omat);
        GB_TRY(hipGetLastError());
    }
    geo->cells.resize(2ull * ncells);
    geo->indices.resize(refs);
    geo->pos.resize(9ull * refs);
    geo->data.resize(15ull * refs);
    geo->mat.resize(refs);
    GB_TRY(hipMemcpyAsync(geo->cells.data(), d_cells, 8ull * ncells, hipMemcpyDeviceToHost, st));
    if (refs) {
        GB_TRY(hipMemcpyAsync(geo->indices.data(), d_idx, 4ull * refs, hipMemcpyDeviceToHost, st));
        GB_TRY(hipMemcpyAsync(geo->pos.data(), d_opos, 36ull * refs, hipMemcpyDeviceToHost, st));
        GB_TRY(hipMemcpyAsync(geo->data.data(), d_odata, 60ull * refs, hipMemcpyDeviceToHost, st));
        GB_TRY(hipMemcpyAsync(geo->mat.data(), d_omat, 4ull * refs, hipMemcpyDeviceToHost, st));
    }
    GB_TRY(hipStreamSynchronize(st));
    return ZRT_OK;
}

}  // namespace

// Load this translation unit's code objects on the current device; called
// by zrt_device_warmup.
int grid_build_warmup() {
    hipFuncAttributes fa;
    return hipFuncGetAttributes(&fa, (const void*)cand_kernel) == hipSuccess ? ZRT_OK : ZRT_ERR_HIP;
}

extern "C" int zrt_geometry_build_device(const float* positions, const float* normals, const float* texcoords,
                                         const uint32_t* material, uint32_t n, const uint32_t resolution[3],
                                         int device, zrt_geometry** out) {
    if (!out) return ZRT_ERR_INVALID_ARG;
    *out = nullptr;
    const int arc = check_build_args(positions, normals, texcoords, material, n, resolution);
    if (arc != ZRT_OK) return arc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ZRT_ERR_NO_DEVICE;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (device < 0) device = prev >= 0 ? prev : 0;
    if (device >= ndev) return ZRT_ERR_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return ZRT_ERR_NO_DEVICE;
    int rc = ZRT_OK;
    zrt_geometry* geo = new (std::nothrow) zrt_geometry();
    hipStream_t st = nullptr;
    if (!geo) {
        rc = ZRT_ERR_OUT_OF_MEMORY;
    } else if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        rc = ZRT_ERR_HIP;
    } else {
        try {
            geo->grid = scene_grid(positions, n, resolution);   // stage2.zig:44-57, host
            geo->ncells = resolution[0] * resolution[1] * resolution[2];
            rc = build_on_device(positions, normals, texcoords, material, n, st, geo, geo->grid, geo->ncells,
                                 nullptr);
        } catch (const std::bad_alloc&) {
            rc = ZRT_ERR_OUT_OF_MEMORY;
        }
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    if (rc != ZRT_OK) {
        delete geo;
        return rc;
    }
    *out = geo;
    return ZRT_OK;
}

// Device build into a render context's arrays on the current device and
// stream (render.hip zrt_context_create_built).  On failure the arrays
// allocated so far are freed.
int grid_build_into_device(const float* positions, const float* normals, const float* texcoords,
                           const uint32_t* material, uint32_t n, const uint32_t resolution[3], hipStream_t st,
                           Grid* grid, DeviceGeometry* dg) {
    const int arc = check_build_args(positions, normals, texcoords, material, n, resolution);
    if (arc != ZRT_OK) return arc;
    *grid = scene_grid(positions, n, resolution);   // stage2.zig:44-57, host
    int rc;
    try {
        rc = build_on_device(positions, normals, texcoords, material, n, st, nullptr, *grid,
                             resolution[0] * resolution[1] * resolution[2], dg);
    } catch (const std::bad_alloc&) {
        rc = ZRT_ERR_OUT_OF_MEMORY;
    }
    if (rc != ZRT_OK) {
        (void)hipStreamSynchronize(st);
        for (void* q : {(void*)dg->cells, (void*)dg->pos, (void*)dg->data})
            if (q) (void)hipFree(q);
        *dg = DeviceGeometry();
    }
    return rc;
}
