// device_geometry.h -- hand-off from the device grid build (grid_build.hip)
// to a render context (render.hip zrt_context_create_built): the baked
// stage-2 arrays, already in the context's HBM layout, never copied to the
// host.
#pragma once

#include <hip/hip_runtime.h>

#include "zrt_internal.h"

struct DeviceGeometry {
    uint2* cells = nullptr;   // ncells {begin, end}
    float4* pos = nullptr;    // refs * 3: v0|0, e1|0, e2|0
    float4* data = nullptr;   // refs * 4: normals, texcoords, material bits
    uint32_t refs = 0;
};

// Build the grid of `n` source triangles on the current device and stream.
// Fills *grid (stage2.zig:44-57) and *dg; on failure frees what it allocated.
int grid_build_into_device(const float* positions, const float* normals, const float* texcoords,
                           const uint32_t* material, uint32_t n, const uint32_t resolution[3], hipStream_t st,
                           zrt::Grid* grid, DeviceGeometry* dg);
