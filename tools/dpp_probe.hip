// DPP lane reads under a partial EXEC mask (gfx950): the root-cause check
// for round 1's park-mode fault ("park mode").
//
// Park mode's wave prefix sum was written as
//     x += (lane & 15) >= 1 ? dpp_row_shr1(x) : 0;
// and hipcc compiled the conditional operator as a branch: the
// v_mov_b32_dpp runs with EXEC = {lanes with (lane & 15) >= 1}, so lane 1
// reads lane 0 while lane 0 is disabled.  On gfx9-family hardware a DPP
// source lane that is disabled in EXEC is "invalid": with bound_ctrl 0 the
// destination is left unwritten (it keeps the zero the compiler put there).
// This program prints, per variant, how many lanes get the true inclusive
// prefix sum of x = lane + 1.
//   hipcc --offload-arch=gfx950 -O3 tools/dpp_probe.hip -o build/dpp_probe
#include <hip/hip_runtime.h>

#include <cstdio>

template <int CTRL>
__device__ __forceinline__ unsigned dpp(unsigned v) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}

// round 1's form: the DPP read is control-dependent on the lane's condition
__device__ __noinline__ unsigned scan_branchy(unsigned x, unsigned lane) {
    const unsigned rl = lane & 15u;
    x += rl >= 1u ? dpp<0x111>(x) : 0u;
    x += rl >= 2u ? dpp<0x112>(x) : 0u;
    x += rl >= 4u ? dpp<0x114>(x) : 0u;
    x += rl >= 8u ? dpp<0x118>(x) : 0u;
    x += (lane & 31u) >= 16u ? dpp<0x142>(x) : 0u;
    x += lane >= 32u ? dpp<0x143>(x) : 0u;
    return x;
}

// fixed form: every DPP read runs with the whole wave enabled, the select after
__device__ __noinline__ unsigned scan_full(unsigned x, unsigned lane) {
    const unsigned rl = lane & 15u;
    unsigned t;
    t = dpp<0x111>(x); x += rl >= 1u ? t : 0u;
    t = dpp<0x112>(x); x += rl >= 2u ? t : 0u;
    t = dpp<0x114>(x); x += rl >= 4u ? t : 0u;
    t = dpp<0x118>(x); x += rl >= 8u ? t : 0u;
    t = dpp<0x142>(x); x += (lane & 31u) >= 16u ? t : 0u;
    t = dpp<0x143>(x); x += lane >= 32u ? t : 0u;
    return x;
}

__global__ void probe(unsigned* out) {
    const unsigned lane = threadIdx.x & 63u;
    out[lane] = scan_branchy(lane + 1u, lane);
    out[64 + lane] = scan_full(lane + 1u, lane);
}

int main() {
    unsigned* d = nullptr;
    unsigned h[128];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 2;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int ok[2] = {0, 0};
    for (int v = 0; v < 2; ++v)
        for (unsigned l = 0; l < 64; ++l) ok[v] += h[64 * v + l] == (l + 1) * (l + 2) / 2;
    printf("{\"branchy_lanes_correct\": %d, \"full_exec_lanes_correct\": %d, \"branchy\": [", ok[0], ok[1]);
    for (int l = 0; l < 64; ++l) printf("%s%u", l ? ", " : "", h[l]);
    printf("]}\n");
    (void)hipFree(d);
    return ok[1] == 64 ? 0 : 1;
}
