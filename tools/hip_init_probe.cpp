// Start-up cost on the GPU box, in the order the zrt CLI pays it: HIP
// runtime + device context (hipFree(0)), then dlopen(libzrt.so), then
// zrt_device_warmup (code objects of render.hip and grid_build.hip).
//   hipcc -O2 tools/hip_init_probe.cpp -o tools/bin/hip_init_probe -ldl
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const char* lib = argc > 1 ? argv[1] : "zig_raytracing_contest_amd/libzrt.so";
    const double t0 = now_ms();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 2;
    const double t1 = now_ms();
    if (hipSetDevice(0) != hipSuccess || hipFree(nullptr) != hipSuccess) return 2;
    const double t2 = now_ms();
    void* h = dlopen(lib, RTLD_NOW);
    if (!h) { fprintf(stderr, "%s\n", dlerror()); return 2; }
    const double t3 = now_ms();
    // grid_build.hip's module first (its hipCUB scans and sorts), then the
    // rest of zrt_device_warmup (render.hip's module)
    auto gwarm = (int (*)())dlsym(h, "_Z17grid_build_warmupv");
    if (gwarm && gwarm() != 0) return 2;
    const double t3b = now_ms();
    auto warm = (int (*)(int))dlsym(h, "zrt_device_warmup");
    if (!warm || warm(0) != 0) return 2;
    const double t4 = now_ms();
    printf("{\"device_count_ms\": %.2f, \"context_ms\": %.2f, \"dlopen_ms\": %.2f, \"grid_module_ms\": %.2f, "
           "\"warmup_rest_ms\": %.2f}\n", t1 - t0, t2 - t1, t3 - t2, t3b - t3, t4 - t3b);
    return 0;
}
