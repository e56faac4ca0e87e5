// Host check of the OccX decision (csrc/zrt_internal.h occx_usable): grids
// whose 4^3-cell bricks overflow the kernels' 24-bit brick index, whose
// occupied-brick prefix overflows u16, or whose blob overflows the LDS budget
// fall back to the lane walk instead of failing the context (round-2 advice).
#include <cstdio>
#include <cstdint>

#include "zrt_internal.h"

static uint64_t bricks(uint32_t a, uint32_t b, uint32_t c) {
    return (uint64_t)((a + 3) / 4) * ((b + 3) / 4) * ((c + 3) / 4);
}

int main() {
    int fails = 0;
    auto expect = [&](bool got, bool want, const char* what) {
        if (got != want) { std::printf("FAIL %s: got %d want %d\n", what, got, want); ++fails; }
    };
    const uint64_t budget = 95 * 1024;
    expect(zrt::occx_usable(bricks(128, 128, 128), 5000, 63328, budget), true, "contest 128^3");
    expect(zrt::occx_usable(bricks(1024, 1024, 1024), 10, budget + 1, budget), false, "2^24 bricks, blob over the LDS budget");
    expect(zrt::occx_usable(bricks(1024, 1024, 1024), 10, 4096, 1ull << 40), true, "exactly 2^24 bricks");
    expect(zrt::occx_usable(bricks(1100, 1100, 900), 10, 4096, 1ull << 40), false, "more than 2^24 bricks");
    expect(zrt::occx_usable(bricks(64, 64, 64), 0xFFFF, 1024, budget), false, "u16 prefix overflow");
    expect(zrt::occx_usable(bricks(64, 64, 64), 0xFFFE, 1024, budget), true, "u16 prefix at the limit");
    expect(zrt::occx_usable(bricks(256, 256, 256), 100, budget + 4, budget), false, "LDS budget");
    std::printf("{\"fails\": %d}\n", fails);
    return fails != 0;
}
