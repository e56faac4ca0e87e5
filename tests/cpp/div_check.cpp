// Host check of the kernels' item division (csrc/dda.h div_magic / div_by):
// for every divisor S in [1, 65535] (a pass's samples per pixel), floor(n / S)
// by multiply-and-shift against the hardware division, over n = 0, S - 1, S,
// the multiples of S around 2^31 - 1, 2^31 - 1 itself and a seeded sample
// of n < 2^31 (argv[1] = random numerators per divisor).
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#include "dda.h"

int main(int argc, char** argv) {
    const uint32_t per = argc > 1 ? (uint32_t)std::strtoul(argv[1], nullptr, 10) : 64;
    uint64_t checked = 0, fails = 0;
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (uint32_t S = 1; S <= 65535u; ++S) {
        const zrt::DivS d = zrt::div_magic(S);
        auto check = [&](uint32_t n) {
            n &= 0x7FFFFFFFu;
            ++checked;
            if (zrt::div_by(n, d) != n / S && fails++ < 10)
                std::fprintf(stderr, "S=%u n=%u got %u want %u\n", S, n, zrt::div_by(n, d), n / S);
        };
        check(0);
        check(S - 1);
        check(S);
        check(0x7FFFFFFFu);
        const uint32_t top = 0x7FFFFFFFu / S * S;
        check(top);
        check(top - 1);
        if (top >= S) check(top - S);
        for (uint32_t i = 0; i < per; ++i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            check((uint32_t)(s >> 33));
            check((uint32_t)(s >> 40) * S + (S - 1));
        }
    }
    std::printf("{\"checked\": %llu, \"fails\": %llu}\n", (unsigned long long)checked, (unsigned long long)fails);
    return fails ? 1 : 0;
}
