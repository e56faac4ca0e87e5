// Host check of the park kernel's pair-refill select (csrc/dda.h select_bit
// over the SEL8_ENTRY byte table): for every mask m and rank r < popcount(m)
// the r-th set bit of m, against a plain bit loop.  Exhaustive over all
// masks with at most 2 set bits, all byte-patterned masks, and a seeded
// sample of random 32-bit masks (argv[1] = sample count).
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#include "dda.h"

static uint32_t select_loop(uint32_t m, uint32_t r) {
    for (uint32_t k = 0; k < 32; ++k)
        if ((m >> k) & 1u) { if (r == 0) return k; --r; }
    return 32;
}

int main(int argc, char** argv) {
    const uint64_t samples = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
    uint8_t sel8[256 * 8];
    for (uint32_t i = 0; i < 256u * 8u; ++i) {
        SEL8_ENTRY(i, pos);
        sel8[i] = (uint8_t)pos;
    }
    uint64_t checked = 0, fails = 0;
    auto check = [&](uint32_t m) {
        const uint32_t n = (uint32_t)__builtin_popcount(m);
        for (uint32_t r = 0; r < n; ++r) {
            const uint32_t got = zrt::select_bit(sel8, m, r), want = select_loop(m, r);
            ++checked;
            if (got != want && fails++ < 10) std::fprintf(stderr, "m=%08x r=%u got %u want %u\n", m, r, got, want);
        }
    };
    check(0u);
    for (uint32_t a = 0; a < 32; ++a)
        for (uint32_t b = a; b < 32; ++b) check((1u << a) | (1u << b));
    for (uint32_t b = 0; b < 256; ++b)
        for (uint32_t mask = 0; mask < 16; ++mask) {
            uint32_t m = 0;
            for (uint32_t k = 0; k < 4; ++k)
                if ((mask >> k) & 1u) m |= b << (8 * k);
            check(m);
            check(~m);
        }
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < samples; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const uint32_t m = (uint32_t)(s >> 32) & ((i & 1) ? 0xFFFFFFFFu : (uint32_t)s);
        check(m);
    }
    std::printf("{\"checked\": %llu, \"fails\": %llu}\n", (unsigned long long)checked, (unsigned long long)fails);
    return fails ? 1 : 0;
}
