/* Exactness check of the division used by libbmfr's fused kernel
 * (bmfr_amd/csrc/bmfr_device.h, div_by_recip): with y = RN(1/b),
 *   q = RN(a*y); r = fma(-q, b, a); q' = fma(r, y, q)
 * must equal RN(a/b).  Exhaustive over divisor mantissas (one binade; the
 * identity is scale-invariant away from under/overflow) x `per` dividends,
 * plus random and adversarial pairs over a wide exponent range.
 * Prints the number of mismatches; exit status 0 iff none. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static long check(float a, float b, float y) {
    const float q = a * y, r = fmaf(-q, b, a), q1 = fmaf(r, y, q);
    return q1 != a / b;
}

int main(int argc, char** argv) {
    const int per = argc > 1 ? atoi(argv[1]) : 8;
    const long random_pairs = argc > 2 ? atol(argv[2]) : 20000000;
    long bad = 0, n = 0;
    for (uint32_t mb = 0; mb < (1u << 23); ++mb) {
        const float b = f_of((127u << 23) | mb), y = 1.0f / b;
        for (int k = 0; k < per; ++k) {
            uint32_t ma = (uint32_t)rnd() & 0x7fffff;
            if (k == 0) ma = 0x7fffff;
            if (k == 1) ma = mb;
            bad += check(f_of(((124u + (k & 7)) << 23) | ma), b, y);
            ++n;
        }
    }
    for (long i = 0; i < random_pairs; ++i) {
        const uint64_t r = rnd();
        const uint32_t ua = (uint32_t)r, ub = (uint32_t)(r >> 32);
        uint32_t mb = ub & 0x7fffff;
        if ((i & 3) == 1) mb = 0x7fffff - (ub & 0xff);
        const float a = f_of((ua & 0x80000000u) | ((80u + (ua >> 24) % 96) << 23) | (ua & 0x7fffff));
        const float b = f_of((ub & 0x80000000u) | ((80u + (ub >> 24) % 96) << 23) | mb);
        bad += check(a, b, 1.0f / b);
        ++n;
    }
    printf("tested %ld bad %ld\n", n, bad);
    return bad != 0;
}
