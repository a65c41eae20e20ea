/* div_check.c — evidence for the march kernel's density normalisation (vr_kernels.hip,
 * div_by_range): on the domain the host enables it for (2^-40 <= b < 2^100, |a| >= 2^-100),
 *     q = a * RN(1/b);  e = fma(-q, b, a);  q' = fma(e, RN(1/b), q)
 * equals the IEEE single-precision quotient RN(a / b).  Compares against x86 SSE division
 * (correctly rounded) with hardware fmaf (-mfma) over random divisors b (random normal,
 * [1, 2), just below 2, integers) and numerators a (random bits, and a/b in [0, 1.01)).
 *   gcc -O2 -mfma -ffp-contract=off tools/div_check.c -o div_check -lm
 *   ./div_check [divisors] [numerators per divisor]      (defaults 200000 x 20000)
 * Prints "tested N mismatches M"; exit status 1 if M > 0. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9E3779B97F4A7C15ull;
static inline uint64_t nx(void)
{
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}
static inline float bits(uint32_t u)
{
    float f;
    memcpy(&f, &u, 4);
    return f;
}

int main(int argc, char **argv)
{
    const long nb = argc > 1 ? atol(argv[1]) : 200000, na = argc > 2 ? atol(argv[2]) : 20000;
    const uint32_t lo = (127u - 40u) << 23, hi = (127u + 100u) << 23;  /* [2^-40, 2^100) */
    long long bad = 0, tot = 0;
    for (long rr = 0; rr < nb; ++rr) {
        float b;
        const long k4 = rr % 4;
        if (k4 == 0) b = bits(0x3F800000u | (uint32_t)(nx() & 0x7FFFFF));            /* [1,2) */
        else if (k4 == 1) b = bits((0x3F800000u | 0x7FFFFF) - (uint32_t)(nx() & 0xFF)); /* ~2 */
        else if (k4 == 2) b = (float)(1 + nx() % 65535);                               /* ints */
        else b = bits((uint32_t)(nx() % (hi - lo)) + lo);                              /* any */
        const float r = 1.0f / b;
        for (long k = 0; k < na; ++k) {
            const uint64_t z = nx();
            float a = (k & 1) ? bits((uint32_t)z & 0x7FFFFFFFu)
                              : b * (float)((z >> 11) * (1.0 / 9007199254740992.0)) * 1.01f;
            if ((z >> 62) & 1) a = -a;
            if (!isfinite(a) || fabsf(a) < 0x1p-100f) continue;
            const float ref = a / b;
            if (isinf(ref)) continue;
            float q = a * r;
            const float e = fmaf(-q, b, a);
            q = fmaf(e, r, q);
            ++tot;
            if (memcmp(&q, &ref, 4) != 0) {
                if (bad < 10) printf("a=%a b=%a ref=%a got=%a\n", a, b, ref, q);
                ++bad;
            }
        }
    }
    printf("tested %lld mismatches %lld\n", tot, bad);
    return bad ? 1 : 0;
}
