/* CPU check of the divc() correction in cfd_amd/csrc/hip/kernels.hpp:
 * q = RN(a * RN(1/d)), q' = RN(q + RN(a - q d) * RN(1/d)) (two FMAs) against
 * the correctly rounded a / d, bit for bit, for the divisors dx^2 of grids of
 * n = 17 .. 1025 points on domains of length 1, 2*pi and 0.5, over random a
 * of either sign with exponents in [-60, 60] (2e7 quotients per divisor).
 *   gcc -O2 -ffp-contract=off -o /tmp/divc_check tools/divc_check.c -lm && /tmp/divc_check
 * Optional argv[1]: quotients per divisor. Prints the number of mismatches
 * (0 expected) and exits 1 on any. */
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static inline uint64_t xorshift(void) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}

int main(int argc, char** argv) {
    const long per = argc > 1 ? atol(argv[1]) : 20000000;
    const int ns[] = {17, 24, 32, 33, 41, 64, 65, 100, 128, 129, 256, 257, 512, 1000, 1024, 1025};
    const double lens[] = {1.0, 2.0 * M_PI, 0.5};
    long bad = 0, tot = 0;
    for (size_t t = 0; t < sizeof ns / sizeof ns[0]; t++) {
        for (int dom = 0; dom < 3; dom++) {
            const double dx = lens[dom] / (ns[t] - 1);
            const double d = dx * dx, r = 1.0 / d;
            for (long n = 0; n < per; n++) {
                const uint64_t b = xorshift();
                const uint64_t e = 1023 - 60 + (b >> 52) % 121;
                const uint64_t bits = (b & 0x000FFFFFFFFFFFFFull) | (e << 52) | ((xorshift() & 1) << 63);
                double a;
                memcpy(&a, &bits, 8);
                const double q = a * r;
                const double q1 = fma(fma(-q, d, a), r, q);
                const double ex = a / d;
                if (memcmp(&q1, &ex, 8) != 0) {
                    if (bad < 5) printf("mismatch n=%d L=%g a=%a got=%a want=%a\n", ns[t], lens[dom], a, q1, ex);
                    bad++;
                }
                tot++;
            }
        }
    }
    printf("divc_check: %ld quotients, %ld mismatches\n", tot, bad);
    return bad ? 1 : 0;
}
