/* Exhaustive check of the row Adam's division by the step constant (csrc/lgcn_rowadam.hip
 * div_step): for every distinct fp32 c_t = (float) sqrt(1 - beta2^t) (t = 1, 2, ... until c_t
 * reaches 1.0f), and every significand of one binade of s, Markstein's
 *     q0 = s * rc,  q = fma(fma(-c, q0, s), rc, q0),  rc = 1.0f / c
 * equals IEEE s / c. Normal-range division is scale invariant (s -> 2^k s scales q0, the exact
 * residual and q by 2^k), so one binade covers every normal s; s = sqrt(v) of a float v >= 0 is
 * never subnormal. usage: gcc -O2 -mfma -ffp-contract=off tools/markstein_check.c -lm && ./a.out [beta2 [max]]
 * (max: stop after that many distinct constants; the CPU test checks the first 64). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

int main(int argc, char** argv) {
    const double beta2 = argc > 1 ? atof(argv[1]) : 0.999;
    const long max = argc > 2 ? atol(argv[2]) : -1;
    long bad = 0, consts = 0;
    float prev = -1.0f;
    for (long t = 1;; ++t) {
        const float c = (float)sqrt(1.0 - pow(beta2, (double)t));
        if (c == prev) continue;
        prev = c;
        ++consts;
        const float rc = 1.0f / c;
        for (uint32_t m = 0; m < (1u << 23); ++m) {
            const float s = f_of((127u << 23) | m);
            const float q0 = s * rc;
            const float q = fmaf(fmaf(-c, q0, s), rc, q0);
            if (q != s / c) {
                if (bad < 10) printf("t=%ld c=%a s=%a: %a vs %a\n", t, c, s, q, s / c);
                ++bad;
            }
        }
        if (c == 1.0f || consts == max) {
            printf("beta2 %g: %ld distinct step constants (t = 1..%ld), %ld mismatches over %ld quotients\n", beta2,
                   consts, t, bad, consts << 23);
            return bad != 0;
        }
    }
}
