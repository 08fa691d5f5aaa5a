/* Exhaustive check of the division-free correctly rounded quotient used by the kernels (soc_device.hpp div_rn):
 * q = a rn, q' = fma(fma(-q, n, a), rn, q) with rn = RN(1 / n) equals RN(a / n) for a = x + 0.5 (pixel centres,
 * x < n) and a = x (x <= n, the clouds' ray uv), for every n <= 16384. Build: gcc -O2 -mfma check_div_rn.c -lm */
#include <stdio.h>
#include <math.h>

static long check(int centre) {
    long bad = 0;
    for (int n = 1; n <= 16384; ++n) {
        const float nf = (float)n, rn = 1.0f / nf;
        const int last = centre ? n - 1 : n;
        for (int x = 0; x <= last; ++x) {
            const float a = centre ? (float)x + 0.5f : (float)x;
            const float q = a * rn;
            const float q1 = fmaf(fmaf(-q, nf, a), rn, q);
            if (q1 != a / nf) bad++;
        }
    }
    return bad;
}

int main(void) {
    const long b0 = check(1), b1 = check(0);
    printf("centre mismatches %ld, integer mismatches %ld\n", b0, b1);
    return (b0 || b1) ? 1 : 0;
}
