/* tests/test_oracle.py::test_ess_quotient_is_ieee_division: k_ess_reg (kernels/stats.hip) forms s / n as
 * q0 = RN(s * rn), q = RN(q0 + (s - n q0) rn) with rn = RN(1 / n) (two fmas); orc_ess divides.  This checks the
 * two agree bit for bit on random, near-exact and all-ones-mantissa quotients for n = 1 .. NMAX.
 * usage: qdiv_check NMAX PER_N  -> prints "checked K mismatches M", exit status 1 on any mismatch */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint64_t st = 88172645463325252ull;
static uint64_t rnd(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static double bits(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
int main(int argc, char** argv) {
    const int nmax = argc > 1 ? atoi(argv[1]) : 1024;
    const long per = argc > 2 ? atol(argv[2]) : 10000;
    long bad = 0, tot = 0;
    for (int n = 1; n <= nmax; ++n) {
        const double nd = (double)n, rn = 1.0 / nd;
        for (long i = 0; i < per; ++i) {
            double x;
            switch (i % 4) {
                case 0: x = bits((rnd() & 0x800fffffffffffffull) | ((uint64_t)(1023 - 60 + rnd() % 120) << 52)); break;
                case 1: x = (double)(int64_t)(rnd() >> 12) * nd + (double)((int64_t)(rnd() % 5) - 2); break;
                case 2: x = bits(((uint64_t)(1023 - 20 + rnd() % 40) << 52) | 0x000fffffffffffffull) * (rnd() & 1 ? 1 : -1); break;
                default: x = nextafter((double)(int64_t)(rnd() % 100000) * nd, (rnd() & 1) ? INFINITY : -INFINITY);
            }
            const double q0 = x * rn;
            const double q = fma(fma(-q0, nd, x), rn, q0);
            const double ref = x / nd;
            ++tot;
            if (memcmp(&q, &ref, 8) != 0) {
                if (bad < 5) printf("n %d x %a: %a vs %a\n", n, x, q, ref);
                ++bad;
            }
        }
    }
    printf("checked %ld mismatches %ld\n", tot, bad);
    return bad != 0;
}
