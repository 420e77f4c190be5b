/* Host check of div_rn (opensim-moco_amd/csrc/core.hpp): the division by a
 * fixed finite-difference step from its reciprocal and two fma residual
 * corrections against the IEEE division a / b, bit for bit (NaNs equal).
 * Built and run by tests/test_div_rn.py (gcc, contraction off).
 *   div_rn_check <samples per step> <seed>  -> prints "mismatches checked" */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static double div_rn(double a, double b, double y) {   /* core.hpp div_rn */
    double q = a * y;
    double r = fma(-q, b, a);
    q = fma(r, y, q);
    r = fma(-q, b, a);
    q = fma(r, y, q);
    const double m = fabs(a);
    if (!(m >= 0x1p-900 && m <= 0x1p+900) && m != 0.0 && m == m) q = a / b;
    return m == 0.0 ? a * y : q;
}

static uint64_t st;
static uint64_t next(void) {   /* splitmix64 */
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static uint64_t ubits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    st = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    /* steps: the solver's (sqrt(eps) multiples, 1e-k), all-ones and
     * power-of-two significands, and random ones across [2^-60, 2^59] */
    double steps[64];
    int ns = 0;
    const double fixed[] = {1e-8, 1e-6, 1e-5, 1e-4, 1.4901161193847656e-08, 2.9802322387695312e-08, 2e-8,
                            0x1.fffffffffffffp-27, 0x1p-30, 0x1.0000000000001p-20, 0x1p-60, 0x1.fffffffffffffp+58,
                            3.0, 0.1, 1.0 / 3.0};
    for (size_t i = 0; i < sizeof fixed / sizeof fixed[0]; ++i) steps[ns++] = fixed[i];
    while (ns < 64) {
        const int e = (int)(next() % 120) - 60;
        steps[ns++] = ldexp(1.0 + (double)(next() >> 12) * 0x1p-52, e) * (ns & 1 ? 1.0 : 0.999);
    }
    const double special[] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 0x1p-1074, -0x1p-1022, 0x1p-900,
                              0x1.fffffffffffffp-901, 0x1p+900, 0x1.0000000000001p+900, 0x1.fffffffffffffp+1023,
                              1.0, -1.0};
    long bad = 0, checked = 0;
    for (int s = 0; s < ns; ++s) {
        const double b = steps[s], y = 1.0 / b;
        for (long k = 0; k < n + (long)(sizeof special / sizeof special[0]); ++k) {
            double a;
            if (k >= n) a = special[k - n];
            else {
                const uint64_t u = next();
                switch (u & 3) {
                case 0:   /* any finite exponent in the fast range, any significand */
                    a = ldexp(1.0 + (double)(next() >> 12) * 0x1p-52, (int)((u >> 2) % 1800) - 900);
                    break;
                case 1: { /* a difference of two nearby values (a perturbed lane minus the base) */
                    const double v = ldexp(1.0 + (double)(next() >> 12) * 0x1p-52, (int)((u >> 2) % 40) - 20);
                    a = (v + v * b * ((double)(next() >> 11) * 0x1p-53)) - v;
                    break;
                }
                case 2:   /* small integers times ulps (quotients near exact) */
                    a = (double)((int64_t)(next() % 2000001) - 1000000) * b * 0x1p-10;
                    break;
                default:  /* raw bits (denormals, huge, NaN, infinities) */
                    a = bits(next());
                }
                if (u & 4) a = -a;
            }
            const double q = div_rn(a, b, y), r = a / b;
            ++checked;
            if (ubits(q) != ubits(r) && !(q != q && r != r)) {
                if (bad < 5) fprintf(stderr, "a=%a b=%a div_rn=%a a/b=%a\n", a, b, q, r);
                ++bad;
            }
        }
    }
    printf("%ld %ld\n", bad, checked);
    return 0;
}
