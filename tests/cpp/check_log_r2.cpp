// log_r2 (the polar transform's table-driven log, df_rng.hpp) against glibc's log: the largest
// difference in ulps over r2 values from the pcg32 polar stream itself, uniform (0, 1], values within
// 2^-20 of 1, and tiny values; and glibc_log (df_rng.hpp, the default) for bit identity over the same
// arguments plus the near-1 band glibc treats apart. argv[1] = count per class.
// Prints "max_ulp N over M ... glibc_log_mismatch K".
#include "df_rng.hpp"
#include <cmath>
#include <cstdio>
#include <cstdlib>
using namespace dfamd;
static long long ulps(double a, double b)
{
    long long x = (long long)dbits(a), y = (long long)dbits(b);
    if (x < 0) x = (long long)0x8000000000000000ull - x;
    if (y < 0) y = (long long)0x8000000000000000ull - y;
    return x > y ? x - y : y - x;
}
int main(int argc, char **argv)
{
    const long long n = argc > 1 ? atoll(argv[1]) : 5000000;
    static LogTabEntry tab[kLogTab];
    build_log_table(tab);
    long long worst = 0, count = 0, off1 = 0, gl_bad = 0;
    double worst_x = 0;
    auto check = [&](double x) {
        if (!(x > 0 && x <= 1)) return;
        const long long u = ulps(log_r2(x, tab), std::log(x));
        if (u > worst) { worst = u; worst_x = x; }
        off1 += u > 0;
        gl_bad += dbits(glibc_log(x)) != dbits(std::log(x));
        ++count;
    };
    uint64_t s = pcg_seed1(42);
    for (long long i = 0; i < n; ++i) { PolarAttempt a = polar_attempt(s); if (a.accept) check(a.r2); }
    uint64_t t = pcg_seed1(7);
    for (long long i = 0; i < n; ++i) {
        uint64_t hi = pcg_output(t); t = t * kPcgMult + kPcgInc;
        uint64_t lo = pcg_output(t); t = t * kPcgMult + kPcgInc;
        const double u = (double)((hi << 21) ^ lo) * 0x1p-53;      // (0, 1)
        check(u > 0 ? u : 1.0);
        check(1.0 - u * 0x1p-20);                                   // near 1 from below
        check(std::ldexp(0.5 + 0.5 * u, -(int)(lo % 100)));         // tiny
        check(1.0 - u * 0x1p-4);                                    // glibc's near-1 band
    }
    check(1.0);
    check(0x1p-106);
    check(0x1.fffffffffffffp-1);
    printf("max_ulp %lld over %lld (differ: %lld) at %.17g glibc_log_mismatch %lld\n", worst, count, off1, worst_x,
           gl_bad);
    return worst > 1 || gl_bad != 0;
}
