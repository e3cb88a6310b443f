// pcg32 + libstdc++-11 polar-normal arithmetic shared by host setup and the HIP
// kernels. This restates (does not include) the reference's third-party RNG:
//   - pcg32 = setseq_xsh_rr_64_32 (pcg-cpp/include/pcg_random.hpp:1866), output
//     from the OLD state (output_previous, :413-437), XSH-RR (:845-872),
//     1-arg seeding state = (seed + inc)*mult + inc (:484-487), Brown jump (:639-662);
//   - generate_canonical<double,53> (random.tcc:3346-3378): lo + hi*2^32, /2^64,
//     clamp to nextafter(1,0);
//   - normal_distribution<double>::operator() polar method (random.tcc:1800-1835):
//     x then y from one attempt of 4 draws, accept 0 < x*x+y*y <= 1, emit y*m
//     first and cache x*m; ret*1.0 + 0.0 maps -0.0 to +0.0.
// Every floating-point line is written so that no FMA can be formed (the library
// is compiled with -ffp-contract=off), matching the reference's x86-64 -O2 code.
#pragma once
#include <cmath>
#include <cstdint>

#include "glibc_log_table.h"

#ifdef __HIPCC__
#define DF_HD __host__ __device__ __forceinline__
#else
#define DF_HD inline
#endif

namespace dfamd {

constexpr uint64_t kPcgMult = 6364136223846793005ULL;
constexpr uint64_t kPcgInc = 1442695040888963407ULL;
// kPcgMult^-1 mod 2^64: the state one step back, s = (s' - kPcgInc) * kPcgMultInv
constexpr uint64_t kPcgMultInv = 0xc097ef87329e28a5ULL;
static_assert(kPcgMult * kPcgMultInv == 1ULL, "pcg multiplier inverse");

DF_HD uint32_t pcg_output(uint64_t s)
{
    uint32_t rot = (uint32_t)(s >> 59);
    s ^= s >> 18;
    uint32_t x = (uint32_t)(s >> 27);
    return (x >> rot) | (x << ((32u - rot) & 31u));
}

DF_HD uint64_t pcg_seed1(uint64_t seed) { return (seed + kPcgInc) * kPcgMult + kPcgInc; }

// Affine jump state -> mult*state + plus that equals `delta` single steps.
struct PcgJump {
    uint64_t mult, plus;
};

DF_HD PcgJump pcg_jump(uint64_t delta)
{
    uint64_t cur_mult = kPcgMult, cur_plus = kPcgInc, acc_mult = 1, acc_plus = 0;
    while (delta > 0) {
        if (delta & 1u) {
            acc_mult *= cur_mult;
            acc_plus = acc_plus * cur_mult + cur_plus;
        }
        cur_plus = (cur_mult + 1) * cur_plus;
        cur_mult *= cur_mult;
        delta >>= 1;
    }
    return {acc_mult, acc_plus};
}

DF_HD uint64_t pcg_advance(uint64_t state, uint64_t delta)
{
    PcgJump j = pcg_jump(delta);
    return j.mult * state + j.plus;
}

// One polar attempt: consumes exactly 4 outputs starting at `state`.
struct PolarAttempt {
    double x, y, r2;
    bool accept;
};

DF_HD double canonical_from(uint32_t lo, uint32_t hi)
{
    double sum = 0.0;
    sum += (double)lo * 1.0;
    sum += (double)hi * 4294967296.0;
    double ret = sum / 18446744073709551616.0;
    // nextafter(1.0, 0.0) == 1 - 2^-53
    if (ret >= 1.0) ret = 0.99999999999999988897769753748434595763683319091796875;
    return ret;
}

DF_HD PolarAttempt polar_attempt(uint64_t &state)
{
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[i] = pcg_output(state);
        state = state * kPcgMult + kPcgInc;
    }
    PolarAttempt a;
    a.x = 2.0 * canonical_from(o[0], o[1]) - 1.0;
    a.y = 2.0 * canonical_from(o[2], o[3]) - 1.0;
    double xx = a.x * a.x;
    double yy = a.y * a.y;
    a.r2 = xx + yy;
    a.accept = !(a.r2 > 1.0 || a.r2 == 0.0);
    return a;
}

// The same attempt from its first state without the fourth step: `s3` is left at the state of the
// fourth output, so the state after the attempt is one more step (s3 * mult + inc), which only the
// call's last attempt needs.
DF_HD PolarAttempt polar_draws(uint64_t s, uint64_t &s3)
{
    uint32_t o[4];
    o[0] = pcg_output(s);
    s = s * kPcgMult + kPcgInc;
    o[1] = pcg_output(s);
    s = s * kPcgMult + kPcgInc;
    o[2] = pcg_output(s);
    s = s * kPcgMult + kPcgInc;
    o[3] = pcg_output(s);
    s3 = s;
    PolarAttempt a;
    a.x = 2.0 * canonical_from(o[0], o[1]) - 1.0;
    a.y = 2.0 * canonical_from(o[2], o[3]) - 1.0;
    double xx = a.x * a.x;
    double yy = a.y * a.y;
    a.r2 = xx + yy;
    a.accept = !(a.r2 > 1.0 || a.r2 == 0.0);
    return a;
}

// Two pcg32 steps at once: state -> mult2*state + inc2 (pcg_jump(2)).
constexpr uint64_t kPcgMult2 = 0x685f98a2018fade9ULL;
constexpr uint64_t kPcgInc2 = 0x1a08ee1184ba6d32ULL;

// K1's accept decision, screened in float from the high words; it decides all but the attempts within
// 1e-5 of the unit circle or of the origin, which take the exact double test:
// |xf - x| <= 2^-24*2 (fl(hi)) + 2^-24 (subtract) + 2^-31 (dropped lo) < 1.9e-7, so
// |r2f - r2| < 2*2*1.9e-7 + 3 float roundings of values <= 2 < 1.2e-6.
// Computed from the attempt's first state s0, without stepping it: it needs
// only the high words o[1] = output(s1) and o[3] = output(s3), i.e. two 64-bit multiply-adds (s1 = one
// step, s3 = two more) and two outputs instead of four of each. Returns 1 (accept), 0 (reject) or -1
// (within 1e-5 of the circle or the origin: the caller redoes the exact double test, polar_attempt).
// The same screen from the states s1, s3 (1 and 3 steps after the attempt's start) directly.
DF_HD int polar_screen13(uint64_t s1, uint64_t s3)
{
    const float xf = (float)pcg_output(s1) * 4.656612873077392578125e-10f - 1.0f; // 2^-31
    const float yf = (float)pcg_output(s3) * 4.656612873077392578125e-10f - 1.0f;
    const float r2f = xf * xf + yf * yf;
    if (r2f > 1e-5f && r2f < 1.0f - 1e-5f) return 1;
    if (r2f > 1.0f + 1e-5f) return 0;
    return -1;
}

DF_HD int polar_screen(uint64_t s0)
{
    const uint64_t s1 = s0 * kPcgMult + kPcgInc;
    return polar_screen13(s1, s1 * kPcgMult2 + kPcgInc2);
}

// ---- log(r2) for the polar transform, r2 in (0, 1] (a normal double: r2 >= 2^-106 > DBL_MIN).
// Table-driven (Tang): r2 = 2^k * m with m in [sqrt(1/2), sqrt(2)); c = the centre of m's cell (width
// 1/256 below 1, 1/128 above; c = 1 exactly for the two cells around 1, so log(1) = 0 and r2 -> 1 has
// no cancellation); r = m * (1/c) - 1 by one FMA, |r| < 2^-7; log(m) = -log(1/c) + log1p(r), log1p by a
// degree-8 polynomial (truncation < 2^-59 relative). k*ln2_hi + T_hi is exact (both on a 2^-43 grid),
// the rest is added small to large. ~25 VALU against ~85 for the device library's log; error about
// 0.5 ulp, within 1 ulp of glibc's log (tests/test_rng_log.py: 2e7 arguments, and the GPU normals
// stay within 2 ulp of the reference's). The host builds the table (build_log_table).
struct LogTabEntry {
    double rinv, thi, tlo, pad; // 1/c rounded; -log(rinv) = thi + tlo, thi on the 2^-43 grid
};
constexpr int kLogTab = 256;     // index: top 7 mantissa bits, +128 in the [1, sqrt 2) binade
constexpr double kLn2Hi = 0x1.62e42fefa3800p-1; // ln 2 on the 2^-43 grid
constexpr double kLn2Lo = 0x1.ef35793c76730p-45; // ln 2 - kLn2Hi

DF_HD uint64_t dbits(double x) { return __builtin_bit_cast(uint64_t, x); }
DF_HD double dfrom(uint64_t b) { return __builtin_bit_cast(double, b); }

DF_HD double log_r2(double x, const LogTabEntry *tab)
{
    uint64_t mb = (dbits(x) & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull; // m in [1, 2)
    int k = (int)(dbits(x) >> 52) - 1023;
    const bool fold = mb >= 0x3FF6A09E667F3BCDull; // m >= sqrt(2): m / 2, k + 1 (exponent field only)
    if (fold) {
        mb -= 0x0010000000000000ull;
        k += 1;
    }
    const LogTabEntry &e = tab[(int)((mb >> 45) & 0x7F) + (fold ? 0 : 128)];
    const double m = dfrom(mb);
    const double r = fma(m, e.rinv, -1.0);
    const double r2 = r * r;
    double q = fma(r, -0.125, 0x1.2492492492492p-3);  // 1/7
    q = fma(r, q, -0x1.5555555555555p-3);             // -1/6
    q = fma(r, q, 0x1.999999999999ap-3);              // 1/5
    q = fma(r, q, -0.25);
    q = fma(r, q, 0x1.5555555555555p-2);              // 1/3
    q = fma(r, q, -0.5);
    const double p = r2 * q;
    const double dk = (double)k;
    const double hi = fma(dk, kLn2Hi, e.thi);          // exact
    const double lo = fma(dk, kLn2Lo, e.tlo);
    return hi + (r + (p + lo));
}

// ---- glibc's own log for r2 in (0, 1] (fast_log 2, the default): the reference's normals come from
// glibc 2.35's log (random.tcc:1831), which on x86-64 CPUs with FMA is the ifunc __log_fma, i.e.
// sysdeps/ieee754/dbl-64/e_log.c built with -mfma: r = fma(z, invc, -1) and GCC's contraction of
// every a*b + c whose product has no other use. Restated here with those fmas explicit, on the
// constants of glibc_log_table.h; it returns glibc's bits for every argument tested
// (tests/test_rng_log.py: 1e8 uniform doubles in (0, 1], the near-1 band, powers of two), so the
// normals, and with them the fields, are bit-identical to the reference's.
// glibc's near-1 band: ix - LO < HI - LO (x in [1 - 2^-4, 1 + 0x1.09p-4)); 6.25% of the polar r2.
constexpr uint64_t kGlNearLo = 0x3FEE000000000000ull; // asuint64(1.0 - 0x1p-4)
constexpr uint64_t kGlNearHi = 0x3FF1090000000000ull; // asuint64(1.0 + 0x1.09p-4)
DF_HD bool glibc_log_near1(double x) { return dbits(x) - kGlNearLo < kGlNearHi - kGlNearLo; }

// The two halves of glibc_log below, for callers that sort their arguments by band first (the dense
// noise generation defers near-1 lanes into batches of their own, so neither half diverges).
DF_HD double glibc_log_band1(double x);
DF_HD double glibc_log_main(double x);

DF_HD double glibc_log(double x)
{
    return glibc_log_near1(x) ? glibc_log_band1(x) : glibc_log_main(x);
}

DF_HD double glibc_log_band1(double x)
{
    {
        if (dbits(x) == 0x3FF0000000000000ull) return 0.0;
        const double r = x - 1.0;
        const double r2 = r * r;
        const double r3 = r * r2;
        const double p3 = fma(r3, kGlB[10], fma(r2, kGlB[9], fma(r, kGlB[8], kGlB[7])));
        const double p2 = fma(r3, p3, fma(r2, kGlB[6], fma(r, kGlB[5], kGlB[4])));
        const double p1 = fma(r3, p2, fma(r2, kGlB[3], fma(r, kGlB[2], kGlB[1])));
        double w = r * 0x1p27;
        const double rhi = r + w - w;
        const double rlo = r - rhi;
        w = rhi * rhi * kGlB[0]; // exact (B[0] = -0.5)
        const double hi = r + w;
        double lo = r - hi + w;
        lo = fma(kGlB[0] * rlo, rhi + r, lo);
        double y = fma(r3, p1, lo); // y = r3 * p1; y += lo
        y += hi;
        return y;
    }
}

DF_HD double glibc_log_main(double x)
{
    const uint64_t ix = dbits(x);
    constexpr uint64_t OFF = 0x3FE6000000000000ull;
    const uint64_t tmp = ix - OFF;
    const int i = (int)((tmp >> 45) & 127);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & (0xFFFull << 52));
    const double invc = kGlTab[2 * i], logc = kGlTab[2 * i + 1];
    const double z = dfrom(iz);
    const double r = fma(z, invc, -1.0);
    const double kd = (double)k;
    const double w = fma(kd, kGlLn2Hi, logc);
    const double hi = w + r;
    const double lo = fma(kd, kGlLn2Lo, w - hi + r);
    const double r2 = r * r;
    const double q = fma(r2, fma(r, kGlA[4], kGlA[3]), fma(r, kGlA[2], kGlA[1]));
    const double y = fma(r * r2, q, fma(r2, kGlA[0], lo)) + hi;
    return y;
}

// The log_r2 table (host): cell centres, 1/c rounded to double, -log(1/c) in x87 long double
// (64-bit significand) split into a 2^-43-grid head and a tail.
inline void build_log_table(LogTabEntry *tab)
{
    for (int idx = 0; idx < kLogTab; ++idx) {
        const bool fold = idx < 128;
        const int j = idx & 127;
        double c;
        if (fold) c = (j == 127) ? 1.0 : 0.5 * (1.0 + (j + 0.5) / 128.0);
        else c = (j == 0) ? 1.0 : 1.0 + (j + 0.5) / 128.0;
        const double rinv = 1.0 / c;
        const long double T = -logl((long double)rinv);
        const long double grid = 8796093022208.0L; // 2^43
        const double thi = (double)(nearbyintl(T * grid) / grid);
        tab[idx] = LogTabEntry{rinv, thi, (double)(T - (long double)thi), 0.0};
    }
}

} // namespace dfamd
