// polar_screen (K1's float-screened accept test, exact polar_attempt where it returns -1) ==
// polar_attempt().accept, the exact double test restated from libstdc++ random.tcc:1800-1835,
// on N attempts per seed (argv[1]).
#include "df_rng.hpp"
#include <cstdio>
#include <cstdlib>
#include <initializer_list>
using namespace dfamd;
int main(int argc, char **argv) {
    const long long per = argc > 1 ? atoll(argv[1]) : 50000000;
    long long n = 0, diff = 0, unsure = 0;
    for (uint64_t seed : {42ull, 1234ull, 7ull, 99991ull}) {
        uint64_t s1 = pcg_seed1(seed);
        for (long long i = 0; i < per; ++i) {
            const uint64_t s0 = s1;
            const bool a = polar_attempt(s1).accept;
            const int v = polar_screen(s0);
            uint64_t s = s0;
            const bool b = v < 0 ? polar_attempt(s).accept : v > 0;
            unsure += v < 0;
            diff += a != b; ++n;
        }
    }
    printf("attempts %lld mismatches %lld unsure %lld\n", n, diff, unsure);
    return diff != 0;
}
