// polar_accept (K1's float-screened accept test) == polar_attempt().accept, the exact double
// test restated from libstdc++ random.tcc:1800-1835, on N attempts per seed (argv[1]).
#include "df_rng.hpp"
#include <cstdio>
#include <cstdlib>
#include <initializer_list>
using namespace dfamd;
int main(int argc, char **argv) {
    const long long per = argc > 1 ? atoll(argv[1]) : 50000000;
    long long n = 0, diff = 0, exact = 0;
    for (uint64_t seed : {42ull, 1234ull, 7ull, 99991ull}) {
        uint64_t s1 = pcg_seed1(seed), s2 = s1;
        for (long long i = 0; i < per; ++i) {
            const bool a = polar_attempt(s1).accept;
            const bool b = polar_accept(s2);
            diff += a != b; ++n;
        }
        if (s1 != s2) { printf("state mismatch\n"); return 1; }
    }
    printf("attempts %lld mismatches %lld\n", n, diff);
    return diff != 0;
}
