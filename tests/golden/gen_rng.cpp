// Golden random streams from this container's libstdc++ (GCC 11.4).
// The reference's sampler / solver selection / LO shuffles all consume
// std::mt19937 through std::uniform_int_distribution<int> and
// std::uniform_real_distribution<double> (src/hybrid_ransac.h:64,79-80,226-229;
// RansacLib sampling.h / utils.h, not vendored).  This program records those
// streams so the product's own RNG restatement can be pinned bit-for-bit.
//
// Build + run (writes tests/golden/rng_gcc11.json):
//   g++ -O2 -std=c++17 tests/golden/gen_rng.cpp -o /tmp/gen_rng && /tmp/gen_rng > tests/golden/rng_gcc11.json
#include <cstdio>
#include <random>
#include <vector>

int main() {
    std::printf("{\n");
    const unsigned seeds[] = {0u, 1u, 42u, 5489u};
    // raw engine outputs
    std::printf("  \"raw\": {");
    for (int si = 0; si < 4; ++si) {
        std::mt19937 g(seeds[si]);
        std::printf("%s\"%u\": [", si ? ", " : "", seeds[si]);
        for (int i = 0; i < 2000; ++i) std::printf("%s%u", i ? "," : "", (unsigned)g());
        std::printf("]");
    }
    std::printf("},\n");
    // uniform_int_distribution<int>(0, n-1)
    const int ns[] = {2, 3, 55, 193, 782, 2000, 4000, 1 << 20, 2147483647};
    std::printf("  \"uint\": {");
    bool first = true;
    for (int si = 0; si < 4; ++si) {
        for (int n : ns) {
            std::mt19937 g(seeds[si]);
            std::uniform_int_distribution<int> d(0, n - 1);
            std::printf("%s\"%u_%d\": [", first ? "" : ", ", seeds[si], n);
            first = false;
            for (int i = 0; i < 1000; ++i) std::printf("%s%d", i ? "," : "", d(g));
            std::printf("]");
        }
    }
    std::printf("},\n");
    // uniform_int_distribution<int>(a, b) with a > 0 (partial Fisher-Yates draws)
    std::printf("  \"uint_ab\": {");
    first = true;
    for (int si = 0; si < 4; ++si) {
        std::mt19937 g(seeds[si]);
        std::printf("%s\"%u\": [", first ? "" : ", ", seeds[si]);
        first = false;
        for (int i = 0; i < 1000; ++i) {
            std::uniform_int_distribution<int> d(i % 300, 300 + (i % 17));
            std::printf("%s%d", i ? "," : "", d(g));
        }
        std::printf("]");
    }
    std::printf("},\n");
    // uniform_real_distribution<double>(0, s) printed with full precision
    std::printf("  \"ureal\": {");
    first = true;
    const double sums[] = {1.0, 2.0};
    for (int si = 0; si < 4; ++si) {
        for (double s : sums) {
            std::mt19937 g(seeds[si]);
            std::uniform_real_distribution<double> d(0.0, s);
            std::printf("%s\"%u_%g\": [", first ? "" : ", ", seeds[si], s);
            first = false;
            for (int i = 0; i < 1000; ++i) std::printf("%s%.17g", i ? "," : "", d(g));
            std::printf("]");
        }
    }
    std::printf("}\n}\n");
    return 0;
}
