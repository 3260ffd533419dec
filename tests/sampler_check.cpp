// Host check of the two-pass batch drawing (madpose_amd/csrc/host/batch_draw.h)
// against the draw-by-draw loop: same solver types, iteration lists, kept sample
// indices, stream snapshots and end states.  Built and run by tests/test_sampler_cpu.py.
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

#include "batch_draw.h"

using namespace mp;

static bool same_stream(Mt19937 a, Mt19937 b) {
    if (a.draws() != b.draws()) return false;
    for (int k = 0; k < 700; ++k) // across a block boundary
        if (a() != b()) return false;
    return true;
}

// argv[1]: the mode under test (1 = scalar two passes, 2 = AVX-512 two passes)
int main(int argc, char **argv) {
    const int mode = argc > 1 ? std::atoi(argv[1]) : 2;
    if (mode == 2 && !draw_simd_available()) {
        std::printf("SKIP no AVX-512 on this host\n");
        return 0;
    }
    struct Case {
        int n, a, c;
        double p0, p1;
        uint32_t seed, B;
    };
    const Case cases[] = {
        {2000, 3, 5, 1.0, 1.0, 0, 32768}, {2000, 3, 5, 0.3, 2.0, 7, 5000}, {7, 3, 5, 1.0, 1.0, 1, 4096},
        {13, 4, 6, 1.0, 0.5, 2, 4096},    {9, 4, 7, 1.0, 1.0, 3, 3000},    {4000, 4, 7, 1.0, 1.0, 4, 32768},
        {2000, 4, 6, 2.0, 1.0, 5, 1},     {2000, 3, 5, 1.0, 0.0, 6, 2048}, {300, 3, 5, 1.0, 1.0, 8, 777},
    };
    double t_one = 0, t_two = 0;
    uint64_t iters = 0;
    for (const Case &c : cases) {
        IterationStream rs;
        rs.seed(c.seed);
        rs.n = c.n;
        rs.prior[0] = c.p0;
        rs.prior[1] = c.p1;
        rs.ss[0][0] = rs.ss[0][1] = c.a;
        rs.ss[1][2] = c.c;
        // two batches in a row, so the second starts mid-block with pick already set
        IterationStream r1 = rs, r2 = rs;
        for (int rep = 0; rep < 2; ++rep) {
            const uint32_t B = c.B;
            std::vector<int> s1(9 * (size_t)B, -1), s2(9 * (size_t)B, -1);
            Batch g1, g2;
            auto t0 = std::chrono::steady_clock::now();
            draw_batch(r1, g1, B, 0, s1.data(), nullptr, 0);
            auto t1 = std::chrono::steady_clock::now();
            draw_batch(r2, g2, B, 0, s2.data(), nullptr, mode);
            auto t2 = std::chrono::steady_clock::now();
            t_one += std::chrono::duration<double>(t1 - t0).count();
            t_two += std::chrono::duration<double>(t2 - t1).count();
            iters += B;
            bool ok = g1.types == g2.types && g1.nmd == g2.nmd && g1.npt == g2.npt &&
                      g1.snaps.size() == g2.snaps.size() && same_stream(r1.sel, r2.sel) &&
                      same_stream(r1.samp, r2.samp);
            for (size_t k = 0; ok && k < g1.snaps.size(); ++k)
                ok = same_stream(g1.snaps[k].sel, g2.snaps[k].sel) && same_stream(g1.snaps[k].samp, g2.snaps[k].samp);
            for (uint32_t j = 0; ok && j < B; ++j) {
                const int kept = g1.types[j] == 0 ? c.a : c.c;
                for (int k = 0; k < kept; ++k) ok = ok && s1[8 * (size_t)j + k] == s2[8 * (size_t)j + k];
            }
            ok = ok && std::memcmp(s1.data() + 8 * (size_t)B, s2.data() + 8 * (size_t)B, sizeof(int) * B) == 0;
            if (!ok) {
                std::printf("MISMATCH mode=%d n=%d a=%d c=%d seed=%u rep=%d\n", mode, c.n, c.a, c.c, c.seed, rep);
                return 1;
            }
        }
    }
    std::printf("OK mode %d, %llu iterations: one-pass %.2f ns/it, two-pass %.2f ns/it\n", mode,
                (unsigned long long)iters, 1e9 * t_one / iters, 1e9 * t_two / iters);
    return 0;
}
