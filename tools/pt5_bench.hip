// The calibrated 5-point root stage two ways on the same random samples: the
// one-lane-per-sample kernel (pt_roots_kernel<kCal>) and the 16-lane-group kernel
// (group_5pt.h).  Checks that they produce the same candidates and times both;
// with phase counters of the group kernel.  Build + run (on an MI355X):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/pt5_bench.hip -o tools/pt5_bench
//   tools/pt5_bench [samples]
#define MP_GROUP5_PROFILE 1
#define MP_GROUP_PROFILE 1
#include "../madpose_amd/csrc/kernels/kernels.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace mp;

#define CHECK(x)                                                                                                      \
    do {                                                                                                               \
        hipError_t e = (x);                                                                                            \
        if (e != hipSuccess) {                                                                                         \
            std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);                \
            std::exit(1);                                                                                              \
        }                                                                                                              \
    } while (0)

int main(int argc, char **argv) {
    const int ns = argc > 1 ? std::atoi(argv[1]) : 16384;
    const int n = 2000;
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> U(-1, 1);
    // a rigid scene: points in front of both cameras, half of them outliers
    std::vector<double> x0u(n), x0v(n), x1u(n), x1v(n), d0(n), d1(n), r0(n), r1(n);
    const double f = 500, cx = 320, cy = 240, ang = 0.2;
    const double R[9] = {std::cos(ang), 0, std::sin(ang), 0, 1, 0, -std::sin(ang), 0, std::cos(ang)};
    const double t[3] = {0.5, 0.05, 0.1};
    for (int i = 0; i < n; ++i) {
        const double X[3] = {2 * U(rng), 1.5 * U(rng), 4 + 2 * U(rng)};
        double Y[3];
        for (int k = 0; k < 3; ++k) Y[k] = R[3 * k] * X[0] + R[3 * k + 1] * X[1] + R[3 * k + 2] * X[2] + t[k];
        x0u[i] = f * X[0] / X[2] + cx;
        x0v[i] = f * X[1] / X[2] + cy;
        x1u[i] = f * Y[0] / Y[2] + cx + (i % 2 ? 0.0 : 80 * U(rng));
        x1v[i] = f * Y[1] / Y[2] + cy;
        d0[i] = X[2];
        d1[i] = Y[2];
        const double a[3] = {(x0u[i] - cx) / f, (x0v[i] - cy) / f, 1}, b[3] = {(x1u[i] - cx) / f, (x1v[i] - cy) / f, 1};
        r0[i] = 1 / std::sqrt(a[0] * a[0] + a[1] * a[1] + 1);
        r1[i] = 1 / std::sqrt(b[0] * b[0] + b[1] * b[1] + 1);
    }
    auto up = [&](const std::vector<double> &v) {
        double *p;
        CHECK(hipMalloc(&p, v.size() * 8));
        CHECK(hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice));
        return p;
    };
    PairData D{up(x0u), up(x0v), up(x1u), up(x1v), up(d0), up(d1), up(r0), up(r1)};
    PairConst C{};
    C.variant = kCal;
    C.n = n;
    const double K[9] = {f, 0, cx, 0, f, cy, 0, 0, 1}, Ki[9] = {1 / f, 0, -cx / f, 0, 1 / f, -cy / f, 0, 0, 1};
    for (int k = 0; k < 9; ++k) {
        C.K0[k] = C.K1[k] = K[k];
        C.K0i[k] = C.K1i[k] = Ki[k];
    }
    std::vector<int> samples((size_t)ns * kSampleStride, 0), list(ns);
    std::uniform_int_distribution<int> UI(0, n - 1);
    for (int s = 0; s < ns; ++s) {
        list[s] = s;
        for (int j = 0; j < 5; ++j) {
            int v;
            bool dup;
            do {
                v = UI(rng);
                dup = false;
                for (int q = 0; q < j; ++q) dup |= samples[(size_t)s * kSampleStride + q] == v;
            } while (dup);
            samples[(size_t)s * kSampleStride + j] = v;
        }
    }
    int *d_samples, *d_list, *d_n1, *d_n2;
    double *d_c1, *d_c2;
    CHECK(hipMalloc(&d_samples, samples.size() * 4));
    CHECK(hipMalloc(&d_list, ns * 4));
    CHECK(hipMemcpy(d_samples, samples.data(), samples.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_list, list.data(), ns * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_n1, ns * 4));
    CHECK(hipMalloc(&d_n2, ns * 4));
    CHECK(hipMalloc(&d_c1, (size_t)ns * kCandStride * 8));
    CHECK(hipMalloc(&d_c2, (size_t)ns * kCandStride * 8));
    CHECK(hipMemset(d_c1, 0, (size_t)ns * kCandStride * 8));
    CHECK(hipMemset(d_c2, 0, (size_t)ns * kCandStride * 8));
    auto run_lane = [&] { pt_roots_kernel<kCal><<<(ns + 63) / 64, 64>>>(D, C, d_list, ns, d_samples, d_c1, d_n1); };
    auto run_group = [&] {
        pt_roots5_group_kernel<<<(ns + kS5 - 1) / kS5, 64>>>(D, C, d_list, ns, d_samples, d_c2, d_n2, kCandStride);
    };
    run_lane();
    run_group();
    CHECK(hipDeviceSynchronize());
    std::vector<int> n1(ns), n2(ns);
    std::vector<double> c1((size_t)ns * kCandStride), c2((size_t)ns * kCandStride);
    CHECK(hipMemcpy(n1.data(), d_n1, ns * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(n2.data(), d_n2, ns * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(c1.data(), d_c1, c1.size() * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(c2.data(), d_c2, c2.size() * 8, hipMemcpyDeviceToHost));
    long tot1 = 0, tot2 = 0, cnt_diff = 0, bit_diff = 0;
    double worst = 0;
    for (int s = 0; s < ns; ++s) {
        tot1 += n1[s];
        tot2 += n2[s];
        if (n1[s] != n2[s]) {
            if (cnt_diff < 5) std::printf("sample %d: lane %d roots, group %d roots\n", s, n1[s], n2[s]);
            ++cnt_diff;
            continue;
        }
        bool shown = false;
        for (int e = 0; e < 9 * n1[s]; ++e) {
            const double a = c1[(size_t)s * kCandStride + e], b = c2[(size_t)s * kCandStride + e];
            if (a != b) ++bit_diff;
            worst = std::max(worst, std::fabs(a - b));
            if (std::fabs(a - b) > 1e-6 && !shown && bit_diff < 40) {
                shown = true;
                std::printf("sample %d (%d roots) differs at value %d:\n", s, n1[s], e);
                for (int k = 0; k < n1[s]; ++k) {
                    std::printf("  lane  E%d:", k);
                    for (int q = 0; q < 9; ++q) std::printf(" %+.6f", c1[(size_t)s * kCandStride + 9 * k + q]);
                    std::printf("\n  group E%d:", k);
                    for (int q = 0; q < 9; ++q) std::printf(" %+.6f", c2[(size_t)s * kCandStride + 9 * k + q]);
                    std::printf("\n");
                }
            }
        }
    }
    std::printf("samples %d: candidates lane %ld group %ld; samples with different counts %ld; values differing %ld "
                "(max abs diff %.3g)\n",
                ns, tot1, tot2, cnt_diff, bit_diff, worst);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int which = 0; which < 2; ++which) {
        unsigned long long z[8] = {0};
        CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g5_prof), z, sizeof(z)));
        CHECK(hipMemcpyToSymbol(HIP_SYMBOL(gs_prof), z, 4 * sizeof(z[0])));
        const int reps = 10;
        CHECK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) which ? run_group() : run_lane();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        std::printf("%s kernel: %.3f ms per launch of %d samples\n", which ? "group" : "lane", ms / reps, ns);
        if (which) {
            CHECK(hipMemcpyFromSymbol(z, HIP_SYMBOL(g5_prof), sizeof(z)));
            const char *names[8] = {"nullspace", "template row", "gauss-jordan", "det B", "sturm chain", "grid counts",
                                    "cells", "refine+E"};
            double tot = 0;
            for (int i = 0; i < 8; ++i) tot += (double)z[i];
            for (int i = 0; i < 8; ++i)
                std::printf("  %-13s %5.1f%%  (%.0f ticks/group)\n", names[i], 100.0 * z[i] / tot,
                            (double)z[i] / (reps * (double)ns));
            unsigned long long zs[4];
            CHECK(hipMemcpyFromSymbol(zs, HIP_SYMBOL(gs_prof), sizeof(zs)));
            const char *sn[4] = {"chain", "grid counts", "cells", "refine"};
            for (int i = 0; i < 4; ++i)
                std::printf("    sturm %-11s %.1f ticks/workgroup\n", sn[i], (double)zs[i] * kS5 / (reps * (double)ns));
        }
    }
    return cnt_diff == 0 ? 0 : 3;
}
