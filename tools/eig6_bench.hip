// The shared-focal 6-point root stage two ways on the same random samples (a rigid
// scene, half of the correspondences outliers, as in an estimator batch): the DFT +
// Sturm group kernel (group_6pt.h) and the deflated eigenproblem (eig6.h: pencil,
// deflation, 15 x 15 eigen kernels).  Times every kernel with HIP events, prints the
// eigen kernel's phase ticks (balance / elmhes / hqr), balancing passes and QR
// iterations per sample, and how often the two root sets agree.  Build + run:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/eig6_bench.hip -o tools/eig6_bench
//   tools/eig6_bench [samples]
#define MP_EIG6_PROFILE 1
#include "../madpose_amd/csrc/kernels/kernels.hip"
#include "ab/group_6pt.h"
#include "ab/eig6_ab.h"

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
    const int ns = argc > 1 ? std::atoi(argv[1]) : 8192;
    const int n = 2000;
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> U(-1, 1);
    std::vector<double> x0u(n), x0v(n), x1u(n), x1v(n), d0(n), d1(n), r0(n, 1.0), r1(n, 1.0);
    const double f = 1.8, ang = 0.2;
    const double R[9] = {std::cos(ang), 0, std::sin(ang), 0, 1, 0, -std::sin(ang), 0, std::cos(ang)};
    const double t[3] = {0.5, 0.05, 0.1};
    for (int i = 0; i < n; ++i) {
        const double X[3] = {2 * U(rng), 1.5 * U(rng), 4 + 2 * U(rng)};
        double Y[3];
        for (int k = 0; k < 3; ++k) Y[k] = R[3 * k] * X[0] + R[3 * k + 1] * X[1] + R[3 * k + 2] * X[2] + t[k];
        x0u[i] = f * X[0] / X[2];
        x0v[i] = f * X[1] / X[2];
        x1u[i] = f * Y[0] / Y[2] + (i % 2 ? 0.0 : 0.3 * U(rng));
        x1v[i] = f * Y[1] / Y[2];
        d0[i] = X[2];
        d1[i] = Y[2];
    }
    auto up = [&](const std::vector<double> &v) {
        double *p;
        CHECK(hipMalloc(&p, v.size() * 8));
        CHECK(hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice));
        return p;
    };
    PairData D{up(x0u), up(x0v), up(x1u), up(x1v), up(d0), up(d1), up(r0), up(r1)};
    PairConst C{};
    C.variant = kSF;
    C.n = n;
    for (int k = 0; k < 9; ++k) C.K0[k] = C.K1[k] = C.K0i[k] = C.K1i[k] = (k % 4 == 0) ? 1.0 : 0.0;
    std::vector<int> samples((size_t)ns * kSampleStride, 0), list(ns);
    std::uniform_int_distribution<int> UI(0, n - 1);
    for (int s = 0; s < ns; ++s) {
        list[s] = s;
        for (int j = 0; j < 6; ++j) {
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
    double *d_c1, *d_c2, *d_pen;
    CHECK(hipMalloc(&d_samples, samples.size() * 4));
    CHECK(hipMalloc(&d_list, ns * 4));
    CHECK(hipMemcpy(d_samples, samples.data(), samples.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_list, list.data(), ns * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_n1, ns * 4));
    CHECK(hipMalloc(&d_n2, ns * 4));
    CHECK(hipMalloc(&d_c1, (size_t)ns * kCandStride * 8));
    CHECK(hipMalloc(&d_c2, (size_t)ns * kCandStride * 8));
    CHECK(hipMalloc(&d_pen, (size_t)ns * kPenStride * 8));
    hipEvent_t ev[9];
    double *d_pen2;
    CHECK(hipMalloc(&d_pen2, (size_t)ns * kPenStride * 8));
    int *d_n3, *d_n4;
    double *d_c3, *d_c4, *d_eig;
    CHECK(hipMalloc(&d_n4, ns * 4));
    CHECK(hipMalloc(&d_c4, (size_t)ns * kCandStride * 8));
    CHECK(hipMalloc(&d_eig, (size_t)ns * 30 * 8));
    CHECK(hipMalloc(&d_n3, ns * 4));
    CHECK(hipMalloc(&d_c3, (size_t)ns * kCandStride * 8));
    for (auto &evk : ev) CHECK(hipEventCreate(&evk));
    auto run = [&](bool timed, float *ms) {
        CHECK(hipEventRecord(ev[0]));
        pt_roots6_group_kernel<<<(ns + kGrpPerWg - 1) / kGrpPerWg, 64>>>(D, C, d_list, ns, d_samples, d_c1, d_n1,
                                                                          kCandStride);
        CHECK(hipEventRecord(ev[1]));
        pt_pencil6_kernel<<<(ns + kGrpPerWg - 1) / kGrpPerWg, 64>>>(D, d_list, ns, d_samples, d_c2, kCandStride,
                                                                      d_pen);
        CHECK(hipMemcpyAsync(d_pen2, d_pen, (size_t)ns * kPenStride * 8, hipMemcpyDeviceToDevice));
        CHECK(hipEventRecord(ev[2]));
        pt_defl6_kernel<<<ns, 64>>>(d_pen, false);
        CHECK(hipEventRecord(ev[3]));
        pt_eig6_kernel<<<ns, 64>>>(d_pen, d_c2, d_n2, kCandStride);
        CHECK(hipEventRecord(ev[4]));
        pt_eig6_lane_kernel<<<(ns + 63) / 64, 64>>>(d_pen, ns, d_c3, d_n3, kCandStride);
        CHECK(hipEventRecord(ev[5]));
        pt_defl6_kernel<<<ns, 64>>>(d_pen2, true); // (the Hessenberg form for the lockstep kernel)
        CHECK(hipEventRecord(ev[6]));
        pt_eig6_reg_kernel<false><<<(ns + 63) / 64, 64>>>(d_pen2, ns, 64, d_c4, d_n4, kCandStride, BatchGate{});
        CHECK(hipEventRecord(ev[7]));
        CHECK(hipEventSynchronize(ev[7]));
        if (timed)
            for (int k = 0; k < 7; ++k) CHECK(hipEventElapsedTime(&ms[k], ev[k], ev[k + 1]));
    };
    float ms[7] = {0, 0, 0, 0, 0, 0, 0}, acc[7] = {0, 0, 0, 0, 0, 0, 0};
    run(false, ms);
    unsigned long long z[8] = {0};
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(e6_prof), z, sizeof(z)));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) {
        run(true, ms);
        for (int k = 0; k < 7; ++k) acc[k] += ms[k] / reps;
    }
    unsigned long long prof[8];
    CHECK(hipMemcpyFromSymbol(prof, HIP_SYMBOL(e6_prof), sizeof(prof)));
    std::printf("samples %d: DFT group %.1f us | pencil %.1f us, deflation %.1f us, eigen (wave) %.1f us, eigen "
                "(lane) %.1f us, deflation + Hessenberg %.1f us, eigen (lockstep) %.1f us\n",
                ns, 1e3 * acc[0], 1e3 * acc[1], 1e3 * acc[2], 1e3 * acc[3], 1e3 * acc[4], 1e3 * acc[5], 1e3 * acc[6]);
    const double per = (double)ns * reps;
    std::printf("eigen kernels per sample (wave + lane kernels together): balance %.0f, elmhes %.0f, hqr %.0f ticks "
                "(100 MHz, lane 0 of each workgroup); %.2f balancing passes, %.2f QR iterations\n",
                prof[0] / per, prof[1] / per, prof[2] / per, prof[4] / per, prof[5] / per);
    {
        std::vector<int> n3(ns);
        std::vector<double> c3((size_t)ns * kCandStride);
        std::vector<int> n2b(ns);
        std::vector<double> c2b((size_t)ns * kCandStride);
        CHECK(hipMemcpy(n3.data(), d_n3, ns * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(c3.data(), d_c3, c3.size() * 8, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(n2b.data(), d_n2, ns * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(c2b.data(), d_c2, c2b.size() * 8, hipMemcpyDeviceToHost));
        long eq = 0;
        for (int s2 = 0; s2 < ns; ++s2) {
            bool same2 = n3[s2] == n2b[s2];
            for (int k = 0; same2 && k < n3[s2]; ++k)
                same2 = std::fabs(c3[(size_t)s2 * kCandStride + 27 + k] - c2b[(size_t)s2 * kCandStride + 27 + k]) <=
                        1e-9 * std::fabs(c2b[(size_t)s2 * kCandStride + 27 + k]);
            eq += same2;
        }
        std::printf("lane vs wave eigen kernels: %ld of %d root sets agree (1e-9)\n", eq, ns);
        std::vector<int> n4(ns);
        std::vector<double> c4((size_t)ns * kCandStride);
        CHECK(hipMemcpy(n4.data(), d_n4, ns * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(c4.data(), d_c4, c4.size() * 8, hipMemcpyDeviceToHost));
        long eq4 = 0, eq4c = 0;
        for (int s2 = 0; s2 < ns; ++s2) {
            bool same2 = n4[s2] == n2b[s2];
            eq4c += same2;
            for (int k = 0; same2 && k < n4[s2]; ++k)
                same2 = std::fabs(c4[(size_t)s2 * kCandStride + 27 + k] - c2b[(size_t)s2 * kCandStride + 27 + k]) <=
                        1e-9 * std::fabs(c2b[(size_t)s2 * kCandStride + 27 + k]);
            eq4 += same2;
            if (!same2 && (long)s2 - eq4 < 4) {
                std::printf("  sample %d: lockstep %d roots, wave %d:", s2, n4[s2], n2b[s2]);
                for (int k = 0; k < n4[s2]; ++k) std::printf(" %.12g", c4[(size_t)s2 * kCandStride + 27 + k]);
                std::printf(" |");
                for (int k = 0; k < n2b[s2]; ++k) std::printf(" %.12g", c2b[(size_t)s2 * kCandStride + 27 + k]);
                std::printf("\n");
            }
        }
        std::printf("lockstep vs wave eigen kernels: %ld of %d root sets agree (1e-9), counts agree %ld\n", eq4, ns,
                    eq4c);
    }
    {
        const double wg = (double)((ns + 63) / 64) * reps;
        std::printf("lockstep kernel per workgroup: hqr %.0f ticks, %.1f rounds\n", prof[6] / wg, prof[7] / wg);
    }
    {
        // the lockstep QR at other samples-per-wave packings: time and bit-equality
        // against 64 per wave (d_c4 / d_n4 from the last run above)
        std::vector<int> n64(ns), nx(ns);
        std::vector<double> c64((size_t)ns * kCandStride), cx((size_t)ns * kCandStride);
        CHECK(hipMemcpy(n64.data(), d_n4, ns * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(c64.data(), d_c4, c64.size() * 8, hipMemcpyDeviceToHost));
        {
            // the 16-lane group kernel: time and bit-equality against the lane kernel
            float t = 0.f, tt = 0.f;
            for (int r = 0; r < 4; ++r) {
                CHECK(hipEventRecord(ev[0]));
                pt_eig6_grp_kernel<<<(ns + 3) / 4, 64>>>(d_pen2, ns, d_c3, d_n3, kCandStride);
                CHECK(hipEventRecord(ev[1]));
                CHECK(hipEventSynchronize(ev[1]));
                CHECK(hipEventElapsedTime(&t, ev[0], ev[1]));
                if (r > 0) tt += t / 3;
            }
            CHECK(hipMemcpy(nx.data(), d_n3, ns * 4, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(cx.data(), d_c3, cx.size() * 8, hipMemcpyDeviceToHost));
            long same = 0, shown = 0;
            for (int s2 = 0; s2 < ns; ++s2) {
                bool eq = nx[s2] == n64[s2];
                for (int k = 0; eq && k < nx[s2]; ++k)
                    eq = cx[(size_t)s2 * kCandStride + 27 + k] == c64[(size_t)s2 * kCandStride + 27 + k];
                same += eq;
                if (!eq && shown++ < 3) {
                    std::printf("  sample %d: group %d roots, lane %d:", s2, nx[s2], n64[s2]);
                    for (int k = 0; k < nx[s2]; ++k) std::printf(" %.17g", cx[(size_t)s2 * kCandStride + 27 + k]);
                    std::printf(" |");
                    for (int k = 0; k < n64[s2]; ++k) std::printf(" %.17g", c64[(size_t)s2 * kCandStride + 27 + k]);
                    std::printf("\n");
                }
            }
            std::printf("group QR (4 samples per wave, %d waves): %.1f us, %ld of %d root sets bit-identical to the lane kernel\n",
                        (ns + 3) / 4, 1e3 * tt, same, ns);
        }
        for (int spw : {64, 16, 8, 2, 1}) {
            float t = 0.f, tt = 0.f;
            for (int r = 0; r < 4; ++r) {
                CHECK(hipEventRecord(ev[0]));
                if (spw == 1)
                    pt_eig6_reg_kernel<true><<<ns, 64>>>(d_pen2, ns, 1, d_c3, d_n3, kCandStride, BatchGate{});
                else
                    pt_eig6_reg_kernel<false><<<(ns + spw - 1) / spw, 64>>>(d_pen2, ns, spw, d_c3, d_n3, kCandStride, BatchGate{});
                CHECK(hipEventRecord(ev[1]));
                CHECK(hipEventSynchronize(ev[1]));
                CHECK(hipEventElapsedTime(&t, ev[0], ev[1]));
                if (r > 0) tt += t / 3;
            }
            CHECK(hipMemcpy(nx.data(), d_n3, ns * 4, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(cx.data(), d_c3, cx.size() * 8, hipMemcpyDeviceToHost));
            long same = 0;
            for (int s2 = 0; s2 < ns; ++s2) {
                bool eq = nx[s2] == n64[s2];
                for (int k = 0; eq && k < nx[s2]; ++k)
                    eq = cx[(size_t)s2 * kCandStride + 27 + k] == c64[(size_t)s2 * kCandStride + 27 + k];
                same += eq;
            }
            std::printf("lockstep QR, %2d samples per wave (%d waves): %.1f us, %ld of %d root sets bit-identical to 64\n",
                        spw, (ns + spw - 1) / spw, 1e3 * tt, same, ns);
        }
    }
    {
        // group deflation (+ balance + Hessenberg) against the one-wave kernel: time, and
        // the roots after the lane QR on either Hessenberg form (1e-9 relative)
        double *d_pen3;
        CHECK(hipMalloc(&d_pen3, (size_t)ns * kPenStride * 8));
        pt_pencil6_kernel<<<(ns + kGrpPerWg - 1) / kGrpPerWg, 64>>>(D, d_list, ns, d_samples, d_c2, kCandStride, d_pen);
        CHECK(hipMemcpy(d_pen2, d_pen, (size_t)ns * kPenStride * 8, hipMemcpyDeviceToDevice));
        CHECK(hipMemcpy(d_pen3, d_pen, (size_t)ns * kPenStride * 8, hipMemcpyDeviceToDevice));
        float tw = 0.f, tg = 0.f, t = 0.f;
        for (int r = 0; r < 4; ++r) {
            CHECK(hipMemcpy(d_pen2, d_pen, (size_t)ns * kPenStride * 8, hipMemcpyDeviceToDevice));
            CHECK(hipMemcpy(d_pen3, d_pen, (size_t)ns * kPenStride * 8, hipMemcpyDeviceToDevice));
            CHECK(hipEventRecord(ev[0]));
            pt_defl6_kernel<<<ns, 64>>>(d_pen2, true);
            CHECK(hipEventRecord(ev[1]));
            pt_defl6_grp_kernel<<<(ns + 3) / 4, 64>>>(d_pen3, ns, BatchGate{});
            CHECK(hipEventRecord(ev[2]));
            CHECK(hipEventSynchronize(ev[2]));
            CHECK(hipEventElapsedTime(&t, ev[0], ev[1]));
            if (r > 0) tw += t / 3;
            CHECK(hipEventElapsedTime(&t, ev[1], ev[2]));
            if (r > 0) tg += t / 3;
        }
        pt_eig6_reg_kernel<false><<<(ns + 63) / 64, 64>>>(d_pen2, ns, 64, d_c3, d_n3, kCandStride, BatchGate{});
        pt_eig6_reg_kernel<false><<<(ns + 63) / 64, 64>>>(d_pen3, ns, 64, d_c4, d_n4, kCandStride, BatchGate{});
        CHECK(hipDeviceSynchronize());
        std::vector<int> na(ns), nb(ns);
        std::vector<double> ca((size_t)ns * kCandStride), cb((size_t)ns * kCandStride);
        CHECK(hipMemcpy(na.data(), d_n3, ns * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(nb.data(), d_n4, ns * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(ca.data(), d_c3, ca.size() * 8, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(cb.data(), d_c4, cb.size() * 8, hipMemcpyDeviceToHost));
        long same = 0, shown = 0, ra = 0, rb = 0;
        for (int s2 = 0; s2 < ns; ++s2) {
            ra += na[s2];
            rb += nb[s2];
            bool eq = na[s2] == nb[s2];
            for (int k = 0; eq && k < na[s2]; ++k)
                eq = std::fabs(ca[(size_t)s2 * kCandStride + 27 + k] - cb[(size_t)s2 * kCandStride + 27 + k]) <=
                     1e-9 * std::fabs(ca[(size_t)s2 * kCandStride + 27 + k]);
            same += eq;
            if (!eq && shown++ < 3) {
                std::printf("  sample %d: wave deflation %d roots, group %d:", s2, na[s2], nb[s2]);
                for (int k = 0; k < na[s2]; ++k) std::printf(" %.12g", ca[(size_t)s2 * kCandStride + 27 + k]);
                std::printf(" |");
                for (int k = 0; k < nb[s2]; ++k) std::printf(" %.12g", cb[(size_t)s2 * kCandStride + 27 + k]);
                std::printf("\n");
            }
        }
        {
            unsigned long long gp[10] = {0}, z10[10] = {0};
            CHECK(hipMemcpyToSymbol(HIP_SYMBOL(e6g_prof), z10, sizeof(z10)));
            CHECK(hipMemcpy(d_pen3, d_pen, (size_t)ns * kPenStride * 8, hipMemcpyDeviceToDevice));
            pt_defl6_grp_kernel<<<(ns + 3) / 4, 64>>>(d_pen3, ns, BatchGate{});
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpyFromSymbol(gp, HIP_SYMBOL(e6g_prof), sizeof(gp)));
            const double waves = (ns + 3) / 4;
            std::printf("group deflation phases per wave (us at 100 MHz ticks): C %.1f, null spaces %.1f, S / c %.1f, "
                        "particular %.1f, similarity %.1f, block %.1f, balance %.1f, elmhes %.1f\n",
                        gp[0] / waves / 100, gp[1] / waves / 100, gp[2] / waves / 100, gp[3] / waves / 100,
                        gp[4] / waves / 100, gp[5] / waves / 100, gp[6] / waves / 100, gp[7] / waves / 100);
        }
        std::printf("deflation + Hessenberg: one wave per sample %.1f us, 16-lane groups %.1f us; roots after the "
                    "lane QR agree (1e-9) on %ld of %d samples (roots %ld / %ld)\n",
                    1e3 * tw, 1e3 * tg, same, ns, ra, rb);
    }
    std::vector<int> n1(ns), n2(ns);
    std::vector<double> c1((size_t)ns * kCandStride), c2((size_t)ns * kCandStride);
    CHECK(hipMemcpy(n1.data(), d_n1, ns * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(n2.data(), d_n2, ns * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(c1.data(), d_c1, c1.size() * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(c2.data(), d_c2, c2.size() * 8, hipMemcpyDeviceToHost));
    long same = 0, nr1 = 0, nr2 = 0;
    for (int s = 0; s < ns; ++s) {
        nr1 += n1[s];
        nr2 += n2[s];
        bool eq = n1[s] == n2[s];
        for (int k = 0; eq && k < n1[s]; ++k) {
            const double a = c1[(size_t)s * kCandStride + 27 + k], b = c2[(size_t)s * kCandStride + 27 + k];
            eq = std::fabs(a - b) <= 1e-6 * std::fabs(b);
        }
        same += eq;
    }
    std::printf("root sets agreeing (1e-6): %ld of %d; roots DFT %ld, eigen %ld\n", same, ns, nr1, nr2);
    return 0;
}
