// Microbenchmark of the exact calibrated MD solver (mp_md_exact.h), stage by stage, in
// the estimator kernel's layout (R lanes per sample, lane r takes roots r, r + R, ...):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I madpose_amd/csrc/include -I include \
//         tools/mdx_bench.hip -o tools/mdx_bench && tools/mdx_bench [samples]
// Stages: -1 = the system up to the quartic (pair terms, QR solve, products), 0 = setup
// (+ the quartic's sorted real roots: companion, balance, hqr), 1 = + root() (polish +
// filters), 2 = + md_pose_exact (Procrustes).  Prints us per launch; differences give
// the cost of each stage; then the setup at several sample counts (a latency-bound
// kernel costs the same at all of them).  Inputs: random calibrated rays and depths.
// Built with -DMDX_COUNT (binary tools/mdx_count): per sample, the balance passes, the
// hqr trips and the setup's shader cycles, and their distribution over samples and
// over waves (a latency-bound launch lasts as long as its slowest wave).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#ifdef MDX_COUNT
constexpr int kMaxCount = 1 << 16;
__device__ int g_bal[kMaxCount], g_trips[kMaxCount];
#define MDX_BAL_HOOK() (g_bal[blockIdx.x * blockDim.x + threadIdx.x] += 1)
#define MDX_TRIP_HOOK() (g_trips[blockIdx.x * blockDim.x + threadIdx.x] += 1)
#endif
#include "mp_md_exact.h"

using namespace mp;

#define CHECK(x)                                                                                                      \
    do {                                                                                                               \
        hipError_t e = (x);                                                                                            \
        if (e != hipSuccess) {                                                                                         \
            std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);                \
            std::exit(1);                                                                                              \
        }                                                                                                              \
    } while (0)

constexpr int kStride = 24; // 3 x (x 3, y 3) + dx 3 + dy 3

template <int R, int STAGE> __global__ void __launch_bounds__(64) kern(const double *in, int n, double *out) {
    const int g = threadIdx.x / R, r = threadIdx.x % R;
    const int idx = blockIdx.x * (64 / R) + g;
    if (idx >= n) return;
    const double *q = in + (size_t)idx * kStride;
    double x[3][3], y[3][3], dx[3], dy[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            x[j][c] = q[3 * j + c];
            y[j][c] = q[9 + 3 * j + c];
        }
        dx[j] = q[18 + j];
        dy[j] = q[21 + j];
    }
    if (STAGE < 0) { // the setup up to the quartic's coefficients (MdxCal::setup's first half)
        double x4[4][3], y4[4][3];
        for (int i = 0; i < 4; ++i)
            for (int c = 0; c < 3; ++c) {
                x4[i][c] = i < 3 ? x[i][c] : 0.0;
                y4[i][c] = i < 3 ? y[i][c] : 0.0;
            }
        const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
        PairTerms T[3];
        for (int k = 0; k < 3; ++k) T[k] = mdx::pair_terms<false>(x4, y4, dx, dy, pr[k][0], pr[k][1]);
        double Q[3][3], Pm[3][3], L[3][3];
        for (int k = 0; k < 3; ++k)
            for (int c = 0; c < 3; ++c) {
                Q[k][c] = T[k].B[c];
                Pm[k][c] = T[k].A[c];
            }
        double acc = mdx::qr_solve<3, 3>(Q, Pm, L) ? 1.0 : 0.0;
        const double l0[3] = {L[0][2], L[0][1], L[0][0]}, l1[3] = {L[1][2], L[1][1], L[1][0]},
                     l2[3] = {L[2][2], L[2][1], L[2][0]};
        double a[5], b[5], quart[5];
        mdx::pmul(l1, l1, a);
        mdx::pmul(l0, l2, b);
        mdx::psub(a, b, quart);
        for (int k = 0; k < 5; ++k) acc += quart[k];
        if (r == 0) out[idx] = acc;
        return;
    }
    MdxCal sys;
    double roots[4];
#ifdef MDX_COUNT
    const long long c0 = clock64();
#endif
    const int nr = sys.setup(x, y, dx, dy, roots);
    double acc = nr;
#ifdef MDX_COUNT
    acc += roots[0] + roots[1] + roots[2] + roots[3];
    const long long c1 = clock64() + (acc == 12345.0 ? 1 : 0);
    if (r == 0) out[idx] = (double)(c1 - c0);
    return;
#endif
    if (STAGE >= 1) {
#pragma unroll
        for (int j = 0; j < 4 / R; ++j) {
            const int k = j * R + r;
            double root = 0.0;
#pragma unroll
            for (int c = 0; c < R; ++c)
                if (c == r) root = opaque(roots[j * R + c]);
            if (k < nr) {
                double sol[6];
                if (sys.root(root, sol)) {
                    acc += sol[1];
                    if (STAGE >= 2) {
                        Model m;
                        if (md_pose_exact<3>(x, y, dx, dy, sol, 1.0, 1.0, m)) acc += m.R[0] + m.t[0];
                    }
                }
            }
        }
    } else {
        acc += roots[0] + roots[1] + roots[2] + roots[3];
    }
    if (r == 0) out[idx] = acc;
}

template <int R, int STAGE> float time_kern(const double *d_in, int n, double *d_out) {
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    const int grid = (n + 64 / R - 1) / (64 / R);
    kern<R, STAGE><<<grid, 64, 0, st>>>(d_in, n, d_out);
    CHECK(hipStreamSynchronize(st));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int reps = 20;
    CHECK(hipEventRecord(a, st));
    for (int k = 0; k < reps; ++k) kern<R, STAGE><<<grid, 64, 0, st>>>(d_in, n, d_out);
    CHECK(hipEventRecord(b, st));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipStreamDestroy(st));
    return 1000.f * ms / reps;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
    std::mt19937 gen(7);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::uniform_real_distribution<double> ud(0.5, 5.0);
    const int nmax = std::max(n, 32768);
    std::vector<double> h((size_t)nmax * kStride);
    for (int s = 0; s < nmax; ++s) {
        double *q = &h[(size_t)s * kStride];
        for (int j = 0; j < 3; ++j) {
            q[3 * j] = 0.4 * nd(gen);
            q[3 * j + 1] = 0.4 * nd(gen);
            q[3 * j + 2] = 1.0;
            q[9 + 3 * j] = q[3 * j] + 0.05 * nd(gen);
            q[9 + 3 * j + 1] = q[3 * j + 1] + 0.05 * nd(gen);
            q[9 + 3 * j + 2] = 1.0;
            q[18 + j] = ud(gen);
            q[21 + j] = ud(gen);
        }
    }
    double *d_in, *d_out;
    CHECK(hipMalloc(&d_in, h.size() * sizeof(double)));
    CHECK(hipMalloc(&d_out, (size_t)nmax * sizeof(double)));
    CHECK(hipMemcpy(d_in, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    std::printf("samples %d\n", n);
#ifdef MDX_COUNT
    {
        const int m = std::min(n, kMaxCount);
        std::vector<int> z(kMaxCount, 0);
        CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_bal), z.data(), sizeof(int) * kMaxCount));
        CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_trips), z.data(), sizeof(int) * kMaxCount));
        kern<1, 0><<<(m + 63) / 64, 64>>>(d_in, m, d_out);
        CHECK(hipDeviceSynchronize());
        std::vector<int> bal(m), trips(m);
        std::vector<double> cyc(m);
        CHECK(hipMemcpyFromSymbol(bal.data(), HIP_SYMBOL(g_bal), sizeof(int) * m));
        CHECK(hipMemcpyFromSymbol(trips.data(), HIP_SYMBOL(g_trips), sizeof(int) * m));
        CHECK(hipMemcpy(cyc.data(), d_out, sizeof(double) * m, hipMemcpyDeviceToHost));
        auto report = [&](const char *what, std::vector<double> v) {
            std::vector<double> wmax;
            for (int w = 0; w < m; w += 16) wmax.push_back(*std::max_element(v.begin() + w, v.begin() + std::min(m, w + 16)));
            std::sort(v.begin(), v.end());
            std::sort(wmax.begin(), wmax.end());
            double mean = 0;
            for (double x : v) mean += x;
            mean /= v.size();
            auto q = [](const std::vector<double> &u, double f) { return u[(size_t)std::min<double>(u.size() - 1, f * u.size())]; };
            std::printf("%s: mean %.1f p50 %.0f p90 %.0f p99 %.0f max %.0f | max of 16: p50 %.0f p90 %.0f max %.0f\n", what,
                        mean, q(v, 0.5), q(v, 0.9), q(v, 0.99), v.back(), q(wmax, 0.5), q(wmax, 0.9), wmax.back());
        };
        report("balance passes", std::vector<double>(bal.begin(), bal.end()));
        report("hqr trips", std::vector<double>(trips.begin(), trips.end()));
        report("setup cycles", cyc);
        // cycles against trips: mean cycles per trip count
        std::vector<double> sum(64, 0.0);
        std::vector<int> cnt(64, 0);
        for (int i = 0; i < m; ++i) {
            const int t = std::min(trips[i], 63);
            sum[t] += cyc[i];
            ++cnt[t];
        }
        for (int t = 0; t < 64; ++t)
            if (cnt[t]) std::printf("  trips %2d: %6d samples, %.0f cycles\n", t, cnt[t], sum[t] / cnt[t]);
    }
#else
    std::printf("R=4: quartic %.1f  setup %.1f  +root %.1f  +pose %.1f us\n", time_kern<4, -1>(d_in, n, d_out),
                time_kern<4, 0>(d_in, n, d_out), time_kern<4, 1>(d_in, n, d_out), time_kern<4, 2>(d_in, n, d_out));
    std::printf("R=2: quartic %.1f  setup %.1f  +root %.1f  +pose %.1f us\n", time_kern<2, -1>(d_in, n, d_out),
                time_kern<2, 0>(d_in, n, d_out), time_kern<2, 1>(d_in, n, d_out), time_kern<2, 2>(d_in, n, d_out));
    std::printf("R=1: quartic %.1f  setup %.1f  +root %.1f  +pose %.1f us\n", time_kern<1, -1>(d_in, n, d_out),
                time_kern<1, 0>(d_in, n, d_out), time_kern<1, 1>(d_in, n, d_out), time_kern<1, 2>(d_in, n, d_out));
    for (int m : {256, 1024, 4096, 16384, 32768})
        std::printf("R=4 setup at %5d samples: %.1f us\n", m, time_kern<4, 0>(d_in, m, d_out));
#endif
    return 0;
}
