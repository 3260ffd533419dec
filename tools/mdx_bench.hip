// Microbenchmark of the exact calibrated MD solver (mp_md_exact.h), stage by stage, in
// the estimator kernel's layout (R lanes per sample, lane r takes roots r, r + R, ...):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I madpose_amd/csrc/include -I include \
//         tools/mdx_bench.hip -o tools/mdx_bench && tools/mdx_bench [samples]
// Stages: 0 = setup (system + sorted roots), 1 = + root() (polish + filters),
// 2 = + md_pose_exact (Procrustes).  Prints us per launch; differences give the cost
// of each stage.  Inputs: random calibrated rays and depths.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

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
    MdxCal sys;
    double roots[4];
    const int nr = sys.setup(x, y, dx, dy, roots);
    double acc = nr;
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
    std::vector<double> h((size_t)n * kStride);
    for (int s = 0; s < n; ++s) {
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
    CHECK(hipMalloc(&d_out, (size_t)n * sizeof(double)));
    CHECK(hipMemcpy(d_in, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    std::printf("samples %d\n", n);
    std::printf("R=4: setup %.1f  +root %.1f  +pose %.1f us\n", time_kern<4, 0>(d_in, n, d_out),
                time_kern<4, 1>(d_in, n, d_out), time_kern<4, 2>(d_in, n, d_out));
    std::printf("R=2: setup %.1f  +root %.1f  +pose %.1f us\n", time_kern<2, 0>(d_in, n, d_out),
                time_kern<2, 1>(d_in, n, d_out), time_kern<2, 2>(d_in, n, d_out));
    std::printf("R=1: setup %.1f  +root %.1f  +pose %.1f us\n", time_kern<1, 0>(d_in, n, d_out),
                time_kern<1, 1>(d_in, n, d_out), time_kern<1, 2>(d_in, n, d_out));
    return 0;
}
