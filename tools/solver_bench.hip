// Microbenchmark of the minimal-solver device code, stage by stage (one sample per
// lane, as in the engine's md_solve / pt_solve kernels).  Build + run:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I madpose_amd/csrc/include -I include \
//         tools/solver_bench.hip -o tools/solver_bench && tools/solver_bench [samples]
// Prints ms per launch for each stage kernel; differences between stages give the
// cost of each stage.  Inputs are random two-view samples (half with outliers).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "mp_md.h"
#include "mp_pt67.h"

using namespace mp;

#define CHECK(x)                                                                                                      \
    do {                                                                                                               \
        hipError_t e = (x);                                                                                            \
        if (e != hipSuccess) {                                                                                         \
            std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);                \
            std::exit(1);                                                                                              \
        }                                                                                                              \
    } while (0)

// in: per sample 7 points x (x0u x0v x1u x1v d0 d1) = 42 doubles
constexpr int kStride = 42;

template <int K> __device__ void load(const double *in, int s, double (&b0)[K][3], double (&b1)[K][3],
                                      double (&p0)[K][2], double (&p1)[K][2], double (&d0)[K], double (&d1)[K]) {
    const double *q = in + (size_t)s * kStride;
    for (int j = 0; j < K; ++j) {
        const double a[3] = {q[6 * j], q[6 * j + 1], 1.0}, c[3] = {q[6 * j + 2], q[6 * j + 3], 1.0};
        const double na = 1.0 / sqrt(dot3(a, a)), nc = 1.0 / sqrt(dot3(c, c));
        for (int r = 0; r < 3; ++r) {
            b0[j][r] = a[r] * na;
            b1[j][r] = c[r] * nc;
        }
        p0[j][0] = a[0];
        p0[j][1] = a[1];
        p1[j][0] = c[0];
        p1[j][1] = c[1];
        d0[j] = q[6 * j + 4];
        d1[j] = q[6 * j + 5];
    }
}


// stage-by-stage copy of sturm_real_roots (mp_math.h) for timing
template <int N, int STOP> __device__ double sturm_dbg(const double *c_in) {
    double c[N + 1], cs[N + 1];
    const double lead = 1.0 / c_in[N];
    for (int j = 0; j <= N; ++j) c[j] = c_in[j] * lead;
    double sigma = 0.0;
    for (int j = 0; j < N; ++j)
        if (c[j] != 0.0) sigma = fmax(sigma, pow(fabs(c[j]), 1.0 / (N - j)));
    if (!(sigma > 0.0) || !(sigma < 1e300)) sigma = 1.0;
    {
        const double inv = 1.0 / sigma;
        double p = 1.0;
        cs[N] = 1.0;
        for (int j = N - 1; j >= 0; --j) {
            p *= inv;
            cs[j] = c[j] * p;
        }
    }
    if (STOP == 1) return cs[0] + sigma;
    SturmChain<N> S;
    sturm_build<N>(cs, S);
    if (STOP == 2) return S.s[S.len - 1][0];
    const double B = 3.0;
    constexpr int kCells = 32;
    const double h = 2.0 * B / kCells;
    const int c_end = sturm_count<N>(S, B);
    double x_lo = -B;
    int v_lo = sturm_count<N>(S, -B);
    double acc = 0;
    for (int i = 0; i < kCells && v_lo > c_end; ++i) {
        const double x_hi = (i + 1 == kCells) ? B : -B + (i + 1) * h;
        const int v_hi = (i + 1 == kCells) ? c_end : sturm_count<N>(S, x_hi);
        const int d = v_lo - v_hi;
        if (STOP == 3) acc += d;
        else if (d >= 1) acc += refine_root<N>(c, sigma * x_lo, sigma * x_hi);
        x_lo = x_hi;
        v_lo = v_hi;
    }
    return acc;
}

template <int STOP> __global__ void __launch_bounds__(64) ksturm(const double *in, int n, double *out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    double b0[5][3], b1[5][3], p0[5][2], p1[5][2], d0[5], d1[5];
    load<5>(in, s, b0, b1, p0, p1, d0, d1);
    FivePtSys S;
    if (!fivept_system(b0, b1, S)) {
        out[s] = -1;
        return;
    }
    out[s] = sturm_dbg<10, STOP>(S.d10);
}

template <int STOP> __global__ void __launch_bounds__(64) k5(const double *in, int n, double *out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    double b0[5][3], b1[5][3], p0[5][2], p1[5][2], d0[5], d1[5];
    load<5>(in, s, b0, b1, p0, p1, d0, d1);
    FivePtSys S;
    if (!fivept_system(b0, b1, S)) {
        out[s] = -1;
        return;
    }
    if (STOP == 1) {
        out[s] = S.d10[0] + S.d10[10];
        return;
    }
    double roots[10];
    const int nr = sturm_real_roots<10>(S.d10, roots);
    if (STOP == 2) {
        double acc = nr;
        for (int r = 0; r < nr; ++r) acc += roots[r];
        out[s] = acc;
        return;
    }
    Model poses[10];
    int np = 0;
    for (int r = 0; r < nr; ++r) np += fivept_poses_for_root(S, roots[r], b0, b1, poses, np, 10);
    if (STOP == 3) {
        out[s] = np + (np ? poses[0].t[0] : 0.0);
        return;
    }
    const double md[2] = {0.0, 0.0};
    int nm = 0;
    for (int k = 0; k < np; ++k) {
        Model m = poses[k];
        if (point_model_tail<5>(p0, p1, d0, d1, 1.0, 1.0, true, true, md, m)) ++nm;
    }
    out[s] = nm;
}

template <int STOP> __global__ void __launch_bounds__(64) k6(const double *in, int n, double *out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    double b0[6][3], b1[6][3], p0[6][2], p1[6][2], d0[6], d1[6];
    load<6>(in, s, b0, b1, p0, p1, d0, d1);
    Model poses[16];
    out[s] = relpose_6pt_sf<STOP>(b0, b1, poses, 16);
}

__global__ void __launch_bounds__(64) k7(const double *in, int n, double *out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    double b0[7][3], b1[7][3], p0[7][2], p1[7][2], d0[7], d1[7];
    load<7>(in, s, b0, b1, p0, p1, d0, d1);
    double F[3][9];
    const int nf = relpose_7pt_F(b0, b1, F);
    double acc = nf;
    for (int k = 0; k < nf; ++k) {
        double f0, f1;
        bougnoux_sq(F[k], &f0, &f1);
        f0 = sqrt(fabs(f0));
        f1 = sqrt(fabs(f1));
        double E[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) E[3 * r + c] = (r < 2 ? f1 : 1.0) * F[k][3 * r + c] * (c < 2 ? f0 : 1.0);
        double R[9], t[3];
        acc += recover_pose_cv<7>(E, p0, p1, 1e9, R, t) + R[0];
    }
    out[s] = acc;
}

template <int V> __global__ void __launch_bounds__(64) kmd(const double *in, int n, double *out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const double *q = in + (size_t)s * kStride;
    int cnt = 0;
    if (V == kCal) {
        double x[3][3], y[3][3], dx[3], dy[3];
        for (int j = 0; j < 3; ++j) {
            x[j][0] = q[6 * j];
            x[j][1] = q[6 * j + 1];
            x[j][2] = 1.0;
            y[j][0] = q[6 * j + 2];
            y[j][1] = q[6 * j + 3];
            y[j][2] = 1.0;
            dx[j] = q[6 * j + 4];
            dy[j] = q[6 * j + 5];
        }
        double sols[4][6];
        const int ns = md_sols_cal(x, y, dx, dy, sols);
        for (int k = 0; k < ns; ++k) {
            Model m;
            m.focal0 = m.focal1 = 1.0;
            cnt += md_pose_from_sol<3>(x, y, dx, dy, sols[k], 1.0, 1.0, m);
        }
    } else {
        double x[4][3], y[4][3], dx[4], dy[4];
        for (int j = 0; j < 4; ++j) {
            x[j][0] = q[6 * j];
            x[j][1] = q[6 * j + 1];
            x[j][2] = 1.0;
            y[j][0] = q[6 * j + 2];
            y[j][1] = q[6 * j + 3];
            y[j][2] = 1.0;
            dx[j] = q[6 * j + 4];
            dy[j] = q[6 * j + 5];
        }
        double sols[8][6];
        const int ns = (V == kSF) ? md_sols_sf(x, y, dx, dy, sols)
                                  : md_sols_tf(x, y, dx, dy, *reinterpret_cast<double(*)[4][6]>(&sols[0][0]));
        for (int k = 0; k < ns; ++k) {
            Model m;
            const double fa = sols[k][4], fb = (V == kSF) ? sols[k][4] : sols[k][5];
            m.focal0 = fa;
            m.focal1 = fb;
            cnt += md_pose_from_sol<4>(x, y, dx, dy, sols[k], fa, fb, m);
        }
    }
    out[s] = cnt;
}

template <class K> float time_kernel(K kern, const double *d_in, int n, double *d_out, hipStream_t st) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const int grid = (n + 63) / 64;
    kern<<<grid, 64, 0, st>>>(d_in, n, d_out); // warm
    CHECK(hipStreamSynchronize(st));
    CHECK(hipEventRecord(a, st));
    const int reps = 3;
    for (int r = 0; r < reps; ++r) kern<<<grid, 64, 0, st>>>(d_in, n, d_out);
    CHECK(hipEventRecord(b, st));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 32768;
    std::mt19937 g(1);
    std::normal_distribution<double> nd;
    std::uniform_real_distribution<double> ud(-1.0, 1.0);
    std::vector<double> h((size_t)n * kStride);
    for (int s = 0; s < n; ++s) {
        // random rotation (small), translation, focal; points in front of both cameras
        const double ax = 0.2 * ud(g), ay = 0.2 * ud(g), az = 0.2 * ud(g);
        const double f = 1.0 + 0.5 * ud(g);
        const double t[3] = {0.3 * ud(g) + 0.5, 0.2 * ud(g), 0.1 * ud(g)};
        for (int j = 0; j < 7; ++j) {
            const double X[3] = {ud(g), ud(g), 4.0 + 2.0 * ud(g)};
            const double Y[3] = {X[0] - az * X[1] + ay * X[2] + t[0], az * X[0] + X[1] - ax * X[2] + t[1],
                                 -ay * X[0] + ax * X[1] + X[2] + t[2]};
            double *q = &h[(size_t)s * kStride + 6 * j];
            q[0] = f * X[0] / X[2] + 1e-3 * nd(g);
            q[1] = f * X[1] / X[2] + 1e-3 * nd(g);
            q[2] = f * Y[0] / Y[2];
            q[3] = f * Y[1] / Y[2];
            if ((s & 1) && j < 2) {
                q[2] = ud(g);
                q[3] = ud(g);
            }
            q[4] = X[2] * (1.0 + 0.05 * nd(g));
            q[5] = Y[2] * (1.0 + 0.05 * nd(g));
        }
    }
    double *d_in, *d_out;
    CHECK(hipMalloc(&d_in, h.size() * sizeof(double)));
    CHECK(hipMalloc(&d_out, (size_t)n * sizeof(double)));
    CHECK(hipMemcpy(d_in, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    std::printf("samples per launch: %d\n", n);
    std::printf("5pt system            %8.3f ms\n", time_kernel(k5<1>, d_in, n, d_out, st));
    std::printf("5pt + sturm roots     %8.3f ms\n", time_kernel(k5<2>, d_in, n, d_out, st));
    std::printf("  sturm: sigma        %8.3f ms\n", time_kernel(ksturm<1>, d_in, n, d_out, st));
    std::printf("  sturm: + build      %8.3f ms\n", time_kernel(ksturm<2>, d_in, n, d_out, st));
    std::printf("  sturm: + grid count %8.3f ms\n", time_kernel(ksturm<3>, d_in, n, d_out, st));
    std::printf("  sturm: + refine     %8.3f ms\n", time_kernel(ksturm<4>, d_in, n, d_out, st));
    std::printf("5pt + poses           %8.3f ms\n", time_kernel(k5<3>, d_in, n, d_out, st));
    std::printf("5pt + depth tail      %8.3f ms\n", time_kernel(k5<4>, d_in, n, d_out, st));
    std::printf("6pt system            %8.3f ms\n", time_kernel(k6<0>, d_in, n, d_out, st));
    std::printf("6pt + pencil det DFT  %8.3f ms\n", time_kernel(k6<1>, d_in, n, d_out, st));
    std::printf("6pt + sturm           %8.3f ms\n", time_kernel(k6<2>, d_in, n, d_out, st));
    std::printf("6pt + polish          %8.3f ms\n", time_kernel(k6<3>, d_in, n, d_out, st));
    std::printf("6pt shared focal      %8.3f ms\n", time_kernel(k6<4>, d_in, n, d_out, st));
    std::printf("7pt + bougnoux + cv   %8.3f ms\n", time_kernel(k7, d_in, n, d_out, st));
    std::printf("MD cal                %8.3f ms\n", time_kernel(kmd<kCal>, d_in, n, d_out, st));
    std::printf("MD sf                 %8.3f ms\n", time_kernel(kmd<kSF>, d_in, n, d_out, st));
    std::printf("MD tf                 %8.3f ms\n", time_kernel(kmd<kTF>, d_in, n, d_out, st));
    CHECK(hipFree(d_in));
    CHECK(hipFree(d_out));
    return 0;
}
