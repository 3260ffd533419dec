// Round-trip latency of the LO sweep (launch -> host sees the completion flag) for a
// few ways of returning its results, on a synthetic calibrated pair of n points:
//   host   the earlier protocol: errors to pinned host memory, the last workgroup to
//          arrive (system-scope counter) sums the partials and raises one flag
//   dev    the same with the error rows in device memory (flag still host)
//   flags  sweep_host_kernel as shipped: one flag per workgroup, host sums
//   flag   a one-workgroup kernel that only raises the flag (the floor)
//   ldonly / stonly / nold_nost   the shipped flag protocol with only the pair loads,
//          only the error-row stores, neither (8 workgroups); nlns_wg1 the last on one
//          workgroup; ls_1024 loads + stores on 1024-lane workgroups
//   noeval / nofence / neither   the shipped protocol without the residuals, without
//          the per-workgroup system fence, without both
// Build + run (on an MI355X):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/sweep_lat.hip -o tools/sweep_lat
//   tools/sweep_lat [n] [reps]
#include "../madpose_amd/csrc/kernels/kernels.hip"

#include <chrono>
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

namespace {
__global__ void flag_only_kernel(int *flag, int seq) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
// one workgroup for the whole sweep: no cross-workgroup counter, one fence per lane
template <int V, int NT>
__global__ void __launch_bounds__(NT) sweep1_kernel(PairData D, PairConst C, ScoreRec r, double *out, int *flag,
                                                    int seq) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < C.n; i += NT) {
        const Corr p = load_corr(C, D, i, V == kCal);
        double e0, e1, e2;
        eval_corr<V>(C, r, p, false, e0, e1, e2);
        out[i] = e0;
        out[C.n + i] = e1;
        out[2 * C.n + i] = e2;
        acc += msac(e0, C.thr[0], C.w[0]) + msac(e1, C.thr[1], C.w[1]) + msac(e2, C.thr[2], C.w[2]);
    }
    __shared__ double wpart[NT / 64];
    const double v = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = v;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        double sc = 0.0;
        for (int w = 0; w < NT / 64; ++w) sc += wpart[w];
        out[3 * C.n] = sc;
        __threadfence_system();
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
// variants of sweep_host_kernel: EVAL = false replaces the residuals by the loaded
// coordinates (isolates the cross-workgroup completion protocol), FENCE = false drops
// each workgroup's system-scope fence before its arrival
template <int V, bool EVAL, bool FENCE>
__global__ void __launch_bounds__(256) sweep_var_kernel(PairData D, PairConst C, ScoreRec r, double *out, int *flag,
                                                        int seq, double *part, unsigned *cnt) {
    double acc = 0.0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < C.n; i += gridDim.x * 256) {
        const Corr p = load_corr(C, D, i, V == kCal);
        double e0 = p.x0u, e1 = p.x1u, e2 = p.d0;
        if (EVAL) eval_corr<V>(C, r, p, false, e0, e1, e2);
        out[i] = e0;
        out[C.n + i] = e1;
        out[2 * C.n + i] = e2;
        acc += msac(e0, C.thr[0], C.w[0]) + msac(e1, C.thr[1], C.w[1]) + msac(e2, C.thr[2], C.w[2]);
    }
    __shared__ double wpart[4];
    __shared__ bool last;
    const double v = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = v;
    if (FENCE) __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        double sc = 0.0;
        for (int w = 0; w < 4; ++w) sc += wpart[w];
        part[blockIdx.x] = sc;
        const unsigned arrived = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
        last = arrived == gridDim.x - 1;
        if (last) {
            double tot = 0.0;
            for (unsigned b = 0; b < gridDim.x; ++b)
                tot += __hip_atomic_load(part + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            out[3 * C.n] = tot;
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}
// isolating loads and stores: LOAD = false uses the index instead of the pair data,
// STORE = false skips the error rows (the partial score and flag protocol stay)
template <bool LOAD, bool STORE, int NT, bool FENCE = true>
__global__ void __launch_bounds__(NT) sweep_ls_kernel(PairData D, PairConst C, double *out, int *flags, int seq) {
    double acc = 0.0;
    for (int i = blockIdx.x * NT + threadIdx.x; i < C.n; i += gridDim.x * NT) {
        const double e0 = LOAD ? D.x0u[i] + D.x0v[i] + D.x1u[i] : (double)i;
        const double e1 = LOAD ? D.x1v[i] + D.d0[i] + D.d1[i] : 1.0;
        const double e2 = LOAD ? D.r0[i] + D.r1[i] : 2.0;
        if (STORE) {
            out[i] = e0;
            out[C.n + i] = e1;
            out[2 * C.n + i] = e2;
        }
        acc += e0 + e1 + e2;
    }
    const double v = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) out[3 * C.n + (NT / 64) * blockIdx.x + (threadIdx.x >> 6)] = v;
    if (FENCE) __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
} // namespace

using Clock = std::chrono::steady_clock;

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 2000;
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> U(-1, 1);
    std::vector<double> x0u(n), x0v(n), x1u(n), x1v(n), d0(n), d1(n), r0(n), r1(n);
    for (int i = 0; i < n; ++i) {
        x0u[i] = 320 + 200 * U(rng);
        x0v[i] = 240 + 200 * U(rng);
        x1u[i] = 320 + 200 * U(rng);
        x1v[i] = 240 + 200 * U(rng);
        d0[i] = 3 + U(rng);
        d1[i] = 3 + U(rng);
        r0[i] = r1[i] = 0.9;
    }
    auto up = [&](const std::vector<double> &v) {
        double *p;
        CHECK(hipMalloc(&p, v.size() * 8));
        CHECK(hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice));
        return (const double *)p;
    };
    PairData D{up(x0u), up(x0v), up(x1u), up(x1v), up(d0), up(d1), up(r0), up(r1)};
    PairConst C{};
    C.variant = kCal;
    C.n = n;
    const double K[9] = {500, 0, 320, 0, 500, 240, 0, 0, 1}, Ki[9] = {1 / 500., 0, -320 / 500., 0, 1 / 500., -240 / 500., 0, 0, 1};
    for (int k = 0; k < 9; ++k) {
        C.K0[k] = C.K1[k] = K[k];
        C.K0i[k] = C.K1i[k] = Ki[k];
    }
    for (int t = 0; t < 3; ++t) {
        C.thr[t] = 4.0;
        C.w[t] = 1.0;
    }
    Model m{};
    m.R[0] = m.R[4] = m.R[8] = 1.0;
    m.t[0] = 0.3;
    m.scale = 1.0;
    m.focal0 = m.focal1 = 1.0;
    ScoreRec rec;
    prepare_score_rec(C, m, rec);

    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    double *h_out, *d_out_h, *d_out_dev, *part;
    int *h_flag, *d_flag;
    unsigned *cnt;
    CHECK(hipHostMalloc(&h_out, sizeof(double) * (3 * n + 1), hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipHostMalloc(&h_flag, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer((void **)&d_out_h, h_out, 0));
    CHECK(hipHostGetDevicePointer((void **)&d_flag, h_flag, 0));
    CHECK(hipMalloc(&d_out_dev, sizeof(double) * (3 * n + 1)));
    double *h_out8, *d_out8;
    int *h_flags, *d_flags;
    const int nbk = sweep_blocks(n);
    CHECK(hipHostMalloc(&h_out8, sizeof(double) * (3 * n + 64), hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipHostMalloc(&h_flags, sizeof(int) * 64, hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer((void **)&d_out8, h_out8, 0));
    CHECK(hipHostGetDevicePointer((void **)&d_flags, h_flags, 0));
    for (int b = 0; b < 64; ++b) h_flags[b] = 0;
    CHECK(hipMalloc(&part, sizeof(double) * sweep_blocks(n)));
    CHECK(hipMalloc(&cnt, sizeof(unsigned)));
    CHECK(hipMemset(cnt, 0, sizeof(unsigned)));
    *h_flag = 0;
    int seq = 0;

    auto run = [&](const char *name, int mode) {
        double t_launch = 0, t_wait = 0;
        for (int r = 0; r < reps + 50; ++r) {
            const int q = ++seq;
            auto t0 = Clock::now();
            if (mode == 0)
                sweep_var_kernel<kCal, true, true><<<nbk, 256, 0, s>>>(D, C, rec, d_out_h, d_flag, q, part, cnt);
            else if (mode == 1)
                sweep_var_kernel<kCal, true, true><<<nbk, 256, 0, s>>>(D, C, rec, d_out_dev, d_flag, q, part, cnt);
            else if (mode == 2)
                flag_only_kernel<<<1, 64, 0, s>>>(d_flag, q);
            else if (mode == 8)
                CHECK(launch_sweep_host(s, D, C, rec, d_out8, d_flags, q));
            else if (mode == 5)
                sweep_var_kernel<kCal, false, true><<<sweep_blocks(n), 256, 0, s>>>(D, C, rec, d_out_h, d_flag, q, part, cnt);
            else if (mode == 6)
                sweep_var_kernel<kCal, true, false><<<sweep_blocks(n), 256, 0, s>>>(D, C, rec, d_out_h, d_flag, q, part, cnt);
            else if (mode == 7)
                sweep_var_kernel<kCal, false, false><<<sweep_blocks(n), 256, 0, s>>>(D, C, rec, d_out_h, d_flag, q, part, cnt);
            else if (mode == 9)
                sweep_ls_kernel<true, false, 256><<<nbk, 256, 0, s>>>(D, C, d_out8, d_flags, q);
            else if (mode == 10)
                sweep_ls_kernel<false, true, 256><<<nbk, 256, 0, s>>>(D, C, d_out8, d_flags, q);
            else if (mode == 11)
                sweep_ls_kernel<false, false, 256><<<nbk, 256, 0, s>>>(D, C, d_out8, d_flags, q);
            else if (mode == 12)
                sweep_ls_kernel<false, false, 256><<<1, 256, 0, s>>>(D, C, d_out8, d_flags, q);
            else if (mode == 13)
                sweep_ls_kernel<true, true, 1024><<<(n + 1023) / 1024, 1024, 0, s>>>(D, C, d_out8, d_flags, q);
            else if (mode == 14)
                sweep_ls_kernel<false, false, 256, false><<<nbk, 256, 0, s>>>(D, C, d_out8, d_flags, q);
            else if (mode == 15)
                sweep_ls_kernel<false, false, 64, true><<<nbk, 64, 0, s>>>(D, C, d_out8, d_flags, q);
            else if (mode == 3)
                sweep1_kernel<kCal, 1024><<<1, 1024, 0, s>>>(D, C, rec, d_out_h, d_flag, q);
            else
                sweep1_kernel<kCal, 256><<<1, 256, 0, s>>>(D, C, rec, d_out_h, d_flag, q);
            auto t1 = Clock::now();
            if (mode >= 8) {
                const int nbw = mode == 12 ? 1 : (mode == 13 ? (n + 1023) / 1024 : nbk);  // (15: nbk blocks of 64)
                for (int b = 0; b < nbw; ++b)
                    while (__atomic_load_n(h_flags + b, __ATOMIC_ACQUIRE) != q) {
                    }
                double tot = 0.0;
                for (int b = 0; b < nbw; ++b) tot += h_out8[3 * n + b];
                h_out[3 * n] = tot;
            } else {
                while (__atomic_load_n(h_flag, __ATOMIC_ACQUIRE) != q) {
                }
            }
            auto t2 = Clock::now();
            if (r >= 50) {
                t_launch += std::chrono::duration<double>(t1 - t0).count();
                t_wait += std::chrono::duration<double>(t2 - t1).count();
            }
        }
        CHECK(hipStreamSynchronize(s));
        std::printf("%-6s n=%d: launch %.2f us, wait %.2f us, round trip %.2f us\n", name, n, 1e6 * t_launch / reps,
                    1e6 * t_wait / reps, 1e6 * (t_launch + t_wait) / reps);
    };
    run("host", 0);
    run("dev", 1);
    run("flag", 2);
    run("flags", 8);
    run("noeval", 5);
    run("nofence", 6);
    run("neither", 7);
    run("ldonly", 9);
    run("stonly", 10);
    run("nold_nost", 11);
    run("nlns_wg1", 12);
    run("ls_1024", 13);
    run("nl_ns_nofence", 14);
    run("nl_ns_wg64", 15);
    run("one1024", 3);
    run("one256", 4);
    run("host", 0);
    std::printf("score %.6f\n", h_out[3 * n]);
    run("flags", 8);
    std::printf("score %.6f\n", h_out[3 * n]);
    return 0;
}
