// score_batch in isolation: one calibrated pair (N = 2000, 30 % outliers), B iterations
// of 1-4 models each (one near-ground-truth model, the rest perturbed poses, as in a
// real batch), timed with HIP events for
//   plain   the sweep without checks (EXIT = false),
//   inf     the early-exit sweep with no finite bound (check overhead only),
//   exit    the early-exit sweep with a realistic bound (1.3 x the best score),
// under a few check schedules; and checks that the early exit keeps every
// iteration's winner (score and slot) whenever that winner is below the bound.
// Build + run (on an MI355X):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/score_bench.hip -o tools/score_bench
//   tools/score_bench [iterations] [variant 0 cal | 1 sf | 2 tf]
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

static void rot(const double *axis, double ang, double *R) {
    const double n = std::sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
    const double x = axis[0] / n, y = axis[1] / n, z = axis[2] / n, c = std::cos(ang), s = std::sin(ang), C = 1 - c;
    const double M[9] = {c + x * x * C,     x * y * C - z * s, x * z * C + y * s, y * x * C + z * s, c + y * y * C,
                         y * z * C - x * s, z * x * C - y * s, z * y * C + x * s, c + z * z * C};
    for (int k = 0; k < 9; ++k) R[k] = M[k];
}

template <int V, int M>
static void bench(int B, std::mt19937 &rng) {
    const int n = V == kTF ? 4000 : 2000;
    std::uniform_real_distribution<double> U(-1, 1);
    std::normal_distribution<double> G(0, 1);
    const double f = 577.87, cx = 319.5, cy = 239.5;
    double Rg[9];
    const double ax[3] = {0.3, 1.0, 0.2};
    rot(ax, 0.25, Rg);
    const double tg[3] = {0.6, 0.05, 0.1};
    std::vector<double> x0u(n), x0v(n), x1u(n), x1v(n), d0(n), d1(n), r0(n), r1(n), ra0(n), ra1(n), rb0(n), rb1(n);
    for (int i = 0; i < n; ++i) {
        const double X[3] = {2 * U(rng), 1.5 * U(rng), 4.5 + 3.5 * U(rng)};
        double Y[3];
        for (int k = 0; k < 3; ++k) Y[k] = Rg[3 * k] * X[0] + Rg[3 * k + 1] * X[1] + Rg[3 * k + 2] * X[2] + tg[k];
        const bool out = (i % 10) < 3;
        x0u[i] = f * X[0] / X[2] + cx + G(rng);
        x0v[i] = f * X[1] / X[2] + cy + G(rng);
        x1u[i] = out ? 320 + 320 * U(rng) : f * Y[0] / Y[2] + cx + G(rng);
        x1v[i] = out ? 240 + 240 * U(rng) : f * Y[1] / Y[2] + cy + G(rng);
        d0[i] = X[2] * std::exp(0.05 * G(rng));
        d1[i] = Y[2] * std::exp(0.05 * G(rng));
        const double a[3] = {(x0u[i] - cx) / f, (x0v[i] - cy) / f, 1}, b[3] = {(x1u[i] - cx) / f, (x1v[i] - cy) / f, 1};
        r0[i] = 1 / std::sqrt(a[0] * a[0] + a[1] * a[1] + 1);
        ra0[i] = a[0];
        ra1[i] = a[1];
        rb0[i] = b[0];
        rb1[i] = b[1];
        r1[i] = 1 / std::sqrt(b[0] * b[0] + b[1] * b[1] + 1);
        if (V != kCal) { // normalized, pp-centred pixels
            x0u[i] = (x0u[i] - cx) / f;
            x0v[i] = (x0v[i] - cy) / f;
            x1u[i] = (x1u[i] - cx) / f;
            x1v[i] = (x1v[i] - cy) / f;
        }
    }
    auto up = [&](const std::vector<double> &v) {
        double *p;
        CHECK(hipMalloc(&p, v.size() * 8));
        CHECK(hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice));
        return p;
    };
    PairData D{up(x0u), up(x0v), up(x1u), up(x1v), up(d0), up(d1), up(r0), up(r1)};
    D.a0 = up(ra0); // (the calibrated ray form's precomputed rays, prep_pair_kernel)
    D.a1 = up(ra1);
    D.b0 = up(rb0);
    D.b1 = up(rb1);
    PairConst C{};
    C.variant = V;
    C.n = n;
    const double K[9] = {f, 0, cx, 0, f, cy, 0, 0, 1}, Ki[9] = {1 / f, 0, -cx / f, 0, 1 / f, -cy / f, 0, 0, 1};
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 9; ++k) {
        C.K0[k] = C.K1[k] = V == kCal ? K[k] : I[k];
        C.K0i[k] = C.K1i[k] = V == kCal ? Ki[k] : I[k];
    }
    C.kstd = 1;
    const double thr = V == kCal ? 64.0 : 64.0 / (f * f), thr2 = V == kCal ? 4.0 : 4.0 / (f * f);
    C.thr[0] = C.thr[1] = thr;
    C.thr[2] = thr2;
    C.w[0] = C.w[1] = 1.0;
    C.w[2] = 2.0 * thr / thr2;
    C.loss_scale = 1.0 / ((1.0 / (2 * f) + 1.0 / (2 * f)) * (1.0 / (2 * f) + 1.0 / (2 * f)));
    C.tie_scale = 1.0;
    margin_consts(C); // (magnitudes left at zero: the margins are only placeholders here)
    std::vector<ScoreRec> recs((size_t)B * M);
    std::vector<int> counts(B);
    std::uniform_int_distribution<int> nmd(1, 4);
    for (int b = 0; b < B; ++b) {
        counts[b] = std::min(M, nmd(rng));
        for (int m = 0; m < counts[b]; ++m) {
            Model md{};
            const bool good = (b % 97 == 0 && m == 0);
            const double ang = good ? 0.002 : 0.03 + 0.4 * std::fabs(U(rng));
            const double a2[3] = {U(rng), U(rng), U(rng)};
            double P[9];
            rot(a2, ang, P);
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    md.R[3 * r + c] = P[3 * r] * Rg[c] + P[3 * r + 1] * Rg[3 + c] + P[3 * r + 2] * Rg[6 + c];
            for (int k = 0; k < 3; ++k) md.t[k] = tg[k] + (good ? 0.001 : 0.3) * U(rng);
            md.scale = 1.0;
            md.offset0 = md.offset1 = 0.0;
            md.focal0 = md.focal1 = 1.0;
            prepare_score_rec(C, md, recs[(size_t)b * M + m]);
        }
    }
    ScoreRec *d_recs;
    int *d_counts, *d_work;
    double *d_scores;
    IterResult *d_res;
    CHECK(hipMalloc(&d_recs, recs.size() * sizeof(ScoreRec)));
    CHECK(hipMemcpy(d_recs, recs.data(), recs.size() * sizeof(ScoreRec), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_counts, B * 4));
    CHECK(hipMemcpy(d_counts, counts.data(), B * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&d_work, B * 4));
    CHECK(hipMalloc(&d_scores, (size_t)B * M * 8));
    CHECK(hipMalloc(&d_res, B * sizeof(IterResult)));
    const int ntrip = (n + kBlock - 1) / kBlock;
    auto launch = [&](bool exit, double cut, int first, int every) {
        ScoreBound sb{cut, first, every, d_work};
        if (exit)
            score_batch_kernel<V, M, true, true><<<B, kBlock>>>(D, C, d_recs, d_counts, d_scores, d_res, sb);
        else
            score_batch_kernel<V, M, true, false><<<B, kBlock>>>(D, C, d_recs, d_counts, d_scores, d_res, sb);
    };
    auto fetch = [&](std::vector<IterResult> &r, std::vector<int> &w) {
        CHECK(hipDeviceSynchronize());
        r.resize(B);
        w.resize(B);
        CHECK(hipMemcpy(r.data(), d_res, B * sizeof(IterResult), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(w.data(), d_work, B * 4, hipMemcpyDeviceToHost));
    };
    std::vector<IterResult> full, ex;
    std::vector<int> wf, we;
    launch(false, __builtin_inf(), 1, 1);
    fetch(full, wf);
    double best = DBL_MAX;
    for (int b = 0; b < B; ++b) best = std::min(best, full[b].best);
    const double bound = 1.3 * best;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](bool exit, double cut, int first, int every) {
        for (int w = 0; w < 3; ++w) launch(exit, cut, first, every);
        const int reps = 20;
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch(exit, cut, first, every);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return 1e3 * ms / reps;
    };
    std::printf("variant %d: N %d, %d iterations, %d trips, best %.6g, bound %.6g\n", V, n, B, ntrip, best, bound);
    std::printf("  plain (no checks)           %8.1f us\n", timeit(false, __builtin_inf(), 1, 1));
    const int scheds[][2] = {{std::max(1, ntrip / 4), 1}, {1, 1}, {2, 2}, {3, 1}, {std::max(1, ntrip / 2), 1},
                             {std::max(1, ntrip / 4), 2}};
    for (auto &sc : scheds) {
        const double t_inf = timeit(true, __builtin_inf(), sc[0], sc[1]);
        const double t_ex = timeit(true, bound * (1.0 + 1e-12), sc[0], sc[1]);
        launch(true, bound * (1.0 + 1e-12), sc[0], sc[1]);
        fetch(ex, we);
        long wsum = 0, wfull = 0, bad = 0;
        for (int b = 0; b < B; ++b) {
            wsum += we[b];
            wfull += (long)counts[b] * ntrip;
            const bool can_win = full[b].best < bound;
            if (can_win && (ex[b].best != full[b].best || ex[b].slot != full[b].slot)) ++bad;
            if (!can_win && ex[b].best < bound) ++bad;
        }
        std::printf("  checks first %d every %d: inf %8.1f us, exit %8.1f us, evaluated %.3f, winner mismatches %ld\n",
                    sc[0], sc[1], t_inf, t_ex, (double)wsum / wfull, bad);
    }
    for (void *p : {(void *)d_recs, (void *)d_counts, (void *)d_work, (void *)d_scores, (void *)d_res}) hipFree(p);
    for (const double *p : {D.x0u, D.x0v, D.x1u, D.x1v, D.d0, D.d1, D.r0, D.r1}) hipFree((void *)p);
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? std::atoi(argv[1]) : 9800;
    const int v = argc > 2 ? std::atoi(argv[2]) : -1;
    std::mt19937 rng(11);
    if (v < 0 || v == 0) bench<kCal, kMaxModelsCal>(B, rng);
    if (v < 0 || v == 1) bench<kSF, kMaxModelsSF>(B, rng);
    if (v < 0 || v == 2) bench<kTF, kMaxModelsTF>(B, rng);
    return 0;
}
