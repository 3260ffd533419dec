// Host LO sweep (see lo_sweep.h).  Built as plain C++ for the host (not a HIP
// translation unit), so that one function can carry an AVX-512 target attribute
// beside the x86-64-v3 (AVX2 + FMA) baseline of the rest of the library.
//
// Exactness: every residual is the operation sequence of the reference's
// EvaluateModelOnPoint as the oracle restates it (oracle/src/estimator.cpp
// evaluate_point; src/hybrid_pose_estimator.cpp:216-261, ..shared..:160-202,
// ..two..:213-257, src/utils.h:64-83, check_cheirality src/solver.cpp:1188-1206):
// the same products and sums in the same association, true IEEE divisions and square
// roots, no FMA contraction (`#pragma clang fp contract(off)`).  Lane-parallel SIMD
// arithmetic rounds exactly like the scalar code, so the errors are bit-identical to
// the oracle's, and the ScoreModel sum in the reference's order makes the score
// bit-identical too (tests/test_lo_sweep_cpu.py).  Model-independent quantities
// (K^-1 x and the unit bearings of the calibrated variant) are formed once per pair
// with the same operations.
#include "lo_sweep.h"
#include "env.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>

namespace mp {

namespace {

void free_aligned(double *p) { std::free(p); }

constexpr double kMax = DBL_MAX;

// o = M v, each row ((M0 v0 + M1 v1) + M2 v2) (oracle mv3)
#define MP_MV3(M, v0, v1, v2, o0, o1, o2)                                                                            \
    const double o0 = M[0] * (v0) + M[1] * (v1) + M[2] * (v2);                                                         \
    const double o1 = M[3] * (v0) + M[4] * (v1) + M[5] * (v2);                                                         \
    const double o2 = M[6] * (v0) + M[7] * (v1) + M[8] * (v2)

// Per-model constants of the sweep, formed exactly as the oracle forms them per point.
struct SweepModel {
    double R[9], t[3], K0[9], K1[9], K0i[9], K1i[9], E[9];
    double o0, o1, s, sampson_scale;
};

void sweep_model(const PairConst &C, const Model &m, SweepModel &M) {
#pragma clang fp contract(off)
    std::memcpy(M.R, m.R, sizeof(M.R));
    std::memcpy(M.t, m.t, sizeof(M.t));
    if (C.variant == kCal) {
        std::memcpy(M.K0, C.K0, sizeof(M.K0));
        std::memcpy(M.K1, C.K1, sizeof(M.K1));
        std::memcpy(M.K0i, C.K0i, sizeof(M.K0i));
        std::memcpy(M.K1i, C.K1i, sizeof(M.K1i));
    } else {
        const double f0 = m.focal0, f1 = (C.variant == kSF) ? m.focal0 : m.focal1;
        const double a[9] = {f0, 0, 0, 0, f0, 0, 0, 0, 1}, b[9] = {f1, 0, 0, 0, f1, 0, 0, 0, 1};
        const double ai[9] = {1.0 / f0, 0, 0, 0, 1.0 / f0, 0, 0, 0, 1};
        const double bi[9] = {1.0 / f1, 0, 0, 0, 1.0 / f1, 0, 0, 0, 1};
        std::memcpy(M.K0, a, sizeof(a));
        std::memcpy(M.K1, b, sizeof(b));
        std::memcpy(M.K0i, ai, sizeof(ai));
        std::memcpy(M.K1i, bi, sizeof(bi));
    }
    const double *R = m.R, *tt = m.t;
    const double tx[9] = {0, -tt[2], tt[1], tt[2], 0, -tt[0], -tt[1], tt[0], 0};
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) M.E[3 * r + c] = tx[3 * r] * R[c] + tx[3 * r + 1] * R[3 + c] + tx[3 * r + 2] * R[6 + c];
    if (C.variant != kCal) // F = K1^-T E K0^-1 (diagonal K)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) M.E[3 * r + c] *= M.K1i[4 * r] * M.K0i[4 * c];
    M.o0 = m.offset0;
    M.o1 = m.offset1;
    M.s = m.scale;
    M.sampson_scale = C.variant == kCal ? C.loss_scale : 1.0;
}

// Squared errors of correspondences [0, n): t = 0 (reprojection 0 -> 1), t = 1
// (1 -> 0), t = 2 (Sampson, cheirality-gated for the calibrated variant).
template <bool CAL>
[[gnu::always_inline]] inline void errors_body(const LoSweepData &D, const SweepModel &Min, int scale_only,
                                               double *__restrict e0o, double *__restrict e1o,
                                               double *__restrict e2o) {
#pragma clang fp contract(off)
    const SweepModel M = Min;
    const double *R = M.R, *tt = M.t, *K0 = M.K0, *K1 = M.K1, *K0i = M.K0i, *K1i = M.K1i, *E = M.E;
    const int n = D.n;
    const bool so = scale_only != 0;
    const double *__restrict x0u = D.x0u, *__restrict x0v = D.x0v, *__restrict x1u = D.x1u, *__restrict x1v = D.x1v;
    const double *__restrict d0 = D.d0, *__restrict d1 = D.d1;
    const double *__restrict ca0 = D.ca[0], *__restrict ca1 = D.ca[1], *__restrict ca2 = D.ca[2];
    const double *__restrict cb0 = D.cb[0], *__restrict cb1 = D.cb[1], *__restrict cb2 = D.cb[2];
    const double *__restrict ua0 = D.ua[0], *__restrict ua1 = D.ua[1], *__restrict ua2 = D.ua[2];
    const double *__restrict ub0 = D.ub[0], *__restrict ub1 = D.ub[1], *__restrict ub2 = D.ub[2];
#pragma clang loop vectorize(enable) interleave_count(1)
    for (int i = 0; i < n; ++i) {
        const double xa0 = x0u[i], xa1 = x0v[i], xb0 = x1u[i], xb1 = x1v[i];
        double c0, c1, c2, g0, g1, g2; // K0^-1 xa, K1^-1 xb
        if (CAL) {
            c0 = ca0[i];
            c1 = ca1[i];
            c2 = ca2[i];
            g0 = cb0[i];
            g1 = cb1[i];
            g2 = cb2[i];
        } else {
            MP_MV3(K0i, xa0, xa1, 1.0, k0, k1, k2);
            MP_MV3(K1i, xb0, xb1, 1.0, l0, l1, l2);
            c0 = k0;
            c1 = k1;
            c2 = k2;
            g0 = l0;
            g1 = l1;
            g2 = l2;
        }
        double e0, e1, e2;
        { // t = 0: K1 (R (K0^-1 xa (d0 + o0)) + t)
            const double p0 = c0 * (d0[i] + M.o0), p1 = c1 * (d0[i] + M.o0), p2 = c2 * (d0[i] + M.o0);
            MP_MV3(R, p0, p1, p2, q0r, q1r, q2r);
            const double q0 = q0r + tt[0], q1 = q1r + tt[1], q2 = q2r + tt[2];
            MP_MV3(K1, q0, q1, q2, r0, r1, z);
            const double u = r0 / z, v = r1 / z;
            const bool bad = z < 1e-2 || (so && d0[i] < 1e-2);
            e0 = bad ? kMax : (u - xb0) * (u - xb0) + (v - xb1) * (v - xb1);
        }
        { // t = 1: K0 (R^T (K1^-1 xb (d1 + o1) s - t))
            const double p0 = g0 * (d1[i] + M.o1) * M.s, p1 = g1 * (d1[i] + M.o1) * M.s,
                         p2 = g2 * (d1[i] + M.o1) * M.s;
            const double q0 = R[0] * (p0 - tt[0]) + R[3] * (p1 - tt[1]) + R[6] * (p2 - tt[2]);
            const double q1 = R[1] * (p0 - tt[0]) + R[4] * (p1 - tt[1]) + R[7] * (p2 - tt[2]);
            const double q2 = R[2] * (p0 - tt[0]) + R[5] * (p1 - tt[1]) + R[8] * (p2 - tt[2]);
            MP_MV3(K0, q0, q1, q2, r0, r1, z);
            const double u = r0 / z, v = r1 / z;
            const bool bad = z < 1e-2 || (so && d1[i] < 1e-2);
            e1 = bad ? kMax : (u - xa0) * (u - xa0) + (v - xa1) * (v - xa1);
        }
        { // t = 2: Sampson (src/utils.h:64-83)
            double ya0, ya1, yb0, yb1;
            bool ok = true;
            if (CAL) {
                // check_cheirality(R, t, unit bearings, 1e-2)
                MP_MV3(R, ua0[i], ua1[i], ua2[i], rx0, rx1, rx2);
                const double a = -(rx0 * ub0[i] + rx1 * ub1[i] + rx2 * ub2[i]);
                const double b1 = -(rx0 * tt[0] + rx1 * tt[1] + rx2 * tt[2]);
                const double b2 = ub0[i] * tt[0] + ub1[i] * tt[1] + ub2[i] * tt[2];
                const double l1 = b1 - a * b2;
                const double l2 = -a * b1 + b2;
                const double md = 1e-2 * (1 - a * a);
                ok = l1 > md && l2 > md;
                ya0 = c0;
                ya1 = c1;
                yb0 = g0;
                yb1 = g1;
            } else {
                ya0 = xa0;
                ya1 = xa1;
                yb0 = xb0;
                yb1 = xb1;
            }
            const double s0 = E[0] * ya0 + E[1] * ya1 + E[2];
            const double s1 = E[3] * ya0 + E[4] * ya1 + E[5];
            const double s2 = E[6] * ya0 + E[7] * ya1 + E[8];
            const double f0 = E[0] * yb0 + E[3] * yb1 + E[6];
            const double f1 = E[1] * yb0 + E[4] * yb1 + E[7];
            const double cc = yb0 * s0 + yb1 * s1 + s2;
            const double r2 = cc * cc / (s0 * s0 + s1 * s1 + f0 * f0 + f1 * f1);
            e2 = ok ? r2 * M.sampson_scale : kMax;
        }
        e0o[i] = e0;
        e1o[i] = e1;
        e2o[i] = e2;
    }
}

// ScoreModel's sum (src/hybrid_ransac.h:274-281): one accumulator, t outer, i
// ascending; std::min(e, thr) is (thr < e) ? thr : e (a NaN error stays NaN); a
// score-type-gated residual is DBL_MAX, i.e. the term thr * w
double ordered_score(const PairConst &C, const double *err, int n) {
#pragma clang fp contract(off)
    const bool gate_md = C.score_type == 1, gate_epi = C.score_type == 2; // EPI_ONLY / MD_ONLY
    double s = 0.0;
    for (int t = 0; t < 3; ++t) {
        const double th = C.thr[t], w = C.w[t];
        const double *e = err + (size_t)t * n;
        if ((t < 2 && gate_md) || (t == 2 && gate_epi)) {
            const double c = ((th < kMax) ? th : kMax) * w;
            for (int i = 0; i < n; ++i) s += c;
        } else {
            for (int i = 0; i < n; ++i) {
                const double m = (th < e[i]) ? th : e[i];
                s += m * w;
            }
        }
    }
    return s;
}

// The fast sum of the same terms: 32 independent accumulators (four 8-lane vectors)
// over each type's terms, then a fixed tree; and sum |term| for the bound.
template <bool W512> [[gnu::always_inline]] inline void fast_sum_body(const PairConst &C, const double *err, int n,
                                                                      double *sum, double *abs_sum) {
#pragma clang fp contract(off)
    const bool gate_md = C.score_type == 1, gate_epi = C.score_type == 2;
    double acc[32], aac[32];
    for (int k = 0; k < 32; ++k) acc[k] = aac[k] = 0.0;
    for (int t = 0; t < 3; ++t) {
        const double th = C.thr[t], w = C.w[t];
        const double *e = err + (size_t)t * n;
        if ((t < 2 && gate_md) || (t == 2 && gate_epi)) {
            const double c = ((th < kMax) ? th : kMax) * w;
            acc[t] += c * n;
            aac[t] += std::fabs(c) * n;
            continue;
        }
        int i = 0;
        for (; i + 32 <= n; i += 32) {
#pragma clang loop vectorize(enable)
            for (int k = 0; k < 32; ++k) {
                const double m = ((th < e[i + k]) ? th : e[i + k]) * w;
                acc[k] += m;
                aac[k] += std::fabs(m);
            }
        }
        for (; i < n; ++i) {
            const double m = ((th < e[i]) ? th : e[i]) * w;
            acc[i & 31] += m;
            aac[i & 31] += std::fabs(m);
        }
    }
    for (int w = 16; w >= 1; w >>= 1)
        for (int k = 0; k < w; ++k) {
            acc[k] += acc[k + w];
            aac[k] += aac[k + w];
        }
    *sum = acc[0];
    *abs_sum = aac[0];
}
void fast_sum_avx2(const PairConst &C, const double *err, int n, double *s, double *a) {
    fast_sum_body<false>(C, err, n, s, a);
}
__attribute__((target("avx512f,avx512dq,avx512vl"))) void fast_sum_avx512(const PairConst &C, const double *err,
                                                                           int n, double *s, double *a) {
    fast_sum_body<true>(C, err, n, s, a);
}

void sweep_avx2(const LoSweepData &D, const SweepModel &M, int so, double *err) {
    if (D.cal)
        errors_body<true>(D, M, so, err, err + D.n, err + 2 * (size_t)D.n);
    else
        errors_body<false>(D, M, so, err, err + D.n, err + 2 * (size_t)D.n);
}

__attribute__((target("avx512f,avx512dq,avx512vl"))) void sweep_avx512(const LoSweepData &D, const SweepModel &M,
                                                                         int so, double *err) {
    if (D.cal)
        errors_body<true>(D, M, so, err, err + D.n, err + 2 * (size_t)D.n);
    else
        errors_body<false>(D, M, so, err, err + D.n, err + 2 * (size_t)D.n);
}

bool use_avx512() {
    static const bool on = [] {
        if (env_avx2("MADPOSE_LO_SWEEP_ISA")) return false; // the 4-wide path (A/B)
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
               __builtin_cpu_supports("avx512vl");
    }();
    return on;
}

} // namespace

void lo_sweep_prepare(const PairConst &C, const double *x0, const double *x1, const double *d0, const double *d1,
                      LoSweepData *D) {
#pragma clang fp contract(off)
    const int n = C.n;
    const size_t stride = ((size_t)std::max(n, 1) + 7) & ~(size_t)7; // 64-byte rows
    const bool cal = C.variant == kCal;
    const int rows = cal ? 18 : 6;
    double *p = static_cast<double *>(std::aligned_alloc(64, sizeof(double) * stride * rows));
    if (!p) throw std::bad_alloc();
    D->store = std::unique_ptr<double[], void (*)(double *)>(p, free_aligned);
    double *row[18];
    for (int k = 0; k < rows; ++k) row[k] = p + stride * k;
    for (int i = 0; i < n; ++i) {
        row[0][i] = x0[2 * i];
        row[1][i] = x0[2 * i + 1];
        row[2][i] = x1[2 * i];
        row[3][i] = x1[2 * i + 1];
        row[4][i] = d0[i];
        row[5][i] = d1[i];
    }
    D->n = n;
    D->cal = cal ? 1 : 0;
    D->x0u = row[0];
    D->x0v = row[1];
    D->x1u = row[2];
    D->x1v = row[3];
    D->d0 = row[4];
    D->d1 = row[5];
    for (int k = 0; k < 3; ++k) D->ca[k] = D->cb[k] = D->ua[k] = D->ub[k] = nullptr;
    if (!cal) return;
    // K0^-1 xa, K1^-1 xb and the unit bearings, as evaluate_point forms them
    const double *K0i = C.K0i, *K1i = C.K1i;
    for (int i = 0; i < n; ++i) {
        MP_MV3(K0i, row[0][i], row[1][i], 1.0, a0, a1, a2);
        MP_MV3(K1i, row[2][i], row[3][i], 1.0, b0, b1, b2);
        const double na = std::sqrt(a0 * a0 + a1 * a1 + a2 * a2);
        const double nb = std::sqrt(b0 * b0 + b1 * b1 + b2 * b2);
        row[6][i] = a0;
        row[7][i] = a1;
        row[8][i] = a2;
        row[9][i] = b0;
        row[10][i] = b1;
        row[11][i] = b2;
        row[12][i] = a0 / na;
        row[13][i] = a1 / na;
        row[14][i] = a2 / na;
        row[15][i] = b0 / nb;
        row[16][i] = b1 / nb;
        row[17][i] = b2 / nb;
    }
    for (int k = 0; k < 3; ++k) {
        D->ca[k] = row[6 + k];
        D->cb[k] = row[9 + k];
        D->ua[k] = row[12 + k];
        D->ub[k] = row[15 + k];
    }
}

double lo_sweep(const PairConst &C, const LoSweepData &D, const Model &m, double *err) {
    SweepModel M;
    sweep_model(C, m, M);
    if (use_avx512())
        sweep_avx512(D, M, C.scale_only, err);
    else
        sweep_avx2(D, M, C.scale_only, err);
    return ordered_score(C, err, D.n);
}

void lo_sweep_fast(const PairConst &C, const LoSweepData &D, const Model &m, double *err, double *fast,
                   double *bound) {
    SweepModel M;
    sweep_model(C, m, M);
    double s = 0.0, a = 0.0;
    if (use_avx512()) {
        sweep_avx512(D, M, C.scale_only, err);
        fast_sum_avx512(C, err, D.n, &s, &a);
    } else {
        sweep_avx2(D, M, C.scale_only, err);
        fast_sum_avx2(C, err, D.n, &s, &a);
    }
    // both sums of the same 3n terms are within gamma_{3n} sum|term| of the exact sum
    // (the fast one's depth is below 3n); |a| itself is computed to within gamma_{3n};
    // an underflowing term can add 2^-1075 per operation
    const double k = 3.0 * D.n + 8.0, u = 0x1p-53;
    const double g = k * u / (1.0 - k * u);
    *fast = s;
    *bound = 2.0 * g * a * (1.0 + 2.0 * g) + 8.0 * k * 0x1p-1074;
}

double lo_ordered_score(const PairConst &C, const double *err, int n) { return ordered_score(C, err, n); }

int lo_sweep_width() { return use_avx512() ? 512 : 256; }

} // namespace mp
