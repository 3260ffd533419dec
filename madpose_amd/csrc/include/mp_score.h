// Per-correspondence residuals of the three estimators, in the form the scoring
// sweep evaluates them (one correspondence per lane, model constants uniform).
//
// Reference: EvaluateModelOnPoint (src/hybrid_pose_estimator.cpp:216-261,
// src/hybrid_pose_shared_focal_estimator.cpp:160-202,
// src/hybrid_pose_two_focal_estimator.cpp:213-257), compute_sampson_error
// (src/utils.h:64-83), check_cheirality (src/solver.cpp:1188-1206), and the MSAC
// term min(e, thr) * w of ScoreModel/ComputeScore (src/hybrid_ransac.h:265-287).
// Sentinels follow the reference: DBL_MAX for z < 1e-2, failed cheirality or a
// score-type-gated residual; min(NaN, thr) stays NaN (std::min semantics).
#pragma once
#include <cfloat>

#include "mp_math.h"

namespace mp {

// ---------------------------------------------------------------------------
// Screening margins.  score_batch's sums decide nothing by themselves:
// the host decides every new best on reference-order sums (host/lo_sweep.h).  The
// device sums screen, and the screen must never hide a model the reference would take.
// For that the device needs, per model, a bound T on |S_dev - S_ref|, where S_ref is
// the reference's ScoreModel sum (src/hybrid_ransac.h:274-281: one running sum, type
// outer, index inner, of min(e, thr_t) w_t with e from EvaluateModelOnPoint) and S_dev
// this kernel's sum of its own residuals (other operations, FMA, another order).
//
// Two sources of difference, bounded separately:
// * summation order: both sums add the same kind of 3n terms, each in [0, thr_t |w_t|]
//   (a gated term is thr_t w_t), so each is within gamma_k * M of the exact sum of its
//   terms (k = 3n for the reference's sequential sum, 3 * trips + 16 for the device's
//   per-lane sums and fixed trees; gamma_k = k u / (1 - k u), u = 2^-53, M = n sum_t
//   thr_t |w_t|), for every n;
// * the terms themselves: min(., thr) is 1-Lipschitz and bounded by thr, so a term
//   differs by at most min(thr, |e_dev - e_ref|), and for a correspondence that is an
//   inlier on either side (e <= thr) |e_dev - e_ref| <= delta (2 sqrt(thr) + delta)
//   when the residual vectors differ by at most delta.  delta is a forward-error bound of
//   both forms against exact arithmetic on the same input doubles, per model from the
//   pair's magnitudes (score_margins below; the z < 1e-2 gate bounds 1 / z for the
//   correspondences it lets through).  That leaves the correspondences where no such
//   bound holds -- a depth within the error window of the z gate, a cheirality quantity
//   within its window, a Sampson denominator so small against |G| |a| |b| that the
//   relative error of the distance is unbounded -- and these the kernel flags
//   (eval_corr*: `flag`); an iteration with a flag is screened out entirely (its
//   models go to the host's reference-order resolution, its early exit stops).
// Every constant below is rounded up, and the whole bound is multiplied by kSafe = 4.
// The bound is exercised against the host's reference-order errors on adversarial
// samples (tests/test_margins_gpu.py).
constexpr double kU = 0x1p-53;
constexpr double kSafe = 4.0;
constexpr double kSampsonKappa = 0x1p-26; // den < kappa g^2 (alpha beta)^2: flagged
MP_HD double gam(double k) { return k * kU / (1.0 - k * kU); }

// reprojection t (0: x0 -> image 1 through K1; 1: x1 -> image 0 through K0): the
// forward-error bound delta of the residual vector (pixels) of both forms, for the
// correspondences the z gate lets through (z >= 1e-2 - wz) that are inliers on either
// side, is linear in Eq, the bound on |q_dev - q| of the point q before projection:
//   delta = kSafe (2 zinv Eq (Ks + U + Ks Qn) + gamma_8 (Ks (Qn + Bp) + U) + 8u Ks KX)
// with zinv <= 1 / (1e-2 - 2 Eq) <= 125 (Eq <= 1e-3, checked), Ks the max row |.|_1 of
// the target K's first two rows, U = X + sqrt(thr) + 1 the bound of an inlier's
// projection (X: max |coordinate| in the target image), Qn = kinv_abs(Ki, U) + 1 the
// bound of |q / q_z| for such a projection, KX = kinv_abs(Ki, X + 1), Bp the source
// ray's absolute sum.  kinv_abs(Ki, X): max over the first two rows of (|Ki_r0| +
// |Ki_r1|) X + |Ki_r2|, a bound of |K^-1 x| for |x| <= X.  c1 and c0 are pair constants
// for the calibrated estimator (margin_consts); with the focal in the model (K =
// diag(f, f, 1)) Ks = f, Qn = U / f + 1, KX = (X + 1) / f.
MP_HD double kinv_abs(const double (&Ki)[9], double X) {
    const double a = (fabs(Ki[0]) + fabs(Ki[1])) * X + fabs(Ki[2]);
    const double b = (fabs(Ki[3]) + fabs(Ki[4])) * X + fabs(Ki[5]);
    return a > b ? a : b;
}
MP_HD void reproj_coefs(double Ks, double U, double Qn, double KX, double Bp, double &c1, double &c0) {
    c1 = kSafe * 2.0 * 125.0 * (Ks + U + Ks * Qn);
    c0 = kSafe * (gam(8) * (Ks * (Qn + Bp) + U) + 8.0 * kU * Ks * KX);
}
// |e_dev - e_ref| bound for a term e = |r|^2 clipped at thr, residual vectors within
// delta (s2 = 2 sqrt(thr))
MP_HD double term_bound(double thr, double s2, double delta) {
    const double b = delta * (s2 + delta) + 8.0 * kU * thr;
    return b < thr ? b : thr;
}

// The model-independent parts of score_margins (host, once per pair, after the
// thresholds and weights are set).
inline void margin_consts(PairConst &C) {
    const bool cal = C.variant == kCal;
    const double X[2] = {C.ex1, C.ex0};
    for (int t = 0; t < 2; ++t) {
        C.mg_s2[t] = 2.0 * sqrt(C.thr[t]);
        C.mg_U[t] = X[t] + sqrt(C.thr[t]) + 1.0;
        C.mg_c0[t] = C.mg_c1[t] = 0.0;
    }
    if (cal) {
        auto rows_abs = [](const double (&K)[9]) {
            const double a = fabs(K[0]) + fabs(K[1]) + fabs(K[2]), b = fabs(K[3]) + fabs(K[4]) + fabs(K[5]);
            return a > b ? a : b;
        };
        reproj_coefs(rows_abs(C.K1), C.mg_U[0], kinv_abs(C.K1i, C.mg_U[0]) + 1.0, kinv_abs(C.K1i, C.ex1 + 1.0), C.ebp,
                     C.mg_c1[0], C.mg_c0[0]);
        reproj_coefs(rows_abs(C.K0), C.mg_U[1], kinv_abs(C.K0i, C.mg_U[1]) + 1.0, kinv_abs(C.K0i, C.ex0 + 1.0), C.eap,
                     C.mg_c1[1], C.mg_c0[1]);
    }
    // Sampson: for an unflagged correspondence (den >= kappa g^2 (alpha beta)^2, g = max
    // |G_ij|, alpha = |a_0| + |a_1| + 1, beta likewise) |c_dev - c_ref| / sqrt(den) <= rho
    // and den is known to a relative rel_den, so the distances sqrt(S) differ by at most
    // rho + sqrt(S) (rel_den / 2 + 4u).  Cc: the coefficient of u g alpha beta in |dc|
    // (the products of the rays' own errors, exi / exj, and of G's formation included).
    // Model-independent: the floor scales with the model's g.
    {
        const double Cc = 8.0 * (2.0 + 2.0 * C.exi + 2.0 * C.exj) + 60.0;
        const double isk = 1.0 / sqrt(kSampsonKappa);
        const double rho = kSafe * 2.0 * Cc * kU * isk;
        const double rel_den = kSafe * 16.0 * Cc * kU * isk + gam(8);
        const double L = cal ? C.loss_scale : 1.0;
        const double thr = C.thr[2] / L;
        const double d2 = rho + sqrt(thr) * (rel_den / 2.0 + 4.0 * kU);
        const double b = L * (d2 * (2.0 * sqrt(thr) + d2)) + 8.0 * kU * C.thr[2];
        C.mg_tau2 = b < C.thr[2] ? b : C.thr[2];
    }
    // summation order: both sums within gamma_k M of the exact sum of their terms
    const double n = C.n;
    const double Mabs = n * (C.thr[0] * fabs(C.w[0]) + C.thr[1] * fabs(C.w[1]) + C.thr[2] * fabs(C.w[2]));
    const double trips = (double)((C.n + 255) / 256);
    const double order = (gam(3.0 * n + 8.0) + gam(3.0 * trips + 16.0)) * Mabs;
    C.mg_fixed = kSafe * order + 16.0 * n * 0x1p-1074;
}

// Per model (device, with every model it solves; host, for the LO's models): the
// margin r.tie and the gate windows wz0, wz1, wl, kg2.  K0i, K1i: the model's inverse
// intrinsics (cal: the pair's).
MP_HD void score_margins(const PairConst &C, const Model &m, const double (&K0i)[9], const double (&K1i)[9],
                         ScoreRec &r, double *taus = nullptr) {
    const double inf = __builtin_inf();
    const bool cal = C.variant == kCal;
    const double *t = m.t;
    const double tinf = fmax(fabs(t[0]), fmax(fabs(t[1]), fabs(t[2])));
    const double t1 = fabs(t[0]) + fabs(t[1]) + fabs(t[2]);
    // |a|_1 and the per-point absolute sums of K^-1 x, in this model's K (uncal: 1/f)
    const double fi0 = K0i[0], fi1 = K1i[0];
    const double A = cal ? C.ea : C.ea * fi0 + 1.0, Ap = cal ? C.eap : A;
    const double B = cal ? C.eb : C.eb * fi1 + 1.0, Bp = cal ? C.ebp : B;
    // the point q before projection, each form within Eq of exact arithmetic
    const double Eq0 = gam(12) * ((A + Ap) * (C.ed0 + fabs(m.offset0)) + tinf);
    const double Eq1 = gam(14) * ((B + Bp) * (C.ed1 + fabs(m.offset1)) * fabs(m.scale) + t1);
    r.wz0 = kSafe * 2.0 * Eq0;
    r.wz1 = kSafe * 2.0 * Eq1;
    double c1[2], c0[2];
    if (cal) {
        c1[0] = C.mg_c1[0];
        c0[0] = C.mg_c0[0];
        c1[1] = C.mg_c1[1];
        c0[1] = C.mg_c0[1];
    } else { // K = diag(f, f, 1): target K1 for t = 0, K0 for t = 1
        const double f0 = m.focal0, f1 = C.variant == kSF ? m.focal0 : m.focal1;
        reproj_coefs(f1, C.mg_U[0], C.mg_U[0] * fi1 + 1.0, (C.ex1 + 1.0) * fi1, Bp, c1[0], c0[0]);
        reproj_coefs(f0, C.mg_U[1], C.mg_U[1] * fi0 + 1.0, (C.ex0 + 1.0) * fi0, Ap, c1[1], c0[1]);
    }
    const double tau0 = Eq0 <= 1e-3 ? term_bound(C.thr[0], C.mg_s2[0], c1[0] * Eq0 + c0[0]) : inf;
    const double tau1 = Eq1 <= 1e-3 ? term_bound(C.thr[1], C.mg_s2[1], c1[1] * Eq1 + c0[1]) : inf;
    const double tau2 = C.mg_tau2;
    double g = 0.0;
    for (int i = 0; i < 9; ++i) g = fmax(g, fabs(r.G[i]));
    // (the floor with the pair's largest (alpha beta)^2: one uniform comparison per
    // correspondence, and for each correspondence at least its own floor)
    r.kg2 = kSampsonKappa * g * g * C.eab2;
    if (taus) { // (test hook: the per-term bounds, before the safety factor of the sum)
        taus[0] = tau0;
        taus[1] = tau1;
        taus[2] = tau2;
    }
    // cheirality (calibrated): l1, l2 and min_depth (1 - a^2) 1e-2 of both forms
    r.wl = cal ? kSafe * gam(16) * (8.0 * t1 + 0.1) : 0.0;
    const double terms = C.n * (fabs(C.w[0]) * tau0 + fabs(C.w[1]) * tau1 + fabs(C.w[2]) * tau2);
    const double T = (kSafe * terms + C.mg_fixed) * (C.tie_scale > 1.0 ? C.tie_scale : 1.0);
    // a non-finite model constant: no screening (its residuals may be NaN where no gate
    // flags them, and the score kernel's minimum would drop the NaN)
    double fin = r.o0 + r.s + r.o1s + m.focal0 + m.focal1;
    for (int i = 0; i < 9; ++i) fin += r.R[i] + r.M0[i] + r.M1[i] + r.G[i];
    for (int i = 0; i < 3; ++i) fin += r.t[i] + r.k0[i] + r.k1[i] + r.nrt[i];
    r.tie = (T == T && fin - fin == 0.0) ? T : inf; // (NaN: no screening)
}

// Prepare the sweep constants of a model (host or device).  taus (nullable): the
// per-term bounds of score_margins (a test hook).
MP_HD void prepare_score_rec(const PairConst &C, const Model &m, ScoreRec &r, double *taus = nullptr) {
    double K0[9], K1[9], K0i[9], K1i[9];
    if (C.variant == kCal) {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            K0[i] = C.K0[i];
            K1[i] = C.K1[i];
            K0i[i] = C.K0i[i];
            K1i[i] = C.K1i[i];
        }
    } else {
        const double f0 = m.focal0, f1 = (C.variant == kSF) ? m.focal0 : m.focal1;
#pragma unroll
        for (int i = 0; i < 9; ++i) K0[i] = K1[i] = K0i[i] = K1i[i] = 0.0;
        K0[0] = K0[4] = f0;
        K1[0] = K1[4] = f1;
        K0i[0] = K0i[4] = 1.0 / f0;
        K1i[0] = K1i[4] = 1.0 / f1;
        K0[8] = K1[8] = K0i[8] = K1i[8] = 1.0;
    }
    const double *R = m.R, *t = m.t;
    double T[9], Rt[9];
    matmul3(R, K0i, T);
    matmul3(K1, T, r.M0);
    matvec3(K1, t, r.k0);
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) Rt[3 * a + b] = R[3 * b + a];
    matmul3(Rt, K1i, T);
    matmul3(K0, T, r.M1);
    double rtt[3];
    matvec3(Rt, t, rtt);
    double k1[3];
    matvec3(K0, rtt, k1);
    r.nrt[0] = -rtt[0];
    r.nrt[1] = -rtt[1];
    r.nrt[2] = -rtt[2];
    r.k1[0] = -k1[0];
    r.k1[1] = -k1[1];
    r.k1[2] = -k1[2];
    const double tx[9] = {0, -t[2], t[1], t[2], 0, -t[0], -t[1], t[0], 0};
    double E[9];
    matmul3(tx, R, E);
    if (C.variant == kCal) {
#pragma unroll
        for (int i = 0; i < 9; ++i) r.G[i] = E[i];
    } else {
        // F = K1^-T E K0^-1 with diagonal K
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) r.G[3 * a + b] = E[3 * a + b] * K1i[4 * a] * K0i[4 * b];
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) r.R[i] = R[i];
    r.t[0] = t[0];
    r.t[1] = t[1];
    r.t[2] = t[2];
    r.o0 = m.offset0;
    r.s = m.scale;
    r.o1s = m.offset1 * m.scale;
    score_margins(C, m, K0i, K1i, r, taus);
}

// One correspondence as the sweeps read it.  For the calibrated estimator the
// model-independent rays are formed once per correspondence (corr_rays), outside the
// loops over models: a = K0^-1 x0, b = K1^-1 x1 (xy; the Sampson terms) and the unit
// bearings n0, n1 (the cheirality test).
struct Corr {
    double x0u, x0v, x1u, x1v, d0, d1, r0, r1;
    double a0, a1, b0, b1, n0[3], n1[3];
};

MP_HD void corr_rays(const PairConst &C, Corr &p) {
    const double *Ki = C.K0i, *Kj = C.K1i;
    const double a0 = Ki[0] * p.x0u + Ki[1] * p.x0v + Ki[2];
    const double a1 = Ki[3] * p.x0u + Ki[4] * p.x0v + Ki[5];
    const double a2 = Ki[6] * p.x0u + Ki[7] * p.x0v + Ki[8];
    const double b0 = Kj[0] * p.x1u + Kj[1] * p.x1v + Kj[2];
    const double b1 = Kj[3] * p.x1u + Kj[4] * p.x1v + Kj[5];
    const double b2 = Kj[6] * p.x1u + Kj[7] * p.x1v + Kj[8];
    p.a0 = a0;
    p.a1 = a1;
    p.b0 = b0;
    p.b1 = b1;
    p.n0[0] = a0 * p.r0;
    p.n0[1] = a1 * p.r0;
    p.n0[2] = a2 * p.r0;
    p.n1[0] = b0 * p.r1;
    p.n1[1] = b1 * p.r1;
    p.n1[2] = b2 * p.r1;
}

// Reciprocals of the sweeps.  On the device, the hardware reciprocal refined by two
// Newton steps (within about an ulp of the correctly rounded quotient; 5 FP64
// instructions instead of the 11 of the IEEE division sequence) where x is finite and
// normal; the IEEE results elsewhere (1/inf = 0, NaN stays NaN, 1/0 and denormal x by
// division).
MP_HD double rcp_newton(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
#else
    return 1.0 / x;
#endif
}
// x >= 1e-2 or NaN (the reprojection depth after its z test)
MP_HD double rcp_depth(double x) { return (x > DBL_MAX) ? 0.0 : rcp_newton(x); }
// q / x for x >= 0 (the Sampson denominator)
MP_HD double div_nonneg(double q, double x) {
    if (__builtin_expect(x >= DBL_MIN && x <= DBL_MAX, 1)) return q * rcp_newton(x);
    return q / x;
}

// `flag` (OR-accumulated): the correspondence lies where the margins of score_margins do
// not hold -- the depth within wz of the z < 1e-2 gate, a cheirality quantity within wl
// of its threshold, or a Sampson denominator below the conditioning floor.
MP_HD double reproj_err(const double *M, const double *k, double u, double v, double a, double tu, double tv,
                        double wz, bool &flag) {
    const double px = (M[0] * u + M[1] * v + M[2]) * a + k[0];
    const double py = (M[3] * u + M[4] * v + M[5]) * a + k[1];
    const double pz = (M[6] * u + M[7] * v + M[8]) * a + k[2];
    flag = flag || !(fabs(pz - 1e-2) > wz); // (NaN: flagged)
    if (pz < 1e-2) return DBL_MAX;
    const double iz = rcp_depth(pz);
    const double ex = px * iz - tu, ey = py * iz - tv;
    return ex * ex + ey * ey;
}

MP_HD double sampson_err(const ScoreRec &r, double au, double av, double bu, double bv, bool &flag) {
    const double *G = r.G;
    const double e0 = G[0] * au + G[1] * av + G[2];
    const double e1 = G[3] * au + G[4] * av + G[5];
    const double e2 = G[6] * au + G[7] * av + G[8];
    const double f0 = G[0] * bu + G[3] * bv + G[6];
    const double f1 = G[1] * bu + G[4] * bv + G[7];
    const double c = bu * e0 + bv * e1 + e2;
    const double den = e0 * e0 + e1 * e1 + f0 * f0 + f1 * f1;
    flag = flag || !(den >= r.kg2);
    return div_nonneg(c * c, den);
}

// check_cheirality(R, t, n0, n1, 1e-2) (src/solver.cpp:1188-1206) given R n0: l1 > md
// and l2 > md decided by the signs of the differences (the same decisions for finite
// values), each flagged when within wl of zero
MP_HD bool cheirality_rn(const double *rn, const double *n1, const double *t, double wl, bool &flag) {
    const double a = -(rn[0] * n1[0] + rn[1] * n1[1] + rn[2] * n1[2]);
    const double b1 = -(rn[0] * t[0] + rn[1] * t[1] + rn[2] * t[2]);
    const double b2 = n1[0] * t[0] + n1[1] * t[1] + n1[2] * t[2];
    const double l1 = b1 - a * b2, l2 = -a * b1 + b2;
    const double md = 1e-2 * (1 - a * a);
    const double d1 = l1 - md, d2 = l2 - md;
    flag = flag || fabs(d1) <= wl || fabs(d2) <= wl;
    return d1 > 0.0 && d2 > 0.0;
}

// Calibrated residuals in ray form (C.kstd: K = [k00 k01 k02; 0 k11 k12; 0 0 1] for
// both views): with a = K0^-1 x0 and b = K1^-1 x1 (third components 1),
//   t=0: q = R a (d0 + o0) + t,       x1 - proj(K1 q) = K1[0:2,0:2] (q_xy / q_z - b_xy)
//   t=1: q = R^T b (d1 s + o1 s) - R^T t, likewise against a through K0,
// the same quantities as EvaluateModelOnPoint (src/hybrid_pose_estimator.cpp:223-246)
// with K1 q / (K1 q)_z rewritten, and R a shared with the cheirality test (R n0 =
// (R a) r0) -- fewer FP64 instructions per (correspondence, model) than the matrix
// form M0 = K1 R K0^-1 of reproj_err.
MP_HD double reproj_ray(const double *q, const double *K, double bu, double bv, double wz, bool &flag) {
    flag = flag || !(fabs(q[2] - 1e-2) > wz); // (NaN: flagged)
    if (q[2] < 1e-2) return DBL_MAX;
    const double iz = rcp_depth(q[2]);
    const double dx = fma(q[0], iz, -bu), dy = fma(q[1], iz, -bv);
    const double ex = fma(K[1], dy, K[0] * dx), ey = K[4] * dy;
    return fma(ex, ex, ey * ey);
}
MP_HD void eval_corr_cal_ray(const PairConst &C, const ScoreRec &r, const Corr &p, double &e0, double &e1, double &e2,
                             bool &flag) {
    const double *R = r.R, *t = r.t;
    // R a and R^T b (a_2 = b_2 = 1)
    const double ra0 = fma(R[0], p.a0, fma(R[1], p.a1, R[2]));
    const double ra1 = fma(R[3], p.a0, fma(R[4], p.a1, R[5]));
    const double ra2 = fma(R[6], p.a0, fma(R[7], p.a1, R[8]));
    const double rb0 = fma(R[0], p.b0, fma(R[3], p.b1, R[6]));
    const double rb1 = fma(R[1], p.b0, fma(R[4], p.b1, R[7]));
    const double rb2 = fma(R[2], p.b0, fma(R[5], p.b1, R[8]));
    {
        const double s0 = p.d0 + r.o0;
        const double q[3] = {fma(ra0, s0, t[0]), fma(ra1, s0, t[1]), fma(ra2, s0, t[2])};
        e0 = reproj_ray(q, C.K1, p.b0, p.b1, r.wz0, flag);
    }
    {
        const double s1 = fma(p.d1, r.s, r.o1s);
        const double q[3] = {fma(rb0, s1, r.nrt[0]), fma(rb1, s1, r.nrt[1]), fma(rb2, s1, r.nrt[2])};
        e1 = reproj_ray(q, C.K0, p.a0, p.a1, r.wz1, flag);
    }
    // check_cheirality(R, t, n0, n1, 1e-2) with R n0 = (R a) r0
    const double rn[3] = {ra0 * p.r0, ra1 * p.r0, ra2 * p.r0};
    if (!cheirality_rn(rn, p.n1, t, r.wl, flag)) {
        e2 = DBL_MAX;
        return;
    }
    e2 = sampson_err(r, p.a0, p.a1, p.b0, p.b1, flag) * C.loss_scale;
}

// Squared errors of the three data types for one correspondence.
// gate: apply the score_type gating of EvaluateModelOnPoint (is_for_inlier == false).
template <int V>
MP_HD void eval_corr(const PairConst &C, const ScoreRec &r, const Corr &p, bool gate, double &e0, double &e1,
                     double &e2, bool &flag) {
    const bool skip_md = gate && C.score_type == 1;  // EPI_ONLY: reprojection gated
    const bool skip_epi = gate && C.score_type == 2; // MD_ONLY: Sampson gated
    e0 = skip_md ? DBL_MAX : reproj_err(r.M0, r.k0, p.x0u, p.x0v, p.d0 + r.o0, p.x1u, p.x1v, r.wz0, flag);
    e1 = skip_md ? DBL_MAX : reproj_err(r.M1, r.k1, p.x1u, p.x1v, p.d1 * r.s + r.o1s, p.x0u, p.x0v, r.wz1, flag);
    if (C.scale_only) { // HybridPoseEstimatorScaleOnly also rejects small priors (:395, :408)
        if (p.d0 < 1e-2) e0 = DBL_MAX;
        if (p.d1 < 1e-2) e1 = DBL_MAX;
    }
    if (skip_epi) {
        e2 = DBL_MAX;
        return;
    }
    if (V == kCal) {
        // calibrated rays and unit bearings (corr_rays)
        double rn[3];
        matvec3(r.R, p.n0, rn);
        if (!cheirality_rn(rn, p.n1, r.t, r.wl, flag)) {
            e2 = DBL_MAX;
            return;
        }
        e2 = sampson_err(r, p.a0, p.a1, p.b0, p.b1, flag) * C.loss_scale;
    } else {
        e2 = sampson_err(r, p.x0u, p.x0v, p.x1u, p.x1v, flag);
    }
}

} // namespace mp
