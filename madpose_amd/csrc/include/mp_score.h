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

// Prepare the sweep constants of a model (host or device).
MP_HD void prepare_score_rec(const PairConst &C, const Model &m, ScoreRec &r) {
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
    r.pad = 0.0;
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

MP_HD double reproj_err(const double *M, const double *k, double u, double v, double a, double tu, double tv) {
    const double px = (M[0] * u + M[1] * v + M[2]) * a + k[0];
    const double py = (M[3] * u + M[4] * v + M[5]) * a + k[1];
    const double pz = (M[6] * u + M[7] * v + M[8]) * a + k[2];
    if (pz < 1e-2) return DBL_MAX;
    const double iz = rcp_depth(pz);
    const double ex = px * iz - tu, ey = py * iz - tv;
    return ex * ex + ey * ey;
}

MP_HD double sampson_err(const double *G, double au, double av, double bu, double bv) {
    const double e0 = G[0] * au + G[1] * av + G[2];
    const double e1 = G[3] * au + G[4] * av + G[5];
    const double e2 = G[6] * au + G[7] * av + G[8];
    const double f0 = G[0] * bu + G[3] * bv + G[6];
    const double f1 = G[1] * bu + G[4] * bv + G[7];
    const double c = bu * e0 + bv * e1 + e2;
    return div_nonneg(c * c, e0 * e0 + e1 * e1 + f0 * f0 + f1 * f1);
}

// Calibrated residuals in ray form (C.kstd: K = [k00 k01 k02; 0 k11 k12; 0 0 1] for
// both views): with a = K0^-1 x0 and b = K1^-1 x1 (third components 1),
//   t=0: q = R a (d0 + o0) + t,       x1 - proj(K1 q) = K1[0:2,0:2] (q_xy / q_z - b_xy)
//   t=1: q = R^T b (d1 s + o1 s) - R^T t, likewise against a through K0,
// the same quantities as EvaluateModelOnPoint (src/hybrid_pose_estimator.cpp:223-246)
// with K1 q / (K1 q)_z rewritten, and R a shared with the cheirality test (R n0 =
// (R a) r0) -- fewer FP64 instructions per (correspondence, model) than the matrix
// form M0 = K1 R K0^-1 of reproj_err.
MP_HD double reproj_ray(const double *q, const double *K, double bu, double bv) {
    if (q[2] < 1e-2) return DBL_MAX;
    const double iz = rcp_depth(q[2]);
    const double dx = fma(q[0], iz, -bu), dy = fma(q[1], iz, -bv);
    const double ex = fma(K[1], dy, K[0] * dx), ey = K[4] * dy;
    return fma(ex, ex, ey * ey);
}
MP_HD void eval_corr_cal_ray(const PairConst &C, const ScoreRec &r, const Corr &p, double &e0, double &e1, double &e2) {
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
        e0 = reproj_ray(q, C.K1, p.b0, p.b1);
    }
    {
        const double s1 = fma(p.d1, r.s, r.o1s);
        const double q[3] = {fma(rb0, s1, r.nrt[0]), fma(rb1, s1, r.nrt[1]), fma(rb2, s1, r.nrt[2])};
        e1 = reproj_ray(q, C.K0, p.a0, p.a1);
    }
    // check_cheirality(R, t, n0, n1, 1e-2) with R n0 = (R a) r0
    const double rn0 = ra0 * p.r0, rn1 = ra1 * p.r0, rn2 = ra2 * p.r0;
    const double a = -(rn0 * p.n1[0] + rn1 * p.n1[1] + rn2 * p.n1[2]);
    const double b1 = -(rn0 * t[0] + rn1 * t[1] + rn2 * t[2]);
    const double b2 = p.n1[0] * t[0] + p.n1[1] * t[1] + p.n1[2] * t[2];
    const double l1 = b1 - a * b2, l2 = -a * b1 + b2;
    const double md = 1e-2 * (1 - a * a);
    if (!(l1 > md && l2 > md)) {
        e2 = DBL_MAX;
        return;
    }
    e2 = sampson_err(r.G, p.a0, p.a1, p.b0, p.b1) * C.loss_scale;
}

// Squared errors of the three data types for one correspondence.
// gate: apply the score_type gating of EvaluateModelOnPoint (is_for_inlier == false).
template <int V>
MP_HD void eval_corr(const PairConst &C, const ScoreRec &r, const Corr &p, bool gate, double &e0, double &e1,
                     double &e2) {
    const bool skip_md = gate && C.score_type == 1;  // EPI_ONLY: reprojection gated
    const bool skip_epi = gate && C.score_type == 2; // MD_ONLY: Sampson gated
    e0 = skip_md ? DBL_MAX : reproj_err(r.M0, r.k0, p.x0u, p.x0v, p.d0 + r.o0, p.x1u, p.x1v);
    e1 = skip_md ? DBL_MAX : reproj_err(r.M1, r.k1, p.x1u, p.x1v, p.d1 * r.s + r.o1s, p.x0u, p.x0v);
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
        if (!check_cheirality(r.R, r.t, p.n0, p.n1, 1e-2)) {
            e2 = DBL_MAX;
            return;
        }
        e2 = sampson_err(r.G, p.a0, p.a1, p.b0, p.b1) * C.loss_scale;
    } else {
        e2 = sampson_err(r.G, p.x0u, p.x0v, p.x1u, p.x1v);
    }
}

} // namespace mp
