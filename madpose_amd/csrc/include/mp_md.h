// Monocular-depth (MD) minimal solvers, GPU formulation.
//
// Reference: src/solver.cpp:35-480 (Groebner templates 12x12 / 36x36 / 40x40 +
// action-matrix eigen decomposition) and the pose stage :482-534, :682-739,
// :986-1043.  The systems are the pairwise distance constraints of rigidly moving,
// affinely corrected back-projections (see oracle/src/md.cpp for the derivation).
// Instead of a 36x36/40x40 template per sample, each thread
//   1. eliminates the monomials that appear linearly (3x3 / 4x4 / 5x5 Gaussian
//      elimination, in registers),
//   2. reduces the rest to one univariate polynomial (quartic / octic resultant),
//   3. finds its real roots with Sturm-sequence bisection,
//   4. polishes every root with Newton steps on the original equations,
//   5. recovers (R, t) with Horn's quaternion method.
// The solution sets equal the reference's (tests/test_engine_gpu.py::test_md_solver_matches_reference_goldens pins this
// against tests/golden/md_solvers.npz).
#pragma once
#include "mp_math.h"

namespace mp {

// a[i] for a runtime i by selects (keeps a small array in registers; indexing it
// with a runtime index would move it to scratch).  The elements pass through opaque()
// so the select chain is not folded back into a load from a selected address.
template <int N> MP_HD double pick(const double (&a)[N], int i) {
    double v = opaque(a[0]);
#pragma unroll
    for (int k = 1; k < N; ++k) v = (i == k) ? opaque(a[k]) : v;
    return v;
}


struct PairTerms {
    double A[3], B[3], dz0, dz1;
};

// full homogeneous 3-vectors (calibrated rays) or xy-only with depth differences
template <bool kXYOnly>
MP_HD PairTerms pair_terms(const double *xi, const double *xj, const double *yi, const double *yj, double dxi, double dxj,
                           double dyi, double dyj) {
    PairTerms p;
    p.A[0] = p.A[1] = p.A[2] = p.B[0] = p.B[1] = p.B[2] = 0.0;
    const int nc = kXYOnly ? 2 : 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        if (c < nc) {
            const double ax = xi[c] - xj[c], ex = dxi * xi[c] - dxj * xj[c];
            const double ay = yi[c] - yj[c], ey = dyi * yi[c] - dyj * yj[c];
            p.A[0] += ax * ax;
            p.A[1] += 2.0 * ex * ax;
            p.A[2] += ex * ex;
            p.B[0] += ay * ay;
            p.B[1] += 2.0 * ey * ay;
            p.B[2] += ey * ey;
        }
    }
    p.dz0 = (dxi - dxj) * (dxi - dxj);
    p.dz1 = (dyi - dyj) * (dyi - dyj);
    return p;
}

template <int A, int B> MP_HD void pmul(const double *a, const double *b, double *o) {
#pragma unroll
    for (int k = 0; k <= A + B; ++k) o[k] = 0.0;
#pragma unroll
    for (int i = 0; i <= A; ++i)
#pragma unroll
        for (int j = 0; j <= B; ++j) o[i + j] += a[i] * b[j];
}
template <int D> MP_HD double peval(const double *a, double x) {
    double v = a[D];
#pragma unroll
    for (int i = D - 1; i >= 0; --i) v = v * x + a[i];
    return v;
}

// Resultant in s of two quadratics in s whose coefficients are quadratics in w.
// X = al2 be0 - al0 be2, Y = al2 be1 - al1 be2, Z = al1 be0 - al0 be1, R = X^2 - Y Z.
MP_HD void quad_resultant(const double *al0, const double *al1, const double *al2, const double *be0,
                          const double *be1, const double *be2, double *X, double *Y, double *R) {
    double t0[5], t1[5], Z[5];
    pmul<2, 2>(al2, be0, t0);
    pmul<2, 2>(al0, be2, t1);
#pragma unroll
    for (int k = 0; k < 5; ++k) X[k] = t0[k] - t1[k];
    pmul<2, 2>(al2, be1, t0);
    pmul<2, 2>(al1, be2, t1);
#pragma unroll
    for (int k = 0; k < 5; ++k) Y[k] = t0[k] - t1[k];
    pmul<2, 2>(al1, be0, t0);
    pmul<2, 2>(al0, be1, t1);
#pragma unroll
    for (int k = 0; k < 5; ++k) Z[k] = t0[k] - t1[k];
    double a[9], b[9];
    pmul<4, 4>(X, X, a);
    pmul<4, 4>(Y, Z, b);
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = a[k] - b[k];
}

// distance-equation residual and gradient for (b1, beta, s, w0, w1):
//   F = w0 A.u + dz0 - s (w1 B.v + dz1),  u = (b1^2, b1, 1), v = (beta^2, beta, 1)
MP_HD double md_eq(const PairTerms &T, const double *z, double *g, bool xy) {
    const double ua = T.A[0] * z[0] * z[0] + T.A[1] * z[0] + T.A[2];
    const double vb = T.B[0] * z[1] * z[1] + T.B[1] * z[1] + T.B[2];
    const double dz0 = xy ? T.dz0 : 0.0, dz1 = xy ? T.dz1 : 0.0;
    g[0] = z[3] * (2.0 * T.A[0] * z[0] + T.A[1]);
    g[1] = -z[2] * z[4] * (2.0 * T.B[0] * z[1] + T.B[1]);
    g[2] = -(z[4] * vb + dz1);
    g[3] = ua;
    g[4] = -z[2] * vb;
    return z[3] * ua + dz0 - z[2] * (z[4] * vb + dz1);
}

// Newton polishing; K equations, unknown map: which of (b1,beta,s,w0,w1) are free.
// kind 0: cal (b1,beta,s; w0=w1=1), kind 1: sf (b1,beta,s,w; w0=w1=w), kind 2: tf (all 5)
template <int K, int KIND> MP_HD void md_polish(const PairTerms *T, double *z) {
    double best[5], rbest = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) best[i] = z[i];
    for (int it = 0; it < 4; ++it) {
        double J[K][K], F[K][1], r = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double g[5];
            double f = md_eq(T[k], z, g, KIND != 0);
            F[k][0] = f;
            r += f * f;
            J[k][0] = g[0];
            J[k][1] = g[1];
            J[k][2] = g[2];
            if (KIND == 1) J[k][3 % K] = g[3] + g[4]; // shared focal: d/dw of w0 = w1 = w
            if (KIND == 2) {
                J[k][3 % K] = g[3];
                J[k][4 % K] = g[4];
            }
        }
        if (it == 0 || r < rbest) {
            rbest = r;
#pragma unroll
            for (int i = 0; i < 5; ++i) best[i] = z[i];
        } else {
            break;
        }
        if (!(r > 0.0)) break;
        if (!gauss_solve<K, 1>(J, F)) break;
        z[0] -= F[0][0];
        z[1] -= F[1][0];
        z[2] -= F[2][0];
        if (KIND == 1) {
            z[3] -= F[3 % K][0];
            z[4] = z[3];
        }
        if (KIND == 2) {
            z[3] -= F[3 % K][0];
            z[4] -= F[4 % K][0];
        }
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) z[i] = best[i];
}

// The solvers in two parts: md_setup_* builds the per-sample system and its
// univariate polynomial (degree 4 / 8 / 4), md_root_* turns one real root into a
// solution (sol = (1, b1, a2, b2*a2, f0, f1)), false if rejected.  md_sols_*_e runs
// both in one lane; the group kernel (group_md.h) runs one root per lane.
struct MdCal {
    PairTerms T[3];
    double l1[3], l2[3];
    double poly[5];
};
MP_HD bool md_setup_cal(const double (&x)[3][3], const double (&y)[3][3], const double *dx, const double *dy,
                        MdCal &S) {
    PairTerms *T = S.T;
    T[0] = pair_terms<false>(x[0], x[1], y[0], y[1], dx[0], dx[1], dy[0], dy[1]);
    T[1] = pair_terms<false>(x[0], x[2], y[0], y[2], dx[0], dx[2], dy[0], dy[2]);
    T[2] = pair_terms<false>(x[1], x[2], y[1], y[2], dx[1], dx[2], dy[1], dy[2]);
    double Q[3][3], L[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            Q[k][c] = T[k].B[c];
            L[k][c] = T[k].A[c];
        }
    if (!gauss_solve<3, 3>(Q, L)) return false;
    // (s beta)^2 = (s beta^2) s, each monomial linear in (b1^2, b1, 1)
    const double l0[3] = {L[0][2], L[0][1], L[0][0]};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        S.l1[c] = L[1][2 - c];
        S.l2[c] = L[2][2 - c];
    }
    double a[5], b[5];
    pmul<2, 2>(S.l1, S.l1, a);
    pmul<2, 2>(l0, S.l2, b);
#pragma unroll
    for (int k = 0; k < 5; ++k) S.poly[k] = a[k] - b[k];
    return true;
}
MP_HD bool md_root_cal(const MdCal &S, double b1, double (&sol)[6]) {
    const double s = peval<2>(S.l2, b1);
    double z[5] = {b1, peval<2>(S.l1, b1) / s, s, 1.0, 1.0};
    md_polish<3, 0>(S.T, z);
    if (!(z[2] > 0.0)) return false;
    const double a2 = sqrt(z[2]);
    sol[0] = 1.0;
    sol[1] = z[0];
    sol[2] = a2;
    sol[3] = z[1] * a2;
    sol[4] = sol[5] = 1.0;
    return true;
}

// solve_scale_and_shift (calibrated): x, y are 3 homogeneous calibrated rays.
// Solutions ascending in b1; returns their count (<= 4).
template <class Emit>
MP_HD int md_sols_cal_e(const double (&x)[3][3], const double (&y)[3][3], const double *dx, const double *dy,
                        Emit &&emit) {
    MdCal S;
    if (!md_setup_cal(x, y, dx, dy, S)) return 0;
    double roots[4];
    const int nr = sturm_real_roots<4>(S.poly, roots);
    int n = 0;
    for (int r = 0; r < nr; ++r) {
        double sol[6];
        if (!md_root_cal(S, pick(roots, r), sol)) continue;
        emit(sol);
        ++n;
    }
    return n;
}

// solutions into sols[] (count <= 4)
MP_HD int md_sols_cal(const double (&x)[3][3], const double (&y)[3][3], const double *dx, const double *dy,
                      double (&sols)[4][6]) {
    int n = 0;
    return md_sols_cal_e(x, y, dx, dy, [&](const double (&sol)[6]) {
        for (int c = 0; c < 6; ++c) sols[n][c] = sol[c];
        ++n;
    });
}

MP_HD double mean_abs_xy(const double (&x)[4][3]) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) s += fabs(x[i][0]) + fabs(x[i][1]);
    return s / 8.0;
}

// solve_scale_and_shift_shared_focal: sol = (1, b1, a2, b2*a2, f, f); count <= 8
struct MdSF {
    PairTerms T[4];
    double q0[4][2], q1[4][2];
    double X[5], Y[5], R[9];
    double f0;
};
MP_HD bool md_setup_sf(const double (&x0)[4][3], const double (&y0)[4][3], const double *dx, const double *dy,
                       MdSF &S) {
    const double f0 = 0.5 * (mean_abs_xy(x0) + mean_abs_xy(y0)); // src/solver.cpp:134-138
    S.f0 = f0;
    double x[4][3], y[4][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[i][0] = x0[i][0] / f0;
        x[i][1] = x0[i][1] / f0;
        x[i][2] = x0[i][2];
        y[i][0] = y0[i][0] / f0;
        y[i][1] = y0[i][1] / f0;
        y[i][2] = y0[i][2];
    }
    const int pr[4][2] = {{0, 1}, {0, 2}, {1, 2}, {0, 3}};
    PairTerms *T = S.T;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        T[k] = pair_terms<true>(x[pr[k][0]], x[pr[k][1]], y[pr[k][0]], y[pr[k][1]], dx[pr[k][0]], dx[pr[k][1]],
                                dy[pr[k][0]], dy[pr[k][1]]);
    double M[4][4], L[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        M[k][0] = T[k].A[0];
        M[k][1] = T[k].A[1];
        M[k][2] = -T[k].B[0];
        M[k][3] = -T[k].B[1];
        L[k][0] = -T[k].A[2];
        L[k][1] = T[k].B[2];
        L[k][2] = T[k].dz1;
        L[k][3] = -T[k].dz0;
    }
    if (!gauss_solve<4, 4>(M, L)) return false;
    // monomial_r = q0_r(w) + s q1_r(w)   (t = s w substituted)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        S.q0[r][0] = L[r][3];
        S.q0[r][1] = L[r][0];
        S.q1[r][0] = L[r][2];
        S.q1[r][1] = L[r][1];
    }
    double al0[3], al1[3], al2[3], be0[3], be1[3], be2[3], t0[3], t1[3];
    pmul<1, 1>(S.q0[1], S.q0[1], t0);
    al0[0] = t0[0];
    al0[1] = t0[1] - S.q0[0][0];
    al0[2] = t0[2] - S.q0[0][1];
    pmul<1, 1>(S.q0[1], S.q1[1], t0);
    al1[0] = 2 * t0[0];
    al1[1] = 2 * t0[1] - S.q1[0][0];
    al1[2] = 2 * t0[2] - S.q1[0][1];
    pmul<1, 1>(S.q1[1], S.q1[1], al2);
    pmul<1, 1>(S.q0[3], S.q0[3], be0);
    pmul<1, 1>(S.q0[3], S.q1[3], t0);
    be1[0] = 2 * t0[0];
    be1[1] = 2 * t0[1] - S.q0[2][0];
    be1[2] = 2 * t0[2] - S.q0[2][1];
    pmul<1, 1>(S.q1[3], S.q1[3], t1);
    be2[0] = t1[0];
    be2[1] = t1[1] - S.q1[2][0];
    be2[2] = t1[2] - S.q1[2][1];
    quad_resultant(al0, al1, al2, be0, be1, be2, S.X, S.Y, S.R);
    return true;
}
MP_HD bool md_root_sf(const MdSF &S, double w, double (&sol)[6]) {
    const double s = -peval<4>(S.X, w) / peval<4>(S.Y, w);
    const double wb1 = peval<1>(S.q0[1], w) + s * peval<1>(S.q1[1], w);
    const double tb = peval<1>(S.q0[3], w) + s * peval<1>(S.q1[3], w);
    double z[5] = {wb1 / w, tb / (s * w), s, w, w};
    md_polish<4, 1>(S.T, z);
    if (z[3] < 0.0) return false; // src/solver.cpp:283
    if (!(z[2] > 0.0)) return false;
    const double a2 = sqrt(z[2]);
    const double f = S.f0 / sqrt(z[3]);
    sol[0] = 1.0;
    sol[1] = z[0];
    sol[2] = a2;
    sol[3] = z[1] * a2;
    sol[4] = sol[5] = f;
    return true;
}
template <class Emit>
MP_HD int md_sols_sf_e(const double (&x0)[4][3], const double (&y0)[4][3], const double *dx, const double *dy,
                       Emit &&emit) {
    MdSF S;
    if (!md_setup_sf(x0, y0, dx, dy, S)) return 0;
    double roots[8];
    const int nr = sturm_real_roots<8>(S.R, roots);
    int n = 0;
    for (int r = 0; r < nr; ++r) {
        double sol[6];
        if (!md_root_sf(S, pick(roots, r), sol)) continue;
        emit(sol);
        ++n;
    }
    return n;
}

// solutions into sols[] (count <= 8)
MP_HD int md_sols_sf(const double (&x0)[4][3], const double (&y0)[4][3], const double *dx, const double *dy,
                     double (&sols)[8][6]) {
    int n = 0;
    return md_sols_sf_e(x0, y0, dx, dy, [&](const double (&sol)[6]) {
        for (int c = 0; c < 6; ++c) sols[n][c] = sol[c];
        ++n;
    });
}

// solve_scale_and_shift_two_focal: sol = (1, b1, a2, b2*a2, f1, f2); count <= 4
struct MdTF {
    PairTerms T[5];
    double q0[5][2], q1[5];
    double X[5], Y[5], R[9]; // (R has degree 4 here)
    double f1, f2;
};
MP_HD bool md_setup_tf(const double (&x0)[4][3], const double (&y0)[4][3], const double *dx, const double *dy,
                       MdTF &S) {
    const double f1 = mean_abs_xy(x0), f2 = mean_abs_xy(y0); // src/solver.cpp:302-305
    S.f1 = f1;
    S.f2 = f2;
    double x[4][3], y[4][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[i][0] = x0[i][0] / f1;
        x[i][1] = x0[i][1] / f1;
        x[i][2] = x0[i][2];
        y[i][0] = y0[i][0] / f2;
        y[i][1] = y0[i][1] / f2;
        y[i][2] = y0[i][2];
    }
    const int pr[5][2] = {{0, 1}, {0, 2}, {1, 2}, {0, 3}, {1, 3}};
    PairTerms *T = S.T;
#pragma unroll
    for (int k = 0; k < 5; ++k)
        T[k] = pair_terms<true>(x[pr[k][0]], x[pr[k][1]], y[pr[k][0]], y[pr[k][1]], dx[pr[k][0]], dx[pr[k][1]],
                                dy[pr[k][0]], dy[pr[k][1]]);
    double M[5][5], L[5][3];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        M[k][0] = T[k].A[0];
        M[k][1] = T[k].A[1];
        M[k][2] = -T[k].B[0];
        M[k][3] = -T[k].B[1];
        M[k][4] = -T[k].dz1;
        L[k][0] = -T[k].A[2];
        L[k][1] = T[k].B[2];
        L[k][2] = -T[k].dz0;
    }
    if (!gauss_solve<5, 3>(M, L)) return false;
    // monomial_r = q0_r(w1) + t q1_r   (q1 constant)
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        S.q0[r][0] = L[r][2];
        S.q0[r][1] = L[r][0];
        S.q1[r] = L[r][1];
    }
    double al0[3], al1[3], al2[3], be0[3], be1[3], be2[3], t0[3];
    pmul<1, 1>(S.q0[1], S.q0[1], t0);
    al0[0] = t0[0];
    al0[1] = t0[1] - S.q0[0][0];
    al0[2] = t0[2] - S.q0[0][1];
    al1[0] = 2 * S.q0[1][0] * S.q1[1];
    al1[1] = 2 * S.q0[1][1] * S.q1[1] - S.q1[0];
    al1[2] = 0.0;
    al2[0] = S.q1[1] * S.q1[1];
    al2[1] = al2[2] = 0.0;
    pmul<1, 1>(S.q0[3], S.q0[3], be0);
    be1[0] = 2 * S.q0[3][0] * S.q1[3] - S.q0[2][0];
    be1[1] = 2 * S.q0[3][1] * S.q1[3] - S.q0[2][1];
    be1[2] = 0.0;
    be2[0] = S.q1[3] * S.q1[3] - S.q1[2];
    be2[1] = be2[2] = 0.0;
    quad_resultant(al0, al1, al2, be0, be1, be2, S.X, S.Y, S.R);
    return true;
}
MP_HD bool md_root_tf(const MdTF &S, double w1, double (&sol)[6]) {
    const double t = -peval<4>(S.X, w1) / peval<4>(S.Y, w1);
    double m[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) m[k] = peval<1>(S.q0[k], w1) + t * S.q1[k];
    const double s = m[4];
    double z[5] = {m[1] / w1, m[3] / t, s, w1, t / s};
    md_polish<5, 2>(S.T, z);
    if (z[3] < 0.0 || z[4] < 0.0) return false; // src/solver.cpp:470
    if (!(z[2] > 0.0)) return false;
    const double a2 = sqrt(z[2]);
    sol[0] = 1.0;
    sol[1] = z[0];
    sol[2] = a2;
    sol[3] = z[1] * a2;
    sol[4] = S.f1 / sqrt(z[3]);
    sol[5] = S.f2 / sqrt(z[4]);
    return true;
}
template <class Emit>
MP_HD int md_sols_tf_e(const double (&x0)[4][3], const double (&y0)[4][3], const double *dx, const double *dy,
                       Emit &&emit) {
    MdTF S;
    if (!md_setup_tf(x0, y0, dx, dy, S)) return 0;
    double roots[4];
    const int nr = sturm_real_roots<4>(S.R, roots); // resultant has degree 4 here
    int n = 0;
    for (int r = 0; r < nr; ++r) {
        double sol[6];
        if (!md_root_tf(S, pick(roots, r), sol)) continue;
        emit(sol);
        ++n;
    }
    return n;
}

// solutions into sols[] (count <= 4)
MP_HD int md_sols_tf(const double (&x0)[4][3], const double (&y0)[4][3], const double *dx, const double *dy,
                     double (&sols)[4][6]) {
    int n = 0;
    return md_sols_tf_e(x0, y0, dx, dy, [&](const double (&sol)[6]) {
        for (int c = 0; c < 6; ++c) sols[n][c] = sol[c];
        ++n;
    });
}

// Pose stage of solve_scale_shift_pose* (scale_on_x = false): positive corrected
// depths, focal division, rigid alignment.  K = 3 (cal) or 4 (sf/tf) points.
template <int K>
MP_HD bool md_pose_from_sol(const double (&x)[K][3], const double (&y)[K][3], const double *dx, const double *dy,
                            const double *sol, double fx, double fy, Model &m, bool check_positive = true) {
    // no FMA contraction: the positivity test of d2 = dy a2 + b2 a2 decides whether a
    // solution becomes a model, and must see the oracle's (md.cpp:400-404) doubles
#pragma clang fp contract(off)
    double X[K][3], Y[K][3], cx[3] = {0, 0, 0}, cy[3] = {0, 0, 0};
    bool ok = true;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const double d1 = dx[i] + sol[1];
        const double d2 = dy[i] * sol[2] + sol[3];
        if (!(d1 > 0.0) || !(d2 > 0.0)) ok = false; // src/solver.cpp:503-504
        X[i][0] = x[i][0] / fx * d1;
        X[i][1] = x[i][1] / fx * d1;
        X[i][2] = x[i][2] * d1;
        Y[i][0] = y[i][0] / fy * d2;
        Y[i][1] = y[i][1] / fy * d2;
        Y[i][2] = y[i][2] * d2;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            cx[c] += X[i][c];
            cy[c] += Y[i][c];
        }
    }
    if (check_positive && !ok) return false;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        cx[c] /= K;
        cy[c] /= K;
    }
    double Mx[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) Mx[a][b] += (X[i][a] - cx[a]) * (Y[i][b] - cy[b]);
    horn_rotation(Mx, m.R);
    double rc[3];
    matvec3(m.R, cx, rc);
#pragma unroll
    for (int c = 0; c < 3; ++c) m.t[c] = cy[c] - rc[c];
    m.scale = sol[2];
    m.offset0 = sol[1];
    m.offset1 = sol[3];
    return true;
}

// estimate_scale_and_pose (src/solver.cpp:5-33) for K points: Y ~ scale R X + t with
// weights W on the centroids and the cross-covariance, R from Horn's quaternion
// method (the Kabsch optimum, identical to the reference's SVD solution).
template <int K>
MP_HD void scale_and_pose(const double (&X)[K][3], const double (&Y)[K][3], const double *W, Model &m) {
    double ws = 0.0, cx[3] = {0, 0, 0}, cy[3] = {0, 0, 0};
#pragma unroll
    for (int i = 0; i < K; ++i) {
        ws += W[i];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            cx[c] += X[i][c] * W[i];
            cy[c] += Y[i][c] * W[i];
        }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        cx[c] /= ws;
        cy[c] /= ws;
    }
    double Mx[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) Mx[a][b] += (X[i][a] - cx[a]) * W[i] * (Y[i][b] - cy[b]);
    horn_rotation(Mx, m.R);
    double num = 0.0, den = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const double xc[3] = {X[i][0] - cx[0], X[i][1] - cx[1], X[i][2] - cx[2]};
        double rx[3];
        matvec3(m.R, xc, rx);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            num += (Y[i][c] - cy[c]) * rx[c];
            den += rx[c] * rx[c];
        }
    }
    m.scale = num / den;
    double rc[3];
    matvec3(m.R, cx, rc);
#pragma unroll
    for (int c = 0; c < 3; ++c) m.t[c] = cy[c] - m.scale * rc[c];
    m.offset0 = m.offset1 = 0.0;
}

// use_shift = false branch of the calibrated MD solver (src/hybrid_pose_estimator.cpp:87-120)
MP_HD void md_pose_noshift_cal(const double (&x)[3][3], const double (&y)[3][3], const double *dx, const double *dy,
                               Model &m) {
    double p0[3][3], p1[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            p0[i][c] = x[i][c] * dx[i];
            p1[i][c] = y[i][c] * dy[i];
        }
    const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    double num = 0.0, den = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double v0 = 0.0, v1 = 0.0;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            v0 += sq(p0[pr[k][0]][c] - p0[pr[k][1]][c]);
            v1 += sq(p1[pr[k][0]][c] - p1[pr[k][1]][c]);
        }
        v0 = sqrt(v0);
        v1 = sqrt(v1);
        num += v1 * v0;
        den += v1 * v1;
    }
    const double scale = num / den;
    double sol[4] = {1.0, 0.0, 1.0, 0.0};
    double dys[3] = {dy[0] * scale, dy[1] * scale, dy[2] * scale};
    md_pose_from_sol<3>(x, y, dx, dys, sol, 1.0, 1.0, m, false);
    m.scale = scale;
    m.offset0 = 0.0;
    m.offset1 = 0.0;
}

} // namespace mp
