// Point minimal solvers of the uncalibrated estimators, GPU formulation (one sample
// per thread, everything in registers / private memory):
//
//   relpose_7pt_F   PoseLib relpose_7pt as called at
//                   src/hybrid_pose_two_focal_estimator.cpp:116 -- Householder null
//                   space of the 7x9 epipolar system, det(a N0 + N1) expanded
//                   multilinearly into a cubic, PoseLib's closed-form solve_cubic_real
//                   (round 6: the oracle's restatement, oracle/src/pt_poselib.cpp).
//   bougnoux_sq     the reference's bougnoux_focals (:11-32) in closed form (the
//                   epipoles are the cross products of rows / columns of the rank-2 F).
//   recover_pose_cv cv::recoverPose(E, p0, p1, I, R, t, 1e9) (:143): R1 = U W V^T,
//                   R2 = U W^T V^T, t = u3; V from a Jacobi eigen-decomposition of
//                   E^T E with the canonical signs documented in oracle/src/pt67.cpp;
//                   per-point DLT triangulation decides "good" points.
//   relpose_6pt_sf  PoseLib relpose_6pt_shared_focal (..shared_focal_estimator.cpp:87):
//                   F = x N0 + y N1 + N2, w = 1/f^2, the ten equations
//                   (M0 + w M1 + w^2 M2) v(x, y) = 0.  With u = 1/w the determinant
//                   det(u^2 M0 + u M1 + M2) = u^5 q(u), deg q = 15; q is recovered by
//                   a 16-point DFT of complex LU determinants on the circle |u| = rho
//                   (rho adapted once to the root magnitudes), its positive real roots
//                   are isolated by Sturm sequences, and each (x, y, w) is polished by
//                   Gauss-Newton on the ten equations before motion_from_essential.
// The CPU oracle solves the same systems by different means (SVD null spaces, a
// 20x20 companion eigenproblem, SVD epipoles), so parity tests cross-check both.
#pragma once
#include "mp_pt.h"

namespace mp {

// Householder null space of a K x 9 system (rows = epipolar constraints).
template <int K> MP_HD void nullspace_kx9(const double (&Q)[K][9], double (&N)[9 - K][9]) {
    double A[9][K];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int e = 0; e < 9; ++e) A[e][i] = Q[i][e];
    double V[K][9], beta[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double nrm = 0.0;
#pragma unroll
        for (int i = 0; i < 9; ++i)
            if (i >= k) nrm += A[i][k] * A[i][k];
        nrm = sqrt(nrm);
        const double alpha = (A[k][k] > 0) ? -nrm : nrm;
        double vn = 0.0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            V[k][i] = (i < k) ? 0.0 : A[i][k];
            if (i == k) V[k][i] -= alpha;
            vn += V[k][i] * V[k][i];
        }
        beta[k] = (vn > 0) ? 2.0 / vn : 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if (j >= k) {
                double d = 0.0;
#pragma unroll
                for (int i = 0; i < 9; ++i) d += V[k][i] * A[i][j];
                d *= beta[k];
#pragma unroll
                for (int i = 0; i < 9; ++i) A[i][j] -= d * V[k][i];
            }
        }
    }
#pragma unroll
    for (int b = 0; b < 9 - K; ++b) {
        double v[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) v[i] = (i == K + b) ? 1.0 : 0.0;
#pragma unroll
        for (int k = K - 1; k >= 0; --k) {
            double d = 0.0;
#pragma unroll
            for (int i = 0; i < 9; ++i) d += V[k][i] * v[i];
            d *= beta[k];
#pragma unroll
            for (int i = 0; i < 9; ++i) v[i] -= d * V[k][i];
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) N[b][i] = v[i];
    }
}

template <int K>
MP_HD void epipolar_rows(const double (&x1)[K][3], const double (&x2)[K][3], double (&Q)[K][9]) {
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) Q[i][3 * r + c] = x2[i][r] * x1[i][c];
}

// det of the 3x3 matrix with rows a, b, c (each 3 consecutive doubles)
MP_HD double det_rows(const double *a, const double *b, const double *c) {
    return a[0] * (b[1] * c[2] - b[2] * c[1]) - a[1] * (b[0] * c[2] - b[2] * c[0]) + a[2] * (b[0] * c[1] - b[1] * c[0]);
}

// ---------------------------------------------------------------------------
// det_rows without FMA contraction (the 7pt cubic: the oracle's expression)
MP_HD double det_rows_x(const double *a, const double *b, const double *c) {
#pragma clang fp contract(off)
    return a[0] * (b[1] * c[2] - b[2] * c[1]) - a[1] * (b[0] * c[2] - b[2] * c[0]) + a[2] * (b[0] * c[1] - b[1] * c[0]);
}

// PoseLib misc/univariate.cc solve_cubic_real (oracle/src/pt_poselib.cpp): real roots of
// x^3 + c2 x^2 + c1 x + c0 -- Cardano when the discriminant term is positive (one
// root), the trigonometric form otherwise (three), one Newton step each.  The root
// count depends on +, -, *, / only, so it is the oracle's; cbrt / acos / cos come from
// the device math library (the host's may differ in the last bit).
MP_HD int solve_cubic_real_x(double c2, double c1, double c0, double (&roots)[3]) {
#pragma clang fp contract(off)
    double a = c1 - c2 * c2 / 3.0;
    double b = (2.0 * c2 * c2 * c2 - 9.0 * c2 * c1) / 27.0 + c0;
    double c = b * b / 4.0 + a * a * a / 27.0;
    int n_roots;
    if (c > 0) {
        c = sqrt(c);
        b *= -0.5;
        roots[0] = cbrt(b + c) + cbrt(b - c) - c2 / 3.0;
        roots[1] = roots[2] = 0.0;
        n_roots = 1;
    } else {
        c = 3.0 * b / (2.0 * a) * sqrt(-3.0 / a);
        const double d = 2.0 * sqrt(-a / 3.0);
        const double theta = acos(c) / 3.0;
        roots[0] = d * cos(theta) - c2 / 3.0;
        roots[1] = d * cos(theta - 2.0 * M_PI / 3.0) - c2 / 3.0;
        roots[2] = d * cos(theta - 4.0 * M_PI / 3.0) - c2 / 3.0;
        n_roots = 3;
    }
    static_for<3>([&](auto i) {
        if (i < n_roots) {
            const double x = roots[i];
            const double x2 = x * x;
            const double x3 = x * x2;
            const double dx = -(x3 + c2 * x2 + c1 * x + c0) / (3 * x2 + 2 * c2 * x + c1);
            roots[i] += dx;
        }
    });
    return n_roots;
}

// 7-point fundamental matrices (PoseLib relpose_7pt, as the oracle's restatement
// oracle/src/pt_poselib.cpp): Householder null space of the 7 x 9 system, det(a N0 +
// N1) expanded by rows into c3 a^3 + .. + c0, normalised by c3, solve_cubic_real, F = a
// N0 + N1 normalised.  Returns k (1 or 3), F[k] row-major with x2^T F x1 = 0.  (Until
// round 5: Sturm bisection of the cubic.)
MP_HD int relpose_7pt_F(const double (&x1)[7][3], const double (&x2)[7][3], double (&F)[3][9]) {
#pragma clang fp contract(off)
    double Q[7][9], N[2][9];
    epipolar_rows<7>(x1, x2, Q);
    householder_nullspace_x<7>(Q, N);
    const double *A = N[0], *B = N[1];
    const double c3 = det_rows_x(A, A + 3, A + 6);
    double c2 = det_rows_x(A, A + 3, B + 6) + det_rows_x(A, B + 3, A + 6) + det_rows_x(B, A + 3, A + 6);
    double c1 = det_rows_x(A, B + 3, B + 6) + det_rows_x(B, A + 3, B + 6) + det_rows_x(B, B + 3, A + 6);
    double c0 = det_rows_x(B, B + 3, B + 6);
    const double inv_c3 = 1.0 / c3;
    c2 *= inv_c3;
    c1 *= inv_c3;
    c0 *= inv_c3;
    double roots[3];
    const int nr = solve_cubic_real_x(c2, c1, c0, roots);
    // (constant indices from the front end on: F and roots stay in registers)
    static_for<3>([&](auto K) {
        constexpr int k = decltype(K)::value;
        if (k < nr) {
            double nn = 0.0;
#pragma unroll
            for (int e = 0; e < 9; ++e) {
                F[k][e] = roots[k] * A[e] + B[e];
                nn += F[k][e] * F[k][e];
            }
            nn = sqrt(nn);
#pragma unroll
            for (int e = 0; e < 9; ++e) F[k][e] /= nn;
        }
    });
    return nr;
}

// unit vector orthogonal to the three given vectors (largest pairwise cross product)
MP_HD void null3(const double *a, const double *b, const double *c, double *n) {
    double ab[3], ac[3], bc[3];
    cross3(a, b, ab);
    cross3(a, c, ac);
    cross3(b, c, bc);
    const double nab = dot3(ab, ab), nac = dot3(ac, ac), nbc = dot3(bc, bc);
#pragma unroll
    for (int r = 0; r < 3; ++r) n[r] = (nab >= nac && nab >= nbc) ? ab[r] : (nac >= nbc ? ac[r] : bc[r]);
}

// bougnoux_focals (src/hybrid_pose_two_focal_estimator.cpp:11-32): squared focals
MP_HD void bougnoux_sq(const double *F, double *f0_sq, double *f1_sq) {
    double e1[3], e2[3];
    null3(F, F + 3, F + 6, e1); // F e1 = 0
    const double c0[3] = {F[0], F[3], F[6]}, c1[3] = {F[1], F[4], F[7]}, c2[3] = {F[2], F[5], F[8]};
    null3(c0, c1, c2, e2); // e2^T F = 0
    const double i1 = svd_rcp(e1[2]), i2 = svd_rcp(e2[2]);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        e1[k] *= i1;
        e2[k] *= i2;
    }
    // row (-e2y, e2x, 0) F  and  row (-e1y, e1x, 0) F^T
    double L[3], M[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        L[c] = -e2[1] * F[c] + e2[0] * F[3 + c];
        M[c] = -e1[1] * F[3 * c] + e1[0] * F[3 * c + 1];
    }
    *f0_sq = -(L[2] * F[8]) * svd_rcp(L[0] * F[6] + L[1] * F[7]);
    *f1_sq = -(M[2] * F[8]) * svd_rcp(M[0] * F[2] + M[1] * F[5]);
}

// Cyclic Jacobi eigen-decomposition of a symmetric 3x3 matrix (A becomes diagonal,
// V accumulates eigenvectors as columns).
MP_HD void jacobi_eig3(double (&A)[3][3], double (&V)[3][3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 16; ++sweep) {
        double off = 0.0, dn = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            dn += A[i][i] * A[i][i];
#pragma unroll
            for (int j = i + 1; j < 3; ++j) off += A[i][j] * A[i][j];
        }
        if (!(off > 1e-32 * dn)) break;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = p + 1; q < 3; ++q) {
                // rotations below 1e-150 of the diagonal are skipped so th*th stays finite
                if (!(fabs(A[p][q]) > 1e-150 * (fabs(A[p][p]) + fabs(A[q][q])))) continue;
                const double th = (A[q][q] - A[p][p]) * svd_rcp(2.0 * A[p][q]);
                const double u = fma(th, th, 1.0);
                const double t = (th >= 0 ? 1.0 : -1.0) * svd_rcp(fabs(th) + u * svd_rsq(u));
                const double c = svd_rsq(fma(t, t, 1.0)), s = t * c;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
}

// cv::recoverPose(E, p0, p1, I, R, t, dist) in three parts: the candidate poses of E
// (OpenCV's decomposeEssentialMat order: (R1, t), (R2, t), (R1, -t), (R2, -t)), the
// per-point DLT test of a candidate, and the choice of the candidate with the most
// good points (first maximum).  recover_pose_cv runs them over K points in one lane;
// the group tail kernel (group_tail.h) runs one point per lane.
struct RecoverCands {
    double R1[9], R2[9], u2[3];
};
MP_HD void recover_pose_candidates(const double *E_in, RecoverCands &rc) {
    // canonical sign of E (largest-magnitude entry positive), as in the oracle
    double emax = E_in[0];
#pragma unroll
    for (int e = 1; e < 9; ++e)
        if (fabs(E_in[e]) > fabs(emax)) emax = E_in[e];
    double E[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) E[e] = emax < 0 ? -E_in[e] : E_in[e];
    double S[3][3], V[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) S[i][j] = E[i] * E[j] + E[3 + i] * E[3 + j] + E[6 + i] * E[6 + j];
    jacobi_eig3(S, V);
    // order eigenpairs by decreasing eigenvalue: indices i0, i1 of the two largest
    const double l0 = S[0][0], l1 = S[1][1], l2 = S[2][2];
    int i0 = 0, i1 = 1;
    if (l1 > l0 && l1 >= l2) {
        i0 = 1;
        i1 = (l0 >= l2) ? 0 : 2;
    } else if (l2 > l0 && l2 > l1) {
        i0 = 2;
        i1 = (l0 >= l1) ? 0 : 1;
    } else {
        i0 = 0;
        i1 = (l1 >= l2) ? 1 : 2;
    }
    // canonical reflection of (v1, v2): v3 = v1 x v2 with its largest-magnitude entry
    // positive (see oracle/src/pt67.cpp); u2 re-orthogonalised against u1
    double v[3][3], u[3][3];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int ik = k == 0 ? i0 : i1;
#pragma unroll
        for (int r = 0; r < 3; ++r) v[k][r] = (ik == 0) ? V[r][0] : ((ik == 1) ? V[r][1] : V[r][2]);
    }
    cross3(v[0], v[1], v[2]);
    {
        double vm = v[2][0];
#pragma unroll
        for (int r = 1; r < 3; ++r)
            if (fabs(v[2][r]) > fabs(vm)) vm = v[2][r];
        if (vm < 0) {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                v[1][r] = -v[1][r];
                v[2][r] = -v[2][r];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int r = 0; r < 3; ++r) u[k][r] = E[3 * r] * v[k][0] + E[3 * r + 1] * v[k][1] + E[3 * r + 2] * v[k][2];
    {
        const double n0 = 1.0 / sqrt(dot3(u[0], u[0]));
#pragma unroll
        for (int r = 0; r < 3; ++r) u[0][r] *= n0;
        const double d = dot3(u[0], u[1]);
#pragma unroll
        for (int r = 0; r < 3; ++r) u[1][r] -= d * u[0][r];
        const double n1 = 1.0 / sqrt(dot3(u[1], u[1]));
#pragma unroll
        for (int r = 0; r < 3; ++r) u[1][r] *= n1;
    }
    cross3(u[0], u[1], u[2]);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            rc.R1[3 * r + c] = -u[1][r] * v[0][c] + u[0][r] * v[1][c] + u[2][r] * v[2][c];
            rc.R2[3 * r + c] = u[1][r] * v[0][c] - u[0][r] * v[1][c] + u[2][r] * v[2][c];
        }
#pragma unroll
    for (int r = 0; r < 3; ++r) rc.u2[r] = u[2][r];
}

// cheirality of one point under candidate k (OpenCV: DLT triangulation, positive and
// finite depth in both views)
MP_HD bool recover_pose_good(const RecoverCands &rc, int k, const double *p0, const double *p1, double dist) {
    const double ts = (k < 2) ? 1.0 : -1.0;
    double P1[3][4];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) P1[r][c] = (k & 1) ? opaque(rc.R2[3 * r + c]) : opaque(rc.R1[3 * r + c]);
        P1[r][3] = ts * rc.u2[r];
    }
    double A[4][4];
    A[0][0] = -1.0;
    A[0][1] = 0.0;
    A[0][2] = p0[0];
    A[0][3] = 0.0;
    A[1][0] = 0.0;
    A[1][1] = -1.0;
    A[1][2] = p0[1];
    A[1][3] = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        A[2][j] = p1[0] * P1[2][j] - P1[0][j];
        A[3][j] = p1[1] * P1[2][j] - P1[1][j];
    }
    // one-sided Jacobi SVD (OpenCV's cv::SVD): for the wrong candidates the two
    // smallest singular values are often close, where inverse iteration (dlt_null4)
    // converges slowly and the cheirality signs rest on the SVD vector (the sweeps'
    // quotients and roots to about an ulp: smallest_right_sv4_fast)
    double Qh[4];
    smallest_right_sv4_fast(A, Qh);
    bool ok = Qh[2] * Qh[3] > 0;
    const double iq = svd_rcp(Qh[3]);
    const double X0 = Qh[0] * iq, X1 = Qh[1] * iq, X2 = Qh[2] * iq;
    ok = ok && X2 < dist;
    const double z1 = P1[2][0] * X0 + P1[2][1] * X1 + P1[2][2] * X2 + P1[2][3];
    return ok && z1 > 0 && z1 < dist;
}

// The same test for the two candidates (R, t) and (R, -t) of one rotation (kr = 0: R1,
// 1: R2) from one SVD.  Their DLT matrices differ by the sign of the last column (A' =
// A diag(1, 1, 1, -1)); every operation of the one-sided Jacobi is odd or even in that
// column's sign (rounding is sign-symmetric), so the sweeps on A' run the mirrored
// rotations of those on A and end at diag(1, 1, 1, -1) times A's vector, up to the
// overall sign: (Qh0, Qh1, Qh2, -Qh3) decides (R, -t) bit for bit as its own SVD would
// (the one exception, zeta == 0 exactly in a rotation, has measure zero).
MP_HD void recover_pose_good_pair(const RecoverCands &rc, int kr, const double *p0, const double *p1, double dist,
                                  bool *good_pos, bool *good_neg) {
    double P1[3][4];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) P1[r][c] = (kr & 1) ? opaque(rc.R2[3 * r + c]) : opaque(rc.R1[3 * r + c]);
        P1[r][3] = rc.u2[r];
    }
    double A[4][4];
    A[0][0] = -1.0;
    A[0][1] = 0.0;
    A[0][2] = p0[0];
    A[0][3] = 0.0;
    A[1][0] = 0.0;
    A[1][1] = -1.0;
    A[1][2] = p0[1];
    A[1][3] = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        A[2][j] = p1[0] * P1[2][j] - P1[0][j];
        A[3][j] = p1[1] * P1[2][j] - P1[1][j];
    }
    double Qh[4];
    smallest_right_sv4_fast(A, Qh);
    const double iq3 = svd_rcp(Qh[3]); // (odd: the two signs' quotients mirror exactly)
#pragma unroll
    for (int sgn = 0; sgn < 2; ++sgn) {
        const double q3 = sgn ? -Qh[3] : Qh[3], t2 = sgn ? -P1[2][3] : P1[2][3], iq = sgn ? -iq3 : iq3;
        bool ok = Qh[2] * q3 > 0;
        const double X0 = Qh[0] * iq, X1 = Qh[1] * iq, X2 = Qh[2] * iq;
        ok = ok && X2 < dist;
        const double z1 = P1[2][0] * X0 + P1[2][1] * X1 + P1[2][2] * X2 + t2;
        ok = ok && z1 > 0 && z1 < dist;
        if (sgn)
            *good_neg = ok;
        else
            *good_pos = ok;
    }
}

// the candidate with the most good points (ties: the first); returns its count
MP_HD int recover_pose_select(const RecoverCands &rc, const int (&good)[4], double *R, double *t) {
    int best = 3;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3])
        best = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3])
        best = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3])
        best = 2;
    const double ts = (best < 2) ? 1.0 : -1.0;
#pragma unroll
    for (int e = 0; e < 9; ++e) R[e] = (best & 1) ? opaque(rc.R2[e]) : opaque(rc.R1[e]); // (rc stays in registers)
#pragma unroll
    for (int r = 0; r < 3; ++r) t[r] = ts * rc.u2[r];
    return (best == 0) ? good[0] : ((best == 1) ? good[1] : ((best == 2) ? good[2] : good[3]));
}

// cv::recoverPose(E, p0, p1, I, R, t, dist); returns the good-point count of the pose
template <int K>
MP_HD int recover_pose_cv(const double *E_in, const double (&p0)[K][2], const double (&p1)[K][2], double dist,
                          double *R, double *t) {
    RecoverCands rc;
    recover_pose_candidates(E_in, rc);
    int good[4] = {0, 0, 0, 0};
#pragma unroll
    for (int kr = 0; kr < 2; ++kr)
        for (int i = 0; i < K; ++i) {
            bool gp, gn;
            recover_pose_good_pair(rc, kr, p0[i], p1[i], dist, &gp, &gn);
            good[kr] += gp ? 1 : 0;
            good[kr + 2] += gn ? 1 : 0;
        }
    return recover_pose_select(rc, good, R, t);
}

// ---------------------------------------------------------------------------
// 6-point shared focal
struct Cx {
    double r, i;
};
MP_HD Cx cmul(Cx a, Cx b) { return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
MP_HD Cx cadd(Cx a, Cx b) { return {a.r + b.r, a.i + b.i}; }
MP_HD Cx csub(Cx a, Cx b) { return {a.r - b.r, a.i - b.i}; }
MP_HD Cx cdiv(Cx a, Cx b) {
    const double d = b.r * b.r + b.i * b.i;
    return {(a.r * b.r + a.i * b.i) / d, (a.i * b.r - a.r * b.i) / d};
}

// monomials of (x, y) up to degree 3 in the order of v:
// x3 x2y xy2 y3 x2 xy y2 x y 1
struct Cub2 {
    double c[10];
};
struct Quad2 {
    double c[6]; // x2 xy y2 x y 1
};
struct Lin2 {
    double c[3]; // x y 1
};
MP_HD void lin2_mul(const Lin2 &a, const Lin2 &b, Quad2 &o) {
    o.c[0] = a.c[0] * b.c[0];
    o.c[1] = a.c[0] * b.c[1] + a.c[1] * b.c[0];
    o.c[2] = a.c[1] * b.c[1];
    o.c[3] = a.c[0] * b.c[2] + a.c[2] * b.c[0];
    o.c[4] = a.c[1] * b.c[2] + a.c[2] * b.c[1];
    o.c[5] = a.c[2] * b.c[2];
}
// o += s * q * l
MP_HD void quad2_lin_acc(const Quad2 &q, const Lin2 &l, double s, Cub2 &o) {
    const double x = l.c[0], y = l.c[1], one = l.c[2];
    o.c[0] += s * q.c[0] * x;                                   // x3
    o.c[1] += s * (q.c[0] * y + q.c[1] * x);                    // x2y
    o.c[2] += s * (q.c[1] * y + q.c[2] * x);                    // xy2
    o.c[3] += s * q.c[2] * y;                                   // y3
    o.c[4] += s * (q.c[0] * one + q.c[3] * x);                  // x2
    o.c[5] += s * (q.c[1] * one + q.c[3] * y + q.c[4] * x);     // xy
    o.c[6] += s * (q.c[2] * one + q.c[4] * y);                  // y2
    o.c[7] += s * (q.c[3] * one + q.c[5] * x);                  // x
    o.c[8] += s * (q.c[4] * one + q.c[5] * y);                  // y
    o.c[9] += s * q.c[5] * one;                                 // 1
}

MP_HD void mono2(double x, double y, double *v, double *dx, double *dy) {
    const double x2 = x * x, y2 = y * y;
    v[0] = x2 * x;
    v[1] = x2 * y;
    v[2] = x * y2;
    v[3] = y2 * y;
    v[4] = x2;
    v[5] = x * y;
    v[6] = y2;
    v[7] = x;
    v[8] = y;
    v[9] = 1.0;
    dx[0] = 3 * x2;
    dx[1] = 2 * x * y;
    dx[2] = y2;
    dx[3] = 0;
    dx[4] = 2 * x;
    dx[5] = y;
    dx[6] = 0;
    dx[7] = 1;
    dx[8] = 0;
    dx[9] = 0;
    dy[0] = 0;
    dy[1] = x2;
    dy[2] = 2 * x * y;
    dy[3] = 3 * y2;
    dy[4] = 0;
    dy[5] = x;
    dy[6] = 2 * y;
    dy[7] = 0;
    dy[8] = 1;
    dy[9] = 0;
}

// det of the complex 10x10 matrix u^2 M0 + u M1 + M2 (LU, partial pivoting)
MP_HD Cx det_pencil10(const double (&M)[3][10][10], Cx u) {
    const Cx u2 = cmul(u, u);
    Cx A[10][10];
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 10; ++c)
            A[r][c] = {u2.r * M[0][r][c] + u.r * M[1][r][c] + M[2][r][c], u2.i * M[0][r][c] + u.i * M[1][r][c]};
    Cx det = {1.0, 0.0};
    for (int k = 0; k < 10; ++k) {
        int p = k;
        double best = fabs(A[k][k].r) + fabs(A[k][k].i);
        for (int r = k + 1; r < 10; ++r) {
            const double v = fabs(A[r][k].r) + fabs(A[r][k].i);
            if (v > best) {
                best = v;
                p = r;
            }
        }
        if (best == 0.0) return {0.0, 0.0};
        if (p != k) {
            for (int c = k; c < 10; ++c) {
                const Cx tmp = A[k][c];
                A[k][c] = A[p][c];
                A[p][c] = tmp;
            }
            det.r = -det.r;
            det.i = -det.i;
        }
        det = cmul(det, A[k][k]);
        const Cx inv = cdiv({1.0, 0.0}, A[k][k]);
        for (int r = k + 1; r < 10; ++r) {
            const Cx l = cmul(A[r][k], inv);
            for (int c = k + 1; c < 10; ++c) A[r][c] = csub(A[r][c], cmul(l, A[k][c]));
        }
    }
    return det;
}

// q(u) = det(u^2 M0 + u M1 + M2) / u^5 (degree 15) by a 16-point DFT on |u| = rho
MP_HD void pencil_poly15(const double (&M)[3][10][10], double rho, double (&c)[16]) {
    Cx qv[9];
    for (int j = 0; j <= 8; ++j) {
        const double th = 2.0 * 3.14159265358979323846 * j / 16.0;
        const Cx u = {rho * cos(th), rho * sin(th)};
        const Cx d = det_pencil10(M, u);
        // divide by u^5
        const double r5 = rho * rho * rho * rho * rho;
        const Cx inv5 = {cos(5.0 * th) / r5, -sin(5.0 * th) / r5};
        qv[j] = cmul(d, inv5);
    }
    for (int k = 0; k < 16; ++k) {
        // sum over the 16 nodes using conjugate symmetry q(conj u) = conj q(u)
        double acc = 0.0;
        for (int j = 0; j < 16; ++j) {
            const int jj = (j <= 8) ? j : 16 - j;
            const Cx q = (j <= 8) ? qv[jj] : Cx{qv[jj].r, -qv[jj].i};
            const double th = -2.0 * 3.14159265358979323846 * j * k / 16.0;
            acc += q.r * cos(th) - q.i * sin(th);
        }
        c[k] = acc / 16.0 / pow(rho, (double)k);
    }
}

// real 10x10 null vector by Gaussian elimination with complete pivoting
MP_HD bool null_vector10(double (&A)[10][10], double (&v)[10]) {
    int perm[10];
    for (int i = 0; i < 10; ++i) perm[i] = i;
    for (int k = 0; k < 9; ++k) {
        int pr = k, pc = k;
        double best = 0.0;
        for (int r = k; r < 10; ++r)
            for (int c = k; c < 10; ++c)
                if (fabs(A[r][c]) > best) {
                    best = fabs(A[r][c]);
                    pr = r;
                    pc = c;
                }
        if (best == 0.0) return false;
        if (pr != k)
            for (int c = 0; c < 10; ++c) {
                const double tmp = A[k][c];
                A[k][c] = A[pr][c];
                A[pr][c] = tmp;
            }
        if (pc != k) {
            for (int r = 0; r < 10; ++r) {
                const double tmp = A[r][k];
                A[r][k] = A[r][pc];
                A[r][pc] = tmp;
            }
            const int tp = perm[k];
            perm[k] = perm[pc];
            perm[pc] = tp;
        }
        for (int r = k + 1; r < 10; ++r) {
            const double l = A[r][k] / A[k][k];
            for (int c = k + 1; c < 10; ++c) A[r][c] -= l * A[k][c];
            A[r][k] = 0.0;
        }
    }
    // free variable: the last (column perm[9]); back substitution for the rest
    double z[10];
    z[9] = 1.0;
    for (int k = 8; k >= 0; --k) {
        double s = 0.0;
        for (int c = k + 1; c < 10; ++c) s += A[k][c] * z[c];
        z[k] = -s / A[k][k];
    }
    for (int i = 0; i < 10; ++i) v[perm[i]] = z[i];
    return true;
}

// The ten equations of the 6-point system, one row at a time: emit(row, t0, t1, t2)
// receives the coefficients of w^0, w^1, w^2 of equation `row` (row 0: det F, which
// has no w terms: t1 = t2 = nullptr; rows 1 + 3r + c: the trace constraint entry
// (r, c)); columns are the monomials of v.  Rows are emitted in ascending order.
template <class Emit> MP_HD void sixpt_rows(const double (&N)[3][9], Emit &&emit) {
    Lin2 F[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        F[e].c[0] = N[0][e];
        F[e].c[1] = N[1][e];
        F[e].c[2] = N[2][e];
    }
    {
        // det F
        Cub2 det;
#pragma unroll
        for (int k = 0; k < 10; ++k) det.c[k] = 0.0;
        Quad2 qa, qb;
        lin2_mul(F[4], F[8], qa);
        lin2_mul(F[5], F[7], qb);
#pragma unroll
        for (int i = 0; i < 6; ++i) qa.c[i] -= qb.c[i];
        quad2_lin_acc(qa, F[0], 1.0, det);
        lin2_mul(F[3], F[8], qa);
        lin2_mul(F[5], F[6], qb);
#pragma unroll
        for (int i = 0; i < 6; ++i) qa.c[i] -= qb.c[i];
        quad2_lin_acc(qa, F[1], -1.0, det);
        lin2_mul(F[3], F[7], qa);
        lin2_mul(F[4], F[6], qb);
#pragma unroll
        for (int i = 0; i < 6; ++i) qa.c[i] -= qb.c[i];
        quad2_lin_acc(qa, F[2], 1.0, det);
        emit(0, det.c, (const double *)nullptr, (const double *)nullptr);
    }
    {
        // G = F D F^T = Ga + w Gb (symmetric; 6 entries each)
        Quad2 Ga[3][3], Gb[3][3];
        for (int r = 0; r < 3; ++r)
            for (int s = r; s < 3; ++s) {
                Quad2 t0, t1;
                lin2_mul(F[3 * r], F[3 * s], t0);
                lin2_mul(F[3 * r + 1], F[3 * s + 1], t1);
                for (int i = 0; i < 6; ++i) Ga[r][s].c[i] = t0.c[i] + t1.c[i];
                lin2_mul(F[3 * r + 2], F[3 * s + 2], Gb[r][s]);
                Ga[s][r] = Ga[r][s];
                Gb[s][r] = Gb[r][s];
            }
        Quad2 tr0, tr1;
        for (int i = 0; i < 6; ++i) {
            tr0.c[i] = Ga[0][0].c[i] + Ga[1][1].c[i];
            tr1.c[i] = Gb[0][0].c[i] + Gb[1][1].c[i] + Ga[2][2].c[i];
        }
        const Quad2 &tr2 = Gb[2][2];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                Cub2 T0, T1, T2;
                for (int k = 0; k < 10; ++k) T0.c[k] = T1.c[k] = T2.c[k] = 0.0;
                quad2_lin_acc(Ga[r][0], F[c], 2.0, T0);
                quad2_lin_acc(Ga[r][1], F[3 + c], 2.0, T0);
                quad2_lin_acc(tr0, F[3 * r + c], -1.0, T0);
                quad2_lin_acc(Gb[r][0], F[c], 2.0, T1);
                quad2_lin_acc(Gb[r][1], F[3 + c], 2.0, T1);
                quad2_lin_acc(Ga[r][2], F[6 + c], 2.0, T1);
                quad2_lin_acc(tr1, F[3 * r + c], -1.0, T1);
                quad2_lin_acc(Gb[r][2], F[6 + c], 2.0, T2);
                quad2_lin_acc(tr2, F[3 * r + c], -1.0, T2);
                emit(1 + 3 * r + c, T0.c, T1.c, T2.c);
            }
    }
}

// One row of the same system, for a caller that owns a single row (the group root
// kernel): F(e) returns entry e of F = x N0 + y N1 + N2 as a Lin2.  Only the entries
// of G that the row uses are formed, each with the operand order of sixpt_rows, and
// every accumulator receives its terms in the order of sixpt_rows.
template <class FGet>
MP_HD void sixpt_row(FGet &&F, int row, double (&t0)[10], double (&t1)[10], double (&t2)[10]) {
    Cub2 T0, T1, T2;
#pragma unroll
    for (int k = 0; k < 10; ++k) T0.c[k] = T1.c[k] = T2.c[k] = 0.0;
    if (row == 0) {
        Quad2 qa, qb;
        auto term = [&](int i0, int i1, int i2, int i3, int i4, double sgn) {
            lin2_mul(F(i1), F(i2), qa);
            lin2_mul(F(i3), F(i4), qb);
#pragma unroll
            for (int i = 0; i < 6; ++i) qa.c[i] -= qb.c[i];
            quad2_lin_acc(qa, F(i0), sgn, T0);
        };
        term(0, 4, 8, 5, 7, 1.0);
        term(1, 3, 8, 5, 6, -1.0);
        term(2, 3, 7, 4, 6, 1.0);
    } else {
        const int a = (row - 1) / 3, c = (row - 1) - 3 * ((row - 1) / 3);
        // G_xy = Ga_xy + w Gb_xy, formed as G_{min max}
        auto Gpair = [&](int x, int y, Quad2 &ga, Quad2 &gb) {
            const int lo = x < y ? x : y, hi = x < y ? y : x;
            Quad2 u0, u1;
            lin2_mul(F(3 * lo), F(3 * hi), u0);
            lin2_mul(F(3 * lo + 1), F(3 * hi + 1), u1);
#pragma unroll
            for (int i = 0; i < 6; ++i) ga.c[i] = u0.c[i] + u1.c[i];
            lin2_mul(F(3 * lo + 2), F(3 * hi + 2), gb);
        };
        Quad2 tr0, tr1, tr2;
        {
            Quad2 ga0, gb0, ga1, gb1, ga2;
            Gpair(0, 0, ga0, gb0);
            Gpair(1, 1, ga1, gb1);
            Gpair(2, 2, ga2, tr2);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                tr0.c[i] = ga0.c[i] + ga1.c[i];
                tr1.c[i] = gb0.c[i] + gb1.c[i] + ga2.c[i];
            }
        }
        const Lin2 Fac = F(3 * a + c);
        Quad2 ga, gb;
        Gpair(a, 0, ga, gb);
        quad2_lin_acc(ga, F(c), 2.0, T0);
        quad2_lin_acc(gb, F(c), 2.0, T1);
        Gpair(a, 1, ga, gb);
        quad2_lin_acc(ga, F(3 + c), 2.0, T0);
        quad2_lin_acc(gb, F(3 + c), 2.0, T1);
        quad2_lin_acc(tr0, Fac, -1.0, T0);
        Gpair(a, 2, ga, gb);
        quad2_lin_acc(ga, F(6 + c), 2.0, T1);
        quad2_lin_acc(gb, F(6 + c), 2.0, T2);
        quad2_lin_acc(tr1, Fac, -1.0, T1);
        quad2_lin_acc(tr2, Fac, -1.0, T2);
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        t0[k] = T0.c[k];
        t1[k] = T1.c[k];
        t2[k] = T2.c[k];
    }
}

// The whole system: M[a] holds the coefficients of w^a.
MP_HD void sixpt_matrices(const double (&N)[3][9], double (&M)[3][10][10]) {
    sixpt_rows(N, [&](int row, const double *t0, const double *t1, const double *t2) {
        for (int k = 0; k < 10; ++k) {
            M[0][row][k] = t0[k];
            M[1][row][k] = t1 ? t1[k] : 0.0;
            M[2][row][k] = t2 ? t2[k] : 0.0;
        }
    });
}

// Positive real roots u = 1/w of det(u^2 M0 + u M1 + M2) / u^5 (ascending).
MP_HD int sixpt_roots(const double (&M)[3][10][10], double (&roots)[15]) {
    // q(u): first pass on |u| = 1, then on the geometric mean of the root moduli
    double c[16];
    pencil_poly15(M, 1.0, c);
    double rho = 1.0;
    if (c[0] != 0.0 && c[15] != 0.0) {
        rho = pow(fabs(c[0] / c[15]), 1.0 / 15.0);
        if (!(rho > 0.0) || !(rho < 1e300)) rho = 1.0;
    }
    if (rho != 1.0) pencil_poly15(M, rho, c);
    double all[15];
    const int nr = sturm_real_roots<15>(c, all);
    int n = 0;
    for (int k = 0; k < nr; ++k)
        if (all[k] > 0.0) roots[n++] = all[k];
    return n;
}

// (x, y) from a null vector v of M(w), v ~ (x^3, x^2 y, x y^2, y^3, x^2, x y, y^2, x,
// y, 1): each coordinate from the ratio of monomials with the largest denominator
// (x = v7/v9 = v4/v7 = v0/v4 = v5/v8 = v2/v6, y = v8/v9 = v6/v8 = v3/v6 = v5/v7 =
// v1/v4).  v7/v9 alone loses the digits of a solution far from the origin (|x| ~ 1e2
// puts v9 ~ 1e-6 of |v|, below the elimination's absolute accuracy) and the polish
// then starts from a wrong point; the largest denominators are accurate relative to
// |v|.  For solutions near the origin the choice is v7/v9, v8/v9 as before.
MP_HD bool sixpt_xy_from_monomials(const double (&v)[10], double *x, double *y) {
    double nx = v[7], dx = v[9], ny = v[8], dy = v[9];
    if (fabs(v[7]) > fabs(dx)) { nx = v[4]; dx = v[7]; }
    if (fabs(v[4]) > fabs(dx)) { nx = v[0]; dx = v[4]; }
    if (fabs(v[8]) > fabs(dx)) { nx = v[5]; dx = v[8]; }
    if (fabs(v[6]) > fabs(dx)) { nx = v[2]; dx = v[6]; }
    if (fabs(v[8]) > fabs(dy)) { ny = v[6]; dy = v[8]; }
    if (fabs(v[6]) > fabs(dy)) { ny = v[3]; dy = v[6]; }
    if (fabs(v[7]) > fabs(dy)) { ny = v[5]; dy = v[7]; }
    if (fabs(v[4]) > fabs(dy)) { ny = v[1]; dy = v[4]; }
    if (dx == 0.0 || dy == 0.0) return false;
    *x = nx / dx;
    *y = ny / dy;
    return true;
}

// Poses of one root u: (x, y) from the null vector of M(w), Gauss-Newton polish of
// (x, y, w), E = K F K, motion_from_essential on the f-calibrated bearings.
MP_HD int sixpt_poses_for_root(const double (&M)[3][10][10], const double (&N)[3][9], double u,
                               const double (&x1)[6][3], const double (&x2)[6][3], Model *out, int nout, int kmax) {
    double w = 1.0 / u;
    double A[10][10];
    for (int r = 0; r < 10; ++r)
        for (int cc = 0; cc < 10; ++cc) A[r][cc] = M[0][r][cc] + w * (M[1][r][cc] + w * M[2][r][cc]);
    double v[10];
    if (!null_vector10(A, v)) return 0;
    double x, y;
    if (!sixpt_xy_from_monomials(v, &x, &y)) return 0;
    // Gauss-Newton polish of (x, y, w) on the ten equations
    for (int it = 0; it < 5; ++it) {
        double mv[10], dxv[10], dyv[10];
        mono2(x, y, mv, dxv, dyv);
        double JtJ[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, Jtr[3][1] = {{0}, {0}, {0}};
        for (int r = 0; r < 10; ++r) {
            double res = 0, jx = 0, jy = 0, jw = 0;
            for (int cc = 0; cc < 10; ++cc) {
                const double m = M[0][r][cc] + w * (M[1][r][cc] + w * M[2][r][cc]);
                res += m * mv[cc];
                jx += m * dxv[cc];
                jy += m * dyv[cc];
                jw += (M[1][r][cc] + 2.0 * w * M[2][r][cc]) * mv[cc];
            }
            const double J[3] = {jx, jy, jw};
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                Jtr[a][0] += J[a] * res;
#pragma unroll
                for (int b = 0; b < 3; ++b) JtJ[a][b] += J[a] * J[b];
            }
        }
        if (!gauss_solve<3, 1>(JtJ, Jtr)) break;
        x -= Jtr[0][0];
        y -= Jtr[1][0];
        w -= Jtr[2][0];
    }
    // a root of the interpolated q(u) that is not a root of the system leaves a
    // residual after the polish: the ten equations must vanish to 1e-8 of their scale
    {
        double mv[10], dxv[10], dyv[10];
        mono2(x, y, mv, dxv, dyv);
        double rr = 0, ss = 0;
        for (int r = 0; r < 10; ++r) {
            double res = 0, mag = 0;
            for (int cc = 0; cc < 10; ++cc) {
                const double t = (M[0][r][cc] + w * (M[1][r][cc] + w * M[2][r][cc])) * mv[cc];
                res += t;
                mag += fabs(t);
            }
            rr += res * res;
            ss += mag * mag;
        }
        if (!(rr <= 1e-16 * ss)) return 0;
    }
    if (!(w > 0.0)) return 0;
    const double foc = 1.0 / sqrt(w);
    double Fm[9], nn = 0.0;
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        Fm[e] = x * N[0][e] + y * N[1][e] + N[2][e];
        nn += Fm[e] * Fm[e];
    }
    nn = 1.0 / sqrt(nn);
    double E[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) E[3 * r + cc] = Fm[3 * r + cc] * nn * (r < 2 ? foc : 1.0) * (cc < 2 ? foc : 1.0);
    // K^-1 x, re-normalised: check_cheirality assumes unit bearings
    double c1[6][3], c2[6][3];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const double a[3] = {x1[i][0] / foc, x1[i][1] / foc, x1[i][2]}, b[3] = {x2[i][0] / foc, x2[i][1] / foc, x2[i][2]};
        const double na = 1.0 / sqrt(dot3(a, a)), nb = 1.0 / sqrt(dot3(b, b));
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            c1[i][q] = a[q] * na;
            c2[i][q] = b[q] * nb;
        }
    }
    const int added = motion_from_essential<6>(E, c1, c2, out, nout, kmax);
    for (int q = 0; q < added; ++q) out[nout + q].focal0 = out[nout + q].focal1 = foc;
    return added;
}

MP_HD int sixpt_poses_for_roots(const double (&M)[3][10][10], const double (&N)[3][9], const double *roots, int nr,
                                const double (&x1)[6][3], const double (&x2)[6][3], Model *out, int kmax);

// kStop < 4 truncates the solver after stage kStop (tools/solver_bench.hip timing).
template <int kStop = 4>
MP_HD int relpose_6pt_sf(const double (&x1)[6][3], const double (&x2)[6][3], Model *out, int kmax) {
    double Q[6][9], N[3][9];
    epipolar_rows<6>(x1, x2, Q);
    nullspace_kx9<6>(Q, N);
    double M[3][10][10];
    sixpt_matrices(N, M);
    if (kStop == 0) return (int)(M[1][3][4] > 0);
    double roots[15];
    const int nr = sixpt_roots(M, roots);
    if (kStop <= 2) return nr;
    return sixpt_poses_for_roots(M, N, roots, nr, x1, x2, out, kmax);
}

// Poses of the roots u of one sample (the stage after the root finder), duplicates
// dropped; N, M: the sample's null space and pencil.
MP_HD int sixpt_poses_for_roots(const double (&M)[3][10][10], const double (&N)[3][9], const double *roots, int nr,
                                const double (&x1)[6][3], const double (&x2)[6][3], Model *out, int kmax) {
    int nout = 0;
    for (int k = 0; k < nr; ++k) nout += sixpt_poses_for_root(M, N, roots[k], x1, x2, out, nout, kmax);
    // two roots that the polish took to the same solution give the same pose twice:
    // keep the first (as pt_compact_kernel does for the estimator's batches)
    int n = 0;
    for (int q = 0; q < nout; ++q) {
        bool dup = false;
        for (int p = 0; p < n && !dup; ++p) {
            bool same = fabs(out[p].focal0 - out[q].focal0) <= 1e-8 * fabs(out[q].focal0);
            for (int e = 0; e < 9 && same; ++e) same = fabs(out[p].R[e] - out[q].R[e]) <= 1e-6;
            for (int e = 0; e < 3 && same; ++e) same = fabs(out[p].t[e] - out[q].t[e]) <= 1e-6 * (1.0 + fabs(out[q].t[e]));
            dup = same;
        }
        if (!dup) out[n++] = out[q];
    }
    return n;
}

// Two-focal candidate of one fundamental matrix: Bougnoux focals, E = K1^T F K0,
// recoverPose on the normalized 2-D points (src/hybrid_pose_two_focal_estimator.cpp:118-146).
template <int K>
MP_HD void twofocal_pose_from_F(const double *F, const double (&p0)[K][2], const double (&p1)[K][2], Model &m) {
    double f0, f1;
    bougnoux_sq(F, &f0, &f1);
    f0 = sqrt(fabs(f0));
    f1 = sqrt(fabs(f1));
    double E[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) E[3 * r + c] = (r < 2 ? f1 : 1.0) * F[3 * r + c] * (c < 2 ? f0 : 1.0);
    recover_pose_cv<K>(E, p0, p1, 1e9, m.R, m.t);
    m.scale = 1.0;
    m.offset0 = m.offset1 = 0.0;
    m.focal0 = f0;
    m.focal1 = f1;
}

} // namespace mp
