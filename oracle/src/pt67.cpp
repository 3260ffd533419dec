// ORACLE -- test infrastructure only.
//
// The uncalibrated point solvers of the shared-focal and two-focal estimators,
// restated from their published algorithms because neither PoseLib v2.0.4 nor
// OpenCV is vendored in the reference (parity "unpinned"):
//
//   relpose_7pt_svd  the 7-point problem of PoseLib relpose_7pt (called at
//                 src/hybrid_pose_two_focal_estimator.cpp:116) by other means than the
//                 estimator's restatement (pt_poselib.cpp), kept as a cross-check:
//                 2-dim null space of the 7x9 epipolar system, F(a) = a N0 + N1,
//                 real roots of the cubic det F(a) = 0, F normalised to unit norm.
//   bougnoux_focals  src/hybrid_pose_two_focal_estimator.cpp:11-32 (the formula is
//                 in the reference; epipoles from the SVD of F).
//   recover_pose  cv::recoverPose(E, p0, p1, I, R, t, 1e9) (:143): SVD
//                 decomposition R1 = U W V^T, R2 = U W^T V^T, t = u3 (OpenCV
//                 decomposeEssentialMat), DLT triangulation per candidate, a point
//                 is good when both depths are in (0, distanceThresh); the candidate
//                 with the most good points wins, ties in the order (R1,t) (R2,t)
//                 (R1,-t) (R2,-t).
//   relpose_6pt_shared_focal  PoseLib relpose_6pt_shared_focal (called at
//                 src/hybrid_pose_shared_focal_estimator.cpp:87): F = x N0 + y N1 + N2
//                 over the 3-dim null space, unknown w = 1/f^2.  The ten equations
//                 det F = 0 and 2 F D F^T D F - tr(F D F^T D) F = 0 (D = diag(1,1,w),
//                 i.e. the essential-matrix trace constraint on E = K F K) are linear
//                 in the ten monomials of (x, y) up to degree 3 with coefficients
//                 quadratic in w: (M0 + w M1 + w^2 M2) v = 0.  Written in u = 1/w this
//                 is a quadratic eigenvalue problem solved through its 20x20
//                 companion matrix; real u with w = 1/u > 0 are kept, (x, y) come from
//                 the null vector of M(w), and motion_from_essential with cheirality
//                 on the six f-calibrated bearings yields the poses.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "la.h"
#include "oracle.h"

namespace oracle {

namespace {

void mm3(const double *A, const double *B, double *C) {
    double T[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) T[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
    std::memcpy(C, T, sizeof(T));
}
void tr3(const double *A, double *T) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) T[3 * c + r] = A[3 * r + c];
}
void cross3v(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
void skew(const double *e, double *S) {
    const double v[9] = {0, -e[2], e[1], e[2], 0, -e[0], -e[1], e[0], 0};
    std::memcpy(S, v, sizeof(v));
}

// null space basis (last k right singular vectors) of the rows x2^T (.) x1 = 0
Mat epipolar_nullspace(const double *x1, const double *x2, int np) {
    Mat A(9, 9);
    for (int i = 0; i < np; ++i)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) A(i, 3 * r + c) = x2[3 * i + r] * x1[3 * i + c];
    Mat U, V;
    std::vector<double> s;
    jacobi_svd(A, &U, &s, &V);
    return V;
}

// polynomials in (x, y) of total degree <= 3: c[i][j] multiplies x^i y^j
struct Q2 {
    double c[4][4];
    Q2() { std::memset(c, 0, sizeof(c)); }
};
Q2 qmul(const Q2 &a, const Q2 &b) {
    Q2 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; i + j < 4; ++j) {
            if (a.c[i][j] == 0.0) continue;
            for (int p = 0; i + j + p < 4; ++p)
                for (int q = 0; i + j + p + q < 4; ++q) r.c[i + p][j + q] += a.c[i][j] * b.c[p][q];
        }
    return r;
}
Q2 qadd(const Q2 &a, const Q2 &b, double s = 1.0) {
    Q2 r = a;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.c[i][j] += s * b.c[i][j];
    return r;
}
// monomial order of the unknown vector v
const int kMono[10][2] = {{3, 0}, {2, 1}, {1, 2}, {0, 3}, {2, 0}, {1, 1}, {0, 2}, {1, 0}, {0, 1}, {0, 0}};

} // namespace

std::vector<std::array<double, 9>> relpose_7pt_svd(const double *x1, const double *x2) {
    Mat V = epipolar_nullspace(x1, x2, 7);
    double N0[9], N1[9];
    for (int e = 0; e < 9; ++e) {
        N0[e] = V(e, 7);
        N1[e] = V(e, 8);
    }
    auto detF = [&](double a) {
        double F[9];
        for (int e = 0; e < 9; ++e) F[e] = a * N0[e] + N1[e];
        return det3(F);
    };
    // exact cubic through four samples
    const double p0 = detF(0.0), p1 = detF(1.0), pm = detF(-1.0), p2 = detF(2.0);
    const double c0 = p0, c2 = 0.5 * (p1 + pm) - p0, s = 0.5 * (p1 - pm);
    const double u = p2 - 4.0 * c2 - c0;
    const double c3 = (u - 2.0 * s) / 6.0, c1 = s - c3;
    std::vector<std::array<double, 9>> out;
    for (double a : poly_real_roots({c0, c1, c2, c3})) {
        std::array<double, 9> F;
        double nn = 0;
        for (int e = 0; e < 9; ++e) {
            F[e] = a * N0[e] + N1[e];
            nn += F[e] * F[e];
        }
        nn = std::sqrt(nn);
        for (int e = 0; e < 9; ++e) F[e] /= nn;
        out.push_back(F);
    }
    return out;
}

void bougnoux_focals(const double F[9], double *f0_sq, double *f1_sq) {
    Mat A(3, 3), At(3, 3);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            A(r, c) = F[3 * r + c];
            At(c, r) = F[3 * r + c];
        }
    Mat U, V, U2, V2;
    std::vector<double> s, s2;
    jacobi_svd(A, &U, &s, &V);
    jacobi_svd(At, &U2, &s2, &V2); // V2 = left singular vectors of F
    double e1[3] = {V(0, 2), V(1, 2), V(2, 2)}, e2[3] = {V2(0, 2), V2(1, 2), V2(2, 2)};
    for (int k = 0; k < 3; ++k) {
        e1[k] /= V(2, 2);
        e2[k] /= V2(2, 2);
    }
    double Se1[9], Se2[9], Ft[9];
    skew(e1, Se1);
    skew(e2, Se2);
    tr3(F, Ft);
    const double II[9] = {1, 0, 0, 0, 1, 0, 0, 0, 0};
    const double PP[9] = {0, 0, 0, 0, 0, 0, 0, 0, 1}; // p p^T with p = (0, 0, 1)
    double L[9], T1[9], T2[9];
    // f1 = -(p2^T [e2]x II F (p1 p1^T) F^T p2) / (p2^T [e2]x II F II F^T p2)
    mm3(Se2, II, L);
    mm3(L, F, L);
    mm3(L, PP, T1);
    mm3(T1, Ft, T1);
    mm3(L, II, T2);
    mm3(T2, Ft, T2);
    *f0_sq = -T1[8] / T2[8];
    // f2 = -(p1^T [e1]x II F^T (p2 p2^T) F p1) / (p1^T [e1]x II F^T II F p1)
    mm3(Se1, II, L);
    mm3(L, Ft, L);
    mm3(L, PP, T1);
    mm3(T1, F, T1);
    mm3(L, II, T2);
    mm3(T2, F, T2);
    *f1_sq = -T1[8] / T2[8];
}

int recover_pose(const double E_in[9], const double *p0, const double *p1, int n, double dist_thresh, double R[9],
                 double t[3]) {
    // The sign of E (inherited from the arbitrary sign of F) only relabels the four
    // candidates; it is fixed canonically (largest-magnitude entry positive).
    double E[9];
    int emax = 0;
    for (int e = 1; e < 9; ++e)
        if (std::fabs(E_in[e]) > std::fabs(E_in[emax])) emax = e;
    for (int e = 0; e < 9; ++e) E[e] = E_in[emax] < 0 ? -E_in[e] : E_in[e];
    Mat A(3, 3);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) A(r, c) = E[3 * r + c];
    Mat U, V;
    std::vector<double> s;
    jacobi_svd(A, &U, &s, &V);
    // OpenCV's SVD sign conventions are not reproducible without its source, and
    // with Bougnoux focals E has two equal singular values, so (v1, v2) is only
    // defined up to an in-plane rotation -- which leaves R1, R2 and u3 unchanged --
    // and a reflection, which relabels the candidates.  The reflection is fixed
    // canonically: v3 = v1 x v2 with its largest-magnitude entry positive (v2 is
    // flipped otherwise); u_k = E v_k / |E v_k|, u2 re-orthogonalised, u3 = u1 x u2.
    double v[3][3], u[3][3];
    for (int k = 0; k < 2; ++k)
        for (int r = 0; r < 3; ++r) v[k][r] = V(r, k);
    cross3v(v[0], v[1], v[2]);
    {
        int im = 0;
        for (int r = 1; r < 3; ++r)
            if (std::fabs(v[2][r]) > std::fabs(v[2][im])) im = r;
        if (v[2][im] < 0)
            for (int r = 0; r < 3; ++r) {
                v[1][r] = -v[1][r];
                v[2][r] = -v[2][r];
            }
    }
    for (int k = 0; k < 2; ++k)
        for (int r = 0; r < 3; ++r) u[k][r] = E[3 * r] * v[k][0] + E[3 * r + 1] * v[k][1] + E[3 * r + 2] * v[k][2];
    {
        double n0 = std::sqrt(u[0][0] * u[0][0] + u[0][1] * u[0][1] + u[0][2] * u[0][2]);
        for (int r = 0; r < 3; ++r) u[0][r] /= n0;
        const double d = u[0][0] * u[1][0] + u[0][1] * u[1][1] + u[0][2] * u[1][2];
        for (int r = 0; r < 3; ++r) u[1][r] -= d * u[0][r];
        double n1 = std::sqrt(u[1][0] * u[1][0] + u[1][1] * u[1][1] + u[1][2] * u[1][2]);
        for (int r = 0; r < 3; ++r) u[1][r] /= n1;
    }
    cross3v(u[0], u[1], u[2]);
    double Um[9], Vt[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            Um[3 * r + c] = u[c][r];
            Vt[3 * r + c] = v[r][c];
        }
    const double W[9] = {0, 1, 0, -1, 0, 0, 0, 0, 1}, Wt[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    double R1[9], R2[9];
    mm3(Um, W, R1);
    mm3(R1, Vt, R1);
    mm3(Um, Wt, R2);
    mm3(R2, Vt, R2);
    const double tu[3] = {Um[2], Um[5], Um[8]};
    const double *Rc[4] = {R1, R2, R1, R2};
    const double ts[4] = {1.0, 1.0, -1.0, -1.0};
    int good[4] = {0, 0, 0, 0};
    for (int k = 0; k < 4; ++k) {
        double P1[12];
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) P1[4 * r + c] = Rc[k][3 * r + c];
            P1[4 * r + 3] = ts[k] * tu[r];
        }
        const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        for (int i = 0; i < n; ++i) {
            // cv::triangulatePoints: homogeneous DLT, smallest right singular vector
            Mat M(4, 4);
            for (int j = 0; j < 4; ++j) {
                M(0, j) = p0[2 * i] * P0[8 + j] - P0[j];
                M(1, j) = p0[2 * i + 1] * P0[8 + j] - P0[4 + j];
                M(2, j) = p1[2 * i] * P1[8 + j] - P1[j];
                M(3, j) = p1[2 * i + 1] * P1[8 + j] - P1[4 + j];
            }
            Mat Um2, Vm2;
            std::vector<double> sm;
            jacobi_svd(M, &Um2, &sm, &Vm2);
            double Q[4] = {Vm2(0, 3), Vm2(1, 3), Vm2(2, 3), Vm2(3, 3)};
            bool ok = Q[2] * Q[3] > 0;
            for (int c = 0; c < 3; ++c) Q[c] /= Q[3];
            ok = ok && Q[2] < dist_thresh;
            const double z1 = P1[8] * Q[0] + P1[9] * Q[1] + P1[10] * Q[2] + P1[11];
            ok = ok && z1 > 0 && z1 < dist_thresh;
            good[k] += ok ? 1 : 0;
        }
    }
    int best = 3;
    if (good[0] >= good[1] && good[0] >= good[2] && good[0] >= good[3])
        best = 0;
    else if (good[1] >= good[0] && good[1] >= good[2] && good[1] >= good[3])
        best = 1;
    else if (good[2] >= good[0] && good[2] >= good[1] && good[2] >= good[3])
        best = 2;
    std::memcpy(R, Rc[best], sizeof(double) * 9);
    for (int r = 0; r < 3; ++r) t[r] = ts[best] * tu[r];
    return good[best];
}

// Positive real roots u = 1/w of det(u^2 M0 + u M1 + M2) / u^5, in eigen-solver
// order.  The companion C on z = [v; u v] (20 x 20) carries a structural 5-fold
// zero eigenvalue: the right null space of M2 (rank 6 -- row 0 is zero and every
// other row is F_22 times a quadratic in (x, y)) and one Jordan vector [a; v] with v
// in null(M2), M1 v in range(M2) and M2 a = -M1 v.  Rounding splits that eigenvalue
// into a cluster reaching ~1e-4 of the largest root (measured over 6000 random
// samples), where genuine roots also occur (down to ~5e-5 of it); no threshold
// separates the two.  So the 5-dimensional invariant subspace is deflated exactly
// (orthogonal similarity by the Householder reflectors of its basis) and the 15
// remaining eigenvalues -- the roots of the degree-15 q(u) -- are computed alone.
std::vector<double> sixpt_roots(const Mat &M0, const Mat &M1, const Mat &M2) {
    std::vector<double> out;
    Mat B(10, 20), X;
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 10; ++c) {
            B(r, c) = M2(r, c);
            B(r, 10 + c) = M1(r, c);
        }
    if (!lu_full_solve(M0, B, &X)) return out;
    Mat C(20, 20);
    for (int i = 0; i < 10; ++i) C(i, 10 + i) = 1.0;
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 20; ++c) C(10 + r, c) = -X(r, c);
    const Mat Nr = right_null_rank(M2, 6);            // 10 x 4
    const Mat Nl = right_null_rank(transpose(M2), 6); // left null vectors as columns
    const Mat S = matmul(matmul(transpose(Nl), M1), Nr);
    const Mat cv = right_null_rank(S, 3);
    std::vector<double> v(10, 0.0), rhs(10, 0.0);
    for (int i = 0; i < 10; ++i)
        for (int f = 0; f < 4; ++f) v[i] += Nr(i, f) * cv(f, 0);
    for (int i = 0; i < 10; ++i) {
        double s = 0.0;
        for (int c = 0; c < 10; ++c) s += M1(i, c) * v[c];
        rhs[i] = -s;
    }
    const std::vector<double> a = particular_solution(M2, rhs, 6);
    Mat Z(20, 5);
    for (int i = 0; i < 10; ++i) {
        for (int f = 0; f < 4; ++f) Z(i, f) = Nr(i, f);
        Z(i, 4) = a[i];
        Z(10 + i, 4) = v[i];
    }
    householder_deflate(C, Z);
    Mat D(15, 15);
    for (int r = 0; r < 15; ++r)
        for (int c = 0; c < 15; ++c) D(r, c) = C(5 + r, 5 + c);
    std::vector<double> wr, wi;
    if (!eig_real(D, &wr, &wi)) return out;
    for (int k = 0; k < 15; ++k)
        if (wi[k] == 0.0 && wr[k] > 0.0) out.push_back(wr[k]);
    return out;
}

// The ten equations of the 6-point system as (M0 + w M1 + w^2 M2) v = 0 over the
// monomials of (x, y) (V: the epipolar null space, F = x V6 + y V7 + V8).
void sixpt_pencil(const double *x1, const double *x2, Mat *Vout, Mat *M0out, Mat *M1out, Mat *M2out) {
    Mat V = epipolar_nullspace(x1, x2, 6);
    Q2 F[9];
    for (int e = 0; e < 9; ++e) {
        F[e].c[1][0] = V(e, 6);
        F[e].c[0][1] = V(e, 7);
        F[e].c[0][0] = V(e, 8);
    }
    auto f = [&](int r, int c) -> const Q2 & { return F[3 * r + c]; };
    // det F
    Q2 det;
    det = qadd(det, qmul(f(0, 0), qadd(qmul(f(1, 1), f(2, 2)), qmul(f(1, 2), f(2, 1)), -1.0)));
    det = qadd(det, qmul(f(0, 1), qadd(qmul(f(1, 0), f(2, 2)), qmul(f(1, 2), f(2, 0)), -1.0)), -1.0);
    det = qadd(det, qmul(f(0, 2), qadd(qmul(f(1, 0), f(2, 1)), qmul(f(1, 1), f(2, 0)), -1.0)));
    // G = F D F^T = Ga + w Gb
    Q2 Ga[3][3], Gb[3][3];
    for (int r = 0; r < 3; ++r)
        for (int s = 0; s < 3; ++s) {
            Ga[r][s] = qadd(qmul(f(r, 0), f(s, 0)), qmul(f(r, 1), f(s, 1)));
            Gb[r][s] = qmul(f(r, 2), f(s, 2));
        }
    const Q2 tr0 = qadd(Ga[0][0], Ga[1][1]);
    const Q2 tr1 = qadd(qadd(Gb[0][0], Gb[1][1]), Ga[2][2]);
    const Q2 tr2 = Gb[2][2];
    Mat M0(10, 10), M1(10, 10), M2(10, 10);
    for (int k = 0; k < 10; ++k) M0(0, k) = det.c[kMono[k][0]][kMono[k][1]];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            Q2 T0 = qadd(qmul(Ga[r][0], f(0, c)), qmul(Ga[r][1], f(1, c)));
            T0 = qadd(qadd(T0, T0), qmul(tr0, f(r, c)), -1.0);
            Q2 T1 = qadd(qadd(qmul(Gb[r][0], f(0, c)), qmul(Gb[r][1], f(1, c))), qmul(Ga[r][2], f(2, c)));
            T1 = qadd(qadd(T1, T1), qmul(tr1, f(r, c)), -1.0);
            Q2 T2 = qmul(Gb[r][2], f(2, c));
            T2 = qadd(qadd(T2, T2), qmul(tr2, f(r, c)), -1.0);
            const int row = 1 + 3 * r + c;
            for (int k = 0; k < 10; ++k) {
                M0(row, k) = T0.c[kMono[k][0]][kMono[k][1]];
                M1(row, k) = T1.c[kMono[k][0]][kMono[k][1]];
                M2(row, k) = T2.c[kMono[k][0]][kMono[k][1]];
            }
        }
    *Vout = V;
    *M0out = M0;
    *M1out = M1;
    *M2out = M2;
}

std::vector<double> sixpt_roots_of(const double *x1, const double *x2) {
    Mat V, M0, M1, M2;
    sixpt_pencil(x1, x2, &V, &M0, &M1, &M2);
    return sixpt_roots(M0, M1, M2);
}

std::vector<Model> relpose_6pt_shared_focal(const double *x1, const double *x2) {
    std::vector<Model> out;
    Mat V, M0, M1, M2;
    sixpt_pencil(x1, x2, &V, &M0, &M1, &M2);
    for (const double uu : sixpt_roots(M0, M1, M2)) {
        double w = 1.0 / uu;
        Mat Mw(10, 10);
        for (int r = 0; r < 10; ++r)
            for (int c = 0; c < 10; ++c) Mw(r, c) = M0(r, c) + w * (M1(r, c) + w * M2(r, c));
        std::vector<double> v = null_vector(Mw);
        // (x, y) from the monomial ratio with the largest denominator (v ~ x^3, x^2 y,
        // x y^2, y^3, x^2, x y, y^2, x, y, 1): v7/v9 alone loses the digits of a
        // solution far from the origin, whose v9 is tiny next to |v|
        const int xr[5][2] = {{7, 9}, {4, 7}, {0, 4}, {5, 8}, {2, 6}};
        const int yr[5][2] = {{8, 9}, {6, 8}, {3, 6}, {5, 7}, {1, 4}};
        int bx = 0, by = 0;
        for (int k = 1; k < 5; ++k) {
            if (std::fabs(v[xr[k][1]]) > std::fabs(v[xr[bx][1]])) bx = k;
            if (std::fabs(v[yr[k][1]]) > std::fabs(v[yr[by][1]])) by = k;
        }
        if (v[xr[bx][1]] == 0.0 || v[yr[by][1]] == 0.0) continue;
        double x = v[xr[bx][0]] / v[xr[bx][1]], y = v[yr[by][0]] / v[yr[by][1]];
        // Gauss-Newton polish of (x, y, w) on the ten equations
        for (int it = 0; it < 5; ++it) {
            double mv[10], dx[10], dy[10];
            for (int q = 0; q < 10; ++q) {
                const int i = kMono[q][0], j = kMono[q][1];
                mv[q] = std::pow(x, i) * std::pow(y, j);
                dx[q] = i ? i * std::pow(x, i - 1) * std::pow(y, j) : 0.0;
                dy[q] = j ? j * std::pow(x, i) * std::pow(y, j - 1) : 0.0;
            }
            double JtJ[3][3] = {{0}}, Jtr[3] = {0};
            for (int r = 0; r < 10; ++r) {
                double res = 0, jx = 0, jy = 0, jw = 0;
                for (int c = 0; c < 10; ++c) {
                    const double m = M0(r, c) + w * (M1(r, c) + w * M2(r, c));
                    res += m * mv[c];
                    jx += m * dx[c];
                    jy += m * dy[c];
                    jw += (M1(r, c) + 2.0 * w * M2(r, c)) * mv[c];
                }
                const double J[3] = {jx, jy, jw};
                for (int a = 0; a < 3; ++a) {
                    Jtr[a] += J[a] * res;
                    for (int b = 0; b < 3; ++b) JtJ[a][b] += J[a] * J[b];
                }
            }
            Mat Am(3, 3), Bm(3, 1), Xm;
            for (int a = 0; a < 3; ++a) {
                Bm(a, 0) = Jtr[a];
                for (int b = 0; b < 3; ++b) Am(a, b) = JtJ[a][b];
            }
            if (!lu_full_solve(Am, Bm, &Xm)) break;
            x -= Xm(0, 0);
            y -= Xm(1, 0);
            w -= Xm(2, 0);
        }
        if (!(w > 0.0)) continue;
        const double foc = 1.0 / std::sqrt(w);
        double Fm[9], nn = 0.0;
        for (int e = 0; e < 9; ++e) {
            Fm[e] = x * V(e, 6) + y * V(e, 7) + V(e, 8);
            nn += Fm[e] * Fm[e];
        }
        nn = std::sqrt(nn);
        double E[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                E[3 * r + c] = Fm[3 * r + c] / nn * (r < 2 ? foc : 1.0) * (c < 2 ? foc : 1.0);
        std::vector<double> c1(18), c2(18);
        // K^-1 x, re-normalised: check_cheirality assumes unit bearings
        for (int i = 0; i < 6; ++i) {
            double n1 = 0.0, n2 = 0.0;
            for (int c = 0; c < 3; ++c) {
                c1[3 * i + c] = x1[3 * i + c] / (c < 2 ? foc : 1.0);
                c2[3 * i + c] = x2[3 * i + c] / (c < 2 ? foc : 1.0);
                n1 += c1[3 * i + c] * c1[3 * i + c];
                n2 += c2[3 * i + c] * c2[3 * i + c];
            }
            n1 = std::sqrt(n1);
            n2 = std::sqrt(n2);
            for (int c = 0; c < 3; ++c) {
                c1[3 * i + c] /= n1;
                c2[3 * i + c] /= n2;
            }
        }
        std::vector<Model> poses;
        motion_from_essential(E, c1.data(), c2.data(), 6, &poses);
        for (Model m : poses) {
            m.focal0 = m.focal1 = foc;
            out.push_back(m);
        }
    }
    return out;
}

} // namespace oracle
