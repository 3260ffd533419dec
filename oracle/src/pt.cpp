// ORACLE -- test infrastructure only.
//
// Point-based minimal solvers and geometry helpers, restated from the literature
// because PoseLib v2.0.4 / OpenCV are not vendored in the reference
// (CMakeLists.txt:25-37): parity for these is "unpinned" (see DESIGN.md).
//
//   relpose_5pt_action -- the 5-point problem of PoseLib relpose_5pt (called at
//                   src/hybrid_pose_estimator.cpp:134) by a different algorithm than the
//                   estimator's restatement (pt_poselib.cpp), kept as a cross-check.
//                   Stewenius' action-matrix form: 4-dim null space of the 5x9
//                   epipolar system, ten cubic constraints (det E = 0 and
//                   2 E E^T E - tr(E E^T) E = 0), Gauss-Jordan of the 10x20 template,
//                   10x10 action matrix for x, real eigenpairs, then
//                   motion_from_essential + cheirality on all five points.
//   motion_from_essential / check_cheirality -- src/solver.cpp:1188-1285 (copies of
//                   PoseLib's functions that the reference ships).
//   triangulate_point -- src/utils.h:24-38 (COLMAP DLT).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "la.h"
#include "oracle.h"

namespace oracle {

namespace {

// polynomials in (x,y,z) of total degree <= 3; coefficient index by exponents
struct P3 {
    double c[4][4][4];
    P3() { std::memset(c, 0, sizeof(c)); }
};

P3 pmul3(const P3 &a, const P3 &b) {
    P3 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j + i < 4; ++j)
            for (int k = 0; k + j + i < 4; ++k) {
                double av = a.c[i][j][k];
                if (av == 0.0) continue;
                for (int p = 0; p + i + j + k < 4; ++p)
                    for (int q = 0; q + p + i + j + k < 4; ++q)
                        for (int s = 0; s + q + p + i + j + k < 4; ++s) r.c[i + p][j + q][k + s] += av * b.c[p][q][s];
            }
    return r;
}
P3 psub3(const P3 &a, const P3 &b) {
    P3 r = a;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 4; ++k) r.c[i][j][k] -= b.c[i][j][k];
    return r;
}
void pacc(P3 &a, const P3 &b, double s) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 4; ++k) a.c[i][j][k] += s * b.c[i][j][k];
}

void cross3(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

} // namespace

void motion_from_essential(const double E[9], const double *x1, const double *x2, int np, std::vector<Model> *out) {
    // columns of E
    double c0[3] = {E[0], E[3], E[6]}, c1[3] = {E[1], E[4], E[7]}, c2[3] = {E[2], E[5], E[8]};
    double u12[3], u13[3], u23[3];
    cross3(c0, c1, u12);
    cross3(c0, c2, u13);
    cross3(c1, c2, u23);
    auto sq = [](const double *v) { return v[0] * v[0] + v[1] * v[1] + v[2] * v[2]; };
    double n12 = sq(u12), n13 = sq(u13), n23 = sq(u23);
    double UW[3][3]; // UW[col][row]
    const double *ec, *uu;
    double nn;
    if (n12 > n13) {
        if (n12 > n23) {
            ec = c0;
            uu = u12;
            nn = n12;
        } else {
            ec = c1;
            uu = u23;
            nn = n23;
        }
    } else {
        if (n13 > n23) {
            ec = c0;
            uu = u13;
            nn = n13;
        } else {
            ec = c1;
            uu = u23;
            nn = n23;
        }
    }
    double en = std::sqrt(sq(ec));
    for (int r = 0; r < 3; ++r) {
        UW[1][r] = ec[r] / en;
        UW[2][r] = uu[r] / std::sqrt(nn);
    }
    double tmp[3];
    cross3(UW[2], UW[1], tmp);
    for (int r = 0; r < 3; ++r) UW[0][r] = -tmp[r];
    double Vt[3][3];
    for (int j = 0; j < 3; ++j) {
        Vt[0][j] = UW[1][0] * E[j] + UW[1][1] * E[3 + j] + UW[1][2] * E[6 + j];
        Vt[1][j] = -(UW[0][0] * E[j] + UW[0][1] * E[3 + j] + UW[0][2] * E[6 + j]);
    }
    double n0 = std::sqrt(sq(Vt[0]));
    for (int j = 0; j < 3; ++j) Vt[0][j] /= n0;
    double d = Vt[0][0] * Vt[1][0] + Vt[0][1] * Vt[1][1] + Vt[0][2] * Vt[1][2];
    for (int j = 0; j < 3; ++j) Vt[1][j] -= d * Vt[0][j];
    double n1 = std::sqrt(sq(Vt[1]));
    for (int j = 0; j < 3; ++j) Vt[1][j] /= n1;
    cross3(Vt[0], Vt[1], Vt[2]);

    auto try_pose = [&](double sgn_rot, double sgn_t) {
        Model m;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                double s = 0;
                for (int k = 0; k < 3; ++k) s += (k < 2 ? sgn_rot : 1.0) * UW[k][r] * Vt[k][c];
                m.R[3 * r + c] = s;
            }
        for (int r = 0; r < 3; ++r) m.t[r] = sgn_t * UW[2][r];
        for (int i = 0; i < np; ++i)
            if (!check_cheirality(m.R, m.t, x1 + 3 * i, x2 + 3 * i, 0.0)) return;
        out->push_back(m);
    };
    try_pose(1.0, 1.0);
    try_pose(1.0, -1.0);
    try_pose(-1.0, -1.0);
    try_pose(-1.0, 1.0);
}

bool check_cheirality(const double R[9], const double t[3], const double x1[3], const double x2[3], double min_depth) {
    double Rx1[3];
    for (int r = 0; r < 3; ++r) Rx1[r] = R[3 * r] * x1[0] + R[3 * r + 1] * x1[1] + R[3 * r + 2] * x1[2];
    const double a = -(Rx1[0] * x2[0] + Rx1[1] * x2[1] + Rx1[2] * x2[2]);
    const double b1 = -(Rx1[0] * t[0] + Rx1[1] * t[1] + Rx1[2] * t[2]);
    const double b2 = x2[0] * t[0] + x2[1] * t[1] + x2[2] * t[2];
    const double l1 = b1 - a * b2;
    const double l2 = -a * b1 + b2;
    min_depth = min_depth * (1 - a * a);
    return l1 > min_depth && l2 > min_depth;
}

std::vector<Model> relpose_5pt_action(const double *x1, const double *x2) {
    std::vector<Model> out;
    // epipolar rows: x2^T E x1 = 0, E row-major
    Mat Q(9, 9);
    for (int i = 0; i < 5; ++i)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Q(i, 3 * r + c) = x2[3 * i + r] * x1[3 * i + c];
    Mat U, V;
    std::vector<double> sv;
    jacobi_svd(Q, &U, &sv, &V);
    // basis of the null space: last four right singular vectors
    P3 Ep[9];
    for (int e = 0; e < 9; ++e) {
        Ep[e].c[1][0][0] = V(e, 5);
        Ep[e].c[0][1][0] = V(e, 6);
        Ep[e].c[0][0][1] = V(e, 7);
        Ep[e].c[0][0][0] = V(e, 8);
    }
    // constraints
    std::vector<P3> eqs;
    {
        P3 det;
        pacc(det, pmul3(Ep[0], psub3(pmul3(Ep[4], Ep[8]), pmul3(Ep[5], Ep[7]))), 1.0);
        pacc(det, pmul3(Ep[1], psub3(pmul3(Ep[3], Ep[8]), pmul3(Ep[5], Ep[6]))), -1.0);
        pacc(det, pmul3(Ep[2], psub3(pmul3(Ep[3], Ep[7]), pmul3(Ep[4], Ep[6]))), 1.0);
        eqs.push_back(det);
    }
    P3 EEt[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            for (int k = 0; k < 3; ++k) pacc(EEt[3 * r + c], pmul3(Ep[3 * r + k], Ep[3 * c + k]), 1.0);
    P3 tr;
    pacc(tr, EEt[0], 1.0);
    pacc(tr, EEt[4], 1.0);
    pacc(tr, EEt[8], 1.0);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            P3 e;
            for (int k = 0; k < 3; ++k) pacc(e, pmul3(EEt[3 * r + k], Ep[3 * k + c]), 2.0);
            pacc(e, pmul3(tr, Ep[3 * r + c]), -1.0);
            eqs.push_back(e);
        }
    // monomial order: cubics then the quotient basis
    const int mon[20][3] = {{3, 0, 0}, {2, 1, 0}, {2, 0, 1}, {1, 2, 0}, {1, 1, 1}, {1, 0, 2}, {0, 3, 0},
                            {0, 2, 1}, {0, 1, 2}, {0, 0, 3}, {2, 0, 0}, {1, 1, 0}, {1, 0, 1}, {0, 2, 0},
                            {0, 1, 1}, {0, 0, 2}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {0, 0, 0}};
    Mat A(10, 10), Bm(10, 10), G;
    for (int r = 0; r < 10; ++r)
        for (int m = 0; m < 20; ++m) {
            double v = eqs[r].c[mon[m][0]][mon[m][1]][mon[m][2]];
            if (m < 10)
                A(r, m) = v;
            else
                Bm(r, m - 10) = v;
        }
    if (!lu_full_solve(A, Bm, &G)) return out; // cubic_r = -G[r] . basis
    Mat Mx(10, 10);
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 10; ++c) Mx(r, c) = -G(r, c);
    Mx(6, 0) = 1.0; // x*x  = x^2
    Mx(7, 1) = 1.0; // x*y  = xy
    Mx(8, 2) = 1.0; // x*z  = xz
    Mx(9, 6) = 1.0; // x*1  = x
    std::vector<double> wr, wi;
    if (!eig_real(Mx, &wr, &wi)) return out;
    struct Sol {
        double x, y, z;
    };
    std::vector<Sol> sols;
    for (int k = 0; k < 10; ++k) {
        if (wi[k] != 0.0) continue;
        Mat T = Mx;
        for (int i = 0; i < 10; ++i) T(i, i) -= wr[k];
        std::vector<double> b = null_vector(T);
        if (b[9] == 0.0) continue;
        sols.push_back({b[6] / b[9], b[7] / b[9], b[8] / b[9]});
    }
    for (const Sol &s : sols) {
        double E[9];
        for (int e = 0; e < 9; ++e) E[e] = s.x * V(e, 5) + s.y * V(e, 6) + s.z * V(e, 7) + V(e, 8);
        motion_from_essential(E, x1, x2, 5, &out);
    }
    return out;
}

namespace {
// Right singular vector of the smallest singular value of a 4 x 4 matrix by one-sided
// (Hestenes) cyclic Jacobi: at most 20 sweeps over (p, q), p < q, a rotation where the
// columns' relative correlation exceeds 1e-16, stop when none exceeds 1e-15; the column
// of the smallest norm (first minimum), picked by one-hot weights
void smallest_right_sv4(const double A0[4][4], double v[4]) {
    double A[4][4], V[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            A[i][j] = A0[i][j];
            V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 20; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < 4; ++i) {
                    al += A[i][p] * A[i][p];
                    be += A[i][q] * A[i][q];
                    ga += A[i][p] * A[i][q];
                }
                const double rel = (ga != 0.0) ? std::fabs(ga) / std::sqrt(al * be) : 0.0;
                off = std::fmax(off, rel);
                if (rel > 1e-16) {
                    const double zeta = (be - al) / (2.0 * ga);
                    const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                    const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
                    for (int i = 0; i < 4; ++i) {
                        const double ap = A[i][p], aq = A[i][q];
                        A[i][p] = c * ap - s * aq;
                        A[i][q] = s * ap + c * aq;
                        const double vp = V[i][p], vq = V[i][q];
                        V[i][p] = c * vp - s * vq;
                        V[i][q] = s * vp + c * vq;
                    }
                }
            }
        if (!(off > 1e-15)) break;
    }
    double nrm[4];
    for (int j = 0; j < 4; ++j) nrm[j] = A[0][j] * A[0][j] + A[1][j] * A[1][j] + A[2][j] * A[2][j] + A[3][j] * A[3][j];
    int k = 0;
    double best = nrm[0];
    for (int j = 1; j < 4; ++j)
        if (nrm[j] < best) {
            best = nrm[j];
            k = j;
        }
    double w[4];
    for (int j = 0; j < 4; ++j) w[j] = (k == j) ? 1.0 : 0.0;
    for (int i = 0; i < 4; ++i) v[i] = w[0] * V[i][0] + w[1] * V[i][1] + w[2] * V[i][2] + w[3] * V[i][3];
}

// The null vector of the 4 x 4 DLT matrix: Householder QR (A^T A = R^T R), then inverse
// iteration on R^T R by triangular solves from R^-1 e4 until two normalised iterates
// agree to 1e-14 (at most 16 steps), else the Jacobi sweeps above.  The device's
// dlt_null4 (madpose_amd/csrc/include/mp_math.h) performs these operations in this
// order without FMA contraction.
void dlt_null4(const double A[4][4], double v[4]) {
    double R[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) R[i][j] = A[i][j];
    for (int k = 0; k < 3; ++k) {
        double nn = 0.0;
        for (int i = k; i < 4; ++i) nn += R[i][k] * R[i][k];
        const double nrm = std::sqrt(nn);
        const double alpha = R[k][k] >= 0.0 ? -nrm : nrm;
        double h[4];
        for (int i = 0; i < 4; ++i) h[i] = i < k ? 0.0 : R[i][k];
        h[k] -= alpha;
        const double hh = nn - 2.0 * alpha * R[k][k] + alpha * alpha;
        const double f2 = hh > 0.0 ? 2.0 / hh : 0.0;
        for (int j = k; j < 4; ++j) {
            double sdot = 0.0;
            for (int i = k; i < 4; ++i) sdot += h[i] * R[i][j];
            const double f = sdot * f2;
            for (int i = k; i < 4; ++i) R[i][j] -= f * h[i];
        }
    }
    double big = 0.0;
    for (int i = 0; i < 4; ++i)
        for (int j = i; j < 4; ++j) big = std::fmax(big, std::fabs(R[i][j]));
    const double floor_ = big * 2.220446049250313e-16;
    double d[4];
    for (int i = 0; i < 4; ++i) {
        const double r = R[i][i];
        d[i] = 1.0 / (std::fabs(r) > floor_ ? r : (r < 0.0 ? -floor_ : floor_));
    }
    double x[4];
    x[3] = d[3];
    x[2] = -(R[2][3] * x[3]) * d[2];
    x[1] = -(R[1][2] * x[2] + R[1][3] * x[3]) * d[1];
    x[0] = -(R[0][1] * x[1] + R[0][2] * x[2] + R[0][3] * x[3]) * d[0];
    bool conv = false;
    for (int it = 0; it < 16 && !conv; ++it) {
        double mx = 0.0;
        for (int i = 0; i < 4; ++i) mx = std::fmax(mx, std::fabs(x[i]));
        const double sc = 1.0 / mx;
        for (int i = 0; i < 4; ++i) x[i] *= sc;
        double y[4], z[4];
        y[0] = x[0] * d[0];
        y[1] = (x[1] - R[0][1] * y[0]) * d[1];
        y[2] = (x[2] - R[0][2] * y[0] - R[1][2] * y[1]) * d[2];
        y[3] = (x[3] - R[0][3] * y[0] - R[1][3] * y[1] - R[2][3] * y[2]) * d[3];
        z[3] = y[3] * d[3];
        z[2] = (y[2] - R[2][3] * z[3]) * d[2];
        z[1] = (y[1] - R[1][2] * z[2] - R[1][3] * z[3]) * d[1];
        z[0] = (y[0] - R[0][1] * z[1] - R[0][2] * z[2] - R[0][3] * z[3]) * d[0];
        double mz = 0.0;
        for (int i = 0; i < 4; ++i) mz = std::fmax(mz, std::fabs(z[i]));
        const double rz = 1.0 / mz;
        double diff = 0.0;
        for (int i = 0; i < 4; ++i) {
            diff = std::fmax(diff, std::fabs(z[i] * rz - x[i]));
            x[i] = z[i];
        }
        conv = diff < 1e-14;
    }
    if (!conv) {
        smallest_right_sv4(A, v);
        return;
    }
    const double n = 1.0 / std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
    for (int i = 0; i < 4; ++i) v[i] = x[i] * n;
}
} // namespace

// COLMAP TriangulatePoint as the reference ships it (src/utils.h:24-38): the DLT matrix,
// its null vector dehomogenised.  The reference takes the null vector from Eigen's
// JacobiSVD (src/utils.h:34); this restatement takes it by Householder QR + inverse
// iteration (dlt_null4 above; the two agree to ~1e-12 -- Eigen is not vendored, so the
// reference's own bits are unpinned either way), because the device performs exactly
// this (a bitwise device restatement of Eigen's two-sided sweeps cost 19 -> 79 us per
// calibrated tail launch, profiles/r06/exact1).  The point solvers' depth tails.
void triangulate_point_qr(const double P0[12], const double P1[12], const double p0[2], const double p1[2],
                          double X[3]) {
    double A[4][4], v[4];
    for (int j = 0; j < 4; ++j) {
        A[0][j] = p0[0] * P0[8 + j] - P0[j];
        A[1][j] = p0[1] * P0[8 + j] - P0[4 + j];
        A[2][j] = p1[0] * P1[8 + j] - P1[j];
        A[3][j] = p1[1] * P1[8 + j] - P1[4 + j];
    }
    dlt_null4(A, v);
    for (int c = 0; c < 3; ++c) X[c] = v[c] / v[3];
}

// the same with the one-sided Jacobi SVD (la.cpp jacobi_svd): recover_pose's tests
void triangulate_point(const double P0[12], const double P1[12], const double p0[2], const double p1[2], double X[3]) {
    Mat A(4, 4);
    for (int j = 0; j < 4; ++j) {
        A(0, j) = p0[0] * P0[8 + j] - P0[j];
        A(1, j) = p0[1] * P0[8 + j] - P0[4 + j];
        A(2, j) = p1[0] * P1[8 + j] - P1[j];
        A(3, j) = p1[1] * P1[8 + j] - P1[4 + j];
    }
    Mat U, V;
    std::vector<double> sv;
    jacobi_svd(A, &U, &sv, &V);
    for (int c = 0; c < 3; ++c) X[c] = V(c, 3) / V(3, 3);
}

} // namespace oracle
