// ORACLE -- test infrastructure only.
//
// The option-gated alternative MD minimal solvers (HybridLORansacOptions::use_ours /
// use_4p4d; gates at src/hybrid_pose_estimator.cpp:75-78,
// src/hybrid_pose_shared_focal_estimator.cpp:62-65,
// src/hybrid_pose_two_focal_estimator.cpp:87-94), restated from src/solver.cpp:
//
//   md_pose_cal_ours   solve_scale_shift_pose_ours (:623-680) + solver_p3p_mono_3d
//                      (:536-621).  Distances between the three lifted points are
//                      preserved: |(d_i+u)x_i - (d_j+u)x_j|^2 = S |(e_i+v)y_i - (e_j+v)y_j|^2
//                      for the pairs (0,1) (0,2) (1,2), S = s^2.  Linear in
//                      (S v^2, S v, S) given u; (S v)^2 = (S v^2) S gives a quartic in u,
//                      solved as the eigenvalues of its companion matrix (|imag| <= 1e-8
//                      accepted); S >= 0.01 kept.  The reference writes the kept
//                      roots into column `ii` of an uninitialised matrix and then keeps
//                      the first `m` columns; columns never written are undefined there
//                      and are dropped here.
//   md_pose_sf_ours    solve_scale_shift_pose_shared_focal_ours (:818-984): three
//                      points, unknown depth of the third point in image 1; 3x3 LU,
//                      4x4 eigenproblem (|imag| <= 1e-3, real >= 0), 2x2 LU, focal and
//                      scale filters, rotation Y X^-1 from two difference vectors.
//   md_pose_tf_ours    solve_scale_shift_pose_two_focal_ours (:1045-1148): one 3x3 LU.
//   md_pose_tf_4p4d    solve_scale_shift_pose_two_focal_4p4d (:1287-1406): 11x11 LU
//                      for F, focals_from_fundamental (:1150-1177), motion_from_essential
//                      (:1219-1285) on the normalized homogeneous points.
// Inputs as md_pose(): x, y = homogeneous points (point-major), dx, dy = depths.
#include <cmath>
#include <cstring>

#include "la.h"
#include "oracle.h"

namespace oracle {

namespace {

void cross(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
double dot(const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// 3x3 inverse by cofactors (Eigen's closed form for 3x3)
bool inv3(const double *M, double *I) {
    const double c00 = M[4] * M[8] - M[5] * M[7], c01 = M[5] * M[6] - M[3] * M[8], c02 = M[3] * M[7] - M[4] * M[6];
    const double det = M[0] * c00 + M[1] * c01 + M[2] * c02;
    I[0] = c00 / det;
    I[1] = (M[2] * M[7] - M[1] * M[8]) / det;
    I[2] = (M[1] * M[5] - M[2] * M[4]) / det;
    I[3] = c01 / det;
    I[4] = (M[0] * M[8] - M[2] * M[6]) / det;
    I[5] = (M[2] * M[3] - M[0] * M[5]) / det;
    I[6] = c02 / det;
    I[7] = (M[1] * M[6] - M[0] * M[7]) / det;
    I[8] = (M[0] * M[4] - M[1] * M[3]) / det;
    return det != 0.0;
}

// R = [v1 v2 v1xv2] [u1 u2 u1xu2]^-1 (columns); not re-orthonormalised
void rot_from_differences(const double *u1, const double *u2, const double *v1, const double *v2, double *R) {
    double u3[3], v3[3], X[9], Xi[9], Y[9];
    cross(u1, u2, u3);
    cross(v1, v2, v3);
    for (int r = 0; r < 3; ++r) {
        X[3 * r] = u1[r];
        X[3 * r + 1] = u2[r];
        X[3 * r + 2] = u3[r];
        Y[3 * r] = v1[r];
        Y[3 * r + 1] = v2[r];
        Y[3 * r + 2] = v3[r];
    }
    inv3(X, Xi);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R[3 * r + c] = Y[3 * r] * Xi[c] + Y[3 * r + 1] * Xi[3 + c] + Y[3 * r + 2] * Xi[6 + c];
}

// partial-pivot LU solve of an n x n system with m right-hand sides (Eigen partialPivLu)
Mat pplu_solve(Mat A, Mat B) {
    const int n = A.r;
    for (int k = 0; k < n; ++k) {
        int p = k;
        for (int r = k + 1; r < n; ++r)
            if (std::fabs(A(r, k)) > std::fabs(A(p, k))) p = r;
        if (p != k) {
            for (int c = 0; c < n; ++c) std::swap(A(k, c), A(p, c));
            for (int c = 0; c < B.c; ++c) std::swap(B(k, c), B(p, c));
        }
        for (int r = k + 1; r < n; ++r) {
            const double l = A(r, k) / A(k, k);
            for (int c = k + 1; c < n; ++c) A(r, c) -= l * A(k, c);
            for (int c = 0; c < B.c; ++c) B(r, c) -= l * B(k, c);
        }
    }
    Mat X(n, B.c);
    for (int c = 0; c < B.c; ++c)
        for (int k = n - 1; k >= 0; --k) {
            double s = B(k, c);
            for (int j = k + 1; j < n; ++j) s -= A(k, j) * X(j, c);
            X(k, c) = s / A(k, k);
        }
    return X;
}

} // namespace

std::vector<Model> md_pose_cal_ours(const double *x, const double *y, const double *dx, const double *dy) {
    std::vector<Model> out;
    const int pairs[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    Mat C0(3, 3), C1(3, 3);
    for (int k = 0; k < 3; ++k) {
        const int i = pairs[k][0], j = pairs[k][1];
        double p[3], q[3], pp[3], qq[3];
        for (int c = 0; c < 3; ++c) {
            p[c] = dx[i] * x[3 * i + c] - dx[j] * x[3 * j + c];
            q[c] = x[3 * i + c] - x[3 * j + c];
            pp[c] = dy[i] * y[3 * i + c] - dy[j] * y[3 * j + c];
            qq[c] = y[3 * i + c] - y[3 * j + c];
        }
        // monomials (S v^2, S v, S) on image 1 and (u^2, u, 1) on image 0
        C0(k, 0) = dot(qq, qq);
        C0(k, 1) = 2.0 * dot(pp, qq);
        C0(k, 2) = dot(pp, pp);
        C1(k, 0) = -dot(q, q);
        C1(k, 1) = -2.0 * dot(p, q);
        C1(k, 2) = -dot(p, p);
    }
    Mat K = pplu_solve(C0, C1);
    for (double &v : K.a) v = -v;
    // (S v)^2 = (S v^2) S, each a quadratic in u (rows 1, 0, 2 of K)
    const double *k0 = &K.a[0], *k1 = &K.a[3], *k2 = &K.a[6];
    const double c4 = 1.0 / (k1[0] * k1[0] - k0[0] * k2[0]);
    const double c3 = c4 * (2 * k1[0] * k1[1] - k0[1] * k2[0] - k0[0] * k2[1]);
    const double c2 = c4 * (k1[1] * k1[1] - k0[0] * k2[2] - k0[1] * k2[1] - k0[2] * k2[0] + 2 * k1[0] * k1[2]);
    const double c1 = c4 * (2 * k1[1] * k1[2] - k0[2] * k2[1] - k0[1] * k2[2]);
    const double c0 = c4 * (k1[2] * k1[2] - k0[2] * k2[2]);
    Mat CC(4, 4);
    CC(0, 1) = CC(1, 2) = CC(2, 3) = 1.0;
    CC(3, 0) = -c0;
    CC(3, 1) = -c1;
    CC(3, 2) = -c2;
    CC(3, 3) = -c3;
    std::vector<double> wr, wi;
    if (!eig_real(CC, &wr, &wi)) return out;
    std::vector<double> roots;
    for (int i = 0; i < 4; ++i)
        if (!(std::fabs(wi[i]) > 1e-8)) roots.push_back(wr[i]);
    // column bookkeeping of solver_p3p_mono_3d: root ii fills column ii, the first
    // m (= number kept) columns are returned
    const int nr = (int)roots.size();
    std::vector<bool> kept(nr, false);
    int m = 0;
    for (int ii = 0; ii < nr; ++ii) {
        const double uu = roots[ii];
        const double S = k2[0] * uu * uu + k2[1] * uu + k2[2];
        if (S < 0.01) continue;
        kept[ii] = true;
        ++m;
    }
    for (int col = 0; col < m; ++col) {
        if (!kept[col]) continue; // never written in the reference (undefined values)
        const double u = roots[col];
        const double S = k2[0] * u * u + k2[1] * u + k2[2];
        const double v = (k1[0] * u * u + k1[1] * u + k1[2]) / S;
        const double s = std::sqrt(S);
        bool ok = true;
        for (int i = 0; i < 3; ++i)
            if (dx[i] + u <= 0 || dy[i] + v <= 0) ok = false;
        if (!ok) continue;
        double v1[3], v2[3], u1[3], u2[3];
        for (int c = 0; c < 3; ++c) {
            v1[c] = s * (dy[0] + v) * y[c] - s * (dy[1] + v) * y[3 + c];
            v2[c] = s * (dy[0] + v) * y[c] - s * (dy[2] + v) * y[6 + c];
            u1[c] = (dx[0] + u) * x[c] - (dx[1] + u) * x[3 + c];
            u2[c] = (dx[0] + u) * x[c] - (dx[2] + u) * x[6 + c];
        }
        Model mo;
        rot_from_differences(u1, u2, v1, v2, mo.R);
        for (int r = 0; r < 3; ++r)
            mo.t[r] = s * (dy[0] + v) * y[r] -
                      (dx[0] + u) * (mo.R[3 * r] * x[0] + mo.R[3 * r + 1] * x[1] + mo.R[3 * r + 2] * x[2]);
        mo.scale = s;
        mo.offset0 = u;
        mo.offset1 = s * v;
        out.push_back(mo);
    }
    return out;
}

std::vector<Model> md_pose_sf_ours(const double *x, const double *y, const double *dx, const double *dy) {
    std::vector<Model> out;
    // lifted points: X1 = [dx_i x_i], X2 = [dy_0 y_0, dy_1 y_1, y_2] (third depth unknown)
    double X1[3][3], X2[3][3]; // [row][col]
    for (int i = 0; i < 3; ++i)
        for (int r = 0; r < 3; ++r) {
            X1[r][i] = dx[i] * x[3 * i + r];
            X2[r][i] = (i < 2 ? dy[i] : 1.0) * y[3 * i + r];
        }
    double a[17];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) a[3 * r + c] = X1[r][c];
    a[9] = X2[0][0];
    a[10] = X2[0][1];
    a[11] = X2[0][2];
    a[12] = X2[1][0];
    a[13] = X2[1][1];
    a[14] = X2[1][2];
    a[15] = X2[2][0];
    a[16] = X2[2][1];
    const double b[12] = {a[0] - a[1], a[3] - a[4],   a[6] - a[7],   a[0] - a[2],  a[3] - a[5],  a[6] - a[8],
                          a[1] - a[2], a[4] - a[5],   a[7] - a[8],   a[9] - a[10], a[12] - a[13], a[15] - a[16]};
    auto sq = [](double v) { return v * v; };
    double c[18];
    c[0] = -sq(b[11]);
    c[1] = sq(b[2]);
    c[2] = -sq(b[9]) - sq(b[10]);
    c[3] = sq(b[0]) + sq(b[1]);
    c[4] = -1.0;
    c[5] = 2 * a[15];
    c[6] = -sq(a[15]);
    c[7] = sq(b[5]);
    c[8] = -sq(a[11]) - sq(a[14]);
    c[9] = 2 * a[9] * a[11] + 2 * a[12] * a[14];
    c[10] = -sq(a[9]) - sq(a[12]);
    c[11] = sq(b[3]) + sq(b[4]);
    c[12] = 2 * a[16] - 2 * a[15];
    c[13] = sq(a[15]) - sq(a[16]);
    c[14] = sq(b[8]) - sq(b[5]);
    c[15] = 2 * a[10] * a[11] - 2 * a[9] * a[11] - 2 * a[12] * a[14] + 2 * a[13] * a[14];
    c[16] = sq(a[9]) - sq(a[10]) + sq(a[12]) - sq(a[13]);
    c[17] = -sq(b[3]) - sq(b[4]) + sq(b[6]) + sq(b[7]);
    double d[21];
    d[6] = 1 / (a[6] - a[7]);
    d[0] = (-c[3] * c[8]) * d[6];
    d[1] = (-c[3] * c[9]) * d[6];
    d[2] = (c[2] * c[11] - c[3] * c[10]) * d[6];
    d[3] = (-c[3] * c[4] - c[1] * c[8]) * d[6];
    d[4] = (-c[3] * c[5] - c[1] * c[9]) * d[6];
    d[5] = (c[2] * c[7] - c[3] * c[6] + c[0] * c[11] - c[1] * c[10]) * d[6];
    d[7] = (a[6] * a[16] - 2 * a[6] * a[15] + a[7] * a[15] + a[8] * a[15] - a[8] * a[16]) * d[6];
    d[8] = 1 / (2 * (a[6] - a[7]) * (a[15] - a[16]));
    d[9] = (-c[3] * c[15]) * d[8];
    d[10] = (c[2] * c[17] - c[3] * c[16]) * d[8];
    d[11] = (-c[3] * c[12] - c[1] * c[15]) * d[8];
    d[12] = (c[2] * c[14] - c[3] * c[13] + c[0] * c[17] - c[1] * c[16]) * d[8];
    d[13] = 1 / (a[6] + a[7] - 2 * a[8]);
    d[14] = (a[8] * a[15] - a[7] * a[15] - a[6] * a[16] + a[8] * a[16]) * d[13];
    d[15] = (c[8] * c[17]) * d[13];
    d[16] = (c[9] * c[17] - c[11] * c[15]) * d[13];
    d[17] = (c[10] * c[17] - c[11] * c[16]) * d[13];
    d[18] = (c[4] * c[17] + c[8] * c[14]) * d[13];
    d[19] = (c[5] * c[17] - c[7] * c[15] + c[9] * c[14] - c[11] * c[12]) * d[13];
    d[20] = (c[6] * c[17] - c[7] * c[16] + c[10] * c[14] - c[11] * c[13]) * d[13];
    Mat C0(3, 3), C1(3, 4);
    const double c0v[9] = {d[2], d[5], d[7], d[10], d[12], 1.0, d[17], d[20], d[14]};
    const double c1v[12] = {d[0] - d[9], d[3] - d[11], d[1] - d[10], d[4] - d[12], 0, 0, d[9], d[11],
                            d[15] - d[9], d[18] - d[11], d[16] - d[10], d[19] - d[12]};
    std::memcpy(C0.a.data(), c0v, sizeof(c0v));
    std::memcpy(C1.a.data(), c1v, sizeof(c1v));
    Mat C2 = pplu_solve(C0, C1);
    Mat AM(4, 4);
    AM(0, 2) = AM(1, 3) = 1.0;
    for (int j = 0; j < 4; ++j) {
        AM(2, j) = -C2(0, j);
        AM(3, j) = -C2(1, j);
    }
    std::vector<double> wr, wi;
    if (!eig_real(AM, &wr, &wi)) return out;
    for (int k = 0; k < 4; ++k) {
        if (std::fabs(wi[k]) > 0.001 || wr[k] < 0.0) continue;
        const double d3 = 1.0 / wr[k];
        Mat A0(2, 2), A1(2, 1);
        A0(0, 0) = (d[3] - d[11]) * d3 * d3 + (d[4] - d[12]) * d3 + d[5];
        A0(0, 1) = d[7];
        A0(1, 0) = d[12] + d[11] * d3;
        A0(1, 1) = 1.0;
        A1(0, 0) = (d[0] - d[9]) * d3 * d3 + (d[1] - d[10]) * d3 + d[2];
        A1(1, 0) = d[10] + d[9] * d3;
        Mat A2 = pplu_solve(A0, A1);
        const double f2 = -A2(0, 0);
        if (f2 < 0.0) continue;
        const double s2 = -(c[1] * f2 + c[3]) / (c[0] * f2 + c[2]);
        if (s2 < 0.001) continue;
        const double s = std::sqrt(s2), f = std::sqrt(f2);
        auto kinv = [&](const double *p, double *o) {
            o[0] = p[0] / f;
            o[1] = p[1] / f;
            o[2] = p[2];
        };
        double ky0[3], ky1[3], ky2[3], kx0[3], kx1[3], kx2[3];
        kinv(y, ky0);
        kinv(y + 3, ky1);
        kinv(y + 6, ky2);
        kinv(x, kx0);
        kinv(x + 3, kx1);
        kinv(x + 6, kx2);
        double v1[3], v2[3], u1[3], u2[3];
        for (int r = 0; r < 3; ++r) {
            v1[r] = s * dy[0] * ky0[r] - s * dy[1] * ky1[r];
            v2[r] = s * dy[0] * ky0[r] - s * d3 * ky2[r];
            u1[r] = dx[0] * kx0[r] - dx[1] * kx1[r];
            u2[r] = dx[0] * kx0[r] - dx[2] * kx2[r];
        }
        Model mo;
        rot_from_differences(u1, u2, v1, v2, mo.R);
        for (int r = 0; r < 3; ++r)
            mo.t[r] = s * dy[0] * ky0[r] - dx[0] * (mo.R[3 * r] * kx0[0] + mo.R[3 * r + 1] * kx0[1] + mo.R[3 * r + 2] * kx0[2]);
        mo.scale = s;
        mo.offset0 = mo.offset1 = 0.0;
        mo.focal0 = mo.focal1 = f;
        out.push_back(mo);
    }
    return out;
}

std::vector<Model> md_pose_tf_ours(const double *x, const double *y, const double *dx, const double *dy) {
    std::vector<Model> out;
    double a[18];
    for (int i = 0; i < 3; ++i) {
        a[i] = x[3 * i] * dx[i];
        a[3 + i] = x[3 * i + 1] * dx[i];
        a[6 + i] = dx[i];
        a[9 + i] = y[3 * i] * dy[i];
        a[12 + i] = y[3 * i + 1] * dy[i];
        a[15 + i] = dy[i];
    }
    // squared distances of the pairs (0,1) (0,2) (1,2), split into xy and z parts
    const int pairs[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    Mat A(3, 3), B(3, 1);
    for (int k = 0; k < 3; ++k) {
        const int i = pairs[k][0], j = pairs[k][1];
        const double bx0 = a[i] - a[j], by0 = a[3 + i] - a[3 + j], bz0 = a[6 + i] - a[6 + j];
        const double bx1 = a[9 + i] - a[9 + j], by1 = a[12 + i] - a[12 + j], bz1 = a[15 + i] - a[15 + j];
        A(k, 0) = bx0 * bx0 + by0 * by0;
        A(k, 1) = -(bx1 * bx1 + by1 * by1);
        A(k, 2) = -bz1 * bz1;
        B(k, 0) = bz0 * bz0;
    }
    Mat sol = pplu_solve(A, B);
    const double s0 = -sol(0, 0), s1 = -sol(1, 0), s2 = -sol(2, 0);
    if (!(s0 > 0 && s1 > 0 && s2 > 0)) return out;
    const double f = std::sqrt(s0), s = std::sqrt(s2), w = std::sqrt(s1 / s2);
    double kx[3][3], ky[3][3]; // diag(f, f, 1) x, diag(w, w, 1) y
    for (int i = 0; i < 3; ++i) {
        kx[i][0] = f * x[3 * i];
        kx[i][1] = f * x[3 * i + 1];
        kx[i][2] = x[3 * i + 2];
        ky[i][0] = w * y[3 * i];
        ky[i][1] = w * y[3 * i + 1];
        ky[i][2] = y[3 * i + 2];
    }
    double v1[3], v2[3], u1[3], u2[3];
    for (int r = 0; r < 3; ++r) {
        v1[r] = s * (dy[0] * ky[0][r] - dy[1] * ky[1][r]);
        v2[r] = s * (dy[0] * ky[0][r] - dy[2] * ky[2][r]);
        u1[r] = dx[0] * kx[0][r] - dx[1] * kx[1][r];
        u2[r] = dx[0] * kx[0][r] - dx[2] * kx[2][r];
    }
    Model mo;
    rot_from_differences(u1, u2, v1, v2, mo.R);
    for (int r = 0; r < 3; ++r)
        mo.t[r] = s * dy[0] * ky[0][r] - dx[0] * (mo.R[3 * r] * kx[0][0] + mo.R[3 * r + 1] * kx[0][1] + mo.R[3 * r + 2] * kx[0][2]);
    mo.scale = s;
    mo.offset0 = mo.offset1 = 0.0;
    mo.focal0 = 1.0 / f;
    mo.focal1 = 1.0 / w;
    out.push_back(mo);
    return out;
}

std::vector<Model> md_pose_tf_4p4d(const double *x, const double *y, const double *dx, const double *dy) {
    std::vector<Model> out;
    Mat Cm(11, 11), rhs(11, 1);
    int row = 0;
    for (int i = 0; i < 4; ++i) {
        const double u1 = x[3 * i] / x[3 * i + 2], v1 = x[3 * i + 1] / x[3 * i + 2];
        const double u2 = y[3 * i] / y[3 * i + 2], v2 = y[3 * i + 1] / y[3 * i + 2];
        const double q = dy[i] / dx[i];
        double r0[12] = {-u1, -v1, -1, 0, 0, 0, 0, 0, 0, 0, q, -q * v2};
        double r1[12] = {0, 0, 0, -u1, -v1, -1, 0, 0, 0, -q, 0, q * u2};
        double r2[12] = {0, 0, 0, 0, 0, 0, -u1, -v1, -1, q * v2, -q * u2, 0};
        const double *rows[3] = {r0, r1, r2};
        for (int k = 0; k < (i == 3 ? 2 : 3); ++k, ++row) {
            for (int c = 0; c < 11; ++c) Cm(row, c) = rows[k][c];
            rhs(row, 0) = -rows[k][11];
        }
    }
    Mat f = pplu_solve(Cm, rhs);
    double F[9];
    for (int e = 0; e < 9; ++e) F[e] = f(e, 0);
    double fsq0, fsq1;
    bougnoux_focals(F, &fsq0, &fsq1);
    const double focal1 = std::sqrt(fsq0), focal2 = std::sqrt(fsq1);
    if (std::isnan(focal1) || std::isnan(focal2)) return out;
    double E[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) E[3 * r + c] = (r < 2 ? focal2 : 1.0) * F[3 * r + c] * (c < 2 ? focal1 : 1.0);
    double b1[12], b2[12];
    for (int i = 0; i < 4; ++i) {
        const double n1 = std::sqrt(dot(x + 3 * i, x + 3 * i)), n2 = std::sqrt(dot(y + 3 * i, y + 3 * i));
        for (int c = 0; c < 3; ++c) {
            b1[3 * i + c] = x[3 * i + c] / n1;
            b2[3 * i + c] = y[3 * i + c] / n2;
        }
    }
    std::vector<Model> poses;
    motion_from_essential(E, b1, b2, 4, &poses);
    for (Model m : poses) {
        m.scale = 1.0;
        m.offset0 = m.offset1 = 0.0;
        m.focal0 = focal1;
        m.focal1 = focal2;
        out.push_back(m);
    }
    return out;
}

} // namespace oracle
