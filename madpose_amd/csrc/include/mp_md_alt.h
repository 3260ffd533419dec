// Option-gated alternative MD minimal solvers (HybridLORansacOptions::use_ours /
// use_4p4d), device versions of src/solver.cpp:536-680 (calibrated), :741-984
// (shared focal), :1045-1148 (two focal) and :1287-1406 (two focal 4p4d); see
// oracle/src/md_alt.cpp for the derivations and the reference quirks reproduced
// (column bookkeeping of solver_p3p_mono_3d, uncalibrated points in the 4p4d
// motion_from_essential).  These paths are off by default and run one sample per
// lane; they are not tuned.
#pragma once
#include "mp_md.h"
#include "mp_pt67.h"

namespace mp {

// ---------------------------------------------------------------------------
// Eigenvalues of a small general real matrix: balancing, Hessenberg reduction by
// Gaussian elimination and the Francis double-shift QR (EISPACK balanc / elmhes /
// hqr), the same sequence as the oracle's eig_real, so the eigenvalue order and the
// real/complex classification agree.  Returns false if QR does not converge.
MP_HD double sign_of(double a, double b) { return b >= 0 ? fabs(a) : -fabs(a); }

template <int N> MP_HD bool eig_small(double (&a)[N][N], double (&wr)[N], double (&wi)[N]) {
    // balance
    const double radix = 2.0, sqrdx = 4.0;
    for (int pass = 0, done = 0; !done && pass < 100; ++pass) {
        done = 1;
        for (int i = 0; i < N; ++i) {
            double r = 0, c = 0;
            for (int j = 0; j < N; ++j)
                if (j != i) {
                    c += fabs(a[j][i]);
                    r += fabs(a[i][j]);
                }
            if (c != 0.0 && r != 0.0) {
                double g = r / radix, f = 1.0, s = c + r;
                while (c < g) {
                    f *= radix;
                    c *= sqrdx;
                }
                g = r * radix;
                while (c > g) {
                    f /= radix;
                    c /= sqrdx;
                }
                if ((c + r) / f < 0.95 * s) {
                    done = 0;
                    g = 1.0 / f;
                    for (int j = 0; j < N; ++j) a[i][j] *= g;
                    for (int j = 0; j < N; ++j) a[j][i] *= f;
                }
            }
        }
    }
    // Hessenberg by elimination with pivoting
    for (int m = 1; m < N - 1; ++m) {
        double x = 0.0;
        int i = m;
        for (int j = m; j < N; ++j)
            if (fabs(a[j][m - 1]) > fabs(x)) {
                x = a[j][m - 1];
                i = j;
            }
        if (i != m) {
            for (int j = m - 1; j < N; ++j) {
                const double tmp = a[i][j];
                a[i][j] = a[m][j];
                a[m][j] = tmp;
            }
            for (int j = 0; j < N; ++j) {
                const double tmp = a[j][i];
                a[j][i] = a[j][m];
                a[j][m] = tmp;
            }
        }
        if (x != 0.0) {
            for (i = m + 1; i < N; ++i) {
                double y = a[i][m - 1];
                if (y != 0.0) {
                    y /= x;
                    a[i][m - 1] = y;
                    for (int j = m; j < N; ++j) a[i][j] -= y * a[m][j];
                    for (int j = 0; j < N; ++j) a[j][m] += y * a[j][i];
                }
            }
        }
    }
    for (int i = 2; i < N; ++i)
        for (int j = 0; j < i - 1; ++j) a[i][j] = 0.0;
    // Francis QR
    for (int i = 0; i < N; ++i) wr[i] = wi[i] = 0.0;
    double anorm = 0.0;
    for (int i = 0; i < N; ++i)
        for (int j = (i > 0 ? i - 1 : 0); j < N; ++j) anorm += fabs(a[i][j]);
    int nn = N - 1;
    double t = 0.0, p = 0, q = 0, r = 0, s = 0, w = 0, x = 0, y = 0, z = 0;
    while (nn >= 0) {
        int its = 0, l;
        do {
            for (l = nn; l >= 1; --l) {
                s = fabs(a[l - 1][l - 1]) + fabs(a[l][l]);
                if (s == 0.0) s = anorm;
                if (fabs(a[l][l - 1]) + s == s) {
                    a[l][l - 1] = 0.0;
                    break;
                }
            }
            x = a[nn][nn];
            if (l == nn) {
                wr[nn] = x + t;
                wi[nn--] = 0.0;
            } else {
                y = a[nn - 1][nn - 1];
                w = a[nn][nn - 1] * a[nn - 1][nn];
                if (l == nn - 1) {
                    p = 0.5 * (y - x);
                    q = p * p + w;
                    z = sqrt(fabs(q));
                    x += t;
                    if (q >= 0.0) {
                        z = p + sign_of(z, p);
                        wr[nn - 1] = wr[nn] = x + z;
                        if (z != 0.0) wr[nn] = x - w / z;
                        wi[nn - 1] = wi[nn] = 0.0;
                    } else {
                        wr[nn - 1] = wr[nn] = x + p;
                        wi[nn] = z;
                        wi[nn - 1] = -z;
                    }
                    nn -= 2;
                } else {
                    if (its == 60) return false;
                    if (its == 10 || its == 20 || its == 40) {
                        t += x;
                        for (int i = 0; i <= nn; ++i) a[i][i] -= x;
                        s = fabs(a[nn][nn - 1]) + fabs(a[nn - 1][nn - 2]);
                        y = x = 0.75 * s;
                        w = -0.4375 * s * s;
                    }
                    ++its;
                    int m;
                    for (m = nn - 2; m >= l; --m) {
                        z = a[m][m];
                        r = x - z;
                        s = y - z;
                        p = (r * s - w) / a[m + 1][m] + a[m][m + 1];
                        q = a[m + 1][m + 1] - z - r - s;
                        r = a[m + 2][m + 1];
                        s = fabs(p) + fabs(q) + fabs(r);
                        p /= s;
                        q /= s;
                        r /= s;
                        if (m == l) break;
                        const double uu = fabs(a[m][m - 1]) * (fabs(q) + fabs(r));
                        const double vv = fabs(p) * (fabs(a[m - 1][m - 1]) + fabs(z) + fabs(a[m + 1][m + 1]));
                        if (uu + vv == vv) break;
                    }
                    for (int i = m + 2; i <= nn; ++i) {
                        a[i][i - 2] = 0.0;
                        if (i != m + 2) a[i][i - 3] = 0.0;
                    }
                    for (int k = m; k <= nn - 1; ++k) {
                        if (k != m) {
                            p = a[k][k - 1];
                            q = a[k + 1][k - 1];
                            r = 0.0;
                            if (k != nn - 1) r = a[k + 2][k - 1];
                            if ((x = fabs(p) + fabs(q) + fabs(r)) != 0.0) {
                                p /= x;
                                q /= x;
                                r /= x;
                            }
                        }
                        if ((s = sign_of(sqrt(p * p + q * q + r * r), p)) != 0.0) {
                            if (k == m) {
                                if (l != m) a[k][k - 1] = -a[k][k - 1];
                            } else
                                a[k][k - 1] = -s * x;
                            p += s;
                            x = p / s;
                            y = q / s;
                            z = r / s;
                            q /= p;
                            r /= p;
                            for (int j = k; j <= nn; ++j) {
                                p = a[k][j] + q * a[k + 1][j];
                                if (k != nn - 1) {
                                    p += r * a[k + 2][j];
                                    a[k + 2][j] -= p * z;
                                }
                                a[k + 1][j] -= p * y;
                                a[k][j] -= p * x;
                            }
                            const int mmin = nn < k + 3 ? nn : k + 3;
                            for (int i = l; i <= mmin; ++i) {
                                p = x * a[i][k] + y * a[i][k + 1];
                                if (k != nn - 1) {
                                    p += z * a[i][k + 2];
                                    a[i][k + 2] -= p * r;
                                }
                                a[i][k + 1] -= p * q;
                                a[i][k] -= p;
                            }
                        }
                    }
                }
            }
        } while (l < nn - 1);
    }
    return true;
}

// partial-pivot LU solve A X = B in place (B becomes X), as Eigen's partialPivLu
template <int N, int M> MP_HD void pplu_solve(double (&A)[N][N], double (&B)[N][M]) {
    for (int k = 0; k < N; ++k) {
        int p = k;
        for (int r = k + 1; r < N; ++r)
            if (fabs(A[r][k]) > fabs(A[p][k])) p = r;
        if (p != k) {
            for (int c = 0; c < N; ++c) {
                const double tmp = A[k][c];
                A[k][c] = A[p][c];
                A[p][c] = tmp;
            }
            for (int c = 0; c < M; ++c) {
                const double tmp = B[k][c];
                B[k][c] = B[p][c];
                B[p][c] = tmp;
            }
        }
        for (int r = k + 1; r < N; ++r) {
            const double l = A[r][k] / A[k][k];
            for (int c = k + 1; c < N; ++c) A[r][c] -= l * A[k][c];
            for (int c = 0; c < M; ++c) B[r][c] -= l * B[k][c];
        }
    }
    for (int c = 0; c < M; ++c)
        for (int k = N - 1; k >= 0; --k) {
            double s = B[k][c];
            for (int j = k + 1; j < N; ++j) s -= A[k][j] * B[j][c];
            B[k][c] = s / A[k][k];
        }
}

// R = [v1 v2 v1xv2] [u1 u2 u1xu2]^-1 (cofactor inverse, no re-orthonormalisation)
MP_HD void rot_from_differences(const double *u1, const double *u2, const double *v1, const double *v2, double *R) {
    double u3[3], v3[3];
    cross3(u1, u2, u3);
    cross3(v1, v2, v3);
    const double X[9] = {u1[0], u2[0], u3[0], u1[1], u2[1], u3[1], u1[2], u2[2], u3[2]};
    const double Y[9] = {v1[0], v2[0], v3[0], v1[1], v2[1], v3[1], v1[2], v2[2], v3[2]};
    const double c00 = X[4] * X[8] - X[5] * X[7], c01 = X[5] * X[6] - X[3] * X[8], c02 = X[3] * X[7] - X[4] * X[6];
    const double det = X[0] * c00 + X[1] * c01 + X[2] * c02;
    const double Xi[9] = {c00 / det,
                          (X[2] * X[7] - X[1] * X[8]) / det,
                          (X[1] * X[5] - X[2] * X[4]) / det,
                          c01 / det,
                          (X[0] * X[8] - X[2] * X[6]) / det,
                          (X[2] * X[3] - X[0] * X[5]) / det,
                          c02 / det,
                          (X[1] * X[6] - X[0] * X[7]) / det,
                          (X[0] * X[4] - X[1] * X[3]) / det};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) R[3 * r + c] = Y[3 * r] * Xi[c] + Y[3 * r + 1] * Xi[3 + c] + Y[3 * r + 2] * Xi[6 + c];
}

// solve_scale_shift_pose_ours (calibrated, 3 points): <= 4 models (scale, offset0 = u,
// offset1 = s v before the estimator's division by the scale)
MP_HD int md_pose_cal_ours(const double (&x)[3][3], const double (&y)[3][3], const double *dx, const double *dy,
                           Model *out) {
    const int pi[3] = {0, 0, 1}, pj[3] = {1, 2, 2};
    double C0[3][3], K[3][3];
    for (int k = 0; k < 3; ++k) {
        const int i = pi[k], j = pj[k];
        double p[3], q[3], pp[3], qq[3];
        for (int c = 0; c < 3; ++c) {
            p[c] = dx[i] * x[i][c] - dx[j] * x[j][c];
            q[c] = x[i][c] - x[j][c];
            pp[c] = dy[i] * y[i][c] - dy[j] * y[j][c];
            qq[c] = y[i][c] - y[j][c];
        }
        C0[k][0] = dot3(qq, qq);
        C0[k][1] = 2.0 * dot3(pp, qq);
        C0[k][2] = dot3(pp, pp);
        K[k][0] = -dot3(q, q);
        K[k][1] = -2.0 * dot3(p, q);
        K[k][2] = -dot3(p, p);
    }
    pplu_solve<3, 3>(C0, K);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) K[r][c] = -K[r][c];
    const double *k0 = K[0], *k1 = K[1], *k2 = K[2];
    const double c4 = 1.0 / (k1[0] * k1[0] - k0[0] * k2[0]);
    double A[4][4] = {{0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}, {0, 0, 0, 0}};
    A[3][3] = -c4 * (2 * k1[0] * k1[1] - k0[1] * k2[0] - k0[0] * k2[1]);
    A[3][2] = -c4 * (k1[1] * k1[1] - k0[0] * k2[2] - k0[1] * k2[1] - k0[2] * k2[0] + 2 * k1[0] * k1[2]);
    A[3][1] = -c4 * (2 * k1[1] * k1[2] - k0[2] * k2[1] - k0[1] * k2[2]);
    A[3][0] = -c4 * (k1[2] * k1[2] - k0[2] * k2[2]);
    double wr[4], wi[4];
    if (!eig_small<4>(A, wr, wi)) return 0;
    double roots[4];
    int nr = 0;
    for (int i = 0; i < 4; ++i)
        if (!(fabs(wi[i]) > 1e-8)) roots[nr++] = wr[i];
    bool kept[4] = {false, false, false, false};
    int m = 0;
    for (int ii = 0; ii < nr; ++ii) {
        const double u = roots[ii];
        if (k2[0] * u * u + k2[1] * u + k2[2] < 0.01) continue;
        kept[ii] = true;
        ++m;
    }
    int n = 0;
    for (int col = 0; col < m; ++col) {
        if (!kept[col]) continue; // column never written by the reference
        const double u = roots[col];
        const double S = k2[0] * u * u + k2[1] * u + k2[2];
        const double v = (k1[0] * u * u + k1[1] * u + k1[2]) / S;
        const double s = sqrt(S);
        bool ok = true;
        for (int i = 0; i < 3; ++i)
            if (dx[i] + u <= 0 || dy[i] + v <= 0) ok = false;
        if (!ok) continue;
        double v1[3], v2[3], u1[3], u2[3];
        for (int c = 0; c < 3; ++c) {
            v1[c] = s * (dy[0] + v) * y[0][c] - s * (dy[1] + v) * y[1][c];
            v2[c] = s * (dy[0] + v) * y[0][c] - s * (dy[2] + v) * y[2][c];
            u1[c] = (dx[0] + u) * x[0][c] - (dx[1] + u) * x[1][c];
            u2[c] = (dx[0] + u) * x[0][c] - (dx[2] + u) * x[2][c];
        }
        Model mo;
        rot_from_differences(u1, u2, v1, v2, mo.R);
        for (int r = 0; r < 3; ++r)
            mo.t[r] = s * (dy[0] + v) * y[0][r] - (dx[0] + u) * (mo.R[3 * r] * x[0][0] + mo.R[3 * r + 1] * x[0][1] +
                                                                 mo.R[3 * r + 2] * x[0][2]);
        mo.scale = s;
        mo.offset0 = u;
        mo.offset1 = s * v;
        mo.focal0 = mo.focal1 = 1.0;
        out[n++] = mo;
    }
    return n;
}

// solve_scale_shift_pose_shared_focal_ours (uses points 0..2): <= 4 models
MP_HD int md_pose_sf_ours(const double (&x)[4][3], const double (&y)[4][3], const double *dx, const double *dy,
                          Model *out) {
    double a[17];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) a[3 * r + c] = dx[c] * x[c][r];
    a[9] = dy[0] * y[0][0];
    a[10] = dy[1] * y[1][0];
    a[11] = y[2][0];
    a[12] = dy[0] * y[0][1];
    a[13] = dy[1] * y[1][1];
    a[14] = y[2][1];
    a[15] = dy[0] * y[0][2];
    a[16] = dy[1] * y[1][2];
    const double b[12] = {a[0] - a[1], a[3] - a[4], a[6] - a[7], a[0] - a[2],  a[3] - a[5],   a[6] - a[8],
                          a[1] - a[2], a[4] - a[5], a[7] - a[8], a[9] - a[10], a[12] - a[13], a[15] - a[16]};
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
    double C0[3][3] = {{d[2], d[5], d[7]}, {d[10], d[12], 1.0}, {d[17], d[20], d[14]}};
    double C[3][4] = {{d[0] - d[9], d[3] - d[11], d[1] - d[10], d[4] - d[12]},
                      {0, 0, d[9], d[11]},
                      {d[15] - d[9], d[18] - d[11], d[16] - d[10], d[19] - d[12]}};
    pplu_solve<3, 4>(C0, C);
    double AM[4][4] = {{0, 0, 1, 0}, {0, 0, 0, 1}, {-C[0][0], -C[0][1], -C[0][2], -C[0][3]},
                       {-C[1][0], -C[1][1], -C[1][2], -C[1][3]}};
    double wr[4], wi[4];
    if (!eig_small<4>(AM, wr, wi)) return 0;
    int n = 0;
    for (int k = 0; k < 4; ++k) {
        if (fabs(wi[k]) > 0.001 || wr[k] < 0.0) continue;
        const double d3 = 1.0 / wr[k];
        double A0[2][2] = {{(d[3] - d[11]) * d3 * d3 + (d[4] - d[12]) * d3 + d[5], d[7]}, {d[12] + d[11] * d3, 1.0}};
        double A1[2][1] = {{(d[0] - d[9]) * d3 * d3 + (d[1] - d[10]) * d3 + d[2]}, {d[10] + d[9] * d3}};
        pplu_solve<2, 1>(A0, A1);
        const double f2 = -A1[0][0];
        if (f2 < 0.0) continue;
        const double s2 = -(c[1] * f2 + c[3]) / (c[0] * f2 + c[2]);
        if (s2 < 0.001) continue;
        const double s = sqrt(s2), f = sqrt(f2);
        double ky[3][3], kx[3][3];
        for (int i = 0; i < 3; ++i) {
            ky[i][0] = y[i][0] / f;
            ky[i][1] = y[i][1] / f;
            ky[i][2] = y[i][2];
            kx[i][0] = x[i][0] / f;
            kx[i][1] = x[i][1] / f;
            kx[i][2] = x[i][2];
        }
        double v1[3], v2[3], u1[3], u2[3];
        for (int r = 0; r < 3; ++r) {
            v1[r] = s * dy[0] * ky[0][r] - s * dy[1] * ky[1][r];
            v2[r] = s * dy[0] * ky[0][r] - s * d3 * ky[2][r];
            u1[r] = dx[0] * kx[0][r] - dx[1] * kx[1][r];
            u2[r] = dx[0] * kx[0][r] - dx[2] * kx[2][r];
        }
        Model mo;
        rot_from_differences(u1, u2, v1, v2, mo.R);
        for (int r = 0; r < 3; ++r)
            mo.t[r] = s * dy[0] * ky[0][r] -
                      dx[0] * (mo.R[3 * r] * kx[0][0] + mo.R[3 * r + 1] * kx[0][1] + mo.R[3 * r + 2] * kx[0][2]);
        mo.scale = s;
        mo.offset0 = mo.offset1 = 0.0;
        mo.focal0 = mo.focal1 = f;
        out[n++] = mo;
    }
    return n;
}

// solve_scale_shift_pose_two_focal_ours (points 0..2): <= 1 model
MP_HD int md_pose_tf_ours(const double (&x)[4][3], const double (&y)[4][3], const double *dx, const double *dy,
                          Model *out) {
    const int pi[3] = {0, 0, 1}, pj[3] = {1, 2, 2};
    double A[3][3], B[3][1];
    for (int k = 0; k < 3; ++k) {
        const int i = pi[k], j = pj[k];
        const double bx0 = x[i][0] * dx[i] - x[j][0] * dx[j], by0 = x[i][1] * dx[i] - x[j][1] * dx[j];
        const double bz0 = dx[i] - dx[j];
        const double bx1 = y[i][0] * dy[i] - y[j][0] * dy[j], by1 = y[i][1] * dy[i] - y[j][1] * dy[j];
        const double bz1 = dy[i] - dy[j];
        A[k][0] = bx0 * bx0 + by0 * by0;
        A[k][1] = -(bx1 * bx1 + by1 * by1);
        A[k][2] = -bz1 * bz1;
        B[k][0] = bz0 * bz0;
    }
    pplu_solve<3, 1>(A, B);
    const double s0 = -B[0][0], s1 = -B[1][0], s2 = -B[2][0];
    if (!(s0 > 0 && s1 > 0 && s2 > 0)) return 0;
    const double f = sqrt(s0), s = sqrt(s2), w = sqrt(s1 / s2);
    double kx[3][3], ky[3][3];
    for (int i = 0; i < 3; ++i) {
        kx[i][0] = f * x[i][0];
        kx[i][1] = f * x[i][1];
        kx[i][2] = x[i][2];
        ky[i][0] = w * y[i][0];
        ky[i][1] = w * y[i][1];
        ky[i][2] = y[i][2];
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
        mo.t[r] = s * dy[0] * ky[0][r] -
                  dx[0] * (mo.R[3 * r] * kx[0][0] + mo.R[3 * r + 1] * kx[0][1] + mo.R[3 * r + 2] * kx[0][2]);
    mo.scale = s;
    mo.offset0 = mo.offset1 = 0.0;
    mo.focal0 = 1.0 / f;
    mo.focal1 = 1.0 / w;
    out[0] = mo;
    return 1;
}

// solve_scale_shift_pose_two_focal_4p4d: <= 4 models
MP_HD int md_pose_tf_4p4d(const double (&x)[4][3], const double (&y)[4][3], const double *dx, const double *dy,
                          Model *out) {
    double C[11][11], rhs[11][1];
    int row = 0;
    for (int i = 0; i < 4; ++i) {
        const double u1 = x[i][0] / x[i][2], v1 = x[i][1] / x[i][2];
        const double u2 = y[i][0] / y[i][2], v2 = y[i][1] / y[i][2];
        const double q = dy[i] / dx[i];
        const double r0[12] = {-u1, -v1, -1, 0, 0, 0, 0, 0, 0, 0, q, -q * v2};
        const double r1[12] = {0, 0, 0, -u1, -v1, -1, 0, 0, 0, -q, 0, q * u2};
        const double r2[12] = {0, 0, 0, 0, 0, 0, -u1, -v1, -1, q * v2, -q * u2, 0};
        for (int k = 0; k < (i == 3 ? 2 : 3); ++k, ++row) {
            const double *rr = (k == 0) ? r0 : ((k == 1) ? r1 : r2);
            for (int c = 0; c < 11; ++c) C[row][c] = rr[c];
            rhs[row][0] = -rr[11];
        }
    }
    pplu_solve<11, 1>(C, rhs);
    double F[9];
    for (int e = 0; e < 9; ++e) F[e] = rhs[e][0];
    // focals_from_fundamental (src/solver.cpp:1150-1177) with zero principal points
    double e1[3], e2[3];
    null3(F, F + 3, F + 6, e1);
    const double c0[3] = {F[0], F[3], F[6]}, c1[3] = {F[1], F[4], F[7]}, c2[3] = {F[2], F[5], F[8]};
    null3(c0, c1, c2, e2);
    double L[3], M[3];
    for (int c = 0; c < 3; ++c) {
        L[c] = -e2[1] * F[c] + e2[0] * F[3 + c];
        M[c] = -e1[1] * F[3 * c] + e1[0] * F[3 * c + 1];
    }
    // the epipoles enter numerator and denominator linearly (scale and sign free)
    const double focal1 = sqrt(-(L[2] * F[8]) / (L[0] * F[6] + L[1] * F[7]));
    const double focal2 = sqrt(-(M[2] * F[8]) / (M[0] * F[2] + M[1] * F[5]));
    if (focal1 != focal1 || focal2 != focal2) return 0; // NaN: negative squared focal
    double E[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) E[3 * r + c] = (r < 2 ? focal2 : 1.0) * F[3 * r + c] * (c < 2 ? focal1 : 1.0);
    double b1[4][3], b2[4][3];
    for (int i = 0; i < 4; ++i) {
        const double n1 = 1.0 / sqrt(dot3(x[i], x[i])), n2 = 1.0 / sqrt(dot3(y[i], y[i]));
        for (int c = 0; c < 3; ++c) {
            b1[i][c] = x[i][c] * n1;
            b2[i][c] = y[i][c] * n2;
        }
    }
    const int n = motion_from_essential<4>(E, b1, b2, out, 0, 4);
    for (int k = 0; k < n; ++k) {
        out[k].scale = 1.0;
        out[k].offset0 = out[k].offset1 = 0.0;
        out[k].focal0 = focal1;
        out[k].focal1 = focal2;
    }
    return n;
}

} // namespace mp
