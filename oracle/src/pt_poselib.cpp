// ORACLE -- test infrastructure only.
//
// The point minimal solvers' ROOT STAGES as PoseLib v2.0.4 computes them (the
// reference calls relpose_5pt at src/hybrid_pose_estimator.cpp:134 and relpose_7pt at
// src/hybrid_pose_two_focal_estimator.cpp:116; PoseLib is a CMake dependency that is
// not vendored, CMakeLists.txt:25-37, so parity with it is UNPINNED: the algorithms
// below are restated from PoseLib's published sources as recalled).
//
//   relpose_5pt   Nister's hidden-variable 5-point solver as in PoseLib
//                 solvers/relpose_5pt.cc: a Householder basis of the null space of
//                 the 5 x 9 epipolar system, the ten cubic constraints (det E = 0 and
//                 2 E E^T E - tr(E E^T) E = 0) in Nister's 20 monomials, Gauss-Jordan
//                 elimination with partial pivoting of the 10 x 20 template, the 3 x 3
//                 polynomial matrix B(z) of rows (e - z f), (g - z h), (i - z j), its
//                 degree-10 determinant, the real roots by PoseLib's Sturm bisection
//                 (misc/sturm.h bisect_sturm<10>: Sturm chain of the monic polynomial,
//                 Cauchy bound, bisection, Ridders' method then Newton), (x, y) from the
//                 null vector of B(z) by the largest cross product of its rows, and
//                 motion_from_essential (pt.cpp, the reference's copy at
//                 src/solver.cpp:1219-1285) with cheirality on the five bearings.
//   relpose_7pt   PoseLib solvers/relpose_7pt.cc: the 2-dim null space of the 7 x 9
//                 system (Householder), det(a N0 + N1) = c3 a^3 + c2 a^2 + c1 a + c0,
//                 normalised by c3 and solved in closed form (misc/univariate.cc
//                 solve_cubic_real: Cardano for one real root, the trigonometric form
//                 for three, one Newton step each), F = a N0 + N1 normalised.
//
// The device root stages (madpose_amd/csrc/kernels/group_5pt.h, mp_pt67.h) perform
// these operations in this order without FMA contraction, so their candidates are
// this code's to the bit (tests/test_pt_roots_gpu.py; the cubic's cbrt / acos / cos
// come from the device and host math libraries and may differ in the last bit).
// Plain C++ without FMA (the oracle is built for baseline x86-64: no FMA instructions).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace oracle {

// Householder null space of a K x 9 system (rows = epipolar constraints): Q = H_0 ..
// H_{K-1} of the QR of Q^T (v = x - alpha e_k, alpha = -sign(x_k) |x|, beta = 2 / v^T v),
// the basis vectors are Q e_{K+b}, b = 0 .. 8 - K.
template <int K> void householder_nullspace(const double (&Q)[K][9], double (&N)[9 - K][9]) {
    double A[9][K];
    for (int i = 0; i < K; ++i)
        for (int e = 0; e < 9; ++e) A[e][i] = Q[i][e];
    double V[K][9], beta[K];
    for (int k = 0; k < K; ++k) {
        double nrm = 0.0;
        for (int i = k; i < 9; ++i) nrm += A[i][k] * A[i][k];
        nrm = std::sqrt(nrm);
        const double alpha = (A[k][k] > 0) ? -nrm : nrm;
        double vn = 0.0;
        for (int i = 0; i < 9; ++i) {
            if (i < k) {
                V[k][i] = 0.0;
            } else {
                V[k][i] = A[i][k];
                if (i == k) V[k][i] -= alpha;
            }
            vn += V[k][i] * V[k][i];
        }
        beta[k] = (vn > 0) ? 2.0 / vn : 0.0;
        for (int j = k; j < K; ++j) {
            double d = 0.0;
            for (int i = 0; i < 9; ++i) d += V[k][i] * A[i][j];
            d *= beta[k];
            for (int i = 0; i < 9; ++i) A[i][j] -= d * V[k][i];
        }
    }
    for (int b = 0; b < 9 - K; ++b) {
        double v[9];
        for (int i = 0; i < 9; ++i) v[i] = (i == K + b) ? 1.0 : 0.0;
        for (int k = K - 1; k >= 0; --k) {
            double d = 0.0;
            for (int i = 0; i < 9; ++i) d += V[k][i] * v[i];
            d *= beta[k];
            for (int i = 0; i < 9; ++i) v[i] -= d * V[k][i];
        }
        for (int i = 0; i < 9; ++i) N[b][i] = v[i];
    }
}

// ---------------------------------------------------------------------------
// PoseLib misc/sturm.h: real roots of a degree-N polynomial by Sturm bisection
namespace sturm {

// the quotients (q0 + q1 x) and the normalisers c of the chain f_k = (q0 + q1 x)
// f_{k+1} + c f_{k+2}, from fvec = [monic f (N + 1) | monic f' / N (N)]
template <int N> void build_sturm_seq(const double *fvec, double *svec) {
    double f[3][N + 1];
    std::memset(f, 0, sizeof(f));
    for (int j = 0; j <= N; ++j) f[0][j] = fvec[j];
    for (int j = 0; j < N; ++j) f[1][j] = fvec[N + 1 + j];
    int i1 = 0, i2 = 1, i3 = 2;
    for (int i = 0; i < N - 1; ++i) {
        const double *f1 = f[i1], *f2 = f[i2];
        double *f3 = f[i3];
        const double q1 = f1[N - i] * f2[N - 1 - i];
        const double q0 = f1[N - 1 - i] * f2[N - 1 - i] - f1[N - i] * f2[N - 2 - i];
        f3[0] = f1[0] - q0 * f2[0];
        for (int j = 1; j < N - 1 - i; ++j) f3[j] = f1[j] - q1 * f2[j - 1] - q0 * f2[j];
        const double c = -std::fabs(f3[N - 2 - i]);
        const double ci = 1.0 / c;
        for (int j = 0; j < N - 1 - i; ++j) f3[j] = f3[j] * ci;
        // (f1, f2, f3) -> (f2, f3, f1)
        const int t = i1;
        i1 = i2;
        i2 = i3;
        i3 = t;
        svec[3 * i] = q0;
        svec[3 * i + 1] = q1;
        svec[3 * i + 2] = c;
    }
    svec[3 * N - 3] = f[i1][0];
    svec[3 * N - 2] = f[i1][1];
    svec[3 * N - 1] = f[i2][0];
}

// Horner on a monic polynomial (f[N] = 1 implied)
template <int N> double polyval(const double *f, double x) {
    double fx = x + f[N - 1];
    for (int i = N - 2; i >= 0; --i) fx = x * fx + f[i];
    return fx;
}

// sign changes of the chain at x (a constant offset -- the sign of the last
// polynomial -- is counted at every x, as PoseLib's flag_negative XOR does)
template <int N> int signchanges(const double *svec, double x) {
    double f[N + 1];
    f[N] = svec[3 * N - 1];
    f[N - 1] = svec[3 * N - 3] + x * svec[3 * N - 2];
    for (int i = N - 2; i >= 0; --i) f[i] = (svec[3 * i] + x * svec[3 * i + 1]) * f[i + 1] + svec[3 * i + 2] * f[i + 2];
    unsigned S = 0;
    for (int k = 0; k <= N; ++k) {
        const unsigned neg_k = f[k] < 0 ? 1u : 0u;
        const unsigned neg_k1 = (k < N) ? (f[k + 1] < 0 ? 1u : 0u) : 0u;
        S |= (neg_k ^ neg_k1) << k;
    }
    return __builtin_popcount(S);
}

template <int N> double get_bounds(const double *fvec) {
    double mx = 0;
    for (int i = 0; i < N; ++i) mx = std::max(mx, std::fabs(fvec[i]));
    return 1.0 + mx;
}

// Ridders' method while the bracket is wider than 1e-3, then Newton (at most 10 steps,
// |f| or |dx| below tol); appends the root
template <int N> void ridders_method_newton(const double *fvec, double a, double b, double *roots, int &n_roots, double tol) {
    double fa = polyval<N>(fvec, a);
    double fb = polyval<N>(fvec, b);
    if (!((fa < 0) ^ (fb < 0))) return;
    const double tol_newton = 1e-3;
    for (int iter = 0; iter < 30; ++iter) {
        if (std::fabs(a - b) < tol_newton) break;
        const double c = (a + b) * 0.5;
        const double fc = polyval<N>(fvec, c);
        const double s = std::sqrt(fc * fc - fa * fb);
        if (!s) break;
        const double d = (fa < fb) ? c + (a - c) * fc / s : c + (c - a) * fc / s;
        const double fd = polyval<N>(fvec, d);
        if (fd >= 0 ? (fc < 0) : (fc > 0)) {
            a = c;
            fa = fc;
            b = d;
            fb = fd;
        } else if (fd >= 0 ? (fa < 0) : (fa > 0)) {
            b = d;
            fb = fd;
        } else {
            a = d;
            fa = fd;
        }
    }
    double x = (a + b) * 0.5;
    const double *fpvec = fvec + N + 1; // the monic derivative / N
    for (int iter = 0; iter < 10; ++iter) {
        const double fx = polyval<N>(fvec, x);
        if (std::fabs(fx) < tol) break;
        const double fpx = static_cast<double>(N) * polyval<N - 1>(fpvec, x);
        const double dx = fx / fpx;
        x = x - dx;
        if (std::fabs(dx) < tol) break;
    }
    if (n_roots < N) roots[n_roots++] = x; // (PoseLib's roots[N]; the cap is never reached with consistent counts)
}

// the shape of the recursion tree, for the capacity rule of the GPU's breadth-first
// walk (kernels/group_bisect.h): intervals halved per depth, leaves
struct TreeCount {
    int pend[302] = {};
    int leaves = 0;
};

template <int N>
void isolate_roots(const double *fvec, const double *svec, double a, double b, int sa, int sb, double *roots,
                   int &n_roots, double tol, int depth, TreeCount &tc) {
    if (depth > 300) return;
    const int n_rts = sa - sb;
    if (n_rts > 1) {
        ++tc.pend[depth];
        const double c = (a + b) * 0.5;
        const int sc = signchanges<N>(svec, c);
        isolate_roots<N>(fvec, svec, a, c, sa, sc, roots, n_roots, tol, depth + 1, tc);
        isolate_roots<N>(fvec, svec, c, b, sc, sb, roots, n_roots, tol, depth + 1, tc);
    } else if (n_rts == 1) {
        ++tc.leaves;
        ridders_method_newton<N>(fvec, a, b, roots, n_roots, tol);
    }
}

// real roots of sum_i coeffs[i] x^i (ascending; degree N), ascending
template <int N> int bisect_sturm(const double *coeffs, double *roots, double tol = 1e-10) {
    if (coeffs[N] == 0.0) return 0;
    double fvec[2 * N + 1];
    double svec[3 * N];
    for (int i = 0; i <= N; ++i) fvec[i] = coeffs[i];
    const double c_inv = 1.0 / fvec[N];
    for (int i = 0; i < N; ++i) fvec[i] *= c_inv;
    fvec[N] = 1.0;
    for (int i = 0; i < N - 1; ++i) fvec[N + 1 + i] = fvec[i + 1] * ((i + 1) / static_cast<double>(N));
    fvec[2 * N] = 1.0;
    // (guard of this restatement: a non-finite coefficient gives no roots)
    for (int i = 0; i <= 2 * N; ++i)
        if (!std::isfinite(fvec[i])) return 0;
    build_sturm_seq<N>(fvec, svec);
    const double r_max = get_bounds<N>(fvec);
    const double a = -r_max, b = r_max;
    const int sa = signchanges<N>(svec, a);
    const int sb = signchanges<N>(svec, b);
    if (sa - sb == 0) return 0;
    int n_roots = 0;
    TreeCount tc;
    isolate_roots<N>(fvec, svec, a, b, sa, sb, roots, n_roots, tol, 0, tc);
    // capacity rule of the GPU walk (group_bisect.h): more than 16 intervals at one depth
    // or more than 16 leaves -- never with counts that do not increase along the line,
    // where a degree-N polynomial has at most N / 2 and N -- give no roots
    if (tc.leaves > 16) return 0;
    for (int d = 0; d <= 300; ++d)
        if (tc.pend[d] > 16) return 0;
    return n_roots;
}

} // namespace sturm

// PoseLib misc/univariate.cc solve_cubic_real: real roots of x^3 + c2 x^2 + c1 x + c0
int solve_cubic_real(double c2, double c1, double c0, double roots[3]) {
    double a = c1 - c2 * c2 / 3.0;
    double b = (2.0 * c2 * c2 * c2 - 9.0 * c2 * c1) / 27.0 + c0;
    double c = b * b / 4.0 + a * a * a / 27.0;
    int n_roots;
    if (c > 0) {
        c = std::sqrt(c);
        b *= -0.5;
        roots[0] = std::cbrt(b + c) + std::cbrt(b - c) - c2 / 3.0;
        n_roots = 1;
    } else {
        c = 3.0 * b / (2.0 * a) * std::sqrt(-3.0 / a);
        const double d = 2.0 * std::sqrt(-a / 3.0);
        const double theta = std::acos(c) / 3.0;
        roots[0] = d * std::cos(theta) - c2 / 3.0;
        roots[1] = d * std::cos(theta - 2.0 * M_PI / 3.0) - c2 / 3.0;
        roots[2] = d * std::cos(theta - 4.0 * M_PI / 3.0) - c2 / 3.0;
        n_roots = 3;
    }
    // one Newton step per root
    for (int i = 0; i < n_roots; ++i) {
        const double x = roots[i];
        const double x2 = x * x;
        const double x3 = x * x2;
        const double dx = -(x3 + c2 * x2 + c1 * x + c0) / (3 * x2 + 2 * c2 * x + c1);
        roots[i] += dx;
    }
    return n_roots;
}

namespace {

// ---- polynomials in (x, y, z) of degree <= 3, Nister's monomial columns ----
// 0 x3, 1 y3, 2 x2y, 3 xy2, 4 x2z, 5 x2, 6 y2z, 7 y2, 8 xyz, 9 xy,
// 10 xz2, 11 xz, 12 x, 13 yz2, 14 yz, 15 y, 16 z3, 17 z2, 18 z, 19 1
int mono_col(int i, int j, int k) {
    if (i == 3) return 0;
    if (j == 3) return 1;
    if (i == 2 && j == 1) return 2;
    if (i == 1 && j == 2) return 3;
    if (i == 2 && k == 1) return 4;
    if (i == 2) return 5;
    if (j == 2 && k == 1) return 6;
    if (j == 2) return 7;
    if (i == 1 && j == 1 && k == 1) return 8;
    if (i == 1 && j == 1) return 9;
    if (i == 1 && k == 2) return 10;
    if (i == 1 && k == 1) return 11;
    if (i == 1) return 12;
    if (j == 1 && k == 2) return 13;
    if (j == 1 && k == 1) return 14;
    if (j == 1) return 15;
    if (k == 3) return 16;
    if (k == 2) return 17;
    if (k == 1) return 18;
    return 19;
}
// products of two of the linear monomials x, y, z, 1 (a <= b)
int quad_index(int a, int b) {
    if (a > b) std::swap(a, b);
    return a == 0 ? b : (a == 1 ? 4 + (b - 1) : (a == 2 ? 7 + (b - 2) : 9));
}
struct Lin {
    double c[4]; // x, y, z, 1
};
struct Quad {
    double c[10];
};
struct Cub {
    double c[20];
};
// o = a b, terms in the order i (a's monomial) outer, j inner
void lin_mul(const Lin &a, const Lin &b, Quad &o) {
    for (double &v : o.c) v = 0.0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) o.c[quad_index(i, j)] += a.c[i] * b.c[j];
}
// o += s q l, terms in the order (A <= B) of q's slot, then C of l
void quad_lin_acc(const Quad &q, const Lin &l, double s, Cub &o) {
    for (int A = 0; A < 4; ++A)
        for (int B = 0; B < 4; ++B)
            for (int C = 0; C < 4; ++C) {
                if (A > B) continue;
                const int ex = (A == 0) + (B == 0) + (C == 0), ey = (A == 1) + (B == 1) + (C == 1),
                          ez = (A == 2) + (B == 2) + (C == 2);
                o.c[mono_col(ex, ey, ez)] += s * q.c[quad_index(A, B)] * l.c[C];
            }
}

// row r of the 10 x 20 template: r = 0 det E, r = 1 + 3a + b entry (a, b) of
// 2 E E^T E - tr(E E^T) E (row a of E E^T formed alone, the same products as the full)
void template_row(const double (&N)[4][9], int r, double (&row)[20]) {
    auto lin = [&](int e) {
        Lin l;
        for (int q = 0; q < 4; ++q) l.c[q] = N[q][e];
        return l;
    };
    Cub acc;
    for (double &v : acc.c) v = 0.0;
    if (r == 0) {
        // det E = E0 (E4 E8 - E5 E7) - E1 (E3 E8 - E5 E6) + E2 (E3 E7 - E4 E6)
        auto term = [&](int i0, int i1, int i2, int i3, int i4, double sgn) {
            Quad qa, qb;
            lin_mul(lin(i1), lin(i2), qa);
            lin_mul(lin(i3), lin(i4), qb);
            for (int i = 0; i < 10; ++i) qa.c[i] -= qb.c[i];
            quad_lin_acc(qa, lin(i0), sgn, acc);
        };
        term(0, 4, 8, 5, 7, 1.0);
        term(1, 3, 8, 5, 6, -1.0);
        term(2, 3, 7, 4, 6, 1.0);
    } else {
        const int a = (r - 1) / 3, b = (r - 1) % 3;
        Quad tr;
        {
            Quad Dg[3];
            for (int d = 0; d < 3; ++d) {
                for (double &v : Dg[d].c) v = 0.0;
                for (int m = 0; m < 3; ++m) {
                    Quad t;
                    const Lin l = lin(3 * d + m);
                    lin_mul(l, l, t);
                    for (int i = 0; i < 10; ++i) Dg[d].c[i] += t.c[i];
                }
            }
            for (int i = 0; i < 10; ++i) tr.c[i] = Dg[0].c[i] + Dg[1].c[i] + Dg[2].c[i];
        }
        for (int k = 0; k < 3; ++k) {
            Quad Q;
            for (double &v : Q.c) v = 0.0;
            for (int m = 0; m < 3; ++m) {
                // (E E^T)_{min(a,k) max(a,k)}: the smaller row index's entry first
                const Lin Lk = lin(3 * k + m), La = lin(3 * a + m);
                Quad t;
                if (k < a)
                    lin_mul(Lk, La, t);
                else
                    lin_mul(La, Lk, t);
                for (int i = 0; i < 10; ++i) Q.c[i] += t.c[i];
            }
            quad_lin_acc(Q, lin(3 * k + b), 2.0, acc);
        }
        quad_lin_acc(tr, lin(3 * a + b), -1.0, acc);
    }
    for (int c = 0; c < 20; ++c) row[c] = acc.c[c];
}

// ascending polynomial product
void pmul(const double *a, int A, const double *b, int B, double *o) {
    for (int k = 0; k <= A + B; ++k) o[k] = 0.0;
    for (int i = 0; i <= A; ++i)
        for (int j = 0; j <= B; ++j) o[i + j] += a[i] * b[j];
}
double peval(const double *a, int D, double x) {
    double v = a[D];
    for (int i = D - 1; i >= 0; --i) v = v * x + a[i];
    return v;
}

struct FivePt {
    double N[4][9];
    double Bx[3][4], By[3][4], B1[3][5];
    double d10[11];
    bool ok = false;
};

// the system up to det B(z); ok = false when the elimination meets no nonzero pivot
FivePt fivept_system(const double *x1, const double *x2) {
    FivePt S;
    double Q[5][9];
    for (int i = 0; i < 5; ++i)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Q[i][3 * r + c] = x2[3 * i + r] * x1[3 * i + c];
    householder_nullspace<5>(Q, S.N);
    double M[10][20];
    for (int r = 0; r < 10; ++r) template_row(S.N, r, M[r]);
    // Gauss-Jordan with partial pivoting: the pivot of column k is the first row of
    // maximal |M[r][k]| among the rows not yet used; rows are not exchanged (logical[r]
    // = the column row r pivoted); every other row is reduced with the unscaled pivot
    // row times 1 / pivot, then the pivot row is scaled
    bool used[10] = {false, false, false, false, false, false, false, false, false, false};
    int logical[10];
    for (int k = 0; k < 10; ++k) {
        double bv = -1.0;
        int bi = -1;
        for (int r = 0; r < 10; ++r) {
            const double v = used[r] ? -1.0 : std::fabs(M[r][k]);
            if (v > bv) {
                bv = v;
                bi = r;
            }
        }
        if (!(bv > 0.0)) return S;
        double piv[20];
        for (int c = 0; c < 20; ++c) piv[c] = M[bi][c];
        const double inv = 1.0 / piv[k];
        for (int r = 0; r < 10; ++r) {
            if (r == bi) continue;
            const double f = M[r][k];
            for (int c = 0; c < 20; ++c) M[r][c] -= f * (piv[c] * inv);
        }
        for (int c = 0; c < 20; ++c) M[bi][c] *= inv;
        used[bi] = true;
        logical[bi] = k;
    }
    double red[6][10];
    for (int r = 0; r < 10; ++r)
        if (logical[r] >= 4)
            for (int c = 0; c < 10; ++c) red[logical[r] - 4][c] = M[r][10 + c];
    // B(z): rows (e - z f), (g - z h), (i - z j) of the reduced rows 4..9
    for (int q = 0; q < 3; ++q) {
        const double *ar = red[2 * q], *br = red[2 * q + 1];
        auto a = [&](int col) { return ar[col - 10]; };
        auto b = [&](int col) { return br[col - 10]; };
        S.Bx[q][0] = a(12);
        S.Bx[q][1] = a(11) - b(12);
        S.Bx[q][2] = a(10) - b(11);
        S.Bx[q][3] = -b(10);
        S.By[q][0] = a(15);
        S.By[q][1] = a(14) - b(15);
        S.By[q][2] = a(13) - b(14);
        S.By[q][3] = -b(13);
        S.B1[q][0] = a(19);
        S.B1[q][1] = a(18) - b(19);
        S.B1[q][2] = a(17) - b(18);
        S.B1[q][3] = a(16) - b(17);
        S.B1[q][4] = -b(16);
    }
    // det = Bx0 (By1 B12 - By2 B11) - By0 (Bx1 B12 - Bx2 B11) + B10 (Bx1 By2 - By1 Bx2)
    double t7a[8], t7b[8], t6a[7], t6b[7], t10[11];
    for (double &v : S.d10) v = 0.0;
    pmul(S.By[1], 3, S.B1[2], 4, t7a);
    pmul(S.By[2], 3, S.B1[1], 4, t7b);
    for (int i = 0; i < 8; ++i) t7a[i] -= t7b[i];
    pmul(S.Bx[0], 3, t7a, 7, t10);
    for (int i = 0; i < 11; ++i) S.d10[i] += t10[i];
    pmul(S.Bx[1], 3, S.B1[2], 4, t7a);
    pmul(S.Bx[2], 3, S.B1[1], 4, t7b);
    for (int i = 0; i < 8; ++i) t7a[i] -= t7b[i];
    pmul(S.By[0], 3, t7a, 7, t10);
    for (int i = 0; i < 11; ++i) S.d10[i] -= t10[i];
    pmul(S.Bx[1], 3, S.By[2], 3, t6a);
    pmul(S.By[1], 3, S.Bx[2], 3, t6b);
    for (int i = 0; i < 7; ++i) t6a[i] -= t6b[i];
    pmul(S.B1[0], 4, t6a, 6, t10);
    for (int i = 0; i < 11; ++i) S.d10[i] += t10[i];
    S.ok = true;
    return S;
}

void cross3v(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
double dot3v(const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// E of the root z: (x, y, 1) spans the null space of B(z) (the largest of the three
// cross products of its rows); false when that vector has no finite (x, y)
bool fivept_E(const FivePt &S, double z, double E[9]) {
    double Bm[3][3];
    for (int q = 0; q < 3; ++q) {
        Bm[q][0] = peval(S.Bx[q], 3, z);
        Bm[q][1] = peval(S.By[q], 3, z);
        Bm[q][2] = peval(S.B1[q], 4, z);
    }
    double v01[3], v02[3], v12[3];
    cross3v(Bm[0], Bm[1], v01);
    cross3v(Bm[0], Bm[2], v02);
    cross3v(Bm[1], Bm[2], v12);
    const double n01 = dot3v(v01, v01), n02 = dot3v(v02, v02), n12 = dot3v(v12, v12);
    const double *v = (n01 >= n02 && n01 >= n12) ? v01 : (n02 >= n12 ? v02 : v12);
    if (v[2] == 0.0) return false;
    const double x = v[0] / v[2], y = v[1] / v[2];
    for (int e = 0; e < 9; ++e) E[e] = x * S.N[0][e] + y * S.N[1][e] + z * S.N[2][e] + S.N[3][e];
    return true;
}

} // namespace

std::vector<std::array<double, 9>> relpose_5pt_E(const double *x1, const double *x2, std::vector<double> *roots_out) {
    std::vector<std::array<double, 9>> out;
    const FivePt S = fivept_system(x1, x2);
    if (roots_out) roots_out->clear();
    if (!S.ok) return out;
    double roots[10];
    const int nr = sturm::bisect_sturm<10>(S.d10, roots);
    for (int k = 0; k < nr; ++k) {
        if (roots_out) roots_out->push_back(roots[k]);
        std::array<double, 9> E;
        if (fivept_E(S, roots[k], E.data())) out.push_back(E);
    }
    return out;
}

std::vector<Model> relpose_5pt(const double *x1, const double *x2) {
    std::vector<Model> out;
    for (const auto &E : relpose_5pt_E(x1, x2, nullptr)) motion_from_essential(E.data(), x1, x2, 5, &out);
    return out;
}

std::vector<std::array<double, 9>> relpose_7pt(const double *x1, const double *x2) {
    double Q[7][9], N[2][9];
    for (int i = 0; i < 7; ++i)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Q[i][3 * r + c] = x2[3 * i + r] * x1[3 * i + c];
    householder_nullspace<7>(Q, N);
    const double *A = N[0], *B = N[1];
    // det(a A + B) by multilinearity in the rows
    auto det_rows = [](const double *a, const double *b, const double *c) {
        return a[0] * (b[1] * c[2] - b[2] * c[1]) - a[1] * (b[0] * c[2] - b[2] * c[0]) +
               a[2] * (b[0] * c[1] - b[1] * c[0]);
    };
    const double c3 = det_rows(A, A + 3, A + 6);
    double c2 = det_rows(A, A + 3, B + 6) + det_rows(A, B + 3, A + 6) + det_rows(B, A + 3, A + 6);
    double c1 = det_rows(A, B + 3, B + 6) + det_rows(B, A + 3, B + 6) + det_rows(B, B + 3, A + 6);
    double c0 = det_rows(B, B + 3, B + 6);
    const double inv_c3 = 1.0 / c3;
    c2 *= inv_c3;
    c1 *= inv_c3;
    c0 *= inv_c3;
    double roots[3];
    const int nr = solve_cubic_real(c2, c1, c0, roots);
    std::vector<std::array<double, 9>> out;
    for (int k = 0; k < nr; ++k) {
        std::array<double, 9> F;
        double nn = 0.0;
        for (int e = 0; e < 9; ++e) {
            F[e] = roots[k] * A[e] + B[e];
            nn += F[e] * F[e];
        }
        nn = std::sqrt(nn);
        for (int e = 0; e < 9; ++e) F[e] /= nn;
        out.push_back(F);
    }
    return out;
}

} // namespace oracle
