// ORACLE -- test infrastructure only.
//
// Monocular-depth (MD) minimal solvers, restated.
//
// The reference builds Groebner-basis elimination templates (12x12 / 36x36 / 40x40,
// src/solver.cpp:35-480) for the "affine depth" systems.  The polynomial systems
// themselves are: for every point pair (i,j) used by the template, rigid motion
// preserves the distance between the two back-projected points,
//     | (d1_i+b1) K0^-1 x_i - (d1_j+b1) K0^-1 x_j |^2
//   = a2^2 | (d2_i+beta) K1^-1 y_i - (d2_j+beta) K1^-1 y_j |^2 ,      beta = b2/a2
// with pairs (0,1),(0,2),(1,2) for the calibrated 3-point case
// (coeffs[0..17], src/solver.cpp:45-74), (0,1),(0,2),(1,2),(0,3) for the shared
// focal case (coeffs[0..31], :144-215) and additionally (1,3) for the two-focal
// case (coeffs[0..39], :311-400).  Pixel coordinates are pre-scaled by the mean
// absolute coordinate exactly as the reference does (:134-138, :302-305).
//
// This oracle solves the same systems by linear elimination of the monomials that
// appear linearly, which leaves
//   cal: a quartic in b1                        (4 solutions, = the 4x4 action matrix)
//   sf : a degree-8 resultant in w = f0^2/f^2   (8 solutions, = the 8x8 action matrix)
//   tf : a quartic in w1 from two conics        (4 solutions, = the 4x4 action matrix)
// whose real roots (companion matrix + Francis QR, wi == 0 exactly, the same
// real-Schur convention as Eigen::EigenSolver) are polished with Newton steps on the
// original distance equations.  The solution sets agree with the reference
// prototypes to ~1e-12 (tests/test_oracle_cpu.py::test_oracle_md_matches_reference_goldens pins this against
// tests/golden/md_solvers.npz).  Root filters follow the reference:
// tf/sf skip negative focal terms (:283, :470); roots with a2^2 <= 0 would give
// NaN scales in the reference and are dropped here (they never survive the
// positivity test of the pose stage, :503-504).
#include <algorithm>
#include <cmath>
#include <cstdio>

#include "la.h"
#include "oracle.h"

namespace oracle {

namespace {

struct PairTerms {
    double A[3]; // |dx|^2, 2 e.dx, |e|^2   for image 0 (unknown b1)
    double B[3]; // same for image 1 (unknown beta)
    double dz0, dz1; // (d0_i - d0_j)^2, (d1_i - d1_j)^2
};

// full 3-component variant (calibrated: homogeneous calibrated rays)
PairTerms pair_terms3(const double *x, const double *y, const double *dx, const double *dy, int i, int j) {
    PairTerms p{};
    double ax[3], ex[3], ay[3], ey[3];
    for (int c = 0; c < 3; ++c) {
        ax[c] = x[3 * i + c] - x[3 * j + c];
        ex[c] = dx[i] * x[3 * i + c] - dx[j] * x[3 * j + c];
        ay[c] = y[3 * i + c] - y[3 * j + c];
        ey[c] = dy[i] * y[3 * i + c] - dy[j] * y[3 * j + c];
    }
    for (int c = 0; c < 3; ++c) {
        p.A[0] += ax[c] * ax[c];
        p.A[1] += 2 * ex[c] * ax[c];
        p.A[2] += ex[c] * ex[c];
        p.B[0] += ay[c] * ay[c];
        p.B[1] += 2 * ey[c] * ay[c];
        p.B[2] += ey[c] * ey[c];
    }
    return p;
}

// xy-only variant with separate depth-difference terms (focal unknown)
PairTerms pair_terms2(const double *x, const double *y, const double *dx, const double *dy, int i, int j) {
    PairTerms p{};
    double ax[2], ex[2], ay[2], ey[2];
    for (int c = 0; c < 2; ++c) {
        ax[c] = x[3 * i + c] - x[3 * j + c];
        ex[c] = dx[i] * x[3 * i + c] - dx[j] * x[3 * j + c];
        ay[c] = y[3 * i + c] - y[3 * j + c];
        ey[c] = dy[i] * y[3 * i + c] - dy[j] * y[3 * j + c];
    }
    for (int c = 0; c < 2; ++c) {
        p.A[0] += ax[c] * ax[c];
        p.A[1] += 2 * ex[c] * ax[c];
        p.A[2] += ex[c] * ex[c];
        p.B[0] += ay[c] * ay[c];
        p.B[1] += 2 * ey[c] * ay[c];
        p.B[2] += ey[c] * ey[c];
    }
    p.dz0 = (dx[i] - dx[j]) * (dx[i] - dx[j]);
    p.dz1 = (dy[i] - dy[j]) * (dy[i] - dy[j]);
    return p;
}

// --- tiny polynomial helpers (ascending coefficients) ---
typedef std::vector<double> Poly;
Poly padd(const Poly &a, const Poly &b) {
    Poly r(std::max(a.size(), b.size()), 0.0);
    for (size_t i = 0; i < a.size(); ++i) r[i] += a[i];
    for (size_t i = 0; i < b.size(); ++i) r[i] += b[i];
    return r;
}
Poly psub(const Poly &a, const Poly &b) {
    Poly r(std::max(a.size(), b.size()), 0.0);
    for (size_t i = 0; i < a.size(); ++i) r[i] += a[i];
    for (size_t i = 0; i < b.size(); ++i) r[i] -= b[i];
    return r;
}
Poly pmul(const Poly &a, const Poly &b) {
    Poly r(a.size() + b.size() - 1, 0.0);
    for (size_t i = 0; i < a.size(); ++i)
        for (size_t j = 0; j < b.size(); ++j) r[i + j] += a[i] * b[j];
    return r;
}
Poly pscale(const Poly &a, double s) {
    Poly r = a;
    for (double &e : r) e *= s;
    return r;
}
double peval(const Poly &a, double x) {
    double v = 0;
    for (int i = (int)a.size() - 1; i >= 0; --i) v = v * x + a[i];
    return v;
}

// Resultant (in s) of  al2 s^2 + al1 s + al0  and  be2 s^2 + be1 s + be0, plus the
// polynomials needed to recover s at a common root:
//   X = al2 be0 - al0 be2,  Y = al2 be1 - al1 be2,  Z = al1 be0 - al0 be1,
//   Res = X^2 - Y Z, and s = -X/Y at a common root.
void quad_resultant(const Poly &al0, const Poly &al1, const Poly &al2, const Poly &be0, const Poly &be1,
                    const Poly &be2, Poly *X, Poly *Y, Poly *res) {
    *X = psub(pmul(al2, be0), pmul(al0, be2));
    *Y = psub(pmul(al2, be1), pmul(al1, be2));
    Poly Z = psub(pmul(al1, be0), pmul(al0, be1));
    *res = psub(pmul(*X, *X), pmul(*Y, Z));
}

// Newton polishing of F(z) = 0 (square system); keeps the iterate with the
// smallest residual.
template <class FJ> void newton_polish(int n, double *z, FJ fj) {
    std::vector<double> F(n), best(z, z + n);
    Mat J(n, n);
    fj(z, F.data(), &J);
    double rbest = 0;
    for (double f : F) rbest += f * f;
    for (int it = 0; it < 3; ++it) {
        Mat Fm(n, 1), dz;
        for (int i = 0; i < n; ++i) Fm(i, 0) = F[i];
        if (!lu_full_solve(J, Fm, &dz)) break;
        std::vector<double> zn(n);
        for (int i = 0; i < n; ++i) zn[i] = z[i] - dz(i, 0);
        Mat Jn(n, n);
        std::vector<double> Fn(n);
        fj(zn.data(), Fn.data(), &Jn);
        double r = 0;
        for (double f : Fn) r += f * f;
        if (!(r < rbest)) break;
        rbest = r;
        for (int i = 0; i < n; ++i) z[i] = zn[i];
        F = Fn;
        J = Jn;
    }
}

std::vector<std::vector<double>> solve_cal(const double *x, const double *y, const double *dx, const double *dy) {
    // unknowns b1, beta, s=a2^2 ; equation per pair: A.[b1^2,b1,1] - s B.[beta^2,beta,1] = 0
    const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
    PairTerms T[3];
    for (int k = 0; k < 3; ++k) T[k] = pair_terms3(x, y, dx, dy, pr[k][0], pr[k][1]);
    // linear elimination: [-B] w = -A u,  w = (s beta^2, s beta, s), u = (b1^2, b1, 1)
    Mat Q(3, 3), Pm(3, 3), L;
    for (int k = 0; k < 3; ++k)
        for (int c = 0; c < 3; ++c) {
            Q(k, c) = T[k].B[c];
            Pm(k, c) = T[k].A[c];
        }
    std::vector<std::vector<double>> out;
    if (!qr_solve(Q, Pm, &L)) return out; // w = L u
    // (s beta)^2 = (s beta^2) s  ->  quartic in b1
    Poly l0 = {L(0, 2), L(0, 1), L(0, 0)}, l1 = {L(1, 2), L(1, 1), L(1, 0)}, l2 = {L(2, 2), L(2, 1), L(2, 0)};
    Poly quart = psub(pmul(l1, l1), pmul(l0, l2));
    std::vector<double> roots = poly_real_roots(quart);
    std::sort(roots.begin(), roots.end());
    for (double b1 : roots) {
        double s = peval(l2, b1);
        double beta = peval(l1, b1) / s;
        double z[3] = {b1, beta, s};
        newton_polish(3, z, [&](const double *v, double *F, Mat *J) {
            for (int k = 0; k < 3; ++k) {
                const double *A = T[k].A, *B = T[k].B;
                double ub = A[0] * v[0] * v[0] + A[1] * v[0] + A[2];
                double vb = B[0] * v[1] * v[1] + B[1] * v[1] + B[2];
                F[k] = ub - v[2] * vb;
                (*J)(k, 0) = 2 * A[0] * v[0] + A[1];
                (*J)(k, 1) = -v[2] * (2 * B[0] * v[1] + B[1]);
                (*J)(k, 2) = -vb;
            }
        });
        if (!(z[2] > 0)) continue;
        double a2 = std::sqrt(z[2]);
        out.push_back({1.0, z[0], a2, z[1] * a2});
    }
    return out;
}

void prescale(const double *x, const double *y, double fx, double fy, double *xs, double *ys, int k) {
    for (int i = 0; i < k; ++i) {
        xs[3 * i] = x[3 * i] / fx;
        xs[3 * i + 1] = x[3 * i + 1] / fx;
        xs[3 * i + 2] = x[3 * i + 2];
        ys[3 * i] = y[3 * i] / fy;
        ys[3 * i + 1] = y[3 * i + 1] / fy;
        ys[3 * i + 2] = y[3 * i + 2];
    }
}

double mean_abs_xy(const double *x, int k) {
    double s = 0;
    for (int i = 0; i < k; ++i) s += std::fabs(x[3 * i]) + std::fabs(x[3 * i + 1]);
    return s / (2 * k);
}

std::vector<std::vector<double>> solve_sf(const double *x0, const double *y0, const double *dx, const double *dy) {
    // src/solver.cpp:134-138 focal pre-scaling
    const double f0 = 0.5 * (mean_abs_xy(x0, 4) + mean_abs_xy(y0, 4));
    double x[12], y[12];
    prescale(x0, y0, f0, f0, x, y, 4);
    // equation per pair:  w A.u + dz0  -  s ( w B.v + dz1 ) = 0 ,  w = 1/f^2, t = s w
    // monomials (w b1^2, w b1, t beta^2, t beta) solved linearly in terms of (w, t, s, 1)
    const int pr[4][2] = {{0, 1}, {0, 2}, {1, 2}, {0, 3}};
    PairTerms T[4];
    Mat M(4, 4), Rh(4, 4), L;
    for (int k = 0; k < 4; ++k) {
        T[k] = pair_terms2(x, y, dx, dy, pr[k][0], pr[k][1]);
        M(k, 0) = T[k].A[0];
        M(k, 1) = T[k].A[1];
        M(k, 2) = -T[k].B[0];
        M(k, 3) = -T[k].B[1];
        Rh(k, 0) = -T[k].A[2]; // w
        Rh(k, 1) = T[k].B[2];  // t
        Rh(k, 2) = T[k].dz1;   // s
        Rh(k, 3) = -T[k].dz0;  // 1
    }
    std::vector<std::vector<double>> out;
    if (!qr_solve(M, Rh, &L)) return out;
    // L row r: monomial_r = L(r,0) w + L(r,1) t + L(r,2) s + L(r,3); substitute t = s w:
    // monomial_r = q0(w) + s q1(w),  q0 = L3 + L0 w,  q1 = L2 + L1 w
    Poly q0[4], q1[4];
    for (int r = 0; r < 4; ++r) {
        q0[r] = {L(r, 3), L(r, 0)};
        q1[r] = {L(r, 2), L(r, 1)};
    }
    const Poly W = {0.0, 1.0};
    // E1: (w b1)^2 - (w b1^2) w = 0 ; E2: (t beta)^2 - (t beta^2) s w = 0 ; both quadratic in s
    Poly al0 = psub(pmul(q0[1], q0[1]), pmul(q0[0], W));
    Poly al1 = psub(pscale(pmul(q0[1], q1[1]), 2.0), pmul(q1[0], W));
    Poly al2 = pmul(q1[1], q1[1]);
    Poly be0 = pmul(q0[3], q0[3]);
    Poly be1 = psub(pscale(pmul(q0[3], q1[3]), 2.0), pmul(q0[2], W));
    Poly be2 = psub(pmul(q1[3], q1[3]), pmul(q1[2], W));
    Poly X, Y, res;
    quad_resultant(al0, al1, al2, be0, be1, be2, &X, &Y, &res);
    std::vector<double> roots = poly_real_roots(res);
    std::sort(roots.begin(), roots.end());
    for (double w : roots) {
        double s = -peval(X, w) / peval(Y, w);
        double wb1 = peval(q0[1], w) + s * peval(q1[1], w);
        double tb = peval(q0[3], w) + s * peval(q1[3], w);
        double z[4] = {wb1 / w, tb / (s * w), s, w};
        newton_polish(4, z, [&](const double *v, double *F, Mat *J) {
            for (int k = 0; k < 4; ++k) {
                const double *A = T[k].A, *B = T[k].B;
                double ua = A[0] * v[0] * v[0] + A[1] * v[0] + A[2];
                double vb = B[0] * v[1] * v[1] + B[1] * v[1] + B[2];
                F[k] = v[3] * ua + T[k].dz0 - v[2] * (v[3] * vb + T[k].dz1);
                (*J)(k, 0) = v[3] * (2 * A[0] * v[0] + A[1]);
                (*J)(k, 1) = -v[2] * v[3] * (2 * B[0] * v[1] + B[1]);
                (*J)(k, 2) = -(v[3] * vb + T[k].dz1);
                (*J)(k, 3) = ua - v[2] * vb;
            }
        });
        if (z[3] < 0) continue; // src/solver.cpp:283
        if (!(z[2] > 0)) continue;
        double a2 = std::sqrt(z[2]);
        out.push_back({1.0, z[0], a2, z[1] * a2, f0 / std::sqrt(z[3])});
    }
    return out;
}

std::vector<std::vector<double>> solve_tf(const double *x0, const double *y0, const double *dx, const double *dy) {
    const double f1 = mean_abs_xy(x0, 4), f2 = mean_abs_xy(y0, 4); // src/solver.cpp:302-305
    double x[12], y[12];
    prescale(x0, y0, f1, f2, x, y, 4);
    // equation per pair: w1 A.u + dz0 - ( t B.v + s dz1 ) = 0,  t = s w2
    // monomials (w1 b1^2, w1 b1, t beta^2, t beta, s) linear in (w1, t, 1)
    const int pr[5][2] = {{0, 1}, {0, 2}, {1, 2}, {0, 3}, {1, 3}};
    PairTerms T[5];
    Mat M(5, 5), Rh(5, 3), L;
    for (int k = 0; k < 5; ++k) {
        T[k] = pair_terms2(x, y, dx, dy, pr[k][0], pr[k][1]);
        M(k, 0) = T[k].A[0];
        M(k, 1) = T[k].A[1];
        M(k, 2) = -T[k].B[0];
        M(k, 3) = -T[k].B[1];
        M(k, 4) = -T[k].dz1;
        Rh(k, 0) = -T[k].A[2]; // w1
        Rh(k, 1) = T[k].B[2];  // t
        Rh(k, 2) = -T[k].dz0;  // 1
    }
    std::vector<std::vector<double>> out;
    if (!qr_solve(M, Rh, &L)) return out;
    // monomial_r = q0(w1) + t q1,  q0 = L2 + L0 w1, q1 = L1 (constant)
    Poly q0[5], q1[5];
    for (int r = 0; r < 5; ++r) {
        q0[r] = {L(r, 2), L(r, 0)};
        q1[r] = {L(r, 1)};
    }
    const Poly W = {0.0, 1.0};
    // conics: (w1 b1)^2 - (w1 b1^2) w1 = 0 ; (t beta)^2 - (t beta^2) t = 0 (quadratic in t)
    Poly al0 = psub(pmul(q0[1], q0[1]), pmul(q0[0], W));
    Poly al1 = psub(pscale(pmul(q0[1], q1[1]), 2.0), pmul(q1[0], W));
    Poly al2 = pmul(q1[1], q1[1]);
    Poly be0 = pmul(q0[3], q0[3]);
    Poly be1 = psub(pscale(pmul(q0[3], q1[3]), 2.0), q0[2]);
    Poly be2 = psub(pmul(q1[3], q1[3]), q1[2]);
    Poly X, Y, res;
    quad_resultant(al0, al1, al2, be0, be1, be2, &X, &Y, &res);
    std::vector<double> roots = poly_real_roots(res);
    std::sort(roots.begin(), roots.end());
    for (double w1 : roots) {
        double t = -peval(X, w1) / peval(Y, w1);
        double m[5];
        for (int r = 0; r < 5; ++r) m[r] = peval(q0[r], w1) + t * q1[r][0];
        double s = m[4];
        // unknowns b1, beta, s, w1, w2
        double z[5] = {m[1] / w1, m[3] / t, s, w1, t / s};
        newton_polish(5, z, [&](const double *v, double *F, Mat *J) {
            for (int k = 0; k < 5; ++k) {
                const double *A = T[k].A, *B = T[k].B;
                double ua = A[0] * v[0] * v[0] + A[1] * v[0] + A[2];
                double vb = B[0] * v[1] * v[1] + B[1] * v[1] + B[2];
                F[k] = v[3] * ua + T[k].dz0 - v[2] * (v[4] * vb + T[k].dz1);
                (*J)(k, 0) = v[3] * (2 * A[0] * v[0] + A[1]);
                (*J)(k, 1) = -v[2] * v[4] * (2 * B[0] * v[1] + B[1]);
                (*J)(k, 2) = -(v[4] * vb + T[k].dz1);
                (*J)(k, 3) = ua;
                (*J)(k, 4) = -v[2] * vb;
            }
        });
        if (z[3] < 0 || z[4] < 0) continue; // src/solver.cpp:470
        if (!(z[2] > 0)) continue;
        double a2 = std::sqrt(z[2]);
        out.push_back({1.0, z[0], a2, z[1] * a2, f1 / std::sqrt(z[3]), f2 / std::sqrt(z[4])});
    }
    return out;
}

// Kabsch/Umeyama without scale: Y ~ R X + t (src/solver.cpp:506-525)
void procrustes(const double *X, const double *Y, int k, double R[9], double t[3]) {
    double cx[3] = {0, 0, 0}, cy[3] = {0, 0, 0};
    for (int i = 0; i < k; ++i)
        for (int c = 0; c < 3; ++c) {
            cx[c] += X[3 * i + c];
            cy[c] += Y[3 * i + c];
        }
    for (int c = 0; c < 3; ++c) {
        cx[c] /= k;
        cy[c] /= k;
    }
    double S[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < k; ++i)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) S[3 * a + b] += (Y[3 * i + a] - cy[a]) * (X[3 * i + b] - cx[b]);
    // Eigen::JacobiSVD<MatrixXd>(S, ComputeFullU | ComputeFullV) (src/solver.cpp:517)
    double U[9], V[9];
    eigen_jacobi_svd3(S, U, V);
    double du = det3(U), dv = det3(V);
    if (du * dv < 0)
        for (int i = 0; i < 3; ++i) U[3 * i + 2] = -U[3 * i + 2];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) {
            double s = 0;
            for (int c = 0; c < 3; ++c) s += U[3 * a + c] * V[3 * b + c];
            R[3 * a + b] = s;
        }
    for (int a = 0; a < 3; ++a) t[a] = cy[a] - (R[3 * a] * cx[0] + R[3 * a + 1] * cx[1] + R[3 * a + 2] * cx[2]);
}

} // namespace

std::vector<std::vector<double>> md_scale_shift(Variant v, const double *x, const double *y, const double *dx,
                                                const double *dy) {
    if (v == CAL) return solve_cal(x, y, dx, dy);
    if (v == SF) return solve_sf(x, y, dx, dy);
    return solve_tf(x, y, dx, dy);
}

std::vector<Model> md_pose(Variant v, const double *x, const double *y, const double *dx, const double *dy) {
    const int k = (v == CAL) ? 3 : 4;
    std::vector<Model> out;
    for (const auto &sol : md_scale_shift(v, x, y, dx, dy)) {
        double d1[4], d2[4];
        bool ok = true;
        for (int i = 0; i < k; ++i) {
            d1[i] = dx[i] + sol[1];
            d2[i] = dy[i] * sol[2] + sol[3];
            if (!(d1[i] > 0) || !(d2[i] > 0)) ok = false; // src/solver.cpp:503-504
        }
        if (!ok) continue;
        double fx = 1.0, fy = 1.0;
        if (v == SF) fx = fy = sol[4];
        if (v == TF) {
            fx = sol[4];
            fy = sol[5];
        }
        double X[12], Y[12];
        for (int i = 0; i < k; ++i) {
            X[3 * i] = x[3 * i] / fx * d1[i];
            X[3 * i + 1] = x[3 * i + 1] / fx * d1[i];
            X[3 * i + 2] = x[3 * i + 2] * d1[i];
            Y[3 * i] = y[3 * i] / fy * d2[i];
            Y[3 * i + 1] = y[3 * i + 1] / fy * d2[i];
            Y[3 * i + 2] = y[3 * i + 2] * d2[i];
        }
        Model m;
        procrustes(X, Y, k, m.R, m.t);
        m.scale = sol[2];
        m.offset0 = sol[1];
        m.offset1 = sol[3];
        if (v == SF) m.focal0 = m.focal1 = sol[4];
        if (v == TF) {
            m.focal0 = sol[4];
            m.focal1 = sol[5];
        }
        out.push_back(m);
    }
    return out;
}

Model md_pose_noshift_cal(const double *x, const double *y, const double *dx, const double *dy) {
    // src/hybrid_pose_estimator.cpp:87-120
    double p0[9], p1[9];
    for (int i = 0; i < 3; ++i)
        for (int c = 0; c < 3; ++c) {
            p0[3 * i + c] = x[3 * i + c] * dx[i];
            p1[3 * i + c] = y[3 * i + c] * dy[i];
        }
    auto dist = [](const double *a, const double *b) {
        return std::sqrt((a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]));
    };
    double v0[3] = {dist(p0, p0 + 3), dist(p0, p0 + 6), dist(p0 + 3, p0 + 6)};
    double v1[3] = {dist(p1, p1 + 3), dist(p1, p1 + 6), dist(p1 + 3, p1 + 6)};
    double scale = (v1[0] * v0[0] + v1[1] * v0[1] + v1[2] * v0[2]) / (v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2]);
    double X[9], Y[9];
    for (int i = 0; i < 3; ++i)
        for (int c = 0; c < 3; ++c) {
            X[3 * i + c] = x[3 * i + c] * dx[i];
            Y[3 * i + c] = y[3 * i + c] * (dy[i] * scale);
        }
    Model m;
    procrustes(X, Y, 3, m.R, m.t);
    m.scale = scale;
    m.offset0 = m.offset1 = 0.0;
    return m;
}

} // namespace oracle
