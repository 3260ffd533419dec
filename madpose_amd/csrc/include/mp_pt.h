// Point-based minimal solver for the calibrated estimator (PoseLib relpose_5pt as
// called at src/hybrid_pose_estimator.cpp:134) and the shared pose tail of the
// point solvers (triangulation + affine depth fit, :140-182).
//
// GPU formulation (one sample per thread):
//   * null space of the 5x9 epipolar system by Householder QR (registers);
//   * the ten cubic constraints det(E) = 0, 2 E E^T E - tr(E E^T) E = 0 expanded
//     over the 20 monomials in Nister's order; Gauss-Jordan on the 10x20 template;
//   * Nister's hidden-variable step: B(z) (3x3, entries of degree 3/3/4 in z),
//     det B(z) = degree-10 polynomial, real roots by Sturm bisection;
//   * (x, y) from the null vector of B(z); E -> poses by motion_from_essential and
//     cheirality on all five points (src/solver.cpp:1188-1285 restate PoseLib's).
// PoseLib is not vendored, so this solver is pinned against the oracle's
// independent Stewenius action-matrix solver (tests/test_point_solvers.py).
#pragma once
#include <utility>

#include "mp_md.h"

namespace mp {

// motion_from_essential (src/solver.cpp:1219-1285): up to 4 candidate poses, kept
// when all points pass cheirality.  Returns number of poses appended at out[k..].
// This lane tests its NP points (use[i]: present); all_ok() combines the verdicts of
// the lanes holding the sample (identity when one lane holds them all); emit(m, q)
// receives the q-th kept pose, for q < cap.
template <int NP, class All, class Emit>
MP_HD int motion_from_essential_r(const double *E, const double (&x1)[NP][3], const double (&x2)[NP][3],
                                  const bool *use, int cap, All &&all_ok, Emit &&emit) {
#pragma clang fp contract(off)
    const double c0[3] = {E[0], E[3], E[6]}, c1[3] = {E[1], E[4], E[7]}, c2[3] = {E[2], E[5], E[8]};
    double u12[3], u13[3], u23[3];
    cross3_x(c0, c1, u12);
    cross3_x(c0, c2, u13);
    cross3_x(c1, c2, u23);
    const double n12 = dot3_x(u12, u12), n13 = dot3_x(u13, u13), n23 = dot3_x(u23, u23);
    double ec[3], uu[3], nn;
    const bool use12 = (n12 > n13) && (n12 > n23);
    const bool use13 = !(n12 > n13) && (n13 > n23);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        ec[r] = (use12 || use13) ? c0[r] : c1[r];
        uu[r] = use12 ? u12[r] : (use13 ? u13[r] : u23[r]);
    }
    nn = use12 ? n12 : (use13 ? n13 : n23);
    double U1[3], U2[3], U0[3], tmp[3];
    const double en = sqrt(dot3_x(ec, ec)), un = sqrt(nn);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        U1[r] = ec[r] / en;
        U2[r] = uu[r] / un;
    }
    cross3_x(U2, U1, tmp);
#pragma unroll
    for (int r = 0; r < 3; ++r) U0[r] = -tmp[r];
    double V0[3], V1[3], V2[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        V0[j] = U1[0] * E[j] + U1[1] * E[3 + j] + U1[2] * E[6 + j];
        V1[j] = -(U0[0] * E[j] + U0[1] * E[3 + j] + U0[2] * E[6 + j]);
    }
    const double n0 = sqrt(dot3_x(V0, V0));
#pragma unroll
    for (int j = 0; j < 3; ++j) V0[j] /= n0;
    const double d = dot3_x(V0, V1);
#pragma unroll
    for (int j = 0; j < 3; ++j) V1[j] -= d * V0[j];
    const double n1 = sqrt(dot3_x(V1, V1));
#pragma unroll
    for (int j = 0; j < 3; ++j) V1[j] /= n1;
    cross3_x(V0, V1, V2);
    int added = 0;
    for (int c = 0; c < 4; ++c) {
        // signs of the candidates (c: R sign, t sign) = (+,+), (+,-), (-,-), (-,+)
        const double sr_c = c < 2 ? 1.0 : -1.0, st_c = (c == 0 || c == 3) ? 1.0 : -1.0;
        Model m;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q) m.R[3 * r + q] = sr_c * (U0[r] * V0[q] + U1[r] * V1[q]) + U2[r] * V2[q];
#pragma unroll
        for (int r = 0; r < 3; ++r) m.t[r] = st_c * U2[r];
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NP; ++i) ok = ok && (!use[i] || check_cheirality(m.R, m.t, x1[i], x2[i], 0.0));
        ok = all_ok(ok);
        if (ok && added < cap) {
            m.scale = 1.0;
            m.offset0 = m.offset1 = 0.0;
            m.focal0 = m.focal1 = 1.0;
            emit(m, added);
            ++added;
        }
    }
    return added;
}

template <int NP>
MP_HD int motion_from_essential(const double *E, const double (&x1)[NP][3], const double (&x2)[NP][3], Model *out,
                                int k, int kmax) {
    bool use[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) use[i] = true;
    return motion_from_essential_r<NP>(E, x1, x2, use, kmax - k, [](bool b) { return b; },
                                       [&](const Model &m, int q) { out[k + q] = m; });
}

// ---- monomials of degree <= 3 in (x, y, z), Nister's column order ----
// 0 x3, 1 y3, 2 x2y, 3 xy2, 4 x2z, 5 x2, 6 y2z, 7 y2, 8 xyz, 9 xy,
// 10 xz2, 11 xz, 12 x, 13 yz2, 14 yz, 15 y, 16 z3, 17 z2, 18 z, 19 1
MP_HD constexpr int mono_col(int i, int j, int k) {
    return (i == 3)                        ? 0
           : (j == 3)                      ? 1
           : (i == 2 && j == 1)            ? 2
           : (i == 1 && j == 2)            ? 3
           : (i == 2 && k == 1)            ? 4
           : (i == 2)                      ? 5
           : (j == 2 && k == 1)            ? 6
           : (j == 2)                      ? 7
           : (i == 1 && j == 1 && k == 1)  ? 8
           : (i == 1 && j == 1)            ? 9
           : (i == 1 && k == 2)            ? 10
           : (i == 1 && k == 1)            ? 11
           : (i == 1)                      ? 12
           : (j == 1 && k == 2)            ? 13
           : (j == 1 && k == 1)            ? 14
           : (j == 1)                      ? 15
           : (k == 3)                      ? 16
           : (k == 2)                      ? 17
           : (k == 1)                      ? 18
                                           : 19;
}
// linear monomials x, y, z, 1 as exponent triples
MP_HD constexpr int lin_e(int a, int v) { return (a == v) ? 1 : 0; } // a in {0,1,2,3}, v exponent slot
// quadratic monomial slots: products of two linear monomials a<=b (10 of them)
// index q(a,b) for a<=b in {x,y,z,1}
MP_HD constexpr int quad_index(int a, int b) {
    return (a > b) ? quad_index(b, a) : (a == 0 ? b : (a == 1 ? 4 + (b - 1) : (a == 2 ? 7 + (b - 2) : 9)));
}

// poly helpers on fixed layouts
struct Lin {
    double c[4];
}; // x, y, z, 1
struct Quad {
    double c[10];
}; // quad_index layout
struct Cub {
    double c[20];
}; // mono_col layout

// The products below are expanded with compile-time indices (fold expressions over
// an index sequence) rather than loops: with loop indices the output slot
// quad_index / mono_col is only constant after unrolling, which comes too late for
// the accumulators to leave private (scratch) memory.  Terms are accumulated in
// the order of the loops they replace: i outer, j inner (lin_mul); a, b >= a, c
// (quad_lin_acc).
// (no FMA contraction in these products: the 5pt root stage is the oracle's to the bit,
// kernels/group_5pt.h)
template <int K> MP_HD void lin_mul_term(const Lin &a, const Lin &b, Quad &o) {
#pragma clang fp contract(off)
    constexpr int slot = quad_index(K / 4, K % 4);
    o.c[slot] += a.c[K / 4] * b.c[K % 4];
}
template <int... K> MP_HD void lin_mul_all(const Lin &a, const Lin &b, Quad &o, std::integer_sequence<int, K...>) {
    (lin_mul_term<K>(a, b, o), ...);
}
MP_HD void lin_mul(const Lin &a, const Lin &b, Quad &o) {
    static_for<10>([&](auto i) { o.c[i] = 0.0; });
    lin_mul_all(a, b, o, std::make_integer_sequence<int, 16>());
}

template <int A, int B, int Cc> MP_HD void quad_lin_term(const Quad &q, const Lin &l, double s, Cub &o) {
#pragma clang fp contract(off)
    if constexpr (A <= B) {
        constexpr int ex = lin_e(A, 0) + lin_e(B, 0) + lin_e(Cc, 0);
        constexpr int ey = lin_e(A, 1) + lin_e(B, 1) + lin_e(Cc, 1);
        constexpr int ez = lin_e(A, 2) + lin_e(B, 2) + lin_e(Cc, 2);
        constexpr int slot = mono_col(ex, ey, ez), qs = quad_index(A, B);
        o.c[slot] += s * q.c[qs] * l.c[Cc];
    }
}
template <int... K>
MP_HD void quad_lin_all(const Quad &q, const Lin &l, double s, Cub &o, std::integer_sequence<int, K...>) {
    (quad_lin_term<K / 16, (K / 4) % 4, K % 4>(q, l, s, o), ...);
}
MP_HD void quad_lin_acc(const Quad &q, const Lin &l, double s, Cub &o) {
    quad_lin_all(q, l, s, o, std::make_integer_sequence<int, 64>());
}

// Householder null space of a K x 9 system (rows = epipolar constraints) without FMA
// contraction: the oracle's householder_nullspace<K> (oracle/src/pt_poselib.cpp) to the
// bit -- Q = H_0 .. H_{K-1} of the QR of Q^T, the basis vectors Q e_{K+b}.  The 5pt
// root stage (K = 5) and the 7pt solver (K = 7).
template <int K> MP_HD void householder_nullspace_x(const double (&Q)[K][9], double (&N)[9 - K][9]) {
#pragma clang fp contract(off)
    double A[9][K];
    static_for<K>([&](auto i) { static_for<9>([&](auto e) { A[e][i] = Q[i][e]; }); });
    double V[K][9], beta[K];
    static_for<K>([&](auto k) {
        double nrm = 0.0;
        static_for<9>([&](auto i) {
            if constexpr (i >= k) nrm += A[i][k] * A[i][k];
        });
        nrm = sqrt(nrm);
        const double alpha = (A[k][k] > 0) ? -nrm : nrm;
        double vn = 0.0;
        static_for<9>([&](auto i) {
            if constexpr (i < k) {
                V[k][i] = 0.0;
            } else {
                V[k][i] = A[i][k];
                if constexpr (i == k) V[k][i] -= alpha;
            }
            vn += V[k][i] * V[k][i];
        });
        beta[k] = (vn > 0) ? 2.0 / vn : 0.0;
        static_for<K>([&](auto j) {
            if constexpr (j >= k) {
                double d = 0.0;
                static_for<9>([&](auto i) { d += V[k][i] * A[i][j]; });
                d *= beta[k];
                static_for<9>([&](auto i) { A[i][j] -= d * V[k][i]; });
            }
        });
    });
    static_for<9 - K>([&](auto b) {
        double v[9];
        static_for<9>([&](auto i) { v[i] = (i == K + b) ? 1.0 : 0.0; });
        static_for<K>([&](auto kk) {
            constexpr int k = K - 1 - kk;
            double d = 0.0;
            static_for<9>([&](auto i) { d += V[k][i] * v[i]; });
            d *= beta[k];
            static_for<9>([&](auto i) { v[i] -= d * V[k][i]; });
        });
        static_for<9>([&](auto i) { N[b][i] = v[i]; });
    });
}

// Householder null space of the 5x9 system (rows = points), returning 4 basis
// vectors of length 9 (E row-major coefficients).
MP_HD void nullspace_5x9(const double (&Q)[5][9], double (&N)[4][9]) {
    // (compile-time indices throughout: see static_for in mp_types.h)
    double A[9][5]; // Q^T
    static_for<5>([&](auto i) { static_for<9>([&](auto e) { A[e][i] = Q[i][e]; }); });
    double V[5][9], beta[5];
    static_for<5>([&](auto k) {
        double nrm = 0.0;
        static_for<9>([&](auto i) {
            if constexpr (i >= k) nrm += A[i][k] * A[i][k];
        });
        nrm = sqrt(nrm);
        const double alpha = (A[k][k] > 0) ? -nrm : nrm;
        double vn = 0.0;
        static_for<9>([&](auto i) {
            if constexpr (i < k) {
                V[k][i] = 0.0;
            } else {
                V[k][i] = A[i][k];
                if constexpr (i == k) V[k][i] -= alpha;
            }
            vn += V[k][i] * V[k][i];
        });
        beta[k] = (vn > 0) ? 2.0 / vn : 0.0;
        static_for<5>([&](auto j) {
            if constexpr (j >= k) {
                double d = 0.0;
                static_for<9>([&](auto i) { d += V[k][i] * A[i][j]; });
                d *= beta[k];
                static_for<9>([&](auto i) { A[i][j] -= d * V[k][i]; });
            }
        });
    });
    // columns 5..8 of Q = H0 H1 H2 H3 H4 applied to unit vectors
    static_for<4>([&](auto b) {
        double v[9];
        static_for<9>([&](auto i) { v[i] = (i == 5 + b) ? 1.0 : 0.0; });
        static_for<5>([&](auto kk) {
            constexpr int k = 4 - kk;
            double d = 0.0;
            static_for<9>([&](auto i) { d += V[k][i] * v[i]; });
            d *= beta[k];
            static_for<9>([&](auto i) { v[i] -= d * V[k][i]; });
        });
        static_for<9>([&](auto i) { N[b][i] = v[i]; });
    });
}

// The 5-point system of one sample: null-space basis, the hidden-variable matrix
// B(z) and its degree-10 determinant (ascending coefficients).
struct FivePtSys {
    double N[4][9];
    double Bx[3][4], By[3][4], B1[3][5];
    double d10[11];
};

// Builds the system; false when the 10x20 elimination hits a zero pivot.
MP_HD bool fivept_system(const double (&x1)[5][3], const double (&x2)[5][3], FivePtSys &S) {
    double Q[5][9];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) Q[i][3 * r + c] = x2[i][r] * x1[i][c];
    double (&N)[4][9] = S.N;
    nullspace_5x9(Q, N);
    Lin E[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        E[e].c[0] = N[0][e];
        E[e].c[1] = N[1][e];
        E[e].c[2] = N[2][e];
        E[e].c[3] = N[3][e];
    }
    double M[10][20];
#pragma unroll
    for (int r = 0; r < 10; ++r)
#pragma unroll
        for (int c = 0; c < 20; ++c) M[r][c] = 0.0;
    {
        // det(E) = E0 (E4 E8 - E5 E7) - E1 (E3 E8 - E5 E6) + E2 (E3 E7 - E4 E6)
        Quad qa, qb;
        Cub det;
#pragma unroll
        for (int c = 0; c < 20; ++c) det.c[c] = 0.0;
        lin_mul(E[4], E[8], qa);
        lin_mul(E[5], E[7], qb);
#pragma unroll
        for (int i = 0; i < 10; ++i) qa.c[i] -= qb.c[i];
        quad_lin_acc(qa, E[0], 1.0, det);
        lin_mul(E[3], E[8], qa);
        lin_mul(E[5], E[6], qb);
#pragma unroll
        for (int i = 0; i < 10; ++i) qa.c[i] -= qb.c[i];
        quad_lin_acc(qa, E[1], -1.0, det);
        lin_mul(E[3], E[7], qa);
        lin_mul(E[4], E[6], qb);
#pragma unroll
        for (int i = 0; i < 10; ++i) qa.c[i] -= qb.c[i];
        quad_lin_acc(qa, E[2], 1.0, det);
#pragma unroll
        for (int c = 0; c < 20; ++c) M[0][c] = det.c[c];
    }
    {
        Quad EEt[6]; // symmetric: (0,0) (0,1) (0,2) (1,1) (1,2) (2,2)
        const int sr[6] = {0, 0, 0, 1, 1, 2}, sc[6] = {0, 1, 2, 1, 2, 2};
#pragma unroll
        for (int p = 0; p < 6; ++p) {
#pragma unroll
            for (int i = 0; i < 10; ++i) EEt[p].c[i] = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                Quad t;
                lin_mul(E[3 * sr[p] + k], E[3 * sc[p] + k], t);
#pragma unroll
                for (int i = 0; i < 10; ++i) EEt[p].c[i] += t.c[i];
            }
        }
        Quad tr;
#pragma unroll
        for (int i = 0; i < 10; ++i) tr.c[i] = EEt[0].c[i] + EEt[3].c[i] + EEt[5].c[i];
        const int symidx[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                Cub e;
#pragma unroll
                for (int i = 0; i < 20; ++i) e.c[i] = 0.0;
#pragma unroll
                for (int k = 0; k < 3; ++k) quad_lin_acc(EEt[symidx[r][k]], E[3 * k + c], 2.0, e);
                quad_lin_acc(tr, E[3 * r + c], -1.0, e);
#pragma unroll
                for (int i = 0; i < 20; ++i) M[1 + 3 * r + c][i] = e.c[i];
            }
    }
    // Gauss-Jordan on the first 10 columns (partial pivoting by rows)
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        int p = k;
        double best = fabs(M[k][k]);
#pragma unroll
        for (int r = k + 1; r < 10; ++r)
            if (fabs(M[r][k]) > best) {
                best = fabs(M[r][k]);
                p = r;
            }
        if (!(best > 0.0)) return false;
#pragma unroll
        for (int r = k + 1; r < 10; ++r)
            if (r == p) {
#pragma unroll
                for (int c = 0; c < 20; ++c) {
                    const double t = M[k][c];
                    M[k][c] = M[r][c];
                    M[r][c] = t;
                }
            }
        const double inv = 1.0 / M[k][k];
#pragma unroll
        for (int c = 0; c < 20; ++c) M[k][c] *= inv;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            if (r != k) {
                const double f = M[r][k];
#pragma unroll
                for (int c = 0; c < 20; ++c) M[r][c] -= f * M[k][c];
            }
        }
    }
    // B(z): rows (e - z f), (g - z h), (i - z j)
    double (&Bx)[3][4] = S.Bx;
    double (&By)[3][4] = S.By;
    double (&B1)[3][5] = S.B1;
    const int ra[3] = {4, 6, 8}, rb[3] = {5, 7, 9};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const double *a = M[ra[q]], *b = M[rb[q]];
        Bx[q][0] = a[12];
        Bx[q][1] = a[11] - b[12];
        Bx[q][2] = a[10] - b[11];
        Bx[q][3] = -b[10];
        By[q][0] = a[15];
        By[q][1] = a[14] - b[15];
        By[q][2] = a[13] - b[14];
        By[q][3] = -b[13];
        B1[q][0] = a[19];
        B1[q][1] = a[18] - b[19];
        B1[q][2] = a[17] - b[18];
        B1[q][3] = a[16] - b[17];
        B1[q][4] = -b[16];
    }
    // det = Bx0 (By1 B12 - B11 By2) - By0 (Bx1 B12 - B11 Bx2) + B10 (Bx1 By2 - By1 Bx2)
    double t7a[8], t7b[8], t6a[7], t6b[7];
    double (&d10)[11] = S.d10;
#pragma unroll
    for (int i = 0; i < 11; ++i) d10[i] = 0.0;
    double t10[11];
    pmul<3, 4>(By[1], B1[2], t7a);
    pmul<3, 4>(By[2], B1[1], t7b);
#pragma unroll
    for (int i = 0; i < 8; ++i) t7a[i] -= t7b[i];
    pmul<3, 7>(Bx[0], t7a, t10);
#pragma unroll
    for (int i = 0; i < 11; ++i) d10[i] += t10[i];
    pmul<3, 4>(Bx[1], B1[2], t7a);
    pmul<3, 4>(Bx[2], B1[1], t7b);
#pragma unroll
    for (int i = 0; i < 8; ++i) t7a[i] -= t7b[i];
    pmul<3, 7>(By[0], t7a, t10);
#pragma unroll
    for (int i = 0; i < 11; ++i) d10[i] -= t10[i];
    pmul<3, 3>(Bx[1], By[2], t6a);
    pmul<3, 3>(By[1], Bx[2], t6b);
#pragma unroll
    for (int i = 0; i < 7; ++i) t6a[i] -= t6b[i];
    pmul<4, 6>(B1[0], t6a, t10);
#pragma unroll
    for (int i = 0; i < 11; ++i) d10[i] += t10[i];
    return true;
}

// Essential matrix of one real root z of det B(z): (x, y) from the null vector of
// B(z).  False when the null vector has no finite (x, y).
MP_HD bool fivept_E_for_root(const FivePtSys &S, double z, double *Ee) {
    double Bm[3][3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        Bm[q][0] = peval<3>(S.Bx[q], z);
        Bm[q][1] = peval<3>(S.By[q], z);
        Bm[q][2] = peval<4>(S.B1[q], z);
    }
    double v01[3], v02[3], v12[3];
    cross3(Bm[0], Bm[1], v01);
    cross3(Bm[0], Bm[2], v02);
    cross3(Bm[1], Bm[2], v12);
    const double n01 = dot3(v01, v01), n02 = dot3(v02, v02), n12 = dot3(v12, v12);
    double v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = (n01 >= n02 && n01 >= n12) ? v01[c] : (n02 >= n12 ? v02[c] : v12[c]);
    if (v[2] == 0.0) return false;
    const double x = v[0] / v[2], y = v[1] / v[2];
#pragma unroll
    for (int e = 0; e < 9; ++e) Ee[e] = x * S.N[0][e] + y * S.N[1][e] + z * S.N[2][e] + S.N[3][e];
    return true;
}

// Poses of one real root: E, then motion_from_essential with cheirality on the five
// points.  Appends at out[k..].
MP_HD int fivept_poses_for_root(const FivePtSys &S, double z, const double (&x1)[5][3], const double (&x2)[5][3],
                                Model *out, int k, int kmax) {
    double Ee[9];
    if (!fivept_E_for_root(S, z, Ee)) return 0;
    return motion_from_essential<5>(Ee, x1, x2, out, k, kmax);
}

// relpose_5pt on unit bearings; returns number of poses written (<= kmax).
MP_HD int relpose_5pt(const double (&x1)[5][3], const double (&x2)[5][3], Model *out, int kmax) {
    FivePtSys S;
    if (!fivept_system(x1, x2, S)) return 0;
    double roots[10];
    const int nr = sturm_real_roots<10>(S.d10, roots);
    int nout = 0;
    for (int r = 0; r < nr; ++r) nout += fivept_poses_for_root(S, roots[r], x1, x2, out, nout, kmax);
    return nout;
}

// DLT triangulation (src/utils.h:24-38) with P0 = diag(fa,fa,1)[I|0], P1 = diag(fb,fb,1)[R|t],
// the null vector by Householder QR + inverse iteration (dlt_null4), no FMA contraction --
// the oracle's triangulate_point_qr (oracle/src/pt.cpp) to the bit.  (The reference takes
// it from Eigen's JacobiSVD, src/utils.h:34; a bitwise restatement of that on the device
// made the calibrated tail 19 -> 79 us per launch, +0.9 ms of GPU solve per pair,
// profiles/r06/exact1 -- the two agree to ~1e-12, and Eigen is absent here either way.)
MP_HD void triangulate(const double *R, const double *t, double fa, double fb, const double *p0, const double *p1,
                       double *X) {
#pragma clang fp contract(off)
    double P1[3][4];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double kr = (r < 2) ? fb : 1.0;
#pragma unroll
        for (int c = 0; c < 3; ++c) P1[r][c] = kr * R[3 * r + c];
        P1[r][3] = kr * t[r];
    }
    const double P0[3][4] = {{fa, 0, 0, 0}, {0, fa, 0, 0}, {0, 0, 1, 0}};
    double A[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        A[0][j] = p0[0] * P0[2][j] - P0[0][j];
        A[1][j] = p0[1] * P0[2][j] - P0[1][j];
        A[2][j] = p1[0] * P1[2][j] - P1[0][j];
        A[3][j] = p1[1] * P1[2][j] - P1[1][j];
    }
    double v[4];
    dlt_null4(A, v);
    X[0] = v[0] / v[3];
    X[1] = v[1] / v[3];
    X[2] = v[2] / v[3];
}

// Least-squares z ~ a d + b over the points with use[i] (src/hybrid_pose_estimator.cpp
// :160-167, the 2x2 normal equations solved in closed form).  Local sums go through
// sum() (identity for one lane holding all n points, a group all-reduce when every
// lane holds one point).
template <int K, class Sum>
MP_HD void ls_affine(const double *d, const double *z, const bool *use, double n, Sum &&sum, double *a, double *b) {
#pragma clang fp contract(off)
    double sdd = 0, sd = 0, sz = 0, sdz = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        sdd += use[i] ? d[i] * d[i] : 0.0;
        sd += use[i] ? d[i] : 0.0;
        sz += use[i] ? z[i] : 0.0;
        sdz += use[i] ? d[i] * z[i] : 0.0;
    }
    sdd = sum(sdd);
    sd = sum(sd);
    sz = sum(sz);
    sdz = sum(sdz);
    const double det = sdd * n - sd * sd;
    *a = (n * sdz - sd * sz) / det;
    *b = (sdd * sz - sd * sdz) / det;
}

// Triangulate the sample with a candidate pose and fit (scale, offsets) to the depth
// priors (src/hybrid_pose_estimator.cpp:136-182; sf :93-126; tf :148-181).
// p0/p1: 2-D image coordinates (calibrated for cal, normalized pixels for sf/tf) of
// the K points this lane holds (use[i]: point present), n: points of the sample over
// all lanes, sum(): the reduction of local sums over the lanes holding the sample.
template <int K, class Sum>
MP_HD bool point_model_tail_r(const double (&p0)[K][2], const double (&p1)[K][2], const double *dd0, const double *dd1,
                              const bool *use, double n, double fa, double fb, bool use_shift,
                              bool min_depth_constraint, const double *min_depth, Model &m, Sum &&sum) {
#pragma clang fp contract(off)
    double X[K][3], z[K];
#pragma unroll
    for (int j = 0; j < K; ++j) triangulate(m.R, m.t, fa, fb, p0[j], p1[j], X[j]);
    double t[3] = {m.t[0], m.t[1], m.t[2]};
    // (the depth fit's outputs are written to m once, at the end: assigned in both
    // branches they kept three fields of m in scratch on the device)
    double sc_o, o0_o, o1_o;
    if (!use_shift) {
        double num = 0, den = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            num += use[j] ? dd0[j] * X[j][2] : 0.0;
            den += use[j] ? dd0[j] * dd0[j] : 0.0;
        }
        const double s0 = sum(num) / sum(den);
#pragma unroll
        for (int c = 0; c < 3; ++c) t[c] /= s0;
        num = den = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double q[3] = {X[j][0] / s0, X[j][1] / s0, X[j][2] / s0};
            const double zz = m.R[6] * q[0] + m.R[7] * q[1] + m.R[8] * q[2] + t[2];
            num += use[j] ? dd1[j] * zz : 0.0;
            den += use[j] ? dd1[j] * dd1[j] : 0.0;
        }
        sc_o = sum(num) / sum(den);
        o0_o = o1_o = 0.0;
    } else {
#pragma unroll
        for (int j = 0; j < K; ++j) z[j] = X[j][2];
        double s0, b0;
        ls_affine<K>(dd0, z, use, n, sum, &s0, &b0);
        const double offset0 = b0 / s0;
        if (min_depth_constraint && offset0 < -min_depth[0]) return false;
#pragma unroll
        for (int c = 0; c < 3; ++c) t[c] /= s0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double q[3] = {X[j][0] / s0, X[j][1] / s0, X[j][2] / s0};
            z[j] = m.R[6] * q[0] + m.R[7] * q[1] + m.R[8] * q[2] + t[2];
        }
        double sc, b1;
        ls_affine<K>(dd1, z, use, n, sum, &sc, &b1);
        const double offset1 = b1 / sc;
        if (min_depth_constraint && offset1 < -min_depth[1]) return false;
        sc_o = sc;
        o0_o = offset0;
        o1_o = offset1;
    }
    m.scale = sc_o;
    m.offset0 = o0_o;
    m.offset1 = o1_o;
    m.t[0] = t[0];
    m.t[1] = t[1];
    m.t[2] = t[2];
    return true;
}

// all K points in this lane
template <int K>
MP_HD bool point_model_tail(const double (&p0)[K][2], const double (&p1)[K][2], const double *dd0, const double *dd1,
                            double fa, double fb, bool use_shift, bool min_depth_constraint, const double *min_depth,
                            Model &m) {
    bool use[K];
#pragma unroll
    for (int j = 0; j < K; ++j) use[j] = true;
    return point_model_tail_r<K>(p0, p1, dd0, dd1, use, (double)K, fa, fb, use_shift, min_depth_constraint, min_depth,
                                 m, [](double v) { return v; });
}

} // namespace mp
