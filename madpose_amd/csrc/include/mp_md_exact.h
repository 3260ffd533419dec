// Monocular-depth (MD) minimal solvers, the oracle's arithmetic to the bit.
//
// Reference: src/solver.cpp:35-480 (solve_scale_and_shift*, Groebner templates +
// Eigen::EigenSolver, real roots where imag() == 0 exactly, :281, :468).  The
// restatement both this file and the oracle follow (oracle/src/md.cpp: linear
// elimination of the monomials that appear linearly, one univariate resultant,
// its real roots as the eigenvalues of the companion matrix with wi == 0 exactly --
// Eigen's real-Schur convention --, Newton polishing on the distance equations) is
// written here operation for operation as oracle/src/md.cpp and oracle/src/la.cpp
// do it (qr_solve :10-76, lu_full_solve :221-244, balance :272-305, hqr :338-461,
// poly_real_roots :474-491, newton_polish md.cpp:136-159), with FMA contraction off,
// so that a sample gives the oracle's solutions bit for bit: the same root count, so
// the estimator's hypothesis count (the headline's unit) equals the oracle's.
//
// Why not the Sturm isolation of mp_md.h: on samples whose resultant has roots
// several orders of magnitude apart (offsets of 10^2..10^5, focal ratios of 10^3),
// the floating-point Sturm chain lost roots and its "even multiplicity" midpoint
// fallback produced non-roots (profiles/r04/s6/diag_sf0.log: 7 of 50k shared-focal
// MD samples, distance residuals 0.04-0.9 against 1e-14 for the oracle's roots).
//
// Everything is register-resident: the elimination matrices, the companion matrix
// through balance + hqr and the Newton LU are fixed-size arrays whose loops unroll to
// compile-time indices, a runtime position (pivot, active QR window) selecting among
// them (a first version kept these in LDS and ran 635 us per shared-focal launch on
// LDS latency, profiles/r04/mdx/).  Only the sorted root list goes to a per-lane
// scratch column (`LaneScratch`: a lane's strided column of an LDS block on the
// device, a plain array on the host), read back by the per-root loop.  One sample
// per lane.  The code compiles for the host as well (tests/md_exact_check.cpp
// checks it against the oracle on the CPU).
#pragma once
#include <cfloat>

#include "mp_md.h"

// instrumentation hooks of the stage microbenchmark (tools/mdx_bench.hip): a balance
// pass, an hqr trip; empty in the library
#ifndef MDX_BAL_HOOK
#define MDX_BAL_HOOK()
#endif
#ifndef MDX_TRIP_HOOK
#define MDX_TRIP_HOOK()
#endif

namespace mp {

// per-lane scratch: element i at p[i * st]
struct LaneScratch {
    double *p;
    int st;
    MP_HD double &operator[](int i) const { return p[i * st]; }
};

namespace mdx {

// --- fixed-size polynomial algebra (ascending coefficients), as the oracle's Poly
// helpers (md.cpp:93-120): every output starts at 0.0 and accumulates in index order
template <int NA, int NB> MP_HD void pmul(const double (&a)[NA], const double (&b)[NB], double (&o)[NA + NB - 1]) {
#pragma clang fp contract(off)
    for (int k = 0; k < NA + NB - 1; ++k) o[k] = 0.0;
    for (int i = 0; i < NA; ++i)
        for (int j = 0; j < NB; ++j) o[i + j] += a[i] * b[j];
}
template <int NA, int NB, int NO>
MP_HD void psub(const double (&a)[NA], const double (&b)[NB], double (&o)[NO]) {
#pragma clang fp contract(off)
    static_assert(NO == (NA > NB ? NA : NB), "psub size");
    for (int i = 0; i < NO; ++i) o[i] = 0.0;
    for (int i = 0; i < NA; ++i) o[i] += a[i];
    for (int i = 0; i < NB; ++i) o[i] -= b[i];
}
template <int N> MP_HD void pscale(double (&a)[N], double s) {
#pragma clang fp contract(off)
    for (int i = 0; i < N; ++i) a[i] *= s;
}
template <int N> MP_HD double peval(const double (&a)[N], double x) {
#pragma clang fp contract(off)
    double v = 0.0;
    for (int i = N - 1; i >= 0; --i) v = v * x + a[i];
    return v;
}

// resultant in s of al2 s^2 + al1 s + al0 and be2 s^2 + be1 s + be0 (md.cpp:126-132)
template <int A0, int A1, int A2, int B0, int B1, int B2, int NX, int NY, int NZ, int NR>
MP_HD void quad_resultant(const double (&al0)[A0], const double (&al1)[A1], const double (&al2)[A2],
                          const double (&be0)[B0], const double (&be1)[B1], const double (&be2)[B2], double (&X)[NX],
                          double (&Y)[NY], double (&R)[NR]) {
    double t0[A2 + B0 - 1], t1[A0 + B2 - 1];
    pmul(al2, be0, t0);
    pmul(al0, be2, t1);
    psub(t0, t1, X);
    double u0[A2 + B1 - 1], u1[A1 + B2 - 1];
    pmul(al2, be1, u0);
    pmul(al1, be2, u1);
    psub(u0, u1, Y);
    double v0[A1 + B0 - 1], v1[A0 + B1 - 1], Z[NZ];
    pmul(al1, be0, v0);
    pmul(al0, be1, v1);
    psub(v0, v1, Z);
    double r0[2 * NX - 1], r1[NY + NZ - 1];
    pmul(X, X, r0);
    pmul(Y, Z, r1);
    psub(r0, r1, R);
}

// pair terms, xy-only with depth differences (md.cpp:69-89) or full rays (:48-66)
template <bool kXY>
MP_HD PairTerms pair_terms(const double (&x)[4][3], const double (&y)[4][3], const double *dx, const double *dy, int i,
                           int j) {
#pragma clang fp contract(off)
    PairTerms p;
    p.A[0] = p.A[1] = p.A[2] = p.B[0] = p.B[1] = p.B[2] = 0.0;
    p.dz0 = p.dz1 = 0.0;
    const int nc = kXY ? 2 : 3;
    double ax[3], ex[3], ay[3], ey[3];
    for (int c = 0; c < nc; ++c) {
        ax[c] = x[i][c] - x[j][c];
        ex[c] = dx[i] * x[i][c] - dx[j] * x[j][c];
        ay[c] = y[i][c] - y[j][c];
        ey[c] = dy[i] * y[i][c] - dy[j] * y[j][c];
    }
    for (int c = 0; c < nc; ++c) {
        p.A[0] += ax[c] * ax[c];
        p.A[1] += 2 * ex[c] * ax[c];
        p.A[2] += ex[c] * ex[c];
        p.B[0] += ay[c] * ay[c];
        p.B[1] += 2 * ey[c] * ay[c];
        p.B[2] += ey[c] * ey[c];
    }
    if (kXY) {
        p.dz0 = (dx[i] - dx[j]) * (dx[i] - dx[j]);
        p.dz1 = (dy[i] - dy[j]) * (dy[i] - dy[j]);
    }
    return p;
}

// Register-resident forms: every array index is a compile-time constant once the
// fixed-size loops are unrolled; a runtime position (a pivot, the active window of
// the QR) selects among the static elements (`opaque` keeps the selects from being
// folded back into a dynamically indexed, scratch-resident array).  Each guarded
// element update performs exactly the oracle's operations on exactly the oracle's
// operands, so the results are the same doubles.
template <int N> MP_HD double pick_diag(const double (&a)[N][N], int i, int off) {
    double v = 0.0;
#pragma unroll
    for (int r = 0; r < N; ++r) {
        const int c = r + off;
        if (c >= 0 && c < N && r == i) v = opaque(a[r][c >= 0 && c < N ? c : 0]);
    }
    return v;
}

// Householder QR with column pivoting, A X = B (la.cpp:10-76)
template <int n, int m> MP_HD bool qr_solve(double (&A)[n][n], double (&B)[n][m], double (&X)[n][m]) {
#pragma clang fp contract(off)
    int perm[n];
#pragma unroll
    for (int i = 0; i < n; ++i) perm[i] = i;
    double maxpiv = 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = -1;
#pragma unroll
        for (int j = k; j < n; ++j) {
            double s = 0;
#pragma unroll
            for (int i = k; i < n; ++i) s += A[i][j] * A[i][j];
            if (s > best) {
                best = s;
                p = j;
            }
        }
#pragma unroll
        for (int j = k + 1; j < n; ++j) {
            const bool sw = j == p;
#pragma unroll
            for (int i = 0; i < n; ++i) {
                const double ak = opaque(A[i][k]), aj = opaque(A[i][j]);
                A[i][k] = sw ? aj : ak;
                A[i][j] = sw ? ak : aj;
            }
            const int pk = perm[k], pj = perm[j];
            perm[k] = sw ? pj : pk;
            perm[j] = sw ? pk : pj;
        }
        double alpha = sqrt(best);
        if (k == 0) maxpiv = alpha;
        if (alpha <= maxpiv * 1e-15 || alpha == 0.0) return false;
        if (A[k][k] > 0) alpha = -alpha;
        double v[n];
#pragma unroll
        for (int i = k; i < n; ++i) v[i] = A[i][k];
        v[k] -= alpha;
        double vn = 0;
#pragma unroll
        for (int i = k; i < n; ++i) vn += v[i] * v[i];
        if (vn > 0) {
#pragma unroll
            for (int j = k; j < n; ++j) {
                double d = 0;
#pragma unroll
                for (int i = k; i < n; ++i) d += v[i] * A[i][j];
                d = 2 * d / vn;
#pragma unroll
                for (int i = k; i < n; ++i) A[i][j] -= d * v[i];
            }
#pragma unroll
            for (int j = 0; j < m; ++j) {
                double d = 0;
#pragma unroll
                for (int i = k; i < n; ++i) d += v[i] * B[i][j];
                d = 2 * d / vn;
#pragma unroll
                for (int i = k; i < n; ++i) B[i][j] -= d * v[i];
            }
        }
    }
    // R z = Q^T B (z in place of B), X = P z
#pragma unroll
    for (int j = 0; j < m; ++j)
#pragma unroll
        for (int i = n - 1; i >= 0; --i) {
            double s = B[i][j];
#pragma unroll
            for (int k = i + 1; k < n; ++k) s -= A[i][k] * B[k][j];
            B[i][j] = s / A[i][i];
        }
    // (a gather by selects: the scatter X[perm[i]] = B[i] stored through a selected
    // pointer, which kept X in scratch)
#pragma unroll
    for (int r = 0; r < n; ++r)
#pragma unroll
        for (int j = 0; j < m; ++j) {
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < n; ++i)
                if (perm[i] == r) v = opaque(B[i][j]);
            X[r][j] = v;
        }
    return true;
}

// LU with complete pivoting + solve of A x = b (la.cpp:78-108, 221-244)
template <int n> MP_HD bool lu_full_solve(double (&A)[n][n], const double (&b)[n], double (&x)[n]) {
#pragma clang fp contract(off)
    int rp[n], cp[n];
#pragma unroll
    for (int i = 0; i < n; ++i) rp[i] = cp[i] = i;
#pragma unroll
    for (int k = 0; k < n; ++k) {
        int pi = k, pj = k;
        double best = -1;
#pragma unroll
        for (int i = k; i < n; ++i)
#pragma unroll
            for (int j = k; j < n; ++j)
                if (fabs(A[i][j]) > best) {
                    best = fabs(A[i][j]);
                    pi = i;
                    pj = j;
                }
#pragma unroll
        for (int i = k + 1; i < n; ++i) { // rows k <-> pi
            const bool sw = i == pi;
#pragma unroll
            for (int j = 0; j < n; ++j) {
                const double ak = opaque(A[k][j]), ai = opaque(A[i][j]);
                A[k][j] = sw ? ai : ak;
                A[i][j] = sw ? ak : ai;
            }
            const int a = rp[k], c = rp[i];
            rp[k] = sw ? c : a;
            rp[i] = sw ? a : c;
        }
#pragma unroll
        for (int j = k + 1; j < n; ++j) { // columns k <-> pj
            const bool sw = j == pj;
#pragma unroll
            for (int i = 0; i < n; ++i) {
                const double ak = opaque(A[i][k]), aj = opaque(A[i][j]);
                A[i][k] = sw ? aj : ak;
                A[i][j] = sw ? ak : aj;
            }
            const int a = cp[k], c = cp[j];
            cp[k] = sw ? c : a;
            cp[j] = sw ? a : c;
        }
        if (A[k][k] != 0.0) {
#pragma unroll
            for (int i = k + 1; i < n; ++i) {
                const double l = A[i][k] / A[k][k];
                A[i][k] = l;
#pragma unroll
                for (int j = k + 1; j < n; ++j) A[i][j] -= l * A[k][j];
            }
        }
    }
    bool ok = true;
#pragma unroll
    for (int k = 0; k < n; ++k) ok = ok && A[k][k] != 0.0;
    if (!ok) return false;
    double y[n];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < n; ++r)
            if (rp[i] == r) s = opaque(b[r]);
#pragma unroll
        for (int k = 0; k < i; ++k) s -= A[i][k] * y[k];
        y[i] = s;
    }
#pragma unroll
    for (int i = n - 1; i >= 0; --i) {
        double s = y[i];
#pragma unroll
        for (int k = i + 1; k < n; ++k) s -= A[i][k] * y[k];
        y[i] = s / A[i][i];
    }
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
        for (int r = 0; r < n; ++r)
            if (cp[i] == r) x[r] = y[i];
    return true;
}

MP_HD double sign_of(double a, double b) { return b >= 0 ? fabs(a) : -fabs(a); }

// EISPACK balance (la.cpp:272-305) of the leading n x n block
template <int N> MP_HD void balance(double (&a)[N][N], int n) {
#pragma clang fp contract(off)
    const double radix = 2.0, sqrdx = 4.0;
    bool done = false;
    // (the pass and scaling caps never bind on finite data -- a scaling loop covers
    // the double range in < 1100 steps -- but keep an infinite entry from hanging a lane)
    for (int pass = 0; !done && pass < 4096; ++pass) {
        MDX_BAL_HOOK();
        done = true;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (i < n) {
                double r = 0, c = 0;
#pragma unroll
                for (int j = 0; j < N; ++j)
                    if (j < n && j != i) {
                        c += fabs(a[j][i]);
                        r += fabs(a[i][j]);
                    }
                if (c != 0.0 && r != 0.0) {
                    double g = r / radix, f = 1.0, s = c + r;
                    for (int it = 0; c < g && it < 2200; ++it) {
                        f *= radix;
                        c *= sqrdx;
                    }
                    g = r * radix;
                    for (int it = 0; c > g && it < 2200; ++it) {
                        f /= radix;
                        c /= sqrdx;
                    }
                    if ((c + r) / f < 0.95 * s) {
                        done = false;
                        g = 1.0 / f;
#pragma unroll
                        for (int j = 0; j < N; ++j)
                            if (j < n) a[i][j] *= g;
#pragma unroll
                        for (int j = 0; j < N; ++j)
                            if (j < n) a[j][i] *= f;
                    }
                }
            }
        }
    }
}

// EISPACK hqr (la.cpp:338-461) on the leading n x n block (upper Hessenberg).  The
// oracle's do / while over windows is one loop here, a trip per deflation or QR
// iteration; l, m and k are runtime positions the static loops compare against.
template <int N> MP_HD bool hqr(double (&a)[N][N], int n, double (&wr)[N], double (&wi)[N]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < N; ++i) wr[i] = wi[i] = 0.0;
    double anorm = 0.0;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = (i - 1 > 0 ? i - 1 : 0); j < N; ++j)
            if (i < n && j < n) anorm += fabs(a[i][j]);
    int nn = n - 1, its = 0;
    double t = 0.0;
    double p = 0, q = 0, r = 0, s = 0, w = 0, x = 0, y = 0, z = 0;
    while (nn >= 0) {
        MDX_TRIP_HOOK();
        // l: the largest l in [1, nn] with a negligible subdiagonal (0 if none)
        int l = 0;
#pragma unroll
        for (int c = N - 1; c >= 1; --c)
            if (l == 0 && c <= nn) {
                double ss = fabs(a[c - 1][c - 1]) + fabs(a[c][c]);
                if (ss == 0.0) ss = anorm;
                if (fabs(a[c][c - 1]) + ss == ss) l = c;
            }
#pragma unroll
        for (int c = 1; c < N; ++c)
            if (c == l) a[c][c - 1] = 0.0;
        x = pick_diag(a, nn, 0);
        if (l == nn) {
#pragma unroll
            for (int c = 0; c < N; ++c)
                if (c == nn) {
                    wr[c] = x + t;
                    wi[c] = 0.0;
                }
            --nn;
            its = 0;
            continue;
        }
        y = pick_diag(a, nn - 1, 0);
        w = pick_diag(a, nn, -1) * pick_diag(a, nn - 1, 1);
        if (l == nn - 1) {
            p = 0.5 * (y - x);
            q = p * p + w;
            z = sqrt(fabs(q));
            x += t;
            double r0, r1, i0, i1;
            if (q >= 0.0) {
                z = p + sign_of(z, p);
                r0 = r1 = x + z;
                if (z != 0.0) r1 = x - w / z;
                i0 = i1 = 0.0;
            } else {
                r0 = r1 = x + p;
                i1 = z;
                i0 = -z;
            }
#pragma unroll
            for (int c = 0; c < N; ++c) {
                if (c == nn - 1) {
                    wr[c] = r0;
                    wi[c] = i0;
                }
                if (c == nn) {
                    wr[c] = r1;
                    wi[c] = i1;
                }
            }
            nn -= 2;
            its = 0;
            continue;
        }
        if (its == 60) return false;
        if (its == 10 || its == 20 || its == 40) {
            t += x;
#pragma unroll
            for (int i = 0; i < N; ++i)
                if (i <= nn) a[i][i] -= x;
            s = fabs(pick_diag(a, nn, -1)) + fabs(pick_diag(a, nn - 1, -1));
            y = x = 0.75 * s;
            w = -0.4375 * s * s;
        }
        ++its;
        // m: from nn - 2 down to l, the first with two small consecutive subdiagonals
        int m = -1;
#pragma unroll
        for (int c = N - 3; c >= 0; --c) {
            if (m < 0 && c <= nn - 2 && c >= l) {
                z = a[c][c];
                r = x - z;
                s = y - z;
                p = (r * s - w) / a[c + 1][c] + a[c][c + 1];
                q = a[c + 1][c + 1] - z - r - s;
                r = a[c + 2][c + 1];
                s = fabs(p) + fabs(q) + fabs(r);
                p /= s;
                q /= s;
                r /= s;
                if (c == l) {
                    m = c;
                } else if (c > 0) {
                    const double u = fabs(a[c][c > 0 ? c - 1 : 0]) * (fabs(q) + fabs(r));
                    const double v = fabs(p) * (fabs(a[c > 0 ? c - 1 : 0][c > 0 ? c - 1 : 0]) + fabs(z) +
                                                fabs(a[c + 1][c + 1]));
                    if (u + v == v) m = c;
                }
            }
        }
#pragma unroll
        for (int i = 2; i < N; ++i)
            if (i >= m + 2 && i <= nn) {
                a[i][i - 2] = 0.0;
                if (i != m + 2 && i >= 3) a[i][i >= 3 ? i - 3 : 0] = 0.0;
            }
#pragma unroll
        for (int k = 0; k < N - 1; ++k) {
            if (k >= m && k <= nn - 1) {
                const bool last = k == nn - 1;
                if (k != m && k > 0) {
                    p = a[k][k > 0 ? k - 1 : 0];
                    q = a[k + 1][k > 0 ? k - 1 : 0];
                    r = 0.0;
                    if (!last && k + 2 < N) r = a[k + 2 < N ? k + 2 : 0][k > 0 ? k - 1 : 0];
                    if ((x = fabs(p) + fabs(q) + fabs(r)) != 0.0) {
                        p /= x;
                        q /= x;
                        r /= x;
                    }
                }
                if ((s = sign_of(sqrt(p * p + q * q + r * r), p)) != 0.0) {
                    if (k == m) {
                        if (l != m && k > 0) a[k][k > 0 ? k - 1 : 0] = -a[k][k > 0 ? k - 1 : 0];
                    } else if (k > 0) {
                        a[k][k > 0 ? k - 1 : 0] = -s * x;
                    }
                    p += s;
                    x = p / s;
                    y = q / s;
                    z = r / s;
                    q /= p;
                    r /= p;
#pragma unroll
                    for (int j = k; j < N; ++j)
                        if (j <= nn) {
                            p = a[k][j] + q * a[k + 1][j];
                            if (!last && k + 2 < N) {
                                const int k2 = k + 2 < N ? k + 2 : 0;
                                p += r * a[k2][j];
                                a[k2][j] -= p * z;
                            }
                            a[k + 1][j] -= p * y;
                            a[k][j] -= p * x;
                        }
                    const int mmin = nn < k + 3 ? nn : k + 3;
#pragma unroll
                    for (int i = 0; i < N && i <= k + 3; ++i)
                        if (i >= l && i <= mmin) {
                            p = x * a[i][k] + y * a[i][k + 1];
                            if (!last && k + 2 < N) {
                                const int k2 = k + 2 < N ? k + 2 : 0;
                                p += z * a[i][k2];
                                a[i][k2] -= p * r;
                            }
                            a[i][k + 1] -= p * q;
                            a[i][k] -= p;
                        }
                }
            }
        }
    }
    return true;
}

// Real roots of the polynomial c (ascending, NC coefficients) as poly_real_roots
// (la.cpp:474-491) followed by the callers' ascending sort: companion matrix,
// balance, hqr (the companion is already upper Hessenberg, so elmhes leaves it
// unchanged and is skipped), the eigenvalues with wi == 0 exactly.  Returns the
// count; roots ascending.
template <int NC> MP_HD int real_roots(const double (&c)[NC], double (&roots)[NC - 1]) {
#pragma clang fp contract(off)
    constexpr int ND = NC - 1;
    int n = ND;
    while (n >= 0 && c[n] == 0.0) --n; // trailing zeros (la.cpp:475)
#pragma unroll
    for (int i = 0; i < ND; ++i) roots[i] = 0.0;
    if (n < 1) return 0;
    if (n == 1) {
        roots[0] = -c[0] / c[1];
        return 1;
    }
    double a[ND][ND], wr[ND], wi[ND];
    double cn = 0.0;
#pragma unroll
    for (int j = 0; j <= ND; ++j)
        if (j == n) cn = c[j];
#pragma unroll
    for (int i = 0; i < ND; ++i)
#pragma unroll
        for (int j = 0; j < ND; ++j) a[i][j] = 0.0;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
        double cj = 0.0; // c[n - 1 - j]
#pragma unroll
        for (int q = 0; q < ND; ++q)
            if (q == n - 1 - j) cj = opaque(c[q]);
        if (j < n) a[0][j] = -cj / cn;
    }
#pragma unroll
    for (int i = 1; i < ND; ++i)
        if (i < n) a[i][i - 1] = 1.0;
    balance(a, n);
    if (!hqr(a, n, wr, wi)) return 0;
    int nr = 0;
#pragma unroll
    for (int i = 0; i < ND; ++i)
        if (i < n && wi[i] == 0.0) {
            const double v = wr[i];
            // insertion into the ascending list (the callers' std::sort)
            int pos = nr;
#pragma unroll
            for (int k = 0; k < ND; ++k)
                if (k < nr && v < roots[k] && pos == nr) pos = k;
#pragma unroll
            for (int k = ND - 1; k > 0; --k)
                if (k > pos && k <= nr) roots[k] = roots[k - 1];
#pragma unroll
            for (int k = 0; k < ND; ++k)
                if (k == pos) roots[k] = v;
            ++nr;
        }
    return nr;
}

// Newton polishing (md.cpp:136-159): at most 3 steps, each kept only if it lowers the
// squared residual.  fj(z, F, J) evaluates the system at z (J: K x K).
template <int K, class FJ> MP_HD void newton_polish(double (&z)[5], FJ fj) {
#pragma clang fp contract(off)
    double F[K], J[K][K];
    fj(z, F, J);
    double rbest = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) rbest += F[k] * F[k];
#pragma unroll 1
    for (int it = 0; it < 3; ++it) {
        double dz[K];
        if (!lu_full_solve<K>(J, F, dz)) break;
        double zn[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) zn[i] = z[i];
#pragma unroll
        for (int i = 0; i < K; ++i) zn[i] = z[i] - dz[i];
        double Fn[K], Jn[K][K];
        fj(zn, Fn, Jn);
        double r = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) r += Fn[k] * Fn[k];
        if (!(r < rbest)) break;
        rbest = r;
#pragma unroll
        for (int i = 0; i < 5; ++i) z[i] = zn[i];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            F[k] = Fn[k];
#pragma unroll
            for (int c = 0; c < K; ++c) J[k][c] = Jn[k][c];
        }
    }
}

// o = M v, each row (M0 v0 + M1 v1) + M2 v2 (oracle/src/estimator.cpp mv3)
MP_HD void mv3_exact(const double *M, const double *v, double *o) {
#pragma clang fp contract(off)
    for (int r = 0; r < 3; ++r) o[r] = M[3 * r] * v[0] + M[3 * r + 1] * v[1] + M[3 * r + 2] * v[2];
}

// prescale x / f (md.cpp:202-217)
MP_HD double mean_abs_xy(const double (&x)[4][3]) {
#pragma clang fp contract(off)
    double s = 0;
    for (int i = 0; i < 4; ++i) s += fabs(x[i][0]) + fabs(x[i][1]);
    return s / (2 * 4);
}

// det3 (la.cpp:570-572), row-major
MP_HD double det3(const double (&M)[3][3]) {
#pragma clang fp contract(off)
    return M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
           M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
}

// The MD poses' SVD as the reference calls it, Eigen::JacobiSVD<MatrixXd>(S,
// ComputeFullU | ComputeFullV) (src/solver.cpp:517, :722, :1026), restated from Eigen
// 3.4 as the oracle restates it (la.cpp eigen_jacobi_svd3): scaling by the largest
// |entry|, two-sided sweeps over (p, q) = (1, 0), (2, 0), (2, 1) until every
// off-diagonal entry is below max(DBL_MIN, 2 eps max|diag|), each a real 2 x 2 Jacobi
// SVD (real_2x2_jacobi_svd, makeJacobi) applied to the rows and columns, the signs of
// the diagonal moved into U, and the singular values sorted descending by swaps.  It
// converges in 3-5 sweeps also on the rank-2 cross-covariance of three points (the
// one-sided Jacobi the oracle used before ran to its cap of 60 sweeps on about 1 % of
// calibrated samples, 85 of 150 us per MD launch, profiles/r05/mdx).
struct Rot2 {
    double c, s;
};
// rows p, q of M: x' = c x + s y, y' = -s x + c y (Eigen apply_rotation_in_the_plane;
// the identity is a no-op)
template <int P, int Q> MP_HD void rot_rows(double (&M)[3][3], Rot2 j) {
#pragma clang fp contract(off)
    if (j.c == 1.0 && j.s == 0.0) return;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double xi = M[P][i], yi = M[Q][i];
        M[P][i] = j.c * xi + j.s * yi;
        M[Q][i] = -j.s * xi + j.c * yi;
    }
}
// columns p, q: MatrixBase::applyOnTheRight(p, q, j) applies j^T = (c, -s)
template <int P, int Q> MP_HD void rot_cols(double (&M)[3][3], Rot2 j) {
#pragma clang fp contract(off)
    const double c = j.c, s = -j.s;
    if (c == 1.0 && s == 0.0) return;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double xi = M[i][P], yi = M[i][Q];
        M[i][P] = c * xi + s * yi;
        M[i][Q] = -s * xi + c * yi;
    }
}
MP_HD Rot2 make_jacobi(double x, double y, double z) {
#pragma clang fp contract(off)
    const double deno = 2.0 * fabs(y);
    if (deno < DBL_MIN) return Rot2{1.0, 0.0};
    const double tau = (x - z) / deno;
    const double w = sqrt(tau * tau + 1.0);
    const double t = tau > 0.0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
    const double sign_t = t > 0.0 ? 1.0 : -1.0;
    const double n = 1.0 / sqrt(t * t + 1.0);
    return Rot2{n, -sign_t * (y / fabs(y)) * fabs(t) * n};
}
// one (p, q) step of the sweep
template <int P, int Q>
MP_HD void jacobi_step(double (&W)[3][3], double (&U)[3][3], double (&V)[3][3], double &max_diag, bool &finished) {
#pragma clang fp contract(off)
    const double pm = 2.0 * DBL_EPSILON * max_diag;
    const double threshold = DBL_MIN < pm ? pm : DBL_MIN;
    if (!(fabs(W[P][Q]) > threshold || fabs(W[Q][P]) > threshold)) return;
    finished = false;
    double m00 = W[P][P], m01 = W[P][Q], m10 = W[Q][P], m11 = W[Q][Q];
    Rot2 rot1{1.0, 0.0};
    const double t = m00 + m11, d = m10 - m01;
    if (!(fabs(d) < DBL_MIN)) {
        const double u = t / d;
        const double tmp = sqrt(1.0 + u * u);
        rot1 = Rot2{u / tmp, 1.0 / tmp};
    }
    if (!(rot1.c == 1.0 && rot1.s == 0.0)) {
        const double x0 = m00, y0 = m10, x1 = m01, y1 = m11;
        m00 = rot1.c * x0 + rot1.s * y0;
        m01 = rot1.c * x1 + rot1.s * y1;
        m11 = -rot1.s * x1 + rot1.c * y1;
    }
    const Rot2 jr = make_jacobi(m00, m01, m11);
    const double c2 = jr.c, s2 = -jr.s; // j_left = rot1 * j_right^T
    const Rot2 jl{rot1.c * c2 - rot1.s * s2, rot1.c * s2 + rot1.s * c2};
    rot_rows<P, Q>(W, jl);
    rot_cols<P, Q>(U, Rot2{jl.c, -jl.s}); // U.applyOnTheRight(p, q, j_left^T)
    rot_cols<P, Q>(W, jr);
    rot_cols<P, Q>(V, jr);
    const double dp = fabs(W[P][P]), dq = fabs(W[Q][Q]);
    const double mm = dp < dq ? dq : dp;
    max_diag = max_diag < mm ? mm : max_diag;
}

MP_HD void svd3(const double (&A)[3][3], double (&U)[3][3], double (&V)[3][3]) {
#pragma clang fp contract(off)
    double scale = 0.0;
    bool nan = false;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double a = fabs(A[i][j]);
            nan = nan || a != a;
            scale = scale < a ? a : scale;
        }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) U[i][j] = V[i][j] = i == j ? 1.0 : 0.0;
    if (nan || !(scale <= DBL_MAX)) return; // Eigen: InvalidInput
    if (scale == 0.0) scale = 1.0;
    double W[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) W[i][j] = A[i][j] / scale;
    double max_diag = fabs(W[0][0]);
    max_diag = max_diag < fabs(W[1][1]) ? fabs(W[1][1]) : max_diag;
    max_diag = max_diag < fabs(W[2][2]) ? fabs(W[2][2]) : max_diag;
    bool finished = false;
    // (a cap far above the 3-6 sweeps finite data takes, against non-termination)
    for (int sweep = 0; !finished && sweep < 1000; ++sweep) {
        finished = true;
        jacobi_step<1, 0>(W, U, V, max_diag, finished);
        jacobi_step<2, 0>(W, U, V, max_diag, finished);
        jacobi_step<2, 1>(W, U, V, max_diag, finished);
    }
    double sv[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double a = W[i][i];
        sv[i] = fabs(a);
        if (a < 0.0)
#pragma unroll
            for (int r = 0; r < 3; ++r) U[r][i] = -U[r][i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) sv[i] *= scale;
    // descending by swaps: position i takes the first maximum of the tail
    bool stop = false;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int pos = i;
        double best = sv[i];
#pragma unroll
        for (int j = i + 1; j < 3; ++j)
            if (sv[j] > best) {
                best = sv[j];
                pos = j;
            }
        stop = stop || best == 0.0;
#pragma unroll
        for (int j = i + 1; j < 3; ++j) {
            const bool sw = !stop && pos == j;
            const double a = opaque(sv[i]), b2 = opaque(sv[j]);
            sv[i] = sw ? b2 : a;
            sv[j] = sw ? a : b2;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const double ui = opaque(U[r][i]), uj = opaque(U[r][j]);
                U[r][i] = sw ? uj : ui;
                U[r][j] = sw ? ui : uj;
                const double vi = opaque(V[r][i]), vj = opaque(V[r][j]);
                V[r][i] = sw ? vj : vi;
                V[r][j] = sw ? vi : vj;
            }
        }
    }
}

// Kabsch without scale, Y ~ R X + t, as the oracle's procrustes (md.cpp:355-383;
// src/solver.cpp:506-525): centroids, cross-covariance S = sum (Y - cy)(X - cx)^T,
// R = U diag(1, 1, sign) V^T with the sign from det U det V, t = cy - R cx.
template <int K> MP_HD void procrustes(const double (&X)[K][3], const double (&Y)[K][3], Model &m) {
#pragma clang fp contract(off)
    double cx[3] = {0, 0, 0}, cy[3] = {0, 0, 0};
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            cx[c] += X[i][c];
            cy[c] += Y[i][c];
        }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        cx[c] /= K;
        cy[c] /= K;
    }
    double S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) S[a][b] += (Y[i][a] - cy[a]) * (X[i][b] - cx[b]);
    double U[3][3], V[3][3];
    svd3(S, U, V);
    const double du = det3(U), dv = det3(V);
    if (du * dv < 0)
#pragma unroll
        for (int i = 0; i < 3; ++i) U[i][2] = -U[i][2];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            double s = 0;
#pragma unroll
            for (int c = 0; c < 3; ++c) s += U[a][c] * V[b][c];
            m.R[3 * a + b] = s;
        }
#pragma unroll
    for (int a = 0; a < 3; ++a)
        m.t[a] = cy[a] - (m.R[3 * a] * cx[0] + m.R[3 * a + 1] * cx[1] + m.R[3 * a + 2] * cx[2]);
}

} // namespace mdx

// Pose stage of the MD solvers as the oracle's md_pose (md.cpp:394-434): the
// positivity test of the corrected depths (src/solver.cpp:503-504), the focal
// division, and the exact Procrustes above -- the model's every double is the
// oracle's.  K = 3 (cal) or 4 (sf/tf) points; fx, fy the solution's focals.
// md_pose_points: the corrected points and the positivity test (the model's scale and
// offsets are the solution's, so whether it is kept is known before the Procrustes).
template <int K>
MP_HD bool md_pose_points(const double (&x)[K][3], const double (&y)[K][3], const double *dx, const double *dy,
                          const double *sol, double fx, double fy, double (&X)[K][3], double (&Y)[K][3]) {
#pragma clang fp contract(off)
    bool ok = true;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const double d1 = dx[i] + sol[1];
        const double d2 = dy[i] * sol[2] + sol[3];
        if (!(d1 > 0.0) || !(d2 > 0.0)) ok = false;
        X[i][0] = x[i][0] / fx * d1;
        X[i][1] = x[i][1] / fx * d1;
        X[i][2] = x[i][2] * d1;
        Y[i][0] = y[i][0] / fy * d2;
        Y[i][1] = y[i][1] / fy * d2;
        Y[i][2] = y[i][2] * d2;
    }
    return ok;
}

template <int K>
MP_HD bool md_pose_exact(const double (&x)[K][3], const double (&y)[K][3], const double *dx, const double *dy,
                         const double *sol, double fx, double fy, Model &m) {
    double X[K][3], Y[K][3];
    if (!md_pose_points<K>(x, y, dx, dy, sol, fx, fy, X, Y)) return false;
    mdx::procrustes<K>(X, Y, m);
    m.scale = sol[2];
    m.offset0 = sol[1];
    m.offset1 = sol[3];
    return true;
}

// The solvers in two parts, as the oracle's loop over roots: setup() builds the
// sample's system and returns the ascending real roots of its resultant; root() turns
// one root into a solution, false when the oracle's filters reject it.  The
// estimator's kernel runs root() on one lane per root (kernels.hip md_exact); the
// mdx_sols_* loops run them in one lane (the direct solver entries, the host check).

// solve_scale_and_shift (calibrated, md.cpp:161-200): rays x, y (3 x 3); solutions in
// ascending b1, sol = (1, b1, a2, b2 * a2, 1, 1).
struct MdxCal {
    static constexpr int NR = 4;
    PairTerms T[3];
    double l1[3], l2[3];
    MP_HD int setup(const double (&x3)[3][3], const double (&y3)[3][3], const double *dx, const double *dy,
                    double (&roots)[NR]) {
#pragma clang fp contract(off)
        double x[4][3], y[4][3];
        for (int i = 0; i < 3; ++i)
            for (int c = 0; c < 3; ++c) {
                x[i][c] = x3[i][c];
                y[i][c] = y3[i][c];
            }
        for (int c = 0; c < 3; ++c) x[3][c] = y[3][c] = 0.0;
        for (int k = 0; k < NR; ++k) roots[k] = 0.0;
        const int pr[3][2] = {{0, 1}, {0, 2}, {1, 2}};
        for (int k = 0; k < 3; ++k) T[k] = mdx::pair_terms<false>(x, y, dx, dy, pr[k][0], pr[k][1]);
        double Q[3][3], Pm[3][3], L[3][3];
        for (int k = 0; k < 3; ++k)
            for (int c = 0; c < 3; ++c) {
                Q[k][c] = T[k].B[c];
                Pm[k][c] = T[k].A[c];
            }
        if (!mdx::qr_solve<3, 3>(Q, Pm, L)) return 0;
        const double l0[3] = {L[0][2], L[0][1], L[0][0]};
        for (int c = 0; c < 3; ++c) {
            l1[c] = L[1][2 - c];
            l2[c] = L[2][2 - c];
        }
        double a[5], b[5], quart[5];
        mdx::pmul(l1, l1, a);
        mdx::pmul(l0, l2, b);
        mdx::psub(a, b, quart);
        return mdx::real_roots(quart, roots);
    }
    MP_HD bool root(double b1, double (&sol)[6]) const {
#pragma clang fp contract(off)
        const double s = mdx::peval(l2, b1);
        const double beta = mdx::peval(l1, b1) / s;
        double z[5] = {b1, beta, s, 0.0, 0.0};
        mdx::newton_polish<3>(z, [&](const double (&v)[5], double (&F)[3], double (&J)[3][3]) {
#pragma clang fp contract(off)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double *A = T[k].A, *B = T[k].B;
                const double ub = A[0] * v[0] * v[0] + A[1] * v[0] + A[2];
                const double vb = B[0] * v[1] * v[1] + B[1] * v[1] + B[2];
                F[k] = ub - v[2] * vb;
                J[k][0] = 2 * A[0] * v[0] + A[1];
                J[k][1] = -v[2] * (2 * B[0] * v[1] + B[1]);
                J[k][2] = -vb;
            }
        });
        if (!(z[2] > 0)) return false;
        const double a2 = sqrt(z[2]);
        sol[0] = 1.0;
        sol[1] = z[0];
        sol[2] = a2;
        sol[3] = z[1] * a2;
        sol[4] = sol[5] = 1.0;
        return true;
    }
};

// solve_scale_and_shift_shared_focal (md.cpp:219-284): x0, y0 pp-centred normalized
// points (homogeneous, 4 x 3); sol = (1, b1, a2, b2 * a2, f, f).
struct MdxSF {
    static constexpr int NR = 8;
    PairTerms T[4];
    double q0[4][2], q1[4][2], X[5], Y[5], f0;
    MP_HD int setup(const double (&x0)[4][3], const double (&y0)[4][3], const double *dx, const double *dy,
                    double (&roots)[NR]) {
#pragma clang fp contract(off)
        for (int k = 0; k < NR; ++k) roots[k] = 0.0;
        f0 = 0.5 * (mdx::mean_abs_xy(x0) + mdx::mean_abs_xy(y0));
        double x[4][3], y[4][3];
        for (int i = 0; i < 4; ++i) {
            x[i][0] = x0[i][0] / f0;
            x[i][1] = x0[i][1] / f0;
            x[i][2] = x0[i][2];
            y[i][0] = y0[i][0] / f0;
            y[i][1] = y0[i][1] / f0;
            y[i][2] = y0[i][2];
        }
        const int pr[4][2] = {{0, 1}, {0, 2}, {1, 2}, {0, 3}};
        double M[4][4], Rh[4][4], L[4][4];
        for (int k = 0; k < 4; ++k) {
            T[k] = mdx::pair_terms<true>(x, y, dx, dy, pr[k][0], pr[k][1]);
            M[k][0] = T[k].A[0];
            M[k][1] = T[k].A[1];
            M[k][2] = -T[k].B[0];
            M[k][3] = -T[k].B[1];
            Rh[k][0] = -T[k].A[2];
            Rh[k][1] = T[k].B[2];
            Rh[k][2] = T[k].dz1;
            Rh[k][3] = -T[k].dz0;
        }
        if (!mdx::qr_solve<4, 4>(M, Rh, L)) return 0;
        for (int r = 0; r < 4; ++r) {
            q0[r][0] = L[r][3];
            q0[r][1] = L[r][0];
            q1[r][0] = L[r][2];
            q1[r][1] = L[r][1];
        }
        const double Wp[2] = {0.0, 1.0};
        double t0[3], t1[3], al0[3], al1[3], al2[3], be0[3], be1[3], be2[3];
        mdx::pmul(q0[1], q0[1], t0);
        mdx::pmul(q0[0], Wp, t1);
        mdx::psub(t0, t1, al0);
        mdx::pmul(q0[1], q1[1], t0);
        mdx::pscale(t0, 2.0);
        mdx::pmul(q1[0], Wp, t1);
        mdx::psub(t0, t1, al1);
        mdx::pmul(q1[1], q1[1], al2);
        mdx::pmul(q0[3], q0[3], be0);
        mdx::pmul(q0[3], q1[3], t0);
        mdx::pscale(t0, 2.0);
        mdx::pmul(q0[2], Wp, t1);
        mdx::psub(t0, t1, be1);
        mdx::pmul(q1[3], q1[3], t0);
        mdx::pmul(q1[2], Wp, t1);
        mdx::psub(t0, t1, be2);
        double R[9];
        mdx::quad_resultant<3, 3, 3, 3, 3, 3, 5, 5, 5, 9>(al0, al1, al2, be0, be1, be2, X, Y, R);
        return mdx::real_roots(R, roots);
    }
    MP_HD bool root(double w, double (&sol)[6]) const {
#pragma clang fp contract(off)
        const double s = -mdx::peval(X, w) / mdx::peval(Y, w);
        const double wb1 = mdx::peval(q0[1], w) + s * mdx::peval(q1[1], w);
        const double tb = mdx::peval(q0[3], w) + s * mdx::peval(q1[3], w);
        double z[5] = {wb1 / w, tb / (s * w), s, w, 0.0};
        mdx::newton_polish<4>(z, [&](const double (&v)[5], double (&F)[4], double (&J)[4][4]) {
#pragma clang fp contract(off)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const double *A = T[k].A, *B = T[k].B;
                const double ua = A[0] * v[0] * v[0] + A[1] * v[0] + A[2];
                const double vb = B[0] * v[1] * v[1] + B[1] * v[1] + B[2];
                F[k] = v[3] * ua + T[k].dz0 - v[2] * (v[3] * vb + T[k].dz1);
                J[k][0] = v[3] * (2 * A[0] * v[0] + A[1]);
                J[k][1] = -v[2] * v[3] * (2 * B[0] * v[1] + B[1]);
                J[k][2] = -(v[3] * vb + T[k].dz1);
                J[k][3] = ua - v[2] * vb;
            }
        });
        if (z[3] < 0) return false; // src/solver.cpp:283
        if (!(z[2] > 0)) return false;
        const double a2 = sqrt(z[2]);
        const double f = f0 / sqrt(z[3]);
        sol[0] = 1.0;
        sol[1] = z[0];
        sol[2] = a2;
        sol[3] = z[1] * a2;
        sol[4] = sol[5] = f;
        return true;
    }
};

// solve_scale_and_shift_two_focal (md.cpp:286-352); sol = (1, b1, a2, b2 * a2, f1, f2).
struct MdxTF {
    static constexpr int NR = 4;
    PairTerms T[5];
    double q0[5][2], q1[5][1], X[3], Y[2], f1, f2;
    MP_HD int setup(const double (&x0)[4][3], const double (&y0)[4][3], const double *dx, const double *dy,
                    double (&roots)[NR]) {
#pragma clang fp contract(off)
        for (int k = 0; k < NR; ++k) roots[k] = 0.0;
        f1 = mdx::mean_abs_xy(x0);
        f2 = mdx::mean_abs_xy(y0);
        double x[4][3], y[4][3];
        for (int i = 0; i < 4; ++i) {
            x[i][0] = x0[i][0] / f1;
            x[i][1] = x0[i][1] / f1;
            x[i][2] = x0[i][2];
            y[i][0] = y0[i][0] / f2;
            y[i][1] = y0[i][1] / f2;
            y[i][2] = y0[i][2];
        }
        const int pr[5][2] = {{0, 1}, {0, 2}, {1, 2}, {0, 3}, {1, 3}};
        double M[5][5], Rh[5][3], L[5][3];
        for (int k = 0; k < 5; ++k) {
            T[k] = mdx::pair_terms<true>(x, y, dx, dy, pr[k][0], pr[k][1]);
            M[k][0] = T[k].A[0];
            M[k][1] = T[k].A[1];
            M[k][2] = -T[k].B[0];
            M[k][3] = -T[k].B[1];
            M[k][4] = -T[k].dz1;
            Rh[k][0] = -T[k].A[2];
            Rh[k][1] = T[k].B[2];
            Rh[k][2] = -T[k].dz0;
        }
        if (!mdx::qr_solve<5, 3>(M, Rh, L)) return 0;
        for (int r = 0; r < 5; ++r) {
            q0[r][0] = L[r][2];
            q0[r][1] = L[r][0];
            q1[r][0] = L[r][1];
        }
        const double Wp[2] = {0.0, 1.0};
        double t0[3], t1[3], s0[2], s1[2], u0[1], al0[3], al1[2], al2[1], be0[3], be1[2], be2[1];
        mdx::pmul(q0[1], q0[1], t0);
        mdx::pmul(q0[0], Wp, t1);
        mdx::psub(t0, t1, al0);
        mdx::pmul(q0[1], q1[1], s0);
        mdx::pscale(s0, 2.0);
        mdx::pmul(q1[0], Wp, s1);
        mdx::psub(s0, s1, al1);
        mdx::pmul(q1[1], q1[1], al2);
        mdx::pmul(q0[3], q0[3], be0);
        mdx::pmul(q0[3], q1[3], s0);
        mdx::pscale(s0, 2.0);
        mdx::psub(s0, q0[2], be1);
        mdx::pmul(q1[3], q1[3], u0);
        mdx::psub(u0, q1[2], be2);
        double R[5];
        mdx::quad_resultant<3, 2, 1, 3, 2, 1, 3, 2, 4, 5>(al0, al1, al2, be0, be1, be2, X, Y, R);
        return mdx::real_roots(R, roots);
    }
    MP_HD bool root(double w1, double (&sol)[6]) const {
#pragma clang fp contract(off)
        const double t = -mdx::peval(X, w1) / mdx::peval(Y, w1);
        double m[5];
        for (int r = 0; r < 5; ++r) m[r] = mdx::peval(q0[r], w1) + t * q1[r][0];
        const double s = m[4];
        double z[5] = {m[1] / w1, m[3] / t, s, w1, t / s};
        mdx::newton_polish<5>(z, [&](const double (&v)[5], double (&F)[5], double (&J)[5][5]) {
#pragma clang fp contract(off)
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const double *A = T[k].A, *B = T[k].B;
                const double ua = A[0] * v[0] * v[0] + A[1] * v[0] + A[2];
                const double vb = B[0] * v[1] * v[1] + B[1] * v[1] + B[2];
                F[k] = v[3] * ua + T[k].dz0 - v[2] * (v[4] * vb + T[k].dz1);
                J[k][0] = v[3] * (2 * A[0] * v[0] + A[1]);
                J[k][1] = -v[2] * v[4] * (2 * B[0] * v[1] + B[1]);
                J[k][2] = -(v[4] * vb + T[k].dz1);
                J[k][3] = ua;
                J[k][4] = -v[2] * vb;
            }
        });
        if (z[3] < 0 || z[4] < 0) return false; // src/solver.cpp:470
        if (!(z[2] > 0)) return false;
        const double a2 = sqrt(z[2]);
        sol[0] = 1.0;
        sol[1] = z[0];
        sol[2] = a2;
        sol[3] = z[1] * a2;
        sol[4] = f1 / sqrt(z[3]);
        sol[5] = f2 / sqrt(z[4]);
        return true;
    }
};

// One lane, every root in turn (the direct solver entries and the host check): the
// sorted roots go through the lane's scratch column, read back by a runtime index.
template <class S, class In, class Emit>
MP_HD int mdx_sols(LaneScratch W, const In &x, const In &y, const double *dx, const double *dy, Emit &&emit) {
    S sys;
    double roots[S::NR];
    const int nr = sys.setup(x, y, dx, dy, roots);
    for (int k = 0; k < S::NR; ++k) W[k] = roots[k];
    int n = 0;
    for (int q = 0; q < nr; ++q) {
        double sol[6];
        if (!sys.root(W[q], sol)) continue;
        emit(sol);
        ++n;
    }
    return n;
}
template <class Emit>
MP_HD int mdx_sols_cal(LaneScratch W, const double (&x)[3][3], const double (&y)[3][3], const double *dx,
                       const double *dy, Emit &&emit) {
    return mdx_sols<MdxCal>(W, x, y, dx, dy, emit);
}
template <class Emit>
MP_HD int mdx_sols_sf(LaneScratch W, const double (&x)[4][3], const double (&y)[4][3], const double *dx,
                      const double *dy, Emit &&emit) {
    return mdx_sols<MdxSF>(W, x, y, dx, dy, emit);
}
template <class Emit>
MP_HD int mdx_sols_tf(LaneScratch W, const double (&x)[4][3], const double (&y)[4][3], const double *dx,
                      const double *dy, Emit &&emit) {
    return mdx_sols<MdxTF>(W, x, y, dx, dy, emit);
}

// per-lane scratch doubles of the three solvers (the root list, read back by a
// runtime index in the per-root loop)
constexpr int kMdxScratchCal = 4, kMdxScratchSF = 8, kMdxScratchTF = 4;

} // namespace mp
