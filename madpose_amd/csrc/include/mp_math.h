// Register-resident small dense math for the per-sample solvers.
// Everything here is fixed-size and fully unrollable so hipcc keeps it in VGPRs
// (no dynamically indexed private arrays -> no scratch traffic).
#pragma once
#include <cfloat>
#include <cmath>

#include "mp_types.h"

namespace mp {

MP_HD double sq(double x) { return x * x; }

MP_HD void cross3(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
MP_HD double dot3(const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// the same without FMA contraction (the exact point-solver stages: the oracle's
// operations to the bit)
MP_HD void cross3_x(const double *a, const double *b, double *c) {
#pragma clang fp contract(off)
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
MP_HD double dot3_x(const double *a, const double *b) {
#pragma clang fp contract(off)
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
MP_HD void matvec3_x(const double *A, const double *v, double *o) {
#pragma clang fp contract(off)
#pragma unroll
    for (int r = 0; r < 3; ++r) o[r] = A[3 * r] * v[0] + A[3 * r + 1] * v[1] + A[3 * r + 2] * v[2];
}

MP_HD void matmul3(const double *A, const double *B, double *C) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) C[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}
MP_HD void matvec3(const double *A, const double *v, double *o) {
#pragma unroll
    for (int r = 0; r < 3; ++r) o[r] = A[3 * r] * v[0] + A[3 * r + 1] * v[1] + A[3 * r + 2] * v[2];
}

// PoseLib check_cheirality (src/solver.cpp:1188-1206); x1, x2 unit vectors
// (no FMA contraction: the oracle's check_cheirality to the bit)
MP_HD bool check_cheirality(const double *R, const double *t, const double *x1, const double *x2, double min_depth) {
#pragma clang fp contract(off)
    double Rx1[3];
    matvec3_x(R, x1, Rx1);
    const double a = -dot3_x(Rx1, x2);
    const double b1 = -dot3_x(Rx1, t);
    const double b2 = dot3_x(x2, t);
    const double l1 = b1 - a * b2;
    const double l2 = -a * b1 + b2;
    min_depth = min_depth * (1 - a * a);
    return l1 > min_depth && l2 > min_depth;
}

// Solve A X = B (N x N, N x M) in place by Gaussian elimination with partial
// pivoting.  Row exchanges are done with predicated selects so all indices are
// compile-time constants.  Returns false on a zero pivot.
template <int N, int M> MP_HD bool gauss_solve(double (&A)[N][N], double (&B)[N][M]) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        // pivot search
        int p = k;
        double best = fabs(A[k][k]);
#pragma unroll
        for (int r = k + 1; r < N; ++r) {
            double v = fabs(A[r][k]);
            if (v > best) {
                best = v;
                p = r;
            }
        }
        // (swaps as selects between opaque values: see opaque() in mp_types.h)
#pragma unroll
        for (int r = k + 1; r < N; ++r) {
            const bool sw = r == p;
#pragma unroll
            for (int c = 0; c < N; ++c) {
                const double akc = opaque(A[k][c]), arc = opaque(A[r][c]);
                A[k][c] = sw ? arc : akc;
                A[r][c] = sw ? akc : arc;
            }
#pragma unroll
            for (int c = 0; c < M; ++c) {
                const double bkc = opaque(B[k][c]), brc = opaque(B[r][c]);
                B[k][c] = sw ? brc : bkc;
                B[r][c] = sw ? bkc : brc;
            }
        }
        if (best == 0.0) ok = false;
        const double inv = 1.0 / A[k][k];
#pragma unroll
        for (int r = k + 1; r < N; ++r) {
            const double l = A[r][k] * inv;
#pragma unroll
            for (int c = k + 1; c < N; ++c) A[r][c] -= l * A[k][c];
#pragma unroll
            for (int c = 0; c < M; ++c) B[r][c] -= l * B[k][c];
        }
    }
    // back substitution
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
        const double inv = 1.0 / A[k][k];
#pragma unroll
        for (int c = 0; c < M; ++c) {
            double s = B[k][c];
#pragma unroll
            for (int j = k + 1; j < N; ++j) s -= A[k][j] * B[j][c];
            B[k][c] = s * inv;
        }
    }
    return ok;
}

// ---------------------------------------------------------------------------
// Real roots of a univariate polynomial by Sturm sequences (root isolation by
// bisection of sign-change counts, then safeguarded Newton/bisection refinement).
// c: ascending coefficients of degree N (c[N] != 0 expected).  Returns the number
// of roots written to roots[] in ascending order.
template <int N> struct SturmChain {
    double s[N + 1][N + 1]; // poly k has degree N-k (ascending coefficients)
    int len;
};

template <int N> MP_HD double horner(const double (&p)[N + 1], int deg, double x) {
    double v = 0.0;
#pragma unroll
    for (int j = N; j >= 0; --j)
        if (j <= deg) v = v * x + p[j];
    return v;
}

template <int N> MP_HD void sturm_build(const double *c, SturmChain<N> &S) {
    double mx = 0.0;
#pragma unroll
    for (int j = 0; j <= N; ++j) mx = fmax(mx, fabs(c[j]));
    const double sc0 = mx > 0 ? 1.0 / mx : 1.0;
#pragma unroll
    for (int j = 0; j <= N; ++j) {
        S.s[0][j] = c[j] * sc0;
        S.s[1][j] = 0.0;
    }
    // derivative (positive scaling)
    mx = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        S.s[1][j] = (j + 1) * S.s[0][j + 1];
        mx = fmax(mx, fabs(S.s[1][j]));
    }
#pragma unroll
    for (int j = 0; j < N; ++j) S.s[1][j] /= mx;
    S.len = 2;
    bool alive = true;
#pragma unroll
    for (int k = 1; k < N; ++k) {
        // a = s[k-1] (deg d+1), b = s[k] (deg d), d = N-k;  next = -(a mod b)
        const int d = N - k;
        double nxt[N + 1];
#pragma unroll
        for (int j = 0; j <= N; ++j) nxt[j] = 0.0;
        const double bd = S.s[k][d];
        double bmax = 0.0;
#pragma unroll
        for (int j = 0; j <= d; ++j) bmax = fmax(bmax, fabs(S.s[k][j]));
        if (!(fabs(bd) > 1e-14 * bmax)) alive = false;
        if (alive) {
            const double q1 = S.s[k - 1][d + 1] / bd;
            const double q0 = (S.s[k - 1][d] - q1 * S.s[k][d - 1]) / bd;
            double rmax = 0.0;
#pragma unroll
            for (int j = 0; j < d; ++j) {
                double bm1 = (j > 0) ? S.s[k][j - 1] : 0.0;
                nxt[j] = -(S.s[k - 1][j] - q1 * bm1 - q0 * S.s[k][j]);
                rmax = fmax(rmax, fabs(nxt[j]));
            }
            double amax = 0.0;
#pragma unroll
            for (int j = 0; j <= d + 1; ++j) amax = fmax(amax, fabs(S.s[k - 1][j]));
            if (!(rmax > 1e-15 * amax)) {
                alive = false; // exact division: gcd found (multiple roots); chain ends here
            } else {
#pragma unroll
                for (int j = 0; j < d; ++j) S.s[k + 1][j] = nxt[j] / rmax;
#pragma unroll
                for (int j = d; j <= N; ++j) S.s[k + 1][j] = 0.0;
                S.len = k + 2;
            }
        }
    }
}

// number of sign changes of the chain at x
template <int N> MP_HD int sturm_count(const SturmChain<N> &S, double x) {
    int changes = 0;
    double prev = 0.0;
#pragma unroll
    for (int k = 0; k <= N; ++k) {
        if (k < S.len) {
            double v = 0.0;
#pragma unroll
            for (int j = N - k; j >= 0; --j) v = v * x + S.s[k][j];
            if (v != 0.0) {
                if (prev != 0.0 && ((v < 0) != (prev < 0))) ++changes;
                prev = v;
            }
        }
    }
    return changes;
}

template <int N> MP_HD double refine_root(const double *c, double lo, double hi) {
    double flo = 0.0, fhi = 0.0;
    for (int j = N; j >= 0; --j) {
        flo = flo * lo + c[j];
        fhi = fhi * hi + c[j];
    }
    if (flo == 0.0) return lo;
    if (fhi == 0.0) return hi;
    if ((flo < 0) == (fhi < 0)) return 0.5 * (lo + hi); // even multiplicity: midpoint
    // a few plain bisection steps first (only the sign of p is needed), so that the
    // Newton phase starts close to the root and rarely falls back to bisection
#pragma unroll
    for (int it = 0; it < 6; ++it) {
        const double mid = 0.5 * (lo + hi);
        double fm = 0.0;
#pragma unroll
        for (int j = N; j >= 0; --j) fm = fm * mid + c[j];
        if (fm == 0.0) return mid;
        if ((fm < 0) == (flo < 0))
            lo = mid;
        else
            hi = mid;
    }
    // safeguarded Newton: a Newton step that leaves the bracket is replaced by
    // bisection; stop once the step is within a few ulps (Newton then oscillates
    // between neighbouring doubles and a tighter test would never fire)
    double x = 0.5 * (lo + hi);
    for (int it = 0; it < 60; ++it) {
        double f = 0.0, df = 0.0;
#pragma unroll
        for (int j = N; j >= 0; --j) {
            df = df * x + f;
            f = f * x + c[j];
        }
        if (f == 0.0) return x;
        if ((f < 0) == (flo < 0))
            lo = x;
        else
            hi = x;
        double xn = x - f / df;
        if (!(xn > lo && xn < hi)) xn = 0.5 * (lo + hi);
        if (fabs(xn - x) <= 4e-16 * fabs(xn) || hi - lo <= 4e-16 * fmax(fabs(lo), fabs(hi))) return xn;
        x = xn;
    }
    return x;
}

// Isolating intervals collected per lane before any refinement, so that the
// refinement loop of a wave runs max(#roots) times instead of once per grid cell
// that holds a root on any lane.  Writes use static indices (registers).
template <int N> struct RootIntervals {
    double lo[N], hi[N];
    int n = 0;
    MP_HD void push(double a, double b) {
#pragma unroll
        for (int k = 0; k < N; ++k)
            if (k == n) {
                lo[k] = a;
                hi[k] = b;
            }
        if (n < N) ++n;
    }
};

// Roots in (lo, hi] (Sturm counts clo > chi) isolated left to right by bisection
// without a stack: shrink onto the leftmost root, record it, continue to its right.
// A cluster narrower than 1e-14 (relative) yields one root.  Used only for grid
// cells that hold several roots.
template <int N>
MP_HD void sturm_isolate(const SturmChain<N> &S, double lo, double hi, int clo, int chi, RootIntervals<N> &I) {
    for (int guard = 0; guard < N && clo > chi; ++guard) {
        double a = lo, b = hi;
        int ca = clo, cb = chi;
        for (int depth = 0; depth < 100; ++depth) {
            if (ca - cb == 1 || b - a <= 1e-14 * fmax(1.0, fmax(fabs(a), fabs(b)))) break;
            const double m = 0.5 * (a + b);
            const int cm = sturm_count<N>(S, m);
            if (ca - cm >= 1) {
                b = m;
                cb = cm;
            } else {
                a = m;
                ca = cm;
            }
        }
        I.push(a, b);
        lo = b;
        clo = cb;
    }
}

template <int N> MP_HD int sturm_real_roots(const double *c_in, double *roots) {
    // trim leading zeros is the caller's job; normalise to avoid overflow
    double c[N + 1], cs[N + 1];
    double mx = 0.0;
#pragma unroll
    for (int j = 0; j <= N; ++j) mx = fmax(mx, fabs(c_in[j]));
    if (!(mx > 0.0) || !(fabs(c_in[N]) > 1e-300)) return 0;
    const double lead = 1.0 / c_in[N];
#pragma unroll
    for (int j = 0; j <= N; ++j) c[j] = c_in[j] * lead; // monic
    // rescale x = sigma * y so the roots are O(1) (Fujiwara-type root-size estimate);
    // the chain is built and searched on the scaled polynomial, roots are refined on c.
    double sigma = 0.0;
#pragma unroll
    for (int j = 0; j < N; ++j)
        if (c[j] != 0.0) sigma = fmax(sigma, pow(fabs(c[j]), 1.0 / (N - j)));
    if (!(sigma > 0.0) || !(sigma < 1e300)) sigma = 1.0;
    {
        const double inv = 1.0 / sigma;
        double p = 1.0;
        cs[N] = 1.0;
#pragma unroll
        for (int j = N - 1; j >= 0; --j) {
            p *= inv;
            cs[j] = c[j] * p;
        }
    }
    const double B = 3.0; // all roots of the scaled monic polynomial satisfy |y| <= 2
    SturmChain<N> S;
    sturm_build<N>(cs, S);
    // Isolation on a uniform grid of kCells cells (the same work on every lane of a
    // wave); cells with several roots are split by stackless bisection.  Then every
    // isolated root is refined.  Output is ascending.
    constexpr int kCells = 32;
    const double h = 2.0 * B / kCells;
    const int c_end = sturm_count<N>(S, B);
    double x_lo = -B;
    int v_lo = sturm_count<N>(S, -B);
    RootIntervals<N> I;
    for (int i = 0; i < kCells && v_lo > c_end; ++i) {
        const double x_hi = (i + 1 == kCells) ? B : -B + (i + 1) * h;
        const int v_hi = (i + 1 == kCells) ? c_end : sturm_count<N>(S, x_hi);
        const int d = v_lo - v_hi;
        if (d == 1)
            I.push(x_lo, x_hi);
        else if (d > 1)
            sturm_isolate<N>(S, x_lo, x_hi, v_lo, v_hi, I);
        x_lo = x_hi;
        v_lo = v_hi;
    }
#pragma unroll
    for (int k = 0; k < N; ++k)
        if (k < I.n) roots[k] = refine_root<N>(c, sigma * I.lo[k], sigma * I.hi[k]);
    return I.n;
}

// ---------------------------------------------------------------------------
// Cyclic Jacobi eigen-decomposition of a symmetric 4x4 matrix (in place, A becomes
// diagonal, V accumulates eigenvectors as columns).
MP_HD void jacobi_eig4(double (&A)[4][4], double (&V)[4][4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 12; ++sweep) {
        double off = 0.0, dn = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            dn += A[i][i] * A[i][i];
#pragma unroll
            for (int j = i + 1; j < 4; ++j) off += A[i][j] * A[i][j];
        }
        if (!(off > 1e-32 * dn)) break;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                const double apq = A[p][q];
                if (apq != 0.0) {
                    const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
                    const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                    const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const double akp = A[k][p], akq = A[k][q];
                        A[k][p] = c * akp - s * akq;
                        A[k][q] = s * akp + c * akq;
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const double apk = A[p][k], aqk = A[q][k];
                        A[p][k] = c * apk - s * aqk;
                        A[q][k] = s * apk + c * aqk;
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const double vkp = V[k][p], vkq = V[k][q];
                        V[k][p] = c * vkp - s * vkq;
                        V[k][q] = s * vkp + c * vkq;
                    }
                }
            }
    }
}

// Rotation minimising sum |Y_i - R X_i|^2 for centred point sets, via Horn's
// unit-quaternion method: q = dominant eigenvector of the 4x4 matrix built from
// M = sum X_i Y_i^T.  Equivalent to the SVD (Kabsch) solution with the det fix
// used by the reference (src/solver.cpp:515-525).
MP_HD void horn_rotation(const double (&M)[3][3], double *R) {
    const double Sxx = M[0][0], Sxy = M[0][1], Sxz = M[0][2];
    const double Syx = M[1][0], Syy = M[1][1], Syz = M[1][2];
    const double Szx = M[2][0], Szy = M[2][1], Szz = M[2][2];
    double N[4][4] = {{Sxx + Syy + Szz, Syz - Szy, Szx - Sxz, Sxy - Syx},
                      {Syz - Szy, Sxx - Syy - Szz, Sxy + Syx, Szx + Sxz},
                      {Szx - Sxz, Sxy + Syx, -Sxx + Syy - Szz, Syz + Szy},
                      {Sxy - Syx, Szx + Sxz, Syz + Szy, -Sxx - Syy + Szz}};
    double V[4][4];
    jacobi_eig4(N, V);
    int best = 0;
    double bv = N[0][0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (N[i][i] > bv) {
            bv = N[i][i];
            best = i;
        }
    double q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double v = V[i][0];
#pragma unroll
        for (int j = 1; j < 4; ++j)
            if (best == j) v = V[i][j];
        q[i] = v;
    }
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const double w = q[0] / n, x = q[1] / n, y = q[2] / n, z = q[3] / n;
    R[0] = 1 - 2 * (y * y + z * z);
    R[1] = 2 * (x * y - w * z);
    R[2] = 2 * (x * z + w * y);
    R[3] = 2 * (x * y + w * z);
    R[4] = 1 - 2 * (x * x + z * z);
    R[5] = 2 * (y * z - w * x);
    R[6] = 2 * (x * z - w * y);
    R[7] = 2 * (y * z + w * x);
    R[8] = 1 - 2 * (x * x + y * y);
}

// Right singular vector of the smallest singular value of a 4x4 matrix
// (one-sided Jacobi), used by DLT triangulation (src/utils.h:24-38).
MP_HD void smallest_right_sv4(const double (&A0)[4][4], double *v) {
#pragma clang fp contract(off)
    double A[4][4], V[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            A[i][j] = A0[i][j];
            V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 20; ++sweep) {
        double off = 0.0;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double al = 0, be = 0, ga = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    al += A[i][p] * A[i][p];
                    be += A[i][q] * A[i][q];
                    ga += A[i][p] * A[i][q];
                }
                const double rel = (ga != 0.0) ? fabs(ga) / sqrt(al * be) : 0.0;
                off = fmax(off, rel);
                if (rel > 1e-16) {
                    const double zeta = (be - al) / (2.0 * ga);
                    const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
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
#pragma unroll
    for (int j = 0; j < 4; ++j) nrm[j] = A[0][j] * A[0][j] + A[1][j] * A[1][j] + A[2][j] * A[2][j] + A[3][j] * A[3][j];
    // column of the smallest norm (first minimum); picked by one-hot weights rather
    // than an index or a select chain, either of which leaves V in scratch (a select
    // of loads becomes a load of a select of addresses before V is promoted)
    int k = 0;
    double best = nrm[0];
#pragma unroll
    for (int j = 1; j < 4; ++j)
        if (nrm[j] < best) {
            best = nrm[j];
            k = j;
        }
    double w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = (k == j) ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = w[0] * V[i][0] + w[1] * V[i][1] + w[2] * V[i][2] + w[3] * V[i][3];
}

// The same Jacobi sweeps with the rotations' quotients and square roots by the hardware
// reciprocal / inverse square root refined by Newton steps (within about an ulp, a third
// of the instructions of the IEEE sequences) on the device, the IEEE operations on the
// host: the two-focal recoverPose tests (mp_pt67.h), whose models are not the oracle's
// to the bit anyway (the 7pt roots differ in the last bits: ocml cbrt / acos / cos).
// smallest_right_sv4 above stays exact: it is dlt_null4's fallback, bit-identical to
// the oracle's.  Every argument is positive and finite here (al be > 0 where ga != 0;
// 1 + zeta^2, 1 + t^2 >= 1), and the sign symmetry recover_pose_good_pair relies on
// holds (the reciprocal is odd, the inverse square root sees even quantities only).
MP_HD double svd_rcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
#else
    return 1.0 / x;
#endif
}
MP_HD double svd_rsq(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = y * fma(-h * y, y, 1.5);
    return y * fma(-h * y, y, 1.5);
#else
    return 1.0 / sqrt(x);
#endif
}
MP_HD void smallest_right_sv4_fast(const double (&A0)[4][4], double *v) {
#pragma clang fp contract(off)
    double A[4][4], V[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            A[i][j] = A0[i][j];
            V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 20; ++sweep) {
        double off = 0.0;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double al = 0, be = 0, ga = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    al += A[i][p] * A[i][p];
                    be += A[i][q] * A[i][q];
                    ga += A[i][p] * A[i][q];
                }
                const double rel = (ga != 0.0) ? fabs(ga) * svd_rsq(al * be) : 0.0;
                off = fmax(off, rel);
                if (rel > 1e-16) {
                    const double zeta = (be - al) * svd_rcp(2.0 * ga);
                    const double u = 1.0 + zeta * zeta;
                    const double t = (zeta >= 0 ? 1.0 : -1.0) * svd_rcp(fabs(zeta) + u * svd_rsq(u));
                    const double c = svd_rsq(1.0 + t * t), s = c * t;
#pragma unroll
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
#pragma unroll
    for (int j = 0; j < 4; ++j) nrm[j] = A[0][j] * A[0][j] + A[1][j] * A[1][j] + A[2][j] * A[2][j] + A[3][j] * A[3][j];
    int k = 0;
    double best = nrm[0];
#pragma unroll
    for (int j = 1; j < 4; ++j)
        if (nrm[j] < best) {
            best = nrm[j];
            k = j;
        }
    double w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = (k == j) ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = w[0] * V[i][0] + w[1] * V[i][1] + w[2] * V[i][2] + w[3] * V[i][3];
}

// The same vector for the DLT triangulation of the depth fits (the chosen pose: A of
// rank 3 up to noise) without the Jacobi sweeps -- round 6: without FMA contraction,
// the oracle's dlt_null4 (oracle/src/pt.cpp) to the bit, fallback included: Householder QR of A (A^T A = R^T R,
// backward stable), then inverse iteration on R^T R by triangular solves, starting
// from R^-1 e4 -- for a rank-3 A that start is already the null vector (R[3][3] ~ 0),
// and each step multiplies the error by (s4 / s3)^2.  The iteration stops once two
// normalised iterates agree to 1e-14 (one to three steps for the depth fits); after
// NIT steps without that it falls back to the sweeps (s3 ~ s4).  About 150-250 FP64
// operations with 4 square roots and 5 reciprocals, against several thousand for
// the sweeps; the accuracy is the SVD's (error ~ eps s1 / s3; agreement with the
// sweeps to ~1e-12 in a host test over noisy two-view points).  Only the direction
// matters to the callers (they dehomogenise).  A zero diagonal of R is replaced by
// eps |R| (inverse iteration on a singular matrix; the DLT matrices have A[0][0] =
// -f != 0, so R != 0).
template <int NIT = 16> MP_HD void dlt_null4(const double (&A)[4][4], double *v) {
#pragma clang fp contract(off)
    double R[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) R[i][j] = A[i][j];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double nn = 0.0;
#pragma unroll
        for (int i = k; i < 4; ++i) nn += R[i][k] * R[i][k];
        const double nrm = sqrt(nn);
        const double alpha = R[k][k] >= 0.0 ? -nrm : nrm;
        double h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = i < k ? 0.0 : R[i][k];
        h[k] -= alpha;
        const double hh = nn - 2.0 * alpha * R[k][k] + alpha * alpha; // |h|^2
        const double f2 = hh > 0.0 ? 2.0 / hh : 0.0;
#pragma unroll
        for (int j = k; j < 4; ++j) {
            double sdot = 0.0;
#pragma unroll
            for (int i = k; i < 4; ++i) sdot += h[i] * R[i][j];
            const double f = sdot * f2;
#pragma unroll
            for (int i = k; i < 4; ++i) R[i][j] -= f * h[i];
        }
    }
    double big = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) big = fmax(big, fabs(R[i][j]));
    const double floor_ = big * 2.220446049250313e-16;
    double d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double r = R[i][i];
        d[i] = 1.0 / (fabs(r) > floor_ ? r : (r < 0.0 ? -floor_ : floor_));
    }
    // x = R^-1 e4
    double x[4];
    x[3] = d[3];
    x[2] = -(R[2][3] * x[3]) * d[2];
    x[1] = -(R[1][2] * x[2] + R[1][3] * x[3]) * d[1];
    x[0] = -(R[0][1] * x[1] + R[0][2] * x[2] + R[0][3] * x[3]) * d[0];
    bool conv = false;
    for (int it = 0; it < NIT && !conv; ++it) {
        double mx = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) mx = fmax(mx, fabs(x[i]));
        const double sc = 1.0 / mx;
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] *= sc;
        // R^T y = x (forward), then R z = y (back)
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
#pragma unroll
        for (int i = 0; i < 4; ++i) mz = fmax(mz, fabs(z[i]));
        const double rz = 1.0 / mz;
        double diff = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            diff = fmax(diff, fabs(z[i] * rz - x[i]));
            x[i] = z[i];
        }
        conv = diff < 1e-14;
    }
    if (!conv) {
        smallest_right_sv4(A, v);
        return;
    }
    const double n = 1.0 / sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = x[i] * n;
}

} // namespace mp
