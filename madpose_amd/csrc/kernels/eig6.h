// Shared-focal 6-point root stage by a deflated eigenproblem: one sample per 64-lane
// wave (one wave per workgroup), every matrix in LDS, the lanes running the inner
// loops (rows / columns) of each step and every lane replaying the step's scalar
// control identically (uniform).
//
// The ten equations (M0 + w M1 + w^2 M2) v = 0 of mp_pt67.h (sixpt_row), written in
// u = 1/w = f^2 as the quadratic eigenproblem (u^2 M0 + u M1 + M2) v = 0 and
// linearised on z = [v; u v]:  C = [0 I; -M0^-1 M2  -M0^-1 M1]  (20 x 20).
// det(u^2 M0 + u M1 + M2) = u^5 q(u) (q of degree 15), so C carries a structural
// 5-fold zero eigenvalue: the right null space of M2 (rank 6: row 0 is zero and every
// other row is F_22 times a quadratic in (x, y)) and one Jordan vector [a; v], v in
// null(M2) with M1 v in range(M2), M2 a = -M1 v.  Rounding splits that eigenvalue
// into a cluster reaching ~1e-4 of the largest root, where genuine roots also occur,
// so the invariant subspace is deflated exactly -- orthogonal similarity by the
// Householder reflectors of its basis -- and the 15 remaining eigenvalues (the roots
// of q) come from balance + elmhes + hqr (EISPACK) on the 15 x 15 block.  Positive
// real ones (wi == 0) are the candidates u, ascending.
//
// This replaces the 16-point DFT of q(u) + Sturm search (group_6pt.h, kept as an A/B
// path): the DFT loses the digits of small coefficients when the roots span several
// orders of magnitude (q's coefficients spanned up to 43 orders on random samples)
// and dropped or shifted roots; on 6000 random samples the deflated eigenvalues
// agree with a 60-digit evaluation of q's roots in all but one ill-conditioned pair
// (scratch prototype recorded in DESIGN.md §5).
//
// The math follows the oracle's restatement (oracle/src/pt67.cpp sixpt_roots: the
// same companion, the same invariant subspace, Householder reflectors of its basis,
// balance + elmhes + hqr); the arithmetic is arranged for a wave: Gauss-Jordan with
// complete pivoting instead of LU + substitutions, wave sums for the dot products,
// elmhes's column eliminations as one similarity.  Three launches: the pencil
// (register-heavy, four samples per wave), the deflation (10 KB of LDS) and the
// 15 x 15 eigenproblem (2 KB of LDS), so that each runs at its own occupancy.
#pragma once
#include "../include/mp_pt67.h"
#include "group_sturm.h"

namespace mp {
namespace {

// Phase timing / counters for tools/eig6_bench.hip (compiled out otherwise): clock
// ticks of balance, elmhes, hqr summed over samples (lane 0), then the QR iterations
// and balancing passes.
#ifdef MP_EIG6_PROFILE
__device__ unsigned long long e6_prof[8];
#define E6_MARK(i)                                                                                                     \
    do {                                                                                                               \
        const unsigned long long t_ = wall_clock64();                                                                 \
        if (threadIdx.x == 0) atomicAdd(&e6_prof[i], t_ - t_prev);                                                     \
        t_prev = t_;                                                                                                   \
    } while (0)
#define E6_START unsigned long long t_prev = wall_clock64()
#define E6_COUNT(i, v)                                                                                                 \
    do {                                                                                                               \
        if (threadIdx.x == 0) atomicAdd(&e6_prof[i], (unsigned long long)(v));                                         \
    } while (0)
#else
#define E6_MARK(i) ((void)0)
#define E6_START ((void)0)
#define E6_COUNT(i, v) ((void)0)
#endif

// ---------------------------------------------------------------------------
// wave helpers (one-wave workgroups: the barrier is cheap and orders LDS accesses)
__device__ inline void e6_bar() { __syncthreads(); }

__device__ inline double e6_readlane(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// sum over the wave (all lanes active), uniform: DPP inside the rows, rows in order
__device__ inline double e6_wsum(double v) {
    v += dpp_d<dpp::kXor1>(v);
    v += dpp_d<dpp::kXor2>(v);
    v += dpp_d<dpp::kHalfMirror>(v);
    v += dpp_d<dpp::kMirror>(v);
    return (e6_readlane(v, 0) + e6_readlane(v, 16)) + (e6_readlane(v, 32) + e6_readlane(v, 48));
}
// wave-wide (value, key) maximum, ties to the smallest key
__device__ inline void e6_argmax(double v, int key, double *bv, int *bk) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(v, off, 64);
        const int ok = __shfl_xor(key, off, 64);
        if (ov > v || (ov == v && ok < key)) {
            v = ov;
            key = ok;
        }
    }
    *bv = v;
    *bk = key;
}

// Gauss-Jordan with complete pivoting over the first np columns of the n x ncol
// matrix G (row stride LD): `steps` pivots, each the largest remaining |G(i, c)|
// (first in row-major order), the pivot row normalised and the pivot column cleared
// from every other row; pivot k at (prow[k], pcol[k]).  Returns false if a pivot
// is zero.  With np = n and steps = n, column j >= np of row prow[k] is then
// (G_left^-1 G_right)(pcol[k], j - np).
template <int LD>
__device__ bool e6_gauss_jordan(double (*G)[LD], int n, int ncol, int np, int steps, double *mul, int *prow,
                                int *pcol) {
    const int lane = threadIdx.x;
    unsigned rows = 0, cols = 0; // pivoted (uniform)
    for (int k = 0; k < steps; ++k) {
        double best = -1.0;
        int bkey = 0x7fffffff;
        for (int e = lane; e < n * np; e += 64) {
            const int i = e / np, c = e - (e / np) * np;
            if (!((rows >> i) & 1u) && !((cols >> c) & 1u)) {
                const double a = fabs(G[i][c]);
                if (a > best) {
                    best = a;
                    bkey = e;
                }
            }
        }
        double bv;
        int bk;
        e6_argmax(best, bkey, &bv, &bk);
        const int pr = bk / np, pc = bk - (bk / np) * np;
        const double piv = G[pr][pc];
        if (!(bv > 0.0)) return false; // (uniform)
        if (lane < n) mul[lane] = G[lane][pc];
        e6_bar();
        for (int c = lane; c < ncol; c += 64) G[pr][c] = G[pr][c] / piv;
        e6_bar();
        for (int e = lane; e < n * ncol; e += 64) {
            const int i = e / ncol, c = e - (e / ncol) * ncol;
            if (i != pr) G[i][c] -= mul[i] * G[pr][c];
        }
        if (lane == 0) {
            prow[k] = pr;
            pcol[k] = pc;
        }
        rows |= 1u << pr;
        cols |= 1u << pc;
        e6_bar();
    }
    return true;
}

// Front of the root stage, four samples per 64-lane wave (16-lane groups): the
// epipolar null space N (every lane of the group) into cand[0, 27) and the pencil
// rows (lane r < 10: row r of M0, M1, M2, sixpt_row) into pen (300 doubles per
// sample, M[a][r][c] at 100 a + 10 r + c).  Split from the eigen kernel so that the
// latter's register allocation is not set by this register-heavy part.
constexpr int kPenStride = 300;
__global__ void __launch_bounds__(64) pt_pencil6_kernel(PairData D, const int *list, int nlist, const int *samples,
                                                        double *cand, int cand_stride, double *pen) {
    __shared__ double shN[kGrpPerWg][27];
    const int g = threadIdx.x / kGrp, r = threadIdx.x % kGrp;
    const int idx = blockIdx.x * kGrpPerWg + g;
    const bool active = idx < nlist;
    const int *smp = samples + (size_t)list[active ? idx : nlist - 1] * kSampleStride;
    {
        double N[3][9];
        {
            double b0[6][3], b1[6][3];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int i = smp[j];
                const double a[3] = {D.x0u[i], D.x0v[i], 1.0}, c[3] = {D.x1u[i], D.x1v[i], 1.0};
                const double na = 1.0 / sqrt(dot3(a, a)), nc = 1.0 / sqrt(dot3(c, c));
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    b0[j][q] = a[q] * na;
                    b1[j][q] = c[q] * nc;
                }
            }
            double Q[6][9];
            epipolar_rows<6>(b0, b1, Q);
            nullspace_kx9<6>(Q, N);
        }
#pragma unroll
        for (int q = 0; q < 27; ++q)
            if (q % kGrp == r) shN[g][q] = N[q / 9][q % 9];
    }
    __syncthreads();
    if (!active) return;
    double *out = cand + (size_t)idx * cand_stride;
    for (int q = r; q < 27; q += kGrp) out[q] = shN[g][q];
    if (r < 10) {
        double m0[10], m1[10], m2[10];
        sixpt_row([&](int e) { return Lin2{{shN[g][e], shN[g][9 + e], shN[g][18 + e]}}; }, r, m0, m1, m2);
        double *P = pen + (size_t)idx * kPenStride;
#pragma unroll
        for (int c = 0; c < 10; ++c) {
            P[10 * r + c] = m0[c];
            P[100 + 10 * r + c] = m1[c];
            P[200 + 10 * r + c] = m2[c];
        }
    }
}

// ---------------------------------------------------------------------------
// Eigenvalues of the deflated 15 x 15 block: balance + elmhes + hqr (EISPACK, as in
// oracle/src/la.cpp), one sample per 64-lane workgroup; the positive real ones
// ascending into cand[27 ..), their number into ncand.
constexpr int kE6 = 15;
struct Eig15Shared {
    double H[kE6][kE6 + 1];
    double y[kE6];
    double wr[kE6], wi[kE6];
    double roots[kE6];
    int cnt;
};
#define E6(i, j) sh.H[i][j]

__device__ inline double e6_sign(double a, double b) { return b >= 0 ? fabs(a) : -fabs(a); }

// balance (EISPACK balanc without permutations); row / column sums as wave sums
__device__ void e6_balance(Eig15Shared &sh) {
    const int lane = threadIdx.x;
    const double radix = 2.0, sqrdx = 4.0;
    bool done = false;
    int pass = 0;
    for (; !done && pass < 64; ++pass) {
        done = true;
        for (int i = 0; i < kE6; ++i) {
            const bool on = lane < kE6 && lane != i;
            double c = e6_wsum(on ? fabs(E6(lane, i)) : 0.0);
            const double r = e6_wsum(on ? fabs(E6(i, lane)) : 0.0);
            if (c != 0.0 && r != 0.0) {
                double g = r / radix, f = 1.0;
                const double s = c + r;
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
                    done = false;
                    g = 1.0 / f;
                    if (lane < kE6) E6(i, lane) *= g;
                    e6_bar();
                    if (lane < kE6) E6(lane, i) *= f;
                    e6_bar();
                }
            }
        }
    }
    E6_COUNT(4, pass);
}

// elmhes: the eliminations of one column as one similarity G^-1 A G (all row
// operations, then the column-m update) -- the product of the sequential steps'
// commuting transforms
__device__ void e6_hessenberg(Eig15Shared &sh) {
    const int lane = threadIdx.x;
    const int n = kE6;
    for (int m = 1; m < n - 1; ++m) {
        double bv;
        int bi;
        e6_argmax((lane >= m && lane < n) ? fabs(E6(lane, m - 1)) : -1.0, lane, &bv, &bi);
        if (!(bv > 0.0)) continue; // x == 0 (uniform)
        const int i = bi;
        if (i != m) {
            if (lane >= m - 1 && lane < n) {
                const double t = E6(i, lane);
                E6(i, lane) = E6(m, lane);
                E6(m, lane) = t;
            }
            e6_bar();
            if (lane < n) {
                const double t = E6(lane, i);
                E6(lane, i) = E6(lane, m);
                E6(lane, m) = t;
            }
            e6_bar();
        }
        const double x = E6(m, m - 1);
        if (lane > m && lane < n) {
            const double y = E6(lane, m - 1) / x;
            sh.y[lane] = y;
            E6(lane, m - 1) = y;
        }
        e6_bar();
        for (int e = lane; e < n * n; e += 64) {
            const int r = e / n, c = e - (e / n) * n;
            if (r > m && c >= m) E6(r, c) -= sh.y[r] * E6(m, c);
        }
        e6_bar();
        if (lane < n) {
            double acc = E6(lane, m);
#pragma unroll
            for (int q = 0; q < kE6; ++q)
                if (q > m) acc += sh.y[q] * E6(lane, q);
            E6(lane, m) = acc;
        }
        e6_bar();
    }
    if (lane < n)
        for (int j = 0; j < lane - 1; ++j) E6(lane, j) = 0.0;
    e6_bar();
}
#undef E6

// ---------------------------------------------------------------------------
// Deflation, one sample per 64-lane workgroup, after pt_pencil6_kernel: the
// companion C, the basis Z of its zero-eigenvalue invariant subspace and the
// trailing 15 x 15 block of Q^T C Q into pen[0, 225) (row-major) -- with hess, its
// balanced upper Hessenberg form (balance + elmhes) -- and pen[225] = 1 (0: M0
// singular, no roots).
struct Defl6Shared {
    union {
        double G[10][31]; // Gauss-Jordan workspace
        Eig15Shared s15;  // balance + elmhes of the deflated block (after the last G use)
    };
    double A[20][21];  // companion, deflated in place
    double Nr[10][4], Nl[10][4];
    double T[4][10], S[4][4];
    double Z[20][5];
    double hv[20];
    double mul[10];
    double v[10], rhs[10], pa[10], cv[4];
    int prow[10], pcol[10], colrow[10];
};

// the right null space (n - rank vectors, columns of out) after a rank-`rank`
// Gauss-Jordan of an n x n G: x_f = 1 on free column f, -G(prow[k], f) on pcol[k]
template <int LD, int LDO>
__device__ void e6_null_gj(const double (*G)[LD], int n, int rank, const int *prow, const int *pcol,
                           double (*out)[LDO]) {
    const int lane = threadIdx.x;
    unsigned piv = 0;
    for (int k = 0; k < rank; ++k) piv |= 1u << pcol[k];
    // free columns in ascending order
    int f = 0;
    for (int c = 0; c < n; ++c) {
        if ((piv >> c) & 1u) continue;
        if (lane < n) {
            double x = (lane == c) ? 1.0 : 0.0;
            for (int k = 0; k < rank; ++k)
                if (pcol[k] == lane) x = -G[prow[k]][c];
            out[lane][f] = x;
        }
        ++f;
    }
    e6_bar();
}

__global__ void __launch_bounds__(64) pt_defl6_kernel(double *pen, bool hess) {
    __shared__ Defl6Shared sh;
    const int lane = threadIdx.x;
    double *P = pen + (size_t)blockIdx.x * kPenStride;
    // M1, M2 are read from the pencil rows in global memory (L2-resident, written by
    // pt_pencil6_kernel) instead of LDS copies: 1.6 KB less LDS per workgroup
    const double *M1 = P + 100, *M2 = P + 200;
#define M1_(r, c) M1[10 * (r) + (c)]
#define M2_(r, c) M2[10 * (r) + (c)]
    // G = [M0 | M2 | M1]
    for (int e = lane; e < 300; e += 64) {
        const int a = e / 100, r = (e / 10) % 10, c = e % 10;
        const double x = P[e];
        if (a == 0) sh.G[r][c] = x;
        if (a == 1) sh.G[r][20 + c] = x;
        if (a == 2) sh.G[r][10 + c] = x;
    }
    e6_bar();
    // ---- C = [0 I; -M0^-1 [M2 M1]] ----
    if (!e6_gauss_jordan<31>(sh.G, 10, 30, 10, 10, sh.mul, sh.prow, sh.pcol)) {
        if (lane == 0) P[225] = 0.0;
        return; // (uniform)
    }
    if (lane < 10) sh.colrow[sh.pcol[lane]] = sh.prow[lane];
    e6_bar();
    for (int e = lane; e < 400; e += 64) {
        const int i = e / 20, j = e % 20;
        sh.A[i][j] = i < 10 ? ((j == 10 + i) ? 1.0 : 0.0) : -sh.G[sh.colrow[i - 10]][10 + j];
    }
    e6_bar();
    // ---- the zero-eigenvalue invariant subspace ----
    // left null space of M2 (Gauss-Jordan of M2^T, rank 6)
    for (int e = lane; e < 100; e += 64) sh.G[e / 10][e % 10] = M2_(e % 10, e / 10);
    e6_bar();
    e6_gauss_jordan<31>(sh.G, 10, 10, 10, 6, sh.mul, sh.prow, sh.pcol);
    e6_null_gj<31, 4>(sh.G, 10, 6, sh.prow, sh.pcol, sh.Nl);
    // right null space of M2
    for (int e = lane; e < 100; e += 64) sh.G[e / 10][e % 10] = M2_(e / 10, e % 10);
    e6_bar();
    e6_gauss_jordan<31>(sh.G, 10, 10, 10, 6, sh.mul, sh.prow, sh.pcol);
    e6_null_gj<31, 4>(sh.G, 10, 6, sh.prow, sh.pcol, sh.Nr);
    // S = Nl^T M1 Nr (4 x 4, rank 3) and its null vector c
    if (lane < 40) {
        const int i = lane / 10, c = lane % 10;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 10; ++k) acc += sh.Nl[k][i] * M1_(k, c);
        sh.T[i][c] = acc;
    }
    e6_bar();
    if (lane < 16) {
        const int i = lane / 4, j = lane % 4;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 10; ++k) acc += sh.T[i][k] * sh.Nr[k][j];
        sh.G[i][j] = acc;
    }
    e6_bar();
    e6_gauss_jordan<31>(sh.G, 4, 4, 4, 3, sh.mul, sh.prow, sh.pcol);
    e6_null_gj<31, 1>(sh.G, 4, 3, sh.prow, sh.pcol, (double(*)[1])sh.cv);
    // v = Nr c, rhs = -M1 v
    if (lane < 10) {
        double acc = 0.0;
#pragma unroll
        for (int f = 0; f < 4; ++f) acc += sh.Nr[lane][f] * sh.cv[f];
        sh.v[lane] = acc;
    }
    e6_bar();
    if (lane < 10) {
        double acc = 0.0;
#pragma unroll
        for (int c = 0; c < 10; ++c) acc += M1_(lane, c) * sh.v[c];
        sh.rhs[lane] = -acc;
    }
    e6_bar();
    // a particular solution of M2 a = rhs: Gauss-Jordan of [M2 | rhs], 6 pivots
    for (int e = lane; e < 110; e += 64) {
        const int i = e / 11, c = e % 11;
        sh.G[i][c] = c < 10 ? M2_(i, c) : sh.rhs[i];
    }
    e6_bar();
    e6_gauss_jordan<31>(sh.G, 10, 11, 10, 6, sh.mul, sh.prow, sh.pcol);
    if (lane < 10) sh.pa[lane] = 0.0;
    e6_bar();
    if (lane < 6) sh.pa[sh.pcol[lane]] = sh.G[sh.prow[lane]][10];
    e6_bar();
    // Z = [Nr a; 0 v]
    if (lane < 20) {
#pragma unroll
        for (int f = 0; f < 4; ++f) sh.Z[lane][f] = lane < 10 ? sh.Nr[lane][f] : 0.0;
        sh.Z[lane][4] = lane < 10 ? sh.pa[lane] : sh.v[lane - 10];
    }
    e6_bar();
    // ---- C <- Q^T C Q, Q = H_0 ... H_4 the Householder reflectors of the QR of Z ----
    for (int k = 0; k < 5; ++k) {
        const double zi = (lane >= k && lane < 20) ? sh.Z[lane][k] : 0.0;
        double alpha = sqrt(e6_wsum(zi * zi));
        if (alpha == 0.0) continue; // (uniform)
        if (sh.Z[k][k] > 0) alpha = -alpha;
        const double hv = zi - (lane == k ? alpha : 0.0);
        const double vn = e6_wsum(hv * hv);
        if (!(vn > 0.0)) continue; // (uniform)
        if (lane < 20) sh.hv[lane] = hv;
        e6_bar();
        const double sc = 2.0 / vn;
        if (lane > k && lane < 5) { // the rest of Z
            double d = 0.0;
#pragma unroll
            for (int i = 0; i < 20; ++i)
                if (i >= k) d += sh.hv[i] * sh.Z[i][lane];
            d *= sc;
#pragma unroll
            for (int i = 0; i < 20; ++i)
                if (i >= k) sh.Z[i][lane] -= d * sh.hv[i];
        }
        if (lane < 20) { // C <- H C: column `lane`
            double d = 0.0;
#pragma unroll
            for (int i = 0; i < 20; ++i)
                if (i >= k) d += sh.hv[i] * sh.A[i][lane];
            d *= sc;
#pragma unroll
            for (int i = 0; i < 20; ++i)
                if (i >= k) sh.A[i][lane] -= d * sh.hv[i];
        }
        e6_bar();
        if (lane < 20) { // C <- C H: row `lane`
            double d = 0.0;
#pragma unroll
            for (int j = 0; j < 20; ++j)
                if (j >= k) d += sh.A[lane][j] * sh.hv[j];
            d *= sc;
#pragma unroll
            for (int j = 0; j < 20; ++j)
                if (j >= k) sh.A[lane][j] -= d * sh.hv[j];
        }
        e6_bar();
    }
    if (!hess) {
        for (int e = lane; e < 225; e += 64) P[e] = sh.A[5 + e / 15][5 + e % 15];
        if (lane == 0) P[225] = 1.0;
        return;
    }
#undef M1_
#undef M2_
    // balanced upper Hessenberg form of the block (for pt_eig6_reg_kernel), in the
    // Gauss-Jordan workspace (free from here on)
    Eig15Shared &s15 = sh.s15;
    for (int e = lane; e < 225; e += 64) s15.H[e / 15][e % 15] = sh.A[5 + e / 15][5 + e % 15];
    e6_bar();
    e6_balance(s15);
    e6_hessenberg(s15);
    for (int e = lane; e < 225; e += 64) P[e] = s15.H[e / 15][e % 15];
    if (lane == 0) P[225] = 1.0;
}

#define E6(i, j) sh.H[i][j]
// hqr (oracle/src/la.cpp, EISPACK); false if an eigenvalue took 60 iterations
__device__ bool e6_hqr(Eig15Shared &sh) {
    const int lane = threadIdx.x;
    const int n = kE6;
    if (lane < n) {
        sh.wr[lane] = 0.0;
        sh.wi[lane] = 0.0;
    }
    double anorm = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = (i - 1 > 0 ? i - 1 : 0); j < n; ++j) anorm += fabs(E6(i, j));
    int nn = n - 1;
    double t = 0.0;
    double p = 0, q = 0, r = 0, s = 0, w = 0, x = 0, y = 0, z = 0;
    while (nn >= 0) {
        int its = 0, l;
        do {
            for (l = nn; l >= 1; --l) {
                s = fabs(E6(l - 1, l - 1)) + fabs(E6(l, l));
                if (s == 0.0) s = anorm;
                if (fabs(E6(l, l - 1)) + s == s) {
                    e6_bar();
                    if (lane == 0) E6(l, l - 1) = 0.0;
                    e6_bar();
                    break;
                }
            }
            x = E6(nn, nn);
            if (l == nn) {
                if (lane == 0) {
                    sh.wr[nn] = x + t;
                    sh.wi[nn] = 0.0;
                }
                nn--;
            } else {
                y = E6(nn - 1, nn - 1);
                w = E6(nn, nn - 1) * E6(nn - 1, nn);
                if (l == nn - 1) {
                    p = 0.5 * (y - x);
                    q = p * p + w;
                    z = sqrt(fabs(q));
                    x += t;
                    if (q >= 0.0) z = p + e6_sign(z, p); // (uniform)
                    if (lane == 0) {
                        if (q >= 0.0) {
                            sh.wr[nn - 1] = sh.wr[nn] = x + z;
                            if (z != 0.0) sh.wr[nn] = x - w / z;
                            sh.wi[nn - 1] = sh.wi[nn] = 0.0;
                        } else {
                            sh.wr[nn - 1] = sh.wr[nn] = x + p;
                            sh.wi[nn] = z;
                            sh.wi[nn - 1] = -z;
                        }
                    }
                    nn -= 2;
                } else {
                    if (its == 60) return false;
                    if (its == 10 || its == 20 || its == 40) {
                        t += x;
                        e6_bar();
                        if (lane <= nn) E6(lane, lane) -= x;
                        e6_bar();
                        s = fabs(E6(nn, nn - 1)) + fabs(E6(nn - 1, nn - 2));
                        y = x = 0.75 * s;
                        w = -0.4375 * s * s;
                    }
                    ++its;
                    E6_COUNT(5, 1);
                    int m;
                    for (m = nn - 2; m >= l; --m) {
                        z = E6(m, m);
                        r = x - z;
                        s = y - z;
                        p = (r * s - w) / E6(m + 1, m) + E6(m, m + 1);
                        q = E6(m + 1, m + 1) - z - r - s;
                        r = E6(m + 2, m + 1);
                        s = fabs(p) + fabs(q) + fabs(r);
                        p /= s;
                        q /= s;
                        r /= s;
                        if (m == l) break;
                        const double u = fabs(E6(m, m - 1)) * (fabs(q) + fabs(r));
                        const double v = fabs(p) * (fabs(E6(m - 1, m - 1)) + fabs(z) + fabs(E6(m + 1, m + 1)));
                        if (u + v == v) break;
                    }
                    e6_bar();
                    if (lane >= m + 2 && lane <= nn) {
                        E6(lane, lane - 2) = 0.0;
                        if (lane != m + 2) E6(lane, lane - 3) = 0.0;
                    }
                    e6_bar();
                    for (int k = m; k <= nn - 1; ++k) {
                        if (k != m) {
                            p = E6(k, k - 1);
                            q = E6(k + 1, k - 1);
                            r = 0.0;
                            if (k != nn - 1) r = E6(k + 2, k - 1);
                            if ((x = fabs(p) + fabs(q) + fabs(r)) != 0.0) {
                                p /= x;
                                q /= x;
                                r /= x;
                            }
                        }
                        if ((s = e6_sign(sqrt(p * p + q * q + r * r), p)) != 0.0) {
                            e6_bar();
                            if (lane == 0) {
                                if (k == m) {
                                    if (l != m) E6(k, k - 1) = -E6(k, k - 1);
                                } else {
                                    E6(k, k - 1) = -s * x;
                                }
                            }
                            p += s;
                            x = p / s;
                            y = q / s;
                            z = r / s;
                            q /= p;
                            r /= p;
                            e6_bar();
                            // rows k..k+2, columns k..nn (lane j)
                            if (lane >= k && lane <= nn) {
                                const int j = lane;
                                double pp = E6(k, j) + q * E6(k + 1, j);
                                if (k != nn - 1) {
                                    pp += r * E6(k + 2, j);
                                    E6(k + 2, j) -= pp * z;
                                }
                                E6(k + 1, j) -= pp * y;
                                E6(k, j) -= pp * x;
                            }
                            e6_bar();
                            // columns k..k+2, rows l..min(nn, k+3) (lane i)
                            const int mmin = nn < k + 3 ? nn : k + 3;
                            if (lane >= l && lane <= mmin) {
                                const int i = lane;
                                double pp = x * E6(i, k) + y * E6(i, k + 1);
                                if (k != nn - 1) {
                                    pp += z * E6(i, k + 2);
                                    E6(i, k + 2) -= pp * r;
                                }
                                E6(i, k + 1) -= pp * q;
                                E6(i, k) -= pp;
                            }
                            e6_bar();
                        }
                    }
                }
            }
        } while (l < nn - 1);
    }
    e6_bar();
    return true;
}
#undef E6

__global__ void __launch_bounds__(64) pt_eig6_kernel(const double *pen, double *cand, int *ncand, int cand_stride) {
    __shared__ Eig15Shared sh;
    const int lane = threadIdx.x, idx = blockIdx.x;
    const double *P = pen + (size_t)idx * kPenStride;
    if (P[225] == 0.0) { // M0 singular: no roots (uniform)
        if (lane == 0) ncand[idx] = 0;
        return;
    }
    for (int e = lane; e < kE6 * kE6; e += 64) sh.H[e / kE6][e % kE6] = P[e];
    e6_bar();
    E6_START;
    e6_balance(sh);
    E6_MARK(0);
    e6_hessenberg(sh);
    E6_MARK(1);
    int nroots = 0;
    const bool conv = e6_hqr(sh);
    E6_MARK(2);
    if (conv) {
        // positive real roots, ascending (insertion sort in lane 0)
        if (lane == 0) {
            int cnt = 0;
            for (int k = 0; k < kE6; ++k) {
                const double u = sh.wr[k];
                if (sh.wi[k] == 0.0 && u > 0.0) {
                    int q = cnt;
                    while (q > 0 && sh.roots[q - 1] > u) {
                        sh.roots[q] = sh.roots[q - 1];
                        --q;
                    }
                    sh.roots[q] = u;
                    ++cnt;
                }
            }
            sh.cnt = cnt;
        }
        e6_bar();
        nroots = sh.cnt;
        double *out = cand + (size_t)idx * cand_stride;
        if (lane < nroots) out[27 + lane] = sh.roots[lane];
    }
    if (lane == 0) ncand[idx] = nroots;
}

// ---------------------------------------------------------------------------
// The same eigenproblem with one sample per LANE (64 samples per wave): every lane
// runs balance + elmhes + hqr serially on its own 15 x 15 matrix, the matrices kept
// in LDS element-major / lane-minor (element e of lane l at [e][l]: the 64 lanes of
// one access always fall in distinct banks, whatever element each lane addresses).
// The control flow diverges between lanes (different QR iteration counts and bulge
// lengths), but each instruction serves up to 64 samples instead of one: measured
// (tools/eig6_bench.hip) far cheaper than the one-sample-per-wave kernel above, whose
// mostly uniform scalar work occupies whole waves.  The code is oracle/src/la.cpp's
// balance / to_hessenberg / hqr line for line.
struct Eig15LaneShared {
    double H[kE6 * kE6][64];
    double wr[kE6][64], wi[kE6][64];
};

__global__ void __launch_bounds__(64) pt_eig6_lane_kernel(const double *pen, int nlist, double *cand, int *ncand,
                                                          int cand_stride) {
    __shared__ Eig15LaneShared sh;
    const int lane = threadIdx.x;
    const int base = blockIdx.x * 64;
    // coalesced load: sample by sample, lanes over the elements
    for (int q = 0; q < 64 && base + q < nlist; ++q) {
        const double *P = pen + (size_t)(base + q) * kPenStride;
        for (int e = lane; e < kE6 * kE6; e += 64) sh.H[e][q] = P[e];
    }
    __syncthreads();
    const int idx = base + lane;
    if (idx >= nlist) return;
    if (pen[(size_t)idx * kPenStride + 225] == 0.0) {
        ncand[idx] = 0;
        return;
    }
#define A(i, j) sh.H[(i) * kE6 + (j)][lane]
    const int n = kE6;
    E6_START;
    // ---- balance ----
    {
        const double radix = 2.0, sqrdx = 4.0;
        bool done = false;
        int pass = 0;
        while (!done && pass < 64) {
            ++pass;
            done = true;
            for (int i = 0; i < n; ++i) {
                double r = 0, c = 0;
                for (int j = 0; j < n; ++j)
                    if (j != i) {
                        c += fabs(A(j, i));
                        r += fabs(A(i, j));
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
                        done = false;
                        g = 1.0 / f;
                        for (int j = 0; j < n; ++j) A(i, j) *= g;
                        for (int j = 0; j < n; ++j) A(j, i) *= f;
                    }
                }
            }
        }
        E6_COUNT(4, pass);
    }
    E6_MARK(0);
    // ---- elmhes ----
    for (int m = 1; m < n - 1; ++m) {
        double x = 0.0;
        int i = m;
        for (int j = m; j < n; ++j)
            if (fabs(A(j, m - 1)) > fabs(x)) {
                x = A(j, m - 1);
                i = j;
            }
        if (i != m) {
            for (int j = m - 1; j < n; ++j) {
                const double t = A(i, j);
                A(i, j) = A(m, j);
                A(m, j) = t;
            }
            for (int j = 0; j < n; ++j) {
                const double t = A(j, i);
                A(j, i) = A(j, m);
                A(j, m) = t;
            }
        }
        if (x != 0.0) {
            for (i = m + 1; i < n; ++i) {
                double y = A(i, m - 1);
                if (y != 0.0) {
                    y /= x;
                    A(i, m - 1) = y;
                    for (int j = m; j < n; ++j) A(i, j) -= y * A(m, j);
                    for (int j = 0; j < n; ++j) A(j, m) += y * A(j, i);
                }
            }
        }
    }
    for (int i = 2; i < n; ++i)
        for (int j = 0; j < i - 1; ++j) A(i, j) = 0.0;
    E6_MARK(1);
    // ---- hqr ----
    bool ok = true;
    {
        for (int i = 0; i < n; ++i) {
            sh.wr[i][lane] = 0.0;
            sh.wi[i][lane] = 0.0;
        }
        double anorm = 0.0;
        for (int i = 0; i < n; ++i)
            for (int j = (i - 1 > 0 ? i - 1 : 0); j < n; ++j) anorm += fabs(A(i, j));
        int nn = n - 1;
        double t = 0.0;
        double p = 0, q = 0, r = 0, s = 0, w = 0, x = 0, y = 0, z = 0;
        while (nn >= 0 && ok) {
            int its = 0, l;
            do {
                for (l = nn; l >= 1; --l) {
                    s = fabs(A(l - 1, l - 1)) + fabs(A(l, l));
                    if (s == 0.0) s = anorm;
                    if (fabs(A(l, l - 1)) + s == s) {
                        A(l, l - 1) = 0.0;
                        break;
                    }
                }
                x = A(nn, nn);
                if (l == nn) {
                    sh.wr[nn][lane] = x + t;
                    sh.wi[nn][lane] = 0.0;
                    nn--;
                } else {
                    y = A(nn - 1, nn - 1);
                    w = A(nn, nn - 1) * A(nn - 1, nn);
                    if (l == nn - 1) {
                        p = 0.5 * (y - x);
                        q = p * p + w;
                        z = sqrt(fabs(q));
                        x += t;
                        if (q >= 0.0) {
                            z = p + e6_sign(z, p);
                            sh.wr[nn - 1][lane] = sh.wr[nn][lane] = x + z;
                            if (z != 0.0) sh.wr[nn][lane] = x - w / z;
                            sh.wi[nn - 1][lane] = sh.wi[nn][lane] = 0.0;
                        } else {
                            sh.wr[nn - 1][lane] = sh.wr[nn][lane] = x + p;
                            sh.wi[nn][lane] = z;
                            sh.wi[nn - 1][lane] = -z;
                        }
                        nn -= 2;
                    } else {
                        if (its == 60) {
                            ok = false;
                            break;
                        }
                        if (its == 10 || its == 20 || its == 40) {
                            t += x;
                            for (int i = 0; i <= nn; ++i) A(i, i) -= x;
                            s = fabs(A(nn, nn - 1)) + fabs(A(nn - 1, nn - 2));
                            y = x = 0.75 * s;
                            w = -0.4375 * s * s;
                        }
                        ++its;
                        E6_COUNT(5, 1);
                        int m;
                        for (m = nn - 2; m >= l; --m) {
                            z = A(m, m);
                            r = x - z;
                            s = y - z;
                            p = (r * s - w) / A(m + 1, m) + A(m, m + 1);
                            q = A(m + 1, m + 1) - z - r - s;
                            r = A(m + 2, m + 1);
                            s = fabs(p) + fabs(q) + fabs(r);
                            p /= s;
                            q /= s;
                            r /= s;
                            if (m == l) break;
                            const double u = fabs(A(m, m - 1)) * (fabs(q) + fabs(r));
                            const double v = fabs(p) * (fabs(A(m - 1, m - 1)) + fabs(z) + fabs(A(m + 1, m + 1)));
                            if (u + v == v) break;
                        }
                        for (int i = m + 2; i <= nn; ++i) {
                            A(i, i - 2) = 0.0;
                            if (i != m + 2) A(i, i - 3) = 0.0;
                        }
                        for (int k = m; k <= nn - 1; ++k) {
                            if (k != m) {
                                p = A(k, k - 1);
                                q = A(k + 1, k - 1);
                                r = 0.0;
                                if (k != nn - 1) r = A(k + 2, k - 1);
                                if ((x = fabs(p) + fabs(q) + fabs(r)) != 0.0) {
                                    p /= x;
                                    q /= x;
                                    r /= x;
                                }
                            }
                            if ((s = e6_sign(sqrt(p * p + q * q + r * r), p)) != 0.0) {
                                if (k == m) {
                                    if (l != m) A(k, k - 1) = -A(k, k - 1);
                                } else
                                    A(k, k - 1) = -s * x;
                                p += s;
                                x = p / s;
                                y = q / s;
                                z = r / s;
                                q /= p;
                                r /= p;
                                for (int j = k; j <= nn; ++j) {
                                    p = A(k, j) + q * A(k + 1, j);
                                    if (k != nn - 1) {
                                        p += r * A(k + 2, j);
                                        A(k + 2, j) -= p * z;
                                    }
                                    A(k + 1, j) -= p * y;
                                    A(k, j) -= p * x;
                                }
                                const int mmin = nn < k + 3 ? nn : k + 3;
                                for (int i = l; i <= mmin; ++i) {
                                    p = x * A(i, k) + y * A(i, k + 1);
                                    if (k != nn - 1) {
                                        p += z * A(i, k + 2);
                                        A(i, k + 2) -= p * r;
                                    }
                                    A(i, k + 1) -= p * q;
                                    A(i, k) -= p;
                                }
                            }
                        }
                    }
                }
            } while (ok && l < nn - 1);
        }
    }
#undef A
    E6_MARK(2);
    int cnt = 0;
    if (ok) {
        double *out = cand + (size_t)idx * cand_stride + 27;
        // positive real roots, ascending (insertion sort in the output row)
        for (int k = 0; k < n; ++k) {
            const double u = sh.wr[k][lane];
            if (sh.wi[k][lane] == 0.0 && u > 0.0) {
                int qq = cnt;
                while (qq > 0 && out[qq - 1] > u) {
                    out[qq] = out[qq - 1];
                    --qq;
                }
                out[qq] = u;
                ++cnt;
            }
        }
    }
    ncand[idx] = cnt;
}

// ---------------------------------------------------------------------------
// The 15 x 15 eigenproblem with one sample per lane, every access static:
// every lane runs balancing, elmhes and the Francis double-shift QR (hqr) on its
// own matrix, but all 64 lanes execute the same static instruction stream -- every
// loop bound is a compile-time constant, every array index a constant after
// unrolling, and the per-lane quantities (active window, pivot rows, deflation)
// enter only through selects.  The matrices live in LDS, element-major / lane-minor
// (115 KB per 64 samples); static offsets let the compiler batch the loads of a
// step (in registers the 225 doubles per lane overflowed the register file).  A QR sweep always runs the 14 bulge positions; a
// position outside a lane's active window [l, nn] applies the identity reflector.
// Row updates run to column 14 and column updates from row 0 (the full Schur-form
// updates), which leaves the window's eigenvalues unchanged.  The chase starts at
// the window's top l (hqr may start lower when a subdiagonal decouples: the same
// similarity up to rounding).  No LDS, no divergence: a wave of 64 samples takes
// about as long as one sample, so one launch handles up to 64 x 1024 samples at
// that latency.  Eigenvalues leave through global memory (wr, wi: 15 + 15 doubles
// per sample in eig, lane-major), roots through cand / ncand.
constexpr int kN15 = 15;
} // namespace
} // namespace mp
#include "eig15_gen.h"
namespace mp {
namespace {

// spw: samples per wave (lanes spw..63 idle).  The kernel is issue-bound on one wave
// per SIMD and a wave runs until its slowest lane's QR has converged, so the launch
// spreads the samples over about one wave per SIMD (kernels.hip launch_sf_eig): fewer
// lanes per wave, fewer rounds.  A lane's arithmetic does not depend on the others
// (its updates are exact no-ops while it waits), so the roots are the same for any spw.
__global__ void __launch_bounds__(64) pt_eig6_reg_kernel(double *pen, int nlist, int spw, double *cand, int *ncand,
                                                         int cand_stride) {
    const int idx = blockIdx.x * spw + threadIdx.x;
    const bool valid = (int)threadIdx.x < spw && idx < nlist;
    const int sidx = valid ? idx : nlist - 1;
    double *P = pen + (size_t)sidx * kPenStride;
    const bool active = valid && P[225] != 0.0;
    // eigenvalues into the sample's own pencil slot past the block (free by now)
    double *wr = P + 240, *wi = wr + kN15;
#ifdef MP_EIG6_PROFILE
    const unsigned long long t_hqr0 = wall_clock64();
#endif
    const bool conv = e15_hqr(P, active, wr, wi);
#ifdef MP_EIG6_PROFILE
    if (threadIdx.x == 0) atomicAdd(&e6_prof[6], wall_clock64() - t_hqr0);
#endif
    if (!valid) return;
    int cnt = 0;
    if (conv) {
        double *out = cand + (size_t)idx * cand_stride + 27;
        for (int k = 0; k < kN15; ++k) {
            const double u = wr[k];
            if (wi[k] == 0.0 && u > 0.0) {
                int qq = cnt;
                while (qq > 0 && out[qq - 1] > u) {
                    out[qq] = out[qq - 1];
                    --qq;
                }
                out[qq] = u;
                ++cnt;
            }
        }
    }
    ncand[idx] = cnt;
}

} // namespace
} // namespace mp
