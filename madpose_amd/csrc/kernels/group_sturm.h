// Group-parallel building blocks of the point-solver root stages: one 16-lane group
// of a 64-lane workgroup per minimal sample (4 samples per workgroup).
//
//   gmax / gbcast / gscan   group reductions, broadcasts and prefix sums (shuffles)
//   group_sturm_roots<NN>   sturm_real_roots<NN> (mp_math.h) spread over the group:
//     * the Sturm chain is built coefficient-parallel (lane j owns coefficient j of
//       every chain polynomial; the chain is kept in LDS),
//     * the sign-change counts at the 33 points of the isolation grid are split over
//       the lanes, the grid cells are isolated lane-parallel,
//     * one lane per isolated root for the safeguarded Newton refinement.
//     The operations per value are those of the one-lane code (same chain, grid,
//     bisection and refinement expressions), so the roots agree with it up to FMA
//     contraction.
// Every lane of the workgroup must call group_sturm_roots (it holds barriers).
#pragma once
#include "../include/mp_math.h"
#include "kernels.h"

namespace mp {
namespace {

constexpr int kGrp = 16;              // lanes per sample
constexpr int kGrpPerWg = 64 / kGrp;  // samples per 64-lane workgroup
constexpr int kGridCells = 32;        // isolation grid of sturm_real_roots

__device__ inline double gmax(double v) {
#pragma unroll
    for (int m = kGrp / 2; m > 0; m >>= 1) v = fmax(v, __shfl_xor(v, m, kGrp));
    return v;
}
__device__ inline double gbcast(double v, int src) { return __shfl(v, src, kGrp); }
__device__ inline int gbcast(int v, int src) { return __shfl(v, src, kGrp); }
// exclusive prefix sum over the group; *total = sum over the group
__device__ inline int gscan(int v, int lane, int *total) {
    int x = v;
#pragma unroll
    for (int d = 1; d < kGrp; d <<= 1) {
        const int y = __shfl_up(x, d, kGrp);
        if (lane >= d) x += y;
    }
    *total = __shfl(x, kGrp - 1, kGrp);
    return x - v;
}

// LDS of one group's root search
template <int NN> struct GroupSturm {
    double chain[NN + 1][NN + 1];   // Sturm chain (poly k: ascending, degree NN - k)
    int cnt[kGridCells + 1];        // sign-change counts at the grid points
    double lo[NN], hi[NN];          // isolating intervals (scaled variable)
};

// Sturm sign changes at x from the chain in LDS
template <int NN> __device__ inline int sturm_count_lds(const double (*ch)[NN + 1], int len, double x) {
    int changes = 0;
    double prev = 0.0;
#pragma unroll
    for (int k = 0; k <= NN; ++k) {
        if (k < len) {
            double v = 0.0;
#pragma unroll
            for (int j = NN - k; j >= 0; --j) v = v * x + ch[k][j];
            if (v != 0.0) {
                if (prev != 0.0 && ((v < 0) != (prev < 0))) ++changes;
                prev = v;
            }
        }
    }
    return changes;
}

// The roots of one cell (x_lo, x_hi] holding clo - chi roots, as in sturm_isolate
template <int NN>
__device__ inline void cell_intervals(const double (*ch)[NN + 1], int len, double lo, double hi, int clo, int chi,
                                      RootIntervals<NN> &I) {
    if (clo - chi == 1) {
        I.push(lo, hi);
        return;
    }
    for (int guard = 0; guard < NN && clo > chi; ++guard) {
        double a = lo, b = hi;
        int ca = clo, cb = chi;
        for (int depth = 0; depth < 100; ++depth) {
            if (ca - cb == 1 || b - a <= 1e-14 * fmax(1.0, fmax(fabs(a), fabs(b)))) break;
            const double m = 0.5 * (a + b);
            const int cm = sturm_count_lds<NN>(ch, len, m);
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

// Real roots of the degree-NN polynomial p (ascending coefficients, held by every
// lane of the group), as sturm_real_roots<NN>.  Returns the number of roots (the same
// in every lane; 0 when !ok); lane r < count receives root r (ascending) in *root.
template <int NN>
__device__ int group_sturm_roots(const double (&p)[NN + 1], int r, GroupSturm<NN> &S, bool ok, double *root) {
    static_assert(NN < kGrp, "one chain coefficient per lane");
    double mx = 0.0;
#pragma unroll
    for (int j = 0; j <= NN; ++j) mx = fmax(mx, fabs(p[j]));
    ok = ok && (mx > 0.0) && (fabs(p[NN]) > 1e-300);
    double c[NN + 1];
    const double lead = 1.0 / p[NN];
#pragma unroll
    for (int j = 0; j <= NN; ++j) c[j] = p[j] * lead; // monic
    // sigma = max_j |c_j|^(1/(N-j)): lane j takes coefficient j
    double sigma;
    {
        double cj = 0.0;
#pragma unroll
        for (int j = 0; j < NN; ++j) cj = (r == j) ? c[j] : cj;
        const double pj = (r < NN && cj != 0.0) ? pow(fabs(cj), 1.0 / (NN - r)) : 0.0;
        sigma = gmax(pj);
        if (!(sigma > 0.0) || !(sigma < 1e300)) sigma = 1.0;
    }
    // this lane's coefficient of the scaled monic polynomial (lane j: cs[j])
    double cs_j;
    {
        const double inv = 1.0 / sigma;
        double q = 1.0, v = (r == NN) ? 1.0 : 0.0;
#pragma unroll
        for (int j = NN - 1; j >= 0; --j) {
            q *= inv;
            v = (r == j) ? c[j] * q : v;
        }
        cs_j = v;
    }
    // chain, coefficient-parallel: lane j holds coefficient j of s[k-1] (a) and s[k] (b)
    int len;
    {
        const double m0 = gmax(fabs(cs_j));
        const double sc0 = m0 > 0 ? 1.0 / m0 : 1.0;
        double a = cs_j * sc0; // s[0]
        const double up = __shfl(a, (r + 1) & (kGrp - 1), kGrp);
        double b = (r < NN) ? (r + 1) * up : 0.0; // derivative
        const double m1 = gmax(fabs(b));
        if (r < NN) b /= m1;
        if (r <= NN) {
            S.chain[0][r] = a;
            S.chain[1][r] = b;
        }
        len = 2;
        bool alive = true;
#pragma unroll
        for (int k = 1; k < NN; ++k) {
            const int d = NN - k;
            const double bd = gbcast(b, d);
            const double bmax = gmax((r <= d) ? fabs(b) : 0.0);
            if (!(fabs(bd) > 1e-14 * bmax)) alive = false;
            const double ad1 = gbcast(a, d + 1), ad = gbcast(a, d), bdm1 = gbcast(b, d - 1);
            const double q1 = ad1 / bd;
            const double q0 = (ad - q1 * bdm1) / bd;
            // (the shuffle runs on every lane: a shuffle inside the conditional would
            // read lane 0 while lane 0 is masked off)
            const double b_left = __shfl(b, (r + kGrp - 1) & (kGrp - 1), kGrp);
            const double bm1 = r > 0 ? b_left : 0.0;
            const double nxt = (r < d) ? -(a - q1 * bm1 - q0 * b) : 0.0;
            const double rmax = gmax(fabs(nxt));
            const double amax = gmax((r <= d + 1) ? fabs(a) : 0.0);
            if (alive && !(rmax > 1e-15 * amax)) alive = false;
            if (alive) {
                const double s_next = (r < d) ? nxt / rmax : 0.0;
                if (r <= NN) S.chain[k + 1][r] = s_next;
                len = k + 2;
                a = b;
                b = s_next;
            }
        }
    }
    __syncthreads();
    const double(*ch)[NN + 1] = S.chain;

    // counts at the grid points x_i = -B + i h (i = 0..32), lanes i and i + 16
    const double Bnd = 3.0, h = 2.0 * Bnd / kGridCells;
    {
        const double xa = -Bnd + r * h, xb = -Bnd + (r + kGrp) * h;
        S.cnt[r] = sturm_count_lds<NN>(ch, len, xa);
        S.cnt[r + kGrp] = sturm_count_lds<NN>(ch, len, xb);
        if (r == 0) S.cnt[kGridCells] = sturm_count_lds<NN>(ch, len, Bnd);
    }
    __syncthreads();

    // cells r and r + 16 isolated by this lane; intervals gathered in cell order
    int nint = 0;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        const int cell = r + pass * kGrp;
        const double x_lo = -Bnd + cell * h, x_hi = (cell + 1 == kGridCells) ? Bnd : -Bnd + (cell + 1) * h;
        const int v_lo = S.cnt[cell], v_hi = S.cnt[cell + 1];
        RootIntervals<NN> I;
        if (ok && v_lo > v_hi) cell_intervals<NN>(ch, len, x_lo, x_hi, v_lo, v_hi, I);
        int total;
        const int off = gscan(I.n, r, &total);
#pragma unroll
        for (int q = 0; q < NN; ++q)
            if (q < I.n && nint + off + q < NN) {
                S.lo[nint + off + q] = I.lo[q];
                S.hi[nint + off + q] = I.hi[q];
            }
        nint = min(nint + total, NN);
    }
    __syncthreads();

    // one lane per root: refinement on the unscaled monic polynomial
    if (ok && r < nint) *root = refine_root<NN>(c, sigma * S.lo[r], sigma * S.hi[r]);
    return ok ? nint : 0;
}

} // namespace
} // namespace mp
