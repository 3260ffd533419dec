// Deflation + balance + Hessenberg form of the shared-focal root stage on 16-lane
// groups (four samples per 64-lane wave), everything in registers, cross-lane traffic
// on DPP broadcasts / reductions and ds_bpermute gathers.  The same construction as
// pt_defl6_kernel (eig6.h: the companion C = [0 I; -M0^-1 M2  -M0^-1 M1], the basis
// Z of its structural zero-eigenvalue subspace, the Householder reflectors of Z applied
// as an orthogonal similarity, then balance + elmhes of the trailing 15 x 15 block),
// arranged so that a sample's work is spread over its 16 lanes instead of a whole wave:
//
//   Gauss-Jordan (complete pivoting): lane r holds row r; the pivot is the group's
//     first maximum in row-major order (DPP arg-max), the pivot row reaches every lane
//     by ds_bpermute, each lane updates its own row;
//   null spaces: lane i forms component i of each null vector, gathering the entry of
//     the row pivoted in column i;
//   the similarity: lane i holds rows i and i + 10 of the 20 x 20 companion; column
//     dot products are group sums (DPP), row dot products lane-local against the
//     reflector broadcast from its lanes;
//   balance / elmhes: lane i holds row i of the block; column sums are group sums, row
//     swaps ds_bpermute, column swaps register selects.
//
// The arithmetic is not the one-wave kernel's operation for operation (reduction
// orders, reciprocal-scaled pivot rows, elmhes as one similarity per column as there),
// so the Hessenberg matrices agree with it to rounding, and the roots to the accuracy
// the parity tests check (oracle, 60-digit fixture).  Output as pt_defl6_kernel's with
// hess = true: the 15 x 15 Hessenberg block row-major in pen[0, 225), pen[225] = 1
// (0: M0 singular, no roots).
#pragma once
#include "eig6.h"

namespace mp {
namespace {

// Phase timing for tools/eig6_bench.hip (compiled out otherwise): wall-clock ticks of
// the kernel's phases, summed over waves (lane 0)
#ifdef MP_EIG6_PROFILE
__device__ unsigned long long e6g_prof[10];
#define E6G_MARK(i)                                                                                                    \
    do {                                                                                                               \
        const unsigned long long t_ = wall_clock64();                                                                 \
        if (threadIdx.x == 0) atomicAdd(&e6g_prof[i], t_ - t_prev);                                                    \
        t_prev = t_;                                                                                                   \
    } while (0)
#define E6G_START unsigned long long t_prev = wall_clock64()
#else
#define E6G_MARK(i) ((void)0)
#define E6G_START ((void)0)
#endif

// value of v at lane `src` (0..15) of the caller's group (src group-uniform)
__device__ inline double e6g_at(double v, int src) { return __shfl(v, (int)(threadIdx.x & ~15u) + src, 64); }


// all-reduce sum over the 16-lane group (identical in every lane: each step adds a
// pair of partial sums, and IEEE addition commutes)
__device__ inline double e6g_sum(double v) {
    v += dpp_d<dpp::kXor1>(v);
    v += dpp_d<dpp::kXor2>(v);
    v += dpp_d<dpp::kHalfMirror>(v);
    return v + dpp_d<dpp::kMirror>(v);
}

// One Gauss-Jordan step with complete pivoting over the first NP columns of the
// group's n x NC matrix (lane r < n holds row r in g).  rows / cols: pivoted sets
// (group-uniform); myrow: in lane c, the row pivoted in column c.  false: zero pivot.
template <int NC, int NP>
__device__ __forceinline__ bool e6g_gj_step(double (&g)[NC], int n, unsigned &rows, unsigned &cols, int &myrow) {
    const int r = threadIdx.x & 15;
    double best = -1.0;
    int bkey = 0x7fffffff;
    if (r < n && !((rows >> r) & 1u)) {
        static_for<NP>([&](auto c) {
            if (!((cols >> c) & 1u)) {
                const double a = fabs(g[c]);
                if (a > best) {
                    best = a;
                    bkey = r * NP + c;
                }
            }
        });
    }
    double vmax;
    int kmin;
    gargmax(best, bkey, &vmax, &kmin);
    if (!(vmax > 0.0)) return false; // (group-uniform)
    const int pr = kmin / NP, pc = kmin - (kmin / NP) * NP;
    double prow[NC];
    static_for<NC>([&](auto c) { prow[c] = e6g_at(g[c], pr); });
    double piv = 0.0, mul = 0.0;
    static_for<NP>([&](auto c) {
        piv = (c == pc) ? prow[c] : piv;
        mul = (c == pc) ? g[c] : mul;
    });
    const double ip = e6_rcp(piv);
    static_for<NC>([&](auto c) {
        const double nv = prow[c] * ip;
        g[c] = (r == pr) ? nv : fma(-mul, nv, g[c]);
    });
    rows |= 1u << pr;
    cols |= 1u << pc;
    if (r == pc) myrow = pr;
    return true;
}

// Component i (lane i < n) of the right null vectors after a rank-`rank` Gauss-Jordan
// of an n x NC matrix (NP = n pivot columns): for the f-th free column fc (ascending),
// x_fc = 1 and x_c = -G(row pivoted in c, fc) on the pivot columns.
template <int NC, int NP, int NF>
__device__ __forceinline__ void e6g_null(const double (&g)[NC], unsigned cols, int myrow, double (&x)[NF]) {
    const int i = threadIdx.x & 15;
    int fc = -1;
    static_for<NF>([&](auto f) {
        // the next free column
        int c = fc + 1;
        while (c < NP && ((cols >> c) & 1u)) ++c;
        fc = c;
        double gf = 0.0;
        static_for<NP>([&](auto q) { gf = (q == fc) ? g[q] : gf; });
        const double piv_entry = e6g_at(gf, myrow < 0 ? 0 : myrow);
        x[f] = (i == fc) ? 1.0 : (i < NP && ((cols >> i) & 1u)) ? -piv_entry : 0.0;
    });
}

__global__ void __launch_bounds__(64) pt_defl6_grp_kernel(double *pen, int nlist, BatchGate gate) {
    if (batch_cancelled(gate.word, gate.hi)) return;
    E6G_START;
    const int i = threadIdx.x & 15;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 4);
    const bool valid = idx < nlist;
    double *P = pen + (size_t)(valid ? idx : nlist - 1) * kPenStride;
    const double *M1 = P + 100, *M2 = P + 200;
    const bool lr = i < 10; // lanes holding a pencil row
    // ---- C = [0 I; -M0^-1 [M2 M1]]: Gauss-Jordan of [M0 | M2 | M1] ----
    double CB[20]; // row 10 + i of C (row i is e_{10+i} until the similarity)
    bool ok = true;
    {
        double g[30];
        static_for<10>([&](auto c) {
            g[c] = lr ? P[10 * i + c] : 0.0;
            g[10 + c] = lr ? M2[10 * i + c] : 0.0;
            g[20 + c] = lr ? M1[10 * i + c] : 0.0;
        });
        unsigned rows = 0, cols = 0;
        int myrow = -1;
        for (int k = 0; k < 10 && ok; ++k) ok = e6g_gj_step<30, 10>(g, 10, rows, cols, myrow);
        // row i of M0^-1 [M2 M1] is the row pivoted in column i
        static_for<20>([&](auto j) { CB[j] = -e6g_at(g[10 + j], myrow < 0 ? 0 : myrow); });
    }
    E6G_MARK(0);
    if (!ok) { // M0 singular: no roots (group-uniform)
        if (valid && i == 0) P[225] = 0.0;
        return;
    }
    // ---- the zero-eigenvalue invariant subspace ----
    double nl[4], nr[4];
    {
        double g[10];
        unsigned rows = 0, cols = 0;
        int myrow = -1;
        // left null space of M2: Gauss-Jordan of M2^T (rank 6)
        static_for<10>([&](auto c) { g[c] = lr ? M2[10 * c + i] : 0.0; });
        for (int k = 0; k < 6; ++k) e6g_gj_step<10, 10>(g, 10, rows, cols, myrow);
        e6g_null<10, 10, 4>(g, cols, myrow, nl);
        // right null space of M2
        rows = cols = 0;
        myrow = -1;
        static_for<10>([&](auto c) { g[c] = lr ? M2[10 * i + c] : 0.0; });
        for (int k = 0; k < 6; ++k) e6g_gj_step<10, 10>(g, 10, rows, cols, myrow);
        e6g_null<10, 10, 4>(g, cols, myrow, nr);
    }
    E6G_MARK(1);
    // S = Nl^T M1 Nr (4 x 4, rank 3): lane c forms column c of T = Nl^T M1
    double S[4][4];
    {
        double tc[4] = {0.0, 0.0, 0.0, 0.0};
        static_for<10>([&](auto k) {
            const double m1 = lr ? M1[10 * k + i] : 0.0;
            static_for<4>([&](auto a) { tc[a] = fma(gbcast<decltype(k)::value>(nl[a]), m1, tc[a]); });
        });
        static_for<4>([&](auto a) {
            static_for<4>([&](auto b) { S[a][b] = e6g_sum(lr ? tc[a] * nr[b] : 0.0); });
        });
    }
    // its null vector: Gauss-Jordan with complete pivoting, 3 steps (every lane alike)
    double cv[4];
    {
        unsigned rows = 0, cols = 0;
        int prow[3] = {0, 0, 0}, pcol[3] = {0, 0, 0};
        static_for<3>([&](auto k) {
            double best = -1.0;
            int br = 0, bc = 0;
            static_for<4>([&](auto r) {
                static_for<4>([&](auto c) {
                    const double a = fabs(opaque(S[r][c]));
                    if (!((rows >> r) & 1u) && !((cols >> c) & 1u) && a > best) {
                        best = a;
                        br = r;
                        bc = c;
                    }
                });
            });
            double prw[4], mulc[4];
            static_for<4>([&](auto c) {
                prw[c] = 0.0;
                static_for<4>([&](auto r) { prw[c] = (r == br) ? opaque(S[r][c]) : prw[c]; });
            });
            static_for<4>([&](auto r) {
                mulc[r] = 0.0;
                static_for<4>([&](auto c) { mulc[r] = (c == bc) ? opaque(S[r][c]) : mulc[r]; });
            });
            double piv = 0.0;
            static_for<4>([&](auto c) { piv = (c == bc) ? prw[c] : piv; });
            const double ip = best > 0.0 ? e6_rcp(piv) : 0.0;
            static_for<4>([&](auto r) {
                static_for<4>([&](auto c) {
                    const double nv = prw[c] * ip;
                    S[r][c] = (r == br) ? nv : fma(-mulc[r], nv, S[r][c]);
                });
            });
            rows |= 1u << br;
            cols |= 1u << bc;
            prow[k] = br;
            pcol[k] = bc;
        });
        int fcol = 0;
        while (fcol < 3 && ((cols >> fcol) & 1u)) ++fcol;
        static_for<4>([&](auto c) {
            double x = (c == fcol) ? 1.0 : 0.0;
            static_for<3>([&](auto k) {
                double e = 0.0;
                static_for<4>([&](auto r) {
                    static_for<4>([&](auto q) { e = (r == prow[k] && q == fcol) ? opaque(S[r][q]) : e; });
                });
                x = (pcol[k] == c) ? -e : x;
            });
            cv[c] = x;
        });
    }
    E6G_MARK(2);
    // v = Nr c (component i), rhs = -M1 v
    const double v = lr ? fma(nr[3], cv[3], fma(nr[2], cv[2], fma(nr[1], cv[1], nr[0] * cv[0]))) : 0.0;
    double rhs = 0.0;
    static_for<10>([&](auto c) {
        const double vc = gbcast<decltype(c)::value>(v);
        rhs = fma(lr ? M1[10 * i + c] : 0.0, vc, rhs);
    });
    rhs = -rhs;
    // a particular solution of M2 a = rhs: Gauss-Jordan of [M2 | rhs], 6 pivots
    double pa;
    {
        double g[11];
        static_for<10>([&](auto c) { g[c] = lr ? M2[10 * i + c] : 0.0; });
        g[10] = lr ? rhs : 0.0;
        unsigned rows = 0, cols = 0;
        int myrow = -1;
        for (int k = 0; k < 6; ++k) e6g_gj_step<11, 10>(g, 10, rows, cols, myrow);
        const double gr = e6g_at(g[10], myrow < 0 ? 0 : myrow);
        pa = (lr && ((cols >> i) & 1u)) ? gr : 0.0;
    }
    E6G_MARK(3);
    // ---- C <- Q^T C Q, Q = H_0 ... H_4 the Householder reflectors of Z = [Nr a; 0 v] ----
    double CA[20];
    static_for<20>([&](auto j) { CA[j] = (lr && j == 10 + i) ? 1.0 : 0.0; });
    if (!lr) static_for<20>([&](auto j) { CB[j] = 0.0; });
    double ZA[5] = {lr ? nr[0] : 0.0, lr ? nr[1] : 0.0, lr ? nr[2] : 0.0, lr ? nr[3] : 0.0, lr ? pa : 0.0};
    double ZB[5] = {0.0, 0.0, 0.0, 0.0, lr ? v : 0.0};
    static_for<5>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        const double zA = (lr && i >= k) ? ZA[k] : 0.0, zB = ZB[k];
        double alpha = sqrt(e6g_sum(fma(zB, zB, zA * zA)));
        if (alpha == 0.0) return; // (uniform)
        if (gbcast<k>(ZA[k]) > 0.0) alpha = -alpha;
        const double hA = zA - (i == k ? alpha : 0.0), hB = zB;
        const double vn = e6g_sum(fma(hB, hB, hA * hA));
        if (!(vn > 0.0)) return; // (uniform)
        const double sc = 2.0 * e6_rcp(vn);
        static_for<5>([&](auto j) {
            if constexpr (decltype(j)::value > k) {
                const double d = sc * e6g_sum(fma(hB, ZB[j], hA * ZA[j]));
                ZA[j] = fma(-d, hA, ZA[j]);
                ZB[j] = fma(-d, hB, ZB[j]);
            }
        });
        // C <- H C (column by column: group sums)
        static_for<20>([&](auto j) {
            const double d = sc * e6g_sum(fma(hB, CB[j], hA * CA[j]));
            CA[j] = fma(-d, hA, CA[j]);
            CB[j] = fma(-d, hB, CB[j]);
        });
        // C <- C H (row by row: the reflector from its lanes)
        double hv[20];
        static_for<10>([&](auto j) {
            hv[j] = gbcast<decltype(j)::value>(hA);
            hv[10 + j] = gbcast<decltype(j)::value>(hB);
        });
        double dA = 0.0, dB = 0.0;
        static_for<20>([&](auto j) {
            dA = fma(CA[j], hv[j], dA);
            dB = fma(CB[j], hv[j], dB);
        });
        dA *= sc;
        dB *= sc;
        static_for<20>([&](auto j) {
            CA[j] = fma(-dA, hv[j], CA[j]);
            CB[j] = fma(-dB, hv[j], CB[j]);
        });
    });
    E6G_MARK(4);
    // ---- the trailing 15 x 15 block, lane i' = row 5 + i' ----
    constexpr int N = 15;
    double h[N];
    {
        const int src = i < 5 ? 5 + i : (i < 15 ? i - 5 : 0);
        static_for<N>([&](auto j) {
            const double a = e6g_at(CA[5 + j], src), b = e6g_at(CB[5 + j], src);
            h[j] = i < 5 ? a : (i < 15 ? b : 0.0);
        });
    }
    E6G_MARK(5);
    // ---- balance (EISPACK balanc without permutations) ----
    {
        const double radix = 2.0, sqrdx = 4.0;
        bool done = false;
        for (int pass = 0; !done && pass < 64; ++pass) {
            done = true;
            static_for<N>([&](auto qq) {
                constexpr int q = decltype(qq)::value;
                double c = e6g_sum((i < N && i != q) ? fabs(h[q]) : 0.0);
                double rs = 0.0;
                static_for<N>([&](auto j) {
                    if (j != q) rs += fabs(h[j]);
                });
                const double r = gbcast<q>(rs);
                if (c != 0.0 && r != 0.0) {
                    // (fi = 1 / f exactly -- f is a power of two -- so (c + r) * fi is the
                    // quotient (c + r) / f to the bit, without a division)
                    double g = r / radix, f = 1.0, fi = 1.0;
                    const double s = c + r;
                    while (c < g) {
                        f *= radix;
                        fi *= 1.0 / radix;
                        c *= sqrdx;
                    }
                    g = r * radix;
                    while (c > g) {
                        f /= radix;
                        fi *= radix;
                        c /= sqrdx;
                    }
                    if ((c + r) * fi < 0.95 * s) {
                        done = false;
                        g = fi;
                        if (i == q) static_for<N>([&](auto j) { h[j] *= g; });
                        h[q] *= f;
                    }
                }
            });
        }
    }
    E6G_MARK(6);
    // ---- elmhes: the eliminations of one column as one similarity ----
    static_for<N - 2>([&](auto mm) {
        constexpr int m = decltype(mm)::value + 1;
        double vmax;
        int ip;
        gargmax((i >= m && i < N) ? fabs(h[m - 1]) : -1.0, i, &vmax, &ip);
        if (!(vmax > 0.0)) return; // x == 0 (uniform)
        if (ip != m) {
            const int src = (i == m) ? ip : (i == ip ? m : i);
            static_for<N>([&](auto j) { h[j] = e6g_at(h[j], src); });
            double t = 0.0;
            static_for<N>([&](auto j) { t = (j == ip) ? h[j] : t; });
            static_for<N>([&](auto j) {
                if (j == ip) h[j] = h[m];
            });
            h[m] = t;
        }
        const double x = gbcast<m>(h[m - 1]);
        const double ix = e6_rcp(x);
        double y = 0.0;
        if (i > m && i < N) {
            y = h[m - 1] * ix;
            h[m - 1] = y;
        }
        static_for<N>([&](auto j) {
            if constexpr (decltype(j)::value >= m) {
                const double hm = gbcast<m>(h[j]);
                if (i > m && i < N) h[j] = fma(-y, hm, h[j]);
            }
        });
        double acc = h[m];
        static_for<N>([&](auto q) {
            if constexpr (decltype(q)::value > m) acc = fma(gbcast<decltype(q)::value>(y), h[q], acc);
        });
        h[m] = acc;
    });
    E6G_MARK(7);
    static_for<N>([&](auto j) {
        if (j < i - 1) h[j] = 0.0;
    });
    if (!valid) return;
    if (i < N) static_for<N>([&](auto j) { P[N * i + j] = h[j]; });
    if (i == 0) P[225] = 1.0;
}

} // namespace
} // namespace mp
