// A/B kernels of the shared-focal root stage, kept for tools/eig6_bench.hip only (not
// built into the library; VERDICT r03 hygiene): the one-sample-per-wave deflation
// (pt_defl6_kernel) and hqr (pt_eig6_kernel), the LDS lane QR (pt_eig6_lane_kernel),
// the 16-lane group QR (pt_eig6_grp_kernel, bit-identical to the default lane QR and no
// faster) and -- in group_6pt.h -- the 16-point DFT + Sturm root stage
// that lost roots.  Include after madpose_amd/csrc/kernels/kernels.hip.
#pragma once

namespace mp {
namespace {

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

__device__ inline int e6g_max(int v) {
    v = max(v, dpp_i<dpp::kXor1>(v));
    v = max(v, dpp_i<dpp::kXor2>(v));
    v = max(v, dpp_i<dpp::kHalfMirror>(v));
    return max(v, dpp_i<dpp::kMirror>(v));
}
// value of v at lane `src` (0..15) of the caller's group (src group-uniform)

__global__ void __launch_bounds__(64) pt_eig6_grp_kernel(const double *pen, int nlist, double *cand, int *ncand,
                                                         int cand_stride) {
#pragma clang fp contract(off)
    constexpr int N = 15;
    const int i = threadIdx.x & 15;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 4);
    const bool valid = idx < nlist;
    const double *P = pen + (size_t)(valid ? idx : nlist - 1) * kPenStride;
    const bool active = valid && P[225] != 0.0; // (group-uniform)
    double a[N];
    static_for<N>([&](auto j) { a[j] = (active && i < N && j >= i - 1) ? P[i * N + j] : 0.0; });
    // anorm: row sums (sequential within a row), then the rows in order
    double anorm = 0.0;
    {
        double rs = 0.0;
        static_for<N>([&](auto j) {
            if (j >= i - 1) rs += fabs(a[j]);
        });
        static_for<N>([&](auto r) { anorm += gbcast<decltype(r)::value>(rs); });
    }
    int nn = N - 1, its = 0;
    double t = 0.0;
    bool done = !active, failed = false;
    double ewr = 0.0, ewi = 0.0; // eigenvalue number i
    // this lane's diagonal H(i,i), subdiagonal H(i,i-1), superdiagonal H(i,i+1)
    auto diag = [&](double &d, double &sub, double &sup) {
        d = 0.0;
        sub = 0.0;
        sup = 0.0;
        static_for<N>([&](auto j) {
            d = (j == i) ? a[j] : d;
            sub = (j == i - 1) ? a[j] : sub;
            sup = (j == i + 1) ? a[j] : sup;
        });
    };
#pragma unroll 1
    for (int round = 0; round < 600 && !__all(done); ++round) {
        int l = 0;
        double x = 0.0, y = 0.0, w = 0.0;
        bool sweep = false;
        double d, sub, sup;
#pragma unroll 1
        for (int rep = 0; rep < 3; ++rep) {
            diag(d, sub, sup);
            // l: the largest q <= nn with a negligible H(q, q-1) (0 if none)
            {
                double s = fabs(dpp_d<dpp::shr(1)>(d)) + fabs(d);
                if (s == 0.0) s = anorm;
                const bool neg = i >= 1 && i <= nn && fabs(sub) + s == s;
                l = e6g_max(neg ? i : 0);
            }
            if (!done && l >= 1) {
                static_for<N>([&](auto j) {
                    if (j == i - 1 && i == l) a[j] = 0.0;
                });
                if (i == l) sub = 0.0;
            }
            x = y = w = 0.0;
            if (nn >= 0) x = e6g_at(d, nn < 0 ? 0 : nn);
            if (nn >= 1) {
                y = e6g_at(d, nn - 1);
                w = e6g_at(sub, nn) * e6g_at(sup, nn - 1);
            }
            sweep = false;
            if (!done) {
                if (l == nn) {
                    if (i == nn) {
                        ewr = x + t;
                        ewi = 0.0;
                    }
                    nn -= 1;
                    its = 0;
                } else if (l == nn - 1) {
                    const double p = 0.5 * (y - x), q = fma(p, p, w);
                    double z = sqrt(fabs(q));
                    const double xx = x + t;
                    if (q >= 0.0) {
                        z = p + e6_sign(z, p);
                        const double w0 = xx + z;
                        const double w1 = (z != 0.0) ? xx - w / z : w0;
                        if (i == nn - 1) ewr = w0;
                        if (i == nn) ewr = w1;
                        if (i == nn - 1 || i == nn) ewi = 0.0;
                    } else {
                        if (i == nn - 1 || i == nn) ewr = xx + p;
                        if (i == nn) ewi = z;
                        if (i == nn - 1) ewi = -z;
                    }
                    nn -= 2;
                    its = 0;
                } else if (its == 60) {
                    failed = true;
                    done = true;
                } else {
                    sweep = true;
                }
                if (nn < 0) done = true;
            }
            if (__all(done || sweep)) break;
        }
        if (!__any(sweep)) continue;
        // the union of the sweeping groups' windows (wave-uniform step range)
        int lo = sweep ? l : N, hi = sweep ? nn : 0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            lo = min(lo, __shfl_xor(lo, off, 64));
            hi = max(hi, __shfl_xor(hi, off, 64));
        }
        lo = __builtin_amdgcn_readfirstlane(lo);
        hi = __builtin_amdgcn_readfirstlane(hi);
        if (sweep && (its == 10 || its == 20 || its == 40)) { // exceptional shift
            t += x;
            static_for<N>([&](auto j) {
                if (j == i && i <= nn) a[j] -= x;
            });
            const double s = fabs(e6g_at(sub, nn)) + fabs(e6g_at(sub, nn - 1));
            y = x = 0.75 * s;
            w = -0.4375 * s * s;
            diag(d, sub, sup);
        }
        if (sweep) ++its;
        // the first reflector, at l
        double p0 = 0.0, q0 = 0.0, r0 = 0.0;
        {
            const int c = sweep ? l : 0;
            const double z = e6g_at(d, c), h10 = e6g_at(sub, c + 1), h01 = e6g_at(sup, c), h11 = e6g_at(d, c + 1),
                         h21 = e6g_at(sub, c + 2 < N ? c + 2 : N - 1);
            if (sweep) {
                const double rr = x - z, ss = y - z;
                p0 = fma(rr, ss, -w) / h10 + h01;
                q0 = h11 - z - rr - ss;
                r0 = h21;
            }
            const double sc = fabs(p0) + fabs(q0) + fabs(r0);
            if (sc != 0.0) {
                p0 /= sc;
                q0 /= sc;
                r0 /= sc;
            }
        }
        static_for<N - 1>([&](auto kk) {
            constexpr int k = decltype(kk)::value;
            if (k >= lo && k < hi) { // (uniform)
                const bool on = sweep && k >= l && k <= nn - 1;
                const bool last = k == nn - 1;
                double p = p0, q = q0, r = r0, xk = 0.0;
                if constexpr (k > 0) {
                    const double bp = gbcast<k>(a[k - 1]), bq = gbcast<k + 1>(a[k - 1]);
                    double br = 0.0;
                    if constexpr (k + 2 < N) br = gbcast<k + 2>(a[k - 1]);
                    if (k > l) {
                        p = bp;
                        q = bq;
                        r = last ? 0.0 : br;
                        xk = fabs(p) + fabs(q) + fabs(r);
                        if (xk != 0.0) {
                            const double ixk = 1.0 / xk;
                            p *= ixk;
                            q *= ixk;
                            r *= ixk;
                        }
                    }
                    // the bulge entries of column k-1 (consumed by this step; zero otherwise)
                    if (i == k + 1 || (k + 2 < N && i == k + 2)) a[k - 1] = 0.0;
                }
                if (last) r = 0.0;
                const double s = e6_sign(sqrt(fma(r, r, fma(q, q, p * p))), p);
                double cx = 0.0, cy = 0.0, cz = 0.0, cq = 0.0, cr = 0.0;
                if (on && s != 0.0) {
                    if constexpr (k > 0) {
                        if (k > l && i == k) a[k - 1] = -s * xk;
                    }
                    const double pp = p + s, is = 1.0 / s, ip = 1.0 / pp;
                    cx = pp * is;
                    cy = q * is;
                    cz = r * is;
                    cq = q * ip;
                    cr = r * ip;
                }
                // rows k..k+2, columns k..nn: the three rows from their lanes
                const double coef = (i == k) ? cx : (i == k + 1) ? cy : (k + 2 < N && i == k + 2) ? cz : 0.0;
                static_for<N - k>([&](auto jj) {
                    constexpr int j = k + decltype(jj)::value;
                    const double r0v = gbcast<k>(a[j]), r1v = gbcast<k + 1>(a[j]);
                    double pj;
                    if constexpr (k + 2 < N)
                        pj = fma(cr, gbcast<k + 2>(a[j]), fma(cq, r1v, r0v));
                    else
                        pj = fma(cq, r1v, r0v);
                    if (on && j <= nn && i >= k && i <= k + 2) a[j] = fma(-pj, coef, a[j]);
                });
                // columns k..k+2, rows l..min(nn, k+3): lane-local
                const int mmin = nn < k + 3 ? nn : k + 3;
                if (on && i >= l && i <= mmin) {
                    double pi;
                    if constexpr (k + 2 < N) {
                        pi = fma(cz, a[k + 2], fma(cy, a[k + 1], cx * a[k]));
                        a[k + 2] = fma(-pi, cr, a[k + 2]);
                    } else {
                        pi = fma(cy, a[k + 1], cx * a[k]);
                    }
                    a[k + 1] = fma(-pi, cq, a[k + 1]);
                    a[k] -= pi;
                }
            }
        });
        // Hessenberg again below the windows
        static_for<N>([&](auto j) {
            if (j == i - 2 || j == i - 3) a[j] = 0.0;
        });
    }
    const bool conv = active && done && !failed;
    // positive real eigenvalues, ascending (ties in index order), into cand[27 ..)
    const bool mine = conv && i < N && ewi == 0.0 && ewr > 0.0;
    int rank = 0, cnt = 0;
    static_for<N>([&](auto j) {
        const double uj = gbcast<decltype(j)::value>(ewr);
        const int vj = gbcast<decltype(j)::value>(mine ? 1 : 0);
        cnt += vj;
        rank += (vj && (uj < ewr || (uj == ewr && j < i))) ? 1 : 0;
    });
    if (!valid) return;
    if (mine) cand[(size_t)idx * cand_stride + 27 + rank] = ewr;
    if (i == 0) ncand[idx] = cnt;
}


} // namespace
} // namespace mp
