// PoseLib's Sturm bisection (misc/sturm.h bisect_sturm<N>, the root finder of PoseLib
// relpose_5pt, called at src/hybrid_pose_estimator.cpp:134) over one 16-lane group,
// with the arithmetic of the oracle's restatement (oracle/src/pt_poselib.cpp) to the bit.
//
// PoseLib recurses depth-first: an interval (a, b] whose Sturm counts differ by more
// than one is halved at c = (a + b) / 2, an interval holding one root goes to Ridders'
// method + Newton, intervals deeper than 300 halvings are dropped.  Every node of that
// recursion depends only on its parent, so the group walks the same tree breadth-first:
// one level per round, lane j halving the j-th pending interval of the level (one
// sign-change count each), the children appended by group prefix sums.  The leaves
// (one root each) come out in another order than the depth-first one, so they are
// ranked by position afterwards -- the disjoint leaves of the tree, ordered left to
// right, ARE the depth-first order -- and lane k refines the k-th leaf.  Each value is
// computed by one lane with the expressions of the oracle, without FMA contraction
// (the chain, every count, Ridders' and Newton's iterates), so the roots are the
// oracle's in value and order.
//
// Capacity (the oracle applies the same rule): at most kGrp pending intervals per level
// and kGrp leaves, otherwise the sample has no roots.  With Sturm counts that do not
// increase along the line -- the case in floating point except at rounding accidents --
// a degree-N polynomial has at most N / 2 pending intervals and N leaves.  The first N
// roots found are kept (PoseLib's roots[N]).
// Every lane of the workgroup must call group_bisect_sturm (it holds barriers).
#pragma once
#include "group_sturm.h"

namespace mp {
namespace {

constexpr int kBisectMaxDepth = 300;

template <int N> struct GroupBisect {
    double fvec[2 * N + 1];        // monic polynomial and monic derivative / N
    double svec[3 * N];            // the Sturm chain's quotients (build_sturm_seq)
    double a[2][kGrp], b[2][kGrp]; // pending intervals of the level (double-buffered)
    int sa[2][kGrp], sb[2][kGrp];
    int npend[2];
    double la[kGrp], lb[kGrp];     // leaves, in discovery order
    int nleaf;
    int overflow;
};

// PoseLib build_sturm_seq<N> on fvec = [monic f (N + 1) | monic f' / N (N)]: the
// quotients and normalisers of the chain (svec: 3 N doubles).  Compile-time indices
// only; the three rotating buffers of PoseLib's pointer juggling are selected
// statically.
template <int N>
__device__ inline void bisect_build_chain(const double (&fvec)[2 * N + 1], double (&svec)[3 * N], bool writer) {
#pragma clang fp contract(off)
    double f[3][N + 1];
    static_for<N + 1>([&](auto j) {
        f[0][j] = fvec[j];
        f[1][j] = (j < N) ? fvec[N + 1 + (j < N ? (int)j : 0)] : 0.0;
        f[2][j] = 0.0;
    });
    static_for<N - 1>([&](auto I) {
        constexpr int i = decltype(I)::value;
        constexpr int i1 = i % 3, i2 = (i + 1) % 3, i3 = (i + 2) % 3;
        const double q1 = f[i1][N - i] * f[i2][N - 1 - i];
        const double q0 = f[i1][N - 1 - i] * f[i2][N - 1 - i] - f[i1][N - i] * f[i2][N - 2 - i];
        f[i3][0] = f[i1][0] - q0 * f[i2][0];
        static_for<N - 2 - i>([&](auto Jm1) {
            constexpr int j = decltype(Jm1)::value + 1;
            f[i3][j] = f[i1][j] - q1 * f[i2][j - 1] - q0 * f[i2][j];
        });
        const double c = -fabs(f[i3][N - 2 - i]);
        const double ci = 1.0 / c;
        static_for<N - 1 - i>([&](auto j) { f[i3][j] = f[i3][j] * ci; });
        if (writer) {
            svec[3 * i] = q0;
            svec[3 * i + 1] = q1;
            svec[3 * i + 2] = c;
        }
    });
    constexpr int e1 = (N - 1) % 3, e2 = N % 3; // f1, f2 after N - 1 rotations
    if (writer) {
        svec[3 * N - 3] = f[e1][0];
        svec[3 * N - 2] = f[e1][1];
        svec[3 * N - 1] = f[e2][0];
    }
}

template <int N> __device__ inline double bisect_polyval(const double *f, double x) {
#pragma clang fp contract(off)
    double fx = x + f[N - 1];
#pragma unroll
    for (int i = N - 2; i >= 0; --i) fx = x * fx + f[i];
    return fx;
}

template <int N> __device__ inline int bisect_signchanges(const double (&svec)[3 * N], double x) {
#pragma clang fp contract(off)
    double f[N + 1];
    f[N] = svec[3 * N - 1];
    f[N - 1] = svec[3 * N - 3] + x * svec[3 * N - 2];
#pragma unroll
    for (int i = N - 2; i >= 0; --i) f[i] = (svec[3 * i] + x * svec[3 * i + 1]) * f[i + 1] + svec[3 * i + 2] * f[i + 2];
    unsigned S = 0;
#pragma unroll
    for (int k = 0; k <= N; ++k) {
        const unsigned nk = f[k] < 0 ? 1u : 0u;
        const unsigned nk1 = (k < N) ? (f[k < N ? k + 1 : N] < 0 ? 1u : 0u) : 0u;
        S |= (nk ^ nk1) << k;
    }
    return __popc(S);
}

// PoseLib ridders_method_newton<N> (tol 1e-10); *x the root when it returns true
template <int N>
__device__ inline bool bisect_ridders_newton(const double (&fvec)[2 * N + 1], double a, double b, double *root) {
#pragma clang fp contract(off)
    double fa = bisect_polyval<N>(fvec, a);
    double fb = bisect_polyval<N>(fvec, b);
    if (!((fa < 0) ^ (fb < 0))) return false;
    const double tol = 1e-10, tol_newton = 1e-3;
    for (int iter = 0; iter < 30; ++iter) {
        if (fabs(a - b) < tol_newton) break;
        const double c = (a + b) * 0.5;
        const double fc = bisect_polyval<N>(fvec, c);
        const double s = sqrt(fc * fc - fa * fb);
        if (!s) break;
        const double d = (fa < fb) ? c + (a - c) * fc / s : c + (c - a) * fc / s;
        const double fd = bisect_polyval<N>(fvec, d);
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
    for (int iter = 0; iter < 10; ++iter) {
        const double fx = bisect_polyval<N>(fvec, x);
        if (fabs(fx) < tol) break;
        const double fpx = static_cast<double>(N) * bisect_polyval<N - 1>(fvec + N + 1, x);
        const double dx = fx / fpx;
        x = x - dx;
        if (fabs(dx) < tol) break;
    }
    *root = x;
    return true;
}

// Real roots of sum_i p[i] x^i (ascending, degree N, held by every lane of the group)
// as bisect_sturm<N>.  Returns whether lane r holds a kept root (in *root); the kept
// roots ascend with the lane index (lanes without one can sit between them).  !ok (a
// failed elimination upstream): no roots.
template <int N>
__device__ bool group_bisect_sturm(const double (&p)[N + 1], int r, GroupBisect<N> &S, bool ok, double *root) {
#pragma clang fp contract(off)
    static_assert(N <= kGrp, "one leaf per lane");
    ok = ok && p[N] != 0.0;
    // the polynomial and the chain are the same in every lane of the group: computed
    // redundantly, kept in LDS (written by lane 0) -- in registers they held the kernel
    // at 186 VGPRs, two waves per SIMD
    double fvec[2 * N + 1];
    {
        static_for<N + 1>([&](auto i) { fvec[i] = p[i]; });
        const double c_inv = 1.0 / fvec[N];
        static_for<N>([&](auto i) { fvec[i] *= c_inv; });
        fvec[N] = 1.0;
        static_for<N - 1>([&](auto i) { fvec[N + 1 + i] = fvec[i + 1] * ((i + 1) / static_cast<double>(N)); });
        fvec[2 * N] = 1.0;
        // (the restatement's guard: a non-finite coefficient gives no roots)
        static_for<2 * N + 1>([&](auto i) { ok = ok && isfinite(fvec[i]); });
    }
    double r_max = 0.0;
    static_for<N>([&](auto i) { r_max = fmax(r_max, fabs(fvec[i])); });
    r_max = 1.0 + r_max;
    // (std::max(mx, |f_i|) keeps mx on a NaN |f_i|, fmax too: the same bound)
    if (r == 0) static_for<2 * N + 1>([&](auto i) { S.fvec[i] = fvec[i]; });
    bisect_build_chain<N>(fvec, S.svec, r == 0);
    __syncthreads();
    const double(&svec)[3 * N] = S.svec;
    const double a0 = -r_max, b0 = r_max;
    const int sa0 = bisect_signchanges<N>(svec, a0), sb0 = bisect_signchanges<N>(svec, b0);
    __syncthreads(); // (S.npend / S.nleaf below: written by lane 0)
    if (r == 0) {
        S.npend[0] = (ok && sa0 - sb0 > 1) ? 1 : 0;
        S.nleaf = (ok && sa0 - sb0 == 1) ? 1 : 0;
        S.overflow = 0;
        S.a[0][0] = a0;
        S.b[0][0] = b0;
        S.sa[0][0] = sa0;
        S.sb[0][0] = sb0;
        S.la[0] = a0;
        S.lb[0] = b0;
    }
    __syncthreads();
    // breadth-first over the depth-first tree of isolate_roots
    int cur = 0;
    for (int depth = 0; depth <= kBisectMaxDepth; ++depth) {
        const int np = S.npend[cur];
        if (np == 0 || S.overflow) break; // (group-uniform: LDS values behind a barrier)
        const bool mine = r < np;
        double a = 0, b = 0, c = 0;
        int sa = 0, sb = 0, sc = 0;
        if (mine) {
            a = S.a[cur][r];
            b = S.b[cur][r];
            sa = S.sa[cur][r];
            sb = S.sb[cur][r];
            c = (a + b) * 0.5;
            sc = bisect_signchanges<N>(svec, c);
        }
        // children at depth + 1 (dropped beyond the maximum depth)
        const bool keep = depth + 1 <= kBisectMaxDepth;
        const int nl = sa - sc, nr = sc - sb;
        const bool pl = mine && keep && nl > 1, pr = mine && keep && nr > 1;
        const bool ll = mine && keep && nl == 1, lr = mine && keep && nr == 1;
        int tot_p, tot_l;
        const int at_p = gscan((pl ? 1 : 0) + (pr ? 1 : 0), &tot_p);
        const int at_l = gscan((ll ? 1 : 0) + (lr ? 1 : 0), &tot_l);
        const int nxt = cur ^ 1, base_l = S.nleaf;
        __syncthreads();
        if (tot_p > kGrp || base_l + tot_l > kGrp) {
            if (r == 0) S.overflow = 1;
        } else {
            int k = at_p;
            if (pl) {
                S.a[nxt][k] = a;
                S.b[nxt][k] = c;
                S.sa[nxt][k] = sa;
                S.sb[nxt][k] = sc;
                ++k;
            }
            if (pr) {
                S.a[nxt][k] = c;
                S.b[nxt][k] = b;
                S.sa[nxt][k] = sc;
                S.sb[nxt][k] = sb;
            }
            int q = base_l + at_l;
            if (ll) {
                S.la[q] = a;
                S.lb[q] = c;
                ++q;
            }
            if (lr) {
                S.la[q] = c;
                S.lb[q] = b;
            }
            if (r == 0) {
                S.npend[nxt] = tot_p;
                S.nleaf = base_l + tot_l;
            }
        }
        __syncthreads();
        cur = nxt;
    }
    const int nleaf = S.overflow ? 0 : S.nleaf;
    // lane k refines the leaf of rank k (leaves are disjoint: rank by left end)
    bool found = false;
    double x = 0.0;
    {
        int rank = 0;
        double la = 0, lb = 0;
        if (r < nleaf) {
            la = S.la[r];
            lb = S.lb[r];
            for (int q = 0; q < nleaf; ++q) rank += S.la[q] < la ? 1 : 0;
        }
        __syncthreads();
        if (r < nleaf) {
            S.la[rank] = la; // (reuse: the leaves in rank order)
            S.lb[rank] = lb;
        }
        __syncthreads();
        if (r < nleaf) found = bisect_ridders_newton<N>(S.fvec, S.la[r], S.lb[r], &x);
    }
    int nf;
    const int before = gscan(found ? 1 : 0, &nf);
    (void)nf;
    *root = x;
    return found && before < N;
}

} // namespace
} // namespace mp
