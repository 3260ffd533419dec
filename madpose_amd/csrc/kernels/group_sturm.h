// Group-parallel building blocks of the point-solver root stages: one 16-lane group
// of a 64-lane workgroup per minimal sample (4 samples per workgroup).
//
//   gmax / gbcast / gscan   group reductions, broadcasts and prefix sums (DPP)
//   group_sturm_roots<NN>   sturm_real_roots<NN> (mp_math.h) spread over the group:
//     * the Sturm chain is built coefficient-parallel (lane j owns coefficient j of
//       every chain polynomial; the chain is kept in LDS),
//     * the sign-change counts at the 33 points of the isolation grid are split over
//       the lanes; cells with several roots are split 16 ways by the whole group
//       (one Sturm count per lane per round) instead of bisected by one lane,
//     * one lane per isolated root for the safeguarded Newton refinement.
//     The chain, grid and refinement are the expressions of the one-lane code; the
//     isolating intervals of multi-root cells differ (16-section instead of
//     bisection), so roots agree with it to the refinement tolerance.
// Every lane of the workgroup must call group_sturm_roots (it holds barriers).
#pragma once
#include "../include/mp_math.h"
#include "kernels.h"

namespace mp {
namespace {

constexpr int kGrp = 16;              // lanes per sample
constexpr int kGrpPerWg = 64 / kGrp;  // samples per 64-lane workgroup
constexpr int kGridCells = 32;        // isolation grid of sturm_real_roots

// Group primitives on DPP (data-parallel primitives: cross-lane moves inside a row of
// 16 lanes, i.e. inside one group, at VALU latency instead of the ~100-cycle LDS
// crossbar of ds_bpermute that __shfl compiles to).  Control codes (gfx9 DPP):
// quad_perm, row_shr:n = 0x110 + n (lane i reads i - n), row_ror:n = 0x120 + n
// (lane i reads (i - n) mod 16), row_mirror 0x140 (i <-> 15 - i), row_half_mirror
// 0x141 (i <-> 7 - i within each half), row_newbcast:n = 0x150 + n (gfx90a+: every
// lane reads lane n of its row).
namespace dpp {
constexpr int kXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kHalfMirror = 0x141;
constexpr int kMirror = 0x140;
constexpr int shr(int n) { return 0x110 + n; }
constexpr int ror(int n) { return 0x120 + n; }
constexpr int bcast(int n) { return 0x150 + n; }
} // namespace dpp

// lanes whose source is outside the row read 0
template <int CTRL> __device__ inline int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true); }
template <int CTRL> __device__ inline double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)dpp_i<CTRL>((int)(b & 0xffffffffLL)), hi = (unsigned)dpp_i<CTRL>((int)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// all-reduce over the group (quad butterflies, then the half and full mirrors)
__device__ inline double gmax(double v) {
    v = fmax(v, dpp_d<dpp::kXor1>(v));
    v = fmax(v, dpp_d<dpp::kXor2>(v));
    v = fmax(v, dpp_d<dpp::kHalfMirror>(v));
    return fmax(v, dpp_d<dpp::kMirror>(v));
}
__device__ inline int gmin(int v) {
    v = min(v, dpp_i<dpp::kXor1>(v));
    v = min(v, dpp_i<dpp::kXor2>(v));
    v = min(v, dpp_i<dpp::kHalfMirror>(v));
    return min(v, dpp_i<dpp::kMirror>(v));
}
// value of lane SRC of the group
template <int SRC> __device__ inline double gbcast(double v) { return dpp_d<dpp::bcast(SRC)>(v); }
template <int SRC> __device__ inline int gbcast(int v) { return dpp_i<dpp::bcast(SRC)>(v); }
// exclusive prefix sum over the group; *total = sum over the group
__device__ inline int gscan(int v, int *total) {
    int x = v;
    x += dpp_i<dpp::shr(1)>(x);
    x += dpp_i<dpp::shr(2)>(x);
    x += dpp_i<dpp::shr(4)>(x);
    x += dpp_i<dpp::shr(8)>(x);
    *total = gbcast<kGrp - 1>(x);
    return x - v;
}
// position of the group maximum of v (ties: smallest key; keys distinct among the
// lanes that can win), as the first-maximum scan of a pivot search
__device__ inline void gargmax(double v, int key, double *vmax, int *kmin) {
    *vmax = gmax(v);
    *kmin = gmin(v == *vmax ? key : 0x7fffffff);
}

// Phase timing of group_sturm_roots for tools/pt*_bench.hip (compiled out otherwise):
// chain, grid counts, cell isolation, refinement; clock ticks summed over workgroups.
#ifdef MP_GROUP_PROFILE
__device__ unsigned long long gs_prof[4];
#define GS_MARK(i)                                                                                                     \
    do {                                                                                                               \
        const unsigned long long t_ = wall_clock64();                                                                 \
        if (threadIdx.x == 0) atomicAdd(&gs_prof[i], t_ - gs_prev);                                                    \
        gs_prev = t_;                                                                                                  \
    } while (0)
#define GS_START unsigned long long gs_prev = wall_clock64()
#else
#define GS_MARK(i) ((void)0)
#define GS_START ((void)0)
#endif

// LDS of one group's root search
template <int NN> struct GroupSturm {
    double chain[NN + 1][NN + 1];   // Sturm chain (poly k: ascending, degree NN - k)
    int cnt[kGridCells + 1];        // sign-change counts at the grid points
    double lo[NN], hi[NN];          // isolating intervals (scaled variable), slot = root index
    // cells holding several roots, split 16 ways by the whole group (a stack)
    double wlo[kGrp], whi[kGrp];
    int wclo[kGrp], wchi[kGrp], wfirst[kGrp];
    int nwork;
    double sx[kGrp]; // section points of the cell being split and their counts
    int sc[kGrp];
};

// Sturm sign changes at x from the chain in LDS.  Polynomial k has degree NN - k and
// its higher coefficients are stored as zeros, so every Horner runs over all NN + 1
// coefficients (leading zeros keep v == 0 exactly): a rolled loop over the chain,
// which keeps only one polynomial's loads in flight instead of the whole chain.
template <int NN> __device__ inline int sturm_count_lds(const double (*ch)[NN + 1], int len, double x) {
    int changes = 0;
    double prev = 0.0;
#pragma unroll 1
    for (int k = 0; k < len; ++k) {
        double v = 0.0;
#pragma unroll
        for (int j = NN; j >= 0; --j) v = v * x + ch[k][j];
        if (v != 0.0) {
            if (prev != 0.0 && ((v < 0) != (prev < 0))) ++changes;
            prev = v;
        }
    }
    return changes;
}

// Append this lane's interval (lo, hi] with clo - chi >= 2 roots, whose first root
// has index `first`, to the group's stack (group-uniform call).
template <int NN>
__device__ inline void push_work(GroupSturm<NN> &S, bool push, double lo, double hi, int clo, int chi, int first) {
    int np;
    const int at = S.nwork + gscan(push ? 1 : 0, &np);
    if (push && at < kGrp) {
        S.wlo[at] = lo;
        S.whi[at] = hi;
        S.wclo[at] = clo;
        S.wchi[at] = chi;
        S.wfirst[at] = first;
    }
    __syncthreads();
    if ((threadIdx.x % kGrp) == 0) S.nwork = min(S.nwork + np, kGrp);
    __syncthreads();
}

// Real roots of the degree-NN polynomial p (ascending coefficients, held by every
// lane of the group), as sturm_real_roots<NN>.  Returns whether this lane holds a
// root (then in *root); the roots ascend with the lane index (none when !ok).
template <int NN>
__device__ bool group_sturm_roots(const double (&p)[NN + 1], int r, GroupSturm<NN> &S, bool ok, double *root) {
    static_assert(NN < kGrp, "one chain coefficient per lane");
    GS_START;
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
        const double up = dpp_d<dpp::ror(kGrp - 1)>(a); // lane r + 1
        double b = (r < NN) ? (r + 1) * up : 0.0;         // derivative
        const double m1 = gmax(fabs(b));
        if (r < NN) b /= m1;
        if (r <= NN) {
            S.chain[0][r] = a;
            S.chain[1][r] = b;
        }
        len = 2;
        bool alive = true;
        static_for<NN - 1>([&](auto km1) {
            constexpr int k = decltype(km1)::value + 1, d = NN - k;
            const double bd = gbcast<d>(b);
            const double bmax = gmax((r <= d) ? fabs(b) : 0.0);
            if (!(fabs(bd) > 1e-14 * bmax)) alive = false;
            const double ad1 = gbcast<d + 1>(a), ad = gbcast<d>(a), bdm1 = gbcast<d - 1>(b);
            const double q1 = ad1 / bd;
            const double q0 = (ad - q1 * bdm1) / bd;
            const double bm1 = dpp_d<dpp::shr(1)>(b); // lane r - 1 (0 for lane 0)
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
        });
    }
    __syncthreads();
    GS_MARK(0);
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

    // Root isolation.  The roots left of grid point i number cnt[0] - cnt[i], so every
    // cell knows the index of its first root = its first slot.  Cells with one root
    // are isolated already; cells with several are split 16 ways by the whole group
    // (15 interior Sturm counts, one per lane, per round) until every piece holds one
    // root or is narrower than 1e-14 (relative), which yields one interval as in
    // sturm_isolate.  Slots a cluster leaves empty stay NaN.
    GS_MARK(1);
    const int total = ok ? min(S.cnt[0] - S.cnt[kGridCells], NN) : 0;
    __syncthreads();
    if (r < NN) S.lo[r] = __builtin_nan("");
    if (r == 0) S.nwork = 0;
    __syncthreads();
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        const int cell = r + pass * kGrp;
        const double x_lo = -Bnd + cell * h, x_hi = (cell + 1 == kGridCells) ? Bnd : -Bnd + (cell + 1) * h;
        const int v_lo = S.cnt[cell], v_hi = S.cnt[cell + 1], first = S.cnt[0] - v_lo;
        const bool valid = ok && v_lo > v_hi && first >= 0 && first + (v_lo - v_hi) <= NN;
        if (valid && v_lo - v_hi == 1) {
            S.lo[first] = x_lo;
            S.hi[first] = x_hi;
        }
        push_work<NN>(S, valid && v_lo - v_hi >= 2, x_lo, x_hi, v_lo, v_hi, first);
    }
    for (int guard = 0; guard < 64; ++guard) {
        const int nw = S.nwork;
        if (nw == 0) break;
        const double lo = S.wlo[nw - 1], hi = S.whi[nw - 1];
        const int clo = S.wclo[nw - 1], chi = S.wchi[nw - 1], first = S.wfirst[nw - 1];
        __syncthreads();
        if (r == 0) S.nwork = nw - 1;
        __syncthreads();
        if (hi - lo <= 1e-14 * fmax(1.0, fmax(fabs(lo), fabs(hi)))) {
            if (r == 0) {
                S.lo[first] = lo;
                S.hi[first] = hi;
            }
            __syncthreads();
            continue;
        }
        const double step = (hi - lo) * (1.0 / kGrp);
        const double x = (r == kGrp - 1) ? hi : lo + (r + 1) * step;
        const int cx = (r == kGrp - 1) ? chi : sturm_count_lds<NN>(ch, len, x);
        S.sx[r] = x;
        S.sc[r] = cx;
        __syncthreads();
        const double xp = r == 0 ? lo : S.sx[r - 1];
        const int cp = r == 0 ? clo : S.sc[r - 1];
        const int d = cp - cx, f = first + (clo - cp);
        const bool piece = d >= 1 && f >= 0 && f + d <= NN;
        if (piece && d == 1) {
            S.lo[f] = xp;
            S.hi[f] = x;
        }
        push_work<NN>(S, piece && d >= 2, xp, x, cp, cx, f);
    }
    __syncthreads();

    GS_MARK(2);
    // one lane per root (slot r): refinement on the unscaled monic polynomial
    const bool has = r < total && S.lo[r] == S.lo[r];
    if (has) *root = refine_root<NN>(c, sigma * S.lo[r], sigma * S.hi[r]);
    GS_MARK(3);
    return has;
}

} // namespace
} // namespace mp
