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
#include "kernels.h"

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

// Front of the root stage, four samples per 64-lane wave (16-lane groups): the
// epipolar null space N (every lane of the group) into cand[0, 27) and the pencil
// rows (lane r < 10: row r of M0, M1, M2, sixpt_row) into pen (300 doubles per
// sample, M[a][r][c] at 100 a + 10 r + c).  Split from the eigen kernel so that the
// latter's register allocation is not set by this register-heavy part.
constexpr int kPenStride = 300;
static_assert(kPenStride == kPtPenStride, "the engine sizes the pencil workspace with kPtPenStride (kernels.h)");
__global__ void __launch_bounds__(64) pt_pencil6_kernel(PairData D, const int *list, int nlist, const int *samples,
                                                        double *cand, int cand_stride, double *pen) {
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
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

// (EISPACK sign transfer, used by the generated QR of eig15_gen.h)
__device__ inline double e6_sign(double a, double b) { return b >= 0 ? fabs(a) : -fabs(a); }
// The bulge reflectors' reciprocals (1 / |p|+|q|+|r|, 1 / s, 1 / (p + s), all nonzero
// there): the hardware reciprocal refined by two Newton steps (within about an ulp, 5
// FP64 instructions on the sweep's serial chain instead of the division's 11), branch-free
// (a range guard's branch cost the straight-line sweep more than it saved).  Both QR
// kernels (one sample per wave, samples per lane) run this code, so their roots stay
// bit-identical to each other.
// sqrt(p^2 + q^2 + r^2) of a reflector whose (p, q, r) were scaled to |p|+|q|+|r| = 1
// (or are all zero): the argument lies in [1/3, 1] or is 0, so the hardware inverse
// square root refined by one Newton step on each of the root and its half reciprocal
// (8 FP64 instructions) needs none of the general sqrt's range scaling (16); within
// about an ulp
__device__ inline double e6_sqrt_unit(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double e = fma(-h, g, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    const double d = fma(-g, g, x);
    g = fma(d, h, g);
    return x == 0.0 ? 0.0 : g;
}
__device__ inline double e6_rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// ---------------------------------------------------------------------------
// The 15 x 15 eigenproblem with one sample per lane, every access static:
// every lane runs the Francis double-shift QR (hqr) on its own balanced Hessenberg
// matrix (balance + elmhes ran in pt_defl6_grp), but all 64 lanes execute the same
// static instruction stream -- every loop bound is a compile-time constant, every
// array index a constant after unrolling, and the per-lane quantities (active window,
// deflation) enter only through selects.  The matrix lives in registers: the code
// generated by tools/gen_eig15.py (eig15_gen.h) keeps the 15 x 15 entries as per-lane
// doubles, which the compiler allocates to 256 VGPRs + 103 AGPRs (2 VGPRs spilled to
// AGPRs, no scratch, no LDS; -Rpass-analysis=kernel-resource-usage, round 4), hence one
// wave per SIMD.  A QR sweep always runs the 14 bulge positions; a position outside a
// lane's active window [l, nn] applies the identity reflector.  Row updates run to
// column 14 and column updates from row 0 (the full Schur-form updates), which leaves
// the window's eigenvalues unchanged.  The chase starts at the window's top l (hqr may
// start lower when a subdiagonal decouples: the same similarity up to rounding).  No
// divergence: a wave of 64 samples takes about as long as one sample, so one launch
// handles up to 64 x 1024 samples at that latency.  Eigenvalues go to the sample's
// pencil slot past the block (wr, wi), the positive real roots to cand / ncand.
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
// U (spw == 1): every lane runs the wave's one sample, which makes the QR's window
// wave-uniform (e15_hqr<true>: scalar branches instead of select chains); lane 0 writes.
template <bool U>
__global__ void __launch_bounds__(64) pt_eig6_reg_kernel(double *pen, int nlist, int spw, double *cand, int *ncand,
                                                         int cand_stride, BatchGate gate) {
    if (batch_cancelled(gate.word, gate.hi)) return;
    const int idx = U ? (int)blockIdx.x : (int)(blockIdx.x * spw + threadIdx.x);
    const bool valid = (U || (int)threadIdx.x < spw) && idx < nlist;
    const int sidx = valid ? idx : nlist - 1;
    double *P = pen + (size_t)sidx * kPenStride;
    const bool active = valid && P[225] != 0.0;
    // eigenvalues into the sample's own pencil slot past the block (free by now)
    double *wr = P + 240, *wi = wr + kN15;
#ifdef MP_EIG6_PROFILE
    const unsigned long long t_hqr0 = wall_clock64();
#endif
    const bool conv = e15_hqr<U>(P, active, wr, wi);
#ifdef MP_EIG6_PROFILE
    if (threadIdx.x == 0) atomicAdd(&e6_prof[6], wall_clock64() - t_hqr0);
#endif
    if (!valid || (U && threadIdx.x != 0)) return;
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
