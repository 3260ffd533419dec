// 6-point shared-focal roots with one 16-lane group per sample (4 samples per
// 64-lane workgroup) -- the root stage of the shared-focal point solver (PoseLib
// relpose_6pt_shared_focal as called at src/hybrid_pose_shared_focal_estimator.cpp:87,
// formulated as in mp_pt67.h: q(u) = det(u^2 M0 + u M1 + M2) / u^5 by a 16-point DFT
// of complex 10x10 determinants, positive real roots by Sturm sequences).
//
// The one-lane formulation (pt_roots_kernel<kSF>) keeps the 3x10x10 pencil and the
// complex 10x10 LU of each of the 18 determinant evaluations in one lane: about
// 500 live doubles, so the compiler spills to scratch and one launch takes
// milliseconds.  Here:
//   * lane r < 10 builds and keeps row r of the pencil (sixpt_row, 30 doubles);
//   * each determinant is an LU over the group: lane r eliminates its own complex
//     row, the pivot is a group argmax (|re| + |im|, ties to the lowest current row
//     position, which is the lane code's first-maximum rule), the pivot row is
//     broadcast through LDS, rows are tracked by position instead of swapped;
//   * the 16 DFT coefficients are one per lane; the rho adaptation of sixpt_roots is
//     applied by always running the second pass (rho = 1 reproduces the first);
//   * the degree-15 Sturm search is group_sturm_roots<15>, one lane per root.
// Per value the operations are those of det_pencil10 / pencil_poly15 /
// sturm_real_roots, so both kernels agree up to FMA contraction.
#pragma once
#include "../../madpose_amd/csrc/include/mp_pt67.h"
#include "../../madpose_amd/csrc/kernels/group_sturm.h"

namespace mp {
namespace {

constexpr int kSixDeg = 15; // degree of q(u)

// Phase timing for tools/pt6_bench.hip (compiled out otherwise): clock ticks per
// phase summed over workgroups (lane 0).
#ifdef MP_GROUP6_PROFILE
__device__ unsigned long long g6_prof[8];
#define G6_MARK(i)                                                                                                     \
    do {                                                                                                               \
        const unsigned long long t_ = wall_clock64();                                                                 \
        if (threadIdx.x == 0) atomicAdd(&g6_prof[i], t_ - t_prev);                                                     \
        t_prev = t_;                                                                                                   \
    } while (0)
#define G6_START unsigned long long t_prev = wall_clock64()
#else
#define G6_MARK(i) ((void)0)
#define G6_START ((void)0)
#endif

struct Group6Shared {
    double N[kGrpPerWg][3][9];          // null-space basis of the epipolar constraints
    double piv[kGrpPerWg][20];          // broadcast pivot row (complex, columns k..9)
    double qv[kGrpPerWg][9][2];         // q at the DFT nodes 0..8
    double q[kGrpPerWg][kSixDeg + 1];   // DFT coefficients gathered from the lanes
    GroupSturm<kSixDeg> st[kGrpPerWg];  // root search of q(u)
};

// det(u^2 M0 + u M1 + M2) by a group LU; lane r < 10 holds row r of M0, M1, M2
// (det_pencil10 in mp_pt67.h).  Every lane of the workgroup must call it.
__device__ inline Cx group_det_pencil10(const double (&m0)[10], const double (&m1)[10], const double (&m2)[10], Cx u,
                                        int r, double *piv) {
    const Cx u2 = cmul(u, u);
    Cx A[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) A[c] = {u2.r * m0[c] + u.r * m1[c] + m2[c], u2.i * m0[c] + u.i * m1[c]};
    const bool row_lane = r < 10;
    int pos = r; // current row position of this lane's row
    Cx det = {1.0, 0.0};
    bool zero = false;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const bool cand = row_lane && pos >= k;
        double bv;
        int bp;
        gargmax(cand ? fabs(A[k].r) + fabs(A[k].i) : -1.0, pos, &bv, &bp);
        if (bv == 0.0) zero = true;
        const bool piv_lane = cand && pos == bp;
        if (piv_lane) {
#pragma unroll
            for (int c = k; c < 10; ++c) {
                piv[2 * c] = A[c].r;
                piv[2 * c + 1] = A[c].i;
            }
        }
        __syncthreads();
        const Cx pk = {piv[2 * k], piv[2 * k + 1]};
        if (bp != k) {
            det.r = -det.r;
            det.i = -det.i;
            if (pos == k) pos = bp;
        }
        if (piv_lane) pos = k;
        det = cmul(det, pk);
        const Cx inv = cdiv({1.0, 0.0}, pk);
        if (row_lane && pos > k) {
            const Cx l = cmul(A[k], inv);
#pragma unroll
            for (int c = k + 1; c < 10; ++c) A[c] = csub(A[c], cmul(l, Cx{piv[2 * c], piv[2 * c + 1]}));
        }
        __syncthreads();
    }
    return zero ? Cx{0.0, 0.0} : det;
}

// cand: N (27 doubles) then the positive roots u (ascending); ncand: their number
// waves per SIMD the register allocation targets (tools/pt6_bench.hip A/B)
#ifndef MP_G6_WAVES
#define MP_G6_WAVES 2
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MP_G6_WAVES))) pt_roots6_group_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                             const int *samples, double *cand, int *ncand,
                                                             int cand_stride) {
    __shared__ Group6Shared sh;
    const int g = threadIdx.x / kGrp, r = threadIdx.x % kGrp;
    const int idx = blockIdx.x * kGrpPerWg + g;
    const bool active = idx < nlist;
    const int *s = samples + (size_t)list[active ? idx : nlist - 1] * kSampleStride;
    G6_START;

    // ---- null space of the epipolar constraints (every lane), row r of the pencil ----
    double m0[10], m1[10], m2[10];
    {
        double N[3][9];
        {
            double b0[6][3], b1[6][3];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int i = s[j];
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
            if (q % kGrp == r) sh.N[g][q / 9][q % 9] = N[q / 9][q % 9];
    }
    __syncthreads();
    if (r < 10) {
        const double(*Nl)[9] = sh.N[g];
        sixpt_row([&](int e) { return Lin2{{Nl[0][e], Nl[1][e], Nl[2][e]}}; }, r, m0, m1, m2);
    } else {
#pragma unroll
        for (int c = 0; c < 10; ++c) m0[c] = m1[c] = m2[c] = 0.0;
    }
    G6_MARK(0);
    // ---- q(u) on |u| = 1, then on |u| = rho (pencil_poly15 / sixpt_roots) ----
    double poly[kSixDeg + 1];
    double rho = 1.0;
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
        // q at the nodes j = 0..8 (the other 7 by conjugate symmetry), kept in LDS
#pragma unroll 1
        for (int j = 0; j <= 8; ++j) {
            const double th = 2.0 * 3.14159265358979323846 * j / 16.0;
            const Cx u = {rho * cos(th), rho * sin(th)};
            const Cx d = group_det_pencil10(m0, m1, m2, u, r, sh.piv[g]);
            const double r5 = rho * rho * rho * rho * rho;
            const Cx inv5 = {cos(5.0 * th) / r5, -sin(5.0 * th) / r5};
            const Cx qj = cmul(d, inv5);
            if (r == 0) {
                sh.qv[g][j][0] = qj.r;
                sh.qv[g][j][1] = qj.i;
            }
        }
        __syncthreads();
        G6_MARK(1 + 2 * pass);
        // coefficient k = r of this lane
        {
            const int k = r;
            double acc = 0.0;
#pragma unroll 1
            for (int j = 0; j < 16; ++j) { // (rolled: one cos/sin in flight keeps registers low)
                const int jj = (j <= 8) ? j : 16 - j;
                const Cx q = (j <= 8) ? Cx{sh.qv[g][jj][0], sh.qv[g][jj][1]} : Cx{sh.qv[g][jj][0], -sh.qv[g][jj][1]};
                const double th = -2.0 * 3.14159265358979323846 * j * k / 16.0;
                acc += q.r * cos(th) - q.i * sin(th);
            }
            sh.q[g][k] = acc / 16.0 / pow(rho, (double)k);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k <= kSixDeg; ++k) poly[k] = sh.q[g][k];
        __syncthreads();
        if (pass == 0) {
            if (poly[0] != 0.0 && poly[kSixDeg] != 0.0) {
                rho = pow(fabs(poly[0] / poly[kSixDeg]), 1.0 / 15.0);
                if (!(rho > 0.0) || !(rho < 1e300)) rho = 1.0;
            }
        }
        G6_MARK(2 + 2 * pass);
    }

    // ---- real roots of q, keep u > 0 ----
    double u = 0.0;
    const bool has_root = group_sturm_roots<kSixDeg>(poly, r, sh.st[g], true, &u);
    G6_MARK(5);
    const bool keep = has_root && u > 0.0;
    int nk;
    const int at = gscan(keep ? 1 : 0, &nk);
    if (active) {
        double *out = cand + (size_t)idx * cand_stride;
#pragma unroll
        for (int q = 0; q < 27; ++q)
            if (q % kGrp == r) out[q] = sh.N[g][q / 9][q % 9];
        if (keep) out[27 + at] = u;
        if (r == 0) ncand[idx] = nk;
    }
    G6_MARK(6);
}

// The same root stage with one sample per 64-lane workgroup: the four 16-lane groups
// evaluate the nine DFT nodes of a pass in parallel (group g takes nodes g, g + 4,
// g + 8), so a pass costs three determinant LUs in sequence instead of nine.  Every
// group builds the pencil rows and runs the DFT and the Sturm search on the same
// values (the barriers inside need every lane); group 0 writes.  Per value the
// operations are those of pt_roots6_group_kernel, so the two agree bit for bit.
// Measured slower at the shared-focal batch sizes (399 vs 291 us per launch: four
// times the waves, and the LU steps are issue-bound, not latency-bound), so it is an
// A/B option (MADPOSE_PT6_WAVE=1), not the default.
struct Group6WaveShared {
    double N[3][9];
    double piv[kGrpPerWg][20];
    double qv[9][2];
    double q[kSixDeg + 1];
    GroupSturm<kSixDeg> st[kGrpPerWg];
};

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MP_G6_WAVES)))
pt_roots6_wave_kernel(PairData D, PairConst C, const int *list, int nlist, const int *samples, double *cand,
                      int *ncand, int cand_stride) {
    __shared__ Group6WaveShared sh;
    const int g = threadIdx.x / kGrp, r = threadIdx.x % kGrp;
    const int idx = blockIdx.x;
    const int *s = samples + (size_t)list[idx] * kSampleStride;

    double m0[10], m1[10], m2[10];
    {
        double N[3][9];
        {
            double b0[6][3], b1[6][3];
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                const int i = s[j];
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
        if (g == 0) {
#pragma unroll
            for (int q = 0; q < 27; ++q)
                if (q % kGrp == r) sh.N[q / 9][q % 9] = N[q / 9][q % 9];
        }
    }
    __syncthreads();
    if (r < 10) {
        sixpt_row([&](int e) { return Lin2{{sh.N[0][e], sh.N[1][e], sh.N[2][e]}}; }, r, m0, m1, m2);
    } else {
#pragma unroll
        for (int c = 0; c < 10; ++c) m0[c] = m1[c] = m2[c] = 0.0;
    }
    double poly[kSixDeg + 1];
    double rho = 1.0;
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll 1
        for (int jb = 0; jb <= 8; jb += kGrpPerWg) {
            const int j = jb + g; // node of this group (j > 8: a discarded LU that keeps the barriers in step)
            const int jn = j <= 8 ? j : 8;
            const double th = 2.0 * 3.14159265358979323846 * jn / 16.0;
            const Cx u = {rho * cos(th), rho * sin(th)};
            const Cx d = group_det_pencil10(m0, m1, m2, u, r, sh.piv[g]);
            const double r5 = rho * rho * rho * rho * rho;
            const Cx inv5 = {cos(5.0 * th) / r5, -sin(5.0 * th) / r5};
            const Cx qj = cmul(d, inv5);
            if (r == 0 && j <= 8) {
                sh.qv[j][0] = qj.r;
                sh.qv[j][1] = qj.i;
            }
        }
        __syncthreads();
        if (g == 0) {
            const int k = r;
            double acc = 0.0;
#pragma unroll 1
            for (int j = 0; j < 16; ++j) {
                const int jj = (j <= 8) ? j : 16 - j;
                const Cx q = (j <= 8) ? Cx{sh.qv[jj][0], sh.qv[jj][1]} : Cx{sh.qv[jj][0], -sh.qv[jj][1]};
                const double th = -2.0 * 3.14159265358979323846 * j * k / 16.0;
                acc += q.r * cos(th) - q.i * sin(th);
            }
            sh.q[k] = acc / 16.0 / pow(rho, (double)k);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k <= kSixDeg; ++k) poly[k] = sh.q[k];
        __syncthreads();
        if (pass == 0) {
            if (poly[0] != 0.0 && poly[kSixDeg] != 0.0) {
                rho = pow(fabs(poly[0] / poly[kSixDeg]), 1.0 / 15.0);
                if (!(rho > 0.0) || !(rho < 1e300)) rho = 1.0;
            }
        }
    }

    double u = 0.0;
    const bool has_root = group_sturm_roots<kSixDeg>(poly, r, sh.st[g], true, &u);
    const bool keep = has_root && u > 0.0;
    int nk;
    const int at = gscan(keep ? 1 : 0, &nk);
    if (g == 0) {
        double *out = cand + (size_t)idx * cand_stride;
#pragma unroll
        for (int q = 0; q < 27; ++q)
            if (q % kGrp == r) out[q] = sh.N[q / 9][q % 9];
        if (keep) out[27 + at] = u;
        if (r == 0) ncand[idx] = nk;
    }
}

} // namespace
} // namespace mp
