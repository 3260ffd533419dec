// Point-solver tails with one 8-lane group per (root, sample): two-focal below, then
// calibrated.  Two-focal
// (src/hybrid_pose_two_focal_estimator.cpp:118-181): Bougnoux focals of the root's F,
// E = K1^T F K0, cv::recoverPose on the seven points, triangulation and the affine
// depth fits.
//
// The one-lane formulation (pt_tail_kernel<kTF>) runs 4 x 7 DLT triangulations for
// recoverPose plus 7 for the depth fit, each a 4x4 Jacobi SVD, back to back in one
// lane.  Here lane j (< 7) holds point j of the sample: it tests its point under each
// candidate pose and triangulates it for the depth fit, and the counts and the fit's
// sums are all-reduced over the group on DPP (quad butterflies + the half-row
// mirror).  The per-root work (focals, E, candidate poses) is computed redundantly in
// every lane.  Per value the operations are those of recover_pose_cv /
// point_model_tail, except that the fit's sums run as a tree over the points.
#pragma once
#include "../include/mp_md.h"
#include "../include/mp_pt67.h"
#include "group_sturm.h"

namespace mp {
namespace {

constexpr int kTail = 8; // lanes per (root, sample)

// all-reduce over the 8-lane group (the half-row of a DPP row)
__device__ inline double gsum8(double v) {
    v += dpp_d<dpp::kXor1>(v);
    v += dpp_d<dpp::kXor2>(v);
    return v + dpp_d<dpp::kHalfMirror>(v);
}
__device__ inline int gsum8(int v) {
    v += dpp_i<dpp::kXor1>(v);
    v += dpp_i<dpp::kXor2>(v);
    return v + dpp_i<dpp::kHalfMirror>(v);
}

// the sum over the 8-lane group in lane order, (((0 + v0) + v1) + ..) + v7, in every lane:
// the oracle's sequential sums over the sample's points (lane j holds point j)
__device__ inline double gsum8_ordered(double v) {
    const bool hi = (threadIdx.x & 8) != 0;
    double s = 0.0;
    static_for<kTail>([&](auto j) {
        const double a = gbcast<decltype(j)::value>(v), b = gbcast<decltype(j)::value + 8>(v);
        s += hi ? b : a;
    });
    return s;
}

// group g of the launch = root k of sample idx, root-major as pt_tail_kernel.
// G = 8: one 8-lane group per (root, sample), every lane tests its point under the
// four recoverPose candidates in turn.  G = 32: four 8-lane subgroups per (root,
// sample), subgroup c tests candidate c (one DLT triangulation per lane instead of
// four), the four good-point counts are exchanged across the subgroups, and the
// subgroups then run the depth fit redundantly (subgroup 0 writes).
template <int G>
__global__ void __launch_bounds__(64) pt_tail7_group_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                            const double *cand, const int *ncand, const int *samples,
                                                            Model *slots, int *valid) {
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
    static_assert(G == 8 || G == 32, "8 or 32 lanes per (root, sample)");
    constexpr int K = 7;
    const int lane = threadIdx.x % kTail;
    const int sub = (threadIdx.x % G) / kTail; // candidate of this subgroup (G = 32)
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G);
    const int k = gid / nlist, idx = gid - k * nlist;
    if (k >= 3 || k >= ncand[idx]) return; // the whole group leaves together
    const int *s = samples + (size_t)list[idx] * kSampleStride;
    const bool has = lane < K;
    const int i = s[has ? lane : K - 1];
    const double p0[1][2] = {{D.x0u[i], D.x0v[i]}}, p1[1][2] = {{D.x1u[i], D.x1v[i]}};
    const double dd0[1] = {D.d0[i]}, dd1[1] = {D.d1[i]};
    const double *F = cand + (size_t)idx * kPtCandStride + 9 * k;

    // twofocal_pose_from_F: focals, E, recoverPose
    double f0, f1;
    bougnoux_sq(F, &f0, &f1);
    f0 = sqrt(fabs(f0));
    f1 = sqrt(fabs(f1));
    double E[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) E[3 * r + c] = (r < 2 ? f1 : 1.0) * F[3 * r + c] * (c < 2 ? f0 : 1.0);
    RecoverCands rc;
    recover_pose_candidates(E, rc);
    int good[4];
    if (G == 8) {
        // one SVD per rotation decides both signs of t (recover_pose_good_pair)
#pragma unroll
        for (int kr = 0; kr < 2; ++kr) {
            bool gp, gn;
            recover_pose_good_pair(rc, kr, p0[0], p1[0], 1e9, &gp, &gn);
            good[kr] = gsum8((has && gp) ? 1 : 0);
            good[kr + 2] = gsum8((has && gn) ? 1 : 0);
        }
    } else {
        const int mine = gsum8((has && recover_pose_good(rc, sub, p0[0], p1[0], 1e9)) ? 1 : 0);
        const int base = (threadIdx.x & 63) & ~(G - 1);
#pragma unroll
        for (int c = 0; c < 4; ++c) good[c] = __shfl(mine, base + kTail * c, 64);
    }
    Model m;
    recover_pose_select(rc, good, m.R, m.t);
    m.scale = 1.0;
    m.offset0 = m.offset1 = 0.0;
    m.focal0 = f0;
    m.focal1 = f1;

    // point_model_tail<7> with one point per lane
    const bool use[1] = {has};
    const bool shift = C.use_shift != 0 && !C.scale_only, mdc = C.min_depth_constraint != 0;
    const bool ok = point_model_tail_r<1>(p0, p1, dd0, dd1, use, (double)K, m.focal0, m.focal1, shift, mdc,
                                          C.min_depth, m, [](double v) { return gsum8(v); });
    if (lane == 0 && sub == 0) {
        const size_t q = (size_t)idx * kPtSlotStride + k; // PtTraits<kTF>::kPosesPerRoot == 1
        if (ok) slots[q] = m;
        valid[q] = ok ? 1 : 0;
    }
}

// Calibrated tail (src/hybrid_pose_estimator.cpp:134-182) with one 8-lane group per
// (root, sample), lane j < 5 holding point j: the cheirality tests of
// motion_from_essential (AND over the group), then for each of the at most two poses
// the triangulation (dlt_null4: Householder QR + inverse iteration, restated in the
// oracle) and depth fit with the group's sums taken in point order -- round 6: the
// oracle's point_model_tail operation for operation, so a calibrated 5pt model is the
// oracle's to the bit (tests/test_ties_gpu.py::test_calibrated_models_are_the_oracles_to_the_bit).
// (the body of workgroup `bid`: pt_tail5_group_kernel, and the fused MD-root + tail
// launch of kernels.hip, which gives it the workgroups past the MD roots')
__device__ __forceinline__ void pt_tail5_group_body(int bid, const PairData &D, const PairConst &C, const int *list,
                                                    int nlist, const double *cand, const int *ncand,
                                                    const int *samples, Model *slots, int *valid) {
#pragma clang fp contract(off)
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
    constexpr int K = 5, kRoots = 10, kPoses = 2;
    const int lane = threadIdx.x % kTail;
    const int gid = (int)((bid * (size_t)blockDim.x + threadIdx.x) / kTail);
    const int k = gid / nlist, idx = gid - k * nlist;
    if (k >= kRoots || k >= ncand[idx]) return; // the whole group leaves together
    const int *s = samples + (size_t)list[idx] * kSampleStride;
    const bool has = lane < K;
    const int i = s[has ? lane : K - 1];
    // one point of the oracle's minimal_solver: calibrated ray c = K^-1 x, unit bearing
    // c / |c|, depth priors (no FMA contraction: the oracle's values to the bit)
    const double xa[3] = {D.x0u[i], D.x0v[i], 1.0}, xb[3] = {D.x1u[i], D.x1v[i], 1.0};
    double a[3], c[3];
    matvec3_x(C.K0i, xa, a);
    matvec3_x(C.K1i, xb, c);
    const double na = sqrt(dot3_x(a, a)), nc = sqrt(dot3_x(c, c));
    const double b1[1][3] = {{a[0] / na, a[1] / na, a[2] / na}}, b2[1][3] = {{c[0] / nc, c[1] / nc, c[2] / nc}};
    const double p0[1][2] = {{a[0], a[1]}}, p1[1][2] = {{c[0], c[1]}};
    const double dd0[1] = {D.d0[i]}, dd1[1] = {D.d1[i]};
    const bool use[1] = {has};
    Model poses[kPoses];
    const int np = motion_from_essential_r<1>(
        cand + (size_t)idx * kPtCandStride + 9 * k, b1, b2, use, kPoses,
        [](bool ok) { return gsum8(ok ? 0 : 1) == 0; },
        [&](const Model &m, int q) { // (static slots: poses[] stays in registers)
            if (q == 0) poses[0] = m;
            if (q == 1) poses[1] = m;
        });
    const bool shift = C.use_shift != 0 && !C.scale_only, mdc = C.min_depth_constraint != 0;
#pragma unroll
    for (int j = 0; j < kPoses; ++j) {
        bool ok = false;
        Model m;
        if (j < np) { // (uniform over the group)
            m = poses[j];
            ok = point_model_tail_r<1>(p0, p1, dd0, dd1, use, (double)K, 1.0, 1.0, shift, mdc, C.min_depth, m,
                                       [](double v) { return gsum8_ordered(v); });
        }
        if (lane == 0) {
            const size_t q = (size_t)idx * kPtSlotStride + kPoses * k + j;
            if (ok) slots[q] = m;
            valid[q] = ok ? 1 : 0;
        }
    }
}

__global__ void __launch_bounds__(64) pt_tail5_group_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                            const double *cand, const int *ncand, const int *samples,
                                                            Model *slots, int *valid) {
    pt_tail5_group_body(blockIdx.x, D, C, list, nlist, cand, ncand, samples, slots, valid);
}

// Shared-focal tail (src/hybrid_pose_shared_focal_estimator.cpp:87-126, the per-root
// part of sixpt_poses_for_root in mp_pt67.h) with one 16-lane group per (root,
// sample): lane r < 10 holds row r of the pencil A(w) = M0 + w M1 + w^2 M2 at the root
// w = 1 / u; the null vector of A comes from a group Gaussian elimination with
// complete pivoting (pivot = group maximum over the remaining rows and columns; the
// pivot rows go to LDS for the back substitution), the Gauss-Newton polish of
// (x, y, w) sums the ten rows' normal equations over the group, and lane j < 6 holds
// point j for motion_from_essential and the depth fit.
struct Tail6Shared {
    double U[kGrpPerWg][9][10]; // pivot rows
    double z[kGrpPerWg][10];    // null vector (original column order)
    int pc[kGrpPerWg][9];       // pivot columns
};

__device__ inline double gsum16(double v) {
    v += dpp_d<dpp::kXor1>(v);
    v += dpp_d<dpp::kXor2>(v);
    v += dpp_d<dpp::kHalfMirror>(v);
    return v + dpp_d<dpp::kMirror>(v);
}
__device__ inline int gsum16(int v) {
    v += dpp_i<dpp::kXor1>(v);
    v += dpp_i<dpp::kXor2>(v);
    v += dpp_i<dpp::kHalfMirror>(v);
    return v + dpp_i<dpp::kMirror>(v);
}

__global__ void __launch_bounds__(64) pt_tail6_group_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                            const double *cand, const int *ncand, const int *samples,
                                                            Model *slots, int *valid) {
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
    constexpr int K = 6, kRoots = 15, kPoses = 2;
    __shared__ Tail6Shared sh;
    const int g = threadIdx.x / kGrp, r = threadIdx.x % kGrp;
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kGrp);
    const int k = gid / nlist, idx = gid - k * nlist;
    if (k >= kRoots || k >= ncand[idx]) return; // the whole group leaves together
    const double *cd = cand + (size_t)idx * kPtCandStride;
    const bool row_lane = r < 10;
    double w = 1.0 / cd[27 + k];
    // a root that yields no pose clears its slots (they hold an earlier batch's models)
    auto no_pose = [&]() {
        if (r == 0)
#pragma unroll
            for (int j = 0; j < kPoses; ++j) valid[(size_t)idx * kPtSlotStride + kPoses * k + j] = 0;
    };

    // ---- row r of the pencil and of A(w) ----
    double m0[10], m1[10], m2[10], a[10];
    if (row_lane) {
        sixpt_row([&](int e) { return Lin2{{cd[e], cd[9 + e], cd[18 + e]}}; }, r, m0, m1, m2);
    } else {
#pragma unroll
        for (int c = 0; c < 10; ++c) m0[c] = m1[c] = m2[c] = 0.0;
    }
#pragma unroll
    for (int c = 0; c < 10; ++c) a[c] = m0[c] + w * (m1[c] + w * m2[c]);

    // ---- null vector: complete pivoting over the group (null_vector10) ----
    bool used = !row_lane, ok = true;
    unsigned cols = 0; // eliminated columns
#pragma unroll
    for (int kk = 0; kk < 9; ++kk) {
        double bv = -1.0;
        int bc = 0;
        if (!used) {
#pragma unroll
            for (int c = 0; c < 10; ++c)
                if (!(cols >> c & 1u) && fabs(a[c]) > bv) {
                    bv = fabs(a[c]);
                    bc = c;
                }
        }
        double vmax;
        int key;
        gargmax(bv, r * 16 + bc, &vmax, &key); // ties: lowest row, then lowest column
        if (!(vmax > 0.0)) ok = false;
        const int prow = key / 16, pcol = key % 16;
        if (r == prow) {
#pragma unroll
            for (int c = 0; c < 10; ++c) sh.U[g][kk][c] = a[c];
            sh.pc[g][kk] = pcol;
            used = true;
        }
        __syncthreads();
        if (!used) {
            // (the quotients by the pivot through its reciprocal: the shared-focal tail is
            // held to the oracle by tolerance, not to the bit)
            const double l = pick(a, pcol) * svd_rcp(sh.U[g][kk][pcol]);
#pragma unroll
            for (int c = 0; c < 10; ++c)
                if (!(cols >> c & 1u) && c != pcol) a[c] -= l * sh.U[g][kk][c];
        }
        cols |= 1u << pcol;
        __syncthreads();
    }
    if (!ok) { // (uniform)
        no_pose();
        return;
    }
    // back substitution (lane 0): free column = the one never pivoted, z = 1 there
    if (r == 0) {
        const int fc = __ffs(~cols & 0x3ffu) - 1;
        for (int c = 0; c < 10; ++c) sh.z[g][c] = 0.0;
        sh.z[g][fc] = 1.0;
        for (int kk = 8; kk >= 0; --kk) {
            double s = 0.0;
            for (int q = kk + 1; q < 9; ++q) s += sh.U[g][kk][sh.pc[g][q]] * sh.z[g][sh.pc[g][q]];
            s += sh.U[g][kk][fc] * sh.z[g][fc];
            sh.z[g][sh.pc[g][kk]] = -s * svd_rcp(sh.U[g][kk][sh.pc[g][kk]]);
        }
    }
    __syncthreads();
    double x, y;
    {
        double zv[10];
#pragma unroll
        for (int c = 0; c < 10; ++c) zv[c] = sh.z[g][c];
        if (!sixpt_xy_from_monomials(zv, &x, &y)) { // (uniform)
            no_pose();
            return;
        }
    }

    // ---- Gauss-Newton polish of (x, y, w), rows summed over the group ----
    for (int it = 0; it < 5; ++it) {
        double mv[10], dxv[10], dyv[10];
        mono2(x, y, mv, dxv, dyv);
        double res = 0, jx = 0, jy = 0, jw = 0;
#pragma unroll
        for (int c = 0; c < 10; ++c) {
            const double m = m0[c] + w * (m1[c] + w * m2[c]);
            res += m * mv[c];
            jx += m * dxv[c];
            jy += m * dyv[c];
            jw += (m1[c] + 2.0 * w * m2[c]) * mv[c];
        }
        const double J[3] = {jx, jy, jw};
        double JtJ[3][3], Jtr[3][1];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            Jtr[p][0] = gsum16(J[p] * res);
#pragma unroll
            for (int q = 0; q < 3; ++q) JtJ[p][q] = q < p ? JtJ[q][p] : gsum16(J[p] * J[q]);
        }
        if (!gauss_solve<3, 1>(JtJ, Jtr)) break;
        x -= Jtr[0][0];
        y -= Jtr[1][0];
        w -= Jtr[2][0];
    }
    // a root of the interpolated q(u) that is not a root of the system (its small
    // coefficients carry rounding) leaves a residual after the polish:
    // keep the root only if the ten equations vanish to 1e-8 of their term scale
    {
        double mv[10], dxv[10], dyv[10];
        mono2(x, y, mv, dxv, dyv);
        double res = 0, mag = 0;
#pragma unroll
        for (int c = 0; c < 10; ++c) {
            const double t = (m0[c] + w * (m1[c] + w * m2[c])) * mv[c];
            res += t;
            mag += fabs(t);
        }
        const double rr = gsum16(res * res), ss = gsum16(mag * mag);
        if (!(rr <= 1e-16 * ss)) w = -1.0; // (uniform)
    }
    if (!(w > 0.0)) {
        no_pose();
        return;
    }
    const double foc = svd_rsq(w), ifoc = w * foc; // (1 / foc = sqrt(w))
    double Fm[9], nn = 0.0;
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        Fm[e] = x * cd[e] + y * cd[9 + e] + cd[18 + e];
        nn += Fm[e] * Fm[e];
    }
    nn = svd_rsq(nn);
    double E[9];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int q = 0; q < 3; ++q) E[3 * p + q] = Fm[3 * p + q] * nn * (p < 2 ? foc : 1.0) * (q < 2 ? foc : 1.0);

    // ---- poses and depth tail, point j = lane j (< 6) ----
    const int *s = samples + (size_t)list[idx] * kSampleStride;
    const bool has = r < K;
    const int i = s[has ? r : K - 1];
    const double pa[3] = {D.x0u[i], D.x0v[i], 1.0}, pb[3] = {D.x1u[i], D.x1v[i], 1.0};
    const double ia = svd_rsq(dot3(pa, pa)), ib = svd_rsq(dot3(pb, pb));
    // the bearing's xy divided by the focal, re-normalised (sixpt_poses_for_root)
    const double ba[3] = {pa[0] * ia * ifoc, pa[1] * ia * ifoc, pa[2] * ia},
                 bb[3] = {pb[0] * ib * ifoc, pb[1] * ib * ifoc, pb[2] * ib};
    const double na = svd_rsq(dot3(ba, ba)), nb = svd_rsq(dot3(bb, bb));
    const double c1[1][3] = {{ba[0] * na, ba[1] * na, ba[2] * na}}, c2[1][3] = {{bb[0] * nb, bb[1] * nb, bb[2] * nb}};
    const double p0[1][2] = {{pa[0], pa[1]}}, p1[1][2] = {{pb[0], pb[1]}};
    const double dd0[1] = {D.d0[i]}, dd1[1] = {D.d1[i]};
    const bool use[1] = {has};
    Model poses[kPoses];
    const int np = motion_from_essential_r<1>(
        E, c1, c2, use, kPoses, [](bool okp) { return gsum16(okp ? 0 : 1) == 0; },
        [&](const Model &m, int q) {
            if (q == 0) poses[0] = m;
            if (q == 1) poses[1] = m;
        });
    const bool shift = C.use_shift != 0 && !C.scale_only, mdc = C.min_depth_constraint != 0;
#pragma unroll
    for (int j = 0; j < kPoses; ++j) {
        bool okm = false;
        Model m;
        if (j < np) { // (uniform over the group)
            m = poses[j];
            m.focal0 = m.focal1 = foc;
            okm = point_model_tail_r<1>(p0, p1, dd0, dd1, use, (double)K, foc, foc, shift, mdc, C.min_depth, m,
                                        [](double v) { return gsum16(v); });
        }
        if (r == 0) {
            const size_t q = (size_t)idx * kPtSlotStride + kPoses * k + j;
            if (okm) slots[q] = m;
            valid[q] = okm ? 1 : 0;
        }
    }
}

} // namespace
} // namespace mp
