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

// group g of the launch = root k of sample idx, root-major as pt_tail_kernel
__global__ void __launch_bounds__(64) pt_tail7_group_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                            const double *cand, const int *ncand, const int *samples,
                                                            Model *slots, int *valid) {
    constexpr int K = 7;
    const int lane = threadIdx.x % kTail;
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kTail);
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
#pragma unroll
    for (int c = 0; c < 4; ++c) good[c] = gsum8((has && recover_pose_good(rc, c, p0[0], p1[0], 1e9)) ? 1 : 0);
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
    if (lane == 0) {
        const size_t q = (size_t)idx * kPtSlotStride + k; // PtTraits<kTF>::kPosesPerRoot == 1
        if (ok) slots[q] = m;
        valid[q] = ok ? 1 : 0;
    }
}

// Calibrated tail (src/hybrid_pose_estimator.cpp:134-182) with one 8-lane group per
// (root, sample), lane j < 5 holding point j: the cheirality tests of
// motion_from_essential (AND over the group), then for each of the at most two poses
// the triangulation and depth fit with the group's sums.
__global__ void __launch_bounds__(64) pt_tail5_group_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                            const double *cand, const int *ncand, const int *samples,
                                                            Model *slots, int *valid) {
    constexpr int K = 5, kRoots = 10, kPoses = 2;
    const int lane = threadIdx.x % kTail;
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / kTail);
    const int k = gid / nlist, idx = gid - k * nlist;
    if (k >= kRoots || k >= ncand[idx]) return; // the whole group leaves together
    const int *s = samples + (size_t)list[idx] * kSampleStride;
    const bool has = lane < K;
    const int i = s[has ? lane : K - 1];
    // one point of load_cal_sample: calibrated ray, unit bearings, depth priors
    const double xa[3] = {D.x0u[i], D.x0v[i], 1.0}, xb[3] = {D.x1u[i], D.x1v[i], 1.0};
    double a[3], c[3];
    matvec3(C.K0i, xa, a);
    matvec3(C.K1i, xb, c);
    const double na = 1.0 / sqrt(dot3(a, a)), nc = 1.0 / sqrt(dot3(c, c));
    const double b1[1][3] = {{a[0] * na, a[1] * na, a[2] * na}}, b2[1][3] = {{c[0] * nc, c[1] * nc, c[2] * nc}};
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
                                       [](double v) { return gsum8(v); });
        }
        if (lane == 0) {
            const size_t q = (size_t)idx * kPtSlotStride + kPoses * k + j;
            if (ok) slots[q] = m;
            valid[q] = ok ? 1 : 0;
        }
    }
}

} // namespace
} // namespace mp
