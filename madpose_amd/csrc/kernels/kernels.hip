// HIP kernels of the MI355X hybrid-RANSAC engine (gfx950, wave64).
//
//  prep_pair          per-pair bearing norms (once per pair)
//  md_exact<V, R>     MD minimal solvers with the oracle's arithmetic, R lanes per
//                     sample (side stream); md_solve<V, ALT> keeps one sample per lane
//                     for the option-gated paths (scale-only, no shift, alternates)
//  pt_solve<V>        point minimal solvers in stages: root stage (group_5pt.h /
//                     group_6pt.h / lane 7pt), tails per root (group_tail.h),
//                     compaction into model slots
//  score_batch<V>     THE hot loop: one workgroup per RANSAC iteration; each lane owns
//                     correspondences i = lane, lane+256, ...; all models of the
//                     iteration are scored from registers with model constants read
//                     through the scalar cache; MSAC sums reduced in-wave (DPP shuffles)
//                     and across the 4 waves in LDS in a fixed order (deterministic);
//                     the workgroup also performs GetBestEstimatedModelId's argmin.
//  sweep<V>           one model, all points (the C ABI's explicit sweeps; LO sweeps
//                     run on the host, host/lo_sweep.h)
#include <cfloat>
#include <cstdlib>
#include <cstring>
#include <algorithm>

#include "../include/mp_md_alt.h"
#include "../include/mp_md_exact.h"
#include "../include/mp_score.h"
#include "group_5pt.h"
#include "group_tail.h"
#include "eig6.h"
#include "eig6_defl_grp.h"
#include "lm_device.h"
#include "kernels.h"
#include "../host/env.h"

namespace mp {

namespace {

constexpr int kBlock = 256;

// Sum over the 64 lanes of a wave (all lanes active), returned uniformly: DPP
// butterflies inside each 16-lane row (every lane of a row ends with the same row
// sum), then the four row sums read out by v_readlane and added in a fixed order --
// no LDS permutes (ds_bpermute) and no lane-index arithmetic; deterministic.
__device__ inline double wave_sum(double v) {
    v += dpp_d<dpp::kXor1>(v);
    v += dpp_d<dpp::kXor2>(v);
    v += dpp_d<dpp::kHalfMirror>(v);
    v += dpp_d<dpp::kMirror>(v);
    const long long bits = __double_as_longlong(v);
    const int lo = (int)(bits & 0xffffffffLL), hi = (int)(bits >> 32);
    auto row = [&](int l) {
        const unsigned a = (unsigned)__builtin_amdgcn_readlane(lo, l), b = (unsigned)__builtin_amdgcn_readlane(hi, l);
        return __longlong_as_double((long long)(((unsigned long long)b << 32) | a));
    };
    return (row(0) + row(16)) + (row(32) + row(48));
}

__device__ inline Corr load_corr(const PairConst &C, const PairData &D, int i, bool cal) {
    Corr p;
    p.x0u = D.x0u[i];
    p.x0v = D.x0v[i];
    p.x1u = D.x1u[i];
    p.x1v = D.x1v[i];
    p.d0 = D.d0[i];
    p.d1 = D.d1[i];
    p.r0 = cal ? D.r0[i] : 0.0;
    p.r1 = cal ? D.r1[i] : 0.0;
    if (cal) corr_rays(C, p);
    return p;
}

__device__ inline double msac(double e, double thr, double w) { return ((thr < e) ? thr : e) * w; }
// the score kernel's term: min(e, thr) w by the hardware minimum (two instructions
// instead of a compare, a product and two selects).  It differs from msac only for
// e = NaN (std::min keeps the NaN, the hardware minimum returns thr), and every NaN
// error of the kernel's residuals comes with a flag (eval_corr*), so its iteration is
// decided on the host's reference-order sums
__device__ inline double msac_min(double e, double thr, double w) {
    // (v_min_f64 directly: fmin() would canonicalize both operands first, two more
    // instructions per term)
    double m;
    asm("v_min_f64 %0, %1, %2" : "=v"(m) : "v"(e), "s"(thr));
    return m * w;
}

__global__ void prep_pair_kernel(PairConst C, PairData D, double *r0, double *r1, double *ra0, double *ra1,
                                 double *rb0, double *rb1) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const double xa[3] = {D.x0u[i], D.x0v[i], 1.0}, xb[3] = {D.x1u[i], D.x1v[i], 1.0};
    double a[3], b[3];
    matvec3(C.K0i, xa, a);
    matvec3(C.K1i, xb, b);
    r0[i] = 1.0 / sqrt(dot3(a, a));
    r1[i] = 1.0 / sqrt(dot3(b, b));
    if (ra0) { // the rays as corr_rays forms them
        Corr p;
        p.x0u = xa[0];
        p.x0v = xa[1];
        p.x1u = xb[0];
        p.x1v = xb[1];
        p.r0 = p.r1 = 1.0;
        corr_rays(C, p);
        ra0[i] = p.a0;
        ra1[i] = p.a1;
        rb0[i] = p.b0;
        rb1[i] = p.b1;
    }
}

// the calibrated ray form's correspondence (eval_corr_cal_ray): the rays from
// prep_pair_kernel, the unit bearing n1 = b r1 (b_2 = 1); x and n0 are not read
__device__ inline Corr load_corr_ray(const PairData &D, int i) {
    Corr p;
    p.x0u = p.x0v = p.x1u = p.x1v = 0.0;
    p.d0 = D.d0[i];
    p.d1 = D.d1[i];
    p.r0 = D.r0[i];
    p.r1 = D.r1[i];
    p.a0 = D.a0[i];
    p.a1 = D.a1[i];
    p.b0 = D.b0[i];
    p.b1 = D.b1[i];
    p.n0[0] = p.n0[1] = p.n0[2] = 0.0;
    p.n1[0] = p.b0 * p.r1;
    p.n1[1] = p.b1 * p.r1;
    p.n1[2] = p.r1;
    return p;
}

// estimator-level min-depth filter of the MD branch (src/hybrid_pose_estimator.cpp:80-85)
__device__ inline bool md_accept(const PairConst &C, Model &m) {
    if (!C.min_depth_constraint || (m.offset0 > -C.min_depth[0] && m.offset1 > -C.min_depth[1] * m.scale)) {
        m.offset1 /= m.scale;
        return true;
    }
    return false;
}

__device__ inline void put_model(const PairConst &C, const Model &m, int b, int slot, int maxm, Model *models,
                                 ScoreRec *recs) {
    models[(size_t)b * maxm + slot] = m;
    ScoreRec r;
    prepare_score_rec(C, m, r);
    recs[(size_t)b * maxm + slot] = r;
}

// ALT: instantiated with the option-gated alternate solvers (use_ours / use_4p4d);
// the default instantiation leaves them out, and with them their scratch use.
template <int V, bool ALT>
__global__ void __launch_bounds__(64) md_solve_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                      const int *samples, Model *models, ScoreRec *recs, int *counts,
                                                      int maxm) {
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nlist) return;
    const int b = list[idx];
    const int *s = samples + (size_t)b * kSampleStride;
    // accepted models go straight to their slots (no per-lane model array: indexing
    // one with the running count would put it in scratch)
    int n = 0;
    auto put = [&](const Model &m) {
        if (n < maxm) put_model(C, m, b, n, maxm, models, recs);
        ++n;
    };
    if (V == kCal) {
        double x[3][3], y[3][3], dx[3], dy[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int i = s[j];
            const double xa[3] = {D.x0u[i], D.x0v[i], 1.0}, xb[3] = {D.x1u[i], D.x1v[i], 1.0};
            matvec3(C.K0i, xa, x[j]);
            matvec3(C.K1i, xb, y[j]);
            dx[j] = D.d0[i];
            dy[j] = D.d1[i];
        }
        if (C.scale_only) {
            // HybridPoseEstimatorScaleOnly::MinimalSolver (src/hybrid_pose_estimator.cpp:319-327)
            const double W[3] = {1.0, 1.0, 1.0};
            Model m;
            m.focal0 = m.focal1 = 1.0;
            scale_and_pose<3>(x, y, W, m);
            m.scale = 1.0 / m.scale;
            put(m);
        } else if (!C.use_shift) {
            Model m;
            m.focal0 = m.focal1 = 1.0;
            md_pose_noshift_cal(x, y, dx, dy, m);
            put(m);
        } else if (ALT && C.md_alt == 1) {
            Model tmp[4];
            const int ns = md_pose_cal_ours(x, y, dx, dy, tmp);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < ns && md_accept(C, tmp[k])) put(tmp[k]);
        }
    } else {
        double x[4][3], y[4][3], dx[4], dy[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = s[j];
            x[j][0] = D.x0u[i];
            x[j][1] = D.x0v[i];
            x[j][2] = 1.0;
            y[j][0] = D.x1u[i];
            y[j][1] = D.x1v[i];
            y[j][2] = 1.0;
            dx[j] = D.d0[i];
            dy[j] = D.d1[i];
        }
        if (ALT && C.md_alt != 0) {
            Model tmp[4];
            const int ns = (V == kSF) ? md_pose_sf_ours(x, y, dx, dy, tmp)
                                      : (C.md_alt == 1 ? md_pose_tf_ours(x, y, dx, dy, tmp)
                                                       : md_pose_tf_4p4d(x, y, dx, dy, tmp));
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < ns && md_accept(C, tmp[k])) put(tmp[k]);
        }
    }
    counts[b] = n < maxm ? n : maxm;
}

// The MD solvers with the oracle's arithmetic (mp_md_exact.h: setup() = system +
// sorted real roots, root() = one root's polish and filters), two layouts:
//  R = 1: one sample per lane, its roots in turn (the kernel is issue-bound, and full
//         waves paid best: 64 / 16 / 8 / 4 samples per wave gave sf 12.9 / 13.4 / 15.0 /
//         16.3 ms per pair, profiles/r04/mdx/);
//  R > 1: R lanes per sample (64 / R per wave), every lane of a group runs the sample's
//         setup (the same doubles in each) and lane r the roots r, r + R, ..., the
//         accepted models compacted in root order by a ballot per turn -- R = 4 for the
//         two-focal quartic, whose roots' polish + pose dominate a lane's serial chain
//         (165 -> 91 us per tf launch, under the 206 us point chain; tf 13.4 -> 12.8 ms
//         per pair, profiles/r04/mdx4/), R = 2 for the shared-focal octic (below).
// Accepted models go to their slots in root order.  Round 5: the calibrated MD solver
// runs this kernel too (it ran md_solve_group, a Sturm isolation on 16-lane groups,
// whose floating-point chain can lose or invent roots on wide-range samples, as it did
// for sf / tf), and the pose stage of every variant is the oracle's Procrustes with its
// Jacobi SVD (md_pose_exact), so an MD model is the oracle's to the bit.
template <int V> struct MdxSys;
template <> struct MdxSys<kCal> {
    using S = MdxCal;
    static constexpr int K = 3;
};
template <> struct MdxSys<kSF> {
    using S = MdxSF;
    static constexpr int K = 4;
};
template <> struct MdxSys<kTF> {
    using S = MdxTF;
    static constexpr int K = 4;
};

// an MD sample's inputs as the oracle forms them: calibrated rays K^-1 x (estimator.cpp
// mv3) or the normalized homogeneous points, and the depth priors
template <int V, int K>
__device__ __forceinline__ void md_sample_inputs(const PairData &D, const PairConst &C, const int *s, double (&x)[K][3],
                                                 double (&y)[K][3], double (&dx)[K], double (&dy)[K]) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int i = s[j];
        const double xa[3] = {D.x0u[i], D.x0v[i], 1.0}, xb[3] = {D.x1u[i], D.x1v[i], 1.0};
        if (V == kCal) {
            mdx::mv3_exact(C.K0i, xa, x[j]);
            mdx::mv3_exact(C.K1i, xb, y[j]);
        } else {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                x[j][q] = xa[q];
                y[j][q] = xb[q];
            }
        }
        dx[j] = D.d0[i];
        dy[j] = D.d1[i];
    }
}

// the body of workgroup `bid` (md_exact_kernel, and the fused MD + 5pt launch below)
template <int V, int R>
__device__ __forceinline__ void md_exact_body(int bid, const PairData &D, const PairConst &C, const int *list,
                                              int nlist, const int *samples, Model *models, ScoreRec *recs,
                                              int *counts, int maxm) {
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
    using Sys = typename MdxSys<V>::S;
    constexpr int K = MdxSys<V>::K, NR = Sys::NR;
    static_assert(R == 1 || R == 2 || R == 4 || R == 8, "1, 2, 4 or 8 lanes per sample");
    static_assert(NR % R == 0, "a sample's lanes take its roots in equal turns");
    __shared__ double scr[R == 1 ? NR * 64 : 1];
    const int g = threadIdx.x / R, r = threadIdx.x % R;
    const int idx = bid * (64 / R) + g;
    const bool active = idx < nlist;
    if (R == 1 && !active) return;
    const int b = list[active ? idx : nlist - 1];
    const int *s = samples + (size_t)b * kSampleStride;
    double x[K][3], y[K][3], dx[K], dy[K];
    md_sample_inputs<V, K>(D, C, s, x, y, dx, dy);
    auto accept = [&](const double (&sol)[6], Model &m) {
        m.focal0 = sol[4];
        m.focal1 = sol[5];
        return md_pose_exact<K>(x, y, dx, dy, sol, sol[4], sol[5], m) && md_accept(C, m);
    };
    if constexpr (R == 1) {
        int n = 0;
        mdx_sols<Sys>(LaneScratch{scr + threadIdx.x, 64}, x, y, dx, dy, [&](const double (&sol)[6]) {
            Model m;
            if (accept(sol, m)) {
                if (n < maxm) put_model(C, m, b, n, maxm, models, recs);
                ++n;
            }
        });
        counts[b] = n < maxm ? n : maxm;
    } else {
        Sys sys;
        double roots[NR];
        const int nr = sys.setup(x, y, dx, dy, roots);
        const int g0 = (threadIdx.x & 63) & ~(R - 1);
        int n = 0; // the sample's accepted models so far (root order: turn j, then lane r)
#pragma unroll
        for (int j = 0; j < NR / R; ++j) {
            const int q = j * R + r;
            double root = 0.0;
#pragma unroll
            for (int c = 0; c < R; ++c)
                if (c == r) root = opaque(roots[j * R + c]);
            Model m;
            double X[K][3], Y[K][3];
            bool keep = false;
            if (active && q < nr) {
                double sol[6];
                if (sys.root(root, sol)) {
                    m.focal0 = sol[4];
                    m.focal1 = sol[5];
                    // whether the solution becomes a model depends on its depths and
                    // offsets only, so the slot is known before the Procrustes
                    if (md_pose_points<K>(x, y, dx, dy, sol, sol[4], sol[5], X, Y)) {
                        m.scale = sol[2];
                        m.offset0 = sol[1];
                        m.offset1 = sol[3];
                        keep = md_accept(C, m);
                    }
                }
            }
            const unsigned long long ball = __ballot(keep);
            const unsigned long long mine = (ball >> g0) & ((1ull << R) - 1);
            const int pos = n + __popcll(mine & ((1ull << r) - 1));
            if (keep && pos < maxm) {
                mdx::procrustes<K>(X, Y, m);
                put_model(C, m, b, pos, maxm, models, recs);
            }
            n += __popcll(mine);
            if (!__any(active && (j + 1) * R < nr)) break; // (uniform) no sample of the wave has more roots
        }
        if (active && r == 0) counts[b] = n < maxm ? n : maxm;
    }
}

// ---- The exact MD solvers in two stages (round 6) ----
// md_exact_body runs a sample's setup -- the system, the resultant, its real roots by
// balance + Hessenberg QR, the longest part -- in each of its R lanes (the same doubles
// in each) before the lanes take the roots: at R = 4 the calibrated kernel issues the
// setup four times, and with big batches (16k-32k MD samples) the waves contend for the
// SIMDs (md_exact<0,4> 155 us per launch against 77 us at 8192 samples, profiles/r06).
// Stage 1 runs the setup once per sample (one lane each) and leaves the system and its
// roots in a workspace (structure of arrays: value k of sample i at ws[k * ld + i],
// coalesced); stage 2 takes one root per lane (NR lanes per sample: 4 calibrated and two
// focal, 8 shared focal), with the same per-root operations, acceptance, Procrustes and
// root-order compaction as md_exact_body -- the models are the same doubles in the same
// slots (the MD bit-exactness tests and the switch-invariance test with
// MADPOSE_MD_TWO_STAGE=0 check it).
template <int V> struct MdxWs {
    using S = typename MdxSys<V>::S;
    static constexpr int W = (int)(sizeof(S) / sizeof(double));
    static_assert(sizeof(S) % sizeof(double) == 0 && W + S::NR <= kMdWsStride, "MD workspace layout");
};

template <int V>
__device__ __forceinline__ void md_setup_body(int bid, const PairData &D, const PairConst &C, const int *list,
                                              int nlist, const int *samples, double *ws, int *ws_nr, int ld) {
    if (batch_cancelled(D.gate, D.gate_hi)) return;
    using Sys = typename MdxSys<V>::S;
    constexpr int K = MdxSys<V>::K, NR = Sys::NR, W = MdxWs<V>::W;
    const int idx = bid * 64 + (int)threadIdx.x;
    if (idx >= nlist) return;
    const int *s = samples + (size_t)list[idx] * kSampleStride;
    double x[K][3], y[K][3], dx[K], dy[K];
    md_sample_inputs<V, K>(D, C, s, x, y, dx, dy);
    Sys sys;
    double roots[NR];
    const int nr = sys.setup(x, y, dx, dy, roots);
    double buf[W];
    __builtin_memcpy(buf, &sys, sizeof(Sys));
    static_for<W>([&](auto k) { ws[(size_t)k * ld + idx] = buf[k]; });
    static_for<NR>([&](auto k) { ws[(size_t)(W + k) * ld + idx] = roots[k]; });
    ws_nr[idx] = nr;
}

template <int V>
__device__ __forceinline__ void md_root_body(int bid, const PairData &D, const PairConst &C, const int *list, int nlist,
                                             const int *samples, const double *ws, const int *ws_nr, int ld,
                                             Model *models, ScoreRec *recs, int *counts, int maxm) {
    if (batch_cancelled(D.gate, D.gate_hi)) return;
    using Sys = typename MdxSys<V>::S;
    constexpr int K = MdxSys<V>::K, NR = Sys::NR, W = MdxWs<V>::W, R = NR;
    const int g = threadIdx.x / R, r = threadIdx.x % R;
    const int idx = bid * (64 / R) + g;
    const bool active = idx < nlist;
    const int ia = active ? idx : nlist - 1;
    const int b = list[ia];
    const int *s = samples + (size_t)b * kSampleStride;
    double x[K][3], y[K][3], dx[K], dy[K];
    md_sample_inputs<V, K>(D, C, s, x, y, dx, dy);
    Sys sys;
    {
        double buf[W];
        static_for<W>([&](auto k) { buf[k] = ws[(size_t)k * ld + ia]; });
        __builtin_memcpy(&sys, buf, sizeof(Sys));
    }
    const int nr = ws_nr[ia];
    const double root = ws[(size_t)(W + r) * ld + ia];
    const int g0 = (threadIdx.x & 63) & ~(R - 1);
    Model m;
    double X[K][3], Y[K][3];
    bool keep = false;
    if (active && r < nr) {
        double sol[6];
        if (sys.root(root, sol)) {
            m.focal0 = sol[4];
            m.focal1 = sol[5];
            if (md_pose_points<K>(x, y, dx, dy, sol, sol[4], sol[5], X, Y)) {
                m.scale = sol[2];
                m.offset0 = sol[1];
                m.offset1 = sol[3];
                keep = md_accept(C, m);
            }
        }
    }
    const unsigned long long ball = __ballot(keep);
    const unsigned long long mine = (ball >> g0) & ((1ull << R) - 1);
    const int pos = __popcll(mine & ((1ull << r) - 1));
    if (keep && pos < maxm) {
        mdx::procrustes<K>(X, Y, m);
        put_model(C, m, b, pos, maxm, models, recs);
    }
    const int n = __popcll(mine);
    if (active && r == 0) counts[b] = n < maxm ? n : maxm;
}

template <int V>
__global__ void __launch_bounds__(64) md_setup_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                      const int *samples, double *ws, int *ws_nr, int ld) {
    md_setup_body<V>(blockIdx.x, D, C, list, nlist, samples, ws, ws_nr, ld);
}

template <int V>
__global__ void __launch_bounds__(64) md_root_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                     const int *samples, const double *ws, const int *ws_nr, int ld,
                                                     Model *models, ScoreRec *recs, int *counts, int maxm) {
    md_root_body<V>(blockIdx.x, D, C, list, nlist, samples, ws, ws_nr, ld, models, recs, counts, maxm);
}

template <int V, int R>
__global__ void __launch_bounds__(64) md_exact_kernel(PairData D, PairConst C, const int *list, int nlist,
                                                      const int *samples, Model *models, ScoreRec *recs, int *counts,
                                                      int maxm) {
    md_exact_body<V, R>(blockIdx.x, D, C, list, nlist, samples, models, recs, counts, maxm);
}

// The calibrated minimal solvers in one launch: workgroups [0, md_blocks) run the
// exact MD solver (4 lanes per sample), the rest the 5pt root stage.  On two streams
// the two needed a fork and a join per batch (four API calls and a cross-stream wait);
// in one grid the MD solver, the longer of the two, still overlaps the root stage, and
// the 5pt tails and the compaction follow on the same stream.
__global__ void __launch_bounds__(64) md_pt5_kernel(PairData D, PairConst C, const int *md_list, int nmd,
                                                    int md_blocks, const int *pt_list, int npt, const int *samples,
                                                    double *cand, int *ncand, int cand_stride, Model *models,
                                                    ScoreRec *recs, int *counts, int maxm) {
    if ((int)blockIdx.x < md_blocks)
        md_exact_body<kCal, 4>(blockIdx.x, D, C, md_list, nmd, samples, models, recs, counts, maxm);
    else
        pt_roots5_group_body(blockIdx.x - md_blocks, D, C, pt_list, npt, samples, cand, ncand, cand_stride);
}

// The calibrated solvers with the two-stage MD: launch 1 = the MD setups (one lane per
// sample, md_blocks workgroups) + the 5pt root stage, launch 2 = the MD roots (4 lanes per
// sample) + the 5pt tails -- the same number of launches as md_pt5 + tails.
__global__ void __launch_bounds__(64) md_setup_pt5_kernel(PairData D, PairConst C, const int *md_list, int nmd,
                                                          int md_blocks, const int *pt_list, int npt,
                                                          const int *samples, double *cand, int *ncand,
                                                          int cand_stride, double *ws, int *ws_nr, int ld) {
    if ((int)blockIdx.x < md_blocks)
        md_setup_body<kCal>(blockIdx.x, D, C, md_list, nmd, samples, ws, ws_nr, ld);
    else
        pt_roots5_group_body(blockIdx.x - md_blocks, D, C, pt_list, npt, samples, cand, ncand, cand_stride);
}

__global__ void __launch_bounds__(64) md_root_tail5_kernel(PairData D, PairConst C, const int *md_list, int nmd,
                                                           int md_blocks, const int *pt_list, int npt,
                                                           const int *samples, const double *ws, const int *ws_nr,
                                                           int ld, Model *models, ScoreRec *recs, int *counts, int maxm,
                                                           const double *cand, const int *ncand, Model *slots,
                                                           int *valid) {
    if ((int)blockIdx.x < md_blocks)
        md_root_body<kCal>(blockIdx.x, D, C, md_list, nmd, samples, ws, ws_nr, ld, models, recs, counts, maxm);
    else
        pt_tail5_group_body(blockIdx.x - md_blocks, D, C, pt_list, npt, cand, ncand, samples, slots, valid);
}

template <int K>
__device__ inline void load_uncal_sample(const PairData &D, const int *s, double (&b0)[K][3], double (&b1)[K][3],
                                         double (&p0)[K][2], double (&p1)[K][2], double (&dd0)[K], double (&dd1)[K]) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int i = s[j];
        const double a[3] = {D.x0u[i], D.x0v[i], 1.0}, c[3] = {D.x1u[i], D.x1v[i], 1.0};
        const double na = 1.0 / sqrt(dot3(a, a)), nc = 1.0 / sqrt(dot3(c, c));
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            b0[j][q] = a[q] * na;
            b1[j][q] = c[q] * nc;
        }
        p0[j][0] = a[0];
        p0[j][1] = a[1];
        p1[j][0] = c[0];
        p1[j][1] = c[1];
        dd0[j] = D.d0[i];
        dd1[j] = D.d1[i];
    }
}

// the same with the oracle's bearings to the bit (c / |c|, no FMA contraction): the
// two-focal 7pt root stage, which is the oracle's relpose_7pt operation for operation
template <int K>
__device__ inline void load_uncal_sample_x(const PairData &D, const int *s, double (&b0)[K][3], double (&b1)[K][3]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int i = s[j];
        const double a[3] = {D.x0u[i], D.x0v[i], 1.0}, c[3] = {D.x1u[i], D.x1v[i], 1.0};
        const double na = sqrt(dot3_x(a, a)), nc = sqrt(dot3_x(c, c));
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            b0[j][q] = a[q] / na;
            b1[j][q] = c[q] / nc;
        }
    }
}

// ---------------------------------------------------------------------------
// Point solvers in three stages, so that the per-root work (pose recovery, depth
// tail) runs one root per lane instead of looping inside one lane per sample:
//   pt_roots   lane per sample: polynomial system + real roots -> candidates
//              (cal: E per root; sf: null-space basis + roots u; tf: F per root)
//   pt_tail    lane per (root, sample), root-major so that waves of high root
//              indices are empty and retire at once: poses + depth tail -> slots
//   pt_compact lane per sample: valid slots in root order -> models + score records
constexpr int kCandStride = kPtCandStride; // doubles of root-stage output per point sample
constexpr int kSlotStride = kPtSlotStride; // candidate model slots per point sample

template <int V> struct PtTraits;
template <> struct PtTraits<kCal> {
    static constexpr int kRoots = 10, kPosesPerRoot = 2, K = 5;
};
template <> struct PtTraits<kSF> {
    static constexpr int kRoots = 15, kPosesPerRoot = 2, K = 6;
};
template <> struct PtTraits<kTF> {
    static constexpr int kRoots = 3, kPosesPerRoot = 1, K = 7;
};

// two-focal root stage, one lane per sample: the 7-point fundamental matrices
// (PoseLib relpose_7pt: cubic by multilinear expansion, closed-form roots; the
// oracle's relpose_7pt operation for operation, oracle/src/pt_poselib.cpp)
__global__ void __launch_bounds__(64) pt_roots7_kernel(PairData D, const int *list, int nlist, const int *samples,
                                                       double *cand, int *ncand) {
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nlist) return;
    const int *s = samples + (size_t)list[idx] * kSampleStride;
    double *out = cand + (size_t)idx * kCandStride;
    double b0[7][3], b1[7][3];
    load_uncal_sample_x<7>(D, s, b0, b1);
    double F[3][9];
    const int n = relpose_7pt_F(b0, b1, F);
    static_for<3>([&](auto K) {
        constexpr int k = decltype(K)::value;
        if (k < n)
#pragma unroll
            for (int e = 0; e < 9; ++e) out[9 * k + e] = F[k][e];
    });
    ncand[idx] = n;
}

// Compaction of a point sample's valid tail slots into its model slots, in slot
// order: one lane per slot (G lanes per sample, G >= the slot count), the kept
// slot's position from a ballot over the group, so the models' score records are
// formed in parallel instead of one after another in one lane.  Shared focal: two
// roots of the interpolated q(u) that the polish took to the same solution give the
// same pose twice; a slot equal to an earlier valid one is dropped (the first stays).
// At most maxm models are kept (the first ones).
template <int V>
__global__ void __launch_bounds__(64) pt_compact_kernel(PairConst C, const int *list, int nlist, const int *ncand,
                                                        const Model *slots, const int *valid, Model *models,
                                                        ScoreRec *recs, int *counts, int maxm, BatchGate gate) {
    if (batch_cancelled(gate.word, gate.hi)) return;
    using T = PtTraits<V>;
    constexpr int kSlots = T::kPosesPerRoot * T::kRoots;
    constexpr int G = kSlots <= 4 ? 4 : 32;
    static_assert(kSlots <= G && kSlots <= kSlotStride && 64 % G == 0, "slot group");
    const int gid = (int)((blockIdx.x * (size_t)blockDim.x + threadIdx.x) / G), q = threadIdx.x % G;
    const bool active = gid < nlist;
    const int idx = active ? gid : nlist - 1;
    const int total = T::kPosesPerRoot * min(ncand[idx], T::kRoots);
    const size_t base = (size_t)idx * kSlotStride;
    bool keep = active && q < total && valid[base + q];
    if (V == kSF && keep) {
        const Model &m = slots[base + q];
        for (int p = 0; p < q && keep; ++p) {
            if (!valid[base + p]) continue;
            const Model &o = slots[base + p];
            bool same = fabs(o.focal0 - m.focal0) <= 1e-8 * fabs(m.focal0);
            for (int e = 0; e < 9 && same; ++e) same = fabs(o.R[e] - m.R[e]) <= 1e-6;
            for (int e = 0; e < 3 && same; ++e) same = fabs(o.t[e] - m.t[e]) <= 1e-6 * (1.0 + fabs(m.t[e]));
            keep = !same;
        }
    }
    const unsigned long long ball = __ballot(keep);
    const int lane = threadIdx.x & 63, g0 = lane & ~(G - 1);
    const unsigned long long mine = (ball >> g0) & (G == 64 ? ~0ull : ((1ull << G) - 1));
    const int pos = __popcll(mine & ((1ull << q) - 1));
    if (keep && pos < maxm) put_model(C, slots[base + q], list[idx], pos, maxm, models, recs);
    if (active && q == 0) {
        const int n = __popcll(mine);
        counts[list[idx]] = n < maxm ? n : maxm;
    }
}

// FAST: score_type 0 (hybrid, no gating) and not scale-only, and for the calibrated
// variant intrinsics of the kstd shape (ray form, mp_score.h eval_corr_cal_ray);
// everything else takes the general path (runtime gating, matrix form).
//
// Screening.  The host decides every new best on reference-order sums
// (host/lo_sweep.h); this kernel's sums only screen.  Each model carries a margin T_m
// (ScoreRec::tie, mp_score.h score_margins) with |S_dev - S_ref| <= T_m unless a
// correspondence of the iteration was flagged.  Per iteration the kernel reports the
// best device score, hi = best + T_best (the best model's reference score is below it),
// lo = min_m (S_m - T_m) (no reference score of the iteration is below it), the argmin
// (first minimum wins), kSlotAmbiguous when another model's interval reaches hi, and
// kSlotUncertain when a correspondence was flagged or a sum is NaN -- then the margins
// say nothing and the host re-scores every model of the iteration.
//
// Exact early exit (`best`: the best minimal-model score before the batch,
// best_min_model_score of src/hybrid_ransac.h:74, 123-131).  An iteration's best score
// is only ever compared with the running best by a strict '<' (:123), the running best
// only decreases inside a batch, and every MSAC term min(e, thr) * w is >= 0 -- so a
// model whose partial device sum minus T_m already reaches `best` has a reference sum
// >= best and can never win: the rest of its sweep is skipped.  Checks run at trip
// boundaries (one trip = 256 correspondences): each live model's workgroup partial
// (wave sums, then the four waves in LDS in a fixed order -- every lane forms the same
// value, so the live mask stays uniform) is compared; the workgroup leaves once no model
// is live.  Once a flag has been seen the exit stops killing (the partial sums are then
// no bound), and a model killed earlier was killed on correspondences without flags.
// Killed models report DBL_MAX and never enter the argmin.
//
// Record skip (ScoreBound::rec, batches at or past lo_starting_iterations only): there
// every new best runs LO, which consumes the selection stream, so the host cuts the
// batch at the first iteration that holds a new best (src/hybrid_ransac.h:123-156) and
// discards every later one.  A workgroup whose hi is below `best` without a flag -- its
// iteration holds a new best in the reference order for certain -- publishes its index
// by an atomic minimum; a workgroup that sees an earlier published record at one of its
// early-exit checks (the word is read at the start and after each check, the check's
// barrier shares the verdict) stops there.  Iterations up to the first record are
// always scored in full, so the host's walk never reads a skipped one.  The word
// carries an epoch in its high half (complemented, so a new batch's first record always
// wins the minimum) and needs no reset between batches.
struct ScoreBound {
    double best;         // +inf: no early exit
    int first, every;    // first check after `first` trips, then every `every` trips
    int *work;           // per iteration: (model, trip) pairs evaluated (profiling)
    int pair;            // two trips per loop step between checks (MADPOSE_SCORE_PAIR=0: one)
    unsigned long long *rec; // nullptr: no record skip
    unsigned epoch_hi;       // ~epoch of this batch
    // record models (nullable): an iteration whose lo is below best (it could hold a new
    // best) writes its best model to rec_out[b] (mapped host memory), so the host reads
    // a new best's model without a copy round trip
    const Model *models;
    Model *rec_out;
    // the host's walk (nullable): per iteration one byte, the model count | 0x80 when the
    // iteration could hold a new best (uncertain, or lo below `best`: a superset of the
    // walk's tests, whose running best only decreases), and for those the IterResult in
    // cand_out[b] (mapped host memory) -- the walk reads B bytes, not B IterResults
    uint8_t *flags8;
    IterResult *cand_out;
};

// EXIT = false (no finite bound yet, or MADPOSE_SCORE_EXIT=0): the plain sweep,
// without the trip-boundary checks and their barriers.
//
// Five waves per SIMD asked of the compiler (FAST instances): the calibrated one
// otherwise takes 99 VGPRs (four waves); at 96 it keeps five without spilling, 50.9 ->
// 47.9 us per launch (sf and tf already fit five / seven; profiles/r05/occ).  The
// general path would spill under the same request and is left alone.
template <int V, int MAXM, bool FAST, bool EXIT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FAST ? 5 : 1)))
score_batch_kernel(PairData D, PairConst C, const ScoreRec *__restrict__ recs, const int *__restrict__ counts,
                   double *scores, IterResult *res, ScoreBound sb) {
    if (batch_cancelled(D.gate, D.gate_hi)) return; // (uniform: the record word is read by every lane)
    const int b = blockIdx.x;
    const int nm = counts[b];
    if (nm == 0) {
        if (threadIdx.x == 0) {
            res[b] = IterResult{DBL_MAX, DBL_MAX, DBL_MAX, 0, 0};
            if (sb.work) sb.work[b] = 0;
            if (sb.flags8) sb.flags8[b] = 0;
        }
        return;
    }
    // the record word, read at the start and decided on at the early-exit checks (their
    // barrier publishes thread 0's verdict), so the load's latency hides behind the
    // first trips instead of stalling the workgroup at entry; reloaded after each check
    unsigned long long recw = ~0ull;
    if (EXIT && sb.rec && threadIdx.x == 0) recw = __hip_atomic_load(sb.rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __shared__ int s_skip[2];
    __shared__ int s_flag[2][kBlock / 64];
    bool skipped = false;
    bool flag = false;       // this lane met a flagged correspondence
    bool uncertain = false;  // (uniform) the workgroup did, as of the last check
    const ScoreRec *R = recs + (size_t)b * MAXM;
    double acc[MAXM];
#pragma unroll
    for (int m = 0; m < MAXM; ++m) acc[m] = 0.0;
    const double t0 = C.thr[0], t1 = C.thr[1], t2 = C.thr[2];
    const double w0 = C.w[0], w1 = C.w[1], w2 = C.w[2];
    __shared__ double part[2][kBlock / 64][MAXM];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned live = (nm >= 32) ? ~0u : ((1u << nm) - 1u); // uniform
    int checks = 0, work = 0;
    const int ntrip = (C.n + kBlock - 1) / kBlock;
    if (!EXIT) {
        for (int i = threadIdx.x; i < C.n; i += kBlock) {
            Corr p = (FAST && V == kCal) ? load_corr_ray(D, i) : load_corr(C, D, i, V == kCal);
#pragma unroll
            for (int m = 0; m < MAXM; ++m) {
                if (m < nm) {
                    double e0, e1, e2;
                    if (FAST && V == kCal)
                        eval_corr_cal_ray(C, R[m], p, e0, e1, e2, flag);
                    else
                        eval_corr<V>(C, R[m], p, !FAST, e0, e1, e2, flag);
                    acc[m] += msac_min(e0, t0, w0) + msac_min(e1, t1, w1) + msac_min(e2, t2, w2);
                }
            }
        }
        work = nm * ntrip;
    }
    // the trip loop over the first NM model slots: a separate instance for iterations with
    // one model (most of them), whose model constants then stay in scalar registers
    // across the trips instead of being reloaded with every trip
    // a check follows `done` trips
    auto check_after = [&](int done) { return done < ntrip && done >= sb.first && (done - sb.first) % sb.every == 0; };
    auto trips = [&](auto nmc) {
        constexpr int NM = decltype(nmc)::value;
        for (int trip = 0; EXIT && trip < ntrip;) {
            // two trips at once where no check falls between them (sb.pair): both
            // correspondences' loads are in flight together, and each model's constants
            // serve two evaluations
            const int step = (sb.pair && trip + 1 < ntrip && !check_after(trip + 1)) ? 2 : 1;
            const int i = trip * kBlock + threadIdx.x, i2 = i + kBlock;
            const bool has = i < C.n, has2 = step == 2 && i2 < C.n;
            Corr p, p2;
            if (has) p = (FAST && V == kCal) ? load_corr_ray(D, i) : load_corr(C, D, i, V == kCal);
            if (has2) p2 = (FAST && V == kCal) ? load_corr_ray(D, i2) : load_corr(C, D, i2, V == kCal);
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                if ((live >> m) & 1u) {
                    if (has) {
                        double e0, e1, e2;
                        if (FAST && V == kCal)
                            eval_corr_cal_ray(C, R[m], p, e0, e1, e2, flag);
                        else
                            eval_corr<V>(C, R[m], p, !FAST, e0, e1, e2, flag);
                        acc[m] += msac_min(e0, t0, w0) + msac_min(e1, t1, w1) + msac_min(e2, t2, w2);
                    }
                    if (has2) {
                        double e0, e1, e2;
                        if (FAST && V == kCal)
                            eval_corr_cal_ray(C, R[m], p2, e0, e1, e2, flag);
                        else
                            eval_corr<V>(C, R[m], p2, !FAST, e0, e1, e2, flag);
                        acc[m] += msac_min(e0, t0, w0) + msac_min(e1, t1, w1) + msac_min(e2, t2, w2);
                    }
                }
            }
            work += __popc(live) * step;
            trip += step;
            const int done = trip;
            if (check_after(done)) {
                const int par = checks & 1; // double-buffered: one barrier per check
                if (threadIdx.x == 0) {
                    s_skip[par] = (unsigned)(recw >> 32) == sb.epoch_hi && (int)(unsigned)(recw & 0xffffffffu) < b;
                    if (sb.rec) recw = __hip_atomic_load(sb.rec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
#pragma unroll
                for (int m = 0; m < NM; ++m) {
                    if ((live >> m) & 1u) {
                        const double v = wave_sum(acc[m]);
                        if (lane == 0) part[par][wave][m] = v;
                    }
                }
                const bool wf = __any(flag);
                if (lane == 0) s_flag[par][wave] = wf;
                __syncthreads();
#pragma unroll
                for (int w = 0; w < kBlock / 64; ++w) uncertain = uncertain || s_flag[par][w] != 0;
                unsigned keep = live;
                if (!uncertain) {
#pragma unroll
                    for (int m = 0; m < NM; ++m) {
                        if ((live >> m) & 1u) {
                            double v = 0.0;
#pragma unroll
                            for (int w = 0; w < kBlock / 64; ++w) v += part[par][w][m];
                            if (v - R[m].tie >= sb.best) keep &= ~(1u << m);
                        }
                    }
                }
                live = __builtin_amdgcn_readfirstlane(keep);
                if (s_skip[par]) { // (uniform) a record earlier in the batch: this iteration is discarded
                    live = 0;
                    skipped = true;
                }
                ++checks;
                if (live == 0) break;
            }
        }
    };
    if (nm == 1)
        trips(std::integral_constant<int, 1>());
    else
        trips(std::integral_constant<int, MAXM>());
    const int par = checks & 1;
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
        if ((live >> m) & 1u) {
            const double v = wave_sum(acc[m]);
            if (lane == 0) part[par][wave][m] = v;
        }
    }
    {
        const bool wf = __any(flag);
        if (lane == 0) s_flag[par][wave] = wf;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) uncertain = uncertain || s_flag[par][w] != 0;
        double bs = DBL_MAX; // best score
        int bi = 0;
        double sc[MAXM];
#pragma unroll
        for (int m = 0; m < MAXM; ++m) {
            double v = DBL_MAX; // killed (or absent): cannot win
            if (m < nm && ((live >> m) & 1u)) {
                v = 0.0;
#pragma unroll
                for (int w = 0; w < kBlock / 64; ++w) v += part[par][w][m];
                uncertain = uncertain || v != v;
            }
            sc[m] = v;
            if (m < nm) {
                scores[(size_t)b * MAXM + m] = v;
                if (v < bs) { // strict '<': first minimum wins (src/hybrid_ransac.h:258)
                    bs = v;
                    bi = m;
                }
            }
        }
        // hi: the best's reference score is below it; lo: no model's is below it; a
        // model other than the best whose interval reaches hi could be the reference's
        // first minimum instead
        double Tb = 0.0;
#pragma unroll
        for (int m = 0; m < MAXM; ++m)
            if (m == bi) Tb = R[m].tie;
        const double hi = bs < DBL_MAX ? bs + Tb : DBL_MAX;
        double lo = DBL_MAX;
        bool amb = false;
#pragma unroll
        for (int m = 0; m < MAXM; ++m) {
            if (m < nm && sc[m] < DBL_MAX) {
                const double l = sc[m] - R[m].tie;
                lo = l < lo ? l : lo;
                amb = amb || (m != bi && l <= hi);
            }
        }
        const int flags = (amb ? kSlotAmbiguous : 0) | (uncertain ? kSlotUncertain : 0);
        const IterResult out = skipped ? IterResult{DBL_MAX, DBL_MAX, DBL_MAX, 0, nm} : IterResult{bs, hi, lo, bi | flags, nm};
        res[b] = out;
        // (a record-skipped iteration reports its trips negated: profiling only)
        if (sb.work) sb.work[b] = skipped ? -work : work;
        if (sb.rec && !skipped && !uncertain && hi < sb.best)
            atomicMin(sb.rec, ((unsigned long long)sb.epoch_hi << 32) | (unsigned long long)(unsigned)b);
        const bool cand = !skipped && (uncertain || lo < sb.best);
        if (sb.flags8) sb.flags8[b] = (uint8_t)(nm | (cand ? 0x80 : 0));
        if (cand && sb.cand_out) sb.cand_out[b] = out;
        if (sb.rec_out && cand) {
            const double *src = (const double *)(sb.models + (size_t)b * MAXM + bi);
            double *dst = (double *)(sb.rec_out + b);
#pragma unroll
            for (int q = 0; q < (int)(sizeof(Model) / sizeof(double)); ++q) dst[q] = src[q];
        }
    }
}

// score_batch's residuals of explicit models, per correspondence, with the flag of
// each (mp_debug_score_terms; a test hook of the screening margins): one workgroup per
// model, the same load and evaluation as score_batch (FAST: the ray form)
template <int V, bool FAST>
__global__ void __launch_bounds__(kBlock) debug_terms_kernel(PairData D, PairConst C, const ScoreRec *recs,
                                                             double *err, int *flags) {
    const ScoreRec &r = recs[blockIdx.x];
    double *e = err + (size_t)blockIdx.x * 3 * C.n;
    for (int i = threadIdx.x; i < C.n; i += kBlock) {
        const Corr p = (FAST && V == kCal) ? load_corr_ray(D, i) : load_corr(C, D, i, V == kCal);
        double e0, e1, e2;
        bool flag = false;
        if (FAST && V == kCal)
            eval_corr_cal_ray(C, r, p, e0, e1, e2, flag);
        else
            eval_corr<V>(C, r, p, !FAST, e0, e1, e2, flag);
        e[i] = e0;
        e[C.n + i] = e1;
        e[2 * C.n + i] = e2;
        flags[(size_t)blockIdx.x * C.n + i] = flag ? 1 : 0;
    }
}

template <int V>
__global__ void __launch_bounds__(1024) sweep_kernel(PairData D, PairConst C, const ScoreRec *rec, double *err,
                                                     double *score) {
    const ScoreRec r = *rec;
    double acc = 0.0;
    const bool gate_md = C.score_type == 1, gate_epi = C.score_type == 2;
    for (int i = threadIdx.x; i < C.n; i += blockDim.x) {
        const Corr p = load_corr(C, D, i, V == kCal);
        double e0, e1, e2;
        bool flag = false; // (unused: an explicit sweep screens nothing)
        eval_corr<V>(C, r, p, false, e0, e1, e2, flag);
        err[i] = e0;
        err[C.n + i] = e1;
        err[2 * C.n + i] = e2;
        acc += gate_md ? C.thr[0] * C.w[0] + C.thr[1] * C.w[1] : msac(e0, C.thr[0], C.w[0]) + msac(e1, C.thr[1], C.w[1]);
        acc += gate_epi ? C.thr[2] * C.w[2] : msac(e2, C.thr[2], C.w[2]);
    }
    __shared__ double part[16];
    const double v = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
        *score = s;
    }
}

template <int V>
__global__ void __launch_bounds__(kBlock) score_models_kernel(PairData D, PairConst C, const ScoreRec *recs,
                                                              double *scores) {
    const ScoreRec r = recs[blockIdx.x];
    double acc = 0.0;
    for (int i = threadIdx.x; i < C.n; i += kBlock) {
        const Corr p = load_corr(C, D, i, V == kCal);
        double e0, e1, e2;
        bool flag = false;
        eval_corr<V>(C, r, p, true, e0, e1, e2, flag);
        acc += msac(e0, C.thr[0], C.w[0]) + msac(e1, C.thr[1], C.w[1]) + msac(e2, C.thr[2], C.w[2]);
    }
    __shared__ double part[kBlock / 64];
    const double v = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < kBlock / 64; ++w) s += part[w];
        scores[blockIdx.x] = s;
    }
}

__global__ void md_direct_kernel(int variant, int alt, const double *in, double *sols_out, int *nsols, Model *poses,
                                 int *nposes) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (variant == kCal && alt != 0) {
        double x[3][3], y[3][3], dx[3], dy[3];
        for (int j = 0; j < 3; ++j) {
            for (int c = 0; c < 3; ++c) {
                x[j][c] = in[3 * j + c];
                y[j][c] = in[9 + 3 * j + c];
            }
            dx[j] = in[18 + j];
            dy[j] = in[21 + j];
        }
        *nposes = *nsols = md_pose_cal_ours(x, y, dx, dy, poses);
        return;
    }
    if (variant != kCal && alt != 0) {
        double x[4][3], y[4][3], dx[4], dy[4];
        for (int j = 0; j < 4; ++j) {
            for (int c = 0; c < 3; ++c) {
                x[j][c] = in[3 * j + c];
                y[j][c] = in[12 + 3 * j + c];
            }
            dx[j] = in[24 + j];
            dy[j] = in[28 + j];
        }
        *nposes = *nsols = (variant == kSF) ? md_pose_sf_ours(x, y, dx, dy, poses)
                                            : (alt == 1 ? md_pose_tf_ours(x, y, dx, dy, poses)
                                                        : md_pose_tf_4p4d(x, y, dx, dy, poses));
        return;
    }
    if (variant == kCal) {
        double x[3][3], y[3][3], dx[3], dy[3];
        for (int j = 0; j < 3; ++j) {
            for (int c = 0; c < 3; ++c) {
                x[j][c] = in[3 * j + c];
                y[j][c] = in[9 + 3 * j + c];
            }
            dx[j] = in[18 + j];
            dy[j] = in[21 + j];
        }
        double sols[4][6], scr[kMdxScratchCal];
        int ns = 0;
        mdx_sols_cal(LaneScratch{scr, 1}, x, y, dx, dy, [&](const double (&sol)[6]) {
            for (int c = 0; c < 6; ++c) sols[ns][c] = sol[c];
            ++ns;
        });
        int np = 0;
        for (int k = 0; k < ns; ++k) {
            for (int c = 0; c < 4; ++c) sols_out[4 * k + c] = sols[k][c];
            Model m;
            m.focal0 = m.focal1 = 1.0;
            if (md_pose_exact<3>(x, y, dx, dy, sols[k], 1.0, 1.0, m)) poses[np++] = m;
        }
        *nsols = ns;
        *nposes = np;
        return;
    }
    double x[4][3], y[4][3], dx[4], dy[4];
    for (int j = 0; j < 4; ++j) {
        for (int c = 0; c < 3; ++c) {
            x[j][c] = in[3 * j + c];
            y[j][c] = in[12 + 3 * j + c];
        }
        dx[j] = in[24 + j];
        dy[j] = in[28 + j];
    }
    double sols[8][6], scr[kMdxScratchSF];
    int ns = 0;
    auto keep = [&](const double (&sol)[6]) {
        for (int c = 0; c < 6; ++c) sols[ns][c] = sol[c];
        ++ns;
    };
    const LaneScratch W{scr, 1};
    if (variant == kSF)
        mdx_sols_sf(W, x, y, dx, dy, keep);
    else
        mdx_sols_tf(W, x, y, dx, dy, keep);
    const int w = (variant == kSF) ? 5 : 6;
    int np = 0;
    for (int k = 0; k < ns; ++k) {
        for (int c = 0; c < w; ++c) sols_out[w * k + c] = sols[k][c];
        Model m;
        const double fa = sols[k][4], fb = (variant == kSF) ? sols[k][4] : sols[k][5];
        m.focal0 = fa;
        m.focal1 = fb;
        if (md_pose_exact<4>(x, y, dx, dy, sols[k], fa, fb, m)) poses[np++] = m;
    }
    *nsols = ns;
    *nposes = np;
}

// standalone point solvers (test hooks): kind 0 = 5pt on unit bearings (5 + 5 x 3
// doubles); kind 2 = two-focal 7pt + Bougnoux + recoverPose on normalized 2-D points
// (K + K x 2 doubles) turned into bearings exactly as the estimator does (the
// shared-focal 6pt runs the estimator's staged root stage, engine.cpp
// solve_point_direct).  Models are returned before the depth fit.
__global__ void point_direct_kernel(int kind, const double *in, Model *poses, int *nposes) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (kind == 0) {
        *nposes = 0; // (launch_point_direct runs the 5pt through the estimator's root stage)
    } else {
        double b0[7][3], b1[7][3], p0[7][2], p1[7][2];
        for (int j = 0; j < 7; ++j) {
            const double a[3] = {in[2 * j], in[2 * j + 1], 1.0}, c[3] = {in[14 + 2 * j], in[14 + 2 * j + 1], 1.0};
            const double na = 1.0 / sqrt(dot3(a, a)), nc = 1.0 / sqrt(dot3(c, c));
            for (int q = 0; q < 3; ++q) {
                b0[j][q] = a[q] * na;
                b1[j][q] = c[q] * nc;
            }
            p0[j][0] = a[0];
            p0[j][1] = a[1];
            p1[j][0] = c[0];
            p1[j][1] = c[1];
        }
        double F[3][9];
        const int nf = relpose_7pt_F(b0, b1, F);
        for (int k = 0; k < nf; ++k) {
            double f0, f1;
            bougnoux_sq(F[k], &f0, &f1);
            f0 = sqrt(fabs(f0));
            f1 = sqrt(fabs(f1));
            double E[9];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) E[3 * r + c] = (r < 2 ? f1 : 1.0) * F[k][3 * r + c] * (c < 2 ? f0 : 1.0);
            Model m;
            recover_pose_cv<7>(E, p0, p1, 1e9, m.R, m.t);
            m.scale = 1.0;
            m.offset0 = m.offset1 = 0.0;
            m.focal0 = f0;
            m.focal1 = f1;
            poses[k] = m;
        }
        *nposes = nf;
    }
}

// estimate_scale_and_pose (src/solver.cpp:5-33) for an arbitrary number of points
__global__ void scale_and_pose_kernel(const double *in, int64_t n, Model *out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const double *X = in, *Y = in + 3 * n, *W = in + 6 * n;
    double ws = 0.0, cx[3] = {0, 0, 0}, cy[3] = {0, 0, 0};
    for (int64_t i = 0; i < n; ++i) {
        ws += W[i];
        for (int c = 0; c < 3; ++c) {
            cx[c] += X[3 * i + c] * W[i];
            cy[c] += Y[3 * i + c] * W[i];
        }
    }
    for (int c = 0; c < 3; ++c) {
        cx[c] /= ws;
        cy[c] /= ws;
    }
    double Mx[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int64_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) Mx[a][b] += (X[3 * i + a] - cx[a]) * W[i] * (Y[3 * i + b] - cy[b]);
    Model m;
    horn_rotation(Mx, m.R);
    double num = 0.0, den = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        const double xc[3] = {X[3 * i] - cx[0], X[3 * i + 1] - cx[1], X[3 * i + 2] - cx[2]};
        double rx[3];
        matvec3(m.R, xc, rx);
        for (int c = 0; c < 3; ++c) {
            num += (Y[3 * i + c] - cy[c]) * rx[c];
            den += rx[c] * rx[c];
        }
    }
    m.scale = num / den;
    double rc[3];
    matvec3(m.R, cx, rc);
    for (int c = 0; c < 3; ++c) m.t[c] = cy[c] - m.scale * rc[c];
    m.offset0 = m.offset1 = 0.0;
    m.focal0 = m.focal1 = 1.0;
    *out = m;
}

template <class F> hipError_t by_variant(int v, F f) {
    if (v == kCal) return f(std::integral_constant<int, kCal>());
    if (v == kSF) return f(std::integral_constant<int, kSF>());
    return f(std::integral_constant<int, kTF>());
}

} // namespace

hipError_t launch_prep_pair(hipStream_t s, const PairConst &C, const PairData &D, double *r0, double *r1, double *a0,
                            double *a1, double *b0, double *b1) {
    if (C.n <= 0) return hipSuccess;
    const bool rays = C.variant == kCal && a0 && a1 && b0 && b1;
    prep_pair_kernel<<<(C.n + 255) / 256, 256, 0, s>>>(C, D, r0, r1, rays ? a0 : nullptr, a1, b0, b1);
    return hipGetLastError();
}

// the default MD solvers (shift on, no alternates) run md_exact
static bool md_plain(const PairConst &C) {
    return C.md_alt == 0 && (C.variant != kCal || (!C.scale_only && C.use_shift));
}
// Where the two-stage exact MD (md_setup + md_root) runs: MADPOSE_MD_TWO_STAGE = 1 (the
// default) in the fused calibrated launch only, 2 in every MD launch, 0 nowhere;
// MADPOSE_MDX_R (the one-stage kernel at R lanes per sample, A/B) turns it off.  Measured
// (profiles/r06/md2): fused calibrated batches md_pt5 86 + tail 23 -> md_setup_pt5 74 +
// md_root_tail5 22 us; the unfused ones gain nothing -- the setup with one lane per sample
// takes 123 us at 16k-32k samples against md_exact<0,4>'s 155 us with the 36 us root stage
// after it: a wave's setup lasts as long as the slowest of its 64 samples' QR trips, where
// four lanes per sample wait for the slowest of 16 -- and the shared-focal setup spills
// (310 VGPRs, 144 B scratch; 252 + 82 against 311 us)
static int md_two_stage_mode() {
    static const int mode = env_int("MADPOSE_MDX_R", 0, 0, 4) != 0 ? 0 : (int)env_int("MADPOSE_MD_TWO_STAGE", 1, 0, 2);
    return mode;
}
static bool md_two_stage() { return md_two_stage_mode() >= 1; }
// md_exact's lanes per sample (MADPOSE_MDX_R=1|2|4 overrides the default)
static int md_lanes(int v) {
    static const int r_env = [] {
        const int r = (int)env_int("MADPOSE_MDX_R", 0, 0, 4);
        if (r == 3) env_reject("MADPOSE_MDX_R", "3", "expected 1, 2 or 4");
        return r;
    }();
    return (r_env == 1 || r_env == 2 || r_env == 4) ? r_env : (v == kSF ? 2 : 4);
}

hipError_t launch_md_solve(hipStream_t s, const PairData &D, const PairConst &C, const int *list, int nlist,
                           const int *samples, Model *models, ScoreRec *recs, int *counts, int maxm) {
    if (nlist <= 0) return hipSuccess;
    const int grid = (nlist + 63) / 64;
    return by_variant(C.variant, [&](auto V) {
        constexpr int v = decltype(V)::value;
        // the default solvers (shift on, no alternates): md_exact, R lanes per sample.
        // sf: two lanes per sample (the kernel 267 -> 212 us per launch, sf gpu_solve 8.17
        // -> 7.74 ms per pair; 4 and 8 lanes shortened it further, 190 / 230 us, but
        // their extra waves slowed the point chain beside it, pt_defl6_grp 80 -> 105 /
        // 124 us, profiles/r04/mdxr/); tf and cal: one lane per root.
        // MADPOSE_MDX_R=1|2|4 overrides (results are the same: a lane's arithmetic never
        // depends on the others; tests/test_switch_invariance_gpu.py)
        if (md_plain(C)) {
            const int r = md_lanes(v);
            if (r == 1)
                md_exact_kernel<v, 1><<<grid, 64, 0, s>>>(D, C, list, nlist, samples, models, recs, counts, maxm);
            else if (r == 2)
                md_exact_kernel<v, 2><<<(nlist + 31) / 32, 64, 0, s>>>(D, C, list, nlist, samples, models, recs,
                                                                       counts, maxm);
            else
                md_exact_kernel<v, 4><<<(nlist + 15) / 16, 64, 0, s>>>(D, C, list, nlist, samples, models, recs,
                                                                       counts, maxm);
            return hipGetLastError();
        }
        // scale-only / no-shift (calibrated) and the use_ours / use_4p4d alternates
        if (C.md_alt != 0)
            md_solve_kernel<decltype(V)::value, true><<<grid, 64, 0, s>>>(D, C, list, nlist, samples, models, recs,
                                                                          counts, maxm);
        else
            md_solve_kernel<decltype(V)::value, false><<<grid, 64, 0, s>>>(D, C, list, nlist, samples, models, recs,
                                                                           counts, maxm);
        return hipGetLastError();
    });
}

hipError_t launch_md_solve_staged(hipStream_t s, const PairData &D, const PairConst &C, const int *list, int nlist,
                                  const int *samples, const PtWorkspace &W, Model *models, ScoreRec *recs,
                                  int *counts, int maxm) {
    if (nlist <= 0) return hipSuccess;
    if (!W.md_ws || md_two_stage_mode() < 2 || !md_plain(C))
        return launch_md_solve(s, D, C, list, nlist, samples, models, recs, counts, maxm);
    if (nlist > W.md_ld) return hipErrorInvalidValue;
    return by_variant(C.variant, [&](auto V) {
        constexpr int v = decltype(V)::value;
        constexpr int spw = 64 / MdxSys<v>::S::NR; // samples per workgroup of the root stage
        md_setup_kernel<v><<<(nlist + 63) / 64, 64, 0, s>>>(D, C, list, nlist, samples, W.md_ws, W.md_nr, W.md_ld);
        md_root_kernel<v><<<(nlist + spw - 1) / spw, 64, 0, s>>>(D, C, list, nlist, samples, W.md_ws, W.md_nr,
                                                                W.md_ld, models, recs, counts, maxm);
        return hipGetLastError();
    });
}

// the shared-focal root stage by the deflated eigenproblem: the pencil (16-lane groups,
// eig6.h), its deflation + balance + Hessenberg form (16-lane groups, eig6_defl_grp.h),
// then the lockstep Francis QR (one sample per lane, eig6.h / eig15_gen.h)
// samples per wave of the lockstep QR: at most 768 waves, three quarters of the SIMDs,
// since the shared-focal MD kernel holds SIMDs beside it (768 / 640 against 1024 and
// 1536: sf gpu_solve 7.33 against 7.56 / 8.30 ms per pair, profiles/r06/eig_waves;
// MADPOSE_EIG_WAVES overrides, MADPOSE_EIG_WAVES=16 packs 64 samples per wave at 1024)
int eig_spw(int nlist) {
    static const int waves = [] {
        return (int)env_int("MADPOSE_EIG_WAVES", 768, 1, 1 << 20);
    }();
    return std::min(64, std::max(1, (nlist + waves - 1) / waves));
}

static void launch_sf_eig(hipStream_t s, const PairData &D, const int *list, int nlist, const int *samples,
                          double *cand, int *ncand, double *pen) {
    pt_pencil6_kernel<<<(nlist + kGrpPerWg - 1) / kGrpPerWg, 64, 0, s>>>(D, list, nlist, samples, cand, kCandStride,
                                                                         pen);
    const BatchGate gate{D.gate, D.gate_hi};
    pt_defl6_grp_kernel<<<(nlist + 3) / 4, 64, 0, s>>>(pen, nlist, gate);
    const int spw = eig_spw(nlist);
    if (spw == 1)
        pt_eig6_reg_kernel<true><<<nlist, 64, 0, s>>>(pen, nlist, 1, cand, ncand, kCandStride, gate);
    else
        pt_eig6_reg_kernel<false><<<(nlist + spw - 1) / spw, 64, 0, s>>>(pen, nlist, spw, cand, ncand, kCandStride,
                                                                         gate);
}

bool solve_fusable(const PairConst &C) {
    static const bool off = [] {
        return !env_flag("MADPOSE_SOLVE_FUSE", true);
    }();
    return !off && C.variant == kCal && md_plain(C) && md_lanes(kCal) == 4;
}

hipError_t launch_solve_fused(hipStream_t s, const PairData &D, const PairConst &C, const int *md_list, int nmd,
                              const int *pt_list, int npt, const int *samples, const PtWorkspace &W, Model *models,
                              ScoreRec *recs, int *counts, int maxm) {
    if (!solve_fusable(C)) return hipErrorInvalidValue;
    if (W.md_ws && md_two_stage()) {
        if (nmd > W.md_ld) return hipErrorInvalidValue;
        // launch 1: MD setups (one lane per sample) + 5pt roots; launch 2: MD roots (four
        // lanes per sample) + 5pt tails; then the 5pt compaction
        const int md1 = (nmd + 63) / 64, md2 = (nmd + 15) / 16, pt_blocks = (npt + kS5 - 1) / kS5;
        const long lanes = (long)npt * PtTraits<kCal>::kRoots;
        const int tgrid = (int)((lanes * kTail + 63) / 64);
        if (md1 + pt_blocks > 0)
            md_setup_pt5_kernel<<<md1 + pt_blocks, 64, 0, s>>>(D, C, md_list, nmd, md1, pt_list, npt, samples, W.cand,
                                                               W.ncand, kCandStride, W.md_ws, W.md_nr, W.md_ld);
        if (md2 + tgrid > 0)
            md_root_tail5_kernel<<<md2 + tgrid, 64, 0, s>>>(D, C, md_list, nmd, md2, pt_list, npt, samples, W.md_ws,
                                                            W.md_nr, W.md_ld, models, recs, counts, maxm, W.cand,
                                                            W.ncand, W.slots, W.valid);
        if (npt > 0) {
            constexpr int kCompactG = 32; // (PtTraits<kCal>: 2 poses x 10 roots > 4)
            pt_compact_kernel<kCal><<<(int)(((size_t)npt * kCompactG + 63) / 64), 64, 0, s>>>(
                C, pt_list, npt, W.ncand, W.slots, W.valid, models, recs, counts, maxm, BatchGate{D.gate, D.gate_hi});
        }
        return hipGetLastError();
    }
    const int md_blocks = (nmd + 15) / 16, pt_blocks = (npt + kS5 - 1) / kS5;
    if (md_blocks + pt_blocks > 0)
        md_pt5_kernel<<<md_blocks + pt_blocks, 64, 0, s>>>(D, C, md_list, nmd, md_blocks, pt_list, npt, samples, W.cand,
                                                          W.ncand, kCandStride, models, recs, counts, maxm);
    return launch_pt_solve(s, D, C, pt_list, npt, samples, W, models, recs, counts, maxm, true);
}

hipError_t launch_pt_solve(hipStream_t s, const PairData &D, const PairConst &C, const int *list, int nlist,
                           const int *samples, const PtWorkspace &W, Model *models, ScoreRec *recs, int *counts,
                           int maxm, bool roots_done) {
    if (nlist <= 0) return hipSuccess;
    return by_variant(C.variant, [&](auto V) {
        constexpr int v = decltype(V)::value;
        // root stage: calibrated 5pt on 16-lane groups (group_5pt.h), shared-focal 6pt by
        // the deflated eigenproblem, two-focal 7pt one lane per sample
        if (roots_done)
            ; // (launched by launch_solve_fused)
        else if (v == kSF)
            launch_sf_eig(s, D, list, nlist, samples, W.cand, W.ncand, W.pen);
        else if (v == kCal)
            pt_roots5_group_kernel<<<(nlist + kS5 - 1) / kS5, 64, 0, s>>>(D, C, list, nlist, samples, W.cand, W.ncand,
                                                                          kCandStride);
        else
            pt_roots7_kernel<<<(nlist + 63) / 64, 64, 0, s>>>(D, list, nlist, samples, W.cand, W.ncand);
        // tails on lane groups per (root, sample) (group_tail.h: 8 lanes for cal / tf, 16
        // for sf), root-major so that waves of high root indices are empty and retire
        const long lanes = (long)nlist * PtTraits<v>::kRoots;
        const int tgrid = (int)((lanes * kTail + 63) / 64);
        if (v == kTF)
            pt_tail7_group_kernel<8><<<tgrid, 64, 0, s>>>(D, C, list, nlist, W.cand, W.ncand, samples, W.slots,
                                                          W.valid);
        else if (v == kCal)
            pt_tail5_group_kernel<<<tgrid, 64, 0, s>>>(D, C, list, nlist, W.cand, W.ncand, samples, W.slots, W.valid);
        else
            pt_tail6_group_kernel<<<(int)((lanes * kGrp + 63) / 64), 64, 0, s>>>(D, C, list, nlist, W.cand, W.ncand,
                                                                                samples, W.slots, W.valid);
        constexpr int kCompactG = PtTraits<v>::kPosesPerRoot * PtTraits<v>::kRoots <= 4 ? 4 : 32;
        pt_compact_kernel<v><<<(int)(((size_t)nlist * kCompactG + 63) / 64), 64, 0, s>>>(
            C, list, nlist, W.ncand, W.slots, W.valid, models, recs, counts, maxm, BatchGate{D.gate, D.gate_hi});
        return hipGetLastError();
    });
}

// Early-exit schedule (MADPOSE_SCORE_EXIT=0 turns the exit off; MADPOSE_SCORE_CHECK
// "first,every" in trips of 256 correspondences overrides the schedule).
static ScoreBound score_bound(const PairConst &C, double best, int *work, unsigned long long *rec, unsigned epoch_hi,
                              const Model *models, Model *rec_out, bool *exit) {
    const int n = C.n;
    static const int mode = [] {
        return env_flag("MADPOSE_SCORE_EXIT", true) ? 1 : 0;
    }();
    // "first,every" (or "first": every trip after it), both >= 1
    static const std::pair<int, int> sched = [] {
        const char *e = std::getenv("MADPOSE_SCORE_CHECK");
        if (!e) return std::pair<int, int>(0, 1);
        int f = 0, v = 1, used = 0;
        const int k = std::sscanf(e, "%d%n,%d%n", &f, &used, &v, &used);
        if (k < 1 || e[used] != '\0' || f < 1 || v < 1) env_reject("MADPOSE_SCORE_CHECK", e, "expected first[,every] >= 1");
        return std::pair<int, int>(f, k == 2 ? v : 1);
    }();
    ScoreBound sb;
    // the exit and the record skip rest on every MSAC term being >= 0 (a partial sum is
    // then a lower bound of the total): errors are squares or DBL_MAX, thresholds are
    // positive (validate()), so it takes non-negative weights; the reference accepts any
    // weights, and with a negative one every iteration is scored in full
    const bool nonneg = C.w[0] >= 0.0 && C.w[1] >= 0.0 && C.w[2] >= 0.0;
    const bool on = mode != 0 && best < DBL_MAX && nonneg;
    *exit = on;
    sb.best = best;
    const int ntrip = (n + kBlock - 1) / kBlock;
    // default: a check every quarter of the trips, at most every two trips (512
    // correspondences; each check costs a wave reduction per live model and a barrier).
    // tools/score_bench.hip, round 2: at N = 2000 checks after trips 2, 4, 6 beat every
    // trip from 2 on, 209 vs 233 us; round 3 (profiles/r03/s11, HIP-event launch
    // averages): cal 44.7 / 45.5 / 47.7 us at 2,2 / 1,1 / 3,3, sf 33.1 / 35.2 us at 2,2 /
    // 1,1, tf (N = 4000) 56.7 us at 2,2 against 60.2 at 4,4
    const int q = std::min(2, std::max(1, ntrip / 4));
    sb.first = sched.first > 0 ? sched.first : q;
    sb.every = sched.first > 0 ? sched.second : q;
    sb.work = work;
    static const int pair = [] {
        return env_flag("MADPOSE_SCORE_PAIR", true) ? 1 : 0;
    }();
    sb.pair = pair;
    static const bool skip = [] {
        return env_flag("MADPOSE_RECORD_SKIP", true);
    }();
    sb.rec = (skip && on) ? rec : nullptr;
    sb.epoch_hi = epoch_hi;
    sb.models = models;
    sb.rec_out = rec_out;
    return sb;
}

hipError_t launch_score_batch(hipStream_t s, const PairData &D, const PairConst &C, const ScoreRec *recs,
                              const int *counts, int nb, int maxm, double *scores, IterResult *res, double best,
                              int *work, unsigned long long *rec, unsigned epoch_hi, const Model *models,
                              Model *rec_out, uint8_t *flags8, IterResult *cand_out) {
    if (nb <= 0) return hipSuccess;
    if (maxm != max_models(C.variant)) return hipErrorInvalidValue;
    const bool fast = C.score_type == 0 && !C.scale_only && (C.variant != kCal || (C.kstd && D.a0));
    bool exit = false;
    ScoreBound sb = score_bound(C, best, work, rec, epoch_hi, models, rec_out, &exit);
    sb.flags8 = flags8;
    sb.cand_out = cand_out;
    auto go = [&](auto V, auto M, auto F) {
        constexpr int kV = decltype(V)::value, kM = decltype(M)::value;
        constexpr bool kF = decltype(F)::value;
        if (exit)
            score_batch_kernel<kV, kM, kF, true><<<nb, kBlock, 0, s>>>(D, C, recs, counts, scores, res, sb);
        else
            score_batch_kernel<kV, kM, kF, false><<<nb, kBlock, 0, s>>>(D, C, recs, counts, scores, res, sb);
    };
    using T = std::true_type;
    using F = std::false_type;
    if (C.variant == kCal) {
        if (fast)
            go(std::integral_constant<int, kCal>(), std::integral_constant<int, kMaxModelsCal>(), T());
        else
            go(std::integral_constant<int, kCal>(), std::integral_constant<int, kMaxModelsCal>(), F());
    } else if (C.variant == kSF) {
        if (fast)
            go(std::integral_constant<int, kSF>(), std::integral_constant<int, kMaxModelsSF>(), T());
        else
            go(std::integral_constant<int, kSF>(), std::integral_constant<int, kMaxModelsSF>(), F());
    } else {
        if (fast)
            go(std::integral_constant<int, kTF>(), std::integral_constant<int, kMaxModelsTF>(), T());
        else
            go(std::integral_constant<int, kTF>(), std::integral_constant<int, kMaxModelsTF>(), F());
    }
    return hipGetLastError();
}

hipError_t launch_pt_roots(hipStream_t s, const PairData &D, const PairConst &C, const int *list, int nlist,
                           const int *samples, double *cand, int *ncand, double *pen) {
    if (nlist <= 0) return hipSuccess;
    if (C.variant == kCal)
        pt_roots5_group_kernel<<<(nlist + kS5 - 1) / kS5, 64, 0, s>>>(D, C, list, nlist, samples, cand, ncand,
                                                                      kCandStride);
    else if (C.variant == kSF && pen)
        launch_sf_eig(s, D, list, nlist, samples, cand, ncand, pen);
    else if (C.variant == kTF)
        pt_roots7_kernel<<<(nlist + 63) / 64, 64, 0, s>>>(D, list, nlist, samples, cand, ncand);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_debug_terms(hipStream_t s, const PairData &D, const PairConst &C, const ScoreRec *recs, int nm,
                              double *err, int *flags) {
    if (nm <= 0) return hipSuccess;
    const bool fast = C.score_type == 0 && !C.scale_only && (C.variant != kCal || (C.kstd && D.a0));
    return by_variant(C.variant, [&](auto V) {
        constexpr int v = decltype(V)::value;
        if (fast)
            debug_terms_kernel<v, true><<<nm, kBlock, 0, s>>>(D, C, recs, err, flags);
        else
            debug_terms_kernel<v, false><<<nm, kBlock, 0, s>>>(D, C, recs, err, flags);
        return hipGetLastError();
    });
}

hipError_t launch_sweep(hipStream_t s, const PairData &D, const PairConst &C, const ScoreRec *rec, double *err,
                        double *score) {
    return by_variant(C.variant, [&](auto V) {
        sweep_kernel<decltype(V)::value><<<1, 1024, 0, s>>>(D, C, rec, err, score);
        return hipGetLastError();
    });
}

hipError_t launch_score_models(hipStream_t s, const PairData &D, const PairConst &C, const ScoreRec *recs, int nm,
                               double *scores) {
    if (nm <= 0) return hipSuccess;
    return by_variant(C.variant, [&](auto V) {
        score_models_kernel<decltype(V)::value><<<nm, kBlock, 0, s>>>(D, C, recs, scores);
        return hipGetLastError();
    });
}

hipError_t launch_md_direct(hipStream_t s, int variant, int alt, const double *in, double *sols, int *nsols, Model *poses,
                            int *nposes) {
    md_direct_kernel<<<1, 64, 0, s>>>(variant, alt, in, sols, nsols, poses, nposes);
    return hipGetLastError();
}

// get_depths over many pairs (madpose/utils.py:4-22): keypoint i of pair p is scaled by
// the pair's (depth-map / image) size ratios, rounded half to even (rint under the
// default rounding mode, as np.round), clipped to the map and looked up at [y, x].
// One lane per keypoint; the pair is found by binary search over the keypoint offsets.
template <typename T>
__global__ void get_depths_kernel(const T *maps, const int64_t *map_off, const int64_t *dims, const double *fac,
                                  const int64_t *pt_off, int32_t num, const double *pts, T *out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= pt_off[num]) return;
    int lo = 0, hi = num - 1; // last pair with pt_off[p] <= i
    while (lo < hi) {
        const int mid = (lo + hi + 1) / 2;
        if (pt_off[mid] <= i)
            lo = mid;
        else
            hi = mid - 1;
    }
    const int p = lo;
    const int64_t h = dims[2 * p], w = dims[2 * p + 1];
    int64_t c = (int64_t)rint(pts[2 * i] * fac[2 * p]), r = (int64_t)rint(pts[2 * i + 1] * fac[2 * p + 1]);
    c = c < 0 ? 0 : (c > w - 1 ? w - 1 : c);
    r = r < 0 ? 0 : (r > h - 1 ? h - 1 : r);
    out[i] = maps[map_off[p] + r * w + c];
}

hipError_t launch_get_depths(hipStream_t s, int dtype, const void *maps, const int64_t *map_off, const int64_t *dims,
                             const double *fac, const int64_t *pt_off, int32_t num, int64_t total, const double *pts,
                             void *out) {
    if (total <= 0) return hipSuccess;
    const int grid = (int)((total + 255) / 256);
    if (dtype == 0)
        get_depths_kernel<float><<<grid, 256, 0, s>>>((const float *)maps, map_off, dims, fac, pt_off, num, pts,
                                                      (float *)out);
    else
        get_depths_kernel<double><<<grid, 256, 0, s>>>((const double *)maps, map_off, dims, fac, pt_off, num, pts,
                                                       (double *)out);
    return hipGetLastError();
}

// bougnoux_focals (src/hybrid_pose_two_focal_estimator.cpp:11-32) of k fundamental
// matrices (row-major, principal points at the origin), one lane each: the squared
// focals exactly as the 7pt tail computes them (mp_pt67.h bougnoux_sq)
__global__ void bougnoux_kernel(const double *F, int64_t k, double *out) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= k) return;
    double f[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) f[e] = F[9 * i + e];
    double f0, f1;
    bougnoux_sq(f, &f0, &f1);
    out[2 * i] = f0;
    out[2 * i + 1] = f1;
}

hipError_t launch_lm_batch(hipStream_t s, const PairData &D, const PairConst &C, const LmJob *jobs, int njobs,
                           const int *idx, Model *out, int *status) {
    if (njobs <= 0) return hipSuccess;
    return by_variant(C.variant, [&](auto V) {
        lm_batch_kernel<decltype(V)::value><<<njobs, kLmBlock, 0, s>>>(D, C, jobs, idx, out, status);
        return hipGetLastError();
    });
}

hipError_t launch_bougnoux(hipStream_t s, const double *F, int64_t k, double *out) {
    if (k <= 0) return hipSuccess;
    bougnoux_kernel<<<(int)((k + 255) / 256), 256, 0, s>>>(F, k, out);
    return hipGetLastError();
}

// compute_pose_error (madpose/utils.py:59-78) of k pairs, one lane each: the
// translation angle folded to [0, 90] (E fixes t up to sign) and the rotation angle
// between R_est and R_gt, in degrees, with numpy's formulas (norm product as the
// divisor, cosine clipped to [-1, 1], err_t = 0 when |t_gt| < t_thres if t_thres >= 0).
// R: k x 9 row-major, t: k x 3, T: k x 16 (row-major 4x4 T_0to1).
__global__ void pose_error_kernel(int64_t k, const double *R, const double *t, const double *T, double t_thres,
                                  double *err_t, double *err_R, double *err_max) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= k) return;
    const double *Ri = R + 9 * i, *ti = t + 3 * i, *Ti = T + 16 * i;
    const double kDeg = 180.0 / M_PI;
    const double tg0 = Ti[3], tg1 = Ti[7], tg2 = Ti[11];
    const double ng = sqrt(tg0 * tg0 + tg1 * tg1 + tg2 * tg2);
    const double n = sqrt(ti[0] * ti[0] + ti[1] * ti[1] + ti[2] * ti[2]) * ng;
    const double ct = (ti[0] * tg0 + ti[1] * tg1 + ti[2] * tg2) / n;
    // np.clip and np.minimum propagate NaN (a zero translation); fmin / fmax do not
    double et = isnan(ct) ? NAN : acos(fmin(fmax(ct, -1.0), 1.0)) * kDeg;
    if (!isnan(et)) et = fmin(et, 180.0 - et);
    if (t_thres >= 0.0 && ng < t_thres) et = 0.0;
    // trace(R_est^T R_gt) = sum over all entries of R_est .* R_gt
    double tr = 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) tr += Ri[c] * Ti[c] + Ri[3 + c] * Ti[4 + c] + Ri[6 + c] * Ti[8 + c];
    double cr = (tr - 1.0) / 2.0;
    const bool nan_r = isnan(cr);
    cr = fmin(fmax(cr, -1.0), 1.0);
    const double er = nan_r ? NAN : fabs(acos(cr)) * kDeg;
    err_t[i] = et;
    err_R[i] = er;
    if (err_max) err_max[i] = isnan(et) || isnan(er) ? NAN : fmax(et, er); // np.maximum propagates NaN
}

// Total order of the pose-AUC sort: ascending error, NaN last (np.sort), equal keys
// by index, so the ranks below are a permutation.
__device__ inline bool auc_before(double a, int64_t ia, double b, int64_t ib) {
    const bool an = isnan(a), bn = isnan(b);
    if (an != bn) return bn;
    if (an) return ia < ib;
    return a < b || (a == b && ia < ib);
}

constexpr int kAucBlock = 256, kAucChunk = 2048;

// Rank sort of the pose errors: lane i counts the elements ordered before e[i]
// (the array streamed through LDS in chunks) and stores e[i] at that rank.
__global__ __launch_bounds__(kAucBlock) void auc_rank_kernel(int64_t k, const double *e, double *sorted) {
    __shared__ double chunk[kAucChunk];
    const int64_t i = blockIdx.x * (int64_t)kAucBlock + threadIdx.x;
    const double ei = i < k ? e[i] : 0.0;
    int64_t rank = 0;
    for (int64_t base = 0; base < k; base += kAucChunk) {
        const int len = (int)(k - base < kAucChunk ? k - base : kAucChunk);
        __syncthreads();
        for (int j = threadIdx.x; j < len; j += kAucBlock) chunk[j] = e[base + j];
        __syncthreads();
        if (i < k)
            for (int j = 0; j < len; ++j) rank += auc_before(chunk[j], base + j, ei, i) ? 1 : 0;
    }
    if (i < k) sorted[rank] = ei;
}

// AUC of the cumulative error curve up to thr[b] (one workgroup per threshold): the
// trapezoid rule over (0, 0), (s_j, j / k) for the m sorted errors s_j < thr, closed
// at (thr, m / k), divided by thr -- the SuperGlue-style pose_auc of madpose_amd/utils.py.
// Lane-strided partial sums in ascending j, then a fixed-order tree: deterministic.
__global__ __launch_bounds__(kAucBlock) void auc_sum_kernel(int64_t k, const double *s, const double *thr,
                                                            double *aucs) {
    __shared__ double part[kAucBlock];
    __shared__ int64_t cnt[kAucBlock];
    const double t = thr[blockIdx.x];
    const double inv = 1.0 / (double)k;
    double acc = 0.0;
    int64_t m = 0;
    for (int64_t j = threadIdx.x; j < k; j += kAucBlock) {
        const double sj = s[j];
        if (!(sj < t)) continue; // sorted: the tail (and NaN) is past the threshold
        ++m;
        const double prev = j == 0 ? 0.0 : s[j - 1];
        const double r0 = j == 0 ? 0.0 : (double)j * inv, r1 = (double)(j + 1) * inv;
        acc += (sj - prev) * (r0 + r1) / 2.0;
    }
    part[threadIdx.x] = acc;
    cnt[threadIdx.x] = m;
    __syncthreads();
    for (int w = kAucBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            part[threadIdx.x] += part[threadIdx.x + w];
            cnt[threadIdx.x] += cnt[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int64_t mm = cnt[0];
        const double last = mm == 0 ? 0.0 : s[mm - 1], rl = mm == 0 ? 0.0 : (double)mm * inv;
        aucs[blockIdx.x] = (part[0] + (t - last) * rl) / t;
    }
}

hipError_t launch_pose_errors(hipStream_t s, int64_t k, const double *R, const double *t, const double *T,
                              double t_thres, double *err_t, double *err_R, double *err_max) {
    if (k <= 0) return hipSuccess;
    pose_error_kernel<<<(int)((k + 255) / 256), 256, 0, s>>>(k, R, t, T, t_thres, err_t, err_R, err_max);
    return hipGetLastError();
}

hipError_t launch_pose_auc(hipStream_t s, int64_t k, const double *e, double *sorted, int nthr, const double *thr,
                           double *aucs) {
    if (k <= 0 || nthr <= 0) return hipSuccess;
    auc_rank_kernel<<<(int)((k + kAucBlock - 1) / kAucBlock), kAucBlock, 0, s>>>(k, e, sorted);
    auc_sum_kernel<<<nthr, kAucBlock, 0, s>>>(k, sorted, thr, aucs);
    return hipGetLastError();
}

hipError_t launch_scale_and_pose(hipStream_t s, const double *in, int64_t n, Model *out) {
    scale_and_pose_kernel<<<1, 64, 0, s>>>(in, n, out);
    return hipGetLastError();
}

// the poses of a shared-focal 6-point sample from the root stage's output (null space
// and roots in cand, as written by pt_roots6_eig_kernel); one lane
__global__ void point_direct_6pt_kernel(const double *in, const double *cand, const int *ncand, Model *poses,
                                        int *nposes) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double b0[6][3], b1[6][3];
    for (int j = 0; j < 6; ++j) {
        const double a[3] = {in[2 * j], in[2 * j + 1], 1.0}, c[3] = {in[12 + 2 * j], in[12 + 2 * j + 1], 1.0};
        const double na = 1.0 / sqrt(dot3(a, a)), nc = 1.0 / sqrt(dot3(c, c));
        for (int q = 0; q < 3; ++q) {
            b0[j][q] = a[q] * na;
            b1[j][q] = c[q] * nc;
        }
    }
    double N[3][9];
    for (int e = 0; e < 27; ++e) N[e / 9][e % 9] = cand[e];
    double M[3][10][10];
    sixpt_matrices(N, M);
    const int nr = ncand[0] < 15 ? ncand[0] : 15;
    *nposes = sixpt_poses_for_roots(M, N, cand + 27, nr, b0, b1, poses, kMaxModelsSF);
}

hipError_t launch_point_direct_6pt(hipStream_t s, const double *in, const double *cand, const int *ncand,
                                   Model *poses, int *nposes) {
    point_direct_6pt_kernel<<<1, 64, 0, s>>>(in, cand, ncand, poses, nposes);
    return hipGetLastError();
}

// the poses of a 5-point sample from the estimator's root stage (E candidates in cand):
// motion_from_essential with cheirality on the five bearings, one lane
__global__ void point_direct_5pt_kernel(const double *in, const double *cand, const int *ncand, Model *poses,
                                        int *nposes) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double b1[5][3], b2[5][3];
    for (int j = 0; j < 5; ++j)
        for (int c = 0; c < 3; ++c) {
            b1[j][c] = in[3 * j + c];
            b2[j][c] = in[15 + 3 * j + c];
        }
    int k = 0;
    for (int e = 0; e < ncand[0] && e < 10; ++e) k += motion_from_essential<5>(cand + 9 * e, b1, b2, poses, k, kMaxModelsCal);
    *nposes = k;
}

hipError_t launch_point_direct(hipStream_t s, int kind, const double *in, Model *poses, int *nposes, double *cand,
                               int *ncand) {
    if (kind == 0) {
        // the estimator's root stage (group_5pt.h) on the one sample, then its poses
        pt_roots5_bearings_kernel<<<1, 64, 0, s>>>(in, 1, cand, ncand, kCandStride);
        point_direct_5pt_kernel<<<1, 64, 0, s>>>(in, cand, ncand, poses, nposes);
        return hipGetLastError();
    }
    point_direct_kernel<<<1, 64, 0, s>>>(kind, in, poses, nposes);
    return hipGetLastError();
}

} // namespace mp
