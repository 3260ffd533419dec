// Shared types of the MI355X hybrid-RANSAC engine (device kernels + host controller).
#pragma once
#include <cstdint>
#include <type_traits>
#include <utility>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MP_HD __host__ __device__ inline
#define MP_DEV __device__ inline
#else
#define MP_HD inline
#define MP_DEV inline
#endif

namespace mp {

// A value the optimiser cannot trace back to the load that produced it.  For selects
// between elements of a local array / struct: select(c, load a, load b) is folded
// into load(select(c, &a, &b)), which keeps the whole aggregate in scratch; selecting
// between opaque values keeps it in registers.
MP_HD double opaque(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x));
#endif
    return x;
}

enum Variant : int { kCal = 0, kSF = 1, kTF = 2, kScaleOnly = 3 }; // kScaleOnly: host-side only

// Model layout == mp_model of include/madpose_mi355x.h (src/pose.h:7-56).
// R row-major, x1 = R x0 + t.
struct Model {
    double R[9];
    double t[3];
    double scale, offset0, offset1, focal0, focal1;
};

// Per-model constants for the scoring sweep, prepared once per hypothesis so the
// per-correspondence work is a handful of FMAs (see DESIGN.md "score_sweep").
//   t=0:  p = M0 (x0,y0,1) * (d0 + o0) + k0      (M0 = K1 R K0^-1, k0 = K1 t)
//   t=1:  p = M1 (x1,y1,1) * (d1*s + o1s) + k1   (M1 = K0 R^T K1^-1, k1 = -K0 R^T t)
//   t=2:  Sampson with G (E for calibrated rays, F for normalized pixels),
//         cheirality with R, t on unit bearings (calibrated variant only).
//   nrt = -R^T t (the ray form of t=1, calibrated intrinsics of the kstd shape)
//   tie:      the model's screening margin, a bound on |device sum - reference-order
//             sum| of its MSAC score when no correspondence is flagged (mp_score.h
//             score_margins)
//   wz0, wz1: half-widths of the z < 1e-2 gates (t = 0, 1) within which the device's
//             and the reference's depth may fall on different sides
//   wl:       the same for the calibrated cheirality test (l1, l2 against min_depth)
//   kg2:      Sampson conditioning floor: den < kg2 flags the correspondence
struct ScoreRec {
    double M0[9], k0[3], M1[9], k1[3], G[9], R[9], t[3], nrt[3];
    double o0, s, o1s, tie, wz0, wz1, wl, kg2;
};

// Per-pair constants (uniform over a launch).
struct PairConst {
    int variant;
    int n;
    int score_type; // 0 hybrid, 1 epi-only, 2 md-only (EstimatorConfig::score_type)
    int min_depth_constraint;
    int use_shift;
    int md_alt; // 0 default MD solvers, 1 use_ours, 2 use_4p4d (two-focal)
    int scale_only; // HybridEstimatePoseAndScale (calibrated geometry, no offsets)
    int kstd;       // calibrated K0, K1 (and inverses) of the form [a b c; 0 d e; 0 0 1] (score ray form)
    double K0[9], K1[9], K0i[9], K1i[9]; // identity for SF/TF (focal lives in the model)
    double thr[3], w[3];                 // squared thresholds / weights after the option transform
    double loss_scale;                   // calibrated Sampson scale (src/hybrid_pose_estimator.h:35-36)
    double min_depth[2];
    // magnitudes of the pair for the screening margins (mp_score.h score_margins):
    // cal: ea = max_i |a_i|_1 with a = K0^-1 x0, eap = max_i sum_jk |K0^-1_jk x0_k|, exi =
    // max_i eap_i / (|a_0| + |a_1| + 1); uncal: ea = eap = max_i |u_i| + |v_i| of the
    // normalized points, exi = 0.  eb, ebp, exj: the same for x1 / K1.  ed0, ed1: max
    // |depth|; ex0, ex1: max |coordinate| of x0, x1 (pixels, or normalized).
    // eab2: max_i (alpha_i beta_i)^2, alpha = |a_0| + |a_1| + 1 (a = K0^-1 x0, or x0),
    // beta likewise (the Sampson conditioning floor, score_margins).
    double ea, eap, exi, eb, ebp, exj, ed0, ed1, ex0, ex1, eab2;
    double tie_scale; // multiplies every margin (MADPOSE_TIE_SCALE: tests force the host resolution)
    // the model-independent parts of the margins (mp_score.h margin_consts): per
    // reprojection t, mg_s2 = 2 sqrt(thr_t), mg_U = the inlier projection bound; cal:
    // delta_t = mg_c1[t] Eq_t + mg_c0[t]; the Sampson term bound; the summation-order
    // part of the margin
    double mg_s2[2], mg_U[2], mg_c0[2], mg_c1[2], mg_tau2, mg_fixed;
};

// Device-resident correspondence arrays of one pair (structure of arrays, doubles).
struct PairData {
    const double *x0u, *x0v, *x1u, *x1v, *d0, *d1; // pixels (CAL) or normalized pixels (SF/TF)
    const double *r0, *r1;                          // 1/|K^-1 x| (CAL bearings), else unused
    // CAL: the rays' first two components a = K0^-1 x0, b = K1^-1 x1 (prep_pair_kernel;
    // the score kernel's ray form reads them instead of forming them per trip)
    const double *a0 = nullptr, *a1 = nullptr, *b0 = nullptr, *b1 = nullptr;
    // Batch gate (nullable): the kernels of a batch launched before the previous batch's
    // results were read leave at once when that batch published a record (score_batch's
    // record word holds ~its epoch, gate_hi), i.e. when the host is bound to run LO and
    // discard this batch (engine.cpp, early continuation)
    const unsigned long long *gate = nullptr;
    unsigned gate_hi = 0;
};
struct BatchGate {
    const unsigned long long *word = nullptr;
    unsigned hi = 0;
};

// Per-iteration outcome of a batch (score_batch): the iteration's best score
// (GetBestEstimatedModelId), its bounds, its model slot and the number of models -- one
// 32-byte record; the walk reads only the marked iterations' records (written to mapped
// host memory) and one flag byte per iteration (engine.cpp).
// hi = best + the best model's margin (its reference-order score is below hi), lo = the
// smallest score - margin over the iteration's models (no reference-order score of the
// iteration is below lo).  slot | kSlotAmbiguous: another model's interval reaches the
// best's; | kSlotUncertain: a correspondence was flagged (a gate or Sampson value the
// margins do not cover), so only the reference-order sums decide (engine.cpp).
struct IterResult {
    double best, hi, lo;
    int slot, count;
};
constexpr int kSlotAmbiguous = 1 << 16;
constexpr int kSlotUncertain = 1 << 17;
constexpr int kSlotMask = kSlotAmbiguous - 1;

// One least-squares problem of the batched device LM (kernels/lm_device.h): residual
// blocks idx[off0 .. off0+n0) (reprojection 0->1), idx[off1 ..) (1->0), idx[off2 ..)
// (Sampson) of the pair, the Ceres settings of the call and the start model.
struct LmJob {
    int off0, n0, off1, n1, off2, n2;
    int use_shift, min_depth_constraint, nonmonotonic, max_iter;
    double w_sampson, ftol, gtol, ptol;
    Model m;
};

constexpr int kMaxModelsCal = 10; // MD <= 4, 5pt <= 10
constexpr int kMaxModelsSF = 16;  // MD <= 8, 6pt <= 15
constexpr int kMaxModelsTF = 4;   // MD <= 4, 7pt <= 3
// static_for<N>(f): f(std::integral_constant<int, 0>()) ... f(<N-1>) -- loop bodies whose
// array indices are constants from the front end on, so small per-lane arrays stay in
// registers (a #pragma unroll loop index only becomes constant after unrolling,
// which can be too late for the arrays it indexes to leave scratch).
template <class F, int... I> MP_HD void static_for_seq(F &&f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>()), ...);
}
template <int N, class F> MP_HD void static_for(F &&f) {
    static_for_seq(static_cast<F &&>(f), std::make_integer_sequence<int, N>());
}

MP_HD int max_models(int v) { return v == kCal ? kMaxModelsCal : (v == kSF ? kMaxModelsSF : kMaxModelsTF); }

} // namespace mp
