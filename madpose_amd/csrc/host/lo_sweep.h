// Host LO sweep: one model over all 3N residuals of a pair, on the CPU core of the LO
// thread that asks for it.
//
// Local optimisation stays on the host (north star), and an LO step is a chain of
// about six (sweep -> inlier lists -> LM) links.  A device sweep costs one launch plus
// a completion round trip (~17-20 us in the engine) for ~10 us of
// 256-lane work; the same 3N residuals take a few microseconds vectorised on the
// host core that needs them.  The minimal-sample scoring (score_batch) stays on the
// GPU; this replaces only the single-model sweeps of LocalOptimization /
// UpdateRANSACTerminationCriteria (src/hybrid_ransac.h:289-349, 351-378, 383-538).
//
// Residuals: the reference's EvaluateModelOnPoint operation sequence (as the oracle
// restates it), ungated (is_for_inlier = true), evaluated 8 (AVX-512) or 4 (AVX2)
// correspondences at a time without FMA contraction: bit-identical to the oracle's
// scalar errors.  Score: the reference's ScoreModel order (src/hybrid_ransac.h:
// 265-287) -- ONE running sum, data type t outer, correspondence i inner and
// ascending, each term std::min(e, thr_t) * w_t (a score-type-gated residual
// contributes thr_t * w_t) -- bit-identical to the oracle's score.
#pragma once
#include <cstdint>
#include <memory>

#include "../include/mp_types.h"

namespace mp {

// Correspondences as the host sweep reads them: structure of arrays, 64-byte aligned.
// Calibrated pairs also carry ca = K0^-1 x0, cb = K1^-1 x1 and the unit bearings
// ua = ca / |ca|, ub = cb / |cb|, formed once per pair.
struct LoSweepData {
    int n = 0;
    int cal = 0;
    const double *x0u = nullptr, *x0v = nullptr, *x1u = nullptr, *x1v = nullptr, *d0 = nullptr, *d1 = nullptr;
    const double *ca[3] = {nullptr, nullptr, nullptr}, *cb[3] = {nullptr, nullptr, nullptr};
    const double *ua[3] = {nullptr, nullptr, nullptr}, *ub[3] = {nullptr, nullptr, nullptr};
    std::unique_ptr<double[], void (*)(double *)> store{nullptr, nullptr};
};

// x0, x1: 2n interleaved (pixels for the calibrated variant, normalized pixels
// otherwise -- the engine's HostPair); d0, d1: n
void lo_sweep_prepare(const PairConst &C, const double *x0, const double *x1, const double *d0, const double *d1,
                      LoSweepData *D);

// errors err[t * n + i] (GetInliers' EvaluateModelOnPoint(.., is_for_inlier = true))
// of model m (problem units); returns the ScoreModel sum
double lo_sweep(const PairConst &C, const LoSweepData &D, const Model &m, double *err);

// The same errors with a fast sum instead: ScoreModel's reference-order sum is one
// chain of 3n dependent additions (about half of a sweep's time), and most of the LO's
// scores only need to be compared with the best score.  The terms are the reference's
// to the bit, so the two sums differ by their order alone: |fast - reference sum| <=
// *bound (both within gamma_3n sum|term| of the exact sum).  A caller takes the
// reference-order sum (lo_ordered_score, from the same errors) only when the fast sum
// cannot decide its comparison.
void lo_sweep_fast(const PairConst &C, const LoSweepData &D, const Model &m, double *err, double *fast, double *bound);

// ScoreModel's sum (src/hybrid_ransac.h:274-281) over errors of lo_sweep / lo_sweep_fast
double lo_ordered_score(const PairConst &C, const double *err, int n);

// the instruction set lo_sweep dispatched to: 512 (AVX-512F) or 256 (AVX2)
int lo_sweep_width();

} // namespace mp
