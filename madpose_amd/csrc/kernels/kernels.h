// Host-side launch wrappers of the HIP kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../include/mp_types.h"

namespace mp {

constexpr int kSampleStride = 8; // sample indices per iteration slot (max minimal sample = 7)

// The batch gate of PairData: true when the record word holds the previous batch's
// epoch, i.e. that batch published a record (and the host will discard this one).
// Every lane of a workgroup reads the same word, so the exit is uniform.
__device__ inline bool batch_cancelled(const unsigned long long *word, unsigned hi) {
    return word != nullptr &&
           (unsigned)(__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == hi;
}

// r0/r1 = 1 / |K^-1 x| for the calibrated bearings; a0 .. b1 (nullable, calibrated):
// the rays' first two components, a = K0^-1 x0 and b = K1^-1 x1 (PairData::a0 .. b1)
hipError_t launch_prep_pair(hipStream_t s, const PairConst &C, const PairData &D, double *r0, double *r1,
                            double *a0 = nullptr, double *a1 = nullptr, double *b0 = nullptr, double *b1 = nullptr);

// MD minimal solver over the listed iterations (md_exact: R lanes per sample).
hipError_t launch_md_solve(hipStream_t s, const PairData &D, const PairConst &C, const int *list, int nlist,
                           const int *samples, Model *models, ScoreRec *recs, int *counts, int maxm);
// Workspace of the staged point solvers (per point sample: candidate roots and model
// slots).  cand: kPtCandStride doubles, slots / valid: kPtSlotStride entries.
constexpr int kPtCandStride = 96, kPtSlotStride = 32;
constexpr int kPtPenStride = 300; // shared focal: the 3 x 10 x 10 pencil of a sample (eig6.h)
struct PtWorkspace {
    double *cand;
    int *ncand;
    Model *slots;
    int *valid;
    double *pen; // kPtPenStride doubles per point sample (shared focal)
    // the two-stage exact MD solver's per-sample state (kMdWsStride doubles per MD sample,
    // structure of arrays with leading dimension md_ld >= the batch's MD samples) and root
    // counts; null: the one-stage kernel
    double *md_ws = nullptr;
    int *md_nr = nullptr;
    int md_ld = 0;
};
constexpr int kMdWsStride = 72; // doubles: the system (<= 62) + its roots (<= 8)
// The exact MD solver in two launches when W.md_ws is set and MADPOSE_MD_TWO_STAGE=2 (the
// setup with one lane per sample, then one lane per root); else launch_md_solve.  (The
// fused calibrated launch, launch_solve_fused, takes the two stages by default.)
hipError_t launch_md_solve_staged(hipStream_t s, const PairData &D, const PairConst &C, const int *list, int nlist,
                                  const int *samples, const PtWorkspace &W, Model *models, ScoreRec *recs,
                                  int *counts, int maxm);
// point minimal solver over the listed iterations (three launches, see kernels.hip;
// roots_done: the root stage ran in launch_solve_fused).
hipError_t launch_pt_solve(hipStream_t s, const PairData &D, const PairConst &C, const int *list, int nlist,
                           const int *samples, const PtWorkspace &W, Model *models, ScoreRec *recs, int *counts,
                           int maxm, bool roots_done = false);
// Calibrated, default MD solver at 4 lanes per sample (MADPOSE_SOLVE_FUSE=0 turns it
// off): the MD solver and the 5pt root stage in one launch, then the 5pt tails and
// compaction -- both solvers on one stream, no fork / join.
bool solve_fusable(const PairConst &C);
hipError_t launch_solve_fused(hipStream_t s, const PairData &D, const PairConst &C, const int *md_list, int nmd,
                              const int *pt_list, int npt, const int *samples, const PtWorkspace &W, Model *models,
                              ScoreRec *recs, int *counts, int maxm);
// scoring sweep: one workgroup per iteration, every model of the iteration scored
// over all correspondences; per-iteration argmin (first minimum wins) into res[b] with
// the screening bounds hi / lo and the kSlotAmbiguous / kSlotUncertain flags (each
// model's margin is ScoreRec::tie, mp_score.h score_margins).  best: the best
// minimal-model score before the batch (DBL_MAX: none yet); with non-negative weights a
// model whose partial sum minus its margin reaches best cannot win and is dropped early
// (exact early exit, kernels.hip ScoreBound), reporting DBL_MAX.  work (nullable): per
// iteration the (model, 256-correspondence trip) pairs evaluated.  rec (nullable): the
// record word of a batch that is cut at its first new best (kernels.hip ScoreBound),
// with epoch_hi = ~epoch, a value unique to the batch; published when hi < best without
// a flag.  rec_out (nullable, device-mapped host memory, nb Models): iterations whose lo
// is below best, or that are uncertain, write their best model (from models, nb x maxm)
// to rec_out[b].
hipError_t launch_score_batch(hipStream_t s, const PairData &D, const PairConst &C, const ScoreRec *recs,
                              const int *counts, int nb, int maxm, double *scores, IterResult *res, double best,
                              int *work, unsigned long long *rec = nullptr, unsigned epoch_hi = 0,
                              const Model *models = nullptr, Model *rec_out = nullptr, uint8_t *flags8 = nullptr,
                              IterResult *cand_out = nullptr);
// score_batch's per-correspondence errors (3 x n per model) and flags (n per model) of
// nm explicit models (test hook)
hipError_t launch_debug_terms(hipStream_t s, const PairData &D, const PairConst &C, const ScoreRec *recs, int nm,
                              double *err, int *flags);
// single-model sweep: per-point squared errors (3 x n, no gating) + gated MSAC score
hipError_t launch_sweep(hipStream_t s, const PairData &D, const PairConst &C, const ScoreRec *rec, double *err,
                        double *score);
// the estimator's point-solver root stage alone, C.variant kCal (5pt, 16-lane groups)
// or kSF (6pt, deflated eigenproblem, eig6.h; pen: kPtPenStride doubles per sample).
// cand: kPtCandStride doubles per sample (cal: 9 per essential matrix; sf: null-space
// basis N (27), then the positive roots u)
hipError_t launch_pt_roots(hipStream_t s, const PairData &D, const PairConst &C, const int *list, int nlist,
                           const int *samples, double *cand, int *ncand, double *pen = nullptr);
// scores of many explicit models (one workgroup per model) -- used by mp_score_models
hipError_t launch_score_models(hipStream_t s, const PairData &D, const PairConst &C, const ScoreRec *recs, int nm,
                               double *scores);

// standalone solvers (mp_solve_* C API): one sample, one thread
hipError_t launch_md_direct(hipStream_t s, int variant, int alt, const double *in /* x(3K) y(3K) dx(K) dy(K) */,
                            double *sols, int *nsols, Model *poses, int *nposes);
// (kind 0: cand / ncand are the root stage's workspace, kPtCandStride doubles and one int)
hipError_t launch_point_direct(hipStream_t s, int kind, const double *in, Model *poses, int *nposes, double *cand,
                               int *ncand);
// shared-focal 6pt poses from a root stage's output (cand: null space + roots of one
// sample, ncand: root count); in: the 6 + 6 normalized 2-D points
hipError_t launch_point_direct_6pt(hipStream_t s, const double *in, const double *cand, const int *ncand,
                                   Model *poses, int *nposes);

// batched device LM: one workgroup per job; out[j] the refined model, status[j] 1
// refined, 0 no residuals, 2 infeasible constant block (unchanged)
hipError_t launch_lm_batch(hipStream_t s, const PairData &D, const PairConst &C, const LmJob *jobs, int njobs,
                           const int *idx, Model *out, int *status);

// squared Bougnoux focals of k fundamental matrices (9 doubles each) into out (2 each)
hipError_t launch_bougnoux(hipStream_t s, const double *F, int64_t k, double *out);

// compute_pose_error of k pairs (R k x 9, t k x 3, T k x 16 row-major T_0to1; t_thres
// < 0: none) into err_t, err_R (degrees) and, when err_max is given, max(err_t, err_R)
hipError_t launch_pose_errors(hipStream_t s, int64_t k, const double *R, const double *t, const double *T,
                              double t_thres, double *err_t, double *err_R, double *err_max);

// pose AUC of k errors at nthr thresholds: rank sort into sorted (k doubles of
// scratch), then one workgroup per threshold
hipError_t launch_pose_auc(hipStream_t s, int64_t k, const double *e, double *sorted, int nthr, const double *thr,
                           double *aucs);

// estimate_scale_and_pose over n points (in = X(3n) Y(3n) W(n)), one thread
hipError_t launch_scale_and_pose(hipStream_t s, const double *in, int64_t n, Model *out);

// get_depths of num pairs in one launch (dtype 0 float32, 1 float64 maps): map p at
// maps + map_off[p] (dims[2p] x dims[2p+1]), size ratios fac[2p] (x), fac[2p+1] (y),
// its keypoints at pts[2 pt_off[p] ..], results at out[pt_off[p] ..]; total = pt_off[num]
hipError_t launch_get_depths(hipStream_t s, int dtype, const void *maps, const int64_t *map_off, const int64_t *dims,
                             const double *fac, const int64_t *pt_off, int32_t num, int64_t total, const double *pts,
                             void *out);

} // namespace mp
