// Host controller of the MI355X hybrid LO-MSAC estimator.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../include/mp_types.h"
#include "lm.h"

namespace mp {

struct RansacOptions {
    uint32_t min_num_iterations = 100, max_num_iterations = 10000, max_num_iterations_per_solver = 10000;
    double success_probability = 0.99;
    double squared_inlier_thresholds[2] = {1.0, 1.0};
    double data_type_weights[2] = {1.0, 1.0};
    uint32_t random_seed = 0;
    int num_lo_steps = 10;
    double threshold_multiplier = 1.4142135623730951;
    int num_lsq_iterations = 4, min_sample_multiplicator = 7, non_min_sample_multiplier = 3;
    int lo_starting_iterations = 50;
    bool final_least_squares = false, use_ours = false, use_4p4d = false;
};

struct EstimatorConfig {
    int solver_type = 0, score_type = 0, lo_type = 0;
    bool min_depth_constraint = true, use_shift = true;
    double ftol = 1e-6, gtol = 1e-8, ptol = 1e-6, max_iter = 25;
    bool nonmonotonic = true; // ceres_use_nonmonotonic_steps
};

struct Stats {
    uint32_t num_iterations_total = 0;
    uint32_t num_iterations_per_solver[2] = {0, 0};
    int best_num_inliers = 0;
    int best_solver_type = -1;
    double best_model_score = 0.0;
    double inlier_ratios[3] = {0, 0, 0};
    std::vector<int> inlier_indices[3];
    int number_lo_iterations = 0;
    uint64_t num_hypotheses = 0, num_lo_sweeps = 0;
    int num_batches = 0;
    double seconds_total = 0, seconds_lo = 0, seconds_gpu_wait = 0;
};

struct PairInput {
    int variant = kCal;
    int64_t n = 0;
    const double *x0 = nullptr, *x1 = nullptr, *d0 = nullptr, *d1 = nullptr;
    double min_depth[2] = {0, 0};
    double cam0[9] = {0}, cam1[9] = {0}; // K (CAL) or principal point (SF/TF)
};

// Runs the full estimator on one pair on `device`; throws std::runtime_error on HIP
// errors and std::invalid_argument on bad input.  The returned model is in user
// units (SF/TF focals multiplied back by the normalisation scale).
void estimate_pair(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, int device, Model *out,
                   Stats *stats);

// Scores explicit models (problem units) on the device (mp_score_models).
void score_models(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, const Model *models,
                  int nm, double *scores, double *errors, int device, double *norm_scale);

// The engine's host LO sweep (host/lo_sweep.h) over explicit models (problem units):
// the errors and ScoreModel sums LO uses (mp_debug_lo_sweep, test hook; no device)
void lo_sweep_models(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, const Model *models,
                     int nm, double *scores, double *errors, double *fast_bounds = nullptr);

// score_batch's residuals of explicit models: errors nm x 3 x n, flags nm x n, taus nm x
// 3 (per-term bounds), ties nm (margins) -- mp_debug_score_terms, test hook
void debug_score_terms(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, const Model *models,
                       int nm, double *errors, int *flags, double *taus, double *ties, int device);

// score_batch over explicit models (mp_debug_score_batch; test hook).  models: nb x
// max_models(variant) (problem units), counts[b] of them used per iteration.  flags: 1
// exact early exit against `best`, 2 record skip.  res_slot keeps kSlotAmbiguous /
// kSlotUncertain; res_hi_lo (nullable): hi, lo per iteration; model_ties (nullable, nb x
// max_models): the margins.
void debug_score_batch(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, int nb,
                       const int *counts, const Model *models, double best, int flags, double *res_best,
                       int *res_slot, Model *rec_models, double *res_hi_lo, double *model_ties, int device);

// Batched device LM (mp_lm_refine_batch): problem j refines models[j] (problem units)
// over the residual blocks idx[offsets[3j] .. offsets[3j+1]) (reproj 0->1),
// [offsets[3j+1] .. offsets[3j+2]) (1->0), [offsets[3j+2] .. offsets[3j+3]) (Sampson),
// with the settings of LeastSquares (kinds[j] 0) or NonMinimalSolver (1).  status[j]:
// 1 refined, 0 no residuals, 2 infeasible constant block, 3 too few data (unchanged).
void lm_refine_batch_device(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, int nprob,
                            const int32_t *kinds, const int64_t *offsets, const int32_t *idx, Model *models,
                            int32_t *status, int device);

void lm_refine_batch_host(const PairInput &in, const RansacOptions &opts, const EstimatorConfig &cfg, int nprob,
                          const int32_t *kinds, const int64_t *offsets, const int32_t *idx, Model *models,
                          int32_t *status);

// Standalone solvers on the device (mp_solve_* / mp_relpose_5pt).
// alt: 0 default MD solver, 1 use_ours, 2 use_4p4d (two-focal)
int solve_md_direct(int variant, const double *x, const double *y, const double *dx, const double *dy, double *sols,
                    int max_sols, Model *poses, int max_poses, int *nposes, int device, int alt = 0);
// kind 0: relpose_5pt on unit bearings; 1: shared-focal 6pt; 2: two-focal 7pt +
// Bougnoux + recoverPose (normalized 2-D points).  Models before the depth fit.
int solve_point_direct(int kind, const double *x1, const double *x2, Model *poses, int max_poses, int device);
// root stage of the calibrated 5-point (variant 0) or shared-focal 6-point (variant 1)
// solver over ns samples of K = 5 / 6 normalized image points each (pts*: ns x K x 2);
// candidates into cand (ns x 96), counts into ncand
void debug_pt_roots(int variant, int64_t ns, const double *pts0, const double *pts1, double *cand, int *ncand,
                    int device);

// estimate_scale_and_pose (src/solver.cpp:5-33) on the device; X, Y point-major n x 3
void scale_and_pose_direct(const double *X, const double *Y, const double *W, int64_t n, Model *out, int device);
// get_depths of num pairs on the device (see launch_get_depths); dims: num x 4
// (depth-map h, w, image h, w); host buffers in and out
// squared Bougnoux focals of k fundamental matrices (device kernel, mp_bougnoux_focals)
void bougnoux_batch(int64_t k, const double *F, double *out, int device);
// compute_pose_error of k pairs and the pose AUC of max(err_R, err_t) at nthr
// thresholds on the device (mp_pose_eval); host buffers in and out
void pose_eval_batch(int64_t k, const double *R, const double *t, const double *T, double t_thres, double *err_t,
                     double *err_R, int nthr, const double *thr, double *aucs, int device);
// the pose AUC of k given errors at nthr thresholds (mp_pose_auc)
void pose_auc_batch(int64_t k, const double *errors, int nthr, const double *thr, double *aucs, int device);
void get_depths_batch(int dtype, int32_t num, const void *maps, const int64_t *dims, const int64_t *pt_off,
                      const double *pts, void *out, int device);

int device_count();

// Per-kernel device timing of the estimator's batch launches, measured with HIP
// events on the engine's own stream (mp_profile_* C API).  Process-wide totals.
struct KernelProfile {
    uint64_t batches = 0;          // speculative batches timed
    uint64_t iterations = 0;       // minimal samples solved
    uint64_t hypotheses = 0;       // models scored by score_batch
    uint64_t correspondences = 0;  // sum over batches of (hypotheses x n)
    uint64_t sweeps = 0;           // single-model LO / termination sweeps
    double solve_ms = 0.0;         // md_solve + pt_solve
    double score_ms = 0.0;         // score_batch
    uint64_t lm_calls = 0;         // host LM solves inside LO
    double lm_wall_ms = 0.0;       // host wall time in the LM
    double sweep_wall_ms = 0.0;    // host wall time of single-model sweeps (incl. copies + sync)
    double sample_wall_ms = 0.0;   // host minimal-sample generation (incl. LO rewinds)
    double wait_wall_ms = 0.0;     // host wait for batch results
    double run_wall_ms = 0.0;      // whole estimator runs
    uint64_t lm_blocks = 0;        // residual blocks over all LM solves
    uint64_t lm_big_calls = 0;     // LM solves with >= kBigLM residual blocks
    double lm_big_wall_ms = 0.0;   // host wall time of those
    uint64_t model_trips = 0;      // score_batch (model, 256-correspondence trip) pairs evaluated
    uint64_t model_trips_full = 0; // ... and without the early exit (models x trips)
    uint64_t accepted = 0;         // hypotheses of the iterations the estimator consumed
    uint64_t scored = 0;           // hypotheses whose score_batch sweep ran (not record-skipped)
    uint64_t tie_checks = 0;       // iterations whose new-best decision needed reference-order re-scoring
};
constexpr size_t kBigLM = 1024;
void profile_enable(bool on);
void profile_reset();
KernelProfile profile_read();

} // namespace mp
