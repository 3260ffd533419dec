/* madpose_mi355x.h -- C ABI of the MI355X-native hybrid-RANSAC relative-pose engine.
 *
 * Drop-in boundary for kocurvik/madpose's Python estimator API.  Each entry point
 * replaces one binding of the reference's pybind11 module (src/bindings.cpp) and
 * keeps its argument meaning; the reference signatures are cited per function.
 * Plain pointers and sizes only.  All buffers are owned by the caller; inputs are
 * copied to device memory inside the call.  Calls are re-entrant per device.
 *
 * Return codes: MP_OK, MP_EINVAL (bad sizes/options), MP_EDEVICE (HIP error; text
 * via mp_last_error()).  There is no CPU fallback: without a usable MI355X device
 * every compute entry point returns MP_EDEVICE.
 */
#ifndef MADPOSE_MI355X_H
#define MADPOSE_MI355X_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MP_OK 0
#define MP_EINVAL 1
#define MP_EDEVICE 2

/* estimator variants */
#define MP_CALIBRATED 0   /* HybridEstimatePoseScaleOffset          */
#define MP_SHARED_FOCAL 1 /* HybridEstimatePoseScaleOffsetSharedFocal */
#define MP_TWO_FOCAL 2    /* HybridEstimatePoseScaleOffsetTwoFocal    */
#define MP_SCALE_ONLY 3   /* HybridEstimatePoseAndScale (K0/K1 as cam0/cam1, min_depth ignored) */

/* ExtendedHybridLORansacOptions (src/hybrid_ransac.h:17-25, src/bindings.cpp:78-95) */
typedef struct mp_ransac_options {
    double success_probability;
    double squared_inlier_thresholds[2]; /* [reprojection^2, epipolar^2] (user units) */
    double data_type_weights[2];         /* [reprojection, epipolar]                  */
    double threshold_multiplier;
    uint32_t min_num_iterations;
    uint32_t max_num_iterations;
    uint32_t max_num_iterations_per_solver;
    uint32_t random_seed;
    int32_t num_lo_steps;
    int32_t num_lsq_iterations;
    int32_t min_sample_multiplicator;
    int32_t non_min_sample_multiplier;
    int32_t lo_starting_iterations;
    int32_t final_least_squares;
    int32_t use_ours;
    int32_t use_4p4d;
} mp_ransac_options;

/* EstimatorConfig (src/estimator_config.h:7-33, src/bindings.cpp:99-109) */
typedef struct mp_estimator_config {
    double ceres_function_tolerance;
    double ceres_gradient_tolerance;
    double ceres_parameter_tolerance;
    double ceres_max_num_iterations;
    int32_t solver_type; /* 0 HYBRID, 1 EPI_ONLY, 2 MD_ONLY */
    int32_t score_type;
    int32_t lo_type;
    int32_t min_depth_constraint;
    int32_t use_shift;
    int32_t ceres_use_nonmonotonic_steps;
    int32_t ceres_num_threads;
    int32_t reserved;
} mp_estimator_config;

/* PoseScaleOffset{,SharedFocal,TwoFocal} (src/pose.h:7-56); R row-major, x1 = R x0 + t */
typedef struct mp_model {
    double R[9];
    double t[3];
    double scale, offset0, offset1;
    double focal0, focal1; /* SF: focal0 == focal1 == focal */
} mp_model;

/* HybridRansacStatistics (src/bindings.cpp:67-76) + engine counters */
typedef struct mp_stats {
    double best_model_score;
    double inlier_ratios[3];
    uint64_t num_hypotheses;       /* models scored by minimal-sample iterations */
    uint64_t num_lo_sweeps;        /* full 3N sweeps issued by LO / termination   */
    uint32_t num_iterations_total;
    uint32_t num_iterations_per_solver[2];
    int32_t best_num_inliers;
    int32_t best_solver_type;
    int32_t number_lo_iterations;
    int32_t num_inliers[3]; /* lengths of the three inlier lists */
    int32_t num_batches;     /* speculative GPU batches issued */
    double seconds_total, seconds_lo, seconds_gpu_wait;
} mp_stats;

/* Full estimator.  Replaces
 *   HybridEstimatePoseScaleOffset            (src/hybrid_pose_estimator.cpp:8-35, bindings.cpp:169-170)
 *   HybridEstimatePoseScaleOffsetSharedFocal (src/hybrid_pose_shared_focal_estimator.cpp:8-51, :171-172)
 *   HybridEstimatePoseScaleOffsetTwoFocal    (src/hybrid_pose_two_focal_estimator.cpp:34-75, :173-174)
 *   HybridEstimatePoseAndScale               (src/hybrid_pose_estimator.cpp:37-63, 297-442, :167-168)
 * x0, x1: n x 2 row-major pixels; d0, d1: n depth priors; min_depth[2];
 * cam0/cam1: K (9, row-major) for MP_CALIBRATED, principal point (2) otherwise.
 * inlier_idx: optional caller buffer of 3*n int32; list t starts at t*n and has
 * stats->num_inliers[t] entries (reproj0, reproj1, sampson). */
int mp_estimate(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                const double *min_depth, const double *cam0, const double *cam1, const mp_ransac_options *options,
                const mp_estimator_config *config, mp_model *out_model, mp_stats *out_stats, int32_t *inlier_idx,
                int device);

/* estimate_scale_and_pose(X, Y, W) (src/solver.cpp:5-33, binding src/bindings.cpp:156):
 * weighted Procrustes with scale, Y ~ scale R X + t; X, Y point-major n x 3. */
int mp_estimate_scale_and_pose(const double *X, const double *Y, const double *W, int64_t n, mp_model *out,
                               int device);

/* Many independent pairs in one call (pairs concatenated; offsets[p]..offsets[p+1]).
 * min_depth: 2 per pair; cams: 9 or 2 doubles per pair; inlier buffers per pair at
 * 3*offsets[p].  Pairs run concurrently on one device. */
int mp_estimate_batch(int variant, int32_t num_pairs, const int64_t *offsets, const double *x0, const double *x1,
                      const double *d0, const double *d1, const double *min_depth, const double *cam0,
                      const double *cam1, const mp_ransac_options *options, const mp_estimator_config *config,
                      mp_model *out_models, mp_stats *out_stats, int32_t *inlier_idx, int device, int num_streams);

/* solve_scale_and_shift{,_shared_focal,_two_focal} (src/solver.cpp:35-480, bindings.cpp:157-161).
 * x_homo, y_homo: K homogeneous points stored point-major (3*K doubles: x,y,w per point),
 * K = 3 (cal) or 4 (sf/tf).  out: max_out rows of width 4/5/6; returns count (>=0) or -code. */
int mp_solve_scale_and_shift(int variant, const double *x_homo, const double *y_homo, const double *depth_x,
                             const double *depth_y, double *out, int max_out, int device);

/* solve_scale_shift_pose{,_shared_focal,_two_focal} (src/solver.cpp:482-534, 682-739, 986-1043,
 * wrappers 1408-1433, bindings.cpp:162-166).  Returns count or -code. */
int mp_solve_scale_shift_pose(int variant, const double *x_homo, const double *y_homo, const double *depth_x,
                              const double *depth_y, mp_model *out, int max_out, int device);

/* Option-gated alternates of the MD solvers (HybridLORansacOptions::use_ours / use_4p4d):
 * alt 1 = solve_scale_shift_pose{,_shared_focal,_two_focal}_ours (src/solver.cpp:623-680,
 * 818-984, 1045-1148), alt 2 = solve_scale_shift_pose_two_focal_4p4d (:1287-1406).
 * Same point layout as mp_solve_scale_shift_pose.  Returns count or -code. */
int mp_solve_scale_shift_pose_alt(int variant, int alt, const double *x_homo, const double *y_homo,
                                  const double *depth_x, const double *depth_y, mp_model *out, int max_out, int device);

/* Batched device sweep over one pair's correspondences (ScoreModel / GetInliers,
 * src/hybrid_ransac.h:265-349) for num_models models given in problem units.
 * Used by tests to check the scoring kernel directly.  scores: num_models;
 * errors (optional): num_models x 3 x n squared errors (is_for_inlier = true). */
int mp_score_models(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                    const double *cam0, const double *cam1, const mp_ransac_options *options,
                    const mp_estimator_config *config, const mp_model *models, int32_t num_models, double *scores,
                    double *errors, int device);

/* mp_debug_score_batch: the estimator's scoring kernel (score_batch) on explicit
 * model lists -- test hook.  models: num_iterations x M (M = 10 / 16 / 4 for the
 * calibrated / shared-focal / two-focal variant, problem units), counts[b] of them
 * used by iteration b.  best: the pre-batch best; flags: 1 the exact early exit
 * against it, 2 the record skip.  Outputs per iteration: res_best, res_slot (bit 16:
 * another model's screening interval reaches the best's; bit 17: a correspondence
 * outside the margins' cover was flagged), rec_models[b] (the mapped record model,
 * written when the iteration could hold a new best), res_hi_lo (nullable, 2 per
 * iteration: best + its margin, min over models of score - margin), model_ties
 * (nullable, num_iterations x M: each model's screening margin). */
int mp_debug_score_batch(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                         const double *d1, const double *cam0, const double *cam1, const mp_ransac_options *options,
                         const mp_estimator_config *config, int32_t num_iterations, const int32_t *counts,
                         const mp_model *models, double best, int32_t flags, double *res_best, int32_t *res_slot,
                         mp_model *rec_models, double *res_hi_lo, double *model_ties, int device);

/* mp_debug_score_terms: score_batch's residual evaluation of explicit models, per
 * correspondence -- test hook of the screening margins.  errors: num_models x 3 x n
 * (reprojection 0 -> 1, 1 -> 0, Sampson; the score kernel's own forms and gating);
 * flags: num_models x n (1: the correspondence lies outside the margins' cover); taus
 * (nullable): num_models x 3 per-term bounds; ties (nullable): each model's margin. */
int mp_debug_score_terms(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                         const double *d1, const double *cam0, const double *cam1, const mp_ransac_options *options,
                         const mp_estimator_config *config, const mp_model *models, int32_t num_models, double *errors,
                         int32_t *flags, double *taus, double *ties, int device);

/* mp_debug_lo_sweep: the same models through the engine's host LO sweep
 * (madpose_amd/csrc/host/lo_sweep.h), the sweep LocalOptimization and
 * UpdateRANSACTerminationCriteria use (src/hybrid_ransac.h:265-349, 383-538): errors
 * and ScoreModel sums in the reference's operation order -- test hook, no device.
 * fast_bounds (nullable, 2 per model): the LO's fast sum of the same terms and its
 * bound on the distance to the reference-order sum (lo_sweep.h lo_sweep_fast). */
int mp_debug_lo_sweep(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                      const double *cam0, const double *cam1, const mp_ransac_options *options,
                      const mp_estimator_config *config, const mp_model *models, int32_t num_models, double *scores,
                      double *errors, double *fast_bounds);

/* get_depths (madpose/utils.py:4-22) for many pairs in one launch: pair p's depth map
 * (dims[4p] x dims[4p+1], row-major, float32 for dtype 0 or float64 for dtype 1) is
 * stored after the previous pairs' maps in depth_maps; dims[4p+2], dims[4p+3] are the
 * image height and width the keypoints refer to; its keypoints (x, y pairs, float64)
 * are keypoints[2 pt_offsets[p] .. 2 pt_offsets[p+1]) and the depths go to
 * out[pt_offsets[p] ..] (dtype of the maps).  Same rounding (half to even), clipping
 * and [y, x] lookup as the reference's numpy code, so results are bit-identical. */
int mp_get_depths(int dtype, int32_t num_pairs, const void *depth_maps, const int64_t *dims, const int64_t *pt_offsets,
                  const double *keypoints, void *out, int device);

/* Batched device Levenberg-Marquardt: the Ceres solves of the local
 * optimisation -- HybridPoseOptimizer* (src/optimizer.h:48-125, SF :265-369, TF
 * :383-499) over the cost functors of src/cost_functions.h:16-387, as called by
 * LeastSquares (kinds[j] = 0; src/hybrid_pose_estimator.cpp:263-295) or
 * NonMinimalSolver (1; :188-214) -- for num_problems problems on one pair, one device
 * workgroup each.  Problem j refines models[j] (in/out, problem units: SF/TF focals
 * divided by the pair's normalize_points scale) over the residual blocks
 * sample_idx[sample_offsets[3j] ..) (reprojection 0->1), [sample_offsets[3j+1] ..)
 * (1->0), [sample_offsets[3j+2] .. sample_offsets[3j+3]) (Sampson).  status[j]: 1
 * refined, 0 no residuals, 2 infeasible constant bounded block, 3 too few data for
 * the solver (model unchanged in cases 0, 2, 3).  Options and config as mp_estimate
 * (thresholds / weights / Ceres settings); min_depth may be NULL (zeros). */
int mp_lm_refine_batch(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                       const double *d1, const double *min_depth, const double *cam0, const double *cam1,
                       const mp_ransac_options *options, const mp_estimator_config *config, int32_t num_problems,
                       const int32_t *kinds, const int64_t *sample_offsets, const int32_t *sample_idx,
                       mp_model *models, int32_t *status, int device);

/* mp_debug_lm_refine_host: the same problems through the engine's host LM (the
 * default LO path) -- test hook, no device needed. */
int mp_debug_lm_refine_host(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                            const double *d1, const double *min_depth, const double *cam0, const double *cam1,
                            const mp_ransac_options *options, const mp_estimator_config *config, int32_t num_problems,
                            const int32_t *kinds, const int64_t *sample_offsets, const int32_t *sample_idx,
                            mp_model *models, int32_t *status);

/* bougnoux_focals (src/hybrid_pose_two_focal_estimator.cpp:11-32; numpy twin
 * madpose/utils.py:25-56 bougnoux_numpy with p1 = p2 = 0): squared focal lengths
 * (f0^2, f1^2) of k fundamental matrices F (k x 9, row-major) into out (k x 2), on
 * the device with the same code the two-focal 7-point tail runs. */
int mp_bougnoux_focals(int64_t k, const double *F, double *out, int device);

/* compute_pose_error (madpose/utils.py:59-78) of k estimated poses against their
 * ground truth on the device, and the pose AUC of the evaluation the reference's
 * README reports (ScanNet-1500 AUC@5/10/20, README.md:18-181):
 * R: k x 9 row-major, t: k x 3, T_0to1: k x 16 (row-major 4x4); t_thres < 0 means
 * none (else err_t = 0 where |t_gt| < t_thres).  err_t, err_R: k degrees each.  When
 * nthr > 0, aucs[b] = area under the recall curve of max(err_R, err_t) up to
 * thresholds[b], divided by it (trapezoid rule, NaN errors sorted last; the
 * SuperGlue-style pose_auc of madpose_amd/utils.py); k = 0 gives NaN. */
int mp_pose_eval(int64_t k, const double *R, const double *t, const double *T_0to1, double t_thres, double *err_t,
                 double *err_R, int32_t nthr, const double *thresholds, double *aucs, int device);
/* The same pose AUC over k given errors (degrees; e.g. max(err_R, err_t) gathered
 * from many ranks): aucs[b] for thresholds[b], b < nthr. */
int mp_pose_auc(int64_t k, const double *errors, int32_t nthr, const double *thresholds, double *aucs, int device);

/* Point minimal solver (PoseLib relpose_5pt, src/hybrid_pose_estimator.cpp:134) on unit bearings
 * (5 points, point-major 3 doubles each).  Returns count or -code. */
int mp_relpose_5pt(const double *x1, const double *x2, mp_model *out, int max_out, int device);
/* mp_debug_pt5_roots: the engine's batched root stage of the calibrated 5-point
 * solver (the part of PoseLib relpose_5pt before pose recovery) over ns samples of
 * five normalized image points (pts0, pts1: ns x 5 x 2, identity intrinsics).
 * impl must be 1 (one 16-lane group per sample, the estimator's stage).  cand: ns x 96
 * doubles, 9 per essential matrix (ascending roots); ncand: ns counts.  Test hook. */
int mp_debug_pt5_roots(int impl, int64_t ns, const double *pts0, const double *pts1, double *cand, int32_t *ncand,
                       int device);
/* mp_debug_pt_roots: the same for variant 0 (calibrated 5-point, impl 1, as above) or
 * 1 (shared-focal 6-point, impl 3: the root stage of PoseLib relpose_6pt_shared_focal
 * as called at src/hybrid_pose_shared_focal_estimator.cpp:87, by the deflated
 * eigenproblem the estimator runs; pts0/pts1: ns x 6 x 2 normalized points; cand per
 * sample: the 3x9 epipolar null-space basis N, then the positive roots u = f^2 of the
 * degree-15 focal polynomial, ascending), or 2 (two-focal 7-point, impl 1: the root stage of
 * PoseLib relpose_7pt as called at src/hybrid_pose_two_focal_estimator.cpp:116; pts0/pts1: ns x 7
 * x 2 normalized points; cand per sample: the unit-norm fundamental matrices, 9 doubles each,
 * in root order).  Other impl values return MP_EINVAL.  Test hook. */
int mp_debug_pt_roots(int variant, int impl, int64_t ns, const double *pts0, const double *pts1, double *cand,
                      int32_t *ncand, int device);

/* Point minimal solvers of the uncalibrated estimators on 2-D points in the
 * estimators' normalized pixel frame ((x - pp) / s, point-major, 2 doubles each),
 * bearings formed as at src/hybrid_pose_shared_focal_estimator.cpp:79-84:
 *   6pt: PoseLib relpose_6pt_shared_focal (:87); out.focal0 = out.focal1 = f.
 *   7pt: PoseLib relpose_7pt + bougnoux_focals + cv::recoverPose
 *        (src/hybrid_pose_two_focal_estimator.cpp:116-146); out.focal0/1 = f0/f1.
 * Models are returned before the depth fit (scale 1, offsets 0).  Returns count or -code. */
int mp_relpose_6pt_shared_focal(const double *x0, const double *x1, mp_model *out, int max_out, int device);
int mp_relpose_7pt_two_focal(const double *x0, const double *x1, mp_model *out, int max_out, int device);

/* Test hooks for the host-side random streams (no device needed).
 * mp_debug_random_stream: kind 0 raw mt19937 words, 1 uniform_int(a, b),
 * 2 uniform_real(0, b), 3 uniform_int(i % 300, 300 + i % 17) for i = 0..count-1.
 * mp_debug_iteration_stream: the solver-type / minimal-sample sequence the engine
 * replays (SelectMinimalSolver + HybridUniformSampling, src/hybrid_ransac.h:64,
 * 98-109); idx holds 8 slots per iteration (unused slots -1). */
int mp_debug_random_stream(int kind, uint32_t seed, int32_t a, int32_t b, int32_t count, double *out);
int mp_debug_iteration_stream(int variant, int32_t n, uint32_t seed, int32_t solver_type, int32_t iterations,
                              int32_t *types, int32_t *idx);

/* Device timing of the estimator's batch kernels (engine-internal; no reference
 * counterpart).  Durations come from HIP events recorded on the engine's stream
 * around each launch and are process-wide totals since the last reset. */
typedef struct mp_kernel_profile {
    uint64_t batches;         /* speculative batches timed                  */
    uint64_t iterations;      /* minimal samples solved                     */
    uint64_t hypotheses;      /* models scored by the score_batch kernel    */
    uint64_t correspondences; /* sum of hypotheses x n over timed batches   */
    uint64_t sweeps;          /* single-model LO / termination sweeps       */
    double solve_ms;          /* md_solve + pt_solve kernels                */
    double score_ms;          /* score_batch kernel                         */
    uint64_t lm_calls;        /* host LM solves inside LO                   */
    double lm_wall_ms;        /* host wall time spent in the LM             */
    double sweep_wall_ms;     /* host wall time of LO sweeps (incl. copies) */
    double sample_wall_ms;    /* host minimal-sample generation + rewinds   */
    double wait_wall_ms;      /* host wait for speculative batch results    */
    double run_wall_ms;       /* whole estimator runs                       */
    uint64_t lm_blocks;       /* residual blocks over all LM solves         */
    uint64_t lm_big_calls;    /* LM solves with >= 1024 residual blocks     */
    double lm_big_wall_ms;    /* host wall time of those                    */
    uint64_t model_trips;     /* score_batch: (model, 256-correspondence trip)
                                 pairs evaluated (early exit stops short)     */
    uint64_t model_trips_full;/* the same without the early exit            */
    uint64_t accepted;        /* hypotheses of the iterations the estimator
                                 consumed (the rest was speculative)          */
    uint64_t scored;          /* hypotheses whose score_batch sweep ran (the
                                 record skip drops iterations past a batch's
                                 first new best; `hypotheses` counts them)     */
    uint64_t tie_checks;      /* iterations whose new-best decision was re-scored
                                 in the reference's order (near ties)         */
} mp_kernel_profile;
int mp_profile_enable(int on);
int mp_profile_reset(void);
int mp_profile_read(mp_kernel_profile *out);

const char *mp_last_error(void);

/* The host LM pool's spin-before-block in microseconds (engine-internal): the
 * MADPOSE_LO_SPIN environment value, else 300, or 0 when the process's CPU affinity
 * share holds fewer than 12 CPUs per rank of LOCAL_WORLD_SIZE. */
int mp_lo_spin_us(void);
int mp_device_count(void);
const char *mp_version(void);

#ifdef __cplusplus
}
#endif
#endif
