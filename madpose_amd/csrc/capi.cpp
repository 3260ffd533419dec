// extern "C" boundary: include/madpose_mi355x.h
#include <atomic>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/madpose_mi355x.h"
#include "host/engine.h"
#include "host/rng.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

mp::RansacOptions to_opts(const mp_ransac_options *o) {
    mp::RansacOptions r;
    r.success_probability = o->success_probability;
    r.squared_inlier_thresholds[0] = o->squared_inlier_thresholds[0];
    r.squared_inlier_thresholds[1] = o->squared_inlier_thresholds[1];
    r.data_type_weights[0] = o->data_type_weights[0];
    r.data_type_weights[1] = o->data_type_weights[1];
    r.threshold_multiplier = o->threshold_multiplier;
    r.min_num_iterations = o->min_num_iterations;
    r.max_num_iterations = o->max_num_iterations;
    r.max_num_iterations_per_solver = o->max_num_iterations_per_solver;
    r.random_seed = o->random_seed;
    r.num_lo_steps = o->num_lo_steps;
    r.num_lsq_iterations = o->num_lsq_iterations;
    r.min_sample_multiplicator = o->min_sample_multiplicator;
    r.non_min_sample_multiplier = o->non_min_sample_multiplier;
    r.lo_starting_iterations = o->lo_starting_iterations;
    r.final_least_squares = o->final_least_squares != 0;
    r.use_ours = o->use_ours != 0;
    r.use_4p4d = o->use_4p4d != 0;
    return r;
}

mp::EstimatorConfig to_cfg(const mp_estimator_config *c) {
    mp::EstimatorConfig r;
    if (!c) return r;
    r.solver_type = c->solver_type;
    r.score_type = c->score_type;
    r.lo_type = c->lo_type;
    r.min_depth_constraint = c->min_depth_constraint != 0;
    r.use_shift = c->use_shift != 0;
    r.ftol = c->ceres_function_tolerance;
    r.gtol = c->ceres_gradient_tolerance;
    r.ptol = c->ceres_parameter_tolerance;
    r.max_iter = c->ceres_max_num_iterations;
    r.nonmonotonic = c->ceres_use_nonmonotonic_steps != 0;
    return r;
}

void to_model(const mp::Model &m, mp_model *o) {
    static_assert(sizeof(mp::Model) == sizeof(mp_model), "model layout");
    std::memcpy(o, &m, sizeof(mp_model));
}

void fill_stats(const mp::Stats &S, int64_t n, mp_stats *o, int32_t *inlier_idx) {
    std::memset(o, 0, sizeof(*o));
    o->best_model_score = S.best_model_score;
    for (int t = 0; t < 3; ++t) {
        o->inlier_ratios[t] = S.inlier_ratios[t];
        o->num_inliers[t] = (int32_t)S.inlier_indices[t].size();
        if (inlier_idx)
            for (size_t k = 0; k < S.inlier_indices[t].size(); ++k) inlier_idx[t * n + (int64_t)k] = S.inlier_indices[t][k];
    }
    o->num_hypotheses = S.num_hypotheses;
    o->num_lo_sweeps = S.num_lo_sweeps;
    o->num_iterations_total = S.num_iterations_total;
    o->num_iterations_per_solver[0] = S.num_iterations_per_solver[0];
    o->num_iterations_per_solver[1] = S.num_iterations_per_solver[1];
    o->best_num_inliers = S.best_num_inliers;
    o->best_solver_type = S.best_solver_type;
    o->number_lo_iterations = S.number_lo_iterations;
    o->num_batches = S.num_batches;
    o->seconds_total = S.seconds_total;
    o->seconds_lo = S.seconds_lo;
    o->seconds_gpu_wait = S.seconds_gpu_wait;
}

mp::PairInput make_input(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                         const double *d1, const double *min_depth, const double *cam0, const double *cam1) {
    mp::PairInput in;
    in.variant = variant;
    in.n = n;
    in.x0 = x0;
    in.x1 = x1;
    in.d0 = d0;
    in.d1 = d1;
    if (min_depth) {
        in.min_depth[0] = min_depth[0];
        in.min_depth[1] = min_depth[1];
    }
    const int nc = (variant == MP_CALIBRATED || variant == MP_SCALE_ONLY) ? 9 : 2;
    if (!cam0 || !cam1) throw std::invalid_argument("camera parameters missing");
    std::memcpy(in.cam0, cam0, sizeof(double) * nc);
    std::memcpy(in.cam1, cam1, sizeof(double) * nc);
    return in;
}

template <class F> int guarded(F f) {
    try {
        return f();
    } catch (const std::invalid_argument &e) {
        return fail(MP_EINVAL, e.what());
    } catch (const std::exception &e) {
        return fail(MP_EDEVICE, e.what());
    } catch (...) {
        return fail(MP_EDEVICE, "unknown error");
    }
}

} // namespace

extern "C" {

int mp_estimate(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                const double *min_depth, const double *cam0, const double *cam1, const mp_ransac_options *options,
                const mp_estimator_config *config, mp_model *out_model, mp_stats *out_stats, int32_t *inlier_idx,
                int device) {
    return guarded([&]() {
        if (!options || !out_model || !out_stats) throw std::invalid_argument("null options / outputs");
        mp::PairInput in = make_input(variant, n, x0, x1, d0, d1, min_depth, cam0, cam1);
        mp::Model m;
        mp::Stats S;
        mp::estimate_pair(in, to_opts(options), to_cfg(config), device, &m, &S);
        to_model(m, out_model);
        fill_stats(S, n, out_stats, inlier_idx);
        return MP_OK;
    });
}

int mp_estimate_batch(int variant, int32_t num_pairs, const int64_t *offsets, const double *x0, const double *x1,
                      const double *d0, const double *d1, const double *min_depth, const double *cam0,
                      const double *cam1, const mp_ransac_options *options, const mp_estimator_config *config,
                      mp_model *out_models, mp_stats *out_stats, int32_t *inlier_idx, int device, int num_streams) {
    return guarded([&]() {
        if (num_pairs < 0 || !offsets || !options || !out_models || !out_stats)
            throw std::invalid_argument("bad batch arguments");
        const int nc = (variant == MP_CALIBRATED || variant == MP_SCALE_ONLY) ? 9 : 2;
        const mp::RansacOptions opts = to_opts(options);
        const mp::EstimatorConfig cfg = to_cfg(config);
        std::atomic<int> next(0);
        std::vector<std::string> errors(num_pairs);
        std::vector<int> codes(num_pairs, MP_OK);
        auto worker = [&]() {
            for (;;) {
                const int p = next.fetch_add(1);
                if (p >= num_pairs) break;
                const int64_t o = offsets[p], n = offsets[p + 1] - offsets[p];
                try {
                    mp::PairInput in = make_input(variant, n, x0 + 2 * o, x1 + 2 * o, d0 + o, d1 + o,
                                                  min_depth + 2 * p, cam0 + nc * p, cam1 + nc * p);
                    mp::Model m;
                    mp::Stats S;
                    mp::estimate_pair(in, opts, cfg, device, &m, &S);
                    to_model(m, &out_models[p]);
                    fill_stats(S, n, &out_stats[p], inlier_idx ? inlier_idx + 3 * o : nullptr);
                } catch (const std::invalid_argument &e) {
                    codes[p] = MP_EINVAL;
                    errors[p] = e.what();
                } catch (const std::exception &e) {
                    codes[p] = MP_EDEVICE;
                    errors[p] = e.what();
                }
            }
        };
        const int nt = std::max(1, std::min(num_streams, std::max(num_pairs, 1)));
        std::vector<std::thread> threads;
        for (int t = 0; t < nt; ++t) threads.emplace_back(worker);
        for (auto &t : threads) t.join();
        for (int p = 0; p < num_pairs; ++p)
            if (codes[p] != MP_OK) return fail(codes[p], "pair " + std::to_string(p) + ": " + errors[p]);
        return MP_OK;
    });
}

int mp_get_depths(int dtype, int32_t num_pairs, const void *depth_maps, const int64_t *dims, const int64_t *pt_offsets,
                  const double *keypoints, void *out, int device) {
    return guarded([&]() {
        if (num_pairs < 0 || (num_pairs > 0 && (!depth_maps || !dims || !pt_offsets || !out)))
            throw std::invalid_argument("bad get_depths arguments");
        mp::get_depths_batch(dtype, num_pairs, depth_maps, dims, pt_offsets, keypoints, out, device);
        return MP_OK;
    });
}

int mp_bougnoux_focals(int64_t k, const double *F, double *out, int device) {
    return guarded([&]() {
        if (k < 0 || (k > 0 && (!F || !out))) throw std::invalid_argument("bad bougnoux arguments");
        mp::bougnoux_batch(k, F, out, device);
        return MP_OK;
    });
}

int mp_pose_eval(int64_t k, const double *R, const double *t, const double *T_0to1, double t_thres, double *err_t,
                 double *err_R, int32_t nthr, const double *thresholds, double *aucs, int device) {
    return guarded([&]() {
        if (k < 0 || nthr < 0 || (k > 0 && (!R || !t || !T_0to1 || !err_t || !err_R)) ||
            (nthr > 0 && (!thresholds || !aucs)))
            throw std::invalid_argument("bad pose_eval arguments");
        for (int b = 0; b < nthr; ++b)
            if (!(thresholds[b] > 0.0)) throw std::invalid_argument("AUC thresholds must be positive");
        mp::pose_eval_batch(k, R, t, T_0to1, t_thres, err_t, err_R, nthr, thresholds, aucs, device);
        return MP_OK;
    });
}

int mp_pose_auc(int64_t k, const double *errors, int32_t nthr, const double *thresholds, double *aucs, int device) {
    return guarded([&]() {
        if (k < 0 || nthr < 0 || (k > 0 && !errors) || (nthr > 0 && (!thresholds || !aucs)))
            throw std::invalid_argument("bad pose_auc arguments");
        for (int b = 0; b < nthr; ++b)
            if (!(thresholds[b] > 0.0)) throw std::invalid_argument("AUC thresholds must be positive");
        mp::pose_auc_batch(k, errors, nthr, thresholds, aucs, device);
        return MP_OK;
    });
}

int mp_estimate_scale_and_pose(const double *X, const double *Y, const double *W, int64_t n, mp_model *out,
                               int device) {
    return guarded([&]() {
        if (!X || !Y || !W || !out || n < 1) throw std::invalid_argument("bad arguments");
        mp::Model m;
        mp::scale_and_pose_direct(X, Y, W, n, &m, device);
        to_model(m, out);
        return MP_OK;
    });
}

int mp_solve_scale_and_shift(int variant, const double *x_homo, const double *y_homo, const double *depth_x,
                             const double *depth_y, double *out, int max_out, int device) {
    int r = guarded([&]() {
        if (variant < 0 || variant > 2) throw std::invalid_argument("bad variant");
        mp::Model poses[8];
        int np = 0;
        int n = mp::solve_md_direct(variant, x_homo, y_homo, depth_x, depth_y, out, max_out, poses, 8, &np, device);
        return -(n + 1000); // encode count through the guard
    });
    return r <= -1000 ? -(r + 1000) : -r;
}

int mp_solve_scale_shift_pose(int variant, const double *x_homo, const double *y_homo, const double *depth_x,
                              const double *depth_y, mp_model *out, int max_out, int device) {
    int r = guarded([&]() {
        if (variant < 0 || variant > 2) throw std::invalid_argument("bad variant");
        double sols[48];
        mp::Model poses[8];
        int np = 0;
        mp::solve_md_direct(variant, x_homo, y_homo, depth_x, depth_y, sols, 8, poses, 8, &np, device);
        for (int i = 0; i < std::min(np, max_out); ++i) to_model(poses[i], &out[i]);
        return -(np + 1000);
    });
    return r <= -1000 ? -(r + 1000) : -r;
}

int mp_solve_scale_shift_pose_alt(int variant, int alt, const double *x_homo, const double *y_homo,
                                  const double *depth_x, const double *depth_y, mp_model *out, int max_out, int device) {
    int r = guarded([&]() {
        if (variant < 0 || variant > 2) throw std::invalid_argument("bad variant");
        if (alt < 1 || alt > 2 || (alt == 2 && variant != 2))
            throw std::invalid_argument("alt must be 1 (use_ours) or 2 (use_4p4d, two-focal only)");
        double sols[48];
        mp::Model poses[8];
        int np = 0;
        mp::solve_md_direct(variant, x_homo, y_homo, depth_x, depth_y, sols, 8, poses, 8, &np, device, alt);
        for (int i = 0; i < std::min(np, max_out); ++i) to_model(poses[i], &out[i]);
        return -(np + 1000);
    });
    return r <= -1000 ? -(r + 1000) : -r;
}

extern "C++" {
namespace {
// the shared argument handling of mp_score_models and mp_debug_lo_sweep: `sweep`
// receives the pair, the converted options and the models
template <class F>
int with_models(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                const double *cam0, const double *cam1, const mp_ransac_options *options,
                const mp_estimator_config *config, const mp_model *models, int32_t num_models, double *scores,
                F &&sweep) {
    return guarded([&]() {
        if (!options || !models || !scores || num_models < 0) throw std::invalid_argument("bad arguments");
        const double md[2] = {0.0, 0.0};
        mp::PairInput in = make_input(variant, n, x0, x1, d0, d1, md, cam0, cam1);
        std::vector<mp::Model> ms(num_models);
        std::memcpy(ms.data(), models, sizeof(mp_model) * num_models);
        sweep(in, to_opts(options), to_cfg(config), ms);
        return MP_OK;
    });
}
} // namespace
} // extern "C++"

int mp_score_models(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                    const double *cam0, const double *cam1, const mp_ransac_options *options,
                    const mp_estimator_config *config, const mp_model *models, int32_t num_models, double *scores,
                    double *errors, int device) {
    return with_models(variant, n, x0, x1, d0, d1, cam0, cam1, options, config, models, num_models, scores,
                       [&](const mp::PairInput &in, const mp::RansacOptions &o, const mp::EstimatorConfig &c,
                           std::vector<mp::Model> &ms) {
                           mp::score_models(in, o, c, ms.data(), num_models, scores, errors, device, nullptr);
                       });
}

int mp_debug_score_batch(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                         const double *d1, const double *cam0, const double *cam1, const mp_ransac_options *options,
                         const mp_estimator_config *config, int32_t num_iterations, const int32_t *counts,
                         const mp_model *models, double best, int32_t flags, double *res_best, int32_t *res_slot,
                         mp_model *rec_models, double *res_hi_lo, double *model_ties, int device) {
    return guarded([&]() {
        if (!options || !counts || !models || !res_best || !res_slot || num_iterations <= 0)
            throw std::invalid_argument("bad arguments");
        const double md[2] = {0.0, 0.0};
        mp::PairInput in = make_input(variant, n, x0, x1, d0, d1, md, cam0, cam1);
        const int maxm = mp::max_models(variant == 3 ? 0 : variant);
        std::vector<mp::Model> ms((size_t)num_iterations * maxm), rm(num_iterations);
        std::memcpy(ms.data(), models, sizeof(mp_model) * ms.size());
        mp::debug_score_batch(in, to_opts(options), to_cfg(config), num_iterations, counts, ms.data(), best, flags,
                              res_best, res_slot, rm.data(), res_hi_lo, model_ties, device);
        if (rec_models)
            for (int b = 0; b < num_iterations; ++b) to_model(rm[b], &rec_models[b]);
        return MP_OK;
    });
}

int mp_debug_score_terms(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                         const double *d1, const double *cam0, const double *cam1, const mp_ransac_options *options,
                         const mp_estimator_config *config, const mp_model *models, int32_t num_models, double *errors,
                         int32_t *flags, double *taus, double *ties, int device) {
    return guarded([&]() {
        if (!options || !models || !errors || !flags || num_models < 0) throw std::invalid_argument("bad arguments");
        const double md[2] = {0.0, 0.0};
        mp::PairInput in = make_input(variant, n, x0, x1, d0, d1, md, cam0, cam1);
        std::vector<mp::Model> ms(num_models);
        std::memcpy(ms.data(), models, sizeof(mp_model) * num_models);
        mp::debug_score_terms(in, to_opts(options), to_cfg(config), ms.data(), num_models, errors, flags, taus, ties,
                              device);
        return MP_OK;
    });
}

int mp_debug_lo_sweep(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                      const double *cam0, const double *cam1, const mp_ransac_options *options,
                      const mp_estimator_config *config, const mp_model *models, int32_t num_models, double *scores,
                      double *errors, double *fast_bounds) {
    return with_models(variant, n, x0, x1, d0, d1, cam0, cam1, options, config, models, num_models, scores,
                       [&](const mp::PairInput &in, const mp::RansacOptions &o, const mp::EstimatorConfig &c,
                           std::vector<mp::Model> &ms) {
                           mp::lo_sweep_models(in, o, c, ms.data(), num_models, scores, errors, fast_bounds);
                       });
}

extern "C++" {
namespace {
// the shared argument handling of mp_lm_refine_batch and mp_debug_lm_refine_host
template <class F>
int with_lm_problems(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                     const double *min_depth, const double *cam0, const double *cam1,
                     const mp_ransac_options *options, const mp_estimator_config *config, int32_t num_problems,
                     const int64_t *sample_offsets, const int32_t *sample_idx, mp_model *models, int32_t *status,
                     F &&refine) {
    return guarded([&]() {
        if (!options || num_problems < 0 || (num_problems > 0 && (!sample_offsets || !models || !status)))
            throw std::invalid_argument("bad arguments");
        if (num_problems > 0 && sample_offsets[3 * num_problems] > 0 && !sample_idx)
            throw std::invalid_argument("null sample indices");
        const double md0[2] = {0.0, 0.0};
        mp::PairInput in = make_input(variant, n, x0, x1, d0, d1, min_depth ? min_depth : md0, cam0, cam1);
        std::vector<mp::Model> ms(num_problems);
        std::memcpy(ms.data(), models, sizeof(mp_model) * num_problems);
        refine(in, to_opts(options), to_cfg(config), ms);
        for (int j = 0; j < num_problems; ++j) to_model(ms[j], &models[j]);
        return MP_OK;
    });
}
} // namespace
} // extern "C++"

int mp_lm_refine_batch(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                       const double *d1, const double *min_depth, const double *cam0, const double *cam1,
                       const mp_ransac_options *options, const mp_estimator_config *config, int32_t num_problems,
                       const int32_t *kinds, const int64_t *sample_offsets, const int32_t *sample_idx,
                       mp_model *models, int32_t *status, int device) {
    return with_lm_problems(variant, n, x0, x1, d0, d1, min_depth, cam0, cam1, options, config, num_problems,
                            sample_offsets, sample_idx, models, status,
                            [&](const mp::PairInput &in, const mp::RansacOptions &o, const mp::EstimatorConfig &c,
                                std::vector<mp::Model> &ms) {
                                mp::lm_refine_batch_device(in, o, c, num_problems, kinds, sample_offsets, sample_idx,
                                                           ms.data(), status, device);
                            });
}

int mp_debug_lm_refine_host(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                            const double *d1, const double *min_depth, const double *cam0, const double *cam1,
                            const mp_ransac_options *options, const mp_estimator_config *config, int32_t num_problems,
                            const int32_t *kinds, const int64_t *sample_offsets, const int32_t *sample_idx,
                            mp_model *models, int32_t *status) {
    return with_lm_problems(variant, n, x0, x1, d0, d1, min_depth, cam0, cam1, options, config, num_problems,
                            sample_offsets, sample_idx, models, status,
                            [&](const mp::PairInput &in, const mp::RansacOptions &o, const mp::EstimatorConfig &c,
                                std::vector<mp::Model> &ms) {
                                mp::lm_refine_batch_host(in, o, c, num_problems, kinds, sample_offsets, sample_idx,
                                                         ms.data(), status);
                            });
}

static int point_direct(int kind, const double *x1, const double *x2, mp_model *out, int max_out, int device) {
    if (!x1 || !x2 || (max_out > 0 && !out)) return -fail(MP_EINVAL, "null argument");
    int r = guarded([&]() {
        mp::Model poses[16];
        int np = mp::solve_point_direct(kind, x1, x2, poses, 16, device);
        for (int i = 0; i < std::min(np, max_out); ++i) to_model(poses[i], &out[i]);
        return -(np + 1000);
    });
    return r <= -1000 ? -(r + 1000) : -r;
}

int mp_debug_pt_roots(int variant, int impl, int64_t ns, const double *pts0, const double *pts1, double *cand,
                      int32_t *ncand, int device) {
    if (!pts0 || !pts1 || !cand || !ncand) return fail(MP_EINVAL, "null pointer");
    // impl names the estimator's root stage: 1 for the 5-point (16-lane groups), 3 for
    // the 6-point (deflated eigenproblem), 1 for the 7-point (lane per sample); the
    // round-2 alternates left the library
    if ((variant == 0 && impl != 1) || (variant == 1 && impl != 3) || (variant == 2 && impl != 1) || variant < 0 ||
        variant > 2)
        return fail(MP_EINVAL, "impl must be 1 (5-point group stage, 7-point) or 3 (6-point eigen stage)");
    return guarded([&] {
        mp::debug_pt_roots(variant, ns, pts0, pts1, cand, ncand, device);
        return MP_OK;
    });
}

int mp_debug_pt5_roots(int impl, int64_t ns, const double *pts0, const double *pts1, double *cand, int32_t *ncand,
                       int device) {
    return mp_debug_pt_roots(0, impl, ns, pts0, pts1, cand, ncand, device);
}

int mp_relpose_5pt(const double *x1, const double *x2, mp_model *out, int max_out, int device) {
    return point_direct(0, x1, x2, out, max_out, device);
}

int mp_relpose_6pt_shared_focal(const double *x0, const double *x1, mp_model *out, int max_out, int device) {
    return point_direct(1, x0, x1, out, max_out, device);
}

int mp_relpose_7pt_two_focal(const double *x0, const double *x1, mp_model *out, int max_out, int device) {
    return point_direct(2, x0, x1, out, max_out, device);
}

int mp_debug_random_stream(int kind, uint32_t seed, int32_t a, int32_t b, int32_t count, double *out) {
    if (!out || count < 0) return fail(MP_EINVAL, "bad arguments");
    mp::Mt19937 g(seed);
    for (int i = 0; i < count; ++i) {
        if (kind == 0)
            out[i] = (double)g();
        else if (kind == 1)
            out[i] = (double)mp::uniform_int(g, a, b);
        else if (kind == 2)
            out[i] = mp::uniform_real(g, 0.0, (double)b);
        else if (kind == 3)
            out[i] = (double)mp::uniform_int(g, i % 300, 300 + (i % 17));
        else
            return fail(MP_EINVAL, "bad kind");
    }
    return MP_OK;
}

int mp_debug_iteration_stream(int variant, int32_t n, uint32_t seed, int32_t solver_type, int32_t iterations,
                              int32_t *types, int32_t *idx) {
    if (!types || !idx || iterations < 0 || n <= 0 || variant < 0 || variant > 2)
        return fail(MP_EINVAL, "bad arguments");
    mp::IterationStream rs;
    const int kmd = variant == MP_CALIBRATED ? 3 : 4;
    const int kpt = variant == MP_CALIBRATED ? 5 : (variant == MP_SHARED_FOCAL ? 6 : 7);
    const int ss[2][3] = {{kmd, kmd, 0}, {0, 0, kpt}};
    for (int s = 0; s < 2; ++s)
        for (int t = 0; t < 3; ++t) {
            rs.ss[s][t] = ss[s][t];
            if (ss[s][t] > n) rs.prior[s] = 0.0;
        }
    if (solver_type == 1) rs.prior[0] = 0.0;
    if (solver_type == 2) rs.prior[1] = 0.0;
    rs.n = n;
    rs.seed(seed);
    for (int k = 0; k < iterations; ++k) {
        int tmp[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
        types[k] = rs.next(tmp);
        for (int j = 0; j < 8; ++j) idx[8 * k + j] = tmp[j];
    }
    return MP_OK;
}

int mp_profile_enable(int on) {
    mp::profile_enable(on != 0);
    return MP_OK;
}
int mp_profile_reset(void) {
    mp::profile_reset();
    return MP_OK;
}
int mp_profile_read(mp_kernel_profile *out) {
    if (!out) return MP_EINVAL;
    const mp::KernelProfile p = mp::profile_read();
    out->batches = p.batches;
    out->iterations = p.iterations;
    out->hypotheses = p.hypotheses;
    out->correspondences = p.correspondences;
    out->sweeps = p.sweeps;
    out->solve_ms = p.solve_ms;
    out->score_ms = p.score_ms;
    out->lm_calls = p.lm_calls;
    out->lm_wall_ms = p.lm_wall_ms;
    out->sweep_wall_ms = p.sweep_wall_ms;
    out->sample_wall_ms = p.sample_wall_ms;
    out->wait_wall_ms = p.wait_wall_ms;
    out->run_wall_ms = p.run_wall_ms;
    out->lm_blocks = p.lm_blocks;
    out->lm_big_calls = p.lm_big_calls;
    out->lm_big_wall_ms = p.lm_big_wall_ms;
    out->model_trips = p.model_trips;
    out->model_trips_full = p.model_trips_full;
    out->accepted = p.accepted;
    out->scored = p.scored;
    out->tie_checks = p.tie_checks;
    return MP_OK;
}

const char *mp_last_error(void) { return g_last_error.c_str(); }

int mp_device_count(void) { return mp::device_count(); }

int mp_lo_spin_us(void) { return mp::lo_spin_us(); }

const char *mp_version(void) { return "madpose-mi355x 0.1.0 (gfx950)"; }

} // extern "C"
