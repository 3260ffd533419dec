// ORACLE -- test infrastructure only.  C entry points used by tests/ via ctypes.
// The option / model / stats structs mirror the field layout of the product's C ABI
// (include/madpose_mi355x.h) so the same Python objects can drive both sides; they
// are declared here independently so the oracle shares no code with the product.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <stdexcept>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

#include "la.h"
#include "oracle.h"

extern "C" {

struct or_ransac_options {
    double success_probability;
    double squared_inlier_thresholds[2];
    double data_type_weights[2];
    double threshold_multiplier;
    uint32_t min_num_iterations, max_num_iterations, max_num_iterations_per_solver, random_seed;
    int32_t num_lo_steps, num_lsq_iterations, min_sample_multiplicator, non_min_sample_multiplier;
    int32_t lo_starting_iterations, final_least_squares, use_ours, use_4p4d;
};
struct or_estimator_config {
    double ftol, gtol, ptol, max_iter;
    int32_t solver_type, score_type, lo_type, min_depth_constraint, use_shift, nonmono, threads, reserved;
};
struct or_model {
    double R[9], t[3], scale, offset0, offset1, focal0, focal1;
};
struct or_stats {
    double best_model_score;
    double inlier_ratios[3];
    uint64_t num_hypotheses, num_lo_sweeps;
    uint32_t num_iterations_total, num_iterations_per_solver[2];
    int32_t best_num_inliers, best_solver_type, number_lo_iterations, num_inliers[3], num_batches;
    double seconds_total, seconds_lo, seconds_gpu_wait;
};

static oracle::Options to_opts(const or_ransac_options *o) {
    oracle::Options r;
    r.success_probability = o->success_probability;
    r.squared_inlier_thresholds = {o->squared_inlier_thresholds[0], o->squared_inlier_thresholds[1]};
    r.data_type_weights = {o->data_type_weights[0], o->data_type_weights[1]};
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
static oracle::EstConfig to_cfg(const or_estimator_config *c) {
    oracle::EstConfig r;
    r.ceres_function_tolerance = c->ftol;
    r.ceres_gradient_tolerance = c->gtol;
    r.ceres_parameter_tolerance = c->ptol;
    r.ceres_max_num_iterations = c->max_iter;
    r.solver_type = c->solver_type;
    r.score_type = c->score_type;
    r.lo_type = c->lo_type;
    r.min_depth_constraint = c->min_depth_constraint != 0;
    r.use_shift = c->use_shift != 0;
    r.ceres_use_nonmonotonic_steps = c->nonmono != 0;
    r.ceres_num_threads = c->threads;
    return r;
}
static void put_model(const oracle::Model &m, or_model *o) {
    std::memcpy(o->R, m.R, sizeof(m.R));
    std::memcpy(o->t, m.t, sizeof(m.t));
    o->scale = m.scale;
    o->offset0 = m.offset0;
    o->offset1 = m.offset1;
    o->focal0 = m.focal0;
    o->focal1 = m.focal1;
}
static oracle::Model get_model(const or_model *o) {
    oracle::Model m;
    std::memcpy(m.R, o->R, sizeof(m.R));
    std::memcpy(m.t, o->t, sizeof(m.t));
    m.scale = o->scale;
    m.offset0 = o->offset0;
    m.offset1 = o->offset1;
    m.focal0 = o->focal0;
    m.focal1 = o->focal1;
    return m;
}

int oracle_md_scale_shift(int variant, const double *x, const double *y, const double *dx, const double *dy,
                          double *out, int max_out) {
    auto sols = oracle::md_scale_shift((oracle::Variant)variant, x, y, dx, dy);
    const int w = variant == 0 ? 4 : (variant == 1 ? 5 : 6);
    int n = std::min((int)sols.size(), max_out);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < w; ++j) out[i * w + j] = sols[i][j];
    return (int)sols.size();
}

// alt: 1 = use_ours, 2 = use_4p4d (two-focal only)
int oracle_md_pose_alt(int variant, int alt, const double *x, const double *y, const double *dx, const double *dy,
                       or_model *out, int max_out) {
    std::vector<oracle::Model> sols;
    if (alt == 1)
        sols = variant == 0 ? oracle::md_pose_cal_ours(x, y, dx, dy)
                            : (variant == 1 ? oracle::md_pose_sf_ours(x, y, dx, dy) : oracle::md_pose_tf_ours(x, y, dx, dy));
    else if (alt == 2 && variant == 2)
        sols = oracle::md_pose_tf_4p4d(x, y, dx, dy);
    int n = std::min((int)sols.size(), max_out);
    for (int i = 0; i < n; ++i) put_model(sols[i], &out[i]);
    return (int)sols.size();
}

int oracle_md_pose(int variant, const double *x, const double *y, const double *dx, const double *dy, or_model *out,
                   int max_out) {
    auto sols = oracle::md_pose((oracle::Variant)variant, x, y, dx, dy);
    int n = std::min((int)sols.size(), max_out);
    for (int i = 0; i < n; ++i) put_model(sols[i], &out[i]);
    return (int)sols.size();
}

int oracle_relpose_5pt(const double *x1, const double *x2, or_model *out, int max_out) {
    auto sols = oracle::relpose_5pt(x1, x2);
    int n = std::min((int)sols.size(), max_out);
    for (int i = 0; i < n; ++i) put_model(sols[i], &out[i]);
    return (int)sols.size();
}

// E candidates of the 5-point root stage and the roots z (ascending); returns the
// number of E (<= max_out written); *nroots = number of real roots (<= 10 written)
int oracle_relpose_5pt_E(const double *x1, const double *x2, double *E_out, int max_out, double *roots, int *nroots) {
    std::vector<double> rz;
    auto Es = oracle::relpose_5pt_E(x1, x2, &rz);
    const int n = std::min((int)Es.size(), max_out);
    for (int i = 0; i < n; ++i)
        for (int e = 0; e < 9; ++e) E_out[9 * i + e] = Es[i][e];
    *nroots = (int)rz.size();
    for (size_t k = 0; k < rz.size() && k < 10; ++k) roots[k] = rz[k];
    return (int)Es.size();
}

int oracle_relpose_5pt_action(const double *x1, const double *x2, or_model *out, int max_out) {
    auto sols = oracle::relpose_5pt_action(x1, x2);
    int n = std::min((int)sols.size(), max_out);
    for (int i = 0; i < n; ++i) put_model(sols[i], &out[i]);
    return (int)sols.size();
}

int oracle_relpose_7pt_svd(const double *x1, const double *x2, double *F_out, int max_out) {
    auto sols = oracle::relpose_7pt_svd(x1, x2);
    int n = std::min((int)sols.size(), max_out);
    for (int i = 0; i < n; ++i)
        for (int e = 0; e < 9; ++e) F_out[9 * i + e] = sols[i][e];
    return (int)sols.size();
}

// Eigen JacobiSVD restatement of a 3 x 3 matrix (la.cpp eigen_jacobi_svd3): U, V row-major
int oracle_eigen_svd3(const double *A, double *U, double *V) {
    oracle::eigen_jacobi_svd3(A, U, V);
    return 0;
}

int oracle_solve_cubic_real(double c2, double c1, double c0, double *roots) {
    return oracle::solve_cubic_real(c2, c1, c0, roots);
}

int oracle_scale_and_pose(const double *X, const double *Y, const double *W, int k, or_model *out) {
    put_model(oracle::estimate_scale_and_pose(X, Y, W, k), out);
    return 0;
}

int oracle_relpose_7pt(const double *x1, const double *x2, double *F_out, int max_out) {
    auto sols = oracle::relpose_7pt(x1, x2);
    int n = std::min((int)sols.size(), max_out);
    for (int i = 0; i < n; ++i)
        for (int e = 0; e < 9; ++e) F_out[9 * i + e] = sols[i][e];
    return (int)sols.size();
}

int oracle_bougnoux(const double *F, double *f_sq) {
    oracle::bougnoux_focals(F, &f_sq[0], &f_sq[1]);
    return 0;
}

int oracle_recover_pose(const double *E, const double *p0, const double *p1, int n, double thresh, double *R,
                        double *t) {
    return oracle::recover_pose(E, p0, p1, n, thresh, R, t);
}

int oracle_6pt_roots(const double *x1, const double *x2, double *out, int max_out) {
    const auto r = oracle::sixpt_roots_of(x1, x2);
    for (int k = 0; k < (int)r.size() && k < max_out; ++k) out[k] = r[k];
    return (int)r.size();
}

int oracle_relpose_6pt(const double *x1, const double *x2, or_model *out, int max_out) {
    auto sols = oracle::relpose_6pt_shared_focal(x1, x2);
    int n = std::min((int)sols.size(), max_out);
    for (int i = 0; i < n; ++i) put_model(sols[i], &out[i]);
    return (int)sols.size();
}

// Scores / per-point errors of given models (models in problem units, i.e. after
// the SF/TF normalisation).  errors: num_models x 3 x n (is_for_inlier = true).
int oracle_score_models(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                        const double *d1, const double *cam0, const double *cam1, const or_ransac_options *o,
                        const or_estimator_config *c, const or_model *models, int32_t nm, double *scores,
                        double *errors, double *norm_scale_out) {
    oracle::Options opts = to_opts(o);
    double md[2] = {0, 0};
    oracle::Problem P =
        oracle::make_problem((oracle::Variant)variant, (int)n, x0, x1, d0, d1, md, cam0, cam1, to_cfg(c), &opts);
    if (norm_scale_out) *norm_scale_out = P.norm_scale;
    for (int m = 0; m < nm; ++m) {
        oracle::Model mm = get_model(&models[m]);
        double s = 0;
        for (int t = 0; t < 3; ++t)
            for (int i = 0; i < n; ++i) {
                double e = oracle::evaluate_point(P, mm, t, i, false);
                s += std::min(e, opts.squared_inlier_thresholds[t]) * opts.data_type_weights[t];
                if (errors) errors[((size_t)m * 3 + t) * n + i] = oracle::evaluate_point(P, mm, t, i, true);
            }
        scores[m] = s;
    }
    return 0;
}

// LeastSquares (kind 0) / NonMinimalSolver (kind 1) of the estimators on one sample
// (three index lists); model in/out in problem units.  Returns 1 when the solver ran,
// 0 when the sample is too small (model unchanged).
int oracle_least_squares(int variant, int64_t n, const double *x0, const double *x1, const double *d0,
                         const double *d1, const double *min_depth, const double *cam0, const double *cam1,
                         const or_ransac_options *o, const or_estimator_config *c, int32_t kind, const int32_t *s0,
                         int32_t n0, const int32_t *s1, int32_t n1, const int32_t *s2, int32_t n2, or_model *model) {
    oracle::Options opts = to_opts(o);
    const double md0[2] = {0, 0};
    oracle::Problem P = oracle::make_problem((oracle::Variant)variant, (int)n, x0, x1, d0, d1,
                                             min_depth ? min_depth : md0, cam0, cam1, to_cfg(c), &opts);
    std::vector<std::vector<int>> sample(3);
    sample[0].assign(s0, s0 + n0);
    sample[1].assign(s1, s1 + n1);
    sample[2].assign(s2, s2 + n2);
    oracle::Model m = get_model(model);
    const int kmd = (variant == 0) ? 3 : 4, kpt = (variant == 0) ? 5 : (variant == 1 ? 6 : 7);
    const bool small = (n0 < kmd && n1 < kmd) || n2 < kpt;
    if (kind == 1)
        oracle::non_minimal_solver(P, sample, 0, &m);
    else
        oracle::least_squares(P, sample, 0, &m);
    put_model(m, model);
    return small ? 0 : 1;
}

int oracle_estimate(int variant, int64_t n, const double *x0, const double *x1, const double *d0, const double *d1,
                    const double *min_depth, const double *cam0, const double *cam1, const or_ransac_options *o,
                    const or_estimator_config *c, or_model *out, or_stats *st, int32_t *inlier_idx) {
    auto t0 = std::chrono::steady_clock::now();
    oracle::Model best;
    oracle::Stats S;
    try {
        oracle::estimate_pose((oracle::Variant)variant, (int)n, x0, x1, d0, d1, min_depth, cam0, cam1, to_opts(o),
                              to_cfg(c), &best, &S);
    } catch (const std::exception &e) { // (ORACLE_MODEL_REPLAY out of step)
        std::fprintf(stderr, "[oracle] %s\n", e.what());
        return -1;
    }
    put_model(best, out);
    std::memset(st, 0, sizeof(*st));
    st->best_model_score = S.best_model_score;
    for (int t = 0; t < 3; ++t) {
        st->inlier_ratios[t] = t < (int)S.inlier_ratios.size() ? S.inlier_ratios[t] : 0.0;
        int cnt = t < (int)S.inlier_indices.size() ? (int)S.inlier_indices[t].size() : 0;
        st->num_inliers[t] = cnt;
        if (inlier_idx)
            for (int k = 0; k < cnt; ++k) inlier_idx[t * n + k] = S.inlier_indices[t][k];
    }
    st->num_hypotheses = S.num_hypotheses;
    st->num_iterations_total = S.num_iterations_total;
    st->num_iterations_per_solver[0] = S.num_iterations_per_solver.size() > 0 ? S.num_iterations_per_solver[0] : 0;
    st->num_iterations_per_solver[1] = S.num_iterations_per_solver.size() > 1 ? S.num_iterations_per_solver[1] : 0;
    st->best_num_inliers = S.best_num_inliers;
    st->best_solver_type = S.best_solver_type;
    st->number_lo_iterations = S.number_lo_iterations;
    st->seconds_total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

// The reference's per-iteration random decisions with libstdc++'s own engine and
// distributions (std::mt19937, uniform_real_distribution, uniform_int_distribution):
// SelectMinimalSolver (src/hybrid_ransac.h:210-243) + HybridUniformSampling.
int oracle_iteration_stream(int variant, int32_t n, uint32_t seed, int32_t solver_type, int32_t iterations,
                            int32_t *types, int32_t *idx) {
    const int kmd = variant == 0 ? 3 : 4, kpt = variant == 0 ? 5 : (variant == 1 ? 6 : 7);
    const int ss[2][3] = {{kmd, kmd, 0}, {0, 0, kpt}};
    double prior[2] = {1.0, 1.0};
    if (solver_type == 1) prior[0] = 0.0;
    if (solver_type == 2) prior[1] = 0.0;
    for (int s = 0; s < 2; ++s)
        for (int t = 0; t < 3; ++t)
            if (ss[s][t] > n) prior[s] = 0.0;
    std::mt19937 rng(seed), samp(seed);
    std::uniform_int_distribution<int> dist(0, n - 1);
    for (int k = 0; k < iterations; ++k) {
        std::uniform_real_distribution<double> ud(0.0, prior[0] + prior[1]);
        const double u = ud(rng);
        int st = -1;
        double acc = 0;
        for (int s = 0; s < 2; ++s) {
            if (prior[s] == 0.0) continue;
            acc += prior[s];
            if (u <= acc) {
                st = s;
                break;
            }
        }
        if (st < 0) st = prior[1] > 0 ? 1 : 0; // only when no solver is feasible (estimator stops earlier)
        types[k] = st;
        for (int j = 0; j < 8; ++j) idx[8 * k + j] = -1;
        for (int t = 0; t < 3; ++t) {
            std::vector<int> smp(ss[st][t]);
            for (int i = 0; i < ss[st][t]; ++i) {
                bool dup = true;
                while (dup) {
                    smp[i] = dist(samp);
                    dup = false;
                    for (int j = 0; j < i; ++j)
                        if (smp[j] == smp[i]) dup = true;
                }
            }
            if ((st == 0 && t == 0) || (st == 1 && t == 2))
                for (int j = 0; j < ss[st][t]; ++j) idx[8 * k + j] = smp[j];
        }
    }
    return 0;
}

} // extern "C"
