// ORACLE -- test infrastructure only.
//
// Restatement of HybridLOMSAC::EstimateModel (src/hybrid_ransac.h:38-206) with its
// helpers, and of the RansacLib pieces it relies on (not vendored, "parity
// unpinned"; the recalled upstream semantics are listed in DESIGN.md):
//   HybridUniformSampling  -- per data type, k draws of uniform_int_distribution
//                             (0, N-1) on the sampler's own mt19937, re-drawing a
//                             value already present in that type's sample.
//   NumRequiredIterations  -- hybrid version: P = prod_t r_t^k_t ...
//   RandomShuffleAndResize -- partial Fisher-Yates with uniform_int_distribution(i, n-1)
//                             for i < k, a no-op when k >= size.
// The random streams are libstdc++'s (std::mt19937, std::uniform_*_distribution),
// i.e. exactly what the reference consumes.
#include <cstdlib>
#include <cstdio>
#include <stdexcept>
#include <algorithm>
#include <cmath>
#include <limits>
#include <random>

#include "oracle.h"

namespace oracle {

namespace {

const double kDMax = std::numeric_limits<double>::max();

std::vector<std::vector<int>> sample_sizes(Variant v) {
    // src/hybrid_pose_estimator.h:45-49, ..shared..h:41-45, ..two..h:43-47
    if (v == CAL) return {{3, 3, 0}, {0, 0, 5}};
    if (v == SF) return {{4, 4, 0}, {0, 0, 6}};
    return {{4, 4, 0}, {0, 0, 7}};
}
int min_sample_size(Variant v) { return v == CAL ? 5 : (v == SF ? 6 : 7); }
int non_minimal_sample_size(Variant v) { return v == CAL ? 35 : 36; }

struct Sampler {
    std::mt19937 rng;
    std::uniform_int_distribution<int> dist;
    explicit Sampler(unsigned seed, int n) : rng(seed), dist(0, std::max(n - 1, 0)) {}
    void draw(int k, std::vector<int> *out) {
        out->resize(k);
        for (int i = 0; i < k; ++i) {
            bool dup = true;
            while (dup) {
                (*out)[i] = dist(rng);
                dup = false;
                for (int j = 0; j < i; ++j)
                    if ((*out)[j] == (*out)[i]) {
                        dup = true;
                        break;
                    }
            }
        }
    }
};

uint32_t num_required_iterations(const std::vector<double> &ratios, double prob_missing, const std::vector<int> &k,
                                 uint32_t min_it, uint32_t max_it) {
    double p_all = 1.0;
    for (size_t t = 0; t < ratios.size(); ++t) p_all *= std::pow(ratios[t], (double)k[t]);
    if (p_all <= 0.0) return max_it;
    if (p_all >= 1.0) return min_it;
    const double p_bad = 1.0 - p_all;
    if (p_bad >= 0.99999999999999) return max_it;
    double it = std::ceil(std::log(prob_missing) / std::log(p_bad) + 0.5);
    uint32_t r = std::min((uint32_t)it, max_it);
    return std::max(min_it, r);
}

void shuffle_resize(int k, std::mt19937 *rng, std::vector<int> *v) {
    const int n = (int)v->size();
    if (n <= k) return;
    for (int i = 0; i < k; ++i) {
        std::uniform_int_distribution<int> d(i, n - 1);
        std::swap((*v)[i], (*v)[d(*rng)]);
    }
    v->resize(k);
}

struct Engine {
    const Problem &P;
    const Options &o;
    std::vector<std::vector<int>> ss;
    const int n;

    Engine(const Problem &p, const Options &opt) : P(p), o(opt), ss(sample_sizes(p.variant)), n(p.n) {}

    double score(const Model &m) const {
        double s = 0.0;
        for (int t = 0; t < 3; ++t)
            for (int i = 0; i < n; ++i) {
                double e = evaluate_point(P, m, t, i, false);
                s += std::min(e, o.squared_inlier_thresholds[t]) * o.data_type_weights[t];
            }
        return s;
    }

    int inliers(const Model &m, const std::vector<double> &thr, std::vector<std::vector<int>> *out) const {
        out->assign(3, {});
        int c = 0;
        for (int t = 0; t < 3; ++t)
            for (int i = 0; i < n; ++i)
                if (evaluate_point(P, m, t, i, true) < thr[t]) {
                    (*out)[t].push_back(i);
                    ++c;
                }
        return c;
    }

    void update_best(double sc, const Model &m, int st, double *best_sc, Model *best, int *best_st) const {
        if (sc < *best_sc) {
            *best_sc = sc;
            *best = m;
            *best_st = st;
        }
    }

    void termination(const Model &m, Stats *S, std::vector<uint32_t> *max_it) const {
        S->best_num_inliers = inliers(m, o.squared_inlier_thresholds, &S->inlier_indices);
        for (int t = 0; t < 3; ++t) S->inlier_ratios[t] = n > 0 ? (double)S->inlier_indices[t].size() / n : 0.0;
        for (int s = 0; s < 2; ++s)
            (*max_it)[s] = num_required_iterations(S->inlier_ratios, 1.0 - o.success_probability, ss[s],
                                                   o.min_num_iterations, o.max_num_iterations_per_solver);
    }

    static std::vector<std::vector<int>> split(const std::vector<int> &all, int n) {
        std::vector<std::vector<int>> s(3);
        for (int idx : all) {
            int t = 0;
            while (idx >= n) {
                idx -= n;
                ++t;
            }
            s[t].push_back(idx);
        }
        return s;
    }

    // LeastSquaresFit (src/hybrid_ransac.h:484-538)
    void lsq_fit(const std::vector<double> &thr, int st, std::mt19937 *rng, Model *m, bool use_all) const {
        std::vector<std::vector<int>> inl;
        inliers(*m, thr, &inl);
        std::vector<int> k = ss[st];
        for (int t = 0; t < 3; ++t) {
            if ((int)inl[t].size() < k[t]) return;
            k[t] = std::min(k[t] * o.min_sample_multiplicator, (int)inl[t].size());
        }
        if (use_all) {
            least_squares(P, inl, st, m);
            return;
        }
        int total = (k[0] + k[1] + k[2]) * o.min_sample_multiplicator;
        std::vector<int> all;
        for (int t = 0; t < 3; ++t)
            for (int idx : inl[t]) all.push_back(idx + t * n);
        shuffle_resize(total, rng, &all);
        least_squares(P, split(all, n), st, m);
    }

    // LocalOptimization (src/hybrid_ransac.h:383-482)
    void local_opt(int st, std::mt19937 *rng, Model *best_min, double *best_min_score, int *best_st) const {
        std::vector<double> thr = o.squared_inlier_thresholds, upd(3);
        for (int t = 0; t < 3; ++t) {
            upd[t] = (o.threshold_multiplier - 1.0) * thr[t] / (int)(o.num_lsq_iterations - 1);
            thr[t] *= o.threshold_multiplier;
        }
        Model m_init = *best_min;
        lsq_fit(thr, st, rng, &m_init, true);
        double sc = score(m_init);
        update_best(sc, m_init, st, best_min_score, best_min, best_st);
        std::vector<std::vector<int>> base;
        inliers(m_init, o.squared_inlier_thresholds, &base);
        std::vector<int> base_all;
        for (int t = 0; t < 3; ++t)
            for (int idx : base[t]) base_all.push_back(idx + t * n);
        const int k_nonmin = std::max(non_minimal_sample_size(P.variant),
                                      std::min(min_sample_size(P.variant) * o.non_min_sample_multiplier,
                                               (int)base_all.size() / 2));
        for (int r = 0; r < o.num_lo_steps; ++r) {
            std::vector<int> sample_all = base_all; // copied BEFORE the shuffle (:439-440)
            shuffle_resize(k_nonmin, rng, &base_all);
            Model m = m_init;
            if (!non_minimal_solver(P, split(sample_all, n), st, &m)) continue;
            sc = score(m);
            update_best(sc, m, st, best_min_score, best_min, best_st);
            lsq_fit(o.squared_inlier_thresholds, st, rng, &m, false);
            std::vector<double> cur = thr;
            for (int i = 0; i < o.num_lsq_iterations; ++i) {
                lsq_fit(cur, st, rng, &m, false);
                sc = score(m);
                update_best(sc, m, st, best_min_score, best_min, best_st);
                for (int t = 0; t < 3; ++t) cur[t] -= upd[t];
            }
        }
    }

    int run(Model *best, Stats *S) const {
        *best = Model();
        *S = Stats();
        S->best_model_score = kDMax;
        S->num_iterations_per_solver.assign(2, 0);
        S->inlier_ratios.assign(3, 0.0);
        S->inlier_indices.assign(3, {});
        std::vector<double> prior = {1.0, 1.0};
        if (P.cfg.solver_type == EPI_ONLY) prior[0] = 0.0;
        if (P.cfg.solver_type == MD_ONLY) prior[1] = 0.0;
        // VerifyData (src/hybrid_ransac.h:552-577)
        for (int s = 0; s < 2; ++s)
            for (int t = 0; t < 3; ++t)
                if (ss[s][t] > n) {
                    prior[s] = 0.0;
                    break;
                }
        if (prior[0] <= 0.0 && prior[1] <= 0.0) {
            S->best_model_score = kDMax;
            return 0;
        }
        Sampler sampler(o.random_seed, n);
        const uint32_t max_total = std::max(o.max_num_iterations, o.min_num_iterations);
        std::vector<uint32_t> max_per(2, std::max(o.max_num_iterations_per_solver, o.min_num_iterations));
        Model best_min;
        double best_min_score = kDMax;
        std::vector<std::vector<int>> sample(3);
        std::vector<Model> models;
        std::mt19937 rng;
        rng.seed(o.random_seed);
        const uint32_t lo_start = (uint32_t)o.lo_starting_iterations;
        // ORACLE_COUNT_DUMP=<file>: one line per iteration (iteration, solver type, model
        // count, the solver's sample) -- a diagnostic (tools/diag_counts.py)
        const char *dump_path = std::getenv("ORACLE_COUNT_DUMP");
        FILE *dump = dump_path ? std::fopen(dump_path, "w") : nullptr;
        struct Closer {
            FILE *f;
            ~Closer() {
                if (f) std::fclose(f);
            }
        } closer{dump};
        // ORACLE_MODEL_REPLAY=<file>: the models of every iteration come from the file
        // (the engine's MADPOSE_MODEL_DUMP: int32 iteration, int32 count, count x 17
        // doubles) instead of the minimal solvers -- the selection, LO and termination
        // logic then runs on the engine's own models (tests/test_ties_gpu.py)
        const char *replay_path = std::getenv("ORACLE_MODEL_REPLAY");
        FILE *replay = replay_path ? std::fopen(replay_path, "rb") : nullptr;
        Closer closer2{replay};
        // ORACLE_MODEL_DUMP=<file>: this loop's own models of every iteration in the
        // engine's MADPOSE_MODEL_DUMP format (tests/test_ties_gpu.py compares the two)
        const char *mdump_path = std::getenv("ORACLE_MODEL_DUMP");
        FILE *mdump = mdump_path ? std::fopen(mdump_path, "wb") : nullptr;
        Closer closer3{mdump};

        for (S->num_iterations_total = 0; S->num_iterations_total < max_total; ++S->num_iterations_total) {
            const uint32_t it = S->num_iterations_total;
            if (it == lo_start && best_min_score < kDMax) {
                ++S->number_lo_iterations;
                local_opt(S->best_solver_type, &rng, best, &S->best_model_score, &S->best_solver_type);
                termination(*best, S, &max_per);
            }
            // SelectMinimalSolver (src/hybrid_ransac.h:210-243)
            double psum = prior[0] + prior[1];
            std::uniform_real_distribution<double> ud(0.0, psum);
            const double u = ud(rng);
            int st = -1;
            double acc = 0.0;
            for (int s = 0; s < 2; ++s) {
                if (prior[s] == 0.0) continue;
                acc += prior[s];
                if (u <= acc) {
                    st = s;
                    break;
                }
            }
            if (st < 0) st = prior[1] > 0 ? 1 : 0; // unreachable: u < psum
            S->num_iterations_per_solver[st] += 1;
            for (int t = 0; t < 3; ++t) sampler.draw(ss[st][t], &sample[t]);
            int nm = minimal_solver(P, sample, st, &models);
            if (replay) {
                int32_t hdr[2] = {-1, 0};
                if (std::fread(hdr, sizeof(hdr), 1, replay) != 1 || hdr[0] != (int32_t)it || hdr[1] < 0)
                    throw std::runtime_error("model replay out of step");
                models.resize(hdr[1]);
                static_assert(sizeof(Model) == 17 * sizeof(double), "Model layout");
                if (hdr[1] > 0 && std::fread(models.data(), sizeof(Model), hdr[1], replay) != (size_t)hdr[1])
                    throw std::runtime_error("model replay truncated");
                nm = hdr[1];
            }
            S->num_hypotheses += nm;
            if (mdump) {
                const int32_t hdr[2] = {(int32_t)it, (int32_t)nm};
                std::fwrite(hdr, sizeof(hdr), 1, mdump);
                if (nm > 0) std::fwrite(models.data(), sizeof(Model), (size_t)nm, mdump);
            }
            if (dump) {
                std::fprintf(dump, "%u %d %d", it, st, nm);
                for (int i : sample[st == 0 ? 0 : 2]) std::fprintf(dump, " %d", i);
                std::fprintf(dump, "\n");
            }
            if (nm > 0) {
                double bl = kDMax;
                int bid = 0;
                for (int m = 0; m < nm; ++m) {
                    double sc = score(models[m]);
                    if (sc < bl) {
                        bl = sc;
                        bid = m;
                    }
                }
                if (bl < best_min_score || it == lo_start) {
                    const bool new_best = bl < best_min_score;
                    if (new_best) {
                        if (std::getenv("ORACLE_TRACE")) std::fprintf(stderr, "[oracle] it=%u new best %.17g (solver %d, %d models)\n", it, bl, st, nm);
                        best_min_score = bl;
                        best_min = models[bid];
                        update_best(best_min_score, best_min, st, &S->best_model_score, best, &S->best_solver_type);
                    }
                    const bool run_lo = it >= lo_start && best_min_score < kDMax;
                    if (new_best || run_lo) {
                        if (run_lo) {
                            ++S->number_lo_iterations;
                            double sc = best_min_score;
                            local_opt(S->best_solver_type, &rng, &best_min, &sc, &S->best_solver_type);
                            if (std::getenv("ORACLE_TRACE")) std::fprintf(stderr, "[oracle] it=%u LO %.17g -> %.17g\n", it, best_min_score, sc);
                            update_best(sc, best_min, st, &S->best_model_score, best, &S->best_solver_type);
                        }
                        termination(*best, S, &max_per);
                    }
                }
            }
            // per-solver cap; `break` skips the loop increment, so num_iterations_total
            // keeps the index of this last iteration (src/hybrid_ransac.h:169-171)
            if (S->num_iterations_per_solver[st] >= max_per[st]) break;
        }
        if (S->num_iterations_total <= lo_start && S->best_model_score < kDMax) {
            ++S->number_lo_iterations;
            local_opt(S->best_solver_type, &rng, best, &S->best_model_score, &S->best_solver_type);
            termination(*best, S, &max_per);
        }
        if (o.final_least_squares) {
            Model refined = *best;
            least_squares(P, S->inlier_indices, S->best_solver_type, &refined);
            double sc = score(refined);
            if (sc < S->best_model_score) {
                S->best_model_score = sc;
                *best = refined;
                termination(*best, S, &max_per);
            }
        }
        return S->best_num_inliers;
    }
};

} // namespace

int estimate(const Problem &P, const Options &opts, Model *best, Stats *stats) {
    Engine e(P, opts);
    return e.run(best, stats);
}

void estimate_pose(Variant v, int n, const double *x0, const double *x1, const double *d0, const double *d1,
                   const double min_depth[2], const double *cam0, const double *cam1, const Options &user_opts,
                   const EstConfig &cfg, Model *best, Stats *stats) {
    Options o = user_opts;
    Problem P = make_problem(v, n, x0, x1, d0, d1, min_depth, cam0, cam1, cfg, &o);
    estimate(P, o, best, stats);
    if (v == SF) {
        best->focal0 *= P.norm_scale;
        best->focal1 = best->focal0;
    } else if (v == TF) {
        best->focal0 *= P.norm_scale;
        best->focal1 *= P.norm_scale;
    }
}

} // namespace oracle
