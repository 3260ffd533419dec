// Host-side Levenberg-Marquardt used by local optimisation (LO).
//
// Replaces the reference's Ceres problems (src/optimizer.h:48-125, 265-369, 383-499)
// built from the cost functors of src/cost_functions.h:16-387.  Ceres is not
// available, so the algorithm is restated (see DESIGN.md "LO"): trust-region LM
// with Jacobi column scaling, LM diagonal clamped to [1e-6, 1e32], initial radius
// 1e4, acceptance at relative decrease > 1e-3, radius update
// mu /= max(1/3, 1-(2 rho-1)^3), QuaternionManifold tangent updates, box bounds by
// projection, and EstimatorConfig's function / gradient / parameter tolerances.
// Jacobians are analytic; normal equations (J^T J, J^T r) are accumulated in one pass.
#pragma once
#include <vector>

#include "../include/mp_types.h"

namespace mp {

struct HostPair {
    int variant = kCal;
    int n = 0;
    std::vector<double> x0, x1; // 2n (pixels for CAL, normalized pixels for SF/TF)
    std::vector<double> d0, d1;
    double K0[9], K1[9], K0i[9], K1i[9];
    double min_depth[2] = {0, 0};
    double sampson_squared_weight = 1.0;
};

struct LMSettings {
    bool use_reproj = true, use_sampson = true, use_shift = true, min_depth_constraint = true;
    double w_sampson = 1.0;
    double ftol = 1e-6, gtol = 1e-8, ptol = 1e-6;
    int max_iter = 25;
    // Ceres use_nonmonotonic_steps (EstimatorConfig default true, src/estimator_config.h:31)
    // with Ceres' default max_consecutive_nonmonotonic_steps = 5
    bool nonmonotonic = true;
};

// Refines m over the residual blocks sample[0] (reproj 0->1), sample[1] (reproj 1->0),
// sample[2] (Sampson).  Returns false when the problem has no residuals (Ceres
// Solve() returning false); m is left unchanged in that case.
bool lm_refine(const HostPair &P, const std::vector<int> *sample, const LMSettings &S, Model *m);
// normal-equation evaluations of this thread's last lm_refine (MADPOSE_LO_TIMING)
extern thread_local int lm_last_evals;

// the LM pool's spin before blocking, in microseconds (MADPOSE_LO_SPIN, or the
// affinity-based default of lm.cpp)
int lo_spin_us();

// quaternion helpers (w, x, y, z) -- Eigen::Quaternion(Matrix3) / toRotationMatrix
void rot_to_quat(const double *R, double *q);
void quat_to_rot(const double *q, double *R);

} // namespace mp
