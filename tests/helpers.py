"""Shared test helpers: option conversion to the oracle's C structs, tolerances."""
import numpy as np

import oracle


def oracle_opts(o):
    r = oracle.OrRansacOptions()
    r.success_probability = o.success_probability
    r.squared_inlier_thresholds[:] = list(o.squared_inlier_thresholds)[:2]
    r.data_type_weights[:] = list(o.data_type_weights)[:2]
    r.threshold_multiplier = o.threshold_multiplier
    r.min_num_iterations = o.min_num_iterations
    r.max_num_iterations = o.max_num_iterations
    r.max_num_iterations_per_solver = o.max_num_iterations_per_solver
    r.random_seed = o.random_seed
    r.num_lo_steps = o.num_lo_steps
    r.num_lsq_iterations = o.num_lsq_iterations
    r.min_sample_multiplicator = o.min_sample_multiplicator
    r.non_min_sample_multiplier = o.non_min_sample_multiplier
    r.lo_starting_iterations = o.lo_starting_iterations
    r.final_least_squares = int(bool(o.final_least_squares))
    r.use_ours = int(bool(o.use_ours))
    r.use_4p4d = int(bool(o.use_4p4d))
    return r


def oracle_cfg(c):
    r = oracle.OrEstimatorConfig()
    r.ceres_function_tolerance = c.ceres_function_tolerance
    r.ceres_gradient_tolerance = c.ceres_gradient_tolerance
    r.ceres_parameter_tolerance = c.ceres_parameter_tolerance
    r.ceres_max_num_iterations = c.ceres_max_num_iterations
    r.solver_type = c.solver_type
    r.score_type = c.score_type
    r.lo_type = c.LO_type
    r.min_depth_constraint = int(bool(c.min_depth_constraint))
    r.use_shift = int(bool(c.use_shift))
    r.ceres_use_nonmonotonic_steps = int(bool(c.ceres_use_nonmonotonic_steps))
    r.ceres_num_threads = c.ceres_num_threads
    return r


def rot_angle_deg(Ra, Rb):
    # chordal form: accurate near zero (arccos of the trace loses ~1e-6 deg there)
    d = np.linalg.norm(np.asarray(Ra) - np.asarray(Rb)) / (2.0 * np.sqrt(2.0))
    return np.rad2deg(2.0 * np.arcsin(min(d, 1.0)))


def solution_sets_match(ref, mine, rtol):
    """Compare two root sets (rows of equal width) as multisets, sorted by column 1 (b1)."""
    ref = np.asarray(ref, dtype=np.float64)
    mine = np.asarray(mine, dtype=np.float64)
    if len(ref) != len(mine):
        return False, np.inf
    if len(ref) == 0:
        return True, 0.0
    ref = ref[np.argsort(ref[:, 1])]
    mine = mine[np.argsort(mine[:, 1])]
    err = float(np.max(np.abs(ref - mine) / (1.0 + np.abs(ref))))
    return err <= rtol, err
