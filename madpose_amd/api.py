"""Python surface of the reference's pybind11 module (src/bindings.cpp), backed by the
MI355X engine through the C ABI.  Names, defaults, argument meaning and return types
follow src/bindings.cpp:34-175 so user code written for `import madpose` runs unchanged.
"""
import ctypes
import math

import numpy as np

from . import _lib as L


# ---------------------------------------------------------------------------
# option / config containers (src/bindings.cpp:78-109, src/hybrid_ransac.h:17-25,
# src/estimator_config.h:7-33; RansacLib defaults as restated in DESIGN.md)
class HybridLORansacOptions:
    def __init__(self):
        self.min_num_iterations = 100
        self.max_num_iterations = 10000
        self.max_num_iterations_per_solver = 10000
        self.success_probability = 0.99
        self.squared_inlier_thresholds = []
        self.data_type_weights = []
        self.random_seed = 0
        self.num_lo_steps = 10
        self.threshold_multiplier = math.sqrt(2.0)
        self.num_lsq_iterations = 4
        self.min_sample_multiplicator = 7
        self.non_min_sample_multiplier = 3
        self.lo_starting_iterations = 50
        self.final_least_squares = False
        self.use_ours = False
        self.use_4p4d = False

    def _to_c(self):
        o = L.mp_ransac_options()
        thr = list(self.squared_inlier_thresholds)
        w = list(self.data_type_weights)
        if len(thr) < 2:
            raise ValueError("squared_inlier_thresholds must hold [reprojection^2, epipolar^2]")
        if len(w) < 2:
            raise ValueError("data_type_weights must hold [reprojection, epipolar]")
        o.success_probability = float(self.success_probability)
        o.squared_inlier_thresholds[0] = float(thr[0])
        o.squared_inlier_thresholds[1] = float(thr[1])
        o.data_type_weights[0] = float(w[0])
        o.data_type_weights[1] = float(w[1])
        o.threshold_multiplier = float(self.threshold_multiplier)
        o.min_num_iterations = int(self.min_num_iterations)
        o.max_num_iterations = int(self.max_num_iterations)
        o.max_num_iterations_per_solver = int(self.max_num_iterations_per_solver)
        o.random_seed = int(self.random_seed)
        o.num_lo_steps = int(self.num_lo_steps)
        o.num_lsq_iterations = int(self.num_lsq_iterations)
        o.min_sample_multiplicator = int(self.min_sample_multiplicator)
        o.non_min_sample_multiplier = int(self.non_min_sample_multiplier)
        o.lo_starting_iterations = int(self.lo_starting_iterations)
        o.final_least_squares = int(bool(self.final_least_squares))
        o.use_ours = int(bool(self.use_ours))
        o.use_4p4d = int(bool(self.use_4p4d))
        return o


class EstimatorConfig:
    HYBRID, EPI_ONLY, MD_ONLY = 0, 1, 2

    def __init__(self, solver=0, score=0, LO=0):
        self.solver_type = int(solver)
        self.score_type = int(score)
        self.LO_type = int(LO)
        self.min_depth_constraint = True
        self.use_shift = True
        self.ceres_function_tolerance = 1e-6
        self.ceres_gradient_tolerance = 1e-8
        self.ceres_parameter_tolerance = 1e-6
        self.ceres_max_num_iterations = 25.0
        self.ceres_use_nonmonotonic_steps = True
        self.ceres_num_threads = 1

    def _to_c(self):
        c = L.mp_estimator_config()
        c.ceres_function_tolerance = float(self.ceres_function_tolerance)
        c.ceres_gradient_tolerance = float(self.ceres_gradient_tolerance)
        c.ceres_parameter_tolerance = float(self.ceres_parameter_tolerance)
        c.ceres_max_num_iterations = float(self.ceres_max_num_iterations)
        c.solver_type = int(self.solver_type)
        c.score_type = int(self.score_type)
        c.lo_type = int(self.LO_type)
        c.min_depth_constraint = int(bool(self.min_depth_constraint))
        c.use_shift = int(bool(self.use_shift))
        c.ceres_use_nonmonotonic_steps = int(bool(self.ceres_use_nonmonotonic_steps))
        c.ceres_num_threads = int(self.ceres_num_threads)
        return c


class RansacOptions:
    def __init__(self):
        self.min_num_iterations_ = 100
        self.max_num_iterations_ = 10000
        self.success_probability_ = 0.99
        self.squared_inlier_threshold_ = 1.0
        self.random_seed_ = 0


class LORansacOptions:
    def __init__(self):
        self.min_num_iterations = 100
        self.max_num_iterations = 10000
        self.success_probability = 0.99
        self.squared_inlier_threshold = 1.0
        self.random_seed = 0
        self.num_lo_steps = 10
        self.threshold_multiplier = math.sqrt(2.0)
        self.num_lsq_iterations = 4
        self.min_sample_multiplicator = 7
        self.non_min_sample_multiplier = 3
        self.lo_starting_iterations = 50
        self.final_least_squares = False


class RansacStats:
    def __init__(self):
        self.num_iterations = 0
        self.best_num_inliers = 0
        self.best_model_score = float("inf")
        self.inlier_ratio = 0.0
        self.inlier_indices = []
        self.number_lo_iterations = 0


class HybridRansacStatistics:
    def __init__(self):
        self.num_iterations_total = 0
        self.num_iterations_per_solver = [0, 0]
        self.best_num_inliers = 0
        self.best_solver_type = -1
        self.best_model_score = float("inf")
        self.inlier_ratios = [0.0, 0.0, 0.0]
        self.inlier_indices = [[], [], []]
        self.number_lo_iterations = 0
        # engine counters (not in the reference)
        self.num_hypotheses = 0
        self.num_lo_sweeps = 0
        self.num_batches = 0
        self.seconds_total = 0.0
        self.seconds_lo = 0.0
        self.seconds_gpu_wait = 0.0

    def __repr__(self):
        return (f"HybridRansacStatistics(iterations={self.num_iterations_total}, per_solver={self.num_iterations_per_solver}, "
                f"inliers={self.best_num_inliers}, score={self.best_model_score:.6g}, lo={self.number_lo_iterations})")


# ---------------------------------------------------------------------------
# model types (src/pose.h:7-56, src/bindings.cpp:111-154)
class PoseAndScale:
    def __init__(self, *args):
        self.pose = np.zeros((3, 4))
        self.scale = 1.0
        if len(args) == 2:
            self.pose = np.array(args[0], dtype=np.float64).reshape(3, 4)
            self.scale = float(args[1])
        elif len(args) == 3:
            self.pose[:, :3] = np.asarray(args[0], dtype=np.float64).reshape(3, 3)
            self.pose[:, 3] = np.asarray(args[1], dtype=np.float64).reshape(3)
            self.scale = float(args[2])
        elif args:
            raise TypeError("PoseAndScale(pose, scale) or PoseAndScale(R, t, scale)")

    def R(self):
        return self.pose[:, :3].copy()

    def t(self):
        return self.pose[:, 3].copy()


class PoseScaleOffset(PoseAndScale):
    _n_extra = 0

    def __init__(self, *args):
        self.pose = np.zeros((3, 4))
        self.scale, self.offset0, self.offset1 = 1.0, 0.0, 0.0
        self._init_extra()
        k = self._n_extra
        if len(args) == 4 + k:  # pose, scale, b0, b1, [focals]
            self.pose = np.array(args[0], dtype=np.float64).reshape(3, 4)
            vals = args[1:]
        elif len(args) == 5 + k:  # R, t, scale, b0, b1, [focals]
            self.pose[:, :3] = np.asarray(args[0], dtype=np.float64).reshape(3, 3)
            self.pose[:, 3] = np.asarray(args[1], dtype=np.float64).reshape(3)
            vals = args[2:]
        elif not args:
            return
        else:
            raise TypeError(f"{type(self).__name__}: unexpected constructor arguments")
        self.scale, self.offset0, self.offset1 = float(vals[0]), float(vals[1]), float(vals[2])
        self._set_extra([float(v) for v in vals[3:]])

    def _init_extra(self):
        pass

    def _set_extra(self, vals):
        pass

    def __repr__(self):
        return f"{type(self).__name__}(scale={self.scale:.6g}, offset0={self.offset0:.6g}, offset1={self.offset1:.6g})"


class PoseScaleOffsetSharedFocal(PoseScaleOffset):
    _n_extra = 1

    def _init_extra(self):
        self.focal = 1.0

    def _set_extra(self, vals):
        self.focal = vals[0]


class PoseScaleOffsetTwoFocal(PoseScaleOffset):
    _n_extra = 2

    def _init_extra(self):
        self.focal0 = 1.0
        self.focal1 = 1.0

    def _set_extra(self, vals):
        self.focal0, self.focal1 = vals[0], vals[1]


def _model_from_c(m, variant):
    R = np.array(m.R[:]).reshape(3, 3)
    t = np.array(m.t[:])
    if variant == L.CALIBRATED:
        return PoseScaleOffset(R, t, m.scale, m.offset0, m.offset1)
    if variant == L.SHARED_FOCAL:
        return PoseScaleOffsetSharedFocal(R, t, m.scale, m.offset0, m.offset1, m.focal0)
    if variant == L.SCALE_ONLY:
        return PoseAndScale(R, t, m.scale)
    return PoseScaleOffsetTwoFocal(R, t, m.scale, m.offset0, m.offset1, m.focal0, m.focal1)


def _model_to_c(p, variant):
    m = L.mp_model()
    pose = np.asarray(p.pose, dtype=np.float64).reshape(3, 4)
    m.R[:] = pose[:, :3].ravel().tolist()
    m.t[:] = pose[:, 3].tolist()
    m.scale, m.offset0, m.offset1 = float(p.scale), float(getattr(p, "offset0", 0.0)), float(getattr(p, "offset1", 0.0))
    if variant == L.SHARED_FOCAL:
        m.focal0 = m.focal1 = float(p.focal)
    elif variant == L.TWO_FOCAL:
        m.focal0, m.focal1 = float(p.focal0), float(p.focal1)
    else:
        m.focal0 = m.focal1 = 1.0
    return m


def _stats_from_c(s, idx, n):
    out = HybridRansacStatistics()
    out.num_iterations_total = int(s.num_iterations_total)
    out.num_iterations_per_solver = [int(s.num_iterations_per_solver[0]), int(s.num_iterations_per_solver[1])]
    out.best_num_inliers = int(s.best_num_inliers)
    out.best_solver_type = int(s.best_solver_type)
    out.best_model_score = float(s.best_model_score)
    out.inlier_ratios = [float(v) for v in s.inlier_ratios]
    out.inlier_indices = [idx[t * n: t * n + s.num_inliers[t]].tolist() for t in range(3)]
    out.number_lo_iterations = int(s.number_lo_iterations)
    out.num_hypotheses = int(s.num_hypotheses)
    out.num_lo_sweeps = int(s.num_lo_sweeps)
    out.num_batches = int(s.num_batches)
    out.seconds_total = float(s.seconds_total)
    out.seconds_lo = float(s.seconds_lo)
    out.seconds_gpu_wait = float(s.seconds_gpu_wait)
    return out


# ---------------------------------------------------------------------------
def _pts(a, name):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if a.ndim != 2 or a.shape[1] != 2:
        raise ValueError(f"{name} must be an N x 2 array of pixel coordinates")
    return a


def _vec(a, n, name):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1))
    if a.shape[0] != n:
        raise ValueError(f"{name} must hold one value per correspondence ({n}), got {a.shape[0]}")
    return a


def _dp(a):
    return a.ctypes.data_as(L.c_double_p)


_DEFAULT_DEVICE = 0


def set_device(device):
    """Select the HIP device used by subsequent calls (one process per GPU)."""
    global _DEFAULT_DEVICE
    _DEFAULT_DEVICE = int(device)


def _estimate(variant, x0, x1, depth0, depth1, min_depth, cam0, cam1, options, est_config, device):
    x0 = _pts(x0, "x0")
    x1 = _pts(x1, "x1")
    n = x0.shape[0]
    if x1.shape[0] != n:
        raise ValueError("x0 and x1 must have the same number of rows")
    d0 = _vec(depth0, n, "depth0")
    d1 = _vec(depth1, n, "depth1")
    md = np.ascontiguousarray(np.asarray(min_depth, dtype=np.float64).reshape(-1))
    if md.shape[0] != 2:
        raise ValueError("min_depth must hold two values")
    ncam = 9 if variant in (L.CALIBRATED, L.SCALE_ONLY) else 2
    c0 = np.ascontiguousarray(np.asarray(cam0, dtype=np.float64).reshape(-1))
    c1 = np.ascontiguousarray(np.asarray(cam1, dtype=np.float64).reshape(-1))
    if c0.shape[0] != ncam or c1.shape[0] != ncam:
        raise ValueError("K0/K1 must be 3x3" if ncam == 9 else "pp0/pp1 must hold two values")
    if est_config is None:
        est_config = EstimatorConfig()
    o = options._to_c()
    c = est_config._to_c()
    model = L.mp_model()
    stats = L.mp_stats()
    idx = np.zeros(3 * max(n, 1), dtype=np.int32)
    code = L.lib().mp_estimate(variant, n, _dp(x0), _dp(x1), _dp(d0), _dp(d1), _dp(md), _dp(c0), _dp(c1),
                               ctypes.byref(o), ctypes.byref(c), ctypes.byref(model), ctypes.byref(stats),
                               idx.ctypes.data_as(L.c_int32_p), _DEFAULT_DEVICE if device is None else int(device))
    L.check(code)
    return _model_from_c(model, variant), _stats_from_c(stats, idx, n)


def HybridEstimatePoseScaleOffset(x0, x1, depth0, depth1, min_depth, K0, K1, options, est_config=None, device=None):
    """src/hybrid_pose_estimator.cpp:8-35 (bindings.cpp:169-170)."""
    return _estimate(L.CALIBRATED, x0, x1, depth0, depth1, min_depth, K0, K1, options, est_config, device)


def HybridEstimatePoseScaleOffsetSharedFocal(x0, x1, depth0, depth1, min_depth, pp0, pp1, options, est_config=None,
                                             device=None):
    """src/hybrid_pose_shared_focal_estimator.cpp:8-51 (bindings.cpp:171-172)."""
    return _estimate(L.SHARED_FOCAL, x0, x1, depth0, depth1, min_depth, pp0, pp1, options, est_config, device)


def HybridEstimatePoseScaleOffsetTwoFocal(x0, x1, depth0, depth1, min_depth, pp0, pp1, options, est_config=None,
                                          device=None):
    """src/hybrid_pose_two_focal_estimator.cpp:34-75 (bindings.cpp:173-174)."""
    return _estimate(L.TWO_FOCAL, x0, x1, depth0, depth1, min_depth, pp0, pp1, options, est_config, device)


def HybridEstimatePoseAndScale(x0, x1, depth0, depth1, K0, K1, options, est_config=None, device=None):
    """src/hybrid_pose_estimator.cpp:37-63, 297-442 (bindings.cpp:167-168): scale-only
    estimator (no depth offsets); returns (PoseAndScale, HybridRansacStatistics)."""
    return _estimate(L.SCALE_ONLY, x0, x1, depth0, depth1, [0.0, 0.0], K0, K1, options, est_config, device)


def estimate_scale_and_pose(X, Y, W):
    """src/solver.cpp:5-33 (bindings.cpp:156): weighted Procrustes with scale on the
    device; X, Y are 3 x N point matrices (columns), W the N weights."""
    X = np.asarray(X, dtype=np.float64)
    Y = np.asarray(Y, dtype=np.float64)
    if X.ndim != 2 or X.shape[0] != 3 or X.shape != Y.shape:
        raise ValueError("X and Y must be 3 x N matrices of the same shape")
    n = X.shape[1]
    W = _vec(W, n, "W")
    Xp = np.ascontiguousarray(X.T)
    Yp = np.ascontiguousarray(Y.T)
    out = L.mp_model()
    L.check(L.lib().mp_estimate_scale_and_pose(_dp(Xp), _dp(Yp), _dp(W), n, ctypes.byref(out), _DEFAULT_DEVICE))
    return _model_from_c(out, L.SCALE_ONLY)


def estimate_batch(variant, pairs, options, est_config=None, device=None, num_streams=4):
    """Many independent pairs on one device (host threads x HIP streams).

    pairs: list of dicts with x0, x1, depth0, depth1, min_depth, and K0/K1 (calibrated)
    or pp0/pp1.  Returns a list of (model, stats)."""
    if est_config is None:
        est_config = EstimatorConfig()
    x0s, x1s, d0s, d1s, mds, c0s, c1s, offs = [], [], [], [], [], [], [], [0]
    for p in pairs:
        x0 = _pts(p["x0"], "x0")
        n = x0.shape[0]
        x0s.append(x0)
        x1s.append(_pts(p["x1"], "x1"))
        d0s.append(_vec(p["depth0"], n, "depth0"))
        d1s.append(_vec(p["depth1"], n, "depth1"))
        mds.append(np.asarray(p["min_depth"], dtype=np.float64).reshape(2))
        if variant == L.CALIBRATED:
            c0s.append(np.asarray(p["K0"], dtype=np.float64).reshape(9))
            c1s.append(np.asarray(p["K1"], dtype=np.float64).reshape(9))
        else:
            c0s.append(np.asarray(p["pp0"], dtype=np.float64).reshape(2))
            c1s.append(np.asarray(p["pp1"], dtype=np.float64).reshape(2))
        offs.append(offs[-1] + n)
    P = len(pairs)
    cat = lambda xs, w: np.ascontiguousarray(np.concatenate(xs).reshape(-1)) if xs else np.zeros(w)
    X0, X1, D0, D1 = cat(x0s, 2), cat(x1s, 2), cat(d0s, 1), cat(d1s, 1)
    MD, C0, C1 = cat(mds, 2), cat(c0s, 9), cat(c1s, 9)
    offsets = np.asarray(offs, dtype=np.int64)
    models = (L.mp_model * max(P, 1))()
    stats = (L.mp_stats * max(P, 1))()
    idx = np.zeros(3 * max(offs[-1], 1), dtype=np.int32)
    o = options._to_c()
    c = est_config._to_c()
    code = L.lib().mp_estimate_batch(variant, P, offsets.ctypes.data_as(L.c_int64_p), _dp(X0), _dp(X1), _dp(D0),
                                     _dp(D1), _dp(MD), _dp(C0), _dp(C1), ctypes.byref(o), ctypes.byref(c), models,
                                     stats, idx.ctypes.data_as(L.c_int32_p),
                                     _DEFAULT_DEVICE if device is None else int(device), int(num_streams))
    L.check(code)
    out = []
    for p in range(P):
        n = offs[p + 1] - offs[p]
        out.append((_model_from_c(models[p], variant), _stats_from_c(stats[p], idx[3 * offs[p]:], n)))
    return out


def lm_refine_batch(variant, x0, x1, depth0, depth1, min_depth, cam0, cam1, options, est_config, problems,
                    device=None, on_host=False):
    """Batched device LM (the LO's Ceres solves, src/optimizer.h:48-125 over
    src/cost_functions.h): problems is a list of (kind, (idx0, idx1, idx2), model) with
    kind 0 = LeastSquares, 1 = NonMinimalSolver, idx* the residual blocks of the three
    data types and model a PoseScaleOffset* in problem units (SF/TF focals divided by
    the pair's normalize_points scale).  One device workgroup per problem.  Returns a
    list of (model, status): 1 refined, 0 no residuals, 2 infeasible constant block,
    3 too few data (unchanged)."""
    if est_config is None:
        est_config = EstimatorConfig()
    x0 = _pts(x0, "x0")
    n = x0.shape[0]
    x1 = _pts(x1, "x1")
    d0, d1 = _vec(depth0, n, "depth0"), _vec(depth1, n, "depth1")
    md = np.asarray(min_depth, dtype=np.float64).reshape(2)
    k = 9 if variant == L.CALIBRATED else 2
    c0 = np.ascontiguousarray(np.asarray(cam0, dtype=np.float64).reshape(k))
    c1 = np.ascontiguousarray(np.asarray(cam1, dtype=np.float64).reshape(k))
    P = len(problems)
    kinds = np.array([int(p[0]) for p in problems] or [0], dtype=np.int32)
    offs, idx = [0], []
    for _, lists, _m in problems:
        for t in range(3):
            a = np.asarray(lists[t], dtype=np.int32).reshape(-1)
            idx.append(a)
            offs.append(offs[-1] + len(a))
    offs = np.asarray(offs, dtype=np.int64)
    idx = np.ascontiguousarray(np.concatenate(idx) if idx and offs[-1] > 0 else np.zeros(1, dtype=np.int32))
    models = (L.mp_model * max(P, 1))()
    for j, (_, _, m) in enumerate(problems):
        models[j] = _model_to_c(m, variant)
    status = np.zeros(max(P, 1), dtype=np.int32)
    o = options._to_c()
    c = est_config._to_c()
    common = (variant, n, _dp(x0), _dp(x1), _dp(d0), _dp(d1), _dp(md), _dp(c0), _dp(c1), ctypes.byref(o),
              ctypes.byref(c), P, kinds.ctypes.data_as(L.c_int32_p), offs.ctypes.data_as(L.c_int64_p),
              idx.ctypes.data_as(L.c_int32_p), models, status.ctypes.data_as(L.c_int32_p))
    if on_host:  # test hook: the engine's host LM (the default LO path) on the same problems
        L.check(L.lib().mp_debug_lm_refine_host(*common))
    else:
        L.check(L.lib().mp_lm_refine_batch(*common, _DEFAULT_DEVICE if device is None else int(device)))
    return [(_model_from_c(models[j], variant), int(status[j])) for j in range(P)]


def bougnoux_focals_batch(F, device=None):
    """Squared Bougnoux focal lengths (f0^2, f1^2) of fundamental matrices F (k x 3 x 3,
    principal points at the origin) on the device: the two-focal 7-point tail's own
    code (src/hybrid_pose_two_focal_estimator.cpp:11-32; madpose/utils.py:25-56)."""
    F = np.ascontiguousarray(np.asarray(F, dtype=np.float64).reshape(-1, 9))
    out = np.zeros((len(F), 2))
    L.check(L.lib().mp_bougnoux_focals(len(F), _dp(F), _dp(out), _DEFAULT_DEVICE if device is None else int(device)))
    return out


def pose_eval_batch(T_0to1, R, t, thresholds=(5, 10, 20), t_thres=None, device=None):
    """compute_pose_error (madpose/utils.py:59-78) of k estimated poses and the pose
    AUC of max(err_R, err_t) at each threshold (degrees), in two device launches
    (SURVEY.md §8(f)4).  T_0to1: k x 4 x 4 ground truths; R: k x 3 x 3; t: k x 3.
    Returns (err_t, err_R, aucs): the per-pair errors as madpose.utils computes them
    and the AUCs of madpose_amd.utils.pose_auc (NaN errors count as misses)."""
    T = np.ascontiguousarray(np.asarray(T_0to1, dtype=np.float64).reshape(-1, 16))
    Rm = np.ascontiguousarray(np.asarray(R, dtype=np.float64).reshape(-1, 9))
    tv = np.ascontiguousarray(np.asarray(t, dtype=np.float64).reshape(-1, 3))
    if not (len(T) == len(Rm) == len(tv)):
        raise ValueError("T_0to1, R and t must hold the same number of poses")
    thr = np.ascontiguousarray(np.asarray(thresholds, dtype=np.float64).reshape(-1))
    if np.any(~(thr > 0)):
        raise ValueError("AUC thresholds must be positive")
    k = len(T)
    et, eR, aucs = np.zeros(max(k, 1)), np.zeros(max(k, 1)), np.zeros(max(len(thr), 1))
    L.check(L.lib().mp_pose_eval(k, _dp(Rm), _dp(tv), _dp(T), -1.0 if t_thres is None else float(t_thres), _dp(et),
                                 _dp(eR), len(thr), _dp(thr), _dp(aucs),
                                 _DEFAULT_DEVICE if device is None else int(device)))
    return et[:k].copy(), eR[:k].copy(), [float(a) for a in aucs[:len(thr)]]


def pose_auc_batch(errors, thresholds=(5, 10, 20), device=None):
    """Pose AUC of given per-pair errors (degrees) at each threshold on the device: the
    evaluator of pose_eval_batch for errors gathered elsewhere (e.g. from all ranks)."""
    e = np.ascontiguousarray(np.asarray(errors, dtype=np.float64).reshape(-1))
    thr = np.ascontiguousarray(np.asarray(thresholds, dtype=np.float64).reshape(-1))
    if np.any(~(thr > 0)):
        raise ValueError("AUC thresholds must be positive")
    aucs = np.zeros(max(len(thr), 1))
    L.check(L.lib().mp_pose_auc(len(e), _dp(e if len(e) else np.zeros(1)), len(thr), _dp(thr), _dp(aucs),
                                _DEFAULT_DEVICE if device is None else int(device)))
    return [float(a) for a in aucs[:len(thr)]]


def get_depths_batch(images, depth_maps, mkpts, device=None):
    """madpose.utils.get_depths (madpose/utils.py:4-22) for many pairs in one device
    launch.  images: the images (only their shapes are used) or (h, w) tuples;
    depth_maps: 2-D float32 or float64 arrays (one dtype for the batch); mkpts: n_p x 2
    keypoints per map.  Returns one array of depths per map (the maps' dtype),
    bit-identical to the numpy reference."""
    if not (len(images) == len(depth_maps) == len(mkpts)):
        raise ValueError("images, depth_maps and mkpts must have the same length")
    P = len(depth_maps)
    if P == 0:
        return []
    dt = np.result_type(*[np.asarray(d).dtype for d in depth_maps])
    if dt not in (np.float32, np.float64):
        dt = np.dtype(np.float64)
    maps, dims, pts, offs = [], [], [], [0]
    for img, dm, kp in zip(images, depth_maps, mkpts):
        dm = np.asarray(dm)
        if dm.ndim != 2:
            raise ValueError("depth maps must be 2-D")
        ih, iw = (img if isinstance(img, tuple) else np.shape(img))[:2]
        kp = np.ascontiguousarray(kp, dtype=np.float64).reshape(-1, 2)
        maps.append(np.ascontiguousarray(dm, dtype=dt).reshape(-1))
        dims.append([dm.shape[0], dm.shape[1], ih, iw])
        pts.append(kp)
        offs.append(offs[-1] + len(kp))
    M = np.ascontiguousarray(np.concatenate(maps))
    D = np.ascontiguousarray(np.asarray(dims, dtype=np.int64).reshape(-1))
    O = np.asarray(offs, dtype=np.int64)
    X = np.ascontiguousarray(np.concatenate(pts).reshape(-1)) if offs[-1] else np.zeros(2)
    out = np.zeros(max(offs[-1], 1), dtype=dt)
    L.check(L.lib().mp_get_depths(0 if dt == np.float32 else 1, P, M.ctypes.data_as(ctypes.c_void_p),
                                  D.ctypes.data_as(L.c_int64_p), O.ctypes.data_as(L.c_int64_p), _dp(X),
                                  out.ctypes.data_as(ctypes.c_void_p),
                                  _DEFAULT_DEVICE if device is None else int(device)))
    return [out[offs[p]:offs[p + 1]].copy() for p in range(P)]


# ---------------------------------------------------------------------------
# standalone solver bindings (src/bindings.cpp:156-166)
def _homog_pm(a, k, name):
    a = np.asarray(a, dtype=np.float64)
    if a.shape == (3, k):
        return np.ascontiguousarray(a.T)
    raise ValueError(f"{name} must be a 3 x {k} matrix of homogeneous points (columns)")


def _solve_ss(variant, x_homo, y_homo, depth_x, depth_y):
    k = 3 if variant == L.CALIBRATED else 4
    x = _homog_pm(x_homo, k, "x_homo")
    y = _homog_pm(y_homo, k, "y_homo")
    dx = _vec(depth_x, k, "depth_x")
    dy = _vec(depth_y, k, "depth_y")
    w = [4, 5, 6][variant]
    out = np.zeros(8 * w)
    n = L.lib().mp_solve_scale_and_shift(variant, _dp(x), _dp(y), _dp(dx), _dp(dy), _dp(out), 8, _DEFAULT_DEVICE)
    if n < 0:
        L.check(-n)
    return [out[i * w:(i + 1) * w].copy() for i in range(n)]


def _solve_pose(variant, x_homo, y_homo, depth_x, depth_y, alt=0):
    k = 3 if variant == L.CALIBRATED else 4
    x = _homog_pm(x_homo, k, "x_homo")
    y = _homog_pm(y_homo, k, "y_homo")
    dx = _vec(depth_x, k, "depth_x")
    dy = _vec(depth_y, k, "depth_y")
    out = (L.mp_model * 8)()
    if alt:
        n = L.lib().mp_solve_scale_shift_pose_alt(variant, alt, _dp(x), _dp(y), _dp(dx), _dp(dy), out, 8,
                                                  _DEFAULT_DEVICE)
    else:
        n = L.lib().mp_solve_scale_shift_pose(variant, _dp(x), _dp(y), _dp(dx), _dp(dy), out, 8, _DEFAULT_DEVICE)
    if n < 0:
        L.check(-n)
    return [_model_from_c(out[i], variant) for i in range(n)]


def solve_scale_and_shift(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:35-125: list of (1, b1, a2, b2*a2)."""
    return _solve_ss(L.CALIBRATED, x_homo, y_homo, depth_x, depth_y)


def solve_scale_and_shift_shared_focal(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:127-293: list of (1, b1, a2, b2*a2, f)."""
    return _solve_ss(L.SHARED_FOCAL, x_homo, y_homo, depth_x, depth_y)


def solve_scale_and_shift_two_focal(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:295-480: list of (1, b1, a2, b2*a2, f1, f2)."""
    return _solve_ss(L.TWO_FOCAL, x_homo, y_homo, depth_x, depth_y)


def solve_scale_shift_pose(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:482-534 (wrapper :1408-1415)."""
    return _solve_pose(L.CALIBRATED, x_homo, y_homo, depth_x, depth_y)


def solve_scale_shift_pose_shared_focal(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:682-739 (wrapper :1417-1424)."""
    return _solve_pose(L.SHARED_FOCAL, x_homo, y_homo, depth_x, depth_y)


def solve_scale_shift_pose_two_focal(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:986-1043 (wrapper :1426-1433)."""
    return _solve_pose(L.TWO_FOCAL, x_homo, y_homo, depth_x, depth_y)


def relpose_5pt(x1, x2):
    """Device 5-point solver on unit bearings (5 x 3 each): list of PoseScaleOffset (scale 1)."""
    b1 = np.ascontiguousarray(np.asarray(x1, dtype=np.float64).reshape(5, 3))
    b2 = np.ascontiguousarray(np.asarray(x2, dtype=np.float64).reshape(5, 3))
    out = (L.mp_model * 16)()
    n = L.lib().mp_relpose_5pt(_dp(b1), _dp(b2), out, 16, _DEFAULT_DEVICE)
    if n < 0:
        L.check(-n)
    return [_model_from_c(out[i], L.CALIBRATED) for i in range(min(n, 16))]


def _point_direct(fn, k, variant, x0, x1):
    a = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).reshape(k, 2))
    b = np.ascontiguousarray(np.asarray(x1, dtype=np.float64).reshape(k, 2))
    out = (L.mp_model * 16)()
    n = fn(_dp(a), _dp(b), out, 16, _DEFAULT_DEVICE)
    if n < 0:
        L.check(-n)
    return [_model_from_c(out[i], variant) for i in range(min(n, 16))]


def relpose_6pt_shared_focal(x0, x1):
    """Device shared-focal 6-point solver on normalized 2-D points (6 x 2 each):
    PoseScaleOffsetSharedFocal candidates before the depth fit."""
    return _point_direct(L.lib().mp_relpose_6pt_shared_focal, 6, L.SHARED_FOCAL, x0, x1)


def relpose_7pt_two_focal(x0, x1):
    """Device 7-point + Bougnoux + recoverPose on normalized 2-D points (7 x 2 each):
    PoseScaleOffsetTwoFocal candidates before the depth fit."""
    return _point_direct(L.lib().mp_relpose_7pt_two_focal, 7, L.TWO_FOCAL, x0, x1)


def solve_scale_shift_pose_ours(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:623-680 (the use_ours calibrated MD solver)."""
    return _solve_pose(L.CALIBRATED, x_homo, y_homo, depth_x, depth_y, alt=1)


def solve_scale_shift_pose_shared_focal_ours(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:818-984 (the use_ours shared-focal MD solver)."""
    return _solve_pose(L.SHARED_FOCAL, x_homo, y_homo, depth_x, depth_y, alt=1)


def solve_scale_shift_pose_two_focal_ours(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:1045-1148 (the use_ours two-focal MD solver)."""
    return _solve_pose(L.TWO_FOCAL, x_homo, y_homo, depth_x, depth_y, alt=1)


def solve_scale_shift_pose_two_focal_4p4d(x_homo, y_homo, depth_x, depth_y):
    """src/solver.cpp:1287-1406 (the use_4p4d two-focal solver)."""
    return _solve_pose(L.TWO_FOCAL, x_homo, y_homo, depth_x, depth_y, alt=2)


def score_models(variant, x0, x1, depth0, depth1, cam0, cam1, options, est_config, models, with_errors=False,
                 host_lo=False, fast_bounds=None):
    """Device ScoreModel over explicit models given in problem units (tests / diagnostics).
    host_lo=True: the engine's host LO sweep instead (mp_debug_lo_sweep; no device);
    fast_bounds (host_lo only): an (nm, 2) float64 array filled with the LO's fast sums
    and their bounds (lo_sweep.h lo_sweep_fast)."""
    x0 = _pts(x0, "x0")
    x1 = _pts(x1, "x1")
    n = x0.shape[0]
    d0 = _vec(depth0, n, "depth0")
    d1 = _vec(depth1, n, "depth1")
    c0 = np.ascontiguousarray(np.asarray(cam0, dtype=np.float64).reshape(-1))
    c1 = np.ascontiguousarray(np.asarray(cam1, dtype=np.float64).reshape(-1))
    nm = len(models)
    arr = (L.mp_model * max(nm, 1))(*[_model_to_c(m, variant) for m in models])
    scores = np.zeros(max(nm, 1))
    errors = np.zeros((max(nm, 1), 3, n)) if with_errors else None
    o = options._to_c()
    c = (est_config or EstimatorConfig())._to_c()
    if host_lo:
        code = L.lib().mp_debug_lo_sweep(variant, n, _dp(x0), _dp(x1), _dp(d0), _dp(d1), _dp(c0), _dp(c1),
                                         ctypes.byref(o), ctypes.byref(c), arr, nm, _dp(scores),
                                         _dp(errors) if with_errors else None,
                                         _dp(fast_bounds) if fast_bounds is not None else None)
    else:
        code = L.lib().mp_score_models(variant, n, _dp(x0), _dp(x1), _dp(d0), _dp(d1), _dp(c0), _dp(c1),
                                       ctypes.byref(o), ctypes.byref(c), arr, nm, _dp(scores),
                                       _dp(errors) if with_errors else None, _DEFAULT_DEVICE)
    L.check(code)
    return (scores[:nm], errors[:nm]) if with_errors else scores[:nm]


def debug_score_batch(variant, x0, x1, depth0, depth1, cam0, cam1, options, est_config, iterations, best,
                      exit=True, record_skip=True):
    """The estimator's scoring kernel on explicit per-iteration model lists (test hook,
    mp_debug_score_batch).  iterations: list of model lists (problem units).  Returns
    (best scores, slots with the ambiguity / uncertainty bits, record models, bounds):
    bounds["hi"], bounds["lo"] per iteration and bounds["tie"][b][m], each model's
    screening margin (mp_score.h score_margins)."""
    x0 = _pts(x0, "x0")
    x1 = _pts(x1, "x1")
    n = x0.shape[0]
    d0 = _vec(depth0, n, "depth0")
    d1 = _vec(depth1, n, "depth1")
    c0 = np.ascontiguousarray(np.asarray(cam0, dtype=np.float64).reshape(-1))
    c1 = np.ascontiguousarray(np.asarray(cam1, dtype=np.float64).reshape(-1))
    M = {0: 10, 1: 16, 2: 4, 3: 10}[variant]
    B = len(iterations)
    arr = (L.mp_model * (B * M))()
    counts = np.zeros(B, dtype=np.int32)
    for b, ms in enumerate(iterations):
        counts[b] = len(ms)
        for m, mod in enumerate(ms):
            arr[b * M + m] = _model_to_c(mod, variant)
    rb = np.zeros(B)
    rs = np.zeros(B, dtype=np.int32)
    rec = (L.mp_model * B)()
    hilo = np.zeros(2 * B)
    ties = np.zeros(B * M)
    o = options._to_c()
    c = (est_config or EstimatorConfig())._to_c()
    flags = (1 if exit else 0) | (2 if record_skip else 0)
    L.check(L.lib().mp_debug_score_batch(variant, n, _dp(x0), _dp(x1), _dp(d0), _dp(d1), _dp(c0), _dp(c1),
                                         ctypes.byref(o), ctypes.byref(c), B, counts.ctypes.data_as(L.c_int32_p),
                                         arr, float(best), flags, _dp(rb), rs.ctypes.data_as(L.c_int32_p), rec,
                                         _dp(hilo), _dp(ties), _DEFAULT_DEVICE))
    bounds = {"hi": hilo[0::2].copy(), "lo": hilo[1::2].copy(),
              "tie": [ties[b * M:b * M + counts[b]].copy() for b in range(B)]}
    return rb, rs, [_model_from_c(rec[b], variant) for b in range(B)], bounds


def debug_score_terms(variant, x0, x1, depth0, depth1, cam0, cam1, options, est_config, models):
    """score_batch's per-correspondence errors of explicit models (test hook,
    mp_debug_score_terms).  Returns (errors [nm x 3 x n], flags [nm x n], taus [nm x 3],
    ties [nm])."""
    x0 = _pts(x0, "x0")
    x1 = _pts(x1, "x1")
    n = x0.shape[0]
    d0 = _vec(depth0, n, "depth0")
    d1 = _vec(depth1, n, "depth1")
    c0 = np.ascontiguousarray(np.asarray(cam0, dtype=np.float64).reshape(-1))
    c1 = np.ascontiguousarray(np.asarray(cam1, dtype=np.float64).reshape(-1))
    nm = len(models)
    arr = (L.mp_model * max(nm, 1))()
    for m, mod in enumerate(models):
        arr[m] = _model_to_c(mod, variant)
    err = np.zeros(max(nm, 1) * 3 * n)
    flags = np.zeros(max(nm, 1) * n, dtype=np.int32)
    taus = np.zeros(max(nm, 1) * 3)
    ties = np.zeros(max(nm, 1))
    o = options._to_c()
    c = (est_config or EstimatorConfig())._to_c()
    L.check(L.lib().mp_debug_score_terms(variant, n, _dp(x0), _dp(x1), _dp(d0), _dp(d1), _dp(c0), _dp(c1),
                                         ctypes.byref(o), ctypes.byref(c), arr, nm, _dp(err),
                                         flags.ctypes.data_as(L.c_int32_p), _dp(taus), _dp(ties), _DEFAULT_DEVICE))
    return (err[:nm * 3 * n].reshape(nm, 3, n), flags[:nm * n].reshape(nm, n), taus[:3 * nm].reshape(nm, 3),
            ties[:nm])


def device_count():
    return int(L.lib().mp_device_count())


def version():
    return L.lib().mp_version().decode()


def profile_enable(on=True):
    """Turn on HIP-event timing of the estimator's batch kernels (process-wide)."""
    L.check(L.lib().mp_profile_enable(1 if on else 0))


def profile_reset():
    L.check(L.lib().mp_profile_reset())


def profile_read():
    """Totals since the last reset: batches, iterations, hypotheses, correspondences,
    sweeps, solve_ms, score_ms (device time from HIP events on the engine stream)."""
    p = L.mp_kernel_profile()
    L.check(L.lib().mp_profile_read(ctypes.byref(p)))
    return {name: getattr(p, name) for name, _ in p._fields_}
