"""ORACLE -- test infrastructure only (see oracle/README.md).

ctypes binding of oracle/_build/liboracle.so, the CPU restatement of the reference's
hybrid LO-MSAC estimator.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package, and only as the checker.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


class OrRansacOptions(ctypes.Structure):
    _fields_ = [
        ("success_probability", ctypes.c_double),
        ("squared_inlier_thresholds", ctypes.c_double * 2),
        ("data_type_weights", ctypes.c_double * 2),
        ("threshold_multiplier", ctypes.c_double),
        ("min_num_iterations", ctypes.c_uint32),
        ("max_num_iterations", ctypes.c_uint32),
        ("max_num_iterations_per_solver", ctypes.c_uint32),
        ("random_seed", ctypes.c_uint32),
        ("num_lo_steps", ctypes.c_int32),
        ("num_lsq_iterations", ctypes.c_int32),
        ("min_sample_multiplicator", ctypes.c_int32),
        ("non_min_sample_multiplier", ctypes.c_int32),
        ("lo_starting_iterations", ctypes.c_int32),
        ("final_least_squares", ctypes.c_int32),
        ("use_ours", ctypes.c_int32),
        ("use_4p4d", ctypes.c_int32),
    ]


class OrEstimatorConfig(ctypes.Structure):
    _fields_ = [
        ("ceres_function_tolerance", ctypes.c_double),
        ("ceres_gradient_tolerance", ctypes.c_double),
        ("ceres_parameter_tolerance", ctypes.c_double),
        ("ceres_max_num_iterations", ctypes.c_double),
        ("solver_type", ctypes.c_int32),
        ("score_type", ctypes.c_int32),
        ("lo_type", ctypes.c_int32),
        ("min_depth_constraint", ctypes.c_int32),
        ("use_shift", ctypes.c_int32),
        ("ceres_use_nonmonotonic_steps", ctypes.c_int32),
        ("ceres_num_threads", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class OrModel(ctypes.Structure):
    _fields_ = [
        ("R", ctypes.c_double * 9),
        ("t", ctypes.c_double * 3),
        ("scale", ctypes.c_double),
        ("offset0", ctypes.c_double),
        ("offset1", ctypes.c_double),
        ("focal0", ctypes.c_double),
        ("focal1", ctypes.c_double),
    ]


class OrStats(ctypes.Structure):
    _fields_ = [
        ("best_model_score", ctypes.c_double),
        ("inlier_ratios", ctypes.c_double * 3),
        ("num_hypotheses", ctypes.c_uint64),
        ("num_lo_sweeps", ctypes.c_uint64),
        ("num_iterations_total", ctypes.c_uint32),
        ("num_iterations_per_solver", ctypes.c_uint32 * 2),
        ("best_num_inliers", ctypes.c_int32),
        ("best_solver_type", ctypes.c_int32),
        ("number_lo_iterations", ctypes.c_int32),
        ("num_inliers", ctypes.c_int32 * 3),
        ("num_batches", ctypes.c_int32),
        ("seconds_total", ctypes.c_double),
        ("seconds_lo", ctypes.c_double),
        ("seconds_gpu_wait", ctypes.c_double),
    ]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"oracle library missing: {_LIB_PATH} (run `make -C oracle`)")
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def model_to_dict(m):
    return dict(
        R=np.array(m.R[:]).reshape(3, 3),
        t=np.array(m.t[:]),
        scale=m.scale,
        offset0=m.offset0,
        offset1=m.offset1,
        focal0=m.focal0,
        focal1=m.focal1,
    )


def md_scale_shift(variant, x_homo_pm, y_homo_pm, dx, dy):
    """x_homo_pm: K x 3 point-major homogeneous points.  Returns (k, width) array."""
    w = [4, 5, 6][variant]
    out = np.zeros((16, w))
    n = lib().oracle_md_scale_shift(
        variant, _dp(_c(x_homo_pm)), _dp(_c(y_homo_pm)), _dp(_c(dx)), _dp(_c(dy)), _dp(out), 16
    )
    return out[:n].copy()


def md_pose(variant, x_homo_pm, y_homo_pm, dx, dy):
    out = (OrModel * 16)()
    n = lib().oracle_md_pose(variant, _dp(_c(x_homo_pm)), _dp(_c(y_homo_pm)), _dp(_c(dx)), _dp(_c(dy)), out, 16)
    return [model_to_dict(out[i]) for i in range(min(n, 16))]


def md_pose_alt(variant, alt, x_homo_pm, y_homo_pm, dx, dy):
    """use_ours (alt=1) / use_4p4d (alt=2, two-focal) MD solvers; same layout as md_pose."""
    out = (OrModel * 16)()
    n = lib().oracle_md_pose_alt(variant, alt, _dp(_c(x_homo_pm)), _dp(_c(y_homo_pm)), _dp(_c(dx)), _dp(_c(dy)),
                                 out, 16)
    return [model_to_dict(out[i]) for i in range(min(n, 16))]


def estimate_scale_and_pose(X, Y, W):
    """src/solver.cpp:5-33; X, Y: k x 3 points, W: k weights."""
    X, Y, W = _c(X), _c(Y), _c(W)
    out = OrModel()
    lib().oracle_scale_and_pose(_dp(X), _dp(Y), _dp(W), len(W), ctypes.byref(out))
    return model_to_dict(out)


def relpose_5pt(b1, b2):
    out = (OrModel * 32)()
    n = lib().oracle_relpose_5pt(_dp(_c(b1)), _dp(_c(b2)), out, 32)
    return [model_to_dict(out[i]) for i in range(min(n, 32))]


def relpose_5pt_E(b1, b2):
    """Root stage of the 5pt restatement (PoseLib: Nister + Sturm bisection): the
    essential matrices (k, 3, 3) and the real roots z of det B(z), ascending."""
    E = np.zeros((16, 9))
    roots = np.zeros(10)
    nr = ctypes.c_int(0)
    n = lib().oracle_relpose_5pt_E(_dp(_c(b1)), _dp(_c(b2)), _dp(E), 16, _dp(roots), ctypes.byref(nr))
    return E[:n].reshape(-1, 3, 3).copy(), roots[:min(nr.value, 10)].copy()


def relpose_5pt_action(b1, b2):
    """The same 5-point problem by Stewenius' action matrix (an independent algorithm)."""
    out = (OrModel * 32)()
    n = lib().oracle_relpose_5pt_action(_dp(_c(b1)), _dp(_c(b2)), out, 32)
    return [model_to_dict(out[i]) for i in range(min(n, 32))]


def relpose_7pt_svd(b1, b2):
    """The 7-point problem by an SVD null space + companion roots (independent cross-check)."""
    out = np.zeros((8, 9))
    n = lib().oracle_relpose_7pt_svd(_dp(_c(b1)), _dp(_c(b2)), _dp(out), 8)
    return out[:n].reshape(-1, 3, 3).copy()


def solve_cubic_real(c2, c1, c0):
    """PoseLib solve_cubic_real: real roots of x^3 + c2 x^2 + c1 x + c0 (1 or 3)."""
    lib().oracle_solve_cubic_real.argtypes = [ctypes.c_double] * 3 + [ctypes.POINTER(ctypes.c_double)]
    out = np.zeros(3)
    n = lib().oracle_solve_cubic_real(float(c2), float(c1), float(c0), _dp(out))
    return out[:n].copy()


def eigen_svd3(A):
    """Eigen JacobiSVD<MatrixXd>(A, ComputeFullU | ComputeFullV) restatement (la.cpp): U, V."""
    A = _c(np.asarray(A).reshape(3, 3))
    U, V = np.zeros((3, 3)), np.zeros((3, 3))
    lib().oracle_eigen_svd3(_dp(A), _dp(U), _dp(V))
    return U, V


def sixpt_roots(b1, b2):
    """Root stage of the 6pt restatement: positive real u = f^2 (deflated companion)."""
    out = np.zeros(32)
    n = lib().oracle_6pt_roots(_dp(_c(b1)), _dp(_c(b2)), _dp(out), 32)
    return np.sort(out[:n])


def relpose_6pt_shared_focal(b1, b2):
    """PoseLib relpose_6pt_shared_focal restatement: list of dicts (focal in focal0)."""
    out = (OrModel * 64)()
    n = lib().oracle_relpose_6pt(_dp(_c(b1)), _dp(_c(b2)), out, 64)
    return [model_to_dict(out[i]) for i in range(min(n, 64))]


def relpose_7pt(b1, b2):
    """PoseLib relpose_7pt restatement: (k, 3, 3) fundamental matrices."""
    out = np.zeros((8, 9))
    n = lib().oracle_relpose_7pt(_dp(_c(b1)), _dp(_c(b2)), _dp(out), 8)
    return out[:n].reshape(-1, 3, 3).copy()


def bougnoux_focals(F):
    out = np.zeros(2)
    lib().oracle_bougnoux(_dp(_c(F)), _dp(out))
    return out


def recover_pose(E, p0, p1, thresh=1e9):
    p0, p1 = _c(p0), _c(p1)
    R = np.zeros(9)
    t = np.zeros(3)
    lib().oracle_recover_pose.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_double] + [ctypes.c_void_p] * 2
    good = lib().oracle_recover_pose(_dp(_c(E)), _dp(p0), _dp(p1), len(p0), thresh, _dp(R), _dp(t))
    return R.reshape(3, 3), t, good


def score_models(variant, x0, x1, d0, d1, cam0, cam1, opts, cfg, models):
    """models: list of OrModel (problem units).  Returns (scores, errors[m,3,n], norm_scale)."""
    n = len(d0)
    nm = len(models)
    arr = (OrModel * max(nm, 1))(*models)
    scores = np.zeros(max(nm, 1))
    errors = np.zeros((max(nm, 1), 3, n))
    ns = ctypes.c_double(0)
    lib().oracle_score_models(
        variant, ctypes.c_int64(n), _dp(_c(x0)), _dp(_c(x1)), _dp(_c(d0)), _dp(_c(d1)), _dp(_c(cam0)), _dp(_c(cam1)),
        ctypes.byref(opts), ctypes.byref(cfg), arr, nm, _dp(scores), _dp(errors), ctypes.byref(ns)
    )
    return scores[:nm], errors[:nm], ns.value


def least_squares(variant, x0, x1, d0, d1, min_depth, cam0, cam1, opts, cfg, kind, samples, model):
    """LeastSquares (kind 0) / NonMinimalSolver (kind 1) on one sample (three index
    lists) from `model` (dict with R, t, scale, offset0, offset1, focal0, focal1;
    problem units).  Returns (refined model dict, ran)."""
    n = len(d0)
    m = OrModel()
    m.R[:] = list(np.asarray(model["R"], dtype=np.float64).reshape(9))
    m.t[:] = list(np.asarray(model["t"], dtype=np.float64).reshape(3))
    for k in ("scale", "offset0", "offset1", "focal0", "focal1"):
        setattr(m, k, float(model[k]))
    ss = [np.ascontiguousarray(np.asarray(s, dtype=np.int32).reshape(-1)) for s in samples]
    ip = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    ran = lib().oracle_least_squares(
        variant, ctypes.c_int64(n), _dp(_c(x0)), _dp(_c(x1)), _dp(_c(d0)), _dp(_c(d1)), _dp(_c(min_depth)),
        _dp(_c(cam0)), _dp(_c(cam1)), ctypes.byref(opts), ctypes.byref(cfg), int(kind), ip(ss[0]), len(ss[0]),
        ip(ss[1]), len(ss[1]), ip(ss[2]), len(ss[2]), ctypes.byref(m))
    return model_to_dict(m), bool(ran)


def estimate(variant, x0, x1, d0, d1, min_depth, cam0, cam1, opts, cfg):
    """Returns (model dict, stats struct, [inlier index arrays x3])."""
    n = len(d0)
    model = OrModel()
    stats = OrStats()
    idx = np.zeros(3 * max(n, 1), dtype=np.int32)
    rc = lib().oracle_estimate(
        variant, ctypes.c_int64(n), _dp(_c(x0)), _dp(_c(x1)), _dp(_c(d0)), _dp(_c(d1)), _dp(_c(min_depth)),
        _dp(_c(cam0)), _dp(_c(cam1)), ctypes.byref(opts), ctypes.byref(cfg), ctypes.byref(model), ctypes.byref(stats),
        idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
    )
    if rc != 0:
        raise RuntimeError("oracle_estimate failed (model replay out of step?)")
    inl = [idx[t * n: t * n + stats.num_inliers[t]].copy() for t in range(3)]
    return model_to_dict(model), stats, inl


def iteration_stream(variant, n, seed, solver_type, iterations):
    types = np.zeros(iterations, dtype=np.int32)
    idx = np.zeros(8 * iterations, dtype=np.int32)
    lib().oracle_iteration_stream(variant, n, ctypes.c_uint32(seed), solver_type, iterations,
                                  types.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                  idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return types, idx.reshape(iterations, 8)
