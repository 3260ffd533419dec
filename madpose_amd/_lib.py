"""ctypes binding of libmadpose_mi355x.so (C ABI: include/madpose_mi355x.h).

The library is built in-tree by madpose_amd/build.py (or __graft_entry__.build()).
There is no CPU fallback: if the library is missing, importing the API raises; if no
MI355X is visible, every compute call raises RuntimeError.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# (MADPOSE_LIB_VARIANT=name loads lib/libmadpose_mi355x_<name>.so instead: same-box A/B
# of two builds)
_VARIANT = os.environ.get("MADPOSE_LIB_VARIANT", "")
LIB_PATH = os.path.join(_HERE, "lib", "libmadpose_mi355x" + (f"_{_VARIANT}" if _VARIANT.isidentifier() else "") + ".so")

MP_OK, MP_EINVAL, MP_EDEVICE = 0, 1, 2
CALIBRATED, SHARED_FOCAL, TWO_FOCAL, SCALE_ONLY = 0, 1, 2, 3

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int32_p = ctypes.POINTER(ctypes.c_int32)
c_int64_p = ctypes.POINTER(ctypes.c_int64)


class mp_ransac_options(ctypes.Structure):
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


class mp_estimator_config(ctypes.Structure):
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


class mp_model(ctypes.Structure):
    _fields_ = [
        ("R", ctypes.c_double * 9),
        ("t", ctypes.c_double * 3),
        ("scale", ctypes.c_double),
        ("offset0", ctypes.c_double),
        ("offset1", ctypes.c_double),
        ("focal0", ctypes.c_double),
        ("focal1", ctypes.c_double),
    ]


class mp_stats(ctypes.Structure):
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


class mp_kernel_profile(ctypes.Structure):
    _fields_ = [
        ("batches", ctypes.c_uint64),
        ("iterations", ctypes.c_uint64),
        ("hypotheses", ctypes.c_uint64),
        ("correspondences", ctypes.c_uint64),
        ("sweeps", ctypes.c_uint64),
        ("solve_ms", ctypes.c_double),
        ("score_ms", ctypes.c_double),
        ("lm_calls", ctypes.c_uint64),
        ("lm_wall_ms", ctypes.c_double),
        ("sweep_wall_ms", ctypes.c_double),
        ("sample_wall_ms", ctypes.c_double),
        ("wait_wall_ms", ctypes.c_double),
        ("run_wall_ms", ctypes.c_double),
        ("lm_blocks", ctypes.c_uint64),
        ("lm_big_calls", ctypes.c_uint64),
        ("lm_big_wall_ms", ctypes.c_double),
        ("model_trips", ctypes.c_uint64),
        ("model_trips_full", ctypes.c_uint64),
        ("accepted", ctypes.c_uint64),
        ("scored", ctypes.c_uint64),
        ("tie_checks", ctypes.c_uint64),
    ]


EXPORTS = {
    "mp_estimate": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p, c_double_p, c_double_p,
                                   c_double_p, c_double_p, c_double_p, ctypes.POINTER(mp_ransac_options),
                                   ctypes.POINTER(mp_estimator_config), ctypes.POINTER(mp_model),
                                   ctypes.POINTER(mp_stats), c_int32_p, ctypes.c_int]),
    "mp_estimate_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int32, c_int64_p, c_double_p, c_double_p, c_double_p,
                                         c_double_p, c_double_p, c_double_p, c_double_p,
                                         ctypes.POINTER(mp_ransac_options), ctypes.POINTER(mp_estimator_config),
                                         ctypes.POINTER(mp_model), ctypes.POINTER(mp_stats), c_int32_p, ctypes.c_int,
                                         ctypes.c_int]),
    "mp_get_depths": (ctypes.c_int, [ctypes.c_int, ctypes.c_int32, ctypes.c_void_p, c_int64_p, c_int64_p, c_double_p,
                                     ctypes.c_void_p, ctypes.c_int]),
    "mp_lm_refine_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p, c_double_p, c_double_p,
                                          c_double_p, c_double_p, c_double_p, ctypes.POINTER(mp_ransac_options),
                                          ctypes.POINTER(mp_estimator_config), ctypes.c_int32, c_int32_p, c_int64_p,
                                          c_int32_p, ctypes.POINTER(mp_model), c_int32_p, ctypes.c_int]),
    "mp_debug_lm_refine_host": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p, c_double_p,
                                               c_double_p, c_double_p, c_double_p, c_double_p,
                                               ctypes.POINTER(mp_ransac_options), ctypes.POINTER(mp_estimator_config),
                                               ctypes.c_int32, c_int32_p, c_int64_p, c_int32_p,
                                               ctypes.POINTER(mp_model), c_int32_p]),
    "mp_bougnoux_focals": (ctypes.c_int, [ctypes.c_int64, c_double_p, c_double_p, ctypes.c_int]),
    "mp_pose_eval": (ctypes.c_int, [ctypes.c_int64, c_double_p, c_double_p, c_double_p, ctypes.c_double, c_double_p,
                                    c_double_p, ctypes.c_int32, c_double_p, c_double_p, ctypes.c_int]),
    "mp_pose_auc": (ctypes.c_int, [ctypes.c_int64, c_double_p, ctypes.c_int32, c_double_p, c_double_p, ctypes.c_int]),
    "mp_estimate_scale_and_pose": (ctypes.c_int, [c_double_p, c_double_p, c_double_p, ctypes.c_int64,
                                                  ctypes.POINTER(mp_model), ctypes.c_int]),
    "mp_solve_scale_and_shift": (ctypes.c_int, [ctypes.c_int, c_double_p, c_double_p, c_double_p, c_double_p,
                                                c_double_p, ctypes.c_int, ctypes.c_int]),
    "mp_solve_scale_shift_pose": (ctypes.c_int, [ctypes.c_int, c_double_p, c_double_p, c_double_p, c_double_p,
                                                 ctypes.POINTER(mp_model), ctypes.c_int, ctypes.c_int]),
    "mp_solve_scale_shift_pose_alt": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_double_p, c_double_p, c_double_p,
                                                     c_double_p, ctypes.POINTER(mp_model), ctypes.c_int, ctypes.c_int]),
    "mp_score_models": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p, c_double_p, c_double_p,
                                       c_double_p, c_double_p, ctypes.POINTER(mp_ransac_options),
                                       ctypes.POINTER(mp_estimator_config), ctypes.POINTER(mp_model), ctypes.c_int32,
                                       c_double_p, c_double_p, ctypes.c_int]),
    "mp_debug_score_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p, c_double_p,
                                            c_double_p, c_double_p, c_double_p, ctypes.POINTER(mp_ransac_options),
                                            ctypes.POINTER(mp_estimator_config), ctypes.c_int32, c_int32_p,
                                            ctypes.POINTER(mp_model), ctypes.c_double, ctypes.c_int32, c_double_p,
                                            c_int32_p, ctypes.POINTER(mp_model), c_double_p, c_double_p,
                                            ctypes.c_int]),
    "mp_debug_score_terms": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p, c_double_p,
                                            c_double_p, c_double_p, c_double_p, ctypes.POINTER(mp_ransac_options),
                                            ctypes.POINTER(mp_estimator_config), ctypes.POINTER(mp_model),
                                            ctypes.c_int32, c_double_p, c_int32_p, c_double_p, c_double_p,
                                            ctypes.c_int]),
    "mp_debug_lo_sweep": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p, c_double_p, c_double_p,
                                         c_double_p, c_double_p, ctypes.POINTER(mp_ransac_options),
                                         ctypes.POINTER(mp_estimator_config), ctypes.POINTER(mp_model), ctypes.c_int32,
                                         c_double_p, c_double_p, c_double_p]),
    "mp_relpose_5pt": (ctypes.c_int, [c_double_p, c_double_p, ctypes.POINTER(mp_model), ctypes.c_int, ctypes.c_int]),
    "mp_debug_pt5_roots": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p, c_double_p,
                                          ctypes.POINTER(ctypes.c_int32), ctypes.c_int]),
    "mp_debug_pt_roots": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int64, c_double_p, c_double_p,
                                         c_double_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]),
    "mp_relpose_6pt_shared_focal": (ctypes.c_int, [c_double_p, c_double_p, ctypes.POINTER(mp_model), ctypes.c_int,
                                                   ctypes.c_int]),
    "mp_relpose_7pt_two_focal": (ctypes.c_int, [c_double_p, c_double_p, ctypes.POINTER(mp_model), ctypes.c_int,
                                                ctypes.c_int]),
    "mp_debug_random_stream": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32,
                                              ctypes.c_int32, c_double_p]),
    "mp_debug_iteration_stream": (ctypes.c_int, [ctypes.c_int, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int32,
                                                 ctypes.c_int32, c_int32_p, c_int32_p]),
    "mp_profile_enable": (ctypes.c_int, [ctypes.c_int]),
    "mp_profile_reset": (ctypes.c_int, []),
    "mp_profile_read": (ctypes.c_int, [ctypes.POINTER(mp_kernel_profile)]),
    "mp_last_error": (ctypes.c_char_p, []),
    "mp_device_count": (ctypes.c_int, []),
    "mp_lo_spin_us": (ctypes.c_int, []),
    "mp_version": (ctypes.c_char_p, []),
}

_lib = None


def lib():
    """Load the engine library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"madpose_amd: native library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)"
            )
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(code):
    if code == MP_OK:
        return
    msg = lib().mp_last_error().decode(errors="replace")
    if code == MP_EINVAL:
        raise ValueError(msg)
    raise RuntimeError(f"madpose_amd device error: {msg}")
