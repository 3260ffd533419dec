"""C ABI / Python surface checks that need no GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import madpose
import madpose_amd
from madpose_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    names = []
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h"):
            txt = open(os.path.join(ROOT, "include", fn)).read()
            names += re.findall(r"^(?:int|const char \*|int64_t|void)\s*\*?\s*(mp_\w+)\s*\(", txt, re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(L.LIB_PATH)
    names = _declared_symbols()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n


def test_python_surface_matches_reference_bindings():
    # src/bindings.cpp:34-175
    for name in ["HybridLORansacOptions", "EstimatorConfig", "PoseScaleOffset", "PoseScaleOffsetSharedFocal",
                 "PoseScaleOffsetTwoFocal", "PoseAndScale", "HybridRansacStatistics", "RansacOptions",
                 "LORansacOptions", "RansacStats", "HybridEstimatePoseScaleOffset",
                 "HybridEstimatePoseScaleOffsetSharedFocal", "HybridEstimatePoseScaleOffsetTwoFocal",
                 "HybridEstimatePoseAndScale", "estimate_scale_and_pose", "solve_scale_and_shift", "solve_scale_and_shift_shared_focal",
                 "solve_scale_and_shift_two_focal", "solve_scale_shift_pose", "solve_scale_shift_pose_shared_focal",
                 "solve_scale_shift_pose_two_focal"]:
        assert hasattr(madpose, name), name
    o = madpose.HybridLORansacOptions()
    assert (o.min_num_iterations, o.max_num_iterations, o.lo_starting_iterations, o.num_lo_steps) == (100, 10000, 50, 10)
    c = madpose.EstimatorConfig()
    assert c.min_depth_constraint and c.use_shift and c.ceres_max_num_iterations == 25
    c2 = madpose.EstimatorConfig(solver=2, score=1, LO=0)
    assert (c2.solver_type, c2.score_type, c2.LO_type) == (2, 1, 0)
    p = madpose.PoseScaleOffsetTwoFocal(np.eye(3), np.array([1.0, 2, 3]), 2.0, 0.1, 0.2, 500.0, 600.0)
    assert np.allclose(p.t(), [1, 2, 3]) and p.focal1 == 600.0 and np.allclose(p.R(), np.eye(3))
    p2 = madpose.PoseScaleOffset(np.hstack([np.eye(3), np.ones((3, 1))]), 1.5, 0.0, 0.0)
    assert p2.scale == 1.5 and np.allclose(p2.t(), 1.0)


def test_input_validation_raises_before_device():
    from madpose_amd import synthetic

    o, c = synthetic.example_options()
    with pytest.raises(ValueError):
        madpose.HybridEstimatePoseScaleOffset(np.zeros((5, 2)), np.zeros((4, 2)), np.ones(5), np.ones(5), [0, 0],
                                              np.eye(3), np.eye(3), o, c)
    bad = madpose.HybridLORansacOptions()
    with pytest.raises(ValueError):
        madpose.HybridEstimatePoseScaleOffset(np.zeros((5, 2)), np.zeros((5, 2)), np.ones(5), np.ones(5), [0, 0],
                                              np.eye(3), np.eye(3), bad, c)


@pytest.mark.skipif(L.lib().mp_device_count() > 0, reason="checks the no-device behaviour")
def test_no_device_fails_loudly():
    """There is no CPU fallback: without a HIP device the estimator raises."""
    from madpose_amd import synthetic

    p = synthetic.make_pair(0, n=50)
    o, c = synthetic.example_options(iterations=100)
    with pytest.raises(RuntimeError):
        madpose.HybridEstimatePoseScaleOffset(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["K0"],
                                              p["K1"], o, c)
