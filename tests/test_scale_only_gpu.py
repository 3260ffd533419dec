"""HybridEstimatePoseAndScale (scale-only estimator, src/hybrid_pose_estimator.cpp:37-63,
297-442) and estimate_scale_and_pose (src/solver.cpp:5-33) on the device vs the oracle."""
import numpy as np
import pytest

import madpose
import oracle
from madpose_amd import synthetic
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


def test_estimate_scale_and_pose_matches_oracle():
    rng = np.random.default_rng(4)
    for _ in range(20):
        n = int(rng.integers(3, 40))
        X = rng.normal(size=(n, 3))
        R = np.linalg.qr(rng.normal(size=(3, 3)))[0]
        R *= np.linalg.det(R)
        Y = rng.uniform(0.5, 2) * X @ R.T + rng.normal(size=3) + rng.normal(0, 0.01, (n, 3))
        W = rng.uniform(0.1, 1.0, n)
        dev = madpose.estimate_scale_and_pose(X.T, Y.T, W)
        ref = oracle.estimate_scale_and_pose(X, Y, W)
        assert np.allclose(dev.R(), ref["R"], atol=1e-10)
        assert np.allclose(dev.t(), ref["t"], atol=1e-10)
        assert abs(dev.scale - ref["scale"]) < 1e-10


@pytest.mark.parametrize("seed,solver", [(0, 0), (1, 0), (2, 1), (3, 2)])
def test_scale_only_estimator_parity(seed, solver):
    p = synthetic.make_pair(70 + seed, n=400)
    o, c = synthetic.example_options("calibrated", iterations=300)
    o.random_seed = seed
    c.solver_type = solver
    pose, st = madpose.HybridEstimatePoseAndScale(p["x0"], p["x1"], p["depth0"], p["depth1"], p["K0"], p["K1"], o, c)
    om, ost, oinl = oracle.estimate(3, p["x0"], p["x1"], p["depth0"], p["depth1"], np.zeros(2), p["K0"], p["K1"],
                                    oracle_opts(o), oracle_cfg(c))
    assert isinstance(pose, madpose.PoseAndScale)
    assert st.num_iterations_total == ost.num_iterations_total
    assert st.num_hypotheses == ost.num_hypotheses, (st.num_hypotheses, ost.num_hypotheses)
    assert st.num_iterations_per_solver == list(ost.num_iterations_per_solver)
    assert st.number_lo_iterations == ost.number_lo_iterations
    for t in range(3):
        assert np.array_equal(np.array(st.inlier_indices[t]), oinl[t])
    assert rot_angle_deg(pose.R(), om["R"]) < 1e-6
    np.testing.assert_allclose(pose.t(), om["t"], rtol=1e-7, atol=1e-9)
    assert abs(pose.scale - om["scale"]) <= 1e-8 * (1 + abs(om["scale"]))
    assert abs(st.best_model_score - ost.best_model_score) <= 1e-9 * abs(ost.best_model_score)
