"""Full-size estimator parity at BASELINE.json's own configurations:
configs[1] calibrated N = 2000 / 100k iterations, configs[2] shared-focal N = 2000 /
100k, configs[3] two-focal N = 4000 / 200k (min = max = per-solver cap, so every run
goes the full length).  GPU path vs the CPU oracle on the same seeded pair: identical
iteration counts (total and per solver), LO count, best solver type and all three
inlier index lists; rotation within 1e-6 deg, the rest within 1e-8 relative, score
within 1e-9 relative.  The oracle needs ~10 s (cal, sf) and ~45 s (tf) per run."""
import numpy as np
import pytest

import madpose
import oracle
from madpose_amd import synthetic
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg

pytestmark = pytest.mark.gpu

CASES = {"cal": (0, "calibrated", 2, 100000), "sf": (1, "shared_focal", 3, 100000),
         "tf": (2, "two_focal", 4, 200000)}


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


@pytest.mark.parametrize("name,seed", [("cal", 0), ("cal", 1), ("sf", 0), ("sf", 1), ("tf", 0)])
def test_full_size_config_parity(name, seed):
    variant, kind, cfg, iters = CASES[name]
    p = synthetic.config_pair(cfg, seed=seed)
    o, c = synthetic.throughput_options(kind, iterations=iters)
    cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
    args = (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1)
    fn = [madpose.HybridEstimatePoseScaleOffset, madpose.HybridEstimatePoseScaleOffsetSharedFocal,
          madpose.HybridEstimatePoseScaleOffsetTwoFocal][variant]
    pose, st = fn(*args, o, c)
    om, ost, oinl = oracle.estimate(variant, *args, oracle_opts(o), oracle_cfg(c))
    assert st.num_iterations_total == ost.num_iterations_total == iters
    assert st.num_hypotheses == ost.num_hypotheses, (st.num_hypotheses, ost.num_hypotheses)  # the headline's unit
    assert st.num_iterations_per_solver == list(ost.num_iterations_per_solver)
    assert st.number_lo_iterations == ost.number_lo_iterations
    assert st.best_solver_type == ost.best_solver_type
    for t in range(3):
        assert np.array_equal(np.array(st.inlier_indices[t]), oinl[t]), f"inlier list {t} differs"
    assert rot_angle_deg(pose.R(), om["R"]) < 1e-6
    np.testing.assert_allclose(pose.t(), om["t"], rtol=1e-8, atol=1e-10)
    for k in ("scale", "offset0", "offset1"):
        assert abs(getattr(pose, k) - om[k]) <= 1e-8 * (1 + abs(om[k])), k
    if variant == 1:
        assert abs(pose.focal - om["focal0"]) <= 1e-8 * om["focal0"]
    elif variant == 2:
        assert abs(pose.focal0 - om["focal0"]) <= 1e-8 * om["focal0"]
        assert abs(pose.focal1 - om["focal1"]) <= 1e-8 * om["focal1"]
    assert abs(st.best_model_score - ost.best_model_score) <= 1e-9 * abs(ost.best_model_score)
    assert rot_angle_deg(pose.R(), p["R"]) < 0.5  # and it found the synthetic pose
