"""The calibrated MD minimal solver on 16-lane groups (md_solve_group_kernel, the default)
against the one-lane-per-sample kernel (MADPOSE_MD_LANE=1): both evaluate the same
md_setup_* / md_root_* restatement of src/solver.cpp:35-480, so whole estimator runs
must agree -- same iteration counts, LO counts, inlier lists, and the same model up to
rounding.  (The shared- and two-focal MD solvers run md_exact_kernel whatever the
switch, tests/test_md_exact_gpu.py.)  The lane run happens in a child process (the switch is read once per
process); it runs after this process's own GPU work has finished, one at a time."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import madpose
from madpose_amd import synthetic

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [(0, 5, 0), (0, 6, 2), (0, 7, 0)]  # (variant, seed, solver_type)

_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import madpose
from madpose_amd import synthetic
from tests.test_md_group_gpu import run_case, CASES
print(json.dumps([run_case(*c) for c in CASES]))
"""


def run_case(variant, seed, solver_type):
    kind = ["calibrated", "shared_focal", "two_focal"][variant]
    p = synthetic.make_pair(seed, n=400)
    o, c = synthetic.example_options(kind, iterations=400)
    o.random_seed = seed
    c.solver_type = solver_type
    if variant == 0:
        pose, st = madpose.HybridEstimatePoseScaleOffset(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"],
                                                         p["K0"], p["K1"], o, c)
        focals = [1.0, 1.0]
    else:
        fn = madpose.HybridEstimatePoseScaleOffsetSharedFocal if variant == 1 else \
            madpose.HybridEstimatePoseScaleOffsetTwoFocal
        pose, st = fn(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["pp0"], p["pp1"], o, c)
        focals = [pose.focal, pose.focal] if variant == 1 else [pose.focal0, pose.focal1]
    return {
        "R": np.asarray(pose.R()).tolist(), "t": np.asarray(pose.t()).tolist(), "scale": pose.scale,
        "offset0": pose.offset0, "offset1": pose.offset1, "focals": focals,
        "iters": st.num_iterations_total, "per_solver": list(st.num_iterations_per_solver),
        "lo": st.number_lo_iterations, "best_solver": st.best_solver_type, "score": st.best_model_score,
        "inliers": [list(map(int, st.inlier_indices[t])) for t in range(3)],
    }


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


def test_group_md_kernel_matches_lane_kernel():
    assert os.environ.get("MADPOSE_MD_LANE") is None
    group = [run_case(*c) for c in CASES]
    env = dict(os.environ, MADPOSE_MD_LANE="1")
    out = subprocess.run([sys.executable, "-c", _SCRIPT, ROOT], env=env, cwd=ROOT, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lane = json.loads(out.stdout.strip().splitlines()[-1])
    for case, g, l in zip(CASES, group, lane):
        for k in ("iters", "per_solver", "lo", "best_solver", "inliers"):
            assert g[k] == l[k], (case, k)
        np.testing.assert_allclose(g["R"], l["R"], rtol=0, atol=1e-9, err_msg=str(case))
        np.testing.assert_allclose(g["t"], l["t"], rtol=1e-9, atol=1e-12, err_msg=str(case))
        for k in ("scale", "offset0", "offset1", "score"):
            assert abs(g[k] - l[k]) <= 1e-9 * (1 + abs(l[k])), (case, k)
        np.testing.assert_allclose(g["focals"], l["focals"], rtol=1e-9, err_msg=str(case))
