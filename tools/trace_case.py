"""Debug helper: run one estimator configuration through the product and the oracle
with best-model / LO tracing enabled (stderr).  Usage on a GPU box:
    python tools/trace_case.py <variant> <seed> <n> <iterations> [solver]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MADPOSE_TRACE"] = "1"
os.environ["ORACLE_TRACE"] = "1"

import madpose  # noqa: E402
import oracle  # noqa: E402
from madpose_amd import synthetic  # noqa: E402
from tests.helpers import oracle_cfg, oracle_opts  # noqa: E402

variant, seed, n, iters = (int(a) for a in sys.argv[1:5])
solver = int(sys.argv[5]) if len(sys.argv) > 5 else 0
p = synthetic.make_pair(seed, n=n)
kind = ["calibrated", "shared_focal", "two_focal"][variant]
o, c = synthetic.example_options(kind, iterations=iters)
c.solver_type = solver
cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
fn = [madpose.HybridEstimatePoseScaleOffset, madpose.HybridEstimatePoseScaleOffsetSharedFocal,
      madpose.HybridEstimatePoseScaleOffsetTwoFocal][variant]
pose, st = fn(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1, o, c)
sys.stderr.flush()
print("engine:", st, flush=True)
om, ost, _ = oracle.estimate(variant, p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1,
                             oracle_opts(o), oracle_cfg(c))
sys.stderr.flush()
print("oracle: iterations", ost.num_iterations_total, "lo", ost.number_lo_iterations, "score", ost.best_model_score)
