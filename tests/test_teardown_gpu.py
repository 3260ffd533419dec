"""Pooled device contexts across pairs of growing size, then a plain process exit.

VERDICT r05 item 1: a rocprofv3 run of the ScanNet stand-in (8 pairs in flight) died
with SIGSEGV in Run::launch_batch on a sampler thread (gpurun_out/r5q/prof_sn.log).  The
engine's answer ("Speculation threads and teardown"): every draw into and
upload from a host sample slot is range-checked, and the pooled contexts' sampler and
LO-worker threads are joined at library teardown.  This test drives the paths the
record points at -- estimate_batch with several pairs in flight, pairs whose N grows so
every pooled context reallocates its buffers (DeviceCtx::ensure), the post-LO
speculation launched from sampler threads -- in a fresh process that then exits without
any cleanup of its own; it must return 0."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r"""
import numpy as np
import madpose
from madpose_amd import api, synthetic
o, c = synthetic.example_options("shared_focal", iterations=1000)
sizes = [300, 800, 1600, 3200, 6400]
total = 0
for rep in range(2):
    pairs = [synthetic.make_pair(100 * rep + k, n=n) for k, n in enumerate(sizes)]
    for pose, st in api.estimate_batch(1, pairs, o, c, num_streams=4):
        assert st.num_iterations_total > 0
        total += 1
# one estimator alone, N growing again (the pooled context of the batch above grows)
oc, cc = synthetic.example_options("calibrated", iterations=3000)
for k, n in enumerate([500, 5000, 9000]):
    p = synthetic.make_pair(1000 + k, n=n)
    pose, st = madpose.HybridEstimatePoseScaleOffset(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"],
                                                     p["K0"], p["K1"], oc, cc)
    assert st.num_iterations_total > 0
    total += 1
print("DONE", total, flush=True)
"""


def test_growing_pairs_then_exit():
    env = {k: v for k, v in os.environ.items() if not k.startswith("MADPOSE_")}
    env["MADPOSE_SEGV_MAPS"] = "1"
    env.setdefault("GPU_MAX_HW_QUEUES", "16")
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stderr[-4000:])
    assert "DONE 13" in r.stdout, r.stdout[-2000:]
