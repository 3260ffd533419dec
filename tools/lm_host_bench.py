"""Host LM timing (the LO's all-inlier fits): one calibrated pair (N = 2000), the
all-inlier problem of every data type started near the ground truth, solved by the
engine's host LM (`lm_refine_batch(..., on_host=True)`, the ctypes call included)
`reps` times; prints microseconds per solve.  Run under MADPOSE_LO_THREADS=1/4/8 or
MADPOSE_LM_ISA=avx2 for the pool / ISA split.  usage: python tools/lm_host_bench.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import madpose
from madpose_amd import synthetic

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
p = synthetic.make_pair(5, n=2000)
o, c = synthetic.example_options("calibrated")
inl = np.flatnonzero(p["inlier_mask"])
rng = np.random.default_rng(0)
ax = rng.standard_normal(3)
ax *= 0.01 / np.linalg.norm(ax)
K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
R = (np.eye(3) + K) @ p["R"]
U, _, Vt = np.linalg.svd(R)
m0 = madpose.PoseScaleOffset(U @ Vt, p["t"] + 0.01 * rng.standard_normal(3), 1.0, 0.0, 0.0)
args = (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["K0"], p["K1"])
for kind in (0, 1):
    probs = [(kind, [inl, inl, inl], m0)]
    madpose.lm_refine_batch(0, *args, o, c, probs, on_host=True)
    t = time.perf_counter()
    for _ in range(reps):
        madpose.lm_refine_batch(0, *args, o, c, probs, on_host=True)
    dt = (time.perf_counter() - t) / reps
    print(f"kind {kind} ({'NonMinimalSolver' if kind else 'LeastSquares'}): {3 * len(inl)} blocks, {1e6 * dt:.1f} us per solve")
