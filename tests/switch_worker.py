"""Worker of tests/test_switch_invariance_gpu.py: runs the full-size estimator cases
(one pair at a time, then four pairs in flight through estimate_batch) in a fresh
process -- the engine reads its A/B switches once per process -- and prints every
result field as exact hex floats / integers, one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import madpose  # noqa: E402
from madpose_amd import api, synthetic  # noqa: E402

CASES = [(0, "calibrated", 2, 100000, 0), (1, "shared_focal", 3, 100000, 0), (2, "two_focal", 4, 200000, 0),
         (1, "shared_focal", 3, 100000, 1)]
FN = [madpose.HybridEstimatePoseScaleOffset, madpose.HybridEstimatePoseScaleOffsetSharedFocal,
      madpose.HybridEstimatePoseScaleOffsetTwoFocal]


def record(variant, pose, st):
    vals = list(np.asarray(pose.pose, dtype=np.float64).reshape(-1)) + [pose.scale, pose.offset0, pose.offset1]
    vals += [pose.focal] if variant == 1 else ([pose.focal0, pose.focal1] if variant == 2 else [])
    return {"model": [float(v).hex() for v in vals], "score": float(st.best_model_score).hex(),
            "iters": int(st.num_iterations_total), "hyp": int(st.num_hypotheses),
            "lo": int(st.number_lo_iterations), "inl": [len(x) for x in st.inlier_indices],
            "inl_sum": [int(np.sum(x)) for x in st.inlier_indices]}


def main():
    out = []
    for variant, kind, cfg, iters, seed in CASES:
        p = synthetic.config_pair(cfg, seed=seed)
        o, c = synthetic.throughput_options(kind, iterations=iters)
        cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
        pose, st = FN[variant](p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1, o, c)
        out.append(record(variant, pose, st))
    # several estimators on the device at once (the early continuation's other regime)
    pairs = [synthetic.scannet_pair(s) for s in range(4)]
    o, c = synthetic.example_options("shared_focal", iterations=1000)
    for pose, st in api.estimate_batch(1, pairs, o, c, num_streams=4):
        out.append(record(1, pose, st))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
