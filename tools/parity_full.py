"""Full-size estimator parity (BASELINE.json configs[1..3]) of the GPU path against the
CPU oracle, one JSON line per case.  Diagnostic driver (the -m gpu tests hold the
asserting versions):  python tools/parity_full.py [cal sf tf] [--seeds 0,1]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import madpose  # noqa: E402
import oracle  # noqa: E402
from madpose_amd import synthetic  # noqa: E402
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg  # noqa: E402

CASES = {"cal": (0, "calibrated", 2, 100000), "sf": (1, "shared_focal", 3, 100000),
         "tf": (2, "two_focal", 4, 200000)}


def compare(variant, p, o, c):
    cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
    fn = [madpose.HybridEstimatePoseScaleOffset, madpose.HybridEstimatePoseScaleOffsetSharedFocal,
          madpose.HybridEstimatePoseScaleOffsetTwoFocal][variant]
    args = (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1)
    t0 = time.perf_counter()
    pose, st = fn(*args, o, c)
    tg = time.perf_counter() - t0
    t0 = time.perf_counter()
    om, ost, oinl = oracle.estimate(variant, *args, oracle_opts(o), oracle_cfg(c))
    to = time.perf_counter() - t0
    same_inl = [bool(np.array_equal(np.array(st.inlier_indices[t]), oinl[t])) for t in range(3)]
    return {"gpu_s": tg, "oracle_s": to, "iterations": [st.num_iterations_total, ost.num_iterations_total],
            "per_solver": [st.num_iterations_per_solver, list(ost.num_iterations_per_solver)],
            "lo": [st.number_lo_iterations, ost.number_lo_iterations],
            "solver_type": [st.best_solver_type, ost.best_solver_type], "inliers_equal": same_inl,
            "inliers": [st.best_num_inliers, ost.best_num_inliers],
            "rot_deg": rot_angle_deg(pose.R(), om["R"]),
            "score_rel": abs(st.best_model_score - ost.best_model_score) / abs(ost.best_model_score),
            "gt_rot_deg": rot_angle_deg(pose.R(), p["R"])}


def main():
    names = [a for a in sys.argv[1:] if a in CASES] or list(CASES)
    seeds = [0]
    for a in sys.argv[1:]:
        if a.startswith("--seeds="):
            seeds = [int(x) for x in a.split("=", 1)[1].split(",")]
    for name in names:
        variant, kind, cfg, iters = CASES[name]
        for seed in seeds:
            p = synthetic.config_pair(cfg, seed=seed)
            o, c = synthetic.throughput_options(kind, iterations=iters)
            r = compare(variant, p, o, c)
            r.update(case=name, seed=seed)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
