"""CPU stand-in for bench.py's engine (tests only): lets the gloo tests drive bench.py's
rank spawning, pair sharding and result gathering without a GPU.  It estimates nothing:
the returned pose is the identity with a unit translation, and the statistics are simple
functions of the pair size, so the gathered records can be checked exactly."""
import numpy as np

from madpose_amd.api import HybridRansacStatistics, PoseScaleOffset


class Engine:
    def __init__(self):
        self.calls = 0

    def estimate(self, variant, args, o, c, device):
        self.calls += 1
        n = len(args[0])
        st = HybridRansacStatistics()
        st.num_iterations_total = o.max_num_iterations
        st.num_hypotheses = 2 * o.max_num_iterations
        st.best_num_inliers = n
        st.best_model_score = float(n)
        st.number_lo_iterations = 1
        st.seconds_lo = 0.0
        return PoseScaleOffset(np.eye(3), np.array([1.0, 0.0, 0.0]), 1.0, 0.0, 0.0), st

    def estimate_batch(self, variant, pairs, o, c, device=None, num_streams=1):
        return [self.estimate(variant, (p["x0"],), o, c, device) for p in pairs]

    def pose_errors(self, T, R, t):
        from madpose_amd import utils

        e = np.array([utils.compute_pose_error(T[k], R[k], t[k]) for k in range(len(T))]).reshape(-1, 2)
        return e[:, 0], e[:, 1]

    def pose_auc(self, errors, thresholds):
        from madpose_amd import utils

        return utils.pose_auc(errors, thresholds)

    def profile_reset(self):
        pass

    def profile_enable(self, on):
        pass

    def profile_read(self):
        keys = ["score_ms", "solve_ms", "hypotheses", "correspondences", "batches", "sweeps", "lm_calls",
                "lm_wall_ms", "sweep_wall_ms", "iterations", "sample_wall_ms", "wait_wall_ms", "run_wall_ms",
                "lm_blocks", "lm_big_calls", "lm_big_wall_ms", "model_trips", "model_trips_full", "accepted", "scored"]
        return {k: 1.0 for k in keys}
