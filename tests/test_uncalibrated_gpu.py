"""GPU parity of the shared-focal / two-focal paths: the 6-point and 7-point point
solvers (PoseLib relpose_6pt_shared_focal / relpose_7pt + bougnoux + cv::recoverPose,
restated in oracle/src/pt67.cpp -- parity unpinned) and the full
HybridEstimatePoseScaleOffsetSharedFocal / TwoFocal estimators against the oracle."""
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


def _rand_rot(rng):
    R = np.linalg.qr(rng.standard_normal((3, 3)))[0]
    return R * np.linalg.det(R)


def _sample(rng, k, shared, outliers, noise):
    while True:
        R = _rand_rot(rng)
        t = rng.standard_normal(3)
        f0, f1 = rng.uniform(0.5, 3.0, 2)
        if shared:
            f1 = f0
        X = np.c_[rng.uniform(-1, 1, (k, 2)), rng.uniform(2, 6, k)]
        X2 = X @ R.T + t
        if np.all(X2[:, 2] > 0.1):
            break
    p0 = f0 * X[:, :2] / X[:, 2:]
    p1 = f1 * X2[:, :2] / X2[:, 2:]
    if outliers:
        p1[:2] = rng.uniform(-1.5, 1.5, (2, 2))
    p0 = p0 + rng.normal(0, noise, p0.shape)
    return p0, p1, R, t, f0, f1


def _bearings(p):
    h = np.c_[p, np.ones(len(p))]
    return h / np.linalg.norm(h, axis=1, keepdims=True)


@pytest.mark.parametrize("seed", [21, 23, 24, 25])
def test_6pt_shared_focal_matches_oracle_and_ground_truth(seed):
    rng = np.random.default_rng(seed)
    n_trials, set_mismatch, gt_found = 500, 0, 0
    for trial in range(n_trials):
        clean = trial % 2 == 0
        p0, p1, R, t, f0, _ = _sample(rng, 6, True, not clean, 0.0)
        dev = madpose.relpose_6pt_shared_focal(p0, p1)
        orc = oracle.relpose_6pt_shared_focal(_bearings(p0), _bearings(p1))
        if len(dev) != len(orc):
            set_mismatch += 1
            continue
        for m in dev:
            d = min(np.abs(m.R() - o["R"]).max() + np.abs(m.t() - o["t"]).max() + abs(m.focal - o["focal0"])
                    for o in orc)
            if d > 1e-6:
                set_mismatch += 1
                break
        if clean:
            tn = t / np.linalg.norm(t)
            err = min(rot_angle_deg(m.R(), R) + abs(m.focal - f0) + np.abs(m.t() / np.linalg.norm(m.t()) - tn).max()
                      for m in dev) if dev else np.inf
            gt_found += err < 1e-5
    # Device and oracle both take the roots u as the eigenvalues of the companion
    # matrix of the pencil, deflated of its structural zero block (device: eig6.h, a
    # lockstep QR over 64 samples per wave; oracle: la.cpp hqr), then (x, y) from the
    # best-conditioned monomial ratios of the null vector and a polish on the ten
    # equations.  Round 2's DFT + Sturm root stage lost roots on 1-8 of 2000 trials of
    # these seeds (the small coefficients of q lost their digits); those
    # samples are tests/golden/sixpt_hard.json.  Measured now (tools/diag_pt67.py, 2000
    # trials per seed, profiles/r03/six/diag.log): 0 mismatches on all four seeds, so
    # none is tolerated here.
    assert set_mismatch == 0, set_mismatch
    assert gt_found == n_trials // 2, gt_found


def test_7pt_two_focal_matches_oracle_and_ground_truth():
    rng = np.random.default_rng(22)
    n_trials, mismatch, gt_found = 160, 0, 0
    for trial in range(n_trials):
        clean = trial % 2 == 0
        p0, p1, R, t, f0, f1 = _sample(rng, 7, False, not clean, 0.0 if clean else 1e-3)
        dev = madpose.relpose_7pt_two_focal(p0, p1)
        Fs = oracle.relpose_7pt(_bearings(p0), _bearings(p1))
        if len(dev) != len(Fs):
            mismatch += 1
            continue
        for m in dev:
            best = np.inf
            for F in Fs:
                fsq = oracle.bougnoux_focals(F.ravel())
                fa, fb = np.sqrt(np.abs(fsq))
                E = np.diag([fb, fb, 1.0]) @ F @ np.diag([fa, fa, 1.0])
                Ro, to, _ = oracle.recover_pose(E.ravel(), p0, p1)
                best = min(best, np.abs(m.R() - Ro).max() + np.abs(m.t() - to).max() + abs(m.focal0 - fa)
                           + abs(m.focal1 - fb))
            mismatch += best > 1e-6
        if clean:
            err = min(abs(m.focal0 - f0) + abs(m.focal1 - f1) for m in dev)
            gt_found += err < 1e-6
    # 0 of 2000 trials disagree (tools/diag_pt67.py, round 2): the candidate labels of
    # recoverPose follow the canonical SVD signs on both sides
    assert mismatch == 0, mismatch
    assert gt_found == n_trials // 2


def _run_both(p, o, c, variant):
    fn = [madpose.HybridEstimatePoseScaleOffset, madpose.HybridEstimatePoseScaleOffsetSharedFocal,
          madpose.HybridEstimatePoseScaleOffsetTwoFocal][variant]
    pose, st = fn(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["pp0"], p["pp1"], o, c)
    om, ost, oinl = oracle.estimate(variant, p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["pp0"],
                                    p["pp1"], oracle_opts(o), oracle_cfg(c))
    return pose, st, om, ost, oinl


def _assert_parity(pose, st, om, ost, oinl, variant):
    assert st.num_iterations_total == ost.num_iterations_total
    assert st.num_hypotheses == ost.num_hypotheses, (st.num_hypotheses, ost.num_hypotheses)
    assert st.num_iterations_per_solver == list(ost.num_iterations_per_solver)
    assert st.number_lo_iterations == ost.number_lo_iterations
    assert st.best_solver_type == ost.best_solver_type
    for t in range(3):
        assert np.array_equal(np.array(st.inlier_indices[t]), oinl[t]), f"inlier list {t} differs"
    assert rot_angle_deg(pose.R(), om["R"]) < 1e-6
    np.testing.assert_allclose(pose.t(), om["t"], rtol=1e-7, atol=1e-9)
    assert abs(pose.scale - om["scale"]) <= 1e-8 * (1 + abs(om["scale"]))
    if variant == 1:
        assert abs(pose.focal - om["focal0"]) <= 1e-8 * om["focal0"]
    else:
        assert abs(pose.focal0 - om["focal0"]) <= 1e-8 * om["focal0"]
        assert abs(pose.focal1 - om["focal1"]) <= 1e-8 * om["focal1"]
    assert abs(st.best_model_score - ost.best_model_score) <= 1e-9 * abs(ost.best_model_score)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_shared_focal_estimator_parity(seed):
    p = synthetic.make_pair(seed, n=400)
    o, c = synthetic.example_options("shared_focal", iterations=300)
    o.random_seed = seed
    _assert_parity(*_run_both(p, o, c, 1), 1)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_two_focal_estimator_parity(seed):
    p = synthetic.config_pair("two_focal", seed=seed)
    sel = slice(0, 500)
    p = {k: (v[sel] if isinstance(v, np.ndarray) and v.ndim >= 1 and len(v) == 4000 else v) for k, v in p.items()}
    o, c = synthetic.example_options("two_focal", iterations=300)
    o.random_seed = seed
    _assert_parity(*_run_both(p, o, c, 2), 2)


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("solver", [1, 2])
def test_uncalibrated_solver_modes(variant, solver):
    p = synthetic.make_pair(30 + variant, n=300)
    o, c = synthetic.example_options("shared_focal" if variant == 1 else "two_focal", iterations=200)
    c.solver_type = solver
    _assert_parity(*_run_both(p, o, c, variant), variant)


@pytest.mark.parametrize("variant", [1, 2])
def test_uncalibrated_recovers_pose(variant):
    p = synthetic.make_pair(40 + variant, n=1000, noise_px=0.5)
    o, c = synthetic.example_options("shared_focal" if variant == 1 else "two_focal", iterations=1000)
    fn = [None, madpose.HybridEstimatePoseScaleOffsetSharedFocal, madpose.HybridEstimatePoseScaleOffsetTwoFocal]
    pose, st = fn[variant](p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["pp0"], p["pp1"], o, c)
    assert rot_angle_deg(pose.R(), p["R"]) < 1.0
    f_est = [pose.focal] if variant == 1 else [pose.focal0, pose.focal1]
    f_gt = [p["f0"]] if variant == 1 else [p["f0"], p["f1"]]
    for fe, fg in zip(f_est, f_gt):
        assert abs(fe - fg) < 0.05 * fg


def _pt6_roots(impl, p0, p1):
    import ctypes

    from madpose_amd import _lib as L

    ns = p0.shape[0]
    cand = np.zeros((ns, 96))
    ncand = np.zeros(ns, dtype=np.int32)
    dp = lambda a: np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    L.check(L.lib().mp_debug_pt_roots(1, impl, ns, dp(p0), dp(p1), cand.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                      ncand.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 0))
    return cand, ncand


def test_eig_6pt_roots_match_oracle():
    """The estimator's shared-focal root stage (impl 3: the pencil, the deflation of its
    structural zero block and the lockstep QR of the 15 x 15 block, eig6.h) against the
    oracle's deflated eigenproblem (oracle.sixpt_roots) on clean and noisy samples: the
    same positive real roots u to 1e-8, and on clean samples the true f^2 among them
    every time (the round-2 DFT + Sturm stage missed it on about 3 %)."""
    rng = np.random.default_rng(13)
    ns = 1500
    p0 = np.zeros((ns, 6, 2))
    p1 = np.zeros((ns, 6, 2))
    f2 = np.zeros(ns)
    for s in range(ns):
        a, b, _, _, f0, _ = _sample(rng, 6, True, False, 0.0 if s % 2 == 0 else 0.01)
        p0[s], p1[s], f2[s] = a, b, f0 * f0
    cand, ncand = _pt6_roots(3, p0, p1)
    hits, bad = 0, []
    for s in range(ns):
        u = np.sort(cand[s, 27: 27 + ncand[s]])
        o = np.sort(np.asarray(oracle.sixpt_roots(_bearings(p0[s]), _bearings(p1[s]))))
        if len(u) != len(o) or np.any(np.abs(u - o) > 1e-8 * np.maximum(1.0, np.abs(o))):
            bad.append((s, u.tolist(), o.tolist()))
        if s % 2 == 0:
            hits += np.any(np.abs(u - f2[s]) <= 1e-6 * f2[s])
    assert not bad, bad[:3]
    assert hits == (ns + 1) // 2, hits
