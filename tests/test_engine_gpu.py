"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the
reference's golden vectors.  Run on an MI355X: pytest -m gpu."""
import os

import numpy as np
import pytest

import madpose
import oracle
from madpose_amd import synthetic
from madpose_amd import _lib as L
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg, solution_sets_match

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


# ---------------------------------------------------------------------------
# minimal solvers
@pytest.mark.parametrize("variant,name", [(0, "cal"), (1, "sf"), (2, "tf")])
def test_md_solver_matches_reference_goldens(variant, name):
    """Device MD solver vs the reference prototypes (solver_py, same templates as
    src/solver.cpp).  Same root count on every instance; values within 1e-6
    relative (the goldens themselves are LU-based: see DESIGN.md)."""
    g = np.load(os.path.join(GOLDEN, "md_solvers.npz"))
    fn = [madpose.solve_scale_and_shift, madpose.solve_scale_and_shift_shared_focal,
          madpose.solve_scale_and_shift_two_focal][variant]
    worst = 0.0
    for i in range(len(g[f"{name}_x"])):
        ref = g[f"{name}_sols"][i, : g[f"{name}_nsols"][i]]
        ref = ref[np.all(np.isfinite(ref), axis=1)]  # a2 = sqrt(<0) roots never survive the pose stage
        mine = np.array(fn(g[f"{name}_x"][i], g[f"{name}_y"][i], g[f"{name}_dx"][i], g[f"{name}_dy"][i]))
        ok, err = solution_sets_match(ref, mine.reshape(-1, ref.shape[1]) if mine.size else mine.reshape(0, ref.shape[1]), 1e-6)
        assert ok, (name, i, ref, mine, err)
        worst = max(worst, err)
    assert worst < 1e-6


@pytest.mark.parametrize("variant,name", [(0, "cal"), (1, "sf"), (2, "tf")])
def test_md_pose_matches_oracle(variant, name):
    g = np.load(os.path.join(GOLDEN, "md_solvers.npz"))
    fn = [madpose.solve_scale_shift_pose, madpose.solve_scale_shift_pose_shared_focal,
          madpose.solve_scale_shift_pose_two_focal][variant]
    for i in range(0, len(g[f"{name}_x"]), 3):
        x, y, dx, dy = g[f"{name}_x"][i], g[f"{name}_y"][i], g[f"{name}_dx"][i], g[f"{name}_dy"][i]
        mine = fn(x, y, dx, dy)
        ref = oracle.md_pose(variant, x.T, y.T, dx, dy)
        assert len(mine) == len(ref), i
        for p in mine:
            j = int(np.argmin([abs(r["offset0"] - p.offset0) for r in ref]))
            r = ref[j]
            assert rot_angle_deg(p.R(), r["R"]) < 1e-6
            assert np.allclose(p.t(), r["t"], rtol=1e-7, atol=1e-7)
            assert abs(p.scale - r["scale"]) <= 1e-7 * (1 + abs(r["scale"]))


@pytest.mark.parametrize("variant,name", [(0, "cal"), (1, "sf"), (2, "tf")])
def test_md_pose_matches_reference_find_transform(variant, name):
    """Pose stage of the MD solvers pinned by the reference itself: md_pose.npz holds,
    for every reference solution that passes the positivity filter of
    src/solver.cpp:503-504, the pose from the reference's find_transform
    (solver_py/scale_and_shift*.py:120-129 / 297 / 356).  Same count per instance,
    rotation within 1e-6 deg, the rest within 1e-6 relative."""
    g = np.load(os.path.join(GOLDEN, "md_solvers.npz"))
    gp = np.load(os.path.join(GOLDEN, "md_pose.npz"))
    fn = [madpose.solve_scale_shift_pose, madpose.solve_scale_shift_pose_shared_focal,
          madpose.solve_scale_shift_pose_two_focal][variant]
    checked = 0
    for i in range(len(g[f"{name}_x"])):
        x, y, dx, dy = g[f"{name}_x"][i], g[f"{name}_y"][i], g[f"{name}_dx"][i], g[f"{name}_dy"][i]
        mine = fn(x, y, dx, dy)
        k = int(gp[f"{name}_npose"][i])
        ref = gp[f"{name}_pose"][i, :k]
        # noisy instances: the reference's LAPACK roots themselves carry ~1e-7 relative
        # error on the worst-conditioned two-focal systems, which the pose inherits
        tol = 1e-4 if g[f"{name}_noise"][i] > 0 else 1e-6
        assert len(mine) == k, (i, len(mine), k)
        for p in mine:
            j = int(np.argmin(np.abs(ref[:, 13] - p.offset0)))
            r = ref[j]
            assert rot_angle_deg(p.R(), r[:9].reshape(3, 3)) < tol, i
            np.testing.assert_allclose(p.t(), r[9:12], rtol=tol, atol=1e-8)
            assert abs(p.scale - r[12]) <= tol * (1 + abs(r[12]))
            assert abs(p.offset0 - r[13]) <= tol * (1 + abs(r[13]))
            assert abs(p.offset1 - r[14]) <= tol * (1 + abs(r[14]))
            if variant == 1:
                assert abs(p.focal - r[15]) <= tol * r[15]
            elif variant == 2:
                assert abs(p.focal0 - r[15]) <= tol * r[15] and abs(p.focal1 - r[16]) <= tol * r[16]
            checked += 1
    assert checked > 200


def test_bougnoux_matches_reference_numpy():
    """Device bougnoux_sq (the two-focal 7pt tail's code) against the reference's
    bougnoux_numpy outputs in utils.npz (madpose/utils.py:25-56).  The goldens carry
    principal points p1, p2; the C++ form has them at the origin, so F is moved to
    centred coordinates first: F' = T1^T F T0 with T = [[1,0,px],[0,1,py],[0,0,1]]."""
    u = np.load(os.path.join(GOLDEN, "utils.npz"))
    Fc = []
    for F, pp in zip(u["bg_F"], u["bg_pp"]):
        T0 = np.array([[1, 0, pp[0]], [0, 1, pp[1]], [0, 0, 1.0]])
        T1 = np.array([[1, 0, pp[2]], [0, 1, pp[3]], [0, 0, 1.0]])
        Fc.append(T1.T @ F @ T0)
    got = madpose.bougnoux_focals_batch(np.array(Fc))
    np.testing.assert_allclose(got, u["bg_out"], rtol=1e-8)


def _rand_rot(rng):
    R = np.linalg.qr(rng.standard_normal((3, 3)))[0]
    return R * np.linalg.det(R)


def test_5pt_matches_oracle_and_ground_truth():
    """The standalone 5pt solver (the estimator's root stage + motion_from_essential)
    equals the oracle's restatement of PoseLib relpose_5pt pose for pose (1e-9), and finds
    the ground truth on noise-free samples -- to 1e-6 on nearly all of them: PoseLib's
    Newton stage stops at |f(z)| < 1e-10 on the monic degree-10 polynomial, which leaves
    roots of a close pair less accurate (the oracle alike; 99.2 % of 4000 samples at 1e-6,
    99.8 % at 1e-4)."""
    rng = np.random.default_rng(3)
    checked = near = 0
    for trial in range(120):
        R = _rand_rot(rng)
        t = rng.standard_normal(3)
        X = np.c_[rng.uniform(-1, 1, (5, 2)), rng.uniform(2, 6, 5)]
        X2 = X @ R.T + t
        if np.any(X2[:, 2] < 0.1):
            continue
        b1 = X / np.linalg.norm(X, axis=1, keepdims=True)
        b2 = X2 / np.linalg.norm(X2, axis=1, keepdims=True)
        dev = madpose.relpose_5pt(b1, b2)
        orc = oracle.relpose_5pt(b1, b2)
        assert len(dev) == len(orc)
        tn = t / np.linalg.norm(t)
        gt_err = min(rot_angle_deg(p.R(), R) + np.abs(p.t() / np.linalg.norm(p.t()) - tn).max() for p in dev)
        assert gt_err < 0.1
        near += gt_err < 1e-6
        for p in dev:
            d = min(np.abs(p.R() - o["R"]).max() + np.abs(p.t() - o["t"]).max() for o in orc)
            assert d < 1e-9
        checked += 1
    assert checked > 80 and near >= checked - 2, (checked, near)


# ---------------------------------------------------------------------------
# scoring sweep
def _models_near_gt(p, rng, k, variant):
    models = []
    for _ in range(k):
        dR = _rand_rot(rng) if rng.random() < 0.2 else np.eye(3)
        ang = rng.normal(0, 0.02, 3)
        Kx = np.array([[0, -ang[2], ang[1]], [ang[2], 0, -ang[0]], [-ang[1], ang[0], 0]])
        Rn = dR @ (np.eye(3) + Kx) @ p["R"]
        U, _, Vt = np.linalg.svd(Rn)
        Rn = U @ Vt
        t = p["t"] + rng.normal(0, 0.05, 3)
        scale, o0, o1 = rng.uniform(0.5, 2), rng.normal(0, 0.2), rng.normal(0, 0.2)
        if variant == 0:
            models.append(madpose.PoseScaleOffset(Rn, t, scale, o0, o1))
        elif variant == 1:
            models.append(madpose.PoseScaleOffsetSharedFocal(Rn, t, scale, o0, o1, rng.uniform(0.8, 1.5)))
        else:
            models.append(madpose.PoseScaleOffsetTwoFocal(Rn, t, scale, o0, o1, rng.uniform(0.8, 1.5),
                                                          rng.uniform(0.8, 1.5)))
    return models


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("score_type", [0, 1, 2])
def test_score_sweep_matches_oracle(variant, score_type):
    rng = np.random.default_rng(10 + variant)
    p = synthetic.make_pair(100 + variant, n=700)
    o, c = synthetic.example_options("two_focal" if variant == 2 else "calibrated")
    c.score_type = score_type
    cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
    models = _models_near_gt(p, rng, 12, variant)
    sc, err = madpose.score_models(variant, p["x0"], p["x1"], p["depth0"], p["depth1"], cam0, cam1, o, c, models,
                                   with_errors=True)
    omods = [madpose_amd_model_to_oracle(m, variant) for m in models]
    osc, oerr, _ = oracle.score_models(variant, p["x0"], p["x1"], p["depth0"], p["depth1"], cam0, cam1,
                                       oracle_opts(o), oracle_cfg(c), omods)
    np.testing.assert_allclose(sc, osc, rtol=1e-10)
    big = np.finfo(np.float64).max
    assert np.array_equal(err == big, oerr == big)
    fin = err < big
    np.testing.assert_allclose(err[fin], oerr[fin], rtol=1e-9, atol=1e-12)


def madpose_amd_model_to_oracle(m, variant):
    om = oracle.OrModel()
    om.R[:] = m.R().ravel().tolist()
    om.t[:] = m.t().tolist()
    om.scale, om.offset0, om.offset1 = m.scale, m.offset0, m.offset1
    if variant == 1:
        om.focal0 = om.focal1 = m.focal
    elif variant == 2:
        om.focal0, om.focal1 = m.focal0, m.focal1
    else:
        om.focal0 = om.focal1 = 1.0
    return om


# ---------------------------------------------------------------------------
# full estimator parity
def _run_both(p, o, c, variant=0):
    cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
    fn = [madpose.HybridEstimatePoseScaleOffset, madpose.HybridEstimatePoseScaleOffsetSharedFocal,
          madpose.HybridEstimatePoseScaleOffsetTwoFocal][variant]
    pose, st = fn(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1, o, c)
    om, ost, oinl = oracle.estimate(variant, p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1,
                                    oracle_opts(o), oracle_cfg(c))
    return pose, st, om, ost, oinl


def _assert_parity(pose, st, om, ost, oinl):
    assert st.num_iterations_total == ost.num_iterations_total
    # the headline's unit: models scored by the minimal-sample iterations the estimator
    # consumed (src/hybrid_ransac.h:120-123 GetBestEstimatedModelId over num_models)
    assert st.num_hypotheses == ost.num_hypotheses, (st.num_hypotheses, ost.num_hypotheses)
    assert st.num_iterations_per_solver == list(ost.num_iterations_per_solver)
    assert st.number_lo_iterations == ost.number_lo_iterations
    assert st.best_solver_type == ost.best_solver_type
    for t in range(3):
        assert np.array_equal(np.array(st.inlier_indices[t]), oinl[t]), f"inlier list {t} differs"
    assert rot_angle_deg(pose.R(), om["R"]) < 1e-6
    np.testing.assert_allclose(pose.t(), om["t"], rtol=1e-7, atol=1e-9)
    assert abs(pose.scale - om["scale"]) <= 1e-8 * (1 + abs(om["scale"]))
    assert abs(pose.offset0 - om["offset0"]) <= 1e-8 * (1 + abs(om["offset0"]))
    assert abs(pose.offset1 - om["offset1"]) <= 1e-8 * (1 + abs(om["offset1"]))
    assert abs(st.best_model_score - ost.best_model_score) <= 1e-9 * abs(ost.best_model_score)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_calibrated_estimator_parity(seed):
    p = synthetic.make_pair(seed, n=400)
    o, c = synthetic.example_options("calibrated", iterations=400)
    o.random_seed = seed
    _assert_parity(*_run_both(p, o, c, 0))


@pytest.mark.parametrize("variant", [0, 1])
def test_large_pair_parity(variant):
    # N = 9000: the LO sweeps span 36 workgroups (one completion flag each) and the
    # batches carry every kernel at a larger size than the other parity cases
    p = synthetic.make_pair(11 + variant, n=9000)
    o, c = synthetic.example_options("calibrated" if variant == 0 else "shared_focal", iterations=150)
    _assert_parity(*_run_both(p, o, c, variant))


@pytest.mark.parametrize("solver,score,lo", [(2, 0, 0), (1, 0, 0), (0, 1, 0), (0, 2, 2), (0, 0, 1)])
def test_calibrated_estimator_config_modes(solver, score, lo):
    p = synthetic.make_pair(7, n=300)
    o, c = synthetic.example_options("calibrated", iterations=300)
    c = madpose.EstimatorConfig(solver, score, lo)
    _assert_parity(*_run_both(p, o, c, 0))


def test_calibrated_no_shift_parity():
    p = synthetic.make_pair(8, n=300)
    o, c = synthetic.example_options("calibrated", iterations=300)
    c.use_shift = False
    _assert_parity(*_run_both(p, o, c, 0))


def test_batch_size_invariance(monkeypatch):
    """The speculative batching must not change any result (rollback correctness)."""
    p = synthetic.make_pair(11, n=600)
    o, c = synthetic.example_options("calibrated", iterations=3000, min_iterations=3000)
    o.max_num_iterations_per_solver = 3000
    outs = []
    for mb in ["8", "37", "8192"]:
        monkeypatch.setenv("MADPOSE_MAX_BATCH", mb)
        monkeypatch.setenv("MADPOSE_MIN_BATCH", mb)
        outs.append(madpose.HybridEstimatePoseScaleOffset(p["x0"], p["x1"], p["depth0"], p["depth1"],
                                                          p["min_depth"], p["K0"], p["K1"], o, c))
    (p0, s0) = outs[0]
    for (pk, sk) in outs[1:]:
        assert np.array_equal(p0.pose, pk.pose)
        assert s0.inlier_indices == sk.inlier_indices
        assert s0.num_iterations_total == sk.num_iterations_total
        assert s0.number_lo_iterations == sk.number_lo_iterations
        assert s0.num_hypotheses == sk.num_hypotheses
        assert s0.best_model_score == sk.best_model_score


def test_full_size_properties():
    """Config 2 size (N = 2000) with a reduced iteration budget: the returned inlier
    sets must equal the thresholded device errors of the returned model, and the
    reported score must equal a fresh sweep of that model."""
    p = synthetic.config_pair("calibrated", seed=0)
    o, c = synthetic.throughput_options("calibrated", iterations=5000)
    pose, st = madpose.HybridEstimatePoseScaleOffset(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"],
                                                     p["K0"], p["K1"], o, c)
    assert st.num_iterations_total == 5000
    sc, err = madpose.score_models(0, p["x0"], p["x1"], p["depth0"], p["depth1"], p["K0"], p["K1"], o, c, [pose],
                                   with_errors=True)
    thr = [o.squared_inlier_thresholds[0]] * 2 + [o.squared_inlier_thresholds[1]]
    for t in range(3):
        assert np.array_equal(np.flatnonzero(err[0, t] < thr[t]), np.array(st.inlier_indices[t]))
    assert abs(sc[0] - st.best_model_score) <= 1e-9 * sc[0]
    assert rot_angle_deg(pose.R(), p["R"]) < 1.0
    assert st.num_hypotheses > 1000


def test_example_pair_runs():
    ex = np.load(os.path.join(GOLDEN, "example_pairs.npz"))
    o, c = synthetic.example_options("calibrated", iterations=1000)
    pose, st = madpose.HybridEstimatePoseScaleOffset(ex["eth3d_m0"], ex["eth3d_m1"], ex["eth3d_depth0"],
                                                     ex["eth3d_depth1"], ex["eth3d_mindepth"], ex["eth3d_K0"],
                                                     ex["eth3d_K1"], o, c)
    err_t, err_R = madpose.utils.compute_pose_error(ex["eth3d_T"], pose.R(), pose.t())
    assert err_R < 10.0
    om, ost, oinl = oracle.estimate(0, ex["eth3d_m0"], ex["eth3d_m1"], ex["eth3d_depth0"], ex["eth3d_depth1"],
                                    ex["eth3d_mindepth"], ex["eth3d_K0"], ex["eth3d_K1"], oracle_opts(o),
                                    oracle_cfg(c))
    _assert_parity(pose, st, om, ost, oinl)


def test_two_focal_example_pair_parity():
    """The reference's two-focal example (examples/two_focal.py:20-100) on its own
    2_2d3ds pair (782 MASt3R matches, DepthAnything priors looked up by the reference's
    get_depths): GPU estimator against the oracle, plus the focal lengths."""
    ex = np.load(os.path.join(GOLDEN, "example_pairs.npz"))
    o, c = synthetic.example_options("two_focal", iterations=1000)
    pp0 = (ex["2d3ds_img0_shape"][::-1].astype(np.float64) - 1) / 2
    pp1 = (ex["2d3ds_img1_shape"][::-1].astype(np.float64) - 1) / 2
    args = (ex["2d3ds_m0"], ex["2d3ds_m1"], ex["2d3ds_depth0"], ex["2d3ds_depth1"], ex["2d3ds_mindepth"], pp0, pp1)
    pose, st = madpose.HybridEstimatePoseScaleOffsetTwoFocal(*args, o, c)
    om, ost, oinl = oracle.estimate(2, *args, oracle_opts(o), oracle_cfg(c))
    _assert_parity(pose, st, om, ost, oinl)
    assert abs(pose.focal0 - om["focal0"]) <= 1e-8 * om["focal0"]
    assert abs(pose.focal1 - om["focal1"]) <= 1e-8 * om["focal1"]
    K0, K1 = ex["2d3ds_K0"], ex["2d3ds_K1"]
    err_f = max(abs(pose.focal0 - K0[0, 0]) / K0[0, 0], abs(pose.focal1 - K1[0, 0]) / K1[0, 0])
    err_t, err_R = madpose.utils.compute_pose_error(ex["2d3ds_T"], pose.R(), pose.t())
    assert err_R < 10.0 and err_f < 0.5, (err_R, err_t, err_f)


def test_nonzero_device_matches_device_zero():
    """estimate(device=1) gives the same results as device 0 (every HIP call of the
    engine, including the sampler thread's post-LO launches, runs on the estimator's
    device).  Needs two visible GPUs."""
    if madpose.device_count() < 2:
        pytest.skip("one visible GPU")
    p = synthetic.make_pair(5, n=800)
    o, c = synthetic.example_options("calibrated", iterations=2000, min_iterations=2000)
    outs = [madpose.HybridEstimatePoseScaleOffset(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"],
                                                  p["K0"], p["K1"], o, c, device=d) for d in (0, 1)]
    (p0, s0), (p1, s1) = outs
    assert np.array_equal(p0.pose, p1.pose) and s0.inlier_indices == s1.inlier_indices
    assert s0.num_iterations_total == s1.num_iterations_total and s0.best_model_score == s1.best_model_score


def test_invalid_inputs_raise():
    with pytest.raises(ValueError):
        madpose.HybridEstimatePoseScaleOffset(np.zeros((5, 2)), np.zeros((4, 2)), np.ones(5), np.ones(5), [0, 0],
                                              np.eye(3), np.eye(3), synthetic.example_options()[0])


def test_too_few_points_returns_default_model():
    o, c = synthetic.example_options("calibrated", iterations=100)
    pose, st = madpose.HybridEstimatePoseScaleOffset(np.zeros((2, 2)), np.zeros((2, 2)), np.ones(2), np.ones(2),
                                                     [0, 0], np.eye(3), np.eye(3), o, c)
    assert st.num_iterations_total == 0 and st.best_num_inliers == 0
    assert np.all(pose.pose == 0) and pose.scale == 1.0


def _pt5_roots(impl, p0, p1):
    import ctypes
    ns = p0.shape[0]
    cand = np.zeros((ns, 96))
    ncand = np.zeros(ns, dtype=np.int32)
    dp = lambda a: np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    L.check(L.lib().mp_debug_pt5_roots(impl, ns, dp(p0), dp(p1), cand.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                       ncand.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 0))
    return cand, ncand


def _five_point_samples(rng, ns, noise_free):
    p0 = np.zeros((ns, 5, 2))
    p1 = np.zeros((ns, 5, 2))
    Es = []
    for s in range(ns):
        R = _rand_rot(rng)
        t = rng.normal(size=3)
        t /= np.linalg.norm(t)
        X = np.c_[rng.uniform(-1, 1, (5, 2)), rng.uniform(2, 6, 5)]
        Y = X @ R.T + t
        p0[s] = X[:, :2] / X[:, 2:]
        p1[s] = Y[:, :2] / Y[:, 2:]
        if not noise_free:
            p1[s] += rng.normal(scale=0.05, size=(5, 2))
        tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
        E = tx @ R
        Es.append(E / np.linalg.norm(E))
    return p0, p1, Es


def test_group_5pt_root_stage_finds_ground_truth():
    """The estimator's 5-point root stage (one 16-lane group per sample): on noise-free
    samples the ground-truth essential matrix is among its candidates (99 % at 1e-6:
    PoseLib's Newton stage stops at |f| < 1e-10 on the monic polynomial, so close root
    pairs come out less accurate -- 1988 of 2000 here; tests/test_pt_roots_gpu.py holds
    the stage to the oracle's bits).  (The one-lane-per-sample kernel it was once
    compared with left the library in round 4; test_5pt_matches_oracle_and_ground_truth
    checks the solver against the oracle.)"""
    rng = np.random.default_rng(5)
    p0, p1, Es = _five_point_samples(rng, 2000, noise_free=True)
    cand, ncand = _pt5_roots(1, p0, p1)
    found = 0
    for s in range(len(Es)):
        best = 1.0
        for k in range(ncand[s]):
            E = cand[s, 9 * k: 9 * k + 9].reshape(3, 3)
            E = E / np.linalg.norm(E)
            best = min(best, np.abs(E - Es[s]).max(), np.abs(E + Es[s]).max())
        found += best < 1e-6
    assert found >= 0.99 * len(Es), found
    # impl values other than the estimator's stage are refused
    with pytest.raises(ValueError):
        _pt5_roots(0, p0[:4], p1[:4])

@pytest.mark.parametrize("variant", [0, 1, 2])
def test_parallel_lo_steps_match_serial(monkeypatch, variant):
    """LO steps run concurrently from predicted random-stream positions and are
    validated afterwards; the whole run must equal the serial LO exactly."""
    kind = ["calibrated", "shared_focal", "two_focal"][variant]
    p = synthetic.make_pair(30 + variant, n=800)
    o, c = synthetic.example_options(kind, iterations=1500, min_iterations=1500)
    o.max_num_iterations_per_solver = 1500
    cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
    fn = [madpose.HybridEstimatePoseScaleOffset, madpose.HybridEstimatePoseScaleOffsetSharedFocal,
          madpose.HybridEstimatePoseScaleOffsetTwoFocal][variant]
    outs = []
    for par in ["0", "1"]:
        monkeypatch.setenv("MADPOSE_LO_PARALLEL", par)
        outs.append(fn(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1, o, c))
    (p0, s0), (p1, s1) = outs
    assert s0.number_lo_iterations > 0
    assert np.array_equal(p0.pose, p1.pose)
    assert s0.inlier_indices == s1.inlier_indices
    assert s0.num_iterations_total == s1.num_iterations_total
    assert s0.number_lo_iterations == s1.number_lo_iterations
    assert s0.num_hypotheses == s1.num_hypotheses
    assert s0.best_model_score == s1.best_model_score
