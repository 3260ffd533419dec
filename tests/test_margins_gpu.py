"""The screening margins of score_batch (mp_score.h score_margins) against
the reference-order sums and errors of the host sweep (host/lo_sweep.h, bit-identical to
the oracle's EvaluateModelOnPoint / ScoreModel, src/hybrid_pose_estimator.cpp:216-261,
src/hybrid_ransac.h:265-287):

* per model, |device sum - reference-order sum| <= the model's margin, for models near
  the truth, random models and far ones, every variant, every score type;
* per correspondence (calibrated, thresholds known in pixels), |min(e_dev, thr) -
  min(e_ref, thr)| <= the per-term bound wherever the correspondence is not flagged;
* correspondences built onto the gates -- a depth at z = 1e-2 to the last bit, a
  cheirality quantity at its threshold, a correspondence at both epipoles (Sampson
  denominator ~0) -- are flagged, and their iterations reported uncertain, so that only
  reference-order sums decide there (VERDICT r04 weak #3b);
* whole estimates on pairs holding such correspondences for the truth match the
  oracle in every field.
"""
import numpy as np
import pytest

import madpose
from madpose_amd import api, synthetic
from tests.test_engine_gpu import _assert_parity, _models_near_gt, _run_both

pytestmark = pytest.mark.gpu

UNC = 1 << 17
BIG = np.finfo(np.float64).max


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


def _cams(p, variant):
    return (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])


def _models(p, rng, variant, k):
    ms = _models_near_gt(p, rng, k, variant)
    for _ in range(k // 2):  # far models: random rotation, translation, depth transform
        A = rng.standard_normal((3, 3))
        U, _, Vt = np.linalg.svd(A)
        R = U @ Vt * np.sign(np.linalg.det(U @ Vt))
        t = rng.standard_normal(3) * rng.uniform(0.1, 3)
        s, o0, o1 = rng.uniform(0.2, 5), rng.normal(0, 2), rng.normal(0, 2)
        if variant == 0:
            ms.append(madpose.PoseScaleOffset(R, t, s, o0, o1))
        elif variant == 1:
            ms.append(madpose.PoseScaleOffsetSharedFocal(R, t, s, o0, o1, rng.uniform(0.3, 3)))
        else:
            ms.append(madpose.PoseScaleOffsetTwoFocal(R, t, s, o0, o1, rng.uniform(0.3, 3), rng.uniform(0.3, 3)))
    return ms


@pytest.mark.parametrize("score_type", [0, 1, 2])
@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_sums_within_margins(variant, score_type):
    """Variant 3 (scale-only): the calibrated geometry without offsets,
    scored by the non-FAST matrix path with its own z < 1e-2 rule and 1/scale models."""
    rng = np.random.default_rng(300 + 3 * variant + score_type)
    p = synthetic.make_pair(300 + variant, n=1700)
    o, c = synthetic.example_options(["calibrated", "shared_focal", "two_focal", "calibrated"][variant])
    c.score_type = score_type
    cam0, cam1 = _cams(p, 0 if variant == 3 else variant)
    if variant == 3:
        ms = [api.PoseAndScale(m.R(), m.t(), m.scale) for m in _models(p, rng, 0, 48)]
    else:
        ms = _models(p, rng, variant, 48)
    args = (variant, p["x0"], p["x1"], p["depth0"], p["depth1"], cam0, cam1, o, c)
    dev, slots, _, bounds = api.debug_score_batch(*args, [[m] for m in ms], best=BIG, exit=False, record_skip=False)
    ref = api.score_models(*args, ms, host_lo=True)
    ties = np.array([t[0] for t in bounds["tie"]])
    checked, worst = 0, 0.0
    for k in range(len(ms)):
        if slots[k] & UNC:
            continue
        assert np.isfinite(ties[k]) and ties[k] > 0
        d = abs(dev[k] - ref[k])
        assert d <= ties[k], (k, dev[k], ref[k], ties[k])
        worst = max(worst, d / ties[k])
        checked += 1
    assert checked >= len(ms) - 2
    assert worst < 0.5  # (the margins are generous; report-level headroom)


@pytest.mark.parametrize("thr", [None, 1e-30, 1e-300])
def test_terms_within_bounds_calibrated(thr):
    rng = np.random.default_rng(7)
    p = synthetic.make_pair(17, n=1200)
    o, c = synthetic.example_options("calibrated")
    if thr is not None:
        o.squared_inlier_thresholds = [thr, thr]
    thr_t = [o.squared_inlier_thresholds[0]] * 2 + [o.squared_inlier_thresholds[1]]
    ms = _models(p, rng, 0, 24)
    args = (0, p["x0"], p["x1"], p["depth0"], p["depth1"], p["K0"], p["K1"], o, c)
    err, flags, taus, ties = api.debug_score_terms(*args, ms)
    _, ref_err = api.score_models(*args, ms, with_errors=True, host_lo=True)
    ref_err = np.asarray(ref_err).reshape(len(ms), 3, -1)
    for k in range(len(ms)):
        ok = flags[k] == 0
        for t in range(3):
            a = np.minimum(err[k, t], thr_t[t])[ok]
            b = np.minimum(ref_err[k, t], thr_t[t])[ok]
            assert np.all(np.abs(a - b) <= taus[k, t]), (k, t, np.max(np.abs(a - b)), taus[k, t])
    assert flags.sum() <= 2


def _ref_z(K0i, R, t, x, d, o0):
    """z of EvaluateModelOnPoint t = 0 in the reference's operation order (oracle mv3)."""
    a = [K0i[j, 0] * x[0] + K0i[j, 1] * x[1] + K0i[j, 2] for j in range(3)]
    s = d + o0
    pp = [a[j] * s for j in range(3)]
    return R[2, 0] * pp[0] + R[2, 1] * pp[1] + R[2, 2] * pp[2]


def test_gate_correspondences_are_flagged():
    """A depth on the z gate, a cheirality quantity on its threshold, a correspondence at
    both epipoles: flagged, and the iterations holding such models uncertain."""
    rng = np.random.default_rng(9)
    p = synthetic.make_pair(19, n=600)
    o, c = synthetic.example_options("calibrated")
    K0, K1 = p["K0"], p["K1"]
    K0i, K1i = np.linalg.inv(K0), np.linalg.inv(K1)
    base = _models_near_gt(p, rng, 3, 0)
    x0, x1 = p["x0"].copy(), p["x1"].copy()
    d0, d1 = p["depth0"].copy(), p["depth1"].copy()
    models, marked = [], []
    # (1) z gate: t_z so that z = 1e-2 in the reference's arithmetic for correspondence 5
    m = base[0]
    R, t = m.R(), m.t().copy()
    i = 5
    t[2] = 0.01 - _ref_z(K0i, R, t, x0[i], d0[i], m.offset0)
    models.append(madpose.PoseScaleOffset(R, t, m.scale, m.offset0, m.offset1))
    marked.append(i)
    # (2) cheirality: l1 = min_depth (1 - a^2) for correspondence 9 (t moved along the
    # gradient of l1 - md in t, which is linear in t)
    m = base[1]
    R, t = m.R(), m.t().copy()
    i = 9
    a0 = K0i @ np.r_[x0[i], 1.0]
    b0 = K1i @ np.r_[x1[i], 1.0]
    n0, n1 = a0 / np.linalg.norm(a0), b0 / np.linalg.norm(b0)
    rn = R @ n0
    a = -rn @ n1
    g = -rn - a * n1  # l1 = b1 - a b2 = g . t
    md = 1e-2 * (1 - a * a)
    t = t + (md - g @ t) / (g @ g) * g
    models.append(madpose.PoseScaleOffset(R, t, m.scale, m.offset0, m.offset1))
    marked.append(i)
    # (3) correspondence 13 at both epipoles of the third model
    m = base[2]
    R, t = m.R(), m.t()
    E = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]]) @ R
    U, _, Vt = np.linalg.svd(E)
    e0, e1 = Vt[2], U[:, 2]  # E e0 = 0, e1^T E = 0
    i = 13
    x0[i] = (K0 @ (e0 / e0[2]))[:2]
    x1[i] = (K1 @ (e1 / e1[2]))[:2]
    models.append(m)
    marked.append(i)
    args = (0, x0, x1, d0, d1, K0, K1, o, c)
    err, flags, taus, ties = api.debug_score_terms(*args, models)
    for k, i in enumerate(marked):
        assert flags[k, i] == 1, (k, i)
    _, slots, _, _ = api.debug_score_batch(*args, [[mm] for mm in models], best=BIG, exit=False, record_skip=False)
    assert np.all(slots & UNC)
    # scale-only (variant 3): the same z-gate correspondence of the first model
    # -- offsets are 0 there, so t_z is rebuilt for o0 = 0 -- flags its iteration too
    m = base[0]
    R, t = m.R(), m.t().copy()
    t[2] = 0.01 - _ref_z(K0i, R, t, x0[5], d0[5], 0.0)
    so = [api.PoseAndScale(R, t, m.scale)]
    args3 = (3, x0, x1, d0, d1, K0, K1, o, c)
    _, slots3, _, _ = api.debug_score_batch(*args3, [so], best=BIG, exit=False, record_skip=False)
    assert slots3[0] & UNC


@pytest.mark.parametrize("seed", [0, 1])
def test_estimator_with_gate_correspondences_matches_oracle(seed):
    """Correspondences placed on the z gate of the pose the engine estimates on a clean
    pair, then the estimate redone on the augmented pair by engine and oracle: full
    parity (the LO and final models pass within rounding of the gate)."""
    p = synthetic.make_pair(40 + seed, n=500, noise_px=0.0, depth_noise=0.0)
    o, c = synthetic.example_options("calibrated", iterations=400)
    o.random_seed = seed
    pose, _ = madpose.HybridEstimatePoseScaleOffset(p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"],
                                                    p["K0"], p["K1"], o, c)
    K0i, K1i = np.linalg.inv(p["K0"]), np.linalg.inv(p["K1"])
    R, t = pose.R(), pose.t()
    rng = np.random.default_rng(seed)
    x0, x1 = list(p["x0"]), list(p["x1"])
    d0, d1 = list(p["depth0"]), list(p["depth1"])
    for _ in range(8):
        # a correspondence whose depth lands on z = 1e-2 under the estimate: choose the
        # depth prior d0 so that (R a (d0 + o0) + t)_z = 1e-2
        u = np.r_[rng.uniform(0, 640), rng.uniform(0, 480)]
        a = K0i @ np.r_[u, 1.0]
        ra = R[2] @ a
        if abs(ra) < 1e-3:
            continue
        dd = (0.01 - t[2]) / ra - pose.offset0
        if dd <= 0:
            continue
        x0.append(u)
        x1.append(np.r_[rng.uniform(0, 640), rng.uniform(0, 480)])
        d0.append(dd)
        d1.append(rng.uniform(1, 8))
    q = dict(p)
    q["x0"], q["x1"] = np.asarray(x0), np.asarray(x1)
    q["depth0"], q["depth1"] = np.asarray(d0), np.asarray(d1)
    q["min_depth"] = np.array([q["depth0"].min(), q["depth1"].min()])
    _assert_parity(*_run_both(q, o, c, 0))
