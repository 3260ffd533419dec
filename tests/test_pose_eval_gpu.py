"""Device pose-error and pose-AUC evaluator (mp_pose_eval): the
reference's compute_pose_error (madpose/utils.py:59-78) pinned by its recorded outputs
(tests/golden/utils.npz pe_*), and the AUC against the host pose_auc on random error
sets with ties, exact-threshold values, NaN errors, several workgroups' worth of pairs
and the empty set.

Tolerances: errors 1e-9 degrees absolute, except at angles within 1e-3 degrees of 0
(after the translation fold, also of 180): there acos is ill-conditioned, and a
one-ulp difference in the trace or dot product (summation order, FMA contraction)
moves an exact 0 to deg(sqrt(2 eps)) ~ 1.2e-6 degrees, so the bound is 2e-6 there;
AUCs 1e-12 relative (the same trapezoid terms, summed in another order)."""
import os

import numpy as np
import pytest

import madpose
from madpose_amd import utils

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


def _close_angles(dev, ref):
    tol = np.where(np.abs(ref) < 1e-3, 2e-6, 1e-9)
    return bool(np.all(np.abs(dev - ref) <= tol))


def _rand_rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def test_pose_errors_match_reference_golden():
    g = np.load(os.path.join(GOLDEN, "utils.npz"))
    et, eR, _ = madpose.pose_eval_batch(g["pe_T"], g["pe_R"], g["pe_t"], thresholds=())
    assert _close_angles(et, g["pe_err"][:, 0])
    assert _close_angles(eR, g["pe_err"][:, 1])


def test_pose_errors_match_numpy_with_t_thres():
    rng = np.random.default_rng(11)
    k = 700
    T = np.tile(np.eye(4), (k, 1, 1))
    R = np.empty((k, 3, 3))
    t = rng.normal(size=(k, 3))
    for i in range(k):
        T[i, :3, :3] = _rand_rot(rng)
        T[i, :3, 3] = rng.normal(size=3) * rng.choice([1e-3, 1.0])
        # estimates from exact to far off, including sign-flipped translations
        R[i] = T[i, :3, :3] if i % 7 == 0 else _rand_rot(rng)
        if i % 5 == 0:
            t[i] = -2.5 * T[i, :3, 3]
    for t_thres in (None, 0.05):
        et, eR, _ = madpose.pose_eval_batch(T, R, t, thresholds=(), t_thres=t_thres)
        ref = np.array([utils.compute_pose_error(T[i], R[i], t[i], t_thres) for i in range(k)])
        assert _close_angles(et, ref[:, 0])
        assert _close_angles(eR, ref[:, 1])


@pytest.mark.parametrize("k", [1, 37, 1500, 5000])
def test_pose_auc_matches_host(k):
    rng = np.random.default_rng(k)
    T = np.tile(np.eye(4), (k, 1, 1))
    R = np.empty((k, 3, 3))
    t = np.empty((k, 3))
    for i in range(k):
        T[i, :3, :3] = _rand_rot(rng)
        T[i, :3, 3] = rng.normal(size=3)
        ang = np.deg2rad(rng.exponential(8.0))
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        Kx = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        dR = np.eye(3) + np.sin(ang) * Kx + (1 - np.cos(ang)) * Kx @ Kx
        R[i] = dR @ T[i, :3, :3]
        t[i] = T[i, :3, 3] + rng.normal(size=3) * 0.1
    if k > 10:  # duplicates (ties) and exact copies of the ground truth (zero errors)
        R[1], t[1] = R[0], t[0]
        T[1] = T[0]
        R[2], t[2] = T[2, :3, :3], T[2, :3, 3]
    et, eR, aucs = madpose.pose_eval_batch(T, R, t, thresholds=(5, 10, 20))
    e = np.maximum(eR, et)
    ref = utils.pose_auc(e, (5, 10, 20))
    assert np.allclose(aucs, ref, rtol=1e-12, atol=1e-15)


def test_pose_auc_ties_threshold_values_and_nan():
    # errors placed exactly on the thresholds, repeated values and a NaN (zero
    # translation): fed through poses whose errors are known
    k = 9
    T = np.tile(np.eye(4), (k, 1, 1))
    T[:, :3, 3] = [1.0, 0.0, 0.0]
    R = np.tile(np.eye(3), (k, 1, 1))
    angles = [0.0, 5.0, 5.0, 2.5, 10.0, 19.0, 30.0, 1.0, 7.0]
    t = np.empty((k, 3))
    for i, a in enumerate(angles):
        r = np.deg2rad(a)
        t[i] = [np.cos(r), np.sin(r), 0.0]
    t[8] = 0.0  # NaN translation error
    et, eR, aucs = madpose.pose_eval_batch(T, R, t, thresholds=(5, 10, 20))
    ref_e = [utils.compute_pose_error(T[i], R[i], t[i]) for i in range(k)]
    assert np.isnan(et[8]) and np.isnan(ref_e[8][0])
    e = np.maximum(eR, et)
    ref = utils.pose_auc(e, (5, 10, 20))
    assert np.allclose(aucs, ref, rtol=1e-12, atol=1e-15)


def test_pose_eval_empty_and_bad_thresholds():
    et, eR, aucs = madpose.pose_eval_batch(np.zeros((0, 4, 4)), np.zeros((0, 3, 3)), np.zeros((0, 3)))
    assert len(et) == 0 and len(eR) == 0 and all(np.isnan(a) for a in aucs)
    with pytest.raises(ValueError):
        madpose.pose_eval_batch(np.eye(4)[None], np.eye(3)[None], np.ones((1, 3)), thresholds=(0.0,))


def test_pose_auc_from_errors_matches_host():
    rng = np.random.default_rng(5)
    e = np.r_[rng.exponential(6.0, 3000), [0.0, 0.0, 5.0, 10.0, 20.0, np.nan]]
    rng.shuffle(e)
    assert np.allclose(madpose.pose_auc_batch(e, (5, 10, 20)), utils.pose_auc(e, (5, 10, 20)), rtol=1e-12, atol=1e-15)
    assert all(np.isnan(a) for a in madpose.pose_auc_batch([], (5,)))
