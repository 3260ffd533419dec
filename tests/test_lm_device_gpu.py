"""Batched device LM (kernels/lm_device.h) against the oracle's
LeastSquares / NonMinimalSolver (the Ceres restatement of src/optimizer.h:48-125 over
src/cost_functions.h:16-387, parity unpinned: Ceres is not vendored).  Many problems of
one pair in one launch: subsets of the three data types as the LO draws them, start
models perturbed from the ground truth, all three variants, both solver kinds, the
non-monotonic step evaluator on and off, and the EPI_ONLY / MD_ONLY LO modes."""
import numpy as np
import pytest

import madpose
import oracle
from madpose_amd import synthetic
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg

pytestmark = pytest.mark.gpu

KIND = {0: "calibrated", 1: "shared_focal", 2: "two_focal"}


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


def _small_rot(rng, deg):
    a = rng.standard_normal(3)
    a *= np.deg2rad(deg) / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    th = np.linalg.norm(a)
    K /= th
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def _problems(rng, p, variant, norm_scale, count, est):
    """LO-like problems: start models near the estimator's own result `est` (problem
    units), residual blocks drawn as the LO draws them (subsets of the inliers, some
    with outliers, and all-inlier fits)."""
    inl = np.flatnonzero(p["inlier_mask"])
    out = []
    for j in range(count):
        sizes = [int(rng.integers(0, 150)), int(rng.integers(0, 150)), int(rng.integers(5, 300))]
        if j % 5 == 0:
            sizes = [len(inl), len(inl), len(inl)]  # an all-inlier fit (the big LO problems)
        lists = [rng.choice(inl, min(s, len(inl)), replace=False) for s in sizes]
        if j % 3 == 0:  # a few outliers, as a relaxed-threshold inlier set holds them
            out_idx = np.flatnonzero(~p["inlier_mask"])
            lists = [np.r_[l, rng.choice(out_idx, len(l) // 30, replace=False)] for l in lists]
        lists = [np.sort(l) for l in lists]
        R = est.R() @ _small_rot(rng, 0.5)
        t = est.t() * (1 + 0.02 * rng.standard_normal(3))
        sc, o0, o1 = est.scale * (1 + 0.01 * rng.standard_normal()), est.offset0, est.offset1
        if variant == 0:
            m = madpose.PoseScaleOffset(R, t, sc, o0, o1)
        elif variant == 1:
            m = madpose.PoseScaleOffsetSharedFocal(R, t, sc, o0, o1, est.focal / norm_scale * 1.02)
        else:
            m = madpose.PoseScaleOffsetTwoFocal(R, t, sc, o0, o1, est.focal0 / norm_scale * 1.02,
                                                est.focal1 / norm_scale * 0.98)
        out.append((j % 2, lists, m))
    return out


def _close(m, ref, variant, tol=1e-7, epi_only=False):
    ok = rot_angle_deg(m.R(), ref["R"]) < 1e-6
    if epi_only:
        # Sampson residuals alone do not observe |t| (E = [t]x R up to scale): the LM
        # moves along that null direction by rounding, so only the direction is compared
        ok &= bool(np.allclose(m.t() / np.linalg.norm(m.t()), ref["t"] / np.linalg.norm(ref["t"]), rtol=tol,
                               atol=1e-9))
    else:
        ok &= bool(np.allclose(m.t(), ref["t"], rtol=tol, atol=1e-9))
    for k in ("scale", "offset0", "offset1"):
        ok &= abs(getattr(m, k) - ref[k]) <= tol * (1 + abs(ref[k]))
    if variant == 1:
        ok &= abs(m.focal - ref["focal0"]) <= tol * ref["focal0"]
    elif variant == 2:
        ok &= abs(m.focal0 - ref["focal0"]) <= tol * ref["focal0"] and abs(m.focal1 - ref["focal1"]) <= tol * ref["focal1"]
    return bool(ok)


def _near_start(ref, m0, variant):
    """The oracle's minimum lies near the start: rotation within 10 degrees, scale
    and focals within a factor 2, offsets within 10 x (1 + |start|) of the start.
    (A two-focal EPI_ONLY fit can run a focal into its 1e-6 bound: Sampson residuals
    alone leave it nearly unobserved, and there implementations part at rounding.)"""
    if rot_angle_deg(ref["R"], m0.R()) > 10.0 or not 0.5 < ref["scale"] / m0.scale < 2.0:
        return False
    f0 = None if variant == 0 else (m0.focal, m0.focal) if variant == 1 else (m0.focal0, m0.focal1)
    if f0 is not None and not all(0.5 < ref[k] / f < 2.0 for k, f in zip(("focal0", "focal1"), f0)):
        return False
    return all(abs(ref[k] - getattr(m0, k)) <= 10.0 * (1.0 + abs(getattr(m0, k))) for k in ("offset0", "offset1"))


def _close_dicts(a, b, variant, tol=1e-7, epi_only=False):
    mk = [madpose.PoseScaleOffset, madpose.PoseScaleOffsetSharedFocal, madpose.PoseScaleOffsetTwoFocal][variant]
    foc = [[], [a["focal0"]], [a["focal0"], a["focal1"]]][variant]
    return _close(mk(a["R"], a["t"], a["scale"], a["offset0"], a["offset1"], *foc), b, variant, tol, epi_only)


def _oracle_model(m, variant):
    d = dict(R=m.R(), t=m.t(), scale=m.scale, offset0=m.offset0, offset1=m.offset1, focal0=1.0, focal1=1.0)
    if variant == 1:
        d["focal0"] = d["focal1"] = m.focal
    elif variant == 2:
        d["focal0"], d["focal1"] = m.focal0, m.focal1
    return d


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("nonmono,lo_type", [(True, 0), (False, 0), (True, 1), (True, 2)])
def test_device_lm_matches_oracle(variant, nonmono, lo_type):
    rng = np.random.default_rng(100 + variant)
    p = synthetic.make_pair(40 + variant, n=800) if variant < 2 else synthetic.config_pair(4, seed=40)
    o, c = synthetic.example_options(KIND[variant], iterations=100)
    c.ceres_use_nonmonotonic_steps = nonmono
    c.LO_type = lo_type
    cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
    args = (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1)
    _, _, norm_scale = oracle.score_models(variant, *args[:4], cam0, cam1, oracle_opts(o), oracle_cfg(c), [])
    # start models near the oracle's own estimate of the pair (problem units)
    m, _, _ = oracle.estimate(variant, *args, oracle_opts(o),
                              oracle_cfg(synthetic.example_options(KIND[variant], iterations=100)[1]))
    mk = [madpose.PoseScaleOffset, madpose.PoseScaleOffsetSharedFocal, madpose.PoseScaleOffsetTwoFocal][variant]
    est = mk(m["R"], m["t"], m["scale"], m["offset0"], m["offset1"], *[[], [m["focal0"]],
                                                                         [m["focal0"], m["focal1"]]][variant])
    # 24 problems whose start lies in the basin of a nearby minimum: the oracle's
    # solution stays near the start.  Some LO-like starts (found with 48 / 38 / 182
    # residuals as with 5) let the non-monotonic evaluator run an offset away to ~1e7,
    # where rounding-level differences between ANY two implementations grow; such a
    # start is a property of the problem, decided by the oracle alone, before the
    # device runs
    probs, refs = [], []
    for cand in _problems(rng, p, variant, norm_scale, 96, est):
        kind, lists, m0 = cand
        ref, ran = oracle.least_squares(variant, *args, oracle_opts(o), oracle_cfg(c), kind, lists,
                                        _oracle_model(m0, variant))
        if ran and not _near_start(ref, m0, variant):
            continue
        if ran:
            # ... and that minimum is stable: the oracle restarted from its own result
            # stays there (Sampson-only two-focal fits can sit on a ridge from which a
            # restart runs off to focals ~0.05, where the implementations' rounding-level
            # differences decide where they stop)
            again, _ = oracle.least_squares(variant, *args, oracle_opts(o), oracle_cfg(c), kind, lists,
                                            dict(ref))
            if not _close_dicts(again, ref, variant, epi_only=lo_type == 1):
                continue
        probs.append(cand)
        refs.append((ref, ran))
        if len(probs) == 24:
            break
    assert len(probs) == 24
    got = madpose.lm_refine_batch(variant, *args, o, c, probs)
    host = madpose.lm_refine_batch(variant, *args, o, c, probs, on_host=True)
    for (kind, lists, m0), (m, st), (mh, sth), (ref, ran) in zip(probs, got, host, refs):
        if not ran:
            assert st == 3 and sth == 3
            assert np.array_equal(m.pose, m0.pose)
            continue
        assert st in (0, 1, 2) and st == sth
        # every problem: the engine's host LM and the device LM both agree with the oracle
        sizes = [len(x) for x in lists]
        assert _close(mh, ref, variant, epi_only=lo_type == 1), ("host", kind, sizes)
        assert _close(m, ref, variant, epi_only=lo_type == 1), ("device", kind, sizes)


def test_device_lm_many_problems_deterministic():
    """Several hundred problems in one launch, twice: bit-identical refined models and
    statuses (the proposal flag of lm_batch_kernel is published once per iteration
    after a barrier; a wave reading it early would leave its loop and sum a stale
    partial row -- ADVICE r02)."""
    variant = 0
    rng = np.random.default_rng(7)
    p = synthetic.make_pair(44, n=800)
    o, c = synthetic.example_options(KIND[variant], iterations=100)
    args = (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["K0"], p["K1"])
    _, _, norm_scale = oracle.score_models(variant, *args[:4], p["K0"], p["K1"], oracle_opts(o), oracle_cfg(c), [])
    m, _, _ = oracle.estimate(variant, *args, oracle_opts(o), oracle_cfg(c))
    est = madpose.PoseScaleOffset(m["R"], m["t"], m["scale"], m["offset0"], m["offset1"])
    probs = _problems(rng, p, variant, norm_scale, 384, est)
    a = madpose.lm_refine_batch(variant, *args, o, c, probs)
    b = madpose.lm_refine_batch(variant, *args, o, c, probs)
    assert len(a) == len(b) == 384
    for (ma, sa), (mb, sb) in zip(a, b):
        assert sa == sb
        assert np.array_equal(ma.pose, mb.pose)
