"""The engine's host LO sweep (madpose_amd/csrc/host/lo_sweep.cpp, through the C ABI
test hook mp_debug_lo_sweep) against the oracle's ScoreModel / GetInliers
(oracle/src/capi.cpp oracle_score_models; src/hybrid_ransac.h:265-349).

The sweep evaluates the reference's residual operation sequence lane-parallel without
FMA contraction and sums the MSAC terms in the reference's order (t outer, i
ascending, one accumulator), so errors AND scores must be bit-identical to the
oracle's scalar loops -- for every variant, score type and both instruction sets
(AVX-512 and the AVX2 baseline, selected by MADPOSE_LO_SWEEP_ISA in a subprocess).
No device is used."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import madpose
import oracle
from madpose_amd import synthetic
from tests.helpers import oracle_cfg, oracle_opts

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rand_rot(rng):
    R = np.linalg.qr(rng.standard_normal((3, 3)))[0]
    return R * np.linalg.det(R)


def _models(p, rng, k, variant):
    """Models near the ground truth (most inliers) plus a few far ones (cheirality
    failures, z < 1e-2 sentinels)."""
    out = []
    for j in range(k):
        far = j % 4 == 3
        dR = _rand_rot(rng) if far else np.eye(3)
        ang = rng.normal(0, 0.01, 3)
        Kx = np.array([[0, -ang[2], ang[1]], [ang[2], 0, -ang[0]], [-ang[1], ang[0], 0]])
        U, _, Vt = np.linalg.svd(dR @ (np.eye(3) + Kx) @ p["R"])
        R = U @ Vt
        t = p["t"] + rng.normal(0, 0.3 if far else 0.02, 3)
        scale, o0, o1 = rng.uniform(0.5, 2), rng.normal(0, 0.2), rng.normal(0, 0.2)
        if variant in (0, 3):
            out.append(madpose.PoseScaleOffset(R, t, scale, o0, o1))
        elif variant == 1:
            out.append(madpose.PoseScaleOffsetSharedFocal(R, t, scale, o0, o1, rng.uniform(0.8, 1.5)))
        else:
            out.append(madpose.PoseScaleOffsetTwoFocal(R, t, scale, o0, o1, rng.uniform(0.8, 1.5),
                                                       rng.uniform(0.8, 1.5)))
    return out


def _to_oracle(m, variant):
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


def _case(variant, score_type, seed, n):
    rng = np.random.default_rng(seed)
    p = synthetic.make_pair(seed, n=n)
    o, c = synthetic.example_options("two_focal" if variant == 2 else "calibrated")
    o.data_type_weights = [1.0, rng.uniform(0.5, 3.0)]
    c.score_type = score_type
    cam0, cam1 = (p["K0"], p["K1"]) if variant in (0, 3) else (p["pp0"], p["pp1"])
    d0, d1 = p["depth0"].copy(), p["depth1"].copy()
    if variant == 3:  # scale-only rejects priors below 1e-2 (src/hybrid_pose_estimator.cpp:395, 408)
        d0[::17] = 1e-3
        d1[::23] = 5e-3
    models = _models(p, rng, 8, variant)
    return p, o, c, cam0, cam1, d0, d1, models


def _compare(variant, score_type, seed, n):
    p, o, c, cam0, cam1, d0, d1, models = _case(variant, score_type, seed, n)
    sc, err = madpose.score_models(variant, p["x0"], p["x1"], d0, d1, cam0, cam1, o, c, models, with_errors=True,
                                   host_lo=True)
    ov = 3 if variant == 3 else variant
    osc, oerr, _ = oracle.score_models(ov, p["x0"], p["x1"], d0, d1, cam0, cam1, oracle_opts(o), oracle_cfg(c),
                                       [_to_oracle(m, variant) for m in models])
    return sc, err, osc, oerr


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("score_type", [0, 1, 2])
def test_host_lo_sweep_bit_identical_to_oracle(variant, score_type):
    for seed, n in ((10 + variant, 701), (20 + variant, 64)):
        sc, err, osc, oerr = _compare(variant, score_type, seed, n)
        # same bits, NaN-aware (np.array_equal with equal_nan compares values)
        assert np.array_equal(err.view(np.uint64), oerr.view(np.uint64)), (
            variant, score_type, seed, int(np.sum(err.view(np.uint64) != oerr.view(np.uint64))))
        assert np.array_equal(sc.view(np.uint64), osc.view(np.uint64)), (sc, osc)
        big = np.finfo(np.float64).max
        assert np.any(err == big) or variant != 0  # the far models hit the sentinels


def test_host_lo_sweep_edge_sizes():
    """n = 0 (empty pair), n = 1 and sizes around the vector width (ragged tails)."""
    for n in (0, 1, 7, 9, 15, 17):
        rng = np.random.default_rng(n)
        p = synthetic.make_pair(5, n=max(n, 1))
        x0, x1, d0, d1 = p["x0"][:n], p["x1"][:n], p["depth0"][:n], p["depth1"][:n]
        o, c = synthetic.example_options("calibrated")
        models = _models(p, rng, 3, 0)
        sc, err = madpose.score_models(0, x0, x1, d0, d1, p["K0"], p["K1"], o, c, models, with_errors=True,
                                       host_lo=True)
        osc, oerr, _ = oracle.score_models(0, x0, x1, d0, d1, p["K0"], p["K1"], oracle_opts(o), oracle_cfg(c),
                                           [_to_oracle(m, 0) for m in models])
        assert np.array_equal(err.view(np.uint64), oerr.view(np.uint64))
        assert np.array_equal(sc.view(np.uint64), osc.view(np.uint64))


_CHILD = r"""
import json, sys
sys.path.insert(0, {root!r})
from tests.test_lo_sweep_cpu import _compare
out = []
for v in (0, 1, 2):
    sc, err, osc, oerr = _compare(v, 0, 40 + v, 333)
    out.append([bool((sc.view('u8') == osc.view('u8')).all()), bool((err.view('u8') == oerr.view('u8')).all())])
print(json.dumps(out))
"""


def test_host_lo_sweep_avx2_path_bit_identical():
    """The 4-wide baseline (MADPOSE_LO_SWEEP_ISA=avx2; the ISA is chosen once per
    process, hence the child process) gives the same bits."""
    env = dict(os.environ, MADPOSE_LO_SWEEP_ISA="avx2")
    r = subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT)], env=env, capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert all(a and b for a, b in res), res


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("case", ["example", "tiny", "negative"])
def test_fast_sum_within_bound(variant, case):
    """The LO decides most of its UpdateBestModel comparisons on a fast sum of the same
    terms (lo_sweep.h lo_sweep_fast) and takes the reference-order sum only when the fast
    one cannot decide: |fast - reference| <= bound for every model, at the example
    thresholds, at tiny ones (subnormal-range sums) and with a negative weight."""
    rng = np.random.default_rng(900 + variant)
    p = synthetic.make_pair(900 + variant, n=1300)
    kind = ["calibrated", "shared_focal", "two_focal"][variant]
    o, c = synthetic.example_options(kind)
    if case == "tiny":
        o.squared_inlier_thresholds = [1e-300, 1e-300]
    if case == "negative":
        o.data_type_weights = [1.0, -0.5]
    cam0, cam1 = (p["K0"], p["K1"]) if variant == 0 else (p["pp0"], p["pp1"])
    ms = _models(p, rng, 40, variant)
    fb = np.zeros((len(ms), 2))
    ref = madpose.score_models(variant, p["x0"], p["x1"], p["depth0"], p["depth1"], cam0, cam1, o, c, ms,
                               host_lo=True, fast_bounds=fb)
    assert np.all(fb[:, 1] >= 0)
    assert np.all(np.abs(fb[:, 0] - ref) <= fb[:, 1]), np.max(np.abs(fb[:, 0] - ref) / fb[:, 1])
    assert np.all(fb[:, 1] <= 1e-11 * np.maximum(np.abs(ref), 1e-300) + 1e-300)
