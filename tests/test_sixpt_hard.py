"""The shared-focal 6pt samples on which the device root stage and the oracle once
disagreed (tests/golden/sixpt_hard.json, built by tests/golden/gen_sixpt_hard.py from
the diagnostic records under profiles/): the oracle's positive roots u of
q(u) = det(u^2 M0 + u M1 + M2) / u^5 against 60-digit roots (CPU), and on the GPU the
device root stage (the deflated eigenproblem) against the same roots and the device
6pt poses against the oracle's (PoseLib relpose_6pt_shared_focal, called at
/root/reference/src/hybrid_pose_shared_focal_estimator.cpp:87; restated in
oracle/src/pt67.cpp)."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
SAMPLES = json.load(open(os.path.join(HERE, "golden", "sixpt_hard.json")))["samples"]
IDS = [s["origin"].split()[-3] + "-" + s["origin"].split()[-1] + "-" + str(i) for i, s in enumerate(SAMPLES)]


def _h(p):
    p = np.asarray(p, float)
    return np.hstack([p, np.ones((len(p), 1))])


def _same_roots(got, want, tol=1e-6):
    got = sorted(got)
    return len(got) == len(want) and all(abs(a - b) <= tol * max(1.0, abs(b)) for a, b in zip(got, want))


def test_fixture_is_well_posed():
    assert len(SAMPLES) >= 11
    assert not any(s["ill_posed"] for s in SAMPLES)


@pytest.mark.parametrize("k", range(len(SAMPLES)), ids=IDS)
def test_oracle_roots_match_60_digit_roots(k):
    s = SAMPLES[k]
    assert _same_roots(oracle.sixpt_roots(_h(s["p0"]), _h(s["p1"])), s["roots_u"])


def _device_roots(p0, p1):
    from madpose_amd import _lib as L

    ns = p0.shape[0]
    cand = np.zeros((ns, 96))
    ncand = np.zeros(ns, dtype=np.int32)
    dp = lambda a: np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    # impl 3: the estimator's shared-focal root stage (pencil, deflation, lockstep QR)
    L.check(L.lib().mp_debug_pt_roots(1, 3, ns, dp(p0), dp(p1), cand.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                      ncand.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 0))
    return [cand[s, 27: 27 + ncand[s]] for s in range(ns)]


@pytest.mark.gpu
def test_device_roots_match_60_digit_roots():
    import madpose

    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")
    p0 = np.array([s["p0"] for s in SAMPLES])
    p1 = np.array([s["p1"] for s in SAMPLES])
    roots = _device_roots(p0, p1)
    bad = [IDS[k] for k, s in enumerate(SAMPLES) if not _same_roots(roots[k], s["roots_u"])]
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(SAMPLES)), ids=IDS)
def test_device_6pt_poses_match_oracle(k):
    import madpose

    s = SAMPLES[k]
    p0, p1 = np.asarray(s["p0"]), np.asarray(s["p1"])
    dev = madpose.relpose_6pt_shared_focal(p0, p1)
    b0 = _h(p0) / np.linalg.norm(_h(p0), axis=1, keepdims=True)
    b1 = _h(p1) / np.linalg.norm(_h(p1), axis=1, keepdims=True)
    orc = oracle.relpose_6pt_shared_focal(b0, b1)
    assert len(dev) == len(orc), (sorted(m.focal for m in dev), sorted(o["focal0"] for o in orc))
    for m in dev:
        d = min(np.abs(m.R() - o["R"]).max() + np.abs(m.t() - o["t"]).max() + abs(m.focal - o["focal0"]) for o in orc)
        assert d <= 1e-6, (d, m.focal)
