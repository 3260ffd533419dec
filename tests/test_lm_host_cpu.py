"""The engine's host LM (the default LO path: madpose_amd/csrc/host/lm.cpp through the C
ABI test hook mp_debug_lm_refine_host, no device) against the oracle's Ceres
restatement on LO-like problems (tests/lm_cases.py), every variant, both solver kinds,
the non-monotonic step evaluator on and off and the EPI_ONLY / MD_ONLY LO modes.

Every drawn problem counts: the oracle alone classifies it (lm_cases.classify); the
share it excludes is bounded and reported, the host LM must agree with the oracle on
every kept problem, and on every problem it must end at no higher cost than its start.
The one divergence found on an excluded problem is pinned: test_lm_ridge_fixture."""
import json
import os

import numpy as np
import pytest

import madpose
import oracle
from tests import lm_cases as LC
from tests.helpers import oracle_cfg, oracle_opts, rot_angle_deg

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
N_PROBLEMS = 48
# most excluded problems per configuration (of N_PROBLEMS): the shared-focal starts
# (focal x 1.02) leave the oracle's basin most often (26-28 of 96 drawn)
MAX_EXCLUDED = {0: 8, 1: 18, 2: 14}


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("nonmono,lo_type", LC.CONFIGS)
def test_host_lm_matches_oracle(variant, nonmono, lo_type):
    rng = np.random.default_rng(100 + variant)
    p, o, c, args, norm_scale, est = LC.setup(variant, nonmono, lo_type)
    cands = LC.problems(rng, p, variant, norm_scale, N_PROBLEMS, est)
    cls = LC.classify(variant, args, o, c, cands, lo_type)
    host = madpose.lm_refine_batch(variant, *args, o, c, cands, on_host=True)
    excluded = {"far": 0, "unstable": 0}
    agree_excluded = 0
    for (kind, lists, m0), (mh, sth), (ref, ran, reason) in zip(cands, host, cls):
        if not ran:
            assert sth == 3 and np.array_equal(mh.pose, m0.pose)
            continue
        assert sth in (0, 1, 2)
        # Ceres returns the lowest-cost parameters it visited: never above the start
        c0 = LC.lm_cost(variant, args, o, c, m0, lists, norm_scale)
        ch = LC.lm_cost(variant, args, o, c, mh, lists, norm_scale)
        assert ch <= c0 * (1 + 1e-9) + 1e-12, (kind, [len(x) for x in lists], ch, c0)
        ok = LC.close(mh, ref, variant, epi_only=lo_type == 1)
        if reason is None:
            assert ok, (kind, [len(x) for x in lists])
        else:
            excluded[reason] += 1
            agree_excluded += ok
    n_ex = sum(excluded.values())
    print(f"variant {variant} nonmono {nonmono} LO {lo_type}: {N_PROBLEMS} problems, excluded {excluded}, "
          f"host LM agrees with the oracle on {agree_excluded} of those anyway")
    assert n_ex <= MAX_EXCLUDED[variant], excluded
    # most excluded problems still agree (a 'far' minimum is usually well defined); the
    # ones that do not are the unstable / ridge cases -- at most 5 of 48 measured
    assert n_ex - agree_excluded <= 6, (excluded, agree_excluded)


def test_lm_ridge_fixture():
    """The problem on which the host LM once left the oracle (two-focal, LO EPI_ONLY,
    blocks [128, 52, 77]; round 3, gpurun_out/s3/pytest_gpu.log:54): a Sampson-only fit
    whose focals are barely observed.  Pinned facts (tests/golden/lm_ridge_tf.json,
    written by tests/golden/gen_lm_ridge.py): the oracle stops on a flat ridge by its
    function tolerance -- restarted from its own solution it moves ~8 degrees to tiny
    focals at a LOWER cost -- and the host LM stops elsewhere on the same ridge, at a
    cost within 1e-6 relative of the oracle's.  A rounding divergence, not a defect."""
    with open(os.path.join(GOLDEN, "lm_ridge_tf.json")) as f:
        g = json.load(f)
    variant, nonmono, lo_type = g["variant"], g["nonmono"], g["lo_type"]
    p, o, c, args, norm_scale, est = LC.setup(variant, nonmono, lo_type)
    lists = [np.asarray(l, dtype=np.int64) for l in g["lists"]]
    m0 = LC.model_of(g["start"], variant)
    ref, ran = oracle.least_squares(variant, *args, oracle_opts(o), oracle_cfg(c), g["kind"], lists,
                                    LC.oracle_model(m0, variant))
    again, _ = oracle.least_squares(variant, *args, oracle_opts(o), oracle_cfg(c), g["kind"], lists, dict(ref))
    (mh, st), = madpose.lm_refine_batch(variant, *args, o, c, [(g["kind"], lists, m0)], on_host=True)
    c0 = LC.lm_cost(variant, args, o, c, m0, lists, norm_scale)
    cr = LC.lm_cost(variant, args, o, c, LC.model_of(ref, variant), lists, norm_scale)
    ca = LC.lm_cost(variant, args, o, c, LC.model_of(again, variant), lists, norm_scale)
    ch = LC.lm_cost(variant, args, o, c, mh, lists, norm_scale)
    assert abs(cr - g["oracle_cost"]) <= 1e-9 * cr and abs(c0 - g["start_cost"]) <= 1e-9 * c0
    assert cr < 0.2 * c0 and ch < 0.2 * c0                      # both fits converge from the start ...
    assert abs(ch - cr) <= 1e-6 * cr                           # ... to the same cost level
    assert ca < cr * (1 - 1e-3) and rot_angle_deg(again["R"], ref["R"]) > 1.0  # the ridge: no isolated minimum
    assert rot_angle_deg(mh.R(), ref["R"]) < 1e-2              # the stops differ along it


def test_lm_gauge_fixture():
    """Why the EPI_ONLY agreement of tests/lm_cases.py close() is 1e-3 deg / 1e-4 in t
    direction instead of 1e-6 deg: with Sampson residuals alone |t| is unobserved (the
    Sampson distance is invariant to the scale of E = [t]x R), so an LM wanders along
    |t| by rounding and stops, by Ceres' function tolerance, where its own path leaves
    it.  Pinned (tests/golden/lm_gauge_cal.json, tests/golden/gen_lm_gauge.py): on this
    calibrated all-inlier fit the host LM and the oracle end at the same cost (8 parts in
    1e9, the host lower) with |t| 1.729 against 1.753 and the rotations 6e-6 deg apart --
    beyond the strict 1e-6 deg, well inside the EPI_ONLY bound; and scaling the oracle's
    t to the host's |t| leaves its cost unchanged to rounding."""
    with open(os.path.join(GOLDEN, "lm_gauge_cal.json")) as f:
        g = json.load(f)
    variant, nonmono, lo_type = g["variant"], g["nonmono"], g["lo_type"]
    p, o, c, args, norm_scale, est = LC.setup(variant, nonmono, lo_type)
    lists = [np.asarray(l, dtype=np.int64) for l in g["lists"]]
    m0 = LC.model_of(g["start"], variant)
    ref, ran = oracle.least_squares(variant, *args, oracle_opts(o), oracle_cfg(c), g["kind"], lists,
                                    LC.oracle_model(m0, variant))
    (mh, st), = madpose.lm_refine_batch(variant, *args, o, c, [(g["kind"], lists, m0)], on_host=True)
    cr = LC.lm_cost(variant, args, o, c, LC.model_of(ref, variant), lists, norm_scale)
    ch = LC.lm_cost(variant, args, o, c, mh, lists, norm_scale)
    assert abs(cr - g["oracle_cost"]) <= 1e-9 * cr and abs(ch - g["host_cost"]) <= 1e-9 * ch
    assert abs(ch - cr) <= 2e-6 * cr  # the same cost level (epi_only_equivalent)
    assert not LC.close(mh, ref, variant)  # the strict agreement fails ...
    assert LC.close(mh, ref, variant, epi_only=True)  # ... the EPI_ONLY one holds
    tn_h, tn_r = np.linalg.norm(mh.t()), np.linalg.norm(ref["t"])
    assert abs(tn_h - tn_r) > 1e-3 * tn_r  # the stops differ along |t|
    scaled = dict(ref)
    scaled["t"] = np.asarray(ref["t"]) * (tn_h / tn_r)
    cs = LC.lm_cost(variant, args, o, c, LC.model_of(scaled, variant), lists, norm_scale)
    assert abs(cs - cr) <= 1e-9 * cr  # |t| is a gauge of the EPI_ONLY cost


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_oracle_lm_ends_are_stationary_on_kept_problems(variant):
    """The oracle's Ceres restatement stops at a stationary point on every problem it
    keeps (start in the basin of an isolated minimum): no single-parameter step of 1e-5
    lowers its end cost by more than 1e-6 of it (lm_cases.is_local_minimum; measured
    < 5e-7).  The device-LM test's 'far' class is where this fails -- the oracle's own
    far ends stop on Ceres' rules short of a minimum -- which is why far starts are
    bounded by cost there instead of compared."""
    from tests import lm_cases as LC

    rng = np.random.default_rng(100 + variant)
    p, o, c, args, ns, est = LC.setup(variant, True, 0)
    cands = LC.problems(rng, p, variant, ns, 32, est)
    cls = LC.classify(variant, args, o, c, cands, 0)
    kept = 0
    for (kind, lists, m0), (ref, ran, reason) in zip(cands, cls):
        if not ran or reason is not None:
            continue
        ok, worst = LC.is_local_minimum(variant, args, o, c, LC.model_of(ref, variant), lists, ns)
        assert ok, (kind, [len(x) for x in lists], worst)
        kept += 1
    assert kept >= 16
