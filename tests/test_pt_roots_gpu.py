"""The point solvers' root stages against the oracle on hard samples.

The calibrated 5-point root stage (kernels/group_5pt.h + group_bisect.h: the estimator's
stage, through mp_debug_pt_roots) performs the oracle's restatement of PoseLib
relpose_5pt (oracle/src/pt_poselib.cpp: Householder null space, Nister's template,
Gauss-Jordan, det B(z), PoseLib's Sturm bisection + Ridders + Newton) operation for
operation without FMA contraction, so its essential matrices must equal the oracle's in
count, order and every bit.  The two-focal 7-point stage (mp_pt67.h relpose_7pt_F: the
Householder null space, the cubic, PoseLib's closed-form solve_cubic_real) decides its
root count with +, -, *, / only, so the counts must be equal; cbrt / acos / cos come
from the device and host math libraries, so the matrices agree to 1e-9 (unit norm).

Samples (tests/pt_samples.py), 10000 of each kind per solver: random scenes (noise-free
and noisy), outlier-contaminated samples, wide-range samples (fields of view, depths and
baselines over decades), and near-double-root samples bisected onto the parameter where
the oracle's real-root count changes.  Reference: /root/reference/src/
hybrid_pose_estimator.cpp:121-185 (5pt), hybrid_pose_two_focal_estimator.cpp:103-182
(7pt), hybrid_ransac.h:123-135."""
import ctypes
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import oracle  # noqa: E402
import pt_samples as ps  # noqa: E402
from madpose_amd import _lib as L  # noqa: E402

pytestmark = pytest.mark.gpu

NS = 10000
KINDS = ["random", "outlier", "wide", "neardouble"]


def _device_roots(variant, impl, p0, p1):
    ns = p0.shape[0]
    cand = np.zeros((ns, 96))
    ncand = np.zeros(ns, dtype=np.int32)
    dp = lambda a: np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    L.check(L.lib().mp_debug_pt_roots(variant, impl, ns, dp(p0), dp(p1),
                                      cand.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                      ncand.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), 0))
    return cand, ncand


def _count5(p0, p1):
    return len(oracle.relpose_5pt_E(ps.bearings(p0), ps.bearings(p1))[1])


def _count7(p0, p1):
    return len(oracle.relpose_7pt(ps.bearings(p0), ps.bearings(p1)))


@pytest.fixture(scope="module")
def samples5():
    return ps.all_kinds(61, NS, 5, _count5)


@pytest.fixture(scope="module")
def samples7():
    return ps.all_kinds(67, NS, 7, _count7)


@pytest.mark.parametrize("kind", KINDS)
def test_5pt_root_stage_is_the_oracles_to_the_bit(samples5, kind):
    p0, p1 = samples5[kind]
    cand, ncand = _device_roots(0, 1, p0, p1)
    b0, b1 = ps.bearings(p0), ps.bearings(p1)
    count_diff, bit_diff, hist = [], [], np.zeros(11, dtype=int)
    for s in range(len(p0)):
        E, _ = oracle.relpose_5pt_E(b0[s], b1[s])
        hist[min(len(E), 10)] += 1
        if ncand[s] != len(E):
            count_diff.append((s, int(ncand[s]), len(E)))
            continue
        dev = cand[s, : 9 * len(E)].reshape(-1, 3, 3)
        if not np.array_equal(dev, E):
            bit_diff.append((s, float(np.abs(dev - E).max())))
    print(f"{kind}: essential-matrix counts {hist.tolist()}")
    assert not count_diff, (kind, len(count_diff), count_diff[:5])
    assert not bit_diff, (kind, len(bit_diff), bit_diff[:5])


@pytest.mark.parametrize("kind", KINDS)
def test_7pt_root_stage_matches_the_oracle(samples7, kind):
    p0, p1 = samples7[kind]
    cand, ncand = _device_roots(2, 1, p0, p1)
    b0, b1 = ps.bearings(p0), ps.bearings(p1)
    count_diff, worst, nbits = [], 0.0, 0
    for s in range(len(p0)):
        F = oracle.relpose_7pt(b0[s], b1[s])
        if ncand[s] != len(F):
            count_diff.append((s, int(ncand[s]), len(F)))
            continue
        dev = cand[s, : 9 * len(F)].reshape(-1, 3, 3)
        fin = np.isfinite(F)
        assert np.array_equal(np.isfinite(dev), fin), s
        if len(F):
            worst = max(worst, float(np.abs(dev[fin] - F[fin]).max()) if fin.any() else 0.0)
            nbits += int(np.array_equal(dev[fin], F[fin]))
    print(f"{kind}: max |F_dev - F_oracle| = {worst:.3g}, bit-identical on {nbits} of {len(p0)}")
    assert not count_diff, (kind, len(count_diff), count_diff[:5])
    assert worst <= 1e-9, (kind, worst)


def test_standalone_5pt_runs_the_estimators_root_stage():
    """mp_relpose_5pt (the C ABI's standalone solver) is the estimator's root stage plus
    motion_from_essential: its pose count equals the oracle's on the same bearings and
    every oracle pose has a device pose within 1e-9."""
    import madpose

    rng = np.random.default_rng(5)
    p0, p1 = ps.random_samples(rng, 300, 5)
    for s in range(len(p0)):
        b0, b1 = ps.bearings(p0[s]), ps.bearings(p1[s])
        dev = madpose.relpose_5pt(b0, b1)
        ref = oracle.relpose_5pt(b0, b1)
        assert len(dev) == len(ref), s
        for m in ref:
            assert min(np.abs(d.R() - m["R"]).max() + np.abs(d.t() - m["t"]).max() for d in dev) <= 1e-9, s


def test_6pt_root_stage_is_independent_of_the_packing():
    """The shared-focal QR runs one sample per wave at <= 1024 samples (the window state
    scalar: columns and rows outside the active window skipped by scalar branches) and
    several samples per wave above (the whole band updated, windows by selects).  Both
    perform the same operations on every entry inside the window, and entries outside
    it are never read again, so a sample's candidates must not depend on the launch:
    the same 600 samples alone (one per wave), inside 3000 (three per wave) and inside
    6000 (six per wave) give the same bits."""
    rng = np.random.default_rng(71)
    r0, r1 = ps.random_samples(rng, 3000, 6)
    o0, o1 = ps.outlier_samples(rng, 1500, 6)
    w0, w1 = ps.wide_samples(rng, 1500, 6)
    p0, p1 = np.concatenate([r0[:300], o0[:150], w0[:150], r0[300:], o0[150:], w0[150:]]), \
        np.concatenate([r1[:300], o1[:150], w1[:150], r1[300:], o1[150:], w1[150:]])
    c6k, n6k = _device_roots(1, 3, p0, p1)
    c3k, n3k = _device_roots(1, 3, p0[:3000], p1[:3000])
    c600, n600 = _device_roots(1, 3, p0[:600], p1[:600])
    assert n600.sum() > 600, n600.sum()
    for c, n, m in ((c3k, n3k, 600), (c6k, n6k, 600), (c6k, n6k, 3000)):
        ref_c, ref_n = (c600, n600) if m == 600 else (c3k, n3k)
        assert np.array_equal(n[:m], ref_n[:m]), m
        diff = np.nonzero(~np.all((c[:m] == ref_c[:m]) | (np.isnan(c[:m]) & np.isnan(ref_c[:m])), axis=1))[0]
        assert diff.size == 0, (m, diff[:10])
