"""The calibrated, shared- and two-focal MD solvers of mp_md_exact.h and their pose stage
(md_pose_exact: the oracle's Procrustes with its Jacobi SVD) against the oracle, bit for
bit, on the CPU: the header is compiled for the host by clang with FMA
available (-march=x86-64-v3) and contraction off by the header's own pragmas, behind
the C ABI of tests/md_exact_check.cpp.  Equal solution lists (count, order, every
double) for random samples, for samples whose resultant's roots span several orders
of magnitude (the class on which the former Sturm isolation lost or invented roots,
profiles/r04/s6/diag_sf0.log), and for the full-size estimator samples where it did.
The device build of the same header is checked against the oracle in
tests/test_md_exact_gpu.py."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle
from madpose_amd import synthetic
from tests.helpers import oracle_cfg, oracle_opts

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang++"
_dp = ctypes.POINTER(ctypes.c_double)

# (case, seed, iteration sample) of the estimator MD samples whose device solutions
# differed from the oracle's before this solver (profiles/r04/s6/diag_{sf,tf}0.log)
DIAG = [("sf", 0, [824, 451, 1708, 1394]), ("sf", 0, [414, 799, 267, 1502]), ("sf", 0, [1366, 1645, 1374, 1587]),
        ("sf", 0, [236, 1756, 1009, 623]), ("sf", 0, [508, 746, 1379, 36]), ("sf", 0, [200, 1495, 1982, 991]),
        ("sf", 0, [704, 971, 594, 851]), ("tf", 0, [2871, 920, 2581, 2674])]


@pytest.fixture(scope="module")
def mdx(tmp_path_factory):
    if not os.path.exists(CLANG):
        pytest.fail(f"{CLANG} missing: the host build of mp_md_exact.h needs ROCm's clang")
    so = str(tmp_path_factory.mktemp("mdx") / "mdx_check.so")
    cmd = [CLANG, "-O3", "-std=c++17", "-march=x86-64-v3", "-fPIC", "-shared", "-I",
           os.path.join(ROOT, "madpose_amd", "csrc", "include"), os.path.join(ROOT, "tests", "md_exact_check.cpp"),
           "-o", so]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    lib = ctypes.CDLL(so)
    lib.mdx_check_solve.restype = ctypes.c_int
    lib.mdx_check_pose.restype = ctypes.c_int

    def solve(v, x, y, dx, dy):
        a = [np.ascontiguousarray(t, dtype=np.float64) for t in (x, y, dx, dy)]
        out = np.zeros(48)
        n = lib.mdx_check_solve(v, *[t.ctypes.data_as(_dp) for t in a], out.ctypes.data_as(_dp))
        return out[:6 * n].reshape(n, 6)[:, :[4, 5, 6][v]]

    def pose(v, x, y, dx, dy):
        a = [np.ascontiguousarray(t, dtype=np.float64) for t in (x, y, dx, dy)]
        out = np.zeros(8 * 17)
        n = lib.mdx_check_pose(v, *[t.ctypes.data_as(_dp) for t in a], out.ctypes.data_as(_dp))
        return out[:17 * n].reshape(n, 17)
    solve.pose = pose
    solve.so_path = so
    return solve


def _oracle(v, x, y, dx, dy):
    s = np.asarray(oracle.md_scale_shift(v, x, y, dx, dy), dtype=np.float64)
    return s.reshape(-1, [4, 5, 6][v])


def oracle_poses(v, x, y, dx, dy):
    """The oracle's md_pose models as rows of 17 doubles (mp_model layout)."""
    rows = []
    for m in oracle.md_pose(v, x, y, dx, dy):
        f0, f1 = (1.0, 1.0) if v == 0 else (m["focal0"], m["focal1"])
        rows.append(np.r_[m["R"].ravel(), m["t"], m["scale"], m["offset0"], m["offset1"], f0, f1])
    return np.asarray(rows, dtype=np.float64).reshape(-1, 17)


def _check(mdx, v, x, y, dx, dy):
    a, b = mdx(v, x, y, dx, dy), _oracle(v, x, y, dx, dy)
    assert a.shape == b.shape and np.array_equal(a, b), (v, a, b)
    pa, pb = mdx.pose(v, x, y, dx, dy), oracle_poses(v, x, y, dx, dy)
    assert pa.shape == pb.shape and np.array_equal(pa, pb), (v, pa, pb)
    return len(a)


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_random_samples_bit_exact(mdx, variant):
    rng = np.random.default_rng(40 + variant)
    k = 3 if variant == 0 else 4
    total = 0
    for _ in range(3000):
        x = np.c_[rng.standard_normal((k, 2)), np.ones(k)]
        y = np.c_[rng.standard_normal((k, 2)), np.ones(k)]
        total += _check(mdx, variant, x, y, rng.uniform(0.5, 5, k), rng.uniform(0.5, 5, k))
    assert total > 1000  # solutions were found and compared


def wide_range_sample(rng, k):
    """Depths spread over several orders of magnitude and nearly collinear points: the
    resultant's roots then span many decades (the Sturm chain's failure class)."""
    x = np.c_[rng.standard_normal((k, 2)) * 10.0 ** rng.uniform(-3, 1), np.ones(k)]
    y = np.c_[x[:, :2] + rng.standard_normal((k, 2)) * 10.0 ** rng.uniform(-4, 0), np.ones(k)]
    return x, y, 10.0 ** rng.uniform(-2, 3, k), 10.0 ** rng.uniform(-2, 3, k)


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_wide_root_range_bit_exact(mdx, variant):
    rng = np.random.default_rng(50 + variant)
    total = 0
    for _ in range(3000):
        total += _check(mdx, variant, *wide_range_sample(rng, 3 if variant == 0 else 4))
    assert total > 300


def test_estimator_diag_samples_bit_exact(mdx):
    from tests.test_full_size_gpu import CASES
    for name, seed, idx in DIAG:
        variant, kind, cfg, iters = CASES[name]
        p = synthetic.config_pair(cfg, seed=seed)
        o, c = synthetic.throughput_options(kind, iterations=iters)
        cam0, cam1 = p["pp0"], p["pp1"]
        _, _, ns = oracle.score_models(variant, p["x0"], p["x1"], p["depth0"], p["depth1"], cam0, cam1,
                                       oracle_opts(o), oracle_cfg(c), [])
        a0 = (np.asarray(p["x0"], float) - np.asarray(cam0, float).reshape(2)) / ns
        a1 = (np.asarray(p["x1"], float) - np.asarray(cam1, float).reshape(2)) / ns
        idx = np.asarray(idx)
        x = np.c_[a0[idx], np.ones(4)]
        y = np.c_[a1[idx], np.ones(4)]
        _check(mdx, variant, x, y, np.asarray(p["depth0"], float)[idx], np.asarray(p["depth1"], float)[idx])


def test_fast_sv4_matches_exact_form(mdx):
    """smallest_right_sv4_fast (the two-focal recoverPose tests) against the exact
    one-sided Jacobi (dlt_null4's fallback) on DLT-shaped and random 4x4 matrices, host
    build: the same right singular vector up to sign, within 1e-10."""
    lib = ctypes.CDLL(mdx.so_path)
    rng = np.random.default_rng(5)
    for t in range(400):
        if t % 2:
            A = rng.normal(size=(4, 4))
        else:  # rank 3 + noise, as a DLT matrix of a consistent point
            B = rng.normal(size=(4, 3))
            A = B @ rng.normal(size=(3, 4)) + 1e-6 * rng.normal(size=(4, 4))
        a = np.ascontiguousarray(A, dtype=np.float64)
        ve, vf = np.zeros(4), np.zeros(4)
        lib.sv4_check(a.ctypes.data_as(_dp), ve.ctypes.data_as(_dp), vf.ctypes.data_as(_dp))
        s = 1.0 if np.dot(ve, vf) >= 0 else -1.0
        assert np.allclose(ve, s * vf, atol=1e-10), (t, ve, vf)
        sv = np.linalg.svd(A)[2][-1]
        assert abs(abs(np.dot(sv, ve)) - 1.0) < 1e-8, (t, sv, ve)
