"""The device build of mp_md_exact.h (the calibrated, shared- and two-focal MD solvers the
estimator runs, md_exact_kernel, the direct solver entries, and their pose stage
md_pose_exact) against the oracle bit for bit:
random samples, samples whose resultant's roots span many decades, and the full-size
estimator samples where the former Sturm isolation lost or invented roots
(profiles/r04/s6/diag_*.log).  Equal solution lists -- count, order, every double --
so the estimator's per-iteration model counts, and the headline's hypothesis count,
are the oracle's (tests/test_full_size_gpu.py asserts num_hypotheses equality)."""
import ctypes

import numpy as np
import pytest

import madpose
from madpose_amd import _lib as L
from madpose_amd import synthetic
from tests.helpers import oracle_cfg, oracle_opts
from tests.test_md_exact_cpu import DIAG, _oracle, oracle_poses, wide_range_sample

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


_FN = {0: madpose.solve_scale_and_shift, 1: madpose.solve_scale_and_shift_shared_focal,
       2: madpose.solve_scale_and_shift_two_focal}


def _device_poses(v, x, y, dx, dy):
    """mp_solve_scale_shift_pose's models as rows of 17 doubles (the mp_model layout)."""
    c = [np.ascontiguousarray(t, dtype=np.float64) for t in (x, y, dx, dy)]
    out = (L.mp_model * 8)()
    n = L.lib().mp_solve_scale_shift_pose(v, *[t.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) for t in c], out, 8,
                                          0)
    assert n >= 0, n
    raw = np.frombuffer(bytes(out), dtype=np.float64).reshape(8, 17)
    return raw[:n].copy()


def _check(v, x, y, dx, dy):
    got = _FN[v](x.T, y.T, dx, dy)
    a = np.asarray(got, dtype=np.float64).reshape(-1, [4, 5, 6][v])
    b = _oracle(v, x, y, dx, dy)
    assert a.shape == b.shape and np.array_equal(a, b), (v, a, b)
    pa, pb = _device_poses(v, x, y, dx, dy), oracle_poses(v, x, y, dx, dy)
    assert pa.shape == pb.shape and np.array_equal(pa, pb), (v, pa, pb)
    return len(a)


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_device_md_random_bit_exact(variant):
    rng = np.random.default_rng(60 + variant)
    k = 3 if variant == 0 else 4
    total = 0
    for _ in range(600):
        x = np.c_[rng.standard_normal((k, 2)), np.ones(k)]
        y = np.c_[rng.standard_normal((k, 2)), np.ones(k)]
        total += _check(variant, x, y, rng.uniform(0.5, 5, k), rng.uniform(0.5, 5, k))
    assert total > 200


@pytest.mark.parametrize("variant", [0, 1, 2])
def test_device_md_wide_range_bit_exact(variant):
    rng = np.random.default_rng(70 + variant)
    for _ in range(600):
        _check(variant, *wide_range_sample(rng, 3 if variant == 0 else 4))


def test_device_md_diag_samples_bit_exact():
    import oracle
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
        _check(variant, np.c_[a0[idx], np.ones(4)], np.c_[a1[idx], np.ones(4)],
               np.asarray(p["depth0"], float)[idx], np.asarray(p["depth1"], float)[idx])
