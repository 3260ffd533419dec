"""The engine's restated random streams vs libstdc++ (GCC 11) golden streams."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle
from madpose_amd import _lib as L

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rng_gcc11.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def _stream(kind, seed, a, b, count):
    out = np.zeros(count)
    code = L.lib().mp_debug_random_stream(kind, seed, a, b, count, out.ctypes.data_as(L.c_double_p))
    assert code == 0
    return out


def test_raw_mt19937(golden):
    for seed, vals in golden["raw"].items():
        assert np.array_equal(_stream(0, int(seed), 0, 0, len(vals)).astype(np.uint64), np.array(vals, dtype=np.uint64))


def test_uniform_int(golden):
    for key, vals in golden["uint"].items():
        seed, n = (int(v) for v in key.split("_"))
        assert np.array_equal(_stream(1, seed, 0, n - 1, len(vals)).astype(np.int64), np.array(vals)), key


def test_uniform_int_shifted_ranges(golden):
    for seed, vals in golden["uint_ab"].items():
        assert np.array_equal(_stream(3, int(seed), 0, 0, len(vals)).astype(np.int64), np.array(vals)), seed


def test_uniform_real(golden):
    for key, vals in golden["ureal"].items():
        seed, s = key.split("_")
        got = _stream(2, int(seed), 0, int(float(s)), len(vals))
        assert np.array_equal(got, np.array(vals, dtype=np.float64)), key


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("solver_type", [0, 1, 2])
def test_iteration_stream_matches_libstdcxx(variant, solver_type):
    """Solver selection + minimal samples as the reference consumes them, against the
    oracle's std::mt19937 / std::uniform_*_distribution implementation."""
    for seed, n in [(0, 55), (42, 2000), (7, 9)]:
        ot, oi = oracle.iteration_stream(variant, n, seed, solver_type, 700)
        t = np.zeros(700, dtype=np.int32)
        i = np.zeros(8 * 700, dtype=np.int32)
        assert L.lib().mp_debug_iteration_stream(variant, n, seed, solver_type, 700, t.ctypes.data_as(L.c_int32_p),
                                                 i.ctypes.data_as(L.c_int32_p)) == 0
        assert np.array_equal(ot, t)
        assert np.array_equal(oi.ravel(), i)
