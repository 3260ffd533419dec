"""Strict parsing of the MADPOSE_* switches (madpose_amd/csrc/host/env.h): a set value
must parse completely and lie in range, or the engine throws (MP_EINVAL / ValueError).
The header is compiled for the host here; tests/test_switch_invariance_gpu.py checks the
same through the estimator on the GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r"""
#include <cstdio>
#include <cstdlib>
#include "env.h"
int main(int argc, char **argv) {
    const char *kind = argv[1];
    try {
        if (kind[0] == 'i') std::printf("%lld\n", mp::env_int("MP_T", 7, 1, 100));
        else if (kind[0] == 'r') std::printf("%.17g\n", mp::env_real("MP_T", 1.5, 1.0, 1e300));
        else std::printf("%d\n", (int)mp::env_flag("MP_T", true));
    } catch (const std::invalid_argument &e) {
        std::printf("EINVAL %s\n", e.what());
    }
    return 0;
}
"""


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    d = tmp_path_factory.mktemp("env")
    src = d / "env_check.cpp"
    src.write_text(PROG)
    exe = d / "env_check"
    subprocess.run([cxx, "-std=c++17", "-O1", "-I", os.path.join(ROOT, "madpose_amd", "csrc", "host"), str(src),
                    "-o", str(exe)], check=True)
    return str(exe)


def _run(prog, kind, val):
    env = dict(os.environ)
    env.pop("MP_T", None)
    if val is not None:
        env["MP_T"] = val
    return subprocess.run([prog, kind], env=env, capture_output=True, text=True, check=True).stdout.strip()


@pytest.mark.parametrize("kind,val,want", [
    ("i", None, "7"), ("i", "42", "42"), ("i", "100", "100"),
    ("r", None, "1.5"), ("r", "1e7", "10000000"), ("r", "10000000.0", "10000000"),
    ("f", None, "1"), ("f", "0", "0"), ("f", "1", "1"),
])
def test_accepted(prog, kind, val, want):
    assert _run(prog, kind, val) == want


@pytest.mark.parametrize("kind,val", [
    ("i", "4k"), ("i", ""), ("i", "0"), ("i", "101"), ("i", "1.0"), ("i", "99999999999999999999"),
    ("r", "np.float64(4.0)"), ("r", "0.5"), ("r", "nan"), ("r", "inf"), ("r", "1e400"),
    ("f", "off"), ("f", "2"), ("f", "00"), ("f", ""),
])
def test_refused(prog, kind, val):
    out = _run(prog, kind, val)
    assert out.startswith("EINVAL MP_T="), out
