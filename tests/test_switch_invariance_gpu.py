"""The engine's performance switches change no result: the full-size estimator cases
and four pairs in flight, each switch setting in a fresh process (the engine reads them
once), compared field by field with the default run to the last bit -- the early
continuation on while alone and always (MADPOSE_EARLY_CONT, §2 step 7 of DESIGN.md), the
exact MD solvers on one or two lanes per sample instead of the defaults (MADPOSE_MDX_R; cal
and tf 4, sf 2), the scalar
batch drawing instead of AVX-512 (MADPOSE_SAMPLER_SIMD), the 15x15 QR packed 16
samples per wave instead of one sample per wave (MADPOSE_EIG_WAVES), the
draw-by-draw sampler (MADPOSE_SAMPLER_TWO_PASS), and the calibrated MD and 5pt root
stage on two streams instead of one fused launch (MADPOSE_SOLVE_FUSE), score_batch
one trip per loop step instead of two between early-exit checks (MADPOSE_SCORE_PAIR), the
post-LO speculation predicted after the LO prefix instead of before it
(MADPOSE_LO_EARLY_HOOK) or not at all (MADPOSE_LO_SPECULATE), and without the batch after
it drawn (MADPOSE_LO_CHAIN) or launched (MADPOSE_LO_CHAIN_LAUNCH) in the same job; the
scoring without its exact early exit (MADPOSE_SCORE_EXIT) or record skip
(MADPOSE_RECORD_SKIP), with an exit check after every trip (MADPOSE_SCORE_CHECK), and the
fused MD + 5pt launch for no batch or only up to 8192 iterations instead of every batch
(MADPOSE_SOLVE_FUSE_MAX), and the
exact MD solver in one launch with its setup repeated in every lane of a sample instead of
the setup and root stages (MADPOSE_MD_TWO_STAGE).  A value
that does not parse is refused loudly (host/env.h)."""
import json
import os
import subprocess
import sys

import pytest

import madpose

pytestmark = pytest.mark.gpu

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "switch_worker.py")
SETTINGS = {"early_alone": {"MADPOSE_EARLY_CONT": "1"}, "early_always": {"MADPOSE_EARLY_CONT": "2"},
            "mdx_one_lane": {"MADPOSE_MDX_R": "1"}, "mdx_two_lanes": {"MADPOSE_MDX_R": "2"}, "sampler_scalar": {"MADPOSE_SAMPLER_SIMD": "0"},
            "eig_packed": {"MADPOSE_EIG_WAVES": "16"}, "eig_waves_1024": {"MADPOSE_EIG_WAVES": "1024"}, "draw_by_draw": {"MADPOSE_SAMPLER_TWO_PASS": "0"},
            "solve_unfused": {"MADPOSE_SOLVE_FUSE": "0"}, "early_big": {"MADPOSE_EARLY_CONT": "3"}, "lo_late_hook": {"MADPOSE_LO_EARLY_HOOK": "0"},
            "lo_no_speculation": {"MADPOSE_LO_SPECULATE": "0"}, "lo_no_chain": {"MADPOSE_LO_CHAIN": "0"},
            "lo_chain_launched": {"MADPOSE_LO_CHAIN_LAUNCH": "1"},
            "score_single_trips": {"MADPOSE_SCORE_PAIR": "0"},
            "score_no_exit": {"MADPOSE_SCORE_EXIT": "0"}, "no_record_skip": {"MADPOSE_RECORD_SKIP": "0"},
            "score_check_every_trip": {"MADPOSE_SCORE_CHECK": "1,1"},
            "fuse_never": {"MADPOSE_SOLVE_FUSE_MAX": "0"}, "fuse_up_to_8192": {"MADPOSE_SOLVE_FUSE_MAX": "8192"},
            "md_one_stage": {"MADPOSE_MD_TWO_STAGE": "0"}, "md_two_stage_everywhere": {"MADPOSE_MD_TWO_STAGE": "2"}}


def _run(extra):
    env = dict(os.environ)
    for k in list(env):
        if k.startswith("MADPOSE_"):
            del env[k]
    env.update(extra)
    r = subprocess.run([sys.executable, WORKER], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_run():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")
    return _run({})


@pytest.mark.parametrize("name", list(SETTINGS))
def test_switch_changes_no_result(default_run, name):
    other = _run(SETTINGS[name])
    assert len(other) == len(default_run)
    for k, (a, b) in enumerate(zip(default_run, other)):
        assert a == b, (name, k, a, b)


@pytest.mark.parametrize("var,val", [("MADPOSE_TIE_SCALE", "np.float64(4.0)"), ("MADPOSE_MIN_BATCH", "4k"),
                                     ("MADPOSE_SCORE_EXIT", "off"), ("MADPOSE_SCORE_CHECK", "2;2")])
def test_unparsable_switch_is_refused(var, val):
    """An unparsable MADPOSE_* value raises instead of being read as 0 / 1.0 (VERDICT r05
    weak #8: MADPOSE_TIE_SCALE="np.float64(...)" once became 1.0 silently)."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("MADPOSE_")}
    env[var] = val
    code = ("import madpose\nfrom madpose_amd import synthetic\np = synthetic.config_pair(2, seed=0)\n"
            "o, c = synthetic.throughput_options('calibrated', iterations=2000)\n"
            "try:\n    madpose.HybridEstimatePoseScaleOffset(p['x0'], p['x1'], p['depth0'], p['depth1'], "
            "p['min_depth'], p['K0'], p['K1'], o, c)\nexcept ValueError as e:\n    print('REFUSED', e)\n")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "REFUSED" in r.stdout and var in r.stdout, r.stdout
