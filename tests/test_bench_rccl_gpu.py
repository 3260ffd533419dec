"""bench.py's result gather through RCCL on the device (configs[4]'s collective, SURVEY.md
§8(e)), exercised on a one-GPU box: MADPOSE_BENCH_DIST=1 makes a fresh bench process
create an `nccl` (= RCCL) process group of one rank before it touches the GPU, and the
per-rank counters and per-pair result records then travel through dist.all_gather on
device tensors -- the same code path the 8-GPU node runs with eight ranks."""
import json
import os
import subprocess
import sys

import pytest

import madpose

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    if madpose.device_count() < 1:
        pytest.fail("no HIP device visible: the GPU tests must run on an MI355X")


def _run(args):
    env = dict(os.environ, MADPOSE_BENCH_DIST="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MADPOSE_BENCH_DIST_BACKEND", "MADPOSE_BENCH_DEVICE",
              "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_one_rank_nccl_gather_of_records():
    out = _run(["--steps", "3", "--warmup", "1", "--cpu-budget", "0", "--in-flight", "1"])
    d = out["dist"]
    assert d["backend"] == "nccl" and d["world_size"] == 1
    # counters + records, both on the device through RCCL
    assert len(d["all_gathers"]) == 2
    assert all(g["backend"] == "nccl" and g["device"].startswith("cuda") for g in d["all_gathers"])
    res = out["results"]
    assert res["records"] == 3 and res["pairs_disjoint"]
    assert res["median_pose_err_deg"] < 1.0
    assert out["n_gpus"] == 1 and out["value"] > 0


def test_one_rank_nccl_scannet_stand_in():
    out = _run(["--workload", "scannet", "--pairs", "6", "--steps", "1", "--warmup", "0", "--cpu-budget", "0",
                "--no-point-only"])
    d = out["dist"]
    assert d["backend"] == "nccl" and len(d["all_gathers"]) == 2
    assert out["results"]["records"] == 6 and out["pose_auc"]["pairs"] == 6
