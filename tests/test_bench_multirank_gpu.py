"""bench.py's multi-rank path on the GPU: `--gpus 2` spawns two rank
processes that run the real HIP engine, shard the pairs and gather the per-pair result
records. A one-GPU box cannot give each rank its own device and RCCL refuses two ranks on
one device, so this rehearsal puts both ranks on device 0 with the gloo backend
(MADPOSE_BENCH_DEVICE, MADPOSE_BENCH_DIST_BACKEND); on the 8-GPU node the same code runs
one rank per device over RCCL."""
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
    env = dict(os.environ, MADPOSE_BENCH_DEVICE="0", MADPOSE_BENCH_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_two_ranks_shard_pairs_and_gather_records():
    out = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--cpu-budget", "0", "--in-flight", "1"])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak"
    res = out["results"]
    assert res["records"] == 2 * 3 and res["pairs_disjoint"]
    assert res["median_pose_err_deg"] < 1.0  # synthetic pairs: the estimates are close to the ground truth
    assert out["value"] > 0


def test_two_ranks_scannet_stand_in():
    out = _run(["--gpus", "2", "--workload", "scannet", "--pairs", "12", "--steps", "1", "--warmup", "0",
                "--cpu-budget", "0", "--no-point-only"])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["results"]["records"] == 12 and out["results"]["pairs_disjoint"]
    assert out["pose_auc"]["pairs"] == 12 and 0.0 <= out["pose_auc"]["5"] <= 1.0
