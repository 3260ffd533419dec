"""The multi-rank plumbing of bench.py on CPU (gloo, world size 2): pairs are sharded
per rank with no data-path collective; the only exchange is the final all_gather of
per-rank counters, and rank 0 reports all ranks' work over the slowest rank's time."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r: elapsed 1 + r seconds, 1000 * (r + 1) hypotheses, ...
    local = [1.0 + rank, 1000.0 * (rank + 1), 500.0, 2.0, 0.5, 10.0, 5.0, 1000.0 * (rank + 1),
             2000.0 * 1000.0 * (rank + 1), 4.0, 7.0, 3.0, 1.0, 2.0, 400.0, 0.3, 0.4, 900.0, 5000.0, 1.0, 0.5]
    allv = bench.gather_counters(local, world)
    if rank == 0:
        res = bench.summarize(allv, bench.WORKLOADS["cal"], 3, 1, world)
        np.save(out_path, np.array([res["value"], res["n_gpus"], res["pairs_per_s"], res["roofline"]["launches"],
                                    res["ms_per_step"]]))
    dist.destroy_process_group()


def test_two_rank_gather_and_summary(tmp_path):
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    value, n_gpus, pairs_per_s, launches, ms = np.load(out)
    assert n_gpus == 2
    assert value == (1000.0 + 2000.0) / 2.0  # all ranks' hypotheses / slowest rank
    assert pairs_per_s == 2 * 3 / 2.0
    assert launches == 8
    assert abs(ms - 2.0 / 3 * 1e3) < 1e-9


def test_single_rank_summary_fields():
    sys.path.insert(0, ROOT)
    import bench

    allv = np.array([[2.0, 3e5, 3e5, 30, 1.0, 100.0, 50.0, 3e5, 3e5 * 2000, 30, 90, 10, 5.0, 6.0, 3e5, 1.0, 2.0, 2000.0,
                      5e4, 3, 2.0]])
    assert allv.shape[1] == len(bench.COUNTERS)
    res = bench.summarize(allv, bench.WORKLOADS["cal"], 3, 1, 1)
    for k in ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]:
        assert k in res
    assert res["scaling"] == "weak" and res["dtype"] == "f64" and res["vs_baseline"] is None
    rf = res["roofline"]
    assert abs(rf["achieved"] - 3e5 * 2000 * 48 / 0.1 / 1e9) < 1e-6
    assert abs(rf["frac"] - rf["achieved"] / 8000.0) < 1e-12


def test_scannet_summary_and_gathered_errors():
    """configs[4] record: pairs/s of all ranks over the slowest rank (strong scaling);
    AUC over every rank's per-pair errors, padding (NaN) dropped."""
    sys.path.insert(0, ROOT)
    import bench
    from madpose_amd import utils

    allv = np.array([[2.0, 10.0, 500.0, 900.0], [4.0, 9.0, 400.0, 800.0]])
    errs = np.array([1.0, 3.0, 30.0, 2.0, 7.0, np.nan])
    res = bench.summarize_scannet(allv, errs, bench.WORKLOADS["scannet"], 1, 0, 2, 19)
    assert res["value"] == 19.0 / 4.0 and res["unit"] == "pairs/s" and res["scaling"] == "strong"
    assert res["pose_auc"]["pairs"] == 5
    ref = utils.pose_auc(errs[:5], (5, 10, 20))
    assert [res["pose_auc"][k] for k in ("5", "10", "20")] == ref
