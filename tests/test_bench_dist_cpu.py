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
             2000.0 * 1000.0 * (rank + 1), 4.0, 7.0, 3.0, 1.0, 2.0, 400.0, 0.3, 0.4, 900.0, 5000.0, 1.0, 0.5,
             4000.0 * (rank + 1), 8000.0 * (rank + 1), 700.0 * (rank + 1), 900.0 * (rank + 1), 3.0]
    allv = bench.gather_counters(local, world)
    if rank == 0:
        res = bench.summarize(allv, bench.WORKLOADS["cal"], 3, 1, world)
        assert res["dist"]["backend"] == "gloo" and res["dist"]["world_size"] == world
        np.save(out_path, np.array([res["value"], res["n_gpus"], res["pairs_per_s"], res["roofline"]["launches"],
                                    res["ms_per_step"], res["roofline"]["evaluated_frac"],
                                    res["speculation"]["scored_over_accepted"],
                                    res["speculation"]["solved_over_accepted"]]))
    dist.destroy_process_group()


def test_two_rank_gather_and_summary(tmp_path):
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    value, n_gpus, pairs_per_s, launches, ms, evaluated, waste, solved = np.load(out)
    assert n_gpus == 2
    assert value == (1000.0 + 2000.0) / 2.0  # all ranks' hypotheses / slowest rank
    assert pairs_per_s == 2 * 3 / 2.0
    assert launches == 8
    assert abs(ms - 2.0 / 3 * 1e3) < 1e-9
    assert evaluated == 0.5  # (4000 + 8000) / (8000 + 16000)
    assert abs(waste - 2700.0 / 2100.0) < 1e-12  # scored / accepted hypotheses
    assert abs(solved - 3000.0 / 2100.0) < 1e-12  # solved / accepted hypotheses


def test_single_rank_summary_fields():
    sys.path.insert(0, ROOT)
    import bench

    allv = np.array([[2.0, 3e5, 3e5, 30, 1.0, 100.0, 50.0, 3e5, 3e5 * 2000, 30, 90, 10, 5.0, 6.0, 3e5, 1.0, 2.0, 2000.0,
                      5e4, 3, 2.0, 1e6, 2.4e6, 2.5e5, 2.75e5, 1.0]])
    assert allv.shape[1] == len(bench.COUNTERS)
    res = bench.summarize(allv, bench.WORKLOADS["cal"], 3, 1, 1)
    for k in ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]:
        assert k in res
    assert res["scaling"] == "weak" and res["dtype"] == "f64" and res["vs_baseline"] is None
    rf = res["roofline"]
    # achieved: the bytes the early-exit kernel read (the evaluated share of the full
    # figure) over the score time; effective_GBps credits the full figure of the
    # hypotheses that were scored (2.75e5 of 3e5: the rest were record-skipped)
    assert abs(rf["effective_GBps"] - 2.75e5 * 2000 * 48 / 0.1 / 1e9) < 1e-6
    assert abs(rf["achieved"] - 3e5 * 2000 * 48 / 0.1 / 1e9 * 1e6 / 2.4e6) < 1e-6
    assert abs(rf["frac"] - rf["achieved"] / 8000.0) < 1e-12
    assert abs(rf["evaluated_frac"] - 1e6 / 2.4e6) < 1e-12
    assert abs(rf["evaluated_bytes_per_launch"] - 3e5 * 2000 * 48 * (1e6 / 2.4e6) / 30) < 1e-3
    assert abs(res["speculation"]["solved_over_accepted"] - 3e5 / 2.5e5) < 1e-12
    assert abs(res["speculation"]["scored_over_accepted"] - 2.75e5 / 2.5e5) < 1e-12
    # the per-pair breakdown averages the profiled pairs (one of the three here)
    assert res["profiled_pairs"] == 1 and abs(res["ms_per_pair"]["run"] - 2000.0) < 1e-9


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


def _run_bench(args, timeout=600, env_extra=None):
    import json
    import subprocess

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "MADPOSE_BENCH_DIST"):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0])


def test_gpus_flag_spawns_ranks_and_gathers_records():
    """bench.py --gpus 2 with no launcher starts two ranks (gloo on CPU), each estimating
    its own pairs through main()'s sharding path; rank 0 reports n_gpus 2 and the
    gathered per-pair records of both ranks, rank-disjoint."""
    res = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--cpu-budget", "0", "--engine-module",
                      "tests.bench_stub_engine"])
    assert res["n_gpus"] == 2
    assert res["results"]["records"] == 6 and res["results"]["pairs_disjoint"]
    assert res["value"] > 0 and res["scaling"] == "weak"
    # rank 0 pinned itself to its share of this host's CPUs (bench.pin_rank)
    share = res["dist"]["cpu_share"]
    assert share is not None and 1 <= share["cpus"] <= len(os.sched_getaffinity(0))
    assert 1 <= share["lo_threads"] <= 8


def test_cpu_partition_follows_gpu_locality():
    """8 GPUs on a two-socket host (GPUs 0-3 local to socket 0: CPUs 0-31 and their SMT
    siblings 64-95; GPUs 4-7 to socket 1): each rank gets a quarter of its socket's cores,
    siblings kept together, disjoint from every other rank's; without topology all ranks
    split the allowed CPUs."""
    sys.path.insert(0, ROOT)
    import bench

    sock = [list(range(0, 32)) + list(range(64, 96)), list(range(32, 64)) + list(range(96, 128))]
    local = [sock[0]] * 4 + [sock[1]] * 4
    core_of = {c: c % 64 for c in range(128)}
    parts = bench.partition_cpus(local, range(128), core_of, list(range(8)))
    seen = set()
    for r, cpus in enumerate(parts):
        assert len(cpus) == 16
        assert set(cpus) <= set(sock[r // 4])
        assert {core_of[c] for c in cpus} == {core_of[c] for c in cpus if c < 64}  # whole cores
        assert not (seen & set(cpus))
        seen |= set(cpus)
    # a restricted allowed set (a container's share): the intersection is split
    parts = bench.partition_cpus(local, range(16, 48), core_of, list(range(8)))
    assert all(parts[r] and set(parts[r]) <= set(range(16, 32)) for r in range(4))
    assert all(parts[r] and set(parts[r]) <= set(range(32, 48)) for r in range(4, 8))
    # no topology, or two ranks on one device (the one-card rehearsal)
    parts = bench.partition_cpus(None, range(8), {c: c for c in range(8)}, [0, 1])
    assert parts == [[0, 1, 2, 3], [4, 5, 6, 7]]
    parts = bench.partition_cpus(local, range(128), core_of, [0, 0])
    assert len(parts[0]) == len(parts[1]) == 32 and not set(parts[0]) & set(parts[1])
    assert bench.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]


def test_gpus_flag_scannet_shards_all_pairs():
    res = _run_bench(["--gpus", "2", "--workload", "scannet", "--pairs", "9", "--steps", "1", "--warmup", "0",
                      "--cpu-budget", "0", "--engine-module", "tests.bench_stub_engine"])
    assert res["n_gpus"] == 2 and res["config"]["pairs"] == 9
    assert res["results"]["records"] == 9 and res["results"]["pairs_disjoint"]
    assert res["pose_auc"]["pairs"] == 9
    assert res["point_only_baseline"]["pose_auc"]["pairs"] == 9


def test_gpus_mismatch_fails_loudly():
    import subprocess

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--engine-module",
                        "tests.bench_stub_engine"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_scannet_sharding_is_a_balanced_partition():
    sys.path.insert(0, ROOT)
    import bench
    from madpose_amd import synthetic

    total, world = 1500, 8
    parts = [bench.shard_scannet(total, world, r) for r in range(world)]
    allp = sorted(s for p in parts for s in p)
    assert allp == list(range(total))
    loads = [sum(synthetic.scannet_size(s) for s in p) for p in parts]
    assert max(loads) - min(loads) <= 2500  # LPT: within one pair of each other


def test_records_summary_and_gather_single_rank():
    sys.path.insert(0, ROOT)
    import bench

    w = len(bench.RECORD_FIELDS)
    recs = [[float(s)] + [0.0] * (w - 3) + [float(s), 2.0 * s] for s in range(4)]
    allr = bench.gather_records(recs, 6, 1)
    assert allr.shape == (4, w)
    s = bench.records_summary(allr)
    assert s["records"] == 4 and s["pairs_disjoint"] and s["median_pose_err_deg"] == np.median([0, 2, 4, 6])


def test_single_rank_in_flight_leg_and_records():
    """One rank: the pairs-in-flight secondary figure (estimate_batch k at a time) sits
    beside `value` without replacing it, and the records carry the engine's pose errors."""
    res = _run_bench(["--steps", "4", "--warmup", "1", "--cpu-budget", "0", "--in-flight", "3", "--engine-module",
                      "tests.bench_stub_engine"])
    assert res["n_gpus"] == 1 and res["value"] > 0
    pf = res["pairs_in_flight"]
    assert pf["pairs"] == 4 and pf["in_flight"] == 3 and pf["hypotheses_per_s"] > 0
    assert res["results"]["records"] == 4
    # the stub returns R = I, t = (1, 0, 0): its pose errors come from compute_pose_error
    assert res["results"]["median_pose_err_deg"] >= 0.0


def test_forced_one_rank_group_gathers_through_the_collective():
    """MADPOSE_BENCH_DIST=1 (the one-GPU rehearsal of the RCCL gather): one rank still
    creates a process group (gloo here) and its counters and records go through
    dist.all_gather."""
    res = _run_bench(["--steps", "2", "--warmup", "1", "--cpu-budget", "0", "--in-flight", "1", "--engine-module",
                      "tests.bench_stub_engine"], env_extra={"MADPOSE_BENCH_DIST": "1"})
    d = res["dist"]
    assert d["backend"] == "gloo" and d["world_size"] == 1
    assert len(d["all_gathers"]) == 2
    assert res["results"]["records"] == 2


def test_cpu_partition_one_l3_domain_per_rank():
    """A two-socket host with 16 CCDs of 8 cores (CPU c and c + 128 are SMT siblings,
    CCD = c // 8 of the core): a single rank gets one whole CCD with its siblings (the
    last one); 8 ranks without GPU locality get 8 distinct CCDs spread over the host; 20
    ranks (more than the domains) fall back to splitting whole cores."""
    sys.path.insert(0, ROOT)
    import bench

    cpus = list(range(256))
    core_of = {c: c % 128 for c in cpus}
    l3_of = {c: (c % 128) // 8 * 8 for c in cpus}
    one = bench.partition_cpus(None, cpus, core_of, [0], l3_of)[0]
    assert one == list(range(120, 128)) + list(range(248, 256))  # the last CCD
    parts = bench.partition_cpus(None, cpus, core_of, list(range(8)), l3_of)
    doms = [{l3_of[c] for c in p} for p in parts]
    assert all(len(d) == 1 and len(p) == 16 for d, p in zip(doms, parts))
    assert len({next(iter(d)) for d in doms}) == 8
    assert {next(iter(d)) for d in doms} == {120 - 16 * j for j in range(8)}  # every other CCD from the top
    parts = bench.partition_cpus(None, cpus, core_of, list(range(20)), l3_of)
    seen = set()
    for p in parts:
        assert p and not set(p) & seen
        seen |= set(p)


def test_gpu_local_cpus_skips_nodes_it_may_not_open(tmp_path, monkeypatch):
    """The pool's boxes let a process open only its own GPU's KFD node (the others raise
    EPERM, profiles/r05/topo.log): those are skipped, not a reason to give up on
    locality; a CPU node (simd_count 0) is skipped; a GPU whose PCI locality is missing
    gets an empty list (every allowed CPU)."""
    sys.path.insert(0, ROOT)
    import bench

    kfd, pci = tmp_path / "nodes", tmp_path / "pci"
    for k, props in {0: "cpu_cores_count 128\nsimd_count 0\n", 1: None,
                     2: "simd_count 1024\nlocation_id 56320\ndomain 0\n",
                     3: "simd_count 1024\nlocation_id 4096\ndomain 0\n"}.items():
        (kfd / str(k)).mkdir(parents=True)
        if props is None:
            (kfd / str(k) / "properties").mkdir()  # opening a directory raises an OSError
        else:
            (kfd / str(k) / "properties").write_text(props)
    (pci / "0000:dc:00.0").mkdir(parents=True)
    (pci / "0000:dc:00.0" / "local_cpulist").write_text("64-66,192\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert bench.gpu_local_cpus(str(kfd), str(pci)) == [[64, 65, 66, 192], []]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert bench.gpu_local_cpus(str(kfd), str(pci)) == [[]]
