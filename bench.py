"""Throughput bench of the MI355X hybrid-RANSAC engine (BASELINE.json metric).

A step is one full HybridEstimatePoseScaleOffset run (solver batches, GPU scoring
sweep, host LO, termination) over one synthetic pair of BASELINE.json configs[1]:
calibrated, N = 2000 correspondences, 100k iterations (min = max = per-solver cap, so
the adaptive bound never stops early).  Every rank runs its own pairs (weak scaling);
the only collective is the final gather of per-rank counters.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cal|sf|tf|scannet]

--workload scannet runs configs[4] instead: a fixed set of 1500 shared-focal pairs
split over the ranks, many pairs in flight per GPU; value = pairs/s, plus pose
AUC@5/10/20 over all pairs.

Prints ONE JSON line on rank 0.  `value` = hypotheses scored per second by the whole
job; `roofline` prices the score_batch kernel at the algorithmic 48*N bytes per
hypothesis against its HIP-event device time; `cpu_baseline` times the CPU oracle
(test infrastructure, a scalar restatement of the reference) on a bounded sample of
the same pair.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md (HBM3E spec peak)
BYTES_PER_CORR = 48    # x0u, x0v, x1u, x1v, d0, d1 in FP64

WORKLOADS = {
    "cal": dict(kind="calibrated", variant=0, config=2, n=2000, iterations=100000,
                name="configs[1]: calibrated solver, 1 pair, 2000 synthetic correspondences, 100k hypotheses"),
    "sf": dict(kind="shared_focal", variant=1, config=3, n=2000, iterations=100000,
               name="configs[2]: shared-focal solver, 2000 synthetic correspondences, 100k hypotheses"),
    "tf": dict(kind="two_focal", variant=2, config=4, n=4000, iterations=200000,
               name="configs[3]: two-focal solver, 4000 synthetic correspondences, 200k hypotheses"),
    # configs[4]: a fixed set of pairs split over the ranks (strong scaling), many pairs
    # in flight per GPU (host workers x HIP streams, mp_estimate_batch)
    "scannet": dict(kind="shared_focal", variant=1, config="scannet", n=2000, iterations=1000, pairs=1500,
                    name="configs[4]: ScanNet-1500 stand-in, 1500 synthetic shared-focal pairs "
                         "(N ~ U{1500..2500}), example options (100..1000 iterations), pairs split over the ranks"),
}


def _pair_args(p, variant):
    if variant == 0:
        return (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["K0"], p["K1"])
    return (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], p["K0"][:2, 2], p["K1"][:2, 2])


def _estimate(madpose, variant, args, o, c, device):
    fn = [madpose.HybridEstimatePoseScaleOffset, madpose.HybridEstimatePoseScaleOffsetSharedFocal,
          madpose.HybridEstimatePoseScaleOffsetTwoFocal][variant]
    return fn(*args, o, c, device=device)


def cpu_baseline(wl, pair, budget_s=15.0):
    """Scalar CPU oracle (kind "port") on a bounded iteration count of the same pair."""
    try:
        import oracle
        from tests.helpers import oracle_cfg, oracle_opts
        from madpose_amd import synthetic
    except Exception as e:  # the oracle is test infrastructure; its absence must not break the bench
        return {"value": None, "unit": "hypotheses/s", "cores": 1, "kind": "port", "sample": f"unavailable: {e}"}
    args = _pair_args(pair, wl["variant"])
    it = 500
    while True:
        o, c = synthetic.throughput_options(wl["kind"], iterations=it)
        t0 = time.perf_counter()
        _, st, _ = oracle.estimate(wl["variant"], *args, oracle_opts(o), oracle_cfg(c))
        dt = time.perf_counter() - t0
        if dt >= budget_s / 3 or it >= wl["iterations"]:
            break
        it = min(wl["iterations"], int(it * max(2.0, budget_s / max(dt, 1e-3))))
    return {"value": st.num_hypotheses / dt, "unit": "hypotheses/s", "cores": 1, "kind": "port",
            "sample": f"same pair, {it} iterations (min=max=per-solver cap), single thread, {dt:.1f} s, "
                      f"{st.num_hypotheses} hypotheses, {st.number_lo_iterations} LO runs"}


def pmc_traffic_model():
    """Latest committed PMC fit (profiles/r*/pmc_score_batch.json): memory-side read
    bytes of one score_batch launch = fixed + per_iteration x iterations."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_score_batch.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        m = json.load(f)
    m["file"] = os.path.relpath(files[-1], ROOT)
    return m


COUNTERS = ["elapsed_s", "hypotheses", "iterations", "lo_runs", "lo_s", "score_ms", "solve_ms", "prof_hypotheses",
            "prof_correspondences", "prof_batches", "prof_sweeps", "lm_calls", "lm_ms", "sweep_ms", "prof_iterations",
            "sample_ms", "wait_ms", "run_ms", "lm_blocks", "lm_big_calls", "lm_big_ms"]


def gather_counters(local, world):
    """All ranks' counter vectors (world x len(COUNTERS)) -- the only collective of the
    bench: one all_gather of a few doubles per rank (RCCL on GPUs, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor(local, dtype=torch.float64)
    if world == 1:
        return t.numpy()[None]
    out = [torch.zeros_like(t) for _ in range(world)]
    if dist.get_backend() == "nccl":
        gl = [g.cuda() for g in out]
        dist.all_gather(gl, t.cuda())
        out = [g.cpu() for g in gl]
    else:
        dist.all_gather(out, t)
    return torch.stack(out).numpy()


def summarize(allv, wl, steps, warmup, world):
    """Whole-job JSON record from the gathered counters: value = all ranks' hypotheses
    divided by the slowest rank's wall time (weak scaling)."""
    c = {k: allv[:, i] for i, k in enumerate(COUNTERS)}
    t_max = float(c["elapsed_s"].max())
    score_ms = float(c["score_ms"].sum())
    achieved = float(c["prof_correspondences"].sum()) * BYTES_PER_CORR / (score_ms * 1e-3) / 1e9 if score_ms > 0 else 0.0
    launches = int(c["prof_batches"].sum())
    traffic, traffic_note = None, None
    tm = pmc_traffic_model()
    if tm is not None and launches > 0:
        it_per_launch = float(c["prof_iterations"].sum()) / launches
        traffic = tm["fetch_bytes_fixed_per_launch"] + tm["fetch_bytes_per_iteration"] * it_per_launch
        traffic_note = (f"bytes per launch from the FETCH_SIZE fit in {tm['file']} ({tm['correction']}) at "
                        f"{it_per_launch:.0f} iterations per launch; algorithmic bytes per launch "
                        f"{float(c['prof_correspondences'].sum()) * BYTES_PER_CORR / launches:.3g}: the pair's "
                        f"arrays stay L2-resident across the workgroups of a launch")
    return {
        "metric": "RANSAC hypotheses/sec + image-pairs/sec on 1xMI355X",
        "value": float(c["hypotheses"].sum()) / t_max,
        "unit": "hypotheses/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": t_max / steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded pairs per SURVEY.md §8d; no datasets on the box)",
        "config": {"workload": wl["name"], "n_correspondences": wl["n"], "iterations": wl["iterations"],
                   "pairs_per_step_per_gpu": 1, "parallelism": f"pairs sharded over {world} rank(s)"},
        "pairs_per_s": world * steps / t_max,
        "iterations_per_s": float(c["iterations"].sum()) / t_max,
        "lo_runs": int(c["lo_runs"].sum()),
        "lo_share": float(c["lo_s"].sum() / c["elapsed_s"].sum()),
        "lo_breakdown": {"lm_calls": int(c["lm_calls"].sum()), "lm_ms": float(c["lm_ms"].sum()),
                         "lm_blocks": int(c["lm_blocks"].sum()), "lm_big_calls": int(c["lm_big_calls"].sum()),
                         "lm_big_ms": float(c["lm_big_ms"].sum()),
                         "sweeps": int(c["prof_sweeps"].sum()), "sweep_ms": float(c["sweep_ms"].sum())},
        # where one pair's wall time goes (host clocks; GPU solve/score from HIP events)
        "ms_per_pair": {k: float(c[src].sum()) / (world * steps) for k, src in
                        [("run", "run_ms"), ("batch_wait", "wait_ms"), ("sampling", "sample_ms"), ("lm", "lm_ms"),
                         ("lo_sweeps", "sweep_ms"), ("gpu_solve", "solve_ms"), ("gpu_score", "score_ms")]},
        "roofline": {
            "bound": "hbm",
            "kernel": "score_batch_kernel",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_note": traffic_note,
            "launches": launches,
            "avg_launch_us": score_ms * 1e3 / max(launches, 1),
            "bytes_per_hypothesis": BYTES_PER_CORR * wl["n"],
            "solve_ms_per_launch": float(c["solve_ms"].sum()) / max(launches, 1),
        },
        "cpu_baseline": None,
    }


def pair_errors(results, pairs):
    """max(rotation error, translation angle error) in degrees per pair
    (madpose/utils.py:70-78 compute_pose_error), the quantity pose AUC integrates."""
    from madpose_amd import utils

    return [max(utils.compute_pose_error(p["T_0to1"], m.R(), m.t())) for (m, _), p in zip(results, pairs)]


def summarize_scannet(allv, errs, wl, steps, warmup, world, total):
    """Whole-job record of the ScanNet-1500 stand-in: value = pairs per second of all
    ranks over the slowest rank's time (total work fixed: strong scaling); AUC@5/10/20
    over the per-pair errors of every rank."""
    from madpose_amd import utils

    t_max = float(allv[:, 0].max())
    done = float(allv[:, 1].sum())
    e = np.asarray(errs, dtype=np.float64)
    e = e[np.isfinite(e)]
    auc = utils.pose_auc(e, (5, 10, 20)) if len(e) else [None] * 3
    return {
        "metric": "image-pairs/sec on 1xMI355X (ScanNet-1500 stand-in) + pose AUC@5/10/20",
        "value": done / t_max,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": t_max / steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded shared-focal pairs per SURVEY.md §8d config 5; no datasets on the box)",
        "config": {"workload": wl["name"], "pairs": total, "iterations": wl["iterations"],
                   "parallelism": f"pairs split over {world} rank(s)"},
        "hypotheses_per_s": float(allv[:, 2].sum()) / t_max,
        "iterations_per_s": float(allv[:, 3].sum()) / t_max,
        "pose_auc": {"5": auc[0], "10": auc[1], "20": auc[2], "pairs": int(len(e))},
        "cpu_baseline": None,
    }


def cpu_baseline_pairs(wl, pairs, budget_s):
    """The scalar CPU oracle on as many of the rank's pairs as fit in budget_s."""
    try:
        import oracle
        from tests.helpers import oracle_cfg, oracle_opts
        from madpose_amd import synthetic
    except Exception as e:
        return {"value": None, "unit": "pairs/s", "cores": 1, "kind": "port", "sample": f"unavailable: {e}"}
    o, c = synthetic.example_options(wl["kind"], iterations=wl["iterations"])
    t0 = time.perf_counter()
    k = 0
    for p in pairs:
        oracle.estimate(wl["variant"], *_pair_args(p, wl["variant"]), oracle_opts(o), oracle_cfg(c))
        k += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": k / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"first {k} pairs of the set, single thread, {dt:.1f} s"}


def run_scannet(a, wl, world, rank, dev, barrier):
    import madpose_amd as madpose
    from madpose_amd import synthetic

    total = a.pairs or wl["pairs"]
    seeds = list(range(rank, total, world))
    pairs = [synthetic.scannet_pair(s) for s in seeds]
    o, c = synthetic.example_options(wl["kind"], iterations=wl["iterations"])
    for _ in range(a.warmup):
        madpose.estimate_batch(wl["variant"], pairs[: min(len(pairs), 2 * a.streams)], o, c, device=dev,
                               num_streams=a.streams)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = madpose.estimate_batch(wl["variant"], pairs, o, c, device=dev, num_streams=a.streams)
    barrier()
    elapsed = time.perf_counter() - t0
    errs = pair_errors(res, pairs)
    local = [elapsed, float(len(pairs) * a.steps), float(sum(st.num_hypotheses for _, st in res) * a.steps),
             float(sum(st.num_iterations_total for _, st in res) * a.steps)]
    allv = gather_counters(local, world)
    per = (total + world - 1) // world
    errs_all = gather_counters(errs + [np.nan] * (per - len(errs)), world).reshape(-1)
    if rank == 0:
        out = summarize_scannet(allv, errs_all, wl, a.steps, a.warmup, world, total)
        if world == 1 and a.cpu_budget > 0:
            out["cpu_baseline"] = cpu_baseline_pairs(wl, pairs, a.cpu_budget)
        print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 40 / 4 pairs for the single-pair workloads (about 0.5 s timed, so the
    # host LO's jitter averages out), 10 / 2 passes over the pair set for scannet
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cal")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU oracle work (0 = skip)")
    ap.add_argument("--pairs", type=int, default=0, help="scannet: total pairs (default 1500)")
    ap.add_argument("--streams", type=int, default=8, help="scannet: pairs in flight per GPU")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = 10 if a.workload == "scannet" else 40
    if a.warmup is None:
        a.warmup = 2 if a.workload == "scannet" else 4
    wl = WORKLOADS[a.workload]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    import madpose_amd as madpose
    from madpose_amd import synthetic

    if world > 1:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)
    dev = local_rank if torch.cuda.is_available() else 0

    def barrier():
        if world > 1:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    if a.workload == "scannet":
        run_scannet(a, wl, world, rank, dev, barrier)
        if world > 1:
            dist.destroy_process_group()
        return

    # per-rank pairs, generated before timing (weak scaling: one pair per rank per step)
    n_pairs = a.warmup + a.steps
    pairs = [synthetic.config_pair(wl["config"], seed=rank * 1000 + k) for k in range(n_pairs)]
    o, c = synthetic.throughput_options(wl["kind"], iterations=wl["iterations"])

    for k in range(a.warmup):
        _estimate(madpose, wl["variant"], _pair_args(pairs[k], wl["variant"]), o, c, dev)

    madpose.profile_reset()
    madpose.profile_enable(True)
    hyps = iters = lo = 0
    t_lo = 0.0
    barrier()
    t0 = time.perf_counter()
    for k in range(a.warmup, n_pairs):
        _, st = _estimate(madpose, wl["variant"], _pair_args(pairs[k], wl["variant"]), o, c, dev)
        hyps += st.num_hypotheses
        iters += st.num_iterations_total
        lo += st.number_lo_iterations
        t_lo += st.seconds_lo
    barrier()
    elapsed = time.perf_counter() - t0
    madpose.profile_enable(False)
    prof = madpose.profile_read()

    local = [elapsed, hyps, iters, lo, t_lo, prof["score_ms"], prof["solve_ms"], prof["hypotheses"],
             prof["correspondences"], prof["batches"], prof["sweeps"], prof["lm_calls"], prof["lm_wall_ms"],
             prof["sweep_wall_ms"], prof["iterations"], prof["sample_wall_ms"], prof["wait_wall_ms"],
             prof["run_wall_ms"], prof["lm_blocks"], prof["lm_big_calls"], prof["lm_big_wall_ms"]]
    allv = gather_counters(local, world)
    if rank == 0:
        res = summarize(allv, wl, a.steps, a.warmup, world)
        if world == 1 and a.cpu_budget > 0:
            res["cpu_baseline"] = cpu_baseline(wl, pairs[a.warmup], a.cpu_budget)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
