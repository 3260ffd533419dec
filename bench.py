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
# FP64 vector peak: 256 CUs x 4 SIMD-32 x 16 FP64 FMA lanes per cycle x 2 x 2.4 GHz (public
# MI355X spec figure; the guide has no FP64 row)
FP64_PEAK_TFLOPS = 78.6
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


def host_cpu_info():
    """nproc, the CPUs this process may run on, physical cores among them, lscpu model."""
    import platform

    aff = sorted(os.sched_getaffinity(0))
    model, tpc = platform.processor() or "unknown", 1
    try:
        with open("/proc/cpuinfo") as f:
            info = f.read()
        for line in info.splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
        sib = [l for l in info.splitlines() if l.startswith("siblings")]
        cores = [l for l in info.splitlines() if l.startswith("cpu cores")]
        if sib and cores:
            tpc = max(1, int(sib[0].split(":")[1]) // max(1, int(cores[0].split(":")[1])))
    except OSError:
        pass
    share = len(aff)
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():  # the GPU box's CPU share per GPU
        share = min(share, int(os.environ["OMP_NUM_THREADS"]))
    return {"nproc": os.cpu_count(), "affinity_cpus": len(aff), "threads_per_core": tpc,
            "physical_cores_used": max(1, share // tpc), "model": model}


def _oracle_pair_run(job):
    """One CPU-baseline process: the scalar oracle on one pair of the workload."""
    wl_key, seed, it = job
    import oracle
    from madpose_amd import synthetic
    from tests.helpers import oracle_cfg, oracle_opts

    wl = WORKLOADS[wl_key]
    pair = synthetic.config_pair(wl["config"], seed=seed)
    o, c = synthetic.throughput_options(wl["kind"], iterations=it)
    t0 = time.perf_counter()
    _, st, _ = oracle.estimate(wl["variant"], *_pair_args(pair, wl["variant"]), oracle_opts(o), oracle_cfg(c))
    return st.num_hypotheses, time.perf_counter() - t0


# the CPU baseline's build (oracle/Makefile): the reference's -O3 without -ffast-math (in a
# shared object it flips FTZ/DAZ process-wide and assumes away the residuals' DBL_MAX / NaN
# sentinels, CMakeLists.txt:14 has -O3 -ffast-math -fno-associative-math); baseline x86-64,
# so -ffp-contract=fast emits no FMA
ORACLE_FLAGS = "g++ -O3 -std=c++17 -fPIC -ffp-contract=fast -fno-math-errno (x86-64 baseline ISA)"


def cpu_baseline(wl, pair, budget_s=15.0, procs=0):
    """Scalar CPU oracle (kind "port", compiled like the reference: -O3, FMA contraction)
    on a bounded iteration count of the workload: (1) one thread on the bench's own pair,
    (2) one process per physical core of this host's CPU share, each on its own pair
    (independent pairs).  `value` is the all-core aggregate."""
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
    single = {"value": st.num_hypotheses / dt, "cores": 1,
              "sample": f"same pair, {it} iterations (min=max=per-solver cap), single thread, {dt:.1f} s, "
                        f"{st.num_hypotheses} hypotheses, {st.number_lo_iterations} LO runs"}
    host = host_cpu_info()
    p = procs or host["physical_cores_used"]
    key = [k for k, v in WORKLOADS.items() if v is wl][0]
    import multiprocessing as mp

    jobs = [(key, 900000 + j, it) for j in range(p)]
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(p) as pool:
        got = pool.map(_oracle_pair_run, jobs)
    wall = time.perf_counter() - t0
    hyps = sum(h for h, _ in got)
    inner = max(d for _, d in got)
    return {"value": hyps / inner, "unit": "hypotheses/s", "cores": p, "kind": "port",
            "sample": f"{p} processes (one per physical core of the host's CPU share), each the oracle on its own "
                      f"pair of the workload for {it} iterations; {hyps} hypotheses over the slowest process's "
                      f"{inner:.1f} s ({wall:.1f} s with process start-up)",
            "iterations": it, "workload_iterations": wl["iterations"], "compile_flags": ORACLE_FLAGS,
            "single_thread": single, "host": host}


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
            "sample_ms", "wait_ms", "run_ms", "lm_blocks", "lm_big_calls", "lm_big_ms", "model_trips",
            "model_trips_full", "prof_accepted", "prof_scored", "prof_pairs"]


def gather_counters(local, world):
    """All ranks' counter vectors (world x len(COUNTERS)) -- the only collective of the
    bench: one all_gather of a few doubles per rank (RCCL on GPUs, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor(local, dtype=torch.float64)
    if not (dist.is_available() and dist.is_initialized()):
        return t.numpy()[None]  # one rank, no process group
    out = [torch.zeros_like(t) for _ in range(world)]
    if dist.get_backend() == "nccl":
        gl = [g.cuda() for g in out]
        dist.all_gather(gl, t.cuda())
        out = [g.cpu() for g in gl]
        GATHER_LOG.append({"backend": "nccl", "device": str(gl[0].device), "doubles": int(t.numel())})
    else:
        dist.all_gather(out, t)
        GATHER_LOG.append({"backend": dist.get_backend(), "device": "cpu", "doubles": int(t.numel())})
    return torch.stack(out).numpy()


GATHER_LOG = []  # the all_gathers this process issued (reported under "dist")


def dist_info(world):
    """Backend and world size as torch.distributed saw them (the N-GPU runs show that
    RCCL had every rank), plus the LO-pool spin setting of this process."""
    info = {"backend": None, "world_size": world}
    try:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            info["backend"] = dist.get_backend()
            info["world_size"] = dist.get_world_size()
        info["all_gathers"] = list(GATHER_LOG)
    except Exception:  # pragma: no cover - informational only
        pass
    try:
        from madpose_amd import _lib

        info["lo_spin_us"] = int(_lib.lib().mp_lo_spin_us())
    except Exception:  # the CPU stand-in engine of the tests has no library
        info["lo_spin_us"] = None
    # rank 0's CPU share (pin_rank; empty when one rank has the node's share)
    info["cpu_share"] = {k: v for k, v in PIN_INFO.items() if k != "cpu_list"} or None
    info["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
    return info


def summarize(allv, wl, steps, warmup, world):
    """Whole-job JSON record from the gathered counters: value = all ranks' hypotheses
    divided by the slowest rank's wall time (weak scaling)."""
    c = {k: allv[:, i] for i, k in enumerate(COUNTERS)}
    t_max = float(c["elapsed_s"].max())
    # the profiled pairs (bench --prof-every), the denominator of the per-pair breakdown
    prof_n = float(c["prof_pairs"].sum()) or float(world * steps)
    score_ms = float(c["score_ms"].sum())
    # the exact early exit (row N1) skips (model, trip) evaluations: the roofline
    # counts the correspondence bytes the launches actually read (the full figure's
    # share model_trips / model_trips_full); "effective" credits the full figure
    full_trips = float(c["model_trips_full"].sum())
    ev_share = float(c["model_trips"].sum()) / full_trips if full_trips > 0 else 1.0
    full_bytes = float(c["prof_correspondences"].sum()) * BYTES_PER_CORR
    achieved = full_bytes * ev_share / (score_ms * 1e-3) / 1e9 if score_ms > 0 else 0.0
    # effective: the algorithmic 48 N bytes of every hypothesis the launches scored (the
    # record skip's iterations, never scored, are not credited)
    hyp = float(c["prof_hypotheses"].sum())
    scored_share = float(c["prof_scored"].sum()) / hyp if hyp > 0 else 1.0
    effective = full_bytes * scored_share / (score_ms * 1e-3) / 1e9 if score_ms > 0 else 0.0
    launches = int(c["prof_batches"].sum())
    traffic, traffic_note = None, None
    tm = pmc_traffic_model()
    if tm is not None and not tm.get("kernel", "").startswith(f"score_batch_kernel<{wl['variant']},"):
        tm = None  # the committed PMC fit is of another variant's kernel
    if tm is not None and launches > 0:
        it_per_launch = float(c["prof_iterations"].sum()) / launches
        traffic = tm["fetch_bytes_fixed_per_launch"] + tm["fetch_bytes_per_iteration"] * it_per_launch
        traffic_note = (f"bytes per launch from the FETCH_SIZE fit in {tm['file']} ({tm['correction']}) at "
                        f"{it_per_launch:.0f} iterations per launch; algorithmic bytes per launch "
                        f"{float(c['prof_correspondences'].sum()) * BYTES_PER_CORR / launches:.3g}: the pair's "
                        f"arrays stay L2-resident across the workgroups of a launch")
    fp64 = None
    if tm is not None and launches > 0 and "f64_flops_per_iteration" in tm and score_ms > 0:
        it_per_launch = float(c["prof_iterations"].sum()) / launches
        flops = tm["f64_flops_fixed_per_launch"] + tm["f64_flops_per_iteration"] * it_per_launch
        tflops = flops / (score_ms * 1e-3 / launches) / 1e12
        fp64 = {"bound": "fp64_valu", "achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": tflops / FP64_PEAK_TFLOPS, "valu_issue_frac": tm.get("valu_issue_frac_median"),
                "f64_share_of_valu": tm.get("f64_share_of_valu"),
                "note": f"FP64 flops per launch from the SQ_INSTS_VALU_*_F64 fit in {tm['file']} at "
                        f"{it_per_launch:.0f} iterations per launch over the HIP-event launch time; "
                        f"valu_issue_frac = VALU issue cycles / SIMD cycles of the profiled dispatches"}
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
        "profiled_pairs": int(c["prof_pairs"].sum()),
        "ms_per_pair": {k: float(c[src].sum()) / prof_n for k, src in
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
            # exact early exit (row N1): the share of (model, 256-correspondence trip)
            # evaluations the kernel actually ran, and the correspondence bytes those
            # evaluations read (48 B each) per launch next to the algorithmic figure
            "evaluated_frac": ev_share if full_trips > 0 else None,
            "evaluated_bytes_per_launch": full_bytes * ev_share / launches if launches > 0 else None,
            "algorithmic_bytes_per_launch": full_bytes / launches if launches > 0 else None,
            "effective_GBps": effective,
            "fp64_valu": fp64,
        },
        "cpu_baseline": None,
        # speculative waste: every hypothesis the solvers produced ("solved") and every
        # one whose scoring sweep ran ("scored": score_batch skips the iterations past a
        # batch's first new best once LO cuts there) against those of the iterations
        # the estimator consumed (batches cut at an LO, discarded post-LO speculation)
        "speculation": {"solved_hypotheses": int(c["prof_hypotheses"].sum()),
                        "scored_hypotheses": int(c["prof_scored"].sum()),
                        "accepted_hypotheses": int(c["prof_accepted"].sum()),
                        "solved_over_accepted": float(c["prof_hypotheses"].sum()) / max(float(c["prof_accepted"].sum()), 1.0),
                        "scored_over_accepted": float(c["prof_scored"].sum()) / max(float(c["prof_accepted"].sum()), 1.0)},
        "dist": dist_info(world),
    }


def pair_errors(results, pairs):
    """max(rotation error, translation angle error) in degrees per pair
    (madpose/utils.py:70-78 compute_pose_error), the quantity pose AUC integrates."""
    from madpose_amd import utils

    return [max(utils.compute_pose_error(p["T_0to1"], m.R(), m.t())) for (m, _), p in zip(results, pairs)]


def summarize_scannet(allv, errs, wl, steps, warmup, world, total, auc_fn=None):
    """Whole-job record of the ScanNet-1500 stand-in: value = pairs per second of all
    ranks over the slowest rank's time (total work fixed: strong scaling); AUC@5/10/20
    over the per-pair errors of every rank (auc_fn: the engine's evaluator, the device
    one for the product engine; default the host pose_auc)."""
    from madpose_amd import utils

    auc_fn = auc_fn or utils.pose_auc
    t_max = float(allv[:, 0].max())
    done = float(allv[:, 1].sum())
    e = np.asarray(errs, dtype=np.float64)
    e = e[np.isfinite(e)]
    auc = auc_fn(e, (5, 10, 20)) if len(e) else [None] * 3
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
        "dist": dist_info(world),
        "cpu_baseline": None,
    }


def _oracle_pairs_run(job):
    """One CPU-baseline process of the ScanNet stand-in: the oracle on its pairs until
    the budget is spent; returns (pairs done, seconds)."""
    wl_key, seeds, budget_s = job
    import oracle
    from madpose_amd import synthetic
    from tests.helpers import oracle_cfg, oracle_opts

    wl = WORKLOADS[wl_key]
    o, c = synthetic.example_options(wl["kind"], iterations=wl["iterations"])
    pairs = [synthetic.scannet_pair(s) for s in seeds]
    t0 = time.perf_counter()
    k = 0
    for p in pairs:
        oracle.estimate(wl["variant"], *_pair_args(p, wl["variant"]), oracle_opts(o), oracle_cfg(c))
        k += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    return k, time.perf_counter() - t0


def cpu_baseline_pairs(wl, seeds, budget_s, procs=0):
    """The scalar CPU oracle on the rank's pairs: one thread on the first pairs that fit
    in budget_s, and one process per physical core over disjoint pairs for budget_s each."""
    try:
        import oracle  # noqa: F401
    except Exception as e:
        return {"value": None, "unit": "pairs/s", "cores": 1, "kind": "port", "sample": f"unavailable: {e}"}
    k, dt = _oracle_pairs_run(("scannet", seeds, budget_s / 2))
    single = {"value": k / dt, "cores": 1, "sample": f"first {k} pairs of the set, single thread, {dt:.1f} s"}
    host = host_cpu_info()
    p = procs or host["physical_cores_used"]
    import multiprocessing as mp

    jobs = [("scannet", seeds[j::p][:64], budget_s / 2) for j in range(p)]
    with mp.get_context("spawn").Pool(p) as pool:
        got = pool.map(_oracle_pairs_run, jobs)
    done = sum(g[0] for g in got)
    rate = sum(g[0] / g[1] for g in got)
    return {"value": rate, "unit": "pairs/s", "cores": p, "kind": "port",
            "sample": f"{p} processes (one per physical core of the host's CPU share) over disjoint pairs of the "
                      f"set, {done} pairs in {budget_s / 2:.1f} s each; value = sum of per-process rates",
            "compile_flags": ORACLE_FLAGS, "single_thread": single, "host": host}


RECORD_FIELDS = (["seed"] + [f"R{i}{j}" for i in range(3) for j in range(3)] + ["t0", "t1", "t2", "scale", "offset0",
                 "offset1", "focal0", "focal1", "num_iterations_total", "best_num_inliers", "best_model_score",
                 "number_lo_iterations", "err_R_deg", "err_t_deg"])


def result_record(seed, model, stats, pair, err=None):
    """One fixed-size result record per pair (pose + stats), the unit
    the ranks exchange at the end: seed, R, t, scale, offsets, focal(s), iteration and
    inlier counts, score, LO count, and the pose error against the synthetic ground truth
    (madpose/utils.py:59-78 compute_pose_error; err: (err_t, err_R) computed already, e.g.
    by the device evaluator)."""
    from madpose_amd import utils

    R, t = np.asarray(model.R(), dtype=np.float64), np.asarray(model.t(), dtype=np.float64)
    f0 = getattr(model, "focal0", getattr(model, "focal", np.nan))
    f1 = getattr(model, "focal1", getattr(model, "focal", np.nan))
    et, eR = utils.compute_pose_error(pair["T_0to1"], R, t) if err is None else err
    rec = ([float(seed)] + list(R.reshape(9)) + list(t.reshape(3)) +
           [getattr(model, "scale", np.nan), getattr(model, "offset0", np.nan), getattr(model, "offset1", np.nan), f0,
            f1, stats.num_iterations_total, stats.best_num_inliers, stats.best_model_score,
            stats.number_lo_iterations, eR, et])
    assert len(rec) == len(RECORD_FIELDS)
    return rec


def gather_records(recs, per_rank, world):
    """All ranks' result records (one all_gather over RCCL / gloo). Ranks own different
    numbers of pairs, so each pads to per_rank rows with NaN; padding is dropped."""
    w = len(RECORD_FIELDS)
    local = np.full((per_rank, w), np.nan)
    if recs:
        local[: len(recs)] = np.asarray(recs, dtype=np.float64)
    allr = gather_counters(local.reshape(-1).tolist(), world).reshape(world * per_rank, w)
    return allr[np.isfinite(allr[:, 0])]


def records_summary(recs):
    """What rank 0 reports about the gathered records."""
    seeds = recs[:, 0]
    err = np.maximum(recs[:, RECORD_FIELDS.index("err_R_deg")], recs[:, RECORD_FIELDS.index("err_t_deg")])
    return {"records": int(len(recs)), "record_doubles": len(RECORD_FIELDS),
            "pairs_disjoint": bool(len(np.unique(seeds)) == len(seeds)),
            "median_pose_err_deg": float(np.median(err)) if len(err) else None}


def records_of(eng, seeds, res, pairs):
    """Result records of a rank's pairs, their pose errors from the engine's evaluator
    in one call (the device evaluator mp_pose_eval for the product engine)."""
    if not res:
        return []
    T = np.stack([p["T_0to1"] for p in pairs])
    R = np.stack([np.asarray(m.R(), dtype=np.float64) for m, _ in res])
    t = np.stack([np.asarray(m.t(), dtype=np.float64).reshape(3) for m, _ in res])
    et, eR = eng.pose_errors(T, R, t)
    return [result_record(s, m, st, p, (et[k], eR[k])) for k, (s, (m, st), p) in enumerate(zip(seeds, res, pairs))]


def shard_scannet(total, world, rank):
    """configs[4] pairs of this rank: longest-processing-time-first over the pair sizes
    (work ~ N x iterations); deterministic, every rank computes the same
    assignment, and the pair of seed s is the same on whichever rank draws it."""
    from madpose_amd import synthetic

    sizes = [synthetic.scannet_size(s) for s in range(total)]
    load = [0] * world
    owner = [0] * total
    for s in sorted(range(total), key=lambda s: (-sizes[s], s)):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[s] = r
        load[r] += sizes[s]
    return [s for s in range(total) if owner[s] == rank]


def run_scannet(a, wl, world, rank, dev, barrier, eng):
    from madpose_amd import synthetic

    total = a.pairs or wl["pairs"]
    seeds = shard_scannet(total, world, rank)
    pairs = [synthetic.scannet_pair(s) for s in seeds]
    o, c = synthetic.example_options(wl["kind"], iterations=wl["iterations"])
    for _ in range(a.warmup):
        eng.estimate_batch(wl["variant"], pairs[: min(len(pairs), 2 * a.streams)], o, c, device=dev,
                           num_streams=a.streams)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = eng.estimate_batch(wl["variant"], pairs, o, c, device=dev, num_streams=a.streams)
    barrier()
    elapsed = time.perf_counter() - t0
    recs = records_of(eng, seeds, res, pairs)
    local = [elapsed, float(len(pairs) * a.steps), float(sum(st.num_hypotheses for _, st in res) * a.steps),
             float(sum(st.num_iterations_total for _, st in res) * a.steps)]
    # point-only baseline (untimed): the examples compare against PoseLib's point-based
    # estimate_relative_pose (examples/calibrated.py:92-122, shared_focal.py:111-130);
    # PoseLib is not vendored, so the reference's own point-only mode stands in:
    # EstimatorConfig(solver=EPI_ONLY, score=EPI_ONLY, LO=EPI_ONLY) on the same pairs
    prec = []
    if a.point_only:
        from madpose_amd.api import EstimatorConfig

        cp = EstimatorConfig(1, 1, 1)
        cp.min_depth_constraint, cp.use_shift = c.min_depth_constraint, c.use_shift
        pres = eng.estimate_batch(wl["variant"], pairs, o, cp, device=dev, num_streams=a.streams)
        prec = records_of(eng, seeds, pres, pairs)
    allv = gather_counters(local, world)
    per = (total + world - 1) // world + 1
    allr = gather_records(recs, per, world)
    allp = gather_records(prec, per, world) if a.point_only else None
    if rank == 0:
        errs = np.maximum(allr[:, RECORD_FIELDS.index("err_R_deg")], allr[:, RECORD_FIELDS.index("err_t_deg")])
        out = summarize_scannet(allv, errs, wl, a.steps, a.warmup, world, total, eng.pose_auc)
        out["results"] = records_summary(allr)
        if allp is not None:
            pe = np.maximum(allp[:, RECORD_FIELDS.index("err_R_deg")], allp[:, RECORD_FIELDS.index("err_t_deg")])
            pe = pe[np.isfinite(pe)]
            auc = eng.pose_auc(pe, (5, 10, 20)) if len(pe) else [None] * 3
            out["point_only_baseline"] = {
                "pose_auc": {"5": auc[0], "10": auc[1], "20": auc[2], "pairs": int(len(pe))},
                "config": "EstimatorConfig(solver=EPI_ONLY, score=EPI_ONLY, LO=EPI_ONLY): the reference's own "
                          "point-only mode (6pt shared-focal solver, Sampson error only), standing in for the "
                          "examples' poselib estimate_*_relative_pose (PoseLib is not vendored); untimed"}
        if world == 1 and a.cpu_budget > 0:
            out["cpu_baseline"] = cpu_baseline_pairs(wl, seeds, a.cpu_budget, a.cpu_procs)
        print(json.dumps(out), flush=True)


class _Engine:
    """The product path: madpose_amd through the C ABI on the HIP device."""

    def __init__(self):
        import madpose_amd

        self.m = madpose_amd

    def estimate(self, variant, args, o, c, device):
        return _estimate(self.m, variant, args, o, c, device)

    def estimate_batch(self, *args, **kw):
        return self.m.estimate_batch(*args, **kw)

    def pose_errors(self, T, R, t):
        return self.m.pose_eval_batch(T, R, t, thresholds=())[:2]

    def pose_auc(self, errors, thresholds):
        return self.m.pose_auc_batch(errors, thresholds)

    def profile_reset(self):
        self.m.profile_reset()

    def profile_enable(self, on):
        self.m.profile_enable(on)

    def profile_read(self):
        return self.m.profile_read()


def _engine(a):
    if a.engine_module:  # tests only: a CPU stand-in that drives the sharding / gather plumbing
        import importlib

        return importlib.import_module(a.engine_module).Engine()
    return _Engine()


def parse_cpulist(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_local_cpus(base="/sys/class/kfd/kfd/topology/nodes", pci="/sys/bus/pci/devices"):
    """The CPUs local to each HIP device, in HIP's order (the GPU nodes of the KFD
    topology, ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES applied), from sysfs only (no
    GPU call); None when the topology cannot be read."""
    try:
        out = []
        for k in sorted(int(d) for d in os.listdir(base) if d.isdigit()):
            try:
                with open(f"{base}/{k}/properties") as f:
                    props = dict(l.split()[:2] for l in f if len(l.split()) >= 2)
            except OSError:
                # a node this process may not open is a GPU it cannot use either: the
                # pool's boxes expose only their own GPU's node (profiles/r05/topo.log)
                continue
            if int(props.get("simd_count", "0")) <= 0:
                continue
            loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
            bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"
            try:
                with open(f"{pci}/{bdf}/local_cpulist") as f:
                    out.append(parse_cpulist(f.read()))
            except OSError:
                out.append([])  # locality unknown: every allowed CPU is a candidate
        for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
            vis = os.environ.get(var)
            if vis:
                ids = [int(v) for v in vis.split(",") if v.strip().isdigit()]
                out = [out[i] for i in ids if i < len(out)]
        return out or None
    except (OSError, ValueError):
        return None


def cpu_siblings(cpus):
    """cpu -> the smallest CPU of its core (SMT siblings share it)."""
    first = {}
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                first[c] = min(parse_cpulist(f.read()))
        except (OSError, ValueError):
            first[c] = c
    return first


def cpu_l3(cpus):
    """cpu -> the smallest CPU sharing its last-level cache (an EPYC CCD), from sysfs."""
    first = {}
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                first[c] = min(parse_cpulist(f.read()))
        except (OSError, ValueError):
            first[c] = c
    return first


def partition_cpus(local, allowed, core_of, devices, l3_of=None):
    """Host CPUs for the ranks of one node: rank r runs on devices[r]; its candidates are
    the allowed CPUs local to that GPU (all allowed CPUs when none is).  With l3_of (cpu
    -> last-level-cache id) and at least as many complete L3 domains among the candidates
    as ranks sharing them, each rank gets one L3 domain (spread evenly over them): the
    estimator's LO threads and LM pool synchronize through that cache.  Otherwise the
    ranks with the same candidates split them into contiguous runs of whole cores.
    local: CPU lists per device (or None); core_of: cpu -> core id.  Returns one sorted
    CPU list per rank."""
    allowed = sorted(set(allowed))
    cand = []
    for d in devices:
        c = sorted(set(local[d]) & set(allowed)) if local and d < len(local) else []
        cand.append(tuple(c or allowed))
    out = [None] * len(devices)
    for key in dict.fromkeys(cand):
        ranks = [r for r in range(len(devices)) if cand[r] == key]
        k = len(ranks)
        if l3_of:
            groups = {}
            for c in key:
                groups.setdefault(l3_of.get(c, c), []).append(c)
            # complete domains only (every CPU of the domain allowed), largest first
            full = [sorted(g) for g in groups.values() if len(g) >= max(len(v) for v in groups.values())]
            full.sort(key=lambda g: g[0])
            if len(full) >= k and len(full[0]) >= 2:
                # (from the last domain down: the first CCD of a host is where its system
                # work runs -- a single pair pinned there once took 20.6 ms instead of
                # 4.8, profiles/r05/r5pb; the last CCD of either socket gave 4.75-5.02,
                # r5pc)
                for j, r in enumerate(ranks):
                    out[r] = full[len(full) - 1 - j * len(full) // k]
                continue
        cores = sorted(dict.fromkeys(core_of.get(c, c) for c in key))
        for j, r in enumerate(ranks):
            lo, hi = len(cores) * j // k, len(cores) * (j + 1) // k
            mine = set(cores[lo:hi]) if hi > lo else {cores[j % len(cores)]}
            out[r] = sorted(c for c in key if core_of.get(c, c) in mine)
    return out


PIN_INFO = {}  # this rank's CPU share (reported under "dist")


def pin_rank(local_rank, local_world, per_ccd=True):
    """Pin this rank (one of local_world on the node, possibly the only one), before any
    GPU call and before the engine's threads exist, to the CPUs local to its GPU -- one
    last-level-cache domain when there are enough of them, else a split of whole cores
    with the ranks that share them (the estimator's host LO runs on these cores: unpinned
    ranks let their LM pools, LO lanes and samplers migrate across CCDs and sockets) --
    and size the LM pool and its spin from the share.  MADPOSE_BENCH_PIN=0: no pinning;
    MADPOSE_BENCH_CPUS=list: exactly these CPUs."""
    explicit = os.environ.get("MADPOSE_BENCH_CPUS")  # an explicit CPU list for this process (A/B)
    if explicit and hasattr(os, "sched_setaffinity"):
        share = parse_cpulist(explicit)
        os.sched_setaffinity(0, share)
        PIN_INFO.update({"cpus": len(share), "cpu_list": share, "pinned": True, "explicit": True})
        return
    if os.environ.get("MADPOSE_BENCH_PIN") == "0" or not hasattr(os, "sched_setaffinity"):
        if hasattr(os, "sched_getaffinity"):
            PIN_INFO.update({"cpus": len(os.sched_getaffinity(0)), "pinned": False})
        return
    allowed = sorted(os.sched_getaffinity(0))
    bench_dev = os.environ.get("MADPOSE_BENCH_DEVICE")
    devices = [int(bench_dev) if bench_dev is not None else r for r in range(local_world)]
    local = gpu_local_cpus()
    # one rank too: unpinned, its threads float over the host (a 16-CPU quota on 256
    # CPUs on the MI355X boxes) and the LO's pool synchronizes across CCDs and sockets --
    # big LM solves 77-86 us unpinned, 28 us pinned to one CCD (8 cores + SMT), cal
    # 5.68-5.91 -> 4.71-4.92 ms per pair (profiles/r05/r5pa)
    if local_world <= 1 and not per_ccd:
        # (a single rank with many pairs in flight, the ScanNet stand-in, wants cores more
        # than one cache: 960 pairs/s unpinned against 883 on one CCD, r5pb)
        PIN_INFO.update({"cpus": len(allowed), "pinned": False})
        return
    share = partition_cpus(local, allowed, cpu_siblings(allowed), devices,
                           cpu_l3(allowed) if per_ccd else None)[local_rank]
    os.sched_setaffinity(0, share)
    # the LM pool: the calling thread plus up to 7 workers, leaving the estimator, the
    # sampler and the LO lanes their cores; spin only on a share of its own
    os.environ.setdefault("MADPOSE_LO_THREADS", str(max(1, min(8, len(share) - 4))))
    os.environ.setdefault("MADPOSE_LO_SPIN", "1000" if len(share) >= 12 else "0")  # (host/lm.cpp lo_spin_us)
    PIN_INFO.update({"cpus": len(share), "cpu_list": share, "gpu_local": bool(local), "pinned": True,
                     "l3_domains": len(set(cpu_l3(share).values())),
                     "lo_threads": int(os.environ["MADPOSE_LO_THREADS"])})


def spawn_ranks(n, argv):
    """--gpus N without a launcher: start N child processes of this script, one per GPU
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), before anything in
    this process touches the GPU, and exit with the worst child status."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # (each child pins itself to its share of the host CPUs, pin_rank)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one process per GPU); default: WORLD_SIZE or 1")
    # defaults: 40 / 4 pairs for the single-pair workloads (about 0.5 s timed, so the
    # host LO's jitter averages out), 10 / 2 passes over the pair set for scannet
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cal")
    ap.add_argument("--prof-every", type=int, default=4,
                    help="profile every k-th timed pair (HIP events, work counts, LO counters; 1 = every pair)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU oracle work (0 = skip)")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="processes of the all-core CPU baseline leg (0 = one per physical core)")
    ap.add_argument("--pairs", type=int, default=0, help="scannet: total pairs (default 1500)")
    ap.add_argument("--streams", type=int, default=8, help="scannet: pairs in flight per GPU")
    ap.add_argument("--in-flight", type=int, default=8,
                    help="configs[1..3]: also time the pairs k at a time on the GPU (secondary figure; 1 = skip)")
    ap.add_argument("--no-point-only", dest="point_only", action="store_false",
                    help="scannet: skip the untimed point-only baseline pass")
    ap.add_argument("--engine-module", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if a.steps is None:
        a.steps = 10 if a.workload == "scannet" else 40
    if a.warmup is None:
        a.warmup = 2 if a.workload == "scannet" else 4
    wl = WORKLOADS[a.workload]

    if "WORLD_SIZE" not in os.environ and a.gpus is not None and a.gpus > 1:
        return spawn_ranks(a.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus is not None and a.gpus != world:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    pin_rank(local_rank, int(os.environ.get("LOCAL_WORLD_SIZE", world)), per_ccd=a.workload != "scannet")
    # hardware queues of the HIP runtime (read once, at its start): every estimator in
    # flight drives three streams (one per batch slot + the MD side stream), and with HIP's default of 4
    # queues the kernels of different pairs serialize behind each other -- ScanNet
    # stand-in 943-946 pairs/s at 4 queues, 1302-1309 at 8, 1281-1337 at 16, 1232-1271
    # at 24 (8 pairs in flight, profiles/r05/r5r).  The boxes export 4, so it is set, not
    # defaulted; MADPOSE_HW_QUEUES overrides the 16.
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("MADPOSE_HW_QUEUES", "16")

    import torch
    import torch.distributed as dist

    from madpose_amd import synthetic

    eng = _engine(a)
    gpu = a.engine_module is None and torch.cuda.is_available()
    # rehearsal knobs for one-GPU boxes (several ranks on one card need gloo: RCCL
    # refuses two ranks on one device): MADPOSE_BENCH_DIST_BACKEND, MADPOSE_BENCH_DEVICE
    dev = int(os.environ.get("MADPOSE_BENCH_DEVICE", local_rank)) if gpu else 0
    # MADPOSE_BENCH_DIST=1: a process group even for one rank, so the result gather runs
    # through RCCL on a one-GPU box as it does on the 8-GPU node (configs[4]'s collective)
    force_dist = os.environ.get("MADPOSE_BENCH_DIST") == "1"
    if world > 1 or force_dist:
        backend = os.environ.get("MADPOSE_BENCH_DIST_BACKEND", "nccl" if gpu else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(dev)
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket

                with socket.socket() as s:
                    s.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
            dist.init_process_group(backend=backend, rank=0, world_size=1)
        else:
            dist.init_process_group(backend=backend)
    distributed = dist.is_available() and dist.is_initialized()

    def barrier():
        if distributed:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    if a.workload == "scannet":
        run_scannet(a, wl, world, rank, dev, barrier, eng)
        if distributed:
            dist.destroy_process_group()
        return 0

    # per-rank pairs, generated before timing (weak scaling: one pair per rank per step;
    # rank r owns seeds r*1000 + k, disjoint across ranks)
    n_pairs = a.warmup + a.steps
    seeds = [rank * 1000 + k for k in range(n_pairs)]
    pairs = [synthetic.config_pair(wl["config"], seed=s) for s in seeds]
    o, c = synthetic.throughput_options(wl["kind"], iterations=wl["iterations"])

    for k in range(a.warmup):
        eng.estimate(wl["variant"], _pair_args(pairs[k], wl["variant"]), o, c, dev)

    # the engine's profile (HIP events around every batch's solve and score, the
    # per-iteration work counts, the host LO counters) on every prof_every-th timed pair:
    # on every pair it cost 7 % of the pair time (4.52 -> 4.19 ms with it off,
    # profiles/r05/prof_off); the per-pair and per-launch figures average the profiled
    # pairs, the headline value counts every pair
    eng.profile_reset()
    hyps = iters = lo = 0
    t_lo = 0.0
    res = []
    prof_pairs = 0
    barrier()
    t0 = time.perf_counter()
    for k in range(a.warmup, n_pairs):
        on = (k - a.warmup) % max(1, a.prof_every) == 0
        prof_pairs += on
        eng.profile_enable(on)
        m, st = eng.estimate(wl["variant"], _pair_args(pairs[k], wl["variant"]), o, c, dev)
        res.append((m, st))
        hyps += st.num_hypotheses
        iters += st.num_iterations_total
        lo += st.number_lo_iterations
        t_lo += st.seconds_lo
    barrier()
    elapsed = time.perf_counter() - t0
    eng.profile_enable(False)
    prof = eng.profile_read()

    recs = records_of(eng, seeds[a.warmup:a.warmup + len(res)], res, pairs[a.warmup:a.warmup + len(res)])
    local = [elapsed, hyps, iters, lo, t_lo, prof["score_ms"], prof["solve_ms"], prof["hypotheses"],
             prof["correspondences"], prof["batches"], prof["sweeps"], prof["lm_calls"], prof["lm_wall_ms"],
             prof["sweep_wall_ms"], prof["iterations"], prof["sample_wall_ms"], prof["wait_wall_ms"],
             prof["run_wall_ms"], prof["lm_blocks"], prof["lm_big_calls"], prof["lm_big_wall_ms"],
             prof["model_trips"], prof["model_trips_full"], prof["accepted"], prof["scored"], prof_pairs]
    allv = gather_counters(local, world)
    allr = gather_records(recs, a.steps, world)
    if rank == 0:
        out = summarize(allv, wl, a.steps, a.warmup, world)
        out["results"] = records_summary(allr)
        if world == 1 and a.in_flight > 1:
            out["pairs_in_flight"] = in_flight_leg(eng, wl, pairs[a.warmup:], o, c, dev, a.in_flight)
        if world == 1 and a.cpu_budget > 0:
            out["cpu_baseline"] = cpu_baseline(wl, pairs[a.warmup], a.cpu_budget, a.cpu_procs)
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()
    return 0


def in_flight_leg(eng, wl, pairs, o, c, dev, k):
    """Secondary figure (never `value`): the same timed pairs with k estimators in flight
    on the one GPU (estimate_batch: k host threads, one HIP stream context each). One
    estimator leaves the GPU idle while its host LO runs; concurrent pairs fill it."""
    eng.estimate_batch(wl["variant"], pairs[:k], o, c, device=dev, num_streams=k)  # warm the contexts
    t0 = time.perf_counter()
    res = eng.estimate_batch(wl["variant"], pairs, o, c, device=dev, num_streams=k)
    el = time.perf_counter() - t0
    hyps = sum(st.num_hypotheses for _, st in res)
    return {"pairs": len(pairs), "in_flight": k, "hypotheses_per_s": hyps / el, "ms_per_pair": el / len(pairs) * 1e3,
            "note": "the timed pairs again, k at a time on one GPU (host threads x streams); a secondary figure, "
                    "not the bench value (which keeps configs[1]'s one pair per step)"}


if __name__ == "__main__":
    sys.exit(main())
