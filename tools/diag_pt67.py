"""Where the device 6pt / 7pt point solvers and the oracle disagree: runs the trial
generators of tests/test_uncalibrated_gpu.py for many trials and prints every
mismatching trial (focals / pose counts on both sides) as JSON lines."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import madpose  # noqa: E402
import oracle  # noqa: E402
from tests.test_uncalibrated_gpu import _bearings, _sample  # noqa: E402


def six(n_trials, seed):
    rng = np.random.default_rng(seed)
    bad = 0
    for trial in range(n_trials):
        clean = trial % 2 == 0
        p0, p1, R, t, f0, _ = _sample(rng, 6, True, not clean, 0.0)
        dev = madpose.relpose_6pt_shared_focal(p0, p1)
        orc = oracle.relpose_6pt_shared_focal(_bearings(p0), _bearings(p1))
        mism = len(dev) != len(orc)
        if not mism:
            for m in dev:
                d = min(np.abs(m.R() - o["R"]).max() + np.abs(m.t() - o["t"]).max() + abs(m.focal - o["focal0"])
                        for o in orc)
                if d > 1e-6:
                    mism = True
                    break
        if mism:
            bad += 1
            print(json.dumps({"solver": "6pt", "seed": seed, "trial": trial, "clean": clean, "f_gt": f0,
                              "dev_f": sorted(m.focal for m in dev), "orc_f": sorted(o["focal0"] for o in orc),
                              "p0": p0.tolist(), "p1": p1.tolist()}), flush=True)
    print(json.dumps({"solver": "6pt", "seed": seed, "trials": n_trials, "mismatch": bad}), flush=True)


def seven(n_trials, seed):
    rng = np.random.default_rng(seed)
    bad = 0
    for trial in range(n_trials):
        clean = trial % 2 == 0
        p0, p1, R, t, f0, f1 = _sample(rng, 7, False, not clean, 0.0 if clean else 1e-3)
        dev = madpose.relpose_7pt_two_focal(p0, p1)
        Fs = oracle.relpose_7pt(_bearings(p0), _bearings(p1))
        info = []
        mism = len(dev) != len(Fs)
        if not mism:
            for m in dev:
                best, arg = np.inf, None
                for F in Fs:
                    fsq = oracle.bougnoux_focals(F.ravel())
                    fa, fb = np.sqrt(np.abs(fsq))
                    E = np.diag([fb, fb, 1.0]) @ F @ np.diag([fa, fa, 1.0])
                    Ro, to, good = oracle.recover_pose(E.ravel(), p0, p1)
                    d = np.abs(m.R() - Ro).max() + np.abs(m.t() - to).max() + abs(m.focal0 - fa) + abs(m.focal1 - fb)
                    if d < best:
                        best, arg = d, (float(fa), float(fb), int(good) if np.ndim(good) == 0 else None)
                if best > 1e-6:
                    mism = True
                    info.append({"dev_f": [m.focal0, m.focal1], "best": best, "orc": arg,
                                 "dev_R": m.R().tolist(), "dev_t": m.t().tolist()})
        if mism:
            bad += 1
            print(json.dumps({"solver": "7pt", "trial": trial, "clean": clean, "ndev": len(dev), "norc": len(Fs),
                              "info": info, "p0": p0.tolist(), "p1": p1.tolist()}), flush=True)
    print(json.dumps({"solver": "7pt", "seed": seed, "trials": n_trials, "mismatch": bad}), flush=True)


if __name__ == "__main__":
    # usage: diag_pt67.py [trials] [6pt seeds, comma-separated] [7pt seeds]
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    s6 = [int(x) for x in sys.argv[2].split(",") if x] if len(sys.argv) > 2 else [21]
    s7 = [int(x) for x in sys.argv[3].split(",") if x] if len(sys.argv) > 3 else [22]
    for sd in s6:
        six(n, sd)
    for sd in s7:
        seven(n, sd)
