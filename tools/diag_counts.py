"""Where the estimator's per-iteration model counts differ from the oracle's (the
num_hypotheses parity of tests/test_full_size_gpu.py): runs one full-size case with
MADPOSE_COUNT_DUMP / ORACLE_COUNT_DUMP, prints every iteration whose count differs
with its sample, and for point-solver iterations the direct device / oracle solver
counts on the estimator's normalised points.  usage: diag_counts.py sf|tf [seed]"""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import madpose  # noqa: E402
import oracle  # noqa: E402
from madpose_amd import synthetic  # noqa: E402
from tests.helpers import oracle_cfg, oracle_opts  # noqa: E402
from tests.test_full_size_gpu import CASES  # noqa: E402


def _read(path):
    out = {}
    for line in open(path):
        v = [int(x) for x in line.split()]
        out[v[0]] = (v[1], v[2], v[3:])
    return out


def _bearings(p):
    h = np.c_[p, np.ones(len(p))]
    return h / np.linalg.norm(h, axis=1, keepdims=True)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "sf"
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    variant, kind, cfg, iters = CASES[name]
    p = synthetic.config_pair(cfg, seed=seed)
    o, c = synthetic.throughput_options(kind, iterations=iters)
    cam0, cam1 = p["pp0"], p["pp1"]
    args = (p["x0"], p["x1"], p["depth0"], p["depth1"], p["min_depth"], cam0, cam1)
    tmp = tempfile.mkdtemp()
    de, do = os.path.join(tmp, "dev.txt"), os.path.join(tmp, "orc.txt")
    os.environ["MADPOSE_COUNT_DUMP"] = de
    os.environ["ORACLE_COUNT_DUMP"] = do
    fn = [None, madpose.HybridEstimatePoseScaleOffsetSharedFocal, madpose.HybridEstimatePoseScaleOffsetTwoFocal][variant]
    _, st = fn(*args, o, c)
    _, ost, _ = oracle.estimate(variant, *args, oracle_opts(o), oracle_cfg(c))
    dev, orc = _read(de), _read(do)
    print(json.dumps({"case": name, "seed": seed, "dev_h": st.num_hypotheses, "orc_h": ost.num_hypotheses,
                      "dev_iters": len(dev), "orc_iters": len(orc)}), flush=True)
    _, _, norm_scale = oracle.score_models(variant, *args[:4], cam0, cam1, oracle_opts(o), oracle_cfg(c), [])
    a0 = (np.asarray(p["x0"], float) - np.asarray(cam0, float).reshape(2)) / norm_scale
    a1 = (np.asarray(p["x1"], float) - np.asarray(cam1, float).reshape(2)) / norm_scale
    nbad = 0
    for it in sorted(set(dev) | set(orc)):
        d, q = dev.get(it), orc.get(it)
        if d is not None and q is not None and d[:2] == q[:2] and d[2] == q[2]:
            continue
        nbad += 1
        rec = {"iter": it, "dev": d, "orc": q}
        if d is not None and q is not None and d[0] == 0 and d[2] == q[2]:
            idx = np.asarray(d[2])
            xh = np.c_[a0[idx], np.ones(len(idx))].T
            yh = np.c_[a1[idx], np.ones(len(idx))].T
            dx, dy = np.asarray(p["depth0"], float)[idx], np.asarray(p["depth1"], float)[idx]
            ss = [madpose.solve_scale_and_shift_shared_focal, madpose.solve_scale_and_shift_two_focal][variant - 1]
            rec["ss_dev"] = [np.asarray(s).tolist() for s in ss(xh, yh, dx, dy)]
            rec["ss_orc"] = np.asarray(oracle.md_scale_shift(variant, xh.T, yh.T, dx, dy)).tolist()
            pose = [madpose.solve_scale_shift_pose_shared_focal, madpose.solve_scale_shift_pose_two_focal][variant - 1]
            rec["pose_dev"] = [[m.scale, m.offset0, m.offset1] for m in pose(xh, yh, dx, dy)]
            rec["pose_orc"] = [[m["scale"], m["offset0"], m["offset1"]] for m in oracle.md_pose(variant, xh.T, yh.T,
                                                                                                  dx, dy)]
            rec["min_depth"] = np.asarray(p["min_depth"], float).tolist()
            rec["use_ours"] = bool(o.use_ours)
        if d is not None and q is not None and d[0] == 1 and d[2] == q[2]:
            idx = np.asarray(d[2])
            if variant == 1:
                dd = madpose.relpose_6pt_shared_focal(a0[idx], a1[idx])
                oo = oracle.relpose_6pt_shared_focal(_bearings(a0[idx]), _bearings(a1[idx]))
                rec["direct"] = {"dev": sorted(m.focal for m in dd), "orc": sorted(x["focal0"] for x in oo)}
                rec["roots"] = sorted(np.asarray(oracle.sixpt_roots(_bearings(a0[idx]), _bearings(a1[idx]))).tolist())
            else:
                dd = madpose.relpose_7pt_two_focal(a0[idx], a1[idx])
                Fs = oracle.relpose_7pt(_bearings(a0[idx]), _bearings(a1[idx]))
                rec["direct"] = {"dev": sorted([m.focal0, m.focal1] for m in dd),
                                 "orc_F": len(Fs),
                                 "orc_fsq": [np.asarray(oracle.bougnoux_focals(F.ravel())).tolist() for F in Fs]}
            rec["a0"] = a0[idx].tolist()
            rec["a1"] = a1[idx].tolist()
        print(json.dumps(rec), flush=True)
        if nbad > 40:
            break
    print(json.dumps({"mismatching_iterations": nbad}), flush=True)


if __name__ == "__main__":
    main()
