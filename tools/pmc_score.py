"""Fit the rocprofv3 PMC passes of score_batch (profiles/r02/pmc_*.csv) per workgroup
(= per RANSAC iteration of the batch) and write profiles/r*/pmc_score_batch.json, the
file bench.py reads for `roofline.traffic` and `roofline.fp64_valu`.

    python tools/pmc_score.py SQ_PASS.csv FETCH_PASS.csv OUT.json "source text"

SQ pass: SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES,
SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64.  FETCH pass: FETCH_SIZE (KiB, x2 on gfx950 for
wide reads, MI355X_MICROARCH.md HBM section), GRBM_GUI_ACTIVE (summed over the 8 XCDs).
FP64 issue model (CDNA4): an FP64 VALU wave64 instruction holds a SIMD-32 for 4 cycles
(16 FP64 FMA lanes per SIMD per cycle = the 78.6 TFLOP/s FP64 vector peak at 2.4 GHz),
other VALU instructions 2 cycles; 1024 SIMDs."""
import csv
import json
import sys
from collections import defaultdict

import numpy as np

SIMDS = 1024


def per_dispatch(path, want):
    d = defaultdict(dict)
    meta = {}
    for row in csv.DictReader(open(path)):
        if want not in row["Kernel_Name"]:
            continue
        k = int(row["Dispatch_Id"])
        d[k][row["Counter_Name"]] = d[k].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        meta[k] = (int(row["Grid_Size"]) // int(row["Workgroup_Size"]),
                   (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9, row["Kernel_Name"])
    return d, meta


def fit(x, y):
    A = np.c_[np.ones(len(x)), np.asarray(x, float)]
    c, *_ = np.linalg.lstsq(A, np.asarray(y, float), rcond=None)
    return float(c[0]), float(c[1])


def main(sq, fetch, out, source, want="score_batch_kernel<0, 10, true, true>"):
    # (round 2's kernel had three template arguments: "score_batch_kernel<0, 10, true>")
    d, meta = per_dispatch(sq, want)
    f, fmeta = per_dispatch(fetch, want)
    wg = [meta[k][0] for k in d]
    f64 = [d[k]["SQ_INSTS_VALU_FMA_F64"] + d[k]["SQ_INSTS_VALU_MUL_F64"] + d[k]["SQ_INSTS_VALU_ADD_F64"] +
           d[k]["SQ_INSTS_VALU_TRANS_F64"] for k in d]
    flops = [64 * (2 * d[k]["SQ_INSTS_VALU_FMA_F64"] + d[k]["SQ_INSTS_VALU_MUL_F64"] + d[k]["SQ_INSTS_VALU_ADD_F64"])
             for k in d]
    valu = [d[k]["SQ_INSTS_VALU"] for k in d]
    # SIMD-cycles the VALU stream needs vs the SIMD-cycles the dispatch lasted
    clocks = []
    for k in f:
        wall = fmeta[k][1]
        if fmeta[k][0] >= 4096 and wall > 0:
            clocks.append(f[k]["GRBM_GUI_ACTIVE"] / 8.0 / wall)
    clock = float(np.median(clocks)) if clocks else 2.4e9
    issue = []
    for k, v, ff in zip(d, valu, f64):
        wall = meta[k][1]
        if meta[k][0] >= 4096 and wall > 0:
            issue.append((4 * ff + 2 * (v - ff)) / (SIMDS * wall * clock))
    fw = [fmeta[k][0] for k in f]
    fetch_b = [2 * 1024 * f[k]["FETCH_SIZE"] for k in f]
    r = {
        "source": source,
        "kernel": want,
        "dispatches_sq": len(d), "dispatches_fetch": len(f),
        "unit": "per workgroup = per RANSAC iteration of the batch (one workgroup each)",
        "valu_instr_fixed_per_launch": fit(wg, valu)[0], "valu_instr_per_iteration": fit(wg, valu)[1],
        "f64_instr_per_iteration": fit(wg, f64)[1],
        "f64_flops_fixed_per_launch": fit(wg, flops)[0], "f64_flops_per_iteration": fit(wg, flops)[1],
        "f64_share_of_valu": float(np.sum(f64) / np.sum(valu)),
        "valu_issue_frac_median": float(np.median(issue)) if issue else None,
        "valu_issue_model": "(4 x F64 + 2 x other VALU wave-instructions) / (1024 SIMDs x dispatch cycles); "
                            "dispatches of >= 4096 workgroups, at the clock GRBM_GUI_ACTIVE / 8 / wall",
        "effective_clock_hz": clock,
        "correction": "x2 (gfx950 FETCH_SIZE counts half of wide reads; 8-byte loads uncalibrated)",
        "fetch_bytes_fixed_per_launch": fit(fw, fetch_b)[0], "fetch_bytes_per_iteration": fit(fw, fetch_b)[1],
    }
    json.dump(r, open(out, "w"), indent=1)
    print(json.dumps(r, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
