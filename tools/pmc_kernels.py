"""Per-kernel summary of the three PMC passes of tools/pmc_kernels.sh.

    python tools/pmc_kernels.py ISSUE_DIR WAIT_DIR FETCH_DIR

Per kernel (all dispatches of the bench run, summed, then per dispatch):
  waves, wave lifetime (SQ_WAVE_CYCLES, quad-cycles x 4 = cycles, per wave),
  VALU / FP64 wave-instructions per wave,
  where a wave's cycles go (MI355X_MICROARCH.md PMC table: SQ_WAIT_ANY parked on
  s_waitcnt / barrier, SQ_WAIT_INST_ANY issue-stalled, SQ_ACTIVE_INST_ANY issuing;
  the three are disjoint and add up to SQ_WAVE_CYCLES),
  VALU-active share of wave cycles (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES),
  SALU and LDS instructions per wave, LDS bank-conflict cycles per LDS instruction,
  FP64 issue fraction of the whole chip over the dispatch ((4 F64 + 2 other VALU) /
  (1024 SIMDs x cycles) at the 2.4 GHz peak clock),
  FETCH_SIZE x 2 (gfx950 counts half of wide reads) per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

SIMDS = 1024


def load(d):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(p)))
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(dict)
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("mp::", "").split("(")[0]
        name = name.replace("void ", "")
        k = int(r["Dispatch_Id"])
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name][k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return acc, disp


def main(issue_dir, wait_dir, fetch_dir):
    a, da = load(issue_dir)
    w, dw = load(wait_dir)
    f, df = load(fetch_dir)
    clocks = [f[n]["GRBM_GUI_ACTIVE"] / 8.0 / sum(df[n].values()) for n in f if sum(df[n].values()) > 0]
    clocks.sort()
    measured = clocks[len(clocks) // 2] if clocks else float("nan")
    # GRBM_GUI_ACTIVE / 8 / wall came out above the 2.4 GHz peak engine clock on the
    # round-6 box (short dispatches), so the issue fraction uses the peak clock: a lower
    # bound on the fraction
    clock = 2.4e9
    print(f"clock: 2.4 GHz peak used (GRBM_GUI_ACTIVE / 8 / wall, median over kernels: {measured / 1e9:.2f} GHz)")
    names = sorted(a, key=lambda n: -sum(da[n].values()))
    for n in names:
        c = a[n]
        nd = len(da[n])
        wall = sum(da[n].values())
        waves = c["SQ_WAVES"] or 1.0
        f64 = sum(c[k] for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                 "SQ_INSTS_VALU_TRANS_F64"))
        valu = c["SQ_INSTS_VALU"]
        cyc = c["SQ_WAVE_CYCLES"]
        issue = (4 * f64 + 2 * (valu - f64)) / (SIMDS * wall * clock) if wall > 0 else float("nan")
        print(f"\n{n[:110]}")
        print(f"  dispatches {nd}, {wall / nd * 1e6:.1f} us per dispatch, {waves / nd:.0f} waves per dispatch")
        print(f"  per wave: lifetime {4 * cyc / waves:.0f} cycles, VALU {valu / waves:.0f} "
              f"(FP64 {f64 / waves:.0f}) wave-instructions, chip FP64-issue fraction {issue:.3f}")
        if n in w:
            x = w[n]
            wc = x["SQ_WAVE_CYCLES"] or 1.0
            wwaves = waves / nd * len(dw[n])  # the wait pass's own dispatch count
            ldsi = x["SQ_INSTS_LDS"]
            print(f"  wave cycles: parked {x['SQ_WAIT_ANY'] / wc:.2f}, issue-stalled {x['SQ_WAIT_INST_ANY'] / wc:.2f}, "
                  f"issuing {x['SQ_ACTIVE_INST_ANY'] / wc:.2f} (VALU {x['SQ_ACTIVE_INST_VALU'] / wc:.2f}); "
                  f"SALU {x['SQ_INSTS_SALU'] / wwaves:.0f}, LDS {ldsi / wwaves:.0f} per wave, bank-conflict cycles per LDS instr "
                  f"{x['SQ_LDS_BANK_CONFLICT'] / ldsi if ldsi else 0.0:.2f}")
        if n in f:
            print(f"  FETCH_SIZE x2: {2 * 1024 * f[n]['FETCH_SIZE'] / max(len(df[n]), 1) / 1e3:.1f} kB per dispatch")


if __name__ == "__main__":
    main(*sys.argv[1:4])
