"""Summarise a rocprofv3 `--pmc FETCH_SIZE` counter-collection CSV per kernel.

    python tools/pmc_traffic.py gpurun_out/pmc_r1/pmc_counter_collection.csv

FETCH_SIZE is in KiB per dispatch (memory-side L2 read requests).  On gfx950 it
counts half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM
section); the corrected column doubles it.  The score kernel's loads are 8-byte
per lane, a width the guide lists as uncalibrated, so both figures are printed.
"""
import csv
import sys
from collections import defaultdict


def main(path):
    acc = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != "FETCH_SIZE":
                continue
            name = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            acc[name][0] += 1
            acc[name][1] += float(row["Counter_Value"])
    print(f"{'kernel':70s} {'dispatches':>10s} {'KiB/dispatch':>14s} {'x2 corrected B/dispatch':>24s}")
    for name, (n, kib) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        print(f"{name[:70]:70s} {n:10d} {kib / n:14.1f} {2 * kib / n * 1024:24.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
