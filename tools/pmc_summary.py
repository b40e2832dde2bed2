"""Aggregate rocprofv3 counter-collection CSVs into profiles/rNN/bench_pmc_hbm.json:
{counter: {kernel_name: {"dispatches": n, "avg_KB_per_dispatch": v}}}.

FETCH_SIZE / WRITE_SIZE are TCC counters in KB summed over the dispatch; bench.py applies
the gfx950 correction (FETCH x2 for 16-B/lane streaming reads, MI355X_MICROARCH.md §HBM).

    python tools/pmc_summary.py OUT.json DIR [DIR ...]
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))  # counter -> kernel -> [n, sum]
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f, newline="") as fh:
                for row in csv.DictReader(fh):
                    k = {c.lower(): c for c in row}
                    name = row[k["kernel_name"]]
                    ctr = row[k["counter_name"]]
                    val = float(row[k["counter_value"]])
                    a = acc[ctr][name]
                    a[0] += 1
                    a[1] += val
    res = {c: {kn: {"dispatches": n, "avg_KB_per_dispatch": s / n} for kn, (n, s) in ks.items()}
           for c, ks in acc.items()}
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(f"{out_path}: " + ", ".join(f"{c} ({len(v)} kernels)" for c, v in res.items()))


if __name__ == "__main__":
    main()
