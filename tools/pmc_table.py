"""Per-kernel table of rocprofv3 counters: each counter summed over the rows of a dispatch,
then averaged over the dispatches of that kernel (SQ cycle counters are per-SE/XCD sums;
compare ratios between kernels of one run, not absolutes across runs).

    python tools/pmc_table.py DIR [kernel-substring ...]
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    for a, b in (("siren::", ""), ("NtCfg<256, 256, 2, 4, ", "Nt<"), ("TnCfg<256, 256, 2, 4, ", "Tn<"),
                 ("gemm_nt_kernel", "nt"), ("gemm_tn_kernel", "tn")):
        name = name.replace(a, b)
    return name.split("(")[0][:60]


def main():
    d, keys = sys.argv[1], sys.argv[2:]
    per = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> sum
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                k = {c.lower(): c for c in row}
                name = row[k["kernel_name"]]
                if keys and not any(s in name for s in keys):
                    continue
                disp = row[k.get("dispatch_id", k.get("correlation_id", "kernel_name"))]
                per[(name, disp)][row[k["counter_name"]]] += float(row[k["counter_value"]])
    agg = defaultdict(lambda: defaultdict(list))
    for (name, _), ctrs in per.items():
        for c, v in ctrs.items():
            agg[name][c].append(v)
    counters = sorted({c for v in agg.values() for c in v})
    print("kernel".ljust(62) + "".join(c[:22].rjust(24) for c in counters))
    for name in sorted(agg):
        row = short(name).ljust(62)
        for c in counters:
            vals = agg[name].get(c, [])
            row += (f"{sum(vals) / len(vals):.4g}" if vals else "-").rjust(24)
        print(row)


if __name__ == "__main__":
    main()
