"""MFMA utilisation per kernel from a rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass.

SQ_VALU_MFMA_BUSY_CYCLES counts MFMA busy cycles summed over all SIMDs (16 per
v_mfma_f32_16x16x32_f16: MI355X_MICROARCH.md, constants table); GRBM_GUI_ACTIVE counts GPU-busy
cycles summed over the 8 XCDs.  So
    clock_GHz   = (GUI / 8) / duration
    mfma_util   = MFMA_BUSY / ((GUI / 8) * SIMDs)      (SIMDs = 4 x CUs = 1024)
i.e. the fraction of the SIMDs' cycles at the clock the kernel actually ran at (the
spec-peak fraction in bench.py's roofline also absorbs the clock drop below 2.4 GHz).

What it is NOT: an independent busy measurement.  On gfx950 SQ_VALU_MFMA_BUSY_CYCLES equals the
issued MFMA count x 16 (2^31 for every 2^20 x 1024 x 1024 GEMM in every profile), so mfma_util is
ideal MFMA cycles / (duration x clock): the kernel time and the clock restated.  Its one use is
the clock (GRBM_GUI_ACTIVE / duration) it folds in.

    python tools/pmc_mfma.py OUT.json DIR [kernel_trace.csv]
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024
XCDS = 8


def main():
    out_path, d = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                k = {c.lower(): c for c in row}
                disp = row[k.get("dispatch_id", k.get("correlation_id", "kernel_name"))]
                per[(row[k["kernel_name"]], disp)][row[k["counter_name"]]] += float(row[k["counter_value"]])
    agg = defaultdict(lambda: defaultdict(list))
    for (name, _), ctrs in per.items():
        for c, v in ctrs.items():
            agg[name][c].append(v)
    res = {}
    for name, ctrs in agg.items():
        busy = ctrs.get("SQ_VALU_MFMA_BUSY_CYCLES", [])
        gui = ctrs.get("GRBM_GUI_ACTIVE", [])
        if not busy or not gui or sum(busy) == 0:
            continue
        b, g = sum(busy) / len(busy), sum(gui) / len(gui)
        res[name] = {"dispatches": len(busy), "mfma_busy_cycles": b, "gui_active_cycles": g,
                     "mfma_util": b / (g / XCDS * SIMDS)}
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
    for name, v in sorted(res.items(), key=lambda kv: -kv[1]["mfma_busy_cycles"]):
        print(f"{v['mfma_util']:.3f}  {name[:110]}")


if __name__ == "__main__":
    main()
