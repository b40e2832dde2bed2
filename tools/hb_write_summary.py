"""Per-library WRITE_SIZE / FETCH_SIZE of the fused last layer from tools/hb_write_probe.py runs under
rocprofv3 --pmc (one counter per pass) and, optionally, mean durations from a --kernel-trace run.

    python tools/hb_write_summary.py OUT.json --probe-log gpurun_out/t2/hbw_write.log \\
        --pmc gpurun_out/t2/hbw_write gpurun_out/t2/hbw_fetch --trace gpurun_out/t2/hbw_trace

FETCH_SIZE is doubled (gfx950: it reports half the bytes of a 16-B/lane streaming read,
MI355X_MICROARCH.md §HBM); WRITE_SIZE is exact.  Both are KB per dispatch.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

HB = re.compile(r"gemm_nt_kernel<siren::NtCfg<[^>]*>, (7|8|9), true")


def _order(log):
    for line in open(log):
        line = line.strip()
        if line.startswith("{") and '"order"' in line:
            return json.loads(line)["order"]
    raise SystemExit(f"{log}: no order line")


def _rows(d, pattern):
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                yield {c.lower(): v for c, v in row.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--probe-log", required=True)
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--trace", default="")
    args = ap.parse_args()
    order = _order(args.probe_log)
    res = defaultdict(dict)
    for d in args.pmc:
        per = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
        for r in _rows(d, "*counter_collection.csv"):
            if not HB.search(r["kernel_name"]):
                continue
            per[r["counter_name"]][int(r["dispatch_id"])] += float(r["counter_value"])
        for ctr, disp in per.items():
            ids = sorted(disp)
            if len(ids) != len(order):
                raise SystemExit(f"{d}: {len(ids)} fused dispatches, {len(order)} launches")
            acc = defaultdict(list)
            for i, nm in zip(ids, order):
                acc[nm].append(disp[i] * (2.0 if ctr == "FETCH_SIZE" else 1.0) * 1024 / 1e9)
            for nm, v in acc.items():
                res[nm][f"{ctr}_GB_per_launch" + ("_x2" if ctr == "FETCH_SIZE" else "")] = sum(v) / len(v)
    if args.trace:
        durs = []
        for r in _rows(args.trace, "*kernel_trace.csv"):
            if HB.search(r["kernel_name"]):
                durs.append((int(r["dispatch_id"]), (int(r["end_timestamp"]) - int(r["start_timestamp"])) / 1e6))
        durs.sort()
        if len(durs) == len(order):
            acc = defaultdict(list)
            for (_, ms), nm in zip(durs, order):
                acc[nm].append(ms)
            for nm, v in acc.items():
                res[nm]["mean_ms"] = sum(v) / len(v)
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
