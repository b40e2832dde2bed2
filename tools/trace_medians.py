"""Per-kind launch statistics of a rocprofv3 --kernel-trace CSV of bench.py (tools/profile_round.sh):
median / mean / min duration of the forward, dX, fused last layer, dX0 and dW GEMMs, beside the
bench line's own event-timed forward.

    python tools/trace_medians.py gpurun_out/prof_r20/trace/run_kernel_trace.csv gpurun_out/prof_r20/bench.json out.json
"""
from __future__ import annotations

import csv
import json
import re
import statistics
import sys

# gemm_nt_kernel<NtCfg<256, 256, ..., true>, MODE, HEAD, QUEUE>: the ping-pong instantiations by mode
KINDS = {"inner_fwd": r"gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, 0,",
         "bwd_dx": r"gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, 1,",
         "head_fwd": r"gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, 7,",
         "bwd_dx0": r"gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, 2,",
         "bwd_dw": r"gemm_tn_kernel<"}


def main(trace: str, bench: str, out: str) -> None:
    durs: dict[str, list[float]] = {k: [] for k in KINDS}
    with open(trace) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            for k, pat in KINDS.items():
                if re.search(re.escape(pat), name):
                    durs[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    res = {k: {"launches": len(v), "median_ms": statistics.median(v), "mean_ms": statistics.fmean(v),
               "min_ms": min(v)} for k, v in durs.items() if v}
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    res["bench_events_inner_fwd_avg_ms"] = line["kernels"]["inner_fwd"]["avg_ms"]
    res["note"] = ("rocprofv3 --kernel-trace of bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-recon-snr "
                   "(tools/profile_round.sh); the mean includes the warm-up steps' first launches, the median "
                   "is the steady state")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v["median_ms"] for k, v in res.items() if isinstance(v, dict)}))


if __name__ == "__main__":
    main(*sys.argv[1:4])
