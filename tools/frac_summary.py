"""The GEMMs' spec-peak fractions three ways, with the clock beside them: HIP events
over bench.py's timed region (the bench line), the rocprofv3 kernel-trace mean and median of the same
build on the same box, and the achieved shader clock = GRBM_GUI_ACTIVE / 8 (cycles per XCD) over the
trace's median duration, so that box-to-box DVFS is told apart from kernel changes.  frac_at_2.4GHz /
clock_ratio = the fraction the same cycles would give at the spec clock.

    python tools/frac_summary.py profiles/r22        (bench.json, kernel_trace_medians.json, bench_pmc_mfma.json)
"""
from __future__ import annotations

import json
import os
import re
import sys

PEAK_TF = 2500.0
SPEC_GHZ = 2.4
FLOP = 2.0 * (1 << 20) * 1024 * 1024  # one 2^20 x 1024 x 1024 GEMM launch (cfg2)
PMC_KIND = {"inner_fwd": r"gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, 0,",
            "bwd_dx": r"gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, 1,",
            "head_fwd": r"gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, 7,",
            "bwd_dx0": r"gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, 2,",
            "bwd_dw": r"gemm_tn_kernel<"}


def frac(ms: float) -> float:
    return FLOP / (ms * 1e-3) / 1e12 / PEAK_TF


def main(d: str) -> None:
    line = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
    med = json.load(open(os.path.join(d, "kernel_trace_medians.json")))
    pmc = json.load(open(os.path.join(d, "bench_pmc_mfma.json")))
    out = {"source": {"events": "bench.json kernels[*].avg_ms", "rocprof": "kernel_trace_medians.json",
                      "clock": "bench_pmc_mfma.json GRBM_GUI_ACTIVE / 8 over the trace median"}}
    for kind, pat in PMC_KIND.items():
        r = {}
        if kind in line.get("kernels", {}):
            ev = line["kernels"][kind]["avg_ms"]
            r["events"] = {"ms": ev, "frac": frac(ev)}
        if kind in med:
            r["rocprof_mean"] = {"ms": med[kind]["mean_ms"], "frac": frac(med[kind]["mean_ms"])}
            r["rocprof_median"] = {"ms": med[kind]["median_ms"], "frac": frac(med[kind]["median_ms"])}
        gui = [v["gui_active_cycles"] for k, v in pmc.items() if re.search(re.escape(pat), k)]
        if gui and "rocprof_median" in r:
            ghz = sum(gui) / len(gui) / 8 / (r["rocprof_median"]["ms"] * 1e-3) / 1e9
            r["clock_ghz"] = ghz
            r["frac_at_own_clock"] = r["rocprof_median"]["frac"] * SPEC_GHZ / ghz
        out[kind] = r
    json.dump(out, open(os.path.join(d, "frac_summary.json"), "w"), indent=1)
    for k, r in out.items():
        if k != "source":
            print(k, {a: (round(b["frac"], 4) if isinstance(b, dict) else round(b, 3)) for a, b in r.items()})


if __name__ == "__main__":
    main(sys.argv[1])
