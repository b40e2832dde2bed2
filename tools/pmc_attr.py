"""Cycle attribution of the NT GEMM kernels from rocprofv3 SQ / TCC counter passes.

Inputs: the counter-collection CSVs of three --pmc passes over tools/ab_bench.py --only fwd,dx
(pass A: SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS + GRBM_GUI_ACTIVE; pass B: SQ_INSTS_VALU SQ_INSTS_MFMA
SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM +
GRBM_GUI_ACTIVE; pass C: TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum + GRBM_GUI_ACTIVE).

Per kernel (averaged over its dispatches):
  * the wave-state split SQ_WAIT_ANY (parked at s_waitcnt / s_barrier) + SQ_WAIT_INST_ANY (issue
    stall: MFMA pipe, dependencies) + SQ_ACTIVE_INST_ANY (issuing) = SQ_WAVE_CYCLES (quad-cycles,
    MI355X_MICROARCH.md PMC notes), as fractions;
  * the SIMD-cycle budget at the clock the kernel ran at (GRBM_GUI_ACTIVE / 8 = cycles per XCD):
    MFMA pipe busy = SQ_INSTS_MFMA x 16 / 1024 SIMDs (v_mfma_f32_16x16x32_f16: 16 cycles), the
    non-MFMA VALU issue = (SQ_INSTS_VALU - SQ_INSTS_MFMA) instructions (SQ_INSTS_VALU counts the
    MFMAs) at their per-instruction issue cost (`--valu-cyc`, 4-cycle wave64 ops plus 8-cycle
    transcendentals: the forward epilogue's mix averages 5.2), and the rest;
  * L2: read-request hit rate and the fabric read / write bytes (x128 / x64 B per request; the
    read count equals FETCH_SIZE / 64 x 2 -- the gfx950 correction).

    python tools/pmc_attr.py OUT.json DIR_A DIR_B DIR_C [--valu-cyc 5.2]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

SIMDS, XCDS, MFMA_CYC = 1024, 8, 16
NT = re.compile(r"gemm_nt_kernel<siren::NtCfg<([^>]*)>, (\d+), (true|false)(?:, (true|false))?(?:, (true|false))?>")
ONE = re.compile(r"nt_fwd_one<(\d+), (\d+)>")
MODES = {"0": "forward (NT_FWD)", "1": "dX (NT_DX)", "2": "dX0", "7": "fused last layer (NT_FWD_HB)"}


def load(dirs):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    for d in dirs:
        acc = defaultdict(float)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f, newline="") as fh:
                for row in csv.DictReader(fh):
                    k = {c.lower(): c for c in row}
                    disp = row[k.get("dispatch_id", k.get("correlation_id", "kernel_name"))]
                    acc[(row[k["kernel_name"]], disp, row[k["counter_name"]])] += float(row[k["counter_value"]])
        for (name, _, ctr), v in acc.items():
            per[name][ctr].append(v)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--valu-cyc", type=float, default=5.2)
    args = ap.parse_args()
    per = load(args.dirs)
    res = {}
    for name, ctrs in per.items():
        m = NT.search(name)
        m1 = ONE.search(name)
        tn = "gemm_tn_kernel<" in name
        if not m and not m1 and not tn:
            continue
        a = {c: sum(v) / len(v) for c, v in ctrs.items()}
        if tn:
            key = "dW (split-K TN)"
        elif m1:
            key = f"forward one wave per SIMD (pipe 5, NK {m1.group(1)}, diag {m1.group(2)})"
        else:
            key = f"{MODES.get(m.group(2), 'mode ' + m.group(2))}{' +head' if m.group(3) == 'true' else ''}" \
                  f"{' queue' if m.group(4) == 'true' else ''}{' lines' if m.group(5) == 'true' else ''}"
        r = {"kernel": name, "dispatches": min(len(v) for v in ctrs.values())}
        gui = a.get("GRBM_GUI_ACTIVE")
        if all(c in a for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")):
            w = a["SQ_WAVE_CYCLES"]
            r["wave_state"] = {"wait_any (waitcnt/barrier)": a["SQ_WAIT_ANY"] / w,
                               "wait_inst_any (issue stall, MFMA pipe)": a["SQ_WAIT_INST_ANY"] / w,
                               "active_inst_any (issuing)": a["SQ_ACTIVE_INST_ANY"] / w,
                               "active_inst_valu": a.get("SQ_ACTIVE_INST_VALU", 0) / w,
                               "active_inst_lds": a.get("SQ_ACTIVE_INST_LDS", 0) / w,
                               "sum_check": (a["SQ_WAIT_ANY"] + a["SQ_WAIT_INST_ANY"] + a["SQ_ACTIVE_INST_ANY"]) / w}
        if gui and "SQ_INSTS_MFMA" in a:
            cyc = gui / XCDS  # cycles per XCD over the dispatch = SIMD-cycles per SIMD
            mfma = a["SQ_INSTS_MFMA"] * MFMA_CYC / SIMDS
            valu_n = (a.get("SQ_INSTS_VALU", 0) - a["SQ_INSTS_MFMA"]) / SIMDS
            valu = valu_n * args.valu_cyc
            r["simd_cycles"] = {"total": cyc, "mfma_pipe": mfma / cyc, "non_mfma_valu_issue": valu / cyc,
                                "rest (barrier / waitcnt / memory stalls, LDS and SALU issue)": 1 - (mfma + valu) / cyc,
                                "non_mfma_valu_instr_per_simd": valu_n,
                                "salu_instr_per_simd": a.get("SQ_INSTS_SALU", 0) / SIMDS,
                                "lds_instr_per_simd": a.get("SQ_INSTS_LDS", 0) / SIMDS,
                                "wait_inst_lds_frac_of_wave_cycles": a.get("SQ_WAIT_INST_LDS", 0) / a["SQ_WAVE_CYCLES"]
                                if "SQ_WAVE_CYCLES" in a else None,
                                "vmem_rd_instr": a.get("SQ_INSTS_VMEM_RD"), "vmem_wr_instr": a.get("SQ_INSTS_VMEM_WR")}
        if "TCC_HIT_sum" in a:
            rd, wr = a.get("TCC_EA0_RDREQ_sum", 0), a.get("TCC_EA0_WRREQ_sum", 0)
            r["l2"] = {"hit_rate (reads and writes)": a["TCC_HIT_sum"] / (a["TCC_HIT_sum"] + a["TCC_MISS_sum"]),
                       "fabric_read_GB (x128 B)": rd * 128 / 1e9, "fabric_write_GB (x64 B)": wr * 64 / 1e9}
        res[key] = r
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, r in res.items():
        s = r.get("simd_cycles", {})
        print(f"{k:40s} mfma {s.get('mfma_pipe', 0):.3f} valu {s.get('non_mfma_valu_issue', 0):.3f} "
              f"rest {s.get('rest (barrier / waitcnt / memory stalls, LDS and SALU issue)', 0):.3f} "
              f"clock {s.get('total', 0):.3g} cyc; l2 {r.get('l2', {})}")


if __name__ == "__main__":
    main()
