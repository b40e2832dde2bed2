#!/usr/bin/env bash
# Round profile on the GPU box (run through gpurun from the repo root):
#   bench.json              the default bench line (incl. cpu_baseline)
#   trace/                  rocprofv3 --kernel-trace --stats of a bench run (20 steps after 5 warm-up)
#   kernel_trace_medians.json, frac_summary.json  per-GEMM mean / median launch, fractions by events,
#                           rocprof mean and median, and the clock each ran at (GRBM_GUI_ACTIVE)
#   bench_pmc_hbm.json      FETCH_SIZE and WRITE_SIZE, each in its own --pmc pass
#   bench_pmc_mfma.json     SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE: MFMA utilisation per kernel
#   bench_pmc_lds.json      SQ_LDS_IDX_ACTIVE / _BANK_CONFLICT / _UNALIGNED_STALL + GRBM_GUI_ACTIVE
#   fwd_dx_pmc_attribution.json  the forward / dX GEMMs' cycle attribution (tools/pmc_attr.py: 3 SQ / TCC passes)
#   bench_cfg{3,4,5}.json   the other BASELINE configs' bench lines (and bench_live / bench_default: the
#                           reference's width-256 stacks, run.py:466 / run.py:30); trace_<config>/ their
#                           rocprofv3 --kernel-trace --stats
# Every GPU step has its own time limit and the steps are chained with &&.
#   bash tools/profile_round.sh r02 [all|main|configs]
set -euo pipefail
TAG=${1:?round tag, e.g. r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
PART=${2:-all}  # all | main (bench, trace, PMC, attribution) | configs (the cfg3 / cfg4 / cfg5 lines)
cd /tmp && export TMPDIR=/tmp
python3 "$ROOT/__graft_entry__.py"
if [ "$PART" != configs ]; then
timeout -k 10 400 python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-recon-snr > "$OUT/trace.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-recon-snr > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-recon-snr > "$OUT/pmc_write.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_mfma" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-recon-snr > "$OUT/pmc_mfma.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_lds" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-recon-snr > "$OUT/pmc_lds.log" 2>&1 &&
AB="python3 $ROOT/tools/ab_bench.py --libs base=inr-for-audio_amd/libsiren_hip.so --only fwd,dx,fwd_hb,dw --rounds 2 --reps 3" &&
(cd "$ROOT" && timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA GRBM_GUI_ACTIVE --output-format csv -d "$OUT/attr_a" -o run -- $AB > "$OUT/attr_a.log" 2>&1) &&
(cd "$ROOT" && timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d "$OUT/attr_b" -o run -- $AB > "$OUT/attr_b.log" 2>&1) &&
(cd "$ROOT" && timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/attr_c" -o run -- $AB > "$OUT/attr_c.log" 2>&1) &&
python3 "$ROOT/tools/pmc_attr.py" "$OUT/fwd_dx_pmc_attribution.json" "$OUT/attr_a" "$OUT/attr_b" "$OUT/attr_c" &&
python3 "$ROOT/tools/pmc_summary.py" "$OUT/bench_pmc_lds.json" "$OUT/pmc_lds" &&
python3 "$ROOT/tools/pmc_summary.py" "$OUT/bench_pmc_hbm.json" "$OUT/pmc_fetch" "$OUT/pmc_write" &&
python3 "$ROOT/tools/pmc_mfma.py" "$OUT/bench_pmc_mfma.json" "$OUT/pmc_mfma" &&
python3 "$ROOT/tools/trace_medians.py" "$(ls "$OUT"/trace/*kernel_trace.csv | head -n 1)" "$OUT/bench.json" "$OUT/kernel_trace_medians.json" &&
python3 "$ROOT/tools/frac_summary.py" "$OUT" || exit 2
fi
[ "$PART" = main ] && { echo "profile $TAG main done"; exit 0; }
for c in cfg3 cfg4 cfg5 live default; do
  # every config line carries its CPU baseline (cfg3 / cfg4: the SIREN port at the job's thread share)
  timeout -k 10 300 python3 "$ROOT/bench.py" --config $c > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$c" -o run -- \
    python3 "$ROOT/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-recon-snr > "$OUT/trace_$c.log" 2>&1 || exit 3
done
echo "profile $TAG done"
