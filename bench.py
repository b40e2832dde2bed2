"""Headline benchmark: coord-samples/sec trained, SIREN 5x1024, 2^20 coords per GPU.

The metric string is BASELINE.json's (quoted on bf16); the path computes on the fp16 MFMA
(v_mfma_f32_16x16x32_f16: same dense peak and bytes as bf16, fp32 accumulate) because fp16
storage is what keeps the fit within 0.1 dB of the fp32 reference (DESIGN.md "Storage
precision") -- the roofline peak is the same 2.5 PF either way.

One "step" = one full-batch optimizer step of the fused HIP path over the rank's 2^20
coordinates (forward, MSE, backward, gradient all-reduce when N > 1, Adam, plateau
scheduler) -- run.py:156-187.  Synthetic data (a two-tone signal on the linspace grid,
weights random-init at seed 0); inputs resident in HBM before timing.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU, RCCL)

Prints ONE JSON line (rank 0).  `roofline` is for the SineLayer forward GEMM (north_star's
"inner GEMM"; SIREN configs), timed with HIP events inside the timed region; `cpu_baseline` times the torch-CPU port of the same
step (oracle/torch_cpu_step.py) on a bounded sample on rank 0 at N = 1.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import re
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "coord-samples/sec trained, SIREN 5×1024 bf16 at 1/2/4/8 MI355X; recon SNR dB"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 / fp16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_HBM_GBS = 8000.0


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


KIND_MATCH = {  # profile kind -> (kernel-name substring, (MODE, HEAD) of gemm_nt_kernel or None)
    # gemm_nt_kernel<Cfg, MODE, HEAD[, QUEUE[, ACTL]]>: statically walked (QUEUE false) or from the
    # dynamic tile queue (gemm_nt.hip), whole-line Snake / Tanh stores (ACTL); neither is part of the kind
    "inner_fwd": ("gemm_nt_kernel", ("0", "false")),
    "bwd_dx": ("gemm_nt_kernel", ("1", "false")),
    "bwd_dx0": ("gemm_nt_kernel", ("2", "false")),
    "bwd_dw": ("gemm_tn_kernel", None),
    # NT_FWD_HB: the last layer fused with the head, the loss gradient and the head backward
    "head_fwd": ("gemm_nt_kernel", ("7", "true")),
}
_NT_ARGS = re.compile(r"gemm_nt_kernel<siren::NtCfg<[^>]*>, (\d+), (true|false)(?:, (?:true|false)){0,2}>")


def kind_match(kind: str, kernel_name: str) -> bool:
    a, mode_head = KIND_MATCH[kind]
    if a not in kernel_name:
        return False
    if mode_head is None:
        return True
    m = _NT_ARGS.search(kernel_name)
    return m is not None and (m.group(1), m.group(2)) == mode_head


def pmc_traffic(kind: str):
    """Per-launch HBM bytes of `kind` from the newest committed PMC summary
    (profiles/r*/bench_pmc_hbm.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate
    passes).  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
    bytes of a 16-B/lane streaming read, so it is doubled; WRITE_SIZE is exact."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "bench_pmc_hbm.json")))
    if not files or kind not in KIND_MATCH:
        return None, None
    with open(files[-1]) as f:
        pmc = json.load(f)
    def avg(counter):
        vals = [v["avg_KB_per_dispatch"] for k, v in pmc.get(counter, {}).items() if kind_match(kind, k)]
        return sum(vals) / len(vals) if vals else None
    fetch, write = avg("FETCH_SIZE"), avg("WRITE_SIZE")
    if fetch is None or write is None:
        return None, None
    return (2.0 * fetch + write) * 1024.0, os.path.relpath(files[-1], ROOT)


def pmc_attribution(kind: str):
    """The newest committed cycle attribution of the forward GEMM (profiles/r*/fwd_dx_pmc_attribution.json,
    tools/pmc_attr.py over three rocprofv3 SQ / TCC passes): the MFMA pipe's busy fraction of the SIMD
    cycles, the non-MFMA VALU issue and the rest, and the L2 numbers -- or None."""
    import glob
    if kind != "inner_fwd":
        return None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "fwd_dx_pmc_attribution.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        pmc = json.load(f)
    fwd = next((v for k, v in pmc.items() if k.startswith("forward (NT_FWD)")), None)
    if not fwd or "simd_cycles" not in fwd:
        return None
    sc = fwd["simd_cycles"]
    return {"mfma_pipe_busy": sc["mfma_pipe"], "non_mfma_valu_issue": sc["non_mfma_valu_issue"],
            "rest": 1.0 - sc["mfma_pipe"] - sc["non_mfma_valu_issue"],
            "l2_hit_rate": fwd.get("l2", {}).get("hit_rate (reads and writes)"),
            "source": os.path.relpath(files[-1], ROOT)}


CONFIGS = {  # name: (hidden, layers, in_dim, coords per GPU, omega0, grid height per GPU or None)
    "cfg2": (1024, 5, 1, 1 << 20, 3000.0, None),
    "cfg3": (1024, 6, 2, 3_600_000, 3000.0, 1_800_000),
    "cfg4": (512, 5, 2, 1024 * 215, 1000.0, 1024),
    # the reference's own live workload (run.py:466: width 256, a first SineLayer at omega 22000 then
    # num_sine=0, num_snake=4, 10 s of 44.1 kHz audio) and train()'s default stack (run.py:30:
    # num_sine=2, num_snake=2, width 256, omega 22000, a_initial 0.5) on the same 10 s
    "live": (256, 5, 1, 441_000, 22000.0, None),
    "default": (256, 5, 1, 441_000, 22000.0, None),
}
# hidden-layer kinds (num_sine, num_snake) of the configs that are not all-sine
STACKS = {"live": (0, 4), "default": (2, 2)}
A_INITIAL = 0.5  # run.py:30


def siren_bytes_per_row(acts, H, in_dim=1):
    """Algorithmic HBM bytes per coordinate of one fused training step, per launch kind (fp16
    activations, 2 B per element; weights, partials and slabs are O(H^2) per launch and left out).
    acts: 'sine' / 'snake' per hidden layer, the last one fused with the head (NT_FWD_HB*):
      first_fwd   reads the coordinate, writes Y0, C0
      inner_fwd   layer i < L-1: reads X_i, writes Y, C (+ E for Snake)
      head_fwd    layer L-1 + head + loss gradient + head backward: reads X, writes dZ_{L-1}
                  (a Snake's E goes to HBM and back inside the launch: scratch, not counted)
      bwd_dx      into layer i-1, i = L-1 .. 1: reads dZ_i, C_i (+ E_i below a Snake), writes dZ_{i-1}
      bwd_dx0     into the first layer: reads dZ_0, C_0 (partials only)
      bwd_dw      layer i: reads Y_i and dZ_i"""
    e = 2 * H
    L = len(acts)
    by = {"first_fwd": 4 * in_dim + 2 * e, "inner_fwd": 0, "head_fwd": 2 * e, "bwd_dx": 0, "bwd_dx0": 2 * e,
          "bwd_dw": 2 * e * L}
    for i in range(L - 1):
        by["inner_fwd"] += e + e * (3 if acts[i] == "snake" else 2)
    for i in range(L - 1, 0, -1):
        by["bwd_dx"] += e * (4 if acts[i - 1] == "snake" else 3)
    return by


PEAK_F32_TFLOPS = 157.3   # MI355X dense fp32 (f32-input MFMA = the vector rate; MI355X_MICROARCH.md)


def kan_work_per_row(widths):
    """Algorithmic work per coordinate of one KAN training step, per launch kind, for the fused
    design (kan.hip): bytes (activations in and out; the expansions A / dA are recomputed in LDS,
    never stored) and GEMM flops (2 x 9 in x out per layer and product; the B-spline recursion's
    own VALU work is not counted, so the flop fraction is a lower bound).  Per layer l (in -> out),
    following siren_kan_train_step's dispatch:
      kan_fwd  reads X_l (4 in), writes X_{l+1} (4 out);                           2*9*in*out flop
               (not the head below, whose forward runs in its training pass)
      l = 0:                      kan_dw  reads X_0, G_1;                           2*9*in*out
      l > 0, out = 1, in <= 64:   kan_dw  (head: forward, MSE gradient, backward) reads X_l,
                                  y, writes out, g, G_l;                            3 * 2*9*in
      l > 0, out <= 64:           kan_dx  (dW + dX) reads X_l, G_{l+1}, writes G_l; 2 * 2*9*in*out
      l > 0, out > 64:            kan_dw as l = 0, and kan_dx reads X_l, G_{l+1}, writes G_l
    Weights, slabs and partials are O(width^2) per launch, not per row, and left out."""
    by = {"kan_fwd": 0, "kan_dw": 0, "kan_dx": 0}
    fl = {"kan_fwd": 0, "kan_dw": 0, "kan_dx": 0}
    for l in range(len(widths) - 1):
        i, o = widths[l], widths[l + 1]
        if l > 0 and o == 1 and i <= 64:
            by["kan_dw"] += 4 * i + 4 + 8 + 4 * i
            fl["kan_dw"] += 54 * i
            continue
        by["kan_fwd"] += 4 * i + 4 * o
        fl["kan_fwd"] += 18 * i * o
        if l == 0:
            by["kan_dw"] += 4 * i + 4 * o
            fl["kan_dw"] += 18 * i * o
        elif o <= 64:
            by["kan_dx"] += 4 * i + 4 * o + 4 * i
            fl["kan_dx"] += 36 * i * o
        else:
            by["kan_dw"] += 4 * i + 4 * o
            fl["kan_dw"] += 18 * i * o
            by["kan_dx"] += 4 * i + 4 * o + 4 * i
            fl["kan_dx"] += 18 * i * o
    return by, fl


def profiled_steps(eng, args, dev, dist, lib, _lib, records_per_step, dom_of):
    """Time args.steps steps with HIP events around only the dominant launch kind.

    Events around every launch cost a step 2-13% (measured: cfg4 2.35 -> 2.66 ms, cfg5 2.37 ->
    2.51, cfg2 27.6 -> 28.2), so the per-kind breakdown comes from a separate pass of up to 5
    steps with every kind bracketed (not timed); the kind dom_of(breakdown) picks is then the only
    one bracketed inside the timed region, which gives the roofline's per-launch duration live.
    Returns (elapsed_s max over ranks, breakdown, breakdown_steps, dom, (dom_ms, dom_launches))."""
    prof_steps = max(1, min(args.steps, 5))
    _lib.check(lib.siren_profile_mask(0xFFFFFFFF), "profile_mask")
    _lib.check(lib.siren_profile_enable(records_per_step * (prof_steps + 1)), "profile_enable")
    for _ in range(prof_steps):
        eng.step()
    torch.cuda.synchronize(dev)
    breakdown = _lib.profile_read()
    dom = dom_of(breakdown, prof_steps)
    _lib.check(lib.siren_profile_enable(records_per_step * (args.steps + 1)), "profile_enable")
    _lib.check(lib.siren_profile_mask(1 << _lib.PROF_KINDS.index(dom)), "profile_mask")
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.step()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timed = _lib.profile_read()[dom]
    _lib.check(lib.siren_profile_enable(0), "profile_disable")
    _lib.check(lib.siren_profile_mask(0xFFFFFFFF), "profile_mask")
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    return elapsed, breakdown, prof_steps, dom, timed


def dp_report(eng, args, dev, dist, steps: int = 5) -> dict:
    """What a data-parallel run saw, measured after the timed region: the process group's backend
    and world size as torch.distributed reports them, the step with and without the gradient
    all-reduce (comm_enabled off: the same launches minus the exchange; timing only, the ranks'
    weights drift apart afterwards), the difference = the all-reduce time NOT hidden under the
    backward (max over ranks), and the all-reduce of the whole flat gradient vector alone."""
    def timed(fn, k):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        e = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        return float(e.item()) / k * 1e3

    with_comm = timed(eng.step, steps)
    eng.comm_enabled = False
    try:
        without = timed(eng.step, steps)
    finally:
        eng.comm_enabled = True
    alone = timed(lambda: dist.all_reduce(eng.grads), steps)
    return {"backend": dist.get_backend(), "world_size_seen": dist.get_world_size(),
            "rccl": dist.get_backend() == "nccl", "bucketed_overlap": eng._buckets is not None,
            "buckets": len(eng._buckets or []), "allreduce_bytes": eng.grads.numel() * 4,
            "ms_per_step_with_allreduce": with_comm, "ms_per_step_without_allreduce": without,
            "exposed_allreduce_ms_per_step": with_comm - without, "allreduce_alone_ms": alone,
            "steps": steps,
            "note": "after the timed region; exposed = step with the bucketed all-reduce minus the same step "
                    "without it (max over ranks)"}


# recon SNR fixtures (the metric's second half), newest first: the reference's own fit of the
# headline model on gt_bach, written by tests/golden/make_golden.py in the build container
RECON_FIXTURES = [("fit_5x1024_w18000_6s.json", "gt_bach_6s.npz"),
                  ("trajectory_5x1024_w3000_lr3e-5_seeds.json", "gt_bach_1s.npz")]


def recon_snr(dev) -> dict | None:
    """BASELINE's "recon SNR dB" on the bench line (outside the timed region): the headline model
    (SIREN 5x1024) fitted on the fixture's clip with the fixture's hyper-parameters, seed 0, then
    SNR_target of the final weights (utils.py:77-97 calculate_snr(target, model(coords)), the
    quantity run.py:302-335 reports) next to the reference's own value for the same run."""
    import numpy as np
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    from inr_for_audio_amd.utils import calculate_snr, get_coord
    gdir = os.path.join(ROOT, "tests", "golden")
    for fname, tname in RECON_FIXTURES:
        path = os.path.join(gdir, fname)
        if os.path.exists(path):
            break
    else:
        return None
    ref = json.load(open(path))
    run = ref["runs"]["0"]
    target = np.load(os.path.join(gdir, tname))["target"].astype(np.float32)
    coords = get_coord(target.size, 1).reshape(-1, 1)
    torch.manual_seed(0)
    model = SirenWithSnakeTanh(1, 1, ref["hidden"], ref["num_sine"], 0, 0, first_omega_0=ref["omega0"],
                               hidden_omega_0=30.0)
    eng = SirenEngine(model, coords, torch.from_numpy(target), lr=ref["lr0"], min_lr=ref.get("min_lr", 1e-6),
                      factor=ref.get("factor", 0.8), patience=ref["patience"], hist_cap=ref["steps"], device=dev)
    t0 = time.perf_counter()
    eng.step()
    eng.capture_graph()
    eng.run(ref["steps"] - 1)
    torch.cuda.synchronize(dev)
    fit_s = time.perf_counter() - t0
    out = eng.infer(coords.to(dev)).cpu().numpy()
    snr = float(calculate_snr(target, out))
    losses, lrs = eng.history()
    return {"snr_target_db": snr, "reference_snr_target_db": run["snr_target"],
            "delta_db": snr - run["snr_target"], "tolerance_db": 0.1,
            "steps": ref["steps"], "coords": int(target.size), "lr0": ref["lr0"], "patience": ref["patience"],
            "final_lr": float(lrs[-1]), "reference_final_lr": float(run["lr"][-1]),
            "fp16_overflow_steps": eng.guard_state()["overflows"], "fit_seconds": fit_s,
            "fixture": os.path.relpath(path, ROOT),
            "workload": f"SIREN {ref['num_sine'] + 1}x{ref['hidden']}, omega0 {ref['omega0']:g}, gt_bach "
                        f"{target.size} samples, full batch, seed 0: SNR_target of the final weights vs the "
                        f"reference's run of the same fit (make_golden.py)"}


def run_kan(args, world, rank, dev, dist, lib, _lib):
    """cfg5: KAN([1, H, H, 1]) full-batch fit step (KanEngine, siren_kan_train_step)."""
    from inr_for_audio_amd.engine import KanEngine
    from inr_for_audio_amd.kan import KAN
    H = args.hidden or 64
    per_gpu = -(-(args.coords or 441_000) // world) if args.strong else (args.coords or 441_000)
    n_total = per_gpu * world
    coords = torch.empty(per_gpu, 1, dtype=torch.float32, device=dev)
    _lib.check(lib.siren_coords_fill(coords.data_ptr(), per_gpu, rank * per_gpu, n_total,
                                     torch.cuda.current_stream(dev).cuda_stream), "coords_fill")
    t = coords[:, 0]
    target = 0.5 * torch.sin(2300.0 * t) + 0.3 * torch.sin(7100.0 * t + 0.5)
    torch.manual_seed(0)
    widths = [1, H, H, 1]
    eng = KanEngine(KAN(widths), coords, target, n_total=n_total, micro_batch=args.micro_batch or per_gpu,
                    hist_cap=args.warmup + args.steps + 6, device=dev)
    for _ in range(args.warmup):
        eng.step()
    torch.cuda.synchronize(dev)
    rows = per_gpu / eng.n_micro
    bpr, fpr = kan_work_per_row(widths)
    elapsed, prof, psteps, dom, (dom_ms, dom_n) = profiled_steps(
        eng, args, dev, dist, lib, _lib, 64 * eng.n_micro,
        lambda pr, n: max((k for k in bpr if pr[k][1]), key=lambda k: pr[k][0]))
    kernels = {}
    for k, (ms, n) in prof.items():
        if n:
            if k == dom:  # the timed region's own events
                ms, n, steps_k = dom_ms, dom_n, args.steps
            else:
                steps_k = psteps
            kernels[k] = {"launches_per_step": n / steps_k, "avg_ms": ms / n, "ms_per_step": ms / steps_k}
            if k in bpr:
                sec = ms / steps_k * 1e-3
                kernels[k]["bytes_per_step"] = bpr[k] * per_gpu
                kernels[k]["gbs"] = bpr[k] * per_gpu / sec / 1e9
                kernels[k]["tflops"] = fpr[k] * per_gpu / sec / 1e12
    ms_per_step = elapsed / args.steps * 1e3
    step_bytes = sum(bpr.values()) * per_gpu
    step_flops = sum(fpr.values()) * per_gpu
    result = {
        "metric": METRIC, "value": n_total * args.steps / elapsed, "unit": "coord-samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic two-tone signal on the linspace(-1, 1) time grid; random-init KAN (seed 0)",
        "config": {"workload": f"cfg5: KAN({widths}) full-batch fit step, {per_gpu} coords/GPU", "name": "cfg5",
                   "global_batch": n_total, "coords_per_gpu": per_gpu, "widths": widths,
                   "micro_batches_per_gpu": eng.n_micro, "parallelism": f"dp{world}",
                   "backend": args.backend if world > 1 else None},
        # compute-bound once the expansions stay on chip: the fp32 dense peak for the dtype
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": kernels[dom]["tflops"], "peak": PEAK_F32_TFLOPS,
                     "unit": "TFLOP/s", "frac": kernels[dom]["tflops"] / PEAK_F32_TFLOPS, "traffic": None,
                     "peak_note": "fp32 dense (f32 MFMA = vector rate); the chunk products run on "
                                  "v_mfma_f32_16x16x4_f32, the out = 1 head on VALU FMAs; GEMM flops only "
                                  "(the B-spline recursion, recomputed in each of the three passes, is extra "
                                  "VALU work)",
                     "flops_per_row": fpr[dom], "rows_per_launch": rows,
                     "hbm": {"achieved": kernels[dom]["gbs"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": kernels[dom]["gbs"] / PEAK_HBM_GBS, "algorithmic_bytes_per_row": bpr[dom]}},
        "step_flop_frac": step_flops / (ms_per_step * 1e-3) / 1e12 / PEAK_F32_TFLOPS,
        "step_hbm_frac": step_bytes / (ms_per_step * 1e-3) / 1e9 / PEAK_HBM_GBS,
        "step_algorithmic_bytes": step_bytes, "step_gemm_flops": step_flops,
        "kernels": kernels,
        "kernels_source": f"{dom}: HIP events inside the timed region (the only kind bracketed there); "
                          f"the other kinds: a separate untimed pass of {psteps} steps with every launch "
                          f"bracketed",
        "final_loss": eng.last_loss(),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # A quarter of the SIREN sample (the B-spline expansion makes a CPU KAN step slow per
        # coordinate), at the box's CPU share only: at os.cpu_count() = 256 threads the KAN step
        # thrashes 40x (26 s a step, measured).
        n_cpu = max(1024, args.cpu_coords // 4)
        what = (f"torch-CPU fp32 port of run.py's KAN step (oracle/torch_cpu_step.py: efficient-KAN "
                f"KANLinear, kan.py:6-166), KAN({widths}), {n_cpu} coords")
        result["cpu_baseline"] = cpu_baseline_sweep(
            lambda threads, steps: torch_cpu_kan(n_cpu, widths, steps, threads), args, what, share_only=True)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def torch_cpu_kan(n, widths, steps, threads):
    from oracle import torch_cpu_step
    return torch_cpu_step.kan_time_steps(n, tuple(widths), steps=steps, threads=threads)


def cpu_baseline_sweep(fn, args, what, share_only=False):
    """Time the CPU port at the box's CPU share and (unless share_only) at os.cpu_count() threads
    (BASELINE.md CPU plan: median of steps 2..k); the faster is the reported value, the sweep is
    kept beside it."""
    cores = os.cpu_count() or 1
    share = min(cores, int(os.environ.get("OMP_NUM_THREADS") or cores))
    legs = [(share, args.cpu_steps)] + ([] if share_only else [(cores, max(3, args.cpu_steps // 2))])
    sweep = {}
    for threads, steps in legs:
        if threads not in sweep:
            sweep[threads] = fn(threads, steps)
    best = sweep[max(sweep, key=lambda k: sweep[k]["coord_samples_per_sec"])]
    return {"value": best["coord_samples_per_sec"], "unit": "coord-samples/s", "cores": best["threads"],
            "kind": "port", "threads": best["threads"], "cpu_count": cores,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "threads_sweep": {str(k): {"value": v["coord_samples_per_sec"], "steps": v["steps"],
                                       "step_s": [round(x, 3) for x in v["step_times"]]} for k, v in sweep.items()},
            "sample": f"{what}, median of steps 2..k, best of torch.set_num_threads({sorted(sweep)}) "
                      f"(os.cpu_count() = {cores}), {cpu_model()}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS) + ["cfg5"], default="cfg2",
                    help="cfg2 (default) .. cfg5: BASELINE.json's configs; live / default: the reference's run.py:466 "
                         "workload / train()'s default stack (width 256, Snake layers)")
    ap.add_argument("--hidden", type=int, default=None, help="override the config's width")
    ap.add_argument("--layers", type=int, default=None, help="SIREN L: sine layers incl. the first")
    ap.add_argument("--coords", type=int, default=None, help="coordinates per GPU (weak scaling), or the global "
                    "batch with --strong")
    ap.add_argument("--strong", action="store_true", help="strong scaling (cfg2 / cfg5): the global batch "
                    "(--coords, default the config's) is fixed and split over the ranks")
    ap.add_argument("--emulate-ranks", type=int, default=None, help="one process runs rank 0's shard of a "
                    "G-rank job (per-rank compute of a scaling curve on one GPU; n_total stays global; with "
                    "--strong the global batch is split G ways); `value` is then this rank's coord-samples/s")
    ap.add_argument("--omega0", type=float, default=None)
    ap.add_argument("--micro-batch", type=int, default=None, help="rows per fused micro-batch "
                    "(default: the whole per-GPU batch)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-recon-snr", action="store_true", help="skip the recon-SNR fit (cfg2, N = 1)")
    ap.add_argument("--cpu-coords", type=int, default=65536)
    ap.add_argument("--cpu-steps", type=int, default=6)
    ap.add_argument("--set-option", action="append", default=[], metavar="K=V",
                    help="measurement only: siren_set_option(K, V) before the engine is built (e.g. 9=0: the last "
                         "layer unfused); the line lists them in config.options")
    ap.add_argument("--lib", default=None, help="measurement only: time another build of the library (a variant "
                    "from tools/variants.py), checked for its ABI; the line then names it in config.lib")
    args = ap.parse_args()

    import __graft_entry__ as ge
    ge.build(diag=False)  # the SIREN_DIAG test library is never loaded here
    from inr_for_audio_amd import _lib
    from inr_for_audio_amd.engine import SirenEngine, round_up
    from inr_for_audio_amd.models import SirenWithSnakeTanh

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; more ranks than GPUs (a rehearsal on a 1-GPU box, --backend gloo) share
    ndev = torch.cuda.device_count()
    dev = torch.device(f"cuda:{local % max(ndev, 1)}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        dist.init_process_group(args.backend)
    lib = _lib.load(os.path.join(ROOT, args.lib)) if args.lib else _lib.load()
    for kv in args.set_option:
        k, v = (int(x) for x in kv.split("="))
        _lib.check(lib.siren_set_option(k, v), f"siren_set_option({k}, {v})")
    ranks = world
    if args.emulate_ranks:
        if world != 1 or args.config not in ("cfg2", "live", "default"):
            raise SystemExit("--emulate-ranks: one process, a 1-D (linspace) config")
        ranks = args.emulate_ranks
    if args.config == "cfg5":
        return run_kan(args, world, rank, dev, dist, lib, _lib)

    cfg_h, cfg_l, in_dim, cfg_coords, cfg_w0, grid_h = CONFIGS[args.config]
    H = args.hidden or cfg_h
    L = (args.layers or cfg_l) - 1
    omega0 = args.omega0 if args.omega0 is not None else cfg_w0
    stream = torch.cuda.current_stream(dev).cuda_stream
    if in_dim == 1:
        per_gpu = round_up(-(-(args.coords or cfg_coords) // ranks) if args.strong else (args.coords or cfg_coords), 128)
        n_total = per_gpu * ranks
        # this rank's shard of the global linspace grid, generated on device (bit-exact linspace)
        coords = torch.empty(per_gpu, 1, dtype=torch.float32, device=dev)
        _lib.check(lib.siren_coords_fill(coords.data_ptr(), per_gpu, rank * per_gpu, n_total, stream),
                   "coords_fill")
        t = coords[:, 0]
        target = 0.5 * torch.sin(2300.0 * t) + 0.3 * torch.sin(7100.0 * t + 0.5)
        grid = "linspace(-1, 1) time grid"
    else:
        # cfg3: (time, channel) rows of a height x 2 grid, time-major (utils.py:211-220);
        # cfg4: (bin, frame) rows of a 1024 x 215 grid, bin-major (utils.py:382-400).  cfg3 shards
        # the global grid over the ranks; cfg4 (1 GPU in BASELINE) replicates it per rank.
        width = 2 if args.config == "cfg3" else (args.coords or cfg_coords) // grid_h
        if args.config == "cfg3":
            per_gpu = (args.coords or cfg_coords) // 2 * 2
            height, offset = per_gpu // 2 * world, rank * per_gpu
            grid = f"MultiWaveformFitting (t, ch) grid, {height} instants x 2 channels"
        else:
            height, offset = grid_h, 0
            per_gpu = height * width
            grid = f"MDCTFitting (bin, frame) grid, {height} bins x {width} frames"
        n_total = per_gpu * world
        coords = torch.empty(per_gpu, 2, dtype=torch.float32, device=dev)
        _lib.check(lib.siren_coords_fill_grid(coords.data_ptr(), per_gpu, offset, height, width, stream),
                   "coords_fill_grid")
        t, ch = coords[:, 0], coords[:, 1]
        target = torch.where(ch < 0, 0.5 * torch.sin(2300.0 * t), 0.4 * torch.sin(3100.0 * t + 1.0)) \
            + 0.2 * torch.sin(7100.0 * t + 0.5 * ch)

    torch.manual_seed(0)
    n_sine, n_snake = STACKS.get(args.config, (L, 0))
    if args.config in STACKS:
        L = n_sine + n_snake
        layers_kind = ["sine"] * n_sine + ["snake"] * n_snake
        model = SirenWithSnakeTanh(in_dim, 1, H, n_sine, n_snake, 0, first_omega_0=omega0, hidden_omega_0=30.0,
                                   a_initial=A_INITIAL)
    else:
        layers_kind = ["sine"] * L
        model = SirenWithSnakeTanh(in_dim, 1, H, L, 0, 0, first_omega_0=omega0, hidden_omega_0=30.0)
    eng = SirenEngine(model, coords, target, n_total=n_total, micro_batch=args.micro_batch or per_gpu,
                      hist_cap=args.warmup + args.steps + 6, device=dev)
    for _ in range(args.warmup):
        eng.step()
    torch.cuda.synchronize(dev)

    gemm_all = ("inner_fwd", "head_fwd", "bwd_dx", "bwd_dw", "bwd_dx0")

    bpr = siren_bytes_per_row(layers_kind, H, in_dim) if args.config in STACKS else None

    def pick(pr, n):
        # the width-256 Snake stacks are HBM-bound: the roofline names the kind with the most time per step
        if bpr is not None:
            return max((k for k in bpr if pr[k][1]), key=lambda k: pr[k][0])
        # pinned to north_star's "inner GEMM": the SineLayer forward (models.py:114-115), which is
        # also the kind with the most time per step by rocprof (3 launches at cfg2).  The forward,
        # dX and dW kinds sit within 3 % of each other per step, so choosing by time in the untimed
        # pre-pass flipped the line's kernel from box to box.  A stack with no plain
        # hidden forward (one hidden layer: only the fused last layer) falls back to the most time.
        if pr["inner_fwd"][1]:
            return "inner_fwd"
        return max((k for k in gemm_all if pr[k][1]), key=lambda k: pr[k][0])

    elapsed, prof, psteps, dom, (dom_ms, dom_n) = profiled_steps(
        eng, args, dev, dist, lib, _lib, 64 * (2 * L + 8) * eng.n_micro, pick)
    loss = eng.last_loss()

    # one hidden-layer GEMM launch (fwd, dX or dW) covers one micro-batch of coordinates
    flops_gemm = 2.0 * (per_gpu / eng.n_micro) * H * H
    kernels = {}
    for k, (ms, n) in prof.items():
        if n:
            if k == dom:  # the timed region's own events
                ms, n, steps_k = dom_ms, dom_n, args.steps
            else:
                steps_k = psteps
            kernels[k] = {"launches_per_step": n / steps_k, "avg_ms": ms / n, "ms_per_step": ms / steps_k}
    for k in gemm_all:
        if k in kernels:
            kernels[k]["tflops"] = flops_gemm / (kernels[k]["avg_ms"] * 1e-3) / 1e12
    gemm_kinds = [k for k in gemm_all if k in kernels]
    achieved = kernels[dom]["tflops"]
    inner_flops_step = 6.0 * per_gpu * H * H * L
    gemm_ms_step = sum(kernels[k]["ms_per_step"] for k in gemm_kinds)

    headline = args.config == "cfg2" and H == 1024 and L == 4 and per_gpu == 1 << 20 and eng.n_micro == 1
    traffic, traffic_src = pmc_traffic(dom) if headline else (None, None)
    ms_per_step = elapsed / args.steps * 1e3
    value = (n_total if ranks == world else per_gpu) * args.steps / elapsed
    layers = L + 1
    result = {
        "metric": METRIC, "value": value, "unit": "coord-samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "strong" if args.strong and in_dim == 1 else "weak",
        "vs_baseline": None, "dtype": "fp16",
        "data": f"synthetic tone mix on the {grid}; random-init weights (seed 0)",
        "config": {"workload": f"{args.config}: SIREN {layers}x{H} (in = {in_dim}) full-batch fit step, "
                               f"{per_gpu} coords/GPU" + (f" (rank 0 of {ranks} emulated, {n_total} global)"
                                                          if ranks != world else ""),
                   "name": args.config, "global_batch": n_total, "coords_per_gpu": per_gpu, "hidden": H,
                   "layers": layers, "in_features": in_dim, "omega0": omega0, "hidden_omega": 30.0,
                   "micro_batches_per_gpu": eng.n_micro, "parallelism": f"dp{world}",
                   "backend": args.backend if world > 1 else None, "lib": args.lib,
                   "options": args.set_option or None},
        "roofline": {"bound": "mfma", "kernel": dom,
                     "kernel_choice": "pinned: the SineLayer forward GEMM (north_star's inner GEMM), "
                                      "timed with HIP events over the timed region",
                     "achieved": achieved, "peak": PEAK_BF16_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / PEAK_BF16_TFLOPS, "traffic": traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     "flops_per_launch": flops_gemm,
                     "hbm_gbs_at_traffic": (traffic / (kernels[dom]["avg_ms"] * 1e-3) / 1e9)
                     if traffic else None,
                     # the committed cycle attribution of this kernel (tools/pmc_attr.py): MFMA pipe
                     # busy = SQ_INSTS_MFMA x 16 cycles / 1024 SIMDs over the dispatch's cycles
                     # (GRBM_GUI_ACTIVE / 8), and the clock it ran at; frac = busy x clock / 2.4 GHz
                     "pmc_attribution": pmc_attribution(dom) if headline else None},
        # every GEMM kind's spec-peak fraction (the dominant one is `roofline`); head_fwd does the
        # forward GEMM's flops plus the head, loss gradient and head backward
        "gemm_frac_by_kind": {k: kernels[k]["tflops"] / PEAK_BF16_TFLOPS for k in gemm_kinds},
        "step_mfma_frac": inner_flops_step / (ms_per_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS,
        "gemm_mfma_frac": inner_flops_step / (gemm_ms_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS,
        "kernels": kernels,
        "kernels_source": f"{dom}: HIP events inside the timed region (the only kind bracketed there); "
                          f"the other kinds: a separate untimed pass of {psteps} steps with every launch "
                          f"bracketed",
        "final_loss": loss,
        "fp16_overflow_steps": eng.guard_state()["overflows"],
    }
    if ranks != world:
        # fill of the persistent GEMM grids at this shard: 256 x 256 tiles over the CUs
        tiles = (round_up(per_gpu // eng.n_micro, 256) // 256) * (H // 256)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        waves = tiles / cus
        result["emulated"] = {
            "ranks": ranks, "rank": 0, "coords_this_rank": per_gpu, "global_batch": n_total,
            "value_is": "this rank's coord-samples/s (the job's would be ranks x value with no exchange cost)",
            "ideal_job_value": value * ranks, "gemm_tiles_per_launch": tiles, "cus": cus,
            "waves": waves, "wave_tail_frac": (math.ceil(waves) - waves) / math.ceil(waves)}
        result["scaling"] = "strong" if args.strong else "weak"
    if bpr is not None:
        # HBM roofline (width 256: 2 H^2 flop per row against >= 8 H bytes, far below the MFMA ridge)
        fused = prof["head_fwd"][1] > 0
        for k, b in bpr.items():
            if k in kernels:
                kernels[k]["bytes_per_step"] = b * per_gpu
                kernels[k]["gbs"] = b * per_gpu / (kernels[k]["ms_per_step"] * 1e-3) / 1e9
        step_bytes = sum(bpr.values()) * per_gpu
        result["config"]["stack"] = {"first": "sine", "hidden": layers_kind, "a_initial": A_INITIAL,
                                     "reference": "run.py:466" if args.config == "live" else "run.py:30 defaults"}
        result["roofline"] = {
            "bound": "hbm", "kernel": dom, "kernel_choice": "the kind with the most time per step (HBM-bound stack)",
            "achieved": kernels[dom]["gbs"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": kernels[dom]["gbs"] / PEAK_HBM_GBS, "traffic": None,
            "algorithmic_bytes_per_row": bpr[dom] / kernels[dom]["launches_per_step"],
            "rows_per_launch": per_gpu / eng.n_micro, "head_fused": fused,
            "mfma": {"achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_BF16_TFLOPS}}
        result["step_hbm_frac"] = step_bytes / (ms_per_step * 1e-3) / 1e9 / PEAK_HBM_GBS
        result["step_algorithmic_bytes"] = step_bytes
        result["bytes_per_row_by_kind"] = bpr
    if dist is not None:
        result["dist"] = dp_report(eng, args, dev, dist)
    if world == 1 and args.config == "cfg2" and not args.no_recon_snr:
        result["recon_snr"] = recon_snr(dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # BASELINE.md CPU plan: median of steps 2..k with torch.set_num_threads(os.cpu_count()).  On
        # the GPU box os.cpu_count() reports the whole host (256) while the job's CPU share is
        # OMP_NUM_THREADS (16), and 256 threads on that share thrash (6x slower, measured): the
        # headline (cfg2) times both counts and reports the faster, the sweep kept beside it; the
        # other configs time the share only (the thrashing leg costs minutes and never wins).
        from oracle import torch_cpu_step
        n_cpu = args.cpu_coords if args.config not in STACKS else 4 * args.cpu_coords  # width 256: 16x less work/row
        what = (f"torch-CPU fp32 port of run.py's step (oracle/torch_cpu_step.py), SIREN {layers}x{H} "
                f"(in = {in_dim}; hidden {'/'.join(layers_kind)}), {n_cpu} coords")
        result["cpu_baseline"] = cpu_baseline_sweep(
            lambda threads, steps: torch_cpu_step.time_steps(n_cpu, H, n_sine, steps=steps, threads=threads,
                                                             omega0=omega0, in_dim=in_dim, n_snake=n_snake,
                                                             a0=A_INITIAL),
            args, what, share_only=args.config != "cfg2")
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
