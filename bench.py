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

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel class, timed with
HIP events inside the timed region; `cpu_baseline` times the torch-CPU port of the same
step (oracle/torch_cpu_step.py) on a bounded sample on rank 0 at N = 1.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
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


KIND_MATCH = {  # profile kind -> substrings of the rocprofv3 kernel name
    "inner_fwd": ("gemm_nt_kernel", ", 0, false>"),
    "bwd_dx": ("gemm_nt_kernel", ", 1, false>"),
    "bwd_dx0": ("gemm_nt_kernel", ", 2, false>"),
    "bwd_dw": ("gemm_tn_kernel", ""),
}


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
    a, b = KIND_MATCH[kind]

    def avg(counter):
        vals = [v["avg_KB_per_dispatch"] for k, v in pmc.get(counter, {}).items() if a in k and b in k]
        return sum(vals) / len(vals) if vals else None
    fetch, write = avg("FETCH_SIZE"), avg("WRITE_SIZE")
    if fetch is None or write is None:
        return None, None
    return (2.0 * fetch + write) * 1024.0, os.path.relpath(files[-1], ROOT)


def pmc_mfma_util(kind: str):
    """MFMA utilisation of `kind` at its actual clock from the newest committed
    profiles/r*/bench_pmc_mfma.json (tools/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES over the SIMD
    cycles implied by GRBM_GUI_ACTIVE), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "bench_pmc_mfma.json")))
    if not files or kind not in KIND_MATCH:
        return None
    with open(files[-1]) as f:
        pmc = json.load(f)
    a, b = KIND_MATCH[kind]
    vals = [v["mfma_util"] for k, v in pmc.items() if a in k and b in k]
    return sum(vals) / len(vals) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=5, help="SIREN L: sine layers incl. the first")
    ap.add_argument("--coords", type=int, default=1 << 20, help="coordinates per GPU (weak scaling)")
    ap.add_argument("--omega0", type=float, default=3000.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-coords", type=int, default=65536)
    ap.add_argument("--cpu-steps", type=int, default=3)
    args = ap.parse_args()

    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd import _lib
    from inr_for_audio_amd.engine import SirenEngine, round_up
    from inr_for_audio_amd.models import SirenWithSnakeTanh

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device(f"cuda:{local}")
    lib = _lib.load()

    H, L = args.hidden, args.layers - 1
    per_gpu = round_up(args.coords, 128)
    n_total = per_gpu * world
    # this rank's shard of the global linspace grid, generated on device (bit-exact linspace)
    coords = torch.empty(per_gpu, dtype=torch.float32, device=dev)
    _lib.check(lib.siren_coords_fill(coords.data_ptr(), per_gpu, rank * per_gpu, n_total,
                                     torch.cuda.current_stream(dev).cuda_stream), "coords_fill")
    target = 0.5 * torch.sin(2300.0 * coords) + 0.3 * torch.sin(7100.0 * coords + 0.5)

    torch.manual_seed(0)
    model = SirenWithSnakeTanh(1, 1, H, L, 0, 0, first_omega_0=args.omega0, hidden_omega_0=30.0)
    eng = SirenEngine(model, coords.reshape(-1, 1), target, n_total=n_total, micro_batch=per_gpu,
                      hist_cap=args.warmup + args.steps + 1, device=dev)
    for _ in range(args.warmup):
        eng.step()
    torch.cuda.synchronize(dev)

    _lib.check(lib.siren_profile_enable(64 * (args.steps + 1) * (2 * L + 8)), "profile_enable")
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
    prof = _lib.profile_read()
    _lib.check(lib.siren_profile_enable(0), "profile_disable")
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    loss = eng.last_loss()

    flops_gemm = 2.0 * per_gpu * H * H          # one hidden-layer GEMM launch (fwd, dX or dW)
    kernels = {}
    for k, (ms, n) in prof.items():
        if n:
            kernels[k] = {"launches_per_step": n / args.steps, "avg_ms": ms / n,
                          "ms_per_step": ms / args.steps}
    for k in ("inner_fwd", "bwd_dx", "bwd_dw", "bwd_dx0"):
        if k in kernels:
            kernels[k]["tflops"] = flops_gemm / (kernels[k]["avg_ms"] * 1e-3) / 1e12
    gemm_kinds = [k for k in ("inner_fwd", "bwd_dx", "bwd_dw", "bwd_dx0") if k in kernels]
    dom = max(gemm_kinds, key=lambda k: kernels[k]["ms_per_step"])
    achieved = kernels[dom]["tflops"]
    inner_flops_step = 6.0 * per_gpu * H * H * L
    gemm_ms_step = sum(kernels[k]["ms_per_step"] for k in gemm_kinds)

    traffic, traffic_src = pmc_traffic(dom) if (H == 1024 and per_gpu == 1 << 20) else (None, None)
    ms_per_step = elapsed / args.steps * 1e3
    value = n_total * args.steps / elapsed
    result = {
        "metric": METRIC, "value": value, "unit": "coord-samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp16",
        "data": "synthetic two-tone signal on the linspace grid; random-init weights (seed 0)",
        "config": {"workload": f"SIREN {args.layers}x{H} full-batch fit step, {per_gpu} coords/GPU",
                   "global_batch": n_total, "coords_per_gpu": per_gpu, "hidden": H,
                   "layers": args.layers, "omega0": args.omega0, "hidden_omega": 30.0,
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": achieved, "peak": PEAK_BF16_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / PEAK_BF16_TFLOPS, "traffic": traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     "flops_per_launch": flops_gemm,
                     "hbm_gbs_at_traffic": (traffic / (kernels[dom]["avg_ms"] * 1e-3) / 1e9)
                     if traffic else None,
                     "mfma_util_at_clock_pmc": pmc_mfma_util(dom) if (H == 1024 and per_gpu == 1 << 20) else None},
        "step_mfma_frac": inner_flops_step / (ms_per_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS,
        "gemm_mfma_frac": inner_flops_step / (gemm_ms_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS,
        "kernels": kernels,
        "final_loss": loss,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import torch_cpu_step
        threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
        cb = torch_cpu_step.time_steps(args.cpu_coords, H, L, steps=args.cpu_steps, threads=threads,
                                       omega0=args.omega0)
        result["cpu_baseline"] = {
            "value": cb["coord_samples_per_sec"], "unit": "coord-samples/s", "cores": cb["threads"],
            "kind": "port",
            "sample": f"torch-CPU fp32 port of run.py's step (oracle/torch_cpu_step.py), SIREN "
                      f"{args.layers}x{H}, {args.cpu_coords} coords, median of steps 2..{args.cpu_steps}, "
                      f"{cpu_model()}"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
