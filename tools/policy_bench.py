"""Cache-policy A/B of the NT GEMM operand streams (measurement only, never the product): builds
libsiren_hip variants whose X / W LDS-DMA loads carry an explicit policy (SIREN_XPOL /
SIREN_WPOL: 0 default, 1 nt, 2 sc1, 3 sc0 sc1) and times siren_inner_fwd / siren_inner_bwd_dx
of each at the headline shape, interleaved rounds in one process (HIP events).

    python tools/policy_bench.py [--variants 00,10,20,01] [--rounds 5] [--reps 5] [--build-only]
    python tools/policy_bench.py --variants 10 --one      (one variant, for a rocprofv3 --pmc pass)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lib_path(v: str) -> str:
    return os.path.join(ROOT, "inr-for-audio_amd", f"libsiren_hip_pol{v}.so")


def build(variants):
    import __graft_entry__ as ge
    for v in variants:
        ge.build_diagnostic([f"SIREN_XPOL={v[0]}", f"SIREN_WPOL={v[1]}"], os.path.basename(lib_path(v)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="00,10,20,01")
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--one", action="store_true", help="time only the first variant (PMC passes)")
    args = ap.parse_args()
    variants = args.variants.split(",")
    if args.build_only:
        build(variants)
        return
    import torch
    from inr_for_audio_amd import _lib
    libs = {}
    for v in variants:
        lb = ctypes.CDLL(lib_path(v), mode=os.RTLD_LOCAL)
        for name in ("siren_inner_fwd", "siren_inner_bwd_dx", "siren_set_option"):
            res, argt = _lib._SIGS[name]
            getattr(lb, name).restype, getattr(lb, name).argtypes = res, argt
        libs[v] = lb
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    s = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.rand(R, H, device=dev, generator=g) * 2 - 1).half()
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * math.sqrt(6 / H) / 30).half()
    WT = W.t().contiguous()
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    Y, C = torch.empty(R, H, dtype=torch.half, device=dev), torch.empty(R, H, dtype=torch.half, device=dev)
    dZ = (torch.randn(R, H, device=dev, generator=g) * 1e-3).half()
    dZp = torch.empty_like(Y)
    part = torch.empty(R // 128, 3, H, device=dev)
    flops = 2.0 * R * H * H
    cases = {}
    for v, lb in libs.items():
        cases[f"fwd_{v}"] = lambda lb=lb: lb.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(Y),
                                                              P(C), None, None, s)
        cases[f"dx_{v}"] = lambda lb=lb: lb.siren_inner_bwd_dx(P(dZ), P(WT), P(C), ctypes.c_float(30.0), R, H, None,
                                                                P(dZp), P(part), s)
        if args.one:
            break
    times = {k: [] for k in cases}
    for _ in range(args.rounds):
        for name, fn in cases.items():
            assert fn() == 0, name
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / args.reps)
    out = {}
    for k, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        out[k] = {"median_ms": med, "min_ms": ts[0], "tflops": flops / (med * 1e-3) / 1e12}
    print(json.dumps({"rows": R, "hidden": H, "results": out}, indent=1))


if __name__ == "__main__":
    main()
