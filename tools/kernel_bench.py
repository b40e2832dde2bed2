"""A/B timing of the individual SIREN kernels at the headline shape (2^20 coords x 1024)
through the C-ABI, with HIP events, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24).  Random fp16 data in realistic ranges.

    python tools/kernel_bench.py [--rows 1048576] [--hidden 1024] [--rounds 5] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tiles", default="128,256")
    ap.add_argument("--pipes", default="1,4", help="256x256 NT K-loop variants to time (0, 1, 4)")
    ap.add_argument("--tn-pipes", default="0,3", help="256x256 dW K-loop variants to time (0..3)")
    ap.add_argument("--only", default="", help="comma list of case-name prefixes to run")
    ap.add_argument("--diags", default="", help="SIREN_OPT_NT_DIAG ablation bits to add as extra "
                    "NT cases (1: L2-resident X; pipe 4: 512 no tiles, 1024 no epilogue); timing only, "
                    "needs --lib of a SIREN_DIAG build")
    ap.add_argument("--dw-splits", default="", help="extra dW cases at these split-K counts (256 tile)")
    ap.add_argument("--grids", default="", help="SIREN_OPT_NT_GRID persistent grid sizes to add as extra "
                    "ping-pong NT cases (measurement: CU-count scaling)")
    ap.add_argument("--queue-ab", action="store_true", help="add a static-walk (SIREN_OPT_NT_QUEUE 0) "
                    "twin of every ping-pong NT case")
    ap.add_argument("--lib", default="", help="load this library instead of the product one "
                    "(a measurement build from __graft_entry__.build_diagnostic)")
    args = ap.parse_args()
    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd import _lib
    # a fresh handle: _lib.load() has already cached the product library (ge.build() loads it), so
    # until round 3 `--lib` silently timed the product library against itself
    lib = _lib.bind(os.path.join(ROOT, args.lib)) if args.lib else _lib.load()
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    P = lambda t: t.data_ptr()  # noqa: E731
    bf = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.rand(R, H, device=dev, generator=g) * 2 - 1).to(bf)
    lim = math.sqrt(6 / H) / 30
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(bf)
    WT = W.t().contiguous()
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    hw = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.02
    Y = torch.empty(R, H, dtype=bf, device=dev)
    C = torch.empty_like(Y)
    dZ = (torch.randn(R, H, device=dev, generator=g) * 1e-3).to(bf)
    dZp = torch.empty_like(Y)
    hp = torch.empty(H // 128, R, device=dev)
    part = torch.empty(R // 128, 3, H, device=dev)
    t = torch.linspace(-1, 1, R, device=dev).reshape(R, 1)
    W0 = torch.rand(H, 1, device=dev) * 2 - 1
    b0 = torch.rand(H, device=dev) * 2 - 1
    tiles = [int(x) for x in args.tiles.split(",")]
    flops = 2.0 * R * H * H

    tq = _lib.new_tileq(dev)

    def run_fwd():
        return lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(Y), P(C), None, None, P(tq), s())

    def run_fwd_head():
        return lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(Y), P(C), P(hw), P(hp), P(tq),
                                   s())

    def run_dx():
        return lib.siren_inner_bwd_dx(P(dZ), P(WT), P(C), ctypes.c_float(30.0), R, H, None, P(dZp), P(part),
                                      s())

    def run_dx0():
        return lib.siren_first_bwd_dx(P(dZ), P(WT), P(C), P(t), 1, ctypes.c_float(3000.0), R, H, None, P(part),
                                      s())

    def run_first():
        return lib.siren_first_fwd(P(t), 1, P(W0), P(b0), ctypes.c_float(3000.0), R, H, P(Y), P(C), s())

    slabs = {}

    def run_dw(tile, splits=None):
        if splits is None:
            splits = lib.siren_default_splits(R, H) if tile == 0 else max(1, (512 if tile == 256 else 1024) // ((H // tile) ** 2))
        if splits not in slabs:
            slabs[splits] = torch.empty(int(lib.siren_slab_floats(H, splits)), device=dev)
        return lib.siren_inner_bwd_dw(P(Y), P(dZ), R, H, splits, tile, P(slabs[splits]), s())

    cases = {}
    pipes = [int(x) for x in args.pipes.split(",")]
    for tile in tiles:
        for pipe in (pipes if tile == 256 else [0]):
            sfx = f"t{tile}" + (f"p{pipe}" if tile == 256 else "")
            for nm, fn in (("fwd", run_fwd), ("fwd_head", run_fwd_head), ("dx", run_dx), ("dx0", run_dx0)):
                cases[f"{nm}_{sfx}"] = (tile, pipe, fn, flops)
        for pipe in ([int(x) for x in args.tn_pipes.split(",")] if tile == 256 else [0]):
            sfx = f"t{tile}" + (f"p{pipe}" if tile == 256 else "")
            cases[f"dw_{sfx}"] = (tile, pipe, (lambda tl=tile: run_dw(tl)), flops)
    cases["first_fwd"] = (0, 1, run_first, 0.0)
    grad = torch.empty(H * H, device=dev)

    def run_dw_reduce(splits):
        st = run_dw(256, splits)
        return st or lib.siren_dw_reduce(P(slabs[splits]), splits, H, 256, P(grad), 0, None, s())

    for sp in [int(x) for x in args.dw_splits.split(",") if x]:
        cases[f"dw_t256p0_s{sp}"] = (256, 0, (lambda sp=sp: run_dw(256, sp)), flops)
        # the default dW K-loop (pipe 4) with its split-K reduce
        cases[f"dwr_t256p4_s{sp}"] = (256, 4, (lambda sp=sp: run_dw_reduce(sp)), flops)
    # library calibration points (hipBLASLt through torch): the same contraction shapes with
    # no epilogue, fp16 and bf16 operands, fp16/bf16 output
    Xb, Wb, dZb = X.to(torch.bfloat16), W.to(torch.bfloat16), dZ.to(torch.bfloat16)
    Yl = torch.empty(R, H, dtype=bf, device=dev)
    Ylb = torch.empty(R, H, dtype=torch.bfloat16, device=dev)
    dWl = torch.empty(H, H, dtype=bf, device=dev)
    dWlb = torch.empty(H, H, dtype=torch.bfloat16, device=dev)
    cases["lib_nt_f16"] = (0, 1, lambda: torch.mm(X, W.t(), out=Yl), flops)
    cases["lib_nt_bf16"] = (0, 1, lambda: torch.mm(Xb, Wb.t(), out=Ylb), flops)
    cases["lib_tn_f16"] = (0, 1, lambda: torch.mm(dZ.t(), X, out=dWl), flops)
    cases["lib_tn_bf16"] = (0, 1, lambda: torch.mm(dZb.t(), Xb, out=dWlb), flops)
    if args.only:
        pre = tuple(args.only.split(","))
        cases = {k: v for k, v in cases.items() if k.startswith(pre)}
    diag = {k: 0 for k in cases}
    for v in [int(x) for x in args.diags.split(",") if x]:
        for k, c in list(cases.items()):
            if k.startswith(("fwd", "dx")) and diag[k] == 0:
                cases[f"{k}_d{v}"] = c
                diag[f"{k}_d{v}"] = v
    queue = {k: 1 for k in cases}
    if args.queue_ab:
        for k, c in list(cases.items()):
            if k.startswith(("fwd", "dx")) and "p4" in k and diag.get(k, 0) == 0:
                for q in (0, 2):
                    cases[f"{k}_q{q}"] = c
                    queue[f"{k}_q{q}"] = q
    grid = {k: 0 for k in cases}
    for v in [int(x) for x in args.grids.split(",") if x]:
        for k, c in list(cases.items()):
            if k.startswith(("fwd", "dx")) and "p4" in k and diag.get(k, 0) == 0 and queue.get(k, 1) == 1 \
                    and grid.get(k, 0) == 0:
                cases[f"{k}_g{v}"] = c
                grid[f"{k}_g{v}"] = v
    times = {k: [] for k in cases}
    for _ in range(args.rounds):
        for name, (tile, pipe, fn, _) in cases.items():
            if name.startswith("lib"):
                fn()
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                for _ in range(args.reps):
                    fn()
                ev1.record()
                torch.cuda.synchronize()
                times[name].append(ev0.elapsed_time(ev1) / args.reps)
                continue
            _lib.check(lib.siren_set_option(6, diag.get(name, 0)), "diag option")
            _lib.check(lib.siren_set_option(8, queue.get(name, 1)), "queue option")
            _lib.check(lib.siren_set_option(4, grid.get(name, 0)), "grid option")
            lib.siren_set_option(0, tile if not name.startswith("dw") else 0)
            if name.startswith("dw"):
                lib.siren_set_option(3, pipe)
            else:
                lib.siren_set_option(2, pipe if tile == 256 else 1)
            for _ in range(1):
                _lib.check(fn(), name)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(args.reps):
                fn()
            ev1.record()
            torch.cuda.synchronize()
            times[name].append(ev0.elapsed_time(ev1) / args.reps)
    lib.siren_set_option(6, 0)
    lib.siren_set_option(8, 1)
    lib.siren_set_option(4, 0)
    lib.siren_set_option(0, 0)
    lib.siren_set_option(2, -1)
    lib.siren_set_option(3, -1)
    out = {}
    for name, (tile, pipe, fn, fl) in cases.items():
        ts = sorted(times[name])
        med = ts[len(ts) // 2]
        out[name] = {"median_ms": med, "min_ms": ts[0], "tflops": (fl / (med * 1e-3) / 1e12) if fl else None}
    print(json.dumps({"rows": R, "hidden": H, "results": out}, indent=1))


if __name__ == "__main__":
    main()
