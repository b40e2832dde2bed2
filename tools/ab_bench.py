"""A/B timing of the product library against measurement builds of it, in ONE process with
interleaved rounds (cdna_hip_programming.md §5.4 rule 24), at the headline shape (2^20 coords x
1024).  Every variant's outputs are also compared with the product library's: a schedule-only
variant must be bit-identical.

    python tools/ab_bench.py --libs base=inr-for-audio_amd/libsiren_hip.so,x1=inr-for-audio_amd/libsiren_x1.so
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
    ap.add_argument("--libs", required=True, help="name=path,... (paths relative to the repo root)")
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="fwd,fwd_head,fwd_hb,dx,dx0,dw", help="cases")
    ap.add_argument("--grid", type=int, default=0, help="SIREN_OPT_NT_GRID for every library (0: one block per CU)")
    ap.add_argument("--queue", type=int, default=1, help="SIREN_OPT_NT_QUEUE for every library")
    ap.add_argument("--own-out", action="store_true", help="time every library on its own output buffers "
                    "(default: all on the first library's, since buffer placement alone moved a forward "
                    "by ~2 %% between identical kernels, profiles/r17)")
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    libs = {}
    for item in args.libs.split(","):
        nm, path = item.split("=")
        # libraries built from older commits (tools/build_at.py) may carry an earlier ABI
        libs[nm] = _lib.bind(os.path.join(ROOT, path), check_abi=False)
    for lib_ in libs.values():
        assert lib_.siren_set_option(4, args.grid) == 0 and lib_.siren_set_option(8, args.queue) == 0
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    P = lambda t: t.data_ptr()  # noqa: E731
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    # X: sin of uniform phases (the forward's real operand distribution)
    X = torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
    lim = math.sqrt(6 / H) / 30
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(f16)
    WT = W.t().contiguous()
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    hw = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.02
    Cp = torch.cos(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
    dZ = (torch.randn(R, H, device=dev, generator=g) * 1e-2).to(f16)
    t = torch.linspace(-1, 1, R, device=dev).reshape(R, 1)
    Ep = ((torch.rand(R, H, device=dev, generator=g) - 0.5) * 0.5).to(f16)  # a Snake layer's dY/da
    a_snake = 0.5 + torch.rand(H, device=dev, generator=g)
    # zero-filled: the parity check compares whole buffers, including what a tile size leaves unwritten
    outs = {nm: {"Y": torch.zeros(R, H, dtype=f16, device=dev), "C": torch.zeros(R, H, dtype=f16, device=dev),
                 "hp": torch.zeros(H // 128, R, device=dev), "dZp": torch.zeros(R, H, dtype=f16, device=dev),
                 "part": torch.zeros(R // 128, 3, H, device=dev), "out": torch.zeros(R, device=dev),
                 "g": torch.zeros(R, device=dev), "sse": torch.zeros(R // 256, device=dev),
                 "gsum": torch.zeros(R // 256, device=dev), "E": torch.zeros(R, H, dtype=f16, device=dev)}
            for nm in libs}
    y = torch.sin(t[:, 0] * 2300.0) * 0.5
    bh = torch.zeros(1, device=dev)
    gs = torch.tensor([2.0 ** 9, 2.0 ** -9], device=dev)
    tq = _lib.new_tileq(dev)
    splits = list(libs.values())[0].siren_default_splits(R, H)
    for nm in libs:  # the dW split-K slab, per library so that the parity check covers dW too
        outs[nm]["slab"] = torch.zeros(int(list(libs.values())[0].siren_slab_floats(H, splits)), device=dev)
    flops = 2.0 * R * H * H

    def case(nm, lib, kind, onm=None):
        o = outs[onm or nm]
        if kind == "fwd":
            return lambda: lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(o["Y"]), P(o["C"]),
                                               None, None, P(tq), s())
        if kind == "fwd_head":
            return lambda: lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(o["Y"]), P(o["C"]),
                                               P(hw), P(o["hp"]), P(tq), s())
        if kind == "fwd_hb":  # the fused last layer + head + MSE gradient + head backward
            return lambda: lib.siren_head_fused_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(hw), P(bh),
                                                    ctypes.c_float(0.0), P(y), R, float(R), 0, P(gs), P(o["hp"]),
                                                    P(o["out"]), P(o["g"]), P(o["sse"]), P(o["gsum"]), P(o["dZp"]),
                                                    P(o["part"]), s())
        if kind == "dx":
            return lambda: lib.siren_inner_bwd_dx(P(dZ), P(WT), P(Cp), ctypes.c_float(30.0), R, H, None,
                                                  P(o["dZp"]), P(o["part"]), s())
        if kind == "dx0":
            return lambda: lib.siren_first_bwd_dx(P(dZ), P(WT), P(Cp), P(t), 1, ctypes.c_float(3000.0), R, H, None,
                                                  P(o["part"]), s())
        if kind in ("dx_snake", "dx_tanh"):  # dX into a Snake / Tanh layer
            act = 1 if kind == "dx_snake" else 2
            return lambda: lib.siren_inner_bwd_dx_act(P(dZ), P(WT), P(Cp), P(Ep), act, ctypes.c_float(1.0), R, H,
                                                      None, P(o["dZp"]), P(o["part"]), s())
        if kind in ("fwd_snake", "fwd_tanh"):
            act = 1 if kind == "fwd_snake" else 2
            return lambda: lib.siren_inner_fwd_act(P(X), P(W), P(b), act, ctypes.c_float(1.0), P(a_snake), R, H,
                                                   P(o["Y"]), P(o["C"]), P(o["E"]), None, None, P(tq), s())
        if kind == "dw":
            return lambda: lib.siren_inner_bwd_dw(P(X), P(dZ), R, H, splits, 0, P(o["slab"]), s())
        raise ValueError(kind)

    kinds = args.only.split(",")
    cases = {(nm, k): case(nm, lib, k) for k in kinds for nm, lib in libs.items()}
    # parity: every variant's outputs equal the first library's (once before and once after the
    # timed rounds, so that reused tile-queue state is covered too)
    base = next(iter(libs))
    mism = {}

    def parity(tag):
        for k in kinds:
            got = {}
            for nm in libs:
                for t_ in outs[nm].values():
                    t_.zero_()
                _lib.check(cases[(nm, k)](), f"{nm} {k}")
                torch.cuda.synchronize()
                o = outs[nm]
                got[nm] = {"fwd": (o["Y"], o["C"]), "fwd_head": (o["Y"], o["C"], o["hp"]), "dx": (o["dZp"], o["part"]),
                           "dx_snake": (o["dZp"], o["part"]), "dx_tanh": (o["dZp"], o["part"]),
                           "fwd_snake": (o["Y"], o["C"], o["E"]), "fwd_tanh": (o["Y"], o["C"]),
                           "dx0": (o["part"],), "fwd_hb": (o["out"], o["g"], o["sse"], o["dZp"], o["part"]),
                           "dw": (o["slab"],)}[k]
                got[nm] = tuple(x.clone() for x in got[nm])
            for nm in libs:
                if nm != base:
                    mism[f"{tag}:{nm}:{k}"] = [bool(torch.equal(a, c)) for a, c in zip(got[nm], got[base])]

    parity("pre")
    if not args.own_out:  # timing on one set of output buffers
        first = next(iter(libs))
        cases = {(nm, k): case(nm, lib, k, first) for k in kinds for nm, lib in libs.items()}
    times = {key: [] for key in cases}
    names = list(libs)
    for rnd in range(args.rounds):
        # the library order rotates every round: the first case of a round runs measurably slower
        # (profiles/r17: 3-4 % in u4's two orders), so no library may always take that place
        order = names[rnd % len(names):] + names[:rnd % len(names)]
        for key, fn in sorted(cases.items(), key=lambda kv: (kinds.index(kv[0][1]), order.index(kv[0][0]))):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[key].append(e0.elapsed_time(e1) / args.reps)
    cases = {(nm, k): case(nm, lib, k) for k in kinds for nm, lib in libs.items()}
    parity("post")
    res = {}
    for (nm, k), ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        res.setdefault(k, {})[nm] = {"median_ms": round(med, 4), "min_ms": round(ts[0], 4),
                                     "frac": round(flops / (med * 1e-3) / 2.5e15, 4)}
    print(json.dumps({"rows": R, "hidden": H, "rounds": args.rounds, "bit_identical": mism, "results": res},
                     indent=1))


if __name__ == "__main__":
    main()
