"""The one-wave-per-SIMD forward (SIREN_OPT_NT_PIPE 5, gemm_nt1.hip) against the ping-pong forward
(pipe 4): bit-identity of Y and C over shapes and grid sizes, then interleaved timing.

    python tools/one_check.py [--time-shapes 1048576x1024,220160x512] [--rounds 7]
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

# (rows, hidden, grid cap): tiles per block 1, 2, 3, odd / even, every K / N variant
PARITY = [(256, 256, 0), (512, 512, 0), (256, 1024, 3), (1024, 1024, 5), (2048, 512, 7), (4096, 1024, 8),
          (4096, 256, 0), (65536, 1024, 0), (220160, 512, 0), (1 << 20, 1024, 0), (1 << 20, 1024, 37)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--time-shapes", default="1048576x1024,220160x512")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--skip-parity", action="store_true")
    ap.add_argument("--pipes", default="5,6", help="NT pipes checked against the ping-pong forward (pipe 4)")
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    tq = _lib.new_tileq(dev)
    f16 = torch.float16

    def make(R, H, seed=0):
        g = torch.Generator(device=dev).manual_seed(seed)
        X = torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
        lim = math.sqrt(6 / H) / 30
        W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(f16)
        b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
        return X, W, b

    def fwd(pipe, grid, X, W, b, Y, C):
        R, H = X.shape
        _lib.check(lib.siren_set_option(2, pipe), "pipe")
        _lib.check(lib.siren_set_option(4, grid), "grid")
        _lib.check(lib.siren_set_option(0, 256), "tile")
        return lib.siren_inner_fwd(X.data_ptr(), W.data_ptr(), b.data_ptr(), ctypes.c_float(30.0), R, H,
                                   Y.data_ptr(), C.data_ptr(), None, None, tq.data_ptr(), s())

    out = {"parity": [], "timing": {}}
    if not args.skip_parity:
        for R, H, grid in PARITY:
            X, W, b = make(R, H, seed=R + H)
            ys = []
            pipes = [4] + [int(x) for x in args.pipes.split(",")]
            for pipe in pipes:
                Y = torch.full((R, H), float("nan"), dtype=f16, device=dev)
                C = torch.full((R, H), float("nan"), dtype=f16, device=dev)
                _lib.check(fwd(pipe, grid, X, W, b, Y, C), f"fwd pipe {pipe}")
                torch.cuda.synchronize()
                ys.append((Y, C))
            row = {"rows": R, "hidden": H, "grid": grid}
            for q in range(1, len(pipes)):
                same = bool(torch.equal(ys[0][0].view(torch.int16), ys[q][0].view(torch.int16)) and
                            torch.equal(ys[0][1].view(torch.int16), ys[q][1].view(torch.int16)))
                nan = bool(torch.isnan(ys[q][0]).any() or torch.isnan(ys[q][1]).any())
                r = {"bit_identical": same, "nan_left": nan}
                if not same:
                    d = (ys[0][0].float() - ys[q][0].float()).abs()
                    r["max_abs_Y"] = float(torch.nan_to_num(d, nan=99.0).max())
                    bad = torch.nonzero(torch.nan_to_num(d, nan=99.0) > 0)
                    r["first_bad"] = bad[:4].tolist()
                    r["n_bad"] = int(bad.shape[0])
                row[f"pipe{pipes[q]}"] = r
            out["parity"].append(row)
            print(json.dumps(row), flush=True)
            del X, W, b, ys
            torch.cuda.empty_cache()
    for shape in [x for x in args.time_shapes.split(",") if x]:
        R, H = (int(v) for v in shape.split("x"))
        X, W, b = make(R, H)
        Y = torch.empty(R, H, dtype=f16, device=dev)
        C = torch.empty_like(Y)
        pl = [4] + [int(x) for x in args.pipes.split(",")]
        times = {q: [] for q in pl}
        for rnd in range(args.rounds):
            for pipe in pl[rnd % len(pl):] + pl[:rnd % len(pl)]:
                _lib.check(fwd(pipe, 0, X, W, b, Y, C), "warm")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fwd(pipe, 0, X, W, b, Y, C)
                e1.record()
                torch.cuda.synchronize()
                times[pipe].append(e0.elapsed_time(e1) / args.reps)
        flops = 2.0 * R * H * H
        res = {}
        for pipe, ts in times.items():
            ts = sorted(ts)
            med = ts[len(ts) // 2]
            res[f"pipe{pipe}"] = {"median_ms": round(med, 4), "min_ms": round(ts[0], 4),
                                  "frac": round(flops / (med * 1e-3) / 2.5e15, 4)}
        out["timing"][shape] = res
        print(shape, json.dumps(res), flush=True)
        del X, W, b, Y, C
        torch.cuda.empty_cache()
    lib.siren_set_option(2, -1)
    lib.siren_set_option(4, 0)
    lib.siren_set_option(0, 0)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
