"""Measurement: the backward's two independent GEMMs of a layer -- dX (NT, store-heavy) and dW
(TN split-K, LDS/MFMA-bound) -- one after the other on the whole chip, or side by side on two
streams, each on part of the CUs (persistent NT grid cap + dW split count).

    python tools/overlap_bench.py [--rows 1048576] [--hidden 1024] [--rounds 5]
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
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--splits", default="96:6,128:8,160:10", help="NT grid cap : dW splits pairs")
    args = ap.parse_args()
    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    Y = (torch.rand(R, H, device=dev, generator=g) * 2 - 1).to(f16)
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * math.sqrt(6 / H) / 30).to(f16)
    WT = W.t().contiguous()
    C = (torch.rand(R, H, device=dev, generator=g) * 2 - 1).to(f16)
    dZ = (torch.randn(R, H, device=dev, generator=g) * 1e-3).to(f16)
    dZp = torch.empty_like(dZ)
    part = torch.empty(R // 128, 3, H, device=dev)
    slabs = {}
    P = lambda t: t.data_ptr()  # noqa: E731
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def dx(stream):
        return lib.siren_inner_bwd_dx(P(dZ), P(WT), P(C), ctypes.c_float(30.0), R, H, None, P(dZp), P(part),
                                      stream.cuda_stream)

    def dw(stream, splits):
        if splits not in slabs:
            slabs[splits] = torch.empty(int(lib.siren_slab_floats(H, splits)), device=dev)
        return lib.siren_inner_bwd_dw(P(Y), P(dZ), R, H, splits, 0, P(slabs[splits]), stream.cuda_stream)

    cases = {"sequential": None}
    for pr in args.splits.split(","):
        cap, sp = (int(x) for x in pr.split(":"))
        cases[f"overlap_g{cap}_s{sp}"] = (cap, sp)
    cases["dx_only"] = "dx"
    cases["dw_only"] = "dw"
    full_splits = int(lib.siren_default_splits(R, H))
    times = {k: [] for k in cases}
    for _ in range(args.rounds):
        for name, c in cases.items():
            cur = torch.cuda.current_stream(dev)
            sa.wait_stream(cur)
            sb.wait_stream(cur)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if c is None or isinstance(c, str):
                lib.siren_set_option(4, 0)
                ev0.record(sa)
                for _ in range(args.reps):
                    if c in (None, "dx"):
                        _lib.check(dx(sa), "dx")
                    if c in (None, "dw"):
                        _lib.check(dw(sa, full_splits), "dw")
                ev1.record(sa)
            else:
                cap, sp = c
                lib.siren_set_option(4, cap)
                ev0.record(sa)
                sb.wait_event(ev0)
                for _ in range(args.reps):
                    _lib.check(dx(sa), "dx")
                    _lib.check(dw(sb, sp), "dw")
                    # next pair starts when both are done (as in the layer chain)
                    e = torch.cuda.Event()
                    e.record(sb)
                    sa.wait_event(e)
                    e2 = torch.cuda.Event()
                    e2.record(sa)
                    sb.wait_event(e2)
                ev1.record(sa)
            torch.cuda.synchronize()
            times[name].append(ev0.elapsed_time(ev1) / args.reps)
    lib.siren_set_option(4, 0)
    out = {k: {"median_ms": sorted(v)[len(v) // 2], "min_ms": min(v)} for k, v in times.items()}
    print(json.dumps({"rows": R, "hidden": H, "default_splits": full_splits, "results": out}, indent=1))


if __name__ == "__main__":
    main()
