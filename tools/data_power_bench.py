"""Same kernels, same instruction stream, different operand data: the forward NT GEMM and the dW
GEMM at 2^20 x 1024 on (a) the real operand distributions (sin of uniform phases, SIREN-init
weights, N(0, 1e-2) gradients) and (b) all-zero operands.  If the GEMMs are held back by the
chip's power limit rather than by their schedule, the zero operands (fewer toggling bits in the
MFMA datapath) run at a higher clock and finish sooner.  Interleaved rounds, HIP events.

    python tools/data_power_bench.py
"""
from __future__ import annotations

import ctypes
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from inr_for_audio_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    R, H = 1 << 20, 1024
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    data = {
        "real": (torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16),
                 ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * math.sqrt(6 / H) / 30).to(f16),
                 (torch.randn(R, H, device=dev, generator=g) * 1e-2).to(f16)),
        "zero": (torch.zeros(R, H, dtype=f16, device=dev), torch.zeros(H, H, dtype=f16, device=dev),
                 torch.zeros(R, H, dtype=f16, device=dev)),
    }
    b = torch.zeros(H, device=dev)
    Y = torch.empty(R, H, dtype=f16, device=dev)
    C = torch.empty(R, H, dtype=f16, device=dev)
    tq = _lib.new_tileq(dev)
    splits = lib.siren_default_splits(R, H)
    slab = torch.empty(int(lib.siren_slab_floats(H, splits)), device=dev)
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    P = lambda t: t.data_ptr()  # noqa: E731

    def fwd(X, W, _):
        _lib.check(lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(Y), P(C), None, None, P(tq),
                                       s()), "fwd")

    def dw(X, _, dZ):
        _lib.check(lib.siren_inner_bwd_dw(P(X), P(dZ), R, H, splits, 0, P(slab), s()), "dw")

    times = {}
    for _ in range(7):
        for kn, fn in (("fwd", fwd), ("dw", dw)):
            for dn, ops in data.items():
                fn(*ops)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    fn(*ops)
                e1.record()
                torch.cuda.synchronize()
                times.setdefault(f"{kn}_{dn}", []).append(e0.elapsed_time(e1) / 5)
    print(json.dumps({k: round(sorted(v)[len(v) // 2], 4) for k, v in times.items()}))


if __name__ == "__main__":
    main()
