"""One NT GEMM launch kind, a few times, for a rocprofv3 --pmc pass per configuration (the kernel
name does not say which diag bits or walk a launch used, so each configuration is its own process).
Attributes the forward GEMM's HBM fetch above its 2.15 GB of X: run it with the
SIREN_DIAG library and diag bit 1 (X from 4 row bands: L2-resident X) or 4 (W from column tile 0:
L2-resident W) against no bits, each under `rocprofv3 --pmc FETCH_SIZE`.

    python tools/fetch_probe.py --lib inr-for-audio_amd/libsiren_diag.so --diag 4 --queue 0 [--mode fwd]
"""
from __future__ import annotations

import argparse
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--diag", type=int, default=0)
    ap.add_argument("--queue", type=int, default=1)
    ap.add_argument("--mode", choices=["fwd", "dx"], default="fwd")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    lib = _lib.bind(os.path.join(ROOT, args.lib)) if args.lib else _lib.load()
    dev = torch.device("cuda:0")
    R, H = 1 << 20, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).half()
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * math.sqrt(6 / H) / 30).half()
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    Y, C = torch.empty(R, H, dtype=torch.float16, device=dev), torch.empty(R, H, dtype=torch.float16, device=dev)
    part = torch.empty(R // 128, 3, H, device=dev)
    tq = _lib.new_tileq(dev)
    _lib.check(lib.siren_set_option(8, args.queue), "queue")
    _lib.check(lib.siren_set_option(6, args.diag), "diag")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(args.reps):
        if args.mode == "fwd":
            st = lib.siren_inner_fwd(X.data_ptr(), W.data_ptr(), b.data_ptr(), ctypes.c_float(30.0), R, H,
                                     Y.data_ptr(), C.data_ptr(), None, None, tq.data_ptr(), s)
        else:
            st = lib.siren_inner_bwd_dx(X.data_ptr(), W.data_ptr(), C.data_ptr(), ctypes.c_float(30.0), R, H, None,
                                        Y.data_ptr(), part.data_ptr(), s)
        _lib.check(st, args.mode)
    torch.cuda.synchronize()
    lib.siren_set_option(6, 0)
    lib.siren_set_option(8, 1)


if __name__ == "__main__":
    main()
