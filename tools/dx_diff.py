"""Where do two builds' dX outputs differ?  (measurement only) Runs siren_inner_bwd_dx of each
library on ab_bench.py's inputs and prints the differing elements of dZ (values, Cprev there).

    python tools/dx_diff.py --libs base=inr-for-audio_amd/libsiren_r4base.so,new=inr-for-audio_amd/libsiren_hip.so
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
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--hidden", type=int, default=1024)
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    libs = [(nm, _lib.bind(os.path.join(ROOT, p))) for nm, p in (x.split("=") for x in args.libs.split(","))]
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    P = lambda t: t.data_ptr()  # noqa: E731
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853)  # ab_bench's draw order: X
    lim = math.sqrt(6 / H) / 30
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(f16)
    WT = W.t().contiguous()
    torch.rand(H, device=dev, generator=g)
    torch.rand(H, device=dev, generator=g)
    Cp = torch.cos(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
    dZ = (torch.randn(R, H, device=dev, generator=g) * 1e-2).to(f16)
    outs = {}
    for nm, lib in libs:
        dzp = torch.zeros(R, H, dtype=f16, device=dev)
        part = torch.zeros(R // 128, 3, H, device=dev)
        _lib.check(lib.siren_inner_bwd_dx(P(dZ), P(WT), P(Cp), ctypes.c_float(30.0), R, H, None, P(dzp), P(part),
                                          torch.cuda.current_stream().cuda_stream), nm)
        torch.cuda.synchronize()
        outs[nm] = (dzp, part)
    (n0, (a, pa)), (n1, (b, pb)) = list(outs.items())[:2]
    ai, bi = a.view(torch.int16), b.view(torch.int16)
    bad = (ai != bi).nonzero()
    res = {"mismatches": int(bad.shape[0]), "part_equal": bool(torch.equal(pa, pb)), "examples": []}
    for r, c in bad[:12].tolist():
        res["examples"].append({"row": r, "col": c, n0: float(a[r, c]), n1: float(b[r, c]),
                                n0 + "_bits": int(ai[r, c]) & 0xffff, n1 + "_bits": int(bi[r, c]) & 0xffff,
                                "cprev": float(Cp[r, c]), "cprev_bits": int(Cp.view(torch.int16)[r, c]) & 0xffff})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
