"""A/B of the first-layer kernel (siren_first_fwd: Y0 and C0 for 2^20 coordinates x 1024) across
builds of the library, interleaved rounds in one process; outputs compared.  Measurement only.

    python tools/first_ab.py --libs base=inr-for-audio_amd/libsiren_hip.so,x=inr-for-audio_amd/libsiren_x.so
"""
from __future__ import annotations

import argparse
import ctypes
import json
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
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    libs = [(nm, _lib.bind(os.path.join(ROOT, p))) for nm, p in (x.split("=") for x in args.libs.split(","))]
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    t = torch.linspace(-1, 1, R, device=dev).reshape(R, 1)
    g = torch.Generator(device=dev).manual_seed(0)
    W0 = (torch.rand(H, 1, device=dev, generator=g) * 2 - 1)
    b0 = (torch.rand(H, device=dev, generator=g) * 2 - 1)
    outs = {nm: (torch.zeros(R, H, dtype=torch.float16, device=dev), torch.zeros(R, H, dtype=torch.float16, device=dev))
            for nm, _ in libs}
    s = torch.cuda.current_stream().cuda_stream

    def run(nm, lib):
        Y, C = outs[nm]
        _lib.check(lib.siren_first_fwd(t.data_ptr(), 1, W0.data_ptr(), b0.data_ptr(), ctypes.c_float(3000.0), R, H,
                                       Y.data_ptr(), C.data_ptr(), s), nm)
    times = {nm: [] for nm, _ in libs}
    for _ in range(args.rounds):
        for nm, lib in libs:
            run(nm, lib)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run(nm, lib)
            e1.record()
            torch.cuda.synchronize()
            times[nm].append(e0.elapsed_time(e1) / args.reps)
    # write-only reference: torch's fill of the same two fp16 arrays
    Y, C = outs[libs[0][0]]
    fill = []
    for _ in range(args.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            Y.fill_(0.5)
            C.fill_(0.5)
        e1.record()
        torch.cuda.synchronize()
        fill.append(e0.elapsed_time(e1) / args.reps)
    times["torch_fill"] = fill
    for nm, lib in libs:
        run(nm, lib)
    torch.cuda.synchronize()
    b = libs[0][0]
    res = {"bit_identical": {nm: [bool(torch.equal(outs[nm][i], outs[b][i])) for i in range(2)] for nm, _ in libs},
           "median_ms": {nm: round(sorted(v)[len(v) // 2], 4) for nm, v in times.items()},
           "tb_per_s": {nm: round(2 * R * H * 2 / (sorted(v)[len(v) // 2] * 1e-3) / 1e12, 3) for nm, v in times.items()}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
