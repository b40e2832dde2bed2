"""Does a padded activation row stride speed the forward up?  (Measurement, not a test.)

X, Y and C rows are 2 KiB apart at H = 1024, so the 128-B segment a K-tile reads from every row of
a band, and the row pieces an epilogue writes, all share their low 11 address bits.  If the L2
channel / set hash leaves those accesses on a few channels, a padded row stride spreads them.  The
SIREN_DIAG library's forward takes a row padding in SIREN_OPT_NT_DIAG bits 16-23 (elements added to
the row stride of X and of Y / C; gemm_nt.hip ldpad).  Every case runs the static tile walk
(SIREN_OPT_NT_QUEUE 0: a diag launch never takes the queue), outputs checked bit-identical to the
dense layout, rounds rotated.

    python tools/ldpad_bench.py [--pads 0,8,64,128] [--rounds 7]
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
    ap.add_argument("--pads", default="0,8,64,128")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    lib = _lib.bind(os.path.join(ROOT, "inr-for-audio_amd", "libsiren_diag.so"))
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
    lim = math.sqrt(6 / H) / 30
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(f16)
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    tq = _lib.new_tileq(dev)
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    pads = [int(x) for x in args.pads.split(",")]
    bufs = {}
    for pad in pads:
        Xp = torch.zeros(R, H + pad, dtype=f16, device=dev)
        Xp[:, :H] = X
        bufs[pad] = (Xp, torch.empty(R, H + pad, dtype=f16, device=dev), torch.empty(R, H + pad, dtype=f16, device=dev))

    def run(pad):
        Xp, Yp, Cp = bufs[pad]
        _lib.check(lib.siren_set_option(6, pad << 16), "diag")
        return lib.siren_inner_fwd(Xp.data_ptr(), W.data_ptr(), b.data_ptr(), ctypes.c_float(30.0), R, H,
                                   Yp.data_ptr(), Cp.data_ptr(), None, None, tq.data_ptr(), s())

    _lib.check(lib.siren_set_option(8, 0), "queue")
    _lib.check(lib.siren_set_option(0, 256), "tile")
    for pad in pads:
        _lib.check(run(pad), f"pad {pad}")
    torch.cuda.synchronize()
    ident = {pad: bool(torch.equal(bufs[pad][1][:, :H].view(torch.int16), bufs[pads[0]][1][:, :H].view(torch.int16))
                       and torch.equal(bufs[pad][2][:, :H].view(torch.int16), bufs[pads[0]][2][:, :H].view(torch.int16)))
             for pad in pads}
    times = {pad: [] for pad in pads}
    for rnd in range(args.rounds):
        order = pads[rnd % len(pads):] + pads[:rnd % len(pads)]
        for pad in order:
            run(pad)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run(pad)
            e1.record()
            torch.cuda.synchronize()
            times[pad].append(e0.elapsed_time(e1) / args.reps)
    lib.siren_set_option(6, 0)
    lib.siren_set_option(8, 1)
    lib.siren_set_option(0, 0)
    res = {}
    for pad, ts in times.items():
        ts = sorted(ts)
        res[str(pad)] = {"median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4),
                         "bit_identical_to_dense": ident[pad], "row_stride_bytes": 2 * (H + pad)}
    print(json.dumps({"rows": R, "hidden": H, "walk": "static (queue 0)", "results": res}, indent=1))


if __name__ == "__main__":
    main()
