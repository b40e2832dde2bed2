"""Does where the activations sit in device memory change the NT GEMMs' speed?  (Measurement, not a test.)

tools/ab_bench.py timed the SAME forward kernel 2 % apart on two sets of output buffers (profiles/r17,
u6 place_own vs place_shared).  Here X, Y and C of one forward launch (and dZ, Cprev, dZprev of one dX
launch) are carved out of ONE pool at chosen byte offsets, so the distance between the streams that
run at the same time is the only variable; rounds rotate the order of the cases.

    python tools/placement_bench.py --rounds 7 [--gaps 0,256,4096,65536,2097152,2101248]
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--gaps", default="0,256,4096,65536,2097152,2101248",
                    help="bytes added between consecutive activation buffers (each also 2 MiB-rounded)")
    args = ap.parse_args()
    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    nbytes = R * H * 2
    gaps = [int(x) for x in args.gaps.split(",")]
    span = 3 * nbytes + 3 * max(gaps) + 4096
    pool = torch.empty(span, dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    f16 = torch.float16
    src_x = torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
    src_c = torch.cos(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
    src_dz = (torch.randn(R, H, device=dev, generator=g) * 1e-2).to(f16)
    lim = math.sqrt(6 / H) / 30
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(f16)
    WT = W.t().contiguous()
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    part = torch.empty(R // 128, 3, H, device=dev)
    tq = _lib.new_tileq(dev)
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    base = pool.data_ptr()

    def view(off):
        return pool[off:off + nbytes].view(f16).view(R, H)

    def layout(gap):
        # three consecutive buffers, each starting `gap` bytes after the previous one's end
        offs = [0, nbytes + gap, 2 * (nbytes + gap)]
        return [view(o) for o in offs], [base + o for o in offs]

    cases = {}
    for gap in gaps:
        (a, bb, c), addrs = layout(gap)
        def fwd(a=a, bb=bb, c=c):  # X = a, Y = bb, C = c
            return lib.siren_inner_fwd(a.data_ptr(), W.data_ptr(), b.data_ptr(), ctypes.c_float(30.0), R, H,
                                       bb.data_ptr(), c.data_ptr(), None, None, tq.data_ptr(), s())
        def dx(a=a, bb=bb, c=c):   # dZ = a, Cprev = bb, dZprev = c
            return lib.siren_inner_bwd_dx(a.data_ptr(), WT.data_ptr(), bb.data_ptr(), ctypes.c_float(30.0), R, H,
                                          None, c.data_ptr(), part.data_ptr(), s())
        cases[("fwd", gap)] = (fwd, a, bb, src_x, None)
        cases[("dx", gap)] = (dx, a, bb, src_dz, src_c)
    times = {k: [] for k in cases}
    keys = list(cases)
    for rnd in range(args.rounds):
        order = keys[rnd % len(keys):] + keys[:rnd % len(keys)]
        for k in order:
            fn, a, bb, sa, sb = cases[k]
            a.copy_(sa)          # the inputs of this layout (the pool is shared)
            if sb is not None:
                bb.copy_(sb)
            _lib.check(fn(), str(k))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / args.reps)
    res = {}
    for (kind, gap), ts in times.items():
        ts = sorted(ts)
        res.setdefault(kind, {})[str(gap)] = {"median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4)}
    print(json.dumps({"rows": R, "hidden": H, "rounds": args.rounds, "pool_base_mod_2MiB": base % (2 << 20),
                      "results": res}, indent=1))


if __name__ == "__main__":
    main()
