"""Does splitting one forward GEMM launch into two half-height launches on two streams (so the
second fills the first's tail round and ramp) pay?  cfg4 shape (220 160 x 512) and cfg2 (2^20 x
1024): one launch on one stream vs two half launches on one stream vs two half launches on two
streams, interleaved rounds, HIP events on the launching stream(s).

    python tools/stream_split_bench.py [--rows 220160 --hidden 512]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=220160)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    assert R % 512 == 0 or (R // 2) % 256 == 0
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
    W = (((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * math.sqrt(6 / H) / 30)).to(f16)
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    Y = torch.empty(R, H, dtype=f16, device=dev)
    C = torch.empty(R, H, dtype=f16, device=dev)
    tq = [_lib.new_tileq(dev) for _ in range(2)]
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    h = R // 2
    P = lambda t: t.data_ptr()  # noqa: E731

    def fwd(lo, n, st, q):
        _lib.check(lib.siren_inner_fwd(P(X) + lo * H * 2, P(W), P(b), ctypes.c_float(30.0), n, H,
                                       P(Y) + lo * H * 2, P(C) + lo * H * 2, None, None, P(q), st.cuda_stream),
                   "inner_fwd")

    def one():
        fwd(0, R, s0, tq[0])

    def halves_one_stream():
        fwd(0, h, s0, tq[0])
        fwd(h, R - h, s0, tq[1])

    def halves_two_streams():
        s1.wait_stream(s0)
        fwd(0, h, s0, tq[0])
        fwd(h, R - h, s1, tq[1])
        s0.wait_stream(s1)

    cases = {"one": one, "halves_1stream": halves_one_stream, "halves_2streams": halves_two_streams}
    ref = None
    times = {k: [] for k in cases}
    for r in range(args.rounds):
        for k, fn in cases.items():
            fn()
            torch.cuda.synchronize()
            if r == 0:
                out = (Y.clone(), C.clone())
                if ref is None:
                    ref = out
                else:
                    assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]), k
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            for _ in range(args.reps):
                fn()
            e1.record(s0)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / args.reps)
    res = {k: round(sorted(v)[len(v) // 2], 4) for k, v in times.items()}
    print(json.dumps({"rows": R, "hidden": H, "median_ms": res, "bit_identical": True}))


if __name__ == "__main__":
    main()
