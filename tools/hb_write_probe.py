"""Where do the fused last layer's extra HBM writes come from?  (measurement only.)

Launches siren_head_fused_fwd (NT_FWD_HB) at the headline shape (2^20 x 1024) `--reps` times from
each library named, one library after the other, in one process, so that a rocprofv3 --pmc pass
over this script gives per-dispatch WRITE_SIZE / FETCH_SIZE for the product kernel and for the
write-attribution variants of tools/variants.py (hb_nostore: no dZ_L stores; hb_nopub: no head
partial hand-off; hb_nopub_nostore: neither).  The dispatch order is printed as JSON so the counter
rows can be matched to the libraries (tools/hb_write_summary.py).

    python tools/variants.py hb_nostore hb_nopub hb_nopub_nostore
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/hbw -o run -- \\
        python3 tools/hb_write_probe.py --libs base=inr-for-audio_amd/libsiren_hip.so,...
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--act", type=int, default=0, help="last layer: 0 sine, 1 Snake, 2 Tanh")
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    libs = []
    for item in args.libs.split(","):
        nm, path = item.split("=")
        libs.append((nm, _lib.bind(os.path.join(ROOT, path))))
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    P = lambda t: t.data_ptr()  # noqa: E731
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(f16)
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * math.sqrt(6 / H) / 30).to(f16)
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    a = 0.5 + torch.rand(H, device=dev, generator=g)
    hw = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.02
    t = torch.linspace(-1, 1, R, device=dev)
    y = torch.sin(t * 2300.0) * 0.5
    bh = torch.zeros(1, device=dev)
    gs = torch.tensor([2.0 ** 9, 2.0 ** -9], device=dev)
    hp, out, gg = torch.zeros(H // 256, R, device=dev), torch.zeros(R, device=dev), torch.zeros(R, device=dev)
    sse, gsum, gmax = (torch.zeros(R // 256, device=dev) for _ in range(3))
    dZ = torch.zeros(R, H, dtype=f16, device=dev)
    E = torch.zeros(R, H, dtype=f16, device=dev)
    part = torch.zeros(R // 256, 3, H, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    order = []
    for nm, lib in libs:
        for _ in range(args.reps):
            _lib.check(lib.siren_head_fused_fwd_act(P(X), P(W), P(b), args.act, ctypes.c_float(30.0), P(a), R, H, P(hw),
                                                    P(bh), ctypes.c_float(0.0), P(y), R, float(R), 0, P(gs), P(hp),
                                                    P(out), P(gg), P(sse), P(gsum), P(gmax), P(dZ), P(part), P(E),
                                                    s),
                       nm)
            order.append(nm)
        torch.cuda.synchronize()
    print(json.dumps({"order": order, "rows": R, "hidden": H, "act": args.act}))


if __name__ == "__main__":
    main()
