"""Whole-step time with eager launches vs one captured HIP graph per step (SirenEngine.capture_graph),
for the bench configs (bench.py CONFIGS): how much of a step is launch gaps.  Rounds alternate two
engines built the same way (one eager, one replaying its graph).

    python tools/graph_step_bench.py --configs cfg4,cfg2 --steps 20 --rounds 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg4,cfg2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import bench
    from inr_for_audio_amd import _lib
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    lib = _lib.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev).cuda_stream
    out = {}
    for cfg in args.configs.split(","):
        H, layers, in_dim, coords, w0, grid_h = bench.CONFIGS[cfg]
        if in_dim == 1:
            n = coords
            xy = torch.empty(n, 1, device=dev)
            _lib.check(lib.siren_coords_fill(xy.data_ptr(), n, 0, n, stream), "fill")
        else:
            n = coords // 2 * 2 if cfg == "cfg3" else grid_h * (coords // grid_h)
            width = 2 if cfg == "cfg3" else coords // grid_h
            height = n // width
            xy = torch.empty(n, 2, device=dev)
            _lib.check(lib.siren_coords_fill_grid(xy.data_ptr(), n, 0, height, width, stream), "fill")
        y = 0.5 * torch.sin(2300.0 * xy[:, 0])
        engs = {}
        for mode in ("eager", "graph"):
            torch.manual_seed(0)
            m = SirenWithSnakeTanh(in_dim, 1, H, layers - 1, 0, 0, first_omega_0=w0, hidden_omega_0=30.0)
            e = SirenEngine(m, xy, y, hist_cap=args.steps * args.rounds * 2 + 16, device=dev)
            e.step()
            if mode == "graph":
                e.capture_graph()
            engs[mode] = e
        t = {"eager": [], "graph": []}
        for _ in range(args.rounds):
            for mode, e in engs.items():
                e.step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    e.step()
                torch.cuda.synchronize()
                t[mode].append((time.perf_counter() - t0) / args.steps * 1e3)
        la, _ = engs["eager"].history()
        lb, _ = engs["graph"].history()
        k = min(len(la), len(lb))
        out[cfg] = {"ms_per_step_eager": float(np.median(t["eager"])), "ms_per_step_graph": float(np.median(t["graph"])),
                    "losses_identical": bool(np.array_equal(la[:k], lb[:k]))}
        print(json.dumps({cfg: out[cfg]}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
