"""Does a captured step replay the same work as an eager one at the headline size?  Two engines built
the same way (SIREN 5x1024, 2^20 coordinates, seed 0): one eager, one replaying its captured step.
Prints per-step times, whether parameters and losses stay bit-identical, and (under rocprofv3
--kernel-trace) the dispatch counts can be read per phase from the markers printed to stderr.

    python tools/graph_check.py [--rows 1048576] [--steps 3]
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
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    from inr_for_audio_amd import _lib
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    lib = _lib.load()
    dev = torch.device("cuda:0")
    n = args.rows
    xy = torch.empty(n, 1, device=dev)
    _lib.check(lib.siren_coords_fill(xy.data_ptr(), n, 0, n, torch.cuda.current_stream().cuda_stream), "fill")
    y = 0.5 * torch.sin(2300.0 * xy[:, 0])
    engs = {}
    for mode in ("eager", "graph"):
        torch.manual_seed(0)
        m = SirenWithSnakeTanh(1, 1, args.hidden, 4, 0, 0, first_omega_0=3000.0, hidden_omega_0=30.0)
        engs[mode] = SirenEngine(m, xy, y, hist_cap=64, device=dev)
    res = {}
    for mode, e in engs.items():
        e.step()
        torch.cuda.synchronize()
        if mode == "graph":
            e.capture_graph()
            torch.cuda.synchronize()
        t = []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            e.step()
            torch.cuda.synchronize()
            t.append((time.perf_counter() - t0) * 1e3)
        res[mode] = {"ms": [round(x, 3) for x in t], "losses": [float(v) for v in e.history()[0]]}
        print(f"phase {mode} done", file=sys.stderr, flush=True)
    res["params_identical"] = bool(torch.equal(engs["eager"].params, engs["graph"].params))
    res["grads_identical"] = bool(torch.equal(engs["eager"].grads, engs["graph"].grads))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
