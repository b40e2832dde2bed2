"""Whole-step time against the dW split-K count (SirenEngine(splits=...)), interleaved rounds in one
process, for a bench config's shape (random coords and target: values do not change the schedule).

    python tools/split_sweep.py --hidden 512 --in-dim 2 --rows 220160 --splits 32,48,64,96,128
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from inr_for_audio_amd import _lib  # noqa: E402
from inr_for_audio_amd.engine import SirenEngine  # noqa: E402
from inr_for_audio_amd.models import SirenWithSnakeTanh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--layers", type=int, default=5)
    ap.add_argument("--in-dim", type=int, default=2)
    ap.add_argument("--rows", type=int, default=220160)
    ap.add_argument("--splits", default="32,48,64,96,128")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    torch.manual_seed(0)
    model = SirenWithSnakeTanh(args.in_dim, 1, args.hidden, args.layers - 1, 0, 0, first_omega_0=1000.0,
                               hidden_omega_0=30.0)
    coords = torch.rand(args.rows, args.in_dim) * 2 - 1
    target = torch.sin(5.0 * coords.sum(1)) * 0.5
    engs = {}
    for s in [int(v) for v in args.splits.split(",")]:
        engs[s] = SirenEngine(model, coords, target, micro_batch=args.rows, splits=s, device=dev)
    default = int(lib.siren_default_splits(args.rows, args.hidden))
    times = {s: [] for s in engs}
    for e in engs.values():
        for _ in range(3):
            e.step()
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for s, e in engs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.steps):
                e.step()
            b.record()
            b.synchronize()
            times[s].append(a.elapsed_time(b) / args.steps)
    med = {s: sorted(v)[len(v) // 2] for s, v in times.items()}
    print(json.dumps({"rows": args.rows, "hidden": args.hidden, "default_splits": default,
                      "ms_per_step_median": med, "all": times}))


if __name__ == "__main__":
    main()
