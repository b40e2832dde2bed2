"""A/B of the fused head backward (SIREN_OPT_HEAD_FUSE 1 vs 0) on the headline step, interleaved in
one process on one engine (cfg2: SIREN 5x1024, 2^20 coords): ms per step (median of rounds) and the
per-kind launch breakdown of each mode (HIP events around every launch, untimed pass).

    python tools/headfuse_ab.py [--rounds 5] [--steps 6] [--rows 1048576]
"""
from __future__ import annotations

import argparse
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
    ap.add_argument("--layers", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd import _lib
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    lib = _lib.load()
    dev = torch.device("cuda:0")
    n = args.rows
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    y = 0.5 * torch.sin(2300.0 * t) + 0.3 * torch.sin(7100.0 * t + 0.5)
    torch.manual_seed(0)
    model = SirenWithSnakeTanh(1, 1, args.hidden, args.layers - 1, 0, 0, first_omega_0=3000.0, hidden_omega_0=30.0)
    eng = SirenEngine(model, t, y, lr=1e-5, device=dev)
    for _ in range(3):
        eng.step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {1: [], 0: []}
    breakdown = {}
    for mode in (1, 0):
        _lib.check(lib.siren_set_option(9, mode), "head fuse option")
        _lib.check(lib.siren_profile_enable(128 * 3), "profile_enable")
        for _ in range(2):
            eng.step()
        torch.cuda.synchronize()
        breakdown[mode] = {k: {"launches_per_step": c / 2, "ms_per_step": ms / 2}
                           for k, (ms, c) in _lib.profile_read().items() if c}
        _lib.check(lib.siren_profile_enable(0), "profile_disable")
    for _ in range(args.rounds):
        for mode in (1, 0):
            _lib.check(lib.siren_set_option(9, mode), "head fuse option")
            eng.step()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.steps):
                eng.step()
            e1.record()
            torch.cuda.synchronize()
            times[mode].append(e0.elapsed_time(e1) / args.steps)
    lib.siren_set_option(9, 1)
    med = {m: sorted(v)[len(v) // 2] for m, v in times.items()}
    print(json.dumps({"rows": n, "hidden": args.hidden, "layers": args.layers, "steps_per_round": args.steps,
                      "rounds": args.rounds, "ms_per_step_median": {"fused": med[1], "unfused": med[0]},
                      "saved_ms_per_step": med[0] - med[1], "ms_per_step_all": {"fused": times[1], "unfused": times[0]},
                      "breakdown": {"fused": breakdown[1], "unfused": breakdown[0]},
                      "final_loss": eng.last_loss() if math.isfinite(eng.last_loss()) else None}, indent=1))


if __name__ == "__main__":
    main()
