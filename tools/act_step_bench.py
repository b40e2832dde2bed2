"""Step time of the Snake / Tanh stacks: run.py's default architecture
(num_sine=2, num_snake=2), run.py:466's __main__ stack (num_snake=4) and a Tanh stack, at H = 1024
over 2^20 coordinates, with the fused last layer on and off (SIREN_OPT_HEAD_FUSE, option 9) and,
optionally, under each 256x256 NT K-loop variant.  Rounds alternate the settings on one engine.

    python tools/act_step_bench.py [--fuse 1,0] [--pipes -1] [--steps 5] [--rounds 3] [--breakdown]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import inr_for_audio_amd  # noqa: E402,F401
from inr_for_audio_amd import _lib  # noqa: E402
from inr_for_audio_amd.engine import SirenEngine  # noqa: E402
from inr_for_audio_amd.models import SirenWithSnakeTanh  # noqa: E402

STACKS = {"sine2_snake2": (2, 2, 0), "snake4": (0, 4, 0), "sine2_tanh2": (2, 0, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipes", default="-1")
    ap.add_argument("--fuse", default="1,0")
    ap.add_argument("--stacks", default=",".join(STACKS))
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--breakdown", action="store_true", help="per-kind kernel ms per step (HIP events around "
                    "every launch, untimed pass)")
    ap.add_argument("--lib", default="", help="time this build of the library (path relative to the repo root)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = _lib.load(os.path.join(root, args.lib)) if args.lib else _lib.load()
    n = args.rows
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    y = 0.5 * torch.sin(2300.0 * t)
    out, times = {}, {}
    for name in args.stacks.split(","):
        ns, nk, nt = STACKS[name]
        torch.manual_seed(0)
        m = SirenWithSnakeTanh(1, 1, 1024, ns, nk, nt, first_omega_0=3000.0, hidden_omega_0=30.0)
        eng = SirenEngine(m, t, y, device=dev)
        eng.step()  # a Snake last layer fuses from the second step on (siren_batch.head_scale_prev)
        settings = [(int(p), int(f)) for p in args.pipes.split(",") for f in args.fuse.split(",")]
        for _ in range(args.rounds):
            for pipe, fuse in settings:
                _lib.check(lib.siren_set_option(2, pipe), "nt pipe")
                _lib.check(lib.siren_set_option(9, fuse), "head fuse")
                eng.step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    eng.step()
                torch.cuda.synchronize()
                times.setdefault(f"{name}_p{pipe}_f{fuse}", []).append((time.perf_counter() - t0) / args.steps * 1e3)
        for pipe, fuse in settings:
            key = f"{name}_p{pipe}_f{fuse}"
            out[key] = float(np.median(times[key]))
            if args.breakdown:
                _lib.check(lib.siren_set_option(2, pipe), "nt pipe")
                _lib.check(lib.siren_set_option(9, fuse), "head fuse")
                _lib.check(lib.siren_profile_enable(4096), "profile_enable")
                for _ in range(args.steps):
                    eng.step()
                torch.cuda.synchronize()
                for k, (ms, cnt) in _lib.profile_read().items():
                    if cnt:
                        out[f"{key}:{k}"] = ms / args.steps
                _lib.check(lib.siren_profile_enable(0), "profile_disable")
        out[f"{name}:overflows"] = eng.guard_state()["overflows"]
    lib.siren_set_option(2, -1)
    lib.siren_set_option(9, 1)
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in out.items()}))


if __name__ == "__main__":
    main()
