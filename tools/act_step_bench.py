"""Step time of the Snake / Tanh stacks under each 256x256 NT K-loop variant:
run.py's default architecture (num_sine=2, num_snake=2) at H = 1024 over 2^20 coordinates.

    python tools/act_step_bench.py [--pipes -1,1] [--steps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import inr_for_audio_amd  # noqa: E402,F401
from inr_for_audio_amd import _lib  # noqa: E402
from inr_for_audio_amd.engine import SirenEngine  # noqa: E402
from inr_for_audio_amd.models import SirenWithSnakeTanh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipes", default="-1,1")
    ap.add_argument("--steps", type=int, default=5)
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
    out = {}
    for name, (ns, nk, nt) in {"sine2_snake2": (2, 2, 0), "sine2_tanh2": (2, 0, 2)}.items():
        torch.manual_seed(0)
        m = SirenWithSnakeTanh(1, 1, 1024, ns, nk, nt, first_omega_0=3000.0, hidden_omega_0=30.0)
        eng = SirenEngine(m, t, y, device=dev)
        for pipe in [int(p) for p in args.pipes.split(",")]:
            _lib.check(lib.siren_set_option(2, pipe), "nt pipe")
            eng.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                eng.step()
            torch.cuda.synchronize()
            out[f"{name}_p{pipe}"] = (time.perf_counter() - t0) / args.steps * 1e3
            if args.breakdown:
                _lib.check(lib.siren_profile_enable(4096), "profile_enable")
                for _ in range(args.steps):
                    eng.step()
                torch.cuda.synchronize()
                for k, (ms, cnt) in _lib.profile_read().items():
                    if cnt:
                        out[f"{name}_p{pipe}:{k}"] = ms / args.steps
                _lib.check(lib.siren_profile_enable(0), "profile_disable")
    lib.siren_set_option(2, -1)
    print(json.dumps({k: round(v, 3) for k, v in out.items()}))


if __name__ == "__main__":
    main()
