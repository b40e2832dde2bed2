"""Dump the HIP path's 300-step loss traces of train()'s default Snake architecture over the
seeds of tests/golden/trajectory_snake_default_seeds.json (fit-stability diagnostics).

    python tools/snake_fit_dump.py OUT.json
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    G = os.path.join(ROOT, "tests", "golden")
    ref = json.load(open(os.path.join(G, "trajectory_snake_default_seeds.json")))
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    t = torch.from_numpy(g["coords"]).reshape(-1, 1)
    y = torch.from_numpy(g["target"])
    out = {}
    for s in sorted(int(k) for k in ref["runs"]):
        torch.manual_seed(s)
        m = SirenWithSnakeTanh(1, 1, 256, 2, 2, 0, first_omega_0=1000.0, hidden_omega_0=30.0, a_initial=0.5)
        eng = SirenEngine(m, t, y, lr=1e-3, hist_cap=ref["steps"], device=torch.device("cuda:0"))
        for _ in range(ref["steps"]):
            eng.step()
        losses, lrs = eng.history()
        out[str(s)] = losses.tolist()
    json.dump(out, open(sys.argv[1], "w"))


if __name__ == "__main__":
    main()
