"""Spread of the 300-step fit quality (SNR_target, dB) over init seeds and summation orders
(micro-batch splits change the order of the gradient sums), on the golden 1 s gt_bach clip
with SIREN 3x256 / omega0 1000 -- the configuration of tests/test_gpu_fit.py.

    python tools/fit_spread.py [--seeds 0,1,2,3,4] [--mbs 0,16384] [--steps 300]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
G = os.path.join(ROOT, "tests", "golden")


def fit(dev, steps, seed, micro_batch, hidden=256, layers=2, w0=1000.0):
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    from inr_for_audio_amd.utils import calculate_snr
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    coords = torch.from_numpy(g["coords"]).reshape(-1, 1)
    target = torch.from_numpy(g["target"])
    torch.manual_seed(seed)
    m = SirenWithSnakeTanh(1, 1, hidden, layers, 0, 0, first_omega_0=w0, hidden_omega_0=30.0)
    kw = {"micro_batch": micro_batch} if micro_batch else {}
    eng = SirenEngine(m, coords, target, lr=1e-3, min_lr=1e-6, hist_cap=steps, device=dev, **kw)
    eng.step()
    eng.capture_graph()
    for _ in range(steps - 1):
        eng.step()
    out = eng.infer(coords.to(dev)).cpu().numpy()
    losses, _ = eng.history()
    return float(calculate_snr(g["target"], out)), losses


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0,1,2,3,4")
    ap.add_argument("--mbs", default="0,16384")
    ap.add_argument("--steps", type=int, default=300)
    args = ap.parse_args()
    import __graft_entry__ as ge
    ge.build()
    dev = torch.device("cuda:0")
    rows = []
    for seed in [int(s) for s in args.seeds.split(",")]:
        for mb in [int(s) for s in args.mbs.split(",")]:
            snr, losses = fit(dev, args.steps, seed, mb)
            cps = {str(k): float(losses[k - 1]) for k in (50, 100, 200, args.steps) if k <= args.steps}
            rows.append({"seed": seed, "micro_batch": mb, "snr": snr, "loss_at": cps})
            print(json.dumps(rows[-1]), flush=True)
    snrs = np.array([r["snr"] for r in rows])
    print(json.dumps({"median": float(np.median(snrs)), "min": float(snrs.min()),
                      "max": float(snrs.max()), "n": len(rows)}))


if __name__ == "__main__":
    main()
