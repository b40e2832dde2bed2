"""How many steps does cfg2's model need on cfg2-scale data to reach a converged SNR?  (Measurement
for the VERDICT r3 item 6 fixture, not a test.)

SIREN 5x1024, omega0 3000 on gt_bach 6 s (264 600 coordinates), full batch, seed 0, at the given lr:
the HIP engine (production settings) and the reference loop in plain fp32 torch on the GPU
(tests/torch_ref.py) side by side; prints SNR_target of the training loss every `--every` steps and
the per-step deviation between the two, so the CPU reference run (make_golden.py --fullsize-seeds
--duration 6) can be sized to the step count where the fit passes ~20 dB while still in the regime
where the trajectory does not depend on summation order.

    python tools/fit6_probe.py --steps 800 --lr 3e-5 > gpurun_out/fit6.json
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
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=800)
    ap.add_argument("--lr", type=float, default=3e-5)
    ap.add_argument("--patience", type=int, default=200)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--every", type=int, default=25)
    ap.add_argument("--omega0", type=float, default=3000.0)
    ap.add_argument("--factor", type=float, default=0.8)
    ap.add_argument("--min-lr", type=float, default=1e-6)
    ap.add_argument("--clip", default="gt_bach_6s.npz", help="tests/golden target file")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 torch comparator")
    args = ap.parse_args()
    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    from inr_for_audio_amd.utils import get_coord
    from torch_ref import fp32_fit
    dev = torch.device("cuda:0")
    target = np.load(os.path.join(ROOT, "tests", "golden", args.clip))["target"]
    var = float(np.mean(target.astype(np.float64) ** 2))
    coords = get_coord(target.size, 1).reshape(-1, 1)
    torch.manual_seed(args.seed)
    m = SirenWithSnakeTanh(1, 1, 1024, 4, 0, 0, first_omega_0=args.omega0, hidden_omega_0=30.0)
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    eng = SirenEngine(m, coords, torch.from_numpy(target), lr=args.lr, min_lr=args.min_lr, factor=args.factor,
                      patience=args.patience, hist_cap=args.steps, device=dev)
    eng.step()
    eng.capture_graph()
    while eng.steps_applied() < args.steps:
        eng.step()
    hip, hip_lr = eng.history()
    from inr_for_audio_amd.utils import calculate_snr
    snr_final_hip = float(calculate_snr(target, eng.infer(coords.to(dev)).cpu().numpy()))
    if args.no_fp32:
        t32, t32_lr = hip, hip_lr
        snr_final_t32 = None
    else:
        t32, t32_lr, o32 = fp32_fit(sd0, 4, args.omega0, coords, target, args.steps, lr=args.lr,
                                    patience=args.patience, device=dev, factor=args.factor, min_lr=args.min_lr,
                                    final=True)
        snr_final_t32 = float(calculate_snr(target, o32))
    db = lambda x: 10 * np.log10(var / np.asarray(x))  # noqa: E731
    rows = []
    for k in range(0, args.steps, args.every):
        rows.append({"step": k, "snr_hip": float(db(hip[k])), "snr_fp32_gpu": float(db(t32[k])),
                     "max_dev_db_so_far": float(np.max(np.abs(db(hip[:k + 1]) - db(t32[:k + 1])))),
                     "lr": float(hip_lr[k])})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"steps": args.steps, "lr": args.lr, "patience": args.patience, "seed": args.seed,
                      "omega0": args.omega0, "factor": args.factor, "clip": args.clip,
                      "snr_target_final_weights_hip": snr_final_hip, "snr_target_final_weights_fp32_gpu": snr_final_t32,
                      "lr_end": float(hip_lr[-1]),
                      "rows": rows, "final_snr_hip": float(db(hip[-1])), "final_snr_fp32_gpu": float(db(t32[-1])),
                      "overflows": eng.guard_state()["overflows"]}))


if __name__ == "__main__":
    main()
