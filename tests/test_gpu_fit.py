"""Fit-quality parity on the reference's own clip: SIREN 3x256, omega0 = 1000, gt_bach.wav
first 1 s (the golden target), full batch, lr 1e-3 Adam + ReduceLROnPlateau -- the GPU fit
vs the reference loop run on CPU by tests/golden/make_golden.py."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fit(dev, steps, seed=0, graph=True):
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    from inr_for_audio_amd.utils import calculate_snr
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    coords = torch.from_numpy(g["coords"]).reshape(-1, 1)
    target = torch.from_numpy(g["target"])
    torch.manual_seed(seed)
    m = SirenWithSnakeTanh(1, 1, 256, 2, 0, 0, first_omega_0=1000.0, hidden_omega_0=30.0)
    eng = SirenEngine(m, coords, target, lr=1e-3, min_lr=1e-6, hist_cap=steps, device=dev)
    eng.step()
    if graph:
        eng.capture_graph()
    for _ in range(steps - 1):
        eng.step()
    out = eng.infer(coords.to(dev)).cpu().numpy()
    return eng, out, float(calculate_snr(g["target"], out))


def test_fit_snr_vs_reference(dev):
    tr = json.load(open(os.path.join(G, "trajectory_3x256_w1000.json")))
    steps = tr["steps"]
    eng, out, snr = _fit(dev, steps)
    losses, lrs = eng.history()
    ref = np.array(tr["loss"])
    print(f"\nGPU SNR_target {snr:.3f} dB vs reference {tr['snr_target']:.3f} dB; "
          f"final loss {losses[-1]:.3e} vs {ref[-1]:.3e}")
    # the first steps track the fp32 reference within bf16 accuracy
    assert np.max(np.abs(losses[:5] - ref[:5]) / ref[:5]) < 5e-2
    assert np.array_equal(lrs, np.array(tr["lr"]))
    assert abs(snr - tr["snr_target"]) < 3.0
