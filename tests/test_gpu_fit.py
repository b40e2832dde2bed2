"""Fit-quality parity on the reference's own clip: SIREN 3x256, omega0 = 1000, gt_bach.wav
first 1 s (the golden target), full batch, lr 1e-3 Adam + ReduceLROnPlateau -- the GPU fit
vs the reference loop run on CPU by tests/golden/make_golden.py.

At 300 steps the lr is still 1e-3 and late Adam loss spikes make ONE run's final SNR a
random draw (reference seeds 0-7 end anywhere between 20.4 and 42.3 dB; a different fp32
summation order on the same seed moves it by as much -- DESIGN.md "Fit parity").  So:
  * the first steps must track the reference trajectory of seed 0 to storage accuracy and
    the lr schedule must be identical;
  * fit quality is compared as statistics over init seeds 0-7 against the reference's
    own runs of the same seeds: the median over seeds of the best-loss SNR
    10 log10(var(target) / min_k loss_k) -- the error floor each run reaches, insensitive
    to where a spike happens to fall -- within 0.5 dB.  The final SNR is a much noisier
    statistic: bootstrapping the reference's 8 seeds gives its median a 5.5 dB standard
    deviation (7.8 dB for a difference of two such medians), so it is only checked one-sided
    at two standard deviations, GPU median >= reference median - 15 dB (a broken optimiser,
    not spike timing).
"""
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


def test_fit_first_steps_track_reference(dev):
    tr = json.load(open(os.path.join(G, "trajectory_3x256_w1000.json")))
    eng, _, _ = _fit(dev, 20)
    losses, lrs = eng.history()
    ref = np.array(tr["loss"][:20])
    # fp16 storage: the first steps track the fp32 reference closely
    assert np.max(np.abs(losses[:5] - ref[:5]) / ref[:5]) < 2e-2
    assert np.array_equal(lrs, np.array(tr["lr"][:20]))


def test_fit_quality_vs_reference_over_seeds(dev):
    ref = json.load(open(os.path.join(G, "trajectory_3x256_w1000_seeds.json")))
    steps = ref["steps"]
    var = float(np.mean(np.load(os.path.join(G, "gt_bach_1s.npz"))["target"].astype(np.float64) ** 2))
    seeds = sorted(int(s) for s in ref["runs"])
    best_gpu, best_ref, fin_gpu, fin_ref = [], [], [], []
    for s in seeds:
        eng, _, snr = _fit(dev, steps, seed=s)
        losses, lrs = eng.history()
        r = ref["runs"][str(s)]
        best_gpu.append(10 * np.log10(var / float(np.min(losses))))
        best_ref.append(10 * np.log10(var / float(np.min(r["loss"]))))
        fin_gpu.append(snr)
        fin_ref.append(r["snr_target"])
    med = lambda x: float(np.median(x))  # noqa: E731
    print(f"\nbest-loss SNR median: GPU {med(best_gpu):.2f} dB, reference {med(best_ref):.2f} dB"
          f"\nfinal SNR median:     GPU {med(fin_gpu):.2f} dB, reference {med(fin_ref):.2f} dB"
          f"\nper seed GPU  best {np.round(best_gpu, 2).tolist()} final {np.round(fin_gpu, 2).tolist()}"
          f"\nper seed ref  best {np.round(best_ref, 2).tolist()} final {np.round(fin_ref, 2).tolist()}")
    assert abs(med(best_gpu) - med(best_ref)) < 0.5
    assert med(fin_gpu) >= med(fin_ref) - 15.0
