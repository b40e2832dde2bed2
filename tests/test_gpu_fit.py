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
    to where a spike happens to fall -- within north_star's 0.1 dB plus the fp32 reference's
    own summation-order sensitivity on this fixture (a fixed 0.35 dB, BOUND_3X256).  The final SNR is a much
    noisier statistic: bootstrapping the reference's 8 seeds gives its median a 5.5 dB
    standard deviation (7.8 dB for a difference of two such medians), so it is only checked
    one-sided at two standard deviations, GPU median >= reference median - 15 dB (a broken
    optimiser, not spike timing); the median over seeds of the tail-median loss (last 100
    steps, 4.0 dB bootstrap deviation) is checked at the same two deviations, +-11 dB.

The headline model itself (SIREN 5x1024, omega0 = 3000) has its own fixture: the reference's
run of 200 full-batch steps on gt_bach 1 s for 8 seeds (lr 1e-4 -- at run.py's 1e-3 this width
does not leave the init plateau in 200 steps -- and patience 10, so ReduceLROnPlateau drops
the lr inside the run).  The best-loss median within a fixed 4.5 dB (BOUND_5X1024_CHAOTIC: at lr
1e-4 the fp32 reference's own median moves 2.7 dB with its summation order), identical lr schedules
while they track, and no fp16 overflow step.  North_star's 0.1 dB is held PER SEED in the stable
regime (lr 3e-5) on gt_bach 1 s and on 6 s (264 600 coordinates, across a plateau lr drop).
"""
import json
import os

import numpy as np
import pytest
import torch

from errlog import log
from torch_ref import fp32_fit

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fit(dev, steps, seed=0, graph=True, H=256, L=2, w0=1000.0, lr=1e-3, patience=200):
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    from inr_for_audio_amd.utils import calculate_snr
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    coords = torch.from_numpy(g["coords"]).reshape(-1, 1)
    target = torch.from_numpy(g["target"])
    torch.manual_seed(seed)
    m = SirenWithSnakeTanh(1, 1, H, L, 0, 0, first_omega_0=w0, hidden_omega_0=30.0)
    eng = SirenEngine(m, coords, target, lr=lr, min_lr=1e-6, patience=patience, hist_cap=steps, device=dev)
    eng.step()
    if graph:
        eng.capture_graph()
    for _ in range(steps - 1):
        eng.step()
    while eng.steps_applied() < steps:
        eng.step()
    assert eng.guard_state()["overflows"] == 0
    out = eng.infer(coords.to(dev)).cpu().numpy()
    return eng, out, float(calculate_snr(g["target"], out))


def _db(var, x):
    return 10 * np.log10(var / float(x))


def _torch_gpu_best(dev, var, seed, steps, H=256, L=2, w0=1000.0, lr=1e-3, patience=200):
    """best-loss SNR of the reference loop in fp32 torch eager on this GPU (tests/torch_ref.py)"""
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    torch.manual_seed(seed)
    sd = SirenWithSnakeTanh(1, 1, H, L, 0, 0, first_omega_0=w0, hidden_omega_0=30.0).state_dict()
    losses, lrs = fp32_fit(sd, L, w0, g["coords"], g["target"], steps, lr=lr, patience=patience, device=dev)
    return _db(var, np.min(losses)), int(np.sum(np.diff(lrs) < 0))


# Fixed bounds on |median over seeds of the GPU's best-loss SNR - the reference's| (dB) for the two
# chaotic multi-seed fixtures: north_star's 0.1 dB plus two standard deviations of how far the
# reference algorithm's OWN median moves when only its summation order changes -- a paired
# bootstrap (20 000 resamples of the seeds) of median(torch fp32 eager on the GPU) - median(CPU
# reference), measured once over the fixture's 8 seeds (round 3: 3x256 +0.15 dB, std 0.11 dB;
# 5x1024 at lr 1e-4 -2.66 dB, std 2.2 dB, the per-seed shifts reaching 10.6 dB).  The torch fp32
# runs are still made and logged, but no longer widen the gate.  The per-seed 0.1 dB gates are the
# stable-regime tests (1 s and 6 s) at the end of this file.
BOUND_3X256 = 0.35
BOUND_5X1024_CHAOTIC = 4.5


def test_fit_first_steps_track_reference(dev):
    tr = json.load(open(os.path.join(G, "trajectory_3x256_w1000.json")))
    eng, _, _ = _fit(dev, 20)
    losses, lrs = eng.history()
    ref = np.array(tr["loss"][:20])
    # fp16 storage: the first steps track the fp32 reference closely
    dev5 = np.max(np.abs(losses[:5] - ref[:5]) / ref[:5])
    log("fit_3x256_first_steps", max_rel_5=dev5)
    assert dev5 < 1e-2  # measured 2.9e-3
    assert np.array_equal(lrs, np.array(tr["lr"][:20]))


def test_fit_quality_vs_reference_over_seeds(dev):
    ref = json.load(open(os.path.join(G, "trajectory_3x256_w1000_seeds.json")))
    steps = ref["steps"]
    var = float(np.mean(np.load(os.path.join(G, "gt_bach_1s.npz"))["target"].astype(np.float64) ** 2))
    seeds = sorted(int(s) for s in ref["runs"])
    best_gpu, best_ref, fin_gpu, fin_ref, tail_gpu, tail_ref, best_t32 = [], [], [], [], [], [], []
    for s in seeds:
        best_t32.append(_torch_gpu_best(dev, var, s, steps)[0])
        eng, _, snr = _fit(dev, steps, seed=s)
        losses, lrs = eng.history()
        r = ref["runs"][str(s)]
        best_gpu.append(_db(var, np.min(losses)))
        best_ref.append(_db(var, np.min(r["loss"])))
        tail_gpu.append(_db(var, np.median(losses[-100:])))
        tail_ref.append(_db(var, np.median(r["loss"][-100:])))
        fin_gpu.append(snr)
        fin_ref.append(r["snr_target"])
    med = lambda x: float(np.median(x))  # noqa: E731
    log("fit_3x256_w1000", best_gpu=med(best_gpu), best_ref=med(best_ref), best_torch_gpu_fp32=med(best_t32),
        tail_gpu=med(tail_gpu), tail_ref=med(tail_ref), final_gpu=med(fin_gpu), final_ref=med(fin_ref),
        per_seed_best_gpu=best_gpu, per_seed_best_ref=best_ref, per_seed_best_torch_gpu_fp32=best_t32)
    print(f"\nbest-loss SNR median: GPU {med(best_gpu):.2f} dB, reference {med(best_ref):.2f} dB"
          f"\nfinal SNR median:     GPU {med(fin_gpu):.2f} dB, reference {med(fin_ref):.2f} dB"
          f"\nper seed GPU  best {np.round(best_gpu, 2).tolist()} final {np.round(fin_gpu, 2).tolist()}"
          f"\nper seed ref  best {np.round(best_ref, 2).tolist()} final {np.round(fin_ref, 2).tolist()}")
    assert abs(med(best_gpu) - med(best_ref)) < BOUND_3X256
    # ... and inside this run's own envelope: the reference's median moved by its summation order
    # alone (fp32 torch on this GPU), plus north_star's 0.1 dB (the fixed bound is the cap)
    assert abs(med(best_gpu) - med(best_ref)) < 0.1 + abs(med(best_t32) - med(best_ref))
    assert med(fin_gpu) >= med(fin_ref) - 15.0
    assert abs(med(tail_gpu) - med(tail_ref)) < 11.0


def test_fit_quality_headline_model_over_seeds(dev):
    """SIREN 5x1024 (BASELINE cfg2's model), omega0 = 3000, gt_bach 1 s, 200 full-batch steps
    per seed against the reference's own runs (tests/golden/trajectory_5x1024_w3000_seeds.json,
    made by make_golden.py --fullsize-seeds): best-loss SNR median within 0.1 dB; every run
    applies its ReduceLROnPlateau drops; the first steps track the reference and the lr trace
    is identical until the first drop."""
    ref = json.load(open(os.path.join(G, "trajectory_5x1024_w3000_seeds.json")))
    var = float(np.mean(np.load(os.path.join(G, "gt_bach_1s.npz"))["target"].astype(np.float64) ** 2))
    best_gpu, best_ref, drops_gpu, drops_ref, fin_gpu, fin_ref, best_t32, drops_t32 = [], [], 0, 0, [], [], [], 0
    for s in sorted(int(k) for k in ref["runs"]):
        r = ref["runs"][str(s)]
        b, d = _torch_gpu_best(dev, var, s, ref["steps"], H=1024, L=4, w0=ref["omega0"], lr=ref["lr0"],
                               patience=ref["patience"])
        best_t32.append(b)
        drops_t32 += d
        eng, _, snr = _fit(dev, ref["steps"], seed=s, H=1024, L=4, w0=ref["omega0"], lr=ref["lr0"],
                           patience=ref["patience"])
        losses, lrs = eng.history()
        rl = np.array(r["loss"])
        best_gpu.append(_db(var, np.min(losses)))
        best_ref.append(_db(var, np.min(rl)))
        fin_gpu.append(snr)
        fin_ref.append(r["snr_target"])
        drops_gpu += int(np.sum(np.diff(lrs) < 0))
        drops_ref += int(np.sum(np.diff(r["lr"]) < 0))
        dev3 = np.max(np.abs(losses[:3] - rl[:3]) / rl[:3])
        log(f"fit_5x1024_first_steps[{s}]", max_rel_3=dev3)
        assert dev3 < 1e-2, s  # measured <= 2.2e-3
        first = int(np.argmax(np.diff(r["lr"]) < 0)) if np.any(np.diff(r["lr"]) < 0) else len(lrs) - 1
        assert np.array_equal(lrs[:min(first, 10)], np.array(r["lr"][:min(first, 10)])), s
    med = lambda x: float(np.median(x))  # noqa: E731
    log("fit_5x1024_w3000", best_gpu=med(best_gpu), best_ref=med(best_ref), best_torch_gpu_fp32=med(best_t32),
        final_gpu=med(fin_gpu), final_ref=med(fin_ref), drops_gpu=drops_gpu, drops_ref=drops_ref, drops_t32=drops_t32,
        per_seed_best_gpu=best_gpu, per_seed_best_ref=best_ref, per_seed_best_torch_gpu_fp32=best_t32)
    print(f"\n5x1024 best-loss SNR median: GPU {med(best_gpu):.2f} dB, reference {med(best_ref):.2f} dB; "
          f"lr drops GPU {drops_gpu} reference {drops_ref}")
    assert drops_ref > 0 and drops_gpu > 0
    assert abs(med(best_gpu) - med(best_ref)) < BOUND_5X1024_CHAOTIC
    # the per-run envelope as well (see test_fit_quality_vs_reference_over_seeds)
    assert abs(med(best_gpu) - med(best_ref)) < 0.1 + abs(med(best_t32) - med(best_ref))


def test_fit_headline_model_stable_regime_per_seed(dev):
    """SIREN 5x1024, omega0 = 3000, gt_bach 1 s at lr 3e-5 (tests/golden/
    trajectory_5x1024_w3000_lr3e-5_seeds.json): a regime where the reference's trajectory does not
    depend on summation order (two CPU thread counts agree to 1.2e-5 in every step's loss over 40
    steps), so the HIP path can be held to north_star's 0.1 dB per seed, not as a median: the
    whole 150-step loss trajectory tracks the reference and each seed's final SNR (the fit of the
    final weights to the target) is within 0.1 dB."""
    from inr_for_audio_amd.utils import calculate_snr
    ref = json.load(open(os.path.join(G, "trajectory_5x1024_w3000_lr3e-5_seeds.json")))
    var = float(np.mean(np.load(os.path.join(G, "gt_bach_1s.npz"))["target"].astype(np.float64) ** 2))
    rows = {}
    for s in sorted(int(k) for k in ref["runs"]):
        r = ref["runs"][str(s)]
        eng, out, snr = _fit(dev, ref["steps"], seed=s, H=1024, L=4, w0=ref["omega0"], lr=ref["lr0"],
                             patience=ref["patience"])
        losses, lrs = eng.history()
        rl = np.array(r["loss"])
        dev_db = np.abs(10 * np.log10(losses / rl))
        rows[s] = {"final_snr_gpu": snr, "final_snr_ref": r["snr_target"], "max_step_db": float(dev_db.max()),
                   "best_gpu": _db(var, np.min(losses)), "best_ref": _db(var, np.min(rl))}
        assert np.array_equal(lrs, np.array(r["lr"])), s
    log("fit_5x1024_stable", seeds=rows)
    print("\n" + json.dumps(rows, indent=1))
    for s, v in rows.items():
        assert abs(v["final_snr_gpu"] - v["final_snr_ref"]) < 0.1, (s, v)
        assert abs(v["best_gpu"] - v["best_ref"]) < 0.1, (s, v)
        assert v["max_step_db"] < 0.1, (s, v)


def _fit6(dev, steps, seed, patience, lr, omega0=3000.0, factor=0.8, min_lr=1e-6):
    """SIREN 5x1024 on gt_bach 6 s (264 600 coordinates: a quarter of cfg2's 2^20 rows, the
    longest whole-second clip of the reference's gt_bach.wav): the fused path with its production
    settings (256 tiles, fused head backward, graph replay)."""
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    from inr_for_audio_amd.utils import calculate_snr, get_coord
    target = np.load(os.path.join(G, "gt_bach_6s.npz"))["target"]
    coords = get_coord(target.size, 1).reshape(-1, 1)
    torch.manual_seed(seed)
    m = SirenWithSnakeTanh(1, 1, 1024, 4, 0, 0, first_omega_0=omega0, hidden_omega_0=30.0)
    eng = SirenEngine(m, coords, torch.from_numpy(target), lr=lr, min_lr=min_lr, factor=factor, patience=patience,
                      hist_cap=steps, device=dev)
    assert eng.lib.siren_nt_tile(eng.rows, 1024) == 256
    eng.step()
    eng.capture_graph()
    while eng.steps_applied() < steps:
        eng.step()
    assert eng.guard_state()["overflows"] == 0
    out = eng.infer(coords.to(dev)).cpu().numpy()
    return eng, float(calculate_snr(target, out)), float(np.mean(target.astype(np.float64) ** 2))


@pytest.mark.parametrize("fixture", ["trajectory_5x1024_w3000_lr3e-5_6s_seeds.json",
                                     "trajectory_5x1024_w3000_lr3e-5_6s_p3.json"])
def test_fit_headline_model_6s_per_seed(dev, fixture):
    """cfg2's model on cfg2-scale data: SIREN 5x1024, omega0 3000, gt_bach 6 s,
    60 full-batch steps at lr 3e-5 per seed against the reference's own runs (make_golden.py
    --fullsize-seeds --duration 6).  The _p3 fixture lowers the plateau patience to 3 so the run
    crosses a ReduceLROnPlateau drop.  Per seed: the lr trace is identical, every step's loss is
    within STEP_DB of the reference's, and the final and best-loss SNR within north_star's 0.1 dB."""
    ref = json.load(open(os.path.join(G, fixture)))
    assert ref["duration"] == 6 and ref["hidden"] == 1024
    rows = {}
    for s in sorted(int(k) for k in ref["runs"]):
        r = ref["runs"][str(s)]
        eng, snr, var = _fit6(dev, ref["steps"], s, ref["patience"], ref["lr0"])
        losses, lrs = eng.history()
        rl = np.array(r["loss"])
        step_db = np.abs(10 * np.log10(losses / rl))
        rows[s] = {"final_snr_gpu": snr, "final_snr_ref": r["snr_target"], "max_step_db": float(step_db.max()),
                   "argmax_step": int(step_db.argmax()), "best_gpu": _db(var, np.min(losses)),
                   "best_ref": _db(var, np.min(rl)), "drops_ref": int(np.sum(np.diff(r["lr"]) < 0))}
        assert np.array_equal(lrs, np.array(r["lr"])), s
    log(f"fit_5x1024_6s[{fixture}]", seeds=rows)
    print("\n" + json.dumps(rows, indent=1))
    if "_p3" in fixture:
        assert all(v["drops_ref"] >= 1 for v in rows.values())
    for s, v in rows.items():
        assert abs(v["final_snr_gpu"] - v["final_snr_ref"]) < 0.1, (s, v)
        assert abs(v["best_gpu"] - v["best_ref"]) < 0.1, (s, v)
        assert v["max_step_db"] < STEP_DB, (s, v)


# every step's loss of a 6 s run within this many dB of the reference's: measured worst step
# 0.0011 dB over the three runs (final SNR within 0.0006 dB); the 0.1 dB SNR gates are north_star's
STEP_DB = 0.01


# the stable window of the 400-step 6 s run: the reference's own steps leave the summation-order-
# independent regime near step 100 (Adam loss oscillations from step 112 on; the fp32 torch run on
# the GPU already deviates 0.055 dB at step 100, tools/fit6_probe.py, profiles/r16/fit6_probe_lr3e-5.json)
STABLE_STEPS_6S = 80


# the fixed-gate reconstruction fixture: omega0 18000 (the 1 s fixtures' 3000 per
# second of audio), lr 1e-5, 140 full-batch steps -- SNR_target 22.3 dB in the regime where the
# reference's trajectory does not depend on summation order.  Probed on the GPU (tools/fit6_probe.py,
# profiles/r17/probe6s_*.json): every run at omega0 9000-24000 and lr 1e-5 .. 1e-4 keeps two
# implementations within 0.01-0.03 dB until Adam's first loss spike (step 130-210 here), after which
# they land 0.1-1 dB apart even when ReduceLROnPlateau anneals (patience 3, factor 0.5: 0.083 dB at
# step 300); 140 steps stay before that spike on every run probed at this setting
FIXED_6S = "fit_5x1024_w18000_6s.json"
STEP_DB_18K = 0.05   # per-step loss gate of that run (fp32 torch on the GPU: <= 0.011 dB by step 150)


def test_fit_headline_model_6s_fixed_snr_gate(dev):
    """North_star's "reconstruction SNR within 0.1 dB of the reference" at a FIXED 0.1 dB: SIREN 5x1024
    on gt_bach 6 s, fitted to SNR_target > 20 dB against the reference's own runs (make_golden.py
    --fullsize-seeds 0,1 --duration 6 --omega0 18000 --lr 1e-5 --trajectory-steps 140).  Per seed:
    SNR_target of the final weights (utils.py:77-97, what run.py:302-335 reports) within 0.1 dB of the
    reference's, every step's loss within STEP_DB_18K, the lr trace identical; and plain fp32 torch on
    the GPU (the reference algorithm with only its summation order changed) lands within 0.05 dB of the
    reference at the last step -- the fixture's own acceptance check."""
    from torch_ref import fp32_fit
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    from inr_for_audio_amd.utils import calculate_snr, get_coord
    ref = json.load(open(os.path.join(G, FIXED_6S)))
    assert ref["duration"] == 6 and ref["hidden"] == 1024 and ref["omega0"] == 18000.0
    target = np.load(os.path.join(G, "gt_bach_6s.npz"))["target"]
    coords = get_coord(target.size, 1).reshape(-1, 1)
    rows = {}
    for s in sorted(int(k) for k in ref["runs"]):
        r = ref["runs"][str(s)]
        assert r["snr_target"] > 20.0, r["snr_target"]
        eng, snr, var = _fit6(dev, ref["steps"], s, ref["patience"], ref["lr0"], omega0=ref["omega0"],
                              factor=ref["factor"], min_lr=ref["min_lr"])
        losses, lrs = eng.history()
        rl = np.array(r["loss"])
        torch.manual_seed(s)
        sd = SirenWithSnakeTanh(1, 1, 1024, 4, 0, 0, first_omega_0=ref["omega0"], hidden_omega_0=30.0).state_dict()
        t32, _, o32 = fp32_fit(sd, 4, ref["omega0"], coords, target, ref["steps"], lr=ref["lr0"],
                               patience=ref["patience"], factor=ref["factor"], min_lr=ref["min_lr"], device=dev,
                               final=True)
        rows[s] = {"snr_target_gpu": snr, "snr_target_ref": r["snr_target"],
                   "snr_target_torch_gpu_fp32": float(calculate_snr(target, o32)),
                   "max_step_db": float(np.max(np.abs(10 * np.log10(losses / rl)))),
                   "max_step_db_torch_gpu_fp32": float(np.max(np.abs(10 * np.log10(t32 / rl))))}
        assert np.array_equal(lrs, np.array(r["lr"])), s
    log("fit_5x1024_6s_fixed_gate", seeds=rows)
    print("\n" + json.dumps(rows, indent=1))
    for s, v in rows.items():
        assert abs(v["snr_target_gpu"] - v["snr_target_ref"]) < 0.1, (s, v)
        assert v["max_step_db"] < STEP_DB_18K, (s, v)
        assert abs(v["snr_target_torch_gpu_fp32"] - v["snr_target_ref"]) < 0.05, (s, v)


def test_fit_headline_model_6s_converged(dev):
    """cfg2's model on cfg2-scale data fitted towards the reference's converged
    reconstruction -- SIREN 5x1024, omega0 3000, gt_bach 6 s (264 600 coordinates), 400 full-batch
    steps at lr 3e-5, seed 0, against the reference's own run (make_golden.py --fullsize-seeds 0
    --duration 6 --trajectory-steps 400: SNR_target 14.53 dB, best-loss SNR 14.79 dB; the SNR still
    rises ~0.2 dB per 25 steps there, so 20 dB is several thousand CPU steps away).  Gates: every
    step of the stable window within STEP_DB and the best-loss SNR within north_star's 0.1 dB.  The
    final reconstruction SNR is logged only: past step ~100 this fit is in the regime where Adam's loss
    oscillations amplify rounding (fp32 torch on the GPU ends 0.36 dB from the CPU run), so it cannot
    carry a fixed 0.1 dB gate; test_fit_headline_model_6s_fixed_snr_gate does."""
    from torch_ref import fp32_fit
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    from inr_for_audio_amd.utils import get_coord
    ref = json.load(open(os.path.join(G, "trajectory_5x1024_w3000_lr3e-5_6s_400.json")))
    assert ref["duration"] == 6 and ref["steps"] == 400
    r = ref["runs"]["0"]
    steps = ref["steps"]
    eng, snr, var = _fit6(dev, steps, 0, ref["patience"], ref["lr0"])
    losses, lrs = eng.history()
    rl = np.array(r["loss"])
    step_db = np.abs(10 * np.log10(losses / rl))
    target = np.load(os.path.join(G, "gt_bach_6s.npz"))["target"]
    torch.manual_seed(0)
    sd = SirenWithSnakeTanh(1, 1, 1024, 4, 0, 0, first_omega_0=3000.0, hidden_omega_0=30.0).state_dict()
    coords = get_coord(target.size, 1).reshape(-1, 1)
    t32, _ = fp32_fit(sd, 4, 3000.0, coords, target, steps, lr=ref["lr0"], patience=ref["patience"], device=dev)
    row = {"final_snr_gpu": snr, "final_snr_ref": r["snr_target"],
           "best_gpu": _db(var, np.min(losses)), "best_ref": _db(var, np.min(rl)), "best_torch_gpu_fp32": _db(var, np.min(t32)),
           "last_gpu": _db(var, losses[-1]), "last_ref": _db(var, rl[-1]), "last_torch_gpu_fp32": _db(var, t32[-1]),
           "max_step_db_stable": float(step_db[:STABLE_STEPS_6S].max()), "max_step_db_all": float(step_db.max()),
           "max_step_db_torch_gpu_fp32": float(np.max(np.abs(10 * np.log10(t32 / rl)))),
           "spikes_gpu": int(np.sum(losses[1:] > 1.05 * losses[:-1])), "spikes_ref": int(np.sum(rl[1:] > 1.05 * rl[:-1]))}
    log("fit_5x1024_6s_converged", **row)
    print("\n" + json.dumps(row, indent=1))
    assert np.array_equal(lrs, np.array(r["lr"]))
    assert row["max_step_db_stable"] < STEP_DB, row
    assert abs(row["best_gpu"] - row["best_ref"]) < 0.1, row
    # the final weights of this run come out of Adam's oscillating regime, where the reference itself
    # is not reproducible to 0.1 dB (fp32 torch on the GPU ends 0.36 dB from it): logged, not gated
    # here -- the fixed 0.1 dB reconstruction gate is test_fit_headline_model_6s_fixed_snr_gate's
