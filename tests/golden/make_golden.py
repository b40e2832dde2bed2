"""Generate the golden fixtures in tests/golden/ from the REFERENCE implementation.

Runs only in the build container, where /root/reference (senyuanfan/inr-for-audio) is
mounted read-only.  Imports the reference's own models.py / utils.py; their top-level
imports of packages absent here (torchaudio, rff, librosa, torchsummary, matplotlib) are
satisfied with empty stub modules -- none of them is used by the code paths exercised
(SURVEY.md §8c).  The reference code itself is never copied: only the numbers it produces
are written, as small .npz / .json data files.

    python tests/golden/make_golden.py [--trajectory-steps 300]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    for name in ["torchaudio", "rff", "librosa", "torchsummary", "matplotlib", "matplotlib.pyplot"]:
        if name not in sys.modules:
            try:
                __import__(name)
            except ImportError:
                mod = types.ModuleType(name)
                if name == "torchsummary":
                    mod.summary = lambda *a, **k: None
                if name == "matplotlib":
                    mod.pyplot = types.ModuleType("matplotlib.pyplot")
                    sys.modules["matplotlib.pyplot"] = mod.pyplot
                sys.modules[name] = mod
    sys.path.insert(0, REF)
    import models as ref_models  # noqa: E402
    import utils as ref_utils  # noqa: E402
    return ref_models, ref_utils


def siren(ref_models, H, L, w0, w=30.0, in_dim=1, seed=0):
    torch.manual_seed(seed)
    return ref_models.SirenWithSnakeTanh(in_features=in_dim, out_features=1, hidden_features=H,
                                         num_sine=L, num_snake=0, num_tanh=0, first_omega_0=w0,
                                         hidden_omega_0=w)


def sd_np(model):
    return {k: v.detach().numpy().astype(np.float32).copy() for k, v in model.state_dict().items()}


def summary(sd):
    return {k: {"shape": list(v.shape), "sum": float(v.astype(np.float64).sum()),
                "sumsq": float((v.astype(np.float64) ** 2).sum()),
                "head": v.reshape(-1)[:8].tolist()} for k, v in sd.items()}


def fwd_bwd(model, coords, target):
    model.zero_grad()
    out = model(coords.reshape(1, -1, coords.shape[-1]))
    loss = torch.nn.MSELoss()(out, target.reshape(1, -1, 1))
    loss.backward()
    grads = {k: p.grad.detach().numpy().copy() for k, p in model.named_parameters()}
    return out.detach().numpy().reshape(-1), float(loss), grads


def restated_loop(model, coords, target, steps, lr=1e-3, min_lr=1e-6, patience=200, factor=0.8):
    """run.py:156-187 on CPU around the reference model (alpha=0: the STFT term is exactly
    zero; best_model aliases model, run.py:173)."""
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=factor, patience=patience,
                                                       min_lr=min_lr)
    mse = torch.nn.MSELoss()
    x = coords.reshape(1, coords.shape[0], -1)
    y = target.reshape(1, -1, 1)
    losses, lrs = [], []
    for _ in range(steps):
        out = model(x)
        loss = mse(out, y)
        losses.append(float(loss.item()))
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step(loss)
        lrs.append(float(sched.get_last_lr()[0]))
    with torch.no_grad():
        final = model(x).numpy().reshape(-1)
    return np.array(losses), np.array(lrs), final


def act_fixtures(ref_models, ref_utils, steps):
    """Snake / Tanh layers (models.py:185-241, 356-372): init, one
    forward/backward and a short full-batch trajectory of train()'s default architecture
    (num_sine=2, num_snake=2, a_initial=0.5) plus a sine/Snake/Tanh mix and an a=None init."""
    wav = os.path.join(REF, "gt_bach.wav")
    coords, target = ref_utils.WaveformFitting(wav, duration=1, decimation=1)[0]
    idx = np.arange(0, 44100, 21)
    c_sub, t_sub = coords[idx], target[idx]
    cfgs = {  # name: (H, num_sine, num_snake, num_tanh, omega0, a_initial, seed, first_linear, last_linear)
        "default": (256, 2, 2, 0, 1000.0, 0.5, 1, False, True),
        "mix": (128, 1, 2, 1, 1000.0, 0.5, 0, False, True),
        "tanh": (128, 1, 0, 2, 1000.0, 0.5, 2, False, True),
        "firstlin": (128, 1, 1, 0, 1000.0, 0.5, 5, True, True),
        "lastsine": (128, 2, 0, 0, 1000.0, 0.5, 6, False, False),
        "both": (128, 1, 1, 1, 1000.0, 2.0, 7, True, False),
    }
    fb = {"subset_idx": idx}
    for name, (H, ns, nk, nt, w0, a0, seed, fl, ll) in cfgs.items():
        torch.manual_seed(seed)
        m = ref_models.SirenWithSnakeTanh(in_features=1, out_features=1, hidden_features=H, num_sine=ns,
                                          num_snake=nk, num_tanh=nt, first_linear=fl, last_linear=ll,
                                          first_omega_0=w0, hidden_omega_0=30.0, a_initial=a0)
        for k, v in sd_np(m).items():
            fb[f"{name}_init_{k}"] = v
        out, loss, grads = fwd_bwd(m, c_sub, t_sub)
        fb[f"{name}_out"] = out
        fb[f"{name}_loss"] = np.array([loss])
        for k, gr in grads.items():
            fb[f"{name}_grad_{k}"] = gr
    torch.manual_seed(4)
    m = ref_models.SirenWithSnakeTanh(in_features=1, out_features=1, hidden_features=128, num_sine=1,
                                      num_snake=1, num_tanh=0, first_omega_0=1000.0, a_initial=None)
    for k, v in sd_np(m).items():
        fb[f"expinit_init_{k}"] = v
    np.savez_compressed(os.path.join(OUT, "fwd_bwd_act.npz"), **fb)
    if steps > 0:
        torch.manual_seed(1)
        m = ref_models.SirenWithSnakeTanh(in_features=1, out_features=1, hidden_features=256, num_sine=2,
                                          num_snake=2, num_tanh=0, first_omega_0=1000.0, a_initial=0.5)
        losses, lrs, final = restated_loop(m, coords, target, steps)
        tgt = target.numpy().reshape(-1)
        json.dump({"steps": steps, "omega0": 1000.0, "hidden": 256, "num_sine": 2, "num_snake": 2,
                   "a_initial": 0.5, "seed": 1, "loss": losses.tolist(), "lr": lrs.tolist(),
                   "snr_target": float(ref_utils.calculate_snr(tgt, final))},
                  open(os.path.join(OUT, "trajectory_snake_default.json"), "w"))
        print(f"snake default: final loss {losses[-1]:.3e} min {losses.min():.3e}", flush=True)


def mdct_fixtures(ref_models, steps):
    """MDCT-domain target: the reference's STMDCT / ISTMDCT on a seeded signal
    (mdct.py), MDCTFitting on gt_bach 1 s with N = 2048 (utils.py:312-414, takelog off / on),
    the run.py:258-290 inversion of a synthetic model output, and a short full-batch fit of
    a SIREN 5x512 on the (bin, frame) grid (in = 2)."""
    import contextlib
    import io
    import mdct as ref_mdct  # noqa: E402  (the reference's own module)
    import utils as ref_utils  # noqa: E402
    rng = np.random.default_rng(7)
    x = rng.uniform(-1, 1, 5000).astype(np.float32)
    kat = {"x": x}
    for N in (1024, 2048):
        c = ref_mdct.STMDCT(x, N=N)
        kat[f"stmdct_{N}"] = c
        kat[f"istmdct_{N}"] = ref_mdct.ISTMDCT(c, N=N)
    np.savez_compressed(os.path.join(OUT, "mdct_kat.npz"), **kat)
    wav = os.path.join(REF, "gt_bach.wav")
    fit = {}
    for takelog in (False, True):
        with contextlib.redirect_stdout(io.StringIO()):
            d = ref_utils.MDCTFitting(wav, duration=1, N=2048, takelog=takelog)
        tag = "log" if takelog else "lin"
        fit[f"{tag}_pixels"] = d.pixels.reshape(-1)
        fit[f"{tag}_stats"] = np.array([d.mean, d.scale, d.shift, d.height, d.width], np.float64)
        # run.py:258-259 and 281-290 applied to a synthetic model output
        out = (0.9 * d.pixels.reshape(-1) + 0.01 * np.sin(np.arange(d.pixels.size))).astype(np.float32)
        o = torch.from_numpy(out)
        if takelog:
            o = torch.exp(o)
        spec = (o.reshape(d.height, d.width) * d.scale + d.mean - d.shift).numpy()
        if takelog:
            spec = np.exp(spec)
        fit[f"{tag}_model_out"] = out
        fit[f"{tag}_signal"] = ref_mdct.ISTMDCT(spec, N=2048).reshape(-1).astype(np.float32)
        if not takelog:
            coords = d.coords
            target = torch.from_numpy(d.pixels)
    np.savez_compressed(os.path.join(OUT, "mdct_fitting_1s.npz"), **fit)
    if steps > 0:
        torch.manual_seed(0)
        m = ref_models.SirenWithSnakeTanh(in_features=2, out_features=1, hidden_features=512, num_sine=4,
                                          num_snake=0, num_tanh=0, first_omega_0=1000.0, hidden_omega_0=30.0)
        losses, lrs, _ = restated_loop(m, coords, target, steps)
        json.dump({"steps": steps, "omega0": 1000.0, "hidden": 512, "num_sine": 4, "seed": 0, "N": 2048,
                   "loss": losses.tolist(), "lr": lrs.tolist()},
                  open(os.path.join(OUT, "trajectory_mdct_5x512.json"), "w"))
        print(f"mdct 5x512: losses {losses[:3]} ... {losses[-1]:.3e}", flush=True)


def kan_fixtures(ref_utils, steps):
    """KAN variant (kan.py, run.py:92-93): init state_dicts (with the grid
    buffers), one forward/backward on the 2100-point gt_bach subset, and a short full-batch
    trajectory of KAN([1, 64, 64, 1]) on gt_bach 1 s."""
    import kan as ref_kan  # noqa: E402  (the reference's own module)
    wav = os.path.join(REF, "gt_bach.wav")
    coords, target = ref_utils.WaveformFitting(wav, duration=1, decimation=1)[0]
    idx = np.arange(0, 44100, 21)
    fb = {"subset_idx": idx}
    for name, widths, seed in (("k64", [1, 64, 64, 1], 0), ("k128", [1, 128, 128, 1], 3)):
        torch.manual_seed(seed)
        m = ref_kan.KAN(widths)
        for k, v in sd_np(m).items():
            fb[f"{name}_init_{k}"] = v
        if name == "k64":
            out, loss, grads = fwd_bwd(m, coords[idx], target[idx])
            fb[f"{name}_out"] = out
            fb[f"{name}_loss"] = np.array([loss])
            for k, gr in grads.items():
                fb[f"{name}_grad_{k}"] = gr
    np.savez_compressed(os.path.join(OUT, "kan_fwd_bwd.npz"), **fb)
    if steps > 0:
        torch.manual_seed(0)
        m = ref_kan.KAN([1, 64, 64, 1])
        losses, lrs, _ = restated_loop(m, coords, target, steps)
        json.dump({"steps": steps, "widths": [1, 64, 64, 1], "seed": 0, "loss": losses.tolist(), "lr": lrs.tolist()},
                  open(os.path.join(OUT, "trajectory_kan_64.json"), "w"))
        print(f"kan: losses {losses[:3]} ... {losses[-1]:.3e}", flush=True)


def snake_seed_trajectories(ref_models, ref_utils, seeds, steps):
    """train()'s default architecture (num_sine=2, num_snake=2, a_initial=0.5, H=256,
    omega0=1000) over several init seeds: loss / lr traces for the multi-seed fit protocol."""
    wav = os.path.join(REF, "gt_bach.wav")
    coords, target = ref_utils.WaveformFitting(wav, duration=1, decimation=1)[0]
    tgt = target.numpy().reshape(-1)
    out = {"steps": steps, "omega0": 1000.0, "hidden": 256, "num_sine": 2, "num_snake": 2,
           "a_initial": 0.5, "runs": {}}
    for s in seeds:
        torch.manual_seed(s)
        m = ref_models.SirenWithSnakeTanh(in_features=1, out_features=1, hidden_features=256, num_sine=2,
                                          num_snake=2, num_tanh=0, first_omega_0=1000.0, a_initial=0.5)
        losses, lrs, final = restated_loop(m, coords, target, steps)
        out["runs"][str(s)] = {"loss": losses.tolist(), "lr": lrs.tolist(),
                               "snr_target": float(ref_utils.calculate_snr(tgt, final))}
        print(f"snake seed {s}: final {losses[-1]:.3e} min {losses.min():.3e}", flush=True)
        json.dump(out, open(os.path.join(OUT, "trajectory_snake_default_seeds.json"), "w"))


def seed_trajectories(ref_models, ref_utils, seeds, steps):
    """The full-batch trajectory of run.py:156-190 for several init seeds: at 300 steps the lr
    is still 1e-3 and late Adam loss spikes make one run's final SNR a random draw, so the
    fit-quality parity test compares statistics over seeds (tests/test_gpu_fit.py)."""
    wav = os.path.join(REF, "gt_bach.wav")
    coords, target = ref_utils.WaveformFitting(wav, duration=1, decimation=1)[0]
    tgt = target.numpy().reshape(-1)
    out = {"steps": steps, "omega0": 1000.0, "hidden": 256, "num_sine": 2, "runs": {}}
    for s in seeds:
        m = siren(ref_models, 256, 2, 1000.0, seed=s)
        losses, lrs, final = restated_loop(m, coords, target, steps)
        out["runs"][str(s)] = {"loss": losses.tolist(), "lr": lrs.tolist(),
                               "snr_target": float(ref_utils.calculate_snr(tgt, final))}
        print(f"seed {s}: final loss {losses[-1]:.3e} min {losses.min():.3e} "
              f"snr {out['runs'][str(s)]['snr_target']:.2f}", flush=True)
    json.dump(out, open(os.path.join(OUT, "trajectory_3x256_w1000_seeds.json"), "w"))


def multiwave_fixtures(ref_utils):
    """MultiWaveformFitting (utils.py:186-231, BASELINE cfg3's (t, ch) grid) on a seeded
    synthetic 3-channel 4 kHz clip (int16 and float32 files): num_channels 2 and 1, with and
    without the FIR decimation (lp=True).  The input clip is stored too, so the test rebuilds
    the same wav files."""
    import contextlib
    import io
    import tempfile
    from scipy.io import wavfile
    rng = np.random.default_rng(11)
    fs, secs = 4000, 2
    t = np.arange(fs * secs + 123) / fs
    clip = np.stack([0.6 * np.sin(2 * np.pi * 440 * t) + 0.05 * rng.standard_normal(t.size),
                     0.4 * np.sin(2 * np.pi * 660 * t + 0.3) + 0.05 * rng.standard_normal(t.size),
                     0.2 * rng.standard_normal(t.size)], axis=1).astype(np.float32)
    fx = {"clip_f32": clip, "clip_i16": (clip * 20000).astype(np.int16), "fs": np.int64(fs)}
    with tempfile.TemporaryDirectory() as d:
        for kind in ("f32", "i16"):
            path = os.path.join(d, f"clip_{kind}.wav")
            wavfile.write(path, fs, fx[f"clip_{kind}"])
            for nc in (2, 1):
                for lp in (False, True):
                    with contextlib.redirect_stdout(io.StringIO()):
                        ds = ref_utils.MultiWaveformFitting(path, duration=1, num_channels=nc, lp=lp)
                    coords, samples = ds[0]
                    tag = f"{kind}_c{nc}_{'lp' if lp else 'raw'}"
                    fx[f"{tag}_coords"] = coords.numpy()
                    fx[f"{tag}_samples"] = np.asarray(samples)
                    fx[f"{tag}_meta"] = np.array([ds.height, ds.width, ds.sample_rate], np.int64)
    np.savez_compressed(os.path.join(OUT, "multiwave.npz"), **fx)


def checkpoint_fixture(ref_models, ref_utils):
    """A checkpoint in the reference's own format (run.py:357-363): train()'s default
    architecture (num_sine=2, num_snake=2, a_initial=0.5; H = 128 to keep the file small,
    omega0 = 1000, seed 2) after 3 Adam steps of the run.py loop on gt_bach 1 s, saved with
    torch.save({'model_state_dict', 'optimizer_state_dict'}) -- the file a prev_ckpt_path
    resume (run.py:84-106) loads.  Also the loss of the NEXT step at the saved weights."""
    wav = os.path.join(REF, "gt_bach.wav")
    coords, target = ref_utils.WaveformFitting(wav, duration=1, decimation=1)[0]
    torch.manual_seed(2)
    m = ref_models.SirenWithSnakeTanh(in_features=1, out_features=1, hidden_features=128, num_sine=2,
                                      num_snake=2, num_tanh=0, first_omega_0=1000.0, a_initial=0.5)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    mse = torch.nn.MSELoss()
    x, y = coords.reshape(1, -1, 1), target.reshape(1, -1, 1)
    for _ in range(3):
        loss = mse(m(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
    torch.save({"model_state_dict": m.state_dict(), "optimizer_state_dict": opt.state_dict()},
               os.path.join(OUT, "ckpt_ref_default_h128.pt"))
    with torch.no_grad():
        nxt = float(mse(m(x), y))
    json.dump({"next_loss": nxt, "steps": 3, "hidden": 128, "omega0": 1000.0, "seed": 2,
               "keys": list(m.state_dict().keys()),
               "shapes": [list(v.shape) for v in m.state_dict().values()]},
              open(os.path.join(OUT, "ckpt_ref_default_h128.json"), "w"), indent=1)


def fullsize_seed_trajectories(ref_models, ref_utils, seeds, steps, patience, omega0=3000.0, lr=1e-3,
                               fname="trajectory_5x1024_w3000_seeds.json", duration=1, factor=0.8, min_lr=1e-6):
    """The headline model (SIREN 5x1024, BASELINE cfg2's shape) fitted full batch on gt_bach
    (`duration` s: 1, or 6 = 264 600 coordinates, the longest whole-second clip gt_bach holds
    and the closest to cfg2's 10 s) over several init seeds -- the 0.1 dB fit-parity fixture at
    the model size the north_star quotes.  The plateau patience can be lowered (run.py:117 uses
    200) so that the CPU-affordable step count contains ReduceLROnPlateau drops; the GPU test
    uses the same patience.  Written after every seed (6 s: ~13 s per step on 8 CPU threads)."""
    wav = os.path.join(REF, "gt_bach.wav")
    coords, target = ref_utils.WaveformFitting(wav, duration=duration, decimation=1)[0]
    tgt = target.numpy().reshape(-1)
    path = os.path.join(OUT, fname)
    out = {"steps": steps, "omega0": omega0, "hidden": 1024, "num_sine": 4, "patience": patience,
           "factor": factor, "lr0": lr, "min_lr": min_lr, "duration": duration, "runs": {}}
    if os.path.exists(path):
        prev = json.load(open(path))
        if all(prev.get(k, {"duration": 1, "factor": 0.8, "min_lr": 1e-6}.get(k)) == out[k]
               for k in ("steps", "omega0", "patience", "lr0", "duration", "factor", "min_lr")):
            out["runs"] = prev["runs"]
            out.update({k: v for k, v in prev.items() if k not in out})  # e.g. fp32_gpu (tools/fit6_probe.py)
    for s in seeds:
        if str(s) in out["runs"]:
            continue
        m = siren(ref_models, 1024, 4, omega0, seed=s)
        losses, lrs, final = restated_loop(m, coords, target, steps, lr=lr, patience=patience, min_lr=min_lr,
                                           factor=factor)
        out["runs"][str(s)] = {"loss": losses.tolist(), "lr": lrs.tolist(),
                               "snr_target": float(ref_utils.calculate_snr(tgt, final))}
        print(f"5x1024 seed {s}: final {losses[-1]:.3e} min {losses.min():.3e} lr_end {lrs[-1]:.3e} "
              f"snr {out['runs'][str(s)]['snr_target']:.2f}", flush=True)
        json.dump(out, open(path, "w"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trajectory-steps", type=int, default=300)
    ap.add_argument("--fullsize-seeds", default="", help="write only the 5x1024 multi-seed trajectories")
    ap.add_argument("--patience", type=int, default=200)
    ap.add_argument("--lr", type=float, default=1e-3, help="--fullsize-seeds: Adam lr")
    ap.add_argument("--fullsize-file", default="trajectory_5x1024_w3000_seeds.json")
    ap.add_argument("--duration", type=int, default=1, help="--fullsize-seeds: seconds of gt_bach")
    ap.add_argument("--omega0", type=float, default=3000.0, help="--fullsize-seeds: first-layer omega_0")
    ap.add_argument("--factor", type=float, default=0.8, help="--fullsize-seeds: ReduceLROnPlateau factor")
    ap.add_argument("--min-lr", type=float, default=1e-6, help="--fullsize-seeds: ReduceLROnPlateau min_lr")
    ap.add_argument("--clip", type=int, default=0, help="write only gt_bach_<clip>s.npz: the WaveformFitting "
                    "target of the first <clip> seconds (the data of the --duration fixtures)")
    ap.add_argument("--seeds", default="0,1,2,3,4", help="init seeds of the multi-seed trajectories")
    ap.add_argument("--only-seeds", action="store_true", help="write only the multi-seed file")
    ap.add_argument("--only-act", action="store_true", help="write only the Snake / Tanh fixtures")
    ap.add_argument("--snake-seeds", default="", help="write only the Snake multi-seed trajectories")
    ap.add_argument("--only-mdct", action="store_true", help="write only the MDCT fixtures")
    ap.add_argument("--only-kan", action="store_true", help="write only the KAN fixtures")
    ap.add_argument("--only-multiwave", action="store_true",
                    help="write only the MultiWaveformFitting and reference-checkpoint fixtures")
    args = ap.parse_args()
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", 0)) or os.cpu_count() or 1)
    ref_models, ref_utils = import_reference()
    if args.clip:
        _, target = ref_utils.WaveformFitting(os.path.join(REF, "gt_bach.wav"), duration=args.clip, decimation=1)[0]
        np.savez_compressed(os.path.join(OUT, f"gt_bach_{args.clip}s.npz"), target=target.numpy().reshape(-1))
        return
    if args.only_multiwave:
        multiwave_fixtures(ref_utils)
        checkpoint_fixture(ref_models, ref_utils)
        return
    if args.only_act:
        act_fixtures(ref_models, ref_utils, args.trajectory_steps)
        return
    if args.only_kan:
        kan_fixtures(ref_utils, args.trajectory_steps)
        return
    if args.only_mdct:
        mdct_fixtures(ref_models, args.trajectory_steps)
        return
    if args.snake_seeds:
        snake_seed_trajectories(ref_models, ref_utils, [int(s) for s in args.snake_seeds.split(",")],
                                args.trajectory_steps)
        return
    if args.fullsize_seeds:
        fullsize_seed_trajectories(ref_models, ref_utils, [int(s) for s in args.fullsize_seeds.split(",")],
                                   args.trajectory_steps, args.patience, lr=args.lr, fname=args.fullsize_file,
                                   duration=args.duration, omega0=args.omega0, factor=args.factor,
                                   min_lr=args.min_lr)
        return
    if args.only_seeds:
        seed_trajectories(ref_models, ref_utils, [int(s) for s in args.seeds.split(",")],
                          args.trajectory_steps)
        return
    from scipy.signal import decimate

    meta = {"generator": "tests/golden/make_golden.py", "torch": torch.__version__,
            "numpy": np.__version__}

    # --- coordinate grid: utils.py:99-109
    lin = {f"n{n}": ref_utils.get_coord(n, 1).numpy().reshape(-1) for n in (7, 100, 4097)}
    np.savez_compressed(os.path.join(OUT, "get_coord.npz"), **lin)

    # --- waveform target: utils.py:111-149 on gt_bach.wav, 1 s
    wav = os.path.join(REF, "gt_bach.wav")
    ds = ref_utils.WaveformFitting(wav, duration=1, decimation=1)
    coords, target = ds[0]
    from scipy.io import wavfile
    fs, raw = wavfile.read(wav)
    raw = raw.astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "gt_bach_1s.npz"), raw=raw[:2 * fs], fs=np.int64(fs),
                        target=target.numpy().reshape(-1), coords=coords.numpy().reshape(-1))
    ds2 = ref_utils.WaveformFitting(wav, duration=2, decimation=2)
    _, target_d2 = ds2[0]
    np.savez_compressed(os.path.join(OUT, "gt_bach_2s_dec2.npz"), target=target_d2.numpy().reshape(-1),
                        sample_rate=np.int64(ds2.sample_rate))

    # --- init: models.py:94-112, 306-386 under torch.manual_seed(0)
    m3 = siren(ref_models, 256, 2, 1000.0)
    np.savez_compressed(os.path.join(OUT, "init_3x256_seed0.npz"), **sd_np(m3))
    m5 = siren(ref_models, 1024, 4, 3000.0)
    json.dump(summary(sd_np(m5)), open(os.path.join(OUT, "init_5x1024_seed0_summary.json"), "w"), indent=1)
    m_st = siren(ref_models, 512, 4, 3000.0, in_dim=2, seed=3)
    json.dump(summary(sd_np(m_st)), open(os.path.join(OUT, "init_5x512_in2_seed3_summary.json"), "w"),
              indent=1)

    # --- one forward/backward (models.py:388-394, run.py:168,185) on a 2100-point subset
    idx = np.arange(0, 44100, 21)
    c_sub, t_sub = coords[idx], target[idx]
    fb = {}
    for w0 in (1000.0, 22000.0):
        m = siren(ref_models, 256, 2, w0)
        out, loss, grads = fwd_bwd(m, c_sub, t_sub)
        acts = m.forward_with_activations(c_sub.reshape(1, -1, 1))
        # SineLayer entries alternate (omega*linear, sin(.)) -- models.py:404-421
        sine = [v.detach().numpy().reshape(-1, v.shape[-1])[:16] for k, v in acts.items()
                if "SineLayer" in k]
        tag = f"w{int(w0)}"
        fb[f"{tag}_out"] = out
        fb[f"{tag}_loss"] = np.array([loss])
        for k, g in grads.items():
            fb[f"{tag}_grad_{k}"] = g
        for j in range(len(sine) // 2):
            fb[f"{tag}_preact{j}"] = sine[2 * j]
            fb[f"{tag}_sin{j}"] = sine[2 * j + 1]
        if w0 == 1000.0:
            opt = torch.optim.Adam(m.parameters(), lr=1e-3)
            opt.step()
            for k, p in m.named_parameters():
                fb[f"{tag}_adam1_{k}"] = p.detach().numpy().copy()
    fb["subset_idx"] = idx
    np.savez_compressed(os.path.join(OUT, "fwd_bwd_3x256.npz"), **fb)

    # --- ReduceLROnPlateau trace (run.py:117,187)
    rng = np.random.default_rng(0)
    seq = np.concatenate([np.linspace(1.0, 0.5, 300), 0.5 + 0.01 * rng.random(1200)])
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=1e-3)
    sch = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.8, patience=200, min_lr=2e-4)
    lrs = []
    for v in seq:
        sch.step(float(np.float32(v)))
        lrs.append(sch.get_last_lr()[0])
    json.dump({"loss": [float(np.float32(v)) for v in seq], "lr": lrs, "patience": 200, "factor": 0.8,
               "min_lr": 2e-4, "lr0": 1e-3}, open(os.path.join(OUT, "plateau_trace.json"), "w"))

    # --- SNR metrics: utils.py:77-97, run.py:302-335 quirks
    tgt = target.numpy().reshape(-1)
    snr = {
        "perfect_fit_reported_1s": float(ref_utils.calculate_snr(decimate(raw[:fs], q=1) + 1e-10, tgt)),
        "lowpass_only_1s": float(ref_utils.calculate_snr(decimate(raw[:fs], q=1) + 1e-10, raw[:fs])),
        "target_vs_half": float(ref_utils.calculate_snr(tgt, 0.5 * tgt)),
        "target_vs_noisy": float(ref_utils.calculate_snr(tgt, tgt + 0.01 * np.sin(np.arange(fs)))),
    }
    json.dump(snr, open(os.path.join(OUT, "snr_cases.json"), "w"), indent=1)

    # --- full-batch trajectory: run.py:156-190, SIREN 3x256, omega0 = 1000, gt_bach 1 s
    if args.trajectory_steps > 0:
        m = siren(ref_models, 256, 2, 1000.0)
        losses, lrs, final = restated_loop(m, coords, target, args.trajectory_steps)
        json.dump({"steps": args.trajectory_steps, "omega0": 1000.0, "hidden": 256, "num_sine": 2,
                   "seed": 0, "loss": losses.tolist(), "lr": lrs.tolist(),
                   "snr_target": float(ref_utils.calculate_snr(tgt, final)),
                   "snr_reported": float(ref_utils.calculate_snr(decimate(raw[:fs], q=1) + 1e-10, final))},
                  open(os.path.join(OUT, "trajectory_3x256_w1000.json"), "w"))
        np.savez_compressed(os.path.join(OUT, "trajectory_3x256_w1000_final.npz"), out=final.astype(np.float32))
        seed_trajectories(ref_models, ref_utils, [int(s) for s in args.seeds.split(",")],
                          args.trajectory_steps)
    act_fixtures(ref_models, ref_utils, args.trajectory_steps)
    mdct_fixtures(ref_models, 20)
    kan_fixtures(ref_utils, 30)
    multiwave_fixtures(ref_utils)
    checkpoint_fixture(ref_models, ref_utils)
    json.dump(meta, open(os.path.join(OUT, "meta.json"), "w"), indent=1)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
