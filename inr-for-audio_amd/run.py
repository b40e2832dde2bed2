"""``train()`` with the reference's keyword API (run.py:30-400) on the HIP engine.

Differences from the reference are limited to what the hot-path scope excludes: no plots
(matplotlib figures), no loss-landscape, no STFT / auraloss-SNR loss terms (alpha must be 0 --
at alpha=0 the reference's STFT term contributes exactly zero; loss_mode 'mse'
and 'mae' (L1Loss, run.py:161-163) are fused on device, 'snr' needs auraloss), no
random-Fourier-feature encoding.  ``multichannel=True`` (keyword-only) fits the (time,
channel) grid of MultiWaveformFitting (utils.py:186-231; the reference's call site,
run.py:59-63, is commented out, with mode == 'lp' selecting its FIR decimation) -- BASELINE
cfg3's data path; its output.wav is written as a (samples, channels) file.  arch='kan' fits KAN([1, H, H, 1]) (SURVEY §8 f4,
kan.py) on its own fp32 HIP kernels.  method='mdct' fits the
MDCT-domain target (utils.MDCTFitting, N = 2048, mode='log' = takelog) with
(bin, frame) coordinates and inverts it as run.py:258-290 does.  Everything the path
produces -- output.wav, the checkpoint dict, parameters.json with the run.py-formula SNR --
keeps the reference's names and formats.  One deliberate deviation: for method='mdct' the
reference's final SNR line (run.py:335) raises a numpy broadcast error whenever
fs * duration is not a multiple of N/2 (the recovered signal has frames * N/2 samples);
here the SNR is taken over the common length instead.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import scipy.io.wavfile as wavfile
import torch

from .engine import KanEngine, SirenEngine
from .kan import KAN
from .models import SirenWithSnakeTanh
from .utils import (MDCTFitting, MultiWaveformFitting, WaveformFitting, calculate_snr, get_coord,
                    load_mono_like_librosa, reported_snr)


def save_parameters(experiment_folder, **kwargs):
    """run.py:25-28."""
    with open(f"{experiment_folder}/parameters.json", "w") as file:
        json.dump(kwargs, file, indent=4)


def _rank0() -> bool:
    d = torch.distributed
    return not (d.is_available() and d.is_initialized()) or d.get_rank() == 0


def _distributed() -> bool:
    d = torch.distributed
    return d.is_available() and d.is_initialized() and d.get_world_size() > 1


def _experiment_folder(experiment_path, inst, method, tag):
    """run.py:34-40 -- append '(2)' to the tag until the folder is new.  Under data
    parallelism rank 0 decides and broadcasts the tag, so every rank returns the same path."""
    if _rank0():
        folder = f"{experiment_path}/{inst}-{method}-{tag}"
        while os.path.exists(folder):
            tag = tag + "(2)"
            folder = f"{experiment_path}/{inst}-{method}-{tag}"
        os.makedirs(folder)
    if _distributed():
        box = [tag]
        torch.distributed.broadcast_object_list(box, src=0)
        tag = box[0]
    return tag, f"{experiment_path}/{inst}-{method}-{tag}"


def train(experiment_path: str, tag: str, inst: str, duration: int, num_channels=1, method='wave',
          arch='mlp', loss_mode='mse', mode=None, decimation=1, bwe=False, num_hidden_features=256,
          num_sine=2, num_snake=2, num_tanh=0, num_freq=None, omega=22000, first_linear=False,
          last_linear=True, hidden_omega=30, a_initial=0.5, total_steps=20000, learning_rate=1e-3,
          min_learning_rate=1e-6, alpha=0.0, prev_ckpt_path=None, visualization=False, *,
          filename=None, data_dir="data", seed=None, micro_batch=1 << 20, use_graph=True,
          device=None, verbose=False, multichannel=False, patience=200):
    """Fit one clip; returns the checkpoint path (run.py:400).  Extra keyword-only knobs:
    ``filename`` (default ``{data_dir}/{inst}.wav`` as run.py:33), ``seed`` (torch.manual_seed
    before model construction), ``micro_batch`` (rows per fused micro-batch), ``use_graph``
    (replay each step as a HIP graph), ``device``, ``multichannel`` (the (t, ch) grid of
    MultiWaveformFitting, run.py:59-63), ``patience`` (ReduceLROnPlateau, run.py:117's 200)."""
    if method not in ("wave", "mdct"):
        raise ValueError("specify the correct fitting method as wave or mdct (run.py:77-78)")
    if method == "mdct" and bwe:
        raise NotImplementedError("bwe is a waveform-mode feature (run.py:127-131)")
    if arch not in ("mlp", "kan"):
        raise NotImplementedError(f"arch={arch!r}: the reference builds 'kan' or the MLP (run.py:92-96)")
    if arch == "kan" and method == "mdct":
        raise NotImplementedError("arch='kan' takes 1-D coordinates (run.py:92 builds KAN([1, H, H, 1]))")
    if loss_mode not in ("mse", "mae") or alpha != 0.0:
        raise NotImplementedError("HIP path implements loss_mode 'mse' / 'mae' with alpha=0 (run.py:161-169)")
    if arch == "kan" and loss_mode != "mse":
        raise NotImplementedError("arch='kan' is fitted with loss_mode='mse'")
    if multichannel and (method != "wave" or arch != "mlp" or bwe):
        raise NotImplementedError("multichannel fits the waveform MLP (run.py:59-63) without bwe")
    if num_freq is not None:
        raise NotImplementedError("random Fourier features (rff) are out of scope")
    if visualization:
        raise NotImplementedError("loss-landscape visualization is out of scope")

    filename = filename or f"{data_dir}/{inst}.wav"
    rank0 = _rank0()
    tag, experiment_folder = _experiment_folder(experiment_path, inst, method, tag)
    decimation = int(decimation)

    takelog = False
    if method == "wave" and multichannel:  # run.py:59-63 (commented out in the reference)
        input_data = MultiWaveformFitting(filename, duration=duration, num_channels=num_channels, lp=mode == "lp")
        model_input, samples = input_data[0]
        ground_truth = torch.from_numpy(np.ascontiguousarray(samples, dtype=np.float32))
        input_dimension = 2
    elif method == "wave":
        input_data = WaveformFitting(filename, duration=duration, decimation=decimation)
        model_input, ground_truth = input_data[0]
        input_dimension = 1
    else:  # run.py:67-76
        N = 2048
        takelog = mode == "log"
        input_data = MDCTFitting(filename, duration=duration, N=N, takelog=takelog)
        model_input, pixels = input_data[0]
        ground_truth = torch.from_numpy(np.ascontiguousarray(pixels))
        input_dimension = 2

    if seed is not None:
        torch.manual_seed(seed)
    if arch == "kan":  # run.py:92-93
        model = KAN([1, num_hidden_features, num_hidden_features, 1])
    else:
        model = SirenWithSnakeTanh(in_features=input_dimension, out_features=1,
                                   hidden_features=num_hidden_features, num_sine=num_sine,
                                   num_snake=num_snake, num_tanh=num_tanh, num_freq=num_freq,
                                   first_linear=first_linear, last_linear=last_linear,
                                   first_omega_0=omega, hidden_omega_0=hidden_omega, a_initial=a_initial)
    ckpt = None
    if prev_ckpt_path is not None:  # run.py:84-106
        ckpt = torch.load(prev_ckpt_path, map_location="cpu", weights_only=True)
        model.load_state_dict(ckpt["model_state_dict"])

    dev = torch.device(device or "cuda")
    Engine = KanEngine if arch == "kan" else SirenEngine
    kw = {} if arch == "kan" else {"loss_mode": loss_mode}
    engine = Engine(model, model_input, ground_truth, lr=learning_rate, min_lr=min_learning_rate,
                    patience=patience, micro_batch=micro_batch, hist_cap=total_steps, device=dev, **kw)
    if ckpt is not None:
        engine.load_adam_state_dict(ckpt["optimizer_state_dict"])

    torch.cuda.synchronize(dev)
    start_time = time.time()
    single = not (torch.distributed.is_available() and torch.distributed.is_initialized())
    if use_graph and single and total_steps > 1:
        engine.step()                    # step 0 eagerly (also warms up the kernels)
        engine.capture_graph()
        for _ in range(total_steps - 1):
            engine.step()
    else:
        for _ in range(total_steps):
            engine.step()
    # steps the fp16 range guard rejected were recomputed by the next call: top up to
    # total_steps applied optimizer steps (one host check, after the loop)
    while engine.steps_applied() < total_steps:
        engine.step()
    torch.cuda.synchronize(dev)
    end_time = time.time()
    total_time = (end_time - start_time) / 60

    raw_losses, raw_lrs = engine.history()
    losses = 10 * np.log10(raw_losses.astype(np.float64) + 1e-10)   # run.py:180
    lrs = 10 * np.log10(raw_lrs)                                     # run.py:190
    best_iter = int(np.argmin(raw_losses)) if len(raw_losses) else -1

    param_size = sum(p.nelement() * p.element_size() for p in model.parameters())
    buffer_size = sum(b.nelement() * b.element_size() for b in model.buffers())
    model_size = (param_size + buffer_size) / 1024

    # inference (run.py:251-256); best_model aliases the final model (run.py:173)
    if bwe:
        coords = get_coord(input_data.original_sample_rate * duration, dim=1)
        recover_sample_rate = input_data.original_sample_rate
    else:
        coords = model_input
        recover_sample_rate = input_data.sample_rate
    model_output = engine.infer(coords.to(dev)).cpu().numpy().astype(np.float32)
    if method == "wave" and multichannel:
        signal_recovered = input_data.to_channels(model_output)      # (samples, channels)
    elif method == "wave":
        signal_recovered = model_output
    else:  # run.py:258-259, 281-290 (double exp in log mode)
        signal_recovered = input_data.to_signal(model_output, takelog=takelog).reshape(-1)

    ckpt_path = f"{experiment_folder}/saved_ckpt.pt"
    if rank0:
        output_filename = f"{experiment_folder}/output.wav"
        wavfile.write(output_filename, recover_sample_rate,
                      signal_recovered if multichannel else signal_recovered.reshape(-1, 1))
        ref, fs_ref = load_mono_like_librosa(filename)
        rec, _ = load_mono_like_librosa(output_filename)
        if method == "mdct":
            m = min(int(fs_ref * duration), len(rec))
            ref, rec = ref[:m], rec[:m]
        # multichannel: librosa.load averages the channels of both files; mode 'lp' halved the rate
        d_snr = (2 if mode == "lp" else 1) if multichannel else decimation
        snr_final = float(reported_snr(ref, fs_ref, rec, duration, d_snr, bwe))
        target = ground_truth.numpy().reshape(-1)
        # the fit in its own (training) domain: waveform or normalised MDCT map
        snr_target = float(calculate_snr(target, model_output)) if not bwe else None

        checkpoint = {"model_state_dict": {k: v.detach().cpu().clone() for k, v in model.state_dict().items()},
                      "optimizer_state_dict": engine.adam_state_dict()}
        torch.save(checkpoint, ckpt_path)

        n_gpus = torch.distributed.get_world_size() if not single else 1
        params = {
            "experiment_path": experiment_path, "tag": tag, "inst": inst, "duration": duration,
            "num_channels": num_channels, "method": method, "arch": arch, "loss_mode": loss_mode,
            "mode": mode, "decimation": decimation, "bwe": bwe,
            "num_hidden_features": num_hidden_features, "num_sine": num_sine,
            "num_snake": num_snake, "num_tanh": num_tanh, "num_freq": num_freq, "omega": omega,
            "hidden_omega": hidden_omega, "a_initial": a_initial, "total_steps": total_steps,
            "learning_rate": learning_rate, "min_learning_rate": min_learning_rate, "alpha": alpha,
            "prev_ckpt_path": prev_ckpt_path, "curr_ckpt_path": ckpt_path,
            "visualization": visualization, "parameter_size(KB)": param_size / 1024,
            "total_model_size(KB)": model_size, "total_trainig_time(min)": total_time,
            "SNR": snr_final,
            # additions of this build
            "SNR_target": snr_target, "best_iter": best_iter,
            "final_loss": float(raw_losses[-1]) if len(raw_losses) else None,
            "coord_samples_per_sec": engine.n_total * total_steps / max(total_time * 60, 1e-9),
            "n_gpus": n_gpus, "fp16_overflow_steps": engine.guard_state()["overflows"],
        }
        save_parameters(experiment_folder, **params)
        if verbose:
            print(json.dumps({"SNR": snr_final, "SNR_target": snr_target, "time_min": total_time}))
    train.last_history = (losses, lrs)
    return ckpt_path
