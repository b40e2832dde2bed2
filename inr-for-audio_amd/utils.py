"""Host-side data preparation and metrics of the reference's waveform path.

Coordinates, targets and the SNR metric are computed once per run on the host, exactly as
the reference does (utils.py:77-149, run.py:300-335); none of this is in the hot loop.
"""
from __future__ import annotations

import numpy as np
import scipy.io.wavfile as wavfile
import torch
from scipy.signal import decimate


def calculate_snr(original_signal, noisy_signal):
    """SNR in dB = 10 log10(mean(ref^2) / mean((rec-ref)^2))  -- utils.py:77-97."""
    original_signal = np.asarray(original_signal)
    noisy_signal = np.asarray(noisy_signal)
    noise = noisy_signal - original_signal
    signal_power = np.mean(original_signal ** 2)
    noise_power = np.mean(noise ** 2)
    return 10 * np.log10(signal_power / noise_power)


def get_coord(sidelen, dim=2, scale=1):
    """Flattened [-scale, scale]^dim grid from torch.linspace  -- utils.py:99-109."""
    tensors = tuple(dim * [torch.linspace(-1 * scale, 1 * scale, steps=sidelen)])
    coord = torch.stack(torch.meshgrid(*tensors, indexing="ij"), dim=-1)
    return coord.reshape(-1, dim)


def read_wav_channel0(filename):
    """wavfile.read + first channel, as WaveformFitting does (utils.py:113-115)."""
    sample_rate, data = wavfile.read(filename)
    if len(data.shape) > 1:
        data = data[:, 0]
    return sample_rate, data


class WaveformFitting:
    """Waveform dataset -- utils.py:111-149.  ``coord`` = linspace(-1,1,N) (N,1);
    ``amplitude()`` = segment / max|segment| (the DataLoader item, utils.py:144-149)."""

    def __init__(self, filename=None, duration=1, decimation=1, *, data=None, sample_rate=None):
        if data is None:
            self.sample_rate, self.data = read_wav_channel0(filename)
        else:
            self.sample_rate, self.data = int(sample_rate), np.asarray(data)
            if self.data.ndim > 1:
                self.data = self.data[:, 0]
        self.data = self.data.astype(np.float32)[0: duration * self.sample_rate]
        self.original_sample_rate = self.sample_rate
        if decimation > 1:
            q = int(decimation)
            self.data = decimate(self.data, q=q)
            self.sample_rate = self.sample_rate // q
        self.height = len(self.data)
        self.width = 1
        self.coord = get_coord(len(self.data), 1)

    def get_num_samples(self):
        return self.coord.shape[0]

    def __len__(self):
        return 1

    def amplitude(self) -> torch.Tensor:
        amplitude = self.data
        scale = np.max(np.abs(amplitude))
        amplitude = amplitude / scale
        return torch.Tensor(amplitude).view(-1, 1)

    def __getitem__(self, idx):
        return self.coord, self.amplitude()


def load_mono_like_librosa(filename):
    """librosa.load(filename, sr=None) for WAV: float32, integer PCM scaled to [-1,1),
    multi-channel averaged to mono (run.py:302-303)."""
    sr, data = wavfile.read(filename)
    if np.issubdtype(data.dtype, np.integer):
        data = data.astype(np.float32) / float(np.iinfo(data.dtype).max + 1)
    data = data.astype(np.float32)
    if data.ndim > 1:
        data = np.mean(data, axis=1).astype(np.float32)
    return data, sr


def reported_snr(ref_raw, fs_ref, rec, duration, decimation=1, bwe=False):
    """The SNR value run.py writes to parameters.json (run.py:302-335), quirks included:
    the reference is NOT peak-normalised like the training target, and decimate(q=1) still
    applies its 8th-order Chebyshev-I low-pass (0.8 * Nyquist)."""
    ref = np.asarray(ref_raw)[:int(fs_ref * duration)]
    d = 1 if bwe else int(decimation)
    ref = decimate(ref, q=d)
    ref = ref + 1e-10
    return calculate_snr(ref, rec)
