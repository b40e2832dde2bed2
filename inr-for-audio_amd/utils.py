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


class MultiWaveformFitting:
    """Multi-channel (t, ch) -> amplitude dataset -- utils.py:186-231 (BASELINE cfg3).

    The clip is cast to float32 and trimmed to `duration` seconds and `num_channels` channels
    (the reference indexes ``data[:T, :num_channels]``, so the file must be multi-channel);
    with ``lp`` each channel is FIR-decimated by 2 (zero phase), which leaves float64 samples
    exactly as the reference's ``np.column_stack`` does.  No peak normalisation (the
    reference's ``__getitem__`` has it commented out).  Coordinates are the height-major
    (time, channel) grid: time = linspace(-1, 1, height), channel = linspace(-1, 1, width)
    (all 0 for one channel), flattened row k = (t[k // width], ch[k % width]) -- so the
    channels of one instant are adjacent rows, and ``samples`` is ``data.reshape(-1, 1)``."""

    def __init__(self, filename=None, duration=1, num_channels=2, lp=False, *, data=None, sample_rate=None):
        if data is None:
            self.sample_rate, self.data = wavfile.read(filename)
        else:
            self.sample_rate, self.data = int(sample_rate), np.asarray(data)
        self.data = self.data.astype(np.float32)[: duration * self.sample_rate, :num_channels]
        self.original_sample_rate = self.sample_rate
        if lp:
            q = 2
            chans = [decimate(self.data[:, i], q, ftype="fir", zero_phase=True) for i in range(num_channels)]
            self.data = np.column_stack(chans)
            self.sample_rate = self.sample_rate // q
        self.height, self.width = self.data.shape
        height_norm = torch.linspace(-1, 1, steps=self.height)
        if num_channels == 1:
            width_norm = torch.linspace(0, 0, steps=self.width)
        else:
            width_norm = torch.linspace(-1, 1, steps=self.width)
        h_grid, w_grid = torch.meshgrid(height_norm, width_norm, indexing="ij")
        self.coords = torch.stack((h_grid, w_grid), dim=-1).reshape(self.height * self.width, -1)
        self.samples = self.data.reshape(-1, 1)

    def get_num_samples(self):
        return self.coords.shape[0]

    def __len__(self):
        return 1

    def __getitem__(self, idx):
        return self.coords, self.samples

    def to_channels(self, model_output) -> np.ndarray:
        """Flat model output in the grid's row order -> [height][width] (time, channel)."""
        return np.asarray(model_output, dtype=np.float32).reshape(self.height, self.width)


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


def hpfilter(data, cutoff, fs):
    """5th-order Butterworth high-pass, zero-phase (utils.py:49-52)."""
    from scipy.signal import butter, filtfilt
    b, a = butter(5, cutoff, btype="highpass", fs=fs)
    return filtfilt(b, a, data)


class MDCTFitting:
    """MDCT-domain fitting target -- utils.py:312-414.

    The clip (channel 1 of a multi-channel file, as the reference reads it) is divided by
    max|x| over the WHOLE file, trimmed to `duration` seconds, and transformed by STMDCT
    (N-sample KBD frames hopping N/2) into a [N/2 bins][frames] float32 map; optionally
    shifted positive and log-compressed (takelog); then mean-removed and scaled by its max
    |.|.  Coordinates are the (bin, frame) linspace grid, bin-major: (height*width, 2)."""

    def __init__(self, filename=None, duration=1, N=1024, highpass=False, takelog=False, *,
                 data=None, sample_rate=None):
        from . import mdct
        if data is None:
            self.sample_rate, self.data = wavfile.read(filename)
        else:
            self.sample_rate, self.data = int(sample_rate), np.asarray(data)
        self.original_sample_rate = self.sample_rate
        if len(self.data.shape) > 1:
            self.data = self.data[:, 1]
        if highpass:
            self.data = hpfilter(self.data, 150, self.sample_rate)
        self.data = torch.from_numpy(self.data.astype(np.float32)[:duration * self.sample_rate]
                                     / np.max(np.abs(self.data)))
        self.N = N
        self.mdct = mdct.STMDCT(self.data.numpy(), N=N).astype(np.float32)
        self.shift = 0.0
        if takelog:
            self.shift = np.abs(np.min(self.mdct)) + 1e-8
            self.mdct = np.log(self.mdct + self.shift)
        self.mean = np.mean(self.mdct)
        self.mdct = self.mdct - self.mean
        self.scale = np.max(np.abs(self.mdct))
        self.mdct = self.mdct / self.scale
        self.height, self.width = self.mdct.shape
        h_grid, w_grid = torch.meshgrid(torch.linspace(-1, 1, steps=self.height),
                                        torch.linspace(-1, 1, steps=self.width), indexing="ij")
        self.coords = torch.stack((h_grid, w_grid), dim=-1).reshape(self.height * self.width, -1)
        self.pixels = self.mdct.reshape(-1, 1)

    def __len__(self):
        return 1

    def __getitem__(self, idx):
        if idx > 0:
            raise IndexError
        return self.coords, self.pixels

    def to_signal(self, model_output, takelog=False):
        """run.py:258-259 + 281-290: normalised model output [height*width] -> waveform.
        With takelog the reference exponentiates TWICE -- once on the raw output, once after
        de-normalisation -- and so does this (drop-in fidelity)."""
        from . import mdct
        out = np.asarray(model_output, dtype=np.float32).reshape(-1)
        if takelog:
            out = np.exp(out)
        spec = out.reshape(self.height, self.width) * self.scale + self.mean - self.shift
        if takelog:
            spec = np.exp(spec)
        return mdct.ISTMDCT(spec, N=self.N).reshape(-1, 1).astype(np.float32)
