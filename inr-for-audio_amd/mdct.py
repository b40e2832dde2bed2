"""MDCT-domain target for the SIREN fit: the reference's framed KBD-windowed
MDCT and its overlap-add inverse (mdct.py:16-111, window.py:39-59), restated as batched numpy /
scipy.fft over all frames at once.  Host-side data preparation, run once per fit (ms-scale);
the fit itself is the same fused HIP path with 2-D (bin, frame) coordinates.

Conventions kept from the reference: N-sample frames hopping N/2, one KBD window (alpha 4) on
both sides, the 2/N factor in the forward transform, zero padding up to the next multiple of
N/2 (a whole extra half-frame when the length already is one), frames = len // (N/2), and the
inverse trimmed to frames * N/2 samples.
"""
from __future__ import annotations

import functools

import numpy as np
from scipy.fft import fft, ifft
from scipy.special import i0


@functools.lru_cache(maxsize=8)
def kbd_window(N: int, alpha: float = 4.0) -> np.ndarray:
    """Kaiser-Bessel-derived window of length N (window.py:39-59): the square root of the
    running sum of a Kaiser kernel over its first N/2 points, normalised by the sum over
    N/2 + 1 points, mirrored for the second half."""
    half = N // 2
    j = np.arange(half + 1)
    kernel = i0(np.pi * alpha * np.sqrt(1 - ((2 * j + 1) / (N / 2 + 1) - 1) ** 2)) / i0(np.pi * alpha)
    total = np.sum(kernel)
    rising = np.sqrt(np.cumsum(kernel[:half]) / total)
    w = np.concatenate([rising, rising[::-1]])
    w.setflags(write=False)
    return w


def KBDWindow(x, alpha: float = 4.0) -> np.ndarray:
    """window.py:39 -- x multiplied by the KBD window of its own length."""
    x = np.asarray(x)
    return kbd_window(x.shape[-1], alpha) * x


def _twiddles(N: int):
    half = N // 2
    n0 = (half + 1) / 2
    n = np.arange(N)
    k = np.arange(half)
    return (np.exp(-1j * np.pi * n / N), np.exp(-2j * np.pi * n0 * (k + 0.5) / N),
            np.exp(2j * np.pi * k * n0 / N), np.exp(1j * np.pi * (n + n0) / N))


def MDCT(data, a: int, b: int, isInverse: bool = False) -> np.ndarray:
    """Forward (N = a + b samples -> N/2 coefficients, scaled 2/N) or inverse (N/2 -> N,
    scaled 2) MDCT of the last axis via one FFT (mdct.py:16-40).  Only a = b = N/2 is used."""
    N = a + b
    if a != b:
        raise NotImplementedError("MDCT with a != b (asymmetric windows) is not used by the fit")
    pre_f, post_f, pre_i, post_i = _twiddles(N)
    x = np.asarray(data)
    if isInverse:
        return 2.0 * (ifft(x * pre_i, N, axis=-1) * N * post_i).real
    return (2.0 / N) * (fft(x * pre_f, axis=-1)[..., : N // 2] * post_f).real


def IMDCT(data, a: int, b: int) -> np.ndarray:
    return MDCT(data, a, b, True)


def _frames(padded: np.ndarray, N: int, n_frames: int) -> np.ndarray:
    half = N // 2
    idx = np.arange(n_frames)[:, None] * half + np.arange(N)[None, :]
    return padded[idx]


def STMDCT(data, N: int = 1024) -> np.ndarray:
    """Framed MDCT of a 1-D signal (mdct.py:48-70) -> [N/2 bins][frames] float64."""
    x = np.asarray(data)
    half = N // 2
    n_frames = len(x) // half
    padded = np.pad(x, (0, half - len(x) % half), "constant", constant_values=(0, 0))
    frames = KBDWindow(_frames(padded, N, n_frames))
    return np.ascontiguousarray(MDCT(frames, half, half).T)


def ISTMDCT(mdct_coefficients, N: int = 1024) -> np.ndarray:
    """Overlap-add inverse of STMDCT (mdct.py:72-111) -> frames * N/2 samples float64."""
    c = np.asarray(mdct_coefficients)
    half = N // 2
    n_frames = c.shape[1]
    blocks = KBDWindow(IMDCT(c.T, half, half))          # [frames][N]
    # output half-block j = second half of frame j-1 + first half of frame j (each sum of
    # two terms is order-independent, so this equals the reference's frame-by-frame add)
    seg = np.zeros((n_frames + 1, half))
    seg[:n_frames] += blocks[:, :half]
    seg[1:] += blocks[:, half:]
    return seg.reshape(-1)[: half * n_frames]
