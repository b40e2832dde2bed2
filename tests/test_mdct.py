"""MDCT-domain target on the host: the restated STMDCT / ISTMDCT / KBD window and
MDCTFitting against the reference's own outputs (tests/golden/mdct_kat.npz, mdct_fitting_1s.npz,
made by tests/golden/make_golden.py from /root/reference's mdct.py / utils.py)."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")


def load(name):
    return np.load(os.path.join(G, name))


@pytest.mark.parametrize("N", [1024, 2048])
def test_stmdct_istmdct_bit_exact(N):
    from inr_for_audio_amd import mdct
    k = load("mdct_kat.npz")
    c = mdct.STMDCT(k["x"], N=N)
    assert c.shape == k[f"stmdct_{N}"].shape and np.array_equal(c, k[f"stmdct_{N}"])
    r = mdct.ISTMDCT(k[f"stmdct_{N}"], N=N)
    assert np.array_equal(r, k[f"istmdct_{N}"])


@pytest.mark.parametrize("N", [256, 1024, 2048])
def test_mdct_perfect_reconstruction_interior(N):
    """Princen-Bradley: KBD analysis + synthesis with 50 % overlap reconstructs the signal
    except in the first and last half-frame (SURVEY §8c known-answer test)."""
    from inr_for_audio_amd import mdct
    x = np.random.default_rng(1).uniform(-1, 1, 40 * N // 2 + 37)
    y = mdct.ISTMDCT(mdct.STMDCT(x, N=N), N=N)
    h = N // 2
    assert len(y) == (len(x) // h) * h
    assert np.max(np.abs(y[h:len(y) - h] - x[h:len(y) - h])) < 1e-12


def _clip():
    g = load("gt_bach_1s.npz")
    # the reference normalises by max|x| over the WHOLE file, which is 1.0 for gt_bach.wav:
    # one 1.0 sample past the clip reproduces that without shipping the file
    return np.concatenate([g["raw"], np.array([1.0], np.float32)]), int(g["fs"])


@pytest.mark.parametrize("tag", ["lin", "log"])
def test_mdct_fitting_matches_reference(tag):
    from inr_for_audio_amd.utils import MDCTFitting
    f = load("mdct_fitting_1s.npz")
    data, fs = _clip()
    d = MDCTFitting(duration=1, N=2048, takelog=(tag == "log"), data=data, sample_rate=fs)
    mean, scale, shift, h, w = f[f"{tag}_stats"]
    assert (d.height, d.width) == (int(h), int(w)) == (1024, 43)
    assert np.array_equal(d.pixels.reshape(-1), f[f"{tag}_pixels"])
    assert (float(d.mean), float(d.scale), float(d.shift)) == (mean, scale, shift)
    c = d.coords.numpy()
    assert c.shape == (1024 * 43, 2)
    assert np.array_equal(c[:43, 0], np.full(43, -1, np.float32)) and c[43, 0] > -1   # bin-major
    sig = d.to_signal(f[f"{tag}_model_out"], takelog=(tag == "log")).reshape(-1)
    ref = f[f"{tag}_signal"]
    assert sig.shape == ref.shape
    # float32 de-normalisation in numpy vs torch: identical up to the last ulp of the spec
    assert np.max(np.abs(sig - ref)) <= 1e-6 * max(1.0, np.max(np.abs(ref)))
