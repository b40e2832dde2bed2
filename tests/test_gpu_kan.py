"""KAN variant (kan.py, run.py:92-93) on the HIP path against the CPU oracle
(tests/test_kan_host.py pins the oracle on the reference's own numbers).  fp32 throughout,
like the reference, so tolerances are fp32-summation-order tight (1e-4 relative L2)."""
import json
import os

import numpy as np
import pytest
import torch
from scipy.io import wavfile

from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _data(n_sub=None):
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    t, y = g["coords"].reshape(-1, 1), g["target"]
    if n_sub:
        idx = np.arange(0, 44100, 44100 // n_sub)[:n_sub]
        t, y = t[idx], y[idx]
    return t, y


def _kan(widths, seed=0):
    from inr_for_audio_amd.kan import KAN
    torch.manual_seed(seed)
    return KAN(widths)


@pytest.mark.parametrize("widths,n,mb,splits", [
    ([1, 64, 64, 1], 2100, 1 << 20, 16), ([1, 64, 64, 1], 2100, 1000, 1), ([1, 32, 64, 1], 44100, 1 << 20, 64),
    ([1, 30, 20, 1], 3000, 1 << 20, 3), ([1, 128, 128, 1], 1024, 1 << 20, 7)])
def test_kan_step_vs_oracle(dev, widths, n, mb, splits):
    from inr_for_audio_amd.engine import KanEngine
    m = _kan(widths)
    sd = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
    t, y = _data(n)
    eng = KanEngine(m, torch.from_numpy(t), torch.from_numpy(y), micro_batch=mb, splits=splits, device=dev)
    eng.step()
    torch.cuda.synchronize()
    L = len(widths) - 1
    out, xs = orc.kan_forward(sd, t, L)
    ref = orc.kan_backward(sd, xs, orc.mse_grad(out, y), L)
    got = {k: v.detach().cpu().numpy() for k, v in zip(eng.layout.names, eng.grad_views())}
    assert set(ref) == set(got)
    for k, r in ref.items():
        rel = np.linalg.norm(got[k].reshape(r.shape) - r) / np.linalg.norm(r)
        assert rel < 1e-4, (k, rel)
    assert abs(eng.last_loss() - orc.mse(out, y)) < 1e-5 * orc.mse(out, y)
    # Adam on the device gradients: bit-exact with the oracle Adam
    for i, k in enumerate(eng.layout.names):
        p1, _, _ = orc.adam_step(sd[k].astype(np.float32), got[k], np.zeros_like(sd[k]), np.zeros_like(sd[k]), 1, 1e-3)
        assert np.array_equal(eng.layout.view(eng.params, i).cpu().numpy(), p1), k


def test_kan_inference_vs_oracle(dev):
    m = _kan([1, 64, 64, 1]).to(dev)
    sd = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    t, _ = _data(5000)
    with torch.no_grad():
        out = m(torch.from_numpy(t).to(dev).reshape(1, -1, 1)).cpu().numpy().reshape(-1)
    ref, _ = orc.kan_forward(sd, t, 3)
    assert np.max(np.abs(out - ref)) < 1e-5 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("width", [1, 3])
def test_kan_forward_bases_bit_exact(dev, width):
    """The forward kernels' B-spline bases are bit-identical to the torch recursion of kan.py:94-104
    (inr_for_audio_amd.kan.bspline_bases, pinned to the reference by tests/test_kan_host.py):
    KAN([width, 1]) with base_weight 0, spline_scaler 1 and a one-hot spline_weight outputs exactly
    B_c(x_i) -- every other term the head kernel adds is an exact zero.  Inputs: uniform draws over
    the grid and past it, every knot, and the floats one ulp either side of each knot."""
    from inr_for_audio_amd.kan import KAN, bspline_bases
    torch.manual_seed(0)
    m = KAN([width, 1])
    lay = m.layers[0]
    grid = lay.grid.detach().clone()
    kn = grid[0].numpy()
    rng = np.random.default_rng(1)
    x1 = np.concatenate([rng.uniform(-2.6, 2.6, 30000), kn, np.nextafter(kn, np.float32(10)),
                         np.nextafter(kn, np.float32(-10)), [0.0, -0.0, 1e-30, -1e-30]]).astype(np.float32)
    x = np.stack([np.roll(x1, 7 * i) for i in range(width)], 1)
    ref = bspline_bases(torch.from_numpy(x), grid, 3).numpy()      # (n, width, 8)
    m = m.to(dev)
    with torch.no_grad():
        lay.base_weight.zero_()
        lay.spline_scaler.fill_(1.0)
    xd = torch.from_numpy(x).to(dev).reshape(1, -1, width)
    for i in range(width):
        for c in range(8):
            with torch.no_grad():
                lay.spline_weight.zero_()
                lay.spline_weight[0, i, c] = 1.0
                out = m(xd).cpu().numpy().reshape(-1)
            bad = np.flatnonzero(out != ref[:, i, c])
            assert bad.size == 0, (i, c, bad[:5], x[bad[:5], i], out[bad[:5]], ref[bad[:5], i, c])


def test_kan_fit_tracks_reference(dev):
    """30 full-batch steps of KAN([1, 64, 64, 1]) on gt_bach 1 s vs the reference's own loop
    (tests/golden/trajectory_kan_64.json): fp32 on both sides, losses within 1e-3 relative."""
    from inr_for_audio_amd.engine import KanEngine
    tr = json.load(open(os.path.join(G, "trajectory_kan_64.json")))
    t, y = _data()
    eng = KanEngine(_kan(tr["widths"], tr["seed"]), torch.from_numpy(t), torch.from_numpy(y), device=dev)
    for _ in range(tr["steps"]):
        eng.step()
    losses, lrs = eng.history()
    ref = np.array(tr["loss"])
    assert np.max(np.abs(losses - ref) / ref) < 1e-3, (losses[:5], ref[:5])
    assert np.array_equal(lrs, np.array(tr["lr"]))


def test_train_kan_end_to_end(dev, tmp_path):
    from inr_for_audio_amd.run import train
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    wav = tmp_path / "clip.wav"
    wavfile.write(wav, int(g["fs"]), g["raw"])
    ckpt = train(str(tmp_path), "k", "clip", 1, arch="kan", num_hidden_features=64, total_steps=25,
                 filename=str(wav), seed=0)
    folder = os.path.dirname(ckpt)
    sr, out = wavfile.read(os.path.join(folder, "output.wav"))
    assert out.shape[0] == 44100 and np.all(np.isfinite(out))
    params = json.load(open(os.path.join(folder, "parameters.json")))
    assert params["arch"] == "kan" and np.isfinite(params["SNR"]) and np.isfinite(params["SNR_target"])
    sd = torch.load(ckpt, weights_only=True)["model_state_dict"]
    assert "layers.1.spline_scaler" in sd and "layers.0.grid" in sd
