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


def _torch_kanlinear(x, lay):
    """kan.py:153-166 restated in plain torch fp64 (differentiable): SiLU base + B-spline term."""
    from inr_for_audio_amd.kan import bspline_bases
    xd = x.double()
    base = torch.nn.functional.silu(xd) @ lay["base_weight"].t()
    bases = bspline_bases(xd, lay["grid"], 3)
    sw = lay["spline_weight"] * lay["spline_scaler"].unsqueeze(-1)
    return base + bases.reshape(xd.shape[0], -1) @ sw.reshape(sw.shape[0], -1).t()


def test_kan_autograd_vs_oracle(dev):
    """KAN(...)(x) + loss.backward() (kan.py:268-273 in a user loop) through _KanFunction: the
    parameter gradients equal the oracle's fp64 autograd of the same MSE (1e-4 relative L2)."""
    m = _kan([1, 32, 48, 1])
    sd = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
    t, y = _data(2100)
    m = m.to(dev)
    out = m(torch.from_numpy(t).to(dev).reshape(1, -1, 1))
    loss = torch.nn.MSELoss()(out, torch.from_numpy(y).to(dev).reshape(1, -1, 1))
    loss.backward()
    ref_out, xs = orc.kan_forward(sd, t, 3)
    ref = orc.kan_backward(sd, xs, orc.mse_grad(ref_out, y), 3)
    assert abs(float(loss) - orc.mse(ref_out, y)) < 1e-5 * orc.mse(ref_out, y)
    for k, p in m.named_parameters():
        r = ref[k]
        rel = np.linalg.norm(p.grad.cpu().numpy().reshape(r.shape) - r) / np.linalg.norm(r)
        assert rel < 1e-4, (k, rel)


def test_kan_autograd_guards(dev):
    """_KanFunction keeps its inputs under torch's version counter (an in-place parameter change
    between forward and backward raises instead of giving silently wrong gradients), and a second
    backward through a retained graph raises a clear RuntimeError."""
    m = _kan([1, 16, 16, 1]).to(dev)
    t, y = _data(600)
    x = torch.from_numpy(t).to(dev).reshape(1, -1, 1)
    yt = torch.from_numpy(y).to(dev).reshape(1, -1, 1)
    loss = torch.nn.MSELoss()(m(x), yt)
    with torch.no_grad():
        m.layers[0].base_weight.add_(1.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        loss.backward()
    m.zero_grad()
    loss = torch.nn.MSELoss()(m(x), yt)
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="run the forward again"):
        loss.backward()


def test_kan_torch_optim_loop_matches_engine(dev):
    """A hand-written torch.optim.Adam loop on the differentiable KAN follows the fused KanEngine
    fit (same gradients, torch's Adam vs the device Adam kernel) and the oracle's Adam on the
    oracle's fp64 gradients, over 6 steps."""
    from inr_for_audio_amd.engine import KanEngine
    widths, steps, lr = [1, 32, 32, 1], 6, 1e-3
    t, y = _data(2100)
    m = _kan(widths).to(dev)
    sd0 = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    opt = torch.optim.Adam(m.parameters(), lr=lr)
    x = torch.from_numpy(t).to(dev).reshape(1, -1, 1)
    yt = torch.from_numpy(y).to(dev).reshape(1, -1, 1)
    for _ in range(steps):
        loss = torch.nn.MSELoss()(m(x), yt)
        opt.zero_grad()
        loss.backward()
        opt.step()
    eng = KanEngine(_kan(widths), torch.from_numpy(t), torch.from_numpy(y), lr=lr, device=dev)
    for _ in range(steps):
        eng.step()
    got = {k: p.detach().cpu().numpy() for k, p in m.named_parameters()}
    for i, k in enumerate(eng.layout.names):
        e = eng.layout.view(eng.params, i).cpu().numpy()
        d = np.linalg.norm(got[k] - e) / np.linalg.norm(e - sd0[k])
        assert d < 1e-3, (k, d)  # relative to the distance the 6 steps moved the parameter
    # oracle: its own gradients and Adam
    sd = {k: v.astype(np.float64) for k, v in sd0.items()}
    mom = {k: np.zeros_like(v) for k, v in sd.items() if not k.endswith("grid")}
    vel = {k: np.zeros_like(v) for k, v in mom.items()}
    for s in range(1, steps + 1):
        o, xs = orc.kan_forward(sd, t, 3)
        g = orc.kan_backward(sd, xs, orc.mse_grad(o, y), 3)
        for k in mom:
            sd[k], mom[k], vel[k] = orc.adam_step(sd[k], g[k], mom[k], vel[k], s, lr)
    for k in mom:
        d = np.linalg.norm(got[k] - sd[k]) / np.linalg.norm(sd[k] - sd0[k])
        assert d < 1e-2, (k, d)


@pytest.mark.parametrize("fin,fout", [(1, 16), (3, 5), (24, 70)])
def test_kanlinear_alone_forward_backward(dev, fin, fout):
    """A lone KANLinear (kan.py:153-166) is a module on the HIP path: output, parameter gradients
    and the input gradient vs plain torch fp64 autograd of the same formula (70 outputs takes the
    two-pass dW + dX kernels, <= 64 the one-pass kernel)."""
    from inr_for_audio_amd.kan import KANLinear
    torch.manual_seed(4)
    lay = KANLinear(fin, fout)
    ref_p = {k: v.detach().clone().double().requires_grad_(k != "grid") for k, v in lay.state_dict().items()}
    x = torch.rand(3000, fin) * 2.4 - 1.2
    xr = x.clone().double().requires_grad_(True)
    out_ref = _torch_kanlinear(xr, ref_p)
    w = torch.randn(3000, fout, dtype=torch.float64)
    (out_ref * w).sum().backward()
    lay = lay.to(dev)
    xg = x.to(dev).requires_grad_(True)
    out = lay(xg)
    assert out.shape == (3000, fout)
    assert float((out.double().cpu() - out_ref.detach()).abs().max()) < 1e-5 * max(1.0, float(out_ref.abs().max()))
    (out * w.float().to(dev)).sum().backward()
    for k, p in lay.named_parameters():
        r = ref_p[k].grad
        rel = float((p.grad.double().cpu() - r).norm() / r.norm())
        assert rel < 1e-4, (k, rel)
    rel = float((xg.grad.double().cpu() - xr.grad).norm() / xr.grad.norm())
    assert rel < 1e-4, rel
