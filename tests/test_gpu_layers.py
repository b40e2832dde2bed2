"""The module API outside the fused step, on the unfused fp32 HIP layer kernels (layer_fp32.hip):
a lone SineLayer (models.py:114-120), Snake (models.py:235-241) and
SirenWithSnakeTanh.forward_with_activations (models.py:396-423) -- against the reference's own
forward_with_activations values (tests/golden/fwd_bwd_3x256.npz) and against plain fp32 PyTorch
of the same ops (forward and autograd)."""
import os

import numpy as np
import pytest
import torch

from errlog import log, rel

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_forward_with_activations_matches_reference(dev):
    from inr_for_audio_amd.models import SineLayer, SirenWithSnakeTanh
    fb = np.load(os.path.join(G, "fwd_bwd_3x256.npz"))
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    t = torch.from_numpy(g["coords"][fb["subset_idx"]]).reshape(1, -1, 1).to(dev)
    torch.manual_seed(0)
    m = SirenWithSnakeTanh(1, 1, 256, 2, 0, 0, first_omega_0=1000.0, hidden_omega_0=30.0).to(dev)
    acts = m.forward_with_activations(t, retain_grad=True)
    sine = [v for k, v in acts.items() if "SineLayer" in k]
    assert len(sine) == 6 and list(acts)[0] == "input"
    errs = {}
    for j in range(3):
        pre = sine[2 * j].detach().reshape(-1, 256)[:16].cpu().numpy()
        y = sine[2 * j + 1].detach().reshape(-1, 256)[:16].cpu().numpy()
        errs[f"preact{j}"] = rel(pre, fb[f"w1000_preact{j}"])
        errs[f"sin{j}"] = float(np.max(np.abs(y - fb[f"w1000_sin{j}"])))
    log("forward_with_activations", **errs)
    # layer 0 agrees to fp32 rounding; the hidden layers inherit sin(|.| ~ 1e3 rad) of layer 0
    # through 256-term sums (the reference's CPU addmm fuses t*w + b for K = 1, this GEMM rounds twice)
    assert errs["preact0"] < 1e-6 and errs["preact1"] < 1e-4 and errs["preact2"] < 1e-4, errs
    assert all(errs[f"sin{j}"] < 2e-3 for j in range(3)), errs   # sin of |.| <= 2e3 rad in fp32
    out = list(acts.values())[-1]
    assert out.shape == (1, t.shape[1], 1)
    assert rel(out.detach().reshape(-1).cpu().numpy(), fb["w1000_out"]) < 1e-3
    # differentiable like the reference's (retain_grad on every entry)
    out.sum().backward()
    assert sine[1].grad is not None and m.net[0].linear.weight.grad is not None
    assert isinstance(m.net[1], SineLayer)


def test_lone_sine_layer_autograd_vs_torch(dev):
    from inr_for_audio_amd.models import SineLayer
    torch.manual_seed(3)
    layer = SineLayer(64, 128, is_first=False, omega_0=30.0).to(dev)
    x = torch.randn(3000, 64, device=dev, requires_grad=True)
    y, pre = layer.forward_with_intermediate(x)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    # plain fp32 PyTorch of the same op
    W = layer.linear.weight.detach().clone().requires_grad_(True)
    b = layer.linear.bias.detach().clone().requires_grad_(True)
    xr = x.detach().clone().requires_grad_(True)
    pr = 30.0 * torch.nn.functional.linear(xr, W, b)
    yr = torch.sin(pr)
    (yr * gy).sum().backward()
    errs = {"y": rel(y.detach().cpu(), yr.detach().cpu().double().numpy()),
            "pre": rel(pre.detach().cpu(), pr.detach().cpu().double().numpy()),
            "gW": rel(layer.linear.weight.grad.cpu(), W.grad.cpu().double().numpy()),
            "gb": rel(layer.linear.bias.grad.cpu(), b.grad.cpu().double().numpy()),
            "gx": rel(x.grad.cpu(), xr.grad.cpu().double().numpy())}
    log("lone_sine_layer", **errs)
    assert all(e < 1e-5 for e in errs.values()), errs
    assert torch.allclose(layer(x), y)
    with pytest.raises(RuntimeError):
        layer.cpu()(torch.zeros(4, 64))


@pytest.mark.parametrize("a0", [0.5, None])
def test_snake_and_tanh_modules_vs_torch(dev, a0):
    from inr_for_audio_amd.models import SirenWithSnakeTanh, Snake
    torch.manual_seed(1)
    sn = Snake(96, a=a0).to(dev)
    x = torch.randn(2000, 96, device=dev, requires_grad=True)
    y = sn(x)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    a = sn.a.detach().clone().requires_grad_(True)
    xr = x.detach().clone().requires_grad_(True)
    yr = xr + (1.0 / a) * torch.pow(torch.sin(xr * a), 2)      # models.py:241
    (yr * gy).sum().backward()
    errs = {"y": rel(y.detach().cpu(), yr.detach().cpu().double().numpy()),
            "gx": rel(x.grad.cpu(), xr.grad.cpu().double().numpy()),
            "ga": rel(sn.a.grad.cpu(), a.grad.cpu().double().numpy())}
    log(f"snake_module[{a0}]", **errs)
    assert all(e < 1e-5 for e in errs.values()), errs
    # a Tanh / Snake stack walks through forward_with_activations as the reference does
    torch.manual_seed(2)
    m = SirenWithSnakeTanh(1, 1, 128, 1, 1, 1, first_omega_0=500.0, a_initial=a0 or 2.0).to(dev)
    t = torch.linspace(-1, 1, 1000, device=dev).reshape(1, -1, 1)
    acts = m.forward_with_activations(t)
    h = torch.sin(500.0 * torch.nn.functional.linear(t, m.net[0].linear.weight, m.net[0].linear.bias))
    h = torch.sin(30.0 * torch.nn.functional.linear(h, m.net[1].linear.weight, m.net[1].linear.bias))
    z = torch.nn.functional.linear(h, m.net[2].weight, m.net[2].bias)
    h = z + (1.0 / m.net[3].a) * torch.pow(torch.sin(z * m.net[3].a), 2)
    h = torch.tanh(torch.nn.functional.linear(h, m.net[4].weight, m.net[4].bias))
    o = torch.nn.functional.linear(h, m.net[6].weight, m.net[6].bias)
    vals = list(acts.values())
    assert len(vals) == 1 + 2 * 2 + 5        # input, 2 SineLayers x 2, Linear/Snake/Linear/Tanh/Linear
    assert rel(vals[-1].detach().cpu(), o.detach().cpu().double().numpy()) < 1e-5


@pytest.mark.parametrize("a_shape", [(), (1,)])
def test_snake_scalar_a_broadcasts(dev, a_shape):
    """A scalar Snake `a` (the reference's formula broadcasts it over the columns, models.py:241)
    is applied to every column and gets the column-summed gradient in its own shape; an `a` of
    another length is refused instead of read out of bounds."""
    from inr_for_audio_amd import _lib
    from inr_for_audio_amd.models import fp32_act
    torch.manual_seed(3)
    x = torch.randn(700, 40, device=dev, requires_grad=True)
    a = torch.full(a_shape, 0.7, device=dev, requires_grad=True)
    y = fp32_act(x, _lib.FP32_SNAKE, a)
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    xr = x.detach().clone().requires_grad_(True)
    ar = a.detach().clone().requires_grad_(True)
    yr = xr + (1.0 / ar) * torch.pow(torch.sin(xr * ar), 2)
    (yr * gy).sum().backward()
    assert a.grad.shape == a.shape
    assert rel(y.detach().cpu(), yr.detach().cpu().double().numpy()) < 1e-5
    assert rel(x.grad.cpu(), xr.grad.cpu().double().numpy()) < 1e-5
    assert rel(a.grad.cpu().reshape(-1), ar.grad.cpu().double().numpy().reshape(-1)) < 1e-5
    with pytest.raises(ValueError):
        fp32_act(x, _lib.FP32_SNAKE, torch.ones(39, device=dev))
