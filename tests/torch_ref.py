"""The reference loop (run.py:156-187) in plain fp32 PyTorch eager on the GPU -- TEST
INFRASTRUCTURE, never the product: a second run of the reference algorithm, same init, same
data, same ops (nn.Linear addmm, omega*sin, MSELoss, torch.optim.Adam, ReduceLROnPlateau),
but with the GPU's fp32 summation orders instead of the CPU's.  The fit-parity tests use it
to measure how far the fp32 reference itself moves between two devices on these chaotic
full-batch fits, next to how far the HIP path moves."""
from __future__ import annotations

import numpy as np
import torch


def fp32_fit(state_dict: dict, n_inner: int, omega0: float, coords, target, steps: int, lr: float = 1e-3,
             patience: int = 200, min_lr: float = 1e-6, omega: float = 30.0, device="cuda", factor: float = 0.8,
             final: bool = False):
    """Sine-only SirenWithSnakeTanh (models.py:114-115, :374-394) fitted full batch; returns
    (losses [steps], lrs [steps]) as float64 numpy, and with final=True also the model output of
    the final weights (float32 numpy)."""
    assert not torch.backends.cuda.matmul.allow_tf32
    p = {k: v.detach().clone().float().to(device).requires_grad_(True) for k, v in state_dict.items()}
    names = list(p)
    x = torch.as_tensor(coords, dtype=torch.float32).reshape(-1, p["net.0.linear.weight"].shape[1]).to(device)
    y = torch.as_tensor(target, dtype=torch.float32).reshape(-1, 1).to(device)
    opt = torch.optim.Adam([p[k] for k in names], lr=lr)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=factor, patience=patience,
                                                       min_lr=min_lr)
    mse = torch.nn.MSELoss()

    def forward():
        h = torch.sin(omega0 * torch.nn.functional.linear(x, p["net.0.linear.weight"], p["net.0.linear.bias"]))
        for j in range(1, n_inner + 1):
            h = torch.sin(omega * torch.nn.functional.linear(h, p[f"net.{j}.linear.weight"], p[f"net.{j}.linear.bias"]))
        j = n_inner + 1
        return torch.nn.functional.linear(h, p[f"net.{j}.weight"], p[f"net.{j}.bias"])

    losses, lrs = [], []
    for _ in range(steps):
        loss = mse(forward(), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step(loss.detach())
        losses.append(loss.detach())
        lrs.append(sched.get_last_lr()[0])
    out = (torch.stack(losses).double().cpu().numpy(), np.array(lrs))
    if final:
        with torch.no_grad():
            out = out + (forward().reshape(-1).cpu().numpy(),)
    return out


def fp32_fit_stack(state_dict: dict, kinds, omega0: float, coords, target, steps: int, lr: float = 1e-3,
                   patience: int = 200, min_lr: float = 1e-6, omega: float = 30.0, device="cuda"):
    """fp32_fit for a sine / Snake / Tanh stack (models.py:306-394): `kinds` names the hidden layers
    after the first SineLayer in order ("sine", "snake", "tanh"), as SirenWithSnakeTanh builds them
    (Snake: x + sin^2(a x)/a, models.py:235-241).  Returns (losses [steps], lrs [steps])."""
    assert not torch.backends.cuda.matmul.allow_tf32
    p = {k: v.detach().clone().float().to(device).requires_grad_(True) for k, v in state_dict.items()}
    names = list(p)
    x = torch.as_tensor(coords, dtype=torch.float32).reshape(-1, p["net.0.linear.weight"].shape[1]).to(device)
    y = torch.as_tensor(target, dtype=torch.float32).reshape(-1, 1).to(device)
    opt = torch.optim.Adam([p[k] for k in names], lr=lr)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.8, patience=patience, min_lr=min_lr)
    mse = torch.nn.MSELoss()
    lin = torch.nn.functional.linear

    def forward():
        h = torch.sin(omega0 * lin(x, p["net.0.linear.weight"], p["net.0.linear.bias"]))
        j = 1
        for kind in kinds:
            if kind == "sine":
                h = torch.sin(omega * lin(h, p[f"net.{j}.linear.weight"], p[f"net.{j}.linear.bias"]))
                j += 1
            elif kind == "snake":
                z = lin(h, p[f"net.{j}.weight"], p[f"net.{j}.bias"])
                a = p[f"net.{j + 1}.a"]
                h = z + (1.0 / a) * torch.pow(torch.sin(z * a), 2)
                j += 2
            else:
                h = torch.tanh(lin(h, p[f"net.{j}.weight"], p[f"net.{j}.bias"]))
                j += 2
        return lin(h, p[f"net.{j}.weight"], p[f"net.{j}.bias"])

    losses, lrs = [], []
    for _ in range(steps):
        loss = mse(forward(), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step(loss.detach())
        losses.append(loss.detach())
        lrs.append(sched.get_last_lr()[0])
    return torch.stack(losses).double().cpu().numpy(), np.array(lrs)
