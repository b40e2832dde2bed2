"""CPU BASELINE (port) of the reference training step -- TEST / BENCH INFRASTRUCTURE ONLY.

A restatement of run.py's hot loop (run.py:156-187) with the same torch CPU ops the
reference uses in fp32: nn.Linear, omega*sin (models.py:114-115), nn.MSELoss,
torch.optim.Adam, ReduceLROnPlateau.  bench.py times it as `cpu_baseline` (kind "port")
because the reference's own code cannot travel to the GPU box.  Never imported by the
product package.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch
from torch import nn


class _Sine(nn.Module):
    def __init__(self, fin, fout, omega, first):
        super().__init__()
        self.omega = omega
        self.linear = nn.Linear(fin, fout)
        with torch.no_grad():
            lim = 1 / fin if first else math.sqrt(6 / fin) / omega
            self.linear.weight.uniform_(-lim, lim)

    def forward(self, x):
        return torch.sin(self.omega * self.linear(x))


class _Snake(nn.Module):
    """nn.Linear + Snake (models.py:235-241): x + (1/a) sin^2(a x), trainable a per channel."""

    def __init__(self, fin, fout, a0):
        super().__init__()
        self.linear = nn.Linear(fin, fout)
        self.a = nn.Parameter(torch.ones(fout) * a0)

    def forward(self, x):
        z = self.linear(x)
        return z + (1.0 / self.a) * torch.pow(torch.sin(z * self.a), 2)


def build(in_dim, hidden, n_inner, omega0, omega, seed=0, n_snake=0, a0=0.5):
    """First SineLayer, n_inner hidden SineLayers, n_snake Linear + Snake layers, final Linear
    (models.py:306-394 with first_linear=False, num_tanh=0, last_linear=True)."""
    torch.manual_seed(seed)
    layers = [_Sine(in_dim, hidden, omega0, True)]
    layers += [_Sine(hidden, hidden, omega, False) for _ in range(n_inner)]
    layers += [_Snake(hidden, hidden, a0) for _ in range(n_snake)]
    last = nn.Linear(hidden, 1)
    with torch.no_grad():
        lim = math.sqrt(6 / hidden) / omega
        last.weight.uniform_(-lim, lim)
    layers.append(last)
    return nn.Sequential(*layers)


def time_steps(n_coords=65536, hidden=1024, n_inner=4, steps=6, threads=None, omega0=3000.0,
               omega=30.0, seed=0, in_dim=1, n_snake=0, a0=0.5):
    """Median wall time of steps 2..k of the full-batch loop (BASELINE.md CPU plan)."""
    if threads:
        torch.set_num_threads(int(threads))
    model = build(in_dim, hidden, n_inner, omega0, omega, seed, n_snake=n_snake, a0=a0)
    t = torch.linspace(-1, 1, n_coords).reshape(1, n_coords, 1)
    y = 0.5 * torch.sin(37 * t) + 0.3 * torch.sin(91 * t + 0.5)
    if in_dim == 2:  # (t, ch) rows: channel -1 / +1 alternating
        ch = torch.where(torch.arange(n_coords) % 2 == 0, -1.0, 1.0).reshape(1, n_coords, 1)
        t = torch.cat([t, ch], -1)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.8, patience=200,
                                                       min_lr=1e-6)
    mse = nn.MSELoss()
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        out = model(t)
        loss = mse(out, y)
        _ = loss.item()
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step(loss)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times[1:])) if len(times) > 1 else times[0]
    return {"sec_per_step": med, "coord_samples_per_sec": n_coords / med,
            "threads": torch.get_num_threads(), "n_coords": n_coords, "steps": steps, "step_times": times}


class _KANLinear(nn.Module):
    """efficient-KAN's KANLinear forward (kan.py:6-166; grid 5, order 3, SiLU base) in torch fp32."""

    def __init__(self, fin, fout, grid_size=5, order=3, grid_range=(-1.0, 1.0)):
        super().__init__()
        self.order = order
        h = (grid_range[1] - grid_range[0]) / grid_size
        g = torch.arange(-order, grid_size + order + 1, dtype=torch.float32) * h + grid_range[0]
        self.register_buffer("grid", g.expand(fin, -1).contiguous())
        self.base_weight = nn.Parameter(torch.empty(fout, fin).uniform_(-1 / math.sqrt(fin), 1 / math.sqrt(fin)))
        self.spline_weight = nn.Parameter(torch.randn(fout, fin, grid_size + order) * 0.1 / grid_size)
        self.spline_scaler = nn.Parameter(torch.empty(fout, fin).uniform_(-1 / math.sqrt(fin), 1 / math.sqrt(fin)))

    def b_splines(self, x):
        g = self.grid
        x = x.unsqueeze(-1)
        b = ((x >= g[:, :-1]) & (x < g[:, 1:])).to(x.dtype)
        for k in range(1, self.order + 1):
            b = ((x - g[:, :-(k + 1)]) / (g[:, k:-1] - g[:, :-(k + 1)]) * b[:, :, :-1]
                 + (g[:, k + 1:] - x) / (g[:, k + 1:] - g[:, 1:(-k)]) * b[:, :, 1:])
        return b

    def forward(self, x):
        base = nn.functional.linear(nn.functional.silu(x), self.base_weight)
        w = (self.spline_weight * self.spline_scaler.unsqueeze(-1)).view(self.spline_weight.shape[0], -1)
        return base + nn.functional.linear(self.b_splines(x).view(x.shape[0], -1), w)


def kan_time_steps(n_coords=65536, widths=(1, 64, 64, 1), steps=6, threads=None, seed=0):
    """Median wall time of steps 2..k of the KAN full-batch loop (run.py:92-93, :156-187)."""
    if threads:
        torch.set_num_threads(int(threads))
    torch.manual_seed(seed)
    model = nn.Sequential(*[_KANLinear(a, b) for a, b in zip(widths[:-1], widths[1:])])
    t = torch.linspace(-1, 1, n_coords).reshape(n_coords, 1)
    y = 0.5 * torch.sin(37 * t) + 0.3 * torch.sin(91 * t + 0.5)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.8, patience=200, min_lr=1e-6)
    mse = nn.MSELoss()
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        loss = mse(model(t), y)
        _ = loss.item()
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step(loss)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times[1:])) if len(times) > 1 else times[0]
    return {"sec_per_step": med, "coord_samples_per_sec": n_coords / med,
            "threads": torch.get_num_threads(), "n_coords": n_coords, "steps": steps, "step_times": times}
