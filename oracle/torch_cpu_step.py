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


def build(in_dim, hidden, n_inner, omega0, omega, seed=0):
    torch.manual_seed(seed)
    layers = [_Sine(in_dim, hidden, omega0, True)]
    layers += [_Sine(hidden, hidden, omega, False) for _ in range(n_inner)]
    last = nn.Linear(hidden, 1)
    with torch.no_grad():
        lim = math.sqrt(6 / hidden) / omega
        last.weight.uniform_(-lim, lim)
    layers.append(last)
    return nn.Sequential(*layers)


def time_steps(n_coords=65536, hidden=1024, n_inner=4, steps=6, threads=None, omega0=3000.0,
               omega=30.0, seed=0, in_dim=1):
    """Median wall time of steps 2..k of the full-batch loop (BASELINE.md CPU plan)."""
    if threads:
        torch.set_num_threads(int(threads))
    model = build(in_dim, hidden, n_inner, omega0, omega, seed)
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
