"""Diagnostic (not the product path): the 300-step golden-clip fit of tests/test_gpu_fit.py
trained by plain torch autograd on the GPU, in fp32 or with the HIP path's bf16 storage
points emulated, to separate the chaos of the reference loop (late Adam loss spikes) from
effects of the HIP path's bf16 activation storage.

Storage points emulated with --bf16 (see inr-for-audio_amd/csrc/gemm_nt.hip): every hidden
layer's input Y (sin) is rounded to bf16 before its GEMM, the GEMM weights are bf16 shadows
of the fp32 master weights, and the backward uses the bf16 cos C and bf16 dZ.

    python tools/fit_torch_diag.py [--seeds 0,1,2,3,4] [--modes fp32,bf16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
G = os.path.join(ROOT, "tests", "golden")


MODES = {
    # name: (forward storage dtype for Y / W, backward storage dtype for C / dZ)
    "fp32": (None, None),
    "bf16": (torch.bfloat16, torch.bfloat16),
    "bf16_fwd": (torch.bfloat16, None),
    "bf16_bwd": (None, torch.bfloat16),
    "fp16": (torch.float16, torch.float16),
    "fp16_fwd": (torch.float16, None),
    # forward storage split by operand: (Y dtype, W dtype), backward fp32
    "bf16_Y": ("Y", torch.bfloat16),
    "bf16_W": ("W", torch.bfloat16),
    "fp16_Y": ("Y", torch.float16),
    "fp16_W": ("W", torch.float16),
}


def _rnd(x, dt):
    if dt is None:
        return x
    if dt == torch.float16:
        # dynamic power-of-two scale so the tensor's max lands near 2^14 (fp16 max 65504)
        m = float(x.abs().max())
        if m == 0.0:
            return x
        s = 2.0 ** (14 - np.ceil(np.log2(m)))
        return (x * s).to(dt).to(torch.float32) / s
    return x.to(dt).to(torch.float32)


class _Q(torch.autograd.Function):
    """Forward storage rounding with an identity gradient (a cast's own backward would round
    the gradient to the storage dtype too -- fp16 underflows there)."""

    @staticmethod
    def forward(ctx, x, dt):
        return x.to(dt).to(torch.float32)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _Sin(torch.autograd.Function):
    """y = sin(a); stores cos in the backward storage dtype; the incoming gradient (dZ of the
    next GEMM) is rounded to it too."""

    @staticmethod
    def forward(ctx, a, dt):
        ctx.dt = dt
        ctx.save_for_backward(_rnd(torch.cos(a), dt))
        return torch.sin(a)

    @staticmethod
    def backward(ctx, g):
        (c,) = ctx.saved_tensors
        return g * c, None


class _RoundGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dt):
        ctx.dt = dt
        return x

    @staticmethod
    def backward(ctx, g):
        return _rnd(g, ctx.dt), None


def forward(params, t, w0, w, mode):
    fdt, bdt = MODES[mode]
    ydt = wdt = fdt
    if fdt in ("Y", "W"):  # one forward operand rounded, backward fp32
        ydt, wdt = (bdt, None) if fdt == "Y" else (None, bdt)
        bdt = None
    W0, b0 = params[0], params[1]
    a = w0 * (t @ W0.t() + b0)
    y = _Sin.apply(a, bdt)
    L = (len(params) - 4) // 2
    for i in range(L):
        W, b = params[2 + 2 * i], params[3 + 2 * i]
        x = y if ydt is None else _Q.apply(y, ydt)
        Wq = W if wdt is None else _Q.apply(W, wdt)
        z = _RoundGrad.apply(x @ Wq.t() + b, bdt)
        y = _Sin.apply(w * z, bdt)
    return y @ params[-2].t() + params[-1]


def fit(dev, steps, seed, mode, hidden=256, layers=2, w0=1000.0):
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    t = torch.from_numpy(g["coords"]).reshape(-1, 1).to(dev)
    y = torch.from_numpy(g["target"]).reshape(-1, 1).to(dev)
    torch.manual_seed(seed)
    m = SirenWithSnakeTanh(1, 1, hidden, layers, 0, 0, first_omega_0=w0, hidden_omega_0=30.0)
    params = [p.detach().clone().to(dev).requires_grad_(True) for p in m.parameters()]
    opt = torch.optim.Adam(params, lr=1e-3)
    sch = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.8, patience=200, min_lr=1e-6)
    losses = []
    for _ in range(steps):
        out = forward(params, t, w0, 30.0, mode)
        loss = torch.mean((out - y) ** 2)
        opt.zero_grad()
        loss.backward()
        opt.step()
        sch.step(loss.detach())
        losses.append(float(loss))
    with torch.no_grad():
        out = forward(params, t, w0, 30.0, mode).cpu().numpy().reshape(-1)
    from inr_for_audio_amd.utils import calculate_snr
    return float(calculate_snr(g["target"], out)), np.array(losses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="0,1,2,3,4")
    ap.add_argument("--modes", default="fp32,bf16")
    ap.add_argument("--steps", type=int, default=300)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.backends.cuda.matmul.allow_tf32 = False
    for mode in args.modes.split(","):
        snrs = []
        for seed in [int(s) for s in args.seeds.split(",")]:
            snr, losses = fit(dev, args.steps, seed, mode)
            snrs.append(snr)
            print(json.dumps({"mode": mode, "seed": seed, "snr": snr, "final": float(losses[-1]),
                              "min": float(losses.min()), "argmin": int(losses.argmin())}), flush=True)
        print(json.dumps({"mode": mode, "median_snr": float(np.median(snrs)), "snrs": [round(x, 2) for x in snrs]}), flush=True)


if __name__ == "__main__":
    main()
