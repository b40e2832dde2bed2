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


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


class _SinBF16(torch.autograd.Function):
    """y = sin(a); stores bf16 cos for the backward; the incoming gradient is rounded to bf16
    after the multiply (dZ storage)."""

    @staticmethod
    def forward(ctx, a):
        ctx.save_for_backward(_bf(torch.cos(a)))
        return torch.sin(a)

    @staticmethod
    def backward(ctx, g):
        (c,) = ctx.saved_tensors
        return g * c


class _RoundGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        return _bf(g)


def forward(params, t, w0, w, bf16):
    W0, b0 = params[0], params[1]
    a = w0 * (t @ W0.t() + b0)
    y = _SinBF16.apply(a) if bf16 else torch.sin(a)
    L = (len(params) - 4) // 2
    for i in range(L):
        W, b = params[2 + 2 * i], params[3 + 2 * i]
        if bf16:
            x = _bf(y)
            z = x @ _bf(W).t() + b
            z = _RoundGrad.apply(z)
            y = _SinBF16.apply(w * z)
        else:
            y = torch.sin(w * (y @ W.t() + b))
    return y @ params[-2].t() + params[-1]


def fit(dev, steps, seed, bf16, hidden=256, layers=2, w0=1000.0):
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
        out = forward(params, t, w0, 30.0, bf16)
        loss = torch.mean((out - y) ** 2)
        opt.zero_grad()
        loss.backward()
        opt.step()
        sch.step(loss)
        losses.append(float(loss))
    with torch.no_grad():
        out = forward(params, t, w0, 30.0, bf16).cpu().numpy().reshape(-1)
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
            snr, losses = fit(dev, args.steps, seed, mode == "bf16")
            snrs.append(snr)
            print(json.dumps({"mode": mode, "seed": seed, "snr": snr, "final": float(losses[-1]),
                              "min": float(losses.min()), "argmin": int(losses.argmin())}), flush=True)
        print(json.dumps({"mode": mode, "median_snr": float(np.median(snrs))}), flush=True)


if __name__ == "__main__":
    main()
