"""SIREN modules with the reference's constructor API, parameter names and init
(models.py:84-120 SineLayer, models.py:306-394 SirenWithSnakeTanh), computing on the
gfx950 HIP kernels.

Parameters are created with exactly the reference's torch calls in the reference's order
(nn.Linear default init, then the SIREN re-draw), so ``torch.manual_seed(s)`` gives
bit-identical weights and the state_dict keys (``net.{i}.linear.weight`` ...,
``net.{L+1}.weight``) load into either implementation.

``forward`` runs the fused HIP forward and has a HIP backward (autograd.Function), so a
user loop of ``model(x)`` / ``loss.backward()`` / ``torch.optim.Adam`` works as a drop-in.
The fast path for fitting is ``engine.SirenEngine`` (used by ``run.train``).  There is no
eager fallback: CPU tensors or unsupported configurations raise.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
from torch import nn

from . import _lib


class SineLayer(nn.Module):
    """sin(omega_0 * Linear(x)) -- models.py:84-120 (init: models.py:105-112)."""

    def __init__(self, in_features, out_features, bias=True, is_first=False, omega_0=30):
        super().__init__()
        self.omega_0 = omega_0
        self.is_first = is_first
        self.in_features = in_features
        self.linear = nn.Linear(in_features, out_features, bias=bias)
        self.init_weights()

    def init_weights(self):
        with torch.no_grad():
            if self.is_first:
                self.linear.weight.uniform_(-1 / self.in_features, 1 / self.in_features)
            else:
                self.linear.weight.uniform_(-np.sqrt(6 / self.in_features) / self.omega_0,
                                            np.sqrt(6 / self.in_features) / self.omega_0)

    def forward(self, input):
        """sin(omega_0 * linear(input)) -- models.py:114-115, on the unfused fp32 HIP layer kernels
        (siren_fp32_linear / siren_fp32_act, differentiable).  Inside SirenWithSnakeTanh the
        fused fp16 path runs instead."""
        return self.forward_with_intermediate(input)[0]

    def forward_with_intermediate(self, input):
        """(sin(intermediate), intermediate) with intermediate = omega_0 * linear(input) --
        models.py:117-120 (activation inspection), fp32 on the GPU."""
        intermediate = fp32_linear(input, self.linear.weight, self.linear.bias, float(self.omega_0))
        return fp32_act(intermediate, _lib.FP32_SIN), intermediate


class Snake(nn.Module):
    """Snake activation y = x + sin^2(a x)/a with per-channel trainable a (models.py:185-241).

    Same parameter, init and RNG use as the reference: a = ones * a, or, for a=None, one
    Exponential(0.1) rsample per channel (models.py:224-229).  `trainable` is stored as the
    reference does (the `requiresGrad` attribute, models.py:231), i.e. a always trains.
    Inside SirenWithSnakeTanh the Linear + Snake pair runs as one fused HIP GEMM epilogue
    (gemm_nt.hip NT_FWD_SNAKE / NT_DX_SNAKE); a lone Snake has no kernel."""

    def __init__(self, in_features, a=None, trainable=True):
        super().__init__()
        self.in_features = in_features if isinstance(in_features, list) else [in_features]
        if a is not None:
            self.a = nn.Parameter(torch.ones(self.in_features) * a)
        else:
            m = torch.distributions.exponential.Exponential(torch.tensor([0.1]))
            self.a = nn.Parameter((m.rsample(self.in_features)).squeeze())
        self.a.requiresGrad = trainable

    def forward(self, x):
        """x + sin^2(a x)/a elementwise (models.py:235-241) on the fp32 HIP kernel
        (siren_fp32_act, differentiable in x and a).  Inside SirenWithSnakeTanh the Linear +
        Snake pair runs as one fused fp16 GEMM epilogue instead."""
        return fp32_act(x, _lib.FP32_SNAKE, self.a)


class SirenWithSnakeTanh(nn.Module):
    """MLP with sine / Snake / Tanh activations -- models.py:306-394.  The HIP path covers
    every configuration of the reference's constructor: a first SineLayer or (first_linear)
    a first Linear+Snake, then num_sine SineLayers, num_snake Linear+Snake and num_tanh
    Linear+Tanh hidden layers, then the final Linear or (last_linear=False) a final
    SineLayer(H, 1)."""

    def __init__(self, in_features, out_features, hidden_features, num_sine, num_snake, num_tanh,
                 first_linear=False, last_linear=True, first_omega_0=30, hidden_omega_0=30.,
                 a_initial=50, num_freq=None, scale=2.0):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.hidden_features = hidden_features
        self.num_sine, self.num_snake, self.num_tanh = num_sine, num_snake, num_tanh
        self.first_linear, self.last_linear = first_linear, last_linear
        self.first_omega_0, self.hidden_omega_0 = first_omega_0, hidden_omega_0
        net = []
        if first_linear:
            net.append(nn.Linear(in_features, hidden_features))
            net.append(Snake(hidden_features, a=a_initial))
        else:
            net.append(SineLayer(in_features, hidden_features, is_first=True, omega_0=first_omega_0))
        for _ in range(num_sine):
            net.append(SineLayer(hidden_features, hidden_features, is_first=False,
                                 omega_0=hidden_omega_0))
        for _ in range(num_snake):
            net.append(nn.Linear(hidden_features, hidden_features))
            net.append(Snake(hidden_features, a=a_initial))
        for _ in range(num_tanh):
            net.append(nn.Linear(hidden_features, hidden_features))
            net.append(nn.Tanh())
        if last_linear:
            final_linear = nn.Linear(hidden_features, out_features)
            with torch.no_grad():
                final_linear.weight.uniform_(-np.sqrt(6 / hidden_features) / hidden_omega_0,
                                             np.sqrt(6 / hidden_features) / hidden_omega_0)
            net.append(final_linear)
        else:
            net.append(SineLayer(hidden_features, out_features, is_first=False,
                                 omega_0=hidden_omega_0))
        self.net = nn.Sequential(*net)

    def hip_spec(self):
        """NetSpec of the fused path; raises for configurations it does not cover."""
        from .engine import NetSpec
        if self.out_features != 1:
            raise NotImplementedError("HIP path: out_features must be 1 (run.py:95,112)")
        n_inner = self.num_sine + self.num_snake + self.num_tanh
        if n_inner < 1:
            raise NotImplementedError("HIP path: at least one hidden layer (num_sine + num_snake + "
                                      "num_tanh >= 1)")
        if self.in_features not in (1, 2):
            raise NotImplementedError("HIP path: in_features must be 1 or 2")
        H = self.hip_width()
        if n_inner > _lib.MAX_INNER:
            raise NotImplementedError(f"HIP path: num_sine + num_snake + num_tanh <= {_lib.MAX_INNER}")
        acts = (_lib.ACT_SINE,) * self.num_sine + (_lib.ACT_SNAKE,) * self.num_snake + \
            (_lib.ACT_TANH,) * self.num_tanh
        return NetSpec(self.in_features, H, n_inner, float(self.first_omega_0),
                       float(self.hidden_omega_0), acts, bool(self.first_linear),
                       0.0 if self.last_linear else float(self.hidden_omega_0))

    def hip_width(self) -> int:
        """The hidden width the kernels run at: hidden_features itself when it is 128, 256, 512,
        1024 or a multiple of 1024 up to SIREN_MAX_HIDDEN (4096: the GEMM epilogues and the
        elementwise kernels run 1024-column windows of it), else the next of those -- the network is
        zero-padded to it (hip_padding), which computes the unpadded network's function and
        gradients exactly (padded units have zero weights in and out: their outputs are 0 and every
        gradient that touches them is 0).  The reference takes any width (models.py:310-311)."""
        H = int(self.hidden_features)
        for w in (128, 256, 512, 1024):
            if H <= w:
                return w
        if H <= _lib.MAX_HIDDEN:
            return -(-H // 1024) * 1024
        raise NotImplementedError(f"HIP path: hidden_features <= {_lib.MAX_HIDDEN} (SIREN_MAX_HIDDEN), got {H}")

    def hip_padding(self) -> dict:
        """{parameter index: (stored shape, fill)} for engine.ParamLayout when hidden_features is
        padded to hip_width(): the hidden axes of W0, b0, every W_i (both), b_i, Snake a (filled
        with 1, so that the padded units' sin^2(a z)/a stays finite), the head weight."""
        H, Hp = int(self.hidden_features), self.hip_width()
        if H == Hp:
            return {}
        ix = self.param_index()
        params = [p for _, p in self.named_parameters()]
        pad = {}

        def put(k, shape, fill=0.0):
            if params[k].dim() != len(shape):
                raise NotImplementedError(f"HIP path: cannot pad a parameter of shape {tuple(params[k].shape)} "
                                          f"to width {Hp}")
            pad[k] = (shape, fill)

        put(ix["W0"], (Hp, self.in_features))
        put(ix["b0"], (Hp,))
        if ix["a0"] is not None:
            put(ix["a0"], (Hp,), 1.0)
        for i in range(len(ix["W"])):
            put(ix["W"][i], (Hp, Hp))
            put(ix["b"][i], (Hp,))
            if ix["a"][i] is not None:
                put(ix["a"][i], (Hp,), 1.0)
        put(ix["wh"], (1, Hp))
        return pad

    def param_index(self):
        """Positions in named_parameters() order (== state_dict order == Adam's state index)
        of every tensor the fused path binds: {'W0', 'b0', 'W': [..], 'b': [..], 'a': [.. or
        None], 'wh', 'bh'} -- SineLayer: net.{i}.linear.{weight,bias}; Linear+Snake:
        net.{i}.{weight,bias} + net.{i+1}.a; Linear+Tanh: net.{i}.{weight,bias}."""
        names = [n for n, _ in self.named_parameters()]
        pos = {n: k for k, n in enumerate(names)}
        if self.first_linear:  # net.0 Linear, net.1 Snake (models.py:330-333)
            idx = {"W0": pos["net.0.weight"], "b0": pos["net.0.bias"], "a0": pos["net.1.a"], "W": [], "b": [],
                   "a": []}
            j = 2
        else:
            idx = {"W0": pos["net.0.linear.weight"], "b0": pos["net.0.linear.bias"], "a0": None, "W": [], "b": [],
                   "a": []}
            j = 1
        mods = list(self.net)
        for _ in range(self.num_sine):
            idx["W"].append(pos[f"net.{j}.linear.weight"])
            idx["b"].append(pos[f"net.{j}.linear.bias"])
            idx["a"].append(None)
            j += 1
        for kind in ["snake"] * self.num_snake + ["tanh"] * self.num_tanh:
            idx["W"].append(pos[f"net.{j}.weight"])
            idx["b"].append(pos[f"net.{j}.bias"])
            idx["a"].append(pos[f"net.{j + 1}.a"] if kind == "snake" else None)
            j += 2
        if self.last_linear:
            assert isinstance(mods[j], nn.Linear), "last layer must be the final Linear"
            idx["wh"], idx["bh"] = pos[f"net.{j}.weight"], pos[f"net.{j}.bias"]
        else:  # final SineLayer(H, 1) (models.py:383-385)
            idx["wh"], idx["bh"] = pos[f"net.{j}.linear.weight"], pos[f"net.{j}.linear.bias"]
        return idx

    def forward_with_activations(self, coords, retain_grad=False):
        """models.py:396-423: the output of every layer, plus each SineLayer's intermediate
        omega * linear(x), keyed like the reference ('<class ...>_<count>').  Visualisation
        only, so it walks the modules one by one on the unfused fp32 HIP kernels (SineLayer /
        Snake forward, siren_fp32_linear for nn.Linear, siren_fp32_act for nn.Tanh) -- the fp32
        values the reference reports, not the fused path's fp16 activations."""
        from collections import OrderedDict
        if not coords.is_cuda:
            raise RuntimeError("forward_with_activations runs on the HIP path only (CUDA tensors)")
        activations = OrderedDict()
        count = 0
        x = coords.clone().detach().requires_grad_(True)
        activations["input"] = x
        for layer in self.net:
            if isinstance(layer, SineLayer):
                x, intermed = layer.forward_with_intermediate(x)
                if retain_grad:
                    x.retain_grad()
                    intermed.retain_grad()
                activations["_".join((str(layer.__class__), "%d" % count))] = intermed
                count += 1
            else:
                if isinstance(layer, nn.Linear):
                    x = fp32_linear(x, layer.weight, layer.bias, 1.0)
                elif isinstance(layer, nn.Tanh):
                    x = fp32_act(x, _lib.FP32_TANH)
                else:
                    x = layer(x)
                if retain_grad:
                    x.retain_grad()
            activations["_".join((str(layer.__class__), "%d" % count))] = x
            count += 1
        return activations

    def forward(self, coords):
        """(1, N, in) or (N, in) CUDA coords -> (..., N, 1) fp32 output, differentiable in the
        parameters (models.py:388-394)."""
        if not coords.is_cuda:
            raise RuntimeError("SirenWithSnakeTanh.forward runs on the HIP path only (CUDA tensors)")
        spec = self.hip_spec()
        lead = coords.shape[:-1]
        params = [p for _, p in self.named_parameters()]
        ix = dict(self.param_index(), pad=self.hip_padding())
        out = _SirenFunction.apply((spec, ix), coords.reshape(-1, spec.in_dim).detach(), *params)
        return out.reshape(*lead, 1)


class _SirenFunction(torch.autograd.Function):
    """HIP forward/backward of the whole SIREN for an arbitrary upstream gradient."""

    @staticmethod
    def forward(ctx, spec_idx, coords, *params):
        from .engine import ROW_TILE, STORE16, Workspace, cast_shadows, make_net, round_up
        spec, ix = spec_idx
        dev = coords.device
        lib = _lib.load()
        L, H = spec.n_inner, spec.hidden
        n = coords.shape[0]
        rows = round_up(max(n, 1), ROW_TILE)
        # the kernels' width: padded copies when hidden_features is not 128/256/512/1024
        pad = ix.get("pad", {})
        p = []
        for k, t in enumerate(params):
            t = t.detach().float()
            if k in pad:
                shp, fill = pad[k]
                full = torch.full(shp, fill, dtype=torch.float32, device=dev)
                full[tuple(slice(0, d) for d in t.shape)] = t
                t = full
            p.append(t.contiguous())
        W = [p[k] for k in ix["W"]]
        Wh = [torch.empty(H, H, dtype=STORE16, device=dev) for _ in range(L)]
        WTh = [torch.empty(H, H, dtype=STORE16, device=dev) for _ in range(L)]
        s = torch.cuda.current_stream(dev).cuda_stream
        cast_shadows(spec, W, Wh, WTh, s)
        net = make_net(spec, p[ix["W0"]], p[ix["b0"]], [p[k] for k in ix["b"]], Wh, WTh, p[ix["wh"]],
                       p[ix["bh"]], [None if k is None else p[k] for k in ix["a"]],
                       None if ix["a0"] is None else p[ix["a0"]])
        ws = Workspace(spec, rows, dev, train=True)
        xc = torch.zeros(rows, spec.in_dim, dtype=torch.float32, device=dev)
        xc[:n] = coords.float()
        tgt = torch.zeros(rows, dtype=torch.float32, device=dev)
        b = ws.batch(xc, tgt, n, float(n))
        _lib.check(lib.siren_forward(ctypes.byref(net), ctypes.byref(b), s), "siren_forward")
        ctx.keep = (spec, ix, net, ws, xc, tgt, p, Wh, WTh, n, [t.shape for t in p], [t.shape for t in params])
        return ws.out[:n].clone()

    @staticmethod
    def backward(ctx, grad_out):
        from .engine import SEG_ALIGN, round_up
        from ._lib import SirenGrads, ptr
        spec, ix, net, ws, xc, tgt, p, Wh, WTh, n, shapes, true_shapes = ctx.keep
        lib = _lib.load()
        dev = xc.device
        L = spec.n_inner
        ws.g.zero_()
        ws.g[:n] = grad_out.reshape(-1).float()
        offs, off = [], 0
        for shp in shapes:
            offs.append(off)
            off = round_up(off + int(np.prod(shp)), SEG_ALIGN)
        flat = torch.zeros(off + SEG_ALIGN, dtype=torch.float32, device=dev)
        views = [flat[o:o + int(np.prod(shp))].view(shp) for o, shp in zip(offs, shapes)]
        gs = SirenGrads()
        gs.W0, gs.b0 = ptr(views[ix["W0"]]), ptr(views[ix["b0"]])
        for i in range(L):
            gs.W[i], gs.b[i] = ptr(views[ix["W"][i]]), ptr(views[ix["b"][i]])
            if ix["a"][i] is not None:
                gs.a[i] = ptr(views[ix["a"][i]])
        gs.w_head, gs.b_head = ptr(views[ix["wh"]]), ptr(views[ix["bh"]])
        if ix["a0"] is not None:
            gs.a0 = ptr(views[ix["a0"]])
        gs.sse, gs.flat, gs.flat_len = flat.data_ptr() + 4 * off, ptr(flat), off + SEG_ALIGN
        b = ws.batch(xc, tgt, n, float(n))
        s = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(lib.siren_backward(ctypes.byref(net), ctypes.byref(gs), ctypes.byref(b), s),
                   "siren_backward")
        ctx.keep = None
        # the model's own blocks of the (possibly padded) gradients
        grads = [v if v.shape == ts else v[tuple(slice(0, d) for d in ts)] for v, ts in zip(views, true_shapes)]
        return (None, None, *grads)


# ---- unfused fp32 layers (layer_fp32.hip): the module API outside the fused step ----------
def _splits(rows: int) -> int:
    return max(1, min(256, rows // 2048))


class _Fp32Linear(torch.autograd.Function):
    """pre = omega * (x W^T + b) in fp32 (siren_fp32_linear) and its autograd
    (siren_fp32_linear_bwd)."""

    @staticmethod
    def forward(ctx, x, W, b, omega):
        lib = _lib.load()
        lead = x.shape[:-1]
        xs = x.reshape(-1, x.shape[-1]).contiguous().float()
        rows, fin = xs.shape
        out = W.shape[0]
        pre = torch.empty(rows, out, dtype=torch.float32, device=x.device)
        s = torch.cuda.current_stream(x.device).cuda_stream
        _lib.check(lib.siren_fp32_linear(_lib.ptr(xs), rows, fin, out, _lib.ptr(W.detach().contiguous()),
                                         _lib.ptr(None if b is None else b.detach().contiguous()),
                                         float(omega), _lib.ptr(pre), s), "siren_fp32_linear")
        ctx.save_for_backward(xs, W, b if b is not None else torch.empty(0, device=x.device))
        ctx.has_b, ctx.omega, ctx.lead = b is not None, float(omega), lead
        return pre.reshape(*lead, out)

    @staticmethod
    def backward(ctx, gpre):
        lib = _lib.load()
        xs, W, b = ctx.saved_tensors
        rows, fin = xs.shape
        out = W.shape[0]
        dev = xs.device
        g = gpre.reshape(rows, out).contiguous().float().clone()  # overwritten with omega * gpre
        gW = torch.empty(out, fin, dtype=torch.float32, device=dev)
        gb = torch.empty(out, dtype=torch.float32, device=dev) if ctx.has_b else None
        gx = torch.empty(rows, fin, dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None
        splits = _splits(rows)
        slab = torch.empty(splits * out * fin if splits > 1 else 1, dtype=torch.float32, device=dev)
        tmp = torch.empty(64 * out, dtype=torch.float32, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(lib.siren_fp32_linear_bwd(_lib.ptr(xs), rows, fin, out, _lib.ptr(W.detach().contiguous()),
                                             ctx.omega, _lib.ptr(g), _lib.ptr(gx), _lib.ptr(gW), _lib.ptr(gb),
                                             _lib.ptr(slab), splits, _lib.ptr(tmp), s), "siren_fp32_linear_bwd")
        return (None if gx is None else gx.reshape(*ctx.lead, fin)), gW, gb, None


class _Fp32Act(torch.autograd.Function):
    """y = act(x) elementwise in fp32 (siren_fp32_act) and its autograd (siren_fp32_act_bwd)."""

    @staticmethod
    def forward(ctx, x, act, a):
        lib = _lib.load()
        xs = x.contiguous().float()
        cols = xs.shape[-1]
        rows = xs.numel() // cols
        y = torch.empty_like(xs)
        s = torch.cuda.current_stream(x.device).cuda_stream
        ac = None
        ctx.a_shape = None
        if a is not None:
            # the kernel reads a[column]: one value per column, or a scalar broadcast to every column
            # (the reference's Snake broadcasts `a` against x; models.py:241)
            if a.numel() not in (1, cols):
                raise ValueError(f"Snake a has {a.numel()} values for {cols} columns (need {cols} or 1)")
            ac = a.detach().reshape(-1).float().expand(cols).contiguous()
            ctx.a_shape = a.shape
        _lib.check(lib.siren_fp32_act(int(act), _lib.ptr(xs), rows, cols, _lib.ptr(ac), _lib.ptr(y), s),
                   "siren_fp32_act")
        ctx.save_for_backward(xs, ac if ac is not None else torch.empty(0, device=x.device))
        ctx.act, ctx.has_a = int(act), a is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = _lib.load()
        xs, ac = ctx.saved_tensors
        cols = xs.shape[-1]
        rows = xs.numel() // cols
        g = gy.contiguous().float()
        gx = torch.empty_like(xs)
        want_da = ctx.has_a and ctx.needs_input_grad[2]
        da = torch.empty(cols, dtype=torch.float32, device=xs.device) if want_da else None
        prod = torch.empty_like(xs) if want_da else None
        tmp = torch.empty(64 * cols, dtype=torch.float32, device=xs.device) if want_da else None
        s = torch.cuda.current_stream(xs.device).cuda_stream
        _lib.check(lib.siren_fp32_act_bwd(ctx.act, _lib.ptr(xs), rows, cols, _lib.ptr(ac if ctx.has_a else None),
                                          _lib.ptr(g), _lib.ptr(gx), _lib.ptr(da), _lib.ptr(prod), _lib.ptr(tmp), s),
                   "siren_fp32_act_bwd")
        if da is not None:  # back to a's own shape (summed over the columns a scalar a was broadcast to)
            da = (da.sum() if math.prod(ctx.a_shape) == 1 and cols > 1 else da).reshape(ctx.a_shape)
        return gx, None, da


def fp32_linear(x, weight, bias, omega=1.0):
    """omega * (x W^T + b) on the fp32 HIP kernels (x [..., in] CUDA)."""
    if not x.is_cuda:
        raise RuntimeError("the HIP layer kernels take CUDA tensors (no CPU fallback)")
    return _Fp32Linear.apply(x, weight, bias, float(omega))


def fp32_act(x, act, a=None):
    """elementwise sin / tanh / Snake(a) / identity on the fp32 HIP kernel (x CUDA)."""
    if not x.is_cuda:
        raise RuntimeError("the HIP layer kernels take CUDA tensors (no CPU fallback)")
    return _Fp32Act.apply(x, act, a)
