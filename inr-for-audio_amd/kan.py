"""KAN variant: efficient-KAN's ``KAN`` / ``KANLinear`` (kan.py:6-285, used by
run.py:92-93 as ``KAN([1, H, H, 1])``) with the reference's constructor API, parameter and
buffer names (``layers.{l}.base_weight``, ``.spline_weight``, ``.spline_scaler``, ``.grid``) and
init, computing on the gfx950 path (kan.hip through the C-ABI siren_kan_*).

Init runs the same torch calls in the same order as the reference (kaiming-uniform base
weight, a uniform-noise curve fitted by least squares onto the B-spline basis, kaiming-uniform
scaler), so ``torch.manual_seed(s)`` gives bit-identical parameters.  The B-spline basis used
for that fit is the Cox-de Boor recursion of kan.py:94-104, vectorised over knots.

Supported like run.py uses it: grid_size 5, spline_order 3, SiLU base activation,
standalone spline scaler.  ``KAN.forward`` and ``KANLinear.forward`` are differentiable
(``_KanFunction``: siren_kan_forward, then siren_kan_backward for any upstream gradient, into the
parameters and, when asked for, the input), so a user loop with ``loss.backward()`` and
``torch.optim`` trains them as it trains the reference's modules (kan.py:153-166, 268-273); the
fused fit goes through ``KanEngine`` / ``run.train(arch='kan')``.  Grid updates and the
regularisation loss (not used by run.py) are not on the path.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from ._lib import SirenKanBatch, SirenKanGrads, SirenKanNet, check, ptr


def bspline_bases(x: torch.Tensor, knots: torch.Tensor, order: int) -> torch.Tensor:
    """(batch, in) inputs on per-input knots (in, G) -> (batch, in, G - 1 - order) bases, by the
    Cox-de Boor recursion with kan.py:94-104's operation order."""
    x = x.unsqueeze(-1)
    lo, hi = knots[:, :-1], knots[:, 1:]
    b = ((x >= lo) & (x < hi)).to(x.dtype)
    for k in range(1, order + 1):
        left = (x - knots[:, :-(k + 1)]) / (knots[:, k:-1] - knots[:, :-(k + 1)]) * b[:, :, :-1]
        right = (knots[:, k + 1:] - x) / (knots[:, k + 1:] - knots[:, 1:(-k)]) * b[:, :, 1:]
        b = left + right
    return b.contiguous()


class KANLinear(torch.nn.Module):
    """kan.py:6-166 (parameters, buffer and init; forward on the HIP path via KAN)."""

    def __init__(self, in_features, out_features, grid_size=5, spline_order=3, scale_noise=0.1,
                 scale_base=1.0, scale_spline=1.0, enable_standalone_scale_spline=True,
                 base_activation=torch.nn.SiLU, grid_eps=0.02, grid_range=[-1, 1]):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.grid_size, self.spline_order = grid_size, spline_order
        step = (grid_range[1] - grid_range[0]) / grid_size
        knots = torch.arange(-spline_order, grid_size + spline_order + 1) * step + grid_range[0]
        self.register_buffer("grid", knots.expand(in_features, -1).contiguous())
        self.base_weight = torch.nn.Parameter(torch.Tensor(out_features, in_features))
        self.spline_weight = torch.nn.Parameter(torch.Tensor(out_features, in_features, grid_size + spline_order))
        if enable_standalone_scale_spline:
            self.spline_scaler = torch.nn.Parameter(torch.Tensor(out_features, in_features))
        self.scale_noise, self.scale_base, self.scale_spline = scale_noise, scale_base, scale_spline
        self.enable_standalone_scale_spline = enable_standalone_scale_spline
        self.base_activation = base_activation()
        self.grid_eps = grid_eps
        self.reset_parameters()

    def reset_parameters(self):
        torch.nn.init.kaiming_uniform_(self.base_weight, a=math.sqrt(5) * self.scale_base)
        with torch.no_grad():
            g = self.grid_size
            noise = (torch.rand(g + 1, self.in_features, self.out_features) - 1 / 2) * self.scale_noise / g
            interior = self.grid.T[self.spline_order:-self.spline_order]
            coeff = self.curve2coeff(interior, noise)
            self.spline_weight.data.copy_((1.0 if self.enable_standalone_scale_spline else self.scale_spline)
                                          * coeff)
            if self.enable_standalone_scale_spline:
                torch.nn.init.kaiming_uniform_(self.spline_scaler, a=math.sqrt(5) * self.scale_spline)

    def b_splines(self, x: torch.Tensor) -> torch.Tensor:
        return bspline_bases(x, self.grid, self.spline_order)

    def curve2coeff(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """Least-squares spline coefficients (out, in, coeff) of curves y (batch, in, out)
        sampled at x (batch, in) -- kan.py:106-135."""
        sol = torch.linalg.lstsq(self.b_splines(x).transpose(0, 1), y.transpose(0, 1)).solution
        return sol.permute(2, 0, 1).contiguous()

    @property
    def scaled_spline_weight(self):
        s = self.spline_scaler.unsqueeze(-1) if self.enable_standalone_scale_spline else 1.0
        return self.spline_weight * s

    def forward(self, x: torch.Tensor):
        """kan.py:153-166: (..., in) -> (..., out), a one-layer KAN on the HIP path (differentiable)."""
        _hip_check_layer(self)
        return _kan_apply([self.in_features, self.out_features], [self], x,
                          [self.base_weight, self.spline_weight, self.spline_scaler])


def _hip_check_layer(lay: "KANLinear"):
    if lay.grid_size != 5 or lay.spline_order != 3:
        raise NotImplementedError("HIP KAN path: grid_size=5, spline_order=3 (kan.py defaults)")
    if not lay.enable_standalone_scale_spline or not isinstance(lay.base_activation, torch.nn.SiLU):
        raise NotImplementedError("HIP KAN path: SiLU base and a standalone spline scaler")
    # kan.hip finds a basis span by counting knots <= x, which equals kan.py:94-96's span predicate
    # for non-decreasing knots (kan.py's grids always are; checked once per grid version)
    key = (lay.grid.data_ptr(), lay.grid._version)
    if getattr(lay, "_knots_checked", None) != key:
        g = lay.grid
        if not bool((g[:, 1:] >= g[:, :-1]).all()):
            raise NotImplementedError("HIP KAN path: every input's knots must be non-decreasing")
        lay._knots_checked = key


def _kan_splits(rows: int) -> int:
    return max(1, min(256, rows // 2048))


def _net(widths, layers, params) -> SirenKanNet:
    n = SirenKanNet()
    n.n_layers = len(layers)
    for l, w in enumerate(widths):
        n.width[l] = w
    for l, lay in enumerate(layers):
        n.grid[l] = ptr(lay.grid)
        n.base_w[l], n.spline_w[l], n.scaler[l] = (ptr(t) for t in params[3 * l:3 * l + 3])
    return n


class _KanFunction(torch.autograd.Function):
    """HIP forward (siren_kan_forward) and backward (siren_kan_backward, any upstream gradient) of
    a KANLinear stack; params = (base_weight, spline_weight, spline_scaler) per layer."""

    @staticmethod
    def forward(ctx, widths, layers, x, *params):
        lib = _lib.load()
        if not x.is_cuda:
            raise RuntimeError("KAN runs on the HIP path only (CUDA tensors)")
        dev = x.device
        p = [t.detach().contiguous().float() for t in params]
        net = _net(widths, layers, p)
        xs = x.detach().reshape(-1, widths[0]).contiguous().float()
        rows = xs.shape[0]
        splits = _kan_splits(rows)
        ws = torch.empty(int(lib.siren_kan_workspace_floats(ctypes.byref(net), rows, splits)), device=dev)
        out = torch.empty(rows, widths[-1], dtype=torch.float32, device=dev)
        g = torch.zeros(rows, widths[-1], dtype=torch.float32, device=dev)
        b = SirenKanBatch()
        b.rows, b.n_valid, b.n_total, b.splits, b.zero_grads = rows, 0, 1.0, splits, 0
        b.coords, b.target, b.out, b.g, b.ws = ptr(xs), 0, ptr(out), ptr(g), ptr(ws)
        check(lib.siren_kan_forward(ctypes.byref(net), ctypes.byref(b), torch.cuda.current_stream(dev).cuda_stream),
              "siren_kan_forward")
        # the input and parameters go through save_for_backward so that torch's version counter
        # catches an in-place change between forward and backward (the workspace holds state
        # computed from them, e.g. the combined spline_w * scaler weights); the rest is non-tensor
        # state and the workspace
        ctx.save_for_backward(x, *params)
        ctx.keep = (net, b, ws, xs, g, p, x.shape, [t.shape for t in params])
        return out.reshape(*x.shape[:-1], widths[-1])

    @staticmethod
    def backward(ctx, grad_out):
        lib = _lib.load()
        _ = ctx.saved_tensors  # raises if x or a parameter was modified in place since the forward
        if ctx.keep is None:
            raise RuntimeError("KAN HIP backward: the forward's workspace is consumed by the first backward; "
                               "run the forward again instead of backward(retain_graph=True) twice")
        net, b, ws, xs, g, p, xshape, shapes = ctx.keep
        dev = xs.device
        g.copy_(grad_out.reshape(g.shape).float())
        grads = [torch.zeros(shp, dtype=torch.float32, device=dev) for shp in shapes]
        gs = SirenKanGrads()
        for l in range(len(shapes) // 3):
            gs.base_w[l], gs.spline_w[l], gs.scaler[l] = (ptr(t) for t in grads[3 * l:3 * l + 3])
        gx = torch.empty_like(xs) if ctx.needs_input_grad[2] else None
        check(lib.siren_kan_backward(ctypes.byref(net), ctypes.byref(gs), ctypes.byref(b), ptr(gx),
                                     torch.cuda.current_stream(dev).cuda_stream), "siren_kan_backward")
        ctx.keep = None
        return (None, None, None if gx is None else gx.reshape(xshape), *grads)


def _kan_apply(widths, layers, x, params):
    return _KanFunction.apply(list(widths), list(layers), x, *params)


class KAN(torch.nn.Module):
    """kan.py:169-285: a stack of KANLinear layers over layers_hidden widths."""

    def __init__(self, layers_hidden, grid_size=5, spline_order=3, scale_noise=0.1, scale_base=1.0,
                 scale_spline=1.0, base_activation=torch.nn.SiLU, grid_eps=0.02, grid_range=[-1, 1]):
        super().__init__()
        self.grid_size, self.spline_order = grid_size, spline_order
        self.widths = list(layers_hidden)
        self.layers = torch.nn.ModuleList(
            KANLinear(i, o, grid_size=grid_size, spline_order=spline_order, scale_noise=scale_noise,
                      scale_base=scale_base, scale_spline=scale_spline, base_activation=base_activation,
                      grid_eps=grid_eps, grid_range=grid_range)
            for i, o in zip(layers_hidden, layers_hidden[1:]))

    def hip_check(self):
        if self.grid_size != 5 or self.spline_order != 3:
            raise NotImplementedError("HIP KAN path: grid_size=5, spline_order=3 (kan.py defaults)")
        if len(self.layers) > _lib.KAN_MAX_LAYERS or self.widths[-1] != 1:
            raise NotImplementedError(f"HIP KAN path: <= {_lib.KAN_MAX_LAYERS} layers, last width 1")
        for lay in self.layers:
            _hip_check_layer(lay)

    def param_index(self):
        pos = {n: k for k, (n, _) in enumerate(self.named_parameters())}
        return [(pos[f"layers.{l}.base_weight"], pos[f"layers.{l}.spline_weight"], pos[f"layers.{l}.spline_scaler"])
                for l in range(len(self.layers))]

    def make_net(self, tensors=None) -> SirenKanNet:
        """C-ABI view of the layers; `tensors` overrides the parameters (list in
        named_parameters order, e.g. views of a flat vector)."""
        self.hip_check()
        n = SirenKanNet()
        n.n_layers = len(self.layers)
        for l, w in enumerate(self.widths):
            n.width[l] = w
        params = tensors if tensors is not None else [p for _, p in self.named_parameters()]
        for l, (ib, isp, isc) in enumerate(self.param_index()):
            n.grid[l] = ptr(self.layers[l].grid)
            n.base_w[l], n.spline_w[l], n.scaler[l] = ptr(params[ib]), ptr(params[isp]), ptr(params[isc])
        return n

    def forward(self, x: torch.Tensor, update_grid=False):
        """kan.py:268-273: (..., in) CUDA coords -> (..., out).  Differentiable when autograd needs
        it (siren_kan_forward + siren_kan_backward); chunked HIP inference otherwise."""
        if update_grid:
            raise NotImplementedError("update_grid is not on the HIP path (run.py never uses it)")
        if not x.is_cuda:
            raise RuntimeError("KAN.forward runs on the HIP path only (CUDA tensors)")
        self.hip_check()
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            params = [t for lay in self.layers for t in (lay.base_weight, lay.spline_weight, lay.spline_scaler)]
            return _kan_apply(self.widths, self.layers, x, params)
        lead = x.shape[:-1]
        with torch.no_grad():
            out = kan_forward(self, x.reshape(-1, self.widths[0]), x.device)
        return out.reshape(*lead, 1)


def kan_forward(model: KAN, coords: torch.Tensor, device, chunk: int = 1 << 20, net=None) -> torch.Tensor:
    lib = _lib.load()
    net = net or model.make_net()
    n = coords.shape[0]
    rows = max(1, min(chunk, n))
    ws = torch.empty(int(lib.siren_kan_workspace_floats(ctypes.byref(net), rows, 1)), device=device)
    out = torch.empty(n, dtype=torch.float32, device=device)
    g = torch.empty(rows, dtype=torch.float32, device=device)
    o = torch.empty(rows, dtype=torch.float32, device=device)
    s = torch.cuda.current_stream(device).cuda_stream
    for lo in range(0, n, rows):
        hi = min(n, lo + rows)
        c = coords[lo:hi].to(device, torch.float32).contiguous()
        b = SirenKanBatch()
        b.rows, b.n_valid, b.n_total, b.splits, b.zero_grads = hi - lo, 0, 1.0, 1, 0
        b.coords, b.target, b.out, b.g, b.ws = ptr(c), 0, ptr(o), ptr(g), ptr(ws)
        check(lib.siren_kan_forward(ctypes.byref(net), ctypes.byref(b), s), "siren_kan_forward")
        out[lo:hi] = o[:hi - lo]
    return out


def make_kan_grads(model: KAN, views, sse_ptr: int, flat: torch.Tensor, flat_len: int) -> SirenKanGrads:
    g = SirenKanGrads()
    for l, (ib, isp, isc) in enumerate(model.param_index()):
        g.base_w[l], g.spline_w[l], g.scaler[l] = ptr(views[ib]), ptr(views[isp]), ptr(views[isc])
    g.sse, g.flat, g.flat_len = sse_ptr, ptr(flat), flat_len
    return g
