"""Device-resident SIREN training engine over the libsiren_hip C-ABI.

Replaces what run.py's hot loop (run.py:156-190) does through torch eager + autograd:
forward, MSELoss, backward, Adam, ReduceLROnPlateau.  The engine owns

* a flat fp32 parameter vector (plus grad / exp_avg / exp_avg_sq vectors of the same
  layout) whose segments the nn.Module parameters are re-pointed at, so
  ``model.state_dict()`` always shows the live weights;
* fp16 shadows W_i and W_i^T of every hidden weight (refreshed by the update kernel);
* one micro-batch workspace (fp16 activations Y_i = sin, C_i = cos, scaled fp16 dZ
  ping-pong and fp32 partial-sum slabs), reused for every micro-batch of the full-batch
  step -- fp16, not bf16: DESIGN.md "Storage precision";
* the optimizer / scheduler state as a device struct, so a step needs no host sync and
  can be captured in a HIP graph.

Data parallel: one process per GPU (torchrun), rank r owns the contiguous coordinate slice
[r*N/G, (r+1)*N/G); the MSE gradient uses the GLOBAL N and the flat gradient vector (whose
tail slot carries the summed squared error) is all-reduced once per step.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import (MAX_INNER, ROW_TILE, SirenBatch, SirenGrads, SirenKanBatch, SirenNet, SirenOptState, check,
                   ptr)

SEG_ALIGN = 64  # floats: every flat segment starts 256-B aligned
STORE16 = torch.float16  # activation / weight-shadow / dZ storage of the HIP path


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class NetSpec:
    in_dim: int
    hidden: int
    n_inner: int
    omega0: float
    omega: float
    acts: tuple = ()   # siren_act per inner layer (empty: all sine)
    first_snake: bool = False   # first_linear=True: net.0 is Linear + Snake
    head_omega: float = 0.0     # last_linear=False: final SineLayer(H, 1, head_omega)

    def act(self, i: int) -> int:
        return self.acts[i] if self.acts else _lib.ACT_SINE


def net_spec(model) -> NetSpec:
    """Validate that `model` is a SirenWithSnakeTanh configuration the HIP path implements."""
    spec = getattr(model, "hip_spec", None)
    if spec is None:
        raise TypeError("expected inr_for_audio_amd.models.SirenWithSnakeTanh")
    return spec()


class ParamLayout:
    """Offsets of every parameter (named_parameters order == state_dict order == the
    order torch.optim.Adam indexes its state) inside the flat fp32 vectors.

    `pad` ({parameter index: (stored shape, fill value)}) stores a parameter zero-padded to the
    width the kernels run at (a hidden width that is not 128/256/512/1024 runs as the next one
    of those; models.SirenWithSnakeTanh.hip_padding): `view` is the stored (padded) tensor the
    C-ABI binds, `true_view` the model's own [:h, ...] block of it.  Pad entries start at their
    fill value (0, or 1 for a Snake a) and their gradients are exactly zero, so Adam never moves
    them and the padded network computes the unpadded one's function and gradients."""

    def __init__(self, model, pad: dict | None = None):
        pad = pad or {}
        self.names, self.shapes, self.offsets, self.numels = [], [], [], []
        self.true_shapes, self.fills = [], []
        off = 0
        for i, (name, p) in enumerate(model.named_parameters()):
            shp, fill = pad.get(i, (tuple(p.shape), 0.0))
            assert len(shp) == p.dim() and all(a >= b for a, b in zip(shp, p.shape)), (name, shp)
            self.names.append(name)
            self.shapes.append(tuple(shp))
            self.true_shapes.append(tuple(p.shape))
            self.fills.append(float(fill))
            self.offsets.append(off)
            self.numels.append(math.prod(shp))
            off = round_up(off + self.numels[-1], SEG_ALIGN)
        self.n_params = off                   # Adam runs over [0, n_params)
        self.sse_offset = off                 # summed squared error rides the all-reduce
        self.flat_len = off + SEG_ALIGN

    def view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        o = self.offsets[i]
        return flat[o:o + self.numels[i]].view(self.shapes[i])

    def true_view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        v = self.view(flat, i)
        if self.shapes[i] == self.true_shapes[i]:
            return v
        return v[tuple(slice(0, d) for d in self.true_shapes[i])]

    def fill_pads(self, flat: torch.Tensor) -> None:
        """Every padded parameter's stored tensor to its fill value (the model block is then
        copied over it)."""
        for i, f in enumerate(self.fills):
            if self.shapes[i] != self.true_shapes[i]:
                self.view(flat, i).fill_(f)


class Workspace:
    """Activations + scratch for `rows` coordinates (rows % 128 == 0).

    Training keeps every layer's Y / C (and Snake E) for the backward.  Inference
    (train=False) needs only the layer input and output at a time: Y ping-pongs between two
    buffers and every C / E points at one write-only scratch buffer, so an inference
    workspace is 3-4 activation buffers whatever the depth."""

    def __init__(self, spec: NetSpec, rows: int, device, train: bool = True, splits: int | None = None):
        lib = _lib.load()
        if rows % ROW_TILE:
            raise ValueError(f"rows={rows} must be a multiple of {ROW_TILE}")
        H, L, R = spec.hidden, spec.n_inner, rows
        h, f32 = STORE16, torch.float32
        e = lambda *s, dtype=f32: torch.empty(*s, dtype=dtype, device=device)  # noqa: E731
        self.rows = R
        if train:
            self.Y = [e(R, H, dtype=h) for _ in range(L + 1)]
            self.C = [e(R, H, dtype=h) for _ in range(L + 1)]
            # dY/da of Snake layers (E[i+1] for inner layer i)
            self.E = [e(R, H, dtype=h) if spec.first_snake else None] + \
                [e(R, H, dtype=h) if spec.act(i) == _lib.ACT_SNAKE else None for i in range(L)]
        else:
            ping = [e(R, H, dtype=h), e(R, H, dtype=h)]
            scratch = e(R, H, dtype=h)
            self.Y = [ping[i % 2] for i in range(L + 1)]
            self.C = [scratch] * (L + 1)
            snake = spec.first_snake or any(spec.act(i) == _lib.ACT_SNAKE for i in range(L))
            escr = e(R, H, dtype=h) if snake else None
            self.E = [escr if spec.first_snake else None] + \
                [escr if spec.act(i) == _lib.ACT_SNAKE else None for i in range(L)]
        self.out = e(R)
        self.g = torch.zeros(R, dtype=f32, device=device)
        self.head_part = e(H // 128, R)
        nsum = (R + 255) // 256
        self.sse_part = e(nsum)
        self.gsum_part = e(nsum)
        self.gmax_part = e(nsum)
        self.gscale = torch.ones(2, dtype=f32, device=device)
        # this workspace's tile-queue counters: its launches are ordered on one stream
        self.tileq = _lib.new_tileq(device)
        self.train = train
        if train:
            self.splits = int(splits or lib.siren_default_splits(R, H))
            self.dZ = [e(R, H, dtype=h) for _ in range(2)]
            self.col_part = e(R // 128, max(2 + spec.in_dim, 2), H)
            self.col_part2 = e(R // 128, H)
            self.red_tmp = e(4, 64, H)  # ABI 10: up to 4 column reductions per launch pair
            self.slab = e(int(lib.siren_slab_floats(H, self.splits)))
        else:
            self.splits = 1
            self.dZ = [None, None]
            self.col_part = self.col_part2 = self.red_tmp = self.slab = None

    def batch(self, coords: torch.Tensor, target, n_valid: int, n_total: float,
              zero_grads: bool = False, guard: torch.Tensor | None = None, loss_mode: int = 0) -> SirenBatch:
        b = SirenBatch()
        b.rows, b.n_valid, b.n_total = self.rows, int(n_valid), float(n_total)
        b.splits, b.zero_grads = self.splits, int(zero_grads)
        b.guard, b.loss_mode = ptr(guard), int(loss_mode)
        b.coords, b.target = ptr(coords), ptr(target)
        for i, y in enumerate(self.Y):
            b.Y[i] = ptr(y)
        for i, c in enumerate(self.C):
            b.C[i] = ptr(c)
        for i, x in enumerate(self.E):
            b.E[i] = ptr(x)
        b.dZ[0], b.dZ[1] = ptr(self.dZ[0]), ptr(self.dZ[1])
        b.out, b.g, b.head_part = ptr(self.out), ptr(self.g), ptr(self.head_part)
        b.sse_part, b.gsum_part = ptr(self.sse_part), ptr(self.gsum_part)
        b.gmax_part, b.gscale = ptr(self.gmax_part), ptr(self.gscale)
        b.col_part, b.col_part2 = ptr(self.col_part), ptr(self.col_part2)
        b.red_tmp, b.slab = ptr(self.red_tmp), ptr(self.slab)
        b.tileq = ptr(self.tileq)
        return b


def make_net(spec: NetSpec, W0, b0, bs, Whs, WThs, w_head, b_head, snake_a=None, a0=None) -> SirenNet:
    n = SirenNet()
    n.in_dim, n.hidden, n.n_inner = spec.in_dim, spec.hidden, spec.n_inner
    n.omega0, n.omega = spec.omega0, spec.omega
    n.W0, n.b0 = ptr(W0), ptr(b0)
    for i in range(spec.n_inner):
        n.b[i], n.Wh[i], n.WTh[i] = ptr(bs[i]), ptr(Whs[i]), ptr(WThs[i])
        n.act[i] = spec.act(i)
        if snake_a is not None and snake_a[i] is not None:
            n.a[i] = ptr(snake_a[i])
    n.w_head, n.b_head = ptr(w_head), ptr(b_head)
    n.first_snake = int(spec.first_snake)
    n.a0 = ptr(a0)
    n.head_omega = float(spec.head_omega)
    return n


def make_grads(spec: NetSpec, layout: ParamLayout, gflat: torch.Tensor, ix: dict) -> SirenGrads:
    """Gradient destinations: views of `gflat` at the positions of model.param_index()."""
    g = SirenGrads()
    v = lambda i: layout.view(gflat, i)  # noqa: E731
    L = spec.n_inner
    g.W0, g.b0 = ptr(v(ix["W0"])), ptr(v(ix["b0"]))
    for i in range(L):
        g.W[i], g.b[i] = ptr(v(ix["W"][i])), ptr(v(ix["b"][i]))
        if ix["a"][i] is not None:
            g.a[i] = ptr(v(ix["a"][i]))
    g.w_head, g.b_head = ptr(v(ix["wh"])), ptr(v(ix["bh"]))
    if ix.get("a0") is not None:
        g.a0 = ptr(v(ix["a0"]))
    g.sse = gflat.data_ptr() + 4 * layout.sse_offset
    g.flat, g.flat_len = ptr(gflat), layout.flat_len
    return g


def cast_shadows(spec, Ws, Whs, WThs, stream):
    lib = _lib.load()
    for W, Wh, WTh in zip(Ws, Whs, WThs):
        check(lib.siren_cast_weight(ptr(W), spec.hidden, spec.hidden, ptr(Wh), ptr(WTh), stream),
              "siren_cast_weight")


LOSS_MODES = {"mse": 0, "mae": 1}   # run.py:161-169 (MSELoss / L1Loss)


def new_guard(device) -> torch.Tensor:
    """A zeroed siren_guard with the default headroom (include/siren_hip.h): flag, headroom, clean,
    overflows, headroom0, stalls."""
    g = torch.zeros(6, dtype=torch.int32)
    g[1] = g[4] = _lib.HEADROOM0
    return g.to(device)


def _dist():
    d = torch.distributed
    if d.is_available() and d.is_initialized() and d.get_world_size() > 1:
        return d
    return None


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous coordinate slice owned by `rank`."""
    return n_total * rank // world, n_total * (rank + 1) // world


class SirenEngine:
    """Full-batch SIREN fit on one GPU (or one DP rank): run.py:108-190 minus the plots.

    Data parallel (torch.distributed initialised, world > 1): the gradients are all-reduced in
    per-layer buckets on a communication stream, each as soon as the backward has finalised it
    (siren_batch.grad_ready events), so RCCL runs under the remaining backward GEMMs."""

    _buckets = None  # [(event index, lo, hi)] in completion order (DP only)
    # bench.py's exposed-communication measurement only: False skips the gradient all-reduce (the
    # ranks' parameters then drift apart -- timing passes after the measured run, never training)
    comm_enabled = True

    def __init__(self, model, coords: torch.Tensor, target: torch.Tensor, *, lr: float = 1e-3,
                 min_lr: float = 1e-6, factor: float = 0.8, patience: int = 200,
                 n_total: int | None = None, micro_batch: int = 1 << 20, hist_cap: int = 20000,
                 splits: int | None = None, device=None, loss_mode: str = "mse"):
        lib = _lib.load()
        self.lib = lib
        if loss_mode not in LOSS_MODES:
            raise NotImplementedError(f"loss_mode={loss_mode!r}: the HIP path has {sorted(LOSS_MODES)}")
        self.device = torch.device(device or "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("SirenEngine runs on the GPU only (HIP kernels; no CPU fallback)")
        self.model = model
        self.spec = spec = net_spec(model)
        self.layout = lay = ParamLayout(model, model.hip_padding())
        dev = self.device

        # flat fp32 parameter storage; module parameters become views into it (the model's own
        # blocks of the padded tensors when the hidden width is padded)
        self.params = torch.zeros(lay.flat_len, dtype=torch.float32, device=dev)
        with torch.no_grad():
            lay.fill_pads(self.params)
            for i, (_, p) in enumerate(model.named_parameters()):
                lay.true_view(self.params, i).copy_(p.detach().to(dev, torch.float32))
        d = _dist()
        if d is not None:
            d.broadcast(self.params, src=0)
        for i, (_, p) in enumerate(model.named_parameters()):
            p.data = lay.true_view(self.params, i)
        self.grads = torch.zeros_like(self.params)
        self.exp_avg = torch.zeros_like(self.params)
        self.exp_avg_sq = torch.zeros_like(self.params)

        L, H = spec.n_inner, spec.hidden
        self.ix = ix = model.param_index()
        pv = lambda i: lay.view(self.params, i)  # noqa: E731
        self.W = [pv(k) for k in ix["W"]]
        self.Wh = [torch.empty(H, H, dtype=STORE16, device=dev) for _ in range(L)]
        self.WTh = [torch.empty(H, H, dtype=STORE16, device=dev) for _ in range(L)]
        self.net = make_net(spec, pv(ix["W0"]), pv(ix["b0"]), [pv(k) for k in ix["b"]], self.Wh, self.WTh,
                            pv(ix["wh"]), pv(ix["bh"]), [None if k is None else pv(k) for k in ix["a"]],
                            None if ix["a0"] is None else pv(ix["a0"]))
        self.grad_struct = make_grads(spec, lay, self.grads, ix)
        self._Wp = (ctypes.c_void_p * L)(*[ptr(w) for w in self.W])
        self._Whp = (ctypes.c_void_p * L)(*[ptr(w) for w in self.Wh])
        self._WThp = (ctypes.c_void_p * L)(*[ptr(w) for w in self.WTh])

        # optimizer + scheduler state (torch defaults of run.py:116-117)
        st = SirenOptState()
        st.lr, st.best, st.step = float(lr), math.inf, 0.0
        st.num_bad, st.last_epoch = 0, 0
        st.min_lr, st.factor, st.threshold, st.eps_lr = float(min_lr), float(factor), 1e-4, 1e-8
        st.patience = int(patience)
        st.beta1, st.beta2, st.eps = 0.9, 0.999, 1e-8
        self.state = torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)
        self.hist_cap = int(hist_cap)
        self.loss_hist = torch.zeros(max(self.hist_cap, 1), dtype=torch.float32, device=dev)
        self.lr_hist = torch.zeros(max(self.hist_cap, 1), dtype=torch.float64, device=dev)

        # data: this rank's contiguous shard, padded per micro-batch
        coords = coords.reshape(-1, spec.in_dim).to(torch.float32)
        target = target.reshape(-1).to(torch.float32)
        n_global = coords.shape[0] if n_total is None else int(n_total)
        rank, world = (d.get_rank(), d.get_world_size()) if d is not None else (0, 1)
        if n_total is None and world > 1:
            lo, hi = shard_range(n_global, rank, world)
            coords, target = coords[lo:hi], target[lo:hi]
        self.n_total = n_global
        self.n_local = n = coords.shape[0]
        # rows padded to 256 (pad rows carry g = 0): the 256x256 GEMM tiles need M % 256 == 0,
        # the 128-row minimum of the C-ABI would drop a 3.6 M-row shard to the 128x128 kernels
        mb = min(round_up(int(micro_batch), 2 * ROW_TILE), round_up(max(n, 1), 2 * ROW_TILE))
        self.rows = mb
        self.n_micro = max(1, -(-n // mb))
        padded = self.n_micro * mb
        self.coords = torch.zeros(padded, spec.in_dim, dtype=torch.float32, device=dev)
        self.target = torch.zeros(padded, dtype=torch.float32, device=dev)
        self.coords[:n] = coords.to(dev)
        self.target[:n] = target.to(dev)
        self.ws = Workspace(spec, mb, dev, train=True, splits=splits)
        self.guard = new_guard(dev)
        self.batches = []
        # max|g| partials per micro-batch: a fused Snake last layer takes its backward scale from the
        # partials of the previous launch over the SAME rows (siren_batch.head_scale_prev), i.e. this
        # micro-batch's in the previous step -- with one shared slice it would be the previous
        # micro-batch's, and a quiet segment after a loud one would drop its dZ into fp16 subnormals
        nsum = (mb + 255) // 256
        self._gmax = torch.zeros(self.n_micro, nsum, dtype=torch.float32, device=dev)
        for k in range(self.n_micro):
            lo = k * mb
            c = self.coords[lo:lo + mb]
            t = self.target[lo:lo + mb]
            b = self.ws.batch(c, t, min(mb, n - lo), n_global, zero_grads=(k == 0),
                              guard=self.guard, loss_mode=LOSS_MODES[loss_mode])
            b.gmax_part = ptr(self._gmax[k])
            self.batches.append(b)
        self.steps_done = 0
        self.graph = None
        if d is not None:
            self._setup_buckets()
        self._refresh_shadows()

    def _setup_buckets(self):
        """One bucket per layer (contiguous in the flat layout): the head (+ the SSE tail slot),
        inner layers L-1 .. 0, then the first layer -- the order the backward finalises them."""
        lay, ix, L = self.layout, self.ix, self.spec.n_inner
        span = lambda ids: (lay.offsets[min(ids)], lay.offsets[max(ids)] + lay.numels[max(ids)])  # noqa: E731
        order = [(L + 1, lay.offsets[ix["wh"]], lay.flat_len)]
        for i in range(L - 1, -1, -1):
            ids = [ix["W"][i], ix["b"][i]] + ([ix["a"][i]] if ix["a"][i] is not None else [])
            order.append((i,) + span(ids))
        order.append((L,) + span([ix["W0"], ix["b0"]] + ([ix["a0"]] if ix["a0"] is not None else [])))
        self._events = []
        with torch.cuda.device(self.device):  # events of the engine's device, whatever is current
            for _ in range(L + 2):
                ev = torch.cuda.Event()
                # materialise the hipEvent_t so its handle can go to the C-ABI
                ev.record(torch.cuda.current_stream(self.device))
                self._events.append(ev)
        last = self.batches[-1]
        for k, ev in enumerate(self._events):
            last.grad_ready[k] = ev.cuda_event
        self._comm = torch.cuda.Stream(self.device)
        self._buckets = order

    # ------------------------------------------------------------------ internals
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _refresh_shadows(self):
        cast_shadows(self.spec, self.W, self.Wh, self.WTh, self._stream())

    def _launch_grads(self):
        s = self._stream()
        for b in self.batches:
            check(self.lib.siren_train_step(ctypes.byref(self.net), ctypes.byref(self.grad_struct),
                                            ctypes.byref(b), s), "siren_train_step")
        # every micro-batch's gmax_part now holds its launch's max|g| partials: from the next step on
        # a Snake last layer may run fused with the head, its backward scale taken from them
        # (include/siren_hip.h siren_batch.head_scale_prev).  Not while capturing a graph: nothing
        # has run, and the graph would record the unfused launch for good (capture_graph)
        if not torch.cuda.is_current_stream_capturing():
            for b in self.batches:
                b.head_scale_prev = 1

    def _launch_update(self):
        check(self.lib.siren_apply_update(
            ctypes.byref(self.net), ptr(self.params), ptr(self.grads), ptr(self.exp_avg),
            ptr(self.exp_avg_sq), self.layout.n_params, self._Wp, self._Whp, self._WThp,
            ptr(self.state), self.grads.data_ptr() + 4 * self.layout.sse_offset, float(self.n_total),
            ptr(self.loss_hist), ptr(self.lr_hist), self.hist_cap, ptr(self.guard), self._stream()),
            "siren_apply_update")

    # ------------------------------------------------------------------ public API
    def step(self):
        """One optimizer step over the full batch (all micro-batches, all ranks)."""
        if self.graph is not None:
            self.graph.replay()
        else:
            self._launch_grads()
            d = _dist() if self.comm_enabled else None
            if d is not None and self._buckets is not None:
                # bucket k goes out as soon as the backward recorded grad_ready[k]
                works = []
                with torch.cuda.stream(self._comm):
                    for k, lo, hi in self._buckets:
                        self._comm.wait_event(self._events[k])
                        works.append(d.all_reduce(self.grads[lo:hi], async_op=True))
                for w in works:
                    w.wait()
                torch.cuda.current_stream(self.device).wait_stream(self._comm)
            elif d is not None:
                d.all_reduce(self.grads)
            self._launch_update()
        self.steps_done += 1

    def capture_graph(self, warmup: int = 0):
        """Capture one whole step as a HIP graph (single-process only).

        The graph replays the launch configuration of the capture.  A stack whose last inner layer
        is a Snake runs that layer fused with the head only once a step has run (its backward scale
        comes from the previous launch's max|g|), so capturing before any step records the unfused
        launches for the whole run: run one step first (warmup >= 1, or step() as run.train does);
        this case warns."""
        if _dist() is not None:
            raise RuntimeError("graph capture is for the single-GPU path")
        for _ in range(warmup):
            self.step()
        if self.steps_done == 0 and self.spec.act(self.spec.n_inner - 1) == _lib.ACT_SNAKE:
            import warnings
            warnings.warn("capture_graph before any step: the Snake last layer is captured unfused "
                          "(run one step first to capture the fused launch)", RuntimeWarning, stacklevel=2)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self._launch_grads()
                self._launch_update()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graph = g
        return g

    def opt_state(self) -> SirenOptState:
        return SirenOptState.from_buffer_copy(bytes(self.state.cpu().numpy().tobytes()))

    def steps_applied(self) -> int:
        """Optimizer steps taken by this engine (scheduler steps of this run); step() calls
        minus the ones the fp16 range guard rejected and recomputed (synchronises).  Raises
        SirenError if a fused last layer's hand-off timed out since the last clear_stalls()."""
        self.guard_state()
        return int(self.opt_state().last_epoch)

    def guard_state(self) -> dict:
        """{'headroom', 'overflows', 'clean', 'stalls'} of the fp16 backward range guard
        (synchronises).  Raises SirenError when `stalls` is non-zero: a fused last layer's band
        hand-off gave up waiting for a partner (include/siren_hip.h siren_guard), so that step's
        loss and gradients were void and its update was skipped -- parameters and optimizer state
        are those of before it.  clear_stalls() re-arms the guard."""
        if getattr(self, "guard", None) is None:
            return {"headroom": None, "overflows": 0, "clean": 0, "stalls": 0}
        g = self.guard.cpu().tolist()
        if g[5]:
            raise _lib.SirenError(
                f"fused last layer: {g[5]} hand-off wait(s) timed out (a band partner never published its "
                "head partial -- CUs held by other work?); the step was voided and not applied. "
                "Call clear_stalls() to train on, or set SIREN_OPT_HEAD_FUSE 0")
        return {"headroom": g[1], "overflows": g[3], "clean": g[2], "stalls": g[5]}

    def clear_stalls(self) -> None:
        """Zero the guard's hand-off stall counter (after guard_state() raised)."""
        self.guard[5] = 0

    def run(self, steps: int) -> None:
        """`steps` optimizer steps: step() calls, plus one more for each step the fp16 range
        guard rejected (checked once at the end -- no per-step host synchronisation)."""
        start = self.steps_applied()
        for _ in range(steps):
            self.step()
        while self.steps_applied() - start < steps:
            self.step()

    def history(self):
        """(losses, lrs) of the optimizer steps applied so far (host copies)."""
        k = min(self.steps_applied(), self.hist_cap)
        return self.loss_hist[:k].cpu().numpy(), self.lr_hist[:k].cpu().numpy()

    def last_loss(self) -> float:
        k = min(self.steps_applied(), self.hist_cap) - 1
        return float(self.loss_hist[k].item()) if k >= 0 else float("nan")

    def grad_views(self):
        """The gradient of every parameter, in the model's own shapes (named_parameters order)."""
        return [self.layout.true_view(self.grads, i) for i in range(len(self.layout.names))]

    @torch.no_grad()
    def infer(self, coords: torch.Tensor, chunk: int | None = None) -> torch.Tensor:
        """model(coords) with the current weights (run.py:249-256); returns [N] fp32.  Runs
        in the training workspace (the next step recomputes every activation), so inference
        allocates nothing beyond the output."""
        chunk = chunk or self.rows
        ws = self.ws if round_up(chunk, ROW_TILE) == self.rows else None
        return forward_net(self.spec, self.net, coords.reshape(-1, self.spec.in_dim), self.device,
                           chunk, shadows_ready=True, ws=ws)

    def adam_state_dict(self):
        """torch.optim.Adam-compatible state_dict (run.py:359-362 checkpoint format)."""
        st = self.opt_state()
        state = {}
        for i in range(len(self.layout.names)):
            state[i] = {
                "step": torch.tensor(float(st.step)),
                "exp_avg": self.layout.true_view(self.exp_avg, i).detach().cpu().clone(),
                "exp_avg_sq": self.layout.true_view(self.exp_avg_sq, i).detach().cpu().clone(),
            }
        group = {"lr": float(st.lr), "betas": (st.beta1, st.beta2), "eps": st.eps, "weight_decay": 0,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "decoupled_weight_decay": False,
                 "params": list(range(len(self.layout.names)))}
        return {"state": state, "param_groups": [group]}

    def load_adam_state_dict(self, sd):
        """Resume from a reference checkpoint's optimizer_state_dict (run.py:104-105)."""
        with torch.no_grad():
            step = 0.0
            for i in range(len(self.layout.names)):
                s = sd["state"].get(i)
                if s is None:
                    continue
                shp = self.layout.true_shapes[i]
                self.layout.true_view(self.exp_avg, i).copy_(s["exp_avg"].reshape(shp))
                self.layout.true_view(self.exp_avg_sq, i).copy_(s["exp_avg_sq"].reshape(shp))
                step = float(s["step"])
            st = self.opt_state()
            st.step = step
            st.lr = float(sd["param_groups"][0]["lr"])
            self.state.copy_(torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(self.device))


def forward_net(spec: NetSpec, net: SirenNet, coords: torch.Tensor, device, chunk: int,
                shadows_ready: bool = True, ws: Workspace | None = None) -> torch.Tensor:
    """Inference through siren_forward in chunks of `chunk` rows (in `ws` when given, else
    in a ping-pong inference workspace)."""
    lib = _lib.load()
    n = coords.shape[0]
    if ws is not None:
        chunk = ws.rows
    else:
        chunk = min(round_up(chunk, ROW_TILE), round_up(max(n, 1), ROW_TILE))
        ws = Workspace(spec, chunk, device, train=False)
    out = torch.empty(n, dtype=torch.float32, device=device)
    buf = torch.zeros(chunk, spec.in_dim, dtype=torch.float32, device=device)
    s = torch.cuda.current_stream(device).cuda_stream
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        buf.zero_()
        buf[:hi - lo] = coords[lo:hi].to(device, torch.float32)
        b = ws.batch(buf, None, 0, 1.0)
        check(lib.siren_forward(ctypes.byref(net), ctypes.byref(b), s), "siren_forward")
        out[lo:hi] = ws.out[:hi - lo]
    return out


def _opt_state_tensor(lr, min_lr, factor, patience, dev) -> torch.Tensor:
    """siren_opt_state for torch.optim.Adam(lr) + ReduceLROnPlateau(min, factor, patience,
    min_lr) with torch's defaults (run.py:116-117), as device bytes."""
    st = SirenOptState()
    st.lr, st.best, st.step = float(lr), math.inf, 0.0
    st.num_bad, st.last_epoch = 0, 0
    st.min_lr, st.factor, st.threshold, st.eps_lr = float(min_lr), float(factor), 1e-4, 1e-8
    st.patience = int(patience)
    st.beta1, st.beta2, st.eps = 0.9, 0.999, 1e-8
    return torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)


class KanEngine(SirenEngine):
    """Full-batch fit of the KAN variant (run.py:92-93 arch='kan') on the HIP
    path: siren_kan_train_step per micro-batch, gradient all-reduce across DP ranks, then the
    same flat Adam + ReduceLROnPlateau kernels as the SIREN path.  Shares the optimizer,
    history, checkpoint and graph-capture methods of SirenEngine."""

    def __init__(self, model, coords: torch.Tensor, target: torch.Tensor, *, lr: float = 1e-3,
                 min_lr: float = 1e-6, factor: float = 0.8, patience: int = 200,
                 n_total: int | None = None, micro_batch: int = 1 << 20, hist_cap: int = 20000,
                 splits: int | None = None, device=None):
        from .kan import make_kan_grads
        lib = _lib.load()
        self.lib = lib
        self.device = dev = torch.device(device or "cuda")
        if dev.type != "cuda":
            raise RuntimeError("KanEngine runs on the GPU only (HIP kernels; no CPU fallback)")
        model.hip_check()
        self.model = model.to(dev)
        self.spec = None
        self.layout = lay = ParamLayout(model)
        self.params = torch.zeros(lay.flat_len, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for i, (_, p) in enumerate(model.named_parameters()):
                lay.view(self.params, i).copy_(p.detach().to(dev, torch.float32))
        d = _dist()
        if d is not None:
            d.broadcast(self.params, src=0)
        for i, (_, p) in enumerate(model.named_parameters()):
            p.data = lay.view(self.params, i)
        self.grads = torch.zeros_like(self.params)
        self.exp_avg = torch.zeros_like(self.params)
        self.exp_avg_sq = torch.zeros_like(self.params)
        views = [lay.view(self.params, i) for i in range(len(lay.names))]
        gviews = [lay.view(self.grads, i) for i in range(len(lay.names))]
        self.net = model.make_net(views)
        self.grad_struct = make_kan_grads(model, gviews, self.grads.data_ptr() + 4 * lay.sse_offset,
                                          self.grads, lay.flat_len)
        self.state = _opt_state_tensor(lr, min_lr, factor, patience, dev)
        self.hist_cap = int(hist_cap)
        self.loss_hist = torch.zeros(max(self.hist_cap, 1), dtype=torch.float32, device=dev)
        self.lr_hist = torch.zeros(max(self.hist_cap, 1), dtype=torch.float64, device=dev)

        in_dim = model.widths[0]
        coords = coords.reshape(-1, in_dim).to(torch.float32)
        target = target.reshape(-1).to(torch.float32)
        n_global = coords.shape[0] if n_total is None else int(n_total)
        rank, world = (d.get_rank(), d.get_world_size()) if d is not None else (0, 1)
        if n_total is None and world > 1:
            lo, hi = shard_range(n_global, rank, world)
            coords, target = coords[lo:hi], target[lo:hi]
        self.n_total = n_global
        self.n_local = n = coords.shape[0]
        self.rows = mb = max(1, min(int(micro_batch), n))
        self.n_micro = max(1, -(-n // mb))
        self.coords = coords.to(dev).contiguous()
        self.target = target.to(dev).contiguous()
        # split-K of the weight-gradient GEMMs (K = coordinates): ~2048 rows per slice keeps
        # ~9 x 200 blocks busy at 441 000 rows (16 slices left 144 blocks: 5.9 ms per launch)
        self.splits = int(splits) if splits else max(1, min(256, mb // 2048))
        self.ws = torch.empty(int(lib.siren_kan_workspace_floats(ctypes.byref(self.net), mb, self.splits)),
                              device=dev)
        self.out = torch.empty(mb, device=dev)
        self.g = torch.empty(mb, device=dev)
        self.batches = []
        for k in range(self.n_micro):
            lo = k * mb
            hi = min(n, lo + mb)
            b = SirenKanBatch()
            b.rows, b.n_valid, b.n_total = hi - lo, hi - lo, float(n_global)
            b.splits, b.zero_grads = self.splits, int(k == 0)
            b.coords, b.target = self.coords[lo:hi].data_ptr(), self.target[lo:hi].data_ptr()
            b.out, b.g, b.ws = ptr(self.out), ptr(self.g), ptr(self.ws)
            self.batches.append(b)
        self.steps_done = 0
        self.graph = None

    def _refresh_shadows(self):
        pass

    def _launch_grads(self):
        s = self._stream()
        for b in self.batches:
            check(self.lib.siren_kan_train_step(ctypes.byref(self.net), ctypes.byref(self.grad_struct),
                                                ctypes.byref(b), s), "siren_kan_train_step")

    def _launch_update(self):
        s = self._stream()
        check(self.lib.siren_adam_step(ptr(self.params), ptr(self.grads), ptr(self.exp_avg), ptr(self.exp_avg_sq),
                                       self.layout.n_params, ptr(self.state), s), "siren_adam_step")
        check(self.lib.siren_plateau_step(ptr(self.state), self.grads.data_ptr() + 4 * self.layout.sse_offset,
                                          float(self.n_total), ptr(self.loss_hist), ptr(self.lr_hist),
                                          self.hist_cap, s), "siren_plateau_step")

    @torch.no_grad()
    def infer(self, coords: torch.Tensor, chunk: int | None = None) -> torch.Tensor:
        from .kan import kan_forward
        return kan_forward(self.model, coords.reshape(-1, self.model.widths[0]), self.device,
                           chunk or self.rows, net=self.net)
