"""CPU ORACLE for the SIREN hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline.  The product package
(inr-for-audio_amd/) never imports it.

A numpy restatement of the reference algorithm (senyuanfan/inr-for-audio):
  * get_coord / torch.linspace                utils.py:99-109
  * WaveformFitting target normalisation      utils.py:111-149
  * SineLayer / SirenWithSnakeTanh forward    models.py:114-115, 388-394
  * Linear + Snake / Linear + Tanh layers       models.py:235-241, 356-372
  * MSELoss / L1Loss + autograd backward       run.py:124-125,161-168,185
  * MultiWaveformFitting (t, ch) grid           utils.py:186-231
  * torch.optim.Adam step                     run.py:116,186
  * ReduceLROnPlateau(min, 0.8, 200)          run.py:117,187
  * calculate_snr + run.py's reported SNR     utils.py:77-97, run.py:302-335

Pinned against golden vectors generated from the reference itself (tests/golden/,
made by tests/golden/make_golden.py, which imports /root/reference in the build
container); see tests/test_oracle.py.

Precision model: `dtype=np.float64` gives the exact-arithmetic answer; `half=True`
rounds exactly the tensors the HIP path stores in fp16 (hidden weights, Y_i = sin,
C_i = cos, and dZ_i multiplied by the power-of-two backward scale S of grad_scale()) so
the GPU can be checked tightly against it.  `bf16_round` is kept for the precision study
(tools/fit_torch_diag.py, DESIGN.md "Storage precision").
"""
from __future__ import annotations

import math

import numpy as np
from scipy.signal import decimate

F32 = np.float32
F64 = np.float64


# ------------------------------------------------------------------ numerics helpers
def bf16_round(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even to bf16, returned as float32 (v_cvt_pk_bf16_f32 semantics)."""
    x = np.ascontiguousarray(x, dtype=F32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(F32).copy()
    nan = np.isnan(x)
    out[nan] = x[nan]
    return out


def f16_round(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even to IEEE fp16 (v_cvt_f16_f32 semantics), returned as float32."""
    return np.asarray(x, F32).astype(np.float16).astype(F32)


def grad_scale(g: np.ndarray, wf: np.ndarray, omega: float, headroom: int = 6) -> float:
    """elementwise.hip grad_scale_kernel: S = 2^(headroom-e) with max|g|*max|w_head|*|omega| in
    [2^(e-1), 2^e) (fp32 product), k clamped to [-100, 100]; S = 1 if the bound is 0.
    `headroom` is 6 unless the fp16 range guard lowered it (siren_guard)."""
    bound = F32(F32(np.max(np.abs(np.asarray(g, F32)))) * F32(np.max(np.abs(np.asarray(wf, F32)))))
    bound = F32(bound * F32(abs(omega)))
    if not (bound > 0 and np.isfinite(bound)):
        return 1.0
    _, e = math.frexp(float(bound))
    return math.ldexp(1.0, int(min(max(headroom - e, -100), 100)))


def grad_scale_bound(y: np.ndarray, n_valid: int, wf: np.ndarray, bf: float, n_total: float, act_bound: float,
                     head_omega: float = 0.0, loss_mode: int = 0, headroom: int = 6) -> float:
    """elementwise.hip grad_scale_bound_kernel -- the backward scale of siren_train_step's fused
    head (gemm_nt.hip NT_FWD_HB), fixed before the forward from a bound of max|g|:
    MSE gfac ((head_omega > 0 ? 1 : sum|w_head| + |b_head|) + max|y|), L1 gfac, times head_omega
    through a final sine; times max|w_head| |act_bound| (1 + 2^-10), then S = 2^(headroom-e) as
    grad_scale.  A different power-of-two S changes no stored dZ bit unless a value leaves fp16's
    normal range, so the oracle's default (grad_scale of the step's max|g|) agrees with the fused
    path to within subnormal rounding; tests of the fused path pass this S to backward(scale=)."""
    gfac = F32((1.0 if loss_mode == 1 else 2.0) / n_total)
    yv = np.abs(np.asarray(y, F32).reshape(-1)[:n_valid])
    ym = F32(yv.max()) if yv.size else F32(0)
    wa = np.abs(np.asarray(wf, F32).reshape(-1))
    wm, ws = F32(wa.max()), F32(wa.astype(F64).sum())
    if loss_mode == 1:
        gb = gfac
    else:
        gb = F32(gfac * F32((F32(1) if head_omega > 0 else F32(ws + F32(abs(float(bf))))) + ym))
    if head_omega > 0:
        gb = F32(gb * F32(head_omega))
    bound = F32(F32(F32(gb * wm) * F32(abs(act_bound))) * F32(1.0 + 2.0 ** -10))
    if not (bound > 0 and np.isfinite(bound)):
        return 1.0
    _, e = math.frexp(float(bound))
    return math.ldexp(1.0, int(min(max(headroom - e, -100), 100)))


def fma32(a, b, c) -> np.ndarray:
    """fp32 fused multiply-add: a*b is exact in fp64, one rounding of the sum to fp32
    (double rounding through fp64 differs from a true fma in < 2^-29 of cases)."""
    return (np.asarray(a, F64) * np.asarray(b, F64) + np.asarray(c, F64)).astype(F32)


# ------------------------------------------------------------------ data (utils.py)
def linspace_f32(n: int, start: float = -1.0, end: float = 1.0) -> np.ndarray:
    """torch.linspace (fp32, CPU kernel): step = (end-start)/(n-1) in fp32; i < n/2:
    fma(step, i, start), else fma(-step, n-1-i, end) -- the contracted form torch's CPU
    build produces (checked bit-exact against torch.linspace in tests/test_oracle.py)."""
    if n == 1:
        return np.array([start], F32)
    step = F32((F32(end) - F32(start)) / F32(n - 1))
    i = np.arange(n, dtype=np.int64)
    half = n // 2
    lo = fma32(step, i[:half].astype(F32), F32(start))
    hi = fma32(-step, (n - 1 - i[half:]).astype(F32), F32(end))
    return np.concatenate([lo, hi]).astype(F32)


def waveform_target(data: np.ndarray, duration: int, sample_rate: int, decimation: int = 1):
    """WaveformFitting (utils.py:111-149): trim, optional decimate, peak-normalise."""
    x = np.asarray(data).astype(F32)[0:duration * sample_rate]
    if decimation > 1:
        x = decimate(x, q=int(decimation))
    return (x / np.max(np.abs(x))).astype(F32)


# ------------------------------------------------------------------ model (models.py)
def first_keys(first_linear: bool = False):
    """(weight, bias, a-or-None) of net.0: SineLayer (net.0.linear.*) or, with first_linear,
    Linear + Snake (net.0.*, net.1.a; models.py:330-333)."""
    if first_linear:
        return "net.0.weight", "net.0.bias", "net.1.a"
    return "net.0.linear.weight", "net.0.linear.bias", None


def layer_keys(num_sine: int, num_snake: int = 0, num_tanh: int = 0, first_linear: bool = False,
               last_linear: bool = True):
    """state_dict keys of SirenWithSnakeTanh (models.py:306-386): per inner layer (kind,
    weight, bias, a-or-None), then the head's (weight, bias).  SineLayer i: net.{i}.linear.*;
    Linear+Snake: net.{j}.* + net.{j+1}.a; Linear+Tanh: net.{j}.* (net.{j+1} is the
    parameterless Tanh); the head is a Linear (net.{j}.*) or, without last_linear, a
    SineLayer (net.{j}.linear.*)."""
    layers, j = [], 2 if first_linear else 1
    for _ in range(num_sine):
        layers.append(("sine", f"net.{j}.linear.weight", f"net.{j}.linear.bias", None))
        j += 1
    for kind in ["snake"] * num_snake + ["tanh"] * num_tanh:
        layers.append((kind, f"net.{j}.weight", f"net.{j}.bias", f"net.{j + 1}.a" if kind == "snake" else None))
        j += 2
    if not last_linear:
        return layers, (f"net.{j}.linear.weight", f"net.{j}.linear.bias")
    return layers, (f"net.{j}.weight", f"net.{j}.bias")


class Params:
    """SirenWithSnakeTanh parameters in nn.Linear layout: W0 [H,in], b0 [H], W[i] [H,H],
    b[i] [H], a[i] [H] (Snake layers, else None), wf [H] (= head weight[0]), bf scalar;
    kinds[i] in {'sine', 'snake', 'tanh'}."""

    def __init__(self, W0, b0, W, b, wf, bf, kinds=None, a=None, a0=None, head_omega=0.0):
        self.W0, self.b0 = np.asarray(W0, F32), np.asarray(b0, F32)
        self.W = [np.asarray(w, F32) for w in W]
        self.b = [np.asarray(x, F32) for x in b]
        self.wf = np.asarray(wf, F32).reshape(-1)
        self.bf = F32(np.asarray(bf).reshape(-1)[0])
        self.kinds = list(kinds) if kinds is not None else ["sine"] * len(self.W)
        self.a = [None if x is None else np.asarray(x, F32).reshape(-1) for x in (a or [None] * len(self.W))]
        self.a0 = None if a0 is None else np.asarray(a0, F32).reshape(-1)   # first_linear Snake a
        self.head_omega = float(head_omega)                                 # >0: final SineLayer

    def counts(self):
        return self.kinds.count("sine"), self.kinds.count("snake"), self.kinds.count("tanh")

    def keys(self):
        return layer_keys(*self.counts(), first_linear=self.a0 is not None, last_linear=self.head_omega == 0)

    @classmethod
    def from_state_dict(cls, sd: dict, n_inner: int, num_snake: int = 0, num_tanh: int = 0,
                        first_linear: bool = False, last_linear: bool = True, hidden_omega: float = 30.0):
        """n_inner = num_sine (the sine-only form) when num_snake = num_tanh = 0."""
        g = lambda k: np.asarray(sd[k], F32)  # noqa: E731
        layers, (hw, hb) = layer_keys(n_inner, num_snake, num_tanh, first_linear, last_linear)
        w0k, b0k, a0k = first_keys(first_linear)
        return cls(g(w0k), g(b0k), [g(w) for _, w, _, _ in layers],
                   [g(b) for _, _, b, _ in layers], g(hw), g(hb), [k for k, _, _, _ in layers],
                   [None if a is None else g(a) for _, _, _, a in layers],
                   None if a0k is None else g(a0k), 0.0 if last_linear else hidden_omega)

    def to_state_dict(self) -> dict:
        layers, (hw, hb) = self.keys()
        w0k, b0k, a0k = first_keys(self.a0 is not None)
        sd = {w0k: self.W0, b0k: self.b0}
        if a0k is not None:
            sd[a0k] = self.a0
        for i, (_, wk, bk, ak) in enumerate(layers):
            sd[wk] = self.W[i]
            sd[bk] = self.b[i]
            if ak is not None:
                sd[ak] = self.a[i]
        sd[hw] = self.wf.reshape(1, -1)
        sd[hb] = np.array([self.bf], F32)
        return sd

    def flat(self) -> list[np.ndarray]:
        return [np.asarray(v) for v in self.to_state_dict().values()]


def first_preact(t: np.ndarray, W0: np.ndarray, b0: np.ndarray, omega0: float) -> np.ndarray:
    """omega0 * (t W0^T + b0) in fp32 with torch-CPU addmm rounding (K=1: fma(t,w,b);
    K=2: fma(t1,w1,t0*w0)+b) then the fp32 multiply."""
    t = np.asarray(t, F32).reshape(t.shape[0], -1)
    if t.shape[1] == 1:
        z = fma32(t[:, :1], W0[None, :, 0], b0[None, :])
    else:
        p = (t[:, :1] * W0[None, :, 0]).astype(F32)
        z = (fma32(t[:, 1:2], W0[None, :, 1], p) + b0[None, :]).astype(F32)
    return (F32(omega0) * z).astype(F32)


def sin32(a: np.ndarray) -> np.ndarray:
    return np.sin(np.asarray(a, F64)).astype(F32)


def cos32(a: np.ndarray) -> np.ndarray:
    return np.cos(np.asarray(a, F64)).astype(F32)


def forward(p: Params, t: np.ndarray, omega0: float, omega: float, half: bool = False,
            dtype=F32):
    """Returns (out [N], cache).  cache: Y[0..L] (layer outputs), A[0..L] (omega*linear),
    C[0..L] cos of the pre-activations; fp16-rounded where the HIP path stores fp16."""
    if p.a0 is None:
        A0 = first_preact(t, p.W0, p.b0, omega0)
        Y0 = sin32(A0)
        C0 = cos32(A0)
        E0 = None
    else:  # first_linear: Linear + Snake (models.py:330-333, :241)
        A0 = first_preact(t, p.W0, p.b0, 1.0)
        z, av = np.asarray(A0, F64), np.asarray(p.a0, F64)[None, :]
        s0, c0 = np.sin(av * z), np.cos(av * z)
        Y0 = (z + s0 * s0 / av).astype(F32)
        C0 = (1.0 + 2.0 * s0 * c0).astype(F32)
        E0 = ((z * 2.0 * s0 * c0) / av - s0 * s0 / (av * av)).astype(F32)
        if half:
            E0 = f16_round(E0)
    Y = [f16_round(Y0) if half else Y0]
    A, C, E = [A0], [f16_round(C0) if half else C0], [E0]
    for Wi, bi, kind, ai in zip(p.W, p.b, p.kinds, p.a):
        Wm = f16_round(Wi) if half else Wi
        z = np.asarray(Y[-1], dtype) @ np.asarray(Wm, dtype).T + np.asarray(bi, dtype)
        e = None
        if kind == "sine":      # models.py:114-115
            a = (F64(omega) * np.asarray(z, F64)) if dtype == F64 else (F32(omega) * z.astype(F32))
            y, c = np.sin(a), np.cos(a)
        elif kind == "snake":   # models.py:241 and its autograd: dY/dz, dY/da
            a = np.asarray(z, F64)
            av = np.asarray(ai, F64)[None, :]
            s, cz = np.sin(av * a), np.cos(av * a)
            y = a + s * s / av
            c = 1.0 + 2.0 * s * cz
            e = (a * 2.0 * s * cz) / av - s * s / (av * av)
        else:                   # tanh, models.py:366-372
            a = np.asarray(z, F64)
            y = np.tanh(a)
            c = 1.0 - y * y
        if half:
            y, c = f16_round(y), f16_round(c)
            e = None if e is None else f16_round(e)
        A.append(a)
        Y.append(np.asarray(y, dtype if not half else F32))
        C.append(np.asarray(c, dtype if not half else F32))
        E.append(None if e is None else np.asarray(e, dtype if not half else F32))
    out = np.asarray(Y[-1], dtype) @ np.asarray(p.wf, dtype) + dtype(p.bf)
    o_lin = out
    if p.head_omega:  # last_linear=False: final SineLayer(H, 1)
        out = np.sin(np.asarray(dtype(p.head_omega) * out, F64)).astype(dtype)
    return out, {"Y": Y, "A": A, "C": C, "E": E, "o": o_lin}


def mse(out: np.ndarray, y: np.ndarray) -> float:
    d = np.asarray(out, F64) - np.asarray(y, F64).reshape(-1)
    return float(np.mean(d * d))


def backward(p: Params, t: np.ndarray, cache: dict, g: np.ndarray, omega0: float, omega: float,
             half: bool = False, dtype=F64, headroom: int = 6, scale: float | None = None) -> dict:
    """Autograd of the SIREN for upstream dLoss/dout = g [N].  Returns a dict of grads in
    nn.Linear layout (same keys as Params.to_state_dict).  With `half`, every dZ_i is
    rounded as the HIP path stores it: fp16(dZ_i * S) / S (exact power-of-two scale, S from
    grad_scale with the given `headroom`, or `scale` when given: grad_scale_bound's S of the
    fused head)."""
    L = len(p.W)
    Y, A, C, E = cache["Y"], cache["A"], cache["C"], cache.get("E", [None] * (L + 1))
    layers, (hw, hb) = p.keys()
    if p.head_omega:  # through the final sine: dLoss/do = g cos(omega o) omega
        o = np.asarray(cache["o"], F64)
        g = (np.asarray(g, F64) * np.cos(p.head_omega * o) * p.head_omega).astype(F32)
    # backward scale bound: |dY/dz| of the last layer (elementwise.hip grad_scale / capi act_bound)
    bound = {"sine": omega, "snake": 2.0, "tanh": 1.0}[p.kinds[-1]]
    S = (scale if scale is not None else grad_scale(g, p.wf, bound, headroom)) if half else 1.0
    g = np.asarray(g, dtype).reshape(-1)
    grads = {}
    grads[hw] = (g @ np.asarray(Y[L], dtype)).reshape(1, -1)
    grads[hb] = np.array([g.sum()])
    dY = g[:, None] * np.asarray(p.wf, dtype)[None, :]
    for i in range(L, 0, -1):
        kind, wk, bk, ak = layers[i - 1]
        if kind == "sine":
            cos_i = np.asarray(C[i], dtype) if half else np.cos(np.asarray(A[i], F64)).astype(dtype)
            dZ = dY * cos_i * dtype(omega)
        else:
            dZ = dY * np.asarray(C[i], dtype)
        if kind == "snake":
            grads[ak] = (dY * np.asarray(E[i], dtype)).sum(0)
        db = dZ.sum(0)
        if half:
            dZ = (np.asarray(dZ * S, F32).astype(np.float16).astype(dtype) / S).astype(dtype)
        grads[wk] = dZ.T @ np.asarray(Y[i - 1], dtype)
        grads[bk] = db
        Wm = f16_round(p.W[i - 1]) if half else p.W[i - 1]
        dY = dZ @ np.asarray(Wm, dtype)
    w0k, b0k, a0k = first_keys(p.a0 is not None)
    if p.a0 is None:
        cos0 = np.asarray(C[0], dtype) if half else np.cos(np.asarray(A[0], F64)).astype(dtype)
        dZ0 = dY * cos0 * dtype(omega0)
    else:
        dZ0 = dY * np.asarray(C[0], dtype)
        grads[a0k] = (dY * np.asarray(E[0], dtype)).sum(0)
    tt = np.asarray(t, dtype).reshape(dZ0.shape[0], -1)
    grads[w0k] = dZ0.T @ tt
    grads[b0k] = dZ0.sum(0)
    return grads


def mse_grad(out: np.ndarray, y: np.ndarray, n_total: int | None = None) -> np.ndarray:
    """MSELoss(mean) backward: (out - y) * (2/N) in fp32 (torch's norm scalar)."""
    n = out.shape[0] if n_total is None else n_total
    return ((np.asarray(out, F32) - np.asarray(y, F32).reshape(-1)) * F32(2.0 / n)).astype(F32)


def l1_grad(out: np.ndarray, y: np.ndarray, n_total: int | None = None) -> np.ndarray:
    """L1Loss(mean) backward (run.py:124, 161-163 loss_mode='mae'): sign(out - y) / N in fp32
    (torch's sign: 0 where out == y)."""
    n = out.shape[0] if n_total is None else n_total
    d = np.asarray(out, F32) - np.asarray(y, F32).reshape(-1)
    return (np.sign(d).astype(F32) * F32(1.0 / n)).astype(F32)


def l1(out: np.ndarray, y: np.ndarray) -> float:
    return float(np.mean(np.abs(np.asarray(out, F64) - np.asarray(y, F64).reshape(-1))))


def multiwave_grid(height: int, width: int) -> np.ndarray:
    """MultiWaveformFitting's (time, channel) grid (utils.py:211-220): row k =
    (linspace(-1,1,height)[k // width], ch[k % width]), ch = linspace(-1,1,width), or 0 for
    one channel.  [height*width][2] fp32."""
    t = linspace_f32(height)
    ch = np.zeros(1, F32) if width == 1 else linspace_f32(width)
    return np.stack([np.repeat(t, width), np.tile(ch, height)], axis=1).astype(F32)


# ------------------------------------------------------------------ optimizer (run.py)
def adam_step(param, grad, exp_avg, exp_avg_sq, step: int, lr: float, beta1=0.9, beta2=0.999,
              eps=1e-8):
    """torch.optim.Adam (CUDA rounding sequence, see elementwise.hip adam_flat_kernel).
    `step` is the 1-based step count after increment.  Returns new (p, m, v) fp32."""
    p, g = np.asarray(param, F32), np.asarray(grad, F32)
    m, v = np.asarray(exp_avg, F32), np.asarray(exp_avg_sq, F32)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    neg_step = F32((lr / bc1) * -1.0)
    bc2_sqrt = F32(math.sqrt(bc2))
    m = fma32(F32(1.0 - beta1), (g - m).astype(F32), m)
    v = fma32((F32(1.0 - beta2) * g).astype(F32), g, (v * F32(beta2)).astype(F32))
    d = ((np.sqrt(v).astype(F32) / bc2_sqrt).astype(F32) + F32(eps)).astype(F32)
    p = (p + ((neg_step * m).astype(F32) / d).astype(F32)).astype(F32)
    return p, m, v


class Plateau:
    """torch.optim.lr_scheduler.ReduceLROnPlateau(mode='min', factor, patience,
    threshold=1e-4 (rel), cooldown=0, min_lr, eps=1e-8)."""

    def __init__(self, lr, factor=0.8, patience=200, min_lr=1e-6, threshold=1e-4, eps=1e-8):
        self.lr, self.factor, self.patience, self.min_lr = lr, factor, patience, min_lr
        self.threshold, self.eps = threshold, eps
        self.best, self.num_bad, self.last_epoch = math.inf, 0, 0

    def step(self, loss: float) -> float:
        cur = float(loss)
        self.last_epoch += 1
        if cur < self.best * (1.0 - self.threshold):
            self.best, self.num_bad = cur, 0
        else:
            self.num_bad += 1
        if self.num_bad > self.patience:
            new_lr = max(self.lr * self.factor, self.min_lr)
            if self.lr - new_lr > self.eps:
                self.lr = new_lr
            self.num_bad = 0
        return self.lr


# ------------------------------------------------------------------ metrics (utils.py / run.py)
def calculate_snr(ref, rec) -> float:
    ref, rec = np.asarray(ref), np.asarray(rec)
    return float(10 * np.log10(np.mean(ref ** 2) / np.mean((rec - ref) ** 2)))


def reported_snr(ref_raw, fs, rec, duration, decimation=1) -> float:
    """run.py:306-335: trim, decimate(q) (a low-pass even at q=1), +1e-10, SNR."""
    ref = np.asarray(ref_raw)[:int(fs * duration)]
    ref = decimate(ref, q=int(decimation)) + 1e-10
    return calculate_snr(ref, rec)


# ------------------------------------------------------------------ full-batch fit (run.py:156-190)
def fit(p: Params, t, y, omega0, omega, steps, lr=1e-3, min_lr=1e-6, half=False):
    """Full-batch fit with the restated loop; returns (params, losses, lrs)."""
    names = list(p.to_state_dict().keys())
    counts = p.counts() + (p.a0 is not None, p.head_omega == 0, p.head_omega or 30.0)
    flat = [x.astype(F32).copy() for x in p.to_state_dict().values()]
    ms = [np.zeros_like(x) for x in flat]
    vs = [np.zeros_like(x) for x in flat]
    sched = Plateau(lr, min_lr=min_lr)
    losses, lrs = [], []
    L = len(p.W)
    for k in range(1, steps + 1):
        cur = Params.from_state_dict(dict(zip(names, flat)), *counts)
        out, cache = forward(cur, t, omega0, omega, half=half)
        loss = F32(mse(out, y))
        grads = backward(cur, t, cache, mse_grad(out, y), omega0, omega, half=half)
        for j, nme in enumerate(names):
            flat[j], ms[j], vs[j] = adam_step(flat[j], grads[nme].astype(F32).reshape(flat[j].shape),
                                              ms[j], vs[j], k, sched.lr)
        losses.append(float(loss))
        lrs.append(sched.step(loss))
    return Params.from_state_dict(dict(zip(names, flat)), *counts), np.array(losses), np.array(lrs)


# ------------------------------------------------------------------ KAN variant (kan.py)
def kan_bases(x: np.ndarray, knots: np.ndarray, order: int = 3, deriv: bool = False):
    """Cox-de Boor bases of kan.py:94-104 in fp32 (same op order), x [N][in], knots [in][G]
    -> [N][in][G-1-order]; with deriv also d bases / dx (the recursion differentiated)."""
    x = np.asarray(x, F32)[:, :, None]
    g = np.asarray(knots, F32)[None]
    b = ((x >= g[..., :-1]) & (x < g[..., 1:])).astype(F32)
    db = np.zeros_like(b)
    for k in range(1, order + 1):
        dl = (g[..., k:-1] - g[..., :-(k + 1)]).astype(F32)
        dr = (g[..., k + 1:] - g[..., 1:(-k)]).astype(F32)
        left = ((x - g[..., :-(k + 1)]) / dl).astype(F32)
        right = ((g[..., k + 1:] - x) / dr).astype(F32)
        if deriv:
            db = (b[..., :-1] / dl + left * db[..., :-1] - b[..., 1:] / dr + right * db[..., 1:]).astype(F32)
        b = (left * b[..., :-1] + right * b[..., 1:]).astype(F32)
    return (b, db) if deriv else b


def kan_forward(sd: dict, x: np.ndarray, n_layers: int, dtype=F64):
    """KAN forward (kan.py:153-166) from a state_dict: per layer A = [SiLU(x) | bases(x)],
    out = A [base_w | spline_w * scaler]^T.  Returns (out [N], cache of per-layer inputs)."""
    xs = [np.asarray(x, F32).reshape(x.shape[0], -1)]
    for l in range(n_layers):
        pre = f"layers.{l}."
        xin = xs[-1]
        bw = np.asarray(sd[pre + "base_weight"], dtype)
        sw = np.asarray(sd[pre + "spline_weight"], dtype) * np.asarray(sd[pre + "spline_scaler"], dtype)[..., None]
        xd = xin.astype(dtype)
        silu = xd / (1 + np.exp(-xd))
        bases = kan_bases(xin, sd[pre + "grid"]).astype(dtype)
        out = silu @ bw.T + bases.reshape(xin.shape[0], -1) @ sw.reshape(sw.shape[0], -1).T
        xs.append(out.astype(F32) if dtype == F32 else out)
    return np.asarray(xs[-1]).reshape(-1), xs


def kan_backward(sd: dict, xs: list, g: np.ndarray, n_layers: int) -> dict:
    """Autograd of kan_forward for dLoss/dout = g [N] (fp64): grads of base_weight,
    spline_weight (x scaler) and spline_scaler (sum_c dW * spline_weight) per layer."""
    grads = {}
    G = np.asarray(g, F64).reshape(-1, 1)
    for l in range(n_layers - 1, -1, -1):
        pre = f"layers.{l}."
        xin = xs[l]
        xd = np.asarray(xin, F64)
        s = 1 / (1 + np.exp(-xd))
        silu, dsilu = xd * s, s * (1 + xd * (1 - s))
        b, db = kan_bases(np.asarray(xin, F32), sd[pre + "grid"], deriv=True)
        b, db = b.astype(F64), db.astype(F64)
        n, i = xin.shape
        bw = np.asarray(sd[pre + "base_weight"], F64)
        spw = np.asarray(sd[pre + "spline_weight"], F64)
        scl = np.asarray(sd[pre + "spline_scaler"], F64)
        dS = (G.T @ b.reshape(n, -1)).reshape(spw.shape)
        grads[pre + "base_weight"] = G.T @ silu
        grads[pre + "spline_weight"] = dS * scl[..., None]
        grads[pre + "spline_scaler"] = (dS * spw).sum(-1)
        if l > 0:
            sw = spw * scl[..., None]
            dA_base = G @ bw
            dA_spl = (G @ sw.reshape(sw.shape[0], -1)).reshape(n, i, -1)
            G = dsilu * dA_base + (db * dA_spl).sum(-1)
    return grads
