"""Snake / Tanh hidden layers on the HIP path (models.py:185-241, 356-372) against
the CPU oracle, which tests/test_oracle.py pins on the reference's own forward/backward numbers
(tests/golden/fwd_bwd_act.npz).

Kernel level: the fused Linear + Snake / Tanh forward epilogues (siren_inner_fwd_act), dX into
a Snake / Tanh layer (siren_inner_bwd_dx_act, with the da column partials) and the head
backward into a Snake layer, each within one fp16 rounding of the fp64 answer computed from the
same fp16 inputs.  Step level: the fused train step on train()'s default architecture
(num_sine=2, num_snake=2, a_initial=0.5) and on sine/Snake/Tanh mixes, gradients within 2 %
(relative L2) of the fp16-storage oracle, the autograd drop-in (model(x).backward()) and a
300-step fit tracked against the reference's own trajectory.
"""
import ctypes
import json
import math
import os

import numpy as np
import pytest
import torch

from inr_for_audio_amd._lib import new_tileq
from oracle import siren_oracle as orc
from errlog import check_grads, log

pytestmark = pytest.mark.gpu

F32 = np.float32
H16 = torch.float16
SINE, SNAKE, TANH = 0, 1, 2
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_KEEP = []


def ptr(t):
    return 0 if t is None else t.data_ptr()


def S():
    return torch.cuda.current_stream().cuda_stream


def ok(status, lib):
    assert status == 0, lib.siren_status_string(status)


def to_dev(a, dev, dtype=torch.float32):
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=F32)).to(dev).to(dtype)
    _KEEP.append(t)
    return t


def f16_np(t):
    return t.float().cpu().numpy().astype(np.float64)


def within_f16(got, ref, abs_slack):
    err = np.abs(np.asarray(got, np.float64) - ref)
    return float(np.max(err - (np.abs(ref) * 2.0 ** -11 + abs_slack + 2.0 ** -25)))


@pytest.fixture(autouse=True)
def _release():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


@pytest.fixture(params=[(128, 0, -1), (256, 0, -1), (256, 2, -1), (256, 0, 1), (256, 2, 1)],
                ids=lambda p: f"t{p[0]}g{p[1]}p{p[2]}")
def tile(request, lib):
    """NT tile edge, persistent grid (grid 2: every block walks several tiles) and 256x256
    K-loop (-1: the automatic ping-pong, 1: the persistent double buffer)."""
    t, grid, pipe = request.param
    ok(lib.siren_set_option(0, t), lib)
    ok(lib.siren_set_option(4, grid), lib)
    ok(lib.siren_set_option(2, pipe), lib)
    yield t
    lib.siren_set_option(0, 0)
    lib.siren_set_option(4, 0)
    lib.siren_set_option(2, -1)


def _inputs(rng, R, H):
    X = orc.f16_round(rng.uniform(-1, 1, (R, H)).astype(F32))
    lim = 1 / math.sqrt(H)     # nn.Linear default init range of the Snake / Tanh Linears
    W = orc.f16_round(rng.uniform(-lim, lim, (H, H)).astype(F32))
    b = rng.uniform(-lim, lim, H).astype(F32)
    return X, W, b


def _snake_ref(z, a):
    s, c = np.sin(a * z), np.cos(a * z)
    return z + s * s / a, 1.0 + 2.0 * s * c, (z * 2.0 * s * c) / a - s * s / (a * a)


@pytest.mark.parametrize("act", [SNAKE, TANH])
@pytest.mark.parametrize("R,H,amag", [(512, 256, 0.5), (512, 512, 50.0), (256, 1024, 3.0)])
@pytest.mark.parametrize("head", [False, True])
def test_inner_fwd_act(lib, dev, tile, act, R, H, amag, head):
    if tile == 256 and (R % 256 or H % 256):
        pytest.skip("256-tile needs multiples of 256")
    rng = np.random.default_rng(21)
    X, W, b = _inputs(rng, R, H)
    a = (amag * rng.uniform(0.5, 1.5, H)).astype(F32)
    hw = rng.uniform(-0.01, 0.01, H).astype(F32)
    Y = torch.empty(R, H, dtype=H16, device=dev)
    C = torch.empty_like(Y)
    E = torch.zeros_like(Y)
    hp = torch.zeros(H // 128, R, device=dev)
    ok(lib.siren_inner_fwd_act(ptr(to_dev(X, dev, H16)), ptr(to_dev(W, dev, H16)), ptr(to_dev(b, dev)), act,
                               ctypes.c_float(30.0), ptr(to_dev(a, dev)), R, H, ptr(Y), ptr(C), ptr(E),
                               ptr(to_dev(hw, dev)) if head else None, ptr(hp) if head else None,
                               ptr(new_tileq(dev)), S()), lib)
    z = X.astype(np.float64) @ W.astype(np.float64).T + b
    # fp32 accumulation of z: |dz| ~ 1e-6; through sin(a z) that is a*|dz|
    slack = 2e-6 * max(1.0, float(amag)) * 4
    if act == SNAKE:
        y, d, e = _snake_ref(z, a.astype(np.float64))
        assert within_f16(f16_np(Y), y, slack) <= 0
        assert within_f16(f16_np(C), d, 2 * slack) <= 0
        assert within_f16(f16_np(E), e, 2 * slack * (np.max(np.abs(z)) + 1) / float(a.min())) <= 0
    else:
        y = np.tanh(z)
        assert within_f16(f16_np(Y), y, 1e-6) <= 0
        assert within_f16(f16_np(C), 1.0 - y * y, 2e-6) <= 0
    if head:
        ref = y @ hw.astype(np.float64)
        got = hp.cpu().numpy().astype(np.float64).sum(0)
        assert np.max(np.abs(got - ref)) < 1e-4 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("act", [SNAKE, TANH])
@pytest.mark.parametrize("H", [256, 512])
def test_inner_fwd_act_lines_queue(lib, dev, act, H):
    """The whole-line Snake / Tanh forward (ACTL, taken at K <= 512) on the dynamic tile queue: 16-32
    tiles of 256 x 256 give a grid that is a multiple of 8, so the queue kernel runs (the
    R = 512 cases above have <= 4 tiles and only ever reach the static walk).  Its outputs must equal
    the static walk's bit for bit and lie within one fp16 rounding of fp64."""
    R = 4096
    rng = np.random.default_rng(33)
    X, W, b = _inputs(rng, R, H)
    a = (0.5 * rng.uniform(0.5, 1.5, H)).astype(F32)
    Xd, Wd, bd, ad = to_dev(X, dev, H16), to_dev(W, dev, H16), to_dev(b, dev), to_dev(a, dev)
    outs = []
    ok(lib.siren_set_option(0, 256), lib)
    try:
        for queue in (1, 0):
            ok(lib.siren_set_option(8, queue), lib)
            Y, C, E = (torch.full((R, H), float("nan"), dtype=H16, device=dev) for _ in range(3))
            ok(lib.siren_inner_fwd_act(ptr(Xd), ptr(Wd), ptr(bd), act, ctypes.c_float(1.0), ptr(ad), R, H, ptr(Y),
                                       ptr(C), ptr(E), None, None, ptr(new_tileq(dev)), S()), lib)
            torch.cuda.synchronize()
            outs.append((Y, C, E) if act == SNAKE else (Y, C))
    finally:
        lib.siren_set_option(8, 1)
        lib.siren_set_option(0, 0)
    for q, s in zip(*outs):
        assert torch.equal(q, s)
    z = X.astype(np.float64) @ W.astype(np.float64).T + b
    slack = 8e-6
    Y, C = outs[0][0], outs[0][1]
    if act == SNAKE:
        y, d, e = _snake_ref(z, a.astype(np.float64))
        assert within_f16(f16_np(Y), y, slack) <= 0
        assert within_f16(f16_np(C), d, 2 * slack) <= 0
        assert within_f16(f16_np(outs[0][2]), e, 2 * slack * (np.max(np.abs(z)) + 1) / float(a.min())) <= 0
    else:
        y = np.tanh(z)
        assert within_f16(f16_np(Y), y, 1e-6) <= 0
        assert within_f16(f16_np(C), 1.0 - y * y, 2e-6) <= 0


def test_snake_small_az_error(lib, dev):
    """The Snake epilogue's double angle (siren_common.h snake_epi: sin^2(az) = (1 - cos 2az)/2) cancels
    for small |az|: t = sin^2(az)/a carries the absolute error of the hardware cos near 1 (~2^-24)
    over 2a, and E = dY/da = (z sin 2az - t)/a that over a again -- an ABSOLUTE error of ~1e-7 at the
    default a = 0.5 where E ~ z^2 is tiny, not a relative one.  Bounded here at small
    |z| against fp64: |E - E_ref| <= one fp16 rounding of E_ref + 4 * 2^-24 / a^2 (+ the fp32 z);
    Y and D stay within one fp16 rounding plus fp32 slack."""
    rng = np.random.default_rng(5)
    R, H = 512, 256
    X = orc.f16_round(rng.uniform(-1, 1, (R, H)).astype(F32))
    W = orc.f16_round(rng.uniform(-1, 1, (H, H)).astype(F32) * 2e-4)   # |z| <~ 1e-2
    b = rng.uniform(-1e-3, 1e-3, H).astype(F32)
    a = np.full(H, 0.5, F32)
    Y = torch.empty(R, H, dtype=H16, device=dev)
    C, E = torch.empty_like(Y), torch.empty_like(Y)
    ok(lib.siren_inner_fwd_act(ptr(to_dev(X, dev, H16)), ptr(to_dev(W, dev, H16)), ptr(to_dev(b, dev)), SNAKE,
                               ctypes.c_float(30.0), ptr(to_dev(a, dev)), R, H, ptr(Y), ptr(C), ptr(E), None, None,
                               ptr(new_tileq(dev)), S()), lib)
    z = X.astype(np.float64) @ W.astype(np.float64).T + b
    y, d, e = _snake_ref(z, a.astype(np.float64))
    eabs = 4.0 * 2.0 ** -24 / 0.25
    err_e = np.abs(f16_np(E) - e)
    log("snake_small_az", max_abs_z=float(np.abs(z).max()), max_abs_e=float(np.abs(e).max()),
        max_err_e=float(err_e.max()), bound_abs=eabs)
    assert within_f16(f16_np(E), e, eabs) <= 0
    assert within_f16(f16_np(Y), y, 1e-7) <= 0
    assert within_f16(f16_np(C), d, 1e-7) <= 0


@pytest.mark.parametrize("act", [SNAKE, TANH])
@pytest.mark.parametrize("R,H,k", [(512, 256, None), (512, 512, 9), (256, 1024, 3)])
def test_inner_bwd_dx_act(lib, dev, tile, act, R, H, k):
    if tile == 256 and (R % 256 or H % 256):
        pytest.skip("256-tile needs multiples of 256")
    rng = np.random.default_rng(22)
    dZ = orc.f16_round((rng.normal(size=(R, H)) * 1e-3).astype(F32))
    _, W, _ = _inputs(rng, R, H)
    D = orc.f16_round(rng.uniform(0, 2, (R, H)).astype(F32))
    Ep = orc.f16_round(rng.normal(size=(R, H)).astype(F32))
    out = torch.empty(R, H, dtype=H16, device=dev)
    part = torch.zeros(R // 128, 2, H, device=dev)
    WT = np.ascontiguousarray(W.T)
    gs = None if k is None else to_dev(np.array([2.0 ** k, 2.0 ** -k], F32), dev)
    ok(lib.siren_inner_bwd_dx_act(ptr(to_dev(dZ, dev, H16)), ptr(to_dev(WT, dev, H16)), ptr(to_dev(D, dev, H16)),
                                  ptr(to_dev(Ep, dev, H16)) if act == SNAKE else None, act, ctypes.c_float(30.0),
                                  R, H, ptr(gs), ptr(out), ptr(part), S()), lib)
    dY = dZ.astype(np.float64) @ W.astype(np.float64)
    ref = dY * D
    scale = np.max(np.abs(ref))
    assert within_f16(f16_np(out), ref, 1e-5 * scale) <= 0
    tile_rows = lib.siren_nt_tile(R, H)
    p = part.cpu().numpy().astype(np.float64)
    if act == SNAKE:
        p = p[: R // tile_rows]
        db, da = p[:, 0].sum(0), p[:, 1].sum(0)
    else:
        db = p.reshape(-1)[: (R // tile_rows) * H].reshape(-1, H).sum(0)
        da = None
    sc = 2.0 ** (k or 0)
    tol = 1e-4 * np.max(np.abs(ref.sum(0))) + 1e-6 * scale * math.sqrt(R)
    assert np.max(np.abs(db * sc - ref.sum(0))) < tol
    if da is not None:
        dref = (dY * Ep).sum(0)
        assert np.max(np.abs(da * sc - dref)) < 1e-4 * np.max(np.abs(dref)) + 1e-6 * np.max(np.abs(dY)) * math.sqrt(R)


@pytest.mark.parametrize("H", [128, 1024])
def test_head_bwd_snake(lib, dev, H):
    rng = np.random.default_rng(23)
    R = 512
    D = orc.f16_round(rng.uniform(0, 2, (R, H)).astype(F32))
    Y = orc.f16_round(rng.uniform(-1, 1, (R, H)).astype(F32))
    Ep = orc.f16_round(rng.normal(size=(R, H)).astype(F32))
    g = (rng.normal(size=R) * 1e-6).astype(F32)
    w = rng.uniform(-0.05, 0.05, H).astype(F32)
    k = 20
    dZ = torch.empty(R, H, dtype=H16, device=dev)
    dbp, dwp, dap = (torch.empty(R // 128, H, device=dev) for _ in range(3))
    gs = to_dev(np.array([2.0 ** k, 2.0 ** -k], F32), dev)
    ok(lib.siren_head_bwd(ptr(to_dev(D, dev, H16)), ptr(to_dev(Y, dev, H16)), ptr(to_dev(g, dev)),
                          ptr(to_dev(w, dev)), ctypes.c_float(1.0), R, H, ptr(gs), ptr(dZ), ptr(dbp), ptr(dwp),
                          ptr(to_dev(Ep, dev, H16)), ptr(dap), S()), lib)
    dY = g[:, None].astype(np.float64) * w[None, :]
    assert within_f16(f16_np(dZ), dY * D * 2.0 ** k, 1e-12) <= 0
    for got, terms in ((dbp, dY * D), (dwp, g[:, None].astype(np.float64) * Y), (dap, dY * Ep)):
        err = np.abs(got.cpu().numpy().astype(np.float64).sum(0) - terms.sum(0))
        assert np.all(err <= 1e-5 * np.abs(terms).sum(0) + 1e-15)


# ------------------------------------------------------------------ fused step / drop-in
def _model(H, ns, nk, nt, w0=1000.0, a0=0.5, seed=0, in_dim=1, fl=False, ll=True):
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    torch.manual_seed(seed)
    return SirenWithSnakeTanh(in_dim, 1, H, ns, nk, nt, first_linear=fl, last_linear=ll, first_omega_0=w0,
                              hidden_omega_0=30.0, a_initial=a0)


def _signal(n, in_dim=1):
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    if in_dim == 2:
        ch = torch.where(torch.arange(n) % 2 == 0, -1.0, 1.0).reshape(n, 1)
        t = torch.cat([t, ch], 1)
    y = 0.5 * torch.sin(37 * t[:, :1]) + 0.3 * torch.sin(91 * t[:, :1] + 0.5)
    return t, y


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("H,cfg,n,a0,in_dim,mb", [
    (256, (2, 2, 0), 2000, 0.5, 1, 1 << 20),     # run.py train() default architecture
    (128, (1, 2, 1), 1500, 0.5, 1, 1024),        # sine + Snake + Tanh, 2 micro-batches
    (512, (1, 1, 2), 1000, 5.0, 2, 1 << 20),     # stereo grid, Tanh last
    (1024, (0, 4, 0), 1024, 50.0, 1, 1 << 20),   # the reference's __main__ run (run.py:466)
    (256, (1, 1, 0, True, True), 1500, 0.5, 1, 1 << 20),    # first_linear: Linear + Snake first
    (256, (2, 0, 0, False, False), 1500, 0.5, 1, 1 << 20),  # last_linear=False: final SineLayer
    (256, (1, 1, 1, True, False), 1500, 2.0, 2, 1024),      # both, stereo grid, micro-batches
])
def test_train_step_act_vs_oracle(dev, H, cfg, n, a0, in_dim, mb):
    from inr_for_audio_amd.engine import SirenEngine
    fl, ll = (cfg[3], cfg[4]) if len(cfg) > 3 else (False, True)
    model = _model(H, *cfg[:3], a0=a0, in_dim=in_dim, fl=fl, ll=ll)
    sd0 = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    t, y = _signal(n, in_dim)
    eng = SirenEngine(model, t, y, lr=1e-3, micro_batch=mb, device=dev)
    eng.step()
    torch.cuda.synchronize()
    got = {k: v.detach().cpu().numpy() for k, v in zip(eng.layout.names, eng.grad_views())}
    p = orc.Params.from_state_dict(sd0, *cfg[:3], fl, ll)
    out, cache = orc.forward(p, t.numpy(), 1000.0, 30.0, half=True, dtype=np.float64)
    ref = orc.backward(p, t.numpy(), cache, orc.mse_grad(out, y.numpy()), 1000.0, 30.0, half=True)
    assert set(ref) == set(got)
    check_grads(f"act_step[{H}x{cfg}x{n}x{in_dim}x{mb}]", got, ref)
    out32, _ = orc.forward(p, t.numpy(), 1000.0, 30.0)
    l32 = orc.mse(out32, y.numpy())
    log(f"act_step_loss[{H}x{cfg}x{n}x{in_dim}x{mb}]", loss=abs(eng.last_loss() - l32) / l32)
    assert abs(eng.last_loss() - l32) < 5e-4 * l32  # measured <= 5.8e-5


@pytest.mark.parametrize("fl,ll", [(False, True), (True, False)])
def test_autograd_dropin_act(dev, fl, ll):
    """model(x) / loss.backward() on the default Snake architecture (and with a first
    Linear+Snake and a final SineLayer): HIP forward and backward through _SirenFunction,
    gradients on every parameter including the Snake a's."""
    model = _model(256, 2, 2, 0, fl=fl, ll=ll).to(dev)
    sd0 = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    t, y = _signal(1500)
    out = model(t.to(dev).reshape(1, -1, 1))
    loss = torch.nn.MSELoss()(out, y.to(dev).reshape(1, -1, 1))
    loss.backward()
    p = orc.Params.from_state_dict(sd0, 2, 2, 0, fl, ll)
    o, cache = orc.forward(p, t.numpy(), 1000.0, 30.0, half=True, dtype=np.float64)
    oerr = np.max(np.abs(out.detach().cpu().numpy().reshape(-1) - o)) / np.max(np.abs(o))
    ref = orc.backward(p, t.numpy(), cache, orc.mse_grad(o, y.numpy()), 1000.0, 30.0, half=True)
    errs = {}
    for name, prm in model.named_parameters():
        assert prm.grad is not None, name
        errs[name] = _rel(prm.grad.cpu().numpy().reshape(ref[name].shape), ref[name])
    log(f"autograd_dropin_act[{fl},{ll}]", out=oerr, **errs)
    assert oerr < 2e-3, oerr                           # measured <= 3.2e-4
    assert all(e < 2e-3 for e in errs.values()), errs  # measured <= 3.2e-4


def _fit_snake(dev, steps, seed):
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.utils import calculate_snr
    g = np.load(os.path.join(GOLDEN, "gt_bach_1s.npz"))
    t = torch.from_numpy(g["coords"]).reshape(-1, 1)
    y = torch.from_numpy(g["target"])
    eng = SirenEngine(_model(256, 2, 2, 0, seed=seed), t, y, lr=1e-3, hist_cap=steps, device=dev)
    eng.step()
    eng.capture_graph()
    for _ in range(steps - 1):
        eng.step()
    out = eng.infer(t.to(dev)).cpu().numpy()
    return eng, float(calculate_snr(g["target"], out))


def test_fit_default_snake_first_steps_track_reference(dev):
    """train()'s default architecture (2 sine + 2 Snake layers after the first SineLayer,
    H = 256, a_initial = 0.5, omega0 = 1000; gt_bach 1 s): the first steps track the
    reference's own run of the same loop (tests/golden/trajectory_snake_default.json, seed 1)."""
    tr = json.load(open(os.path.join(GOLDEN, "trajectory_snake_default.json")))
    eng, _ = _fit_snake(dev, 20, tr["seed"])
    losses, lrs = eng.history()
    ref = np.array(tr["loss"][:20])
    dev8 = np.max(np.abs(losses[:8] - ref[:8]) / ref[:8])
    log("fit_snake_first_steps", max_rel_8=dev8)
    assert dev8 < 2e-2  # measured 5.7e-3
    assert np.array_equal(lrs, np.array(tr["lr"][:20]))


def test_fit_default_snake_quality_over_seeds(dev):
    """Multi-seed fit protocol of tests/test_gpu_fit.py on the Snake default architecture, vs
    the reference's runs of the same seeds (tests/golden/trajectory_snake_default_seeds.json).
    At lr 1e-3 this architecture spends ~40 % of its 300 steps inside Adam loss spikes (loss > 10x
    the running minimum) -- the reference itself ends 3 of 8 seeds at ~0 dB -- so the final SNR is
    a coin flip per seed, and the per-seed best-loss SNR moves by +-2 dB with the summation order
    alone.  Gates: the median over seeds of the best-loss SNR within 0.5 dB of the reference's,
    plus how far the reference algorithm itself lands when only its summation order changes (the
    same fits in fp32 torch on this GPU, same init and data: tests/torch_ref.py), capped at 1.5 dB;
    and the spike rate summed over seeds within a factor 1.5."""
    from torch_ref import fp32_fit_stack
    ref = json.load(open(os.path.join(GOLDEN, "trajectory_snake_default_seeds.json")))
    var = float(np.mean(np.load(os.path.join(GOLDEN, "gt_bach_1s.npz"))["target"].astype(np.float64) ** 2))

    def spikes(x):
        x = np.asarray(x)
        return int(np.sum(x > 10 * np.minimum.accumulate(x)))

    g = np.load(os.path.join(GOLDEN, "gt_bach_1s.npz"))
    best_gpu, best_ref, best_t32, sp_gpu, sp_ref = [], [], [], 0, 0
    for s in sorted(int(k) for k in ref["runs"]):
        eng, _ = _fit_snake(dev, ref["steps"], s)
        losses, _ = eng.history()
        r = ref["runs"][str(s)]
        best_gpu.append(10 * np.log10(var / float(np.min(losses))))
        best_ref.append(10 * np.log10(var / float(np.min(r["loss"]))))
        sp_gpu += spikes(losses)
        sp_ref += spikes(r["loss"])
        t32, _ = fp32_fit_stack(_model(256, 2, 2, 0, seed=s).state_dict(), ["sine", "sine", "snake", "snake"],
                                1000.0, g["coords"], g["target"], ref["steps"], device=dev)
        best_t32.append(10 * np.log10(var / float(np.min(t32))))
    med = lambda x: float(np.median(x))  # noqa: E731
    d_gpu, d_t32 = abs(med(best_gpu) - med(best_ref)), abs(med(best_t32) - med(best_ref))
    log("fit_snake_default_seeds", med_gpu=med(best_gpu), med_ref=med(best_ref), med_torch_gpu_fp32=med(best_t32),
        spikes_gpu=sp_gpu, spikes_ref=sp_ref)
    print(f"\nSnake default best-loss SNR median: GPU {med(best_gpu):.2f} dB, reference {med(best_ref):.2f} dB, "
          f"fp32 torch on the GPU {med(best_t32):.2f} dB\nspike steps: GPU {sp_gpu}, reference {sp_ref}"
          f"\nper seed GPU best {np.round(best_gpu, 2).tolist()}\nper seed ref best {np.round(best_ref, 2).tolist()}"
          f"\nper seed t32 best {np.round(best_t32, 2).tolist()}")
    assert d_gpu < min(0.5 + d_t32, 1.5), (d_gpu, d_t32)
    assert sp_ref / 1.5 <= sp_gpu <= sp_ref * 1.5
