"""The fused last layer for Snake and Tanh stacks (gemm_nt.hip NT_FWD_HB_SNAKE / NT_FWD_HB_TANH).

run.py:30's train() defaults to num_sine=2, num_snake=2 and its only live __main__ call is
num_sine=0, num_snake=4 (run.py:466): those stacks end in Linear + Snake (models.py:356-364), the
Tanh stacks in Linear + Tanh (models.py:366-372).  siren_train_step runs that last layer, the head
(models.py:374-381), the loss gradient (run.py:161-169) and the head backward (its autograd) as one
launch, as for a sine last layer (test_gpu_headfuse.py).

Backward scale: a Tanh output is bounded by 1, so S comes from grad_scale_bound like the sine
case.  A Snake output is not bounded, so S is the unfused path's own rule (grad_scale) applied to
the max|g| of the previous launch on the workspace (siren_batch.head_scale_prev; the engine sets
it after its first step, and the range guard catches a step whose |g| outgrew S).

Checked against the unfused launches (siren_inner_fwd_act + head -> siren_head_loss ->
siren_head_bwd at the same S: outputs, dLoss/dout, loss partials, max|g| partials and dZ_L bit
for bit) and, whole step, against the unfused step and the fp16-storage oracle."""
import ctypes

import numpy as np
import pytest
import torch

from errlog import check_grads, log
from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu

OPT_NT_TILE, OPT_NT_GRID, OPT_HEAD_FUSE = 0, 4, 9
DEFAULTS = {OPT_NT_TILE: 0, OPT_NT_GRID: 0, OPT_HEAD_FUSE: 1}
SINE, SNAKE, TANH = 0, 1, 2


@pytest.fixture
def opts(lib):
    touched = []

    def set_(o, v):
        assert lib.siren_set_option(o, v) == 0, (o, v)
        touched.append(o)

    yield set_
    for o in touched:
        lib.siren_set_option(o, DEFAULTS[o])


@pytest.mark.parametrize("act", [SNAKE, TANH])
@pytest.mark.parametrize("H,R,n_valid,grid,amag", [
    (1024, 4096, 4096, 0, 0.5),
    (1024, 4096, 3000, 8, 50.0),   # pad rows; 2 band groups walking 8 bands each; __main__'s a = 50
    (512, 2048, 2048, 2, 3.0),
    (256, 2048, 1500, 0, 0.5),
])
def test_kernel_act_vs_unfused_launches(dev, lib, opts, act, H, R, n_valid, grid, amag):
    from inr_for_audio_amd._lib import new_tileq
    opts(OPT_NT_TILE, 256)
    opts(OPT_NT_GRID, grid)
    g_ = torch.Generator(device=dev).manual_seed(H + R + act)
    f16 = torch.float16
    P = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    X = torch.sin(torch.rand(R, H, device=dev, generator=g_) * 6.2831853).to(f16)
    W = ((torch.rand(H, H, device=dev, generator=g_) * 2 - 1) * (6 / H) ** 0.5).to(f16)
    b = (torch.rand(H, device=dev, generator=g_) - 0.5) * 0.2
    a = (0.5 + torch.rand(H, device=dev, generator=g_)) * amag
    wh = (torch.rand(H, device=dev, generator=g_) - 0.5) * 2 / H ** 0.5
    bh = torch.tensor([0.01], device=dev)
    y = (torch.rand(R, device=dev, generator=g_) - 0.5)
    gs = torch.tensor([2.0 ** 9, 2.0 ** -9], device=dev)
    nq = 3 if act == SNAKE else 2
    e = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=dev)  # noqa: E731
    hp1, out1, g1, dZ1, E1 = e(H // 256, R), e(R), e(R), e(R, H, dt=f16), e(R, H, dt=f16)
    sse1, gsum1, gmax1, part1 = e(R // 256), e(R // 256), e(R // 256), e(R // 256, nq, H)
    st = lib.siren_head_fused_fwd_act(P(X), P(W), P(b), act, ctypes.c_float(30.0), P(a), R, H, P(wh), P(bh),
                                      ctypes.c_float(0.0), P(y), n_valid, float(n_valid), 0, P(gs), P(hp1),
                                      P(out1), P(g1), P(sse1), P(gsum1), P(gmax1), P(dZ1), P(part1), P(E1), s)
    assert st == 0, lib.siren_status_string(st)
    Y, C, E, hp2 = e(R, H, dt=f16), e(R, H, dt=f16), e(R, H, dt=f16), e(H // 256, R)
    out2, g2, sse2, gsum2, gmax2, dZ2 = e(R), e(R), e(R // 256), e(R // 256), e(R // 256), e(R, H, dt=f16)
    db2, dw2, da2 = e(R // 128, H), e(R // 128, H), e(R // 128, H)
    tq = new_tileq(dev)
    snake = act == SNAKE
    for st in (lib.siren_inner_fwd_act(P(X), P(W), P(b), act, ctypes.c_float(30.0), P(a), R, H, P(Y), P(C),
                                       P(E) if snake else None, P(wh), P(hp2), P(tq), s),
               lib.siren_head_loss(P(hp2), H // 256, R, P(bh), P(y), n_valid, float(n_valid), P(out2), P(g2), P(sse2),
                                   P(gsum2), P(gmax2), s),
               lib.siren_head_bwd(P(C), P(Y), P(g2), P(wh), ctypes.c_float(1.0), R, H, P(gs), P(dZ2), P(db2), P(dw2),
                                  P(E) if snake else None, P(da2) if snake else None, s)):
        assert st == 0, lib.siren_status_string(st)
    torch.cuda.synchronize()
    assert torch.equal(out1, out2) and torch.equal(g1, g2)
    assert torch.equal(sse1, sse2) and torch.equal(gsum1, gsum2) and torch.equal(gmax1, gmax2)
    assert torch.equal(dZ1, dZ2)
    if snake:  # the fused kernel leaves the layer's dY/da where the unfused forward writes it
        assert torch.equal(E1, E)
    pairs = [(part1[:, 0], db2), (part1[:, 1], dw2)] + ([(part1[:, 2], da2)] if snake else [])
    for got, ref in pairs:
        got, ref = got.double().sum(0), ref.double().sum(0)
        assert float((got - ref).abs().max()) <= 1e-5 * float(ref.abs().max()) + 1e-12


def _engine(dev, H, cfg, n, *, a0=0.5, mb=1 << 20, seed=0, w0=3000.0, loss="mse"):
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    torch.manual_seed(seed)
    model = SirenWithSnakeTanh(1, 1, H, *cfg, first_omega_0=w0, hidden_omega_0=30.0, a_initial=a0)
    sd0 = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    y = 0.5 * torch.sin(37 * t) + 0.3 * torch.sin(91 * t + 0.5)
    eng = SirenEngine(model, t, y, micro_batch=mb, loss_mode=loss, device=dev)
    return eng, sd0, t, y


def _grads(eng, lib):
    from inr_for_audio_amd import _lib
    _lib.check(lib.siren_profile_enable(64 * eng.n_micro), "profile_enable")
    eng._launch_grads()
    torch.cuda.synchronize()
    prof = _lib.profile_read()
    _lib.check(lib.siren_profile_enable(0), "profile_disable")
    return eng.grads.clone(), eng.ws.out.clone(), eng.ws.g.clone(), {k: n for k, (_, n) in prof.items()}


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


@pytest.mark.parametrize("H,cfg,n,grid,a0,mb,loss", [
    (1024, (2, 2, 0), 8192, 0, 0.5, 1 << 20, "mse"),   # run.py:30 train() default stack
    (1024, (0, 4, 0), 8000, 8, 50.0, 1 << 20, "mse"),  # run.py:466 __main__: 4 Snake layers, a = 50
    (512, (1, 1, 1), 4096, 6, 0.5, 1 << 20, "mae"),    # Tanh last, L1Loss
    (1024, (1, 1, 0), 6000, 4, 0.5, 2048, "mse"),      # Snake last, 3 micro-batches
])
def test_fused_act_matches_unfused(dev, lib, opts, H, cfg, n, grid, a0, mb, loss):
    opts(OPT_NT_TILE, 256)
    opts(OPT_NT_GRID, grid)
    eng, _, _, _ = _engine(dev, H, cfg, n, a0=a0, mb=mb, loss=loss)
    L = sum(cfg)
    snake_last = cfg[2] == 0
    # the first launch of a Snake-last stack runs unfused (no max|g| of a previous launch yet)
    g0, o0, gg0, k0 = _grads(eng, lib)
    assert k0["head_fwd"] == (0 if snake_last else eng.n_micro)
    ga, oa, gga, ka = _grads(eng, lib)
    opts(OPT_HEAD_FUSE, 0)
    gb, ob, ggb, kb = _grads(eng, lib)
    assert ka["head_fwd"] == eng.n_micro and kb["head_fwd"] == 0
    assert ka["inner_fwd"] == (L - 1) * eng.n_micro and kb["inner_fwd"] == L * eng.n_micro
    assert torch.equal(oa, ob) and torch.equal(gga, ggb)
    sse = eng.layout.sse_offset
    assert torch.equal(ga[sse], gb[sse])
    lay = eng.layout
    errs = {k: _rel(lay.view(ga, i), lay.view(gb, i)) for i, k in enumerate(lay.names)}
    log(f"headfuse_act_vs_unfused[{H}x{cfg}x{n}x{grid}x{mb}x{loss}]", errs=errs)
    # Snake: the same S (the previous launch's max|g| is this one's: no update in between), so only
    # the fp32 order of the db_L / dw_head / da_L column sums differs; Tanh: S from the bound
    for k, e in errs.items():
        assert e < 2e-5, (k, e)
    if snake_last and eng.n_micro == 1:
        # one micro-batch, no update: the unfused launch and the previous one wrote the same partials
        errs0 = {k: _rel(lay.view(ga, i), lay.view(g0, i)) for i, k in enumerate(lay.names)}
        assert max(errs0.values()) < 2e-5, errs0


@pytest.mark.parametrize("H,cfg,n,a0", [
    (1024, (2, 2, 0), 4096, 0.5),
    (512, (1, 0, 2), 4096, 0.5),
    (1024, (0, 4, 0), 4096, 50.0),
])
def test_fused_act_vs_oracle(dev, lib, opts, H, cfg, n, a0):
    opts(OPT_NT_TILE, 256)
    eng, sd0, t, y = _engine(dev, H, cfg, n, a0=a0)
    _grads(eng, lib)                      # a Snake last layer's first launch: unfused
    got_g, _, _, kinds = _grads(eng, lib)
    assert kinds["head_fwd"] == 1
    S = float(eng.ws.gscale[0])
    assert float(eng.ws.gscale[1]) == 1.0 / S
    p = orc.Params.from_state_dict(sd0, *cfg)
    out, cache = orc.forward(p, t.numpy(), 3000.0, 30.0, half=True, dtype=np.float64)
    gl = orc.mse_grad(out, y.numpy())
    if cfg[2]:  # Tanh last: the bound of grad_scale_bound, as the sine case
        assert S == orc.grad_scale_bound(y.numpy(), n, p.wf, float(np.asarray(p.bf).reshape(-1)[0]), n, 1.0)
    else:       # Snake last: grad_scale on the previous launch's max|g| (= this launch's: no update)
        assert S == orc.grad_scale(eng.ws.g.cpu().numpy(), p.wf, 2.0)
    ref = orc.backward(p, t.numpy(), cache, gl, 3000.0, 30.0, half=True, scale=S)
    got = {k: eng.layout.view(got_g, i).cpu().numpy() for i, k in enumerate(eng.layout.names)}
    check_grads(f"headfuse_act_vs_oracle[{H}x{cfg}x{n}]", got, ref)
    lref = orc.mse(out, y.numpy())
    lgot = float(got_g[eng.layout.sse_offset]) / n
    assert abs(lgot - lref) <= 5e-4 * lref, (lgot, lref)


def test_fused_act_training_graph_and_determinism(dev, opts):
    """The default train() stack (2 sine + 2 Snake): eager steps (first unfused, then fused) and a
    captured step replayed give bit-identical parameters and losses; no fp16 overflow."""
    opts(OPT_NT_TILE, 256)
    a, _, _, _ = _engine(dev, 1024, (2, 2, 0), 8192)
    b, _, _, _ = _engine(dev, 1024, (2, 2, 0), 8192)
    for _ in range(5):
        a.step()
    b.step()
    b.step()
    b.capture_graph()
    for _ in range(3):
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params)
    la, _ = a.history()
    lb, _ = b.history()
    assert np.array_equal(la, lb)
    assert a.guard_state()["overflows"] == 0


def test_snake_head_scale_per_micro_batch(dev, lib, opts):
    """A fused Snake last layer takes its backward scale S from the max|g| partials of the previous
    launch over the SAME rows (siren_batch.head_scale_prev): each micro-batch has its own partials
    (engine._gmax), not the workspace's one slice.  Micro-batches of very different
    loudness -- a quiet segment, a loud one, a quiet one, in the order a long clip would give them --
    then each keep the unfused path's scale: no fp16 overflow is ever caught, and the fused step's
    gradients match the unfused step's at the same weights.  (With one shared slice the loud
    micro-batch would run on the quiet one's S, ~2^11 too large, and the quiet one after it on the
    loud one's; the same engine with its batches pointed at one slice is run beside it and its
    overflow count and gradient error are logged.)"""
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    opts(OPT_NT_TILE, 256)
    torch.manual_seed(0)
    H, mb, n = 1024, 4096, 12288
    model = SirenWithSnakeTanh(1, 1, H, 1, 1, 0, first_omega_0=3000.0, hidden_omega_0=30.0, a_initial=0.5)
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    amp = torch.ones(n)
    amp[mb:2 * mb] = 2000.0  # the loud segment: |g| ~ 10^3 x the quiet ones'
    y = amp * (0.5 * torch.sin(37 * t[:, 0]) + 0.3 * torch.sin(91 * t[:, 0] + 0.5))
    eng = SirenEngine(model, t, y, micro_batch=mb, device=dev)
    assert eng.n_micro == 3
    for _ in range(4):
        eng.step()
    torch.cuda.synchronize()
    assert eng.guard_state()["overflows"] == 0
    assert eng.steps_applied() == 4
    gmax = eng._gmax.amax(dim=1).cpu()
    assert float(gmax[1]) > 100 * float(max(gmax[0], gmax[2])), gmax  # really a loud segment between quiet ones
    _grads(eng, lib)                      # every micro-batch's partials at these weights
    ga, oa, gga, ka = _grads(eng, lib)    # fused, each at its own scale
    opts(OPT_HEAD_FUSE, 0)
    gb, ob, ggb, kb = _grads(eng, lib)    # unfused: the scale from this launch's own max|g|
    assert ka["head_fwd"] == 3 and kb["head_fwd"] == 0
    assert torch.equal(oa, ob) and torch.equal(gga, ggb)
    lay = eng.layout
    errs = {k: _rel(lay.view(ga, i), lay.view(gb, i)) for i, k in enumerate(lay.names)}
    for k, e in errs.items():
        assert e < 2e-5, (k, e)
    # the round-4 behaviour, for the record: every micro-batch on one max|g| slice
    opts(OPT_HEAD_FUSE, 1)
    torch.manual_seed(0)
    model2 = SirenWithSnakeTanh(1, 1, H, 1, 1, 0, first_omega_0=3000.0, hidden_omega_0=30.0, a_initial=0.5)
    eng2 = SirenEngine(model2, t, y, micro_batch=mb, device=dev)
    for b in eng2.batches:
        b.gmax_part = eng2.batches[0].gmax_part
    for _ in range(4):
        eng2.step()
    torch.cuda.synchronize()
    shared_overflows = eng2.guard_state()["overflows"]
    _grads(eng2, lib)
    gc, _, _, _ = _grads(eng2, lib)
    opts(OPT_HEAD_FUSE, 0)
    gd, _, _, _ = _grads(eng2, lib)
    lay2 = eng2.layout
    shared_errs = {k: _rel(lay2.view(gc, i), lay2.view(gd, i)) for i, k in enumerate(lay2.names)}
    log("headfuse_snake_scale_per_micro_batch", errs=errs, gmax=gmax.tolist(), shared_slice_overflows=shared_overflows,
        shared_slice_errs=shared_errs)
