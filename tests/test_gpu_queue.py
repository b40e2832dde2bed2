"""Dynamic tile queue of the ping-pong NT GEMM (SIREN_OPT_NT_QUEUE; caller-owned counter sets,
include/siren_hip.h SIREN_TILEQ_INTS).

The queue only changes WHICH persistent block computes a tile, never how, so every output must be
bit-identical to the static walk: forward (with the head partials) over grids where the shards
hold one or several blocks, several launches in a row on one set, a second stream with its own
set, and a set handed over full of garbage (the launcher zeroes it on the stream first).  The
backward modes through the queue (option 2) are checked on the fused step, whose siren_batch
carries the set.  One case is also checked against fp64.
"""
import ctypes
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

F32 = np.float32
H16 = torch.float16


def ok(status, lib):
    assert status == 0, lib.siren_status_string(status)


@pytest.fixture(autouse=True)
def _reset(lib):
    yield
    torch.cuda.synchronize()
    for opt, v in ((0, 0), (2, -1), (4, 0), (8, 1)):
        lib.siren_set_option(opt, v)


def P(t):
    return 0 if t is None else t.data_ptr()


def _inputs(dev, R, H, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    X = (torch.rand(R, H, device=dev, generator=g) * 2 - 1).to(H16)
    lim = math.sqrt(6 / H) / 30
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(H16)
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    hw = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.02
    dZ = (torch.randn(R, H, device=dev, generator=g) * 1e-3).to(H16)
    Cp = (torch.rand(R, H, device=dev, generator=g) * 2 - 1).to(H16)
    t = torch.rand(R, 2, device=dev, generator=g) * 2 - 1
    return X, W, b, hw, dZ, Cp, t


def _run_all(lib, dev, R, H, inp, stream, tq):
    """Forward with and without the head partials; tq: tile-queue set (None: static walk)."""
    X, W, b, hw, dZ, Cp, t = inp
    s = stream.cuda_stream
    res = []
    for head in (False, True):
        Y = torch.full((R, H), float("nan"), dtype=H16, device=dev)
        C = torch.full_like(Y, float("nan"))
        hp = torch.full((H // 128, R), float("nan"), device=dev)
        stream.wait_stream(torch.cuda.current_stream())  # the fills above ran on the current stream
        ok(lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(Y), P(C), P(hw) if head else 0,
                               P(hp) if head else 0, P(tq), s), lib)
        stream.synchronize()
        # the 256-tile launches write H/256 partial rows; the rest stays NaN in both runs
        res += [Y, C] + ([hp[:H // 256]] if head else [])
    return res


def _same(a, b):
    return all(torch.equal(torch.nan_to_num(x.float(), 7.0), torch.nan_to_num(y.float(), 7.0))
               for x, y in zip(a, b))


@pytest.mark.parametrize("R,H,grid", [(4096, 1024, 8), (4096, 1024, 16), (4096, 1024, 24), (4096, 1024, 0),
                                      (3072, 512, 8), (6144, 256, 16),
                                      # 20 tiles: shards of 2 and 3 tiles (uneven eighths)
                                      (2560, 512, 8), (2560, 512, 16)])
def test_queue_bit_identical_to_static_walk(lib, dev, R, H, grid):
    from inr_for_audio_amd._lib import new_tileq
    ok(lib.siren_set_option(0, 256), lib)
    ok(lib.siren_set_option(2, 4), lib)
    ok(lib.siren_set_option(4, grid), lib)
    inp = _inputs(dev, R, H, seed=R + H + grid)
    st = torch.cuda.current_stream()
    ref = _run_all(lib, dev, R, H, inp, st, None)
    tq = new_tileq(dev)
    for _ in range(3):  # back to back on one set
        assert _same(_run_all(lib, dev, R, H, inp, st, tq), ref)
    side = torch.cuda.Stream(device=dev)
    assert _same(_run_all(lib, dev, R, H, inp, side, new_tileq(dev)), ref)
    assert _same(_run_all(lib, dev, R, H, inp, st, tq), ref)


@pytest.mark.parametrize("fill", [1, -1, 1 << 30, "random"])
def test_queue_set_handed_over_dirty(lib, dev, fill):
    """A counter set left non-zero (an aborted launch, a caller's garbage) must not change any
    output: every queue launch zeroes its set on the stream first, and every pulled tile id is
    range-checked, so no block can skip a tile or walk past its shard."""
    from inr_for_audio_amd._lib import TILEQ_INTS
    R, H, grid = 4096, 1024, 16
    ok(lib.siren_set_option(0, 256), lib)
    ok(lib.siren_set_option(2, 4), lib)
    ok(lib.siren_set_option(4, grid), lib)
    inp = _inputs(dev, R, H, seed=5)
    st = torch.cuda.current_stream()
    ref = _run_all(lib, dev, R, H, inp, st, None)
    if fill == "random":
        g = torch.Generator(device=dev).manual_seed(1)
        tq = torch.randint(-(1 << 31), (1 << 31) - 1, (TILEQ_INTS,), dtype=torch.int64, device=dev,
                           generator=g).to(torch.int32)
    else:
        tq = torch.full((TILEQ_INTS,), fill, dtype=torch.int32, device=dev)
    assert _same(_run_all(lib, dev, R, H, inp, st, tq), ref)


@pytest.mark.parametrize("act", ["snake", "tanh"])
@pytest.mark.parametrize("grid", [8, 0])
def test_queue_act_forward_bit_identical(lib, dev, act, grid):
    """The Snake / Tanh forward epilogues (modes NT_FWD_SNAKE / NT_FWD_TANH, with and without the
    head partials) from the queue == from the static walk."""
    R, H = 4096, 512
    code = {"snake": 1, "tanh": 2}[act]  # SIREN_ACT_SNAKE, SIREN_ACT_TANH
    ok(lib.siren_set_option(0, 256), lib)
    ok(lib.siren_set_option(2, 4), lib)
    ok(lib.siren_set_option(4, grid), lib)
    from inr_for_audio_amd._lib import new_tileq
    X, W, b, hw, *_ = _inputs(dev, R, H, seed=11)
    a = 0.5 + torch.rand(H, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def run(tq):
        res = []
        for head in (False, True):
            Y = torch.full((R, H), float("nan"), dtype=H16, device=dev)
            C = torch.full_like(Y, float("nan"))
            E = torch.full_like(Y, float("nan"))
            hp = torch.full((H // 128, R), float("nan"), device=dev)
            ok(lib.siren_inner_fwd_act(P(X), P(W), P(b), code, ctypes.c_float(1.0), P(a), R, H, P(Y), P(C),
                                       P(E) if act == "snake" else 0, P(hw) if head else 0, P(hp) if head else 0,
                                       P(tq), s), lib)
            torch.cuda.synchronize()
            res += [Y, C] + ([E] if act == "snake" else []) + ([hp[:H // 256]] if head else [])
        return res
    ref = run(None)
    assert _same(run(new_tileq(dev)), ref)


def test_queue_forward_vs_fp64(lib, dev):
    R, H = 4096, 512
    ok(lib.siren_set_option(0, 256), lib)
    ok(lib.siren_set_option(2, 4), lib)
    ok(lib.siren_set_option(4, 16), lib)
    from inr_for_audio_amd._lib import new_tileq
    X, W, b, hw, *_ = _inputs(dev, R, H, seed=3)
    Y, C, hp = _run_all(lib, dev, R, H, _inputs(dev, R, H, seed=3), torch.cuda.current_stream(), new_tileq(dev))[2:]
    a = 30.0 * (X.double() @ W.double().t() + b.double())
    for got, ref in ((Y, torch.sin(a)), (C, torch.cos(a))):
        err = (got.double() - ref).abs() - ref.abs() * 2.0 ** -11 - 2e-5
        assert float(err.max()) <= 0
    head = hp.double().sum(0)
    assert float((head - torch.sin(a) @ hw.double()).abs().max()) < 1e-4


def _engine(dev, seed, H=512, n=65536):
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    torch.manual_seed(seed)
    model = SirenWithSnakeTanh(1, 1, H, 2, 0, 0, first_omega_0=2000.0, hidden_omega_0=30.0)
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    y = torch.sin(37 * t + seed) * 0.5
    return SirenEngine(model, t, y, device=dev)


def test_queue_every_mode_in_the_fused_step(lib, dev):
    """SIREN_OPT_NT_QUEUE 2 sends the dX / dX0 launches of siren_train_step through the batch's
    set too: the step's gradients are bit-identical to the static walk's (0) and the default (1)."""
    assert lib.siren_nt_tile(65536, 512) == 256
    grads = []
    for q in (0, 1, 2):
        ok(lib.siren_set_option(8, q), lib)
        e = _engine(dev, 0)
        e.step()
        torch.cuda.synchronize()
        grads.append(e.grads.clone())
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[0], grads[2])


def test_two_captured_graphs_replayed_concurrently(lib, dev):
    """Two engines, each step captured as a HIP graph (each workspace owns its counter set), are
    replayed at the same time on two streams: both stay bit-identical to their eager twins.  (The
    round-2 design keyed one global set per capture stream, which two replays could share.)"""
    eager = [_engine(dev, s) for s in (1, 2)]
    graphed = [_engine(dev, s) for s in (1, 2)]
    for e in eager:
        for _ in range(4):
            e.step()
    for e in graphed:
        e.step()
        e.capture_graph()
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    for _ in range(3):
        for e, st in zip(graphed, streams):
            with torch.cuda.stream(st):
                e.graph.replay()
    torch.cuda.synchronize()
    for a, b in zip(eager, graphed):
        assert torch.equal(a.params, b.params)
