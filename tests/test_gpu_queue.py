"""Dynamic tile queue of the ping-pong NT GEMM (SIREN_OPT_NT_QUEUE, gemm_nt.hip tileq_*).

The queue only changes WHICH persistent block computes a tile, never how, so every output must be
bit-identical to the static walk: forward (with the head partials), dX and dX into layer 0, over
grids where the shards hold one or several blocks, several launches in a row (the queue re-zeroes
itself) and a second stream (its own counter set).  One case is also checked against fp64.
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


def _run_all(lib, dev, R, H, inp, stream):
    X, W, b, hw, dZ, Cp, t = inp
    s = stream.cuda_stream
    Y = torch.full((R, H), float("nan"), dtype=H16, device=dev)
    C = torch.full_like(Y, float("nan"))
    hp = torch.full((H // 128, R), float("nan"), device=dev)
    dZp = torch.full_like(Y, float("nan"))
    dbp = torch.full((R // 128, H), float("nan"), device=dev)
    p0 = torch.full((R // 128, 3, H), float("nan"), device=dev)
    WT = W.t().contiguous()
    stream.wait_stream(torch.cuda.current_stream())  # the fills above ran on the current stream
    ok(lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(Y), P(C), P(hw), P(hp), s), lib)
    ok(lib.siren_inner_bwd_dx(P(dZ), P(WT), P(Cp), ctypes.c_float(30.0), R, H, None, P(dZp), P(dbp), s), lib)
    ok(lib.siren_first_bwd_dx(P(dZ), P(WT), P(Cp), P(t), 2, ctypes.c_float(3000.0), R, H, None, P(p0), s), lib)
    stream.synchronize()
    # the 256-tile launches write R/256 partial rows; the rest stays NaN in both runs
    return [Y, C, hp[:H // 256], dZp, dbp[:R // 256], p0[:R // 256]]


def _same(a, b):
    return all(torch.equal(torch.nan_to_num(x.float(), 7.0), torch.nan_to_num(y.float(), 7.0))
               for x, y in zip(a, b))


@pytest.mark.parametrize("R,H,grid", [(4096, 1024, 8), (4096, 1024, 16), (4096, 1024, 24), (4096, 1024, 0),
                                      (3072, 512, 8), (6144, 256, 16),
                                      # 20 tiles: shards of 2 and 3 tiles (uneven eighths)
                                      (2560, 512, 8), (2560, 512, 16)])
def test_queue_bit_identical_to_static_walk(lib, dev, R, H, grid):
    ok(lib.siren_set_option(0, 256), lib)
    ok(lib.siren_set_option(2, 4), lib)
    ok(lib.siren_set_option(4, grid), lib)
    inp = _inputs(dev, R, H, seed=R + H + grid)
    st = torch.cuda.current_stream()
    ok(lib.siren_set_option(8, 0), lib)
    ref = _run_all(lib, dev, R, H, inp, st)
    ok(lib.siren_set_option(8, 2), lib)  # every mode
    for _ in range(3):  # back to back: each launch's last block re-zeroes the queue
        assert _same(_run_all(lib, dev, R, H, inp, st), ref)
    side = torch.cuda.Stream(device=dev)
    assert _same(_run_all(lib, dev, R, H, inp, side), ref)
    assert _same(_run_all(lib, dev, R, H, inp, st), ref)


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
    X, W, b, hw, *_ = _inputs(dev, R, H, seed=11)
    a = 0.5 + torch.rand(H, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def run():
        res = []
        for head in (False, True):
            Y = torch.full((R, H), float("nan"), dtype=H16, device=dev)
            C = torch.full_like(Y, float("nan"))
            E = torch.full_like(Y, float("nan"))
            hp = torch.full((H // 128, R), float("nan"), device=dev)
            ok(lib.siren_inner_fwd_act(P(X), P(W), P(b), code, ctypes.c_float(1.0), P(a), R, H, P(Y), P(C),
                                       P(E) if act == "snake" else 0, P(hw) if head else 0, P(hp) if head else 0,
                                       s), lib)
            torch.cuda.synchronize()
            res += [Y, C] + ([E] if act == "snake" else []) + ([hp[:H // 256]] if head else [])
        return res
    ok(lib.siren_set_option(8, 0), lib)
    ref = run()
    ok(lib.siren_set_option(8, 1), lib)
    assert _same(run(), ref)


def test_queue_forward_vs_fp64(lib, dev):
    R, H = 4096, 512
    ok(lib.siren_set_option(0, 256), lib)
    ok(lib.siren_set_option(2, 4), lib)
    ok(lib.siren_set_option(4, 16), lib)
    X, W, b, hw, *_ = _inputs(dev, R, H, seed=3)
    Y, C, hp = _run_all(lib, dev, R, H, _inputs(dev, R, H, seed=3), torch.cuda.current_stream())[:3]
    a = 30.0 * (X.double() @ W.double().t() + b.double())
    for got, ref in ((Y, torch.sin(a)), (C, torch.cos(a))):
        err = (got.double() - ref).abs() - ref.abs() * 2.0 ** -11 - 2e-5
        assert float(err.max()) <= 0
    head = hp.double().sum(0)
    assert float((head - torch.sin(a) @ hw.double()).abs().max()) < 1e-4
