"""The step's consolidated launches (ABI 10) against the per-call C-ABI kernels, bit for bit.

* The column reductions of one epilogue share one launch pair (`col_reduce_multi`: db0 and the
  in columns of dW0 of the NT_DX0 epilogue, row partials [rows/tile][1+in][H]).  After a step with
  one micro-batch the engine's b0 / W0 gradients must equal `siren_col_reduce` of each segment,
  on both the one-pass (<= 256 partial rows) and the two-pass path.
* The fp16 shadows of every hidden layer are refreshed by one launch (`cast_weights`) after Adam:
  they must equal `siren_cast_weight` of the updated fp32 weights.
"""
from __future__ import annotations

import pytest
import torch

from inr_for_audio_amd import _lib
from inr_for_audio_amd.engine import SirenEngine
from inr_for_audio_amd.models import SirenWithSnakeTanh

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
H = 256


def _engine(rows: int, in_dim: int, seed: int = 0) -> SirenEngine:
    torch.manual_seed(seed)
    model = SirenWithSnakeTanh(in_dim, 1, H, 2, 0, 0, first_omega_0=300.0, hidden_omega_0=30.0)
    g = torch.Generator().manual_seed(seed)
    t = torch.rand(rows, in_dim, generator=g) * 2 - 1
    y = torch.sin(7.0 * t.sum(1)) * 0.5
    return SirenEngine(model, t, y, device=DEV)


@pytest.mark.parametrize("rows,in_dim", [(4096, 1), (4096, 2), (1 << 17, 1), (1 << 17, 2)])
def test_first_layer_partials_match_per_segment_reduce(rows, in_dim):
    eng = _engine(rows, in_dim)
    assert eng.n_micro == 1
    eng._launch_grads()
    torch.cuda.synchronize()
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    prow = eng.rows // lib.siren_nt_tile(eng.rows, H)
    assert (prow > 256) == (rows > 4096)  # both reduce paths are covered
    nred = 1 + in_dim
    base = eng.ws.col_part.data_ptr()
    tmp = torch.empty(64 * H, device=DEV)
    db0 = torch.full((H,), float("nan"), device=DEV)
    _lib.check(lib.siren_col_reduce(base, nred * H, prow, H, db0.data_ptr(), 1, 0, tmp.data_ptr(), s), "col_reduce")
    W0 = torch.full((H, in_dim), float("nan"), device=DEV)
    for j in range(in_dim):
        _lib.check(lib.siren_col_reduce(base + 4 * (1 + j) * H, nred * H, prow, H, W0.data_ptr() + 4 * j, in_dim, 0,
                                        tmp.data_ptr(), s), "col_reduce")
    torch.cuda.synchronize()
    g_b0 = eng.layout.view(eng.grads, eng.ix["b0"])
    g_W0 = eng.layout.view(eng.grads, eng.ix["W0"])
    assert torch.isfinite(db0).all() and torch.isfinite(W0).all()
    assert torch.equal(g_b0, db0)
    assert torch.equal(g_W0, W0)


def test_batched_shadow_cast_matches_per_layer_cast():
    eng = _engine(4096, 1, seed=3)
    eng.step()
    eng.step()
    torch.cuda.synchronize()
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    for i, W in enumerate(eng.W):
        Wh = torch.empty_like(eng.Wh[i])
        WTh = torch.empty_like(eng.WTh[i])
        _lib.check(lib.siren_cast_weight(W.data_ptr(), H, H, Wh.data_ptr(), WTh.data_ptr(), s), "cast_weight")
        torch.cuda.synchronize()
        assert torch.equal(Wh.view(torch.int16), eng.Wh[i].view(torch.int16)), i
        assert torch.equal(WTh.view(torch.int16), eng.WTh[i].view(torch.int16)), i


@pytest.mark.parametrize("mask_all", [True, False])
def test_profile_records_count_launches(mask_all):
    """ABI 10: the run of back-to-back plain forward launches is one profiling record, and
    siren_profile_read still returns the launch count (bench.py's per-launch average divides by
    it).  A 2^17 x 256 SIREN with 3 hidden layers: 2 plain forwards + the fused last layer per
    step, 3 dX launches... per kind, launches = steps x launches per step."""
    lib = _lib.load()
    torch.manual_seed(0)
    model = SirenWithSnakeTanh(1, 1, H, 3, 0, 0, first_omega_0=300.0, hidden_omega_0=30.0)
    t = torch.linspace(-1, 1, 1 << 17).reshape(-1, 1)
    eng = SirenEngine(model, t, torch.sin(9.0 * t[:, 0]), device=DEV)
    L = eng.spec.n_inner
    eng.step()
    torch.cuda.synchronize()
    kinds = _lib.PROF_KINDS
    mask = 0xFFFFFFFF if mask_all else (1 << kinds.index("inner_fwd"))
    _lib.check(lib.siren_profile_mask(mask), "mask")
    _lib.check(lib.siren_profile_enable(4096), "enable")
    try:
        steps = 3
        for _ in range(steps):
            eng.step()
        torch.cuda.synchronize()
        pr = _lib.profile_read()
    finally:
        _lib.check(lib.siren_profile_enable(0), "disable")
        _lib.check(lib.siren_profile_mask(0xFFFFFFFF), "mask")
    fused = pr["head_fwd"][1] > 0 if mask_all else lib.siren_nt_tile(1 << 17, H) == 256
    n_fwd = pr["inner_fwd"][1]
    assert n_fwd == steps * (L - 1 if fused else L), pr
    assert pr["inner_fwd"][0] > 0
    if mask_all:
        assert pr["bwd_dw"][1] == steps * L and pr["bwd_dx"][1] == steps * (L - 1) and pr["bwd_dx0"][1] == steps
    else:
        assert all(n == 0 for k, (ms, n) in pr.items() if k != "inner_fwd")
