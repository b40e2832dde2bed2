"""Per-kernel parity of libsiren_hip.so against the CPU oracle (called through the C-ABI).

Tolerances: fp16-stored outputs (Y = sin, C = cos, dZ) must be within one fp16 rounding of
the fp64 answer computed from the same fp16 inputs (|err| <= 2^-11 |x| + small fp32
accumulation slack); fp32 reductions within 1e-5 relative; Adam, the coordinate grid, the
weight shadows and the backward scale bit-exact.  The backward storage scale S (gscale =
{S, 1/S}) is exercised both as NULL (S = 1) and as a non-trivial power of two.
"""
import ctypes
import math

import numpy as np
import pytest
import torch

from inr_for_audio_amd._lib import new_tileq
from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu

F32 = np.float32


def ptr(t):
    return 0 if t is None else t.data_ptr()


def S():
    return torch.cuda.current_stream().cuda_stream


def ok(status, lib):
    assert status == 0, lib.siren_status_string(status)


_KEEP = []


def to_dev(a, dev, dtype=torch.float32):
    """Host array -> device tensor.  Kept alive (module list) so a pointer taken from a
    temporary inside one call can never be recycled by the caching allocator."""
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=F32)).to(dev).to(dtype)
    _KEEP.append(t)
    return t


@pytest.fixture(autouse=True)
def _release():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


@pytest.fixture(params=[(128, 0, 0), (256, 0, 0), (256, 1, 0), (256, 1, 2), (256, 1, 3), (256, 4, 0),
                        (256, 4, 2), (256, 4, 3), (256, 4, 5), (256, 5, 0), (256, 5, 3), (256, 6, 0),
                        (256, 6, 3), (256, 7, 0), (256, 7, 3)],
                ids=lambda p: f"t{p[0]}p{p[1]}g{p[2]}")
def nt_tile(request, lib):
    """Force the NT GEMM tile edge, persistence and persistent grid size (siren_set_option)
    for one test; grid 2 makes every block walk several tiles across the LDS ring."""
    tile, pipe, grid = request.param
    ok(lib.siren_set_option(0, tile), lib)
    ok(lib.siren_set_option(2, pipe), lib)
    ok(lib.siren_set_option(4, grid), lib)
    yield tile
    lib.siren_set_option(0, 0)
    lib.siren_set_option(2, -1)
    lib.siren_set_option(4, 0)


@pytest.fixture(params=[0, 1, 2, 3, 4], ids=lambda p: f"p{p}")
def tn_pipe(request, lib):
    ok(lib.siren_set_option(3, request.param), lib)
    yield request.param
    lib.siren_set_option(3, -1)


def _skip_tile(tile, R, H):
    if tile == 256 and (R % 256 or H % 256):
        pytest.skip("256-tile needs rows and hidden multiples of 256")


H16 = torch.float16


def f16_np(t: torch.Tensor) -> np.ndarray:
    return t.float().cpu().numpy()


def within_f16(got, ref, abs_slack=1e-5):
    """|got - ref| <= 2^-11 * |ref| + abs_slack elementwise (one fp16 rounding + slack;
    2^-25 covers the subnormal spacing)."""
    err = np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64))
    bound = np.abs(np.asarray(ref, np.float64)) * 2.0 ** -11 + abs_slack + 2.0 ** -25
    return float(np.max(err - bound))


def gscale_dev(dev, k):
    """{S, 1/S} with S = 2^k, or None (NULL: unscaled)."""
    return None if k is None else to_dev(np.array([2.0 ** k, 2.0 ** -k], F32), dev)


@pytest.mark.parametrize("n,rows,offset", [(1, 128, 0), (7, 128, 0), (44100, 44160, 0),
                                          (1 << 20, 1 << 20, 0), (441000, 1024, 220000),
                                          (441000, 1024, 440500)])
def test_coords_fill_bit_exact(lib, dev, n, rows, offset):
    t = torch.full((rows,), float("nan"), device=dev)
    ok(lib.siren_coords_fill(ptr(t), rows, offset, n, S()), lib)
    got = t.cpu().numpy()
    ref_full = orc.linspace_f32(n)
    valid = max(0, min(rows, n - offset))
    assert np.array_equal(got[:valid], ref_full[offset:offset + valid])
    assert np.all(got[valid:] == 0)


@pytest.mark.parametrize("in_dim", [1, 2])
@pytest.mark.parametrize("omega0", [30.0, 1000.0, 22000.0])
def test_first_fwd(lib, dev, in_dim, omega0):
    rng = np.random.default_rng(1)
    R, H = 1024, 256
    t = rng.uniform(-1, 1, (R, in_dim)).astype(F32)
    W0 = rng.uniform(-1, 1, (H, in_dim)).astype(F32)
    b0 = rng.uniform(-1, 1, H).astype(F32)
    Y0 = torch.empty(R, H, dtype=H16, device=dev)
    C0 = torch.empty_like(Y0)
    ok(lib.siren_first_fwd(ptr(to_dev(t, dev)), in_dim, ptr(to_dev(W0, dev)), ptr(to_dev(b0, dev)),
                           ctypes.c_float(omega0), R, H, ptr(Y0), ptr(C0), S()), lib)
    a0 = orc.first_preact(t, W0, b0, omega0)  # fp32 restatement (torch addmm rounding)
    for got, ref in ((f16_np(Y0), orc.sin32(a0)), (f16_np(C0), orc.cos32(a0))):
        assert within_f16(got, ref, abs_slack=1e-6) <= 0
        assert np.mean(got == orc.f16_round(ref)) > 0.995


def _inner_inputs(rng, R, H):
    X = orc.f16_round(rng.uniform(-1, 1, (R, H)).astype(F32))
    lim = math.sqrt(6 / H) / 30
    W = rng.uniform(-lim, lim, (H, H)).astype(F32)
    b = rng.uniform(-1 / math.sqrt(H), 1 / math.sqrt(H), H).astype(F32)
    return X, W, b


@pytest.mark.parametrize("R,H", [(256, 128), (512, 256), (384, 512), (256, 1024), (768, 512)])
@pytest.mark.parametrize("head", [False, True])
def test_inner_fwd(lib, dev, R, H, head, nt_tile):
    _skip_tile(nt_tile, R, H)
    rng = np.random.default_rng(2)
    X, W, b = _inner_inputs(rng, R, H)
    Wh = orc.f16_round(W)
    hw = rng.uniform(-0.01, 0.01, H).astype(F32)
    Y = torch.empty(R, H, dtype=H16, device=dev)
    C = torch.empty_like(Y)
    hp = torch.zeros(H // 128, R, device=dev)
    ok(lib.siren_inner_fwd(ptr(to_dev(X, dev, H16)), ptr(to_dev(Wh, dev, H16)),
                           ptr(to_dev(b, dev)), ctypes.c_float(30.0), R, H, ptr(Y), ptr(C),
                           ptr(to_dev(hw, dev)) if head else None, ptr(hp) if head else None,
                           ptr(new_tileq(dev)), S()), lib)
    a = 30.0 * (X.astype(np.float64) @ Wh.astype(np.float64).T + b)
    assert within_f16(f16_np(Y), np.sin(a), 2e-5) <= 0
    assert within_f16(f16_np(C), np.cos(a), 2e-5) <= 0
    if head:
        ref = np.sin(a) @ hw.astype(np.float64)
        got = hp.cpu().numpy().astype(np.float64).sum(0)
        assert np.max(np.abs(got - ref)) < 1e-4 * max(1.0, np.max(np.abs(ref)))


@pytest.mark.parametrize("R,H,grid", [(512, 256, 0), (4096, 512, 7), (65536, 1024, 0), (220160, 512, 0),
                                      (262144, 1024, 37)])
def test_inner_fwd_pipes_bit_identical(lib, dev, R, H, grid):
    """The one-wave-per-SIMD forwards (SIREN_OPT_NT_PIPE 5: 128x256 tiles with the epilogue under the
    next tile's MFMAs, gemm_nt1.hip; 7: the same K loop with the epilogue at the tile's end; 6: 256x256
    tiles, BK 32, 4-stage ring, gemm_nt2.hip) against the
    ping-pong forward (pipe 4): Y and C bit-identical (same K order per output, same epilogue
    arithmetic), every block walking 1 .. 100+ tiles."""
    g = torch.Generator(device=dev).manual_seed(R + H)
    X = torch.sin(torch.rand(R, H, device=dev, generator=g) * 6.2831853).to(H16)
    lim = math.sqrt(6 / H) / 30
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(H16)
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    tq = new_tileq(dev)
    outs = {}
    try:
        ok(lib.siren_set_option(0, 256), lib)
        ok(lib.siren_set_option(4, grid), lib)
        for pipe in (4, 5, 6, 7):
            ok(lib.siren_set_option(2, pipe), lib)
            Y = torch.full((R, H), float("nan"), dtype=H16, device=dev)
            C = torch.full_like(Y, float("nan"))
            ok(lib.siren_inner_fwd(ptr(X), ptr(W), ptr(b), ctypes.c_float(30.0), R, H, ptr(Y), ptr(C), None,
                                   None, ptr(tq), S()), lib)
            torch.cuda.synchronize()
            outs[pipe] = (Y.view(torch.int16), C.view(torch.int16))
    finally:
        lib.siren_set_option(0, 0)
        lib.siren_set_option(2, -1)
        lib.siren_set_option(4, 0)
    for pipe in (5, 6, 7):
        assert torch.equal(outs[pipe][0], outs[4][0]), pipe
        assert torch.equal(outs[pipe][1], outs[4][1]), pipe


def test_head_loss(lib, dev):
    rng = np.random.default_rng(3)
    R, nparts, n_valid, n_total = 1024, 4, 1000, 5000
    hp = rng.normal(size=(nparts, R)).astype(F32)
    y = rng.normal(size=R).astype(F32)
    bh = np.array([0.25], F32)
    out = torch.empty(R, device=dev)
    g = torch.empty(R, device=dev)
    sse = torch.empty((R + 255) // 256, device=dev)
    gs = torch.empty_like(sse)
    gm = torch.empty_like(sse)
    ok(lib.siren_head_loss(ptr(to_dev(hp, dev)), nparts, R, ptr(to_dev(bh, dev)), ptr(to_dev(y, dev)),
                           n_valid, ctypes.c_double(n_total), ptr(out), ptr(g), ptr(sse), ptr(gs),
                           ptr(gm), S()),
       lib)
    o_ref = hp.astype(np.float64).sum(0) + 0.25
    assert np.allclose(out.cpu().numpy(), o_ref, atol=1e-5)
    g_ref = np.where(np.arange(R) < n_valid, (o_ref - y) * (2.0 / n_total), 0.0)
    assert np.allclose(g.cpu().numpy(), g_ref, rtol=1e-5, atol=1e-9)
    assert abs(sse.cpu().numpy().astype(np.float64).sum() - np.sum((o_ref - y)[:n_valid] ** 2)) < 1e-3
    assert abs(gs.cpu().numpy().astype(np.float64).sum() - g_ref.sum()) < 1e-6
    g_dev = g.cpu().numpy()
    assert np.array_equal(gm.cpu().numpy(), np.abs(g_dev).reshape(-1, 256).max(1))


@pytest.mark.parametrize("gmag,wmag,omega", [(1e-3, 0.01, 30.0), (3e-10, 0.2, 30.0), (0.0, 0.1, 30.0),
                                             (5e-6, 1e-30, 3000.0), (1.0, 1.0, 1.0)])
def test_grad_scale_bit_exact(lib, dev, gmag, wmag, omega):
    rng = np.random.default_rng(12)
    R, H = 4096, 512
    g = (rng.normal(size=R) * gmag).astype(F32)
    w = (rng.uniform(-1, 1, H) * wmag).astype(F32)
    part = np.abs(g).reshape(-1, 256).max(1).astype(F32)
    out = torch.zeros(2, device=dev)
    ok(lib.siren_grad_scale(ptr(to_dev(part, dev)), part.size, ptr(to_dev(w, dev)), H,
                            ctypes.c_float(omega), ptr(out), S()), lib)
    s_ref = orc.grad_scale(g, w, omega)
    got = out.cpu().numpy()
    assert got[0] == np.float32(s_ref) and got[1] == np.float32(1.0 / s_ref)
    bound = float(np.max(np.abs(g))) * float(np.max(np.abs(w))) * omega
    if bound > 0:
        assert 2.0 ** 5 <= bound * s_ref < 2.0 ** 6 or s_ref in (2.0 ** 100, 2.0 ** -100)


@pytest.mark.parametrize("H", [128, 256, 1024])
@pytest.mark.parametrize("gmag,k", [(1e-3, None), (1e-9, 27)])
def test_head_bwd(lib, dev, H, gmag, k):
    """dZ is stored x S (k = log2 S; 1e-9 gradients would underflow fp16 unscaled); the db /
    dw_head partials stay unscaled."""
    rng = np.random.default_rng(4)
    R = 512
    C = orc.f16_round(rng.uniform(-1, 1, (R, H)).astype(F32))
    Y = orc.f16_round(rng.uniform(-1, 1, (R, H)).astype(F32))
    g = rng.normal(size=R).astype(F32) * gmag
    w = rng.uniform(-0.01, 0.01, H).astype(F32)
    dZ = torch.empty(R, H, dtype=H16, device=dev)
    dbp = torch.empty(R // 128, H, device=dev)
    dwp = torch.empty(R // 128, H, device=dev)
    ok(lib.siren_head_bwd(ptr(to_dev(C, dev, H16)), ptr(to_dev(Y, dev, H16)),
                          ptr(to_dev(g, dev)), ptr(to_dev(w, dev)), ctypes.c_float(30.0), R, H,
                          ptr(gscale_dev(dev, k)), ptr(dZ), ptr(dbp), ptr(dwp), None, None, S()), lib)
    sc = 2.0 ** (k or 0)
    dz_ref = g[:, None].astype(np.float64) * w[None, :] * C * 30.0
    assert within_f16(f16_np(dZ), dz_ref * sc, 1e-12) <= 0
    # fp32 partial sums vs fp64, tolerance relative to the sum of |terms| (cancellation)
    gy = g[:, None].astype(np.float64) * Y
    for got, terms in ((dbp, dz_ref), (dwp, gy)):
        err = np.abs(got.cpu().numpy().astype(np.float64).sum(0) - terms.sum(0))
        assert np.all(err <= 1e-5 * np.abs(terms).sum(0) + 1e-12)


@pytest.mark.parametrize("R,H", [(256, 128), (512, 256), (256, 1024), (768, 512)])
@pytest.mark.parametrize("k", [None, 9])
def test_inner_bwd_dx(lib, dev, R, H, k, nt_tile):
    """dZprev carries the input's scale; the db partials come out x 1/S."""
    _skip_tile(nt_tile, R, H)
    rng = np.random.default_rng(5)
    dZ = orc.f16_round((rng.normal(size=(R, H)) * 1e-3).astype(F32))
    _, W, _ = _inner_inputs(rng, R, H)
    Wh = orc.f16_round(W)
    Cp = orc.f16_round(rng.uniform(-1, 1, (R, H)).astype(F32))
    out = torch.empty(R, H, dtype=H16, device=dev)
    dbp = torch.zeros(R // 128, H, device=dev)  # R / siren_nt_tile rows are written
    WT = np.ascontiguousarray(Wh.T)
    ok(lib.siren_inner_bwd_dx(ptr(to_dev(dZ, dev, H16)), ptr(to_dev(WT, dev, H16)),
                              ptr(to_dev(Cp, dev, H16)), ctypes.c_float(30.0), R, H,
                              ptr(gscale_dev(dev, k)), ptr(out), ptr(dbp), S()), lib)
    ref = (dZ.astype(np.float64) @ Wh.astype(np.float64)) * Cp * 30.0
    scale = np.max(np.abs(ref))
    assert within_f16(f16_np(out), ref, 1e-5 * scale) <= 0
    db = dbp.cpu().numpy().astype(np.float64).sum(0) * 2.0 ** (k or 0)
    assert np.max(np.abs(db - ref.sum(0))) < 1e-4 * np.max(np.abs(ref.sum(0))) + 1e-6 * scale


@pytest.mark.parametrize("in_dim", [1, 2])
@pytest.mark.parametrize("omega0", [1000.0, 22000.0])
def test_first_bwd_dx(lib, dev, in_dim, omega0, nt_tile):
    rng = np.random.default_rng(6)
    R, H = 512, 256
    k = 5 if in_dim == 2 else None
    dZ1 = orc.f16_round((rng.normal(size=(R, H)) * 1e-3).astype(F32))
    _, W, _ = _inner_inputs(rng, R, H)
    Wh = orc.f16_round(W)
    t = rng.uniform(-1, 1, (R, in_dim)).astype(F32)
    W0 = rng.uniform(-1 / in_dim, 1 / in_dim, (H, in_dim)).astype(F32)
    b0 = rng.uniform(-1, 1, H).astype(F32)
    part = torch.zeros(R // 128, 1 + in_dim, H, device=dev)
    WT = np.ascontiguousarray(Wh.T)
    A0 = orc.first_preact(t, W0, b0, omega0)
    C0 = orc.f16_round(orc.cos32(A0))  # as siren_first_fwd stores it
    ok(lib.siren_first_bwd_dx(ptr(to_dev(dZ1, dev, H16)), ptr(to_dev(WT, dev, H16)),
                              ptr(to_dev(C0, dev, H16)), ptr(to_dev(t, dev)), in_dim,
                              ctypes.c_float(omega0), R, H, ptr(gscale_dev(dev, k)), ptr(part), S()), lib)
    dz0 = (dZ1.astype(np.float64) @ Wh.astype(np.float64)) * C0 * omega0
    got = part.cpu().numpy().astype(np.float64).sum(0) * 2.0 ** (k or 0)
    ref_db = dz0.sum(0)
    scale = np.max(np.abs(dz0)) * math.sqrt(R)
    assert np.max(np.abs(got[0] - ref_db)) < 1e-4 * scale
    for j in range(in_dim):
        ref_w = (dz0 * t[:, j:j + 1]).sum(0)
        assert np.max(np.abs(got[1 + j] - ref_w)) < 1e-4 * scale


@pytest.mark.parametrize("R,H,splits,tile", [(256, 128, 1, 128), (1024, 256, 3, 128), (2048, 256, 16, 128),
                                             (512, 1024, 2, 128), (640, 512, 5, 128), (1024, 256, 3, 256),
                                             (2048, 512, 7, 256), (512, 1024, 2, 256), (320, 256, 9, 256)])
def test_inner_bwd_dw(lib, dev, R, H, splits, tile, tn_pipe):
    if tile == 128 and tn_pipe != 0:
        pytest.skip("pipeline variants apply to the 256x256 tile")
    rng = np.random.default_rng(7)
    k = 12 if splits % 2 else None   # odd split counts also check the 1/S of dw_reduce
    Y = orc.f16_round(rng.uniform(-1, 1, (R, H)).astype(F32))
    dZ = orc.f16_round((rng.normal(size=(R, H)) * 1e-3).astype(F32))
    slab = torch.empty(int(lib.siren_slab_floats(H, splits)), device=dev)
    grad = torch.full((H, H), 0.5, device=dev)
    ok(lib.siren_inner_bwd_dw(ptr(to_dev(Y, dev, H16)), ptr(to_dev(dZ, dev, H16)),
                              R, H, splits, tile, ptr(slab), S()), lib)
    ok(lib.siren_dw_reduce(ptr(slab), splits, H, tile, ptr(grad), 1, ptr(gscale_dev(dev, k)), S()), lib)
    ref = (dZ.astype(np.float64).T @ Y.astype(np.float64)) * 2.0 ** -(k or 0) + 0.5
    got = grad.cpu().numpy().astype(np.float64)
    # + one fp32 half-ulp of the 0.5 accumulated into
    assert np.max(np.abs(got - ref)) < 1e-5 * np.max(np.abs(ref - 0.5)) + 1e-7 * 2.0 ** -(k or 0) + 3e-8


@pytest.mark.parametrize("H,splits,tile", [(256, 15, 256), (256, 16, 256), (256, 17, 256), (256, 256, 256),
                                           (512, 33, 256), (256, 7, 128), (256, 40, 128)])
def test_dw_reduce_split_order(lib, dev, H, splits, tile):
    """The slab reduce sums the splits strictly in order s = 0, 1, ..., splits-1 in fp32 (its loads go
    out 16 at a time, the last chunk too): checked bit for bit against numpy's sequential fp32 sum on
    a slab whose magnitudes make the order matter.  Which slab position lands in which dW entry is
    the kernel's MFMA-order decode, so the two are compared as sorted multisets."""
    rng = np.random.default_rng(11)
    n = int(lib.siren_slab_floats(H, splits)) // splits
    slab = (rng.normal(size=(splits, n)) * 10.0 ** rng.uniform(-3, 3, size=(splits, n))).astype(F32)
    ref = slab[0].copy()
    for s in range(1, splits):
        ref = (ref + slab[s]).astype(F32)
    grad = torch.full((H, H), 7.0, device=dev)
    ok(lib.siren_dw_reduce(ptr(to_dev(slab.reshape(-1), dev)), splits, H, tile, ptr(grad), 0, None, S()), lib)
    got = grad.cpu().numpy().reshape(-1)
    assert np.array_equal(np.sort(got).view(np.uint32), np.sort(ref).view(np.uint32))


def test_col_reduce(lib, dev):
    rng = np.random.default_rng(8)
    for nrows, ncols, stride in [(3, 70, 1), (300, 256, 1), (8192, 1024, 2)]:
        part = rng.normal(size=(nrows, ncols)).astype(F32)
        out = torch.full((ncols * stride,), 1.0, device=dev)
        tmp = torch.empty(64, ncols, device=dev)
        ok(lib.siren_col_reduce(ptr(to_dev(part, dev)), ncols, nrows, ncols, ptr(out), stride, 1, ptr(tmp),
                                S()), lib)
        got = out.cpu().numpy()[::stride]
        assert np.allclose(got, part.astype(np.float64).sum(0) + 1.0, rtol=1e-5, atol=1e-4)


def _state_tensor(dev, **kw):
    from inr_for_audio_amd._lib import SirenOptState
    st = SirenOptState()
    st.lr, st.best, st.step = kw.get("lr", 1e-3), math.inf, kw.get("step", 0.0)
    st.min_lr, st.factor, st.threshold, st.eps_lr = kw.get("min_lr", 1e-6), 0.8, 1e-4, 1e-8
    st.patience = kw.get("patience", 200)
    st.beta1, st.beta2, st.eps = 0.9, 0.999, 1e-8
    return torch.frombuffer(bytearray(bytes(st)), dtype=torch.uint8).to(dev)


def _read_state(t):
    from inr_for_audio_amd._lib import SirenOptState
    return SirenOptState.from_buffer_copy(bytes(t.cpu().numpy().tobytes()))


def test_adam_bit_exact(lib, dev):
    rng = np.random.default_rng(9)
    n = 100003
    p = (rng.normal(size=n) * 0.05).astype(F32)
    m = np.zeros(n, F32)
    v = np.zeros(n, F32)
    pd, md, vd = to_dev(p, dev), to_dev(m, dev), to_dev(v, dev)
    for step in range(1, 6):
        g = (rng.normal(size=n) * 10.0 ** rng.uniform(-6, 0, n)).astype(F32)
        st = _state_tensor(dev, lr=1e-3 * step, step=float(step - 1))
        ok(lib.siren_adam_step(ptr(pd), ptr(to_dev(g, dev)), ptr(md), ptr(vd), n, ptr(st), S()), lib)
        p, m, v = orc.adam_step(p, g, m, v, step, 1e-3 * step)
        assert np.array_equal(md.cpu().numpy(), m)
        assert np.array_equal(vd.cpu().numpy(), v)
        assert np.array_equal(pd.cpu().numpy(), p)


def test_plateau_trace(lib, dev):
    rng = np.random.default_rng(10)
    steps, patience = 400, 20
    st = _state_tensor(dev, lr=1e-3, patience=patience, min_lr=2e-4)
    lh = torch.zeros(steps, device=dev)
    rh = torch.zeros(steps, dtype=torch.float64, device=dev)
    sse = torch.zeros(1, device=dev)
    ref = orc.Plateau(1e-3, patience=patience, min_lr=2e-4)
    losses = np.concatenate([np.linspace(1, 0.5, 100), 0.5 + 0.01 * rng.random(300)]).astype(F32)
    n_total = 1000.0
    for k in range(steps):
        sse.fill_(float(losses[k]) * n_total)
        ok(lib.siren_plateau_step(ptr(st), ptr(sse), ctypes.c_double(n_total), ptr(lh), ptr(rh), steps, S()),
           lib)
        loss32 = float(np.float32(np.float64(np.float32(float(losses[k]) * n_total)) / n_total))
        ref.step(loss32)
    got_lr = rh.cpu().numpy()
    s = _read_state(st)
    assert s.step == steps and s.last_epoch == steps
    assert abs(got_lr[-1] - ref.lr) < 1e-15
    assert s.num_bad == ref.num_bad


@pytest.mark.parametrize("H", [128, 1024])
def test_cast_weight(lib, dev, H):
    rng = np.random.default_rng(11)
    W = rng.normal(size=(H, H)).astype(F32)
    Wh = torch.empty(H, H, dtype=H16, device=dev)
    WTh = torch.empty_like(Wh)
    ok(lib.siren_cast_weight(ptr(to_dev(W, dev)), H, H, ptr(Wh), ptr(WTh), S()), lib)
    assert np.array_equal(f16_np(Wh), orc.f16_round(W))
    assert np.array_equal(f16_np(WTh), orc.f16_round(W).T)
