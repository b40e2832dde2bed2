"""The C-ABI library loads on a GPU-less host and exports exactly what include/siren_hip.h
declares; argument validation returns status codes without touching the device."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "siren_hip.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?(?:int|int32_t|int64_t|char\s*\*)\s*\**\s*(siren_\w+)\s*\(",
                          src, flags=re.M))


def test_header_parses():
    names = declared()
    assert {"siren_train_step", "siren_apply_update", "siren_inner_fwd", "siren_inner_bwd_dw",
            "siren_adam_step", "siren_plateau_step"} <= names
    assert len(names) >= 24


def test_header_constants_match_binding():
    """The ctypes binding's constants are the header's #defines."""
    from inr_for_audio_amd import _lib
    src = open(HEADER).read()
    defs = dict(re.findall(r"^#define (SIREN_\w+) (\d+)", src, flags=re.M))
    assert int(defs["SIREN_MAX_HIDDEN"]) == _lib.MAX_HIDDEN
    assert int(defs["SIREN_MAX_INNER"]) == _lib.MAX_INNER
    assert int(defs["SIREN_ROW_TILE"]) == _lib.ROW_TILE
    assert int(defs["SIREN_TILEQ_INTS"]) == _lib.TILEQ_INTS
    assert int(defs["SIREN_ABI_VERSION"]) == _lib.ABI_VERSION


def test_library_exports_every_declared_symbol(lib):
    for name in declared():
        assert hasattr(lib, name), name


def test_binding_table_matches_header(lib):
    from inr_for_audio_amd import _lib
    assert set(_lib._SIGS) == declared()


def test_struct_layouts_match(lib):
    """ctypes mirrors of the ABI structs have the C sizes (load() also refuses a mismatch)."""
    import ctypes
    from inr_for_audio_amd import _lib
    for k, st in enumerate(_lib.STRUCTS):
        assert lib.siren_struct_size(k) == ctypes.sizeof(st), st.__name__
    assert lib.siren_struct_size(99) == -1


def test_host_only_helpers(lib):
    assert lib.siren_abi_version() == 12
    assert lib.siren_status_string(0) == b"ok"
    assert b"shape" in lib.siren_status_string(1001)
    assert lib.siren_dw_tile(1 << 20, 1024) == 256 and lib.siren_nt_tile(1 << 20, 1024) == 256
    assert lib.siren_dw_tile(44288, 256) == 128 and lib.siren_nt_tile(44160, 256) == 128
    assert lib.siren_default_splits(1 << 20, 1024) == 16        # 16 tiles x 16 slices = 256 blocks, one per CU
    assert lib.siren_default_splits(220160, 512) == 64          # cfg4: 4 tiles x 64 slices
    assert lib.siren_default_splits(44160, 256) >= 1
    assert lib.siren_slab_floats(1024, 16) == 16 * 1024 * 1024


def test_validation_without_device(lib):
    from inr_for_audio_amd._lib import SirenBatch, SirenGrads, SirenNet
    net = SirenNet()
    assert lib.siren_train_step(None, None, None, None) == 1002          # NULL net
    net.in_dim, net.hidden, net.n_inner = 3, 256, 2
    assert lib.siren_train_step(ctypes.byref(net), ctypes.byref(SirenGrads()),
                                ctypes.byref(SirenBatch()), None) == 1003  # in_dim 3 unsupported
    net.in_dim, net.hidden = 1, 384
    assert lib.siren_forward(ctypes.byref(net), ctypes.byref(SirenBatch()), None) == 1001
    assert lib.siren_inner_fwd(None, None, None, ctypes.c_float(30), 128, 256, None, None, None, None,
                               None, None) == 1002
    assert lib.siren_inner_bwd_dw(1, 1, 100, 256, 1, 0, 1, None) == 1001  # rows % 64
    assert lib.siren_inner_bwd_dw(1, 1, 128, 256, 1, 64, 1, None) == 1003  # bad tile
    assert lib.siren_dw_reduce(1, 1, 256, 0, 1, 1, None, None) == 1003     # tile must be explicit
    assert lib.siren_grad_scale(None, 1, 1, 256, ctypes.c_float(30), 1, None) == 1002
    assert lib.siren_grad_scale(1, 0, 1, 256, ctypes.c_float(30), 1, None) == 1001
    assert lib.siren_first_fwd(1, 3, 1, 1, ctypes.c_float(1.0), 128, 256, 1, 1, None) == 1003
    assert lib.siren_coords_fill_grid(None, 8, 0, 4, 2, None) == 1002
    assert lib.siren_coords_fill_grid(1, 8, 0, 0, 2, None) == 1001        # height 0
    # the fused head: NULL operands, rows not a multiple of 256, a loss mode other than MSE / L1
    f = ctypes.c_float
    assert lib.siren_head_fused_fwd(None, 1, 1, f(30), 1024, 256, 1, 1, f(0), 1, 1024, 1024.0, 0, 1, 1, 1, 1, 1, 1,
                                    1, 1, None) == 1002
    assert lib.siren_head_fused_fwd(1, 1, 1, f(30), 1152, 256, 1, 1, f(0), 1, 1152, 1152.0, 0, 1, 1, 1, 1, 1, 1,
                                    1, 1, None) == 1001
    assert lib.siren_head_fused_fwd(1, 1, 1, f(30), 1024, 256, 1, 1, f(0), 1, 1024, 1024.0, 2, 1, 1, 1, 1, 1, 1,
                                    1, 1, None) == 1003
    # ... and for a last layer of any kind: a Snake without its a, an unknown activation
    A = lambda act, a, rows=1024, lm=0, e=1: lib.siren_head_fused_fwd_act(  # noqa: E731
        1, 1, 1, act, f(30), a, rows, 256, 1, 1, f(0), 1, rows, float(rows), lm, 1, 1, 1, 1, 1, 1, None, 1, 1, e, None)
    assert A(1, None) == 1002
    assert A(1, 1, e=None) == 1002                                         # a Snake needs its E buffer
    assert A(3, 1) == 1003
    assert A(2, None, rows=1152) == 1001
    assert A(2, None, lm=2) == 1003
    assert lib.siren_grad_scale_bound(None, 10, None, 1, 1, 256, 10.0, f(0), 0, f(30), 1, None) == 1002
    assert lib.siren_grad_scale_bound(1, -1, 1, 1, 1, 256, 10.0, f(0), 0, f(30), 1, None) == 1001
    assert lib.siren_grad_scale_bound(1, 10, 1, 1, 1, 256, 10.0, f(0), 3, f(30), 1, None) == 1003
    b = SirenBatch()
    b.loss_mode = 7                                                          # not MSE / L1
    net.hidden = 256
    assert lib.siren_forward(ctypes.byref(net), ctypes.byref(b), None) in (1001, 1002, 1003)


@pytest.mark.parametrize("hidden", [128, 256, 512, 1024])
def test_supported_hidden_sizes_validate(lib, hidden):
    # only shape checks run (NULL outputs make it return before any launch)
    assert lib.siren_head_bwd(None, None, None, None, ctypes.c_float(30), 128, hidden, None, None, None,
                              None, None, None, None) == 1002


@pytest.mark.parametrize("hidden,ok", [(128, True), (1024, True), (2048, True), (3072, True), (4096, True),
                                       (384, False), (1536, False), (5120, False)])
def test_hidden_width_shapes(lib, hidden, ok):
    """Kernel widths: 128, 256, 512, 1024, then multiples of 1024 up to SIREN_MAX_HIDDEN (column windows);
    a width outside them is a shape error before any other check (here the bad tile 64: 1003)."""
    assert lib.siren_inner_bwd_dw(1, 1, 128, hidden, 1, 64, 1, None) == (1003 if ok else 1001)


def test_set_option_ranges(lib):
    """siren_set_option validates every knob on the host (SIREN_OPT_* in siren_hip.h) and leaves
    the defaults restored; SIREN_OPT_NT_QUEUE takes 0 (static walk), 1 (forward modes), 2 (all).
    The product library carries no measurement ablation: SIREN_OPT_NT_DIAG accepts only 0, and
    the retired stagger (5) and prefetch-distance (7) options are rejected; SIREN_OPT_HEAD_FUSE (9)
    takes 0 or 1; the hand-off fault hook SIREN_OPT_HB_FAULT (10) only 0.  SIREN_OPT_NT_PIPE takes the
    measurement forwards 5-7 (one wave per SIMD, gemm_nt1.hip / gemm_nt2.hip) besides -1, 0, 1, 4."""
    bad = 1003  # SIREN_ERR_CONFIG
    for opt, good, wrong in ((0, (0, 128, 256), (64,)), (1, (0, 128, 256), (512,)), (2, (-1, 0, 1, 4, 5, 6, 7), (2, 3, 8, -2)),
                             (3, (-1, 4), (5,)), (4, (0, 16), (-1,)), (5, (), (0, 1)),
                             (6, (0,), (1, 4, 512, 1024, 2, 8)), (7, (), (1, 2)), (8, (0, 1, 2), (3, -1)),
                             (9, (0, 1), (2, -1)), (10, (0,), (1, 1 << 8, -1))):
        for v in good:
            assert lib.siren_set_option(opt, v) == 0, (opt, v)
        for v in wrong:
            assert lib.siren_set_option(opt, v) == bad, (opt, v)
    assert lib.siren_set_option(99, 0) == bad
    for opt, v in ((0, 0), (1, 0), (2, -1), (3, -1), (4, 0), (6, 0), (8, 1), (9, 1)):
        assert lib.siren_set_option(opt, v) == 0


def test_build_id_is_the_source_hash(lib):
    """The library embeds the SHA-256 of the sources it was compiled from (siren_build_id); the build
    step reads it from the file and rebuilds on a mismatch, and _lib.load() refuses a library whose
    id is not the hash of the sources beside it (no file times involved)."""
    import __graft_entry__ as ge
    from inr_for_audio_amd import _lib, buildinfo
    bid = lib.siren_build_id().decode()
    assert re.fullmatch(r"[0-9a-f]{64}", bid)
    assert bid == buildinfo.source_hash() == buildinfo.lib_build_id(ge.LIB)
    assert not ge._stale()
    # the SIREN_DIAG test library: its own defines, its own id
    diag = buildinfo.lib_build_id(ge.DIAG_LIB)
    assert diag == buildinfo.source_hash(ge.DIAG_DEFINES) != bid
    assert _lib.bind(ge.DIAG_LIB, expect_build_id=diag).siren_build_id().decode() == diag
    with pytest.raises(_lib.SirenError, match="other sources"):
        _lib.bind(ge.LIB, expect_build_id="0" * 64)
    # a one-byte change of any source changes the hash
    src = os.path.join(buildinfo.CSRC, "gemm_nt.hip")
    data = open(src, "rb").read()
    try:
        open(src, "wb").write(data + b"\n")
        assert buildinfo.source_hash() != bid and ge._stale()
    finally:
        open(src, "wb").write(data)
    assert buildinfo.source_hash() == bid


def test_diag_library_accepts_the_fault_hook():
    """-DSIREN_DIAG builds take SIREN_OPT_HB_FAULT (the product refuses it: test_set_option_ranges)."""
    import __graft_entry__ as ge
    from inr_for_audio_amd import _lib
    d = _lib.bind(ge.DIAG_LIB)
    for v in (1, (64 << 8) | 1, 0):
        assert d.siren_set_option(10, v) == 0, v
    assert d.siren_set_option(10, -1) == 1003
