"""ctypes binding of libsiren_hip.so (the C-ABI declared in include/siren_hip.h).

This is the only place Python touches the native library.  There is deliberately no
fallback: if the shared object is missing or was built for another ABI, importing the
compute path raises, so a GPU run can never silently degrade to eager PyTorch.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- load torch's HIP runtime first so the library binds to it

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsiren_hip.so")
ABI_VERSION = 12
MAX_INNER = 16
MAX_HIDDEN = 4096  # SIREN_MAX_HIDDEN: hidden widths 128, 256, 512, 1024, then multiples of 1024 up to this
ROW_TILE = 128
TILEQ_INTS = 768  # SIREN_TILEQ_INTS: one tile-queue counter set
ACT_SINE, ACT_SNAKE, ACT_TANH = 0, 1, 2  # siren_act
FP32_IDENTITY, FP32_SIN, FP32_TANH, FP32_SNAKE = 0, 1, 2, 3  # siren_fp32_act

_p = ctypes.c_void_p
_f32p = ctypes.POINTER(ctypes.c_float)
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64


class SirenOptState(ctypes.Structure):
    """siren_opt_state: Adam step + ReduceLROnPlateau state (run.py:116-117)."""
    _fields_ = [
        ("lr", ctypes.c_double), ("best", ctypes.c_double), ("step", ctypes.c_double),
        ("num_bad", _i32), ("last_epoch", _i32),
        ("min_lr", ctypes.c_double), ("factor", ctypes.c_double),
        ("threshold", ctypes.c_double), ("eps_lr", ctypes.c_double),
        ("patience", _i32), ("pad0", _i32),
        ("beta1", ctypes.c_double), ("beta2", ctypes.c_double), ("eps", ctypes.c_double),
    ]


class SirenGuard(ctypes.Structure):
    """siren_guard: fp16 backward range guard (include/siren_hip.h)."""
    _fields_ = [("flag", _i32), ("headroom", _i32), ("clean", _i32), ("overflows", _i32),
                ("headroom0", _i32), ("stalls", _i32)]


HEADROOM0 = 6


class SirenNet(ctypes.Structure):
    _fields_ = [
        ("in_dim", _i32), ("hidden", _i32), ("n_inner", _i32), ("pad0", _i32),
        ("omega0", ctypes.c_float), ("omega", ctypes.c_float),
        ("W0", _p), ("b0", _p),
        ("b", _p * MAX_INNER), ("Wh", _p * MAX_INNER), ("WTh", _p * MAX_INNER),
        ("w_head", _p), ("b_head", _p),
        ("act", _i32 * MAX_INNER), ("a", _p * MAX_INNER),
        ("first_snake", _i32), ("pad1", _i32), ("a0", _p), ("head_omega", ctypes.c_float), ("pad2", ctypes.c_float),
    ]


class SirenGrads(ctypes.Structure):
    _fields_ = [
        ("W0", _p), ("b0", _p),
        ("W", _p * MAX_INNER), ("b", _p * MAX_INNER),
        ("w_head", _p), ("b_head", _p), ("sse", _p),
        ("flat", _p), ("flat_len", _i64),
        ("a", _p * MAX_INNER), ("a0", _p),
    ]


class SirenBatch(ctypes.Structure):
    _fields_ = [
        ("rows", _i32), ("n_valid", _i32), ("n_total", ctypes.c_double),
        ("splits", _i32), ("zero_grads", _i32),
        ("coords", _p), ("target", _p),
        ("Y", _p * (MAX_INNER + 1)), ("C", _p * (MAX_INNER + 1)), ("dZ", _p * 2),
        ("out", _p), ("g", _p), ("head_part", _p), ("sse_part", _p), ("gsum_part", _p),
        ("gmax_part", _p), ("gscale", _p), ("col_part", _p), ("col_part2", _p), ("red_tmp", _p), ("slab", _p),
        ("E", _p * (MAX_INNER + 1)),
        ("grad_ready", _p * (MAX_INNER + 2)),
        ("loss_mode", _i32), ("head_scale_prev", _i32), ("guard", _p), ("tileq", _p),
    ]


KAN_MAX_LAYERS = 8


class SirenKanNet(ctypes.Structure):
    _fields_ = [
        ("n_layers", _i32), ("pad0", _i32), ("width", _i32 * (KAN_MAX_LAYERS + 1)),
        ("grid", _p * KAN_MAX_LAYERS), ("base_w", _p * KAN_MAX_LAYERS),
        ("spline_w", _p * KAN_MAX_LAYERS), ("scaler", _p * KAN_MAX_LAYERS),
    ]


class SirenKanGrads(ctypes.Structure):
    _fields_ = [
        ("base_w", _p * KAN_MAX_LAYERS), ("spline_w", _p * KAN_MAX_LAYERS), ("scaler", _p * KAN_MAX_LAYERS),
        ("sse", _p), ("flat", _p), ("flat_len", _i64),
    ]


class SirenKanBatch(ctypes.Structure):
    _fields_ = [
        ("rows", _i32), ("n_valid", _i32), ("n_total", ctypes.c_double), ("splits", _i32),
        ("zero_grads", _i32), ("coords", _p), ("target", _p), ("out", _p), ("g", _p), ("ws", _p),
    ]


# name -> (restype, argtypes).  Mirrors include/siren_hip.h one-to-one; the CPU test
# suite checks that every symbol the header declares is exported.
_SIGS = {
    "siren_abi_version": (ctypes.c_int, []),
    "siren_build_id": (ctypes.c_char_p, []),
    "siren_struct_size": (_i64, [_i32]),
    "siren_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "siren_default_splits": (_i32, [_i32, _i32]),
    "siren_slab_floats": (_i64, [_i32, _i32]),
    "siren_forward": (ctypes.c_int, [ctypes.POINTER(SirenNet), ctypes.POINTER(SirenBatch), _p]),
    "siren_train_step": (ctypes.c_int, [ctypes.POINTER(SirenNet), ctypes.POINTER(SirenGrads),
                                        ctypes.POINTER(SirenBatch), _p]),
    "siren_backward": (ctypes.c_int, [ctypes.POINTER(SirenNet), ctypes.POINTER(SirenGrads),
                                      ctypes.POINTER(SirenBatch), _p]),
    "siren_apply_update": (ctypes.c_int, [ctypes.POINTER(SirenNet), _p, _p, _p, _p, _i64,
                                          ctypes.POINTER(_p), ctypes.POINTER(_p), ctypes.POINTER(_p),
                                          _p, _p, ctypes.c_double, _p, _p, _i64, _p, _p]),
    "siren_coords_fill": (ctypes.c_int, [_p, _i64, _i64, _i64, _p]),
    "siren_coords_fill_grid": (ctypes.c_int, [_p, _i64, _i64, _i64, _i32, _p]),
    "siren_first_fwd": (ctypes.c_int, [_p, _i32, _p, _p, ctypes.c_float, _i32, _i32, _p, _p, _p]),
    "siren_inner_fwd": (ctypes.c_int, [_p, _p, _p, ctypes.c_float, _i32, _i32, _p, _p, _p, _p, _p, _p]),
    "siren_head_loss": (ctypes.c_int, [_p, _i32, _i32, _p, _p, _i32, ctypes.c_double, _p, _p, _p, _p,
                                       _p, _p]),
    "siren_grad_scale": (ctypes.c_int, [_p, _i32, _p, _i32, ctypes.c_float, _p, _p]),
    "siren_inner_fwd_act": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_float, _p, _i32, _i32, _p, _p, _p, _p,
                                           _p, _p, _p]),
    "siren_head_bwd": (ctypes.c_int, [_p, _p, _p, _p, ctypes.c_float, _i32, _i32, _p, _p, _p, _p, _p, _p,
                                      _p]),
    "siren_inner_bwd_dx_act": (ctypes.c_int, [_p, _p, _p, _p, _i32, ctypes.c_float, _i32, _i32, _p, _p, _p,
                                              _p]),
    "siren_inner_bwd_dx": (ctypes.c_int, [_p, _p, _p, ctypes.c_float, _i32, _i32, _p, _p, _p, _p]),
    "siren_first_bwd_dx": (ctypes.c_int, [_p, _p, _p, _p, _i32, ctypes.c_float, _i32, _i32, _p, _p,
                                          _p]),
    "siren_inner_bwd_dw": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _i32, _p, _p]),
    "siren_dw_reduce": (ctypes.c_int, [_p, _i32, _i32, _i32, _p, _i32, _p, _p]),
    "siren_nt_tile": (_i32, [_i32, _i32]),
    "siren_dw_tile": (_i32, [_i32, _i32]),
    "siren_col_reduce": (ctypes.c_int, [_p, _i64, _i32, _i32, _p, _i32, _i32, _p, _p]),
    "siren_adam_step": (ctypes.c_int, [_p, _p, _p, _p, _i64, _p, _p]),
    "siren_plateau_step": (ctypes.c_int, [_p, _p, ctypes.c_double, _p, _p, _i64, _p]),
    "siren_cast_weight": (ctypes.c_int, [_p, _i32, _i32, _p, _p, _p]),
    "siren_head_fused_fwd": (ctypes.c_int, [_p, _p, _p, ctypes.c_float, _i32, _i32, _p, _p, ctypes.c_float, _p, _i32,
                                            ctypes.c_double, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "siren_head_fused_fwd_act": (ctypes.c_int, [_p, _p, _p, _i32, ctypes.c_float, _p, _i32, _i32, _p, _p,
                                                ctypes.c_float, _p, _i32, ctypes.c_double, _i32, _p, _p, _p, _p, _p,
                                                _p, _p, _p, _p, _p, _p]),
    "siren_grad_scale_bound": (ctypes.c_int, [_p, _i32, _p, _p, _p, _i32, ctypes.c_double, ctypes.c_float, _i32,
                                              ctypes.c_float, _p, _p]),
    "siren_set_option": (ctypes.c_int, [_i32, _i32]),
    "siren_fp32_linear": (ctypes.c_int, [_p, _i64, _i32, _i32, _p, _p, ctypes.c_float, _p, _p]),
    "siren_fp32_act": (ctypes.c_int, [_i32, _p, _i64, _i32, _p, _p, _p]),
    "siren_fp32_act_bwd": (ctypes.c_int, [_i32, _p, _i64, _i32, _p, _p, _p, _p, _p, _p, _p]),
    "siren_fp32_linear_bwd": (ctypes.c_int, [_p, _i64, _i32, _i32, _p, ctypes.c_float, _p, _p, _p, _p, _p, _i32, _p,
                                              _p]),
    "siren_kan_workspace_floats": (_i64, [ctypes.POINTER(SirenKanNet), _i32, _i32]),
    "siren_kan_forward": (ctypes.c_int, [ctypes.POINTER(SirenKanNet), ctypes.POINTER(SirenKanBatch), _p]),
    "siren_kan_train_step": (ctypes.c_int, [ctypes.POINTER(SirenKanNet), ctypes.POINTER(SirenKanGrads),
                                            ctypes.POINTER(SirenKanBatch), _p]),
    "siren_kan_backward": (ctypes.c_int, [ctypes.POINTER(SirenKanNet), ctypes.POINTER(SirenKanGrads),
                                          ctypes.POINTER(SirenKanBatch), _p, _p]),
    "siren_profile_enable": (ctypes.c_int, [_i32]),
    "siren_profile_reset": (ctypes.c_int, []),
    "siren_profile_mask": (ctypes.c_int, [ctypes.c_uint32]),
    "siren_profile_read": (ctypes.c_int, [_i32, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(_i64)]),
}

STRUCTS = [SirenNet, SirenGrads, SirenBatch, SirenOptState, SirenKanNet, SirenKanGrads, SirenKanBatch, SirenGuard]

PROF_KINDS = ["first_fwd", "inner_fwd", "head", "bwd_dw", "bwd_dx", "bwd_dx0", "reduce", "update",
              "kan_fwd", "kan_dw", "kan_dx", "kan_misc", "head_fwd"]


def profile_read() -> dict:
    """{kind: (total_ms, launches)} for every profiled launch kind since the last reset."""
    lib = load()
    out = {}
    for k, name in enumerate(PROF_KINDS):
        ms, n = ctypes.c_double(0), _i64(0)
        check(lib.siren_profile_read(k, ctypes.byref(ms), ctypes.byref(n)), "siren_profile_read")
        out[name] = (ms.value, n.value)
    return out

_lib = None


class SirenError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load (once) and return the native library; raises if it is absent or mismatched: wrong ABI,
    or (when the sources are beside it) a build id that is not the hash of those sources."""
    global _lib
    if _lib is not None:
        return _lib
    # another library file (tools/lib_ab.py: a build of another commit) is checked for its ABI only
    own = os.path.abspath(path) == os.path.abspath(LIB_PATH)
    _lib = bind(path, expect_build_id=expected_build_id() if own else None)
    return _lib


def expected_build_id(defines=()) -> str | None:
    """buildinfo.source_hash of the sources in this tree (None when they are not shipped)."""
    from . import buildinfo
    return buildinfo.source_hash(defines) if buildinfo.sources_present() else None


def bind(path: str, expect_build_id: str | None = None, check_abi: bool = True):
    """A freshly bound (uncached) handle of the library at `path`: tools/ab_bench.py loads the
    product library beside measurement builds of it under other file names.  expect_build_id: refuse
    a library compiled from other sources (siren_build_id, include/siren_hip.h).  check_abi=False
    (measurement tools only): bind a library of an earlier ABI built from an older commit, for the
    entry points whose signatures did not change; symbols it lacks are left unbound."""
    if not os.path.exists(path):
        raise SirenError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the SIREN path has no eager fallback)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        if not check_abi and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if not check_abi:
        return lib
    if lib.siren_abi_version() != ABI_VERSION:
        raise SirenError(f"libsiren_hip ABI {lib.siren_abi_version()} != expected {ABI_VERSION}")
    if expect_build_id is not None and lib.siren_build_id().decode() != expect_build_id:
        raise SirenError(f"{path} was built from other sources (build id {lib.siren_build_id().decode()[:12]}, "
                         f"sources {expect_build_id[:12]}): rebuild with __graft_entry__.build()")
    for k, st in enumerate(STRUCTS):
        if lib.siren_struct_size(k) != ctypes.sizeof(st):
            raise SirenError(f"{st.__name__}: ctypes size {ctypes.sizeof(st)} != C size {lib.siren_struct_size(k)}")
    return lib


def check(status: int, what: str = "siren") -> None:
    """Map a non-zero C-ABI status to SirenError (siren_status_string text)."""
    if status != 0:
        msg = load().siren_status_string(status)
        raise SirenError(f"{what} failed with status {status}: {msg.decode() if msg else '?'}")


def ptr(t) -> int:
    """Device/host address of a torch tensor (0 for None)."""
    return 0 if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def new_tileq(device) -> torch.Tensor:
    """A tile-queue counter set (SIREN_TILEQ_INTS int32 on `device`; the library zeroes it before
    each launch that uses it).  One per stream of concurrent launches."""
    return torch.zeros(TILEQ_INTS, dtype=torch.int32, device=device)
