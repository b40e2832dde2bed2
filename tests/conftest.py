import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# The parity group: one whole-step check against the oracle per BASELINE config and per fused
# kernel of the default training step. These run first, so that a `-x` stop anywhere later in the
# GPU suite still leaves every config's parity verdict on record, and the first failure names its
# row. Order inside the group: the fused step itself, then one step per config.
PARITY_FIRST = (
    "test_gpu_headfuse.py::test_fused_vs_oracle",               # a5/a6/a8/a9: fused last layer
    "test_gpu_headfuse.py::test_kernel_vs_unfused_launches",    # NT_FWD_HB bit identity
    "test_gpu_queue.py::test_queue_bit_identical_to_static_walk",
    "test_gpu_kernels.py::test_inner_fwd",                      # a5 vs fp64
    "test_gpu_kernels.py::test_inner_bwd_dx",
    "test_gpu_kernels.py::test_inner_bwd_dw",
    "test_gpu_engine.py::test_train_step_grads_vs_oracle",      # cfg1 shapes, whole step
    "test_gpu_fullsize.py::test_cfg2_parity_vs_torch_fp32",     # cfg2
    "test_gpu_cfg3.py::test_cfg3_step_vs_oracle_slice",         # cfg3
    "test_gpu_mdct.py::test_mdct_step_grads_vs_oracle",         # cfg4
    "test_gpu_kan.py::test_kan_step_vs_oracle",                 # cfg5
    "test_gpu_act.py::test_train_step_act_vs_oracle",           # f3 Snake / Tanh
)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libsiren_hip.so")


def _parity_rank(item) -> int:
    node = item.nodeid.split("/")[-1].split("[")[0]
    for i, key in enumerate(PARITY_FIRST):
        if node == key:
            return i
    return len(PARITY_FIRST)


@pytest.hookimpl(trylast=True)
def pytest_collection_modifyitems(session, config, items):
    # stable: everything outside the group keeps its file order
    items[:] = sorted(items, key=_parity_rank)


@pytest.fixture(scope="session")
def lib():
    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def dev(lib):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda:0")
