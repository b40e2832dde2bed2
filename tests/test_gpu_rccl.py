"""RCCL on the box: the engine's data-parallel path over the `nccl` backend (RCCL), one rank.

RCCL refuses two ranks on one GPU, so the multi-rank tests use gloo (test_gpu_dist.py).  This
one runs the code the 8-GPU node runs -- init_process_group("nccl"), the parameter broadcast, the
per-layer gradient buckets all-reduced on the communication stream behind the backward's
grad_ready events -- through RCCL itself, with a world of one (the engine's world > 1 gate is
lifted for the test only).  An all-reduce over one rank is the identity, so the step must be
bit-identical to the single-process step, and bench.py under torchrun with --backend nccl must
print its line."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model_data():
    sys.path.insert(0, ROOT)
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    torch.manual_seed(0)
    m = SirenWithSnakeTanh(1, 1, 256, 2, 2, 0, first_omega_0=2000.0, hidden_omega_0=30.0, a_initial=0.5)
    n = 5001
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    y = 0.5 * torch.sin(37 * t) + 0.2 * torch.sin(91 * t)
    return m, t, y


def _steps(eng):
    eng.step()
    g1 = eng.grads.cpu().numpy().copy()
    eng.step()
    torch.cuda.synchronize()
    return g1, eng.params.cpu().numpy().copy(), eng.history()[0]


def _rank(port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    from inr_for_audio_amd import engine
    engine._dist = lambda: dist  # lift the world > 1 gate: the bucketed RCCL path at world 1
    m, t, y = _model_data()
    eng = engine.SirenEngine(m, t, y, micro_batch=1024, device=torch.device("cuda:0"))
    assert eng._buckets is not None and eng.n_micro == 5
    q.put(_steps(eng))
    dist.destroy_process_group()


def test_engine_over_rccl_matches_single(lib):
    from inr_for_audio_amd.engine import SirenEngine
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank, args=(_free_port(), q))
    p.start()
    g1, params, hist = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    m, t, y = _model_data()
    ref = _steps(SirenEngine(m, t, y, micro_batch=1024, device=torch.device("cuda:0")))
    assert np.array_equal(g1, ref[0])
    assert np.array_equal(params, ref[1])
    assert np.array_equal(hist, ref[2])


def test_bench_torchrun_nccl_one_rank():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus",
                        "1", "--backend", "nccl", "--steps", "2", "--warmup", "1", "--coords", "65536", "--hidden",
                        "256", "--layers", "3", "--no-cpu-baseline"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and res["value"] > 0
