"""Data-parallel math on CPU with gloo (world_size 2): contiguous coordinate shards with the
GLOBAL-N MSE scaling, summed by one all-reduce of the flat gradient (whose tail slot
carries the squared-error sum), equal the full-batch gradient."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _problem():
    import sys
    sys.path.insert(0, ROOT)
    from oracle import siren_oracle as orc
    rng = np.random.default_rng(0)
    H, L, n = 128, 2, 999
    lim = np.sqrt(6 / H) / 30
    p = orc.Params(rng.uniform(-1, 1, (H, 1)), rng.uniform(-1, 1, H),
                   [rng.uniform(-lim, lim, (H, H)) for _ in range(L)],
                   [rng.uniform(-0.05, 0.05, H) for _ in range(L)], rng.uniform(-lim, lim, H), 0.01)
    t = orc.linspace_f32(n).reshape(-1, 1)
    y = (0.5 * np.sin(37 * t[:, 0])).astype(np.float32)
    return orc, p, t, y, n


def _flat(orc, p, grads, sse):
    keys = list(p.to_state_dict().keys())
    return np.concatenate([grads[k].reshape(-1) for k in keys] + [np.array([sse])])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    from inr_for_audio_amd.engine import shard_range
    orc, p, t, y, n = _problem()
    lo, hi = shard_range(n, rank, world)
    out, cache = orc.forward(p, t[lo:hi], 1000.0, 30.0, dtype=np.float64)
    g = orc.mse_grad(out, y[lo:hi], n_total=n)          # global-N scaling
    grads = orc.backward(p, t[lo:hi], cache, g, 1000.0, 30.0)
    sse = float(np.sum((out - y[lo:hi]) ** 2))
    flat = torch.from_numpy(_flat(orc, p, grads, sse))
    dist.all_reduce(flat)
    q.put((rank, flat.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gradient_equals_full_batch(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    orc, p, t, y, n = _problem()
    out, cache = orc.forward(p, t, 1000.0, 30.0, dtype=np.float64)
    grads = orc.backward(p, t, cache, orc.mse_grad(out, y), 1000.0, 30.0)
    full = _flat(orc, p, grads, float(np.sum((out - y) ** 2)))
    for r in range(world):
        assert np.allclose(res[r], full, rtol=1e-6, atol=1e-12)
        assert np.array_equal(res[r], res[0])            # every rank holds the same reduced vector
