"""BASELINE cfg3 on the HIP path: 5 min of 48 kHz stereo as MultiWaveformFitting's (time,
channel) grid (utils.py:186-231) -> SIREN 6x1024 with in = 2, sharded over 8 GPUs.

* the device grid generator (siren_coords_fill_grid) is bit-exact with the reference's
  meshgrid of torch.linspace at cfg3's full height, at a shard offset;
* one fused step on a 4096-row slice of that grid against the fp16-storage oracle;
* one GPU's full 3.6 M-row shard through size-independent properties: determinism,
  train/inference loss consistency and micro-batch linearity of the full-batch gradient.
(The 2-rank data-parallel step on this architecture is in test_gpu_dist.py.)"""
import numpy as np
import pytest
import torch

from errlog import STEP_TOL, check_grads
from oracle import siren_oracle as orc

pytestmark = pytest.mark.gpu

HEIGHT = 300 * 48000          # 14.4 M instants x 2 channels = 28.8 M coordinates
SHARD = HEIGHT * 2 // 8       # one GPU's contiguous share at DP = 8


def _grid(rows, offset, dev, height=HEIGHT, width=2):
    from inr_for_audio_amd import _lib
    lib = _lib.load()
    xy = torch.empty(rows, 2, dtype=torch.float32, device=dev)
    _lib.check(lib.siren_coords_fill_grid(xy.data_ptr(), rows, offset, height, width,
                                          torch.cuda.current_stream(dev).cuda_stream), "coords_fill_grid")
    return xy


def _stereo_target(xy):
    """a synthetic stereo signal on the grid: different tone mixes per channel"""
    t, ch = xy[:, 0], xy[:, 1]
    left = 0.5 * torch.sin(2300.0 * t) + 0.2 * torch.sin(9100.0 * t + 0.3)
    right = 0.4 * torch.sin(3100.0 * t + 1.0) + 0.2 * torch.sin(7700.0 * t)
    return torch.where(ch < 0, left, right)


def _model(seed=0):
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    torch.manual_seed(seed)
    return SirenWithSnakeTanh(2, 1, 1024, 5, 0, 0, first_omega_0=3000.0, hidden_omega_0=30.0)


def test_grid_fill_bit_exact(dev):
    from inr_for_audio_amd.utils import MultiWaveformFitting
    # a whole small grid against the reference-identical host dataset
    data = np.zeros((4801, 2), np.float32)
    ds = MultiWaveformFitting(duration=1, num_channels=2, data=data, sample_rate=4801)
    xy = _grid(ds.height * 2 + 256, 0, dev, ds.height, 2).cpu()
    assert torch.equal(xy[:ds.height * 2], ds.coords)
    assert not xy[ds.height * 2:].any()                                  # pad rows are (0, 0)
    one = _grid(100, 0, dev, 100, 1).cpu()
    assert torch.equal(one, torch.from_numpy(orc.multiwave_grid(100, 1)))
    # cfg3's full height, rank 5's shard start (offset not a multiple of anything convenient)
    off = 5 * SHARD + 12345 * 2 + 1
    got = _grid(1 << 16, off, dev).cpu().numpy()
    k = off + np.arange(1 << 16)
    t = orc.linspace_f32(HEIGHT)[k // 2]
    assert np.array_equal(got[:, 0], t) and np.array_equal(got[:, 1], np.where(k % 2 == 0, -1.0, 1.0))


def test_cfg3_step_vs_oracle_slice(dev):
    """SIREN 6x1024, in = 2: one fused step on 4096 rows of the cfg3 grid (rank 3's shard),
    gradients vs the fp64 oracle with the HIP path's fp16 storage emulated."""
    from inr_for_audio_amd.engine import SirenEngine
    n = 4096
    xy = _grid(n, 3 * SHARD + 777_000, dev)
    y = _stereo_target(xy)
    m = _model()
    sd0 = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
    eng = SirenEngine(m, xy, y, device=dev)
    eng.step()
    torch.cuda.synchronize()
    got = {k: v.detach().cpu().numpy() for k, v in zip(eng.layout.names, eng.grad_views())}
    p = orc.Params.from_state_dict(sd0, 5)
    t, yy = xy.cpu().numpy(), y.cpu().numpy()
    out, cache = orc.forward(p, t, 3000.0, 30.0, half=True, dtype=np.float64)
    ref = orc.backward(p, t, cache, orc.mse_grad(out, yy), 3000.0, 30.0, half=True)
    check_grads("cfg3_slice_6x1024_in2", got, ref, STEP_TOL)
    assert abs(eng.last_loss() - orc.mse(out, yy)) <= 1e-4 * orc.mse(out, yy)


def _shard_engine(dev, micro_batch):
    from inr_for_audio_amd.engine import SirenEngine
    xy = _grid(SHARD, 0, dev)
    return SirenEngine(_model(), xy, _stereo_target(xy), n_total=2 * HEIGHT, micro_batch=micro_batch,
                       hist_cap=4, device=dev), xy


def test_cfg3_full_shard_properties(dev):
    """One GPU's 3.6 M-row cfg3 shard (global N = 28.8 M in the MSE mean)."""
    eng, xy = _shard_engine(dev, SHARD)
    assert eng.n_micro == 1 and eng.rows % 256 == 0
    p0, st0 = eng.params.clone(), eng.state.clone()
    # consistency: the fused step's loss == MSE of the inference output on the same weights
    out = eng.infer(xy).double()
    y = _stereo_target(xy).double()
    sse = float(((out - y) ** 2).sum())
    eng.step()
    torch.cuda.synchronize()
    g1 = eng.grads.clone()
    assert abs(float(g1[eng.layout.sse_offset]) - sse) <= 1e-5 * sse
    assert torch.isfinite(g1).all()
    # determinism: rewind the weights and optimizer, step again -> bit-identical gradients
    eng.params.copy_(p0)
    eng.exp_avg.zero_()
    eng.exp_avg_sq.zero_()
    eng.state.copy_(st0)
    eng._refresh_shadows()
    eng.step()
    torch.cuda.synchronize()
    assert torch.equal(eng.grads, g1)
    p_after = eng.params.clone()
    del eng
    torch.cuda.empty_cache()
    # linearity: the same full-batch gradient from 2^20-row micro-batches (fp16 dZ storage per
    # micro-batch scale), and the same first update
    eng4, _ = _shard_engine(dev, 1 << 20)
    assert eng4.n_micro == 4
    eng4.step()
    torch.cuda.synchronize()
    g4 = eng4.grads
    # per parameter: the first layer's gradient (x omega0) dominates the whole-vector norm
    lay = eng4.layout
    got = {k: lay.view(g4, i).double().cpu().numpy() for i, k in enumerate(lay.names)}
    ref = {k: lay.view(g1, i).double().cpu().numpy() for i, k in enumerate(lay.names)}
    check_grads("cfg3_shard_microbatch_linearity", got, ref, STEP_TOL)
    assert abs(float(g4[eng4.layout.sse_offset]) - sse) <= 1e-5 * sse
    d = (eng4.params - p_after).abs()
    assert float(d.max()) <= 2 * 1e-3 + 1e-6 and float((d > 1e-6).float().mean()) < 0.01
