"""Host-side logic of the package (no GPU): reference-compatible construction and init,
parameter layout, configuration validation, data prep and metrics, train() API."""
import inspect
import json
import os

import numpy as np
import pytest
import torch

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _model(H=256, L=2, w0=1000.0, in_dim=1, seed=0):
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    torch.manual_seed(seed)
    return SirenWithSnakeTanh(in_features=in_dim, out_features=1, hidden_features=H, num_sine=L,
                              num_snake=0, num_tanh=0, first_omega_0=w0, hidden_omega_0=30)


def test_init_bit_exact_with_reference_3x256():
    ref = np.load(os.path.join(G, "init_3x256_seed0.npz"))
    sd = _model().state_dict()
    assert list(sd.keys()) == list(ref.files)
    for k in ref.files:
        assert np.array_equal(sd[k].numpy(), ref[k]), k


@pytest.mark.parametrize("fname,H,L,in_dim,seed", [("init_5x1024_seed0_summary.json", 1024, 4, 1, 0),
                                                   ("init_5x512_in2_seed3_summary.json", 512, 4, 2, 3)])
def test_init_matches_reference_large(fname, H, L, in_dim, seed):
    ref = json.load(open(os.path.join(G, fname)))
    sd = _model(H, L, 3000.0, in_dim, seed).state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k, r in ref.items():
        v = sd[k].numpy().astype(np.float64)
        assert list(v.shape) == r["shape"]
        assert v.reshape(-1)[:8].astype(np.float32).tolist() == r["head"]
        assert v.sum() == pytest.approx(r["sum"], rel=1e-12, abs=1e-12)
        assert (v ** 2).sum() == pytest.approx(r["sumsq"], rel=1e-12)


def test_param_layout():
    from inr_for_audio_amd.engine import SEG_ALIGN, ParamLayout
    m = _model(1024, 4)
    lay = ParamLayout(m)
    assert lay.names == list(m.state_dict().keys())
    assert all(o % SEG_ALIGN == 0 for o in lay.offsets)
    assert sum(lay.numels) == 4201473          # 5x1024 parameter count
    assert lay.sse_offset == lay.n_params and lay.flat_len == lay.n_params + SEG_ALIGN
    flat = torch.arange(lay.flat_len, dtype=torch.float32)
    for i, shp in enumerate(lay.shapes):
        v = lay.view(flat, i)
        assert tuple(v.shape) == shp and int(v.reshape(-1)[0]) == lay.offsets[i]


@pytest.mark.parametrize("H,cfg,fl,ll,Hp", [
    (100, (2, 0, 0), False, True, 128), (384, (1, 1, 1), False, True, 512), (200, (0, 2, 0), True, False, 256),
    (1000, (1, 0, 0), False, True, 1024), (3, (1, 1, 0), False, True, 128),
    (1500, (2, 0, 0), False, True, 2048), (2048, (1, 0, 1), False, True, 2048), (3000, (1, 1, 1), True, False, 3072)])
def test_hidden_width_padding(H, cfg, fl, ll, Hp):
    """Any hidden_features <= 4096 runs zero-padded to the next kernel width (128, 256, 512, 1024,
    then multiples of 1024; models.py:310 accepts
    any width): the layout stores the padded tensors, the model's parameters are their [:H] blocks,
    a Snake a's pad entries are 1 and every other pad entry is 0."""
    from inr_for_audio_amd.engine import ParamLayout
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    torch.manual_seed(0)
    m = SirenWithSnakeTanh(1, 1, H, *cfg, first_linear=fl, last_linear=ll, first_omega_0=300.0, a_initial=0.5)
    assert m.hip_width() == Hp and m.hip_spec().hidden == Hp
    pad = m.hip_padding()
    lay = ParamLayout(m, pad)
    flat = torch.full((lay.flat_len,), 7.0)
    lay.fill_pads(flat)
    sd = m.state_dict()
    for i, (name, p) in enumerate(m.named_parameters()):
        tv = lay.true_view(flat, i)
        assert tuple(tv.shape) == tuple(p.shape), name
        tv.copy_(p.detach())
        v = lay.view(flat, i)
        assert all(d in (Hp, 1, m.in_features) for d in v.shape), (name, v.shape)
        assert torch.equal(lay.true_view(flat, i), sd[name])
        if i in pad:
            mask = torch.ones_like(v, dtype=torch.bool)
            mask[tuple(slice(0, d) for d in p.shape)] = False
            want = 1.0 if name.endswith(".a") else 0.0
            assert bool((v[mask] == want).all()), name
    assert (m.hip_padding() == {}) == (H == Hp)


def test_hip_spec_validation():
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    spec = _model(256, 2, 22000.0).hip_spec()
    assert (spec.in_dim, spec.hidden, spec.n_inner, spec.omega0, spec.omega) == (1, 256, 2, 22000.0, 30.0)
    bad = [dict(hidden_features=4097), dict(num_sine=0), dict(in_features=3), dict(out_features=2),
           dict(num_sine=10, num_snake=4, num_tanh=3)]
    for kw in bad:
        args = dict(in_features=1, out_features=1, hidden_features=256, num_sine=2, num_snake=0, num_tanh=0)
        args.update(kw)
        with pytest.raises(NotImplementedError):
            SirenWithSnakeTanh(**args).hip_spec()


def test_reference_default_snake_config_constructs():
    """train()'s defaults (num_sine=2, num_snake=2, a_initial=0.5) build the reference's
    module tree and parameter names, and the fused path's spec / parameter index."""
    from inr_for_audio_amd import _lib
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    m = SirenWithSnakeTanh(1, 1, 256, 2, 2, 0, a_initial=0.5)
    names = list(m.state_dict().keys())
    assert names[-2:] == ["net.7.weight", "net.7.bias"] and "net.4.a" in names
    spec = m.hip_spec()
    assert spec.n_inner == 4 and spec.acts == (_lib.ACT_SINE,) * 2 + (_lib.ACT_SNAKE,) * 2
    ix = m.param_index()
    assert [names[k] for k in ix["W"]] == ["net.1.linear.weight", "net.2.linear.weight", "net.3.weight",
                                          "net.5.weight"]
    assert [None if k is None else names[k] for k in ix["a"]] == [None, None, "net.4.a", "net.6.a"]
    assert (names[ix["wh"]], names[ix["bh"]]) == ("net.7.weight", "net.7.bias")
    t = SirenWithSnakeTanh(2, 1, 128, 1, 1, 2, a_initial=None)
    assert t.hip_spec().acts == (_lib.ACT_SINE, _lib.ACT_SNAKE, _lib.ACT_TANH, _lib.ACT_TANH)
    assert [t.state_dict()[k].shape for k in ("net.3.a",)] == [(128,)]


def test_shard_range_partitions():
    from inr_for_audio_amd.engine import shard_range
    for n in (1, 7, 1000, 28_800_000):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_train_signature_matches_reference():
    """run.py:30 -- same positional/keyword parameters and defaults, extras keyword-only."""
    from inr_for_audio_amd.run import train
    ref = [("experiment_path", None), ("tag", None), ("inst", None), ("duration", None),
           ("num_channels", 1), ("method", "wave"), ("arch", "mlp"), ("loss_mode", "mse"), ("mode", None),
           ("decimation", 1), ("bwe", False), ("num_hidden_features", 256), ("num_sine", 2),
           ("num_snake", 2), ("num_tanh", 0), ("num_freq", None), ("omega", 22000),
           ("first_linear", False), ("last_linear", True), ("hidden_omega", 30), ("a_initial", 0.5),
           ("total_steps", 20000), ("learning_rate", 1e-3), ("min_learning_rate", 1e-6), ("alpha", 0.0),
           ("prev_ckpt_path", None), ("visualization", False)]
    params = inspect.signature(train).parameters
    pos = [p for p in params.values() if p.kind == p.POSITIONAL_OR_KEYWORD]
    assert [p.name for p in pos] == [r[0] for r in ref]
    for p, (name, default) in zip(pos, ref):
        if default is not None:
            assert p.default == default, name
    assert all(p.kind == p.KEYWORD_ONLY for p in params.values() if p not in pos)


def test_waveform_fitting_and_reported_snr(tmp_path):
    from scipy.io import wavfile
    from inr_for_audio_amd import utils
    g = np.load(os.path.join(G, "gt_bach_1s.npz"))
    fs = int(g["fs"])
    wav = str(tmp_path / "x.wav")
    wavfile.write(wav, fs, g["raw"])
    ds = utils.WaveformFitting(wav, duration=1)
    coords, amp = ds[0]
    assert np.array_equal(amp.numpy().reshape(-1), g["target"])
    assert np.array_equal(coords.numpy().reshape(-1), g["coords"])
    ref, fs2 = utils.load_mono_like_librosa(wav)
    snr = json.load(open(os.path.join(G, "snr_cases.json")))
    assert abs(utils.reported_snr(ref, fs2, g["target"], 1) - snr["perfect_fit_reported_1s"]) < 1e-5
    d2 = utils.WaveformFitting(wav, duration=2, decimation=2)
    ref2 = np.load(os.path.join(G, "gt_bach_2s_dec2.npz"))
    assert np.allclose(d2.amplitude().numpy().reshape(-1), ref2["target"], atol=1e-7)
    assert d2.sample_rate == int(ref2["sample_rate"])


@pytest.mark.parametrize("kind", ["f32", "i16"])
def test_multiwave_fitting_bit_exact(tmp_path, kind):
    """MultiWaveformFitting (utils.py:186-231, BASELINE cfg3's (t, ch) grid) against the
    reference's own output (tests/golden/multiwave.npz): channel trim, FIR decimation,
    height-major (time, channel) coordinates, no normalisation."""
    from scipy.io import wavfile
    from inr_for_audio_amd.utils import MultiWaveformFitting, get_coord
    g = np.load(os.path.join(G, "multiwave.npz"))
    wav = str(tmp_path / "c.wav")
    wavfile.write(wav, int(g["fs"]), g[f"clip_{kind}"])
    for nc in (2, 1):
        for lp in (False, True):
            tag = f"{kind}_c{nc}_{'lp' if lp else 'raw'}"
            ds = MultiWaveformFitting(wav, duration=1, num_channels=nc, lp=lp)
            coords, samples = ds[0]
            assert [ds.height, ds.width, ds.sample_rate] == g[f"{tag}_meta"].tolist()
            assert coords.dtype == torch.float32 and np.array_equal(coords.numpy(), g[f"{tag}_coords"]), tag
            assert samples.dtype == g[f"{tag}_samples"].dtype
            assert np.array_equal(samples, g[f"{tag}_samples"]), tag
            # time column = get_coord(height) repeated per channel; channel column alternates
            t = get_coord(ds.height, 1).numpy().reshape(-1)
            assert np.array_equal(coords.numpy()[:, 0], np.repeat(t, ds.width))
            assert np.array_equal(ds.to_channels(samples.reshape(-1))[:, -1], samples.reshape(-1)[nc - 1::nc])
    with pytest.raises(IndexError):  # the reference indexes [:T, :nc]: a mono file is rejected
        mono = str(tmp_path / "m.wav")
        wavfile.write(mono, int(g["fs"]), g["clip_f32"][:, 0].copy())
        MultiWaveformFitting(mono, duration=1, num_channels=1)


def test_unsupported_train_options_raise(tmp_path):
    from inr_for_audio_amd.run import train
    for kw in (dict(method="mdct", bwe=True), dict(arch="kan", method="mdct"), dict(arch="rbf"),
               dict(loss_mode="snr"), dict(alpha=0.5), dict(multichannel=True, bwe=True)):
        with pytest.raises(NotImplementedError):
            train(str(tmp_path), "t", "x", 1, **kw)
    with pytest.raises(ValueError):
        train(str(tmp_path), "t", "x", 1, method="stft")


def test_package_never_imports_oracle():
    root = os.path.join(os.path.dirname(G), "..", "inr-for-audio_amd")
    for dirpath, _, files in os.walk(root):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in src.replace("# oracle", ""), f


def test_bench_kernel_kinds_cover_every_template_form():
    """bench.py maps rocprof kernel names to launch kinds for the roofline's PMC fields: every
    gemm_nt_kernel<Cfg, MODE, HEAD[, QUEUE]> form the library instantiates must resolve to exactly
    one kind (a dX launch with QUEUE = false once fell through and left `traffic` null)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    cfg = "void siren::gemm_nt_kernel<siren::NtCfg<256, 256, 2, 4, 64, 2, true>, {}>(siren::NtParams)"
    want = {"0, false": "inner_fwd", "0, false, true": "inner_fwd", "0, false, false": "inner_fwd",
            "1, false": "bwd_dx", "1, false, false": "bwd_dx", "1, false, true": "bwd_dx",
            "2, false, false": "bwd_dx0", "7, true, false": "head_fwd", "7, true": "head_fwd",
            "3, false, false": None, "3, false, true, true": None, "0, false, true, false": "inner_fwd"}
    for args, kind in want.items():
        hits = [k for k in bench.KIND_MATCH if bench.kind_match(k, cfg.format(args))]
        assert hits == ([kind] if kind else []), (args, hits)
    tn = "void siren::gemm_tn_kernel<siren::TnCfg<256, 256, 2, 4, 64, 2, 2> >(siren::TnParams)"
    assert [k for k in bench.KIND_MATCH if bench.kind_match(k, tn)] == ["bwd_dw"]


def test_bench_bytes_per_row_live_stack():
    """bench.py's HBM byte model for the width-256 Snake stacks (--config live / default): per row, fp16
    activations (2 B), the last hidden layer fused with the head."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    e = 2 * 256
    live = bench.siren_bytes_per_row(["snake"] * 4, 256)
    assert live == {"first_fwd": 4 + 2 * e, "inner_fwd": 3 * 4 * e, "head_fwd": 2 * e, "bwd_dx": 3 * 4 * e,
                    "bwd_dx0": 2 * e, "bwd_dw": 4 * 2 * e}
    dflt = bench.siren_bytes_per_row(["sine", "sine", "snake", "snake"], 256)
    # forwards: sine 3e, sine 3e, snake 4e; dX into snake (i=3), sine (2), sine (1): 4e + 3e + 3e
    assert dflt["inner_fwd"] == 10 * e and dflt["bwd_dx"] == 10 * e and dflt["bwd_dw"] == 8 * e
    assert bench.STACKS["live"] == (0, 4) and bench.CONFIGS["live"][0] == 256 and bench.CONFIGS["live"][3] == 441_000
