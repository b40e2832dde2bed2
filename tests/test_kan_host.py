"""KAN variant on the host: the module mirror's init and the CPU oracle against
the reference's own numbers (tests/golden/kan_fwd_bwd.npz from /root/reference's kan.py)."""
import os

import numpy as np
import pytest
import torch

from oracle import siren_oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")


def load(name):
    return np.load(os.path.join(G, name))


def _sd(name):
    f = load("kan_fwd_bwd.npz")
    pre = f"{name}_init_"
    return {k[len(pre):]: f[k] for k in f.files if k.startswith(pre)}


@pytest.mark.parametrize("name,widths,seed", [("k64", [1, 64, 64, 1], 0), ("k128", [1, 128, 128, 1], 3)])
def test_kan_init_bit_exact(name, widths, seed):
    from inr_for_audio_amd.kan import KAN
    torch.manual_seed(seed)
    m = KAN(widths)
    ref = _sd(name)
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k, v in sd.items():
        if k.endswith("spline_weight"):
            # torch.linalg.lstsq (kan.py:126-128) is not bit-reproducible run to run: the
            # reference itself, re-run, differs from its own fixture by a few ulps here
            assert np.max(np.abs(v.numpy() - ref[k])) < 1e-7, k
        else:
            assert np.array_equal(v.numpy(), ref[k]), k


def test_kan_bases_bit_exact_vs_torch_recursion():
    """The oracle's fp32 bases equal the module's torch recursion (kan.py:94-104 op order)."""
    from inr_for_audio_amd.kan import bspline_bases
    sd = _sd("k64")
    x = np.random.default_rng(0).uniform(-1.2, 1.2, (500, 64)).astype(np.float32)
    x[:5, 0] = [-1.0, 1.0, 0.2, -0.6, 1.4]
    ref = bspline_bases(torch.from_numpy(x), torch.from_numpy(sd["layers.1.grid"]), 3).numpy()
    assert np.array_equal(orc.kan_bases(x, sd["layers.1.grid"]), ref)


def test_kan_oracle_matches_reference():
    f = load("kan_fwd_bwd.npz")
    g = load("gt_bach_1s.npz")
    idx = f["subset_idx"]
    t, y = g["coords"][idx].reshape(-1, 1), g["target"][idx]
    sd = _sd("k64")
    out, xs = orc.kan_forward(sd, t, 3)
    ref = f["k64_out"]
    assert np.max(np.abs(out - ref)) < 1e-5 * max(1.0, np.max(np.abs(ref)))
    assert abs(orc.mse(out, y) - float(f["k64_loss"][0])) < 1e-5 * float(f["k64_loss"][0])
    grads = orc.kan_backward(sd, xs, orc.mse_grad(out, y), 3)
    for k, gr in grads.items():
        r = f[f"k64_grad_{k}"]
        rel = np.linalg.norm(gr.reshape(r.shape) - r) / np.linalg.norm(r)
        assert rel < 1e-4, (k, rel)


def test_span_by_count_equals_span_predicate():
    """kan.hip kan_bases_window (KAN_WINDOW_GATHER): for non-decreasing knots the span found by
    counting, s = #{j : g[j] <= x} - 1 if that count is 1 .. 11 else -1, equals the span of the
    per-span predicate g[j] <= x < g[j+1] (kan.py:94-96's order-0 bases), for x on, between and
    outside the knots, +-inf and NaN, on uniform grids (efficient-KAN init) and on sorted grids
    with repeated knots (what update_grid can produce)."""
    rng = np.random.default_rng(0)
    grids = [(np.arange(-3, 9, dtype=np.float32) * np.float32(0.4) - np.float32(1.0))]
    for _ in range(40):
        g = np.sort(rng.normal(size=12).astype(np.float32))
        if rng.random() < 0.5:  # repeated knots
            k = rng.integers(0, 11)
            g[k + 1] = g[k]
        grids.append(g)
    for g in grids:
        xs = np.concatenate([g, np.nextafter(g, np.float32(np.inf)), np.nextafter(g, np.float32(-np.inf)),
                             rng.uniform(g[0] - 1, g[-1] + 1, 200).astype(np.float32),
                             np.array([np.inf, -np.inf, np.nan], dtype=np.float32)])
        for x in xs:
            s_pred = -1
            for j in range(11):
                if g[j] <= x < g[j + 1]:
                    s_pred = j
            cnt = int(np.sum(x >= g))
            s_cnt = cnt - 1 if 1 <= cnt <= 11 else -1
            assert s_cnt == s_pred, (g, x)


def test_hip_path_rejects_unsorted_knots():
    """The HIP KAN path counts knots to find a span, which needs non-decreasing knots: a grid
    that is not is rejected before any launch; after the grid is restored the layer passes."""
    from inr_for_audio_amd import kan as hk
    torch.manual_seed(0)
    lay = hk.KANLinear(4, 3)
    hk._hip_check_layer(lay)
    keep = lay.grid.clone()
    with torch.no_grad():
        lay.grid[2, 5], lay.grid[2, 6] = lay.grid[2, 6].item(), lay.grid[2, 5].item()
    with pytest.raises(NotImplementedError, match="non-decreasing"):
        hk._hip_check_layer(lay)
    with torch.no_grad():
        lay.grid.copy_(keep)
    hk._hip_check_layer(lay)
