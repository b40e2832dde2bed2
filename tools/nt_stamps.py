"""Where the persistent NT GEMM's time goes, from in-kernel s_memtime stamps.

Builds a measurement-only variant of the library with -DSIREN_NT_STAMPS
(inr-for-audio_amd/libsiren_hip_stamps.so, never loaded by the package), runs the NT forward
/ dx / dx0 kernels at the headline shape, and prints per-tile medians (cycles) of:
  main    tile start -> end of the last K-step's MFMAs
  wait    of which spent in the K-step vmcnt waits + barriers
  epi     end of MFMAs -> end of the epilogue (incl. the early prefetch issue)
  gap     end of epilogue -> next tile's start
plus the spread of the blocks' first-tile start times.  The stamps themselves cost a few %.

    python tools/nt_stamps.py [--rows 1048576] [--hidden 1024]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarize(st, ntiles_block):
    """st: [grid][256][4] u64 -> dict of medians."""
    out = {}
    g = st.shape[0]
    nt = ntiles_block
    s = st[:, :nt, :].astype(np.float64)
    start, wait, mend, eend = s[..., 0], s[..., 1], s[..., 2], s[..., 3]
    main = mend - start
    epi = eend - mend
    gap = start[:, 1:] - eend[:, :-1]
    out["main_cyc"] = float(np.median(main))
    out["wait_cyc"] = float(np.median(wait))
    out["epi_cyc"] = float(np.median(epi))
    out["gap_cyc"] = float(np.median(gap)) if nt > 1 else 0.0
    out["first_tile_main_cyc"] = float(np.median(main[:, 0]))
    out["first_tile_wait_cyc"] = float(np.median(wait[:, 0]))
    t0 = start[:, 0]
    out["start_spread_cyc"] = float(t0.max() - t0.min())
    out["block_total_cyc_med"] = float(np.median(eend[:, -1] - start[:, 0]))
    out["block_total_cyc_max"] = float(np.max(eend[:, -1] - start[:, 0]))
    out["kernel_span_cyc"] = float(eend[:, -1].max() - start[:, 0].min())
    # by tile index: is the first/last tile special?
    out["main_by_tile"] = [float(np.median(main[:, i])) for i in (0, 1, 2, nt // 2, nt - 1)]
    out["epi_by_tile"] = [float(np.median(epi[:, i])) for i in (0, 1, 2, nt // 2, nt - 1)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--stagger", type=int, default=0)
    args = ap.parse_args()
    import __graft_entry__ as ge
    path = ge.build_diagnostic(["SIREN_NT_STAMPS"], "libsiren_hip_stamps.so")
    from inr_for_audio_amd import _lib
    lib = _lib.load(path)
    lib.siren_debug_nt_stamps.argtypes = [ctypes.c_void_p]
    lib.siren_debug_nt_stamps.restype = None
    dev = torch.device("cuda:0")
    R, H = args.rows, args.hidden
    s = torch.cuda.current_stream().cuda_stream
    P = lambda t: t.data_ptr()  # noqa: E731
    bf = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.rand(R, H, device=dev, generator=g) * 2 - 1).to(bf)
    lim = math.sqrt(6 / H) / 30
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * lim).to(bf)
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    Y = torch.empty(R, H, dtype=bf, device=dev)
    C = torch.empty_like(Y)
    dZ = (torch.randn(R, H, device=dev, generator=g) * 1e-3).to(bf)
    dZp = torch.empty_like(Y)
    part = torch.empty(R // 128, 3, H, device=dev)
    t = torch.linspace(-1, 1, R, device=dev).reshape(R, 1)
    cases = {
        "fwd": lambda: lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(Y), P(C), None, None, s),
        "dx": lambda: lib.siren_inner_bwd_dx(P(dZ), P(W), P(C), ctypes.c_float(30.0), R, H, None, P(dZp), P(part), s),
        "dx0": lambda: lib.siren_first_bwd_dx(P(dZ), P(W), P(C), P(t), 1, ctypes.c_float(3000.0), R, H, None, P(part), s),
    }
    lib.siren_set_option(5, args.stagger)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    ntiles = (R // 256) * (H // 256)
    per_block = ntiles // ncu
    buf = torch.zeros(ncu * 256 * 4, dtype=torch.int64, device=dev)
    res = {"rows": R, "hidden": H, "cus": ncu, "tiles_per_block": per_block, "stagger": args.stagger}
    for name, fn in cases.items():
        for _ in range(5):  # warm clocks, no stamps
            _lib.check(fn(), name)
        lib.siren_debug_nt_stamps(ctypes.c_void_p(P(buf)))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        _lib.check(fn(), name)
        ev1.record()
        torch.cuda.synchronize()
        lib.siren_debug_nt_stamps(None)
        st = buf.cpu().numpy().view(np.uint64).reshape(ncu, 256, 4)
        r = summarize(st, per_block)
        r["ms"] = ev0.elapsed_time(ev1)
        r["clock_ghz_est"] = r["kernel_span_cyc"] / (r["ms"] * 1e6)
        res[name] = r
        print(name, json.dumps(r), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
