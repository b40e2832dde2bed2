"""Are the persistent NT GEMM blocks' epilogues synchronised, and what does that cost?

Measurement only.  Builds the SIREN_NT_STAMPS variant of the library (tools/nt_stamps.py),
runs the ping-pong forward / dX at the headline shape with the tile queue on or off and with
start staggers, and reads per tile {start, tile id, end of MFMAs, end of epilogue} from the
chip-wide 100 MHz real-time counter.  Prints per case:
  main_us / epi_us     medians per tile (K-loop; epilogue + stores)
  conc_med             median number of blocks whose epilogue is running at the middle of a
                       block's epilogue (256 = every CU stores at once)
  epi_by_conc          median epilogue time for tiles binned by that concurrency
  burst                peak / mean of the epilogue-start histogram (1 us bins)

    python tools/nt_sync.py [--staggers 0,1,2] [--queue 0,1]
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


def analyse(st, ms):
    """st [grid][256][4] u64: {start, shader-clock count, end of MFMAs, end of epilogue}, times in
    10 ns ticks (unused slots 0)."""
    rows = []
    for b in range(st.shape[0]):
        for i in range(st.shape[1]):
            s0, g, tm, te = (int(x) for x in st[b, i])
            if te == 0:
                break
            rows.append((b, i, s0, g, tm, te))
    a = np.array(rows, dtype=np.float64)
    t0 = a[:, 2].min()
    start, tm, te = (a[:, 2] - t0) * 0.01, (a[:, 4] - t0) * 0.01, (a[:, 5] - t0) * 0.01  # us
    main, epi = tm - start, te - tm
    mid = 0.5 * (tm + te)
    order = np.argsort(tm)
    tms, tes = tm[order], te[order]
    # blocks in their epilogue at each epilogue's midpoint: started before mid and ended after mid
    started = np.searchsorted(tms, mid, side="right")
    ended = np.searchsorted(np.sort(te), mid, side="right")
    conc = started - ended
    bins = [(0, 32), (32, 64), (64, 128), (128, 192), (192, 257)]
    by = {f"{lo}-{hi - 1}": (float(np.median(epi[(conc >= lo) & (conc < hi)])) if np.any((conc >= lo) & (conc < hi)) else None,
                             int(np.sum((conc >= lo) & (conc < hi))))
          for lo, hi in bins}
    h, _ = np.histogram(tm, bins=np.arange(0, te.max() + 1.0, 1.0))
    ti = a[:, 1]
    first = start[ti == 0]
    conc_early = float(np.median(conc[ti <= 2]))
    conc_late = float(np.median(conc[ti >= 10]))
    per = float(np.median(te[ti >= 1] - start[ti >= 1]))
    # shader clock between consecutive tiles of a block: d(s_memtime) / d(real time)
    cyc = a[:, 3]
    same = a[1:, 0] == a[:-1, 0]
    dcyc, dt = (cyc[1:] - cyc[:-1])[same], (te[1:] - te[:-1])[same]
    clk = float(np.median(dcyc / np.maximum(dt, 1e-3)) / 1e3)  # cycles per us / 1e3 = GHz
    return {"ms": ms, "tiles": len(a), "main_us": float(np.median(main)), "epi_us": float(np.median(epi)),
            "conc_med": float(np.median(conc)), "epi_by_conc": by,
            "burst": float(h.max() / max(h.mean(), 1e-9)), "span_us": float(te.max()),
            "first_start_spread_us": float(first.max() - first.min()), "conc_tiles_0_2": conc_early,
            "conc_tiles_10plus": conc_late, "tile_period_us": per, "clock_ghz": clk}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--staggers", default="0,1,2")
    ap.add_argument("--queue", default="0,1")
    ap.add_argument("--cases", default="fwd,dx")
    ap.add_argument("--grid", type=int, default=0, help="SIREN_OPT_NT_GRID (0 = one block per CU)")
    ap.add_argument("--diags", default="0", help="SIREN_OPT_NT_DIAG values (timing-only ablations; the "
                    "queue is off while one is set)")
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
    f16 = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.rand(R, H, device=dev, generator=g) * 2 - 1).to(f16)
    W = ((torch.rand(H, H, device=dev, generator=g) * 2 - 1) * math.sqrt(6 / H) / 30).to(f16)
    b = (torch.rand(H, device=dev, generator=g) - 0.5) * 0.06
    Y, C = torch.empty(R, H, dtype=f16, device=dev), torch.empty(R, H, dtype=f16, device=dev)
    dZ = (torch.randn(R, H, device=dev, generator=g) * 1e-3).to(f16)
    dZp = torch.empty_like(Y)
    part = torch.empty(R // 128, 3, H, device=dev)
    fns = {
        "fwd": lambda: lib.siren_inner_fwd(P(X), P(W), P(b), ctypes.c_float(30.0), R, H, P(Y), P(C), None, None, s),
        "dx": lambda: lib.siren_inner_bwd_dx(P(dZ), P(W), P(C), ctypes.c_float(30.0), R, H, None, P(dZp), P(part), s),
    }
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    buf = torch.zeros(ncu * 256 * 4, dtype=torch.int64, device=dev)
    out = {}
    for name in args.cases.split(","):
        for q in [int(x) for x in args.queue.split(",")]:
            for stg, dg in [(int(x), int(d)) for x in args.staggers.split(",") for d in args.diags.split(",")]:
                _lib.check(lib.siren_set_option(8, 2 if q else 0), "queue")
                _lib.check(lib.siren_set_option(6, dg), "diag")
                _lib.check(lib.siren_set_option(5, stg), "stagger")
                _lib.check(lib.siren_set_option(4, args.grid), "grid")
                for _ in range(3):
                    _lib.check(fns[name](), name)
                buf.zero_()
                lib.siren_debug_nt_stamps(ctypes.c_void_p(P(buf)))
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                _lib.check(fns[name](), name)
                ev1.record()
                torch.cuda.synchronize()
                lib.siren_debug_nt_stamps(None)
                st = buf.cpu().numpy().view(np.uint64).reshape(ncu, 256, 4)
                r = analyse(st, ev0.elapsed_time(ev1))
                key = f"{name}_q{q}_s{stg}_d{dg}"
                out[key] = r
                print(key, json.dumps(r), flush=True)
    lib.siren_set_option(5, 0)
    lib.siren_set_option(6, 0)
    lib.siren_set_option(8, 1)


if __name__ == "__main__":
    main()
