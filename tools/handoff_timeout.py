"""How long a fused last layer's hand-off timeout takes (the per-wait figure was a guess).

Runs the SIREN_DIAG library's fault hook (SIREN_OPT_HB_FAULT bit 0: column tile 1 never publishes its
head partial) at several poll limits and at the product's default (kHeadSpinLimit), one step each,
and prints the wall time per step and per poll.  With the fail-fast stall check every wait of the
launch stops once the first one has given up, so a voided step costs about one timeout.

    python tools/handoff_timeout.py [--rows 65536] [--limits 16384,65536,262144,0]   (0 = default)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIMIT = 1 << 23  # gemm_nt.hip kHeadSpinLimit (2^25 until round 6: 5.4 s per voided launch)
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--limits", default="16384,65536,262144,0")
    args = ap.parse_args()
    import __graft_entry__ as ge
    from inr_for_audio_amd import _lib
    diag = _lib.bind(ge.DIAG_LIB, expect_build_id=_lib.expected_build_id(ge.DIAG_DEFINES))
    _lib._lib = diag
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    n = args.rows
    model = SirenWithSnakeTanh(1, 1, 1024, 2, 0, 0, first_omega_0=3000.0, hidden_omega_0=30.0)
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    eng = SirenEngine(model, t, 0.5 * torch.sin(37 * t), device=dev)
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.step()
    torch.cuda.synchronize()
    clean = time.perf_counter() - t0
    out = {"rows": n, "clean_step_s": clean, "runs": []}
    for lim in [int(x) for x in args.limits.split(",")]:
        assert diag.siren_set_option(10, (lim << 8) | 1) == 0
        try:
            t0 = time.perf_counter()
            eng.step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        finally:
            assert diag.siren_set_option(10, 0) == 0
        stalls = int(eng.guard[5].item())
        eng.clear_stalls()
        polls = lim if lim > 0 else DEFAULT_LIMIT
        out["runs"].append({"limit": lim or "default", "polls": polls, "step_s": round(dt, 4), "stalls": stalls,
                            "us_per_poll": round((dt - clean) / polls * 1e6, 4)})
        print(json.dumps(out["runs"][-1]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
