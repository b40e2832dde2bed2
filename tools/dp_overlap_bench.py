"""Single-GPU emulation of the data-parallel step's communication/compute overlap (VERDICT r2
item 5).  The DP step all-reduces each per-layer gradient bucket on a communication
stream as soon as the backward records its grad_ready event (engine.py SirenEngine.step); RCCL's
kernels then hold CUs while the remaining dX / dW GEMMs run, and those GEMMs are persistent (one
block per CU).  Here the RCCL kernels are replaced by a CU-occupying stand-in
(tools/micro/rccl_standin.hip: `blocks` blocks reduce-copying the bucket `reps` times into scratch)
and the step is timed three ways, interleaved in one process:
  none     the 1-GPU step (no communication)
  overlap  stand-ins on the communication stream behind the grad_ready events (the DP schedule)
  serial   the same stand-ins after the whole backward (no overlap)
for the default forward-only tile queue and with the dX / dX0 GEMMs on the queue too
(SIREN_OPT_NT_QUEUE 2: late blocks take fewer tiles instead of stretching the launch).

    python tools/dp_overlap_bench.py [--blocks 32] [--reps 6] [--steps 6] [--rounds 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MICRO = os.path.join(ROOT, "tools", "micro")


def standin_lib():
    so = os.path.join(MICRO, "librccl_standin.so")
    src = os.path.join(MICRO, "rccl_standin.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", so],
                       check=True)
    lib = ctypes.CDLL(so)
    lib.rccl_standin.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p]
    lib.rccl_standin.restype = ctypes.c_int
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--blocks", type=int, default=32, help="stand-in blocks per bucket (RCCL channels)")
    ap.add_argument("--reps", type=int, default=6, help="reduce-copy passes per bucket")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    sl = standin_lib()
    if args.build_only:
        return
    import __graft_entry__ as ge
    ge.build()
    from inr_for_audio_amd import _lib
    from inr_for_audio_amd.engine import SirenEngine
    from inr_for_audio_amd.models import SirenWithSnakeTanh
    lib = _lib.load()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = SirenWithSnakeTanh(1, 1, 1024, 4, 0, 0, first_omega_0=3000.0, hidden_omega_0=30.0)
    n = args.rows
    t = torch.linspace(-1, 1, n).reshape(n, 1)
    y = 0.5 * torch.sin(2 * math.pi * 440 * t) + 0.3 * torch.sin(2 * math.pi * 3100 * t + 0.5)
    eng = SirenEngine(model, t, y, lr=1e-5, device=dev)
    eng._setup_buckets()  # grad_ready events on the last micro-batch, bucket spans, comm stream
    comm = eng._comm
    scratch = torch.empty(eng.grads.numel() + 64, device=dev)

    def standins(stream):
        for k, lo, hi in eng._buckets:
            m = (hi - lo) // 4 * 4
            if m:
                st = sl.rccl_standin(scratch[lo:lo + m].data_ptr(), eng.grads[lo:lo + m].data_ptr(), m, args.blocks,
                                     args.reps, stream.cuda_stream)
                assert st == 0, st

    cur = torch.cuda.current_stream(dev)

    def step(mode):
        eng._launch_grads()
        if mode == "overlap":
            with torch.cuda.stream(comm):
                # one stand-in per bucket, each behind its own event
                for k, lo, hi in eng._buckets:
                    comm.wait_event(eng._events[k])
                    m = (hi - lo) // 4 * 4
                    if m:
                        assert sl.rccl_standin(scratch[lo:lo + m].data_ptr(), eng.grads[lo:lo + m].data_ptr(), m,
                                               args.blocks, args.reps, comm.cuda_stream) == 0
            cur.wait_stream(comm)
        elif mode == "serial":
            standins(cur)
        eng._launch_update()

    # the stand-in alone, for its duration per bucket
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        standins(cur)
    e1.record()
    torch.cuda.synchronize()
    alone_ms = e0.elapsed_time(e1) / 5
    cases = [(mode, q) for q in (1, 2) for mode in ("none", "overlap", "serial")]
    times = {c: [] for c in cases}
    for _ in range(2):
        step("none")
    for _ in range(args.rounds):
        for mode, q in cases:
            _lib.check(lib.siren_set_option(8, q), "queue option")
            step(mode)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.steps):
                step(mode)
            e1.record()
            torch.cuda.synchronize()
            times[(mode, q)].append(e0.elapsed_time(e1) / args.steps)
    lib.siren_set_option(8, 1)
    res = {f"{mode}_q{q}": round(sorted(v)[len(v) // 2], 4) for (mode, q), v in times.items()}
    print(json.dumps({"rows": n, "buckets": len(eng._buckets), "standin_blocks": args.blocks,
                      "standin_reps": args.reps, "standin_all_buckets_ms": round(alone_ms, 4),
                      "ms_per_step_median": res}, indent=1))


if __name__ == "__main__":
    main()
