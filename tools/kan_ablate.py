"""KAN kernel ablation (measurement only, never the product): builds libsiren_hip variants with
KAN_ABL = 1 (trivial basis stand-in), 2 (no chunk products), 3 (both) and runs
`bench.py --config cfg5` on each in a child process, printing each variant's per-kind kernel
times.  Separates the fused kernels' basis work, their MFMA products and their load / barrier
skeleton.

    python tools/kan_ablate.py --build-only          (here, on the CPU)
    python tools/kan_ablate.py [--variants 0,1,2,3]  (on the GPU box)
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lib_path(v: str) -> str:
    return os.path.join(ROOT, "inr-for-audio_amd", "libsiren_hip.so" if v == "0" else f"libsiren_hip_kanabl{v}.so")


CHILD = """
import runpy, sys
sys.path.insert(0, {root!r})
from inr_for_audio_amd import _lib
_lib.load({lib!r})
sys.argv = ["bench.py", "--config", "cfg5", "--steps", "10", "--warmup", "3", "--no-cpu-baseline"]
runpy.run_path({bench!r}, run_name="__main__")
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--build-only", action="store_true")
    args = ap.parse_args()
    variants = args.variants.split(",")
    if args.build_only:
        import __graft_entry__ as ge
        for v in variants:
            if v != "0":
                ge.build_diagnostic([f"KAN_ABL={v}"], os.path.basename(lib_path(v)))
        return
    for v in variants:
        code = CHILD.format(root=ROOT, lib=lib_path(v), bench=os.path.join(ROOT, "bench.py"))
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=ROOT)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not line:
            print(json.dumps({"variant": v, "error": r.stderr[-1500:]}))
            sys.exit(1)
        d = json.loads(line[0])
        print(json.dumps({"variant": v, "ms_per_step": d["ms_per_step"],
                          "kernels": {k: round(x["avg_ms"], 4) for k, x in d["kernels"].items()}}), flush=True)


if __name__ == "__main__":
    main()
