"""A/B of whole bench steps across builds of the library: `bench.py --config C` in a child process
per (round, library), libraries alternating, per-kind kernel ms per step printed per run.

    python tools/lib_ab.py --config cfg5 --libs base=inr-for-audio_amd/libsiren_hip.so,x=inr-for-audio_amd/libsiren_x.so
    python tools/lib_ab.py --config cfg4 --libs a=inr-for-audio_amd/libsiren_hip.so,q2=inr-for-audio_amd/libsiren_hip.so --opts q2=8:2
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = """
import runpy, sys
sys.path.insert(0, {root!r})
from inr_for_audio_amd import _lib
lib = _lib.load({lib!r})
for opt, val in {opts!r}:
    _lib.check(lib.siren_set_option(opt, val), "set_option")
sys.argv = ["bench.py", "--config", {cfg!r}, "--steps", "10", "--warmup", "3", "--no-cpu-baseline", "--no-recon-snr"]
runpy.run_path({bench!r}, run_name="__main__")
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5")
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--opts", default="", help="per-library siren_set_option pairs: name=OPT:VAL[;OPT:VAL],...")
    args = ap.parse_args()
    libs = dict(item.split("=") for item in args.libs.split(","))
    opts = {}
    for item in filter(None, args.opts.split(",")):
        nm, pairs = item.split("=")
        opts[nm] = [tuple(int(v) for v in pr.split(":")) for pr in pairs.split(";")]
    res = {nm: [] for nm in libs}
    for _ in range(args.rounds):
        for nm, path in libs.items():
            code = CHILD.format(root=ROOT, lib=os.path.join(ROOT, path), cfg=args.config, opts=opts.get(nm, []),
                                bench=os.path.join(ROOT, "bench.py"))
            out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600,
                                 check=True).stdout
            d = json.loads(out.strip().splitlines()[-1])
            row = {"ms_per_step": round(d["ms_per_step"], 4),
                   **{k: round(v["ms_per_step"], 4) for k, v in d["kernels"].items()}}
            res[nm].append(row)
            print(json.dumps({"lib": nm, **row}), flush=True)
    med = {nm: {k: sorted(r[k] for r in rows)[len(rows) // 2] for k in rows[0]} for nm, rows in res.items()}
    print(json.dumps({"config": args.config, "median": med}))


if __name__ == "__main__":
    main()
