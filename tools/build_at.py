"""Build libsiren_hip.so from the sources of an earlier commit, for same-box A/B and PMC
bisects (tools/ab_bench.py binds it with check_abi=False):

    python tools/build_at.py b067ce9 r15        # -> inr-for-audio_amd/libsiren_r15.so
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    commit, tag = sys.argv[1], sys.argv[2]
    out = os.path.join(ROOT, "inr-for-audio_amd", f"libsiren_{tag}.so")
    with tempfile.TemporaryDirectory() as td:
        arch = subprocess.run(["git", "-C", ROOT, "archive", commit, "inr-for-audio_amd/csrc", "include"],
                              check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", td], input=arch, check=True)
        csrc = os.path.join(td, "inr-for-audio_amd", "csrc")
        srcs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".hip"))
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-w", *srcs, "-o", out]
        subprocess.run(cmd, check=True)
    print(out)


if __name__ == "__main__":
    main()
