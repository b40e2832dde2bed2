"""Provenance of libsiren_hip.so: which sources and defines a library was compiled from.

__graft_entry__._compile embeds source_hash(defines) in the library (capi.hip siren_build_id, behind
the marker ``SIREN_BUILD_ID=``); the build step compares the id read from the file with the hash of
the sources beside it (no file times involved) and rebuilds on a mismatch, and _lib.load() refuses a
library whose id does not match them.  No torch import here: the build step uses it before the
package can be imported.
"""
from __future__ import annotations

import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
HEADER = os.path.join(os.path.dirname(PKG), "include", "siren_hip.h")
SOURCES = ["capi.hip", "gemm_nt.hip", "gemm_nt1.hip", "gemm_nt2.hip", "gemm_tn.hip", "elementwise.hip", "kan.hip", "layer_fp32.hip"]
HEADERS = ["siren_common.h", "siren_kernels.h", "gemm_pipeline.h"]
ARCH = "gfx950"
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
         "-Wno-unused-variable", "-Wno-unused-function"]
MARKER = b"SIREN_BUILD_ID="


def sources_present() -> bool:
    return all(os.path.exists(os.path.join(CSRC, f)) for f in SOURCES + HEADERS) and os.path.exists(HEADER)


def source_hash(defines=()) -> str:
    """SHA-256 over every source, header and the include/ C-ABI header (name and bytes, fixed
    order), the compile flags and the sorted extra defines."""
    h = hashlib.sha256()
    for name in SOURCES + HEADERS:
        h.update(name.encode() + b"\0")
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    h.update(b"include/siren_hip.h\0")
    with open(HEADER, "rb") as f:
        h.update(f.read())
    h.update(" ".join(FLAGS).encode() + b"\0")
    h.update(" ".join(sorted(defines)).encode())
    return h.hexdigest()


def lib_build_id(path: str) -> str | None:
    """The id embedded in a built library, read from the file (None: no marker / no file)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    i = data.find(MARKER)
    if i < 0:
        return None
    j = i + len(MARKER)
    k = data.find(b"\0", j)
    return data[j:k].decode(errors="replace")
