"""Condensed instruction stream of one kernel in a hipcc `-S` (device-only) listing: MFMAs,
ds_reads, LDS-DMA, global loads/stores and VALU/SALU runs collapsed, waits / barriers /
branches and block labels kept -- for reading a K-loop's schedule at a glance.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S gemm_nt.hip -o /tmp/nt.s
    python tools/isa_summary.py /tmp/nt.s <substring of the mangled kernel name> [max_lines]
"""
from __future__ import annotations

import sys


def classify(t: str) -> str:
    op = t.split()[0]
    if op.startswith("v_mfma"):
        return "MFMA"
    if op.startswith("ds_read"):
        return "DSR"
    if op.startswith("ds_write"):
        return "DSW"
    if op == "global_load_lds_dwordx4":
        return "GLDS"
    if op.startswith("global_store"):
        return "GST"
    if op.startswith("global_load"):
        return "GLD"
    if op.startswith("s_waitcnt") or op in ("s_barrier", "s_setprio", "s_sleep") or "branch" in op:
        return t
    if op.startswith("v_"):
        return "V"
    if op.startswith("s_"):
        return "S"
    return op


def main():
    path, key = sys.argv[1], sys.argv[2]
    limit = int(sys.argv[3]) if len(sys.argv) > 3 else 600
    s = open(path).read()
    heads = (ln.split(";")[0].strip() for ln in s.split("\n"))
    names = [h[:-1] for h in heads if h.endswith(":") and key in h and not h.startswith(".")]
    if not names:
        sys.exit(f"no kernel matching {key}")
    name = names[0]
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    ops = []
    for ln in s[i:j].split("\n")[1:]:
        t = ln.strip()
        if not t or t.startswith(";"):
            continue
        if t.startswith("."):
            if t.startswith(".LBB"):
                ops.append(t)
            continue
        ops.append(classify(t))
    res, prev, n = [], None, 0
    for o in ops + [None]:
        if o == prev:
            n += 1
            continue
        if prev is not None:
            res.append(f"{prev} x{n}" if n > 1 else prev)
        prev, n = o, 1
    print(name)
    counts = {k: sum(1 for o in ops if o == k) for k in ("MFMA", "DSR", "GLDS", "GST", "GLD")}
    print("totals:", counts, "barriers:", sum(1 for o in ops if o == "s_barrier"))
    print("\n".join(res[:limit]))


if __name__ == "__main__":
    main()
