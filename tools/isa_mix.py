#!/usr/bin/env python3
"""Static instruction mix of libbmfr kernels (CPU only: the built library's
gfx950 code objects, disassembled): per kernel whose demangled name contains
every filter word, the count of VALU / SALU / LDS / vector-memory / DPP
instructions and the most frequent VALU opcodes.  A K1 block runs most of its
code once per wave (phase 1 and 3 unrolled; the fit's column branches are
wave-uniform, so a wave runs about a quarter of the fit's static code).

  python tools/isa_mix.py [--lib bmfr_amd/libbmfr.so] [--top 40] FILTER...
  e.g. python tools/isa_mix.py k_fused_cols "<4, 9, _Float16, true, false>"
"""
import argparse
import collections
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_hazards  # noqa: E402


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return dict(zip(names, out))


def category(op: str) -> str:
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith(("global_atomic", "buffer_atomic")):
        return "vmem_atomic"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_", )):
        return "salu/smem/ctrl"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "bmfr_amd", "libbmfr.so"))
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("filters", nargs="*")
    a = ap.parse_args(argv)
    with tempfile.TemporaryDirectory() as d:
        funcs = {}
        for co in isa_hazards.code_objects(a.lib, d):
            funcs.update(isa_hazards.disassemble(co))
    dm = demangle(list(funcs))
    for sym, insts in sorted(funcs.items(), key=lambda kv: dm[kv[0]]):
        name = dm[sym]
        if not all(f in name for f in a.filters):
            continue
        ops = [s.split(None, 1)[0] for s in insts if s]
        cats = collections.Counter(category(o) for o in ops)
        dpp = sum(1 for s in insts if s and ("row_" in s or "quad_perm" in s or "dpp" in s.split(None, 1)[0]))
        print(f"== {name}\n   {len(ops)} instructions: " + ", ".join(f"{k} {v}" for k, v in cats.most_common())
              + f", dpp {dpp}")
        valu = collections.Counter(o for o in ops if o.startswith("v_"))
        print("   " + "  ".join(f"{o} {n}" for o, n in valu.most_common(a.top)))


if __name__ == "__main__":
    main(sys.argv[1:])
