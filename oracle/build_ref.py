#!/usr/bin/env python3
"""Compile the reference OpenCL kernels for gfx950 into oracle/_ref/.

TEST INFRASTRUCTURE ONLY.  The reference source is compiled where it lies
(/root/reference/opencl/bmfr.cl, pulled in by oracle/ref_wrappers.cl via
#include); nothing of it is copied into the repository.  The compiler is ROCm's
clang with its own OpenCL device libraries, i.e. the toolchain the reference's
OpenCL runtime would use on this GPU; nothing is stubbed.

Outputs per (config, mode): `<name>_<mode>.hsaco` and `<name>_<mode>.json`
(kernel argument offsets read from the code object's metadata).  The .hsaco
files are git-ignored but travel to the GPU box with the gpurun snapshot.

Usage: python oracle/build_ref.py [--ref /root/reference/opencl] [--force]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from ref_configs import FULL_REF_CONFIGS, REF_CONFIGS, REF_MODES  # noqa: E402

CLANG = "/opt/rocm/lib/llvm/bin/clang"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
OUT = os.path.join(HERE, "_ref")


def kernel_layouts(hsaco: str) -> dict:
    notes = subprocess.run([READELF, "--notes", hsaco], check=True,
                           capture_output=True, text=True).stdout
    start = notes.index("---")
    end = notes.index("\n...", start)
    meta = yaml.safe_load(notes[start:end])
    out = {}
    for k in meta["amdhsa.kernels"]:
        args = [
            {"offset": a[".offset"], "size": a[".size"], "kind": a[".value_kind"]}
            for a in k[".args"]
            if not a[".value_kind"].startswith("hidden_")
        ]
        out[k[".name"]] = {
            "args": args,
            "kernarg_size": k[".kernarg_segment_size"],
            "group_segment_fixed_size": k[".group_segment_fixed_size"],
            "vgpr_count": k[".vgpr_count"],
        }
    return out


def build(ref_dir: str, force: bool = False) -> list:
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(HERE, "ref_wrappers.cl")
    built = []
    for name, cfg in {**REF_CONFIGS, **FULL_REF_CONFIGS}.items():
        for mode, flags in REF_MODES.items():
            hsaco = os.path.join(OUT, f"{name}_{mode}.hsaco")
            meta = os.path.join(OUT, f"{name}_{mode}.json")
            if not force and os.path.exists(hsaco) and os.path.exists(meta) and \
                    os.path.getmtime(hsaco) >= os.path.getmtime(src):
                built.append(hsaco)
                continue
            cmd = [CLANG, "-x", "cl", "-cl-std=CL1.2", "-target", "amdgcn-amd-amdhsa",
                   "-mcpu=gfx950", "-O3", "-Xclang", "-finclude-default-header",
                   "-Wno-everything", "-I", ref_dir, *flags, *cfg.ref_build_options(),
                   src, "-o", hsaco]
            subprocess.run(cmd, check=True)
            with open(meta, "w") as f:
                json.dump({"config": name, "mode": mode, "flags": flags,
                           "kernels": kernel_layouts(hsaco)}, f, indent=1)
            built.append(hsaco)
    return built


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/opencl")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    if not os.path.exists(os.path.join(a.ref, "bmfr.cl")):
        sys.exit(f"reference source not found under {a.ref}")
    for p in build(a.ref, a.force):
        print(p)


if __name__ == "__main__":
    main()
