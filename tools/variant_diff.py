#!/usr/bin/env python3
"""Bitwise comparison of libbmfr builds (GPU box): the same synthetic frames
through the default library and each named variant (BMFR_LIB, built with
tools/ab.py build), fast_fit, headline and config-5 configurations; prints
per variant and configuration the number of frames whose output differs and
the largest relative L2 of a differing frame.

  python tools/variant_diff.py [W H N] VARIANT...
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = sys.argv[1:]
W, H, N = (int(args[0]), int(args[1]), int(args[2])) if args and args[0].isdigit() else (640, 360, 12)
names = [a for a in args if not a.isdigit()]


def frames(lib, cfg, d):
    out = os.path.join(d, f"{lib or 'base'}_{cfg}.npy")
    env = dict(os.environ, BMFR_LIB=lib, BMFR_ALLOW_FOREIGN_BUILD="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "variant_frames.py"), str(W), str(H), str(N),
                        "1", out, cfg], env=env, capture_output=True, text=True, timeout=300)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    return np.load(out)


with tempfile.TemporaryDirectory() as d:
    for cfg in ("default", "cfg5"):
        base = frames("", cfg, d)
        for n in names:
            v = frames(n, cfg, d)
            diff = [f for f in range(N) if v[f].tobytes() != base[f].tobytes()]
            rel = max((float(np.linalg.norm(v[f].astype(np.float64) - base[f]) / np.linalg.norm(base[f]))
                       for f in diff), default=0.0)
            print(f"{cfg:8s} {n:12s} frames differing {len(diff)}/{N}  worst rel-L2 {rel:.3e}", flush=True)
