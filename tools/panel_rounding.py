#!/usr/bin/env python3
"""How far a blocked (compact-WY) trailing update lands from the reference
when tmp_data is half -- the numerical half of the MFMA question.

A compact-WY Householder QR applies the NB steps of a panel to the trailing
columns as one contraction, X - V (T^T (V^T X)): the one shape in the fitter
MFMA can run.  But the reference rounds every trailing column to half after
EVERY step (bmfr.cl:640-653, vstore_half); a blocked update rounds it once per
panel.  This runs the CPU oracle twice on the same frames -- the reference's
rounding (panel 0) and the blocked rounding (panel NB: trailing columns beyond
the panel rounded only at its last step, tools build oracle/bmfr_oracle.c with
-DORACLE_PANEL_EXPERIMENT) -- and reports the TAA output's relative L2
distance per frame, next to north_star's 1e-4 and to the distance of the
reference's own f32-tmp_data build.  MFMA would also change the sums'
association (f32 accumulation in another order): not modelled, it only adds.

  python tools/panel_rounding.py [W H frames] [--third-order]  -> JSON on stdout
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
LIB = os.path.join(ROOT, "tools", "liboracle_panel.so")


def build():
    src = os.path.join(ROOT, "oracle", "bmfr_oracle.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["gcc", "-O2", "-std=c99", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                        "-DORACLE_PANEL_EXPERIMENT", "-shared", "-o", LIB, src, "-lm"], check=True)


def run(W, H, n, scaled, half_tmp, panel):
    import pyoracle
    import bmfr_amd
    pyoracle.LIB_PATH = LIB
    lib = pyoracle.load()
    lib.oracle_set_panel.argtypes = [C.c_int]
    lib.oracle_set_panel(panel)
    loop = pyoracle.OracleLoop(pyoracle.make_cfg(W, H, bmfr_amd.NOT_SCALED_DEFAULT, scaled, half_tmp))
    outs = []
    for f in range(n):
        fr = bmfr_amd.synth_frame_host(W, H, f)
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        loop.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        rec = {}
        loop.run_stages(vp, jit, f, record=rec)
        loop.swap()
        outs.append(rec["result"].astype(np.float64))
    return outs


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def main(argv):
    third = "--third-order" in argv
    args = [int(a) for a in argv if a.isdigit()]
    W, H, n = (args + [640, 360, 8])[:3] if args else (640, 360, 8)
    import bmfr_amd
    scaled = bmfr_amd.SCALED_THIRD_ORDER if third else bmfr_amd.SCALED_DEFAULT
    build()
    ref = run(W, H, n, scaled, 1, 0)
    res = {"image": f"{W}x{H}", "frames": n, "buffer_count": 4 + len(scaled) + 3,
           "metric": "TAA output relative L2 vs the reference rounding (oracle == reference strict build)"}
    f32 = run(W, H, n, scaled, 0, 0)
    res["f32_tmp_data"] = [rel(a, b) for a, b in zip(f32, ref)]
    for nb in (2, 4, 8, 16):
        o = run(W, H, n, scaled, 1, nb)
        res[f"panel_{nb}"] = [rel(a, b) for a, b in zip(o, ref)]
    # MFMA for the dot products only (V^T X and the WY identity, from values
    # not rounded since the panel began), every update still rounded per step
    for nb in (2, 4, 8):
        o = run(W, H, n, scaled, 1, -nb)
        res[f"dots_only_panel_{nb}"] = [rel(a, b) for a, b in zip(o, ref)]
    res["worst"] = {k: max(v) for k, v in res.items() if isinstance(v, list)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
