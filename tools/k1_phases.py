#!/usr/bin/env python3
"""Per-phase timing of the fused K1 kernel from in-kernel timestamps.

Needs the diagnostic library (python bmfr_amd/_build.py --diag) and runs with
BMFR_LIB=diag BMFR_STAMPS=1 (set here before importing bmfr_amd).  Prints,
over all blocks of the last frame, the median / mean shader cycles spent in
each phase and the spread of block start times.
"""
import os
import sys

os.environ["BMFR_LIB"] = "diag"
os.environ["BMFR_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bmfr_amd  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tool_cfg import parse  # noqa: E402

# W H [FRAMES] (FRAMES = the last frame whose K1 phases to report; frames
# 0..FRAMES run twice, the second pass reported) + bench.py's config flags
a, cfg = parse(default_frames=3)
W, H = a.W, a.H
report = [a.frames]
den = bmfr_amd.Denoiser(cfg)
G = den.sizes.blocks
names = ["accumulate_noisy", "min/max scale", "QR", "back-subst", "weighted+blend"]
# frames rendered up front; a first pass over them untimed (GPU at its working clock)
frames = [a.render(f) for f in range(max(report) + 1)]
for f in range(len(frames) * 2):
    fr = frames[f % len(frames)]
    g = f % len(frames)
    vp, _ = bmfr_amd.synth_camera(W, H, max(g - 1, 0))
    _, jit = bmfr_amd.synth_camera(W, H, g)
    den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, g)
    if f < len(frames) or g not in report:
        continue
    f = g
    torch.cuda.synchronize()
    buf = np.zeros(G * 8, np.uint64)
    rc = den.lib.bmfr_debug_stamps(den.handle, buf.ctypes.data_as(C.c_void_p), buf.size)
    assert rc == 0, rc
    st = buf.reshape(G, 8).astype(np.int64)
    d = np.diff(st[:, :6], axis=1)
    tot = st[:, 5] - st[:, 0]
    print(f"{W}x{H} frame {f}: {G} blocks; block lifetime cycles median {np.median(tot):.0f} mean {tot.mean():.0f}")
    for i, n in enumerate(names):
        print(f"  {n:18s} median {np.median(d[:, i]):8.0f}  mean {d[:, i].mean():8.0f}  share {d[:, i].sum() / tot.sum():.2%}")
    rt = st[:, 7] - st[:, 6]
    ok = rt > 0
    print(f"  shader clock (block cycles / 100 MHz realtime) median {np.median(tot[ok] / rt[ok]) * 0.1:.3f} GHz")
    span = st[:, 5].max() - st[:, 0].min()
    print(f"  kernel span (cycles) {span}, start spread {st[:, 0].max() - st[:, 0].min()}", flush=True)
