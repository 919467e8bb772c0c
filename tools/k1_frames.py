#!/usr/bin/env python3
"""K1 / K2 device time of every frame of the synthetic sequence (libbmfr's
profiling events, stride 1), to see how the per-frame cost moves along the
sequence (spp growth, reprojection acceptance).

  python tools/k1_frames.py [W H FRAMES [PASSES]] [--third-order] [--input-half] [--f32-tmp]

With PASSES > 1 the whole sequence runs again from frame 0 in a fresh
context, back to back (separates a per-frame data effect from the GPU's
clock ramp at the start of a run).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bmfr_amd  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tool_cfg import parse  # noqa: E402

a, cfg = parse(default_passes=1)
W, H, N, PASSES = a.W, a.H, a.frames, a.passes
frames = [a.render(f) for f in range(N)]
for ps in range(PASSES):
    den = bmfr_amd.Denoiser(cfg)
    den.set_profiling(True, capacity=N, stride=1)
    for f in range(N):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        fr = frames[f]
        den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
    torch.cuda.synchronize()
    prof = den.profile()
    k1 = np.array([p[1] for p in prof])
    k2 = np.array([p[2] for p in prof])
    print(f"pass {ps}")
    for lo in range(0, N, 10):
        print(f"frames {lo:3d}-{min(lo + 9, N - 1):3d}: K1 {k1[lo:lo + 10].mean():.4f} ms  "
              f"K2 {k2[lo:lo + 10].mean():.4f} ms")
    print(f"frames 5-24 K1 {k1[5:25].mean():.4f}  frames 5-{N - 1} K1 {k1[5:].mean():.4f}")
    del den
