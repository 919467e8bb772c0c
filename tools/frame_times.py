#!/usr/bin/env python3
"""Device time of every bmfr_process_frame call of the synthetic sequence
(HIP events on the stream around each call -- the frames keep their
production schedule, one launch each, unlike libbmfr's per-kernel
profiling, which splits K1 and K2), averaged over runs of 10 frames.

  python tools/frame_times.py [W H FRAMES [PASSES]] [--third-order] [--input-half] [--f32-tmp]
  (FRAME_LAUNCHES=1 or 2 forces one launch per frame or K1, K2)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bmfr_amd  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tool_cfg import parse  # noqa: E402

a, cfg = parse(default_passes=2)
W, H, N, P = a.W, a.H, a.frames, a.passes
frames = [a.render(f) for f in range(N)]
# All passes enqueued back to back (contexts made up front, one synchronize at
# the end): the GPU never idles between passes.
dens = [bmfr_amd.Denoiser(cfg) for _ in range(P)]
if os.environ.get("FRAME_LAUNCHES"):  # 1 / 2: force the frame's launch form (bmfr_debug_frame_launches)
    for d in dens:
        d.debug_frame_launches(int(os.environ["FRAME_LAUNCHES"]))
evs = [[torch.cuda.Event(enable_timing=True) for _ in range(N + 1)] for _ in range(P)]
torch.cuda.synchronize()
for rep in range(P):
    den, ev = dens[rep], evs[rep]
    ev[0].record()
    for f in range(N):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        fr = frames[f]
        den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        ev[f + 1].record()
torch.cuda.synchronize()
for rep in range(P):
    ev = evs[rep]
    t = np.array([ev[f].elapsed_time(ev[f + 1]) for f in range(N)])
    print(f"pass {rep}: " + "  ".join(f"{lo}-{min(lo + 9, N - 1)}: {t[lo:lo + 10].mean():.4f}" for lo in range(0, N, 10)))
    print(f"  frames 5-24 {t[5:25].mean():.4f}  frames 5-{N - 1} {t[5:].mean():.4f}")
