#!/usr/bin/env python3
"""Device time of every bmfr_process_frame call of the synthetic sequence
(HIP events on the stream around each call -- the frames keep their
production schedule, one launch each, unlike libbmfr's per-kernel
profiling, which splits K1 and K2), averaged over runs of 10 frames.

  python tools/frame_times.py [W H FRAMES [PASSES]]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bmfr_amd  # noqa: E402

W, H, N = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (3840, 2160, 100)))
frames = [bmfr_amd.synth_frame_device(W, H, f) for f in range(N)]
P = int(sys.argv[4]) if len(sys.argv) > 4 else 2
# All passes enqueued back to back (contexts made up front, one synchronize at
# the end): the GPU never idles between passes.
dens = [bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H)) for _ in range(P)]
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
