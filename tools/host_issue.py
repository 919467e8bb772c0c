#!/usr/bin/env python3
"""Host cost of one tiled frame on the native exchange path, without RCCL:
every tile of a TX x TY grid of the W x H frame as its own context on ONE
GPU, the halo exchange through libbmfr's bmfr_exchange_run_all (the same
plans and pack / unpack kernels as bmfr_exchange_run, the transfers as
device copies).  Per frame, each tile's process_frame_interior, then one
run_all, then each tile's process_frame_border -- what the ranks of a
multi-GPU run enqueue, all from one host thread.  Prints the host time to
enqueue a frame (no synchronisation inside it), per frame and per tile (=
per rank), and the device time per frame of all tiles together.

  [FAST_FIT=1] python tools/host_issue.py [W H TX TY FRAMES]   (default 7680 4320 4 2 12)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bmfr_amd  # noqa: E402
from bmfr_amd import tiling  # noqa: E402

W, H, TX, TY, FR = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (7680, 4320, 4, 2, 12)))
FAST = int(os.environ.get("FAST_FIT", "0"))
grid = tiling.TileGrid(W, H, TX, TY, halo=64)
dens, xs, frames = [], [], []
for r in range(grid.ranks):
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r), tile_halo=64, fast_fit=FAST)
    d = bmfr_amd.Denoiser(cfg)
    dens.append(d)
    frames.append([bmfr_amd.synth_region_device(W, H, d.region, f) for f in range(FR)])
xs = [tiling.NativeExchange(d, grid, r, None) for r, d in enumerate(dens)]
cams = [(bmfr_amd.synth_camera(W, H, max(f - 1, 0))[0], bmfr_amd.synth_camera(W, H, f)[1]) for f in range(FR)]
torch.cuda.synchronize()
host, dev = [], []
for f in range(FR):
    vp, jit = cams[f]
    args = [(fr[f]["noisy"], fr[f]["normals"], fr[f]["positions"], fr[f]["albedo"], vp, jit, f) for fr in frames]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for d, a in zip(dens, args):
        d.process_frame_interior(*a)
    if f > 0:
        tiling.NativeExchange.run_all(xs, f)
    for d, a in zip(dens, args):
        d.process_frame_border(*a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if f >= 2:
        host.append(t1 - t0)
        dev.append(t2 - t0)
for d in dens:
    d.halo_status()  # raises if a frame reprojected past the halo
h = 1e3 * float(np.mean(host))
print(f"{TX}x{TY} tiles of {W}x{H} on one GPU, native exchange (device copies), fast_fit = {FAST}, "
      f"frames 2..{FR - 1}")
print(f"host enqueue per frame: {h:.3f} ms for {grid.ranks} tiles = {h / grid.ranks:.3f} ms per tile (rank)")
print(f"wall per frame (all tiles on one GPU): {1e3 * float(np.mean(dev)):.3f} ms")
for x in xs:
    x.close()
