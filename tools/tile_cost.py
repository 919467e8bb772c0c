#!/usr/bin/env python3
"""Cost of the tiled frame path on one GPU, without the exchange: rank r's
tile of a tx x ty grid of W x H tiles, each frame as process_frame or as
process_frame_interior + process_frame_border (halo left stale: timing only),
against the untiled W x H frame.  Prints ms/frame for each.

  [FAST_FIT=1] python tools/tile_cost.py [W H TX TY RANK]   (default: 3840 2160 4 2 5;
  the 8K strong-scaling tile of 8 GPUs: 1920 2160 4 2 5)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bmfr_amd  # noqa: E402
from bmfr_amd import tiling  # noqa: E402

W, H, TX, TY, RANK = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (3840, 2160, 4, 2, 5)))
FR = 30
grid = tiling.TileGrid(W * TX, H * TY, TX, TY, halo=64)


def run(cfg, split):
    den = bmfr_amd.Denoiser(cfg)
    reg = den.region
    frames = [bmfr_amd.synth_region_device(cfg.image_width, cfg.image_height, reg, f) for f in range(FR)]
    cams = [(bmfr_amd.synth_camera(cfg.image_width, cfg.image_height, max(f - 1, 0))[0],
             bmfr_amd.synth_camera(cfg.image_width, cfg.image_height, f)[1]) for f in range(FR)]
    t0 = None
    for f in range(FR):
        if f == 5:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        fr, (vp, jit) = frames[f], cams[f]
        args = (fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        if split:
            den.process_frame_interior(*args)
            den.process_frame_border(*args)
        else:
            den.process_frame(*args)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / (FR - 5)


FAST = int(os.environ.get("FAST_FIT", "0"))  # FAST_FIT=1: bmfr_config.fast_fit (the bench headline's fit)
full = bmfr_amd.BmfrConfig(image_width=W, image_height=H, fast_fit=FAST)
tile = bmfr_amd.BmfrConfig(image_width=W * TX, image_height=H * TY, tile=grid.tile(RANK), tile_halo=64, fast_fit=FAST)
print(f"fast_fit = {FAST}")
print(f"untiled {W}x{H}: {run(full, False):.4f} ms/frame")
print(f"tile {grid.tile(RANK)} of {W * TX}x{H * TY}, one call: {run(tile, False):.4f} ms/frame")
print(f"same tile, interior + border calls: {run(tile, True):.4f} ms/frame")
