#!/usr/bin/env python3
"""Predicted multi-GPU strong scaling of the 8K frame from one-GPU measurements
(BASELINE config 4; the 8-GPU run itself is the driver's).

For a TX x TY grid of the W x H frame, every rank's tile runs on this one GPU
as its own tiled context, frame after frame, as bench.py --gpus N runs it:
bmfr_process_frame_interior, then bmfr_process_frame_border (the halo left
stale: timing only -- the exchange is what this predicts), with HIP events
around each part.  Per rank: interior and border ms (means over frames
5..FR-1; every tile alone on the whole GPU, as it is on its own GPU), the halo
bytes it sends / receives per frame (bmfr_halo_plan, mean over the 16 grid
shifts) and the largest message to one peer.  The untiled W x H frame is timed
the same way (the 1-GPU point).

Prediction per rank (bench.py's overlap: the exchange on its own stream under
the interior blocks, the border after both):
    frame = max(interior, pack + transfer + unpack) + border
with transfer = the largest single-peer message / LINK_GBS (each peer pair has
its own xGMI link; messages to different peers run in parallel) + RCCL_US of
fixed cost per grouped batch, pack / unpack at HBM rate (PACK_GBS); the job's
frame = the slowest rank.  Printed for LINK_GBS = 50 (a conservative RCCL
point-to-point rate on one link) and 100 GB/s.

  [FAST_FIT=1] python tools/scale_predict.py [W H TX TY [FRAMES]]   (default 7680 4320 4 2 20)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bmfr_amd  # noqa: E402
from bmfr_amd import tiling  # noqa: E402

args = [int(x) for x in sys.argv[1:]]
W, H, TX, TY = (args[:4] if len(args) >= 4 else [7680, 4320, 4, 2])
FR = args[4] if len(args) > 4 else 20
FAST = int(os.environ.get("FAST_FIT", "1"))
HALO = 64
RCCL_US = 30.0   # fixed cost of one grouped send / receive batch (launch + handshake), assumed
PACK_GBS = 3000.0  # pack / unpack kernels: strided 2D copies at ~0.4 of the HBM roof, assumed
grid = tiling.TileGrid(W, H, TX, TY, halo=HALO)


def frames_for(cfg, region):
    fr = [bmfr_amd.synth_region_device(W, H, region, f) for f in range(FR)]
    cams = [(bmfr_amd.synth_camera(W, H, max(f - 1, 0))[0], bmfr_amd.synth_camera(W, H, f)[1]) for f in range(FR)]
    return fr, cams


def time_ctx(cfg, split):
    den = bmfr_amd.Denoiser(cfg)
    fr, cams = frames_for(cfg, den.region)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(FR)]
    for f in range(FR):
        a = (fr[f]["noisy"], fr[f]["normals"], fr[f]["positions"], fr[f]["albedo"], cams[f][0], cams[f][1], f)
        ev[f][0].record()
        if split:
            den.process_frame_interior(*a)
            ev[f][1].record()
            den.process_frame_border(*a)
        else:
            den.process_frame(*a)
            ev[f][1].record()
        ev[f][2].record()
    torch.cuda.synchronize()
    it = float(np.mean([ev[f][0].elapsed_time(ev[f][1]) for f in range(5, FR)]))
    bd = float(np.mean([ev[f][1].elapsed_time(ev[f][2]) for f in range(5, FR)]))
    return den, it, bd


def plan_bytes(den, rank):
    """Per frame (mean over the 16 shifts): bytes sent, received, largest
    single-peer message (either direction)."""
    sent, recv, big = [], [], []
    for f in range(16, 32):
        p = tiling.native_plan(den.cfg, grid, rank, f)
        s_tot = r_tot = m = 0
        for _peer, send, rcv in p:
            sb = sum(den_bytes(den, rec) for rec in send)
            rb = sum(den_bytes(den, rec) for rec in rcv)
            s_tot += sb
            r_tot += rb
            m = max(m, sb, rb)
        sent.append(s_tot)
        recv.append(r_tot)
        big.append(m)
    return float(np.mean(sent)), float(np.mean(recv)), float(np.mean(big))


def den_bytes(den, rec):
    """Packed bytes of one bmfr_halo_copy record {x, y, w, h, planes}."""
    x, y, w, h, planes = rec
    bpp = {1: 12, 2: 1, 4: 12, 8: 12}
    n = 0
    for bit, b in bpp.items():
        if planes & bit:
            n += (w * h * b + 15) // 16 * 16
    return n


full = bmfr_amd.BmfrConfig(image_width=W, image_height=H, fast_fit=FAST)
d1, t1, _ = time_ctx(full, False)
del d1
print(f"{W}x{H} untiled on one GPU, fast_fit = {FAST}: {t1:.4f} ms/frame (frames 5..{FR - 1})")
print(f"grid {TX}x{TY}, halo {HALO}: per rank interior / border ms, halo MB sent / received per frame, "
      f"largest single-peer message MB")
rows = []
for r in range(grid.ranks):
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r), tile_halo=HALO, fast_fit=FAST)
    den, it, bd = time_ctx(cfg, True)
    s, rv, big = plan_bytes(den, r)
    rows.append((r, it, bd, s, rv, big))
    print(f"  rank {r} tile {grid.tile(r)}: interior {it:.4f}  border {bd:.4f}  (sum {it + bd:.4f})  "
          f"sent {s / 1e6:.2f}  received {rv / 1e6:.2f}  largest message {big / 1e6:.2f}", flush=True)
    del den
    torch.cuda.empty_cache()
for gbs in (50.0, 100.0):
    worst = 0.0
    for r, it, bd, s, rv, big in rows:
        xch = (s + rv) / (PACK_GBS * 1e9) * 1e3 + big / (gbs * 1e9) * 1e3 + RCCL_US * 1e-3
        worst = max(worst, max(it, xch) + bd)
    print(f"predicted {grid.ranks}-GPU frame at {gbs:.0f} GB/s per link: {worst:.4f} ms  "
          f"(speedup {t1 / worst:.2f}x vs the untiled frame's {t1:.4f} ms)")
no_x = max(it + bd for _, it, bd, *_ in rows)
print(f"without any exchange cost (slowest rank's interior + border): {no_x:.4f} ms, speedup {t1 / no_x:.2f}x")
