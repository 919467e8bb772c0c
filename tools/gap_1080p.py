#!/usr/bin/env python3
"""Where the per-frame time of a small frame goes between its kernels.

The 1080p frame is one launch (include/bmfr.h bmfr_sizes.frame_launches):
its kernel takes ~92 us under rocprofv3 while bench.py's 1080p line reads
~100-104 us per frame.  This runs the same frames (the bench's configuration,
frames W..W+K-1 after a spin-up with the workload) through several issue
forms, each on its own context, enqueued back to back without the GPU idling
between forms, and prints ms/frame of each:

  events    bmfr_process_frame + a timing event after every frame (bench.py's
            one-launch form up to round 5)
  plain     bmfr_process_frame only; wall clock around the K frames
  graph     the K frames captured once into a HIP graph (hipStreamBeginCapture
            via torch.cuda.graph) and replayed: the launch cost without the host
  sequence  bmfr_process_sequence over the K frames (one call)
  two       plain, but forced to two launches per frame (K1 then K2)

plus the host time to enqueue one frame (`host_us`: perf_counter around each
bmfr_process_frame call of the plain form).  With --trace CSV (a rocprofv3
kernel-trace CSV of this script) it instead prints, per kernel name, the
dispatch count, mean duration and the mean idle gap from the previous
dispatch's end to this one's start.

  python tools/gap_1080p.py [W H FRAMES] [--exact]      (default 1920 1080 40)
  python tools/gap_1080p.py --trace gpurun_out/prof/..._kernel_trace.csv
"""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def trace_gaps(path: str) -> None:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    by = {}
    for i, (s, e, n) in enumerate(rows):
        gap = s - rows[i - 1][1] if i else 0
        d = by.setdefault(n, [0, 0.0, 0.0, []])
        d[0] += 1
        d[1] += e - s
        d[2] += gap
        d[3].append(gap)
    for n, (c, dur, gap, gaps) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        gaps.sort()
        med = gaps[len(gaps) // 2] / 1e3
        print(f"{c:6d}  dur {dur / c / 1e3:9.2f} us  gap mean {gap / c / 1e3:8.2f} us  median {med:8.2f} us  {n[:110]}")


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--trace":
        trace_gaps(sys.argv[2])
        return
    import numpy as np
    import torch

    import bmfr_amd
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    W, H, K = (int(x) for x in (args + ["1920", "1080", "40"][len(args):]))
    fast = "--exact" not in sys.argv
    WARM = 5
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, fast_fit=int(fast))
    n = WARM + K
    frames = [bmfr_amd.synth_frame_device(W, H, f) for f in range(n)]
    cams = [(bmfr_amd.synth_camera(W, H, max(f - 1, 0))[0], bmfr_amd.synth_camera(W, H, f)[1]) for f in range(n)]

    def one(d, f):
        fr = frames[f]
        d.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], cams[f][0], cams[f][1], f)

    # spin-up: ~1 s of the same frames (clock ramp, bench.py spin_up)
    scratch = bmfr_amd.Denoiser(cfg)
    t0, f = time.perf_counter(), 0
    while time.perf_counter() - t0 < 1.0:
        for _ in range(16):
            one(scratch, f % n)
            f += 1
        torch.cuda.synchronize()

    res = {}
    host = []
    for rep in range(2):
        for form in ("events", "plain", "graph", "sequence", "two"):
            d = bmfr_amd.Denoiser(cfg)
            if form == "two":
                d.debug_frame_launches(2)
            for f in range(WARM):
                one(d, f)
            if form == "graph":
                # frames WARM.. captured once (the context's frame state advances in
                # the capture exactly as in a run; the replay repeats those frames:
                # frame WARM's inputs again, so its state slots match the capture)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        for f in range(WARM, n):
                            one(d, f)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g.replay()
                torch.cuda.synchronize()
                res.setdefault(form, []).append(1e3 * (time.perf_counter() - t0) / K)
                del g
                continue
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)] if form == "events" else None
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if form == "sequence":
                d.process_sequence(frames[WARM:n], cams[WARM:n], WARM)
            else:
                if ev:
                    ev[0].record()
                for i, f in enumerate(range(WARM, n)):
                    h0 = time.perf_counter()
                    one(d, f)
                    if form == "plain":
                        host.append(time.perf_counter() - h0)
                    if ev:
                        ev[i + 1].record()
            torch.cuda.synchronize()
            res.setdefault(form, []).append(1e3 * (time.perf_counter() - t0) / K)
            if ev:
                res.setdefault("events_device", []).append(
                    float(np.mean([ev[i].elapsed_time(ev[i + 1]) for i in range(K)])))
    print(f"{W}x{H}, fast_fit={int(fast)}, frames {WARM}..{n - 1}, two rounds of each form:")
    for k, v in res.items():
        print(f"  {k:14s} " + "  ".join(f"{x:.4f}" for x in v) + " ms/frame")
    print(f"  host_us        {1e6 * float(np.mean(host)):.1f} us per bmfr_process_frame call (plain form)")


if __name__ == "__main__":
    main()
