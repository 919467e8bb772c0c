#!/usr/bin/env python3
"""BMFR frame throughput on MI355X.

One step = one frame of the BMFR hot path (bmfr.cpp:417-485: accumulate_noisy
-> fitter -> weighted_sum -> accumulate_filtered -> taa), run by libbmfr's
fused kernels (K1 per 32x32 block + K2 TAA) on synthetic 1-spp frames that
are rendered on the GPU and resident in HBM before timing starts (the
reference also excludes uploads and readback, bmfr.cpp:415-416,478).

Workload at N=1: 3840x2160, reference default parameters (B = 13 features,
half tmp_data, 32x32 blocks), frames W..W+K-1 of the sequence (temporal path
active on every timed frame), with bmfr_config.fast_fit (--fit fast, the
default): the fitter's Householder trailing update as one fused FMA per
element, its wave-wide reductions as butterflies and its pivot square roots /
reciprocals at hardware precision -- within north_star's 1e-4 relative L2 of
the reference (measured 1.2e-5 against its strict build, 1.6e-5 against its
default build, which is itself 1.2e-5 from the strict one;
tests/test_gpu_fast_fit.py pins exactly this configuration at 4K) -- and the exact path (bit-exact to the reference's
strict build, the library's default) as `ms_per_frame_exact` beside it
(--fit exact swaps the two).

The N = 1 line also carries the metric's other sizes, untiled on the same
GPU: `ms_per_frame_1080p` (1920x1080) and `ms_per_frame_8k` (7680x4320, the
1-GPU point of the north star's scaling target); BASELINE's other 4K
configurations with their own rooflines: `ms_per_frame_cfg5` (config 5:
half input planes, 3rd-order features, B = 16) and `ms_per_frame_f32tmp`
(f32 tmp_data), both with the headline's fit; `ms_per_frame_exact` (or,
with --fit exact, `ms_per_frame_fast_fit`): the headline configuration with
the other fit; and
`ms_per_frame_sequence`: the same 4K frames through bmfr_process_sequence
(K2 of frame f inside K1 of f + 1's launch, as the reference's frame loop
enqueues every frame without waiting).  `value` stays the per-frame API's
number (bmfr_process_frame: each frame's output complete at its return).

Multi-GPU (torchrun, one process per GPU): BASELINE config 4 -- one
7680x4320 frame cut into a tile grid (2x1, 2x2, 4x2 for N = 2, 4, 8), one
tile per rank (--scaling strong, the default for N > 1), each rank
denoising its tile with a tiled context; before every frame the ranks
exchange the halo ring of the previous frame's temporal state over RCCL
(bmfr_amd/tiling.py, DESIGN.md "Multi-GPU"), overlapped with the tile's
interior blocks.  Rank 0 first times the same frames untiled on its own GPU
(`ms_per_frame_1gpu`, `speedup_vs_1gpu`); per-rank exchange / interior /
border times and halo bytes come back in `ranks`.  --scaling weak instead
gives every rank a --width x --height tile.  Timing: barrier + synchronize
around K frames (exchange included), max over ranks.

Untiled per-frame runs (the N = 1 `value`): below 4096 K1 blocks (1080p) a
frame is one launch (K1 blocks, then the frame's TAA tiles, include/bmfr.h
bmfr_sizes.frame_launches) and the timed frames run with nothing between
their launches (an event between two frames costs ~5 us of GPU time at
1080p, profiles/r06_gap_1080p.txt): two HIP events around the timed region
give the device's frame period (`device_ms_per_frame`); an untimed pass over
the same frames with events around each launch gives the frame kernel's
duration (`roofline.launch_ms`, `kernel_ms.frame_one_launch`), and another
with libbmfr's per-kernel events K1 and K2 timed as separate launches.  Larger frames (4K, 8K) are two launches, K1
then K2; they, sequence and tiled runs record libbmfr's per-kernel events
(on the launch stream) on every 10th timed frame.

Extra JSON fields: `roofline` for the dominant kernel of the timed region
(the one-launch frame kernel, with the frame's algorithmic bytes; K1 where
frames are not one launch), `roofline_k1` / `roofline_k2` for K1 and the TAA
kernel timed apart (compulsory bytes: bench.k1_bytes_per_px /
k2_bytes_per_px); `cpu_baseline` = the CPU oracle
(oracle/liboracle.so, OpenMP) on a bounded sample of the same sequence.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bmfr_amd  # noqa: E402
from bmfr_amd import tiling  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def k1_bytes_per_px(s: int) -> int:
    """Algorithmic bytes per pixel (SURVEY.md §8d, 18*s + 74; s = 4 for f32
    input planes, 2 for half), split over the two kernels by which one
    touches each compulsory byte.  K1 reads noisy/normal/position (9s) +
    previous normal/position (6s) + accumulated noisy (12) + spp (1) +
    accumulated filtered (12) and writes accumulated noisy (12) + spp (1) +
    accumulated filtered (12): 15s + 50 (110 for f32)."""
    return 15 * s + 50


def k2_bytes_per_px(s: int) -> int:
    """K2's compulsory bytes: albedo (3s) + previous TAA output (12) + output
    (12); the accumulated filtered colour and the reprojected positions it
    reads are K1's intermediates (their bytes are not compulsory)."""
    return 3 * s + 24


def frame_bytes_per_px(s: int) -> int:
    """K1's plus K2's: albedo (3s) + previous TAA output (12) + output (12)."""
    return 18 * s + 74


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--width", type=int, default=None, help="default 3840 (N = 1), 7680 (N > 1)")
    ap.add_argument("--height", type=int, default=None, help="default 2160 (N = 1), 4320 (N > 1)")
    ap.add_argument("--half-tmp", type=int, default=1)
    ap.add_argument("--third-order", action="store_true", help="B = 16 feature set (BASELINE config 5)")
    ap.add_argument("--input-half", action="store_true",
                    help="half3 input planes (BASELINE config 5's fp16 feature buffers)")
    ap.add_argument("--library-powr", action="store_true",
                    help="tone map with the device library's powr (bit-identical to the reference kernel "
                         "on gfx950) instead of the correctly rounded one")
    ap.add_argument("--fit", choices=("fast", "exact"), default="fast",
                    help="fast (default): bmfr_config.fast_fit = 1, the fitter's trailing update as one fused FMA "
                         "(not bit-exact; within 1e-4 -- measured 1.2e-5 -- rel-L2 of the reference's strict build, "
                         "tests/test_gpu_fast_fit.py); exact: upstream's roundings, bit-exact to the reference's "
                         "strict build (the library default)")
    ap.add_argument("--no-1080p", action="store_true", help="skip the 1920x1080 line (N = 1 only)")
    ap.add_argument("--spin-up", type=float, default=1.0,
                    help="seconds of untimed frames (a scratch context) before each measured run (clock ramp)")
    ap.add_argument("--no-sequence", action="store_true", help="skip the sequence-mode field of the N = 1 line")
    ap.add_argument("--no-8k", action="store_true", help="skip the untiled 7680x4320 line (N = 1) / the 1-GPU "
                                                         "reference time (N > 1)")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the N = 1 line's config-5 (half inputs, B = 16) and f32-tmp_data fields")
    ap.add_argument("--frames-8k", type=int, default=30, help="timed frames of the untiled 8K line (N = 1)")
    ap.add_argument("--cpu-frames", type=int, default=12,
                    help="timed CPU-oracle frames (0 = skip); 12 at 4K is ~10 s of host work")
    ap.add_argument("--seed", type=int, default=0x424D4652)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="multi-GPU: strong = one --width x --height frame split (default), "
                         "weak = one --width x --height tile per GPU")
    ap.add_argument("--halo", type=int, default=64, help="tile halo in pixels (>= 34 + max motion)")
    ap.add_argument("--grid", default=None,
                    help="multi-GPU tile grid COLSxROWS (default: 2x1, 2x2, 4x2 for N = 2, 4, 8 -- the 4x2 tiles "
                         "of 8K are 1920x2160, a shorter halo perimeter than 2x4's 3840x1080)")
    ap.add_argument("--sequence", action="store_true",
                    help="single GPU: the timed frames as one bmfr_process_sequence call (TAA of frame f beside "
                         "K1 of frame f+1) instead of one bmfr_process_frame per frame")
    ap.add_argument("--exchange", choices=("native", "torch"), default="torch",
                    help="multi-GPU over RCCL: torch (default) = torch.distributed isend / irecv between libbmfr's "
                         "pack / unpack kernels -- the path the gloo rehearsals run end to end; native = libbmfr's "
                         "bmfr_exchange_run (pack + grouped ncclSend / ncclRecv + unpack, one C call per frame), "
                         "whose RCCL branch has not yet run between two ranks (tests/test_gpu_exchange.py "
                         "test_rccl_two_gpus_matches_untiled needs a multi-GPU box)")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false",
                    help="multi-GPU: exchange the halo before the frame instead of under K1's interior blocks")
    a = ap.parse_args(argv)
    a.fast_fit = a.fit == "fast"
    return a


def psnr(a: np.ndarray, b: np.ndarray) -> float:
    mse = float(np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2))
    return 10 * np.log10(1.0 / mse) if mse > 0 else float("inf")


def cpu_model() -> str:
    """The host CPU's model string (/proc/cpuinfo), for cpu_baseline."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(cfg: bmfr_amd.BmfrConfig, frames: int, seed: int):
    """CPU oracle on the first frames+1 frames of the same sequence; frame 0
    untimed (the reference's Total also starts at frame 1, bmfr.cpp:497-502)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    W, H = cfg.image_width, cfg.image_height
    loop = pyoracle.OracleLoop(pyoracle.make_cfg(W, H, cfg.not_scaled, cfg.scaled,
                                                 cfg.use_half_precision_in_tmp_data))
    times = []
    for f in range(frames + 1):
        # the frame the GPU runs process (the GPU renderer), copied to host memory
        g = bmfr_amd.synth_frame_device(W, H, f, seed=seed)
        fr = {k: g[k].cpu().numpy().reshape(H, W, 3) for k in ("noisy", "normals", "positions", "albedo")}
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        loop.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        t0 = time.perf_counter()
        loop.run_stages(vp, jit, f)
        dt = time.perf_counter() - t0
        loop.swap()
        if f > 0:
            times.append(dt)
    ms = 1e3 * float(np.mean(times))
    return {"value": round(ms, 2), "unit": "ms/frame", "cores": pyoracle.load().oracle_threads(),
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "kind": "port",
            "sample": f"{W}x{H} frames 1..{frames} of the same synthetic sequence (frame 0 untimed), "
                      f"oracle/bmfr_oracle.c with OpenMP"}


def pmc_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), when one exists for this
    workload: `<workload>` K1, `<workload>_k2` K2, `<workload>_frame` the
    one-launch frame kernel, `<workload>_two_launch` K1 + K2 of one frame."""
    p = os.path.join(ROOT, "profiles", "pmc_k1.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    return d.get(workload, {}).get("hbm_bytes_per_launch")


def with_traffic(roof: dict, workload_key: str, launch_ms: float) -> dict:
    """roof plus the launch's measured HBM bytes (pmc_traffic) as a rate:
    the algorithmic roofline counts compulsory bytes only, while K2 also
    re-reads K1's intermediates (accumulated colour, reprojected positions:
    20 B/px) -- its bound is the bytes it actually moves."""
    t = pmc_traffic(workload_key)
    roof["traffic"] = t
    if t and launch_ms:
        g = t / (launch_ms * 1e-3) / 1e9
        roof["traffic_gbs"] = round(g, 1)
        roof["traffic_frac"] = round(g / HBM_PEAK_GBS, 4)
    return roof


PROF_STRIDE = 10  # timed frames between two recorded with per-kernel events


class NativeTransport:
    """DistTransport's interface over libbmfr's native exchange (bmfr_exchange_run)."""

    def __init__(self, x, comm):
        self.x, self.comm = x, comm  # the communicator outlives the exchange

    @property
    def last_bytes(self):
        return self.x.last_bytes

    def exchange_ctx(self, denoiser, frame):
        self.x.run(frame)


def run_sequence(a, W, H, tile, grid, rank, world, dev, backend, steps, warmup, per_frame=False):
    """Denoise frames 0..warmup+steps-1 of the synthetic W x H sequence (this
    rank's tile of it); time the last `steps` frames.  Returns the timings,
    per-kernel HIP-event means and the PSNR of the last output."""
    scaled = bmfr_amd.SCALED_THIRD_ORDER if a.third_order else bmfr_amd.SCALED_DEFAULT
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, scaled=scaled,
                              use_half_precision_in_tmp_data=a.half_tmp,
                              tile=tile if grid else None, tile_halo=a.halo if grid else 0,
                              input_half=int(a.input_half), library_powr=int(a.library_powr),
                              fast_fit=int(a.fast_fit))
    local = dev.index
    den = bmfr_amd.Denoiser(cfg, device=local)
    region = den.region
    # Per-kernel HIP events are recorded on every PROF_STRIDE-th frame of the
    # timed region (libbmfr's profiling stride), so the kernel breakdown and
    # the roofline come from the timed frames at a small cost to the rest.
    nfr = warmup + steps
    seed = a.seed

    # Render every frame's region into HBM up front (untimed).
    frames = [bmfr_amd.synth_region_device(W, H, region, f, seed=seed, device=local) for f in range(nfr)]
    if a.input_half:  # the planes as half3 (the f32 render rounded to nearest)
        frames = [{k: (v.half() if k in ("noisy", "normals", "positions", "albedo") else v) for k, v in fr.items()}
                  for fr in frames]
    cams = []
    for f in range(nfr):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        cams.append((vp, jit))
    scratch = spin_up(a, cfg, local, frames, cams)  # its last frames still run under the warm-up frames
    transport = None
    if grid:
        # torch.distributed point-to-point (RCCL with the nccl backend; gloo, host-staged, in the
        # one-GPU rehearsal) between libbmfr's pack / unpack kernels; --exchange native: libbmfr's
        # own exchange (one C call per frame enqueues pack, the grouped ncclSend / ncclRecv batch
        # and unpack)
        transport = tiling.DistTransport(grid, rank, dev, host_staging=backend != "nccl")
        if backend == "nccl" and a.exchange == "native":
            comm_handle = tiling.RcclComm(world, rank, local)
            transport = NativeTransport(tiling.NativeExchange(den, grid, rank, comm_handle), comm_handle)
    # Tiled: the halo exchange runs on its own stream while K1's interior
    # blocks (which need no halo) run on the compute stream
    # (bmfr_process_frame_interior / _border, include/bmfr.h).
    compute = torch.cuda.current_stream(dev)
    comm = torch.cuda.Stream(dev) if grid else None
    frame_done = torch.cuda.Event() if grid else None
    # Split timings of sampled timed frames: (interior start/end, exchange
    # start/end, border end) events, on the streams the work runs on.
    marks = []

    host_issue = []  # tiled frames: host wall time to enqueue one frame (interior, pack, exchange, unpack, border)

    def run(f, mark=False):
        t_issue = time.perf_counter()
        fr = frames[f]
        prev = frames[f - 1] if f > 0 else None
        args = (fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], cams[f][0], cams[f][1], f)
        kw = dict(prev_normals=prev["normals"] if prev else None, prev_positions=prev["positions"] if prev else None)
        if transport is None or f == 0:
            den.process_frame(*args, **kw)
        elif not a.overlap:
            transport.exchange_ctx(den, f)
            den.process_frame(*args, **kw)
        else:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if mark else None
            comm.wait_event(frame_done)  # the previous frame's state is complete
            if ev:
                ev[0].record(compute)
            den.process_frame_interior(*args, **kw)
            if ev:
                ev[1].record(compute)
            with torch.cuda.stream(comm):  # one pack and one unpack kernel around the RCCL batch
                if ev:
                    ev[2].record(comm)
                transport.exchange_ctx(den, f)
                if ev:
                    ev[3].record(comm)
            compute.wait_stream(comm)
            den.process_frame_border(*args, **kw)
            if ev:
                ev[4].record(compute)
                marks.append((ev, transport.last_bytes))
        if frame_done is not None:
            frame_done.record(compute)
            if f > 0:
                host_issue.append(time.perf_counter() - t_issue)

    # Untiled: the whole run as bmfr_process_sequence calls (frames pipelined),
    # unless per_frame; tiled: frame by frame around the halo exchange.
    pipelined = grid is None and not per_frame
    # Untiled per-frame: each frame is one launch (K1 blocks + the frame's TAA
    # tiles), and nothing else is enqueued between the timed frames: an event
    # between two frames' kernels costs ~5 us of GPU time per frame at 1080p
    # (profiles/r06_gap_1080p.txt).  Two HIP events bracket the whole timed
    # region on its stream (`device_ms_per_frame`: the device's frame period);
    # the frame kernel's own duration comes from an untimed pass over the same
    # frames with events around each launch, and the K1 / K2 split from
    # another with libbmfr's per-kernel events (which time the two as separate
    # launches).  Elsewhere the per-kernel events run inside the timed region
    # on every PROF_STRIDE-th frame.
    one_launch = grid is None and per_frame and cfg.sizes().frame_launches == 1
    stride = PROF_STRIDE if steps >= PROF_STRIDE else 1
    tev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if one_launch else None

    def run_range(f0, f1, timed=False):
        if pipelined:
            den.process_sequence(frames[f0:f1], cams[f0:f1], f0)
        else:
            if tev and timed:
                tev[0].record(compute)
            for f in range(f0, f1):
                run(f, mark=timed and not one_launch and f % stride == 0)
            if tev and timed:
                tev[1].record(compute)

    if warmup:
        run_range(0, warmup)
    if not one_launch:
        den.set_profiling(True, capacity=steps, stride=stride)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_range(warmup, warmup + steps, timed=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    frame_kernel_ms = period_ms = None
    if one_launch:
        period_ms = tev[0].elapsed_time(tev[1]) / steps
        # untimed: the same frames again with events around each frame's launch
        # (the frame kernel's duration), then once more with K1 and K2 timed as
        # separate launches
        prof = bmfr_amd.Denoiser(cfg, device=local)
        fev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * steps)]
        for f in range(nfr):
            fr = frames[f]
            if f >= warmup:
                fev[2 * (f - warmup)].record(compute)
            prof.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], cams[f][0], cams[f][1], f)
            if f >= warmup:
                fev[2 * (f - warmup) + 1].record(compute)
        torch.cuda.synchronize()
        frame_kernel_ms = float(np.mean([fev[2 * i].elapsed_time(fev[2 * i + 1]) for i in range(steps)]))
        for f in range(nfr):
            if f == warmup:
                prof.set_profiling(True, capacity=steps, stride=1)
            fr = frames[f]
            prof.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], cams[f][0], cams[f][1], f)
        torch.cuda.synchronize()
        kprof = prof.profile()
        del prof
    else:
        kprof = den.profile()
        den.set_profiling(False)
    overshoot = den.halo_status() if grid else 0  # raises if a frame reprojected past the halo

    # Quality: PSNR of this rank's tile of the last output against the clean render.
    clean = bmfr_amd.synth_region_device(W, H, region, nfr - 1, seed=seed, device=local, clean=True)["clean"]
    out = den.copy_output(torch.empty(region[2] * region[3] * 3, device=dev))
    torch.cuda.synchronize()

    def tile_of(x):
        x = x.view(region[3], region[2], 3)
        return x[tile[1] - region[1]:tile[1] - region[1] + tile[3], tile[0] - region[0]:tile[0] - region[0] + tile[2]]

    last = frames[nfr - 1]
    noisy_tm = torch.clamp(torch.clamp(last["albedo"].float() * last["noisy"].float(), min=0) ** 0.454545, 0, 1)
    split = None
    if marks:
        mean = lambda i, j: float(np.mean([e[i].elapsed_time(e[j]) for e, _ in marks]))  # noqa: E731
        # halo bytes per frame (the exchanged rectangles change with frame % 16)
        split = {"interior_ms": mean(0, 1), "exchange_ms": mean(2, 3), "border_ms": mean(1, 4),
                 "frame_ms": mean(0, 4),
                 "halo_bytes_sent": int(np.mean([b[0] for _, b in marks])),
                 "halo_bytes_received": int(np.mean([b[1] for _, b in marks])),
                 "halo_overshoot_px": overshoot,
                 # host time to enqueue one tiled frame (mean over timed frames > 0);
                 # with gloo this includes the blocking host-staged transfer
                 "host_issue_ms": 1e3 * float(np.mean(host_issue[-steps:])) if host_issue else 0.0}
    res = {
        "cfg": cfg,
        "ms_per_frame": 1e3 * elapsed / steps,
        "k1_ms": float(np.mean([p[1] for p in kprof])),
        "k2_ms": float(np.mean([p[2] for p in kprof])),
        "dev_ms": period_ms if one_launch else float(np.mean([p[3] for p in kprof])),
        "frame_kernel_ms": frame_kernel_ms,
        "psnr": psnr(tile_of(out).cpu().numpy(), tile_of(clean).cpu().numpy()),
        "psnr_in": psnr(tile_of(noisy_tm).cpu().numpy(), tile_of(clean).cpu().numpy()),
        "split": split,
    }
    if isinstance(transport, NativeTransport):
        torch.cuda.synchronize()
        transport.x.close()
        transport.comm.close()
    del frames, den, out, clean, noisy_tm, last, scratch, transport
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def valu_roofline(fast_fit: bool = False):
    """K1's other roof: VALU issue.  From the committed rocprofv3 SQ pass of
    the same bench command (profiles/*sq_counters.json, newest round):
    K1's VALU instructions per SIMD x the achievable issue cost of a wave64
    f32 instruction (3.24 cycles, profiles/r01_valu_rate.txt) / K1's cycles.
    The guide's nominal issue rate (2 cycles, MI355X_MICROARCH.md) gives
    `valu_frac_nominal`.  K1 runs below both roofs -- its limiter is the
    latency of phase 1's dependent gathers and of the fit's pivot chain
    (DESIGN.md section 5)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_sq_counters.json")))
    if fast_fit:  # the SQ passes of the fast_fit K1, when there are any
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_sq_counters_fastfit.json"))) or files
    if not files:
        return {}
    with open(files[-1]) as f:
        d = json.load(f)
    c = d.get("K1 k_fused_cols")
    if not c:
        return {}
    return {"valu_frac": round(c["valu_instr_per_simd"] * 3.24 / c["kernel_cycles_per_xcd"], 3),
            "valu_frac_nominal": round(c["valu_instr_per_simd"] * 2.0 / c["kernel_cycles_per_xcd"], 3),
            "limiter": "latency (phase-1 gathers, the fit's pivot chain) under the HBM and VALU roofs",
            "valu_source": os.path.relpath(files[-1], ROOT) + ": SQ_INSTS_VALU / GRBM_GUI_ACTIVE, "
                                                                "3.24 cycles per wave64 VALU instruction"}


def side_line(r):
    """A secondary-size field of the N = 1 line."""
    d = {"value": round(r["ms_per_frame"], 4), "device_ms_per_frame": round(r["dev_ms"], 4),
         "kernel_ms": {"fused_block_k1": round(r["k1_ms"], 4), "taa_k2": round(r["k2_ms"], 4)},
         "psnr_db": round(r["psnr"], 2)}
    if r["frame_kernel_ms"] is not None:  # one-launch frames: the frame kernel (untimed pass, events around it)
        d["kernel_ms"]["frame_one_launch"] = round(r["frame_kernel_ms"], 4)
        # the frame's time outside its kernel: wall clock per frame minus the
        # device's frame period (host issue / launch boundary), and the device
        # period minus the kernel's own duration (idle between kernels; negative
        # when the events around a lone kernel cost more than back-to-back launches)
        d["gap_ms"] = {"wall_minus_device": round(r["ms_per_frame"] - r["dev_ms"], 4),
                       "device_minus_kernel": round(r["dev_ms"] - r["frame_kernel_ms"], 4)}
    return d


def variant_line(r, s: int, W: int, H: int, workload: str, kernel: str, k1_kernel: str):
    """A same-size configuration field of the N = 1 line (BASELINE config 5,
    f32 tmp_data): side_line plus the roofline of its dominant kernel -- the
    one-launch frame kernel (the frame's 18 s + 74 B/px over the kernel's
    HIP-event duration), or K1 where the frame is two launches."""
    if r["frame_kernel_ms"] is None:
        kb = k1_bytes_per_px(s) * W * H
        ka = kb / (r["k1_ms"] * 1e-3) / 1e9
        return dict(side_line(r), workload=workload,
                    roofline=with_traffic({"bound": "hbm", "achieved": round(ka, 1), "peak": HBM_PEAK_GBS,
                                           "unit": "GB/s", "frac": round(ka / HBM_PEAK_GBS, 4),
                                           "kernel": k1_kernel + " (K1; frame = K1, K2)",
                                           "algorithmic_bytes_per_launch": kb, "launch_ms": round(r["k1_ms"], 4)},
                                          workload, r["k1_ms"]))
    fb = frame_bytes_per_px(s) * W * H
    fa = fb / (r["frame_kernel_ms"] * 1e-3) / 1e9
    return dict(side_line(r), workload=workload,
                roofline={"bound": "hbm", "achieved": round(fa, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(fa / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(workload + "_frame"),
                          "kernel": kernel + " (K1 + K2 of the frame, one launch)",
                          "algorithmic_bytes_per_launch": fb, "launch_ms": round(r["frame_kernel_ms"], 4)})


def spin_up(a, cfg, local, frames, cams):
    """Untimed: the same frames through a scratch context for --spin-up
    seconds before the measured context starts; returns that context, whose
    last frames are still in flight (the caller keeps it alive until after
    the timed region).  The GPU's power management sets the shader clock by
    the load: in-kernel timestamps (tools/k1_phases.py: block cycles over the
    100 MHz real-time counter) read 1.5-1.9 GHz for the first ~30 frames
    after the GPU idled for a few milliseconds, 2.2-2.3 GHz in steady
    state -- so the warm-up is this workload, and it hands over to the
    warm-up frames of the measured context without the GPU going idle
    (tools/frame_times.py: passes enqueued back to back have no slow early
    frames).  A tiled run spins up on an untiled context of its region's
    size over the same rendered planes: no halo exchange to stand in for, no
    never-written ring state read, no reach check that could stop the run."""
    if a.spin_up <= 0:
        return None
    if cfg.tile is not None:
        import dataclasses
        sz = cfg.sizes()
        cfg = dataclasses.replace(cfg, image_width=sz.region_width, image_height=sz.region_height, tile=None,
                                  tile_halo=0)
    scratch = bmfr_amd.Denoiser(cfg, device=local)
    t0, f = time.perf_counter(), 0
    while True:
        for _ in range(8):
            g = f % len(frames)
            fr = frames[g]
            scratch.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], cams[g][0], cams[g][1],
                                  g)
            f += 1
        if time.perf_counter() - t0 >= a.spin_up:
            return scratch
        torch.cuda.synchronize()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # BMFR_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks
    # on one GPU (messages staged through host memory); default RCCL.
    backend = os.environ.get("BMFR_DIST_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    # N = 1: the 4K headline (BASELINE config 3); N > 1: config 4's 8K frame.
    a.width = a.width or (3840 if world == 1 else 7680)
    a.height = a.height or (2160 if world == 1 else 4320)

    tx, ty = tiling.grid_for(world) if not a.grid else tuple(int(v) for v in a.grid.lower().split("x"))
    if tx * ty != world:
        raise SystemExit(f"--grid {a.grid}: {tx * ty} tiles for {world} ranks")
    if a.scaling == "weak":
        W, H = a.width * tx, a.height * ty
    else:
        W, H = a.width, a.height
    grid = tiling.TileGrid(W, H, tx, ty, halo=a.halo) if world > 1 else None
    tile = grid.tile(rank) if grid else (0, 0, W, H)
    # N > 1: rank 0 first times the same frames of the whole frame on its own
    # GPU (the 1-GPU point of the scaling curve); the other ranks wait.
    r1 = None
    if world > 1 and rank == 0 and not a.no_8k:
        r1 = run_sequence(a, W, H, (0, 0, W, H), None, 0, 1, dev, backend, a.steps, a.warmup, per_frame=True)
    if world > 1:
        dist.barrier()
    r = run_sequence(a, W, H, tile, grid, rank, world, dev, backend, a.steps, a.warmup, per_frame=not a.sequence)
    cfg = r["cfg"]
    # The metric's other resolutions (BASELINE.json: ms/frame @1080p & 4K, and
    # the 8K frame of the scaling target), single GPU only.
    r1080 = r8k = rseq = None
    # The same frames as one bmfr_process_sequence call per 64 frames (K2 of
    # frame f in K1 of f + 1's tail): the reference's own frame loop
    # (bmfr.cpp:417-485) enqueues every frame without waiting, as this does.
    if world == 1 and not a.sequence and not a.no_sequence:
        rseq = run_sequence(a, W, H, (0, 0, W, H), None, 0, 1, dev, backend, a.steps, a.warmup, per_frame=False)
    if world == 1 and not a.no_1080p and (W, H) != (1920, 1080):
        r1080 = run_sequence(a, 1920, 1080, (0, 0, 1920, 1080), None, 0, 1, dev, backend, a.steps, a.warmup,
                             per_frame=not a.sequence)
    if world == 1 and not a.no_8k and (W, H) != (7680, 4320):
        n8 = min(a.steps, a.frames_8k)
        r8k = run_sequence(a, 7680, 4320, (0, 0, 7680, 4320), None, 0, 1, dev, backend, n8, a.warmup,
                           per_frame=not a.sequence)
        r8k["steps"] = n8
    # The other same-size configurations BASELINE.json names (N = 1): config 5
    # (fp16 feature buffers + 3rd-order features) and config 3 with f32
    # tmp_data, per-frame API, each with its own roofline.
    rvar = {}
    if world == 1 and not a.no_variants and not a.sequence:
        import copy
        other = ("exact", dict(third_order=False, input_half=False, half_tmp=1, fast_fit=False)) if a.fast_fit \
            else ("fast_fit", dict(third_order=False, input_half=False, half_tmp=1, fast_fit=True))
        for key, upd in (("cfg5", dict(third_order=True, input_half=True, half_tmp=1, fast_fit=a.fast_fit)),
                         ("f32tmp", dict(third_order=False, input_half=False, half_tmp=0, fast_fit=a.fast_fit)),
                         other):
            if all(getattr(a, k) == v for k, v in upd.items()):
                continue  # the main line already is this configuration
            b = copy.copy(a)
            b.__dict__.update(upd)
            rvar[key] = (b, run_sequence(b, W, H, (0, 0, W, H), None, 0, 1, dev, backend, a.steps, a.warmup,
                                         per_frame=True))
    ranks = None
    if world > 1 and r["split"] is not None:
        keys = ("interior_ms", "exchange_ms", "border_ms", "frame_ms", "host_issue_ms", "halo_bytes_sent",
                "halo_overshoot_px")
        v = torch.zeros(world, len(keys), dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        v[rank] = torch.tensor([float(r["split"][k]) for k in keys], dtype=torch.float64)
        dist.all_reduce(v)
        ranks = [{k: (round(float(x), 4) if k.endswith("_ms") else int(x)) for k, x in zip(keys, row)}
                 for row in v.cpu().tolist()]

    s = 2 if a.input_half else 4
    tile_px = tile[2] * tile[3]
    tmp = "half" if a.half_tmp else "f32"
    workload = f"bmfr_{W}x{H}_B{cfg.buffer_count}_{tmp}tmp" + ("_f16in" if a.input_half else "") + \
        ("_fastfit" if a.fast_fit else "")
    ms_per_frame = r["ms_per_frame"]
    if rank == 0:
        achieved = k1_bytes_per_px(s) * tile_px / (r["k1_ms"] * 1e-3) / 1e9
        k1_roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                   "kernel": "k_fused_cols (K1)" if a.half_tmp or a.fast_fit else "k_fused (K1)",
                   "algorithmic_bytes_per_launch": k1_bytes_per_px(s) * tile_px}
        if world == 1:
            with_traffic(k1_roof, workload, r["k1_ms"])
        if world == 1:
            k1_roof.update(valu_roofline(a.fast_fit))
        # Untiled per-frame runs below kTwoLaunchBlocks K1 blocks (bmfr_sizes
        # frame_launches): the frame is one launch (K1 blocks + TAA tiles),
        # the dominant -- only -- kernel of the timed region; its roofline is
        # the frame's algorithmic bytes over its duration, and K1's own (timed
        # apart, untimed pass) is roofline_k1.  Larger frames are two launches
        # and K1, timed live by libbmfr's events, is the dominant kernel.
        one_launch = r["frame_kernel_ms"] is not None
        if one_launch:
            fb = frame_bytes_per_px(s) * tile_px
            fa = fb / (r["frame_kernel_ms"] * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(fa, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(fa / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(workload + "_frame"),
                    "kernel": ("k_fused_cols_taa<..., SAME = true>" if a.half_tmp or a.fast_fit
                               else "k_fused_rows_taa<...>")
                              + " (K1 + K2 of the frame, one launch)",
                    "algorithmic_bytes_per_launch": fb, "launch_ms": round(r["frame_kernel_ms"], 4),
                    "launch_ms_source": "HIP events around each frame's launch on its stream, in an untimed "
                                        "pass over the same frames (the timed frames run without events between "
                                        "them); the rocprofv3 kernel-trace mean of the same command is in "
                                        "profiles/*_kernel_stats.md",
                    "limiter": "K1 blocks: latency of phase-1 gathers and of the fit's pivot chain, VALU issue "
                               "(roofline_k1); TAA tiles: texture path / latency (roofline_k2) -- not HBM"}
        else:
            roof = k1_roof
        roof["frame_frac"] = round(frame_bytes_per_px(s) * W * H / (ms_per_frame * 1e-3) / 1e9 / (HBM_PEAK_GBS * world),
                                   4)
        line = {
            "metric": "ms/frame @1080p & 4K, 1/2/4/8 GPU; PSNR vs 4096spp reference",
            "value": round(ms_per_frame, 4),
            "unit": "ms/frame",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_frame, 4),
            "higher_is_better": False,
            "scaling": a.scaling if world > 1 else "strong",
            "vs_baseline": None,
            "dtype": "f32" + ("+f16 tmp_data" if a.half_tmp else "") + ("+f16 input planes" if a.input_half else ""),
            "data": "synthetic (GPU-rendered 1-spp frames + features, resident in HBM)",
            "config": {"workload": workload, "image": f"{W}x{H}", "buffer_count": cfg.buffer_count,
                       "half_tmp_data": a.half_tmp, "input_half": int(a.input_half),
                       "powr": "device library" if a.library_powr else "correctly rounded",
                       "fit": ("fast_fit: fused trailing update, butterfly reductions, within 1e-4 rel-L2 of the "
                               "reference (measured 1.2e-5 vs its strict build, 1.6e-5 vs its default build; "
                               "tests/test_gpu_fast_fit.py)"
                               if a.fast_fit else "exact: bit-exact to the reference's strict build"),
                       "frames_timed": a.steps,
                       # SHA-256 of the sources libbmfr.so was built from (the loader
                       # refuses a library that is not this tree's: bmfr_amd/_lib.py)
                       "build_id": bmfr_amd.build_id(),
                       "frames_pipelined": world == 1 and a.sequence,
                       "parallelism": (f"tiles {tx}x{ty}, halo {a.halo} px, "
                                       f"{'RCCL' if backend == 'nccl' else backend} halo exchange"
                                       f"{' (libbmfr bmfr_exchange_run)' if backend == 'nccl' and a.exchange == 'native' else ' (torch.distributed)'}"
                                       f"{' overlapped with interior blocks' if a.overlap else ''}")
                       if world > 1 else "single GPU"},
            "device_ms_per_frame": round(r["dev_ms"], 4),
            "kernel_ms": {"fused_block_k1": round(r["k1_ms"], 4), "taa_k2": round(r["k2_ms"], 4)},
            "psnr_db": {"output": round(r["psnr"], 2), "noisy_input": round(r["psnr_in"], 2)},
            "roofline": roof,
        }
        if one_launch:
            line["roofline_k1"] = k1_roof
        if world == 1:
            k2 = k2_bytes_per_px(s) * tile_px / (r["k2_ms"] * 1e-3) / 1e9 if not a.sequence else None
            if k2:
                line["roofline_k2"] = with_traffic(
                    {"bound": "hbm", "achieved": round(k2, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(k2 / HBM_PEAK_GBS, 4), "kernel": "k_fused_taa (K2)",
                     "algorithmic_bytes_per_launch": k2_bytes_per_px(s) * tile_px}, workload + "_k2", r["k2_ms"])
        if rseq is not None:
            line["ms_per_frame_sequence"] = side_line(rseq)
        if r1080 is not None:  # the metric's 1080p half: its frame kernel's roofline too
            wl1080 = workload.replace(f"bmfr_{W}x{H}_", "bmfr_1920x1080_", 1)
            line["ms_per_frame_1080p"] = variant_line(r1080, s, 1920, 1080, wl1080,
                                                      "k_fused_cols_taa<..., SAME = true>" if a.half_tmp or a.fast_fit
                                                      else "k_fused_rows_taa<...>",
                                                      "k_fused_cols" if a.half_tmp or a.fast_fit else "k_fused")
        if r8k is not None:
            line["ms_per_frame_8k"] = dict(side_line(r8k), frames_timed=r8k["steps"])
        if r1 is not None:
            line["ms_per_frame_1gpu"] = side_line(r1)
            line["speedup_vs_1gpu"] = round(r1["ms_per_frame"] / ms_per_frame, 3)
        if world > 1:
            # `value` here is the whole W x H frame cut into tiles; the N = 1
            # line's `value` is the 4K frame -- the 1-GPU point of this curve is
            # ms_per_frame_1gpu (and the N = 1 line's ms_per_frame_8k)
            line["scaling_reference"] = (f"ms_per_frame_1gpu ({W}x{H} untiled, rank 0's GPU)"
                                         if a.scaling == "strong" else "none (weak scaling: one tile per GPU)")
        if ranks is not None:
            line["ranks"] = ranks
        for key, (b, rv) in rvar.items():
            vs = 2 if b.input_half else 4
            wl = f"bmfr_{W}x{H}_B{rv['cfg'].buffer_count}_{'half' if b.half_tmp else 'f32'}tmp" + \
                 ("_f16in" if b.input_half else "") + ("_fastfit" if b.fast_fit else "")
            line[f"ms_per_frame_{key}"] = variant_line(rv, vs, W, H, wl, "k_fused_cols_taa<..., SAME = true>"
                                                       if b.half_tmp or b.fast_fit else "k_fused_rows_taa<...>",
                                                       "k_fused_cols" if b.half_tmp or b.fast_fit else "k_fused")
        if world == 1 and a.cpu_frames > 0:
            line["cpu_baseline"] = cpu_baseline(cfg, a.cpu_frames, a.seed)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
