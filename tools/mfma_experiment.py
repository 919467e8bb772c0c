#!/usr/bin/env python3
"""EXPERIMENT: settle the MFMA trailing-panel question with data (DESIGN.md
section 4).  Runs on the GPU box.

The f32-tmp_data stage pipeline (StagePipeline, library_powr = 1) is run on
the synthetic 3840x2160 sequence with libbmfr's exact VALU fitter
(bmfr_fitter) and with the compact-WY fitter of tools/wy_fitter.hip whose
trailing-panel update runs on MFMA (tools/libwy.so; build:
hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/wy_fitter.hip -o tools/libwy.so)
at each panel width NB (4, 8, 16 = the whole QR as one panel).
Reported: each fitter's kernel time on the same tmp_data (HIP events,
median of 10), the fused f32 K1 for context, and the TAA output's relative L2
to the reference kernels' default build (contraction on) and strict build.

  python tools/mfma_experiment.py [W H FRAMES [B [NB,...]]]   (B = 13 or 16)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bmfr_amd  # noqa: E402
import ref_run  # noqa: E402
from mfma_common import load_wy, run_stages  # noqa: E402
from bmfr_amd._lib import check  # noqa: E402
from bmfr_amd.pipeline import _ptr  # noqa: E402
from ref_configs import FULL_REF_CONFIGS  # noqa: E402

W, H, FR = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (3840, 2160, 4)))
BC = int(sys.argv[4]) if len(sys.argv) > 4 else 13
NBS = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [4, 8, 16]
rc = FULL_REF_CONFIGS.get(f"f{W}x{H}_f{BC}")
wy = load_wy(os.path.join(ROOT, "tools", "libwy.so"))
cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, use_half_precision_in_tmp_data=0, library_powr=1,
                          scaled=bmfr_amd.SCALED_THIRD_ORDER if BC == 16 else bmfr_amd.SCALED_DEFAULT)


def valu_fitter(sp, f):
    check(sp.lib.bmfr_fitter(sp.handle, torch.cuda.current_stream().cuda_stream, _ptr(sp.weights),
                             _ptr(sp.mins_maxs), _ptr(sp.tmp_data), f), "fitter")


def wy_fitter_nb(nb):
    def fit(sp, f):
        G = sp.sizes.blocks
        err = wy.wy_fitter(G, _ptr(sp.tmp_data), _ptr(sp.weights), _ptr(sp.mins_maxs), f, cfg.noise_amount * 2.0,
                           torch.cuda.current_stream().cuda_stream, BC, nb)
        assert err == 0, err
    return fit


def rel_l2(a, b):
    a, b = a.double(), b.double()
    return float(torch.linalg.norm(a - b) / torch.linalg.norm(b))


def time_ms(fn, reps=10):
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return float(np.median(out))


exact = bmfr_amd.StagePipeline(cfg)
blocked = {nb: bmfr_amd.StagePipeline(cfg) for nb in NBS}
refs = {m: ref_run.RefLoop(rc, m) for m in ("strict", "default")} if rc and ref_run.available(rc.name) else {}
res = {"image": f"{W}x{H}", "buffer_count": BC, "tmp_data": "f32", "panel_widths": NBS, "frames": []}
for f in range(FR):
    fr = bmfr_amd.synth_frame_device(W, H, f)
    vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
    _, jit = bmfr_amd.synth_camera(W, H, f)
    for sp, fit in [(exact, valu_fitter)] + [(blocked[nb], wy_fitter_nb(nb)) for nb in NBS]:
        sp.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        run_stages(sp, vp, jit, f, fit)
    row = {"frame": f}
    for m, rl in refs.items():
        rec = {}
        rl.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        rl.run_stages(vp, jit, f, record=rec)
        rl.swap()
        row[f"valu_vs_ref_{m}"] = rel_l2(exact.cur(exact.result), rec["result"])
        for nb in NBS:
            row[f"wy{nb}_vs_ref_{m}"] = rel_l2(blocked[nb].cur(blocked[nb].result), rec["result"])
    for nb in NBS:
        row[f"wy{nb}_vs_valu"] = rel_l2(blocked[nb].cur(blocked[nb].result), exact.cur(exact.result))
    res["frames"].append(row)
    print(json.dumps(row), flush=True)
    if f == FR - 1:  # every fitter on the same tmp_data of this frame's stage 1
        saved = exact.tmp_data.clone()

        def again(fn):
            def go():
                exact.tmp_data.copy_(saved)
                fn(exact, f)
            return go
        copy_only = time_ms(lambda: exact.tmp_data.copy_(saved))
        res["fitter_ms"] = {"valu_exact": time_ms(again(valu_fitter)) - copy_only}
        for nb in NBS:
            res["fitter_ms"][f"mfma_compact_wy_nb{nb}"] = time_ms(again(wy_fitter_nb(nb))) - copy_only
    for sp in [exact] + list(blocked.values()):
        sp.swap()
# the production K1 (f32 tmp_data) for context: fit + everything else of the frame
den = bmfr_amd.Denoiser(cfg)
frames = [bmfr_amd.synth_frame_device(W, H, f) for f in range(8)]
den.set_profiling(True, capacity=8)
for f in range(8):
    vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
    _, jit = bmfr_amd.synth_camera(W, H, f)
    den.process_frame(frames[f]["noisy"], frames[f]["normals"], frames[f]["positions"], frames[f]["albedo"], vp, jit, f)
torch.cuda.synchronize()
res["fused_k1_f32_ms"] = float(np.mean([p[1] for p in den.profile()[2:]]))
print("RESULT " + json.dumps(res), flush=True)
