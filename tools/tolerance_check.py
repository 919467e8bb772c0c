#!/usr/bin/env python3
"""Relative L2 of a libbmfr build's TAA output (the frame output) against the
reference kernels (oracle/_ref, strict and default builds) frame by frame,
for builds that are not bit-exact by design (experiments such as
-DBMFR_FAST_FIT; BMFR_LIB selects the build).  Runs on the GPU box.

  [FAST_FIT=1] BMFR_LIB=NAME python tools/tolerance_check.py [CONFIG [FRAMES]]
  (CONFIG: a FULL_REF_CONFIGS name, default f3840x2160_h13)

The Denoiser runs with library_powr = 1 (the reference kernel's powr), so a
bit-exact build reads 0 against the strict reference."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bmfr_amd  # noqa: E402
import ref_run  # noqa: E402
from ref_configs import FULL_REF_CONFIGS  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "f3840x2160_h13"
rc = FULL_REF_CONFIGS[name]
N = int(sys.argv[2]) if len(sys.argv) > 2 else rc.frames
W, H = rc.width, rc.height
cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, scaled=rc.scaled, use_half_precision_in_tmp_data=rc.half_tmp,
                          library_powr=1, fast_fit=int(os.environ.get("FAST_FIT", "0")))
den = bmfr_amd.Denoiser(cfg)
refs = {m: ref_run.RefLoop(rc, m) for m in ("strict", "default") if ref_run.available(rc.name, m)}
out = torch.empty(W * H * 3, device="cuda")
worst = {m: 0.0 for m in refs}
for f in range(N):
    fr = bmfr_amd.synth_frame_device(W, H, f)
    vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
    _, jit = bmfr_amd.synth_camera(W, H, f)
    den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
    den.copy_output(out)
    row = {"frame": f}
    for m, rl in refs.items():
        rec = {}
        rl.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        rl.run_stages(vp, jit, f, record=rec)
        rl.swap()
        a, b = out.double(), rec["result"].double()
        e = float(torch.linalg.norm(a - b) / torch.linalg.norm(b))
        row[m] = e
        worst[m] = max(worst[m], e)
    print(json.dumps(row), flush=True)
print("RESULT " + json.dumps({"config": name, "frames": N, "lib": os.environ.get("BMFR_LIB", ""),
                              "worst_rel_l2": worst}), flush=True)
