"""A long sequence: spp saturates at 255 (bmfr.cl:433-442, `sample_spp >
254.f ? 255 : ...`) after ~255 frames of accepted reprojection, and the noise
tables roll over four 64-frame batches.  The fused per-frame path must equal
the CPU oracle (oracle/bmfr_oracle.c) bit for bit on every frame's output,
accumulated colour and spp through and past the saturation.

At 64x64 a moving camera's taps land a whole pixel (~0.4 scene units) from
their surface points and fail POSITION_LIMIT_SQUARED, so spp would stay
small: the scene and camera are held still after frame 16 (frame 16's
inputs and camera every frame -- each pixel reprojects onto itself), while
the per-frame noise terms still change."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest
import torch

import bmfr_amd

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))


def test_spp_saturation_matches_oracle(gpu):
    import pyoracle
    W, H, N = 64, 64, 270
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H)
    den = bmfr_amd.Denoiser(cfg)
    orc = pyoracle.OracleLoop(pyoracle.make_cfg(W, H, cfg.not_scaled, cfg.scaled, 1))
    out = torch.empty(W * H * 3, device="cuda")
    acc = torch.empty(W * H * 3, device="cuda")
    spp = torch.empty(W * H, dtype=torch.uint8, device="cuda")
    top = 0
    for f in range(N):
        g = min(f, 16)
        fr = bmfr_amd.synth_frame_host(W, H, g)
        vp, _ = bmfr_amd.synth_camera(W, H, max(g - 1, 0) if f <= 16 else 16)
        _, jit = bmfr_amd.synth_camera(W, H, g)
        d = {k: torch.from_numpy(v.reshape(-1)).cuda() for k, v in fr.items()}
        den.process_frame(d["noisy"], d["normals"], d["positions"], d["albedo"], vp, jit, f)
        orc.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        rec = {}
        orc.run_stages(vp, jit, f, record=rec)
        orc.swap()
        den.copy_output(out)
        den.copy_state("filtered_accumulated", acc)
        den.copy_state("spp", spp)
        got_spp = spp.cpu().numpy()
        assert out.cpu().numpy().tobytes() == rec["result"].tobytes(), f"frame {f}: output"
        assert acc.cpu().numpy().tobytes() == rec["acc"].tobytes(), f"frame {f}: accumulated colour"
        assert got_spp.tobytes() == np.ascontiguousarray(rec["spp"]).astype(np.uint8).tobytes(), f"frame {f}: spp"
        top = max(top, int(got_spp.max()))
    assert top == 255, top
