"""bmfr_process_sequence (include/bmfr.h): frames pipelined -- by default one
launch per frame with K1 of frame f and the TAA tiles of frame f-1
(k_fused_cols_taa), or (BMFR_SEQUENCE=streams, and configurations the
combined kernel does not cover) over two streams, K2 of frame f beside K1 of
frame f+1 -- must give every frame's output and the final temporal state bit
for bit as bmfr_process_frame does, frame by frame -- across chunk
boundaries and mixed with per-frame calls."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import bmfr_amd

pytestmark = pytest.mark.gpu

FRAMES = 9


def _bits(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint32)


def _frames(W, H, half):
    out = []
    for f in range(FRAMES):
        fr = bmfr_amd.synth_frame_device(W, H, f)
        if half:
            fr = {k: v.half() for k, v in fr.items()}
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        out.append((fr, (vp, jit)))
    return out


@pytest.mark.parametrize("streams", [False, True])
@pytest.mark.parametrize("W,H,kw", [
    (160, 96, {}),
    (136, 76, {}),  # partial TAA tiles at the right and bottom edges
    (128, 80, {"use_half_precision_in_tmp_data": 0}),
    (160, 96, {"scaled": bmfr_amd.SCALED_THIRD_ORDER, "input_half": 1}),
    (96, 64, {"scaled": bmfr_amd.SCALED_THIRD_ORDER[:3] + bmfr_amd.SCALED_THIRD_ORDER[6:]}),  # generic K1: serial
])
def test_sequence_matches_per_frame(W, H, kw, streams, gpu, monkeypatch):
    if streams:
        monkeypatch.setenv("BMFR_SEQUENCE", "streams")
    else:
        monkeypatch.delenv("BMFR_SEQUENCE", raising=False)
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, **kw)
    seq = _frames(W, H, kw.get("input_half", 0))
    n = W * H * 3
    ref = bmfr_amd.Denoiser(cfg)
    want = []
    for f, (fr, (vp, jit)) in enumerate(seq):
        ref.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        want.append(_bits(ref.copy_output(torch.empty(n, device="cuda"))))
    den = bmfr_amd.Denoiser(cfg)
    outs = [torch.full((n,), float("nan"), device="cuda") for _ in range(FRAMES)]
    # chunks [0, 4), then one per-frame call, then [5, 9)
    den.process_sequence([s[0] for s in seq[:4]], [s[1] for s in seq[:4]], 0, outputs=outs[:4])
    fr, (vp, jit) = seq[4]
    den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, 4)
    den.copy_output(outs[4])
    den.process_sequence([s[0] for s in seq[5:]], [s[1] for s in seq[5:]], 5, outputs=outs[5:])
    torch.cuda.synchronize()
    for f in range(FRAMES):
        assert np.array_equal(_bits(outs[f]), want[f]), f"frame {f}"
    assert np.array_equal(_bits(den.copy_output(torch.empty(n, device="cuda"))), want[-1])
    for name in ("noisy_accumulated", "filtered_accumulated"):
        a = den.copy_state(name, torch.empty(n, device="cuda"))
        b = ref.copy_state(name, torch.empty(n, device="cuda"))
        assert np.array_equal(_bits(a), _bits(b)), name
