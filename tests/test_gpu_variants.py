"""The A/B kernel variants selected by BMFR_FUSED_KERNEL (rows: row-split
K1; k1tone: tone map in K1 + LDS TAA; tonecols: column-split K1 with tone
map + register-only stencil TAA) compute the same frames bit for bit as the
default path, per frame and pipelined (bmfr_process_sequence)."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

import bmfr_amd

pytestmark = pytest.mark.gpu

W, H, FRAMES = 160, 96, 6


def _bits(t):
    return t.cpu().numpy().view(np.uint32)


def _run(variant, sequence, half_tmp):
    old = os.environ.pop("BMFR_FUSED_KERNEL", None)
    if variant:
        os.environ["BMFR_FUSED_KERNEL"] = variant
    try:
        den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H,
                                                    use_half_precision_in_tmp_data=half_tmp))
    finally:
        os.environ.pop("BMFR_FUSED_KERNEL", None)
        if old is not None:
            os.environ["BMFR_FUSED_KERNEL"] = old
    frames, cams = [], []
    for f in range(FRAMES):
        frames.append(bmfr_amd.synth_frame_device(W, H, f))
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        cams.append((vp, jit))
    n = W * H * 3
    outs = [torch.empty(n, device="cuda") for _ in range(FRAMES)]
    if sequence:
        den.process_sequence(frames, cams, 0, outputs=outs)
    else:
        for f, (fr, (vp, jit)) in enumerate(zip(frames, cams)):
            den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
            den.copy_output(outs[f])
    torch.cuda.synchronize()
    return [_bits(o) for o in outs]


@pytest.mark.parametrize("variant,sequence,half_tmp", [
    ("tonecols", False, 1), ("tonecols", True, 1), ("tonecols", False, 0),
    ("k1tone", False, 1), ("k1tone", True, 1), ("rows", False, 1), ("colstone", False, 1),
    ("colstone", True, 1)])
def test_variant_matches_default(variant, sequence, half_tmp, gpu):
    want = _run(None, False, half_tmp)
    got = _run(variant, sequence, half_tmp)
    for f in range(FRAMES):
        assert np.array_equal(got[f], want[f]), (variant, sequence, f)
