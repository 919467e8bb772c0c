"""Half-precision input planes (bmfr_config.input_half, BASELINE config 5's
"fp16 feature buffers").

The kernels widen each half value to f32 exactly on load, so denoising the
half planes must give, bit for bit, what the f32 path gives on the same
planes widened to f32 -- every frame, output and temporal state.  The f32
path itself is pinned to the reference kernels by test_gpu_parity.py."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import bmfr_amd

pytestmark = pytest.mark.gpu

FRAMES = 6
PLANES = ("noisy", "normals", "positions", "albedo")


def _bits(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("fast_fit", [0, 1])
@pytest.mark.parametrize("W,H,scaled,half_tmp", [
    (160, 96, bmfr_amd.SCALED_DEFAULT, 1),       # column-split K1, B = 13
    (160, 96, bmfr_amd.SCALED_THIRD_ORDER, 1),   # column-split K1, B = 16 (config 5's feature set)
    (128, 80, bmfr_amd.SCALED_DEFAULT, 0),       # row-split K1 (f32 tmp_data)
    (100, 72, bmfr_amd.SCALED_THIRD_ORDER, 0),
])
def test_half_inputs_match_widened_f32(W, H, scaled, half_tmp, fast_fit, gpu):
    """(fast_fit too: the fused update changes the fit's arithmetic, not how
    the inputs are read, so half planes == widened planes bit for bit there
    as well -- config 5's timed configuration.)"""
    base = dict(image_width=W, image_height=H, scaled=scaled, use_half_precision_in_tmp_data=half_tmp,
                fast_fit=fast_fit)
    den_h = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(**base, input_half=1))
    den_f = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(**base))
    n = W * H * 3
    for f in range(FRAMES):
        fr = bmfr_amd.synth_frame_device(W, H, f)
        h = {k: fr[k].half() for k in PLANES}
        w = {k: h[k].float() for k in PLANES}
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        den_h.process_frame(h["noisy"], h["normals"], h["positions"], h["albedo"], vp, jit, f)
        den_f.process_frame(w["noisy"], w["normals"], w["positions"], w["albedo"], vp, jit, f)
        out_h = den_h.copy_output(torch.empty(n, device="cuda"))
        out_f = den_f.copy_output(torch.empty(n, device="cuda"))
        assert np.array_equal(_bits(out_h), _bits(out_f)), f"frame {f}: output differs"
        for name in ("noisy_accumulated", "filtered_accumulated"):
            a = den_h.copy_state(name, torch.empty(n, device="cuda"))
            b = den_f.copy_state(name, torch.empty(n, device="cuda"))
            assert np.array_equal(_bits(a), _bits(b)), f"frame {f}: {name} differs"
    # The half path really read half planes: the widened-f32 result differs
    # from the result on the original f32 planes.
    den_o = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(**base))
    fr = bmfr_amd.synth_frame_device(W, H, 0)
    vp, jit = bmfr_amd.synth_camera(W, H, 0)
    den_o.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, 0)
    assert not np.array_equal(_bits(den_o.copy_output(torch.empty(n, device="cuda"))), _bits(out_h))


def test_half_inputs_rejected_where_unsupported(gpu):
    # generic feature lists run the generic K1, which reads f32 planes only
    cfg = bmfr_amd.BmfrConfig(image_width=64, image_height=64, scaled=(bmfr_amd.SCALED_DEFAULT[0],), input_half=1)
    den = bmfr_amd.Denoiser(cfg)
    fr = bmfr_amd.synth_frame_device(64, 64, 0)
    h = {k: fr[k].half() for k in PLANES}
    vp, jit = bmfr_amd.synth_camera(64, 64, 0)
    with pytest.raises(bmfr_amd.BmfrError) as e:
        den.process_frame(h["noisy"], h["normals"], h["positions"], h["albedo"], vp, jit, 0)
    assert "unsupported" in str(e.value)
