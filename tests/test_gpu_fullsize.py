"""Full-size parity (BASELINE.json configs: 1920x1080, 3840x2160, 7680x4320).

The CPU oracle is too slow at these sizes, so the check is transitive: the
stage kernels are pinned bit for bit to the reference kernels at small sizes
(test_gpu_parity.py) and follow the reference's dataflow exactly; here the
fused production path must equal them bit for bit on every output and state
plane at the full sizes (3 frames, so the temporal path and two block-grid
offsets are exercised), plus the half-input and B = 16 configuration at 4K."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import bmfr_amd

pytestmark = pytest.mark.gpu

FRAMES = 3


@pytest.mark.parametrize("W,H,third", [(1920, 1080, False), (3840, 2160, False), (7680, 4320, False),
                                       (3840, 2160, True)])
def test_fused_equals_stages_full_size(W, H, third, gpu):
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H,
                              scaled=bmfr_amd.SCALED_THIRD_ORDER if third else bmfr_amd.SCALED_DEFAULT)
    st = bmfr_amd.StagePipeline(cfg)
    den = bmfr_amd.Denoiser(cfg)
    n = W * H
    for f in range(FRAMES):
        fr = bmfr_amd.synth_frame_device(W, H, f)
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        rec = {}
        st.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        st.run_stages(vp, jit, f, record=rec)
        st.swap()
        den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        got = {
            "result": den.copy_output(torch.empty(3 * n, device="cuda")),
            "acc": den.copy_state("filtered_accumulated", torch.empty(3 * n, device="cuda")),
            "noisy": den.copy_state("noisy_accumulated", torch.empty(3 * n, device="cuda")),
            "spp": den.copy_state("spp", torch.empty(n, dtype=torch.uint8, device="cuda")),
        }
        for k, v in got.items():
            a = v.cpu().numpy()
            b = rec[k].reshape(-1).cpu().numpy() if hasattr(rec[k], "cpu") else np.asarray(rec[k]).reshape(-1)
            b = b[:a.size]
            assert a.tobytes() == b.tobytes(), (W, H, third, f, k, int((a != b).sum()))
        del fr, rec
        torch.cuda.empty_cache()
