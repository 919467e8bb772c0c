"""The MFMA compact-WY fitter experiment (tools/wy_fitter.hip, DESIGN.md
section 4; BASELINE config 5's "wider panel, MFMA path") as a GPU test: the
blocked Householder QR whose trailing-panel update runs on
v_mfma_f32_16x16x4_f32, at B = 13 and B = 16 and panel widths 4 and 16 (one
full-width panel), inside the f32-tmp_data stage pipeline, against the exact
VALU fitter of libbmfr on the same frames.  The WY form re-associates the
trailing update, so it is not bit-exact: the TAA output must stay within the
north star's 1e-4 relative L2 (bmfr.cl:606-655 is the update it replaces).
Not a product path: libbmfr ships only the exact fitter."""
from __future__ import annotations

import ctypes as C
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,nb", [(13, 4), (13, 16), (16, 4), (16, 16)])
def test_wy_mfma_fitter_within_tolerance(B, nb, gpu):
    import torch

    import bmfr_amd
    from bmfr_amd._lib import check
    from bmfr_amd.pipeline import _ptr
    import mfma_common as mc

    path = os.path.join(ROOT, "tools", "libwy.so")
    assert os.path.exists(path), "tools/libwy.so is built by __graft_entry__.build()"
    wy = mc.load_wy(path)
    W, H = 256, 144
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, use_half_precision_in_tmp_data=0, library_powr=1,
                              scaled=bmfr_amd.SCALED_THIRD_ORDER if B == 16 else bmfr_amd.SCALED_DEFAULT)
    assert cfg.buffer_count == B
    exact, blocked = bmfr_amd.StagePipeline(cfg), bmfr_amd.StagePipeline(cfg)

    def valu(sp, f):
        check(sp.lib.bmfr_fitter(sp.handle, torch.cuda.current_stream().cuda_stream, _ptr(sp.weights),
                                 _ptr(sp.mins_maxs), _ptr(sp.tmp_data), f), "fitter")

    def mfma(sp, f):
        err = wy.wy_fitter(sp.sizes.blocks, _ptr(sp.tmp_data), _ptr(sp.weights), _ptr(sp.mins_maxs), f,
                           cfg.noise_amount * 2.0, torch.cuda.current_stream().cuda_stream, B, nb)
        assert err == 0, err

    worst = 0.0
    for f in range(4):
        fr = bmfr_amd.synth_frame_device(W, H, f)
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        for sp, fit in ((exact, valu), (blocked, mfma)):
            sp.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
            mc.run_stages(sp, vp, jit, f, fit)
        torch.cuda.synchronize()
        a, b = blocked.cur(blocked.result).double(), exact.cur(exact.result).double()
        assert torch.isfinite(a).all()
        worst = max(worst, float(torch.linalg.norm(a - b) / torch.linalg.norm(b)))
        exact.swap()
        blocked.swap()
    print(f"B={B} nb={nb}: worst TAA-output rel-L2 vs the exact fitter {worst:.3g}")
    assert 0.0 < worst <= 1e-4  # re-associated (not bit-exact), within the north star's tolerance
