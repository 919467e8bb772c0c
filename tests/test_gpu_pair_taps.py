"""Half input planes load a reprojection tap row's two pixels in one 12-byte
load (bmfr_kernels.h noisy_taps_issue, kPairTaps).  A pair that would start
before the plane (taps at x = -1 on the first row) or end past it (taps at
x = W - 1 on the last row) is read one pixel over and its in-image tap taken
from the other half; pairs at a row's ends read into the neighbouring row.

Here every pixel of a frame is reprojected to one chosen point: the previous
camera matrix maps every world position to the same clip-space point
(u = M[12], v = M[13], w = M[15] = 1; bmfr.cl:343-356), so all taps of the
frame sit at that point.  Points at the plane's last pixel, its first pixel,
and the right / left ends of an inner row, one per frame, each on the
bit-exact path with half inputs against the reference kernels (strict build,
inputs widened) -- every buffer of the state and the output bit for bit; the
same input planes every frame, so each corner pixel accepts the tap at its
own position, the one the fix-up supplies.  (A build without the fix-up,
-DBMFR_PROBE_NO_PAIR_FIX, fails here at frame 1: 251 of 30,720 output values
differ.)
"""
from __future__ import annotations

import dataclasses

import pytest
import torch

import bmfr_amd
import ref_run
from ref_configs import REF_CONFIGS
from test_gpu_reference_fullsize import assert_same, hip_cfg

pytestmark = pytest.mark.gpu


def constant_camera(W: int, H: int, px: float, py: float):
    """(prev_vp, jitter) reprojecting every pixel to (px, py): pfx = u W - jx,
    pfy = v H - (1 - jy) with u = (cx + 1) / 2, v = (cy + 1) / 2, jitter (0, 1)."""
    cx = 2.0 * px / W - 1.0
    cy = 2.0 * py / H - 1.0
    m = [0.0] * 16
    m[12], m[13], m[15] = cx, cy, 1.0
    return m, [0.0, 1.0]


def test_pair_taps_at_plane_ends_match_reference(gpu):
    rc = dataclasses.replace(REF_CONFIGS["s128x80_h13"], frames=6)
    if not ref_run.available(rc.name, "strict"):
        pytest.skip("reference build missing")
    W, H = rc.width, rc.height
    # frame 0: no reprojection; then the last pixel (hi fix), the first pixel
    # (lo fix), the right end of row 40 (pair into row 41), the left end of
    # row 40 (pair from row 39), and the last pixel again
    points = [None, (W - 0.7, H - 0.7), (-0.7, -0.7), (W - 0.7, 40.3), (-0.7, 40.3), (W - 0.2, H - 0.2)]
    ref = ref_run.RefLoop(rc, "strict")
    den = bmfr_amd.Denoiser(hip_cfg(rc, 1))
    n = W * H
    # the same planes every frame: a pixel's own previous position and
    # normal then match at its own tap, so the corner pixels accept the tap
    # the fix-up supplies (spp grows there)
    fr = bmfr_amd.synth_frame_device(W, H, 0, seed=rc.seed)
    for f, pt in enumerate(points):
        half = {k: fr[k].half() for k in ("noisy", "normals", "positions", "albedo")}
        wide = {k: v.float() for k, v in half.items()}
        if pt is None:
            vp, jit = bmfr_amd.synth_camera(W, H, 0)
        else:
            vp, jit = constant_camera(W, H, *pt)
        rec = {}
        ref.upload(wide["noisy"], wide["normals"], wide["positions"], wide["albedo"])
        ref.run_stages(vp, jit, f, record=rec)
        ref.swap()
        den.process_frame(half["noisy"], half["normals"], half["positions"], half["albedo"], vp, jit, f)
        got = {
            "result": den.copy_output(torch.empty(3 * n, device="cuda")),
            "acc": den.copy_state("filtered_accumulated", torch.empty(3 * n, device="cuda")),
            "noisy": den.copy_state("noisy_accumulated", torch.empty(3 * n, device="cuda")),
            "spp": den.copy_state("spp", torch.empty(n, dtype=torch.uint8, device="cuda")),
            "prev_pixel": den.copy_state("prev_frame_pixel", torch.empty(2 * n, device="cuda")),
        }
        for k, v in got.items():
            assert_same(v, rec[k], f"frame {f} (taps at {pt}) {k}")
        if pt is not None:
            # the reprojection really put every pixel at the chosen point
            pp = rec["prev_pixel"].view(-1, 2)
            assert float(pp[:, 0].min()) == float(pp[:, 0].max()) and abs(float(pp[0, 0]) - pt[0]) < 1e-3
            # the corner pixel accepts its own tap -- the pair's fixed-up half
            corner = {1: n - 1, 2: 0, 5: n - 1}.get(f)
            if corner is not None:
                assert int(rec["spp"][corner]) >= 2, (f, int(rec["spp"][corner]))
