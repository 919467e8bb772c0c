"""Tiled contexts detect reprojection past the exchanged halo instead of
diverging silently (include/bmfr.h tile_halo, bmfr_halo_status).

The reference reprojects to any pixel (bmfr.cl:343-356); a tile holds the
previous frame's state only for its region (tile + halo), and only for its
tile before the halo exchange.  A camera that moves by more than the halo
allows must therefore surface as BMFR_ERROR_HALO_EXCEEDED, and motion inside
the allowance must stay bit-exact with the untiled frame."""
from __future__ import annotations

import pytest
import torch

import bmfr_amd
from bmfr_amd import _lib
from bmfr_amd.tiling import LoopbackTransport, TileGrid

pytestmark = pytest.mark.gpu

W, H, HALO = 320, 256, 40


def shifted(vp, dx: float, width: int):
    """The column-major VP with clip x += (2 dx / width) w: every reprojection
    lands dx pixels further right (bmfr.cl:343-355)."""
    k = 2.0 * dx / width
    m = list(vp)
    for c in range(4):  # row 0 += k * row 3
        m[4 * c] += k * m[4 * c + 3]
    return m


def run(dx: float, frames: int = 3, split: bool = True):
    grid = TileGrid(W, H, 2, 2, halo=HALO)
    full = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    tiles = [bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r),
                                                   tile_halo=HALO)) for r in range(grid.ranks)]
    loop = LoopbackTransport(grid)
    prev = [None] * grid.ranks
    status = []
    for f in range(frames):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        vp = shifted(vp, dx, W) if f > 0 else vp
        fr = bmfr_amd.synth_frame_device(W, H, f)
        full.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        inps = [bmfr_amd.synth_region_device(W, H, d.region, f) for d in tiles]
        kws = [dict(prev_normals=p["normals"], prev_positions=p["positions"]) if p else {} for p in prev]
        args = [(i["noisy"], i["normals"], i["positions"], i["albedo"], vp, jit, f) for i in inps]
        if split and f > 0:
            for r in range(grid.ranks):
                tiles[r].process_frame_interior(*args[r], **kws[r])
            loop.exchange_all_ctx(tiles, f)
            for r in range(grid.ranks):
                tiles[r].process_frame_border(*args[r], **kws[r])
        else:
            if f > 0:
                loop.exchange_all_ctx(tiles, f)
            for r in range(grid.ranks):
                tiles[r].process_frame(*args[r], **kws[r])
        prev = inps
        st = []
        for d in tiles:
            try:
                st.append(d.halo_status())
            except _lib.BmfrError as e:
                assert e.status == _lib.HALO_EXCEEDED, e
                st.append(-1)
        status.append(st)
    return grid, full, tiles, status, (prev, vp, jit)


def test_motion_inside_halo_is_exact(gpu):
    grid, full, tiles, status, _ = run(dx=5.0)
    assert all(s == 0 for st in status for s in st), status
    n = W * H
    want = full.copy_output(torch.empty(3 * n, device="cuda")).view(H, W, 3)
    for r, d in enumerate(tiles):
        rx, ry, rw, rh = d.region
        x, y, w, h = grid.tile(r)
        got = d.copy_output(torch.empty(3 * rw * rh, device="cuda")).view(rh, rw, 3)
        assert torch.equal(got[y - ry:y - ry + h, x - rx:x - rx + w].view(torch.int32),
                           want[y:y + h, x:x + w].view(torch.int32)), r


@pytest.mark.parametrize("dx", [40.0, -40.0])
@pytest.mark.parametrize("split", [True, False])
def test_motion_past_halo_is_reported(dx, split, gpu):
    """40 px of motion with a 40 px halo: the tiles whose neighbour lies in
    the direction of motion read past their state and report it; the others
    read only valid state (or off-image taps) and stay bit-exact."""
    grid, full, tiles, status, (prev, vp, jit) = run(dx=dx, frames=2, split=split)
    assert all(s == 0 for s in status[0]), status  # frame 0 reprojects nothing
    flagged = [r for r in range(grid.ranks) if (r % 2 == 0) == (dx > 0)]
    assert [r for r, s in enumerate(status[1]) if s == -1] == flagged, status
    n = W * H
    want = full.copy_output(torch.empty(3 * n, device="cuda")).view(H, W, 3)
    for r, d in enumerate(tiles):
        if r in flagged:
            continue
        rx, ry, rw, rh = d.region
        x, y, w, h = grid.tile(r)
        got = d.copy_output(torch.empty(3 * rw * rh, device="cuda")).view(rh, rw, 3)
        assert torch.equal(got[y - ry:y - ry + h, x - rx:x - rx + w].view(torch.int32),
                           want[y:y + h, x:x + w].view(torch.int32)), r
    # sticky: the next frame is refused until frame 0 restarts the sequence
    r = flagged[0]
    inp = bmfr_amd.synth_region_device(W, H, tiles[r].region, 2)
    with pytest.raises(_lib.BmfrError) as e:
        tiles[r].process_frame(inp["noisy"], inp["normals"], inp["positions"], inp["albedo"], vp, jit, 2,
                               prev_normals=prev[r]["normals"], prev_positions=prev[r]["positions"])
    assert e.value.status == _lib.HALO_EXCEEDED
    inp0 = bmfr_amd.synth_region_device(W, H, tiles[r].region, 0)
    tiles[r].process_frame(inp0["noisy"], inp0["normals"], inp0["positions"], inp0["albedo"], vp, jit, 0)
    assert tiles[r].halo_status() == 0


def test_untiled_never_reports(gpu):
    den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    for f in range(2):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        fr = bmfr_amd.synth_frame_device(W, H, f)
        den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], shifted(vp, 200.0, W), jit, f)
    assert den.halo_status() == 0
