"""The fused kernels' bounded waits report instead of running on silently
(include/bmfr.h BMFR_ERROR_SYNC_TIMEOUT, bmfr_frame_status; the knobs are
include/bmfr_debug.h bmfr_debug_sync).

Two waits exist: a K1 wave waiting in LDS for the Householder pivot another
wave of its work-group publishes (bmfr_fused_cols.hip wait_flag), and, in
the one-launch frame (frames below 4096 K1 blocks, bmfr_sizes.frame_launches;
4K and up run K1 and K2 as two launches), a TAA tile waiting for the
completion flags of the K1 blocks under it (bmfr_taa_tile.h wait_k1_blocks)."""
from __future__ import annotations

import pytest
import torch

import bmfr_amd
from bmfr_amd import _lib

pytestmark = pytest.mark.gpu


def _frames(W, H, n):
    out = []
    for f in range(n):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        out.append((bmfr_amd.synth_frame_device(W, H, f), vp, jit))
    return out


def _run(den, frames, first=0):
    for i, (fr, vp, jit) in enumerate(frames):
        den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, first + i)


def _planes(den, W, H):
    n = W * H
    return {"result": den.copy_output(torch.empty(3 * n, device="cuda")),
            "filtered_accumulated": den.copy_state("filtered_accumulated", torch.empty(3 * n, device="cuda")),
            "noisy_accumulated": den.copy_state("noisy_accumulated", torch.empty(3 * n, device="cuda")),
            "spp": den.copy_state("spp", torch.empty(n, dtype=torch.uint8, device="cuda")),
            "prev_frame_pixel": den.copy_state("prev_frame_pixel", torch.empty(2 * n, device="cuda"))}


def test_default_bounds_report_ok(gpu):
    W, H = 3840, 2160
    den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    _run(den, _frames(W, H, 3))
    assert den.frame_status() == 0


@pytest.mark.parametrize("W,H,half_tmp", [(3840, 2160, 1), (2560, 1440, 1), (2560, 1440, 0)])
def test_exhausted_waits_report_sync_timeout(W, H, half_tmp, gpu):
    """max_polls = 0: a wait gives up at the first flag that is not ready yet.
    Thousands of K1 blocks wait for pivots (half tmp_data) and, in the
    one-launch frame (2560x1440: 3726 K1 blocks), the TAA tiles in K1's tail
    wait for blocks still running, so the frame must report; the report is
    sticky (the next frame's call returns it) until frame 0."""
    assert bmfr_amd.BmfrConfig(image_width=W, image_height=H).sizes().frame_launches == (2 if W == 3840 else 1)
    den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H,
                                                use_half_precision_in_tmp_data=half_tmp))
    frames = _frames(W, H, 3)
    den.debug_sync(max_polls=0)
    _run(den, frames[:2])
    # half tmp_data: K1's pivot waits (and the tiles' waits of a one-launch
    # frame); f32 (row-split K1, work-group barriers): the tiles' waits
    assert den.frame_status() == _lib.SYNC_TIMEOUT
    with pytest.raises(bmfr_amd.BmfrError) as e:
        _run(den, frames[2:3], first=2)
    assert e.value.status == _lib.SYNC_TIMEOUT
    den.debug_sync(max_polls=-1)  # default bounds; frame 0 starts over and clears the report
    _run(den, frames)
    assert den.frame_status() == 0


def test_sequence_api_reports_sync_timeout(gpu):
    W, H = 1920, 1080
    den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    frames = _frames(W, H, 4)
    den.debug_sync(max_polls=0)
    den.process_sequence([f for f, _, _ in frames], [(vp, jit) for _, vp, jit in frames], 0)
    assert den.frame_status() == _lib.SYNC_TIMEOUT
    den.debug_sync(max_polls=-1)
    den.process_sequence([f for f, _, _ in frames], [(vp, jit) for _, vp, jit in frames], 0)
    assert den.frame_status() == 0


@pytest.mark.parametrize("W,H,half_tmp", [(2560, 1440, 1), (1920, 1080, 1), (2560, 1440, 0)])
def test_delayed_k1_blocks_one_launch_exact(W, H, half_tmp, gpu):
    """One K1 block in 61 sleeps ~0.3 ms before it raises its completion
    flag, so the TAA tiles over it really wait on the flags: the one-launch
    frame must still equal the two-launch frame (profiling on: K1 and K2 as
    separate launches, no flags) bit for bit on the output and every state
    plane, and report no timeout."""
    frames = _frames(W, H, 4)
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, use_half_precision_in_tmp_data=half_tmp)
    one = bmfr_amd.Denoiser(cfg)
    one.debug_sync(k1_delay=40)
    two = bmfr_amd.Denoiser(cfg)
    two.set_profiling(True, capacity=16)
    for i, fr in enumerate(frames):
        _run(one, [fr], first=i)
        _run(two, [fr], first=i)
        a, b = _planes(one, W, H), _planes(two, W, H)
        for k in a:
            ia = a[k].view(torch.uint8) if a[k].dtype == torch.uint8 else a[k].view(torch.int32)
            ib = b[k].view(torch.uint8) if b[k].dtype == torch.uint8 else b[k].view(torch.int32)
            assert torch.equal(ia, ib), (W, H, i, k, int((ia != ib).sum()))
    assert one.frame_status() == 0
    assert len(two.profile()) == len(frames)


def test_delayed_k1_blocks_tiled_border_launch_exact(gpu):
    """Tiled contexts run a frame's border ring of K1 blocks and the tile's TAA
    in one launch (completion flags; the launch's last work-group forwards
    the reach report after every ring block): with one K1 block in 61
    delayed, every tile of a 4x2 grid still equals the untiled frame bit for
    bit, through the interior / exchange / border split, and reports
    neither a timeout nor a halo overshoot."""
    from bmfr_amd.tiling import LoopbackTransport, TileGrid
    W, H, halo = 960, 544, 40
    grid = TileGrid(W, H, 4, 2, halo=halo)
    full = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    tiles = [bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r), tile_halo=halo))
             for r in range(grid.ranks)]
    for d in tiles:
        d.debug_sync(k1_delay=40)
    loop = LoopbackTransport(grid)
    prev = [None] * grid.ranks
    for f in range(6):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        fr = bmfr_amd.synth_frame_device(W, H, f)
        full.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        inps = [bmfr_amd.synth_region_device(W, H, d.region, f) for d in tiles]
        kws = [dict(prev_normals=p["normals"], prev_positions=p["positions"]) if p else {} for p in prev]
        args = [(i["noisy"], i["normals"], i["positions"], i["albedo"], vp, jit, f) for i in inps]
        if f == 0:
            for r in range(grid.ranks):
                tiles[r].process_frame(*args[r], **kws[r])
        else:
            for r in range(grid.ranks):
                tiles[r].process_frame_interior(*args[r], **kws[r])
            loop.exchange_all_ctx(tiles, f)
            for r in range(grid.ranks):
                tiles[r].process_frame_border(*args[r], **kws[r])
        prev = inps
        want = full.copy_output(torch.empty(3 * W * H, device="cuda")).view(H, W, 3)
        for r, d in enumerate(tiles):
            assert d.frame_status() == 0
            rx, ry, rw, rh = d.region
            x, y, w, h = grid.tile(r)
            got = d.copy_output(torch.empty(3 * rw * rh, device="cuda")).view(rh, rw, 3)
            a = got[y - ry:y - ry + h, x - rx:x - rx + w].contiguous().view(torch.int32)
            b = want[y:y + h, x:x + w].contiguous().view(torch.int32)
            assert torch.equal(a, b), (f, r, int((a != b).sum()))


@pytest.mark.parametrize("W,H", [(1920, 1080), (3840, 2160)])
def test_frame_status_waits_for_the_last_frames_stream(W, H, gpu):
    """bmfr_frame_status records its event when called, on the stream of the
    last enqueued frame (no marker between frames): after it returns, that
    stream has drained -- here a side stream whose frames carry delayed K1
    blocks (one in 61 sleeps ~40 us x 40), one-launch (1080p) and two-launch
    (4K) frames alike -- and frame 0 of a new sequence waits the same way."""
    den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    frames = _frames(W, H, 3)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    den.debug_sync(k1_delay=40)
    with torch.cuda.stream(s):
        _run(den, frames)
    assert den.frame_status() == 0
    assert s.query(), "bmfr_frame_status returned before the last frame's stream drained"
    with torch.cuda.stream(s):
        _run(den, frames)  # frame 0 again: waits for the frames above, clears the reports
    assert den.frame_status() == 0
    assert s.query()
