"""Tiled contexts reproduce the untiled frame bit for bit.

All tiles of a grid run in one process on one GPU, each its own tiled
libbmfr context over its region, with the halo exchange done by the
loopback transport (the same plan the RCCL transport sends).  Every frame,
each tile's output and temporal state must equal the same pixels of the
untiled run."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import bmfr_amd
from bmfr_amd.tiling import HipCopier, LoopbackTransport, TileGrid, halo_rects, state_planes

pytestmark = pytest.mark.gpu

FRAMES = 8


def _tile_of(a: np.ndarray, region, tile, ch):
    rx, ry, rw, rh = region
    x, y, w, h = tile
    a = a.reshape(rh, rw, ch)
    return a[y - ry:y - ry + h, x - rx:x - rx + w]


@pytest.mark.parametrize("shape", [(320, 256, 2, 2, 40), (352, 224, 2, 1, 48), (256, 320, 1, 2, 40),
                                   (480, 288, 4, 2, 38)])
@pytest.mark.parametrize("half,split,kernel_copy", [(1, False, False), (0, False, False), (1, True, False),
                                                    (1, True, True)])
def test_tiled_matches_untiled_bitwise(shape, half, split, kernel_copy, gpu):
    """split: each frame as bmfr_process_frame_interior, halo exchange,
    bmfr_process_frame_border -- with the halo ring poisoned (all-ones bytes:
    NaN colours, spp 255) until the exchange, so an interior block that read
    the halo would break the bitwise match."""
    W, H, tx, ty, halo = shape
    grid = TileGrid(W, H, tx, ty, halo=halo)
    full = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H,
                                                 use_half_precision_in_tmp_data=half))
    tiles = [bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r),
                                                   tile_halo=halo, use_half_precision_in_tmp_data=half))
             for r in range(grid.ranks)]
    for r, d in enumerate(tiles):
        assert d.region == grid.region(r)
    loop = LoopbackTransport(grid)
    copier = HipCopier()
    prev = [None] * grid.ranks
    for f in range(FRAMES):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        fr = bmfr_amd.synth_frame_device(W, H, f)
        full.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        inps = [bmfr_amd.synth_region_device(W, H, d.region, f) for d in tiles]

        def call(method, r):
            inp = inps[r]
            getattr(tiles[r], method)(inp["noisy"], inp["normals"], inp["positions"], inp["albedo"], vp, jit, f,
                                      prev_normals=prev[r]["normals"] if prev[r] else None,
                                      prev_positions=prev[r]["positions"] if prev[r] else None)

        if split:
            if f > 0:
                for r, d in enumerate(tiles):
                    for p in state_planes(d):
                        for h in halo_rects(d.region, grid.tile(r)):
                            copier.fill2d(p.rect_ptr(h), p.pitch, 0xFF, h[2] * p.bpp, h[3])
            for r in range(grid.ranks):
                call("process_frame_interior", r)
            if f > 0:
                if kernel_copy:  # libbmfr's one-launch pack / unpack (bmfr_halo_copy)
                    loop.exchange_all_ctx(tiles, f)
                else:
                    loop.exchange_all([state_planes(d) for d in tiles], copier)
            for r in range(grid.ranks):
                call("process_frame_border", r)
        else:
            if f > 0:
                loop.exchange_all([state_planes(d) for d in tiles], copier)
            for r in range(grid.ranks):
                call("process_frame", r)
        prev = inps
        torch.cuda.synchronize()
        n = W * H
        want = {
            "result": full.copy_output(torch.empty(3 * n, device="cuda")).cpu().numpy(),
            "noisy_accumulated": full.copy_state("noisy_accumulated", torch.empty(3 * n, device="cuda")).cpu().numpy(),
            "filtered_accumulated": full.copy_state("filtered_accumulated",
                                                    torch.empty(3 * n, device="cuda")).cpu().numpy(),
            "spp": full.copy_state("spp", torch.empty(n, dtype=torch.uint8, device="cuda")).cpu().numpy(),
        }
        for r, d in enumerate(tiles):
            reg, tile = d.region, grid.tile(r)
            m = reg[2] * reg[3]
            got = {
                "result": d.copy_output(torch.empty(3 * m, device="cuda")).cpu().numpy(),
                "noisy_accumulated": d.copy_state("noisy_accumulated", torch.empty(3 * m, device="cuda")).cpu().numpy(),
                "filtered_accumulated": d.copy_state("filtered_accumulated",
                                                     torch.empty(3 * m, device="cuda")).cpu().numpy(),
                "spp": d.copy_state("spp", torch.empty(m, dtype=torch.uint8, device="cuda")).cpu().numpy(),
            }
            for k, v in got.items():
                ch = 1 if k == "spp" else 3
                a = _tile_of(v, reg, tile, ch)
                b = _tile_of(want[k], (0, 0, W, H), tile, ch)
                bad = np.argwhere(a != b)
                assert bad.size == 0, (shape, half, f, r, k, len(bad), bad[:3].tolist())


@pytest.mark.parametrize("gx,gy", [(4, 2), (2, 4)], ids=["4x2", "2x4"])
def test_8k_tiled_matches_untiled(gx, gy, gpu):
    """BASELINE config 4 at its own size: 7680x4320 as bench.py's 4x2 grid
    and as the 2x4 grid BASELINE.json names (3840x1080 tiles), halo 64,
    every frame split into bmfr_process_frame_interior, the bmfr_halo_copy
    exchange and bmfr_process_frame_border, == the untiled 8K frame bit for
    bit (output and exchanged state), 3 frames.  The untiled 8K frame is
    itself pinned to the reference kernels (test_gpu_reference_fullsize.py,
    f7680x4320_h13)."""
    W, H, halo = 7680, 4320, 64
    grid = TileGrid(W, H, gx, gy, halo=halo)
    full = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    tiles = [bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r),
                                                   tile_halo=halo)) for r in range(grid.ranks)]
    loop = LoopbackTransport(grid)
    prev = [None] * grid.ranks
    n = W * H
    for f in range(3):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        fr = bmfr_amd.synth_frame_device(W, H, f)
        full.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        del fr
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
        want = {"result": full.copy_output(torch.empty(3 * n, device="cuda")).view(H, W, 3),
                "filtered_accumulated": full.copy_state("filtered_accumulated",
                                                        torch.empty(3 * n, device="cuda")).view(H, W, 3),
                "noisy_accumulated": full.copy_state("noisy_accumulated", torch.empty(3 * n, device="cuda")).view(H, W, 3)}
        for r, d in enumerate(tiles):
            assert d.halo_status() == 0
            rx, ry, rw, rh = d.region
            x, y, w, h = grid.tile(r)
            for k, v in want.items():
                t = torch.empty(3 * rw * rh, device="cuda")
                got = (d.copy_output(t) if k == "result" else d.copy_state(k, t)).view(rh, rw, 3)
                a = got[y - ry:y - ry + h, x - rx:x - rx + w].contiguous().view(torch.int32)
                b = v[y:y + h, x:x + w].contiguous().view(torch.int32)
                assert torch.equal(a, b), (f, r, k, int((a != b).sum()))
        del want


def test_halo_copy_plane_masks(gpu):
    """bmfr_halo_copy records {x, y, w, h, planes}: each mask packs exactly
    its planes (segment sizes padded to 16 bytes), a pack / unpack round trip
    through another context moves only those planes, and masks outside
    1..15 are rejected."""
    import ctypes as C

    from bmfr_amd import tiling
    W, H = 320, 256
    grid = TileGrid(W, H, 2, 2, halo=40)
    a, b = (bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r), tile_halo=40))
            for r in (0, 1))
    # rectangle of tile 0 inside region 1
    rect = tiling.intersect(grid.tile(0), grid.region(1))
    assert rect is not None
    n = rect[2] * rect[3]
    pad = lambda x: (x + 15) // 16 * 16  # noqa: E731
    sizes = {1: 12 * n, 2: n, 4: 12 * n, 8: 12 * n}
    for mask in range(1, 16):
        want = sum(pad(v) for k, v in sizes.items() if mask & k)
        assert tiling.halo_bytes(a, [(*rect, mask)]) == want
    for bad in (0, 16, -1):
        with pytest.raises(bmfr_amd.BmfrError):
            tiling.halo_bytes(a, [(*rect, bad)])
    # one frame so both contexts hold state; then move only the spp and result planes
    for d in (a, b):
        inp = bmfr_amd.synth_region_device(W, H, d.region, 0)
        vp, jit = bmfr_amd.synth_camera(W, H, 0)
        d.process_frame(inp["noisy"], inp["normals"], inp["positions"], inp["albedo"], vp, jit, 0)
    torch.cuda.synchronize()

    def planes(d):
        m = d.region[2] * d.region[3]
        return {k: (d.copy_output(torch.empty(3 * m, device="cuda")) if k == "result" else
                    d.copy_state(k, torch.empty(m if k == "spp" else 3 * m,
                                                dtype=torch.uint8 if k == "spp" else torch.float32, device="cuda")))
                .cpu().numpy().copy() for k in ("noisy_accumulated", "spp", "filtered_accumulated", "result")}

    before_a, before_b = planes(a), planes(b)
    recs = [(*rect, 2 | 8)]
    buf = torch.empty(tiling.halo_bytes(a, recs), dtype=torch.uint8, device="cuda")
    tiling.halo_copy(a, recs, buf.data_ptr(), unpack=False)
    tiling.halo_copy(b, recs, buf.data_ptr(), unpack=True)
    torch.cuda.synchronize()
    after_b = planes(b)
    ra, rb = a.region, b.region
    x, y, w, h = rect
    for k in before_b:
        ch = 1 if k == "spp" else 3
        va = before_a[k].reshape(ra[3], ra[2], ch)[y - ra[1]:y - ra[1] + h, x - ra[0]:x - ra[0] + w]
        vb0 = before_b[k].reshape(rb[3], rb[2], ch)
        vb1 = after_b[k].reshape(rb[3], rb[2], ch)
        inside = vb1[y - rb[1]:y - rb[1] + h, x - rb[0]:x - rb[0] + w]
        if k in ("spp", "result"):
            assert inside.tobytes() == va.tobytes(), k
        else:
            assert vb1.tobytes() == vb0.tobytes(), k  # untouched plane
        outside = vb1.copy()
        outside[y - rb[1]:y - rb[1] + h, x - rb[0]:x - rb[0] + w] = 0
        ref = vb0.copy()
        ref[y - rb[1]:y - rb[1] + h, x - rb[0]:x - rb[0] + w] = 0
        assert outside.tobytes() == ref.tobytes(), k
