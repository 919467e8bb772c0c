"""libbmfr's native halo exchange (bmfr_exchange_*, include/bmfr.h): the
plan, pack, messages and unpack of one frame behind one C call.

On one GPU the grid's ranks run in one process and the messages move as
device copies (bmfr_exchange_run_all without communicators) -- the same
plans and buffers the RCCL path sends from, checked bit for bit against the
untiled frame with the halo ring poisoned until the exchange.  RCCL itself
(bmfr_comm_*) is exercised as far as one GPU allows: communicators of one
rank, made both ways, and an exchange through them."""
from __future__ import annotations

import pytest
import torch

import bmfr_amd
from bmfr_amd.tiling import HipCopier, NativeExchange, TileGrid, halo_bytes, halo_rects, packed_bytes, state_planes

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(320, 256, 2, 2, 40), (480, 288, 4, 2, 38), (352, 224, 1, 2, 48)])
@pytest.mark.parametrize("fast_fit", [0, 1])
def test_native_exchange_matches_untiled(shape, fast_fit, gpu):
    W, H, tx, ty, halo = shape
    grid = TileGrid(W, H, tx, ty, halo=halo)
    full = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, fast_fit=fast_fit))
    tiles = [bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r),
                                                   tile_halo=halo, fast_fit=fast_fit)) for r in range(grid.ranks)]
    xs = [NativeExchange(d, grid, r, None) for r, d in enumerate(tiles)]
    copier = HipCopier()
    prev = [None] * grid.ranks
    for f in range(8):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        fr = bmfr_amd.synth_frame_device(W, H, f)
        full.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        inps = [bmfr_amd.synth_region_device(W, H, d.region, f) for d in tiles]
        kws = [dict(prev_normals=p["normals"], prev_positions=p["positions"]) if p else {} for p in prev]
        args = [(i["noisy"], i["normals"], i["positions"], i["albedo"], vp, jit, f) for i in inps]
        if f > 0:  # poison the halo ring: only the exchange may fill what the frame reads
            for r, d in enumerate(tiles):
                for p in state_planes(d):
                    for h in halo_rects(d.region, grid.tile(r)):
                        copier.fill2d(p.rect_ptr(h), p.pitch, 0xFF, h[2] * p.bpp, h[3])
            for r in range(grid.ranks):
                tiles[r].process_frame_interior(*args[r], **kws[r])
            NativeExchange.run_all(xs, f)
            for r in range(grid.ranks):
                tiles[r].process_frame_border(*args[r], **kws[r])
        else:
            for r in range(grid.ranks):
                tiles[r].process_frame(*args[r], **kws[r])
        prev = inps
        torch.cuda.synchronize()
        want = full.copy_output(torch.empty(3 * W * H, device="cuda")).view(H, W, 3)
        for r, d in enumerate(tiles):
            assert d.halo_status() == 0
            rx, ry, rw, rh = d.region
            x, y, w, h = grid.tile(r)
            got = d.copy_output(torch.empty(3 * rw * rh, device="cuda")).view(rh, rw, 3)
            a = got[y - ry:y - ry + h, x - rx:x - rx + w].contiguous().view(torch.int32)
            b = want[y:y + h, x:x + w].contiguous().view(torch.int32)
            assert torch.equal(a, b), (shape, f, r, int((a != b).sum()))
        if f > 0:
            sent = sum(x.bytes(f)[0] for x in xs)
            recv = sum(x.bytes(f)[1] for x in xs)
            assert sent == recv > 0
            for r, x in enumerate(xs):  # the host mirror of the packed layout (tests/test_tiling.py)
                plan = grid.frame_plan(r, f)
                assert x.bytes(f) == (sum(packed_bytes(s) for _, s, _ in plan),
                                      sum(packed_bytes(q) for _, _, q in plan))
                for _, s, q in plan:
                    for recs in (s, q):
                        if recs:
                            assert halo_bytes(tiles[r], recs) == packed_bytes(recs)


def _multi_gpu_run(W, H, tx, ty, halo, frames, fast_fit):
    """Each tile of a tx x ty grid on its own GPU (devices 0..n-1 of this
    process), the halo exchange through RCCL communicators made by
    bmfr_comm_create_all (every rank's ncclSend / ncclRecv in one group),
    compared with the untiled frame on device 0."""
    import ctypes as C

    from bmfr_amd import _lib
    lib = _lib.load()
    grid = TileGrid(W, H, tx, ty, halo=halo)
    n = grid.ranks
    devs = (C.c_int * n)(*range(n))
    comms = (C.c_void_p * n)()
    assert lib.bmfr_comm_create_all(n, devs, comms) == 0
    full = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, fast_fit=fast_fit), device=0)
    tiles = [bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(r), tile_halo=halo,
                                                   fast_fit=fast_fit), device=r) for r in range(n)]

    class _C:
        def __init__(self, h):
            self.handle = h

    xs = [NativeExchange(d, grid, r, _C(comms[r])) for r, d in enumerate(tiles)]
    streams = [torch.cuda.Stream(device=r) for r in range(n)]
    prev = [None] * n
    for f in range(frames):
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        fr = bmfr_amd.synth_frame_device(W, H, f)
        full.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        inps = []
        for r, d in enumerate(tiles):
            with torch.cuda.device(r):
                inps.append(bmfr_amd.synth_region_device(W, H, d.region, f, device=r, stream=streams[r]))
        if f > 0:
            NativeExchange.run_all(xs, f, streams)
        for r, d in enumerate(tiles):
            kw = dict(prev_normals=prev[r]["normals"], prev_positions=prev[r]["positions"]) if prev[r] else {}
            i = inps[r]
            with torch.cuda.device(r):
                d.process_frame(i["noisy"], i["normals"], i["positions"], i["albedo"], vp, jit, f, stream=streams[r],
                                **kw)
        prev = inps
        for r in range(n):
            torch.cuda.synchronize(r)
        want = full.copy_output(torch.empty(3 * W * H, device="cuda:0")).view(H, W, 3)
        for r, d in enumerate(tiles):
            assert d.halo_status() == 0
            rx, ry, rw, rh = d.region
            x, y, w, h = grid.tile(r)
            with torch.cuda.device(r):
                got = d.copy_output(torch.empty(3 * rw * rh, device=f"cuda:{r}"), stream=streams[r]).view(rh, rw, 3)
                torch.cuda.synchronize(r)
            a = got[y - ry:y - ry + h, x - rx:x - rx + w].contiguous().cpu().view(torch.int32)
            b = want[y:y + h, x:x + w].contiguous().cpu().view(torch.int32)
            assert torch.equal(a, b), (f, r, int((a != b).sum()))
    for x in xs:
        x.close()
    for r in range(n):
        assert lib.bmfr_comm_destroy(comms[r]) == 0


@pytest.mark.multi_gpu
@pytest.mark.timeout(240, method="thread")  # a stuck RCCL call ends the run instead of hanging it
@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL between ranks needs two GPUs")
@pytest.mark.parametrize("fast_fit", [0, 1])
def test_rccl_two_gpus_matches_untiled(fast_fit, gpu):
    """The RCCL branch of bmfr_exchange_run_all (pack, one grouped ncclSend /
    ncclRecv batch over the grid's communicators, unpack) on a 2 x 1 grid of
    two GPUs == the untiled frame bit for bit (skipped on one-GPU boxes)."""
    _multi_gpu_run(320, 256, 2, 1, 40, 6, fast_fit)


def test_rccl_single_rank_communicators(gpu):
    """RCCL loads, a one-rank communicator is made both ways
    (bmfr_comm_unique_id + bmfr_comm_create, bmfr_comm_create_all), and an
    exchange through it on a 1x1 grid (no neighbours: an empty group) runs."""
    import ctypes as C

    from bmfr_amd import _lib
    lib = _lib.load()
    uid = (C.c_char * 128)()
    assert lib.bmfr_comm_unique_id(uid) == 0
    comm = C.c_void_p()
    assert lib.bmfr_comm_create(uid, 1, 0, 0, C.byref(comm)) == 0
    devs = (C.c_int * 1)(0)
    comms = (C.c_void_p * 1)()
    assert lib.bmfr_comm_create_all(1, devs, comms) == 0
    W, H = 256, 128
    grid = TileGrid(W, H, 1, 1, halo=40)
    d = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(0), tile_halo=40))

    class _C:
        handle = comm

    x = NativeExchange(d, grid, 0, _C())
    for f in range(3):
        inp = bmfr_amd.synth_region_device(W, H, d.region, f)
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        if f > 0:
            x.run(f)
        d.process_frame(inp["noisy"], inp["normals"], inp["positions"], inp["albedo"], vp, jit, f)
    torch.cuda.synchronize()
    assert x.bytes(1) == (0, 0)
    x.close()
    assert lib.bmfr_comm_destroy(comm) == 0
    assert lib.bmfr_comm_destroy(comms[0]) == 0
