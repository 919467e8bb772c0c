"""Multi-GPU sharding: tile geometry, the exchange plan, and
the halo exchange itself over torch.distributed with the gloo backend on CPU
(world sizes 2 and 4).  The GPU side -- tiled contexts reproducing the
untiled frame bit for bit -- is tests/test_gpu_tiled.py."""
from __future__ import annotations

import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bmfr_amd.tiling import (STATE_PLANES, DistTransport, HostCopier, Plane, TileGrid, grid_for, intersect,
                             rect_bytes)


@pytest.mark.parametrize("n,expect", [(1, (1, 1)), (2, (2, 1)), (4, (2, 2)), (8, (4, 2))])
def test_grid_for(n, expect):
    assert grid_for(n) == expect


@pytest.mark.parametrize("shape", [(3840, 2160, 2, 2), (7680, 4320, 4, 2), (250, 130, 2, 1), (1000, 700, 1, 4)])
def test_tiles_partition_and_plan_is_symmetric(shape):
    g = TileGrid(*shape, halo=40)
    cover = np.zeros((g.height, g.width), np.int32)
    for r in range(g.ranks):
        x, y, w, h = g.tile(r)
        cover[y:y + h, x:x + w] += 1
        rx, ry, rw, rh = g.region(r)
        assert rx <= x and ry <= y and rx + rw >= x + w and ry + rh >= y + h
        assert intersect(g.region(r), (0, 0, g.width, g.height)) == g.region(r)
    assert (cover == 1).all()
    for r in range(g.ranks):
        for peer, s, rcv in g.plan(r):
            back = {p: (s2, r2) for p, s2, r2 in g.plan(peer)}
            assert back[r][1] == s and back[r][0] == rcv
        # the region is covered by my tile and what I receive
        reg = np.zeros((g.height, g.width), bool)
        x, y, w, h = g.tile(r)
        reg[y:y + h, x:x + w] = True
        for _, _, rcv in g.plan(r):
            if rcv:
                reg[rcv[1]:rcv[1] + rcv[3], rcv[0]:rcv[0] + rcv[2]] = True
        rx, ry, rw, rh = g.region(r)
        assert reg[ry:ry + rh, rx:rx + rw].all()
        assert reg.sum() == rw * rh


OFFSETS = [(-14, -14), (4, -6), (-8, 14), (8, 0), (-10, -8), (2, 12), (12, -12), (-10, 0),
           (12, 14), (-8, -16), (6, 6), (-2, -2), (6, -14), (-16, 12), (14, -4), (-6, 4)]  # bmfr.cl:267-285


def _need_restated(g, rank, frame):
    """bmfr_halo_need restated: blocks of frame's shifted grid reaching the
    tile + 1 px, their mirrored pixels grown by halo - 33; the tile grown by
    the same; clipped to the region."""
    x, y, w, h = g.tile(rank)
    rx, ry, rw, rh = g.region(rank)
    reach = g.halo - 33
    out_s, out_r = [], []
    for t0, t1, size, off, r0, r1 in ((x, x + w, g.width, OFFSETS[frame % 16][0], rx, rx + rw),
                                      (y, y + h, g.height, OFFSETS[frame % 16][1], ry, ry + rh)):
        nb = (32 * ((size + 31) // 32) + 32) // 32
        lo, hi = size, -1
        for b in range(nb):
            p0 = 32 * b - 16 + off
            if p0 < min(size, t1 + 1) and p0 + 32 > max(0, t0 - 1):
                for p in range(p0, p0 + 32):
                    m = -p - 1 if p < 0 else (2 * size - p - 1 if p >= size else p)
                    lo, hi = min(lo, m), max(hi, m)
        out_s.append((max(lo - reach, r0), min(hi + 1 + reach, r1)))
        out_r.append((max(t0 - reach, r0), min(t1 + reach, r1)))
    rect = lambda a: (a[0][0], a[1][0], a[0][1] - a[0][0], a[1][1] - a[1][0])  # noqa: E731
    return rect(out_s), rect(out_r)


@pytest.mark.parametrize("shape", [(7680, 4320, 4, 2, 64), (7680, 4320, 2, 4, 64), (3840, 2160, 2, 2, 40), (480, 288, 4, 2, 38),
                                   (320, 256, 2, 2, 40), (1000, 700, 1, 4, 50)])
def test_frame_plan_sends_what_each_frame_reads(shape):
    """The per-frame exchange (bmfr_halo_need, TileGrid.frame_plan): the C ABI
    equals the restatement; the result rectangle lies inside the state one,
    which lies inside the region and covers the tile + 1 px; every rank
    receives exactly the parts of its need rectangles outside its tile, each
    from the peer that owns them; the plan is symmetric; and it moves fewer
    bytes than the whole halo ring."""
    W, H, tx, ty, halo = shape
    g = TileGrid(W, H, tx, ty, halo=halo)
    bpp = {1: 12, 2: 1, 4: 12, 8: 12}
    for frame in range(1, 17):
        ring_bytes = plan_bytes = 0
        for r in range(g.ranks):
            st, rs = g.need(r, frame)
            assert (st, rs) == _need_restated(g, r, frame)
            x, y, w, h = g.tile(r)
            assert intersect(st, rs) == rs and intersect(g.region(r), st) == st
            assert intersect(st, (x - 1, y - 1, w + 2, h + 2)) == intersect((0, 0, W, H), (x - 1, y - 1, w + 2, h + 2))
            plan = g.frame_plan(r, frame)
            back = {p: (s2, r2) for p, s2, r2 in []}
            for peer, send, recv in plan:
                back = {p: (s2, r2) for p, s2, r2 in g.frame_plan(peer, frame)}
                assert back[r][0] == recv and back[r][1] == send
            for k, need in ((1, st), (8, rs)):
                got = np.zeros((H, W), np.int32)
                for peer, _, recv in plan:
                    pt = g.tile(peer)
                    for (qx, qy, qw, qh, m) in recv:
                        if m & k:
                            assert intersect(pt, (qx, qy, qw, qh)) == (qx, qy, qw, qh)
                            got[qy:qy + qh, qx:qx + qw] += 1
                want = np.zeros((H, W), np.int32)
                want[need[1]:need[1] + need[3], need[0]:need[0] + need[2]] = 1
                want[y:y + h, x:x + w] = 0
                assert (got == want).all(), (frame, r, k)
            ring_bytes += sum(rect_bytes([Plane(0, g.region(r), b) for _, b in STATE_PLANES], rc) for _, _, rc in g.plan(r))
            plan_bytes += sum(q[2] * q[3] * sum(bpp[b] for b in bpp if q[4] & b) for _, _, recv in plan for q in recv)
        assert plan_bytes < ring_bytes


def _truth(name, bpp, W, H):
    """Deterministic per-plane content of the whole frame (bytes)."""
    idx = np.arange(W * H * bpp, dtype=np.uint64).reshape(H, W * bpp)
    salt = sum(map(ord, name))
    return ((idx * 2654435761 + salt) >> 7).astype(np.uint8)


def _worker(rank, world, port, shape, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        g = TileGrid(*shape, halo=40)
        rx, ry, rw, rh = g.region(rank)
        tx, ty, tw, th = g.tile(rank)
        arrays, planes = [], []
        for name, bpp in STATE_PLANES:
            full = _truth(name, bpp, g.width, g.height)
            a = np.full((rh, rw * bpp), 0xEE, np.uint8)
            # my tile holds its values; the ring is stale
            a[ty - ry:ty - ry + th, (tx - rx) * bpp:(tx - rx + tw) * bpp] = full[ty:ty + th, tx * bpp:(tx + tw) * bpp]
            arrays.append((a, full))
            planes.append(Plane(a.ctypes.data, (rx, ry, rw, rh), bpp))
        t = DistTransport(g, rank, torch.device("cpu"))
        t.exchange(planes, HostCopier())
        ok = all((a == full[ry:ry + rh, rx * p.bpp:(rx + rw) * p.bpp]).all() for (a, full), p in zip(arrays, planes))
        sent = sum(rect_bytes(planes, s) for _, s, _ in g.plan(rank))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok, sent))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e), 0))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("shape", [(300, 200, 2, 1), (256, 256, 2, 2), (200, 300, 1, 2)])
def test_halo_exchange_gloo(shape):
    world = shape[2] * shape[3]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, sent in res:
        assert ok is True, (rank, ok)
        assert sent > 0


@pytest.mark.parametrize("region,tile", [((0, 0, 100, 80), (20, 10, 50, 40)), ((0, 0, 100, 80), (0, 0, 60, 80)),
                                         ((10, 20, 70, 50), (10, 20, 70, 50))])
def test_halo_rects_partition_region_minus_tile(region, tile):
    from bmfr_amd.tiling import halo_rects
    m = np.zeros((200, 200), np.int32)
    for x, y, w, h in halo_rects(region, tile):
        m[y:y + h, x:x + w] += 1
    x, y, w, h = tile
    m[y:y + h, x:x + w] += 1
    rx, ry, rw, rh = region
    assert (m[ry:ry + rh, rx:rx + rw] == 1).all() and m.sum() == rw * rh


@pytest.mark.parametrize("W,H,tx,ty,halo", [(7680, 4320, 4, 2, 64), (7680, 4320, 2, 4, 64), (7680, 4320, 2, 2, 64),
                                            (7680, 4320, 2, 1, 64), (480, 288, 4, 2, 38), (352, 224, 2, 1, 48)])
def test_native_plan_equals_frame_plan(W, H, tx, ty, halo):
    """libbmfr's bmfr_halo_plan (the plan bmfr_exchange_* sends on) is
    TileGrid.frame_plan record for record, for every rank and all 16
    block-grid shifts."""
    import bmfr_amd
    from bmfr_amd import tiling
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H)
    g = tiling.TileGrid(W, H, tx, ty, halo=halo)
    for r in range(g.ranks):
        for f in range(16):
            want = [(p, [tuple(x) for x in s], [tuple(x) for x in q]) for p, s, q in g.frame_plan(r, f)]
            assert tiling.native_plan(cfg, g, r, f) == want, (r, f)


@pytest.mark.parametrize("W,H,tx,ty,halo", [(320, 256, 2, 2, 40), (480, 288, 4, 2, 38), (352, 224, 1, 2, 48),
                                            (7680, 4320, 4, 2, 64), (7680, 4320, 2, 4, 64)])
def test_native_messages_match_at_both_ends(W, H, tx, ty, halo):
    """Every message of libbmfr's exchange plan (bmfr_halo_plan, what
    bmfr_exchange_* posts as one ncclSend / ncclRecv pair) is described the
    same way at both ends, for every rank and all 16 block-grid shifts: the
    sender's records for a peer equal that peer's receive records from it,
    hence the packed byte counts agree (packed_bytes == bmfr_halo_copy's
    layout; a mismatch would truncate an RCCL receive or leave it waiting).
    The messages are also laid out in the send / receive buffers in peer
    order at both ends, which the device-copy form of bmfr_exchange_run_all
    reproduces (tests/test_gpu_exchange.py)."""
    import bmfr_amd
    from bmfr_amd import tiling
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H)
    g = tiling.TileGrid(W, H, tx, ty, halo=halo)
    for f in range(16):
        plans = {r: {p: (s, q) for p, s, q in tiling.native_plan(cfg, g, r, f)} for r in range(g.ranks)}
        total_sent = total_recv = 0
        for r, peers in plans.items():
            for p, (send, recv) in peers.items():
                assert r in plans[p], (f, r, p)
                assert plans[p][r][1] == send, (f, r, p)  # the peer receives what I send
                assert plans[p][r][0] == recv, (f, r, p)  # and sends what I receive
                assert tiling.packed_bytes(send) == tiling.packed_bytes(plans[p][r][1])
                total_sent += tiling.packed_bytes(send)
                total_recv += tiling.packed_bytes(recv)
        assert total_sent == total_recv > 0


def test_packed_bytes_pads_segments():
    from bmfr_amd.tiling import HALO_ALL, HALO_RESULT, packed_bytes
    # 3 x 1 px: noisy 36 -> 48, spp 3 -> 16, filtered 36 -> 48, result 36 -> 48
    assert packed_bytes([(0, 0, 3, 1, HALO_ALL)]) == 48 + 16 + 48 + 48
    assert packed_bytes([(0, 0, 4, 4, HALO_RESULT), (5, 5, 1, 1, 2)]) == 192 + 16


def test_native_plan_rejects_bad_grids():
    import ctypes as C

    import bmfr_amd
    from bmfr_amd import _lib
    lib = _lib.load()
    c = bmfr_amd.BmfrConfig(image_width=256, image_height=128, tile=(0, 0, 128, 128), tile_halo=40).to_c()
    n = C.c_int()
    for tiles, rank in [([0, 0, 128, 128, 100, 0, 156, 128], 0),   # overlapping tiles
                        ([0, 0, 128, 128], 0),                     # do not cover the frame
                        ([0, 0, 128, 128, 128, 0, 128, 128], 2)]:  # rank out of range
        arr = (C.c_int * len(tiles))(*tiles)
        assert lib.bmfr_halo_plan(C.byref(c), arr, len(tiles) // 4, rank, 0, None, None, None, None, 0,
                                  C.byref(n)) == 1
