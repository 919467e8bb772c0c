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
