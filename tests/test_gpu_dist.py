"""The multi-rank tiled path as bench.py runs it, in 2, 4 and 8 processes on
one GPU (gloo with host-staged messages stands in for RCCL; 8 ranks = the
4x2 grid of the driver's 8-GPU node): each rank denoises its
tile with bmfr_process_frame_interior, the halo exchange on its own stream
(DistTransport.exchange_ctx: bmfr_halo_copy pack, isend/irecv, unpack) and
bmfr_process_frame_border, and must reproduce its tile of the untiled frame
bit for bit every frame."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, FRAMES = 320, 192, 6


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist

        import bmfr_amd
        from bmfr_amd import tiling
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        grid = tiling.TileGrid(W, H, *tiling.grid_for(world), halo=40)
        full = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
        den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H, tile=grid.tile(rank),
                                                    tile_halo=40))
        transport = tiling.DistTransport(grid, rank, torch.device("cuda", 0), host_staging=True)
        compute, comm = torch.cuda.current_stream(), torch.cuda.Stream()
        done = torch.cuda.Event()
        reg, (tx, ty, tw, th) = den.region, grid.tile(rank)
        prev, bad = None, []
        for f in range(FRAMES):
            vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
            _, jit = bmfr_amd.synth_camera(W, H, f)
            fr = bmfr_amd.synth_frame_device(W, H, f)
            full.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
            inp = bmfr_amd.synth_region_device(W, H, reg, f)
            args = (inp["noisy"], inp["normals"], inp["positions"], inp["albedo"], vp, jit, f)
            kw = dict(prev_normals=prev["normals"] if prev else None,
                      prev_positions=prev["positions"] if prev else None)
            if f == 0:
                den.process_frame(*args, **kw)
            else:
                comm.wait_event(done)
                den.process_frame_interior(*args, **kw)
                with torch.cuda.stream(comm):
                    transport.exchange_ctx(den, f)
                compute.wait_stream(comm)
                den.process_frame_border(*args, **kw)
            done.record(compute)
            prev = inp
            a = den.copy_output(torch.empty(reg[2] * reg[3] * 3, device="cuda")).cpu().numpy()
            b = full.copy_output(torch.empty(W * H * 3, device="cuda")).cpu().numpy()
            a = a.reshape(reg[3], reg[2], 3)[ty - reg[1]:ty - reg[1] + th, tx - reg[0]:tx - reg[0] + tw]
            b = b.reshape(H, W, 3)[ty:ty + th, tx:tx + tw]
            if a.tobytes() != b.tobytes():
                bad.append((f, int((a != b).sum())))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, bad))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 4, 8])  # 8: the driver node's 4x2 plan (bench.py --gpus 8), rehearsed
def test_two_process_tiled_frames_match_untiled(world, gpu):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=400) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == [] for v in results.values()), results
