"""Spatial sharding of a frame over ranks, with the per-frame halo exchange
(include/bmfr.h tile_*).

Every rank owns one tile of the frame and runs a tiled libbmfr context over
the tile's *region* (the tile grown by `halo` pixels, clipped to the frame).
The fused K1 covers the blocks of the frame's shifted block grid that reach
the tile plus one pixel, so its block fits are the untiled ones; what a rank
cannot compute itself is the previous frame's temporal state in the halo
ring, which its neighbours own.  Before each frame > 0, `HaloExchange` moves
exactly that: for every pair of ranks, the part of the sender's tile that
lies inside the receiver's region, for the four state planes the next frame
reads (accumulated noisy colour, spp, accumulated filtered colour, TAA
output).  Current-frame inputs need no exchange: each rank reads (renders)
its own region.  What a frame reads of that ring is narrower
(`bmfr_halo_need`, include/bmfr.h): the three accumulation planes over the
pixels of the frame's K1 blocks grown by the reprojection reach, the TAA
output over the tile grown by the reach -- so `frame_plan` sends only those
parts (per frame: the block grid shifts with frame % 16).

Transports: `DistTransport` (torch.distributed point-to-point; RCCL over
xGMI with the nccl backend, gloo on CPU) and `LoopbackTransport` (all tiles
in one process -- the single-GPU parity test of the tiled path).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import functools

# (plane name in bmfr_state_view, bytes per pixel)
STATE_PLANES = (("noisy_accumulated", 12), ("spp", 1), ("filtered_accumulated", 12), ("result", 12))
MIN_HALO = 34  # include/bmfr.h: blocks reach 32 px past the tile, + TAA and bilinear taps
# plane masks of bmfr_halo_copy rectangles (include/bmfr.h BMFR_HALO_*)
HALO_STATE, HALO_RESULT = 1 | 2 | 4, 8
HALO_ALL = HALO_STATE | HALO_RESULT


def _split(n: int, parts: int, i: int) -> tuple[int, int]:
    """[start, end) of part i of n split into `parts` near-equal runs, multiples of 32 where possible."""
    edges = [round(n * k / parts / 32) * 32 for k in range(parts + 1)]
    edges[-1] = n
    return edges[i], edges[i + 1]


def grid_for(n_ranks: int) -> tuple[int, int]:
    """Tile grid (columns, rows) for n ranks: 1x1, 2x1, 2x2, 4x2, ..."""
    tx, ty = 1, 1
    while tx * ty < n_ranks:
        if tx <= ty:
            tx *= 2
        else:
            ty *= 2
    if tx * ty != n_ranks:
        raise ValueError(f"no power-of-two tile grid for {n_ranks} ranks")
    return tx, ty


Rect = tuple  # (x, y, w, h)


def intersect(a: Rect, b: Rect) -> Rect | None:
    x0, y0 = max(a[0], b[0]), max(a[1], b[1])
    x1, y1 = min(a[0] + a[2], b[0] + b[2]), min(a[1] + a[3], b[1] + b[3])
    return (x0, y0, x1 - x0, y1 - y0) if x1 > x0 and y1 > y0 else None


@functools.lru_cache(maxsize=None)
def _need(width, height, tile, halo, frame16):
    """bmfr_halo_need for one tile: (state_rect, result_rect)."""
    from . import _lib
    from .pipeline import BmfrConfig
    cfg = BmfrConfig(image_width=width, image_height=height, tile=tile, tile_halo=halo).to_c()
    st, rs = (C.c_int * 4)(), (C.c_int * 4)()
    _lib.check(_lib.load().bmfr_halo_need(C.byref(cfg), frame16, st, rs), "bmfr_halo_need")
    return tuple(st), tuple(rs)


def _masked(part_of: Rect, state: Rect, result: Rect) -> list:
    """The parts of `part_of` inside the state / result rectangles, as
    bmfr_halo_copy records (x, y, w, h, planes)."""
    s, r = intersect(part_of, state), intersect(part_of, result)
    if s and s == r:
        return [(*s, HALO_ALL)]
    return ([(*s, HALO_STATE)] if s else []) + ([(*r, HALO_RESULT)] if r else [])


@dataclasses.dataclass(frozen=True)
class TileGrid:
    """A width x height frame cut into tiles_x x tiles_y tiles (rank = ty * tiles_x + tx)."""
    width: int
    height: int
    tiles_x: int
    tiles_y: int
    halo: int = 64

    def __post_init__(self):
        if self.halo < MIN_HALO:
            raise ValueError(f"halo must be >= {MIN_HALO}")

    @property
    def ranks(self) -> int:
        return self.tiles_x * self.tiles_y

    def tile(self, rank: int) -> Rect:
        tx, ty = rank % self.tiles_x, rank // self.tiles_x
        x0, x1 = _split(self.width, self.tiles_x, tx)
        y0, y1 = _split(self.height, self.tiles_y, ty)
        return (x0, y0, x1 - x0, y1 - y0)

    def region(self, rank: int) -> Rect:
        x, y, w, h = self.tile(rank)
        x0, y0 = max(0, x - self.halo), max(0, y - self.halo)
        x1, y1 = min(self.width, x + w + self.halo), min(self.height, y + h + self.halo)
        return (x0, y0, x1 - x0, y1 - y0)

    def need(self, rank: int, frame: int):
        """(state_rect, result_rect): what `rank`'s frame `frame` reads of the
        previous state (bmfr_halo_need)."""
        return _need(self.width, self.height, self.tile(rank), self.halo, frame % 16)

    def frame_plan(self, rank: int, frame: int):
        """[(peer, send, recv)] for the exchange before `frame`: send = the
        parts of my tile that the peer's frame reads, recv = the parts of the
        peer's tile that mine reads, as bmfr_halo_copy records."""
        out = []
        for peer in range(self.ranks):
            if peer == rank:
                continue
            send = _masked(self.tile(rank), *self.need(peer, frame))
            recv = _masked(self.tile(peer), *self.need(rank, frame))
            if send or recv:
                out.append((peer, send, recv))
        return out

    def plan(self, rank: int):
        """[(peer, send_rect, recv_rect)]: send the part of my tile inside the
        peer's region, receive the part of the peer's tile inside mine."""
        out = []
        for peer in range(self.ranks):
            if peer == rank:
                continue
            s = intersect(self.tile(rank), self.region(peer))
            r = intersect(self.tile(peer), self.region(rank))
            if s or r:
                out.append((peer, s, r))
        return out


# ---------------------------------------------------------------- copies ----
class Plane:
    """A plane of a region-sized buffer: base pointer, region origin/stride, bytes per pixel."""

    def __init__(self, ptr: int, region: Rect, bpp: int):
        self.ptr, self.region, self.bpp = ptr, region, bpp

    def rect_ptr(self, r: Rect) -> int:
        return self.ptr + ((r[1] - self.region[1]) * self.region[2] + (r[0] - self.region[0])) * self.bpp

    @property
    def pitch(self) -> int:
        return self.region[2] * self.bpp


class HipCopier:
    """Rectangle copies between device planes and flat device buffers (hipMemcpy2DAsync)."""

    def __init__(self, stream=None):
        self.hip = C.CDLL("libamdhip64.so.7")
        self.hip.hipMemcpy2DAsync.restype = C.c_int
        self.hip.hipMemcpy2DAsync.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t,
                                              C.c_size_t, C.c_int, C.c_void_p]
        self.stream = stream

    def copy2d(self, dst: int, dpitch: int, src: int, spitch: int, width: int, rows: int) -> None:
        err = self.hip.hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, 3, self.stream)
        if err != 0:
            raise RuntimeError(f"hipMemcpy2DAsync failed: {err}")

    def fill2d(self, dst: int, pitch: int, value: int, width: int, rows: int) -> None:
        self.hip.hipMemset2DAsync.restype = C.c_int
        self.hip.hipMemset2DAsync.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_size_t, C.c_size_t, C.c_void_p]
        err = self.hip.hipMemset2DAsync(dst, pitch, value, width, rows, self.stream)
        if err != 0:
            raise RuntimeError(f"hipMemset2DAsync failed: {err}")


class HostCopier:
    """The same on host memory (CPU tests)."""

    def copy2d(self, dst: int, dpitch: int, src: int, spitch: int, width: int, rows: int) -> None:
        for y in range(rows):
            C.memmove(dst + y * dpitch, src + y * spitch, width)


def pack(copier, planes, rect: Rect, dst: int) -> int:
    """Copy `rect` of every plane back to back into the flat buffer at dst; returns bytes."""
    off = 0
    for p in planes:
        w = rect[2] * p.bpp
        copier.copy2d(dst + off, w, p.rect_ptr(rect), p.pitch, w, rect[3])
        off += w * rect[3]
    return off


def unpack(copier, planes, rect: Rect, src: int) -> int:
    off = 0
    for p in planes:
        w = rect[2] * p.bpp
        copier.copy2d(p.rect_ptr(rect), p.pitch, src + off, w, w, rect[3])
        off += w * rect[3]
    return off


def rect_bytes(planes, r: Rect | None) -> int:
    return 0 if r is None else sum(r[2] * r[3] * p.bpp for p in planes)


# ------------------------------------------------- libbmfr halo copies ----
def _rect_array(rects):
    """bmfr_halo_copy records: (x, y, w, h[, planes]) -> 5 ints each (all planes by default)."""
    recs = [tuple(r) if len(r) == 5 else (*r, HALO_ALL) for r in rects]
    return (C.c_int * max(5 * len(recs), 1))(*[v for r in recs for v in r])


def packed_bytes(records) -> int:
    """bmfr_halo_copy's packed size of bmfr_halo_copy records (x, y, w, h,
    planes), host only: rectangle after rectangle, plane after plane, each
    segment padded to 16 bytes (include/bmfr.h) -- the message size both ends
    of an exchange compute (bmfr_amd/csrc/bmfr_capi.hip bmfr_halo_copy)."""
    bpp = [b for _, b in STATE_PLANES]
    total = 0
    for x, y, w, h, mask in records:
        for k, b in enumerate(bpp):
            if mask & (1 << k):
                total += (w * b * h + 15) & ~15
    return total


def halo_bytes(denoiser, rects) -> int:
    """Packed size of the rectangles' segments (bmfr_halo_copy layout)."""
    from ._lib import check
    n = C.c_size_t()
    check(denoiser.lib.bmfr_halo_copy(denoiser.handle, None, _rect_array(rects), len(rects), None, 0, C.byref(n)),
          "bmfr_halo_copy")
    return n.value


def halo_copy(denoiser, rects, buf_ptr: int, unpack: bool, stream=None) -> None:
    """Pack (or unpack) the rectangles of the state planes into (from) a device
    buffer in one kernel launch on `stream` (torch stream; default current)."""
    import torch

    from ._lib import check
    if not rects:
        return
    s = (stream or torch.cuda.current_stream()).cuda_stream
    check(denoiser.lib.bmfr_halo_copy(denoiser.handle, s, _rect_array(rects), len(rects), buf_ptr, int(unpack),
                                      None), "bmfr_halo_copy")


# ------------------------------------------------------------- transports ----
class DistTransport:
    """torch.distributed point-to-point: one grouped batch of isend/irecv per frame."""

    def __init__(self, grid: TileGrid, rank: int, device, host_staging: bool = False):
        """host_staging: the planes are on a GPU but the process group is gloo
        (rehearsal of the multi-rank path on one GPU): messages go through host
        memory."""
        import torch
        self.torch = torch
        self.grid, self.rank, self.device = grid, rank, device
        self.host_staging = host_staging
        self._bufs = {}
        self._layouts = {}
        self.last_bytes = (0, 0)

    def buffer(self, key, nbytes, device=None):
        b = self._bufs.get(key)
        if b is None or b.numel() < nbytes:
            b = self.torch.empty(max(nbytes, 1), dtype=self.torch.uint8, device=device or self.device)
            self._bufs[key] = b
        return b

    def exchange_ctx(self, denoiser, frame: int) -> None:
        """The exchange before `frame` on a tiled Denoiser (TileGrid.frame_plan)
        with libbmfr's one-launch pack and unpack (bmfr_halo_copy) on the
        current stream: two kernels around one grouped isend/irecv batch
        (RCCL orders it on that stream).  self.last_bytes = (sent, received)."""
        import torch.distributed as dist
        key = frame % 16
        if key not in self._layouts:
            plan = self.grid.frame_plan(self.rank, frame)
            sends = [(p, s) for p, s, _ in plan if s]
            recvs = [(p, r) for p, _, r in plan if r]
            self._layouts[key] = (sends, [halo_bytes(denoiser, s) for _, s in sends],
                                  recvs, [halo_bytes(denoiser, r) for _, r in recvs])
        sends, s_sizes, recvs, r_sizes = self._layouts[key]
        ns, nr = sum(s_sizes), sum(r_sizes)
        self.last_bytes = (ns, nr)
        if not sends and not recvs:
            return
        sbuf = self.buffer("S", ns)
        rbuf = self.buffer("R", nr)
        halo_copy(denoiser, [q for _, s in sends for q in s], sbuf.data_ptr(), unpack=False)
        s_msg, r_msg = sbuf, rbuf
        if self.host_staging:  # gloo: the messages travel through host memory
            cpu = self.torch.device("cpu")
            s_msg, r_msg = self.buffer("SH", ns, cpu), self.buffer("RH", nr, cpu)
            s_msg[:ns].copy_(sbuf[:ns])  # synchronous device-to-host copy on the current stream
        ops, off = [], 0
        for (peer, _), n in zip(sends, s_sizes):
            ops.append(dist.P2POp(dist.isend, s_msg[off:off + n], peer))
            off += n
        off = 0
        for (peer, _), n in zip(recvs, r_sizes):
            ops.append(dist.P2POp(dist.irecv, r_msg[off:off + n], peer))
            off += n
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if self.host_staging:
            rbuf[:nr].copy_(r_msg[:nr])
        halo_copy(denoiser, [q for _, r in recvs for q in r], rbuf.data_ptr(), unpack=True)

    def exchange(self, planes, copier) -> None:
        import torch.distributed as dist
        ops, recvs = [], []
        cpu = self.torch.device("cpu")
        for peer, s, r in self.grid.plan(self.rank):
            if s:
                n = rect_bytes(planes, s)
                buf = self.buffer(("s", peer), n)
                pack(copier, planes, s, buf.data_ptr())
                if self.host_staging:
                    self.torch.cuda.synchronize()
                    sb = self.buffer(("sh", peer), n, cpu)
                    sb[:n].copy_(buf[:n])
                    buf = sb
                ops.append(dist.P2POp(dist.isend, buf[:n], peer))
            if r:
                n = rect_bytes(planes, r)
                buf = self.buffer(("rh" if self.host_staging else "r", peer), n, cpu if self.host_staging else None)
                ops.append(dist.P2POp(dist.irecv, buf[:n], peer))
                recvs.append((r, n, buf))
        if not ops:
            return
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for r, n, buf in recvs:
            if self.host_staging:
                dbuf = self.buffer(("r", r), n)
                dbuf[:n].copy_(buf[:n])
                self.torch.cuda.synchronize()
                buf = dbuf
            unpack(copier, planes, r, buf.data_ptr())


class LoopbackTransport:
    """All tiles in one process: copy each peer's tile part straight into my region."""

    def __init__(self, grid: TileGrid):
        self.grid = grid

    def exchange_all_ctx(self, denoisers, frame: int) -> None:
        """The exchange before `frame` through libbmfr's pack / unpack kernels
        (bmfr_halo_copy): each message packed from the sender's context and
        unpacked into the receiver's, as DistTransport.exchange_ctx moves them."""
        import torch
        for rank in range(self.grid.ranks):
            for peer, s, _ in self.grid.frame_plan(rank, frame):
                if not s:
                    continue
                buf = torch.empty(halo_bytes(denoisers[rank], s), dtype=torch.uint8, device="cuda")
                halo_copy(denoisers[rank], s, buf.data_ptr(), unpack=False)
                halo_copy(denoisers[peer], s, buf.data_ptr(), unpack=True)

    def exchange_all(self, planes_by_rank, copier) -> None:
        for rank in range(self.grid.ranks):
            for peer, _, r in self.grid.plan(rank):
                if not r:
                    continue
                for src, dst in zip(planes_by_rank[peer], planes_by_rank[rank]):
                    w = r[2] * src.bpp
                    copier.copy2d(dst.rect_ptr(r), dst.pitch, src.rect_ptr(r), src.pitch, w, r[3])


def halo_rects(region: Rect, tile: Rect) -> list:
    """The region minus the tile as up to four rectangles."""
    rx, ry, rw, rh = region
    x, y, w, h = tile
    out = [(rx, ry, rw, y - ry), (rx, y + h, rw, ry + rh - y - h), (rx, y, x - rx, h), (x + w, y, rx + rw - x - w, h)]
    return [r for r in out if r[2] > 0 and r[3] > 0]


def state_planes(denoiser) -> list:
    """The four exchanged planes of a tiled Denoiser's last frame (the next frame's previous state)."""
    v = denoiser.state(previous=False)
    reg = denoiser.region
    return [Plane(getattr(v, name), reg, bpp) for name, bpp in STATE_PLANES]


# ------------------------------------------- libbmfr's native exchange ----
def native_plan(cfg, grid: TileGrid, rank: int, frame: int):
    """bmfr_halo_plan (the C plan) in frame_plan's format: [(peer, send, recv)]."""
    from . import _lib
    lib = _lib.load()
    c = dataclasses.replace(cfg, tile=grid.tile(rank), tile_halo=grid.halo).to_c()
    tiles = (C.c_int * (4 * grid.ranks))(*[v for r in range(grid.ranks) for v in grid.tile(r)])
    n = C.c_int()
    _lib.check(lib.bmfr_halo_plan(C.byref(c), tiles, grid.ranks, rank, frame, None, None, None, None, 0,
                                  C.byref(n)), "bmfr_halo_plan")
    cap = 8 * grid.ranks
    peers, sc, rc = (C.c_int * max(n.value, 1))(), (C.c_int * max(n.value, 1))(), (C.c_int * max(n.value, 1))()
    recs = (C.c_int * (5 * cap))()
    _lib.check(lib.bmfr_halo_plan(C.byref(c), tiles, grid.ranks, rank, frame, peers, sc, rc, recs, cap,
                                  C.byref(n)), "bmfr_halo_plan")
    out, k = [], 0
    for i in range(n.value):
        send = [tuple(recs[5 * (k + j):5 * (k + j) + 5]) for j in range(sc[i])]
        k += sc[i]
        recv = [tuple(recs[5 * (k + j):5 * (k + j) + 5]) for j in range(rc[i])]
        k += rc[i]
        out.append((peers[i], send, recv))
    return out


def _tiles_array(grid: TileGrid):
    return (C.c_int * (4 * grid.ranks))(*[v for r in range(grid.ranks) for v in grid.tile(r)])


class RcclComm:
    """libbmfr's RCCL communicator for one rank (bmfr_comm_create); the
    unique id travels over the torch.distributed group (gloo or nccl)."""

    def __init__(self, world: int, rank: int, device: int):
        import torch
        import torch.distributed as dist

        from . import _lib
        self.lib = _lib.load()
        uid = (C.c_char * 128)()
        if rank == 0:
            _lib.check(self.lib.bmfr_comm_unique_id(uid), "bmfr_comm_unique_id")
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8)
        if dist.get_backend() == "nccl":
            t = t.cuda(device)
        dist.broadcast(t, 0)
        uid = (C.c_char * 128)(*t.cpu().tolist())
        h = C.c_void_p()
        _lib.check(self.lib.bmfr_comm_create(uid, world, rank, device, C.byref(h)), "bmfr_comm_create")
        self.handle = h

    def close(self):
        if self.handle:
            self.lib.bmfr_comm_destroy(self.handle)
            self.handle = None


class NativeExchange:
    """One rank's halo exchange inside libbmfr (bmfr_exchange_*): pack, the
    grouped ncclSend / ncclRecv batch and unpack enqueued by ONE C call per
    frame -- the per-frame host work of DistTransport.exchange_ctx (plan
    lookup, P2POp lists, two pack / unpack calls) gone.  comm=None: an
    in-process grid, driven by run_all."""

    def __init__(self, denoiser, grid: TileGrid, rank: int, comm: RcclComm | None):
        from . import _lib
        self.lib = _lib.load()
        self.grid, self.rank, self.comm = grid, rank, comm
        h = C.c_void_p()
        self._tiles = _tiles_array(grid)
        _lib.check(self.lib.bmfr_exchange_create(denoiser.handle, C.byref(denoiser.cfg.to_c()), self._tiles,
                                                 grid.ranks, rank, comm.handle if comm else None, C.byref(h)),
                   "bmfr_exchange_create")
        self.handle = h
        self.last_bytes = (0, 0)

    def bytes(self, frame: int):
        s, r = C.c_size_t(), C.c_size_t()
        self.lib.bmfr_exchange_bytes(self.handle, frame, C.byref(s), C.byref(r))
        return s.value, r.value

    def run(self, frame: int, stream=None) -> None:
        import torch

        from . import _lib
        s = (stream or torch.cuda.current_stream()).cuda_stream
        _lib.check(self.lib.bmfr_exchange_run(self.handle, s, frame), "bmfr_exchange_run")
        self.last_bytes = self.bytes(frame)

    @staticmethod
    def run_all(exchanges, frame: int, streams=None) -> None:
        import torch

        from . import _lib
        n = len(exchanges)
        xs = (C.c_void_p * n)(*[x.handle.value for x in exchanges])
        ss = streams or [torch.cuda.current_stream()] * n
        st = (C.c_void_p * n)(*[s.cuda_stream for s in ss])
        _lib.check(exchanges[0].lib.bmfr_exchange_run_all(xs, n, st, frame), "bmfr_exchange_run_all")

    def close(self):
        if self.handle:
            self.lib.bmfr_exchange_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
