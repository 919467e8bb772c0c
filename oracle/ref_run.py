"""Run the reference's own OpenCL kernels (compiled by build_ref.py into
oracle/_ref/*.hsaco) on an MI355X through the HIP module API.

TEST INFRASTRUCTURE ONLY: used by tests/ to pin the CPU oracle to the
reference and to produce the golden vectors.  `RefLoop` replays tasks()'
frame loop (bmfr.cpp:417-485) with the reference's launch geometry
(bmfr.cpp:245-249): 8x8 work-groups over the (WORKSET+32)^2 margin grid for
accumulate_noisy_data, 256-thread work-groups per block for the fitter, 8x8
work-groups over WORKSET for the three per-pixel kernels.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import struct

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")


class _Hip:
    def __init__(self):
        lib = C.CDLL("libamdhip64.so.7")  # the runtime torch already loaded
        lib.hipModuleLoad.argtypes = [C.POINTER(C.c_void_p), C.c_char_p]
        lib.hipModuleGetFunction.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_char_p]
        lib.hipModuleLaunchKernel.argtypes = [C.c_void_p, C.c_uint, C.c_uint, C.c_uint, C.c_uint, C.c_uint,
                                              C.c_uint, C.c_uint, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.hipModuleUnload.argtypes = [C.c_void_p]
        for n in ("hipModuleLoad", "hipModuleGetFunction", "hipModuleLaunchKernel", "hipModuleUnload"):
            getattr(lib, n).restype = C.c_int
        self.lib = lib


_HIP = None


def hip() -> _Hip:
    global _HIP
    if _HIP is None:
        _HIP = _Hip()
    return _HIP


def available(config: str, mode: str = "strict") -> bool:
    return os.path.exists(os.path.join(REF_DIR, f"{config}_{mode}.hsaco"))


class RefModule:
    """One compiled reference program (one -D configuration)."""

    def __init__(self, config: str, mode: str = "strict"):
        torch.cuda.init()
        path = os.path.join(REF_DIR, f"{config}_{mode}.hsaco")
        with open(os.path.join(REF_DIR, f"{config}_{mode}.json")) as f:
            self.meta = json.load(f)["kernels"]
        self.h = hip()
        mod = C.c_void_p()
        err = self.h.lib.hipModuleLoad(C.byref(mod), path.encode())
        if err:
            raise RuntimeError(f"hipModuleLoad({path}) failed: {err}")
        self.mod = mod
        self.fns = {}

    def fn(self, name: str):
        if name not in self.fns:
            f = C.c_void_p()
            err = self.h.lib.hipModuleGetFunction(C.byref(f), self.mod, name.encode())
            if err:
                raise RuntimeError(f"hipModuleGetFunction({name}) failed: {err}")
            self.fns[name] = f
        return self.fns[name]

    def launch(self, name: str, grid, block, args, stream=None) -> None:
        """args: list of tensors (global pointers) / ('f', [floats]) / ('i', int)
        in declaration order; packed at the metadata's offsets."""
        layout = self.meta[name]["args"]
        assert len(layout) == len(args), (name, len(layout), len(args))
        end = max(a["offset"] + a["size"] for a in layout)
        buf = bytearray(end)
        for a, v in zip(layout, args):
            off, size = a["offset"], a["size"]
            if isinstance(v, torch.Tensor):
                assert size == 8
                struct.pack_into("<Q", buf, off, v.data_ptr())
            elif isinstance(v, tuple) and v[0] == "f":
                vals = list(v[1])
                assert size == 4 * len(vals), (name, size, len(vals))
                struct.pack_into(f"<{len(vals)}f", buf, off, *vals)
            elif isinstance(v, tuple) and v[0] == "i":
                assert size == 4
                struct.pack_into("<i", buf, off, v[1])
            else:
                raise TypeError(v)
        cbuf = (C.c_char * len(buf)).from_buffer(buf)
        size = C.c_size_t(len(buf))
        # HIP_LAUNCH_PARAM_BUFFER_POINTER = 1, _BUFFER_SIZE = 2, _END = 3
        extra = (C.c_void_p * 5)(1, C.cast(cbuf, C.c_void_p), 2, C.cast(C.pointer(size), C.c_void_p), 3)
        st = (stream or torch.cuda.current_stream()).cuda_stream
        err = self.h.lib.hipModuleLaunchKernel(self.fn(name), grid[0], grid[1], grid[2], block[0], block[1],
                                               block[2], 0, st, None, extra)
        if err:
            raise RuntimeError(f"hipModuleLaunchKernel({name}) failed: {err}")


class RefLoop:
    """tasks()' frame loop over the reference kernels (torch-owned buffers)."""

    def __init__(self, rc, mode: str = "strict", device: int = 0):
        from ref_configs import RefConfig  # noqa: F401  (rc is a RefConfig)
        self.rc = rc
        self.m = RefModule(rc.name, mode)
        dev = torch.device("cuda", device)
        W, H = rc.width, rc.height
        ww, wh = rc.workset
        mw, mh = rc.margins
        B = rc.buffer_count
        f32 = dict(dtype=torch.float32, device=dev)
        # Allocation sizes as bmfr.cpp:316-343 (OUTPUT_SIZE-based); kernels use W stride.
        out_sz = ww * wh
        img = lambda n=out_sz: torch.zeros(n * 3, **f32)  # noqa: E731
        self.normals, self.positions, self.noisy = [img(), img()], [img(), img()], [img(), img()]
        self.out = [img(mw * mh), img(mw * mh)]
        self.result = [img(), img()]
        self.spp = [torch.zeros(out_sz, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.albedo, self.tone = img(W * H), img(W * H)
        self.filtered = img()
        self.prev_pixels = torch.zeros(out_sz * 2, **f32)
        self.accept = torch.zeros(out_sz, dtype=torch.uint8, device=dev)
        self.tmp = torch.zeros(mw * mh * B, dtype=torch.float16 if rc.half_tmp else torch.float32, device=dev)
        G = rc.blocks
        self.weights = torch.zeros(G * (B - 3) * 3, **f32)
        self.mins_maxs = torch.zeros(G * len(rc.scaled) * 2, **f32)
        self.swapped = False

    def cur(self, pair):
        return pair[0] if self.swapped else pair[1]

    def prev(self, pair):
        return pair[1] if self.swapped else pair[0]

    def upload(self, noisy, normals, positions, albedo) -> None:
        n = self.rc.width * self.rc.height * 3
        self.cur(self.noisy)[:n].copy_(noisy.reshape(-1))
        self.cur(self.normals)[:n].copy_(normals.reshape(-1))
        self.cur(self.positions)[:n].copy_(positions.reshape(-1))
        self.albedo.copy_(albedo.reshape(-1))

    def run_stages(self, prev_vp, jitter, frame: int, record=None, upstream_launch: bool = False,
                   marks=None) -> None:
        """One frame of tasks().  upstream_launch: accumulate_noisy_data as
        the reference launches it (its own kernel, one launch over the margin
        grid, bmfr.cpp:446-447) instead of the race-free margin / owner pass
        pair -- the form the reference-speed test times; its margin values
        may then differ by the A.4 race, so parity tests keep the default.
        marks: a list that receives a recorded timing event after each
        kernel (the per-kernel split of the reference-speed test)."""
        rc, m = self.rc, self.m

        def mark():
            if marks is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                marks.append(ev)

        ww, wh = rc.workset
        mw, mh = rc.margins
        fr = ("i", frame)
        acc_args = [self.prev_pixels, self.accept, self.cur(self.normals), self.prev(self.normals),
                    self.cur(self.positions), self.prev(self.positions), self.cur(self.noisy),
                    self.prev(self.noisy), self.prev(self.spp), self.cur(self.spp), self.tmp,
                    ("f", prev_vp), ("f", jitter), fr]
        if upstream_launch:
            m.launch("accumulate_noisy_data", (mw // 8, mh // 8, 1), (8, 8, 1), acc_args)
        else:
            for pas in (0, 1):  # margins first, then owners (race-free semantics)
                m.launch("ref_accumulate_noisy_data", (mw // 8, mh // 8, 1), (8, 8, 1), acc_args + [("i", pas)])
        mark()
        if record is not None:
            record["tmp_noisy"] = self.tmp.clone()
        m.launch("ref_fitter", (rc.blocks, 1, 1), (256, 1, 1), [self.weights, self.mins_maxs, self.tmp, fr])
        mark()
        g8 = (ww // 8, wh // 8, 1)
        m.launch("weighted_sum", g8, (8, 8, 1), [self.weights, self.mins_maxs, self.filtered,
                                                 self.cur(self.normals), self.cur(self.positions),
                                                 self.cur(self.noisy), fr])
        mark()
        m.launch("accumulate_filtered_data", g8, (8, 8, 1),
                 [self.filtered, self.prev_pixels, self.accept, self.albedo, self.tone, self.cur(self.spp),
                  self.prev(self.out), self.cur(self.out), fr])
        mark()
        m.launch("taa", g8, (8, 8, 1), [self.prev_pixels, self.tone, self.cur(self.result),
                                        self.prev(self.result), fr])
        mark()
        if record is not None:
            W, H = rc.width, rc.height
            n = W * H
            record.update(
                tmp_fit=self.tmp.clone(), weights=self.weights.clone(), mins_maxs=self.mins_maxs.clone(),
                filtered=self.filtered[:3 * n].clone(), acc=self.cur(self.out)[:3 * n].clone(),
                tone=self.tone.clone(), result=self.cur(self.result)[:3 * n].clone(),
                spp=self.cur(self.spp)[:n].clone(), accept=self.accept[:n].clone(),
                prev_pixel=self.prev_pixels[:2 * n].clone(), noisy=self.cur(self.noisy)[:3 * n].clone())

    def swap(self) -> None:
        self.swapped = not self.swapped
