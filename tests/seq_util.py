"""Shared helpers for the sequence tests: drive any frame loop (CPU oracle,
reference kernels, libbmfr stages) over the synthetic sequence and compare
the recorded buffers."""
from __future__ import annotations

import hashlib

import numpy as np

import bmfr_amd
from ref_configs import RefConfig

# Buffers whose values are pinned bit for bit.  tone / result go through
# powr(), which the GPU library does not round correctly, so the CPU oracle
# is held to a tolerance there (GPU vs GPU stays bit-exact).
EXACT_KEYS = ("tmp_noisy", "tmp_fit", "weights", "mins_maxs", "filtered", "acc", "spp", "accept",
              "prev_pixel", "noisy")
POWR_KEYS = ("tone", "result")
ALL_KEYS = EXACT_KEYS + POWR_KEYS


def frame_inputs(rc: RefConfig, frame: int):
    return bmfr_amd.synth_frame_host(rc.width, rc.height, frame, seed=rc.seed)


def camera(rc: RefConfig, frame: int):
    """(camera_matrices[max(frame-1,0)], pixel_offsets[frame]), bmfr.cpp:440-444."""
    vp, _ = bmfr_amd.synth_camera(rc.width, rc.height, max(frame - 1, 0))
    _, jit = bmfr_amd.synth_camera(rc.width, rc.height, frame)
    return vp, jit


def input_digest(fr) -> str:
    h = hashlib.sha256()
    for k in ("noisy", "normals", "positions", "albedo"):
        h.update(np.ascontiguousarray(fr[k], np.float32).tobytes())
    return h.hexdigest()


def to_np(x) -> np.ndarray:
    if hasattr(x, "detach"):
        x = x.detach().cpu()
        if str(x.dtype) == "torch.float16":
            return x.view(__import__("torch").int16).numpy().view(np.uint16)
        return x.numpy()
    return np.asarray(x)


def digest(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(to_np(a)).tobytes()).hexdigest()


def sample_idx(n: int, k: int = 8192) -> np.ndarray:
    return np.unique(np.linspace(0, n - 1, min(n, k)).astype(np.int64))


def run_loop(loop, rc: RefConfig, frames: int, to_device=None, sync=None):
    """Run `frames` frames; returns a list of per-frame dicts of numpy arrays."""
    out = []
    for f in range(frames):
        fr = frame_inputs(rc, f)
        if to_device is not None:
            fr = {k: to_device(v) for k, v in fr.items()}
        loop.upload(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"])
        vp, jit = camera(rc, f)
        rec = {}
        loop.run_stages(vp, jit, f, record=rec)
        if sync is not None:
            sync()
        out.append({k: to_np(v).copy() for k, v in rec.items()})
        loop.swap()
    return out


def rel_l2(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    d = np.linalg.norm(a - b)
    n = np.linalg.norm(b)
    return float(d / n) if n > 0 else float(d)


def compare_exact(got, ref, keys=EXACT_KEYS, where=""):
    """Assert bitwise equality of every key (as raw bytes); report the first
    mismatching frame with a useful summary."""
    for f, (g, r) in enumerate(zip(got, ref)):
        for k in keys:
            a, b = g[k], r[k]
            assert a.shape == b.shape, (where, f, k, a.shape, b.shape)
            if a.tobytes() != b.tobytes():
                av = a.view(np.uint8) if a.dtype == np.uint8 else a
                bad = np.flatnonzero(av != b)
                msg = f"{where} frame {f} {k}: {bad.size} of {a.size} differ, first at {bad[:5]}: " \
                      f"{a.reshape(-1)[bad[:5]]} vs {b.reshape(-1)[bad[:5]]}"
                if a.dtype == np.float32:
                    msg += f", rel_l2 {rel_l2(a, b):.3e}"
                raise AssertionError(msg)
