"""The C++ host program (host/bmfr_host.cpp: bmfr.cpp's tasks() on libbmfr)
end to end on the GPU: a synthetic dataset written as EXR files +
camera_matrices.h, read back and denoised, must give bit for bit the
outputs of the in-memory synthetic path and of the Python Denoiser."""
from __future__ import annotations

import ctypes as C
import subprocess

import numpy as np
import pytest
import torch

import bmfr_amd
from bmfr_amd import _build

pytestmark = pytest.mark.gpu

W, H, F = 160, 96, 5


def _run(args, cwd):
    exe = _build.build_host()
    r = subprocess.run([exe, *args], cwd=cwd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def _read(path):
    lib = C.CDLL(_build.IO_LIB)
    lib.bmfr_exr_read_rgb.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p]
    out = np.empty((H, W, 3), np.float32)
    assert lib.bmfr_exr_read_rgb(str(path).encode(), W, H, out.ctypes.data) == 0
    return out


def test_host_dataset_roundtrip_matches_denoiser(tmp_path, gpu):
    ds = tmp_path / "ds"
    ds.mkdir()
    size = ["--width", str(W), "--height", str(H), "--frames", str(F)]
    _run(["--write-synthetic", str(ds), *size], tmp_path)
    log = _run(["--input", str(ds), *size, "--exr", "--output", str(tmp_path / "file_")], tmp_path)
    assert "Total (device" in log
    _run(["--synthetic", *size, "--exr", "--output", str(tmp_path / "syn_"), "--no-pipeline"], tmp_path)
    den = bmfr_amd.Denoiser(bmfr_amd.BmfrConfig(image_width=W, image_height=H))
    problems = []
    for f in range(F):
        # bmfr_host renders with the CPU renderer (bmfr_synth_frame_host); feed the
        # Denoiser the same bytes (the device renderer's libm may differ by an ulp).
        fr = {k: torch.from_numpy(v.reshape(-1)).cuda() for k, v in bmfr_amd.synth_frame_host(W, H, f).items()}
        vp, _ = bmfr_amd.synth_camera(W, H, max(f - 1, 0))
        _, jit = bmfr_amd.synth_camera(W, H, f)
        den.process_frame(fr["noisy"], fr["normals"], fr["positions"], fr["albedo"], vp, jit, f)
        want = den.copy_output(torch.empty(W * H * 3, device="cuda")).cpu().numpy().reshape(H, W, 3)
        a, b = _read(tmp_path / f"file_{f}.exr"), _read(tmp_path / f"syn_{f}.exr")
        for name, got in (("exr dataset", a), ("in-memory synthetic", b)):
            bad = got.view(np.uint32) != want.view(np.uint32)
            if bad.any():
                problems.append(f"frame {f}, {name}: {int(bad.sum())} of {bad.size} floats differ, "
                                f"first at {np.argwhere(bad)[0].tolist()}, "
                                f"max |diff| {float(np.abs(got - want).max()):.3g}")
    assert not problems, "\n".join(problems)

def test_device_renderer_matches_host_renderer(gpu):
    """The GPU renderer (bench inputs) and the CPU renderer (bmfr_host, the
    CPU baseline) draw the same scene: geometry bit for bit, shading within
    the libm ulp differences of logf/powf."""
    for f in (0, 1, 4):
        h = bmfr_amd.synth_frame_host(W, H, f)
        d = bmfr_amd.synth_frame_device(W, H, f)
        for k in ("normals", "positions", "albedo"):
            assert d[k].cpu().numpy().tobytes() == h[k].reshape(-1).tobytes(), (f, k)
        np.testing.assert_allclose(d["noisy"].cpu().numpy(), h["noisy"].reshape(-1), rtol=1e-5, atol=0)


@pytest.mark.parametrize("grid,halo", [("2x2", 40), ("4x1", 38)])
def test_host_tile_grid_matches_untiled(tmp_path, grid, halo, gpu):
    """bmfr_host --tile-grid: the frame sharded into tiles, one context per
    tile, the halo exchanged by bmfr_exchange_run_all (all tiles on one GPU:
    device copies), == the untiled host run bit for bit, every frame."""
    size = ["--width", str(W), "--height", str(H), "--frames", str(F), "--synthetic", "--exr"]
    _run([*size, "--output", str(tmp_path / "full_")], tmp_path)
    log = _run([*size, "--output", str(tmp_path / "tile_"), "--tile-grid", grid, "--tile-halo", str(halo)], tmp_path)
    assert "Tiled:" in log, log
    for f in range(F):
        a, b = _read(tmp_path / f"tile_{f}.exr"), _read(tmp_path / f"full_{f}.exr")
        bad = a.view(np.uint32) != b.view(np.uint32)
        assert not bad.any(), (grid, f, int(bad.sum()), np.argwhere(bad)[:3].tolist())
