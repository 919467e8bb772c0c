"""C-ABI checks that need no GPU: every symbol include/bmfr.h declares is
exported, host-side functions behave, device entry points fail cleanly."""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np
import pytest

import bmfr_amd
from bmfr_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    inc = os.path.join(ROOT, "include")
    text = "".join(open(os.path.join(inc, f)).read() for f in sorted(os.listdir(inc)) if f.endswith(".h"))
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bmfr_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def reference_sizes(W, H, ns, fs, half):
    """bmfr.cpp:104-118 and 316-343, restated."""
    ww, wh = 32 * ((W + 31) // 32), 32 * ((H + 31) // 32)
    mw, mh = ww + 32, wh + 32
    B = ns + fs + 3
    G = (mw // 32) * (mh // 32)
    return dict(buffer_count=B, r_edge=B - 2, workset_width=ww, workset_height=wh,
                workset_with_margins_width=mw, workset_with_margins_height=mh, blocks=G,
                tmp_data_bytes=mw * mh * B * (2 if half else 4), weights_bytes=G * (B - 3) * 12,
                mins_maxs_bytes=G * fs * 8, image_bytes=W * H * 12)


@pytest.mark.parametrize("W,H,third,half", [(1280, 720, False, 1), (1920, 1080, False, 1), (3840, 2160, False, 0),
                                            (3840, 2160, True, 1), (7680, 4320, False, 1), (100, 72, True, 1),
                                            (48, 48, False, 1)])
def test_config_sizes_match_reference(W, H, third, half):
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H, use_half_precision_in_tmp_data=half,
                              scaled=bmfr_amd.SCALED_THIRD_ORDER if third else bmfr_amd.SCALED_DEFAULT)
    s = cfg.sizes()
    want = reference_sizes(W, H, 4, 9 if third else 6, half)
    got = {k: getattr(s, k) for k in want}
    assert got == want
    # untiled per-frame launches: one below 4096 K1 blocks, two from there
    assert s.frame_launches == (2 if s.blocks >= 4096 else 1)


@pytest.mark.parametrize("W,H", [(40, 64), (64, 40), (46, 100), (33, 33), (0, 10), (31, 200)])
def test_config_rejects_images_mirror_cannot_cover(W, H):
    # mirror() (bmfr.cl:207-216) needs every margin pixel within one image
    # size of the border; below that the reference reads out of bounds.
    cfg = bmfr_amd.BmfrConfig(image_width=W, image_height=H)
    with pytest.raises(bmfr_amd.BmfrError) as e:
        cfg.sizes()
    assert e.value.status == 1


def test_config_rejects_bad_features():
    lib = _lib.load()
    c = bmfr_amd.BmfrConfig().to_c()
    c.feature_buffers[2] = 99
    s = _lib.Sizes()
    assert lib.bmfr_config_sizes(C.byref(c), C.byref(s)) == 1
    c = bmfr_amd.BmfrConfig().to_c()
    c.features_scaled = 20
    assert lib.bmfr_config_sizes(C.byref(c), C.byref(s)) == 1


def test_default_config_is_reference_defines():
    lib = _lib.load()
    c = _lib.Config()
    lib.bmfr_config_default(C.byref(c), 1280, 720)
    assert (c.image_width, c.image_height) == (1280, 720)
    assert (c.features_not_scaled, c.features_scaled) == (4, 6)
    assert list(c.feature_buffers[:10]) == list(range(10))
    assert c.noise_amount == 1e-2
    assert np.float32(c.blend_alpha) == np.float32(0.2)
    assert np.float32(c.second_blend_alpha) == np.float32(0.1)
    assert np.float32(c.taa_blend_alpha) == np.float32(0.2)
    assert c.use_half_precision_in_tmp_data == 1
    # the options beyond the reference's defines default to its behaviour:
    # untiled, f32 inputs, exact fit (library_powr 0 = the correctly rounded powr)
    assert (c.tile_width, c.tile_height, c.input_half, c.library_powr, c.fast_fit) == (0, 0, 0, 0, 0)


def test_status_strings():
    lib = _lib.load()
    for s in range(6):
        assert lib.bmfr_status_string(s).decode() == _lib.STATUS[s]


def test_null_arguments_are_errors_not_crashes():
    lib = _lib.load()
    assert lib.bmfr_destroy(None) == 1
    assert lib.bmfr_fitter(None, None, None, None, None, 0) == 1
    assert lib.bmfr_process_frame(None, None, None, None, None, 0) == 1
    assert lib.bmfr_output(None) is None
    n = C.c_int()
    assert lib.bmfr_get_profile(None, None, 0, C.byref(n)) == 1


def test_synth_camera_is_column_major_projection():
    W, H = 640, 360
    vp, off = bmfr_amd.synth_camera(W, H, 3)
    M = np.array(vp, np.float64).reshape(4, 4).T  # column-major -> row-major
    fr = bmfr_amd.synth_frame_host(W, H, 3)
    # A pixel's world position reprojected with its own frame's matrix lands
    # on (x + jx, y + 1 - jy) in the reference's uv -> pixel convention
    # (bmfr.cl:343-355).
    for (x, y) in [(10, 20), (320, 180), (600, 50)]:
        p = np.append(fr["positions"][y, x].astype(np.float64), 1.0)
        c = M @ p
        u, v = (c[0] / c[3] + 1) / 2 * W, (c[1] / c[3] + 1) / 2 * H
        assert abs(u - (x + off[0])) < 2e-2 and abs(v - (y + 1 - off[1])) < 2e-2, (x, y, u, v, off)
    assert 0 <= off[0] < 1 and 0 <= off[1] < 1


def test_synth_frame_properties():
    fr = bmfr_amd.synth_frame_host(96, 64, 0, clean=True)
    n = fr["normals"]
    assert np.allclose(np.linalg.norm(n, axis=-1), 1, atol=1e-5)
    assert np.abs(fr["positions"]).max() <= 16
    assert fr["albedo"].min() >= 0.1 - 1e-6 and fr["albedo"].max() <= 0.9 + 1e-6
    assert (fr["noisy"] >= 0).all() and np.isfinite(fr["noisy"]).all()
    assert 0 <= fr["clean"].min() and fr["clean"].max() <= 1
    again = bmfr_amd.synth_frame_host(96, 64, 0, clean=True)
    for k in fr:
        assert fr[k].tobytes() == again[k].tobytes()


def test_config_struct_matches_header():
    """The ctypes mirror of bmfr_config has the header's size (fast_fit is the last field)."""
    import subprocess
    import tempfile
    src = '#include <stdio.h>\n#include "bmfr.h"\nint main(void){printf("%zu %zu", sizeof(bmfr_config), ' \
          'sizeof(bmfr_frame_inputs));return 0;}\n'
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        cfg_size, in_size = map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split())
    assert cfg_size == C.sizeof(_lib.Config)
    assert in_size == C.sizeof(_lib.FrameInputs)


def test_split_frame_calls_validate_arguments():
    lib = _lib.load()
    assert lib.bmfr_process_frame_interior(None, None, None, None, None, 0) == 1
    assert lib.bmfr_process_frame_border(None, None, None, None, None, 0) == 1


def test_library_build_id_is_the_tree():
    """libbmfr.so carries the SHA-256 of the sources it was built from, and
    it is this tree's (the loader refuses anything else)."""
    from bmfr_amd import _build
    lib = _lib.load()
    assert lib.bmfr_build_id().decode() == _build.source_hash()
    assert _build.embedded_id(_lib.LIB_PATH) == _build.source_hash()


def _fake_lib(tmp_path, ident: str, name: str) -> str:
    import subprocess
    src = tmp_path / f"{name}.c"
    src.write_text('const char* bmfr_build_id(void) { return "%s"; }\n' % ident)
    so = str(tmp_path / f"lib{name}.so")
    subprocess.run(["gcc", "-shared", "-fPIC", str(src), "-o", so], check=True)
    return so


def test_mismatched_library_is_refused(tmp_path, monkeypatch):
    from bmfr_amd import _build
    so = _fake_lib(tmp_path, "0" * 64, "stale")
    with pytest.raises(_lib.StaleLibraryError, match="other sources"):
        _lib.check_build_id(C.CDLL(so), so)
    # a probe build of the right sources is refused too, unless asked for
    probe = _fake_lib(tmp_path, _build.source_hash() + "+-DBMFR_PROBE_NOSC1", "probe")
    monkeypatch.delenv("BMFR_ALLOW_PROBE", raising=False)
    with pytest.raises(_lib.StaleLibraryError, match="probe build"):
        _lib.check_build_id(C.CDLL(probe), probe)
    monkeypatch.setenv("BMFR_ALLOW_PROBE", "1")
    assert _lib.check_build_id(C.CDLL(probe), probe).endswith("BMFR_PROBE_NOSC1")
    # a variant of the right sources is accepted
    ok = _fake_lib(tmp_path, _build.source_hash() + "+-DBMFR_FAST_SCHED_BARRIER=0", "variant")
    assert _lib.check_build_id(C.CDLL(ok), ok)
