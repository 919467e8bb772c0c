"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
section 5; GPU sanitizers are not available on this pool, so these cover the
CPU side):

* the CPU restatement oracle/bmfr_oracle.c, all five stages over several
  configurations (tests/native/oracle_asan_main.c);
* the EXR reader host/image_io.cpp (PIZ, PXR24, B44 / B44A and DWAA / DWAB
  decoders, scanline and tiled files) -- the one component that parses external files -- over a
  corpus of malformed files derived from valid ones:
  every truncation length of a small file, seeded random byte corruption,
  and hand-made hostile headers (huge chunk offsets, attribute sizes past
  the end, empty single-byte attributes, overflowing data windows).

Both must finish with exit status 0 and no sanitizer report; a malformed
file must be rejected with an error status."""
from __future__ import annotations

import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

import exr_dwa_py
from test_image_io import DWA_OPTS, _attr, _dwa_image, _img, write_exr_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")


def _run(cmd, **kw):
    r = subprocess.run(cmd, capture_output=True, text=True, env=ENV, timeout=600, **kw)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
    return out


def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_asan")
    _run(["gcc", "-std=c99", "-ffp-contract=off", *SAN, "-I", os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests", "native", "oracle_asan_main.c"), os.path.join(ROOT, "oracle", "bmfr_oracle.c"),
          "-lm", "-o", exe])
    out = _run([exe])
    assert out.count("checksum") == 4, out


def _hostile(tmp_path, W=9, H=5):
    """Hand-made headers whose fields point past the file or overflow."""
    chl = b"".join(n + b"\0" + struct.pack("<iIii", 2, 0, 1, 1) for n in (b"B", b"G", b"R")) + b"\0"

    def hdr(box=(0, 0, W - 1, H - 1), comp=b"\0", extra=b""):
        return (struct.pack("<II", 20000630, 2) + _attr("channels", "chlist", chl) +
                _attr("compression", "compression", comp) + _attr("dataWindow", "box2i", struct.pack("<iiii", *box)) +
                _attr("lineOrder", "lineOrder", b"\0") + extra + b"\0")

    files = {
        "offset_near_2_64": hdr() + struct.pack("<Q", 2 ** 64 - 4) * H,
        "offset_past_end": hdr() + struct.pack("<Q", 10 ** 9) * H,
        "chunk_size_huge": None,
        "empty_compression": hdr(comp=b""),
        "window_overflow": hdr(box=(-2 ** 31, -2 ** 31, 2 ** 31 - 1, 2 ** 31 - 1)),
        "window_huge": hdr(box=(0, 0, 2 ** 30, 2 ** 30)),
        "attr_size_past_end": struct.pack("<II", 20000630, 2) + b"channels\0chlist\0" + struct.pack("<i", 2 ** 31 - 1),
        "attr_size_negative": struct.pack("<II", 20000630, 2) + b"channels\0chlist\0" + struct.pack("<i", -8),
        "no_terminator": struct.pack("<II", 20000630, 2) + b"channels",
        "empty": b"",
    }
    h = hdr()
    first = len(h) + 8 * H
    files["chunk_size_huge"] = h + struct.pack("<Q", first) * H + struct.pack("<ii", 0, 2 ** 31 - 1)
    out = []
    for name, data in files.items():
        p = tmp_path / f"hostile_{name}.exr"
        p.write_bytes(data)
        out.append(str(p))
    return out


def test_exr_reader_malformed_corpus_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "exr_fuzz")
    _run(["g++", "-std=c++17", *SAN, "-I", os.path.join(ROOT, "host"),
          os.path.join(ROOT, "tests", "native", "exr_fuzz_main.cpp"), os.path.join(ROOT, "host", "image_io.cpp"),
          "-lz", "-o", exe])
    img = _img(H=7, W=11)
    corpus = []
    rng = np.random.default_rng(0x424D4652)
    for comp, half, tile in ((0, False, None), (1, False, None), (2, True, None), (3, False, None),
                             (4, False, None), (4, True, None), (5, False, None), (5, True, None),
                             (6, True, None), (7, True, None), (7, True, (4, 4)),
                             (3, False, (4, 4)), (4, False, (8, 2)), (5, False, (4, 4)),
                             (8, True, None), (9, True, None), (8, True, (16, 16)), (-8, True, None),
                             (9, False, None)):
        name = f"{comp}_{int(half)}" + (f"_t{tile[0]}x{tile[1]}" if tile else "")
        src = tmp_path / f"valid_{name}.exr"
        if abs(comp) >= 8:  # DWA: an image the codec shrinks (tiny noisy ones are stored raw); -8: deflated AC;
            # (9, False): FLOAT R, G, B under the FLOAT LOSSY_DCT rules (decoded as halves, widened)
            r, g, b = _dwa_image(24, 40, 3)
            chans = {"R": r, "G": g, "B": b, "A": np.full(r.shape, 0.5, np.float32), "Z": r * 10}
            types = {"Z": False} if half else {"R": False, "G": False, "B": False, "Z": False}
            DWA_OPTS.update(ac_mode=int(comp < 0))
            if not half:
                DWA_OPTS.update(rules=exr_dwa_py.DEFAULT_RULES_FLOAT)
            try:
                write_exr_py(str(src), chans, abs(comp), half=True, tile=tile, types=types)
            finally:
                DWA_OPTS.update(ac_mode=0)
                DWA_OPTS.pop("rules", None)
        else:
            write_exr_py(str(src), {"R": img[..., 0], "G": img[..., 1], "B": img[..., 2]}, comp, half=half, tile=tile)
        data = src.read_bytes()
        corpus.append(str(src))
        for n in range(0, len(data), max(1, len(data) // 97)):  # truncations
            p = tmp_path / f"trunc_{name}_{n}.exr"
            p.write_bytes(data[:n])
            corpus.append(str(p))
        for k in range(120):  # 1..8 corrupted bytes anywhere
            b = bytearray(data)
            for i in rng.integers(0, len(b), rng.integers(1, 9)):
                b[i] = int(rng.integers(0, 256))
            p = tmp_path / f"flip_{name}_{k}.exr"
            p.write_bytes(bytes(b))
            corpus.append(str(p))
    hostile = _hostile(tmp_path)
    # a DWA file whose lossy G channel carries the pLinear flag: refused
    src = tmp_path / "valid_8_1.exr"
    b = bytearray(src.read_bytes())
    i = b.index(b"G\0", b.index(b"chlist"))
    b[i + 2 + 4] = 1
    (tmp_path / "dwa_plinear.exr").write_bytes(bytes(b))
    hostile.append(str(tmp_path / "dwa_plinear.exr"))
    out = _run([exe, *corpus, *hostile])
    assert f"files {len(corpus) + len(hostile)}" in out, out
    # every hostile file is rejected, every valid one read
    out_h = _run([exe, *hostile])
    assert f"rejected {len(hostile)}" in out_h, out_h
    out_v = _run([exe, *[c for c in corpus if "valid_" in c]])
    assert "rejected 0" in out_v, out_v
