"""EXR / PNG I/O of the host (host/image_io.cpp), checked
against an independent numpy + zlib implementation of the same published
formats written here: OpenEXR 2 scanline and tiled files (HALF / FLOAT
channels, NONE / RLE / ZIPS / ZIP / PXR24 / B44 / B44A compression, PIZ
through the independent encoder tests/exr_piz_py.py and DWAA / DWAB through
tests/exr_dwa_py.py; one-level and mip-mapped tiles) and
8-bit RGB PNG.  EXR parity is unpinned: no OpenEXR library and no reference
.exr file exist here, so the reader is only as right as these encoders'
reading of the published format."""
from __future__ import annotations

import ctypes as C
import os
import struct
import zlib

import numpy as np
import pytest

from bmfr_amd import _build
import exr_dwa_py
import exr_piz_py
from exr_piz_py import piz_compress

LIB = None


def lib():
    global LIB
    if LIB is None:
        _build.build_host()
        LIB = C.CDLL(_build.IO_LIB)
        LIB.bmfr_exr_info.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        LIB.bmfr_exr_read_rgb.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p]
        LIB.bmfr_exr_write_rgb.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t, C.c_int]
        LIB.bmfr_png_write_rgb.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t]
        LIB.bmfr_io_error.restype = C.c_char_p
    return LIB


# ---------------------------------------------------- reference encoder ----
def _attr(name, typ, data):
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def _predict(raw: bytes) -> bytes:
    a = np.frombuffer(raw, np.uint8)
    t = np.concatenate([a[0::2], a[1::2]]).astype(np.int32)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128 + 256) & 255
    return d.astype(np.uint8).tobytes()


def _rle(data: bytes) -> bytes:
    out, i, n = bytearray(), 0, len(data)
    while i < n:
        j = i
        while j < n and j - i < 127 and data[j] == data[i]:
            j += 1
        if j - i >= 3:
            out += struct.pack("b", j - i - 1) + data[i:i + 1]
            i = j
        else:
            k = i
            while k < n and k - i < 127 and not (k + 2 < n and data[k] == data[k + 1] == data[k + 2]):
                k += 1
            out += struct.pack("b", -(k - i)) + data[i:k]
            i = k
    return bytes(out)


def f24(a: np.ndarray) -> np.ndarray:
    """PXR24's float -> 24-bit conversion (published OpenEXR scheme): the top
    24 bits of the float, rounded half up in the mantissa, not rounding into
    infinity; NaN stays NaN."""
    i = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.int64)
    s, e, m = i & 0x80000000, i & 0x7f800000, i & 0x007fffff
    r = ((e | m) + (m & 0x80)) >> 8
    r = np.where(r >= 0x7f8000, (e | m) >> 8, r)
    m8 = m >> 8
    special = np.where(m != 0, (e >> 8) | m8 | (m8 == 0), e >> 8)
    return (np.where(e == 0x7f800000, special, r) | (s >> 8)).astype(np.int64)


def f24_values(a: np.ndarray) -> np.ndarray:
    """What a PXR24 FLOAT sample decodes to: the 24 bits, low byte zero."""
    return (f24(a) << 8).astype(np.uint32).view(np.float32).reshape(np.shape(a))


def _pxr24(img, names, y0, lines, x0, w, half):
    """One PXR24 chunk: per line and channel, sample differences split into
    byte planes (most significant first), deflated."""
    out = bytearray()
    for y in range(y0, y0 + lines):
        for n in names:
            row = np.ascontiguousarray(img[n][y, x0:x0 + w])
            if half:
                v = row.astype(np.float16).view(np.uint16).astype(np.int64)
                nb = 2
            else:
                v = f24(row)
                nb = 3
            d = np.diff(np.concatenate([[0], v])) & 0xffffffff
            for k in range(nb):
                out += ((d >> (8 * (nb - 1 - k))) & 255).astype(np.uint8).tobytes()
    return zlib.compress(bytes(out))


def _b44_shift_round(x, shift):
    """B44's x / 2^shift rounded to nearest, ties to even (published OpenEXR scheme)."""
    x = x << 1
    a = (1 << shift) - 1
    b = (x >> (shift + 1)) & 1
    return (x + a + b) >> (shift + 1)


def _b44_ordered(h16: np.ndarray) -> np.ndarray:
    """Half bit patterns -> B44's ordered 16-bit codes (inf / NaN -> 0x8000)."""
    h = h16.astype(np.int64)
    t = np.where(h & 0x8000, (~h) & 0xffff, h | 0x8000)
    return np.where((h & 0x7c00) == 0x7c00, 0x8000, t)


def _b44_block(s: np.ndarray, flat: bool):
    """One 4x4 block (16 half bit patterns, row-major) -> (bytes, decoded bit
    patterns).  The decoded block in closed form: t_max - (d_i << shift)."""
    t = _b44_ordered(s)
    tmax = int(t.max())
    bias = 0x20
    shift = -1
    while True:
        shift += 1
        d = np.array([_b44_shift_round(tmax - int(v), shift) for v in t])
        r = [d[0] - d[4], d[4] - d[8], d[8] - d[12],
             d[0] - d[1], d[4] - d[5], d[8] - d[9], d[12] - d[13],
             d[1] - d[2], d[5] - d[6], d[9] - d[10], d[13] - d[14],
             d[2] - d[3], d[6] - d[7], d[10] - d[11], d[14] - d[15]]
        r = [int(v) + bias for v in r]
        if min(r) >= 0 and max(r) <= 0x3f:
            break
    if flat and min(r) == bias and max(r) == bias:
        t0 = int(t[0])
        dec = np.full(16, t0, np.int64)
        out = bytes([t0 >> 8, t0 & 255, 0xfc])
    else:
        t0 = (tmax - (int(d[0]) << shift)) & 0xffff
        dec = (tmax - (d.astype(np.int64) << shift)) & 0xffff
        b = [t0 >> 8, t0 & 255, (shift << 2) | (r[0] >> 4), (r[0] << 4) | (r[1] >> 2), (r[1] << 6) | r[2],
             (r[3] << 2) | (r[4] >> 4), (r[4] << 4) | (r[5] >> 2), (r[5] << 6) | r[6],
             (r[7] << 2) | (r[8] >> 4), (r[8] << 4) | (r[9] >> 2), (r[9] << 6) | r[10],
             (r[11] << 2) | (r[12] >> 4), (r[12] << 4) | (r[13] >> 2), (r[13] << 6) | r[14]]
        out = bytes(v & 255 for v in b)
    dec = np.where(dec & 0x8000, dec & 0x7fff, (~dec) & 0xffff)  # ordered code -> half bits
    return out, dec.astype(np.uint16), shift


B44_DECODED = {}  # channel -> {(y0, x0): half bit patterns of the chunk as B44 decodes it}
B44_SHIFTS = []   # shift of every block written (-1: a B44A flat block)


def _b44(img, names, y0, lines, x0, w, half, flat, types):
    """One B44 / B44A chunk: channel after channel over the chunk; HALF
    channels as 4x4 blocks (edge blocks padded by repeating the last row /
    column), other channels raw."""
    out = bytearray()
    for n in names:
        a = np.ascontiguousarray(img[n][y0:y0 + lines, x0:x0 + w])
        if not types.get(n, half):
            out += a.astype(np.float32).tobytes()
            continue
        h = a.astype(np.float16).view(np.uint16)
        ph, pw = (lines + 3) // 4 * 4, (w + 3) // 4 * 4
        hp = np.pad(h, ((0, ph - lines), (0, pw - w)), mode="edge")
        dec = np.zeros((ph, pw), np.uint16)
        for by in range(0, ph, 4):
            for bx in range(0, pw, 4):
                blk, d, sh = _b44_block(hp[by:by + 4, bx:bx + 4].reshape(16), flat)
                B44_SHIFTS.append(-1 if len(blk) == 3 else sh)  # -1: a 3-byte flat block
                out += blk
                dec[by:by + 4, bx:bx + 4] = d.reshape(4, 4)
        B44_DECODED.setdefault(n, {})[(y0, x0)] = dec[:lines, :w]
    return bytes(out)


RAW_CHUNKS = []  # (level, y0, lines, x0, w) of the chunks write_exr_py stored uncompressed
DWA_DECODED = {}  # channel -> {(y0, x0): the chunk's samples as a DWA decoder produces them}
DWA_OPTS = {"version": 2, "ac_mode": 0, "drop": 0.02}  # DWA chunks' form (exr_dwa_py.dwa_compress)


def _chunk_data(img, names, dt, compression, y0, lines, x0, w, half, level=0, types=None):
    types = types or {}
    raw = b"".join(np.ascontiguousarray(img[n][y, x0:x0 + w]).astype(
        (np.float16 if types[n] else np.float32) if n in types else dt).tobytes()
                   for y in range(y0, y0 + lines) for n in names)
    if compression == 1:
        data = _rle(_predict(raw))
    elif compression in (2, 3):
        data = zlib.compress(_predict(raw))
    elif compression == 4:
        data = piz_compress(raw, w, lines, [1 if half else 2] * len(names))
    elif compression == 5:
        data = _pxr24(img, names, y0, lines, x0, w, half)
    elif compression in (6, 7):
        data = _b44(img, names, y0, lines, x0, w, half, compression == 7, types)
    elif compression in (8, 9):
        ptypes = {n: (1 if types.get(n, half) else 2) for n in names}
        data, dec = exr_dwa_py.dwa_compress({n: img[n][y0:y0 + lines, x0:x0 + w] for n in names}, ptypes, lines, w,
                                            **DWA_OPTS)
        for n in names:
            DWA_DECODED.setdefault(n, {})[(y0, x0)] = dec[n]
    else:
        data = raw
    if compression and len(data) >= len(raw):  # OpenEXR stores such a chunk as it is
        RAW_CHUNKS.append((level, y0, lines, x0, w))
        return raw
    return data


def write_exr_py(path, img: dict, compression: int, half: bool, tile=None, mipmap=False, types=None):
    """img: channel name -> (H, W) float array.  Channels are stored sorted by
    name.  compression 0 NONE, 1 RLE, 2 ZIPS, 3 ZIP, 4 PIZ, 5 PXR24, 6 B44,
    7 B44A, 8 DWAA, 9 DWAB.  types: channel name -> True (HALF) / False
    (FLOAT) where it differs from `half` (B44 / DWA chunks only).
    tile = (tw, th): a tiled file (ONE_LEVEL, or MIPMAP_LEVELS round-down
    with mipmap=True: the lower levels follow level 0, box-filtered)."""
    names = sorted(img)
    H, W = img[names[0]].shape
    ptype, dt = (1, np.float16) if half else (2, np.float32)
    types = types or {}
    chl = b"".join(n.encode() + b"\0" + struct.pack("<iIii", (1 if types[n] else 2) if n in types else ptype, 0, 1, 1)
                   for n in names) + b"\0"
    box = struct.pack("<iiii", 0, 0, W - 1, H - 1)
    version = 2 | (0x200 if tile else 0)
    hdr = (struct.pack("<II", 20000630, version) + _attr("channels", "chlist", chl) +
           _attr("compression", "compression", bytes([compression])) + _attr("dataWindow", "box2i", box) +
           _attr("displayWindow", "box2i", box) + _attr("lineOrder", "lineOrder", b"\0") +
           _attr("pixelAspectRatio", "float", struct.pack("<f", 1)) +
           _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0, 0)) +
           _attr("screenWindowWidth", "float", struct.pack("<f", 1)))
    if tile:
        hdr += _attr("tiles", "tiledesc", struct.pack("<IIB", tile[0], tile[1], 1 if mipmap else 0))
    hdr += b"\0"
    chunks = []
    if tile:
        tw, th = tile
        levels = [img]
        while mipmap and max(levels[-1][names[0]].shape) > 1:
            h2, w2 = (max(1, d // 2) for d in levels[-1][names[0]].shape)
            levels.append({n: levels[-1][n][:2 * h2:2, :2 * w2:2][:h2, :w2] for n in names})
        for lv, im in enumerate(levels):
            lh, lw = im[names[0]].shape
            for ty in range((lh + th - 1) // th):
                for tx in range((lw + tw - 1) // tw):
                    x0, y0 = tx * tw, ty * th
                    w, lines = min(tw, lw - x0), min(th, lh - y0)
                    data = _chunk_data(im, names, dt, compression, y0, lines, x0, w, half, lv, types)
                    chunks.append(struct.pack("<iiiii", tx, ty, lv, lv, len(data)) + data)
    else:
        lpc = {0: 1, 1: 1, 2: 1, 3: 16, 4: 32, 5: 16, 6: 32, 7: 32, 8: 32, 9: 256}[compression]
        for y0 in range(0, H, lpc):
            data = _chunk_data(img, names, dt, compression, y0, min(H, y0 + lpc) - y0, 0, W, half, types=types)
            chunks.append(struct.pack("<ii", y0, len(data)) + data)
    off = len(hdr) + 8 * len(chunks)
    table = b""
    for c in chunks:
        table += struct.pack("<Q", off)
        off += len(c)
    with open(path, "wb") as f:
        f.write(hdr + table + b"".join(chunks))


def read_exr_py(path):
    """Independent decoder for the FLOAT/NONE/ZIP files the host writes."""
    b = open(path, "rb").read()
    assert struct.unpack_from("<I", b, 0)[0] == 20000630
    p, attrs = 8, {}
    while b[p]:
        e = b.index(b"\0", p)
        name = b[p:e].decode()
        e2 = b.index(b"\0", e + 1)
        size = struct.unpack_from("<i", b, e2 + 1)[0]
        attrs[name] = b[e2 + 5:e2 + 5 + size]
        p = e2 + 5 + size
    p += 1
    x0, y0, x1, y1 = struct.unpack("<iiii", attrs["dataWindow"])
    W, H = x1 - x0 + 1, y1 - y0 + 1
    comp = attrs["compression"][0]
    lpc = 16 if comp == 3 else 1
    n_chunks = (H + lpc - 1) // lpc
    offs = struct.unpack_from(f"<{n_chunks}Q", b, p)
    out = np.zeros((H, W, 3), np.float32)
    for o in offs:
        y, size = struct.unpack_from("<ii", b, o)
        data = b[o + 8:o + 8 + size]
        lines = min(lpc, H - y)
        raw_size = lines * W * 12
        if size < raw_size:
            t = np.frombuffer(zlib.decompress(data), np.uint8).astype(np.int64)
            t = (t[0] + np.concatenate([[0], np.cumsum(t[1:] - 128)])) & 255  # undo the delta predictor
            half = (len(t) + 1) // 2
            r = np.empty(len(t), np.uint8)
            r[0::2] = t[:half]
            r[1::2] = t[half:]
            data = r.tobytes()
        a = np.frombuffer(data, np.float32).reshape(lines, 3, W)  # B, G, R
        out[y:y + lines] = a[:, ::-1, :].transpose(0, 2, 1)
    return out


def read_png_py(path):
    b = open(path, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    p, idat, W = 8, b"", 0
    while p < len(b):
        n = struct.unpack(">I", b[p:p + 4])[0]
        typ, data = b[p + 4:p + 8], b[p + 8:p + 8 + n]
        assert zlib.crc32(typ + data) == struct.unpack(">I", b[p + 8 + n:p + 12 + n])[0]
        if typ == b"IHDR":
            W, H, depth, ctype = struct.unpack(">IIBB", data[:10])
            assert (depth, ctype) == (8, 2)
        elif typ == b"IDAT":
            idat += data
        p += 12 + n
    rows = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(H, 1 + 3 * W)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(H, W, 3)


def _img(H=37, W=53, seed=1):
    rng = np.random.default_rng(seed)
    img = rng.normal(0, 3, (H, W, 3)).astype(np.float32)
    img[0, 0] = [np.inf, -0.0, 65504.0]
    img[1, :5, 0] = 0.25  # runs for RLE
    img[2, :] = 1.0
    return img


# ------------------------------------------------------------------ tests --
@pytest.mark.parametrize("comp", [0, 3])
def test_exr_write_read_roundtrip(tmp_path, comp):
    img = _img()
    H, W, _ = img.shape
    path = str(tmp_path / f"rt{comp}.exr").encode()
    assert lib().bmfr_exr_write_rgb(path, W, H, img.ctypes.data, W * 3, comp) == 0, lib().bmfr_io_error()
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    assert lib().bmfr_exr_info(path, C.byref(w), C.byref(h), C.byref(c)) == 0
    assert (w.value, h.value, c.value) == (W, H, 3)
    back = np.empty_like(img)
    assert lib().bmfr_exr_read_rgb(path, W, H, back.ctypes.data) == 0, lib().bmfr_io_error()
    assert back.tobytes() == img.tobytes()
    # an independent decoder reads the same values
    assert read_exr_py(path.decode()).tobytes() == img.tobytes()


@pytest.mark.parametrize("comp", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("half", [False, True])
def test_exr_reader_against_reference_encoder(tmp_path, comp, half):
    img = _img(41, 29, seed=comp + 7 * half)
    chans = {"R": img[..., 0], "G": img[..., 1], "B": img[..., 2], "A": np.ones(img.shape[:2], np.float32)}
    path = str(tmp_path / f"ref{comp}{int(half)}.exr")
    write_exr_py(path, chans, comp, half)
    H, W, _ = img.shape
    out = np.empty_like(img)
    assert lib().bmfr_exr_read_rgb(path.encode(), W, H, out.ctypes.data) == 0, lib().bmfr_io_error()
    want = img.astype(np.float16).astype(np.float32) if half else img
    np.testing.assert_array_equal(out, want)


def test_exr_errors(tmp_path):
    p = tmp_path / "bad.exr"
    p.write_bytes(b"not an exr file at all")
    out = np.empty(3, np.float32)
    assert lib().bmfr_exr_read_rgb(str(p).encode(), 1, 1, out.ctypes.data) != 0
    assert b"OpenEXR" in lib().bmfr_io_error()
    img = _img(8, 8)
    path = str(tmp_path / "wrongsize.exr").encode()
    assert lib().bmfr_exr_write_rgb(path, 8, 8, img.ctypes.data, 24, 0) == 0
    big = np.empty((9, 8, 3), np.float32)
    assert lib().bmfr_exr_read_rgb(path, 8, 9, big.ctypes.data) != 0


def test_png_quantisation(tmp_path):
    img = _img(23, 31)
    img[3, 3] = [np.nan, 0.5, 1.5]
    H, W, _ = img.shape
    path = str(tmp_path / "o.png").encode()
    assert lib().bmfr_png_write_rgb(path, W, H, img.ctypes.data, W * 3) == 0, lib().bmfr_io_error()
    got = read_png_py(path.decode())
    want = np.floor(np.clip(np.nan_to_num(img, nan=0.0), 0, 1) * 255 + 0.5).astype(np.uint8)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("shape", [(1, 1), (33, 70), (7, 300), (64, 5), (40, 300)])
@pytest.mark.parametrize("half", [False, True])
def test_exr_piz_shapes(tmp_path, shape, half):
    """PIZ: partial last chunks, one-pixel and very wide / narrow images (odd
    wavelet rows / columns at every level), smooth data (14-bit wavelet,
    long runs) and noise (16-bit wavelet: many distinct words)."""
    H, W = shape
    rng = np.random.default_rng(H * 1000 + W)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    smooth = (np.sin(xx / 9.0) + yy / 50.0).astype(np.float32)
    img = np.stack([smooth, rng.normal(0, 10, (H, W)).astype(np.float32), np.zeros((H, W), np.float32)], -1)
    img[:, :, 2][::3] = 0.5  # runs
    chans = {"R": img[..., 0], "G": img[..., 1], "B": img[..., 2]}
    path = str(tmp_path / "piz.exr")
    exr_piz_py.MAX_VALUES.clear()
    write_exr_py(path, chans, 4, half)
    if shape == (40, 300) and not half:  # both wavelet forms: the first chunk 16-bit, the 8-line tail 14-bit
        assert max(exr_piz_py.MAX_VALUES) >= 1 << 14 and min(exr_piz_py.MAX_VALUES) < 1 << 14
    out = np.empty_like(img)
    assert lib().bmfr_exr_read_rgb(path.encode(), W, H, out.ctypes.data) == 0, lib().bmfr_io_error()
    want = img.astype(np.float16).astype(np.float32) if half else img
    np.testing.assert_array_equal(out, want)


@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("shape", [(41, 29), (16, 16), (1, 70), (33, 1)])
def test_exr_pxr24(tmp_path, shape, half):
    """PXR24 (OpenImageIO reads it, bmfr.cpp:145-163): lossless for HALF,
    FLOAT samples rounded to 24 bits (f24_values); partial 16-line chunks."""
    H, W = shape
    img = np.random.default_rng(H + W).normal(0, 3, (H, W, 3)).astype(np.float32)
    img[0, 0] = [np.inf, -0.0, np.float32(1.0 + 2 ** -16)]  # the dropped byte's top bit: rounds up
    img[-1, -1] = [np.nan, 65504.0, np.float32(3.4028235e38)]  # NaN; no rounding into infinity
    chans = {"R": img[..., 0], "G": img[..., 1], "B": img[..., 2]}
    path = str(tmp_path / "pxr24.exr")
    RAW_CHUNKS.clear()
    write_exr_py(path, chans, 5, half)
    out = np.empty_like(img)
    assert lib().bmfr_exr_read_rgb(path.encode(), W, H, out.ctypes.data) == 0, lib().bmfr_io_error()
    want = img.astype(np.float16).astype(np.float32) if half else f24_values(img)
    for _, y0, n, x0, w in RAW_CHUNKS if not half else []:  # FLOAT chunks stored uncompressed: exact
        want[y0:y0 + n, x0:x0 + w] = img[y0:y0 + n, x0:x0 + w]
    np.testing.assert_array_equal(out, want)


@pytest.mark.parametrize("comp", [0, 1, 3, 4, 5])
@pytest.mark.parametrize("tile,mipmap", [((16, 16), False), ((32, 8), False), ((64, 64), False),
                                         ((16, 16), True)])
def test_exr_tiled(tmp_path, comp, tile, mipmap):
    """Tiled single-part files (renderer output): partial edge tiles, a tile
    larger than the image, and a mip map whose full-resolution level is read."""
    img = _img(37, 53, seed=comp)
    chans = {"R": img[..., 0], "G": img[..., 1], "B": img[..., 2], "A": np.ones(img.shape[:2], np.float32)}
    path = str(tmp_path / "tiled.exr")
    RAW_CHUNKS.clear()
    write_exr_py(path, chans, comp, False, tile=tile, mipmap=mipmap)
    H, W, _ = img.shape
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    assert lib().bmfr_exr_info(path.encode(), C.byref(w), C.byref(h), C.byref(c)) == 0
    assert (w.value, h.value, c.value) == (W, H, 4)
    out = np.empty_like(img)
    assert lib().bmfr_exr_read_rgb(path.encode(), W, H, out.ctypes.data) == 0, lib().bmfr_io_error()
    want = f24_values(img) if comp == 5 else img.copy()
    for lv, y0, n, x0, w in RAW_CHUNKS:  # level-0 tiles stored uncompressed are exact
        if lv == 0:
            want[y0:y0 + n, x0:x0 + w] = img[y0:y0 + n, x0:x0 + w]
    np.testing.assert_array_equal(out, want)


def test_exr_tiled_rejects_bad_tiles(tmp_path):
    """A tiled file without a tile description, or a tile of another level
    where level (0, 0) is expected, is rejected with a message."""
    img = _img(8, 8)
    chans = {"R": img[..., 0], "G": img[..., 1], "B": img[..., 2]}
    path = tmp_path / "t.exr"
    write_exr_py(str(path), chans, 0, False, tile=(4, 4))
    data = path.read_bytes()
    i = data.index(b"tiles\0tiledesc\0")
    no_desc = data[:i] + b"tileX\0" + data[i + 6:]  # attribute renamed: no tile description
    out = np.empty_like(img)
    (tmp_path / "nodesc.exr").write_bytes(no_desc)
    assert lib().bmfr_exr_read_rgb(str(tmp_path / "nodesc.exr").encode(), 8, 8, out.ctypes.data) != 0
    assert b"tile" in lib().bmfr_io_error()
    # the first tile's level x -> 1
    p = 8
    while data[p]:  # attributes: name, type, size, value
        e2 = data.index(b"\0", data.index(b"\0", p) + 1)
        p = e2 + 5 + struct.unpack_from("<i", data, e2 + 1)[0]
    first = struct.unpack_from("<Q", data, p + 1)[0]  # the offset table follows the terminating null
    b = bytearray(data)
    struct.pack_into("<i", b, first + 8, 1)
    (tmp_path / "level.exr").write_bytes(bytes(b))
    assert lib().bmfr_exr_read_rgb(str(tmp_path / "level.exr").encode(), 8, 8, out.ctypes.data) != 0
    assert b"bad tile" in lib().bmfr_io_error()


def _b44_want(shape, chunks_of, names):
    """The decoded image of B44_DECODED's chunks, as float32, (H, W) per channel."""
    H, W = shape
    out = {}
    for n in names:
        a = np.zeros((H, W), np.uint16)
        for (y0, x0), d in B44_DECODED[n].items():
            a[y0:y0 + d.shape[0], x0:x0 + d.shape[1]] = d
        out[n] = a.view(np.float16).astype(np.float32)
    return out


@pytest.mark.parametrize("comp", [6, 7])
@pytest.mark.parametrize("shape,tile", [((41, 29), None), ((32, 32), None), ((3, 70), None), ((70, 2), None),
                                        ((37, 53), (16, 8))])
def test_exr_b44(tmp_path, comp, shape, tile):
    """B44 / B44A (OpenImageIO reads them, bmfr.cpp:145-163): HALF channels in
    4x4 blocks -- lossless where a block's samples differ little (shift 0),
    rounded to 2^shift steps below the block maximum elsewhere (the closed
    form t_max - (d << shift) of the published scheme, independent of the
    decoder's running sums), flat blocks in 3 bytes (B44A), partial edge
    blocks; a FLOAT channel in the same chunk is stored raw."""
    H, W = shape
    rng = np.random.default_rng(H * W + comp)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    img = np.stack([1.0 + xx / 512.0,                                  # smooth: shift 0, lossless
                    rng.normal(0, 3, (H, W)).astype(np.float32),      # noise: lossy blocks
                    np.where(yy < H // 8 * 4, 0.5, -2.0).astype(np.float32)], -1)  # flat blocks
    img[0, 0, 1] = np.inf
    img[-1, -1, 1] = -0.0
    chans = {"R": img[..., 0], "G": img[..., 1], "B": img[..., 2], "A": rng.normal(0, 1, (H, W)).astype(np.float32)}
    types = {"A": False}
    path = str(tmp_path / "b44.exr")
    B44_DECODED.clear()
    B44_SHIFTS.clear()
    RAW_CHUNKS.clear()
    write_exr_py(path, chans, comp, True, tile=tile, types=types)
    out = np.empty_like(img)
    assert lib().bmfr_exr_read_rgb(path.encode(), W, H, out.ctypes.data) == 0, lib().bmfr_io_error()
    want = _b44_want((H, W), B44_DECODED, "RGB")
    for _, y0, n, x0, w in RAW_CHUNKS:  # chunks B44 would not shrink are stored as they are
        for c, ch in enumerate("RGB"):
            want[ch][y0:y0 + n, x0:x0 + w] = img[y0:y0 + n, x0:x0 + w, c].astype(np.float16)
    np.testing.assert_array_equal(out[..., 0], want["R"])
    np.testing.assert_array_equal(out[..., 1], want["G"])
    np.testing.assert_array_equal(out[..., 2], want["B"])
    # lossless where the scheme is: smooth and flat channels
    np.testing.assert_array_equal(out[..., 0], img[..., 0].astype(np.float16).astype(np.float32))
    np.testing.assert_array_equal(out[..., 2], img[..., 2].astype(np.float16).astype(np.float32))
    # the noisy channel: lossy, each sample within half a step (2^shift of the
    # ordered code) of its own -- measured in the ordered code, where the
    # scheme rounds
    g = img[..., 1].astype(np.float16)
    fin = np.isfinite(g)
    code = lambda a: _b44_ordered(a.view(np.uint16))  # noqa: E731
    err = np.abs(code(out[..., 1].astype(np.float16))[fin] - code(g)[fin])
    assert err.max() <= 1 << (max(B44_SHIFTS) - 1)
    assert err.max() > 0 or RAW_CHUNKS
    assert (-1 in B44_SHIFTS) == (comp == 7)  # 3-byte flat blocks: B44A only


def test_exr_b44_rejects_plinear(tmp_path):
    img = _img(8, 8)
    chans = {"R": img[..., 0], "G": img[..., 1], "B": img[..., 2]}
    path = tmp_path / "lin.exr"
    write_exr_py(str(path), chans, 6, True)
    b = bytearray(path.read_bytes())
    i = b.index(b"R\0", b.index(b"chlist"))
    b[i + 2 + 4] = 1  # R's pLinear flag
    path.write_bytes(bytes(b))
    out = np.empty_like(img)
    assert lib().bmfr_exr_read_rgb(str(path).encode(), 8, 8, out.ctypes.data) != 0
    assert b"pLinear" in lib().bmfr_io_error()


def _dwa_image(H, W, seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    r = 0.5 + 0.4 * np.sin(xx / 7.0) * np.cos(yy / 5.0)                       # smooth, below 1
    g = np.abs(0.3 + 0.1 * np.sin(yy / 3.0) + rng.normal(0, 0.03, (H, W))).astype(np.float32)  # noise
    b = (1.0 + 30.0 * (xx + yy) / (W + H)).astype(np.float32)                 # above 1: the log branch
    b[::5, ::3] *= -1.0                                                      # negative samples
    g[0, 0] = np.inf                                                          # non-finite -> 0 on the codec's scale
    return r.astype(np.float32), g, b


def _dwa_want(shape, names, raw_img, types):
    """The decoded R, G, B of DWA_DECODED's chunks (HALF channels: half bit
    patterns; FLOAT: the samples), raw chunks as stored, as float32."""
    H, W = shape
    out = {}
    for n in names:
        half = types.get(n, True)
        a = np.zeros((H, W), np.uint16 if half else np.float32)
        for (y0, x0), d in DWA_DECODED[n].items():
            a[y0:y0 + d.shape[0], x0:x0 + d.shape[1]] = d
        out[n] = a.view(np.float16).astype(np.float32) if half else a
    for _, y0, ln, x0, w in RAW_CHUNKS:  # chunks DWA would not shrink are stored as they are
        for n in names:
            v = raw_img[n][y0:y0 + ln, x0:x0 + w]
            out[n][y0:y0 + ln, x0:x0 + w] = v.astype(np.float16).astype(np.float32) if types.get(n, True) else v
    return out


@pytest.mark.parametrize("comp", [8, 9])
@pytest.mark.parametrize("shape,tile", [((41, 29), None), ((300, 21), None), ((3, 9), None), ((67, 53), (32, 16))])
@pytest.mark.parametrize("version,ac_mode", [(2, 0), (2, 1), (1, 0)])
def test_exr_dwa(tmp_path, comp, shape, tile, version, ac_mode):
    """DWAA / DWAB (OpenImageIO reads them, bmfr.cpp:145-163): an R, G, B set
    of HALF channels through the lossy DCT with the colour transform, an
    alpha (RLE) and a FLOAT depth channel (UNKNOWN) in the same chunks,
    static-Huffman and deflated AC terms, version-2 rules and version 1's
    fixed set, partial 8x8 blocks and partial chunks (DWAB: 256 lines), tiles.
    Bit for bit against the decode exr_dwa_py.py predicts from the
    coefficients it wrote; and close to the input (the codec is lossy)."""
    H, W = shape
    r, g, b = _dwa_image(H, W, H * W + comp)
    chans = {"R": r, "G": g, "B": b, "A": np.full((H, W), 0.5, np.float32), "Z": (r * 100).astype(np.float32)}
    types = {"Z": False}
    path = str(tmp_path / "dwa.exr")
    DWA_DECODED.clear()
    RAW_CHUNKS.clear()
    DWA_OPTS.update(version=version, ac_mode=ac_mode, drop=0.02)
    try:
        write_exr_py(path, chans, comp, True, tile=tile, types=types)
    finally:
        DWA_OPTS.update(version=2, ac_mode=0, drop=0.02)
    out = np.empty((H, W, 3), np.float32)
    assert lib().bmfr_exr_read_rgb(path.encode(), W, H, out.ctypes.data) == 0, lib().bmfr_io_error()
    want = _dwa_want((H, W), "RGB", chans, types)
    for c, n in enumerate("RGB"):
        np.testing.assert_array_equal(out[..., c], want[n], err_msg=n)
    # lossy, but close: relative error on the finite samples
    for c, src in enumerate((r, g, b)):
        fin = np.isfinite(src)
        err = np.abs(out[..., c][fin] - src[fin]) / np.maximum(np.abs(src[fin]), 0.05)
        assert np.median(err) < 0.05, (c, np.median(err))
    assert len(RAW_CHUNKS) < len(DWA_DECODED["R"]) or H * W < 64  # DWA-coded chunks (tiny images: stored)


def test_exr_dwa_partial_colour_set(tmp_path):
    """R and G without a HALF B (here FLOAT: an UNKNOWN channel) form no
    colour set: each is its own lossy decoder, no colour transform."""
    H, W = 20, 19
    r, g, b = _dwa_image(H, W, 5)
    chans = {"R": r, "G": g, "B": b}
    types = {"B": False}
    path = str(tmp_path / "dwa_rg.exr")
    DWA_DECODED.clear()
    RAW_CHUNKS.clear()
    write_exr_py(path, chans, 8, True, types=types)
    out = np.empty((H, W, 3), np.float32)
    assert lib().bmfr_exr_read_rgb(path.encode(), W, H, out.ctypes.data) == 0, lib().bmfr_io_error()
    want = _dwa_want((H, W), "RGB", chans, types)
    for c, n in enumerate("RGB"):
        np.testing.assert_array_equal(out[..., c], want[n], err_msg=n)
    np.testing.assert_array_equal(out[..., 2], b)  # UNKNOWN: lossless


def test_exr_dwa_float_lossy_channels(tmp_path):
    """FLOAT R, G, B under OpenEXR's version-2 default rules, which mark them
    LOSSY_DCT too: decoded as halves (colour transform included) and widened
    exactly to float."""
    H, W = 24, 37
    r, g, b = _dwa_image(H, W, 11)
    chans = {"R": r, "G": g, "B": b}
    types = {"R": False, "G": False, "B": False}
    path = str(tmp_path / "dwa_f.exr")
    DWA_DECODED.clear()
    RAW_CHUNKS.clear()
    DWA_OPTS.update(rules=exr_dwa_py.DEFAULT_RULES_FLOAT)
    try:
        write_exr_py(path, chans, 9, True, types=types)
    finally:
        DWA_OPTS.pop("rules")
    assert not RAW_CHUNKS
    out = np.empty((H, W, 3), np.float32)
    assert lib().bmfr_exr_read_rgb(path.encode(), W, H, out.ctypes.data) == 0, lib().bmfr_io_error()
    want = _dwa_want((H, W), "RGB", chans, types)
    for c, n in enumerate("RGB"):
        np.testing.assert_array_equal(out[..., c], want[n], err_msg=n)
        assert (want[n] == want[n].astype(np.float16).astype(np.float32)).all()  # halves, widened


def test_exr_dwa_rejects_plinear_lossy_channel(tmp_path):
    """A LOSSY_DCT channel with the pLinear flag is refused as unsupported
    (not reported as corrupt data)."""
    H, W = 32, 64
    r, g, b = _dwa_image(H, W, 13)
    path = tmp_path / "dwa_lin.exr"
    DWA_DECODED.clear()
    RAW_CHUNKS.clear()
    write_exr_py(str(path), {"R": r, "G": g, "B": b}, 8, True)
    assert not RAW_CHUNKS
    bb = bytearray(path.read_bytes())
    i = bb.index(b"G\0", bb.index(b"chlist"))
    bb[i + 2 + 4] = 1  # G's pLinear flag
    path.write_bytes(bytes(bb))
    out = np.empty((H, W, 3), np.float32)
    assert lib().bmfr_exr_read_rgb(str(path).encode(), W, H, out.ctypes.data) != 0
    err = lib().bmfr_io_error()
    assert b"unsupported" in err and b"pLinear" in err and b"corrupt" not in err, err


def test_exr_dwa_rejects_corrupt_chunks(tmp_path):
    """Bad sizes, an unknown version or AC mode, and a truncated AC stream
    are errors, not crashes (the ASan corpus in test_sanitizers.py covers
    random damage)."""
    H, W = 32, 64
    r, g, b = _dwa_image(H, W, 9)
    path = tmp_path / "dwa.exr"
    DWA_DECODED.clear()
    RAW_CHUNKS.clear()
    write_exr_py(str(path), {"R": r, "G": g, "B": b}, 8, True)
    data = path.read_bytes()
    p = 8
    while data[p]:  # attributes: name, type, size, value
        e2 = data.index(b"\0", data.index(b"\0", p) + 1)
        p = e2 + 5 + struct.unpack_from("<i", data, e2 + 1)[0]
    first = struct.unpack_from("<Q", data, p + 1)[0] + 8  # the first chunk's DWA sizes (after y, size)
    assert struct.unpack_from("<Q", data, first)[0] == 2
    out = np.empty((H, W, 3), np.float32)
    for field, value in ((0, 7), (10, 5), (8, 10 ** 6), (9, 3)):  # version, AC mode, AC count, DC count
        bb = bytearray(data)
        struct.pack_into("<Q", bb, first + 8 * field, value)
        (tmp_path / "bad.exr").write_bytes(bytes(bb))
        assert lib().bmfr_exr_read_rgb(str(tmp_path / "bad.exr").encode(), W, H, out.ctypes.data) != 0, field
        assert b"corrupt chunk" in lib().bmfr_io_error()
