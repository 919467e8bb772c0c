"""Independent DWAA / DWAB encoder for the EXR reader's tests (test infrastructure).

A numpy statement of the published OpenEXR DWA scheme, encoder side (the
reader in host/image_io.cpp implements the decoder side), together with the
values a decoder of the scheme must produce from what it writes:

* a chunk = 11 little-endian u64 sizes (version, UNKNOWN uncompressed /
  compressed, AC compressed, DC compressed, RLE compressed / uncompressed /
  raw, AC and DC value counts, AC compression: 0 static Huffman -- PIZ's
  coder, tests/exr_piz_py.py --, 1 deflate), version 2's channel rules (u16
  byte count including itself; per rule the name suffix, a byte (CSC index +
  1) << 4 | scheme << 2 | case-insensitive, a pixel type), then the UNKNOWN,
  AC, DC and RLE sections;
* a channel takes the scheme of the first rule matching its name's last
  '.'-component and its type; UNKNOWN channels: raw lines, zlib; RLE
  channels: byte planes of the samples, OpenEXR RLE, zlib;
* LOSSY_DCT (HALF) channels: the samples mapped to the codec's perceptual
  scale (|x|^(1/2.2) up to 1, ln|x| / 2.2 + 1 above), an R, G, B set under
  one prefix converted to Y'CbCr (BT.709), 8 x 8 blocks (edges padded by
  repetition), the orthonormal DCT, coefficients rounded to half (small AC
  terms dropped: zero runs), in zig-zag order: DC terms per channel into the
  DC section (ZIP's interleave + byte predictor, zlib), AC terms block by
  block (each channel of a set in turn) as words -- 0xff00 ends a block,
  0xffnn skips nn zeros.

The expected decode repeats the decoder's arithmetic in float32 in the same
order (inverse DCT rows then columns, the inverse colour transform, rounding
to half, the perceptual-to-linear table), so the reader is checked bit for
bit.  Parity with the OpenEXR library is unpinned: neither OpenEXR nor a
reference DWA file is available here.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

from exr_piz_py import huf_compress

UNKNOWN, LOSSY_DCT, RLE = 0, 1, 2
UINT, HALF, FLOAT = 0, 1, 2

# (suffix, csc index, scheme, case-insensitive, pixel type): the default rules
# a version-2 chunk carries.
DEFAULT_RULES = [("R", 0, LOSSY_DCT, True, HALF), ("G", 1, LOSSY_DCT, True, HALF), ("B", 2, LOSSY_DCT, True, HALF),
                 ("Y", -1, LOSSY_DCT, True, HALF), ("BY", -1, LOSSY_DCT, True, HALF),
                 ("RY", -1, LOSSY_DCT, True, HALF), ("A", -1, RLE, True, UINT), ("A", -1, RLE, True, HALF),
                 ("A", -1, RLE, True, FLOAT)]
# OpenEXR's version-2 default rules also list the colour / luminance names for
# FLOAT channels (stored as halves, widened on decode).
DEFAULT_RULES_FLOAT = DEFAULT_RULES + [(n, c, LOSSY_DCT, True, FLOAT) for n, c in
                                       (("R", 0), ("G", 1), ("B", 2), ("Y", -1), ("BY", -1), ("RY", -1))]
LEGACY_RULES = [("r", 0, LOSSY_DCT, True, HALF), ("red", 0, LOSSY_DCT, True, HALF), ("g", 1, LOSSY_DCT, True, HALF),
                ("grn", 1, LOSSY_DCT, True, HALF), ("green", 1, LOSSY_DCT, True, HALF),
                ("b", 2, LOSSY_DCT, True, HALF), ("blu", 2, LOSSY_DCT, True, HALF),
                ("blue", 2, LOSSY_DCT, True, HALF), ("y", -1, LOSSY_DCT, True, HALF),
                ("by", -1, LOSSY_DCT, True, HALF), ("ry", -1, LOSSY_DCT, True, HALF), ("a", -1, RLE, True, UINT),
                ("a", -1, RLE, True, HALF), ("a", -1, RLE, True, FLOAT)]

ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                   13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59,
                   52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])

_K = np.arange(8)
T64 = (np.where(_K == 0, np.sqrt(0.5), 1.0)[:, None] * 0.5 *
       np.cos((2 * _K[None, :] + 1) * _K[:, None] * np.pi / 16))  # T[k, n]
T32 = T64.astype(np.float32)


def _lin_table() -> np.ndarray:
    h = np.arange(1 << 16, dtype=np.uint32).astype(np.uint16).view(np.float16).astype(np.float64)
    a = np.abs(h)
    with np.errstate(over="ignore", invalid="ignore"):
        lin = np.where(a <= 1.0, a ** 2.2, np.exp(2.2 * (a - 1.0)))
    lin = np.where(np.isfinite(h), np.where(h < 0, -lin, lin), 0.0)
    with np.errstate(over="ignore"):
        return lin.astype(np.float32).astype(np.float16).view(np.uint16)


TO_LINEAR = _lin_table()


def to_nonlinear(x: np.ndarray) -> np.ndarray:
    a = np.abs(x.astype(np.float64))
    with np.errstate(divide="ignore"):
        y = np.where(a <= 1.0, a ** (1 / 2.2), np.log(np.maximum(a, 1e-300)) / 2.2 + 1.0)
    return np.where(np.isfinite(x), np.where(x < 0, -y, y), 0.0)


def classify(name: str, ptype: int, rules) -> tuple:
    suffix = name.rsplit(".", 1)[-1]
    for suf, csc, scheme, nocase, t in rules:
        if t == ptype and (suffix.lower() == suf.lower() if nocase else suffix == suf):
            return scheme, csc
    return UNKNOWN, -1


def _rle(data: bytes) -> bytes:
    """OpenEXR RLE: (n - 1, byte) for a run of n >= 3 equal bytes, (-n, n bytes) literals."""
    out, i, n = bytearray(), 0, len(data)
    while i < n:
        j = i
        while j < n and j - i < 128 and data[j] == data[i]:
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


def _zip_predict(raw: bytes) -> bytes:
    a = np.frombuffer(raw, np.uint8)
    t = np.concatenate([a[0::2], a[1::2]]).astype(np.int32)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128 + 256) & 255
    return d.astype(np.uint8).tobytes()


def _blocks(a: np.ndarray) -> np.ndarray:
    """(lines, w) -> (nb, 8, 8) blocks, rows of blocks top to bottom; edges padded by repetition."""
    lines, w = a.shape
    ph, pw = (lines + 7) // 8 * 8, (w + 7) // 8 * 8
    p = np.pad(a, ((0, ph - lines), (0, pw - w)), mode="edge")
    return p.reshape(ph // 8, 8, pw // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 8, 8)


def _idct32(z: np.ndarray) -> np.ndarray:
    """The decoder's float32 inverse DCT of (nb, 64) zig-zag halves: rows, then columns, sums in k order."""
    b = np.zeros(z.shape, np.float32)
    b[:, ZIGZAG] = z.view(np.float16).astype(np.float32)
    b = b.reshape(-1, 8, 8)
    t = np.zeros_like(b)
    for k in range(8):  # t[r, n] = sum_k T[k, n] b[r, k]
        t = t + T32[k][None, None, :] * b[:, :, k:k + 1]
    out = np.zeros_like(b)
    for k in range(8):  # out[n, c] = sum_k T[k, n] t[k, c]
        out = out + T32[k][None, :, None] * t[:, k:k + 1, :]
    return out


def _unblock(blk: np.ndarray, lines: int, w: int) -> np.ndarray:
    bx = (w + 7) // 8
    by = blk.shape[0] // bx
    return blk.reshape(by, bx, 8, 8).transpose(0, 2, 1, 3).reshape(by * 8, bx * 8)[:lines, :w]


def dwa_compress(chans: dict, types: dict, lines: int, w: int, version: int = 2, ac_mode: int = 0,
                 drop: float = 0.02, rules=None):
    """One DWA chunk of `lines` x `w` samples.

    chans: channel name -> (lines, w) float array; types: name -> HALF / FLOAT
    / UINT.  Channels are taken in sorted-name order (the EXR channel list).
    drop: AC coefficients of magnitude below it become zeros.  Returns (chunk
    bytes, {name: decoded samples}) -- HALF as uint16 bit patterns, FLOAT as
    float32, UINT as uint32 -- what a decoder of the scheme must produce."""
    rules = rules if rules is not None else (DEFAULT_RULES if version == 2 else LEGACY_RULES)
    names = sorted(chans)
    info = {n: classify(n, types[n], rules) for n in names}
    decoded = {}

    def samples(n):
        a = np.ascontiguousarray(chans[n][:lines, :w])
        t = types[n]
        return a.astype(np.float16) if t == HALF else (a.astype(np.float32) if t == FLOAT else a.astype(np.uint32))

    # UNKNOWN: raw lines
    unk = bytearray()
    for y in range(lines):
        for n in names:
            if info[n][0] == UNKNOWN:
                unk += samples(n)[y].tobytes()
    for n in names:
        if info[n][0] == UNKNOWN:
            s = samples(n)
            decoded[n] = s.view(np.uint16) if types[n] == HALF else s
    # RLE: byte planes per channel
    rle_raw = bytearray()
    for n in names:
        if info[n][0] == RLE:
            s = samples(n)
            b = s.view(np.uint8).reshape(lines * w, -1)
            for k in range(b.shape[1]):
                rle_raw += b[:, k].tobytes()
            decoded[n] = s.view(np.uint16) if types[n] == HALF else s
    rle_unc = _rle(bytes(rle_raw)) if rle_raw else b""
    # LOSSY_DCT: the colour sets, then the other channels
    prefix = {n: (n.rsplit(".", 1)[0] + "." if "." in n else "") for n in names}
    used, sets = set(), []
    for n in names:
        sch, csc = info[n]
        if sch != LOSSY_DCT or csc < 0 or n in used:
            continue
        s = [None, None, None]
        for m in names:
            if info[m][0] == LOSSY_DCT and info[m][1] >= 0 and m not in used and prefix[m] == prefix[n] \
                    and s[info[m][1]] is None:
                s[info[m][1]] = m
        if None not in s:
            used.update(s)
            sets.append(s)
    decoders = sets + [[n] for n in names if info[n][0] == LOSSY_DCT and n not in used]
    nb = ((lines + 7) // 8) * ((w + 7) // 8)
    dc_words, ac_words = [], []
    for dec in decoders:
        x = [to_nonlinear(samples(n).astype(np.float64)) for n in dec]
        if len(dec) == 3:
            r, g, b = x
            yv = 0.2126 * r + 0.7152 * g + 0.0722 * b
            x = [yv, (b - yv) / 1.8556, (r - yv) / 1.5747]
        zz = []
        for c in x:
            blk = _blocks(c)
            coef = np.einsum("kn,bnm,lm->bkl", T64, blk, T64).reshape(nb, 64)[:, ZIGZAG]
            ac = coef[:, 1:]
            coef[:, 1:] = np.where(np.abs(ac) < drop, 0.0, ac)
            with np.errstate(over="ignore"):
                z = coef.astype(np.float16).view(np.uint16).copy()
            z[:, 1:] = np.where(z[:, 1:] == 0x8000, 0, z[:, 1:])  # -0 as 0: runs
            zz.append(z)
            dc_words.extend(z[:, 0].tolist())
        for bi in range(nb):
            for ci, z in enumerate(zz):
                row = z[bi, 1:].tolist()
                last = max([i for i, v in enumerate(row) if v] + [-1])
                i, k = 0, 0
                while i <= last:
                    if row[i]:
                        ac_words.append(row[i])
                        i += 1
                        continue
                    run = 0
                    while row[i + run] == 0:
                        run += 1
                    # zero runs both ways: a single zero sometimes as a plain 0 word
                    if run == 1 and (bi + ci + k) % 2:
                        ac_words.append(0)
                    else:
                        ac_words.append(0xff00 | run)
                    i += run
                    k += 1
                if last < 62:
                    ac_words.append(0xff00)
        # expected decode
        out = [_idct32(z) for z in zz]
        if len(dec) == 3:
            yv, cb, cr = out
            out = [yv + np.float32(1.5747) * cr, yv - np.float32(0.1873) * cb - np.float32(0.4682) * cr,
                   yv + np.float32(1.8556) * cb]
        for n, o in zip(dec, out):
            with np.errstate(over="ignore"):
                hb = o.astype(np.float16).view(np.uint16)
            d = _unblock(TO_LINEAR[hb], lines, w)
            # a FLOAT lossy channel: the half, widened exactly
            decoded[n] = d.view(np.float16).astype(np.float32) if types[n] == FLOAT else d
    # sections
    unk_c = zlib.compress(bytes(unk)) if unk else b""
    if ac_words:
        ac_c = huf_compress(ac_words) if ac_mode == 0 else zlib.compress(np.array(ac_words, np.uint16).tobytes())
        dc_c = zlib.compress(_zip_predict(np.array(dc_words, np.uint16).tobytes()))
    else:
        ac_c = b""
        dc_c = zlib.compress(_zip_predict(np.array(dc_words, np.uint16).tobytes())) if dc_words else b""
    rle_c = zlib.compress(rle_unc) if rle_raw else b""
    sizes = [version, len(unk), len(unk_c), len(ac_c), len(dc_c), len(rle_c), len(rle_unc), len(rle_raw),
             len(ac_words), len(dc_words), ac_mode]
    head = struct.pack("<11Q", *sizes)
    if version == 2:
        body = b"".join(s.encode() + b"\0" + bytes([((c + 1) << 4) | (sch << 2) | int(nc), t])
                        for s, c, sch, nc, t in rules)
        head += struct.pack("<H", len(body) + 2) + body
    return head + unk_c + ac_c + dc_c + rle_c, decoded
