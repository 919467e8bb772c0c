"""Independent PIZ encoder for the EXR reader's tests (test infrastructure).

A pure-Python statement of the published OpenEXR PIZ scheme, encoder side
(the reader in host/image_io.cpp implements the decoder side):

* a chunk's samples as 16-bit little-endian words, channel by channel, each
  channel's lines one after the other (a FLOAT / UINT sample is two words,
  low half first);
* range map: a bitmap of the word values present (value 0 implicit), each
  word replaced by its rank among them; the bitmap bytes [min, max] of the
  non-zero bitmap bytes are stored;
* a 2-D Haar-like wavelet per channel and word component, finest level
  first: 14-bit lifting when the largest rank is below 2^14, modular 16-bit
  otherwise;
* Huffman coding: code lengths from the word frequencies plus one
  pseudo-symbol (frequency 1) that repeats the previous word 0..255 more
  times; canonical codes (longer codes numerically lower); the lengths
  stored as 6-bit fields with zero runs (59..62: 2..5 zeros, 63 + 8 bits:
  6..261 zeros); header = min symbol, max symbol, table bytes, bit count, 0.

Parity with the OpenEXR library is unpinned: neither OpenEXR nor a
reference PIZ file is available here.  Pure Python, for small test images.
"""
from __future__ import annotations

import heapq
import struct

USHORT_RANGE = 1 << 16
BITMAP_SIZE = USHORT_RANGE >> 3
SHORT_ZEROCODE_RUN, LONG_ZEROCODE_RUN = 59, 63
SHORTEST_LONG_RUN = 2 + LONG_ZEROCODE_RUN - SHORT_ZEROCODE_RUN
LONGEST_LONG_RUN = 255 + SHORTEST_LONG_RUN
MAX_VALUES = []  # the range map's largest rank of every chunk compressed (tests check both wavelet modes)


# ------------------------------------------------------------- wavelet ----
def _s16(v: int) -> int:
    v &= 0xFFFF
    return v - 0x10000 if v & 0x8000 else v


def _wenc14(a: int, b: int):
    as_, bs = _s16(a), _s16(b)
    return ((as_ + bs) >> 1) & 0xFFFF, (as_ - bs) & 0xFFFF


def _wenc16(a: int, b: int):
    ao = (a + (1 << 15)) & 0xFFFF
    m = (ao + b) >> 1
    d = ao - b
    if d < 0:
        m = (m + (1 << 15)) & 0xFFFF
    return m, d & 0xFFFF


def wav2_encode(buf: list, start: int, nx: int, ox: int, ny: int, oy: int, mx: int) -> None:
    """Forward wavelet of the nx x ny words at buf[start + x*ox + y*oy], in place."""
    enc = _wenc14 if mx < (1 << 14) else _wenc16
    n = min(nx, ny)
    p, p2 = 1, 2
    while p2 <= n:
        oy1, oy2, ox1, ox2 = oy * p, oy * p2, ox * p, ox * p2
        py = start
        ey = start + oy * (ny - p2)
        while py <= ey:
            px = py
            ex = py + ox * (nx - p2)
            while px <= ex:
                p01, p10 = px + ox1, px + oy1
                p11 = p10 + ox1
                i00, i01 = enc(buf[px], buf[p01])
                i10, i11 = enc(buf[p10], buf[p11])
                buf[px], buf[p10] = enc(i00, i10)
                buf[p01], buf[p11] = enc(i01, i11)
                px += ox2
            if nx & p:  # odd column
                p10 = px + oy1
                buf[px], buf[p10] = enc(buf[px], buf[p10])
            py += oy2
        if ny & p:  # odd line
            px = py
            ex = py + ox * (nx - p2)
            while px <= ex:
                p01 = px + ox1
                buf[px], buf[p01] = enc(buf[px], buf[p01])
                px += ox2
        p = p2
        p2 <<= 1


# ------------------------------------------------------------- Huffman ----
def _code_lengths(freq: dict) -> dict:
    """Huffman code lengths of the symbols with non-zero frequency."""
    if len(freq) == 1:
        return {next(iter(freq)): 1}
    heap = [(f, i, [s]) for i, (s, f) in enumerate(sorted(freq.items()))]
    heapq.heapify(heap)
    length = {s: 0 for s in freq}
    tie = len(heap)
    while len(heap) > 1:
        f1, _, a = heapq.heappop(heap)
        f2, _, b = heapq.heappop(heap)
        for s in a + b:
            length[s] += 1
        heapq.heappush(heap, (f1 + f2, tie, a + b))
        tie += 1
    return length


def _canonical(lengths: dict) -> dict:
    """symbol -> (code, length), canonical as the format defines it."""
    n = [0] * 59
    for l in lengths.values():
        n[l] += 1
    c = 0
    for i in range(58, 0, -1):
        nc = (c + n[i]) >> 1
        n[i] = c
        c = nc
    out = {}
    for s in sorted(lengths):
        l = lengths[s]
        out[s] = (n[l], l)
        n[l] += 1
    return out


class _BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.c = 0
        self.lc = 0

    def bits(self, n: int, v: int) -> None:
        self.c = (self.c << n) | v
        self.lc += n
        while self.lc >= 8:
            self.lc -= 8
            self.out.append((self.c >> self.lc) & 0xFF)
        self.c &= (1 << self.lc) - 1

    def flush(self) -> int:
        """Pad the last byte; returns the number of bits written."""
        nbits = 8 * len(self.out) + self.lc
        if self.lc:
            self.out.append((self.c << (8 - self.lc)) & 0xFF)
        return nbits


def huf_compress(words: list) -> bytes:
    if not words:
        return b""
    freq = {}
    for w in words:
        freq[w] = freq.get(w, 0) + 1
    im, iM = min(freq), max(freq)
    rlc = iM + 1  # the run pseudo-symbol
    freq[rlc] = 1
    codes = _canonical(_code_lengths(freq))
    assert max(l for _, l in codes.values()) <= 56
    # code-length table, zero runs packed
    tw = _BitWriter()
    s = im
    while s <= rlc:
        l = codes[s][1] if s in codes else 0
        if l == 0:
            run = 1
            while s + run <= rlc and run < LONGEST_LONG_RUN and (s + run) not in codes:
                run += 1
            if run >= 2:
                if run >= SHORTEST_LONG_RUN:
                    tw.bits(6, LONG_ZEROCODE_RUN)
                    tw.bits(8, run - SHORTEST_LONG_RUN)
                else:
                    tw.bits(6, SHORT_ZEROCODE_RUN + run - 2)
                s += run
                continue
        tw.bits(6, l)
        s += 1
    tw.flush()
    table = bytes(tw.out)
    # data: runs of one value as value + run symbol + 8-bit count when shorter
    dw = _BitWriter()

    def send(sym: int, run: int) -> None:
        c, l = codes[sym]
        rc, rl = codes[rlc]
        if l + rl + 8 < l * run:
            dw.bits(l, c)
            dw.bits(rl, rc)
            dw.bits(8, run)
        else:
            for _ in range(run + 1):
                dw.bits(l, c)

    s, cs = words[0], 0
    for w in words[1:]:
        if w == s and cs < 255:
            cs += 1
        else:
            send(s, cs)
            cs = 0
        s = w
    send(s, cs)
    nbits = dw.flush()
    return struct.pack("<IIIII", im, rlc, len(table), nbits, 0) + table + bytes(dw.out)


# ----------------------------------------------------------------- PIZ ----
def piz_compress(raw: bytes, width: int, lines: int, words_per_sample: list) -> bytes:
    """One chunk in the file's line-then-channel layout -> PIZ bytes."""
    nch = len(words_per_sample)
    per_line = [width * w for w in words_per_sample]
    line_words = sum(per_line)
    allw = list(struct.unpack(f"<{line_words * lines}H", raw))
    # channel by channel, each channel's lines in order
    chans, starts = [], []
    for c in range(nch):
        off = sum(per_line[:c])
        starts.append(len(chans))
        for y in range(lines):
            base = y * line_words + off
            chans.extend(allw[base:base + per_line[c]])
    bitmap = bytearray(BITMAP_SIZE)
    for v in chans:
        bitmap[v >> 3] |= 1 << (v & 7)
    bitmap[0] &= 0xFE
    nz = [i for i in range(BITMAP_SIZE) if bitmap[i]]
    lo, hi = (min(nz), max(nz)) if nz else (BITMAP_SIZE - 1, 0)
    lut, k = [0] * USHORT_RANGE, 0
    for i in range(USHORT_RANGE):
        if i == 0 or bitmap[i >> 3] & (1 << (i & 7)):
            lut[i] = k
            k += 1
    max_value = k - 1
    MAX_VALUES.append(max_value)
    chans = [lut[v] for v in chans]
    for c in range(nch):
        wps = words_per_sample[c]
        for j in range(wps):
            wav2_encode(chans, starts[c] + j, width, wps, lines, width * wps, max_value)
    huf = huf_compress(chans)
    out = struct.pack("<HH", lo, hi)
    if lo <= hi:
        out += bytes(bitmap[lo:hi + 1])
    return out + struct.pack("<i", len(huf)) + huf
