// image_io.cpp -- OpenEXR (scanline and tiled, NONE/RLE/ZIPS/ZIP/PIZ/PXR24/B44/B44A/DWAA/DWAB) and
// PNG I/O over zlib.  See image_io.h.  The EXR layout follows the published
// OpenEXR 2 file format: magic + version, attribute list, per-chunk offset
// table, chunks of (y, size, data) -- tiled files: (tile x, tile y, level x,
// level y, size, data) -- with each scanline's channels stored in
// channel-list order.
#include "image_io.h"

#include <zlib.h>

#include <algorithm>
#include <array>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_error;

int fail(const std::string& msg) {
    g_error = msg;
    return -1;
}

// ------------------------------------------------------------------ EXR --
constexpr uint32_t kExrMagic = 20000630;
enum PixelType { kUint = 0, kHalf = 1, kFloat = 2 };

struct Channel {
    std::string name;
    int type;
    int xs, ys;
    bool linear = false;  // pLinear (B44 stores such HALF samples on a log scale)
};

struct ExrHeader {
    std::vector<Channel> channels;
    int compression = -1;
    int x0 = 0, y0 = 0, x1 = -1, y1 = -1;
    int line_order = 0;
    bool tiled = false;
    // tiled files ("tiles" attribute, tiledesc): tile size, level mode
    // (0 ONE_LEVEL, 1 MIPMAP_LEVELS, 2 RIPMAP_LEVELS; only level (0, 0) is read)
    uint32_t tile_w = 0, tile_h = 0;
    int level_mode = -1;
    int width() const { return x1 - x0 + 1; }
    int height() const { return y1 - y0 + 1; }
};

int lines_per_chunk(int compression) {
    switch (compression) {
        case BMFR_EXR_NONE: case BMFR_EXR_RLE: case BMFR_EXR_ZIPS: return 1;
        case BMFR_EXR_ZIP: case BMFR_EXR_PXR24: return 16;
        case BMFR_EXR_PIZ: case BMFR_EXR_B44: case BMFR_EXR_B44A: case BMFR_EXR_DWAA: return 32;
        case BMFR_EXR_DWAB: return 256;
        default: return 0;
    }
}

int type_bytes(int t) { return t == kHalf ? 2 : 4; }

struct Reader {
    const std::vector<uint8_t>& b;
    size_t p = 0;
    bool ok = true;
    template <class T>
    T get() {
        T v{};
        if (p + sizeof(T) > b.size()) {
            ok = false;
            return v;
        }
        std::memcpy(&v, b.data() + p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    std::string cstr() {
        std::string s;
        while (p < b.size() && b[p]) s.push_back((char)b[p++]);
        if (p >= b.size()) ok = false;
        ++p;
        return s;
    }
};

bool read_file(const char* path, std::vector<uint8_t>& out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    const bool ok = n >= 0 && std::fread(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

bool parse_header(const std::vector<uint8_t>& file, ExrHeader& h, size_t& end, std::string& err) {
    Reader r{file};
    if (r.get<uint32_t>() != kExrMagic) return err = "not an OpenEXR file", false;
    const uint32_t version = r.get<uint32_t>();
    if ((version & 0xff) != 2) return err = "unsupported OpenEXR version", false;
    if (version & 0x200) h.tiled = true;
    if (version & (0x800 | 0x1000)) return err = "deep / multi-part OpenEXR files are not supported", false;
    for (;;) {
        const std::string name = r.cstr();
        if (!r.ok) return err = "truncated header", false;
        if (name.empty()) break;
        const std::string type = r.cstr();
        const int32_t size = r.get<int32_t>();
        if (!r.ok || size < 0 || (size_t)size > file.size() - r.p) return err = "truncated attribute " + name, false;
        const size_t next = r.p + size;
        if (name == "channels" && type == "chlist") {
            while (r.p < next) {
                Channel c;
                c.name = r.cstr();
                if (c.name.empty()) break;
                c.type = r.get<int32_t>();
                c.linear = (r.get<uint32_t>() & 0xff) != 0;  // pLinear + reserved
                c.xs = r.get<int32_t>();
                c.ys = r.get<int32_t>();
                h.channels.push_back(c);
            }
        } else if (name == "compression") {
            if (size < 1) return err = "bad compression attribute", false;
            h.compression = file[r.p];
        } else if (name == "dataWindow" && size == 16) {
            h.x0 = r.get<int32_t>();
            h.y0 = r.get<int32_t>();
            h.x1 = r.get<int32_t>();
            h.y1 = r.get<int32_t>();
        } else if (name == "lineOrder") {
            if (size < 1) return err = "bad lineOrder attribute", false;
            h.line_order = file[r.p];
        } else if (name == "tiles" && type == "tiledesc") {
            if (size < 9) return err = "bad tiles attribute", false;
            h.tile_w = r.get<uint32_t>();
            h.tile_h = r.get<uint32_t>();
            h.level_mode = file[r.p] & 0xf;
        }
        r.p = next;
    }
    end = r.p;
    if (h.tiled && (h.level_mode < 0 || h.level_mode > 2 || h.tile_w == 0 || h.tile_h == 0 ||
                    h.tile_w > (1u << 16) || h.tile_h > (1u << 16)))
        return err = "bad or missing tile description", false;
    if (lines_per_chunk(h.compression) == 0) return err = "unsupported OpenEXR compression " + std::to_string(h.compression), false;
    // data window extents in 64-bit (x1 - x0 overflows int for hostile corners)
    const int64_t w64 = (int64_t)h.x1 - h.x0 + 1, h64 = (int64_t)h.y1 - h.y0 + 1;
    if (h.channels.empty() || w64 <= 0 || h64 <= 0 || w64 > (1 << 20) || h64 > (1 << 20) ||
        h.channels.size() > 1024)
        return err = "bad channels / data window", false;
    for (const Channel& c : h.channels)
        if (c.xs != 1 || c.ys != 1 || c.type < 0 || c.type > 2) return err = "subsampled or unknown channel " + c.name, false;
    if (h.compression == BMFR_EXR_B44 || h.compression == BMFR_EXR_B44A)
        for (const Channel& c : h.channels)
            if (c.linear && c.type == kHalf) return err = "B44 pLinear channel " + c.name + " is not supported", false;
    return true;
}

float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31;
    uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff;
    uint32_t bits;
    if (e == 0) {
        if (m == 0) {
            bits = s;
        } else {  // subnormal: normalise
            e = 127 - 15 + 1;
            while (!(m & 0x400)) {
                m <<= 1;
                --e;
            }
            m &= 0x3ff;
            bits = s | (e << 23) | (m << 13);
        }
    } else if (e == 31) {
        bits = s | 0x7f800000u | (m << 13);
    } else {
        bits = s | ((e + 127 - 15) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

// float -> half, rounded to nearest even (overflow -> inf, NaN kept quiet).
uint16_t float_to_half(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint16_t s = (uint16_t)((x >> 16) & 0x8000);
    const uint32_t a = x & 0x7fffffffu;
    if (a >= 0x7f800000u) return (uint16_t)(s | 0x7c00 | (a > 0x7f800000u ? 0x200 : 0));
    if (a >= 0x477ff000u) return (uint16_t)(s | 0x7c00);  // rounds past 65504
    if (a < 0x38800000u) {  // half subnormal (or zero)
        if (a < 0x33000000u) return s;  // below half the smallest subnormal: +-0
        const uint32_t e = a >> 23, m = (a & 0x7fffff) | 0x800000;
        const int shift = 126 - (int)e;  // 14 .. 24: value = m * 2^(e - 150), subnormal unit 2^-24
        const uint32_t q = m >> shift, r = m & ((1u << shift) - 1), half_ = 1u << (shift - 1);
        return (uint16_t)(s | (q + (r > half_ || (r == half_ && (q & 1)))));
    }
    const uint32_t q = (a - 0x38000000u) >> 13, r = a & 0x1fff;
    return (uint16_t)(s | (q + (r > 0x1000 || (r == 0x1000 && (q & 1)))));
}

// Undo ZIP/RLE preprocessing: delta predictor, then de-interleave the two halves.
void unpredict_deinterleave(std::vector<uint8_t>& t, uint8_t* out) {
    const size_t n = t.size();
    for (size_t i = 1; i < n; ++i) t[i] = (uint8_t)(t[i - 1] + t[i] - 128);
    const uint8_t* t1 = t.data();
    const uint8_t* t2 = t.data() + (n + 1) / 2;
    for (size_t i = 0; i < n; ++i) out[i] = (i & 1) ? *t2++ : *t1++;
}

void interleave_predict(const uint8_t* in, size_t n, std::vector<uint8_t>& t) {
    t.resize(n);
    uint8_t* t1 = t.data();
    uint8_t* t2 = t.data() + (n + 1) / 2;
    for (size_t i = 0; i < n; ++i) ((i & 1) ? *t2++ : *t1++) = in[i];
    int p = t[0];
    for (size_t i = 1; i < n; ++i) {
        const int d = (int)t[i] - p + (128 + 256);
        p = t[i];
        t[i] = (uint8_t)d;
    }
}

bool rle_decode(const uint8_t* in, size_t n, std::vector<uint8_t>& out, size_t expect) {
    out.clear();
    size_t i = 0;
    while (i < n) {
        const int c = (int8_t)in[i++];
        if (c < 0) {
            if (i + (size_t)(-c) > n) return false;
            out.insert(out.end(), in + i, in + i - c);
            i += -c;
        } else {
            if (i >= n) return false;
            out.insert(out.end(), (size_t)c + 1, in[i++]);
        }
        if (out.size() > expect) return false;
    }
    return out.size() == expect;
}

// ------------------------------------------------------------------ PIZ --
// The published OpenEXR PIZ scheme, decoder side: a chunk of 32 scanlines is
// held as 16-bit words, channel by channel (a FLOAT / UINT sample is two
// words, low half first); the words went through (1) a range map onto
// 0..maxValue given by a bitmap of the values present, (2) a 2-D Haar-like
// wavelet per channel and word component (14-bit lifting when maxValue <
// 2^14, modular 16-bit otherwise), (3) Huffman coding with a canonical code
// whose 6-bit code lengths are stored run-length packed, plus one
// pseudo-symbol that repeats the previous word.  Parity is unpinned: no
// OpenEXR library and no reference PIZ file exist here; tests/exr_piz_py.py
// is an independent encoder of the same scheme.
namespace piz {

constexpr int kUshortRange = 1 << 16;
constexpr int kBitmapSize = kUshortRange >> 3;
constexpr int kEncSize = (1 << 16) + 1;  // symbols 0..65535 + the run pseudo-symbol
constexpr int kDecBits = 14;             // first-level decoding table index bits
constexpr int kDecSize = 1 << kDecBits;
constexpr int kShortZeroRun = 59, kLongZeroRun = 63;
constexpr int kShortestLongRun = 2 + kLongZeroRun - kShortZeroRun;
constexpr int kMaxCodeLength = 56;  // keeps every bit window inside 64 bits

uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

// Code lengths -> (length | code << 6), canonical: per length, consecutive
// codes in symbol order; longer codes take the numerically lower values.
void canonical_codes(std::vector<uint64_t>& hcode) {
    uint64_t n[59] = {};
    for (uint64_t l : hcode) ++n[l];
    uint64_t c = 0;
    for (int i = 58; i > 0; --i) {
        const uint64_t nc = (c + n[i]) >> 1;
        n[i] = c;
        c = nc;
    }
    for (uint64_t& h : hcode)
        if (h > 0) h = h | (n[h]++ << 6);
}

struct BitReader {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t c = 0;
    int lc = 0;
    bool byte() {
        if (p >= end) return false;
        c = (c << 8) | *p++;
        lc += 8;
        return true;
    }
    bool bits(int n, uint32_t& v) {
        while (lc < n)
            if (!byte()) return false;
        lc -= n;
        v = (uint32_t)((c >> lc) & ((1u << n) - 1));
        return true;
    }
};

// Packed code lengths of symbols im..iM (6 bits each; 59..62: a run of
// 2..5 zero lengths; 63 + 8 bits: a run of 6..261).
bool unpack_table(BitReader& in, uint32_t im, uint32_t iM, std::vector<uint64_t>& hcode) {
    hcode.assign(kEncSize, 0);
    for (uint32_t i = im; i <= iM; ++i) {
        uint32_t l;
        if (!in.bits(6, l)) return false;
        if (l == (uint32_t)kLongZeroRun || l >= (uint32_t)kShortZeroRun) {
            uint32_t run;
            if (l == (uint32_t)kLongZeroRun) {
                if (!in.bits(8, run)) return false;
                run += kShortestLongRun;
            } else {
                run = l - kShortZeroRun + 2;
            }
            if ((uint64_t)i + run > (uint64_t)iM + 1) return false;
            i += run - 1;  // the lengths are already zero
        } else {
            if (l > (uint32_t)kMaxCodeLength) return false;
            hcode[i] = l;
        }
    }
    canonical_codes(hcode);
    return true;
}

struct DecEntry {
    int len = 0;             // > 0: a code of this length (<= kDecBits) starts here
    int sym = 0;             // its symbol
    std::vector<int> longs;  // symbols of the longer codes with this prefix
};

bool build_decoder(const std::vector<uint64_t>& hcode, uint32_t im, uint32_t iM, std::vector<DecEntry>& dec) {
    dec.assign(kDecSize, DecEntry{});
    for (uint32_t i = im; i <= iM; ++i) {
        const uint64_t c = hcode[i] >> 6;
        const int l = (int)(hcode[i] & 63);
        if (l == 0) continue;
        if (c >> l) return false;  // not an l-bit code
        if (l > kDecBits) {
            DecEntry& e = dec[c >> (l - kDecBits)];
            if (e.len) return false;
            e.longs.push_back((int)i);
        } else {
            const uint64_t base = c << (kDecBits - l);
            for (uint64_t k = 0; k < (1ull << (kDecBits - l)); ++k) {
                DecEntry& e = dec[base + k];
                if (e.len || !e.longs.empty()) return false;
                e.len = l;
                e.sym = (int)i;
            }
        }
    }
    return true;
}

// nbits bits of codes from in -> no words; symbol rlc repeats the previous
// word (8-bit count).
bool huf_decode(const std::vector<uint64_t>& hcode, const std::vector<DecEntry>& dec, const uint8_t* in,
                const uint8_t* in_end, uint64_t nbits, int rlc, uint16_t* out, size_t no) {
    BitReader r{in, in + (nbits + 7) / 8};
    size_t o = 0;
    auto emit = [&](int sym) -> bool {
        if (sym == rlc) {
            if (r.lc < 8) {  // the count may sit in the byte past the coded bits
                if (r.p >= in_end) return false;
                r.c = (r.c << 8) | *r.p++;
                r.lc += 8;
            }
            r.lc -= 8;
            const uint32_t cs = (uint32_t)(r.c >> r.lc) & 0xff;
            if (o == 0 || o + cs > no) return false;
            const uint16_t s = out[o - 1];
            for (uint32_t k = 0; k < cs; ++k) out[o++] = s;
            return true;
        }
        if (o >= no) return false;
        out[o++] = (uint16_t)sym;
        return true;
    };
    while (r.p < r.end) {
        r.byte();
        while (r.lc >= kDecBits) {
            const DecEntry& e = dec[(r.c >> (r.lc - kDecBits)) & (kDecSize - 1)];
            if (e.len) {
                r.lc -= e.len;
                if (!emit(e.sym)) return false;
                continue;
            }
            bool found = false;
            for (int sym : e.longs) {
                const int l = (int)(hcode[sym] & 63);
                while (r.lc < l && r.p < r.end) r.byte();
                if (r.lc >= l && (hcode[sym] >> 6) == ((r.c >> (r.lc - l)) & ((1ull << l) - 1))) {
                    r.lc -= l;
                    if (!emit(sym)) return false;
                    found = true;
                    break;
                }
            }
            if (!found) return false;
        }
    }
    // the last, short codes: drop the padding bits of the final byte
    const int pad = (int)((8 - nbits) & 7);
    if (pad > r.lc) return false;
    r.c >>= pad;
    r.lc -= pad;
    while (r.lc > 0) {
        const DecEntry& e = dec[(r.c << (kDecBits - r.lc)) & (kDecSize - 1)];
        if (!e.len || e.len > r.lc) return false;
        r.lc -= e.len;
        if (!emit(e.sym)) return false;
    }
    return o == no;
}

bool huf_uncompress(const uint8_t* comp, size_t n, uint16_t* raw, size_t nraw) {
    if (n == 0) return nraw == 0;
    if (n < 20) return false;
    const uint32_t im = rd32(comp), iM = rd32(comp + 4), nbits = rd32(comp + 12);
    if (im >= (uint32_t)kEncSize || iM >= (uint32_t)kEncSize || im > iM) return false;
    BitReader table{comp + 20, comp + n};
    std::vector<uint64_t> hcode;
    if (!unpack_table(table, im, iM, hcode)) return false;
    const uint8_t* data = table.p;
    if ((uint64_t)nbits > 8ull * (uint64_t)(comp + n - data)) return false;
    std::vector<DecEntry> dec;
    if (!build_decoder(hcode, im, iM, dec)) return false;
    return huf_decode(hcode, dec, data, comp + n, nbits, (int)iM, raw, nraw);
}

// One level of the wavelet, inverse: 14-bit lifting or modular 16-bit.
inline void wdec14(uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
    const int hi = (int16_t)h;
    const int ai = (int16_t)l + (hi & 1) + (hi >> 1);
    a = (uint16_t)(int16_t)ai;
    b = (uint16_t)(int16_t)(ai - hi);
}
inline void wdec16(uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
    constexpr int kOff = 1 << 15, kMask = (1 << 16) - 1;
    const int m = l, d = h;
    const int bb = (m - (d >> 1)) & kMask;
    const int aa = (d + bb - kOff) & kMask;
    b = (uint16_t)bb;
    a = (uint16_t)aa;
}

// Inverse 2-D wavelet of an nx x ny array of words at stride ox (x) and oy (y).
void wav2_decode(uint16_t* in, int nx, int ox, int ny, int oy, uint16_t mx) {
    const bool w14 = mx < (1 << 14);
    auto dec = [w14](uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
        if (w14) wdec14(l, h, a, b);
        else wdec16(l, h, a, b);
    };
    const int n = nx > ny ? ny : nx;
    int p = 1;
    while (p <= n) p <<= 1;
    p >>= 1;
    int p2 = p;
    p >>= 1;
    while (p >= 1) {
        uint16_t* py = in;
        uint16_t* const ey = in + (ptrdiff_t)oy * (ny - p2);
        const int oy1 = oy * p, oy2 = oy * p2, ox1 = ox * p, ox2 = ox * p2;
        uint16_t i00, i01, i10, i11;
        for (; py <= ey; py += oy2) {
            uint16_t* px = py;
            uint16_t* const ex = py + (ptrdiff_t)ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t* p01 = px + ox1;
                uint16_t* p10 = px + oy1;
                uint16_t* p11 = p10 + ox1;
                dec(*px, *p10, i00, i10);
                dec(*p01, *p11, i01, i11);
                dec(i00, i01, *px, *p01);
                dec(i10, i11, *p10, *p11);
            }
            if (nx & p) {  // odd column
                uint16_t* p10 = px + oy1;
                dec(*px, *p10, i00, *p10);
                *px = i00;
            }
        }
        if (ny & p) {  // odd line
            uint16_t* px = py;
            uint16_t* const ex = py + (ptrdiff_t)ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t* p01 = px + ox1;
                dec(*px, *p01, i00, *p01);
                *px = i00;
            }
        }
        p2 = p;
        p >>= 1;
    }
}

// One PIZ chunk -> `lines` scanlines of `words` (per channel: 1 for HALF, 2
// for FLOAT / UINT) x width samples, in the file's line-then-channel layout.
bool uncompress(const uint8_t* in, size_t n, int width, int lines, const std::vector<int>& words,
                std::vector<uint8_t>& raw) {
    size_t total = 0;
    std::vector<size_t> start(words.size());
    for (size_t c = 0; c < words.size(); ++c) {
        start[c] = total;
        total += (size_t)width * lines * words[c];
    }
    if (n < 4) return false;
    const uint16_t lo = (uint16_t)(in[0] | in[1] << 8), hi = (uint16_t)(in[2] | in[3] << 8);
    size_t p = 4;
    if (hi >= kBitmapSize) return false;
    std::vector<uint8_t> bitmap(kBitmapSize, 0);
    if (lo <= hi) {
        const size_t nb = (size_t)hi - lo + 1;
        if (nb > n - p) return false;
        std::memcpy(bitmap.data() + lo, in + p, nb);
        p += nb;
    }
    // reverse range map: the k-th value present (0 always) -> k
    std::vector<uint16_t> lut(kUshortRange, 0);
    int k = 0;
    for (int i = 0; i < kUshortRange; ++i)
        if (i == 0 || (bitmap[i >> 3] & (1 << (i & 7)))) lut[k++] = (uint16_t)i;
    const uint16_t max_value = (uint16_t)(k - 1);
    if (n - p < 4) return false;
    const uint32_t length = rd32(in + p);
    p += 4;
    if (length > n - p) return false;
    std::vector<uint16_t> tmp(total);
    if (!huf_uncompress(in + p, length, tmp.data(), total)) return false;
    for (size_t c = 0; c < words.size(); ++c)
        for (int j = 0; j < words[c]; ++j)
            wav2_decode(tmp.data() + start[c] + j, width, words[c], lines, width * words[c], max_value);
    for (uint16_t& v : tmp) v = lut[v];
    raw.resize(total * 2);
    uint8_t* o = raw.data();
    for (int y = 0; y < lines; ++y)
        for (size_t c = 0; c < words.size(); ++c) {
            const uint16_t* s = tmp.data() + start[c] + (size_t)y * width * words[c];
            for (size_t x = 0; x < (size_t)width * words[c]; ++x) {
                *o++ = (uint8_t)(s[x] & 0xff);
                *o++ = (uint8_t)(s[x] >> 8);
            }
        }
    return true;
}

}  // namespace piz

// ---------------------------------------------------------------- PXR24 --
// The published OpenEXR PXR24 scheme, decoder side: per scanline and
// channel, the samples as integers -- HALF 16 bits, UINT 32 bits, FLOAT the
// top 24 bits of the float rounded (lossy) -- replaced by their differences
// from the previous sample of the line, split into byte planes (most
// significant first, each `width` bytes), all planes zlib-deflated.  The
// decoded FLOAT is the 24-bit value in the top bits, low byte zero.
bool pxr24_uncompress(const ExrHeader& h, const uint8_t* in, size_t n, int width, int lines,
                      std::vector<uint8_t>& raw) {
    size_t planes = 0;  // bytes per pixel of all channels, packed form
    for (const Channel& c : h.channels) planes += c.type == kHalf ? 2 : (c.type == kFloat ? 3 : 4);
    const size_t packed = planes * (size_t)width * lines;
    std::vector<uint8_t> t(packed);
    uLongf got = (uLongf)packed;
    if (uncompress(t.data(), &got, in, (uLong)n) != Z_OK || got != packed) return false;
    uint8_t* o = raw.data();
    const uint8_t* p = t.data();
    for (int y = 0; y < lines; ++y)
        for (const Channel& c : h.channels) {
            const size_t w = (size_t)width;
            uint32_t pixel = 0;
            if (c.type == kHalf) {
                for (size_t x = 0; x < w; ++x) {
                    pixel += (uint32_t)p[x] << 8 | p[w + x];
                    const uint16_t v = (uint16_t)pixel;
                    std::memcpy(o + 2 * x, &v, 2);
                }
                p += 2 * w;
                o += 2 * w;
            } else if (c.type == kFloat) {
                for (size_t x = 0; x < w; ++x) {
                    pixel += (uint32_t)p[x] << 24 | (uint32_t)p[w + x] << 16 | (uint32_t)p[2 * w + x] << 8;
                    std::memcpy(o + 4 * x, &pixel, 4);
                }
                p += 3 * w;
                o += 4 * w;
            } else {
                for (size_t x = 0; x < w; ++x) {
                    pixel += (uint32_t)p[x] << 24 | (uint32_t)p[w + x] << 16 | (uint32_t)p[2 * w + x] << 8 |
                             p[3 * w + x];
                    std::memcpy(o + 4 * x, &pixel, 4);
                }
                p += 4 * w;
                o += 4 * w;
            }
        }
    return true;
}

// ------------------------------------------------------------------ B44 --
// The published OpenEXR B44 / B44A scheme, decoder side.  The chunk holds
// its channels one after another, each over the whole chunk: FLOAT / UINT
// channels as their raw bytes (rows of the chunk), HALF channels as 4 x 4
// blocks of samples, rows of blocks top to bottom.  A block is 14 bytes --
// the first sample (mapped to an ordered 16-bit code: negative halves
// complemented, positive ones with the top bit set), a 6-bit shift and 15
// 6-bit differences (biased by 0x20, scaled by 2^shift) down the block's
// first column and along each row -- or, B44A only, 3 bytes for a flat block
// (third byte >= 13 << 2: every sample equal to the first).  Edge blocks are
// padded; the decoder drops what lies outside the chunk.  Channels with the
// pLinear flag (samples stored on a log scale) are rejected at the header.
namespace b44 {

void ordered_to_half(uint16_t (&s)[16]) {
    for (uint16_t& v : s) v = (v & 0x8000) ? (uint16_t)(v & 0x7fff) : (uint16_t)~v;
}

void unpack14(const uint8_t* b, uint16_t (&s)[16]) {
    const int shift = b[2] >> 2, bias = 0x20 << shift;
    // (column, row) order of the differences: column 0 downwards, then each row rightwards
    auto step = [&](int from, int r6) { return (uint16_t)(from + (r6 << shift) - bias); };
    s[0] = (uint16_t)(b[0] << 8 | b[1]);
    s[4] = step(s[0], ((b[2] << 4) | (b[3] >> 4)) & 0x3f);
    s[8] = step(s[4], ((b[3] << 2) | (b[4] >> 6)) & 0x3f);
    s[12] = step(s[8], b[4] & 0x3f);
    s[1] = step(s[0], b[5] >> 2);
    s[5] = step(s[4], ((b[5] << 4) | (b[6] >> 4)) & 0x3f);
    s[9] = step(s[8], ((b[6] << 2) | (b[7] >> 6)) & 0x3f);
    s[13] = step(s[12], b[7] & 0x3f);
    s[2] = step(s[1], b[8] >> 2);
    s[6] = step(s[5], ((b[8] << 4) | (b[9] >> 4)) & 0x3f);
    s[10] = step(s[9], ((b[9] << 2) | (b[10] >> 6)) & 0x3f);
    s[14] = step(s[13], b[10] & 0x3f);
    s[3] = step(s[2], b[11] >> 2);
    s[7] = step(s[6], ((b[11] << 4) | (b[12] >> 4)) & 0x3f);
    s[11] = step(s[10], ((b[12] << 2) | (b[13] >> 6)) & 0x3f);
    s[15] = step(s[14], b[13] & 0x3f);
    ordered_to_half(s);
}

void unpack3(const uint8_t* b, uint16_t (&s)[16]) {
    const uint16_t v = (uint16_t)(b[0] << 8 | b[1]);
    for (uint16_t& x : s) x = v;
    ordered_to_half(s);
}

bool uncompress(const ExrHeader& h, const uint8_t* in, size_t n, int width, int lines, std::vector<uint8_t>& raw) {
    // per channel, its samples over the chunk (row-major), then interleaved per line
    std::vector<std::vector<uint8_t>> planes;
    size_t p = 0;
    for (const Channel& c : h.channels) {
        const size_t row = (size_t)width * type_bytes(c.type);
        std::vector<uint8_t> pl(row * lines);
        if (c.type != kHalf) {
            if (n - p < pl.size()) return false;
            std::memcpy(pl.data(), in + p, pl.size());
            p += pl.size();
        } else {
            for (int y = 0; y < lines; y += 4)
                for (int x = 0; x < width; x += 4) {
                    uint16_t s[16];
                    if (n - p < 3) return false;
                    if (in[p + 2] >= (13 << 2)) {
                        unpack3(in + p, s);
                        p += 3;
                    } else {
                        if (n - p < 14) return false;
                        unpack14(in + p, s);
                        p += 14;
                    }
                    for (int dy = 0; dy < 4 && y + dy < lines; ++dy)
                        for (int dx = 0; dx < 4 && x + dx < width; ++dx) {
                            uint8_t* o = pl.data() + (size_t)(y + dy) * row + 2 * (size_t)(x + dx);
                            o[0] = (uint8_t)(s[4 * dy + dx] & 0xff);
                            o[1] = (uint8_t)(s[4 * dy + dx] >> 8);
                        }
                }
        }
        planes.push_back(std::move(pl));
    }
    if (p != n) return false;
    uint8_t* o = raw.data();
    for (int y = 0; y < lines; ++y)
        for (size_t c = 0; c < planes.size(); ++c) {
            const size_t row = (size_t)width * type_bytes(h.channels[c].type);
            std::memcpy(o, planes[c].data() + (size_t)y * row, row);
            o += row;
        }
    return true;
}

}  // namespace b44

// ------------------------------------------------------------------ DWA --
// The published OpenEXR DWAA / DWAB scheme (DreamWorks' lossy DCT codec),
// decoder side.  A chunk (32 lines DWAA, 256 DWAB) is
//   11 little-endian u64: version, unknown uncompressed / compressed size,
//     AC compressed size, DC compressed size, RLE compressed / uncompressed /
//     raw size, AC and DC value counts, AC compression (0 static Huffman --
//     PIZ's coder --, 1 deflate);
//   version 2: the channel rules, a u16 byte count (itself included) and
//     rules of (channel-name suffix, a byte (CSC index + 1) << 4 | scheme << 2
//     | case-insensitive, a pixel type); version 1 uses the fixed legacy set;
//   then the UNKNOWN, AC, DC and RLE sections.
// Each channel takes the scheme of the first rule matching its name's last
// '.'-component and its type (none: UNKNOWN).
//   UNKNOWN: the channels' raw lines (each line: those channels in order),
//     zlib-compressed.
//   RLE: per channel, its samples' bytes as byte planes (plane k: byte k of
//     every sample, rows in order), the channels one after another, then
//     OpenEXR RLE, then zlib.
//   LOSSY_DCT (HALF only): 8 x 8 blocks, rows of blocks top to bottom; each
//     block's 64 DCT coefficients are halves in zig-zag order -- the DC term
//     in the DC section (per decoded channel, all its blocks; zlib with
//     ZIP's byte predictor and interleave), the 63 AC terms in the AC section,
//     block after block (per block, each channel of a colour set in turn):
//     0xff00 ends the block (the rest zero), 0xffnn skips nn zeros, any other
//     word is the next coefficient.  The decoder forms the inverse DCT
//     (x = sum_k c_k / 2 X_k cos((2n + 1) k pi / 16), c_0 = 1/sqrt 2, rows then
//     columns) in float, for an R, G, B set (CSC indices 0, 1, 2 under one
//     prefix) converts Y'CbCr to RGB (BT.709: R = Y + 1.5747 Cr, G = Y -
//     0.1873 Cb - 0.4682 Cr, B = Y + 1.8556 Cb), rounds each value to half
//     and maps it from the codec's perceptual scale to linear (table below:
//     |y|^2.2 up to 1, exp(2.2 (|y| - 1)) above, sign kept; non-finite -> 0).
//     Decoded channels come in this order: the colour sets, then the other
//     LOSSY_DCT channels, in channel-list order.
// Parity is unpinned: no OpenEXR library and no reference DWA file exist
// here; tests/exr_dwa_py.py is an independent encoder of the same scheme.
// Why the last chunk decode failed when the file is valid but uses a feature
// this reader does not implement ("" = corrupt data); the caller reports it.
thread_local std::string g_chunk_unsupported;
bool unsupported(const std::string& what) {
    g_chunk_unsupported = what;
    return false;
}

namespace dwa {

enum Scheme { kUnknown = 0, kLossyDct = 1, kRle = 2 };

struct Rule {
    std::string suffix;
    int csc;  // -1, or the colour index 0 / 1 / 2 (R / G / B)
    int scheme;
    bool nocase;
    int type;
};

const std::vector<Rule>& legacy_rules() {
    static const std::vector<Rule> r = {
        {"r", 0, kLossyDct, true, kHalf},     {"red", 0, kLossyDct, true, kHalf},
        {"g", 1, kLossyDct, true, kHalf},     {"grn", 1, kLossyDct, true, kHalf},
        {"green", 1, kLossyDct, true, kHalf}, {"b", 2, kLossyDct, true, kHalf},
        {"blu", 2, kLossyDct, true, kHalf},   {"blue", 2, kLossyDct, true, kHalf},
        {"y", -1, kLossyDct, true, kHalf},    {"by", -1, kLossyDct, true, kHalf},
        {"ry", -1, kLossyDct, true, kHalf},   {"a", -1, kRle, true, kUint},
        {"a", -1, kRle, true, kHalf},         {"a", -1, kRle, true, kFloat},
    };
    return r;
}

std::string lower(std::string s) {
    for (char& ch : s) ch = (char)std::tolower((unsigned char)ch);
    return s;
}

// The channel's rule: scheme and CSC index.
void classify(const std::vector<Rule>& rules, const Channel& c, int& scheme, int& csc) {
    const size_t dot = c.name.rfind('.');
    const std::string suffix = dot == std::string::npos ? c.name : c.name.substr(dot + 1);
    for (const Rule& r : rules) {
        if (r.type != c.type) continue;
        if (r.nocase ? lower(suffix) == lower(r.suffix) : suffix == r.suffix) {
            scheme = r.scheme;
            csc = r.csc;
            return;
        }
    }
    scheme = kUnknown;
    csc = -1;
}

// Perceptual half -> linear half (the codec's inverse transfer).
const std::vector<uint16_t>& to_linear() {
    static const std::vector<uint16_t> t = [] {
        std::vector<uint16_t> v(1 << 16);
        for (uint32_t b = 0; b < (1u << 16); ++b) {
            const float f = half_to_float((uint16_t)b);
            double lin = 0.0;
            if (std::isfinite(f)) {
                const double a = std::fabs((double)f);
                lin = a <= 1.0 ? std::pow(a, 2.2) : std::exp(2.2 * (a - 1.0));
                if (f < 0) lin = -lin;
            }
            v[b] = float_to_half((float)lin);
        }
        return v;
    }();
    return t;
}

constexpr int kZigZag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// In-place 8 x 8 inverse DCT (rows, then columns), float.
void idct8x8(float (&b)[64]) {
    static const std::vector<float> T = [] {
        std::vector<float> m(64);
        const double pi = 3.14159265358979323846;
        for (int k = 0; k < 8; ++k)
            for (int n = 0; n < 8; ++n)
                m[k * 8 + n] = (float)((k == 0 ? std::sqrt(0.5) : 1.0) * 0.5 * std::cos((2 * n + 1) * k * pi / 16));
        return m;
    }();
    float t[64];
    for (int r = 0; r < 8; ++r)
        for (int n = 0; n < 8; ++n) {
            float s = 0.f;
            for (int k = 0; k < 8; ++k) s += T[k * 8 + n] * b[r * 8 + k];
            t[r * 8 + n] = s;
        }
    for (int c = 0; c < 8; ++c)
        for (int n = 0; n < 8; ++n) {
            float s = 0.f;
            for (int k = 0; k < 8; ++k) s += T[k * 8 + n] * t[k * 8 + c];
            b[n * 8 + c] = s;
        }
}

uint64_t rd64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
}

// zlib into exactly `want` bytes.
bool inflate_exact(const uint8_t* in, uint64_t n, std::vector<uint8_t>& out, uint64_t want) {
    if (want > (1ull << 31) || n > (1ull << 31)) return false;
    out.resize((size_t)want);
    if (want == 0) return n == 0;
    uLongf got = (uLongf)want;
    return uncompress(out.data(), &got, in, (uLong)n) == Z_OK && got == want;
}

bool uncompress(const ExrHeader& h, const uint8_t* in, size_t n, int width, int lines, std::vector<uint8_t>& raw) {
    constexpr int kSizes = 11;
    if (n < 8 * kSizes) return false;
    uint64_t sz[kSizes];
    for (int i = 0; i < kSizes; ++i) sz[i] = rd64(in + 8 * i);
    const uint64_t version = sz[0], unk_raw = sz[1], unk_comp = sz[2], ac_comp = sz[3], dc_comp = sz[4],
                   rle_comp = sz[5], rle_unc = sz[6], rle_raw = sz[7], ac_count = sz[8], dc_count = sz[9],
                   ac_mode = sz[10];
    if (version > 2 || ac_mode > 1) return false;
    const uint8_t* p = in + 8 * kSizes;
    const uint8_t* const end = in + n;
    std::vector<Rule> rules;
    if (version == 2) {
        if (end - p < 2) return false;
        const uint16_t rule_bytes = (uint16_t)(p[0] | p[1] << 8);
        if (rule_bytes < 2 || rule_bytes > end - p) return false;
        const uint8_t* r = p + 2;
        const uint8_t* const rend = p + rule_bytes;
        while (r < rend) {
            const uint8_t* z = (const uint8_t*)std::memchr(r, 0, (size_t)(rend - r));
            if (!z || rend - z < 3) return false;
            Rule ru;
            ru.suffix.assign((const char*)r, (size_t)(z - r));
            const uint8_t v = z[1];
            ru.csc = (v >> 4) - 1;
            ru.scheme = (v >> 2) & 3;
            ru.nocase = (v & 1) != 0;
            ru.type = z[2];
            if (ru.csc > 2 || ru.scheme > kRle || ru.type > kFloat) return false;
            rules.push_back(ru);
            r = z + 3;
        }
        p = rend;
    } else {
        rules = legacy_rules();
    }
    // the sections, in order, inside the chunk
    const uint64_t left = (uint64_t)(end - p);
    if (unk_comp > left || ac_comp > left - unk_comp || dc_comp > left - unk_comp - ac_comp ||
        rle_comp > left - unk_comp - ac_comp - dc_comp)
        return false;
    const uint8_t* unk_p = p;
    const uint8_t* ac_p = unk_p + unk_comp;
    const uint8_t* dc_p = ac_p + ac_comp;
    const uint8_t* rle_p = dc_p + dc_comp;

    // channel schemes and colour sets
    const size_t nc = h.channels.size();
    std::vector<int> scheme(nc), csc(nc);
    for (size_t i = 0; i < nc; ++i) classify(rules, h.channels[i], scheme[i], csc[i]);
    std::vector<std::array<int, 3>> sets;  // channel indices of complete R, G, B sets
    std::vector<int> in_set(nc, 0);
    {
        std::vector<std::string> prefix(nc);
        for (size_t i = 0; i < nc; ++i) {
            const size_t dot = h.channels[i].name.rfind('.');
            prefix[i] = dot == std::string::npos ? std::string() : h.channels[i].name.substr(0, dot + 1);
        }
        std::vector<int> used(nc, 0);
        for (size_t i = 0; i < nc; ++i) {
            if (scheme[i] != kLossyDct || csc[i] < 0 || used[i]) continue;
            std::array<int, 3> s = {-1, -1, -1};
            for (size_t j = 0; j < nc; ++j)
                if (scheme[j] == kLossyDct && csc[j] >= 0 && !used[j] && prefix[j] == prefix[i] && s[csc[j]] < 0)
                    s[csc[j]] = (int)j;
            if (s[0] >= 0 && s[1] >= 0 && s[2] >= 0) {
                for (int k : s) used[k] = in_set[k] = 1;
                sets.push_back(s);
            }
        }
    }
    // LOSSY_DCT channels hold halves; a FLOAT channel under a LOSSY_DCT rule
    // (OpenEXR's version-2 default rules list R, G, B, Y, BY, RY for HALF and
    // FLOAT) is decoded as half and widened to float.  UINT cannot be lossy.
    // A pLinear channel would skip the perceptual-to-linear table in some
    // writers: without a reference decoder to pin that here it is refused.
    for (size_t i = 0; i < nc; ++i) {
        if (scheme[i] != kLossyDct) continue;
        if (h.channels[i].type == kUint) return false;
        if (h.channels[i].linear) return unsupported("DWA pLinear channel " + h.channels[i].name);
    }

    // per-channel decoded planes (row-major, type_bytes per sample)
    std::vector<std::vector<uint8_t>> plane(nc);
    const size_t W = (size_t)width, L = (size_t)lines;

    // UNKNOWN
    {
        size_t line_bytes = 0;
        for (size_t i = 0; i < nc; ++i)
            if (scheme[i] == kUnknown) line_bytes += W * type_bytes(h.channels[i].type);
        if (unk_raw != line_bytes * L) return false;
        std::vector<uint8_t> u;
        if (!inflate_exact(unk_p, unk_comp, u, unk_raw)) return false;
        size_t o = 0;
        for (size_t y = 0; y < L; ++y)
            for (size_t i = 0; i < nc; ++i) {
                if (scheme[i] != kUnknown) continue;
                const size_t row = W * type_bytes(h.channels[i].type);
                plane[i].resize(row * L);
                std::memcpy(plane[i].data() + y * row, u.data() + o, row);
                o += row;
            }
    }
    // RLE
    {
        size_t want = 0;
        for (size_t i = 0; i < nc; ++i)
            if (scheme[i] == kRle) want += W * L * type_bytes(h.channels[i].type);
        if (rle_raw != want) return false;
        std::vector<uint8_t> r;
        if (want > 0) {
            std::vector<uint8_t> z;
            if (!inflate_exact(rle_p, rle_comp, z, rle_unc)) return false;
            if (!rle_decode(z.data(), z.size(), r, want)) return false;
        } else if (rle_comp != 0 || rle_unc != 0) {
            return false;
        }
        size_t o = 0;
        for (size_t i = 0; i < nc; ++i) {
            if (scheme[i] != kRle) continue;
            const int tb = type_bytes(h.channels[i].type);
            plane[i].resize(W * L * tb);
            for (int k = 0; k < tb; ++k)
                for (size_t s = 0; s < W * L; ++s) plane[i][s * tb + k] = r[o + k * W * L + s];
            o += W * L * tb;
        }
    }
    // LOSSY_DCT
    const size_t bx = (W + 7) / 8, by = (L + 7) / 8, nb = bx * by;
    size_t n_dct = 0;
    for (size_t i = 0; i < nc; ++i) n_dct += scheme[i] == kLossyDct;
    if (dc_count != nb * n_dct || ac_count > (uint64_t)63 * nb * n_dct) return false;
    std::vector<uint16_t> ac((size_t)ac_count), dc((size_t)dc_count);
    if (n_dct > 0) {
        if (ac_mode == 0) {
            if (!piz::huf_uncompress(ac_p, (size_t)ac_comp, ac.data(), ac.size())) return false;
        } else {
            std::vector<uint8_t> t;
            if (!inflate_exact(ac_p, ac_comp, t, 2 * ac_count)) return false;
            std::memcpy(ac.data(), t.data(), t.size());
        }
        std::vector<uint8_t> t;
        if (!inflate_exact(dc_p, dc_comp, t, 2 * dc_count)) return false;
        std::vector<uint8_t> d(t.size());
        if (!t.empty()) unpredict_deinterleave(t, d.data());
        std::memcpy(dc.data(), d.data(), d.size());
    } else if (ac_count || dc_count || ac_comp || dc_comp) {
        return false;
    }
    // decoders: the colour sets, then the other lossy channels
    std::vector<std::vector<int>> decoders;
    for (const auto& s : sets) decoders.push_back({s[0], s[1], s[2]});
    for (size_t i = 0; i < nc; ++i)
        if (scheme[i] == kLossyDct && !in_set[i]) decoders.push_back({(int)i});
    const std::vector<uint16_t>& lin = to_linear();
    size_t ai = 0, di = 0;
    for (const auto& dec : decoders) {
        const size_t k = dec.size();
        for (int c : dec) plane[c].assign(W * L * type_bytes(h.channels[c].type), 0);
        for (size_t b = 0; b < nb; ++b) {
            float blk[3][64];
            for (size_t c = 0; c < k; ++c) {
                uint16_t z[64] = {};
                z[0] = dc[di + c * nb + b];
                int pos = 1;
                while (pos < 64) {
                    if (ai >= ac.size()) return false;
                    const uint16_t v = ac[ai++];
                    if (v == 0xff00) {
                        pos = 64;
                    } else if ((v >> 8) == 0xff) {
                        pos += v & 0xff;
                        if (pos > 64) return false;
                    } else {
                        z[pos++] = v;
                    }
                }
                for (int j = 0; j < 64; ++j) blk[c][kZigZag[j]] = half_to_float(z[j]);
                idct8x8(blk[c]);
            }
            if (k == 3) {
                for (int j = 0; j < 64; ++j) {
                    const float y = blk[0][j], cb = blk[1][j], cr = blk[2][j];
                    blk[0][j] = y + 1.5747f * cr;
                    blk[1][j] = y - 0.1873f * cb - 0.4682f * cr;
                    blk[2][j] = y + 1.8556f * cb;
                }
            }
            const size_t x0 = (b % bx) * 8, y0 = (b / bx) * 8;
            for (size_t c = 0; c < k; ++c)
                for (size_t dy = 0; dy < 8 && y0 + dy < L; ++dy)
                    for (size_t dx = 0; dx < 8 && x0 + dx < W; ++dx) {
                        const uint16_t v = lin[float_to_half(blk[c][dy * 8 + dx])];
                        if (h.channels[dec[c]].type == kFloat) {  // widened exactly
                            const float f = half_to_float(v);
                            std::memcpy(plane[dec[c]].data() + ((y0 + dy) * W + x0 + dx) * 4, &f, 4);
                        } else {
                            uint8_t* o = plane[dec[c]].data() + ((y0 + dy) * W + x0 + dx) * 2;
                            o[0] = (uint8_t)(v & 0xff);
                            o[1] = (uint8_t)(v >> 8);
                        }
                    }
        }
        di += k * nb;
    }
    if (ai != ac.size()) return false;
    // interleave per line, channel-list order
    uint8_t* o = raw.data();
    for (size_t y = 0; y < L; ++y)
        for (size_t i = 0; i < nc; ++i) {
            const size_t row = W * type_bytes(h.channels[i].type);
            std::memcpy(o, plane[i].data() + y * row, row);
            o += row;
        }
    return true;
}

}  // namespace dwa

// One chunk (scanline block, or tile) of `lines` lines x `width` pixels.
bool decode_chunk(const ExrHeader& h, const uint8_t* data, size_t size, size_t raw_size, int width, int lines,
                  std::vector<uint8_t>& raw) {
    const int compression = h.compression;
    raw.resize(raw_size);
    if (compression == BMFR_EXR_NONE || size == raw_size) {  // stored uncompressed
        if (size != raw_size) return false;
        std::memcpy(raw.data(), data, size);
        return true;
    }
    if (compression == BMFR_EXR_PIZ) {
        std::vector<int> words;
        for (const Channel& c : h.channels) words.push_back(type_bytes(c.type) / 2);
        return piz::uncompress(data, size, width, lines, words, raw) && raw.size() == raw_size;
    }
    if (compression == BMFR_EXR_PXR24) return pxr24_uncompress(h, data, size, width, lines, raw);
    if (compression == BMFR_EXR_B44 || compression == BMFR_EXR_B44A)
        return b44::uncompress(h, data, size, width, lines, raw);
    if (compression == BMFR_EXR_DWAA || compression == BMFR_EXR_DWAB)
        return dwa::uncompress(h, data, size, width, lines, raw);
    std::vector<uint8_t> t;
    if (compression == BMFR_EXR_RLE) {
        if (!rle_decode(data, size, t, raw_size)) return false;
    } else {  // ZIPS / ZIP
        t.resize(raw_size);
        uLongf n = (uLongf)raw_size;
        if (uncompress(t.data(), &n, data, (uLong)size) != Z_OK || n != raw_size) return false;
    }
    unpredict_deinterleave(t, raw.data());
    return true;
}

// ------------------------------------------------------------------ out --
void put_u32(std::vector<uint8_t>& b, uint32_t v) { b.insert(b.end(), (uint8_t*)&v, (uint8_t*)&v + 4); }
void put_i32(std::vector<uint8_t>& b, int32_t v) { b.insert(b.end(), (uint8_t*)&v, (uint8_t*)&v + 4); }
void put_f32(std::vector<uint8_t>& b, float v) { b.insert(b.end(), (uint8_t*)&v, (uint8_t*)&v + 4); }
void put_str(std::vector<uint8_t>& b, const char* s) { b.insert(b.end(), s, s + std::strlen(s) + 1); }
void put_attr(std::vector<uint8_t>& b, const char* name, const char* type, const std::vector<uint8_t>& v) {
    put_str(b, name);
    put_str(b, type);
    put_i32(b, (int32_t)v.size());
    b.insert(b.end(), v.begin(), v.end());
}

bool write_file(const char* path, const std::vector<uint8_t>& b) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    const bool ok = std::fwrite(b.data(), 1, b.size(), f) == b.size();
    return std::fclose(f) == 0 && ok;
}

void put_be32(std::vector<uint8_t>& b, uint32_t v) {
    const uint8_t x[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    b.insert(b.end(), x, x + 4);
}

void png_chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    put_be32(out, (uint32_t)data.size());
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put_be32(out, (uint32_t)crc32(0L, out.data() + start, (uInt)(out.size() - start)));
}

}  // namespace

extern "C" {

const char* bmfr_io_error(void) { return g_error.c_str(); }

int bmfr_exr_info(const char* path, int* width, int* height, int* channels) {
    std::vector<uint8_t> file;
    if (!read_file(path, file)) return fail(std::string("cannot read ") + path);
    ExrHeader h;
    size_t end = 0;
    std::string err;
    if (!parse_header(file, h, end, err)) return fail(std::string(path) + ": " + err);
    if (width) *width = h.width();
    if (height) *height = h.height();
    if (channels) *channels = (int)h.channels.size();
    return 0;
}

int bmfr_exr_read_rgb(const char* path, int width, int height, float* rgb) {
    std::vector<uint8_t> file;
    if (!read_file(path, file)) return fail(std::string("cannot read ") + path);
    ExrHeader h;
    size_t p = 0;
    std::string err;
    if (!parse_header(file, h, p, err)) return fail(std::string(path) + ": " + err);
    if (h.width() != width || h.height() != height)
        return fail(std::string(path) + ": image is " + std::to_string(h.width()) + "x" + std::to_string(h.height()));
    // Which stored channel feeds R, G, B.
    int src[3] = {-1, -1, -1};
    for (size_t i = 0; i < h.channels.size(); ++i) {
        const std::string& n = h.channels[i].name;
        const char last = n.empty() ? 0 : n.back();
        const bool plain = n.size() == 1 || (n.size() > 1 && n[n.size() - 2] == '.');
        if (plain && last == 'R') src[0] = (int)i;
        if (plain && last == 'G') src[1] = (int)i;
        if (plain && last == 'B') src[2] = (int)i;
    }
    if (src[0] < 0 || src[1] < 0 || src[2] < 0) {
        if (h.channels.size() != 3) return fail(std::string(path) + ": needs R, G, B channels");
        src[0] = 0, src[1] = 1, src[2] = 2;
    }
    // Rows [line0, line0 + lines) x columns [x0, x0 + w) of decoded chunk
    // data (per line: each channel's w samples) into the RGB buffer.
    auto scatter = [&](const std::vector<uint8_t>& raw, int x0, int w, int line0, int lines) {
        size_t line_bytes = 0;
        std::vector<size_t> ch_off(h.channels.size());
        for (size_t i = 0; i < h.channels.size(); ++i) {
            ch_off[i] = line_bytes;
            line_bytes += (size_t)w * type_bytes(h.channels[i].type);
        }
        for (int l = 0; l < lines; ++l) {
            const uint8_t* line = raw.data() + line_bytes * l;
            float* dst = rgb + ((size_t)(line0 + l) * width + x0) * 3;
            for (int k = 0; k < 3; ++k) {
                const Channel& ch = h.channels[src[k]];
                const uint8_t* s = line + ch_off[src[k]];
                for (int x = 0; x < w; ++x) {
                    float v;
                    if (ch.type == kHalf) {
                        uint16_t u;
                        std::memcpy(&u, s + 2 * x, 2);
                        v = half_to_float(u);
                    } else if (ch.type == kFloat) {
                        std::memcpy(&v, s + 4 * x, 4);
                    } else {
                        uint32_t u;
                        std::memcpy(&u, s + 4 * x, 4);
                        v = (float)u;
                    }
                    dst[3 * x + k] = v;
                }
            }
        }
    };
    size_t px_bytes = 0;  // all channels of one pixel
    for (const Channel& c : h.channels) px_bytes += type_bytes(c.type);
    std::vector<uint8_t> raw;
    g_chunk_unsupported.clear();
    if (h.tiled) {
        // Level (0, 0): the first nx * ny entries of the offset table (tiles
        // in row-major order; the other levels of a mip / rip map follow).
        const int64_t nx = ((int64_t)width + h.tile_w - 1) / h.tile_w, ny = ((int64_t)height + h.tile_h - 1) / h.tile_h;
        if (p > file.size() || (uint64_t)(nx * ny) > (file.size() - p) / 8) return fail(std::string(path) + ": truncated offset table");
        std::vector<uint8_t> seen((size_t)(nx * ny), 0);
        for (int64_t c = 0; c < nx * ny; ++c) {
            uint64_t off;
            std::memcpy(&off, file.data() + p + 8 * (size_t)c, 8);
            if (file.size() < 20 || off > file.size() - 20) return fail(std::string(path) + ": bad tile offset");
            int32_t hd[5];  // tile x, tile y, level x, level y, data size
            std::memcpy(hd, file.data() + off, 20);
            if (hd[0] < 0 || hd[0] >= nx || hd[1] < 0 || hd[1] >= ny || hd[2] != 0 || hd[3] != 0 || hd[4] < 0 ||
                (uint64_t)hd[4] > file.size() - off - 20 || seen[(size_t)(hd[1] * nx + hd[0])])
                return fail(std::string(path) + ": bad tile");
            seen[(size_t)(hd[1] * nx + hd[0])] = 1;
            const int x0 = (int)(hd[0] * (int64_t)h.tile_w), y0 = (int)(hd[1] * (int64_t)h.tile_h);
            const int w = std::min((int)h.tile_w, width - x0), lines = std::min((int)h.tile_h, height - y0);
            if (!decode_chunk(h, file.data() + off + 20, (size_t)hd[4], px_bytes * w * lines, w, lines, raw))
                return fail(std::string(path) + (g_chunk_unsupported.empty() ? ": corrupt tile " : ": unsupported: " +
                            g_chunk_unsupported + ", tile ") + std::to_string(hd[0]) + "," + std::to_string(hd[1]));
            scatter(raw, x0, w, y0, lines);
        }
        return 0;
    }
    const int lpc = lines_per_chunk(h.compression);
    const int chunks = (height + lpc - 1) / lpc;
    if (p > file.size() || (size_t)chunks > (file.size() - p) / 8) return fail(std::string(path) + ": truncated offset table");
    for (int c = 0; c < chunks; ++c) {
        uint64_t off;
        std::memcpy(&off, file.data() + p + 8 * (size_t)c, 8);
        // (compared without overflow: an offset near 2^64 must not wrap)
        if (file.size() < 8 || off > file.size() - 8) return fail(std::string(path) + ": bad chunk offset");
        int32_t y, size;
        std::memcpy(&y, file.data() + off, 4);
        std::memcpy(&size, file.data() + off + 4, 4);
        const int line0 = (int)((int64_t)y - h.y0);
        if ((int64_t)y - h.y0 < 0 || (int64_t)y - h.y0 >= height || size < 0 || (uint64_t)size > file.size() - off - 8)
            return fail(std::string(path) + ": bad chunk");
        const int lines = std::min(lpc, height - line0);
        if (!decode_chunk(h, file.data() + off + 8, (size_t)size, px_bytes * width * lines, width, lines, raw))
            return fail(std::string(path) + (g_chunk_unsupported.empty() ? ": corrupt chunk" : ": unsupported: " +
                        g_chunk_unsupported + ",") + " at y=" + std::to_string(y));
        scatter(raw, 0, width, line0, lines);
    }
    return 0;
}

int bmfr_exr_write_rgb(const char* path, int width, int height, const float* rgb, size_t stride,
                       bmfr_exr_compression compression) {
    if (width <= 0 || height <= 0 || !rgb || stride < (size_t)width * 3 ||
        (compression != BMFR_EXR_NONE && compression != BMFR_EXR_ZIP))
        return fail("bmfr_exr_write_rgb: bad arguments");
    std::vector<uint8_t> b;
    put_u32(b, kExrMagic);
    put_u32(b, 2);
    std::vector<uint8_t> v;
    for (const char* n : {"B", "G", "R"}) {  // channel list is sorted by name
        put_str(v, n);
        put_i32(v, kFloat);
        put_u32(v, 0);
        put_i32(v, 1);
        put_i32(v, 1);
    }
    v.push_back(0);
    put_attr(b, "channels", "chlist", v);
    put_attr(b, "compression", "compression", {(uint8_t)compression});
    v.clear();
    for (int x : {0, 0, width - 1, height - 1}) put_i32(v, x);
    put_attr(b, "dataWindow", "box2i", v);
    put_attr(b, "displayWindow", "box2i", v);
    put_attr(b, "lineOrder", "lineOrder", {0});
    v.clear();
    put_f32(v, 1.f);
    put_attr(b, "pixelAspectRatio", "float", v);
    v.clear();
    put_f32(v, 0.f);
    put_f32(v, 0.f);
    put_attr(b, "screenWindowCenter", "v2f", v);
    v.clear();
    put_f32(v, 1.f);
    put_attr(b, "screenWindowWidth", "float", v);
    b.push_back(0);
    const int lpc = lines_per_chunk(compression);
    const int chunks = (height + lpc - 1) / lpc;
    const size_t table = b.size();
    b.resize(b.size() + 8 * (size_t)chunks);
    const size_t line_bytes = (size_t)width * 4 * 3;
    std::vector<uint8_t> raw, t, z;
    for (int c = 0; c < chunks; ++c) {
        const int y0 = c * lpc, lines = std::min(lpc, height - y0);
        raw.resize(line_bytes * lines);
        for (int l = 0; l < lines; ++l) {
            const float* row = rgb + (size_t)(y0 + l) * stride;
            for (int k = 0; k < 3; ++k)  // B, G, R
                for (int x = 0; x < width; ++x)
                    std::memcpy(raw.data() + line_bytes * l + (size_t)k * width * 4 + 4 * (size_t)x, &row[3 * x + 2 - k], 4);
        }
        const uint8_t* data = raw.data();
        size_t size = raw.size();
        if (compression == BMFR_EXR_ZIP) {
            interleave_predict(raw.data(), raw.size(), t);
            uLongf zn = compressBound((uLong)t.size());
            z.resize(zn);
            if (compress2(z.data(), &zn, t.data(), (uLong)t.size(), Z_DEFAULT_COMPRESSION) != Z_OK)
                return fail("zlib compress failed");
            if (zn < raw.size()) {
                data = z.data();
                size = zn;
            }
        }
        const uint64_t off = b.size();
        std::memcpy(b.data() + table + 8 * (size_t)c, &off, 8);
        put_i32(b, y0);
        put_i32(b, (int32_t)size);
        b.insert(b.end(), data, data + size);
    }
    if (!write_file(path, b)) return fail(std::string("cannot write ") + path);
    return 0;
}

int bmfr_png_write_rgb(const char* path, int width, int height, const float* rgb, size_t stride) {
    if (width <= 0 || height <= 0 || !rgb || stride < (size_t)width * 3) return fail("bmfr_png_write_rgb: bad arguments");
    std::vector<uint8_t> rows((size_t)height * (1 + (size_t)width * 3));
    for (int y = 0; y < height; ++y) {
        uint8_t* r = rows.data() + (size_t)y * (1 + (size_t)width * 3);
        r[0] = 0;  // filter: none
        for (int i = 0; i < width * 3; ++i) {
            const float v = rgb[(size_t)y * stride + i];
            const float c = v > 0.f ? (v < 1.f ? v : 1.f) : 0.f;  // NaN -> 0
            r[1 + i] = (uint8_t)std::floor(c * 255.f + 0.5f);
        }
    }
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)width);
    put_be32(ihdr, (uint32_t)height);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
    png_chunk(out, "IHDR", ihdr);
    uLongf zn = compressBound((uLong)rows.size());
    std::vector<uint8_t> z(zn);
    if (compress2(z.data(), &zn, rows.data(), (uLong)rows.size(), 6) != Z_OK) return fail("zlib compress failed");
    z.resize(zn);
    png_chunk(out, "IDAT", z);
    png_chunk(out, "IEND", {});
    if (!write_file(path, out)) return fail(std::string("cannot write ") + path);
    return 0;
}

}  // extern "C"
