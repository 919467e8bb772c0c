// image_io.cpp -- OpenEXR (scanline, NONE/RLE/ZIPS/ZIP) and PNG I/O over zlib.
// See image_io.h.  The EXR layout follows the published OpenEXR 2 file
// format: magic + version, attribute list, per-chunk offset table, chunks of
// (y, size, data) with each scanline's channels stored in channel-list order.
#include "image_io.h"

#include <zlib.h>

#include <algorithm>
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
};

struct ExrHeader {
    std::vector<Channel> channels;
    int compression = -1;
    int x0 = 0, y0 = 0, x1 = -1, y1 = -1;
    int line_order = 0;
    bool tiled = false;
    int width() const { return x1 - x0 + 1; }
    int height() const { return y1 - y0 + 1; }
};

int lines_per_chunk(int compression) {
    switch (compression) {
        case BMFR_EXR_NONE: case BMFR_EXR_RLE: case BMFR_EXR_ZIPS: return 1;
        case BMFR_EXR_ZIP: return 16;
        default: return 0;  // PIZ (4), PXR24 (5), B44 (6, 7), DWAA/B (8, 9): unsupported
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
                r.get<uint32_t>();  // pLinear + reserved
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
        }
        r.p = next;
    }
    end = r.p;
    if (h.tiled) return err = "tiled OpenEXR files are not supported", false;
    if (lines_per_chunk(h.compression) == 0) return err = "unsupported OpenEXR compression " + std::to_string(h.compression), false;
    // data window extents in 64-bit (x1 - x0 overflows int for hostile corners)
    const int64_t w64 = (int64_t)h.x1 - h.x0 + 1, h64 = (int64_t)h.y1 - h.y0 + 1;
    if (h.channels.empty() || w64 <= 0 || h64 <= 0 || w64 > (1 << 20) || h64 > (1 << 20) ||
        h.channels.size() > 1024)
        return err = "bad channels / data window", false;
    for (const Channel& c : h.channels)
        if (c.xs != 1 || c.ys != 1 || c.type < 0 || c.type > 2) return err = "subsampled or unknown channel " + c.name, false;
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

bool decode_chunk(int compression, const uint8_t* data, size_t size, size_t raw_size, std::vector<uint8_t>& raw) {
    raw.resize(raw_size);
    if (compression == BMFR_EXR_NONE || size == raw_size) {  // stored uncompressed
        if (size != raw_size) return false;
        std::memcpy(raw.data(), data, size);
        return true;
    }
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
    size_t line_bytes = 0;
    std::vector<size_t> ch_off(h.channels.size());
    for (size_t i = 0; i < h.channels.size(); ++i) {
        ch_off[i] = line_bytes;
        line_bytes += (size_t)width * type_bytes(h.channels[i].type);
    }
    const int lpc = lines_per_chunk(h.compression);
    const int chunks = (height + lpc - 1) / lpc;
    if (p > file.size() || (size_t)chunks > (file.size() - p) / 8) return fail(std::string(path) + ": truncated offset table");
    std::vector<uint8_t> raw;
    for (int c = 0; c < chunks; ++c) {
        uint64_t off;
        std::memcpy(&off, file.data() + p + 8 * (size_t)c, 8);
        // (compared without overflow: an offset near 2^64 must not wrap)
        if (file.size() < 8 || off > file.size() - 8) return fail(std::string(path) + ": bad chunk offset");
        int32_t y, size;
        std::memcpy(&y, file.data() + off, 4);
        std::memcpy(&size, file.data() + off + 4, 4);
        const int line0 = y - h.y0;
        if (line0 < 0 || line0 >= height || size < 0 || (uint64_t)size > file.size() - off - 8)
            return fail(std::string(path) + ": bad chunk");
        const int lines = std::min(lpc, height - line0);
        if (!decode_chunk(h.compression, file.data() + off + 8, (size_t)size, line_bytes * lines, raw))
            return fail(std::string(path) + ": corrupt chunk at y=" + std::to_string(y));
        for (int l = 0; l < lines; ++l) {
            const uint8_t* line = raw.data() + line_bytes * l;
            float* dst = rgb + (size_t)(line0 + l) * width * 3;
            for (int k = 0; k < 3; ++k) {
                const Channel& ch = h.channels[src[k]];
                const uint8_t* s = line + ch_off[src[k]];
                for (int x = 0; x < width; ++x) {
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
