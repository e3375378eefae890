// vcf_png.cpp -- native PNG reader for the frame-ingest path (host code in
// libvcf_amd.so).
//
// Replaces the image read of EIC.encode_read_fn (src/entropy_image_coding.py
// :51-65: cv2.imread(IMREAD_UNCHANGED) + BGR2RGB, assumption A9: the same RGB
// array PIL's convert("RGB") gives) for the PNGs the III runner ingests
// (/tmp/original_%04d.png, III.py:73-89).  SURVEY.md §8(f) row 1: once the
// kernels run near the HBM roofline, host PNG decoding bounds the end-to-end
// rate; PIL's decoder spends ~55-70 ms on a 1080p frame, this one ~2-3x less
// (one inflate of the concatenated IDAT data, row unfiltering in place).
//
// Covered: the colour images the reference reads as RGB -- bit depth 8 RGB
// (type 2) and RGBA (type 6, alpha dropped: cv2 BGR2RGB of a 4-channel image),
// palette images (type 3, depth 1/2/4/8, looked up: libpng expands them), no
// interlace -- as PIL's convert("RGB") gives them.  Gray images are not
// colour frames to the reference (cvtColor(BGR2RGB) of a 2-D array fails,
// entropy_image_coding.py:55-60): like 16-bit and Adam7 files they return
// VCF_ERR_UNSUPPORTED and the caller reads them the generic way.  Chunk CRCs
// are verified; a corrupt file is VCF_ERR_INVALID.
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "vcf_amd.h"
#include "vcf_internal.h"

namespace vcf {
namespace {

// libdeflate's decompressor and crc32, resolved once (null members: absent)
struct Libdeflate {
    void *(*alloc_decompressor)() = nullptr;
    void (*free_decompressor)(void *) = nullptr;
    int (*zlib_decompress_ex)(void *, const void *, size_t, void *, size_t, size_t *, size_t *) = nullptr;
    uint32_t (*crc32)(uint32_t, const void *, size_t) = nullptr;
    bool ok() const { return alloc_decompressor && free_decompressor && zlib_decompress_ex && crc32; }
};

const Libdeflate &libdeflate()
{
    static const Libdeflate L = [] {
        Libdeflate l;
        const char *off = getenv("VCF_PNG_NO_LIBDEFLATE");   // tests: force the zlib path
        if (off && *off && *off != '0') return l;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return l;
        l.alloc_decompressor = reinterpret_cast<void *(*)()>(dlsym(h, "libdeflate_alloc_decompressor"));
        l.free_decompressor = reinterpret_cast<void (*)(void *)>(dlsym(h, "libdeflate_free_decompressor"));
        l.zlib_decompress_ex = reinterpret_cast<int (*)(void *, const void *, size_t, void *, size_t, size_t *,
                                                        size_t *)>(dlsym(h, "libdeflate_zlib_decompress_ex"));
        l.crc32 = reinterpret_cast<uint32_t (*)(uint32_t, const void *, size_t)>(dlsym(h, "libdeflate_crc32"));
        return l;
    }();
    return L;
}

// one decompressor per thread (the III runner reads frames on a pool)
struct Inflater {
    void *d = nullptr;
    ~Inflater() { if (d) libdeflate().free_decompressor(d); }
};

uint32_t chunk_crc(const uint8_t *p, size_t n)
{
    const Libdeflate &L = libdeflate();
    if (L.ok()) return L.crc32(0, p, n);
    return (uint32_t)crc32(crc32(0L, Z_NULL, 0), p, (uInt)n);
}

// the whole zlib stream of the IDAT data into out (exactly out_len bytes);
// false: libdeflate absent or the stream not clean (the zlib path then
// reports the precise error)
bool inflate_libdeflate(const std::vector<std::pair<const uint8_t *, uint32_t>> &idat, uint8_t *out, size_t out_len)
{
    const Libdeflate &L = libdeflate();
    if (!L.ok()) return false;
    thread_local Inflater inf;
    if (!inf.d) inf.d = L.alloc_decompressor();
    if (!inf.d) return false;
    thread_local std::vector<uint8_t> joined;
    const uint8_t *in = idat.empty() ? nullptr : idat[0].first;
    size_t in_len = idat.empty() ? 0 : idat[0].second;
    if (idat.size() > 1) {
        size_t tot = 0;
        for (const auto &c : idat) tot += c.second;
        joined.resize(tot);
        size_t at = 0;
        for (const auto &c : idat) { std::memcpy(joined.data() + at, c.first, c.second); at += c.second; }
        in = joined.data();
        in_len = tot;
    }
    if (!in) return false;
    size_t used = 0, got = 0;
    const int r = L.zlib_decompress_ex(inf.d, in, in_len, out, out_len, &used, &got);
    return r == 0 && got == out_len;   // LIBDEFLATE_SUCCESS, every scanline byte
}

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

struct PngHeader {
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0;
    int channels() const { return ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : 4; }
    bool covered() const
    {
        if (interlace != 0) return false;
        if (depth == 8) return ctype == 2 || ctype == 3 || ctype == 6;
        return (depth == 1 || depth == 2 || depth == 4) && ctype == 3;
    }
};

const uint8_t kSig[8] = {137, 80, 78, 71, 13, 10, 26, 10};

// Walk the chunks: header, palette, IDAT pieces (pointers into data).
int parse(const uint8_t *data, int64_t n, PngHeader &h, const uint8_t **plte, uint32_t *plte_len,
          std::vector<std::pair<const uint8_t *, uint32_t>> *idat)
{
    if (!data || n < 8 + 25 || std::memcmp(data, kSig, 8) != 0) return set_error(VCF_ERR_INVALID, "not a PNG file");
    int64_t off = 8;
    bool have_ihdr = false, have_iend = false;
    while (off + 12 <= n) {
        const uint32_t len = be32(data + off);
        const uint8_t *type = data + off + 4;
        if (len > (uint32_t)0x7fffffff || off + 12 + (int64_t)len > n)
            return set_error(VCF_ERR_INVALID, "truncated PNG chunk");
        const uint8_t *body = data + off + 8;
        const uint32_t crc = be32(body + len);
        if (chunk_crc(type, 4 + (size_t)len) != crc)
            return set_error(VCF_ERR_INVALID, "broken PNG file (chunk CRC)");
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13) return set_error(VCF_ERR_INVALID, "bad IHDR");
            h.w = be32(body);
            h.h = be32(body + 4);
            h.depth = body[8];
            h.ctype = body[9];
            h.interlace = body[12];
            if (body[10] != 0 || body[11] != 0) return set_error(VCF_ERR_INVALID, "bad PNG compression/filter method");
            have_ihdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            if (plte) { *plte = body; *plte_len = len; }
        } else if (!std::memcmp(type, "IDAT", 4)) {
            if (idat) idat->push_back({body, len});
        } else if (!std::memcmp(type, "IEND", 4)) {
            have_iend = true;
            break;
        }
        off += 12 + (int64_t)len;
    }
    if (!have_ihdr) return set_error(VCF_ERR_INVALID, "PNG without IHDR");
    if (idat && !have_iend) return set_error(VCF_ERR_INVALID, "truncated PNG (no IEND)");
    if (h.w == 0 || h.h == 0) return set_error(VCF_ERR_INVALID, "empty PNG");
    return VCF_OK;
}

inline uint8_t paeth(int a, int b, int c)
{
    const int p = a + b - c;
    const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    return pb <= pc ? (uint8_t)b : (uint8_t)c;
}

// PNG filters 0..4 (ISO 15948 §9) on one scanline, bpp bytes per pixel
int unfilter(uint8_t *row, const uint8_t *prev, size_t len, int bpp, int ftype)
{
    switch (ftype) {
    case 0: return VCF_OK;
    case 1:
        if (bpp == 3) {   // the running pixel in registers: no store-to-load chain through memory
            uint8_t a = 0, b = 0, c = 0;
            for (size_t i = 0; i + 2 < len; i += 3) {
                a = (uint8_t)(a + row[i]); b = (uint8_t)(b + row[i + 1]); c = (uint8_t)(c + row[i + 2]);
                row[i] = a; row[i + 1] = b; row[i + 2] = c;
            }
            return VCF_OK;
        }
        for (size_t i = bpp; i < len; ++i) row[i] = (uint8_t)(row[i] + row[i - bpp]);
        return VCF_OK;
    case 2:
        if (prev) for (size_t i = 0; i < len; ++i) row[i] = (uint8_t)(row[i] + prev[i]);
        return VCF_OK;
    case 3:
        for (size_t i = 0; i < len; ++i) {
            const int a = i >= (size_t)bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
            row[i] = (uint8_t)(row[i] + ((a + b) >> 1));
        }
        return VCF_OK;
    case 4:
        for (size_t i = 0; i < len; ++i) {
            const int a = i >= (size_t)bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
            const int c = (prev && i >= (size_t)bpp) ? prev[i - bpp] : 0;
            row[i] = (uint8_t)(row[i] + paeth(a, b, c));
        }
        return VCF_OK;
    default: return set_error(VCF_ERR_INVALID, "bad PNG filter type %d", ftype);
    }
}

void put32(std::vector<uint8_t> &o, uint32_t v)
{
    o.push_back((uint8_t)(v >> 24)); o.push_back((uint8_t)(v >> 16)); o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

void put_chunk(std::vector<uint8_t> &o, const char *type, const uint8_t *body, size_t len)
{
    put32(o, (uint32_t)len);
    const size_t at = o.size();
    o.insert(o.end(), (const uint8_t *)type, (const uint8_t *)type + 4);
    if (len) o.insert(o.end(), body, body + len);
    put32(o, (uint32_t)crc32(0L, o.data() + at, (uInt)(len + 4)));
}

// One piece of a pigz-style parallel deflate: raw deflate of in[0, n) primed
// with the preceding 32 KiB as dictionary, ended by a sync flush (or the
// final block).
int deflate_piece(const uint8_t *dict, size_t ndict, const uint8_t *in, size_t n, int level, bool last,
                  std::vector<uint8_t> &out)
{
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
    if (ndict && deflateSetDictionary(&zs, dict, (uInt)ndict) != Z_OK) { deflateEnd(&zs); return -1; }
    out.resize(deflateBound(&zs, (uLong)n) + 64);
    zs.next_in = const_cast<Bytef *>(in);
    zs.avail_in = (uInt)n;
    zs.next_out = out.data();
    zs.avail_out = (uInt)out.size();
    const int zr = deflate(&zs, last ? Z_FINISH : Z_SYNC_FLUSH);
    const bool ok = last ? zr == Z_STREAM_END : (zr == Z_OK && zs.avail_in == 0);
    out.resize(out.size() - zs.avail_out);
    deflateEnd(&zs);
    return ok ? 0 : -1;
}

}  // namespace
}  // namespace vcf

using namespace vcf;

extern "C" {

int vcf_png_info(const uint8_t *data, int64_t nbytes, int32_t *H, int32_t *W, int32_t *supported)
{
    PngHeader h;
    int rc = parse(data, nbytes, h, nullptr, nullptr, nullptr);
    if (rc != VCF_OK) return rc;
    if (H) *H = (int32_t)h.h;
    if (W) *W = (int32_t)h.w;
    if (supported) *supported = h.covered() ? 1 : 0;
    return VCF_OK;
}

int vcf_png_decode_rgb(const uint8_t *data, int64_t nbytes, uint8_t *rgb_out, int64_t out_capacity)
{
    PngHeader h;
    const uint8_t *plte = nullptr;
    uint32_t plte_len = 0;
    std::vector<std::pair<const uint8_t *, uint32_t>> idat;
    int rc = parse(data, nbytes, h, &plte, &plte_len, &idat);
    if (rc != VCF_OK) return rc;
    if (!h.covered())
        return set_error(VCF_ERR_UNSUPPORTED, "PNG depth %d colour type %d interlace %d", h.depth, h.ctype,
                         h.interlace);
    if (!rgb_out) return set_error(VCF_ERR_INVALID, "null output");
    const int bpp = h.depth == 8 ? h.channels() : 1;   // filter unit: bytes per pixel, at least 1
    const size_t stride = h.depth == 8 ? (size_t)h.w * bpp : ((size_t)h.w * h.depth + 7) / 8;
    const size_t need = (size_t)h.h * h.w * 3;
    if ((int64_t)need > out_capacity) return set_error(VCF_ERR_INVALID, "output buffer too small");
    if (h.ctype == 3 && (!plte || plte_len % 3 != 0)) return set_error(VCF_ERR_INVALID, "palette PNG without PLTE");

    // inflate all IDAT data into filtered scanlines (1 filter byte + stride);
    // the buffer is kept per thread (no zero fill, no fresh pages per frame)
    thread_local std::vector<uint8_t> raw;
    raw.resize((stride + 1) * h.h);
    if (!inflate_libdeflate(idat, raw.data(), raw.size())) {
        z_stream zs;
        std::memset(&zs, 0, sizeof(zs));
        if (inflateInit(&zs) != Z_OK) return set_error(VCF_ERR_INVALID, "inflateInit failed");
        zs.next_out = raw.data();
        zs.avail_out = (uInt)raw.size();
        int zr = Z_OK;
        for (size_t c = 0; c < idat.size() && zr != Z_STREAM_END; ++c) {
            zs.next_in = const_cast<Bytef *>(idat[c].first);
            zs.avail_in = idat[c].second;
            while (zs.avail_in > 0 && zs.avail_out > 0) {
                zr = inflate(&zs, Z_NO_FLUSH);
                if (zr == Z_STREAM_END) break;
                if (zr != Z_OK && zr != Z_BUF_ERROR) {
                    inflateEnd(&zs);
                    return set_error(VCF_ERR_INVALID, "broken PNG data stream (zlib %d)", zr);
                }
                if (zr == Z_BUF_ERROR) break;
            }
        }
        const size_t got = raw.size() - zs.avail_out;
        inflateEnd(&zs);
        if (got != raw.size()) return set_error(VCF_ERR_INVALID, "image file is truncated (%zu of %zu bytes)", got,
                                                raw.size());
    }

    // unfilter in place, then expand to RGB
    const uint8_t *prev = nullptr;
    for (uint32_t y = 0; y < h.h; ++y) {
        uint8_t *line = raw.data() + (size_t)y * (stride + 1);
        rc = unfilter(line + 1, prev, stride, bpp, line[0]);
        if (rc != VCF_OK) return rc;
        prev = line + 1;
        const uint8_t *s = line + 1;
        uint8_t *d = rgb_out + (size_t)y * h.w * 3;
        if (h.depth < 8) {   // packed samples, most significant bits first
            const int per = 8 / h.depth, mask = (1 << h.depth) - 1;
            for (uint32_t x = 0; x < h.w; ++x) {
                const int v = (s[x / per] >> ((per - 1 - (int)(x % per)) * h.depth)) & mask;
                if (3u * v + 2 < plte_len) {
                    d[3 * x] = plte[3 * v]; d[3 * x + 1] = plte[3 * v + 1]; d[3 * x + 2] = plte[3 * v + 2];
                } else {
                    d[3 * x] = d[3 * x + 1] = d[3 * x + 2] = 0;
                }
            }
            continue;
        }
        switch (h.ctype) {
        case 2: std::memcpy(d, s, stride); break;
        case 6:
            for (uint32_t x = 0; x < h.w; ++x) { d[3 * x] = s[4 * x]; d[3 * x + 1] = s[4 * x + 1]; d[3 * x + 2] = s[4 * x + 2]; }
            break;
        case 0:
            for (uint32_t x = 0; x < h.w; ++x) d[3 * x] = d[3 * x + 1] = d[3 * x + 2] = s[x];
            break;
        case 4:
            for (uint32_t x = 0; x < h.w; ++x) d[3 * x] = d[3 * x + 1] = d[3 * x + 2] = s[2 * x];
            break;
        case 3:
            for (uint32_t x = 0; x < h.w; ++x) {
                const uint32_t i = s[x];
                if (3 * i + 2 < plte_len) { d[3 * x] = plte[3 * i]; d[3 * x + 1] = plte[3 * i + 1]; d[3 * x + 2] = plte[3 * i + 2]; }
                else { d[3 * x] = d[3 * x + 1] = d[3 * x + 2] = 0; }
            }
            break;
        }
    }
    return VCF_OK;
}

/* RGB u8 (H x W x 3) -> a PNG file image: 8-bit truecolour, no interlace,
 * every scanline "Up"-filtered, one zlib stream deflated at `level` in
 * pieces on up to `threads` threads (each piece primed with the previous
 * 32 KiB, joined by sync flushes, adler32 combined: pigz's construction).
 * The writer the decode side uses for its PNGs (EIC.decode_write_fn,
 * entropy_image_coding.py:101-112) and IPP for its frame dumps: pixel-exact,
 * though not byte-identical to another library's PNG writer. */
int vcf_png_encode_rgb(const uint8_t *rgb, int32_t H, int32_t W, int32_t level, int32_t threads, uint8_t *out,
                       int64_t out_capacity, int64_t *out_bytes)
{
    if (!rgb || !out_bytes || H <= 0 || W <= 0) return set_error(VCF_ERR_INVALID, "bad PNG encode arguments");
    if (level < 0 || level > 9) return set_error(VCF_ERR_INVALID, "zlib level %d", level);
    const size_t stride = (size_t)W * 3, raw_len = (stride + 1) * (size_t)H;
    std::vector<uint8_t> raw(raw_len);
    for (int32_t y = 0; y < H; ++y) {
        uint8_t *d = raw.data() + (size_t)y * (stride + 1);
        const uint8_t *s = rgb + (size_t)y * stride;
        if (y == 0) {
            d[0] = 0;
            std::memcpy(d + 1, s, stride);
        } else {
            d[0] = 2;   // Up
            const uint8_t *p = s - stride;
            for (size_t i = 0; i < stride; ++i) d[1 + i] = (uint8_t)(s[i] - p[i]);
        }
    }
    const size_t kPiece = 1u << 20;
    const size_t npieces = std::max<size_t>(1, (raw_len + kPiece - 1) / kPiece);
    std::vector<std::vector<uint8_t>> parts(npieces);
    std::vector<int> rcs(npieces, 0);
    const int nth = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(1, threads), npieces));
    auto work = [&](int t) {
        for (size_t i = (size_t)t; i < npieces; i += (size_t)nth) {
            const size_t a = i * kPiece, b = std::min(raw_len, a + kPiece);
            const size_t nd = std::min<size_t>(a, 32768);
            rcs[i] = deflate_piece(raw.data() + a - nd, nd, raw.data() + a, b - a, level, i + 1 == npieces, parts[i]);
        }
    };
    if (nth == 1) {
        work(0);
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < nth; ++t) pool.emplace_back(work, t);
        for (auto &th : pool) th.join();
    }
    for (int r : rcs)
        if (r) return set_error(VCF_ERR_INVALID, "deflate failed");
    // zlib stream: header, the pieces, adler32 of the whole scanline buffer
    uLong adler = adler32(0L, Z_NULL, 0);
    for (size_t i = 0; i < npieces; ++i) {
        const size_t a = i * kPiece, b = std::min(raw_len, a + kPiece);
        adler = adler32_combine(adler, adler32(1L, raw.data() + a, (uInt)(b - a)), (z_off_t)(b - a));
    }
    std::vector<uint8_t> z;
    z.push_back(0x78);
    z.push_back(level >= 7 ? 0xDA : level >= 6 ? 0x9C : level >= 2 ? 0x5E : 0x01);
    for (auto &p : parts) z.insert(z.end(), p.begin(), p.end());
    put32(z, (uint32_t)adler);

    std::vector<uint8_t> png(kSig, kSig + 8);
    uint8_t ihdr[13];
    ihdr[0] = (uint8_t)(W >> 24); ihdr[1] = (uint8_t)(W >> 16); ihdr[2] = (uint8_t)(W >> 8); ihdr[3] = (uint8_t)W;
    ihdr[4] = (uint8_t)(H >> 24); ihdr[5] = (uint8_t)(H >> 16); ihdr[6] = (uint8_t)(H >> 8); ihdr[7] = (uint8_t)H;
    ihdr[8] = 8; ihdr[9] = 2; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    put_chunk(png, "IHDR", ihdr, 13);
    const size_t kIdat = 1u << 20;
    for (size_t a = 0; a < z.size(); a += kIdat) put_chunk(png, "IDAT", z.data() + a, std::min(kIdat, z.size() - a));
    put_chunk(png, "IEND", nullptr, 0);
    *out_bytes = (int64_t)png.size();
    if (!out || (int64_t)png.size() > out_capacity) return set_error(VCF_ERR_INVALID, "output buffer too small");
    std::memcpy(out, png.data(), png.size());
    return VCF_OK;
}

int64_t vcf_png_encode_bound(int32_t H, int32_t W)
{
    if (H <= 0 || W <= 0) return 0;
    const int64_t raw = ((int64_t)W * 3 + 1) * H;
    return raw + raw / 8 + ((raw >> 20) + 2) * 96 + 4096;
}

}  // extern "C"
