// png.cpp -- PNG codec on zlib (no libpng/stb headers in the image).
//
// Decode follows what stb_image does for stbi_loadf(..., req_comp = 4), the
// loader the reference uses for glTF images (src/stage1.zig:58): expansion to
// RGBA, 16-bit -> top byte, low-bit gray scaled by {255, 85, 17}, palette via
// PLTE/tRNS, and the channel count reported as stb's *comp (palette: 3 or 4
// with tRNS; otherwise the file's channels -- tRNS on gray/RGB adds alpha to
// the pixels but not to the count, which the reference's transparency test
// `actual_c == 4 or actual_c == 2` (stage1.zig:452) then sees).
#include "png.h"

#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <thread>
#include <vector>

#include "zrt_internal.h"

namespace zrt {

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
void put32(std::vector<uint8_t>* o, uint32_t v) {
    o->push_back((uint8_t)(v >> 24)); o->push_back((uint8_t)(v >> 16));
    o->push_back((uint8_t)(v >> 8)); o->push_back((uint8_t)v);
}
int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}
bool unfilter(uint8_t* data, size_t rows, size_t rowbytes, size_t bpp) {
    std::vector<uint8_t> prev(rowbytes, 0);
    for (size_t y = 0; y < rows; ++y) {
        uint8_t* line = data + y * (rowbytes + 1);
        const uint8_t f = line[0];
        uint8_t* cur = line + 1;
        for (size_t i = 0; i < rowbytes; ++i) {
            const int a = i >= bpp ? cur[i - bpp] : 0;
            const int b = prev[i];
            const int c = i >= bpp ? prev[i - bpp] : 0;
            int v = cur[i];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: return false;
            }
            cur[i] = (uint8_t)v;
        }
        memcpy(prev.data(), cur, rowbytes);
    }
    return true;
}

}  // namespace

int png_decode(const uint8_t* d, size_t n, Image8* out) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (n < 8 || memcmp(d, sig, 8) != 0) return ZRT_ERR_PARSE;
    size_t pos = 8;
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    bool have_trns = false;
    while (pos + 12 <= n) {
        const uint32_t len = be32(d + pos);
        if (len > n - pos - 12) return ZRT_ERR_PARSE;
        const uint8_t* tag = d + pos + 4;
        const uint8_t* body = d + pos + 8;
        if (!memcmp(tag, "IHDR", 4)) {
            if (len < 13) return ZRT_ERR_PARSE;
            w = be32(body); h = be32(body + 4);
            depth = body[8]; ctype = body[9]; interlace = body[12];
            if (body[10] != 0 || body[11] != 0) return ZRT_ERR_PARSE;
        } else if (!memcmp(tag, "PLTE", 4)) {
            plte.assign(body, body + len);
        } else if (!memcmp(tag, "tRNS", 4)) {
            trns.assign(body, body + len);
            have_trns = true;
        } else if (!memcmp(tag, "IDAT", 4)) {
            idat.insert(idat.end(), body, body + len);
        } else if (!memcmp(tag, "IEND", 4)) {
            break;
        }
        pos += 12 + len;
    }
    if (w == 0 || h == 0 || w > (1u << 24) || h > (1u << 24)) return ZRT_ERR_PARSE;
    int chans;
    switch (ctype) {
        case 0: chans = 1; break;
        case 2: chans = 3; break;
        case 3: chans = 1; break;
        case 4: chans = 2; break;
        case 6: chans = 4; break;
        default: return ZRT_ERR_PARSE;
    }
    if (!(depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) return ZRT_ERR_PARSE;
    if ((ctype == 2 || ctype == 4 || ctype == 6) && depth < 8) return ZRT_ERR_PARSE;
    if (ctype == 3 && (depth == 16 || plte.size() < 3)) return ZRT_ERR_PARSE;
    if (interlace > 1) return ZRT_ERR_PARSE;

    // passes: (x0, y0, dx, dy); non-interlaced = one pass
    struct Pass { int x0, y0, dx, dy; };
    static const Pass adam7[7] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                  {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    static const Pass single[1] = {{0, 0, 1, 1}};
    const Pass* passes = interlace ? adam7 : single;
    const int npass = interlace ? 7 : 1;
    const size_t bits_pp = (size_t)chans * depth;
    const size_t bpp = std::max<size_t>(1, bits_pp / 8);
    size_t total = 0;
    for (int k = 0; k < npass; ++k) {
        const size_t pw = (w > (uint32_t)passes[k].x0) ? (w - passes[k].x0 + passes[k].dx - 1) / passes[k].dx : 0;
        const size_t ph = (h > (uint32_t)passes[k].y0) ? (h - passes[k].y0 + passes[k].dy - 1) / passes[k].dy : 0;
        if (pw && ph) total += ph * (1 + (pw * bits_pp + 7) / 8);
    }
    // deflate expands at most ~1032:1: a header promising more than the
    // IDAT data can hold is corrupt (and must not drive a huge allocation)
    if ((uint64_t)w * h > (1ull << 27) || total > (size_t)1 << 31 || total > idat.size() * (size_t)1040 + 1024)
        return ZRT_ERR_PARSE;
    std::vector<uint8_t> raw(total);
    {
        z_stream zs;
        memset(&zs, 0, sizeof zs);
        if (inflateInit(&zs) != Z_OK) return ZRT_ERR_PARSE;
        zs.next_in = idat.data();
        zs.avail_in = (uInt)idat.size();
        zs.next_out = raw.data();
        zs.avail_out = (uInt)raw.size();
        const int rc = inflate(&zs, Z_FINISH);
        const size_t got = raw.size() - zs.avail_out;
        inflateEnd(&zs);
        if ((rc != Z_STREAM_END && rc != Z_BUF_ERROR && rc != Z_OK) || got != raw.size()) return ZRT_ERR_PARSE;
    }
    // sample fetch in the file's depth, scaled to 8 bits as stb does
    static const int scale[17] = {0, 0xff, 0x55, 0, 0x11, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1};
    out->w = (int)w;
    out->h = (int)h;
    out->rgba.assign((size_t)w * h * 4, 0);
    int trns_g = -1, trns_rgb[3] = {-1, -1, -1};
    if (have_trns && ctype == 0 && trns.size() >= 2) {
        const int v = (trns[0] << 8) | trns[1];
        trns_g = depth == 16 ? v : (v & 255) * scale[depth];
    }
    if (have_trns && ctype == 2 && trns.size() >= 6)
        for (int k = 0; k < 3; ++k) {
            const int v = (trns[2 * k] << 8) | trns[2 * k + 1];
            trns_rgb[k] = depth == 16 ? v : (v & 255);
        }
    size_t off = 0;
    for (int k = 0; k < npass; ++k) {
        const Pass& ps = passes[k];
        const size_t pw = (w > (uint32_t)ps.x0) ? (w - ps.x0 + ps.dx - 1) / ps.dx : 0;
        const size_t ph = (h > (uint32_t)ps.y0) ? (h - ps.y0 + ps.dy - 1) / ps.dy : 0;
        if (!pw || !ph) continue;
        const size_t rb = (pw * bits_pp + 7) / 8;
        if (!unfilter(raw.data() + off, ph, rb, bpp)) return ZRT_ERR_PARSE;
        for (size_t yy = 0; yy < ph; ++yy) {
            const uint8_t* row = raw.data() + off + yy * (rb + 1) + 1;
            for (size_t xx = 0; xx < pw; ++xx) {
                int s16[4] = {0, 0, 0, 0};   // raw samples in file depth
                for (int c = 0; c < chans; ++c) {
                    const size_t idx = xx * chans + c;
                    if (depth == 16) s16[c] = (row[2 * idx] << 8) | row[2 * idx + 1];
                    else if (depth == 8) s16[c] = row[idx];
                    else {
                        const size_t bit = idx * depth;
                        s16[c] = (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1 << depth) - 1);
                    }
                }
                const size_t px = ((size_t)(ps.y0 + yy * ps.dy) * w + ps.x0 + xx * ps.dx) * 4;
                uint8_t* o = &out->rgba[px];
                auto to8 = [&](int v) -> uint8_t { return depth == 16 ? (uint8_t)(v >> 8) : (uint8_t)(v * scale[depth]); };
                switch (ctype) {
                    case 0: {
                        const uint8_t g = to8(s16[0]);
                        o[0] = o[1] = o[2] = g;
                        const int cmp = depth == 16 ? s16[0] : g;
                        o[3] = (trns_g >= 0 && cmp == trns_g) ? 0 : 255;
                        break;
                    }
                    case 2: {
                        for (int c = 0; c < 3; ++c) o[c] = to8(s16[c]);
                        bool t = trns_rgb[0] >= 0;
                        for (int c = 0; c < 3 && t; ++c) t = s16[c] == trns_rgb[c];
                        o[3] = t ? 0 : 255;
                        break;
                    }
                    case 3: {
                        const int i = s16[0];
                        if ((size_t)(3 * i + 2) >= plte.size()) return ZRT_ERR_PARSE;
                        o[0] = plte[3 * i]; o[1] = plte[3 * i + 1]; o[2] = plte[3 * i + 2];
                        o[3] = (size_t)i < trns.size() ? trns[i] : 255;
                        break;
                    }
                    case 4: {
                        const uint8_t g = to8(s16[0]);
                        o[0] = o[1] = o[2] = g;
                        o[3] = to8(s16[1]);
                        break;
                    }
                    case 6:
                        for (int c = 0; c < 4; ++c) o[c] = to8(s16[c]);
                        break;
                }
            }
        }
        off += ph * (rb + 1);
    }
    out->actual_c = ctype == 3 ? (have_trns ? 4 : 3) : chans;
    return ZRT_OK;
}

int png_encode_rgb(const uint8_t* rgb, int w, int h, int level, std::vector<uint8_t>* out) {
    if (!rgb || w <= 0 || h <= 0 || !out) return ZRT_ERR_INVALID_ARG;
    const size_t rb = (size_t)w * 3;
    const size_t row = rb + 1;
    // zlib stream deflated in parallel: row-aligned pieces,
    // each filtered, deflated as a raw stream ended by a sync flush
    // (byte-aligned, non-final blocks) except the last, and checksummed on
    // its own thread; the pieces are concatenated behind one zlib header, the
    // Adler-32 of the whole and the IDAT CRC-32 combined from the pieces'.  A
    // valid single stream: any inflater (and stbi) reads it; only the file
    // bytes differ from a one-thread deflate (each piece starts with an empty
    // window).
    const unsigned hw = zrt::host_threads();
    const size_t min_piece = 256 * 1024;
    size_t np = std::min<size_t>(std::min<size_t>(hw, 32), std::max<size_t>(1, row * (size_t)h / min_piece));
    np = std::min<size_t>(np, (size_t)h);
    std::vector<std::vector<uint8_t>> zp(np);
    std::vector<uLong> ad(np, 0), cr(np, 0);
    std::vector<int> ok(np, 0);
    auto piece = [&](size_t k) {
        const size_t y0 = (size_t)h * k / np, y1 = (size_t)h * (k + 1) / np;
        const size_t len = (y1 - y0) * row;
        std::vector<uint8_t> raw(len);
        for (size_t y = y0; y < y1; ++y) {
            uint8_t* line = raw.data() + (y - y0) * row;
            line[0] = 1;   // Sub filter: cheap and compresses smooth images well
            const uint8_t* src = rgb + y * rb;
            line[1] = src[0];
            line[2] = src[1];
            line[3] = src[2];
            for (size_t i = 3; i < rb; ++i) line[1 + i] = (uint8_t)(src[i] - src[i - 3]);
        }
        z_stream zs;
        memset(&zs, 0, sizeof zs);
        if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return;
        zp[k].resize(deflateBound(&zs, (uLong)len) + 16);
        zs.next_in = raw.data();
        zs.avail_in = (uInt)len;
        zs.next_out = zp[k].data();
        zs.avail_out = (uInt)zp[k].size();
        const int r = deflate(&zs, k + 1 == np ? Z_FINISH : Z_SYNC_FLUSH);
        const bool done = k + 1 == np ? r == Z_STREAM_END : (r == Z_OK && zs.avail_in == 0);
        zp[k].resize(zs.total_out);
        deflateEnd(&zs);
        ad[k] = adler32(adler32(0L, Z_NULL, 0), raw.data(), (uInt)len);
        cr[k] = crc32(0L, zp[k].data(), (uInt)zp[k].size());
        ok[k] = done ? 1 : 0;
    };
    {
        std::vector<std::thread> th;
        for (size_t k = 1; k < np; ++k) th.emplace_back(piece, k);
        piece(0);
        for (auto& t : th) t.join();
    }
    size_t zn = 2 + 4;                        // zlib header + Adler-32
    uLong adl = adler32(0L, Z_NULL, 0);
    for (size_t k = 0; k < np; ++k) {
        if (!ok[k]) return ZRT_ERR_IO;
        zn += zp[k].size();
        const size_t y0 = (size_t)h * k / np, y1 = (size_t)h * (k + 1) / np;
        adl = adler32_combine(adl, ad[k], (z_off_t)((y1 - y0) * row));
    }
    out->clear();
    out->reserve(8 + 25 + 12 + zn + 12);
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    out->insert(out->end(), sig, sig + 8);
    auto chunk = [&](const char* tag, const uint8_t* body, size_t len) {
        put32(out, (uint32_t)len);
        const size_t s = out->size();
        out->insert(out->end(), tag, tag + 4);
        if (len) out->insert(out->end(), body, body + len);
        put32(out, (uint32_t)crc32(0, out->data() + s, (uInt)(len + 4)));
    };
    uint8_t ihdr[13];
    const uint32_t ww = (uint32_t)w, hh = (uint32_t)h;
    ihdr[0] = (uint8_t)(ww >> 24); ihdr[1] = (uint8_t)(ww >> 16); ihdr[2] = (uint8_t)(ww >> 8); ihdr[3] = (uint8_t)ww;
    ihdr[4] = (uint8_t)(hh >> 24); ihdr[5] = (uint8_t)(hh >> 16); ihdr[6] = (uint8_t)(hh >> 8); ihdr[7] = (uint8_t)hh;
    ihdr[8] = 8; ihdr[9] = 2; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    chunk("IHDR", ihdr, 13);
    // IDAT: "IDAT", zlib header, the pieces, Adler-32; its CRC from the
    // pieces' CRCs (crc32_combine), not a second pass over the bytes
    put32(out, (uint32_t)zn);
    static const uint8_t idat_head[6] = {'I', 'D', 'A', 'T', 0x78, 0x9C};   // CM 8, 32K window; FCHECK valid
    out->insert(out->end(), idat_head, idat_head + 6);
    uLong crc = crc32(0L, idat_head, 6);
    for (size_t k = 0; k < np; ++k) {
        out->insert(out->end(), zp[k].begin(), zp[k].end());
        crc = crc32_combine(crc, cr[k], (z_off_t)zp[k].size());
    }
    uint8_t tail[4] = {(uint8_t)(adl >> 24), (uint8_t)(adl >> 16), (uint8_t)(adl >> 8), (uint8_t)adl};
    out->insert(out->end(), tail, tail + 4);
    crc = crc32(crc, tail, 4);
    put32(out, (uint32_t)crc);
    chunk("IEND", nullptr, 0);
    return ZRT_OK;
}

int png_write_rgb(const char* path, const uint8_t* rgb, int w, int h, int level) {
    std::vector<uint8_t> buf;
    const int rc = png_encode_rgb(rgb, w, h, level, &buf);
    if (rc != ZRT_OK) return rc;
    FILE* f = fopen(path, "wb");
    if (!f) return ZRT_ERR_IO;
    const size_t wr = fwrite(buf.data(), 1, buf.size(), f);
    const int cl = fclose(f);
    return (wr == buf.size() && cl == 0) ? ZRT_OK : ZRT_ERR_IO;
}

void rgba8_to_linear(const Image8& img, std::vector<float>* o) {
    const size_t n = (size_t)img.w * img.h;
    o->resize(4 * n);
    for (size_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k)
            (*o)[4 * i + k] = (float)(pow((double)(img.rgba[4 * i + k] / 255.0f), (double)2.2f) * (double)1.0f);
        (*o)[4 * i + 3] = img.rgba[4 * i + 3] / 255.0f;
    }
}

}  // namespace zrt

// zlib level 3: on the rendered contest frame (1080p, 3 spp; tools/png_bench,
// 16 threads of the GPU host) 9.1 ms and the smallest file, against 13.6 ms
// at 6 and 8.1 ms (+1%) at 1
extern "C" int zrt_png_write(const char* path, const uint8_t* rgb, uint32_t w, uint32_t h) {
    return zrt::png_write_rgb(path, rgb, (int)w, (int)h, 3);
}
