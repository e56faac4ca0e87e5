// jpeg.cpp -- JPEG textures for the glTF loader: the
// reference decodes every glTF image with stb_image's stbi_loadf_from_memory
// (src/stage1.zig:58), whose JPEG path is what this file provides.
//
// ITU-T T.81 Huffman JPEG: baseline and extended sequential (SOF0/SOF1) and
// progressive (SOF2, spectral selection + successive approximation), 8-bit
// samples, 1 or 3 components, any sampling factors up to 4x4, restart
// intervals, Adobe APP14 RGB.  Decoding: coefficients of all scans into
// per-component block planes, then dequantisation, an integer separable IDCT
// (Loeffler-Ligtenberg-Moschytz flow, 13-bit constants, 2 extra bits between
// passes), triangle-filter chroma upsampling for 2x factors (replication for
// others) and BT.601 full-range YCbCr -> RGB in 20-bit fixed point.  Output
// is RGBA8 (alpha 255); the caller applies stb's loadf gamma like for PNG.
//
// Parity: stb_image is an un-vendored submodule (empty in the reference), so
// its exact integer rounding is not available to pin against: JPEG texels
// are "parity unpinned" (DESIGN.md §2); tests compare with an independent
// decoder within a small per-channel tolerance.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "png.h"
#include "zrt_internal.h"

namespace zrt {
namespace {

// natural index of the k-th coefficient in zigzag order
const uint8_t kZig[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    // overrun guard for corrupt streams: extra positions land on 63
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huff {
    bool defined = false;
    uint8_t val[256];
    int mincode[17], maxcode[18], valptr[17];
    uint16_t fast[512];   // 9-bit lookahead: (len << 8) | value, 0 = slow path
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0;
    int bw = 0, bh = 0;            // blocks per row / column (whole MCUs)
    int cw = 0, ch = 0;            // blocks covering the component's own size
    std::vector<int16_t> coef;     // bw*bh blocks x 64, natural order, quantised
    std::vector<uint8_t> pix;      // bw*8 x bh*8 samples
    int dc_pred = 0;
    int td = 0, ta = 0;
};

struct Decoder {
    const uint8_t* p;
    size_t n, pos = 0;
    uint64_t bits = 0;
    int nbits = 0;
    bool marker_hit = false;
    uint16_t q[4][64];             // zigzag order
    bool q_defined[4] = {false, false, false, false};
    Huff dc[4], ac[4];
    Comp comp[3];
    int ncomp = 0, width = 0, height = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool progressive = false, have_frame = false, adobe_rgb = false, adobe_seen = false;
    int restart = 0, eobrun = 0;

    int u8() { return pos < n ? p[pos++] : -1; }
    int u16() {
        const int a = u8(), b = u8();
        return (a < 0 || b < 0) ? -1 : (a << 8) | b;
    }

    // entropy-coded data: 0xFF00 is a data 0xFF; any other marker stops input
    void fill() {
        while (nbits <= 56) {
            int b = 0;
            if (!marker_hit && pos < n) {
                b = p[pos];
                if (b == 0xFF) {
                    const int nx = pos + 1 < n ? p[pos + 1] : 0xD9;
                    if (nx == 0) {
                        pos += 2;
                    } else {
                        marker_hit = true;
                        b = 0;
                    }
                } else {
                    ++pos;
                }
            }
            bits |= (uint64_t)b << (56 - nbits);
            nbits += 8;
        }
    }
    int getbits(int k) {
        if (k == 0) return 0;
        if (nbits < k) fill();
        const int v = (int)(bits >> (64 - k));
        bits <<= k;
        nbits -= k;
        return v;
    }
    int getbit() { return getbits(1); }
    // T.81 F.12 EXTEND
    static int extend(int v, int s) { return s == 0 ? 0 : (v < (1 << (s - 1)) ? v - (1 << s) + 1 : v); }
    int receive_extend(int s) { return extend(getbits(s), s); }

    int decode(const Huff& h) {
        if (nbits < 16) fill();
        const uint16_t f = h.fast[bits >> (64 - 9)];
        if (f) {
            const int len = f >> 8;
            bits <<= len;
            nbits -= len;
            return f & 0xFF;
        }
        int code = 0;
        for (int l = 1; l <= 16; ++l) {
            code = (code << 1) | getbit();
            if (code <= h.maxcode[l]) return h.val[h.valptr[l] + code - h.mincode[l]];
        }
        return -1;   // corrupt
    }

    void reset_entropy() {
        bits = 0;
        nbits = 0;
        marker_hit = false;
        for (int i = 0; i < ncomp; ++i) comp[i].dc_pred = 0;
        eobrun = 0;
    }
    // after an interval: skip to the RSTn marker (and past it)
    bool restart_marker() {
        while (pos + 1 < n && !(p[pos] == 0xFF && p[pos + 1] >= 0xD0 && p[pos + 1] <= 0xD7)) ++pos;
        if (pos + 1 >= n) return false;
        pos += 2;
        reset_entropy();
        return true;
    }

    bool build_huff(Huff& h, const uint8_t counts[16], const uint8_t* vals, int total) {
        memcpy(h.val, vals, total);
        int code = 0, k = 0;
        memset(h.fast, 0, sizeof h.fast);
        for (int l = 1; l <= 16; ++l) {
            h.valptr[l] = k;
            h.mincode[l] = code;
            for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
                if (code >= (1 << l)) return false;        // over-subscribed: not a prefix code
                if (l <= 9) {
                    const int shift = 9 - l;
                    for (int j = 0; j < (1 << shift); ++j)
                        h.fast[(code << shift) | j] = (uint16_t)((l << 8) | vals[k]);
                }
            }
            h.maxcode[l] = counts[l - 1] ? code - 1 : -1;
            if (code > (1 << l)) return false;
            code <<= 1;
        }
        h.maxcode[17] = 0x7FFFFFFF;
        h.defined = true;
        return true;
    }

    int16_t* block(Comp& c, int bx, int by) { return c.coef.data() + 64 * ((size_t)by * c.bw + bx); }

    // ---- block decoders (T.81 F.2 / G.1.2) ----
    bool dec_baseline(Comp& c, int16_t* b) {
        const int t = decode(dc[c.td]);
        if (t < 0 || t > 16) return false;
        c.dc_pred += receive_extend(t);
        b[0] = (int16_t)c.dc_pred;
        for (int k = 1; k < 64;) {
            const int rs = decode(ac[c.ta]);
            if (rs < 0) return false;
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r != 15) break;
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return false;
            b[kZig[k++]] = (int16_t)receive_extend(s);
        }
        return true;
    }
    bool dec_dc_first(Comp& c, int16_t* b, int al) {
        const int t = decode(dc[c.td]);
        if (t < 0 || t > 16) return false;
        c.dc_pred += receive_extend(t);
        b[0] = (int16_t)(c.dc_pred * (1 << al));
        return true;
    }
    void dec_dc_refine(int16_t* b, int al) {
        if (getbit()) b[0] = (int16_t)(b[0] | (1 << al));
    }
    bool dec_ac_first(Comp& c, int16_t* b, int ss, int se, int al) {
        if (eobrun > 0) {
            --eobrun;
            return true;
        }
        for (int k = ss; k <= se;) {
            const int rs = decode(ac[c.ta]);
            if (rs < 0) return false;
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r < 15) {
                    eobrun = (1 << r) - 1;
                    if (r) eobrun += getbits(r);
                    break;
                }
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return false;
            b[kZig[k++]] = (int16_t)(receive_extend(s) * (1 << al));
        }
        return true;
    }
    void refine_nonzero(int16_t* z, int p1, int m1) {
        if (getbit() && (*z & p1) == 0) *z = (int16_t)(*z + (*z >= 0 ? p1 : m1));
    }
    bool dec_ac_refine(Comp& c, int16_t* b, int ss, int se, int al) {
        const int p1 = 1 << al, m1 = -1 * (1 << al);
        int k = ss;
        if (eobrun <= 0) {
            for (; k <= se; ++k) {
                const int rs = decode(ac[c.ta]);
                if (rs < 0) return false;
                int r = rs >> 4, s = rs & 15;
                if (s) {
                    s = getbit() ? p1 : m1;
                } else if (r != 15) {
                    eobrun = 1 << r;
                    if (r) eobrun += getbits(r);
                    break;
                }
                // advance over r zero-history coefficients, refining the others
                for (; k <= se; ++k) {
                    int16_t* z = b + kZig[k];
                    if (*z != 0) refine_nonzero(z, p1, m1);
                    else if (--r < 0) break;
                }
                if (s && k <= 63) b[kZig[k]] = (int16_t)s;
            }
        }
        if (eobrun > 0) {
            for (; k <= se; ++k) {
                int16_t* z = b + kZig[k];
                if (*z != 0) refine_nonzero(z, p1, m1);
            }
            --eobrun;
        }
        return true;
    }

    bool scan(const int* sc, int ns, int ss, int se, int ah, int al) {
        reset_entropy();
        if (!progressive) { ss = 0; se = 63; ah = 0; al = 0; }
        for (int i = 0; i < ns; ++i) {
            const Comp& c = comp[sc[i]];
            const bool need_dc = !progressive || ss == 0;
            const bool need_ac = !progressive || se > 0;
            if (need_dc && ah == 0 && !dc[c.td].defined) return false;
            if (need_ac && !ac[c.ta].defined) return false;
        }
        if (progressive && (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1))) return false;
        auto one = [&](Comp& c, int bx, int by) -> bool {
            int16_t* b = block(c, bx, by);
            if (!progressive) return dec_baseline(c, b);
            if (ss == 0) {
                if (ah == 0) return dec_dc_first(c, b, al);
                dec_dc_refine(b, al);
                return true;
            }
            return ah == 0 ? dec_ac_first(c, b, ss, se, al) : dec_ac_refine(c, b, ss, se, al);
        };
        int todo = restart;
        if (ns == 1) {   // non-interleaved: the component's own blocks in raster order
            Comp& c = comp[sc[0]];
            for (int by = 0; by < c.ch; ++by)
                for (int bx = 0; bx < c.cw; ++bx) {
                    if (restart && todo-- == 0) {
                        if (!restart_marker()) return false;
                        todo = restart - 1;
                    }
                    if (!one(c, bx, by)) return false;
                }
        } else {         // interleaved: MCUs of h x v blocks per component
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    if (restart && todo-- == 0) {
                        if (!restart_marker()) return false;
                        todo = restart - 1;
                    }
                    for (int i = 0; i < ns; ++i) {
                        Comp& c = comp[sc[i]];
                        for (int v = 0; v < c.v; ++v)
                            for (int h = 0; h < c.h; ++h)
                                if (!one(c, mx * c.h + h, my * c.v + v)) return false;
                    }
                }
        }
        // resynchronise on the next marker
        while (pos + 1 < n && !(p[pos] == 0xFF && p[pos + 1] != 0 && !(p[pos + 1] >= 0xD0 && p[pos + 1] <= 0xD7)))
            ++pos;
        return true;
    }
};

// ---- IDCT (LLM flow; 13-bit fixed-point constants) -------------------------
constexpr int kCB = 13, kP1 = 2;
constexpr int fx(double x) { return (int)(x * (1 << kCB) + 0.5); }

// 64-bit: a corrupt stream can carry coefficients whose products overflow
// 32 bits (UB; tests/test_sanitize.py); valid data gives the same values.
using ilong = long long;
inline void idct_1d(const ilong* in, int stride, ilong& o0, ilong& o1, ilong& o2, ilong& o3, ilong& o4, ilong& o5,
                    ilong& o6, ilong& o7) {
    // even part: inputs 0, 2, 4, 6
    ilong z2 = in[2 * stride], z3 = in[6 * stride];
    ilong z1 = (z2 + z3) * fx(0.541196100);
    const ilong t2 = z1 + z3 * -fx(1.847759065);
    const ilong t3 = z1 + z2 * fx(0.765366865);
    z2 = in[0];
    z3 = in[4 * stride];
    const ilong t0 = (z2 + z3) * (1 << kCB), t1 = (z2 - z3) * (1 << kCB);
    const ilong e10 = t0 + t3, e13 = t0 - t3, e11 = t1 + t2, e12 = t1 - t2;
    // odd part: inputs 7, 5, 3, 1
    ilong a0 = in[7 * stride], a1 = in[5 * stride], a2 = in[3 * stride], a3 = in[1 * stride];
    z1 = a0 + a3;
    z2 = a1 + a2;
    z3 = a0 + a2;
    ilong z4 = a1 + a3;
    const ilong z5 = (z3 + z4) * fx(1.175875602);
    a0 *= fx(0.298631336);
    a1 *= fx(2.053119869);
    a2 *= fx(3.072711026);
    a3 *= fx(1.501321110);
    z1 *= -fx(0.899976223);
    z2 *= -fx(2.562915447);
    z3 = z3 * -fx(1.961570560) + z5;
    z4 = z4 * -fx(0.390180644) + z5;
    a0 += z1 + z3;
    a1 += z2 + z4;
    a2 += z2 + z3;
    a3 += z1 + z4;
    o0 = e10 + a3; o7 = e10 - a3;
    o1 = e11 + a2; o6 = e11 - a2;
    o2 = e12 + a1; o5 = e12 - a1;
    o3 = e13 + a0; o4 = e13 - a0;
}

inline uint8_t clamp8(ilong v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

void idct_block(const int16_t* coef, const uint16_t* qz, uint8_t* out, int stride) {
    ilong d[64], ws[64];
    for (int k = 0; k < 64; ++k) d[kZig[k]] = (ilong)coef[kZig[k]] * (ilong)qz[k];
    for (int c = 0; c < 8; ++c) {                 // columns
        const ilong* in = d + c;
        if (!in[8] && !in[16] && !in[24] && !in[32] && !in[40] && !in[48] && !in[56]) {
            const ilong dcv = in[0] * (1 << kP1);
            for (int r = 0; r < 8; ++r) ws[8 * r + c] = dcv;
            continue;
        }
        ilong o[8];
        idct_1d(in, 8, o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]);
        const int sh = kCB - kP1;
        const ilong rnd = 1ll << (sh - 1);
        // (a corrupt block: keep the row pass's products inside 64 bits)
        for (int r = 0; r < 8; ++r) ws[8 * r + c] = std::max<ilong>(-(1ll << 40), std::min<ilong>(1ll << 40, (o[r] + rnd) >> sh));
    }
    for (int r = 0; r < 8; ++r) {                 // rows: descale, +128, clamp
        ilong o[8];
        idct_1d(ws + 8 * r, 1, o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]);
        const int sh = kCB + kP1 + 3;
        const ilong rnd = (1ll << (sh - 1)) + (128ll << sh);
        for (int k = 0; k < 8; ++k) out[(size_t)r * stride + k] = clamp8((o[k] + rnd) >> sh);
    }
}

// component plane -> full-resolution row y (w samples)
void upsample_row(const Comp& c, int hmax, int vmax, int y, int w, uint8_t* out) {
    const int pw = c.bw * 8;
    const int fh = hmax / c.h, fv = vmax / c.v;
    const int rows = c.bh * 8;
    const int cy = y / fv;
    const uint8_t* near = c.pix.data() + (size_t)std::min(cy, rows - 1) * pw;
    if (fh == 1 && fv == 1) {
        memcpy(out, near, w);
        return;
    }
    // chroma rows actually covered by the image: the last one is the edge
    const int cw_used = (w + fh - 1) / fh;
    if (fv == 2) {
        // triangle filter across rows: 3/4 nearer + 1/4 farther row
        const int far_y = std::max(0, std::min((y & 1) ? cy + 1 : cy - 1, (int)((c.ch * 8 - 1))));
        const uint8_t* far = c.pix.data() + (size_t)std::min(far_y, rows - 1) * pw;
        if (fh == 2) {
            std::vector<int> t(cw_used);
            for (int i = 0; i < cw_used; ++i) t[i] = 3 * near[i] + far[i];
            if (cw_used == 1) {
                const uint8_t v = (uint8_t)((t[0] + 2) >> 2);
                for (int x = 0; x < w; ++x) out[x] = v;
                return;
            }
            for (int i = 0; i < cw_used; ++i) {
                const int l = t[i > 0 ? i - 1 : 0], r = t[i + 1 < cw_used ? i + 1 : cw_used - 1];
                const int a = (i == 0) ? (t[0] * 4 + 8) >> 4 : (3 * t[i] + l + 8) >> 4;
                const int b = (i + 1 == cw_used) ? (t[i] * 4 + 8) >> 4 : (3 * t[i] + r + 8) >> 4;
                if (2 * i < w) out[2 * i] = (uint8_t)a;
                if (2 * i + 1 < w) out[2 * i + 1] = (uint8_t)b;
            }
            return;
        }
        if (fh == 1) {
            for (int x = 0; x < w; ++x) out[x] = (uint8_t)((3 * near[x] + far[x] + 2) >> 2);
            return;
        }
    } else if (fv == 1 && fh == 2) {
        if (cw_used == 1) {
            for (int x = 0; x < w; ++x) out[x] = near[0];
            return;
        }
        for (int i = 0; i < cw_used; ++i) {
            const int l = near[i > 0 ? i - 1 : 0], r = near[i + 1 < cw_used ? i + 1 : cw_used - 1];
            const int a = (i == 0) ? near[0] : (3 * near[i] + l + 2) >> 2;
            const int b = (i + 1 == cw_used) ? near[i] : (3 * near[i] + r + 2) >> 2;
            if (2 * i < w) out[2 * i] = (uint8_t)a;
            if (2 * i + 1 < w) out[2 * i + 1] = (uint8_t)b;
        }
        return;
    }
    for (int x = 0; x < w; ++x) out[x] = near[x / fh];   // other factors: replicate
}

// BT.601 full range, 20-bit fixed point
inline void ycc_to_rgb(int y, int cb, int cr, uint8_t* o) {
    auto f = [](double x) { return (int)(x * 4096.0 + 0.5) << 8; };
    const int yf = (y << 20) + (1 << 19);
    cb -= 128;
    cr -= 128;
    o[0] = clamp8((yf + cr * f(1.40200)) >> 20);
    o[1] = clamp8((yf - cr * f(0.71414) - cb * f(0.34414)) >> 20);
    o[2] = clamp8((yf + cb * f(1.77200)) >> 20);
}

}  // namespace

int jpeg_decode(const uint8_t* data, size_t len, Image8* out) {
    if (!data || !out || len < 4 || data[0] != 0xFF || data[1] != 0xD8) return ZRT_ERR_PARSE;
    Decoder D;
    D.p = data;
    D.n = len;
    D.pos = 2;
    bool done = false;
    while (!done) {
        // next marker: skip anything up to 0xFF, then fill bytes 0xFF
        int m = D.u8();
        while (m >= 0 && m != 0xFF) m = D.u8();
        while (m == 0xFF) m = D.u8();
        if (m < 0) break;   // truncated after the last scan: decode what is there
        if (m == 0xD9) break;                                  // EOI
        if (m >= 0xD0 && m <= 0xD7) continue;                  // stray RSTn
        const int L = D.u16();
        if (L < 2 || D.pos + (size_t)(L - 2) > D.n) return ZRT_ERR_PARSE;
        const size_t seg = D.pos, end = D.pos + L - 2;
        if (m == 0xDB) {                                       // DQT
            while (D.pos < end) {
                const int pq = D.u8();
                const int prec = pq >> 4, t = pq & 15;
                if (t > 3 || prec > 1) return ZRT_ERR_PARSE;
                for (int k = 0; k < 64; ++k) D.q[t][k] = (uint16_t)(prec ? D.u16() : D.u8());
                D.q_defined[t] = true;
            }
        } else if (m == 0xC4) {                                // DHT
            while (D.pos < end) {
                const int tc = D.u8();
                const int cls = tc >> 4, th = tc & 15;
                if (cls > 1 || th > 3) return ZRT_ERR_PARSE;
                uint8_t counts[16];
                int total = 0;
                for (int i = 0; i < 16; ++i) { counts[i] = (uint8_t)D.u8(); total += counts[i]; }
                if (total > 256 || D.pos + total > end) return ZRT_ERR_PARSE;
                if (!D.build_huff(cls ? D.ac[th] : D.dc[th], counts, D.p + D.pos, total)) return ZRT_ERR_PARSE;
                D.pos += total;
            }
        } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {      // SOF0/1/2 (Huffman)
            if (D.have_frame) return ZRT_ERR_PARSE;
            D.progressive = m == 0xC2;
            if (D.u8() != 8) return ZRT_ERR_UNSUPPORTED;      // 12-bit
            D.height = D.u16();
            D.width = D.u16();
            D.ncomp = D.u8();
            if (D.width <= 0 || D.height <= 0) return ZRT_ERR_UNSUPPORTED;   // DNL not supported
            if ((uint64_t)D.width * D.height > (1ull << 27)) return ZRT_ERR_UNSUPPORTED;   // > 128 MP
            if (D.ncomp != 1 && D.ncomp != 3) return ZRT_ERR_UNSUPPORTED;   // CMYK / YCCK
            for (int i = 0; i < D.ncomp; ++i) {
                Comp& c = D.comp[i];
                c.id = D.u8();
                const int hv = D.u8();
                c.h = hv >> 4;
                c.v = hv & 15;
                c.tq = D.u8();
                if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) return ZRT_ERR_PARSE;
                D.hmax = std::max(D.hmax, c.h);
                D.vmax = std::max(D.vmax, c.v);
            }
            D.mcux = (D.width + 8 * D.hmax - 1) / (8 * D.hmax);
            D.mcuy = (D.height + 8 * D.vmax - 1) / (8 * D.vmax);
            for (int i = 0; i < D.ncomp; ++i) {
                Comp& c = D.comp[i];
                if (D.hmax % c.h || D.vmax % c.v) return ZRT_ERR_UNSUPPORTED;   // fractional factors
                c.bw = D.mcux * c.h;
                c.bh = D.mcuy * c.v;
                c.cw = ((D.width * c.h + D.hmax - 1) / D.hmax + 7) / 8;
                c.ch = ((D.height * c.v + D.vmax - 1) / D.vmax + 7) / 8;
                c.coef.assign((size_t)c.bw * c.bh * 64, 0);
            }
            D.have_frame = true;
        } else if ((m >= 0xC3 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return ZRT_ERR_UNSUPPORTED;                        // lossless / arithmetic coding
        } else if (m == 0xDD) {                                // DRI
            D.restart = D.u16();
        } else if (m == 0xDA) {                                // SOS
            if (!D.have_frame) return ZRT_ERR_PARSE;
            const int ns = D.u8();
            if (ns < 1 || ns > D.ncomp) return ZRT_ERR_PARSE;
            int sc[3];
            for (int i = 0; i < ns; ++i) {
                const int cs = D.u8(), t = D.u8();
                int k = 0;
                while (k < D.ncomp && D.comp[k].id != cs) ++k;
                if (k == D.ncomp) return ZRT_ERR_PARSE;
                sc[i] = k;
                D.comp[k].td = t >> 4;
                D.comp[k].ta = t & 15;
                if (D.comp[k].td > 3 || D.comp[k].ta > 3) return ZRT_ERR_PARSE;
            }
            const int ss = D.u8(), se = D.u8(), a = D.u8();
            D.pos = end;
            if (!D.scan(sc, ns, ss, se, a >> 4, a & 15)) return ZRT_ERR_PARSE;
            continue;   // D.pos is at the next marker
        } else if (m == 0xEE) {                                // APP14 Adobe: colour transform
            if (L >= 14 && !memcmp(D.p + seg, "Adobe", 5)) {
                D.adobe_seen = true;
                D.adobe_rgb = D.p[seg + 11] == 0;
            }
        }
        D.pos = end;   // APPn, COM and the rest: skip
    }
    if (!D.have_frame) return ZRT_ERR_PARSE;
    for (int i = 0; i < D.ncomp; ++i) {
        Comp& c = D.comp[i];
        if (!D.q_defined[c.tq]) return ZRT_ERR_PARSE;
        c.pix.assign((size_t)c.bw * 8 * c.bh * 8, 0);
        for (int by = 0; by < c.bh; ++by)
            for (int bx = 0; bx < c.bw; ++bx)
                idct_block(D.block(c, bx, by), D.q[c.tq], c.pix.data() + (size_t)by * 8 * (c.bw * 8) + bx * 8,
                           c.bw * 8);
    }
    const int w = D.width, h = D.height;
    out->w = w;
    out->h = h;
    out->actual_c = D.ncomp;
    out->rgba.assign((size_t)w * h * 4, 255);
    std::vector<uint8_t> r0(w), r1(w), r2(w);
    for (int y = 0; y < h; ++y) {
        uint8_t* o = out->rgba.data() + (size_t)y * w * 4;
        upsample_row(D.comp[0], D.hmax, D.vmax, y, w, r0.data());
        if (D.ncomp == 1) {
            for (int x = 0; x < w; ++x) o[4 * x] = o[4 * x + 1] = o[4 * x + 2] = r0[x];
            continue;
        }
        upsample_row(D.comp[1], D.hmax, D.vmax, y, w, r1.data());
        upsample_row(D.comp[2], D.hmax, D.vmax, y, w, r2.data());
        // RGB when Adobe says so, or the classic component ids 'R','G','B'
        const bool rgb = (D.adobe_seen && D.adobe_rgb) ||
                         (!D.adobe_seen && D.comp[0].id == 'R' && D.comp[1].id == 'G' && D.comp[2].id == 'B');
        for (int x = 0; x < w; ++x) {
            if (rgb) {
                o[4 * x] = r0[x];
                o[4 * x + 1] = r1[x];
                o[4 * x + 2] = r2[x];
            } else {
                ycc_to_rgb(r0[x], r1[x], r2[x], o + 4 * x);
            }
        }
    }
    return ZRT_OK;
}

}  // namespace zrt
