// jpeg.cpp -- host-side JPEG and Radiance .hdr decoding for the scene / envmap loaders
// (mpt/image.py).  The reference decodes every texture with stb_image's stbi_load
// (Image8Bit::read_image, Image.cpp:33-61; its textured scene, the-white-room, ships JPEGs) and
// its envmaps and baked LUTs with stbi_loadf (Image32Bit::read_image_hdr, Image.cpp:342-370).
// This file restates the decoder the reference compiles (thirdparties/stbi/stb_image.h, x86-64
// build: the SSE2 kernels) so that a texture decodes to the same bytes:
//   * baseline + extended (SOF0/1) and progressive (SOF2) Huffman JPEG, 1 / 3 / 4 components,
//     any integer sampling ratio, restart intervals, DNL, junk after scans;
//   * dequantisation into 16-bit coefficients (products truncated to short, as stb stores them);
//   * the islow integer IDCT (jidctint constants scaled by 4096) with the SSE2 kernel's 16-bit
//     behaviour: the column pass saturates to int16, the row-pair sums wrap in int16;
//   * chroma upsampling: 1:1, the 2:1 triangle filters (h, v, hv) and nearest replication for the
//     other ratios, fed row by row with stb's near / far line state machine;
//   * YCbCr -> RGB in 20-bit fixed point with the Cb term of green truncated to 16 fractional bits
//     (identical to the SSE2 kernel), 'R','G','B' component ids or Adobe transform 0 without JFIF
//     = RGB, Adobe CMYK / YCCK through the rounded 8x8-bit product, and the requested channel
//     count (Y = (77 r + 150 g + 29 b) >> 8 for grey from RGB);
//   * .hdr: the RADIANCE / RGBE header, flat and new-style RLE scanlines (including stb's fallback
//     that reads a non-RLE first scanline as flat data), RGBE -> float with ldexp(1, e - 136).
// A vertical flip (stbi_set_flip_vertically_on_load) is the caller's (mpt/image.py).
#include <cstdint>
#include <cstdlib>
#include <climits>
#include <cstring>
#include <cmath>
#include <string>
#include <vector>

#include "mpt.h"

namespace mpt {
int api_fail(int code, const char* msg);   // mpt_api.cpp: sets mpt_last_error
}

namespace {

// zigzag position -> natural (row-major) index; 15 extra entries let a corrupt run end at 63
const uint8_t kDezigzag[64 + 15] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

constexpr int NO_MARKER = 0xff;

struct Huff {
    uint8_t size[257];
    uint16_t code[256];
    uint8_t values[256];
    uint32_t maxcode[18];
    int delta[17];
    bool defined = false;
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0, hd = 0, ha = 0, dc_pred = 0;
    int x = 0, y = 0, w2 = 0, h2 = 0, coeff_w = 0;
    std::vector<uint8_t> plane;    // w2 x h2 samples
    std::vector<int16_t> coeff;    // progressive: 64 per block
};

struct Jpeg {
    const uint8_t* p;
    const uint8_t* end;
    std::string err;
    int img_x = 0, img_y = 0, img_n = 0;
    Huff hdc[4], hac[4];
    uint16_t dequant[4][64];
    Comp comp[4];
    int h_max = 1, v_max = 1, mcu_x = 0, mcu_y = 0;
    bool progressive = false;
    int jfif = 0, app14 = -1, rgb_ids = 0;
    int scan_n = 0, order[4] = {0, 0, 0, 0};
    int spec_start = 0, spec_end = 0, succ_high = 0, succ_low = 0, eob_run = 0;
    int restart_interval = 0, todo = 0;
    uint32_t code_buffer = 0;
    int code_bits = 0;
    int marker = NO_MARKER;
    bool nomore = false;

    bool fail(const char* m) { if (err.empty()) err = m; return false; }
    bool at_eof() const { return p >= end; }
    int get8() { return p < end ? *p++ : 0; }
    int get16() { int a = get8(); return (a << 8) | get8(); }
    void skip(int n) { p = (n < 0 || end - p < n) ? end : p + n; }

    // ---- entropy-coded bits: 0xff00 stuffing, a marker ends the data (zeros are fed after it) ----
    void grow() {
        do {
            unsigned b = nomore ? 0 : (unsigned)get8();
            if (b == 0xff) {
                int c = get8();
                while (c == 0xff) c = get8();
                if (c != 0) { marker = c; nomore = true; return; }
            }
            code_buffer |= b << (24 - code_bits);
            code_bits += 8;
        } while (code_bits <= 24);
    }
    // canonical Huffman decode (JPEG F.2.2.3): the code length is the first k whose
    // left-aligned limit exceeds the next 16 bits
    int decode(const Huff& h) {
        if (code_bits < 16) grow();
        const uint32_t top = code_buffer >> 16;
        int k = 1;
        while (k <= 16 && top >= h.maxcode[k]) k++;
        if (k == 17) { code_bits -= 16; return -1; }
        if (k > code_bits) return -1;
        const int c = (int)((code_buffer >> (32 - k)) & ((1u << k) - 1)) + h.delta[k];
        if (c < 0 || c >= 256) return -1;
        code_bits -= k;
        code_buffer <<= k;
        return h.values[c];
    }
    // receive n bits and sign-extend (JPEG F.2.2.1 EXTEND)
    int receive_extend(int n) {
        if (code_bits < n) grow();
        if (code_bits < n) return 0;
        const bool neg = (code_buffer >> 31) == 0;
        const uint32_t k = n ? (code_buffer >> (32 - n)) : 0;
        code_buffer = n ? code_buffer << n : code_buffer;
        code_bits -= n;
        return neg ? (int)k - (1 << n) + 1 : (int)k;
    }
    int get_bits(int n) {
        if (code_bits < n) grow();
        if (code_bits < n) return 0;
        const uint32_t k = n ? (code_buffer >> (32 - n)) : 0;
        code_buffer = n ? code_buffer << n : code_buffer;
        code_bits -= n;
        return (int)k;
    }
    int get_bit() {
        if (code_bits < 1) grow();
        if (code_bits < 1) return 0;
        const uint32_t k = code_buffer & 0x80000000u;
        code_buffer <<= 1;
        code_bits--;
        return k != 0;
    }

    int get_marker() {
        if (marker != NO_MARKER) { int x = marker; marker = NO_MARKER; return x; }
        int x = get8();
        if (x != 0xff) return NO_MARKER;
        while (x == 0xff) x = get8();
        return x;
    }
    void reset() {
        code_bits = 0;
        code_buffer = 0;
        nomore = false;
        for (Comp& c : comp) c.dc_pred = 0;
        marker = NO_MARKER;
        todo = restart_interval ? restart_interval : 0x7fffffff;
        eob_run = 0;
    }
    // after an MCU: the restart interval's countdown; false = the scan stops here (not a restart)
    bool restart_countdown() {
        if (--todo <= 0) {
            if (code_bits < 24) grow();
            if (!(marker >= 0xd0 && marker <= 0xd7)) return false;
            reset();
        }
        return true;
    }

    bool build_huffman(Huff& h, const int* count) {
        int k = 0;
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < count[i]; j++) {
                h.size[k++] = (uint8_t)(i + 1);
                if (k >= 257) return fail("bad size list");
            }
        h.size[k] = 0;
        unsigned code = 0;
        k = 0;
        for (int j = 1; j <= 16; j++) {
            h.delta[j] = k - (int)code;
            if (h.size[k] == j) {
                while (h.size[k] == j) h.code[k++] = (uint16_t)(code++);
                if (code - 1 >= (1u << j)) return fail("bad code lengths");
            }
            h.maxcode[j] = code << (16 - j);
            code <<= 1;
        }
        h.maxcode[17] = 0xffffffffu;
        h.defined = true;
        return true;
    }

    // corrupt-stream guards of stb_image 2.28 (stbi__addints_valid / stbi__mul2shorts_valid,
    // stb_image.h:1068-1083): a DC prediction that would overflow int, or a dequantised DC
    // beyond int16 (of the int16-truncated operands, as stb computes it), ends the decode
    static bool addints_valid(int a, int b) {
        if ((a >= 0) != (b >= 0)) return true;
        if (a < 0 && b < 0) return a >= INT_MIN - b;
        return a <= INT_MAX - b;
    }
    static bool mul2shorts_valid(int16_t a, int16_t b) {
        if (b == 0 || b == -1) return true;
        if ((a >= 0) == (b >= 0)) return a <= SHRT_MAX / b;
        if (b < 0) return a <= SHRT_MIN / b;
        return a >= SHRT_MIN / b;
    }

    // ---- one 8x8 block ----
    bool decode_block(int16_t data[64], int b) {
        Comp& c = comp[b];
        const uint16_t* dq = dequant[c.tq];
        const int t = decode(hdc[c.hd]);
        if (t < 0 || t > 15) return fail("bad huffman code");
        std::memset(data, 0, 64 * sizeof(int16_t));
        const int diff = t ? receive_extend(t) : 0;
        if (!addints_valid(c.dc_pred, diff)) return fail("bad delta");
        const int dc = c.dc_pred + diff;
        c.dc_pred = dc;
        if (!mul2shorts_valid((int16_t)dc, (int16_t)dq[0])) return fail("can't merge dc and ac");
        data[0] = (int16_t)(dc * dq[0]);
        int k = 1;
        do {
            const int rs = decode(hac[c.ha]);
            if (rs < 0) return fail("bad huffman code");
            const int s = rs & 15, r = rs >> 4;
            if (s == 0) {
                if (rs != 0xf0) break;   // end of block
                k += 16;
            } else {
                k += r;
                const int zig = kDezigzag[k++];
                data[zig] = (int16_t)(receive_extend(s) * dq[zig]);
            }
        } while (k < 64);
        return true;
    }
    bool decode_block_prog_dc(int16_t data[64], int b) {
        if (spec_end != 0) return fail("can't merge dc and ac");
        if (succ_high == 0) {
            std::memset(data, 0, 64 * sizeof(int16_t));
            const int t = decode(hdc[comp[b].hd]);
            if (t < 0 || t > 15) return fail("bad huffman code");
            const int diff = t ? receive_extend(t) : 0;
            if (!addints_valid(comp[b].dc_pred, diff)) return fail("bad delta");
            const int dc = comp[b].dc_pred + diff;
            comp[b].dc_pred = dc;
            if (!mul2shorts_valid((int16_t)dc, (int16_t)(1 << succ_low))) return fail("can't merge dc and ac");
            data[0] = (int16_t)(dc * (1 << succ_low));
        } else if (get_bit()) {
            data[0] = (int16_t)(data[0] + (1 << succ_low));
        }
        return true;
    }
    // a nonzero coefficient's correction bit in a refinement scan
    void refine(int16_t* q, int16_t bit) {
        if (get_bit() && (*q & bit) == 0) *q = (int16_t)(*q > 0 ? *q + bit : *q - bit);
    }
    bool decode_block_prog_ac(int16_t data[64], int b) {
        if (spec_start == 0) return fail("can't merge dc and ac");
        const Huff& h = hac[comp[b].ha];
        if (succ_high == 0) {
            if (eob_run) { eob_run--; return true; }
            int k = spec_start;
            do {
                const int rs = decode(h);
                if (rs < 0) return fail("bad huffman code");
                const int s = rs & 15, r = rs >> 4;
                if (s == 0) {
                    if (r < 15) {
                        eob_run = (1 << r);
                        if (r) eob_run += get_bits(r);
                        eob_run--;
                        break;
                    }
                    k += 16;
                } else {
                    k += r;
                    const int zig = kDezigzag[k++];
                    data[zig] = (int16_t)(receive_extend(s) * (1 << succ_low));
                }
            } while (k <= spec_end);
        } else {
            const int16_t bit = (int16_t)(1 << succ_low);
            if (eob_run) {
                eob_run--;
                for (int k = spec_start; k <= spec_end; k++) {
                    int16_t* q = &data[kDezigzag[k]];
                    if (*q != 0) refine(q, bit);
                }
            } else {
                int k = spec_start;
                do {
                    const int rs = decode(h);
                    if (rs < 0) return fail("bad huffman code");
                    int s = rs & 15, r = rs >> 4;
                    if (s == 0) {
                        if (r < 15) {
                            eob_run = (1 << r) - 1;
                            if (r) eob_run += get_bits(r);
                            r = 64;   // the rest of the band is refinement only
                        }
                    } else {
                        if (s != 1) return fail("bad huffman code");
                        s = get_bit() ? bit : -bit;
                    }
                    while (k <= spec_end) {
                        int16_t* q = &data[kDezigzag[k++]];
                        if (*q != 0) {
                            refine(q, bit);
                        } else {
                            if (r == 0) { *q = (int16_t)s; break; }
                            r--;
                        }
                    }
                } while (k <= spec_end);
            }
        }
        return true;
    }

    bool parse_scan_data();
    bool process_marker(int m);
    bool frame_header(bool alloc = true);
    bool scan_header();
    bool decode_image();
};

// ---- IDCT: jidctint "islow" in 12-bit fixed point, as stb's SSE2 kernel evaluates it ----------
int f2f(double x) { return (int)(x * 4096 + 0.5); }
int16_t sat16(int v) { return (int16_t)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }
int16_t wrap16(int v) { return (int16_t)(uint16_t)(uint32_t)v; }

// One 1-D pass over 8 values (int16 in): returns the 8 int32 sums before the final shift,
// pairwise (out[i] = even_i + odd_i, out[7 - i] = even_i - odd_i) with `bias` added to the even part
void idct_1d(const int16_t* s, int stride, int bias, int shift, int* out) {
    const int r0 = s[0], r1 = s[stride], r2 = s[2 * stride], r3 = s[3 * stride];
    const int r4 = s[4 * stride], r5 = s[5 * stride], r6 = s[6 * stride], r7 = s[7 * stride];
    // even part: rotation of (r2, r6), (r0 +- r4) << 12 with 16-bit sums
    const int t2 = r2 * f2f(0.5411961) + r6 * (f2f(0.5411961) + f2f(-1.847759065));
    const int t3 = r2 * (f2f(0.5411961) + f2f(0.765366865)) + r6 * f2f(0.5411961);
    const int t0 = (int)wrap16(r0 + r4) * 4096, t1 = (int)wrap16(r0 - r4) * 4096;
    const int x0 = t0 + t3, x3 = t0 - t3, x1 = t1 + t2, x2 = t1 - t2;
    // odd part
    const int s17 = wrap16(r1 + r7), s35 = wrap16(r3 + r5);
    const int y0 = r7 * (f2f(-1.961570560) + f2f(0.298631336)) + r3 * f2f(-1.961570560);
    const int y2 = r7 * f2f(-1.961570560) + r3 * (f2f(-1.961570560) + f2f(3.072711026));
    const int y1 = r5 * (f2f(-0.390180644) + f2f(2.053119869)) + r1 * f2f(-0.390180644);
    const int y3 = r5 * f2f(-0.390180644) + r1 * (f2f(-0.390180644) + f2f(1.501321110));
    const int y4 = s17 * (f2f(1.175875602) + f2f(-0.899976223)) + s35 * f2f(1.175875602);
    const int y5 = s17 * f2f(1.175875602) + s35 * (f2f(1.175875602) + f2f(-2.562915447));
    const int x4 = y0 + y4, x5 = y1 + y5, x6 = y2 + y5, x7 = y3 + y4;
    const int e[4] = {x0 + bias, x1 + bias, x2 + bias, x3 + bias}, o[4] = {x7, x6, x5, x4};
    for (int i = 0; i < 4; i++) {
        out[i] = (e[i] + o[i]) >> shift;
        out[7 - i] = (e[i] - o[i]) >> shift;
    }
}

void idct_block(uint8_t* out, int stride, const int16_t data[64]) {
    int16_t col[64];
    int v[8];
    for (int i = 0; i < 8; i++) {   // columns: (x + 512) >> 10, saturated to int16
        idct_1d(data + i, 8, 512, 10, v);
        for (int k = 0; k < 8; k++) col[k * 8 + i] = sat16(v[k]);
    }
    for (int r = 0; r < 8; r++) {   // rows: (x + 65536 + (128 << 17)) >> 17, saturated to int16 then to 0..255
        idct_1d(col + r * 8, 1, 65536 + (128 << 17), 17, v);
        for (int k = 0; k < 8; k++) {
            const int16_t s = sat16(v[k]);
            out[r * stride + k] = (uint8_t)(s < 0 ? 0 : s > 255 ? 255 : s);
        }
    }
}

bool Jpeg::parse_scan_data() {
    reset();
    int16_t blk[64];
    if (scan_n == 1) {
        // non-interleaved: the component's own blocks in raster order
        const int n = order[0];
        Comp& c = comp[n];
        const int w = (c.x + 7) >> 3, h = (c.y + 7) >> 3;
        for (int j = 0; j < h; j++)
            for (int i = 0; i < w; i++) {
                if (!progressive) {
                    if (!decode_block(blk, n)) return false;
                    idct_block(c.plane.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, blk);
                } else {
                    int16_t* d = c.coeff.data() + 64 * ((size_t)i + (size_t)j * c.coeff_w);
                    if (spec_start == 0 ? !decode_block_prog_dc(d, n) : !decode_block_prog_ac(d, n)) return false;
                }
                if (!restart_countdown()) return true;
            }
        return true;
    }
    for (int j = 0; j < mcu_y; j++)
        for (int i = 0; i < mcu_x; i++) {
            for (int k = 0; k < scan_n; k++) {
                const int n = order[k];
                Comp& c = comp[n];
                for (int y = 0; y < c.v; y++)
                    for (int x = 0; x < c.h; x++) {
                        const int bx = i * c.h + x, by = j * c.v + y;
                        if (!progressive) {
                            if (!decode_block(blk, n)) return false;
                            idct_block(c.plane.data() + (size_t)c.w2 * by * 8 + bx * 8, c.w2, blk);
                        } else if (!decode_block_prog_dc(c.coeff.data() + 64 * ((size_t)bx + (size_t)by * c.coeff_w), n)) {
                            return false;
                        }
                    }
            }
            if (!restart_countdown()) return true;
        }
    return true;
}

bool Jpeg::process_marker(int m) {
    if (m == NO_MARKER) return fail("expected marker");
    if (m == 0xdd) {   // DRI
        if (get16() != 4) return fail("bad DRI len");
        restart_interval = get16();
        return true;
    }
    if (m == 0xdb) {   // DQT
        int L = get16() - 2;
        while (L > 0) {
            const int q = get8(), pq = q >> 4, t = q & 15;
            if (pq != 0 && pq != 1) return fail("bad DQT type");
            if (t > 3) return fail("bad DQT table");
            for (int i = 0; i < 64; i++) dequant[t][kDezigzag[i]] = (uint16_t)(pq ? get16() : get8());
            L -= pq ? 129 : 65;
        }
        return L == 0 || fail("bad DQT len");
    }
    if (m == 0xc4) {   // DHT
        int L = get16() - 2;
        while (L > 0) {
            int sizes[16], n = 0;
            const int q = get8(), tc = q >> 4, th = q & 15;
            if (tc > 1 || th > 3) return fail("bad DHT header");
            for (int i = 0; i < 16; i++) { sizes[i] = get8(); n += sizes[i]; }
            if (n > 256) return fail("bad DHT header");
            L -= 17;
            Huff& h = tc == 0 ? hdc[th] : hac[th];
            if (!build_huffman(h, sizes)) return false;
            for (int i = 0; i < n; i++) h.values[i] = (uint8_t)get8();
            L -= n;
        }
        return L == 0 || fail("bad DHT len");
    }
    if ((m >= 0xe0 && m <= 0xef) || m == 0xfe) {   // APPn / COM
        int L = get16();
        if (L < 2) return fail(m == 0xfe ? "bad COM len" : "bad APP len");
        L -= 2;
        if (m == 0xe0 && L >= 5) {   // JFIF
            static const uint8_t tag[5] = {'J', 'F', 'I', 'F', 0};
            bool ok = true;
            for (int i = 0; i < 5; i++) ok = (get8() == tag[i]) && ok;
            L -= 5;
            if (ok) jfif = 1;
        } else if (m == 0xee && L >= 12) {   // Adobe APP14: the colour transform
            static const uint8_t tag[6] = {'A', 'd', 'o', 'b', 'e', 0};
            bool ok = true;
            for (int i = 0; i < 6; i++) ok = (get8() == tag[i]) && ok;
            L -= 6;
            if (ok) {
                get8();
                get16();
                get16();
                app14 = get8();
                L -= 6;
            }
        }
        skip(L);
        return true;
    }
    return fail("unknown marker");
}

// alloc = false: the checks only (mpt_jpeg_decode's header query), no sample planes
bool Jpeg::frame_header(bool alloc) {
    const int Lf = get16();
    if (Lf < 11) return fail("bad SOF len");
    if (get8() != 8) return fail("only 8-bit JPEG");
    img_y = get16();
    if (img_y == 0) return fail("no header height");
    img_x = get16();
    if (img_x == 0) return fail("0 width");
    if (img_x > (1 << 24) || img_y > (1 << 24)) return fail("too large");
    const int c = get8();
    if (c != 1 && c != 3 && c != 4) return fail("bad component count");
    img_n = c;
    if (Lf != 8 + 3 * c) return fail("bad SOF len");
    rgb_ids = 0;
    static const int rgb[3] = {'R', 'G', 'B'};
    for (int i = 0; i < c; i++) {
        Comp& k = comp[i];
        k.id = get8();
        if (c == 3 && k.id == rgb[i]) rgb_ids++;
        const int q = get8();
        k.h = q >> 4;
        if (!k.h || k.h > 4) return fail("bad H");
        k.v = q & 15;
        if (!k.v || k.v > 4) return fail("bad V");
        k.tq = get8();
        if (k.tq > 3) return fail("bad TQ");
    }
    if ((int64_t)img_x * img_y * img_n > ((int64_t)1 << 31)) return fail("image too large");
    h_max = v_max = 1;
    for (int i = 0; i < c; i++) { h_max = comp[i].h > h_max ? comp[i].h : h_max; v_max = comp[i].v > v_max ? comp[i].v : v_max; }
    for (int i = 0; i < c; i++)
        if (h_max % comp[i].h || v_max % comp[i].v) return fail("non-integer sampling ratio");
    mcu_x = (img_x + h_max * 8 - 1) / (h_max * 8);
    mcu_y = (img_y + v_max * 8 - 1) / (v_max * 8);
    if (!alloc) return true;
    for (int i = 0; i < c; i++) {
        Comp& k = comp[i];
        k.x = (img_x * k.h + h_max - 1) / h_max;
        k.y = (img_y * k.v + v_max - 1) / v_max;
        k.w2 = mcu_x * k.h * 8;
        k.h2 = mcu_y * k.v * 8;
        k.plane.assign((size_t)k.w2 * k.h2, 0);
        if (progressive) {
            k.coeff_w = k.w2 / 8;
            k.coeff.assign((size_t)k.w2 * k.h2, 0);
        }
    }
    return true;
}

bool Jpeg::scan_header() {
    const int Ls = get16();
    scan_n = get8();
    if (scan_n < 1 || scan_n > 4 || scan_n > img_n) return fail("bad SOS component count");
    if (Ls != 6 + 2 * scan_n) return fail("bad SOS len");
    for (int i = 0; i < scan_n; i++) {
        const int id = get8(), q = get8();
        int which = 0;
        while (which < img_n && comp[which].id != id) which++;
        if (which == img_n) return fail("SOS names an unknown component");
        comp[which].hd = q >> 4;
        comp[which].ha = q & 15;
        if (comp[which].hd > 3 || comp[which].ha > 3) return fail("bad huffman table index");
        order[i] = which;
    }
    spec_start = get8();
    spec_end = get8();
    const int aa = get8();
    succ_high = aa >> 4;
    succ_low = aa & 15;
    if (progressive) {
        if (spec_start > 63 || spec_end > 63 || spec_start > spec_end || succ_high > 13 || succ_low > 13) return fail("bad SOS");
    } else {
        if (spec_start != 0 || succ_high != 0 || succ_low != 0) return fail("bad SOS");
        spec_end = 63;
    }
    return true;
}

bool Jpeg::decode_image() {
    jfif = 0;
    app14 = -1;
    marker = NO_MARKER;
    restart_interval = 0;
    if (get_marker() != 0xd8) return fail("no SOI");
    int m = get_marker();
    while (!(m == 0xc0 || m == 0xc1 || m == 0xc2)) {
        if (!process_marker(m)) return false;
        m = get_marker();
        while (m == NO_MARKER) {   // padding after a segment
            if (at_eof()) return fail("no SOF");
            m = get_marker();
        }
    }
    progressive = m == 0xc2;
    if (!frame_header()) return false;
    m = get_marker();
    while (m != 0xd9) {
        if (m == 0xda) {
            if (!scan_header() || !parse_scan_data()) return false;
            if (marker == NO_MARKER) {
                // junk after the entropy-coded data: resume at what looks like a marker
                int found = NO_MARKER;
                while (!at_eof() && found == NO_MARKER) {
                    int x = get8();
                    while (x == 0xff) {
                        if (at_eof()) break;
                        x = get8();
                        if (x != 0x00 && x != 0xff) { found = x; break; }
                    }
                }
                marker = found;
            }
            m = get_marker();
            if (m >= 0xd0 && m <= 0xd7) m = get_marker();
        } else if (m == 0xdc) {   // DNL
            const int Ld = get16(), NL = get16();
            if (Ld != 4) return fail("bad DNL len");
            if (NL != img_y) return fail("bad DNL height");
            m = get_marker();
        } else {
            if (!process_marker(m)) { err.clear(); break; }   // stb keeps what it decoded
            m = get_marker();
        }
        if (m == NO_MARKER && at_eof()) break;
    }
    if (progressive)   // dequantise (16-bit products) and transform every block
        for (int n = 0; n < img_n; n++) {
            Comp& c = comp[n];
            const int w = (c.x + 7) >> 3, h = (c.y + 7) >> 3;
            for (int j = 0; j < h; j++)
                for (int i = 0; i < w; i++) {
                    int16_t* d = c.coeff.data() + 64 * ((size_t)i + (size_t)j * c.coeff_w);
                    for (int k = 0; k < 64; k++) d[k] = (int16_t)(d[k] * dequant[c.tq][k]);
                    idct_block(c.plane.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, d);
                }
        }
    return true;
}

// ---- upsampling of one output row (the near row is the closer source row) ----
uint8_t div4(int x) { return (uint8_t)(x >> 2); }
uint8_t div16(int x) { return (uint8_t)(x >> 4); }

const uint8_t* resample_row(uint8_t* out, const uint8_t* nr, const uint8_t* fr, int w, int hs, int vs) {
    if (hs == 1 && vs == 1) return nr;
    if (hs == 1 && vs == 2) {
        for (int i = 0; i < w; i++) out[i] = div4(3 * nr[i] + fr[i] + 2);
        return out;
    }
    if (hs == 2 && vs == 1) {
        if (w == 1) { out[0] = out[1] = nr[0]; return out; }
        out[0] = nr[0];
        out[1] = div4(nr[0] * 3 + nr[1] + 2);
        int i = 1;
        for (; i < w - 1; i++) {
            const int n = 3 * nr[i] + 2;
            out[2 * i] = div4(n + nr[i - 1]);
            out[2 * i + 1] = div4(n + nr[i + 1]);
        }
        out[2 * i] = div4(nr[w - 2] * 3 + nr[w - 1] + 2);
        out[2 * i + 1] = nr[w - 1];
        return out;
    }
    if (hs == 2 && vs == 2) {
        if (w == 1) { out[0] = out[1] = div4(3 * nr[0] + fr[0] + 2); return out; }
        int t1 = 3 * nr[0] + fr[0];
        out[0] = div4(t1 + 2);
        for (int i = 1; i < w; i++) {
            const int t0 = t1;
            t1 = 3 * nr[i] + fr[i];
            out[2 * i - 1] = div16(3 * t0 + t1 + 8);
            out[2 * i] = div16(3 * t1 + t0 + 8);
        }
        out[2 * w - 1] = div4(t1 + 2);
        return out;
    }
    for (int i = 0; i < w; i++)   // other ratios: nearest
        for (int j = 0; j < hs; j++) out[i * hs + j] = nr[i];
    return out;
}

uint8_t compute_y(int r, int g, int b) { return (uint8_t)((r * 77 + g * 150 + 29 * b) >> 8); }
uint8_t blinn(uint8_t x, uint8_t y) { const unsigned t = (unsigned)x * y + 128; return (uint8_t)((t + (t >> 8)) >> 8); }

void ycbcr_to_rgb(uint8_t* out, const uint8_t* y, const uint8_t* pcb, const uint8_t* pcr, int count, int step) {
    auto fx = [](float v) { return ((int)(v * 4096.0f + 0.5f)) << 8; };
    for (int i = 0; i < count; i++) {
        const int yf = (y[i] << 20) + (1 << 19);
        const int cr = pcr[i] - 128, cb = pcb[i] - 128;
        int r = yf + cr * fx(1.40200f);
        int g = yf + cr * -fx(0.71414f) + (int)((unsigned)(cb * -fx(0.34414f)) & 0xffff0000u);
        int b = yf + cb * fx(1.77200f);
        r >>= 20; g >>= 20; b >>= 20;
        out[0] = (uint8_t)(r < 0 ? 0 : r > 255 ? 255 : r);
        out[1] = (uint8_t)(g < 0 ? 0 : g > 255 ? 255 : g);
        out[2] = (uint8_t)(b < 0 ? 0 : b > 255 ? 255 : b);
        if (step == 4) out[3] = 255;
        out += step;
    }
}

// load_jpeg_image: upsample + colour convert into n channels
void jpeg_output(Jpeg& z, int n, uint8_t* output) {
    const bool is_rgb = z.img_n == 3 && (z.rgb_ids == 3 || (z.app14 == 0 && !z.jfif));
    const int decode_n = (z.img_n == 3 && n < 3 && !is_rgb) ? 1 : z.img_n;
    struct Res { int hs, vs, ystep, ypos, w_lores; const uint8_t* line0; const uint8_t* line1; std::vector<uint8_t> buf; };
    Res rs[4];
    for (int k = 0; k < decode_n; k++) {
        Res& r = rs[k];
        r.hs = z.h_max / z.comp[k].h;
        r.vs = z.v_max / z.comp[k].v;
        r.ystep = r.vs >> 1;
        r.w_lores = (z.img_x + r.hs - 1) / r.hs;
        r.ypos = 0;
        r.line0 = r.line1 = z.comp[k].plane.data();
        r.buf.assign((size_t)z.img_x + 3, 0);
    }
    const uint8_t* co[4] = {nullptr, nullptr, nullptr, nullptr};
    for (int j = 0; j < z.img_y; j++) {
        uint8_t* out = output + (size_t)n * z.img_x * j;
        for (int k = 0; k < decode_n; k++) {
            Res& r = rs[k];
            const bool y_bot = r.ystep >= (r.vs >> 1);
            co[k] = resample_row(r.buf.data(), y_bot ? r.line1 : r.line0, y_bot ? r.line0 : r.line1, r.w_lores, r.hs, r.vs);
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.line0 = r.line1;
                if (++r.ypos < z.comp[k].y) r.line1 += z.comp[k].w2;
            }
        }
        const int W = z.img_x;
        if (n >= 3) {
            if (z.img_n == 3) {
                if (is_rgb) {
                    for (int i = 0; i < W; i++, out += n) {
                        out[0] = co[0][i]; out[1] = co[1][i]; out[2] = co[2][i];
                        if (n == 4) out[3] = 255;
                    }
                } else {
                    ycbcr_to_rgb(out, co[0], co[1], co[2], W, n);
                }
            } else if (z.img_n == 4) {
                if (z.app14 == 0) {   // CMYK
                    for (int i = 0; i < W; i++, out += n) {
                        const uint8_t m = co[3][i];
                        out[0] = blinn(co[0][i], m); out[1] = blinn(co[1][i], m); out[2] = blinn(co[2][i], m);
                        if (n == 4) out[3] = 255;
                    }
                } else if (z.app14 == 2) {   // YCCK
                    ycbcr_to_rgb(out, co[0], co[1], co[2], W, n);
                    for (int i = 0; i < W; i++, out += n) {
                        const uint8_t m = co[3][i];
                        out[0] = blinn((uint8_t)(255 - out[0]), m);
                        out[1] = blinn((uint8_t)(255 - out[1]), m);
                        out[2] = blinn((uint8_t)(255 - out[2]), m);
                    }
                } else {   // YCbCr + an ignored fourth channel
                    ycbcr_to_rgb(out, co[0], co[1], co[2], W, n);
                }
            } else {
                for (int i = 0; i < W; i++, out += n) {
                    out[0] = out[1] = out[2] = co[0][i];
                    if (n == 4) out[3] = 255;
                }
            }
        } else {
            if (is_rgb) {
                for (int i = 0; i < W; i++, out += n) {
                    out[0] = compute_y(co[0][i], co[1][i], co[2][i]);
                    if (n == 2) out[1] = 255;
                }
            } else if (z.img_n == 4 && z.app14 == 0) {
                for (int i = 0; i < W; i++, out += n) {
                    const uint8_t m = co[3][i];
                    out[0] = compute_y(blinn(co[0][i], m), blinn(co[1][i], m), blinn(co[2][i], m));
                    if (n == 2) out[1] = 255;
                }
            } else if (z.img_n == 4 && z.app14 == 2) {
                for (int i = 0; i < W; i++, out += n) {
                    out[0] = blinn((uint8_t)(255 - co[0][i]), co[3][i]);
                    if (n == 2) out[1] = 255;
                }
            } else {
                for (int i = 0; i < W; i++, out += n) {
                    out[0] = co[0][i];
                    if (n == 2) out[1] = 255;
                }
            }
        }
    }
}

// ---- Radiance .hdr --------------------------------------------------------------------------
struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool eof() const { return p >= end; }
    int get8() { return p < end ? *p++ : 0; }
    std::string token() {   // one header line (stbi__hdr_gettoken, 1023 characters at most)
        std::string s;
        char c = (char)get8();
        while (!eof() && c != '\n') {
            s.push_back(c);
            if (s.size() == 1023) { while (!eof() && get8() != '\n') {} break; }
            c = (char)get8();
        }
        return s;
    }
};

void hdr_convert(float* o, const uint8_t* in, int req) {
    if (in[3] != 0) {
        const float f1 = (float)std::ldexp(1.0f, in[3] - (128 + 8));
        if (req <= 2) {
            o[0] = (float)(in[0] + in[1] + in[2]) * f1 / 3;
        } else {
            o[0] = in[0] * f1; o[1] = in[1] * f1; o[2] = in[2] * f1;
        }
        if (req == 2) o[1] = 1;
        if (req == 4) o[3] = 1;
    } else {
        if (req == 4) o[3] = 1;
        if (req >= 3) o[0] = o[1] = o[2] = 0;
        if (req == 2) o[1] = 1;
        if (req <= 2) o[0] = 0;
    }
}

}  // namespace

extern "C" int mpt_jpeg_decode(const uint8_t* data, int64_t size, int32_t req_comp, uint8_t* out, int64_t out_cap,
                               int32_t* out_w, int32_t* out_h, int32_t* out_comp) {
    if (!data || size <= 0 || !out_w || !out_h) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "jpeg: NULL argument");
    if (req_comp < 0 || req_comp > 4) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "jpeg: req_comp must be 0..4");
    Jpeg z{};   // stb memsets its decoder (stb_image.h:4031): undefined tables decode from zeros
    z.p = data;
    z.end = data + size;
    if (!out) {   // header only: the size of the decoded image
        z.jfif = 0;
        z.app14 = -1;
        if (z.get_marker() != 0xd8) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "jpeg: no SOI");
        int m = z.get_marker();
        while (!(m == 0xc0 || m == 0xc1 || m == 0xc2)) {
            if (!z.process_marker(m)) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, ("jpeg: " + z.err).c_str());
            m = z.get_marker();
            while (m == NO_MARKER) {
                if (z.at_eof()) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "jpeg: no SOF");
                m = z.get_marker();
            }
        }
        z.progressive = m == 0xc2;
        // the frame header's checks (Lf, precision, zero / oversized dimensions, components,
        // sampling factors, the 2^31-byte limit) without allocating planes
        if (!z.frame_header(false)) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, ("jpeg: " + z.err).c_str());
        *out_h = z.img_y;
        *out_w = z.img_x;
        if (out_comp) *out_comp = z.img_n;
        return MPT_OK;
    }
    if (!z.decode_image()) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, ("jpeg: " + z.err).c_str());
    const int n = req_comp ? req_comp : (z.img_n >= 3 ? 3 : 1);
    if (out_cap < (int64_t)n * z.img_x * z.img_y) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "jpeg: output buffer too small");
    jpeg_output(z, n, out);
    *out_w = z.img_x;
    *out_h = z.img_y;
    if (out_comp) *out_comp = z.img_n;
    return MPT_OK;
}

extern "C" int mpt_hdr_decode(const uint8_t* data, int64_t size, int32_t req_comp, float* out, int64_t out_cap,
                              int32_t* out_w, int32_t* out_h) {
    if (!data || size <= 0 || !out_w || !out_h) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: NULL argument");
    if (req_comp < 0 || req_comp > 4) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: req_comp must be 0..4");
    Reader s{data, data + size};
    const std::string head = s.token();
    if (head != "#?RADIANCE" && head != "#?RGBE") return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: not a Radiance HDR file");
    bool valid = false;
    for (;;) {
        const std::string t = s.token();
        if (t.empty()) break;
        if (t == "FORMAT=32-bit_rle_rgbe") valid = true;
    }
    if (!valid) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: unsupported format");
    const std::string dims = s.token();
    if (dims.compare(0, 3, "-Y ") != 0) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: unsupported data layout");
    char* q = nullptr;
    const int height = (int)std::strtol(dims.c_str() + 3, &q, 10);
    while (*q == ' ') q++;
    if (std::strncmp(q, "+X ", 3) != 0) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: unsupported data layout");
    const int width = (int)std::strtol(q + 3, nullptr, 10);
    if (width <= 0 || height <= 0 || width > (1 << 24) || height > (1 << 24))
        return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: bad dimensions");
    *out_w = width;
    *out_h = height;
    const int req = req_comp ? req_comp : 3;
    if (!out) return MPT_OK;
    if (out_cap < (int64_t)width * height * req) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: output buffer too small");
    auto flat = [&](int j0, int i0) {
        for (int j = j0; j < height; j++)
            for (int i = (j == j0 ? i0 : 0); i < width; i++) {
                uint8_t rgbe[4];
                for (int k = 0; k < 4; k++) rgbe[k] = (uint8_t)s.get8();
                hdr_convert(out + ((size_t)j * width + i) * req, rgbe, req);
            }
    };
    if (width < 8 || width >= 32768) {
        flat(0, 0);
        return MPT_OK;
    }
    std::vector<uint8_t> line((size_t)width * 4);
    for (int j = 0; j < height; j++) {
        const int c1 = s.get8(), c2 = s.get8();
        int len = s.get8();
        if (c1 != 2 || c2 != 2 || (len & 0x80)) {
            // not run-length encoded: these bytes are a pixel and the whole image is read flat
            // from the start (stb_image's behaviour, whatever row this happens on)
            uint8_t rgbe[4] = {(uint8_t)c1, (uint8_t)c2, (uint8_t)len, (uint8_t)s.get8()};
            hdr_convert(out, rgbe, req);
            flat(0, 1);
            return MPT_OK;
        }
        len = (len << 8) | s.get8();
        if (len != width) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: invalid decoded scanline length");
        for (int k = 0; k < 4; k++) {
            int i = 0, left;
            while ((left = width - i) > 0) {
                int count = s.get8();
                if (count > 128) {
                    const int value = s.get8();
                    count -= 128;
                    if (count == 0 || count > left) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: bad RLE data");
                    for (int z = 0; z < count; z++) line[(size_t)(i++) * 4 + k] = (uint8_t)value;
                } else {
                    if (count == 0 || count > left) return mpt::api_fail(MPT_ERR_INVALID_ARGUMENT, "hdr: bad RLE data");
                    for (int z = 0; z < count; z++) line[(size_t)(i++) * 4 + k] = (uint8_t)s.get8();
                }
            }
        }
        for (int i = 0; i < width; i++) hdr_convert(out + ((size_t)j * width + i) * req, line.data() + (size_t)i * 4, req);
    }
    return MPT_OK;
}
