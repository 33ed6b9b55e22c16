// image.cpp -- native env-map decoding for EnvLight(file) (src/texture.cu:64-171,
// include/picture.h:19-45).  The reference decodes through FreeImage (bundled
// libjpeg); this restates what that path produces for the formats an env map
// ships in:
//   * JPEG, baseline and progressive Huffman (SOF0/1/2), 3-component YCbCr
//     (JFIF), any sampling factors.  The arithmetic follows libjpeg's defaults
//     bit for bit: the "islow" integer IDCT, "fancy" triangle upsampling for
//     2x1 and 2x2 chroma planes wider than 2 samples (otherwise replication),
//     and the fixed-point
//     YCbCr->RGB tables.  Grayscale and CMYK JPEGs are rejected, as the
//     reference's Texture rejects anything but 3 or 4 channels.
//   * binary PPM (P6, maxval 255).
// Output: RGBA8, row 0 = bottom (FreeImage's order), alpha 255 -- exactly the
// texel array Texture uploads after its BGR->RGB swizzle (texture.cu:33-47).
#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <iterator>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "tpt_internal.hpp"

namespace tpt {
namespace {

struct DecodeError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Canonical Huffman table with a 9-bit lookahead.
struct Huffman {
    bool present = false;
    uint8_t symbols[256] = {};
    int32_t maxcode[18] = {};   // largest code of each length, -1 if none
    int32_t valoff[17] = {};    // symbol index offset per length
    uint16_t look[512] = {};    // (length << 8) | symbol, 0 = not resolvable in 9 bits

    void build(const uint8_t counts[16], const uint8_t* syms, int n) {
        std::memcpy(symbols, syms, (size_t)n);
        int code = 0, k = 0;
        std::memset(look, 0, sizeof look);
        for (int len = 1; len <= 16; ++len) {
            valoff[len] = k - code;
            if (counts[len - 1]) {
                for (int i = 0; i < counts[len - 1]; ++i, ++k, ++code) {
                    // a code must fit in len bits (libjpeg: JERR_BAD_HUFF_TABLE); checked
                    // before it indexes the lookahead table
                    if (code >= (1 << len)) throw DecodeError("bad Huffman table");
                    if (len <= 9) {
                        const int shift = 9 - len;
                        for (int f = 0; f < (1 << shift); ++f)
                            look[(code << shift) | f] = (uint16_t)((len << 8) | symbols[k]);
                    }
                }
                maxcode[len] = code - 1;
            } else {
                maxcode[len] = -1;
            }
            if (code > (1 << len)) throw DecodeError("bad Huffman table");
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        present = true;
    }
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;                 // Huffman table ids of the current scan
    int bw = 0, bh = 0;                 // blocks across / down, padded to whole MCUs
    int cw = 0, ch = 0;                 // downsampled size (ceil(W*h/hmax), ceil(H*v/vmax))
    int pred = 0;                       // DC predictor
    std::vector<int16_t> coef;          // bw*bh*64, natural order (quantized)
};

class Jpeg {
public:
    Jpeg(const uint8_t* p, size_t n) : d_(p), n_(n) {}

    void decode(std::vector<uint8_t>& rgba, int& w, int& h) {
        if (n_ < 4 || d_[0] != 0xFF || d_[1] != 0xD8) throw DecodeError("not a JPEG file");
        pos_ = 2;
        bool frame = false, eoi = false;
        while (!eoi) {
            const int m = next_marker();
            switch (m) {
                case 0xC0: case 0xC1: case 0xC2:
                    read_sof(m == 0xC2);
                    frame = true;
                    break;
                case 0xC4: read_dht(); break;
                case 0xDB: read_dqt(); break;
                case 0xDD: read_dri(); break;
                case 0xDA:
                    if (!frame) throw DecodeError("scan before frame header");
                    read_sos_and_scan();
                    break;
                case 0xD9: eoi = true; break;
                case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
                case 0xCD: case 0xCE: case 0xCF:
                    throw DecodeError("unsupported JPEG process (lossless / hierarchical / arithmetic)");
                default:
                    if (m == 0xEE) read_app14();
                    else skip_segment();
                    break;
            }
        }
        if (!frame) throw DecodeError("no frame in JPEG");
        finish(rgba, w, h);
    }

private:
    const uint8_t* d_;
    size_t n_, pos_ = 0;
    int width_ = 0, height_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
    bool progressive_ = false;
    int restart_ = 0;
    int adobe_transform_ = -1;
    uint16_t qt_[4][64] = {};
    bool qt_present_[4] = {};
    Huffman dc_[4], ac_[4];
    std::vector<Component> comp_;
    // entropy decoder state
    uint32_t bits_ = 0;
    int nbits_ = 0;
    bool hit_marker_ = false;
    int eobrun_ = 0;

    uint8_t byte() {
        if (pos_ >= n_) throw DecodeError("truncated JPEG");
        return d_[pos_++];
    }
    int u16() {
        const int hi = byte();
        return (hi << 8) | byte();
    }
    int next_marker() {
        uint8_t b = byte();
        while (b != 0xFF) b = byte();   // tolerate garbage between segments
        while (b == 0xFF) b = byte();
        return b;
    }
    void skip_segment() {
        const int len = u16();
        if (len < 2 || pos_ + (size_t)(len - 2) > n_) throw DecodeError("bad segment length");
        pos_ += (size_t)(len - 2);
    }
    void read_app14() {   // Adobe: transform flag (0 = no YCbCr conversion)
        const size_t start = pos_;
        const int len = u16();
        if (len >= 14 && pos_ + 12 <= n_ && std::memcmp(d_ + pos_, "Adobe", 5) == 0) adobe_transform_ = d_[pos_ + 11];
        pos_ = start + (size_t)len;
    }
    void read_dri() {
        const int len = u16();
        if (len != 4) throw DecodeError("bad DRI");
        restart_ = u16();
    }
    void read_dqt() {
        int len = u16() - 2;
        while (len > 0) {
            const int pq_tq = byte();
            const int pq = pq_tq >> 4, tq = pq_tq & 15;
            if (tq > 3 || pq > 1) throw DecodeError("bad DQT");
            for (int i = 0; i < 64; ++i) qt_[tq][kZigzag[i]] = (uint16_t)(pq ? u16() : byte());
            qt_present_[tq] = true;
            len -= 1 + 64 * (pq ? 2 : 1);
        }
        if (len != 0) throw DecodeError("bad DQT length");
    }
    void read_dht() {
        int len = u16() - 2;
        while (len > 0) {
            const int tc_th = byte();
            const int tc = tc_th >> 4, th = tc_th & 15;
            if (tc > 1 || th > 3) throw DecodeError("bad DHT");
            uint8_t counts[16];
            int total = 0;
            for (int i = 0; i < 16; ++i) total += counts[i] = byte();
            if (total > 256) throw DecodeError("bad DHT counts");
            uint8_t syms[256];
            for (int i = 0; i < total; ++i) syms[i] = byte();
            (tc ? ac_[th] : dc_[th]).build(counts, syms, total);
            len -= 17 + total;
        }
        if (len != 0) throw DecodeError("bad DHT length");
    }
    void read_sof(bool progressive) {
        if (!comp_.empty()) throw DecodeError("multiple frames");
        progressive_ = progressive;
        u16();
        if (byte() != 8) throw DecodeError("only 8-bit JPEG samples are supported");
        height_ = u16();
        width_ = u16();
        const int nc = byte();
        if (width_ <= 0 || height_ <= 0) throw DecodeError("JPEG without a height (DNL) is not supported");
        if ((int64_t)width_ * height_ > (int64_t)1 << 28) throw DecodeError("JPEG too large");
        if (nc == 1 || nc == 4)   // Texture accepts 3 or 4 channels only (texture.cu:64-85)
            throw DecodeError("only 3-component (YCbCr/RGB) JPEGs are supported (grayscale/CMYK env maps are "
                              "rejected, as the reference's Texture rejects non-RGB pictures)");
        if (nc != 3) throw DecodeError("unsupported JPEG component count");
        comp_.resize((size_t)nc);
        for (auto& c : comp_) {
            c.id = byte();
            const int hv = byte();
            c.h = hv >> 4;
            c.v = hv & 15;
            c.tq = byte();
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) throw DecodeError("bad component");
            hmax_ = std::max(hmax_, c.h);
            vmax_ = std::max(vmax_, c.v);
        }
        mcux_ = (width_ + 8 * hmax_ - 1) / (8 * hmax_);
        mcuy_ = (height_ + 8 * vmax_ - 1) / (8 * vmax_);
        for (auto& c : comp_) {
            c.bw = mcux_ * c.h;
            c.bh = mcuy_ * c.v;
            c.cw = (width_ * c.h + hmax_ - 1) / hmax_;
            c.ch = (height_ * c.v + vmax_ - 1) / vmax_;
            c.coef.assign((size_t)c.bw * (size_t)c.bh * 64, 0);
        }
    }

    // ---- bit reader (0xFF00 stuffing; a marker stops the data: zeros follow) ----
    void fill() {
        while (nbits_ <= 24) {
            uint32_t b = 0;
            if (!hit_marker_ && pos_ < n_) {
                b = d_[pos_];
                if (b == 0xFF) {
                    const uint8_t nx = pos_ + 1 < n_ ? d_[pos_ + 1] : 0xD9;
                    if (nx == 0x00) {
                        pos_ += 2;
                    } else {
                        hit_marker_ = true;
                        b = 0;
                    }
                } else {
                    ++pos_;
                }
            }
            bits_ |= b << (24 - nbits_);
            nbits_ += 8;
        }
    }
    int get_bits(int n) {
        if (n == 0) return 0;
        fill();
        const int v = (int)(bits_ >> (32 - n));
        bits_ <<= n;
        nbits_ -= n;
        return v;
    }
    int get_bit() { return get_bits(1); }
    int decode(const Huffman& t) {
        if (!t.present) throw DecodeError("missing Huffman table");
        fill();
        const uint16_t e = t.look[bits_ >> 23];
        if (e) {
            const int len = e >> 8;
            bits_ <<= len;
            nbits_ -= len;
            return e & 0xff;
        }
        int code = (int)(bits_ >> 23), len = 9;
        bits_ <<= 9;
        nbits_ -= 9;
        while (code > t.maxcode[len]) {
            code = (code << 1) | get_bit();
            if (++len > 16) throw DecodeError("bad Huffman code");
        }
        return t.symbols[t.valoff[len] + code];
    }
    static int extend(int v, int s) { return s == 0 ? 0 : (v < (1 << (s - 1)) ? v - (1 << s) + 1 : v); }
    int receive_extend(int s) { return extend(get_bits(s), s); }

    void restart_marker() {
        // discard the remaining bits, expect RSTn
        bits_ = 0;
        nbits_ = 0;
        if (hit_marker_) {
            hit_marker_ = false;
            if (pos_ + 1 < n_ && d_[pos_] == 0xFF && d_[pos_ + 1] >= 0xD0 && d_[pos_ + 1] <= 0xD7) pos_ += 2;
        } else {
            // data ended without the marker in the bit stream yet: search for it
            while (pos_ + 1 < n_ && !(d_[pos_] == 0xFF && d_[pos_ + 1] >= 0xD0 && d_[pos_ + 1] <= 0xD7)) ++pos_;
            if (pos_ + 1 < n_) pos_ += 2;
        }
        for (auto& c : comp_) c.pred = 0;
        eobrun_ = 0;
    }

    // ---- scans ----
    void read_sos_and_scan() {
        u16();
        const int ns = byte();
        if (ns < 1 || ns > 4) throw DecodeError("bad SOS");
        std::vector<Component*> sc;
        for (int i = 0; i < ns; ++i) {
            const int cid = byte(), t = byte();
            Component* c = nullptr;
            for (auto& cc : comp_)
                if (cc.id == cid) c = &cc;
            if (!c) throw DecodeError("scan names an unknown component");
            c->td = t >> 4;
            c->ta = t & 15;
            if (c->td > 3 || c->ta > 3) throw DecodeError("bad table selector");
            sc.push_back(c);
        }
        const int ss = byte(), se = byte(), a = byte();
        const int ah = a >> 4, al = a & 15;
        if (!progressive_) {
            if (ss != 0 || se != 63 || ah != 0 || al != 0) throw DecodeError("bad baseline scan parameters");
        } else {
            if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || al > 13)
                throw DecodeError("bad progressive scan parameters");
        }
        bits_ = 0;
        nbits_ = 0;
        hit_marker_ = false;
        eobrun_ = 0;
        for (auto* c : sc) c->pred = 0;

        auto block = [&](Component* c, int bx, int by) {
            int16_t* b = &c->coef[((size_t)by * (size_t)c->bw + (size_t)bx) * 64];
            if (!progressive_) decode_baseline(c, b);
            else if (ss == 0) decode_dc_prog(c, b, ah, al);
            else if (ah == 0) decode_ac_first(c, b, ss, se, al);
            else decode_ac_refine(c, b, ss, se, al);
        };
        int mcus = 0;
        if (ns == 1) {   // non-interleaved: the component's own block grid
            Component* c = sc[0];
            const int bw = (c->cw + 7) / 8, bh = (c->ch + 7) / 8;
            for (int by = 0; by < bh; ++by)
                for (int bx = 0; bx < bw; ++bx) {
                    if (restart_ && mcus > 0 && mcus % restart_ == 0) restart_marker();
                    block(c, bx, by);
                    ++mcus;
                }
        } else {
            for (int my = 0; my < mcuy_; ++my)
                for (int mx = 0; mx < mcux_; ++mx) {
                    if (restart_ && mcus > 0 && mcus % restart_ == 0) restart_marker();
                    for (auto* c : sc)
                        for (int v = 0; v < c->v; ++v)
                            for (int u = 0; u < c->h; ++u) block(c, mx * c->h + u, my * c->v + v);
                    ++mcus;
                }
        }
        // position the reader after the entropy-coded data (at the next marker)
        while (pos_ + 1 < n_ && !(d_[pos_] == 0xFF && d_[pos_ + 1] != 0x00 && !(d_[pos_ + 1] >= 0xD0 && d_[pos_ + 1] <= 0xD7)))
            ++pos_;
    }

    void decode_baseline(Component* c, int16_t* b) {
        const int t = decode(dc_[c->td]);
        if (t > 11) throw DecodeError("bad DC magnitude");
        c->pred += receive_extend(t);
        b[0] = (int16_t)c->pred;
        const Huffman& ac = ac_[c->ta];
        for (int k = 1; k < 64;) {
            const int rs = decode(ac);
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r != 15) break;   // EOB
                k += 16;              // ZRL
                continue;
            }
            k += r;
            if (k > 63) throw DecodeError("AC index out of range");
            b[kZigzag[k]] = (int16_t)receive_extend(s);
            ++k;
        }
    }
    void decode_dc_prog(Component* c, int16_t* b, int ah, int al) {
        if (ah == 0) {
            const int t = decode(dc_[c->td]);
            if (t > 11) throw DecodeError("bad DC magnitude");
            c->pred += receive_extend(t);
            b[0] = (int16_t)(c->pred * (1 << al));
        } else if (get_bit()) {
            b[0] = (int16_t)(b[0] | (1 << al));
        }
    }
    void decode_ac_first(Component* c, int16_t* b, int ss, int se, int al) {
        if (eobrun_ > 0) {
            --eobrun_;
            return;
        }
        const Huffman& ac = ac_[c->ta];
        for (int k = ss; k <= se;) {
            const int rs = decode(ac);
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r < 15) {
                    eobrun_ = (1 << r) - 1;
                    if (r) eobrun_ += get_bits(r);
                    break;
                }
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) throw DecodeError("AC index out of range");
            b[kZigzag[k]] = (int16_t)(receive_extend(s) * (1 << al));
            ++k;
        }
    }
    void decode_ac_refine(Component* c, int16_t* b, int ss, int se, int al) {
        const int p1 = 1 << al, m1 = -1 * (1 << al);
        int k = ss;
        auto refine = [&](int16_t& coef) {   // correction bit of an already-nonzero coefficient
            if (get_bit() && (coef & p1) == 0) coef = (int16_t)(coef >= 0 ? coef + p1 : coef + m1);
        };
        if (eobrun_ == 0) {
            const Huffman& ac = ac_[c->ta];
            for (; k <= se; ++k) {
                const int rs = decode(ac);
                int r = rs >> 4;
                const int s = rs & 15;
                int val = 0;
                if (s) {
                    if (s != 1) throw DecodeError("bad refinement magnitude");
                    val = get_bit() ? p1 : m1;
                } else if (r != 15) {
                    eobrun_ = 1 << r;
                    if (r) eobrun_ += get_bits(r);
                    break;   // the rest of the band is handled as an EOB run
                }
                // skip r zero coefficients (refining the nonzero ones passed over), then place val
                for (; k <= se; ++k) {
                    int16_t& coef = b[kZigzag[k]];
                    if (coef != 0) {
                        refine(coef);
                    } else {
                        if (r == 0) {
                            if (val) coef = (int16_t)val;
                            break;
                        }
                        --r;
                    }
                }
            }
        }
        if (eobrun_ > 0) {
            for (; k <= se; ++k) {
                int16_t& coef = b[kZigzag[k]];
                if (coef != 0) refine(coef);
            }
            --eobrun_;
        }
    }

    // ---- reconstruction: islow IDCT, fancy upsampling, YCbCr -> RGB ----
    static uint8_t idct_limit(int32_t x) {   // libjpeg's IDCT range-limit table (RANGE_MASK 1023)
        const int v = x & 1023;
        if (v < 128) return (uint8_t)(v + 128);
        if (v < 512) return 255;
        if (v < 896) return 0;
        return (uint8_t)(v - 896);
    }
    static void idct_islow(const int16_t* in, const uint16_t* q, uint8_t* out, int stride) {
        constexpr int CB = 13, P1 = 2;
        constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                          F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
        auto descale = [](int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); };
        int32_t ws[64];
        for (int c = 0; c < 8; ++c) {
            const int16_t* ip = in + c;
            if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
                const int32_t dc = ((int32_t)ip[0] * q[c]) * (1 << P1);
                for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
                continue;
            }
            int64_t z2 = (int32_t)ip[16] * q[16 + c], z3 = (int32_t)ip[48] * q[48 + c];
            int64_t z1 = (z2 + z3) * F0541;
            const int64_t t2 = z1 + z3 * -F1847, t3 = z1 + z2 * F0765;
            z2 = (int32_t)ip[0] * q[c];
            z3 = (int32_t)ip[32] * q[32 + c];
            const int64_t t0 = (z2 + z3) * (1 << CB), t1 = (z2 - z3) * (1 << CB);
            const int64_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
            int64_t o0 = (int32_t)ip[56] * q[56 + c], o1 = (int32_t)ip[40] * q[40 + c],
                    o2 = (int32_t)ip[24] * q[24 + c], o3 = (int32_t)ip[8] * q[8 + c];
            int64_t y1 = o0 + o3, y2 = o1 + o2, y3 = o0 + o2, y4 = o1 + o3;
            const int64_t y5 = (y3 + y4) * F1175;
            o0 *= F0298;
            o1 *= F2053;
            o2 *= F3072;
            o3 *= F1501;
            y1 *= -F0899;
            y2 *= -F2562;
            y3 *= -F1961;
            y4 *= -F0390;
            y3 += y5;
            y4 += y5;
            o0 += y1 + y3;
            o1 += y2 + y4;
            o2 += y2 + y3;
            o3 += y1 + y4;
            ws[0 * 8 + c] = descale(t10 + o3, CB - P1);
            ws[7 * 8 + c] = descale(t10 - o3, CB - P1);
            ws[1 * 8 + c] = descale(t11 + o2, CB - P1);
            ws[6 * 8 + c] = descale(t11 - o2, CB - P1);
            ws[2 * 8 + c] = descale(t12 + o1, CB - P1);
            ws[5 * 8 + c] = descale(t12 - o1, CB - P1);
            ws[3 * 8 + c] = descale(t13 + o0, CB - P1);
            ws[4 * 8 + c] = descale(t13 - o0, CB - P1);
        }
        for (int r = 0; r < 8; ++r) {
            const int32_t* w = ws + r * 8;
            uint8_t* op = out + (size_t)r * stride;
            int64_t z2 = w[2], z3 = w[6];
            int64_t z1 = (z2 + z3) * F0541;
            const int64_t t2 = z1 + z3 * -F1847, t3 = z1 + z2 * F0765;
            const int64_t t0 = ((int64_t)w[0] + w[4]) * (1 << CB), t1 = ((int64_t)w[0] - w[4]) * (1 << CB);
            const int64_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
            int64_t o0 = w[7], o1 = w[5], o2 = w[3], o3 = w[1];
            int64_t y1 = o0 + o3, y2 = o1 + o2, y3 = o0 + o2, y4 = o1 + o3;
            const int64_t y5 = (y3 + y4) * F1175;
            o0 *= F0298;
            o1 *= F2053;
            o2 *= F3072;
            o3 *= F1501;
            y1 *= -F0899;
            y2 *= -F2562;
            y3 *= -F1961;
            y4 *= -F0390;
            y3 += y5;
            y4 += y5;
            o0 += y1 + y3;
            o1 += y2 + y4;
            o2 += y2 + y3;
            o3 += y1 + y4;
            constexpr int S = CB + P1 + 3;
            op[0] = idct_limit(descale(t10 + o3, S));
            op[7] = idct_limit(descale(t10 - o3, S));
            op[1] = idct_limit(descale(t11 + o2, S));
            op[6] = idct_limit(descale(t11 - o2, S));
            op[2] = idct_limit(descale(t12 + o1, S));
            op[5] = idct_limit(descale(t12 - o1, S));
            op[3] = idct_limit(descale(t13 + o0, S));
            op[4] = idct_limit(descale(t13 - o0, S));
        }
    }

    void finish(std::vector<uint8_t>& rgba, int& w, int& h) {
        const int W = width_, H = height_;
        // component planes at their padded block size
        std::vector<std::vector<uint8_t>> plane(comp_.size());
        for (size_t ci = 0; ci < comp_.size(); ++ci) {
            Component& c = comp_[ci];
            if (!qt_present_[c.tq]) throw DecodeError("missing quantization table");
            const int pw = c.bw * 8;
            plane[ci].assign((size_t)pw * (size_t)(c.bh * 8), 0);
            for (int by = 0; by < c.bh; ++by)
                for (int bx = 0; bx < c.bw; ++bx)
                    idct_islow(&c.coef[((size_t)by * c.bw + bx) * 64], qt_[c.tq],
                               &plane[ci][(size_t)by * 8 * pw + (size_t)bx * 8], pw);
        }
        // full-resolution component rows (fancy upsampling as libjpeg's jdsample.c)
        std::vector<std::vector<uint8_t>> full(comp_.size());
        for (size_t ci = 0; ci < comp_.size(); ++ci) {
            const Component& c = comp_[ci];
            const int pw = c.bw * 8;
            const int fx = hmax_ / c.h, fy = vmax_ / c.v;
            const bool integral = hmax_ % c.h == 0 && vmax_ % c.v == 0;
            if (!integral) throw DecodeError("non-integral sampling factors are not supported");
            const int ow = c.cw * fx;   // >= W
            std::vector<uint8_t>& f = full[ci];
            f.assign((size_t)ow * (size_t)H, 0);
            const uint8_t* P = plane[ci].data();
            auto row = [&](int y) { return P + (size_t)(y < 0 ? 0 : (y >= c.ch ? c.ch - 1 : y)) * pw; };
            // libjpeg (jinit_upsampler) uses the fancy filters only for planes
            // wider than 2 samples; narrower ones are replicated
            const bool fancy = c.cw > 2;
            if (fx == 1 && fy == 1) {
                for (int y = 0; y < H; ++y) std::memcpy(&f[(size_t)y * ow], row(y), (size_t)ow);
            } else if (fancy && fx == 2 && fy == 1) {   // h2v1_fancy_upsample
                for (int y = 0; y < H; ++y) {
                    const uint8_t* in = row(y);
                    uint8_t* o = &f[(size_t)y * ow];
                    const int n = c.cw;
                    o[0] = in[0];
                    o[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
                    for (int i = 1; i < n - 1; ++i) {
                        const int v = in[i] * 3;
                        o[2 * i] = (uint8_t)((v + in[i - 1] + 1) >> 2);
                        o[2 * i + 1] = (uint8_t)((v + in[i + 1] + 2) >> 2);
                    }
                    o[2 * n - 2] = (uint8_t)((in[n - 1] * 3 + in[n - 2] + 1) >> 2);
                    o[2 * n - 1] = in[n - 1];
                }
            } else if (fancy && fx == 2 && fy == 2) {   // h2v2_fancy_upsample, edge rows replicated
                for (int y = 0; y < H; ++y) {
                    const int r = y >> 1;
                    const uint8_t* i0 = row(r);
                    const uint8_t* i1 = row((y & 1) ? r + 1 : r - 1);
                    uint8_t* o = &f[(size_t)y * ow];
                    const int n = c.cw;
                    int thiss = i0[0] * 3 + i1[0];
                    int nexts = i0[1] * 3 + i1[1];
                    o[0] = (uint8_t)((thiss * 4 + 8) >> 4);
                    o[1] = (uint8_t)((thiss * 3 + nexts + 7) >> 4);
                    int last = thiss;
                    thiss = nexts;
                    for (int i = 1; i < n - 1; ++i) {
                        nexts = i0[i + 1] * 3 + i1[i + 1];
                        o[2 * i] = (uint8_t)((thiss * 3 + last + 8) >> 4);
                        o[2 * i + 1] = (uint8_t)((thiss * 3 + nexts + 7) >> 4);
                        last = thiss;
                        thiss = nexts;
                    }
                    o[2 * n - 2] = (uint8_t)((thiss * 3 + last + 8) >> 4);
                    o[2 * n - 1] = (uint8_t)((thiss * 4 + 7) >> 4);
                }
            } else {   // other factors and narrow planes: pixel replication (int_upsample / h2v*_upsample)
                for (int y = 0; y < H; ++y) {
                    const uint8_t* in = row(y / fy);
                    uint8_t* o = &f[(size_t)y * ow];
                    for (int x = 0; x < ow; ++x) o[x] = in[x / fx];
                }
            }
        }
        // color conversion (jdcolor.c ycc_rgb_convert tables), rows stored bottom-up
        constexpr int SB = 16;
        constexpr int32_t HALF = 1 << (SB - 1);
        auto FIX = [](double x) { return (int32_t)(x * (1 << SB) + 0.5); };
        int32_t crr[256], cbb[256], crg[256], cbg[256];
        for (int i = 0; i < 256; ++i) {
            const int32_t x = i - 128;
            crr[i] = (FIX(1.40200) * x + HALF) >> SB;
            cbb[i] = (FIX(1.77200) * x + HALF) >> SB;
            crg[i] = -FIX(0.71414) * x;
            cbg[i] = -FIX(0.34414) * x + HALF;
        }
        auto clamp8 = [](int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); };
        // JFIF: YCbCr unless an Adobe marker says "no transform" (then RGB)
        const bool ycc = adobe_transform_ != 0;
        rgba.assign((size_t)W * (size_t)H * 4, 255);
        const int ow0 = comp_[0].cw * (hmax_ / comp_[0].h), ow1 = comp_[1].cw * (hmax_ / comp_[1].h),
                  ow2 = comp_[2].cw * (hmax_ / comp_[2].h);
        for (int y = 0; y < H; ++y) {
            const uint8_t* Y = &full[0][(size_t)y * ow0];
            const uint8_t* Cb = &full[1][(size_t)y * ow1];
            const uint8_t* Cr = &full[2][(size_t)y * ow2];
            uint8_t* o = &rgba[(size_t)(H - 1 - y) * W * 4];
            for (int x = 0; x < W; ++x) {
                if (ycc) {
                    const int yy = Y[x], cb = Cb[x], cr = Cr[x];
                    o[4 * x + 0] = clamp8(yy + crr[cr]);
                    o[4 * x + 1] = clamp8(yy + ((cbg[cb] + crg[cr]) >> SB));
                    o[4 * x + 2] = clamp8(yy + cbb[cb]);
                } else {
                    o[4 * x + 0] = Y[x];
                    o[4 * x + 1] = Cb[x];
                    o[4 * x + 2] = Cr[x];
                }
            }
        }
        w = W;
        h = H;
    }
};

void read_ppm(const std::vector<uint8_t>& d, std::vector<uint8_t>& rgba, int& w, int& h) {
    size_t p = 2;
    auto token = [&]() -> long {
        for (;;) {
            while (p < d.size() && std::isspace(d[p])) ++p;
            if (p < d.size() && d[p] == '#') {
                while (p < d.size() && d[p] != '\n') ++p;
                continue;
            }
            break;
        }
        long v = 0;
        bool any = false;
        while (p < d.size() && d[p] >= '0' && d[p] <= '9') {
            v = v * 10 + (d[p++] - '0');
            any = true;
            if (v > (1L << 30)) throw DecodeError("bad PPM header");
        }
        if (!any) throw DecodeError("bad PPM header");
        return v;
    };
    const long W = token(), H = token(), maxv = token();
    ++p;   // the single whitespace byte before the raster
    if (W <= 0 || H <= 0 || maxv != 255) throw DecodeError("only 8-bit binary PPM (P6) is supported");
    if (p + (size_t)W * (size_t)H * 3 > d.size()) throw DecodeError("truncated PPM");
    rgba.assign((size_t)W * (size_t)H * 4, 255);
    for (long y = 0; y < H; ++y)
        for (long x = 0; x < W; ++x) {
            const uint8_t* s = &d[p + ((size_t)y * W + x) * 3];
            uint8_t* o = &rgba[((size_t)(H - 1 - y) * W + x) * 4];   // bottom-up
            o[0] = s[0];
            o[1] = s[1];
            o[2] = s[2];
        }
    w = (int)W;
    h = (int)H;
}

}  // namespace

void load_image(const std::string& path, std::vector<uint8_t>& rgba, int& w, int& h) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw io_error("Failed to open file " + path);
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    try {
        if (d.size() >= 2 && d[0] == 0xFF && d[1] == 0xD8) {
            Jpeg(d.data(), d.size()).decode(rgba, w, h);
        } else if (d.size() >= 2 && d[0] == 'P' && d[1] == '6') {
            read_ppm(d, rgba, w, h);
        } else {
            throw DecodeError("unsupported image format (JPEG or binary PPM expected)");
        }
    } catch (const DecodeError& e) {
        throw std::runtime_error(path + ": " + e.what());
    }
}

}  // namespace tpt
