// output.cpp — the reference CLI's output muxers (tools/output/{md5,yuv,y4m2,null}.rs) as a
// C ABI (include/mi_av1out.h): what rav1d writes per displayed picture, byte for byte.
//
// md5:  the visible rows of every plane, w << hbd bytes each, luma then U then V
//       (md5_write, tools/output/md5.rs:541-576), hashed with MD5 (RFC 1321; md5_finish
//       :578-586 is the standard padding), printed as the four state words in little-endian
//       byte order (md5_close :588-606) — the digest the meson test vectors list.
// yuv:  the same rows, raw (yuv_write, tools/output/yuv.rs).
// y4m2: a "YUV4MPEG2 W H F Ip A C" header before the first picture (write_header,
//       tools/output/y4m2.rs: the aspect ratio is (h * render_w) : (w * render_h) reduced by
//       their gcd, the colour-space tag from layout, bit depth and chroma sample position),
//       then "FRAME\n" + the rows per picture (y4m2_write).
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "mi_av1out.h"

namespace {

struct Md5 {
    uint32_t s[4] = { 0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u };
    uint64_t len = 0;          // bytes
    uint8_t buf[64];
    bool done = false;

    static uint32_t rol(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

    void block(const uint8_t *p) {
        // RFC 1321 section 3.4: four rounds of 16 steps; per-step shift amounts and the
        // constants floor(|sin(i + 1)| * 2^32)
        static const int R[4][4] = { { 7, 12, 17, 22 }, { 5, 9, 14, 20 }, { 4, 11, 16, 23 }, { 6, 10, 15, 21 } };
        struct KT {
            uint32_t v[64];
            KT() {
                for (int i = 0; i < 64; i++) v[i] = (uint32_t)(std::fabs(std::sin((double)(i + 1))) * 4294967296.0);
            }
        };
        static const KT kt;   // thread-safe one-time initialisation
        const uint32_t *K = kt.v;
        uint32_t x[16];
        for (int i = 0; i < 16; i++)
            x[i] = (uint32_t)p[4 * i] | (uint32_t)p[4 * i + 1] << 8 | (uint32_t)p[4 * i + 2] << 16 | (uint32_t)p[4 * i + 3] << 24;
        uint32_t a = s[0], b = s[1], c = s[2], d = s[3];
        for (int i = 0; i < 64; i++) {
            const int r = i >> 4;
            uint32_t f;
            int g;
            if (r == 0) { f = (b & c) | (~b & d); g = i; }
            else if (r == 1) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
            else if (r == 2) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
            else { f = c ^ (b | ~d); g = (7 * i) & 15; }
            const uint32_t t = d;
            d = c;
            c = b;
            b = b + rol(a + f + K[i] + x[g], R[r][i & 3]);
            a = t;
        }
        s[0] += a; s[1] += b; s[2] += c; s[3] += d;
    }

    void update(const uint8_t *p, size_t n) {
        size_t fill = len & 63;
        len += n;
        if (fill) {
            const size_t k = n < 64 - fill ? n : 64 - fill;
            memcpy(buf + fill, p, k);
            p += k; n -= k; fill += k;
            if (fill < 64) return;
            block(buf);
        }
        for (; n >= 64; p += 64, n -= 64) block(p);
        memcpy(buf, p, n);
    }

    void finish() {
        if (done) return;
        const uint64_t bits = len << 3;
        const uint8_t one = 0x80, zero = 0;
        update(&one, 1);
        while ((len & 63) != 56) update(&zero, 1);
        uint8_t l[8];
        for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (8 * i));
        update(l, 8);
        done = true;
    }

    void hex(char out[33]) const {
        for (int i = 0; i < 4; i++)
            snprintf(out + 8 * i, 9, "%02x%02x%02x%02x", s[i] & 0xff, (s[i] >> 8) & 0xff, (s[i] >> 16) & 0xff, s[i] >> 24);
    }
};

enum Kind { MD5, YUV, Y4M2, NUL };

}  // namespace

struct MiMuxer {
    Kind kind;
    FILE *f = nullptr;
    bool own = false, first = true;
    MiOutParams p;
    unsigned fps[2] = { 25, 1 };
    Md5 md5;
};

namespace {

int open_file(MiMuxer *m, const char *file) {
    if (!file) return m->kind == MD5 || m->kind == NUL ? 0 : -EINVAL;
    if (!strcmp(file, "-")) { m->f = stdout; return 0; }
    m->f = fopen(file, "wb");
    if (!m->f) return -EIO;
    m->own = true;
    return 0;
}

// y4m2 colour-space tag (tools/output/y4m2.rs write_header)
const char *y4m_tag(const MiOutParams &p) {
    static const char *ss[4][3] = { { "mono", "mono10", "mono12" },
                                    { nullptr, "420p10", "420p12" },
                                    { "422", "422p10", "422p12" },
                                    { "444", "444p10", "444p12" } };
    static const char *c420[3] = { "420jpeg", "420mpeg2", "420" };
    if (p.layout == 1 && p.bpc == 8) return c420[p.chr > 2 || p.chr < 0 ? 0 : p.chr];
    const int hbd = p.bpc == 8 ? 0 : p.bpc == 10 ? 1 : 2;
    return ss[p.layout & 3][hbd];
}

int y4m_header(MiMuxer *m, const MiPicture *pic) {
    uint64_t aw = (uint64_t)(uint32_t)pic->h * (uint64_t)(uint32_t)m->p.render_w;
    uint64_t ah = (uint64_t)(uint32_t)pic->w * (uint64_t)(uint32_t)m->p.render_h;
    uint64_t g = ah, a = aw;
    while (g) { const uint64_t b = a % g; a = g; g = b; }    // gcd(aw, ah) = a
    if (a) { aw /= a; ah /= a; }
    MiOutParams hp = m->p;
    hp.layout = pic->layout;
    hp.bpc = pic->bpc;
    return fprintf(m->f, "YUV4MPEG2 W%u H%u F%u:%u Ip A%llu:%llu C%s\n", (unsigned)pic->w, (unsigned)pic->h,
                   m->fps[0], m->fps[1], (unsigned long long)aw, (unsigned long long)ah, y4m_tag(hp)) < 0 ? -EIO : 0;
}

// the visible rows of every plane, w << hbd bytes each (md5_write / yuv_write / y4m2_write)
template <typename F>
int for_rows(const MiPicture *pic, F &&emit) {
    const int hbd = pic->bpc > 8;
    const uint8_t *y = (const uint8_t *)pic->data[0];
    for (int r = 0; r < pic->h; r++)
        if (int e = emit(y + (ptrdiff_t)r * pic->stride[0], (size_t)pic->w << hbd)) return e;
    if (pic->layout) {
        const int ss_ver = pic->layout == 1, ss_hor = pic->layout != 3;
        const int cw = (pic->w + ss_hor) >> ss_hor, ch = (pic->h + ss_ver) >> ss_ver;
        for (int pl = 1; pl <= 2; pl++) {
            const uint8_t *c = (const uint8_t *)pic->data[pl];
            for (int r = 0; r < ch; r++)
                if (int e = emit(c + (ptrdiff_t)r * pic->stride[1], (size_t)cw << hbd)) return e;
        }
    }
    return 0;
}

}  // namespace

extern "C" {

int mi_muxer_open(MiMuxer **out, const char *name, const char *file, const MiOutParams *p, const unsigned fps[2]) {
    if (!out || !name) return -EINVAL;
    *out = nullptr;
    Kind k;
    if (!strcmp(name, "md5")) k = MD5;
    else if (!strcmp(name, "yuv")) k = YUV;
    else if (!strcmp(name, "y4m2")) k = Y4M2;
    else if (!strcmp(name, "null")) k = NUL;
    else return -EINVAL;
    if (k == Y4M2 && !p) return -EINVAL;
    MiMuxer *m = new MiMuxer();
    m->kind = k;
    if (p) m->p = *p;
    else memset(&m->p, 0, sizeof(m->p));
    if (fps) { m->fps[0] = fps[0]; m->fps[1] = fps[1]; }
    if (int e = open_file(m, file)) { delete m; return e; }
    *out = m;
    return 0;
}

int mi_muxer_write(MiMuxer *m, const MiPicture *pic) {
    if (!m || !pic || !pic->data[0] || pic->w <= 0 || pic->h <= 0 || pic->layout < 0 || pic->layout > 3 ||
        (pic->bpc != 8 && pic->bpc != 10 && pic->bpc != 12) || (pic->layout && (!pic->data[1] || !pic->data[2])))
        return -EINVAL;
    switch (m->kind) {
    case NUL:
        return 0;
    case MD5:
        if (m->md5.done) return -EINVAL;
        return for_rows(pic, [&](const uint8_t *row, size_t n) { m->md5.update(row, n); return 0; });
    case Y4M2:
        if (m->first) {
            m->first = false;
            if (int e = y4m_header(m, pic)) return e;
        }
        if (fputs("FRAME\n", m->f) < 0) return -EIO;
        [[fallthrough]];
    case YUV:
        return for_rows(pic, [&](const uint8_t *row, size_t n) { return fwrite(row, n, 1, m->f) == 1 ? 0 : -EIO; });
    }
    return -EINVAL;
}

int mi_muxer_verify(MiMuxer *m, const char *md5_str) {
    if (!m || m->kind != MD5 || !md5_str) return -EINVAL;
    if (strlen(md5_str) < 32) return -1;
    m->md5.finish();
    for (int i = 0; i < 4; i++) {
        uint32_t w = 0;
        for (int j = 0; j < 4; j++) {
            const char t[3] = { md5_str[8 * i + 2 * j], md5_str[8 * i + 2 * j + 1], 0 };
            w |= (uint32_t)strtoul(t, nullptr, 16) << (8 * j);
        }
        if (w != m->md5.s[i]) return 1;
    }
    return 0;
}

int mi_muxer_digest(MiMuxer *m, char out[33]) {
    if (!m || m->kind != MD5 || !out) return -EINVAL;
    m->md5.finish();
    m->md5.hex(out);
    return 0;
}

void mi_muxer_close(MiMuxer *m) {
    if (!m) return;
    if (m->kind == MD5 && m->f) {
        char h[33];
        m->md5.finish();
        m->md5.hex(h);
        fprintf(m->f, "%s\n", h);
    }
    if (m->own) fclose(m->f);
    else if (m->f) fflush(m->f);
    delete m;
}

}  // extern "C"
