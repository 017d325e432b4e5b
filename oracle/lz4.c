/* lz4.c — CPU restatement of the LZ4 block and frame formats as mpx uses them (TEST
 * INFRASTRUCTURE ONLY).
 *
 * mpx compresses a connection with github.com/pierrec/lz4/v4 v4.1.21 (mpx/conn_writer.go:42-56:
 * lz4.NewWriter + BlockSizeOption(Block256Kb); mpx/conn_reader.go:53-62: lz4.NewReader).  That
 * module is not in /root/reference, so this file restates the published LZ4 formats:
 *   - block: sequences of [token][literal length ext][literals][offset u16 LE][match length ext],
 *     min match 4; decode semantics follow pierrec's decodeBlock (internal/lz4block/
 *     decode_other.go): empty input, offset 0, offset beyond the output start, input or output
 *     overrun, a final token with a match nibble but no offset => error;
 *   - frame: magic 0x184D2204, FLG (version 01, B.Indep, B.Checksum, C.Size, C.Checksum, DictID),
 *     BD (block max 64K..4M), optional content size / dict id, HC = (xxh32(descriptor) >> 8) &
 *     0xFF; blocks [u32 LE size, bit 31 = stored uncompressed][data][xxh32 if B.Checksum]; end
 *     mark 0; xxh32 of the content if C.Checksum; skippable frames 0x184D2A5x.
 * The compressor is a plain greedy one (any valid compressor: the decoder is what is pinned);
 * parity against pierrec's exact compressed bytes is unpinned (module absent), decompression
 * parity is pinned by round trips and hand-made blocks (tests/test_oracle_lz4.py). */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "spec_oracle.h"

/* ---- xxHash32 (the published algorithm) ---- */
static const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint32_t round32(uint32_t acc, uint32_t in) { return rotl32(acc + in * P2, 13) * P1; }

uint32_t so_xxh32(const void *data, size_t len, uint32_t seed) {
    const uint8_t *p = (const uint8_t *)data, *end = p + len;
    uint32_t h;
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const uint8_t *lim = end - 16;
        do {
            v1 = round32(v1, rd32(p));
            v2 = round32(v2, rd32(p + 4));
            v3 = round32(v3, rd32(p + 8));
            v4 = round32(v4, rd32(p + 12));
            p += 16;
        } while (p <= lim);
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    while (p + 4 <= end) {
        h = rotl32(h + rd32(p) * P3, 17) * P4;
        p += 4;
    }
    while (p < end) {
        h = rotl32(h + (*p) * P5, 11) * P1;
        p++;
    }
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

/* ---- block decode (pierrec/lz4/v4 internal/lz4block decodeBlock, no dictionary) ----
 * Returns the decompressed size, or -1 on any error. */
long long so_lz4_decompress_block(const uint8_t *src, size_t n, uint8_t *dst, size_t cap) {
    if (n == 0) return -1;
    size_t si = 0, di = 0;
    while (si < n) {
        const uint32_t b = src[si++];
        size_t ll = b >> 4;
        if (ll == 15) {
            for (;;) {
                if (si >= n) return -1;
                const uint32_t x = src[si++];
                ll += x;
                if (x != 255) break;
            }
        }
        if (ll) {
            if (si + ll > n || di + ll > cap) return -1;
            memcpy(dst + di, src + si, ll);
            si += ll;
            di += ll;
        }
        size_t ml = b & 15;
        if (si == n && ml == 0) break;
        if (si + 2 > n) return -1;
        const size_t off = (size_t)src[si] | ((size_t)src[si + 1] << 8);
        si += 2;
        if (off == 0) return -1;
        ml += 4;
        if (ml == 19) {
            for (;;) {
                if (si >= n) return -1;
                const uint32_t x = src[si++];
                ml += x;
                if (x != 255) break;
            }
        }
        if (off > di || di + ml > cap) return -1;
        for (size_t i = 0; i < ml; i++) dst[di + i] = dst[di - off + i]; /* overlapping copies repeat */
        di += ml;
    }
    return (long long)di;
}

/* ---- block encode: greedy, 4-byte hash of the last position seen ----
 * Returns the compressed size, or -1 if it does not fit cap. */
static uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> 16; }
static int put_len(uint8_t *dst, size_t cap, size_t *o, size_t v) {
    while (v >= 255) {
        if (*o >= cap) return -1;
        dst[(*o)++] = 255;
        v -= 255;
    }
    if (*o >= cap) return -1;
    dst[(*o)++] = (uint8_t)v;
    return 0;
}
long long so_lz4_compress_block(const uint8_t *src, size_t n, uint8_t *dst, size_t cap) {
    size_t o = 0, anchor = 0, i = 0;
    int32_t *tab = (int32_t *)malloc(sizeof(int32_t) << 16);
    if (!tab) return -1;
    for (size_t k = 0; k < (1u << 16); k++) tab[k] = -1;
    /* format rules: the last 5 bytes are literals, the last match starts >= 12 bytes before the end */
    const size_t mflimit = n > 12 ? n - 12 : 0;
    while (n >= 13 && i < mflimit) {
        const uint32_t v = rd32(src + i), h = hash4(v);
        const int32_t ref = tab[h];
        tab[h] = (int32_t)i;
        if (ref < 0 || i - (size_t)ref > 65535 || rd32(src + ref) != v) {
            i++;
            continue;
        }
        size_t ml = 4;
        while (i + ml < n - 5 && src[ref + ml] == src[i + ml]) ml++;
        const size_t ll = i - anchor;
        if (o >= cap) goto fail;
        uint8_t *tok = dst + o++;
        *tok = (uint8_t)(((ll >= 15 ? 15 : ll) << 4) | (ml - 4 >= 15 ? 15 : ml - 4));
        if (ll >= 15 && put_len(dst, cap, &o, ll - 15)) goto fail;
        if (o + ll + 2 > cap) goto fail;
        memcpy(dst + o, src + anchor, ll);
        o += ll;
        const size_t off = i - (size_t)ref;
        dst[o++] = (uint8_t)off;
        dst[o++] = (uint8_t)(off >> 8);
        if (ml - 4 >= 15 && put_len(dst, cap, &o, ml - 4 - 15)) goto fail;
        for (size_t k = i + 1; k < i + ml && k + 4 <= n; k++) tab[hash4(rd32(src + k))] = (int32_t)k;
        i += ml;
        anchor = i;
    }
    {
        const size_t ll = n - anchor;
        if (o >= cap) goto fail;
        dst[o++] = (uint8_t)((ll >= 15 ? 15 : ll) << 4);
        if (ll >= 15 && put_len(dst, cap, &o, ll - 15)) goto fail;
        if (o + ll > cap) goto fail;
        memcpy(dst + o, src + anchor, ll);
        o += ll;
    }
    free(tab);
    return (long long)o;
fail:
    free(tab);
    return -1;
}

/* ---- frames ---- */
static void wr32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}
static int bd_code(uint32_t block_max) {
    switch (block_max) {
    case 64u << 10: return 4;
    case 256u << 10: return 5;
    case 1u << 20: return 6;
    case 4u << 20: return 7;
    }
    return -1;
}

/* One frame as pierrec's Writer produces it for a connection: header (B.Indep, C.Checksum as
 * given, block checksums as given), then for every flush segment [flush_ends[k-1], flush_ends[k])
 * its data in blocks of block_max (a Flush compresses the pending partial block), each block
 * stored uncompressed when compression does not shrink it; `close` appends the end mark and
 * the content checksum.  Returns the frame size, or -1. */
long long so_lz4_frame_write(const uint8_t *data, const uint64_t *flush_ends, size_t nflush, uint32_t block_max,
                             int content_checksum, int block_checksum, int close, uint8_t *out, size_t cap) {
    const int bd = bd_code(block_max);
    if (bd < 0 || cap < 7) return -1;
    size_t o = 0;
    wr32(out, 0x184D2204u);
    out[4] = (uint8_t)(0x40 | 0x20 | (block_checksum ? 0x10 : 0) | (content_checksum ? 0x04 : 0));
    out[5] = (uint8_t)(bd << 4);
    out[6] = (uint8_t)((so_xxh32(out + 4, 2, 0) >> 8) & 0xff);
    o = 7;
    uint8_t *tmp = (uint8_t *)malloc(block_max + block_max / 255 + 64);
    if (!tmp) return -1;
    uint64_t prev = 0;
    for (size_t k = 0; k < nflush; k++) {
        for (uint64_t p = prev; p < flush_ends[k]; p += block_max) {
            const size_t bn = (size_t)(flush_ends[k] - p < block_max ? flush_ends[k] - p : block_max);
            const long long c = so_lz4_compress_block(data + p, bn, tmp, bn - 1 > 0 ? bn - 1 : 0);
            const int stored = c < 0;
            const size_t sz = stored ? bn : (size_t)c;
            if (o + 4 + sz + 4 > cap) goto fail;
            wr32(out + o, (uint32_t)sz | (stored ? 0x80000000u : 0));
            memcpy(out + o + 4, stored ? data + p : tmp, sz);
            o += 4 + sz;
            if (block_checksum) {
                wr32(out + o, so_xxh32(out + o - sz, sz, 0));
                o += 4;
            }
        }
        prev = flush_ends[k];
    }
    if (close) {
        if (o + 8 > cap) goto fail;
        wr32(out + o, 0);
        o += 4;
        if (content_checksum) {
            wr32(out + o, so_xxh32(data, (size_t)prev, 0));
            o += 4;
        }
    }
    free(tmp);
    return (long long)o;
fail:
    free(tmp);
    return -1;
}

/* The reader side (pierrec Reader over a byte buffer): every frame in buf (and skippable
 * frames), every COMPLETE block decompressed into out.  *consumed = bytes of buf used (an
 * incomplete block or header at the end is left); returns 0, or a negative error:
 * -1 bad magic/version/reserved bits, -2 header checksum, -3 block size > block max,
 * -4 corrupt block, -5 block checksum, -6 content checksum, -7 out too small. */
int so_lz4_frame_read(const uint8_t *buf, size_t len, uint8_t *out, size_t cap, size_t *out_len, size_t *consumed) {
    size_t p = 0, o = 0;
    *out_len = 0;
    *consumed = 0;
    while (p + 4 <= len) {
        const uint32_t magic = rd32(buf + p);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) { /* skippable frame */
            if (p + 8 > len) break;
            const size_t sz = rd32(buf + p + 4);
            if (p + 8 + sz > len) break;
            p += 8 + sz;
            *consumed = p;
            continue;
        }
        if (magic != 0x184D2204u) return -1;
        if (p + 7 > len) break;
        const uint8_t flg = buf[p + 4], bd = buf[p + 5];
        if ((flg >> 6) != 1 || (flg & 0x02) || (bd & 0x8F)) return -1;
        const int bcs = (flg >> 4) & 1, csz = (flg >> 3) & 1, ccs = (flg >> 2) & 1, dict = flg & 1;
        const size_t hlen = 2 + (csz ? 8 : 0) + (dict ? 4 : 0);
        if (p + 4 + hlen + 1 > len) break;
        if (((so_xxh32(buf + p + 4, hlen, 0) >> 8) & 0xff) != buf[p + 4 + hlen]) return -2;
        const int code = (bd >> 4) & 7;
        if (code < 4) return -1;
        const size_t bmax = (size_t)1 << (8 + 2 * code);
        size_t q = p + 4 + hlen + 1, frame_start_o = o;
        int closed = 0;
        while (q + 4 <= len) {
            const uint32_t w = rd32(buf + q);
            if (w == 0) { /* end mark */
                if (ccs) {
                    if (q + 8 > len) break;
                    if (so_xxh32(out + frame_start_o, o - frame_start_o, 0) != rd32(buf + q + 4)) return -6;
                    q += 8;
                } else {
                    q += 4;
                }
                closed = 1;
                break;
            }
            const size_t sz = w & 0x7FFFFFFFu;
            if (sz > bmax) return -3;
            if (q + 4 + sz + (bcs ? 4 : 0) > len) break;
            if (bcs && so_xxh32(buf + q + 4, sz, 0) != rd32(buf + q + 4 + sz)) return -5;
            if (w & 0x80000000u) {
                if (o + sz > cap) return -7;
                memcpy(out + o, buf + q + 4, sz);
                o += sz;
            } else {
                const size_t room = cap - o < bmax ? cap - o : bmax;
                const long long d = so_lz4_decompress_block(buf + q + 4, sz, out + o, room);
                if (d < 0) return room < bmax ? -7 : -4;
                o += (size_t)d;
            }
            q += 4 + sz + (bcs ? 4 : 0);
            *out_len = o;
            *consumed = q;
        }
        *out_len = o;
        if (!closed) break;
        p = q;
        *consumed = p;
    }
    *out_len = o;
    return 0;
}
