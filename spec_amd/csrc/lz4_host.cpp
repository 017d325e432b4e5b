// lz4_host.cpp — spec_lz4_frame_blocks (host walk of LZ4 frame headers and block size words)
// and the C-ABI entry points of the device LZ4 path (lz4_device.hip).
//
// What pierrec/lz4/v4's Reader checks before it decodes a block (mpx/conn_reader.go:53-62 wraps
// the connection in lz4.NewReader), restated from the LZ4 frame format: magic 0x184D2204 (and
// skippable frames 0x184D2A5x), FLG version 01 with reserved bit 0, BD reserved bits 0 and a
// block max code 4..7, the header checksum byte (xxh32 of the descriptor >> 8), a block size no
// larger than the block max, and the block checksum when the frame carries them.
#include <hip/hip_runtime.h>

#include <string.h>

#include "spec_internal.hpp"

namespace {

uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// xxHash32 (the published algorithm), for the frame header and block checksums
uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
uint32_t xxh32(const uint8_t *p, size_t len, uint32_t seed) {
    const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
    const uint8_t *end = p + len;
    uint32_t h;
    if (len >= 16) {
        uint32_t v[4] = {seed + P1 + P2, seed + P2, seed, seed - P1};
        for (; p + 16 <= end; p += 16)
            for (int i = 0; i < 4; i++) v[i] = rotl32(v[i] + rd32(p + 4 * i) * P2, 13) * P1;
        h = rotl32(v[0], 1) + rotl32(v[1], 7) + rotl32(v[2], 12) + rotl32(v[3], 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    for (; p + 4 <= end; p += 4) h = rotl32(h + rd32(p) * P3, 17) * P4;
    for (; p < end; p++) h = rotl32(h + (*p) * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

} // namespace

extern "C" {

int spec_lz4_frame_blocks(const uint8_t *buf, uint64_t len, spec_lz4_state *state, spec_lz4_block *blocks,
                          uint64_t cap, uint64_t *nblocks, uint64_t *consumed, uint32_t *block_max) {
    if ((!buf && len) || !state || !nblocks || !consumed || !block_max || (cap && !blocks))
        return SPEC_E_INVALID_ARGUMENT;
    uint64_t p = 0, k = 0;
    uint32_t bmax_all = state->in_frame ? state->block_max : 0;
    state->flags &= 3u; // bit 2 reports this call only
    *nblocks = 0;
    *consumed = 0;
    int rc = SPEC_OK;
    while (rc == SPEC_OK) {
        if (!state->in_frame) { // a frame header (or a skippable frame)
            if (p + 4 > len) break;
            const uint32_t magic = rd32(buf + p);
            if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
                if (p + 8 > len) break;
                const uint64_t sz = rd32(buf + p + 4);
                if (p + 8 + sz > len) break;
                p += 8 + sz;
                *consumed = p;
                continue;
            }
            if (magic != 0x184D2204u) {
                rc = SPEC_E_CORRUPT;
                break;
            }
            if (p + 7 > len) break;
            const uint8_t flg = buf[p + 4], bd = buf[p + 5];
            if ((flg >> 6) != 1 || (flg & 0x02) || (bd & 0x8F) || ((bd >> 4) & 7) < 4) {
                rc = SPEC_E_CORRUPT;
                break;
            }
            const uint64_t hlen = 2 + ((flg & 0x08) ? 8 : 0) + ((flg & 0x01) ? 4 : 0);
            if (p + 4 + hlen + 1 > len) break;
            if (((xxh32(buf + p + 4, hlen, 0) >> 8) & 0xff) != buf[p + 4 + hlen]) {
                rc = SPEC_E_CORRUPT;
                break;
            }
            state->in_frame = 1;
            state->block_max = 1u << (8 + 2 * ((bd >> 4) & 7));
            state->flags = ((flg & 0x10) ? 1u : 0u) | ((flg & 0x04) ? 2u : 0u) | (state->flags & 4u);
            if (state->block_max > bmax_all) bmax_all = state->block_max;
            p += 4 + hlen + 1;
            *consumed = p;
        }
        // the open frame's blocks
        const bool bcs = state->flags & 1, ccs = state->flags & 2;
        bool more = false;
        while (p + 4 <= len) {
            const uint32_t w = rd32(buf + p);
            if (w == 0) { // end mark (+ content checksum: reported, see include/spec_amd.h)
                const uint64_t tail = 4 + (ccs ? 4 : 0);
                if (p + tail > len) break;
                if (ccs) {
                    state->flags |= 4u;
                    state->content_checksum = rd32(buf + p + 4);
                }
                p += tail;
                *consumed = p;
                state->in_frame = 0;
                more = true;
                break;
            }
            const uint64_t sz = w & 0x7FFFFFFFu;
            if (sz > state->block_max) {
                rc = SPEC_E_CORRUPT;
                break;
            }
            if (p + 4 + sz + (bcs ? 4 : 0) > len) break;
            if (bcs && xxh32(buf + p + 4, sz, 0) != rd32(buf + p + 4 + sz)) {
                rc = SPEC_E_CORRUPT;
                break;
            }
            if (k == cap) {
                rc = SPEC_E_CAPACITY;
                break;
            }
            blocks[k].src_off = p + 4;
            blocks[k].src_len = (uint32_t)sz;
            blocks[k].stored = (w >> 31) & 1;
            k++;
            p += 4 + sz + (bcs ? 4 : 0);
            *consumed = p;
        }
        if (!more) break;
    }
    *nblocks = k;
    *block_max = bmax_all;
    return rc;
}

int spec_lz4_decompress(const uint8_t *src, uint64_t src_len, const spec_lz4_block *blocks, uint64_t nblocks,
                        uint8_t *slots, uint64_t slot_bytes, uint32_t *sizes, uint8_t *status, void *stream) {
    if (nblocks == 0) return SPEC_OK;
    if (!src || !blocks || !slots || !sizes || !status || slot_bytes == 0 || slot_bytes > (64u << 20) ||
        (slot_bytes & 15) || ((uintptr_t)slots & 15))
        return SPEC_E_INVALID_ARGUMENT;
    if (src_len >= (1ull << 32)) return SPEC_E_TOO_LARGE;
    if (spec::launch_lz4_decompress(src, src_len, blocks, nblocks, slots, slot_bytes, sizes, status,
                                    (hipStream_t)stream))
        return SPEC_E_HIP;
    return SPEC_OK;
}

size_t spec_lz4_pack_workspace_size(uint64_t nblocks) { return (size_t)(nblocks + 1) * 8; }

int spec_lz4_content_update(spec_lz4_content *content, const uint8_t *data, uint64_t len, void *stream) {
    if (!content || (len && !data)) return SPEC_E_INVALID_ARGUMENT;
    return spec::launch_lz4_content(content, data, len, nullptr, (hipStream_t)stream) ? SPEC_E_HIP : SPEC_OK;
}

int spec_lz4_content_digest(const spec_lz4_content *content, uint32_t *digest, void *stream) {
    if (!content || !digest) return SPEC_E_INVALID_ARGUMENT;
    return spec::launch_lz4_content((spec_lz4_content *)content, nullptr, 0, digest, (hipStream_t)stream) ? SPEC_E_HIP
                                                                                                          : SPEC_OK;
}

int spec_lz4_pack(const uint8_t *slots, uint64_t slot_bytes, const uint32_t *sizes, uint64_t nblocks, uint8_t *out,
                  uint64_t out_cap, uint64_t *total, void *workspace, size_t workspace_size, void *stream) {
    if (!total || !workspace || (nblocks && (!slots || !sizes)) || (out_cap && !out)) return SPEC_E_INVALID_ARGUMENT;
    if (workspace_size < spec_lz4_pack_workspace_size(nblocks)) return SPEC_E_WORKSPACE;
    if (spec::launch_lz4_pack(slots, slot_bytes, sizes, nblocks, out, out_cap, (uint64_t *)workspace, total,
                              (hipStream_t)stream))
        return SPEC_E_HIP;
    return SPEC_OK;
}

} // extern "C"
