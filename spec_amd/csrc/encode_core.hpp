// encode_core.hpp — device code shared by the flat and nested encoders (gfx950).
//
// Restates, per message, what the reference Writer produces (internal/writer/writer.go:376-553,
// internal/encode/...): field values in write order, the table sorted by tag with the
// insertion-sort tie rule (internal/writer/stack_msg.go:37-61, precomputed on the host as
// `order`), the trailer rvarint(dataSize) | rvarint(tableSize) | type (internal/encode/msg.go:15-77).
#pragma once

#include "spec_device.hpp"

#ifndef SPEC_MAX_FIELDS
#define SPEC_MAX_FIELDS 64
#endif

namespace spec {

// The columns one message's fields are written from.
struct EncFields {
    uint32_t nfields;
    uint16_t tags[SPEC_MAX_FIELDS];
    uint8_t kinds[SPEC_MAX_FIELDS];
    uint8_t order[SPEC_MAX_FIELDS]; // table order: order[j] = schema index of j-th table entry
    const void *cols[SPEC_MAX_FIELDS];
    const uint8_t *heaps[SPEC_MAX_FIELDS];
    uint64_t heap_lens[SPEC_MAX_FIELDS];
    uint32_t table_big_forced; // 1 if any tag > 255 (IsBigMessage holds for every record)
};

constexpr uint64_t MAX_SIZE = 2147483647ull; // format.MaxSize, type.go:14

__device__ __forceinline__ uint32_t vlen64(uint64_t v) {
    uint32_t bits = v ? 64 - __builtin_clzll(v) : 1;
    return (bits + 6) / 7;
}
__device__ __forceinline__ uint32_t vlen32(uint32_t v) { return vlen64(v); }
__device__ __forceinline__ uint32_t zigzag32(int32_t v) { return ((uint32_t)v << 1) ^ (uint32_t)(v >> 31); }
__device__ __forceinline__ uint64_t zigzag64(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }

__device__ __forceinline__ uint32_t kind_width(uint32_t k) {
    switch (k) {
    case K_BOOL: case K_BYTE: return 1;
    case K_INT16: case K_UINT16: return 2;
    case K_INT32: case K_UINT32: case K_FLOAT32: return 4;
    case K_BIN128: return 16;
    case K_BIN256: return 32;
    default: return 8;
    }
}

// Encoded size of field f of record r (value | type, internal/encode/...); err set on an
// encoder error (string/bytes > MaxSize or outside its heap).
__device__ __forceinline__ uint64_t field_size(const EncFields &a, uint32_t f, uint64_t r, bool check_heaps,
                                               bool &err) {
    const uint8_t *col = (const uint8_t *)a.cols[f];
    switch (a.kinds[f]) {
    case K_BOOL: return 1;
    case K_BYTE: return 2;
    case K_INT16: return vlen32(zigzag32(((const int16_t *)col)[r])) + 1;
    case K_INT32: return vlen32(zigzag32(((const int32_t *)col)[r])) + 1;
    case K_INT64: return vlen64(zigzag64(((const int64_t *)col)[r])) + 1;
    case K_UINT16: return vlen32(((const uint16_t *)col)[r]) + 1;
    case K_UINT32: return vlen32(((const uint32_t *)col)[r]) + 1;
    case K_UINT64: return vlen64(((const uint64_t *)col)[r]) + 1;
    case K_FLOAT32: return 5;
    case K_FLOAT64: return 9;
    case K_BIN64: return 9;
    case K_BIN128: return 17;
    case K_BIN256: return 33;
    case K_STRING:
    case K_BYTES: {
        uint2 sp = ((const uint2 *)col)[r];
        if ((uint64_t)sp.y > MAX_SIZE || (check_heaps && (uint64_t)sp.x + sp.y > a.heap_lens[f])) err = true;
        return (uint64_t)sp.y + vlen32(sp.y) + 1 + (a.kinds[f] == K_STRING ? 1 : 0);
    }
    }
    return 0;
}

struct RecSize {
    uint64_t total, data;
    bool big;
};

// lists(f, r) returns the encoded size of a K_LIST field (nested encode); flat schemas have none.
struct NoLists {
    __device__ __forceinline__ uint64_t operator()(uint32_t, uint64_t) const { return 0; }
};

template <class Lists = NoLists>
__device__ __forceinline__ RecSize record_size(const EncFields &a, uint64_t r, bool check_heaps, bool &err,
                                               const Lists &lists = Lists()) {
    uint64_t data = 0;
    for (uint32_t f = 0; f < a.nfields; f++)
        data += a.kinds[f] == K_LIST ? lists(f, r) : field_size(a, f, r, check_heaps, err);
    // IsBigMessage (internal/format/msg.go:43-61): any tag > 255 or any end offset > 65535;
    // ends grow in write order so the largest is the data size.
    bool big = a.table_big_forced || (a.nfields > 0 && data > 65535);
    uint64_t tsize = (uint64_t)a.nfields * (big ? 6 : 3);
    if (data > MAX_SIZE) err = true; // EncodeMessageTable: message too large
    RecSize s;
    s.data = data;
    s.big = big;
    s.total = data + tsize + vlen32((uint32_t)data) + vlen32((uint32_t)tsize) + 1;
    return s;
}

// ---- pass 2: exclusive scan of block sums (one workgroup), total ----------------------

// One 1024-thread workgroup: block_sums[0..nblocks) -> exclusive offsets, block_sums[nblocks]
// and *total = the total (all-ones if any block reported an encoder error).
__device__ __forceinline__ void scan_block_sums(uint64_t *block_sums, uint64_t nblocks, uint64_t *total) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry_s;
    __shared__ int err_s;
    if (threadIdx.x == 0) {
        carry_s = 0;
        err_s = 0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t base = 0; base < nblocks; base += 1024) {
        uint64_t i = base + threadIdx.x;
        uint64_t v = i < nblocks ? block_sums[i] : 0;
        if (v == ~0ull) {
            err_s = 1;
            v = 0;
        }
        uint64_t x = v; // inclusive wave scan
        for (int o = 1; o < 64; o <<= 1) {
            uint64_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint64_t wpre = 0;
        for (int w = 0; w < wave; w++) wpre += wsum[w];
        uint64_t carry = carry_s;
        if (i < nblocks) block_sums[i] = carry + wpre + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry_s = carry + wpre + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        uint64_t t = err_s ? ~0ull : carry_s;
        block_sums[nblocks] = t;
        if (total) *total = t;
    }
}

// Byte sinks.  Positions are in sink coordinates; `lo` is the first byte this lane owns (a
// dword straddling lo is written bytewise so neighbouring records are never clobbered).
struct LdsSink {
    uint8_t *slab;
    __device__ __forceinline__ void st1(int p, uint32_t b) const { slab[p] = (uint8_t)b; }
    __device__ __forceinline__ void st4a(int p, uint32_t w) const { *(uint32_t *)(slab + p) = w; }
};

struct GlobalSink {
    uint8_t *out;
    __device__ __forceinline__ void st1(long long p, uint32_t b) const { out[p] = (uint8_t)b; }
    __device__ __forceinline__ void st4a(long long p, uint32_t w) const {
        out[p] = (uint8_t)w;
        out[p + 1] = (uint8_t)(w >> 8);
        out[p + 2] = (uint8_t)(w >> 16);
        out[p + 3] = (uint8_t)(w >> 24);
    }
};

// Sequential emitter that merges bytes into dwords (aligned in sink coordinates).
template <class Sink, class Pos>
struct Emit {
    const Sink &k;
    Pos pos;   // next byte position
    Pos lo;    // first owned byte
    uint32_t acc; // pending bytes of the dword containing pos (bytes below pos&3)

    __device__ __forceinline__ Emit(const Sink &sink, Pos p) : k(sink), pos(p), lo(p), acc(0) {}

    __device__ __forceinline__ void flush_dword(Pos d, uint32_t w) {
        if (d >= lo) {
            k.st4a(d, w);
        } else {
            for (int i = 0; i < 4; i++)
                if (d + i >= lo) k.st1(d + i, (w >> (8 * i)) & 0xff);
        }
    }
    __device__ __forceinline__ void put1(uint32_t b) {
        uint32_t sh = (uint32_t)(pos & 3) * 8;
        acc |= (b & 0xff) << sh;
        pos++;
        if ((pos & 3) == 0) {
            flush_dword(pos - 4, acc);
            acc = 0;
        }
    }
    // 4 bytes in memory order packed little-endian
    __device__ __forceinline__ void put4(uint32_t w) {
        uint32_t k4 = (uint32_t)(pos & 3);
        if (k4 == 0) {
            flush_dword(pos, w);
        } else {
            uint32_t sh = 8 * k4;
            flush_dword(pos - k4, acc | (w << sh));
            acc = w >> (32 - sh);
        }
        pos += 4;
    }
    __device__ __forceinline__ void put8(uint64_t w) {
        put4((uint32_t)w);
        put4((uint32_t)(w >> 32));
    }
    // k (0..8) bytes of v, lowest byte first, merged into the pending dword
    __device__ __forceinline__ void put_n(uint64_t v, uint32_t k) {
        const uint32_t ph = (uint32_t)(pos & 3), sh = 8 * ph;
        const uint64_t lo64 = (uint64_t)acc | (v << sh);
        const uint32_t hi32 = sh ? (uint32_t)(v >> (64 - sh)) : 0u;
        const uint32_t total = ph + k;
        const Pos d = pos & ~(Pos)3;
        if (total >= 4) flush_dword(d, (uint32_t)lo64);
        if (total >= 8) flush_dword(d + 4, (uint32_t)(lo64 >> 32));
        const uint32_t full = total >> 2;
        const uint32_t rest = full == 0 ? (uint32_t)lo64 : (full == 1 ? (uint32_t)(lo64 >> 32) : hi32);
        const uint32_t keep = total & 3;
        acc = keep ? (rest & (0xffffffffu >> (32 - 8 * keep))) : 0u;
        pos += k;
    }
    // reverse varint (oracle/compactint.c so_put_reverse_*): top group first, MSB clear;
    // following groups carry 0x80; the least-significant group is the last byte.  Up to 8
    // bytes (values < 2^56) are built in a register and appended at once.
    __device__ __forceinline__ void rvarint(uint64_t v) {
        const uint32_t L = vlen64(v);
        if (L <= 8) {
            uint64_t x = v & 0x00ffffffffffffffull; // 7-bit groups -> bytes (inverse of rvarint_bf)
            x = (x & 0x000000000fffffffull) | ((x << 4) & 0x0fffffff00000000ull);
            x = (x & 0x00003fff00003fffull) | ((x << 2) & 0x3fff00003fff0000ull);
            x = (x & 0x007f007f007f007full) | ((x << 1) & 0x7f007f007f007f00ull);
            const uint32_t drop = 8 * (8 - L);
            uint64_t out = __builtin_bswap64(x) >> drop;        // byte i = group L-1-i
            const uint64_t cont = (0x8080808080808080ull >> drop) & ~0xffull; // all but the first byte
            put_n(out | cont, L);
            return;
        }
        for (uint32_t i = 0; i < L; i++) {
            uint32_t g = (uint32_t)(v >> (7 * (L - 1 - i))) & 0x7f;
            put1(g | (i ? 0x80 : 0));
        }
    }
    __device__ __forceinline__ void finish() {
        Pos d = pos & ~(Pos)3;
        for (int i = 0; i < (int)(pos - d); i++)
            if (d + i >= lo) k.st1(d + i, (acc >> (8 * i)) & 0xff);
        acc = 0;
    }
};

// 16 heap bytes at dword-aligned offset a (range-checked; a straddling access reads per dword)
__device__ __forceinline__ uint4 heap_ld128(__amdgpu_buffer_rsrc_t hr, uint32_t a, uint64_t hlen) {
    if ((uint64_t)a + 16 <= hlen) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(hr, a, 0, 0);
        return make_uint4(v[0], v[1], v[2], v[3]);
    }
    return make_uint4(buf_ld32(hr, a, hlen), buf_ld32(hr, a + 4, hlen), buf_ld32(hr, a + 8, hlen),
                      buf_ld32(hr, a + 12, hlen));
}

// Copy len bytes of heap[off..] into the emitter: 64 bytes per round from five 16-byte
// range-checked loads issued together (one memory latency per round, not one per dword).
template <class E>
__device__ __forceinline__ void emit_heap(E &em, __amdgpu_buffer_rsrc_t hr, uint64_t hlen, uint32_t off,
                                          uint32_t len) {
    const uint32_t a = off & ~3u, sh = off & 3;
    for (uint32_t i = 0; i < len; i += 64) {
        uint32_t w[20];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const uint4 q = heap_ld128(hr, a + i + 16 * k, hlen);
            w[4 * k] = q.x;
            w[4 * k + 1] = q.y;
            w[4 * k + 2] = q.z;
            w[4 * k + 3] = q.w;
        }
        const uint32_t n = len - i < 64 ? len - i : 64;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if ((uint32_t)(4 * j + 4) <= n) {
                em.put4(__builtin_amdgcn_alignbyte(w[j + 1], w[j], sh));
            } else if ((uint32_t)(4 * j) < n) {
                em.put_n(__builtin_amdgcn_alignbyte(w[j + 1], w[j], sh), n - 4 * j);
            }
        }
    }
}

// lists(em, f, r) emits a K_LIST field's value (nested encode); flat schemas have none.
struct NoListEmit {
    template <class E>
    __device__ __forceinline__ void operator()(E &, uint32_t, uint64_t) const {}
};

// One message (internal/writer/writer.go:376-553): fields in write order, table entries at
// their sorted positions, trailer.  Returns the end position.
template <class Sink, class Pos, class Lists = NoListEmit>
__device__ __forceinline__ Pos emit_message(const EncFields &a, const Sink &k, Pos start, uint64_t r,
                                            const RecSize &rs, const uint8_t *inv_order,
                                            const Lists &lists = Lists()) {
    Emit<Sink, Pos> em(k, start);
    const Pos tstart = start + (Pos)rs.data;
    const uint32_t esize = rs.big ? 6 : 3;
    uint64_t end = 0;
    for (uint32_t f = 0; f < a.nfields; f++) {
        const uint8_t *col = (const uint8_t *)a.cols[f];
        uint32_t kind = a.kinds[f];
        switch (kind) {
        case K_LIST: lists(em, f, r); break;
        case K_BOOL: em.put1(col[r] ? T_TRUE : T_FALSE); break;
        case K_BYTE: em.put1(col[r]); em.put1(T_BYTE); break;
        case K_INT16: em.rvarint(zigzag32(((const int16_t *)col)[r])); em.put1(T_INT16); break;
        case K_INT32: em.rvarint(zigzag32(((const int32_t *)col)[r])); em.put1(T_INT32); break;
        case K_INT64: em.rvarint(zigzag64(((const int64_t *)col)[r])); em.put1(T_INT64); break;
        case K_UINT16: em.rvarint(((const uint16_t *)col)[r]); em.put1(T_UINT16); break;
        case K_UINT32: em.rvarint(((const uint32_t *)col)[r]); em.put1(T_UINT32); break;
        case K_UINT64: em.rvarint(((const uint64_t *)col)[r]); em.put1(T_UINT64); break;
        case K_FLOAT32: em.put4(bswap32(((const uint32_t *)col)[r])); em.put1(T_FLOAT32); break;
        case K_FLOAT64: {
            uint64_t v = ((const uint64_t *)col)[r];
            em.put4(bswap32((uint32_t)(v >> 32)));
            em.put4(bswap32((uint32_t)v));
            em.put1(T_FLOAT64);
            break;
        }
        case K_BIN64: em.put8(((const uint64_t *)col)[r]); em.put1(T_BIN64); break;
        case K_BIN128: {
            ulonglong2 v = ((const ulonglong2 *)col)[r];
            em.put8(v.x);
            em.put8(v.y);
            em.put1(T_BIN128);
            break;
        }
        case K_BIN256: {
            const ulonglong2 *c = (const ulonglong2 *)col + 2 * r;
            ulonglong2 v0 = c[0], v1 = c[1];
            em.put8(v0.x);
            em.put8(v0.y);
            em.put8(v1.x);
            em.put8(v1.y);
            em.put1(T_BIN256);
            break;
        }
        case K_STRING:
        case K_BYTES: {
            uint2 sp = ((const uint2 *)col)[r];
            __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(
                (void *)a.heaps[f], (short)0,
                (int)(uint32_t)(a.heap_lens[f] > 0xffffffffull ? 0xffffffffull : a.heap_lens[f]), 0x00020000);
            emit_heap(em, hr, a.heap_lens[f], sp.x, sp.y);
            if (kind == K_STRING) em.put1(0);
            em.rvarint(sp.y);
            em.put1(kind == K_STRING ? T_STRING : T_BYTES);
            break;
        }
        }
        end = (uint64_t)(em.pos - start);
        // table entry for this field at its sorted position (encode/msg.go:58-72)
        Pos p = tstart + (Pos)(inv_order[f] * esize);
        uint32_t tag = a.tags[f];
        if (rs.big) {
            k.st1(p, tag >> 8);
            k.st1(p + 1, tag & 0xff);
            k.st1(p + 2, (uint32_t)(end >> 24) & 0xff);
            k.st1(p + 3, (uint32_t)(end >> 16) & 0xff);
            k.st1(p + 4, (uint32_t)(end >> 8) & 0xff);
            k.st1(p + 5, (uint32_t)end & 0xff);
        } else {
            k.st1(p, tag & 0xff);
            k.st1(p + 1, (uint32_t)(end >> 8) & 0xff);
            k.st1(p + 2, (uint32_t)end & 0xff);
        }
    }
    em.finish();
    // trailer: rvarint(dataSize) | rvarint(tableSize) | type (encode/msg.go:36-39)
    Emit<Sink, Pos> tr(k, tstart + (Pos)((uint64_t)a.nfields * esize));
    tr.rvarint((uint32_t)rs.data);
    tr.rvarint((uint32_t)(a.nfields * esize));
    tr.put1(rs.big ? T_BIG_MESSAGE : T_MESSAGE);
    tr.finish();
    return tr.pos;
}

} // namespace spec
