// encode_core.hpp — device code shared by the flat and nested encoders (gfx950).
//
// Restates, per message, what the reference Writer produces (internal/writer/writer.go:376-553,
// internal/encode/...): field values in write order, the table sorted by tag with the
// insertion-sort tie rule (internal/writer/stack_msg.go:37-61, precomputed on the host as
// `order`), the trailer rvarint(dataSize) | rvarint(tableSize) | type (internal/encode/msg.go:15-77).
#pragma once

#include "spec_device.hpp"


namespace spec {

// The columns one message's fields are written from.
struct EncFields {
    uint32_t nfields;
    uint16_t tags[SPEC_KFIELDS];
    uint8_t kinds[SPEC_KFIELDS];
    uint8_t order[SPEC_KFIELDS]; // table order: order[j] = schema index of j-th table entry
    const void *cols[SPEC_KFIELDS];
    const uint8_t *heaps[SPEC_KFIELDS];
    uint64_t heap_lens[SPEC_KFIELDS];
    uint32_t table_big_forced; // 1 if any tag > 255 (IsBigMessage holds for every record)
};

// The field set of a schema with more than SPEC_KFIELDS fields: the same members as EncFields,
// as arrays in device memory (the caller's workspace, uploaded per call), so the kernel argument
// stays small.  field_size / record_size / emit_message read either through the same names.
struct WideEncFields {
    uint32_t nfields;
    uint32_t table_big_forced;
    const uint16_t *tags;
    const uint8_t *kinds;
    const uint16_t *inv_order; // table position of each field (the inverse of the Writer's order)
    const void *const *cols;
    const uint8_t *const *heaps;
    const uint64_t *heap_lens;
};

// Passed by value as the kernel argument (lives in the kernarg segment => scalar loads,
// the per-field loop branches are wave-uniform).
struct EncodeArgs {
    uint64_t n;
    EncFields f;
    uint32_t check_heaps;  // 1 when heaps/heap_lens are known (full encode, not size-only)
    uint8_t *out;
    uint64_t out_cap;
    uint64_t *ends;
    uint64_t ends_base;    // added to every end offset (a shard's first byte in the whole batch)
    uint64_t *block_sums;  // workspace: per-block encoded bytes, then exclusive offsets
    uint64_t nblocks;
    uint64_t *total;
    static constexpr bool kWide = false;
};

// EncodeArgs of a schema with more than SPEC_KFIELDS fields (encode_flat.hip wide kernels).
struct WideEncodeArgs {
    uint64_t n;
    WideEncFields f;
    uint32_t check_heaps;
    uint8_t *out;
    uint64_t out_cap;
    uint64_t *ends;
    uint64_t ends_base;
    uint64_t *block_sums;
    uint64_t nblocks;
    uint64_t *total;
    static constexpr bool kWide = true;
};

constexpr int ENC_BLOCK = 256;            // records per encode block (4 waves, one record per lane)
constexpr int ENC_SLAB = 20 * 1024 - 128; // per-wave output staging (LDS)
constexpr int ENC_LDS_HEAD = 128;         // write kernel LDS header: wave sums + inverse table order

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
template <class FS>
__device__ __forceinline__ uint64_t field_size(const FS &a, uint32_t f, uint64_t r, bool check_heaps, bool &err) {
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

template <class Lists = NoLists, class FS>
__device__ __forceinline__ RecSize record_size(const FS &a, uint64_t r, bool check_heaps, bool &err,
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
// and *total = the total (all-ones if any block reported an encoder error).  Tiles of 8 x 1024
// sums: loaded coalesced (all loads in flight) into LDS, each thread scans 8 CONSECUTIVE sums
// serially, one block scan of the thread sums per tile (a block scan costs ~1 us of barriers
// and shuffles on the one CU), results back through LDS, coalesced stores.
__device__ __forceinline__ void scan_block_sums(uint64_t *block_sums, uint64_t nblocks, uint64_t *total) {
    constexpr int PER = 8, TILE = 1024 * PER;
    __shared__ uint64_t tv[TILE + TILE / 16]; // +1 pad per 16: thread-contiguous reads spread banks
    __shared__ uint64_t wsum[16];
    __shared__ int err_s;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    auto at = [](int k) { return k + (k >> 4); };
    if (t == 0) err_s = 0;
    __syncthreads();
    uint64_t carry = 0;
    for (uint64_t tile = 0; tile < nblocks; tile += TILE) {
        uint64_t v[PER];
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint64_t k = tile + (uint64_t)i * 1024 + t;
            v[i] = k < nblocks ? block_sums[k] : 0;
        }
#pragma unroll
        for (int i = 0; i < PER; i++) {
            if (v[i] == ~0ull) {
                err_s = 1;
                v[i] = 0;
            }
            tv[at(i * 1024 + t)] = v[i];
        }
        __syncthreads();
        uint64_t mine[PER], sum = 0;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            mine[i] = tv[at(t * PER + i)];
            sum += mine[i];
        }
        uint64_t x = sum; // inclusive wave scan of the thread sums
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint64_t before = 0, tile_total = 0;
#pragma unroll
        for (int w = 0; w < 16; w++) {
            before += w < wave ? wsum[w] : 0;
            tile_total += wsum[w];
        }
        uint64_t run = before + x - sum;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            tv[at(t * PER + i)] = run;
            run += mine[i];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint64_t k = tile + (uint64_t)i * 1024 + t;
            if (k < nblocks) block_sums[k] = carry + tv[at(i * 1024 + t)];
        }
        carry += tile_total;
        __syncthreads();
    }
    if (t == 0) {
        const uint64_t tot = err_s ? ~0ull : carry;
        block_sums[nblocks] = tot;
        if (total) *total = tot;
    }
}

// Byte sinks.  Positions are in sink coordinates; `lo` is the first byte this lane owns (a
// dword straddling lo is written bytewise so neighbouring records are never clobbered).
struct LdsSink {
    // An emitter that owns a record from its first to its last byte (SpecEnc::emit) may store
    // its first dword whole even when it starts below the record (HEAD_ST4 below): the bytes
    // below belong to the previous lane's record, which writes them later, in its finish().
    static constexpr bool kHeadSt4 = true;
    uint8_t *slab;
    int dummy; // slab-relative dword nobody reads: target of the stores a HEAD_ST4 emitter skips
    __device__ __forceinline__ void st1(int p, uint32_t b) const { slab[p] = (uint8_t)b; }
    __device__ __forceinline__ void st4a(int p, uint32_t w) const { *(uint32_t *)(slab + p) = w; }
    // store w at p if c, else at the dummy dword: one store, no divergent branch
    __device__ __forceinline__ void st4a_if(bool c, int p, uint32_t w) const { st4a(c ? p : dummy, w); }
};

struct GlobalSink {
    static constexpr bool kHeadSt4 = false;
    uint8_t *out;
    __device__ __forceinline__ void st1(long long p, uint32_t b) const { out[p] = (uint8_t)b; }
    __device__ __forceinline__ void st4a(long long p, uint32_t w) const {
        out[p] = (uint8_t)w;
        out[p + 1] = (uint8_t)(w >> 8);
        out[p + 2] = (uint8_t)(w >> 16);
        out[p + 3] = (uint8_t)(w >> 24);
    }
    __device__ __forceinline__ void st4a_if(bool c, long long p, uint32_t w) const {
        if (c) st4a(p, w);
    }
};

// Sequential emitter that merges bytes into dwords (aligned in sink coordinates).
// HEAD_ST4: the dword straddling `lo` is stored whole (no per-byte path, no divergent branch
// per flush) — only for an emitter that writes a whole record in one sequence, in lockstep
// with its neighbours (see LdsSink::kHeadSt4); otherwise bytes below `lo` are never written.
template <class Sink, class Pos, bool HEAD_ST4 = false>
struct Emit {
    static constexpr bool kHeadSt4 = HEAD_ST4;
    const Sink &k;
    Pos pos;   // next byte position
    Pos lo;    // first owned byte
    uint32_t acc; // pending bytes of the dword containing pos (bytes below pos&3)

    __device__ __forceinline__ Emit(const Sink &sink, Pos p) : k(sink), pos(p), lo(p), acc(0) {}

    __device__ __forceinline__ void flush_dword(Pos d, uint32_t w) {
        if (HEAD_ST4 || d >= lo) {
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
        if constexpr (HEAD_ST4) {
            const bool full = (pos & 3) == 0;
            k.st4a_if(full, pos - 4, acc);
            acc = full ? 0u : acc;
        } else if ((pos & 3) == 0) {
            flush_dword(pos - 4, acc);
            acc = 0;
        }
    }
    // 4 bytes in memory order packed little-endian
    __device__ __forceinline__ void put4(uint32_t w) {
        uint32_t k4 = (uint32_t)(pos & 3);
        if constexpr (HEAD_ST4) {
            const uint32_t sh = 8 * k4;
            k.st4a(pos - k4, acc | (w << sh));
            acc = k4 ? (w >> (32 - sh)) : 0u;
        } else if (k4 == 0) {
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
    __device__ __forceinline__ void put_n(uint64_t v, uint32_t nb) {
        const uint32_t ph = (uint32_t)(pos & 3), sh = 8 * ph;
        const uint64_t lo64 = (uint64_t)acc | (v << sh);
        const uint32_t hi32 = sh ? (uint32_t)(v >> (64 - sh)) : 0u;
        const uint32_t total = ph + nb;
        const Pos d = pos & ~(Pos)3;
        if constexpr (HEAD_ST4) {
            k.st4a_if(total >= 4, d, (uint32_t)lo64);
            k.st4a_if(total >= 8, d + 4, (uint32_t)(lo64 >> 32));
        } else {
            if (total >= 4) flush_dword(d, (uint32_t)lo64);
            if (total >= 8) flush_dword(d + 4, (uint32_t)(lo64 >> 32));
        }
        const uint32_t full = total >> 2;
        const uint32_t rest = full == 0 ? (uint32_t)lo64 : (full == 1 ? (uint32_t)(lo64 >> 32) : hi32);
        const uint32_t keep = total & 3;
        acc = keep ? (rest & (0xffffffffu >> (32 - 8 * keep))) : 0u;
        pos += nb;
    }
    // HEAD_ST4 only: n (<= 64) bytes whose first is heap byte `off`, from h[0..19] = the heap
    // dwords starting at off & ~3.  Output dword m of the run (byte d0 + 4m, d0 = pos & ~3) is
    // one funnel shift of two heap dwords, so a 64-byte string costs 17 shifts and 17 dword
    // stores instead of 16 byte-merging appends.
    template <class H>
    __device__ __forceinline__ void put_heap64(const H &h, uint32_t off, uint32_t n) {
        static_assert(HEAD_ST4, "put_heap64: whole-record emitters only");
        const uint32_t ph = (uint32_t)(pos & 3);
        const Pos d0 = pos & ~(Pos)3;
        const uint32_t s = (off & 3) + 4 - ph; // g-byte of output byte d0, g = [0, h0, h1, ...]
        const bool hi = s >= 4;
        const uint32_t b = s & 3;
        const uint32_t total = ph + n, full = total >> 2;
        uint32_t v[17];
#pragma unroll
        for (int m = 0; m < 17; m++) {
            const uint32_t g0 = m == 0 ? 0u : h[m - 1], g1 = h[m], g2 = h[m + 1];
            v[m] = hi ? __builtin_amdgcn_alignbyte(g2, g1, b) : __builtin_amdgcn_alignbyte(g1, g0, b);
        }
        v[0] = (v[0] & (0xffffffffu << (8 * ph))) | acc;
#pragma unroll
        for (int m = 0; m < 17; m++) k.st4a_if((uint32_t)m < full, d0 + 4 * m, v[m]);
        // the pending (partial) dword: v[full], by a select tree on full's bits
        uint32_t t[17];
#pragma unroll
        for (int m = 0; m < 17; m++) t[m] = v[m];
        asm("" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7]),
            "+v"(t[8]), "+v"(t[9]), "+v"(t[10]), "+v"(t[11]), "+v"(t[12]), "+v"(t[13]), "+v"(t[14]), "+v"(t[15]),
            "+v"(t[16]));
        const uint32_t l1[9] = {full & 1 ? t[1] : t[0],   full & 1 ? t[3] : t[2],   full & 1 ? t[5] : t[4],
                                full & 1 ? t[7] : t[6],   full & 1 ? t[9] : t[8],   full & 1 ? t[11] : t[10],
                                full & 1 ? t[13] : t[12], full & 1 ? t[15] : t[14], t[16]};
        const uint32_t l2[5] = {full & 2 ? l1[1] : l1[0], full & 2 ? l1[3] : l1[2], full & 2 ? l1[5] : l1[4],
                                full & 2 ? l1[7] : l1[6], l1[8]};
        const uint32_t l3[3] = {full & 4 ? l2[1] : l2[0], full & 4 ? l2[3] : l2[2], l2[4]};
        const uint32_t l4[2] = {full & 8 ? l3[1] : l3[0], l3[2]};
        const uint32_t last = full & 16 ? l4[1] : l4[0];
        const uint32_t keep = total & 3;
        acc = keep ? (last & (0xffffffffu >> (32 - 8 * keep))) : 0u;
        pos += n;
    }
    // put_heap64 for n <= 4 * (M - 1) bytes (short strings, or a run of bytes built in
    // registers with off = 0): M output dwords from h[0..M].
    template <int M, class H>
    __device__ __forceinline__ void put_heap_short(const H &h, uint32_t off, uint32_t n) {
        static_assert(HEAD_ST4 && M <= 18, "put_heap_short: whole-record emitters, <= 68 bytes");
        const uint32_t ph = (uint32_t)(pos & 3);
        const Pos d0 = pos & ~(Pos)3;
        const uint32_t s = (off & 3) + 4 - ph;
        const bool hi = s >= 4;
        const uint32_t b = s & 3;
        const uint32_t total = ph + n, full = total >> 2;
        uint32_t v[M];
#pragma unroll
        for (int m = 0; m < M; m++) {
            const uint32_t g0 = m == 0 ? 0u : h[m - 1], g1 = h[m], g2 = h[m + 1];
            v[m] = hi ? __builtin_amdgcn_alignbyte(g2, g1, b) : __builtin_amdgcn_alignbyte(g1, g0, b);
        }
        v[0] = (v[0] & (0xffffffffu << (8 * ph))) | acc;
        uint32_t last = v[0];
#pragma unroll
        for (int m = 0; m < M; m++) {
            k.st4a_if((uint32_t)m < full, d0 + 4 * m, v[m]);
            if (m) last = full == (uint32_t)m ? v[m] : last;
        }
        const uint32_t keep = total & 3;
        acc = keep ? (last & (0xffffffffu >> (32 - 8 * keep))) : 0u;
        pos += n;
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
    // [npre bytes of pre] | rvarint(v) | type as ONE append (v < 2^32: the varint is <= 5
    // bytes, so the run is <= 8 bytes with npre <= 1): 32-bit ints, string/bytes lengths.
    __device__ __forceinline__ void varint32_type(uint32_t v, uint32_t type, uint32_t pre = 0, uint32_t npre = 0) {
        const uint32_t L = vlen32(v);
        uint64_t x = v; // 7-bit groups -> bytes
        x = (x & 0x000000000fffffffull) | ((x << 4) & 0x0000000f00000000ull);
        x = (x & 0x00003fff00003fffull) | ((x << 2) & 0x3fff00003fff0000ull);
        x = (x & 0x007f007f007f007full) | ((x << 1) & 0x7f007f007f007f00ull);
        const uint32_t drop = 8 * (8 - L);
        const uint64_t out = (__builtin_bswap64(x) >> drop) | ((0x8080808080808080ull >> drop) & ~0xffull);
        const uint32_t sh = 8 * npre;
        put_n((uint64_t)pre | (out << sh) | ((uint64_t)type << (sh + 8 * L)), npre + L + 1);
    }
    // rvarint(v) | type for any 64-bit v (<= 10 + 1 bytes) without a per-length branch: the 10
    // reversed groups built in 128 bits, the leading (10 - L) bytes shifted out, continuation
    // bits set, the type appended, the run stored as dwords (HEAD_ST4 emitters only).
    __device__ __forceinline__ void varint64_type(uint64_t v, uint32_t type) {
        const uint32_t L = vlen64(v);
        uint64_t x = v & 0x00ffffffffffffffull; // groups 0..7 -> bytes 0..7
        x = (x & 0x000000000fffffffull) | ((x << 4) & 0x0fffffff00000000ull);
        x = (x & 0x00003fff00003fffull) | ((x << 2) & 0x3fff00003fff0000ull);
        x = (x & 0x007f007f007f007full) | ((x << 1) & 0x7f007f007f007f00ull);
        // memory order [g9 g8 g7 ... g0]: lo = first 8 bytes, hi = last 2 (little-endian u128)
        const uint64_t g98 = ((v >> 63) & 1) | (((v >> 56) & 0x7f) << 8);
        const uint64_t rev = __builtin_bswap64(x); // [g7 .. g0]
        uint64_t lo = g98 | (rev << 16), hi = rev >> 48;
        // drop the 10 - L leading bytes (shift right by 8 * (10 - L) in 128 bits)
        const uint32_t d = 8 * (10 - L);
        if (d >= 64) {
            lo = hi >> (d - 64);
            hi = 0;
        } else if (d) {
            lo = (lo >> d) | (hi << (64 - d));
            hi >>= d;
        }
        // continuation bits on bytes 1..L-1, then the type at byte L
        const uint64_t c = 0x8080808080808080ull;
        lo |= L >= 8 ? (c & ~0xffull) : ((c & ((1ull << (8 * L)) - 1)) & ~0xffull);
        hi |= L > 8 ? (c & ((1ull << (8 * (L - 8))) - 1)) : 0ull;
        if (L >= 8) hi |= (uint64_t)type << (8 * (L - 8));
        else lo |= (uint64_t)type << (8 * L);
        const uint32_t w[5] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32), 0u};
        put_heap_short<4>(w, 0u, L + 1);
    }
    // NW payload dwords (memory order) then the type byte, as one run (HEAD_ST4 only)
    template <int NW>
    __device__ __forceinline__ void words_type(const uint32_t (&p)[NW], uint32_t type) {
        uint32_t w[NW + 3];
#pragma unroll
        for (int i = 0; i < NW; i++) w[i] = p[i];
        w[NW] = type;
        w[NW + 1] = w[NW + 2] = 0;
        put_heap_short<NW + 2>(w, 0u, 4 * NW + 1);
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
template <class Sink, class Pos, class Lists = NoListEmit, class FS, class Inv>
__device__ __forceinline__ Pos emit_message(const FS &a, const Sink &k, Pos start, uint64_t r, const RecSize &rs,
                                            const Inv *inv_order, const Lists &lists = Lists()) {
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
            const __amdgpu_buffer_rsrc_t hr = uniform_rsrc(a.heaps[f], a.heap_lens[f]);
            emit_heap(em, hr, a.heap_lens[f], sp.x, sp.y);
            if (kind == K_STRING) em.put1(0);
            em.rvarint(sp.y);
            em.put1(kind == K_STRING ? T_STRING : T_BYTES);
            break;
        }
        }
        end = (uint64_t)(em.pos - start);
        // table entry for this field at its sorted position (encode/msg.go:58-72)
        Pos p = tstart + (Pos)((uint32_t)inv_order[f] * esize);
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

// ---- kernel bodies shared by the precompiled and the schema-specialised encoders -------
//
// A record policy P supplies
//   P::Rec                         the record's column values, loaded by
//   P::load(a, r)                  (all loads of a lane issued together)
//   P::size(a, rec, r, check, err) RecSize of the record
//   P::emit(a, sink, pos, r, rec, rs, inv_order)   the record's bytes
// RuntimeEnc reads the schema from the kernel arguments (one switch per field);
// SpecEnc<Spec> has it as compile-time constants (jit.cpp).

struct RuntimeEnc {
    struct Rec {};
    template <class FS>
    static __device__ __forceinline__ Rec load(const FS &, uint64_t) { return Rec{}; }
    template <class FS>
    static __device__ __forceinline__ void load_cols(const FS &, uint64_t, Rec &) {}
    template <class FS>
    static __device__ __forceinline__ void load_heaps(const FS &, Rec &) {}
    template <class Lists = NoLists, class FS>
    static __device__ __forceinline__ RecSize size(const FS &f, const Rec &, uint64_t r, bool check, bool &err,
                                                   const Lists &lists = Lists()) {
        return record_size(f, r, check, err, lists);
    }
    template <class Sink, class Pos, class Lists = NoListEmit, class FS, class Inv>
    static __device__ __forceinline__ void emit(const FS &f, const Sink &k, Pos p, uint64_t r, const Rec &,
                                                const RecSize &rs, const Inv *inv_order,
                                                const Lists &lists = Lists()) {
        emit_message(f, k, p, r, rs, inv_order, lists);
    }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t heap_rsrc(const EncFields &f, int i) {
    return uniform_rsrc(f.heaps[i], f.heap_lens[i]);
}

// Spec: N (1..), kind[N], tag[N] in write order, order[N] (table order, as EncFields.order),
// big_forced (some tag > 255).  Every per-field step is instantiated per field index
// (template recursion), so the record lives in registers.
template <class Spec>
struct SpecEnc {
    static constexpr int N = Spec::N;
    static constexpr bool kBigForced = Spec::big_forced;
    static constexpr bool has_list() {
        for (int f = 0; f < N; f++)
            if (Spec::kind[f] == K_LIST) return true;
        return false;
    }
    static constexpr bool kHasList = has_list();
    template <int F>
    static constexpr bool heap_kind() { return Spec::kind[F] == K_STRING || Spec::kind[F] == K_BYTES; }
    struct Rec {
        uint64_t v[N][4]; // raw column bits (string/bytes: off | len << 32)
        uint32_t h[N][20]; // string/bytes: first 80 heap bytes from off & ~3
        uint32_t end[N];  // emit: end offset of each field
    };

    template <int F, int E = N>
    static __device__ __forceinline__ void load_col(const EncFields &f, uint64_t r, Rec &x) {
        if constexpr (F < E) {
            const void *col = f.cols[F];
            constexpr uint32_t k = Spec::kind[F];
            if constexpr (k == K_LIST) {
                // no column: written from the item columns by the nested encoder's list hook
            } else if constexpr (k == K_BOOL || k == K_BYTE) {
                x.v[F][0] = ((const uint8_t *)col)[r];
            } else if constexpr (k == K_INT16 || k == K_UINT16) {
                x.v[F][0] = ((const uint16_t *)col)[r];
            } else if constexpr (k == K_INT32 || k == K_UINT32 || k == K_FLOAT32) {
                x.v[F][0] = ((const uint32_t *)col)[r];
            } else if constexpr (k == K_BIN128) {
                const ulonglong2 q = ((const ulonglong2 *)col)[r];
                x.v[F][0] = q.x;
                x.v[F][1] = q.y;
            } else if constexpr (k == K_BIN256) {
                const ulonglong2 *c = (const ulonglong2 *)col + 2 * r;
                const ulonglong2 q0 = c[0], q1 = c[1];
                x.v[F][0] = q0.x;
                x.v[F][1] = q0.y;
                x.v[F][2] = q1.x;
                x.v[F][3] = q1.y;
            } else { // 64-bit kinds, string/bytes spans
                x.v[F][0] = ((const uint64_t *)col)[r];
            }
            load_col<F + 1, E>(f, r, x);
        }
    }

    template <int F, int E = N>
    static __device__ __forceinline__ void load_heap(const EncFields &f, Rec &x) {
        if constexpr (F < E) {
            if constexpr (heap_kind<F>()) {
                const __amdgpu_buffer_rsrc_t hr = heap_rsrc(f, F);
                const uint32_t off = (uint32_t)x.v[F][0] & ~3u;
                // the first 32 bytes always (short strings need no more), the rest only
                // for lanes whose string runs past them
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const uint4 w = heap_ld128(hr, off + 16 * q, f.heap_lens[F]);
                    x.h[F][4 * q] = w.x;
                    x.h[F][4 * q + 1] = w.y;
                    x.h[F][4 * q + 2] = w.z;
                    x.h[F][4 * q + 3] = w.w;
                }
#pragma unroll
                for (int q = 8; q < 20; q++) x.h[F][q] = 0;
                if (((uint32_t)x.v[F][0] & 3u) + (uint32_t)(x.v[F][0] >> 32) > 32) {
#pragma unroll
                    for (int q = 2; q < 5; q++) {
                        const uint4 w = heap_ld128(hr, off + 16 * q, f.heap_lens[F]);
                        x.h[F][4 * q] = w.x;
                        x.h[F][4 * q + 1] = w.y;
                        x.h[F][4 * q + 2] = w.z;
                        x.h[F][4 * q + 3] = w.w;
                    }
                }
            }
            load_heap<F + 1, E>(f, x);
        }
    }

    // every column load of the record, then the heap loads they address, all in flight at once
    static __device__ __forceinline__ Rec load(const EncFields &f, uint64_t r) {
        Rec x;
        load_col<0>(f, r, x);
        load_heap<0>(f, x);
        return x;
    }
    // the two halves of load(), for pipelines that issue them an iteration apart
    static __device__ __forceinline__ void load_cols(const EncFields &f, uint64_t r, Rec &x) { load_col<0>(f, r, x); }
    static __device__ __forceinline__ void load_heaps(const EncFields &f, Rec &x) { load_heap<0>(f, x); }

    template <int F, class Lists, int E = N>
    static __device__ __forceinline__ uint64_t data_size(const EncFields &f, const Rec &x, uint64_t r, bool check,
                                                         bool &err, const Lists &lists) {
        if constexpr (F >= E) {
            return 0;
        } else {
            const uint64_t v = x.v[F][0];
            constexpr uint32_t k = Spec::kind[F];
            uint64_t s;
            if constexpr (k == K_LIST) s = lists((uint32_t)F, r);
            else if constexpr (k == K_BOOL) s = 1;
            else if constexpr (k == K_BYTE) s = 2;
            else if constexpr (k == K_INT16) s = vlen32(zigzag32((int16_t)v)) + 1;
            else if constexpr (k == K_INT32) s = vlen32(zigzag32((int32_t)v)) + 1;
            else if constexpr (k == K_INT64) s = vlen64(zigzag64((int64_t)v)) + 1;
            else if constexpr (k == K_UINT16 || k == K_UINT32 || k == K_UINT64) s = vlen64(v) + 1;
            else if constexpr (k == K_FLOAT32) s = 5;
            else if constexpr (k == K_FLOAT64 || k == K_BIN64) s = 9;
            else if constexpr (k == K_BIN128) s = 17;
            else if constexpr (k == K_BIN256) s = 33;
            else {
                const uint32_t off = (uint32_t)v, len = (uint32_t)(v >> 32);
                err |= ((uint64_t)len > MAX_SIZE) | (check & ((uint64_t)off + len > f.heap_lens[F]));
                s = (uint64_t)len + vlen32(len) + 1 + (k == K_STRING ? 1 : 0);
            }
            return s + data_size<F + 1, Lists, E>(f, x, r, check, err, lists);
        }
    }

    template <class Lists = NoLists>
    static __device__ __forceinline__ RecSize size(const EncFields &f, const Rec &x, uint64_t r, bool check,
                                                   bool &err, const Lists &lists = Lists()) {
        const uint64_t data = data_size<0>(f, x, r, check, err, lists);
        const bool big = Spec::big_forced | (data > 65535); // IsBigMessage, internal/format/msg.go:43-61
        const uint64_t tsize = (uint64_t)N * (big ? 6 : 3);
        err |= data > MAX_SIZE;
        RecSize s;
        s.data = data;
        s.big = big;
        s.total = data + tsize + vlen32((uint32_t)data) + vlen32((uint32_t)tsize) + 1;
        return s;
    }

    template <int F, class E, class Lists, int FE = N>
    static __device__ __forceinline__ void emit_values(const EncFields &f, E &em, Rec &x, decltype(em.pos) start,
                                                       uint64_t r, const Lists &lists) {
        if constexpr (F < FE) {
            const uint64_t v = x.v[F][0];
            constexpr uint32_t k = Spec::kind[F];
            if constexpr (k == K_LIST) {
                lists(em, (uint32_t)F, r);
            } else if constexpr (k == K_BOOL) {
                em.put1(v ? T_TRUE : T_FALSE);
            } else if constexpr (k == K_BYTE) {
                em.put_n(v | (T_BYTE << 8), 2);
            } else if constexpr (k == K_INT16) {
                em.varint32_type(zigzag32((int16_t)v), T_INT16);
            } else if constexpr (k == K_INT32) {
                em.varint32_type(zigzag32((int32_t)v), T_INT32);
            } else if constexpr (k == K_INT64 || k == K_UINT64) {
                const uint64_t u = k == K_INT64 ? zigzag64((int64_t)v) : v;
                const uint32_t ty = k == K_INT64 ? T_INT64 : T_UINT64;
                if constexpr (E::kHeadSt4) {
                    em.varint64_type(u, ty);
                } else {
                    em.rvarint(u);
                    em.put1(ty);
                }
            } else if constexpr (k == K_UINT16 || k == K_UINT32) {
                em.varint32_type((uint32_t)v, k == K_UINT16 ? T_UINT16 : T_UINT32);
            } else if constexpr (k == K_FLOAT32) {
                em.put_n(bswap32((uint32_t)v) | ((uint64_t)T_FLOAT32 << 32), 5);
            } else if constexpr (E::kHeadSt4 && (k == K_FLOAT64 || k == K_BIN64 || k == K_BIN128 || k == K_BIN256)) {
                // fixed-width payload + type as one run of dwords
                if constexpr (k == K_FLOAT64) {
                    const uint32_t p[2] = {bswap32((uint32_t)(v >> 32)), bswap32((uint32_t)v)};
                    em.words_type(p, T_FLOAT64);
                } else if constexpr (k == K_BIN64) {
                    const uint32_t p[2] = {(uint32_t)v, (uint32_t)(v >> 32)};
                    em.words_type(p, T_BIN64);
                } else if constexpr (k == K_BIN128) {
                    const uint32_t p[4] = {(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)x.v[F][1],
                                           (uint32_t)(x.v[F][1] >> 32)};
                    em.words_type(p, T_BIN128);
                } else {
                    uint32_t p[8];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        p[2 * q] = (uint32_t)x.v[F][q];
                        p[2 * q + 1] = (uint32_t)(x.v[F][q] >> 32);
                    }
                    em.words_type(p, T_BIN256);
                }
            } else if constexpr (k == K_FLOAT64) {
                em.put4(bswap32((uint32_t)(v >> 32)));
                em.put4(bswap32((uint32_t)v));
                em.put1(T_FLOAT64);
            } else if constexpr (k == K_BIN64) {
                em.put8(v);
                em.put1(T_BIN64);
            } else if constexpr (k == K_BIN128) {
                em.put8(v);
                em.put8(x.v[F][1]);
                em.put1(T_BIN128);
            } else if constexpr (k == K_BIN256) {
                em.put8(v);
                em.put8(x.v[F][1]);
                em.put8(x.v[F][2]);
                em.put8(x.v[F][3]);
                em.put1(T_BIN256);
            } else { // string/bytes: the prefetched 64 bytes, then the rest from the heap
                const uint32_t off = (uint32_t)v, len = (uint32_t)(v >> 32), sh = off & 3;
                const uint32_t n = len < 64 ? len : 64;
                if constexpr (E::kHeadSt4) {
                    if (__ballot(n > 16) == 0) em.template put_heap_short<5>(x.h[F], off, n); // wave-uniform
                    else em.put_heap64(x.h[F], off, n);
                } else {
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        const uint32_t w = __builtin_amdgcn_alignbyte(x.h[F][j + 1], x.h[F][j], sh);
                        if ((uint32_t)(4 * j + 4) <= n) {
                            em.put4(w);
                        } else if ((uint32_t)(4 * j) < n) {
                            em.put_n(w, n - 4 * j);
                        }
                    }
                }
                if (len > 64) emit_heap(em, heap_rsrc(f, F), f.heap_lens[F], off + 64, len - 64);
                // [NUL] | rvarint(len) | type in one append
                if constexpr (k == K_STRING) em.varint32_type(len, T_STRING, 0u, 1u);
                else em.varint32_type(len, T_BYTES);
            }
            x.end[F] = (uint32_t)(em.pos - start);
            emit_values<F + 1, E, Lists, FE>(f, em, x, start, r, lists);
        }
    }

    // table (internal/encode/msg.go:58-72): small {u8 tag, u16 end}, big {u16 tag, u32 end}
    template <int J, class E>
    static __device__ __forceinline__ void emit_table(E &em, const Rec &x, bool big) {
        if constexpr (J < N) {
            constexpr int f = Spec::order[J];
            constexpr uint32_t tag = Spec::tag[f];
            const uint32_t e = x.end[f];
            const uint64_t small = (tag & 0xff) | ((uint64_t)(__builtin_bswap16((uint16_t)e)) << 8);
            const uint64_t bigv = (uint64_t)__builtin_bswap16((uint16_t)tag) | ((uint64_t)bswap32(e) << 16);
            em.put_n(big ? bigv : small, big ? 6 : 3);
            emit_table<J + 1>(em, x, big);
        }
    }

    // The record as one sequential byte run: values in write order, the table entries in
    // table order (their ends kept in registers), the trailer.
    // Small table + trailer as ONE run of bytes built in registers (every entry's byte position
    // is a compile-time constant), appended with one phase-shifted store per dword:
    //   table {u8 tag, u16 BE end} x N | rvarint(dataSize) (<= 3 bytes: data <= 65535) |
    //   rvarint(3N) (1 byte: 3N < 128) | TypeMessage          (internal/encode/msg.go:27-77)
    static constexpr int TB = 3 * N;
    static constexpr int RUN_M = (TB + 5 + 3) / 4 + 1; // output dwords covering the run at any phase
    template <class E>
    static __device__ __forceinline__ void emit_small_table_trailer(E &em, const Rec &x, uint32_t data) {
        uint32_t w[RUN_M + 1];
#pragma unroll
        for (int i = 0; i <= RUN_M; i++) w[i] = 0;
#pragma unroll
        for (int j = 0; j < N; j++) {
            const int f = Spec::order[j];
            const uint32_t ent = Spec::tag[f] | ((uint32_t)__builtin_bswap16((uint16_t)x.end[f]) << 8);
            const int b = 3 * j, d = b >> 2, s = 8 * (b & 3);
            w[d] |= ent << s;
            if (s > 8) w[d + 1] |= ent >> (32 - s);
        }
        // trailer bytes: the reverse varint of data (top group first, continuation bits on all
        // but the first), then 3N, then the type
        const uint32_t L = vlen32(data);
        uint64_t v = data & 0x1fffff; // 3 groups of 7 bits -> bytes (inverse of rvarint_bf)
        v = (v & 0x7f) | ((v & 0x3f80) << 1) | ((v & 0x1fc000) << 2);
        const uint64_t be = (__builtin_bswap32((uint32_t)v) >> 8) >> (8 * (3 - L)); // byte i = group L-1-i
        const uint64_t cont = (0x808080ull >> (8 * (3 - L))) & ~0xffull;
        const uint64_t T = (be | cont) | ((uint64_t)TB << (8 * L)) | ((uint64_t)T_MESSAGE << (8 * (L + 1)));
        {
            constexpr int d = TB >> 2, s = 8 * (TB & 3);
            w[d] |= (uint32_t)(T << s);
            w[d + 1] |= (uint32_t)((T << s) >> 32);
        }
        em.template put_heap_short<RUN_M>(w, 0u, (uint32_t)TB + L + 2);
    }

    // ---- the write pass on a wave pair (encode_write_pair_body): wave 0 emits fields [0, H),
    // wave 1 fields [H, N), the table and the trailer ----
    // x.end[F..E) = base + the field sizes through each field: the ends the emitter records,
    // known from the sizes before any byte is written
    template <int F, int E>
    static __device__ __forceinline__ uint32_t range_ends(const EncFields &f, Rec &x, uint64_t r, uint32_t base) {
        if constexpr (F < E) {
            bool err = false;
            const uint32_t s = (uint32_t)data_size<F, NoLists, F + 1>(f, x, r, false, err, NoLists());
            x.end[F] = base + s;
            return range_ends<F + 1, E>(f, x, r, base + s);
        } else {
            return base;
        }
    }
    // the values of fields [F0, F1) from em.pos (no finish: the pending dword stays in em.acc)
    template <int F0, int F1, class E, class Lists = NoListEmit>
    static __device__ __forceinline__ void emit_range(const EncFields &f, E &em, Rec &x, decltype(em.pos) start,
                                                      uint64_t r, const Lists &lists = Lists()) {
        emit_values<F0, E, Lists, F1>(f, em, x, start, r, lists);
    }
    // the K_LIST field's index (-1: none)
    static constexpr int list_field() {
        for (int f = 0; f < N; f++)
            if (Spec::kind[f] == K_LIST) return f;
        return -1;
    }
    // the table and trailer after the values (x.end[] of every field set; no finish)
    template <class E>
    static __device__ __forceinline__ void emit_table_trailer(E &em, const Rec &x, const RecSize &rs) {
        if constexpr (E::kHeadSt4 && !Spec::big_forced && RUN_M <= 18) {
            if (__ballot(rs.big) == 0) {
                emit_small_table_trailer(em, x, (uint32_t)rs.data);
                return;
            }
        }
        emit_table<0>(em, x, rs.big);
        em.rvarint((uint32_t)rs.data);
        em.rvarint((uint32_t)(N * (rs.big ? 6 : 3)));
        em.put1(rs.big ? T_BIG_MESSAGE : T_MESSAGE);
    }

    // With a list field the emitter jumps over the list's items (written later by other lanes:
    // encode_nested_core.hpp phase B).  HEAD_ST4 stays valid: the first store after the jump may
    // clobber <= 3 bytes of the last item, which phase B then writes.
    template <class Sink, class Pos, class Lists = NoListEmit>
    static __device__ __forceinline__ void emit(const EncFields &f, const Sink &k, Pos start, uint64_t r,
                                                const Rec &rec, const RecSize &rs, const uint8_t *,
                                                const Lists &lists = Lists()) {
        Rec x = rec;
        Emit<Sink, Pos, Sink::kHeadSt4> em(k, start);
        emit_values<0>(f, em, x, start, r, lists);
        if constexpr (Sink::kHeadSt4 && !Spec::big_forced && RUN_M <= 18) {
            if (__ballot(rs.big) == 0) { // wave-uniform: every record of the wave has a small table
                emit_small_table_trailer(em, x, (uint32_t)rs.data);
                em.finish();
                return;
            }
        }
        emit_table<0>(em, x, rs.big);
        // trailer: rvarint(dataSize) | rvarint(tableSize) | type (internal/encode/msg.go:36-39)
        em.rvarint((uint32_t)rs.data);
        em.rvarint((uint32_t)(N * (rs.big ? 6 : 3)));
        em.put1(rs.big ? T_BIG_MESSAGE : T_MESSAGE);
        em.finish();
    }
};

// Pass 1: per-block encoded bytes (all-ones on an encoder error).
template <class P, class A>
__device__ __forceinline__ void encode_size_body(const A &a) {
    __shared__ uint64_t part[ENC_BLOCK / 64];
    __shared__ int errs;
    if (threadIdx.x == 0) errs = 0;
    __syncthreads();
    const uint64_t r = (uint64_t)blockIdx.x * ENC_BLOCK + threadIdx.x;
    const bool valid = r < a.n;
    typename P::Rec rec; // sizes need the columns only (string/bytes: their spans), not heap bytes
    P::load_cols(a.f, valid ? r : a.n - 1, rec);
    bool err = false;
    const RecSize rs = P::size(a.f, rec, r, a.check_heaps, err);
    if (valid & err) errs = 1;
    uint64_t s = valid ? rs.total : 0;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < ENC_BLOCK / 64; w++) t += part[w];
        a.block_sums[blockIdx.x] = errs ? ~0ull : t;
    }
}

// Copy slab [head, lim) -> gbase[head, lim) (gbase 16-B aligned), one 16-B store per lane.
__device__ __forceinline__ void copy_slab_out(const uint8_t *slab, uint8_t *gbase, uint64_t head, uint64_t lim,
                                              int lane) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const v4u lds_v4;
    typedef __attribute__((address_space(3))) const uint8_t lds_b;
    lds_v4 *s4 = (lds_v4 *)(lds_b *)slab; // ds_read_b128 (a generic pointer would be a flat load)
    lds_b *sb = (lds_b *)slab;
    v4u *g4 = (v4u *)gbase;
    // the whole 16-byte chunks [h16, l16): four per lane per round, every LDS read before the stores
    const uint64_t h16 = (head + 15) >> 4, l16 = lim >> 4;
    for (uint64_t q = h16 + lane; q < l16; q += 256) {
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t qq = q + 64 * u;
            v[u] = s4[qq < l16 ? qq : q]; // q < l16: in range
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (q + 64 * u < l16) g4[q + 64 * u] = v[u];
    }
    // the partial chunks at either end, a byte per lane
    const uint64_t hend = (h16 << 4) < lim ? (h16 << 4) : lim;
    const uint64_t tb = (l16 << 4) > hend ? (l16 << 4) : hend;
    if (lane < 16 && head + lane < hend) gbase[head + lane] = sb[head + lane];
    if (lane >= 16 && lane < 32 && tb + (lane - 16) < lim) gbase[tb + (lane - 16)] = sb[tb + (lane - 16)];
}

// Pass 3: block scan of the recomputed sizes -> record offsets; each lane emits its record
// into the wave's LDS slab, the wave copies the slab to HBM with 16-byte stores; ends[]
// written coalesced.  A wave whose output span does not fit the slab emits straight to HBM.
// smem: ENC_LDS_HEAD bytes of header, then ENC_BLOCK / 64 slabs of ENC_SLAB bytes.
template <class P, class A>
__device__ __forceinline__ void encode_write_body(const A &a, uint8_t *smem) {
    uint64_t *wsum = (uint64_t *)smem;
    // the table position of every field: built in LDS from the Writer's order, or (a wide
    // schema) precomputed in device memory
    uint8_t *inv_lds = smem + 8 * (ENC_BLOCK / 64);
    const auto *inv_order = [&] {
        if constexpr (A::kWide) return a.f.inv_order;
        else return (const uint8_t *)inv_lds;
    }();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t r = (uint64_t)blockIdx.x * ENC_BLOCK + threadIdx.x;
    const bool valid = r < a.n;
    // the record's loads, the total and this block's offset all in flight together (the check
    // that nothing is written after an error or a capacity overflow waits for the total only now)
    const typename P::Rec rec = P::load(a.f, valid ? r : a.n - 1);
    const uint64_t total = a.block_sums[a.nblocks], blk_pre = a.block_sums[blockIdx.x];
    if (total > a.out_cap) return; // capacity error or encoder error (total == ~0)
    if constexpr (!A::kWide)
        if (threadIdx.x < a.f.nfields) inv_lds[a.f.order[threadIdx.x]] = (uint8_t)threadIdx.x;
    bool err = false;
    RecSize rs = P::size(a.f, rec, r, false, err);
    if (!valid) rs.total = 0;
    uint64_t x = rs.total; // block exclusive scan of sizes
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    lds_barrier(); // (heap loads still in flight)
    uint64_t pre = blk_pre;
    for (int w = 0; w < wave; w++) pre += wsum[w];
    const uint64_t start = pre + x - rs.total;
    if (valid) a.ends[r] = a.ends_base + start + rs.total;

    // wave output span [S, E)
    const uint64_t wbase = (uint64_t)blockIdx.x * ENC_BLOCK + wave * 64;
    if (wbase >= a.n) return;
    const uint64_t S = __builtin_amdgcn_readfirstlane((uint32_t)start) |
                       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(start >> 32)) << 32);
    const int last = (int)((a.n - wbase) < 64 ? a.n - wbase - 1 : 63);
    const uint64_t Ev = __shfl(start + rs.total, last);
    const uint64_t E = __builtin_amdgcn_readfirstlane((uint32_t)Ev) |
                       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(Ev >> 32)) << 32);
    const uint64_t head = ((uint64_t)(a.out + S)) & 15; // slab pos of byte S keeps 16-B phase
    if (head + (E - S) + 16 <= (uint64_t)ENC_SLAB) {
        uint8_t *slab = smem + ENC_LDS_HEAD + wave * ENC_SLAB;
        LdsSink k{slab, (int)(smem + ENC_LDS_HEAD - 4 - slab)}; // dummy: last header dword (unused)
        if (valid) P::emit(a.f, k, (int)(head + (start - S)), r, rec, rs, inv_order);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        copy_slab_out(slab, a.out + S - head, head, head + (E - S), lane);
    } else if (valid) {
        GlobalSink k{a.out};
        P::emit(a.f, k, (long long)start, r, rec, rs, inv_order);
    }
}

constexpr size_t enc_write_lds_bytes() { return ENC_LDS_HEAD + (size_t)(ENC_BLOCK / 64) * ENC_SLAB; }

// ---- the write pass on wave PAIRS (schema-specialised encoders) ---------------------------
// A 512-thread block takes the size pass's 256-record block as four groups of 64 records; each
// group is written by a wave PAIR sharing one LDS slab: wave 0 emits fields [0, H) of the 64
// records, wave 1 fields [H, N) from each record's position of field H, then the table and the
// trailer (the ends of fields [0, H) come from wave 0 through LDS, known from the sizes before
// any byte is written).  Twice the waves per slab: one wave's LDS stores and heap loads overlap
// the other's emission (the decoder's wave pairs, decode_flat_pair, are the same lever).
// Ordering: a HEAD_ST4 emitter's first dword store covers <= 3 bytes below its start (the bytes
// of the previous lane's record, or of wave 0's half of the same record), and every emitter
// keeps its last partial dword pending; all whole-dword stores of both waves happen before a
// block barrier and every pending tail is stored bytewise after it, so each byte's last writer
// is its owner.
// LDS: wsum[4] | per group: d0 (u32 x 64) | wave 0's field ends (u16 x H x 64) | slab.
constexpr int ENC_PAIR_BLOCK = 512;
constexpr int ENC_PAIR_HEAD = 64;
__host__ __device__ constexpr uint32_t enc_pair_xch_bytes(int h) { return (uint32_t)(256 + 128 * h + 15) & ~15u; }
// the slab of one group: four groups' slabs and exchanges in <= 80 KiB (two blocks per CU)
__host__ __device__ constexpr uint32_t enc_pair_slab_bytes(int h) {
    return ((81920u - ENC_PAIR_HEAD) / 4 - enc_pair_xch_bytes(h)) & ~15u;
}
__host__ __device__ constexpr uint32_t enc_pair_lds_bytes(int h) {
    return ENC_PAIR_HEAD + 4 * (enc_pair_xch_bytes(h) + enc_pair_slab_bytes(h));
}

// copy_slab_out by T threads (one 16-byte store per thread and chunk)
template <int T>
__device__ __forceinline__ void copy_slab_out_t(const uint8_t *slab, uint8_t *gbase, uint64_t head, uint64_t lim,
                                                int tid) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const v4u lds_v4;
    typedef __attribute__((address_space(3))) const uint8_t lds_b;
    lds_v4 *s4 = (lds_v4 *)(lds_b *)slab;
    lds_b *sb = (lds_b *)slab;
    v4u *g4 = (v4u *)gbase;
    const uint64_t h16 = (head + 15) >> 4, l16 = lim >> 4;
    for (uint64_t q = h16 + tid; q < l16; q += 4 * T) {
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t qq = q + T * u;
            v[u] = s4[qq < l16 ? qq : q];
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (q + T * u < l16) g4[q + T * u] = v[u];
    }
    const uint64_t hend = (h16 << 4) < lim ? (h16 << 4) : lim;
    const uint64_t tb = (l16 << 4) > hend ? (l16 << 4) : hend;
    if (tid < 16 && head + tid < hend) gbase[head + tid] = sb[head + tid];
    if (tid >= 16 && tid < 32 && tb + (tid - 16) < lim) gbase[tb + (tid - 16)] = sb[tb + (tid - 16)];
}

template <class P, int H>
__device__ __forceinline__ void encode_write_pair_body(const EncodeArgs &a, uint8_t *smem) {
    static_assert(H >= 1 && H < P::N, "the split leaves fields on both waves");
    constexpr uint32_t XB = enc_pair_xch_bytes(H), SB = enc_pair_slab_bytes(H);
    uint64_t *wsum = (uint64_t *)smem;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, grp = wave >> 1, half = wave & 1;
    uint8_t *gx = smem + ENC_PAIR_HEAD + grp * (XB + SB);
    uint32_t *xd0 = (uint32_t *)gx;                   // wave 0's data bytes per record
    uint16_t *xend = (uint16_t *)(gx + 256);          // wave 0's field ends [field][lane]
    uint8_t *slab = gx + XB;
    const uint64_t r = (uint64_t)blockIdx.x * ENC_BLOCK + grp * 64 + lane;
    const bool valid = r < a.n;
    const uint64_t rr = valid ? r : a.n - 1;
    typename P::Rec x;
    if (half == 0) {
        P::template load_col<0, H>(a.f, rr, x);
        P::template load_heap<0, H>(a.f, x);
    } else {
        P::template load_col<H, P::N>(a.f, rr, x);
        P::template load_heap<H, P::N>(a.f, x);
    }
    const uint64_t total = a.block_sums[a.nblocks], blk_pre = a.block_sums[blockIdx.x];
    if (total > a.out_cap) return; // capacity error or encoder error (total == ~0): block-uniform
    bool err = false;
    uint32_t dmine;
    if (half == 0) {
        dmine = P::template range_ends<0, H>(a.f, x, rr, 0u);
        xd0[lane] = dmine;
#pragma unroll
        for (int f = 0; f < H; f++) xend[f * 64 + lane] = (uint16_t)x.end[f];
    } else {
        dmine = (uint32_t)P::template data_size<H, NoLists, P::N>(a.f, x, rr, false, err, NoLists());
    }
    __syncthreads(); // (1) wave 0's sizes and ends are in LDS
    const uint32_t d0 = half == 0 ? dmine : xd0[lane];
    const uint64_t data = (uint64_t)d0 + (half == 0 ? 0u : dmine);
    uint64_t tot = 0, data_all = data;
    RecSize rs;
    if (half == 1) {
        rs.data = data_all;
        rs.big = P::kBigForced | (data_all > 65535);
        const uint64_t tsize = (uint64_t)P::N * (rs.big ? 6 : 3);
        rs.total = data_all + tsize + vlen32((uint32_t)data_all) + vlen32((uint32_t)tsize) + 1;
        tot = valid ? rs.total : 0;
    }
    // wave 1 owns the record sizes: its scan gives the group's offsets; wave 0 reads its starts
    uint64_t xs = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(xs, o);
        if (lane >= o) xs += y;
    }
    uint64_t *xstart = (uint64_t *)slab; // (the slab is free until the emission starts)
    if (half == 1) {
        if (lane == 63) wsum[grp] = xs;
        xstart[lane] = xs - tot; // group-relative start of the record
    }
    __syncthreads(); // (2) group sums and starts
    uint64_t pre = blk_pre;
    for (int g = 0; g < grp; g++) pre += wsum[g];
    const uint64_t start = pre + xstart[lane];
    const uint64_t gtot = wsum[grp];
    if (half == 1 && valid) a.ends[r] = a.ends_base + start + rs.total;
    const uint64_t gbase_r = (uint64_t)blockIdx.x * ENC_BLOCK + grp * 64;
    const bool live = gbase_r < a.n; // group-uniform
    const uint64_t S = pre, E = pre + gtot;
    const uint64_t head = ((uint64_t)(a.out + S)) & 15;
    const bool fits = live && head + (E - S) + 16 <= (uint64_t)SB;
    __syncthreads(); // (3) xstart read: the slab may be written
    if (!live) return;
    if (!fits) {
        // a group larger than its slab: wave 0 writes each record straight to HBM (every field)
        if (half == 0 && valid) {
            const typename P::Rec all = P::load(a.f, r);
            RecSize rs0 = P::size(a.f, all, r, false, err);
            GlobalSink k{a.out};
            P::emit(a.f, k, (long long)start, r, all, rs0, (const uint8_t *)nullptr);
        }
        return;
    }
    LdsSink k{slab, (int)(smem + ENC_PAIR_HEAD - 4 - slab)}; // dummy: the last header dword
    const int p0 = (int)(head + (start - S));
    Emit<LdsSink, int, true> em(k, half == 0 ? p0 : p0 + (int)d0);
    if (valid) {
        if (half == 0) {
            P::template emit_range<0, H>(a.f, em, x, p0, r);
        } else {
#pragma unroll
            for (int f = 0; f < H; f++) x.end[f] = xend[f * 64 + lane];
            P::template emit_range<H, P::N>(a.f, em, x, p0, r);
            P::emit_table_trailer(em, x, rs);
        }
    }
    __syncthreads(); // (4) every whole-dword store of the group is done
    if (valid) em.finish(); // the pending tails, bytewise: the owners write last
    __syncthreads(); // (5) the slab is complete
    copy_slab_out_t<128>(slab, a.out + S - head, head, head + (E - S), threadIdx.x & 127);
}

} // namespace spec
