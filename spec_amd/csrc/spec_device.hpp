// spec_device.hpp — device-side primitives of the MI355X spec engine (gfx950 / CDNA4).
//
// Wire format (reference: basecomplextech/spec, internal/format/type.go:13-52,
// internal/decode/...): every value ENDS with a 1-byte type tag and is parsed backwards from
// its end.  This header holds the pieces both kernels share:
//   * byte sources: LdsSrc (a wave's staged byte span in LDS) and GlobalSrc (bounds-checked
//     buffer loads straight from HBM, used when a wave's span does not fit its LDS slab);
//   * tail windows: the 16 bytes that end at a value's end, fetched with 3 aligned 8-byte
//     reads and funnel-shifted into two big-endian u64 views — this one fetch yields the
//     type byte, any fixed-width payload up to 8 bytes and the reverse varint;
//   * the reverse varint (compactint reconstruction, see oracle/compactint.c) decoded
//     branch-free from that window;
//   * IEEE f32<->f64 conversions done in integer arithmetic so Go's float32(float64(x))
//     semantics (NaN quieting, round-to-nearest-even, subnormals) hold bit for bit
//     independently of the GPU's FP mode registers.
#pragma once

#ifdef __HIPCC_RTC__
// compiled at run time by hiprtc (schema-specialised kernels, jit.cpp): no system headers
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint64_t uint64_t;
typedef __hip_internal::int16_t int16_t;
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::int64_t int64_t;
#define INT32_MIN (-2147483647 - 1)
#define INT32_MAX 2147483647
#else
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

// Fields of one kernel-side field set (decode_core.hpp FieldSet, encode_core.hpp EncFields): a
// schema with more fields (include/spec_amd.h SPEC_MAX_FIELDS) is decoded in chunks of this many
// fields and encoded by the wide kernels, whose field set lives in device memory.
#define SPEC_KFIELDS 64

namespace spec {

// ---- type codes, internal/format/type.go:20-52
enum : uint32_t {
    T_TRUE = 1, T_FALSE = 2, T_BYTE = 3,
    T_INT16 = 10, T_INT32 = 11, T_INT64 = 12,
    T_UINT16 = 20, T_UINT32 = 21, T_UINT64 = 22,
    T_BIN64 = 30, T_BIN128 = 31, T_BIN256 = 32,
    T_FLOAT32 = 40, T_FLOAT64 = 41,
    T_BYTES = 50, T_STRING = 60,
    T_LIST = 70, T_BIG_LIST = 71,
    T_MESSAGE = 80, T_BIG_MESSAGE = 81,
    T_STRUCT = 90,
};

// ---- column kinds (include/spec_amd.h)
enum : uint32_t {
    K_BOOL = 1, K_BYTE, K_INT16, K_INT32, K_INT64, K_UINT16, K_UINT32, K_UINT64,
    K_FLOAT32, K_FLOAT64, K_BIN64, K_BIN128, K_BIN256, K_STRING, K_BYTES,
    K_LIST, // list<message> field of a nested schema (spec_decode_nested); no flat column
};

// ---- record status (include/spec_amd.h spec_status)
enum : uint32_t {
    ST_OK = 0, ST_INVALID_TYPE = 1, ST_INVALID_TABLE_SIZE = 2, ST_INVALID_DATA_SIZE = 3,
    ST_INVALID_TABLE = 4, ST_INVALID_DATA = 5, ST_PANIC = 6, ST_INVALID_VALUE = 7, ST_TOO_DEEP = 8,
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Big-endian u64 from 8 little-endian-packed bytes held in (lo = bytes 0..3, hi = 4..7).
__device__ __forceinline__ uint64_t be64_of(uint32_t lo, uint32_t hi) {
    return ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
}

// ---- byte sources ------------------------------------------------------------------------
// Positions are signed so lower-bound checks (reads below a message start) are plain
// compares.  `d64(p)` returns the 8 bytes at an 8-aligned position p (little-endian packed).

typedef __attribute__((address_space(3))) const uint8_t lds_u8;
typedef __attribute__((address_space(3))) const uint32_t lds_u32;
typedef __attribute__((address_space(3))) const uint64_t lds_u64;

struct LdsSrc {
    using pos_t = int;
    lds_u8 *lds; // slab base inside the dynamic LDS array (explicit LDS address space)
    __device__ __forceinline__ uint32_t u8(int p) const { return lds[p]; }
    // Each qword is its own ds_read_b64: the address goes through an empty asm so the
    // backend cannot pair neighbouring reads into ds_read2_b64, which on CDNA4 costs 8 LDS
    // cycles with (a/4) mod 32 banking against 2 x 2 cycles, (a/4) mod 64, for two b64 reads
    // (MI355X_MICROARCH.md, LDS table).  The record windows are read at random lane
    // addresses, so the wider banking also halves the conflicts.
    __device__ __forceinline__ uint64_t d64(int p) const {
        asm("" : "+v"(p));
        return *(lds_u64 *)(lds + p);
    }
    __device__ __forceinline__ uint32_t d32(int p) const { return *(lds_u32 *)(lds + p); }
};

// A workgroup barrier that orders LDS only: the waves' global loads stay in flight across it
// (__syncthreads' fence also covers global memory, so it waits for every outstanding load).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// A buffer load that straddles num_records returns 0 for the WHOLE access (not just the
// bytes past the end), so the last partial word of a buffer is read bytewise.
__device__ __forceinline__ uint32_t buf_ld32(__amdgpu_buffer_rsrc_t r, uint32_t off, uint64_t len) {
    if ((uint64_t)off + 4 <= len) return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    uint32_t w = 0;
    for (int i = 0; i < 4; i++) w |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, off + i, 0, 0) << (8 * i);
    return w;
}

// A range-checked buffer descriptor over [p, p + len) (len clamped to 4 GiB - 1), built from
// readfirstlane'd scalars: the callers' p / len are wave-uniform, but a value that went through
// memory or a call is not KNOWN to be, and every buffer load through a descriptor in VGPRs
// becomes a waterfall loop (readfirstlane x 4, compare, loop).  Free when they sit in SGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void *p, uint64_t len) {
    const uint64_t b = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(len > 0xffffffffull ? 0xffffffffu : (uint32_t)len);
    return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0, (int)n, 0x00020000);
}

struct GlobalSrc {
    using pos_t = long long;
    const uint8_t *base; // range-checked: reads outside [0, len) return 0
    uint64_t len;
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const { return uniform_rsrc(base, len); }
    __device__ __forceinline__ uint32_t u8(long long p) const {
        return __builtin_amdgcn_raw_buffer_load_b8(rsrc(), (uint32_t)p, 0, 0);
    }
    __device__ __forceinline__ uint64_t d64(long long p) const {
        // p may be negative near the stream start: wrap to a huge offset => range check => 0
        if (p >= 0 && (uint64_t)p + 8 > len) {
            uint64_t v = 0;
            for (int i = 0; i < 8; i++) v |= (uint64_t)u8(p + i) << (8 * i);
            return v;
        }
        auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc(), (uint32_t)p, 0, 0);
        return (uint64_t)v[0] | ((uint64_t)v[1] << 32);
    }
    __device__ __forceinline__ uint32_t d32(long long p) const {
        if (p >= 0) return buf_ld32(rsrc(), (uint32_t)p, len);
        return 0;
    }
};

// 8 bytes starting at arbitrary position p, little-endian packed (byte p in bits 0..7).
template <class Src>
__device__ __forceinline__ uint64_t load_le64(const Src &s, typename Src::pos_t p) {
    typename Src::pos_t a = p & ~(typename Src::pos_t)7;
    uint32_t sh = (uint32_t)(p - a); // 0..7
    uint64_t x = s.d64(a), y = s.d64(a + 8);
    uint32_t w0 = (uint32_t)x, w1 = (uint32_t)(x >> 32), w2 = (uint32_t)y, w3 = (uint32_t)(y >> 32);
    // select dword pair by sh>>2, then funnel-shift by sh&3 bytes
    bool hi = sh >= 4;
    uint32_t a0 = hi ? w1 : w0, a1 = hi ? w2 : w1, a2 = hi ? w3 : w2;
    uint32_t b = sh & 3;
    uint32_t lo32 = __builtin_amdgcn_alignbyte(a1, a0, b);
    uint32_t hi32 = __builtin_amdgcn_alignbyte(a2, a1, b);
    return ((uint64_t)hi32 << 32) | lo32;
}

// The 16 bytes [e-16, e) as two big-endian views: q0 = BE64([e-8, e)), q1 = BE64([e-16, e-8)).
// q0 & 0xff is the type byte at e-1.
struct Tail {
    uint64_t q0, q1;
};

template <class Src>
__device__ __forceinline__ Tail load_tail(const Src &s, typename Src::pos_t e) {
    typename Src::pos_t p = e - 16;
    typename Src::pos_t a = p & ~(typename Src::pos_t)7;
    uint32_t sh = (uint32_t)(p - a);
    uint64_t x = s.d64(a), y = s.d64(a + 8), z = s.d64(a + 16);
    uint32_t w0 = (uint32_t)x, w1 = (uint32_t)(x >> 32), w2 = (uint32_t)y, w3 = (uint32_t)(y >> 32);
    uint32_t w4 = (uint32_t)z, w5 = (uint32_t)(z >> 32);
    bool hi = sh >= 4;
    uint32_t a0 = hi ? w1 : w0, a1 = hi ? w2 : w1, a2 = hi ? w3 : w2, a3 = hi ? w4 : w3;
    uint32_t a4 = hi ? w5 : w4;
    uint32_t b = sh & 3;
    uint32_t l0 = __builtin_amdgcn_alignbyte(a1, a0, b); // bytes e-16..e-13
    uint32_t l1 = __builtin_amdgcn_alignbyte(a2, a1, b); // e-12..e-9
    uint32_t l2 = __builtin_amdgcn_alignbyte(a3, a2, b); // e-8..e-5
    uint32_t l3 = __builtin_amdgcn_alignbyte(a4, a3, b); // e-4..e-1
    Tail t;
    t.q0 = be64_of(l2, l3);
    t.q1 = be64_of(l0, l1);
    return t;
}

// Reverse varint ending at the type byte: R = BE64([e-9, e-1)) puts the byte adjacent to the
// type byte (the least-significant 7-bit group) in bits 0..7; R2 holds bytes e-10 (bits 0..7)
// and e-11 (bits 8..15).
__device__ __forceinline__ uint64_t tail_r(const Tail &t) { return (t.q0 >> 8) | (t.q1 << 56); }
__device__ __forceinline__ uint32_t tail_r2(const Tail &t) { return (uint32_t)(t.q1 >> 8) & 0xffff; }

// Reverse varint decode (oracle/compactint.c so_reverse_uint{32,64}): r/r2 hold the candidate
// bytes in read order, avail = bytes available before the lower bound.  Returns the value and
// sets n = bytes consumed (>0) or a negative error (incomplete / overflow).
template <int MAXLEN>
__device__ __forceinline__ uint64_t rvarint(uint64_t r, uint32_t r2, long long avail, int &n) {
    // terminator: first byte (from index 0) with MSB clear
    uint64_t t = ~r & 0x8080808080808080ull;
    int ta;
    if (t) {
        ta = (int)(__builtin_ctzll(t) >> 3);
    } else {
        uint32_t t2 = ~r2 & 0x8080u;
        ta = t2 ? 8 + (int)(__builtin_ctz(t2) >> 3) : 10;
    }
    long long lim = avail < MAXLEN ? avail : MAXLEN;
    if ((long long)ta >= lim) {
        n = -(int)(lim + 1);
        return 0;
    }
    // keep bytes 0..ta
    uint64_t w = r & 0x7f7f7f7f7f7f7f7full;
    if (ta < 7) w &= (~0ull) >> (56 - 8 * ta);
    // compact 7-bit groups: 8x7 -> 56 bits
    w = (w & 0x007f007f007f007full) | ((w & 0x7f007f007f007f00ull) >> 1);
    w = (w & 0x00003fff00003fffull) | ((w & 0x3fff00003fff0000ull) >> 2);
    w = (w & 0x000000000fffffffull) | ((w & 0x0fffffff00000000ull) >> 4);
    uint32_t last;
    if (ta >= 8) {
        uint32_t b8 = r2 & 0x7f;
        w |= (uint64_t)b8 << 56;
        if (ta == 9) w |= (uint64_t)((r2 >> 8) & 0x7f) << 63;
        last = (r2 >> (8 * (ta - 8))) & 0xff;
    } else {
        last = (uint32_t)(r >> (8 * ta)) & 0xff;
    }
    if (ta == MAXLEN - 1 && last > (MAXLEN == 10 ? 1u : 0x0fu)) {
        n = -(ta + 1);
        return 0;
    }
    n = ta + 1;
    return w;
}

// Branch-free form of rvarint (same results) with a run-time MaxLen (5 or 10): every
// intermediate is computed eagerly and combined with selects, so a specialised kernel's
// fields stay straight-line code the compiler can interleave.
__device__ __forceinline__ uint32_t ctz_or(uint32_t x, uint32_t none) { return __builtin_ctzg(x, (int)none); }

__device__ __forceinline__ uint64_t rvarint_bf(uint64_t r, uint32_t r2, long long avail, int maxlen, int &n) {
    const uint64_t t = ~r & 0x8080808080808080ull;
    const uint32_t t2 = ~r2 & 0x8080u;
    // index of the first byte with MSB clear: bit index / 8, 10 if none among the 10 bytes
    const uint32_t b0 = ctz_or((uint32_t)t, 96u);
    const uint32_t b1 = ctz_or((uint32_t)(t >> 32), 64u) + 32u;
    const uint32_t b2 = ctz_or(t2, 16u) + 64u;
    const int ta = (int)(__builtin_elementwise_min(__builtin_elementwise_min(b0, b1), b2) >> 3);
    const long long lim = avail < maxlen ? avail : (long long)maxlen;
    const bool incomplete = (long long)ta >= lim;
    const uint64_t keep = ~0ull >> (56 - 8 * (ta < 7 ? ta : 7)); // bytes 0..ta (all 8 when ta >= 7)
    uint64_t w = r & 0x7f7f7f7f7f7f7f7full & keep;
    w = (w & 0x007f007f007f007full) | ((w & 0x7f007f007f007f00ull) >> 1);
    w = (w & 0x00003fff00003fffull) | ((w & 0x3fff00003fff0000ull) >> 2);
    w = (w & 0x000000000fffffffull) | ((w & 0x0fffffff00000000ull) >> 4);
    const uint64_t h8 = (uint64_t)(r2 & 0x7f) << 56;
    const uint64_t h9 = (uint64_t)((r2 >> 8) & 0x7f) << 63;
    w |= (ta >= 8 ? h8 : 0ull) | (ta == 9 ? h9 : 0ull);
    const uint32_t lo_last = (uint32_t)(r >> (8 * (ta & 7))) & 0xff;
    const uint32_t hi_last = (r2 >> (8 * ((ta - 8) & 1))) & 0xff;
    const uint32_t last = ta >= 8 ? hi_last : lo_last;
    const uint32_t cap = maxlen == 10 ? 1u : 0x0fu;
    const bool over = (ta == maxlen - 1) & (last > cap);
    const int n_inc = -(int)(lim + 1), n_over = -(ta + 1), n_ok = ta + 1;
    n = incomplete ? n_inc : (over ? n_over : n_ok);
    return (incomplete | over) ? 0ull : w;
}

__device__ __forceinline__ int64_t unzigzag64(uint64_t u) { return (int64_t)(u >> 1) ^ -(int64_t)(u & 1); }
__device__ __forceinline__ int32_t unzigzag32(uint32_t u) { return (int32_t)(u >> 1) ^ -(int32_t)(u & 1); }

// ---- IEEE conversions in integer arithmetic ------------------------------------------------

// float64(float32): exact widening, a NaN is quieted (x86 CVTSS2SD, Go on amd64).
__device__ __forceinline__ uint64_t f32_to_f64_bits(uint32_t f) {
    uint64_t s = (uint64_t)(f >> 31) << 63;
    uint32_t e = (f >> 23) & 0xff, m = f & 0x7fffff;
    if (e == 0xff) {
        if (m) return s | 0x7ff8000000000000ull | ((uint64_t)m << 29);
        return s | 0x7ff0000000000000ull;
    }
    if (e == 0) {
        if (m == 0) return s;
        int p = 31 - __builtin_clz(m); // highest set bit, 0..22
        uint64_t E = (uint64_t)(p - 149 + 1023);
        uint64_t M = ((uint64_t)m << (52 - p)) & 0xfffffffffffffull;
        return s | (E << 52) | M;
    }
    return s | ((uint64_t)(e - 127 + 1023) << 52) | ((uint64_t)m << 29);
}

// float32(float64) for a NaN or a finite value within +-MaxFloat32 (callers range-check):
// round to nearest even, subnormal results kept, NaN payload truncated and quieted.
__device__ __forceinline__ uint32_t f64_to_f32_bits(uint64_t d) {
    uint32_t s = (uint32_t)(d >> 63) << 31;
    int E = (int)((d >> 52) & 0x7ff);
    uint64_t M = d & 0xfffffffffffffull;
    if (E == 0x7ff) return s | 0x7fc00000u | (uint32_t)(M >> 29); // NaN (Inf excluded by caller)
    if (E == 0) return s;                                           // |d| < 2^-1022 -> +-0
    int e = E - 1023;
    uint64_t sig = M | (1ull << 52);
    int r; // right shift that leaves the f32 mantissa field
    uint32_t base;
    if (e >= -126) {
        r = 29;
        base = (uint32_t)(e + 127) << 23;
        sig = M; // implicit bit carried by the exponent field
    } else {
        r = 29 + (-126 - e);
        base = 0;
        if (r >= 64) return s;
    }
    uint64_t q = sig >> r;
    uint64_t rem = sig & ((1ull << r) - 1);
    uint64_t half = 1ull << (r - 1);
    if (rem > half || (rem == half && (q & 1))) q += 1;
    return s | (base + (uint32_t)q); // mantissa carry rolls into the exponent correctly
}

// Branch-free forms of the two conversions above (same bits).
__device__ __forceinline__ uint64_t f32_to_f64_bits_bf(uint32_t f) {
    const uint64_t sgn = (uint64_t)(f >> 31) << 63;
    const uint32_t e = (f >> 23) & 0xff, m = f & 0x7fffff;
    const uint64_t norm = sgn | ((uint64_t)(e + 896) << 52) | ((uint64_t)m << 29);
    const uint64_t qnan = 0x0008000000000000ull | ((uint64_t)m << 29);
    const uint64_t infnan = sgn | 0x7ff0000000000000ull | (m != 0 ? qnan : 0ull);
    const int p = 31 - (int)__builtin_clz(m | 1u);
    const uint64_t sub = sgn | ((uint64_t)(p + 874) << 52) | (((uint64_t)m << (52 - p)) & 0xfffffffffffffull);
    const uint64_t zs = m != 0 ? sub : sgn;
    return e == 0xff ? infnan : (e == 0 ? zs : norm);
}

__device__ __forceinline__ uint32_t f64_to_f32_bits_bf(uint64_t d) {
    const uint32_t sgn = (uint32_t)(d >> 63) << 31;
    const int E = (int)((d >> 52) & 0x7ff);
    const uint64_t M = d & 0xfffffffffffffull;
    const int e = E - 1023;
    const bool normal = e >= -126;
    const int rr = normal ? 29 : 29 + (-126 - e);
    const bool tiny = rr >= 64;
    const int r = tiny ? 63 : rr;
    const uint64_t sig = normal ? M : (M | (1ull << 52));
    const uint32_t base = normal ? (uint32_t)(e + 127) << 23 : 0u;
    uint64_t q = sig >> r;
    const uint64_t rem = sig & ((1ull << r) - 1);
    const uint64_t half = 1ull << (r - 1);
    q += ((rem > half) | ((rem == half) & ((q & 1) != 0))) ? 1 : 0;
    const uint32_t fin = tiny ? sgn : sgn | (base + (uint32_t)q);
    const uint32_t nanr = sgn | 0x7fc00000u | (uint32_t)(M >> 29);
    return E == 0x7ff ? nanr : (E == 0 ? sgn : fin);
}

// ---- tiny helpers ------------------------------------------------------------------------

__device__ __forceinline__ int lane_id() { return __lane_id(); }

} // namespace spec
