// decode_core.hpp — device code of the flat-message decoder (gfx950), shared by the
// precompiled generic kernel (decode_flat.hip) and the schema-specialised kernels that
// jit.cpp compiles at run time with hiprtc.
//
// Replaces, per record, spec.OpenMessageErr (internal/types/msg.go:43-55 ->
// internal/decode/msg.go:14-99) followed by one typed getter per schema field
// (internal/types/msg.go:219-475: m.field(tag) = table.Offset(tag) binary search
// (internal/format/msg.go:227-265) + decode.Decode<Kind>(bytes[:end])).
//
// Mapping (MI355X, wave64):
//   * one wave = 64 consecutive records, one record per lane;
//   * the wave's contiguous byte span [ends[base-1], ends[base+63]) is staged into the wave's
//     private LDS slab with LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per instruction,
//     range-checked by the buffer descriptor) — one fully coalesced HBM read of the stream;
//   * each lane parses its record from LDS.  Two code paths:
//       - the FAST path (schema known at compile time: `Spec` = a generated struct) reads the
//         whole field table with a few wide LDS reads, checks that it holds exactly the
//         schema's tags in the order a Writer emits them (then the reference's binary search
//         provably lands on the same entries), and decodes every field with straight-line,
//         kind-specialised code the compiler can interleave (ILP across fields);
//       - the GENERIC path (any table, any record) restates the reference step by step:
//         trailer, sortedness check, probe at the expected index or exact binary search,
//         per-kind decode selected at run time.  Records the fast path rejects go here,
//         so results never depend on which path ran;
//   * column writes are lane-strided => coalesced per field;
//   * a wave whose span exceeds its slab parses straight from HBM via range-checked buffer
//     loads (GlobalSrc, generic path) — correctness never depends on record sizes.
#pragma once

#include "spec_device.hpp"

namespace spec {


// The fields a record decode produces: one column per schema field + the status column.
struct FieldSet {
    uint8_t *status;
    uint64_t *errmask; // optional: bit f = field f's <Kind>Err getter errs
    uint32_t nfields;
    uint16_t tags[SPEC_KFIELDS];
    uint8_t kinds[SPEC_KFIELDS];
    uint16_t rank[SPEC_KFIELDS]; // index of the field's tag in the sorted table a writer emits
    void *cols[SPEC_KFIELDS];
};

// Passed by value as the kernel argument (lives in the kernarg segment => scalar loads,
// the per-field loop branches are wave-uniform).
struct DecodeArgs {
    const uint8_t *stream;
    uint64_t stream_len;
    const uint64_t *ends;
    uint64_t n;  // records [r0, n) of the batch are decoded (columns indexed by record)
    uint64_t r0;
    uint32_t head; // bytes before each record (mpx frame head = 4: [u32 BE size][message])
    uint32_t slab; // LDS bytes per wave (0: every wave parses from HBM)
    uint32_t xcd;  // 1: XCD-aware block order (consecutive groups on one XCD's L2)
    FieldSet f;
};

// spec_decode_nested (decode_nested.hip): outer records with one list<message> field.
struct NestedArgs {
    const uint8_t *stream;
    uint64_t stream_len;
    const uint64_t *ends;
    uint64_t n;
    FieldSet outer; // the outer message; its K_LIST field is decoded into item_begin
    FieldSet item;  // the list items
    uint32_t list_tag, list_rank;
    uint32_t *item_begin; // [n + 1]
    uint64_t item_cap;    // item columns hold this many items
    uint64_t *group_base; // workspace: per 64-record group item total, then exclusive offsets
    uint64_t *total;      // device: total items
    uint32_t slab;        // LDS bytes per wave
    uint32_t xcd;         // decode pass: 1 = XCD-aware block order (grid a multiple of 8)
};

constexpr int DEC_WAVES = 4; // waves per block of the nested kernels
constexpr int SLAB_GUARD = 48; // >= the deepest read below a value end (bin256: 33 + 7)

// LDS slab per wave: guard + the 1 KiB DMA chunks a 64-record span needs + pad.  Sized at
// launch from the batch's mean record size with a margin (4 % for flat records; 16 % for
// nested ones, whose item counts vary: on config 4, 4 % left 17.8 % of the groups over the
// slab, 16 % leaves 0.05 %); a wave whose span does not fit is staged in halves or parses
// from HBM, so the margin only affects speed.
constexpr int SLAB_MAX_CHUNKS = 40;
__host__ __device__ inline uint32_t decode_slab_bytes(double avg_record, double margin = 1.04) {
    const double span = avg_record * 64 * margin;
    int chunks = (int)(span / 1024.0) + 1;
    if (chunks > SLAB_MAX_CHUNKS) return 0;
    return (uint32_t)(SLAB_GUARD + chunks * 1024 + 32);
}
// The nested kernels run DEC_WAVES waves per block, each with its slab plus (RANGES mode) a 1 KiB
// item-range window: the block's LDS must stay within gfx950's 160 KiB, so a slab over
// NESTED_SLAB_MAX is not used (0: the groups parse from HBM).
constexpr uint32_t NESTED_SLAB_MAX = 163840 / DEC_WAVES - 1024;
__host__ __device__ inline uint32_t nested_slab_bytes(double avg_record) {
    const uint32_t s = decode_slab_bytes(avg_record, 1.16);
    return s <= NESTED_SLAB_MAX ? s : 0u;
}

// ---- message table lookup --------------------------------------------------------------

// exact reference binary search (offset_small/offset_big), returns end offset or -1
template <class Src>
__device__ __noinline__ long long table_search(const Src s, typename Src::pos_t tstart, uint32_t nent,
                                               bool big, uint32_t tag) {
    int left = 0, right = (int)nent - 1;
    while (left <= right) {
        int mid = (int)((unsigned)(left + right) >> 1);
        uint32_t cur;
        typename Src::pos_t p;
        if (big) {
            p = tstart + (typename Src::pos_t)mid * 6;
            cur = (s.u8(p) << 8) | s.u8(p + 1);
        } else {
            p = tstart + (typename Src::pos_t)mid * 3;
            cur = s.u8(p);
        }
        if (cur < tag) {
            left = mid + 1;
        } else if (cur > tag) {
            right = mid - 1;
        } else {
            if (big)
                return ((long long)s.u8(p + 2) << 24) | (s.u8(p + 3) << 16) | (s.u8(p + 4) << 8) | s.u8(p + 5);
            return (s.u8(p + 1) << 8) | s.u8(p + 2);
        }
    }
    return -1;
}

// ---- value decoders: field slice [lo, e), type at e-1 (internal/decode/...) ------------

struct Val {
    uint64_t v0, v1, v2, v3; // up to 32 bytes of column payload, little-endian
};

// Decode the value ending at e (field slice [lo, e), flen = e - lo; flen <= 0 => zero value)
// from its 16-byte tail window t; bin128/bin256 read their leading bytes from s.
// Straight-line code (selects, no branches): every byte it reads lies within 40 bytes below
// e, which callers keep inside the source even for an empty field.
// The bytes a value's decode reads: its 16-byte tail window, plus for bin128/bin256 the
// leading payload qwords.
struct Win {
    Tail t;
    uint64_t x0, x1, x2;
};

// Kinds whose value, once its type is the one the Writer emits (cross_kind_type), ends in at
// most 8 bytes: type byte + <= 5-byte reverse varint (32-bit ints, string/bytes lengths),
// 4-byte float32, byte, bool.  The fast path reads an 8-byte window for them (2 LDS reads,
// not 3); bytes below the window read as 0, which a <= 5-byte varint never looks at.
template <uint32_t KIND>
__host__ __device__ constexpr bool narrow_kind() {
    return KIND == K_BOOL || KIND == K_BYTE || KIND == K_INT16 || KIND == K_INT32 || KIND == K_UINT16 ||
           KIND == K_UINT32 || KIND == K_FLOAT32 || KIND == K_STRING || KIND == K_BYTES;
}

// Fixed-width payloads (bin64/128/256, float64): NQ payload qwords [e-1-8NQ, e-1) and the
// type byte at e-1, from the NQ+1 aligned qwords that cover them (a 16-byte tail window plus
// separate payload reads would take 3 / 5 / 9 reads for 8 / 16 / 32 bytes; this takes 2 / 3 / 5).
// Packed as a Win: x0.. = leading payload qwords (little-endian), t = the tail view decode_tail_k
// reads (type byte + the last 8 payload bytes, big-endian).
template <int NQ, class Src>
__device__ __forceinline__ Win load_fixed(const Src &s, typename Src::pos_t e) {
    using pos_t = typename Src::pos_t;
    const pos_t p = e - 1 - 8 * NQ;
    const pos_t base = p & ~(pos_t)7;
    const uint32_t sh = 8u * (uint32_t)(p - base);
    uint64_t q[NQ + 1], c[NQ];
#pragma unroll
    for (int j = 0; j <= NQ; j++) q[j] = s.d64(base + 8 * j);
#pragma unroll
    for (int j = 0; j < NQ; j++) c[j] = (q[j] >> sh) | ((q[j + 1] << 1) << (63 - sh));
    const uint32_t type = (uint32_t)(q[NQ] >> sh) & 0xff;
    const uint64_t B = __builtin_bswap64(c[NQ - 1]);
    Win w;
    w.t.q0 = (B << 8) | type;
    w.t.q1 = B >> 56;
    w.x0 = NQ > 1 ? c[0] : 0;
    w.x1 = NQ > 2 ? c[1 % NQ] : 0;
    w.x2 = NQ > 3 ? c[2 % NQ] : 0;
    return w;
}

template <uint32_t KIND, bool NARROW = false, class Src>
__device__ __forceinline__ Win load_win(const Src &s, typename Src::pos_t e) {
    Win w;
    if constexpr (NARROW && narrow_kind<KIND>()) {
        w.t.q0 = __builtin_bswap64(load_le64(s, e - 8)); // BE64([e-8, e))
        w.t.q1 = 0;
        w.x0 = w.x1 = w.x2 = 0;
        return w;
    } else if constexpr (NARROW && (KIND == K_FLOAT64 || KIND == K_BIN64)) {
        return load_fixed<1>(s, e);
    } else if constexpr (NARROW && KIND == K_BIN128) {
        return load_fixed<2>(s, e);
    } else if constexpr (NARROW && KIND == K_BIN256) {
        return load_fixed<4>(s, e);
    }
    w.t = load_tail(s, e);
    w.x0 = w.x1 = w.x2 = 0;
    if constexpr (KIND == K_BIN128) {
        w.x0 = load_le64(s, e - 17);
    } else if constexpr (KIND == K_BIN256) {
        w.x0 = load_le64(s, e - 33);
        w.x1 = load_le64(s, e - 25);
        w.x2 = load_le64(s, e - 17);
    }
    return w;
}

// The type a Writer emits for a column kind, for the kinds whose getter also accepts other
// types (ints of other widths, float32 <-> float64); 0 for kinds that accept one type only.
__host__ __device__ constexpr uint32_t cross_kind_type(uint32_t k) {
    return k == K_INT16 ? T_INT16 : k == K_INT32 ? T_INT32 : k == K_INT64 ? T_INT64
         : k == K_UINT16 ? T_UINT16 : k == K_UINT32 ? T_UINT32 : k == K_UINT64 ? T_UINT64
         : k == K_FLOAT32 ? T_FLOAT32 : k == K_FLOAT64 ? T_FLOAT64 : 0u;
}

// NAT = true: the caller has checked that the value's type byte is cross_kind_type(KIND) (or
// the field is empty), so the cross-width branches fold away; results are those of NAT = false
// for such values.
// okp (optional): set to false when the decoder returns an error (the getter's *Err variant,
// internal/types/msg.go:233-459); a non-empty field only (callers handle flen <= 0).
template <uint32_t KIND, bool NAT = false, class Pos>
__device__ __forceinline__ Val decode_tail_k(const Win &w, Pos lo, Pos e, long long to_stream, bool *okp = nullptr) {
    const Tail &t = w.t;
    Val out = {0, 0, 0, 0};
    bool okv = true;
    const long long flen = (long long)(e - lo);
    constexpr uint32_t NT = cross_kind_type(KIND);
    const uint32_t type = (NAT && NT) ? NT : (uint32_t)t.q0 & 0xff;
    const uint64_t R = tail_r(t);
    const uint32_t R2 = tail_r2(t);
    const long long avail = flen - 1; // bytes before the type byte
    int m;
    if constexpr (KIND == K_BOOL) { // DecodeBool, byte.go:38-51: true iff type == TypeTrue
        out.v0 = ((flen > 0) & (type == T_TRUE)) ? 1 : 0;
    } else if constexpr (KIND == K_BYTE) { // DecodeByte, byte.go:16-34
        okv = (type == T_BYTE) & (flen >= 2);
        out.v0 = okv ? (R & 0xff) : 0;
    } else if constexpr (KIND == K_INT16 | KIND == K_INT32 | KIND == K_INT64) {
        // DecodeInt16/32/64, int.go:16-135: 32-bit routine for Int16/Int32, 64-bit for Int64
        const bool w32 = (type == T_INT16) | (type == T_INT32);
        const uint64_t u = rvarint_bf(R, R2, avail, w32 ? 5 : 10, m);
        const long long x = w32 ? (long long)unzigzag32((uint32_t)u) : (long long)unzigzag64(u);
        bool ok = (flen > 0) & (w32 | (type == T_INT64)) & (m >= 0);
        if (KIND == K_INT16) ok = ok & (x >= -32768) & (x <= 32767);
        if (KIND == K_INT32) ok = ok & (w32 | ((x >= INT32_MIN) & (x <= INT32_MAX)));
        okv = ok;
        out.v0 = ok ? (uint64_t)x : 0;
        if (KIND == K_INT16) out.v0 &= 0xffff;
        if (KIND == K_INT32) out.v0 &= 0xffffffffu;
    } else if constexpr (KIND == K_UINT16 | KIND == K_UINT32 | KIND == K_UINT64) {
        // DecodeUint16/32/64, uint.go:16-125
        const bool w32 = (type == T_UINT16) | (type == T_UINT32);
        const uint64_t x = rvarint_bf(R, R2, avail, w32 ? 5 : 10, m);
        bool ok = (flen > 0) & (w32 | (type == T_UINT64)) & (m >= 0);
        if (KIND == K_UINT16) ok = ok & (x <= 0xffffull);
        if (KIND == K_UINT32) ok = ok & (x <= 0xffffffffull);
        okv = ok;
        out.v0 = ok ? x : 0;
    } else if constexpr (KIND == K_FLOAT32) { // DecodeFloat32, float.go:15-32 (via float64 + range check)
        uint32_t b = (uint32_t)(R & 0xffffffffu);
        const uint32_t ex = (b >> 23) & 0xff;
        const bool inf = (ex == 0xff) & ((b & 0x7fffff) == 0); // +-Inf fails the +-MaxFloat32 check
        b = ex == 0xff ? (b | 0x00400000u) : b;             // NaN: quieted by the float64 round trip
        const uint64_t d = R;
        const uint32_t dx = (uint32_t)(d >> 52) & 0x7ff;
        const bool nan = (dx == 0x7ff) & ((d & 0xfffffffffffffull) != 0);
        // |d| > MaxFloat32 (0x47EFFFFFE0000000) => overflow error => 0
        const bool over = !nan & ((d & 0x7fffffffffffffffull) > 0x47EFFFFFE0000000ull);
        const uint32_t from64 = f64_to_f32_bits_bf(d);
        const bool ok32 = (type == T_FLOAT32) & (flen >= 5) & !inf, ok64 = (type == T_FLOAT64) & (flen >= 9) & !over;
        okv = ok32 | ok64;
        out.v0 = ok32 ? b : (ok64 ? from64 : 0u);
    } else if constexpr (KIND == K_FLOAT64) { // DecodeFloat64, float.go:34-78
        const uint64_t from32 = f32_to_f64_bits_bf((uint32_t)(R & 0xffffffffu));
        const bool ok32 = (type == T_FLOAT32) & (flen >= 5), ok64 = (type == T_FLOAT64) & (flen >= 9);
        okv = ok32 | ok64;
        out.v0 = ok32 ? from32 : (ok64 ? R : 0ull);
    } else if constexpr (KIND == K_BIN64) { // DecodeBin64, bin.go:15-44: raw 8 bytes before the type byte
        okv = (type == T_BIN64) & (flen >= 9);
        out.v0 = okv ? __builtin_bswap64(R) : 0;
    } else if constexpr (KIND == K_BIN128) {
        const bool ok = (type == T_BIN128) & (flen >= 17);
        okv = ok;
        out.v0 = ok ? w.x0 : 0;
        out.v1 = ok ? __builtin_bswap64(R) : 0;
    } else if constexpr (KIND == K_BIN256) {
        const bool ok = (type == T_BIN256) & (flen >= 33);
        okv = ok;
        out.v0 = ok ? w.x0 : 0;
        out.v1 = ok ? w.x1 : 0;
        out.v2 = ok ? w.x2 : 0;
        out.v3 = ok ? __builtin_bswap64(R) : 0;
    } else if constexpr (KIND == K_STRING | KIND == K_BYTES) {
        // DecodeString (string.go:15-70) / DecodeBytes (bytes.go:14-58)
        constexpr bool str = KIND == K_STRING;
        const uint32_t len = (uint32_t)rvarint_bf(R, R2, avail, 5, m);
        const long long end = (long long)(e - 1) - m - (str ? 1 : 0); // skip the NUL for strings
        const long long off = end - (long long)len;
        const bool ok = (type == (str ? T_STRING : T_BYTES)) & (flen > 0) & (m >= 0) & (end >= (long long)lo) &
                        (off >= (long long)lo) & (len != 0);
        okv = (type == (str ? T_STRING : T_BYTES)) & (m >= 0) & (end >= (long long)lo) & (off >= (long long)lo);
        out.v0 = ok ? ((uint64_t)(uint32_t)(off + to_stream) | ((uint64_t)len << 32)) : 0;
    }
    if (okp) *okp = okv;
    return out;
}

template <uint32_t KIND, class Src>
__device__ __forceinline__ Val decode_value_k(const Src &s, typename Src::pos_t lo, typename Src::pos_t e,
                                              long long to_stream) {
    if ((long long)(e - lo) <= 0) return Val{0, 0, 0, 0}; // empty => zero value, no error
    return decode_tail_k<KIND>(load_win<KIND>(s, e), lo, e, to_stream);
}

template <class T>
__device__ __forceinline__ void col_store(T *p, T v) {
#if !defined(SPEC_CACHED_STORE)
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

template <uint32_t KIND>
__device__ __forceinline__ void store_value_k(void *colp, uint64_t r, const Val &v) {
    uint8_t *col = (uint8_t *)colp;
#if !defined(SPEC_CACHED_STORE)
    if constexpr (KIND == K_BOOL || KIND == K_BYTE) {
        col_store(col + r, (uint8_t)v.v0);
    } else if constexpr (KIND == K_INT16 || KIND == K_UINT16) {
        col_store((uint16_t *)col + r, (uint16_t)v.v0);
    } else if constexpr (KIND == K_INT32 || KIND == K_UINT32 || KIND == K_FLOAT32) {
        col_store((uint32_t *)col + r, (uint32_t)v.v0);
    } else if constexpr (KIND == K_BIN128) {
        col_store((uint64_t *)col + 2 * r, v.v0);
        col_store((uint64_t *)col + 2 * r + 1, v.v1);
    } else if constexpr (KIND == K_BIN256) {
        col_store((uint64_t *)col + 4 * r, v.v0);
        col_store((uint64_t *)col + 4 * r + 1, v.v1);
        col_store((uint64_t *)col + 4 * r + 2, v.v2);
        col_store((uint64_t *)col + 4 * r + 3, v.v3);
    } else {
        col_store((uint64_t *)col + r, v.v0);
    }
    return;
#endif
    if constexpr (KIND == K_BOOL || KIND == K_BYTE) {
        col[r] = (uint8_t)v.v0;
    } else if constexpr (KIND == K_INT16 || KIND == K_UINT16) {
        ((uint16_t *)col)[r] = (uint16_t)v.v0;
    } else if constexpr (KIND == K_INT32 || KIND == K_UINT32 || KIND == K_FLOAT32) {
        ((uint32_t *)col)[r] = (uint32_t)v.v0;
    } else if constexpr (KIND == K_BIN128) {
        ((ulonglong2 *)col)[r] = make_ulonglong2(v.v0, v.v1);
    } else if constexpr (KIND == K_BIN256) {
        ulonglong2 *c = (ulonglong2 *)col + 2 * r;
        c[0] = make_ulonglong2(v.v0, v.v1);
        c[1] = make_ulonglong2(v.v2, v.v3);
    } else {
        ((uint64_t *)col)[r] = v.v0;
    }
}

// run-time kind dispatch for the generic path (wave-uniform switches around ONE shared
// tail-window load, so the generic kernel stays compact)
// returns false when the field is present and its decoder errs (the *Err getter's error)
template <class Src>
__device__ __forceinline__ bool decode_store(const Src &s, uint32_t kind, typename Src::pos_t lo, long long end,
                                             long long to_stream, void *col, uint64_t r) {
    Val v = {0, 0, 0, 0};
    bool ok = true;
    if (end > 0) {
        const typename Src::pos_t e = lo + (typename Src::pos_t)end;
#define SPEC_CASE(K) \
    case K: v = decode_tail_k<K>(load_win<K>(s, e), lo, e, to_stream, &ok); break;
        switch (kind) {
            SPEC_CASE(K_BOOL)
            SPEC_CASE(K_BYTE)
            SPEC_CASE(K_INT16)
            SPEC_CASE(K_INT32)
            SPEC_CASE(K_INT64)
            SPEC_CASE(K_UINT16)
            SPEC_CASE(K_UINT32)
            SPEC_CASE(K_UINT64)
            SPEC_CASE(K_FLOAT32)
            SPEC_CASE(K_FLOAT64)
            SPEC_CASE(K_BIN64)
            SPEC_CASE(K_BIN128)
            SPEC_CASE(K_BIN256)
            SPEC_CASE(K_STRING)
            SPEC_CASE(K_BYTES)
        }
#undef SPEC_CASE
    }
    uint8_t *c = (uint8_t *)col;
    switch (kind) {
    case K_BOOL:
    case K_BYTE: c[r] = (uint8_t)v.v0; break;
    case K_INT16:
    case K_UINT16: ((uint16_t *)c)[r] = (uint16_t)v.v0; break;
    case K_INT32:
    case K_UINT32:
    case K_FLOAT32: ((uint32_t *)c)[r] = (uint32_t)v.v0; break;
    case K_BIN128: store_value_k<K_BIN128>(col, r, v); break;
    case K_BIN256: store_value_k<K_BIN256>(col, r, v); break;
    default: ((uint64_t *)c)[r] = v.v0; break;
    }
    return ok;
}

// ---- record trailer: DecodeMessageTable, internal/decode/msg.go:14-99 -------------------

struct Trailer {
    uint32_t st;     // spec_status
    bool big;
    long long tstart, dstart; // source positions
    uint32_t dsize, tsize;
};

// LIST = false: DecodeMessageTable (internal/decode/msg.go:14-99), 3/6-byte entries;
// LIST = true: DecodeListTable (internal/decode/list.go:14-98), 2/4-byte entries.
template <bool LIST = false, class Src>
__device__ __forceinline__ Trailer parse_trailer(const Src &s, typename Src::pos_t rs, typename Src::pos_t re) {
    Trailer tr = {ST_OK, false, 0, 0, 0, 0};
    long long len = (long long)(re - rs);
    Tail t = load_tail(s, re);
    uint32_t type = (uint32_t)t.q0 & 0xff;
    const uint32_t T_SMALL = LIST ? T_LIST : T_MESSAGE, T_BIG = LIST ? T_BIG_LIST : T_BIG_MESSAGE;
    const uint32_t ESMALL = LIST ? 2u : 3u, EBIG = LIST ? 4u : 6u;
    if (type != T_SMALL && type != T_BIG) {
        tr.st = ST_INVALID_TYPE;
        return tr;
    }
    tr.big = type == T_BIG;
    uint64_t R = tail_r(t);
    uint32_t R2 = tail_r2(t);
    int m1, m2;
    uint32_t tsz = (uint32_t)rvarint<5>(R, R2, len - 1, m1);
    if (m1 < 0) {
        tr.st = ST_INVALID_TABLE_SIZE;
        return tr;
    }
    // the data-size varint ends m1 bytes further down: shift the window
    uint64_t Rs = (R >> (8 * m1)) | ((uint64_t)R2 << (64 - 8 * m1));
    uint32_t R2s = m1 >= 2 ? 0u : (R2 >> (8 * m1));
    uint32_t dsz = (uint32_t)rvarint<5>(Rs, R2s, len - 1 - m1, m2);
    if (m2 < 0) {
        tr.st = ST_INVALID_DATA_SIZE;
        return tr;
    }
    long long tend = (long long)(re - 1) - m1 - m2;
    long long ts = tend - (long long)tsz;
    if (ts < (long long)rs || tsz % (tr.big ? EBIG : ESMALL) != 0) {
        tr.st = ST_INVALID_TABLE;
        return tr;
    }
    if (ts - (long long)dsz < (long long)rs) {
        tr.st = ST_INVALID_DATA;
        return tr;
    }
    tr.tstart = ts;
    tr.dstart = ts - (long long)dsz;
    tr.dsize = dsz;
    tr.tsize = tsz;
    return tr;
}

// ---- generic path: any record, run-time schema -----------------------------------------

// OpenMessageErr of one record: trailer + whether the table's tags are strictly increasing
// (then a probe at a field's expected index finds what the reference's binary search finds).
struct RecInfo {
    Trailer tr;
    bool ok, sorted;
    uint32_t nent;
};

template <class Src>
__device__ __forceinline__ RecInfo rec_open(const Src &s, typename Src::pos_t rs, typename Src::pos_t re) {
    using pos_t = typename Src::pos_t;
    RecInfo ri;
    ri.tr = Trailer{ST_OK, false, 0, 0, 0, 0};
    ri.ok = false;
    ri.sorted = true;
    ri.nent = 0;
    if (re > rs) {
        ri.tr = parse_trailer(s, rs, re);
        ri.ok = ri.tr.st == ST_OK;
        ri.nent = ri.tr.tsize / (ri.tr.big ? 6u : 3u);
    }
    if (ri.ok) {
        // the tags 8 entries at a time, every read of a step issued before any is compared (one
        // dependent read per entry costs a memory round trip per entry when parsing from HBM)
        const pos_t tstart = (pos_t)ri.tr.tstart;
        const uint32_t esz = ri.tr.big ? 6u : 3u;
        uint32_t prev = 0;
        bool sorted = true;
        for (uint32_t i0 = 0; i0 < ri.nent; i0 += 8) {
            uint32_t tg[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t i = i0 + u < ri.nent ? i0 + u : ri.nent - 1;
                const pos_t p = tstart + (pos_t)(i * esz);
                const uint32_t b0 = s.u8(p), b1 = s.u8(p + 1);
                tg[u] = ri.tr.big ? ((b0 << 8) | b1) : b0;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t i = i0 + u;
                const bool in = i < ri.nent;
                sorted = sorted & !(in & (i > 0) & (tg[u] <= prev));
                prev = in ? tg[u] : prev;
            }
        }
        ri.sorted = sorted;
    }
    return ri;
}

// m.field(tag) (internal/types/msg.go:466-475): the field's end offset relative to the data
// start, or -1 (absent, or end > dataSize).  k = the tag's index in a Writer's table.
template <class Src>
__device__ __forceinline__ long long rec_field_end(const Src &s, const RecInfo &ri, uint32_t tag, uint32_t k) {
    using pos_t = typename Src::pos_t;
    if (!ri.ok) return -1;
    const pos_t tstart = (pos_t)ri.tr.tstart;
    long long end = -1;
    bool hit = false;
    if (ri.sorted && k < ri.nent) {
        if (ri.tr.big) {
            pos_t p = tstart + (pos_t)k * 6;
            uint32_t tg = (s.u8(p) << 8) | s.u8(p + 1);
            if (tg == tag) {
                end = ((long long)s.u8(p + 2) << 24) | (s.u8(p + 3) << 16) | (s.u8(p + 4) << 8) | s.u8(p + 5);
                hit = true;
            }
        } else {
            pos_t p = tstart + (pos_t)k * 3;
            if (s.u8(p) == tag) {
                end = (s.u8(p + 1) << 8) | s.u8(p + 2);
                hit = true;
            }
        }
    }
    if (!hit) end = table_search(s, tstart, ri.nent, ri.tr.big, tag);
    if (end > (long long)ri.tr.dsize) end = -1; // m.field: end > dataSize => nil
    return end;
}

// Parse record r occupying [rs, re) of the source into fs's columns; to_stream converts a
// source position to a stream offset (string/bytes spans).  Kind K_LIST fields are skipped.
template <class Src>
__device__ __forceinline__ void decode_record_generic(const Src &s, typename Src::pos_t rs, typename Src::pos_t re,
                                                      uint64_t r, const FieldSet &fs, long long to_stream) {
    using pos_t = typename Src::pos_t;
    const RecInfo ri = rec_open(s, rs, re);
    if (fs.status) fs.status[r] = (uint8_t)ri.tr.st;
    const pos_t dstart = (pos_t)ri.tr.dstart;
    uint64_t errs = 0;
    for (uint32_t f = 0; f < fs.nfields; f++) {
        const uint32_t kind = fs.kinds[f];
        if (kind == K_LIST) continue;
        const long long end = rec_field_end(s, ri, fs.tags[f], fs.rank[f]);
        const bool ok = decode_store(s, kind, dstart, end, to_stream, fs.cols[f], r);
        if (!ok && f < 64) errs |= 1ull << f;
    }
    if (fs.errmask) fs.errmask[r] = errs;
}

// ---- fast path: compile-time schema ------------------------------------------------------

// A run-time schema has no fast path.
struct RuntimeSpec {
    static constexpr int N = 0;
    static constexpr bool big = false;
};

// Spec (generated by jit.cpp) provides:
//   N              number of fields (1..SPEC_KFIELDS; the register-resident fast path below
//                  takes up to FAST_MAX_FIELDS small-table fields, fast_wide the rest)
//   kind[f], rank[f]  per schema field
//   stag[k]        k-th tag of the table a Writer emits (strictly increasing)
//   order[k]       the schema field of table entry k (rank's inverse)
//   big            the Writer's tables are big for every record (a tag > 255: IsBigMessage,
//                  internal/format/msg.go:43-61)
constexpr int FAST_MAX_FIELDS = 24;

// Unrolled at compile time: field F's kind and table index are constants, so every field
// is straight-line code.  Phase 1 issues every field's LDS reads, phase 2 decodes and
// stores, so the LDS latency is paid once per record, not once per field.
template <class Spec>
struct FastRec {
    Win w[Spec::N];
    int e[Spec::N], lo[Spec::N];
};

template <class Spec, int F>
struct FieldLoad {
    static __device__ __forceinline__ void run(FastRec<Spec> &fr, const LdsSrc &s, int ds, const uint32_t *ends,
                                               uint32_t dsize) {
        if constexpr (F < Spec::N) {
            constexpr uint32_t K = Spec::kind[F];
            const uint32_t end = ends[Spec::rank[F]];
            // end > dataSize => nil; an empty field decodes to zero: read a harmless window
            const bool has = (end <= dsize) & (end > 0);
            if constexpr (K == K_LIST) {
                // list<message> of a nested schema: only its extent [lo, e) (empty if absent)
                fr.lo[F] = ds;
                fr.e[F] = has ? ds + (int)end : ds;
            } else {
                fr.e[F] = has ? ds + (int)end : SLAB_GUARD;
                fr.lo[F] = has ? ds : SLAB_GUARD;
                // narrow windows are valid because fast_prepare only accepts natural-type records
                fr.w[F] = load_win<K, true>(s, fr.e[F]);
            }
            FieldLoad<Spec, F + 1>::run(fr, s, ds, ends, dsize);
        }
    }
};

// true iff every int/float field F is empty or has type cross_kind_type(kind[F])
template <class Spec, int F>
struct FieldNat {
    static __device__ __forceinline__ bool ok(const FastRec<Spec> &fr) {
        if constexpr (F >= Spec::N) {
            return true;
        } else {
            constexpr uint32_t NT = cross_kind_type(Spec::kind[F]);
            bool good = true;
            if constexpr (NT != 0) good = (fr.e[F] <= fr.lo[F]) | (((uint32_t)fr.w[F].t.q0 & 0xff) == NT);
            return good & FieldNat<Spec, F + 1>::ok(fr);
        }
    }
};

// ERR: also collect field F's <Kind>Err outcome into bit F of errs (a present, non-empty field
// whose decoder errs; internal/types/msg.go:233-459)
template <class Spec, int F, bool ERR = false>
struct FieldStore {
    static __device__ __forceinline__ void run(const FastRec<Spec> &fr, long long to_stream, const FieldSet &fs,
                                               uint64_t r, uint64_t &errs) {
        if constexpr (F < Spec::N) {
            constexpr uint32_t K = Spec::kind[F];
            if constexpr (K != K_LIST) {
                bool ok = true;
                const Val v = decode_tail_k<K, true>(fr.w[F], fr.lo[F], fr.e[F], to_stream, ERR ? &ok : nullptr);
                store_value_k<K>(fs.cols[F], r, v);
                if constexpr (ERR && F < 64) errs |= (!ok & (fr.e[F] > fr.lo[F])) ? (1ull << F) : 0ull;
            }
            FieldStore<Spec, F + 1, ERR>::run(fr, to_stream, fs, r, errs);
        }
    }
};

// Fast path, part 1 (LdsSrc only): trailer, table check and every field's window read into
// registers.  Returns false (nothing read into fr, nothing written) when the record needs
// the generic path.  After it returns the record's LDS bytes are no longer needed.
// Compact records (3N + 4 <= 16: list items, small messages): trailer AND table come from the
// one 16-byte tail window — [table 3N][rvarint dataSize, 1-2 bytes][3N][TypeMessage] — so
// the table needs no second round of LDS reads.  Accepts exactly what the general fast path
// accepts, restricted to a 1-2 byte data size (anything else returns false: generic path).
template <class Spec>
__device__ __forceinline__ bool fast_prepare_compact(const LdsSrc &s, int rs, int re, FastRec<Spec> &fr) {
    constexpr int N = Spec::N;
    static_assert(3 * N + 4 <= 16, "compact records only");
    const Tail t = load_tail(s, re);
    const uint32_t type = (uint32_t)t.q0 & 0xff, tsz = (uint32_t)(t.q0 >> 8) & 0xff;
    const uint32_t b3 = (uint32_t)(t.q0 >> 16) & 0xff, b4 = (uint32_t)(t.q0 >> 24) & 0xff;
    const bool two = (b3 & 0x80) != 0; // data size: reverse varint ending at re-3
    const uint32_t L = two ? 2u : 1u;
    const uint32_t dsz = two ? ((b3 & 0x7f) | ((b4 & 0x7f) << 7)) : b3;
    const int ts = re - 2 - (int)L - 3 * N, ds = ts - (int)dsz;
    bool ok = (type == T_MESSAGE) & (tsz == 3u * N) & (!two | ((b4 & 0x80) == 0)) & (ds >= rs);
    // table: shift the 128-bit tail (q1:q0, byte re-1 lowest) right past the trailer; entry
    // N-1-k then sits in bits [24k, 24k + 24) as tag | end_hi | end_lo
    const uint32_t sh = 8u * (2u + L);
    const uint64_t lo = (t.q0 >> sh) | (t.q1 << (64 - sh)), hi = t.q1 >> sh;
    uint32_t ends[N];
#pragma unroll
    for (int j = 0; j < N; j++) {
        const int bo = 24 * (N - 1 - j);
        const uint32_t ent =
            (uint32_t)((bo >= 64 ? hi >> (bo - 64) : (lo >> bo) | (bo ? hi << (64 - bo) : 0ull)) & 0xffffff);
        ok = ok & ((ent >> 16) == Spec::stag[j]);
        ends[j] = ent & 0xffff;
    }
    if (!ok) return false;
    FieldLoad<Spec, 0>::run(fr, s, ds, ends, dsz);
    return FieldNat<Spec, 0>::ok(fr);
}

template <class Spec>
__device__ __forceinline__ bool fast_prepare(const LdsSrc &s, int rs, int re, FastRec<Spec> &fr) {
    constexpr int N = Spec::N;
    if (re <= rs) return false;
#if !defined(SPEC_NO_COMPACT)
    if constexpr (3 * N + 4 <= 16) return fast_prepare_compact<Spec>(s, rs, re, fr);
#endif
    Trailer tr = parse_trailer(s, rs, re);
    if ((tr.st != ST_OK) | tr.big | (tr.tsize != 3u * N)) return false;
    const int ts = (int)tr.tstart;
    // the table's 3N bytes, re-aligned into qwords: c[j] = bytes [ts+8j, ts+8j+8), each a
    // 64-bit funnel shift of two aligned qwords.  (No select between array elements here: in
    // the not-yet-unrolled loop LLVM folds `hi ? d[i+1] : d[i]` into a load at a variable
    // index, which after unrolling is a 2N-deep v_cndmask chain per dword.)
    constexpr int NC = (3 * N + 7) / 8;  // realigned qwords holding the table
    constexpr int NQ = NC + 1;           // aligned qwords covering [ts & ~7, ts + 3N)
    const int base = ts & ~7;
    const uint32_t sh = 8u * (uint32_t)(ts & 7);
    uint64_t q[NQ];
#pragma unroll
    for (int j = 0; j < NQ; j++) q[j] = s.d64(base + 8 * j);
    uint64_t c[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) c[j] = (q[j] >> sh) | ((q[j + 1] << 1) << (63 - sh));
    // entry k = bytes 3k (tag), 3k+1..3k+2 (end, big-endian): the table must hold exactly the
    // Writer's tags (strictly increasing), so binary search would land on entry rank[f]
    auto byte_at = [&](int j) -> uint32_t { return (uint32_t)(c[j >> 3] >> (8 * (j & 7))) & 0xff; };
    bool hit = true;
    uint32_t ends[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        hit = hit & (byte_at(3 * k) == Spec::stag[k]);
        ends[k] = (byte_at(3 * k + 1) << 8) | byte_at(3 * k + 2);
    }
    if (!hit) return false;
    FieldLoad<Spec, 0>::run(fr, s, (int)tr.dstart, ends, tr.dsize);
    // every int/float field holds the type the Writer emits for its kind (or is empty): the
    // decode needs no cross-width branches (a record written under another schema version
    // takes the generic path)
    return FieldNat<Spec, 0>::ok(fr);
}

// Fast path, part 2: decode every field from registers and store the columns.
template <class Spec, bool ERR = false>
__device__ __forceinline__ void fast_finish(const FastRec<Spec> &fr, uint64_t r, const FieldSet &fs,
                                            long long to_stream) {
    uint64_t errs = 0;
    FieldStore<Spec, 0, ERR>::run(fr, to_stream, fs, r, errs);
    if (fs.status) fs.status[r] = ST_OK;
    if constexpr (ERR) fs.errmask[r] = errs;
}

// ---- fast path for wide schemas and big tables --------------------------------------------
// Schemas with more than FAST_MAX_FIELDS fields, or whose tags make every table big (u16 tag |
// u32 end entries, internal/format/msg.go:138-186).  The trailer is checked as by fast_prepare;
// then the table is walked in batches of FAST_BATCH entries: the batch's entries read with a few
// wide LDS reads and checked against the Writer's tags (strictly increasing, so the reference's
// binary search lands on entry k for the k-th tag), its fields' windows read, their types checked
// (the type a Writer emits for the kind), decoded and stored.  A record rejected after some
// batches were stored runs the generic path, which rewrites every column and the status, so the
// result never depends on where the fast path gave up.
constexpr int FAST_BATCH = 8;

template <class Spec, int J0, int K, int NB>
struct WideField {
    static __device__ __forceinline__ void load(Win (&w)[NB], int (&e)[NB], int (&lo)[NB], const LdsSrc &s, int ds,
                                                const uint32_t (&ends)[NB], uint32_t dsize) {
        if constexpr (K < NB) {
            constexpr uint32_t KD = Spec::kind[Spec::order[J0 + K]];
            const bool has = (ends[K] <= dsize) & (ends[K] > 0);
            e[K] = has ? ds + (int)ends[K] : SLAB_GUARD;
            lo[K] = has ? ds : SLAB_GUARD;
            w[K] = load_win<KD, true>(s, e[K]);
            WideField<Spec, J0, K + 1, NB>::load(w, e, lo, s, ds, ends, dsize);
        }
    }
    static __device__ __forceinline__ bool nat(const Win (&w)[NB], const int (&e)[NB], const int (&lo)[NB]) {
        if constexpr (K >= NB) {
            return true;
        } else {
            constexpr uint32_t NT = cross_kind_type(Spec::kind[Spec::order[J0 + K]]);
            bool good = true;
            if constexpr (NT != 0) good = (e[K] <= lo[K]) | (((uint32_t)w[K].t.q0 & 0xff) == NT);
            return good & WideField<Spec, J0, K + 1, NB>::nat(w, e, lo);
        }
    }
    template <bool ERR>
    static __device__ __forceinline__ void store(const Win (&w)[NB], const int (&e)[NB], const int (&lo)[NB],
                                                 long long to_stream, const FieldSet &fs, uint64_t r, uint64_t &errs) {
        if constexpr (K < NB) {
            constexpr int F = Spec::order[J0 + K];
            constexpr uint32_t KD = Spec::kind[F];
            bool ok = true;
            const Val v = decode_tail_k<KD, true>(w[K], lo[K], e[K], to_stream, ERR ? &ok : nullptr);
            store_value_k<KD>(fs.cols[F], r, v);
            if constexpr (ERR && F < 64) errs |= (!ok & (e[K] > lo[K])) ? (1ull << F) : 0ull;
            WideField<Spec, J0, K + 1, NB>::template store<ERR>(w, e, lo, to_stream, fs, r, errs);
        }
    }
};

// table entries [J0, J1): false when the record needs the generic path
template <class Spec, int J0, int J1, bool ERR>
__device__ __forceinline__ bool wide_batch(const LdsSrc &s, int ts, int ds, uint32_t dsize, uint64_t r,
                                           const FieldSet &fs, long long to_stream, uint64_t &errs) {
    constexpr int NB = J1 - J0;
    constexpr int ESZ = Spec::big ? 6 : 3;
    constexpr int NC = (ESZ * NB + 7) / 8, NQ = NC + 1;
    const int p0 = ts + ESZ * J0;
    const int base = p0 & ~7;
    const uint32_t sh = 8u * (uint32_t)(p0 & 7);
    uint64_t q[NQ];
#pragma unroll
    for (int j = 0; j < NQ; j++) q[j] = s.d64(base + 8 * j);
    uint64_t c[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) c[j] = (q[j] >> sh) | ((q[j + 1] << 1) << (63 - sh));
    auto byte_at = [&](int j) -> uint32_t { return (uint32_t)(c[j >> 3] >> (8 * (j & 7))) & 0xff; };
    bool hit = true;
    uint32_t ends[NB];
#pragma unroll
    for (int k = 0; k < NB; k++) {
        if constexpr (Spec::big) {
            hit = hit & (((byte_at(6 * k) << 8) | byte_at(6 * k + 1)) == Spec::stag[J0 + k]);
            ends[k] = (byte_at(6 * k + 2) << 24) | (byte_at(6 * k + 3) << 16) | (byte_at(6 * k + 4) << 8) |
                      byte_at(6 * k + 5);
        } else {
            hit = hit & (byte_at(3 * k) == Spec::stag[J0 + k]);
            ends[k] = (byte_at(3 * k + 1) << 8) | byte_at(3 * k + 2);
        }
    }
    if (!hit) return false;
    Win w[NB];
    int e[NB], lo[NB];
    WideField<Spec, J0, 0, NB>::load(w, e, lo, s, ds, ends, dsize);
    if (!WideField<Spec, J0, 0, NB>::nat(w, e, lo)) return false;
    WideField<Spec, J0, 0, NB>::template store<ERR>(w, e, lo, to_stream, fs, r, errs);
    return true;
}

template <class Spec, int J0, bool ERR>
struct WideBatches {
    static __device__ __forceinline__ bool run(const LdsSrc &s, int ts, int ds, uint32_t dsize, uint64_t r,
                                               const FieldSet &fs, long long to_stream, uint64_t &errs) {
        if constexpr (J0 >= Spec::N) {
            return true;
        } else {
            constexpr int J1 = J0 + FAST_BATCH < Spec::N ? J0 + FAST_BATCH : Spec::N;
            if (!wide_batch<Spec, J0, J1, ERR>(s, ts, ds, dsize, r, fs, to_stream, errs)) return false;
            return WideBatches<Spec, J1, ERR>::run(s, ts, ds, dsize, r, fs, to_stream, errs);
        }
    }
};

// table entries [J0, JE) in batches of FAST_BATCH (a wave pair's half of a wide record)
template <class Spec, int J0, int JE, bool ERR = false>
struct WideBatchesTo {
    static __device__ __forceinline__ bool run(const LdsSrc &s, int ts, int ds, uint32_t dsize, uint64_t r,
                                               const FieldSet &fs, long long to_stream, uint64_t &errs) {
        if constexpr (J0 >= JE) {
            return true;
        } else {
            constexpr int J1 = J0 + FAST_BATCH < JE ? J0 + FAST_BATCH : JE;
            if (!wide_batch<Spec, J0, J1, ERR>(s, ts, ds, dsize, r, fs, to_stream, errs)) return false;
            return WideBatchesTo<Spec, J1, JE, ERR>::run(s, ts, ds, dsize, r, fs, to_stream, errs);
        }
    }
};

// Part h of P of a record's fields (table entries [lo(h), lo(h + 1)); for a pair the boundary is
// the batch boundary near N/2) for the waves of one group (decode_flat_pair): false when this part
// needs the generic path.  No status: the group's first wave writes it once every part succeeded.
// ERR: this part's error-mask bits in errs.
template <class Spec, int P>
__host__ __device__ constexpr int flat_part_lo(int h) {
    if (h >= P) return Spec::N;
    if (P == 2) return h == 0 ? 0 : ((Spec::N / 2 + FAST_BATCH - 1) / FAST_BATCH) * FAST_BATCH;
    return (h * Spec::N) / P;
}
template <class Spec, bool ERR, int P, int H = 0>
__device__ __forceinline__ bool wide_part_run(const LdsSrc &s, const Trailer &tr, uint64_t r, const FieldSet &fs,
                                              long long to_stream, int h, uint64_t &errs) {
    if constexpr (H >= P) {
        return true;
    } else {
        constexpr int J0 = flat_part_lo<Spec, P>(H), J1 = flat_part_lo<Spec, P>(H + 1);
        if (h == H)
            return WideBatchesTo<Spec, J0, J1, ERR>::run(s, (int)tr.tstart, (int)tr.dstart, tr.dsize, r, fs, to_stream, errs);
        return wide_part_run<Spec, ERR, P, H + 1>(s, tr, r, fs, to_stream, h, errs);
    }
}
template <class Spec, bool ERR = false, int P = 2>
__device__ __forceinline__ bool fast_wide_half(const LdsSrc &s, int rs, int re, uint64_t r, const FieldSet &fs,
                                               long long to_stream, int h, uint64_t &errs) {
    if (re <= rs) return false;
    const Trailer tr = parse_trailer(s, rs, re);
    if ((tr.st != ST_OK) | (tr.big != Spec::big) | (tr.tsize != (Spec::big ? 6u : 3u) * (uint32_t)Spec::N)) return false;
    return wide_part_run<Spec, ERR, P>(s, tr, r, fs, to_stream, h, errs);
}

// The whole record (columns, status, errmask); false: nothing final written, run the generic path.
template <class Spec, bool ERR = false>
__device__ __forceinline__ bool fast_wide(const LdsSrc &s, int rs, int re, uint64_t r, const FieldSet &fs,
                                          long long to_stream) {
    if (re <= rs) return false;
    const Trailer tr = parse_trailer(s, rs, re);
    if ((tr.st != ST_OK) | (tr.big != Spec::big) | (tr.tsize != (Spec::big ? 6u : 3u) * (uint32_t)Spec::N)) return false;
    uint64_t errs = 0;
    if (!WideBatches<Spec, 0, ERR>::run(s, (int)tr.tstart, (int)tr.dstart, tr.dsize, r, fs, to_stream, errs))
        return false;
    if (fs.status) fs.status[r] = ST_OK;
    if constexpr (ERR) fs.errmask[r] = errs;
    return true;
}

// ---- kernel body -------------------------------------------------------------------------

// One wave's group of 64 consecutive records: per-lane record bounds and the wave's span.
struct Group {
    uint64_t rec_lo, rec_hi; // this lane's record [rec_lo, rec_hi) in the stream
    uint64_t aligned_lo;     // span start rounded down to 16 (wave-uniform)
    uint32_t chunks;         // 1 KiB DMA chunks covering the span (wave-uniform)
    bool in_lds;             // span fits the slab (wave-uniform)
};

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    return __builtin_amdgcn_readfirstlane((uint32_t)v) |
           ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

// ends[] of group g, as (lo, hi) per lane: lo = ends[r-1] (0 for record 0), hi = ends[r].
__device__ __forceinline__ void load_group_ends(const DecodeArgs &a, uint64_t base, int lane, uint64_t &lo,
                                                uint64_t &hi) {
    const uint64_t r = base + lane;
    const uint64_t last = a.n - 1;
    hi = a.ends[r < last ? r : last];
    lo = (r == 0 ? 0 : a.ends[(r - 1) < last ? r - 1 : last]) + a.head;
}

__device__ __forceinline__ Group make_group(const DecodeArgs &a, uint64_t base, int lane, uint64_t lo, uint64_t hi,
                                            uint32_t slab) {
    Group gr;
    gr.rec_lo = lo;
    gr.rec_hi = hi < lo ? lo : hi; // malformed ends: treat as empty
    const uint64_t nrec = a.n - base < 64 ? a.n - base : 64;
    const uint64_t span_lo = uniform64(__shfl(lo, 0));
    const uint64_t span_hi = uniform64(__shfl(hi, (int)nrec - 1));
    gr.aligned_lo = span_lo & ~15ull;
    const uint64_t bytes = span_hi > gr.aligned_lo ? span_hi - gr.aligned_lo : 0;
    const uint64_t chunks = (bytes + 1023) >> 10;
    gr.chunks = (uint32_t)chunks;
    gr.in_lds = slab > 0 && span_hi >= span_lo && SLAB_GUARD + chunks * 1024 + 16 <= (uint64_t)slab;
    return gr;
}

__device__ __forceinline__ void issue_dma(__amdgpu_buffer_rsrc_t rsrc, uint8_t *slab, const Group &gr, int lane) {
    for (uint32_t c = 0; c < gr.chunks; c++) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsrc, (__attribute__((address_space(3))) void *)(slab + SLAB_GUARD + c * 1024), 16,
            (uint32_t)gr.aligned_lo + c * 1024 + lane * 16, 0, 0, 0);
    }
}

// The DMA'd 16-byte chunk holding the stream's last bytes came back zeroed if it straddles
// the end (whole-access range check): refill it bytewise.
__device__ __forceinline__ void fix_stream_tail(const DecodeArgs &a, __amdgpu_buffer_rsrc_t rsrc, uint8_t *slab,
                                                const Group &gr, int lane) {
    const uint64_t tail = a.stream_len & ~15ull;
    const uint64_t span_end = gr.aligned_lo + (uint64_t)gr.chunks * 1024;
    if (tail < a.stream_len && tail >= gr.aligned_lo && tail < span_end) {
        if (lane < 16 && tail + lane < a.stream_len)
            slab[SLAB_GUARD + (tail - gr.aligned_lo) + lane] =
                (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (uint32_t)(tail + lane), 0, 0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// Persistent waves: wave w of the grid decodes groups w, w + W, w + 2W, ... (W = waves in the
// grid, sized by the launcher to what the CUs hold at once).  Per group:
//   wait for its DMA -> fast_prepare (trailer, table, all field windows into registers) and
//   the generic path for any rejected record -> the slab is free: issue the NEXT group's DMA
//   -> decode + store this group from registers while that DMA is in flight.
template <class Spec, bool ERR = false>
__device__ __forceinline__ void decode_flat_body(const DecodeArgs &a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int nw = blockDim.x >> 6;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const uint64_t ngroups = (a.n - a.r0 + 63) / 64;
    const uint64_t stride = (uint64_t)gridDim.x * nw;
    uint64_t g = (uint64_t)blockIdx.x * nw + wave;
    if (g >= ngroups) return;
    uint8_t *slab = smem + wave * a.slab;
    __amdgpu_buffer_rsrc_t rsrc =
        uniform_rsrc(a.stream, a.stream_len);

    uint64_t lo, hi;
    load_group_ends(a, a.r0 + g * 64, lane, lo, hi);
    Group cur = make_group(a, a.r0 + g * 64, lane, lo, hi, a.slab);
    if (cur.in_lds) issue_dma(rsrc, slab, cur, lane);
    // the next group's ends are always one iteration ahead
    uint64_t gn = g + stride, nlo = 0, nhi = 0;
    if (gn < ngroups) load_group_ends(a, a.r0 + gn * 64, lane, nlo, nhi);

    while (true) {
        const uint64_t base = a.r0 + g * 64;
        const uint64_t r = base + lane;
        const bool valid = r < a.n;
        const bool has_next = gn < ngroups;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this group's DMA, the next group's ends
        const Group nxt = make_group(a, has_next ? a.r0 + gn * 64 : base, lane, nlo, nhi, a.slab);
        const uint64_t g2 = gn + stride;
        uint64_t lo2 = 0, hi2 = 0;

        if (cur.in_lds) {
            fix_stream_tail(a, rsrc, slab, cur, lane);
            LdsSrc s{(lds_u8 *)slab};
            const int rs = SLAB_GUARD + (int)(cur.rec_lo - cur.aligned_lo);
            const int re = SLAB_GUARD + (int)(cur.rec_hi - cur.aligned_lo);
            const long long to_stream = (long long)cur.aligned_lo - SLAB_GUARD;
            if constexpr (Spec::N > 0) {
                FastRec<Spec> fr;
                bool fast = valid && fast_prepare<Spec>(s, rs, re, fr);
                if (valid && !fast) decode_record_generic(s, rs, re, r, a.f, to_stream);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // every LDS read of this group done
                if (has_next && nxt.in_lds) issue_dma(rsrc, slab, nxt, lane);
                if (g2 < ngroups) load_group_ends(a, a.r0 + g2 * 64, lane, lo2, hi2);
                if (fast) fast_finish<Spec, ERR>(fr, r, a.f, to_stream);
            } else {
                if (valid) decode_record_generic(s, rs, re, r, a.f, to_stream);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (has_next && nxt.in_lds) issue_dma(rsrc, slab, nxt, lane);
                if (g2 < ngroups) load_group_ends(a, a.r0 + g2 * 64, lane, lo2, hi2);
            }
        } else {
            if (has_next && nxt.in_lds) issue_dma(rsrc, slab, nxt, lane);
            if (g2 < ngroups) load_group_ends(a, a.r0 + g2 * 64, lane, lo2, hi2);
            if (valid) {
                GlobalSrc s{a.stream, a.stream_len};
                decode_record_generic(s, (long long)cur.rec_lo, (long long)cur.rec_hi, r, a.f, 0);
            }
        }
        if (!has_next) break;
        g = gn;
        gn = g2;
        cur = nxt;
        nlo = lo2;
        nhi = hi2;
    }
}

// One group per wave (the default grid): stage, decode, done.  Same steps as one iteration of
// decode_flat_body without the hand-off to a next group, so nothing fences the fast path's
// LDS reads from its decode and stores.
template <class Spec, bool ERR = false>
__device__ __forceinline__ void decode_flat_once(const DecodeArgs &a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    // blocks are dealt round-robin to the 8 XCDs: with xcd = 1, block b takes the b/8-th slot
    // of XCD b%8's contiguous share of the groups, so neighbouring groups (which share the
    // narrow columns' cache lines) are written through one L2
    uint64_t blk = blockIdx.x;
    if (a.xcd) {
        const uint64_t per = (gridDim.x + 7) / 8;
        blk = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    }
    const uint64_t base = a.r0 + (blk * (blockDim.x >> 6) + wave) * 64;
    if (base >= a.n) return;
    const uint64_t r = base + lane;
    const bool valid = r < a.n;
    uint8_t *slab = smem + wave * a.slab;
    __amdgpu_buffer_rsrc_t rsrc =
        uniform_rsrc(a.stream, a.stream_len);
    const uint64_t hi = a.ends[valid ? r : a.n - 1];
    uint64_t lo = __shfl_up(hi, 1);
    if (lane == 0) lo = r == 0 ? 0 : a.ends[r - 1];
    lo += a.head;
    const Group cur = make_group(a, base, lane, lo, hi, a.slab);
    if (cur.in_lds) {
        issue_dma(rsrc, slab, cur, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        fix_stream_tail(a, rsrc, slab, cur, lane);
        if (!valid) return;
        LdsSrc s{(lds_u8 *)slab};
        const int rs = SLAB_GUARD + (int)(cur.rec_lo - cur.aligned_lo);
        const int re = SLAB_GUARD + (int)(cur.rec_hi - cur.aligned_lo);
        const long long to_stream = (long long)cur.aligned_lo - SLAB_GUARD;
        if constexpr (Spec::N > 0) {
            if constexpr (Spec::N <= FAST_MAX_FIELDS && !Spec::big) {
                FastRec<Spec> fr;
                if (fast_prepare<Spec>(s, rs, re, fr)) {
                    fast_finish<Spec, ERR>(fr, r, a.f, to_stream);
                    return;
                }
            } else {
                if (fast_wide<Spec, ERR>(s, rs, re, r, a.f, to_stream)) return;
            }
        }
        decode_record_generic(s, rs, re, r, a.f, to_stream);
    } else if (valid) {
        GlobalSrc s{a.stream, a.stream_len};
        decode_record_generic(s, (long long)cur.rec_lo, (long long)cur.rec_hi, r, a.f, 0);
    }
}

// A wide schema's group of 64 records on a wave PAIR (a 128-thread block): both waves stage the
// group's span once in the block's slab (each issues half the LDS-DMA chunks), each decodes half
// of the fields (fast_wide_half), wave 1 hands its verdict to wave 0 through LDS, and wave 0
// writes the status — or, where either half needs it, runs the generic path over the whole
// record (it rewrites every column).  Same LDS per 64 records, twice the waves: one wave's LDS
// and memory latency overlaps the other's decode.  ERR: every wave's mask bits, OR-ed by wave 0.
// P waves per group in general (P parts of the fields; build-time A/B, jit.cpp SPEC_AB_FLAT_WAVES).
template <class Spec, bool ERR = false, int P = 2>
__device__ __forceinline__ void decode_flat_pair(const DecodeArgs &a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    uint64_t blk = blockIdx.x;
    if (a.xcd) {
        const uint64_t per = (gridDim.x + 7) / 8;
        blk = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    }
    const uint64_t base = a.r0 + blk * 64;
    if (base >= a.n) return; // (block-uniform)
    const uint64_t r = base + lane;
    const bool valid = r < a.n;
    uint8_t *slab = smem;
    uint32_t *xch = (uint32_t *)(smem + a.slab);
    __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(a.stream, a.stream_len);
    const uint64_t hi = a.ends[valid ? r : a.n - 1];
    uint64_t lo = __shfl_up(hi, 1);
    if (lane == 0) lo = r == 0 ? 0 : a.ends[r - 1];
    lo += a.head;
    const Group cur = make_group(a, base, lane, lo, hi, a.slab);
    if (!cur.in_lds) {
        if (wave == 0 && valid) {
            GlobalSrc s{a.stream, a.stream_len};
            decode_record_generic(s, (long long)cur.rec_lo, (long long)cur.rec_hi, r, a.f, 0);
        }
        return;
    }
    for (uint32_t c = (uint32_t)wave; c < cur.chunks; c += P)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(slab + SLAB_GUARD + c * 1024),
                                                 16, (uint32_t)cur.aligned_lo + c * 1024 + lane * 16, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the chunk straddling the stream end is refilled by the wave that loaded it
    const uint64_t tail = a.stream_len & ~15ull;
    if (tail < a.stream_len && tail >= cur.aligned_lo && tail < cur.aligned_lo + (uint64_t)cur.chunks * 1024 &&
        (int)(((tail - cur.aligned_lo) >> 10) % P) == wave && lane < 16 && tail + lane < a.stream_len)
        slab[SLAB_GUARD + (tail - cur.aligned_lo) + lane] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (uint32_t)(tail + lane), 0, 0);
    __syncthreads(); // the slab is whole
    LdsSrc s{(lds_u8 *)slab};
    const int rs = SLAB_GUARD + (int)(cur.rec_lo - cur.aligned_lo);
    const int re = SLAB_GUARD + (int)(cur.rec_hi - cur.aligned_lo);
    const long long to_stream = (long long)cur.aligned_lo - SLAB_GUARD;
    uint64_t errs = 0;
    const bool ok = valid && fast_wide_half<Spec, ERR, P>(s, rs, re, r, a.f, to_stream, wave, errs);
    // waves 1 .. P-1: verdicts at slab + 256 (w - 1), ERR: mask bits after them (512 B per wave)
    uint64_t *xerr = (uint64_t *)(xch + 64 * (P - 1));
    if (wave > 0) {
        xch[64 * (wave - 1) + lane] = ok ? 1u : 0u;
        if constexpr (ERR) xerr[64 * (wave - 1) + lane] = errs;
    }
    __syncthreads(); // the other waves' verdicts (and their column stores) are in
    if (wave == 0 && valid) {
        bool all = ok;
        uint64_t m = errs;
#pragma unroll
        for (int w = 1; w < P; w++) {
            all = all && xch[64 * (w - 1) + lane] != 0;
            if constexpr (ERR) m |= xerr[64 * (w - 1) + lane];
        }
        if (all) {
            if (a.f.status) a.f.status[r] = ST_OK;
            if constexpr (ERR) a.f.errmask[r] = m;
        } else {
            decode_record_generic(s, rs, re, r, a.f, to_stream);
        }
    }
}

// Kernel entry: PERSIST selects the persistent, software-pipelined loop; ERR the variant that
// also writes the per-record field error masks (a.f.errmask, spec_decode_flat_errors).
template <bool PERSIST, class Spec, bool ERR = false>
__device__ __forceinline__ void decode_flat_entry(const DecodeArgs &a) {
    if constexpr (PERSIST)
        decode_flat_body<Spec, ERR>(a);
    else
        decode_flat_once<Spec, ERR>(a);
}

bool xcd_swizzle_decode(); // XCD-aware block order, default on; build-time SPEC_AB_NOXCD off (decode_flat.hip)

// Launch shape of the flat decode: per-wave slab, waves per block, grid.
struct DecodeLaunch {
    uint32_t slab;   // bytes per wave
    unsigned wpb;    // waves per block
    unsigned blocks;
    size_t lds;      // dynamic LDS per block
};

// One group per wave (default): `wpb` waves per block (1 packs the most slabs per CU: LDS
// is the occupancy limit).  Persistent: as many blocks as the CUs hold at once, each wave
// looping over groups with the next group's DMA overlapping this group's decode.
__host__ inline DecodeLaunch decode_launch(uint64_t nrec, double avg_record, int cus, bool persistent, unsigned wpb) {
    DecodeLaunch L;
    L.slab = decode_slab_bytes(avg_record);
    L.wpb = wpb < 1 ? 1 : (wpb > 4 ? 4 : wpb);
    const uint64_t groups = (nrec + 63) / 64;
    uint64_t need = (groups + L.wpb - 1) / L.wpb;
    if (xcd_swizzle_decode() && !persistent) need = (need + 7) / 8 * 8; // 8 equal XCD shares
    if (persistent) {
        int per_cu = L.slab > 0 ? (int)((160 * 1024) / (L.wpb * L.slab)) : 8;
        per_cu = per_cu < 1 ? 1 : (per_cu > 8 ? 8 : per_cu);
        const uint64_t cap = (uint64_t)cus * per_cu;
        need = need < cap ? need : cap;
    }
    L.blocks = (unsigned)need;
    L.lds = (size_t)L.wpb * L.slab;
    return L;
}

} // namespace spec
