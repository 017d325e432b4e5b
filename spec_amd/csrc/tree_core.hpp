// tree_core.hpp — device code of the schema-tree decoder and encoder (spec_decode_tree /
// spec_encode_tree, include/spec_amd.h): every kind a generated reader/writer handles —
// structs, sub-messages, value lists, lists of structs and of messages, any, enums (int32).
//
// The work is one lane per ROW of a table (a record, a sub-message, a list element), table by
// table, so a row's bytes are whatever range its parent row found for it:
//   decode  index   per row of a message table: OpenMessage, the range of every sub-message
//                   field (rows 1:1) and the element count of every list field;
//           scan    counts -> CSR begin (a list table's rows);
//           expand  per owner row: the range of every list element (List.GetBytes);
//           decode  per row: the table's columns (getters, Decode<Kind>, struct Decode, OpenValue);
//   encode  size    per row, bottom-up: encoded size (values, structs, lists and sub-messages
//                   from their already-sized rows), IsBigMessage / IsBigList;
//           scan    record sizes -> record offsets, ends, total;
//           write   per row, top-down: its bytes, and the start of every child row.
// The reads go through range-checked buffer loads (GlobalSrc): this is the general path for
// any schema; the benchmark schemas have the LDS-staged, schema-specialised kernels.
#pragma once

#include "decode_nested_core.hpp"
#include "encode_core.hpp"

namespace spec {

constexpr int TB = 256; // threads per block of the row kernels
constexpr int TREE_MAX_F = 1024, TREE_MAX_T = 128, TREE_MAX_C = 2048, TREE_MAX_D = 1024;
constexpr int TREE_MAX_SD = 16; // structs nested in structs (include/spec_amd.h SPEC_TREE_MAX_STRUCT_DEPTH)
enum : uint32_t { K_STRUCT = 17, K_MESSAGE = 18, K_ANY = 19 };
enum : uint32_t { REL_ROOT = 0, REL_ONE = 1, REL_MANY = 2 };
enum : uint32_t { SHAPE_MESSAGE = 0, SHAPE_VALUE = 1, SHAPE_STRUCT = 2 };
constexpr uint32_t RNG_PANIC = 0xffffffffu; // range (RNG_PANIC, 0): Go panics on this element

struct TField {
    uint16_t tag;
    uint8_t kind, elem;
    int16_t parent;
    int16_t table;   // MESSAGE / LIST: the table it defines
    int16_t col;     // VALUE column (scalar, any, struct member; a value list's element column)
    int16_t present; // MESSAGE / LIST: PRESENT column; ANY: TYPE column
    uint16_t rank;   // index of the tag in the writer's table of all direct fields (lookup probe)
    uint16_t nmem, mem0; // STRUCT / LIST<STRUCT>: members[mem0 .. mem0 + nmem)
    uint16_t send;       // one past the last field of this field's subtree (pre-order)
    uint8_t nested;      // STRUCT / LIST<STRUCT>: some member is itself a struct
    uint8_t pad;
};

struct TTable {
    int16_t parent, field;
    uint8_t rel, shape, has_children, pad;
    int16_t begin_col, status_col;
    uint16_t nd, d0; // MESSAGE shape: direct[d0 .. d0 + nd) (write order), sorted[...] (table order)
    int16_t err_col; // MESSAGE shape: ERRMASK column
    int16_t pad2;
    // decode groups: a group root (the records or a list table) and the sub-message tables
    // hanging off it 1:1, decoded in one pass (tree_decode.hip)
    uint16_t groot;  // this table's group root
    uint16_t gslot;  // a sub-message table: its range slot within the group (0-based)
    uint16_t g0, gn; // a group root: its tables group[g0 .. g0 + gn), pre-order, itself first
};

struct TreeDesc {
    uint32_t nfields, ntables, ncols, pad;
    TField f[TREE_MAX_F];
    TTable t[TREE_MAX_T];
    uint16_t direct[TREE_MAX_F];
    uint16_t sorted[TREE_MAX_F];
    uint16_t sslot[TREE_MAX_F]; // sorted[d0 + k]'s index in direct[d0 ..] (its write slot)
    uint16_t members[TREE_MAX_F];
    uint16_t width[TREE_MAX_C];
    uint16_t group[TREE_MAX_T];
};

struct TreeBufs {
    void *cols[TREE_MAX_C];
    const uint8_t *heaps[TREE_MAX_C];
    uint64_t heap_lens[TREE_MAX_C];
    uint2 *rng[TREE_MAX_T];     // decode: LIST tables: element ranges (stream offsets lo, hi)
    uint32_t *cnt[TREE_MAX_T];  // decode: LIST tables: element count per owner row
    uint4 *lh[TREE_MAX_T];      // decode: LIST tables: per owner row (table start, data start, data size, count | big << 31)
    uint64_t caps[TREE_MAX_T];  // decode: row capacity per table (a list table's buffers)
    uint64_t *rowsd;            // decode: device row counts of the list tables
    uint32_t *size[TREE_MAX_T]; // encode: encoded bytes per row
    uint64_t *pos[TREE_MAX_T];  // encode: start of each row in out (tables 1..)
    uint64_t rows[TREE_MAX_T];
    const uint8_t *stream;
    uint64_t stream_len;
    const uint64_t *ends;
    const uint2 *spans; // decode over spans (Field(tag).Message() values) instead of ends
    uint64_t n;
    uint8_t *out;
    uint64_t out_cap;
    uint64_t *ends_out;
    uint64_t *offsets; // encode: record starts (exclusive scan of size[0])
    uint64_t *total;
    uint32_t *err;
    uint32_t *tblk;  // encode, record-tile writer: per record, the offsets of its field blocks (jit.cpp gen_tile)
    uint64_t *tmask; // encode, record-tile writer: per record, its present direct fields
};

__device__ __forceinline__ uint64_t grid_stride() { return (uint64_t)gridDim.x * blockDim.x; }
__device__ __forceinline__ uint64_t grid_first() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }

// ---- decode helpers ----------------------------------------------------------------------

__device__ __forceinline__ __amdgpu_buffer_rsrc_t stream_rsrc(const TreeBufs &B) {
    return uniform_rsrc(B.stream, B.stream_len);
}

// The byte range of row `row` of table x (record, sub-message field slice, list element).
__device__ __forceinline__ void row_range(const TreeBufs &B, uint32_t x, uint64_t row, long long &lo, long long &hi,
                                          bool &panic) {
    panic = false;
    if (x == 0) {
        if (B.spans) { // a value span (off, len); one past the stream would panic in Go
            const uint2 sp = B.spans[row];
            const bool out = (uint64_t)sp.x + sp.y > B.stream_len;
            panic = out;
            lo = out ? 0 : sp.x;
            hi = out ? 0 : (long long)sp.x + sp.y;
            return;
        }
        lo = row ? (long long)B.ends[row - 1] : 0;
        hi = (long long)B.ends[row];
        if (hi < lo) hi = lo;
        return;
    }
    const uint2 r = B.rng[x][row];
    panic = r.x == RNG_PANIC && r.y == 0;
    lo = panic ? 0 : r.x;
    hi = panic ? 0 : r.y;
}

__device__ __forceinline__ void store_kind(void *colp, uint64_t r, uint32_t kind, const Val &v) {
    uint8_t *c = (uint8_t *)colp;
    if (!c) return;
    switch (kind) {
    case K_BOOL:
    case K_BYTE: c[r] = (uint8_t)v.v0; break;
    case K_INT16:
    case K_UINT16: ((uint16_t *)c)[r] = (uint16_t)v.v0; break;
    case K_INT32:
    case K_UINT32:
    case K_FLOAT32: ((uint32_t *)c)[r] = (uint32_t)v.v0; break;
    case K_BIN128:
        ((uint64_t *)c)[2 * r] = v.v0;
        ((uint64_t *)c)[2 * r + 1] = v.v1;
        break;
    case K_BIN256:
        ((uint64_t *)c)[4 * r] = v.v0;
        ((uint64_t *)c)[4 * r + 1] = v.v1;
        ((uint64_t *)c)[4 * r + 2] = v.v2;
        ((uint64_t *)c)[4 * r + 3] = v.v3;
        break;
    default: ((uint64_t *)c)[r] = v.v0; break;
    }
}

__device__ __forceinline__ void store_u8(void *colp, uint64_t r, uint32_t v) {
    if (colp) ((uint8_t *)colp)[r] = (uint8_t)v;
}

// Decode<Kind>(b) of the value [lo, e) with Go's (value, n, err) (internal/decode/...; the
// value rules are decode_tail_k's, n = bytes consumed from the end).  Returns !err.  K is a
// compile-time kind (the schema-specialised tree kernels); decode_value_n dispatches a run-time one.
template <uint32_t K, class Src>
__device__ __forceinline__ bool decode_value_kn(const Src &s, typename Src::pos_t lo, typename Src::pos_t e,
                                                long long to_stream, Val &v, int &n) {
    v = Val{0, 0, 0, 0};
    n = 0;
    const long long flen = (long long)(e - lo);
    if (flen <= 0) return true; // empty input: zero value, n = 0, no error
    const Tail t = load_tail(s, e);
    const uint32_t type = (uint32_t)t.q0 & 0xff;
    const uint64_t R = tail_r(t);
    const uint32_t R2 = tail_r2(t);
    const long long avail = flen - 1;
    int m = 0;
    bool ok = false;
    if constexpr (K == K_BOOL) {
        n = 1; // DecodeBool: any type, no error (byte.go:38-51)
        ok = true;
    } else if constexpr (K == K_BYTE) {
        ok = (type == T_BYTE) & (flen >= 2);
        n = 2;
    } else if constexpr (K == K_INT16 || K == K_INT32 || K == K_INT64) {
        const bool w32 = (type == T_INT16) | (type == T_INT32);
        if (w32 || type == T_INT64) {
            const uint64_t u = rvarint_bf(R, R2, avail, w32 ? 5 : 10, m);
            if (m >= 0) {
                const long long x = w32 ? (long long)unzigzag32((uint32_t)u) : (long long)unzigzag64(u);
                ok = K == K_INT16 ? (x >= -32768) & (x <= 32767)
                     : K == K_INT32 ? (w32 | ((x >= INT32_MIN) & (x <= INT32_MAX)))
                                    : true;
                n = 1 + m;
            }
        }
    } else if constexpr (K == K_UINT16 || K == K_UINT32 || K == K_UINT64) {
        const bool w32 = (type == T_UINT16) | (type == T_UINT32);
        if (w32 || type == T_UINT64) {
            const uint64_t x = rvarint_bf(R, R2, avail, w32 ? 5 : 10, m);
            if (m >= 0) {
                ok = K == K_UINT16 ? x <= 0xffffull : K == K_UINT32 ? x <= 0xffffffffull : true;
                n = 1 + m;
            }
        }
    } else if constexpr (K == K_FLOAT32 || K == K_FLOAT64) {
        const bool f32 = (type == T_FLOAT32) & (flen >= 5), f64 = (type == T_FLOAT64) & (flen >= 9);
        if (f32 || f64) {
            n = f32 ? 5 : 9;
            ok = true;
            if constexpr (K == K_FLOAT32) { // +-MaxFloat32 range check (float.go:15-32); NaN passes
                if (f32) {
                    const uint32_t b = (uint32_t)(R & 0xffffffffu);
                    ok = !((((b >> 23) & 0xff) == 0xff) & ((b & 0x7fffff) == 0));
                } else {
                    const bool nan = (((R >> 52) & 0x7ff) == 0x7ff) & ((R & 0xfffffffffffffull) != 0);
                    ok = nan | ((R & 0x7fffffffffffffffull) <= 0x47EFFFFFE0000000ull);
                }
            }
        }
    } else if constexpr (K == K_BIN64) {
        ok = (type == T_BIN64) & (flen >= 9);
        n = 9;
    } else if constexpr (K == K_BIN128) {
        ok = (type == T_BIN128) & (flen >= 17);
        n = 17;
    } else if constexpr (K == K_BIN256) {
        ok = (type == T_BIN256) & (flen >= 33);
        n = 33;
    } else if constexpr (K == K_STRING || K == K_BYTES) {
        constexpr bool str = K == K_STRING;
        if (type == (str ? T_STRING : T_BYTES)) {
            const uint32_t len = (uint32_t)rvarint_bf(R, R2, avail, 5, m);
            if (m >= 0) {
                const long long end = (long long)(e - 1) - m - (str ? 1 : 0);
                const long long off = end - (long long)len;
                ok = (end >= (long long)lo) & (off >= (long long)lo);
                n = 1 + m + (str ? 1 : 0) + (int)len;
            }
        }
    }
    if (!ok) {
        n = 0;
        return false;
    }
    v = decode_tail_k<K>(load_win<K>(s, e), lo, e, to_stream);
    return true;
}

template <class Src>
__device__ __noinline__ bool decode_value_n(const Src &s, uint32_t kind, typename Src::pos_t lo,
                                            typename Src::pos_t e, long long to_stream, Val &v, int &n) {
#define SPEC_CASE(K) \
    case K: return decode_value_kn<K>(s, lo, e, to_stream, v, n);
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
    v = Val{0, 0, 0, 0};
    n = 0;
    return e <= lo; // not a scalar kind: empty input decodes without error
}

// DecodeStruct (internal/decode/struct.go:14-42) of the value ending at e over [lo, e), then
// the generated Decode's `b = b[len(b)-size:]` (a panic when size > len(b)): the struct's start S
// and data size; ST_OK, ST_INVALID_VALUE or ST_PANIC.  e > lo.
template <class Src>
__device__ __forceinline__ uint32_t struct_open(const Src &s, long long lo, long long e, long long &S, uint32_t &ds) {
    if (s.u8((typename Src::pos_t)(e - 1)) != T_STRUCT) return ST_INVALID_VALUE; // invalid type
    const Tail t = load_tail(s, (typename Src::pos_t)e);
    int m;
    ds = (uint32_t)rvarint_bf(tail_r(t), tail_r2(t), e - 1 - lo, 5, m);
    if (m < 0) return ST_INVALID_VALUE; // invalid data size
    const long long size = 1 + m + (long long)ds;
    if (size > e - lo) return ST_PANIC;
    S = e - size;
    return ST_OK;
}

// A generated struct's Decode (internal/lang/generator/struct.go:75-113) over [lo, e):
// DecodeStruct, then the members from the LAST to the first over b[:off]; the first error
// stops it and members decoded so far keep their values.  An inner struct member is decoded by
// its own DecodeXxx over b[:off] (its bytes end at off, its lower bound is the outer struct's
// start), consuming its size.  Returns ST_OK, ST_INVALID_VALUE, or ST_PANIC where Go slices
// b[len(b)-size:] with size > len(b) (at any depth).
template <class Src>
__device__ __noinline__ uint32_t tree_struct(const Src &s, const TreeDesc &D, const TreeBufs &B, uint32_t sf,
                                                long long lo, long long e, uint64_t row, long long to_stream) {
    const TField &F = D.f[sf];
    const Val zero = {0, 0, 0, 0};
    for (uint32_t i = sf + 1; i < F.send; i++) {
        const TField &M = D.f[i];
        if (M.kind != K_STRUCT) store_kind(B.cols[M.col], row, M.kind, zero);
    }
    if (e <= lo) return ST_OK;
    long long S;
    uint32_t ds;
    uint32_t st = struct_open(s, lo, e, S, ds);
    if (st != ST_OK) return st;
    long long off = S + ds;
    if (!F.nested) {
        for (int k = (int)F.nmem - 1; k >= 0; k--) {
            const TField &M = D.f[D.members[F.mem0 + k]];
            Val v;
            int n;
            const bool ok = decode_value_n(s, M.kind, (typename Src::pos_t)S, (typename Src::pos_t)off, to_stream, v, n);
            store_kind(B.cols[M.col], row, M.kind, v);
            if (!ok) return ST_INVALID_VALUE;
            off -= n;
        }
        return ST_OK;
    }
    // structs inside structs: an explicit stack of the open structs (field, next member, start)
    uint16_t sfi[TREE_MAX_SD];
    int16_t kk[TREE_MAX_SD];
    long long Sb[TREE_MAX_SD];
    int d = 0;
    sfi[0] = (uint16_t)sf;
    kk[0] = (int16_t)F.nmem - 1;
    Sb[0] = S;
    for (;;) {
        if (kk[d] < 0) { // this struct is done: its parent continues below its start
            if (d == 0) return ST_OK;
            off = Sb[d];
            d--;
            continue;
        }
        const uint32_t mi = D.members[D.f[sfi[d]].mem0 + kk[d]];
        kk[d]--;
        const TField &M = D.f[mi];
        if (M.kind == K_STRUCT) {
            if (off <= Sb[d]) continue; // empty input: DecodeStruct => size 0, the members stay zero
            long long S2;
            uint32_t ds2;
            st = struct_open(s, Sb[d], off, S2, ds2);
            if (st != ST_OK) return st;
            d++;
            sfi[d] = (uint16_t)mi;
            kk[d] = (int16_t)M.nmem - 1;
            Sb[d] = S2;
            off = S2 + ds2;
        } else {
            Val v;
            int n;
            const bool ok = decode_value_n(s, M.kind, (typename Src::pos_t)Sb[d], (typename Src::pos_t)off, to_stream, v, n);
            store_kind(B.cols[M.col], row, M.kind, v);
            if (!ok) return ST_INVALID_VALUE;
            off -= n;
        }
    }
}

// compactint.ReverseSize (oracle/compactint.c so_reverse_size) over the bytes below e down to lo
template <class Src>
__device__ __forceinline__ int reverse_size(const Src &s, long long lo, long long e) {
    for (int i = 0; i < 10; i++) {
        if (e - 1 - i < lo) return -(i + 1);
        if (s.u8((typename Src::pos_t)(e - 1 - i)) < 0x80) return i + 1;
    }
    return -11;
}

// decodeSize = ReverseUint32 of the bytes below e (>= lo): value, m (< 0 on error)
template <class Src>
__device__ __forceinline__ uint32_t rsize32(const Src &s, long long lo, long long e, int &m) {
    if (e <= lo) {
        m = -1;
        return 0;
    }
    const Tail t = load_tail(s, (typename Src::pos_t)e + 1); // window ending just above e: R = bytes e-1..
    return (uint32_t)rvarint_bf(tail_r(t), tail_r2(t), e - lo, 5, m);
}

// DecodeTypeSize (internal/decode/type.go:27-203) of the value ending at e over [lo, e):
// returns false on an error; n may be negative (the struct case checks n, not m: the bug is
// kept, type.go:185-191).
template <class Src>
__device__ __forceinline__ bool type_size_inl(const Src &s, long long lo, long long e, long long &n) {
    n = 0;
    if (e <= lo) return true;
    const uint32_t t = s.u8((typename Src::pos_t)(e - 1));
    const long long len = e - lo, end = e - 1;
    int m;
    switch (t) {
    case T_TRUE:
    case T_FALSE: n = 1; return true;
    case T_BYTE: n = 2; return end - lo >= 1;
    case T_INT16: case T_INT32: case T_INT64:
    case T_UINT16: case T_UINT32: case T_UINT64:
        m = reverse_size(s, lo, end);
        n = 1 + m;
        return m > 0;
    case T_FLOAT32: n = 5; return end - lo >= 4;
    case T_FLOAT64: n = 9; return end - lo >= 8;
    case T_BIN64: n = 9; return end - lo >= 8;
    case T_BIN128: n = 17; return end - lo >= 16;
    case T_BIN256: n = 33; return end - lo >= 32;
    case T_BYTES:
    case T_STRING: {
        const uint32_t ds = rsize32(s, lo, end, m);
        if (m < 0) return false;
        n = 1 + m + (long long)ds + (t == T_STRING ? 1 : 0);
        return len >= n;
    }
    case T_LIST: case T_BIG_LIST: case T_MESSAGE: case T_BIG_MESSAGE: {
        const uint32_t ts = rsize32(s, lo, end, m);
        if (m < 0) return false;
        long long size = 1 + m + (long long)ts;
        const long long end2 = end - m;
        int m2;
        const uint32_t ds = rsize32(s, lo, end2, m2);
        if (m2 < 0) return false;
        size += m2 + (long long)ds;
        n = size;
        return len >= size;
    }
    case T_STRUCT: {
        const uint32_t ds = rsize32(s, lo, end, m);
        const long long size = 1 + m + (long long)ds; // m unchecked (n is checked instead)
        n = size;
        return !(len < size);
    }
    }
    return false;
}

template <class Src>
__device__ __noinline__ bool type_size(const Src &s, long long lo, long long e, long long &n) {
    return type_size_inl(s, lo, e, n);
}

// ---- encode helpers ----------------------------------------------------------------------

__device__ __forceinline__ const uint8_t *cell(const TreeBufs &B, const TreeDesc &D, int c, uint64_t row) {
    return (const uint8_t *)B.cols[c] + row * D.width[c];
}

// Encoded size of a column element of a scalar kind (encode_core.hpp field_size rules)
__device__ __forceinline__ uint64_t value_size(const TreeBufs &B, const TreeDesc &D, int c, uint32_t kind,
                                               uint64_t row, bool &err) {
    const uint8_t *p = cell(B, D, c, row);
    switch (kind) {
    case K_BOOL: return 1;
    case K_BYTE: return 2;
    case K_INT16: return vlen32(zigzag32(*(const int16_t *)p)) + 1;
    case K_INT32: return vlen32(zigzag32(*(const int32_t *)p)) + 1;
    case K_INT64: return vlen64(zigzag64(*(const int64_t *)p)) + 1;
    case K_UINT16: return vlen32(*(const uint16_t *)p) + 1;
    case K_UINT32: return vlen32(*(const uint32_t *)p) + 1;
    case K_UINT64: return vlen64(*(const uint64_t *)p) + 1;
    case K_FLOAT32: return 5;
    case K_FLOAT64: case K_BIN64: return 9;
    case K_BIN128: return 17;
    case K_BIN256: return 33;
    case K_STRING:
    case K_BYTES:
    case K_ANY: {
        const uint2 sp = *(const uint2 *)p;
        if ((uint64_t)sp.y > MAX_SIZE || (uint64_t)sp.x + sp.y > B.heap_lens[c]) err = true;
        if (kind == K_ANY) return sp.y;
        return (uint64_t)sp.y + vlen32(sp.y) + 1 + (kind == K_STRING ? 1 : 0);
    }
    }
    return 0;
}

// The generated EncodeXxxTo's size (internal/lang/generator/struct.go:115-142): the members'
// encoded sizes, then EncodeStruct's rvarint(dataSize) | TypeStruct; inner structs likewise.
__device__ __forceinline__ uint64_t struct_size(const TreeBufs &B, const TreeDesc &D, uint32_t sf, uint64_t row,
                                                bool &err) {
    const TField &F = D.f[sf];
    if (!F.nested) {
        uint64_t data = 0;
        for (uint32_t k = 0; k < F.nmem; k++) {
            const TField &M = D.f[D.members[F.mem0 + k]];
            data += value_size(B, D, M.col, M.kind, row, err);
        }
        if (data > MAX_SIZE) err = true; // EncodeStruct: struct too large
        return data + vlen64(data) + 1;
    }
    uint64_t acc[TREE_MAX_SD];
    uint16_t endi[TREE_MAX_SD];
    int d = 0;
    acc[0] = 0;
    endi[0] = F.send;
    auto close = [&]() {
        const uint64_t data = acc[d];
        if (data > MAX_SIZE) err = true;
        d--;
        acc[d] += data + vlen64(data) + 1;
    };
    for (uint32_t i = sf + 1; i < F.send; i++) { // the subtree in pre-order = declaration order
        while (d > 0 && i >= endi[d]) close();
        const TField &M = D.f[i];
        if (M.kind == K_STRUCT) {
            d++;
            acc[d] = 0;
            endi[d] = M.send;
        } else {
            acc[d] += value_size(B, D, M.col, M.kind, row, err);
        }
    }
    while (d > 0) close();
    if (acc[0] > MAX_SIZE) err = true;
    return acc[0] + vlen64(acc[0]) + 1;
}

// [begin[row], begin[row + 1]) of list table y, from its BEGIN column (checked)
__device__ __forceinline__ void list_span(const TreeBufs &B, const TreeDesc &D, uint32_t y, uint64_t row, uint32_t &j0,
                                          uint32_t &j1, bool &err) {
    const uint32_t *b = (const uint32_t *)B.cols[D.t[y].begin_col];
    j0 = b[row];
    j1 = b[row + 1];
    if (j1 < j0 || (uint64_t)j1 > B.rows[y]) {
        err = true;
        j1 = j0;
    }
}

struct TreeListSize {
    uint64_t total, data;
    uint32_t count;
    bool big;
};

// EncodeListTable (internal/encode/list.go:15-75) over the elements' encoded sizes; IsBigList
// (internal/format/list.go:40-54): count > 255 or the LAST end offset > 65535
__device__ __forceinline__ TreeListSize list_size(const TreeBufs &B, const TreeDesc &D, uint32_t y, uint64_t row, bool &err) {
    uint32_t j0, j1;
    list_span(B, D, y, row, j0, j1, err);
    TreeListSize L;
    L.data = 0;
    for (uint32_t j = j0; j < j1; j++) L.data += B.size[y][j];
    L.count = j1 - j0;
    L.big = L.count > 255 || (L.count > 0 && L.data > 65535);
    const uint64_t tsize = (uint64_t)L.count * (L.big ? 4 : 2);
    if (L.data > MAX_SIZE) err = true;
    L.total = L.data + tsize + vlen64(L.data) + vlen64(tsize) + 1;
    return L;
}

// Byte emitter over the output (one lane writes one row's own bytes; child rows are written by
// later launches into the gaps this one skips).
// A row's bytes at out[pos..]: bytes are merged into the dword they fall in and stored as whole
// dwords (a byte store per byte costs a VMEM instruction per byte); the row's first and last
// dwords, which it shares with the neighbouring rows (other lanes), are stored bytewise from
// `lo` (the row start) and up to the end (finish()).  skip(n) jumps over a child's bytes (a
// sub-message, list elements) written by a LATER launch: a dword stored across such a gap may
// hold zeros for the child's bytes, which the child's own launch then overwrites.
// The emitter's memory: GSink the output in HBM (dword phase = the byte offset's), LSink a
// workgroup's LDS image of an output range (the tile writer, jit.cpp gen_tile): out byte p lives
// at img[p - sh], sh chosen so that LDS and memory agree on p's position in its 16-byte chunk.
struct GSink {
    uint8_t *out;
    __device__ __forceinline__ uint32_t ph(uint64_t p) const { return (uint32_t)(p & 3); }
    __device__ __forceinline__ void st32(uint64_t p, uint32_t v) const { *(uint32_t *)(out + p) = v; }
    __device__ __forceinline__ void st8(uint64_t p, uint32_t b) const { out[p] = (uint8_t)b; }
    // bytes [from, end) of the dword v at base (from >= base, end <= base + 4): whole, or bytewise
    // where the dword is shared with a neighbour
    __device__ __forceinline__ void word(uint64_t base, uint64_t from, uint64_t end, uint32_t v) const {
        if (from == base && end == base + 4) {
            st32(base, v);
        } else {
            for (uint64_t q = from; q < end; q++) st8(q, v >> (8 * (q - base)));
        }
    }
};
// (a tile's range may exceed the image: bytes past the image's window [sh, sh + cap) are stored
// straight to the output — dwords are 4-byte aligned in both, so none straddles the window's end)
#ifndef SPEC_TILE_OR
#define SPEC_TILE_OR 0
#endif
typedef __attribute__((address_space(3))) uint8_t TileU8; // (writable: spec_device.hpp's lds_u8 is const)
typedef __attribute__((address_space(3))) uint32_t TileU32;
typedef __attribute__((address_space(3))) uint64_t TileU64;
struct LSink {
    TileU8 *img;
    uint8_t *out;
    uint64_t lim;  // sh + cap: bytes at or past it go to HBM
    uint32_t sh32; // sh's low 32 bits: every byte of the tile is >= sh and an in-window one < sh + cap, so
                   // its image offset p - sh is (uint32_t)p - sh32 (32-bit arithmetic: fewer VALU per store)
    __device__ __forceinline__ uint32_t at(uint64_t p) const { return (uint32_t)p - sh32; }
    __device__ __forceinline__ uint32_t ph(uint64_t p) const { return at(p) & 3; }
    __device__ __forceinline__ void st32(uint64_t p, uint32_t v) const {
        if (p < lim) *(TileU32 *)(img + at(p)) = v;
        else *(uint32_t *)(out + p) = v;
    }
    __device__ __forceinline__ void st8(uint64_t p, uint32_t b) const {
        if (p < lim) img[at(p)] = (uint8_t)b;
        else out[p] = (uint8_t)b;
    }
    __device__ __forceinline__ void word(uint64_t base, uint64_t from, uint64_t end, uint32_t v) const {
#if SPEC_TILE_OR
        // the image starts zeroed and every byte belongs to one row: v's bytes outside [from, end)
        // are zero (a row's pending dword holds only its own bytes), so an OR merges the dword
        // with its neighbours' without the edge cases
        if (base < lim) {
            __hip_atomic_fetch_or((TileU32 *)(img + at(base)), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
#endif
        if (from == base && end == base + 4) {
            st32(base, v);
        } else {
            for (uint64_t q = from; q < end; q++) st8(q, v >> (8 * (q - base)));
        }
    }
};

template <class S>
struct DEmit {
    S k;
    uint64_t pos;
    uint64_t lo;    // first byte of the row (bytes below belong to another row)
    uint32_t w = 0; // pending bytes of the dword holding pos
    __device__ __forceinline__ void store_word(uint64_t base, uint64_t end, uint32_t v) { // bytes [base, end) of v
        k.word(base, base > lo ? base : lo, end, v);
    }
    __device__ __forceinline__ void store_pending(uint64_t base, uint64_t end) { store_word(base, end, w); }
    __device__ __forceinline__ void put1(uint32_t b) {
        const uint32_t ph = k.ph(pos);
        w |= (b & 0xffu) << (8 * ph);
        pos++;
        if (ph == 3) {
            store_pending(pos - 4, pos);
            w = 0;
        }
    }
    // nb (<= 8) bytes of v, lowest first, merged with the pending bytes: the full dwords stored
    __device__ __forceinline__ void put_n(uint64_t v, uint32_t nb) {
        const uint32_t ph = k.ph(pos), sh = 8 * ph;
        const uint64_t lo64 = (uint64_t)w | (v << sh);
        const uint32_t hi32 = sh ? (uint32_t)(v >> (64 - sh)) : 0u;
        const uint32_t total = ph + nb;
        const uint64_t d = pos - ph;
        if (total >= 4) store_word(d, d + 4, (uint32_t)lo64);
        if (total >= 8) store_word(d + 4, d + 8, (uint32_t)(lo64 >> 32));
        const uint32_t full = total >> 2;
        const uint32_t rest = full == 0 ? (uint32_t)lo64 : (full == 1 ? (uint32_t)(lo64 >> 32) : hi32);
        const uint32_t keep = total & 3;
        w = keep ? (rest & (0xffffffffu >> (32 - 8 * keep))) : 0u;
        pos += nb;
    }
    __device__ __forceinline__ void skip(uint64_t n) {
        if (!n) return;
        const uint32_t ph = k.ph(pos);
        const uint64_t d = pos - ph;
        pos += n;
        if (pos >= d + 4) {
            if (ph) store_pending(d, d + 4); // the gap's bytes: the child's
            w = 0;
        }
    }
    __device__ __forceinline__ void finish() {
        const uint32_t ph = k.ph(pos);
        if (ph) store_pending(pos - ph, pos);
        w = 0;
    }
    // nb (<= 8) bytes of v, lowest first, at p, bytewise (a table entry: its neighbours are
    // other fields' entries, written by other waves)
    __device__ __forceinline__ void put_at(uint64_t p, uint64_t v, uint32_t nb) {
        for (uint32_t i = 0; i < nb; i++) k.st8(p + i, (uint32_t)(v >> (8 * i)));
    }
    // reverse varint (oracle/compactint.c so_put_reverse_*): top group first, MSB clear, the
    // following groups with 0x80; up to 8 bytes (values < 2^56) built in a register at once
    __device__ __forceinline__ void rvarint(uint64_t v) {
        const uint32_t L = vlen64(v);
        if (L <= 8) {
            uint64_t x = v & 0x00ffffffffffffffull; // 7-bit groups -> bytes
            x = (x & 0x000000000fffffffull) | ((x << 4) & 0x0fffffff00000000ull);
            x = (x & 0x00003fff00003fffull) | ((x << 2) & 0x3fff00003fff0000ull);
            x = (x & 0x007f007f007f007full) | ((x << 1) & 0x7f007f007f007f00ull);
            const uint32_t drop = 8 * (8 - L);
            put_n((__builtin_bswap64(x) >> drop) | ((0x8080808080808080ull >> drop) & ~0xffull), L);
            return;
        }
        for (uint32_t i = 0; i < L; i++) put1(((uint32_t)(v >> (7 * (L - 1 - i))) & 0x7f) | (i ? 0x80 : 0));
    }
    __device__ __forceinline__ void be(uint64_t v, int nb) { // the low nb bytes of v, big-endian
        put_n(__builtin_bswap64(v) >> (8 * (8 - nb)), (uint32_t)nb);
    }
    __device__ __forceinline__ void le(uint64_t v, int nb) { put_n(v, (uint32_t)nb); }
    // heap bytes [off, off + len): 16 at a time from one 16-byte load (4-byte aligned; a load
    // straddling the heap's end reads per dword, bytes past it as 0 and never used), appended 8
    // at a time
    __device__ __forceinline__ void heap(const uint8_t *h, uint64_t hlen, uint32_t off, uint32_t len) {
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(h, hlen);
        uint32_t i = 0;
        while (i < len) {
            const uint32_t a = (off + i) & ~3u;
            uint64_t lo, hi;
            if ((uint64_t)a + 16 <= hlen) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0);
                lo = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
                hi = (uint64_t)q[2] | ((uint64_t)q[3] << 32);
            } else {
                lo = (uint64_t)buf_ld32(r, a, hlen) | ((uint64_t)buf_ld32(r, a + 4, hlen) << 32);
                hi = (uint64_t)buf_ld32(r, a + 8, hlen) | ((uint64_t)buf_ld32(r, a + 12, hlen) << 32);
            }
            const uint32_t q = off + i - a; // 0..3: bytes [q, 16) of (lo, hi) are heap bytes
            const uint32_t n1 = min(8u, len - i);
            put_n((lo >> (8 * q)) | (q ? hi << (64 - 8 * q) : 0ull), n1);
            i += n1;
            if (i < len) {
                const uint32_t n2 = min(8u - q, len - i); // the rest of the 16 loaded bytes
                put_n(hi >> (8 * q), n2);
                i += n2;
            }
        }
    }
};
using BEmit = DEmit<GSink>;
using LEmit = DEmit<LSink>;


// BEmit16: the same contract with 16-byte chunks (the generated writer of the records' table,
// whose rows are long: jit.cpp gen_write_table).  A row's bytes at out[pos..] are merged into the
// 16-byte chunk (16-byte aligned in memory) they
// fall in, and a chunk the row covers whole is stored with ONE 16-byte store: the 64 lanes of a
// store instruction write 64 different rows, i.e. 64 different cache lines, and the memory pipe
// takes such an instruction a line at a time, so wide stores move 4x the bytes per line slot of
// dword stores.  The row's first and last chunks, which it shares with the neighbouring rows
// (other lanes), are stored as whole dwords where they lie inside the row and bytewise at its
// edges, from `lo` (the row start) and up to the end (finish()).  skip(n) jumps over a child's
// bytes (a sub-message, list elements) written by a LATER launch: a chunk stored across such a
// gap may hold zeros for the child's bytes, which the child's own launch then overwrites.
struct BEmit16 {
    uint8_t *out;
    uint64_t pos;
    uint64_t lo;             // first byte of the row (bytes below belong to another row)
    uint64_t c0 = 0, c1 = 0; // the chunk holding pos: bytes below pos (emitted, or gap zeros)

    // the position of pos within its 16-byte memory chunk
    __device__ __forceinline__ uint32_t phase(uint64_t p) const { return (uint32_t)(((unsigned long long)out + p) & 15); }
    // bytes [max(base, lo), end) of the chunk at base (16-byte aligned in memory), end <= base + 16
    __device__ __forceinline__ void store_chunk(uint64_t base, uint64_t end) {
        if (base >= lo && end == base + 16) {
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            v4u v = {(uint32_t)c0, (uint32_t)(c0 >> 32), (uint32_t)c1, (uint32_t)(c1 >> 32)};
            *(v4u *)(out + base) = v;
            return;
        }
        for (uint64_t q = base > lo ? base : lo; q < end;) {
            const uint32_t k = (uint32_t)(q - base);
            const uint64_t word = k < 8 ? c0 : c1;
            const uint32_t sh = 8 * (k & 7);
            if ((k & 3) == 0 && q + 4 <= end) {
                *(uint32_t *)(out + q) = (uint32_t)(word >> sh);
                q += 4;
            } else {
                out[q] = (uint8_t)(word >> sh);
                q++;
            }
        }
    }
    // nb (<= 8) bytes of v, lowest first (bytes of v above nb are ignored)
    __device__ __forceinline__ void put_n(uint64_t v, uint32_t nb) {
        v &= nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
        const uint32_t p = phase(pos), sh = 8 * (p & 7);
        const uint64_t l64 = v << sh, h64 = sh ? v >> (64 - sh) : 0ull;
        uint64_t carry = 0;
        if (p < 8) {
            c0 |= l64;
            c1 |= h64;
        } else {
            c1 |= l64;
            carry = h64; // the next chunk's first bytes
        }
        pos += nb;
        if (p + nb >= 16) { // the chunk is complete (p >= 8 here: nb <= 8)
            store_chunk(pos - (p + nb - 16) - 16, pos - (p + nb - 16));
            c0 = carry;
            c1 = 0;
        }
    }
    __device__ __forceinline__ void put1(uint32_t b) { put_n(b, 1); }
    __device__ __forceinline__ void skip(uint64_t n) {
        if (!n) return;
        const uint32_t p = phase(pos);
        const uint64_t base = pos - p;
        pos += n;
        if (pos >= base + 16) { // leaves the chunk: store it (the rest of it is the child's gap)
            if (p) store_chunk(base, base + 16);
            c0 = c1 = 0;
        }
    }
    __device__ __forceinline__ void finish() {
        const uint32_t p = phase(pos);
        if (p) store_chunk(pos - p, pos);
        c0 = c1 = 0;
    }
    // reverse varint (oracle/compactint.c so_put_reverse_*): top group first, MSB clear, the
    // following groups with 0x80; up to 8 bytes (values < 2^56) built in a register at once
    __device__ __forceinline__ void rvarint(uint64_t v) {
        const uint32_t L = vlen64(v);
        if (L <= 8) {
            uint64_t x = v & 0x00ffffffffffffffull; // 7-bit groups -> bytes
            x = (x & 0x000000000fffffffull) | ((x << 4) & 0x0fffffff00000000ull);
            x = (x & 0x00003fff00003fffull) | ((x << 2) & 0x3fff00003fff0000ull);
            x = (x & 0x007f007f007f007full) | ((x << 1) & 0x7f007f007f007f00ull);
            const uint32_t drop = 8 * (8 - L);
            put_n((__builtin_bswap64(x) >> drop) | ((0x8080808080808080ull >> drop) & ~0xffull), L);
            return;
        }
        for (uint32_t i = 0; i < L; i++) put1(((uint32_t)(v >> (7 * (L - 1 - i))) & 0x7f) | (i ? 0x80 : 0));
    }
    __device__ __forceinline__ void be(uint64_t v, int nb) { // the low nb bytes of v, big-endian
        put_n(__builtin_bswap64(v) >> (8 * (8 - nb)), (uint32_t)nb);
    }
    __device__ __forceinline__ void le(uint64_t v, int nb) { put_n(v, (uint32_t)nb); }
    // heap bytes [off, off + len): 16 at a time from one 16-byte load (4-byte aligned; a load
    // straddling the heap's end reads per dword, bytes past it as 0 and never used), appended 8
    // at a time
    __device__ __forceinline__ void heap(const uint8_t *h, uint64_t hlen, uint32_t off, uint32_t len) {
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(h, hlen);
        uint32_t i = 0;
        while (i < len) {
            const uint32_t a = (off + i) & ~3u;
            uint64_t lo, hi;
            if ((uint64_t)a + 16 <= hlen) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0);
                lo = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
                hi = (uint64_t)q[2] | ((uint64_t)q[3] << 32);
            } else {
                lo = (uint64_t)buf_ld32(r, a, hlen) | ((uint64_t)buf_ld32(r, a + 4, hlen) << 32);
                hi = (uint64_t)buf_ld32(r, a + 8, hlen) | ((uint64_t)buf_ld32(r, a + 12, hlen) << 32);
            }
            const uint32_t q = off + i - a; // 0..3: bytes [q, 16) of (lo, hi) are heap bytes
            const uint32_t n1 = min(8u, len - i);
            put_n((lo >> (8 * q)) | (q ? hi << (64 - 8 * q) : 0ull), n1);
            i += n1;
            if (i < len) {
                const uint32_t n2 = min(8u - q, len - i); // the rest of the 16 loaded bytes
                put_n(hi >> (8 * q), n2);
                i += n2;
            }
        }
    }
};

// ---- schema-specialised writer pieces (jit.cpp generate_tree: spec_tree_write_<t>) ---------

// A scalar column element of constant kind K as raw bits (v[0..3]; string/bytes/any: the span)
template <uint32_t K>
__device__ __forceinline__ void load_value_k(const void *col, uint64_t row, uint64_t (&v)[4]) {
    const uint8_t *c = (const uint8_t *)col;
    v[1] = v[2] = v[3] = 0;
    if constexpr (K == K_BOOL || K == K_BYTE) v[0] = c[row];
    else if constexpr (K == K_INT16 || K == K_UINT16) v[0] = ((const uint16_t *)c)[row];
    else if constexpr (K == K_INT32 || K == K_UINT32 || K == K_FLOAT32) v[0] = ((const uint32_t *)c)[row];
    else if constexpr (K == K_BIN128) {
        const ulonglong2 q = ((const ulonglong2 *)c)[row];
        v[0] = q.x;
        v[1] = q.y;
    } else if constexpr (K == K_BIN256) {
        const ulonglong2 q0 = ((const ulonglong2 *)c)[2 * row], q1 = ((const ulonglong2 *)c)[2 * row + 1];
        v[0] = q0.x;
        v[1] = q0.y;
        v[2] = q1.x;
        v[3] = q1.y;
    } else v[0] = ((const uint64_t *)c)[row]; // 64-bit kinds, string/bytes/any spans
}

// The element through its encoder (internal/encode/...), as emit_value; string/bytes from heap h
template <uint32_t K, class E>
__device__ __forceinline__ void emit_value_k(E &em, const uint64_t (&v)[4], const uint8_t *h, uint64_t hlen) {
    if constexpr (K == K_BOOL) em.put1(v[0] ? T_TRUE : T_FALSE);
    else if constexpr (K == K_BYTE) em.put_n(v[0] | ((uint64_t)T_BYTE << 8), 2);
    else if constexpr (K == K_INT16) { em.rvarint(zigzag32((int16_t)v[0])); em.put1(T_INT16); }
    else if constexpr (K == K_INT32) { em.rvarint(zigzag32((int32_t)v[0])); em.put1(T_INT32); }
    else if constexpr (K == K_INT64) { em.rvarint(zigzag64((int64_t)v[0])); em.put1(T_INT64); }
    else if constexpr (K == K_UINT16 || K == K_UINT32 || K == K_UINT64) {
        em.rvarint(v[0]);
        em.put1(K == K_UINT16 ? T_UINT16 : K == K_UINT32 ? T_UINT32 : T_UINT64);
    } else if constexpr (K == K_FLOAT32) em.put_n(bswap32((uint32_t)v[0]) | ((uint64_t)T_FLOAT32 << 32), 5);
    else if constexpr (K == K_FLOAT64) { em.be(v[0], 8); em.put1(T_FLOAT64); }
    else if constexpr (K == K_BIN64) { em.le(v[0], 8); em.put1(T_BIN64); }
    else if constexpr (K == K_BIN128) { em.le(v[0], 8); em.le(v[1], 8); em.put1(T_BIN128); }
    else if constexpr (K == K_BIN256) {
        em.le(v[0], 8);
        em.le(v[1], 8);
        em.le(v[2], 8);
        em.le(v[3], 8);
        em.put1(T_BIN256);
    } else if constexpr (K == K_STRING || K == K_BYTES) {
        const uint32_t off = (uint32_t)v[0], len = (uint32_t)(v[0] >> 32);
        em.heap(h, hlen, off, len);
        if constexpr (K == K_STRING) em.put1(0);
        em.rvarint(len);
        em.put1(K == K_STRING ? T_STRING : T_BYTES);
    } else if constexpr (K == K_ANY) {
        em.heap(h, hlen, (uint32_t)v[0], (uint32_t)(v[0] >> 32));
    }
}

// One column element through its encoder (internal/encode/...)
template <class E>
__device__ __forceinline__ void emit_value(E &em, const TreeBufs &B, const TreeDesc &D, int c, uint32_t kind,
                                           uint64_t row) {
    const uint8_t *p = cell(B, D, c, row);
    switch (kind) {
    case K_BOOL: em.put1(p[0] ? T_TRUE : T_FALSE); break;
    case K_BYTE: em.put1(p[0]); em.put1(T_BYTE); break;
    case K_INT16: em.rvarint(zigzag32(*(const int16_t *)p)); em.put1(T_INT16); break;
    case K_INT32: em.rvarint(zigzag32(*(const int32_t *)p)); em.put1(T_INT32); break;
    case K_INT64: em.rvarint(zigzag64(*(const int64_t *)p)); em.put1(T_INT64); break;
    case K_UINT16: em.rvarint(*(const uint16_t *)p); em.put1(T_UINT16); break;
    case K_UINT32: em.rvarint(*(const uint32_t *)p); em.put1(T_UINT32); break;
    case K_UINT64: em.rvarint(*(const uint64_t *)p); em.put1(T_UINT64); break;
    case K_FLOAT32: em.be(*(const uint32_t *)p, 4); em.put1(T_FLOAT32); break;
    case K_FLOAT64: em.be(*(const uint64_t *)p, 8); em.put1(T_FLOAT64); break;
    case K_BIN64: em.le(*(const uint64_t *)p, 8); em.put1(T_BIN64); break;
    case K_BIN128:
        em.le(((const uint64_t *)p)[0], 8);
        em.le(((const uint64_t *)p)[1], 8);
        em.put1(T_BIN128);
        break;
    case K_BIN256:
        for (int i = 0; i < 4; i++) em.le(((const uint64_t *)p)[i], 8);
        em.put1(T_BIN256);
        break;
    case K_STRING:
    case K_BYTES: {
        const uint2 sp = *(const uint2 *)p;
        em.heap(B.heaps[c], B.heap_lens[c], sp.x, sp.y);
        if (kind == K_STRING) em.put1(0);
        em.rvarint(sp.y);
        em.put1(kind == K_STRING ? T_STRING : T_BYTES);
        break;
    }
    case K_ANY: {
        const uint2 sp = *(const uint2 *)p;
        em.heap(B.heaps[c], B.heap_lens[c], sp.x, sp.y);
        break;
    }
    }
}

template <class E>
__device__ __forceinline__ void emit_struct(E &em, const TreeBufs &B, const TreeDesc &D, uint32_t sf, uint64_t row) {
    const TField &F = D.f[sf];
    if (!F.nested) {
        const uint64_t start = em.pos;
        for (uint32_t k = 0; k < F.nmem; k++) {
            const TField &M = D.f[D.members[F.mem0 + k]];
            emit_value(em, B, D, M.col, M.kind, row);
        }
        em.rvarint(em.pos - start); // EncodeStruct: rvarint(dataSize) | TypeStruct
        em.put1(T_STRUCT);
        return;
    }
    // members in declaration order; an inner struct is its own EncodeXxxTo (members, then
    // EncodeStruct) in place
    uint64_t st[TREE_MAX_SD];
    uint16_t endi[TREE_MAX_SD];
    int d = 0;
    st[0] = em.pos;
    endi[0] = F.send;
    for (uint32_t i = sf + 1; i < F.send; i++) {
        while (d > 0 && i >= endi[d]) {
            em.rvarint(em.pos - st[d]);
            em.put1(T_STRUCT);
            d--;
        }
        const TField &M = D.f[i];
        if (M.kind == K_STRUCT) {
            d++;
            st[d] = em.pos;
            endi[d] = M.send;
        } else {
            emit_value(em, B, D, M.col, M.kind, row);
        }
    }
    for (; d >= 0; d--) {
        em.rvarint(em.pos - st[d]);
        em.put1(T_STRUCT);
    }
}

// list_size's total over elements [j0, j1) of list table y (its BEGIN range, already read): the
// elements' sizes loaded 8 at a time (one round of loads for a short list)
__device__ __forceinline__ uint64_t list_total(const TreeBufs &B, uint32_t y, uint32_t j0, uint32_t j1, bool &err) {
    if (j1 < j0 || (uint64_t)j1 > B.rows[y]) { // (list_span's check)
        err = true;
        j1 = j0;
    }
    const uint32_t *sz = B.size[y];
    uint64_t data = 0;
    for (uint32_t j = j0; j < j1; j += 8) {
        uint32_t s[8];
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) s[i] = j + i < j1 ? sz[j + i] : 0u;
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) data += s[i];
    }
    const uint32_t count = j1 - j0;
    const bool big = count > 255 || (count > 0 && data > 65535);
    const uint64_t tsize = (uint64_t)count * (big ? 4 : 2);
    if (data > MAX_SIZE) err = true;
    return data + tsize + vlen64(data) + vlen64(tsize) + 1;
}

// A present list field's bytes (EncodeListTable, internal/encode/list.go:15-75) over elements
// [j0, j1) of list table y: the elements' gaps (their rows' positions), the offset table
// (IsBigList: count > 255 or data > 65535), the trailer.  Up to 8 elements take one round of size
// loads (issued together, kept in registers for the table); longer lists loop 4 at a time.
template <class E>
__device__ __forceinline__ void emit_list(E &em, const TreeBufs &B, uint32_t y, uint32_t j0, uint32_t j1) {
    const uint32_t *sz = B.size[y];
    uint64_t *pos = B.pos[y];
    const uint32_t cnt = j1 - j0;
    if (cnt <= 8) {
        uint32_t s[8];
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) s[i] = i < cnt ? sz[j0 + i] : 0u;
        uint64_t p = em.pos;
#pragma unroll
        for (uint32_t i = 0; i < 8; i++)
            if (i < cnt) {
                pos[j0 + i] = p;
                p += s[i];
            }
        const uint64_t data = p - em.pos;
        em.skip(data);
        const bool big = data > 65535;
        uint64_t off = 0;
#pragma unroll
        for (uint32_t i = 0; i < 8; i++)
            if (i < cnt) {
                off += s[i];
                em.be(off, big ? 4 : 2);
            }
        em.rvarint(data);
        em.rvarint((uint64_t)cnt * (big ? 4 : 2));
        em.put1(big ? T_BIG_LIST : T_LIST);
        return;
    }
    uint64_t data = 0;
    for (uint32_t j = j0; j < j1; j += 4) {
        uint32_t s[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) s[i] = j + i < j1 ? sz[j + i] : 0u;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++)
            if (j + i < j1) {
                pos[j + i] = em.pos + data;
                data += s[i];
            }
    }
    em.skip(data);
    const bool big = cnt > 255 || data > 65535;
    uint64_t off = 0;
    for (uint32_t j = j0; j < j1; j += 4) {
        uint32_t s[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) s[i] = j + i < j1 ? sz[j + i] : 0u;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++)
            if (j + i < j1) {
                off += s[i];
                em.be(off, big ? 4 : 2);
            }
    }
    em.rvarint(data);
    em.rvarint((uint64_t)cnt * (big ? 4 : 2));
    em.put1(big ? T_BIG_LIST : T_LIST);
}

// ---- level-fused encode launches (jit.cpp spec_tree_size_set / spec_tree_write_set) ---------
// Tables with no size dependency between them (the same height: every child sized first) are
// sized in ONE launch, tables at the same depth (every owner written first) written in one:
// blockIdx.y picks the table of the set, the blocks stride over its rows.
struct TableSet {
    uint32_t n;
    uint32_t t[TREE_MAX_T];
};

// the size of row `row` of a VALUE or STRUCT table (tree.hip tree_size_kernel's run-time rules)
__device__ __forceinline__ uint64_t size_row_shaped(const TreeDesc &D, const TreeBufs &B, uint32_t x, uint64_t row,
                                                    bool &err) {
    const TTable &T = D.t[x];
    if (T.shape == SHAPE_VALUE) {
        const TField &F = D.f[T.field];
        return value_size(B, D, F.col, F.elem, row, err);
    }
    return struct_size(B, D, T.field, row, err);
}

// A list table's rows its owners' BEGIN ranges cover: [begin[0], begin[owner rows]) (the writers
// check BEGIN is monotonic: an encoder error otherwise).  Rows outside belong to no owner and are
// not written (a message row outside marks its own children unplaced, jit.cpp gen_unplace_*);
// every row inside gets its position (or ~0: an absent / unplaced owner) from its owner's write,
// so the level-fused writers need no position fill first.
__device__ __forceinline__ bool list_row_covered(const TreeDesc &D, const TreeBufs &B, uint32_t y, uint64_t row) {
    const uint32_t *b = (const uint32_t *)B.cols[D.t[y].begin_col];
    return row >= b[0] && row < b[B.rows[D.t[y].parent]];
}

// the bytes of row `row` of a VALUE or STRUCT table (a list element) through emitter em
template <class E>
__device__ __forceinline__ void emit_row_shaped(E &em, const TreeDesc &D, const TreeBufs &B, uint32_t x, uint64_t row) {
    const TTable &T = D.t[x];
    if (T.shape == SHAPE_VALUE) {
        const TField &F = D.f[T.field];
        emit_value(em, B, D, F.col, F.elem, row);
    } else {
        emit_struct(em, B, D, T.field, row);
    }
    em.finish();
}

// the bytes of row `row` of a VALUE or STRUCT table (list elements) at its position
// (tree_write_kernel's rules)
__device__ __forceinline__ void write_row_shaped(const TreeDesc &D, const TreeBufs &B, uint32_t x, uint64_t row) {
    if (!list_row_covered(D, B, x, row)) return;
    const uint64_t start = B.pos[x][row];
    if (start == ~0ull) return; // a row no written owner placed
    BEmit em{{B.out}, start, start};
    emit_row_shaped(em, D, B, x, row);
}

// ---- the record-tile writer (jit.cpp gen_tile: spec_tree_write_tile) ------------------------
// One workgroup writes 64 consecutive records with every row under them, depth by depth, into an
// LDS image of their output range, then stores the image once with 16-byte stores.  The bytes of
// a range longer than the image past its first cap bytes go straight to HBM (LSink).
struct MkL { // emitters over the LDS image of the window [sh, sh + cap), HBM past it
    TileU8 *img;
    uint8_t *out;
    uint64_t sh;
    uint32_t cap;
    __device__ __forceinline__ LEmit operator()(uint64_t p) const { return LEmit{{img, out, sh + cap, (uint32_t)sh}, p, p}; }
};

// zeroes the image's first `len` bytes (SPEC_TILE_OR: the rows OR their dwords into it)
__device__ __forceinline__ void tile_clear(TileU8 *img, uint32_t len) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    for (uint32_t a = threadIdx.x * 16u; a < len; a += blockDim.x * 16u) *(__attribute__((address_space(3))) v4u *)(img + a) = v4u{0, 0, 0, 0};
}

// out[org, fin) from the image (out byte p at img[p - sh]; out + sh is 16-byte aligned): whole
// chunks with 16-byte stores, the partial chunks at the ends bytewise (the neighbours' bytes)
__device__ __forceinline__ void tile_copy_out(uint8_t *out, const TileU8 *img, uint64_t sh, uint64_t org, uint64_t fin) {
    const uint32_t q0 = (uint32_t)(org - sh), q1 = (uint32_t)(fin - sh);
    uint8_t *o = out + sh;
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const v4u lds_v4u;
    for (uint32_t a = threadIdx.x * 16u; a < q1; a += blockDim.x * 16u) {
        if (a >= q0 && a + 16 <= q1) {
            *(v4u *)(o + a) = *(lds_v4u *)(img + a);
        } else {
            const uint32_t b1 = a + 16 < q1 ? a + 16 : q1;
            for (uint32_t b = a > q0 ? a : q0; b < b1; b++) o[b] = img[b];
        }
    }
}

} // namespace spec
