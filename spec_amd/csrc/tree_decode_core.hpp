// tree_decode_core.hpp — device code of the schema-tree decoder (tree_decode.hip), shared by the
// precompiled run-time-schema group kernel and the schema-specialised group kernels jit.cpp
// compiles with hiprtc (the generated readers of internal/lang/generator/message.go:97-186 with
// their tags, kinds and columns as constants).
//
// A wave's 64 rows are staged in LDS before they are parsed: the rows' whole span with LDS-DMA
// when it fits the wave's slab (consecutive records; the elements of neighbouring lists), else
// each row in its own lane window (small rows far apart), else the rows parse from HBM through
// range-checked loads.
#pragma once

#include "tree_core.hpp"

namespace spec {

constexpr int LANE_W = 256;          // bytes of a lane's window (lane staging)
constexpr int LANE_CHUNKS = LANE_W / 16;
constexpr int GUARD = 64;            // bytes staged below a row (value windows read below its start)

// Staged stream bytes [off, off + size) at lds: reads are clamped into the window (every read
// of a row's parse lies in [lo - 64, hi + 16), which the staging covers).
struct TreeLds {
    using pos_t = long long;
    lds_u8 *lds;
    long long off;
    int size;
    // 32-bit window offset (the stream is < 4 GiB): a position below the window wraps to a huge
    // value and, like one past it, is clamped to the window's last n bytes (only reads the
    // decoders mask out go outside [lo - 64, hi + 16))
    __device__ __forceinline__ int at(long long p, int n) const {
        const uint32_t i = (uint32_t)p - (uint32_t)off;
        const uint32_t lim = (uint32_t)(size - n);
        return (int)(i < lim ? i : lim);
    }
    __device__ __forceinline__ uint32_t u8(long long p) const { return lds[at(p, 1)]; }
    __device__ __forceinline__ uint64_t d64(long long p) const {
        int i = at(p, 8);
        asm("" : "+v"(i)); // one ds_read_b64 per qword (LdsSrc::d64)
        return *(lds_u64 *)(lds + i);
    }
    __device__ __forceinline__ uint32_t d32(long long p) const { return *(lds_u32 *)(lds + at(p, 4)); }
};

__device__ __forceinline__ void tree_wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Rows of table x during a decode: the records (n) or a list table's device-counted rows,
// capped by its capacity (a sub-message table has its owner's rows).
__device__ __forceinline__ uint64_t dec_rows(const TreeDesc &D, const TreeBufs &B, uint32_t x) {
    const uint32_t g = D.t[x].groot;
    if (g == 0) return B.n;
    const uint64_t r = B.rowsd[g];
    return r < B.caps[g] ? r : B.caps[g];
}

// Every wave of the grid over the rows of group root x, 64 at a time: for its valid rows
// lds_body(src, row, lo, hi, panic) with src = the staged bytes (TreeLds), or glob_body(...) with
// src = HBM (GlobalSrc) when the rows fit neither staging.  Each body has one call site, so a
// specialised row body is inlined once.
// rpw = rows per wave, 64 or 32: with 32 the wave's lanes 32..63 idle and its slab holds half
// the span, so twice the waves share a CU's LDS (rows too large for 64 per slab at good occupancy).
template <class LdsBody, class GlobBody>
__device__ __forceinline__ void tree_rows(const TreeBufs &B, uint32_t x, uint64_t rows, uint32_t slab_bytes,
                                          uint32_t wave_bytes, uint32_t rpw, LdsBody lds_body, GlobBody glob_body) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint8_t *slab = smem + wave * wave_bytes;
    const __amdgpu_buffer_rsrc_t rsrc = stream_rsrc(B);
    const GlobalSrc gs{B.stream, B.stream_len};
    const uint64_t wpb = blockDim.x >> 6; // (fewer than TB / 64 waves when the range slots are large)
    const uint64_t wstride = (uint64_t)gridDim.x * wpb * rpw;
    for (uint64_t base = ((uint64_t)blockIdx.x * wpb + wave) * rpw; base < rows; base += wstride) {
        const uint64_t row = base + lane;
        const bool valid = row < rows && (uint32_t)lane < rpw;
        long long lo = 0, hi = 0;
        bool panic = false;
        if (valid) row_range(B, x, row, lo, hi, panic);
        const bool some = valid && hi > lo;
        long long slo = some ? lo : (long long)B.stream_len, shi = some ? hi : 0, len = some ? hi - lo : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const long long a = __shfl_xor(slo, d), b2 = __shfl_xor(shi, d), l2 = __shfl_xor(len, d);
            slo = a < slo ? a : slo;
            shi = b2 > shi ? b2 : shi;
            len = l2 > len ? l2 : len;
        }
        slo = (long long)uniform64((uint64_t)slo);
        shi = (long long)uniform64((uint64_t)shi);
        len = (long long)uniform64((uint64_t)len);
        const long long sb = (slo > GUARD ? slo - GUARD : 0) & ~15ll, se = (shi + 16 + 15) & ~15ll;
        const bool span = slab_bytes && slo < shi && se - sb + 16 <= (long long)slab_bytes;
        const bool lanes = !span && slab_bytes >= 64 * LANE_W && len + GUARD + 48 <= LANE_W;
        if (span) {
            // the span: LDS-DMA, 1 KiB per instruction, all in flight at once
            const uint32_t chunks = (uint32_t)((se - sb + 1023) >> 10);
            for (uint32_t c = 0; c < chunks; c++)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(slab + c * 1024),
                                                         16, (uint32_t)sb + c * 1024 + lane * 16, 0, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // a 16-byte chunk straddling the stream end comes back zeroed: refill it bytewise
            const uint64_t tail = B.stream_len & ~15ull;
            if (tail < B.stream_len && (long long)tail >= sb && (long long)tail < sb + (long long)chunks * 1024 &&
                lane < 16 && tail + lane < B.stream_len)
                slab[tail - sb + lane] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (uint32_t)(tail + lane), 0, 0);
        } else if (lanes) {
            // each row in its lane's window: its 16-byte chunks, all loads issued before the stores
            uint8_t *win = slab + lane * LANE_W;
            const long long lb = (lo > GUARD ? lo - GUARD : 0) & ~15ll;
            const int nch = some ? (int)((((hi + 16 + 15) & ~15ll) - lb) >> 4) : 0;
            uint4 v[LANE_CHUNKS];
#pragma unroll
            for (int c = 0; c < LANE_CHUNKS; c++) {
                const long long p = lb + 16ll * c;
                if (c < nch) {
                    if ((uint64_t)p + 16 <= B.stream_len) {
                        const auto q = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (uint32_t)p, 0, 0);
                        v[c] = make_uint4(q[0], q[1], q[2], q[3]);
                    } else {
                        v[c] = make_uint4(gs.d32(p), gs.d32(p + 4), gs.d32(p + 8), gs.d32(p + 12));
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < LANE_CHUNKS; c++)
                if (c < nch) *(uint4 *)(win + 16 * c) = v[c];
        }
        if (span || lanes) {
            tree_wave_fence();
            const long long off = span ? sb : ((lo > GUARD ? lo - GUARD : 0) & ~15ll);
            if (valid)
                lds_body(TreeLds{(lds_u8 *)(span ? slab : slab + lane * LANE_W), off, span ? (int)slab_bytes : LANE_W}, row,
                         lo, hi, panic);
        } else if (valid) {
            glob_body(gs, row, lo, hi, panic);
        }
        tree_wave_fence(); // the staged bytes are read before the next rows overwrite them
    }
}

// The root table's outcome on one wave of a wave group (tree_rows_pair): its status, whether
// the table took the specialised path, and the *Err bits of the fields that wave decoded.
struct RowOut {
    uint64_t errs;
    uint32_t st, fast;
};

// tree_rows for a group of P waves (a 64 P-thread block): every wave takes the same 64 rows,
// staged ONCE in the block's slab (the waves issue the LDS-DMA chunks round-robin), and decodes
// its share of the group's fields (jit.cpp gen_pair_rows); waves 1..P-1 then hand their RowOut
// to wave 0 through LDS (xch, 64 entries each) and fin(row, panic, ro0, ro_rest) stores the root
// table's status and *Err mask (ro_rest: the others' bits ORed, ST_PANIC if any panicked).
// P waves per 64 rows at the same LDS per row: a SIMD holds P waves, so one's LDS round trips
// overlap the others' decode.  Rows whose span exceeds the slab parse from HBM (the lane windows
// of tree_rows are not used here).
template <int P, class LdsBody, class GlobBody, class Fin>
__device__ __forceinline__ void tree_rows_pair(const TreeBufs &B, uint32_t x, uint64_t rows, uint32_t slab_bytes,
                                               uint4 *xch, LdsBody lds_body, GlobBody glob_body, Fin fin) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint8_t *slab = smem;
    const __amdgpu_buffer_rsrc_t rsrc = stream_rsrc(B);
    const GlobalSrc gs{B.stream, B.stream_len};
    for (uint64_t base = (uint64_t)blockIdx.x * 64; base < rows; base += (uint64_t)gridDim.x * 64) {
        const uint64_t row = base + lane;
        const bool valid = row < rows;
        long long lo = 0, hi = 0;
        bool panic = false;
        if (valid) row_range(B, x, row, lo, hi, panic);
        const bool some = valid && hi > lo;
        long long slo = some ? lo : (long long)B.stream_len, shi = some ? hi : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const long long a = __shfl_xor(slo, d), b2 = __shfl_xor(shi, d);
            slo = a < slo ? a : slo;
            shi = b2 > shi ? b2 : shi;
        }
        slo = (long long)uniform64((uint64_t)slo);
        shi = (long long)uniform64((uint64_t)shi);
        const long long sb = (slo > GUARD ? slo - GUARD : 0) & ~15ll, se = (shi + 16 + 15) & ~15ll;
        const bool span = slab_bytes && slo < shi && se - sb + 16 <= (long long)slab_bytes;
        if (span) {
            const uint32_t chunks = (uint32_t)((se - sb + 1023) >> 10);
            for (uint32_t c = (uint32_t)wave; c < chunks; c += P)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(slab + c * 1024),
                                                         16, (uint32_t)sb + c * 1024 + lane * 16, 0, 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // the straddling chunk is refilled by the wave that loaded it (after its own DMA landed)
            const uint64_t tail = B.stream_len & ~15ull;
            if (tail < B.stream_len && (long long)tail >= sb && (long long)tail < sb + (long long)chunks * 1024 &&
                (int)(((tail - sb) >> 10) % P) == wave && lane < 16 && tail + lane < B.stream_len)
                slab[tail - sb + lane] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (uint32_t)(tail + lane), 0, 0);
        }
        __syncthreads(); // the slab is whole; the previous rows' exchange has been read
        RowOut ro = {0, 0, 0};
        if (valid) {
            if (span)
                lds_body(TreeLds{(lds_u8 *)slab, sb, (int)slab_bytes}, row, lo, hi, ro);
            else
                glob_body(gs, row, lo, hi, ro);
        }
        if (wave) xch[(wave - 1) * 64 + lane] = make_uint4((uint32_t)ro.errs, (uint32_t)(ro.errs >> 32), ro.st, ro.fast);
        __syncthreads(); // the others' outcomes are in xch; every wave is done with the slab
        if (wave == 0 && valid) {
            RowOut r = {0, 0, 0};
#pragma unroll
            for (int w = 1; w < P; w++) {
                const uint4 q = xch[(w - 1) * 64 + lane];
                r.errs |= (uint64_t)q.x | ((uint64_t)q.y << 32);
                r.st = q.z == ST_PANIC ? (uint32_t)ST_PANIC : r.st;
            }
            fin(row, panic, ro, r);
        }
    }
}

// tree_rows without staging (slab 0): every row parsed from HBM.  A kernel of its own, so its
// register budget is the row code's alone (the staging paths' 16-chunk lane windows would
// otherwise set it) and the CU holds as many waves as the latency of the reads needs.
template <class GlobBody>
__device__ __forceinline__ void tree_rows_global(const TreeBufs &B, uint32_t x, uint64_t rows, GlobBody glob_body) {
    const GlobalSrc gs{B.stream, B.stream_len};
    for (uint64_t row = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; row < rows; row += (uint64_t)gridDim.x * blockDim.x) {
        long long lo = 0, hi = 0;
        bool panic = false;
        row_range(B, x, row, lo, hi, panic);
        glob_body(gs, row, lo, hi, panic);
    }
}

// ---- the run-time-schema row code ------------------------------------------------------------

template <class Src>
__device__ __forceinline__ bool tree_scalar(const Src &s, uint32_t kind, long long ds, long long end, void *col,
                                            uint64_t row, bool want_err) {
    if (!col && !want_err) return true;
    Val v;
    int n;
    const bool ok = decode_value_n(s, kind, ds, end >= 0 ? ds + end : ds, 0, v, n); // m.<Kind>(tag)
    store_kind(col, row, kind, v);
    return ok;
}

// A message row of table t over [lo, hi): OpenMessageErr, every direct field's getter into its
// column, *Err bits, and for its children: sub-message ranges (into the group's LDS range
// slots), list counts + list table positions (for the scan).  Returns the row's status.
// Out of line, once per source: the generic row code is large (every kind's decoder), and one
// copy per call site overflowed the instruction cache (98K instructions: the waves of one
// kernel executing different fields' code missed it constantly).
template <class Src>
__device__ __forceinline__ uint32_t tree_message_row_inl(const Src &s, const TreeDesc &D, const TreeBufs &B, uint32_t t,
                                                         uint64_t row, long long lo, long long hi, uint2 *gr) {
    const TTable &T = D.t[t];
    const RecInfo ri = rec_open(s, lo, hi); // empty (or panicked) range => empty message
    uint32_t st = ri.tr.st;
    const long long ds = ri.tr.dstart;
    // ERRMASK: W words per row (a bit per direct field), each stored once its 64 fields are done
    // (the index pass runs with no columns: a null column stays null, not null + row * W)
    uint64_t *const ecol = T.err_col >= 0 ? (uint64_t *)B.cols[T.err_col] : nullptr;
    uint64_t *errp = ecol ? ecol + row * ((uint32_t)D.width[T.err_col] / 8) : nullptr;
    uint64_t errs = 0;
    for (uint32_t k = 0; k < T.nd; k++) {
        const uint32_t fi = D.direct[T.d0 + k];
        const TField &F = D.f[fi];
        const long long end = rec_field_end(s, ri, F.tag, F.rank);
        const long long e = end >= 0 ? ds + end : ds;
        bool bad = false; // the field's *Err getter errs
        switch (F.kind) {
        case K_MESSAGE: {
            store_u8(B.cols[F.present], row, end >= 0 ? 1u : 0u);
            // its table decodes next in this group, over m.field(tag) (Message(tag), msg.go:447-451)
            gr[D.t[F.table].gslot * 64] = end >= 0 ? make_uint2((uint32_t)ds, (uint32_t)e) : make_uint2(0, 0);
            if (errp && e > ds) bad = parse_trailer<false>(s, ds, e).st != ST_OK; // MessageErr
            break;
        }
        case K_LIST: {
            store_u8(B.cols[F.present], row, end >= 0 ? 1u : 0u);
            // OpenList(m.field(tag)): errors => an empty list (internal/types/list.go:22-25)
            ListInfo li = {0, 0, 0, 0, false};
            if (e > ds) {
                const Trailer lt = parse_trailer<true>(s, ds, e);
                if (lt.st == ST_OK) {
                    li.big = lt.big;
                    li.count = lt.tsize / (lt.big ? 4u : 2u);
                    li.dstart = lt.dstart;
                    li.tstart = lt.tstart;
                    li.dsize = lt.dsize;
                } else {
                    bad = true; // ListErr
                }
            }
            B.cnt[F.table][row] = li.count;
            B.lh[F.table][row] = make_uint4((uint32_t)li.tstart, (uint32_t)li.dstart, li.dsize,
                                            li.count | (li.big ? 0x80000000u : 0u));
            break;
        }
        case K_STRUCT: {
            const uint32_t sst = tree_struct(s, D, B, fi, ds, e, row, 0);
            if (sst == ST_PANIC) st = ST_PANIC;
            bad = sst != ST_OK;
            break;
        }
        case K_ANY: {
            // Field(tag) = OpenValue(bytes[:end]): nil on error or len < n; n < 0 panics
            long long n = 0;
            uint2 sp = make_uint2(0, 0);
            if (e > ds) {
                if (type_size(s, ds, e, n)) {
                    if (n < 0) st = ST_PANIC;
                    else if (n > 0 && n <= e - ds) sp = make_uint2((uint32_t)(e - n), (uint32_t)n);
                } else {
                    bad = true; // OpenValueErr: DecodeTypeSize's error
                }
            }
            if (B.cols[F.col]) ((uint2 *)B.cols[F.col])[row] = sp;
            // Value.Type(): the value's last byte (DecodeType), 0 for a nil value
            store_u8(B.cols[F.present], row, sp.y ? s.u8((long long)sp.x + sp.y - 1) : 0u);
            break;
        }
        default:
            bad = !tree_scalar(s, F.kind, ds, end, B.cols[F.col], row, errp != nullptr);
        }
        if (bad) errs |= 1ull << (k & 63);
        if ((k & 63) == 63 && k + 1 < T.nd) {
            if (errp) errp[k >> 6] = errs;
            errs = 0;
        }
    }
    if (errp) errp[T.nd ? (T.nd - 1) >> 6 : 0] = errs;
    return st;
}

template <class Src>
__device__ __noinline__ uint32_t tree_message_row(const Src &s, const TreeDesc &D, const TreeBufs &B, uint32_t t,
                                                  uint64_t row, long long lo, long long hi, uint2 *gr) {
    return tree_message_row_inl(s, D, B, t, row, lo, hi, gr);
}

// The schema-specialised rows' fallback for a table the fast path rejects: out of line when the
// row is parsed from LDS (the kernel's register budget is set by its staging code anyway), inline
// when it is parsed from HBM (a call's register saves would set the no-staging kernel's budget).
// the run-time path of a wave-group kernel (gen_pair_rows): out of line from either source, one
// instance per group size Tag, so the kernel's register budget (amdgpu_waves_per_eu) reaches it
template <int Tag, class Src>
__device__ __noinline__ uint32_t tree_message_fallback_p(const Src &s, const TreeDesc &D, const TreeBufs &B, uint32_t t,
                                                         uint64_t row, long long lo, long long hi, uint2 *gr) {
    return tree_message_row_inl(s, D, B, t, row, lo, hi, gr);
}
__device__ __forceinline__ uint32_t tree_message_fallback(const TreeLds &s, const TreeDesc &D, const TreeBufs &B,
                                                          uint32_t t, uint64_t row, long long lo, long long hi,
                                                          uint2 *gr) {
    return tree_message_row(s, D, B, t, row, lo, hi, gr);
}
__device__ __forceinline__ uint32_t tree_message_fallback(const GlobalSrc &s, const TreeDesc &D, const TreeBufs &B,
                                                          uint32_t t, uint64_t row, long long lo, long long hi,
                                                          uint2 *gr) {
    return tree_message_row_inl(s, D, B, t, row, lo, hi, gr);
}

// One row of group root x (run-time schema): the root table's row, then the group's
// sub-message tables, each over the range its owner found.
template <class Src>
__device__ __forceinline__ void tree_group_row(const Src &s, const TreeDesc &D, const TreeBufs &B, uint32_t x,
                                               uint64_t row, long long lo, long long hi, bool panic, uint2 *gr) {
    const TTable &T = D.t[x];
    uint32_t st;
    if (T.shape == SHAPE_VALUE) {
        const TField &F = D.f[T.field];
        Val v;
        int n;
        const bool ok = decode_value_n(s, F.elem, lo, hi, 0, v, n);
        store_kind(B.cols[F.col], row, F.elem, v);
        st = panic ? ST_PANIC : (ok ? ST_OK : ST_INVALID_VALUE);
        store_u8(B.cols[T.status_col], row, st);
        return;
    }
    if (T.shape == SHAPE_STRUCT) {
        st = tree_struct(s, D, B, T.field, lo, hi, row, 0);
        store_u8(B.cols[T.status_col], row, panic ? ST_PANIC : st);
        return;
    }
    st = tree_message_row(s, D, B, x, row, lo, hi, gr);
    store_u8(B.cols[T.status_col], row, panic ? ST_PANIC : st);
    for (uint32_t g = 1; g < T.gn; g++) {
        const uint32_t y = D.group[T.g0 + g];
        const uint2 r = gr[D.t[y].gslot * 64];
        const uint32_t sy = tree_message_row(s, D, B, y, row, (long long)r.x, (long long)r.y, gr);
        store_u8(B.cols[D.t[y].status_col], row, sy);
    }
}

// ---- pieces of the schema-specialised row code (jit.cpp generates the rest) -----------------

// OpenMessageErr of a row whose schema is known: the trailer, then the table's tags checked
// against the schema's tag set (M0..M3: a 256-bit mask of its tags, all <= 255).  fast = the
// table is small, strictly increasing and holds schema tags only: then the reference's binary
// search for a schema tag finds the entry at index popcount(P below its rank) (P bit r = the
// field of rank r is present), so every lookup is one table read.  Otherwise the row takes the
// run-time path (tree_message_row), which restates the search itself.
struct TOpen {
    uint32_t st;      // DecodeMessageTable's status (ST_OK for an empty range)
    bool fast;
    long long ds, ts; // data start, table start (0 when the row is empty or invalid)
    uint32_t dsize;
    uint64_t P;
};

template <uint64_t M0, uint64_t M1, uint64_t M2, uint64_t M3>
__device__ __forceinline__ uint32_t tag_rank(uint32_t t, bool &in) {
    const uint32_t w = t >> 6, b = t & 63;
    const uint64_t m = w == 0 ? M0 : w == 1 ? M1 : w == 2 ? M2 : M3;
    constexpr uint32_t c1 = __builtin_popcountll(M0), c2 = c1 + __builtin_popcountll(M1),
                       c3 = c2 + __builtin_popcountll(M2);
    const uint32_t before = w == 0 ? 0u : w == 1 ? c1 : w == 2 ? c2 : c3;
    in = ((m >> b) & 1) != 0;
    return before + (uint32_t)__builtin_popcountll(m & ((1ull << b) - 1));
}

template <int N, uint64_t M0, uint64_t M1, uint64_t M2, uint64_t M3, class Src>
__device__ __forceinline__ TOpen tree_open(const Src &s, long long lo, long long hi) {
    TOpen o = {ST_OK, true, 0, 0, 0, 0};
    if (hi <= lo) return o; // an empty message: every field absent
    const Trailer tr = parse_trailer(s, lo, hi);
    o.st = tr.st;
    if (tr.st != ST_OK) return o; // OpenMessageErr fails: every getter returns zero
    o.ds = tr.dstart;
    o.ts = tr.tstart;
    o.dsize = tr.dsize;
    const uint32_t nent = tr.tsize / (tr.big ? 6u : 3u);
    bool ok = !tr.big && nent <= (uint32_t)N;
    uint32_t prev = 0;
    uint64_t P = 0;
    if constexpr (N == 0) {
        o.fast = ok;
        return o;
    } else {
    // the table's first 3N bytes, re-aligned into qwords (as decode_core.hpp fast_prepare): tag i
    // is byte 3i, a compile-time position
    constexpr int NC = (3 * N + 7) / 8, NQ = NC + 1;
    const long long base = tr.tstart & ~7ll;
    const uint32_t sh = 8u * (uint32_t)(tr.tstart & 7);
    uint64_t q[NQ];
#pragma unroll
    for (int j = 0; j < NQ; j++) q[j] = s.d64(base + 8 * j);
    uint64_t c[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) c[j] = (q[j] >> sh) | ((q[j + 1] << 1) << (63 - sh));
#pragma unroll
    for (int i = 0; i < N; i++) {
        const bool use = (uint32_t)i < nent;
        const uint32_t t = (uint32_t)(c[(3 * i) >> 3] >> (8 * ((3 * i) & 7))) & 0xff;
        bool in;
        const uint32_t r = tag_rank<M0, M1, M2, M3>(t, in);
        ok = ok & (!use | (in & (i == 0 || t > prev)));
        P |= use ? (1ull << (r & 63)) : 0ull;
        prev = t;
    }
    o.fast = ok;
    o.P = P;
    return o;
    }
}

// m.field(tag) of the field of rank R: its end offset (data-relative), or -1 (absent or
// end > dataSize: nil, internal/types/msg.go:466-475)
template <int R, class Src>
__device__ __forceinline__ long long tree_end(const Src &s, const TOpen &o) {
    const bool has = ((o.P >> R) & 1) != 0;
    const uint32_t idx = (uint32_t)__builtin_popcountll(o.P & ((1ull << R) - 1));
    const long long p = o.ts + 3ll * idx;
    const long long end = (long long)((s.u8(p + 1) << 8) | s.u8(p + 2));
    return (has && end <= (long long)o.dsize) ? end : -1;
}

// m.<Kind>(tag) of a field of constant kind K into its column (nullable); returns !err
// The value's window is read for the type a Writer emits for K (decode_core.hpp load_win<K, true>:
// 8 bytes for the narrow kinds, the payload qwords for the fixed-width ones); a value of another
// accepted type (an int of another width, float32 <-> float64) takes the general decode.  For
// kinds that accept one type only the narrow window holds everything a valid value needs, and a
// value of another type fails on its type byte either way.
template <uint32_t K, class Src>
__device__ __forceinline__ bool tree_field_k(const Src &s, long long ds, long long end, void *col, uint64_t row) {
    using pos_t = typename Src::pos_t;
    Val v = {0, 0, 0, 0};
    bool ok = true;
    if (end > 0) {
        const pos_t e = (pos_t)(ds + end), lo = (pos_t)ds;
        constexpr uint32_t NT = cross_kind_type(K);
        const Win w = load_win<K, true>(s, e);
        if (NT == 0 || ((uint32_t)w.t.q0 & 0xff) == NT) v = decode_tail_k<K, true>(w, lo, e, 0, &ok);
        else v = decode_tail_k<K>(load_win<K>(s, e), lo, e, 0, &ok);
    }
    if (col) store_value_k<K>(col, row, v);
    return ok;
}

} // namespace spec
