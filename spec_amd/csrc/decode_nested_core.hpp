// decode_nested_core.hpp — device code of the list<message> decoder (BASELINE config 4),
// shared by the precompiled kernels (decode_nested.hip, run-time schema) and the
// schema-specialised one-pass kernel jit.cpp compiles with hiprtc.
//
// Per record the reference runs (generated reader, internal/lang/generator/message.go:154-162):
//   m, err := spec.OpenMessageErr(b)                       internal/types/msg.go:43-55
//   outer getters as for a flat message                     internal/types/msg.go:219-475
//   items := spec.NewMessageList(m.msg.List(tag), OpenItemErr)   list_msg.go:20-26
//     m.List(tag) = OpenList(m.field(tag))                  internal/types/msg.go:441-444 (errors => empty list)
//     items.Len() = table.Len()                             list_msg.go:67-69, internal/types/list.go:70-72
//     items.Get(i) = open(List.GetBytes(i))                 list_msg.go:88-92, internal/types/list.go:100-116
//       GetBytes: start = end(i-1) (0 for i = 0), end = end(i); end > dataSize => nil;
//       start > end panics in Go (slice bounds) => item status SPEC_STATUS_PANIC here
//     item getters on the opened item message
// Output: outer columns [n] + status; item_begin [n+1] (CSR, uint32); item columns [m] +
// item status, items in record order.
//
// A wave decodes a group of 64 consecutive records: stage the span into LDS (as the flat
// decoder), decode each outer record (one lane per record), wave prefix-sum of the item
// counts, then the group's items ITEM-PARALLEL: item j of the group goes to lane j % 64 (owner
// record found by a binary search over the lanes' prefix sums), so item columns are written
// coalesced and no lane idles on a short list.  Outer records and items take the
// schema-specialised fast path (decode_core.hpp) when the kernel has one (OSpec / ISpec), the
// generic path otherwise.
//
// Where the group's first item goes:
//   * two-pass (spec_decode_nested_index + spec_decode_nested): a count kernel and a scan
//     kernel write every group's item offset first;
//   * one pass (spec_decode_nested_onepass): groups are taken in order from an atomic ticket
//     and publish their item count, then their inclusive prefix, in a per-group state word;
//     a group finds its offset by looking back over its predecessors' words (decoupled
//     look-back: a window of 64 predecessors per step, one per lane).
#pragma once

#include "decode_core.hpp"

namespace spec {

// What OpenList(m.field(tag)) gives: count and where the table / data are (source positions).
struct ListInfo {
    uint32_t count;
    long long dstart, tstart; // list data start, table start
    uint32_t dsize;
    bool big;
};

// OpenList over the list value [lo, e) (e <= lo: absent or empty => empty list)
template <class Src>
__device__ __forceinline__ ListInfo list_at(const Src &s, typename Src::pos_t lo, typename Src::pos_t e) {
    ListInfo li = {0, 0, 0, 0, false};
    if (e <= lo) return li;
    const Trailer lt = parse_trailer<true>(s, lo, e);
    if (lt.st != ST_OK) return li; // OpenList: error => List{}
    li.big = lt.big;
    li.count = lt.tsize / (lt.big ? 4u : 2u);
    li.dstart = lt.dstart;
    li.tstart = lt.tstart;
    li.dsize = lt.dsize;
    return li;
}

template <class Src>
__device__ __forceinline__ ListInfo list_open(const Src &s, const RecInfo &ri, const NestedArgs &a) {
    const long long end = rec_field_end(s, ri, a.list_tag, a.list_rank);
    using pos_t = typename Src::pos_t;
    const pos_t lo = (pos_t)ri.tr.dstart;
    return list_at(s, lo, end <= 0 ? lo : lo + (pos_t)end);
}

template <class Src>
__device__ __forceinline__ uint32_t be16_at(const Src &s, long long p) {
    return (s.u8((typename Src::pos_t)p) << 8) | s.u8((typename Src::pos_t)p + 1);
}
template <class Src>
__device__ __forceinline__ uint32_t be32_at(const Src &s, long long p) {
    typename Src::pos_t q = (typename Src::pos_t)p;
    return (s.u8(q) << 24) | (s.u8(q + 1) << 16) | (s.u8(q + 2) << 8) | s.u8(q + 3);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

// Stage one wave's group (records [base, base+64)) into its slab: returns the group; if
// gr.in_lds the bytes are in LDS when this returns.
__device__ __forceinline__ Group nested_stage(const NestedArgs &a, __amdgpu_buffer_rsrc_t rsrc, uint8_t *slab,
                                              uint64_t base, int lane) {
    uint64_t lo, hi;
    DecodeArgs d;
    d.stream = a.stream;
    d.stream_len = a.stream_len;
    d.ends = a.ends;
    d.n = a.n;
    d.r0 = 0;
    d.head = 0;
    load_group_ends(d, base, lane, lo, hi);
    Group gr = make_group(d, base, lane, lo, hi, a.slab);
    if (gr.in_lds) {
        issue_dma(rsrc, slab, gr, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        fix_stream_tail(d, rsrc, slab, gr, lane);
    }
    return gr;
}

// Lanes [l0, l1) of the group only (a group whose whole span exceeds the slab is staged and
// decoded in two halves): the part's span, staged into the slab if it fits.
__device__ __forceinline__ Group nested_stage_part(const NestedArgs &a, __amdgpu_buffer_rsrc_t rsrc, uint8_t *slab,
                                                   uint64_t base, int lane, int l0, int l1) {
    uint64_t lo, hi;
    DecodeArgs d;
    d.stream = a.stream;
    d.stream_len = a.stream_len;
    d.ends = a.ends;
    d.n = a.n;
    d.r0 = 0;
    d.head = 0;
    load_group_ends(d, base, lane, lo, hi);
    Group gr;
    gr.rec_lo = lo;
    gr.rec_hi = hi < lo ? lo : hi;
    const int nrec = (int)(a.n - base < 64 ? a.n - base : 64);
    const int last = (l1 < nrec ? l1 : nrec) - 1;
    const uint64_t span_lo = uniform64(__shfl(lo, l0));
    const uint64_t span_hi = uniform64(__shfl(hi, last));
    gr.aligned_lo = span_lo & ~15ull;
    const uint64_t bytes = span_hi > gr.aligned_lo ? span_hi - gr.aligned_lo : 0;
    gr.chunks = (uint32_t)((bytes + 1023) >> 10);
    gr.in_lds = a.slab > 0 && l0 <= last && span_hi >= span_lo && SLAB_GUARD + (uint64_t)gr.chunks * 1024 + 16 <= a.slab;
    if (gr.in_lds) {
        issue_dma(rsrc, slab, gr, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        fix_stream_tail(d, rsrc, slab, gr, lane);
    }
    return gr;
}

// Item count of record [rs, re) (generic path).
template <class Src>
__device__ __forceinline__ uint32_t record_count(const Src &s, long long rs, long long re, const NestedArgs &a) {
    const RecInfo ri = rec_open(s, (typename Src::pos_t)rs, (typename Src::pos_t)re);
    return list_open(s, ri, a).count;
}

// index of the K_LIST field in a compile-time outer schema
template <class Spec>
__host__ __device__ constexpr int list_field() {
    for (int f = 0; f < Spec::N; f++)
        if (Spec::kind[f] == K_LIST) return f;
    return -1;
}

// Outer record r at [rs, re): its columns + status, and its list.
template <class OSpec, class Src>
__device__ __forceinline__ ListInfo decode_outer(const Src &s, long long rs, long long re, uint64_t r,
                                                 long long to_stream, const NestedArgs &a) {
    using pos_t = typename Src::pos_t;
    if constexpr (OSpec::N > 0 && __is_same(Src, LdsSrc)) {
        FastRec<OSpec> fr;
        if (fast_prepare<OSpec>(s, (int)rs, (int)re, fr)) {
            constexpr int LF = list_field<OSpec>();
            const ListInfo li = list_at(s, fr.lo[LF], fr.e[LF]);
            fast_finish<OSpec>(fr, r, a.outer, to_stream);
            return li;
        }
    }
    decode_record_generic(s, (pos_t)rs, (pos_t)re, r, a.outer, to_stream);
    const RecInfo ri = rec_open(s, (pos_t)rs, (pos_t)re);
    return list_open(s, ri, a);
}

// Item `out` = List.GetBytes(i) of the list li (internal/types/list.go:100-116 with
// format.ListTable.Offset), opened and decoded.
template <class ISpec, class Src>
__device__ __forceinline__ void decode_item(const Src &s, const ListInfo &li, uint32_t i, uint64_t out,
                                            long long to_stream, const NestedArgs &a) {
    using pos_t = typename Src::pos_t;
    uint32_t start, end;
    if (li.big) {
        end = be32_at(s, li.tstart + 4ll * i);
        start = i ? be32_at(s, li.tstart + 4ll * (i - 1)) : 0;
    } else {
        end = be16_at(s, li.tstart + 2ll * i);
        start = i ? be16_at(s, li.tstart + 2ll * (i - 1)) : 0;
    }
    if (end > li.dsize) {
        // nil item => OpenItemErr(nil): empty message, zero fields, no error
        decode_record_generic(s, (pos_t)0, (pos_t)0, out, a.item, to_stream);
        return;
    }
    if (start > end) {
        decode_record_generic(s, (pos_t)0, (pos_t)0, out, a.item, to_stream);
        if (a.item.status) a.item.status[out] = ST_PANIC;
        return;
    }
    const pos_t ib = (pos_t)(li.dstart + start), ie = (pos_t)(li.dstart + end);
    if constexpr (ISpec::N > 0 && __is_same(Src, LdsSrc)) {
        FastRec<ISpec> fr;
        if (fast_prepare<ISpec>(s, (int)ib, (int)ie, fr)) {
            fast_finish<ISpec>(fr, out, a.item, to_stream);
            return;
        }
    }
    decode_record_generic(s, ib, ie, out, a.item, to_stream);
}

// The group's items, item-parallel: item j of the group (j = excl[owner] + i) on lane j % 64.
// owner of group item j: the largest lane whose exclusive prefix is <= j (it has count > 0);
// i = j's index in the owner's list
__device__ __forceinline__ ListInfo item_owner(const ListInfo &li, uint32_t excl, uint32_t j, uint32_t &i) {
    int l = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
        const uint32_t ex = __shfl(excl, l + step < 64 ? l + step : 63);
        if (l + step < 64 && ex <= j) l += step;
    }
    ListInfo own;
    i = j - __shfl(excl, l);
    own.dstart = __shfl(li.dstart, l);
    own.tstart = __shfl(li.tstart, l);
    own.dsize = __shfl(li.dsize, l);
    own.big = __shfl((int)li.big, l) != 0;
    own.count = 0;
    return own;
}

// The group's items, item-parallel: item j of the group (j = excl[owner] + i) on lane j % 64.
// Two chunks of 64 items per iteration (NESTED_ITEM_U = 2): their owner searches and LDS
// reads are independent, so each wave keeps twice the LDS traffic in flight.
#ifndef NESTED_ITEM_U
#define NESTED_ITEM_U 2
#endif
// (j_first, j_step: a wave pair's waves take alternate rounds of 64 * U items, nested_decode_pair)
template <class ISpec, int U = NESTED_ITEM_U, class Src>
__device__ __forceinline__ void decode_group_items(const Src &s, const ListInfo &li, uint32_t excl, uint32_t total,
                                                   uint64_t item_base, int lane, long long to_stream,
                                                   const NestedArgs &a, uint32_t j_first = 0,
                                                   uint32_t j_step = 64 * U) {
    for (uint32_t j0 = j_first; j0 < total; j0 += j_step) {
        ListInfo own[U];
        uint32_t idx[U];
#pragma unroll
        for (int u = 0; u < U; u++) own[u] = item_owner(li, excl, j0 + 64 * u + lane, idx[u]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t j = j0 + 64 * u + lane;
            const uint64_t out = item_base + j;
            if (j < total && out < a.item_cap) decode_item<ISpec>(s, own[u], idx[u], out, to_stream, a);
        }
    }
}

// The group's items from PRECOMPUTED ranges (LdsSrc only): each record's lane first writes the
// slab range [lo, hi) of each of its items (its list table entries, List.GetBytes) into an LDS
// array indexed by the group item, a window of NESTED_RANGE_ITEMS at a time; then item j of the
// window reads its range with one LDS read — no owner search and no table reads on the item's
// dependency chain.  Ranges pack two 16-bit slab positions (slabs are < 64 KiB); a nil item
// (end > dataSize) is the empty range, a panicking one (start > end) RANGE_PANIC.
constexpr uint32_t NESTED_RANGE_ITEMS = 256;
constexpr uint32_t NESTED_RANGE_BYTES = NESTED_RANGE_ITEMS * 4;
constexpr uint32_t RANGE_PANIC = 0xffffu;

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class ISpec>
__device__ __forceinline__ void decode_group_items_ranges(const LdsSrc &s, const ListInfo &li, uint32_t excl,
                                                          uint32_t total, uint64_t item_base, int lane,
                                                          long long to_stream, uint32_t *rng,
                                                          const NestedArgs &a) {
    constexpr int U = NESTED_ITEM_U;
    for (uint32_t w0 = 0; w0 < total; w0 += NESTED_RANGE_ITEMS) {
        const uint32_t w1 = total - w0 < NESTED_RANGE_ITEMS ? total : w0 + NESTED_RANGE_ITEMS;
        // this record's items [excl, excl + count) within the window [w0, w1)
        const uint32_t i0 = w0 > excl ? w0 - excl : 0u;
        const uint32_t e1 = excl + li.count < w1 ? excl + li.count : w1;
        const uint32_t i1 = e1 > excl ? e1 - excl : 0u;
        for (uint32_t i = i0; i < i1; i++) {
            uint32_t start, end;
            if (li.big) {
                end = be32_at(s, li.tstart + 4ll * i);
                start = i ? be32_at(s, li.tstart + 4ll * (i - 1)) : 0;
            } else {
                end = be16_at(s, li.tstart + 2ll * i);
                start = i ? be16_at(s, li.tstart + 2ll * (i - 1)) : 0;
            }
            uint32_t v;
            if (end > li.dsize) v = 0u;              // nil: OpenItemErr(nil), an empty message
            else if (start > end) v = RANGE_PANIC;   // Go panics on the slice
            else v = (uint32_t)(li.dstart + start) | ((uint32_t)(li.dstart + end) << 16);
            rng[excl + i - w0] = v;
        }
        wave_lds_sync();
        for (uint32_t j0 = w0; j0 < w1; j0 += 64 * U) {
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t j = j0 + 64 * u + lane;
                v[u] = j < w1 ? rng[j - w0] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t j = j0 + 64 * u + lane;
                const uint64_t out = item_base + j;
                if (j >= w1 || out >= a.item_cap) continue;
                if (v[u] == RANGE_PANIC) {
                    decode_record_generic(s, 0, 0, out, a.item, to_stream);
                    if (a.item.status) a.item.status[out] = ST_PANIC;
                    continue;
                }
                const int ib = (int)(v[u] & 0xffffu), ie = (int)(v[u] >> 16);
                if constexpr (ISpec::N > 0) {
                    FastRec<ISpec> fr;
                    if (fast_prepare<ISpec>(s, ib, ie, fr)) {
                        fast_finish<ISpec>(fr, out, a.item, to_stream);
                        continue;
                    }
                }
                decode_record_generic(s, ib, ie, out, a.item, to_stream);
            }
        }
        wave_lds_sync(); // the next window's ranges overwrite this one's
    }
}

// ---- decoupled look-back (one pass) ------------------------------------------------------

constexpr uint64_t LB_AGG = 1ull << 62;       // word holds the group's own item count
constexpr uint64_t LB_PRE = 2ull << 62;       // word holds the inclusive prefix (items up to and incl. the group)
constexpr uint64_t LB_VAL = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

// Publish unit g's item count `agg`, return the items of units [0, g).  Units are blocks of
// DEC_WAVES groups in block order (workgroups are dispatched in increasing id, so every unit < g
// is resident or done and will publish: the wait ends).  The window looks back 256 units per
// round (4 per lane, nearest first); 1,024 per round (16 per lane) measured no faster.
__device__ __forceinline__ uint64_t lookback(uint64_t *state, uint64_t g, uint64_t agg, int lane) {
    constexpr int K = 4;
    if (lane == 0) lb_store(&state[g], (g == 0 ? LB_PRE : LB_AGG) | agg);
    if (g == 0) return 0;
    uint64_t excl = 0;
    long long hi = (long long)g - 1; // window: group hi - (lane + 64 k) on lane `lane`, slot k
    while (true) {
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const long long j = hi - lane - 64 * k;
            v[k] = j >= 0 ? lb_load(&state[j]) : LB_PRE; // before group 0: prefix 0
        }
        int first = 64 * K; // distance of the nearest inclusive prefix
        bool wait = false;
#pragma unroll
        for (int k = K - 1; k >= 0; k--) {
            const uint64_t pre = __ballot((v[k] >> 62) == 2);
            if (pre) first = 64 * k + __builtin_ctzll(pre);
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint64_t none = __ballot((v[k] >> 62) == 0);
            const int lim = first - 64 * k; // lanes of slot k nearer than `first`, or at it
            if (lim >= 0 && none & (lim >= 63 ? ~0ull : ((2ull << lim) - 1))) wait = true;
        }
        if (wait) { // a nearer group has not published yet
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t part = 0;
#pragma unroll
        for (int k = 0; k < K; k++)
            if (lane + 64 * k <= first) part += v[k] & LB_VAL;
        excl += wave_sum64(part);
        if (first < 64 * K) break;
        hi -= 64 * K;
    }
    if (lane == 0) lb_store(&state[g], LB_PRE | (excl + agg));
    return excl;
}

// ONEPASS: the block's groups (one per wave) sum their item totals in LDS (xch); wave 0 publishes
// the block's total and looks back over the earlier blocks; each wave's first item = the block's
// base + the totals of the block's earlier waves.  Every wave of the block calls this once (a
// wave past the batch's end with total 0).
__device__ __forceinline__ uint64_t onepass_base(const NestedArgs &a, uint32_t total, int lane, uint64_t *xch) {
    const int wave = threadIdx.x >> 6;
    if (lane == 0) xch[wave] = total;
    __syncthreads();
    uint64_t before = 0, bt = 0;
#pragma unroll
    for (int w = 0; w < DEC_WAVES; w++) {
        const uint64_t t = xch[w];
        before += w < wave ? t : 0;
        bt += t;
    }
    if (wave == 0) {
        const uint64_t b = uniform64(lookback(a.group_base, blockIdx.x, bt, lane));
        if (lane == 0) xch[DEC_WAVES] = b;
    }
    __syncthreads();
    return uniform64(xch[DEC_WAVES] + before);
}

// Decode a group: outer records (lane = record), then items (item-parallel).  item_base =
// the group's first item; ONEPASS: item_base is found here by look-back (state = a.group_base).
template <class OSpec, class ISpec, bool ONEPASS, int U = NESTED_ITEM_U, class Src>
__device__ __forceinline__ uint32_t nested_group_body(const Src &s, long long rs, long long re, bool valid,
                                                      uint64_t r, uint64_t g, uint64_t item_base, int lane,
                                                      long long to_stream, const NestedArgs &a,
                                                      uint32_t *rng = nullptr, uint64_t *xch = nullptr) {
    ListInfo li = {0, 0, 0, 0, false};
    if (valid) li = decode_outer<OSpec>(s, rs, re, r, to_stream, a);
    const uint32_t incl = wave_incl_scan(li.count, lane);
    const uint32_t excl = incl - li.count;
    const uint32_t total = __shfl(incl, 63);
    if constexpr (ONEPASS) {
        item_base = onepass_base(a, total, lane, xch);
        if (g == (a.n - 1) / 64 && lane == 0) *a.total = item_base + total;
    }
    if (valid) {
        a.item_begin[r] = (uint32_t)(item_base + excl);
        if (r == a.n - 1) a.item_begin[a.n] = (uint32_t)(item_base + incl);
    }
    if constexpr (__is_same(Src, LdsSrc)) {
        if (rng) {
            decode_group_items_ranges<ISpec>(s, li, excl, total, item_base, lane, to_stream, rng, a);
            return total;
        }
    }
    decode_group_items<ISpec, U>(s, li, excl, total, item_base, lane, to_stream, a);
    return total;
}

// A part of a group (lanes [l0, l1)) from the slab when it fits, from HBM otherwise; the part's items
// start at item_base.  Returns the part's item count.
template <class OSpec, class ISpec, bool RANGES, int U = NESTED_ITEM_U>
__device__ __forceinline__ uint32_t nested_decode_part(const NestedArgs &a, __amdgpu_buffer_rsrc_t rsrc,
                                                       uint8_t *slab, uint64_t g, uint64_t item_base, int lane,
                                                       int l0, int l1) {
    const uint64_t base = g * 64;
    const Group gr = nested_stage_part(a, rsrc, slab, base, lane, l0, l1);
    const uint64_t r = base + lane;
    const bool valid = r < a.n && lane >= l0 && lane < l1;
    if (gr.in_lds) {
        LdsSrc s{(lds_u8 *)slab};
        return nested_group_body<OSpec, ISpec, false, U>(s, SLAB_GUARD + (long long)(gr.rec_lo - gr.aligned_lo),
                                                      SLAB_GUARD + (long long)(gr.rec_hi - gr.aligned_lo), valid, r,
                                                      g, item_base, lane, (long long)gr.aligned_lo - SLAB_GUARD, a,
                                                      RANGES ? (uint32_t *)(slab + a.slab) : nullptr);
    }
    GlobalSrc s{a.stream, a.stream_len};
    return nested_group_body<OSpec, ISpec, false, U>(s, (long long)gr.rec_lo, (long long)gr.rec_hi, valid, r, g,
                                                  item_base, lane, 0, a);
}

// Kernel body for one group per wave.  ONEPASS: group = wave index, a.group_base = one state word
// per block (zeroed by the launcher); else group = wave index and a.group_base holds the
// exclusive item offsets from the index kernels.
template <class OSpec, class ISpec, bool ONEPASS, bool RANGES = false, int U = NESTED_ITEM_U>
__device__ __forceinline__ void nested_decode_body(const NestedArgs &a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint64_t g;
    if constexpr (ONEPASS) {
        // group = block order: workgroups are dispatched in increasing id, so every group a
        // group waits on (a smaller id) is running or done — the lowest running group never waits
        // (round 4 took a ticket from one global counter: 16 K agent-scope atomics on one address)
        g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    } else {
        // blocks are dealt round-robin to the 8 XCDs: with xcd = 1, block b takes the b/8-th slot
        // of XCD b%8's contiguous share, so neighbouring groups (sharing the item columns' cache
        // lines) are written through one L2
        uint64_t blk = blockIdx.x;
        if (a.xcd) {
            const uint64_t per = (gridDim.x + 7) / 8;
            blk = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
        }
        g = blk * (blockDim.x >> 6) + wave;
    }
    const uint64_t base = g * 64;
    __shared__ uint64_t xch[DEC_WAVES + 1]; // ONEPASS: the block's wave totals, then its base
    if (base >= a.n) {
        if constexpr (ONEPASS) onepass_base(a, 0u, lane, xch); // the block's barriers
        return;
    }
    // per wave: the slab, then (RANGES) the item range window
    uint8_t *slab = smem + wave * (a.slab + (RANGES ? NESTED_RANGE_BYTES : 0u));
    __amdgpu_buffer_rsrc_t rsrc =
        uniform_rsrc(a.stream, a.stream_len);
    if constexpr (!ONEPASS) {
        // the whole group in the slab; a group whose span exceeds it (a batch whose record sizes
        // vary a lot) as two halves of 32 records, each staged on its own
        const uint64_t item_base = uniform64(a.group_base[g]);
        const Group whole = nested_stage_part(a, rsrc, slab, base, lane, 0, 64);
        const uint64_t r = base + lane;
        if (whole.in_lds) {
            LdsSrc s{(lds_u8 *)slab};
            nested_group_body<OSpec, ISpec, false, U>(s, SLAB_GUARD + (long long)(whole.rec_lo - whole.aligned_lo),
                                                   SLAB_GUARD + (long long)(whole.rec_hi - whole.aligned_lo),
                                                   r < a.n, r, g, item_base, lane,
                                                   (long long)whole.aligned_lo - SLAB_GUARD, a,
                                                   RANGES ? (uint32_t *)(slab + a.slab) : nullptr);
            return;
        }
        const uint32_t first = nested_decode_part<OSpec, ISpec, RANGES, U>(a, rsrc, slab, g, item_base, lane, 0, 32);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the first half's LDS reads done
        __builtin_amdgcn_wave_barrier();
        nested_decode_part<OSpec, ISpec, RANGES, U>(a, rsrc, slab, g, item_base + first, lane, 32, 64);
        return;
    }
    const Group gr = nested_stage(a, rsrc, slab, base, lane);
    const uint64_t r = base + lane;
    const bool valid = r < a.n;
    const uint64_t item_base = 0;
    if (gr.in_lds) {
        LdsSrc s{(lds_u8 *)slab};
        nested_group_body<OSpec, ISpec, ONEPASS>(s, SLAB_GUARD + (long long)(gr.rec_lo - gr.aligned_lo),
                                                 SLAB_GUARD + (long long)(gr.rec_hi - gr.aligned_lo), valid, r, g,
                                                 item_base, lane, (long long)gr.aligned_lo - SLAB_GUARD, a,
                                                 RANGES ? (uint32_t *)(slab + a.slab) : nullptr, xch);
    } else {
        GlobalSrc s{a.stream, a.stream_len};
        nested_group_body<OSpec, ISpec, ONEPASS>(s, (long long)gr.rec_lo, (long long)gr.rec_hi, valid, r, g,
                                                 item_base, lane, 0, a, nullptr, xch);
    }
}

// Two-pass decode on a WAVE PAIR (round 5; decode_core.hpp decode_flat_pair is the flat
// analogue): a 128-thread block takes one group of 64 records.  Both waves stage the group's
// span into ONE slab (1 KiB DMA chunks issued round-robin; the chunk straddling the stream end
// refilled by the wave that issued it), wave 0 decodes the 64 outer records and posts each
// record's list (count, data / table start, data size, big) to LDS after the slab, then both
// waves decode the group's items, alternating rounds of 64 * U items.  Twice the waves per
// staged byte: the items' LDS reads are latency-bound.  A group larger
// than the slab: wave 0 alone, in two halves of 32 records (nested_decode_part).
// SELF: the other waves open each record's list themselves (rec_open + list_open, the generic
// path's lookup) instead of waiting for wave 0's posted lists.
// ONEPASS (round 6): no index kernels.  The group's item total is known once wave 0 has posted
// the lists; wave 0 then publishes it and finds the group's first item by the decoupled
// look-back over the earlier groups (lookback: groups in block order, a.group_base = one state
// word per group, zeroed by the launcher), both waves wait for it at a barrier and decode the
// items.  The stream is read once (the count pass re-read each record's tail).
template <class OSpec, class ISpec, int U = NESTED_ITEM_U, int P = 2, bool SELF = false, bool ONEPASS = false>
__device__ __forceinline__ void nested_decode_pair(const NestedArgs &a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint64_t g = blockIdx.x;
    if (a.xcd && !ONEPASS) {
        const uint64_t per = (gridDim.x + 7) / 8;
        g = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    }
    const uint64_t base = g * 64;
    if (base >= a.n) return; // (block-uniform)
    uint8_t *slab = smem;
    uint32_t *xl = (uint32_t *)(smem + a.slab); // [4][64]: count, dsize | big << 31, dstart, tstart
    __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(a.stream, a.stream_len);
    uint64_t item_base = ONEPASS ? 0 : uniform64(a.group_base[g]);
    DecodeArgs d;
    d.stream = a.stream;
    d.stream_len = a.stream_len;
    d.ends = a.ends;
    d.n = a.n;
    d.r0 = 0;
    d.head = 0;
    uint64_t lo, hi;
    load_group_ends(d, base, lane, lo, hi);
    const Group gr = make_group(d, base, lane, lo, hi, a.slab);
    if (!gr.in_lds) {
        if (wave == 0) {
            if constexpr (ONEPASS) { // the group's item total from HBM first, then its base
                GlobalSrc gs{a.stream, a.stream_len};
                const uint32_t cnt = base + lane < a.n ? record_count(gs, (long long)gr.rec_lo, (long long)gr.rec_hi, a) : 0u;
                const uint32_t tot = wave_sum(cnt);
                item_base = uniform64(lookback(a.group_base, g, tot, lane));
                if (g == (a.n - 1) / 64 && lane == 0) *a.total = item_base + tot;
            }
            const uint32_t first = nested_decode_part<OSpec, ISpec, false, U>(a, rsrc, slab, g, item_base, lane, 0, 32);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the first half's LDS reads done
            __builtin_amdgcn_wave_barrier();
            nested_decode_part<OSpec, ISpec, false, U>(a, rsrc, slab, g, item_base + first, lane, 32, 64);
        }
        return;
    }
    for (uint32_t c = (uint32_t)wave; c < gr.chunks; c += P)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(slab + SLAB_GUARD + c * 1024),
                                                 16, (uint32_t)gr.aligned_lo + c * 1024 + lane * 16, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t tail = a.stream_len & ~15ull;
    if (tail < a.stream_len && tail >= gr.aligned_lo && tail < gr.aligned_lo + (uint64_t)gr.chunks * 1024 &&
        (int)(((tail - gr.aligned_lo) >> 10) % P) == wave && lane < 16 && tail + lane < a.stream_len)
        slab[SLAB_GUARD + (tail - gr.aligned_lo) + lane] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (uint32_t)(tail + lane), 0, 0);
    __syncthreads(); // the slab is whole
    LdsSrc s{(lds_u8 *)slab};
    const long long to_stream = (long long)gr.aligned_lo - SLAB_GUARD;
    const uint64_t r = base + lane;
    const bool valid = r < a.n;
    ListInfo li = {0, 0, 0, 0, false};
    const int rs = SLAB_GUARD + (int)(gr.rec_lo - gr.aligned_lo), re = SLAB_GUARD + (int)(gr.rec_hi - gr.aligned_lo);
    if constexpr (SELF) {
        if (valid) {
            if (wave == 0) li = decode_outer<OSpec>(s, rs, re, r, to_stream, a);
            else li = list_open(s, rec_open(s, rs, re), a);
        }
    } else if (wave == 0) {
        if (valid) li = decode_outer<OSpec>(s, rs, re, r, to_stream, a);
        xl[lane] = li.count;
        xl[64 + lane] = li.dsize | ((uint32_t)li.big << 31);
        xl[128 + lane] = (uint32_t)li.dstart;
        xl[192 + lane] = (uint32_t)li.tstart;
    }
    if constexpr (!SELF) __syncthreads(); // the lists are posted
    if (!SELF && wave != 0) {
        li.count = xl[lane];
        const uint32_t ds = xl[64 + lane];
        li.dsize = ds & 0x7fffffffu;
        li.big = (ds >> 31) != 0;
        li.dstart = xl[128 + lane];
        li.tstart = xl[192 + lane];
    }
    const uint32_t incl = wave_incl_scan(li.count, lane);
    const uint32_t excl = incl - li.count;
    const uint32_t total = __shfl(incl, 63);
    if constexpr (ONEPASS) {
        uint64_t *xb = (uint64_t *)(xl + 256); // the group's base, from wave 0 to the others
        if (wave == 0) {
            const uint64_t b = uniform64(lookback(a.group_base, g, total, lane));
            if (lane == 0) {
                *xb = b;
                if (g == (a.n - 1) / 64) *a.total = b + total;
            }
        }
        __syncthreads(); // the base is posted
        item_base = uniform64(*xb);
    }
    if (wave == 0 && valid) {
        a.item_begin[r] = (uint32_t)(item_base + excl);
        if (r == a.n - 1) a.item_begin[a.n] = (uint32_t)(item_base + incl);
    }
    decode_group_items<ISpec, U>(s, li, excl, total, item_base, lane, to_stream, a, (uint32_t)wave * 64 * U,
                                 P * 64 * U);
}

// Count kernel of the two-pass index: per group, the item total.
__device__ __forceinline__ void nested_count_body(const NestedArgs &a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const uint64_t base = g * 64;
    if (base >= a.n) return;
    uint8_t *slab = smem + wave * a.slab;
    __amdgpu_buffer_rsrc_t rsrc =
        uniform_rsrc(a.stream, a.stream_len);
    uint32_t cnt = 0;
    // the whole group, or (span larger than the slab) two halves of 32 records
    for (int part = 0; part < 2; part++) {
        const int l0 = part ? 32 : 0;
        const int l1 = part ? 64 : 32;
        const Group gr = nested_stage_part(a, rsrc, slab, base, lane, part ? l0 : 0, part ? l1 : 64);
        const bool whole = part == 0 && gr.in_lds;
        Group h = gr;
        if (!whole && part == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            h = nested_stage_part(a, rsrc, slab, base, lane, 0, 32);
        }
        const int hl0 = whole ? 0 : l0, hl1 = whole ? 64 : l1;
        const bool valid = base + lane < a.n && lane >= hl0 && lane < hl1;
        if (valid) {
            if (h.in_lds) {
                LdsSrc s{(lds_u8 *)slab};
                cnt = record_count(s, SLAB_GUARD + (long long)(h.rec_lo - h.aligned_lo),
                                   SLAB_GUARD + (long long)(h.rec_hi - h.aligned_lo), a);
            } else {
                GlobalSrc s{a.stream, a.stream_len};
                cnt = record_count(s, (long long)h.rec_lo, (long long)h.rec_hi, a);
            }
        }
        if (whole) break;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // this half's LDS reads done
        __builtin_amdgcn_wave_barrier();
    }
    const uint32_t sum = wave_sum(cnt);
    if (lane == 0) a.group_base[g] = sum;
}

// ---- count from tail windows --------------------------------------------------------------
// The count pass needs, per record, only OpenMessage's trailer and table, the list field's
// table entry and the list's own trailer.  A Writer emits the table and trailer last and, for a
// record whose list is its last field, the list's trailer right below the table: all within the
// record's last few dozen bytes.  So instead of staging the whole span, each lane loads the 40
// bytes [a, a + 40) (a = (end - 32) & ~7: at least the last 32 bytes, 8-byte aligned so the
// parse's qword reads stay in the window) into its own LDS window and parses from there; a read
// outside the window (big tables, a list followed by other fields, malformed records) goes to HBM
// through the same range-checked loads GlobalSrc uses, so the count is the same whatever the
// record looks like.  The count is bound by the 128-byte lines the windows touch: 1 + 39/128 per
// record on average (round 3's 64-byte window at a 16-byte boundary: 1 + 63/128).
constexpr int TAIL_WIN = 40;
constexpr int TAIL_BACK = 32; // bytes below the record end the window always holds
// Windows sit TAIL_STRIDE = 11 dwords apart: lane i's byte k is in bank (11 i + k / 4) mod 32,
// so the 32 lanes of a ds_write_b32 / ds_read group never share a bank at equal k (an even
// stride of 16 dwords put every other lane on the same 4 banks: 10.4 conflict cycles per LDS
// instruction, r02h).
constexpr int TAIL_STRIDE = TAIL_WIN + 4;

struct WinSrc {
    using pos_t = long long;
    lds_u8 *lds;  // this lane's window (4-byte aligned): stream bytes [a, a + TAIL_WIN)
    long long a;
    GlobalSrc g;
    __device__ __forceinline__ uint32_t u8(long long p) const {
        const unsigned long long k = (unsigned long long)(p - a);
        return k < (unsigned long long)TAIL_WIN ? (uint32_t)lds[k] : g.u8(p);
    }
    __device__ __forceinline__ uint64_t d64(long long p) const {
        const unsigned long long k = (unsigned long long)(p - a);
        if (k <= (unsigned long long)(TAIL_WIN - 8) && !(k & 7))
            return (uint64_t)*(lds_u32 *)(lds + k) | ((uint64_t)*(lds_u32 *)(lds + k + 4) << 32);
        return g.d64(p);
    }
    __device__ __forceinline__ uint32_t d32(long long p) const {
        const unsigned long long k = (unsigned long long)(p - a);
        if (k <= (unsigned long long)(TAIL_WIN - 4) && !(k & 3)) return *(lds_u32 *)(lds + k);
        return g.d32(p);
    }
};

// 16 stream bytes at o as GlobalSrc reads them (a piece straddling the end bytewise, beyond: 0)
__device__ __forceinline__ uint4 win_piece(__amdgpu_buffer_rsrc_t rsrc, uint64_t o, uint64_t len) {
    const uint32_t o32 = (uint32_t)o;
    if ((uint64_t)o32 + 16 <= len) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o32, 0, 0);
        return make_uint4(v[0], v[1], v[2], v[3]);
    }
    return make_uint4(buf_ld32(rsrc, o32, len), buf_ld32(rsrc, o32 + 4, len), buf_ld32(rsrc, o32 + 8, len),
                      buf_ld32(rsrc, o32 + 12, len));
}

__device__ __forceinline__ void nested_count_tail_body(const NestedArgs &a, uint8_t *wins) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const uint64_t base = g * 64;
    if (base >= a.n) return;
    __amdgpu_buffer_rsrc_t rsrc =
        uniform_rsrc(a.stream, a.stream_len);
    DecodeArgs d;
    d.ends = a.ends;
    d.n = a.n;
    d.head = 0;
    uint64_t lo, hi;
    load_group_ends(d, base, lane, lo, hi);
    if (hi < lo) hi = lo; // malformed ends: an empty record (make_group)
    uint32_t cnt = 0;
    if (base + lane < a.n) {
        const uint64_t w0 = hi >= TAIL_BACK ? (hi - TAIL_BACK) & ~7ull : 0;
        uint8_t *win = wins + threadIdx.x * TAIL_STRIDE;
        static_assert(TAIL_WIN == 40, "two 16-byte pieces and one 8-byte piece");
        const uint4 v0 = win_piece(rsrc, w0, a.stream_len), v1 = win_piece(rsrc, w0 + 16, a.stream_len);
        const uint32_t o2 = (uint32_t)(w0 + 32);
        uint32_t v2x, v2y;
        if ((uint64_t)o2 + 8 <= a.stream_len) {
            const auto q = __builtin_amdgcn_raw_buffer_load_b64(rsrc, o2, 0, 0);
            v2x = q[0];
            v2y = q[1];
        } else {
            v2x = buf_ld32(rsrc, o2, a.stream_len);
            v2y = buf_ld32(rsrc, o2 + 4, a.stream_len);
        }
        uint32_t *d = (uint32_t *)win;
        d[0] = v0.x;
        d[1] = v0.y;
        d[2] = v0.z;
        d[3] = v0.w;
        d[4] = v1.x;
        d[5] = v1.y;
        d[6] = v1.z;
        d[7] = v1.w;
        d[8] = v2x;
        d[9] = v2y;
        WinSrc s{(lds_u8 *)win, (long long)w0, GlobalSrc{a.stream, a.stream_len}};
        cnt = record_count(s, (long long)lo, (long long)hi, a);
    }
    const uint32_t sum = wave_sum(cnt);
    if (lane == 0) a.group_base[g] = sum;
}

} // namespace spec
