// encode_nested_core.hpp — device code of the list<message> encoder (BASELINE config 4), shared
// by the precompiled kernels (encode_nested.hip: RuntimeEnc record policies) and the
// schema-specialised ones (jit.cpp: SpecEnc<outer>, SpecEnc<item>).
//
// Per record, what a generated Write() does over the Writer:
//   w.Field(tag).<Kind>(v) for the outer scalar fields, in write order
//   l := w.Field(list_tag).List()           FieldWriter.List, internal/writer/msg.go:219-222
//   for each item: m := l.Add()             MessageListWriter.Add, writer_list_msg.go:22-25
//       m.Field(t).<Kind>(v)...; m.End()     -> endMessage + endElement (element offset =
//                                              item end - list start), internal/writer/writer.go:299-337
//   l.End()                                 -> endList: EncodeListTable (IsBigList: count > 255 or
//                                              last offset > 65535), internal/writer/writer.go:339-372,
//                                              internal/encode/list.go:15-75, internal/format/list.go:40-54
//   w.Build()                               -> the outer table + trailer
//
// Layout of the work: one wave = 64 consecutive records (one per lane) and the items they own,
// which are contiguous ([item_begin[first], item_begin[last + 1])).  Item sizes are computed
// ITEM-parallel (item k of the wave on lane k % 64, coalesced item column loads) and
// prefix-summed into LDS; a record's list size and every item's position follow from that
// prefix.  Emission into the wave's LDS slab:
//   A. lane per record: the outer fields, jumping over the list's items, then the list table
//      (element ends from the prefix), list trailer, later fields, outer table, trailer;
//   B. item per lane, chunks of 64 items from the LAST chunk to the first: each item as one
//      straight run (HEAD_ST4 emitter: its first dword is stored whole, clobbering <= 3 bytes
//      below the item, which belong to the previous item — written later, lockstep or a later
//      chunk — or to the record's bytes before the list, restored in C);
//   C. each record restores the dword under its list start from a copy taken after A.
// The wave then copies the slab to HBM with 16-byte stores.  Waves with more than
// NENC_ITEM_CAP items, invalid item ranges, or output that does not fit the slab take the
// per-lane generic path straight to HBM (same bytes).
#pragma once

#include "encode_core.hpp"

namespace spec {

struct NestedEncodeArgs {
    uint64_t n;
    EncFields outer; // its K_LIST field is written from item_begin + item
    EncFields item;
    const uint32_t *item_begin; // [n + 1]
    uint64_t nitems;            // item columns hold this many items
    uint32_t check_heaps;
    uint8_t *out;
    uint64_t out_cap;
    uint64_t *ends;
    uint64_t *block_sums;
    uint64_t nblocks;
    uint64_t *total;
    uint32_t xcd; // write pass: 1 = XCD-aware block order (grid padded to a multiple of 8)
    // optional (workspace large enough): the size pass leaves every item's wave prefix
    // (item_pre[i] = bytes of the wave's items up to and including item i) and each wave's
    // item-parallel verdict (wave_ok), so the write pass reads them instead of reloading every
    // item column and heap to recompute the sizes and scans
    uint32_t *item_pre;
    uint8_t *wave_ok;
};

constexpr int NENC_BLOCK = 256;               // records per block (4 waves, one record per lane)
constexpr int NENC_ITEM_CAP = 512;            // items per wave on the item-parallel path
constexpr int NENC_PRE = (NENC_ITEM_CAP + 4) * 4; // per-wave item prefix (u32), 16-B multiple
constexpr int NENC_SLAB = 17920;              // per-wave output staging
constexpr int NENC_HEAD = 256;                // wsum[4] | inv_outer[64] | inv_item[64] | dummy | errs
constexpr int NENC_WAVE_LDS = NENC_PRE + NENC_SLAB;
constexpr size_t nenc_size_lds_bytes() { return NENC_HEAD + (size_t)(NENC_BLOCK / 64) * NENC_PRE; }
constexpr size_t nenc_write_lds_bytes() { return NENC_HEAD + (size_t)(NENC_BLOCK / 64) * NENC_WAVE_LDS; }
static_assert(NENC_PRE % 16 == 0 && NENC_WAVE_LDS % 16 == 0, "slab alignment");

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- generic per-lane path (the whole list of a record on its lane) ------------------------

struct ListSize {
    uint64_t total, data;
    uint32_t count;
    bool big;
};

__device__ __forceinline__ ListSize list_size(const NestedEncodeArgs &a, uint64_t r, bool check, bool &err) {
    ListSize ls = {0, 0, 0, false};
    const uint32_t b = a.item_begin[r], e = a.item_begin[r + 1];
    if (e < b || e > a.nitems) {
        err = true;
        return ls;
    }
    uint64_t data = 0;
    for (uint32_t i = b; i < e; i++) data += record_size(a.item, i, check, err).total;
    ls.count = e - b;
    ls.data = data;
    ls.big = ls.count > 255 || data > 65535; // IsBigList, internal/format/list.go:40-54
    const uint64_t tsize = (uint64_t)ls.count * (ls.big ? 4 : 2);
    if (data > MAX_SIZE || tsize > MAX_SIZE) err = true; // EncodeListTable: list too large
    ls.total = data + tsize + vlen32((uint32_t)data) + vlen32((uint32_t)tsize) + 1;
    return ls;
}

// Emits the list value of record r at the emitter's position (flushing it first) and moves
// the emitter past it.
template <class Sink, class Pos>
struct ListEmitter {
    const NestedEncodeArgs *a;
    const Sink *k;
    const uint8_t *item_inv;
    template <class E>
    __device__ __forceinline__ void operator()(E &em, uint32_t, uint64_t r) const {
        em.finish();
        bool err = false;
        const ListSize ls = list_size(*a, r, false, err);
        const Pos lstart = em.pos;
        const Pos tstart = lstart + (Pos)ls.data;
        const uint32_t esize = ls.big ? 4 : 2;
        Pos p = lstart;
        const uint32_t b = a->item_begin[r];
        for (uint32_t j = 0; j < ls.count; j++) {
            const RecSize irs = record_size(a->item, b + j, false, err);
            p = emit_message(a->item, *k, p, (uint64_t)(b + j), irs, item_inv);
            // element offset = item end - list start (writer.go:327-330), big-endian
            const uint32_t off = (uint32_t)(p - lstart);
            const Pos q = tstart + (Pos)(j * esize);
            if (ls.big) {
                k->st1(q, off >> 24);
                k->st1(q + 1, (off >> 16) & 0xff);
                k->st1(q + 2, (off >> 8) & 0xff);
                k->st1(q + 3, off & 0xff);
            } else {
                k->st1(q, (off >> 8) & 0xff);
                k->st1(q + 1, off & 0xff);
            }
        }
        // trailer: rvarint(dataSize) | rvarint(tableSize) | type (internal/encode/list.go:36-43)
        Emit<Sink, Pos> tr(*k, tstart + (Pos)((uint64_t)ls.count * esize));
        tr.rvarint((uint32_t)ls.data);
        tr.rvarint(ls.count * esize);
        tr.put1(ls.big ? T_BIG_LIST : T_LIST);
        tr.finish();
        em.pos = tr.pos;
        em.lo = tr.pos;
        em.acc = 0;
    }
};

// ---- item-parallel path ---------------------------------------------------------------

// list size hook: the list's encoded size, known from the wave's item prefix
struct KnownListSize {
    uint64_t total;
    __device__ __forceinline__ uint64_t operator()(uint32_t, uint64_t) const { return total; }
};

// list emit hook (phase A): skips the items, writes the list table and trailer, records where
// the items start.  An empty list is no jump: the emitter keeps its pending bytes (a HEAD_ST4
// emitter restarting at the same position would zero the bytes below it, and no item would
// rewrite them).
// merge_slab (the pair write pass's A2, run once the items are final): after the jump the
// HEAD_ST4 emitter resumes with the bytes already in the slab below the list's end (the last
// item's tail) as its pending bytes, so its first whole-dword store writes them back unchanged.
struct WaveListEmit {
    const uint32_t *pre; // wave item prefix at this record's first item
    uint32_t count, data;
    bool big;
    mutable int lstart;
    const uint8_t *merge_slab = nullptr;
    template <class E>
    __device__ __forceinline__ void operator()(E &em, uint32_t, uint64_t) const {
        lstart = (int)em.pos;
        if (data) {
            em.finish();
            em.pos += data;
            em.lo = em.pos;
            em.acc = 0;
            if (merge_slab && (em.pos & 3)) {
                const uint32_t w = *(const uint32_t *)(merge_slab + (em.pos & ~3));
                em.acc = w & (0xffffffffu >> (32 - 8 * (uint32_t)(em.pos & 3)));
            }
        }
        const uint32_t p0 = pre[0];
        if constexpr (E::kHeadSt4) {
            if (__ballot(count > 8 || big) == 0) { // wave-uniform: short small lists
                // table {u16 BE end} x count | rvarint(data) (<= 3 bytes: data <= 65535) |
                // rvarint(2 count) (1 byte) | TypeList as ONE run built in registers
                // (internal/encode/list.go:36-75), appended with one store per dword
                uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const bool in = j < (int)count;
                    // element offset = item end - list start; the last item ends at the list's data
                    // size (pre[count] belongs to the next record, whose entries the pair write
                    // pass may already have turned into slab positions)
                    const uint32_t end = in ? (j + 1 < (int)count ? pre[j + 1] - p0 : data) : 0u;
                    w[j >> 1] |= (in ? (uint32_t)__builtin_bswap16((uint16_t)end) : 0u) << (16 * (j & 1));
                }
                const uint32_t L = vlen32(data);
                uint64_t x = data & 0x1fffff; // 3 groups of 7 bits -> bytes (inverse of rvarint_bf)
                x = (x & 0x7f) | ((x & 0x3f80) << 1) | ((x & 0x1fc000) << 2);
                const uint64_t be = (__builtin_bswap32((uint32_t)x) >> 8) >> (8 * (3 - L)); // top group first
                const uint64_t cont = (0x808080ull >> (8 * (3 - L))) & ~0xffull;
                const uint64_t T = (be | cont) | ((uint64_t)(2 * count) << (8 * L)) | ((uint64_t)T_LIST << (8 * (L + 1)));
                const uint32_t q = count >> 1;
                const uint64_t Ts = T << (16 * (count & 1)); // the trailer starts at byte 2 count
#pragma unroll
                for (int d = 0; d < 7; d++) {
                    w[d] |= d == (int)q ? (uint32_t)Ts : 0u;
                    w[d] |= d == (int)q + 1 ? (uint32_t)(Ts >> 32) : 0u;
                }
                em.template put_heap_short<7>(w, 0u, 2 * count + L + 2);
                return;
            }
        }
        for (uint32_t j = 0; j < count; j++) {
            const uint32_t end = j + 1 < count ? pre[j + 1] - p0 : data; // item end - list start
            em.put_n(big ? bswap32(end) : (uint32_t)__builtin_bswap16((uint16_t)end), big ? 4 : 2);
        }
        em.rvarint(data);
        em.rvarint(count * (big ? 4u : 2u));
        em.put1(big ? T_BIG_LIST : T_LIST);
    }
};

// Encoded sizes of the wave's items [I0, I0 + cnt) -> pre[k] = bytes of items I0..I0+k-1
// (pre[0] = 0).  Returns false if the wave's item bytes do not fit 31 bits.
template <class IP>
__device__ __forceinline__ bool wave_item_prefix(const NestedEncodeArgs &a, uint32_t I0, uint32_t cnt,
                                                 uint32_t *pre, int lane, bool check, bool &err) {
    uint64_t carry = 0;
    if (lane == 0) pre[0] = 0;
    // groups of 4 chunks (256 items): every load of the group in flight before the first
    // size is needed; lanes past the end re-read the last item
    for (uint32_t c0 = 0; c0 < cnt; c0 += 256) {
        typename IP::Rec rec[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t k = c0 + 64 * j + lane;
            IP::load_cols(a.item, I0 + (k < cnt ? k : cnt - 1), rec[j]); // sizes: columns only
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t k = c0 + 64 * j + lane;
            const bool iv = k < cnt;
            bool e = false;
            const uint64_t s = IP::size(a.item, rec[j], I0 + (iv ? k : cnt - 1), check, e).total;
            err |= iv & e;
            uint64_t x = iv ? s : 0;
            for (int o = 1; o < 64; o <<= 1) {
                const uint64_t y = __shfl_up(x, o);
                if (lane >= o) x += y;
            }
            if (iv) pre[k + 1] = (uint32_t)(carry + x);
            carry += __shfl(x, 63);
        }
    }
    return carry <= MAX_SIZE;
}

// The lane's record and the wave's item range.
struct LaneRecord {
    uint64_t r;
    bool valid;
    uint32_t b, e; // items [b, e) (e = b for lanes past n)
    uint32_t I0, cnt;
    bool fast; // wave-uniform: item-parallel path
};

// cached = the size pass's prefix is read from a.item_pre (write pass with the cache)
template <class IP>
__device__ __forceinline__ LaneRecord lane_record(const NestedEncodeArgs &a, uint32_t *pre, int lane, bool check,
                                                  bool &err, uint64_t blk, bool cached = false) {
    LaneRecord L;
    L.r = blk * NENC_BLOCK + threadIdx.x;
    L.valid = L.r < a.n;
    L.b = a.item_begin[L.valid ? L.r : a.n];
    L.e = L.valid ? a.item_begin[L.r + 1] : L.b;
    const bool bad = L.valid && (L.e < L.b || (uint64_t)L.e > a.nitems);
    L.I0 = __builtin_amdgcn_readfirstlane(L.b);
    const uint32_t I1 = __builtin_amdgcn_readfirstlane(__shfl(L.e, 63));
    L.cnt = I1 - L.I0;
    if (cached) {
        const uint64_t w = (blk * NENC_BLOCK + threadIdx.x) >> 6;
        L.fast = (w << 6) < a.n && a.wave_ok[w] != 0; // (waves past n return before using it)
        if (L.fast) {
            if (lane == 0) pre[0] = 0;
            for (uint32_t k = lane; k < L.cnt; k += 64) pre[k + 1] = a.item_pre[L.I0 + k];
        }
        return L;
    }
    L.fast = __ballot(bad) == 0 && L.cnt <= (uint32_t)NENC_ITEM_CAP;
    if (L.fast) L.fast = wave_item_prefix<IP>(a, L.I0, L.cnt, pre, lane, check, err);
    return L;
}

// Encoded size of the lane's record (valid lanes), list from the prefix or the generic path.
template <class OP>
__device__ __forceinline__ RecSize lane_record_size(const NestedEncodeArgs &a, const LaneRecord &L,
                                                    const typename OP::Rec &orec, const uint32_t *pre, bool check,
                                                    bool &err, ListSize &ls) {
    if (L.fast) {
        ls.count = L.e - L.b;
        ls.data = L.valid ? pre[L.e - L.I0] - pre[L.b - L.I0] : 0;
        ls.big = ls.count > 255 || ls.data > 65535; // IsBigList, internal/format/list.go:40-54
        const uint32_t tsize = ls.count * (ls.big ? 4 : 2);
        ls.total = ls.data + tsize + vlen32((uint32_t)ls.data) + vlen32(tsize) + 1;
    } else {
        ls = L.valid ? list_size(a, L.r, check, err) : ListSize{0, 0, 0, false};
    }
    return OP::size(a.outer, orec, L.r, check, err, KnownListSize{ls.total});
}

// Pass 1: per-block encoded bytes (all-ones on an encoder error).
template <class OP, class IP>
__device__ __forceinline__ void nested_enc_size_body(const NestedEncodeArgs &a, uint8_t *smem) {
    uint64_t *part = (uint64_t *)smem;
    int *errs = (int *)(smem + 164);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t *pre = (uint32_t *)(smem + NENC_HEAD + wave * NENC_PRE);
    if (threadIdx.x == 0) *errs = 0;
    __syncthreads();
    bool err = false;
    const LaneRecord L = lane_record<IP>(a, pre, lane, a.check_heaps, err, blockIdx.x);
    if (a.item_pre && L.r - lane < a.n) { // this wave's prefix and verdict, for the write pass
        if (lane == 0) a.wave_ok[L.r >> 6] = L.fast ? 1 : 0;
        if (L.fast) {
            wave_sync();
            for (uint32_t k = lane; k < L.cnt; k += 64) a.item_pre[L.I0 + k] = pre[k + 1];
        }
    }
    typename OP::Rec orec; // sizes: columns only
    OP::load_cols(a.outer, L.valid ? L.r : a.n - 1, orec);
    ListSize ls;
    const RecSize rs = lane_record_size<OP>(a, L, orec, pre, a.check_heaps, err, ls);
    if (L.valid & err) *errs = 1;
    uint64_t s = L.valid ? rs.total : 0;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) part[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < NENC_BLOCK / 64; w++) t += part[w];
        a.block_sums[blockIdx.x] = *errs ? ~0ull : t;
    }
}

// Pass 3: record offsets from the block scan, ends[], the records' bytes.
template <class OP, class IP>
__device__ __forceinline__ void nested_enc_write_body(const NestedEncodeArgs &a, uint8_t *smem) {
    uint64_t *wsum = (uint64_t *)smem;
    uint8_t *inv_outer = smem + 32, *inv_item = smem + 96;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // blocks dealt to the 8 XCDs in contiguous shares (xcd = 1): neighbouring blocks, whose
    // outputs share a cache line at each boundary, write through one L2
    uint64_t blk = blockIdx.x;
    if (a.xcd) blk = (blockIdx.x & 7) * ((gridDim.x + 7) / 8) + (blockIdx.x >> 3);
    if (blk >= a.nblocks) return;
    const uint64_t total = a.block_sums[a.nblocks], blk_pre = a.block_sums[blk];
    if (threadIdx.x < a.outer.nfields) inv_outer[a.outer.order[threadIdx.x]] = (uint8_t)threadIdx.x;
    if (threadIdx.x < a.item.nfields) inv_item[a.item.order[threadIdx.x]] = (uint8_t)threadIdx.x;
    uint32_t *pre = (uint32_t *)(smem + NENC_HEAD + wave * NENC_WAVE_LDS);
    uint8_t *slab = (uint8_t *)pre + NENC_PRE;

    bool err = false;
    // the outer record's loads first: in flight while the item prefix is built
    const uint64_t r0 = blk * NENC_BLOCK + threadIdx.x;
    const typename OP::Rec orec = OP::load(a.outer, r0 < a.n ? r0 : a.n - 1);
    const LaneRecord L = lane_record<IP>(a, pre, lane, false, err, blk, a.item_pre != nullptr);
    // (checked once the loads above are in flight: nothing is written before this point)
    if (total > a.out_cap) return; // capacity error or encoder error (total == ~0)
    wave_sync(); // the prefix (from the cache) is in LDS
    ListSize ls;
    RecSize rs = lane_record_size<OP>(a, L, orec, pre, false, err, ls);
    if (!L.valid) rs.total = 0;
    uint64_t x = rs.total; // block exclusive scan of sizes
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    lds_barrier();
    uint64_t pre_b = blk_pre;
    for (int w = 0; w < wave; w++) pre_b += wsum[w];
    const uint64_t start = pre_b + x - rs.total;
    if (L.valid) a.ends[L.r] = start + rs.total;

    const uint64_t wbase = blk * NENC_BLOCK + wave * 64;
    if (wbase >= a.n) return;
    const uint64_t S = __builtin_amdgcn_readfirstlane((uint32_t)start) |
                       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(start >> 32)) << 32);
    const int last = (int)((a.n - wbase) < 64 ? a.n - wbase - 1 : 63);
    const uint64_t Ev = __shfl(start + rs.total, last);
    const uint64_t E = __builtin_amdgcn_readfirstlane((uint32_t)Ev) |
                       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(Ev >> 32)) << 32);
    const uint64_t head = ((uint64_t)(a.out + S)) & 15; // slab pos of byte S keeps 16-B phase
    if (!(L.fast && head + (E - S) + 16 <= (uint64_t)NENC_SLAB)) {
        if (L.valid) {
            GlobalSink k{a.out};
            ListEmitter<GlobalSink, long long> le{&a, &k, inv_item};
            emit_message(a.outer, k, (long long)start, L.r, rs, inv_outer, le);
        }
        return;
    }
    LdsSink k{slab, (int)(smem + 160 - slab)}; // dummy dword in the header
    // A: outer records, the items skipped
    WaveListEmit le{pre + (L.b - L.I0), ls.count, (uint32_t)ls.data, ls.big, 0};
    if (L.valid) OP::emit(a.outer, k, (int)(head + (start - S)), L.r, orec, rs, inv_outer, le);
    wave_sync();
    const int lst = le.lstart;
    const bool fix = L.valid && ls.count > 0 && (lst & 3);
    const uint32_t saved = fix ? *(const uint32_t *)(slab + (lst & ~3)) : 0u;
    // the prefix has been read (list tables): each record turns its items' entries into their
    // slab positions, so an item lane reads its position instead of searching for its owner
    if (L.valid && ls.count > 0) {
        const uint32_t k0 = L.b - L.I0, k1 = L.e - L.I0;
        const int delta = lst - (int)pre[k0];
        for (uint32_t q = k0; q < k1; q++) pre[q] = (uint32_t)((int)pre[q] + delta);
    }
    wave_sync();
    // B: items, last chunk first, three chunks in flight: the column loads of chunk c-128 and
    // the heap loads of chunk c-64 (addressed by the spans its column loads brought one
    // iteration earlier) are issued before chunk c is emitted
    int c = ((int)L.cnt - 1) & ~63;
    typename IP::Rec cur, nxt, nn;
    if (c >= 0) {
        const uint32_t kk = (uint32_t)c + lane;
        cur = IP::load(a.item, L.I0 + (kk < L.cnt ? kk : L.cnt - 1));
    }
    if (c >= 64) IP::load_cols(a.item, L.I0 + (uint32_t)(c - 64) + lane, nxt);
    for (; c >= 0; c -= 64) {
        if (c >= 128) IP::load_cols(a.item, L.I0 + (uint32_t)(c - 128) + lane, nn);
        if (c >= 64) IP::load_heaps(a.item, nxt);
        const uint32_t kk = (uint32_t)c + lane;
        const bool iv = kk < L.cnt;
        const uint32_t i = L.I0 + (iv ? kk : 0u);
        const int pos = (int)pre[iv ? kk : 0u];
        if (iv) {
            bool e2 = false;
            const RecSize irs = IP::size(a.item, cur, i, false, e2);
            IP::emit(a.item, k, pos, i, cur, irs, inv_item);
        }
        wave_sync();
        cur = nxt;
        nxt = nn;
    }
    // C: the bytes under the list start that the first item's head store overwrote
    if (fix) {
        uint32_t *d = (uint32_t *)(slab + (lst & ~3));
        const uint32_t m = 0xffffffffu >> (32 - 8 * (lst & 3));
        *d = (saved & m) | (*d & ~m);
    }
    wave_sync();
    copy_slab_out(slab, a.out + S - head, head, head + (E - S), lane);
}


// ---- the write pass on wave PAIRS (schema-specialised outer encoder, size-pass prefix cache) ----
// Items [klo, khi) of the wave's item range (prefix entries already turned into slab positions),
// chunks of 64 from the LAST to the first, three chunks in flight (as nested_enc_write_body B).
template <class IP, class Sink>
__device__ __forceinline__ void emit_item_range(const NestedEncodeArgs &a, const Sink &k, const uint32_t *pre,
                                                uint32_t I0, uint32_t klo, uint32_t khi, const uint8_t *inv_item,
                                                int lane) {
    if (khi <= klo) return;
    auto idx = [&](int cc) {
        const uint32_t kk = (uint32_t)cc + (uint32_t)lane;
        return I0 + (kk < khi ? kk : khi - 1);
    };
    int c = (int)(klo + ((khi - klo - 1) & ~63u));
    typename IP::Rec cur, nxt, nn;
    cur = IP::load(a.item, idx(c));
    if (c - 64 >= (int)klo) IP::load_cols(a.item, idx(c - 64), nxt);
    for (; c >= (int)klo; c -= 64) {
        if (c - 128 >= (int)klo) IP::load_cols(a.item, idx(c - 128), nn);
        if (c - 64 >= (int)klo) IP::load_heaps(a.item, nxt);
        const uint32_t kk = (uint32_t)c + (uint32_t)lane;
        if (kk < khi) {
            const uint32_t i = I0 + kk;
            bool e2 = false;
            const RecSize irs = IP::size(a.item, cur, i, false, e2);
            IP::emit(a.item, k, (int)pre[kk], i, cur, irs, inv_item);
        }
        wave_sync();
        cur = nxt;
        nxt = nn;
    }
}

// A 512-thread block takes the size pass's 256-record block as four 64-record groups, each
// written by a wave PAIR sharing the group's prefix and slab (the same LDS per group as the
// one-wave pass, twice the waves per CU).  Wave 0 emits the records' outer fields before the
// list field (A1) and the items of records [0, R0); wave 1 the items of records [R0, 64)
// concurrently (R0: the record boundary near SPEC_AB_NENC_SPLIT % of the group's items); after a
// barrier wave 0 emits the rest of each record (A2: list table and trailer, later fields, outer
// table and trailer) with an emitter that never stores below its start, and both copy the slab
// out.  Ordering: the HEAD_ST4 emitters of A1 and of the items store whole dwords, the first
// covering <= 3 bytes below its start; those bytes are a previous item's (same wave: written
// later in chunk order, as in the one-wave pass), the record's A1 tail (kept pending across the
// barrier, then stored bytewise) or the previous record's A2 bytes (emitted after the barrier).
// The split is at a record boundary, so no item byte is covered by the other wave's stores.
#ifndef SPEC_AB_NENC_SPLIT
#define SPEC_AB_NENC_SPLIT 45
#endif
// measurement builds only (wrong bytes): skip the items (1), the copy-out (2), the outer records (4)
#ifndef SPEC_AB_NENC_SKIP
#define SPEC_AB_NENC_SKIP 0
#endif
template <class OP, class IP>
__device__ __forceinline__ void nested_enc_write_pair_body(const NestedEncodeArgs &a, uint8_t *smem) {
    constexpr int LF = OP::list_field();
    static_assert(LF >= 0, "the outer schema holds the list field");
    uint64_t *wsum = (uint64_t *)smem;
    uint8_t *inv_outer = smem + 32, *inv_item = smem + 96;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, grp = wave >> 1, half = wave & 1;
    uint64_t blk = blockIdx.x;
    if (a.xcd) blk = (blockIdx.x & 7) * ((gridDim.x + 7) / 8) + (blockIdx.x >> 3);
    if (blk >= a.nblocks) return; // block-uniform
    const uint64_t total = a.block_sums[a.nblocks], blk_pre = a.block_sums[blk];
    if (threadIdx.x < a.outer.nfields) inv_outer[a.outer.order[threadIdx.x]] = (uint8_t)threadIdx.x;
    if (threadIdx.x < a.item.nfields) inv_item[a.item.order[threadIdx.x]] = (uint8_t)threadIdx.x;
    uint32_t *pre = (uint32_t *)(smem + NENC_HEAD + grp * NENC_WAVE_LDS);
    uint8_t *slab = (uint8_t *)pre + NENC_PRE;
    const uint64_t r = blk * NENC_BLOCK + grp * 64 + lane, gbase = blk * NENC_BLOCK + grp * 64;
    const bool valid = r < a.n, live = gbase < a.n; // live: group-uniform
    typename OP::Rec orec;
    if (half == 0) orec = OP::load(a.outer, valid ? r : a.n - 1); // in flight across the prefix
    // the group's items and the size pass's verdict and prefix (both waves load half the prefix)
    const uint32_t b = live ? a.item_begin[valid ? r : a.n] : 0u;
    const uint32_t e = valid ? a.item_begin[r + 1] : b;
    const uint32_t I0 = __builtin_amdgcn_readfirstlane(b);
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(__shfl(e, 63)) - I0;
    const bool fast = live && a.wave_ok[gbase >> 6] != 0;
    if (fast) {
        if (half == 0 && lane == 0) pre[0] = 0;
        for (uint32_t q = (uint32_t)(half * 64 + lane); q < cnt; q += 128) pre[q + 1] = a.item_pre[I0 + q];
    }
    if (total > a.out_cap) return; // capacity or encoder error: block-uniform, before any barrier
    __syncthreads(); // (1) prefix and inverse orders in LDS
    ListSize ls = {0, 0, 0, false};
    RecSize rs = {0, 0, false};
    bool err = false;
    if (half == 0 && live) {
        LaneRecord L;
        L.r = r;
        L.valid = valid;
        L.b = b;
        L.e = e;
        L.I0 = I0;
        L.cnt = cnt;
        L.fast = fast;
        rs = lane_record_size<OP>(a, L, orec, pre, false, err, ls);
        if (!valid) rs.total = 0;
    }
    uint64_t x = rs.total; // group exclusive scan of sizes (wave 0)
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (half == 0 && lane == 63) wsum[grp] = live ? x : 0;
    __syncthreads(); // (2) group sums
    uint64_t S = blk_pre;
    for (int g = 0; g < grp; g++) S += wsum[g];
    const uint64_t E = S + wsum[grp];
    const uint64_t start = S + x - rs.total; // (wave 0)
    const uint64_t head = ((uint64_t)(a.out + S)) & 15;
    const bool staged = live && fast && head + (E - S) + 16 <= (uint64_t)NENC_SLAB; // group-uniform
    if (half == 0 && valid) a.ends[r] = start + rs.total;
    const int p0 = (int)(head + (start - S));
    int lst = 0;
    if (half == 0 && staged && valid) {
        // the list's slab position from the sizes of the fields before it; the record's prefix
        // entries become its items' slab positions
        bool e1 = false;
        lst = p0 + (int)OP::template data_size<0, KnownListSize, LF>(a.outer, orec, r, false, e1, KnownListSize{0});
        if (ls.count > 0) {
            const uint32_t k0 = b - I0, k1 = e - I0;
            const int delta = lst - (int)pre[k0];
            for (uint32_t q = k0; q < k1; q++) pre[q] = (uint32_t)((int)pre[q] + delta);
        }
    }
    // the split: the first record whose items start at or past SPEC_AB_NENC_SPLIT % of the group's
    uint32_t K0 = cnt;
    if (staged) {
        const uint64_t m = __ballot(valid && (uint64_t)(b - I0) * 100 >= (uint64_t)cnt * SPEC_AB_NENC_SPLIT);
        if (m) K0 = __builtin_amdgcn_readlane(b, __builtin_ctzll(m)) - I0;
    }
    __syncthreads(); // (3) item positions
    LdsSink k{slab, (int)(smem + 160 - slab)}; // dummy dword in the header
    typename OP::Rec xo = orec;
    Emit<LdsSink, int, true> em(k, p0);
    if (staged) {
        if (half == 0) {
            if (valid && !(SPEC_AB_NENC_SKIP & 4)) OP::template emit_range<0, LF>(a.outer, em, xo, p0, r); // A1, its tail left pending
            if (!(SPEC_AB_NENC_SKIP & 1)) emit_item_range<IP>(a, k, pre, I0, 0u, K0, inv_item, lane);
        } else if (!(SPEC_AB_NENC_SKIP & 1)) {
            emit_item_range<IP>(a, k, pre, I0, K0, cnt, inv_item, lane);
        }
    } else if (half == 0 && valid) {
        // a group that does not fit the slab (or without the item-parallel verdict): each record
        // straight to HBM on its lane
        GlobalSink g{a.out};
        ListEmitter<GlobalSink, long long> le{&a, &g, inv_item};
        emit_message(a.outer, g, (long long)start, r, rs, inv_outer, le);
    }
    __syncthreads(); // (4) every whole-dword store of A1 and of the items is done
    if (staged && half == 0 && valid && !(SPEC_AB_NENC_SKIP & 4)) {
        // A2: the same emitter from the list field on; the hook stores A1's pending tail bytewise
        // and resumes past the items with their last bytes read back (WaveListEmit merge_slab)
        WaveListEmit le{pre + (b - I0), ls.count, (uint32_t)ls.data, ls.big, 0, slab};
        OP::template emit_range<LF, OP::N>(a.outer, em, xo, p0, r, le);
        OP::emit_table_trailer(em, xo, rs);
        em.finish();
    }
    __syncthreads(); // (5) the group's slab is complete
    if (staged && !(SPEC_AB_NENC_SKIP & 2)) copy_slab_out_t<128>(slab, a.out + S - head, head, head + (E - S), threadIdx.x & 127);
}

} // namespace spec
