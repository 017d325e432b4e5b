// encode_nested.hip — bulk encode of messages with a list<message> field (BASELINE config 4).
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
// Input: outer columns [n], item_begin [n+1] (CSR, uint32) and item columns [m].
// Three launches, no host sync: sizes (record per lane; the lane sums its items' sizes) ->
// scan of block sums -> write (each lane emits its record — items included — into the wave's
// LDS slab; the wave copies the slab out with 16-byte stores; ends written coalesced).
#include <hip/hip_runtime.h>

#include "encode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

namespace {

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

struct ListSizer {
    const NestedEncodeArgs *a;
    bool check;
    bool *err;
    __device__ __forceinline__ uint64_t operator()(uint32_t, uint64_t r) const { return list_size(*a, r, check, *err).total; }
};

__device__ __forceinline__ RecSize outer_size(const NestedEncodeArgs &a, uint64_t r, bool check, bool &err) {
    ListSizer ls{&a, check, &err};
    return record_size(a.outer, r, check, err, ls);
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

__global__ __launch_bounds__(ENC_BLOCK) void nested_enc_size_kernel(NestedEncodeArgs a) {
    __shared__ uint64_t part[ENC_BLOCK / 64];
    __shared__ int errs;
    if (threadIdx.x == 0) errs = 0;
    __syncthreads();
    const uint64_t r = (uint64_t)blockIdx.x * ENC_BLOCK + threadIdx.x;
    uint64_t sz = 0;
    bool err = false;
    if (r < a.n) sz = outer_size(a, r, a.check_heaps, err).total;
    if (err) errs = 1;
    uint64_t s = sz;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < ENC_BLOCK / 64; w++) t += part[w];
        a.block_sums[blockIdx.x] = errs ? ~0ull : t;
    }
}

__global__ __launch_bounds__(1024) void nested_enc_scan_kernel(NestedEncodeArgs a) {
    scan_block_sums(a.block_sums, a.nblocks, a.total);
}

constexpr int NENC_SLAB = 20 * 1024 - 128; // per-wave output staging

__global__ __launch_bounds__(ENC_BLOCK) void nested_enc_write_kernel(NestedEncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint64_t wsum[ENC_BLOCK / 64];
    __shared__ uint8_t inv_outer[SPEC_MAX_FIELDS], inv_item[SPEC_MAX_FIELDS];
    const uint64_t total = a.block_sums[a.nblocks];
    if (total > a.out_cap) return; // capacity error or encoder error (total == ~0)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < a.outer.nfields) inv_outer[a.outer.order[threadIdx.x]] = (uint8_t)threadIdx.x;
    if (threadIdx.x < a.item.nfields) inv_item[a.item.order[threadIdx.x]] = (uint8_t)threadIdx.x;

    const uint64_t r = (uint64_t)blockIdx.x * ENC_BLOCK + threadIdx.x;
    const bool valid = r < a.n;
    bool err = false;
    RecSize rs = {0, 0, false};
    if (valid) rs = outer_size(a, r, false, err);
    uint64_t x = rs.total;
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint64_t pre = a.block_sums[blockIdx.x];
    for (int w = 0; w < wave; w++) pre += wsum[w];
    const uint64_t start = pre + x - rs.total;
    if (valid) a.ends[r] = start + rs.total;

    const uint64_t wbase = (uint64_t)blockIdx.x * ENC_BLOCK + wave * 64;
    if (wbase >= a.n) return;
    const uint64_t S = __builtin_amdgcn_readfirstlane((uint32_t)start) |
                       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(start >> 32)) << 32);
    const int last = (int)((a.n - wbase) < 64 ? a.n - wbase - 1 : 63);
    const uint64_t Ev = __shfl(start + rs.total, last);
    const uint64_t E = __builtin_amdgcn_readfirstlane((uint32_t)Ev) |
                       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(Ev >> 32)) << 32);
    const uint64_t head = ((uintptr_t)(a.out + S)) & 15;
    if (head + (E - S) + 16 <= (uint64_t)NENC_SLAB) {
        uint8_t *slab = smem + wave * NENC_SLAB;
        LdsSink k{slab, 0}; // emit_message never uses the dummy (no HEAD_ST4 emitter)
        if (valid) {
            ListEmitter<LdsSink, int> le{&a, &k, inv_item};
            emit_message(a.outer, k, (int)(head + (start - S)), r, rs, inv_outer, le);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint8_t *gbase = a.out + S - head; // 16-B aligned
        const uint64_t lim = head + (E - S);
        for (uint64_t c = 0; c < lim; c += 1024) {
            uint64_t p = c + (uint64_t)lane * 16;
            if (p >= lim) break;
            if (p >= head && p + 16 <= lim) {
                *(uint4 *)(gbase + p) = *(const uint4 *)(slab + p);
            } else {
                for (int i = 0; i < 16; i++)
                    if (p + i >= head && p + i < lim) gbase[p + i] = slab[p + i];
            }
        }
    } else if (valid) {
        GlobalSink k{a.out};
        ListEmitter<GlobalSink, long long> le{&a, &k, inv_item};
        emit_message(a.outer, k, (long long)start, r, rs, inv_outer, le);
    }
}

} // namespace

int launch_nested_encode(const NestedEncodeArgs &a, bool write, hipStream_t stream) {
    if (a.nblocks)
        hipLaunchKernelGGL(nested_enc_size_kernel, dim3((unsigned)a.nblocks), dim3(ENC_BLOCK), 0, stream, a);
    hipLaunchKernelGGL(nested_enc_scan_kernel, dim3(1), dim3(1024), 0, stream, a);
    if (write && a.nblocks)
        hipLaunchKernelGGL(nested_enc_write_kernel, dim3((unsigned)a.nblocks), dim3(ENC_BLOCK),
                           (size_t)(ENC_BLOCK / 64) * NENC_SLAB, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
