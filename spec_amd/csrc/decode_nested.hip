// decode_nested.hip — bulk decode of messages with a list<message> field (BASELINE config 4).
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
// Two calls (no host sync inside either):
//   spec_decode_nested_index: nested_count_kernel (per 64-record group: item total) +
//     nested_scan_kernel (exclusive scan of group totals in the workspace, total items);
//   spec_decode_nested: nested_decode_kernel — per group: stage the span into LDS (as the
//     flat decoder), decode each outer record (one lane per record), wave prefix-sum of the
//     item counts => item_begin, then decode the group's items ITEM-PARALLEL: item j of the
//     group goes to lane j % 64 (owner record found by a binary search over the lanes' prefix
//     sums with ds_bpermute), so item columns are written coalesced and no lane idles on a
//     short list.
#include <hip/hip_runtime.h>

#include "decode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

namespace {

// What OpenList(m.field(tag)) gives: count and where the table / data are (source positions).
struct ListInfo {
    uint32_t count;
    long long dstart, tstart; // list data start, table start
    uint32_t dsize;
    bool big;
};

template <class Src>
__device__ __forceinline__ ListInfo list_open(const Src &s, const RecInfo &ri, const NestedArgs &a) {
    ListInfo li = {0, 0, 0, 0, false};
    const long long end = rec_field_end(s, ri, a.list_tag, a.list_rank);
    if (end <= 0) return li; // absent or empty => empty list
    using pos_t = typename Src::pos_t;
    const pos_t lo = (pos_t)ri.tr.dstart, e = lo + (pos_t)end;
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
__device__ __forceinline__ Group stage(const NestedArgs &a, __amdgpu_buffer_rsrc_t rsrc, uint8_t *slab, uint64_t base,
                                       int lane) {
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

// Item count of record [rs, re).
template <class Src>
__device__ __forceinline__ uint32_t record_count(const Src &s, long long rs, long long re, const NestedArgs &a) {
    const RecInfo ri = rec_open(s, (typename Src::pos_t)rs, (typename Src::pos_t)re);
    return list_open(s, ri, a).count;
}

// Decode a group: outer records (lane = record), then items (item-parallel).
template <class Src>
__device__ __forceinline__ void decode_group(const Src &s, long long rs, long long re, bool valid, uint64_t r,
                                             uint64_t item_base, int lane, long long to_stream,
                                             const NestedArgs &a) {
    using pos_t = typename Src::pos_t;
    ListInfo li = {0, 0, 0, 0, false};
    if (valid) {
        decode_record_generic(s, (pos_t)rs, (pos_t)re, r, a.outer, to_stream);
        const RecInfo ri = rec_open(s, (pos_t)rs, (pos_t)re);
        li = list_open(s, ri, a);
    }
    const uint32_t incl = wave_incl_scan(li.count, lane);
    const uint32_t excl = incl - li.count;
    const uint32_t total = __shfl(incl, 63);
    if (valid) {
        a.item_begin[r] = (uint32_t)(item_base + excl);
        if (r == a.n - 1) a.item_begin[a.n] = (uint32_t)(item_base + incl);
    }
    for (uint32_t j0 = 0; j0 < total; j0 += 64) {
        const uint32_t j = j0 + lane;
        // owner: the largest lane whose exclusive prefix is <= j (it has count > 0)
        int l = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1) {
            const uint32_t ex = __shfl(excl, l + step < 64 ? l + step : 63);
            if (l + step < 64 && ex <= j) l += step;
        }
        const uint32_t i = j - __shfl(excl, l);
        const long long ldstart = __shfl(li.dstart, l);
        const long long ltstart = __shfl(li.tstart, l);
        const uint32_t ldsize = __shfl(li.dsize, l);
        const bool lbig = __shfl((int)li.big, l) != 0;
        if (j >= total) continue;
        const uint64_t out = item_base + j;
        if (out >= a.item_cap) continue;
        // List.GetBytes(i), internal/types/list.go:100-116 with format.ListTable.Offset
        uint32_t start, end;
        if (lbig) {
            end = be32_at(s, ltstart + 4ll * i);
            start = i ? be32_at(s, ltstart + 4ll * (i - 1)) : 0;
        } else {
            end = be16_at(s, ltstart + 2ll * i);
            start = i ? be16_at(s, ltstart + 2ll * (i - 1)) : 0;
        }
        if (end > ldsize) {
            // nil item => OpenItemErr(nil): empty message, zero fields, no error
            decode_record_generic(s, (pos_t)0, (pos_t)0, out, a.item, to_stream);
        } else if (start > end) {
            decode_record_generic(s, (pos_t)0, (pos_t)0, out, a.item, to_stream);
            if (a.item.status) a.item.status[out] = ST_PANIC;
        } else {
            const pos_t ib = (pos_t)(ldstart + start), ie = (pos_t)(ldstart + end);
            decode_record_generic(s, ib, ie, out, a.item, to_stream);
        }
    }
}

__global__ __launch_bounds__(256) void nested_count_kernel(NestedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * DEC_WAVES + wave;
    const uint64_t base = g * 64;
    if (base >= a.n) return;
    uint8_t *slab = smem + wave * a.slab;
    __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.stream, (short)0, (int)(uint32_t)a.stream_len, 0x00020000);
    const Group gr = stage(a, rsrc, slab, base, lane);
    const bool valid = base + lane < a.n;
    uint32_t cnt = 0;
    if (valid) {
        if (gr.in_lds) {
            LdsSrc s{(lds_u8 *)slab};
            cnt = record_count(s, SLAB_GUARD + (long long)(gr.rec_lo - gr.aligned_lo),
                               SLAB_GUARD + (long long)(gr.rec_hi - gr.aligned_lo), a);
        } else {
            GlobalSrc s{rsrc, a.stream_len};
            cnt = record_count(s, (long long)gr.rec_lo, (long long)gr.rec_hi, a);
        }
    }
    const uint32_t sum = wave_sum(cnt);
    if (lane == 0) a.group_base[g] = sum;
}

// Exclusive scan of the group totals (one 1024-thread workgroup, chunked) + total items.
__global__ __launch_bounds__(1024) void nested_scan_kernel(NestedArgs a) {
    __shared__ uint64_t part[1024 / 64];
    __shared__ uint64_t carry;
    const uint64_t ngroups = (a.n + 63) / 64;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint64_t c0 = 0; c0 < ngroups; c0 += 1024) {
        const uint64_t i = c0 + t;
        const uint64_t v = i < ngroups ? a.group_base[i] : 0;
        uint64_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint64_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) part[w] = x;
        __syncthreads();
        if (t == 0) {
            uint64_t run = carry;
            for (int k = 0; k < 1024 / 64; k++) {
                uint64_t p = part[k];
                part[k] = run;
                run += p;
            }
            carry = run;
        }
        __syncthreads();
        if (i < ngroups) a.group_base[i] = part[w] + x - v;
        __syncthreads();
    }
    if (t == 0) *a.total = carry;
}

__global__ __launch_bounds__(256) void nested_decode_kernel(NestedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t g = (uint64_t)blockIdx.x * DEC_WAVES + wave;
    const uint64_t base = g * 64;
    if (base >= a.n) return;
    uint8_t *slab = smem + wave * a.slab;
    __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.stream, (short)0, (int)(uint32_t)a.stream_len, 0x00020000);
    const Group gr = stage(a, rsrc, slab, base, lane);
    const uint64_t r = base + lane;
    const bool valid = r < a.n;
    const uint64_t item_base = a.group_base[g];
    if (gr.in_lds) {
        LdsSrc s{(lds_u8 *)slab};
        decode_group(s, SLAB_GUARD + (long long)(gr.rec_lo - gr.aligned_lo),
                     SLAB_GUARD + (long long)(gr.rec_hi - gr.aligned_lo), valid, r, item_base, lane,
                     (long long)gr.aligned_lo - SLAB_GUARD, a);
    } else {
        GlobalSrc s{rsrc, a.stream_len};
        decode_group(s, (long long)gr.rec_lo, (long long)gr.rec_hi, valid, r, item_base, lane, 0, a);
    }
}

} // namespace

int launch_nested_index(NestedArgs a, double avg_record, hipStream_t stream) {
    if (a.n == 0) {
        (void)hipMemsetAsync(a.total, 0, sizeof(uint64_t), stream);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    a.slab = decode_slab_bytes(avg_record);
    const uint64_t groups = (a.n + 63) / 64;
    dim3 grid((unsigned)((groups + DEC_WAVES - 1) / DEC_WAVES)), block(64 * DEC_WAVES);
    hipLaunchKernelGGL(nested_count_kernel, grid, block, (size_t)DEC_WAVES * a.slab, stream, a);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(nested_scan_kernel, dim3(1), dim3(1024), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_nested_decode(NestedArgs a, double avg_record, hipStream_t stream) {
    if (a.n == 0) return 0;
    a.slab = decode_slab_bytes(avg_record);
    const uint64_t groups = (a.n + 63) / 64;
    dim3 grid((unsigned)((groups + DEC_WAVES - 1) / DEC_WAVES)), block(64 * DEC_WAVES);
    hipLaunchKernelGGL(nested_decode_kernel, grid, block, (size_t)DEC_WAVES * a.slab, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
