// validate.hip — bulk ParseMessage / ParseList / ParseValue: recursive validation of every record
// (SURVEY.md §8(f) #2).
//
// What mpx runs on every received frame (mpx/conn_reader.go:119: pmpx.ParseMessage):
//   ParseMessage(b)  internal/types/msg.go:58-82  — DecodeMessageTable, then ParseValue on
//                    every non-empty field slice m.bytes[:end_i] in table order (fieldAt,
//                    msg.go:477-486: end > dataSize => nil, skipped)
//   ParseList(b)     internal/types/list.go:35-53 — DecodeListTable, then ParseValue on every
//                    non-empty element (GetBytes: end > dataSize => nil; start > end panics)
//   ParseValue(b)    internal/types/value.go:49-113 — per type: the decoder's error checks,
//                    recursion into lists/messages, "unsupported type" otherwise.
// One lane per record, depth-first with an explicit stack of VAL_MAX_DEPTH frames (the reference
// recurses).  Records are staged in LDS like the decoders'; larger spans parse from HBM.  A record
// nested deeper than VAL_MAX_DEPTH is listed and parsed again by deep_kernel (round 6; the call
// returned SPEC_STATUS_TOO_DEEP for it before) with its stack in an HBM arena: 8,192 frames per
// thread, then, for a record deeper still, DEEP_ARENA / sizeof(Frame) = 2,097,152 frames on one
// thread.  Only deeper nesting reports SPEC_STATUS_TOO_DEEP: the reference's recursion (ParseValue
// -> ParseMessage / ParseList -> ParseValue per level) would exhaust Go's 1 GB goroutine stack at a
// depth of that order and crash.
#include <hip/hip_runtime.h>

#include "decode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

namespace {

constexpr int VAL_MAX_DEPTH = 32;

struct Frame {
    long long base, tstart; // data start, table start (source positions)
    uint32_t nent, i, dsize;
    uint8_t list, big;
};

// the main pass's stack (registers / scratch) and the deep pass's (a slice of the HBM arena)
struct LocalStack {
    Frame f[VAL_MAX_DEPTH];
    static constexpr int cap = VAL_MAX_DEPTH;
    __device__ __forceinline__ Frame &operator[](int i) { return f[i]; }
};
struct ArenaStack {
    Frame *f;
    int cap;
    __device__ __forceinline__ Frame &operator[](int i) const { return f[i]; }
};

// the deep pass's workspace (stream-ordered scratch of the call): the records the main pass found
// too deep, then the frame arena
constexpr uint32_t DEEP_LIST_CAP = 1u << 16;
constexpr size_t DEEP_ARENA = 64ull << 20;
constexpr int DEEP_THREADS = 256;
struct DeepWs {
    uint32_t count, pad;
    uint32_t list[DEEP_LIST_CAP];
};
constexpr size_t DEEP_WS_BYTES = ((sizeof(DeepWs) + 255) & ~(size_t)255) + DEEP_ARENA;

// The decoder error checks ParseValue runs for a scalar of type `type` ending at e, and the size
// it reports (value.go:49-113: n = bytes the decoder consumed from the end): 0 ok, 1 an error,
// 2 a Go panic (value.go:110 returns b[len(b)-n:]: DecodeStruct does not bound its data size, so
// a struct larger than its slice panics).
template <class Src>
__device__ __forceinline__ int scalar_check(const Src &s, uint32_t type, long long lo, long long e, uint32_t &n) {
    const long long flen = e - lo;
    const Tail t = load_tail(s, (typename Src::pos_t)e);
    const uint64_t R = tail_r(t);
    const uint32_t R2 = tail_r2(t);
    const long long avail = flen - 1;
    int m;
    n = 0;
    switch (type) {
    case T_TRUE:
    case T_FALSE: n = 1; return 0;
    case T_BYTE: n = 2; return flen >= 2 ? 0 : 1;                     // byte.go:16-34
    case T_INT16: {                                                  // int.go:16-62
        const int32_t x = unzigzag32((uint32_t)rvarint_bf(R, R2, avail, 5, m));
        n = 1 + (uint32_t)m;
        return m >= 0 && x >= -32768 && x <= 32767 ? 0 : 1;
    }
    case T_INT32:
    case T_UINT32: rvarint_bf(R, R2, avail, 5, m); n = 1 + (uint32_t)m; return m >= 0 ? 0 : 1; // int.go:64-103
    case T_INT64:
    case T_UINT64: rvarint_bf(R, R2, avail, 10, m); n = 1 + (uint32_t)m; return m >= 0 ? 0 : 1; // int.go:105-135
    case T_UINT16: {                                                 // uint.go:16-56
        const uint64_t x = rvarint_bf(R, R2, avail, 5, m);
        n = 1 + (uint32_t)m;
        return m >= 0 && x <= 0xffff ? 0 : 1;
    }
    case T_BIN64: n = 9; return flen >= 9 ? 0 : 1;                   // bin.go:15-112
    case T_BIN128: n = 17; return flen >= 17 ? 0 : 1;
    case T_BIN256: n = 33; return flen >= 33 ? 0 : 1;
    case T_FLOAT32: {                                                // float.go:15-32: +-Inf > MaxFloat32
        const uint32_t b = (uint32_t)(R & 0xffffffffu);
        n = 5;
        return flen >= 5 && (b & 0x7fffffffu) != 0x7f800000u ? 0 : 1;
    }
    case T_FLOAT64: n = 9; return flen >= 9 ? 0 : 1;                 // float.go:34-49
    case T_BYTES: {                                                  // bytes.go:14-58
        const uint32_t ds = (uint32_t)rvarint_bf(R, R2, avail, 5, m);
        n = 1 + (uint32_t)m + ds;
        return m >= 0 && (e - 1 - m) - (long long)ds >= lo ? 0 : 1;
    }
    case T_STRING: {                                                 // string.go:15-47 (+1: the NUL)
        const uint32_t ds = (uint32_t)rvarint_bf(R, R2, avail, 5, m);
        const long long end = e - 1 - m - 1;
        n = 2 + (uint32_t)m + ds;
        return m >= 0 && end >= lo && end - (long long)ds >= lo ? 0 : 1;
    }
    case T_STRUCT: {                                                 // struct.go:14-42 (no bound check)
        const uint32_t ds = (uint32_t)rvarint_bf(R, R2, avail, 5, m);
        if (m < 0) return 1;
        const long long size = 1 + (long long)m + ds;
        n = (uint32_t)size;
        return size > flen ? 2 : 0;
    }
    }
    return 1; // "unsupported type", value.go:103-104
}

template <class Src>
__device__ __forceinline__ uint32_t be_at(const Src &s, long long p, int bytes) {
    uint32_t v = 0;
    for (int k = 0; k < bytes; k++) v = (v << 8) | s.u8((typename Src::pos_t)(p + k));
    return v;
}

// ParseMessage (root PARSE_MESSAGE), ParseList (PARSE_LIST) or ParseValue (PARSE_VALUE) of record
// [rs, re): status and size (the parsed size; 0 on error).
template <class Src, class Stack>
__device__ __forceinline__ uint32_t parse_record(const Src &s, long long rs, long long re, uint32_t root,
                                                 uint32_t &size, Stack &stk) {
    using pos_t = typename Src::pos_t;
    size = 0;
    bool list = root == SPEC_PARSE_LIST;
    if (root == SPEC_PARSE_VALUE) {
        if (re <= rs) return ST_INVALID_VALUE; // DecodeType(empty) = TypeUndefined: "unsupported type 0"
        const uint32_t type = s.u8((pos_t)(re - 1));
        if (type != T_LIST && type != T_BIG_LIST && type != T_MESSAGE && type != T_BIG_MESSAGE) {
            uint32_t n;
            const int r = scalar_check(s, type, rs, re, n);
            if (r) return r == 2 ? ST_PANIC : ST_INVALID_VALUE;
            size = n;
            return ST_OK;
        }
        list = type == T_LIST || type == T_BIG_LIST;
    }
    if (re <= rs) return ST_OK; // empty input: zero message / list, no error
    const Trailer top = list ? parse_trailer<true>(s, (pos_t)rs, (pos_t)re) : parse_trailer<false>(s, (pos_t)rs, (pos_t)re);
    if (top.st != ST_OK) return root == SPEC_PARSE_VALUE ? (uint32_t)ST_INVALID_VALUE : top.st;
    int sp = 0;
    const uint32_t es0 = list ? (top.big ? 4u : 2u) : (top.big ? 6u : 3u);
    stk[sp++] = Frame{top.dstart, top.tstart, top.tsize / es0, 0, top.dsize, (uint8_t)list, (uint8_t)top.big};
    while (sp > 0) {
        Frame &f = stk[sp - 1];
        if (f.i >= f.nent) {
            sp--;
            continue;
        }
        const uint32_t i = f.i++;
        long long lo = f.base, e;
        if (!f.list) { // fieldAt(i): table entry i's end
            const uint32_t end = f.big ? be_at(s, f.tstart + 6ll * i + 2, 4) : be_at(s, f.tstart + 3ll * i + 1, 2);
            if (end > f.dsize) continue; // nil
            e = f.base + end;
        } else { // GetBytes(i)
            const int w = f.big ? 4 : 2;
            const uint32_t end = be_at(s, f.tstart + (long long)w * i, w);
            const uint32_t start = i ? be_at(s, f.tstart + (long long)w * (i - 1), w) : 0;
            if (end > f.dsize) continue; // nil
            if (start > end) return ST_PANIC; // Go: slice bounds out of range
            lo = f.base + start;
            e = f.base + end;
        }
        if (e <= lo) continue; // empty value: skipped
        const uint32_t type = s.u8((pos_t)(e - 1));
        if (type == T_LIST || type == T_BIG_LIST || type == T_MESSAGE || type == T_BIG_MESSAGE) {
            const bool sub = type == T_LIST || type == T_BIG_LIST;
            const Trailer tr = sub ? parse_trailer<true>(s, (pos_t)lo, (pos_t)e) : parse_trailer<false>(s, (pos_t)lo, (pos_t)e);
            if (tr.st != ST_OK) return ST_INVALID_VALUE;
            if (sp == stk.cap) return ST_TOO_DEEP;
            const uint32_t es = sub ? (tr.big ? 4u : 2u) : (tr.big ? 6u : 3u);
            stk[sp++] = Frame{tr.dstart, tr.tstart, tr.tsize / es, 0, tr.dsize, (uint8_t)sub, (uint8_t)tr.big};
        } else {
            uint32_t n;
            const int r = scalar_check(s, type, lo, e, n);
            if (r) return r == 2 ? ST_PANIC : ST_INVALID_VALUE;
        }
    }
    size = (uint32_t)(re - top.dstart);
    return ST_OK;
}

__global__ __launch_bounds__(256) void parse_kernel(DecodeArgs a, uint32_t *sizes, uint32_t root, DeepWs *deep) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t base = a.r0 + ((uint64_t)blockIdx.x * (blockDim.x >> 6) + wave) * 64;
    if (base >= a.n) return;
    const uint64_t r = base + lane;
    const bool valid = r < a.n;
    uint8_t *slab = smem + wave * a.slab;
    __amdgpu_buffer_rsrc_t rsrc =
        uniform_rsrc(a.stream, a.stream_len);
    uint64_t lo, hi;
    load_group_ends(a, base, lane, lo, hi);
    const Group gr = make_group(a, base, lane, lo, hi, a.slab);
    uint32_t st = ST_OK, size = 0;
    if (gr.in_lds) {
        issue_dma(rsrc, slab, gr, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        fix_stream_tail(a, rsrc, slab, gr, lane);
        if (!valid) return;
        LdsSrc s{(lds_u8 *)slab};
        LocalStack stk;
        st = parse_record(s, SLAB_GUARD + (long long)(gr.rec_lo - gr.aligned_lo),
                          SLAB_GUARD + (long long)(gr.rec_hi - gr.aligned_lo), root, size, stk);
    } else {
        if (!valid) return;
        GlobalSrc s{a.stream, a.stream_len};
        LocalStack stk;
        st = parse_record(s, (long long)gr.rec_lo, (long long)gr.rec_hi, root, size, stk);
    }
    a.f.status[r] = (uint8_t)st;
    if (sizes) sizes[r] = size;
    if (st == ST_TOO_DEEP) { // for the deep pass
        const uint32_t j = atomicAdd(&deep->count, 1u);
        if (j < DEEP_LIST_CAP) deep->list[j] = (uint32_t)(r - a.r0);
    }
}

// The records the main pass found nested deeper than VAL_MAX_DEPTH, parsed from HBM with their
// stacks in the arena: DEEP_THREADS threads with 8,192 frames each, then one thread with the whole
// arena for any still too deep.  More than DEEP_LIST_CAP such records: every record's status is
// scanned instead.  Exits at once when the main pass listed none.
__device__ __forceinline__ void deep_one(const DecodeArgs &a, uint32_t *sizes, uint32_t root, uint64_t r,
                                         ArenaStack stk) {
    const uint64_t lo = (r == 0 ? 0 : a.ends[r - 1]) + a.head, hi0 = a.ends[r];
    const uint64_t hi = hi0 < lo ? lo : hi0;
    GlobalSrc s{a.stream, a.stream_len};
    uint32_t size = 0;
    const uint32_t st = parse_record(s, (long long)lo, (long long)hi, root, size, stk);
    a.f.status[r] = (uint8_t)st;
    if (sizes) sizes[r] = size;
}

__global__ __launch_bounds__(DEEP_THREADS) void deep_kernel(DecodeArgs a, uint32_t *sizes, uint32_t root, DeepWs *deep) {
    const uint32_t count = deep->count;
    if (count == 0) return;
    Frame *arena = (Frame *)((uint8_t *)deep + ((sizeof(DeepWs) + 255) & ~(size_t)255));
    const int slice = (int)(DEEP_ARENA / sizeof(Frame) / DEEP_THREADS);
    const bool listed = count <= DEEP_LIST_CAP;
    const uint64_t m = listed ? count : a.n - a.r0;
    for (uint64_t j = threadIdx.x; j < m; j += DEEP_THREADS) {
        const uint64_t r = a.r0 + (listed ? deep->list[j] : j);
        if (a.f.status[r] == ST_TOO_DEEP) deep_one(a, sizes, root, r, ArenaStack{arena + threadIdx.x * slice, slice});
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint64_t j = 0; j < m; j++) {
            const uint64_t r = a.r0 + (listed ? deep->list[j] : j);
            if (a.f.status[r] == ST_TOO_DEEP)
                deep_one(a, sizes, root, r, ArenaStack{arena, (int)(DEEP_ARENA / sizeof(Frame))});
        }
    }
}

} // namespace

int launch_parse(DecodeArgs a, uint32_t *sizes, uint32_t root, double avg_record, hipStream_t stream) {
    if (a.n <= a.r0) return 0;
    const DecodeLaunch L = decode_launch(a.n - a.r0, avg_record, device_cus(), false, 1);
    a.slab = L.slab;
    // the deep pass's list and arena: stream-ordered scratch of this call
    DeepWs *deep = nullptr;
    if (hipMallocAsync((void **)&deep, DEEP_WS_BYTES, stream) != hipSuccess) return -1;
    if (hipMemsetAsync(deep, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
    hipLaunchKernelGGL(parse_kernel, dim3(L.blocks), dim3(64 * L.wpb), L.lds, stream, a, sizes, root, deep);
    hipLaunchKernelGGL(deep_kernel, dim3(1), dim3(DEEP_THREADS), 0, stream, a, sizes, root, deep);
    if (hipFreeAsync(deep, stream) != hipSuccess) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
