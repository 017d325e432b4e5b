// frames_device.hip — spec_frames_index_device: the mpx frame index (mpx/conn_reader.go:179-194:
// `[u32 BE size][message]` frames back to back) computed on the GPU, with exactly the results of
// the host walk spec_frames_index (capi.hip).
//
// The head chain is serial (frame k+1 starts where frame k ends), so the walk is split:
//   1. segments of 32 KiB, staged in LDS; for EVERY entry offset e < W (2048) of a segment, the
//      chain is walked to the segment end: exit offset into the next segment, frames completed.
//      Inside the segment the walk is itself split into 8 sub-segments of 4 KiB: every entry
//      o < WS (1024) of sub-segments 1..7 is walked to the first position past its sub-segment
//      that lies in some later sub-segment's window (or past the segment end), the results kept
//      in LDS; a segment entry then walks sub-segment 0 and composes the tables (at most 7
//      dependent LDS reads), so no thread walks more than ~4 KiB of frames (a false entry reads a
//      random big size and leaves at once).  Entries that leave the segment (live: the true one
//      and the others on the same chain, ~8 per segment) keep their pieces for step 5;
//   2. groups of 16 segments compose their tables (every entry, 16 dependent table reads), and
//      super-groups of 16 groups compose those (every entry, 16 reads);
//   3. one thread chains the super-groups from offset 0 (nseg / 256 dependent reads);
//   4. each super-group resolves its groups' entries and frame bases, each group its segments';
//   5. each segment on the chain: one lane per sub-segment piece of its true chain (from the
//      live record of its entry) reads the heads from HBM and writes ends[]; a segment without a
//      record (the chain ends in it) rebuilds its tables in LDS (a short work list).
// A frame that straddles a segment boundary by W bytes or more, or a segment with more than
// 4096 frames, sets the overflow flag: a single-thread serial walk over HBM then produces the
// same results (slow but exact).  One call, no host sync; count / consumed / status land in
// device memory.
#include <hip/hip_runtime.h>

#include "spec_internal.hpp"

namespace spec {

namespace {

constexpr uint32_t FI_SEG = 32768, FI_W = 2048, FI_STEPCAP = 4096;
constexpr uint32_t FI_G1 = 16, FI_G2 = 16; // segments per group, groups per super-group
constexpr uint32_t FI_BLOCK = 1024; // threads of the segment / group kernels (a constant: blockDim
                                    // is a load from the dispatch packet)
constexpr uint32_t FI_SUB = 4096, FI_NSUB = FI_SEG / FI_SUB, FI_WS = 512;
// LDS: the segment (+16 halo), T (window walks), C (segment-entry walks), the survivor list
constexpr uint32_t FI_LDS_T = FI_SEG + 16, FI_LDS = FI_LDS_T + (FI_NSUB - 1) * FI_WS * 4;
constexpr uint32_t FI_LDS_L = FI_LDS + FI_W * 4, FI_LDS_END = FI_LDS_L + ((FI_NSUB - 1) * FI_WS + FI_W) * 4;
// a segment table entry: exit x (< W) | frames << 16; FI_TERM | position | frames << 16; FI_OVF
constexpr uint32_t FI_CNT_SHIFT = 16, FI_CNT_MASK = 0x1fffu, FI_POS_MASK = 0x7fffu;
// a sub-segment walk result: [31] TERM, [30:17] frames, [16:0] segment-relative position
// a segment's live entries (walks that leave it): entry, then per sub-segment piece of its chain
// (position << 16 | frames before it, ~0u where the chain jumps over the sub-segment)
constexpr uint32_t FI_LIVE = 32, FI_LREC = 1 + FI_NSUB;
constexpr uint32_t FI_T_TERM = 1u << 31, FI_T_OVF = 0xffffffffu, FI_T_POS = 0x1ffffu;
constexpr uint32_t FI_OVF = 0xffffffffu, FI_TERM = 0x80000000u, FI_NONE = 0xffffffffu;
constexpr uint64_t FI_G_TERM = 1ull << 63, FI_G_OVF = 1ull << 62;

struct FiArgs {
    const uint8_t *buf;
    uint64_t len, cap;
    uint64_t *ends, *count, *consumed;
    int32_t *status;
    uint32_t nseg, ng1, ng2;
    uint32_t *exitT;           // [nseg * W] packed: exit / TERM position, frames
    uint64_t *g1T, *g2T;       // [ng1 * W], [ng2 * W]: entry into the next, FI_G_TERM | position, FI_G_OVF
    uint32_t *g1Cnt, *g2Cnt;   // frames
    uint32_t *g1_entry;        // [ng1]
    uint64_t *g1_base;         // [ng1]
    uint32_t *g2_entry;        // [ng2]
    uint64_t *g2_base;         // [ng2]
    uint32_t *seg_entry;       // [nseg]
    uint64_t *seg_base;        // [nseg]
    uint64_t *misc;            // [0] overflow, [1] total frames, [2] consumed
    uint32_t *live_n;          // [nseg] live entries recorded (may exceed FI_LIVE)
    uint32_t *live;            // [nseg * FI_LIVE * FI_LREC]
    uint32_t *work;            // [1 + nseg] count, then segments the emit must rebuild
};

// A workgroup barrier for LDS data only: __syncthreads also waits for every global load and
// store in flight (vmcnt), which would stall on the next segment's prefetch and on this
// segment's table stores.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// the big-endian u32 at byte o of the staged segment: two dword reads and a funnel shift
__device__ __forceinline__ uint32_t be32_lds(const uint8_t *l, uint32_t o) {
    const uint32_t *w = (const uint32_t *)l;
    const uint64_t d = ((uint64_t)w[(o >> 2) + 1] << 32) | w[o >> 2];
    return __builtin_bswap32((uint32_t)(d >> (8 * (o & 3))));
}

constexpr uint32_t FI_QPT = FI_SEG / 16 / FI_BLOCK; // 16-byte quads of a segment per thread
static_assert(FI_QPT == 2 && FI_QPT * 16 * FI_BLOCK == FI_SEG, "two 16-byte quads of a segment per thread");

// a segment the quad path stages: whole (with its 16 halo bytes) from a 16-byte aligned buffer
// (the ABI only promises 4-byte alignment: other buffers, and the tail, take the dword loop)
__device__ __forceinline__ bool quad_segment(const FiArgs &a, uint64_t s0) {
    return s0 + FI_SEG + 16 <= a.len && ((uintptr_t)a.buf & 15) == 0;
}

// bytes [s0, s0 + SEG + 16) of buf into lds (zeros past len; buf is 4-byte aligned), then a barrier
__device__ __forceinline__ void stage_segment(const FiArgs &a, uint64_t s0, uint8_t *lds) {
    if (quad_segment(a, s0)) {
        const uint4 *src = (const uint4 *)(a.buf + s0);
        uint4 *dst = (uint4 *)lds;
        const uint4 v0 = src[threadIdx.x], v1 = src[threadIdx.x + FI_BLOCK];
        dst[threadIdx.x] = v0;
        dst[threadIdx.x + FI_BLOCK] = v1;
        if (threadIdx.x == 0) dst[FI_SEG / 16] = src[FI_SEG / 16];
        __syncthreads();
        return;
    }
    uint32_t *l32 = (uint32_t *)lds;
    for (uint32_t i = threadIdx.x; i < (FI_SEG + 16) / 4; i += FI_BLOCK) {
        const uint64_t p = s0 + 4ull * i;
        uint32_t w = 0;
        if (p + 4 <= a.len) {
            w = *(const uint32_t *)(a.buf + p);
        } else {
            for (uint32_t b = 0; b < 4; b++)
                if (p + b < a.len) w |= (uint32_t)a.buf[p + b] << (8 * b);
        }
        l32[i] = w;
    }
    __syncthreads();
}

// The walks of a staged segment.  Jobs j < NT = (NSUB-1) * WS: entry j % WS of the window of
// sub-segment 1 + j / WS, into T[j]; then, with `entries`, the W segment entries e = j - NT of
// sub-segment 0, into C[e] right after T.  A walk follows the chain until it stands on a
// position at or past its stop (the next sub-segment) that lies in the first WS bytes of a
// sub-segment, or past the segment end (segend = s1 - s0, lenrel = len - s0).  A jump W or more
// past the segment end, or more than STEPCAP frames, is overflow (the serial fallback).
//  1. every job takes its first step at once (one LDS read per job, no loop): nearly all of
//     them (a false entry reads a random big size) finish there; the survivors (job, position
//     after the first step) are appended to a list in LDS;
//  2. the survivors are walked, one frame step per iteration with 32-bit arithmetic (the size
//     saturates; the exact TERM test only decides a finished walk's code), shared out to the
//     waves 64 at a time — the others skip the loop — and handed to whichever lanes just
//     finished (ballot + mbcnt).
// Then a barrier.  *nsurv (LDS) must be 0 on entry; it is 0 again on return.
__device__ __forceinline__ void fi_tables(const FiArgs &a, uint64_t s0, uint32_t segend, uint8_t *lds, bool entries,
                                          uint32_t *nsurv) {
    constexpr uint32_t NT = (FI_NSUB - 1) * FI_WS, NWAVES = FI_BLOCK / 64;
    static_assert(FI_LDS == FI_LDS_T + NT * 4, "C follows T");
    static_assert((FI_SUB - FI_WS) == 0xe00u, "window test by mask");
    static_assert(NT + FI_W <= (1u << 13) && FI_SEG + FI_W <= (1u << 19), "a survivor packs job | position << 13");
    uint32_t *out = (uint32_t *)(lds + FI_LDS_T), *list = (uint32_t *)(lds + FI_LDS_L);
    const uint64_t lenrel = a.len - s0;
    const uint32_t far = (uint32_t)((uint64_t)segend + FI_W < lenrel + 1 ? (uint64_t)segend + FI_W : lenrel + 1);
    const uint32_t njobs = entries ? NT + FI_W : NT;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    auto stop_of = [](uint32_t j) -> uint32_t { return j < NT ? (2 + j / FI_WS) * FI_SUB : FI_SUB; };
    // 1. first steps
    for (uint32_t j = threadIdx.x; j < (NT + FI_W + FI_BLOCK - 1) / FI_BLOCK * FI_BLOCK; j += FI_BLOCK) {
        const bool valid = j < njobs;
        const uint32_t p = j < NT ? (1 + j / FI_WS) * FI_SUB + j % FI_WS : j - NT;
        const uint32_t v = be32_lds(lds, p & (FI_SEG - 1));
        const uint32_t q = p + 4 + (v < 0x7fffffffu ? v : 0x7fffffffu);
        const bool exit = p >= segend, fin = exit | (q >= far);
        if (valid & fin) out[j] = exit ? p : (uint64_t)p + 4 + v > lenrel ? FI_T_TERM | p : FI_T_OVF;
        const bool alive = valid & !fin;
        const uint64_t m = __ballot(alive);
        if (m) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(nsurv, (uint32_t)__popcll(m));
            base = __builtin_amdgcn_readlane(base, 0);
            if (alive)
                list[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                    j | (q << 13);
        }
    }
    lds_barrier();
    // 2. the survivors, 64 per wave at a time
    const uint32_t S = *nsurv, share = (S + NWAVES * 64 - 1) / (NWAVES * 64) * 64;
    const uint32_t j0 = wave * share, j1 = j0 + share < S ? j0 + share : S;
    uint32_t i = j0 + lane, next = j0 + 64, job = 0, p = 0, stop = 0, steps = 1;
    bool active = i < j1;
    if (active) {
        const uint32_t e = list[i];
        job = e & 0x1fffu;
        p = e >> 13;
        stop = stop_of(job);
    }
    while (__ballot(active)) {
        const uint32_t v = be32_lds(lds, p & (FI_SEG - 1)); // in the staged bytes
        const uint32_t q = p + 4 + (v < 0x7fffffffu ? v : 0x7fffffffu);
        const bool exit = (p >= segend) | ((p >= stop) & ((p & 0xe00u) == 0));
        const bool fin = active & (exit | (q >= far) | (steps >= FI_STEPCAP));
        if (fin)
            out[job] = exit ? (steps << 17) | p
                            : (uint64_t)p + 4 + v > lenrel ? FI_T_TERM | (steps << 17) | p : FI_T_OVF;
        const uint64_t fm = __ballot(fin);
        const uint32_t in = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
        next += (uint32_t)__popcll(fm);
        const uint32_t e = list[in < j1 ? in : j0]; // (a real entry either way)
        active = fin ? in < j1 : active;
        job = fin ? e & 0x1fffu : job;
        p = fin ? e >> 13 : q;
        stop = fin ? stop_of(e & 0x1fffu) : stop;
        steps = fin ? 1 : steps + 1;
    }
    lds_barrier();
    if (threadIdx.x == 0) *nsurv = 0;
}

// a segment entry's result from its sub-segment 0 walk c: exit offset into the next segment
// (< W), FI_TERM | position, or FI_OVF; frames in *steps.  piece(j, p, before) for every later
// sub-segment piece of the chain (entry position, frames before it).
template <class Piece>
__device__ __forceinline__ uint32_t fi_compose(const uint32_t *T, uint32_t c, uint32_t segend, uint32_t *steps_out,
                                               Piece piece) {
    uint32_t steps = 0;
    while (true) {
        if (c == FI_T_OVF) return FI_OVF;
        steps += (c >> 17) & 0x3fffu;
        if (steps > FI_STEPCAP) return FI_OVF;
        const uint32_t p = c & FI_T_POS;
        *steps_out = steps;
        if (c & FI_T_TERM) return FI_TERM | p;
        if (p >= segend) return p - segend < FI_W ? p - segend : FI_OVF;
        piece(p / FI_SUB, p, steps);
        c = T[(p / FI_SUB - 1) * FI_WS + (p & (FI_SUB - 1))];
    }
}

// Persistent: a block strides over the segments; the next segment's bytes are loaded into
// registers while this one is walked, so HBM latency hides behind the walks.
__global__ __launch_bounds__(FI_BLOCK) void fi_seg_kernel(FiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t nlive, nsurv;
    const uint32_t stride = gridDim.x;
    if (threadIdx.x == 0) nsurv = 0; // (fi_tables leaves it 0; the first barrier is the staging's)
    const uint4 *src = (const uint4 *)a.buf; // quad_segment: 16-byte aligned
    uint4 v0 = {}, v1 = {}, halo = {};
    uint32_t k = blockIdx.x;
    if (k < a.nseg && quad_segment(a, (uint64_t)k * FI_SEG)) {
        const uint64_t q0 = (uint64_t)k * (FI_SEG / 16);
        v0 = src[q0 + threadIdx.x];
        v1 = src[q0 + threadIdx.x + FI_BLOCK];
        if (threadIdx.x == 0) halo = src[q0 + FI_SEG / 16];
    }
    for (; k < a.nseg; k += stride) {
        const uint64_t s0 = (uint64_t)k * FI_SEG, s1 = s0 + FI_SEG < a.len ? s0 + FI_SEG : a.len;
        const uint32_t segend = (uint32_t)(s1 - s0);
        if (threadIdx.x == 0) nlive = 0;
        if (quad_segment(a, s0)) {
            uint4 *dst = (uint4 *)lds;
            dst[threadIdx.x] = v0;
            dst[threadIdx.x + FI_BLOCK] = v1;
            if (threadIdx.x == 0) dst[FI_SEG / 16] = halo;
            lds_barrier();
        } else {
            stage_segment(a, s0, lds);
        }
        if (k + stride < a.nseg && quad_segment(a, (uint64_t)(k + stride) * FI_SEG)) { // the next, in flight
            const uint64_t q0 = (uint64_t)(k + stride) * (FI_SEG / 16);
            v0 = src[q0 + threadIdx.x];
            v1 = src[q0 + threadIdx.x + FI_BLOCK];
            if (threadIdx.x == 0) halo = src[q0 + FI_SEG / 16];
        }
        fi_tables(a, s0, segend, lds, true, &nsurv);
        const uint32_t *T = (const uint32_t *)(lds + FI_LDS_T), *C = (const uint32_t *)(lds + FI_LDS);
        uint32_t *live = a.live + (uint64_t)k * FI_LIVE * FI_LREC;
        for (uint32_t e = threadIdx.x; e < FI_W; e += FI_BLOCK) { // a lane composes its own walks
            // an entry that survives sub-segment 0 may be live: a record slot for its pieces
            // (marked dead again if the chain ends in the segment after all)
            const uint32_t c0 = C[e];
            uint32_t *rec = nullptr;
            if (c0 != FI_T_OVF && !(c0 & FI_T_TERM)) {
                const uint32_t slot = atomicAdd(&nlive, 1u);
                if (slot < FI_LIVE) {
                    rec = live + slot * FI_LREC;
                    rec[1] = e << 16;
                    for (uint32_t j = 1; j < FI_NSUB; j++) rec[1 + j] = ~0u;
                }
            }
            uint32_t steps = 0;
            const uint32_t code = fi_compose(T, c0, segend, &steps, [&](uint32_t j, uint32_t p, uint32_t before) {
                if (rec) rec[1 + j] = (p << 16) | before;
            });
            if (rec) rec[0] = code < FI_W ? e : ~0u;
            a.exitT[(uint64_t)k * FI_W + e] = code == FI_OVF ? FI_OVF : code | (steps << FI_CNT_SHIFT);
        }
        lds_barrier(); // nlive final; the LDS free for the next segment
        if (threadIdx.x == 0) a.live_n[k] = nlive;
    }
}

// groups of G1 segments: every entry's exit composed over the group's tables (G1 dependent reads)
__global__ __launch_bounds__(FI_BLOCK) void fi_group1_kernel(FiArgs a) {
    const uint32_t g = blockIdx.x, k0 = g * FI_G1, k1 = k0 + FI_G1 < a.nseg ? k0 + FI_G1 : a.nseg;
    for (uint32_t e = threadIdx.x; e < FI_W; e += FI_BLOCK) {
        uint32_t x = e, cnt = 0;
        uint64_t code = 0;
        bool open = true;
        for (uint32_t k = k0; k < k1 && open; k++) {
            const uint32_t c = a.exitT[(uint64_t)k * FI_W + x];
            if (c == FI_OVF) {
                code = FI_G_OVF;
                open = false;
                break;
            }
            cnt += (c >> FI_CNT_SHIFT) & FI_CNT_MASK;
            if (c & FI_TERM) {
                code = FI_G_TERM | ((uint64_t)k * FI_SEG + (c & FI_POS_MASK));
                open = false;
            } else {
                x = c & 0xffffu;
            }
        }
        if (open) code = x; // entry into segment k1
        a.g1T[(uint64_t)g * FI_W + e] = code;
        a.g1Cnt[(uint64_t)g * FI_W + e] = cnt;
    }
}

// super-groups of G2 groups: the same over the group tables
__global__ __launch_bounds__(FI_BLOCK) void fi_group2_kernel(FiArgs a) {
    const uint32_t g = blockIdx.x, j0 = g * FI_G2, j1 = j0 + FI_G2 < a.ng1 ? j0 + FI_G2 : a.ng1;
    for (uint32_t e = threadIdx.x; e < FI_W; e += FI_BLOCK) {
        uint64_t code = e;
        uint32_t cnt = 0;
        for (uint32_t j = j0; j < j1; j++) {
            const uint64_t c = a.g1T[(uint64_t)j * FI_W + code];
            cnt += a.g1Cnt[(uint64_t)j * FI_W + code];
            code = c;
            if (c & (FI_G_TERM | FI_G_OVF)) break;
        }
        a.g2T[(uint64_t)g * FI_W + e] = code;
        a.g2Cnt[(uint64_t)g * FI_W + e] = cnt;
    }
}

// one thread: the super-groups chained from offset 0
__global__ void fi_chain_kernel(FiArgs a) {
    if (threadIdx.x != 0) return;
    uint64_t x = 0, base = 0, consumed = a.len, ovf = 0;
    uint32_t g = 0;
    for (; g < a.ng2; g++) {
        a.g2_entry[g] = (uint32_t)x;
        a.g2_base[g] = base;
        const uint64_t c = a.g2T[(uint64_t)g * FI_W + x];
        base += a.g2Cnt[(uint64_t)g * FI_W + x];
        if (c & FI_G_OVF) {
            ovf = 1;
            break;
        }
        if (c & FI_G_TERM) {
            consumed = c & ~FI_G_TERM;
            g++;
            break;
        }
        x = c;
    }
    for (; g < a.ng2; g++) a.g2_entry[g] = FI_NONE;
    a.work[0] = 0;
    a.misc[0] = ovf;
    a.misc[1] = base;
    a.misc[2] = consumed;
}

// per super-group (one thread): its groups' entries and frame bases
__global__ void fi_resolve2_kernel(FiArgs a) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.ng2 || a.misc[0]) return;
    const uint32_t j0 = g * FI_G2, j1 = j0 + FI_G2 < a.ng1 ? j0 + FI_G2 : a.ng1;
    uint32_t x = a.g2_entry[g];
    uint64_t base = a.g2_base[g];
    for (uint32_t j = j0; j < j1; j++) {
        a.g1_entry[j] = x;
        a.g1_base[j] = base;
        if (x == FI_NONE) continue;
        const uint64_t c = a.g1T[(uint64_t)j * FI_W + x];
        base += a.g1Cnt[(uint64_t)j * FI_W + x];
        x = (c & (FI_G_TERM | FI_G_OVF)) ? FI_NONE : (uint32_t)c;
    }
}

// per group (one thread): its segments' entries and frame bases
__global__ void fi_segentry_kernel(FiArgs a) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.ng1 || a.misc[0]) return;
    const uint32_t k0 = g * FI_G1, k1 = k0 + FI_G1 < a.nseg ? k0 + FI_G1 : a.nseg;
    uint32_t x = a.g1_entry[g];
    uint64_t base = a.g1_base[g];
    for (uint32_t k = k0; k < k1; k++) {
        a.seg_entry[k] = x;
        a.seg_base[k] = base;
        if (x == FI_NONE) continue;
        const uint32_t c = a.exitT[(uint64_t)k * FI_W + x];
        if (c == FI_OVF) { // the chain kernel has raised the overflow flag
            x = FI_NONE;
            continue;
        }
        base += (c >> FI_CNT_SHIFT) & FI_CNT_MASK;
        x = (c & FI_TERM) ? FI_NONE : c & 0xffffu;
    }
}

// the big-endian u32 at byte o of buf (zeros past len; buf is 4-byte aligned)
__device__ __forceinline__ uint32_t be32_global(const uint8_t *buf, uint64_t len, uint64_t o) {
    if (o + 8 <= len) {
        const uint32_t *w = (const uint32_t *)(buf + (o & ~3ull));
        const uint64_t d = ((uint64_t)w[1] << 32) | w[0];
        return __builtin_bswap32((uint32_t)(d >> (8 * (o & 3))));
    }
    uint32_t v = 0;
    for (uint32_t b = 0; b < 4; b++) v = (v << 8) | (o + b < len ? buf[o + b] : 0u);
    return v;
}

// One piece of a segment's true chain (from segment-relative p, frames before it in i): the
// frames up to the next window position past `stop` (or the segment end), ends[] written.
template <class Read>
__device__ __forceinline__ void fi_emit_piece(const FiArgs &a, uint64_t s0, uint32_t segend, uint32_t stop,
                                              uint32_t p, uint64_t i, Read be32) {
    const uint64_t lenrel = a.len - s0;
    while (!(p >= segend || (p >= stop && (p & (FI_SUB - 1)) < FI_WS)) && (uint64_t)p + 4 <= lenrel) {
        const uint64_t q = (uint64_t)p + 4 + be32(p);
        if (q > lenrel) break;
        if (i < a.cap) a.ends[i] = s0 + q;
        i++;
        p = (uint32_t)q;
    }
}

// per segment on the chain: its entry's pieces from the seg kernel's live records, one lane per
// sub-segment piece reading the heads from HBM and writing ends[]; a segment whose entry has no
// record (the chain ends in it, or more than FI_LIVE live entries) goes to the work list
__global__ __launch_bounds__(64) void fi_emit_kernel(FiArgs a) {
    const uint32_t k = blockIdx.x, lane = threadIdx.x;
    if (a.misc[0]) return;
    const uint32_t e = a.seg_entry[k];
    if (e == FI_NONE) return;
    const uint32_t n = a.live_n[k];
    const uint32_t *live = a.live + (uint64_t)k * FI_LIVE * FI_LREC;
    const uint64_t hit = __ballot(lane < n && lane < FI_LIVE && live[lane * FI_LREC] == e);
    if (hit == 0) {
        if (lane == 0) a.work[1 + atomicAdd(&a.work[0], 1u)] = k;
        return;
    }
    if (lane >= FI_NSUB) return;
    const uint32_t v = live[(__ffsll((unsigned long long)hit) - 1) * FI_LREC + 1 + lane];
    if (v == ~0u) return;
    const uint64_t s0 = (uint64_t)k * FI_SEG, s1 = s0 + FI_SEG < a.len ? s0 + FI_SEG : a.len;
    fi_emit_piece(a, s0, (uint32_t)(s1 - s0), (lane + 1) * FI_SUB, v >> 16, a.seg_base[k] + (v & 0xffffu),
                  [&](uint32_t p) { return be32_global(a.buf, a.len, s0 + p); });
}

// the work list's segments: tables again in LDS, the true entry composed once, one thread per
// piece (a grid of at most 256 blocks striding the list; usually one segment, the chain's last)
__global__ __launch_bounds__(FI_BLOCK) void fi_emit_slow_kernel(FiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t ent[FI_NSUB], before[FI_NSUB], nsurv;
    if (threadIdx.x == 0) nsurv = 0;
    const uint32_t nwork = a.work[0];
    for (uint32_t w = blockIdx.x; w < nwork; w += gridDim.x) {
        const uint32_t k = a.work[1 + w], e = a.seg_entry[k];
        const uint64_t s0 = (uint64_t)k * FI_SEG, s1 = s0 + FI_SEG < a.len ? s0 + FI_SEG : a.len;
        const uint32_t segend = (uint32_t)(s1 - s0);
        if (threadIdx.x < FI_NSUB) ent[threadIdx.x] = threadIdx.x ? ~0u : e, before[threadIdx.x] = 0;
        stage_segment(a, s0, lds);
        fi_tables(a, s0, segend, lds, true, &nsurv);
        if (threadIdx.x == 0) {
            uint32_t steps;
            const uint32_t *C = (const uint32_t *)(lds + FI_LDS);
            fi_compose((const uint32_t *)(lds + FI_LDS_T), C[e], segend, &steps, [&](uint32_t j, uint32_t p, uint32_t b) {
                ent[j] = p;
                before[j] = b;
            });
        }
        __syncthreads();
        if (threadIdx.x < FI_NSUB && ent[threadIdx.x] != ~0u)
            fi_emit_piece(a, s0, segend, (threadIdx.x + 1) * FI_SUB, ent[threadIdx.x],
                          a.seg_base[k] + before[threadIdx.x], [&](uint32_t p) { return be32_lds(lds, p); });
        __syncthreads();
    }
}

// overflow: the serial walk over HBM (exact, slow); then count / consumed / status
__global__ void fi_finish_kernel(FiArgs a) {
    if (threadIdx.x != 0) return;
    uint64_t total = a.misc[1], consumed = a.misc[2];
    if (a.misc[0]) {
        uint64_t p = 0, i = 0;
        while (p + 4 <= a.len) {
            const uint64_t q = p + 4 +
                               (((uint32_t)a.buf[p] << 24) | ((uint32_t)a.buf[p + 1] << 16) |
                                ((uint32_t)a.buf[p + 2] << 8) | a.buf[p + 3]);
            if (q > a.len) break;
            if (i < a.cap) a.ends[i] = q;
            i++;
            p = q;
        }
        total = i;
        consumed = p;
    }
    if (total > a.cap) { // as the host walk: the first cap frames, SPEC_E_CAPACITY
        *a.count = a.cap;
        *a.consumed = a.cap ? a.ends[a.cap - 1] : 0;
        *a.status = SPEC_E_CAPACITY;
    } else {
        *a.count = total;
        *a.consumed = consumed;
        *a.status = SPEC_OK;
    }
}

struct FiLayout {
    uint32_t nseg, ng1, ng2;
    size_t off[15], bytes;
};

FiLayout fi_layout(uint64_t len) {
    FiLayout L;
    L.nseg = (uint32_t)((len + FI_SEG - 1) / FI_SEG);
    if (L.nseg == 0) L.nseg = 1;
    L.ng1 = (L.nseg + FI_G1 - 1) / FI_G1;
    L.ng2 = (L.ng1 + FI_G2 - 1) / FI_G2;
    const size_t W = FI_W;
    const size_t sz[15] = {L.nseg * W * 4,  L.ng1 * W * 8, L.ng1 * W * 4, L.ng2 * W * 8,
                           L.ng2 * W * 4,   (size_t)L.ng1 * 4, (size_t)L.ng1 * 8, (size_t)L.ng2 * 4,
                           (size_t)L.ng2 * 8, (size_t)L.nseg * 4, (size_t)L.nseg * 8, 64,
                           (size_t)L.nseg * 4, (size_t)L.nseg * FI_LIVE * FI_LREC * 4, ((size_t)L.nseg + 1) * 4};
    size_t o = 0;
    for (int i = 0; i < 15; i++) {
        L.off[i] = o;
        o += (sz[i] + 255) / 256 * 256;
    }
    L.bytes = o;
    return L;
}

} // namespace

size_t frames_index_device_workspace(uint64_t len) { return fi_layout(len).bytes; }

int launch_frames_index_device(const uint8_t *buf, uint64_t len, uint64_t *ends, uint64_t cap, uint64_t *count,
                               uint64_t *consumed, int32_t *status, void *ws, hipStream_t stream) {
    const FiLayout L = fi_layout(len);
    uint8_t *w = (uint8_t *)ws;
    FiArgs a;
    a.buf = buf;
    a.len = len;
    a.cap = cap;
    a.ends = ends;
    a.count = count;
    a.consumed = consumed;
    a.status = status;
    a.nseg = L.nseg;
    a.ng1 = L.ng1;
    a.ng2 = L.ng2;
    a.exitT = (uint32_t *)(w + L.off[0]);
    a.g1T = (uint64_t *)(w + L.off[1]);
    a.g1Cnt = (uint32_t *)(w + L.off[2]);
    a.g2T = (uint64_t *)(w + L.off[3]);
    a.g2Cnt = (uint32_t *)(w + L.off[4]);
    a.g1_entry = (uint32_t *)(w + L.off[5]);
    a.g1_base = (uint64_t *)(w + L.off[6]);
    a.g2_entry = (uint32_t *)(w + L.off[7]);
    a.g2_base = (uint64_t *)(w + L.off[8]);
    a.seg_entry = (uint32_t *)(w + L.off[9]);
    a.seg_base = (uint64_t *)(w + L.off[10]);
    a.misc = (uint64_t *)(w + L.off[11]);
    a.live_n = (uint32_t *)(w + L.off[12]);
    a.live = (uint32_t *)(w + L.off[13]);
    a.work = (uint32_t *)(w + L.off[14]);
    const size_t lds = FI_LDS_END;
    const uint32_t seg_blocks = 2u * (uint32_t)device_cus(); // two 70 KiB-LDS blocks per CU, persistent
    hipLaunchKernelGGL(fi_seg_kernel, dim3(L.nseg < seg_blocks ? L.nseg : seg_blocks), dim3(FI_BLOCK), lds, stream, a);
    hipLaunchKernelGGL(fi_group1_kernel, dim3(L.ng1), dim3(FI_BLOCK), 0, stream, a);
    hipLaunchKernelGGL(fi_group2_kernel, dim3(L.ng2), dim3(FI_BLOCK), 0, stream, a);
    hipLaunchKernelGGL(fi_chain_kernel, dim3(1), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(fi_resolve2_kernel, dim3((L.ng2 + 63) / 64), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(fi_segentry_kernel, dim3((L.ng1 + 63) / 64), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(fi_emit_kernel, dim3(L.nseg), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(fi_emit_slow_kernel, dim3(L.nseg < 256 ? L.nseg : 256), dim3(FI_BLOCK), lds, stream, a);
    hipLaunchKernelGGL(fi_finish_kernel, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
