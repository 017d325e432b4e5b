// frames_device.hip — spec_frames_index_device: the mpx frame index (mpx/conn_reader.go:179-194:
// `[u32 BE size][message]` frames back to back) computed on the GPU, with exactly the results of
// the host walk spec_frames_index (capi.hip).
//
// The head chain is serial (frame k+1 starts where frame k ends), so the walk is split:
//   1. segments of 64 KiB, staged in LDS; for EVERY entry offset e < W (2048) of a segment, the
//      chain is walked to the segment end: exit offset into the next segment, frames completed.
//      Inside the segment the walk is itself split into 16 sub-segments of 4 KiB: every entry
//      o < WS (1024) of sub-segments 1..15 is walked to the first position past its sub-segment
//      that lies in some later sub-segment's window (or past the segment end), the results kept
//      in LDS; a segment entry then walks sub-segment 0 and composes the tables (at most 15
//      dependent LDS reads), so no thread walks more than ~4 KiB of frames (a false entry reads a
//      random big size and leaves at once);
//   2. groups of 64 segments compose their tables (every entry, 64 dependent table reads);
//   3. one thread chains the groups from offset 0 (a few hundred dependent reads);
//   4. each group resolves its segments' entries and frame bases;
//   5. each segment on the chain rebuilds its sub-segment tables, composes its true entry once,
//      and 16 threads walk the 16 sub-segment pieces of the true chain writing ends[];
#include <hip/hip_runtime.h>

#include "spec_internal.hpp"

namespace spec {

namespace {

constexpr uint32_t FI_SEG = 65536, FI_W = 2048, FI_G = 64, FI_STEPCAP = 4096;
constexpr uint32_t FI_BLOCK = 1024; // threads of the segment / group kernels (a constant: blockDim
                                    // is a load from the dispatch packet)
constexpr uint32_t FI_SUB = 4096, FI_NSUB = FI_SEG / FI_SUB, FI_WS = 1024;
constexpr uint32_t FI_LDS_T = FI_SEG + 16, FI_LDS = FI_LDS_T + (FI_NSUB - 1) * FI_WS * 4;
// a sub-segment walk result: [31] TERM, [30:17] frames, [16:0] segment-relative position
constexpr uint32_t FI_T_TERM = 1u << 31, FI_T_OVF = 0xffffffffu, FI_T_POS = 0x1ffffu;
constexpr uint32_t FI_OVF = 0xffffffffu, FI_TERM = 0x80000000u, FI_NONE = 0xffffffffu;
constexpr uint64_t FI_G_TERM = 1ull << 63, FI_G_OVF = 1ull << 62;

struct FiArgs {
    const uint8_t *buf;
    uint64_t len, cap;
    uint64_t *ends, *count, *consumed;
    int32_t *status;
    uint32_t nseg, ngroups;
    uint32_t *exitT, *cntT;    // [nseg * W]
    uint64_t *grpT;            // [ngroups * W]
    uint32_t *grpCnt;          // [ngroups * W]
    uint32_t *grp_entry;       // [ngroups]
    uint64_t *grp_base;        // [ngroups]
    uint32_t *seg_entry;       // [nseg]
    uint64_t *seg_base;        // [nseg]
    uint64_t *misc;            // [0] overflow, [1] total frames, [2] consumed
};

// the big-endian u32 at byte o of the staged segment: two dword reads and a funnel shift
__device__ __forceinline__ uint32_t be32_lds(const uint8_t *l, uint32_t o) {
    const uint32_t *w = (const uint32_t *)l;
    const uint64_t d = ((uint64_t)w[(o >> 2) + 1] << 32) | w[o >> 2];
    return __builtin_bswap32((uint32_t)(d >> (8 * (o & 3))));
}

// bytes [s0, s0 + SEG + 16) of buf into lds (zeros past len); buf is 4-byte aligned
__device__ __forceinline__ void stage_segment(const FiArgs &a, uint64_t s0, uint8_t *lds) {
    // a whole segment from a 16-byte aligned buffer: 16-byte loads, all of a thread's in flight
    // (the ABI only promises 4-byte alignment: other buffers take the dword loop)
    if (s0 + FI_SEG + 16 <= a.len && ((uintptr_t)a.buf & 15) == 0) {
        const uint4 *src = (const uint4 *)(a.buf + s0);
        uint4 *dst = (uint4 *)lds;
        for (uint32_t i0 = 0; i0 < FI_SEG / 16; i0 += 4 * FI_BLOCK) {
            const uint32_t i = i0 + threadIdx.x; // FI_SEG / 16 is a multiple of 4 * FI_BLOCK
            const uint4 v0 = src[i], v1 = src[i + FI_BLOCK], v2 = src[i + 2 * FI_BLOCK],
                        v3 = src[i + 3 * FI_BLOCK];
            dst[i] = v0;
            dst[i + FI_BLOCK] = v1;
            dst[i + 2 * FI_BLOCK] = v2;
            dst[i + 3 * FI_BLOCK] = v3;
        }
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

// Walk jobs i = threadIdx.x + m * FI_BLOCK < njobs: from start(i) -> (p, stop), the chain
// until it stands on a position at or past `stop` that lies in the first WS bytes of a
// sub-segment, or past the segment end (segend = s1 - s0, lenrel = len - s0); out[i] = code.  A
// jump W or more past the segment end, or more than STEPCAP frames, is overflow (the serial
// fallback).  One frame step per iteration, selects instead of branches, one predicated store:
// a lane that finishes a walk starts its next at once, so a wave runs for its busiest lane's
// steps, not for the sum over jobs of the longest walk.
template <class Start>
__device__ __forceinline__ void fi_walk_all(const uint8_t *lds, uint32_t njobs, uint32_t segend, uint64_t lenrel,
                                            Start start, uint32_t *out) {
    uint32_t i = threadIdx.x, p, stop, steps = 0;
    if (i >= njobs) return;
    start(i, p, stop);
    const uint64_t far = (uint64_t)segend + FI_W;
    while (true) {
        const bool exit = p >= segend || (p >= stop && (p & (FI_SUB - 1)) < FI_WS);
        const uint64_t q = (uint64_t)p + 4 + be32_lds(lds, p & 0xffffu); // in the staged bytes
        const bool term = q > lenrel;
        const bool fin = exit || term || q >= far || steps >= FI_STEPCAP;
        const uint32_t code = exit ? (steps << 17) | p : term ? FI_T_TERM | (steps << 17) | p : FI_T_OVF;
        if (fin) out[i] = code;
        const uint32_t inext = fin ? i + FI_BLOCK : i;
        if (inext >= njobs) break;
        uint32_t p2, stop2;
        start(inext, p2, stop2);
        p = fin ? p2 : (uint32_t)q;
        stop = fin ? stop2 : stop;
        steps = fin ? 0 : steps + 1;
        i = inext;
    }
}

// stage the segment and walk every window entry of sub-segments 1..15 (tables after the data)
__device__ __forceinline__ void fi_tables(const FiArgs &a, uint64_t s0, uint32_t segend, uint8_t *lds) {
    stage_segment(a, s0, lds);
    uint32_t *T = (uint32_t *)(lds + FI_LDS_T);
    fi_walk_all(
        lds, (FI_NSUB - 1) * FI_WS, segend, a.len - s0,
        [](uint32_t i, uint32_t &p, uint32_t &stop) {
            stop = (2 + i / FI_WS) * FI_SUB;
            p = stop - FI_SUB + i % FI_WS;
        },
        T);
    __syncthreads();
}

// a segment entry's result from its sub-segment 0 walk c: exit offset into the next segment
// (< W), FI_TERM | position, or FI_OVF; frames in *steps.  With `ent`, the sub-segment pieces'
// entries and frame counts before them (ent[j] = ~0u for sub-segments the chain jumps over).
__device__ __forceinline__ uint32_t fi_compose(const uint32_t *T, uint32_t c, uint32_t segend, uint32_t *steps_out,
                                               uint32_t *ent = nullptr, uint32_t *before = nullptr) {
    uint32_t steps = 0;
    while (true) {
        if (c == FI_T_OVF) return FI_OVF;
        steps += (c >> 17) & 0x3fffu;
        if (steps > FI_STEPCAP) return FI_OVF;
        const uint32_t p = c & FI_T_POS;
        *steps_out = steps;
        if (c & FI_T_TERM) return FI_TERM | p;
        if (p >= segend) return p - segend < FI_W ? p - segend : FI_OVF;
        if (ent) {
            ent[p / FI_SUB] = p;
            before[p / FI_SUB] = steps;
        }
        c = T[(p / FI_SUB - 1) * FI_WS + (p & (FI_SUB - 1))];
    }
}

__global__ __launch_bounds__(FI_BLOCK) void fi_seg_kernel(FiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t k = blockIdx.x;
    const uint64_t s0 = (uint64_t)k * FI_SEG, s1 = s0 + FI_SEG < a.len ? s0 + FI_SEG : a.len;
    const uint32_t segend = (uint32_t)(s1 - s0);
    fi_tables(a, s0, segend, lds);
    const uint32_t *T = (const uint32_t *)(lds + FI_LDS_T);
    uint32_t *C = (uint32_t *)(lds + FI_LDS);
    fi_walk_all(
        lds, FI_W, segend, a.len - s0,
        [](uint32_t e, uint32_t &p, uint32_t &stop) {
            p = e;
            stop = FI_SUB;
        },
        C);
    for (uint32_t e = threadIdx.x; e < FI_W; e += FI_BLOCK) { // a lane composes its own walks
        uint32_t steps = 0;
        const uint32_t code = fi_compose(T, C[e], segend, &steps);
        a.exitT[(uint64_t)k * FI_W + e] = code;
        a.cntT[(uint64_t)k * FI_W + e] = steps;
    }
}

__global__ __launch_bounds__(FI_BLOCK) void fi_group_kernel(FiArgs a) {
    const uint32_t g = blockIdx.x, k0 = g * FI_G, k1 = k0 + FI_G < a.nseg ? k0 + FI_G : a.nseg;
    for (uint32_t e = threadIdx.x; e < FI_W; e += FI_BLOCK) {
        uint32_t x = e, cnt = 0;
        uint64_t code = 0;
        bool open = true;
        for (uint32_t k = k0; k < k1 && open; k++) {
            const uint32_t c = a.exitT[(uint64_t)k * FI_W + x];
            cnt += a.cntT[(uint64_t)k * FI_W + x];
            if (c < FI_W) {
                x = c;
            } else if (c == FI_OVF) {
                code = FI_G_OVF;
                open = false;
            } else {
                code = FI_G_TERM | ((uint64_t)k * FI_SEG + (c & 0xffffu));
                open = false;
            }
        }
        if (open) code = x; // entry into segment k1
        a.grpT[(uint64_t)g * FI_W + e] = code;
        a.grpCnt[(uint64_t)g * FI_W + e] = cnt;
    }
}

// one thread: the groups chained from offset 0
__global__ void fi_chain_kernel(FiArgs a) {
    if (threadIdx.x != 0) return;
    uint64_t x = 0, base = 0, consumed = a.len, ovf = 0;
    uint32_t g = 0;
    for (; g < a.ngroups; g++) {
        a.grp_entry[g] = (uint32_t)x;
        a.grp_base[g] = base;
        const uint64_t c = a.grpT[(uint64_t)g * FI_W + x];
        base += a.grpCnt[(uint64_t)g * FI_W + x];
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
    for (; g < a.ngroups; g++) a.grp_entry[g] = FI_NONE;
    a.misc[0] = ovf;
    a.misc[1] = base;
    a.misc[2] = consumed;
}

// per group (one thread): its segments' entries and frame bases
__global__ void fi_segentry_kernel(FiArgs a) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.ngroups || a.misc[0]) return;
    const uint32_t k0 = g * FI_G, k1 = k0 + FI_G < a.nseg ? k0 + FI_G : a.nseg;
    uint32_t x = a.grp_entry[g];
    uint64_t base = a.grp_base[g];
    for (uint32_t k = k0; k < k1; k++) {
        a.seg_entry[k] = x;
        a.seg_base[k] = base;
        if (x == FI_NONE) continue;
        const uint32_t c = a.exitT[(uint64_t)k * FI_W + x];
        base += a.cntT[(uint64_t)k * FI_W + x];
        x = c < FI_W ? c : FI_NONE;
    }
}

// per segment on the chain: tables again, the true entry composed once, then one thread per
// sub-segment piece of the true chain writes its ends[]
__global__ __launch_bounds__(FI_BLOCK) void fi_emit_kernel(FiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t ent[FI_NSUB], before[FI_NSUB];
    const uint32_t k = blockIdx.x;
    if (a.misc[0]) return;
    const uint32_t e = a.seg_entry[k];
    if (e == FI_NONE) return;
    const uint64_t s0 = (uint64_t)k * FI_SEG, s1 = s0 + FI_SEG < a.len ? s0 + FI_SEG : a.len;
    const uint32_t segend = (uint32_t)(s1 - s0);
    const uint64_t lenrel = a.len - s0;
    if (threadIdx.x < FI_NSUB) ent[threadIdx.x] = threadIdx.x ? ~0u : e, before[threadIdx.x] = 0;
    fi_tables(a, s0, segend, lds);
    if (threadIdx.x == 0) {
        uint32_t steps;
        uint32_t *C = (uint32_t *)(lds + FI_LDS);
        fi_walk_all(
            lds, 1, segend, lenrel,
            [&](uint32_t, uint32_t &p, uint32_t &stop) {
                p = e;
                stop = FI_SUB;
            },
            C);
        fi_compose((const uint32_t *)(lds + FI_LDS_T), C[0], segend, &steps, ent, before);
    }
    __syncthreads();
    if (threadIdx.x >= FI_NSUB || ent[threadIdx.x] == ~0u) return;
    const uint32_t stop = (threadIdx.x + 1) * FI_SUB;
    uint32_t p = ent[threadIdx.x];
    uint64_t i = a.seg_base[k] + before[threadIdx.x];
    while (!(p >= segend || (p >= stop && (p & (FI_SUB - 1)) < FI_WS)) && (uint64_t)p + 4 <= lenrel) {
        const uint64_t q = (uint64_t)p + 4 + be32_lds(lds, p);
        if (q > lenrel) break;
        if (i < a.cap) a.ends[i] = s0 + q;
        i++;
        p = (uint32_t)q;
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
    uint32_t nseg, ngroups;
    size_t off[9], bytes;
};

FiLayout fi_layout(uint64_t len) {
    FiLayout L;
    L.nseg = (uint32_t)((len + FI_SEG - 1) / FI_SEG);
    if (L.nseg == 0) L.nseg = 1;
    L.ngroups = (L.nseg + FI_G - 1) / FI_G;
    const size_t sz[9] = {(size_t)L.nseg * FI_W * 4, (size_t)L.nseg * FI_W * 4, (size_t)L.ngroups * FI_W * 8,
                          (size_t)L.ngroups * FI_W * 4, (size_t)L.ngroups * 4, (size_t)L.ngroups * 8,
                          (size_t)L.nseg * 4, (size_t)L.nseg * 8, 64};
    size_t o = 0;
    for (int i = 0; i < 9; i++) {
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
    a.ngroups = L.ngroups;
    a.exitT = (uint32_t *)(w + L.off[0]);
    a.cntT = (uint32_t *)(w + L.off[1]);
    a.grpT = (uint64_t *)(w + L.off[2]);
    a.grpCnt = (uint32_t *)(w + L.off[3]);
    a.grp_entry = (uint32_t *)(w + L.off[4]);
    a.grp_base = (uint64_t *)(w + L.off[5]);
    a.seg_entry = (uint32_t *)(w + L.off[6]);
    a.seg_base = (uint64_t *)(w + L.off[7]);
    a.misc = (uint64_t *)(w + L.off[8]);
    const size_t lds = FI_LDS + FI_W * 4; // + the segment walks' sub-segment 0 codes
    hipLaunchKernelGGL(fi_seg_kernel, dim3(L.nseg), dim3(FI_BLOCK), lds, stream, a);
    hipLaunchKernelGGL(fi_group_kernel, dim3(L.ngroups), dim3(FI_BLOCK), 0, stream, a);
    hipLaunchKernelGGL(fi_chain_kernel, dim3(1), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(fi_segentry_kernel, dim3((L.ngroups + 63) / 64), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(fi_emit_kernel, dim3(L.nseg), dim3(FI_BLOCK), lds, stream, a);
    hipLaunchKernelGGL(fi_finish_kernel, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
