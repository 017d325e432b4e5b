// frames_device.hip — spec_frames_index_device: the mpx frame index (mpx/conn_reader.go:179-194:
// `[u32 BE size][message]` frames back to back) computed on the GPU, with exactly the results of
// the host walk spec_frames_index (capi.hip).
//
// The head chain is serial (frame k+1 starts where frame k ends), so the walk is split:
//   1. segments of 64 KiB, staged in LDS; for EVERY entry offset e < W (2048) of a segment, the
//      chain is walked to the segment end: exit offset into the next segment, frames completed
//      (a false entry reads a random big size and leaves at once; the true one walks ~S/frame
//      steps in LDS);
//   2. groups of 64 segments compose their tables (every entry, 64 dependent table reads);
//   3. one thread chains the groups from offset 0 (a few hundred dependent reads);
//   4. each group resolves its segments' entries and frame bases;
//   5. each segment walks its true chain again in LDS and writes ends[];
// A frame that straddles a segment boundary by W bytes or more, or a segment with more than
// 4096 frames, sets the overflow flag: a single-thread serial walk over HBM then produces the
// same results (slow but exact).  One call, no host sync; count / consumed / status land in
// device memory.
#include <hip/hip_runtime.h>

#include "spec_internal.hpp"

namespace spec {

namespace {

constexpr uint32_t FI_SEG = 65536, FI_W = 2048, FI_G = 64, FI_STEPCAP = 4096;
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

__device__ __forceinline__ uint32_t be32_lds(const uint8_t *l, uint32_t o) {
    return ((uint32_t)l[o] << 24) | ((uint32_t)l[o + 1] << 16) | ((uint32_t)l[o + 2] << 8) | l[o + 3];
}

// bytes [s0, s0 + SEG + 16) of buf into lds (zeros past len); buf is 4-byte aligned
__device__ __forceinline__ void stage_segment(const FiArgs &a, uint64_t s0, uint8_t *lds) {
    constexpr uint32_t NQ = (FI_SEG + 16) / 16;
    // a whole segment from a 16-byte aligned buffer: 16-byte loads, four in flight per thread
    // (the ABI only promises 4-byte alignment: other buffers take the dword loop)
    if (s0 + FI_SEG + 16 <= a.len && ((uintptr_t)a.buf & 15) == 0) {
        for (uint32_t i0 = 0; i0 < NQ; i0 += 4 * blockDim.x) {
            uint4 v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
                if (i < NQ) v[j] = *(const uint4 *)(a.buf + s0 + 16ull * i);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t i = i0 + threadIdx.x + j * blockDim.x;
                if (i < NQ) *(uint4 *)(lds + 16 * i) = v[j];
            }
        }
        __syncthreads();
        return;
    }
    uint32_t *l32 = (uint32_t *)lds;
    for (uint32_t i = threadIdx.x; i < (FI_SEG + 16) / 4; i += blockDim.x) {
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

__global__ __launch_bounds__(1024) void fi_seg_kernel(FiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t k = blockIdx.x;
    const uint64_t s0 = (uint64_t)k * FI_SEG, s1 = s0 + FI_SEG < a.len ? s0 + FI_SEG : a.len;
    stage_segment(a, s0, lds);
    for (uint32_t e = threadIdx.x; e < FI_W; e += blockDim.x) {
        uint64_t p = s0 + e;
        uint32_t steps = 0, code;
        while (true) {
            if (p >= s1) {
                const uint64_t x = p - s1;
                code = x < FI_W ? (uint32_t)x : FI_OVF;
                break;
            }
            if (p + 4 > a.len) {
                code = FI_TERM | (uint32_t)(p - s0);
                break;
            }
            const uint64_t q = p + 4 + be32_lds(lds, (uint32_t)(p - s0));
            if (q > a.len) {
                code = FI_TERM | (uint32_t)(p - s0);
                break;
            }
            p = q;
            if (++steps > FI_STEPCAP) {
                code = FI_OVF;
                break;
            }
        }
        a.exitT[(uint64_t)k * FI_W + e] = code;
        a.cntT[(uint64_t)k * FI_W + e] = steps;
    }
}

__global__ __launch_bounds__(1024) void fi_group_kernel(FiArgs a) {
    const uint32_t g = blockIdx.x, k0 = g * FI_G, k1 = k0 + FI_G < a.nseg ? k0 + FI_G : a.nseg;
    for (uint32_t e = threadIdx.x; e < FI_W; e += blockDim.x) {
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

// per segment: its true chain walked again in LDS, ends[] written
__global__ __launch_bounds__(256) void fi_emit_kernel(FiArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t k = blockIdx.x;
    if (a.misc[0]) return;
    const uint32_t e = a.seg_entry[k];
    if (e == FI_NONE) return;
    const uint64_t s0 = (uint64_t)k * FI_SEG, s1 = s0 + FI_SEG < a.len ? s0 + FI_SEG : a.len;
    stage_segment(a, s0, lds);
    if (threadIdx.x != 0) return;
    uint64_t p = s0 + e, i = a.seg_base[k];
    while (p < s1 && p + 4 <= a.len) {
        const uint64_t q = p + 4 + be32_lds(lds, (uint32_t)(p - s0));
        if (q > a.len) break;
        if (i < a.cap) a.ends[i] = q;
        i++;
        p = q;
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
    const size_t lds = FI_SEG + 16;
    hipLaunchKernelGGL(fi_seg_kernel, dim3(L.nseg), dim3(1024), lds, stream, a);
    hipLaunchKernelGGL(fi_group_kernel, dim3(L.ngroups), dim3(1024), 0, stream, a);
    hipLaunchKernelGGL(fi_chain_kernel, dim3(1), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(fi_segentry_kernel, dim3((L.ngroups + 63) / 64), dim3(64), 0, stream, a);
    hipLaunchKernelGGL(fi_emit_kernel, dim3(L.nseg), dim3(256), lds, stream, a);
    hipLaunchKernelGGL(fi_finish_kernel, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
