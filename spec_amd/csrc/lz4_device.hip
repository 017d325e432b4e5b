// lz4_device.hip — LZ4 blocks of an mpx connection stream decompressed on the GPU
// (spec_lz4_decompress / spec_lz4_pack, include/spec_amd.h).
//
// mpx wraps the connection in one LZ4 frame of independent 256 KiB blocks (mpx/conn_writer.go:
// 42-56, pierrec/lz4/v4).  The host walks the frame's block headers (spec_lz4_frame_blocks:
// one u32 per block) and hands the block table over; here ONE WAVE DECODES ONE BLOCK:
//   * the sequence chain (token, literal length, offset, match length) is serial, so it is
//     parsed by the scalar unit: the compressed bytes sit in a 768-byte register window (3
//     VGPRs x 64 lanes, refilled 256 bytes at a time) read with v_readlane at uniform indices;
//   * literal and match bytes are moved by all 64 lanes (64 bytes per instruction): literals
//     by ds_bpermute out of the window, matches out of a 64 KiB LDS ring holding the block's
//     last 64 KiB of output (every LZ4 offset is < 64 KiB) — a match whose source would be
//     overwritten in the ring during the copy (offset + length > 64 KiB) reads the output back
//     from HBM instead, with L1-bypassing loads after its own stores have drained;
//   * output bytes go to the block's slot in HBM.
// Errors are those of pierrec's decodeBlock (oracle/lz4.c so_lz4_decompress_block): the block's
// status is 1 and its size all-ones.  spec_lz4_pack then gathers the slots into one contiguous
// stream (exclusive scan of the sizes + a copy).
#include <hip/hip_runtime.h>

#include "spec_internal.hpp"

namespace spec {

namespace {

constexpr uint32_t RING = 65536, RMASK = RING - 1;

struct Lz4Args {
    const uint8_t *src;
    uint64_t src_len;
    const spec_lz4_block *blocks;
    uint64_t nblocks;
    uint8_t *slots;
    uint64_t slot;
    uint32_t *sizes;
    uint8_t *status;
};

// 4 source bytes at absolute offset o (zeros past the end; the last partial dword bytewise)
__device__ __forceinline__ uint32_t src_dword(const Lz4Args &a, __amdgpu_buffer_rsrc_t r, uint64_t o) {
    if (o + 4 <= a.src_len) return __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)o, 0, 0);
    uint32_t w = 0;
    for (uint32_t b = 0; b < 4; b++)
        if (o + b < a.src_len) w |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (uint32_t)(o + b), 0, 0) << (8 * b);
    return w;
}

struct Window {
    uint32_t w0, w1, w2; // bytes [wb, wb + 256), [wb + 256, +512), [wb + 512, +768) of the block
    uint32_t wb;
};

__device__ __forceinline__ uint32_t win_byte(const Window &W, uint32_t p) { // p uniform, wb <= p < wb + 768
    const uint32_t rel = p - W.wb, l = (rel >> 2) & 63, sh = 8 * (rel & 3);
    const uint32_t sel = rel >> 8;
    const uint32_t w = sel == 0 ? __builtin_amdgcn_readlane(W.w0, l)
                                : (sel == 1 ? __builtin_amdgcn_readlane(W.w1, l) : __builtin_amdgcn_readlane(W.w2, l));
    return (w >> sh) & 0xff;
}

__device__ __forceinline__ void win_advance(const Lz4Args &a, __amdgpu_buffer_rsrc_t r, uint64_t base, Window &W,
                                            int lane) {
    W.w0 = W.w1;
    W.w1 = W.w2;
    W.wb += 256;
    W.w2 = src_dword(a, r, base + W.wb + 512 + 4 * (uint32_t)lane);
}

// ring[from, to) -> dst[from, to), 16 bytes per lane (from 16-aligned; up to 15 bytes past `to`
// may be written: the slot is a multiple of 16 and bytes past the block's size are never read)
__device__ __forceinline__ void ring_flush(const uint8_t *ring, uint8_t *dst, uint32_t from, uint32_t to, int lane) {
    for (uint32_t p = from + 16 * (uint32_t)lane; p < to; p += 1024)
        *(uint4 *)(dst + p) = *(const uint4 *)(ring + (p & RMASK));
}

__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Output goes to the LDS ring only; the ring is flushed to the slot 4 KiB at a time with
// 16-byte stores (kept at most ~8 KiB behind), so the sequence loop issues no global stores —
// on gfx9 stores count in vmcnt, and a store in flight would make every window read wait.
__device__ __forceinline__ void ring_keep_up(const uint8_t *ring, uint8_t *dst, uint32_t upto, uint32_t &flushed,
                                             int lane) {
    if (upto - flushed >= 8192) {
        wave_fence();
        ring_flush(ring, dst, flushed, flushed + 4096, lane);
        flushed += 4096;
    }
}

__global__ __launch_bounds__(64) void lz4_block_kernel(Lz4Args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t ring[];
    const uint64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const spec_lz4_block blk = a.blocks[b];
    const uint64_t base = blk.src_off;
    const uint32_t n = blk.src_len;
    uint8_t *dst = a.slots + b * a.slot;
    const uint32_t cap = (uint32_t)a.slot;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.src, (short)0, (int)(uint32_t)(a.src_len > 0xffffffffull ? 0xffffffffull : a.src_len), 0x00020000);
    bool err = base + n > a.src_len;
    if (!err && blk.stored) { // a block the writer stored uncompressed
        err = n > cap;
        if (!err)
            for (uint32_t i = lane; i < n; i += 64) dst[i] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, (uint32_t)(base + i), 0, 0);
        if (lane == 0) {
            a.sizes[b] = err ? 0xffffffffu : n;
            a.status[b] = err ? 1 : 0;
        }
        return;
    }
    err |= n == 0;
    Window W;
    W.wb = 0;
    W.w0 = src_dword(a, r, base + 4 * (uint32_t)lane);
    W.w1 = src_dword(a, r, base + 256 + 4 * (uint32_t)lane);
    W.w2 = src_dword(a, r, base + 512 + 4 * (uint32_t)lane);
    uint32_t ip = 0, op = 0, flushed = 0;
    while (!err && ip < n) {
        while (ip - W.wb >= 256) win_advance(a, r, base, W, lane);
        const uint32_t token = win_byte(W, ip++);
        uint32_t ll = token >> 4;
        if (ll == 15) {
            for (;;) {
                if (ip >= n) {
                    err = true;
                    break;
                }
                while (ip - W.wb >= 256) win_advance(a, r, base, W, lane);
                const uint32_t x = win_byte(W, ip++);
                ll += x;
                if (x != 255) break;
            }
            if (err) break;
        }
        if (ll) {
            if (ll > n - ip || ll > cap - op) {
                err = true;
                break;
            }
            for (uint32_t c = 0; c < ll; c += 64) {
                ring_keep_up(ring, dst, op + c, flushed, lane);
                while (ip + c - W.wb >= 256) win_advance(a, r, base, W, lane);
                const uint32_t rel = ip + c - W.wb + (uint32_t)lane; // < 320
                const uint32_t addr = ((rel >> 2) & 63) * 4;
                const uint32_t v0 = __builtin_amdgcn_ds_bpermute(addr, W.w0);
                const uint32_t v1 = __builtin_amdgcn_ds_bpermute(addr, W.w1);
                const uint32_t v = (rel >> 8) ? v1 : v0;
                const uint8_t byte = (uint8_t)(v >> (8 * (rel & 3)));
                if (c + lane < ll) ring[(op + c + lane) & RMASK] = byte;
            }
            ip += ll;
            op += ll;
        }
        uint32_t ml = token & 15;
        if (ip == n && ml == 0) break;
        if (ip + 2 > n) {
            err = true;
            break;
        }
        while (ip - W.wb >= 256) win_advance(a, r, base, W, lane);
        const uint32_t off = win_byte(W, ip) | (win_byte(W, ip + 1) << 8);
        ip += 2;
        if (off == 0) {
            err = true;
            break;
        }
        ml += 4;
        if (ml == 19) {
            for (;;) {
                if (ip >= n) {
                    err = true;
                    break;
                }
                while (ip - W.wb >= 256) win_advance(a, r, base, W, lane);
                const uint32_t x = win_byte(W, ip++);
                ml += x;
                if (x != 255) break;
            }
            if (err) break;
        }
        if (off > op || ml > cap - op) {
            err = true;
            break;
        }
        wave_fence();
        const bool from_ring = off + ml <= RING;
        __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc((void *)dst, (short)0, (int)cap, 0x00020000);
        if (!from_ring) { // the source is read back from the slot: everything before op stored first
            ring_flush(ring, dst, flushed, op, lane);
            flushed = op & ~15u;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        for (uint32_t c = 0; c < ml; c += 64) {
            ring_keep_up(ring, dst, op + c, flushed, lane);
            const uint32_t i = c + lane;
            // out[op + i] = out[op - off + (i mod off)]: the source is always output before op
            const uint32_t s = op - off + (off >= ml ? i : i % off);
            uint8_t byte = 0;
            if (i < ml) {
                byte = from_ring ? ring[s & RMASK]
                                 : (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(dr, s, 0, 16); // sc1: L2, not L1
            }
            __builtin_amdgcn_wave_barrier();
            if (i < ml) ring[(op + i) & RMASK] = byte;
        }
        wave_fence();
        op += ml;
    }
    if (!err) {
        wave_fence();
        ring_flush(ring, dst, flushed, op, lane);
    }
    if (lane == 0) {
        a.sizes[b] = err ? 0xffffffffu : op;
        a.status[b] = err ? 1 : 0;
    }
}

// exclusive scan of the block sizes (one workgroup) -> offsets[0..nblocks], all-ones if any
// block failed
__global__ __launch_bounds__(1024) void lz4_scan_kernel(const uint32_t *sizes, uint64_t nblocks, uint64_t *offsets,
                                                        uint64_t *total) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry_s;
    __shared__ int err_s;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) {
        carry_s = 0;
        err_s = 0;
    }
    __syncthreads();
    for (uint64_t b0 = 0; b0 < nblocks; b0 += 1024) {
        const uint64_t i = b0 + t;
        uint64_t v = i < nblocks ? sizes[i] : 0;
        if (v == 0xffffffffu) {
            err_s = 1;
            v = 0;
        }
        uint64_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint64_t before = 0;
        for (int k = 0; k < w; k++) before += wsum[k];
        const uint64_t carry = carry_s;
        if (i < nblocks) offsets[i] = carry + before + x - v;
        __syncthreads();
        if (t == 1023) carry_s = carry + before + x;
        __syncthreads();
    }
    if (t == 0) {
        offsets[nblocks] = carry_s;
        *total = err_s ? ~0ull : carry_s;
    }
}

// one workgroup per block: slot -> out + offset (16-byte loads from the slot, byte-aligned
// destination assembled with dword stores where aligned)
__global__ __launch_bounds__(256) void lz4_gather_kernel(const uint8_t *slots, uint64_t slot, const uint32_t *sizes,
                                                         const uint64_t *offsets, uint64_t nblocks, uint8_t *out,
                                                         uint64_t out_cap, const uint64_t *total) {
    const uint64_t b = blockIdx.x;
    if (*total == ~0ull || *total > out_cap) return;
    const uint32_t n = sizes[b];
    const uint8_t *s = slots + b * slot;
    uint8_t *d = out + offsets[b];
    // head bytes until d is 4-aligned, then dwords (unaligned source reads), then the tail
    uint32_t head = (uint32_t)((4 - ((uint64_t)d & 3)) & 3);
    if (head > n) head = n;
    if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
    const uint32_t body = (n - head) / 4;
    for (uint32_t i = threadIdx.x; i < body; i += blockDim.x) {
        const uint8_t *q = s + head + 4 * i;
        const uint32_t v = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
        *(uint32_t *)(d + head + 4 * i) = v;
    }
    const uint32_t done = head + 4 * body;
    if (threadIdx.x < n - done) d[done + threadIdx.x] = s[done + threadIdx.x];
}

} // namespace

int launch_lz4_decompress(const uint8_t *src, uint64_t src_len, const spec_lz4_block *blocks, uint64_t nblocks,
                          uint8_t *slots, uint64_t slot, uint32_t *sizes, uint8_t *status, hipStream_t stream) {
    if (nblocks == 0) return 0;
    Lz4Args a = {src, src_len, blocks, nblocks, slots, slot, sizes, status};
    hipLaunchKernelGGL(lz4_block_kernel, dim3((unsigned)nblocks), dim3(64), RING, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lz4_pack(const uint8_t *slots, uint64_t slot, const uint32_t *sizes, uint64_t nblocks, uint8_t *out,
                    uint64_t out_cap, uint64_t *offsets, uint64_t *total, hipStream_t stream) {
    hipLaunchKernelGGL(lz4_scan_kernel, dim3(1), dim3(1024), 0, stream, sizes, nblocks, offsets, total);
    if (nblocks)
        hipLaunchKernelGGL(lz4_gather_kernel, dim3((unsigned)nblocks), dim3(256), 0, stream, slots, slot, sizes,
                           (const uint64_t *)offsets, nblocks, out, out_cap, (const uint64_t *)total);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
