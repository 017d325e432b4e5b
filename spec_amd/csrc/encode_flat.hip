// encode_flat.hip — bulk encode of SoA columns into flat spec messages (gfx950).
//
// Replaces, per record, the generated Write() sequence over the Writer stack machine:
//   w := spec.NewMessageWriterBuffer(buf)                       writer_msg.go:26-31
//   w.Field(tag).<Kind>(v) for each field in schema order         internal/writer/msg.go:99-211
//     -> ValueWriter.<Kind> -> encode.Encode<Kind> (internal/encode/...) + pushData
//     -> writer.field(tag): insertion-sorted table entry {tag, end - message.start}
//                                                                 internal/writer/writer.go:409-436,
//                                                                 internal/writer/stack_msg.go:37-61
//   w.Build() -> endMessage -> encode.EncodeMessageTable          internal/writer/writer.go:520-553,
//                                                                 internal/encode/msg.go:15-77
// The table order depends only on the schema's tags, so the host computes it once
// (`order`, same insertion-sort tie rule); per record only the sizes vary.
//
// Three launches, no host sync:
//   1. encode_size_kernel  : per-record encoded size, per-block sums (reads only the columns
//                            that affect sizes: varint and string/bytes columns)
//   2. encode_scan_kernel  : exclusive scan of block sums (one workgroup) + total
//   3. encode_write_kernel : per-block scan of recomputed sizes -> record offsets; each lane
//                            emits its record into the wave's LDS slab (dword-merging byte
//                            emitter), then the wave copies the slab to HBM with 16-byte
//                            stores; ends[] written coalesced.  A wave whose output span does
//                            not fit the slab emits straight to HBM.
#include <hip/hip_runtime.h>

#include "../../include/spec_amd.h"
#include "encode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

// ---- pass 1: block sums ------------------------------------------------------------------

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__global__ __launch_bounds__(ENC_BLOCK) void encode_size_kernel(EncodeArgs a) {
    __shared__ uint64_t part[ENC_BLOCK / 64];
    __shared__ int errs;
    if (threadIdx.x == 0) errs = 0;
    __syncthreads();
    uint64_t r = (uint64_t)blockIdx.x * ENC_BLOCK + threadIdx.x;
    uint64_t sz = 0;
    bool err = false;
    if (r < a.n) sz = record_size(a.f, r, a.check_heaps, err).total;
    if (err) errs = 1;
    uint64_t s = wave_sum(sz);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < ENC_BLOCK / 64; w++) t += part[w];
        a.block_sums[blockIdx.x] = errs ? ~0ull : t;
    }
}

// ---- pass 2: exclusive scan of block sums (one workgroup), total ----------------------

__global__ __launch_bounds__(1024) void encode_scan_kernel(EncodeArgs a) { scan_block_sums(a.block_sums, a.nblocks, a.total); }

// ---- pass 3: write ------------------------------------------------------------------------

constexpr int ENC_SLAB = 20 * 1024 - 128; // per-wave output staging

__global__ __launch_bounds__(ENC_BLOCK) void encode_write_kernel(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint64_t wsum[ENC_BLOCK / 64];
    __shared__ uint8_t inv_order[SPEC_MAX_FIELDS];
    const uint64_t total = a.block_sums[a.nblocks];
    if (total > a.out_cap) return; // capacity error or encoder error (total == ~0)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < a.f.nfields) inv_order[a.f.order[threadIdx.x]] = (uint8_t)threadIdx.x;

    const uint64_t r = (uint64_t)blockIdx.x * ENC_BLOCK + threadIdx.x;
    const bool valid = r < a.n;
    bool err = false;
    RecSize rs = {0, 0, false};
    if (valid) rs = record_size(a.f, r, a.check_heaps, err);
    // block exclusive scan of sizes
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

    // wave output span [S, E)
    if ((uint64_t)blockIdx.x * ENC_BLOCK + wave * 64 >= a.n) return;
    const uint64_t S = __builtin_amdgcn_readfirstlane((uint32_t)start) |
                       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(start >> 32)) << 32);
    const int last = (int)((a.n - ((uint64_t)blockIdx.x * ENC_BLOCK + wave * 64)) < 64
                               ? a.n - ((uint64_t)blockIdx.x * ENC_BLOCK + wave * 64) - 1
                               : 63);
    const uint64_t Ev = __shfl(start + rs.total, last);
    const uint64_t E = __builtin_amdgcn_readfirstlane((uint32_t)Ev) |
                       ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(Ev >> 32)) << 32);
    const uint64_t head = ((uintptr_t)(a.out + S)) & 15; // slab pos of byte S keeps 16-B phase
    if (head + (E - S) + 16 <= (uint64_t)ENC_SLAB) {
        uint8_t *slab = smem + wave * ENC_SLAB;
        LdsSink k{slab};
        if (valid) emit_message(a.f, k, (int)(head + (start - S)), r, rs, inv_order);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // copy slab [head, head + E - S) -> out[S, E) with 16-B stores
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
        emit_message(a.f, k, (long long)start, r, rs, inv_order);
    }
}

static size_t enc_lds_bytes() { return (size_t)(ENC_BLOCK / 64) * ENC_SLAB; }

int launch_encode_size(const EncodeArgs &a, hipStream_t stream) {
    if (a.nblocks) hipLaunchKernelGGL(encode_size_kernel, dim3((unsigned)a.nblocks), dim3(ENC_BLOCK), 0, stream, a);
    hipLaunchKernelGGL(encode_scan_kernel, dim3(1), dim3(1024), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_write(const EncodeArgs &a, hipStream_t stream) {
    if (a.nblocks)
        hipLaunchKernelGGL(encode_write_kernel, dim3((unsigned)a.nblocks), dim3(ENC_BLOCK), enc_lds_bytes(), stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
