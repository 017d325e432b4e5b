// decode_nested.hip — precompiled (run-time schema) kernels of the list<message> decoder and
// their launchers.  The device code lives in decode_nested_core.hpp; jit.cpp compiles the
// one-pass kernel specialised to the outer and item schemas.
//
// Two ways to place the items (include/spec_amd.h):
//   spec_decode_nested_index + spec_decode_nested: nested_count_tail_kernel (per 64-record
//     group: item total, from each record's last 64 bytes; nested_count_kernel parses the staged
//     span instead) + nested_scan_kernel (exclusive scan of group totals, total items), then
//     nested_decode_kernel;
//   spec_decode_nested_onepass: nested_onepass_kernel alone (decoupled look-back over the
//     groups' item counts), after zeroing the look-back words.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "decode_nested_core.hpp"
#include "spec_internal.hpp"

namespace spec {

namespace {

__global__ __launch_bounds__(256) void nested_count_kernel(NestedArgs a) { nested_count_body(a); }

__global__ __launch_bounds__(256) void nested_count_tail_kernel(NestedArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t wins[256 * TAIL_STRIDE];
    nested_count_tail_body(a, wins);
}

// Exclusive scan of the group totals + total items: one 1024-thread workgroup.  Tiles of
// 16 x 1024 totals: loaded coalesced (all 16 loads in flight) into LDS as u32 (item counts of
// 64 records), each thread then scans 16 CONSECUTIVE totals serially, one block scan of the
// thread sums, results back through LDS, coalesced stores.  (A block scan per 1024 totals
// costs ~1 us of barriers and shuffles on the one CU; this does one per tile.)
__global__ __launch_bounds__(1024) void nested_scan_kernel(NestedArgs a) {
    constexpr int PER = 16, TILE = 1024 * PER;
    __shared__ uint32_t tv[TILE + TILE / 32]; // +1 pad word per 32: thread-contiguous reads spread banks
    __shared__ uint64_t wsum[1024 / 64];
    const uint64_t ngroups = (a.n + 63) / 64;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    auto at = [](int k) { return k + (k >> 5); };
    uint64_t carry = 0;
    for (uint64_t tile = 0; tile < ngroups; tile += TILE) {
        uint64_t v[PER];
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint64_t k = tile + (uint64_t)i * 1024 + t;
            v[i] = k < ngroups ? a.group_base[k] : 0;
        }
#pragma unroll
        for (int i = 0; i < PER; i++) tv[at(i * 1024 + t)] = (uint32_t)v[i];
        __syncthreads();
        uint32_t mine[PER], sum = 0;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            mine[i] = tv[at(t * PER + i)];
            sum += mine[i];
        }
        uint64_t x = sum; // inclusive wave scan of the thread sums
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint64_t before = 0, tile_total = 0;
#pragma unroll
        for (int k = 0; k < 1024 / 64; k++) {
            before += k < w ? wsum[k] : 0;
            tile_total += wsum[k];
        }
        // exclusive offsets within the tile fit 32 bits (item_begin is uint32)
        uint32_t run = (uint32_t)(before + x - sum);
#pragma unroll
        for (int i = 0; i < PER; i++) {
            tv[at(t * PER + i)] = run;
            run += mine[i];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const uint64_t k = tile + (uint64_t)i * 1024 + t;
            if (k < ngroups) a.group_base[k] = carry + tv[at(i * 1024 + t)];
        }
        carry += tile_total;
        __syncthreads();
    }
    if (t == 0) *a.total = carry;
}

__global__ __launch_bounds__(256) void nested_decode_kernel(NestedArgs a) {
    nested_decode_body<RuntimeSpec, RuntimeSpec, false>(a);
}

__global__ __launch_bounds__(64 * DEC_WAVES) void nested_onepass_kernel(NestedArgs a) {
    nested_decode_body<RuntimeSpec, RuntimeSpec, true>(a);
}

__global__ __launch_bounds__(256) void nested_decode_ranges_kernel(NestedArgs a) {
    nested_decode_body<RuntimeSpec, RuntimeSpec, false, true>(a);
}

int g_nested_mode = NESTED_XCD;

} // namespace

// NESTED_HALVES: slabs sized for half a group (32 records), so twice the waves fit a CU's LDS;
// every group is then staged and decoded as two halves (the path a group larger than its
// slab takes anyway).
uint32_t nested_slab_for_mode(double avg_record) {
    return nested_slab_bytes(g_nested_mode == NESTED_HALVES ? avg_record * 0.5 : avg_record);
}

int launch_nested_index(NestedArgs a, double avg_record, hipStream_t stream) {
    if (a.n == 0) {
        (void)hipMemsetAsync(a.total, 0, sizeof(uint64_t), stream);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    a.slab = nested_slab_for_mode(avg_record);
    const uint64_t groups = (a.n + 63) / 64;
    if (g_nested_mode == NESTED_TAILCOUNT || g_nested_mode == NESTED_XCD) {
        hipLaunchKernelGGL(nested_count_tail_kernel, dim3((unsigned)((groups + 3) / 4)), dim3(256), 0, stream, a);
    } else {
        dim3 grid((unsigned)((groups + DEC_WAVES - 1) / DEC_WAVES)), block(64 * DEC_WAVES);
        hipLaunchKernelGGL(nested_count_kernel, grid, block, (size_t)DEC_WAVES * a.slab, stream, a);
    }
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(nested_scan_kernel, dim3(1), dim3(1024), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The decode pass after the index kernels: a wave per 64-record group; its items found by an
// owner search (NESTED_GROUPS, default) or from ranges precomputed into LDS (NESTED_RANGES).
int launch_nested_decode(const spec_nested_schema *schema, NestedArgs a, double avg_record, hipStream_t stream) {
    if (a.n == 0) return 0;
    a.slab = nested_slab_for_mode(avg_record);
    a.xcd = g_nested_mode == NESTED_XCD ? 1u : 0u;
    const int mode = g_nested_mode >= NESTED_HALVES ? NESTED_GROUPS : g_nested_mode;
    const int j = jit_launch_nested(schema, a, mode, stream);
    if (j != 0) return j > 0 ? 0 : -1;
    const uint64_t groups = (a.n + 63) / 64;
    unsigned blocks = (unsigned)((groups + DEC_WAVES - 1) / DEC_WAVES);
    if (a.xcd) blocks = (blocks + 7) / 8 * 8;
    dim3 grid(blocks), block(64 * DEC_WAVES);
    if (mode == NESTED_RANGES)
        hipLaunchKernelGGL(nested_decode_ranges_kernel, grid, block,
                           (size_t)DEC_WAVES * (a.slab + NESTED_RANGE_BYTES), stream, a);
    else
        hipLaunchKernelGGL(nested_decode_kernel, grid, block, (size_t)DEC_WAVES * a.slab, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The look-back one-pass kernel (0.31 ms vs 0.13 ms for the index kernels + decode on config 4)
// is chosen at build time only (-DSPEC_AB_LOOKBACK=1), never by the environment.
#ifndef SPEC_AB_LOOKBACK
#define SPEC_AB_LOOKBACK 0
#endif
bool nested_lookback() { return SPEC_AB_LOOKBACK != 0; }
// -DSPEC_AB_NESTED_PAIR_LB=1: spec_decode_nested_onepass on the wave-pair kernel with one
// look-back per group (round 6, nested_decode_pair ONEPASS: the stream read once).  Config 4:
// 0.1754-0.1764 ms against 0.1109-0.1131 ms for the count + scan + two-pass pair decode
// (gpurun_out/nencp2, two runs each on one box): 16 K groups each waiting on the agent-scope
// look-back words of the groups before it hold their slabs idle; off by default.
#ifndef SPEC_AB_NESTED_PAIR_LB
#define SPEC_AB_NESTED_PAIR_LB 0
#endif

// The two-pass decode on a wave pair per group (decode_nested_core.hpp nested_decode_pair; the
// JIT kernels only): -DSPEC_AB_NESTED_PAIR=0 runs a wave per group instead.
#ifndef SPEC_AB_NESTED_PAIR
#define SPEC_AB_NESTED_PAIR 1
#endif
bool nested_pair() { return SPEC_AB_NESTED_PAIR != 0; }

// spec_decode_nested_onepass: by default the index kernels + the decode kernel back to back
// (no host round trip); with SPEC_AB_LOOKBACK: DEC_WAVES groups per block (one per wave), one
// look-back per block over the earlier blocks, the look-back words (group_base[0 .. blocks])
// zeroed first, on the same stream.
int launch_nested_onepass(const spec_nested_schema *schema, NestedArgs a, double avg_record, hipStream_t stream) {
    if (a.n == 0) {
        (void)hipMemsetAsync(a.total, 0, sizeof(uint64_t), stream);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (!nested_lookback()) {
        if (SPEC_AB_NESTED_PAIR_LB && nested_pair()) {
            // the wave-pair decode with one look-back per group: the stream read once
            a.slab = nested_slab_bytes(avg_record);
            const uint64_t groups = (a.n + 63) / 64;
            if (hipMemsetAsync(a.group_base, 0, (groups + 1) * sizeof(uint64_t), stream) != hipSuccess) return -1;
            const int j = jit_launch_nested(schema, a, NESTED_PAIR_ONEPASS, stream);
            if (j < 0) return -1;
            if (j > 0) return 0;
        }
        if (launch_nested_index(a, avg_record, stream)) return -1;
        return launch_nested_decode(schema, a, avg_record, stream);
    }
    a.slab = nested_slab_bytes(avg_record);
    const uint64_t groups = (a.n + 63) / 64;
    const uint64_t blocks = (groups + DEC_WAVES - 1) / DEC_WAVES;
    if (hipMemsetAsync(a.group_base, 0, (blocks + 1) * sizeof(uint64_t), stream) != hipSuccess) return -1;
    const int j = jit_launch_nested(schema, a, NESTED_ONEPASS, stream);
    if (j < 0) return -1;
    if (j == 0)
        hipLaunchKernelGGL(nested_onepass_kernel, dim3((unsigned)blocks), dim3(64 * DEC_WAVES),
                           (size_t)DEC_WAVES * a.slab, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec

extern "C" void spec_set_nested_mode(int mode) {
    if (mode == spec::NESTED_GROUPS || mode == spec::NESTED_RANGES || mode == spec::NESTED_HALVES ||
        mode == spec::NESTED_TAILCOUNT || mode == spec::NESTED_XCD)
        spec::g_nested_mode = mode;
}
