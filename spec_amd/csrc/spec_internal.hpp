// spec_internal.hpp — kernel argument blocks and launcher declarations shared by the HIP
// translation units of libspec_amd.so (not part of the public C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/spec_amd.h"
#include "decode_core.hpp"
#include "encode_core.hpp"
#include "encode_nested_core.hpp"
#include "decode_nested_core.hpp"

namespace spec {

// Build-time A/B (make HIPFLAGS+="-DSPEC_AB_TREE_TILE=0"): 1 generates the tree encoder's
// record-tile writer (jit.cpp gen_tile) where it applies, 0 the level-fused write sets always.
#ifndef SPEC_AB_TREE_TILE
#define SPEC_AB_TREE_TILE 1
#endif
// the tile writer's waves per workgroup (= field blocks of the records' table) and waves per SIMD
// (its register budget): 4 WPE / W workgroups per CU share the LDS, per workgroup the image of
// the tile's output range and a dummy dword
#ifndef SPEC_AB_TREE_TILE_W
#define SPEC_AB_TREE_TILE_W 4
#endif
#ifndef SPEC_AB_TREE_TILE_WPE
#define SPEC_AB_TREE_TILE_WPE 4 // waves per SIMD the kernel is compiled for (amdgpu_waves_per_eu)
#endif
constexpr int TREE_TILE_W = SPEC_AB_TREE_TILE_W, TREE_TILE_WPE = SPEC_AB_TREE_TILE_WPE;
// measurement build (-DSPEC_AB_TILE_CLOCK=1, tools/tile_clock.py): each tile's workgroup stores the
// wall clock at its phase boundaries over its records' B.tmask entries (read back from the workspace)
#ifndef SPEC_AB_TILE_CLOCK
#define SPEC_AB_TILE_CLOCK 0
#endif
// the tile writer's rows below the records in rounds over the tables of a depth (jit.cpp
// tile_round_ok); 0: one loop per table.  Measured on pkg1: depth-1 phase 24.0 vs 23.7 us per
// tile (tools/tile_clock.py), encode 0.2864 vs 0.2844 ms — no gain, off
#ifndef SPEC_AB_TILE_ROUNDS
#define SPEC_AB_TILE_ROUNDS 0
#endif
// the tile writer's LDS image starts zeroed and rows OR their dwords into it (tree_core.hpp
// LSink::word), so the emitter's stores need no edge cases
#ifndef SPEC_AB_TILE_OR
#define SPEC_AB_TILE_OR 1
#endif
constexpr uint32_t TREE_TILE_IMG = ((163840u / (4u * TREE_TILE_WPE / TREE_TILE_W)) - 32u) & ~15u;

// encode_nested.hip
int launch_nested_encode(const spec_nested_schema *schema, const NestedEncodeArgs &a, bool write,
                         hipStream_t stream);
// jit.cpp: schema-specialised nested encode pass 1 (write=false) or 3; 1 launched, 0 use the
// precompiled kernel, <0 HIP error.
int jit_launch_nested_encode(const spec_nested_schema *schema, const NestedEncodeArgs &a, bool write,
                             hipStream_t stream);
long long jit_compile_only_nested_encode(const spec_nested_schema *schema);
int launch_decode_flat(DecodeArgs a, double avg_record, hipStream_t stream);
// lz4_device.hip
int launch_lz4_decompress(const uint8_t *src, uint64_t src_len, const spec_lz4_block *blocks, uint64_t nblocks,
                          uint8_t *slots, uint64_t slot, uint32_t *sizes, uint8_t *status, hipStream_t stream);
int launch_lz4_pack(const uint8_t *slots, uint64_t slot, const uint32_t *sizes, uint64_t nblocks, uint8_t *out,
                    uint64_t out_cap, uint64_t *offsets, uint64_t *total, hipStream_t stream);
// xxHash32 of the frame content: data != null appends data[0, len); digest != null writes the digest
int launch_lz4_content(spec_lz4_content *c, const uint8_t *data, uint64_t len, uint32_t *digest, hipStream_t stream);
// frames_device.hip
size_t frames_index_device_workspace(uint64_t len);
int launch_frames_index_device(const uint8_t *buf, uint64_t len, uint64_t *ends, uint64_t cap, uint64_t *count,
                               uint64_t *consumed, int32_t *status, void *ws, hipStream_t stream);
int device_cus(); // CUs of the current device (cached)
void note_hip_error(hipError_t e); // capi.hip: remembered for spec_last_hip_error()
// capi.hip: bytes copied to the device on st from a pooled pinned slot of the current device (no
// host wait: the pool grows while every slot's copy is in flight; not graph-capturable)
hipError_t pinned_upload(void *dst, const void *src, size_t bytes, hipStream_t st);
bool persistent_decode(); // build-time A/B variants (decode_flat.hip): SPEC_AB_PERSIST
unsigned decode_wpb();     // SPEC_AB_WPB (waves per block, default 1)
int flat_pair();
bool nested_pair(); // decode_nested.hip: SPEC_AB_NESTED_PAIR           // SPEC_AB_FLAT_PAIR: 1 wide schemas / 2 every schema on wave pairs (decode_flat_pair)
int launch_parse(DecodeArgs a, uint32_t *sizes, uint32_t root, double avg_record, hipStream_t stream);
int launch_nested_index(NestedArgs a, double avg_record, hipStream_t stream);
int launch_nested_decode(const spec_nested_schema *schema, NestedArgs a, double avg_record, hipStream_t stream);
int launch_nested_onepass(const spec_nested_schema *schema, NestedArgs a, double avg_record, hipStream_t stream);
// jit.cpp: nested decode specialised to the outer and item schemas (onepass: look-back kernel,
// else the decode pass after the index kernels); 1 launched, 0 use the precompiled kernel,
// <0 HIP error.  a.slab must be set.
// mode: NESTED_ONEPASS (look-back kernel), NESTED_GROUPS (a wave per group after the index
// kernels, items found by an owner search), NESTED_RANGES (same, items from ranges precomputed
// into LDS by their records' lanes), NESTED_HALVES (as GROUPS, slabs for half a group),
// NESTED_TAILCOUNT (as GROUPS, the count pass from each record's last 64 bytes), NESTED_XCD (as
// TAILCOUNT with an XCD-aware block order for the decode pass: the default)
// NESTED_PAIR_ONEPASS (round 6): the decode on wave pairs with one look-back per group, no
// index kernels (spec_decode_nested_onepass)
enum { NESTED_ONEPASS = 0, NESTED_GROUPS = 1, NESTED_RANGES = 2, NESTED_HALVES = 3, NESTED_TAILCOUNT = 4, NESTED_XCD = 5,
       NESTED_PAIR_ONEPASS = 6 };
int jit_launch_nested(const spec_nested_schema *schema, const NestedArgs &a, int mode, hipStream_t stream);
bool nested_lookback(); // build-time SPEC_AB_LOOKBACK: spec_decode_nested_onepass runs the look-back kernel
long long jit_compile_only_nested(const spec_nested_schema *schema);
// jit.cpp: schema-specialised decode kernel (hiprtc); returns 1 if launched, 0 if the caller
// should launch the generic kernel, <0 on a HIP error.
int jit_launch_decode_flat(const spec_schema *schema, const DecodeArgs &a, double avg_record, hipStream_t stream);
int jit_prepare_decode_flat(const spec_schema *schema, double avg_record);
void jit_set_enabled(int on);
long long jit_compile_only(const spec_schema *schema, double avg_record);
long long jit_compile_only_encode(const spec_schema *schema);
int launch_encode_size(const spec_schema *schema, const EncodeArgs &a, hipStream_t stream);
// capi.hip: spec_encode_flat's passes (ENC_PASS_SIZE: sizes + scan into the workspace, heaps
// checked; ENC_PASS_WRITE: the write pass over a workspace the size pass filled), every end
// offset + ends_base (shard.hip: a shard's first byte in the whole batch).
enum { ENC_PASS_SIZE = 1, ENC_PASS_WRITE = 2 };
int encode_flat_passes(const spec_schema *schema, const void *const *columns, const uint8_t *const *heaps,
                       const uint64_t *heap_lens, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *ends,
                       uint64_t ends_base, void *workspace, size_t workspace_size, uint64_t *total, int passes,
                       hipStream_t stream);
int launch_encode_write(const spec_schema *schema, const EncodeArgs &a, hipStream_t stream);
int launch_encode_wide_size(const WideEncodeArgs &a, hipStream_t stream);
int launch_encode_wide_write(const WideEncodeArgs &a, hipStream_t stream);
// jit.cpp: schema-specialised encode pass 1 (write=false) or 3; 1 launched, 0 use the
// precompiled kernel, <0 HIP error.
int jit_launch_encode(const spec_schema *schema, const EncodeArgs &a, bool write, hipStream_t stream);

// jit.cpp: schema-specialised schema-tree group kernels (tree_decode.hip)
struct TreeDesc;
const hipFunction_t *jit_tree_kernels(const TreeDesc &D);
long long jit_compile_only_tree(const TreeDesc &D);

} // namespace spec
