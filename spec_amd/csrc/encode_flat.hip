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
// Passes 1 and 3 are, for schemas jit.cpp accepts, schema-specialised kernels compiled at run
// time (all column loads of a record issued together, the table emitted from registers).
#include <hip/hip_runtime.h>

#include "../../include/spec_amd.h"
#include "encode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

// Kernel bodies: encode_core.hpp (RuntimeEnc here; jit.cpp instantiates them per schema).

__global__ __launch_bounds__(ENC_BLOCK) void encode_size_kernel(EncodeArgs a) { encode_size_body<RuntimeEnc>(a); }

__global__ __launch_bounds__(1024) void encode_scan_kernel(EncodeArgs a) { scan_block_sums(a.block_sums, a.nblocks, a.total); }

__global__ __launch_bounds__(ENC_BLOCK) void encode_write_kernel(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    encode_write_body<RuntimeEnc>(a, smem);
}

// Schemas with more than SPEC_KFIELDS fields: the same bodies over a field set in device memory
// (RuntimeEnc reads it through WideEncFields' pointers; no schema-specialised kernel).
__global__ __launch_bounds__(ENC_BLOCK) void encode_wide_size_kernel(WideEncodeArgs a) {
    encode_size_body<RuntimeEnc>(a);
}

__global__ __launch_bounds__(1024) void encode_wide_scan_kernel(WideEncodeArgs a) {
    scan_block_sums(a.block_sums, a.nblocks, a.total);
}

__global__ __launch_bounds__(ENC_BLOCK) void encode_wide_write_kernel(WideEncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    encode_write_body<RuntimeEnc>(a, smem);
}

int launch_encode_wide_size(const WideEncodeArgs &a, hipStream_t stream) {
    if (a.nblocks) hipLaunchKernelGGL(encode_wide_size_kernel, dim3((unsigned)a.nblocks), dim3(ENC_BLOCK), 0, stream, a);
    hipLaunchKernelGGL(encode_wide_scan_kernel, dim3(1), dim3(1024), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_wide_write(const WideEncodeArgs &a, hipStream_t stream) {
    if (!a.nblocks) return 0;
    hipLaunchKernelGGL(encode_wide_write_kernel, dim3((unsigned)a.nblocks), dim3(ENC_BLOCK), enc_write_lds_bytes(),
                       stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_size(const spec_schema *schema, const EncodeArgs &a, hipStream_t stream) {
    int j = a.nblocks ? jit_launch_encode(schema, a, false, stream) : 1;
    if (j < 0) return -1;
    if (j == 0) hipLaunchKernelGGL(encode_size_kernel, dim3((unsigned)a.nblocks), dim3(ENC_BLOCK), 0, stream, a);
    hipLaunchKernelGGL(encode_scan_kernel, dim3(1), dim3(1024), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_write(const spec_schema *schema, const EncodeArgs &a, hipStream_t stream) {
    if (!a.nblocks) return 0;
    int j = jit_launch_encode(schema, a, true, stream);
    if (j < 0) return -1;
    if (j == 0)
        hipLaunchKernelGGL(encode_write_kernel, dim3((unsigned)a.nblocks), dim3(ENC_BLOCK), enc_write_lds_bytes(),
                           stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
