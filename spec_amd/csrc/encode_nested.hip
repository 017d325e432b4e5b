// encode_nested.hip — bulk encode of messages with a list<message> field (BASELINE config 4):
// the precompiled kernels (schema read from the kernel arguments, RuntimeEnc policies) and the
// launcher, which prefers the schema-specialised kernels of jit.cpp.  Device code and the
// algorithm: encode_nested_core.hpp.  Three launches, no host sync: sizes -> scan of block
// sums -> write.
#include <hip/hip_runtime.h>

#include "encode_nested_core.hpp"
#include "spec_internal.hpp"

namespace spec {

namespace {

__global__ __launch_bounds__(NENC_BLOCK) void nested_enc_size_kernel(NestedEncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    nested_enc_size_body<RuntimeEnc, RuntimeEnc>(a, smem);
}

__global__ __launch_bounds__(1024) void nested_enc_scan_kernel(NestedEncodeArgs a) {
    scan_block_sums(a.block_sums, a.nblocks, a.total);
}

__global__ __launch_bounds__(NENC_BLOCK) void nested_enc_write_kernel(NestedEncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    nested_enc_write_body<RuntimeEnc, RuntimeEnc>(a, smem);
}

} // namespace

int launch_nested_encode(const spec_nested_schema *schema, const NestedEncodeArgs &a, bool write,
                         hipStream_t stream) {
    if (a.nblocks) {
        const int j = jit_launch_nested_encode(schema, a, false, stream);
        if (j < 0) return -1;
        if (j == 0)
            hipLaunchKernelGGL(nested_enc_size_kernel, dim3((unsigned)a.nblocks), dim3(NENC_BLOCK),
                               nenc_size_lds_bytes(), stream, a);
    }
    hipLaunchKernelGGL(nested_enc_scan_kernel, dim3(1), dim3(1024), 0, stream, a);
    if (write && a.nblocks) {
        const int j = jit_launch_nested_encode(schema, a, true, stream);
        if (j < 0) return -1;
        if (j == 0)
            hipLaunchKernelGGL(nested_enc_write_kernel, dim3((unsigned)a.nblocks), dim3(NENC_BLOCK),
                               nenc_write_lds_bytes(), stream, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
