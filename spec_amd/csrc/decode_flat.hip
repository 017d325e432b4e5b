// decode_flat.hip — the precompiled (run-time schema) decode kernels and their launcher.
// The device code lives in decode_core.hpp; schema-specialised variants of the same body
// are compiled at run time by jit.cpp.
#include <hip/hip_runtime.h>

#include "decode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

constexpr int GENERIC_RECS = 64;

template <int SLAB>
__global__ __launch_bounds__(256) void decode_flat_kernel(DecodeArgs a) {
    decode_flat_body<GENERIC_RECS, SLAB, RuntimeSpec>(a);
}

int launch_decode_flat(const DecodeArgs &a, double avg_record, hipStream_t stream) {
    constexpr int R = GENERIC_RECS;
    uint64_t waves = (a.n + R - 1) / R;
    uint64_t blocks = (waves + DEC_WAVES - 1) / DEC_WAVES;
    if (blocks == 0) return 0;
    dim3 grid((unsigned)blocks), block(256);
    switch (decode_slab_class(avg_record, R)) {
    case 0: hipLaunchKernelGGL(decode_flat_kernel<slab_bytes(R, 0)>, grid, block, DEC_WAVES * slab_bytes(R, 0), stream, a); break;
    case 1: hipLaunchKernelGGL(decode_flat_kernel<slab_bytes(R, 1)>, grid, block, DEC_WAVES * slab_bytes(R, 1), stream, a); break;
    case 2: hipLaunchKernelGGL(decode_flat_kernel<slab_bytes(R, 2)>, grid, block, DEC_WAVES * slab_bytes(R, 2), stream, a); break;
    default: hipLaunchKernelGGL(decode_flat_kernel<0>, grid, block, 0, stream, a); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
