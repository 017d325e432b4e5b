// decode_flat.hip — the precompiled (run-time schema) decode kernels and their launcher.
// The device code lives in decode_core.hpp; schema-specialised variants of the same body
// are compiled at run time by jit.cpp.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "decode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

template <int SLAB>
__global__ __launch_bounds__(256) void decode_flat_kernel(DecodeArgs a) {
    decode_flat_entry<false, SLAB, RuntimeSpec>(a);
}

template <int SLAB>
__global__ __launch_bounds__(256) void decode_flat_kernel_persistent(DecodeArgs a) {
    decode_flat_entry<true, SLAB, RuntimeSpec>(a);
}

bool persistent_decode() {
    static int v = [] {
        const char *e = getenv("SPEC_AMD_PERSIST");
        return (e && e[0] == '1') ? 1 : 0;
    }();
    return v == 1;
}

int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cus[dev] = v;
    }
    return cus[dev];
}

int launch_decode_flat(const DecodeArgs &a, double avg_record, hipStream_t stream) {
    if (a.n <= a.r0) return 0;
    const int cls = decode_slab_class(avg_record);
    const int slab = cls < 3 ? slab_bytes(cls) : 0;
    dim3 grid(decode_grid(a.n - a.r0, device_cus(), slab, persistent_decode())), block(256);
#define SPEC_LAUNCH(K)                                                                                          \
    switch (cls) {                                                                                              \
    case 0: hipLaunchKernelGGL(K<slab_bytes(0)>, grid, block, DEC_WAVES * slab_bytes(0), stream, a); break;     \
    case 1: hipLaunchKernelGGL(K<slab_bytes(1)>, grid, block, DEC_WAVES * slab_bytes(1), stream, a); break;     \
    case 2: hipLaunchKernelGGL(K<slab_bytes(2)>, grid, block, DEC_WAVES * slab_bytes(2), stream, a); break;     \
    default: hipLaunchKernelGGL(K<0>, grid, block, 0, stream, a); break;                                        \
    }
    if (persistent_decode()) {
        SPEC_LAUNCH(decode_flat_kernel_persistent)
    } else {
        SPEC_LAUNCH(decode_flat_kernel)
    }
#undef SPEC_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
