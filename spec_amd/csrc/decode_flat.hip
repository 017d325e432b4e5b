// decode_flat.hip — the precompiled (run-time schema) decode kernels and their launcher.
// The device code lives in decode_core.hpp; schema-specialised variants of the same body
// are compiled at run time by jit.cpp.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "decode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

__global__ __launch_bounds__(256) void decode_flat_kernel(DecodeArgs a) { decode_flat_entry<false, RuntimeSpec>(a); }

__global__ __launch_bounds__(256) void decode_flat_kernel_persistent(DecodeArgs a) {
    decode_flat_entry<true, RuntimeSpec>(a);
}

bool persistent_decode() {
    static int v = [] {
        const char *e = getenv("SPEC_AMD_PERSIST");
        return (e && e[0] == '1') ? 1 : 0;
    }();
    return v == 1;
}

// XCD-aware block order (consecutive groups on one XCD's L2) is the default: 1.3 % faster on the
// 1M Flat16 decode (tools/ab.py, 6 interleaved rounds, r02); SPEC_AMD_XCD=0 turns it off
bool xcd_swizzle_decode() {
    static int v = [] {
        const char *e = getenv("SPEC_AMD_XCD");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    return v == 1;
}

unsigned decode_wpb() {
    static unsigned v = [] {
        const char *e = getenv("SPEC_AMD_WPB");
        int w = e ? atoi(e) : 1;
        return (unsigned)(w >= 1 && w <= 4 ? w : 1);
    }();
    return v;
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

int launch_decode_flat(DecodeArgs a, double avg_record, hipStream_t stream) {
    if (a.n <= a.r0) return 0;
    const DecodeLaunch L = decode_launch(a.n - a.r0, avg_record, device_cus(), persistent_decode(), decode_wpb());
    a.slab = L.slab;
    a.xcd = xcd_swizzle_decode() && !persistent_decode();
    dim3 grid(L.blocks), block(64 * L.wpb);
    if (persistent_decode())
        hipLaunchKernelGGL(decode_flat_kernel_persistent, grid, block, L.lds, stream, a);
    else
        hipLaunchKernelGGL(decode_flat_kernel, grid, block, L.lds, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
