// decode_flat.hip — the precompiled (run-time schema) decode kernels and their launcher.
// The device code lives in decode_core.hpp; schema-specialised variants of the same body
// are compiled at run time by jit.cpp.
#include <hip/hip_runtime.h>

#include "decode_core.hpp"
#include "spec_internal.hpp"

namespace spec {

__global__ __launch_bounds__(256) void decode_flat_kernel(DecodeArgs a) { decode_flat_entry<false, RuntimeSpec>(a); }

__global__ __launch_bounds__(256) void decode_flat_kernel_persistent(DecodeArgs a) {
    decode_flat_entry<true, RuntimeSpec>(a);
}

// Launch variants measured in rounds 1-3 and not kept as defaults are chosen when the library
// is BUILT (make HIPFLAGS+="-DSPEC_AB_PERSIST=1 ..."), never by a process's environment:
//   SPEC_AB_PERSIST=1  persistent, software-pipelined decode (no faster on MI355X);
//   SPEC_AB_NOXCD=1    blocks in launch order instead of XCD-aware contiguous shares (1.3 %
//                      slower on the 1M Flat16 decode, tools/ab.py, 6 interleaved rounds, r02);
//   SPEC_AB_WPB=k      k waves per block (1 packs the most slabs per CU: LDS is the limit).
#ifndef SPEC_AB_PERSIST
#define SPEC_AB_PERSIST 0
#endif
#ifndef SPEC_AB_NOXCD
#define SPEC_AB_NOXCD 0
#endif
#ifndef SPEC_AB_WPB
#define SPEC_AB_WPB 1
#endif
bool persistent_decode() { return SPEC_AB_PERSIST != 0; }
bool xcd_swizzle_decode() { return SPEC_AB_NOXCD == 0; }
unsigned decode_wpb() { return SPEC_AB_WPB >= 1 && SPEC_AB_WPB <= 4 ? SPEC_AB_WPB : 1; }
//   SPEC_AB_FLAT_PAIR    2 (default): every schema's group of 64 records on a wave pair sharing
//                        one staged slab, half the fields each (decode_core.hpp decode_flat_pair;
//                        Flat16: 0.0745 -> 0.0684 ms, 0.68 -> 0.74 of HBM; wide40 0.181 -> 0.154 ms);
//                        1: only the fast_wide schemas; 0: none (a wave per group)
#ifndef SPEC_AB_FLAT_PAIR
#define SPEC_AB_FLAT_PAIR 2
#endif
int flat_pair() { return SPEC_AB_FLAT_PAIR; }

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
