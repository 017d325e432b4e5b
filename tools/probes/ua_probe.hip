// Probe: are unaligned LDS stores (ds_write_b16/b32/b64 at any byte address) exact on this GPU,
// and what do they cost against aligned ones?  Build: hipcc --offload-arch=gfx950 -O3 ua_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __attribute__((address_space(3))) uint8_t lds8;


template <int NB>
__device__ __forceinline__ void stn(lds8 *p, uint64_t v) {
    if constexpr (NB == 8) { typedef __attribute__((address_space(3), aligned(1))) uint64_t u; *(u *)p = v; }
    else if constexpr (NB == 4) { typedef __attribute__((address_space(3), aligned(1))) uint32_t u; *(u *)p = (uint32_t)v; }
    else if constexpr (NB == 2) { typedef __attribute__((address_space(3), aligned(1))) uint16_t u; *(u *)p = (uint16_t)v; }
    else *p = (uint8_t)v;
}

// each lane writes 8 pieces of sizes 1,2,4,8 at consecutive unaligned positions of its own 64-B row
extern "C" __global__ void probe(uint8_t *out, int shift) {
    __shared__ uint8_t s[64 * 64];
    lds8 *S = (lds8 *)s;
    const int t = threadIdx.x;
    for (int i = 0; i < 64; i++) S[t * 64 + i] = 0xEE;
    __syncthreads();
    int p = t * 64 + ((t + shift) & 7);
    uint64_t v = 0x0102030405060708ull * (uint64_t)(t + 1);
    stn<1>(S + p, v); p += 1;
    stn<2>(S + p, v >> 8); p += 2;
    stn<4>(S + p, v >> 16); p += 4;
    stn<8>(S + p, v ^ 0xA5A5A5A5A5A5A5A5ull); p += 8;
    stn<4>(S + p, v >> 3); p += 4;
    stn<2>(S + p, v >> 5); p += 2;
    stn<8>(S + p, ~v); p += 8;
    stn<1>(S + p, 0x5A); p += 1;
    __syncthreads();
    for (int i = 0; i < 64; i++) out[t * 64 + i] = S[t * 64 + i];
}

template <bool UNALIGNED>
__global__ void speed(uint64_t *cyc, uint32_t *sink, int iters) {
    __shared__ uint8_t s[64 * 256];
    lds8 *S = (lds8 *)s;
    const int t = threadIdx.x & 63;
    uint64_t v = t * 0x9E3779B97F4A7C15ull;
    int p = t * 256 + (UNALIGNED ? ((t * 3) & 7) : 0);
    const uint64_t c0 = clock64();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 16; j++) stn<8>(S + p + 8 * (j & 15), v + j);
        v = v * 6364136223846793005ull + 1;
    }
    __syncthreads();
    const uint64_t c1 = clock64();
    if (t == 0) cyc[blockIdx.x] = c1 - c0;
    sink[blockIdx.x * 64 + t] = S[t * 256 + 5];
}

int main() {
    uint8_t *d;
    hipMalloc(&d, 64 * 64);
    int bad = 0;
    for (int shift = 0; shift < 8; shift++) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, shift);
        uint8_t h[64 * 64];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        for (int t = 0; t < 64; t++) {
            uint8_t want[64];
            memset(want, 0xEE, 64);
            int p = (t + shift) & 7;
            uint64_t v = 0x0102030405060708ull * (uint64_t)(t + 1);
            auto put = [&](uint64_t x, int nb) { memcpy(want + p, &x, nb); p += nb; };
            put(v, 1); put(v >> 8, 2); put(v >> 16, 4); put(v ^ 0xA5A5A5A5A5A5A5A5ull, 8); put(v >> 3, 4);
            put(v >> 5, 2); put(~v, 8); put(0x5A, 1);
            if (memcmp(want, h + 64 * t, 64)) bad++;
        }
    }
    printf("unaligned LDS stores: %s (%d bad rows of 512)\n", bad ? "MISMATCH" : "exact", bad);
    uint64_t *cyc;
    uint32_t *sink;
    hipMalloc(&cyc, 1024 * 8);
    hipMalloc(&sink, 1024 * 64 * 4);
    for (int u = 0; u < 2; u++) {
        for (int rep = 0; rep < 2; rep++) {
            if (u) hipLaunchKernelGGL(speed<true>, dim3(1024), dim3(64), 0, 0, cyc, sink, 1000);
            else hipLaunchKernelGGL(speed<false>, dim3(1024), dim3(64), 0, 0, cyc, sink, 1000);
        }
        uint64_t h[1024];
        hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < 1024; i++) m += h[i];
        printf("%s b64 stores: %.2f cycles per wave-instruction\n", u ? "unaligned" : "aligned  ", m / 1024 / 16000);
    }
    return bad ? 1 : 0;
}
