// decode_flat.hip — bulk decode of flat spec messages into SoA columns (gfx950).
//
// Replaces, per record, spec.OpenMessageErr (internal/types/msg.go:43-55 ->
// internal/decode/msg.go:14-99) followed by one typed getter per schema field
// (internal/types/msg.go:219-475: m.field(tag) = table.Offset(tag) binary search
// (internal/format/msg.go:227-265) + decode.Decode<Kind>(bytes[:end])).
//
// Mapping (MI355X, wave64):
//   * one wave = 64 consecutive records, one record per lane;
//   * the wave's contiguous byte span [ends[base-1], ends[base+63]) is staged into the wave's
//     private LDS slab with LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per instruction,
//     range-checked by the buffer descriptor) — one fully coalesced HBM read of the stream;
//   * each lane then parses its record from LDS: trailer (type, two reverse varints) from
//     one 16-byte tail window, table sortedness check, one probe per field at the field's
//     expected table index (falling back to the reference's exact binary search), value
//     decode from the field's 16-byte tail window;
//   * column writes are lane-strided => coalesced per field;
//   * a wave whose span exceeds its slab parses straight from HBM via range-checked buffer
//     loads (same code, GlobalSrc) — correctness never depends on record sizes.
#include <hip/hip_runtime.h>

#include "../../include/spec_amd.h"
#include "spec_device.hpp"
#include "spec_internal.hpp"

namespace spec {

constexpr int DEC_WAVES = 4; // waves per 256-thread block
constexpr int SLAB_GUARD = 16;

// ---- message table lookup --------------------------------------------------------------

// exact reference binary search (offset_small/offset_big), returns end offset or -1
template <class Src>
__device__ __noinline__ long long table_search(const Src &s, typename Src::pos_t tstart, uint32_t nent,
                                               bool big, uint32_t tag) {
    int left = 0, right = (int)nent - 1;
    while (left <= right) {
        int mid = (int)((unsigned)(left + right) >> 1);
        uint32_t cur;
        typename Src::pos_t p;
        if (big) {
            p = tstart + (typename Src::pos_t)mid * 6;
            cur = (s.u8(p) << 8) | s.u8(p + 1);
        } else {
            p = tstart + (typename Src::pos_t)mid * 3;
            cur = s.u8(p);
        }
        if (cur < tag) {
            left = mid + 1;
        } else if (cur > tag) {
            right = mid - 1;
        } else {
            if (big)
                return ((long long)s.u8(p + 2) << 24) | (s.u8(p + 3) << 16) | (s.u8(p + 4) << 8) | s.u8(p + 5);
            return (s.u8(p + 1) << 8) | s.u8(p + 2);
        }
    }
    return -1;
}

// ---- value decoders: field slice [lo, e), type at e-1 (internal/decode/...) ------------

struct Val {
    uint64_t v0, v1, v2, v3; // up to 32 bytes of column payload, little-endian
};

template <class Src>
__device__ __forceinline__ Val decode_value(const Src &s, uint32_t kind, typename Src::pos_t lo,
                                            typename Src::pos_t e, long long to_stream) {
    Val out = {0, 0, 0, 0};
    long long flen = (long long)(e - lo);
    if (flen <= 0) return out; // empty => zero value, no error
    Tail t = load_tail(s, e);
    uint32_t type = (uint32_t)t.q0 & 0xff;
    uint64_t R = tail_r(t);
    uint32_t R2 = tail_r2(t);
    long long avail = flen - 1; // bytes before the type byte
    int m;
    switch (kind) {
    case K_BOOL: // DecodeBool, byte.go:38-51: true iff type == TypeTrue
        out.v0 = type == T_TRUE;
        break;
    case K_BYTE: // DecodeByte, byte.go:16-34
        if (type == T_BYTE && flen >= 2) out.v0 = R & 0xff;
        break;
    case K_INT16:
    case K_INT32:
    case K_INT64: { // DecodeInt16/32/64, int.go:16-135
        long long x;
        if (type == T_INT16 || type == T_INT32) {
            uint32_t u = (uint32_t)rvarint<5>(R, R2, avail, m);
            x = unzigzag32(u);
        } else if (type == T_INT64) {
            x = unzigzag64(rvarint<10>(R, R2, avail, m));
        } else {
            break;
        }
        if (m < 0) break;
        if (kind == K_INT16 && (x < -32768 || x > 32767)) break;
        if (kind == K_INT32 && type == T_INT64 && (x < INT32_MIN || x > INT32_MAX)) break;
        out.v0 = (uint64_t)x;
        if (kind == K_INT16) out.v0 &= 0xffff;
        if (kind == K_INT32) out.v0 &= 0xffffffffu;
        break;
    }
    case K_UINT16:
    case K_UINT32:
    case K_UINT64: { // DecodeUint16/32/64, uint.go:16-125
        uint64_t x;
        if (type == T_UINT16 || type == T_UINT32) {
            x = rvarint<5>(R, R2, avail, m);
        } else if (type == T_UINT64) {
            x = rvarint<10>(R, R2, avail, m);
        } else {
            break;
        }
        if (m < 0) break;
        if (kind == K_UINT16 && x > 0xffffull) break;
        if (kind == K_UINT32 && x > 0xffffffffull) break;
        out.v0 = x;
        break;
    }
    case K_FLOAT32: { // DecodeFloat32, float.go:15-32 (via float64 + range check)
        if (type == T_FLOAT32) {
            if (flen < 5) break;
            uint32_t b = (uint32_t)(R & 0xffffffffu);
            uint32_t ex = (b >> 23) & 0xff;
            if (ex == 0xff) {
                if ((b & 0x7fffff) == 0) break; // +-Inf fails the +-MaxFloat32 range check
                b |= 0x00400000u;               // NaN: quieted by the float64 round trip
            }
            out.v0 = b;
        } else if (type == T_FLOAT64) {
            if (flen < 9) break;
            uint64_t d = R;
            uint32_t ex = (uint32_t)(d >> 52) & 0x7ff;
            bool nan = ex == 0x7ff && (d & 0xfffffffffffffull);
            if (!nan) {
                // |d| > MaxFloat32 (0x47EFFFFFE0000000) => overflow error => 0
                if ((d & 0x7fffffffffffffffull) > 0x47EFFFFFE0000000ull) break;
            }
            out.v0 = f64_to_f32_bits(d);
        }
        break;
    }
    case K_FLOAT64: { // DecodeFloat64, float.go:34-78
        if (type == T_FLOAT32) {
            if (flen < 5) break;
            out.v0 = f32_to_f64_bits((uint32_t)(R & 0xffffffffu));
        } else if (type == T_FLOAT64) {
            if (flen < 9) break;
            out.v0 = R;
        }
        break;
    }
    case K_BIN64: // DecodeBin64, bin.go:15-44: raw 8 bytes before the type byte
        if (type == T_BIN64 && flen >= 9) out.v0 = __builtin_bswap64(R);
        break;
    case K_BIN128:
        if (type == T_BIN128 && flen >= 17) {
            out.v0 = load_le64(s, e - 17);
            out.v1 = __builtin_bswap64(R);
        }
        break;
    case K_BIN256:
        if (type == T_BIN256 && flen >= 33) {
            out.v0 = load_le64(s, e - 33);
            out.v1 = load_le64(s, e - 25);
            out.v2 = load_le64(s, e - 17);
            out.v3 = __builtin_bswap64(R);
        }
        break;
    case K_STRING:
    case K_BYTES: { // DecodeString (string.go:15-70) / DecodeBytes (bytes.go:14-58)
        bool str = kind == K_STRING;
        if (type != (str ? T_STRING : T_BYTES)) break;
        uint32_t len = (uint32_t)rvarint<5>(R, R2, avail, m);
        if (m < 0) break;
        long long end = (long long)(e - 1) - m - (str ? 1 : 0); // skip the NUL for strings
        long long off = end - (long long)len;
        if (end < (long long)lo || off < (long long)lo) break;
        if (len) out.v0 = (uint64_t)(uint32_t)(off + to_stream) | ((uint64_t)len << 32);
        break;
    }
    }
    return out;
}

template <class Src>
__device__ __forceinline__ void store_value(const DecodeArgs &a, uint32_t f, uint32_t kind, uint64_t r,
                                            const Val &v) {
    uint8_t *col = (uint8_t *)a.cols[f];
    switch (kind) {
    case K_BOOL:
    case K_BYTE: col[r] = (uint8_t)v.v0; break;
    case K_INT16:
    case K_UINT16: ((uint16_t *)col)[r] = (uint16_t)v.v0; break;
    case K_INT32:
    case K_UINT32:
    case K_FLOAT32: ((uint32_t *)col)[r] = (uint32_t)v.v0; break;
    case K_INT64:
    case K_UINT64:
    case K_FLOAT64:
    case K_BIN64:
    case K_STRING:
    case K_BYTES: ((uint64_t *)col)[r] = v.v0; break;
    case K_BIN128: ((ulonglong2 *)col)[r] = make_ulonglong2(v.v0, v.v1); break;
    case K_BIN256: {
        ulonglong2 *c = (ulonglong2 *)col + 2 * r;
        c[0] = make_ulonglong2(v.v0, v.v1);
        c[1] = make_ulonglong2(v.v2, v.v3);
        break;
    }
    }
}

// Parse record r occupying [rs, re) of the source; to_stream converts a source position to a
// stream offset (string/bytes spans).
template <class Src>
__device__ __forceinline__ void decode_record(const Src &s, typename Src::pos_t rs, typename Src::pos_t re,
                                              uint64_t r, const DecodeArgs &a, long long to_stream) {
    using pos_t = typename Src::pos_t;
    uint32_t st = ST_OK;
    bool ok = false, big = false, sorted = true;
    pos_t dstart = 0, tstart = 0;
    uint32_t dsize = 0, nent = 0;
    long long len = (long long)(re - rs);
    if (len > 0) {
        // DecodeMessageTable, internal/decode/msg.go:14-73
        Tail t = load_tail(s, re);
        uint32_t type = (uint32_t)t.q0 & 0xff;
        if (type != T_MESSAGE && type != T_BIG_MESSAGE) {
            st = ST_INVALID_TYPE;
        } else {
            big = type == T_BIG_MESSAGE;
            uint64_t R = tail_r(t);
            uint32_t R2 = tail_r2(t);
            int m1, m2;
            uint32_t tsz = (uint32_t)rvarint<5>(R, R2, len - 1, m1);
            if (m1 < 0) {
                st = ST_INVALID_TABLE_SIZE;
            } else {
                // the data-size varint ends m1 bytes further down: shift the window
                uint64_t Rs = (R >> (8 * m1)) | ((uint64_t)R2 << (64 - 8 * m1));
                uint32_t R2s = m1 >= 2 ? 0u : (R2 >> (8 * m1));
                uint32_t dsz = (uint32_t)rvarint<5>(Rs, R2s, len - 1 - m1, m2);
                if (m2 < 0) {
                    st = ST_INVALID_DATA_SIZE;
                } else {
                    long long tend = (long long)(re - 1) - m1 - m2;
                    long long ts = tend - (long long)tsz;
                    if (ts < (long long)rs || tsz % (big ? 6u : 3u) != 0) {
                        st = ST_INVALID_TABLE;
                    } else if (ts - (long long)dsz < (long long)rs) {
                        st = ST_INVALID_DATA;
                    } else {
                        ok = true;
                        tstart = (pos_t)ts;
                        dstart = (pos_t)(ts - (long long)dsz);
                        dsize = dsz;
                        nent = tsz / (big ? 6u : 3u);
                    }
                }
            }
        }
    }
    if (ok) {
        // strictly increasing tags => a probe at the expected index is what binary search finds
        uint32_t prev = 0;
        for (uint32_t i = 0; i < nent; i++) {
            pos_t p = tstart + (pos_t)i * (big ? 6 : 3);
            uint32_t tg = big ? ((s.u8(p) << 8) | s.u8(p + 1)) : s.u8(p);
            if (i > 0 && tg <= prev) sorted = false;
            prev = tg;
        }
    }
    if (a.status) a.status[r] = (uint8_t)st;

    for (uint32_t f = 0; f < a.nfields; f++) {
        uint32_t tag = a.tags[f];
        uint32_t kind = a.kinds[f];
        long long end = -1;
        if (ok) {
            uint32_t k = a.rank[f];
            bool hit = false;
            if (sorted && k < nent) {
                pos_t p = tstart + (pos_t)k * (big ? 6 : 3);
                if (big) {
                    uint32_t tg = (s.u8(p) << 8) | s.u8(p + 1);
                    if (tg == tag) {
                        end = ((long long)s.u8(p + 2) << 24) | (s.u8(p + 3) << 16) | (s.u8(p + 4) << 8) | s.u8(p + 5);
                        hit = true;
                    }
                } else {
                    if (s.u8(p) == tag) {
                        end = (s.u8(p + 1) << 8) | s.u8(p + 2);
                        hit = true;
                    }
                }
            }
            if (!hit) end = table_search(s, tstart, nent, big, tag);
            if (end > (long long)dsize) end = -1; // m.field: end > dataSize => nil
        }
        Val v = {0, 0, 0, 0};
        if (end > 0) v = decode_value(s, kind, dstart, dstart + (pos_t)end, to_stream);
        store_value<Src>(a, f, kind, r, v);
    }
}

template <int SLAB>
__global__ __launch_bounds__(256) void decode_flat_kernel(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const uint64_t base = ((uint64_t)blockIdx.x * DEC_WAVES + wave) * 64;
    if (base >= a.n) return;
    const uint64_t r = base + lane;
    const bool valid = r < a.n;
    const uint64_t last = (a.n - base) < 64 ? a.n - 1 : base + 63;

    uint64_t rec_hi = valid ? a.ends[r] : 0;
    uint64_t prev = __shfl_up(rec_hi, 1);
    if (lane == 0) prev = base ? a.ends[base - 1] : 0;
    const uint64_t rec_lo = prev;
    const uint64_t span_lo = __builtin_amdgcn_readfirstlane((uint32_t)rec_lo) |
                             ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(rec_lo >> 32)) << 32);
    const uint64_t span_hi_v = __shfl(rec_hi, (int)(last - base));
    const uint64_t span_hi = __builtin_amdgcn_readfirstlane((uint32_t)span_hi_v) |
                             ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(span_hi_v >> 32)) << 32);

    __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.stream, (short)0, (int)(uint32_t)a.stream_len, 0x00020000);

    bool use_lds = false;
    uint64_t aligned_lo = span_lo & ~15ull;
    if (SLAB > 0) {
        uint64_t bytes = span_hi - aligned_lo;
        uint64_t chunks = (bytes + 1023) >> 10;
        use_lds = span_hi >= span_lo && SLAB_GUARD + chunks * 1024 + 16 <= (uint64_t)SLAB;
        if (use_lds) {
            uint8_t *slab = smem + wave * SLAB;
            for (uint32_t c = 0; c < (uint32_t)chunks; c++) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsrc, (__attribute__((address_space(3))) void *)(slab + SLAB_GUARD + c * 1024), 16,
                    (uint32_t)aligned_lo + c * 1024 + lane * 16, 0, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            // the 16-byte chunk holding the stream's last bytes came back zeroed if it
            // straddles the end (whole-access range check): refill it bytewise
            const uint64_t tail = a.stream_len & ~15ull;
            if (tail < a.stream_len && tail >= aligned_lo && tail < span_hi) {
                if (lane < 16 && tail + lane < a.stream_len)
                    slab[SLAB_GUARD + (tail - aligned_lo) + lane] =
                        (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (uint32_t)(tail + lane), 0, 0);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (valid) {
                LdsSrc s{(lds_u8 *)slab};
                int rs = SLAB_GUARD + (int)(rec_lo - aligned_lo);
                int re = SLAB_GUARD + (int)(rec_hi - aligned_lo);
                if (rec_hi < rec_lo) re = rs; // malformed ends: treat as empty
                decode_record(s, rs, re, r, a, (long long)aligned_lo - SLAB_GUARD);
            }
            return;
        }
    }
    if (valid) {
        GlobalSrc s{rsrc, a.stream_len};
        long long rs = (long long)rec_lo, re = (long long)rec_hi;
        if (re < rs) re = rs;
        decode_record(s, rs, re, r, a, 0);
    }
}

// slab bytes per wave for each instantiation (guard + DMA chunks + pad)
constexpr int SLAB_S = SLAB_GUARD + 11 * 1024 + 16 + 16;  // spans <= 11 KiB  (avg rec <~ 150 B)
constexpr int SLAB_M = SLAB_GUARD + 19 * 1024 + 16 + 16;  // spans <= 19 KiB  (avg rec <~ 270 B)
constexpr int SLAB_L = SLAB_GUARD + 35 * 1024 + 16 + 16;  // spans <= 35 KiB  (avg rec <~ 500 B)

int launch_decode_flat(const DecodeArgs &a, double avg_record, hipStream_t stream) {
    uint64_t waves = (a.n + 63) / 64;
    uint64_t blocks = (waves + DEC_WAVES - 1) / DEC_WAVES;
    if (blocks == 0) return 0;
    dim3 grid((unsigned)blocks), block(256);
    double span = avg_record * 64.0 * 1.08 + 64.0;
    if (span <= 11 * 1024) {
        hipLaunchKernelGGL(decode_flat_kernel<SLAB_S>, grid, block, DEC_WAVES * SLAB_S, stream, a);
    } else if (span <= 19 * 1024) {
        hipLaunchKernelGGL(decode_flat_kernel<SLAB_M>, grid, block, DEC_WAVES * SLAB_M, stream, a);
    } else if (span <= 35 * 1024) {
        hipLaunchKernelGGL(decode_flat_kernel<SLAB_L>, grid, block, DEC_WAVES * SLAB_L, stream, a);
    } else {
        hipLaunchKernelGGL(decode_flat_kernel<0>, grid, block, 0, stream, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
