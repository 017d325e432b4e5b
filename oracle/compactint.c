/*
 * compactint.c — reconstruction of github.com/basecomplextech/baselibrary/encoding/compactint
 * (pinned in the reference at v0.0.0-20250218120829-9ca66e53fd5f, go.mod:6, go.sum:1).
 *
 * TEST INFRASTRUCTURE (oracle).  The module is NOT present in /root/reference, so this
 * file restates its published contract as the reference's call sites and tests use it:
 *   - PutReverse{Uint,Int}{32,64}(p [MaxLen]byte, v) write into the TAIL of p and return
 *     n; callers copy p[MaxLen-n:]          (internal/encode/int.go:14-22, size.go:10-17)
 *   - Reverse{Uint,Int}{32,64}(b) read the varint that ENDS at len(b) and return (v, n),
 *     n < 0 on error, INCLUDING a buffer that ends mid-varint: the tests
 *     internal/decode/msg_test.go:88-108 and list_test.go:89-109 require a lone 0xff to
 *     produce "invalid table size"/"invalid data size", which only a negative n can do.
 *   - ReverseSize(b) <= 0 on error          (internal/decode/type.go:53-57)
 * Byte layout (UNPINNED — no golden vector exists in the reference): LEB128 7-bit groups,
 * continuation bit 0x80, byte order reversed so the least-significant group is the LAST
 * byte (adjacent to the type byte) and the most-significant group (MSB clear) is first.
 * Signed values use zigzag like Go's encoding/binary.PutVarint.  Overflow rules follow
 * encoding/binary.Uvarint with MaxLen32 = 5, MaxLen64 = 10.
 * Keep this the ONLY place the varint layout is defined on the oracle side; the device
 * side mirror is spec_amd/csrc/spec_device.hpp (rvarint_bf and the encoders' varint emitters).
 */
#include "spec_oracle.h"

int so_put_reverse_uint64(uint8_t p[SO_MAX_LEN64], uint64_t v) {
    int i = SO_MAX_LEN64 - 1;
    while (v >= 0x80) {
        p[i--] = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    p[i] = (uint8_t)v;
    return SO_MAX_LEN64 - i;
}

int so_put_reverse_uint32(uint8_t p[SO_MAX_LEN32], uint32_t v) {
    int i = SO_MAX_LEN32 - 1;
    while (v >= 0x80) {
        p[i--] = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    p[i] = (uint8_t)v;
    return SO_MAX_LEN32 - i;
}

int so_put_reverse_int32(uint8_t p[SO_MAX_LEN32], int32_t v) {
    uint32_t ux = (uint32_t)v << 1;
    if (v < 0) ux = ~ux;
    return so_put_reverse_uint32(p, ux);
}

int so_put_reverse_int64(uint8_t p[SO_MAX_LEN64], int64_t v) {
    uint64_t ux = (uint64_t)v << 1;
    if (v < 0) ux = ~ux;
    return so_put_reverse_uint64(p, ux);
}

/* Reads backwards from b[len-1]; i counts bytes consumed so far. */
uint64_t so_reverse_uint64(const uint8_t *b, size_t len, int *n) {
    uint64_t x = 0;
    unsigned s = 0;
    for (int i = 0;; i++) {
        if (i == SO_MAX_LEN64) {
            *n = -(i + 1); /* overflow: too long */
            return 0;
        }
        if ((size_t)i >= len) {
            *n = -(i + 1); /* incomplete */
            return 0;
        }
        uint8_t c = b[len - 1 - (size_t)i];
        if (c < 0x80) {
            if (i == SO_MAX_LEN64 - 1 && c > 1) {
                *n = -(i + 1); /* overflow: value > 64 bits */
                return 0;
            }
            *n = i + 1;
            return x | ((uint64_t)c << s);
        }
        x |= (uint64_t)(c & 0x7f) << s;
        s += 7;
    }
}

uint32_t so_reverse_uint32(const uint8_t *b, size_t len, int *n) {
    uint32_t x = 0;
    unsigned s = 0;
    for (int i = 0;; i++) {
        if (i == SO_MAX_LEN32) {
            *n = -(i + 1);
            return 0;
        }
        if ((size_t)i >= len) {
            *n = -(i + 1);
            return 0;
        }
        uint8_t c = b[len - 1 - (size_t)i];
        if (c < 0x80) {
            if (i == SO_MAX_LEN32 - 1 && c > 0x0f) {
                *n = -(i + 1); /* value > 32 bits */
                return 0;
            }
            *n = i + 1;
            return x | ((uint32_t)c << s);
        }
        x |= (uint32_t)(c & 0x7f) << s;
        s += 7;
    }
}

int32_t so_reverse_int32(const uint8_t *b, size_t len, int *n) {
    uint32_t ux = so_reverse_uint32(b, len, n);
    int32_t x = (int32_t)(ux >> 1);
    if (ux & 1) x = ~x;
    return x;
}

int64_t so_reverse_int64(const uint8_t *b, size_t len, int *n) {
    uint64_t ux = so_reverse_uint64(b, len, n);
    int64_t x = (int64_t)(ux >> 1);
    if (ux & 1) x = ~x;
    return x;
}

int so_reverse_size(const uint8_t *b, size_t len) {
    for (int i = 0; i < SO_MAX_LEN64; i++) {
        if ((size_t)i >= len) return -(i + 1);
        if (b[len - 1 - (size_t)i] < 0x80) return i + 1;
    }
    return -(SO_MAX_LEN64 + 1);
}
