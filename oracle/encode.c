/*
 * encode.c — restatement of internal/encode/...: append `value | type` encoders.
 * TEST INFRASTRUCTURE (oracle).
 */
#include <string.h>

#include "spec_oracle.h"

/* encodeSize / encodeSizeType, internal/encode/size.go:9-30 */
static int encode_size(so_buf *b, uint32_t size) {
    uint8_t p[SO_MAX_LEN32];
    int n = so_put_reverse_uint32(p, size);
    memcpy(so_buf_grow(b, (size_t)n), p + (SO_MAX_LEN32 - n), (size_t)n);
    return n;
}

static int encode_size_type(so_buf *b, uint32_t size, uint8_t type) {
    uint8_t p[SO_MAX_LEN32];
    int n = so_put_reverse_uint32(p, size);
    uint8_t *q = so_buf_grow(b, (size_t)n + 1);
    memcpy(q, p + (SO_MAX_LEN32 - n), (size_t)n);
    q[n] = type;
    return n + 1;
}

/* EncodeBool / EncodeByte, internal/encode/byte.go:12-27 */
so_err so_encode_bool(so_buf *b, int v, int *n) {
    so_buf_grow(b, 1)[0] = v ? SO_TYPE_TRUE : SO_TYPE_FALSE;
    *n = 1;
    return NULL;
}

so_err so_encode_byte(so_buf *b, uint8_t v, int *n) {
    uint8_t *p = so_buf_grow(b, 2);
    p[0] = v;
    p[1] = SO_TYPE_BYTE;
    *n = 2;
    return NULL;
}

/* EncodeInt16/32/64, internal/encode/int.go:13-47 (Int16 goes through the 32-bit routine) */
static int put32(so_buf *b, const uint8_t *p, int n, uint8_t type) {
    uint8_t *q = so_buf_grow(b, (size_t)n + 1);
    memcpy(q, p, (size_t)n);
    q[n] = type;
    return n + 1;
}

so_err so_encode_int16(so_buf *b, int16_t v, int *n) {
    uint8_t p[SO_MAX_LEN32];
    int m = so_put_reverse_int32(p, (int32_t)v);
    *n = put32(b, p + (SO_MAX_LEN32 - m), m, SO_TYPE_INT16);
    return NULL;
}

so_err so_encode_int32(so_buf *b, int32_t v, int *n) {
    uint8_t p[SO_MAX_LEN32];
    int m = so_put_reverse_int32(p, v);
    *n = put32(b, p + (SO_MAX_LEN32 - m), m, SO_TYPE_INT32);
    return NULL;
}

so_err so_encode_int64(so_buf *b, int64_t v, int *n) {
    uint8_t p[SO_MAX_LEN64];
    int m = so_put_reverse_int64(p, v);
    *n = put32(b, p + (SO_MAX_LEN64 - m), m, SO_TYPE_INT64);
    return NULL;
}

/* EncodeUint16/32/64, internal/encode/uint.go:13-47 */
so_err so_encode_uint16(so_buf *b, uint16_t v, int *n) {
    uint8_t p[SO_MAX_LEN32];
    int m = so_put_reverse_uint32(p, (uint32_t)v);
    *n = put32(b, p + (SO_MAX_LEN32 - m), m, SO_TYPE_UINT16);
    return NULL;
}

so_err so_encode_uint32(so_buf *b, uint32_t v, int *n) {
    uint8_t p[SO_MAX_LEN32];
    int m = so_put_reverse_uint32(p, v);
    *n = put32(b, p + (SO_MAX_LEN32 - m), m, SO_TYPE_UINT32);
    return NULL;
}

so_err so_encode_uint64(so_buf *b, uint64_t v, int *n) {
    uint8_t p[SO_MAX_LEN64];
    int m = so_put_reverse_uint64(p, v);
    *n = put32(b, p + (SO_MAX_LEN64 - m), m, SO_TYPE_UINT64);
    return NULL;
}

/* EncodeFloat32/64, internal/encode/float.go:15-27: big-endian IEEE bits + type */
so_err so_encode_float32(so_buf *b, float v, int *n) {
    uint32_t u;
    memcpy(&u, &v, 4);
    uint8_t *p = so_buf_grow(b, 5);
    for (int i = 0; i < 4; i++) p[i] = (uint8_t)(u >> (24 - 8 * i));
    p[4] = SO_TYPE_FLOAT32;
    *n = 5;
    return NULL;
}

so_err so_encode_float64(so_buf *b, double v, int *n) {
    uint64_t u;
    memcpy(&u, &v, 8);
    uint8_t *p = so_buf_grow(b, 9);
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(u >> (56 - 8 * i));
    p[8] = SO_TYPE_FLOAT64;
    *n = 9;
    return NULL;
}

/* EncodeBin64/128/256, internal/encode/bin.go:13-39: opaque bytes (bin.MarshalTo) + type */
static so_err encode_bin(so_buf *b, const uint8_t *v, int w, uint8_t type, int *n) {
    uint8_t *p = so_buf_grow(b, (size_t)w + 1);
    memcpy(p, v, (size_t)w);
    p[w] = type;
    *n = w + 1;
    return NULL;
}

so_err so_encode_bin64(so_buf *b, const uint8_t v[8], int *n) { return encode_bin(b, v, 8, SO_TYPE_BIN64, n); }
so_err so_encode_bin128(so_buf *b, const uint8_t v[16], int *n) { return encode_bin(b, v, 16, SO_TYPE_BIN128, n); }
so_err so_encode_bin256(so_buf *b, const uint8_t v[32], int *n) { return encode_bin(b, v, 32, SO_TYPE_BIN256, n); }

/* EncodeBytes, internal/encode/bytes.go:14-26: data | rvarint(len) | type */
so_err so_encode_bytes(so_buf *b, const uint8_t *v, size_t len, int *n) {
    *n = 0;
    if (len > SO_MAX_SIZE) return "encode: bytes too large";
    if (len) memcpy(so_buf_grow(b, len), v, len);
    *n = (int)len + encode_size_type(b, (uint32_t)len, SO_TYPE_BYTES);
    return NULL;
}

/* EncodeString, internal/encode/string.go:14-26: data | 0x00 | rvarint(len) | type */
so_err so_encode_string(so_buf *b, const char *s, size_t len, int *n) {
    *n = 0;
    if (len > SO_MAX_SIZE) return "encode: string too large";
    uint8_t *p = so_buf_grow(b, len + 1);
    if (len) memcpy(p, s, len);
    p[len] = 0;
    *n = (int)len + 1 + encode_size_type(b, (uint32_t)len, SO_TYPE_STRING);
    return NULL;
}

/* EncodeStruct, internal/encode/struct.go:14-21 */
so_err so_encode_struct(so_buf *b, int64_t data_size, int *n) {
    *n = 0;
    if (data_size > SO_MAX_SIZE) return "encode: struct too large";
    *n = encode_size_type(b, (uint32_t)data_size, SO_TYPE_STRUCT);
    return NULL;
}

/* EncodeListTable, internal/encode/list.go:15-75: table | rvarint(data) | rvarint(table) | 70/71 */
so_err so_encode_list_table(so_buf *b, int64_t data_size, const so_list_element *t, size_t cnt, int *n) {
    *n = 0;
    if (data_size > SO_MAX_SIZE) return "encode: list too large";
    int big = so_is_big_list(t, cnt);
    uint8_t type = big ? SO_TYPE_BIG_LIST : SO_TYPE_LIST;
    size_t esize = big ? 4 : 2;
    size_t size = cnt * esize;
    if (size > SO_MAX_SIZE) return "encode: list table too large";
    uint8_t *p = so_buf_grow(b, size);
    for (size_t i = 0; i < cnt; i++) {
        uint32_t o = t[i].offset;
        uint8_t *q = p + i * esize;
        if (big) {
            q[0] = (uint8_t)(o >> 24);
            q[1] = (uint8_t)(o >> 16);
            q[2] = (uint8_t)(o >> 8);
            q[3] = (uint8_t)o;
        } else {
            q[0] = (uint8_t)(o >> 8); /* uint16(elem.Offset) truncates */
            q[1] = (uint8_t)o;
        }
    }
    int m = (int)size;
    m += encode_size(b, (uint32_t)data_size);
    m += encode_size_type(b, (uint32_t)size, type);
    *n = m;
    return NULL;
}

/* EncodeMessageTable, internal/encode/msg.go:15-77: small entry u8 tag + u16 BE end,
 * big entry u16 BE tag + u32 BE end */
so_err so_encode_message_table(so_buf *b, int64_t data_size, const so_message_field *t, size_t cnt, int *n) {
    *n = 0;
    if (data_size > SO_MAX_SIZE) return "encode: message too large";
    int big = so_is_big_message(t, cnt);
    uint8_t type = big ? SO_TYPE_BIG_MESSAGE : SO_TYPE_MESSAGE;
    size_t fsize = big ? 6 : 3;
    size_t size = cnt * fsize;
    if (size > SO_MAX_SIZE) return "encode: message table too large";
    uint8_t *p = so_buf_grow(b, size);
    for (size_t i = 0; i < cnt; i++) {
        uint8_t *q = p + i * fsize;
        uint16_t tag = t[i].tag;
        uint32_t o = t[i].offset;
        if (big) {
            q[0] = (uint8_t)(tag >> 8);
            q[1] = (uint8_t)tag;
            q[2] = (uint8_t)(o >> 24);
            q[3] = (uint8_t)(o >> 16);
            q[4] = (uint8_t)(o >> 8);
            q[5] = (uint8_t)o;
        } else {
            q[0] = (uint8_t)tag;
            q[1] = (uint8_t)(o >> 8);
            q[2] = (uint8_t)o;
        }
    }
    int m = (int)size;
    m += encode_size(b, (uint32_t)data_size);
    m += encode_size_type(b, (uint32_t)size, type);
    *n = m;
    return NULL;
}
