/*
 * decode.c — restatement of internal/decode/....  Every decoder parses the value that
 * ENDS at b+len and reports n = bytes consumed from the end.  Empty input => zero value,
 * n = 0, no error.  Arithmetic on sizes is done in int64 like Go's int.
 * TEST INFRASTRUCTURE (oracle).
 */
#include <math.h>
#include <string.h>

#include "spec_oracle.h"

/* decodeType / decodeSize, internal/decode/type.go:206-217 */
static inline int decode_type(const uint8_t *b, size_t len, uint8_t *t) {
    if (len == 0) {
        *t = SO_TYPE_UNDEFINED;
        return 0;
    }
    *t = b[len - 1];
    return 1;
}

static inline uint32_t decode_size(const uint8_t *b, size_t len, int *n) {
    return so_reverse_uint32(b, len, n);
}

/* DecodeType, type.go:16-25 */
so_err so_decode_type(const uint8_t *b, size_t len, uint8_t *t, int *n) {
    *n = decode_type(b, len, t);
    return NULL;
}

/* DecodeTypeSize, type.go:27-203 */
so_err so_decode_type_size(const uint8_t *b, size_t len, uint8_t *tp, int *np) {
    *tp = 0;
    *np = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int n = decode_type(b, len, &t);
    int64_t end = (int64_t)len - n;
    int64_t size;
    int m;
    uint32_t ds, ts;
    switch (t) {
    case SO_TYPE_TRUE:
    case SO_TYPE_FALSE:
        size = n;
        break;
    case SO_TYPE_BYTE:
        if (end < 1) return "decode byte: invalid data";
        size = n + 1;
        break;
    case SO_TYPE_INT16: case SO_TYPE_INT32: case SO_TYPE_INT64:
        m = so_reverse_size(b, (size_t)end);
        if (m <= 0) return "decode int: invalid data";
        size = n + m;
        break;
    case SO_TYPE_UINT16: case SO_TYPE_UINT32: case SO_TYPE_UINT64:
        m = so_reverse_size(b, (size_t)end);
        if (m <= 0) return "decode uint: invalid data";
        size = n + m;
        break;
    case SO_TYPE_FLOAT32:
        if (end < 4) return "decode float32: invalid data";
        size = n + 4;
        break;
    case SO_TYPE_FLOAT64:
        if (end < 8) return "decode float64: invalid data";
        size = n + 8;
        break;
    case SO_TYPE_BIN64:
        if (end < 8) return "decode bin64: invalid data";
        size = n + 8;
        break;
    case SO_TYPE_BIN128:
        if (end < 16) return "decode bin128: invalid data";
        size = n + 16;
        break;
    case SO_TYPE_BIN256:
        if (end < 32) return "decode bin256: invalid data";
        size = n + 32;
        break;
    case SO_TYPE_BYTES:
        ds = decode_size(b, (size_t)end, &m);
        if (m < 0) return "decode bytes: invalid data size";
        size = (int64_t)n + m + ds;
        if ((int64_t)len < size) return "decode bytes: invalid data";
        break;
    case SO_TYPE_STRING:
        ds = decode_size(b, (size_t)end, &m);
        if (m < 0) return "decode string: invalid data size";
        size = (int64_t)n + m + ds + 1;
        if ((int64_t)len < size) return "decode string: invalid data";
        break;
    case SO_TYPE_LIST:
    case SO_TYPE_BIG_LIST:
        size = n;
        ts = decode_size(b, (size_t)end, &m);
        if (m < 0) return "decode list: invalid table size";
        end -= m;
        size += m + (int64_t)ts;
        ds = decode_size(b, (size_t)end, &m);
        if (m < 0) return "decode list: invalid data size";
        end -= m;
        size += m + (int64_t)ds;
        if ((int64_t)len < size) return "decode list: invalid data";
        break;
    case SO_TYPE_MESSAGE:
    case SO_TYPE_BIG_MESSAGE:
        size = n;
        ts = decode_size(b, (size_t)end, &m);
        if (m < 0) return "decode message: invalid table size";
        end -= m;
        size += m + (int64_t)ts;
        ds = decode_size(b, (size_t)end, &m);
        if (m < 0) return "decode message: invalid data size";
        end -= m;
        size += m + (int64_t)ds;
        if ((int64_t)len < size) return "decode message: invalid data";
        break;
    case SO_TYPE_STRUCT:
        size = n;
        ds = decode_size(b, (size_t)end, &m);
        /* type.go:185-191 checks n (the type size) instead of m: preserved. */
        if (n < 0) return "decode struct: invalid data size";
        size += m + (int64_t)ds;
        if ((int64_t)len < size) return "decode struct: invalid data";
        break;
    default:
        return "decode: invalid type";
    }
    *tp = t;
    *np = (int)size;
    return NULL;
}

/* DecodeByte / DecodeBool, internal/decode/byte.go:16-51 */
so_err so_decode_byte(const uint8_t *b, size_t len, uint8_t *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    decode_type(b, len, &t);
    if (t != SO_TYPE_BYTE) return "decode byte: invalid type";
    if (len < 2) return "decode byte: invalid data";
    *v = b[len - 2];
    *n = 2;
    return NULL;
}

so_err so_decode_bool(const uint8_t *b, size_t len, int *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    *n = decode_type(b, len, &t);
    *v = (t == SO_TYPE_TRUE); /* any other type => false, no error */
    return NULL;
}

/* DecodeInt16/32/64, internal/decode/int.go:16-135 */
so_err so_decode_int16(const uint8_t *b, size_t len, int16_t *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    size_t end = len - (size_t)k;
    int m;
    int64_t x;
    if (t == SO_TYPE_INT16 || t == SO_TYPE_INT32) {
        x = so_reverse_int32(b, end, &m);
    } else if (t == SO_TYPE_INT64) {
        x = so_reverse_int64(b, end, &m);
    } else {
        return "decode int16: invalid type";
    }
    if (m < 0) return "decode int16: invalid data";
    if (x < -32768) return "decode int16: overflow, value too small";
    if (x > 32767) return "decode int16: overflow, value too large";
    *v = (int16_t)x;
    *n = k + m;
    return NULL;
}

so_err so_decode_int32(const uint8_t *b, size_t len, int32_t *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    size_t end = len - (size_t)k;
    int m;
    if (t == SO_TYPE_INT16 || t == SO_TYPE_INT32) {
        int32_t x = so_reverse_int32(b, end, &m);
        if (m < 0) return "decode int32: invalid data";
        *v = x;
        *n = k + m;
        return NULL;
    }
    if (t == SO_TYPE_INT64) {
        int64_t x = so_reverse_int64(b, end, &m);
        if (m < 0) return "decode int32: invalid data";
        if (x < INT32_MIN) return "decode int32: overflow, value too small";
        if (x > INT32_MAX) return "decode int32: overflow, value too large";
        *v = (int32_t)x;
        *n = k + m;
        return NULL;
    }
    return "decode int32: invalid type";
}

so_err so_decode_int64(const uint8_t *b, size_t len, int64_t *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    size_t end = len - (size_t)k;
    int m;
    int64_t x;
    if (t == SO_TYPE_INT16 || t == SO_TYPE_INT32) {
        x = so_reverse_int32(b, end, &m);
    } else if (t == SO_TYPE_INT64) {
        x = so_reverse_int64(b, end, &m);
    } else {
        return "decode int64: invalid type";
    }
    if (m < 0) return "decode int64: invalid data";
    *v = x;
    *n = k + m;
    return NULL;
}

/* DecodeUint16/32/64, internal/decode/uint.go:16-125 */
so_err so_decode_uint16(const uint8_t *b, size_t len, uint16_t *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    size_t end = len - (size_t)k;
    int m;
    uint64_t x;
    if (t == SO_TYPE_UINT16 || t == SO_TYPE_UINT32) {
        x = so_reverse_uint32(b, end, &m);
    } else if (t == SO_TYPE_UINT64) {
        x = so_reverse_uint64(b, end, &m);
    } else {
        return "decode uint32: invalid type"; /* sic, uint.go:52 */
    }
    if (m < 0) return "decode uint16: invalid data";
    if (x > 65535) return "decode int16: overflow, value too large";
    *v = (uint16_t)x;
    *n = k + m;
    return NULL;
}

so_err so_decode_uint32(const uint8_t *b, size_t len, uint32_t *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    size_t end = len - (size_t)k;
    int m;
    uint64_t x;
    if (t == SO_TYPE_UINT16 || t == SO_TYPE_UINT32) {
        x = so_reverse_uint32(b, end, &m);
    } else if (t == SO_TYPE_UINT64) {
        x = so_reverse_uint64(b, end, &m);
        if (m >= 0 && x > UINT32_MAX) return "decode int32: overflow, value too large";
    } else {
        return "decode uint32: invalid type";
    }
    if (m < 0) return "decode uint32: invalid data";
    *v = (uint32_t)x;
    *n = k + m;
    return NULL;
}

so_err so_decode_uint64(const uint8_t *b, size_t len, uint64_t *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    size_t end = len - (size_t)k;
    int m;
    uint64_t x;
    if (t == SO_TYPE_UINT16 || t == SO_TYPE_UINT32) {
        x = so_reverse_uint32(b, end, &m);
    } else if (t == SO_TYPE_UINT64) {
        x = so_reverse_uint64(b, end, &m);
    } else {
        return "decode uint64: invalid type";
    }
    if (m < 0) return "decode uint64: invalid data";
    *v = x;
    *n = k + m;
    return NULL;
}

/* decodeFloat64, internal/decode/float.go:51-78: either width read as float64 */
static double decode_float64(const uint8_t *b, size_t len, int *n) {
    uint8_t t;
    decode_type(b, len, &t);
    if (t == SO_TYPE_FLOAT32) {
        if (len < 5) {
            *n = -1;
            return 0;
        }
        const uint8_t *p = b + len - 5;
        uint32_t u = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
        float f;
        memcpy(&f, &u, 4);
        *n = 5;
        return (double)f; /* float64(f): IEEE widening (quiets a signalling NaN) */
    }
    if (t == SO_TYPE_FLOAT64) {
        if (len < 9) {
            *n = -1;
            return 0;
        }
        const uint8_t *p = b + len - 9;
        uint64_t u = 0;
        for (int i = 0; i < 8; i++) u = (u << 8) | p[i];
        double d;
        memcpy(&d, &u, 8);
        *n = 9;
        return d;
    }
    *n = -1;
    return 0;
}

/* DecodeFloat32, float.go:15-32: via float64 with a +-MaxFloat32 range check (so a
 * float32 +-Inf decodes to an error => 0 through the getter; NaN passes) */
so_err so_decode_float32(const uint8_t *b, size_t len, float *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    int k;
    double d = decode_float64(b, len, &k);
    if (k < 0) return "decode float32: invalid data";
    if (d < -3.40282346638528859811704183484516925440e+38) return "decode float32: overflow, value too small";
    if (d > 3.40282346638528859811704183484516925440e+38) return "decode float32: overflow, value too large";
    *v = (float)d;
    *n = k;
    return NULL;
}

so_err so_decode_float64(const uint8_t *b, size_t len, double *v, int *n) {
    *v = 0;
    *n = 0;
    if (len == 0) return NULL;
    int k;
    double d = decode_float64(b, len, &k);
    if (k < 0) {
        *n = k;
        return "decode float64: invalid data";
    }
    *v = d;
    *n = k;
    return NULL;
}

/* DecodeBin64/128/256, internal/decode/bin.go:15-112 */
static so_err decode_bin(const uint8_t *b, size_t len, uint8_t *v, int w, uint8_t type, int *n,
                         const char *etype, const char *edata) {
    memset(v, 0, (size_t)w);
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    decode_type(b, len, &t);
    if (t != type) return etype;
    if ((int64_t)len - (1 + w) < 0) return edata;
    memcpy(v, b + len - 1 - w, (size_t)w);
    *n = 1 + w;
    return NULL;
}

so_err so_decode_bin64(const uint8_t *b, size_t len, uint8_t v[8], int *n) {
    return decode_bin(b, len, v, 8, SO_TYPE_BIN64, n, "decode bin64: invalid type", "decode bin64: invalid data");
}
so_err so_decode_bin128(const uint8_t *b, size_t len, uint8_t v[16], int *n) {
    return decode_bin(b, len, v, 16, SO_TYPE_BIN128, n, "decode bin128: invalid type", "decode bin128: invalid data");
}
so_err so_decode_bin256(const uint8_t *b, size_t len, uint8_t v[32], int *n) {
    return decode_bin(b, len, v, 32, SO_TYPE_BIN256, n, "decode bin256: invalid type", "decode bin256: invalid data");
}

/* DecodeBytes, internal/decode/bytes.go:14-58 */
so_err so_decode_bytes(const uint8_t *b, size_t len, size_t *off, size_t *vlen, int *n) {
    *off = 0;
    *vlen = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    if (t != SO_TYPE_BYTES) return "decode bytes: invalid type";
    int64_t size = k;
    int64_t end = (int64_t)len - size;
    int m;
    uint32_t ds = decode_size(b, (size_t)end, &m);
    if (m < 0) return "decode bytes: invalid data size";
    size += m;
    end -= m;
    int64_t o = end - (int64_t)ds;
    if (o < 0) return "decode bytes: invalid data size";
    size += ds;
    *off = (size_t)o;
    *vlen = ds;
    *n = (int)size;
    return NULL;
}

/* DecodeString, internal/decode/string.go:15-70 (the NUL byte is skipped, not checked) */
so_err so_decode_string(const uint8_t *b, size_t len, size_t *off, size_t *vlen, int *n) {
    *off = 0;
    *vlen = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    if (t != SO_TYPE_STRING) return "decode string: invalid type";
    int64_t size = k;
    int64_t end = (int64_t)len - size;
    int m;
    uint32_t ds = decode_size(b, (size_t)end, &m);
    if (m < 0) return "decode string: invalid data size";
    size += m + 1;
    end -= (m + 1);
    /* decodeStringData(b[:end], size): Go would panic on a negative end (slice bound);
     * a negative end can only come from a 1-byte varint with no room for the NUL, and
     * then off = end - ds < 0 as well: reported as invalid data size. */
    int64_t o = end - (int64_t)ds;
    if (end < 0 || o < 0) return "decode string: invalid data size";
    size += ds;
    *off = (size_t)o;
    *vlen = ds;
    *n = (int)size;
    return NULL;
}

/* DecodeStruct, internal/decode/struct.go:14-42 */
so_err so_decode_struct(const uint8_t *b, size_t len, int *data_size, int *n) {
    *data_size = 0;
    *n = 0;
    if (len == 0) return NULL;
    uint8_t t;
    int k = decode_type(b, len, &t);
    if (t != SO_TYPE_STRUCT) return "decode struct: invalid type";
    int m;
    uint32_t ds = decode_size(b, len - (size_t)k, &m);
    if (m < 0) return "decode struct: invalid data size";
    *data_size = (int)ds;
    *n = (int)(k + m + (int64_t)ds);
    return NULL;
}

/* DecodeListTable, internal/decode/list.go:14-98 */
so_err so_decode_list_table(const uint8_t *b, size_t len, so_list_table *t, int *np) {
    memset(t, 0, sizeof(*t));
    *np = 0;
    if (len == 0) return NULL;
    uint8_t typ;
    int k = decode_type(b, len, &typ);
    if (typ != SO_TYPE_LIST && typ != SO_TYPE_BIG_LIST) return "decode list: invalid type";
    int64_t size = k;
    int64_t end = (int64_t)len - k;
    int big = typ == SO_TYPE_BIG_LIST;
    int m;
    uint32_t ts = decode_size(b, (size_t)end, &m);
    if (m < 0) return "decode list: invalid table size";
    end -= m;
    size += m;
    uint32_t ds = decode_size(b, (size_t)end, &m);
    if (m < 0) return "decode list: invalid data size";
    end -= m;
    size += m;
    /* decodeListTable, list.go:76-98 */
    int64_t start = end - (int64_t)ts;
    if (start < 0) return "decode list: invalid table";
    if (ts % (uint32_t)(big ? 4 : 2) != 0) return "decode list: invalid table";
    const uint8_t *table = b + start;
    end -= (int64_t)ts + (int64_t)ds;
    size += ts;
    if (end < 0) return "decode list: invalid data";
    size += ds;
    t->table = table;
    t->table_len = ts;
    t->data = ds;
    t->big = big;
    *np = (int)size;
    return NULL;
}

/* DecodeMessageTable, internal/decode/msg.go:14-99 */
so_err so_decode_message_table(const uint8_t *b, size_t len, so_message_table *t, int *np) {
    memset(t, 0, sizeof(*t));
    *np = 0;
    if (len == 0) return NULL;
    uint8_t typ;
    int k = decode_type(b, len, &typ);
    if (typ != SO_TYPE_MESSAGE && typ != SO_TYPE_BIG_MESSAGE) return "decode message: invalid type";
    int64_t size = k;
    int64_t end = (int64_t)len - k;
    int big = typ == SO_TYPE_BIG_MESSAGE;
    int m;
    uint32_t ts = decode_size(b, (size_t)end, &m);
    if (m < 0) return "decode message: invalid table size";
    end -= m;
    size += m;
    uint32_t ds = decode_size(b, (size_t)end, &m);
    if (m < 0) return "decode message: invalid data size";
    end -= m;
    size += m;
    /* decodeMessageTable, msg.go:77-99 */
    int64_t start = end - (int64_t)ts;
    if (start < 0) return "decode message: invalid table";
    if (ts % (uint32_t)(big ? 6 : 3) != 0) return "decode message: invalid table";
    const uint8_t *table = b + start;
    end -= (int64_t)ts + (int64_t)ds;
    size += ts;
    if (end < 0) return "decode message: invalid data";
    size += ds;
    t->table = table;
    t->table_len = ts;
    t->data = ds;
    t->big = big;
    *np = (int)size;
    return NULL;
}
