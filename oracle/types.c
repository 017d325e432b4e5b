/*
 * types.c — restatement of internal/types (Message, List, Value readers).
 * TEST INFRASTRUCTURE (oracle).
 */
#include <string.h>

#include "spec_oracle.h"

/* OpenMessageErr, internal/types/msg.go:43-55: bytes = b[len(b)-size:] */
so_err so_open_message_err(const uint8_t *b, size_t len, so_message *m) {
    memset(m, 0, sizeof(*m));
    int size;
    so_err e = so_decode_message_table(b, len, &m->table, &size);
    if (e) {
        memset(m, 0, sizeof(*m));
        return e;
    }
    m->bytes = b + (len - (size_t)size);
    m->len = (size_t)size;
    return NULL;
}

/* OpenMessage, msg.go:28-40: empty message on error */
void so_open_message(const uint8_t *b, size_t len, so_message *m) {
    if (so_open_message_err(b, len, m)) memset(m, 0, sizeof(*m));
}

int so_message_fields(const so_message *m) { return so_message_table_len(&m->table); }

/* HasField, msg.go:101-106 */
int so_message_has_field(const so_message *m, uint16_t tag) {
    int64_t end = so_message_table_offset(&m->table, tag);
    return end >= 0 && end <= (int64_t)m->table.data;
}

/* field(tag), msg.go:466-475: bytes[:end] when 0 <= end <= dataSize, else nil */
const uint8_t *so_message_field_raw(const so_message *m, uint16_t tag, size_t *len) {
    int64_t end = so_message_table_offset(&m->table, tag);
    if (end < 0 || end > (int64_t)m->table.data) {
        *len = 0;
        return NULL;
    }
    *len = (size_t)end;
    return m->bytes;
}

/* fieldAt(i), msg.go:477-486 */
const uint8_t *so_message_field_at_raw(const so_message *m, int i, size_t *len) {
    int64_t end = so_message_table_offset_by_index(&m->table, i);
    if (end < 0 || end > (int64_t)m->table.data) {
        *len = 0;
        return NULL;
    }
    *len = (size_t)end;
    return m->bytes;
}

/* Typed getters, msg.go:219-421: decode errors are swallowed, zero value returned. */
#define FIELD(m, tag)        \
    size_t flen;             \
    const uint8_t *f = so_message_field_raw(m, tag, &flen); \
    int n

int so_message_bool(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    int v;
    so_decode_bool(f, flen, &v, &n);
    return v;
}

uint8_t so_message_byte(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    uint8_t v;
    if (so_decode_byte(f, flen, &v, &n)) return 0;
    return v;
}

int16_t so_message_int16(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    int16_t v;
    if (so_decode_int16(f, flen, &v, &n)) return 0;
    return v;
}

int32_t so_message_int32(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    int32_t v;
    if (so_decode_int32(f, flen, &v, &n)) return 0;
    return v;
}

int64_t so_message_int64(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    int64_t v;
    if (so_decode_int64(f, flen, &v, &n)) return 0;
    return v;
}

uint16_t so_message_uint16(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    uint16_t v;
    if (so_decode_uint16(f, flen, &v, &n)) return 0;
    return v;
}

uint32_t so_message_uint32(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    uint32_t v;
    if (so_decode_uint32(f, flen, &v, &n)) return 0;
    return v;
}

uint64_t so_message_uint64(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    uint64_t v;
    if (so_decode_uint64(f, flen, &v, &n)) return 0;
    return v;
}

float so_message_float32(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    float v;
    if (so_decode_float32(f, flen, &v, &n)) return 0;
    return v;
}

double so_message_float64(const so_message *m, uint16_t tag) {
    FIELD(m, tag);
    double v;
    if (so_decode_float64(f, flen, &v, &n)) return 0;
    return v;
}

void so_message_bin64(const so_message *m, uint16_t tag, uint8_t v[8]) {
    FIELD(m, tag);
    if (so_decode_bin64(f, flen, v, &n)) memset(v, 0, 8);
}

void so_message_bin128(const so_message *m, uint16_t tag, uint8_t v[16]) {
    FIELD(m, tag);
    if (so_decode_bin128(f, flen, v, &n)) memset(v, 0, 16);
}

void so_message_bin256(const so_message *m, uint16_t tag, uint8_t v[32]) {
    FIELD(m, tag);
    if (so_decode_bin256(f, flen, v, &n)) memset(v, 0, 32);
}

const uint8_t *so_message_bytes(const so_message *m, uint16_t tag, size_t *len) {
    FIELD(m, tag);
    size_t off, vlen;
    *len = 0;
    if (!f || so_decode_bytes(f, flen, &off, &vlen, &n)) return NULL;
    *len = vlen;
    return f + off;
}

const uint8_t *so_message_string(const so_message *m, uint16_t tag, size_t *len) {
    FIELD(m, tag);
    size_t off, vlen;
    *len = 0;
    if (!f || so_decode_string(f, flen, &off, &vlen, &n)) return NULL;
    *len = vlen;
    return f + off;
}

/* List(tag) / Message(tag), msg.go:441-454 */
void so_message_list(const so_message *m, uint16_t tag, so_list *l) {
    size_t flen;
    const uint8_t *f = so_message_field_raw(m, tag, &flen);
    if (so_open_list_err(f, flen, l)) memset(l, 0, sizeof(*l));
}

void so_message_message(const so_message *m, uint16_t tag, so_message *sub) {
    size_t flen;
    const uint8_t *f = so_message_field_raw(m, tag, &flen);
    so_open_message(f, flen, sub);
}

/* ---- List, internal/types/list.go ---- */

/* decodeList, list.go:55-67 */
so_err so_open_list_err(const uint8_t *b, size_t len, so_list *l) {
    memset(l, 0, sizeof(*l));
    int size;
    so_err e = so_decode_list_table(b, len, &l->table, &size);
    if (e) {
        memset(l, 0, sizeof(*l));
        return e;
    }
    l->bytes = b + (len - (size_t)size);
    l->len = (size_t)size;
    return NULL;
}

int so_list_len(const so_list *l) { return so_list_table_len(&l->table); }

/* GetBytes, list.go:101-113: -1 where Go panics (index out of range, or a slice with
 * start > end from a malformed table); nil when end > dataSize. */
int so_list_get_bytes(const so_list *l, int i, const uint8_t **p, size_t *len) {
    int64_t start, end;
    so_list_table_offset(&l->table, i, &start, &end);
    *p = NULL;
    *len = 0;
    if (start < 0) return -1;
    if (end > (int64_t)l->table.data) return 0;
    if (start > end) return -1;
    *p = l->bytes + start;
    *len = (size_t)(end - start);
    return 0;
}

/* ---- ParseMessage / ParseList / ParseValue (recursive validation) ---- */

/* ParseList, internal/types/list.go:35-53 */
so_err so_parse_list(const uint8_t *b, size_t len, int *size) {
    so_list l;
    so_err e = so_open_list_err(b, len, &l);
    *size = 0;
    if (e) return e;
    int n = so_list_len(&l);
    for (int i = 0; i < n; i++) {
        const uint8_t *p;
        size_t plen;
        if (so_list_get_bytes(&l, i, &p, &plen) < 0) return "list: index out of range";
        if (plen == 0) continue;
        int vn;
        if ((e = so_parse_value(p, plen, &vn))) return e;
    }
    *size = (int)l.len;
    return NULL;
}

/* ParseMessage, internal/types/msg.go:58-82 */
so_err so_parse_message(const uint8_t *b, size_t len, so_message *m, int *size) {
    *size = 0;
    so_err e = so_open_message_err(b, len, m);
    if (e) return e;
    int num = so_message_fields(m);
    for (int i = 0; i < num; i++) {
        size_t flen;
        const uint8_t *f = so_message_field_at_raw(m, i, &flen);
        if (flen == 0) continue;
        int vn;
        if ((e = so_parse_value(f, flen, &vn))) return e;
    }
    *size = (int)m->len;
    return NULL;
}

/* ParseValue, internal/types/value.go:49-113 */
so_err so_parse_value(const uint8_t *b, size_t len, int *n) {
    uint8_t t;
    so_err e = so_decode_type(b, len, &t, n);
    if (e) return e;
    union {
        int i;
        uint8_t u8;
        int16_t i16;
        int32_t i32;
        int64_t i64;
        uint16_t u16;
        uint32_t u32;
        uint64_t u64;
        float f32;
        double f64;
        uint8_t bin[32];
    } v;
    size_t off, vlen;
    so_message m;
    switch (t) {
    case SO_TYPE_TRUE:
    case SO_TYPE_FALSE:
        break;
    case SO_TYPE_BYTE: e = so_decode_byte(b, len, &v.u8, n); break;
    case SO_TYPE_INT16: e = so_decode_int16(b, len, &v.i16, n); break;
    case SO_TYPE_INT32: e = so_decode_int32(b, len, &v.i32, n); break;
    case SO_TYPE_INT64: e = so_decode_int64(b, len, &v.i64, n); break;
    case SO_TYPE_UINT16: e = so_decode_uint16(b, len, &v.u16, n); break;
    case SO_TYPE_UINT32: e = so_decode_uint32(b, len, &v.u32, n); break;
    case SO_TYPE_UINT64: e = so_decode_uint64(b, len, &v.u64, n); break;
    case SO_TYPE_BIN64: e = so_decode_bin64(b, len, v.bin, n); break;
    case SO_TYPE_BIN128: e = so_decode_bin128(b, len, v.bin, n); break;
    case SO_TYPE_BIN256: e = so_decode_bin256(b, len, v.bin, n); break;
    case SO_TYPE_FLOAT32: e = so_decode_float32(b, len, &v.f32, n); break;
    case SO_TYPE_FLOAT64: e = so_decode_float64(b, len, &v.f64, n); break;
    case SO_TYPE_BYTES: e = so_decode_bytes(b, len, &off, &vlen, n); break;
    case SO_TYPE_STRING: e = so_decode_string(b, len, &off, &vlen, n); break;
    case SO_TYPE_LIST:
    case SO_TYPE_BIG_LIST: e = so_parse_list(b, len, n); break;
    case SO_TYPE_MESSAGE:
    case SO_TYPE_BIG_MESSAGE: e = so_parse_message(b, len, &m, n); break;
    case SO_TYPE_STRUCT: e = so_decode_struct(b, len, &v.i, n); break;
    default:
        *n = 0;
        return "unsupported type";
    }
    /* value.go:110: return b[len(b)-n:] — a size past the slice (DecodeStruct does not bound its
     * data size) panics: slice bounds out of range */
    if (!e && (size_t)*n > len) return "parse value: slice bounds out of range (index out of range)";
    return e;
}
