/*
 * format.c — restatement of internal/format (type codes, message/list tables) and the
 * baselibrary buffer.Buffer append semantics.  TEST INFRASTRUCTURE (oracle).
 */
#include <stdlib.h>
#include <string.h>

#include "spec_oracle.h"

/* Type.Check, internal/format/type.go:54-90 */
int so_type_check(uint8_t t) {
    switch (t) {
    case SO_TYPE_TRUE: case SO_TYPE_FALSE: case SO_TYPE_BYTE:
    case SO_TYPE_INT16: case SO_TYPE_INT32: case SO_TYPE_INT64:
    case SO_TYPE_UINT16: case SO_TYPE_UINT32: case SO_TYPE_UINT64:
    case SO_TYPE_FLOAT32: case SO_TYPE_FLOAT64:
    case SO_TYPE_BIN64: case SO_TYPE_BIN128: case SO_TYPE_BIN256:
    case SO_TYPE_BYTES: case SO_TYPE_STRING:
    case SO_TYPE_LIST: case SO_TYPE_BIG_LIST:
    case SO_TYPE_MESSAGE: case SO_TYPE_BIG_MESSAGE:
    case SO_TYPE_STRUCT:
        return 0;
    }
    return -1;
}

/* ---- buffer.Buffer ---- */

so_buf *so_buf_new(size_t cap) {
    so_buf *b = (so_buf *)calloc(1, sizeof(so_buf));
    if (cap == 0) cap = 64;
    b->data = (uint8_t *)malloc(cap);
    b->cap = cap;
    b->owned = 1;
    return b;
}

void so_buf_init_fixed(so_buf *b, uint8_t *mem, size_t cap) {
    b->data = mem;
    b->len = 0;
    b->cap = cap;
    b->owned = 0;
    b->overflow = 0;
}

void so_buf_free(so_buf *b) {
    if (!b) return;
    if (b->owned) free(b->data);
    free(b);
}

void so_buf_reset(so_buf *b) {
    b->len = 0;
    b->overflow = 0;
}

/* Grow(n) returns the next n bytes at the end (a fixed buffer that overflows keeps
 * writing into a scratch area and records the overflow; callers check it). */
static uint8_t so_scratch_sink[1 << 16];

uint8_t *so_buf_grow(so_buf *b, size_t n) {
    if (b->len + n > b->cap) {
        if (!b->owned) {
            b->overflow = 1;
            if (n > sizeof(so_scratch_sink)) abort();
            b->len += n;
            return so_scratch_sink;
        }
        size_t c = b->cap * 2;
        while (c < b->len + n) c *= 2;
        b->data = (uint8_t *)realloc(b->data, c);
        b->cap = c;
    }
    uint8_t *p = b->data + b->len;
    b->len += n;
    return p;
}

size_t so_buf_len(const so_buf *b) { return b->len; }
uint8_t *so_buf_bytes(const so_buf *b) { return b->data; }

/* ---- message table, internal/format/msg.go ---- */

#define FIELD_SMALL 3 /* MessageFieldSize_Small, msg.go:14 */
#define FIELD_BIG 6   /* MessageFieldSize_Big,   msg.go:15 */
#define ELEM_SMALL 2  /* ListElementSize_Small, list.go:13 */
#define ELEM_BIG 4    /* ListElementSize_Big,   list.go:14 */

static inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* IsBigMessage, msg.go:43-61: any tag > 255 or any offset > 65535 */
int so_is_big_message(const so_message_field *f, size_t n) {
    for (size_t i = n; i-- > 0;) {
        if (f[i].tag > 255) return 1;
        if (f[i].offset > 65535) return 1;
    }
    return 0;
}

/* IsBigList, list.go:40-54: count > 255, or the LAST offset > 65535 */
int so_is_big_list(const so_list_element *e, size_t n) {
    if (n == 0) return 0;
    if (n > 255) return 1;
    return e[n - 1].offset > 65535;
}

int so_message_table_len(const so_message_table *t) {
    return (int)(t->table_len / (t->big ? FIELD_BIG : FIELD_SMALL));
}

/* offset_big / offset_small, msg.go:138-186 and 227-265: binary search by tag over the
 * sorted table; returns the field END offset or -1.  The exact midpoint sequence is kept
 * because tables may hold duplicate tags (the writer never deduplicates). */
int64_t so_message_table_offset(const so_message_table *t, uint16_t tag) {
    int size = t->big ? FIELD_BIG : FIELD_SMALL;
    if ((int)t->table_len < size) return -1;
    int n = (int)(t->table_len / (size_t)size);
    int left = 0, right = n - 1;
    while (left <= right) {
        int middle = (int)((unsigned)(left + right) >> 1);
        const uint8_t *p = t->table + (size_t)middle * (size_t)size;
        uint16_t cur = t->big ? be16(p) : p[0];
        if (cur < tag) {
            left = middle + 1;
        } else if (cur > tag) {
            right = middle - 1;
        } else {
            return t->big ? (int64_t)be32(p + 2) : (int64_t)be16(p + 1);
        }
    }
    return -1;
}

/* offsetByIndex_big/_small, msg.go:303-339 */
int64_t so_message_table_offset_by_index(const so_message_table *t, int i) {
    int size = t->big ? FIELD_BIG : FIELD_SMALL;
    int n = (int)(t->table_len / (size_t)size);
    if (i < 0 || i >= n) return -1;
    const uint8_t *p = t->table + (size_t)i * (size_t)size;
    return t->big ? (int64_t)be32(p + 2) : (int64_t)be16(p + 1);
}

/* field_big/_small, msg.go:343-390 */
int so_message_table_field(const so_message_table *t, int i, so_message_field *f) {
    int size = t->big ? FIELD_BIG : FIELD_SMALL;
    int n = (int)(t->table_len / (size_t)size);
    if (i < 0 || i >= n) return 0;
    const uint8_t *p = t->table + (size_t)i * (size_t)size;
    if (t->big) {
        f->tag = be16(p);
        f->offset = be32(p + 2);
    } else {
        f->tag = p[0];
        f->offset = be16(p + 1);
    }
    return 1;
}

/* ---- list table, internal/format/list.go ---- */

int so_list_table_len(const so_list_table *t) {
    return (int)(t->table_len / (t->big ? ELEM_BIG : ELEM_SMALL));
}

/* offset_big/offset_small, list.go:130-176: element i = [end(i-1), end(i)) */
void so_list_table_offset(const so_list_table *t, int i, int64_t *start, int64_t *end) {
    int size = t->big ? ELEM_BIG : ELEM_SMALL;
    int n = (int)(t->table_len / (size_t)size);
    if (i < 0 || i >= n) {
        *start = -1;
        *end = -1;
        return;
    }
    const uint8_t *p = t->table + (size_t)i * (size_t)size;
    int64_t s = 0;
    if (i > 0) s = t->big ? (int64_t)be32(p - 4) : (int64_t)be16(p - 2);
    *start = s;
    *end = t->big ? (int64_t)be32(p) : (int64_t)be16(p);
}
