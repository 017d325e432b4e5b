/*
 * writer.c — restatement of the internal/writer stack machine (writer.go, stack.go,
 * stack_list.go, stack_msg.go, value.go, msg.go, list.go).
 * TEST INFRASTRUCTURE (oracle).
 */
#include <stdlib.h>
#include <string.h>

#include "spec_oracle.h"

/* entryType, internal/writer/stack.go:7-16 */
enum { E_UNDEFINED = 0, E_DATA, E_LIST, E_ELEMENT, E_MESSAGE, E_FIELD };

typedef struct entry {
    int64_t start;
    int64_t table_start; /* data: end; list/message: side-stack offset; field: tag */
    int type;
} entry;

struct so_message_stack {
    so_message_field *v;
    int len, cap;
};

typedef struct list_stack {
    so_list_element *v;
    int len, cap;
} list_stack;

struct so_writer {
    so_buf *buf;
    entry *stack;
    int slen, scap;
    list_stack elements;
    struct so_message_stack fields;
    so_err err;
};

static const char *err_closed = "operation on closed writer"; /* writer.go:62 */

/* ---- messageStack, stack_msg.go:23-81 ---- */

static void ms_push(struct so_message_stack *s, so_message_field f) {
    if (s->len == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 48;
        s->v = (so_message_field *)realloc(s->v, (size_t)s->cap * sizeof(*s->v));
    }
    s->v[s->len++] = f;
}

/* insert: append then insertion-sort backwards; a tie (left.Tag == right.Tag) also
 * swaps, so a field written later with an equal tag lands BEFORE the earlier one. */
static void ms_insert(struct so_message_stack *s, int table_offset, so_message_field f) {
    ms_push(s, f);
    so_message_field *t = s->v + table_offset;
    int n = s->len - table_offset;
    for (int i = n - 1; i > 0; i--) {
        so_message_field left = t[i - 1], right = t[i];
        if (left.tag < right.tag) break;
        t[i - 1] = right;
        t[i] = left;
    }
}

/* hasField: sort.Search for the first tag >= tag, then equality */
static int ms_has_field(struct so_message_stack *s, int table_offset, uint16_t tag) {
    so_message_field *t = s->v + table_offset;
    int n = s->len - table_offset;
    int lo = 0, hi = n;
    while (lo < hi) {
        int h = (int)((unsigned)(lo + hi) >> 1);
        if (!(t[h].tag >= tag)) lo = h + 1;
        else hi = h;
    }
    if (lo >= n) return 0;
    return t[lo].tag == tag;
}

so_message_stack *so_message_stack_new(void) { return (so_message_stack *)calloc(1, sizeof(so_message_stack)); }
void so_message_stack_free(so_message_stack *s) {
    if (!s) return;
    free(s->v);
    free(s);
}
void so_message_stack_insert(so_message_stack *s, int table_offset, uint16_t tag, uint32_t off) {
    so_message_field f = {tag, off};
    ms_insert(s, table_offset, f);
}
int so_message_stack_pop(so_message_stack *s, int table_offset, so_message_field *out, int cap) {
    int n = s->len - table_offset;
    for (int i = 0; i < n && i < cap; i++) out[i] = s->v[table_offset + i];
    s->len = table_offset;
    return n;
}
int so_message_stack_has_field(so_message_stack *s, int table_offset, uint16_t tag) {
    return ms_has_field(s, table_offset, tag);
}

/* ---- listStack, stack_list.go:20-49 ---- */

static void ls_push(list_stack *s, uint32_t off) {
    if (s->len == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 48;
        s->v = (so_list_element *)realloc(s->v, (size_t)s->cap * sizeof(*s->v));
    }
    s->v[s->len++].offset = off;
}

/* ---- stack, stack.go ---- */

static void push(so_writer *w, int type, int64_t start, int64_t ts) {
    if (w->slen == w->scap) {
        w->scap = w->scap ? w->scap * 2 : 14;
        w->stack = (entry *)realloc(w->stack, (size_t)w->scap * sizeof(entry));
    }
    entry e = {start, ts, type};
    w->stack[w->slen++] = e;
}

static int peek(so_writer *w, entry *e) {
    if (w->slen == 0) return 0;
    *e = w->stack[w->slen - 1];
    return 1;
}

static int peek_second_last(so_writer *w, entry *e) {
    if (w->slen < 2) return 0;
    *e = w->stack[w->slen - 2];
    return 1;
}

static int pop(so_writer *w, entry *e) {
    if (w->slen == 0) return 0;
    *e = w->stack[--w->slen];
    return 1;
}

/* ---- writer ---- */

so_writer *so_writer_new(so_buf *buf) {
    so_writer *w = (so_writer *)calloc(1, sizeof(so_writer));
    so_writer_reset(w, buf);
    return w;
}

void so_writer_free(so_writer *w) {
    if (!w) return;
    free(w->stack);
    free(w->elements.v);
    free(w->fields.v);
    free(w);
}

/* Reset, writer.go:95-108 */
void so_writer_reset(so_writer *w, so_buf *buf) {
    w->err = NULL;
    w->buf = buf;
    w->slen = 0;
    w->elements.len = 0;
    w->fields.len = 0;
}

so_err so_writer_err(const so_writer *w) { return w->err; }

/* close / fail, writer.go:585-625 (state release is a no-op here) */
static so_err wclose(so_writer *w) {
    if (w->err) return w->err;
    w->err = err_closed;
    return NULL;
}

static so_err fail(so_writer *w, so_err e) {
    if (w->err) return w->err;
    if (!e) return wclose(w);
    w->err = e;
    return e;
}

/* pushData / popData, writer.go:557-582 */
static so_err push_data(so_writer *w, int64_t start, int64_t end) {
    entry e;
    if (peek(w, &e) && e.type == E_DATA)
        return fail(w, "cannot push more data, element/field must be written first");
    push(w, E_DATA, start, end);
    return NULL;
}

static so_err pop_data(so_writer *w, int64_t *start, int64_t *end) {
    entry e;
    if (!pop(w, &e)) return fail(w, "cannot pop data, no data");
    if (e.type != E_DATA) return fail(w, "cannot pop data, not data");
    *start = e.start;
    *end = e.table_start;
    return NULL;
}

static so_err result(so_writer *w, int64_t start, int64_t end, const uint8_t **out, size_t *out_len) {
    if (out) *out = so_buf_bytes(w->buf) + start;
    if (out_len) *out_len = (size_t)(end - start);
    return NULL;
}

/* endValue, writer.go:191-214 */
static so_err end_value(so_writer *w, const uint8_t **out, size_t *out_len) {
    if (w->err) return w->err;
    if (w->slen > 1) return fail(w, "end value: cannot end value, not root value");
    entry e;
    if (!pop(w, &e)) return fail(w, "end value: no data entry");
    if (e.type != E_DATA) return fail(w, "end value: not data entry");
    return result(w, e.start, (int64_t)so_buf_len(w->buf), out, out_len);
}

/* beginList / beginElement / element / listLen / endElement / endList, writer.go:218-372 */
so_err so_writer_begin_list(so_writer *w) {
    if (w->err) return w->err;
    push(w, E_LIST, (int64_t)so_buf_len(w->buf), w->elements.len);
    return NULL;
}

static so_err begin_element(so_writer *w) {
    if (w->err) return w->err;
    entry l;
    if (!peek(w, &l) || l.type != E_LIST) return fail(w, "begin element: cannot begin element, parent not list");
    push(w, E_ELEMENT, (int64_t)so_buf_len(w->buf), 0);
    return NULL;
}

static so_err element(so_writer *w) {
    if (w->err) return w->err;
    int64_t s, e;
    so_err err = pop_data(w, &s, &e);
    if (err) return err;
    entry l;
    if (!peek(w, &l) || l.type != E_LIST) return fail(w, "element: cannot encode element, parent not list");
    ls_push(&w->elements, (uint32_t)(e - l.start));
    return NULL;
}

int so_writer_list_len(so_writer *w) {
    if (w->err) return 0;
    entry l;
    if (!peek(w, &l) || l.type != E_LIST) return 0;
    /* writer.go:285-287 indexes the element stack by list.start (a BUFFER offset), not
     * list.tableStart; kept as is (Go panics when start > len). */
    if (l.start > w->elements.len) return -1;
    return w->elements.len - (int)l.start;
}

static so_err end_element(so_writer *w, const uint8_t **out, size_t *out_len) {
    if (w->err) return w->err;
    int64_t s, e;
    so_err err = pop_data(w, &s, &e);
    if (err) return err;
    entry el;
    if (!pop(w, &el) || el.type != E_ELEMENT) return fail(w, "end element: not element");
    entry l;
    if (!peek(w, &l) || l.type != E_LIST) return fail(w, "end element: parent not list");
    ls_push(&w->elements, (uint32_t)(e - l.start));
    return result(w, el.start, e, out, out_len);
}

static so_err end_list(so_writer *w, const uint8_t **out, size_t *out_len) {
    if (w->err) return w->err;
    entry l;
    if (!pop(w, &l) || l.type != E_LIST) return fail(w, "end list: not list");
    int64_t body = (int64_t)so_buf_len(w->buf) - l.start;
    int ts = (int)l.table_start;
    int cnt = w->elements.len - ts;
    int n;
    so_err err = so_encode_list_table(w->buf, body, w->elements.v + ts, (size_t)cnt, &n);
    w->elements.len = ts;
    if (err) return fail(w, err);
    int64_t end = (int64_t)so_buf_len(w->buf);
    if ((err = push_data(w, l.start, end))) return err;
    return result(w, l.start, end, out, out_len);
}

/* beginMessage / beginField / field / fieldAny / hasField / endField / endMessage,
 * writer.go:376-553 */
so_err so_writer_begin_message(so_writer *w) {
    if (w->err) return w->err;
    push(w, E_MESSAGE, (int64_t)so_buf_len(w->buf), w->fields.len);
    return NULL;
}

static so_err begin_field(so_writer *w, uint16_t tag) {
    if (w->err) return w->err;
    entry m;
    if (!peek(w, &m) || m.type != E_MESSAGE) return fail(w, "begin field: cannot begin field, parent not message");
    push(w, E_FIELD, (int64_t)so_buf_len(w->buf), tag);
    return NULL;
}

static so_err field(so_writer *w, uint16_t tag) {
    if (w->err) return w->err;
    int64_t s, e;
    so_err err = pop_data(w, &s, &e);
    if (err) return err;
    entry m;
    if (!peek(w, &m) || m.type != E_MESSAGE) return fail(w, "field: cannot encode field, parent not message");
    so_message_field f = {tag, (uint32_t)(e - m.start)};
    ms_insert(&w->fields, (int)m.table_start, f);
    return NULL;
}

int so_writer_has_field(so_writer *w, uint16_t tag) {
    if (w->err) return 0;
    entry m;
    if (!peek(w, &m) || m.type != E_MESSAGE) return 0;
    return ms_has_field(&w->fields, (int)m.table_start, tag);
}

static so_err end_field(so_writer *w, const uint8_t **out, size_t *out_len) {
    if (w->err) return w->err;
    int64_t s, e;
    so_err err = pop_data(w, &s, &e);
    if (err) return err;
    entry fe;
    if (!pop(w, &fe) || fe.type != E_FIELD) return fail(w, "end field: not field");
    entry m;
    if (!peek(w, &m) || m.type != E_MESSAGE) return fail(w, "field: cannot encode field, parent not message");
    so_message_field f = {(uint16_t)fe.table_start, (uint32_t)(e - m.start)};
    ms_insert(&w->fields, (int)m.table_start, f);
    return result(w, fe.start, e, out, out_len);
}

static so_err end_message(so_writer *w, const uint8_t **out, size_t *out_len) {
    if (w->err) return w->err;
    entry m;
    if (!pop(w, &m) || m.type != E_MESSAGE) return fail(w, "end message: parent not message");
    int64_t data_size = (int64_t)so_buf_len(w->buf) - m.start;
    int ts = (int)m.table_start;
    int cnt = w->fields.len - ts;
    int n;
    so_err err = so_encode_message_table(w->buf, data_size, w->fields.v + ts, (size_t)cnt, &n);
    w->fields.len = ts;
    if (err) return fail(w, err);
    int64_t end = (int64_t)so_buf_len(w->buf);
    if ((err = push_data(w, m.start, end))) return err;
    return result(w, m.start, end, out, out_len);
}

/* end, writer.go:141-188 */
so_err so_writer_end(so_writer *w, const uint8_t **out, size_t *out_len) {
    if (out) *out = NULL;
    if (out_len) *out_len = 0;
    if (w->err) return w->err;
    entry e;
    if (!peek(w, &e)) return fail(w, "end: stack is empty");
    so_err err;
    const uint8_t *r = NULL;
    size_t rlen = 0;
    switch (e.type) {
    case E_DATA: err = end_value(w, &r, &rlen); break;
    case E_LIST: err = end_list(w, &r, &rlen); break;
    case E_MESSAGE: err = end_message(w, &r, &rlen); break;
    default: return fail(w, "end: cannot end object, invalid entry type");
    }
    if (err) return err;
    if (!peek_second_last(w, &e)) {
        if (out) *out = r;
        if (out_len) *out_len = rlen;
        return wclose(w);
    }
    if (e.type == E_ELEMENT) return end_element(w, out, out_len);
    if (e.type == E_FIELD) return end_field(w, out, out_len);
    if (out) *out = r;
    if (out_len) *out_len = rlen;
    return NULL;
}

/* ---- ValueWriter + FieldWriter + ListWriter front-ends (value.go, msg.go, list.go) ---- */

#define VALUE(call)                                   \
    do {                                              \
        if (w->err) return w->err;                    \
        int64_t start_ = (int64_t)so_buf_len(w->buf); \
        int n_;                                       \
        so_err e_ = (call);                           \
        if (e_) return fail(w, e_);                   \
        (void)n_;                                     \
        so_err p_ = push_data(w, start_, (int64_t)so_buf_len(w->buf)); \
        if (p_) return p_;                            \
    } while (0)

#define FIELD_OF(call)   \
    VALUE(call);         \
    return field(w, tag)

so_err so_field_bool(so_writer *w, uint16_t tag, int v) { FIELD_OF(so_encode_bool(w->buf, v, &n_)); }
so_err so_field_byte(so_writer *w, uint16_t tag, uint8_t v) { FIELD_OF(so_encode_byte(w->buf, v, &n_)); }
so_err so_field_int16(so_writer *w, uint16_t tag, int16_t v) { FIELD_OF(so_encode_int16(w->buf, v, &n_)); }
so_err so_field_int32(so_writer *w, uint16_t tag, int32_t v) { FIELD_OF(so_encode_int32(w->buf, v, &n_)); }
so_err so_field_int64(so_writer *w, uint16_t tag, int64_t v) { FIELD_OF(so_encode_int64(w->buf, v, &n_)); }
so_err so_field_uint16(so_writer *w, uint16_t tag, uint16_t v) { FIELD_OF(so_encode_uint16(w->buf, v, &n_)); }
so_err so_field_uint32(so_writer *w, uint16_t tag, uint32_t v) { FIELD_OF(so_encode_uint32(w->buf, v, &n_)); }
so_err so_field_uint64(so_writer *w, uint16_t tag, uint64_t v) { FIELD_OF(so_encode_uint64(w->buf, v, &n_)); }
so_err so_field_float32(so_writer *w, uint16_t tag, float v) { FIELD_OF(so_encode_float32(w->buf, v, &n_)); }
so_err so_field_float64(so_writer *w, uint16_t tag, double v) { FIELD_OF(so_encode_float64(w->buf, v, &n_)); }
so_err so_field_bin64(so_writer *w, uint16_t tag, const uint8_t v[8]) { FIELD_OF(so_encode_bin64(w->buf, v, &n_)); }
so_err so_field_bin128(so_writer *w, uint16_t tag, const uint8_t v[16]) { FIELD_OF(so_encode_bin128(w->buf, v, &n_)); }
so_err so_field_bin256(so_writer *w, uint16_t tag, const uint8_t v[32]) { FIELD_OF(so_encode_bin256(w->buf, v, &n_)); }
so_err so_field_bytes(so_writer *w, uint16_t tag, const uint8_t *v, size_t len) { FIELD_OF(so_encode_bytes(w->buf, v, len, &n_)); }
so_err so_field_string(so_writer *w, uint16_t tag, const char *v, size_t len) { FIELD_OF(so_encode_string(w->buf, v, len, &n_)); }

/* fieldAny, writer.go:438-456 (DecodeType never fails) */
so_err so_field_any(so_writer *w, uint16_t tag, const uint8_t *v, size_t len) {
    if (w->err) return w->err;
    int64_t start = (int64_t)so_buf_len(w->buf);
    if (len) memcpy(so_buf_grow(w->buf, len), v, len);
    so_err e = push_data(w, start, (int64_t)so_buf_len(w->buf));
    if (e) return e;
    return field(w, tag);
}

/* FieldWriter.List / Message, msg.go:215-227 */
so_err so_field_begin_list(so_writer *w, uint16_t tag) {
    begin_field(w, tag);
    return so_writer_begin_list(w);
}

so_err so_field_begin_message(so_writer *w, uint16_t tag) {
    begin_field(w, tag);
    return so_writer_begin_message(w);
}

#define ELEM_OF(call) \
    VALUE(call);      \
    return element(w)

so_err so_elem_int64(so_writer *w, int64_t v) { ELEM_OF(so_encode_int64(w->buf, v, &n_)); }
so_err so_elem_string(so_writer *w, const char *v, size_t len) { ELEM_OF(so_encode_string(w->buf, v, len, &n_)); }

/* ValueWriter.Any, value.go:21-36, then element() (list.go:46-51) */
so_err so_elem_any(so_writer *w, const uint8_t *v, size_t len) {
    if (w->err) return w->err;
    int64_t start = (int64_t)so_buf_len(w->buf);
    if (len) memcpy(so_buf_grow(w->buf, len), v, len);
    so_err e = push_data(w, start, (int64_t)so_buf_len(w->buf));
    if (e) return e;
    return element(w);
}

/* ListWriter.List / Message, list.go:169-178 */
so_err so_elem_begin_list(so_writer *w) {
    begin_element(w);
    return so_writer_begin_list(w);
}

so_err so_elem_begin_message(so_writer *w) {
    begin_element(w);
    return so_writer_begin_message(w);
}

so_err so_value_int64(so_writer *w, int64_t v) {
    VALUE(so_encode_int64(w->buf, v, &n_));
    return NULL;
}

so_err so_value_string(so_writer *w, const char *v, size_t len) {
    VALUE(so_encode_string(w->buf, v, len, &n_));
    return NULL;
}

/* ---- generic values by column kind (the generated writers' per-kind calls) ---- */

/* One column element of `kind` appended through its encoder (internal/encode/...): v is the
 * column element (so_kind_width(kind) bytes); string/bytes elements are {u32 off, u32 len}
 * into heap. */
static so_err encode_kind(so_buf *b, int kind, const uint8_t *v, const uint8_t *heap, int *n) {
    switch (kind) {
    case SO_KIND_BOOL: return so_encode_bool(b, v[0] != 0, n);
    case SO_KIND_BYTE: return so_encode_byte(b, v[0], n);
    case SO_KIND_INT16: { int16_t x; memcpy(&x, v, 2); return so_encode_int16(b, x, n); }
    case SO_KIND_INT32: { int32_t x; memcpy(&x, v, 4); return so_encode_int32(b, x, n); }
    case SO_KIND_INT64: { int64_t x; memcpy(&x, v, 8); return so_encode_int64(b, x, n); }
    case SO_KIND_UINT16: { uint16_t x; memcpy(&x, v, 2); return so_encode_uint16(b, x, n); }
    case SO_KIND_UINT32: { uint32_t x; memcpy(&x, v, 4); return so_encode_uint32(b, x, n); }
    case SO_KIND_UINT64: { uint64_t x; memcpy(&x, v, 8); return so_encode_uint64(b, x, n); }
    case SO_KIND_FLOAT32: { float x; memcpy(&x, v, 4); return so_encode_float32(b, x, n); }
    case SO_KIND_FLOAT64: { double x; memcpy(&x, v, 8); return so_encode_float64(b, x, n); }
    case SO_KIND_BIN64: return so_encode_bin64(b, v, n);
    case SO_KIND_BIN128: return so_encode_bin128(b, v, n);
    case SO_KIND_BIN256: return so_encode_bin256(b, v, n);
    case SO_KIND_STRING:
    case SO_KIND_BYTES: {
        uint32_t span[2];
        memcpy(span, v, 8);
        const uint8_t *p = heap ? heap + span[0] : (const uint8_t *)"";
        return kind == SO_KIND_STRING ? so_encode_string(b, (const char *)p, span[1], n)
                                      : so_encode_bytes(b, p, span[1], n);
    }
    }
    return "encode: unsupported kind";
}

/* The generated EncodeXxxTo of a struct (internal/lang/generator/struct.go:115-142): every
 * member through its encoder in declaration order, then EncodeStruct(dataSize)
 * (internal/encode/struct.go:14-21).  An inner struct member (kinds[i] == SO_KIND_STRUCT,
 * nmem[i] direct members following it in the arrays) is its own EncodeXxxTo in place.
 * `top` members from *at on; *at advances past them. */
static so_err encode_struct_at(so_buf *b, int top, int *at, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                               const uint8_t *const *heaps, const int *nmem, int *n) {
    int64_t data = 0;
    for (int i = 0; i < top; i++) {
        if (*at >= nm) return "encode struct: member list too short";
        const int j = (*at)++;
        int k = 0;
        so_err e = kinds[j] == SO_KIND_STRUCT ? encode_struct_at(b, nmem ? nmem[j] : 0, at, nm, kinds, vals, heaps, nmem, &k)
                                              : encode_kind(b, kinds[j], vals[j], heaps ? heaps[j] : NULL, &k);
        if (e) return e;
        data += k;
    }
    int k = 0;
    so_err e = so_encode_struct(b, data, &k);
    if (e) return e;
    *n = (int)(data + k);
    return NULL;
}

static so_err encode_struct(so_buf *b, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                            const uint8_t *const *heaps, int *n) {
    int at = 0;
    return encode_struct_at(b, nm, &at, nm, kinds, vals, heaps, NULL, n);
}

static so_err encode_struct_tree(so_buf *b, int top, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                                 const uint8_t *const *heaps, const int *nmem, int *n) {
    int at = 0;
    so_err e = encode_struct_at(b, top, &at, nm, kinds, vals, heaps, nmem, n);
    return e ? e : (at == nm ? NULL : "encode struct: member list too long");
}

/* FieldWriter.<Kind>(v) (internal/writer/msg.go:99-211) by column kind */
so_err so_field_value(so_writer *w, uint16_t tag, int kind, const uint8_t *v, const uint8_t *heap) {
    FIELD_OF(encode_kind(w->buf, kind, v, heap, &n_));
}

/* ListWriter.<Kind>(v) / ValueListWriter.Add (writer_list_value.go:26-29): value + element() */
so_err so_elem_value(so_writer *w, int kind, const uint8_t *v, const uint8_t *heap) {
    ELEM_OF(encode_kind(w->buf, kind, v, heap, &n_));
}

/* spec.WriteField(w.Field(tag), v, EncodeXxxTo) for a struct field (generator/message.go:402-408,
 * internal/writer/msg.go:75-80): the struct through WriteValue, then field(tag) */
so_err so_field_struct(so_writer *w, uint16_t tag, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                       const uint8_t *const *heaps) {
    FIELD_OF(encode_struct(w->buf, nm, kinds, vals, heaps, &n_));
}

/* ValueListWriter[Struct].Add = WriteElement(list, v, EncodeXxxTo) (internal/writer/list.go:37-43) */
so_err so_elem_struct(so_writer *w, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                      const uint8_t *const *heaps) {
    ELEM_OF(encode_struct(w->buf, nm, kinds, vals, heaps, &n_));
}

/* Structs with inner structs: members in pre-order (see encode_struct_at) */
so_err so_field_struct_tree(so_writer *w, uint16_t tag, int top, int nm, const uint8_t *kinds,
                            const uint8_t *const *vals, const uint8_t *const *heaps, const int *nmem) {
    FIELD_OF(encode_struct_tree(w->buf, top, nm, kinds, vals, heaps, nmem, &n_));
}

so_err so_elem_struct_tree(so_writer *w, int top, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                           const uint8_t *const *heaps, const int *nmem) {
    ELEM_OF(encode_struct_tree(w->buf, top, nm, kinds, vals, heaps, nmem, &n_));
}
