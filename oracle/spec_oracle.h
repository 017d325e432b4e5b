/*
 * spec_oracle.h — CPU restatement of basecomplextech/spec's binary format, codecs,
 * Writer and Message/List readers.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the MI355X engine
 * in spec_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.  The product path never links or calls it.
 *
 * Parity status:
 *   - Behaviour is pinned against every assertion of the reference's own tests for
 *     this path (internal/decode/..._test.go, internal/writer/..._test.go), ported under
 *     tests/test_oracle_*.py.
 *   - The reference holds NO byte-level golden vectors, and its varint codec lives in the
 *     absent third-party module github.com/basecomplextech/baselibrary
 *     v0.0.0-20250218120829-9ca66e53fd5f (encoding/compactint).  The varint byte layout
 *     is therefore a reconstruction (compactint.c): "parity unpinned" at the varint byte
 *     level.  Everything else (type codes, tables, trailers, writer ordering) follows the
 *     reference source directly and is cited per function.
 *
 * Reference paths are relative to the reference repo root.
 */
#ifndef SPEC_ORACLE_H
#define SPEC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- format (internal/format/type.go:13-52) ---- */
enum {
    SO_TYPE_UNDEFINED = 0,
    SO_TYPE_TRUE = 1,
    SO_TYPE_FALSE = 2,
    SO_TYPE_BYTE = 3,
    SO_TYPE_INT16 = 10,
    SO_TYPE_INT32 = 11,
    SO_TYPE_INT64 = 12,
    SO_TYPE_UINT16 = 20,
    SO_TYPE_UINT32 = 21,
    SO_TYPE_UINT64 = 22,
    SO_TYPE_BIN64 = 30,
    SO_TYPE_BIN128 = 31,
    SO_TYPE_BIN256 = 32,
    SO_TYPE_FLOAT32 = 40,
    SO_TYPE_FLOAT64 = 41,
    SO_TYPE_BYTES = 50,
    SO_TYPE_STRING = 60,
    SO_TYPE_LIST = 70,
    SO_TYPE_BIG_LIST = 71,
    SO_TYPE_MESSAGE = 80,
    SO_TYPE_BIG_MESSAGE = 81,
    SO_TYPE_STRUCT = 90,
};

#define SO_MAX_SIZE 2147483647 /* format.MaxSize = math.MaxInt32, type.go:14 */
#define SO_MAX_LEN32 5         /* compactint.MaxLen32 (reconstruction) */
#define SO_MAX_LEN64 10        /* compactint.MaxLen64 (reconstruction) */

/* Errors are static strings (NULL = no error) whose text follows the reference's
 * error messages, so tests can match the same substrings the Go tests match. */
typedef const char *so_err;

int so_type_check(uint8_t t); /* 0 ok, -1 unsupported (type.go:54-90) */

/* ---- compactint reconstruction (compactint.c) ---- */
int so_put_reverse_uint32(uint8_t p[SO_MAX_LEN32], uint32_t v);
int so_put_reverse_uint64(uint8_t p[SO_MAX_LEN64], uint64_t v);
int so_put_reverse_int32(uint8_t p[SO_MAX_LEN32], int32_t v);
int so_put_reverse_int64(uint8_t p[SO_MAX_LEN64], int64_t v);
uint32_t so_reverse_uint32(const uint8_t *b, size_t len, int *n);
uint64_t so_reverse_uint64(const uint8_t *b, size_t len, int *n);
int32_t so_reverse_int32(const uint8_t *b, size_t len, int *n);
int64_t so_reverse_int64(const uint8_t *b, size_t len, int *n);
int so_reverse_size(const uint8_t *b, size_t len);

/* ---- append buffer (baselibrary buffer.Buffer semantics: Grow/Len/Bytes) ---- */
typedef struct so_buf {
    uint8_t *data;
    size_t len;
    size_t cap;
    int owned; /* 1: realloc-able heap memory; 0: fixed caller memory */
    int overflow;
} so_buf;

so_buf *so_buf_new(size_t cap);
void so_buf_init_fixed(so_buf *b, uint8_t *mem, size_t cap);
void so_buf_free(so_buf *b);
void so_buf_reset(so_buf *b);
uint8_t *so_buf_grow(so_buf *b, size_t n);
size_t so_buf_len(const so_buf *b);
uint8_t *so_buf_bytes(const so_buf *b);

/* ---- format tables (internal/format/msg.go, list.go) ---- */
typedef struct so_message_field {
    uint16_t tag;
    uint32_t offset;
} so_message_field;

typedef struct so_list_element {
    uint32_t offset;
} so_list_element;

typedef struct so_message_table {
    const uint8_t *table;
    size_t table_len;
    uint32_t data;
    int big;
} so_message_table;

typedef struct so_list_table {
    const uint8_t *table;
    size_t table_len;
    uint32_t data;
    int big;
} so_list_table;

int so_is_big_message(const so_message_field *fields, size_t n);
int so_is_big_list(const so_list_element *elems, size_t n);
int so_message_table_len(const so_message_table *t);
int64_t so_message_table_offset(const so_message_table *t, uint16_t tag);
int64_t so_message_table_offset_by_index(const so_message_table *t, int i);
int so_message_table_field(const so_message_table *t, int i, so_message_field *f);
int so_list_table_len(const so_list_table *t);
void so_list_table_offset(const so_list_table *t, int i, int64_t *start, int64_t *end);

/* ---- encode (internal/encode/...) ---- */
so_err so_encode_bool(so_buf *b, int v, int *n);
so_err so_encode_byte(so_buf *b, uint8_t v, int *n);
so_err so_encode_int16(so_buf *b, int16_t v, int *n);
so_err so_encode_int32(so_buf *b, int32_t v, int *n);
so_err so_encode_int64(so_buf *b, int64_t v, int *n);
so_err so_encode_uint16(so_buf *b, uint16_t v, int *n);
so_err so_encode_uint32(so_buf *b, uint32_t v, int *n);
so_err so_encode_uint64(so_buf *b, uint64_t v, int *n);
so_err so_encode_float32(so_buf *b, float v, int *n);
so_err so_encode_float64(so_buf *b, double v, int *n);
so_err so_encode_bin64(so_buf *b, const uint8_t v[8], int *n);
so_err so_encode_bin128(so_buf *b, const uint8_t v[16], int *n);
so_err so_encode_bin256(so_buf *b, const uint8_t v[32], int *n);
so_err so_encode_bytes(so_buf *b, const uint8_t *v, size_t len, int *n);
so_err so_encode_string(so_buf *b, const char *s, size_t len, int *n);
so_err so_encode_struct(so_buf *b, int64_t data_size, int *n);
so_err so_encode_list_table(so_buf *b, int64_t data_size, const so_list_element *t, size_t cnt, int *n);
so_err so_encode_message_table(so_buf *b, int64_t data_size, const so_message_field *t, size_t cnt, int *n);

/* ---- decode (internal/decode/...); every decoder parses the value ENDING at b+len ---- */
so_err so_decode_type(const uint8_t *b, size_t len, uint8_t *t, int *n);
so_err so_decode_type_size(const uint8_t *b, size_t len, uint8_t *t, int *n);
so_err so_decode_bool(const uint8_t *b, size_t len, int *v, int *n);
so_err so_decode_byte(const uint8_t *b, size_t len, uint8_t *v, int *n);
so_err so_decode_int16(const uint8_t *b, size_t len, int16_t *v, int *n);
so_err so_decode_int32(const uint8_t *b, size_t len, int32_t *v, int *n);
so_err so_decode_int64(const uint8_t *b, size_t len, int64_t *v, int *n);
so_err so_decode_uint16(const uint8_t *b, size_t len, uint16_t *v, int *n);
so_err so_decode_uint32(const uint8_t *b, size_t len, uint32_t *v, int *n);
so_err so_decode_uint64(const uint8_t *b, size_t len, uint64_t *v, int *n);
so_err so_decode_float32(const uint8_t *b, size_t len, float *v, int *n);
so_err so_decode_float64(const uint8_t *b, size_t len, double *v, int *n);
so_err so_decode_bin64(const uint8_t *b, size_t len, uint8_t v[8], int *n);
so_err so_decode_bin128(const uint8_t *b, size_t len, uint8_t v[16], int *n);
so_err so_decode_bin256(const uint8_t *b, size_t len, uint8_t v[32], int *n);
/* bytes/string return a view: *off = offset of the payload from b, *vlen = its length */
so_err so_decode_bytes(const uint8_t *b, size_t len, size_t *off, size_t *vlen, int *n);
so_err so_decode_string(const uint8_t *b, size_t len, size_t *off, size_t *vlen, int *n);
so_err so_decode_struct(const uint8_t *b, size_t len, int *data_size, int *n);
so_err so_decode_list_table(const uint8_t *b, size_t len, so_list_table *t, int *n);
so_err so_decode_message_table(const uint8_t *b, size_t len, so_message_table *t, int *n);

/* ---- types.Message / types.List (internal/types/msg.go, list.go) ---- */
typedef struct so_message {
    so_message_table table;
    const uint8_t *bytes;
    size_t len;
} so_message;

typedef struct so_list {
    so_list_table table;
    const uint8_t *bytes;
    size_t len;
} so_list;

so_err so_open_message_err(const uint8_t *b, size_t len, so_message *m);
void so_open_message(const uint8_t *b, size_t len, so_message *m);
so_err so_parse_message(const uint8_t *b, size_t len, so_message *m, int *size);
int so_message_fields(const so_message *m);
int so_message_has_field(const so_message *m, uint16_t tag);
/* field(tag): the raw slice bytes[:end] or NULL/0 (msg.go:466-475) */
const uint8_t *so_message_field_raw(const so_message *m, uint16_t tag, size_t *len);
const uint8_t *so_message_field_at_raw(const so_message *m, int i, size_t *len);
int so_message_bool(const so_message *m, uint16_t tag);
uint8_t so_message_byte(const so_message *m, uint16_t tag);
int16_t so_message_int16(const so_message *m, uint16_t tag);
int32_t so_message_int32(const so_message *m, uint16_t tag);
int64_t so_message_int64(const so_message *m, uint16_t tag);
uint16_t so_message_uint16(const so_message *m, uint16_t tag);
uint32_t so_message_uint32(const so_message *m, uint16_t tag);
uint64_t so_message_uint64(const so_message *m, uint16_t tag);
float so_message_float32(const so_message *m, uint16_t tag);
double so_message_float64(const so_message *m, uint16_t tag);
void so_message_bin64(const so_message *m, uint16_t tag, uint8_t v[8]);
void so_message_bin128(const so_message *m, uint16_t tag, uint8_t v[16]);
void so_message_bin256(const so_message *m, uint16_t tag, uint8_t v[32]);
/* returns pointer to payload (NULL if absent/error) and its length */
const uint8_t *so_message_bytes(const so_message *m, uint16_t tag, size_t *len);
const uint8_t *so_message_string(const so_message *m, uint16_t tag, size_t *len);
void so_message_list(const so_message *m, uint16_t tag, so_list *l);
void so_message_message(const so_message *m, uint16_t tag, so_message *sub);

so_err so_open_list_err(const uint8_t *b, size_t len, so_list *l);
int so_list_len(const so_list *l);
/* GetBytes(i): returns 0 ok, -1 index out of range (Go panics); slice may be NULL/0 */
int so_list_get_bytes(const so_list *l, int i, const uint8_t **p, size_t *len);

so_err so_parse_value(const uint8_t *b, size_t len, int *n);
so_err so_parse_list(const uint8_t *b, size_t len, int *size);

/* ---- Writer (internal/writer/...) ---- */
typedef struct so_writer so_writer;

so_writer *so_writer_new(so_buf *buf);
void so_writer_free(so_writer *w);
void so_writer_reset(so_writer *w, so_buf *buf);
so_err so_writer_err(const so_writer *w);
/* Root objects */
so_err so_writer_begin_message(so_writer *w); /* Writer.Message() */
so_err so_writer_begin_list(so_writer *w);    /* Writer.List() */
/* Value().X(v) followed by field(tag): FieldWriter.X (writer/msg.go:99-211) */
so_err so_field_bool(so_writer *w, uint16_t tag, int v);
so_err so_field_byte(so_writer *w, uint16_t tag, uint8_t v);
so_err so_field_int16(so_writer *w, uint16_t tag, int16_t v);
so_err so_field_int32(so_writer *w, uint16_t tag, int32_t v);
so_err so_field_int64(so_writer *w, uint16_t tag, int64_t v);
so_err so_field_uint16(so_writer *w, uint16_t tag, uint16_t v);
so_err so_field_uint32(so_writer *w, uint16_t tag, uint32_t v);
so_err so_field_uint64(so_writer *w, uint16_t tag, uint64_t v);
so_err so_field_float32(so_writer *w, uint16_t tag, float v);
so_err so_field_float64(so_writer *w, uint16_t tag, double v);
so_err so_field_bin64(so_writer *w, uint16_t tag, const uint8_t v[8]);
so_err so_field_bin128(so_writer *w, uint16_t tag, const uint8_t v[16]);
so_err so_field_bin256(so_writer *w, uint16_t tag, const uint8_t v[32]);
so_err so_field_bytes(so_writer *w, uint16_t tag, const uint8_t *v, size_t len);
so_err so_field_string(so_writer *w, uint16_t tag, const char *v, size_t len);
so_err so_field_any(so_writer *w, uint16_t tag, const uint8_t *v, size_t len);
so_err so_field_begin_list(so_writer *w, uint16_t tag);    /* FieldWriter.List() */
so_err so_field_begin_message(so_writer *w, uint16_t tag); /* FieldWriter.Message() */
int so_writer_has_field(so_writer *w, uint16_t tag);
/* ListWriter element writes (writer/list.go) */
so_err so_elem_int64(so_writer *w, int64_t v);
so_err so_elem_string(so_writer *w, const char *v, size_t len);
so_err so_elem_any(so_writer *w, const uint8_t *v, size_t len);
so_err so_elem_begin_list(so_writer *w);    /* ListWriter.List() */
so_err so_elem_begin_message(so_writer *w); /* ListWriter.Message() */
int so_writer_list_len(so_writer *w);
/* ValueWriter (writer/value.go) for root values */
/* FieldWriter / ListWriter calls by column kind (v = column element; string/bytes = {u32 off,
 * u32 len} into heap), and struct fields/elements (generated EncodeXxxTo: members then
 * EncodeStruct, internal/lang/generator/struct.go:115-142) */
so_err so_field_value(so_writer *w, uint16_t tag, int kind, const uint8_t *v, const uint8_t *heap);
so_err so_elem_value(so_writer *w, int kind, const uint8_t *v, const uint8_t *heap);
so_err so_field_struct(so_writer *w, uint16_t tag, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                       const uint8_t *const *heaps);
so_err so_elem_struct(so_writer *w, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                      const uint8_t *const *heaps);
/* structs with inner structs: nm members in pre-order, an inner struct = SO_KIND_STRUCT followed
 * by its nmem[i] direct members; `top` = the outer struct's direct members */
so_err so_field_struct_tree(so_writer *w, uint16_t tag, int top, int nm, const uint8_t *kinds,
                            const uint8_t *const *vals, const uint8_t *const *heaps, const int *nmem);
so_err so_elem_struct_tree(so_writer *w, int top, int nm, const uint8_t *kinds, const uint8_t *const *vals,
                           const uint8_t *const *heaps, const int *nmem);
so_err so_value_int64(so_writer *w, int64_t v);
so_err so_value_string(so_writer *w, const char *v, size_t len);
/* end(): MessageWriter.Build / ListWriter.Build / ValueWriter.Build (writer.go:141-188) */
so_err so_writer_end(so_writer *w, const uint8_t **out, size_t *out_len);
/* message-stack test hooks (stack_msg.go) */
typedef struct so_message_stack so_message_stack;
so_message_stack *so_message_stack_new(void);
void so_message_stack_free(so_message_stack *s);
void so_message_stack_insert(so_message_stack *s, int table_offset, uint16_t tag, uint32_t off);
int so_message_stack_pop(so_message_stack *s, int table_offset, so_message_field *out, int cap);
int so_message_stack_has_field(so_message_stack *s, int table_offset, uint16_t tag);

/* ---- batch harness (batch.c): the reference's per-record loops over a record batch ---- */
/* Column kinds: same numbering as include/spec_amd.h SPEC_KIND_* */
enum {
    SO_KIND_BOOL = 1,
    SO_KIND_BYTE = 2,
    SO_KIND_INT16 = 3,
    SO_KIND_INT32 = 4,
    SO_KIND_INT64 = 5,
    SO_KIND_UINT16 = 6,
    SO_KIND_UINT32 = 7,
    SO_KIND_UINT64 = 8,
    SO_KIND_FLOAT32 = 9,
    SO_KIND_FLOAT64 = 10,
    SO_KIND_BIN64 = 11,
    SO_KIND_BIN128 = 12,
    SO_KIND_BIN256 = 13,
    SO_KIND_STRING = 14,
    SO_KIND_BYTES = 15,
};

int so_kind_width(int kind);

/* Decode N flat records: per record OpenMessageErr + one typed getter per field
 * (internal/bench/parse_test.go:48-111 pattern).  Column i is an array of
 * so_kind_width(kinds[i]) bytes per record; string/bytes columns hold
 * {uint32 off (from stream base), uint32 len}.  status[r] = SPEC_STATUS_* code. */
int so_decode_flat_batch(int nfields, const uint16_t *tags, const uint8_t *kinds,
                         const uint8_t *stream, const uint64_t *ends, uint64_t n,
                         void *const *columns, uint8_t *status, int nthreads);

/* Per record, which *Err getters err (internal/types/msg.go:233-459): errmask bit f. */
int so_decode_flat_errors(int nfields, const uint16_t *tags, const uint8_t *kinds, const uint8_t *stream,
                          const uint64_t *ends, uint64_t n, uint64_t *errmask);

/* Encode N flat records with the Writer (write_test.go:16-78 pattern:
 * NewMessageWriterBuffer + one FieldWriter call per field in schema order + Build).
 * string/bytes columns are {uint32 off, uint32 len} into heaps[i].
 * Returns 0, or -1 on writer error / -2 if out_cap is too small. */
int so_encode_flat_batch(int nfields, const uint16_t *tags, const uint8_t *kinds,
                         const void *const *columns, const uint8_t *const *heaps, uint64_t n,
                         uint8_t *out, uint64_t out_cap, uint64_t *ends);

/* Nested schema (config 4): outer {1 bin128 id, 2 int64 seq, 3 string name,
 * 4 list<Item>}, Item {1 int32 key, 2 float64 value, 3 string label}.
 * item_begin[r] is the CSR offset of record r's first item (n+1 entries). */
int so_encode_nested_batch(const uint8_t *id, const int64_t *seq, const uint32_t *name,
                           const uint8_t *name_heap, const uint32_t *item_begin,
                           const int32_t *key, const double *value, const uint32_t *label,
                           const uint8_t *label_heap, uint64_t n, uint8_t *out,
                           uint64_t out_cap, uint64_t *ends);
/* Decode pass 1: item count per record (MessageList.Len after m.List(4)). */
int so_decode_nested_counts(const uint8_t *stream, const uint64_t *ends, uint64_t n,
                            uint32_t *counts, uint8_t *status);
/* Decode pass 2: all columns; items written at item_begin[r]. */
int so_decode_nested_batch(const uint8_t *stream, const uint64_t *ends, uint64_t n,
                           const uint32_t *item_begin, uint8_t *id, int64_t *seq,
                           uint32_t *name, int32_t *key, double *value, uint32_t *label,
                           uint8_t *item_status, uint8_t *status);
/* The CPU baseline loops on nthreads host threads (contiguous record shards; an encode shard t
 * writes its records into out + t * (out_cap / nthreads), ends relative to that region). */
int so_encode_flat_batch_mt(int nfields, const uint16_t *tags, const uint8_t *kinds, const void *const *columns,
                            const uint8_t *const *heaps, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *ends,
                            int nthreads);
int so_encode_nested_batch_mt(const uint8_t *id, const int64_t *seq, const uint32_t *name, const uint8_t *name_heap,
                              const uint32_t *item_begin, const int32_t *key, const double *value,
                              const uint32_t *label, const uint8_t *label_heap, uint64_t n, uint8_t *out,
                              uint64_t out_cap, uint64_t *ends, int nthreads);
int so_decode_nested_batch_mt(const uint8_t *stream, const uint64_t *ends, uint64_t n, const uint32_t *item_begin,
                              uint8_t *id, int64_t *seq, uint32_t *name, int32_t *key, double *value, uint32_t *label,
                              uint8_t *item_status, uint8_t *status, int nthreads);

/* ParseMessage per record (spec_parse_messages semantics): status 0 ok, 1-5 trailer class,
 * 6 panic (list element start > end), 7 nested value error; sizes = message bytes or 0.
 * head = bytes before each record (4 for mpx frames). */
int so_parse_batch_root(int root, const uint8_t *stream, const uint64_t *ends, uint64_t n, uint32_t head,
                        uint8_t *status, uint32_t *sizes);
int so_parse_batch(const uint8_t *stream, const uint64_t *ends, uint64_t n, uint32_t head, uint8_t *status,
                   uint32_t *sizes);

/* ---- schema trees (tree.c): structs, sub-messages, value lists, lists of structs/messages,
 * any — the generated readers/writers of internal/lang/generator over a batch ----
 * Field descriptors mirror include/spec_amd.h spec_tree_field (same layout and rules); the
 * table/column layout is restated independently (tree.c) and compared with the engine's in
 * the tests. */
enum { SO_KIND_LIST = 16, SO_KIND_STRUCT = 17, SO_KIND_MESSAGE = 18, SO_KIND_ANY = 19 };
typedef struct so_tree_field {
    uint16_t tag;
    uint8_t kind;
    uint8_t elem;
    int16_t parent;
    uint16_t reserved;
} so_tree_field;
typedef struct so_tree_table {
    int16_t parent, field;
    uint8_t rel, shape;
    uint16_t first_column, ncolumns;
} so_tree_table;
typedef struct so_tree_column {
    uint16_t table;
    int16_t field;
    uint8_t role, kind;
    uint16_t width;
} so_tree_column;
/* 0 ok, -1 invalid tree */
int so_tree_layout(const so_tree_field *f, int nf, so_tree_table *tables, int *ntables, so_tree_column *cols,
                   int *ncols);
/* Per record: the generated reader's getters over the whole tree (OpenMessageErr, getters,
 * HasField, Message(tag), List(tag) + Get(i), OpenStruct, Field(tag)).  rows[t] = rows of
 * table t; columns (may be NULL: rows only) in layout order, sized by rows. */
int so_decode_tree_batch(const so_tree_field *f, int nf, const uint8_t *stream, const uint64_t *ends, uint64_t n,
                         void *const *columns, uint64_t *rows);
int so_decode_tree_spans(const so_tree_field *f, int nf, const uint8_t *stream, uint64_t stream_len,
                         const uint32_t *spans, uint64_t n, void *const *columns, uint64_t *rows);
int so_decode_values(int kind, const uint8_t *stream, uint64_t stream_len, const uint32_t *spans, uint64_t n,
                     uint8_t *out, uint8_t *err);
/* Per record: the generated Write() over the tree (scalars always written; sub-messages and
 * lists when their PRESENT byte is set; any when its span is non-empty), Build().
 * heaps[c] backs string/bytes/any column c.  0 ok, -1 writer error, -2 out too small. */
int so_encode_tree_batch(const so_tree_field *f, int nf, const void *const *columns, const uint8_t *const *heaps,
                         uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *ends);

/* mpx frame read loop over a received buffer (mpx/conn_reader.go:179-194): frame count and
 * ends (offset past each complete frame's message), -1 if more than cap frames are complete. */
long long so_frames_read(const uint8_t *buf, uint64_t len, uint64_t *ends, uint64_t cap, uint64_t *consumed);

/* ---- LZ4 block + frame formats (oracle/lz4.c; mpx compression, pierrec/lz4/v4 restated) ---- */
uint32_t so_xxh32(const void *data, size_t len, uint32_t seed);
long long so_lz4_decompress_block(const uint8_t *src, size_t n, uint8_t *dst, size_t cap);
long long so_lz4_compress_block(const uint8_t *src, size_t n, uint8_t *dst, size_t cap);
long long so_lz4_frame_write(const uint8_t *data, const uint64_t *flush_ends, size_t nflush, uint32_t block_max,
                             int content_checksum, int block_checksum, int close, uint8_t *out, size_t cap);
int so_lz4_frame_read(const uint8_t *buf, size_t len, uint8_t *out, size_t cap, size_t *out_len, size_t *consumed);

#ifdef __cplusplus
}
#endif

#endif
