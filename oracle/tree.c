/*
 * tree.c — the generated readers and writers of a whole schema tree, per record: structs,
 * enums (int32), sub-messages, value lists, lists of structs and of messages, any.
 * TEST INFRASTRUCTURE (oracle): the parity checker for spec_decode_tree / spec_encode_tree.
 *
 * What a generated reader does per field (internal/lang/generator/message.go:97-186):
 *   scalar         m.msg.<Kind>(tag)                         internal/types/msg.go:219-421
 *   struct         OpenXxx(m.msg.FieldRaw(tag))              message.go:176-183, msg.go:139-150,
 *                  = Xxx.Decode: DecodeStruct, members in REVERSE order   generator/struct.go:75-113
 *   any            m.msg.Field(tag) = OpenValue(bytes[:end]) internal/types/msg.go:108-124,
 *                                                            internal/types/value.go:18-31
 *   message        NewXxx(m.msg.Message(tag)); HasXxx = HasField       msg.go:447-451
 *   list<value>    spec.NewValueList(m.msg.List(tag), DecodeX); Get(i) list_value.go:87-92
 *   list<message>  spec.NewMessageList(m.msg.List(tag), OpenXxxErr)    list_msg.go:88-92
 * and a generated writer (message.go:319-439, struct.go:115-142; the calls pkg1/object.go makes):
 *   scalar  w.Field(tag).<Kind>(v); struct spec.WriteField(w.Field(tag), v, EncodeXxxTo);
 *   any     w.Field(tag).Any(v); message w.Field(tag).Message() ... End();
 *   list    w.Field(tag).List() + Add(v) / Add() ... End() ... End().
 *
 * Output layout (restated from include/spec_amd.h, independently of the engine): tables —
 * the root (one row per record), one per MESSAGE field (rows = its owner's rows), one per
 * LIST field (rows = elements, CSR `begin` over the owner's rows); columns table by table:
 * [BEGIN], then per direct field VALUE (scalar), VALUE per member (struct), VALUE span (any),
 * PRESENT (message, list); a value list's VALUE, a struct list's member VALUEs; then STATUS.
 */
#include <stdlib.h>
#include <string.h>

#include "spec_oracle.h"

enum { REL_ROOT = 0, REL_ONE = 1, REL_MANY = 2 };
enum { SHAPE_MESSAGE = 0, SHAPE_VALUE = 1, SHAPE_STRUCT = 2 };
enum { ROLE_VALUE = 0, ROLE_PRESENT = 1, ROLE_BEGIN = 2, ROLE_STATUS = 3, ROLE_ERRMASK = 4, ROLE_TYPE = 5 };
enum { ST_OK = 0, ST_PANIC = 6, ST_INVALID_VALUE = 7 };
#define MAX_F 1024
#define MAX_T 128
#define MAX_C 2048

static int scalar(int k) { return k >= SO_KIND_BOOL && k <= SO_KIND_BYTES; }

typedef struct {
    const so_tree_field *f;
    int nf;
    so_tree_table T[MAX_T];
    so_tree_column C[MAX_C];
    int nt, nc;
    int table_of[MAX_F]; /* table a MESSAGE / LIST field defines */
    int col_of[MAX_F];   /* VALUE column of a field (a struct member: its own; a value list: its elements) */
    int present_of[MAX_F]; /* PRESENT column of a MESSAGE / LIST field */
    int status_col[MAX_T], begin_col[MAX_T], err_col[MAX_T];
    int type_of[MAX_F]; /* TYPE column of an ANY field */
    const uint8_t *stream;
    void *const *cols;
    const uint8_t *const *heaps;
    uint64_t rows[MAX_T];
} tree;

static int owner_table(const tree *t, int i) {
    int p = t->f[i].parent;
    while (p >= 0 && t->f[p].kind == SO_KIND_STRUCT) p = t->f[p].parent;
    return p < 0 ? 0 : t->table_of[p];
}

static int add_col(tree *t, int table, int field, int role, int kind, int width) {
    if (t->nc >= MAX_C) return -1;
    so_tree_column c = {(uint16_t)table, (int16_t)field, (uint8_t)role, (uint8_t)kind, (uint16_t)width};
    t->C[t->nc] = c;
    return t->nc++;
}

/* The columns of struct field sf in table x: its members in declaration order, an inner
 * struct's members (recursively) in its place. */
static int struct_cols(tree *t, int x, int sf) {
    for (int j = sf + 1; j < t->nf; j++) {
        if (t->f[j].parent != sf) continue;
        int c;
        if (t->f[j].kind == SO_KIND_STRUCT)
            c = struct_cols(t, x, j);
        else
            c = t->col_of[j] = add_col(t, x, j, ROLE_VALUE, t->f[j].kind, so_kind_width(t->f[j].kind));
        if (c < 0) return -1;
    }
    return 0;
}

static int build(tree *t, const so_tree_field *f, int nf) {
    memset(t, 0, sizeof(*t));
    t->f = f;
    t->nf = nf;
    if (nf < 0 || nf > MAX_F) return -1;
    for (int i = 0; i < nf; i++) {
        int k = f[i].kind, p = f[i].parent;
        t->table_of[i] = -1;
        t->col_of[i] = t->present_of[i] = -1;
        if (p < -1 || p >= i) return -1;
        if (!scalar(k) && k != SO_KIND_LIST && k != SO_KIND_STRUCT && k != SO_KIND_MESSAGE && k != SO_KIND_ANY) return -1;
        if (k == SO_KIND_LIST && !scalar(f[i].elem) && f[i].elem != SO_KIND_STRUCT && f[i].elem != SO_KIND_MESSAGE)
            return -1;
        if (p >= 0) {
            int pk = f[p].kind;
            /* struct members: value types or other structs (model/struct_field.go:57-70) */
            if (pk == SO_KIND_STRUCT && !scalar(k) && k != SO_KIND_STRUCT) return -1;
            if (pk == SO_KIND_LIST && f[p].elem == SO_KIND_STRUCT && !scalar(k) && k != SO_KIND_STRUCT) return -1;
            if (pk == SO_KIND_LIST && scalar(f[p].elem)) return -1;
            if (pk != SO_KIND_STRUCT && pk != SO_KIND_MESSAGE && pk != SO_KIND_LIST) return -1;
        }
    }
    /* struct nesting depth (at most 16 structs deep, spec_amd.h SPEC_TREE_MAX_STRUCT_DEPTH) */
    for (int i = 0; i < nf; i++) {
        int depth = f[i].kind == SO_KIND_STRUCT;
        for (int p = f[i].parent; p >= 0; p = f[p].parent)
            depth += f[p].kind == SO_KIND_STRUCT || (f[p].kind == SO_KIND_LIST && f[p].elem == SO_KIND_STRUCT);
        if (depth > 16) return -1;
    }
    /* tables: the root, then one per MESSAGE / LIST field in field order */
    so_tree_table root = {-1, -1, REL_ROOT, SHAPE_MESSAGE, 0, 0};
    t->T[t->nt++] = root;
    for (int i = 0; i < nf; i++) {
        int k = f[i].kind;
        if (k != SO_KIND_MESSAGE && k != SO_KIND_LIST) continue;
        if (t->nt >= MAX_T) return -1;
        so_tree_table tb;
        tb.parent = (int16_t)owner_table(t, i);
        tb.field = (int16_t)i;
        tb.rel = k == SO_KIND_MESSAGE ? REL_ONE : REL_MANY;
        tb.shape = k == SO_KIND_MESSAGE || f[i].elem == SO_KIND_MESSAGE ? SHAPE_MESSAGE
                   : f[i].elem == SO_KIND_STRUCT                        ? SHAPE_STRUCT
                                                                         : SHAPE_VALUE;
        tb.first_column = tb.ncolumns = 0;
        t->table_of[i] = t->nt;
        t->T[t->nt++] = tb;
    }
    /* columns, table by table */
    for (int x = 0; x < t->nt; x++) {
        so_tree_table *tb = &t->T[x];
        int d = tb->field;
        tb->first_column = (uint16_t)t->nc;
        t->begin_col[x] = -1;
        if (tb->rel == REL_MANY && (t->begin_col[x] = add_col(t, x, d, ROLE_BEGIN, 0, 4)) < 0) return -1;
        if (tb->shape == SHAPE_VALUE) {
            if ((t->col_of[d] = add_col(t, x, d, ROLE_VALUE, f[d].elem, so_kind_width(f[d].elem))) < 0) return -1;
        } else if (tb->shape == SHAPE_STRUCT) {
            if (struct_cols(t, x, d) < 0) return -1;
        } else {
            for (int i = d + 1; i < nf; i++) {
                if (f[i].parent != d) continue;
                int k = f[i].kind;
                int c = 0;
                if (scalar(k)) {
                    c = t->col_of[i] = add_col(t, x, i, ROLE_VALUE, k, so_kind_width(k));
                } else if (k == SO_KIND_ANY) { /* the span, then Value.Type() */
                    c = t->col_of[i] = add_col(t, x, i, ROLE_VALUE, k, 8);
                    if (c >= 0) c = t->type_of[i] = add_col(t, x, i, ROLE_TYPE, 0, 1);
                } else if (k == SO_KIND_MESSAGE || k == SO_KIND_LIST) {
                    c = t->present_of[i] = add_col(t, x, i, ROLE_PRESENT, 0, 1);
                } else { /* struct: one column per scalar member, inner structs' members in place */
                    c = struct_cols(t, x, i);
                }
                if (c < 0) return -1;
            }
        }
        t->err_col[x] = -1;
        if (tb->shape == SHAPE_MESSAGE) { /* a bit per direct field: ceil(direct / 64) words, at least 1 */
            int nd = 0;
            for (int i = d + 1; i < t->nf; i++) nd += t->f[i].parent == d;
            if ((t->err_col[x] = add_col(t, x, d, ROLE_ERRMASK, 0, 8 * (nd > 64 ? (nd + 63) / 64 : 1))) < 0) return -1;
        }
        if ((t->status_col[x] = add_col(t, x, d, ROLE_STATUS, 0, 1)) < 0) return -1;
        tb->ncolumns = (uint16_t)(t->nc - tb->first_column);
    }
    return 0;
}

int so_tree_layout(const so_tree_field *f, int nf, so_tree_table *tables, int *ntables, so_tree_column *cols,
                   int *ncols) {
    tree *t = (tree *)malloc(sizeof(tree));
    int rc = build(t, f, nf);
    if (rc == 0) {
        memcpy(tables, t->T, sizeof(so_tree_table) * (size_t)t->nt);
        memcpy(cols, t->C, sizeof(so_tree_column) * (size_t)t->nc);
        *ntables = t->nt;
        *ncols = t->nc;
    }
    free(t);
    return rc;
}

/* ---------------------------------------------------------------- decode */

static uint8_t *slot(tree *t, int c, uint64_t row) {
    if (!t->cols || c < 0) return NULL;
    return (uint8_t *)t->cols[c] + row * t->C[c].width;
}

static void put(tree *t, int c, uint64_t row, const void *v, int w) {
    uint8_t *p = slot(t, c, row);
    if (p) memcpy(p, v, (size_t)w);
}

static void put_u8(tree *t, int c, uint64_t row, uint8_t v) { put(t, c, row, &v, 1); }

/* Map a DecodeMessageTable error to its class (batch.c classify; msg.go:22-66). */
static uint8_t classify(so_err e) {
    if (!e) return ST_OK;
    const char *s = strstr(e, ": ");
    s = s ? s + 2 : e;
    if (!strncmp(s, "invalid type", 12)) return 1;
    if (!strncmp(s, "invalid table size", 18)) return 2;
    if (!strncmp(s, "invalid data size", 17)) return 3;
    if (!strncmp(s, "invalid table", 13)) return 4;
    return 5;
}

/* Decode<Kind>(b) of a value ending at b+len: value into dst (column element), bytes consumed
 * into *n; returns the decoder's error.  string/bytes: a span into the stream ({0,0} if empty). */
static so_err decode_kind(tree *t, int kind, const uint8_t *b, size_t len, uint8_t *dst, int *n) {
    so_err e = NULL;
    *n = 0;
    switch (kind) {
    case SO_KIND_BOOL: { int v; e = so_decode_bool(b, len, &v, n); dst[0] = (uint8_t)v; } break;
    case SO_KIND_BYTE: e = so_decode_byte(b, len, dst, n); break;
    case SO_KIND_INT16: { int16_t v; e = so_decode_int16(b, len, &v, n); memcpy(dst, &v, 2); } break;
    case SO_KIND_INT32: { int32_t v; e = so_decode_int32(b, len, &v, n); memcpy(dst, &v, 4); } break;
    case SO_KIND_INT64: { int64_t v; e = so_decode_int64(b, len, &v, n); memcpy(dst, &v, 8); } break;
    case SO_KIND_UINT16: { uint16_t v; e = so_decode_uint16(b, len, &v, n); memcpy(dst, &v, 2); } break;
    case SO_KIND_UINT32: { uint32_t v; e = so_decode_uint32(b, len, &v, n); memcpy(dst, &v, 4); } break;
    case SO_KIND_UINT64: { uint64_t v; e = so_decode_uint64(b, len, &v, n); memcpy(dst, &v, 8); } break;
    case SO_KIND_FLOAT32: { float v; e = so_decode_float32(b, len, &v, n); memcpy(dst, &v, 4); } break;
    case SO_KIND_FLOAT64: { double v; e = so_decode_float64(b, len, &v, n); memcpy(dst, &v, 8); } break;
    case SO_KIND_BIN64: e = so_decode_bin64(b, len, dst, n); break;
    case SO_KIND_BIN128: e = so_decode_bin128(b, len, dst, n); break;
    case SO_KIND_BIN256: e = so_decode_bin256(b, len, dst, n); break;
    case SO_KIND_STRING:
    case SO_KIND_BYTES: {
        size_t off = 0, vlen = 0;
        e = kind == SO_KIND_STRING ? so_decode_string(b, len, &off, &vlen, n) : so_decode_bytes(b, len, &off, &vlen, n);
        uint32_t span[2] = {0, 0};
        if (!e && vlen) {
            span[0] = (uint32_t)(b + off - t->stream);
            span[1] = (uint32_t)vlen;
        }
        memcpy(dst, span, 8);
    } break;
    }
    if (e) { /* every decoder returns the zero value with its error */
        memset(dst, 0, (size_t)so_kind_width(kind));
        *n = 0;
    }
    return e;
}

/* Zero the columns of every scalar member of struct sf (inner structs' too). */
static void zero_struct(tree *t, int sf, uint64_t row) {
    uint8_t zero[32] = {0};
    for (int j = sf + 1; j < t->nf; j++) {
        if (t->f[j].parent != sf) continue;
        if (t->f[j].kind == SO_KIND_STRUCT)
            zero_struct(t, j, row);
        else
            put(t, t->col_of[j], row, zero, so_kind_width(t->f[j].kind));
    }
}

/* Xxx.Decode(b) of a generated struct (generator/struct.go:75-113) over the value ending at
 * b+len, members = the fields whose parent is `sf`.  Members decoded from the LAST to the
 * first over b[:off]; an inner struct member through its own DecodeXxx(b[:off]) = this function
 * (n = its size); the first error stops the decode, members decoded so far keep their values.
 * Returns ST_OK, ST_INVALID_VALUE (an error), or ST_PANIC (b[len(b)-size:] with size > len),
 * and the struct's size in *nsize. */
static int decode_struct_n(tree *t, int sf, const uint8_t *b, size_t len, uint64_t row, int *nsize) {
    int mem[MAX_F], nm = 0;
    for (int j = sf + 1; j < t->nf; j++)
        if (t->f[j].parent == sf) mem[nm++] = j;
    zero_struct(t, sf, row);
    *nsize = 0;
    int ds = 0, size = 0;
    if (so_decode_struct(b, len, &ds, &size)) return ST_INVALID_VALUE;
    if (size == 0) return ST_OK;
    if ((size_t)size > len) return ST_PANIC;
    *nsize = size;
    b = b + len - (size_t)size;
    int n = size - ds;
    int64_t off = (int64_t)size - n; /* = dataSize */
    for (int k = nm - 1; k >= 0; k--) {
        const int mk = t->f[mem[k]].kind;
        int m = 0;
        if (mk == SO_KIND_STRUCT) {
            const int st = decode_struct_n(t, mem[k], b, (size_t)off, row, &m);
            if (st != ST_OK) return st;
        } else {
            uint8_t v[32];
            so_err e = decode_kind(t, mk, b, (size_t)off, v, &m);
            put(t, t->col_of[mem[k]], row, v, so_kind_width(mk));
            if (e) return ST_INVALID_VALUE;
        }
        off -= m;
    }
    return ST_OK;
}

static int decode_struct(tree *t, int sf, const uint8_t *b, size_t len, uint64_t row) {
    int n;
    return decode_struct_n(t, sf, b, len, row, &n);
}

static void decode_message(tree *t, int x, uint64_t row, const uint8_t *b, size_t len, int item);

/* One element row of list table x: GetBytes(j) already applied (p, plen) */
static void decode_element(tree *t, int x, uint64_t row, const uint8_t *p, size_t plen) {
    const so_tree_table *tb = &t->T[x];
    const int d = tb->field;
    if (tb->shape == SHAPE_MESSAGE) {
        decode_message(t, x, row, p, plen, 1);
    } else if (tb->shape == SHAPE_STRUCT) {
        put_u8(t, t->status_col[x], row, (uint8_t)decode_struct(t, d, p, plen, row));
    } else {
        uint8_t v[32];
        int m;
        so_err e = decode_kind(t, t->f[d].elem, p, plen, v, &m);
        put(t, t->col_of[d], row, v, so_kind_width(t->f[d].elem));
        put_u8(t, t->status_col[x], row, e ? ST_INVALID_VALUE : ST_OK);
    }
}

/* Zero every column of table x at `row` (and, recursively, its ONE children): what the reader
 * sees for an element Go would panic on, before the panic status is set. */
static void zero_row(tree *t, int x, uint64_t row) {
    const so_tree_table *tb = &t->T[x];
    for (int c = tb->first_column; c < tb->first_column + tb->ncolumns; c++) {
        if (t->C[c].role == ROLE_BEGIN) continue;
        uint8_t z[32] = {0};
        put(t, c, row, z, t->C[c].width);
    }
    for (int y = x + 1; y < t->nt; y++)
        if (t->T[y].parent == x) {
            if (t->T[y].rel == REL_ONE) {
                zero_row(t, y, row);
            } else {
                uint32_t b = (uint32_t)t->rows[y];
                put(t, t->begin_col[y], row, &b, 4);
            }
        }
}

/* A message row of table x over the value ending at b+len: OpenMessageErr (root, sub-message)
 * or OpenItemErr (item) — status = its error class, errors => an empty message — then every
 * field's getter, and (ERRMASK) whether each direct field's *Err getter errs (msg.go:233-463,
 * value.go:35-46, generator/struct.go:60-64). */
static void decode_message(tree *t, int x, uint64_t row, const uint8_t *b, size_t len, int item) {
    (void)item;
    so_message m;
    so_err e = so_open_message_err(b, len, &m);
    if (e) memset(&m, 0, sizeof(m));
    uint8_t st = classify(e);
    uint64_t errs[MAX_F / 64] = {0};
    int kth = 0;
    const int d = t->T[x].field;
    for (int i = d + 1; i < t->nf; i++) {
        if (t->f[i].parent != d) continue;
        const so_tree_field *fi = &t->f[i];
        const int k = fi->kind;
        const int bit = kth++;
        int bad = 0;
        size_t rl = 0;
        const uint8_t *raw = so_message_field_raw(&m, fi->tag, &rl);
        if (scalar(k)) {
            uint8_t v[32];
            int n;
            bad = decode_kind(t, k, raw, rl, v, &n) != NULL; /* m.<Kind>(tag) swallows it; <Kind>Err not */
            put(t, t->col_of[i], row, v, so_kind_width(k));
        } else if (k == SO_KIND_STRUCT) {
            const int sst = decode_struct(t, i, raw, rl, row); /* DecodeXxx(m.FieldRaw(tag)) */
            if (sst == ST_PANIC) st = ST_PANIC;
            bad = sst != ST_OK;
        } else if (k == SO_KIND_ANY) {
            /* OpenValue(bytes[:end]) (value.go:18-31): nil on error or len < n; Go slices
             * b[len(b)-n:] with n < 0 (DecodeTypeSize's struct quirk) and panics; OpenValueErr
             * errs with DecodeTypeSize only (value.go:35-46) */
            uint32_t span[2] = {0, 0};
            uint8_t ty;
            int n = 0;
            if (rl) {
                if (so_decode_type_size(raw, rl, &ty, &n)) {
                    bad = 1;
                } else if (n < 0) {
                    st = ST_PANIC;
                } else if ((size_t)n <= rl && n > 0) {
                    span[0] = (uint32_t)(raw + rl - (size_t)n - t->stream);
                    span[1] = (uint32_t)n;
                }
            }
            put(t, t->col_of[i], row, span, 8);
            /* Value.Type() = DecodeType(v) (value.go:115-119): the last byte, Undefined for nil */
            put_u8(t, t->type_of[i], row, span[1] ? t->stream[span[0] + span[1] - 1] : 0);
        } else if (k == SO_KIND_MESSAGE) {
            put_u8(t, t->present_of[i], row, (uint8_t)so_message_has_field(&m, fi->tag));
            so_message sm;
            bad = so_open_message_err(raw, rl, &sm) != NULL; /* MessageErr(tag) */
            decode_message(t, t->table_of[i], row, raw, rl, 0);
        } else { /* list */
            const int y = t->table_of[i];
            put_u8(t, t->present_of[i], row, (uint8_t)so_message_has_field(&m, fi->tag));
            so_list l;
            if (so_open_list_err(raw, rl, &l)) { /* m.List(tag): errors => empty; ListErr errs */
                memset(&l, 0, sizeof(l));
                bad = 1;
            }
            const int cnt = so_list_len(&l);
            uint32_t b0 = (uint32_t)t->rows[y];
            put(t, t->begin_col[y], row, &b0, 4);
            for (int j = 0; j < cnt; j++) {
                const uint64_t er = t->rows[y]++;
                const uint8_t *p;
                size_t plen;
                if (so_list_get_bytes(&l, j, &p, &plen) < 0) { /* Go panics (start > end) */
                    zero_row(t, y, er);
                    put_u8(t, t->status_col[y], er, ST_PANIC);
                    continue;
                }
                decode_element(t, y, er, p, plen);
            }
        }
        if (bad) errs[bit >> 6] |= 1ull << (bit & 63);
    }
    put(t, t->err_col[x], row, errs, t->C[t->err_col[x]].width);
    put_u8(t, t->status_col[x], row, st);
}

/* The generated reader over n messages: record r = [ends[r-1], ends[r]) of the stream, or
 * (spans != NULL) the value span r — m.Field(tag).Message() = OpenMessage(value)
 * (internal/types/value.go:318-321); a span past the stream is a Go panic. */
static int decode_tree(const so_tree_field *f, int nf, const uint8_t *stream, uint64_t stream_len, const uint64_t *ends,
                       const uint32_t *spans, uint64_t n, void *const *columns, uint64_t *rows) {
    tree *t = (tree *)malloc(sizeof(tree));
    if (build(t, f, nf)) {
        free(t);
        return -1;
    }
    t->stream = stream;
    t->cols = columns;
    t->rows[0] = n;
    for (uint64_t r = 0; r < n; r++) {
        if (spans) {
            const uint64_t off = spans[2 * r], len = spans[2 * r + 1];
            const int past = off + len > stream_len;
            decode_message(t, 0, r, past ? stream : stream + off, past ? 0 : (size_t)len, 0);
            if (past) put_u8(t, t->status_col[0], r, ST_PANIC);
        } else {
            const uint64_t s = r ? ends[r - 1] : 0;
            decode_message(t, 0, r, stream + s, (size_t)(ends[r] - s), 0);
        }
    }
    /* CSR closers: begin[parent rows] = total */
    for (int x = 1; x < t->nt; x++) {
        if (t->T[x].rel == REL_ONE) t->rows[x] = t->rows[t->T[x].parent];
    }
    for (int x = 1; x < t->nt; x++) {
        if (t->T[x].rel != REL_MANY) continue;
        uint32_t tot = (uint32_t)t->rows[x];
        put(t, t->begin_col[x], t->rows[t->T[x].parent], &tot, 4);
    }
    memcpy(rows, t->rows, sizeof(uint64_t) * (size_t)t->nt);
    free(t);
    return 0;
}

int so_decode_tree_batch(const so_tree_field *f, int nf, const uint8_t *stream, const uint64_t *ends, uint64_t n,
                         void *const *columns, uint64_t *rows) {
    return decode_tree(f, nf, stream, 0, ends, NULL, n, columns, rows);
}

int so_decode_tree_spans(const so_tree_field *f, int nf, const uint8_t *stream, uint64_t stream_len,
                         const uint32_t *spans, uint64_t n, void *const *columns, uint64_t *rows) {
    return decode_tree(f, nf, stream, stream_len, NULL, spans, n, columns, rows);
}

/* Value.<Kind>Err() over value spans (internal/types/value.go:120-310): Decode<Kind> of the
 * span's bytes; err = 1 on a decoder error, 2 for a span past the stream (a Go panic). */
int so_decode_values(int kind, const uint8_t *stream, uint64_t stream_len, const uint32_t *spans, uint64_t n,
                     uint8_t *out, uint8_t *err) {
    if (!scalar(kind)) return -1;
    tree *t = (tree *)calloc(1, sizeof(tree));
    t->stream = stream;
    const int w = so_kind_width(kind);
    for (uint64_t r = 0; r < n; r++) {
        const uint64_t off = spans[2 * r], len = spans[2 * r + 1];
        const int past = off + len > stream_len;
        int m;
        so_err e = decode_kind(t, kind, past ? stream : stream + off, past ? 0 : (size_t)len, out + r * (uint64_t)w, &m);
        err[r] = past ? 2 : (e ? 1 : 0);
    }
    free(t);
    return 0;
}

/* ---------------------------------------------------------------- encode */

static const uint8_t *cell(tree *t, int c, uint64_t row) {
    return (const uint8_t *)t->cols[c] + row * t->C[c].width;
}

/* The member list of struct sf for the Writer's struct calls: pre-order (an inner struct is
 * SO_KIND_STRUCT followed by its members; nmem[] = direct member counts of the structs). */
static void struct_members(tree *t, int sf, uint64_t row, uint8_t *kinds, const uint8_t **vals, const uint8_t **heaps,
                           int *nmem, int *nm) {
    for (int j = sf + 1; j < t->nf; j++) {
        if (t->f[j].parent != sf) continue;
        const int at = (*nm)++;
        kinds[at] = t->f[j].kind;
        nmem[at] = 0;
        if (t->f[j].kind == SO_KIND_STRUCT) {
            vals[at] = NULL;
            heaps[at] = NULL;
            for (int q = j + 1; q < t->nf; q++) nmem[at] += t->f[q].parent == j;
            struct_members(t, j, row, kinds, vals, heaps, nmem, nm);
        } else {
            const int c = t->col_of[j];
            vals[at] = cell(t, c, row);
            heaps[at] = t->heaps ? t->heaps[c] : NULL;
        }
    }
}

static so_err write_struct(tree *t, so_writer *w, int sf, uint64_t row, int field, uint16_t tag) {
    uint8_t kinds[MAX_F];
    const uint8_t *vals[MAX_F], *heaps[MAX_F];
    int nmem[MAX_F], nm = 0, top = 0;
    for (int j = sf + 1; j < t->nf; j++) top += t->f[j].parent == sf;
    struct_members(t, sf, row, kinds, vals, heaps, nmem, &nm);
    return field ? so_field_struct_tree(w, tag, top, nm, kinds, vals, heaps, nmem)
                 : so_elem_struct_tree(w, top, nm, kinds, vals, heaps, nmem);
}

static uint32_t begin_at(tree *t, int y, uint64_t row) {
    uint32_t v;
    memcpy(&v, cell(t, t->begin_col[y], row), 4);
    return v;
}

static void write_message(tree *t, so_writer *w, int x, uint64_t row) {
    const int d = t->T[x].field;
    for (int i = d + 1; i < t->nf; i++) {
        if (t->f[i].parent != d) continue;
        const so_tree_field *fi = &t->f[i];
        const int k = fi->kind, c = t->col_of[i];
        if (scalar(k)) {
            so_field_value(w, fi->tag, k, cell(t, c, row), t->heaps ? t->heaps[c] : NULL);
        } else if (k == SO_KIND_STRUCT) {
            write_struct(t, w, i, row, 1, fi->tag);
        } else if (k == SO_KIND_ANY) {
            uint32_t span[2];
            memcpy(span, cell(t, c, row), 8);
            if (span[1]) so_field_any(w, fi->tag, t->heaps[c] + span[0], span[1]);
        } else if (k == SO_KIND_MESSAGE) {
            if (!cell(t, t->present_of[i], row)[0]) continue;
            so_field_begin_message(w, fi->tag);
            write_message(t, w, t->table_of[i], row);
            so_writer_end(w, NULL, NULL);
        } else { /* list */
            if (!cell(t, t->present_of[i], row)[0]) continue;
            const int y = t->table_of[i];
            const so_tree_table *tb = &t->T[y];
            so_field_begin_list(w, fi->tag);
            const uint32_t j0 = begin_at(t, y, row), j1 = begin_at(t, y, row + 1);
            for (uint32_t j = j0; j < j1; j++) {
                if (tb->shape == SHAPE_MESSAGE) {
                    so_elem_begin_message(w);
                    write_message(t, w, y, j);
                    so_writer_end(w, NULL, NULL);
                } else if (tb->shape == SHAPE_STRUCT) {
                    write_struct(t, w, i, j, 0, 0);
                } else {
                    const int vc = t->col_of[i];
                    so_elem_value(w, fi->elem, cell(t, vc, j), t->heaps ? t->heaps[vc] : NULL);
                }
            }
            so_writer_end(w, NULL, NULL);
        }
    }
}

int so_encode_tree_batch(const so_tree_field *f, int nf, const void *const *columns, const uint8_t *const *heaps,
                         uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *ends) {
    tree *t = (tree *)malloc(sizeof(tree));
    if (build(t, f, nf)) {
        free(t);
        return -1;
    }
    t->cols = (void *const *)columns;
    t->heaps = heaps;
    so_buf buf;
    so_buf_init_fixed(&buf, out, (size_t)out_cap);
    so_writer *w = so_writer_new(&buf);
    int rc = 0;
    for (uint64_t r = 0; r < n; r++) {
        so_writer_reset(w, &buf);
        so_writer_begin_message(w);
        write_message(t, w, 0, r);
        if (so_writer_end(w, NULL, NULL)) {
            rc = -1;
            break;
        }
        if (buf.overflow) {
            rc = -2;
            break;
        }
        ends[r] = buf.len;
    }
    so_writer_free(w);
    free(t);
    return rc;
}
