/*
 * batch.c — the reference's per-record loops over a batch of records, used as the
 * parity oracle for the bulk GPU kernels and as the CPU baseline in bench.py.
 * TEST INFRASTRUCTURE (oracle).
 *
 *   decode: BenchmarkReadMessage pattern, internal/bench/parse_test.go:48-111
 *           (OpenMessageErr + one typed getter per field)
 *   encode: BenchmarkWrite_* pattern, internal/bench/write_test.go:16-78
 *           (NewMessageWriterBuffer + one FieldWriter call per field + Build)
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "spec_oracle.h"

/* Record status codes, shared with include/spec_amd.h SPEC_STATUS_*. */
enum {
    ST_OK = 0,
    ST_INVALID_TYPE = 1,
    ST_INVALID_TABLE_SIZE = 2,
    ST_INVALID_DATA_SIZE = 3,
    ST_INVALID_TABLE = 4,
    ST_INVALID_DATA = 5,
    ST_PANIC = 6, /* the reference would panic (malformed list table) */
};

/* Map a DecodeMessageTable / DecodeListTable error to its class (msg.go:22-66). */
static uint8_t classify(so_err e) {
    if (!e) return ST_OK;
    const char *s = strstr(e, ": ");
    s = s ? s + 2 : e;
    if (!strncmp(s, "invalid type", 12)) return ST_INVALID_TYPE;
    if (!strncmp(s, "invalid table size", 18)) return ST_INVALID_TABLE_SIZE;
    if (!strncmp(s, "invalid data size", 17)) return ST_INVALID_DATA_SIZE;
    if (!strncmp(s, "invalid table", 13)) return ST_INVALID_TABLE;
    if (!strncmp(s, "invalid data", 12)) return ST_INVALID_DATA;
    return ST_INVALID_DATA;
}

int so_kind_width(int kind) {
    switch (kind) {
    case SO_KIND_BOOL: case SO_KIND_BYTE: return 1;
    case SO_KIND_INT16: case SO_KIND_UINT16: return 2;
    case SO_KIND_INT32: case SO_KIND_UINT32: case SO_KIND_FLOAT32: return 4;
    case SO_KIND_INT64: case SO_KIND_UINT64: case SO_KIND_FLOAT64: case SO_KIND_BIN64: return 8;
    case SO_KIND_BIN128: return 16;
    case SO_KIND_BIN256: return 32;
    case SO_KIND_STRING: case SO_KIND_BYTES: return 8;
    }
    return 0;
}

static inline uint64_t rec_start(const uint64_t *ends, uint64_t r) { return r ? ends[r - 1] : 0; }

/* Decode one field of one record into its column slot via the typed getter. */
static void getter(const so_message *m, const uint8_t *stream, uint16_t tag, int kind, uint8_t *dst) {
    switch (kind) {
    case SO_KIND_BOOL: dst[0] = (uint8_t)so_message_bool(m, tag); break;
    case SO_KIND_BYTE: dst[0] = so_message_byte(m, tag); break;
    case SO_KIND_INT16: { int16_t v = so_message_int16(m, tag); memcpy(dst, &v, 2); } break;
    case SO_KIND_INT32: { int32_t v = so_message_int32(m, tag); memcpy(dst, &v, 4); } break;
    case SO_KIND_INT64: { int64_t v = so_message_int64(m, tag); memcpy(dst, &v, 8); } break;
    case SO_KIND_UINT16: { uint16_t v = so_message_uint16(m, tag); memcpy(dst, &v, 2); } break;
    case SO_KIND_UINT32: { uint32_t v = so_message_uint32(m, tag); memcpy(dst, &v, 4); } break;
    case SO_KIND_UINT64: { uint64_t v = so_message_uint64(m, tag); memcpy(dst, &v, 8); } break;
    case SO_KIND_FLOAT32: { float v = so_message_float32(m, tag); memcpy(dst, &v, 4); } break;
    case SO_KIND_FLOAT64: { double v = so_message_float64(m, tag); memcpy(dst, &v, 8); } break;
    case SO_KIND_BIN64: so_message_bin64(m, tag, dst); break;
    case SO_KIND_BIN128: so_message_bin128(m, tag, dst); break;
    case SO_KIND_BIN256: so_message_bin256(m, tag, dst); break;
    case SO_KIND_STRING:
    case SO_KIND_BYTES: {
        size_t len;
        const uint8_t *p = kind == SO_KIND_STRING ? so_message_string(m, tag, &len) : so_message_bytes(m, tag, &len);
        /* empty or absent => {0, 0}: a zero-length view carries no offset */
        uint32_t span[2] = {p && len ? (uint32_t)(p - stream) : 0u, p ? (uint32_t)len : 0u};
        memcpy(dst, span, 8);
    } break;
    }
}

typedef struct {
    int nfields;
    const uint16_t *tags;
    const uint8_t *kinds;
    const uint8_t *stream;
    const uint64_t *ends;
    uint64_t lo, hi;
    void *const *columns;
    uint8_t *status;
} decode_job;

static void *decode_range(void *arg) {
    decode_job *j = (decode_job *)arg;
    int widths[1024];
    if (j->nfields > 1024) return NULL;
    for (int f = 0; f < j->nfields; f++) widths[f] = so_kind_width(j->kinds[f]);
    for (uint64_t r = j->lo; r < j->hi; r++) {
        uint64_t s = rec_start(j->ends, r);
        so_message m;
        so_err e = so_open_message_err(j->stream + s, (size_t)(j->ends[r] - s), &m);
        j->status[r] = classify(e);
        for (int f = 0; f < j->nfields; f++) {
            uint8_t *dst = (uint8_t *)j->columns[f] + r * (uint64_t)widths[f];
            getter(&m, j->stream, j->tags[f], j->kinds[f], dst);
        }
    }
    return NULL;
}

int so_decode_flat_batch(int nfields, const uint16_t *tags, const uint8_t *kinds,
                         const uint8_t *stream, const uint64_t *ends, uint64_t n,
                         void *const *columns, uint8_t *status, int nthreads) {
    if (nfields > 1024) return -1;
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
    decode_job jobs[256];
    pthread_t th[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        decode_job j = {nfields, tags, kinds, stream, ends, n * (uint64_t)t / (uint64_t)nthreads,
                        n * (uint64_t)(t + 1) / (uint64_t)nthreads, columns, status};
        jobs[t] = j;
    }
    if (nthreads == 1) {
        decode_range(&jobs[0]);
        return 0;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, decode_range, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* Write one field through the FieldWriter method for its kind. */
static so_err write_field(so_writer *w, uint16_t tag, int kind, const uint8_t *src, const uint8_t *heap) {
    switch (kind) {
    case SO_KIND_BOOL: return so_field_bool(w, tag, src[0] != 0);
    case SO_KIND_BYTE: return so_field_byte(w, tag, src[0]);
    case SO_KIND_INT16: { int16_t v; memcpy(&v, src, 2); return so_field_int16(w, tag, v); }
    case SO_KIND_INT32: { int32_t v; memcpy(&v, src, 4); return so_field_int32(w, tag, v); }
    case SO_KIND_INT64: { int64_t v; memcpy(&v, src, 8); return so_field_int64(w, tag, v); }
    case SO_KIND_UINT16: { uint16_t v; memcpy(&v, src, 2); return so_field_uint16(w, tag, v); }
    case SO_KIND_UINT32: { uint32_t v; memcpy(&v, src, 4); return so_field_uint32(w, tag, v); }
    case SO_KIND_UINT64: { uint64_t v; memcpy(&v, src, 8); return so_field_uint64(w, tag, v); }
    case SO_KIND_FLOAT32: { float v; memcpy(&v, src, 4); return so_field_float32(w, tag, v); }
    case SO_KIND_FLOAT64: { double v; memcpy(&v, src, 8); return so_field_float64(w, tag, v); }
    case SO_KIND_BIN64: return so_field_bin64(w, tag, src);
    case SO_KIND_BIN128: return so_field_bin128(w, tag, src);
    case SO_KIND_BIN256: return so_field_bin256(w, tag, src);
    case SO_KIND_STRING:
    case SO_KIND_BYTES: {
        uint32_t span[2];
        memcpy(span, src, 8);
        const uint8_t *p = heap + span[0];
        return kind == SO_KIND_STRING ? so_field_string(w, tag, (const char *)p, span[1])
                                      : so_field_bytes(w, tag, p, span[1]);
    }
    }
    return "unknown kind";
}

/* Records [r0, r1) written back to back into out (ends[r] relative to out). */
static int encode_flat_range(int nfields, const uint16_t *tags, const uint8_t *kinds, const void *const *columns,
                             const uint8_t *const *heaps, uint64_t r0, uint64_t r1, uint8_t *out, uint64_t out_cap,
                             uint64_t *ends) {
    so_buf buf;
    so_buf_init_fixed(&buf, out, (size_t)out_cap);
    so_writer *w = so_writer_new(&buf);
    int widths[1024];
    if (nfields > 1024) return -1;
    for (int f = 0; f < nfields; f++) widths[f] = so_kind_width(kinds[f]);
    int rc = 0;
    for (uint64_t r = r0; r < r1; r++) {
        so_writer_reset(w, &buf);
        so_writer_begin_message(w);
        for (int f = 0; f < nfields; f++) {
            const uint8_t *src = (const uint8_t *)columns[f] + r * (uint64_t)widths[f];
            write_field(w, tags[f], kinds[f], src, heaps ? heaps[f] : NULL);
        }
        so_err e = so_writer_end(w, NULL, NULL);
        if (e) {
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
    return rc;
}

int so_encode_flat_batch(int nfields, const uint16_t *tags, const uint8_t *kinds,
                         const void *const *columns, const uint8_t *const *heaps, uint64_t n,
                         uint8_t *out, uint64_t out_cap, uint64_t *ends) {
    return encode_flat_range(nfields, tags, kinds, columns, heaps, 0, n, out, out_cap, ends);
}

/* ---- the CPU baseline on several host threads (bench.py): contiguous record shards, one per
 * thread, each with its own output region out + t * (out_cap / nthreads) and ends relative to
 * it — what nthreads goroutines each running the reference's loop with their own buffer do ---- */

typedef struct {
    int kind; /* 0 flat encode, 1 nested encode, 2 nested decode */
    uint64_t r0, r1;
    uint8_t *out;
    uint64_t cap;
    int rc;
    /* flat */
    int nfields;
    const uint16_t *tags;
    const uint8_t *kinds;
    const void *const *columns;
    const uint8_t *const *heaps;
    /* nested: id, seq, name, name_heap, item_begin, key, value, label, label_heap; decode adds
     * stream, ends and the output columns */
    const void *nv[9];
    const uint8_t *stream;
    const uint64_t *ends_in;
    void *dv[8];
    uint64_t *ends;
} mt_job;

static int encode_nested_range(const uint8_t *id, const int64_t *seq, const uint32_t *name, const uint8_t *name_heap,
                               const uint32_t *item_begin, const int32_t *key, const double *value,
                               const uint32_t *label, const uint8_t *label_heap, uint64_t r0, uint64_t r1,
                               uint8_t *out, uint64_t out_cap, uint64_t *ends);
static void decode_nested_range(const uint8_t *stream, const uint64_t *ends, uint64_t r0, uint64_t r1,
                                const uint32_t *item_begin, uint8_t *id, int64_t *seq, uint32_t *name, int32_t *key,
                                double *value, uint32_t *label, uint8_t *item_status, uint8_t *status);

static void *mt_run(void *arg) {
    mt_job *j = (mt_job *)arg;
    if (j->kind == 0) {
        j->rc = encode_flat_range(j->nfields, j->tags, j->kinds, j->columns, j->heaps, j->r0, j->r1, j->out, j->cap,
                                  j->ends);
    } else if (j->kind == 1) {
        j->rc = encode_nested_range(j->nv[0], j->nv[1], j->nv[2], j->nv[3], j->nv[4], j->nv[5], j->nv[6], j->nv[7],
                                    j->nv[8], j->r0, j->r1, j->out, j->cap, j->ends);
    } else {
        decode_nested_range(j->stream, j->ends_in, j->r0, j->r1, j->nv[4], j->dv[0], j->dv[1], j->dv[2], j->dv[3],
                            j->dv[4], j->dv[5], j->dv[6], j->dv[7]);
        j->rc = 0;
    }
    return NULL;
}

static int mt_launch(mt_job *proto, uint64_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
    mt_job jobs[256];
    pthread_t th[256];
    const uint64_t share = proto->cap / (uint64_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = *proto;
        jobs[t].r0 = n * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].r1 = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
        jobs[t].out = proto->out ? proto->out + share * (uint64_t)t : NULL;
        jobs[t].cap = share;
    }
    if (nthreads == 1) {
        mt_run(&jobs[0]);
        return jobs[0].rc;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, mt_run, &jobs[t]);
    int rc = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    return rc;
}

int so_encode_flat_batch_mt(int nfields, const uint16_t *tags, const uint8_t *kinds, const void *const *columns,
                            const uint8_t *const *heaps, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *ends,
                            int nthreads) {
    mt_job j;
    memset(&j, 0, sizeof(j));
    j.kind = 0;
    j.nfields = nfields;
    j.tags = tags;
    j.kinds = kinds;
    j.columns = columns;
    j.heaps = heaps;
    j.out = out;
    j.cap = out_cap;
    j.ends = ends;
    return mt_launch(&j, n, nthreads);
}

int so_encode_nested_batch_mt(const uint8_t *id, const int64_t *seq, const uint32_t *name, const uint8_t *name_heap,
                              const uint32_t *item_begin, const int32_t *key, const double *value,
                              const uint32_t *label, const uint8_t *label_heap, uint64_t n, uint8_t *out,
                              uint64_t out_cap, uint64_t *ends, int nthreads) {
    mt_job j;
    memset(&j, 0, sizeof(j));
    j.kind = 1;
    const void *nv[9] = {id, seq, name, name_heap, item_begin, key, value, label, label_heap};
    memcpy(j.nv, nv, sizeof(nv));
    j.out = out;
    j.cap = out_cap;
    j.ends = ends;
    return mt_launch(&j, n, nthreads);
}

int so_decode_nested_batch_mt(const uint8_t *stream, const uint64_t *ends, uint64_t n, const uint32_t *item_begin,
                              uint8_t *id, int64_t *seq, uint32_t *name, int32_t *key, double *value, uint32_t *label,
                              uint8_t *item_status, uint8_t *status, int nthreads) {
    mt_job j;
    memset(&j, 0, sizeof(j));
    j.kind = 2;
    j.stream = stream;
    j.ends_in = ends;
    j.nv[4] = item_begin;
    void *dv[8] = {id, seq, name, key, value, label, item_status, status};
    memcpy(j.dv, dv, sizeof(dv));
    return mt_launch(&j, n, nthreads);
}

/* ---- Nested (config 4) ---- */

int so_encode_nested_batch(const uint8_t *id, const int64_t *seq, const uint32_t *name,
                           const uint8_t *name_heap, const uint32_t *item_begin,
                           const int32_t *key, const double *value, const uint32_t *label,
                           const uint8_t *label_heap, uint64_t n, uint8_t *out,
                           uint64_t out_cap, uint64_t *ends) {
    return encode_nested_range(id, seq, name, name_heap, item_begin, key, value, label, label_heap, 0, n, out,
                               out_cap, ends);
}

static int encode_nested_range(const uint8_t *id, const int64_t *seq, const uint32_t *name, const uint8_t *name_heap,
                               const uint32_t *item_begin, const int32_t *key, const double *value,
                               const uint32_t *label, const uint8_t *label_heap, uint64_t r0, uint64_t r1,
                               uint8_t *out, uint64_t out_cap, uint64_t *ends) {
    so_buf buf;
    so_buf_init_fixed(&buf, out, (size_t)out_cap);
    so_writer *w = so_writer_new(&buf);
    int rc = 0;
    for (uint64_t r = r0; r < r1; r++) {
        so_writer_reset(w, &buf);
        so_writer_begin_message(w);
        so_field_bin128(w, 1, id + 16 * r);
        so_field_int64(w, 2, seq[r]);
        so_field_string(w, 3, (const char *)name_heap + name[2 * r], name[2 * r + 1]);
        so_field_begin_list(w, 4); /* FieldWriter.List() */
        for (uint32_t i = item_begin[r]; i < item_begin[r + 1]; i++) {
            so_elem_begin_message(w); /* MessageListWriter.Add() */
            so_field_int32(w, 1, key[i]);
            so_field_float64(w, 2, value[i]);
            so_field_string(w, 3, (const char *)label_heap + label[2 * i], label[2 * i + 1]);
            so_writer_end(w, NULL, NULL); /* item End() */
        }
        so_writer_end(w, NULL, NULL); /* list End() */
        so_err e = so_writer_end(w, NULL, NULL); /* Build() */
        if (e) {
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
    return rc;
}

int so_decode_nested_counts(const uint8_t *stream, const uint64_t *ends, uint64_t n,
                            uint32_t *counts, uint8_t *status) {
    for (uint64_t r = 0; r < n; r++) {
        uint64_t s = rec_start(ends, r);
        so_message m;
        so_err e = so_open_message_err(stream + s, (size_t)(ends[r] - s), &m);
        status[r] = classify(e);
        so_list l;
        so_message_list(&m, 4, &l);
        counts[r] = (uint32_t)so_list_len(&l);
    }
    return 0;
}

int so_decode_nested_batch(const uint8_t *stream, const uint64_t *ends, uint64_t n,
                           const uint32_t *item_begin, uint8_t *id, int64_t *seq,
                           uint32_t *name, int32_t *key, double *value, uint32_t *label,
                           uint8_t *item_status, uint8_t *status) {
    decode_nested_range(stream, ends, 0, n, item_begin, id, seq, name, key, value, label, item_status, status);
    return 0;
}

/* Per record: OpenMessageErr, the outer getters, MessageList Len/Get + the item getters
 * (list_msg.go:88-92); items land at item_begin[r] + i. */
static void decode_nested_range(const uint8_t *stream, const uint64_t *ends, uint64_t r0, uint64_t r1,
                                const uint32_t *item_begin, uint8_t *id, int64_t *seq, uint32_t *name, int32_t *key,
                                double *value, uint32_t *label, uint8_t *item_status, uint8_t *status) {
    for (uint64_t r = r0; r < r1; r++) {
        uint64_t s = rec_start(ends, r);
        so_message m;
        so_err e = so_open_message_err(stream + s, (size_t)(ends[r] - s), &m);
        status[r] = classify(e);
        so_message_bin128(&m, 1, id + 16 * r);
        seq[r] = so_message_int64(&m, 2);
        size_t len;
        const uint8_t *p = so_message_string(&m, 3, &len);
        name[2 * r] = p && len ? (uint32_t)(p - stream) : 0;
        name[2 * r + 1] = p ? (uint32_t)len : 0;
        so_list l;
        so_message_list(&m, 4, &l);
        uint32_t cnt = (uint32_t)so_list_len(&l);
        for (uint32_t i = 0; i < cnt; i++) {
            uint32_t o = item_begin[r] + i;
            const uint8_t *ib;
            size_t ilen;
            so_message it;
            if (so_list_get_bytes(&l, (int)i, &ib, &ilen) < 0) {
                memset(&it, 0, sizeof(it));
                item_status[o] = ST_PANIC;
            } else {
                item_status[o] = classify(so_open_message_err(ib, ilen, &it));
            }
            key[o] = so_message_int32(&it, 1);
            value[o] = so_message_float64(&it, 2);
            const uint8_t *q = so_message_string(&it, 3, &len);
            label[2 * o] = q && len ? (uint32_t)(q - stream) : 0;
            label[2 * o + 1] = q ? (uint32_t)len : 0;
        }
    }
}

/* ---- ParseMessage over a batch (spec_parse_messages semantics) ---- */
int so_parse_batch(const uint8_t *stream, const uint64_t *ends, uint64_t n, uint32_t head, uint8_t *status,
                   uint32_t *sizes) {
    for (uint64_t r = 0; r < n; r++) {
        uint64_t s = (r ? ends[r - 1] : 0) + head;
        uint64_t e = ends[r] < s ? s : ends[r];
        so_message m;
        sizes[r] = 0;
        so_err err = so_open_message_err(stream + s, (size_t)(e - s), &m);
        if (err) {
            status[r] = classify(err);
            continue;
        }
        int size = 0;
        err = so_parse_message(stream + s, (size_t)(e - s), &m, &size);
        if (err) {
            status[r] = strstr(err, "index out of range") ? ST_PANIC : 7;
            continue;
        }
        status[r] = 0;
        sizes[r] = (uint32_t)size;
    }
    return 0;
}

/* spec_parse_batch semantics: root 0 = ParseMessage (so_parse_batch), 1 = ParseList
 * (internal/types/list.go:35-53: DecodeListTable's error class, then ParseValue on every non-empty
 * element), 2 = ParseValue (internal/types/value.go:49-113: any error => 7, INVALID_VALUE; an
 * empty value is "unsupported type 0").  Nested errors => 7, Go panics => ST_PANIC; sizes[r] =
 * the parsed size (ParseValue's n). */
int so_parse_batch_root(int root, const uint8_t *stream, const uint64_t *ends, uint64_t n, uint32_t head,
                        uint8_t *status, uint32_t *sizes) {
    if (root == 0) return so_parse_batch(stream, ends, n, head, status, sizes);
    for (uint64_t r = 0; r < n; r++) {
        uint64_t s = (r ? ends[r - 1] : 0) + head;
        uint64_t e = ends[r] < s ? s : ends[r];
        const uint8_t *b = stream + s;
        const size_t len = (size_t)(e - s);
        sizes[r] = 0;
        so_err err = NULL;
        int size = 0;
        if (root == 1) {
            so_list l;
            err = so_open_list_err(b, len, &l);
            if (err) {
                status[r] = classify(err);
                continue;
            }
            err = so_parse_list(b, len, &size);
        } else {
            err = so_parse_value(b, len, &size);
        }
        if (err) {
            status[r] = strstr(err, "index out of range") ? ST_PANIC : 7;
            continue;
        }
        status[r] = 0;
        sizes[r] = (uint32_t)size;
    }
    return 0;
}

/* mpx frame read loop (mpx/conn_reader.go:179-194, connReader.read): io.ReadFull of the 4-byte
 * head, size = binary.BigEndian.Uint32(head), then io.ReadFull of size bytes — repeated over a
 * received buffer.  A read that would run past len stops the loop (ReadFull would block for
 * more bytes): ends[k] = offset just past frame k's message, *consumed = ends of the last
 * complete frame.  Returns the frame count, or -1 when more than cap frames are complete
 * (ends[0, cap) written). */
long long so_frames_read(const uint8_t *buf, uint64_t len, uint64_t *ends, uint64_t cap, uint64_t *consumed) {
    uint64_t p = 0, k = 0;
    *consumed = 0;
    while (p + 4 <= len) {
        const uint64_t size = ((uint64_t)buf[p] << 24) | ((uint64_t)buf[p + 1] << 16) | ((uint64_t)buf[p + 2] << 8) |
                              (uint64_t)buf[p + 3];
        if (p + 4 + size > len) break; /* incomplete message: the next read continues it */
        if (k == cap) return -1;
        p += 4 + size;
        ends[k++] = p;
        *consumed = p;
    }
    return (long long)k;
}

/* The *Err getters (internal/types/msg.go:233-459) of every field of every record:
 * errmask[r] bit f = m.<Kind>Err(tag_f) returns an error (decode.Decode<Kind>(m.field(tag)):
 * an absent field is nil and decodes without error).  More than 64 fields: ceil(nfields / 64)
 * words per record, word-major (errmask[c * n + r] bit f = field 64 c + f), as
 * spec_decode_flat_errors lays them out. */
int so_decode_flat_errors(int nfields, const uint16_t *tags, const uint8_t *kinds, const uint8_t *stream,
                          const uint64_t *ends, uint64_t n, uint64_t *errmask) {
    for (uint64_t r = 0; r < n; r++) {
        const uint64_t s = rec_start(ends, r);
        so_message m;
        if (so_open_message_err(stream + s, (size_t)(ends[r] - s), &m)) memset(&m, 0, sizeof(m));
        uint64_t bits = 0;
        for (int f = 0; f < nfields; f++) {
            if (f && (f & 63) == 0) { /* the next word */
                errmask[(uint64_t)(f / 64 - 1) * n + r] = bits;
                bits = 0;
            }
            size_t len;
            const uint8_t *b = so_message_field_raw(&m, tags[f], &len);
            int k;
            so_err e = NULL;
            union {
                int i; uint8_t u8; int16_t i16; int32_t i32; int64_t i64; uint16_t u16; uint32_t u32; uint64_t u64;
                float f32; double f64; uint8_t bin[32];
            } v;
            size_t off, vlen;
            switch (kinds[f]) {
            case SO_KIND_BOOL: e = so_decode_bool(b, len, &v.i, &k); break;
            case SO_KIND_BYTE: e = so_decode_byte(b, len, &v.u8, &k); break;
            case SO_KIND_INT16: e = so_decode_int16(b, len, &v.i16, &k); break;
            case SO_KIND_INT32: e = so_decode_int32(b, len, &v.i32, &k); break;
            case SO_KIND_INT64: e = so_decode_int64(b, len, &v.i64, &k); break;
            case SO_KIND_UINT16: e = so_decode_uint16(b, len, &v.u16, &k); break;
            case SO_KIND_UINT32: e = so_decode_uint32(b, len, &v.u32, &k); break;
            case SO_KIND_UINT64: e = so_decode_uint64(b, len, &v.u64, &k); break;
            case SO_KIND_FLOAT32: e = so_decode_float32(b, len, &v.f32, &k); break;
            case SO_KIND_FLOAT64: e = so_decode_float64(b, len, &v.f64, &k); break;
            case SO_KIND_BIN64: e = so_decode_bin64(b, len, v.bin, &k); break;
            case SO_KIND_BIN128: e = so_decode_bin128(b, len, v.bin, &k); break;
            case SO_KIND_BIN256: e = so_decode_bin256(b, len, v.bin, &k); break;
            case SO_KIND_STRING: e = so_decode_string(b, len, &off, &vlen, &k); break;
            case SO_KIND_BYTES: e = so_decode_bytes(b, len, &off, &vlen, &k); break;
            }
            if (e) bits |= 1ull << (f & 63);
        }
        errmask[(uint64_t)(nfields > 0 ? (nfields - 1) / 64 : 0) * n + r] = bits;
    }
    return 0;
}
