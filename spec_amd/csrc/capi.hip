// capi.hip — the C ABI of libspec_amd.so (include/spec_amd.h): argument validation, schema
// preprocessing (table order) and kernel launches.  No host sync on any path.
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/spec_amd.h"
#include "spec_internal.hpp"

namespace {

thread_local int g_last_hip_error = 0;

int kind_width(int kind) {
    switch (kind) {
    case SPEC_KIND_BOOL: case SPEC_KIND_BYTE: return 1;
    case SPEC_KIND_INT16: case SPEC_KIND_UINT16: return 2;
    case SPEC_KIND_INT32: case SPEC_KIND_UINT32: case SPEC_KIND_FLOAT32: return 4;
    case SPEC_KIND_INT64: case SPEC_KIND_UINT64: case SPEC_KIND_FLOAT64: case SPEC_KIND_BIN64: return 8;
    case SPEC_KIND_BIN128: return 16;
    case SPEC_KIND_BIN256: return 32;
    case SPEC_KIND_STRING: case SPEC_KIND_BYTES: return 8;
    }
    return 0;
}

// Table order a Writer produces for this schema: messageStack.insert over the tags in write
// order, insertion sort where an equal tag written later moves before the earlier one
// (internal/writer/stack_msg.go:37-61).  order[j] = schema index of the j-th table entry.
void table_order(const spec_schema *s, uint8_t *order) {
    uint16_t tags[SPEC_MAX_FIELDS];
    uint8_t idx[SPEC_MAX_FIELDS];
    for (uint32_t f = 0; f < s->nfields; f++) {
        tags[f] = s->fields[f].tag;
        idx[f] = (uint8_t)f;
        for (int i = (int)f; i > 0; i--) {
            if (tags[i - 1] < tags[i]) break;
            uint16_t t = tags[i - 1];
            tags[i - 1] = tags[i];
            tags[i] = t;
            uint8_t x = idx[i - 1];
            idx[i - 1] = idx[i];
            idx[i] = x;
        }
    }
    memcpy(order, idx, s->nfields);
}

int check_schema(const spec_schema *s) {
    if (!s || s->nfields > SPEC_MAX_FIELDS) return SPEC_E_INVALID_ARGUMENT;
    for (uint32_t f = 0; f < s->nfields; f++)
        if (kind_width(s->fields[f].kind) == 0) return SPEC_E_INVALID_ARGUMENT;
    return SPEC_OK;
}

// outer schema of a nested decode: flat kinds plus exactly one SPEC_KIND_LIST; *list_f = its index
int check_nested(const spec_nested_schema *s, uint32_t *list_f) {
    if (!s || s->outer.nfields > SPEC_MAX_FIELDS || check_schema(&s->item)) return SPEC_E_INVALID_ARGUMENT;
    int lists = 0;
    for (uint32_t f = 0; f < s->outer.nfields; f++) {
        if (s->outer.fields[f].kind == SPEC_KIND_LIST) {
            lists++;
            *list_f = f;
        } else if (kind_width(s->outer.fields[f].kind) == 0) {
            return SPEC_E_INVALID_ARGUMENT;
        }
    }
    return lists == 1 ? SPEC_OK : SPEC_E_INVALID_ARGUMENT;
}

int hip_rc(hipError_t e) {
    if (e == hipSuccess) return SPEC_OK;
    g_last_hip_error = (int)e;
    return SPEC_E_HIP;
}

void fill_field_set(spec::FieldSet &fs, const spec_schema *schema, void *const *columns, uint8_t *status) {
    memset(&fs, 0, sizeof(fs));
    fs.status = status;
    fs.errmask = nullptr;
    fs.nfields = schema->nfields;
    uint8_t order[SPEC_MAX_FIELDS];
    table_order(schema, order);
    for (uint32_t j = 0; j < schema->nfields; j++) fs.rank[order[j]] = (uint8_t)j;
    for (uint32_t f = 0; f < schema->nfields; f++) {
        fs.tags[f] = schema->fields[f].tag;
        fs.kinds[f] = schema->fields[f].kind;
        fs.cols[f] = columns ? columns[f] : nullptr;
    }
}

void fill_enc_fields(spec::EncFields &e, const spec_schema *schema, const void *const *columns) {
    memset(&e, 0, sizeof(e));
    e.nfields = schema->nfields;
    for (uint32_t f = 0; f < schema->nfields; f++) {
        e.tags[f] = schema->fields[f].tag;
        e.kinds[f] = schema->fields[f].kind;
        e.cols[f] = columns ? columns[f] : nullptr;
        if (schema->fields[f].tag > 255) e.table_big_forced = 1;
    }
    table_order(schema, e.order);
}

void fill_encode_args(spec::EncodeArgs &a, const spec_schema *schema, const void *const *columns, uint64_t n) {
    memset(&a, 0, sizeof(a));
    a.n = n;
    fill_enc_fields(a.f, schema, columns);
    a.nblocks = (n + spec::ENC_BLOCK - 1) / spec::ENC_BLOCK;
}

} // namespace

namespace spec {
void note_hip_error(hipError_t e) {
    if (e != hipSuccess) g_last_hip_error = (int)e;
}

int encode_flat_passes(const spec_schema *schema, const void *const *columns, const uint8_t *const *heaps,
                       const uint64_t *heap_lens, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *ends,
                       uint64_t ends_base, void *workspace, size_t workspace_size, uint64_t *total, int passes,
                       hipStream_t stream) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (!columns || !workspace || (n && (!ends || !out))) return SPEC_E_INVALID_ARGUMENT;
    if (workspace_size < spec_encode_flat_workspace_size(n)) return SPEC_E_WORKSPACE;
    EncodeArgs a{};
    fill_encode_args(a, schema, columns, n);
    for (uint32_t f = 0; f < schema->nfields; f++) {
        int k = schema->fields[f].kind;
        if (k == SPEC_KIND_STRING || k == SPEC_KIND_BYTES) {
            if (!heaps || !heap_lens || (!heaps[f] && heap_lens[f])) return SPEC_E_INVALID_ARGUMENT;
            a.f.heaps[f] = heaps[f];
            a.f.heap_lens[f] = heap_lens[f];
        }
    }
    a.check_heaps = 1;
    a.out = out;
    a.out_cap = out_cap;
    a.ends = ends;
    a.ends_base = ends_base;
    a.block_sums = (uint64_t *)workspace;
    a.total = total;
    if ((passes & ENC_PASS_SIZE) && launch_encode_size(schema, a, stream)) return hip_rc(hipGetLastError());
    if ((passes & ENC_PASS_WRITE) && launch_encode_write(schema, a, stream)) return hip_rc(hipGetLastError());
    return SPEC_OK;
}
} // namespace spec

extern "C" {

int spec_abi_version(void) { return SPEC_AMD_ABI_VERSION; }

int spec_kind_width(int kind) { return kind_width(kind); }

int spec_last_hip_error(void) { return g_last_hip_error; }

const char *spec_strerror(int rc) {
    switch (rc) {
    case SPEC_OK: return "ok";
    case SPEC_E_INVALID_ARGUMENT: return "invalid argument";
    case SPEC_E_HIP: return "HIP runtime error";
    case SPEC_E_TOO_LARGE: return "batch too large (stream >= 4 GiB or record > format.MaxSize)";
    case SPEC_E_CAPACITY: return "output capacity too small";
    case SPEC_E_WORKSPACE: return "workspace too small";
    case SPEC_E_CORRUPT: return "corrupt LZ4 frame";
    case SPEC_E_ENCODE: return "encoder error (a span outside its heap or a value > format.MaxSize)";
    }
    return "unknown error";
}

int spec_set_device(int device) { return hip_rc(hipSetDevice(device)); }
int spec_device_alloc(size_t bytes, void **ptr) {
    if (!ptr) return SPEC_E_INVALID_ARGUMENT;
    return hip_rc(hipMalloc(ptr, bytes ? bytes : 1));
}
int spec_device_free(void *ptr) { return hip_rc(hipFree(ptr)); }
int spec_host_alloc(size_t bytes, void **ptr) {
    if (!ptr) return SPEC_E_INVALID_ARGUMENT;
    return hip_rc(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault));
}
int spec_host_free(void *ptr) { return hip_rc(hipHostFree(ptr)); }
int spec_stream_create(void **stream) {
    if (!stream) return SPEC_E_INVALID_ARGUMENT;
    return hip_rc(hipStreamCreateWithFlags((hipStream_t *)stream, hipStreamNonBlocking));
}
int spec_stream_destroy(void *stream) { return hip_rc(hipStreamDestroy((hipStream_t)stream)); }
int spec_stream_sync(void *stream) { return hip_rc(hipStreamSynchronize((hipStream_t)stream)); }
int spec_copy_h2d(void *dst, const void *src, size_t bytes, void *stream) {
    return hip_rc(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
}
int spec_copy_d2h(void *dst, const void *src, size_t bytes, void *stream) {
    return hip_rc(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
}
int spec_copy_d2d(void *dst, const void *src, size_t bytes, void *stream) {
    return hip_rc(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
}

static int decode_flat_impl(const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                            const uint64_t *ends, uint64_t r0, uint64_t r1, uint64_t range_bytes, uint32_t head,
                            void *const *columns, uint8_t *status, void *stream, uint64_t *errmask = nullptr) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (r1 < r0) return SPEC_E_INVALID_ARGUMENT;
    if (r1 == r0) return SPEC_OK;
    if (!ends || !columns || (!stream_bytes && stream_len)) return SPEC_E_INVALID_ARGUMENT;
    if (stream_len >= (1ull << 32)) return SPEC_E_TOO_LARGE;
    for (uint32_t f = 0; f < schema->nfields; f++)
        if (!columns[f]) return SPEC_E_INVALID_ARGUMENT;
    spec::DecodeArgs a;
    memset(&a, 0, sizeof(a));
    a.stream = stream_bytes;
    a.stream_len = stream_len;
    a.ends = ends;
    a.n = r1;
    a.r0 = r0;
    a.head = head;
    fill_field_set(a.f, schema, columns, status);
    a.f.errmask = errmask;
    // LDS slab from the mean record size of the range (the caller knows the range's bytes;
    // for a whole batch it is stream_len / n)
    double avg = range_bytes ? (double)range_bytes / (double)(r1 - r0) : (double)stream_len / (double)r1;
    // field error masks: the schema-specialised kernel's errmask variant (or the generic path)
    int j = spec::jit_launch_decode_flat(schema, a, avg, (hipStream_t)stream);
    if (j < 0) return hip_rc(hipGetLastError());
    if (j == 0 && spec::launch_decode_flat(a, avg, (hipStream_t)stream)) return hip_rc(hipGetLastError());
    return SPEC_OK;
}

int spec_decode_flat_range(const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                           const uint64_t *ends, uint64_t r0, uint64_t r1, uint64_t range_bytes, void *const *columns,
                           uint8_t *status, void *stream) {
    return decode_flat_impl(schema, stream_bytes, stream_len, ends, r0, r1, range_bytes, 0, columns, status, stream);
}

int spec_decode_flat(const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                     const uint64_t *ends, uint64_t n, void *const *columns, uint8_t *status,
                     void *stream) {
    return decode_flat_impl(schema, stream_bytes, stream_len, ends, 0, n, 0, 0, columns, status, stream);
}

int spec_decode_flat_errors(const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                            const uint64_t *ends, uint64_t n, void *const *columns, uint8_t *status, uint64_t *errmask,
                            void *stream) {
    if (!errmask && n) return SPEC_E_INVALID_ARGUMENT;
    return decode_flat_impl(schema, stream_bytes, stream_len, ends, 0, n, 0, 0, columns, status, stream, errmask);
}

int spec_decode_frames(const spec_schema *schema, const uint8_t *frames, uint64_t frames_len,
                       const uint64_t *ends, uint64_t r0, uint64_t r1, uint64_t range_bytes, void *const *columns,
                       uint8_t *status, void *stream) {
    return decode_flat_impl(schema, frames, frames_len, ends, r0, r1, range_bytes, 4, columns, status, stream);
}

// mpx framing, mpx/conn_reader.go:179-194 (read) / mpx/conn_writer.go:84-97 (write):
// [u32 big-endian size][size message bytes], back to back.
int spec_frames_index(const uint8_t *buf, uint64_t len, uint64_t *ends, uint64_t cap, uint64_t *count,
                      uint64_t *consumed) {
    if ((!buf && len) || !count || !consumed || (cap && !ends)) return SPEC_E_INVALID_ARGUMENT;
    uint64_t p = 0, k = 0;
    while (p + 4 <= len) {
        const uint64_t size = ((uint64_t)buf[p] << 24) | ((uint64_t)buf[p + 1] << 16) | ((uint64_t)buf[p + 2] << 8) |
                              (uint64_t)buf[p + 3];
        if (p + 4 + size > len) break; // incomplete frame: the caller reads more
        if (k == cap) {
            *count = k;
            *consumed = p;
            return SPEC_E_CAPACITY;
        }
        p += 4 + size;
        ends[k++] = p;
    }
    *count = k;
    *consumed = p;
    return SPEC_OK;
}

size_t spec_frames_index_device_workspace_size(uint64_t len) { return spec::frames_index_device_workspace(len); }

int spec_frames_index_device(const uint8_t *buf, uint64_t len, uint64_t *ends, uint64_t cap, uint64_t *count,
                             uint64_t *consumed, int32_t *status, void *workspace, size_t workspace_size,
                             void *stream) {
    if ((!buf && len) || ((uintptr_t)buf & 3) || !count || !consumed || !status || (cap && !ends) || !workspace)
        return SPEC_E_INVALID_ARGUMENT;
    if (len >= (1ull << 48)) return SPEC_E_TOO_LARGE;
    if (workspace_size < spec::frames_index_device_workspace(len)) return SPEC_E_WORKSPACE;
    if (spec::launch_frames_index_device(buf, len, ends, cap, count, consumed, status, workspace, (hipStream_t)stream))
        return hip_rc(hipGetLastError());
    return SPEC_OK;
}

int spec_parse_messages(const uint8_t *stream_bytes, uint64_t stream_len, const uint64_t *ends, uint64_t n,
                        uint32_t head, uint8_t *status, uint32_t *sizes, void *stream) {
    if (n == 0) return SPEC_OK;
    if (!ends || !status || (!stream_bytes && stream_len)) return SPEC_E_INVALID_ARGUMENT;
    if (stream_len >= (1ull << 32)) return SPEC_E_TOO_LARGE;
    spec::DecodeArgs a;
    memset(&a, 0, sizeof(a));
    a.stream = stream_bytes;
    a.stream_len = stream_len;
    a.ends = ends;
    a.n = n;
    a.head = head;
    a.f.status = status;
    if (spec::launch_parse(a, sizes, (double)stream_len / (double)n, (hipStream_t)stream))
        return hip_rc(hipGetLastError());
    return SPEC_OK;
}

int spec_decode_flat_prepare(const spec_schema *schema, uint64_t stream_len, uint64_t n) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (n == 0) return 0;
    return spec::jit_prepare_decode_flat(schema, (double)stream_len / (double)n);
}

void spec_set_jit(int enabled) { spec::jit_set_enabled(enabled); }

long long spec_decode_flat_jit_compile(const spec_schema *schema, uint64_t stream_len, uint64_t n) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (n == 0) return 0;
    return spec::jit_compile_only(schema, (double)stream_len / (double)n);
}

long long spec_encode_flat_jit_compile(const spec_schema *schema) {
    int rc = check_schema(schema);
    if (rc) return rc;
    return spec::jit_compile_only_encode(schema);
}

size_t spec_decode_nested_workspace_size(uint64_t n) { return (size_t)(((n + 63) / 64 + 1) * sizeof(uint64_t)); }

static int nested_args(spec::NestedArgs &a, const spec_nested_schema *schema, const uint8_t *stream_bytes,
                       uint64_t stream_len, const uint64_t *ends, uint64_t n, void *workspace,
                       size_t workspace_size) {
    uint32_t list_f = 0;
    int rc = check_nested(schema, &list_f);
    if (rc) return rc;
    if (n && (!ends || (!stream_bytes && stream_len) || !workspace)) return SPEC_E_INVALID_ARGUMENT;
    if (stream_len >= (1ull << 32)) return SPEC_E_TOO_LARGE;
    if (workspace_size < spec_decode_nested_workspace_size(n)) return SPEC_E_WORKSPACE;
    memset(&a, 0, sizeof(a));
    a.stream = stream_bytes;
    a.stream_len = stream_len;
    a.ends = ends;
    a.n = n;
    fill_field_set(a.outer, &schema->outer, nullptr, nullptr);
    fill_field_set(a.item, &schema->item, nullptr, nullptr);
    a.list_tag = schema->outer.fields[list_f].tag;
    a.list_rank = a.outer.rank[list_f];
    a.group_base = (uint64_t *)workspace;
    return SPEC_OK;
}

int spec_decode_nested_index(const spec_nested_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                             const uint64_t *ends, uint64_t n, void *workspace, size_t workspace_size,
                             uint64_t *total_items, void *stream) {
    spec::NestedArgs a{};
    int rc = nested_args(a, schema, stream_bytes, stream_len, ends, n, workspace, workspace_size);
    if (rc) return rc;
    if (!total_items) return SPEC_E_INVALID_ARGUMENT;
    a.total = total_items;
    double avg = n ? (double)stream_len / (double)n : 0.0;
    if (spec::launch_nested_index(a, avg, (hipStream_t)stream)) return hip_rc(hipGetLastError());
    return SPEC_OK;
}

int spec_decode_nested(const spec_nested_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                       const uint64_t *ends, uint64_t n, void *const *outer_columns, uint8_t *status,
                       uint32_t *item_begin, void *const *item_columns, uint8_t *item_status, uint64_t item_cap,
                       void *workspace, size_t workspace_size, void *stream) {
    spec::NestedArgs a{};
    int rc = nested_args(a, schema, stream_bytes, stream_len, ends, n, workspace, workspace_size);
    if (rc) return rc;
    if (n == 0) return SPEC_OK;
    if (!outer_columns || !item_begin || (item_cap && !item_columns)) return SPEC_E_INVALID_ARGUMENT;
    for (uint32_t f = 0; f < schema->outer.nfields; f++) {
        if (schema->outer.fields[f].kind == SPEC_KIND_LIST) continue;
        if (!outer_columns[f]) return SPEC_E_INVALID_ARGUMENT;
        a.outer.cols[f] = outer_columns[f];
    }
    for (uint32_t f = 0; f < schema->item.nfields && item_cap; f++) {
        if (!item_columns[f]) return SPEC_E_INVALID_ARGUMENT;
        a.item.cols[f] = item_columns[f];
    }
    a.outer.status = status;
    a.item.status = item_cap ? item_status : nullptr;
    a.item_begin = item_begin;
    a.item_cap = item_cap;
    double avg = (double)stream_len / (double)n;
    if (spec::launch_nested_decode(schema, a, avg, (hipStream_t)stream)) return hip_rc(hipGetLastError());
    return SPEC_OK;
}

int spec_decode_nested_onepass(const spec_nested_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                               const uint64_t *ends, uint64_t n, void *const *outer_columns, uint8_t *status,
                               uint32_t *item_begin, void *const *item_columns, uint8_t *item_status,
                               uint64_t item_cap, void *workspace, size_t workspace_size, uint64_t *total_items,
                               void *stream) {
    spec::NestedArgs a{};
    int rc = nested_args(a, schema, stream_bytes, stream_len, ends, n, workspace, workspace_size);
    if (rc) return rc;
    if (!total_items) return SPEC_E_INVALID_ARGUMENT;
    a.total = total_items;
    if (n) {
        if (!outer_columns || !item_begin || (item_cap && !item_columns)) return SPEC_E_INVALID_ARGUMENT;
        for (uint32_t f = 0; f < schema->outer.nfields; f++) {
            if (schema->outer.fields[f].kind == SPEC_KIND_LIST) continue;
            if (!outer_columns[f]) return SPEC_E_INVALID_ARGUMENT;
            a.outer.cols[f] = outer_columns[f];
        }
        for (uint32_t f = 0; f < schema->item.nfields && item_cap; f++) {
            if (!item_columns[f]) return SPEC_E_INVALID_ARGUMENT;
            a.item.cols[f] = item_columns[f];
        }
    }
    a.outer.status = status;
    a.item.status = item_cap ? item_status : nullptr;
    a.item_begin = item_begin;
    a.item_cap = item_cap;
    double avg = n ? (double)stream_len / (double)n : 0.0;
    if (spec::launch_nested_onepass(schema, a, avg, (hipStream_t)stream)) return hip_rc(hipGetLastError());
    return SPEC_OK;
}

long long spec_decode_nested_jit_compile(const spec_nested_schema *schema) {
    uint32_t list_f = 0;
    int rc = check_nested(schema, &list_f);
    if (rc) return rc;
    return spec::jit_compile_only_nested(schema);
}

long long spec_encode_nested_jit_compile(const spec_nested_schema *schema) {
    uint32_t list_f = 0;
    int rc = check_nested(schema, &list_f);
    if (rc) return rc;
    return spec::jit_compile_only_nested_encode(schema);
}

size_t spec_encode_nested_workspace_size(uint64_t n) { return spec_encode_flat_workspace_size(n); }

// block sums | item prefixes (u32 per item) | wave verdicts (one byte per 64 records)
static size_t nested_ws_base(uint64_t n) { return (spec_encode_flat_workspace_size(n) + 255) & ~(size_t)255; }
size_t spec_encode_nested_workspace_size_items(uint64_t n, uint64_t nitems) {
    return nested_ws_base(n) + (((size_t)nitems * 4 + 255) & ~(size_t)255) + (size_t)((n + 63) / 64);
}

static int heaps_of(spec::EncFields &e, const spec_schema *s, const uint8_t *const *heaps, const uint64_t *lens) {
    for (uint32_t f = 0; f < s->nfields; f++) {
        int k = s->fields[f].kind;
        if (k == SPEC_KIND_STRING || k == SPEC_KIND_BYTES) {
            if (!heaps || !lens || (!heaps[f] && lens[f])) return SPEC_E_INVALID_ARGUMENT;
            e.heaps[f] = heaps[f];
            e.heap_lens[f] = lens[f];
        }
    }
    return SPEC_OK;
}

int spec_encode_nested(const spec_nested_schema *schema, const void *const *outer_columns,
                       const uint8_t *const *outer_heaps, const uint64_t *outer_heap_lens, const uint32_t *item_begin,
                       const void *const *item_columns, const uint8_t *const *item_heaps,
                       const uint64_t *item_heap_lens, uint64_t nitems, uint64_t n, uint8_t *out, uint64_t out_cap,
                       uint64_t *ends, void *workspace, size_t workspace_size, uint64_t *total, void *stream) {
    uint32_t list_f = 0;
    int rc = check_nested(schema, &list_f);
    if (rc) return rc;
    if (!workspace || !total || (n && (!item_begin || !outer_columns))) return SPEC_E_INVALID_ARGUMENT;
    if (nitems && !item_columns) return SPEC_E_INVALID_ARGUMENT;
    if (out && !ends && n) return SPEC_E_INVALID_ARGUMENT;
    if (workspace_size < spec_encode_nested_workspace_size(n)) return SPEC_E_WORKSPACE;
    spec::NestedEncodeArgs a{};
    memset(&a, 0, sizeof(a));
    a.n = n;
    fill_enc_fields(a.outer, &schema->outer, outer_columns);
    fill_enc_fields(a.item, &schema->item, nitems ? item_columns : nullptr);
    for (uint32_t f = 0; f < schema->outer.nfields; f++)
        if (f != list_f && !outer_columns[f]) return SPEC_E_INVALID_ARGUMENT;
    a.outer.cols[list_f] = nullptr;
    if ((rc = heaps_of(a.outer, &schema->outer, outer_heaps, outer_heap_lens))) return rc;
    if ((rc = heaps_of(a.item, &schema->item, item_heaps, item_heap_lens))) return rc;
    a.item_begin = item_begin;
    a.nitems = nitems;
    a.check_heaps = 1;
    a.out = out;
    a.out_cap = out ? out_cap : 0;
    a.ends = ends;
    a.block_sums = (uint64_t *)workspace;
    a.nblocks = (n + spec::ENC_BLOCK - 1) / spec::ENC_BLOCK;
    a.total = total;
    if (workspace_size >= spec_encode_nested_workspace_size_items(n, nitems)) {
        a.item_pre = (uint32_t *)((uint8_t *)workspace + nested_ws_base(n));
        a.wave_ok = (uint8_t *)a.item_pre + (((size_t)nitems * 4 + 255) & ~(size_t)255);
    }
    if (spec::launch_nested_encode(schema, a, out != nullptr, (hipStream_t)stream))
        return hip_rc(hipGetLastError());
    return SPEC_OK;
}

size_t spec_encode_flat_workspace_size(uint64_t n) {
    uint64_t nblocks = (n + spec::ENC_BLOCK - 1) / spec::ENC_BLOCK;
    return (size_t)((nblocks + 1) * sizeof(uint64_t));
}

int spec_encode_flat_size(const spec_schema *schema, const void *const *columns, uint64_t n,
                          void *workspace, size_t workspace_size, uint64_t *total, void *stream) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (!columns || !workspace) return SPEC_E_INVALID_ARGUMENT;
    if (workspace_size < spec_encode_flat_workspace_size(n)) return SPEC_E_WORKSPACE;
    spec::EncodeArgs a{};
    fill_encode_args(a, schema, columns, n);
    a.block_sums = (uint64_t *)workspace;
    a.total = total;
    if (spec::launch_encode_size(schema, a, (hipStream_t)stream)) return hip_rc(hipGetLastError());
    return SPEC_OK;
}

int spec_encode_flat(const spec_schema *schema, const void *const *columns,
                     const uint8_t *const *heaps, const uint64_t *heap_lens, uint64_t n,
                     uint8_t *out, uint64_t out_cap, uint64_t *ends, void *workspace,
                     size_t workspace_size, uint64_t *total, void *stream) {
    return spec::encode_flat_passes(schema, columns, heaps, heap_lens, n, out, out_cap, ends, 0, workspace,
                                    workspace_size, total, spec::ENC_PASS_SIZE | spec::ENC_PASS_WRITE,
                                    (hipStream_t)stream);
}

} // extern "C"
