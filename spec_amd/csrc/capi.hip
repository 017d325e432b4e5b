// capi.hip — the C ABI of libspec_amd.so (include/spec_amd.h): argument validation, schema
// preprocessing (table order) and kernel launches.  No host sync on any path.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

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
// The insertion moves a new entry left past every entry whose tag is >= its own, so the result
// is the unique order by (tag ascending, write index descending): sorted in O(n log n) here
// (a 1024-field schema in reverse tag order cost ~0.5 M swaps per call as an insertion sort).
template <class T>
void table_order(const spec_schema *s, T *order) {
    uint32_t key[SPEC_MAX_FIELDS]; // tag << 16 | (0xffff - index): ascending = the Writer's order
    for (uint32_t f = 0; f < s->nfields; f++) key[f] = (uint32_t)s->fields[f].tag << 16 | (0xffffu - f);
    std::sort(key, key + s->nfields);
    for (uint32_t j = 0; j < s->nfields; j++) order[j] = (T)(0xffffu - (key[j] & 0xffffu));
}

int check_schema(const spec_schema *s) {
    if (!s || s->nfields > SPEC_MAX_FIELDS) return SPEC_E_INVALID_ARGUMENT;
    for (uint32_t f = 0; f < s->nfields; f++)
        if (kind_width(s->fields[f].kind) == 0) return SPEC_E_INVALID_ARGUMENT;
    return SPEC_OK;
}

// outer schema of a nested decode: flat kinds plus exactly one SPEC_KIND_LIST; *list_f = its index
int check_nested(const spec_nested_schema *s, uint32_t *list_f) {
    // (a half of more than SPEC_KFIELDS fields: decoded in field chunks, encoded through the tree
    // encoder — nested_decode_chunks, nested_encode_wide)
    if (!s || s->outer.nfields > SPEC_MAX_FIELDS || check_schema(&s->item))
        return SPEC_E_INVALID_ARGUMENT;
    // a wide schema encodes as one schema tree of outer + item fields: the same limit for decode,
    // so a schema either decodes and encodes or is rejected up front
    if ((s->outer.nfields > SPEC_KFIELDS || s->item.nfields > SPEC_KFIELDS) &&
        s->outer.nfields + s->item.nfields > SPEC_TREE_MAX_FIELDS)
        return SPEC_E_INVALID_ARGUMENT;
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

} // namespace

namespace spec {
// ---- pinned uploads: per-call kernel data too large for the kernel arguments (a wide schema's
// field set, a schema tree's descriptor block) goes to the device from a pool of pinned slots
// per device.  A slot is reused once the copy out of it has run (its event has completed,
// hipEventQuery: no wait); when every slot is still in flight the pool grows by one, so a call
// never waits on the device, and the lock (one per device) is held only to claim or release a
// slot, never across a HIP copy.  Such a call cannot be captured into a HIP graph (its copy
// source is a pooled slot that later calls refill).
namespace {
struct UploadSlot {
    uint8_t *p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    bool busy = false; // claimed by a call that has not yet recorded its event
};
struct UploadPool {
    std::mutex mu;
    std::vector<UploadSlot *> slots;
};
UploadPool g_upload[64];
} // namespace

hipError_t pinned_upload(void *dst, const void *src, size_t bytes, hipStream_t st) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    UploadPool &P = g_upload[dev];
    UploadSlot *S = nullptr;
    {
        std::lock_guard<std::mutex> lk(P.mu);
        for (UploadSlot *s : P.slots)
            if (!s->busy && (!s->ev || hipEventQuery(s->ev) == hipSuccess)) {
                S = s;
                break;
            }
        if (!S) {
            S = new (std::nothrow) UploadSlot();
            if (!S) return hipErrorOutOfMemory;
            P.slots.push_back(S);
        }
        S->busy = true;
    }
    auto fill = [&]() -> hipError_t {
        hipError_t r;
        if (!S->ev && (r = hipEventCreateWithFlags(&S->ev, hipEventDisableTiming)) != hipSuccess) return r;
        if (S->cap < bytes) {
            if (S->p) (void)hipHostFree(S->p);
            S->p = nullptr;
            S->cap = 0;
            if ((r = hipHostMalloc((void **)&S->p, bytes, hipHostMallocDefault)) != hipSuccess) return r;
            S->cap = bytes;
        }
        memcpy(S->p, src, bytes);
        if ((r = hipMemcpyAsync(dst, S->p, bytes, hipMemcpyHostToDevice, st)) != hipSuccess) return r;
        return hipEventRecord(S->ev, st);
    };
    e = fill();
    std::lock_guard<std::mutex> lk(P.mu);
    S->busy = false;
    return e;
}
} // namespace spec

namespace {
hipError_t upload_async(void *dst, const void *src, size_t bytes, hipStream_t st) {
    return spec::pinned_upload(dst, src, bytes, st);
}

int hip_rc(hipError_t e) {
    if (e == hipSuccess) return SPEC_OK;
    g_last_hip_error = (int)e;
    return SPEC_E_HIP;
}

// Fields [f0, f1) (at most SPEC_KFIELDS) of the schema as one kernel field set; rank = the
// field's index in the table a Writer emits for the WHOLE schema (a chunk of a wide schema is
// looked up in the full table).
void fill_field_set(spec::FieldSet &fs, const spec_schema *schema, void *const *columns, uint8_t *status,
                    uint32_t f0 = 0, uint32_t f1 = ~0u) {
    memset(&fs, 0, sizeof(fs));
    if (f1 > schema->nfields) f1 = schema->nfields;
    fs.status = status;
    fs.errmask = nullptr;
    fs.nfields = f1 - f0;
    uint16_t order[SPEC_MAX_FIELDS], rank[SPEC_MAX_FIELDS];
    table_order(schema, order);
    for (uint32_t j = 0; j < schema->nfields; j++) rank[order[j]] = (uint16_t)j;
    for (uint32_t f = f0; f < f1; f++) {
        fs.tags[f - f0] = schema->fields[f].tag;
        fs.kinds[f - f0] = schema->fields[f].kind;
        fs.rank[f - f0] = rank[f];
        fs.cols[f - f0] = columns ? columns[f] : nullptr;
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

// Encode workspace: the block sums (nblocks + 1 words), then room for a wide schema's field set.
constexpr size_t WIDE_FIELDS_BYTES = 32768; // >= SPEC_MAX_FIELDS x (2 + 1 + 2 + 8 + 8 + 8) + alignment
size_t enc_ws_sums(uint64_t n) {
    const uint64_t nblocks = (n + spec::ENC_BLOCK - 1) / spec::ENC_BLOCK;
    return (size_t)(((nblocks + 1) * sizeof(uint64_t) + 255) & ~(uint64_t)255);
}

// A schema with more than SPEC_KFIELDS fields: its field set (tags, kinds, table positions,
// columns, heaps) written into the workspace after the block sums, from a pinned slot on the
// call's stream; the kernel argument holds the pointers.
int fill_wide_encode_args(spec::WideEncodeArgs &a, const spec_schema *schema, const void *const *columns,
                          const uint8_t *const *heaps, const uint64_t *heap_lens, uint64_t n, void *workspace,
                          hipStream_t st) {
    memset(&a, 0, sizeof(a));
    const uint32_t N = schema->nfields;
    a.n = n;
    a.nblocks = (n + spec::ENC_BLOCK - 1) / spec::ENC_BLOCK;
    uint8_t *dev = (uint8_t *)workspace + enc_ws_sums(n);
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t o_tags = 0, o_kinds = al(o_tags + 2 * N), o_inv = al(o_kinds + N), o_cols = al(o_inv + 2 * N),
                 o_heaps = o_cols + 8 * N, o_lens = o_heaps + 8 * N, bytes = o_lens + 8 * N;
    if (bytes > WIDE_FIELDS_BYTES) return SPEC_E_INVALID_ARGUMENT;
    std::vector<uint8_t> h(bytes, 0);
    uint16_t order[SPEC_MAX_FIELDS];
    table_order(schema, order);
    for (uint32_t f = 0; f < N; f++) {
        ((uint16_t *)(h.data() + o_tags))[f] = schema->fields[f].tag;
        h[o_kinds + f] = schema->fields[f].kind;
        ((uint16_t *)(h.data() + o_inv))[order[f]] = (uint16_t)f;
        ((const void **)(h.data() + o_cols))[f] = columns ? columns[f] : nullptr;
        const int k = schema->fields[f].kind;
        if (heaps && heap_lens && (k == SPEC_KIND_STRING || k == SPEC_KIND_BYTES)) {
            if (!heaps[f] && heap_lens[f]) return SPEC_E_INVALID_ARGUMENT;
            ((const uint8_t **)(h.data() + o_heaps))[f] = heaps[f];
            ((uint64_t *)(h.data() + o_lens))[f] = heap_lens[f];
        }
        if (schema->fields[f].tag > 255) a.f.table_big_forced = 1;
    }
    a.f.nfields = N;
    a.f.tags = (const uint16_t *)(dev + o_tags);
    a.f.kinds = dev + o_kinds;
    a.f.inv_order = (const uint16_t *)(dev + o_inv);
    a.f.cols = (const void *const *)(dev + o_cols);
    a.f.heaps = (const uint8_t *const *)(dev + o_heaps);
    a.f.heap_lens = (const uint64_t *)(dev + o_lens);
    const hipError_t e = upload_async(dev, h.data(), bytes, st);
    return e == hipSuccess ? SPEC_OK : hip_rc(e);
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
    if (schema->nfields > SPEC_KFIELDS) {
        for (uint32_t f = 0; f < schema->nfields; f++) {
            const int k = schema->fields[f].kind;
            if ((k == SPEC_KIND_STRING || k == SPEC_KIND_BYTES) && (!heaps || !heap_lens)) return SPEC_E_INVALID_ARGUMENT;
        }
        WideEncodeArgs w{};
        if ((rc = fill_wide_encode_args(w, schema, columns, heaps, heap_lens, n, workspace, stream))) return rc;
        w.check_heaps = 1;
        w.out = out;
        w.out_cap = out_cap;
        w.ends = ends;
        w.ends_base = ends_base;
        w.block_sums = (uint64_t *)workspace;
        w.total = total;
        if ((passes & ENC_PASS_SIZE) && launch_encode_wide_size(w, stream)) return hip_rc(hipGetLastError());
        if ((passes & ENC_PASS_WRITE) && launch_encode_wide_write(w, stream)) return hip_rc(hipGetLastError());
        return SPEC_OK;
    }
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

size_t spec_struct_size(int which) {
    switch (which) {
    case SPEC_ABI_SPAN: return sizeof(spec_span);
    case SPEC_ABI_FIELD: return sizeof(spec_field);
    case SPEC_ABI_SCHEMA: return sizeof(spec_schema);
    case SPEC_ABI_NESTED_SCHEMA: return sizeof(spec_nested_schema);
    case SPEC_ABI_TREE_FIELD: return sizeof(spec_tree_field);
    case SPEC_ABI_TREE: return sizeof(spec_tree);
    case SPEC_ABI_TREE_TABLE: return sizeof(spec_tree_table);
    case SPEC_ABI_TREE_COLUMN: return sizeof(spec_tree_column);
    case SPEC_ABI_LZ4_BLOCK: return sizeof(spec_lz4_block);
    case SPEC_ABI_LZ4_STATE: return sizeof(spec_lz4_state);
    case SPEC_ABI_LZ4_CONTENT: return sizeof(spec_lz4_content);
    }
    return 0;
}

size_t spec_struct_offset(int which, int member) {
#define SPEC_OFFS(T, ...)                                                                                              \
    do {                                                                                                               \
        const size_t o[] = {__VA_ARGS__};                                                                              \
        return member >= 0 && member < (int)(sizeof(o) / sizeof(o[0])) ? o[member] : (size_t)-1;                       \
    } while (0)
    switch (which) {
    case SPEC_ABI_SPAN: SPEC_OFFS(spec_span, offsetof(spec_span, off), offsetof(spec_span, len));
    case SPEC_ABI_FIELD:
        SPEC_OFFS(spec_field, offsetof(spec_field, tag), offsetof(spec_field, kind), offsetof(spec_field, reserved));
    case SPEC_ABI_SCHEMA: SPEC_OFFS(spec_schema, offsetof(spec_schema, nfields), offsetof(spec_schema, fields));
    case SPEC_ABI_NESTED_SCHEMA:
        SPEC_OFFS(spec_nested_schema, offsetof(spec_nested_schema, outer), offsetof(spec_nested_schema, item));
    case SPEC_ABI_TREE_FIELD:
        SPEC_OFFS(spec_tree_field, offsetof(spec_tree_field, tag), offsetof(spec_tree_field, kind),
                  offsetof(spec_tree_field, elem), offsetof(spec_tree_field, parent),
                  offsetof(spec_tree_field, reserved));
    case SPEC_ABI_TREE: SPEC_OFFS(spec_tree, offsetof(spec_tree, nfields), offsetof(spec_tree, fields));
    case SPEC_ABI_TREE_TABLE:
        SPEC_OFFS(spec_tree_table, offsetof(spec_tree_table, parent), offsetof(spec_tree_table, field),
                  offsetof(spec_tree_table, rel), offsetof(spec_tree_table, shape),
                  offsetof(spec_tree_table, first_column), offsetof(spec_tree_table, ncolumns));
    case SPEC_ABI_TREE_COLUMN:
        SPEC_OFFS(spec_tree_column, offsetof(spec_tree_column, table), offsetof(spec_tree_column, field),
                  offsetof(spec_tree_column, role), offsetof(spec_tree_column, kind),
                  offsetof(spec_tree_column, width));
    case SPEC_ABI_LZ4_BLOCK:
        SPEC_OFFS(spec_lz4_block, offsetof(spec_lz4_block, src_off), offsetof(spec_lz4_block, src_len),
                  offsetof(spec_lz4_block, stored));
    case SPEC_ABI_LZ4_STATE:
        SPEC_OFFS(spec_lz4_state, offsetof(spec_lz4_state, in_frame), offsetof(spec_lz4_state, block_max),
                  offsetof(spec_lz4_state, flags), offsetof(spec_lz4_state, content_checksum));
    case SPEC_ABI_LZ4_CONTENT:
        SPEC_OFFS(spec_lz4_content, offsetof(spec_lz4_content, v), offsetof(spec_lz4_content, total),
                  offsetof(spec_lz4_content, buf), offsetof(spec_lz4_content, buffered),
                  offsetof(spec_lz4_content, started));
    }
#undef SPEC_OFFS
    return (size_t)-1;
}

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
    // LDS slab from the mean record size of the range (the caller knows the range's bytes;
    // for a whole batch it is stream_len / n)
    double avg = range_bytes ? (double)range_bytes / (double)(r1 - r0) : (double)stream_len / (double)r1;
    if (schema->nfields > SPEC_KFIELDS) {
        // a wide schema: the generic kernel once per chunk of SPEC_KFIELDS fields, each chunk's
        // getters against the record's whole table (ranks in the full Writer table); chunk 0
        // writes the status (OpenMessageErr, the same for every chunk), chunk c the errmask words
        // errmask[c * r1 + r] (bit f = field 64 c + f)
        for (uint32_t f0 = 0; f0 < schema->nfields; f0 += SPEC_KFIELDS) {
            fill_field_set(a.f, schema, columns, f0 ? nullptr : status, f0, f0 + SPEC_KFIELDS);
            a.f.errmask = errmask ? errmask + (uint64_t)(f0 / SPEC_KFIELDS) * r1 : nullptr;
            if (spec::launch_decode_flat(a, avg, (hipStream_t)stream)) return hip_rc(hipGetLastError());
        }
        return SPEC_OK;
    }
    fill_field_set(a.f, schema, columns, status);
    a.f.errmask = errmask;
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
    return spec_parse_batch(SPEC_PARSE_MESSAGE, stream_bytes, stream_len, ends, n, head, status, sizes, stream);
}

int spec_parse_batch(uint32_t root, const uint8_t *stream_bytes, uint64_t stream_len, const uint64_t *ends,
                     uint64_t n, uint32_t head, uint8_t *status, uint32_t *sizes, void *stream) {
    if (root > SPEC_PARSE_VALUE) return SPEC_E_INVALID_ARGUMENT;
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
    if (spec::launch_parse(a, sizes, root, (double)stream_len / (double)n, (hipStream_t)stream))
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
    fill_field_set(a.outer, &schema->outer, nullptr, nullptr, 0, SPEC_KFIELDS);
    fill_field_set(a.item, &schema->item, nullptr, nullptr, 0, SPEC_KFIELDS);
    a.list_tag = schema->outer.fields[list_f].tag;
    uint16_t order[SPEC_MAX_FIELDS];
    table_order(&schema->outer, order);
    for (uint32_t j = 0; j < schema->outer.nfields; j++)
        if (order[j] == list_f) a.list_rank = j; // the list field's index in the whole Writer table
    a.group_base = (uint64_t *)workspace;
    return SPEC_OK;
}

// The nested decode pass over the columns: one launch, or for a schema with a half of more than
// SPEC_KFIELDS fields one launch per chunk of SPEC_KFIELDS fields of each half (every chunk's
// getters against the records' whole tables; chunk 0 writes both status columns, every chunk
// the same item_begin)
static int nested_decode_chunks(const spec_nested_schema *schema, spec::NestedArgs &a, void *const *outer_columns,
                                uint8_t *status, void *const *item_columns, uint8_t *item_status, double avg,
                                hipStream_t stream) {
    const uint32_t no = schema->outer.nfields, ni = schema->item.nfields;
    const uint32_t chunks = std::max<uint32_t>(1, std::max((no + SPEC_KFIELDS - 1) / SPEC_KFIELDS, (ni + SPEC_KFIELDS - 1) / SPEC_KFIELDS));
    std::vector<void *> oc(no, nullptr);
    for (uint32_t f = 0; f < no; f++)
        if (schema->outer.fields[f].kind != SPEC_KIND_LIST) oc[f] = outer_columns[f];
    for (uint32_t c = 0; c < chunks; c++) {
        const uint32_t f0 = c * SPEC_KFIELDS;
        if (f0 < no) fill_field_set(a.outer, &schema->outer, oc.data(), c ? nullptr : status, f0, f0 + SPEC_KFIELDS);
        else fill_field_set(a.outer, &schema->outer, nullptr, nullptr, no, no);
        if (f0 < ni && a.item_cap)
            fill_field_set(a.item, &schema->item, item_columns, c ? nullptr : item_status, f0, f0 + SPEC_KFIELDS);
        else fill_field_set(a.item, &schema->item, nullptr, c ? nullptr : (a.item_cap ? item_status : nullptr), ni, ni);
        if (spec::launch_nested_decode(schema, a, avg, stream)) return hip_rc(hipGetLastError());
    }
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
    for (uint32_t f = 0; f < schema->outer.nfields; f++)
        if (schema->outer.fields[f].kind != SPEC_KIND_LIST && !outer_columns[f]) return SPEC_E_INVALID_ARGUMENT;
    for (uint32_t f = 0; f < schema->item.nfields && item_cap; f++)
        if (!item_columns[f]) return SPEC_E_INVALID_ARGUMENT;
    a.item_begin = item_begin;
    a.item_cap = item_cap;
    double avg = (double)stream_len / (double)n;
    return nested_decode_chunks(schema, a, outer_columns, status, item_columns, item_status, avg, (hipStream_t)stream);
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
            if (f < SPEC_KFIELDS) a.outer.cols[f] = outer_columns[f];
        }
        for (uint32_t f = 0; f < schema->item.nfields && item_cap; f++) {
            if (!item_columns[f]) return SPEC_E_INVALID_ARGUMENT;
            if (f < SPEC_KFIELDS) a.item.cols[f] = item_columns[f];
        }
    }
    a.item_begin = item_begin;
    a.item_cap = item_cap;
    double avg = n ? (double)stream_len / (double)n : 0.0;
    if (schema->outer.nfields > SPEC_KFIELDS || schema->item.nfields > SPEC_KFIELDS) {
        // a wide schema: the index kernels, then the decode in field chunks
        if (n == 0) {
            if (hipMemsetAsync(total_items, 0, sizeof(uint64_t), (hipStream_t)stream) != hipSuccess)
                return hip_rc(hipGetLastError());
            return SPEC_OK;
        }
        if (spec::launch_nested_index(a, avg, (hipStream_t)stream)) return hip_rc(hipGetLastError());
        return nested_decode_chunks(schema, a, outer_columns, status, item_columns, item_status, avg, (hipStream_t)stream);
    }
    a.outer.status = status;
    a.item.status = item_cap ? item_status : nullptr;
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

// A nested schema with a half of more than SPEC_KFIELDS fields, encoded by the schema-tree
// encoder (spec_encode_tree): the records' message with the list field as a LIST of MESSAGE
// items — the same Writer calls (writer_list_msg.go:8-47), so the same bytes.  The list is always
// written (its PRESENT column all ones, from scratch), item_begin is the list table's BEGIN; the
// tree encoder's workspace is stream-ordered scratch (hipMallocAsync / hipFreeAsync), so the
// call stays asynchronous and the nested workspace contract is unchanged.
static int nested_encode_wide(const spec_nested_schema *schema, uint32_t list_f, const void *const *outer_columns,
                              const uint8_t *const *outer_heaps, const uint64_t *outer_heap_lens,
                              const uint32_t *item_begin, const void *const *item_columns,
                              const uint8_t *const *item_heaps, const uint64_t *item_heap_lens, uint64_t nitems,
                              uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *ends, uint64_t *total,
                              hipStream_t st) {
    const uint32_t no = schema->outer.nfields, ni = schema->item.nfields;
    if (no + ni > SPEC_TREE_MAX_FIELDS) return SPEC_E_INVALID_ARGUMENT;
    std::vector<spec_tree> tv(1);
    spec_tree &T = tv[0];
    memset(&T, 0, sizeof(T));
    std::vector<int> half(no + ni), idx(no + ni); // tree field -> (0 outer / 1 item, schema index)
    uint32_t k = 0;
    int list_tf = -1;
    for (uint32_t f = 0; f < no; f++) {
        const spec_field &F = schema->outer.fields[f];
        T.fields[k].tag = F.tag;
        T.fields[k].parent = -1;
        half[k] = 0;
        idx[k] = (int)f;
        if (f == list_f) {
            T.fields[k].kind = SPEC_KIND_LIST;
            T.fields[k].elem = SPEC_KIND_MESSAGE;
            list_tf = (int)k++;
            for (uint32_t g = 0; g < ni; g++, k++) { // the items' fields, pre-order under the list
                T.fields[k].tag = schema->item.fields[g].tag;
                T.fields[k].kind = schema->item.fields[g].kind;
                T.fields[k].parent = (int16_t)list_tf;
                half[k] = 1;
                idx[k] = (int)g;
            }
        } else {
            T.fields[k++].kind = F.kind;
        }
    }
    T.nfields = k;
    std::vector<spec_tree_table> tables(SPEC_TREE_MAX_TABLES);
    std::vector<spec_tree_column> cols(SPEC_TREE_MAX_COLUMNS);
    uint32_t nt = 0, nc = 0;
    if (spec_tree_layout(&T, tables.data(), &nt, cols.data(), &nc) || nt != 2) return SPEC_E_INVALID_ARGUMENT;
    const uint64_t rows[2] = {n, nitems};
    const size_t tws = (spec_encode_tree_workspace_size(&T, rows) + 255) & ~(size_t)255;
    uint8_t *scratch = nullptr;
    if (hipMallocAsync((void **)&scratch, tws + std::max<uint64_t>(n, 1), st) != hipSuccess) return hip_rc(hipGetLastError());
    uint8_t *present = scratch + tws;
    std::vector<const void *> tc(nc, nullptr);
    std::vector<const uint8_t *> th(nc, nullptr);
    std::vector<uint64_t> tl(nc, 0);
    for (uint32_t c = 0; c < nc; c++) {
        const spec_tree_column &C = cols[c];
        if (C.role == SPEC_COL_PRESENT) {
            tc[c] = present;
        } else if (C.role == SPEC_COL_BEGIN) {
            tc[c] = item_begin;
        } else if (C.role == SPEC_COL_VALUE) {
            const int f = idx[C.field];
            tc[c] = half[C.field] ? (item_columns ? item_columns[f] : nullptr) : outer_columns[f];
            th[c] = half[C.field] ? (item_heaps ? item_heaps[f] : nullptr) : (outer_heaps ? outer_heaps[f] : nullptr);
            tl[c] = half[C.field] ? (item_heap_lens ? item_heap_lens[f] : 0) : (outer_heap_lens ? outer_heap_lens[f] : 0);
        }
    }
    int rc = SPEC_OK;
    if (hipMemsetAsync(present, 1, std::max<uint64_t>(n, 1), st) != hipSuccess) rc = hip_rc(hipGetLastError());
    if (!rc)
        rc = spec_encode_tree(&T, tc.data(), th.data(), tl.data(), rows, out, out_cap, ends, scratch, tws, total, st);
    if (hipFreeAsync(scratch, st) != hipSuccess && !rc) rc = hip_rc(hipGetLastError());
    return rc;
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
    if (schema->outer.nfields > SPEC_KFIELDS || schema->item.nfields > SPEC_KFIELDS) {
        for (uint32_t f = 0; f < schema->outer.nfields && n; f++)
            if (f != list_f && !outer_columns[f]) return SPEC_E_INVALID_ARGUMENT;
        return nested_encode_wide(schema, list_f, outer_columns, outer_heaps, outer_heap_lens, item_begin, item_columns,
                                  item_heaps, item_heap_lens, nitems, n, out, out_cap, ends, total, (hipStream_t)stream);
    }
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

size_t spec_encode_flat_workspace_size(uint64_t n) { return enc_ws_sums(n) + WIDE_FIELDS_BYTES; }

int spec_encode_flat_size(const spec_schema *schema, const void *const *columns, uint64_t n,
                          void *workspace, size_t workspace_size, uint64_t *total, void *stream) {
    int rc = check_schema(schema);
    if (rc) return rc;
    if (!columns || !workspace) return SPEC_E_INVALID_ARGUMENT;
    if (workspace_size < spec_encode_flat_workspace_size(n)) return SPEC_E_WORKSPACE;
    if (schema->nfields > SPEC_KFIELDS) {
        spec::WideEncodeArgs w{};
        if ((rc = fill_wide_encode_args(w, schema, columns, nullptr, nullptr, n, workspace, (hipStream_t)stream)))
            return rc;
        w.block_sums = (uint64_t *)workspace;
        w.total = total;
        if (spec::launch_encode_wide_size(w, (hipStream_t)stream)) return hip_rc(hipGetLastError());
        return SPEC_OK;
    }
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
