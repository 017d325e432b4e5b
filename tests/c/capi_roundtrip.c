/* capi_roundtrip.c — drives libspec_amd.so through include/spec_amd.h only (no torch), the
 * way a cgo binding would: device/pinned buffers, a stream, H2D copies,
 * spec_decode_flat, D2H; then spec_encode_flat from the decoded columns.  The CPU oracle
 * (test infrastructure) writes the input records and checks both directions bit for bit.
 * Exit 0 = pass.  Built and run by tests/test_gpu_capi.py. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "spec_amd.h"
#include "spec_oracle.h"

#define CHECK(x)                                                                          \
    do {                                                                                  \
        int rc_ = (x);                                                                    \
        if (rc_ != 0) {                                                                   \
            fprintf(stderr, "%s:%d: %s -> %d (%s, hip=%d)\n", __FILE__, __LINE__, #x, rc_, \
                    spec_strerror(rc_), spec_last_hip_error());                           \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

int main(void) {
    const uint64_t n = 10007;
    /* the load-time check a binding makes (the Go init()) */
    if (spec_abi_version() != SPEC_AMD_ABI_VERSION || spec_struct_size(SPEC_ABI_SCHEMA) != sizeof(spec_schema) ||
        spec_struct_offset(SPEC_ABI_NESTED_SCHEMA, 1) != offsetof(spec_nested_schema, item)) {
        fprintf(stderr, "ABI mismatch\n");
        return 1;
    }
    /* schema: 1 int64, 2 string, 5 float64, 9 bool, 300 uint32 (big table) */
    spec_schema s;
    memset(&s, 0, sizeof(s));
    const uint16_t tags[5] = {1, 2, 5, 9, 300};
    const uint8_t kinds[5] = {SPEC_KIND_INT64, SPEC_KIND_STRING, SPEC_KIND_FLOAT64, SPEC_KIND_BOOL, SPEC_KIND_UINT32};
    s.nfields = 5;
    for (int f = 0; f < 5; f++) {
        s.fields[f].tag = tags[f];
        s.fields[f].kind = kinds[f];
    }
    /* input columns */
    int64_t *c_i64 = malloc(n * 8);
    uint32_t *c_str = malloc(n * 8);
    double *c_f64 = malloc(n * 8);
    uint8_t *c_b = malloc(n);
    uint32_t *c_u32 = malloc(n * 4);
    uint8_t *heap = malloc(n * 40);
    uint64_t hp = 0, x = 0x5EC0DE;
    for (uint64_t i = 0; i < n; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        c_i64[i] = (int64_t)x >> (x & 63);
        uint32_t len = (uint32_t)(x >> 59) + (i % 3);
        c_str[2 * i] = (uint32_t)hp;
        c_str[2 * i + 1] = len;
        for (uint32_t k = 0; k < len; k++) heap[hp++] = (uint8_t)('a' + (x >> (k % 50)) % 26);
        c_f64[i] = (double)(int64_t)x / 3.0;
        c_b[i] = (uint8_t)(x >> 7) & 1;
        c_u32[i] = (uint32_t)(x >> 20);
    }
    const void *cols[5] = {c_i64, c_str, c_f64, c_b, c_u32};
    const uint8_t *heaps[5] = {NULL, heap, NULL, NULL, NULL};
    uint64_t cap = n * 128 + hp, *ends = malloc(n * 8);
    uint8_t *stream = malloc(cap);
    if (so_encode_flat_batch(5, tags, kinds, cols, heaps, n, stream, cap, ends) != 0) return 2;
    const uint64_t total = ends[n - 1];

    /* device round trip through the C ABI only */
    void *st, *d_stream, *d_ends, *d_cols[5], *d_status, *h_stream, *h_ends;
    CHECK(spec_set_device(0));
    CHECK(spec_stream_create(&st));
    CHECK(spec_host_alloc(total, &h_stream));
    CHECK(spec_host_alloc(n * 8, &h_ends));
    memcpy(h_stream, stream, total);
    memcpy(h_ends, ends, n * 8);
    CHECK(spec_device_alloc(total, &d_stream));
    CHECK(spec_device_alloc(n * 8, &d_ends));
    CHECK(spec_device_alloc(n, &d_status));
    for (int f = 0; f < 5; f++) CHECK(spec_device_alloc(n * (uint64_t)spec_kind_width(kinds[f]), &d_cols[f]));
    CHECK(spec_copy_h2d(d_stream, h_stream, total, st));
    CHECK(spec_copy_h2d(d_ends, h_ends, n * 8, st));
    CHECK(spec_decode_flat(&s, d_stream, total, d_ends, n, d_cols, d_status, st));
    uint8_t *got[5], *want[5], *gst = malloc(n), *wst = malloc(n);
    void *wcols[5];
    for (int f = 0; f < 5; f++) {
        size_t b = n * (uint64_t)spec_kind_width(kinds[f]);
        got[f] = malloc(b);
        want[f] = malloc(b);
        wcols[f] = want[f];
        CHECK(spec_copy_d2h(got[f], d_cols[f], b, st));
    }
    CHECK(spec_copy_d2h(gst, d_status, n, st));
    CHECK(spec_stream_sync(st));
    so_decode_flat_batch(5, tags, kinds, stream, ends, n, wcols, wst, 4);
    if (memcmp(gst, wst, n)) {
        fprintf(stderr, "status mismatch\n");
        return 3;
    }
    for (int f = 0; f < 5; f++)
        if (memcmp(got[f], want[f], n * (uint64_t)spec_kind_width(kinds[f]))) {
            fprintf(stderr, "decode column %d mismatch\n", f);
            return 3;
        }

    /* the host pipeline (pinned host in, pinned host out, chunk-major outputs) */
    spec_host_decoder *hd = NULL;
    CHECK(spec_host_decoder_create(&s, n, total, 7, &hd));
    void *h_out;
    const uint64_t out_bytes = spec_host_decoder_out_bytes(hd, n);
    CHECK(spec_host_alloc(out_bytes, &h_out));
    CHECK(spec_host_decoder_run(hd, h_stream, total, h_ends, n, h_out));
    for (uint32_t k = 0; k < 7; k++) {
        uint64_t r0, r1, offs[5], soff;
        CHECK(spec_host_decoder_chunk(hd, n, k, &r0, &r1, offs, &soff));
        if (memcmp((uint8_t *)h_out + soff, wst + r0, r1 - r0)) {
            fprintf(stderr, "host pipeline status mismatch (chunk %u)\n", k);
            return 5;
        }
        for (int f = 0; f < 5; f++) {
            const uint64_t w = (uint64_t)spec_kind_width(kinds[f]);
            if (memcmp((uint8_t *)h_out + offs[f], want[f] + r0 * w, (r1 - r0) * w)) {
                fprintf(stderr, "host pipeline column %d mismatch (chunk %u)\n", f, k);
                return 5;
            }
        }
    }
    spec_host_decoder_destroy(hd);
    CHECK(spec_host_free(h_out));

    /* encode on the device from the input columns: bytes must equal the oracle Writer's */
    void *d_in[5], *d_heap, *d_out, *d_ends2, *d_ws, *d_total;
    for (int f = 0; f < 5; f++) {
        size_t b = n * (uint64_t)spec_kind_width(kinds[f]);
        CHECK(spec_device_alloc(b, &d_in[f]));
        CHECK(spec_copy_h2d(d_in[f], cols[f], b, st));
    }
    CHECK(spec_device_alloc(hp, &d_heap));
    CHECK(spec_copy_h2d(d_heap, heap, hp, st));
    size_t ws = spec_encode_flat_workspace_size(n);
    CHECK(spec_device_alloc(ws, &d_ws));
    CHECK(spec_device_alloc(8, &d_total));
    CHECK(spec_device_alloc(total, &d_out));
    CHECK(spec_device_alloc(n * 8, &d_ends2));
    const uint8_t *d_heaps[5] = {NULL, d_heap, NULL, NULL, NULL};
    const uint64_t heap_lens[5] = {0, hp, 0, 0, 0};
    CHECK(spec_encode_flat(&s, (const void *const *)d_in, d_heaps, heap_lens, n, d_out, total, d_ends2, d_ws, ws,
                           d_total, st));
    uint8_t *out = malloc(total);
    uint64_t *ends2 = malloc(n * 8), tot2 = 0;
    CHECK(spec_copy_d2h(out, d_out, total, st));
    CHECK(spec_copy_d2h(ends2, d_ends2, n * 8, st));
    CHECK(spec_copy_d2h(&tot2, d_total, 8, st));
    CHECK(spec_stream_sync(st));
    if (tot2 != total || memcmp(ends2, ends, n * 8) || memcmp(out, stream, total)) {
        fprintf(stderr, "encode mismatch (total %llu vs %llu)\n", (unsigned long long)tot2, (unsigned long long)total);
        return 4;
    }
    printf("capi roundtrip ok: %llu records, %llu bytes\n", (unsigned long long)n, (unsigned long long)total);
    return 0;
}
