// host_pipeline.cpp — spec_host_decoder_* (include/spec_amd.h): decode of a batch that starts
// and ends in host memory, the way an mpx receiver holds it (mpx/conn_reader.go:179-194:
// frames read into connection buffers, decoded messages handed back to Go code).
//
// The batch is split into `chunks` record ranges.  Three HIP streams overlap, per chunk k:
//   s_in : H2D of ends[r0, r1) and the chunk's bytes            (chunk k+1 while k decodes)
//   s_dec: spec_decode_flat_range(r0, r1) once s_in's event fires
//   s_out: ONE D2H of the chunk's output region once s_dec's event fires
// Outputs are chunk-major (columns of the chunk's records back to back, then its status), so
// the device side of chunk k is one contiguous region and leaves the device in one copy: on
// MI355X the two PCIe directions overlap only when the traffic is split into chunks, and
// every extra copy costs a launch (tools/pcie_probe.py).
#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include "../../include/spec_amd.h"

struct spec_host_decoder {
    spec_schema schema;
    uint64_t n_cap, stream_cap;
    uint32_t chunks;
    int device;
    uint8_t *d_stream;
    uint64_t *d_ends;
    uint8_t *d_out;
    uint64_t out_cap;
    hipStream_t s_in, s_dec, s_out;
    hipEvent_t *ev_in, *ev_dec; // one pair per chunk
};

namespace {

constexpr uint64_t ALIGN = 256;
uint64_t align_up(uint64_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

// chunk k of an n-record batch: records [r0, r1); offsets (bytes) of its columns and status
// relative to the start of the output buffer; returns the chunk region's end.
uint64_t chunk_layout(const spec_host_decoder *d, uint64_t n, uint32_t k, uint64_t *r0, uint64_t *r1,
                      uint64_t *col_off, uint64_t *status_off) {
    uint64_t base = 0;
    for (uint32_t j = 0;; j++) {
        const uint64_t a = n * j / d->chunks, b = n * (j + 1) / d->chunks, nk = b - a;
        uint64_t o = base;
        for (uint32_t f = 0; f < d->schema.nfields; f++) {
            if (j == k && col_off) col_off[f] = o;
            o = align_up(o + nk * (uint64_t)spec_kind_width(d->schema.fields[f].kind));
        }
        if (j == k) {
            if (r0) *r0 = a;
            if (r1) *r1 = b;
            if (status_off) *status_off = o;
            return align_up(o + nk);
        }
        base = align_up(o + nk);
    }
}

int hip_fail(hipError_t e) {
    (void)e;
    return SPEC_E_HIP;
}

} // namespace

namespace spec {
// shard.hip: ends[0, n) -= base on `stream`
int launch_rebase_ends(uint64_t *ends, uint64_t n, uint64_t base, hipStream_t stream);

// spec_host_decoder_run over a batch whose end offsets are all `ends_base` too large: a shard of
// a larger host batch (stream_host = the shard's first byte, ends_host = the shard's ends as
// they are in the whole batch).  The device copy of `ends` is rebased chunk by chunk after its
// H2D, so spans come out shard-relative.  spec_shard_host_decode runs one per device.
int host_decoder_run_based(spec_host_decoder *d, const uint8_t *stream_host, uint64_t stream_len,
                           const uint64_t *ends_host, uint64_t n, uint64_t ends_base, uint8_t *out_host);
} // namespace spec

extern "C" {

uint64_t spec_host_decoder_out_bytes(const spec_host_decoder *d, uint64_t n) {
    if (!d) return 0;
    return chunk_layout(d, n, d->chunks - 1, nullptr, nullptr, nullptr, nullptr);
}

int spec_host_decoder_chunk(const spec_host_decoder *d, uint64_t n, uint32_t k, uint64_t *r0, uint64_t *r1,
                            uint64_t *col_offsets, uint64_t *status_offset) {
    if (!d || k >= d->chunks) return SPEC_E_INVALID_ARGUMENT;
    chunk_layout(d, n, k, r0, r1, col_offsets, status_offset);
    return SPEC_OK;
}

void spec_host_decoder_destroy(spec_host_decoder *d) {
    if (!d) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(d->device);
    if (d->s_in) (void)hipStreamSynchronize(d->s_in);
    if (d->s_dec) (void)hipStreamSynchronize(d->s_dec);
    if (d->s_out) (void)hipStreamSynchronize(d->s_out);
    for (uint32_t k = 0; d->ev_in && k < d->chunks; k++) {
        if (d->ev_in[k]) (void)hipEventDestroy(d->ev_in[k]);
        if (d->ev_dec[k]) (void)hipEventDestroy(d->ev_dec[k]);
    }
    free(d->ev_in);
    free(d->ev_dec);
    if (d->s_in) (void)hipStreamDestroy(d->s_in);
    if (d->s_dec) (void)hipStreamDestroy(d->s_dec);
    if (d->s_out) (void)hipStreamDestroy(d->s_out);
    (void)hipFree(d->d_stream);
    (void)hipFree(d->d_ends);
    (void)hipFree(d->d_out);
    (void)hipSetDevice(prev);
    free(d);
}

int spec_host_decoder_create(const spec_schema *schema, uint64_t n_cap, uint64_t stream_cap, uint32_t chunks,
                             spec_host_decoder **out) {
    if (!schema || !out || chunks == 0 || schema->nfields > SPEC_MAX_FIELDS) return SPEC_E_INVALID_ARGUMENT;
    for (uint32_t f = 0; f < schema->nfields; f++)
        if (spec_kind_width(schema->fields[f].kind) == 0 || schema->fields[f].kind == SPEC_KIND_LIST)
            return SPEC_E_INVALID_ARGUMENT;
    if (stream_cap >= (1ull << 32)) return SPEC_E_TOO_LARGE;
    *out = nullptr;
    spec_host_decoder *d = (spec_host_decoder *)calloc(1, sizeof(spec_host_decoder));
    if (!d) return SPEC_E_INVALID_ARGUMENT;
    d->schema = *schema;
    d->n_cap = n_cap;
    d->stream_cap = stream_cap;
    d->chunks = chunks;
    (void)hipGetDevice(&d->device);
    // any n <= n_cap fits: sum over chunks of (columns + status), each rounded up per piece
    uint64_t rec = 1;
    for (uint32_t f = 0; f < schema->nfields; f++) rec += (uint64_t)spec_kind_width(schema->fields[f].kind);
    d->out_cap = n_cap * rec + (uint64_t)chunks * (schema->nfields + 1) * ALIGN + ALIGN;
    d->ev_in = (hipEvent_t *)calloc(chunks, sizeof(hipEvent_t));
    d->ev_dec = (hipEvent_t *)calloc(chunks, sizeof(hipEvent_t));
    hipError_t e = hipSuccess;
    if (!d->ev_in || !d->ev_dec) {
        spec_host_decoder_destroy(d);
        return SPEC_E_INVALID_ARGUMENT;
    }
    if ((e = hipMalloc(&d->d_stream, stream_cap ? stream_cap : 1)) != hipSuccess ||
        (e = hipMalloc(&d->d_ends, n_cap ? n_cap * 8 : 8)) != hipSuccess ||
        (e = hipMalloc(&d->d_out, d->out_cap)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&d->s_in, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&d->s_dec, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&d->s_out, hipStreamNonBlocking)) != hipSuccess) {
        spec_host_decoder_destroy(d);
        return hip_fail(e);
    }
    for (uint32_t k = 0; k < chunks; k++) {
        if ((e = hipEventCreateWithFlags(&d->ev_in[k], hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&d->ev_dec[k], hipEventDisableTiming)) != hipSuccess) {
            spec_host_decoder_destroy(d);
            return hip_fail(e);
        }
    }
    *out = d;
    return SPEC_OK;
}

int spec_host_decoder_run(spec_host_decoder *d, const uint8_t *stream_host, uint64_t stream_len,
                          const uint64_t *ends_host, uint64_t n, uint8_t *out_host) {
    return spec::host_decoder_run_based(d, stream_host, stream_len, ends_host, n, 0, out_host);
}

} // extern "C"

int spec::host_decoder_run_based(spec_host_decoder *d, const uint8_t *stream_host, uint64_t stream_len,
                                 const uint64_t *ends_host, uint64_t n, uint64_t ends_base, uint8_t *out_host) {
    if (!d || n > d->n_cap || stream_len > d->stream_cap) return SPEC_E_INVALID_ARGUMENT;
    if (n == 0) return SPEC_OK;
    if (!stream_host || !ends_host || !out_host) return SPEC_E_INVALID_ARGUMENT;
    if (ends_host[n - 1] < ends_base || ends_host[n - 1] - ends_base > stream_len) return SPEC_E_INVALID_ARGUMENT;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != d->device) (void)hipSetDevice(d->device);
    int rc = SPEC_OK;
    hipError_t e = hipSuccess;
    uint64_t col_off[SPEC_MAX_FIELDS], status_off = 0, base = 0;
    void *cols[SPEC_MAX_FIELDS];
    for (uint32_t k = 0; k < d->chunks && rc == SPEC_OK; k++) {
        uint64_t r0 = 0, r1 = 0;
        const uint64_t end = chunk_layout(d, n, k, &r0, &r1, col_off, &status_off);
        if (r1 > r0) {
            const uint64_t a0 = r0 ? ends_host[r0 - 1] : ends_base, a1 = ends_host[r1 - 1];
            if (a1 < a0 || a0 < ends_base) {
                rc = SPEC_E_INVALID_ARGUMENT;
                break;
            }
            const uint64_t b0 = a0 - ends_base, b1 = a1 - ends_base;
            if ((e = hipMemcpyAsync(d->d_ends + r0, ends_host + r0, (r1 - r0) * 8, hipMemcpyHostToDevice,
                                    d->s_in)) != hipSuccess ||
                (b1 > b0 && (e = hipMemcpyAsync(d->d_stream + b0, stream_host + b0, b1 - b0, hipMemcpyHostToDevice,
                                                d->s_in)) != hipSuccess)) {
                rc = hip_fail(e);
                break;
            }
            if (ends_base && spec::launch_rebase_ends(d->d_ends + r0, r1 - r0, ends_base, d->s_in)) {
                rc = SPEC_E_HIP;
                break;
            }
            if ((e = hipEventRecord(d->ev_in[k], d->s_in)) != hipSuccess ||
                (e = hipStreamWaitEvent(d->s_dec, d->ev_in[k], 0)) != hipSuccess) {
                rc = hip_fail(e);
                break;
            }
            // column f of this chunk, shifted by -r0 rows (the kernel indexes by record)
            for (uint32_t f = 0; f < d->schema.nfields; f++)
                cols[f] = d->d_out + col_off[f] - r0 * (uint64_t)spec_kind_width(d->schema.fields[f].kind);
            rc = spec_decode_flat_range(&d->schema, d->d_stream, stream_len, d->d_ends, r0, r1, b1 - b0, cols,
                                        d->d_out + status_off - r0, d->s_dec);
            if (rc != SPEC_OK) break;
            if ((e = hipEventRecord(d->ev_dec[k], d->s_dec)) != hipSuccess ||
                (e = hipStreamWaitEvent(d->s_out, d->ev_dec[k], 0)) != hipSuccess ||
                (e = hipMemcpyAsync(out_host + base, d->d_out + base, end - base, hipMemcpyDeviceToHost,
                                    d->s_out)) != hipSuccess) {
                rc = hip_fail(e);
                break;
            }
        }
        base = end;
    }
    // every stream drained before returning, also after an error (no copy outlives the call)
    hipError_t s1 = hipStreamSynchronize(d->s_in), s2 = hipStreamSynchronize(d->s_dec),
               s3 = hipStreamSynchronize(d->s_out);
    if (rc == SPEC_OK && (s1 != hipSuccess || s2 != hipSuccess || s3 != hipSuccess)) rc = SPEC_E_HIP;
    if (prev != d->device) (void)hipSetDevice(prev);
    return rc;
}
