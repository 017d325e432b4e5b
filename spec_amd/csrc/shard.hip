// shard.hip — one host process driving several MI355X (include/spec_amd.h spec_shard_*):
// a batch's records split into contiguous shards (records are independent: SURVEY.md §8(e)),
// one stream and one RCCL communicator per device (ncclCommInitAll), and per device:
//   decode  — a device-resident shard into ONE packed buffer (its columns back to back, each
//             256-byte aligned, then the status bytes); from host memory, the shard is copied
//             in record chunks (pinned staging for pageable sources) with each chunk's decode
//             ordered after its copy, one host thread per device;
//   gather  — one grouped RCCL send/recv of every packed buffer to a root device over xGMI;
//   encode  — the flat encoder's size and write passes on every device (a record's bytes do not
//             depend on its offset: internal/writer/writer.go:520-553 ->
//             internal/encode/msg.go:15-77 per record), the host waiting for the size passes
//             only; one N-entry scan of the shard totals on the host (the shards' byte bases)
//             while the write passes run, then each shard's end offsets moved by its base;
//   host    — host batch in, host columns out: a spec_host_decoder per device (H2D / decode /
//             D2H overlapped in chunks), all devices at once on their own host threads.
// The reference has no multi-device code; this is what a Go host calls through cgo
//  instead of N processes.
//
// RCCL is loaded on first use (dlopen): inside a process that already holds an RCCL (torch's),
// that copy is reused, so both talk to the same HIP runtime.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>

#include "../../include/spec_amd.h"
#include "spec_internal.hpp"

namespace spec {
int host_decoder_run_based(spec_host_decoder *d, const uint8_t *stream_host, uint64_t stream_len,
                           const uint64_t *ends_host, uint64_t n, uint64_t ends_base, uint8_t *out_host);
} // namespace spec

namespace {

// ---- the RCCL entry points used (rccl.h: ncclGetVersion, ncclCommInitAll, ncclSend, ncclRecv) ----
typedef void *nccl_comm_t;
typedef int nccl_result_t; // ncclSuccess = 0
enum { NCCL_UINT8 = 1 };   // ncclUint8 (ncclDataType_t, rccl.h)

struct Rccl {
    nccl_result_t (*get_version)(int *) = nullptr;
    nccl_result_t (*comm_init_all)(nccl_comm_t *, int, const int *) = nullptr;
    nccl_result_t (*comm_destroy)(nccl_comm_t) = nullptr;
    nccl_result_t (*group_start)() = nullptr;
    nccl_result_t (*group_end)() = nullptr;
    nccl_result_t (*send)(const void *, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
    nccl_result_t (*recv)(void *, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
    bool ok = false;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // an RCCL already in the process first (torch links librccl.so.1), then the ROCm one
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        r.get_version = (decltype(r.get_version))dlsym(h, "ncclGetVersion");
        r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.send = (decltype(r.send))dlsym(h, "ncclSend");
        r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
        r.ok = r.get_version && r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.send && r.recv;
    });
    return r;
}

constexpr uint64_t PACK_ALIGN = 256;
constexpr uint32_t MAX_CHUNKS = 64;

uint64_t align_up(uint64_t x) { return (x + PACK_ALIGN - 1) / PACK_ALIGN * PACK_ALIGN; }

// Restores the calling thread's current device on scope exit.
struct DeviceGuard {
    int prev = 0;
    bool have = false;
    DeviceGuard() { have = hipGetDevice(&prev) == hipSuccess; }
    ~DeviceGuard() {
        if (have) (void)hipSetDevice(prev);
    }
};

int hip_err(hipError_t e) {
    spec::note_hip_error(e);
    return SPEC_E_HIP;
}

bool is_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

__global__ void rebase_ends_kernel(uint64_t *ends, uint64_t n, uint64_t base) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        ends[i] -= base;
}

// Per-device state.
struct Dev {
    int dev = 0;
    hipStream_t st = nullptr;   // decode / encode / gather
    hipStream_t s_in = nullptr; // host -> device copies of spec_shard_decode_host
    nccl_comm_t comm = nullptr;
    void *buf = nullptr;        // spec_shard_decode_host: the shard's ends, then its bytes
    size_t cap = 0;
    void *pin[2] = {nullptr, nullptr}; // pinned staging slots for pageable host sources
    size_t pin_cap = 0;
    hipEvent_t ev_in[MAX_CHUNKS] = {};
    hipEvent_t ev_done = nullptr; // gather without a communicator: the part is ready
    hipEvent_t ev_drained = nullptr; // decode_host: the previous call's decodes (readers of buf)
    void *ws = nullptr;         // encode workspace (block sums), then the total
    size_t ws_cap = 0;
    spec_host_decoder *hd = nullptr;
};

} // namespace

namespace spec {
int launch_rebase_ends(uint64_t *ends, uint64_t n, uint64_t base, hipStream_t stream) {
    if (!n) return 0;
    const unsigned blocks = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(rebase_ends_kernel, dim3(blocks), dim3(256), 0, stream, ends, n, base);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
} // namespace spec

struct spec_shard {
    int ndev = 0;
    uint32_t flags = 0;
    uint32_t chunks = 8;
    uint32_t split = SPEC_SHARD_SPLIT_RECORDS;
    Dev d[SPEC_SHARD_MAX_DEVICES];
    uint64_t *host_totals = nullptr; // pinned: the encode size passes' totals
};

namespace {

// Grow device i's staging buffer to `need` bytes (after its streams drained).
int ensure_buf(Dev &D, size_t need) {
    if (need <= D.cap) return SPEC_OK;
    hipError_t e;
    if ((e = hipStreamSynchronize(D.st)) != hipSuccess || (e = hipStreamSynchronize(D.s_in)) != hipSuccess)
        return hip_err(e);
    if (D.buf) (void)hipFree(D.buf);
    D.buf = nullptr;
    D.cap = 0;
    if ((e = hipMalloc(&D.buf, need)) != hipSuccess) return hip_err(e);
    D.cap = need;
    return SPEC_OK;
}

int ensure_pin(Dev &D, size_t need) {
    if (need <= D.pin_cap) return SPEC_OK;
    hipError_t e;
    if ((e = hipStreamSynchronize(D.s_in)) != hipSuccess) return hip_err(e);
    for (void *&p : D.pin) {
        if (p) (void)hipHostFree(p);
        p = nullptr;
    }
    D.pin_cap = 0;
    for (void *&p : D.pin)
        if ((e = hipHostMalloc(&p, need, hipHostMallocDefault)) != hipSuccess) return hip_err(e);
    D.pin_cap = need;
    return SPEC_OK;
}

// Device i's part of spec_shard_decode_host: records [R0, R1) of the batch, bytes [B0, B1).
int decode_host_dev(spec_shard *c, int i, const spec_schema *schema, const uint8_t *stream_host,
                    const uint64_t *ends_host, uint64_t R0, uint64_t R1, uint64_t B0, uint64_t B1, uint8_t *packed,
                    bool staged) {
    Dev &D = c->d[i];
    hipError_t e;
    if ((e = hipSetDevice(D.dev)) != hipSuccess) return hip_err(e);
    const uint64_t ns = R1 - R0, len = B1 - B0;
    const uint64_t eb = align_up(ns * 8);
    int rc = ensure_buf(D, eb + len + 16);
    if (rc) return rc;
    uint64_t *de = (uint64_t *)D.buf;
    uint8_t *ds = (uint8_t *)D.buf + eb;
    uint64_t offs[SPEC_MAX_FIELDS], soff;
    spec_packed_layout(schema, ns, offs, &soff);
    void *cols[SPEC_MAX_FIELDS];
    for (uint32_t f = 0; f < schema->nfields; f++) cols[f] = packed + offs[f];
    if (ns == 0) return SPEC_OK;
    const uint32_t nch = (uint32_t)std::min<uint64_t>(std::min<uint32_t>(c->chunks, MAX_CHUNKS), ns);
    if (staged) {
        // the previous call's copies out of the slots have drained before they are refilled
        if ((e = hipStreamSynchronize(D.s_in)) != hipSuccess) return hip_err(e);
        size_t slot = 0;
        for (uint32_t k = 0; k < nch; k++) {
            const uint64_t r0 = ns * k / nch, r1 = ns * (k + 1) / nch;
            if (r1 == r0) continue;
            const uint64_t a0 = r0 ? ends_host[R0 + r0 - 1] : B0, a1 = ends_host[R0 + r1 - 1];
            slot = std::max<size_t>(slot, align_up((r1 - r0) * 8) + (a1 > a0 ? a1 - a0 : 0));
        }
        if ((rc = ensure_pin(D, slot))) return rc;
    }
    // this call's copies overwrite buf, which the previous call's decodes (on st) may still
    // read: order them after those decodes (no host wait: back-to-back
    // calls need no spec_shard_sync between them)
    if ((e = hipEventRecord(D.ev_drained, D.st)) != hipSuccess || (e = hipStreamWaitEvent(D.s_in, D.ev_drained, 0)) != hipSuccess)
        return hip_err(e);
    for (uint32_t k = 0; k < nch; k++) {
        const uint64_t r0 = ns * k / nch, r1 = ns * (k + 1) / nch;
        if (r1 == r0) continue;
        const uint64_t a0 = r0 ? ends_host[R0 + r0 - 1] : B0, a1 = ends_host[R0 + r1 - 1];
        if (a0 < B0 || a1 < a0 || a1 > B1) return SPEC_E_INVALID_ARGUMENT;
        const uint64_t b0 = a0 - B0, b1 = a1 - B0;
        const void *se = ends_host + R0 + r0;
        const void *ss = stream_host + a0;
        if (!D.ev_in[k] && (e = hipEventCreateWithFlags(&D.ev_in[k], hipEventDisableTiming)) != hipSuccess)
            return hip_err(e);
        if (staged) {
            uint8_t *p = (uint8_t *)D.pin[k & 1];
            if (k >= 2 && (e = hipEventSynchronize(D.ev_in[k - 2])) != hipSuccess) return hip_err(e);
            memcpy(p, se, (r1 - r0) * 8);
            memcpy(p + align_up((r1 - r0) * 8), ss, b1 - b0);
            se = p;
            ss = p + align_up((r1 - r0) * 8);
        }
        if ((e = hipMemcpyAsync(de + r0, se, (r1 - r0) * 8, hipMemcpyHostToDevice, D.s_in)) != hipSuccess)
            return hip_err(e);
        if (b1 > b0 && (e = hipMemcpyAsync(ds + b0, ss, b1 - b0, hipMemcpyHostToDevice, D.s_in)) != hipSuccess)
            return hip_err(e);
        if (B0 && spec::launch_rebase_ends(de + r0, r1 - r0, B0, D.s_in)) return hip_err(hipGetLastError());
        if ((e = hipEventRecord(D.ev_in[k], D.s_in)) != hipSuccess || (e = hipStreamWaitEvent(D.st, D.ev_in[k], 0)) != hipSuccess)
            return hip_err(e);
        rc = spec_decode_flat_range(schema, ds, len, de, r0, r1, b1 - b0, cols, packed + soff, (void *)D.st);
        if (rc) return rc;
    }
    return SPEC_OK;
}

// Shard i's first record under the shard's split mode (i == ndev: n).
void shard_split(const spec_shard *c, const uint64_t *ends, uint64_t n, int i, uint64_t *r0) {
    if (c->split == SPEC_SHARD_SPLIT_BYTES) spec_shard_bounds_bytes(ends, n, c->ndev, i, r0, nullptr);
    else spec_shard_bounds(n, c->ndev, i, r0, nullptr);
}

// Run fn(i) for every device, each on its own host thread (inline for one device); returns the
// first device's non-zero code.
template <class F>
int per_device(int ndev, F fn) {
    if (ndev == 1) return fn(0);
    int rcs[SPEC_SHARD_MAX_DEVICES] = {0};
    std::thread th[SPEC_SHARD_MAX_DEVICES];
    for (int i = 0; i < ndev; i++) th[i] = std::thread([&, i] { rcs[i] = fn(i); });
    for (int i = 0; i < ndev; i++) th[i].join();
    for (int i = 0; i < ndev; i++)
        if (rcs[i]) return rcs[i];
    return SPEC_OK;
}

} // namespace

extern "C" {

uint64_t spec_packed_layout(const spec_schema *schema, uint64_t n, uint64_t *col_offsets, uint64_t *status_offset) {
    if (!schema || schema->nfields > SPEC_MAX_FIELDS) return 0;
    uint64_t off = 0;
    for (uint32_t f = 0; f < schema->nfields; f++) {
        if (col_offsets) col_offsets[f] = off;
        const uint64_t w = (uint64_t)spec_kind_width(schema->fields[f].kind);
        off = align_up(off + n * w);
    }
    if (status_offset) *status_offset = off;
    return off + n;
}

void spec_shard_bounds(uint64_t n, int nshards, int k, uint64_t *r0, uint64_t *r1) {
    if (nshards < 1) nshards = 1;
    const unsigned __int128 N = n;
    if (r0) *r0 = (uint64_t)(N * (unsigned)k / (unsigned)nshards);
    if (r1) *r1 = (uint64_t)(N * (unsigned)(k + 1) / (unsigned)nshards);
}

void spec_shard_bounds_bytes(const uint64_t *ends, uint64_t n, int nshards, int k, uint64_t *r0, uint64_t *r1) {
    if (nshards < 1) nshards = 1;
    // split point j: the record boundary nearest to byte quantile total * j / nshards
    auto split = [&](int j) -> uint64_t {
        if (j <= 0 || !n || !ends) return 0;
        if (j >= nshards) return n;
        const uint64_t q = (uint64_t)((unsigned __int128)ends[n - 1] * (unsigned)j / (unsigned)nshards);
        const uint64_t i = (uint64_t)(std::lower_bound(ends, ends + n, q) - ends); // first end >= q
        if (i >= n) return n;
        const uint64_t below = i ? ends[i - 1] : 0; // records [0, i) end at or below q
        return ends[i] - q <= q - below ? i + 1 : i;
    };
    if (r0) *r0 = split(k);
    if (r1) *r1 = split(k + 1);
}

int spec_shard_set_split(spec_shard *c, uint32_t split) {
    if (!c || split > SPEC_SHARD_SPLIT_BYTES) return SPEC_E_INVALID_ARGUMENT;
    c->split = split;
    return SPEC_OK;
}

int spec_shard_create_ex(const int *devices, int ndev, uint32_t flags, spec_shard **out) {
    if (!out || !devices || ndev < 1 || ndev > SPEC_SHARD_MAX_DEVICES) return SPEC_E_INVALID_ARGUMENT;
    if (flags & ~(uint32_t)(SPEC_SHARD_FORCE_COMM | SPEC_SHARD_SHARED)) return SPEC_E_INVALID_ARGUMENT;
    if ((flags & SPEC_SHARD_FORCE_COMM) && (flags & SPEC_SHARD_SHARED)) return SPEC_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (!(flags & SPEC_SHARD_SHARED))
        for (int i = 0; i < ndev; i++)
            for (int j = 0; j < i; j++)
                if (devices[i] == devices[j]) return SPEC_E_INVALID_ARGUMENT; // one communicator rank per GPU
    spec_shard *c = new (std::nothrow) spec_shard();
    if (!c) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    c->ndev = ndev;
    c->flags = flags;
    hipError_t e = hipSuccess;
    for (int i = 0; i < ndev; i++) {
        Dev &D = c->d[i];
        D.dev = devices[i];
        if ((e = hipSetDevice(devices[i])) != hipSuccess ||
            (e = hipStreamCreateWithFlags(&D.st, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipStreamCreateWithFlags(&D.s_in, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&D.ev_done, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&D.ev_drained, hipEventDisableTiming)) != hipSuccess) {
            spec_shard_destroy(c);
            return hip_err(e);
        }
    }
    if ((e = hipHostMalloc((void **)&c->host_totals, SPEC_SHARD_MAX_DEVICES * sizeof(uint64_t), hipHostMallocDefault)) !=
        hipSuccess) {
        c->host_totals = nullptr;
        spec_shard_destroy(c);
        return hip_err(e);
    }
    if ((ndev > 1 && !(flags & SPEC_SHARD_SHARED)) || (flags & SPEC_SHARD_FORCE_COMM)) {
        const Rccl &r = rccl();
        nccl_comm_t comms[SPEC_SHARD_MAX_DEVICES] = {nullptr};
        int devs[SPEC_SHARD_MAX_DEVICES];
        for (int i = 0; i < ndev; i++) devs[i] = devices[i];
        if (!r.ok || r.comm_init_all(comms, ndev, devs) != 0) {
            spec_shard_destroy(c);
            return SPEC_E_HIP;
        }
        for (int i = 0; i < ndev; i++) c->d[i].comm = comms[i];
    }
    *out = c;
    return SPEC_OK;
}

int spec_shard_create(const int *devices, int ndev, spec_shard **out) {
    return spec_shard_create_ex(devices, ndev, 0, out);
}

void spec_shard_destroy(spec_shard *c) {
    if (!c) return;
    DeviceGuard g;
    for (int i = 0; i < c->ndev; i++) {
        Dev &D = c->d[i];
        if (hipSetDevice(D.dev) != hipSuccess) continue;
        if (D.hd) spec_host_decoder_destroy(D.hd);
        if (D.st) {
            (void)hipStreamSynchronize(D.st);
            (void)hipStreamDestroy(D.st);
        }
        if (D.s_in) {
            (void)hipStreamSynchronize(D.s_in);
            (void)hipStreamDestroy(D.s_in);
        }
        for (hipEvent_t &ev : D.ev_in)
            if (ev) (void)hipEventDestroy(ev);
        if (D.ev_done) (void)hipEventDestroy(D.ev_done);
        if (D.ev_drained) (void)hipEventDestroy(D.ev_drained);
        for (void *p : D.pin)
            if (p) (void)hipHostFree(p);
        if (D.buf) (void)hipFree(D.buf);
        if (D.ws) (void)hipFree(D.ws);
        if (D.comm && rccl().ok) rccl().comm_destroy(D.comm);
    }
    if (c->host_totals) (void)hipHostFree(c->host_totals);
    delete c;
}

int spec_shard_ndev(const spec_shard *c) { return c ? c->ndev : 0; }

int spec_shard_has_comm(const spec_shard *c) { return c && c->d[0].comm ? 1 : 0; }

int spec_shard_rccl_version(void) {
    const Rccl &r = rccl();
    int v = 0;
    if (!r.ok || r.get_version(&v) != 0) return -1;
    return v;
}

int spec_shard_set_chunks(spec_shard *c, uint32_t chunks) {
    if (!c || chunks < 1 || chunks > MAX_CHUNKS) return SPEC_E_INVALID_ARGUMENT;
    c->chunks = chunks;
    return SPEC_OK;
}

void *spec_shard_stream(const spec_shard *c, int k) {
    return c && k >= 0 && k < c->ndev ? (void *)c->d[k].st : nullptr;
}

int spec_shard_decode(spec_shard *c, const spec_schema *schema, const uint8_t *const *streams,
                      const uint64_t *stream_lens, const uint64_t *const *ends, const uint64_t *ns,
                      uint8_t *const *packed) {
    if (!c || !schema || !streams || !stream_lens || !ends || !ns || !packed) return SPEC_E_INVALID_ARGUMENT;
    if (schema->nfields == 0 || schema->nfields > SPEC_MAX_FIELDS) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    for (int i = 0; i < c->ndev; i++) {
        hipError_t e;
        if ((e = hipSetDevice(c->d[i].dev)) != hipSuccess) return hip_err(e);
        uint64_t offs[SPEC_MAX_FIELDS], soff;
        spec_packed_layout(schema, ns[i], offs, &soff);
        void *cols[SPEC_MAX_FIELDS];
        for (uint32_t f = 0; f < schema->nfields; f++) cols[f] = packed[i] + offs[f];
        const int rc = spec_decode_flat(schema, streams[i], stream_lens[i], ends[i], ns[i], cols, packed[i] + soff,
                                        (void *)c->d[i].st);
        if (rc) return rc;
    }
    return SPEC_OK;
}

int spec_shard_decode_host(spec_shard *c, const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                           const uint64_t *ends, uint64_t n, uint8_t *const *packed, uint64_t *byte_bases) {
    if (!c || !schema || (n && (!stream_bytes || !ends)) || !packed) return SPEC_E_INVALID_ARGUMENT;
    if (schema->nfields == 0 || schema->nfields > SPEC_MAX_FIELDS) return SPEC_E_INVALID_ARGUMENT;
    uint64_t R[SPEC_SHARD_MAX_DEVICES + 1], B[SPEC_SHARD_MAX_DEVICES + 1];
    for (int i = 0; i <= c->ndev; i++) {
        shard_split(c, ends, n, i, &R[i]);
        B[i] = R[i] ? ends[R[i] - 1] : 0;
        if ((i && (R[i] < R[i - 1] || B[i] < B[i - 1])) || B[i] > stream_len) return SPEC_E_INVALID_ARGUMENT;
        if (byte_bases && i < c->ndev) byte_bases[i] = B[i];
    }
    for (int i = 0; i < c->ndev; i++)
        if (B[i + 1] - B[i] >= (1ull << 32)) return SPEC_E_TOO_LARGE; // spans are shard-relative u32
    const bool staged = n && !(is_pinned(stream_bytes) && is_pinned(ends));
    DeviceGuard g;
    return per_device(c->ndev, [&](int i) {
        return decode_host_dev(c, i, schema, stream_bytes, ends, R[i], R[i + 1], B[i], B[i + 1], packed[i], staged);
    });
}

int spec_shard_gather(spec_shard *c, const uint64_t *nbytes, uint8_t *const *packed, int root, uint8_t *gathered) {
    if (!c || !nbytes || !packed || !gathered || root < 0 || root >= c->ndev) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    uint64_t off[SPEC_SHARD_MAX_DEVICES], o = 0;
    for (int i = 0; i < c->ndev; i++) {
        off[i] = o;
        o += nbytes[i];
    }
    const bool comm = c->d[root].comm != nullptr;
    hipError_t e;
    // without a communicator (one device, or SPEC_SHARD_SHARED): device copies on the root's
    // stream, each after its part's stream reached this point
    if (!comm) {
        for (int i = 0; i < c->ndev; i++) {
            if (!nbytes[i] || i == root) continue;
            if ((e = hipSetDevice(c->d[i].dev)) != hipSuccess || (e = hipEventRecord(c->d[i].ev_done, c->d[i].st)) != hipSuccess)
                return hip_err(e);
        }
        if ((e = hipSetDevice(c->d[root].dev)) != hipSuccess) return hip_err(e);
        for (int i = 0; i < c->ndev; i++) {
            if (!nbytes[i]) continue;
            if (i != root && (e = hipStreamWaitEvent(c->d[root].st, c->d[i].ev_done, 0)) != hipSuccess) return hip_err(e);
            if ((e = hipMemcpyAsync(gathered + off[i], packed[i], nbytes[i], hipMemcpyDeviceToDevice,
                                    c->d[root].st)) != hipSuccess)
                return hip_err(e);
        }
        return SPEC_OK;
    }
    // one grouped send/recv per part (RCCL over xGMI, point to point); the root's own part too
    // (a send to itself), so every byte takes the same path
    const Rccl &r = rccl();
    if (!r.ok) return SPEC_E_HIP;
    if (r.group_start() != 0) return SPEC_E_HIP;
    int bad = 0;
    for (int i = 0; i < c->ndev; i++) {
        if (!nbytes[i]) continue;
        bad |= r.send(packed[i], nbytes[i], NCCL_UINT8, root, c->d[i].comm, c->d[i].st);
        bad |= r.recv(gathered + off[i], nbytes[i], NCCL_UINT8, i, c->d[root].comm, c->d[root].st);
    }
    if (r.group_end() != 0 || bad) return SPEC_E_HIP;
    return SPEC_OK;
}

int spec_shard_encode(spec_shard *c, const spec_schema *schema, const void *const *const *columns,
                      const uint8_t *const *const *heaps, const uint64_t *const *heap_lens, const uint64_t *ns,
                      uint8_t *const *outs, const uint64_t *out_caps, uint64_t *const *ends, uint64_t *totals,
                      uint64_t *byte_bases) {
    if (!c || !schema || !columns || !ns || !outs || !out_caps || !ends) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    hipError_t e;
    int rc;
    // 1. per device: the size pass (heaps checked), its total copied to the host, then at once
    //    the write pass with shard-relative ends (a record's bytes do not depend on where the
    //    shard lands; the write pass skips everything itself when the total exceeds the capacity
    //    or is an encoder error)
    for (int i = 0; i < c->ndev; i++) {
        Dev &D = c->d[i];
        if ((e = hipSetDevice(D.dev)) != hipSuccess) return hip_err(e);
        const size_t wsb = (spec_encode_flat_workspace_size(ns[i]) + 255) & ~(size_t)255;
        if (wsb + 8 > D.ws_cap) {
            if ((e = hipStreamSynchronize(D.st)) != hipSuccess) return hip_err(e);
            if (D.ws) (void)hipFree(D.ws);
            D.ws = nullptr;
            D.ws_cap = 0;
            if ((e = hipMalloc(&D.ws, wsb + 8)) != hipSuccess) return hip_err(e);
            D.ws_cap = wsb + 8;
        }
        uint64_t *dtotal = (uint64_t *)((uint8_t *)D.ws + D.ws_cap - 8);
        const uint8_t *const *hp = heaps ? heaps[i] : nullptr;
        const uint64_t *hl = heap_lens ? heap_lens[i] : nullptr;
        if ((rc = spec::encode_flat_passes(schema, columns[i], hp, hl, ns[i], outs[i], out_caps[i], ends[i], 0, D.ws,
                                           D.ws_cap - 8, dtotal, spec::ENC_PASS_SIZE, D.st)))
            return rc;
        if ((e = hipMemcpyAsync(c->host_totals + i, dtotal, 8, hipMemcpyDeviceToHost, D.st)) != hipSuccess ||
            (e = hipEventRecord(D.ev_done, D.st)) != hipSuccess)
            return hip_err(e);
        if ((rc = spec::encode_flat_passes(schema, columns[i], hp, hl, ns[i], outs[i], out_caps[i], ends[i], 0, D.ws,
                                           D.ws_cap - 8, dtotal, spec::ENC_PASS_WRITE, D.st)))
            return rc;
    }
    // 2. the totals (the host waits for the size passes only; the write passes keep running):
    //    the shards' byte bases are their exclusive scan
    for (int i = 0; i < c->ndev; i++)
        if ((e = hipEventSynchronize(c->d[i].ev_done)) != hipSuccess) return hip_err(e);
    uint64_t base[SPEC_SHARD_MAX_DEVICES], o = 0;
    rc = SPEC_OK;
    for (int i = 0; i < c->ndev; i++) {
        const uint64_t t = c->host_totals[i];
        if (totals) totals[i] = t;
        base[i] = o;
        if (byte_bases) byte_bases[i] = o;
        if (t == ~0ull) rc = SPEC_E_ENCODE;
        else if (t > out_caps[i] && rc == SPEC_OK) rc = SPEC_E_CAPACITY;
        o += t == ~0ull ? 0 : t;
    }
    // a shard over its capacity or in error wrote nothing (its write pass checks its own total);
    // the shards that fit hold their bytes, with shard-relative ends
    if (rc) return rc;
    // 3. every shard's ends moved to the whole batch, after its write pass
    for (int i = 0; i < c->ndev; i++) {
        if (!base[i] || !ns[i]) continue;
        if ((e = hipSetDevice(c->d[i].dev)) != hipSuccess) return hip_err(e);
        if (spec::launch_rebase_ends(ends[i], ns[i], (uint64_t)0 - base[i], c->d[i].st)) return hip_err(hipGetLastError());
    }
    return SPEC_OK;
}

int spec_shard_host_prepare(spec_shard *c, const spec_schema *schema, uint64_t n_cap, uint64_t stream_cap,
                            uint32_t chunks) {
    if (!c || !schema) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    for (int i = 0; i < c->ndev; i++) {
        Dev &D = c->d[i];
        hipError_t e;
        if ((e = hipSetDevice(D.dev)) != hipSuccess) return hip_err(e);
        if (D.hd) spec_host_decoder_destroy(D.hd);
        D.hd = nullptr;
        const int rc = spec_host_decoder_create(schema, n_cap, stream_cap, chunks, &D.hd);
        if (rc) return rc;
    }
    return SPEC_OK;
}

spec_host_decoder *spec_shard_host_decoder(const spec_shard *c, int k) {
    return c && k >= 0 && k < c->ndev ? c->d[k].hd : nullptr;
}

int spec_shard_host_decode(spec_shard *c, const uint8_t *stream_host, uint64_t stream_len, const uint64_t *ends_host,
                           uint64_t n, uint8_t *const *out_host, uint64_t *byte_bases) {
    if (!c || (n && (!stream_host || !ends_host)) || !out_host) return SPEC_E_INVALID_ARGUMENT;
    uint64_t R[SPEC_SHARD_MAX_DEVICES + 1], B[SPEC_SHARD_MAX_DEVICES + 1];
    for (int i = 0; i <= c->ndev; i++) {
        if (i < c->ndev && !c->d[i].hd) return SPEC_E_INVALID_ARGUMENT; // spec_shard_host_prepare first
        shard_split(c, ends_host, n, i, &R[i]);
        B[i] = R[i] ? ends_host[R[i] - 1] : 0;
        if ((i && (R[i] < R[i - 1] || B[i] < B[i - 1])) || B[i] > stream_len) return SPEC_E_INVALID_ARGUMENT;
        if (byte_bases && i < c->ndev) byte_bases[i] = B[i];
    }
    DeviceGuard g;
    return per_device(c->ndev, [&](int i) {
        return spec::host_decoder_run_based(c->d[i].hd, stream_host + B[i], B[i + 1] - B[i], ends_host + R[i],
                                            R[i + 1] - R[i], B[i], out_host[i]);
    });
}

int spec_shard_sync(spec_shard *c) {
    if (!c) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    for (int i = 0; i < c->ndev; i++) {
        hipError_t e;
        if ((e = hipSetDevice(c->d[i].dev)) != hipSuccess || (e = hipStreamSynchronize(c->d[i].s_in)) != hipSuccess ||
            (e = hipStreamSynchronize(c->d[i].st)) != hipSuccess)
            return hip_err(e);
    }
    return SPEC_OK;
}

} // extern "C"
