// shard.hip — one host process driving several MI355X (include/spec_amd.h spec_shard_*):
// a batch's records split into contiguous shards (records are independent: SURVEY.md §8(e)),
// one stream and one RCCL communicator per device (ncclCommInitAll), every shard decoded on
// its device into ONE packed buffer (its columns back to back, each 256-byte aligned, then the
// status bytes), and one grouped RCCL send/recv gathering the packed buffers to a root device
// over xGMI.  The reference has no multi-device code; this is what a Go host calls through cgo
//  instead of N processes.
//
// RCCL is loaded on first use (dlopen of librccl.so), so the decode-only library does not pull
// it in.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>

#include "../../include/spec_amd.h"

namespace {

// ---- the RCCL entry points used (rccl.h: ncclCommInitAll :236, ncclSend :700, ncclRecv :722) ----
typedef void *nccl_comm_t;
typedef int nccl_result_t; // ncclSuccess = 0
enum { NCCL_UINT8 = 1 };   // ncclUint8 (ncclDataType_t)

struct Rccl {
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
        void *h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.send = (decltype(r.send))dlsym(h, "ncclSend");
        r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
        r.ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.send && r.recv;
    });
    return r;
}

constexpr uint64_t PACK_ALIGN = 256;

// Restores the calling thread's current device on scope exit.
struct DeviceGuard {
    int prev = 0;
    bool have = false;
    DeviceGuard() { have = hipGetDevice(&prev) == hipSuccess; }
    ~DeviceGuard() {
        if (have) (void)hipSetDevice(prev);
    }
};

__global__ void rebase_ends_kernel(uint64_t *ends, uint64_t n, uint64_t base) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        ends[i] -= base;
}

} // namespace

struct spec_shard {
    int ndev = 0;
    int dev[SPEC_SHARD_MAX_DEVICES] = {0};
    hipStream_t st[SPEC_SHARD_MAX_DEVICES] = {nullptr};
    nccl_comm_t comm[SPEC_SHARD_MAX_DEVICES] = {nullptr};
    // staging of spec_shard_decode_host: per device, the shard's stream bytes and ends
    void *buf[SPEC_SHARD_MAX_DEVICES] = {nullptr};
    size_t cap[SPEC_SHARD_MAX_DEVICES] = {0};
};

extern "C" {

uint64_t spec_packed_layout(const spec_schema *schema, uint64_t n, uint64_t *col_offsets, uint64_t *status_offset) {
    if (!schema || schema->nfields > SPEC_MAX_FIELDS) return 0;
    uint64_t off = 0;
    for (uint32_t f = 0; f < schema->nfields; f++) {
        if (col_offsets) col_offsets[f] = off;
        const uint64_t w = (uint64_t)spec_kind_width(schema->fields[f].kind);
        off = (off + n * w + PACK_ALIGN - 1) / PACK_ALIGN * PACK_ALIGN;
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

int spec_shard_create(const int *devices, int ndev, spec_shard **out) {
    if (!out || !devices || ndev < 1 || ndev > SPEC_SHARD_MAX_DEVICES) return SPEC_E_INVALID_ARGUMENT;
    *out = nullptr;
    for (int i = 0; i < ndev; i++)
        for (int j = 0; j < i; j++)
            if (devices[i] == devices[j]) return SPEC_E_INVALID_ARGUMENT; // one communicator rank per GPU
    spec_shard *c = new (std::nothrow) spec_shard();
    if (!c) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    c->ndev = ndev;
    for (int i = 0; i < ndev; i++) {
        c->dev[i] = devices[i];
        if (hipSetDevice(devices[i]) != hipSuccess ||
            hipStreamCreateWithFlags(&c->st[i], hipStreamNonBlocking) != hipSuccess) {
            spec_shard_destroy(c);
            return SPEC_E_HIP;
        }
    }
    if (ndev > 1) {
        const Rccl &r = rccl();
        if (!r.ok || r.comm_init_all(c->comm, ndev, c->dev) != 0) {
            spec_shard_destroy(c);
            return SPEC_E_HIP;
        }
    }
    *out = c;
    return SPEC_OK;
}

void spec_shard_destroy(spec_shard *c) {
    if (!c) return;
    DeviceGuard g;
    for (int i = 0; i < c->ndev; i++) {
        if (hipSetDevice(c->dev[i]) != hipSuccess) continue;
        if (c->st[i]) {
            (void)hipStreamSynchronize(c->st[i]);
            (void)hipStreamDestroy(c->st[i]);
        }
        if (c->buf[i]) (void)hipFree(c->buf[i]);
        if (c->comm[i] && rccl().ok) rccl().comm_destroy(c->comm[i]);
    }
    delete c;
}

int spec_shard_ndev(const spec_shard *c) { return c ? c->ndev : 0; }

void *spec_shard_stream(const spec_shard *c, int k) {
    return c && k >= 0 && k < c->ndev ? (void *)c->st[k] : nullptr;
}

int spec_shard_decode(spec_shard *c, const spec_schema *schema, const uint8_t *const *streams,
                      const uint64_t *stream_lens, const uint64_t *const *ends, const uint64_t *ns,
                      uint8_t *const *packed) {
    if (!c || !schema || !streams || !stream_lens || !ends || !ns || !packed) return SPEC_E_INVALID_ARGUMENT;
    if (schema->nfields == 0 || schema->nfields > SPEC_MAX_FIELDS) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    for (int i = 0; i < c->ndev; i++) {
        if (hipSetDevice(c->dev[i]) != hipSuccess) return SPEC_E_HIP;
        uint64_t offs[SPEC_MAX_FIELDS], soff;
        spec_packed_layout(schema, ns[i], offs, &soff);
        void *cols[SPEC_MAX_FIELDS];
        for (uint32_t f = 0; f < schema->nfields; f++) cols[f] = packed[i] + offs[f];
        const int rc = spec_decode_flat(schema, streams[i], stream_lens[i], ends[i], ns[i], cols, packed[i] + soff,
                                        (void *)c->st[i]);
        if (rc) return rc;
    }
    return SPEC_OK;
}

int spec_shard_decode_host(spec_shard *c, const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                           const uint64_t *ends, uint64_t n, uint8_t *const *packed, uint64_t *byte_bases) {
    if (!c || !schema || (n && (!stream_bytes || !ends)) || !packed) return SPEC_E_INVALID_ARGUMENT;
    const uint8_t *sp[SPEC_SHARD_MAX_DEVICES];
    const uint64_t *ep[SPEC_SHARD_MAX_DEVICES];
    uint64_t lens[SPEC_SHARD_MAX_DEVICES], ns[SPEC_SHARD_MAX_DEVICES];
    {
        DeviceGuard g;
        for (int i = 0; i < c->ndev; i++) {
            uint64_t r0, r1;
            spec_shard_bounds(n, c->ndev, i, &r0, &r1);
            const uint64_t b0 = r0 ? ends[r0 - 1] : 0, b1 = r1 ? ends[r1 - 1] : 0;
            if (b1 < b0 || b1 > stream_len) return SPEC_E_INVALID_ARGUMENT;
            if (byte_bases) byte_bases[i] = b0;
            ns[i] = r1 - r0;
            lens[i] = b1 - b0;
            const size_t eb = (ns[i] * sizeof(uint64_t) + 255) & ~(size_t)255;
            const size_t need = eb + lens[i] + 16;
            if (hipSetDevice(c->dev[i]) != hipSuccess) return SPEC_E_HIP;
            if (need > c->cap[i]) {
                if (hipStreamSynchronize(c->st[i]) != hipSuccess) return SPEC_E_HIP;
                if (c->buf[i]) (void)hipFree(c->buf[i]);
                c->buf[i] = nullptr;
                c->cap[i] = 0;
                if (hipMalloc(&c->buf[i], need) != hipSuccess) return SPEC_E_HIP;
                c->cap[i] = need;
            }
            uint64_t *de = (uint64_t *)c->buf[i];
            uint8_t *ds = (uint8_t *)c->buf[i] + eb;
            if ((ns[i] && hipMemcpyAsync(de, ends + r0, ns[i] * sizeof(uint64_t), hipMemcpyHostToDevice, c->st[i]) != hipSuccess) ||
                (lens[i] && hipMemcpyAsync(ds, stream_bytes + b0, lens[i], hipMemcpyHostToDevice, c->st[i]) != hipSuccess))
                return SPEC_E_HIP;
            if (ns[i] && b0) {
                const unsigned blocks = (unsigned)std::min<uint64_t>((ns[i] + 255) / 256, 4096);
                hipLaunchKernelGGL(rebase_ends_kernel, dim3(blocks), dim3(256), 0, c->st[i], de, ns[i], b0);
                if (hipGetLastError() != hipSuccess) return SPEC_E_HIP;
            }
            sp[i] = ds;
            ep[i] = de;
        }
    }
    return spec_shard_decode(c, schema, sp, lens, ep, ns, packed);
}

int spec_shard_gather(spec_shard *c, const uint64_t *nbytes, uint8_t *const *packed, int root, uint8_t *gathered) {
    if (!c || !nbytes || !packed || !gathered || root < 0 || root >= c->ndev) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    uint64_t off[SPEC_SHARD_MAX_DEVICES], o = 0;
    for (int i = 0; i < c->ndev; i++) {
        off[i] = o;
        o += nbytes[i];
    }
    // the root's own part: a device copy on its stream
    if (hipSetDevice(c->dev[root]) != hipSuccess) return SPEC_E_HIP;
    if (nbytes[root] && hipMemcpyAsync(gathered + off[root], packed[root], nbytes[root], hipMemcpyDeviceToDevice,
                                       c->st[root]) != hipSuccess)
        return SPEC_E_HIP;
    if (c->ndev == 1) return SPEC_OK;
    // every other part: one grouped send/recv per device pair (RCCL over xGMI, point to point)
    const Rccl &r = rccl();
    if (!r.ok) return SPEC_E_HIP;
    if (r.group_start() != 0) return SPEC_E_HIP;
    int bad = 0;
    for (int i = 0; i < c->ndev; i++) {
        if (i == root || !nbytes[i]) continue;
        bad |= r.send(packed[i], nbytes[i], NCCL_UINT8, root, c->comm[i], c->st[i]);
        bad |= r.recv(gathered + off[i], nbytes[i], NCCL_UINT8, i, c->comm[root], c->st[root]);
    }
    if (r.group_end() != 0 || bad) return SPEC_E_HIP;
    return SPEC_OK;
}

int spec_shard_sync(spec_shard *c) {
    if (!c) return SPEC_E_INVALID_ARGUMENT;
    DeviceGuard g;
    for (int i = 0; i < c->ndev; i++)
        if (hipSetDevice(c->dev[i]) != hipSuccess || hipStreamSynchronize(c->st[i]) != hipSuccess) return SPEC_E_HIP;
    return SPEC_OK;
}

} // extern "C"
