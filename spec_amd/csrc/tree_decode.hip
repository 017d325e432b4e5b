// tree_decode.hip — the generated readers of a schema tree over a batch (include/spec_amd.h
// spec_tree_decoder_*, spec_decode_values): internal/lang/generator/message.go:97-186 (getters),
// struct.go:75-113 (struct Decode), list_msg.go / list_value.go (lists), value.go (any).
//
// One pass over the batch, no host round trip (device-resident row counts):
//   for every GROUP in pre-order — the records, or one list table — with the sub-message tables
//   hanging off it 1:1 (a sub-message's bytes lie inside its owner row's bytes):
//     decode   a lane per row: the group's tables top-down within the row (getters, structs,
//              any, PRESENT / TYPE / ERRMASK / STATUS), and for every list owned in the group
//              its element count and table position (List.Len, internal/types/list.go:22-67);
//     scan     the group's list counts -> CSR begin (BEGIN columns), row counts of the lists;
//              every element's byte range (List.GetBytes: end > dataSize => nil, start > end =>
//              Go panics) while the offsets are in registers.
// A wave's 64 rows are staged in LDS before they are parsed: the rows' whole span with LDS-DMA
// when it fits the wave's slab (consecutive records; the elements of neighbouring lists), else
// each row in its own lane window (small rows far apart), else the rows parse from HBM through
// range-checked loads.  Parsing from LDS turns the field walk's chain of dependent reads from
// HBM-latency round trips into LDS round trips.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>

#include "spec_internal.hpp"
#include "tree_decode_core.hpp"
#include "tree_internal.hpp"

namespace spec {
namespace {

// Build-time A/B (make HIPFLAGS+="-DSPEC_AB_TREE_PAIR=0"), never the environment: 0 runs the
// root group's staged kernel one wave per 64 rows instead of two (gen_pair_rows; pkg1: 158 vs
// 100 us).
#ifndef SPEC_AB_TREE_PAIR
#define SPEC_AB_TREE_PAIR 2
#endif
constexpr int tree_pair() { return SPEC_AB_TREE_PAIR == 2 ? 2 : 0; }

// Group root x (the records or a list table) and the sub-message tables below it, a lane per
// row, run-time schema.  LDS per wave: the staging slab, then a range slot per sub-message table
// of the group.
__global__ __launch_bounds__(TB) void tree_group_kernel(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x,
                                                         uint32_t slab, uint32_t wave_bytes, uint32_t rpw) {
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const uint64_t rows = dec_rows(D, B, x);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint2 *gr = (uint2 *)(smem + (threadIdx.x >> 6) * wave_bytes + slab) + (threadIdx.x & 63);
    auto body = [&](const auto &s, uint64_t row, long long lo, long long hi, bool panic) {
        tree_group_row(s, D, B, x, row, lo, hi, panic, gr);
    };
    tree_rows(B, x, rows, slab, wave_bytes, rpw, body, body);
}

// ---- the group's list counts -> CSR begin, row counts, element ranges ----------------------

// one owner row per thread: the apply pass's per-row element loads are the latency to hide
constexpr int SCAN_T = 1024, SCAN_PER = 1, SCAN_TILE = SCAN_T * SCAN_PER;

// Exclusive block scan through LDS (lds_barrier, spec_device.hpp: a caller's loads issued before it
// overlap it).
__device__ __forceinline__ uint64_t block_scan(uint64_t v, uint64_t *sh, uint64_t &block_total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) sh[wave] = incl;
    lds_barrier();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
            const uint64_t t = sh[w];
            sh[w] = acc;
            acc += t;
        }
        sh[16] = acc;
    }
    lds_barrier();
    const uint64_t r = sh[wave] + incl - v;
    block_total = sh[16];
    lds_barrier();
    return r;
}

// The list tables scanned together (every list owned in one group: same owner rows).
struct ListSet {
    uint32_t n;                 // lists
    uint32_t owner;             // the group root (its rows are the lists' owner rows)
    uint32_t top;               // 1: list_top_kernel turned the tile sums into offsets (many tiles)
    uint32_t y[TREE_MAX_T];     // the list tables
    uint64_t *ws[TREE_MAX_T];   // per list: tile sums, then their exclusive offsets
};

// pass 1: per tile of SCAN_TILE owner rows and list j (blockIdx.y), the tile's element total
__global__ __launch_bounds__(SCAN_T) void list_tiles_kernel(const TreeDesc *Dp, const TreeBufs *Bp, ListSet m) {
    __shared__ uint64_t sh[17];
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const uint64_t rows = dec_rows(D, B, m.owner);
    if ((uint64_t)blockIdx.x * SCAN_TILE >= rows && blockIdx.x) return;
    const uint32_t *cnt = B.cnt[m.y[blockIdx.y]];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER;
    uint64_t v = 0;
    for (int k = 0; k < SCAN_PER; k++)
        if (base + k < rows) v += cnt[base + k];
    uint64_t tot;
    block_scan(v, sh, tot);
    if (threadIdx.x == 0) m.ws[blockIdx.y][blockIdx.x] = tot;
}

// Many tiles (owner rows > FOLD_TILES tiles): per list j (blockIdx.x), exclusive offsets of the
// tile totals in place, and the list's row count (rows_out_kernel compares it with the capacity).
constexpr uint64_t FOLD_TILES = 1024;
__global__ __launch_bounds__(SCAN_T) void list_top_kernel(const TreeDesc *Dp, const TreeBufs *Bp, ListSet m) {
    __shared__ uint64_t sh[17];
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const uint64_t rows = dec_rows(D, B, m.owner);
    const uint64_t ntiles = (rows + SCAN_TILE - 1) / SCAN_TILE;
    uint64_t *ws = m.ws[blockIdx.x];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < ntiles; b += SCAN_T) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < ntiles ? ws[i] : 0;
        uint64_t tot;
        const uint64_t e = block_scan(v, sh, tot);
        if (i < ntiles) ws[i] = carry + e;
        carry += tot;
    }
    if (threadIdx.x == 0) B.rowsd[m.y[blockIdx.x]] = carry;
}

// per tile, every owner row's begin (BEGIN column) and its elements' byte ranges.  Up to
// FOLD_TILES tiles the tile's element offset is the sum of the earlier tiles' totals
// (list_tiles_kernel), summed by the block itself (one load per thread) instead of a top-level
// scan launch, and block 0 sums every tile: the list's row count (rowsd, for rows_out and the next
// level's groups); beyond, list_top_kernel ran first (m.top) and left the offsets in place.
__global__ __launch_bounds__(SCAN_T) void list_apply_kernel(const TreeDesc *Dp, const TreeBufs *Bp, ListSet m) {
    __shared__ uint64_t sh[17];
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const uint64_t rows = dec_rows(D, B, m.owner);
    if ((uint64_t)blockIdx.x * SCAN_TILE >= rows && blockIdx.x) return;
    const uint32_t y = m.y[blockIdx.y];
    const uint32_t *cnt = B.cnt[y];
    uint32_t *beg = (uint32_t *)B.cols[D.t[y].begin_col];
    const uint64_t cap = B.caps[y];
    uint2 *rng = B.rng[y];
    const uint4 *lh = B.lh[y];
    const GlobalSrc gs{B.stream, B.stream_len};
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER;
    static_assert(SCAN_PER == 1, "one owner row per thread");
    // the row's count, table position and first 16 table bytes are loaded before the block
    // scan (they do not depend on it): only the element ranges' positions wait for it
    const uint64_t r = base;
    const uint32_t v0 = r < rows ? cnt[r] : 0;
    const uint4 h = r < rows ? lh[r] : make_uint4(0, 0, 0, 0); // with cnt, not after it
    const uint64_t *tiles = m.ws[blockIdx.y];
    const uint64_t ntiles = (rows + SCAN_TILE - 1) / SCAN_TILE;
    const uint64_t lim = m.top ? 0 : (blockIdx.x ? (uint64_t)blockIdx.x : ntiles);
    uint64_t part = 0;
    for (uint64_t i = threadIdx.x; i < lim; i += SCAN_T) part += tiles[i];
    const uint64_t t0 = v0 ? load_le64(gs, (long long)h.x) : 0, t1 = v0 ? load_le64(gs, (long long)h.x + 8) : 0;
    uint64_t sum = 0, tot;
    if (!m.top) (void)block_scan(part, sh, sum); // sum: earlier tiles (block 0: every tile)
    uint64_t p = (m.top ? tiles[blockIdx.x] : (blockIdx.x ? sum : 0)) + block_scan(v0, sh, tot);
    const uint32_t v[1] = {v0};
    for (int k = 0; k < SCAN_PER; k++) {
        if (r >= rows) break;
        if (beg) beg[r] = (uint32_t)p;
        if (v[k]) {
            // List.GetBytes(i) (internal/types/list.go:100-116, format/list.go:152-176): the
            // table's entries 16 bytes at a time (8 small / 4 big), both loads in flight at once
            const bool big = (h.w & 0x80000000u) != 0;
            const uint32_t esz = big ? 4u : 2u, per = 16u / esz;
            uint32_t a = 0;
            for (uint32_t j0 = 0; j0 < v[k] && p + j0 < cap; j0 += per) {
                const long long q = (long long)h.x + (long long)j0 * esz;
                const uint64_t w0 = j0 ? load_le64(gs, q) : t0, w1 = j0 ? load_le64(gs, q + 8) : t1;
#pragma unroll
                for (uint32_t u = 0; u < 8; u++) {
                    const uint32_t j = j0 + u;
                    if (u >= per || j >= v[k] || p + j >= cap) break;
                    const uint64_t w = u * esz < 8 ? w0 >> (8 * (u * esz)) : w1 >> (8 * (u * esz - 8));
                    const uint32_t b = big ? __builtin_bswap32((uint32_t)w) : (uint32_t)__builtin_bswap16((uint16_t)w);
                    uint2 rr;
                    if (b > h.z) rr = make_uint2(0, 0);               // end > dataSize: nil element
                    else if (a > b) rr = make_uint2(RNG_PANIC, 0);     // start > end: Go panics
                    else rr = make_uint2(h.y + a, h.y + b);
                    rng[p + j] = rr;
                    a = b;
                }
            }
        }
        p += v[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (!m.top) B.rowsd[y] = sum; // the list's row count
        if (beg) beg[rows] = (uint32_t)(m.top ? B.rowsd[y] : sum); // the closing entry
    }
}

// Value.<Kind>() / <Kind>Err() over value spans (internal/types/value.go:120-310): Decode<Kind>
// of exactly the span's bytes; err[row] = 1 where the decoder errs.  A span past the stream
// (Go would panic slicing it) decodes as empty and reports 2.
__global__ __launch_bounds__(256) void values_kernel(const uint8_t *stream, uint64_t stream_len, const uint2 *spans,
                                                     uint64_t n, uint32_t kind, void *out, uint8_t *err) {
    const GlobalSrc gs{stream, stream_len};
    for (uint64_t row = grid_first(); row < n; row += grid_stride()) {
        const uint2 sp = spans[row];
        const bool past = (uint64_t)sp.x + sp.y > stream_len;
        const long long lo = past ? 0 : sp.x, e = past ? 0 : (long long)sp.x + sp.y;
        Val v;
        int nn;
        const bool ok = decode_value_n(gs, kind, lo, e, 0, v, nn);
        store_kind(out, row, kind, v);
        if (err) err[row] = past ? 2 : (ok ? 0 : 1);
    }
}

// rows_out[t] = rows of table t, or ~0 where its group or any group above it (the list tables
// it hangs under) overflowed the capacity: a table under a truncated list is incomplete too
__global__ void rows_out_kernel(const TreeDesc *Dp, const TreeBufs *Bp, uint64_t *out) {
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const uint32_t t = threadIdx.x;
    if (t >= D.ntables) return;
    const uint32_t g = D.t[t].groot;
    bool ovf = false;
    for (uint32_t x = g; x != 0; x = D.t[D.t[x].parent].groot) // x: a list group root
        ovf = ovf || B.rowsd[x] > B.caps[x];
    out[t] = g == 0 ? B.n : (ovf ? ~0ull : B.rowsd[g]);
}

} // namespace
} // namespace spec

using namespace spec;

// ---- host side ------------------------------------------------------------------------------

struct spec_tree_decoder {
    Layout L;
    int device = 0;
    DevBuf desc, bufs, misc, ws_scan;
    DevBuf rng[TREE_MAX_T], cnt[TREE_MAX_T], lh[TREE_MAX_T];
    uint64_t caps[TREE_MAX_T] = {0}; // capacities of the list tables' row buffers
    TreeBufs B;          // host copy of the call's device block
    TreeBufs uploaded;   // what the device block holds
    bool have_upload = false;
    TreeBufs *pinned = nullptr;     // staging for the async upload (ring of slots)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    int slot = 0;
    uint64_t rows[TREE_MAX_T] = {0}; // from the last index
    bool indexed = false;
    const hipFunction_t *jit = nullptr; // schema-specialised group kernels (jit.cpp), per group root
    bool jit_looked = false;
    ~spec_tree_decoder() {
        for (hipEvent_t &e : ev)
            if (e) (void)hipEventDestroy(e);
        if (pinned) (void)hipHostFree(pinned);
    }
};

namespace {

// LDS per wave of group x: the staging slab and one range slot per sub-message table
struct GroupShape {
    uint32_t slab, wave_bytes, rpw; // rpw: rows per wave (tree_rows)
};

// A block's 4 waves share a CU's 160 KiB: a wave gets at most 40 KiB.
constexpr uint32_t WAVE_LDS_MAX = 40960;

GroupShape group_shape(const Layout &L, uint32_t x, uint64_t stream_len, uint64_t rows) {
    const TTable &T = L.desc.t[x];
    const uint32_t extra = 512u * (T.gn > 1 ? T.gn - 1 : 0) + 16; // sub-message range slots
    GroupShape g;
    g.slab = 0;
    g.rpw = 64;
    if (rows) {
        // a wave's 64 consecutive rows span about 64 / rows of the stream (the records: 64 mean
        // records; a list table's elements are spread over every record holding the list):
        // staged when that fits a wave's share of the CU's LDS, else the rows parse straight
        // from HBM (small rows far apart: a slab would hold mostly other rows' bytes, and
        // without one the CU holds 8 waves per SIMD to cover the reads' latency)
        const double span = 64.0 * (double)stream_len / (double)rows * 1.15 + 128 + GUARD;
        const uint32_t lim = x == 0 ? WAVE_LDS_MAX : 16384u;
        const double slab = (double)(((uint64_t)span + 1023) & ~1023ull);
        // (32 rows per wave in half the slab, two waves per SIMD: measured slower for pkg1's
        // 473-byte records, 183 vs 177 us: the waves are VALU-bound at half their lanes)
        if (slab + extra <= lim) {
            g.slab = (uint32_t)slab;
        }
    }
    g.wave_bytes = (g.slab + extra + 15) & ~15u;
    return g;
}

// Waves per block of a group kernel: TB / 64, fewer when the waves' LDS (slab + one 512-byte
// range slot per sub-message table of the group: up to 127 of them) would pass a CU's 160 KiB.
unsigned group_waves(uint32_t wave_bytes) {
    return std::max<unsigned>(1, std::min<unsigned>(TB / 64, 163840u / std::max<uint32_t>(wave_bytes, 1)));
}

int grow(DevBuf &b, size_t bytes) { return b.reserve(std::max<size_t>(bytes, 256)); }

// Buffers for the batch (n records) and the current list capacities; fills d->B.
int prepare(spec_tree_decoder *d, uint64_t n) {
    Layout &L = d->L;
    TreeBufs &B = d->B;
    const TreeDesc &D = L.desc;
    for (uint32_t x = 1; x < L.nt; x++) {
        const TTable &T = D.t[x];
        const uint64_t cap = T.groot == 0 ? n : d->caps[T.groot];
        B.caps[x] = cap;
        if (T.rel == REL_MANY) {
            const uint32_t o = T.parent;
            const uint64_t ocap = D.t[o].groot == 0 ? n : d->caps[D.t[o].groot];
            if (grow(d->rng[x], std::max<uint64_t>(cap, 1) * sizeof(uint2)) ||
                grow(d->cnt[x], (ocap + 1) * sizeof(uint32_t)) || grow(d->lh[x], std::max<uint64_t>(ocap, 1) * sizeof(uint4)))
                return SPEC_E_HIP;
            B.rng[x] = (uint2 *)d->rng[x].p;
            B.cnt[x] = (uint32_t *)d->cnt[x].p;
            B.lh[x] = (uint4 *)d->lh[x].p;
        }
    }
    B.caps[0] = n;
    // scan workspace: per list table, the tile sums of its owner rows
    size_t ws = 0;
    for (uint32_t x = 1; x < L.nt; x++) {
        if (D.t[x].rel != REL_MANY) continue;
        const uint32_t o = D.t[D.t[x].parent].groot;
        const uint64_t ocap = o == 0 ? n : d->caps[o];
        ws += ((ocap + SCAN_TILE - 1) / SCAN_TILE + 1) * sizeof(uint64_t) + 256;
    }
    if (grow(d->ws_scan, ws)) return SPEC_E_HIP;
    return SPEC_OK;
}

// Upload d->B if it differs from what the device holds (stream-ordered, from pinned staging).
int upload(spec_tree_decoder *d, hipStream_t st) {
    if (d->have_upload && memcmp(&d->uploaded, &d->B, sizeof(TreeBufs)) == 0) return SPEC_OK;
    const int k = d->slot;
    d->slot = (d->slot + 1) & 3;
    if (d->ev[k] && hipEventSynchronize(d->ev[k]) != hipSuccess) return SPEC_E_HIP; // slot's last copy done
    memcpy(&d->pinned[k], &d->B, sizeof(TreeBufs));
    if (hipMemcpyAsync(d->bufs.p, &d->pinned[k], sizeof(TreeBufs), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(d->ev[k], st) != hipSuccess)
        return SPEC_E_HIP;
    memcpy(&d->uploaded, &d->B, sizeof(TreeBufs));
    d->have_upload = true;
    return SPEC_OK;
}

// The whole decode of a batch, asynchronous on st: every group's kernel, then its lists' scans.
// col_rows (optional, host, per table): rows the caller's columns hold; every group's rows are
// clamped to them (its tables' columns, and the BEGIN columns of the lists it owns: owner rows +
// 1 entries), so nothing is written past a column; a clamped list reports ~0 in rows_out.
int run(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len, const uint64_t *ends,
        const uint2 *spans, uint64_t n, void *const *columns, const uint64_t *col_rows, hipStream_t st) {
    if (stream_len >= (1ull << 32)) return SPEC_E_TOO_LARGE;
    if (n && (!stream_bytes || (!ends && !spans))) return SPEC_E_INVALID_ARGUMENT;
    Layout &L = d->L;
    TreeBufs &B = d->B;
    const TreeDesc &D = L.desc;
    int rc = prepare(d, n);
    if (rc) return rc;
    if (col_rows) {
        for (uint32_t x = 0; x < L.nt; x++) {
            const uint32_t g = D.t[x].groot;
            if (g == 0) {
                if (col_rows[x] < n) return SPEC_E_CAPACITY; // a row per record: no clamp possible
            } else {
                B.caps[g] = std::min(B.caps[g], col_rows[x]);
            }
        }
        for (uint32_t x = 1; x < L.nt; x++) B.caps[x] = B.caps[D.t[x].groot == 0 ? 0 : D.t[x].groot];
        B.caps[0] = n;
    }
    B.stream = stream_bytes;
    B.stream_len = stream_len;
    B.ends = ends;
    B.spans = spans;
    B.n = n;
    B.rowsd = (uint64_t *)d->misc.p;
    bool all_cols = columns != nullptr; // the schema-specialised kernels store every column unconditionally
    for (uint32_t c = 0; c < L.nc; c++) {
        B.cols[c] = columns ? columns[c] : nullptr;
        all_cols = all_cols && B.cols[c];
    }
    if ((rc = upload(d, st))) return rc;
    // a group with no capacity yet is skipped, and with it the scans of the lists it owns: their
    // row counts must read 0, not a previous batch's (and n == 0 skips every scan)
    bool skipped = n == 0;
    for (uint32_t x = 1; x < L.nt; x++) skipped = skipped || (D.t[x].groot == x && d->caps[x] == 0);
    if (skipped && hipMemsetAsync(B.rowsd, 0, TREE_MAX_T * sizeof(uint64_t), st) != hipSuccess) return SPEC_E_HIP;
    if (!d->jit_looked) { // compiled (or read from the code-object cache) on first use
        d->jit = jit_tree_kernels(D);
        d->jit_looked = true;
    }
    const TreeDesc *Dd = (const TreeDesc *)d->desc.p;
    const TreeBufs *Bd = (const TreeBufs *)d->bufs.p;
    uint8_t *wsp = (uint8_t *)d->ws_scan.p;
    // Groups by level: the records' group is level 0, a list's group one level below its owner's
    // group.  The groups of one level are independent (their rows come from the previous level's
    // scans); every list owned in a group gets one batched scan after the group's kernel.
    uint32_t lv[TREE_MAX_T] = {};
    uint32_t maxlv = 0;
    ListSet ms[TREE_MAX_T];
    for (uint32_t x = 0; x < L.nt; x++) {
        if (D.t[x].groot != x) continue; // decoded inside its group
        if (x) lv[x] = lv[D.t[D.t[x].parent].groot] + 1; // the owner's group precedes it
        maxlv = std::max(maxlv, lv[x]);
        const uint64_t cap = x == 0 ? n : d->caps[x];
        ListSet &m = ms[x];
        m.n = 0;
        m.owner = x;
        m.top = (cap + SCAN_TILE - 1) / SCAN_TILE > FOLD_TILES ? 1u : 0u;
        for (uint32_t y = x + 1; y < L.nt; y++) {
            if (D.t[y].rel != REL_MANY || D.t[D.t[y].parent].groot != x) continue;
            m.y[m.n] = y;
            m.ws[m.n] = (uint64_t *)wsp;
            wsp += (((cap + SCAN_TILE - 1) / SCAN_TILE + 1) * sizeof(uint64_t) + 255) & ~(size_t)255;
            m.n++;
        }
    }
    const hipFunction_t set_fn = d->jit && all_cols ? d->jit[4 * TREE_MAX_T + 2] : nullptr;
    for (uint32_t level = 0; n && level <= maxlv; level++) {
        // the level's groups parsed from HBM by generated kernels: one level-fused launch when
        // there are two or more (pkg1's five list groups: 89.5 -> 70.5 us)
        bool in_set[TREE_MAX_T] = {};
        TableSet fused;
        fused.n = 0;
        uint32_t fused_wb = 16;
        unsigned fused_grid = 1;
        for (uint32_t x = 1; set_fn && x < L.nt; x++) {
            if (D.t[x].groot != x || lv[x] != level || d->caps[x] == 0 || !d->jit[x]) continue;
            const GroupShape gs = group_shape(L, x, stream_len, d->caps[x]);
            if (gs.slab) continue;
            fused.t[fused.n++] = x;
            fused_wb = std::max(fused_wb, gs.wave_bytes);
            fused_grid = std::max(fused_grid, row_grid(d->caps[x]));
        }
        if (fused.n >= 2) { // (one group: its own kernel below)
            for (uint32_t j = 0; j < fused.n; j++) in_set[fused.t[j]] = true;
            void *args[] = {(void *)&Dd, (void *)&Bd, &fused, &fused_wb};
            const unsigned fw = group_waves(fused_wb);
            const hipError_t le = hipModuleLaunchKernel(set_fn, fused_grid, fused.n, 1, 64 * fw, 1, 1,
                                                        (unsigned)(fw * fused_wb), st, args, nullptr);
            if (le != hipSuccess) {
                note_hip_error(le);
                return SPEC_E_HIP;
            }
        }
        for (uint32_t x = 0; x < L.nt; x++) {
            if (D.t[x].groot != x || lv[x] != level || in_set[x]) continue;
            const uint64_t cap = x == 0 ? n : d->caps[x];
            if (cap == 0) continue;
            const GroupShape gs = group_shape(L, x, stream_len, cap);
            const unsigned wpb = group_waves(gs.wave_bytes);
            const uint64_t per_block = (uint64_t)wpb * gs.rpw;
            const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((cap + per_block - 1) / per_block, 1u << 20));
            const size_t lds = (size_t)wpb * gs.wave_bytes;
            const hipFunction_t pair_fn =
                tree_pair() && d->jit && all_cols && gs.slab ? d->jit[2 * TREE_MAX_T + x] : nullptr;
            if (pair_fn) {
                // the root group on P waves per 64 rows: one slab, the waves decoding it
                // (tree_rows_pair), one set of range slots, a 1 KiB exchange per extra wave (pkg1:
                // 35 KiB slab + 2 KiB slots + 1-3 KiB = four blocks per CU)
                const uint32_t gn = D.t[x].gn, P = (uint32_t)tree_pair();
                uint32_t xx = x, slab = gs.slab, slots = 512u * (gn > 1 ? gn - 1 : 0), rpw = 64;
                void *args[] = {(void *)&Dd, (void *)&Bd, &xx, &slab, &slots, &rpw};
                const unsigned grid = (unsigned)std::min<uint64_t>((cap + 63) / 64, 1u << 20);
                const hipError_t le = hipModuleLaunchKernel(pair_fn, grid, 1, 1, 64 * P, 1, 1, slab + slots + (P - 1) * 1024,
                                                            st, args, nullptr);
                if (le != hipSuccess) {
                    note_hip_error(le);
                    return SPEC_E_HIP;
                }
            } else if (d->jit && d->jit[x] && all_cols) {
                uint32_t xx = x, slab = gs.slab, wb = gs.wave_bytes, rpw = gs.rpw;
                void *args[] = {(void *)&Dd, (void *)&Bd, &xx, &slab, &wb, &rpw};
                // rows from HBM: the kernel without staging code (fewer registers, more waves)
                const hipFunction_t fn = gs.slab == 0 && d->jit[TREE_MAX_T + x] ? d->jit[TREE_MAX_T + x] : d->jit[x];
                const unsigned grid = gs.slab == 0 ? row_grid(cap) : (unsigned)blocks;
                const hipError_t le =
                    hipModuleLaunchKernel(fn, grid, 1, 1, 64 * wpb, 1, 1, (unsigned)lds, st, args, nullptr);
                if (le != hipSuccess) {
                    note_hip_error(le);
                    return SPEC_E_HIP;
                }
            } else {
                hipLaunchKernelGGL(tree_group_kernel, dim3((unsigned)blocks), dim3(64 * wpb), lds, st, Dd, Bd, x, gs.slab,
                                   gs.wave_bytes, gs.rpw);
            }
        }
        // every list owned in the level's groups: one batched scan per owner group
        for (uint32_t x = 0; x < L.nt; x++) {
            if (D.t[x].groot != x || lv[x] != level || !ms[x].n) continue;
            const uint64_t cap = x == 0 ? n : d->caps[x];
            if (cap == 0) continue;
            const ListSet &m = ms[x];
            const uint64_t tiles = std::max<uint64_t>(1, (cap + SCAN_TILE - 1) / SCAN_TILE);
            hipLaunchKernelGGL(list_tiles_kernel, dim3((unsigned)tiles, m.n), dim3(SCAN_T), 0, st, Dd, Bd, m);
            if (m.top) hipLaunchKernelGGL(list_top_kernel, dim3(m.n), dim3(SCAN_T), 0, st, Dd, Bd, m);
            hipLaunchKernelGGL(list_apply_kernel, dim3((unsigned)tiles, m.n), dim3(SCAN_T), 0, st, Dd, Bd, m);
        }
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        note_hip_error(e);
        return SPEC_E_HIP;
    }
    return SPEC_OK;
}

// index: a decode without columns, then the row counts on the host; list capacities grow and
// the pass reruns when a list outgrew them (at most once per growth).
int index(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len, const uint64_t *ends,
          const uint2 *spans, uint64_t n, uint64_t *rows, hipStream_t st) {
    Layout &L = d->L;
    // an inner list's count is exact only once its owner list fits: at most one growth per level
    // of list nesting (bounded by the table count)
    for (uint32_t attempt = 0; attempt <= L.nt; attempt++) {
        int rc = run(d, stream_bytes, stream_len, ends, spans, n, nullptr, nullptr, st);
        if (rc) return rc;
        uint64_t got[TREE_MAX_T];
        if (hipMemcpyAsync(got, d->B.rowsd, sizeof(uint64_t) * TREE_MAX_T, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return SPEC_E_HIP;
        bool again = false;
        for (uint32_t x = 1; x < L.nt; x++) {
            const TTable &T = L.desc.t[x];
            if (T.rel != REL_MANY) continue;
            if (n && got[x] > d->caps[x]) {
                if (got[x] > 0xffffffffull) return SPEC_E_TOO_LARGE;
                d->caps[x] = got[x] + got[x] / 8 + 64;
                again = true;
            }
        }
        if (again) continue;
        for (uint32_t x = 0; x < L.nt; x++) {
            const uint32_t g = L.desc.t[x].groot;
            d->rows[x] = n == 0 ? 0 : (g == 0 ? n : got[g]);
        }
        if (rows) memcpy(rows, d->rows, sizeof(uint64_t) * L.nt);
        d->indexed = true;
        return SPEC_OK;
    }
    return SPEC_E_TOO_LARGE; // the capacities did not settle (cannot happen for a finite tree)
}

} // namespace

extern "C" {

int spec_tree_decoder_create(const spec_tree *tree, spec_tree_decoder **out) {
    if (!out) return SPEC_E_INVALID_ARGUMENT;
    *out = nullptr;
    spec_tree_decoder *d = new (std::nothrow) spec_tree_decoder();
    if (!d) return SPEC_E_INVALID_ARGUMENT;
    if (!build_layout(tree, d->L)) {
        delete d;
        return SPEC_E_INVALID_ARGUMENT;
    }
    memset(&d->B, 0, sizeof(d->B));
    memset(&d->uploaded, 0, sizeof(d->uploaded));
    bool ok = hipGetDevice(&d->device) == hipSuccess && !d->desc.reserve(sizeof(TreeDesc)) &&
              !d->bufs.reserve(sizeof(TreeBufs)) && !d->misc.reserve(TREE_MAX_T * sizeof(uint64_t) + 256) &&
              hipHostMalloc((void **)&d->pinned, 4 * sizeof(TreeBufs), hipHostMallocDefault) == hipSuccess &&
              hipMemcpy(d->desc.p, &d->L.desc, sizeof(TreeDesc), hipMemcpyHostToDevice) == hipSuccess &&
              hipMemset(d->misc.p, 0, TREE_MAX_T * sizeof(uint64_t) + 256) == hipSuccess;
    for (hipEvent_t &e : d->ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        note_hip_error(hipGetLastError());
        delete d;
        return SPEC_E_HIP;
    }
    *out = d;
    return SPEC_OK;
}

void spec_tree_decoder_destroy(spec_tree_decoder *d) { delete d; }

int spec_tree_decoder_index(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len,
                            const uint64_t *ends, uint64_t n, uint64_t *rows, void *stream) {
    if (!d) return SPEC_E_INVALID_ARGUMENT;
    return index(d, stream_bytes, stream_len, ends, nullptr, n, rows, (hipStream_t)stream);
}

int spec_tree_decoder_index_spans(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len,
                                  const spec_span *spans, uint64_t n, uint64_t *rows, void *stream) {
    if (!d || (n && !spans)) return SPEC_E_INVALID_ARGUMENT;
    return index(d, stream_bytes, stream_len, nullptr, (const uint2 *)spans, n, rows, (hipStream_t)stream);
}

int spec_tree_decoder_decode(spec_tree_decoder *d, void *const *columns, void *stream) {
    if (!d || !d->indexed || !columns) return SPEC_E_INVALID_ARGUMENT;
    const TreeBufs &B = d->B;
    return run(d, B.stream, B.stream_len, B.ends, B.spans, B.n, columns, nullptr, (hipStream_t)stream);
}

int spec_tree_decoder_run(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len, const uint64_t *ends,
                          uint64_t n, void *const *columns, const uint64_t *col_rows, uint64_t *rows_out,
                          void *stream) {
    if (!d || !columns) return SPEC_E_INVALID_ARGUMENT;
    const int rc = run(d, stream_bytes, stream_len, ends, nullptr, n, columns, col_rows, (hipStream_t)stream);
    if (rc || !rows_out) return rc;
    hipLaunchKernelGGL(rows_out_kernel, dim3(1), dim3(TREE_MAX_T), 0, (hipStream_t)stream,
                       (const TreeDesc *)d->desc.p, (const TreeBufs *)d->bufs.p, rows_out);
    return hipGetLastError() == hipSuccess ? SPEC_OK : SPEC_E_HIP;
}

int spec_tree_decoder_capacity(const spec_tree_decoder *d, uint64_t *rows) {
    if (!d || !rows) return SPEC_E_INVALID_ARGUMENT;
    for (uint32_t x = 0; x < d->L.nt; x++) {
        const uint32_t g = d->L.desc.t[x].groot;
        rows[x] = g == 0 ? 0 : d->caps[g];
    }
    return SPEC_OK;
}

int spec_tree_decoder_reserve(spec_tree_decoder *d, const uint64_t *rows) {
    if (!d || !rows) return SPEC_E_INVALID_ARGUMENT;
    for (uint32_t x = 1; x < d->L.nt; x++)
        if (d->L.desc.t[x].rel == REL_MANY) d->caps[x] = std::max(d->caps[x], rows[x]);
    return SPEC_OK;
}

long long spec_tree_jit_compile(const spec_tree *tree) {
    Layout *L = new (std::nothrow) Layout();
    if (!L) return SPEC_E_INVALID_ARGUMENT;
    long long r = SPEC_E_INVALID_ARGUMENT;
    if (build_layout(tree, *L)) r = jit_compile_only_tree(L->desc);
    delete L;
    return r;
}

int spec_decode_values(int kind, const uint8_t *stream_bytes, uint64_t stream_len, const spec_span *spans, uint64_t n,
                       void *out, uint8_t *err, void *stream) {
    if (!is_scalar(kind)) return SPEC_E_INVALID_ARGUMENT;
    if (n == 0) return SPEC_OK;
    if (!spans || !out || (!stream_bytes && stream_len)) return SPEC_E_INVALID_ARGUMENT;
    if (stream_len >= (1ull << 32)) return SPEC_E_TOO_LARGE;
    hipLaunchKernelGGL(values_kernel, dim3(row_grid(n)), dim3(TB), 0, (hipStream_t)stream, stream_bytes, stream_len,
                       (const uint2 *)spans, n, (uint32_t)kind, out, err);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        note_hip_error(e);
        return SPEC_E_HIP;
    }
    return SPEC_OK;
}

} // extern "C"
