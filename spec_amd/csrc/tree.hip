// tree.hip — schema trees on the GPU (include/spec_amd.h spec_tree_*): the generated readers
// and writers of internal/lang/generator (message.go:97-439, struct.go:75-142) over a batch,
// for every kind — structs, sub-messages, value lists, lists of structs/messages, any.
// Device code: tree_core.hpp.  Host side: the layout, the descriptor, the launch sequences.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "spec_internal.hpp"
#include "tree_core.hpp"

namespace spec {
namespace {

constexpr int TB = 256; // threads per block of the row kernels

unsigned row_grid(uint64_t rows) {
    const uint64_t b = (rows + TB - 1) / TB;
    const uint64_t cap = (uint64_t)device_cus() * 16;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, cap));
}

// ---- decode kernels ------------------------------------------------------------------------
//
// A wave takes 64 consecutive rows of a table; the rows' bytes usually lie close together in
// the stream (consecutive records, their sub-messages, the elements of neighbouring lists), so
// the span [min lo, max hi) of the wave's rows is staged in an LDS slab with 16-byte loads and
// parsed from there (SlabSrc); reads outside the staged bytes, and waves whose span does not fit,
// go to HBM (GlobalSrc) — the same bytes either way.

constexpr int TSLAB = 16384 + 128; // per wave

// LDS per wave for the rows of a table: a slab when 64 consecutive rows are expected to fit it
// (mean span of 64 rows, estimated as if the table's rows covered the whole stream, + 10 %),
// else none: staging would almost never happen and the slab only halves the waves a CU holds
// (the row kernels are latency-bound gathers: pkg1's ~470-byte records never fit).
uint32_t tree_slab(uint64_t stream_len, uint64_t rows) {
    if (!rows) return 0;
    const double span = 64.0 * (double)stream_len / (double)rows;
    return span * 1.1 + 256 <= TSLAB ? (uint32_t)TSLAB : 0u;
}

struct SlabSrc {
    using pos_t = long long;
    lds_u8 *lds;    // stream bytes [base, end)
    long long base, end;
    GlobalSrc g;
    __device__ __forceinline__ bool in(long long p, int n) const { return p >= base && p + n <= end; }
    __device__ __forceinline__ uint32_t u8(long long p) const { return in(p, 1) ? lds[p - base] : g.u8(p); }
    __device__ __forceinline__ uint64_t d64(long long p) const {
        return in(p, 8) ? *(lds_u64 *)(lds + (p - base)) : g.d64(p);
    }
    __device__ __forceinline__ uint32_t d32(long long p) const {
        return in(p, 4) ? *(lds_u32 *)(lds + (p - base)) : g.d32(p);
    }
};

__device__ __forceinline__ void tree_wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Every wave of the grid over the rows of table x, 64 at a time: body(src, row, lo, hi, panic)
// for its valid rows, src = the staged slab when the wave's span fits, else HBM.
template <class Body>
__device__ __forceinline__ void tree_rows(const TreeBufs &B, uint32_t x, uint64_t rows, uint32_t slab_bytes,
                                          Body body) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint8_t *slab = smem + wave * slab_bytes;
    const GlobalSrc gs{stream_rsrc(B), B.stream_len};
    const uint64_t wstride = (uint64_t)gridDim.x * (TB / 64) * 64;
    for (uint64_t base = ((uint64_t)blockIdx.x * (TB / 64) + wave) * 64; base < rows; base += wstride) {
        const uint64_t row = base + lane;
        const bool valid = row < rows;
        long long lo = 0, hi = 0;
        bool panic = false;
        if (valid) row_range(B, x, row, lo, hi, panic);
        const bool some = valid && hi > lo;
        long long slo = some ? lo : (long long)B.stream_len, shi = some ? hi : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const long long a = __shfl_xor(slo, d), b2 = __shfl_xor(shi, d);
            slo = a < slo ? a : slo;
            shi = b2 > shi ? b2 : shi;
        }
        slo = (long long)uniform64((uint64_t)slo);
        shi = (long long)uniform64((uint64_t)shi);
        const long long sb = (slo > 64 ? slo - 64 : 0) & ~15ll, se = (shi + 16 + 15) & ~15ll;
        if (slab_bytes && slo < shi && se - sb <= (long long)slab_bytes) {
            for (long long off = 16ll * lane; off < se - sb; off += 1024) {
                const long long p = sb + off;
                uint4 v;
                if ((uint64_t)p + 16 <= B.stream_len) {
                    const auto q = __builtin_amdgcn_raw_buffer_load_b128(gs.rsrc, (uint32_t)p, 0, 0);
                    v = make_uint4(q[0], q[1], q[2], q[3]);
                } else {
                    v = make_uint4(gs.d32(p), gs.d32(p + 4), gs.d32(p + 8), gs.d32(p + 12));
                }
                *(uint4 *)(slab + off) = v;
            }
            tree_wave_fence();
            const SlabSrc ss{(lds_u8 *)slab, sb, se, gs};
            if (valid) body(ss, row, lo, hi, panic);
        } else if (valid) {
            body(gs, row, lo, hi, panic);
        }
        tree_wave_fence(); // the slab is read before the next rows overwrite it
    }
}

// Per row of message table x: the range of every sub-message field (its child row) and the
// element count of every list field (m.field(tag), internal/types/msg.go:466-475; OpenList,
// internal/types/list.go:22-25: errors => an empty list).
__global__ __launch_bounds__(TB) void tree_index_kernel(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x,
                                                         uint64_t rows, uint32_t slab) {
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const TTable &T = D.t[x];
    tree_rows(B, x, rows, slab, [&](const auto &s, uint64_t row, long long lo, long long hi, bool) {
        const RecInfo ri = rec_open(s, lo, hi);
        const long long ds = ri.tr.dstart;
        for (uint32_t k = 0; k < T.nd; k++) {
            const TField &F = D.f[D.direct[T.d0 + k]];
            if (F.kind != K_MESSAGE && F.kind != K_LIST) continue;
            const long long end = rec_field_end(s, ri, F.tag, F.rank);
            if (F.kind == K_MESSAGE) {
                B.rng[F.table][row] = end >= 0 ? make_uint2((uint32_t)ds, (uint32_t)(ds + end)) : make_uint2(0, 0);
            } else {
                const ListInfo li = list_at(s, (long long)ds, end >= 0 ? ds + end : ds);
                B.cnt[F.table][row] = li.count;
            }
        }
    });
}

// Per owner row of table x: the range of every element of each of x's list tables y (one pass
// over the owner rows for all of them: List.GetBytes, internal/types/list.go:100-116: end >
// dataSize => nil; start > end => Go panics).
__global__ __launch_bounds__(TB) void tree_expand_kernel(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x,
                                                          uint64_t rows, uint32_t slab) {
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    tree_rows(B, x, rows, slab, [&](const auto &s, uint64_t row, long long lo, long long hi, bool) {
        const RecInfo ri = rec_open(s, lo, hi);
        const long long ds = ri.tr.dstart;
        for (uint32_t y = x + 1; y < D.ntables; y++) {
            const TTable &Ty = D.t[y];
            if (Ty.parent != (int)x || Ty.rel != REL_MANY) continue;
            const TField &F = D.f[Ty.field];
            const long long end = rec_field_end(s, ri, F.tag, F.rank);
            const ListInfo li = list_at(s, (long long)ds, end >= 0 ? ds + end : ds);
            uint2 *out = B.rng[y] + B.cnt[y][row];
            for (uint32_t j = 0; j < li.count; j++) {
                uint32_t a, b;
                if (li.big) {
                    b = be32_at(s, li.tstart + 4ll * j);
                    a = j ? be32_at(s, li.tstart + 4ll * (j - 1)) : 0;
                } else {
                    b = be16_at(s, li.tstart + 2ll * j);
                    a = j ? be16_at(s, li.tstart + 2ll * (j - 1)) : 0;
                }
                uint2 r;
                if (b > li.dsize) r = make_uint2(0, 0);           // nil element
                else if (a > b) r = make_uint2(RNG_PANIC, 0);      // Go panics on the slice
                else r = make_uint2((uint32_t)(li.dstart + a), (uint32_t)(li.dstart + b));
                out[j] = r;
            }
        }
    });
}

// Every column of table x.
__global__ __launch_bounds__(TB) void tree_decode_kernel(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x,
                                                          uint64_t rows, uint32_t slab) {
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const TTable &T = D.t[x];
    tree_rows(B, x, rows, slab, [&](const auto &s, uint64_t row, long long lo, long long hi, bool panic) {
        uint32_t st = ST_OK;
        if (T.shape == SHAPE_VALUE) {
            const TField &F = D.f[T.field];
            Val v;
            int n;
            const bool ok = decode_value_n(s, F.elem, lo, hi, 0, v, n);
            store_kind(B.cols[F.col], row, F.elem, v);
            st = panic ? ST_PANIC : (ok ? ST_OK : ST_INVALID_VALUE);
        } else if (T.shape == SHAPE_STRUCT) {
            st = tree_struct(s, D, B, T.field, lo, hi, row, 0);
            st = panic ? ST_PANIC : st;
        } else {
            const RecInfo ri = rec_open(s, lo, hi); // empty (or panicked) range => empty message
            st = ri.tr.st;
            const long long ds = ri.tr.dstart;
            uint64_t *errp = (uint64_t *)B.cols[T.err_col];
            uint64_t errs = 0;
            for (uint32_t k = 0; k < T.nd; k++) {
                const uint32_t fi = D.direct[T.d0 + k];
                const TField &F = D.f[fi];
                const long long end = rec_field_end(s, ri, F.tag, F.rank);
                const long long e = end >= 0 ? ds + end : ds;
                bool bad = false; // the field's *Err getter errs
                switch (F.kind) {
                case K_MESSAGE:
                case K_LIST:
                    store_u8(B.cols[F.present], row, end >= 0 ? 1u : 0u);
                    // MessageErr / ListErr: OpenMessageErr / OpenListErr of m.field(tag)
                    if (errp && e > ds)
                        bad = (F.kind == K_MESSAGE ? parse_trailer<false>(s, ds, e).st : parse_trailer<true>(s, ds, e).st) != ST_OK;
                    break;
                case K_STRUCT: {
                    const uint32_t sst = tree_struct(s, D, B, fi, ds, e, row, 0);
                    if (sst == ST_PANIC) st = ST_PANIC;
                    bad = sst != ST_OK;
                    break;
                }
                case K_ANY: {
                    // Field(tag) = OpenValue(bytes[:end]): nil on error or len < n; n < 0 panics
                    long long n = 0;
                    uint2 sp = make_uint2(0, 0);
                    if (e > ds) {
                        if (type_size(s, ds, e, n)) {
                            if (n < 0) st = ST_PANIC;
                            else if (n > 0 && n <= e - ds) sp = make_uint2((uint32_t)(e - n), (uint32_t)n);
                        } else {
                            bad = true; // OpenValueErr: DecodeTypeSize's error
                        }
                    }
                    if (B.cols[F.col]) ((uint2 *)B.cols[F.col])[row] = sp;
                    // Value.Type(): the value's last byte (DecodeType), 0 for a nil value
                    store_u8(B.cols[F.present], row, sp.y ? s.u8((long long)sp.x + sp.y - 1) : 0u);
                    break;
                }
                default:
                    if (B.cols[F.col]) bad = !decode_store(s, F.kind, (long long)ds, end, 0, B.cols[F.col], row);
                    else if (errp) {
                        Val v;
                        int n;
                        bad = !decode_value_n(s, F.kind, (long long)ds, e, 0, v, n);
                    }
                }
                if (bad && k < 64) errs |= 1ull << k;
            }
            if (errp) errp[row] = errs;
            if (panic) st = ST_PANIC;
        }
        store_u8(B.cols[T.status_col], row, st);
    });
}

// Value.<Kind>() / <Kind>Err() over value spans (internal/types/value.go:120-310): Decode<Kind>
// of exactly the span's bytes; err[row] = 1 where the decoder errs.  A span past the stream
// (Go would panic slicing it) decodes as empty and reports 2.
__global__ __launch_bounds__(256) void values_kernel(const uint8_t *stream, uint64_t stream_len, const uint2 *spans,
                                                     uint64_t n, uint32_t kind, void *out, uint8_t *err) {
    const GlobalSrc gs{__builtin_amdgcn_make_buffer_rsrc((void *)stream, (short)0, (int)(uint32_t)stream_len, 0x00020000),
                       stream_len};
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

// ---- encode kernels ------------------------------------------------------------------------

// Encoded size of every row of table x (its children already sized).
__global__ __launch_bounds__(TB) void tree_size_kernel(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x,
                                                        uint64_t rows) {
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const TTable &T = D.t[x];
    bool err = false;
    for (uint64_t row = grid_first(); row < rows; row += grid_stride()) {
        uint64_t total;
        if (T.shape == SHAPE_VALUE) {
            const TField &F = D.f[T.field];
            total = value_size(B, D, F.col, F.elem, row, err);
        } else if (T.shape == SHAPE_STRUCT) {
            total = struct_size(B, D, T.field, row, err);
        } else {
            uint64_t data = 0;
            uint32_t nf = 0, maxtag = 0;
            for (uint32_t k = 0; k < T.nd; k++) {
                const TField &F = D.f[D.direct[T.d0 + k]];
                uint64_t sz;
                if (F.kind == K_MESSAGE || F.kind == K_LIST) {
                    if (!cell(B, D, F.present, row)[0]) continue;
                    sz = F.kind == K_MESSAGE ? B.size[F.table][row] : list_size(B, D, F.table, row, err).total;
                } else if (F.kind == K_STRUCT) {
                    sz = struct_size(B, D, D.direct[T.d0 + k], row, err);
                } else {
                    sz = value_size(B, D, F.col, F.kind, row, err);
                    if (F.kind == K_ANY && sz == 0) continue;
                }
                data += sz;
                nf++;
                maxtag = F.tag > maxtag ? F.tag : maxtag;
            }
            // IsBigMessage (internal/format/msg.go:43-61): a tag > 255 or an end offset > 65535
            const bool big = maxtag > 255 || (nf > 0 && data > 65535);
            const uint64_t tsize = (uint64_t)nf * (big ? 6 : 3);
            if (data > MAX_SIZE) err = true;
            total = data + tsize + vlen64(data) + vlen64(tsize) + 1;
        }
        if (total > 0xffffffffull) err = true;
        B.size[x][row] = (uint32_t)total;
    }
    if (err) *B.err = 1;
}

// Bytes of every row of table x at its start; the starts of its child rows.
__global__ __launch_bounds__(TB) void tree_write_kernel(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x,
                                                         uint64_t rows) {
    const TreeDesc &D = *Dp;
    const TreeBufs &B = *Bp;
    const TTable &T = D.t[x];
    if (!B.out || *B.err || *B.total > B.out_cap) return;
    extern __shared__ uint32_t tw_ends[]; // MESSAGE tables: [wave][field][lane]
    uint32_t *ends = tw_ends + (threadIdx.x >> 6) * (uint32_t)T.nd * 64 + (threadIdx.x & 63);
    for (uint64_t row = grid_first(); row < rows; row += grid_stride()) {
        const uint64_t start = x == 0 ? B.offsets[row] : B.pos[x][row];
        if (start == ~0ull) continue; // a row no written owner placed (absent message / list)
        if (x == 0 && B.ends_out) B.ends_out[row] = start + B.size[0][row];
        BEmit em{B.out, start, start};
        if (T.shape == SHAPE_VALUE) {
            const TField &F = D.f[T.field];
            emit_value(em, B, D, F.col, F.elem, row);
            em.finish();
            continue;
        }
        if (T.shape == SHAPE_STRUCT) {
            emit_struct(em, B, D, T.field, row);
            em.finish();
            continue;
        }
        // a message (internal/writer/writer.go:376-553): fields in write order, each field's
        // end offset (relative to the message start) kept for the table, in LDS
        // ([field][lane] per wave: a per-lane array indexed at run time would live in scratch)
        uint32_t maxtag = 0, nf = 0;
        for (uint32_t k = 0; k < T.nd; k++) {
            const uint32_t fi = D.direct[T.d0 + k];
            const TField &F = D.f[fi];
            ends[k * 64] = 0xffffffffu; // absent
            if (F.kind == K_MESSAGE || F.kind == K_LIST) {
                if (!cell(B, D, F.present, row)[0]) continue;
                if (F.kind == K_MESSAGE) {
                    B.pos[F.table][row] = em.pos; // the sub-message, written by table F.table
                    em.skip(B.size[F.table][row]);
                } else {
                    // elements (written by table F.table), then EncodeListTable's table and trailer
                    bool e2 = false;
                    uint32_t j0, j1;
                    list_span(B, D, F.table, row, j0, j1, e2);
                    const TreeListSize L = list_size(B, D, F.table, row, e2);
                    const uint64_t lstart = em.pos;
                    for (uint32_t j = j0; j < j1; j++) {
                        B.pos[F.table][j] = em.pos;
                        em.skip(B.size[F.table][j]);
                    }
                    uint64_t off = 0;
                    for (uint32_t j = j0; j < j1; j++) {
                        off += B.size[F.table][j];
                        em.be(off, L.big ? 4 : 2);
                    }
                    (void)lstart;
                    em.rvarint(L.data);
                    em.rvarint((uint64_t)L.count * (L.big ? 4 : 2));
                    em.put1(L.big ? T_BIG_LIST : T_LIST);
                }
            } else if (F.kind == K_STRUCT) {
                emit_struct(em, B, D, fi, row);
            } else {
                if (F.kind == K_ANY && ((const uint2 *)cell(B, D, F.col, row))->y == 0) continue;
                emit_value(em, B, D, F.col, F.kind, row);
            }
            ends[k * 64] = (uint32_t)(em.pos - start);
            nf++;
            maxtag = F.tag > maxtag ? F.tag : maxtag;
        }
        const uint64_t data = em.pos - start;
        const bool big = maxtag > 255 || (nf > 0 && data > 65535);
        // the table in the writer's order (insertion sort, equal tags: later first,
        // internal/writer/stack_msg.go:37-61), present fields only (encode/msg.go:58-72)
        for (uint32_t k = 0; k < T.nd; k++) {
            const uint32_t fi = D.sorted[T.d0 + k];
            const uint32_t e = ends[D.sslot[T.d0 + k] * 64];
            if (e == 0xffffffffu) continue;
            em.be(D.f[fi].tag, big ? 2 : 1);
            em.be(e, big ? 4 : 2);
        }
        em.rvarint(data);
        em.rvarint((uint64_t)nf * (big ? 6 : 3));
        em.put1(big ? T_BIG_MESSAGE : T_MESSAGE);
        em.finish();
    }
}

// ---- exclusive scans ---------------------------------------------------------------------

constexpr int SCAN_T = 1024, SCAN_PER = 4, SCAN_TILE = SCAN_T * SCAN_PER;

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *sh, uint64_t &block_total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) sh[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
            const uint64_t t = sh[w];
            sh[w] = acc;
            acc += t;
        }
        sh[16] = acc;
    }
    __syncthreads();
    const uint64_t r = sh[wave] + incl - v;
    block_total = sh[16];
    __syncthreads();
    return r;
}

// pass 1: tile sums of a u32 array
__global__ __launch_bounds__(SCAN_T) void scan_tiles_kernel(const uint32_t *in, uint64_t n, uint64_t *tile_sums) {
    __shared__ uint64_t sh[17];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER;
    uint64_t v = 0;
    for (int k = 0; k < SCAN_PER; k++)
        if (base + k < n) v += in[base + k];
    uint64_t tot;
    block_excl_scan(v, sh, tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

// pass 2: exclusive scan of the tile sums (one workgroup), total
__global__ __launch_bounds__(SCAN_T) void scan_top_kernel(uint64_t *tile_sums, uint64_t ntiles, uint64_t *total) {
    __shared__ uint64_t sh[17];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < ntiles; b += SCAN_T) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < ntiles ? tile_sums[i] : 0;
        uint64_t tot;
        const uint64_t e = block_excl_scan(v, sh, tot);
        if (i < ntiles) tile_sums[i] = carry + e;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

// pass 3: per tile, the exclusive prefix of every element: into out32 (u32, + out32[n] = total)
// or out64 (u64); ends64 (optional) = prefix + element
__global__ __launch_bounds__(SCAN_T) void scan_apply_kernel(const uint32_t *in, uint64_t n, const uint64_t *tile_sums,
                                                            const uint64_t *total, uint32_t *out32, uint64_t *out64,
                                                            uint64_t *ends64) {
    __shared__ uint64_t sh[17];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER;
    uint32_t v[SCAN_PER];
    uint64_t sum = 0;
    for (int k = 0; k < SCAN_PER; k++) {
        v[k] = base + k < n ? in[base + k] : 0;
        sum += v[k];
    }
    uint64_t tot;
    uint64_t p = tile_sums[blockIdx.x] + block_excl_scan(sum, sh, tot);
    for (int k = 0; k < SCAN_PER; k++) {
        if (base + k < n) {
            if (out32) out32[base + k] = (uint32_t)p;
            if (out64) out64[base + k] = p;
            if (ends64) ends64[base + k] = p + v[k];
        }
        p += v[k];
    }
    if (out32 && blockIdx.x == 0 && threadIdx.x == 0) out32[n] = (uint32_t)*total;
}

// The same three passes over several u32 arrays of n elements at once (the list tables of one
// owner table): array j = blockIdx.y (tiles, apply) / blockIdx.x (top); out32 in place allowed.
struct ScanMulti {
    const uint32_t *in[TREE_MAX_T];
    uint32_t *out32[TREE_MAX_T];
    uint64_t *ws[TREE_MAX_T];
    uint64_t *total[TREE_MAX_T];
};

__global__ __launch_bounds__(SCAN_T) void scan_tiles_multi_kernel(ScanMulti m, uint64_t n) {
    __shared__ uint64_t sh[17];
    const uint32_t j = blockIdx.y;
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER;
    uint64_t v = 0;
    for (int k = 0; k < SCAN_PER; k++)
        if (base + k < n) v += m.in[j][base + k];
    uint64_t tot;
    block_excl_scan(v, sh, tot);
    if (threadIdx.x == 0) m.ws[j][blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_T) void scan_top_multi_kernel(ScanMulti m, uint64_t ntiles) {
    __shared__ uint64_t sh[17];
    const uint32_t j = blockIdx.x;
    uint64_t carry = 0;
    for (uint64_t b = 0; b < ntiles; b += SCAN_T) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < ntiles ? m.ws[j][i] : 0;
        uint64_t tot;
        const uint64_t e = block_excl_scan(v, sh, tot);
        if (i < ntiles) m.ws[j][i] = carry + e;
        carry += tot;
    }
    if (threadIdx.x == 0) *m.total[j] = carry;
}

__global__ __launch_bounds__(SCAN_T) void scan_apply_multi_kernel(ScanMulti m, uint64_t n) {
    __shared__ uint64_t sh[17];
    const uint32_t j = blockIdx.y;
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER;
    uint32_t v[SCAN_PER];
    uint64_t sum = 0;
    for (int k = 0; k < SCAN_PER; k++) {
        v[k] = base + k < n ? m.in[j][base + k] : 0;
        sum += v[k];
    }
    uint64_t tot;
    uint64_t p = m.ws[j][blockIdx.x] + block_excl_scan(sum, sh, tot);
    for (int k = 0; k < SCAN_PER; k++) {
        if (base + k < n) m.out32[j][base + k] = (uint32_t)p;
        p += v[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) m.out32[j][n] = (uint32_t)*m.total[j];
}

// Every child table's row positions to ~0 (unplaced) in one launch: table blockIdx.y
struct PosFill {
    uint64_t *p[TREE_MAX_T];
    uint64_t n[TREE_MAX_T];
};
__global__ __launch_bounds__(256) void tree_pos_fill_kernel(PosFill f) {
    uint64_t *p = f.p[blockIdx.y];
    const uint64_t n = f.n[blockIdx.y];
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) p[i] = ~0ull;
}

__global__ void tree_err_kernel(const uint32_t *err, uint64_t *total) {
    if (*err) *total = ~0ull;
}

size_t scan_ws_bytes(uint64_t n) { return ((n + SCAN_TILE - 1) / SCAN_TILE + 1) * sizeof(uint64_t); }

// k exclusive scans of n >= 1 elements each (ScanMulti filled for j < k), three launches
int launch_scan_multi(const ScanMulti &m, uint32_t k, uint64_t n, hipStream_t st) {
    const uint64_t tiles = std::max<uint64_t>(1, (n + SCAN_TILE - 1) / SCAN_TILE);
    hipLaunchKernelGGL(scan_tiles_multi_kernel, dim3((unsigned)tiles, k), dim3(SCAN_T), 0, st, m, n);
    hipLaunchKernelGGL(scan_top_multi_kernel, dim3(k), dim3(SCAN_T), 0, st, m, tiles);
    hipLaunchKernelGGL(scan_apply_multi_kernel, dim3((unsigned)tiles, k), dim3(SCAN_T), 0, st, m, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// exclusive scan of in[0, n) (in place allowed for out32); *total (device) = the sum
int launch_scan(const uint32_t *in, uint64_t n, uint32_t *out32, uint64_t *out64, uint64_t *ends64, uint64_t *ws,
                uint64_t *total, hipStream_t st) {
    const uint64_t tiles = std::max<uint64_t>(1, (n + SCAN_TILE - 1) / SCAN_TILE);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3((unsigned)tiles), dim3(SCAN_T), 0, st, in, n, ws);
    hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(SCAN_T), 0, st, ws, tiles, total);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)tiles), dim3(SCAN_T), 0, st, in, n, ws, total, out32, out64,
                       ends64);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- layout ---------------------------------------------------------------------------------

bool is_scalar(int k) { return k >= SPEC_KIND_BOOL && k <= SPEC_KIND_BYTES; }

// The whole host-side description of a tree: the ABI layout + the device descriptor.
struct Layout {
    spec_tree_table tables[TREE_MAX_T];
    spec_tree_column cols[TREE_MAX_C];
    uint32_t nt = 0, nc = 0;
    TreeDesc desc;
};

int add_col(Layout &L, int table, int field, int role, int kind, int width) {
    if (L.nc >= (uint32_t)TREE_MAX_C) return -1;
    spec_tree_column c;
    c.table = (uint16_t)table;
    c.field = (int16_t)field;
    c.role = (uint8_t)role;
    c.kind = (uint8_t)kind;
    c.width = (uint16_t)width;
    L.desc.width[L.nc] = (uint16_t)width;
    L.cols[L.nc] = c;
    return (int)L.nc++;
}

// Builds the layout; false on an invalid tree (rules: include/spec_amd.h spec_tree).
bool build_layout(const spec_tree *tr, Layout &L) {
    if (!tr || tr->nfields > (uint32_t)TREE_MAX_F) return false;
    const uint32_t nf = tr->nfields;
    const spec_tree_field *f = tr->fields;
    TreeDesc &D = L.desc;
    memset(&D, 0, sizeof(D));
    D.nfields = nf;
    for (uint32_t i = 0; i < nf; i++) {
        const int k = f[i].kind, p = f[i].parent;
        if (p < -1 || p >= (int)i) return false;
        if (!is_scalar(k) && k != SPEC_KIND_LIST && k != SPEC_KIND_STRUCT && k != SPEC_KIND_MESSAGE && k != SPEC_KIND_ANY)
            return false;
        if (k == SPEC_KIND_LIST && !is_scalar(f[i].elem) && f[i].elem != SPEC_KIND_STRUCT && f[i].elem != SPEC_KIND_MESSAGE)
            return false;
        if (p >= 0) {
            const int pk = f[p].kind;
            if (pk != SPEC_KIND_STRUCT && pk != SPEC_KIND_MESSAGE && pk != SPEC_KIND_LIST) return false;
            // struct members: value types or other structs (internal/lang/model/struct_field.go:57-70)
            if (pk == SPEC_KIND_STRUCT && !is_scalar(k) && k != SPEC_KIND_STRUCT) return false;
            if (pk == SPEC_KIND_LIST && is_scalar(f[p].elem)) return false;
            if (pk == SPEC_KIND_LIST && f[p].elem == SPEC_KIND_STRUCT && !is_scalar(k) && k != SPEC_KIND_STRUCT)
                return false;
        }
        TField &F = D.f[i];
        F.tag = f[i].tag;
        F.kind = (uint8_t)k;
        F.elem = f[i].elem;
        F.parent = (int16_t)p;
        F.table = F.col = F.present = -1;
        F.send = (uint16_t)(i + 1);
    }
    // subtree ends (pre-order: a field's descendants follow it) and struct nesting depth
    for (uint32_t i = 0; i < nf; i++) {
        int depth = 0;
        for (int p = f[i].parent; p >= 0; p = f[p].parent) {
            D.f[p].send = (uint16_t)std::max<uint32_t>(D.f[p].send, i + 1);
            if (f[p].kind == SPEC_KIND_STRUCT || (f[p].kind == SPEC_KIND_LIST && f[p].elem == SPEC_KIND_STRUCT)) depth++;
        }
        if (f[i].kind == SPEC_KIND_STRUCT) {
            depth++;
            if (f[i].parent >= 0 && (f[f[i].parent].kind == SPEC_KIND_STRUCT ||
                                     (f[f[i].parent].kind == SPEC_KIND_LIST && f[f[i].parent].elem == SPEC_KIND_STRUCT)))
                D.f[f[i].parent].nested = 1;
        }
        if (depth > TREE_MAX_SD) return false;
    }
    // a field's subtree must be contiguous (pre-order): every field inside [i + 1, send) descends from i
    for (uint32_t i = 0; i < nf; i++)
        for (uint32_t j = i + 1; j < D.f[i].send; j++) {
            int p = f[j].parent;
            while (p > (int)i) p = f[p].parent;
            if (p != (int)i) return false;
        }
    auto owner = [&](int i) {
        int p = f[i].parent;
        while (p >= 0 && f[p].kind == SPEC_KIND_STRUCT) p = f[p].parent;
        return p < 0 ? 0 : (int)D.f[p].table;
    };
    // tables
    L.tables[0] = spec_tree_table{-1, -1, SPEC_REL_ROOT, SPEC_SHAPE_MESSAGE, 0, 0};
    L.nt = 1;
    for (uint32_t i = 0; i < nf; i++) {
        const int k = f[i].kind;
        if (k != SPEC_KIND_MESSAGE && k != SPEC_KIND_LIST) continue;
        if (L.nt >= (uint32_t)TREE_MAX_T) return false;
        spec_tree_table t;
        t.parent = (int16_t)owner((int)i);
        t.field = (int16_t)i;
        t.rel = k == SPEC_KIND_MESSAGE ? SPEC_REL_ONE : SPEC_REL_MANY;
        t.shape = (k == SPEC_KIND_MESSAGE || f[i].elem == SPEC_KIND_MESSAGE) ? SPEC_SHAPE_MESSAGE
                  : f[i].elem == SPEC_KIND_STRUCT                             ? SPEC_SHAPE_STRUCT
                                                                              : SPEC_SHAPE_VALUE;
        t.first_column = t.ncolumns = 0;
        D.f[i].table = (int16_t)L.nt;
        L.tables[L.nt++] = t;
    }
    // members of structs (struct fields and lists of structs)
    uint32_t nm = 0;
    for (uint32_t i = 0; i < nf; i++) {
        const bool has_members = f[i].kind == SPEC_KIND_STRUCT || (f[i].kind == SPEC_KIND_LIST && f[i].elem == SPEC_KIND_STRUCT);
        if (!has_members) continue;
        D.f[i].mem0 = (uint16_t)nm;
        for (uint32_t j = i + 1; j < nf; j++)
            if (f[j].parent == (int)i) D.members[nm++] = (uint16_t)j;
        D.f[i].nmem = (uint16_t)(nm - D.f[i].mem0);
        if (D.f[i].nmem > (uint32_t)TREE_MAX_D) return false;
    }
    // columns, table by table; direct-field lists of message tables
    uint32_t nd_all = 0;
    for (uint32_t x = 0; x < L.nt; x++) {
        spec_tree_table &t = L.tables[x];
        TTable &T = D.t[x];
        const int d = t.field;
        T.parent = t.parent;
        T.field = (int16_t)d;
        T.rel = t.rel;
        T.shape = t.shape;
        T.begin_col = -1;
        t.first_column = (uint16_t)L.nc;
        if (t.rel == SPEC_REL_MANY && (T.begin_col = (int16_t)add_col(L, x, d, SPEC_COL_BEGIN, 0, 4)) < 0) return false;
        if (t.shape == SPEC_SHAPE_VALUE) {
            const int c = add_col(L, x, d, SPEC_COL_VALUE, f[d].elem, spec_kind_width(f[d].elem));
            if (c < 0) return false;
            D.f[d].col = (int16_t)c;
        } else if (t.shape == SPEC_SHAPE_STRUCT) {
            for (uint32_t j = (uint32_t)d + 1; j < D.f[d].send; j++) { // scalar members, pre-order
                if (!is_scalar(f[j].kind)) continue;
                const int c = add_col(L, x, (int)j, SPEC_COL_VALUE, f[j].kind, spec_kind_width(f[j].kind));
                if (c < 0) return false;
                D.f[j].col = (int16_t)c;
            }
        } else {
            T.d0 = (uint16_t)nd_all;
            for (uint32_t i = (uint32_t)(d + 1); i < nf; i++) {
                if (f[i].parent != d) continue;
                D.direct[nd_all++] = (uint16_t)i;
                const int k = f[i].kind;
                int c = 0;
                if (is_scalar(k)) {
                    c = D.f[i].col = (int16_t)add_col(L, x, i, SPEC_COL_VALUE, k, spec_kind_width(k));
                } else if (k == SPEC_KIND_ANY) {
                    c = D.f[i].col = (int16_t)add_col(L, x, i, SPEC_COL_VALUE, k, 8);
                    if (c >= 0) c = D.f[i].present = (int16_t)add_col(L, x, i, SPEC_COL_TYPE, 0, 1);
                } else if (k == SPEC_KIND_MESSAGE || k == SPEC_KIND_LIST) {
                    c = D.f[i].present = (int16_t)add_col(L, x, i, SPEC_COL_PRESENT, 0, 1);
                    T.has_children = 1;
                } else { // a struct: its scalar members (inner structs' in place), pre-order
                    for (uint32_t j = i + 1; j < D.f[i].send && c >= 0; j++) {
                        if (!is_scalar(f[j].kind)) continue;
                        c = D.f[j].col = (int16_t)add_col(L, x, (int)j, SPEC_COL_VALUE, f[j].kind, spec_kind_width(f[j].kind));
                    }
                }
                if (c < 0) return false;
            }
            T.nd = (uint16_t)(nd_all - T.d0);
            if (T.nd > (uint32_t)TREE_MAX_D) return false;
            // the writer's table order (insertion sort by tag; an equal tag written later goes
            // first: internal/writer/stack_msg.go:37-61) and each field's index in it
            uint16_t *srt = D.sorted + T.d0;
            for (uint32_t k = 0; k < T.nd; k++) {
                srt[k] = D.direct[T.d0 + k];
                for (int q = (int)k; q > 0 && D.f[srt[q - 1]].tag >= D.f[srt[q]].tag; q--) std::swap(srt[q - 1], srt[q]);
            }
            for (uint32_t k = 0; k < T.nd; k++) D.f[srt[k]].rank = (uint16_t)k;
            for (uint32_t k = 0; k < T.nd; k++)
                for (uint32_t q = 0; q < T.nd; q++)
                    if (D.direct[T.d0 + q] == srt[k]) D.sslot[T.d0 + k] = (uint16_t)q;
        }
        T.err_col = -1;
        if (t.shape == SPEC_SHAPE_MESSAGE && (T.err_col = (int16_t)add_col(L, x, d, SPEC_COL_ERRMASK, 0, 8)) < 0)
            return false;
        if ((T.status_col = (int16_t)add_col(L, x, d, SPEC_COL_STATUS, 0, 1)) < 0) return false;
        t.ncolumns = (uint16_t)(L.nc - t.first_column);
    }
    D.ntables = L.nt;
    D.ncols = L.nc;
    return true;
}

// grow-only device buffer
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int reserve(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes, 256);
        if (hipMalloc(&p, want) != hipSuccess) return -1;
        cap = want;
        return 0;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

} // namespace
} // namespace spec

using namespace spec;

struct spec_tree_decoder {
    Layout L;
    TreeBufs B;
    DevBuf desc, bufs, scan_ws, total;
    DevBuf rng[TREE_MAX_T], cnt[TREE_MAX_T];
    int device = 0;
    bool indexed = false;
};

extern "C" {

int spec_tree_layout(const spec_tree *tree, spec_tree_table *tables, uint32_t *ntables, spec_tree_column *columns,
                     uint32_t *ncolumns) {
    Layout *L = new (std::nothrow) Layout();
    if (!L) return SPEC_E_INVALID_ARGUMENT;
    const bool ok = build_layout(tree, *L);
    if (ok) {
        if (tables) memcpy(tables, L->tables, sizeof(spec_tree_table) * L->nt);
        if (columns) memcpy(columns, L->cols, sizeof(spec_tree_column) * L->nc);
        if (ntables) *ntables = L->nt;
        if (ncolumns) *ncolumns = L->nc;
    }
    delete L;
    return ok ? SPEC_OK : SPEC_E_INVALID_ARGUMENT;
}

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
    if (hipGetDevice(&d->device) != hipSuccess || d->desc.reserve(sizeof(TreeDesc)) ||
        d->bufs.reserve(sizeof(TreeBufs)) || d->total.reserve(sizeof(uint64_t) * TREE_MAX_T) ||
        hipMemcpy(d->desc.p, &d->L.desc, sizeof(TreeDesc), hipMemcpyHostToDevice) != hipSuccess) {
        note_hip_error(hipGetLastError());
        delete d;
        return SPEC_E_HIP;
    }
    *out = d;
    return SPEC_OK;
}

void spec_tree_decoder_destroy(spec_tree_decoder *d) { delete d; }

static int tree_index_impl(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len,
                           const uint64_t *ends, const uint2 *spans, uint64_t n, uint64_t *rows, void *stream) {
    if (!d || (n && (!stream_bytes || (!ends && !spans)))) return SPEC_E_INVALID_ARGUMENT;
    if (stream_len >= (1ull << 32)) return SPEC_E_TOO_LARGE;
    hipStream_t st = (hipStream_t)stream;
    Layout &L = d->L;
    TreeBufs &B = d->B;
    B.stream = stream_bytes;
    B.stream_len = stream_len;
    B.ends = ends;
    B.spans = spans;
    B.n = n;
    B.rows[0] = n;
    const TreeDesc *Dd = (const TreeDesc *)d->desc.p;
    TreeBufs *Bd = (TreeBufs *)d->bufs.p;
    auto upload = [&]() {
        return hipMemcpyAsync(Bd, &B, sizeof(TreeBufs), hipMemcpyHostToDevice, st) == hipSuccess &&
               hipStreamSynchronize(st) == hipSuccess;
    };
    for (uint32_t x = 0; x < L.nt; x++) {
        const uint64_t R = B.rows[x];
        const TTable &T = L.desc.t[x];
        if (T.shape != SHAPE_MESSAGE || !T.has_children) continue;
        // buffers of the child tables this table's rows feed
        for (uint32_t y = x + 1; y < L.nt; y++) {
            if (L.desc.t[y].parent != (int)x) continue;
            if (L.desc.t[y].rel == REL_ONE) {
                B.rows[y] = R;
                if (d->rng[y].reserve(std::max<uint64_t>(R, 1) * sizeof(uint2))) return SPEC_E_HIP;
                B.rng[y] = (uint2 *)d->rng[y].p;
            } else {
                if (d->cnt[y].reserve((R + 1) * sizeof(uint32_t))) return SPEC_E_HIP;
                B.cnt[y] = (uint32_t *)d->cnt[y].p;
            }
        }
        if (!upload()) return SPEC_E_HIP;
        const uint32_t slab = tree_slab(stream_len, R);
        if (R) hipLaunchKernelGGL(tree_index_kernel, dim3(row_grid(R)), dim3(TB), (TB / 64) * slab, st, Dd, Bd, x, R, slab);
        // every list child: counts -> begin (in place), its total into totals[y] (one batched scan
        // for all of them); then ONE copy of the totals to the host and one sync
        ScanMulti sm;
        uint32_t nl = 0;
        for (uint32_t y = x + 1; y < L.nt; y++) {
            if (L.desc.t[y].parent != (int)x || L.desc.t[y].rel != REL_MANY) continue;
            uint64_t *tot_y = (uint64_t *)d->total.p + y;
            if (R == 0) {
                (void)hipMemsetAsync(B.cnt[y], 0, sizeof(uint32_t), st);
                (void)hipMemsetAsync(tot_y, 0, sizeof(uint64_t), st);
            }
            sm.in[nl] = B.cnt[y];
            sm.out32[nl] = B.cnt[y];
            sm.total[nl] = tot_y;
            nl++;
        }
        if (!nl) continue;
        if (R) {
            const size_t wsb = (scan_ws_bytes(R) + 255) & ~(size_t)255;
            if (d->scan_ws.reserve(wsb * nl)) return SPEC_E_HIP;
            for (uint32_t j = 0; j < nl; j++) sm.ws[j] = (uint64_t *)((uint8_t *)d->scan_ws.p + wsb * j);
            if (launch_scan_multi(sm, nl, R, st)) return SPEC_E_HIP;
        }
        uint64_t tot[TREE_MAX_T];
        if (hipMemcpyAsync(tot, d->total.p, sizeof(uint64_t) * L.nt, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return SPEC_E_HIP;
        for (uint32_t y = x + 1; y < L.nt; y++) {
            if (L.desc.t[y].parent != (int)x || L.desc.t[y].rel != REL_MANY) continue;
            B.rows[y] = tot[y];
            if (d->rng[y].reserve(std::max<uint64_t>(tot[y], 1) * sizeof(uint2))) return SPEC_E_HIP;
            B.rng[y] = (uint2 *)d->rng[y].p;
        }
        if (!upload()) return SPEC_E_HIP;
        if (R) hipLaunchKernelGGL(tree_expand_kernel, dim3(row_grid(R)), dim3(TB), (TB / 64) * slab, st, Dd, Bd, x, R, slab);
    }
    // tables whose owner has no rows to index (empty batch / no message children) keep 0 rows
    for (uint32_t y = 1; y < L.nt; y++)
        if (L.desc.t[y].rel == REL_ONE) B.rows[y] = B.rows[L.desc.t[y].parent];
    if (rows) memcpy(rows, B.rows, sizeof(uint64_t) * L.nt);
    d->indexed = true;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        note_hip_error(e);
        return SPEC_E_HIP;
    }
    return SPEC_OK;
}

int spec_tree_decoder_index(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len,
                            const uint64_t *ends, uint64_t n, uint64_t *rows, void *stream) {
    return tree_index_impl(d, stream_bytes, stream_len, ends, nullptr, n, rows, stream);
}

int spec_tree_decoder_index_spans(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len,
                                  const spec_span *spans, uint64_t n, uint64_t *rows, void *stream) {
    if (n && !spans) return SPEC_E_INVALID_ARGUMENT;
    return tree_index_impl(d, stream_bytes, stream_len, nullptr, (const uint2 *)spans, n, rows, stream);
}

int spec_tree_decoder_decode(spec_tree_decoder *d, void *const *columns, void *stream) {
    if (!d || !d->indexed || !columns) return SPEC_E_INVALID_ARGUMENT;
    hipStream_t st = (hipStream_t)stream;
    Layout &L = d->L;
    TreeBufs &B = d->B;
    for (uint32_t c = 0; c < L.nc; c++) B.cols[c] = columns[c];
    // tables without an indexed owner row set still need range buffers for their (0) rows
    for (uint32_t y = 1; y < L.nt; y++) {
        if (!B.rng[y]) {
            if (d->rng[y].reserve(sizeof(uint2))) return SPEC_E_HIP;
            B.rng[y] = (uint2 *)d->rng[y].p;
        }
    }
    if (hipMemcpyAsync(d->bufs.p, &B, sizeof(TreeBufs), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return SPEC_E_HIP;
    const TreeDesc *Dd = (const TreeDesc *)d->desc.p;
    const TreeBufs *Bd = (const TreeBufs *)d->bufs.p;
    for (uint32_t x = 0; x < L.nt; x++) {
        const uint64_t R = B.rows[x];
        const TTable &T = L.desc.t[x];
        if (T.rel == REL_MANY && columns[T.begin_col]) {
            const uint64_t owner_rows = B.rows[T.parent];
            if (B.cnt[x]) {
                if (hipMemcpyAsync(columns[T.begin_col], B.cnt[x], (owner_rows + 1) * sizeof(uint32_t),
                                   hipMemcpyDeviceToDevice, st) != hipSuccess)
                    return SPEC_E_HIP;
            } else if (hipMemsetAsync(columns[T.begin_col], 0, (owner_rows + 1) * sizeof(uint32_t), st) != hipSuccess) {
                return SPEC_E_HIP;
            }
        }
        const uint32_t slab = tree_slab(B.stream_len, R);
        if (R) hipLaunchKernelGGL(tree_decode_kernel, dim3(row_grid(R)), dim3(TB), (TB / 64) * slab, st, Dd, Bd, x, R, slab);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        note_hip_error(e);
        return SPEC_E_HIP;
    }
    return SPEC_OK;
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

// ---- encode ----

namespace {
struct EncWs {
    size_t desc, bufs, size[TREE_MAX_T], pos[TREE_MAX_T], offsets, scan, err, total;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t enc_plan(const Layout &L, const uint64_t *rows, EncWs &w) {
    size_t o = 0;
    w.desc = o;
    o += align256(sizeof(TreeDesc));
    w.bufs = o;
    o += align256(sizeof(TreeBufs));
    for (uint32_t x = 0; x < L.nt; x++) {
        w.size[x] = o;
        o += align256(std::max<uint64_t>(rows[x], 1) * sizeof(uint32_t));
        w.pos[x] = o;
        o += align256(x ? std::max<uint64_t>(rows[x], 1) * sizeof(uint64_t) : 0);
    }
    w.offsets = o;
    o += align256(std::max<uint64_t>(rows[0], 1) * sizeof(uint64_t));
    w.scan = o;
    o += align256(scan_ws_bytes(rows[0]));
    w.err = o;
    o += 256;
    w.total = o;
    o += 256;
    return o;
}
} // namespace

size_t spec_encode_tree_workspace_size(const spec_tree *tree, const uint64_t *rows) {
    Layout *L = new (std::nothrow) Layout();
    if (!L || !rows || !build_layout(tree, *L)) {
        delete L;
        return 0;
    }
    EncWs w;
    const size_t s = enc_plan(*L, rows, w);
    delete L;
    return s;
}

int spec_encode_tree(const spec_tree *tree, const void *const *columns, const uint8_t *const *heaps,
                     const uint64_t *heap_lens, const uint64_t *rows, uint8_t *out, uint64_t out_cap, uint64_t *ends,
                     void *workspace, size_t workspace_size, uint64_t *total, void *stream) {
    if (!columns || !rows || !total || !workspace) return SPEC_E_INVALID_ARGUMENT;
    Layout *Lp = new (std::nothrow) Layout();
    if (!Lp) return SPEC_E_INVALID_ARGUMENT;
    if (!build_layout(tree, *Lp)) {
        delete Lp;
        return SPEC_E_INVALID_ARGUMENT;
    }
    Layout &L = *Lp;
    EncWs w;
    if (enc_plan(L, rows, w) > workspace_size) {
        delete Lp;
        return SPEC_E_WORKSPACE;
    }
    hipStream_t st = (hipStream_t)stream;
    uint8_t *ws = (uint8_t *)workspace;
    TreeBufs *B = new (std::nothrow) TreeBufs();
    if (!B) {
        delete Lp;
        return SPEC_E_INVALID_ARGUMENT;
    }
    memset(B, 0, sizeof(*B));
    int rc = SPEC_OK;
    for (uint32_t c = 0; c < L.nc; c++) {
        B->cols[c] = (void *)columns[c];
        B->heaps[c] = heaps ? heaps[c] : nullptr;
        B->heap_lens[c] = heap_lens ? heap_lens[c] : 0;
        const spec_tree_column &col = L.cols[c];
        const bool spans = col.role == SPEC_COL_VALUE && (col.kind == SPEC_KIND_STRING || col.kind == SPEC_KIND_BYTES ||
                                                         col.kind == SPEC_KIND_ANY);
        // a BEGIN column has owner rows + 1 entries: needed whenever the owner table has rows
        // (an owner whose lists are all empty still reads begin[row], begin[row + 1])
        const uint64_t col_rows = col.role == SPEC_COL_BEGIN ? rows[L.tables[col.table].parent] : rows[col.table];
        const bool input = col.role == SPEC_COL_VALUE || col.role == SPEC_COL_PRESENT || col.role == SPEC_COL_BEGIN;
        if (input && !columns[c] && col_rows) rc = SPEC_E_INVALID_ARGUMENT;
        if (spans && rows[col.table] && !B->heaps[c]) rc = SPEC_E_INVALID_ARGUMENT;
    }
    for (uint32_t x = 0; x < L.nt; x++) {
        B->rows[x] = rows[x];
        B->size[x] = (uint32_t *)(ws + w.size[x]);
        B->pos[x] = x ? (uint64_t *)(ws + w.pos[x]) : nullptr;
        if (L.tables[x].rel == SPEC_REL_ONE && rows[x] != rows[L.tables[x].parent]) rc = SPEC_E_INVALID_ARGUMENT;
    }
    if (rc) {
        delete B;
        delete Lp;
        return rc;
    }
    const uint64_t n = rows[0];
    B->n = n;
    B->out = out;
    B->out_cap = out ? out_cap : 0;
    B->ends_out = ends;
    B->offsets = (uint64_t *)(ws + w.offsets);
    B->total = total;
    B->err = (uint32_t *)(ws + w.err);
    const TreeDesc *Dd = (const TreeDesc *)(ws + w.desc);
    TreeBufs *Bd = (TreeBufs *)(ws + w.bufs);
    bool ok = hipMemcpyAsync(ws + w.desc, &L.desc, sizeof(TreeDesc), hipMemcpyHostToDevice, st) == hipSuccess &&
              hipMemcpyAsync(Bd, B, sizeof(TreeBufs), hipMemcpyHostToDevice, st) == hipSuccess &&
              hipMemsetAsync(B->err, 0, sizeof(uint32_t), st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
    // sizes bottom-up (children before their owners: table order is pre-order)
    for (int x = (int)L.nt - 1; ok && x >= 0; x--)
        if (rows[x]) hipLaunchKernelGGL(tree_size_kernel, dim3(row_grid(rows[x])), dim3(TB), 0, st, Dd, Bd, (uint32_t)x, rows[x]);
    // record offsets, ends, total
    if (ok) {
        if (n) {
            ok = launch_scan(B->size[0], n, nullptr, B->offsets, nullptr, (uint64_t *)(ws + w.scan), total, st) == 0;
        } else {
            ok = hipMemsetAsync(total, 0, sizeof(uint64_t), st) == hipSuccess;
        }
    }
    // an encoder error: total = all-ones
    if (ok) hipLaunchKernelGGL(tree_err_kernel, dim3(1), dim3(1), 0, st, (const uint32_t *)B->err, total);
    // child rows start unplaced: only rows their owner writes get a position
    if (ok && out && L.nt > 1) {
        PosFill pf;
        uint64_t most = 0;
        for (uint32_t x = 1; x < L.nt; x++) {
            pf.p[x - 1] = B->pos[x];
            pf.n[x - 1] = rows[x];
            most = std::max(most, rows[x]);
        }
        if (most) {
            const unsigned gx = (unsigned)std::min<uint64_t>((most + 255) / 256, 1024);
            hipLaunchKernelGGL(tree_pos_fill_kernel, dim3(gx, L.nt - 1), dim3(256), 0, st, pf);
        }
    }
    for (uint32_t x = 0; ok && out && x < L.nt; x++)
        if (rows[x]) {
            const TTable &T = L.desc.t[x];
            const size_t lds = T.shape == SHAPE_MESSAGE ? (size_t)(TB / 64) * T.nd * 64 * sizeof(uint32_t) : 0;
            hipLaunchKernelGGL(tree_write_kernel, dim3(row_grid(rows[x])), dim3(TB), lds, st, Dd, Bd, x, rows[x]);
        }
    const hipError_t e = hipGetLastError();
    delete B;
    delete Lp;
    if (!ok || e != hipSuccess) {
        note_hip_error(e);
        return SPEC_E_HIP;
    }
    return SPEC_OK;
}

} // extern "C"
