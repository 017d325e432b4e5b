// tree.hip — schema trees on the GPU (include/spec_amd.h spec_tree_*): the layout of a tree and
// the generated writers of internal/lang/generator (message.go:319-439, struct.go:115-142) over
// a batch, for every kind — structs, sub-messages, value lists, lists of structs/messages, any.
// Device code: tree_core.hpp; the decoder (generated readers): tree_decode.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "spec_internal.hpp"
#include "tree_internal.hpp"

namespace spec {

// Build-time measurement switch (make HIPFLAGS+="-DSPEC_AB_TREE_ENC_SPLIT=1"): the encoder's
// level-fused size / write launches split into one launch per table.
#ifndef SPEC_AB_TREE_ENC_SPLIT
#define SPEC_AB_TREE_ENC_SPLIT 0
#endif

unsigned row_grid(uint64_t rows) {
    const uint64_t b = (rows + TB - 1) / TB;
    const uint64_t cap = (uint64_t)device_cus() * 16;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, cap));
}

bool is_scalar(int k) { return k >= SPEC_KIND_BOOL && k <= SPEC_KIND_BYTES; }

namespace {

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
        BEmit em{{B.out}, start, start};
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
__global__ __launch_bounds__(SCAN_T) void scan_top_kernel(uint64_t *tile_sums, uint64_t ntiles, uint64_t *total,
                                                          const uint32_t *err) {
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
    if (threadIdx.x == 0) *total = err && *err ? ~0ull : carry; // an encoder error: all-ones
}

// pass 3: per tile, the exclusive prefix of every element: into out32 (u32, + out32[n] = total)
// or out64 (u64); ends64 (optional) = prefix + element.  fold (up to FOLD_TILES tiles, no pass 2):
// the tile's offset is the sum of the earlier tiles' totals, summed by the block itself (one load
// per thread), and block 0 sums every tile into *total (all-ones when *err).
constexpr uint64_t FOLD_TILES = 1024;
__global__ __launch_bounds__(SCAN_T) void scan_apply_kernel(const uint32_t *in, uint64_t n, const uint64_t *tile_sums,
                                                            uint64_t *total, uint32_t *out32, uint64_t *out64,
                                                            uint64_t *ends64, uint32_t fold, const uint32_t *err) {
    __shared__ uint64_t sh[17];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER;
    uint32_t v[SCAN_PER];
    uint64_t sum = 0;
    for (int k = 0; k < SCAN_PER; k++) {
        v[k] = base + k < n ? in[base + k] : 0;
        sum += v[k];
    }
    uint64_t tot, off = 0, grand = 0;
    if (fold) {
        const uint64_t ntiles = gridDim.x, lim = blockIdx.x ? (uint64_t)blockIdx.x : ntiles;
        uint64_t part = 0;
        for (uint64_t i = threadIdx.x; i < lim; i += SCAN_T) part += tile_sums[i];
        (void)block_excl_scan(part, sh, grand); // earlier tiles (block 0: every tile)
        off = blockIdx.x ? grand : 0;
        if (blockIdx.x == 0) grand = err && *err ? ~0ull : grand; // an encoder error: all-ones
        if (blockIdx.x == 0 && threadIdx.x == 0) *total = grand;
    } else {
        off = tile_sums[blockIdx.x];
    }
    uint64_t p = off + block_excl_scan(sum, sh, tot);
    for (int k = 0; k < SCAN_PER; k++) {
        if (base + k < n) {
            if (out32) out32[base + k] = (uint32_t)p;
            if (out64) out64[base + k] = p;
            if (ends64) ends64[base + k] = p + v[k];
        }
        p += v[k];
    }
    if (out32 && blockIdx.x == 0 && threadIdx.x == 0) out32[n] = (uint32_t)(fold ? grand : *total);
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

size_t scan_ws_bytes(uint64_t n) { return ((n + SCAN_TILE - 1) / SCAN_TILE + 1) * sizeof(uint64_t); }

// exclusive scan of in[0, n) (in place allowed for out32); *total (device) = the sum, or all-ones
// when *err (optional) is set
int launch_scan(const uint32_t *in, uint64_t n, uint32_t *out32, uint64_t *out64, uint64_t *ends64, uint64_t *ws,
                uint64_t *total, const uint32_t *err, hipStream_t st) {
    const uint64_t tiles = std::max<uint64_t>(1, (n + SCAN_TILE - 1) / SCAN_TILE);
    const uint32_t fold = tiles <= FOLD_TILES ? 1u : 0u;
    hipLaunchKernelGGL(scan_tiles_kernel, dim3((unsigned)tiles), dim3(SCAN_T), 0, st, in, n, ws);
    if (!fold) hipLaunchKernelGGL(scan_top_kernel, dim3(1), dim3(SCAN_T), 0, st, ws, tiles, total, err);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)tiles), dim3(SCAN_T), 0, st, in, n, ws, total, out32, out64,
                       ends64, fold, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace

// ---- layout (spec_tree_layout) ---------------------------------------------------------------------------------

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
            for (uint32_t q = 0; q < T.nd; q++) D.sslot[T.d0 + D.f[D.direct[T.d0 + q]].rank] = (uint16_t)q;
        }
        T.err_col = -1;
        // ERRMASK: a bit per direct field, ceil(nd / 64) words (at least one)
        if (t.shape == SPEC_SHAPE_MESSAGE &&
            (T.err_col = (int16_t)add_col(L, x, d, SPEC_COL_ERRMASK, 0, 8 * std::max<uint32_t>(1, (T.nd + 63) / 64))) < 0)
            return false;
        if ((T.status_col = (int16_t)add_col(L, x, d, SPEC_COL_STATUS, 0, 1)) < 0) return false;
        t.ncolumns = (uint16_t)(L.nc - t.first_column);
    }
    D.ntables = L.nt;
    D.ncols = L.nc;
    // decode groups (tree_decode.hip): every table hangs 1:1 off its owner's group unless it is a
    // list table, which starts its own; groups listed in pre-order, root first
    uint32_t ng = 0;
    for (uint32_t x = 0; x < L.nt; x++) {
        TTable &T = D.t[x];
        T.groot = (x == 0 || T.rel == REL_MANY) ? (uint16_t)x : D.t[T.parent].groot;
        T.gslot = 0xffff;
        T.gn = 0;
    }
    for (uint32_t x = 0; x < L.nt; x++) {
        TTable &T = D.t[x];
        if (T.groot != x) continue;
        T.g0 = (uint16_t)ng;
        for (uint32_t y = x; y < L.nt; y++) {
            if (D.t[y].groot != x) continue;
            if (y != x) D.t[y].gslot = (uint16_t)(T.gn - 1);
            D.group[ng++] = (uint16_t)y;
            T.gn++;
        }
    }
    return true;
}


} // namespace spec

using namespace spec;

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

// ---- encode ----

namespace {
struct EncWs {
    size_t desc, bufs, size[TREE_MAX_T], pos[TREE_MAX_T], offsets, scan, err, total, tblk, tmask;
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// [desc | bufs | err] first and contiguous: ONE upload (from a pinned slot) sets all three, the
// error word to zero
constexpr size_t ENC_HEAD_DESC = 0;
constexpr size_t ENC_HEAD_BUFS = (sizeof(TreeDesc) + 255) & ~(size_t)255;
constexpr size_t ENC_HEAD_ERR = ENC_HEAD_BUFS + ((sizeof(TreeBufs) + 255) & ~(size_t)255);
constexpr size_t ENC_HEAD = ENC_HEAD_ERR + 256;

size_t enc_plan(const Layout &L, const uint64_t *rows, EncWs &w) {
    size_t o = 0;
    w.desc = ENC_HEAD_DESC;
    w.bufs = ENC_HEAD_BUFS;
    w.err = ENC_HEAD_ERR;
    o = ENC_HEAD;
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
    w.total = o;
    o += 256;
    // the record-tile writer's per-record field-block offsets and presence masks (size pass)
    w.tblk = o;
    o += align256(std::max<uint64_t>(rows[0], 1) * TREE_TILE_W * sizeof(uint32_t));
    w.tmask = o;
    o += align256(std::max<uint64_t>(rows[0], 1) * sizeof(uint64_t));
    return o;
}
} // namespace

namespace {
// copies the workspace head [desc | bufs | err = 0] (ENC_HEAD bytes) to the device on st through
// the library's pinned upload pool (spec::pinned_upload: no host wait on the device); false on a
// HIP error
bool upload_head(const TreeDesc &desc, const TreeBufs &bufs, void *dhead, hipStream_t st) {
    thread_local std::vector<uint8_t> h;
    h.assign(ENC_HEAD, 0);
    memcpy(h.data() + ENC_HEAD_DESC, &desc, sizeof(TreeDesc));
    memcpy(h.data() + ENC_HEAD_BUFS, &bufs, sizeof(TreeBufs));
    return spec::pinned_upload(dhead, h.data(), ENC_HEAD, st) == hipSuccess;
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
    B->tblk = (uint32_t *)(ws + w.tblk);
    B->tmask = (uint64_t *)(ws + w.tmask);
    B->total = total;
    B->err = (uint32_t *)(ws + w.err);
    const TreeDesc *Dd = (const TreeDesc *)(ws + w.desc);
    TreeBufs *Bd = (TreeBufs *)(ws + w.bufs);
    // the generated writers and size passes (jit.cpp) for message tables, else the run-time row kernels
    const hipFunction_t *jit = jit_tree_kernels(L.desc);
    // level-fused launches (tree_core.hpp TableSet) when the generated module has them: the
    // tables of one height sized together (children have smaller heights), the tables of one
    // depth written together (owners have smaller depths)
    const bool sets = jit && jit[4 * TREE_MAX_T] && (jit[4 * TREE_MAX_T + 1] || jit[4 * TREE_MAX_T + 3]);
    // the run-time writer keeps a message's field ends in LDS ([wave][field][lane], 256 B per field
    // per wave, 160 KiB per block at most): a table of more than 640 direct fields needs the
    // generated writer (jit.cpp).  Checked before anything is issued, so a call that cannot run
    // leaves the stream, *total and out untouched.
    for (uint32_t x = 0; !sets && out && x < L.nt; x++)
        if (rows[x] && L.desc.t[x].shape == SHAPE_MESSAGE && (size_t)L.desc.t[x].nd * 64 * sizeof(uint32_t) > 163840) {
            delete B;
            delete Lp;
            return SPEC_E_TOO_LARGE;
        }
    bool ok = upload_head(L.desc, *B, ws, st);
    int height[TREE_MAX_T] = {0}, depth[TREE_MAX_T] = {0}, maxh = 0, maxd = 0;
    for (uint32_t x = 1; x < L.nt; x++) depth[x] = depth[L.desc.t[x].parent] + 1;
    for (int x = (int)L.nt - 1; x > 0; x--) {
        const int par = L.desc.t[x].parent;
        height[par] = std::max(height[par], height[x] + 1);
    }
    for (uint32_t x = 0; x < L.nt; x++) {
        maxh = std::max(maxh, height[x]);
        maxd = std::max(maxd, depth[x]);
    }
    auto launch_set = [&](hipFunction_t fn, const int *level, int lv) -> bool {
        TableSet ts;
        ts.n = 0;
        uint64_t most = 0;
        for (uint32_t x = 0; x < L.nt; x++)
            if (level[x] == lv && rows[x]) {
                ts.t[ts.n++] = x;
                most = std::max(most, rows[x]);
            }
        if (!ts.n) return true;
#if SPEC_AB_TREE_ENC_SPLIT
        // (measurement build: one launch per table, so a kernel trace times each table)
        for (uint32_t j = 0; j < ts.n; j++) {
            TableSet one;
            one.n = 1;
            one.t[0] = ts.t[j];
            void *a1[] = {(void *)&Dd, (void *)&Bd, &one};
            const hipError_t l1 = hipModuleLaunchKernel(fn, row_grid(rows[ts.t[j]]), 1, 1, TB, 1, 1, 0, st, a1, nullptr);
            if (l1 != hipSuccess) {
                note_hip_error(l1);
                return false;
            }
        }
        return true;
#endif
        void *args[] = {(void *)&Dd, (void *)&Bd, &ts};
        const hipError_t le = hipModuleLaunchKernel(fn, row_grid(most), ts.n, 1, TB, 1, 1, 0, st, args, nullptr);
        if (le != hipSuccess) note_hip_error(le);
        return le == hipSuccess;
    };
    for (int h = 0; sets && ok && h <= maxh; h++) ok = launch_set(jit[4 * TREE_MAX_T], height, h);
    // (no generated module: the run-time row kernels) sizes bottom-up (children before their
    // owners: table order is pre-order)
    for (int x = (int)L.nt - 1; !sets && ok && x >= 0; x--)
        if (rows[x])
            hipLaunchKernelGGL(tree_size_kernel, dim3(row_grid(rows[x])), dim3(TB), 0, st, Dd, Bd, (uint32_t)x, rows[x]);
    // record offsets, total (all-ones on an encoder error)
    if (ok) {
        if (n) {
            ok = launch_scan(B->size[0], n, nullptr, B->offsets, nullptr, (uint64_t *)(ws + w.scan), total, B->err,
                             st) == 0;
        } else {
            ok = hipMemsetAsync(total, 0, sizeof(uint64_t), st) == hipSuccess;
        }
    }
    // child rows start unplaced: only rows their owner writes get a position (the generated
    // writers mark the rows under an absent or unplaced owner themselves)
    if (!sets && ok && out && L.nt > 1) {
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
    const bool tile = sets && jit[4 * TREE_MAX_T + 3];
    if (tile && ok && out && n) {
        uint32_t cap = TREE_TILE_IMG;
        void *args[] = {(void *)&Dd, (void *)&Bd, &cap};
        const hipError_t le = hipModuleLaunchKernel(jit[4 * TREE_MAX_T + 3], (unsigned)((n + 63) / 64), 1, 1,
                                                    64 * TREE_TILE_W, 1, 1, TREE_TILE_IMG + 16, st, args,
                                                    nullptr);
        if (le != hipSuccess) note_hip_error(le);
        ok = le == hipSuccess;
    }
    for (int d = 0; sets && !tile && ok && out && d <= maxd; d++) ok = launch_set(jit[4 * TREE_MAX_T + 1], depth, d);
    bool too_wide = false;
    for (uint32_t x = 0; !sets && ok && out && !too_wide && x < L.nt; x++)
        if (rows[x]) {
            const TTable &T = L.desc.t[x];
            // a message's field ends live in LDS ([wave][field][lane], 256 B per field per wave):
            // fewer waves per block for a wide table (160 KiB per block at most); a table of more
            // than 640 direct fields needs the generated writer (jit.cpp)
            const size_t per_wave = T.shape == SHAPE_MESSAGE ? (size_t)T.nd * 64 * sizeof(uint32_t) : 0;
            const unsigned wpb = per_wave ? (unsigned)std::min<size_t>(TB / 64, 163840 / per_wave) : TB / 64;
            if (wpb == 0) {
                too_wide = true;
                break;
            }
            const uint64_t blocks = std::min<uint64_t>((rows[x] + 64 * wpb - 1) / (64 * wpb), (uint64_t)row_grid(rows[x]) * (TB / 64) / wpb);
            hipLaunchKernelGGL(tree_write_kernel, dim3((unsigned)std::max<uint64_t>(blocks, 1)), dim3(64 * wpb), wpb * per_wave, st,
                               Dd, Bd, x, rows[x]);
        }
    const hipError_t e = hipGetLastError();
    delete B;
    delete Lp;
    if (too_wide) return SPEC_E_TOO_LARGE;
    if (!ok || e != hipSuccess) {
        note_hip_error(e);
        return SPEC_E_HIP;
    }
    return SPEC_OK;
}

} // extern "C"
