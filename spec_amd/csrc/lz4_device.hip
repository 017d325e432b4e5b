// lz4_device.hip — LZ4 blocks of an mpx connection stream decompressed on the GPU
// (spec_lz4_decompress / spec_lz4_pack, include/spec_amd.h).
//
// mpx wraps the connection in one LZ4 frame of independent 256 KiB blocks (mpx/conn_writer.go:
// 42-56, pierrec/lz4/v4).  The host walks the frame's block headers (spec_lz4_frame_blocks:
// one u32 per block) and hands the block table over; here ONE WAVE DECODES ONE BLOCK, in
// batches of up to 64 sequences:
//   * PARSE (serial, uniform): the compressed bytes stream through a 16 KiB LDS ring (2 KiB
//     chunks loaded 4 KiB ahead); a sequence's token and, for literal runs up to 5 bytes, its
//     offset come from one 8-byte LDS read.  Each sequence is checked exactly as the reference
//     decoder checks it and recorded in the registers of lane k (k-th sequence of the batch):
//     literal source, literal length, output position, offset, match length;
//   * EXECUTE (the batch's output, at most 8 KiB, is assembled in an LDS window): every lane
//     copies its own short literal, long literals go wave-wide; matches read out[mop - off +
//     (i mod off)] — always bytes before mop — so a match whose source ends before the batch
//     (far) is read back from HBM by its own lane, all far matches at once; matches whose source
//     lies in the window (near; the few that straddle the window start read that part from HBM)
//     run in order, 64 bytes per instruction; then the window is stored to the block's slot;
//   * a sequence longer than 4 KiB (literal + match) runs alone, HBM to HBM.
// Errors are those of pierrec's decodeBlock (oracle/lz4.c so_lz4_decompress_block): the block's
// status is 1 and its size all-ones.  spec_lz4_pack then gathers the slots into one contiguous
// stream (exclusive scan of the sizes + a copy).
#include <hip/hip_runtime.h>

#include "spec_internal.hpp"

namespace spec {

namespace {

constexpr uint32_t CR = 16384, CRW = CR / 4, CHUNK = 2048, LOOK = 4096; // compressed ring
constexpr uint32_t WIN = 8192, SOLO = 4096, BATCH = 64;                 // output window

struct Lz4Args {
    const uint8_t *src;
    uint64_t src_len;
    const spec_lz4_block *blocks;
    uint64_t nblocks;
    uint8_t *slots;
    uint64_t slot;
    uint32_t *sizes;
    uint8_t *status;
};

// 4 source bytes at absolute offset o (zeros past the end; the last partial dword bytewise)
__device__ __forceinline__ uint32_t src_dword(const Lz4Args &a, __amdgpu_buffer_rsrc_t r, uint64_t o) {
    if (o + 4 <= a.src_len) return __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)o, 0, 0);
    uint32_t w = 0;
    for (uint32_t b = 0; b < 4; b++)
        if (o + b < a.src_len) w |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (uint32_t)(o + b), 0, 0) << (8 * b);
    return w;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// a byte of the block's output already stored by this wave (L2: sc1 bypasses the L1)
__device__ __forceinline__ uint8_t out_byte(__amdgpu_buffer_rsrc_t dr, uint32_t o) {
    return (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(dr, o, 0, 16);
}

__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(128) void lz4_block_kernel(Lz4Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t ringw[CRW];
    __shared__ __attribute__((aligned(16))) uint8_t win[WIN + 16];
    // the batch queue: two slots of per-lane records (literal source, literal length, output
    // position, offset, match length) and their batch's size / window / ring start
    __shared__ uint32_t q_desc[2][5][64], q_meta[2][3];
    __shared__ uint32_t q_posted, q_taken, q_done; // q_done: 1 parser finished, 2 failed
    const uint8_t *ring = (const uint8_t *)ringw;
    const uint64_t b = blockIdx.x;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        q_posted = 0;
        q_taken = 0;
        q_done = 0;
    }
    __syncthreads();
    const spec_lz4_block blk = a.blocks[b];
    const uint64_t base = blk.src_off;
    const uint32_t n = blk.src_len;
    uint8_t *dst = a.slots + b * a.slot;
    const uint32_t cap = (uint32_t)a.slot;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.src, (short)0, (int)(uint32_t)(a.src_len > 0xffffffffull ? 0xffffffffull : a.src_len), 0x00020000);
    __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc((void *)dst, (short)0, (int)cap, 0x00020000);
    bool err = base + n > a.src_len;
    if (!err && blk.stored) { // a block the writer stored uncompressed
        if (wave != 0) return;
        err = n > cap;
        if (!err)
            for (uint32_t i = lane; i < n; i += 64) dst[i] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, (uint32_t)(base + i), 0, 0);
        if (lane == 0) {
            a.sizes[b] = err ? 0xffffffffu : n;
            a.status[b] = err ? 1 : 0;
        }
        return;
    }
    err |= n == 0;
    if (err && wave != 0) return;
    if (wave == 1) { // ---- the copier: runs the parser's batches in order
        uint32_t taken = 0;
        for (;;) {
            for (;;) {
                if (__hip_atomic_load(&q_posted, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) > taken) break;
                const uint32_t d = __hip_atomic_load(&q_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (d == 2) return;
                if (d == 1 && __hip_atomic_load(&q_posted, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= taken)
                    return;
                __builtin_amdgcn_s_sleep(1);
            }
            const uint32_t slot = taken & 1;
            const uint32_t nb = q_meta[slot][0], first_op = q_meta[slot][1], wb = q_meta[slot][2];
            const uint32_t r_lit = q_desc[slot][0][lane], r_ll = q_desc[slot][1][lane], r_op = q_desc[slot][2][lane];
            const uint32_t r_off = q_desc[slot][3][lane], r_ml = q_desc[slot][4][lane];
            const bool mine = lane < nb;
            const uint32_t mop = r_op + r_ll, msrc = mop - r_off, mspan = r_off < r_ml ? r_off : r_ml;
            wave_lds_fence();
            // (1) literals (all in the ring): each lane its first 16 bytes, longer ones wave-wide
#pragma unroll
            for (uint32_t t = 0; t < 16; t++)
                if (mine && t < r_ll) win[r_op + t - wb] = ring[(r_lit + t) & (CR - 1)];
            uint64_t longlit = __ballot(mine && r_ll > 16);
            while (longlit) {
                const uint32_t k = (uint32_t)__builtin_ctzll(longlit);
                longlit &= longlit - 1;
                const uint32_t lit = uni(__builtin_amdgcn_readlane(r_lit, k)), ll = uni(__builtin_amdgcn_readlane(r_ll, k));
                const uint32_t o = uni(__builtin_amdgcn_readlane(r_op, k));
                for (uint32_t c = 16; c < ll; c += 64)
                    if (c + lane < ll) win[o + c + lane - wb] = ring[(lit + c + lane) & (CR - 1)];
            }
            // (2) far matches (source before the window): each lane reads its own from HBM
            const bool far = mine && r_ml > 0 && msrc + mspan <= first_op;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // earlier batches' stores have landed
            uint32_t farmax = 0;
            {
                uint32_t m = far ? r_ml : 0;
                for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d));
                farmax = uni(m);
            }
            for (uint32_t c = 0; c < farmax; c += 16) {
                uint8_t v[16];
#pragma unroll
                for (uint32_t t = 0; t < 16; t++) {
                    const uint32_t i = c + t;
                    v[t] = (far && i < r_ml) ? out_byte(dr, msrc + (r_off >= r_ml ? i : i % r_off)) : 0;
                }
#pragma unroll
                for (uint32_t t = 0; t < 16; t++)
                    if (far && c + t < r_ml) win[mop + c + t - wb] = v[t];
            }
            // (3) near (and straddling) matches, in order, 64 bytes per instruction
            uint64_t near = __ballot(mine && r_ml > 0 && !far);
            while (near) {
                const uint32_t k = (uint32_t)__builtin_ctzll(near);
                near &= near - 1;
                const uint32_t o = uni(__builtin_amdgcn_readlane(mop, k)), off = uni(__builtin_amdgcn_readlane(r_off, k));
                const uint32_t ml = uni(__builtin_amdgcn_readlane(r_ml, k));
                wave_lds_fence();
                for (uint32_t c = 0; c < ml; c += 64) {
                    const uint32_t i = c + lane;
                    const uint32_t sidx = o - off + (off >= ml ? i : i % off);
                    uint8_t v = 0;
                    if (i < ml) v = sidx >= first_op ? win[sidx - wb] : out_byte(dr, sidx);
                    __builtin_amdgcn_wave_barrier();
                    if (i < ml) win[o + i - wb] = v;
                }
            }
            wave_lds_fence();
            // (4) the window [first_op, end) to the slot: dwords where whole, bytes at the edges
            const uint32_t end = uni(__builtin_amdgcn_readlane(r_op + r_ll + r_ml, nb - 1));
            for (uint32_t u = first_op & ~3u; u < end; u += 256) {
                const uint32_t ad = u + 4 * lane;
                if (ad >= first_op && ad + 4 <= end) {
                    *(uint32_t *)(dst + ad) = *(const uint32_t *)(win + (ad - wb));
                } else {
                    for (uint32_t t = 0; t < 4; t++)
                        if (ad + t >= first_op && ad + t < end) dst[ad + t] = win[ad + t - wb];
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // landed: the parser's alone-sequences read them
            taken++;
            __hip_atomic_store(&q_taken, taken, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }

    // ---- ring: compressed bytes [max(vlo, filled - CR), filled) are in ring[x mod CR]; a chunk
    // is only loaded while it leaves the batch's literals (>= bs) in place
    uint32_t filled = 0, vlo = 0, bs = 0;
    // one chunk is kept in flight in registers (pf, for the bytes at pf_at) while the batch runs
    uint32_t pf[CHUNK / 256], pf_at = ~0u;
    auto fetch = [&](uint32_t at, uint32_t *v) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t j = 0; j < CHUNK / 256; j++) v[j] = src_dword(a, r, base + at + 4 * (lane + 64 * j));
    };
    auto load_chunk = [&]() __attribute__((always_inline)) {
        uint32_t v[CHUNK / 256];
        if (pf_at == filled) {
#pragma unroll
            for (uint32_t j = 0; j < CHUNK / 256; j++) v[j] = pf[j];
        } else {
            fetch(filled, v);
        }
#pragma unroll
        for (uint32_t j = 0; j < CHUNK / 256; j++) ringw[((filled >> 2) + lane + 64 * j) & (CRW - 1)] = v[j];
        filled += CHUNK;
    };
    // 8 bytes at x (uniform; must be loaded)
    auto rd8 = [&](uint32_t x) __attribute__((always_inline)) -> uint64_t {
        const uint32_t d = x >> 2, sh = 8 * (x & 3);
        const uint32_t w0 = ringw[d & (CRW - 1)], w1 = ringw[(d + 1) & (CRW - 1)], w2 = ringw[(d + 2) & (CRW - 1)];
        const uint64_t lo = (((uint64_t)w1 << 32) | w0) >> sh;
        const uint64_t v = sh ? lo | ((uint64_t)w2 << (64 - sh)) : lo;
        return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
    };

    // ---- the parser: lane k holds sequence k of the batch being assembled
    uint32_t nb = 0, first_op = 0, wb = 0, posted = 0, bs_of[2] = {0, 0};
    uint32_t r_lit = 0, r_ll = 0, r_op = 0, r_off = 0, r_ml = 0;
    auto taken_now = [&]() __attribute__((always_inline)) -> uint32_t {
        return uni(__hip_atomic_load(&q_taken, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
    };
    // hand the batch to the copier (waiting for a free slot)
    auto post = [&]() __attribute__((always_inline)) {
        while (posted - taken_now() >= 2) __builtin_amdgcn_s_sleep(1);
        const uint32_t slot = posted & 1;
        q_desc[slot][0][lane] = r_lit;
        q_desc[slot][1][lane] = r_ll;
        q_desc[slot][2][lane] = r_op;
        q_desc[slot][3][lane] = r_off;
        q_desc[slot][4][lane] = r_ml;
        if (lane == 0) {
            q_meta[slot][0] = nb;
            q_meta[slot][1] = first_op;
            q_meta[slot][2] = wb;
        }
        bs_of[slot] = bs;
        posted++;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&q_posted, posted, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        nb = 0;
    };
    // the ring start that unconsumed batches still need (their literals)
    auto oldest = [&](uint32_t cur) __attribute__((always_inline)) -> uint32_t {
        const uint32_t t = taken_now();
        return t < posted ? (bs_of[t & 1] < cur ? bs_of[t & 1] : cur) : cur;
    };

    // 8 bytes at x: from the ring when loaded, else (the headers of sequences too long for the
    // ring's look-ahead) straight from HBM
    auto rd = [&](uint32_t x) __attribute__((always_inline)) -> uint64_t {
        if (x + 8 <= filled && x + CR >= filled + 8 && x >= vlo) return rd8(x);
        uint64_t v = 0;
        for (uint32_t t = 0; t < 8; t++)
            v |= (uint64_t)(x + t < n ? __builtin_amdgcn_raw_buffer_load_b8(r, (uint32_t)(base + x + t), 0, 0) : 0u) << (8 * t);
        return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
    };
    // a length extension starting at x: adds bytes until one is not 255; false past the block
    auto ext = [&](uint32_t &x, uint32_t &len) __attribute__((always_inline)) -> bool {
        for (;;) {
            if (x >= n) return false;
            const uint32_t v = (uint32_t)(rd(x++) & 0xff);
            len += v;
            if (v != 255) return true;
        }
    };

    uint32_t ip = 0, op = 0, guard = 0;
    bool end = false;
    // every pass of either loop below consumes input or runs a batch; the guard only turns a
    // logic slip into a failed block instead of a wave that never finishes
    const uint32_t guard_max = 4 * n + 4096;
    while (!err && !end) {
        if (++guard > guard_max) {
            err = true;
            break;
        }
        // ---- top up the ring to LOOK bytes past ip, keeping what unconsumed batches need
        bs = oldest(ip);
        if (filled < n && ip + LOOK > filled) {
            if (filled + CR < ip || filled < (ip & ~3u)) { // skip what nobody reads from the ring
                filled = ip & ~3u;
                vlo = filled;
            }
            while (filled < ip + LOOK && filled < n && filled + CHUNK <= bs + CR) load_chunk();
            wave_lds_fence();
        }
        if (filled < n && pf_at != filled) { // the next chunk, in flight while this batch runs
            fetch(filled, pf);
            pf_at = filled;
        }
        if (filled < n && ip + 8 > filled) { // the ring is full of unconsumed batches: wait for the copier
            const uint32_t t = taken_now();
            if (t >= posted) { // nothing to wait for: cannot happen
                err = true;
                break;
            }
            while (taken_now() == t) __builtin_amdgcn_s_sleep(1);
            guard--;
            continue;
        }
        const uint32_t lim = filled >= n ? 0xffffffffu : filled;
        bs = ip; // this batch's literals start here
        // ---- the chain: up to 64 sequences (lengths only; lane k records sequence k) whose
        // bytes are all in the ring and whose output fits the window
        first_op = op;
        wb = op & ~15u;
        uint32_t o = op, c_pos = 0, c_op = 0;
        bool solo = false;
        uint32_t s_lit = 0, s_ll = 0, s_ml = 0, s_q = 0;
        // Speculative next-pointers: for each of the 256 positions x of a window, as if a token
        // sat at x, (next token - x) | (literal + match length) << 16 — or ~0 when that
        // sequence needs the careful path (a length extension of 255s, bytes past the ring or
        // the block, an error).  The chain then costs one readlane per sequence.
        auto spec_next = [&](uint32_t x) __attribute__((always_inline)) -> uint32_t {
            // straight-line: every byte read (masked into the ring), the verdict by selects
            const uint32_t t = ring[x & (CR - 1)], b1 = ring[(x + 1) & (CR - 1)];
            const uint32_t llnib = t >> 4, mlnib = t & 15;
            const bool e1 = llnib == 15, e2 = mlnib == 15;
            const uint32_t ll = llnib + (e1 ? b1 : 0u), lit = x + 1 + (e1 ? 1u : 0u), q = lit + ll;
            const uint32_t b2 = ring[(q + 2) & (CR - 1)];
            const uint32_t ml = mlnib + 4 + (e2 ? b2 : 0u), nx = q + 2 + (e2 ? 1u : 0u);
            const bool last = q == n && mlnib == 0;
            const bool bad = (x + 4 > lim) | (x >= n) | (e1 & (b1 == 255)) | (lit > n) | (ll > n - lit) |
                             (!last & ((q + 2 > n) | (q + 3 > lim) | (e2 & ((q + 2 >= n) | (b2 == 255))) |
                                       (nx + 8 > lim)));
            const uint32_t res = last ? (n - x) | (ll << 16) : (nx - x) | ((ll + ml) << 16);
            return bad ? ~0u : res;
        };
        uint32_t swb = 0, sp0 = 0, sp1 = 0, sp2 = 0, sp3 = 0;
        bool sval = false, full = false; // sval: the window [swb, swb + 256) is computed
        while (nb < BATCH) {
            // the fast chain: one readlane per sequence while the window knows the next token
            for (;;) {
                if (ip >= n || ip + 8 > lim || nb >= BATCH) break;
                if (!sval || ip - swb >= 256) {
                    sval = true;
                    swb = ip;
                    sp0 = spec_next(swb + lane);
                    sp1 = spec_next(swb + 64 + lane);
                    sp2 = spec_next(swb + 128 + lane);
                    sp3 = spec_next(swb + 192 + lane);
                }
                const uint32_t rel = ip - swb, l = rel & 63, kq = rel >> 6;
                const uint32_t v0 = __builtin_amdgcn_readlane(sp0, l), v1 = __builtin_amdgcn_readlane(sp1, l);
                const uint32_t v2 = __builtin_amdgcn_readlane(sp2, l), v3 = __builtin_amdgcn_readlane(sp3, l);
                const uint32_t v = kq == 0 ? v0 : kq == 1 ? v1 : kq == 2 ? v2 : v3;
                if (v == ~0u || (v & 0xffff) == 0) break; // the careful path
                const uint32_t total = v >> 16;
                if (o + total - wb > WIN) { // the batch is full: run it, top up
                    full = true;
                    break;
                }
                if (lane == nb) {
                    c_pos = ip;
                    c_op = o;
                }
                nb++;
                o += total;
                ip += v & 0xffff;
            }
            if (full || nb >= BATCH) break;
            if (ip >= n) { // the last sequence ended exactly at the block end
                end = true;
                break;
            }
            if (ip + 8 > lim || ++guard > guard_max) break;
            // ---- the careful path: this sequence parsed and checked serially
            const uint32_t token = (uint32_t)(rd8(ip) & 0xff);
            uint32_t ll = token >> 4, x = ip + 1;
            if (ll == 15 && !ext(x, ll)) {
                err = true;
                break;
            }
            const uint32_t lit = x;
            if (ll > n - lit || ll > cap - o) { // the reference: si + ll > n || di + ll > cap
                err = true;
                break;
            }
            const uint32_t q = lit + ll;
            uint32_t ml = token & 15, nxt;
            const bool last = q == n && ml == 0;
            if (last) {
                nxt = n;
            } else {
                if (q + 2 > n) {
                    err = true;
                    break;
                }
                ml += 4;
                nxt = q + 2;
                if (ml == 19 && !ext(nxt, ml)) {
                    err = true;
                    break;
                }
            }
            const uint32_t total = ll + ml;
            const bool fits = nxt + 8 <= lim || lim == 0xffffffffu;
            if (total > SOLO || (!fits && nb == 0)) { // alone, after the batch
                if (nb > 0) break;
                solo = true;
                s_lit = lit;
                s_ll = ll;
                s_ml = ml;
                s_q = last ? ~0u : q;
                ip = nxt;
                end = last;
                break;
            }
            if (!fits || o + total - wb > WIN) break; // the batch is full: run it, top up
            if (lane == nb) {
                c_pos = ip;
                c_op = o;
            }
            nb++;
            o += total;
            ip = nxt;
        }
        if (err) break;
        // ---- every lane parses its own sequence again (all its bytes are in the ring) and makes
        // the reference's remaining checks
        if (nb > 0) {
            const bool mine = lane < nb;
            uint32_t ll = 0, ml = 0, off = 0, lit = 0;
            bool bad = false;
            if (mine) {
                const uint32_t t = ring[c_pos & (CR - 1)];
                uint32_t x = c_pos + 1;
                ll = t >> 4;
                if (ll == 15)
                    for (uint32_t v = 255, i = 0; v == 255 && i < 32; i++) { // <= SOLO: < 17 bytes
                        v = ring[(x++) & (CR - 1)];
                        ll += v;
                    }
                lit = x;
                const uint32_t q = lit + ll, mlnib = t & 15;
                if (!(q == n && mlnib == 0)) {
                    off = (uint32_t)ring[q & (CR - 1)] | ((uint32_t)ring[(q + 1) & (CR - 1)] << 8);
                    ml = mlnib + 4;
                    if (mlnib == 15)
                        for (uint32_t v = 255, y = q + 2, i = 0; v == 255 && i < 32; i++) {
                            v = ring[(y++) & (CR - 1)];
                            ml += v;
                        }
                    const uint32_t di = c_op + ll;
                    bad = off == 0 || off > di || ml > cap - di;
                }
                bad |= ll > cap - c_op;
            }
            if (__ballot(bad)) {
                err = true;
                break;
            }
            r_lit = lit;
            r_ll = ll;
            r_op = c_op;
            r_off = off;
            r_ml = ml;
            op = o;
            post();
        }
        if (solo) { // HBM to HBM, once the copier has stored every batch before it
            while (taken_now() < posted) __builtin_amdgcn_s_sleep(1);
            uint32_t off = 0;
            if (s_q != ~0u) {
                off = (uint32_t)(rd(s_q) & 0xffff);
                if (off == 0 || off > op + s_ll || s_ml > cap - op - s_ll) {
                    err = true;
                    break;
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t mop = op + s_ll;
            for (uint32_t c = 0; c < s_ll; c += 64)
                if (c + lane < s_ll)
                    dst[op + c + lane] = (uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, (uint32_t)(base + s_lit + c + lane), 0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            for (uint32_t c = 0; c < s_ml; c += 64) {
                const uint32_t i = c + lane;
                if (i < s_ml) dst[mop + i] = out_byte(dr, mop - off + (off >= s_ml ? i : i % off));
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            op = mop + s_ml;
        }
    }
    if (lane == 0) __hip_atomic_store(&q_done, err ? 2u : 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!err)
        while (taken_now() < posted) __builtin_amdgcn_s_sleep(1);
    if (lane == 0) {
        a.sizes[b] = err ? 0xffffffffu : op;
        a.status[b] = err ? 1 : 0;
    }
}

// exclusive scan of the block sizes (one workgroup) -> offsets[0..nblocks], all-ones if any
// block failed
__global__ __launch_bounds__(1024) void lz4_scan_kernel(const uint32_t *sizes, uint64_t nblocks, uint64_t *offsets,
                                                        uint64_t *total) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry_s;
    __shared__ int err_s;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) {
        carry_s = 0;
        err_s = 0;
    }
    __syncthreads();
    for (uint64_t b0 = 0; b0 < nblocks; b0 += 1024) {
        const uint64_t i = b0 + t;
        uint64_t v = i < nblocks ? sizes[i] : 0;
        if (v == 0xffffffffu) {
            err_s = 1;
            v = 0;
        }
        uint64_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint64_t before = 0;
        for (int k = 0; k < w; k++) before += wsum[k];
        const uint64_t carry = carry_s;
        if (i < nblocks) offsets[i] = carry + before + x - v;
        __syncthreads();
        if (t == 1023) carry_s = carry + before + x;
        __syncthreads();
    }
    if (t == 0) {
        offsets[nblocks] = carry_s;
        *total = err_s ? ~0ull : carry_s;
    }
}

// one workgroup per block: slot -> out + offset (16-byte loads from the slot, byte-aligned
// destination assembled with dword stores where aligned)
__global__ __launch_bounds__(256) void lz4_gather_kernel(const uint8_t *slots, uint64_t slot, const uint32_t *sizes,
                                                         const uint64_t *offsets, uint64_t nblocks, uint8_t *out,
                                                         uint64_t out_cap, const uint64_t *total) {
    const uint64_t b = blockIdx.x;
    if (*total == ~0ull || *total > out_cap) return;
    const uint32_t n = sizes[b];
    const uint8_t *s = slots + b * slot;
    uint8_t *d = out + offsets[b];
    // head bytes until d is 4-aligned, then dwords (unaligned source reads), then the tail
    uint32_t head = (uint32_t)((4 - ((uint64_t)d & 3)) & 3);
    if (head > n) head = n;
    if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
    const uint32_t body = (n - head) / 4;
    for (uint32_t i = threadIdx.x; i < body; i += blockDim.x) {
        const uint8_t *q = s + head + 4 * i;
        const uint32_t v = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
        *(uint32_t *)(d + head + 4 * i) = v;
    }
    const uint32_t done = head + 4 * body;
    if (threadIdx.x < n - done) d[done + threadIdx.x] = s[done + threadIdx.x];
}

} // namespace

int launch_lz4_decompress(const uint8_t *src, uint64_t src_len, const spec_lz4_block *blocks, uint64_t nblocks,
                          uint8_t *slots, uint64_t slot, uint32_t *sizes, uint8_t *status, hipStream_t stream) {
    if (nblocks == 0) return 0;
    Lz4Args a = {src, src_len, blocks, nblocks, slots, slot, sizes, status};
    hipLaunchKernelGGL(lz4_block_kernel, dim3((unsigned)nblocks), dim3(128), 0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- the frame's content checksum: xxHash32 (seed 0) streamed over the decompressed bytes ----
// (the published algorithm; oracle/lz4.c so_xxh32 and lz4_host.cpp xxh32 are the host versions).
// One wave: lane 0 merges a partial stripe carried in the state, lanes 0..3 run the four
// accumulators over the 16-byte stripes (each lane dword i of every stripe, from aligned dword
// loads funnel-shifted to the data's byte phase, 32 stripes ahead of the chain), lane 0 keeps the
// tail.  (Byte-wise loads of unaligned words: 0.58 GB/s with a lane per accumulator, 0.31 GB/s
// with the four chains interleaved in one lane.)
namespace {
constexpr uint32_t XP1 = 2654435761u, XP2 = 2246822519u, XP3 = 3266489917u, XP4 = 668265263u, XP5 = 374761393u;

__device__ __forceinline__ uint32_t xrotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t xround(uint32_t v, uint32_t x) { return xrotl(v + x * XP2, 13) * XP1; }
__device__ __forceinline__ uint32_t ld32u(const uint8_t *p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}

__global__ __launch_bounds__(64) void lz4_content_kernel(spec_lz4_content *c, const uint8_t *data, uint64_t len,
                                                          uint32_t *digest) {
    __shared__ uint32_t vv[4];
    __shared__ uint64_t head_bytes;
    const int lane = threadIdx.x;
    if (lane == 0) {
        if (!c->started) {
            c->v[0] = XP1 + XP2;
            c->v[1] = XP2;
            c->v[2] = 0;
            c->v[3] = 0u - XP1;
            c->started = 1;
        }
        uint64_t take = 0;
        if (data && c->buffered) { // complete the carried stripe
            take = 16 - c->buffered < len ? 16 - c->buffered : len;
            for (uint64_t i = 0; i < take; i++) c->buf[c->buffered + i] = data[i];
            c->buffered += (uint32_t)take;
            if (c->buffered == 16) {
                for (int i = 0; i < 4; i++) c->v[i] = xround(c->v[i], ld32u(c->buf + 4 * i));
                c->buffered = 0;
            }
        }
        head_bytes = take;
        for (int i = 0; i < 4; i++) vv[i] = c->v[i];
    }
    __syncthreads();
    if (data) {
        const uint64_t p0 = head_bytes;
        const uint64_t ns = len > p0 ? (len - p0) / 16 : 0;
        if (lane < 4) {
            // lane i: accumulator i over dword i of every stripe, read as aligned dwords and
            // funnel-shifted (the data may start at any byte; an aligned dword that holds a byte
            // of the data lies in a mapped page), 32 stripes' loads ahead of the chain
            const uintptr_t qa = (uintptr_t)(data + p0);
            const uint32_t *w = (const uint32_t *)(qa & ~(uintptr_t)3) + lane;
            const uint32_t sh = (uint32_t)(qa & 3);
            uint32_t v = vv[lane];
            constexpr int U = 32;
            uint64_t s = 0;
            auto word = [&](uint64_t st) __attribute__((always_inline)) {
                const uint32_t lo = w[4 * st], hi = sh ? w[4 * st + 1] : 0u;
                return __builtin_amdgcn_alignbyte(hi, lo, sh);
            };
            if (ns >= U) {
                uint32_t x[U];
#pragma unroll
                for (int k = 0; k < U; k++) x[k] = word(k);
                for (; s + 2 * U <= ns; s += U) {
                    uint32_t y[U];
#pragma unroll
                    for (int k = 0; k < U; k++) y[k] = word(s + U + k); // the next batch in flight
#pragma unroll
                    for (int k = 0; k < U; k++) v = xround(v, x[k]);
#pragma unroll
                    for (int k = 0; k < U; k++) x[k] = y[k];
                }
#pragma unroll
                for (int k = 0; k < U; k++) v = xround(v, x[k]);
                s += U;
            }
            for (; s < ns; s++) v = xround(v, word(s));
            vv[lane] = v;
        }
        __syncthreads();
        if (lane == 0) {
            for (int i = 0; i < 4; i++) c->v[i] = vv[i];
            const uint64_t done = p0 + 16 * ns;
            for (uint64_t i = done; i < len; i++) c->buf[c->buffered++] = data[i];
            c->total += len;
        }
    }
    if (digest && lane == 0) {
        uint32_t h = c->total >= 16 ? xrotl(c->v[0], 1) + xrotl(c->v[1], 7) + xrotl(c->v[2], 12) + xrotl(c->v[3], 18)
                                    : XP5;
        h += (uint32_t)c->total;
        uint32_t i = 0;
        for (; i + 4 <= c->buffered; i += 4) h = xrotl(h + ld32u(c->buf + i) * XP3, 17) * XP4;
        for (; i < c->buffered; i++) h = xrotl(h + c->buf[i] * XP5, 11) * XP1;
        h ^= h >> 15;
        h *= XP2;
        h ^= h >> 13;
        h *= XP3;
        h ^= h >> 16;
        *digest = h;
    }
}
} // namespace

int launch_lz4_content(spec_lz4_content *c, const uint8_t *data, uint64_t len, uint32_t *digest, hipStream_t stream) {
    hipLaunchKernelGGL(lz4_content_kernel, dim3(1), dim3(64), 0, stream, c, len ? data : nullptr, len, digest);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lz4_pack(const uint8_t *slots, uint64_t slot, const uint32_t *sizes, uint64_t nblocks, uint8_t *out,
                    uint64_t out_cap, uint64_t *offsets, uint64_t *total, hipStream_t stream) {
    hipLaunchKernelGGL(lz4_scan_kernel, dim3(1), dim3(1024), 0, stream, sizes, nblocks, offsets, total);
    if (nblocks)
        hipLaunchKernelGGL(lz4_gather_kernel, dim3((unsigned)nblocks), dim3(256), 0, stream, slots, slot, sizes,
                           (const uint64_t *)offsets, nblocks, out, out_cap, (const uint64_t *)total);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace spec
