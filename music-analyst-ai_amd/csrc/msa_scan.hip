// msa_scan.hip -- record/field scan and lyric tokenizer over a CSV in HBM.
//
// Replaces the byte-serial reader of the reference (read_csv_record,
// parallel_spotify.c:549-633; parse_csv_line 258-304; process_lyrics 350-394)
// with a three-kernel data-parallel scan:
//
//   K1 k_chunk_summary  one wave per 16 KiB chunk: the chunk's transfer
//                       function over the reader state, for BOTH possible
//                       incoming quote parities (wave-ballot prefix-xor)
//   K2 k_fn_reduce /    scan the chunk functions (associative composition)
//      k_fn_top /       and apply the initial state -> exact reader state at
//      k_fn_down        every chunk
//   K3 k_scan_main      one wave per chunk again, now knowing its state:
//                       record terminators, the first three unquoted commas
//                       of every record, NUL truncation, and -- for the
//                       lyric field -- token starts, lengths, lower-cased
//                       keys, counted in an LDS-private table (Zipf head)
//                       with device-scope atomics only on overflow.
//
// Every wave moves 1 KiB per iteration as one coalesced dwordx4 per lane; all
// cross-lane work is ballot/mbcnt based (64-wide wavefronts).
#include "msa_internal.h"
#include "msa_k1.h"
#include "msa_tables.h"

namespace {

__device__ __forceinline__ uint4 ld16(const u8 *p) { return *reinterpret_cast<const uint4 *>(p); }

__device__ __forceinline__ u32 valid_mask(u64 lpos, u64 end) {
    if (lpos >= end) return 0;
    u64 r = end - lpos;
    return r >= 16 ? 0xFFFFu : ((1u << r) - 1u);
}

__device__ __forceinline__ u32 range_mask(u32 from, u32 to) {  // bits [from, to)
    return ((0xFFFFu << from) & (0xFFFFu >> (16 - to))) & 0xFFFFu;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

// ---------------------------------------------------------------------------
// K1: per-chunk transfer function, both parity hypotheses.  A hypothesis
// needs only wave totals and the values at the last lane holding a
// terminator: the terminator count from ballot bit-planes, the commas after
// the last terminator as saturating ballot counts (min(popc, 3) per lane; the
// state saturates at 3), the rest by readlane at that lane (scalar work).
// Input is loaded two iterations ahead (the buffers are padded).
// 64 bytes per lane per iteration (4 KiB per wave, u64 masks per lane): the
// cross-lane ballot work is per iteration, so more bytes per lane make it
// cheaper per byte.
#define K1_ITER 4096
struct Classes64 {
    u64 Q, C, NL, CR, Z;
    bool rare;  // the wave's 4 KiB hold a '\r' or NUL (CR / Z computed)
};
// "byte == c" per byte as 0x80 flags (exact) / "some byte == c" (cheap)
__device__ __forceinline__ u32 k1_eq80(u32 x, u32 c) {
    const u32 y = x ^ (c * 0x01010101u);
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
}
__device__ __forceinline__ u32 k1_has80(u32 x, u32 c) {
    const u32 y = x ^ (c * 0x01010101u);
    return (y - 0x01010101u) & ~y & 0x80808080u;
}
// The lane's 64 bytes: '"', ',' and '\n' always; '\r' and NUL only when the
// wave's 4 KiB hold one (a cheap has-byte test, then a wave-uniform branch).
__device__ __forceinline__ Classes64 classify64(const uint4 (&v)[4], u64 lpos, u64 end) {
    Classes64 k{0, 0, 0, 0, 0, false};
    u32 rare = 0;
    u32 q0 = 0, q1 = 0, c0 = 0, c1 = 0, n0 = 0, n1 = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const u32 w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
        for (int d = 0; d < 4; ++d) rare |= k1_has80(w[d], '\r') | k1_has80(w[d], 0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // dword pairs: byte 2q + h of each mask
            const int kb = 2 * q + h;
            const u32 a = w[2 * h], b = w[2 * h + 1];
            const u32 a7 = a & 0x7F7F7F7Fu, b7 = b & 0x7F7F7F7Fu;
            swar_put8(q0, q1, kb, swar_pack8x128(eq80x(a, a7, '"'), eq80x(b, b7, '"')));
            swar_put8(c0, c1, kb, swar_pack8x128(eq80x(a, a7, ','), eq80x(b, b7, ',')));
            swar_put8(n0, n1, kb, swar_pack8x128(eq80x(a, a7, '\n'), eq80x(b, b7, '\n')));
        }
    }
    k.Q = mk64(q0, q1); k.C = mk64(c0, c1); k.NL = mk64(n0, n1);
    if (__ballot(rare != 0)) {
        u32 r0 = 0, r1 = 0, z0 = 0, z1 = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32 w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int kb = 2 * q + h;
                swar_put8(r0, r1, kb, swar_pack8x128(k1_eq80(w[2 * h], '\r'), k1_eq80(w[2 * h + 1], '\r')));
                swar_put8(z0, z1, kb, swar_pack8x128(k1_eq80(w[2 * h], 0), k1_eq80(w[2 * h + 1], 0)));
            }
        }
        k.CR = mk64(r0, r1);
        k.Z = mk64(z0, z1);
        k.rare = true;
    }
    const u64 r = lpos < end ? end - lpos : 0;
    const u64 vm = r >= 64 ? ~0ull : ((1ull << r) - 1ull);
    k.Q &= vm; k.C &= vm; k.NL &= vm; k.CR &= vm; k.Z &= vm;
    return k;
}
#ifndef K1_LDS
#define K1_LDS 0  // 1: blocks loaded coalesced (lane l: bytes 1024 q + 16 l) and transposed through LDS
#endif
#ifndef K1_MINW
#define K1_MINW 5  // min waves per SIMD: 96 VGPRs, 5 waves (4 at 111 VGPRs: 0.362 -> 0.338 ms; 6 and 8 spill: 0.43, 0.89)
#endif
__global__ __launch_bounds__(256, K1_MINW) void k_chunk_summary(const u8 *__restrict__ buf, u64 seg_begin,
                                                       u64 seg_end, u32 nchunks,
                                                       ChunkSum *__restrict__ out) {
    const u32 lane = lane_id();
    const u32 gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const u32 nw = (gridDim.x * blockDim.x) >> 6;
    // the byte after a block (raw '\n' there: the '\r\n' swallow at lane 63),
    // loaded with the block, an iteration ahead and BEFORE that block's data:
    // vector loads complete in order, so a byte load issued after the next
    // block's prefetch made every iteration wait for that prefetch
    auto nbyte = [&](u64 pos) -> u32 { return pos < seg_end ? (u32)buf[pos] : 0u; };
#if K1_LDS
    __shared__ uint4 k1st[256 / 64][256];
    uint4 *st = k1st[threadIdx.x >> 6];
    Blk4 raw{};  // the next block as loaded (coalesced), in flight during the current one
    u32 nb_cur = 0;
    if (gw < nchunks) {
        const u64 b0 = seg_begin + (u64)gw * MSA_CHUNK;
        nb_cur = nbyte(b0 + K1_ITER);
        raw = blk_load_co(buf + b0);
    }
    for (u32 c = gw; c < nchunks; c += nw) {
        const u64 cbase = seg_begin + (u64)c * MSA_CHUNK;
        const u64 cend = min(cbase + (u64)MSA_CHUNK, seg_end);
        K1Acc acc;
        k1_init(acc);
        for (u64 ibase = cbase; ibase < cend; ibase += K1_ITER) {
            const u64 lpos = ibase + lane * 64;
            uint4 cur[4];
            blk_transpose(st, raw, cur);
            u32 nb_next = 0;
            if (ibase + K1_ITER < cend) {
                nb_next = nbyte(ibase + 2 * K1_ITER);
                raw = blk_load_co(buf + ibase + K1_ITER);
            } else if (c + nw < nchunks) {
                const u64 b1 = seg_begin + (u64)(c + nw) * MSA_CHUNK;
                nb_next = nbyte(b1 + K1_ITER);
                raw = blk_load_co(buf + b1);
            }
            const Classes64 k = classify64(cur, lpos, cend);
            const u32 nb_nl = nb_cur == '\n' ? 1u : 0u;
            const u32 lastb = (u32)(min(ibase + (u64)K1_ITER, cend) - 1 - ibase);
            k1_block(acc, k.Q, k.C, k.NL, k.CR, k.Z, k.rare, nb_nl, (u32)(ibase - cbase), lastb);
            nb_cur = nb_next;
        }
        const ChunkSum sum = k1_finish(acc);
        if (lane == 0) out[c] = sum;
    }
#else
    uint4 cur[4];  // a chunk's first block: loaded during the previous chunk's last one
    u32 nb_cur = 0;
    if (gw < nchunks) {
        const u64 b0 = seg_begin + (u64)gw * MSA_CHUNK;
        nb_cur = nbyte(b0 + K1_ITER);
#pragma unroll
        for (int q = 0; q < 4; ++q) cur[q] = ld16(buf + b0 + lane * 64 + 16 * q);
    }
    for (u32 c = gw; c < nchunks; c += nw) {
        const u64 cbase = seg_begin + (u64)c * MSA_CHUNK;
        const u64 cend = min(cbase + (u64)MSA_CHUNK, seg_end);
        K1Acc acc;
        k1_init(acc);
        for (u64 ibase = cbase; ibase < cend; ibase += K1_ITER) {
            const u64 lpos = ibase + lane * 64;
            // one iteration ahead: the chunk's next block, else the wave's next
            // chunk (reads end < cend + 4096, MSA_INPUT_PAD); its following byte first
            uint4 nxt[4] = {cur[0], cur[1], cur[2], cur[3]};
            u32 nb_next = 0;
            if (ibase + K1_ITER < cend) {
                nb_next = nbyte(ibase + 2 * K1_ITER);
#pragma unroll
                for (int q = 0; q < 4; ++q) nxt[q] = ld16(buf + lpos + K1_ITER + 16 * q);
            } else if (c + nw < nchunks) {
                const u64 b1 = seg_begin + (u64)(c + nw) * MSA_CHUNK;
                nb_next = nbyte(b1 + K1_ITER);
#pragma unroll
                for (int q = 0; q < 4; ++q) nxt[q] = ld16(buf + b1 + lane * 64 + 16 * q);
            }
            const Classes64 k = classify64(cur, lpos, cend);
            const u32 nb_nl = nb_cur == '\n' ? 1u : 0u;
            const u32 lastb = (u32)(min(ibase + (u64)K1_ITER, cend) - 1 - ibase);
            k1_block(acc, k.Q, k.C, k.NL, k.CR, k.Z, k.rare, nb_nl, (u32)(ibase - cbase), lastb);
#pragma unroll
            for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
            nb_cur = nb_next;
        }
        const ChunkSum sum = k1_finish(acc);
        if (lane == 0) out[c] = sum;
    }
#endif
}

// ---------------------------------------------------------------------------
// K2: exact reader state at every chunk start = the initial state pushed
// through the composition of all earlier chunk functions (an exclusive scan
// over the associative "f then g" monoid), in three launches:
//   k_fn_reduce  one block per 256 chunks: tree-compose -> block total
//   k_fn_top     one block: runs of block totals -> each block's start state
//   k_fn_down    one block per 256 chunks: Hillis-Steele scan in LDS, apply
#define FN_T 256

__device__ __forceinline__ Fn chunk_fn(const ChunkSum *__restrict__ sums, u64 seg_begin, u32 nchunks, u32 c) {
    const u64 base = seg_begin + (u64)c * MSA_CHUNK;
    if (c >= nchunks) return fn_identity(base);
    const ChunkSum cs = sums[c];
    Fn g;
    g.e[0] = chunk_entry(cs, base, 0);
    g.e[1] = chunk_entry(cs, base, 1);
    g.e[2] = chunk_entry(cs, base, 2);
    return g;
}

__global__ __launch_bounds__(FN_T) void k_fn_reduce(const ChunkSum *__restrict__ sums, u64 seg_begin, u32 nchunks,
                                                    Fn *__restrict__ btot) {
    __shared__ Fn sh[FN_T];
    const u32 t = threadIdx.x;
    sh[t] = chunk_fn(sums, seg_begin, nchunks, blockIdx.x * FN_T + t);
    __syncthreads();
    for (u32 w = 1; w < FN_T; w <<= 1) {
        if ((t & (2 * w - 1)) == 0) sh[t] = fn_compose(sh[t], sh[t + w]);
        __syncthreads();
    }
    if (t == 0) btot[blockIdx.x] = sh[0];
}

__global__ __launch_bounds__(FN_T) void k_fn_top(const Fn *__restrict__ btot, u32 nb, u64 seg_begin,
                                                 const State init, State *__restrict__ bstate,
                                                 Fn *__restrict__ total) {
    // tiles of FN_T block totals: an inclusive scan in LDS per tile (as
    // k_fn_down), the state carried from tile to tile -- one element per
    // thread, no per-thread serial composition (that one lived in scratch)
    __shared__ Fn sh[2][FN_T];
    __shared__ State carry_s;
    __shared__ Fn tot_s;
    const u32 t = threadIdx.x;
    if (t == 0) {
        carry_s = init;
        tot_s = fn_identity(seg_begin);
    }
    for (u32 base = 0; base < nb; base += FN_T) {
        const u32 i = base + t;
        sh[0][t] = i < nb ? btot[i] : fn_identity(seg_begin);
        __syncthreads();
        u32 cur = 0;
        for (u32 off = 1; off < FN_T; off <<= 1) {  // inclusive scan, ping-pong buffers
            const u32 src = (t >= off) ? t - off : t;
            Fn g = fn_compose(sh[cur][src], sh[cur][t]);
            if (t < off) g = sh[cur][t];
            sh[cur ^ 1][t] = g;
            cur ^= 1;
            __syncthreads();
        }
        const State s0 = carry_s;
        State s = s0;
        if (t > 0) s = fn_apply(s0, sh[cur][t - 1]);
        if (i < nb) bstate[i] = s;
        __syncthreads();  // every thread has read carry_s
        if (t == FN_T - 1) {
            carry_s = fn_apply(s0, sh[cur][t]);
            if (total) tot_s = fn_compose(tot_s, sh[cur][t]);
        }
        __syncthreads();
    }
    if (t == 0 && total) *total = tot_s;
}

__global__ __launch_bounds__(FN_T) void k_fn_down(const ChunkSum *__restrict__ sums, u64 seg_begin, u32 nchunks,
                                                  const State *__restrict__ bstate, State *__restrict__ carry,
                                                  State *__restrict__ final_state) {
    __shared__ Fn sh[2][FN_T];
    const u32 t = threadIdx.x;
    const u32 c = blockIdx.x * FN_T + t;
    sh[0][t] = chunk_fn(sums, seg_begin, nchunks, c);
    __syncthreads();
    u32 cur = 0;
    for (u32 off = 1; off < FN_T; off <<= 1) {  // inclusive scan, ping-pong buffers
        const u32 src = (t >= off) ? t - off : t;
        Fn g = fn_compose(sh[cur][src], sh[cur][t]);
        if (t < off) g = sh[cur][t];
        sh[cur ^ 1][t] = g;
        cur ^= 1;
        __syncthreads();
    }
    State s = bstate[blockIdx.x];
    if (t > 0) s = fn_apply(s, sh[cur][t - 1]);
    if (c < nchunks) carry[c] = s;
    if (c + 1 == nchunks) *final_state = fn_apply(bstate[blockIdx.x], sh[cur][t]);
}

// ---------------------------------------------------------------------------
// K3: the main pass.  Default: one 1024-thread workgroup per CU (16 waves)
// sharing one LDS count table -- the larger the table, the fewer Zipf-tail
// words miss it.
#ifndef K3_THREADS
#define K3_THREADS 1024
#endif
#define K3_WAVES (K3_THREADS / 64)
#ifndef LSLOTS
#define LSLOTS 4096
#endif
#ifndef MSLOTS
#define MSLOTS 1024
#endif
#ifndef K3_BLOCKS_PER_CU
#define K3_BLOCKS_PER_CU 1
#endif
// Per-wave LDS: a 2 KiB ring (this and the next 1 KiB of input), 1 KiB of
// token entries in three lists -- S words (3..8 bytes) at [0, 256), M words
// (9..16) at [256, 384), long words at [384, 512) -- and the deferred-miss
// buffer: keys that miss the LDS tables are inserted into HBM in batches of
// > K3_MISS_CAP - 64, so a wave waits on HBM once per batch, not once per
// token pass.
#define K3_MISS_CAP 128
#define ST_M 256
#define ST_L 384
#define WAVE_LDS (2048 + 1024 + K3_MISS_CAP * 16)
#define TAB_LDS (LSLOTS * 12 + MSLOTS * 20 + (K3_DOORKEEPER ? DK_WORDS * 4 : 0))
#define K3_LDS (TAB_LDS + K3_WAVES * WAVE_LDS)

// LDS count tables are bucketised: 4 keys per 32-byte bucket, read with two
// 16-byte LDS loads, so a lookup costs one round trip whether it hits or
// misses (a linear probe chain made the whole wave wait for its slowest lane).
// A key lives in its bucket or the next; a miss in both goes to HBM.
#define LB 4
#ifndef K3_DOORKEEPER
#define K3_DOORKEEPER 0
#endif
#define DK_WORDS 2048  // doorkeeper bitset: 64 Ki bits of LDS
static_assert(K3_LDS * K3_BLOCKS_PER_CU <= 160 * 1024, "K3 LDS exceeds the CU's 160 KiB");
static_assert(TAB_LDS % 16 == 0 && WAVE_LDS % 16 == 0, "K3 LDS carve-outs must stay 16-byte aligned");
// Admission filter: a key claims an LDS slot only on its second sighting in
// this workgroup, so words seen once (the Zipf tail) do not fill the table.
__device__ __forceinline__ bool dk_admit(u32 *dk, u64 h) {
    if (!K3_DOORKEEPER) return true;
    const u32 bit = (u32)(h >> 17) & (DK_WORDS * 32 - 1);
    const u32 m = 1u << (bit & 31);
    return (atomicOr(&dk[bit >> 5], m) & m) != 0;
}
__device__ __forceinline__ u32 lds_find_s(u64 *lkey, u32 *dk, u64 key) {
    const u32 nb = LSLOTS / LB;
    u32 b = lds_hash(key) & (nb - 1);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const u32 base = b * LB;
        const ulonglong2 q0 = *reinterpret_cast<const ulonglong2 *>(&lkey[base]);
        const ulonglong2 q1 = *reinterpret_cast<const ulonglong2 *>(&lkey[base + 2]);
        const u64 kk[4] = {q0.x, q0.y, q1.x, q1.y};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (kk[i] == key) return base + i;
        if (p == 0 && (kk[0] == 0 || kk[1] == 0 || kk[2] == 0 || kk[3] == 0) && !dk_admit(dk, key * 0x9E3779B97F4A7C15ULL))
            return ~0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (kk[i] == 0) {
                const u64 old = atomicCAS((unsigned long long *)&lkey[base + i], 0ull, (unsigned long long)key);
                if (old == 0 || old == key) return base + i;
            }
        }
        b = (b + 1) & (nb - 1);
    }
    return ~0u;
}

// 9..16-byte keys (k0, k1): claimed by CAS on k0, k1 published after the
// claim; a prober that finds k0 but not (yet) k1 moves on -- a key may then
// own two slots, and both flush into the same HBM entry.
__device__ __forceinline__ u32 lds_find_m(u64 *mk0, u64 *mk1, u32 *dk, u64 x0, u64 x1) {
    const u32 nb = MSLOTS / LB;
    u32 b = lds_hash(x0 ^ (x1 * 0xC2B2AE3D27D4EB4FULL)) & (nb - 1);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const u32 base = b * LB;
        const ulonglong2 q0 = *reinterpret_cast<const ulonglong2 *>(&mk0[base]);
        const ulonglong2 q1 = *reinterpret_cast<const ulonglong2 *>(&mk0[base + 2]);
        const u64 kk[4] = {q0.x, q0.y, q1.x, q1.y};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (kk[i] == x0 && mk1[base + i] == x1) return base + i;
        if (p == 0 && (kk[0] == 0 || kk[1] == 0 || kk[2] == 0 || kk[3] == 0) &&
            !dk_admit(dk, (x0 ^ (x1 * 0xC2B2AE3D27D4EB4FULL)) * 0x9E3779B97F4A7C15ULL))
            return ~0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (kk[i] == 0) {
                const u64 old = atomicCAS((unsigned long long *)&mk0[base + i], 0ull, (unsigned long long)x0);
                if (old == 0) {
                    mk1[base + i] = x1;
                    return base + i;
                }
            }
        }
        b = (b + 1) & (nb - 1);
    }
    return ~0u;
}

// Deferred HBM inserts of LDS-table misses (k1 == 0: an S word).
__device__ __forceinline__ void flush_misses(const ScanArgs &a, const ulonglong2 *miss, u32 n) {
    wave_sync();
    for (u32 t = lane_id(); t < n; t += 64) {
        const ulonglong2 x = miss[t];
        if (x.y == 0) s_insert<false>(a.s_tab, a.s_mask, x.x, 1, a.s_list, a.s_list_cap, a.ctr);
        else m_insert<false>(a.m_tab, a.m_mask, x.x, x.y, 1, a.m_list, a.m_list_cap, a.ctr);
    }
    wave_sync();
}
// Called by every lane of the wave; appends the keys of the lanes with `m`.
__device__ __forceinline__ void push_miss(ulonglong2 *miss, u32 &nmiss, bool m, u64 x0, u64 x1) {
    const u64 B = __ballot(m);
    if (m) miss[nmiss + mbcnt(B)] = make_ulonglong2(x0, x1);
    nmiss += (u32)__popcll(B);
}

// MODE 0 = CSV (records, fields, lyric tokens), 1 = LINES (records only),
//      2 = FLAT (every byte is lyric text: tokens only, no record structure)
template <int MODE>
__global__ __launch_bounds__(K3_THREADS) void k_scan_main(ScanArgs a) {
    constexpr bool TOK = MODE != 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64 *lkey = reinterpret_cast<u64 *>(smem);
    u32 *lcnt = reinterpret_cast<u32 *>(smem + LSLOTS * 8);
    // M words (9..16 bytes): key (k0, k1), claimed by CAS on k0; k1 is published
    // after the claim, and a prober that finds k0 but not yet k1 moves on (a
    // key may then own two slots -- both flush into the same HBM entry).
    u64 *mk0 = reinterpret_cast<u64 *>(smem + LSLOTS * 12);
    u64 *mk1 = mk0 + MSLOTS;
    u32 *mcnt = reinterpret_cast<u32 *>(mk1 + MSLOTS);
    u32 *dk = mcnt + MSLOTS;  // doorkeeper bitset (K3_DOORKEEPER)
    const u32 lane = lane_id();
    const u32 wib = threadIdx.x >> 6;
    unsigned char *wl = smem + TAB_LDS + wib * WAVE_LDS;
    u64 *ring = reinterpret_cast<u64 *>(wl);             // 2 KiB: two 1 KiB iteration slots
    u16 *starts = reinterpret_cast<u16 *>(wl + 2048);    // token entries: pos | len << 10
    ulonglong2 *miss = reinterpret_cast<ulonglong2 *>(wl + 3072);
    u32 nmiss = 0;  // wave-uniform
    const u64 lt = (1ull << lane) - 1ull;

    if (TOK) {
        for (u32 i = threadIdx.x; i < LSLOTS; i += K3_THREADS) { lkey[i] = 0; lcnt[i] = 0; }
        for (u32 i = threadIdx.x; i < MSLOTS; i += K3_THREADS) { mk0[i] = 0; mk1[i] = 0; mcnt[i] = 0; }
        if (K3_DOORKEEPER)
            for (u32 i = threadIdx.x; i < DK_WORDS; i += K3_THREADS) dk[i] = 0;
        __syncthreads();
    }
    const u32 gw = blockIdx.x * K3_WAVES + wib;
    const u32 nw = gridDim.x * K3_WAVES;
    u64 words = 0;

    for (u32 c = gw; c < a.nchunks; c += nw) {
        State st = a.carry[c];
        const u64 cbase = a.seg_begin + (u64)c * MSA_CHUNK;
        const u64 cend = min(cbase + (u64)MSA_CHUNK, a.seg_end);
        u32 prevT = 0;
        if (TOK && cbase > 0) {
            const u32 b = a.buf[cbase - 1];
            prevT = (u32)(((b | 0x20u) >= 'a' && (b | 0x20u) <= 'z') || (b >= '0' && b <= '9') || b == '\'');
        }
        uint4 cur = ld16(a.buf + cbase + lane * 16);
        uint4 nxt = ld16(a.buf + cbase + MSA_ITER + lane * 16);
        if (TOK) {
            reinterpret_cast<uint4 *>(ring)[lane] = cur;
        }
        u32 it = 0;
        for (u64 ibase = cbase; ibase < cend; ibase += MSA_ITER, ++it) {
            const u64 lpos = ibase + lane * 16;
            const u64 npos = ibase + MSA_ITER;
            u32 tnext = 0;  // token mask of the following 1 KiB (token continuation)
            uint4 nn = ld16(a.buf + npos + MSA_ITER + lane * 16);  // prefetch it+2
            if (TOK) {
                // stage the following 1 KiB (token continuation only) in the other ring slot
                const u32 slot = (it + 1) & 1u;
                reinterpret_cast<uint4 *>(ring)[slot * 64 + lane] = nxt;
                tnext = tok16(nxt, valid_mask(npos + lane * 16, a.seg_end));
            }
            const u32 vmask = valid_mask(lpos, cend);
            const Classes k = classify16(cur, vmask);
            const u32 lastb = (u32)(min(ibase + (u64)MSA_ITER, cend) - 1 - ibase);
            const int Lz = (int)(lastb >> 4);
            const u32 bz = lastb & 15u;
            u32 live = (MODE == 2) ? 0xFFFFu : 0u;  // lyric bytes of this lane
            if (MODE != 2) {
            const u64 B = __ballot(__popc(k.Q) & 1u);
            const u32 pin = st.p ^ (mbcnt(B) & 1u);
            const u32 inq = pxor_excl16(k.Q) ^ (pin ? 0xFFFFu : 0u);
            const u32 CRu = k.CR & ~inq, NLu = k.NL & ~inq;
            const u32 Cu = (MODE == 0) ? (k.C & ~inq) : 0u;
            const u32 Zm = (MODE == 0) ? k.Z : 0u;
            const u32 upCR = __shfl_up(CRu, 1);
            const u32 pc0 = lane ? ((upCR >> 15) & 1u) : st.cr;
            const u32 TERM = (CRu | (NLu & ~((CRu << 1) | pc0))) & 0xFFFFu;
            const u32 nb_nl = (npos < a.seg_end) ? ((readlane(nxt.x, 0) & 0xFFu) == '\n') : 0u;
            const u32 dn = __shfl_down(k.NL, 1);
            const u32 nlnext = (k.NL >> 1) | (((lane == 63) ? nb_nl : (dn & 1u)) << 15);
            const u32 SW = CRu & nlnext;
            // segmented (per-record) state at this lane's first byte
            const u32 nt = __popc(TERM);
            const u32 lastT = nt ? 31u - __clz(TERM) : 0u;
            const u32 above = nt ? ((0xFFFFu << (lastT + 1)) & 0xFFFFu) : 0xFFFFu;
            const u32 cC = __popc(Cu);
            const u32 tailC = __popc(Cu & above);
            const u32 tailZ = (Zm & above) != 0;
            const u64 endpos = lpos + lastT + 1 + ((SW >> lastT) & 1u);
            u32 totC, totT;
            const u32 PC = wave_prefix<5>(cC, totC);
            const u32 PT = wave_prefix<5>(nt, totT);
            const u64 Bh = __ballot(nt != 0);
            const u64 Bz = __ballot(Zm != 0);
            const u64 J = Bh & lt;
            const int j = J ? (63 - __clzll(J)) : (int)lane;
            const u32 pk = tailC | (tailZ << 5) | ((PC + cC) << 6);
            const u32 gpk = __shfl(pk, j);
            const u64 gend = __shfl(endpos, j);
            u32 cin, zin;
            u64 rs;
            if (J) {
                cin = (gpk & 31u) + (PC - (gpk >> 6));
                const u64 between = lt & ~((2ull << j) - 1ull);
                zin = ((gpk >> 5) & 1u) | ((Bz & between) != 0);
                rs = gend;
            } else {
                cin = st.c + PC;
                zin = st.z | ((Bz & lt) != 0);
                rs = st.rs;
            }
            u32 cs = cin > 3 ? 3 : cin, zs = zin;
            u64 rr = st.rec + PT;
            // walk this lane's events (terminators, unquoted commas, NULs)
            u32 E = TERM | Cu | Zm;
            u32 from = 0;
            if (a.ablate & 8) E = TERM;  // ablation: skip field events
            while (E) {
                const u32 b = __ffs(E) - 1;
                E &= E - 1;
                if (MODE == 0 && rr >= a.first_rec && cs >= 3 && !zs) live |= range_mask(from, b);
                const u64 bpos = lpos + b;
                if ((TERM >> b) & 1u) {
                    const u64 ns = bpos + 1 + ((SW >> b) & 1u);
                    ++rr;
                    if (rr < a.rec_cap) a.rec_start[rr] = ns;
                    cs = 0;
                    zs = 0;
                    rs = ns;
                } else if ((Zm >> b) & 1u) {
                    if (!zs) {
                        zs = 1;
                        if (a.want_nul && rr < a.rec_cap) a.nulrel[rr] = (u32)(bpos - rs) + 1u;
                    }
                } else if (cs < 3) {
                    ++cs;  // the field offsets themselves are found later (k_rec_fields)
                }
                from = b + 1;
            }
            if (MODE == 0 && rr >= a.first_rec && cs >= 3 && !zs) live |= range_mask(from, 16);

            // carry to the next iteration (lane 63 has seen every byte)
            st.p ^= (u32)__popcll(B) & 1u;
            st.cr = (readlane(CRu, Lz) >> bz) & 1u;
            st.c = readlane(cs, 63);
            st.z = readlane(zs, 63);
            st.rec = readlane64(rr, 63);
            st.rs = readlane64(rs, 63);
            }

            if (TOK && !(a.ablate & 1)) {
                // ---- tokens of the lyric field (process_lyrics, parallel_spotify.c:350-394)
                // token starts S and each start's length class from run masks of this
                // lane's and the next lane's token bits: r_k bit b = bytes b..b+k-1 are
                // token bytes (b + 16 <= 31 for every start of this lane).  Tokens of
                // fewer than 3 bytes are not counted and never leave the producer.
                const u32 upT = __shfl_up(k.T, 1);
                const u32 pt0 = lane ? ((upT >> 15) & 1u) : prevT;
                const u32 S = (k.T & live) & ~((k.T << 1) | pt0) & 0xFFFFu;
                prevT = (readlane(k.T, Lz) >> bz) & 1u;
                const u32 n0 = readlane(tnext, 0);
                const u32 d1 = __shfl_down(k.T, 1);
                const u32 w = k.T | ((lane == 63 ? n0 : d1) << 16);
                const u32 r2 = w & (w >> 1), r3 = r2 & (w >> 2), r4 = r2 & (r2 >> 2);
                const u32 r8 = r4 & (r4 >> 4), r9 = r8 & (w >> 8), r16 = r8 & (r8 >> 8), r17 = r16 & (w >> 16);
                const u32 sS = S & r3 & ~r9, sM = S & r9 & ~r17, sL = S & r17;
                const u32 cS = __popc(sS), cM = __popc(sM), cL = __popc(sL);  // <= 4, 2, 1 per lane
                words += cS + cM + cL;
                u32 tS, tM, tL;
                u32 iS = wave_prefix<3>(cS, tS);
                u32 iM = ST_M + wave_prefix<2>(cM, tM);
                u32 iL = ST_L + wave_prefix<1>(cL, tL);
                for (u32 sm = sS | sM | sL; sm; sm &= sm - 1) {
                    const u32 b = __ffs(sm) - 1;
                    const u32 len = min((u32)__ffs(~(w >> b)) - 1u, 31u);  // exact up to 16
                    const u16 e = (u16)((lane * 16 + b) | (len << 10));
                    if ((sL >> b) & 1u) starts[iL++] = e;
                    else if ((sM >> b) & 1u) starts[iM++] = e;
                    else starts[iS++] = e;
                }
                wave_sync();
                const u32 slot_off = (it & 1u) << 10;
                // S words: dense passes over the wave's list (every lane stays in the
                // loop: nmiss is wave-uniform)
                for (u32 t0 = 0; t0 < tS && !(a.ablate & 2); t0 += 64) {
                    const u32 t = t0 + lane;
                    bool m = false;
                    u64 key = 0;
                    if (t < tS && !(a.ablate & 32)) {
                        const u32 ent = starts[t];
                        const u32 len = ent >> 10;
                        const u32 o = slot_off + (ent & 1023u);
                        const u32 q = o >> 3, sh = (o & 7u) * 8u;
                        const u64 w0 = ring[q], w1 = ring[(q + 1) & 255u];
                        u64 k0 = sh ? ((w0 >> sh) | (w1 << (64 - sh))) : w0;
                        if (len < 8) k0 &= (1ull << (8 * len)) - 1ull;
                        key = lower8(k0);
                        const u32 slot = lds_find_s(lkey, dk, key);
                        if (slot != ~0u) atomicAdd(&lcnt[slot], 1u);
                        else m = !(a.ablate & 4);
                    }
                    push_miss(miss, nmiss, m, key, 0ull);
                    if (nmiss > K3_MISS_CAP - 64) {
                        flush_misses(a, miss, nmiss);
                        nmiss = 0;
                    }
                }
                // M words (9..16 bytes)
                for (u32 t0 = 0; t0 < tM && !(a.ablate & 2); t0 += 64) {
                    const u32 t = t0 + lane;
                    bool m = false;
                    u64 x0 = 0, x1 = 0;
                    if (t < tM && !(a.ablate & 16)) {
                        const u32 ent = starts[ST_M + t];
                        const u32 len = ent >> 10;
                        const u32 o = slot_off + (ent & 1023u);
                        const u32 q = o >> 3, sh = (o & 7u) * 8u;
                        const u64 w0 = ring[q], w1 = ring[(q + 1) & 255u], w2 = ring[(q + 2) & 255u];
                        const u64 k0 = sh ? ((w0 >> sh) | (w1 << (64 - sh))) : w0;
                        u64 k1 = sh ? ((w1 >> sh) | (w2 << (64 - sh))) : w1;
                        if (len < 16) k1 &= (1ull << (8 * (len - 8))) - 1ull;
                        x0 = lower8(k0);
                        x1 = lower8(k1);
                        const u32 slot = lds_find_m(mk0, mk1, dk, x0, x1);
                        if (slot != ~0u) atomicAdd(&mcnt[slot], 1u);
                        else m = true;
                    }
                    push_miss(miss, nmiss, m, x0, x1);
                    if (nmiss > K3_MISS_CAP - 64) {
                        flush_misses(a, miss, nmiss);
                        nmiss = 0;
                    }
                }
                // long words (> 16 bytes; <= 57 per KiB): positions for k_long_insert,
                // one occurrence-counter bump per wave
                if (tL && !(a.ablate & 2)) {
                    u64 base = 0;
                    if (lane == 0) base = atomicAdd((unsigned long long *)&a.ctr->l_occ, (unsigned long long)tL);
                    base = readlane64(base, 0);
                    if (lane < tL) {
                        const u64 i = base + lane;
                        const u32 ent = starts[ST_L + lane];
                        if (i < a.l_cap) a.l_pos[i] = (ibase + (ent & 1023u)) | a.lpos_tag;
                        else atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_L);
                    }
                }
                wave_sync();
            }
            cur = nxt;
            nxt = nn;
        }
    }
    if (TOK) {
        if (nmiss) flush_misses(a, miss, nmiss);
        words = wave_sum64(words);
        if (lane == 0 && words) atomicAdd((unsigned long long *)&a.ctr->total_words, (unsigned long long)words);
        __syncthreads();
        for (u32 i = threadIdx.x; i < LSLOTS; i += K3_THREADS) {
            const u32 n = lcnt[i];
            if (n) s_insert<false>(a.s_tab, a.s_mask, lkey[i], n, a.s_list, a.s_list_cap, a.ctr);
        }
        for (u32 i = threadIdx.x; i < MSLOTS; i += K3_THREADS) {
            const u32 n = mcnt[i];
            if (n) m_insert<false>(a.m_tab, a.m_mask, mk0[i], mk1[i], n, a.m_list, a.m_list_cap, a.ctr);
        }
    }
}

// ---------------------------------------------------------------------------
// First record end in a shard (multi-GPU boundary resolution): one wave walks
// the shard from its first byte with the reader state (p, cr) it inherits from
// the shards before it, and stops at the first unquoted terminator (a '\r'
// swallows one '\n', as in read_csv_record, parallel_spotify.c:609-627).
// Writes the offset just past that record, or n if the shard has none.
__global__ __launch_bounds__(64) void k_first_end(const u8 *__restrict__ buf, u64 n, u32 p0, u32 cr0,
                                                  u64 *__restrict__ out) {
    const u32 lane = lane_id();
    u32 p = p0, cr = cr0;
    for (u64 ibase = 0; ibase < n; ibase += MSA_ITER) {
        const u64 lpos = ibase + lane * 16;
        const uint4 v = ld16(buf + lpos);
        const Classes k = classify16(v, valid_mask(lpos, n));
        const u64 B = __ballot(__popc(k.Q) & 1u);
        const u32 pin = p ^ (mbcnt(B) & 1u);
        const u32 inq = pxor_excl16(k.Q) ^ (pin ? 0xFFFFu : 0u);
        const u32 CRu = k.CR & ~inq, NLu = k.NL & ~inq;
        const u32 upCR = __shfl_up(CRu, 1);
        const u32 pc0 = lane ? ((upCR >> 15) & 1u) : cr;
        const u32 TERM = (CRu | (NLu & ~((CRu << 1) | pc0))) & 0xFFFFu;
        const u64 Bt = __ballot(TERM != 0);
        if (Bt) {
            const int jl = __ffsll((long long)Bt) - 1;
            const u32 tm = readlane(TERM, jl);
            const u64 pos = ibase + (u64)jl * 16 + (u64)(__ffs(tm) - 1);
            if (lane == 0) {
                u64 end = pos + 1;
                if (buf[pos] == '\r' && end < n && buf[end] == '\n') ++end;
                *out = end;
            }
            return;
        }
        p ^= (u32)__popcll(B) & 1u;
        const u32 lastb = (u32)(min(ibase + (u64)MSA_ITER, n) - 1 - ibase);
        cr = (readlane(CRu, (int)(lastb >> 4)) >> (lastb & 15u)) & 1u;
    }
    if (lane == 0) *out = n;
}

// Quote parity of a byte range (the boundary resolution of the multi-GPU
// path needs only the reader state at each shard's end: the parity of its
// '"' bytes and its last byte, see msa_shard_function).  A streaming read,
// 16 bytes per lane per step; the unaligned head and tail by byte; one
// atomic XOR per wave.
__global__ __launch_bounds__(256) void k_quote_parity(const u8 *__restrict__ buf, u64 n, u32 *__restrict__ out) {
    const u64 a0 = (16 - ((size_t)buf & 15)) & 15;  // bytes before the first 16-byte boundary
    const u64 head = a0 < n ? a0 : n;
    const u64 nv = (n - head) / 16;
    const uint4 *v = reinterpret_cast<const uint4 *>(buf + head);
    const u64 tid = (u64)blockIdx.x * blockDim.x + threadIdx.x, nt = (u64)gridDim.x * blockDim.x;
    u32 par = 0;
    for (u64 i = tid; i < nv; i += nt) {
        const uint4 x = v[i];
        par ^= __popc(k1_eq80(x.x, '"') ^ k1_eq80(x.y, '"') ^ k1_eq80(x.z, '"') ^ k1_eq80(x.w, '"'));
    }
    if (tid < head) par ^= buf[tid] == '"';
    const u64 t0 = head + nv * 16;
    if (tid < n - t0) par ^= buf[t0 + tid] == '"';
    par &= 1u;
    const u64 b = __ballot(par);
    if (lane_id() == 0 && (__popcll(b) & 1)) atomicXor(out, 1u);
}
hipError_t msa_launch_quote_parity(const u8 *buf, u64 n, u32 *out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, 4, s);
    if (e != hipSuccess || !n) return e;
    u64 blocks = (n / 16 + 255) / 256;
    const u64 cap = 2048;  // 8 workgroups per CU of a 256-CU MI355X
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_quote_parity, dim3((u32)blocks), dim3(256), 0, s, buf, n, out);
    return hipGetLastError();
}

hipError_t msa_launch_first_end(const u8 *buf, u64 n, u32 p, u32 cr, u64 *out, hipStream_t s) {
    hipLaunchKernelGGL(k_first_end, dim3(1), dim3(64), 0, s, buf, n, p, cr, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// host launchers
static int g_cus = 0;
static int num_cus() {
    if (!g_cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, dev) == hipSuccess) g_cus = p.multiProcessorCount;
        if (g_cus <= 0) g_cus = 256;
    }
    return g_cus;
}

hipError_t msa_launch_summary(const u8 *buf, u64 seg_begin, u64 seg_end, u32 nchunks, ChunkSum *out,
                              hipStream_t s) {
    if (!nchunks) return hipSuccess;
    u32 blocks = (nchunks + 3) / 4;
    u32 cap = (u32)num_cus() * 8;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(k_chunk_summary, dim3(blocks), dim3(256), 0, s, buf, seg_begin, seg_end, nchunks, out);
    return hipGetLastError();
}

u32 msa_fn_blocks(u32 nchunks) { return (nchunks + FN_T - 1) / FN_T; }

hipError_t msa_launch_fn(const ChunkSum *sums, u64 seg_begin, u32 nchunks, Fn *btot, State *bstate, Fn *total,
                         State init, State *carry, State *final_state, hipStream_t s) {
    if (!nchunks) return hipSuccess;
    const u32 nb = msa_fn_blocks(nchunks);
    hipLaunchKernelGGL(k_fn_reduce, dim3(nb), dim3(FN_T), 0, s, sums, seg_begin, nchunks, btot);
    hipLaunchKernelGGL(k_fn_top, dim3(1), dim3(FN_T), 0, s, (const Fn *)btot, nb, seg_begin, init, bstate, total);
    hipLaunchKernelGGL(k_fn_down, dim3(nb), dim3(FN_T), 0, s, sums, seg_begin, nchunks, (const State *)bstate, carry,
                       final_state);
    return hipGetLastError();
}

hipError_t msa_launch_scan(const ScanArgs &a, int mode, hipStream_t s) {
    if (!a.nchunks) return hipSuccess;
    u32 blocks = (a.nchunks + K3_WAVES - 1) / K3_WAVES;
    u32 cap = (u32)num_cus() * K3_BLOCKS_PER_CU;
    if (blocks > cap) blocks = cap;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)k_scan_main<0>, hipFuncAttributeMaxDynamicSharedMemorySize, K3_LDS);
        (void)hipFuncSetAttribute((const void *)k_scan_main<2>, hipFuncAttributeMaxDynamicSharedMemorySize, K3_LDS);
        attr = true;
    }
    if (mode == 0) hipLaunchKernelGGL(k_scan_main<0>, dim3(blocks), dim3(K3_THREADS), K3_LDS, s, a);
    else if (mode == 2) hipLaunchKernelGGL(k_scan_main<2>, dim3(blocks), dim3(K3_THREADS), K3_LDS, s, a);
    else hipLaunchKernelGGL(k_scan_main<1>, dim3(blocks), dim3(K3_THREADS), 0, s, a);
    return hipGetLastError();
}
