// msa_k3.hip -- K3 for the CSV: record/field structure, lyric tokens and word
// counting in one pass over each 16 KiB chunk (reader state at the chunk start
// from K1/K2, msa_scan.hip).
//
// Replaces the byte-serial reader and tokenizer of the reference
// (read_csv_record, parallel_spotify.c:549-633; parse_csv_line 258-304;
// process_lyrics 350-394; ht_put 126-149) for the lyric column.
//
// Layout of the work (gfx950, wave64):
//   * a wave moves 4 KiB per iteration; lane l owns the 64 contiguous bytes
//     [64 l, 64 l + 64) as four dwordx4 loads, so every byte class is a u64
//     mask per lane and every cross-lane step (quote parity, record index,
//     comma count) is a handful of ballots per 4 KiB;
//   * per-record structure is computed per lane segment (between record
//     terminators) with bit arithmetic, not per byte;
//   * the wave's token starts go to a per-wave LDS list; the lanes take them
//     64 at a time, re-read each key (<= 16 bytes) from the just-loaded input
//     (L1/L2) and count it in ONE workgroup-wide LDS table of 16-byte keys
//     (4-slot buckets); keys the LDS table cannot hold are batched per wave
//     and inserted into the HBM tables asynchronously (pipelined loads).
#include "msa_internal.h"
#include "msa_k1.h"
#include "msa_tables.h"

#include <algorithm>

namespace {

#ifndef Q_T
#define Q_T 1024                 // 16 waves: one workgroup per CU
#endif
#ifndef Q_WGCU
#define Q_WGCU 1                 // token-pass workgroups per CU (2: each with half the LDS -- 8 waves per SIMD)
#endif
#define Q_W (Q_T / 64)
#define Q_BLK 4096               // bytes per wave-iteration
#ifndef Q_TDL
#define Q_TDL 0                  // 1: fewer bytes through the texture data path (see k_scan_tokens)
#endif
#ifndef Q_KAL
#define Q_KAL 0                  // 1: keys re-read as two 16-byte-aligned dwordx4 loads (a 32-byte window) + selects
#endif
#ifndef Q_PROBE1
#define Q_PROBE1 0               // 1: a bucket's second half read only by lanes its first half left open
#endif
#ifndef Q_LIST2
#define Q_LIST2 1                // 1: the token list built two starts a trip (lowest + highest)
#endif
#ifndef Q_X2
#define Q_X2 0                   // 1: two probe batches a trip in the token pass
#endif
#ifndef TOK_PF
#define TOK_PF 1                 // batches of key loads in flight ahead of the probed one
#endif
static_assert(!(Q_KAL && TOK_PF > 1), "Q_KAL keeps one batch of key loads in flight");
// Token keys are re-read from the input (just loaded: L1/L2) rather than
// from an LDS copy of the block, which leaves the LDS to the word table and
// to a per-wave list of the block's token starts: the lanes share the tokens
// evenly (compaction) instead of each walking its own.
#define Q_LIST 1024              // token entries per wave-iteration (>= 4 bytes per token)
// Each probe batch's misses go straight to the logs in one buffer store per
// wave (round 4; the per-wave LDS miss buffers of round 3 are gone).
#define Q_WLDS (Q_LIST * 2)
#define Q_CUR ((MSA_MLOG_PARTS + 4) * 4)  // log cursors per partition + the dropped-entry count
// LDS word table: 3..8-byte words (92 % of the tokens of lyric text) as
// single u64 keys (12 bytes a slot, 4-slot buckets read as two ds_read_b128);
// 9..16-byte words are logged for k_miss_agg.  Measured on configs[2]
// (csv_scan + k_miss_agg, round 2): S and M words listed apart with a 1024-slot
// M table 1.95 ms, mixed with an M table 1.99, mixed without an M table (the S
// table takes the whole LDS) 1.82 -- the design kept.
#ifndef Q_SSLOTS                 // the rest of the workgroup's share of the CU's LDS
#define Q_SSLOTS (((163840 / Q_WGCU - Q_W * Q_WLDS - Q_CUR) / 12) & ~31)
#endif
#define Q_SNB (Q_SSLOTS / 4)
#define Q_TAB (Q_SSLOTS * 12)
#define Q_LDS (Q_TAB + Q_W * Q_WLDS + Q_CUR)
static_assert(Q_LDS * Q_WGCU <= 163840, "K3 LDS exceeds the CU's 160 KiB");
static_assert(Q_SNB < 4096, "lds_find8 scales 20 hash bits by Q_SNB in 32 bits");
static_assert(Q_SSLOTS % 32 == 0 && Q_TAB % 16 == 0 && Q_WLDS % 16 == 0,
              "LDS carve-outs stay 16-byte aligned");

// Every key byte of a token is < 0x80 (alnum or '\''), so bit 63 of the
// second key word is free: it marks a published slot (an S word has k1 == 0).
#define KMARK 0x8000000000000000ull

// diagnostic ablations of tools/ablate.py (MSA_ABLATE bits) are compiled in
// only with -DK3_ABLATE=1: the production kernel carries no test of them
#ifndef K3_ABLATE
#define K3_ABLATE 0
#endif

// Lower-cases token bytes ('0'..'9', 'A'..'Z', 'a'..'z', '\'', or zero
// padding): of those only 'A'..'Z' have bit 6 set and bit 5 clear, so setting
// bit 5 wherever bit 6 is set is the whole mapping
__device__ __forceinline__ u64 lower_tok8(u64 x) { return x | ((x >> 1) & 0x2020202020202020ull); }

__device__ __forceinline__ uint4 ldg16(const u8 *p) { return *reinterpret_cast<const uint4 *>(p); }
// a wave-uniform read of data no kernel writes while this one runs: through
// the constant address space, i.e. a scalar load (counted in lgkmcnt, so it
// does not wait behind the wave's vector loads)
#ifndef K3_SLOAD
#define K3_SLOAD 1
#endif
#if K3_SLOAD
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T *sload(const T *p) {
    return (const __attribute__((address_space(4))) T *)(size_t)p;
}
#else
template <class T>
__device__ __forceinline__ const T *sload(const T *p) { return p; }
#endif
__device__ __forceinline__ State sload_state(const State *p) {
    const auto q = sload(p);
    State s;
    s.rec = q->rec;
    s.rs = q->rs;
    s.p = q->p;
    s.cr = q->cr;
    s.c = q->c;
    s.z = q->z;
    return s;
}

// lane l receives lane l+1's value (lane 63: 0) / lane l-1's (lane 0: 0): DPP wave shifts
__device__ __forceinline__ u32 from_next32(u32 v) { return __builtin_amdgcn_update_dpp(0u, v, 0x130, 0xF, 0xF, false); }
__device__ __forceinline__ u32 from_prev32(u32 v) { return __builtin_amdgcn_update_dpp(0u, v, 0x138, 0xF, 0xF, false); }
__device__ __forceinline__ u64 from_next(u64 v) {
    return ((u64)from_next32((u32)(v >> 32)) << 32) | from_next32((u32)v);
}
__device__ __forceinline__ u64 from_prev(u64 v) {
    return ((u64)from_prev32((u32)(v >> 32)) << 32) | from_prev32((u32)v);
}

__device__ __forceinline__ u64 bits_lo(u32 n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }  // [0, n)
__device__ __forceinline__ u64 bits_hi(u32 n) { return n >= 64 ? 0ull : (~0ull << n); }           // [n, 64)

__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 4 packed 0x80-per-byte masks of one dword -> 4 bits
__device__ __forceinline__ u32 pk4(u32 m) { return (((m >> 7) * 0x00204081u) >> 21) & 0xFu; }

struct Masks {
    u64 Q, C, NL, CR, Z, T;
};

// An opaque use/def: the value is computed before this point and not
// recomputed after it.
__device__ __forceinline__ void pin64(u64 &x) { asm volatile("" : "+v"(x)); }

// "byte == c" per byte as 0x80 flags (exact: no cross-byte carries)
__device__ __forceinline__ u32 eq80(u32 x, u32 c) {
    const u32 y = x ^ (c * 0x01010101u);
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
}
// any byte == c (cheap, may not locate it): the classic has-zero test
__device__ __forceinline__ u32 has80(u32 x, u32 c) {
    const u32 y = x ^ (c * 0x01010101u);
    return (y - 0x01010101u) & ~y & 0x80808080u;
}
// 'A'..'Z' -> 'a'..'z' in place (every other byte unchanged, bytes >= 0x80
// stay >= 0x80) and the token-byte flags of process_lyrics (alnum or '\'')
__device__ __forceinline__ u32 lower_tok(u32 &x) {
    const u32 hi = x & 0x80808080u, y = x & 0x7F7F7F7Fu;
    const u32 up = (y + 0x3F3F3F3Fu) & ~(y + 0x25252525u) & ~hi & 0x80808080u;  // 'A'..'Z'
    x |= up >> 2;
    const u32 z = y | (up >> 2);
    const u32 lo = (z + 0x1F1F1F1Fu) & ~(z + 0x05050505u);                     // 'a'..'z'
    const u32 dg = (z + 0x50505050u) & ~(z + 0x46464646u);                     // '0'..'9'
    return (((lo | dg) & ~hi) & 0x80808080u) | eq80(x, '\'');
}

// Byte classes of the lane's 64 bytes (bit i = byte i; bytes at or past
// `nvalid` cleared).  '\r' and NUL masks are computed only when the wave's block holds
// one (a wave-uniform branch).
__device__ __forceinline__ Masks classify64x(uint4 (&v)[4], u32 nvalid, bool test_rare) {
    Masks k{0, 0, 0, 0, 0, 0};
    u32 rare = 0;
    u32 q0 = 0, q1 = 0, c0 = 0, c1 = 0, n0 = 0, n1 = 0, t0 = 0, t1 = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        u32 w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
        for (int d = 0; d < 4; ++d)
            if (test_rare) rare |= has80(w[d], '\r') | has80(w[d], 0);
        // dwords in pairs: byte k = 2q + h of each 64-bit mask (dot4 packing)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kb = 2 * q + h;
            const u32 a = w[2 * h], b = w[2 * h + 1];
            const u32 a7 = a & 0x7F7F7F7Fu, b7 = b & 0x7F7F7F7Fu;
            swar_put8(q0, q1, kb, swar_pack8x128(eq80x(a, a7, '"'), eq80x(b, b7, '"')));
            swar_put8(c0, c1, kb, swar_pack8x128(eq80x(a, a7, ','), eq80x(b, b7, ',')));
            swar_put8(n0, n1, kb, swar_pack8x128(eq80x(a, a7, '\n'), eq80x(b, b7, '\n')));
            swar_put8(t0, t1, kb, swar_pack8x128(tok80x(a, a7), tok80x(b, b7)));
        }
    }
    k.Q = mk64(q0, q1); k.C = mk64(c0, c1); k.NL = mk64(n0, n1); k.T = mk64(t0, t1);
    if (__ballot(rare != 0)) {
        u32 r0 = 0, r1 = 0, z0 = 0, z1 = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const u32 w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int kb = 2 * q + h;
                swar_put8(r0, r1, kb, swar_pack8x128(eq80(w[2 * h], '\r'), eq80(w[2 * h + 1], '\r')));
                swar_put8(z0, z1, kb, swar_pack8x128(eq80(w[2 * h], 0), eq80(w[2 * h + 1], 0)));
            }
        }
        k.CR = mk64(r0, r1);
        k.Z = mk64(z0, z1);
    }
    const u64 vm = bits_lo(nvalid);
    k.Q &= vm; k.C &= vm; k.NL &= vm; k.CR &= vm; k.Z &= vm; k.T &= vm;
    // materialise the masks here: left alone, the scheduler sinks the byte
    // tests to their first use (the token phase) and keeps all 64 input bytes
    // live across the structure code, spilling to scratch
    pin64(k.Q); pin64(k.C); pin64(k.NL); pin64(k.CR); pin64(k.Z); pin64(k.T);
    return k;
}

__device__ __forceinline__ u64 pxor_ex64(u64 q) {  // bit j = parity of bits < j
    u64 x = q << 1;
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    x ^= x << 32;
    return x;
}

// 128-bit (hi:lo) >> k, low 64 bits, 0 < k < 64
__device__ __forceinline__ u64 shr128(u64 lo, u64 hi, u32 k) { return (lo >> k) | (hi << (64 - k)); }

// 9..10-byte words in the LDS table (Q_PK10): a lower-cased token byte has
// one of 37 values, coded in 6 bits, nonzero -- 'a'..'z' 33..58, '0'..'9'
// 16..25, '\'' 7: (c & 0x1F) | ((c >> 1) & 0x20) -- so ten of them pack into
// 60 bits (zero codes past the word's end); bit 63 tags the packed key, which
// an S key (bytes < 0x80) never has.  The 9..10-byte words (~2/3 of the
// 9..16-byte tokens of lyric text) are then counted in LDS instead of logged.
// Measured and not kept (profiles/r06_ab_pk10.txt): WRITE_SIZE -15 %,
// k_miss_agg 0.305 -> 0.28 ms, but the pack's VALU (+18 %) made the token pass
// 0.80 -> 0.90 ms, 2.885 -> 2.95 ms/step.
#ifndef Q_PK10
#define Q_PK10 0
#endif
#define PK10_TAG 0x8000000000000000ull
__device__ __forceinline__ u64 pk6x8(u64 y) {  // 8 token bytes -> 48 bits of codes
    y = (y & 0x1F1F1F1F1F1F1F1Full) | ((y >> 1) & 0x2020202020202020ull);
    y = (y & 0x003F003F003F003Full) | ((y >> 2) & 0x0FC00FC00FC00FC0ull);
    y = (y & 0x00000FFF00000FFFull) | ((y >> 4) & 0x00FFF00000FFF000ull);
    return (y & 0xFFFFFFull) | ((y >> 8) & 0xFFFFFF000000ull);
}
__device__ __forceinline__ u64 pk10(u64 k0, u64 k1m) {  // k1m: bytes 8, 9 (| KMARK)
    const u32 h = (u32)k1m & 0xFFFFu;
    const u32 c = (h & 0x1F1Fu) | ((h >> 1) & 0x2020u);
    return pk6x8(k0) | ((u64)((c & 0x3Fu) | ((c >> 2) & 0xFC0u)) << 48) | PK10_TAG;
}
__device__ __forceinline__ u32 unpk6(u32 c) { return c ? c + (c >= 32 ? 0x40u : 0x20u) : 0u; }
__device__ __forceinline__ void unpk10(u64 p, u64 &k0, u64 &k1m) {  // the inverse of pk10
    k0 = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) k0 |= (u64)unpk6((u32)(p >> (6 * j)) & 63u) << (8 * j);
    k1m = KMARK | unpk6((u32)(p >> 48) & 63u) | (unpk6((u32)(p >> 54) & 63u) << 8);
}

// LDS lookup of an S key (3..8 bytes, nonzero).  Returns the slot or ~0u.
// The bucket: full-rate 24-bit multiplies only (v_mul_u32_u24; the 32-bit
// ones are quarter rate), the top 20 bits scaled to Q_SNB (< 2^12) (HIP's
// __umul24 returns int: the products are taken as u32 before any shift)
__device__ __forceinline__ u32 lds_bucket8(u64 k0) {
    const u32 lo = (u32)k0, hi = (u32)(k0 >> 32);
    u32 t = lo + ((hi << 13) | (hi >> 19));
    t ^= t >> 17;
    u32 h = (u32)__umul24(t, 0x9E3779u);
    h ^= h >> 13;
    return (u32)__umul24(h >> 12, (u32)Q_SNB) >> 20;
}
__device__ __forceinline__ u32 match4(const ulonglong2 &s01, const ulonglong2 &s23, u64 k) {
    return s01.x == k ? 0u : (s01.y == k ? 1u : (s23.x == k ? 2u : (s23.y == k ? 3u : 4u)));
}
// a key not among bucket b's four (s01, s23): claim its first empty slot
// (CAS; a racing claim of the same key is a hit), else the next bucket
__device__ __forceinline__ u32 lds_find8_rest(u64 *skeys, u64 k0, u32 b, ulonglong2 s01, ulonglong2 s23) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const u32 base = b * 4;
        if (p) {
            s01 = *reinterpret_cast<const ulonglong2 *>(&skeys[base]);
            s23 = *reinterpret_cast<const ulonglong2 *>(&skeys[base + 2]);
            const u32 hit = match4(s01, s23, k0);
            if (hit < 4) return base + hit;
        }
        u32 i = s01.x == 0 ? 0u : (s01.y == 0 ? 1u : (s23.x == 0 ? 2u : (s23.y == 0 ? 3u : 4u)));
        for (; i < 4; ++i) {
            const u64 old = atomicCAS((unsigned long long *)&skeys[base + i], 0ull, (unsigned long long)k0);
            if (old == 0 || old == k0) return base + i;
        }
        b = (b + 1 == Q_SNB) ? 0 : b + 1;
    }
    return ~0u;
}
__device__ __forceinline__ u32 lds_find8(u64 *skeys, u64 k0) {
    u32 b = lds_bucket8(k0);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const u32 base = b * 4;
        const ulonglong2 s01 = *reinterpret_cast<const ulonglong2 *>(&skeys[base]);
#if Q_PROBE1
        // the bucket's second half read only by the lanes its first half did
        // not settle (keys are claimed in slot order, so the Zipf head -- seen
        // first -- sits in slots 0 / 1): fewer lanes per ds_read_b128, fewer
        // bank conflicts
        if (s01.x == k0) return base;
        if (s01.y == k0) return base + 1;
        const ulonglong2 s23 = *reinterpret_cast<const ulonglong2 *>(&skeys[base + 2]);
        const u32 hit = s23.x == k0 ? 2u : (s23.y == k0 ? 3u : 4u);
#else
        const ulonglong2 s23 = *reinterpret_cast<const ulonglong2 *>(&skeys[base + 2]);
        const u32 hit = match4(s01, s23, k0);
#endif
        if (hit < 4) return base + hit;
        u32 i = s01.x == 0 ? 0u : (s01.y == 0 ? 1u : (s23.x == 0 ? 2u : (s23.y == 0 ? 3u : 4u)));
        for (; i < 4; ++i) {
            const u64 old = atomicCAS((unsigned long long *)&skeys[base + i], 0ull, (unsigned long long)k0);
            if (old == 0 || old == k0) return base + i;
        }
        b = (b + 1 == Q_SNB) ? 0 : b + 1;
    }
    return ~0u;
}
// Two keys a lane (Q_X2): both buckets' four reads in flight together, then
// the hits; the rest one key after the other.  p*: probe this key at all.
__device__ __forceinline__ void lds_find8x2(u64 *skeys, bool pa, u64 ka, bool pb, u64 kb, u32 &sa, u32 &sb) {
    const u32 ba = lds_bucket8(ka), bb = lds_bucket8(kb);
    const ulonglong2 a01 = *reinterpret_cast<const ulonglong2 *>(&skeys[ba * 4]);
    const ulonglong2 a23 = *reinterpret_cast<const ulonglong2 *>(&skeys[ba * 4 + 2]);
    const ulonglong2 b01 = *reinterpret_cast<const ulonglong2 *>(&skeys[bb * 4]);
    const ulonglong2 b23 = *reinterpret_cast<const ulonglong2 *>(&skeys[bb * 4 + 2]);
    const u32 ha = match4(a01, a23, ka), hb = match4(b01, b23, kb);
    sa = ha < 4 ? ba * 4 + ha : ~0u;
    sb = hb < 4 ? bb * 4 + hb : ~0u;
    if (pa && ha >= 4) sa = lds_find8_rest(skeys, ka, ba, a01, a23);
    if (pb && hb >= 4) sb = lds_find8_rest(skeys, kb, bb, b01, b23);
}

template <bool CASF = (TAB_CAS_FIRST != 0)>
__device__ __forceinline__ void hbm_insert16(const ScanArgs &a, u64 k0, u64 k1m, u64 cnt) {
    if (k1m == KMARK) s_insert<false, CASF>(a.s_tab, a.s_mask, k0, cnt, a.s_list, a.s_list_cap, a.ctr);
    else m_insert<false, CASF>(a.m_tab, a.m_mask, k0, k1m & ~KMARK, cnt, a.m_list, a.m_list_cap, a.ctr);
}

// Keys the LDS table cannot hold are not counted in HBM one atomic at a
// time (scattered device-scope atomics run at a few tens of G/s chip-wide and
// made up a third of the kernel).  They are logged instead: per workgroup and
// key partition (16 by key hash), plain 16-byte stores behind an LDS cursor;
// k_miss_agg then counts each partition in LDS and adds each distinct key to
// the HBM table once per aggregating workgroup.  A full log partition drops
// the entry and flags OVF_MLOG (the split runs again with larger logs); only
// at the 2^24-entry partition limit do entries go straight into the HBM table.
__device__ __forceinline__ u32 mlog_part(u64 k0, u64 k1m) {
    // full-rate operations only: two 64-bit multiplies had cost six
    // quarter-rate v_mul_lo/hi_u32 per probe batch of the token pass
    u32 t = (u32)k0 ^ __builtin_amdgcn_alignbit((u32)(k0 >> 32), (u32)(k0 >> 32), 11) ^ (u32)k1m ^
            __builtin_amdgcn_alignbit((u32)(k1m >> 32), (u32)(k1m >> 32), 23);
    t ^= t >> 15;
    u32 h;  // v_mul_u32_u24 (full rate) by hand: the compiler turns the masked __umul24 into v_mul_lo_u32
    asm("v_mul_u32_u24 %0, 0x9e3779, %1" : "=v"(h) : "v"(t ^ (t >> 16)));
    return (h >> 20) & 15u;
}

// The workgroup's LDS table is flushed into the same logs at the end of the
// scan (k_miss_agg then inserts each distinct key once per aggregating
// workgroup, not once per scan workgroup): a flushed entry carries its count
// (1..32767) in the bytes' free high bits -- bit 7 of every key byte (token
// bytes are < 0x80) except KMARK.  A logged miss has none set: count 1.
#define MLOG_CMAX 32767u
__device__ __forceinline__ u64 spread8(u32 c) {  // bit j of c -> bit 8j + 7
    u64 r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r |= (u64)((c >> j) & 1u) << (8 * j + 7);
    return r;
}
__device__ __forceinline__ u32 gather8(u64 x) {  // bit 8j + 7 -> bit j
    u32 r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r |= (u32)((x >> (8 * j + 7)) & 1u) << j;
    return r;
}
#define MLOG_KEYBITS 0x7F7F7F7F7F7F7F7Full

// Record structure of one 4 KiB block (read_csv_record 549-633 + parse_csv_line
// 258-304): from the reader state st at the block start (updated to the state
// after it) and the block's byte classes, the per-record arrays (rec_start,
// f0, tss, tse, nulrel) and the lane's live lyric bytes (returned).  tail /
// tvm: the 16 bytes after the block and their validity; prevQ: the byte
// before the block is a '"'.
__device__ __forceinline__ u64 struct_block(const ScanArgs &a, State &st, const Masks &k, uint4 tail, u32 tvm,
                                            u64 lpos, u32 prevQ) {
    const u32 lane = lane_id();
    const u64 lt = (1ull << lane) - 1ull;
    // ---- record structure (read_csv_record + parse_csv_line) ----
    const u64 B = __ballot(__popcll(k.Q) & 1u);
    const u32 pin = st.p ^ (mbcnt(B) & 1u);
    const u64 inq = pxor_ex64(k.Q) ^ (pin ? ~0ull : 0ull);
    const u64 CRu = k.CR & ~inq, NLu = k.NL & ~inq, Cu = k.C & ~inq;
    // DPP and bpermute read the source lane's register only when that
    // lane is active: every cross-lane move below runs on all 64 lanes,
    // the per-lane choice is a select afterwards
    const u64 CRp = from_prev(CRu) >> 63;
    const u64 NLn = from_next(k.NL) & 1ull;
    const u64 pCR = lane ? CRp : (u64)st.cr;
    const u64 TERM = CRu | (NLu & ~((CRu << 1) | pCR));
    const u32 tail_nl = ((tail.x & 0xFFu) == '\n' && (tvm & 1u)) ? 1u : 0u;
    const u64 nNL = lane == 63 ? (u64)tail_nl : NLn;
    // '"' at the byte after the lane (text start after a comma at byte
    // 63) and at the byte before it (text end before a terminator at byte 0)
    const u32 tail_q = ((tail.x & 0xFFu) == '"' && (tvm & 1u)) ? 1u : 0u;
    const u64 Qnx = from_next(k.Q) & 1ull, Qpv = from_prev(k.Q) >> 63;
    const u32 qnext = lane == 63 ? tail_q : (u32)Qnx;
    const u32 qprev = lane ? (u32)Qpv : prevQ;
    const u64 SW = CRu & ((k.NL >> 1) | (nNL << 63));  // '\r' terminators that swallow a '\n'

    const u32 nt = (u32)__popcll(TERM);
    const u32 lastT = nt ? 63u - (u32)__clzll(TERM) : 0u;
    const u64 above = nt ? bits_hi(lastT + 1) : ~0ull;
    const u32 cq = min((u32)__popcll(Cu & above), 3u);
    const bool zq = (k.Z & above) != 0;
    const u64 C1 = __ballot(cq >= 1), C2 = __ballot(cq >= 2), C3 = __ballot(cq >= 3);
    const u64 Zb = __ballot(zq), Bh = __ballot(nt != 0);
    const u64 J = Bh & lt;
    u64 M;
    u32 cin;
    bool zin;
    if (J) {
        const u32 jl = 63u - (u32)__clzll(J);
        M = lt & ~bits_lo(jl);
        cin = 0;
        zin = (Zb & M) != 0;
    } else {
        M = lt;
        cin = st.c;
        zin = st.z || ((Zb & M) != 0);
    }
    cin = min(cin + (u32)__popcll(C1 & M) + (u32)__popcll(C2 & M) + (u32)__popcll(C3 & M), 3u);
    // record index at the lane's first byte: prefix of terminator counts
    const u64 T1 = __ballot(nt >= 1), T2 = __ballot(nt >= 2), T3 = __ballot(nt >= 3);
    u64 rin = st.rec + (u64)__popcll(T1 & lt) + (u64)__popcll(T2 & lt);
    if (T3) {  // records shorter than 32 bytes (rare): full prefix of nt
        u32 tot;
        rin = st.rec + wave_prefix<7>(nt, tot);
    }
    // record start at the lane's first byte (for NUL offsets; only
    // when a NUL is anywhere in this block's wave)
    const u64 endp = nt ? lpos + lastT + 1 + ((SW >> lastT) & 1ull) : 0;
    const u64 Zany = __ballot(k.Z != 0);
    u64 rsin = st.rs;
    if (Zany) {  // wave-uniform branch: the shuffle runs on every lane
        const u64 rsj = __shfl(endp, J ? 63 - __clzll(J) : (int)lane);
        if (J) rsin = rsj;
    }

    // per segment of the lane (between terminators): live lyric bytes,
    // record starts, first NUL
    u64 live = 0;
    {
        u64 E = TERM;
        u32 lo = 0, cc = cin;
        bool zz = zin;
        u64 r = rin, rs = rsin;
        for (;;) {
            const u32 hi = E ? (u32)__ffsll((long long)E) - 1 : 64u;
            const u64 seg = bits_hi(lo) & bits_lo(hi);
            const u64 zs = k.Z & seg;
            if (zs && !zz && a.want_nul && r < a.rec_cap) {
                const u32 zp = (u32)__ffsll((long long)zs) - 1;
                a.nulrel[r] = (u32)(lpos + zp - rs) + 1u;
            }
            bool ok = false;  // the record's third comma is at or before this segment's end
            if (r >= a.first_rec && !zz) {
                // commas after a NUL do not count (the C string ends there)
                u64 x = Cu & seg & (zs ? bits_lo((u32)__ffsll((long long)zs) - 1) : ~0ull);
                u32 from = lo;
                ok = true;
                for (u32 n = cc; n < 3; ++n) {
                    if (!x) { ok = false; break; }
                    from = (u32)__ffsll((long long)x);  // one past that comma
                    x &= x - 1;
                    // field 0 ends here (artist span for k_rec_fast)
                    if (n == 0 && r < a.rec_cap) a.f0[r] = lpos + from - 1;
                }
                if (ok) {
                    u64 lv = bits_hi(from) & bits_lo(hi);
                    if (zs) lv &= bits_lo((u32)__ffsll((long long)zs) - 1);
                    live |= lv;
                    if (cc < 3 && r < a.rec_cap) {  // field 3 starts here; '"' there?
                        const u32 q = from < 64 ? (u32)(k.Q >> from) & 1u : qnext;
                        a.tss[r] = (lpos + from) | (q ? SPAN_Q : 0ull);
                    }
                }
            }
            if (!E) break;
            if (r < a.rec_cap) {  // the record ends at this terminator
                const u32 q = hi ? (u32)(k.Q >> (hi - 1)) & 1u : qprev;
                u64 fl = q ? SPAN_Q : 0ull;
                if (zz || zs) fl |= SPAN_NUL;  // the C string ends before: exact path
                else if (!ok) fl |= SPAN_NOLINE;  // header, or < 3 commas (parse_csv_line fails)
                a.tse[r] = (lpos + hi) | fl;
            }
            const u64 ns = lpos + hi + 1 + ((SW >> hi) & 1ull);
            ++r;
            if (r < a.rec_cap) a.rec_start[r] = ns;
            rs = ns;
            cc = 0;
            zz = false;
            lo = hi + 1;
            E &= E - 1;
        }
    }
    // carry the reader state to the next block (lane 63 has seen every byte)
    {
        const u32 cout = nt ? cq : min(cin + cq, 3u);
        const bool zout = nt ? zq : (zin || zq);
        st.p ^= (u32)__popcll(B) & 1u;
        st.cr = readlane((u32)(CRu >> 63), 63);
        st.c = readlane(cout, 63);
        st.z = readlane((u32)zout, 63);
        st.rec = rin + nt;
        st.rec = readlane64(st.rec, 63);
        if (Bh) st.rs = readlane64(endp, 63 - __clzll(Bh));
    }
    return live;
}

// The token phase of one 4 KiB block (process_lyrics, parallel_spotify.c:
// 350-394): w = the lane's 64 token-byte bits, Tn = the 64 after them, S0 =
// the counted token starts.
// the workgroup's miss logs as a buffer resource: a store out of its range
// (lanes without a miss) is dropped by the bounds check
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mlog_rsrc(const ScanArgs &a) {
    ulonglong2 *base = a.mlog + (u64)blockIdx.x * MSA_MLOG_PARTS * a.mlog_cap;
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)(MSA_MLOG_PARTS * a.mlog_cap * 16u), 0x00020000);
}
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Long-word positions: each wave takes ranges of l_pos from Counters::l_occ
// lch slots at a time (one device atomic per range, not per block: every
// wave adding to that one word once per 4 KiB block serialised at the
// memory side -- 3.1 of configs[4]'s 3.9 ms token pass); the slots of a range
// a wave does not fill are set to LP_NONE (k_long_insert skips them).
#define LP_NONE (~0ull)
__device__ __forceinline__ void lpos_fill(const ScanArgs &a, u64 from, u64 to) {
    for (u64 k = from + lane_id(); k < to && k < a.l_cap; k += 64) a.l_pos[k] = LP_NONE;
}
static_assert(!(Q_X2 && (Q_KAL || Q_TDL || TOK_PF > 1 || K3_ABLATE || Q_PK10)), "Q_X2: the plain key loads only");
__device__ __forceinline__ void tok_phase(const ScanArgs &a, u64 ib, u64 lpos, u64 w, u64 Tn, u64 S0, u64 *skeys,
                                          u32 *scnts, u16 *list, u32 *lcur,
                                          u64 &words, __amdgpu_buffer_rsrc_t rsrc, u64 &lres, u64 &lend, u64 lch) {
    const u32 lane = lane_id();
    // runs: rK bit b = bytes b .. b+K-1 are token bytes (w = Tn:T)
    const u64 r2 = w & shr128(w, Tn, 1), r2h = Tn & (Tn >> 1);
    const u64 r3 = r2 & shr128(w, Tn, 2);
    const u64 r4 = r2 & shr128(r2, r2h, 2), r4h = r2h & (r2h >> 2);
    const u64 r8 = r4 & shr128(r4, r4h, 4), r8h = r4h & (r4h >> 4);
    const u64 r16 = r8 & shr128(r8, r8h, 8);
    const u64 r17 = r16 & shr128(w, Tn, 16);
    const u64 r9 = r8 & shr128(w, Tn, 8);
    const u64 sS = S0 & r3 & ~r9, sM = S0 & r9 & ~r17, sL = S0 & r17;
    words += (u64)__popcll(S0 & r3);

    // long words (> 16 bytes): positions for k_long_insert
    const u64 BL = (K3_ABLATE && (a.ablate & 256)) ? 0ull : __ballot(sL != 0);  // 256: no long-word positions
    if (BL) {
        const u32 nl = (u32)__popcll(sL);
        u32 tot;
        const u32 pre = wave_prefix<6>(nl, tot);
        if (lres + tot > lend) {  // a new range (the rest of the old one unused)
            lpos_fill(a, lres, lend);
            const u64 want = tot > lch ? (u64)tot : lch;
            u64 b = 0;
            if (lane == 0) b = atomicAdd((unsigned long long *)&a.ctr->l_occ, (unsigned long long)want);
            lres = readlane64(b, 0);
            lend = lres + want;
        }
        u64 base = lres + pre;
        lres += tot;
        for (u64 m = sL; m; m &= m - 1) {
            const u32 b = (u32)__ffsll((long long)m) - 1;
            if (base < a.l_cap) a.l_pos[base] = (lpos + b) | a.lpos_tag;
            else atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_L);
            ++base;
        }
    }

    // 3..16-byte words.  The wave's token starts go to its LDS list
    // (block offset | (length - 3) << 12); then the lanes take them 64
    // at a time: 3..8-byte words probe the LDS table, 9..16-byte words
    // go to the miss logs.  Diagnostic ablations (K3_ABLATE builds,
    // MSA_ABLATE; results invalid): 1 no tokens at all, 2 no counting,
    // 32 keys without the LDS table, 4 LDS misses dropped, 128 keys not
    // re-read from memory
    u64 m = (K3_ABLATE && (a.ablate & 3)) ? 0ull : (sS | sM);
    u32 nS;
    const u32 ntl = (u32)__popcll(m);
    u32 li = wave_prefix<5>(ntl, nS);
    // token length (<= 16 here): first non-token bit at or after b, from the
    // 32 bits [b, b + 32) of (Tn:T)
    const u32 d0 = (u32)w, d1 = (u32)(w >> 32), d2 = (u32)Tn;
    auto entry = [&](u32 b) -> u16 {
        const u32 run = __builtin_amdgcn_alignbit(b >= 32 ? d2 : d1, b >= 32 ? d1 : d0, b & 31u);
        const u32 len = (u32)__ffs(~run) - 1;  // 3..16
        return (u16)((lane * 64 + b) | ((len - 3) << 12));
    };
#if Q_LIST2
    // two tokens a trip, the lowest and the highest start left (half the
    // trips of the loop-carried chain; the lane's list range filled from
    // both ends)
    u32 hi = li + ntl;
    while (__ballot(m != 0)) {
        if (m) {
            const u32 b = (u32)__ffsll((long long)m) - 1;
            const u32 bh = 63u - (u32)__clzll(m);
            m &= m - 1;
            list[li++] = entry(b);
            if (bh != b) {
                m &= ~(1ull << bh);
                list[--hi] = entry(bh);
            }
        }
    }
#else
    while (__ballot(m != 0)) {
        if (m) {
            const u32 b = (u32)__ffsll((long long)m) - 1;
            m &= m - 1;
            list[li++] = entry(b);
        }
    }
#endif
    wsync();
    // Keys are re-read from the block (L2) as dwords from the token's
    // dword; the next 64 tokens' loads are issued before this batch is
    // probed, so their latency hides behind the LDS work.
    const u32 nb = (nS + 63) >> 6;
    // key loads of batch j (a stale list entry past the list's end addresses
    // a byte inside the block: harmless, and the loop's vector memory sequence
    // stays the same every trip)
#if Q_KAL
    // the 32 bytes from the 16-byte boundary at or before the token: two
    // aligned dwordx4 loads (k4 unused; kv2 = the second half)
    uint4 kv2, kv2n;
    auto kload = [&](u32 j, u32 &e, uint4 &v, u32 &v4) {
        e = list[min(j * 64 + lane, (u32)Q_LIST - 1u)];
        const size_t pa = (size_t)(a.buf + ib + (e & 4095u)) & ~(size_t)15;
        const uint4 *gp = reinterpret_cast<const uint4 *>(pa);
        v = gp[0];
        kv2n = gp[1];
        v4 = 0;
    };
#elif Q_TDL
    // 12 bytes from the token's dword (a 3..8-byte word and its offset in
    // the dword fit), the next 8 only for 9..16-byte words: fewer bytes
    // returned through the texture data path, which the key gathers kept
    // ~84 % busy (TD_TD_BUSY, profiles/r06_pmc_tok_explore.txt)
    auto kload = [&](u32 j, u32 &e, uint4 &v, u32 &v4) {
        e = list[min(j * 64 + lane, (u32)Q_LIST - 1u)];
        const u32 *gp = reinterpret_cast<const u32 *>(a.buf + ((ib + (e & 4095u)) & ~3ull));
        const uint3 w3 = *reinterpret_cast<const uint3 *>(gp);
        uint2 w2 = make_uint2(0, 0);
        if ((e >> 12) >= 6) w2 = *reinterpret_cast<const uint2 *>(gp + 3);  // length >= 9
        v = make_uint4(w3.x, w3.y, w3.z, w2.x);
        v4 = w2.y;
    };
#else
    auto kload = [&](u32 j, u32 &e, uint4 &v, u32 &v4) {
        e = list[min(j * 64 + lane, (u32)Q_LIST - 1u)];
        const u32 *gp = reinterpret_cast<const u32 *>(a.buf + ((ib + (e & 4095u)) & ~3ull));
        v = *reinterpret_cast<const uint4 *>(gp);
        v4 = gp[4];
    };
#endif
#if Q_X2
    // two batches a trip (the lanes' j-th tokens of batches 2i and 2i + 1):
    // two independent key builds, probes and log stores in flight together
    // -- the pass waits on each batch's dependent chain at 4 waves per SIMD
    u32 enA, k4A, enB, k4B;
    uint4 kvA, kvB;
    kload(0, enA, kvA, k4A);
    kload(1, enB, kvB, k4B);
    auto keyof = [&](u32 e, const uint4 &v, u32 v4, u64 &k0, u64 &k1) {
        const u32 len = (e >> 12) + 3;
        const u32 sh = (u32)(ib + (e & 4095u)) & 3u;
        u64 x0 = mk64(__builtin_amdgcn_alignbyte(v.y, v.x, sh), __builtin_amdgcn_alignbyte(v.z, v.y, sh));
        u64 x1 = mk64(__builtin_amdgcn_alignbyte(v.w, v.z, sh), __builtin_amdgcn_alignbyte(v4, v.w, sh));
        const u32 nbits = 8 * len;  // 24..128
        x0 &= bits_lo(nbits);
        x1 = nbits <= 64 ? 0ull : (x1 & bits_lo(nbits - 64));
        k0 = lower_tok8(x0);
        k1 = lower_tok8(x1) | KMARK;
        return len;
    };
    auto logmiss = [&](bool mis, u64 k0, u64 k1) {
        u32 off = 0xFFFFFFF0u;
        if (mis) {
            const u32 part = mlog_part(k0, k1);
            const u32 at = atomicAdd(&lcur[part], 1u);
            if (at < a.mlog_cap) off = ((u32)__umul24(part, a.mlog_cap) + at) * 16u;  // cap < 2^24
            else if (a.mlog_direct) hbm_insert16<false>(a, k0, k1, 1);  // logs at their size limit
            else atomicAdd(&lcur[MSA_MLOG_PARTS], 1u);
        }
        const u32x4_t ent = {(u32)k0, (u32)(k0 >> 32), (u32)k1, (u32)(k1 >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(ent, rsrc, (int)off, 0, 0);
    };
    for (u32 bt = 0; bt < nb; bt += 2) {
        const u32 eA = enA, v4A = k4A, eB = enB, v4B = k4B;
        const uint4 vA = kvA, vB = kvB;
        const bool hA = bt * 64 + lane < nS, hB = (bt + 1) * 64 + lane < nS;
        kload(bt + 2, enA, kvA, k4A);
        kload(bt + 3, enB, kvB, k4B);
        u64 a0 = 0, a1 = KMARK, b0 = 0, b1 = KMARK;
        const u32 lA = keyof(eA, vA, v4A, a0, a1), lB = keyof(eB, vB, v4B, b0, b1);
        const bool pA = hA && lA <= 8, pB = hB && lB <= 8;
        u32 sA, sB;
        lds_find8x2(skeys, pA, a0, pB, b0, sA, sB);
        if (pA && sA != ~0u) atomicAdd(&scnts[sA], 1u);
        if (pB && sB != ~0u) atomicAdd(&scnts[sB], 1u);
        logmiss(hA && !(pA && sA != ~0u), a0, a1);
        if (bt + 1 < nb) logmiss(hB && !(pB && sB != ~0u), b0, b1);
    }
#else
    u32 en, k4;
    uint4 kv;
    kload(0, en, kv, k4);
#if Q_KAL
    kv2 = kv2n;
#endif
#if TOK_PF > 1
    u32 en2, k42;  // batch bt + 2's, TOK_PF = 2: two batches of key loads in flight
    uint4 kv2;
    kload(1, en2, kv2, k42);
#endif
    for (u32 bt = 0; bt < nb; ++bt) {
        bool mis = false;
        u64 k0 = 0, k1 = KMARK;
        const u32 e = en;
        const uint4 v = kv;
        const u32 v4 = k4;
#if Q_KAL
        const uint4 vb = kv2;
#endif
        const bool have = bt * 64 + lane < nS;
#if TOK_PF > 1
        en = en2;
        kv = kv2;
        k4 = k42;
        kload(bt + 2, en2, kv2, k42);
#else
        kload(bt + 1, en, kv, k4);
#if Q_KAL
        kv2 = kv2n;
#endif
#endif
        if (have) {
            const u32 len = (e >> 12) + 3;
#if Q_KAL
            const u32 s16 = (u32)(size_t)(a.buf + ib + (e & 4095u)) & 15u, sh = s16 & 3u;
            const bool h2 = (s16 & 8u) != 0, h1 = (s16 & 4u) != 0;
            const u32 t0 = h2 ? v.z : v.x, t1 = h2 ? v.w : v.y, t2 = h2 ? vb.x : v.z, t3 = h2 ? vb.y : v.w,
                      t4 = h2 ? vb.z : vb.x, t5 = h2 ? vb.w : vb.y;
            const u32 d0 = h1 ? t1 : t0, d1 = h1 ? t2 : t1, d2 = h1 ? t3 : t2, d3 = h1 ? t4 : t3, d4 = h1 ? t5 : t4;
            (void)v4;
            u64 x0 = mk64(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh));
            u64 x1 = mk64(__builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
#else
            const u32 sh = (u32)(ib + (e & 4095u)) & 3u;
            u64 x0 = mk64(__builtin_amdgcn_alignbyte(v.y, v.x, sh), __builtin_amdgcn_alignbyte(v.z, v.y, sh));
            u64 x1 = mk64(__builtin_amdgcn_alignbyte(v.w, v.z, sh), __builtin_amdgcn_alignbyte(v4, v.w, sh));
#endif
            if (K3_ABLATE && (a.ablate & 128)) {  // diagnostic: keys made up from the list entry (no re-read)
                x0 = (u64)e * 0x9E3779B97F4A7C15ull & 0x7F7F7F7F7F7F7F7Full;
                x1 = x0 >> 3;
            }
            // the token's bytes only (selects, no branches), lower-cased
            const u32 nbits = 8 * len;  // 24..128
            x0 &= bits_lo(nbits);
            x1 = nbits <= 64 ? 0ull : (x1 & bits_lo(nbits - 64));
            k0 = lower_tok8(x0);
            k1 = lower_tok8(x1) | KMARK;
            if (K3_ABLATE && (a.ablate & 32)) {
                words += (k0 ^ k1) == 1;  // keep the key build alive
            } else if (len <= (Q_PK10 ? 10u : 8u)) {
                const u64 sk = (Q_PK10 && len > 8) ? pk10(k0, k1) : k0;
                const u32 slot = lds_find8(skeys, sk);
                if (slot != ~0u) atomicAdd(&scnts[slot], 1u);
                else mis = !(K3_ABLATE && (a.ablate & 4));
            } else {
                mis = !(K3_ABLATE && (a.ablate & 4));
            }
        }
        // the batch's misses straight to their log partitions: a slot from the
        // partition's LDS cursor, then one store for the whole wave -- every
        // trip, lanes without a miss out of the buffer's range -- so waiting for
        // the next batch's key loads never waits for this store.  A full
        // partition drops the entry and counts it: the split runs again with
        // larger logs (Counters::mlog_full, OVF_MLOG) -- unless the logs are at
        // their size limit (2^24 - 1 entries a partition: mlog_direct), where
        // the entry goes straight into the HBM table
        u32 off = 0xFFFFFFF0u;
        if (K3_ABLATE && (a.ablate & 512)) mis = false;  // 512: misses neither counted nor stored
        if (mis) {
            const u32 part = mlog_part(k0, k1);
            const u32 at = atomicAdd(&lcur[part], 1u);
            if (at < a.mlog_cap) off = ((u32)__umul24(part, a.mlog_cap) + at) * 16u;  // cap < 2^24
            else if (a.mlog_direct) hbm_insert16<false>(a, k0, k1, 1);  // logs at their size limit
            else atomicAdd(&lcur[MSA_MLOG_PARTS], 1u);
        }
        const u32x4_t ent = {(u32)k0, (u32)(k0 >> 32), (u32)k1, (u32)(k1 >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(ent, rsrc, (int)off, 0, 0);
    }
#endif
    wsync();
}

// End of a counting workgroup: the wave's pending misses, total_words, the
// LDS table flushed into the logs (counts encoded) and the log lengths.  Only
// this flush inserts into the HBM table when a partition is full (its entries
// carry counts, at most Q_SSLOTS of them); a full partition during the token
// walk drops the miss and flags OVF_MLOG instead (tok_batches).
__device__ __forceinline__ void tok_epilogue(const ScanArgs &a, u64 *skeys, u32 *scnts, u32 *lcur, u64 words) {
    const u32 lane = lane_id();
    words = wave_sum64(words);
    if (lane == 0 && words) atomicAdd((unsigned long long *)&a.ctr->total_words, (unsigned long long)words);
    __syncthreads();
    // the LDS table into the logs, counts encoded (a full partition: HBM insert)
    for (u32 i = threadIdx.x; i < Q_SSLOTS && !(K3_ABLATE && (a.ablate & 32768)); i += Q_T) {  // 32768: no flush
        u32 n = scnts[i];
        if (!n) continue;
        ulonglong2 kk = make_ulonglong2(skeys[i], KMARK);
        if (Q_PK10 && (kk.x & PK10_TAG)) {  // a 9..10-byte word
            u64 u0, u1;
            unpk10(kk.x, u0, u1);
            kk = make_ulonglong2(u0, u1);
        }
        const u32 part = mlog_part(kk.x, kk.y);
        const u64 base = ((u64)blockIdx.x * MSA_MLOG_PARTS + part) * a.mlog_cap;
        while (n) {
            const u32 c = min(n, MLOG_CMAX);
            const u32 at = atomicAdd(&lcur[part], 1u);
            if (at < a.mlog_cap) a.mlog[base + at] = make_ulonglong2(kk.x | spread8(c), kk.y | spread8(c >> 8));
            else hbm_insert16(a, kk.x, kk.y, c);
            n -= c;
        }
    }
    __syncthreads();
    if (threadIdx.x < MSA_MLOG_PARTS) {
        const u32 n = lcur[threadIdx.x];
        a.mlog_n[blockIdx.x * MSA_MLOG_PARTS + threadIdx.x] = min(n, a.mlog_cap);
        // the next split sizes the logs from this (a full partition drops its
        // further entries: OVF_MLOG, the split runs again with larger logs)
        if (n > a.mlog_cap) atomicAdd((unsigned long long *)&a.ctr->mlog_full, (unsigned long long)(n - a.mlog_cap));
    }
    if (threadIdx.x == 0 && lcur[MSA_MLOG_PARTS])  // misses dropped: this split is repeated
        atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_MLOG);
}

}  // namespace

// k_scan_struct: the record structure alone, no LDS, 256-thread workgroups at
// SA_MINW waves per SIMD; instead of counting it writes the lyric token-byte
// mask (ScanArgs::lmask) that k_scan_tokens counts.  (The fused pass of rounds
// 1-3 -- structure, tokens and LDS counting in one 1024-thread workgroup per CU
// -- was 0.25 ms/step slower and is gone.)
#ifndef SA_T
#define SA_T 256
#endif
#ifndef SA_MINW
#define SA_MINW 5
#endif
// k_scan_struct: the split scan's structure pass.  Each wave walks its
// blocks (the 4 KiB blocks of chunks gw, gw + nw, ...) with the input loaded
// SA_PF blocks ahead (1: the next block; 2: two blocks in flight -- one
// block's structure work alone did not cover the HBM latency at these wave
// counts).  Per block: byte classes, record structure (struct_block), and the
// lyric token-byte mask for k_scan_tokens.
#ifndef SA_PF
#define SA_PF 1
#endif
#ifndef SA_TAIL1
#define SA_TAIL1 0
#endif
#ifndef SA_LDS
#define SA_LDS 0  // 1: blocks loaded coalesced and transposed through the wave's LDS image (msa_k1.h blk_*)
#endif
__global__ __launch_bounds__(SA_T, SA_MINW) void k_scan_struct(ScanArgs a) {
    const u32 lane = lane_id();
    const u32 wib = threadIdx.x >> 6;
    const u32 gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (SA_T / 64) + wib);
    const u32 nw = gridDim.x * (SA_T / 64);
    if (gw >= a.nchunks) return;
    // block s of this wave: chunk gw + (s / 4) nw, block s % 4 of it (past the
    // segment end: no block -- its loads re-read the wave's first block)
    auto blk_at = [&](u32 s, u64 &ib) -> bool {
        const u32 c = gw + (s >> 2) * nw;
        ib = a.seg_begin + (u64)c * MSA_CHUNK + (u64)(s & 3u) * Q_BLK;
        return c < a.nchunks && ib < a.seg_end;
    };
    auto load_blk = [&](u32 s, uint4 (&v)[4], uint4 &t) {
        u64 ib;
        if (!blk_at(s, ib)) ib = a.seg_begin + (u64)gw * MSA_CHUNK;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ldg16(a.buf + ib + lane * 64 + 16 * q);
        // a vector load (a uniform address would become a scalar load, which
        // drops the low address bits -- a.buf is a view at any alignment)
        u64 ta = ib + Q_BLK < a.seg_end ? ib + Q_BLK : ib;
        pin64(ta);
#if SA_TAIL1
        // only lane 63 reads the bytes after the block (struct_block): one
        // active lane, not 64 copies of the same 16 bytes through the texture
        // data path (a fifth of the block's own bytes)
        t = make_uint4(0, 0, 0, 0);
        if (lane == 63) t = ldg16(a.buf + ta);
#else
        t = ldg16(a.buf + ta);
#endif
    };
#if SA_LDS
    static_assert(SA_PF == 1, "SA_LDS prefetches one block");
    __shared__ uint4 sast[SA_T / 64][256];
    uint4 *bst = sast[threadIdx.x >> 6];
    auto load_raw = [&](u32 s, Blk4 &r, uint4 &t) {
        u64 ib;
        if (!blk_at(s, ib)) ib = a.seg_begin + (u64)gw * MSA_CHUNK;
        r = blk_load_co(a.buf + ib);
        u64 ta = ib + Q_BLK < a.seg_end ? ib + Q_BLK : ib;
        pin64(ta);
#if SA_TAIL1
        t = make_uint4(0, 0, 0, 0);
        if (lane == 63) t = ldg16(a.buf + ta);
#else
        t = ldg16(a.buf + ta);
#endif
    };
    Blk4 raw;
    uint4 tl;
    load_raw(0, raw, tl);
#else
    uint4 cur[4], tl;
    load_blk(0, cur, tl);
#endif
#if SA_PF > 1
    uint4 nx[4], ntl;
    load_blk(1, nx, ntl);
#endif
    State st{};
    bool rare_chunk = true;
    u32 prevQ = 0;
    for (u32 s = 0;; ++s) {
        u64 ib;
        const bool valid = blk_at(s, ib);
        const u32 c = gw + (s >> 2) * nw;
        if (c >= a.nchunks) break;
        if ((s & 3u) == 0) {  // a chunk starts: its reader state and '"' before it
            st = sload_state(a.carry + c);
            rare_chunk = !a.sums || ((*sload(&a.sums[c].h[0]) >> 22) & 1u);
            prevQ = 0;
            if (ib > a.seg_begin) {
                const size_t pa = (size_t)(a.buf + ib - 1);
                const u32 b = (*sload(reinterpret_cast<const u32 *>(pa & ~(size_t)3)) >> (8 * (pa & 3))) & 0xFFu;
                prevQ = (u32)(b == '"');
            }
        }
        const uint4 tail = tl;
        const u64 cend = min(a.seg_begin + (u64)c * MSA_CHUNK + (u64)MSA_CHUNK, a.seg_end);
        const u64 lpos = ib + lane * 64;
        const u64 rem = valid && cend > lpos ? cend - lpos : 0;
#if SA_LDS
        uint4 cur[4];
        blk_transpose(bst, raw, cur);
        load_raw(s + 1, raw, tl);
        const Masks k = classify64x(cur, (u32)min(rem, (u64)64), rare_chunk);
#else
        const Masks k = classify64x(cur, (u32)min(rem, (u64)64), rare_chunk);
#endif
        // the block's bytes now live in the masks: rotate the prefetch
#if SA_LDS
#elif SA_PF > 1
#pragma unroll
        for (int q = 0; q < 4; ++q) cur[q] = nx[q];
        tl = ntl;
        load_blk(s + 2, nx, ntl);
#else
        load_blk(s + 1, cur, tl);
#endif
        if (!valid) continue;
        const u64 tpos = ib + Q_BLK;
        const u32 tvm = tpos < a.seg_end ? (a.seg_end - tpos >= 16 ? 0xFFFFu : (1u << (a.seg_end - tpos)) - 1u) : 0u;
        const u64 live = struct_block(a, st, k, tail, tvm, lpos, prevQ);
        prevQ = readlane((u32)(k.Q >> 63), 63);
        // the lyric token bytes (every lane of the block writes its word, past
        // the segment end too: zero)
        a.lmask[1 + ((ib - a.seg_begin) >> 6) + lane] = k.T & live;
    }
}

// ---------------------------------------------------------------------------
// k_scan_fold: K1 + K2 + k_scan_struct in one pass over the input.  A
// workgroup of FD_CH waves takes a tile of FD_CH consecutive chunks (a wave
// each) in ticket order and
//   A. classifies its chunk's four blocks once, keeping the byte-class masks
//      in registers, and builds the chunk's transfer function from them (K1's
//      k1_block over the same masks);
//   B. wave 0 composes the tile's function, publishes it, and looks back over
//      the earlier tiles' published functions / end states (decoupled
//      look-back, 64 tiles a round trip, a log-depth composition across the
//      wave) for the tile's entry state; it publishes the tile's end state
//      and hands every chunk its entry state through LDS;
//   C. every wave runs the record structure over its masks (struct_block)
//      and writes the token-byte mask, as k_scan_struct does.
// The input is read once (k_chunk_summary + k_scan_struct read it twice).
// Statuses are self-validating 64-bit words (epoch in bits 48-63, relaxed
// agent-scope atomics: no fence, no memset between launches): entries of the
// tile function pack nterm (17 bits), rs - tile start (17), p, cr, c, z; the
// end state packs rec (40) | p, cr, c, z and rs (48).
#define FD_CH 4
#define FD_T (FD_CH * 64)
#ifndef FD_MINW
#define FD_MINW 4
#endif
#define FD_SPIN_LIMIT (1u << 24)  // polls before a look-back gives up (error, never a hang)

__device__ __forceinline__ u64 fd_ld(const u64 *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void fd_st(u64 *p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ u64 fd_pack_ent(const FnEnt &e, u64 tb, u64 ep) {
    return e.nterm | ((e.rs - tb) << 17) | ((u64)e.p << 34) | ((u64)e.cr << 35) | ((u64)e.c << 36) |
           ((u64)e.z << 38) | (ep << 48);
}
__device__ __forceinline__ u64 fd_pack_rec(const State &s, u64 ep) {
    return s.rec | ((u64)s.p << 40) | ((u64)s.cr << 41) | ((u64)s.c << 42) | ((u64)s.z << 44) | (ep << 48);
}
__device__ __forceinline__ State fd_unpack_state(u64 wa, u64 wb) {
    State s;
    s.rec = wa & ((1ull << 40) - 1ull);
    s.p = (u32)(wa >> 40) & 1u;
    s.cr = (u32)(wa >> 41) & 1u;
    s.c = (u32)(wa >> 42) & 3u;
    s.z = (u32)(wa >> 44) & 1u;
    s.rs = wb & ((1ull << 48) - 1ull);
    return s;
}
// The look-back's functions in registers: three named entries (no array --
// an entry picked by (p, cr) out of an array is a dynamic index, i.e. scratch
// memory), picked by masks.  fl = p | cr << 1 | c << 3 | z << 5; has = nt != 0.
struct LEnt {
    u64 nt, rs;
    u32 fl;
};
struct LFn {
    LEnt e0, e1, e2;
};
__device__ __forceinline__ LEnt le_unpack(u64 w, u64 tb) {
    LEnt e;
    e.nt = w & 0x1FFFFull;
    e.rs = tb + ((w >> 17) & 0x1FFFFull);
    e.fl = ((u32)(w >> 34) & 3u) | (((u32)(w >> 36) & 7u) << 3);
    return e;
}
__device__ __forceinline__ LEnt le_identity(u32 idx) {
    LEnt e;
    e.nt = 0;
    e.rs = 0;
    e.fl = idx == 1 ? 1u : (idx == 2 ? 2u : 0u);
    return e;
}
__device__ __forceinline__ LFn lf_identity() { return LFn{le_identity(0), le_identity(1), le_identity(2)}; }
__device__ __forceinline__ LEnt le_pick(const LFn &g, u32 p, u32 cr) {
    const u64 m2 = cr ? ~0ull : 0ull, m1 = (!cr && p) ? ~0ull : 0ull, m0 = ~(m1 | m2);
    LEnt r;
    r.nt = (g.e0.nt & m0) | (g.e1.nt & m1) | (g.e2.nt & m2);
    r.rs = (g.e0.rs & m0) | (g.e1.rs & m1) | (g.e2.rs & m2);
    r.fl = (g.e0.fl & (u32)m0) | (g.e1.fl & (u32)m1) | (g.e2.fl & (u32)m2);
    return r;
}
// fn_then (msa_internal.h) on LEnt
__device__ __forceinline__ LEnt le_then(const LEnt &a, const LFn &g) {
    const LEnt b = le_pick(g, a.fl & 1u, (a.fl >> 1) & 1u);
    LEnt r;
    r.nt = a.nt + b.nt;
    if (b.nt) {
        r.fl = b.fl;
        r.rs = b.rs;
    } else {
        const u32 c = min(((a.fl >> 3) & 3u) + ((b.fl >> 3) & 3u), 3u);
        r.fl = (b.fl & 3u) | (c << 3) | ((a.fl | b.fl) & 32u);
        r.rs = a.rs;
    }
    return r;
}
__device__ __forceinline__ LFn lf_compose(const LFn &f, const LFn &g) {  // f then g
    return LFn{le_then(f.e0, g), le_then(f.e1, g), le_then(f.e2, g)};
}
// fn_apply (msa_internal.h) on LFn
__device__ __forceinline__ State lf_apply(const State &s, const LFn &f) {
    const LEnt b = le_pick(f, s.p, s.cr);
    State r;
    r.p = b.fl & 1u;
    r.cr = (b.fl >> 1) & 1u;
    r.rec = s.rec + b.nt;
    if (b.nt) {
        r.c = (b.fl >> 3) & 3u;
        r.z = (b.fl >> 5) & 1u;
        r.rs = b.rs;
    } else {
        r.c = min(s.c + ((b.fl >> 3) & 3u), 3u);
        r.z = s.z | ((b.fl >> 5) & 1u);
        r.rs = s.rs;
    }
    return r;
}
__device__ __forceinline__ LEnt le_shfl_up(const LEnt &e, u32 d) {
    return LEnt{__shfl_up(e.nt, d), __shfl_up(e.rs, d), __shfl_up(e.fl, d)};
}
__device__ __forceinline__ LEnt le_readlane(const LEnt &e, int l) {
    return LEnt{readlane64(e.nt, l), readlane64(e.rs, l), readlane(e.fl, l)};
}
__device__ __forceinline__ LFn lf_readlane(const LFn &f, int l) {
    return LFn{le_readlane(f.e0, l), le_readlane(f.e1, l), le_readlane(f.e2, l)};
}
__device__ __forceinline__ State fd_uniform(const State &s) {
    State r;
    r.rec = readlane64(s.rec, 0);
    r.rs = readlane64(s.rs, 0);
    r.p = readlane(s.p, 0);
    r.cr = readlane(s.cr, 0);
    r.c = readlane(s.c, 0);
    r.z = readlane(s.z, 0);
    return r;
}

// The entry state of tile `tile` (> 0), by wave 0: 64 earlier tiles' statuses
// a round trip (lane l: tile j0 - l).  The nearest published end state
// (lane k) with every tile after it published at least as a function: that
// state pushed through lanes k-1 .. 0 (H_{k-1} = F_{k-1} then ... then F_0,
// an inclusive scan across the lanes) and through the compositions of the
// newer windows (acc).  A window without an end state is composed whole and
// the look-back moves 64 tiles further.
__device__ __forceinline__ State fd_lookback(const ScanArgs &a, u32 tile, u64 ep) {
    const u32 lane = lane_id();
    const u64 *W0 = a.fold_stat, *W1 = W0 + a.fold_n, *W2 = W1 + a.fold_n, *W3 = W2 + a.fold_n,
              *W4 = W3 + a.fold_n;
    const u64 tile_bytes = (u64)FD_CH * MSA_CHUNK;
    LFn acc = lf_identity();
    bool have_acc = false;
    long long j0 = (long long)tile - 1;
    u32 spins = 0;
    for (;;) {
        const long long t = j0 - (long long)lane;
        u64 w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0;
        if (t >= 0) {
            w3 = fd_ld(W3 + t);
            w4 = fd_ld(W4 + t);
            w0 = fd_ld(W0 + t);
            w1 = fd_ld(W1 + t);
            w2 = fd_ld(W2 + t);
        }
        const bool inc = (w3 >> 48) == ep && (w4 >> 48) == ep;
        const bool agg = (w0 >> 48) == ep && (w1 >> 48) == ep && (w2 >> 48) == ep;
        const u64 Bin = __ballot(t >= 0), Binc = __ballot(t >= 0 && inc), Bok = __ballot(t >= 0 && (inc || agg));
        const u32 k = Binc ? (u32)__ffsll((long long)Binc) - 1u : 64u;
        const u64 need = Binc ? bits_lo(k) : Bin;
        if ((Bok & need) != need) {  // a tile in between has not published yet
            if (++spins > FD_SPIN_LIMIT) {
                if (lane == 0) atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_FOLD);
                return a.fold_init;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        const u32 nl = Binc ? k : (u32)__popcll(Bin);
        const u64 tb = a.seg_begin + (u64)(t >= 0 ? t : 0) * tile_bytes;
        LFn F = lf_identity();
        if (lane < nl) F = LFn{le_unpack(w0, tb), le_unpack(w1, tb), le_unpack(w2, tb)};
        for (u32 d = 1; d < nl; d <<= 1) {  // X_l = X_l then X_{l-d} (older first)
            const LFn Y{le_shfl_up(F.e0, d), le_shfl_up(F.e1, d), le_shfl_up(F.e2, d)};
            if (lane >= d) F = lf_compose(F, Y);
        }
        if (Binc) {
            State S = fd_unpack_state(readlane64(w3, (int)k), readlane64(w4, (int)k));
            if (k) S = lf_apply(S, lf_readlane(F, (int)k - 1));
            if (have_acc) S = lf_apply(S, acc);
            return S;
        }
        const LFn Wn = lf_readlane(F, (int)nl - 1);
        acc = have_acc ? lf_compose(Wn, acc) : Wn;
        have_acc = true;
        j0 -= 64;
    }
}

__global__ __launch_bounds__(FD_T, FD_MINW) void k_scan_fold(ScanArgs a) {
    __shared__ Fn s_fn[FD_CH];
    __shared__ State s_st[FD_CH];
    __shared__ u32 s_tile;
    const u32 lane = lane_id();
    const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u32 ntiles = (a.nchunks + FD_CH - 1) / FD_CH;
    const u64 ep = a.fold_ep;
    // a chunk's block j and the 16 bytes after it (no block: the chunk's first
    // block again, which exists)
    auto load_blk = [&](u64 cbase, u64 cend, u32 j, uint4 (&v)[4], uint4 &t) {
        u64 ib = cbase + (u64)j * Q_BLK;
        if (ib >= cend) ib = cbase;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ldg16(a.buf + ib + lane * 64 + 16 * q);
        u64 ta = ib + Q_BLK < a.seg_end ? ib + Q_BLK : ib;
        pin64(ta);
        t = ldg16(a.buf + ta);
    };
    // (measured: taking the next tile's ticket during the look-back, to load its
    // first block while this tile's structure runs, made the kernel 1.37 ms
    // instead of 0.85 -- tiles then start a whole phase after their tickets and
    // their successors' look-backs wait for them)
    for (;;) {
        if (threadIdx.x == 0) {
            const u64 tk = atomicAdd((unsigned long long *)a.fold_ticket, 1ull) - a.fold_tbase;
            s_tile = (u32)min(tk, (u64)ntiles);
        }
        __syncthreads();
        const u32 tile = __builtin_amdgcn_readfirstlane(s_tile);
        if (tile >= ntiles) break;
        const u32 c = tile * FD_CH + wib;
        const bool has = c < a.nchunks;
        const u64 cbase = a.seg_begin + (u64)c * MSA_CHUNK;
        const u64 cend = has ? min(cbase + (u64)MSA_CHUNK, a.seg_end) : cbase;
        // ---- A: the chunk's byte classes (kept) and its transfer function
        Masks m[4];
        u32 tb[4];  // the byte after each block | (it exists) << 8
        Fn g = fn_identity(cbase);
        if (has) {
            K1Acc acc;
            k1_init(acc);
            uint4 v[4], t;
            load_blk(cbase, cend, 0, v, t);
#pragma unroll
            for (u32 j = 0; j < 4; ++j) {
                const u64 ib = cbase + (u64)j * Q_BLK;
                const bool valid = ib < cend;
                uint4 cv[4] = {v[0], v[1], v[2], v[3]};
                const uint4 ct = t;
                if (j + 1 < 4) load_blk(cbase, cend, j + 1, v, t);
                const u64 lpos = ib + lane * 64;
                const u64 rem = valid && cend > lpos ? cend - lpos : 0;
                m[j] = classify64x(cv, (u32)min(rem, (u64)64), true);
                const u32 tex = ib + Q_BLK < a.seg_end ? 1u : 0u;
                tb[j] = (ct.x & 0xFFu) | (tex << 8);
                if (valid) {
                    const u32 nb_nl = (tex && (ct.x & 0xFFu) == '\n') ? 1u : 0u;
                    const u32 lastb = (u32)(min(ib + (u64)Q_BLK, cend) - 1 - ib);
                    k1_block(acc, m[j].Q, m[j].C, m[j].NL, m[j].CR, m[j].Z, false, nb_nl, j * Q_BLK, lastb);
                }
            }
            const ChunkSum cs = k1_finish(acc);
#pragma unroll
            for (u32 i = 0; i < 3; ++i) g.e[i] = chunk_entry(cs, cbase, i);
        }
        if (lane == 0) s_fn[wib] = g;
        __syncthreads();
        // ---- B: the tile's function published, its entry state looked up
        if (wib == 0) {
            // (the functions stay in LDS: a local copy of an Fn is an array the
            // entry selects index, i.e. scratch memory)
            const u64 tbase = a.seg_begin + (u64)tile * FD_CH * MSA_CHUNK;
            State S;
            if (tile == 0) {
                S = a.fold_init;
            } else {
                u64 pk[3];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const FnEnt e = fn_then(fn_then(fn_then(s_fn[0].e[i], s_fn[1]), s_fn[2]), s_fn[3]);
                    pk[i] = fd_pack_ent(e, tbase, ep);
                }
                if (lane < 3) fd_st(a.fold_stat + (u64)lane * a.fold_n + tile, lane == 0 ? pk[0] : (lane == 1 ? pk[1] : pk[2]));
                S = fd_uniform(fd_lookback(a, tile, ep));
            }
            const State s1 = fn_apply(S, s_fn[0]), s2 = fn_apply(s1, s_fn[1]), s3 = fn_apply(s2, s_fn[2]),
                        E = fn_apply(s3, s_fn[3]);
            const u64 wa = fd_pack_rec(E, ep), wb = E.rs | (ep << 48);
            if (lane < 2) fd_st(a.fold_stat + (u64)(3 + lane) * a.fold_n + tile, lane == 0 ? wa : wb);
            if (lane == 0) {
                s_st[0] = S;
                s_st[1] = s1;
                s_st[2] = s2;
                s_st[3] = s3;
                if (tile + 1 == ntiles) {
                    *a.fold_fin = E;
                    if (a.fold_fin_host) *a.fold_fin_host = E;
                }
            }
        }
        __syncthreads();
        // ---- C: the record structure of the chunk from its masks
        if (has) {
            State st = fd_uniform(s_st[wib]);
            u32 prevQ = 0;
            if (cbase > a.seg_begin) {
                const size_t pa = (size_t)(a.buf + cbase - 1);
                const u32 b = (*sload(reinterpret_cast<const u32 *>(pa & ~(size_t)3)) >> (8 * (pa & 3))) & 0xFFu;
                prevQ = (u32)(b == '"');
            }
#pragma unroll
            for (u32 j = 0; j < 4; ++j) {
                const u64 ib = cbase + (u64)j * Q_BLK;
                if (ib < cend) {
                    const u64 lpos = ib + lane * 64;
                    const u64 live = struct_block(a, st, m[j], make_uint4(tb[j] & 0xFFu, 0, 0, 0), tb[j] >> 8, lpos, prevQ);
                    prevQ = readlane((u32)(m[j].Q >> 63), 63);
                    a.lmask[1 + ((ib - a.seg_begin) >> 6) + lane] = m[j].T & live;
                }
            }
        }
    }
}

// k_scan_tokens: the token phase of the split scan over k_scan_struct's
// lmask -- no reader state, no byte classes: a wave per 4 KiB block (grid
// stride), token starts and lengths from the mask, keys re-read from the
// input, counted in the workgroup's LDS table.  The next
// block's mask words and one 16-byte load per lane of its bytes (the keys'
// cache lines) are in flight while a block is counted.  (Measured and
// removed: the token lists software-pipelined across blocks, the next
// block's list built before the current block's last batch is probed --
// 1.02 vs 0.81 ms.)
__global__ __launch_bounds__(Q_T, Q_WGCU) void k_scan_tokens(ScanArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    u64 *skeys = reinterpret_cast<u64 *>(smem);
    u32 *scnts = reinterpret_cast<u32 *>(smem + Q_SSLOTS * 8);
    const u32 lane = lane_id();
    const u32 wib = threadIdx.x >> 6;
    unsigned char *wl = smem + Q_TAB + wib * Q_WLDS;
    u16 *list = reinterpret_cast<u16 *>(wl);
    u32 *lcur = reinterpret_cast<u32 *>(smem + Q_TAB + Q_W * Q_WLDS);
    for (u32 i = threadIdx.x; i < Q_SSLOTS; i += Q_T) {
        skeys[i] = 0;
        scnts[i] = 0;
    }
    if (threadIdx.x < MSA_MLOG_PARTS + 1) lcur[threadIdx.x] = 0;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rsrc = mlog_rsrc(a);

    const u64 nblk = (a.seg_end - a.seg_begin + Q_BLK - 1) / Q_BLK;
    const u64 nwords = nblk * 64;  // k_scan_struct writes every lane's word of every block
    const u32 gw = __builtin_amdgcn_readfirstlane(blockIdx.x * Q_W + wib);
    const u32 nw = gridDim.x * Q_W;
    u64 words = 0;
    // this wave's range of l_pos; ranges of ~a quarter of an even share of the
    // occurrences expected (the capacity when none are), 8..1024 -- a floor of
    // 64 had let ~1 K waves with one long word each reserve a 64 K-slot
    // capacity whole (OVF_L and a repeated split for a few long words); unused
    // range slots are walked by k_long_insert, so ranges follow the expected
    // occurrences, not the (generous) capacity
    u64 lres = 0, lend = 0;
    const u64 lch = min<u64>(1024, max<u64>(8, min(a.l_expect ? a.l_expect : a.l_cap, a.l_cap) / ((u64)nw * 4)));
    // mask words of the block: this lane's, the one after it and the one before
    u64 Lc = 0, Ln = 0, Lp = 0;
#if Q_TDL
    // the neighbours' mask words by DPP from the lane's own (only the block's
    // two edge words loaded, by one lane each); the lines warmed by one dword
    // a lane, not 16 bytes
    u32 warm = 0;
    u64 Le = 0;  // lane 0: the word before the block; lane 63: the word after it
    auto fetch = [&](u64 blk) {
        u64 wi = blk * 64 + lane;
        pin64(wi);
        Lc = a.lmask[1 + wi];
        if (lane == 0) Le = a.lmask[wi];  // lmask[0] is the zero pad
        else if (lane == 63) Le = wi + 1 < nwords ? a.lmask[2 + wi] : 0ull;
        warm = *reinterpret_cast<const u32 *>(a.buf + ((a.seg_begin + blk * Q_BLK + lane * 64) & ~3ull));
    };
#else
    uint4 warm = make_uint4(0, 0, 0, 0);
    auto fetch = [&](u64 blk) {
        u64 wi = blk * 64 + lane;
        pin64(wi);
        Lc = a.lmask[1 + wi];
        Ln = wi + 1 < nwords ? a.lmask[2 + wi] : 0ull;
        Lp = a.lmask[wi];  // lmask[0] is the zero pad
        warm = ldg16(a.buf + a.seg_begin + blk * Q_BLK + lane * 64);
    };
#endif
    if (gw < nblk) fetch(gw);
    for (u64 blk = gw; blk < nblk; blk += nw) {
#if Q_TDL
        const u64 L = Lc, Le_ = Le;
        const u64 dn = from_next(L), dp = from_prev(L);
        const u64 Lnext = lane == 63 ? Le_ : dn, Lprev = lane == 0 ? Le_ : dp;
        asm volatile("" ::"v"(warm));  // the block's lines are in cache
#else
        const u64 L = Lc, Lnext = Ln, Lprev = Lp;
        asm volatile("" ::"v"(warm.x));  // the block's lines are in cache
#endif
        if (blk + nw < nblk) fetch(blk + nw);
        const u64 ib = a.seg_begin + blk * Q_BLK;
        const u64 lpos = ib + lane * 64;
        const u64 S0 = L & ~((L << 1) | (Lprev >> 63));
        tok_phase(a, ib, lpos, L, Lnext, S0, skeys, scnts, list, lcur, words, rsrc, lres, lend, lch);
    }
    lpos_fill(a, lres, lend);
    tok_epilogue(a, skeys, scnts, lcur, words);
}

// k_miss_agg: workgroup (partition p, group g) counts partition p of the
// logs of K3 workgroups g, g + G, ... in an LDS table (the whole LDS: ~8000
// 16-byte keys), then adds each distinct key once to the HBM tables.
#ifndef MA_T
#define MA_T 1024
#endif
#ifndef MA_SLOTS
#define MA_SLOTS 8176
#endif
#ifndef MA_FLY
#define MA_FLY 4  // log entries in flight per thread
#endif
#define MA_NB (MA_SLOTS / 4)
__device__ __forceinline__ u32 ma_hash(u64 k0, u64 k1) {
    u32 h = (u32)k0 * 0x9E3779B1u + (u32)(k0 >> 32) * 0x85EBCA77u + (u32)k1 * 0xC2B2AE3Du + (u32)(k1 >> 32);
    h ^= h >> 15;
    return h * 0x2C1B3C6Du;
}
// PROBES buckets of 4 slots are tried (k_miss_agg: 2, then the HBM table;
// the dense aggregation: 16, its table a third full at configs[4] -- two
// buckets left ~1 in 300 keys without a slot there)
template <int PROBES = 2>
__device__ __forceinline__ u32 ma_find(ulonglong2 *keys, u64 k0, u64 k1) {
    const u32 h = ma_hash(k0, k1);
    u32 b = __umulhi(h, (u32)MA_NB);
    // the four slot reads start at a key-dependent slot: a ds_read_b128 lane
    // group spreads over 16 positions of the bank row, not 4 (measured: the
    // aggregation 0.22 -> 0.19 ms; in K3's table it did not pay)
    const u32 ro = h & 3u;
    for (int p = 0; p < PROBES; ++p) {
        const u32 base = b * 4;
        const ulonglong2 s0 = keys[base + (ro & 3u)], s1 = keys[base + ((ro + 1) & 3u)];
        const ulonglong2 s2 = keys[base + ((ro + 2) & 3u)], s3 = keys[base + ((ro + 3) & 3u)];
        const bool e0 = (s0.x == k0) & (s0.y == k1), e1 = (s1.x == k0) & (s1.y == k1);
        const bool e2 = (s2.x == k0) & (s2.y == k1), e3 = (s3.x == k0) & (s3.y == k1);
        const u32 hit = e0 ? 0u : (e1 ? 1u : (e2 ? 2u : (e3 ? 3u : 4u)));
        if (hit < 4) return base + ((ro + hit) & 3u);
        // a slot is claimed word by word, each by a CAS: the first word by the
        // key's first 8 bytes, the second by the rest -- lanes of one key that
        // meet a slot whose second word is not written yet write the same
        // value, so a key never takes two slots (a plain store of the second
        // word had let them move on and claim another)
#pragma unroll
        for (u32 i = 0; i < 4; ++i) {
            const ulonglong2 sn = i == 0 ? s0 : (i == 1 ? s1 : (i == 2 ? s2 : s3));
            if ((sn.x != 0 && sn.x != k0) || (sn.y != 0 && sn.y != k1)) continue;  // another key's
            const u32 sl = base + ((ro + i) & 3u);
            u64 *kp = reinterpret_cast<u64 *>(&keys[sl]);
            u64 w0 = sn.x;
            if (w0 == 0) {
                const u64 o = atomicCAS((unsigned long long *)kp, 0ull, (unsigned long long)k0);
                w0 = o == 0 ? k0 : o;
            }
            if (w0 != k0) continue;
            u64 w1 = sn.y;
            if (w1 == 0) {
                const u64 o = atomicCAS((unsigned long long *)(kp + 1), 0ull, (unsigned long long)k1);
                w1 = o == 0 ? k1 : o;
            }
            if (w1 == k1) return sl;
        }
        b = (b + 1 == MA_NB) ? 0 : b + 1;
    }
    return ~0u;
}
#ifndef MA_FLAT
#define MA_FLAT 1  // 0: one source log at a time, no load pipelining (A/B)
#endif
#ifndef MA_DIAG
#define MA_DIAG 0  // timing diagnostics only, results wrong (profiles/r06_ab_miss_agg.txt): 1 no flush,
                   // 2 LDS-full entries dropped, 4 plain adds, 8 no probe (hash slot), 32 a slot per thread
#endif
#ifndef MA_PB
#define MA_PB 0  // 1: the batch's bucket reads issued together before the first count (MA_FLAT)
#endif
__device__ __forceinline__ void ma_count(const ScanArgs &a, ulonglong2 *keys, u32 *cnts, ulonglong2 x) {
    const u32 c = gather8(x.x) | ((gather8(x.y) & 0x7Fu) << 8);
    const u64 k0 = x.x & MLOG_KEYBITS, k1 = x.y & (MLOG_KEYBITS | KMARK);
#if MA_DIAG & 32
    const u32 slot = threadIdx.x;  // timing diagnostic: no probe, no two lanes on one slot
#elif MA_DIAG & 8
    const u32 slot = ma_hash(k0, k1) % MA_SLOTS;  // timing diagnostic: no probe
#else
    const u32 slot = ma_find(keys, k0, k1);
#endif
#if MA_DIAG & 4
    if (slot != ~0u) cnts[slot] += c ? c : 1u;  // timing diagnostic: plain add (races)
#else
    if (slot != ~0u) atomicAdd(&cnts[slot], c ? c : 1u);
#endif
#if MA_DIAG & 2
    else {}  // timing diagnostic: dropped
#else
    else hbm_insert16<false>(a, k0, k1, c ? c : 1u);  // table full: one insert per entry
#endif
}
__global__ __launch_bounds__(MA_T) void k_miss_agg(ScanArgs a, u32 nsrc, u32 groups) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ulonglong2 *keys = reinterpret_cast<ulonglong2 *>(smem);
    u32 *cnts = reinterpret_cast<u32 *>(smem + MA_SLOTS * 16);
    for (u32 i = threadIdx.x; i < MA_SLOTS; i += MA_T) {
        keys[i] = make_ulonglong2(0, 0);
        cnts[i] = 0;
    }
    __syncthreads();
    const u32 part = blockIdx.x % MSA_MLOG_PARTS, g = blockIdx.x / MSA_MLOG_PARTS;
#if MA_FLAT
    // The workgroup's source logs (K3 workgroups g, g + G, ...) as ONE stream
    // per thread, 64 sources at a time: a thread's entries are i = t, t + T, ...
    // of each log in turn, so every batch is full (one log at a time had left
    // a partial batch per log: ~32 batches per thread instead of ~22), and the
    // next batch's loads are in flight while this one is counted.
    __shared__ u32 sn[64];
    for (u32 c0 = 0; g + c0 * groups < nsrc; c0 += 64) {
        __syncthreads();  // the previous chunk's readers of sn are done
        if (threadIdx.x < 64) {
            const u32 src = g + (c0 + threadIdx.x) * groups;
            const u32 n = src < nsrc ? a.mlog_n[src * MSA_MLOG_PARTS + part] : 0u;
            sn[threadIdx.x] = n;
            u64 tot = n;
            for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
            if (threadIdx.x == 0 && tot) atomicAdd((unsigned long long *)&a.ctr->k3_misses, (unsigned long long)tot);
        }
        __syncthreads();
        u32 k = 0, i = threadIdx.x;
        while (k < 64 && i >= sn[k]) { ++k; i = threadIdx.x; }
        auto fetch = [&](ulonglong2 (&x)[MA_FLY], u32 &nx) {
            nx = 0;
#pragma unroll
            for (int q = 0; q < MA_FLY; ++q) {
                if (k < 64) {
                    const u64 src = g + (c0 + k) * groups;
                    x[q] = a.mlog[(src * MSA_MLOG_PARTS + part) * a.mlog_cap + i];
                    ++nx;
                    i += MA_T;
                    while (k < 64 && i >= sn[k]) { ++k; i = threadIdx.x; }
                }
            }
        };
        ulonglong2 cur[MA_FLY], nxt[MA_FLY];
        u32 ncur, nnxt;
        fetch(cur, ncur);
        while (ncur) {
            fetch(nxt, nnxt);
#if MA_PB
            // the batch's first bucket reads together (stale reads are safe:
            // a hit is an exact key match, a slot that looked free goes through
            // ma_find's CAS claim)
            ulonglong2 sl[MA_FLY][4];
            u32 bs[MA_FLY];
#pragma unroll
            for (int q = 0; q < MA_FLY; ++q) {
                if ((u32)q < ncur) {
                    const u64 k0 = cur[q].x & MLOG_KEYBITS, k1 = cur[q].y & (MLOG_KEYBITS | KMARK);
                    const u32 h = ma_hash(k0, k1);
                    bs[q] = __umulhi(h, (u32)MA_NB) * 4;
#pragma unroll
                    for (int j = 0; j < 4; ++j) sl[q][j] = keys[bs[q] + j];
                }
            }
#pragma unroll
            for (int q = 0; q < MA_FLY; ++q) {
                if ((u32)q >= ncur) break;
                const ulonglong2 x = cur[q];
                const u64 k0 = x.x & MLOG_KEYBITS, k1 = x.y & (MLOG_KEYBITS | KMARK);
                u32 hit = 4;
#pragma unroll
                for (int j = 3; j >= 0; --j)
                    if (sl[q][j].x == k0 && sl[q][j].y == k1) hit = (u32)j;
                if (hit < 4) {
                    const u32 c = gather8(x.x) | ((gather8(x.y) & 0x7Fu) << 8);
                    atomicAdd(&cnts[bs[q] + hit], c ? c : 1u);
                } else {
                    ma_count(a, keys, cnts, x);
                }
            }
#else
#pragma unroll
            for (int q = 0; q < MA_FLY; ++q)
                if ((u32)q < ncur) ma_count(a, keys, cnts, cur[q]);
#endif
#pragma unroll
            for (int q = 0; q < MA_FLY; ++q) cur[q] = nxt[q];
            ncur = nnxt;
        }
    }
#else
    for (u32 src = g; src < nsrc; src += groups) {
        const u64 base = ((u64)src * MSA_MLOG_PARTS + part) * a.mlog_cap;
        const u32 n = a.mlog_n[src * MSA_MLOG_PARTS + part];
        if (threadIdx.x == 0 && n) atomicAdd((unsigned long long *)&a.ctr->k3_misses, (unsigned long long)n);
        // four entries per thread in flight: their loads are issued before
        // the first LDS probe
        for (u32 i0 = threadIdx.x; i0 < n; i0 += MA_FLY * MA_T) {
            ulonglong2 xs[MA_FLY];
#pragma unroll
            for (int q = 0; q < MA_FLY; ++q) {
                const u32 i = i0 + q * MA_T;
                xs[q] = i < n ? a.mlog[base + i] : make_ulonglong2(0, 0);
            }
#pragma unroll
            for (int q = 0; q < MA_FLY; ++q) {
                if (i0 + q * MA_T >= n) break;
                ma_count(a, keys, cnts, xs[q]);
            }
        }
    }
#endif
    __syncthreads();
#if !(MA_DIAG & 1)
    for (u32 i = threadIdx.x; i < MA_SLOTS; i += MA_T) {
        const u32 c = cnts[i];
        if (c) {
            const ulonglong2 kk = keys[i];
            hbm_insert16(a, kk.x, kk.y, c);
        }
    }
#endif
}

// ---------------------------------------------------------------------------
// High-cardinality aggregation (configs[4]: 70 M logged misses, 50 M distinct
// keys).  k_miss_agg's LDS table fills after ~8 K keys per workgroup and then
// every further entry is one HBM insert (probe + claim + count: ~2 memory-side
// atomics per entry, 6.5 ms).  Here the logs are first bucketed by a second
// key hash -- MB_B buckets per partition, small enough that a bucket's
// distinct keys fit one workgroup's LDS table -- with a counting sort
// (k_mb_hist: per-tile bucket counts, bucket-major; one exclusive scan;
// k_mb_scatter).  k_mb_agg then counts each bucket in LDS and inserts each
// distinct key once, claim first (CAS) and count (no-return add), with no
// load-first probe.  The count stays an atomic add: the LDS table can hold a
// key twice (a prober that meets a slot claimed but not yet keyed moves on)
// and an entry that finds the LDS table full takes the atomic insert -- a
// plain count store lost those adds (caught by test_gpu_miss_buckets).
// Opt-in (MSA_MISS_BUCKETS=1): slower than k_miss_agg at both configs[2] and
// configs[4] (msa_ctx::mb_mode).
#define MB_B 1024u       // buckets per partition
#define MB_TT 512u       // threads per tile
#define MB_TILE 8192u    // log entries per tile
__device__ __forceinline__ u32 mb_bucket(u64 k0, u64 k1m) {
    u64 h = (k0 & MLOG_KEYBITS) * 0x9E3779B97F4A7C15ull ^ (k1m & (MLOG_KEYBITS | KMARK)) * 0xC2B2AE3D27D4EB4Full;
    h ^= h >> 29;
    return (u32)(h >> 40) & (MB_B - 1);  // independent of mlog_part's bits (low 32 of a different mix)
}
// tile (part p, source s, chunk c) = entries [c MB_TILE, (c + 1) MB_TILE) of log (s, p);
// t = s * chunks + c; hist[(p * MB_B + b) * T + t]
// XCD-aware tile order: workgroup w runs on XCD w % 8, so the tiles t that
// share a line of hist (and of the scatter's offsets and output runs) are
// given to workgroups of one XCD -- the hist lines are then merged in that
// XCD's L2 instead of written partially from eight (T a multiple of 8; else
// the identity)
__device__ __forceinline__ u32 mb_tile(u32 x, u32 T) {
#ifdef MB_NOXCD  // (A/B builds)
    return x;
#endif
    return (T & 7u) ? x : (x & 7u) * (T >> 3) + (x >> 3);
}
__global__ __launch_bounds__(MB_TT) void k_mb_hist(ScanArgs a, u32 chunks, u32 T, u64 *__restrict__ hist) {
    __shared__ u32 h[MB_B];
    const u32 p = blockIdx.y, t = mb_tile(blockIdx.x, T), src = t / chunks, c = t % chunks;
    for (u32 k = threadIdx.x; k < MB_B; k += MB_TT) h[k] = 0;
    __syncthreads();
    const u32 n = a.mlog_n[src * MSA_MLOG_PARTS + p];
    if (c == 0 && threadIdx.x == 0 && n) atomicAdd((unsigned long long *)&a.ctr->k3_misses, (unsigned long long)n);
    const u32 lo = c * MB_TILE, hi = min(n, lo + MB_TILE);
    const u64 base = ((u64)src * MSA_MLOG_PARTS + p) * a.mlog_cap;
    for (u32 i = lo + threadIdx.x; i < hi; i += MB_TT) {
        const ulonglong2 x = a.mlog[base + i];
        atomicAdd(&h[mb_bucket(x.x, x.y)], 1u);
    }
    __syncthreads();
    for (u32 k = threadIdx.x; k < MB_B; k += MB_TT) hist[((u64)p * MB_B + k) * T + t] = h[k];
}
// The tile sorted by bucket in LDS (counting sort), then written bucket run by
// bucket run with consecutive lanes on consecutive entries (a scattered
// 16-byte store per entry had taken 2.0 ms at configs[4]).  LDS: the staged
// tile (MB_TILE x 16 B), its bucket ids (MB_TILE x 2 B), the bucket counts and
// offsets (later overlaid by each bucket's output base).
#define MS_PER (MB_TILE / MB_TT)
#define MS_LDS (MB_TILE * 18u + MB_B * 8u)
__global__ __launch_bounds__(MB_TT) void k_mb_scatter(ScanArgs a, u32 chunks, u32 T, const u64 *__restrict__ off,
                                                      ulonglong2 *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ulonglong2 *stage = reinterpret_cast<ulonglong2 *>(smem);
    u16 *bid = reinterpret_cast<u16 *>(smem + MB_TILE * 16u);
    u32 *cnt = reinterpret_cast<u32 *>(smem + MB_TILE * 18u);
    u32 *loff = cnt + MB_B;
    u64 *gdel = reinterpret_cast<u64 *>(cnt);  // (after the staging) bucket b's output index - loff[b]
    __shared__ u32 wsum[MB_TT / 64];
    const u32 p = blockIdx.y, t = mb_tile(blockIdx.x, T), src = t / chunks, c = t % chunks;
    const u32 n = a.mlog_n[src * MSA_MLOG_PARTS + p];
    const u32 lo = c * MB_TILE, hi = min(n, lo + MB_TILE);
    if (lo >= hi) return;  // whole workgroup
    const u32 m = hi - lo, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    for (u32 k = tid; k < MB_B; k += MB_TT) cnt[k] = 0;
    __syncthreads();
    const u64 base = ((u64)src * MSA_MLOG_PARTS + p) * a.mlog_cap + lo;
    ulonglong2 x[MS_PER];
    u32 bk[MS_PER], r[MS_PER];
#pragma unroll
    for (u32 q = 0; q < MS_PER; ++q) {
        const u32 i = tid + q * MB_TT;
        x[q] = i < m ? a.mlog[base + i] : make_ulonglong2(0, 0);
    }
#pragma unroll
    for (u32 q = 0; q < MS_PER; ++q) {
        bk[q] = mb_bucket(x[q].x, x[q].y);
        r[q] = tid + q * MB_TT < m ? atomicAdd(&cnt[bk[q]], 1u) : 0u;
    }
    __syncthreads();
    // exclusive scan of the 1024 counts (2 per thread)
    static_assert(MB_B == 2 * MB_TT, "two buckets per thread");
    const u32 c0 = cnt[2 * tid], c1 = cnt[2 * tid + 1];
    u32 wt;
    const u32 pre = wave_prefix<14>(c0 + c1, wt);  // <= MB_TILE per tile
    if (lane == 0) wsum[w] = wt;
    __syncthreads();
    u32 wb = 0;
    for (u32 v = 0; v < w; ++v) wb += wsum[v];
    const u32 l0 = wb + pre, l1 = l0 + c0;
    loff[2 * tid] = l0;
    loff[2 * tid + 1] = l1;
    __syncthreads();
#pragma unroll
    for (u32 q = 0; q < MS_PER; ++q) {
        if (tid + q * MB_TT >= m) continue;
        const u32 pos = loff[bk[q]] + r[q];
        stage[pos] = x[q];
        bid[pos] = (u16)bk[q];
    }
    __syncthreads();  // (every loff read is done before gdel overlays it)
    gdel[2 * tid] = off[((u64)p * MB_B + 2 * tid) * T + t] - l0;
    gdel[2 * tid + 1] = off[((u64)p * MB_B + 2 * tid + 1) * T + t] - l1;
    __syncthreads();
    for (u32 j = tid; j < m; j += MB_TT) out[gdel[bid[j]] + j] = stage[j];
}
// one claim per distinct key of a bucket (CAS first: most keys are new)
__device__ __forceinline__ void mb_insert_once(const ScanArgs &a, u64 k0, u64 k1m, u64 cnt) {
    if (k1m == KMARK) {
        u64 h = fmix64(k0) & a.s_mask, rest;
        const u64 claim = tab_claim(k0, cnt, &rest);
        for (u32 probe = 0; probe < MSA_MAX_PROBE; ++probe) {
            u64 *slot = a.s_tab + 2 * h;
            const u64 old = atomicCAS((unsigned long long *)slot, 0ull, (unsigned long long)claim);
            if (old == 0 || (old & TAB_KEY7) == k0) {
                const u64 add = old == 0 ? rest : cnt;
                if (add) atomicAdd((unsigned long long *)(slot + 1), (unsigned long long)add);
                return;
            }
            if (table_full(probe, a.ctr, OVF_S)) break;
            h = (h + 1) & a.s_mask;
        }
        atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_S);
        return;
    }
    const u64 k1 = k1m & ~KMARK;
    u64 h = fmix64(k0 ^ fmix64(k1)) & a.m_mask, rest;
    const u64 claim = tab_claim(k0, cnt, &rest);
    u32 probe = 0, spins = 0;
    while (probe < MSA_MAX_PROBE) {
        u64 *slot = a.m_tab + 4 * h;
        const u64 c0 = atomicCAS((unsigned long long *)slot, 0ull, (unsigned long long)claim);
        if (c0 == 0) {
            __hip_atomic_store(slot + 1, k1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (rest) atomicAdd((unsigned long long *)(slot + 2), (unsigned long long)rest);
            return;
        }
        if ((c0 & TAB_KEY7) == k0) {
            const u64 c1 = __hip_atomic_load(slot + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c1 == 0) {  // claimed, k1 not yet visible: retry this slot
                if (++spins > (1u << 24)) break;
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            if (c1 == k1) {
                atomicAdd((unsigned long long *)(slot + 2), (unsigned long long)cnt);
                return;
            }
        }
        if (table_full(probe, a.ctr, OVF_M)) break;
        h = (h + 1) & a.m_mask;
        ++probe;
    }
    atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_M);
}
// workgroup (p, b): bucket b of partition p = bucketed entries [off[(p B + b) T], off[(p B + b + 1) T])
#define MBA_T 512
__global__ __launch_bounds__(MBA_T) void k_mb_agg(ScanArgs a, u32 T, const u64 *__restrict__ off,
                                                  const u64 *__restrict__ total, const ulonglong2 *__restrict__ in) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ulonglong2 *keys = reinterpret_cast<ulonglong2 *>(smem);
    u32 *cnts = reinterpret_cast<u32 *>(smem + MA_SLOTS * 16);
    const u64 q = (u64)blockIdx.y * MB_B + blockIdx.x;
    const u64 lo = off[q * T], hi = q + 1 < (u64)MSA_MLOG_PARTS * MB_B ? off[(q + 1) * T] : *total;
    if (lo >= hi) return;
    for (u32 i = threadIdx.x; i < MA_SLOTS; i += MBA_T) {
        keys[i] = make_ulonglong2(0, 0);
        cnts[i] = 0;
    }
    __syncthreads();
    for (u64 i0 = lo + threadIdx.x; i0 < hi; i0 += (u64)MA_FLY * MBA_T) {
        ulonglong2 xs[MA_FLY];
#pragma unroll
        for (int f = 0; f < MA_FLY; ++f) {
            const u64 i = i0 + (u64)f * MBA_T;
            xs[f] = i < hi ? in[i] : make_ulonglong2(0, 0);
        }
#pragma unroll
        for (int f = 0; f < MA_FLY; ++f) {
            if (i0 + (u64)f * MBA_T >= hi) break;
            const ulonglong2 x = xs[f];
            const u32 c = gather8(x.x) | ((gather8(x.y) & 0x7Fu) << 8);
            const u64 k0 = x.x & MLOG_KEYBITS, k1 = x.y & (MLOG_KEYBITS | KMARK);
            const u32 slot = ma_find(keys, k0, k1);
            if (slot != ~0u) atomicAdd(&cnts[slot], c ? c : 1u);
            else hbm_insert16<true>(a, k0, k1, c ? c : 1u);  // table full: this key's every entry
        }
    }
    __syncthreads();
    for (u32 i = threadIdx.x; i < MA_SLOTS; i += MBA_T) {
        const u32 c = cnts[i];
        if (c) {
            const ulonglong2 kk = keys[i];
            mb_insert_once(a, kk.x, kk.y, c);
        }
    }
}

// k_mb_dense (ScanArgs::dn_*, single GPU, high cardinality): no HBM table at
// all -- a bucket's distinct keys are final once counted (no other workgroup
// sees them), so each becomes its ranking entry right here (the K2 / K1 / K0 /
// val / ref / cnt planes k_word_entries would have written from the table: no
// inserts, no slot lists, no table clears).  Persistent: a workgroup per CU
// takes buckets blockIdx.x, + gridDim.x, ... with one LDS table, cleared as
// its entries are written out (no clear pass per bucket, no launch of a
// workgroup per bucket).  A key the LDS table cannot hold, or entries past
// the planes' capacity, flag OVF_DENSE: the split runs again through the
// tables.  The planes' OR / AND: one partial per workgroup
// (dn_vary[6 + blockIdx.x * 6 ..]), reduced by k_dn_vary into dn_vary[0..5].
#ifndef MBD_T
#define MBD_T 1024  // 16 waves: 512 threads (8 waves) 1.57 ms at configs[4]
#endif
#define MBD_KS ((MA_SLOTS + MBD_T - 1) / MBD_T)
__global__ __launch_bounds__(MBD_T) void k_mb_dense(ScanArgs a, u32 T, const u64 *__restrict__ off,
                                                    const u64 *__restrict__ total, const ulonglong2 *__restrict__ in) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ulonglong2 *keys = reinterpret_cast<ulonglong2 *>(smem);
    u32 *cnts = reinterpret_cast<u32 *>(smem + MA_SLOTS * 16);
    __shared__ u32 s_wbase[MBD_T / 64], s_tot, s_ns;
    __shared__ u64 s_gbase, s_vary[6];
    const u32 lane = lane_id(), wv = threadIdx.x >> 6;
    for (u32 i = threadIdx.x; i < MA_SLOTS; i += MBD_T) {
        keys[i] = make_ulonglong2(0, 0);
        cnts[i] = 0;
    }
    u64 vo[3] = {0, 0, 0}, va[3] = {~0ull, ~0ull, ~0ull};
    const u64 nq = (u64)MSA_MLOG_PARTS * MB_B;
    // bucket q's bounds and first batch of entries, loaded while the bucket
    // before it is written out
    u64 nlo = 0, nhi = 0;
    ulonglong2 pf[MA_FLY];
    auto prefetch = [&](u64 q) {
        if (q >= nq) return;
        nlo = off[q * T];
        nhi = q + 1 < nq ? off[(q + 1) * T] : *total;
#pragma unroll
        for (int f = 0; f < MA_FLY; ++f) {
            const u64 i = nlo + threadIdx.x + (u64)f * MBD_T;
            pf[f] = i < nhi ? in[i] : make_ulonglong2(0, 0);
        }
    };
    prefetch(blockIdx.x);
    for (u64 q = blockIdx.x; q < nq; q += gridDim.x) {
        if (threadIdx.x == 0) s_tot = s_ns = 0;
        __syncthreads();  // (the table clear / the last bucket's flush done)
        const u64 lo = nlo, hi = nhi;
        for (u64 i0 = lo + threadIdx.x; i0 < hi; i0 += (u64)MA_FLY * MBD_T) {
            ulonglong2 xs[MA_FLY];
            if (i0 == lo + threadIdx.x) {
#pragma unroll
                for (int f = 0; f < MA_FLY; ++f) xs[f] = pf[f];
            } else {
#pragma unroll
                for (int f = 0; f < MA_FLY; ++f) {
                    const u64 i = i0 + (u64)f * MBD_T;
                    xs[f] = i < hi ? in[i] : make_ulonglong2(0, 0);
                }
            }
#pragma unroll
            for (int f = 0; f < MA_FLY; ++f) {
                if (i0 + (u64)f * MBD_T >= hi) break;
                const ulonglong2 x = xs[f];
                const u32 c = gather8(x.x) | ((gather8(x.y) & 0x7Fu) << 8);
                const u64 k0 = x.x & MLOG_KEYBITS, k1 = x.y & (MLOG_KEYBITS | KMARK);
                const u32 slot = ma_find<16>(keys, k0, k1);
                if (slot != ~0u) atomicAdd(&cnts[slot], c ? c : 1u);
                else atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_DENSE);
            }
        }
        __syncthreads();
        // the bucket's entries (each key holds one slot: ma_find's claims): a
        // range per wave (slots threadIdx.x + k MBD_T), the bucket's range
        // from one device atomic; each wave's k-th batch of entries is
        // contiguous (coalesced stores)
        u32 nw = 0, nsw = 0;
        for (u32 k = 0; k < MBD_KS; ++k) {
            const u32 i = threadIdx.x + k * MBD_T;
            const bool live = i < MA_SLOTS && cnts[i] != 0;
            const u64 bm = __ballot(live), bs = __ballot(live && keys[i].y == KMARK);
            nw += (u32)__popcll(bm);
            nsw += (u32)__popcll(bs);
        }
        if (lane == 0) {
            s_wbase[wv] = atomicAdd(&s_tot, nw);
            atomicAdd(&s_ns, nsw);
        }
        __syncthreads();
        if (threadIdx.x == 0 && s_tot) {
            s_gbase = atomicAdd((unsigned long long *)&a.ctr->dense_n, (unsigned long long)s_tot);
            atomicAdd((unsigned long long *)&a.ctr->s_claimed, (unsigned long long)s_ns);
            atomicAdd((unsigned long long *)&a.ctr->m_claimed, (unsigned long long)(s_tot - s_ns));
            if (s_gbase + s_tot > a.dn_cap)
                atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_DENSE);
        }
        prefetch(q + gridDim.x);  // (in flight across the barrier and the write-out)
        __syncthreads();
        u64 idx = s_gbase + s_wbase[wv];
        for (u32 k = 0; k < MBD_KS; ++k) {
            const u32 i = threadIdx.x + k * MBD_T;
            const u32 c = i < MA_SLOTS ? cnts[i] : 0u;
            const u64 bm = __ballot(c != 0);
            const u64 e = idx + mbcnt(bm);
            idx += (u64)__popcll(bm);
            if (c == 0) continue;
            const ulonglong2 kk = keys[i];
            keys[i] = make_ulonglong2(0, 0);  // the table clear for the next bucket
            cnts[i] = 0;
            if (e >= a.dn_cap) continue;
            const bool sk = kk.y == KMARK;
            const u64 k2 = ~(u64)c, k1 = __builtin_bswap64(kk.x), k0 = sk ? 0ull : __builtin_bswap64(kk.y & ~KMARK);
            a.dn_K2[e] = k2;
            a.dn_K1[e] = k1;
            a.dn_K0[e] = k0;
            a.dn_val[e] = (u32)e;
            a.dn_ref[e] = ((u64)(sk ? KIND_S : KIND_M) << 60) | e;
            a.dn_cnt[e] = c;
            vo[0] |= k0; vo[1] |= k1; vo[2] |= k2;
            va[0] &= k0; va[1] &= k1; va[2] &= k2;
        }
    }
#pragma unroll
    for (int w = 0; w < 3; ++w) {
        for (int o = 32; o > 0; o >>= 1) {
            vo[w] |= (u64)__shfl_xor((long long)vo[w], o);
            va[w] &= (u64)__shfl_xor((long long)va[w], o);
        }
    }
    if (threadIdx.x < 6) s_vary[threadIdx.x] = threadIdx.x < 3 ? 0ull : ~0ull;
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int w = 0; w < 3; ++w) {
            atomicOr((unsigned long long *)&s_vary[w], (unsigned long long)vo[w]);
            atomicAnd((unsigned long long *)&s_vary[3 + w], (unsigned long long)va[w]);
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) a.dn_vary[6 + (u64)blockIdx.x * 6 + threadIdx.x] = s_vary[threadIdx.x];
}
// The dense planes' OR / AND from the bucket workgroups' partials (one
// workgroup) into vary[0..5] (k_word_entries adds the long words' to them).
#define DV_T 1024
__global__ __launch_bounds__(DV_T) void k_dn_vary(const u64 *__restrict__ part, u32 nq, u64 *__restrict__ vary) {
    __shared__ u64 r[DV_T / 64][6];
    u64 v[6] = {0, 0, 0, ~0ull, ~0ull, ~0ull};
    for (u32 q = threadIdx.x; q < nq; q += DV_T) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            v[k] |= part[(u64)q * 6 + k];
            v[3 + k] &= part[(u64)q * 6 + 3 + k];
        }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k)
        for (int o = 32; o > 0; o >>= 1) {
            const u64 y = (u64)__shfl_xor((long long)v[k], o);
            v[k] = k < 3 ? (v[k] | y) : (v[k] & y);
        }
    if (lane_id() == 0)
        for (int k = 0; k < 6; ++k) r[threadIdx.x >> 6][k] = v[k];
    __syncthreads();
    if (threadIdx.x < 6) {
        const u32 k = threadIdx.x;
        u64 x = r[0][k];
        for (u32 w = 1; w < DV_T / 64; ++w) x = k < 3 ? (x | r[w][k]) : (x & r[w][k]);
        vary[k] = x;
    }
}

static int g_q_cus = 0;
// Counting workgroups: one per CU (k_scan_tokens: a wave per 4 KiB block);
// k_miss_agg reads their logs.
static u32 scan_blocks(const ScanArgs &a) {
    if (!g_q_cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        hipDeviceProp_t p;
        g_q_cus = (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ? p.multiProcessorCount
                                                                                                 : 256;
        (void)hipFuncSetAttribute((const void *)k_scan_tokens, hipFuncAttributeMaxDynamicSharedMemorySize, Q_LDS);
        (void)hipFuncSetAttribute((const void *)k_miss_agg, hipFuncAttributeMaxDynamicSharedMemorySize, MA_SLOTS * 20);
    }
    const u64 units = (a.seg_end - a.seg_begin + Q_BLK - 1) / Q_BLK;
    const u64 blocks = (units + Q_W - 1) / Q_W;
    return blocks > (u64)g_q_cus * Q_WGCU ? (u32)g_q_cus * Q_WGCU : (u32)blocks;
}
u32 msa_tok_wgcu() { return Q_WGCU; }
// The split scan's first kernel, k_scan_struct (msa_launch_scan_tokens then
// runs the second on the same stream).
hipError_t msa_launch_scan_csv(const ScanArgs &a, hipStream_t s) {
    if (!a.nchunks) return hipSuccess;
    (void)scan_blocks(a);  // the device's CU count
    // a wave per chunk, SA_MINW waves per SIMD while chunks last
    const u32 waves = std::min<u32>(a.nchunks, (u32)g_q_cus * 4 * SA_MINW);
    hipLaunchKernelGGL(k_scan_struct, dim3((waves + SA_T / 64 - 1) / (SA_T / 64)), dim3(SA_T), 0, s, a);
    return hipGetLastError();
}
// The folded split scan (k_scan_fold); *tickets = the tickets it takes (the
// next launch's fold_tbase advances by that many)
u32 msa_fold_tiles(u32 nchunks) { return (nchunks + FD_CH - 1) / FD_CH; }
hipError_t msa_launch_scan_fold(const ScanArgs &a, u64 *tickets, hipStream_t s) {
    *tickets = 0;
    if (!a.nchunks) return hipSuccess;
    (void)scan_blocks(a);  // the device's CU count
    const u32 ntiles = msa_fold_tiles(a.nchunks);
    const u32 grid = std::min<u32>(ntiles, (u32)g_q_cus * FD_MINW);
    hipLaunchKernelGGL(k_scan_fold, dim3(grid), dim3(FD_T), 0, s, a);
    *tickets = (u64)ntiles + grid;
    return hipGetLastError();
}
hipError_t msa_launch_scan_tokens(const ScanArgs &a, hipStream_t s) {
    if (!a.nchunks) return hipSuccess;
    hipLaunchKernelGGL(k_scan_tokens, dim3(scan_blocks(a)), dim3(Q_T), Q_LDS, s, a);
    return hipGetLastError();
}
// after k_scan_tokens on the same stream: fold the logged misses, 16 partitions x
// groups, one workgroup per CU
// the bucketed aggregation: scratch sizes (entries = every log's capacity)
u64 msa_mb_hist_words(const ScanArgs &a, u32 nsrc) {
    const u32 chunks = (a.mlog_cap + MB_TILE - 1) / MB_TILE;
    return (u64)MSA_MLOG_PARTS * MB_B * nsrc * chunks;
}
hipError_t msa_exclusive_scan(const u64 *in, u64 n, u64 *out, u64 *bsum_scratch, u64 *total, hipStream_t s);
// k_mb_dense's workgroups: one per CU (its LDS table is the whole LDS)
static u32 msa_dn_groups() {
    if (!g_q_cus) {
        int dev = 0;
        hipDeviceProp_t pr;
        (void)hipGetDevice(&dev);
        g_q_cus = (hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0) ? pr.multiProcessorCount
                                                                                                   : 256;
    }
    return (u32)g_q_cus;
}
// hist / off: msa_mb_hist_words u64 each; bsum: (that + 1023) / 1024 + 1 words;
// total: one word; out: nsrc * PARTS * mlog_cap entries
hipError_t msa_launch_miss_buckets(const ScanArgs &a, u64 *hist, u64 *off, u64 *bsum, u64 *total, ulonglong2 *out,
                                   hipStream_t s) {
    if (!a.nchunks) return hipSuccess;
    const u32 nsrc = scan_blocks(a);
    const u32 chunks = (a.mlog_cap + MB_TILE - 1) / MB_TILE, T = nsrc * chunks;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)k_mb_agg, hipFuncAttributeMaxDynamicSharedMemorySize, MA_SLOTS * 20);
        (void)hipFuncSetAttribute((const void *)k_mb_dense, hipFuncAttributeMaxDynamicSharedMemorySize, MA_SLOTS * 20);
        (void)hipFuncSetAttribute((const void *)k_mb_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, MS_LDS);
        attr = true;
    }
    hipLaunchKernelGGL(k_mb_hist, dim3(T, MSA_MLOG_PARTS), dim3(MB_TT), 0, s, a, chunks, T, hist);
    hipError_t e = msa_exclusive_scan(hist, msa_mb_hist_words(a, nsrc), off, bsum, total, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mb_scatter, dim3(T, MSA_MLOG_PARTS), dim3(MB_TT), MS_LDS, s, a, chunks, T, (const u64 *)off,
                       out);
    if (a.dn_K2) {  // dense entries (the caller zeroed Counters::dense_n with the split's counters)
        const u32 g = msa_dn_groups();
        hipLaunchKernelGGL(k_mb_dense, dim3(g), dim3(MBD_T), MA_SLOTS * 20, s, a, T, (const u64 *)off,
                           (const u64 *)total, (const ulonglong2 *)out);
        hipLaunchKernelGGL(k_dn_vary, dim3(1), dim3(DV_T), 0, s, (const u64 *)a.dn_vary + 6, g, a.dn_vary);
    } else {
        hipLaunchKernelGGL(k_mb_agg, dim3(MB_B, MSA_MLOG_PARTS), dim3(MBA_T), MA_SLOTS * 20, s, a, T,
                           (const u64 *)off, (const u64 *)total, (const ulonglong2 *)out);
    }
    return hipGetLastError();
}
u32 msa_scan_blocks(const ScanArgs &a) { return scan_blocks(a); }
// the dense planes' OR / AND: dn_vary holds msa_dn_vary_words() words, the
// reduced six first (the radix sort's varying-byte mask), then the partials
u64 msa_dn_vary_words() { return (u64)msa_dn_groups() * 6 + 6; }
hipError_t msa_launch_miss_agg(const ScanArgs &a, hipStream_t s) {
    if (!a.nchunks) return hipSuccess;
    const u32 blocks = scan_blocks(a);
#ifndef MA_GROUP_MUL
#define MA_GROUP_MUL 1  // aggregating workgroups per CU
#endif
    const u32 groups = std::max<u32>(1, std::min<u32>(blocks, MA_GROUP_MUL * (u32)g_q_cus / MSA_MLOG_PARTS));
    hipLaunchKernelGGL(k_miss_agg, dim3(groups * MSA_MLOG_PARTS), dim3(MA_T), MA_SLOTS * 20, s, a, blocks, groups);
    return hipGetLastError();
}
