// msa_internal.h -- shared device/host definitions of libmsa_hip (gfx950).
//
// Byte layout in HBM: the CSV is one flat byte array; all per-record data is
// structure-of-arrays indexed by record number; hash tables are open-address
// arrays of 16/32-byte slots.  Scan granularity:
//   MSA_ITER  = 1 KiB  = one wave-iteration (64 lanes x 16 B, one dwordx4 each)
//   MSA_CHUNK = 16 KiB = the unit whose reader-state transfer function is
//               summarised (K1) and scanned (K2) before the main pass (K3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;

#define MSA_ITER 1024
#define MSA_CHUNK 16384
#define MSA_ITERS (MSA_CHUNK / MSA_ITER)

// ---------------------------------------------------------------------------
// Reader state.  The reference's record reader (parallel_spotify.c:549-633)
// and field splitter (258-304) are a finite-state machine over bytes; what a
// later byte needs from everything before it is:
//   p     quote parity (1 = inside a quoted run)
//   cr    previous byte was an unquoted '\r' (a following '\n' is swallowed)
//   c     unquoted commas since the record start, saturated at 3
//   z     a NUL was seen since the record start (C-string truncation)
//   rec   index of the current record (terminators so far)
//   rs    absolute offset where the current record starts
struct State {
    u64 rec;
    u64 rs;
    u32 p, cr, c, z;
};

// Transfer function of a byte range, one entry per input (p, cr) in
// {(0,0), (1,0), (0,1)}.  If the range holds a terminator ("has"), c/z/rs are
// the values after its last terminator; otherwise c adds (saturating) and z ORs.
struct FnEnt {
    u64 nterm;
    u64 rs;       // absolute start of the record open at the range end (if has)
    u32 p, cr, has, c, z, pad;
};
struct Fn {
    FnEnt e[3];
};

// K1 output per chunk: the chunk's function for hypotheses p=0 / p=1 with
// cr=0 (the cr=1 entry is derived from first_nl).  Packed flags word:
//   [15:0] nterm  [17:16] c  [18] z  [19] cr_out  [20] parity  [21] first_nl
//   [22] the chunk holds a '\r' or NUL byte (both hypotheses)
struct ChunkSum {
    u32 h[2];
    u32 last_end[2];  // offset in chunk just past the last terminator
};

__host__ __device__ inline u32 st_index(u32 p, u32 cr) { return cr ? 2u : p; }

__host__ __device__ inline FnEnt chunk_entry(const ChunkSum &s, u64 base, u32 idx) {
    FnEnt e;
    u32 hyp = (idx == 1) ? 1u : 0u;
    u32 f = s.h[hyp];
    u32 nterm = f & 0xFFFFu;
    e.pad = 0;
    e.p = hyp ^ ((f >> 20) & 1u);
    e.cr = (f >> 19) & 1u;
    e.c = (f >> 16) & 3u;
    e.z = (f >> 18) & 1u;
    e.rs = base + s.last_end[hyp];
    if (idx == 2 && ((f >> 21) & 1u)) nterm -= 1;  // leading '\n' swallowed by the carried '\r'
    e.nterm = nterm;
    e.has = nterm > 0;
    return e;
}

// g's entry for input state (p, cr), by value selects (a dynamic index into
// the entry array would put Fn in scratch memory).
__host__ __device__ inline FnEnt fn_pick(const Fn &g, u32 p, u32 cr) {
    const bool two = cr != 0, one = p != 0;
    FnEnt r;
#define MSA_PICK(f) r.f = two ? g.e[2].f : (one ? g.e[1].f : g.e[0].f)
    MSA_PICK(nterm); MSA_PICK(rs); MSA_PICK(p); MSA_PICK(cr); MSA_PICK(has); MSA_PICK(c); MSA_PICK(z);
#undef MSA_PICK
    r.pad = 0;
    return r;
}

__host__ __device__ inline FnEnt fn_then(const FnEnt &a, const Fn &g) {
    const FnEnt b = fn_pick(g, a.p, a.cr);
    FnEnt r;
    r.p = b.p;
    r.cr = b.cr;
    r.nterm = a.nterm + b.nterm;
    r.has = a.has | b.has;
    if (b.has) {
        r.c = b.c; r.z = b.z; r.rs = b.rs;
    } else {
        u32 c = a.c + b.c;
        r.c = c > 3 ? 3 : c;
        r.z = a.z | b.z;
        r.rs = a.rs;
    }
    r.pad = 0;
    return r;
}

__host__ __device__ inline Fn fn_compose(const Fn &f, const Fn &g) {  // f then g
    Fn r;
    r.e[0] = fn_then(f.e[0], g);
    r.e[1] = fn_then(f.e[1], g);
    r.e[2] = fn_then(f.e[2], g);
    return r;
}

__host__ __device__ inline Fn fn_identity(u64 pos) {
    Fn r;
    for (u32 i = 0; i < 3; ++i) {
        r.e[i].nterm = 0; r.e[i].rs = pos; r.e[i].has = 0; r.e[i].c = 0; r.e[i].z = 0; r.e[i].pad = 0;
        r.e[i].p = (i == 1); r.e[i].cr = (i == 2);
    }
    return r;
}

__host__ __device__ inline State fn_apply(const State &s, const Fn &f) {
    const FnEnt b = fn_pick(f, s.p, s.cr);
    State r;
    r.p = b.p;
    r.cr = b.cr;
    r.rec = s.rec + b.nterm;
    if (b.has) { r.c = b.c; r.z = b.z; r.rs = b.rs; }
    else { u32 c = s.c + b.c; r.c = c > 3 ? 3 : c; r.z = s.z | b.z; r.rs = s.rs; }
    return r;
}

// ---------------------------------------------------------------------------
// SWAR byte classification (4 bytes per u32, exact, no cross-byte carries).
__device__ __forceinline__ u32 swar_eq(u32 x, u32 byte) {
    u32 y = x ^ (byte * 0x01010101u);
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);  // 0x80 where equal
}
__device__ __forceinline__ u32 swar_ge7(u32 y7, u32 c) {  // y7 bytes < 0x80; 0x80 where byte >= c
    return (y7 + (0x80u - c) * 0x01010101u) & 0x80808080u;
}
// 0x80-per-byte mask -> 4-bit mask (byte j -> bit j): one v_dot4_u32_u8 (the
// bytes weighted 1, 2, 4, 8), not a 32-bit multiply (quarter rate)
__device__ __forceinline__ u32 swar_pack4(u32 m) { return __builtin_amdgcn_udot4(m, 0x08040201u, 0u, false) >> 7; }
// Two dwords of 0x80 flags -> 128 x (8-bit mask): bytes of a -> bits 0..3, of
// b -> bits 4..7 (two chained dot4s)
__device__ __forceinline__ u32 swar_pack8x128(u32 a, u32 b) {
    return __builtin_amdgcn_udot4(b, 0x80402010u, __builtin_amdgcn_udot4(a, 0x08040201u, 0u, false), false);
}
// Byte k (0..7) of a 64-bit mask kept as two dwords, from swar_pack8x128
__device__ __forceinline__ void swar_put8(u32 &lo, u32 &hi, int k, u32 p128) {
    const int s = 8 * (k & 3) - 7;
    const u32 v = s < 0 ? (p128 >> 7) : (p128 << s);
    if (k < 4) lo |= v;
    else hi |= v;
}
__device__ __forceinline__ u64 mk64(u32 lo, u32 hi) { return ((u64)hi << 32) | lo; }

// The same tests with x7 = x & 0x7F7F7F7F shared by every class of one dword:
// "byte == c" (c < 0x80) is one v_xad_u32 + one v_bitop3_b32, and the token
// class of process_lyrics (isalnum or '\'', parallel_spotify.c:359) a dozen ops.
__device__ __forceinline__ u32 eq80x(u32 x, u32 x7, u32 c) {
    const u32 t = (x7 ^ (c * 0x01010101u)) + 0x7F7F7F7Fu;  // bit 7 of a byte: low 7 bits != c
    return ~(t | x) & 0x80808080u;
}
__device__ __forceinline__ u32 tok80x(u32 x, u32 x7) {
    const u32 z = x7 | 0x20202020u;                           // case folded
    const u32 al = (z + 0x1F1F1F1Fu) & ~(z + 0x05050505u);    // 'a'..'z'
    const u32 dg = (x7 + 0x50505050u) & ~(x7 + 0x46464646u);  // '0'..'9'
    return ((al | dg) & ~x & 0x80808080u) | eq80x(x, x7, '\'');
}

// Token byte of process_lyrics (parallel_spotify.c:359): isalnum (C locale) or '\''.
__device__ __forceinline__ u32 swar_tok(u32 x) {
    u32 hi = x & 0x80808080u;
    u32 y = x & 0x7F7F7F7Fu;
    u32 l = y | 0x20202020u;
    u32 alpha = swar_ge7(l, 'a') & ~swar_ge7(l, 'z' + 1);
    u32 digit = swar_ge7(y, '0') & ~swar_ge7(y, '9' + 1);
    return ((alpha | digit) & ~hi) | swar_eq(x, '\'');
}

struct Classes {
    u32 Q, C, NL, CR, Z, T;  // 16-bit masks, bit j = byte j of the lane's 16 bytes
};

__device__ __forceinline__ Classes classify16(uint4 v, u32 vmask) {
    Classes k;
    u32 w[4] = {v.x, v.y, v.z, v.w};
    u32 Q = 0, C = 0, NL = 0, CR = 0, Z = 0, T = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        Q |= swar_pack4(swar_eq(w[i], '"')) << (4 * i);
        C |= swar_pack4(swar_eq(w[i], ',')) << (4 * i);
        NL |= swar_pack4(swar_eq(w[i], '\n')) << (4 * i);
        CR |= swar_pack4(swar_eq(w[i], '\r')) << (4 * i);
        Z |= swar_pack4(swar_eq(w[i], 0)) << (4 * i);
        T |= swar_pack4(swar_tok(w[i])) << (4 * i);
    }
    k.Q = Q & vmask; k.C = C & vmask; k.NL = NL & vmask; k.CR = CR & vmask; k.Z = Z & vmask; k.T = T & vmask;
    return k;
}

__device__ __forceinline__ u32 tok16(uint4 v, u32 vmask) {
    return (swar_pack4(swar_tok(v.x)) | (swar_pack4(swar_tok(v.y)) << 4) |
            (swar_pack4(swar_tok(v.z)) << 8) | (swar_pack4(swar_tok(v.w)) << 12)) & vmask;
}

// exclusive prefix-xor over 16 bits: bit j = xor of bits < j
__device__ __forceinline__ u32 pxor_excl16(u32 q) {
    u32 x = q << 1;
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    return x & 0xFFFFu;
}

// ---------------------------------------------------------------------------
// Wave (64-lane) helpers.
__device__ __forceinline__ u32 lane_id() { return __lane_id(); }
__device__ __forceinline__ u32 mbcnt(u64 m) {  // popcount of m's bits below this lane
    return __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
}
// Exclusive wave prefix sum of small values (< 2^BITS) via ballot bit-planes.
template <int BITS>
__device__ __forceinline__ u32 wave_prefix(u32 x, u32 &total) {
    u32 pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < BITS; ++k) {
        u64 b = __ballot((x >> k) & 1u);
        pre += mbcnt(b) << k;
        tot += (u32)__popcll(b) << k;
    }
    total = tot;
    return pre;
}
__device__ __forceinline__ u32 readlane(u32 x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ u64 readlane64(u64 x, int l) {
    return ((u64)readlane((u32)(x >> 32), l) << 32) | readlane((u32)x, l);
}
__device__ __forceinline__ u64 wave_sum64(u64 v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ---------------------------------------------------------------------------
// Hashing.
__host__ __device__ __forceinline__ u64 fmix64(u64 k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}
__device__ __forceinline__ u32 lds_hash(u64 k) { return (u32)((k * 0x9E3779B97F4A7C15ULL) >> 40); }

// Lower-case ASCII letters in 8 packed bytes (all bytes < 0x80 here).
__device__ __forceinline__ u64 lower8(u64 x) {
    u64 y = x & 0x7F7F7F7F7F7F7F7FULL;
    u64 ge_a = (y + 0x3F3F3F3F3F3F3F3FULL) & 0x8080808080808080ULL;  // >= 'A' (0x41)
    u64 ge_z = (y + 0x2525252525252525ULL) & 0x8080808080808080ULL;  // >= 'Z'+1 (0x5B)
    return x | ((ge_a & ~ge_z) >> 2);
}

// ---------------------------------------------------------------------------
// Device-resident run counters (one struct, zeroed per run).
struct Counters {
    u64 total_words;
    u64 s_claimed, m_claimed, l_occ, l_claimed, a_claimed;
    u64 overflow;    // bitmask of capacity overflows
    u64 collision;   // hash-collision detections
    u64 songs;
    // split: some accepted record's artist field holds a '"' without being a
    // quoted field, so artist.csv lines may not be artist.csv records (the
    // artist pass then runs the exact record reader over artist.csv)
    u64 a_quoted;
    u64 a_long;      // bytes used in the long-key arena (k_rec_spans)
    u64 k3_misses;   // K3 log entries folded by k_miss_agg: LDS-table misses + flushed table entries (diagnostic)
    u64 col_body[2]; // artist.csv / text.csv body bytes (the line-offset scans' totals)
    u64 span_fix;    // records k_rec_fast hands to k_rec_fix (the exact per-record path)
    u64 mlog_full;   // K3 misses that found their log partition full (dropped: the split runs again with
                     // larger logs; at the logs' size limit inserted straight into HBM)
    u64 dense_n;     // dense S/M entries written (the bucketed aggregation's cursor)
};

enum { OVF_S = 1, OVF_M = 2, OVF_L = 4, OVF_LT = 8, OVF_A = 16, OVF_REC = 32, OVF_MLOG = 64, OVF_FOLD = 128, OVF_DENSE = 256 };

// Artist keys built by k_rec_spans for the lines shortcut of the artist pass:
// per record the key bytes (duplicate_field(duplicate_field(field0, 1), 0))
// in the arena -- a 32-byte slot per record, longer or escaped keys in the
// long area behind an atomic cursor -- and two independent 64-bit hashes.
struct AKeys {
    u8 *arena;
    u64 *key_off;
    u32 *key_len;
    u64 *kh1, *kh2;
    u64 long_base, long_cap;  // long area = arena + [long_base, long_base + long_cap)
};

// Arguments of the main scan (K3) and of the ranking-entry builder.
struct ScanArgs {
    const u8 *buf;
    u64 seg_begin, seg_end;
    u32 nchunks;
    const State *carry;
    u64 *rec_start;
    u32 *nulrel;
    u64 rec_cap;
    // per record, for the column spans (k_rec_fast): f0 = position of field
    // 0's comma; tss = start of field 3 (| SPAN_Q: it is a '"'); tse = the
    // record's terminator (| SPAN_Q: the byte before is a '"', | SPAN_NUL /
    // SPAN_NOLINE)
    u64 *f0, *tss, *tse;
    u64 *s_tab;
    u64 s_mask;
    u32 *s_list;
    u64 s_list_cap;
    u64 *m_tab;
    u64 m_mask;
    u32 *m_list;
    u64 m_list_cap;
    u64 *l_pos;
    u64 l_cap;
    u64 l_expect;    // long-word occurrences expected (the last split's; sizes the waves' l_pos ranges)
    // K1's chunk summaries of this segment (bit 22 of h[0]: the chunk holds a
    // '\r' or NUL), or null: test every block
    const ChunkSum *sums;
    u64 lpos_tag;    // OR'ed into recorded long-token positions (MSA_POS_EXTRA: the side buffer)
    Counters *ctr;
    int want_nul;    // record the first NUL of each record (text column)
    int ablate;
    u32 first_rec;   // records before this index are not data (the header: 1; a continuation shard: 0)
    // K3 misses of the LDS word table, logged per (workgroup, key partition)
    // for k_miss_agg (MSA_MLOG_PARTS partitions, mlog_cap entries each)
    ulonglong2 *mlog;
    u32 *mlog_n;
    u32 mlog_cap;
    int mlog_direct; // the logs are at their size limit: a full partition's entries go to the HBM tables
    // folded split scan (k_scan_fold: K1 + K2 + k_scan_struct in one pass):
    // tiles of 4 chunks taken in ticket order (ticket - fold_tbase), each
    // publishing its chunk functions' composition, then its end state, as
    // self-validating words (epoch fold_ep in bits 48-63) in fold_stat: 5
    // arrays of fold_n words (3 function entries, 2 state words)
    u64 *fold_stat;
    u64 *fold_ticket;
    u64 fold_tbase;
    u32 fold_n, fold_ep;
    State fold_init;
    State *fold_fin;       // the state after the segment (device)
    State *fold_fin_host;  // the same, into pinned host memory
    // split scan (k_scan_struct -> k_scan_tokens): bit i of lmask[1 + i / 64]
    // = byte seg_begin + i is a token byte of a counted lyric field
    // (process_lyrics input, parallel_spotify.c:350-394); lmask[0] = 0 pad
    u64 *lmask;
    // dense S/M entries (high cardinality, single GPU): the bucketed
    // aggregation writes each distinct 3..16-byte word's ranking entry
    // straight into these planes (null: into the HBM tables) -- see k_mb_agg
    u64 *dn_K2, *dn_K1, *dn_K0, *dn_ref, *dn_cnt, *dn_vary;
    u32 *dn_val;
    u64 dn_cap;
};

#define MSA_MLOG_PARTS 16

#define SPAN_Q (1ull << 63)
#define SPAN_NUL (1ull << 62)
#define SPAN_NOLINE (1ull << 61)
#define SPAN_FIX (1ull << 60)   // set by the host on an unterminated last record
#define SPAN_POS ((1ull << 60) - 1)

// A long-token position with this bit set indexes the context's side buffer
// (text.csv header-label remainder, see do_split) instead of the CSV.
#define MSA_POS_EXTRA (1ull << 63)
__host__ __device__ inline const u8 *tok_at(const u8 *buf, const u8 *extra, u64 pos) {
    return (pos & MSA_POS_EXTRA) ? extra + (pos & ~MSA_POS_EXTRA) : buf + pos;
}
// ranking entries' ref = (kind << 60) | index: an S / M table slot (or a
// dense entry's own index), a long word's occurrence, an artist record
enum { KIND_S = 0, KIND_M = 1, KIND_L = 2, KIND_A = 3 };
struct EntryArgs {
    const u64 *s_tab;
    const u32 *s_list;
    u64 ns;
    const u64 *m_tab;
    const u32 *m_list;
    u64 nm;
    const u64 *l_tab;
    const u32 *l_list;
    u64 nl;
    const u8 *buf;
    const u8 *extra;
    const u64 *l_pos;
    const u32 *l_len;
    u64 *K2, *K1, *K0;
    u32 *val;
    u64 *ref;
    u64 *cnt;
    u64 vbase;  // val[i] = vbase + i (the planes start at entry vbase: the dense S/M entries before them)
    // optional: OR of each key plane over all entries ([0..2] = K0, K1, K2)
    // and their AND ([3..5]), for the radix sort's varying-byte mask (the
    // caller zeroes the ORs and sets the ANDs to all ones)
    u64 *vary;
};

// Export source: the counted table (words or artists) of one GPU.
struct ExpSrc {
    const u64 *s_tab;
    const u32 *s_list;
    u64 ns;
    const u64 *m_tab;
    const u32 *m_list;
    u64 nm;
    const u64 *l_tab;
    const u32 *l_list;
    u64 nl;
    const u8 *buf, *extra;
    const u64 *l_pos;
    const u32 *l_len;
    const u64 *a_tab;
    const u32 *a_list;
    u64 na;
    const u8 *arena;
    const u64 *key_off;
    const u32 *key_len;
    int artists;
    // words counted as dense entries (k_mb_dense): entries [0, nd) come from
    // their planes -- K1 / K0 the key's big-endian bytes, cnt the count -- in
    // place of the S / M tables (ns = nm = 0); the long words from the table
    const u64 *d_K1, *d_K0, *d_cnt;
    u64 nd;
};
// Import destination: the (cleared) tables that receive a key partition.
struct ImpDst {
    u64 *s_tab;
    u64 s_mask;
    u32 *s_list;
    u64 s_list_cap;
    u64 *m_tab;
    u64 m_mask;
    u32 *m_list;
    u64 m_list_cap;
    u64 *l_tab;
    u64 l_mask;
    u32 *l_list;
    u64 l_list_cap;
    u64 *l_pos;
    u32 *l_len;
    u64 *l_slot;
    u64 l_cap;
    u64 *a_tab;
    u64 a_mask;
    u32 *a_list;
    u64 a_list_cap;
    u64 *key_off;
    u32 *key_len;
    u64 *key_slot;
    Counters *ctr;
    int artists;
};

#define MSA_HIP_CHECK(x)                                                     \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) return msa_fail_hip(e_, #x, __FILE__, __LINE__); \
    } while (0)
