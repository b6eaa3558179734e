// msa_wcs.hip -- per-song word counter on gfx950 (DESIGN.md row f): the GPU
// path of /root/reference/scripts/word_count_per_song.py.
//
// What the script does (file:line in word_count_per_song.py):
//   * reads the CSV with csv.DictReader over open(newline="", "utf-8-sig")
//     (108-117): Python's _csv state machine, lines split at \n, \r\n, \r
//   * tokenize (28-38): runs of [0-9A-Za-zÀ-ÖØ-öø-ÿ'], lower-cased, >= 3
//     characters, not only apostrophes
//   * process_row (91-99): Counter per song (first-occurrence order), rows
//     without tokens dropped; artist/song .strip()
//   * main (124-146): global Counter (first-occurrence order) and
//     most_common() = stable sort by count descending
//
// GPU pipeline (one context, everything resident in HBM):
//   k_wcs_validate   UTF-8 + NUL check of every byte (the decoder / _csv errors)
//   k_wcs_map        per 256-byte segment: the reader's transfer function over
//                    its 6 states (3 bits each) + row ends per entering state
//   k_wcs_state_*    block scan of the maps (composition) -> entering state of
//                    every segment -> row-end counts
//   k_wcs_emit       row ends at their scanned offsets
//   k_wcs_rows       one thread per row: fields, field limit, tokenizer on the
//                    unescaped text field, 64-bit word hash into the global
//                    table (count, first occurrence, h2 checksum), per-row
//                    table of (word, order, count) in a private scratch region
//   k_wcs_list / sort / k_wcs_words  global ranking (count desc, first
//                    occurrence asc -- exactly most_common's stable order),
//                    word bytes in rank order, collision check
//   k_wcs_pairs      by-song lines (rank of word, count) in file order
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "msa_hip.h"
#include "msa_internal.h"

hipError_t msa_exclusive_scan(const u64 *in, u64 n, u64 *out, u64 *bsum_scratch, u64 *total, hipStream_t s);
hipError_t msa_launch_gather_lines(const u8 *buf, const u64 *len, const u64 *off, const u64 *src, u64 nrec,
                                   const u64 *body_p, u8 *col, hipStream_t s);
hipError_t msa_launch_sort(u64 *const K2[3], u64 *const K1[3], u64 *const K0[3], u32 *const V[3], u64 n, int *which,
                           hipStream_t s);

namespace {

// Reader states of CPython's _csv.c (3.10) for the dialect the script uses.
enum : u32 { SR = 0, SF = 1, IF = 2, IQ = 3, QQ = 4, EC = 5 };
#define PK(a, b, c, d, e, f) ((a) | ((b) << 3) | ((c) << 6) | ((d) << 9) | ((e) << 12) | ((f) << 15))
// next state for input state SR SF IF IQ QQ EC
constexpr u32 T_Q = PK(IQ, IQ, IF, QQ, IQ, EC);    // '"'
constexpr u32 T_D = PK(SF, SF, SF, IQ, SF, EC);    // ','
constexpr u32 T_NL = PK(EC, EC, EC, IQ, EC, EC);   // '\r' or '\n'
constexpr u32 T_O = PK(IF, IF, IF, IQ, IF, EC);    // anything else
constexpr u32 T_EOL = PK(SR, SR, SR, IQ, SR, SR);  // end of a line
// ' ' with skipinitialspace (the column splitter's sniffed dialect): ignored
// at a field's start (START_FIELD tests it before the delimiter), otherwise an
// ordinary byte; when ' ' is also the delimiter it moves as T_D but saves no
// field at a field's start
constexpr u32 T_SP = PK(SF, SF, IF, IQ, IF, EC);
constexpr u32 MAP_ID = PK(0, 1, 2, 3, 4, 5);
#undef PK
// actions per (byte class, state), 2 bits per state: bit 0 = the byte is
// added to the field, bit 1 = the field is saved (ends) before it
#define PA(a, b, c, d, e, f) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6) | ((e) << 8) | ((f) << 10))
constexpr u32 A_Q = PA(0, 0, 1, 0, 1, 0);
constexpr u32 A_D = PA(2, 2, 2, 1, 2, 0);
constexpr u32 A_NL = PA(0, 2, 2, 1, 2, 0);
constexpr u32 A_O = PA(1, 1, 1, 1, 1, 0);
constexpr u32 A_SP = PA(0, 0, 1, 1, 1, 0);
constexpr u32 A_SPD = PA(0, 0, 2, 1, 2, 0);
#undef PA

#ifndef CC_IQ
#define CC_IQ 1  // 0: the splitter's pass 0 and the row-end walk step through line ends inside quotes too (A/B)
#endif
#ifndef WCS_PF
#define WCS_PF 1  // 0: the row-split walks and the splitter's row walk without the next vector's load in flight (A/B)
#endif
constexpr u32 SEG = 256;        // bytes per lane in the map / emit passes
constexpr u32 BLK = 256;        // threads per block in the state scan
constexpr u32 PER = 4;          // segments per thread in the state scan
constexpr u32 BSEG = BLK * PER; // segments per block
constexpr u32 FIELD_LIMIT = 131072;

enum : u32 { E_UTF8 = 1, E_NUL = 2, E_LIMIT = 3, E_SHORT = 4 };
enum : u32 { OVF_G = 1 };

struct WCtr {
    u64 err;        // min over (row << 8 | code), ~0 = none
    u64 total_rows; // non-blank data rows
    u64 song_rows;  // rows with >= 1 token
    u64 tokens;
    u64 distinct;   // claimed global slots
    u64 overflow;
    u64 collision;
    u64 listed;
    u64 fallback;   // rows k_wcs_wrows left to the per-thread walk
};

// The reader's dialect: delimiter, quotechar (default '"'), skipinitialspace.
// The per-song counter always reads the default dialect with its delimiter.
struct Dia {
    u32 delim, quote, skip;
};
// byte class in the precedence of _csv.c's START_FIELD: quotechar, then a
// skipped space, then the delimiter, CR/LF, anything else
enum : u32 { C_Q = 0, C_D = 1, C_NL = 2, C_O = 3, C_SP = 4, C_SPD = 5 };
__host__ __device__ __forceinline__ u32 cls_of(u32 b, const Dia &d) {
    if (b == d.quote) return C_Q;
    if (b == ' ' && d.skip) return b == d.delim ? C_SPD : C_SP;
    if (b == d.delim) return C_D;
    return (b == '\r' || b == '\n') ? C_NL : C_O;
}
__host__ __device__ __forceinline__ u32 cls_next(u32 c) {
    return c == C_Q ? T_Q : (c == C_D || c == C_SPD ? T_D : (c == C_NL ? T_NL : (c == C_SP ? T_SP : T_O)));
}
__host__ __device__ __forceinline__ u32 cls_act(u32 c) {
    return c == C_Q ? A_Q : (c == C_D ? A_D : (c == C_NL ? A_NL : (c == C_SP ? A_SP : (c == C_SPD ? A_SPD : A_O))));
}
__host__ __device__ __forceinline__ u32 tpk(u32 b, const Dia &d) { return cls_next(cls_of(b, d)); }
__host__ __device__ __forceinline__ u32 step(u32 t, u32 s) { return (t >> (3 * s)) & 7u; }
__device__ __forceinline__ u32 map_apply(u32 t, u32 m) {  // m then t
    u32 r = 0;
#pragma unroll
    for (u32 k = 0; k < 6; ++k) r |= step(t, (m >> (3 * k)) & 7u) << (3 * k);
    return r;
}
__device__ __forceinline__ u32 compose(u32 f, u32 g) { return map_apply(g, f); }  // f then g

__device__ __forceinline__ u32 byte_of(const uint4 &v, u32 j) {
    const u32 w = j < 8 ? (j < 4 ? v.x : v.y) : (j < 12 ? v.z : v.w);
    return (w >> (8 * (j & 3))) & 0xFFu;
}

__device__ __forceinline__ u32 mask16(const uint4 &v, u32 c) {
    return swar_pack4(swar_eq(v.x, c)) | (swar_pack4(swar_eq(v.y, c)) << 4) | (swar_pack4(swar_eq(v.z, c)) << 8) |
           (swar_pack4(swar_eq(v.w, c)) << 12);
}

// ---------------------------------------------------------------------------
// UTF-8 (strict, as Python's decoder) and NUL check.
__device__ __forceinline__ u32 lead_len(u32 b) {
    return b < 0x80 ? 1 : (b < 0xC2 ? 0 : (b < 0xE0 ? 2 : (b < 0xF0 ? 3 : (b < 0xF5 ? 4 : 0))));
}

// utf8 0: a single-byte --encoding (every byte one character): NULs only
__global__ __launch_bounds__(256) void k_wcs_validate(const u8 *__restrict__ buf, u64 n, WCtr *ctr, u32 utf8) {
    const u64 base = ((u64)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (base >= n) return;
    const uint4 v = *(const uint4 *)(buf + base);
    if (!utf8) {
        bool nul = false;
        for (u32 j = 0; j < 16 && base + j < n; ++j) nul |= byte_of(v, j) == 0;
        if (nul) atomicMin((unsigned long long *)&ctr->err, (unsigned long long)E_NUL);
        return;
    }
    // fast path: 16 bytes without NUL of ASCII and whole 2-byte sequences (lead
    // C2..DF, then a continuation byte) -- almost all of a lyrics file
    if (base + 16 <= n && !mask16(v, 0)) {
        if (!((v.x | v.y | v.z | v.w) & 0x80808080u)) return;
        const u32 w[4] = {v.x, v.y, v.z, v.w};
        u32 X = 0, L2 = 0, C = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32 x = w[k], x7 = x & 0x7F7F7F7Fu;
            X |= swar_pack4(x & 0x80808080u) << (4 * k);
            L2 |= swar_pack4((x7 + 0x3E3E3E3Eu) & ~(x7 + 0x20202020u) & x & 0x80808080u) << (4 * k);
            C |= swar_pack4(x & ~(x << 1) & 0x80808080u) << (4 * k);
        }
        if (!(X & ~(L2 | C)) && C == ((L2 << 1) & 0xFFFFu) && !(L2 & 0x8000u)) return;
    }
    u32 bad = 0;
    for (u32 j = 0; j < 16; ++j) {
        const u64 i = base + j;
        if (i >= n) break;
        const u32 b = byte_of(v, j);
        if (b == 0) { bad = bad ? bad : E_NUL; continue; }
        if (b < 0x80) continue;
        if (b < 0xC0) {  // continuation: must be covered by a lead at most 3 back
            u32 k = 1;
            bool ok = false;
            for (; k <= 3 && i >= k; ++k) {
                const u32 c = buf[i - k];
                if ((c & 0xC0) != 0x80) { ok = lead_len(c) > k; break; }
            }
            if (!ok) bad = E_UTF8;
            continue;
        }
        const u32 L = lead_len(b);
        if (L == 0 || i + L > n) { bad = E_UTF8; continue; }
        const u32 c1 = buf[i + 1];
        u32 lo = 0x80, hi = 0xBF;
        if (b == 0xE0) lo = 0xA0;
        else if (b == 0xED) hi = 0x9F;
        else if (b == 0xF0) lo = 0x90;
        else if (b == 0xF4) hi = 0x8F;
        if (c1 < lo || c1 > hi) { bad = E_UTF8; continue; }
        for (u32 k = 2; k < L; ++k)
            if ((buf[i + k] & 0xC0) != 0x80) bad = E_UTF8;
    }
    if (bad) atomicMin((unsigned long long *)&ctr->err, (unsigned long long)bad);  // row 0: before any row
}

// ---------------------------------------------------------------------------
// Row splitting.  An end of line follows byte i when it is '\n', a '\r' not
// followed by '\n', or the last byte (the final line has no terminator).  A
// row ends at an end of line that takes the reader to SR.
__device__ __forceinline__ bool eol_after(u32 b, u32 next, u64 i, u64 n) {
    return b == '\n' || (b == '\r' && (i + 1 >= n || next != '\n')) || i + 1 == n;
}

// Segment walk shared by k_wcs_map and k_wcs_emit.  Only '"', ',', '\r',
// '\n' (and the last byte of the input) are visited one by one: T_O, the
// step of every other byte, is idempotent, so a run of ordinary bytes is one
// T_O step.  SWAR masks over each 16-byte vector find the visited bytes.
// S: the walker; S::step(t) applies a transfer table, S::eol(i) handles the
// end of a line after byte i.
template <typename W>
__device__ __forceinline__ void seg_walk(const u8 *__restrict__ buf, u64 base, u64 ds, u64 n, Dia dia, W &wk) {
#if WCS_PF
    uint4 vn = base < n ? *(const uint4 *)(buf + base) : make_uint4(0, 0, 0, 0);
#endif
    for (u32 q = 0; q < SEG / 16; ++q) {
        const u64 b0 = base + q * 16;
        if (b0 >= n) break;
#if WCS_PF
        // the next vector's load in flight while this one is walked
        const uint4 v = vn;
        if (q + 1 < SEG / 16 && b0 + 16 < n) vn = *(const uint4 *)(buf + b0 + 16);
#else
        const uint4 v = *(const uint4 *)(buf + b0);
#endif
        u32 vm = 0xFFFFu;
        if (b0 < ds) vm &= 0xFFFFu << (u32)(ds - b0);
        if (b0 + 16 > n) vm &= (1u << (u32)(n - b0)) - 1u;
        if (!vm) continue;
        const u32 Q = mask16(v, dia.quote), D = mask16(v, dia.delim), NL = mask16(v, '\n'), CR = mask16(v, '\r');
        const u32 S = (Q | D | NL | CR | (dia.skip ? mask16(v, ' ') : 0u)) & vm;
        const u32 O = vm & ~S;
        u32 E = S;
        const bool has_last = b0 + 16 >= n;  // the input's last byte is in this vector
        const u32 pl = has_last ? (u32)(n - 1 - b0) : 0u;
        if (has_last && ((vm >> pl) & 1u)) E |= 1u << pl;
        int prev = -1;
        while (E) {
#if CC_IQ
            if (W::single() && wk.in_iq()) {
                // inside quotes nothing but a quotechar moves a one-state walker
                // (line ends there are no row ends): straight to the next one
                const u32 qn = Q & vm & (prev < 0 ? 0xFFFFu : ~((2u << prev) - 1u));
                if (!qn) {
                    prev = 15;
                    break;
                }
                const u32 pq = (u32)__builtin_ctz(qn);
                prev = (int)pq - 1;
                E &= ~((1u << pq) - 1u);
            }
#endif
            const u32 p = (u32)__builtin_ctz(E);
            E &= E - 1;
            const u32 upto_prev = prev < 0 ? 0u : ((2u << prev) - 1u);
            if (O & ((1u << p) - 1u) & ~upto_prev) wk.step(T_O);  // ordinary bytes in (prev, p)
            const u32 c = byte_of(v, p);
            wk.step(tpk(c, dia));
            const u64 i = b0 + p;
            bool eol = i + 1 == n || c == '\n';
            if (c == '\r' && !eol) eol = (p < 15 ? byte_of(v, p + 1) : (u32)buf[i + 1]) != '\n';
            if (eol) wk.eol(i);
            prev = (int)p;
        }
        if (O & ~(prev < 0 ? 0u : ((2u << prev) - 1u))) wk.step(T_O);  // ordinary bytes after the last visited one
    }
}

struct MapWalker {
    static constexpr bool single() { return false; }  // the states of all 6 entering states
    __device__ __forceinline__ bool in_iq() const { return false; }
    u32 m;
    u64 c6;
    __device__ __forceinline__ void step(u32 t) { m = map_apply(t, m); }
    __device__ __forceinline__ void eol(u64) {
#pragma unroll
        for (u32 k = 0; k < 6; ++k) {
            const u32 s = (m >> (3 * k)) & 7u;
            if (s != SR && s != IQ) c6 += 1ull << (9 * k);
        }
        m = map_apply(T_EOL, m);
    }
};

// Per segment: map over the 6 entering states; row ends per entering state
// (9 bits each: at most 256 per segment).
__global__ __launch_bounds__(256) void k_wcs_map(const u8 *__restrict__ buf, u64 ds, u64 n, u64 nseg, Dia dia,
                                                 u32 *__restrict__ map, u64 *__restrict__ cnt6) {
    const u64 seg = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= nseg) return;
    MapWalker wk{MAP_ID, 0};
    seg_walk(buf, seg * SEG, ds, n, dia, wk);
    map[seg] = wk.m;
    cnt6[seg] = wk.c6;
}

// Inclusive scan of the 256 thread composites of a block (Hillis-Steele in LDS).
__device__ u32 block_map_scan(u32 x, u32 *sh) {
    const u32 t = threadIdx.x;
    sh[t] = x;
    __syncthreads();
    for (u32 o = 1; o < BLK; o <<= 1) {
        const u32 y = t >= o ? sh[t - o] : MAP_ID;
        __syncthreads();
        x = compose(y, x);
        sh[t] = x;
        __syncthreads();
    }
    return x;
}

__global__ __launch_bounds__(BLK) void k_wcs_state_block(const u32 *__restrict__ map, u64 nseg,
                                                         u32 *__restrict__ bmap) {
    __shared__ u32 sh[BLK];
    const u64 s0 = (u64)blockIdx.x * BSEG + (u64)threadIdx.x * PER;
    u32 x = MAP_ID;
    for (u32 k = 0; k < PER; ++k)
        if (s0 + k < nseg) x = compose(x, map[s0 + k]);
    x = block_map_scan(x, sh);
    if (threadIdx.x == BLK - 1) bmap[blockIdx.x] = x;
}

constexpr u32 TOP_T = 1024;

// The block maps' entering states with every thread: a chunk of TOP2_PER
// block maps each, a scan of the chunks' composites in LDS, then each thread
// steps through its chunk (k_wcs_state_top's one-thread loop over configs[2]'s
// 4.5 K block maps took 100 us)
constexpr u32 TOP2_PER = 16;
__global__ __launch_bounds__(TOP_T) void k_wcs_state_top2(u32 *__restrict__ bmap, u64 nb, u32 *__restrict__ final_state) {
    __shared__ u32 sh[TOP_T];
    __shared__ u32 carry;
    const u32 t = threadIdx.x;
    if (t == 0) carry = SR;
    __syncthreads();
    for (u64 c0 = 0; c0 < nb; c0 += (u64)TOP_T * TOP2_PER) {
        const u64 k0 = c0 + (u64)t * TOP2_PER;
        u32 x = MAP_ID;
        for (u32 k = 0; k < TOP2_PER; ++k)
            if (k0 + k < nb) x = compose(x, bmap[k0 + k]);
        sh[t] = x;
        __syncthreads();
        for (u32 o = 1; o < TOP_T; o <<= 1) {  // inclusive scan of the chunk composites
            const u32 y = t >= o ? sh[t - o] : MAP_ID;
            __syncthreads();
            x = compose(y, x);
            sh[t] = x;
            __syncthreads();
        }
        const u32 cin = carry;
        u32 st = ::step(t ? sh[t - 1] : MAP_ID, cin);
        for (u32 k = 0; k < TOP2_PER; ++k) {
            if (k0 + k >= nb) break;
            const u32 tm = bmap[k0 + k];
            bmap[k0 + k] = st;
            st = ::step(tm, st);
        }
        __syncthreads();
        if (t == TOP_T - 1) carry = ::step(sh[TOP_T - 1], cin);
        __syncthreads();
    }
    if (t == 0) *final_state = carry;
}

__global__ __launch_bounds__(BLK) void k_wcs_state_down(const u32 *__restrict__ map, const u64 *__restrict__ cnt6,
                                                        u64 nseg, const u32 *__restrict__ bstate,
                                                        u32 *__restrict__ sstate, u64 *__restrict__ cnt) {
    __shared__ u32 sh[BLK];
    const u64 s0 = (u64)blockIdx.x * BSEG + (u64)threadIdx.x * PER;
    u32 x = MAP_ID;
    for (u32 k = 0; k < PER; ++k)
        if (s0 + k < nseg) x = compose(x, map[s0 + k]);
    const u32 inc = block_map_scan(x, sh);
    const u32 excl = threadIdx.x ? sh[threadIdx.x - 1] : MAP_ID;
    (void)inc;
    u32 s = step(excl, bstate[blockIdx.x]);
    for (u32 k = 0; k < PER; ++k) {
        const u64 g = s0 + k;
        if (g >= nseg) break;
        sstate[g] = s;
        cnt[g] = (cnt6[g] >> (9 * s)) & 511u;
        s = step(map[g], s);
    }
}

struct EmitWalker {
    static constexpr bool single() { return true; }
    u32 s;
    u64 o;
    u64 *rend;
    __device__ __forceinline__ bool in_iq() const { return s == IQ; }
    __device__ __forceinline__ void step(u32 t) { s = ::step(t, s); }
    __device__ __forceinline__ void eol(u64 i) {
        if (s != SR && s != IQ) rend[o++] = i + 1;
        s = ::step(T_EOL, s);
    }
};

__global__ __launch_bounds__(256) void k_wcs_emit(const u8 *__restrict__ buf, u64 ds, u64 n, u64 nseg, Dia dia,
                                                  const u32 *__restrict__ sstate, const u64 *__restrict__ roff,
                                                  u64 *__restrict__ rend) {
    const u64 seg = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= nseg) return;
    EmitWalker wk{sstate[seg], roff[seg], rend};
    seg_walk(buf, seg * SEG, ds, n, dia, wk);
}

// ---------------------------------------------------------------------------
// Per-row pass.
struct ByteReader {
    const u32 *w;
    u64 wi;
    u32 cur;
    __device__ ByteReader(const u8 *buf) : w((const u32 *)buf), wi(~0ull), cur(0) {}
    __device__ __forceinline__ u32 get(u64 i) {
        const u64 k = i >> 2;
        if (k != wi) { wi = k; cur = w[k]; }
        return (cur >> (8 * (i & 3))) & 0xFFu;
    }
};

__host__ __device__ __forceinline__ bool tok_ascii(u32 c) {
    return (c >= '0' && c <= '9') || ((c | 0x20u) >= 'a' && (c | 0x20u) <= 'z') || c == '\'';
}
// second byte d of a 0xC3 pair: U+00C0..U+00FF minus U+00D7 / U+00F7
__host__ __device__ __forceinline__ bool tok_c3(u32 d) { return d >= 0x80 && d <= 0xBF && d != 0x97 && d != 0xB7; }
__host__ __device__ __forceinline__ u32 low_ascii(u32 c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
__host__ __device__ __forceinline__ u32 low_c3(u32 d) { return d <= 0x9E ? d + 32 : d; }

// Word hash: bytes are packed 8 at a time into a u64 and absorbed by two
// independent mixers (h1 = table key, h2 = check); one multiply pair per 8
// bytes instead of per byte.
struct TokHash {
    u64 h1, h2, acc;
    u32 nacc, len;
    __host__ __device__ __forceinline__ void reset() {
        h1 = 0xcbf29ce484222325ull; h2 = 0x2545F4914F6CDD1Dull; acc = 0; nacc = 0; len = 0;
    }
    __host__ __device__ __forceinline__ void absorb() {
        h1 = (h1 ^ acc) * 0x87c37b91114253d5ull;
        h1 = (h1 << 31) | (h1 >> 33);
        h2 = (h2 + acc) * 0x9E3779B97F4A7C15ull;
        h2 ^= h2 >> 32;
        acc = 0;
        nacc = 0;
    }
    __host__ __device__ __forceinline__ void add(u32 c) {
        acc |= (u64)c << (8 * nacc);
        ++len;
        if (++nacc == 8) absorb();
    }
    __host__ __device__ __forceinline__ u64 key() const {  // h1 of the finished word (nonzero)
        u64 x = h1;
        if (nacc) { x = (x ^ acc) * 0x87c37b91114253d5ull; x = (x << 31) | (x >> 33); }
        const u64 k = fmix64(x ^ ((u64)len * 0xD6E8FEB86659FD93ull));
        return k ? k : 1;
    }
    __host__ __device__ __forceinline__ u64 check() const {  // h2 of the finished word (nonzero)
        u64 x = h2;
        if (nacc) { x = (x + acc) * 0x9E3779B97F4A7C15ull; x ^= x >> 32; }
        const u64 k = fmix64(x + len);
        return k ? k : 1;
    }
};

struct RowArgs {
    const u8 *buf;
    u64 n;
    const u64 *rend;
    u64 ds;
    u64 nrows;
    u32 ia, isg, it, need;
    u32 delim;      // the field delimiter byte (',' unless sniffed / given otherwise)
    u64 *gtab;      // 4 u64 per slot: key, h2 of the word, ~first (pos << 20 | raw len), count
    u64 gmask;
    u64 glimit;
    u64 *scratch;   // per-row work areas, row at scratch + 2 * row start (3 tmax + 2 ntok <= 2 L)
    u64 *nd;        // distinct words per row
    u64 *spans;     // 4 per row: artist start/end, song start/end (raw)
    WCtr *ctr;
    const u64 *rows;  // k_wcs_rows: the rows to walk (null: every row)
    u64 *fb;          // k_wcs_wrows: rows it leaves to k_wcs_rows
    int ablate;     // timing diagnostics only (MSA_WCS_ABLATE): 1 no token loop, 4 no per-row
                    // table, 8 no wave-per-row pass, 16 (wave pass) no global slot claim (no
                    // words: nothing to rank), 32 neither the claim nor the workgroup aggregate
                    // -- results are wrong when set
};

// The token's h2 against its slot's (set once by the first CAS); a second,
// independent 64-bit hash, so a mismatch is a 64-bit h1 collision.
__device__ __forceinline__ void h2_check(const RowArgs &a, u64 *gt, u64 seen, u64 h2v) {
    if (seen == 0) seen = atomicCAS((unsigned long long *)(gt + 1), 0ull, (unsigned long long)h2v);
    if (seen != 0 && seen != h2v) atomicAdd((unsigned long long *)&a.ctr->collision, 1ull);
}
// Global slot of a word: `cur` = the (key, h2) pair at key & gmask, loaded by
// the caller (its load can be in flight while the caller does LDS work).
__device__ __forceinline__ ulonglong2 g_probe(const RowArgs &a, u64 key) {
    return *(const ulonglong2 *)(a.gtab + (key & a.gmask) * 4);  // plain (cached) load: a key never
                                                                 // changes once set; a stale 0 goes to the CAS
}
__device__ __forceinline__ u64 g_insert(const RowArgs &a, u64 key, u64 h2v, ulonglong2 cur) {
    u64 slot = key & a.gmask;
    for (u64 p = 0; p <= a.gmask; ++p) {
        u64 *k = a.gtab + slot * 4;
        if (cur.x == key) { h2_check(a, k, cur.y, h2v); return slot; }
        if (cur.x == 0) {
            const u64 old = atomicCAS((unsigned long long *)k, 0ull, (unsigned long long)key);
            if (old == 0) {
                const u64 d = atomicAdd((unsigned long long *)&a.ctr->distinct, 1ull);
                if (d >= a.glimit) atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_G);
                h2_check(a, k, 0, h2v);
                return slot;
            }
            if (old == key) { h2_check(a, k, 0, h2v); return slot; }
        }
        slot = (slot + 1) & a.gmask;
        cur = *(const ulonglong2 *)(a.gtab + slot * 4);
    }
    atomicOr((unsigned long long *)&a.ctr->overflow, (unsigned long long)OVF_G);
    return ~0ull;
}

__device__ __forceinline__ void wcs_err(WCtr *ctr, u64 row, u32 code) {
    atomicMin((unsigned long long *)&ctr->err, (unsigned long long)((row << 8) | code));
}

// Workgroup-private aggregation of the global word updates (the Zipf head
// would otherwise serialise every token on a few device-scope atomics): per
// word seen by the workgroup, LDS holds the count and the max of ~first.
// Flushed once per workgroup.  (The h2 check is g_insert's.)
constexpr u32 LW = 2048, LW_PROBE = 8;
struct WgAgg {
    u32 *id;
    u32 *cnt;
    u64 *first;
    u64 *rows;  // [0] rows, [1] song rows, [2] tokens
};

template <u32 N = LW>
__device__ __forceinline__ void word_update(const RowArgs &a, WgAgg &g, u64 slot, u64 nfirst) {
    static_assert((N & (N - 1)) == 0 && N >= 256, "LDS aggregate size");
    const u32 id = (u32)slot + 1;
    u32 h = (id * 0x9E3779B1u) >> (32 - __builtin_ctz(N));
    for (u32 p = 0; p < LW_PROBE; ++p, h = (h + 1) & (N - 1)) {
        u32 cur = g.id[h];
        if (cur == 0) {
            const u32 old = atomicCAS(&g.id[h], 0u, id);
            cur = old == 0 ? id : old;
        }
        if (cur != id) continue;
        atomicAdd(&g.cnt[h], 1u);
        // first changes rarely: a plain LDS read filters out most atomics
        if (nfirst > g.first[h]) atomicMax((unsigned long long *)&g.first[h], (unsigned long long)nfirst);
        return;
    }
    u64 *gt = a.gtab + slot * 4;  // LDS table full here: straight to HBM
    atomicAdd((unsigned long long *)(gt + 3), 1ull);
    atomicMax((unsigned long long *)(gt + 2), (unsigned long long)nfirst);
}

// flush of a workgroup's aggregate
__device__ __forceinline__ void agg_flush(const RowArgs &a, const WgAgg &g, u32 n) {
    for (u32 k = threadIdx.x; k < n; k += blockDim.x) {
        const u32 id = g.id[k];
        if (!id) continue;
        u64 *gt = a.gtab + (u64)(id - 1) * 4;
        atomicAdd((unsigned long long *)(gt + 3), (unsigned long long)g.cnt[k]);
        atomicMax((unsigned long long *)(gt + 2), (unsigned long long)g.first[k]);
    }
    if (threadIdx.x == 0) {
        atomicAdd((unsigned long long *)&a.ctr->total_rows, (unsigned long long)g.rows[0]);
        atomicAdd((unsigned long long *)&a.ctr->song_rows, (unsigned long long)g.rows[1]);
        atomicAdd((unsigned long long *)&a.ctr->tokens, (unsigned long long)g.rows[2]);
    }
}

__device__ __forceinline__ void wcs_row(const RowArgs &a, WgAgg &agg, u64 r) {
    const u64 rs = a.rend[r - 1], re = a.rend[r];
    ByteReader rd(a.buf);
    u32 s = SR, f = 0, chars = 0;
    bool any = false;  // a field was saved (blank rows have none)
    u64 fstart = rs;
    u64 sp[4] = {0, 0, 0, 0};
    // tokenizer over the added characters of field `it`
    bool in_tok = false, alnum = false, skip = false;
    u32 cps = 0;
    TokHash th;
    th.reset();
    u64 tstart = 0;
    // scratch of this row (u64 units, disjoint from every other row's):
    //   [0, 3*tmax)            token records (h1, h2, ~first) from the byte walk;
    //                          its front is reused as the u32 order->slot list
    //   [tmax, tmax + nd)      the row's (word id, count) lines in order
    //   [3*tmax, +2*ntok)      per-row hash table (id, order, count)
    u64 *sc = a.scratch + 2 * rs;
    const u64 tmax = (re - rs) / 4 + 1;
    u32 nd = 0, ntok = 0;
    bool limit = false;

    auto tok_end = [&](u64 end) {
        if (in_tok && cps >= 3 && alnum) {  // record only: the walk stays free of memory round trips
            u64 *t = sc + 3 * (u64)ntok++;
            t[0] = th.key();
            t[1] = th.check();
            t[2] = ~((tstart << 20) | (end - tstart));
        }
        in_tok = false;
    };
    auto save = [&](u64 end) {
        if (f == a.it) tok_end(end);
        if (f == a.ia) { sp[0] = fstart; sp[1] = end; }
        if (f == a.isg) { sp[2] = fstart; sp[3] = end; }
        ++f;
        chars = 0;
        any = true;
    };
    auto add = [&](u64 i, u32 b) {
        if ((b & 0xC0) != 0x80 && ++chars > FIELD_LIMIT) limit = true;
        if (f != a.it) return;
        if (skip) { skip = false; return; }
        u32 lo0 = 0, lo1 = 0, nb = 0;
        if (b < 0x80 && tok_ascii(b)) { lo0 = low_ascii(b); nb = 1; }
        else if (b == 0xC3) {
            const u32 d = rd.get(i + 1);
            if (tok_c3(d)) { lo0 = 0xC3; lo1 = low_c3(d); nb = 2; skip = true; }
        }
        if (!nb) { tok_end(i); return; }
        if (!in_tok) { in_tok = true; alnum = false; cps = 0; th.reset(); tstart = i; }
        th.add(lo0);
        if (nb == 2) th.add(lo1);
        alnum |= b != '\'';
        ++cps;
    };

    // 16-byte SWAR blocks: quote/comma/CR/LF bytes (and the input's last byte)
    // go through the reader's table step one by one; a run of other bytes is
    // one (idempotent) T_O step -- its bytes are all added to the field: fed
    // to the tokenizer in the text field, only counted in the others
    for (u64 b0 = rs & ~15ull; b0 < re; b0 += 16) {
        const uint4 v = *(const uint4 *)(a.buf + b0);
        u32 vm = 0xFFFFu;
        if (b0 < rs) vm &= 0xFFFFu << (u32)(rs - b0);
        if (b0 + 16 > re) vm &= (1u << (u32)(re - b0)) - 1u;
        const u32 S = (mask16(v, '"') | mask16(v, a.delim) | mask16(v, '\n') | mask16(v, '\r')) & vm;
        const u32 O = vm & ~S;
        u32 E = S;
        if (b0 + 16 >= a.n && a.n > b0 && ((vm >> (u32)(a.n - 1 - b0)) & 1u)) E |= 1u << (u32)(a.n - 1 - b0);
        auto run = [&](u32 m) {
            if (!m) return;
            if (s == SR) fstart = b0 + (u32)__builtin_ctz(m);
            if (f == a.it) {
                for (u32 mm = m; mm; mm &= mm - 1) {
                    const u32 p = (u32)__builtin_ctz(mm);
                    add(b0 + p, byte_of(v, p));
                }
            } else {
                const u32 W[4] = {v.x, v.y, v.z, v.w};
                u32 cont = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) cont |= swar_pack4(W[k] & ~(W[k] << 1) & 0x80808080u) << (4 * k);
                chars += (u32)__popc(m & ~cont);
                if (chars > FIELD_LIMIT) limit = true;
            }
            s = step(T_O, s);
        };
        int prev = -1;
        while (E) {
            const u32 p = (u32)__builtin_ctz(E);
            E &= E - 1;
            run(O & ((1u << p) - 1u) & ~(prev < 0 ? 0u : ((2u << prev) - 1u)));
            const u32 b = byte_of(v, p);
            const u64 i = b0 + p;
            // end of line: after '\n', after '\r' not followed by '\n', after the last byte
            bool eol = i + 1 == a.n;
            if (b == '\n') eol = true;
            else if (b == '\r' && !eol) eol = (p < 15 ? byte_of(v, p + 1) : (u32)a.buf[i + 1]) != '\n';
            const u32 cls = b == '"' ? 0u : (b == a.delim ? 1u : ((b == '\r' || b == '\n') ? 2u : 3u));
            const u32 tnext = cls == 0 ? T_Q : (cls == 1 ? T_D : (cls == 2 ? T_NL : T_O));
            const u32 tact = cls == 0 ? A_Q : (cls == 1 ? A_D : (cls == 2 ? A_NL : A_O));
            const u32 act = (tact >> (2 * s)) & 3u;
            if (s == SR && cls != 2) fstart = i;
            if (act & 2u) {
                save(i);
                if (cls == 1) fstart = i + 1;
            }
            if (act & 1u) add(i, b);
            s = step(tnext, s);
            if (eol) {
                if (s == SF || s == IF || s == QQ) save(i + 1);
                if (s != IQ) s = SR;
            }
            prev = (int)p;
        }
        run(O & ~(prev < 0 ? 0u : ((2u << prev) - 1u)));
    }
    if (s == IQ) save(re);  // input ended inside a quoted field
    if (limit) wcs_err(a.ctr, r, E_LIMIT);
    if (!any) { a.nd[r] = 0; return; }  // blank line: DictReader skips it
    // tokens -> global table (via the workgroup aggregate) and per-row table;
    // every lane runs the same loop, one iteration per token
    if (ntok && !(a.ablate & 1)) {
        const u32 rcap = 2 * ntok;
        u64 *rt = sc + 3 * tmax;
        u32 *list = (u32 *)sc;
        for (u32 k = 0; k < rcap; ++k) rt[k] = 0;
        for (u32 t = 0; t < ntok; ++t) {
            const u64 key = sc[3 * t], h2v = sc[3 * t + 1], nfirst = sc[3 * t + 2];
            const u64 slot = g_insert(a, key, h2v, g_probe(a, key));
            if (slot == ~0ull) continue;  // overflow: the run repeats with a larger table
            word_update(a, agg, slot, nfirst);
            if (a.ablate & 4) continue;
            const u64 id = slot + 1;
            u32 h = (u32)(((id * 0x9E3779B97F4A7C15ull) >> 32) % rcap);
            for (;;) {
                const u64 v = rt[h];
                if (v == 0) { rt[h] = (id << 32) | 1u; list[nd++] = h; break; }
                if ((v >> 32) == id) { rt[h] = v + 1; break; }
                h = h + 1 == rcap ? 0 : h + 1;
            }
        }
        for (u32 k = 0; k < nd; ++k) sc[tmax + k] = rt[list[k]];
    }
    atomicAdd((unsigned long long *)&agg.rows[0], 1ull);
    if (f <= a.need) wcs_err(a.ctr, r, E_SHORT);
    a.nd[r] = nd;
    if (nd) {
        atomicAdd((unsigned long long *)&agg.rows[1], 1ull);
        atomicAdd((unsigned long long *)&agg.rows[2], (unsigned long long)ntok);  // counted tokens
    }
    u64 *o = a.spans + r * 4;
    o[0] = sp[0]; o[1] = sp[1]; o[2] = sp[2]; o[3] = sp[3];
}

__global__ __launch_bounds__(256) void k_wcs_rows(RowArgs a) {
    __shared__ u32 l_id[LW], l_cnt[LW];
    __shared__ u64 l_first[LW], l_rows[4];
    for (u32 k = threadIdx.x; k < LW; k += blockDim.x) { l_id[k] = 0; l_cnt[k] = 0; l_first[k] = 0; }
    if (threadIdx.x < 4) l_rows[threadIdx.x] = 0;
    __syncthreads();
    WgAgg agg{l_id, l_cnt, l_first, l_rows};
    // row k of the file spans [rend[k], rend[k+1]); kernel index r = k + 1,
    // r = 1 is the header row
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 r = a.rows ? (i < a.ctr->fallback ? a.rows[i] : a.nrows) : i + 2;
    if (r < a.nrows) wcs_row(a, agg, r);
    __syncthreads();
    agg_flush(a, agg, LW);
}

// ---------------------------------------------------------------------------
// Wave-per-window pass (the common case; k_wcs_rows walks what it leaves).
// A wave takes WR_ROWS consecutive rows and cuts them into windows: as many
// whole rows (at most WR_M) as fit in 1 KiB from the first row's 16-byte
// aligned start, 16 bytes per lane, classified with SWAR masks.  A row's
// quoting is "standard" when every '"' sits where the reader's quote parity
// predicts a structural or doubled quote:
//   * a quote outside quotes (parity 0) follows the row start, a delimiter or
//     another quote (the second of a doubled pair),
//   * a quote inside quotes is followed by a quote, a delimiter, an end of line
//     or the row end,
//   * the row starts and ends outside quotes, and ends of line outside quotes
//     are only the row's own terminator.
// Then parity 0 <=> the reader is outside a quoted field, the fields are
// split by the delimiters at parity 0, no quote lies inside a token (so a
// token's raw span is its bytes), and every quote is a token separator like
// the character it stands for.  Other rows (and rows over 1 KiB, or all rows
// of a window with more than WR_TCAP token runs) go to the fallback list,
// before anything of theirs is committed.  Per-row values (delimiter counts,
// field bounds, flags) are reduced through small LDS arrays indexed by the
// row's place in the window (row-start bits + prefix counts give a byte's
// row).  Tokens: one lane per token (start / end from LDS) hashes its
// lower-cased bytes (same TokHash as k_wcs_rows), claims the global slot and
// updates the workgroup aggregate; the rows' Counters share one per-wave LDS
// table keyed by (row, h1) -- the row in h1's top 5 bits, so two words of one
// window merge only if their 64-bit keys agree in the other 59 -- written out
// in first-occurrence order.
#ifndef WR_LW
#define WR_LW 4096  // workgroup aggregate of k_wcs_wrows (2048 at 2 workgroups per CU 12.66 ms, 1024 at 3: 14.2)
#endif
#ifndef WR_WAVES
#define WR_WAVES 10  // waves per workgroup (LDS: 10 x 9 KiB + the 64 KiB aggregate; 8 waves: 12.28 vs 11.67 ms)
#endif
#ifndef WR_GPC
#define WR_GPC 1    // resident workgroups per CU (LDS: 152 KiB)
#endif
constexpr u32 WR_W = WR_WAVES, WR_ROWS = 64, WR_M = 32, WR_TCAP = 192, WR_DCAP = 256;
struct WrWave {
    u64 key[WR_DCAP];      // (row, h1)
    u32 slot[WR_DCAP];     // its global slot
    u32 cnt[WR_DCAP];
    u32 first[WR_DCAP];    // order of the first token
    u32 row[264];          // the window (1 KiB) + 32 bytes of zeros
    u32 rbits[64];         // row-start bits per lane
    u32 tgl[64];           // text-field start / end toggles per lane
    u16 ts[WR_TCAP], te[WR_TCAP];
    // per row of the window
    u32 db[WR_M + 1];      // delimiters outside quotes before the row ([m]: all)
    u32 flag[WR_M];        // 1 bad, 2 blank, 4 odd quote parity at the row start
    u32 eol[WR_M];         // first end-of-line byte outside quotes, else the row end
    u32 fp[WR_M][6];       // start / end of the artist, song, text fields
    u32 lb[WR_M];          // rank of the row's first line in the window
    u32 nd[WR_M];          // its lines
    u32 nv[WR_M];          // its counted tokens
};

__device__ __forceinline__ u32 wr_mask(u64 lb, u64 lo, u64 hi) {  // bits j with lb + j in [lo, hi)
    const u64 a = lo > lb ? (lo - lb < 16 ? lo - lb : 16) : 0;
    const u64 b = hi > lb ? (hi - lb < 16 ? hi - lb : 16) : 0;
    return ((1u << b) - 1u) & ~((1u << a) - 1u);
}
// 0x80 per byte in [0x41, 0x5A] or [0x80, 0x9E] (the bytes a token lower-cases by + 0x20)
__device__ __forceinline__ u32 swar_upper(u32 x) {
    const u32 x7 = x & 0x7F7F7F7Fu;
    const u32 up = (x7 + 0x3F3F3F3Fu) & ~(x7 + 0x25252525u) & ~x;
    const u32 c3 = ~(x7 + 0x61616161u) & x;
    return (up | c3) & 0x80808080u;
}
__device__ __forceinline__ u64 shfl64(u64 x, u32 l) {
    return ((u64)(u32)__shfl((int)(x >> 32), (int)l) << 32) | (u32)__shfl((int)(u32)x, (int)l);
}

struct WrCount {
    u64 rows, song, tok;
};

// One window: rows i .. i + m - 1 of the wave's set (row i + j owned by lane j),
// bytes [base, base + 1024) in v.  rsj / rej: the owner lane's row bounds.
__device__ __forceinline__ void wr_window(const RowArgs &a, WgAgg &agg, WrWave &W, u64 r_first, u32 m, u64 base,
                                          u64 rsj, u64 rej, uint4 v, WrCount &cnt) {
    const u32 lane = lane_id();
    const u64 lb = base + 16 * lane;
    const u64 ws = readlane64(rsj, 0), we = readlane64(rej, (int)m - 1);
    const u32 V = wr_mask(lb, ws, we);
    const bool own = lane < m;
    const u32 fi[3] = {a.ia, a.isg, a.it};
    // ---- row starts, per-row defaults
    W.rbits[lane] = 0;
    W.tgl[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    if (own) {
        const u32 o = (u32)(rsj - base);
        atomicOr(&W.rbits[o >> 4], 1u << (o & 15));
        W.flag[lane] = 0;
        W.eol[lane] = (u32)(rej - base);
        W.nd[lane] = 0;
        W.nv[lane] = 0;
        W.lb[lane] = ~0u;
#pragma unroll
        for (int f = 0; f < 3; ++f) { W.fp[lane][2 * f] = fi[f] == 0 ? o : 0u; W.fp[lane][2 * f + 1] = ~0u; }
    }
    __builtin_amdgcn_wave_barrier();
    const u32 RB = W.rbits[lane];
    // ---- classes
    const u32 w[4] = {v.x, v.y, v.z, v.w};
    u32 Q = 0, D = 0, E = 0, C3 = 0, T2 = 0, TA = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const u32 x = w[k], x7 = x & 0x7F7F7F7Fu;
        Q |= swar_pack4(eq80x(x, x7, '"')) << (4 * k);
        D |= swar_pack4(eq80x(x, x7, a.delim)) << (4 * k);
        E |= swar_pack4(eq80x(x, x7, '\n') | eq80x(x, x7, '\r')) << (4 * k);
        TA |= swar_pack4(tok80x(x, x7)) << (4 * k);
        C3 |= swar_pack4(swar_eq(x, 0xC3)) << (4 * k);
        // second byte of a token 0xC3 pair: 0x80..0xBF minus 0x97 / 0xB7
        T2 |= swar_pack4(x & ~(x << 1) & 0x80808080u & ~swar_eq(x, 0x97) & ~swar_eq(x, 0xB7)) << (4 * k);
    }
    Q &= V; D &= V; E &= V; C3 &= V; T2 &= V; TA &= V;
    // neighbours: bit 15 of the lane below, bits 0-1 of the lane above
    const u32 lo_bits = (D >> 15) | ((Q >> 15) << 1) | ((C3 >> 15) << 2);
    const u32 hi_bits = (Q & 1u) | ((D & 1u) << 1) | ((E & 1u) << 2) | ((T2 & 1u) << 3) | ((RB & 3u) << 4);
    u32 pb = __shfl_up(lo_bits, 1), nb = __shfl_down(hi_bits, 1);
    if (lane == 0) pb = 0;
    if (lane == 63) nb = 0;
    // quote parity before each byte
    const u64 qodd = __ballot(__popc(Q) & 1u);
    const u32 carry = (u32)__popcll(qodd & ((1ull << lane) - 1ull)) & 1u;
    const u32 P = pxor_excl16(Q) ^ (carry ? 0xFFFFu : 0u);
    // last and second-to-last byte of each row
    const u32 END = (((RB >> 1) | (((nb >> 4) & 1u) << 15)) & V) | wr_mask(lb, we - 1, we);
    const u32 END2 = (((RB >> 2) | (((nb >> 4) & 3u) << 14)) & V) | wr_mask(lb, we - 2, we - 1);
    const u32 prevD = (D << 1) | (pb & 1u), prevQ = (Q << 1) | ((pb >> 1) & 1u);
    const u32 nextQ = (Q >> 1) | ((nb & 1u) << 15), nextD = (D >> 1) | (((nb >> 1) & 1u) << 15);
    const u32 nextE = (E >> 1) | (((nb >> 2) & 1u) << 15);
    const u32 E0 = E & ~P, D0 = D & ~P;
    const u32 bad = (Q & ~P & ~(prevD | prevQ | RB)) | (Q & P & ~(nextQ | nextD | nextE | END)) |
                    (E0 & ~(END | END2));
    // a byte's row: rows started at or before it
    u32 nrows_tot, nd_tot;
    const u32 rpre = wave_prefix<6>((u32)__popc(RB), nrows_tot);
    const u32 dpre = wave_prefix<5>((u32)__popc(D0), nd_tot);
    for (u32 mm = bad; mm; mm &= mm - 1) {
        const u32 b = (u32)__builtin_ctz(mm);
        atomicOr(&W.flag[rpre + __popc(RB & ((2u << b) - 1u)) - 1], 1u);
    }
    for (u32 mm = RB, j = rpre; mm; mm &= mm - 1, ++j) {
        const u32 b = (u32)__builtin_ctz(mm);
        const u32 fl = (((P >> b) & 1u) << 2) | (((E0 >> b) & 1u) << 1);
        if (fl) atomicOr(&W.flag[j], fl);
        W.db[j] = dpre + __popc(D0 & ((1u << b) - 1u));
    }
    if (lane == 0) W.db[m] = nd_tot;
    __builtin_amdgcn_wave_barrier();
    // ---- fields
    for (u32 mm = D0, g = dpre; mm; mm &= mm - 1, ++g) {
        const u32 b = (u32)__builtin_ctz(mm);
        const u32 j = rpre + __popc(RB & ((2u << b) - 1u)) - 1;
        const u32 idx = g - W.db[j], pos = 16 * lane + b;
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            if (idx + 1 == fi[f]) W.fp[j][2 * f] = pos + 1;
            if (idx == fi[f]) W.fp[j][2 * f + 1] = pos;
        }
    }
    for (u32 mm = E0; mm; mm &= mm - 1) {
        const u32 b = (u32)__builtin_ctz(mm);
        atomicMin(&W.eol[rpre + __popc(RB & ((2u << b) - 1u)) - 1], 16 * lane + b);
    }
    __builtin_amdgcn_wave_barrier();
    u32 nf = 0, rflag = 0;
    if (own) {
        const u32 fl = W.flag[lane];
        const bool odd_end = lane + 1 < m ? (W.flag[lane + 1] & 4u) != 0 : (__popcll(qodd) & 1) != 0;
        rflag = ((fl & 5u) || odd_end) ? 1u : (fl & 2u);
        nf = W.db[lane + 1] - W.db[lane] + 1;
        const u32 eo = W.eol[lane];
#pragma unroll
        for (int f = 0; f < 3; ++f)
            if (W.fp[lane][2 * f + 1] == ~0u) W.fp[lane][2 * f + 1] = eo;
        if (rflag == 0 && nf > a.it) {
            const u32 ts = W.fp[lane][4], te = W.fp[lane][5];
            // a last row without a newline can end at window byte 1023 with
            // an empty text field: then ts == 1024, outside the window
            if (ts < 1024) atomicXor(&W.tgl[ts >> 4], 1u << (ts & 15));
            if (te < 1024) atomicXor(&W.tgl[te >> 4], 1u << (te & 15));
        }
    }
    __builtin_amdgcn_wave_barrier();
    // ---- tokens of the text fields
    u32 R = W.tgl[lane];
    const u32 tcarry = (u32)__popcll(__ballot(__popc(R) & 1u) & ((1ull << lane) - 1ull)) & 1u;
    R ^= R << 1; R ^= R << 2; R ^= R << 4; R ^= R << 8;
    R = (R ^ (tcarry ? 0xFFFFu : 0u)) & V;
    const u32 lead = C3 & ((T2 >> 1) | (((nb >> 3) & 1u) << 15));
    const u32 sec = T2 & ((C3 << 1) | ((pb >> 2) & 1u));
    const u32 TB = (TA | lead | sec) & R;
    u32 pt = __shfl_up(TB >> 15, 1), nt = __shfl_down(TB & 1u, 1);
    if (lane == 0) pt = 0;
    if (lane == 63) nt = 0;
    const u32 TS = TB & ~((TB << 1) | pt), TE = TB & ~((TB >> 1) | (nt << 15));
    u32 ntok, tot_e;
    const u32 tpre = wave_prefix<5>((u32)__popc(TS), ntok);
    const bool over = ntok > WR_TCAP;  // every row of the window to the fallback
    u32 nval = 0, nlead = 0;
    if (!over) {
        const u32 je = wave_prefix<5>((u32)__popc(TE), tot_e);  // the k-th end closes the k-th start
        W.row[4 * lane] = v.x; W.row[4 * lane + 1] = v.y; W.row[4 * lane + 2] = v.z; W.row[4 * lane + 3] = v.w;
        if (lane < 8) W.row[256 + lane] = 0;
        for (u32 mm = TS, j = tpre; mm; mm &= mm - 1, ++j) {
            const u32 b = (u32)__builtin_ctz(mm);
            W.ts[j] = (u16)((16 * lane + b) | ((rpre + __popc(RB & ((2u << b) - 1u)) - 1) << 10));
        }
        for (u32 mm = TE, j = je; mm; mm &= mm - 1, ++j) W.te[j] = (u16)(16 * lane + (u32)__builtin_ctz(mm) + 1u);
        for (u32 k = lane; k < WR_DCAP; k += 64) { W.key[k] = 0; W.cnt[k] = 0; W.first[k] = ~0u; W.slot[k] = ~0u; }
        __builtin_amdgcn_wave_barrier();
        // one token per lane: lower-cased bytes hashed 8 at a time (TokHash)
        for (u32 t0 = 0; t0 < ntok; t0 += 64) {
            const u32 t = t0 + lane;
            bool ok = false;
            u64 key = 0, h2v = 0;
            u32 s = 0, len = 0, rj = 0;
            if (t < ntok) {
                const u32 tsv = W.ts[t];
                s = tsv & 1023u;
                rj = tsv >> 10;
                len = W.te[t] - s;
                TokHash th;
                th.reset();
                th.len = len;
                u32 c3 = 0;
                bool alnum = false;
                for (u32 off = 0; off < len; off += 8) {
                    const u32 q = (s + off) >> 2, sh = (s + off) & 3u;
                    const u32 w0 = W.row[q], w1 = W.row[q + 1], w2 = W.row[q + 2];
                    u32 x0 = __builtin_amdgcn_alignbyte(w1, w0, sh), x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
                    const u32 nbt = len - off < 8 ? len - off : 8;
                    const u32 k0 = nbt >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nbt)) - 1u);
                    const u32 k1 = nbt >= 8 ? 0xFFFFFFFFu : (nbt <= 4 ? 0u : ((1u << (8 * (nbt - 4))) - 1u));
                    x0 &= k0;
                    x1 &= k1;
                    c3 += __popc(swar_eq(x0, 0xC3) & k0 & 0x80808080u) + __popc(swar_eq(x1, 0xC3) & k1 & 0x80808080u);
                    alnum |= ((~swar_eq(x0, '\'') & k0) | (~swar_eq(x1, '\'') & k1)) & 0x80808080u;
                    x0 |= swar_upper(x0) >> 2;
                    x1 |= swar_upper(x1) >> 2;
                    th.acc = ((u64)x1 << 32) | x0;
                    if (nbt == 8) th.absorb();
                    else th.nacc = nbt;
                }
                ok = alnum && len - c3 >= 3;
                if (ok) { key = th.key(); h2v = th.check(); }
            }
            const u64 okm = __ballot(ok);
            const u32 ord = nval + mbcnt(okm);
            nval += (u32)__popcll(okm);
            u32 h = 0;
            if (ok) {
                const ulonglong2 cur = (a.ablate & 48) ? ulonglong2{0, 0} : g_probe(a, key);  // in flight
                const u64 rk = (key & ~(31ull << 59)) | ((u64)rj << 59);
                h = (u32)(rk >> 40) & (WR_DCAP - 1);
                for (;;) {
                    u64 c = W.key[h];
                    if (c == 0) {
                        const u64 old = atomicCAS((unsigned long long *)&W.key[h], 0ull, (unsigned long long)rk);
                        c = old == 0 ? rk : old;
                    }
                    if (c == rk) break;
                    h = (h + 1) & (WR_DCAP - 1);
                }
                atomicAdd(&W.cnt[h], 1u);
                atomicMin(&W.first[h], ord);
                atomicAdd(&W.nv[rj], 1u);
                const u64 slot = (a.ablate & 48) ? (key & a.gmask) : g_insert(a, key, h2v, cur);
                if (slot != ~0ull) {  // else overflow: the run repeats with a larger table
                    if (!(a.ablate & 32)) word_update<WR_LW>(a, agg, slot, ~(((base + s) << 20) | (u64)len));
                    // the same value from every token of the word; two words
                    // whose (row, h1) keys agree in the window's 59 hash bits
                    // but that own different global slots are a collision
                    // (detected and reported, like the global h1 check)
                    const u32 prev = atomicCAS(&W.slot[h], ~0u, (u32)slot);
                    if (prev != ~0u && prev != (u32)slot) atomicAdd((unsigned long long *)&a.ctr->collision, 1ull);
                }
            }
            if (t < ntok) { W.ts[t] = (u16)(h | (rj << 10)); W.te[t] = (u16)(ok ? ord : 0xFFFFu); }
        }
        __builtin_amdgcn_wave_barrier();
        // leaders (first tokens of a word in a row): window rank, row base, row count
        for (u32 t0 = 0; t0 < ntok; t0 += 64) {
            const u32 t = t0 + lane;
            bool ld = false;
            u32 rj = 0;
            if (t < ntok) {
                const u32 tsv = W.ts[t], ord = W.te[t];
                rj = tsv >> 10;
                ld = ord != 0xFFFFu && W.first[tsv & 1023u] == ord;
            }
            const u64 lm = __ballot(ld);
            if (ld) {
                atomicMin(&W.lb[rj], nlead + mbcnt(lm));
                atomicAdd(&W.nd[rj], 1u);
            }
            nlead += (u32)__popcll(lm);
        }
        __builtin_amdgcn_wave_barrier();
        // the rows' (word id, count) lines in first-occurrence order
        u32 nl = 0;
        for (u32 t0 = 0; t0 < ntok; t0 += 64) {
            const u32 t = t0 + lane;
            bool ld = false;
            u32 rj = 0, h = 0;
            if (t < ntok) {
                const u32 tsv = W.ts[t], ord = W.te[t];
                rj = tsv >> 10;
                h = tsv & 1023u;
                ld = ord != 0xFFFFu && W.first[h] == ord;
            }
            const u64 lm = __ballot(ld);
            const u64 r_s = shfl64(rsj, rj), r_e = shfl64(rej, rj);
            if (ld) {
                u64 *lines = a.scratch + 2 * r_s + (r_e - r_s) / 4 + 1;
                lines[nl + mbcnt(lm) - W.lb[rj]] = ((u64)(W.slot[h] + 1) << 32) | W.cnt[h];
            }
            nl += (u32)__popcll(lm);
        }
        __builtin_amdgcn_wave_barrier();
    }
    // ---- per row: fallback, blank, or nd / spans / counters
    if (own) {
        const u64 r = r_first + lane;
        if (rflag == 1 || (over && rflag == 0)) {
            const u64 i = atomicAdd((unsigned long long *)&a.ctr->fallback, 1ull);
            a.fb[i] = r;
        } else if (rflag == 2) {
            a.nd[r] = 0;
        } else {
            if (nf <= a.need) wcs_err(a.ctr, r, E_SHORT);
            const u32 nd = W.nd[lane];
            a.nd[r] = nd;
            u64 *sp = a.spans + r * 4;
            sp[0] = base + W.fp[lane][0]; sp[1] = base + W.fp[lane][1];
            sp[2] = base + W.fp[lane][2]; sp[3] = base + W.fp[lane][3];
            ++cnt.rows;
            if (nd) { ++cnt.song; cnt.tok += W.nv[lane]; }
        }
    }
    __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(WR_W * 64) void k_wcs_wrows(RowArgs a) {
    __shared__ u32 l_id[WR_LW], l_cnt[WR_LW];
    __shared__ u64 l_first[WR_LW], l_rows[4];
    __shared__ WrWave l_w[WR_W];
    for (u32 k = threadIdx.x; k < WR_LW; k += blockDim.x) { l_id[k] = 0; l_cnt[k] = 0; l_first[k] = 0; }
    if (threadIdx.x < 4) l_rows[threadIdx.x] = 0;
    __syncthreads();
    WgAgg agg{l_id, l_cnt, l_first, l_rows};
    const u32 lane = lane_id(), wv = threadIdx.x >> 6;
    WrWave &W = l_w[wv];
    WrCount cnt{0, 0, 0};
    for (u64 blk = (u64)blockIdx.x * WR_W + wv;; blk += (u64)gridDim.x * WR_W) {
        const u64 r0 = 2 + blk * WR_ROWS;
        if (r0 >= a.nrows) break;
        const u32 nr = (u32)(a.nrows - r0 < WR_ROWS ? a.nrows - r0 : WR_ROWS);
        // lane k: row r0 + k spans [s_k, e_k)
        const u64 s_k = lane < nr ? a.rend[r0 - 1 + lane] : 0;
        const u64 e_k = lane < nr ? a.rend[r0 + lane] : 0;
        // window starting at row i: rows i .. i + m - 1 (every one ends within
        // 1 KiB of the first's aligned start, at most WR_M)
        auto window = [&](u32 i, u64 &wbase) -> u32 {
            wbase = readlane64(s_k, (int)i) & ~15ull;
            const bool fit = lane >= i && lane < nr && lane < i + WR_M && e_k - wbase <= 1024;
            const u64 nf = ~__ballot(fit) >> i;  // first row past the window
            return nf ? (u32)__builtin_ctzll(nf) : 64u - i;
        };
        u32 i = 0;
        u64 base;
        u32 m = window(0, base);
        uint4 v = *(const uint4 *)(a.buf + base + 16 * lane);
        while (i < nr) {
            if (m == 0) {  // a row over 1 KiB
                if (lane == 0) {
                    const u64 k = atomicAdd((unsigned long long *)&a.ctr->fallback, 1ull);
                    a.fb[k] = r0 + i;
                }
                i += 1;
                if (i < nr) { m = window(i, base); v = *(const uint4 *)(a.buf + base + 16 * lane); }
                continue;
            }
            // the next window's bytes are in flight while this one is processed
            const u32 i2 = i + m;
            u64 base2 = 0;
            u32 m2 = 0;
            uint4 v2 = make_uint4(0, 0, 0, 0);
            if (i2 < nr) {
                m2 = window(i2, base2);
                v2 = *(const uint4 *)(a.buf + base2 + 16 * lane);
            }
            const u32 src = i + (lane < m ? lane : 0);
            wr_window(a, agg, W, r0 + i, m, base, shfl64(s_k, src), shfl64(e_k, src), v, cnt);
            i = i2;
            base = base2;
            m = m2;
            v = v2;
        }
    }
    cnt.rows = wave_sum64(cnt.rows);
    cnt.song = wave_sum64(cnt.song);
    cnt.tok = wave_sum64(cnt.tok);
    if (lane == 0 && cnt.rows) {
        atomicAdd((unsigned long long *)&l_rows[0], (unsigned long long)cnt.rows);
        atomicAdd((unsigned long long *)&l_rows[1], (unsigned long long)cnt.song);
        atomicAdd((unsigned long long *)&l_rows[2], (unsigned long long)cnt.tok);
    }
    __syncthreads();
    agg_flush(a, agg, WR_LW);
}

// ---------------------------------------------------------------------------
// Global ranking: most_common() = stable sort by count desc over the
// first-occurrence order, i.e. the key (count desc, first position asc).
__global__ __launch_bounds__(256) void k_wcs_list(const u64 *__restrict__ gtab, u64 nslots, WCtr *ctr,
                                                  u64 *__restrict__ K2, u64 *__restrict__ K1, u64 *__restrict__ K0,
                                                  u32 *__restrict__ V) {
    const u64 slot = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 *g = gtab + slot * 4;
    const bool used = slot < nslots && g[0] != 0;
    // one claim per wave (a claim per used slot on the one counter had
    // serialised: 256 us for 33 K words); the list order does not matter,
    // the sort keys are unique
    const u64 um = __ballot(used);
    if (!um) return;
    const u32 lead = (u32)__builtin_ctzll(um);
    u64 base = 0;
    if (lane_id() == lead) base = atomicAdd((unsigned long long *)&ctr->listed, (unsigned long long)__popcll(um));
    base = readlane64(base, (int)lead);
    if (!used) return;
    const u64 idx = base + mbcnt(um);
    K2[idx] = 0xFFFFFFFFull - g[3];
    K1[idx] = (~g[2]) >> 20;
    K0[idx] = 0;
    V[idx] = (u32)slot;
}

// Word bytes of rank i: the first occurrence's raw span without its (at most
// one, structural) '"', lower-cased; re-hashed to check the slot's key and h2 sum.
__global__ __launch_bounds__(256) void k_wcs_wordlen(const u8 *__restrict__ buf, const u64 *__restrict__ gtab,
                                                     const u32 *__restrict__ order, u64 nw, u32 *__restrict__ rank_of,
                                                     u64 *__restrict__ len, u32 *__restrict__ counts, WCtr *ctr) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nw) return;
    const u32 slot = order[i];
    const u64 *g = gtab + (u64)slot * 4;
    const u64 fe = ~g[2];
    const u64 pos = fe >> 20, raw = fe & ((1u << 20) - 1);
    TokHash th;
    th.reset();
    for (u64 k = 0; k < raw; ++k) {
        const u32 b = buf[pos + k];
        if (b == '"') continue;
        u32 c;
        if (b == 0xC3) c = 0xC3;
        else if (k > 0 && buf[pos + k - 1] == 0xC3) c = low_c3(b);
        else c = low_ascii(b);
        th.add(c);
    }
    const u64 cnt = g[3];
    const u64 l = th.len;
    if (th.key() != g[0] || th.check() != g[1])
        atomicAdd((unsigned long long *)&ctr->collision, 1ull);
    rank_of[slot] = (u32)i;
    len[i] = l;
    counts[i] = (u32)cnt;
}

__global__ __launch_bounds__(256) void k_wcs_wordblob(const u8 *__restrict__ buf, const u64 *__restrict__ gtab,
                                                      const u32 *__restrict__ order, u64 nw,
                                                      const u64 *__restrict__ off, u8 *__restrict__ blob,
                                                      WCtr *ctr) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nw) return;
    const u64 fe = ~gtab[(u64)order[i] * 4 + 2];
    const u64 pos = fe >> 20, raw = fe & ((1u << 20) - 1);
    const u64 o0 = off[i];
    u64 j = o0;
    u32 prev = 0;
    for (u64 k = 0; k < raw; ++k) {
        const u32 b = buf[pos + k];
        const u32 c = b == 0xC3 ? b : (prev == 0xC3 ? low_c3(b) : low_ascii(b));
        prev = b;
        if (b != '"') blob[j++] = (u8)c;
    }
    if (j != off[i + 1]) atomicAdd((unsigned long long *)&ctr->collision, 1ull);
}

// by-song lines of row r at poff[r] + k: (rank << 32) | count
__global__ __launch_bounds__(256) void k_wcs_pairs(const u64 *__restrict__ rend, u64 nrows,
                                                   const u64 *__restrict__ nd, const u64 *__restrict__ poff,
                                                   const u64 *__restrict__ scratch, const u32 *__restrict__ rank_of,
                                                   u64 *__restrict__ pairs) {
    // One wave covers 64 consecutive rows and writes their lines [wbeg, wend)
    // contiguously: lane-strided over the lines, each lane finds the owning
    // row by a binary search over the lanes' first-line offsets (shuffles), so
    // stores are coalesced and reads run along each row's compact area.
    const u32 lane = lane_id();
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x + 2;
    const bool act = r < nrows;
    const u64 p0 = act ? poff[r] : ~0ull;
    const u64 cnt = act ? nd[r] : 0;
    const u64 rs = act ? rend[r - 1] : 0, re = act ? rend[r] : 0;
    const u64 cbase = act ? 2 * rs + (re - rs) / 4 + 1 : 0;
    const u64 wbeg = readlane64(p0, 0);
    if (wbeg == ~0ull) return;  // no row of this wave exists (wave-uniform)
    u64 wend = act ? p0 + cnt : 0;
    for (int o = 32; o > 0; o >>= 1) wend = max(wend, (u64)__shfl_xor(wend, o));
    const u64 iters = (wend - wbeg + 63) / 64;
    for (u64 it = 0; it < iters; ++it) {
        const u64 p = wbeg + it * 64 + lane;
        int l = 0;
        for (int st = 32; st > 0; st >>= 1) {
            const u64 v = __shfl(p0, l + st);
            if (v <= p) l += st;
        }
        const u64 k0 = __shfl(p0, l), cb = __shfl(cbase, l);
        if (p < wend) {
            const u64 v = scratch[cb + (p - k0)];
            pairs[p] = ((u64)rank_of[(v >> 32) - 1] << 32) | (v & 0xFFFFFFFFu);
        }
    }
}

// ---------------------------------------------------------------------------
// Column splitter (/root/reference/scripts/split_csv_columns.py main 124-199):
// csv.reader rows (blank lines are rows with no fields) -> one file body per
// column, each value written by csv.writer([value]) with lineterminator "\n",
// QUOTE_MINIMAL: quoted when it holds ',', '"' or '\n' (quotes doubled), and
// a lone empty value is written as "".  Fields past ncols are dropped, missing
// ones are "".  Pass 0 computes each (column, row) output length (+ a quoted
// flag), pass 1 writes the bytes at the scanned offsets (column-major, so the
// columns end up contiguous one after another).
struct ColArgs {
    const u8 *buf;
    u64 n;
    const u64 *rend;
    u64 first, nrows;  // kernel rows [first, nrows)
    u64 ncols, R;      // R = rows per column block
    u64 *len;          // [ncols * R]
    u8 *quoted;        // [ncols * R]
    const u64 *off;    // [ncols * R] (pass 1)
    u8 *out;
    WCtr *ctr;
    Dia dia;           // the reader's dialect; the writer quotes with its delimiter and quotechar
    u64 *src;          // [ncols * R]: a raw-copy value's source bytes (pass 0, CC_RAW)
    u64 *fix;          // rows with a value that is not a raw copy (pass 0 lists them, pass 1 walks them)
    u64 *nfix;
};

// Raw copies (CC_RAW): most values are written exactly as they stand in the
// input -- an unquoted value that needs no quoting, or a quoted one that
// needs quoting (the reader's and the writer's quotechar and doubling agree),
// its quotes included -- so pass 0 records each value's source and whether
// it is such a copy, a segmented gather (k_col_gather, msa_post.hip) copies
// every column's lines with coalesced 16-byte stores, and pass 1 walks only
// the rows holding another value, writing those values over the gather's.
// (Pass 1 over every row, one thread a row through an 8-byte write combiner,
// had been latency-bound: 4.4 ms for configs[2]'s 5 M rows.)
#ifndef CC_RAW
#define CC_RAW 1
#endif
template <int PASS>
__global__ __launch_bounds__(256) void k_csvcol(ColArgs a) {
    u64 r;
    if (PASS == 1 && a.fix) {
        const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= *a.nfix) return;
        r = a.fix[i];
    } else {
        r = (u64)blockIdx.x * blockDim.x + threadIdx.x + a.first;
        if (r >= a.nrows) return;
    }
    const u64 rs = a.rend[r - 1], re = a.rend[r];
    const u64 j = r - a.first;  // output row
    u32 s = SR, chars = 0;
    u64 f = 0, clen = 0;
    bool special = false, limit = false;
    // write combiner: byte stores up to an 8-byte boundary, then whole u64s
    u8 *dst = nullptr;
    u64 acc = 0;
    u32 nacc = 0;
    bool q = false;
    bool wr = true;  // pass 1: this value is written here (not a raw copy)
    // pass 0, raw-copy tracking: the value's first source byte (its opening
    // quote when quoted), quoted, bytes after a closing quote, any value of
    // the row left to pass 1
    u64 fs = ~0ull;
    bool qin = false, bad = false, anyfix = false;
    auto put = [&](u32 c) {
        if (PASS == 1 && !wr) return;
        if (nacc == 0 && ((uintptr_t)dst & 7u) != 0) { *dst++ = (u8)c; return; }
        acc |= (u64)c << (8 * nacc);
        if (++nacc == 8) { *(u64 *)dst = acc; dst += 8; acc = 0; nacc = 0; }
    };
    auto flush = [&]() {
        if (PASS == 1 && !wr) return;
        for (u32 k = 0; k < nacc; ++k) dst[k] = (u8)(acc >> (8 * k));
        dst += nacc;
        acc = 0;
        nacc = 0;
    };
    auto open_field = [&]() {
        clen = 0;
        special = false;
        fs = ~0ull;
        qin = bad = false;
        if (PASS == 1 && f < a.ncols) {
            const u64 k = f * a.R + j;
            dst = a.out + a.off[k];
            wr = (a.quoted[k] & 2u) == 0;
            q = (a.quoted[k] & 1u) != 0;
            if (q) put(a.dia.quote);
        }
    };
    // fend: one past the value's last source byte; sv: the reader's state there
    auto save = [&](u64 fend, u32 sv) {
        if (f < a.ncols) {
            if (PASS == 0) {
                const u64 k = f * a.R + j;
                const bool qq = special || clen == 0;  // clen already counts doubled quotes
                a.len[k] = qq ? clen + 3 : clen + 1;
                bool raw = CC_RAW && !bad && fs != ~0ull;
                if (qq) raw = raw && qin && sv == QQ && fend - fs == clen + 2;
                else raw = raw && !qin && fend - fs == clen;
                a.quoted[k] = (qq ? 1u : 0u) | (raw ? 2u : 0u);
                if (a.src) a.src[k] = raw ? fs : 0;
                anyfix |= !raw;
            } else {
                if (q) put(a.dia.quote);
                put('\n');
                flush();
            }
        }
        ++f;
        chars = 0;
        open_field();
    };
    open_field();
    bool any = false;
    {
        // quote/comma/CR/LF bytes one by one, every run of other bytes at once
        // (all of them are added to the field and never need quoting or
        // doubling): pass 0 counts them (field-limit characters =
        // non-continuation bytes), pass 1 copies them through the combiner
#if WCS_PF
        uint4 vn = (rs & ~15ull) < re ? *(const uint4 *)(a.buf + (rs & ~15ull)) : make_uint4(0, 0, 0, 0);
#endif
        for (u64 b0 = rs & ~15ull; b0 < re; b0 += 16) {
#if WCS_PF
            const uint4 v = vn;  // the next vector's load in flight while this one is walked
            if (b0 + 16 < re) vn = *(const uint4 *)(a.buf + b0 + 16);
#else
            const uint4 v = *(const uint4 *)(a.buf + b0);
#endif
            u32 vm = 0xFFFFu;
            if (b0 < rs) vm &= 0xFFFFu << (u32)(rs - b0);
            if (b0 + 16 > re) vm &= (1u << (u32)(re - b0)) - 1u;
            const u32 Qm = mask16(v, a.dia.quote) & vm, DNm = (mask16(v, a.dia.delim) | mask16(v, '\n')) & vm;
            const u32 S = (Qm | DNm | mask16(v, '\r') | (a.dia.skip ? mask16(v, ' ') : 0u)) & vm;
            const u32 O = vm & ~S;
            const u32 W[4] = {v.x, v.y, v.z, v.w};
            u32 CONT = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) CONT |= swar_pack4(W[k] & ~(W[k] << 1) & 0x80808080u) << (4 * k);
            u32 E = S;
            if (b0 + 16 >= a.n && a.n > b0 && ((vm >> (u32)(a.n - 1 - b0)) & 1u)) E |= 1u << (u32)(a.n - 1 - b0);
            int prev = -1;
            auto run = [&](u32 m) {
                if (!m) return;
                if (s == SR || s == SF) {  // an unquoted value starts here
                    if (fs == ~0ull) fs = b0 + (u32)__builtin_ctz(m);
                } else if (s == QQ) {
                    bad = true;  // bytes after a closing quote
                }
                if (PASS == 0) {
                    chars += (u32)__popc(m & ~CONT);
                    if (chars > FIELD_LIMIT) limit = true;
                    if (f < a.ncols) clen += (u32)__popc(m);
                } else if (f < a.ncols) {
                    for (u32 mm = m; mm; mm &= mm - 1) put(byte_of(v, (u32)__builtin_ctz(mm)));
                }
                s = step(T_O, s);
            };
            while (E) {
#if CC_IQ
                if (PASS == 0 && s == IQ) {
                    // inside quotes every byte up to the next quotechar is added
                    // to the value (delimiters and line ends too): one step to it
                    // (the lyric fields' line breaks had each been a trip)
                    const u32 after = prev < 0 ? vm : (vm & ~((2u << prev) - 1u));
                    const u32 qn = Qm & after;
                    const u32 rng = qn ? (after & ((1u << __builtin_ctz(qn)) - 1u)) : after;
                    if (rng) {
                        chars += (u32)__popc(rng & ~CONT);
                        if (chars > FIELD_LIMIT) limit = true;
                        if (f < a.ncols) {
                            clen += (u32)__popc(rng);
                            special |= (rng & DNm) != 0;
                        }
                    }
                    if (!qn) {
                        prev = 15;
                        break;
                    }
                    const u32 pq = (u32)__builtin_ctz(qn);
                    prev = (int)pq - 1;
                    E &= ~((1u << pq) - 1u);  // (the quote's own bit stays)
                }
#endif
                const u32 p = (u32)__builtin_ctz(E);
                E &= E - 1;
                run(O & ((1u << p) - 1u) & ~(prev < 0 ? 0u : ((2u << prev) - 1u)));
                const u32 b = byte_of(v, p);
                const u64 i = b0 + p;
                bool eol = i + 1 == a.n || b == '\n';
                if (b == '\r' && !eol) eol = (p < 15 ? byte_of(v, p + 1) : (u32)a.buf[i + 1]) != '\n';
                const u32 cls = cls_of(b, a.dia);
                const u32 tnext = cls_next(cls);
                const u32 act = (cls_act(cls) >> (2 * s)) & 3u;
                if (act & 2u) save(i, s);
                if (s == SR || s == SF) {
                    if (cls == C_Q) {  // an opening quote
                        qin = true;
                        fs = i;
                    } else if ((act & 1u) && fs == ~0ull) {
                        fs = i;
                    }
                } else if (s == QQ && cls != C_Q && !(act & 2u)) {
                    bad = true;
                }
                if (act & 1u) {
                    if ((b & 0xC0) != 0x80 && ++chars > FIELD_LIMIT) limit = true;
                    if (f < a.ncols) {
                        if (PASS == 0) {
                            clen += 1 + (b == a.dia.quote);  // a quotechar is doubled if the value is quoted
                            special |= b == a.dia.delim || b == a.dia.quote || b == '\n';
                        } else {
                            put(b);
                            if (q && b == a.dia.quote) put(a.dia.quote);
                        }
                    }
                }
                s = step(tnext, s);
                if (eol) {
                    if (s == SF || s == IF || s == QQ) save(i + 1, s);
                    if (s != IQ) s = SR;
                }
                prev = (int)p;
            }
            run(O & ~(prev < 0 ? 0u : ((2u << prev) - 1u)));
        }
    }
    if (s == IQ) { save(re, s); any = true; }
    if (PASS == 0 && limit) wcs_err(a.ctr, r, E_LIMIT);
    (void)any;
    // missing fields (and every field of a blank row) are ""
    for (; f < a.ncols; ++f) {
        const u64 k = f * a.R + j;
        if (PASS == 0) {
            a.len[k] = 3;
            a.quoted[k] = 1;
            if (a.src) a.src[k] = 0;
            anyfix = true;
        } else {
            u8 *d = a.out + a.off[k];
            d[0] = (u8)a.dia.quote; d[1] = (u8)a.dia.quote; d[2] = '\n';
        }
    }
    if (PASS == 0 && a.fix && anyfix) a.fix[atomicAdd((unsigned long long *)a.nfix, 1ull)] = r;
}

inline dim3 grid1(u64 n, u32 t = 256) { return dim3((u32)((n + t - 1) / t)); }

}  // namespace

// ===========================================================================
// Host side.
struct msa_wcs {
    int device = 0;
    int cus = 0;  // compute units (k_wcs_wrows runs WR_GPC workgroups per CU)
    hipStream_t stream = nullptr;
    char err[512] = {0};
    // input
    u8 *d_buf = nullptr;
    u64 n = 0, cap = 0;
    // rows
    u64 nrows = 0;  // incl. header
    u64 fallback_rows = 0;  // last run: rows left to k_wcs_rows
    u64 *d_rend = nullptr;
    u64 rend_cap = 0;
    // results (device)
    u64 nw = 0, np = 0, blob_len = 0;
    u32 *d_counts = nullptr;
    u64 *d_woff = nullptr;
    u8 *d_blob = nullptr;
    u64 *d_pairs = nullptr;
    u64 *d_nd = nullptr;
    u64 *d_spans = nullptr;
    msa_wcs_summary sum{};
    u64 gbits = 0;  // global table size of the next run (log2), 0 = auto
    u32 delim = ',';  // field delimiter (msa_wcs_set_delimiter: the script's --delimiter or csv.Sniffer's guess)
    hipEvent_t ev_a = nullptr, ev_b = nullptr;  // k_wcs_wrows of the last run (msa_wcs_kernel_ms)
    float wrows_ms = 0;
    float csvcol_ms = 0;  // the copy phase of the last msa_csvcol_run (msa_csvcol_kernel): the gathers + k_csvcol<1>
    u64 csvcol_out = 0;   // its output bytes
    u32 quote = '"';  // quotechar and skipinitialspace (msa_wcs_set_quoting): the column splitter's dialect
    u32 skipsp = 0;
    bool keep_bom = false;  // msa_wcs_set_encoding: "utf-8" keeps a leading BOM as data ("utf-8-sig" drops it)
    bool one_byte = false;  // msa_wcs_set_encoding 2: a single-byte codec (column splitter only)
    Dia dia() const { return Dia{delim, quote, skipsp}; }
    bool have = false;
    // column splitter results
    u64 cc_ncols = 0, cc_rows = 0;
    std::vector<std::string> cc_hdr;
    u64 *d_ccoff = nullptr;  // [ncols * rows + 1]
    u8 *d_ccout = nullptr;
    bool cc_have = false;
    // scratch owned by the run
    void *scr[29] = {nullptr};  // grow-only pool: buffers persist across runs
    u64 scr_cap[29] = {0};
};

static int wfail(msa_wcs *w, int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(w->err, sizeof w->err, fmt, ap);
    va_end(ap);
    return code;
}
#define WCHECK(x)                                                                                           \
    do {                                                                                                    \
        hipError_t e_ = (x);                                                                                \
        if (e_ != hipSuccess) return wfail(w, MSA_ERR_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, \
                                           __LINE__);                                                       \
    } while (0)

static void wfree(void *&p) {
    if (p) {  // nothing in flight may still touch it (its memory can be handed out again at once)
        (void)hipDeviceSynchronize();
        (void)hipFree(p);
    }
    p = nullptr;
}
template <typename T>
static hipError_t walloc(T *&p, u64 bytes) {
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, bytes ? bytes : 16);
    p = (T *)q;
    return e;
}

// Pool slot k holds at least `bytes` (contents not preserved on growth).
template <typename T>
static hipError_t wpool(msa_wcs *w, int k, u64 bytes, T *&p) {
    if (bytes == 0) bytes = 16;
    if (w->scr_cap[k] < bytes) {
        wfree(w->scr[k]);
        w->scr_cap[k] = 0;
        hipError_t e = hipMalloc(&w->scr[k], bytes);
        if (e != hipSuccess) {
            w->scr[k] = nullptr;
            return e;
        }
        w->scr_cap[k] = bytes;
    }
    p = (T *)w->scr[k];
    return hipSuccess;
}

static void wcs_release_results(msa_wcs *w) { w->have = false; w->cc_have = false; }

extern "C" int msa_wcs_create(int device, msa_wcs **out) {
    if (!out) return MSA_ERR_ARG;
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd <= device || device < 0) return MSA_ERR_HIP;
    if (hipSetDevice(device) != hipSuccess) return MSA_ERR_HIP;
    msa_wcs *w = new msa_wcs();
    w->device = device;
    if (hipDeviceGetAttribute(&w->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || w->cus < 1)
        w->cus = 1;
    if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&w->ev_a) != hipSuccess || hipEventCreate(&w->ev_b) != hipSuccess) {
        delete w;
        return MSA_ERR_HIP;
    }
    *out = w;
    return MSA_OK;
}

// Not part of include/msa_hip.h: the last run's k_wcs_wrows time (HIP events
// on the context's stream), for tools/bench_wcs.py's roofline.
extern "C" double msa_wcs_kernel_ms(msa_wcs *w) { return w ? (double)w->wrows_ms : 0.0; }
// The column splitter's copy kernel (k_csvcol<1>) of the last msa_csvcol_run:
// HIP-event time and output bytes (tools/bench_wcs.py --path split: roofline)
extern "C" int msa_csvcol_kernel(msa_wcs *w, double *ms, uint64_t *out_bytes) {
    if (!w || !ms || !out_bytes) return MSA_ERR_ARG;
    *ms = w->csvcol_ms;
    *out_bytes = w->csvcol_out;
    return MSA_OK;
}

extern "C" void msa_wcs_destroy(msa_wcs *w) {
    if (!w) return;
    (void)hipSetDevice(w->device);
    (void)hipStreamSynchronize(w->stream);
    for (auto &p : w->scr) wfree(p);
    wfree((void *&)w->d_buf);
    wfree((void *&)w->d_rend);
    if (w->ev_a) (void)hipEventDestroy(w->ev_a);
    if (w->ev_b) (void)hipEventDestroy(w->ev_b);
    (void)hipStreamDestroy(w->stream);
    delete w;
}

extern "C" const char *msa_wcs_last_error(const msa_wcs *w) { return w ? w->err : "null context"; }
extern "C" void *msa_wcs_stream(msa_wcs *w) { return w ? (void *)w->stream : nullptr; }

extern "C" int msa_wcs_load_csv(msa_wcs *w, const void *host_csv, size_t n) {
    if (!w || (!host_csv && n)) return MSA_ERR_ARG;
    WCHECK(hipSetDevice(w->device));
    if (n + MSA_INPUT_PAD > w->cap) {
        wfree((void *&)w->d_buf);
        w->cap = n + MSA_INPUT_PAD;
        WCHECK(walloc(w->d_buf, w->cap));
    }
    WCHECK(hipMemsetAsync(w->d_buf + n, 0, MSA_INPUT_PAD, w->stream));
    if (n) WCHECK(hipMemcpyAsync(w->d_buf, host_csv, n, hipMemcpyHostToDevice, w->stream));
    WCHECK(hipStreamSynchronize(w->stream));
    w->n = n;
    w->have = false;
    return MSA_OK;
}

// The field delimiter of the reader (and of the column splitter's writer):
// one ASCII byte other than '"', '\r', '\n' and NUL.  Invalidates results.
extern "C" int msa_wcs_set_delimiter(msa_wcs *w, int delim) {
    if (!w || delim <= 0 || delim > 127 || (u32)delim == w->quote || delim == '\r' || delim == '\n') return MSA_ERR_ARG;
    if ((u32)delim != w->delim) wcs_release_results(w);
    w->delim = (u32)delim;
    return MSA_OK;
}

// The column splitter's quoting (split_csv_columns.py --quotechar, 90-95, and
// the sniffed skipinitialspace of detect_csv_params, 58): one ASCII byte other
// than the delimiter, CR, LF and NUL.  The per-song counter reads the default
// dialect only (msa_wcs_run refuses another).  Invalidates results.
extern "C" int msa_wcs_set_quoting(msa_wcs *w, int quotechar, int skipinitialspace) {
    if (!w || quotechar <= 0 || quotechar > 127 || (u32)quotechar == w->delim || quotechar == '\r' ||
        quotechar == '\n')
        return MSA_ERR_ARG;
    if ((u32)quotechar != w->quote || (u32)(skipinitialspace != 0) != w->skipsp) wcs_release_results(w);
    w->quote = (u32)quotechar;
    w->skipsp = skipinitialspace != 0;
    return MSA_OK;
}

// Both at once, the pair validated together (the column splitter: a new
// quotechar may equal the current delimiter and vice versa).
extern "C" int msa_wcs_set_dialect(msa_wcs *w, int delim, int quotechar, int skipinitialspace) {
    auto bad = [](int b) { return b <= 0 || b > 127 || b == '\r' || b == '\n'; };
    if (!w || bad(delim) || bad(quotechar) || delim == quotechar) return MSA_ERR_ARG;
    if ((u32)delim != w->delim || (u32)quotechar != w->quote || (u32)(skipinitialspace != 0) != w->skipsp)
        wcs_release_results(w);
    w->delim = (u32)delim;
    w->quote = (u32)quotechar;
    w->skipsp = skipinitialspace != 0;
    return MSA_OK;
}

// The scripts' --encoding: utf8_sig = 1 ("utf-8-sig", their default) drops a
// leading BOM; 0 ("utf-8") keeps it as the first field's first character.
// Invalidates results.
extern "C" int msa_wcs_set_encoding(msa_wcs *w, int utf8_sig) {
    if (!w || utf8_sig < 0 || utf8_sig > 2) return MSA_ERR_ARG;
    const bool keep = utf8_sig != 1, one = utf8_sig == 2;
    if (keep != w->keep_bom || one != w->one_byte) wcs_release_results(w);
    w->keep_bom = keep;
    w->one_byte = one;
    return MSA_OK;
}

extern "C" int msa_wcs_set_table_bits(msa_wcs *w, int bits) {
    if (!w || bits < 0 || bits > 31) return MSA_ERR_ARG;
    w->gbits = (u64)bits;
    return MSA_OK;
}

// Header row -> column indices ("dict(zip(fieldnames, row))": the last
// duplicate name wins).  Host restatement of the same reader for one row.
static int parse_header(msa_wcs *w, const u8 *h, u64 len, u32 *ia, u32 *isg, u32 *it) {
    long long col[3] = {-1, -1, -1};
    static const char *names[3] = {"artist", "song", "text"};
    char *fld = (char *)malloc(len + 1);
    u64 fl = 0;
    u32 f = 0, s = SR;
    bool any = false;
    auto save = [&]() {
        for (int k = 0; k < 3; ++k)
            if (fl == strlen(names[k]) && memcmp(fld, names[k], fl) == 0) col[k] = f;
        ++f;
        fl = 0;
        any = true;
    };
    for (u64 i = 0; i < len; ++i) {
        const u32 b = h[i];
        const bool eol = b == '\n' || (b == '\r' && (i + 1 >= len || h[i + 1] != '\n')) || i + 1 == len;
        switch (s) {
            case SR:
                if (b == '\r' || b == '\n') { s = EC; break; }
                s = SF;
                [[fallthrough]];
            case SF:
                if (b == '\r' || b == '\n') { save(); s = EC; }
                else if (b == '"') s = IQ;
                else if (b == w->delim) save();
                else { fld[fl++] = (char)b; s = IF; }
                break;
            case IF:
                if (b == '\r' || b == '\n') { save(); s = EC; }
                else if (b == w->delim) { save(); s = SF; }
                else fld[fl++] = (char)b;
                break;
            case IQ:
                if (b == '"') s = QQ;
                else fld[fl++] = (char)b;
                break;
            case QQ:
                if (b == '"') { fld[fl++] = '"'; s = IQ; }
                else if (b == w->delim) { save(); s = SF; }
                else if (b == '\r' || b == '\n') { save(); s = EC; }
                else { fld[fl++] = (char)b; s = IF; }
                break;
            default:
                break;
        }
        if (eol) {
            if (s == SF || s == IF || s == QQ) save();
            if (s != IQ) s = SR;
        }
    }
    if (s == IQ) save();
    free(fld);
    (void)any;
    if (col[0] < 0 || col[1] < 0 || col[2] < 0)
        return wfail(w, MSA_ERR_BADHEADER, "CSV sem colunas esperadas. Campos necessários: artist, song, text.");
    *ia = (u32)col[0];
    *isg = (u32)col[1];
    *it = (u32)col[2];
    return MSA_OK;
}

static int wcs_input_error(msa_wcs *w, u64 e) {
    const u32 code = (u32)(e & 0xFF);
    const u64 row = e >> 8;
    switch (code) {
        case E_UTF8: return wfail(w, MSA_ERR_INPUT, "invalid UTF-8 in the input");
        case E_NUL: return wfail(w, MSA_ERR_INPUT, "line contains NUL");
        case E_LIMIT: return wfail(w, MSA_ERR_INPUT, "field larger than field limit (131072) (row %llu)",
                                   (unsigned long long)row);
        default: return wfail(w, MSA_ERR_INPUT, "row %llu has no artist/song/text value", (unsigned long long)row);
    }
}

// Validation + row ends of the loaded CSV (shared by the per-song counter and
// the column splitter).  d_rend[0] = ds, d_rend[k + 1] = end of file row k.
static int wcs_split_rows(msa_wcs *w, WCtr **ctr_out, u64 *ds_out, u64 *nrows_out) {
    hipStream_t st = w->stream;
    const u8 *buf = w->d_buf;
    const u64 n = w->n;
    WCtr *ctr;
    WCHECK(wpool(w, 0, sizeof(WCtr), ctr));
    WCtr h0{};
    h0.err = ~0ull;
    WCHECK(hipMemcpyAsync(ctr, &h0, sizeof h0, hipMemcpyHostToDevice, st));
    if (n) hipLaunchKernelGGL(k_wcs_validate, grid1((n + 15) / 16), dim3(256), 0, st, buf, n, ctr, w->one_byte ? 0u : 1u);
    // BOM ("utf-8-sig")
    u8 bom[3] = {0, 0, 0};
    if (n >= 3) WCHECK(hipMemcpyAsync(bom, buf, 3, hipMemcpyDeviceToHost, st));
    WCHECK(hipStreamSynchronize(st));
    const u64 ds = (!w->keep_bom && n >= 3 && bom[0] == 0xEF && bom[1] == 0xBB && bom[2] == 0xBF) ? 3 : 0;

    // ---- rows
    const u64 nseg = (n + SEG - 1) / SEG;
    u64 nrows = 0;
    u32 fin = SR;
    if (nseg) {
        const u64 nb = (nseg + BSEG - 1) / BSEG;
        u32 *map, *bmap, *sstate, *dfin;
        u64 *cnt6, *cnt, *roff, *bsum, *total;
        WCHECK(wpool(w, 1, nseg * 4, map));
        WCHECK(wpool(w, 2, nseg * 8, cnt6));
        WCHECK(wpool(w, 3, nseg * 8, cnt));
        WCHECK(wpool(w, 4, nseg * 8, roff));
        WCHECK(wpool(w, 5, nb * 4 + 16, bmap));
        WCHECK(wpool(w, 6, nseg * 4, sstate));
        WCHECK(wpool(w, 7, (nseg / 1024 + 2) * 8, bsum));
        WCHECK(wpool(w, 8, 16, total));
        dfin = bmap + nb;
        hipLaunchKernelGGL(k_wcs_map, grid1(nseg), dim3(256), 0, st, buf, ds, n, nseg, w->dia(), map, cnt6);
        hipLaunchKernelGGL(k_wcs_state_block, dim3((u32)nb), dim3(BLK), 0, st, (const u32 *)map, nseg, bmap);
        hipLaunchKernelGGL(k_wcs_state_top2, dim3(1), dim3(TOP_T), 0, st, bmap, nb, dfin);
        hipLaunchKernelGGL(k_wcs_state_down, dim3((u32)nb), dim3(BLK), 0, st, (const u32 *)map, (const u64 *)cnt6,
                           nseg, (const u32 *)bmap, sstate, cnt);
        WCHECK(msa_exclusive_scan(cnt, nseg, roff, bsum, total, st));
        u64 nend = 0;
        WCHECK(hipMemcpyAsync(&nend, total, 8, hipMemcpyDeviceToHost, st));
        WCHECK(hipMemcpyAsync(&fin, dfin, 4, hipMemcpyDeviceToHost, st));
        WCHECK(hipStreamSynchronize(st));
        nrows = nend + (fin == IQ ? 1 : 0);
        if (nrows + 1 > w->rend_cap) {
            wfree((void *&)w->d_rend);
            w->rend_cap = nrows + 1;
            WCHECK(walloc(w->d_rend, w->rend_cap * 8));
        }
        // rend[-1] = ds: rows are [rend[r-1], rend[r]) with d_rend shifted by one
        WCHECK(hipMemcpyAsync(w->d_rend, &ds, 8, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_wcs_emit, grid1(nseg), dim3(256), 0, st, buf, ds, n, nseg, w->dia(), (const u32 *)sstate,
                           (const u64 *)roff, w->d_rend + 1);
        if (fin == IQ) WCHECK(hipMemcpyAsync(w->d_rend + nrows, &n, 8, hipMemcpyHostToDevice, st));
    }
    WCtr hc{};
    WCHECK(hipMemcpyAsync(&hc, ctr, sizeof hc, hipMemcpyDeviceToHost, st));
    WCHECK(hipStreamSynchronize(st));
    if (hc.err != ~0ull) return wcs_input_error(w, hc.err);
    *ctr_out = ctr;
    *ds_out = ds;
    *nrows_out = nrows;
    return MSA_OK;
}


extern "C" int msa_wcs_run(msa_wcs *w) {
    if (!w || !w->d_buf) return MSA_ERR_ARG;
    if (w->quote != '"' || w->skipsp)  // csv.DictReader(fh, delimiter=...): the default dialect otherwise
        return wfail(w, MSA_ERR_ARG, "the per-song counter reads quotechar '\"' without skipinitialspace");
    if (w->one_byte)  // its tokens are Unicode words of UTF-8 text
        return wfail(w, MSA_ERR_ARG, "the per-song counter reads UTF-8 only (single-byte encodings: column splitter)");
    WCHECK(hipSetDevice(w->device));
    wcs_release_results(w);
    hipStream_t st = w->stream;
    const u8 *buf = w->d_buf;
    const u64 n = w->n;
    WCtr *ctr;
    u64 ds = 0, nrows = 0;
    int rc0 = wcs_split_rows(w, &ctr, &ds, &nrows);
    if (rc0) return rc0;
    if (nrows == 0) return wfail(w, MSA_ERR_BADHEADER, "CSV sem colunas esperadas. Campos necessários: artist, song, text.");
    WCtr h0{};
    h0.err = ~0ull;
    WCtr hc{};

    // ---- header (host)
    u64 he = 0;
    WCHECK(hipMemcpyAsync(&he, w->d_rend + 1, 8, hipMemcpyDeviceToHost, st));
    WCHECK(hipStreamSynchronize(st));
    u8 *hb = (u8 *)malloc(he - ds + 1);
    if (he > ds) WCHECK(hipMemcpy(hb, buf + ds, he - ds, hipMemcpyDeviceToHost));
    u32 ia = 0, isg = 0, it = 0;
    int rc = parse_header(w, hb, he - ds, &ia, &isg, &it);
    free(hb);
    if (rc) return rc;
    const u32 need = ia > isg ? (ia > it ? ia : it) : (isg > it ? isg : it);

    // ---- per-row pass: d_rend[0] = ds, d_rend[k + 1] = end of file row k;
    // per-row arrays are indexed by k + 1 (the header is index 1)
    const u64 R = nrows + 1;
    WCHECK(wpool(w, 18, R * 8, w->d_nd));
    WCHECK(wpool(w, 19, R * 32, w->d_spans));
    WCHECK(hipMemsetAsync(w->d_nd, 0, R * 8, st));
    u64 *scratch;
    WCHECK(wpool(w, 9, (2 * n + 64) * 8, scratch));
    u64 *fb;
    WCHECK(wpool(w, 24, R * 8, fb));
    u64 bits = w->gbits;
    if (!bits) {
        bits = 16;
        while (bits < 28 && (1ull << bits) < n / 1024) ++bits;  // regrown (the run repeats) past 3/4 full
    }
    u64 *gtab = nullptr;
    for (;;) {
        const u64 slots = 1ull << bits;
        WCHECK(wpool(w, 10, slots * 32, gtab));
        WCHECK(hipMemsetAsync(gtab, 0, slots * 32, st));
        WCHECK(hipMemcpyAsync(ctr, &h0, sizeof h0, hipMemcpyHostToDevice, st));
        RowArgs a;
        a.buf = buf; a.n = n; a.rend = w->d_rend; a.ds = ds; a.nrows = R;
        a.ia = ia; a.isg = isg; a.it = it; a.need = need; a.delim = w->delim;
        a.gtab = gtab; a.gmask = slots - 1; a.glimit = slots / 4 * 3;
        a.scratch = scratch; a.nd = w->d_nd; a.spans = w->d_spans; a.ctr = ctr;
        a.ablate = getenv("MSA_WCS_ABLATE") ? atoi(getenv("MSA_WCS_ABLATE")) : 0;
        a.rows = nullptr;
        a.fb = fb;
        // wave per row first; the rows it leaves (long, unusual quoting, many
        // token runs) are walked one thread per row (ablate bit 8: all of them)
        if (R > 2 && !(a.ablate & 8)) {
            // persistent workgroups: each keeps its LDS aggregate over many
            // row blocks, so the flush (device-scope atomics on the Zipf head)
            // happens a few hundred times, not once per 256 rows
            const u64 per = (u64)WR_W * WR_ROWS, blocks = (R - 2 + per - 1) / per;
            const u64 g = (u64)w->cus * WR_GPC;
            WCHECK(hipEventRecord(w->ev_a, st));
            hipLaunchKernelGGL(k_wcs_wrows, dim3((u32)(blocks < g ? blocks : g)), dim3(WR_W * 64), 0, st, a);
            WCHECK(hipGetLastError());
            WCHECK(hipEventRecord(w->ev_b, st));
            WCHECK(hipMemcpyAsync(&hc, ctr, sizeof hc, hipMemcpyDeviceToHost, st));
            WCHECK(hipStreamSynchronize(st));
            WCHECK(hipEventElapsedTime(&w->wrows_ms, w->ev_a, w->ev_b));
            // (the count is the summary's fallback_rows)
            w->fallback_rows = hc.fallback;
            if (hc.fallback) {
                a.rows = fb;
                hipLaunchKernelGGL(k_wcs_rows, grid1(hc.fallback), dim3(256), 0, st, a);
            }
        } else if (R > 2) {
            w->fallback_rows = R - 2;
            hipLaunchKernelGGL(k_wcs_rows, grid1(R - 2), dim3(256), 0, st, a);
        }
        WCHECK(hipGetLastError());
        WCHECK(hipMemcpyAsync(&hc, ctr, sizeof hc, hipMemcpyDeviceToHost, st));
        WCHECK(hipStreamSynchronize(st));
        if (hc.err != ~0ull) return wcs_input_error(w, hc.err);
        if (!(hc.overflow & OVF_G)) break;
        if (bits >= 31) return wfail(w, MSA_ERR_CAPACITY, "word table overflow at 2^31 slots");
        bits += 2;
    }
    const u64 slots = 1ull << bits;
    const u64 nw = hc.distinct;

    // ---- ranking
    u64 *K2[3], *K1[3], *K0[3];
    u32 *V[3];
    u64 *kmem;
    u32 *vmem;
    WCHECK(wpool(w, 11, (nw + 1) * 8 * 9, kmem));
    WCHECK(wpool(w, 12, (nw + 1) * 4 * 3, vmem));
    for (int k = 0; k < 3; ++k) {
        K2[k] = kmem + (u64)(3 * k + 0) * (nw + 1);
        K1[k] = kmem + (u64)(3 * k + 1) * (nw + 1);
        K0[k] = kmem + (u64)(3 * k + 2) * (nw + 1);
        V[k] = vmem + (u64)k * (nw + 1);
    }
    hipLaunchKernelGGL(k_wcs_list, grid1(slots), dim3(256), 0, st, (const u64 *)gtab, slots, ctr, K2[0], K1[0], K0[0],
                       V[0]);
    int which = 1;
    WCHECK(msa_launch_sort(K2, K1, K0, V, nw, &which, st));
    const u32 *order = V[which];
    u32 *rank_of;
    WCHECK(wpool(w, 13, slots * 4, rank_of));
    u64 *wlen, *bsum2, *total2;
    WCHECK(wpool(w, 14, (nw + 1) * 8, wlen));
    WCHECK(wpool(w, 20, (nw + 1) * 4, w->d_counts));
    WCHECK(wpool(w, 21, (nw + 1) * 8, w->d_woff));
    WCHECK(wpool(w, 15, ((R > nw ? R : nw) / 1024 + 2) * 8, bsum2));
    WCHECK(wpool(w, 16, 16, total2));
    if (nw) {
        hipLaunchKernelGGL(k_wcs_wordlen, grid1(nw), dim3(256), 0, st, buf, (const u64 *)gtab, order, nw, rank_of, wlen,
                           w->d_counts, ctr);
        WCHECK(msa_exclusive_scan(wlen, nw, w->d_woff, bsum2, total2, st));
        WCHECK(hipMemcpyAsync(w->d_woff + nw, total2, 8, hipMemcpyDeviceToDevice, st));
    } else {
        WCHECK(hipMemsetAsync(w->d_woff, 0, 8, st));
    }
    u64 blob_len = 0;
    WCHECK(hipMemcpyAsync(&blob_len, w->d_woff + nw, 8, hipMemcpyDeviceToHost, st));
    WCHECK(hipStreamSynchronize(st));
    WCHECK(wpool(w, 22, blob_len + 16, w->d_blob));
    if (nw)
        hipLaunchKernelGGL(k_wcs_wordblob, grid1(nw), dim3(256), 0, st, buf, (const u64 *)gtab, order, nw,
                           (const u64 *)w->d_woff, w->d_blob, ctr);

    // ---- by-song lines
    u64 *poff;
    WCHECK(wpool(w, 17, R * 8, poff));
    WCHECK(msa_exclusive_scan(w->d_nd, R, poff, bsum2, total2, st));
    u64 np = 0;
    WCHECK(hipMemcpyAsync(&np, total2, 8, hipMemcpyDeviceToHost, st));
    WCHECK(hipStreamSynchronize(st));
    WCHECK(wpool(w, 23, np * 8 + 16, w->d_pairs));
    if (R > 2)
        hipLaunchKernelGGL(k_wcs_pairs, grid1(R - 2), dim3(256), 0, st, (const u64 *)w->d_rend, R,
                           (const u64 *)w->d_nd, (const u64 *)poff, (const u64 *)scratch, (const u32 *)rank_of,
                           w->d_pairs);
    WCHECK(hipGetLastError());
    WCHECK(hipMemcpyAsync(&hc, ctr, sizeof hc, hipMemcpyDeviceToHost, st));
    WCHECK(hipStreamSynchronize(st));
    if (hc.collision) return wfail(w, MSA_ERR_COLLISION, "64-bit word-hash collision detected (%llu words)",
                                   (unsigned long long)hc.collision);
    w->nrows = R;
    w->nw = nw;
    w->np = np;
    w->blob_len = blob_len;
    w->sum.total_rows = hc.total_rows;
    w->sum.song_rows = hc.song_rows;
    w->sum.total_tokens = hc.tokens;
    w->sum.n_words = nw;
    w->sum.n_pairs = np;
    w->sum.fallback_rows = w->fallback_rows;
    w->have = true;
    return MSA_OK;
}

extern "C" int msa_wcs_get_summary(msa_wcs *w, msa_wcs_summary *out) {
    if (!w || !out || !w->have) return MSA_ERR_ARG;
    *out = w->sum;
    return MSA_OK;
}

// ---------------------------------------------------------------------------
// Output formatting (csv.writer, QUOTE_MINIMAL, "\r\n").
namespace {
struct Out {
    char *p = nullptr;
    size_t n = 0, cap = 0;
    bool put(const void *s, size_t k) {
        if (n + k > cap) {
            size_t c = cap ? cap : 1 << 16;
            while (c < n + k) c *= 2;
            char *q = (char *)realloc(p, c);
            if (!q) return false;
            p = q;
            cap = c;
        }
        memcpy(p + n, s, k);
        n += k;
        return true;
    }
    bool num(u64 v) {
        char t[24];
        int k = snprintf(t, sizeof t, "%llu", (unsigned long long)v);
        return put(t, (size_t)k);
    }
};

// Field content of a raw span: the reader's added characters.
void field_content(const u8 *b, u64 s, u64 e, std::string &o) {
    o.clear();
    u32 st = SF;
    for (u64 i = s; i < e; ++i) {
        const u8 c = b[i];
        switch (st) {
            case SF:
                if (c == '"') st = IQ;
                else { o.push_back((char)c); st = IF; }
                break;
            case IF: o.push_back((char)c); break;
            case IQ:
                if (c == '"') st = QQ;
                else o.push_back((char)c);
                break;
            default:  // QQ
                o.push_back((char)c);
                st = c == '"' ? IQ : IF;
                break;
        }
    }
}
bool py_space(u32 cp) {
    return (cp >= 0x9 && cp <= 0xD) || (cp >= 0x1C && cp <= 0x20) || cp == 0x85 || cp == 0xA0 || cp == 0x1680 ||
           (cp >= 0x2000 && cp <= 0x200A) || cp == 0x2028 || cp == 0x2029 || cp == 0x202F || cp == 0x205F ||
           cp == 0x3000;
}
u32 cp_at(const std::string &s, size_t i, size_t *len) {
    const u8 c = (u8)s[i];
    if (c < 0x80) { *len = 1; return c; }
    if (c < 0xE0) { *len = 2; return ((c & 0x1Fu) << 6) | ((u8)s[i + 1] & 0x3Fu); }
    if (c < 0xF0) { *len = 3; return ((c & 0x0Fu) << 12) | (((u8)s[i + 1] & 0x3Fu) << 6) | ((u8)s[i + 2] & 0x3Fu); }
    *len = 4;
    return ((c & 0x07u) << 18) | (((u8)s[i + 1] & 0x3Fu) << 12) | (((u8)s[i + 2] & 0x3Fu) << 6) | ((u8)s[i + 3] & 0x3Fu);
}
// str.strip() over UTF-8
void py_strip(std::string &s) {
    size_t a = 0, z = s.size(), l;
    while (a < z && py_space(cp_at(s, a, &l))) a += l;
    while (z > a) {
        size_t k = z - 1;
        while (k > a && ((u8)s[k] & 0xC0) == 0x80) --k;
        if (!py_space(cp_at(s, k, &l))) break;
        z = k;
    }
    s = s.substr(a, z - a);
}
bool csv_field(Out &o, const std::string &s) {
    if (s.find_first_of(",\"\r\n") == std::string::npos) return o.put(s.data(), s.size());
    if (!o.put("\"", 1)) return false;
    for (char c : s) {
        if (c == '"' && !o.put("\"", 1)) return false;
        if (!o.put(&c, 1)) return false;
    }
    return o.put("\"", 1);
}
}  // namespace

extern "C" int msa_wcs_get_csv(msa_wcs *w, int which, char **out, size_t *len) {
    if (!w || !out || !len || !w->have || (which != MSA_WCS_GLOBAL && which != MSA_WCS_BY_SONG)) return MSA_ERR_ARG;
    WCHECK(hipSetDevice(w->device));
    const u64 nw = w->nw;
    u32 *counts = (u32 *)malloc((nw + 1) * 4);
    u64 *woff = (u64 *)malloc((nw + 1) * 8);
    u8 *blob = (u8 *)malloc(w->blob_len + 1);
    WCHECK(hipMemcpy(counts, w->d_counts, nw * 4, hipMemcpyDeviceToHost));
    WCHECK(hipMemcpy(woff, w->d_woff, (nw + 1) * 8, hipMemcpyDeviceToHost));
    WCHECK(hipMemcpy(blob, w->d_blob, w->blob_len, hipMemcpyDeviceToHost));
    Out o;
    bool ok = true;
    if (which == MSA_WCS_GLOBAL) {
        ok = o.put("word,count\r\n", 12);
        for (u64 i = 0; ok && i < nw; ++i) {
            ok = o.put(blob + woff[i], woff[i + 1] - woff[i]) && o.put(",", 1) && o.num(counts[i]) && o.put("\r\n", 2);
        }
    } else {
        const u64 R = w->nrows;
        u64 *nd = (u64 *)malloc(R * 8), *sp = (u64 *)malloc(R * 32), *pairs = (u64 *)malloc(w->np * 8 + 8);
        u8 *csv = (u8 *)malloc(w->n + 1);
        WCHECK(hipMemcpy(nd, w->d_nd, R * 8, hipMemcpyDeviceToHost));
        WCHECK(hipMemcpy(sp, w->d_spans, R * 32, hipMemcpyDeviceToHost));
        WCHECK(hipMemcpy(pairs, w->d_pairs, w->np * 8, hipMemcpyDeviceToHost));
        WCHECK(hipMemcpy(csv, w->d_buf, w->n, hipMemcpyDeviceToHost));
        ok = o.put("artist,song,word,count\r\n", 24);
        std::string fa, fs;
        Out pre;
        u64 p = 0;
        for (u64 r = 2; ok && r < R; ++r) {
            if (!nd[r]) continue;
            field_content(csv, sp[r * 4 + 0], sp[r * 4 + 1], fa);
            field_content(csv, sp[r * 4 + 2], sp[r * 4 + 3], fs);
            py_strip(fa);
            py_strip(fs);
            pre.n = 0;
            ok = csv_field(pre, fa) && pre.put(",", 1) && csv_field(pre, fs) && pre.put(",", 1);
            for (u64 k = 0; ok && k < nd[r]; ++k, ++p) {
                const u64 v = pairs[p];
                const u64 rank = v >> 32;
                ok = o.put(pre.p, pre.n) && o.put(blob + woff[rank], woff[rank + 1] - woff[rank]) && o.put(",", 1) &&
                     o.num(v & 0xFFFFFFFFu) && o.put("\r\n", 2);
            }
        }
        free(pre.p);
        free(nd); free(sp); free(pairs); free(csv);
    }
    free(counts); free(woff); free(blob);
    if (!ok) { free(o.p); return wfail(w, MSA_ERR_HIP, "out of host memory"); }
    *out = o.p ? o.p : (char *)malloc(1);
    *len = o.n;
    return MSA_OK;
}

extern "C" int msa_wcs_write_outputs(msa_wcs *w, const char *outdir) {
    if (!w || !outdir || !w->have) return MSA_ERR_ARG;
    static const char *names[2] = {"word_counts_global.csv", "word_counts_by_song.csv"};
    for (int k = 0; k < 2; ++k) {
        char *d = nullptr;
        size_t len = 0;
        int rc = msa_wcs_get_csv(w, k, &d, &len);
        if (rc) return rc;
        char path[4096];
        snprintf(path, sizeof path, "%s/%s", outdir, names[k]);
        FILE *f = fopen(path, "wb");
        if (!f) { free(d); return wfail(w, MSA_ERR_IO, "cannot open %s", path); }
        const bool ok = fwrite(d, 1, len, f) == len;
        free(d);
        if (fclose(f) != 0 || !ok) return wfail(w, MSA_ERR_IO, "write failed: %s", path);
    }
    return MSA_OK;
}

// ---------------------------------------------------------------------------
// Column splitter host side.
static void row_fields(const u8 *h, u64 len, const Dia &dia, std::vector<std::string> &out) {
    out.clear();
    std::string fld;
    u32 s = SR;
    for (u64 i = 0; i < len; ++i) {
        const u32 b = h[i];
        const bool eol = b == '\n' || (b == '\r' && (i + 1 >= len || h[i + 1] != '\n')) || i + 1 == len;
        const u32 cls = cls_of(b, dia);
        const u32 tnext = cls_next(cls);
        const u32 act = (cls_act(cls) >> (2 * s)) & 3u;
        if (act & 2u) { out.push_back(fld); fld.clear(); }
        if (act & 1u) fld.push_back((char)b);
        s = step(tnext, s);
        if (eol) {
            if (s == SF || s == IF || s == QQ) { out.push_back(fld); fld.clear(); }
            if (s != IQ) s = SR;
        }
    }
    if (s == IQ) out.push_back(fld);
}

extern "C" int msa_csvcol_run(msa_wcs *w, int has_header, uint64_t *ncols, uint64_t *nrows) {
    if (!w || !w->d_buf || !ncols || !nrows) return MSA_ERR_ARG;
    WCHECK(hipSetDevice(w->device));
    w->cc_have = false;
    w->have = false;  // the two paths share the context's buffer pool
    hipStream_t st = w->stream;
    WCtr *ctr;
    u64 ds = 0, nr = 0;
    int rc = wcs_split_rows(w, &ctr, &ds, &nr);
    if (rc) return rc;
    if (nr == 0) return wfail(w, MSA_ERR_NOHEADER, "CSV vazio.");
    u64 he = 0;
    WCHECK(hipMemcpy(&he, w->d_rend + 1, 8, hipMemcpyDeviceToHost));
    std::vector<u8> hb(he - ds + 1);
    if (he > ds) WCHECK(hipMemcpy(hb.data(), w->d_buf + ds, he - ds, hipMemcpyDeviceToHost));
    row_fields(hb.data(), he - ds, w->dia(), w->cc_hdr);
    const u64 nc = w->cc_hdr.size();
    const u64 first = has_header ? 2 : 1;  // kernel row index of the first data row
    const u64 R = nr + 1 - first;
    const u64 cells = nc * R;
    u64 *len, *bsum, *total;
    u8 *quoted;
    WCHECK(wpool(w, 9, (cells + 1) * 8, len));
    WCHECK(wpool(w, 1, cells + 16, quoted));
    WCHECK(wpool(w, 17, (cells + 1) * 8, w->d_ccoff));
    WCHECK(wpool(w, 15, (cells / 1024 + 2) * 8, bsum));
    WCHECK(wpool(w, 16, 16, total));
    ColArgs a;
    a.buf = w->d_buf; a.n = w->n; a.rend = w->d_rend; a.first = first; a.nrows = nr + 1;
    a.ncols = nc; a.R = R; a.len = len; a.quoted = quoted; a.off = w->d_ccoff; a.out = nullptr; a.ctr = ctr;
    a.dia = w->dia();
    a.src = nullptr; a.fix = nullptr; a.nfix = nullptr;
#if CC_RAW
    WCHECK(wpool(w, 26, (cells + 1) * 8, a.src));
    WCHECK(wpool(w, 27, (R + 1) * 8, a.fix));
    WCHECK(wpool(w, 28, 16, a.nfix));
    WCHECK(hipMemsetAsync(a.nfix, 0, 8, st));
#endif
    if (cells) {
        hipLaunchKernelGGL(k_csvcol<0>, grid1(R), dim3(256), 0, st, a);
        WCHECK(msa_exclusive_scan(len, cells, w->d_ccoff, bsum, total, st));
        WCHECK(hipMemcpyAsync(w->d_ccoff + cells, total, 8, hipMemcpyDeviceToDevice, st));
    } else {
        WCHECK(hipMemsetAsync(w->d_ccoff, 0, 8, st));
    }
    u64 outlen = 0;
    WCHECK(hipMemcpyAsync(&outlen, w->d_ccoff + cells, 8, hipMemcpyDeviceToHost, st));
    WCtr hc{};
    WCHECK(hipMemcpyAsync(&hc, ctr, sizeof hc, hipMemcpyDeviceToHost, st));
    WCHECK(hipStreamSynchronize(st));
    if (hc.err != ~0ull) return wcs_input_error(w, hc.err);
    WCHECK(wpool(w, 22, outlen + 16, w->d_ccout));
    a.out = w->d_ccout;
    WCHECK(hipEventRecord(w->ev_a, st));
#if CC_RAW
    // every column's lines as raw copies, then the rows holding another value
    for (u64 f = 0; cells && f < nc; ++f)
        WCHECK(msa_launch_gather_lines(w->d_buf, len + f * R, w->d_ccoff + f * R, a.src + f * R, R,
                                       w->d_ccoff + (f + 1) * R, a.out, st));
    if (cells) hipLaunchKernelGGL(k_csvcol<1>, grid1(R), dim3(256), 0, st, a);
#else
    if (cells) hipLaunchKernelGGL(k_csvcol<1>, grid1(R), dim3(256), 0, st, a);
#endif
    WCHECK(hipGetLastError());
    WCHECK(hipEventRecord(w->ev_b, st));
    WCHECK(hipStreamSynchronize(st));
    WCHECK(hipEventElapsedTime(&w->csvcol_ms, w->ev_a, w->ev_b));
    w->csvcol_out = outlen;
    w->cc_ncols = nc;
    w->cc_rows = R;
    w->cc_have = true;
    *ncols = nc;
    *nrows = R;
    return MSA_OK;
}

extern "C" int msa_csvcol_header(msa_wcs *w, uint64_t col, char **out, size_t *len) {
    if (!w || !w->cc_have || col >= w->cc_ncols || !out || !len) return MSA_ERR_ARG;
    const std::string &h = w->cc_hdr[col];
    char *p = (char *)malloc(h.size() + 1);
    memcpy(p, h.data(), h.size());
    *out = p;
    *len = h.size();
    return MSA_OK;
}

extern "C" int msa_csvcol_get(msa_wcs *w, uint64_t col, char **out, size_t *len) {
    if (!w || !w->cc_have || col >= w->cc_ncols || !out || !len) return MSA_ERR_ARG;
    WCHECK(hipSetDevice(w->device));
    u64 o[2];
    WCHECK(hipMemcpy(&o[0], w->d_ccoff + col * w->cc_rows, 8, hipMemcpyDeviceToHost));
    WCHECK(hipMemcpy(&o[1], w->d_ccoff + (col + 1) * w->cc_rows, 8, hipMemcpyDeviceToHost));
    char *p = (char *)malloc(o[1] - o[0] + 1);
    if (o[1] > o[0]) WCHECK(hipMemcpy(p, w->d_ccout + o[0], o[1] - o[0], hipMemcpyDeviceToHost));
    *out = p;
    *len = o[1] - o[0];
    return MSA_OK;
}
