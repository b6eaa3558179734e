// msa_post.hip -- everything after the main scan:
//   * artist column: duplicate_field (parallel_spotify.c:215-255) of field 0,
//     split_dataset_columns' artist.csv (640-721), and the artist pass's
//     duplicate_field(line, 0) + ht_put (948-998) as exact 64-bit-hash counts
//   * words longer than 16 bytes (H-table + byte-exact verification)
//   * ranking: sort on (count desc, first 16 key bytes) -- bitonic tiles in
//     LDS, then merge passes by rank -- with an exact strcmp fix-up of the
//     rare equal-prefix runs: the order of entry_compare_desc (178-188)
//   * generic exclusive scan (u64)
#include <algorithm>

#include "msa_hip.h"
#include "msa_internal.h"
#include "msa_tables.h"

namespace {
__device__ __forceinline__ bool c_space(u32 c) { return c == ' ' || (c >= 9 && c <= 13); }
__device__ __forceinline__ bool c_tok(u32 c) {
    return ((c | 0x20u) >= 'a' && (c | 0x20u) <= 'z') || (c >= '0' && c <= '9') || c == '\'';
}
__device__ __forceinline__ u64 bswap64(u64 x) { return __builtin_bswap64(x); }
}  // namespace

// ---------------------------------------------------------------------------
// generic exclusive scan over u64 (3 phases), for up to two arrays at once
// (blockIdx.y picks the array: both column line-length arrays in one launch
// sequence)
#define SCAN_T 256
#define SCAN_PER 4
#define SCAN_TILE (SCAN_T * SCAN_PER)

struct ScanJob {
    const u64 *in;
    u64 *out, *bsum, *total;
    u64 n;
};
struct ScanJobs {
    ScanJob j[2];
    u64 tile;  // elements per block: SCAN_TILE, or SCAN_TILE_BIG for long arrays
};
// long arrays (configs[4]'s 50 M blob lengths): 16 elements a thread, so the
// single-workgroup top scan sees 12 K block sums instead of 49 K (96 us)
#define SCAN_PER_BIG 16
#define SCAN_TILE_BIG (SCAN_T * SCAN_PER_BIG)

template <int PER>
__global__ __launch_bounds__(SCAN_T) void k_scan_reduce(ScanJobs js) {
    const ScanJob &J = js.j[blockIdx.y];
    __shared__ u64 red[SCAN_T / 64];
    const u64 base = (u64)blockIdx.x * (SCAN_T * PER);
    if (base >= J.n) return;
    u64 s = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const u64 idx = base + (u64)i * SCAN_T + threadIdx.x;
        if (idx < J.n) s += J.in[idx];
    }
    s = wave_sum64(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 t = 0;
        for (int w = 0; w < SCAN_T / 64; ++w) t += red[w];
        J.bsum[blockIdx.x] = t;
    }
}

// exclusive scan of the block sums in place: per-thread runs, then a block
// scan of the run totals (wave shuffles + wave totals)
__global__ void k_scan_zero_totals(ScanJobs js) {
    if (threadIdx.x < 2 && js.j[threadIdx.x].total)
        __hip_atomic_store(js.j[threadIdx.x].total, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one workgroup per array: SCAN_TOP_T threads for long block-sum arrays
// (configs[4]'s 50 M blob lengths: 49 K sums), 256 otherwise (a 1024-thread
// workgroup waited ~70 us for a CU beside the text gather); each thread's
// run is read 8 loads at a time (one dependent load per element had made the
// top scan 105 us)
#define SCAN_TOP_T 1024
#define SCAN_TOP_BIG 16384
__global__ __launch_bounds__(SCAN_TOP_T) void k_scan_top(ScanJobs js) {
    const ScanJob &J = js.j[blockIdx.y];
    if (!J.n) {
        if (threadIdx.x == 0 && J.total) __hip_atomic_store(J.total, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    __shared__ u64 wtot[SCAN_TOP_T / 64];
    const u32 T = blockDim.x;
    const u64 nb = (J.n + js.tile - 1) / js.tile;
    const u64 per = (nb + T - 1) / T;
    const u64 a = min(nb, (u64)threadIdx.x * per), b = min(nb, a + per);
    u64 s = 0;
    for (u64 i = a; i < b; i += 8) {
        u64 x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = i + k < b ? J.bsum[i + k] : 0ull;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += x[k];
    }
    const u32 lane = lane_id(), w = threadIdx.x >> 6;
    u64 x = s;  // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
        const u64 y = __shfl_up(x, o);
        if (lane >= (u32)o) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    u64 acc = x - s;
    for (u32 i = 0; i < w; ++i) acc += wtot[i];
    // the total may live in the run's Counters, whose other fields kernels on
    // other streams update meanwhile (e.g. the column spans beside the token
    // pass): a write-through store, so no dirty copy of that line stays in
    // this XCD's L2 to be written back over their updates later
    if (threadIdx.x == T - 1 && J.total) __hip_atomic_store(J.total, acc + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (u64 i = a; i < b; i += 8) {
        u64 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = i + k < b ? J.bsum[i + k] : 0ull;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (i + k < b) {
                J.bsum[i + k] = acc;
                acc += v[k];
            }
    }
}

// CH chunks of SCAN_TILE elements a block (CH = SCAN_PER_BIG / SCAN_PER for
// long arrays), each in the blocked SCAN_PER-a-thread layout -- 16 elements
// a thread in one run had made the lanes' loads and stores 128 bytes apart
// (320 vs 171 us for 50 M) -- with every chunk's loads issued up front and
// the prefix carried from chunk to chunk
template <int CH>
__global__ __launch_bounds__(SCAN_T) void k_scan_down(ScanJobs js) {
    const ScanJob &J = js.j[blockIdx.y];
    __shared__ u64 wsum[CH][SCAN_T / 64];
    const u64 base0 = (u64)blockIdx.x * (SCAN_TILE * CH);
    if (base0 >= J.n) return;
    const u32 lane = lane_id(), w = threadIdx.x >> 6;
    // thread t owns elements base + t*SCAN_PER .. +SCAN_PER (blocked) of each chunk
    u64 v[CH][SCAN_PER], s[CH], x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        s[c] = 0;
#pragma unroll
        for (int i = 0; i < SCAN_PER; ++i) {
            const u64 idx = base0 + (u64)c * SCAN_TILE + (u64)threadIdx.x * SCAN_PER + i;
            v[c][i] = idx < J.n ? J.in[idx] : 0;
        }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
#pragma unroll
        for (int i = 0; i < SCAN_PER; ++i) s[c] += v[c][i];
        // inclusive wave scan of s
        x[c] = s[c];
        for (int o = 1; o < 64; o <<= 1) {
            const u64 y = __shfl_up(x[c], o);
            if (lane >= (u32)o) x[c] += y;
        }
        if (lane == 63) wsum[c][w] = x[c];
    }
    __syncthreads();
    u64 carry = J.bsum[blockIdx.x];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        u64 pre = carry;
        for (u32 i = 0; i < w; ++i) pre += wsum[c][i];
        pre += x[c] - s[c];
        const u64 base = base0 + (u64)c * SCAN_TILE;
#pragma unroll
        for (int i = 0; i < SCAN_PER; ++i) {
            const u64 idx = base + (u64)threadIdx.x * SCAN_PER + i;
            if (idx < J.n) J.out[idx] = pre;
            pre += v[c][i];
        }
        for (u32 i = 0; i < SCAN_T / 64; ++i) carry += wsum[c][i];
    }
}

// Exclusive scans of one or two u64 arrays (in2 null: one), totals to the
// device; bsum scratch: (n + 1023) / 1024 entries per array.
hipError_t msa_exclusive_scan2(const u64 *in, u64 n, u64 *out, u64 *bsum, u64 *total, const u64 *in2, u64 n2,
                               u64 *out2, u64 *bsum2, u64 *total2, hipStream_t s) {
    ScanJobs js{};
    js.j[0] = ScanJob{in, out, bsum, total, n};
    js.j[1] = ScanJob{in2, out2, bsum2, total2, in2 ? n2 : 0};
    const u32 ny = in2 ? 2 : 1;
    const u64 nmax = std::max(js.j[0].n, js.j[1].n);
    if (nmax == 0) {  // empty: the totals are 0 (write-through, as k_scan_top stores them)
        hipLaunchKernelGGL(k_scan_zero_totals, dim3(1), dim3(64), 0, s, js);
        return hipGetLastError();
    }
    const bool big = (nmax + SCAN_TILE - 1) / SCAN_TILE > SCAN_TOP_BIG;
    js.tile = big ? SCAN_TILE_BIG : SCAN_TILE;
    const u64 nb = (nmax + js.tile - 1) / js.tile;
    if (big) hipLaunchKernelGGL(k_scan_reduce<SCAN_PER_BIG>, dim3((u32)nb, ny), dim3(SCAN_T), 0, s, js);
    else hipLaunchKernelGGL(k_scan_reduce<SCAN_PER>, dim3((u32)nb, ny), dim3(SCAN_T), 0, s, js);
    hipLaunchKernelGGL(k_scan_top, dim3(1, ny), dim3(big ? SCAN_TOP_T : SCAN_T), 0, s, js);
    if (big) hipLaunchKernelGGL(k_scan_down<SCAN_PER_BIG / SCAN_PER>, dim3((u32)nb, ny), dim3(SCAN_T), 0, s, js);
    else hipLaunchKernelGGL(k_scan_down<1>, dim3((u32)nb, ny), dim3(SCAN_T), 0, s, js);
    return hipGetLastError();
}
hipError_t msa_exclusive_scan(const u64 *in, u64 n, u64 *out, u64 *bsum_scratch, u64 *total, hipStream_t s) {
    return msa_exclusive_scan2(in, n, out, bsum_scratch, total, nullptr, 0, nullptr, nullptr, nullptr, s);
}

// ---------------------------------------------------------------------------
// duplicate_field (parallel_spotify.c:215-255).  Writes to `out` when given;
// returns the result as (offset into out, length) -- the final trim is done
// by offset so no byte moves twice.
struct Span {
    u64 off, len;
};

__device__ Span dup_field(const u8 *f, u64 len, int preserve, u8 *out) {
    u64 s = 0, e = len;
    while (s < len && c_space(f[s])) ++s;
    while (e > s && c_space(f[e - 1])) --e;
    const bool quoted = (e > s + 1 && f[s] == '"' && f[e - 1] == '"');
    u64 j = 0;
    if (preserve && quoted) {
        if (out)
            for (u64 i = s; i < e; ++i) out[i - s] = f[i];
        Span r = {0, e - s};
        return r;  // already trimmed at both ends
    }
    u64 a = s, z = e;
    if (quoted) { ++a; --z; }
    u64 first_ns = ~0ull, last_ns = 0;
    for (u64 i = a; i < z; ++i) {
        u8 c = f[i];
        if (c == '"' && i + 1 < z && f[i + 1] == '"') ++i;
        if (out) out[j] = c;
        if (!c_space(c)) {
            if (first_ns == ~0ull) first_ns = j;
            last_ns = j;
        }
        ++j;
    }
    Span r;
    if (first_ns == ~0ull) { r.off = 0; r.len = 0; }
    else { r.off = first_ns; r.len = last_ns + 1 - first_ns; }
    return r;
}

// Bytes [off, off + 16) of the 32-byte window (a, b).
__device__ __forceinline__ u32 sel4(const uint4 &v, u32 i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
__device__ __forceinline__ uint4 funnel16(const uint4 &a, const uint4 &b, u32 off) {
    if (off == 0) return a;
    const u32 dw = off >> 2, sh = (off & 3) * 8;
    u32 d[5];
#pragma unroll
    for (u32 i = 0; i < 5; ++i) {
        const u32 k = dw + i;  // 0..7
        d[i] = k < 4 ? sel4(a, k) : sel4(b, k - 4);
    }
    uint4 r;
    r.x = (u32)((((u64)d[1] << 32) | d[0]) >> sh);
    r.y = (u32)((((u64)d[2] << 32) | d[1]) >> sh);
    r.z = (u32)((((u64)d[3] << 32) | d[2]) >> sh);
    r.w = (u32)((((u64)d[4] << 32) | d[3]) >> sh);
    return r;
}

// ---------------------------------------------------------------------------
// Short fields in registers: a 64-byte window of four aligned dwordx4 loads
// and SWAR byte-class masks (bit i = window byte i).
struct Win64 {
    uint4 q[4];
};
__device__ __forceinline__ Win64 load_win64(const u8 *__restrict__ buf, u64 s) {
    const uint4 *p = reinterpret_cast<const uint4 *>(buf + (s & ~15ull));
    Win64 w;
#pragma unroll
    for (int i = 0; i < 4; ++i) w.q[i] = p[i];
    return w;
}
__device__ __forceinline__ u32 swar_space(u32 x) {  // isspace, C locale: ' ' and 9..13
    const u32 hi = x & 0x80808080u, y = x & 0x7F7F7F7Fu;
    const u32 ctl = swar_ge7(y, 9) & ~swar_ge7(y, 14);
    return (ctl & ~hi) | swar_eq(x, ' ');
}
template <int CLS>  // 0 = space, 1 = '"', 2 = '\n' or '\r', 3 = ',', 4 = NUL
__device__ __forceinline__ u64 win_mask(const Win64 &w) {
    u64 m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const u32 d[4] = {w.q[i].x, w.q[i].y, w.q[i].z, w.q[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u32 v;
            if (CLS == 0) v = swar_space(d[k]);
            else if (CLS == 1) v = swar_eq(d[k], '"');
            else if (CLS == 2) v = swar_eq(d[k], '\n') | swar_eq(d[k], '\r');
            else if (CLS == 3) v = swar_eq(d[k], ',');
            else v = swar_eq(d[k], 0);
            m |= (u64)swar_pack4(v) << (16 * i + 4 * k);
        }
    }
    return m;
}
// w.q[i] for a run-time i, as selects on single dwords (a select of whole
// array elements is lowered to a scratch-memory index)
__device__ __forceinline__ u32 sel_d(u32 i, u32 a, u32 b, u32 c, u32 d) {
    const u32 lo = (i & 1u) ? b : a, hi = (i & 1u) ? d : c;
    return (i & 2u) ? hi : lo;
}
__device__ __forceinline__ uint4 sel_q(const Win64 &w, u32 i) {
    return make_uint4(sel_d(i, w.q[0].x, w.q[1].x, w.q[2].x, w.q[3].x), sel_d(i, w.q[0].y, w.q[1].y, w.q[2].y, w.q[3].y),
                      sel_d(i, w.q[0].z, w.q[1].z, w.q[2].z, w.q[3].z), sel_d(i, w.q[0].w, w.q[1].w, w.q[2].w, w.q[3].w));
}
// 32 window bytes starting at byte `at` (at + len <= 64), bytes >= len zeroed.
__device__ __forceinline__ void win_take32(const Win64 &w, u32 at, u32 len, uint4 *o0, uint4 *o1) {
    const u32 qi = at >> 4, off = at & 15;
    const uint4 a = sel_q(w, qi), b = sel_q(w, min(qi + 1, 3u)), c = sel_q(w, min(qi + 2, 3u));
    const uint4 x0 = funnel16(a, b, off), x1 = funnel16(b, c, off);
    u32 d[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (u32 k = 0; k < 8; ++k) {
        const u32 lo = 4 * k;
        const u32 keep = len <= lo ? 0u : (len >= lo + 4 ? 4u : len - lo);
        d[k] &= keep == 4 ? 0xFFFFFFFFu : ((1u << (8 * keep)) - 1u);
    }
    *o0 = make_uint4(d[0], d[1], d[2], d[3]);
    *o1 = make_uint4(d[4], d[5], d[6], d[7]);
}
// bytes_hash (msa_tables.h) of <= 32 bytes given as little-endian words
__device__ __forceinline__ u64 bytes_hash_words(const uint4 &o0, const uint4 &o1, u32 n) {
    const u64 w[4] = {((u64)o0.y << 32) | o0.x, ((u64)o0.w << 32) | o0.z, ((u64)o1.y << 32) | o1.x,
                      ((u64)o1.w << 32) | o1.z};
    u64 h = 0x243F6A8885A308D3ULL ^ ((u64)n * 0x9E3779B97F4A7C15ULL);
    const u32 full = n >> 3, rem = n & 7;
#pragma unroll
    for (u32 i = 0; i < 4; ++i)
        if (i < full) h = fmix64(h ^ w[i]) * 0x9E3779B97F4A7C15ULL;
    const u64 acc = rem ? (full == 0 ? w[0] : (full == 1 ? w[1] : (full == 2 ? w[2] : w[3]))) : 0ull;
    return fmix64(h ^ acc ^ ((u64)rem << 59));
}
__device__ __forceinline__ u64 bits_from(u32 lo) { return lo >= 64 ? 0ull : (~0ull << lo); }
__device__ __forceinline__ u64 bits_below(u32 hi) { return hi >= 64 ? ~0ull : ((1ull << hi) - 1ull); }
// 16 bytes at any byte address: dword-aligned loads (4 + 1) and v_alignbyte.
__device__ __forceinline__ uint4 align16(const uint4 &v, u32 d4, u32 sh) {
    return make_uint4(__builtin_amdgcn_alignbyte(v.y, v.x, sh), __builtin_amdgcn_alignbyte(v.z, v.y, sh),
                      __builtin_amdgcn_alignbyte(v.w, v.z, sh), __builtin_amdgcn_alignbyte(d4, v.w, sh));
}
__device__ __forceinline__ uint4 load16u(const u8 *__restrict__ buf, u64 s) {
    const u32 *p = reinterpret_cast<const u32 *>(buf + (s & ~3ull));
    return align16(make_uint4(p[0], p[1], p[2], p[3]), p[4], (u32)(s & 3));
}
// funnel16 without the branch: dword selects + v_alignbyte
__device__ __forceinline__ uint4 funnel16a(const uint4 &X, const uint4 &Y, u32 ph) {
    const u32 d = ph >> 2, s = ph & 3u;
    const u32 w[8] = {X.x, X.y, X.z, X.w, Y.x, Y.y, Y.z, Y.w};
    u32 c[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) c[i] = d == 0 ? w[i] : (d == 1 ? w[i + 1] : (d == 2 ? w[i + 2] : w[i + 3]));
    return make_uint4(__builtin_amdgcn_alignbyte(c[1], c[0], s), __builtin_amdgcn_alignbyte(c[2], c[1], s),
                      __builtin_amdgcn_alignbyte(c[3], c[2], s), __builtin_amdgcn_alignbyte(c[4], c[3], s));
}
// lane l receives lane l + 1's value (lane 63: 0): DPP wave shift; every lane active
__device__ __forceinline__ u32 dpp_next32(u32 v) { return __builtin_amdgcn_update_dpp(0u, v, 0x130, 0xF, 0xF, false); }
#ifndef CG_AL
#define CG_AL 0  // 1: text.csv's single-line slots by one aligned 16-byte load + the next lane's (k_col_gather)
#endif
// out with its bytes [a, b) (0 <= a <= b <= 16) taken from v
__device__ __forceinline__ uint4 bytes_blend(const uint4 &out, const uint4 &v, u32 a, u32 b) {
    const u64 lo = bits_from(8 * a) & bits_below(8 * b);
    const u64 hi = bits_from(a >= 8 ? 8 * a - 64 : 0) & (b > 8 ? bits_below(8 * b - 64) : 0ull);
    const u32 m[4] = {(u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32)};
    return make_uint4(((out.x & ~m[0]) | (v.x & m[0])), (out.y & ~m[1]) | (v.y & m[1]),
                      (out.z & ~m[2]) | (v.z & m[2]), (out.w & ~m[3]) | (v.w & m[3]));
}
__device__ __forceinline__ uint4 byte_put(uint4 o, u32 i, u32 ch) {
    const u32 s = 8 * (i & 3), m = 0xFFu << s, v = ch << s;
    if (i < 4) o.x = (o.x & ~m) | v;
    else if (i < 8) o.y = (o.y & ~m) | v;
    else if (i < 12) o.z = (o.z & ~m) | v;
    else o.w = (o.w & ~m) | v;
    return o;
}

// greedy "" pairs (duplicate_field's collapse) in a quote mask: sum of floor(run/2)
__device__ __forceinline__ u32 quote_pairs(u64 q) {
    u32 pairs = 0;
    while (q) {
        const u32 st = (u32)__ffsll((long long)q) - 1;
        const u64 rest = ~(q >> st);
        const u32 rl = rest ? (u32)__ffsll((long long)rest) - 1 : 64 - st;
        pairs += rl >> 1;
        q &= ~(bits_below(rl) << st);
    }
    return pairs;
}

// Any '"' in bytes [as, as + n): 16-byte pieces, SWAR test.
__device__ __forceinline__ bool field_has_quote(const u8 *__restrict__ buf, u64 as, u64 n) {
    for (u64 b = 0; b < n; b += 16) {
        const uint4 c = load16u(buf, as + b);
        const u32 m = swar_pack4(swar_eq(c.x, '"')) | (swar_pack4(swar_eq(c.y, '"')) << 4) |
                      (swar_pack4(swar_eq(c.z, '"')) << 8) | (swar_pack4(swar_eq(c.w, '"')) << 12);
        const u64 left = n - b;
        if (m & (left >= 16 ? 0xFFFFu : ((1u << left) - 1u))) return true;
    }
    return false;
}

// 8 dwords = 32 bytes; bytes moved up by o (0..31) positions, the top ones
// dropped: a barrel shifter (16 / 8 / 4 bytes by selects, then v_alignbyte).
__device__ __forceinline__ void v32_shl(u32 (&d)[8], u32 o) {
#pragma unroll
    for (int k = 7; k >= 0; --k) d[k] = (o & 16) ? (k >= 4 ? d[k - 4] : 0u) : d[k];
#pragma unroll
    for (int k = 7; k >= 0; --k) d[k] = (o & 8) ? (k >= 2 ? d[k - 2] : 0u) : d[k];
#pragma unroll
    for (int k = 7; k >= 0; --k) d[k] = (o & 4) ? (k >= 1 ? d[k - 1] : 0u) : d[k];
    const u32 sh = o & 3u;
    if (sh) {
#pragma unroll
        for (int k = 7; k >= 1; --k) d[k] = __builtin_amdgcn_alignbyte(d[k], d[k - 1], 4 - sh);
        d[0] <<= 8 * sh;
    }
}

// Key of a quoted artist field whose outer quotes are window bytes a < b:
// duplicate_field(line, 0) = trim(collapse(inner)), built in registers (the
// "" pairs' second quotes dropped, the kept runs shifted into place).  False
// when the key is longer than 32 bytes.
__device__ bool quoted_key_window(const Win64 &w, u32 a, u32 b, uint4 *k0, uint4 *k1, u32 *klen) {
    const u64 IM = bits_from(a + 1) & bits_below(b);
    u64 R = 0;
    for (u64 q = win_mask<1>(w) & IM; q;) {  // greedy pairs: runs of quotes
        const u32 st = (u32)__ffsll((long long)q) - 1;
        const u64 rest = ~(q >> st);
        const u32 rl = rest ? (u32)__ffsll((long long)rest) - 1 : 64u - st;
        const u64 run = bits_below(rl) << st;
        R |= run & ((st & 1u) ? 0x5555555555555555ull : 0xAAAAAAAAAAAAAAAAull);
        q &= ~run;
    }
    u64 K = IM & ~R;
    const u64 NS = K & ~win_mask<0>(w);
    if (!NS) {
        *klen = 0;
        return true;
    }
    K &= bits_from((u32)__ffsll((long long)NS) - 1) & bits_below(64u - (u32)__clzll((long long)NS));
    const u32 n = (u32)__popcll(K);
    if (n > 32) return false;
    u32 out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    u32 o = 0;
    while (K) {
        const u32 rs = (u32)__ffsll((long long)K) - 1;
        const u64 rest = ~(K >> rs);
        const u32 rl = rest ? (u32)__ffsll((long long)rest) - 1 : 64u - rs;
        uint4 t0, t1;
        win_take32(w, rs, rl, &t0, &t1);
        u32 t[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
        v32_shl(t, o);
#pragma unroll
        for (int k = 0; k < 8; ++k) out[k] |= t[k];
        o += rl;
        K &= ~(bits_below(rl) << rs);
    }
    *k0 = make_uint4(out[0], out[1], out[2], out[3]);
    *k1 = make_uint4(out[4], out[5], out[6], out[7]);
    *klen = n;
    return true;
}

// The artist pass's key for one record when artist.csv lines are its records:
// duplicate_field(line, 0) with line = duplicate_field(field0, 1) (the
// artist.csv line without its '\n'), i.e. for the trimmed field [as, ae):
//   quote-free           -> the field itself
//   quoted "..."         -> trim(collapse(inner))
//   anything else        -> the general path (byte loop, long area)
// An unquoted field with a '"' makes the shortcut unavailable (a_quoted is
// set by the caller), so its key is never used.
__device__ void artist_key_of(const u8 *__restrict__ buf, const Win64 &w0, u64 b0, u64 as, u64 ae, u64 r,
                              const AKeys &ak, Counters *ctr, int ab = 0) {
    const u64 n = ae - as;
    if (n == 0) {
        ak.key_len[r] = 0;
        return;
    }
    bool quoted, plain = false;
    if (ae - b0 <= 64) {  // the field is inside the record's first window
        const u32 a = (u32)(as - b0), b = (u32)(ae - 1 - b0);
        const u64 Q = win_mask<1>(w0) & bits_from(a) & bits_below(b + 1);
        quoted = n >= 2 && ((Q >> a) & 1) && ((Q >> b) & 1);
        plain = !Q;
        u32 ka = a, kb = b + 1;  // key = window bytes [ka, kb)
        bool ok = false;
        uint4 k0, k1;
        u32 klen = 0;
        if (!Q) {
            ok = true;
        } else if (!quoted) {
            // an unquoted field holding a '"': the shortcut is off (the caller
            // raised a_quoted), this key is never read
            ak.key_len[r] = 0;
            return;
        } else if (!(Q & bits_from(a + 1) & bits_below(b))) {
            const u64 inner = bits_from(a + 1) & bits_below(b);
            const u64 nsp = inner & ~win_mask<0>(w0);
            if (!nsp) {
                ak.key_len[r] = 0;
                return;
            }
            ka = (u32)__ffsll((long long)nsp) - 1;
            kb = 64u - (u32)__clzll((long long)nsp);
            ok = true;
        } else if (quoted_key_window(w0, a, b, &k0, &k1, &klen)) {  // inner quotes
            if (!klen) {
                ak.key_len[r] = 0;
                return;
            }
            ok = true;
            ka = 0;
            kb = klen;  // k0 / k1 hold the key already
        }
        if (ok && kb - ka <= 32) {
            if (!klen) {
                klen = kb - ka;
                win_take32(w0, ka, klen, &k0, &k1);
            }
            uint4 *dst = reinterpret_cast<uint4 *>(ak.arena + 32 * r);
            if (ab & 16384) {  // diagnostic: the key built and hashed, one store
                const u64 w0 = ((u64)k0.y << 32) | k0.x, w1 = ((u64)k0.w << 32) | k0.z;
                const u64 w2 = ((u64)k1.y << 32) | k1.x, w3 = ((u64)k1.w << 32) | k1.z;
                ak.kh1[r] = akey_fold(akey_seed(klen, 0), w0, w1, w2, w3, 0) ^
                            akey_fold(akey_seed(klen, 1), w0, w1, w2, w3, 1);
                return;
            }
            if (!(ab & 8192)) {
                dst[0] = k0;
                dst[1] = k1;
            }
            ak.key_off[r] = 32 * r;
            ak.key_len[r] = klen;
            const u64 w0 = ((u64)k0.y << 32) | k0.x, w1 = ((u64)k0.w << 32) | k0.z;
            const u64 w2 = ((u64)k1.y << 32) | k1.x, w3 = ((u64)k1.w << 32) | k1.z;
            if (ab & 2048) {
                ak.kh1[r] = w0 ^ w1 ^ w2 ^ w3;
                ak.kh2[r] = w0;
            } else {
                ak.kh1[r] = akey_fold(akey_seed(klen, 0), w0, w1, w2, w3, 0);
                ak.kh2[r] = akey_fold(akey_seed(klen, 1), w0, w1, w2, w3, 1);
            }
            return;
        }
    } else {
        quoted = n >= 2 && buf[as] == '"' && buf[ae - 1] == '"';
    }
    // A field without any '"' (the long names of the synthetic corpora): its
    // line and key are the trimmed field itself.  Copied to the long area in
    // 16-byte pieces and hashed per 32 bytes as akey_hash_bytes does -- the
    // byte loops below cost a dependent load per byte, and a wave waits for
    // its slowest lane.
    if (!plain && !quoted) plain = !field_has_quote(buf, as, n);
    if (plain) {
        const u64 room32 = (n + 31) & ~31ull;
        const u64 at = atomicAdd((unsigned long long *)&ctr->a_long, (unsigned long long)room32);
        if (at + room32 > ak.long_cap) {
            atomicOr((unsigned long long *)&ctr->a_quoted, 2ull);
            ak.key_len[r] = 0;
            return;
        }
        uint4 *dst = reinterpret_cast<uint4 *>(ak.arena + ak.long_base + at);
        u64 h1 = akey_seed(n, 0), h2 = akey_seed(n, 1);
        for (u64 b = 0; b < n; b += 32) {
            uint4 c0 = load16u(buf, as + b), c1 = load16u(buf, as + b + 16);
            const u64 left = n - b;
            if (left < 32) {
                c0 = bytes_blend(make_uint4(0, 0, 0, 0), c0, 0, (u32)min(left, (u64)16));
                c1 = left > 16 ? bytes_blend(make_uint4(0, 0, 0, 0), c1, 0, (u32)(left - 16)) : make_uint4(0, 0, 0, 0);
            }
            dst[b / 16] = c0;
            dst[b / 16 + 1] = c1;
            const u64 w0 = ((u64)c0.y << 32) | c0.x, w1 = ((u64)c0.w << 32) | c0.z;
            const u64 w2 = ((u64)c1.y << 32) | c1.x, w3 = ((u64)c1.w << 32) | c1.z;
            h1 = akey_fold(h1, w0, w1, w2, w3, 0);
            h2 = akey_fold(h2, w0, w1, w2, w3, 1);
        }
        ak.key_off[r] = ak.long_base + at;
        ak.key_len[r] = (u32)n;
        ak.kh1[r] = h1;
        ak.kh2[r] = h2;
        return;
    }
    // general path: the line (collapse "" pairs of an unquoted field), then
    // duplicate_field(line, 0) in place, in the long area
    const u64 room = n + 1;
    const u64 at = atomicAdd((unsigned long long *)&ctr->a_long, (unsigned long long)((room + 15) & ~15ull));
    if (at + room > ak.long_cap) {  // no room: the shortcut is given up, the exact reader runs
        atomicOr((unsigned long long *)&ctr->a_quoted, 2ull);
        ak.key_len[r] = 0;
        return;
    }
    u8 *dst = ak.arena + ak.long_base + at;
    u64 m = 0;
    if (quoted) {
        for (u64 i = as; i < ae; ++i) dst[m++] = buf[i];
    } else {
        for (u64 i = as; i < ae; ++i) {
            const u8 ch = buf[i];
            if (ch == '"' && i + 1 < ae && buf[i + 1] == '"') ++i;
            dst[m++] = ch;
        }
        while (m > 0 && c_space(dst[m - 1])) --m;  // trim_inplace (the front is non-space)
    }
    const Span sp = dup_field(dst, m, 0, dst);
    ak.key_off[r] = ak.long_base + at + sp.off;
    ak.key_len[r] = (u32)sp.len;
    if (sp.len) {
        ak.kh1[r] = akey_hash_bytes(dst + sp.off, sp.len, 0);
        ak.kh2[r] = akey_hash_bytes(dst + sp.off, sp.len, 1);
    }
}

// Per record (thread): the first three unquoted commas (parse_csv_line,
// parallel_spotify.c:258-304), then the spans of both column lines
// (split_dataset_columns 699-714): line = duplicate_field(field, preserve=1)
// + '\n'.  After the outer trim a quoted field -- every lyric of the real
// corpus -- is copied raw; an unquoted one has its "" pairs collapsed and
// needs no second trim (its first and last bytes are non-space and a
// collapsed pair yields '"').  Outputs per record: line length (0 = no line:
// the header, or a record parse_csv_line rejects), source offset, pairs.
//
// Commas: record-local (a record starts outside quotes), 64-byte windows
// (four dwordx4 loads) with the quote parity carried; a NUL ends the C string
// the reference splits, so commas after it do not count.  The artist field
// (<= 48 bytes) is trimmed and its pairs counted in the first window.
struct SpanOut {
    u64 *alen, *asrc;
    u32 *apairs;
    u64 *tlen, *tsrc;
    u32 *tpairs;
};

// Artist line span of record r = field 0 = [s, s + f0) (w0 = the 64-byte
// window at s & ~15), and the artist key of the lines shortcut.
__device__ __forceinline__ void rec_artist(const u8 *__restrict__ buf, const Win64 &w0, u64 s, u32 f0, u64 r,
                                           const SpanOut &o, Counters *ctr, const AKeys &ak, bool no_key = false,
                                           int ab = 0) {
    const u64 b0 = s & ~15ull;
    u64 as = s, ae = s + f0;
    u32 pairs = 0;
    if (f0 <= 48) {
        const u32 o16 = (u32)(s & 15);
        const u64 fm = bits_from(o16) & bits_below(o16 + f0);
        const u64 nsp = fm & ~win_mask<0>(w0);
        if (!nsp) {
            ae = as;
        } else {
            const u32 a = (u32)__ffsll((long long)nsp) - 1, b = 63u - (u32)__clzll((long long)nsp);
            const u64 Q = win_mask<1>(w0) & bits_from(a) & bits_below(b + 1);
            if (!(b > a && ((Q >> a) & 1) && ((Q >> b) & 1))) {
                pairs = quote_pairs(Q);
                if (Q) atomicOr((unsigned long long *)&ctr->a_quoted, 1ull);
            }
            as = b0 + a;
            ae = b0 + b + 1;
        }
    } else {
        while (as < ae && c_space(buf[as])) ++as;
        while (ae > as && c_space(buf[ae - 1])) --ae;
        if (!(ae > as + 1 && buf[as] == '"' && buf[ae - 1] == '"') && field_has_quote(buf, as, ae - as)) {
            bool anyq = false;
            for (u64 i = as; i < ae; ++i) {
                if (buf[i] != '"') continue;
                anyq = true;
                if (i + 1 < ae && buf[i + 1] == '"') { ++pairs; ++i; }
            }
            if (anyq) atomicOr((unsigned long long *)&ctr->a_quoted, 1ull);
        }
    }
    o.alen[r] = (ae - as) - pairs + 1;
    o.asrc[r] = as;
    o.apairs[r] = pairs;
    if (!no_key) artist_key_of(buf, w0, b0, as, ae, r, ak, ctr, ab);
}

__device__ __forceinline__ void rec_noline(u64 r, int want_text, const SpanOut &o, const AKeys &ak) {
    o.alen[r] = 0;
    ak.key_len[r] = 0;
    if (want_text) o.tlen[r] = 0;
}

// Per record, the exact path: the first three commas (parse_csv_line,
// parallel_spotify.c:258-304), then the spans of both column lines
// (split_dataset_columns 699-714): line = duplicate_field(field, preserve=1)
// + '\n'.  After the outer trim a quoted field -- every lyric of the real
// corpus -- is copied raw; an unquoted one has its "" pairs collapsed and
// needs no second trim (its first and last bytes are non-space and a
// collapsed pair yields '"').  Outputs per record: line length (0 = no line:
// the header, or a record parse_csv_line rejects), source offset, pairs.
//
// Commas: record-local (a record starts outside quotes), 64-byte windows
// (four dwordx4 loads) with the quote parity carried; a NUL ends the C string
// the reference splits, so commas after it do not count.  The artist field
// (<= 48 bytes) is trimmed and its pairs counted in the first window.
__device__ void rec_full(const u8 *__restrict__ buf, const u64 *__restrict__ rec_start,
                         const u32 *__restrict__ nulrel, u64 r, u64 first_rec, int want_text, const SpanOut &o,
                         Counters *ctr, const AKeys &ak, bool want_artist = true) {
    const u64 s = rec_start[r], e = rec_start[r + 1];
    const u64 b0 = s & ~15ull;
    const Win64 w0 = load_win64(buf, s);
    u32 par = 0, nc = 0, f0 = 0, f3 = 0;
    for (u64 base = b0; base < e; base += 64) {
        const Win64 w = base == b0 ? w0 : load_win64(buf, base);
        u64 valid = bits_below((u32)min(e - base, (u64)64));
        if (base < s) valid &= bits_from((u32)(s - base));
        const u64 Q = win_mask<1>(w) & valid, Z = win_mask<4>(w) & valid;
        u64 x = Q << 1;  // exclusive prefix-xor: bit i = parity of the quotes before byte i
        x ^= x << 1;
        x ^= x << 2;
        x ^= x << 4;
        x ^= x << 8;
        x ^= x << 16;
        x ^= x << 32;
        const u64 inq = x ^ (par ? ~0ull : 0ull);
        par ^= (u32)__popcll(Q) & 1u;
        u64 cu = win_mask<3>(w) & valid & ~inq;
        if (Z) cu &= bits_below((u32)__ffsll((long long)Z) - 1);
        while (cu && nc < 3) {
            const u32 b = (u32)__ffsll((long long)cu) - 1;
            cu &= cu - 1;
            ++nc;
            if (nc == 1) f0 = (u32)(base + b - s);
            if (nc == 3) f3 = (u32)(base + b + 1 - s);
        }
        if (nc >= 3 || Z) break;
    }
    if (r < first_rec || nc < 3) {
        if (want_artist) rec_noline(r, want_text, o, ak);
        else o.tlen[r] = 0;
        return;
    }
    if (want_artist) rec_artist(buf, w0, s, f0, r, o, ctr, ak);
    if (want_text) {  // field 3: after the third comma up to the first NUL; the
                      // terminator is part of the record and trimmed as whitespace
        u64 ts = s + f3, te = e;
        if (nulrel[r]) te = min(te, s + nulrel[r] - 1);
        if (te < ts) te = ts;
        while (ts < te && c_space(buf[ts])) ++ts;
        while (te > ts && c_space(buf[te - 1])) --te;
        u32 pairs = 0;
        if (!(te > ts + 1 && buf[ts] == '"' && buf[te - 1] == '"'))
            for (u64 i = ts; i + 1 < te; ++i)
                if (buf[i] == '"' && buf[i + 1] == '"') { ++pairs; ++i; }
        o.tlen[r] = (te - ts) - pairs + 1;
        o.tsrc[r] = ts;
        o.tpairs[r] = pairs;
    }
}

// Thread per record, every record on the exact path (A/B runs with the
// round-1 scan kernel, which records no spans).
__global__ __launch_bounds__(256) void k_rec_spans(const u8 *__restrict__ buf, const u64 *__restrict__ rec_start,
                                                   const u32 *__restrict__ nulrel, u64 nrec, u64 first_rec,
                                                   int want_text, SpanOut o, Counters *ctr, AKeys ak) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < nrec) rec_full(buf, rec_start, nulrel, r, first_rec, want_text, o, ctr, ak);
}

// Thread per record, from what K3 recorded (f0 / tss / tse): no comma search
// and no reads at the record's end.  The common record -- field 3 opens with
// a '"' right after its comma and the record's terminator follows a '"' --
// has the text line [tss, tse) copied raw (duplicate_field keeps a quoted
// field as is); the artist span comes from the record's first window.  Every
// other record (unquoted or space-padded lyrics, a NUL, the unterminated last
// record) is listed for k_rec_fix, the exact path.
#ifndef RF_MINW
#define RF_MINW 1  // waves per SIMD k_rec_fast is compiled for (8: <= 64 VGPRs, 4 beside the token pass's 4)
#endif
__global__ __launch_bounds__(256, RF_MINW) void k_rec_fast(const u8 *__restrict__ buf, const u64 *__restrict__ rec_start,
                                                  const u64 *__restrict__ f0p, const u64 *__restrict__ tss,
                                                  const u64 *__restrict__ tse, u64 nrec, u64 first_rec,
                                                  int want_text, SpanOut o, Counters *ctr, AKeys ak,
                                                  u64 *__restrict__ fix, int ablate) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrec) return;
    const u64 E = tse[r];
    if (r < first_rec || (E & (SPAN_NOLINE | SPAN_NUL | SPAN_FIX)) == SPAN_NOLINE) {
        rec_noline(r, want_text, o, ak);
        return;
    }
    const u64 S = tss[r];
    const u64 ts = S & SPAN_POS, te = E & SPAN_POS;
    const bool quoted = (S & SPAN_Q) && (E & SPAN_Q) && te >= ts + 2;
    if ((E & (SPAN_NUL | SPAN_FIX)) || (want_text && !quoted)) {
        const u64 at = atomicAdd((unsigned long long *)&ctr->span_fix, 1ull);
        fix[at] = r;
        return;
    }
    const u64 s = rec_start[r];
    // diagnostic ablations (results invalid): 256 no artist span, 512 no artist
    // window / key, 1024 no artist key
    if (ablate & 256) {
        o.alen[r] = 0;
    } else if (ablate & 512) {
        o.alen[r] = f0p[r] - s + 1;
        o.asrc[r] = s;
        o.apairs[r] = 0;
    } else {
        // the window's second half only when field 0 reaches into it
        const u64 f0 = f0p[r] - s;
        const uint4 *p = reinterpret_cast<const uint4 *>(buf + (s & ~15ull));
        Win64 w0;
        w0.q[0] = p[0];
        w0.q[1] = p[1];
        if ((s & 15) + f0 > 32) {
            w0.q[2] = p[2];
            w0.q[3] = p[3];
        } else {
            w0.q[2] = w0.q[3] = make_uint4(0, 0, 0, 0);
        }
        rec_artist(buf, w0, s, (u32)f0, r, o, ctr, ak, (ablate & 1024) != 0, ablate);
    }
    if (want_text) {
        o.tlen[r] = te - ts + 1;
        o.tsrc[r] = ts;
        o.tpairs[r] = 0;
    }
}

// The records k_rec_fast listed, on the exact path (count on the device).
__global__ __launch_bounds__(256) void k_rec_fix(const u8 *__restrict__ buf, const u64 *__restrict__ rec_start,
                                                 const u32 *__restrict__ nulrel, u64 first_rec, int want_text,
                                                 SpanOut o, Counters *ctr, AKeys ak, const u64 *__restrict__ fix) {
    const u64 n = *(volatile const u64 *)&ctr->span_fix;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        rec_full(buf, rec_start, nulrel, fix[i], first_rec, want_text, o, ctr, ak);
}

// Segmented gather.  A workgroup owns 256 consecutive lines (their metadata
// is one coalesced load into LDS) and therefore the contiguous output range
// [off[r0], off[r0+256]).  Its threads walk the 16-byte slots (aligned in
// memory) of that range: a slot inside one line is five dword loads +
// v_alignbyte and one 16-byte store; a slot that meets a line end is composed
// in registers from the lines it meets (byte blends + the '\n').  Only the
// range's ragged first/last slot is stored byte by byte (only the bytes this
// workgroup owns).  Lines whose "" pairs collapse get raw bytes here and are
// rewritten by k_col_collapse, launched after this kernel on the same stream.
#ifndef CG_T
#define CG_T 256
#endif
#define CG_SLOT 16
#ifndef CG_MAXS
#define CG_MAXS 4096
#endif  // slot->line map capacity (LDS); larger ranges binary-search
__global__ __launch_bounds__(CG_T) void k_col_gather(const u8 *__restrict__ buf, const u64 *__restrict__ line_len,
                                                     const u64 *__restrict__ line_off,
                                                     const u64 *__restrict__ span_src,
                                                     const u32 *__restrict__ span_pairs, u64 nrec, u64 hdr,
                                                     const u64 *__restrict__ body_p, u8 *__restrict__ col) {
    __shared__ u64 w_off[CG_T + 1], w_src[CG_T];
    const u64 body = *body_p;  // column body bytes (the scan's total, left on the device)
    __shared__ u32 smap[CG_MAXS];  // slot -> line holding the slot's first byte
    __shared__ u32 tmax[CG_T];
    const u64 r0 = (u64)blockIdx.x * CG_T;
    const u32 wn = (u32)min((u64)CG_T, nrec - r0);
    const u32 t = threadIdx.x;
    if (t < wn) {
        w_off[t] = line_off[r0 + t];
        w_src[t] = span_src[r0 + t];
    }
    if (t == 0) w_off[wn] = (r0 + wn < nrec) ? line_off[r0 + wn] : body;
    __syncthreads();
    const u64 O0 = hdr + w_off[0], O1 = hdr + w_off[wn];  // absolute column bytes owned
    if (O1 <= O0) return;
    const u64 S0 = O0 & ~(u64)(CG_SLOT - 1);
    const u64 nslots = (O1 - S0 + CG_SLOT - 1) / CG_SLOT;
    const bool mapped = nslots <= CG_MAXS;
    if (mapped) {
        // scatter each line to the first slot starting inside it, then prefix-max
        for (u32 i = t; i < nslots; i += CG_T) smap[i] = 0;
        __syncthreads();
        if (t < wn) {
            const u64 fs = (hdr + w_off[t] - S0 + CG_SLOT - 1) / CG_SLOT;
            if (fs < nslots) atomicMax(&smap[fs], (u32)t);
        }
        __syncthreads();
        const u32 per = (u32)((nslots + CG_T - 1) / CG_T);
        const u32 a = min((u32)nslots, t * per), b = min((u32)nslots, a + per);
        u32 m = 0;
        for (u32 i = a; i < b; ++i) m = max(m, smap[i]);
        tmax[t] = m;
        __syncthreads();
        if (t < 64) {  // exclusive prefix-max of the 256 per-thread maxima, one wave
            const u32 v0 = tmax[4 * t], v1 = max(v0, tmax[4 * t + 1]), v2 = max(v1, tmax[4 * t + 2]),
                      v3 = max(v2, tmax[4 * t + 3]);
            u32 inc = v3;
            for (u32 o = 1; o < 64; o <<= 1) {
                const u32 y = __shfl_up(inc, o);
                if (t >= o) inc = max(inc, y);
            }
            u32 ex = __shfl_up(inc, 1);
            if (t == 0) ex = 0;
            tmax[4 * t] = ex;
            tmax[4 * t + 1] = max(ex, v0);
            tmax[4 * t + 2] = max(ex, v1);
            tmax[4 * t + 3] = max(ex, v2);
        }
        __syncthreads();
        u32 run = tmax[t];
        for (u32 i = a; i < b; ++i) { run = max(run, smap[i]); smap[i] = run; }
        __syncthreads();
    }
    // slots in batches of CG_B per thread: every single-line slot's loads of
    // the batch are issued before the first store (memory-level parallelism)
#ifndef CG_B
#define CG_B 2
#endif
#if CG_AL
    const u32 lane = t & 63u;
#endif
    for (u64 s0 = t; s0 < nslots; s0 += (u64)CG_B * CG_T) {
        uint4 va[CG_B];
        u32 jj[CG_B], d4[CG_B], sh[CG_B];
        bool fast[CG_B];
#if CG_AL
        uint4 vb[CG_B];  // the 16 aligned bytes after va's: own load, or the next lane's va
        bool ownb[CG_B];
#endif
#pragma unroll
        for (int k = 0; k < CG_B; ++k) {
            const u64 si = s0 + (u64)k * CG_T;
            fast[k] = false;
            jj[k] = 0;
            sh[k] = 0;
            d4[k] = 0;
#if CG_AL
            va[k] = vb[k] = make_uint4(0, 0, 0, 0);
            ownb[k] = false;
#endif
            if (si >= nslots) continue;
            const u64 A = S0 + si * CG_SLOT;
            const u64 lo = max(A, O0), hi = min(A + CG_SLOT, O1);
            u32 j;
            if (mapped) {
                j = smap[si];
            } else {  // last j with hdr + w_off[j] <= lo
                u32 jl = 0, jh = wn;
                while (jh - jl > 1) {
                    const u32 mid = (jl + jh) >> 1;
                    if (hdr + w_off[mid] <= lo) jl = mid;
                    else jh = mid;
                }
                j = jl;
            }
            while (j + 1 < wn && hdr + w_off[j + 1] <= lo) ++j;  // skip empty lines
            jj[k] = j;
            const u64 lstart = hdr + w_off[j], lend = hdr + w_off[j + 1];  // '\n' at lend-1
            if (lo == A && hi == A + CG_SLOT && A + CG_SLOT < lend) {
                const u64 src = w_src[j] + (A - lstart);
#if CG_AL
                // one aligned 16-byte load; the 16 bytes after it are the next
                // lane's load when that lane's slot is the next slot of this
                // line (a fast one too), else this lane loads them as well
                const size_t pa = (size_t)(buf + src);
                const uint4 *p = reinterpret_cast<const uint4 *>(pa & ~(size_t)15);
                va[k] = p[0];
                sh[k] = (u32)(pa & 15);
                ownb[k] = sh[k] && (lane == 63 || !(A + 2 * CG_SLOT < lend && A + 2 * CG_SLOT <= O1));
                if (ownb[k]) vb[k] = p[1];
#else
                const u32 *p = reinterpret_cast<const u32 *>(buf + (src & ~3ull));
                va[k] = make_uint4(p[0], p[1], p[2], p[3]);
                d4[k] = p[4];
                sh[k] = (u32)(src & 3);
#endif
                fast[k] = true;
            }
        }
#if CG_AL
#pragma unroll
        for (int k = 0; k < CG_B; ++k) {  // every lane active: DPP reads the source lane's register
            const uint4 nx = make_uint4(dpp_next32(va[k].x), dpp_next32(va[k].y), dpp_next32(va[k].z),
                                        dpp_next32(va[k].w));
            if (!ownb[k]) vb[k] = nx;
        }
#endif
#pragma unroll
        for (int k = 0; k < CG_B; ++k) {
            const u64 si = s0 + (u64)k * CG_T;
            if (si >= nslots) continue;
            const u64 A = S0 + si * CG_SLOT;
            if (fast[k]) {
#if CG_AL
                *reinterpret_cast<uint4 *>(col + A) = funnel16a(va[k], vb[k], sh[k]);
#else
                *reinterpret_cast<uint4 *>(col + A) = align16(va[k], d4[k], sh[k]);
#endif
                continue;
            }
            // the slot holds a line end: compose it from the (usually two) lines
            // it meets, in registers
            const u64 lo = max(A, O0), hi = min(A + CG_SLOT, O1);
            {  // the common case: line j's tail, its '\n', line j+1's head to the
               // slot's end -- two unaligned loads and a byte-mask select (the
               // line loop below costs ~3x the instructions, and every wave has
               // a few such slots per batch)
                const u32 j = jj[k];
                const u64 ls = hdr + w_off[j], le = hdr + w_off[j + 1];  // '\n' at le - 1
                if (lo == A && hi == A + CG_SLOT && j + 1 < wn && ls <= A && le - 1 >= A && le - 1 < A + CG_SLOT &&
                    hdr + w_off[j + 2] > A + CG_SLOT && w_src[j + 1] + A >= le) {
                    const u32 e = (u32)(le - 1 - A);  // 0..15
                    const uint4 X = load16u(buf, w_src[j] + (A - ls));
                    const uint4 Y = load16u(buf, w_src[j + 1] + A - le);
                    const u64 xl = e >= 8 ? ~0ull : bits_below(8 * e), xh = e >= 8 ? bits_below(8 * e - 64) : 0ull;
                    const u64 nl = e >= 8 ? 0ull : (0x0Aull << (8 * e)), nh = e >= 8 ? (0x0Aull << (8 * e - 64)) : 0ull;
                    const u64 yl = ~(xl | (0xFFull << (8 * (e & 7))) * (e < 8));
                    const u64 yh = ~(xh | (e >= 8 ? (0xFFull << (8 * (e - 8))) : 0ull));
                    const u64 Xl = ((u64)X.y << 32) | X.x, Xh = ((u64)X.w << 32) | X.z;
                    const u64 Yl = ((u64)Y.y << 32) | Y.x, Yh = ((u64)Y.w << 32) | Y.z;
                    const u64 ol = (Xl & xl) | (Yl & yl) | nl, oh = (Xh & xh) | (Yh & yh) | nh;
                    *reinterpret_cast<uint4 *>(col + A) = make_uint4((u32)ol, (u32)(ol >> 32), (u32)oh, (u32)(oh >> 32));
                    continue;
                }
            }
            uint4 out = make_uint4(0, 0, 0, 0);
            bool ok = true;
            for (u32 j = jj[k]; j < wn; ++j) {
                const u64 ls = hdr + w_off[j], le = hdr + w_off[j + 1];
                if (ls >= hi) break;
                if (le > ls) {
                    const u64 a = max(A, ls), b = min(A + CG_SLOT, le - 1);
                    if (b > a) {
                        if (w_src[j] + A < ls) { ok = false; break; }  // window would start before the buffer
                        out = bytes_blend(out, load16u(buf, w_src[j] + A - ls), (u32)(a - A), (u32)(b - A));
                    }
                    if (le - 1 >= A && le - 1 < A + CG_SLOT) out = byte_put(out, (u32)(le - 1 - A), '\n');
                }
                if (le >= hi) break;
            }
            if (ok && lo == A && hi == A + CG_SLOT) {
                *reinterpret_cast<uint4 *>(col + A) = out;
            } else if (ok) {  // the workgroup's ragged first / last slot: owned bytes only
                const u32 d[4] = {out.x, out.y, out.z, out.w};
                for (u64 p = lo; p < hi; ++p) col[p] = (u8)(d[(p - A) >> 2] >> (8 * ((p - A) & 3)));
            } else {
                u32 j = jj[k];
                for (u64 p = lo; p < hi; ++p) {
                    while (p >= hdr + w_off[j + 1]) ++j;
                    const u64 ls = hdr + w_off[j], le = hdr + w_off[j + 1];
                    col[p] = (p + 1 == le) ? (u8)'\n' : buf[w_src[j] + (p - ls)];
                }
            }
        }
    }
}

// Short lines (the artist column, ~15 bytes a line): one thread per line
// writes its bytes into LDS at the line's output offset (source from a 64-byte
// register window; longer lines and lines with "" pairs by a byte loop), then
// the workgroup stores its contiguous output range with aligned 16-byte
// stores (ragged first/last chunk byte by byte).  A workgroup whose range does
// not fit the stage writes its lines straight to the column.
#define CL_T 256
#define CL_LDS 16384
template <typename P>
__device__ __forceinline__ void put_line(P dst, const u8 *__restrict__ buf, u64 s, u64 len, u32 pairs,
                                         const uint4 *__restrict__ key32 = nullptr) {
    if (key32) {  // the line is the record's artist key: its 32-byte arena slot (dense, just written)
        const uint4 x0 = key32[0], x1 = key32[1];
        const u32 d[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (u32 k = 0; k < 8; ++k) {
            if (4 * k >= len) break;
#pragma unroll
            for (u32 b = 0; b < 4; ++b)
                if (4 * k + b < len) dst[4 * k + b] = (u8)(d[k] >> (8 * b));
        }
    } else if (!pairs && (s & 15) + len <= 64) {
        const Win64 w = load_win64(buf, s);
        const u32 o = (u32)(s & 15);
        uint4 x0, x1, y0, y1;
        win_take32(w, o, (u32)min(len, (u64)32), &x0, &x1);
        win_take32(w, o + 32, len > 32 ? (u32)len - 32 : 0u, &y0, &y1);
        const u32 d[16] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w,
                           y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
#pragma unroll
        for (u32 k = 0; k < 16; ++k) {
            if (4 * k >= len) break;
#pragma unroll
            for (u32 b = 0; b < 4; ++b)
                if (4 * k + b < len) dst[4 * k + b] = (u8)(d[k] >> (8 * b));
        }
    } else {
        const u64 n = len + pairs;
        u64 j = 0;
        for (u64 i = 0; i < n; ++i) {
            const u8 ch = buf[s + i];
            if (pairs && ch == '"' && i + 1 < n && buf[s + i + 1] == '"') ++i;
            dst[j++] = ch;
        }
    }
    dst[len] = '\n';
}

__global__ __launch_bounds__(CL_T) void k_col_lines(const u8 *__restrict__ buf, const u64 *__restrict__ line_len,
                                                    const u64 *__restrict__ line_off, const u64 *__restrict__ span_src,
                                                    const u32 *__restrict__ span_pairs, u64 nrec, u64 hdr,
                                                    const u64 *__restrict__ body_p, u8 *__restrict__ col,
                                                    const u8 *__restrict__ arena, const u64 *__restrict__ key_off,
                                                    const u32 *__restrict__ key_len) {
    const u64 body = *body_p;
    __shared__ __attribute__((aligned(16))) u8 st[CL_LDS];
    const u64 r0 = (u64)blockIdx.x * CL_T;
    const u32 t = threadIdx.x;
    const u64 r = r0 + t;
    const u64 wn = min((u64)CL_T, nrec - r0);
    const u64 B0 = line_off[r0];
    const u64 B1 = (r0 + wn < nrec) ? line_off[r0 + wn] : body;
    const u64 A0 = hdr + B0, A1 = hdr + B1;  // this workgroup's output bytes
    const u64 lead = A0 & 15;                // st[i] <-> col[(A0 & ~15) + i]
    const bool staged = (A1 - A0) + lead <= CL_LDS;
    if (r < nrec) {
        const u64 L = line_len[r];
        if (L) {
            // an artist line equal to its key (same length: nothing stripped,
            // nothing collapsed) is read from the key's arena slot
            const uint4 *k32 = (arena && key_off[r] == 32 * r && (u64)key_len[r] + 1 == L)
                                   ? reinterpret_cast<const uint4 *>(arena + 32 * r) : nullptr;
            if (staged) put_line(st + lead + (line_off[r] - B0), buf, span_src[r], L - 1, span_pairs[r], k32);
            else put_line(col + hdr + line_off[r], buf, span_src[r], L - 1, span_pairs[r], k32);
        }
    }
    if (!staged) return;
    __syncthreads();
    const u64 C0 = A0 & ~15ull;
    const u64 nch = (A1 - C0 + 15) / 16;
    for (u64 k = t; k < nch; k += CL_T) {
        const u64 a = C0 + 16 * k;
        if (a >= A0 && a + 16 <= A1) {
            *reinterpret_cast<uint4 *>(col + a) = *reinterpret_cast<const uint4 *>(st + 16 * k);
        } else {
            for (u32 b = 0; b < 16; ++b) {
                const u64 x = a + b;
                if (x >= A0 && x < A1) col[x] = st[16 * k + b];
            }
        }
    }
}

// Lines with "" pairs to collapse (duplicate_field, parallel_spotify.c:243-250).
__global__ void k_col_collapse(const u8 *__restrict__ buf, const u64 *__restrict__ line_len,
                               const u64 *__restrict__ line_off, const u64 *__restrict__ span_src,
                               const u32 *__restrict__ span_pairs, u64 nrec, u64 hdr, u8 *__restrict__ col) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrec || !span_pairs[r] || !line_len[r]) return;
    const u64 len = line_len[r] - 1, n = len + span_pairs[r];
    const u8 *src = buf + span_src[r];
    u8 *dst = col + hdr + line_off[r];
    u64 j = 0;
    for (u64 i = 0; i < n; ++i) {
        const u8 ch = src[i];
        if (ch == '"' && i + 1 < n && src[i + 1] == '"') ++i;
        dst[j++] = ch;
    }
    dst[len] = '\n';
}

// Artist pass (parallel_spotify.c:948-998): per artist.csv record, strip EOL,
// duplicate_field(line, 0), count non-empty names.  Records are either the
// artist.csv records found by the exact reader (ar_start) or -- when every
// artist line is one artist.csv record (no unquoted artist field holds a
// '"', checked by k_rec_spans) -- the lines themselves (hdr + line_off[j],
// line_len[j]; a record without a line has length 0 and is no song).
//
// Key bytes go to the arena (<= 32 bytes: an aligned 32-byte slot per record,
// built in registers; longer / escaped names: at the record's own offset).
// Counting is privatised in ONE workgroup-wide LDS table per CU (64-bit key
// hash, 4-slot buckets, 8192 slots); each distinct key is added to the HBM
// table once per workgroup.  Exactness: every record's bytes are compared
// with its workgroup's first record of that hash (after the workgroup
// barrier, so the bytes are visible), and each workgroup's first record with
// the global representative (k_artist_verify_reps, next launch).
#define AK_T 1024
#define AK_SLOTS 8192
#define AK_NB (AK_SLOTS / 4)
#define AK_LOCAL (1ull << 63)
#define AK_VREP (1ull << 62)   // verify against the HBM table's representative
#define AK_SLOTMASK ((1ull << 62) - 1)
static_assert(AK_SLOTS * 16 <= 160 * 1024, "artist LDS table exceeds the CU");

__device__ __forceinline__ bool keys_equal(const u8 *__restrict__ arena, u64 oa, u32 na, u64 ob, u32 nb) {
    if (na != nb) return false;
    if (na <= 32 && ((oa | ob) & 15) == 0) {  // aligned 32-byte slots: vector compare
        const uint4 *pa = reinterpret_cast<const uint4 *>(arena + oa), *pb = reinterpret_cast<const uint4 *>(arena + ob);
        const uint4 a0 = pa[0], b0 = pb[0];
        const uint4 a1 = na > 16 ? pa[1] : make_uint4(0, 0, 0, 0), b1 = na > 16 ? pb[1] : make_uint4(0, 0, 0, 0);
        const u32 x[8] = {a0.x ^ b0.x, a0.y ^ b0.y, a0.z ^ b0.z, a0.w ^ b0.w,
                          a1.x ^ b1.x, a1.y ^ b1.y, a1.z ^ b1.z, a1.w ^ b1.w};
        u32 acc = 0;
#pragma unroll
        for (u32 k = 0; k < 8; ++k) {
            const u32 lo = 4 * k;
            const u32 keep = na <= lo ? 0u : (na >= lo + 4 ? 4u : na - lo);
            acc |= x[k] & (keep == 4 ? 0xFFFFFFFFu : ((1u << (8 * keep)) - 1u));
        }
        return acc == 0;
    }
    const u8 *a = arena + oa, *b = arena + ob;
    for (u32 i = 0; i < na; ++i)
        if (a[i] != b[i]) return false;
    return true;
}

// One artist record (the body of k_artist_key's phase 1).
template <bool LINES>
__device__ __forceinline__ void artist_one(u64 j, u64 s, u64 L, const Win64 win, const u8 *__restrict__ col,
                                           u8 *__restrict__ arena, u64 *__restrict__ key_off,
                                           u32 *__restrict__ key_len, u64 *__restrict__ key_slot, u64 *atab,
                                           u64 amask, u32 *alist, u64 alist_cap, Counters *ctr, u64 short_base,
                                           u64 *lh, u32 *lc, u32 *lrep, u32 &songs) {
    if (L == 0) {  // no line: not an artist.csv record
        key_len[j] = 0;
        key_slot[j] = ~0ull;
        return;
    }
    ++songs;
    u64 h = 0;
    u32 klen = 0;
    bool fast = false;
    if (L <= 48) {
        // registers: strip EOL, trim; a line without '"' is its own key
        const Win64 &w = win;
        const u32 o = (u32)(s & 15);
        const u64 fm = bits_from(o) & bits_below(o + (u32)L);
        const u64 ne = fm & ~win_mask<2>(w);
        const u32 endp = ne ? 64u - (u32)__clzll((long long)ne) : o;  // past the last non-EOL byte
        const u64 f2 = fm & bits_below(endp);
        const u64 nsp = f2 & ~win_mask<0>(w);
        if (!nsp) {
            fast = true;  // empty name: a song, not an artist
        } else if (!(f2 & win_mask<1>(w))) {
            const u32 a = (u32)__ffsll((long long)nsp) - 1, b = 63u - (u32)__clzll((long long)nsp);
            if (b - a + 1 <= 32) {
                klen = b - a + 1;
                uint4 k0, k1;
                win_take32(w, a, klen, &k0, &k1);
                h = bytes_hash_words(k0, k1, klen);
                uint4 *dst = reinterpret_cast<uint4 *>(arena + short_base + 32 * j);
                dst[0] = k0;
                dst[1] = k1;
                key_off[j] = short_base + 32 * j;
                fast = true;
            }
        }
    }
    if (!fast) {
        u64 n = L;
        const u8 *p = col + s;
        while (n > 0 && (p[n - 1] == '\n' || p[n - 1] == '\r')) --n;
        const Span sp = dup_field(p, n, 0, arena + s);
        key_off[j] = s + sp.off;
        klen = (u32)sp.len;
        if (klen) h = bytes_hash(arena + s + sp.off, sp.len, 0);
    }
    key_len[j] = klen;
    if (klen == 0) {
        key_slot[j] = ~0ull;
        return;
    }
    if (h == 0) h = 0x8000000000000000ULL;
    u32 b = (u32)(((h >> 32) * (u64)AK_NB) >> 32);
    u64 ks = ~0ull;
#pragma unroll
    for (int p = 0; p < 2 && ks == ~0ull; ++p) {
        const u32 base = b * 4;
        const ulonglong2 q0 = *reinterpret_cast<const ulonglong2 *>(&lh[base]);
        const ulonglong2 q1 = *reinterpret_cast<const ulonglong2 *>(&lh[base + 2]);
        const u64 kk[4] = {q0.x, q0.y, q1.x, q1.y};
        u32 hit = kk[0] == h ? 0u : (kk[1] == h ? 1u : (kk[2] == h ? 2u : (kk[3] == h ? 3u : 4u)));
        if (hit < 4) {
            atomicAdd(&lc[base + hit], 1u);
            ks = AK_LOCAL | (base + hit);
            break;
        }
        for (u32 i = 0; i < 4; ++i) {
            if (kk[i] != 0) continue;
            const u64 old = atomicCAS((unsigned long long *)&lh[base + i], 0ull, (unsigned long long)h);
            if (old == 0) lrep[base + i] = (u32)j;
            if (old == 0 || old == h) {
                atomicAdd(&lc[base + i], 1u);
                ks = AK_LOCAL | (base + i);
                break;
            }
        }
        b = (b + 1 == AK_NB) ? 0 : b + 1;
    }
    if (ks == ~0ull) {  // the workgroup's table is full: straight to HBM
        const u64 g = h_insert(atab, amask, h, 1, j, alist, alist_cap, &ctr->a_claimed, ctr, OVF_A);
        ks = g == ~0ull ? ~0ull : (g | AK_VREP);
    }
    key_slot[j] = ks;
}

template <bool LINES>
__global__ __launch_bounds__(AK_T) void k_artist_key(const u8 *__restrict__ col, const u64 *__restrict__ ar_start,
                                                     const u64 *__restrict__ line_off,
                                                     const u64 *__restrict__ line_len, u64 hdr, u64 nrec,
                                                     u8 *__restrict__ arena, u64 *__restrict__ key_off,
                                                     u32 *__restrict__ key_len, u64 *__restrict__ key_slot, u64 *atab,
                                                     u64 amask, u32 *alist, u64 alist_cap, Counters *ctr,
                                                     u64 short_base, int abl) {
    __shared__ u64 lh[AK_SLOTS];   // key hash; after the flush: the global slot
    __shared__ u32 lc[AK_SLOTS];   // count
    __shared__ u32 lrep[AK_SLOTS]; // the workgroup's first record with this hash
    __shared__ u32 songs_wg;
    for (u32 i = threadIdx.x; i < AK_SLOTS; i += AK_T) { lh[i] = 0; lc[i] = 0; }
    if (threadIdx.x == 0) songs_wg = 0;
    __syncthreads();
    const u64 stride = (u64)gridDim.x * AK_T;
    u32 songs = 0;
    // AK_B records per thread and step, their loads issued together (memory-
    // level parallelism: each record is a chain of dependent loads)
#define AK_B 2
    for (u64 jb = (u64)blockIdx.x * AK_T + threadIdx.x; jb < nrec; jb += AK_B * stride) {
    u64 sB[AK_B], LB[AK_B];
    Win64 wB[AK_B];
#pragma unroll
    for (int u = 0; u < AK_B; ++u) {
        const u64 j = jb + u * stride;
        sB[u] = 0;
        LB[u] = 0;
        if (j < nrec) {
            if (LINES) {
                LB[u] = line_len[j];
                sB[u] = hdr + line_off[j];
            } else {
                sB[u] = ar_start[j];
                LB[u] = ar_start[j + 1] - sB[u];  // the record incl. its terminator
            }
        }
    }
#pragma unroll
    for (int u = 0; u < AK_B; ++u) wB[u] = load_win64(col, sB[u]);  // in bounds for every record (padding)
#pragma unroll
    for (int u = 0; u < AK_B; ++u) {
        const u64 j = jb + u * stride;
        if (j < nrec)
            artist_one<LINES>(j, sB[u], LB[u], wB[u], col, arena, key_off, key_len, key_slot, atab, amask, alist,
                              alist_cap, ctr, short_base, lh, lc, lrep, songs);
    }
    }
    if (LINES && songs) atomicAdd(&songs_wg, songs);
    __syncthreads();
    // one HBM insert per distinct key of the workgroup
    for (u32 i = threadIdx.x; i < AK_SLOTS; i += AK_T) {
        const u32 cnt = lc[i];
        if (cnt) {  // MSA_ABLATE 512: no HBM inserts (diagnostic, results invalid; no slot is used)
            lh[i] = (abl & 512) ? ~0ull
                                : h_insert(atab, amask, lh[i], cnt, lrep[i], alist, alist_cap, &ctr->a_claimed, ctr, OVF_A);
        }
    }
    if (LINES && threadIdx.x == 0 && songs_wg) atomicAdd((unsigned long long *)&ctr->songs, (unsigned long long)songs_wg);
    __syncthreads();
    // global slots; every record's bytes against its workgroup representative
    for (u64 jb = (u64)blockIdx.x * AK_T + threadIdx.x; jb < nrec; jb += AK_B * stride) {
        u64 kB[AK_B];
#pragma unroll
        for (int u = 0; u < AK_B; ++u) kB[u] = jb + u * stride < nrec ? key_slot[jb + u * stride] : ~0ull;
        u64 oa[AK_B], ob[AK_B];
        u32 na[AK_B], nb[AK_B];
        bool cmp[AK_B];
#pragma unroll
        for (int u = 0; u < AK_B; ++u) {
            const u64 j = jb + u * stride, k = kB[u];
            cmp[u] = false;
            if (k == ~0ull || !(k & AK_LOCAL)) continue;
            const u32 q = (u32)(k & (AK_SLOTS - 1));
            const u64 g = lh[q];
            if (g == ~0ull) {  // the HBM table overflowed: the run is repeated with a bigger table
                key_slot[j] = ~0ull;
                continue;
            }
            const u32 rep = lrep[q];
            if (rep == (u32)j) {
                key_slot[j] = g | AK_VREP;
            } else {
                key_slot[j] = g;
                cmp[u] = true;
                oa[u] = key_off[j];
                na[u] = key_len[j];
                ob[u] = key_off[rep];
                nb[u] = key_len[rep];
            }
        }
#pragma unroll
        for (int u = 0; u < AK_B; ++u)
            if (cmp[u] && !(abl & 256) && !keys_equal(arena, oa[u], na[u], ob[u], nb[u]))
                atomicAdd((unsigned long long *)&ctr->collision, 1ull);
    }
}

// The artist pass when artist.csv lines are its records: count the keys
// k_rec_spans built.  One workgroup per CU counts a contiguous range of
// records in an LDS table (64-bit hash h1; per slot the count, the sum of the
// second hashes h2 and the first record); each distinct key then goes to the
// HBM table once per workgroup, flushes staggered so that the workgroups do
// not all hit the same keys at once.  A slot whose sum of h2 is not
// count x h2(first record) holds two different keys: reported, never merged
// silently (k_artist_h2_check does the same for the HBM table).
#define AC_T 1024
#ifndef AC_SLOTS
#define AC_SLOTS 6144
#endif
#define AC_PARTS 16       // hash partitions of the flush logs (k_artist_merge)
#define AC_NB (AC_SLOTS / 4)
static_assert(AC_SLOTS * 24 + 16 <= 160 * 1024, "artist count LDS exceeds the CU");

__global__ __launch_bounds__(AC_T) void k_artist_count(const u64 *__restrict__ line_len,
                                                       const u32 *__restrict__ key_len, const u64 *__restrict__ kh1,
                                                       const u64 *__restrict__ kh2, u64 nrec, u64 *atab, u64 amask,
                                                       u32 *alist, u64 alist_cap, Counters *ctr, int ablate,
                                                       ulonglong2 *__restrict__ alog, u32 *__restrict__ alog_n,
                                                       u32 alog_cap) {
    __shared__ u64 lh[AC_SLOTS];
    __shared__ u64 lsum[AC_SLOTS];
    __shared__ u32 lc[AC_SLOTS];
    __shared__ u32 lrep[AC_SLOTS];
    __shared__ u32 songs_wg;
    for (u32 i = threadIdx.x; i < AC_SLOTS; i += AC_T) { lh[i] = 0; lsum[i] = 0; lc[i] = 0; }
    if (threadIdx.x == 0) songs_wg = 0;
    __syncthreads();
    const u64 per = (nrec + gridDim.x - 1) / gridDim.x;
    const u64 r0 = (u64)blockIdx.x * per, r1 = min(nrec, r0 + per);
    u32 songs = 0;
    for (u64 r = r0 + threadIdx.x; r < r1; r += AC_T) {
        if (!line_len[r]) continue;  // no line: no artist.csv record
        ++songs;
        const u32 klen = key_len[r];
        if (!klen) continue;         // empty name: a song, not an artist
        u64 h = kh1[r];
        const u64 h2 = kh2[r];
        if (h == 0) h = 0x8000000000000000ULL;
        u32 b = (u32)(((h >> 32) * (u64)AC_NB) >> 32);
        bool done = false;
#pragma unroll
        for (int p = 0; p < 2 && !done; ++p) {
            const u32 base = b * 4;
            const ulonglong2 q0 = *reinterpret_cast<const ulonglong2 *>(&lh[base]);
            const ulonglong2 q1 = *reinterpret_cast<const ulonglong2 *>(&lh[base + 2]);
            const u64 kk[4] = {q0.x, q0.y, q1.x, q1.y};
            u32 i = kk[0] == h ? 0u : (kk[1] == h ? 1u : (kk[2] == h ? 2u : (kk[3] == h ? 3u : 4u)));
            if (i == 4) {
                for (u32 e = 0; e < 4 && !done; ++e) {
                    if (kk[e] != 0) continue;
                    const u64 old = atomicCAS((unsigned long long *)&lh[base + e], 0ull, (unsigned long long)h);
                    if (old == 0) lrep[base + e] = (u32)(r - r0);
                    if (old == 0 || old == h) { i = e; done = true; }
                }
            } else {
                done = true;
            }
            if (done) {
                atomicAdd(&lc[base + i], 1u);
                atomicAdd((unsigned long long *)&lsum[base + i], (unsigned long long)h2);
            }
            b = (b + 1 == AC_NB) ? 0 : b + 1;
        }
        if (!done)  // the workgroup's table is full: straight to HBM
            h_insert2(atab, amask, h, 1, r, h2, alist, alist_cap, &ctr->a_claimed, ctr, OVF_A);
    }
    if (songs) atomicAdd(&songs_wg, songs);
    __syncthreads();
    if (threadIdx.x == 0 && songs_wg) atomicAdd((unsigned long long *)&ctr->songs, (unsigned long long)songs_wg);
    // flush: every workgroup holds the Zipf head of the artists, so the entries
    // go to per-(workgroup, hash partition) logs and k_artist_merge inserts
    // each distinct key once per merging workgroup (a full log partition:
    // straight to HBM)
    __shared__ u32 lcur[AC_PARTS];
    if (threadIdx.x < AC_PARTS) lcur[threadIdx.x] = 0;
    __syncthreads();
    for (u32 i = threadIdx.x; i < AC_SLOTS && !(ablate & 65536); i += AC_T) {  // 65536: no flush (diagnostic)
        const u32 cnt = lc[i];
        if (!cnt) continue;
        const u64 rep = r0 + lrep[i];
        if (lsum[i] != (u64)cnt * kh2[rep]) atomicAdd((unsigned long long *)&ctr->collision, 1ull);
        const u32 part = (u32)(lh[i] >> 60) & (AC_PARTS - 1);
        const u32 at = atomicAdd(&lcur[part], 1u);
        if (at < alog_cap) {
            ulonglong2 *e = alog + 2 * (((u64)blockIdx.x * AC_PARTS + part) * alog_cap + at);
            e[0] = make_ulonglong2(lh[i], (u64)cnt);
            e[1] = make_ulonglong2(lsum[i], rep);
        } else {
            h_insert2(atab, amask, lh[i], cnt, rep, lsum[i], alist, alist_cap, &ctr->a_claimed, ctr, OVF_A);
        }
    }
    __syncthreads();
    if (threadIdx.x < AC_PARTS) alog_n[blockIdx.x * AC_PARTS + threadIdx.x] = min(lcur[threadIdx.x], alog_cap);
}

// Workgroup (partition p, group g) folds partition p of the artist logs of
// count workgroups g, g + G, ... in LDS (counts and h2 sums added, the lowest
// representative kept), then adds each distinct hash to the HBM table once.
#define AM_T 1024
#define AM_SLOTS 4096
#define AM_STAGE 4096
__global__ __launch_bounds__(AM_T) void k_artist_merge(const ulonglong2 *__restrict__ alog,
                                                       const u32 *__restrict__ alog_n, u32 alog_cap, u32 nsrc,
                                                       u32 groups, u64 *atab, u64 amask, u32 *alist, u64 alist_cap,
                                                       Counters *ctr) {
    __shared__ u64 mh[AM_SLOTS], mc[AM_SLOTS], ms[AM_SLOTS], mr[AM_SLOTS];
    __shared__ u32 staged[AM_STAGE], nst;  // the workgroup's new HBM slots (stage_new)
    __shared__ u64 gbase;
    for (u32 i = threadIdx.x; i < AM_SLOTS; i += AM_T) { mh[i] = 0; mc[i] = 0; ms[i] = 0; mr[i] = ~0ull; }
    if (threadIdx.x == 0) nst = 0;
    __syncthreads();
    const u32 part = blockIdx.x % AC_PARTS, g = blockIdx.x / AC_PARTS;
    for (u32 src = g; src < nsrc; src += groups) {
        const u32 n = alog_n[src * AC_PARTS + part];
        const ulonglong2 *e = alog + 2 * ((u64)src * AC_PARTS + part) * alog_cap;
        for (u32 i = threadIdx.x; i < n; i += AM_T) {
            const ulonglong2 x = e[2 * i], y = e[2 * i + 1];  // (hash, count), (h2 sum, representative)
            u32 b = (u32)((x.x * 0x9E3779B97F4A7C15ull) >> 52) & (AM_SLOTS - 1);
            bool done = false;
            for (u32 p = 0; p < 64 && !done; ++p, b = (b + 1) & (AM_SLOTS - 1)) {
                u64 cur = mh[b];
                if (cur == 0) {
                    const u64 old = atomicCAS((unsigned long long *)&mh[b], 0ull, (unsigned long long)x.x);
                    cur = old ? old : x.x;
                }
                if (cur == x.x) {
                    atomicAdd((unsigned long long *)&mc[b], (unsigned long long)x.y);
                    atomicAdd((unsigned long long *)&ms[b], (unsigned long long)y.x);
                    atomicMin((unsigned long long *)&mr[b], (unsigned long long)y.y);
                    done = true;
                }
            }
            bool isnew = false;
            u64 sl = 0;
            if (!done)
                sl = h_insert2<false>(atab, amask, x.x, x.y, y.y, y.x, alist, alist_cap, &ctr->a_claimed, ctr, OVF_A,
                                      &isnew);
            stage_new(isnew, sl, staged, &nst, AM_STAGE, alist, alist_cap, &ctr->a_claimed, ctr, OVF_A);
        }
    }
    __syncthreads();
    for (u32 i = threadIdx.x; i < AM_SLOTS; i += AM_T) {
        bool isnew = false;
        u64 sl = 0;
        if (mc[i])
            sl = h_insert2<false>(atab, amask, mh[i], mc[i], mr[i], ms[i], alist, alist_cap, &ctr->a_claimed, ctr, OVF_A,
                                  &isnew);
        stage_new(isnew, sl, staged, &nst, AM_STAGE, alist, alist_cap, &ctr->a_claimed, ctr, OVF_A);
    }
    __syncthreads();
    stage_flush(staged, &nst, AM_STAGE, &gbase, alist, alist_cap, &ctr->a_claimed, ctr, OVF_A);
}

// Every HBM artist entry: sum of h2 == count x h2(representative).
__global__ void k_artist_h2_check(const u64 *__restrict__ atab, const u32 *__restrict__ alist, u64 cap,
                                  const u64 *__restrict__ kh2, Counters *ctr) {
    const u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= cap || e >= ctr->a_claimed) return;
    const u64 *slot = atab + 4 * (u64)alist[e];
    if (slot[3] != slot[1] * kh2[slot[2]]) atomicAdd((unsigned long long *)&ctr->collision, 1ull);
}

// Workgroup representatives (and records inserted straight into HBM) against
// the HBM table's representative.
__global__ void k_artist_verify_reps(const u8 *__restrict__ arena, const u64 *__restrict__ key_off,
                                     const u32 *__restrict__ key_len, u64 *__restrict__ key_slot, u64 nrec,
                                     const u64 *__restrict__ atab, Counters *ctr) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nrec) return;
    const u64 k = key_slot[j];
    if (k == ~0ull || !(k & AK_VREP)) return;
    const u64 slot = k & AK_SLOTMASK;
    key_slot[j] = slot;
    const u64 rep = atab[4 * slot + 2];
    if (rep == j) return;
    if (!keys_equal(arena, key_off[j], key_len[j], key_off[rep], key_len[rep]))
        atomicAdd((unsigned long long *)&ctr->collision, 1ull);
}

__global__ void k_artist_verify(const u8 *__restrict__ arena, const u64 *__restrict__ key_off,
                                const u32 *__restrict__ key_len, const u64 *__restrict__ key_slot, u64 nrec,
                                const u64 *__restrict__ atab, Counters *ctr) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nrec || key_len[j] == 0 || key_slot[j] == ~0ull) return;
    const u64 rep = atab[4 * key_slot[j] + 2];
    if (rep == j) return;
    const u32 n = key_len[j];
    bool same = key_len[rep] == n;
    const u64 oa = key_off[j], ob = key_off[rep];
    if (same && n <= 32 && ((oa | ob) & 15) == 0) {  // keys in 16-byte aligned storage: vector compare
        const uint4 *pa = reinterpret_cast<const uint4 *>(arena + oa), *pb = reinterpret_cast<const uint4 *>(arena + ob);
        const uint4 a0 = pa[0], b0 = pb[0];
        const uint4 a1 = n > 16 ? pa[1] : make_uint4(0, 0, 0, 0), b1 = n > 16 ? pb[1] : make_uint4(0, 0, 0, 0);
        const u32 x[8] = {a0.x ^ b0.x, a0.y ^ b0.y, a0.z ^ b0.z, a0.w ^ b0.w,
                          a1.x ^ b1.x, a1.y ^ b1.y, a1.z ^ b1.z, a1.w ^ b1.w};
        u32 acc = 0;
#pragma unroll
        for (u32 k = 0; k < 8; ++k) {
            const u32 lo = 4 * k;
            const u32 keep = n <= lo ? 0u : (n >= lo + 4 ? 4u : n - lo);
            acc |= x[k] & (keep == 4 ? 0xFFFFFFFFu : ((1u << (8 * keep)) - 1u));
        }
        same = acc == 0;
    } else {
        const u8 *a = arena + oa, *b = arena + ob;
        for (u32 i = 0; same && i < n; ++i) same = a[i] == b[i];
    }
    if (!same) atomicAdd((unsigned long long *)&ctr->collision, 1ull);
}

// ---------------------------------------------------------------------------
// words > 16 bytes (one occurrence per thread: 1024-thread workgroups of 4
// occurrences per thread with the new slots listed once per workgroup were
// slower, 1.48 -> 1.75 ms for configs[4] and 0.04 -> 0.44 ms for configs[2]:
// the list claims were not what bound it, the inserts in flight are)
__device__ __forceinline__ u64 long_hash(const u8 *__restrict__ buf, u64 seg_end, const u8 *__restrict__ extra,
                                         u64 extra_len, u64 p, u32 &len) {
    const u8 *src = tok_at(buf, extra, p);
    const u64 lim = (p & MSA_POS_EXTRA) ? extra_len - (p & ~MSA_POS_EXTRA) : seg_end - p;
    // the token's first 48 bytes from 13 dword loads (the buffers are padded
    // past their end), aligned in registers: its length and its hash
    // (bytes_hash's 8-byte groups) without a byte loop through memory
    const u32 *wp = reinterpret_cast<const u32 *>(reinterpret_cast<uintptr_t>(src) & ~(uintptr_t)3);
    const u32 sh = (u32)(reinterpret_cast<uintptr_t>(src) & 3);
    u32 w[13], a[12];
#pragma unroll
    for (int k = 0; k < 13; ++k) w[k] = wp[k];
#pragma unroll
    for (int k = 0; k < 12; ++k) a[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
    len = 48;
#pragma unroll
    for (int k = 47; k >= 0; --k)
        if (!c_tok((a[k >> 2] >> (8 * (k & 3))) & 0xFFu)) len = (u32)k;
    if ((u64)len > lim) len = (u32)lim;
    u64 h;
    if (len < 48) {
        h = 0x243F6A8885A308D3ULL ^ ((u64)len * 0x9E3779B97F4A7C15ULL);
        u64 acc = 0;
#pragma unroll
        for (u32 g = 0; g < 6; ++g) {
            u64 x = ((u64)a[2 * g + 1] << 32) | a[2 * g];
            x |= (x >> 1) & 0x2020202020202020ull;  // lower-case (token bytes: letters, digits, ')
            if (8 * g + 8 <= len) {
                h = fmix64(h ^ x) * 0x9E3779B97F4A7C15ULL;
            } else if (8 * g < len) {
                acc = x & ((1ull << (8 * (len - 8 * g))) - 1ull);
            }
        }
        h = fmix64(h ^ acc ^ ((u64)(len & 7u) << 59));
    } else {  // a longer token: the byte loops
        u64 L = 48;
        while (L < lim && c_tok(src[L])) ++L;
        len = (u32)L;
        h = bytes_hash(src, L, 1);
    }
    return h;
}
__global__ void k_long_insert(const u8 *__restrict__ buf, u64 seg_end, const u8 *__restrict__ extra, u64 extra_len,
                              const u64 *__restrict__ l_pos, u64 n, u32 *__restrict__ l_len, u64 *__restrict__ l_slot,
                              u64 *ltab, u64 lmask, u32 *llist, u64 llist_cap, Counters *ctr) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (l_pos[i] == ~0ull) {  // a slot of a token-pass range left unused (msa_k3.hip LP_NONE)
        l_len[i] = 0;
        l_slot[i] = ~0ull;
        return;
    }
    u32 len;
    const u64 h = long_hash(buf, seg_end, extra, extra_len, l_pos[i], len);
    l_len[i] = len;
    l_slot[i] = h_insert<true, true>(ltab, lmask, h, 1, i, llist, llist_cap, &ctr->l_claimed, ctr, OVF_LT);
}

__device__ __forceinline__ u64 lower8x(u64 x) {  // 'A'..'Z' -> 'a'..'z' in each byte (bytes >= 0x80 kept)
    const u64 h = 0x8080808080808080ull, o = 0x0101010101010101ull;
    const u64 t = x & ~h;
    const u64 ge = (t + (0x80 - 0x41) * o) & h, gt = (t + (0x80 - 0x5B) * o) & h;
    return x | ((ge & ~gt & ~x) >> 2);
}
__device__ __forceinline__ u32 lower1(u32 c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

__global__ void k_long_verify(const u8 *__restrict__ buf, const u8 *__restrict__ extra, const u64 *__restrict__ l_pos,
                              const u32 *__restrict__ l_len, const u64 *__restrict__ l_slot, u64 n,
                              const u64 *__restrict__ ltab, Counters *ctr) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || l_slot[i] == ~0ull) return;
    const u64 rep = ltab[4 * l_slot[i] + 2];
    if (rep == i) return;
    const u32 len = l_len[i];
    bool same = l_len[rep] == len;
    // 16 bytes of each at a time (dword-aligned bases, padded inputs), lower-cased in registers
    const u64 pa = l_pos[i], pb = l_pos[rep];
    const u8 *ba = (pa & MSA_POS_EXTRA) ? extra : buf, *bb = (pb & MSA_POS_EXTRA) ? extra : buf;
    const u64 oa = pa & ~MSA_POS_EXTRA, ob = pb & ~MSA_POS_EXTRA;
    for (u32 k = 0; same && k < len; k += 16) {
        const uint4 x = load16u(ba, oa + k), y = load16u(bb, ob + k);
        u64 x0 = ((u64)x.y << 32) | x.x, x1 = ((u64)x.w << 32) | x.z;
        u64 y0 = ((u64)y.y << 32) | y.x, y1 = ((u64)y.w << 32) | y.z;
        const u32 r = len - k;  // bytes of this piece that belong to the words
        const u64 m0 = r >= 8 ? ~0ull : bits_below(8 * r), m1 = r >= 16 ? ~0ull : (r > 8 ? bits_below(8 * (r - 8)) : 0ull);
        same = ((lower8x(x0) ^ lower8x(y0)) & m0) == 0 && ((lower8x(x1) ^ lower8x(y1)) & m1) == 0;
    }
    if (!same) atomicAdd((unsigned long long *)&ctr->collision, 1ull);
}

// ---------------------------------------------------------------------------
// Ranking entries.  Sort key = (K2 = ~count, K1 = key bytes 0..7 big-endian,
// K0 = key bytes 8..15 big-endian); ascending == entry_compare_desc for all
// keys that differ within their first 16 bytes (zero padding sorts first,
// exactly like strcmp's terminator).  ref = (kind << 60) | index (KIND_*:
// msa_internal.h).

__device__ __forceinline__ void be16(const u8 *p, u64 n, int lower, u64 *hi, u64 *lo) {
    u64 h = 0, l = 0;
    for (u64 i = 0; i < 16; ++i) {
        u32 c = i < n ? p[i] : 0;
        if (lower) c = lower1(c);
        if (i < 8) h = (h << 8) | c;
        else l = (l << 8) | c;
    }
    *hi = h;
    *lo = l;
}

// be16 from one unaligned 16-byte load (base dword-aligned, padded past the
// key): a byte load per key byte left each long word's lane waiting on 16
// loads in turn
__device__ __forceinline__ void be16w(const u8 *base, u64 off, u64 n, int lower, u64 *hi, u64 *lo) {
    const uint4 v = load16u(base, off);
    u64 a = ((u64)v.y << 32) | v.x, b = ((u64)v.w << 32) | v.z;  // bytes 0..7, 8..15 (little-endian)
    if (n < 16) {
        if (n <= 8) {
            a &= bits_below(8 * (u32)n);
            b = 0;
        } else {
            b &= bits_below(8 * (u32)(n - 8));
        }
    }
    if (lower) {
        a = lower8x(a);
        b = lower8x(b);
    }
    *hi = __builtin_bswap64(a);
    *lo = __builtin_bswap64(b);
}

// Dense list of the claimed slots of an S or M word table.  The main scan
// inserts without appending to the list (every new key would serialise on one
// claim counter); this pass reads the keys once (16 slots per thread,
// coalesced) and adds to the claim counter once per workgroup.
__global__ __launch_bounds__(256) void k_list_build(const u64 *__restrict__ tab, u64 nslots, u32 stride,
                                                    u32 *__restrict__ list, u64 cap, u64 *claimed, Counters *ctr,
                                                    u64 ovf_bit) {
    __shared__ u32 wsum[4];
    __shared__ u64 gbase;
    const u32 t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const u64 s0 = (u64)blockIdx.x * 4096;
    u32 used = 0;
#pragma unroll
    for (u32 k = 0; k < 16; ++k) {
        const u64 sl = s0 + k * 256 + t;
        if (sl < nslots && tab[sl * stride] != 0) used |= 1u << k;
    }
    u32 wt;
    const u32 pre = wave_prefix<5>((u32)__popc(used), wt);
    if (lane == 0) wsum[w] = wt;
    __syncthreads();
    if (t == 0) {
        const u32 all = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        gbase = all ? atomicAdd((unsigned long long *)claimed, (unsigned long long)all) : 0ull;
    }
    __syncthreads();
    u64 i = gbase + pre;
    for (u32 v = 0; v < w; ++v) i += wsum[v];
    for (u32 k = 0; k < 16; ++k) {
        if (!((used >> k) & 1u)) continue;
        if (i < cap) list[i] = (u32)(s0 + k * 256 + t);
        else atomicOr((unsigned long long *)&ctr->overflow, (unsigned long long)ovf_bit);
        ++i;
    }
}

__global__ __launch_bounds__(256) void k_word_entries(EntryArgs a) {
    const u64 n = a.ns + a.nm + a.nl;
    // the key planes' OR / AND (a.vary): per thread over its grid-stride
    // entries, then per workgroup, one atomic per plane and workgroup (one per
    // wave on the same six words serialised at the L2: 47 ms at 50 M entries)
    u64 vo[3] = {0, 0, 0}, va[3] = {~0ull, ~0ull, ~0ull};
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        u64 c, hi, lo, ref;
        if (i < a.ns) {
            const u64 slot = a.s_list[i];
            const u64 w0 = a.s_tab[2 * slot], key = w0 & TAB_KEY7;
            c = a.s_tab[2 * slot + 1] + tab_gather8(w0);
            hi = __builtin_bswap64(key);
            lo = 0;
            ref = ((u64)KIND_S << 60) | slot;
        } else if (i < a.ns + a.nm) {
            const u64 slot = a.m_list[i - a.ns];
            const u64 w0 = a.m_tab[4 * slot];
            hi = __builtin_bswap64(w0 & TAB_KEY7);
            lo = __builtin_bswap64(a.m_tab[4 * slot + 1]);
            c = a.m_tab[4 * slot + 2] + tab_gather8(w0);
            ref = ((u64)KIND_M << 60) | slot;
        } else {
            const u64 slot = a.l_list[i - a.ns - a.nm];
            c = a.l_tab[4 * slot + 1] + 1;  // h_insert IMPL1: the first occurrence is implicit
            const u64 rep = a.l_tab[4 * slot + 2];
            const u64 lp = a.l_pos[rep];
            be16w((lp & MSA_POS_EXTRA) ? a.extra : a.buf, lp & ~MSA_POS_EXTRA, a.l_len[rep], 1, &hi, &lo);
            ref = ((u64)KIND_L << 60) | rep;
        }
        a.K2[i] = ~c;
        a.K1[i] = hi;
        a.K0[i] = lo;
        a.val[i] = (u32)(a.vbase + i);
        a.ref[i] = ref;
        if (a.cnt) a.cnt[i] = c;
        vo[0] |= lo; vo[1] |= hi; vo[2] |= ~c;
        va[0] &= lo; va[1] &= hi; va[2] &= ~c;
    }
    if (!a.vary) return;
    __shared__ u64 r[4][6];
#pragma unroll
    for (int w = 0; w < 3; ++w) {
        for (int o = 32; o > 0; o >>= 1) {
            vo[w] |= __shfl_xor(vo[w], o);
            va[w] &= __shfl_xor(va[w], o);
        }
    }
    const u32 wv = threadIdx.x >> 6;
    if (lane_id() == 0)
        for (int w = 0; w < 3; ++w) { r[wv][w] = vo[w]; r[wv][3 + w] = va[w]; }
    __syncthreads();
    if (threadIdx.x < 6) {
        const u32 k = threadIdx.x;
        u64 x = r[0][k];
        for (u32 q = 1; q < blockDim.x / 64; ++q) x = k < 3 ? (x | r[q][k]) : (x & r[q][k]);
        if (k < 3) atomicOr((unsigned long long *)&a.vary[k], (unsigned long long)x);
        else atomicAnd((unsigned long long *)&a.vary[k], (unsigned long long)x);
    }
}

__global__ void k_artist_entries(const u64 *__restrict__ atab, const u32 *__restrict__ alist, u64 n,
                                 const u8 *__restrict__ arena, const u64 *__restrict__ key_off,
                                 const u32 *__restrict__ key_len, u64 *K2, u64 *K1, u64 *K0, u32 *val, u64 *ref,
                                 u64 *cnt) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 slot = alist[i];
    const u64 c = atab[4 * slot + 1];
    const u64 rep = atab[4 * slot + 2];
    u64 hi, lo;
    be16w(arena, key_off[rep], key_len[rep], 0, &hi, &lo);
    K2[i] = ~c;
    K1[i] = hi;
    K0[i] = lo;
    val[i] = (u32)i;
    ref[i] = ((u64)KIND_A << 60) | rep;
    cnt[i] = c;
}

// ---------------------------------------------------------------------------
// Sort of (K2, K1, K0) ascending with u32 values.  Tables hold 10^3..10^6
// distinct keys, so the sort is launch- and latency-bound: 1024-element tiles
// are bitonic-sorted in LDS (one launch), then log2(n / 1024) merge passes,
// each element finding its output position by one binary search in the
// partner run (A-elements count partner keys <, B-elements <=, so equal keys
// keep A before B and every position is written once).  Equal keys (long
// words sharing 16 bytes and a count) are ordered by k_tie_fixup.
#define TS_T 512
#define TS_N 1024
__device__ __forceinline__ bool key_lt(u64 a2, u64 a1, u64 a0, u64 b2, u64 b1, u64 b0) {
    return a2 != b2 ? a2 < b2 : (a1 != b1 ? a1 < b1 : a0 < b0);
}

__global__ __launch_bounds__(TS_T) void k_tile_sort(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                    const u64 *__restrict__ K0, const u32 *__restrict__ V, u64 n,
                                                    u64 *__restrict__ O2, u64 *__restrict__ O1,
                                                    u64 *__restrict__ O0, u32 *__restrict__ OV) {
    __shared__ u64 s2[TS_N], s1[TS_N], s0[TS_N];
    __shared__ u32 sv[TS_N];
    const u64 base = (u64)blockIdx.x * TS_N;
    const u32 t = threadIdx.x;
    for (u32 i = t; i < TS_N; i += TS_T) {
        const u64 g = base + i;
        const bool ok = g < n;  // padding sorts last
        s2[i] = ok ? K2[g] : ~0ull;
        s1[i] = ok ? K1[g] : ~0ull;
        s0[i] = ok ? K0[g] : ~0ull;
        sv[i] = ok ? V[g] : ~0u;
    }
    __syncthreads();
    for (u32 k = 2; k <= TS_N; k <<= 1) {
        for (u32 j = k >> 1; j > 0; j >>= 1) {
            const u32 i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), l = i | j;
            const u64 a2 = s2[i], a1 = s1[i], a0 = s0[i], b2 = s2[l], b1 = s1[l], b0 = s0[l];
            const bool asc = (i & k) == 0;
            if (key_lt(b2, b1, b0, a2, a1, a0) == asc) {
                s2[i] = b2; s1[i] = b1; s0[i] = b0;
                s2[l] = a2; s1[l] = a1; s0[l] = a0;
                const u32 x = sv[i];
                sv[i] = sv[l];
                sv[l] = x;
            }
            __syncthreads();
        }
    }
    for (u32 i = t; i < TS_N; i += TS_T) {
        const u64 g = base + i;
        if (g < n) {
            O2[g] = s2[i];
            O1[g] = s1[i];
            O0[g] = s0[i];
            OV[g] = sv[i];
        }
    }
}

__global__ __launch_bounds__(256) void k_merge_pass(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                    const u64 *__restrict__ K0, const u32 *__restrict__ V, u64 n,
                                                    u64 width, u64 *__restrict__ O2, u64 *__restrict__ O1,
                                                    u64 *__restrict__ O0, u32 *__restrict__ OV) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 run = i / width, base = (run & ~1ull) * width;
    const bool left = (run & 1ull) == 0;
    const u64 a2 = K2[i], a1 = K1[i], a0 = K0[i];
    const u64 lo = left ? min(base + width, n) : base, hi = left ? min(base + 2 * width, n) : base + width;
    u64 L = lo, H = hi;
    while (L < H) {
        const u64 m = (L + H) >> 1;
        const u64 b2 = K2[m], b1 = K1[m], b0 = K0[m];
        const bool before = left ? key_lt(b2, b1, b0, a2, a1, a0) : !key_lt(a2, a1, a0, b2, b1, b0);
        if (before) L = m + 1;
        else H = m;
    }
    const u64 out = base + (i - (left ? base : base + width)) + (L - lo);
    O2[out] = a2;
    O1[out] = a1;
    O0[out] = a0;
    OV[out] = V[i];
}

// ---------------------------------------------------------------------------
// Exact tie fix-up: runs of equal (K2, K1, K0) (keys sharing 16 leading bytes
// and a count) are re-ordered by full strcmp.  Run sizes are tiny.
__device__ __forceinline__ void key_bytes(u64 ref, u64 k1, u64 k0, const u8 *buf, const u8 *extra, const u64 *l_pos,
                                          const u32 *l_len, const u8 *arena, const u64 *key_off,
                                          const u32 *key_len, const u8 **p, u64 *n, int *lower) {
    const u32 kind = (u32)(ref >> 60);
    const u64 idx = ref & ((1ull << 60) - 1);
    *lower = 0;
    if (kind == KIND_L) { *p = tok_at(buf, extra, l_pos[idx]); *n = l_len[idx]; *lower = 1; }
    else if (kind == KIND_A) { *p = arena + key_off[idx]; *n = key_len[idx]; }
    else { *p = nullptr; *n = 0; }
}

__device__ int full_cmp(u64 refa, u64 refb, u64 k1, u64 k0, const u8 *buf, const u8 *extra, const u64 *l_pos,
                        const u32 *l_len,
                        const u8 *arena, const u64 *key_off, const u32 *key_len) {
    const u8 *pa, *pb;
    u64 na, nb;
    int la, lb;
    key_bytes(refa, k1, k0, buf, extra, l_pos, l_len, arena, key_off, key_len, &pa, &na, &la);
    key_bytes(refb, k1, k0, buf, extra, l_pos, l_len, arena, key_off, key_len, &pb, &nb, &lb);
    // S/M keys are fully described by (k1, k0): 16 bytes, zero padded
    u8 tmp[16];
    for (int i = 0; i < 8; ++i) { tmp[i] = (u8)(k1 >> (56 - 8 * i)); tmp[8 + i] = (u8)(k0 >> (56 - 8 * i)); }
    if (!pa) { pa = tmp; na = 0; while (na < 16 && tmp[na]) ++na; la = 0; }
    if (!pb) { pb = tmp; nb = 0; while (nb < 16 && tmp[nb]) ++nb; lb = 0; }
    const u64 m = na < nb ? na : nb;
    // tied entries agree in (k1, k0) = their first 16 key bytes, zero padded;
    // key bytes are never 0, so the first min(16, na, nb) bytes are equal
    for (u64 i = m < 16 ? m : 16; i < m; ++i) {
        u32 x = pa[i], y = pb[i];
        if (la) x = lower1(x);
        if (lb) y = lower1(y);
        if (x != y) return x < y ? -1 : 1;
    }
    return na < nb ? -1 : (na > nb ? 1 : 0);
}

__global__ void k_tie_fixup(const u64 *__restrict__ K2, const u64 *__restrict__ K1, const u64 *__restrict__ K0,
                            const u32 *__restrict__ V, u64 n, const u64 *__restrict__ ref, const u8 *buf,
                            const u8 *extra, const u64 *l_pos, const u32 *l_len, const u8 *arena, const u64 *key_off,
                            const u32 *key_len, u32 *__restrict__ out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // K0 is required (msa_launch_fixup refuses null): full_cmp takes tied
    // entries as equal in their first 16 key bytes (K1, K0)
    const u64 a2 = K2[i], a1 = K1[i], a0 = K0[i];
    const bool eq_prev = i > 0 && K2[i - 1] == a2 && K1[i - 1] == a1 && K0[i - 1] == a0;
    const bool eq_next = i + 1 < n && K2[i + 1] == a2 && K1[i + 1] == a1 && K0[i + 1] == a0;
    if (!eq_prev && !eq_next) { out[i] = V[i]; return; }
    u64 s = i, e = i + 1;
    while (s > 0 && K2[s - 1] == a2 && K1[s - 1] == a1 && K0[s - 1] == a0) --s;
    while (e < n && K2[e] == a2 && K1[e] == a1 && K0[e] == a0) ++e;
    const u64 me = ref[V[i]];
    u64 rank = 0;
    for (u64 j = s; j < e; ++j) {
        if (j == i) continue;
        const int c = full_cmp(ref[V[j]], me, a1, a0, buf, extra, l_pos, l_len, arena, key_off, key_len);
        if (c < 0 || (c == 0 && j < i)) ++rank;
    }
    out[s + rank] = V[i];
}

// ---------------------------------------------------------------------------
// Tie refinement (radix path): instead of comparing every pair of a tie run,
// the tied entries are sorted again by (run, next 16 key bytes), round after
// round, until no two adjacent keys are equal.  A run of thousands of artists
// sharing 16 bytes and a count (configs[4]) costs one small radix sort, not
// run^2 string compares.
// Tie runs by stream compaction: a block of TB_N consecutive entries counts
// its run heads and tied entries (k_tie_count), the block counts are scanned,
// and k_tie_build recomputes the flags, ranks them within the block (wave
// ballots) and writes only the tied entries.  (Per-entry head / tie / run-id /
// position arrays and their two full scans had cost ~1.3 ms for configs[4]'s
// 50 M words, to find a few hundred thousand tied entries.)
#define TB_T 256
#define TB_PER 4
#define TB_N (TB_T * TB_PER)
struct TieFlags {
    bool head, tie;
};
// K0 null: the sort covered K2 and K1 only (K0's bytes are the first refinement round's)
__device__ __forceinline__ TieFlags tie_flags(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                              const u64 *__restrict__ K0, u64 n, u64 i) {
    // K1 == K2: one plane (the composite key's sort)
    const bool k1s = K1 != K2;
    const u64 a2 = K2[i], a1 = k1s ? K1[i] : 0, a0 = K0 ? K0[i] : 0;
    const bool eq_prev = i > 0 && K2[i - 1] == a2 && (!k1s || K1[i - 1] == a1) && (!K0 || K0[i - 1] == a0);
    const bool eq_next = i + 1 < n && K2[i + 1] == a2 && (!k1s || K1[i + 1] == a1) && (!K0 || K0[i + 1] == a0);
    return TieFlags{!eq_prev, eq_prev || eq_next};
}
// Runs of at most TIE_SEG entries are ordered by k_tie_seg instead of the
// radix sort; k_tie_count flags a longer one (its head equal to the entry
// TIE_SEG places on) in *big.
#define TIE_SEG 64
__device__ __forceinline__ bool tie_same(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                         const u64 *__restrict__ K0, u64 i, u64 j) {
    return K2[i] == K2[j] && (K1 == K2 || K1[i] == K1[j]) && (!K0 || K0[i] == K0[j]);
}
// entry (row k, thread t) of block b is entry b * TB_N + k * TB_T + t
__global__ __launch_bounds__(TB_T) void k_tie_count(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                    const u64 *__restrict__ K0, u64 n, u64 *__restrict__ bh,
                                                    u64 *__restrict__ bt, u64 *__restrict__ big) {
    __shared__ u32 ws[2][TB_T / 64];
    const u32 t = threadIdx.x;
    u32 h = 0, q = 0;
#pragma unroll
    for (u32 k = 0; k < TB_PER; ++k) {
        const u64 i = (u64)blockIdx.x * TB_N + k * TB_T + t;
        if (i < n) {
            const TieFlags f = tie_flags(K2, K1, K0, n, i);
            h += f.head;
            q += f.tie;
            if (f.head && f.tie && i + TIE_SEG < n && tie_same(K2, K1, K0, i, i + TIE_SEG)) big[0] = 1;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        h += __shfl_xor(h, o);
        q += __shfl_xor(q, o);
    }
    if (lane_id() == 0) {
        ws[0][t >> 6] = h;
        ws[1][t >> 6] = q;
    }
    __syncthreads();
    if (t == 0) {
        u32 H = 0, Q = 0;
        for (u32 w = 0; w < TB_T / 64; ++w) {
            H += ws[0][w];
            Q += ws[1][w];
        }
        bh[blockIdx.x] = H;
        bt[blockIdx.x] = Q;
    }
}

// key bytes [skip, skip + 16) of an entry as two big-endian words (zero past its end)
__device__ __forceinline__ void key16_round(u64 refv, u32 skip, const u8 *buf, const u8 *extra, const u64 *l_pos,
                                            const u32 *l_len, const u8 *arena, const u64 *key_off,
                                            const u32 *key_len, u64 *hi, u64 *lo) {
    const u8 *p;
    u64 n;
    int lower;
    key_bytes(refv, 0, 0, buf, extra, l_pos, l_len, arena, key_off, key_len, &p, &n, &lower);
    if (!p || n <= skip) {  // the key ends before (S/M keys: within their first 16 bytes)
        *hi = 0;
        *lo = 0;
        return;
    }
    be16(p + skip, n - skip, lower, hi, lo);
}

// hoff / toff: exclusive scans of the blocks' head / tie counts.  Tied entry
// i of the current level (value Vc[i], order position Pc ? Pc[i] : i) goes to
// slot j of the next level's subset, keyed by (its run's inclusive head count,
// key bytes [skip, skip + 16)).
__global__ __launch_bounds__(TB_T) void k_tie_build(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                    const u64 *__restrict__ K0, u64 mc, const u64 *__restrict__ hoff,
                                                    const u64 *__restrict__ toff, const u32 *__restrict__ Vc,
                                                    const u64 *__restrict__ Pc, u32 skip,
                                                    const u64 *__restrict__ K1u, const u64 *__restrict__ K0u,
                                                    const u64 *__restrict__ ref, const u8 *buf, const u8 *extra,
                                                    const u64 *l_pos, const u32 *l_len, const u8 *arena,
                                                    const u64 *key_off, const u32 *key_len, u64 *__restrict__ K2n,
                                                    u64 *__restrict__ K1n, u64 *__restrict__ K0n, u32 *__restrict__ Vid,
                                                    u32 *__restrict__ Vn, u64 *__restrict__ Pn) {
    __shared__ u32 ws[2][TB_PER][TB_T / 64];
    const u32 t = threadIdx.x, lane = lane_id(), w = t >> 6;
    TieFlags f[TB_PER];
    u32 hp[TB_PER], tp[TB_PER];
#pragma unroll
    for (u32 k = 0; k < TB_PER; ++k) {
        const u64 i = (u64)blockIdx.x * TB_N + k * TB_T + t;
        f[k] = i < mc ? tie_flags(K2, K1, K0, mc, i) : TieFlags{false, false};
        const u64 H = __ballot(f[k].head), Q = __ballot(f[k].tie);
        hp[k] = mbcnt(H);
        tp[k] = mbcnt(Q);
        if (lane == 0) {
            ws[0][k][w] = (u32)__popcll(H);
            ws[1][k][w] = (u32)__popcll(Q);
        }
    }
    __syncthreads();
    bool any = false;
#pragma unroll
    for (u32 k = 0; k < TB_PER; ++k) any |= f[k].tie;
    if (!any) return;
    // exclusive offsets of (row k, wave w) within the block: earlier rows, then earlier waves of row k
    u32 hb = 0, tb = 0;
#pragma unroll
    for (u32 k = 0; k < TB_PER; ++k) {
        u32 hw = hb, tw = tb;
        for (u32 v = 0; v < w; ++v) {
            hw += ws[0][k][v];
            tw += ws[1][k][v];
        }
        if (f[k].tie) {
            const u64 i = (u64)blockIdx.x * TB_N + k * TB_T + t;
            const u64 j = toff[blockIdx.x] + tw + tp[k];
            const u32 e = Vc[i];
            u64 hi, lo;
            if (skip <= 8) {  // after a sort of fewer than 16 key bytes: bytes skip .. 15 are in K1/K0 (S/M keys
                              // have no byte source), bytes 16 .. from the key's bytes
                u64 h2, l2;
                key16_round(ref[e], 16, buf, extra, l_pos, l_len, arena, key_off, key_len, &h2, &l2);
                const u64 k0 = K0u[e];
                if (skip == 8) {
                    hi = k0;
                    lo = h2;
                } else {  // the composite key's sort (skip 6 or 7: msa_radix_sort_comp)
                    const u32 sb = 8 * skip;
                    const u64 k1 = K1u[e];
                    hi = (k1 << sb) | (k0 >> (64 - sb));
                    lo = (k0 << sb) | (h2 >> (64 - sb));
                }
            } else {
                key16_round(ref[e], skip, buf, extra, l_pos, l_len, arena, key_off, key_len, &hi, &lo);
            }
            K2n[j] = hoff[blockIdx.x] + hw + hp[k] + (f[k].head ? 1 : 0);  // the same for every entry of a run
            K1n[j] = hi;
            K0n[j] = lo;
            Vid[j] = (u32)j;
            Vn[j] = e;
            Pn[j] = Pc ? Pc[i] : i;
        }
        for (u32 v = 0; v < TB_T / 64; ++v) {
            hb += ws[0][k][v];
            tb += ws[1][k][v];
        }
    }
}

// the subset sorted (perm): its entries take the same order positions, in order
// (and the sorted K0 plane at those positions: after a K2/K1-only sort the
// tied entries' K0 differ, and the key blob reads K0 in rank order)
__global__ void k_tie_apply(const u32 *__restrict__ perm, const u32 *__restrict__ Vn, const u64 *__restrict__ Pn,
                            u64 m, u32 *__restrict__ order, u32 *__restrict__ Vc, u64 *__restrict__ Pc,
                            const u64 *__restrict__ K1u, const u64 *__restrict__ K0u, u64 *__restrict__ ks1,
                            u64 *__restrict__ ks0) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const u32 e = Vn[perm[j]];
    order[Pn[j]] = e;
    if (ks0) ks0[Pn[j]] = K0u[e];
    if (ks1) ks1[Pn[j]] = K1u[e];  // the composite key's sort: tied entries share only bytes 0 .. skip-1
    Vc[j] = e;
    Pc[j] = Pn[j];
}

// A tie round whose runs all hold <= TIE_SEG entries (k_tie_count's flag
// clear): each entry of the subset counts the members of its run -- contiguous,
// equal run id K2n -- that the radix sort would put before it ((K1n, K0n),
// then subset position: the sort is stable) and writes itself and its keys
// at that place of set 1.  Same output as msa_radix_sort, without its ~20
// launch-bound passes and its host round trip.
__global__ void k_tie_seg(const u64 *__restrict__ K2n, const u64 *__restrict__ K1n, const u64 *__restrict__ K0n,
                          const u32 *__restrict__ Vid, u64 m, u64 *__restrict__ O2, u64 *__restrict__ O1,
                          u64 *__restrict__ O0, u32 *__restrict__ OV) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const u64 r = K2n[j], a1 = K1n[j], a0 = K0n[j];
    u64 s = j, e = j + 1;
    while (s > 0 && K2n[s - 1] == r) --s;
    while (e < m && K2n[e] == r) ++e;
    u64 rank = 0;
    for (u64 i = s; i < e; ++i) {
        const u64 b1 = K1n[i], b0 = K0n[i];
        rank += b1 < a1 || (b1 == a1 && (b0 < a0 || (b0 == a0 && i < j)));
    }
    const u64 o = s + rank;
    O2[o] = r;
    O1[o] = a1;
    O0[o] = a0;
    OV[o] = Vid[j];
}

// ---------------------------------------------------------------------------
// Ranked key blob: lengths, then bytes (in rank order).
__device__ __forceinline__ u64 entry_key_len(u64 ref, u64 k1, u64 k0, const u32 *l_len, const u32 *key_len) {
    const u32 kind = (u32)(ref >> 60);
    const u64 idx = ref & ((1ull << 60) - 1);
    if (kind == KIND_L) return l_len[idx];
    if (kind == KIND_A) return key_len[idx];
    // S/M key bytes are nonzero and big-endian here, zero padded: the length
    // is the nonzero bytes above the trailing zero bytes
    const u64 n1 = k1 ? 8 - ((u64)__builtin_ctzll(k1) >> 3) : 0;
    if (n1 < 8) return n1;
    return 8 + (k0 ? 8 - ((u64)__builtin_ctzll(k0) >> 3) : 0);
}

// SortedKeys: the sorted (K2, K1, K0) planes, position i = rank i (entries tied
// on all 24 bytes share them, so the tie order does not matter); entries below
// `lthr` are S/M words whose K1/K0 are the whole key.  Those need no random
// reads of ref/K/cnt: only the long words' and artists' keys do.
struct SortedKeys {
    const u64 *K2, *K1, *K0;
    u64 lthr;
};

__global__ void k_blob_len(const u32 *__restrict__ order, u64 n, const u64 *__restrict__ ref,
                           const u64 *__restrict__ K1u, const u64 *__restrict__ K0u, const u32 *l_len,
                           const u32 *key_len, SortedKeys sk, u64 *__restrict__ len) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 e = order[i];
    len[i] = e < sk.lthr ? entry_key_len((u64)KIND_S << 60, sk.K1[i], sk.K0[i], l_len, key_len)
                         : entry_key_len(ref[e], K1u[e], K0u[e], l_len, key_len);
}

// one entry's key bytes to dst (rank i, entry e = order[i])
__device__ __forceinline__ void blob_key_bytes(u64 i, u32 e, const u64 *__restrict__ ref, const u64 *__restrict__ K1u,
                                               const u64 *__restrict__ K0u, const u8 *buf, const u8 *extra,
                                               const u64 *l_pos, const u32 *l_len, const u8 *arena,
                                               const u64 *key_off, const u32 *key_len, const SortedKeys &sk, u8 *dst) {
    if (e < sk.lthr) {  // S/M word: the key is the sorted K1/K0
        const u64 k1 = sk.K1[i], k0 = sk.K0[i];
        for (int k = 0; k < 16; ++k) {
            const u8 b = (u8)((k < 8 ? k1 : k0) >> (56 - 8 * (k & 7)));
            if (!b) break;
            dst[k] = b;
        }
        return;
    }
    const u64 r = ref[e];
    const u32 kind = (u32)(r >> 60);
    const u64 idx = r & ((1ull << 60) - 1);
    if (kind == KIND_L || kind == KIND_A) {
        // 16-byte unaligned loads, two in flight (a byte load per key byte
        // left each long word's lane waiting on ~20 loads in turn); the input,
        // the side buffer and the key arena are padded past their last key
        const bool low = kind == KIND_L;
        const u64 lp = low ? l_pos[idx] : 0;
        // an aligned base and a byte offset (load16u's dword loads stay aligned)
        const u8 *base = low ? ((lp & MSA_POS_EXTRA) ? extra : buf) : arena;
        const u64 o = low ? (lp & ~MSA_POS_EXTRA) : key_off[idx];
        const u32 L = low ? l_len[idx] : key_len[idx];
        for (u32 k = 0; k < L; k += 32) {
            const uint4 a = load16u(base, o + k), b = load16u(base, o + k + 16);
            const u32 w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            const u32 m = min(32u, L - k);
#pragma unroll
            for (u32 q = 0; q < 32; ++q) {
                if (q >= m) break;
                const u32 ch = (w[q >> 2] >> (8 * (q & 3))) & 0xFFu;
                dst[k + q] = (u8)(low ? lower1(ch) : ch);
            }
        }
    } else {
        const u64 k1 = K1u[e], k0 = K0u[e];
        for (int k = 0; k < 16; ++k) {
            const u8 b = (u8)((k < 8 ? k1 : k0) >> (56 - 8 * (k & 7)));
            if (!b) break;
            dst[k] = b;
        }
    }
}

// A workgroup writes the keys of BW_T consecutive ranks: their bytes are one
// contiguous range of the blob, composed in LDS at the blob's 16-byte phase
// and written as whole 16-byte chunks (the range's first and last chunk byte
// by byte: they share bytes with the neighbouring workgroups).  Byte stores
// of every key straight to the blob (one lane per key, 1-16 byte stores at
// scattered offsets) had cost 1.6 ms for configs[4]'s 50 M words.  A range
// longer than the staging buffer (long keys), or past the blob's capacity,
// is written key by key.
#define BW_T 256
#define BW_LDS 16384
__global__ __launch_bounds__(BW_T) void k_blob_write(const u32 *__restrict__ order, u64 n, const u64 *__restrict__ ref,
                                                     const u64 *__restrict__ K1u, const u64 *__restrict__ K0u,
                                                     const u64 *__restrict__ cnt, const u8 *buf, const u8 *extra,
                                                     const u64 *l_pos, const u32 *l_len, const u8 *arena,
                                                     const u64 *key_off, const u32 *key_len,
                                                     const u64 *__restrict__ off, const u64 *__restrict__ len,
                                                     SortedKeys sk, u8 *__restrict__ blob,
                                                     u64 *__restrict__ counts_out, u64 blob_cap) {
    __shared__ __attribute__((aligned(16))) u8 stage[BW_LDS + 32];
    const u32 t = threadIdx.x;
    const u64 i0 = (u64)blockIdx.x * BW_T, i = i0 + t;
    const u64 last = min(n, i0 + BW_T) - 1;
    const bool live = i < n;
    const u32 e = live ? order[i] : 0u;
    if (live) counts_out[i] = sk.K2 ? ~sk.K2[i] : cnt[e];
    const u64 base = off[i0], end = off[last] + len[last];
    const u32 ph = (u32)(base & 15u);
    if (end - base > BW_LDS || end > blob_cap) {  // key by key (uniform per workgroup)
        // the blob was sized before its length came back to the host: a key
        // that does not fit is skipped (the host sees the total, grows the
        // blob and writes it again)
        if (live && off[i] + len[i] <= blob_cap)
            blob_key_bytes(i, e, ref, K1u, K0u, buf, extra, l_pos, l_len, arena, key_off, key_len, sk, blob + off[i]);
        return;
    }
    if (live)
        blob_key_bytes(i, e, ref, K1u, K0u, buf, extra, l_pos, l_len, arena, key_off, key_len, sk,
                       stage + ph + (off[i] - base));
    __syncthreads();
    // chunks c = 0 .. nc-1 cover blob bytes [base - ph + 16 c, + 16)
    const u64 L = end - base;
    if (!L) return;
    const u32 nc = (u32)((ph + L + 15) >> 4);
    u8 *gb = blob + (base - ph);
    for (u32 c = t; c < nc; c += BW_T) {
        const u32 lo = c * 16u, hi = lo + 16u;
        if (lo >= ph && hi <= ph + L) {
            *reinterpret_cast<uint4 *>(gb + lo) = *reinterpret_cast<const uint4 *>(stage + lo);
        } else {
            const u32 a = max(lo, ph), b = min(hi, (u32)(ph + L));
            for (u32 k = a; k < b; ++k) gb[k] = stage[k];
        }
    }
}

// ---------------------------------------------------------------------------
// Small tables (<= MR_MAXN keys) in two launches after k_tile_sort, with no
// dependent global loads (the ranking runs beside the text column's gather,
// which makes every L2 miss slow):
//   k_rank_count  workgroup u: tile u's keys in LDS; every key counts the
//                 keys of tile u smaller than it (binary search in LDS) and
//                 flags an equal one (keys tied on all 24 bytes: long words
//                 sharing 16 bytes and a count) -> cnt[u][i].  One workgroup
//                 per tile: few, long workgroups (beside the gather, a grid
//                 of tile pairs waited for CU slots: 320 us)
//   k_rank_place  rank = sum over u; tied keys ordered by full_cmp (rare);
//                 writes the entry id and its key length at that rank
// (the merge passes, the tie fix-up and k_blob_len in two launches).
#define MR_MAXT 64
#define MR_MAXN ((u64)MR_MAXT * TS_N)
#define RC_T 1024
// tiles: [u TS_N, (u + 1) TS_N), or [ts[u], ts[u + 1]) (<= TS_N keys each)
__global__ __launch_bounds__(RC_T) void k_rank_count(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                     const u64 *__restrict__ K0, u64 n, u32 *__restrict__ cnt,
                                                     const u64 *__restrict__ ts) {
    __shared__ u64 s2[TS_N], s1[TS_N], s0[TS_N];
    const u32 u = blockIdx.x;
    const u64 ub = ts ? ts[u] : (u64)u * TS_N;
    const u32 un = (u32)(ts ? ts[u + 1] - ub : min((u64)TS_N, n - ub));
    for (u32 j = threadIdx.x; j < un; j += RC_T) {
        s2[j] = K2[ub + j];
        s1[j] = K1[ub + j];
        s0[j] = K0[ub + j];
    }
    __syncthreads();
    for (u64 i = threadIdx.x; i < n; i += RC_T) {
        const u64 a2 = K2[i], a1 = K1[i], a0 = K0[i];
        const u32 j = (u32)(i - ub);  // own tile: its index in the tile
        u32 lo = 0, hi = un;  // first key of tile u not smaller than a
        while (lo < hi) {
            const u32 m = (lo + hi) >> 1;
            if (key_lt(s2[m], s1[m], s0[m], a2, a1, a0)) lo = m + 1;
            else hi = m;
        }
        bool tie;
        if (i >= ub && i < ub + un) {
            tie = (j > 0 && s2[j - 1] == a2 && s1[j - 1] == a1 && s0[j - 1] == a0) ||
                  (j + 1 < un && s2[j + 1] == a2 && s1[j + 1] == a1 && s0[j + 1] == a0);
        } else {
            tie = lo < un && s2[lo] == a2 && s1[lo] == a1 && s0[lo] == a0;
        }
        cnt[(u64)u * n + i] = lo | (tie ? 0x80000000u : 0u);
    }
}

__global__ __launch_bounds__(256) void k_rank_place(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                    const u64 *__restrict__ K0, const u32 *__restrict__ V, u64 n,
                                                    const u32 *__restrict__ cnt, const u64 *__restrict__ ref,
                                                    const u8 *buf, const u8 *extra, const u64 *l_pos,
                                                    const u32 *l_len, const u8 *arena, const u64 *key_off,
                                                    const u32 *key_len, u32 *__restrict__ order,
                                                    u64 *__restrict__ len) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 T = (u32)((n + TS_N - 1) / TS_N);
    u64 less = 0;
    u32 tie = 0;
    for (u32 u = 0; u < T; ++u) {
        const u32 c = cnt[(u64)u * n + i];
        less += c & 0x7FFFFFFFu;
        tie |= c;
    }
    const u64 a2 = K2[i], a1 = K1[i], a0 = K0[i];
    const u32 v = V[i];
    const u64 me = ref[v];
    if (tie & 0x80000000u) {  // rare: rank among the tied entries of every tile by full key
        for (u32 u = 0; u < T; ++u) {
            const u64 b = (u64)u * TS_N, e = min(b + TS_N, n);
            u64 lo = b + (cnt[(u64)u * n + i] & 0x7FFFFFFFu);
            for (u64 j = lo; j < e && K2[j] == a2 && K1[j] == a1 && K0[j] == a0; ++j)
                if (j != i && full_cmp(ref[V[j]], me, a1, a0, buf, extra, l_pos, l_len, arena, key_off, key_len) < 0)
                    ++less;
        }
    }
    order[less] = v;
    len[less] = entry_key_len(me, a1, a0, l_len, key_len);
}

// The small-table path's count in one sum per key (k_rank_total + k_rank_put):
// workgroup u keeps tile u's keys in registers (thread = key) and streams every
// tile v through LDS -- double-buffered, the next tile's coalesced loads in
// flight while the current one is searched -- counting the smaller keys of all
// tiles in a register.  Beside the text column's gather every dependent L2 miss
// of k_rank_count's per-key loads waited behind the gather's traffic (386 us
// for 33 K words against ~0.1 ms alone); here each workgroup issues T bulk
// tile loads, each one tile ahead.  Keys equal in all 24 bytes (long words
// sharing 16 bytes and a count) are ordered here too, by full_cmp against the
// equal run the search lands on in each tile (rare; it had been a global
// binary search per tile in k_rank_put: 0.11 ms of the words' chain).
// cnt[i] = the key's rank.
// Small workgroups (RT_T threads, RT_T keys, one 24 KiB tile buffer in LDS,
// the next tile held in registers): the gather's workgroups fill every CU, and
// a workgroup of this size fits in what one finished gather workgroup frees.
#ifndef RC_TOT
#define RC_TOT 1
#endif
#ifndef RT_T
#define RT_T 256
#endif
#define RT_K (TS_N / RT_T)  // tile elements per thread
__global__ __launch_bounds__(RT_T) void k_rank_total(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                     const u64 *__restrict__ K0, const u32 *__restrict__ V, u64 n,
                                                     const u64 *__restrict__ ref, const u8 *buf, const u8 *extra,
                                                     const u64 *l_pos, const u32 *l_len, const u8 *arena,
                                                     const u64 *key_off, const u32 *key_len, u32 *__restrict__ cnt) {
    __shared__ u64 s2[TS_N], s1[TS_N], s0[TS_N];
    const u32 T = (u32)((n + TS_N - 1) / TS_N);
    const u32 t = threadIdx.x;
    const u32 u = blockIdx.x / RT_K;                     // the keys' tile
    const u32 j = (blockIdx.x % RT_K) * RT_T + t;        // the key's place in it
    const u64 i = (u64)u * TS_N + j;
    const bool mine = i < n;
    u64 a2 = 0, a1 = 0, a0 = 0;
    if (mine) { a2 = K2[i]; a1 = K1[i]; a0 = K0[i]; }
    u64 p2[RT_K], p1[RT_K], p0[RT_K];
#pragma unroll
    for (int k = 0; k < RT_K; ++k) {
        const u64 e = (u64)k * RT_T + t;
        p2[k] = p1[k] = p0[k] = 0;
        if (e < n) { p2[k] = K2[e]; p1[k] = K1[e]; p0[k] = K0[e]; }
    }
    u32 less = 0;
    u64 me = ~0ull;  // this entry's ref, loaded at its first tie
    for (u32 v = 0; v < T; ++v) {
#pragma unroll
        for (int k = 0; k < RT_K; ++k) {
            s2[k * RT_T + t] = p2[k];
            s1[k * RT_T + t] = p1[k];
            s0[k * RT_T + t] = p0[k];
        }
        __syncthreads();
        if (v + 1 < T) {  // the next tile's loads in flight during the search
#pragma unroll
            for (int k = 0; k < RT_K; ++k) {
                const u64 e = (u64)(v + 1) * TS_N + (u64)k * RT_T + t;
                if (e < n) { p2[k] = K2[e]; p1[k] = K1[e]; p0[k] = K0[e]; }
            }
        }
        const u32 un = (u32)min((u64)TS_N, n - (u64)v * TS_N);
        if (mine) {
            u32 lo = 0, hi = un;  // first key of tile v not smaller than a
            while (lo < hi) {
                const u32 m = (lo + hi) >> 1;
                if (key_lt(s2[m], s1[m], s0[m], a2, a1, a0)) lo = m + 1;
                else hi = m;
            }
            less += lo;
            // the run of keys equal to this one in tile v (itself excluded):
            // the ones whose full key is smaller come first
            for (u32 q = lo; q < un && s2[q] == a2 && s1[q] == a1 && s0[q] == a0; ++q) {
                if (v == u && q == j) continue;
                if (me == ~0ull) me = ref[V[i]];
                const u64 vb = (u64)v * TS_N;
                if (full_cmp(ref[V[vb + q]], me, a1, a0, buf, extra, l_pos, l_len, arena, key_off, key_len) < 0) ++less;
            }
        }
        __syncthreads();  // tile v read by every thread before the next one is stored
    }
    if (mine) cnt[i] = less;
}

// order[rank] = entry id, len[rank] = its key length
__global__ __launch_bounds__(256) void k_rank_put(const u64 *__restrict__ K1, const u64 *__restrict__ K0,
                                                  const u32 *__restrict__ V, u64 n, const u32 *__restrict__ cnt,
                                                  const u64 *__restrict__ ref, const u32 *l_len, const u32 *key_len,
                                                  u32 *__restrict__ order, u64 *__restrict__ len) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 r = cnt[i], v = V[i];
    order[r] = v;
    len[r] = entry_key_len(ref[v], K1[i], K0[i], l_len, key_len);
}

// ---------------------------------------------------------------------------
// Root-GPU merge of ranked partitions (msa_import_ranked): every received
// block is one GPU's ranked key partition (msa_export_ranked), the blocks'
// keys are disjoint, so the global ranking is their k-way merge -- no
// re-insertion and no sort.  Co-rank: a record's global rank is its index in
// its own block plus, for every other block, the number of that block's keys
// smaller than it (k_mr_corank: one workgroup per tile of <= TS_N records,
// each other block's window of keys between the tile's first and last key
// streamed through LDS; ties on 24 key bytes ordered by the key bytes);
// k_mr_blob writes the counts and the key blob in rank order.  O(n x blocks)
// coalesced loads and O(n) scratch at any table size.
//   block: u64 n, u64 blob_bytes, u64 0, u64 0 | n x {u64 count, u32 len,
//          u32 blob_off, u8 key[16]} | blob (keys in rank order)
__global__ void k_mr_keys(const u8 *__restrict__ in, const u64 *__restrict__ blk_off, const u64 *__restrict__ rec_base,
                          u32 nblk, u64 n, u64 *__restrict__ K2, u64 *__restrict__ K1, u64 *__restrict__ K0,
                          u64 *__restrict__ kptr, u64 *__restrict__ cntv) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 lo = 0, hi = nblk;  // block p: rec_base[p] <= i < rec_base[p + 1]
    while (hi - lo > 1) {
        const u32 m = (lo + hi) >> 1;
        if (rec_base[m] <= i) lo = m;
        else hi = m;
    }
    const u64 p0 = blk_off[lo], j = i - rec_base[lo];
    const u64 nb = rec_base[lo + 1] - rec_base[lo];
    const u64 *rec = reinterpret_cast<const u64 *>(in + p0 + 32 + 32 * j);
    const u64 c = rec[0], w = rec[1];
    const u32 len = (u32)w;
    const u64 kp = p0 + 32 + 32 * nb + (w >> 32);
    u64 h, l;
    be16(in + kp, len, 0, &h, &l);
    K2[i] = ~c;
    K1[i] = h;
    K0[i] = l;
    kptr[i] = kp | ((u64)len << 40);
    cntv[i] = c;
}
__device__ __forceinline__ int mr_cmp(const u8 *in, u64 a, u64 b) {  // strcmp of two keys (a, b: kptr)
    const u8 *pa = in + (a & ((1ull << 40) - 1)), *pb = in + (b & ((1ull << 40) - 1));
    const u64 na = a >> 40, nb = b >> 40, m = na < nb ? na : nb;
    for (u64 k = 16 < m ? 16 : m; k < m; ++k)
        if (pa[k] != pb[k]) return pa[k] < pb[k] ? -1 : 1;
    return na < nb ? -1 : (na > nb ? 1 : 0);
}
#define CR_T TS_N
__global__ __launch_bounds__(CR_T) void k_mr_corank(const u64 *__restrict__ K2, const u64 *__restrict__ K1,
                                                   const u64 *__restrict__ K0, const u64 *__restrict__ ts,
                                                   const u64 *__restrict__ rec_base, u32 nblk,
                                                   const u8 *__restrict__ in, const u64 *__restrict__ kptr,
                                                   u32 *__restrict__ order, u64 *__restrict__ len) {
    __shared__ u64 s2[CR_T], s1[CR_T], s0[CR_T];
    __shared__ u64 win[2];
    const u32 t = threadIdx.x;
    const u64 tb = ts[blockIdx.x], te = ts[blockIdx.x + 1];
    u32 p = 0, ph = nblk;  // the tile's block: rec_base[p] <= tb < rec_base[p + 1]
    while (ph - p > 1) {
        const u32 m = (p + ph) >> 1;
        if (rec_base[m] <= tb) p = m;
        else ph = m;
    }
    const u64 i = tb + t;
    const bool mine = i < te;
    u64 a2 = 0, a1 = 0, a0 = 0;
    if (mine) { a2 = K2[i]; a1 = K1[i]; a0 = K0[i]; }
    u64 less = mine ? i - rec_base[p] : 0;  // its own block is ranked: the index is its rank there
    bool tie = false;
    const u64 f2 = K2[tb], f1 = K1[tb], f0 = K0[tb], l2 = K2[te - 1], l1 = K1[te - 1], l0 = K0[te - 1];
    for (u32 q = 0; q < nblk; ++q) {
        const u64 qb = rec_base[q], qe = rec_base[q + 1];
        if (q == p || qb == qe) continue;
        // block q's window: [first key >= the tile's first, first key > the tile's last)
        if (t < 2) {
            u64 lo = qb, hi = qe;
            while (lo < hi) {
                const u64 m = (lo + hi) >> 1;
                const bool go = t == 0 ? key_lt(K2[m], K1[m], K0[m], f2, f1, f0) : !key_lt(l2, l1, l0, K2[m], K1[m], K0[m]);
                if (go) lo = m + 1;
                else hi = m;
            }
            win[t] = lo;
        }
        __syncthreads();
        const u64 L = win[0], H = win[1];
        __syncthreads();  // read by every thread before the next block's window is stored
        less += L - qb;
        for (u64 c0 = L; c0 < H; c0 += CR_T) {
            const u32 cn = (u32)min((u64)CR_T, H - c0);
            if (t < cn) { s2[t] = K2[c0 + t]; s1[t] = K1[c0 + t]; s0[t] = K0[c0 + t]; }
            __syncthreads();
            if (mine) {
                u32 lo = 0, hi = cn;  // first key of the chunk not smaller than this one
                while (lo < hi) {
                    const u32 m = (lo + hi) >> 1;
                    if (key_lt(s2[m], s1[m], s0[m], a2, a1, a0)) lo = m + 1;
                    else hi = m;
                }
                less += lo;
                tie |= lo < cn && s2[lo] == a2 && s1[lo] == a1 && s0[lo] == a0;
            }
            __syncthreads();
        }
    }
    if (!mine) return;
    const u64 me = kptr[i];
    if (tie)  // rare: a key of another block shares the count and 16 bytes; order by the key bytes
        for (u32 q = 0; q < nblk; ++q) {
            if (q == p) continue;
            u64 lo = rec_base[q], hi = rec_base[q + 1];
            const u64 qe = hi;
            while (lo < hi) {
                const u64 m = (lo + hi) >> 1;
                if (key_lt(K2[m], K1[m], K0[m], a2, a1, a0)) lo = m + 1;
                else hi = m;
            }
            for (u64 j = lo; j < qe && K2[j] == a2 && K1[j] == a1 && K0[j] == a0; ++j)
                if (mr_cmp(in, kptr[j], me) < 0) ++less;
        }
    order[less] = (u32)i;
    len[less] = me >> 40;
}
__global__ void k_mr_blob(const u32 *__restrict__ order, u64 n, const u8 *__restrict__ in, const u64 *__restrict__ kptr,
                          const u64 *__restrict__ cntv, const u64 *__restrict__ off, u8 *__restrict__ blob,
                          u64 *__restrict__ counts) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const u32 i = order[r];
    const u64 kp = kptr[i];
    const u8 *src = in + (kp & ((1ull << 40) - 1));
    u8 *dst = blob + off[r];
    for (u64 k = 0; k < (kp >> 40); ++k) dst[k] = src[k];
    counts[r] = cntv[i];
}

// ---------------------------------------------------------------------------
// host launchers
static inline dim3 grid1(u64 n, u32 t = 256) { return dim3((u32)((n + t - 1) / t)); }

hipError_t msa_launch_rec_spans(const u8 *buf, const u64 *rs, const u32 *nul, u64 nrec, u64 first_rec, int text,
                                u64 *alen, u64 *asrc, u32 *apairs, u64 *tlen, u64 *tsrc, u32 *tpairs, Counters *ctr,
                                const AKeys &ak, const u64 *f0, const u64 *tss, const u64 *tse, u64 *fix,
                                int ablate, hipStream_t s, hipEvent_t fast_end) {
    const SpanOut o{alen, asrc, apairs, tlen, tsrc, tpairs};
    if (!nrec) return fast_end ? hipEventRecord(fast_end, s) : hipSuccess;
    if (!f0) {
        hipLaunchKernelGGL(k_rec_spans, grid1(nrec), dim3(256), 0, s, buf, rs, nul, nrec, first_rec, text, o, ctr, ak);
        if (fast_end) (void)hipEventRecord(fast_end, s);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_rec_fast, grid1(nrec), dim3(256), 0, s, buf, rs, f0, tss, tse, nrec, first_rec, text, o, ctr,
                       ak, fix, ablate);
    if (fast_end) (void)hipEventRecord(fast_end, s);  // its own profiling stage ends here
    // the listed records: a fixed grid, the count read on the device
    const u64 fb = (nrec + 255) / 256 < 1024 ? (nrec + 255) / 256 : 1024;
    hipLaunchKernelGGL(k_rec_fix, dim3((u32)fb), dim3(256), 0, s, buf, rs, nul, first_rec, text, o, ctr, ak, fix);
    return hipGetLastError();
}
// body_p: the column body length on the device (the offsets' scan total);
// the PAD bytes after the column are zeroed here too
__global__ void k_zero_tail(u8 *__restrict__ col, u64 hdr, const u64 *__restrict__ body_p, u32 pad) {
    const u64 at = hdr + *body_p;
    for (u32 k = threadIdx.x; k < pad; k += blockDim.x) col[at + k] = 0;
}
hipError_t msa_launch_col_write(int text, const u8 *buf, const u64 *len, const u64 *off, const u64 *src,
                                const u32 *pairs, u64 nrec, u64 hdr, const u64 *body_p, u8 *col, const u8 *arena,
                                const u64 *key_off, const u32 *key_len, hipStream_t s) {
    hipLaunchKernelGGL(k_zero_tail, dim3(1), dim3(256), 0, s, col, hdr, body_p, (u32)MSA_INPUT_PAD);
    if (!nrec) return hipGetLastError();
    if (!text) {
        hipLaunchKernelGGL(k_col_lines, dim3((u32)((nrec + CL_T - 1) / CL_T)), dim3(CL_T), 0, s, buf, len, off, src,
                           pairs, nrec, hdr, body_p, col, arena, key_off, key_len);
        return hipGetLastError();
    }
    const u64 groups = (nrec + CG_T - 1) / CG_T;
    hipLaunchKernelGGL(k_col_gather, dim3((u32)groups), dim3(CG_T), 0, s, buf, len, off, src, pairs, nrec, hdr, body_p,
                       col);
    hipLaunchKernelGGL(k_col_collapse, grid1(nrec), dim3(256), 0, s, buf, len, off, src, pairs, nrec, hdr, col);
    return hipGetLastError();
}
// Lines of one column laid out at absolute offsets: line j = the source
// bytes [src[j], src[j] + off[j+1] - off[j] - 1) and a '\n' (the column
// splitter's raw-copy values; body_p = the offset right after the column)
hipError_t msa_launch_gather_lines(const u8 *buf, const u64 *len, const u64 *off, const u64 *src, u64 nrec,
                                   const u64 *body_p, u8 *col, hipStream_t s) {
    if (!nrec) return hipSuccess;
    const u64 groups = (nrec + CG_T - 1) / CG_T;
    hipLaunchKernelGGL(k_col_gather, dim3((u32)groups), dim3(CG_T), 0, s, buf, len, off, src, (const u32 *)nullptr,
                       nrec, (u64)0, body_p, col);
    return hipGetLastError();
}
// text.csv's body with the LDS-free gather (beside the token pass)
hipError_t msa_launch_artist_key(const u8 *col, const u64 *ar_start, const u64 *line_off, const u64 *line_len, u64 hdr,
                                 u64 nrec, u8 *arena, u64 *key_off, u32 *key_len, u64 *key_slot, u64 *atab, u64 amask,
                                 u32 *alist, u64 alist_cap, Counters *ctr, u64 short_base, int cus, int abl,
                                 hipStream_t s) {
    if (nrec) {
        u64 blocks = (nrec + AK_T - 1) / AK_T;
        if (blocks > (u64)cus) blocks = (u64)cus;  // one workgroup (one LDS table) per CU
        if (line_len)
            hipLaunchKernelGGL(k_artist_key<true>, dim3((u32)blocks), dim3(AK_T), 0, s, col, ar_start, line_off,
                               line_len, hdr, nrec, arena, key_off, key_len, key_slot, atab, amask, alist, alist_cap,
                               ctr, short_base, abl);
        else
            hipLaunchKernelGGL(k_artist_key<false>, dim3((u32)blocks), dim3(AK_T), 0, s, col, ar_start, line_off,
                               line_len, hdr, nrec, arena, key_off, key_len, key_slot, atab, amask, alist, alist_cap,
                               ctr, short_base, abl);
        hipLaunchKernelGGL(k_artist_verify_reps, grid1(nrec), dim3(256), 0, s, (const u8 *)arena, key_off, key_len,
                           key_slot, nrec, (const u64 *)atab, ctr);
    }
    return hipGetLastError();
}
hipError_t msa_launch_artist_count(const u64 *line_len, const u32 *key_len, const u64 *kh1, const u64 *kh2, u64 nrec,
                                   u64 *atab, u64 amask, u32 *alist, u64 alist_cap, Counters *ctr, int cus,
                                   int ablate, ulonglong2 *alog, u32 *alog_n, u32 alog_cap, hipStream_t s) {
    if (nrec) {
        u64 blocks = (nrec + AC_T - 1) / AC_T;
        if (blocks > (u64)cus) blocks = (u64)cus;
        hipLaunchKernelGGL(k_artist_count, dim3((u32)blocks), dim3(AC_T), 0, s, line_len, key_len, kh1, kh2, nrec, atab,
                           amask, alist, alist_cap, ctr, ablate, alog, alog_n, alog_cap);
        u32 groups = (u32)cus / AC_PARTS;
        if (groups > (u32)blocks) groups = (u32)blocks;
        if (groups < 1) groups = 1;
        hipLaunchKernelGGL(k_artist_merge, dim3(groups * AC_PARTS), dim3(AM_T), 0, s, (const ulonglong2 *)alog,
                           (const u32 *)alog_n, alog_cap, (u32)blocks, groups, atab, amask, alist, alist_cap, ctr);
        hipLaunchKernelGGL(k_artist_h2_check, grid1(alist_cap), dim3(256), 0, s, (const u64 *)atab, (const u32 *)alist,
                           alist_cap, kh2, ctr);
    }
    return hipGetLastError();
}
hipError_t msa_launch_long(const u8 *buf, u64 seg_end, const u8 *extra, u64 extra_len, const u64 *l_pos, u64 n,
                           u32 *l_len, u64 *l_slot, u64 *ltab, u64 lmask, u32 *llist, u64 llist_cap, Counters *ctr,
                           hipStream_t s) {
    if (n) {
        hipLaunchKernelGGL(k_long_insert, grid1(n), dim3(256), 0, s, buf, seg_end, extra, extra_len, l_pos, n, l_len,
                           l_slot, ltab, lmask, llist, llist_cap, ctr);
        hipLaunchKernelGGL(k_long_verify, grid1(n), dim3(256), 0, s, buf, extra, l_pos, (const u32 *)l_len,
                           (const u64 *)l_slot, n, (const u64 *)ltab, ctr);
    }
    return hipGetLastError();
}
hipError_t msa_launch_artist_verify(const u8 *arena, const u64 *key_off, const u32 *key_len, const u64 *key_slot,
                                    u64 n, const u64 *atab, Counters *ctr, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_artist_verify, grid1(n), dim3(256), 0, s, arena, key_off, key_len, key_slot, n, atab, ctr);
    return hipGetLastError();
}
hipError_t msa_launch_long_verify(const u8 *buf, const u8 *extra, const u64 *l_pos, const u32 *l_len,
                                  const u64 *l_slot, u64 n, const u64 *ltab, Counters *ctr, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_long_verify, grid1(n), dim3(256), 0, s, buf, extra, l_pos, l_len, l_slot, n, ltab, ctr);
    return hipGetLastError();
}
hipError_t msa_launch_list_build(const u64 *tab, u64 nslots, u32 stride, u32 *list, u64 cap, u64 *claimed,
                                 Counters *ctr, u64 ovf_bit, hipStream_t s) {
    if (nslots)
        hipLaunchKernelGGL(k_list_build, dim3((u32)((nslots + 4095) / 4096)), dim3(256), 0, s, tab, nslots, stride, list,
                           cap, claimed, ctr, ovf_bit);
    return hipGetLastError();
}
hipError_t msa_launch_word_entries(const EntryArgs &a, hipStream_t s) {
    const u64 n = a.ns + a.nm + a.nl;
    // a grid-stride launch (its key-plane reduction ends in one atomic per workgroup)
    if (n) hipLaunchKernelGGL(k_word_entries, dim3((u32)std::min<u64>(4096, (n + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t msa_launch_artist_entries(const u64 *atab, const u32 *alist, u64 n, const u8 *arena, const u64 *key_off,
                                     const u32 *key_len, u64 *K2, u64 *K1, u64 *K0, u32 *val, u64 *ref, u64 *cnt,
                                     hipStream_t s) {
    if (n)
        hipLaunchKernelGGL(k_artist_entries, grid1(n), dim3(256), 0, s, atab, alist, n, arena, key_off, key_len, K2,
                           K1, K0, val, ref, cnt);
    return hipGetLastError();
}
// Sorts set `in` into one of the two ping-pong sets; returns the set holding
// the result in *which (1 or 2).
hipError_t msa_launch_sort(u64 *const K2[3], u64 *const K1[3], u64 *const K0[3], u32 *const V[3], u64 n, int *which,
                           hipStream_t s) {
    *which = 1;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_tile_sort, dim3((u32)((n + TS_N - 1) / TS_N)), dim3(TS_T), 0, s, K2[0], K1[0], K0[0], V[0],
                       n, K2[1], K1[1], K0[1], V[1]);
    int cur = 1;
    for (u64 w = TS_N; w < n; w <<= 1) {
        const int nx = cur == 1 ? 2 : 1;
        hipLaunchKernelGGL(k_merge_pass, grid1(n), dim3(256), 0, s, K2[cur], K1[cur], K0[cur], V[cur], n, w, K2[nx],
                           K1[nx], K0[nx], V[nx]);
        cur = nx;
    }
    *which = cur;
    return hipGetLastError();
}
// Root-GPU merge of ranked blocks (see k_mr_keys).  Scratch: K2/K1/K0,
// kptr, cntv (n each), cnt (T x n u32), ts (T + 1).  Ends with len / off /
// total (blob offsets) in rank order; k_mr_blob then writes counts + blob.
hipError_t msa_launch_merge_ranked(const u8 *in, const u64 *blk_off, const u64 *rec_base, u32 nblk, u64 n,
                                   const u64 *ts, u32 T, u64 *K2, u64 *K1, u64 *K0, u64 *kptr, u64 *cntv,
                                   u32 *order, u64 *len, u64 *off, u64 *bsum, u64 *total, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_mr_keys, grid1(n), dim3(256), 0, s, in, blk_off, rec_base, nblk, n, K2, K1, K0, kptr, cntv);
    hipLaunchKernelGGL(k_mr_corank, dim3(T), dim3(CR_T), 0, s, (const u64 *)K2, (const u64 *)K1, (const u64 *)K0, ts,
                       rec_base, nblk, in, (const u64 *)kptr, order, len);
    return msa_exclusive_scan(len, n, off, bsum, total, s);
}
hipError_t msa_launch_merge_blob(const u32 *order, u64 n, const u8 *in, const u64 *kptr, const u64 *cntv,
                                 const u64 *off, u8 *blob, u64 *counts, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_mr_blob, grid1(n), dim3(256), 0, s, order, n, in, kptr, cntv, off, blob, counts);
    return hipGetLastError();
}
u64 msa_rank_small_max() { return MR_MAXN; }
// k_rank_total writes one count per key; the per-tile k_rank_count path T x n
u64 msa_rank_small_scratch(u64 n) { return RC_TOT ? n * 4 : ((n + TS_N - 1) / TS_N) * n * 4; }
// Small-table ranking: k_tile_sort + k_rank_count + k_rank_place (entry ids
// and key lengths in rank order) + the blob offsets' scan (total to *total).
// Set 1 of K2/K1/K0/V holds the sorted tiles; cnt: msa_rank_small_scratch(n)
// bytes.
hipError_t msa_launch_rank_small(u64 *const K2[3], u64 *const K1[3], u64 *const K0[3], u32 *const V[3], u64 n,
                                 const u64 *ref, const u8 *buf, const u8 *extra, const u64 *l_pos, const u32 *l_len,
                                 const u8 *arena, const u64 *key_off, const u32 *key_len, u32 *order, u64 *len,
                                 u64 *off, u64 *bsum, u64 *total, u32 *cnt, hipStream_t s) {
    if (!n || n > MR_MAXN) return hipErrorInvalidValue;
    const u32 T = (u32)((n + TS_N - 1) / TS_N);
    hipLaunchKernelGGL(k_tile_sort, dim3(T), dim3(TS_T), 0, s, K2[0], K1[0], K0[0], V[0], n, K2[1], K1[1], K0[1], V[1]);
#if RC_TOT
    hipLaunchKernelGGL(k_rank_total, dim3(T * RT_K), dim3(RT_T), 0, s, K2[1], K1[1], K0[1], (const u32 *)V[1], n, ref,
                       buf, extra, l_pos, l_len, arena, key_off, key_len, cnt);
    hipLaunchKernelGGL(k_rank_put, grid1(n), dim3(256), 0, s, K1[1], K0[1], V[1], n, (const u32 *)cnt, ref, l_len,
                       key_len, order, len);
#else
    hipLaunchKernelGGL(k_rank_count, dim3(T), dim3(RC_T), 0, s, K2[1], K1[1], K0[1], n, cnt, (const u64 *)nullptr);
    hipLaunchKernelGGL(k_rank_place, grid1(n), dim3(256), 0, s, K2[1], K1[1], K0[1], V[1], n, (const u32 *)cnt, ref,
                       buf, extra, l_pos, l_len, arena, key_off, key_len, order, len);
#endif
    return msa_exclusive_scan(len, n, off, bsum, total, s);
}
hipError_t msa_launch_fixup(const u64 *K2, const u64 *K1, const u64 *K0, const u32 *V, u64 n, const u64 *ref,
                            const u8 *buf, const u8 *extra, const u64 *l_pos, const u32 *l_len, const u8 *arena, const u64 *key_off,
                            const u32 *key_len, u32 *out, hipStream_t s) {
    if (!K0) return hipErrorInvalidValue;  // k_tie_fixup compares 16-byte prefixes
    if (n)
        hipLaunchKernelGGL(k_tie_fixup, grid1(n), dim3(256), 0, s, K2, K1, K0, V, n, ref, buf, extra, l_pos, l_len, arena,
                           key_off, key_len, out);
    return hipGetLastError();
}
hipError_t msa_launch_blob(const u32 *order, u64 n, const u64 *ref, const u64 *K1u, const u64 *K0u, const u64 *cnt,
                           const u8 *buf, const u8 *extra, const u64 *l_pos, const u32 *l_len, const u8 *arena, const u64 *key_off,
                           const u32 *key_len, u64 *len, u64 *off, u64 *bsum, u64 *total, u8 *blob, u64 *counts_out,
                           u64 blob_cap, hipStream_t s, int phase, const u64 *Ks2, const u64 *Ks1, const u64 *Ks0,
                           u64 lthr) {
    if (!n) return hipSuccess;
    const SortedKeys sk{Ks2, Ks1, Ks0, Ks1 ? lthr : 0};
    if (phase == 0) {
        hipLaunchKernelGGL(k_blob_len, grid1(n), dim3(256), 0, s, order, n, ref, K1u, K0u, l_len, key_len, sk, len);
        return msa_exclusive_scan(len, n, off, bsum, total, s);
    }
    hipLaunchKernelGGL(k_blob_write, grid1(n, BW_T), dim3(BW_T), 0, s, order, n, ref, K1u, K0u, cnt, buf, extra, l_pos, l_len, arena,
                       key_off, key_len, (const u64 *)off, (const u64 *)len, sk, blob, counts_out, blob_cap);
    return hipGetLastError();
}

u64 msa_tie_blocks(u64 n) { return (n + TB_N - 1) / TB_N; }
hipError_t msa_launch_tie_count(const u64 *K2, const u64 *K1, const u64 *K0, u64 n, u64 *bh, u64 *bt, u64 *big,
                                hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_tie_count, dim3((u32)msa_tie_blocks(n)), dim3(TB_T), 0, s, K2, K1, K0, n, bh, bt, big);
    return hipGetLastError();
}
hipError_t msa_launch_tie_seg(const u64 *K2n, const u64 *K1n, const u64 *K0n, const u32 *Vid, u64 m, u64 *O2, u64 *O1,
                              u64 *O0, u32 *OV, hipStream_t s) {
    if (m) hipLaunchKernelGGL(k_tie_seg, grid1(m), dim3(256), 0, s, K2n, K1n, K0n, Vid, m, O2, O1, O0, OV);
    return hipGetLastError();
}
hipError_t msa_launch_tie_build(const u64 *K2, const u64 *K1, const u64 *K0, u64 mc, const u64 *hoff, const u64 *toff,
                                const u32 *Vc, const u64 *Pc, u32 skip, const u64 *K1u, const u64 *K0u, const u64 *ref,
                                const u8 *buf, const u8 *extra, const u64 *l_pos, const u32 *l_len, const u8 *arena,
                                const u64 *key_off, const u32 *key_len, u64 *K2n, u64 *K1n, u64 *K0n, u32 *Vid,
                                u32 *Vn, u64 *Pn, hipStream_t s) {
    if (mc)
        hipLaunchKernelGGL(k_tie_build, dim3((u32)msa_tie_blocks(mc)), dim3(TB_T), 0, s, K2, K1, K0, mc, hoff, toff, Vc,
                           Pc, skip, K1u, K0u, ref, buf, extra, l_pos, l_len, arena, key_off, key_len, K2n, K1n, K0n,
                           Vid, Vn, Pn);
    return hipGetLastError();
}
hipError_t msa_launch_tie_apply(const u32 *perm, const u32 *Vn, const u64 *Pn, u64 m, u32 *order, u32 *Vc, u64 *Pc,
                                const u64 *K1u, const u64 *K0u, u64 *ks1, u64 *ks0, hipStream_t s) {
    if (m) hipLaunchKernelGGL(k_tie_apply, grid1(m), dim3(256), 0, s, perm, Vn, Pn, m, order, Vc, Pc, K1u, K0u, ks1, ks0);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// word_counts.csv / top_artists.csv lines on the device (write_table_csv +
// write_csv_entry, parallel_spotify.c:307-344): entry i of the ranked table
// becomes `"<key with '"' doubled>",<count>\n`.  k_csv_len sizes every line,
// one exclusive scan places them, k_csv_put writes them: a workgroup stages its
// entries' keys (contiguous in the rank-ordered blob) and its lines (contiguous
// in the output) in LDS, so both the key loads and the line stores are
// coalesced; a workgroup whose keys or lines do not fit (very long keys)
// writes straight to global memory.  The host copies the bytes out and writes
// the file once (the per-entry formatting loop on the host had taken 2.4 s for
// configs[4]'s 50 M words).
#define CSV_T 256
#define CSV_KEY_LDS 12288
#define CSV_OUT_LDS 20480
__device__ __forceinline__ u32 csv_digits(u64 v) {
    u32 d = 1;
    while (v >= 10) {
        v /= 10;
        ++d;
    }
    return d;
}
__device__ __forceinline__ u64 csv_key_end(const u64 *off, u64 i, u64 n, u64 blob_len) {
    return i + 1 < n ? off[i + 1] : blob_len;
}
__global__ __launch_bounds__(CSV_T) void k_csv_len(const u64 *__restrict__ off, const u8 *__restrict__ blob,
                                                   const u64 *__restrict__ cnt, u64 n, u64 m, u64 blob_len,
                                                   int quotes, u64 *__restrict__ len) {
    const u64 i = (u64)blockIdx.x * CSV_T + threadIdx.x;
    if (i >= m) return;
    const u64 b = off[i], e = csv_key_end(off, i, n, blob_len);
    u64 dq = 0;
    if (quotes)  // artists may hold '"' (word keys never do: token bytes are alnum and '\'')
        for (u64 k = b; k < e; ++k) dq += blob[k] == '"';
    len[i] = (e - b) + dq + csv_digits(cnt[i]) + 4;  // '"' key '"' ',' digits '\n'
}
__device__ __forceinline__ u8 *csv_line(u8 *o, const u8 *key, u64 klen, u64 count) {
    *o++ = '"';
    for (u64 k = 0; k < klen; ++k) {
        const u8 ch = key[k];
        if (ch == '"') *o++ = '"';
        *o++ = ch;
    }
    *o++ = '"';
    *o++ = ',';
    const u32 d = csv_digits(count);
    for (u32 k = d; k-- > 0;) {
        o[k] = (u8)('0' + count % 10);
        count /= 10;
    }
    o += d;
    *o++ = '\n';
    return o;
}
// pos: the scan of len (exclusive), pos_total: its total
__global__ __launch_bounds__(CSV_T) void k_csv_put(const u64 *__restrict__ off, const u8 *__restrict__ blob,
                                                   const u64 *__restrict__ cnt, u64 n, u64 m, u64 blob_len,
                                                   const u64 *__restrict__ pos, const u64 *__restrict__ pos_total,
                                                   u8 *__restrict__ out) {
    __shared__ u8 kbuf[CSV_KEY_LDS];
    __shared__ u8 obuf[CSV_OUT_LDS];
    const u64 first = (u64)blockIdx.x * CSV_T, last = min(first + CSV_T, m);  // entries [first, last)
    const u64 i = first + threadIdx.x;
    const u64 kb = off[first], ke = csv_key_end(off, last - 1, n, blob_len);
    const u64 ob = pos[first], oe = last < m ? pos[last] : *pos_total;
    if (ke - kb <= CSV_KEY_LDS && oe - ob <= CSV_OUT_LDS) {
        for (u64 j = threadIdx.x; j < ke - kb; j += CSV_T) kbuf[j] = blob[kb + j];
        __syncthreads();
        if (i < last) {
            const u64 b = off[i], e = csv_key_end(off, i, n, blob_len);
            csv_line(obuf + (pos[i] - ob), kbuf + (b - kb), e - b, cnt[i]);
        }
        __syncthreads();
        for (u64 j = threadIdx.x; j < oe - ob; j += CSV_T) out[ob + j] = obuf[j];
        return;
    }
    if (i < last) {
        const u64 b = off[i], e = csv_key_end(off, i, n, blob_len);
        csv_line(out + pos[i], blob + b, e - b, cnt[i]);
    }
}
// lines of entries [0, m) of a ranked table (n entries, keys off / blob, counts
// cnt).  phase 0: their lengths (len) and offsets (pos, total: the exclusive
// scan, bsum its scratch); phase 1: the bytes into out (total bytes)
hipError_t msa_launch_csv_lines(int phase, const u64 *off, const u8 *blob, const u64 *cnt, u64 n, u64 m, u64 blob_len,
                                int quotes, u64 *len, u64 *pos, u64 *bsum, u64 *total, u8 *out, hipStream_t s) {
    if (!m) return hipSuccess;
    if (phase == 0) {
        hipLaunchKernelGGL(k_csv_len, grid1(m, CSV_T), dim3(CSV_T), 0, s, off, blob, cnt, n, m, blob_len, quotes, len);
        return msa_exclusive_scan(len, m, pos, bsum, total, s);
    }
    hipLaunchKernelGGL(k_csv_put, grid1(m, CSV_T), dim3(CSV_T), 0, s, off, blob, cnt, n, m, blob_len,
                       (const u64 *)pos, (const u64 *)total, out);
    return hipGetLastError();
}
